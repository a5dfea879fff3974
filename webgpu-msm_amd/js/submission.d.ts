// Type surface of submission.mjs — identical to the reference's (src/reference/types.ts:1-13,
// src/submission/submission.ts:25-28).
export type BigIntPoint = { x: bigint; y: bigint; t: bigint; z: bigint };
export type U32ArrayPoint = { x: Uint32Array; y: Uint32Array; t: Uint32Array; z: Uint32Array };

// Extensions: flat wire buffers (n x 32 / n x 8 BE words: the fast form, no per-point
// marshalling) and options { windowSize, devices, cpuWorkRatio } (devices: gfx950 HIP ordinals to
// shard over; cpuWorkRatio: the reference's CPU/GPU split, submission.ts:94-154).
export declare const compute_msm: (
  baseAffinePoints: BigIntPoint[] | U32ArrayPoint[] | Uint32Array,
  scalars: bigint[] | Uint32Array[] | Uint32Array,
  options?: { windowSize?: number; devices?: number[]; cpuWorkRatio?: number }
) => Promise<{ x: bigint; y: bigint }>;
export declare function flattenU32(points: U32ArrayPoint[], scalars: Uint32Array[]): [Uint32Array, Uint32Array];

export declare function getBestWindowSize(n: number): number;
export declare function u32ArrayToBigInts(u32Array: Uint32Array): bigint[];
export declare const split_dynamic: (windowSize: number, scalars: Uint32Array) => Uint32Array;
export declare const point_add_affine: (a: Uint32Array, b: Uint32Array) => Uint32Array;
export declare const init: () => number;
export declare const deviceCount: () => number;
export declare const deviceOrdinals: () => number[];
export declare const nUint32PerScalar: 8;
export declare const nUint32PerPoint: 32;
export declare const loadTestCase: (
  pointsPath: string,
  scalarsPath: string
) => Promise<{ baseAffinePoints: BigIntPoint[]; scalars: bigint[] }>;
export declare const expectedPowersResult: Record<16 | 17 | 18 | 19 | 20, { x: bigint; y: bigint }>;
