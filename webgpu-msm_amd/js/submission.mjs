// compute_msm — drop-in for the reference's public entry point
// (src/submission/submission.ts:25-157), routed through the N-API addon (addon.cc) into
// libmsm's HIP kernels on MI355X.  Same signature and result:
//
//   compute_msm(baseAffinePoints: BigIntPoint[] | U32ArrayPoint[],
//               scalars: bigint[] | Uint32Array[]) => Promise<{ x: bigint, y: bigint }>
//
// Also accepted (an extension, and the fast form): flat wire buffers, a Uint32Array of n x 32
// point words and one of n x 8 scalar words -- the layout flattenU32 builds -- which skips the JS
// marshalling of n point objects (at 2^20 that marshalling is ~25x the MSM itself).  Flat arrays
// over a SharedArrayBuffer (as the reference allocates them, submission.ts:35-39) are read in
// place; over a plain ArrayBuffer the addon copies them first (they could be detached meanwhile).
//
// The browser-only knobs (?windowSize=, submission.ts:29-33) become an optional third
// argument { windowSize } or the MSM_WINDOW_SIZE environment variable.  { devices: [0, 1, ...] }
// shards the MSM over those gfx950 devices inside this one call (one host thread and PCIe link
// each, partials joined with one EC add each) -- the multi-device form of the reference's
// CPU/GPU split.  { cpuWorkRatio } (or MSM_CPU_WORK_RATIO) is that split itself (?cpuWorkRatio,
// submission.ts:94-154): the first floor(ratio n) points on libmsm's host Pippenger beside the GPU
// share, joined with one EC add (msm_compute_cocompute).  Same result for every ratio; on MI355X
// any share above ~0.1% only delays it (the host is ~800x slower than one GPU).
// There is no WebGPU/WGSL/CPU fallback: without the addon or a gfx950 device this rejects.
import { createRequire } from "module";
import fs from "fs";

const require = createRequire(import.meta.url);
const addon = require("./msm_napi.node");

export const nUint32PerScalar = 8; // consts.ts:1
export const nUint32PerPoint = 4 * nUint32PerScalar; // consts.ts:3

// getBestWindowSize (submission.ts:18-23), tuned for libmsm's signed-digit pipeline.
export function getBestWindowSize(n) {
  return addon.bestWindowSize(n);
}

function windowFrom(options) {
  if (options && options.windowSize) return options.windowSize | 0;
  const env = typeof process !== "undefined" && process.env ? process.env.MSM_WINDOW_SIZE : undefined;
  return env ? parseInt(env, 10) : 0;
}

// u32ArrayToBigInts (submission.ts:159-175): 8 big-endian words per value.
export function u32ArrayToBigInts(u32Array) {
  const out = [];
  for (let i = 0; i < u32Array.length; i += 8) {
    let v = 0n;
    for (let j = 0; j < 8 && i + j < u32Array.length; j++) v = (v << 32n) | BigInt(u32Array[i + j]);
    out.push(v);
  }
  return out;
}

// U32ArrayPoint[] / Uint32Array[] -> flat wire buffers (submission.ts:75-86 layout x|y|t|z).
// Element-wise copies: on Node 12 a per-coordinate TypedArray.set() costs more than the 8 word
// copies it replaces (2^20 points: ~15-30% faster flatten, measured locally).
// Exported for tools/node_e2e.mjs, which times this JS marshalling share of compute_msm.
// The buffers live on SharedArrayBuffers (as in submission.ts:35-39), so the addon reads them in
// place.
export function flattenU32(points, scalars) {
  const n = Math.min(points.length, scalars.length);
  const pb = new Uint32Array(new SharedArrayBuffer(n * nUint32PerPoint * 4));
  const sb = new Uint32Array(new SharedArrayBuffer(n * nUint32PerScalar * 4));
  flattenInto(points, scalars, n, pb, sb);
  return [pb, sb];
}

// Staging buffers of compute_msm's object inputs, kept between calls: the first touch of fresh
// SharedArrayBuffer pages costs ~50 ms per 160 MiB (2^20 points) in page faults, more than the
// word copies.  A call takes a free pair (or makes one) and gives it back when its promise settles,
// so concurrent calls never share one; at most two pairs of up to 2^21 points are kept.
const stagingFree = [];
function takeStaging(n) {
  for (let i = 0; i < stagingFree.length; i++) if (stagingFree[i].cap >= n) return stagingFree.splice(i, 1)[0];
  return { cap: n, pb: new Uint32Array(new SharedArrayBuffer(n * nUint32PerPoint * 4)),
           sb: new Uint32Array(new SharedArrayBuffer(n * nUint32PerScalar * 4)) };
}
function giveStaging(st) {
  if (st.cap <= 1 << 21 && stagingFree.length < 2) stagingFree.push(st);
}
// Exported for tools/node_e2e.mjs: compute_msm's marshalling of object inputs into reused staging.
export function flattenStaged(points, scalars) {
  const n = Math.min(points.length, scalars.length);
  const st = takeStaging(n);
  flattenInto(points, scalars, n, st.pb, st.sb);
  return { st, pb: st.pb.subarray(0, n * nUint32PerPoint), sb: st.sb.subarray(0, n * nUint32PerScalar) };
}
export const releaseStaged = (staged) => giveStaging(staged.st);

function flattenInto(points, scalars, n, pb, sb) {
  for (let i = 0; i < n; i++) {
    const p = points[i];
    const o = i * 32;
    const x = p.x, y = p.y, t = p.t, z = p.z, s = scalars[i];
    pb[o] = x[0]; pb[o + 1] = x[1]; pb[o + 2] = x[2]; pb[o + 3] = x[3];
    pb[o + 4] = x[4]; pb[o + 5] = x[5]; pb[o + 6] = x[6]; pb[o + 7] = x[7];
    pb[o + 8] = y[0]; pb[o + 9] = y[1]; pb[o + 10] = y[2]; pb[o + 11] = y[3];
    pb[o + 12] = y[4]; pb[o + 13] = y[5]; pb[o + 14] = y[6]; pb[o + 15] = y[7];
    pb[o + 16] = t[0]; pb[o + 17] = t[1]; pb[o + 18] = t[2]; pb[o + 19] = t[3];
    pb[o + 20] = t[4]; pb[o + 21] = t[5]; pb[o + 22] = t[6]; pb[o + 23] = t[7];
    pb[o + 24] = z[0]; pb[o + 25] = z[1]; pb[o + 26] = z[2]; pb[o + 27] = z[3];
    pb[o + 28] = z[4]; pb[o + 29] = z[5]; pb[o + 30] = z[6]; pb[o + 31] = z[7];
    const q = i * 8;
    sb[q] = s[0]; sb[q + 1] = s[1]; sb[q + 2] = s[2]; sb[q + 3] = s[3];
    sb[q + 4] = s[4]; sb[q + 5] = s[5]; sb[q + 6] = s[6]; sb[q + 7] = s[7];
  }
}

function ratioFrom(options) {
  if (options && options.cpuWorkRatio !== undefined && options.cpuWorkRatio !== null) return Number(options.cpuWorkRatio);
  const env = typeof process !== "undefined" && process.env ? process.env.MSM_CPU_WORK_RATIO : undefined;
  return env ? parseFloat(env) : 0;
}

function devicesFrom(options) {
  if (!options || options.devices === undefined || options.devices === null) return undefined;
  if (!Array.isArray(options.devices)) throw new TypeError("options.devices must be an array of device ordinals");
  return options.devices;
}

export const compute_msm = async (baseAffinePoints, scalars, options) => {
  const windowSize = windowFrom(options);
  const devices = devicesFrom(options);
  const cpuWorkRatio = ratioFrom(options);
  if (baseAffinePoints instanceof Uint32Array && scalars instanceof Uint32Array) {
    // already flat wire buffers (x|y|t|z BE words per point, BE words per scalar): no marshalling
    const n = Math.min(Math.floor(baseAffinePoints.length / nUint32PerPoint), Math.floor(scalars.length / nUint32PerScalar));
    const result = await addon.computeMsmU32(baseAffinePoints.subarray(0, n * nUint32PerPoint),
                                             scalars.subarray(0, n * nUint32PerScalar), windowSize, devices, cpuWorkRatio);
    const [x, y] = u32ArrayToBigInts(result);
    return { x, y };
  }
  const hasBigInt =
    (baseAffinePoints.length > 0 && typeof baseAffinePoints[0].x === "bigint") ||
    (scalars.length > 0 && typeof scalars[0] === "bigint");
  let result;
  if (hasBigInt) {
    // native marshalling (napi_get_value_bigint_words) replaces convert_worker.ts
    const pts = typeof baseAffinePoints[0].x === "bigint" ? baseAffinePoints : baseAffinePoints.map(toBigIntPoint);
    const sc = typeof scalars[0] === "bigint" ? scalars : scalars.map((s) => u32ArrayToBigInts(s)[0]);
    result = await addon.computeMsmBigInt(pts, sc, windowSize, devices, cpuWorkRatio);
  } else {
    const staged = flattenStaged(baseAffinePoints, scalars);
    try {
      result = await addon.computeMsmU32(staged.pb, staged.sb, windowSize, devices, cpuWorkRatio);
    } finally {
      giveStaging(staged.st);
    }
  }
  const [x, y] = u32ArrayToBigInts(result);
  return { x, y };
};

function toBigIntPoint(p) {
  return {
    x: u32ArrayToBigInts(p.x)[0],
    y: u32ArrayToBigInts(p.y)[0],
    t: u32ArrayToBigInts(p.t)[0],
    z: u32ArrayToBigInts(p.z)[0],
  };
}

// Reference helper entry points (lib.rs:196-253), exposed for parity with the wasm module.
export const split_dynamic = (windowSize, scalarsU32) => addon.split(windowSize, scalarsU32);
export const point_add_affine = (a16, b16) => addon.pointAddAffine(a16, b16);
export const init = () => addon.init();
export const deviceCount = () => addon.deviceCount();
export const deviceOrdinals = () => addon.deviceOrdinals();

// loadTestCase (src/test-data/testCases.ts:34-52): JSON-lines points whose string fields are
// BigInts, and one decimal scalar per line.  Paths instead of fetch() URLs (Node, not a browser).
export const loadTestCase = async (pointsPath, scalarsPath) => {
  const pointsText = await fs.promises.readFile(pointsPath, "utf8");
  if (pointsText.startsWith("version https://git-lfs.github.com/spec/v1"))
    throw new Error(`${pointsPath} is a Git-LFS pointer stub, not the test data`);
  const baseAffinePoints = pointsText
    .trim()
    .split("\n")
    .filter((l) => l.length)
    .map((line) => JSON.parse(line, (key, value) => (typeof value === "string" ? BigInt(value) : value)));
  const scalarsText = await fs.promises.readFile(scalarsPath, "utf8");
  const scalars = scalarsText
    .trim()
    .split("\n")
    .filter((l) => l.length)
    .map((line) => BigInt(line));
  return { baseAffinePoints, scalars };
};

// Expected results of the reference's 2^16..2^20 cases (testCases.ts:11-32).
export const expectedPowersResult = {
  16: { x: 4490298471131273381350715833932091894064554978284853693957586604825823442429n, y: 207233051598812890797414182362695316831408959017076683749810755208551572458n },
  17: { x: 405755281347735151880827575059343698498813029460786026451708154294960743560n, y: 7112985356832152643523650125935205310677117771129806490701829425450717492869n },
  18: { x: 4020134989704514076121556080357844499902614818105934254331815581426895427831n, y: 2694327822589008080344499645494473764166611881342421427746308662023437975766n },
  19: { x: 3856727778963570638772781884183843350150969534777451295534564482755471873113n, y: 1398750101296346671684024297455637342909036274728274942667983346895370713922n },
  20: { x: 5201851187583570844529445080011852189038251929148722905178398320328749074909n, y: 3586360219804356686204324370397321114669962278596135149389460948678051407803n },
};
