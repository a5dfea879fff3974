// End-to-end compute_msm time through the Node surface, the reference's own timing semantics
// (src/ui/Benchmark.tsx:29-39: performance.now() around `await msmFunc(points, scalars)`), for the
// input forms the reference's callers use:
//   flat_input_ms        flat wire buffers over a SharedArrayBuffer (what submission.ts:35-39
//                        allocates; read in place by the addon)
//   flat_copied_input_ms flat wire buffers over a plain ArrayBuffer (copied by the addon first)
//   node_e2e_ms          U32ArrayPoint[] / Uint32Array[] objects (AllBenchmarks.tsx:81-94), with
//                        marshal_ms = their JS flatten alone into compute_msm's reused staging
//                        (flattenStaged), marshal_fresh_ms = into fresh buffers (flattenU32)
//   bigint_input_ms      BigIntPoint[] / bigint[] (the test-data loader's form, testCases.ts:34-52),
//                        marshalled natively by the addon (napi_get_value_bigint_words)
// The flat forms run first, on a fresh heap: millions of live point objects make V8's collector
// pause the main thread, which delays the promise's resolution (the round-3 harness measured the
// flat forms after building the objects and read 7-9 ms for a 4 ms call).
//
//   node --max-old-space-size=16384 tools/node_e2e.mjs <points.bin> <scalars.bin> <n> <runs> [x y]
//
// points.bin / scalars.bin: wire words (x|y|t|z BE u32[8] each / BE u32[8]), as bench.py writes
// them.  Prints one JSON line: medians and all run times (ms), and whether every result matched.
import fs from "fs";
import { performance } from "perf_hooks";
import { compute_msm, flattenStaged, flattenU32, releaseStaged, u32ArrayToBigInts } from "../webgpu-msm_amd/js/submission.mjs";

const [, , pPath, sPath, nArg, runsArg, xArg, yArg] = process.argv;
const n = parseInt(nArg, 10);
const runs = parseInt(runsArg || "5", 10);
const expect = xArg ? { x: BigInt(xArg), y: BigInt(yArg) } : null;
const med = (xs) => [...xs].sort((a, b) => a - b)[Math.floor(xs.length / 2)];
let ok = true;

// runs + 1 awaited calls of compute_msm(p(), s()); the first warms the addon, context and graphs
async function timeCalls(p, s) {
  const ts = [];
  for (let r = 0; r <= runs; r++) {
    const t0 = performance.now();
    const res = await compute_msm(p, s);
    const t1 = performance.now();
    if (r > 0) ts.push(t1 - t0);
    if (expect && (res.x !== expect.x || res.y !== expect.y)) ok = false;
  }
  return ts;
}

(async () => {
  let pw = new Uint32Array(fs.readFileSync(pPath).buffer.slice(0));
  let sw = new Uint32Array(fs.readFileSync(sPath).buffer.slice(0));
  const share = (a) => {
    const b = new Uint32Array(new SharedArrayBuffer(a.length * 4));
    b.set(a);
    return b;
  };
  let spw = share(pw), ssw = share(sw);
  const flatTimes = await timeCalls(spw, ssw);
  const copyTimes = await timeCalls(pw, sw);
  spw = ssw = null;
  // U32ArrayPoint[] objects: one Uint32Array per coordinate and per scalar, as bigIntToU32Array
  // gives the reference's harness
  let points = new Array(n);
  let scalars = new Array(n);
  for (let i = 0; i < n; i++) {
    const o = 32 * i;
    points[i] = { x: pw.slice(o, o + 8), y: pw.slice(o + 8, o + 16), t: pw.slice(o + 16, o + 24), z: pw.slice(o + 24, o + 32) };
    scalars[i] = sw.slice(8 * i, 8 * i + 8);
  }
  const objTimes = await timeCalls(points, scalars);
  const flat = [], fresh = [];
  for (let r = 0; r < runs; r++) {
    let t0 = performance.now();
    releaseStaged(flattenStaged(points, scalars));  // what compute_msm does: reused staging
    flat.push(performance.now() - t0);
    t0 = performance.now();
    flattenU32(points, scalars);  // fresh SharedArrayBuffers (page faults on first touch)
    fresh.push(performance.now() - t0);
  }
  points = scalars = null;
  // BigIntPoint[] / bigint[]
  const big = (o) => u32ArrayToBigInts(pw.subarray(o, o + 8))[0];
  let bpoints = new Array(n);
  let bscalars = new Array(n);
  for (let i = 0; i < n; i++) {
    const o = 32 * i;
    bpoints[i] = { x: big(o), y: big(o + 8), t: big(o + 16), z: big(o + 24) };
    bscalars[i] = u32ArrayToBigInts(sw.subarray(8 * i, 8 * i + 8))[0];
  }
  const bigTimes = await timeCalls(bpoints, bscalars);
  console.log(JSON.stringify({
    flat_input_ms: med(flatTimes), flat_copied_input_ms: med(copyTimes), node_e2e_ms: med(objTimes),
    marshal_ms: med(flat), marshal_fresh_ms: med(fresh), bigint_input_ms: med(bigTimes), runs_ms: { flat: flatTimes, flat_copied: copyTimes,
    objects: objTimes, bigint: bigTimes }, correct: expect ? ok : null,
  }));
})().catch((e) => {
  console.log(JSON.stringify({ error: String(e) }));
  process.exit(1);
});
