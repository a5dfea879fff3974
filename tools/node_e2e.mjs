// End-to-end compute_msm time through the Node surface, the reference's own timing semantics
// (src/ui/Benchmark.tsx:29-39: performance.now() around `await msmFunc(points, scalars)`, with
// the U32ArrayPoint[] / Uint32Array[] inputs AllBenchmarks.tsx:81-94 builds).
//
//   node --max-old-space-size=8192 tools/node_e2e.mjs <points.bin> <scalars.bin> <n> <runs> [x y]
//
// points.bin / scalars.bin: wire words (x|y|t|z BE u32[8] each / BE u32[8]), as bench.py writes
// them.  Prints one JSON line: median and all run times (ms), and whether every result matched.
import fs from "fs";
import { performance } from "perf_hooks";
import { compute_msm, flattenU32 } from "../webgpu-msm_amd/js/submission.mjs";

const [, , pPath, sPath, nArg, runsArg, xArg, yArg] = process.argv;
const n = parseInt(nArg, 10);
const runs = parseInt(runsArg || "5", 10);
const pw = new Uint32Array(fs.readFileSync(pPath).buffer.slice(0));
const sw = new Uint32Array(fs.readFileSync(sPath).buffer.slice(0));
// one Uint32Array per coordinate and per scalar, as bigIntToU32Array gives the harness
const points = new Array(n);
const scalars = new Array(n);
for (let i = 0; i < n; i++) {
  const o = 32 * i;
  points[i] = {
    x: pw.slice(o, o + 8),
    y: pw.slice(o + 8, o + 16),
    t: pw.slice(o + 16, o + 24),
    z: pw.slice(o + 24, o + 32),
  };
  scalars[i] = sw.slice(8 * i, 8 * i + 8);
}
const expect = xArg ? { x: BigInt(xArg), y: BigInt(yArg) } : null;
(async () => {
  const times = [];
  let ok = true;
  for (let r = 0; r <= runs; r++) {
    const t0 = performance.now();
    const res = await compute_msm(points, scalars);
    const t1 = performance.now();
    if (r > 0) times.push(t1 - t0); // run 0 warms the addon, device context and graphs
    if (expect && (res.x !== expect.x || res.y !== expect.y)) ok = false;
  }
  // the JS marshalling share alone: compute_msm's flatten of the U32ArrayPoint[] objects
  const flat = [];
  for (let r = 0; r < runs; r++) {
    const t0 = performance.now();
    flattenU32(points, scalars);
    flat.push(performance.now() - t0);
  }
  // the same MSM from flat wire buffers (no marshalling): the addon + libmsm share.  Over a
  // SharedArrayBuffer (as the reference allocates its buffers, submission.ts:35-39) the addon reads
  // them in place; over a plain ArrayBuffer (pw, sw) it copies them first (detachable memory).
  const share = (a) => {
    const b = new Uint32Array(new SharedArrayBuffer(a.length * 4));
    b.set(a);
    return b;
  };
  const spw = share(pw), ssw = share(sw);
  const timeFlat = async (p, s) => {
    const ts = [];
    for (let r = 0; r <= runs; r++) {
      const t0 = performance.now();
      const res = await compute_msm(p, s);
      const t1 = performance.now();
      if (r > 0) ts.push(t1 - t0);
      if (expect && (res.x !== expect.x || res.y !== expect.y)) ok = false;
    }
    return ts;
  };
  const flatTimes = await timeFlat(spw, ssw);
  const copyTimes = await timeFlat(pw, sw);
  const med = (xs) => [...xs].sort((a, b) => a - b)[Math.floor(xs.length / 2)];
  console.log(JSON.stringify({ node_e2e_ms: med(times), marshal_ms: med(flat), flat_input_ms: med(flatTimes),
                               flat_copied_input_ms: med(copyTimes), runs_ms: times, correct: expect ? ok : null }));
})().catch((e) => {
  console.log(JSON.stringify({ error: String(e) }));
  process.exit(1);
});
