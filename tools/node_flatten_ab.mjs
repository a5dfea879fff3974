// A/B of the two flattenings of compute_msm's U32ArrayPoint[] inputs (what AllBenchmarks.tsx:124-132
// builds: one Uint32Array(8) per coordinate and per scalar) into flat wire buffers: the JS loop
// (submission.mjs flattenU32) against the addon's native flattenU32.  No GPU needed.
//   node tools/node_flatten_ab.mjs [log2 n] [rounds]
import { createRequire } from "module";
import { flattenU32 } from "../webgpu-msm_amd/js/submission.mjs";

const require = createRequire(import.meta.url);
const addon = require("../webgpu-msm_amd/js/msm_napi.node");
const lg = parseInt(process.argv[2] || "20", 10);
const rounds = parseInt(process.argv[3] || "5", 10);
const n = 1 << lg;
const mk = (seed) => {
  const a = new Uint32Array(8);
  for (let i = 0; i < 8; i++) a[i] = (Math.imul(seed + 1, 2654435761) ^ (i * 40503)) >>> 0;
  return a;
};
const pts = [];
const sc = [];
for (let i = 0; i < n; i++) {
  pts.push({ x: mk(4 * i), y: mk(4 * i + 1), t: mk(4 * i + 2), z: mk(4 * i + 3) });
  sc.push(mk(-i));
}
const js = [];
const nat = [];
let same = true;
for (let r = 0; r < rounds; r++) {
  let t0 = process.hrtime.bigint();
  const [pb, sb] = flattenU32(pts, sc);
  js.push(Number(process.hrtime.bigint() - t0) / 1e6);
  t0 = process.hrtime.bigint();
  const pw = new Uint32Array(new SharedArrayBuffer(n * 128));
  const sw = new Uint32Array(new SharedArrayBuffer(n * 32));
  addon.flattenU32(pts, sc, pw, sw);
  nat.push(Number(process.hrtime.bigint() - t0) / 1e6);
  if (r === 0) for (let i = 0; i < n * 32 && same; i++) same = pb[i] === pw[i] && (i >= n * 8 || sb[i] === sw[i]);
}
const med = (a) => [...a].sort((x, y) => x - y)[a.length >> 1];
console.log(JSON.stringify({ n, rounds, js_ms: js.map((x) => +x.toFixed(1)), native_ms: nat.map((x) => +x.toFixed(1)),
  js_median_ms: +med(js).toFixed(1), native_median_ms: +med(nat).toFixed(1), identical: same }));
