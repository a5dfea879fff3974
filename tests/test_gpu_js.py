"""The TypeScript/JS drop-in (webgpu-msm_amd/js/submission.mjs) end to end on the GPU:
compute_msm with BigIntPoint[]/bigint[] and U32ArrayPoint[]/Uint32Array[] inputs, and with
flat wire buffers (the marshalling-free extension), and with { cpuWorkRatio } (the reference's
CPU/GPU split, submission.ts:94-154: msm_compute_cocompute)."""
import json
import os
import shutil
import subprocess

import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JS = os.path.join(ROOT, "webgpu-msm_amd", "js", "submission.mjs")
NODE = shutil.which("node")


@pytest.mark.skipif(NODE is None, reason="node not installed")
@pytest.mark.parametrize("form,ratio", [("bigint", None), ("u32", None), ("flat", None), ("bigint", 0.3),
                                        ("u32", 0.001), ("flat", 0.5), ("flat", 1.0)])
def test_compute_msm_js(form, ratio, tmp_path):
    n = 500
    pts = O.gen_points(n, k0=21, step=13)
    ss = O.xorshift_scalars(n, seed=77)
    exp = O.closed_form_msm([21 + 13 * i for i in range(n)], ss)
    rows = [[O.be_words_to_int(pts[i, 8 * j: 8 * j + 8]) for j in range(4)] for i in range(n)]
    data = json.dumps({"pts": [[str(v) for v in r] for r in rows], "sc": [str(s) for s in ss]})
    script = f"""
import * as m from {json.dumps(JS)};
const d = {data};
const toWords = (v) => {{ const w = new Uint32Array(8); let b = BigInt(v);
  for (let i = 7; i >= 0; i--) {{ w[i] = Number(b & 0xffffffffn); b >>= 32n; }} return w; }};
let points, scalars;
if ("{form}" === "bigint") {{
  points = d.pts.map(([x, y, t, z]) => ({{x: BigInt(x), y: BigInt(y), t: BigInt(t), z: BigInt(z)}}));
  scalars = d.sc.map(BigInt);
}} else if ("{form}" === "u32") {{
  points = d.pts.map(([x, y, t, z]) => ({{x: toWords(x), y: toWords(y), t: toWords(t), z: toWords(z)}}));
  scalars = d.sc.map(toWords);
}} else {{  // flat wire buffers (the extension): n x 32 and n x 8 words
  points = new Uint32Array(d.pts.length * 32);
  d.pts.forEach((r, i) => r.forEach((v, j) => points.set(toWords(v), 32 * i + 8 * j)));
  scalars = new Uint32Array(d.sc.length * 8);
  d.sc.forEach((v, i) => scalars.set(toWords(v), 8 * i));
}}
m.compute_msm(points, scalars, {json.dumps({"cpuWorkRatio": ratio} if ratio is not None else None)}).then((r) => console.log(r.x.toString() + "," + r.y.toString()),
  (e) => {{ console.error(e); process.exit(3); }});
"""
    path = tmp_path / "run_js.mjs"
    path.write_text(script)
    out = subprocess.run([NODE, str(path)], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    x, y = out.stdout.strip().split(",")
    assert (int(x), int(y)) == exp
