"""The reference's on-disk test-case format (src/test-data/testCases.ts:34-52): loader round trip,
LFS-stub detection, the reference's expected results, and the JS loader (CPU only)."""
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

from msm_amd import testdata as TD
from oracle import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JS = os.path.join(ROOT, "webgpu-msm_amd", "js", "submission.mjs")
NODE = shutil.which("node")


def _case(tmp_path, n=40, z_scale=False):
    pts = [O.scalar_mul(O.G, 3 + 5 * i) for i in range(n)]
    quads = []
    for i, (x, y) in enumerate(pts):
        z = (7 + i) if z_scale else 1  # projective inputs are legal (README.md:92)
        quads.append((x * z % O.P, y * z % O.P, x * y % O.P * z % O.P, z))
    ss = O.xorshift_scalars(n, seed=77)
    pp, sp = str(tmp_path / "pts.txt"), str(tmp_path / "sc.txt")
    TD.write_test_case(pp, sp, quads, ss)
    return pp, sp, quads, ss


def test_round_trip_matches_wire(tmp_path):
    pp, sp, quads, ss = _case(tmp_path)
    pts, sc = TD.load_test_case(pp, sp)
    assert pts.shape == (40, 32) and sc.shape == (40, 8)
    for i, q in enumerate(quads):
        assert [O.be_words_to_int(pts[i, 8 * j: 8 * j + 8]) for j in range(4)] == list(q)
    assert np.array_equal(sc, O.ints_to_be_words(ss))
    # the reference's format: one JSON object of decimal strings per line
    first = json.loads(open(pp).readline())
    assert set(first) == {"x", "y", "t", "z"} and all(isinstance(v, str) for v in first.values())
    assert TD.load_test_case(pp, sp, limit=5)[0].shape == (5, 32)


def test_lfs_pointer_stub_is_rejected(tmp_path):
    stub = tmp_path / "16-power-points.txt"
    stub.write_text("version https://git-lfs.github.com/spec/v1\noid sha256:00\nsize 17472283\n")
    assert TD.is_lfs_pointer(str(stub))
    with pytest.raises(FileNotFoundError):
        TD.load_test_case(str(stub), str(stub))


def test_expected_results_are_subgroup_points():
    # transcription check of testCases.ts:11-32: on the curve and of order r
    for power, (x, y) in TD.EXPECTED_POWERS.items():
        assert O.on_curve((x, y)), power
        assert O.scalar_mul((x, y), O.R_ORDER) == O.IDENTITY, power


@pytest.mark.skipif(NODE is None, reason="node not installed")
def test_js_load_test_case(tmp_path):
    pp, sp, quads, ss = _case(tmp_path, n=6)
    script = (
        "import { loadTestCase } from %s;\n"
        "(async () => { const tc = await loadTestCase(%s, %s);\n"
        "console.log(JSON.stringify({p: tc.baseAffinePoints.map(q => [q.x, q.y, q.t, q.z].map(String)),"
        " s: tc.scalars.map(String)})); })();\n" % (json.dumps(JS), json.dumps(pp), json.dumps(sp)))
    out = subprocess.run([NODE, "--input-type=module", "-e", script], capture_output=True, text=True, timeout=120,
                         cwd=os.path.dirname(JS))
    assert out.returncode == 0, out.stderr
    got = json.loads(out.stdout)
    assert got["p"] == [[str(v) for v in q] for q in quads]
    assert got["s"] == [str(s) for s in ss]
