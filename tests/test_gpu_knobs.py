"""GPU parity of libmsm's measured-and-kept-off launch paths (the environment knobs DESIGN.md §2.4
lists): every knob is read once per process, so each setting runs in a child process of its own
(one at a time, a few seconds each) over the same cases, checked bit-exact against the closed form
sum s_i (k_i G) = ((sum s_i k_i) mod r) G (tests/golden/msm_vectors.json pins it to the oracle).

Cases per setting: msm_compute from host arrays below the split (2^17 + 777 points, run_host) and
through it (2^19 + 5: four slices in two launches, the last one short), with one projective point
in each; and 5 MSMs of 2^16 points through the pipelined entry from host arrays (msm_compute_many).
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, sys
import numpy as np
sys.path[:0] = [{root!r}, {root!r} + "/webgpu-msm_amd", {root!r} + "/tests"]
import msm_amd as M
from _closed_form import as_xy, closed_form
from oracle import oracle as O

def projective(pts, i, z):
    x, y, t = (O.be_words_to_int(pts[i, 8 * j: 8 * j + 8]) for j in range(3))
    for j, v in enumerate((x * z % O.P, y * z % O.P, t * z % O.P, z)):
        pts[i, 8 * j: 8 * j + 8] = O.int_to_be_words(v)

out = []
for n, k0, step, seed in ((131072 + 777, 6, 11, 19), ((1 << 19) + 5, 9, 7, 77)):
    pts = M.gen_points(n, k0=k0, step=step)
    sc = M.gen_scalars(n, seed=seed)
    projective(pts, n // 2 + 3, 12345)
    out.append(M.compute_msm_wire(pts, sc) == closed_form(k0, step, sc))
n = 65536
pl, sl, ex = [], [], []
for b in range(5):
    pl.append(M.gen_points(n, k0=3 + b, step=5))
    sl.append(M.gen_scalars(n, seed=100 + b))
    ex.append(closed_form(3 + b, 5, sl[-1]))
res = M.compute_msm_many(pl, sl, n)
out.append([tuple(as_xy(r)) for r in res] == [tuple(e) for e in ex])
print(json.dumps(out))
"""


@pytest.mark.parametrize("env", [
    {"MSM_HOST_PACK": "0"},                        # host points uploaded whole (x|y|t|z, pageable)
    {"MSM_HOST_OWN_PTS": "0"},                     # the split's points into the slots' wire buffers
    {"MSM_HOST_SC_FIRST": "0"},                    # scalars per launch beside the points
    {"MSM_HOST_TAIL_LOG": "15"},                   # graded tail launch of short slices
    {"MSM_RED2_TREE": "0"},                        # k_bucket_reduce_2 for the second stage
    {"MSM_HORNER_THREADS": "0", "MSM_FORK_PREP_PIPE": "1"},  # tails inline, preparation forked
    {"MSM_HOST_SORT_EARLY": "0", "MSM_HOST_PACK_THREADS": "1"},
    {"MSM_PIN_MAX_MB": "1"},                       # staging ring over its cap: every entry unpacked
    {"MSM_RED1_PAIRS": "1"},                       # first reduction stage on lane pairs
    {"MSM_RED_FOLD": "1"},                         # first stage and group trees in one launch
    {"MSM_RECODE_FIXED": "0"},                     # the generic recode loop at every width
    {"MSM_STAGGER": "0"},                          # pipelined launches not staggered
])
def test_knob_paths_bit_exact(env):
    e = dict(os.environ)
    e.update(env)
    r = subprocess.run([sys.executable, "-c", CHILD.format(root=ROOT)], env=e, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    assert json.loads(r.stdout.strip().splitlines()[-1]) == [True, True, True], (env, r.stdout[-500:])


TAIL_CHILD = r"""
import json, sys
sys.path[:0] = [{root!r}, {root!r} + "/webgpu-msm_amd", {root!r} + "/tests"]
import msm_amd as M
from _closed_form import closed_form
n = 1 << 22
pts = M.gen_points(n, k0=5, step=3)
sc = M.gen_scalars(n, seed=2024)
print(json.dumps(M.compute_msm_wire(pts, sc) == closed_form(5, 3, sc)))
"""


def test_tail_slices_longer_than_body_slices():
    # MSM_HOST_TAIL_LOG = 18 at 2^22 points asks for tail slices of 2^18 while the body's 16 slices
    # hold (2^22 - 2^19) / 16 = 229,376: the tail is dropped (every slice runs as an MSM of the
    # body's length; a longer tail slice would lose points)
    e = dict(os.environ, MSM_HOST_TAIL_LOG="18")
    r = subprocess.run([sys.executable, "-c", TAIL_CHILD.format(root=ROOT)], env=e, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    assert json.loads(r.stdout.strip().splitlines()[-1]) is True
