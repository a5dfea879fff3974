"""CPU/GPU co-compute (msm_compute_cocompute, the reference's ?cpuWorkRatio branch,
submission.ts:94-154): the first floor(ratio n) points on libmsm's host Pippenger beside the GPU
share, joined with one EC add.  Every ratio must give msm_compute's result (closed form / oracle),
including the reference's edge branches: a share that floors to 0 (GPU only) and a share >= n
(host only)."""
import numpy as np
import pytest

import msm_amd as M
from _closed_form import closed_form
from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("ratio", [1e-4, 0.001, 0.1, 0.5, 0.999, 1.0, 2.5])
def test_cocompute_ratios_match_closed_form(ratio):
    n = 5000
    pts = M.gen_points(n, k0=5, step=11)
    sc = M.gen_scalars(n, seed=31)
    exp = closed_form(5, 11, sc)
    assert M.compute_msm_wire(pts, sc, cpu_work_ratio=ratio, cpu_threads=4) == exp
    assert M.compute_msm_wire(pts, sc) == exp


def test_cocompute_split_host_path():
    """The GPU share large enough for the host-input slice pipeline (>= 2^18 points)."""
    n = (1 << 18) + 4099
    pts = M.gen_points(n, k0=2, step=3)
    sc = M.gen_scalars(n, seed=8)
    assert M.compute_msm_wire(pts, sc, cpu_work_ratio=0.015) == closed_form(2, 3, sc)


def test_cocompute_edges():
    empty_p, empty_s = np.zeros((0, 32), np.uint32), np.zeros((0, 8), np.uint32)
    assert M.compute_msm_wire(empty_p, empty_s, cpu_work_ratio=0.5) == (0, 1)
    pts = M.gen_points(1, k0=9, step=1)
    sc = M.gen_scalars(1, seed=2)
    exp = closed_form(9, 1, sc)
    for ratio in (0.5, 1.0, 3.0):  # share 0 (GPU only), then 1 = n (host only)
        assert M.compute_msm_wire(pts, sc, cpu_work_ratio=ratio) == exp


def test_cocompute_projective_inputs_and_errors():
    """Projective wire points (z != 1) on both sides of the split; a bad coordinate in the host
    share reports the same error as the device path."""
    n = 60
    rng = np.random.default_rng(12)
    ks = list(range(3, 3 + n))
    ss = [int(rng.integers(1, 2**63)) for _ in range(n)]
    pts = np.zeros((n, 32), np.uint32)
    for i, k in enumerate(ks):
        x, y = O.scalar_mul(O.G, k)
        z = int(rng.integers(2, 2**62)) if i % 3 else 1
        for j, v in enumerate((x * z % O.P, y * z % O.P, x * y % O.P * z % O.P, z)):
            pts[i, 8 * j: 8 * j + 8] = O.int_to_be_words(v)
    sw = O.ints_to_be_words(ss)
    exp = O.closed_form_msm(ks, ss)
    for ratio in (0.25, 0.5, 0.9):
        assert M.compute_msm_wire(pts, sw, cpu_work_ratio=ratio, cpu_threads=2) == exp
    bad = pts.copy()
    bad[4, 0:8] = O.int_to_be_words(O.P)  # inside the host share at ratio 0.5
    with pytest.raises(M.MsmError) as e:
        M.compute_msm_wire(bad, sw, cpu_work_ratio=0.5)
    assert e.value.code == -3


def test_cocompute_with_device_list():
    n = 20000
    pts = M.gen_points(n, k0=7, step=5)
    sc = M.gen_scalars(n, seed=4)
    ords = [M.load().msm_device_ordinal(0)]
    assert M.compute_msm_wire(pts, sc, devices=ords, cpu_work_ratio=0.05) == closed_form(7, 5, sc)


def test_compute_msm_objects_with_ratio():
    """compute_msm (BigIntPoint-like objects) forwards cpu_work_ratio."""
    n = 300
    pts = O.gen_points(n, k0=21, step=13)
    ss = O.xorshift_scalars(n, seed=77)
    objs = [{"x": O.be_words_to_int(pts[i, 0:8]), "y": O.be_words_to_int(pts[i, 8:16]),
             "t": O.be_words_to_int(pts[i, 16:24]), "z": O.be_words_to_int(pts[i, 24:32])} for i in range(n)]
    assert M.compute_msm(objs, ss, cpu_work_ratio=0.3) == O.closed_form_msm([21 + 13 * i for i in range(n)], ss)
