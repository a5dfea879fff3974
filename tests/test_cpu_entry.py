"""msm_compute_cpu: libmsm's own host Pippenger (the reference's CPU-only path, cpuWorkRatio = 1 ->
msm_end_to_end, lib.rs:106-121).  Runs without a GPU; checked against the oracle (C restatement
and closed form)."""
import numpy as np
import pytest

import msm_amd as M
from _closed_form import closed_form
from oracle import oracle as O


def test_cpu_entry_closed_form_sizes():
    for n, seed in ((1, 1), (2, 2), (255, 3), (4097, 4), (30000, 5)):
        pts = M.gen_points(n, k0=3, step=7)
        sc = M.gen_scalars(n, seed=seed)
        assert M.compute_msm_cpu(pts, sc, threads=4) == closed_form(3, 7, sc), n


@pytest.mark.parametrize("window", [4, 7, 12, 16])
def test_cpu_entry_full_scalars_vs_c_oracle(window):
    rng = np.random.default_rng(window)
    n = 700
    pts = M.gen_points(n, k0=11, step=3)
    sc = rng.integers(0, 2**32, size=(n, 8), dtype=np.uint64).astype(np.uint32)  # full 256-bit
    assert M.compute_msm_cpu(pts, sc, window_size=window, threads=3) == O.msm(pts, sc, window=10, threads=2)


def test_cpu_entry_edges():
    assert M.compute_msm_cpu(np.zeros((0, 32), np.uint32), np.zeros((0, 8), np.uint32)) == (0, 1)
    n = 40
    rng = np.random.default_rng(5)
    ks = list(range(7, 7 + n))
    ss = [int(rng.integers(1, 2**63)) for _ in range(n)]
    pts = np.zeros((n, 32), np.uint32)
    for i, k in enumerate(ks):  # projective inputs, z != 1 on two thirds of them
        x, y = O.scalar_mul(O.G, k)
        z = int(rng.integers(2, 2**62)) if i % 3 else 1
        for j, v in enumerate((x * z % O.P, y * z % O.P, x * y % O.P * z % O.P, z)):
            pts[i, 8 * j: 8 * j + 8] = O.int_to_be_words(v)
    assert M.compute_msm_cpu(pts, O.ints_to_be_words(ss)) == O.closed_form_msm(ks, ss)
    bad = pts.copy()
    bad[3, 0:8] = O.int_to_be_words(O.P)
    with pytest.raises(M.MsmError) as e:
        M.compute_msm_cpu(bad, O.ints_to_be_words(ss))
    assert e.value.code == -3
    bad = pts.copy()
    bad[5, 24:32] = 0
    with pytest.raises(M.MsmError) as e:
        M.compute_msm_cpu(bad, O.ints_to_be_words(ss))
    assert e.value.code == -4
    with pytest.raises(M.MsmError) as e:
        M.compute_msm_cpu(pts, O.ints_to_be_words(ss), window_size=21)
    assert e.value.code == -2
