"""Seeded random sweep of libmsm's entry points: sizes from 1 to 2^19 (log-uniform, ragged; the
MSM_SWEEP_* variables below run other seeds, counts and sizes),
explicit or automatic window widths 4..20, run lengths, host / device / pipelined / shared-base
entries, batch counts and split partials, every result bit-exact against the closed form
sum s_i (k_i G) = ((sum s_i k_i) mod r) G over P_i = (k0 + i step) G (tests/_closed_form.py; pinned to the Aleo-wasm oracle
through tests/golden).  Complements the targeted cases of test_gpu_msm.py / test_gpu_paths.py
with plan combinations nobody picked by hand.
"""
import numpy as np
import pytest

import msm_amd as M
from _closed_form import as_xy, closed_form

pytestmark = pytest.mark.gpu

import os

# MSM_SWEEP_SEED / MSM_SWEEP_CASES run a different or longer sweep (profiles/r5/random_sweep_*.txt)
SEED = int(os.environ.get("MSM_SWEEP_SEED", "20261016"))
N_CASES = int(os.environ.get("MSM_SWEEP_CASES", "120"))
MAX_LOG = int(os.environ.get("MSM_SWEEP_MAXLOG", "19"))  # sizes up to 2^MAX_LOG


def _cases():
    rng = np.random.default_rng(SEED)
    out = []
    for i in range(N_CASES):
        n = int(np.exp(rng.uniform(0, np.log(1 << MAX_LOG))))
        window = int(rng.choice([0, 0, 4, 7, 9, 11, 13, 14, 15, 16, 17, 20]))
        if window and n > (1 << 17) and window < 9:
            window = 0  # keep the number of narrow windows (and the runtime) bounded
        run_length = int(rng.choice([0, 0, 0, 1, 4, 16, 64]))
        entry = str(rng.choice(["host", "device", "many_device", "many_host", "shared_device", "shared_host",
                                "partial"]))
        count = int(rng.integers(1, 6)) if entry.startswith(("many", "shared")) else 1
        if entry in ("many_host", "shared_host"):
            n = min(n, 1 << 17)
        out.append(dict(n=max(1, n), window=window or None, run_length=run_length or None, entry=entry,
                        count=count, k0=int(rng.integers(1, 1000)), step=int(rng.integers(1, 50)),
                        seed=int(rng.integers(1, 2**62))))
    return out


def _dev(a):
    import torch

    return torch.from_numpy(np.ascontiguousarray(a).view(np.int32)).cuda()


@pytest.mark.parametrize("case", _cases(), ids=lambda c: f"{c['entry']}-n{c['n']}-w{c['window']}-k{c['run_length']}")
def test_random_plan(case):
    n, w, k = case["n"], case["window"], case["run_length"]
    pts = M.gen_points(n, k0=case["k0"], step=case["step"])
    scs = [M.gen_scalars(n, seed=case["seed"] + j) for j in range(case["count"])]
    exps = [closed_form(case["k0"], case["step"], s) for s in scs]
    if case["entry"] == "host":
        assert M.compute_msm_wire(pts, scs[0], window_size=w, run_length=k) == exps[0]
    elif case["entry"] == "device":
        import torch

        d_pts, d_sc = _dev(pts), _dev(scs[0])
        torch.cuda.synchronize()
        assert M.compute_msm_device(d_pts, d_sc, n, window_size=w, run_length=k) == exps[0]
    elif case["entry"] == "many_device":
        import torch

        d_pts = _dev(pts)
        d_scs = [_dev(s) for s in scs]
        torch.cuda.synchronize()
        out = M.compute_msm_many_device([d_pts] * len(scs), d_scs, n, window_size=w, run_length=k)
        for j, exp in enumerate(exps):
            assert as_xy(out[j]) == exp, j
    elif case["entry"] == "many_host":
        out = M.compute_msm_many([pts] * len(scs), scs, n, window_size=w, run_length=k)
        for j, exp in enumerate(exps):
            assert as_xy(out[j]) == exp, j
    elif case["entry"] == "shared_device":
        import torch

        d_pts = _dev(pts)
        d_scs = [_dev(s) for s in scs]
        torch.cuda.synchronize()
        out = M.compute_msm_shared_device(d_pts, d_scs, n, window_size=w, run_length=k)
        for j, exp in enumerate(exps):
            assert as_xy(out[j]) == exp, j
    elif case["entry"] == "shared_host":
        out = M.compute_msm_shared(pts, scs, n, window_size=w, run_length=k)
        for j, exp in enumerate(exps):
            assert as_xy(out[j]) == exp, j
    else:  # projective partial of the two halves, joined on the host (the multi-GPU identity)
        h = n // 2
        parts = [M.compute_msm_partial(pts[a:b], scs[0][a:b], window_size=w)
                 for a, b in ((0, h), (h, n)) if b > a]
        assert M.combine_partials(np.asarray(parts, dtype=np.uint32).reshape(-1, 32)) == exps[0]
