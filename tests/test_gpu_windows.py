"""Window ranges (msm_opts MSM_FLAG_WINDOWS, include/msm.h): an MSM restricted to signed-digit
windows [lo, hi) returns sum over those windows of 2^(offset w) G_w, so the partials of a partition
of the windows join (projective adds, msm_combine_partials) into the whole MSM -- the second way of
sharding one MSM over devices.  Every result is checked against the closed form
sum_i s_i (k_i G) = ((sum s_i k_i) mod r) G, including full 256-bit scalars (the overflow window).
Half-window ranges (MSM_FLAG_HALF_WINDOWS, (lo, hi, 2)) cut a window between the lower and upper
halves of its bucket magnitudes: their partitions join the same way."""
import numpy as np
import pytest

import msm_amd as M
from _closed_form import closed_form

pytestmark = pytest.mark.gpu


def _dev(a):
    import torch

    return torch.from_numpy(np.ascontiguousarray(a).view(np.int32)).cuda()


def _full_scalars(n, seed):
    rng = np.random.default_rng(seed)
    return rng.integers(0, 1 << 32, size=(n, 8), dtype=np.uint64).astype(np.uint32)  # 256-bit, not reduced


def _ranges(wm, cuts):
    edges = [0] + sorted(set(c for c in cuts if 0 < c < wm)) + [wm]
    return list(zip(edges[:-1], edges[1:]))


@pytest.mark.parametrize("n,c,cuts", [
    (1000, 10, [5, 12]),
    (70001, 13, [1, 2, 3, 10, 19]),
    ((1 << 18) + 5, 16, [4, 8, 12]),
    ((1 << 20), 16, [2, 4, 6, 8, 10, 12, 14]),
    ((1 << 17), 15, [9]),
])
@pytest.mark.parametrize("full", [False, True])
def test_window_partition_joins_to_msm(n, c, cuts, full):
    pts = M.gen_points(n, k0=3, step=7)
    sc = _full_scalars(n, n + c) if full else M.gen_scalars(n, seed=n + c)
    exp = closed_form(3, 7, sc)
    wm = M.window_count(c)
    rs = _ranges(wm, cuts)
    host = [M.compute_msm_partial(pts, sc, window_size=c, windows=r) for r in rs]
    assert M.combine_partials(np.stack(host)) == exp, rs
    dp, ds = _dev(pts), _dev(sc)
    dev = [M.compute_msm_device_partial(dp, ds, n, window_size=c, windows=r) for r in rs]
    assert M.combine_partials(np.stack(dev)) == exp, rs


@pytest.mark.parametrize("n,c,nr", [(1 << 17, 15, 4), ((1 << 19) + 3, 16, 2), (50000, 12, 3)])
def test_pipelined_window_ranges(n, c, nr):
    """The pipelined entry (several MSMs per launch, launches in flight) per window range: every
    range's K partials, joined per MSM, equal the K closed forms."""
    K = 5
    pts = M.gen_points(n, k0=1, step=1)
    scs = [M.gen_scalars(n, seed=900 + j) for j in range(K)]
    exps = [closed_form(1, 1, s) for s in scs]
    dp = _dev(pts)
    dss = [_dev(s) for s in scs]
    wm = M.window_count(c)
    edges = [round(wm * i / nr) for i in range(nr + 1)]
    parts = [M.compute_msm_many_device_partial([dp] * K, dss, n, window_size=c, windows=(edges[i], edges[i + 1]))
             for i in range(nr)]
    got = M.combine_partials_many(np.stack(parts))
    assert got == exps


def test_full_range_equals_plain_msm():
    n, c = 30000, 14
    pts, sc = M.gen_points(n, k0=2, step=3), M.gen_scalars(n, seed=4)
    wm = M.window_count(c)
    whole = M.compute_msm_partial(pts, sc, window_size=c, windows=(0, wm))
    assert M.combine_partials(whole.reshape(1, 32)) == M.compute_msm_wire(pts, sc, window_size=c) == closed_form(2, 3, sc)


@pytest.mark.parametrize("c,rng", [(0, (0, 2)), (16, (3, 3)), (16, (5, 2)), (16, (0, 18)), (13, (0, 99))])
def test_bad_window_ranges_rejected(c, rng):
    pts, sc = M.gen_points(64), M.gen_scalars(64)
    with pytest.raises(M.MsmError) as e:
        M.compute_msm_partial(pts, sc, window_size=c or None, windows=rng)
    assert e.value.code == -1


@pytest.mark.parametrize("n,c,cuts", [
    (1000, 10, [11]),                      # window 5 split in its middle
    (70001, 13, [1, 2, 7, 20, 39]),        # odd cuts everywhere, the overflow window halved too
    ((1 << 17) + 3, 15, [17]),             # the 8-GPU split's 8.5 / 8.5 windows
    ((1 << 18), 15, [9, 17, 26]),          # four half-window ranges
])
@pytest.mark.parametrize("full", [False, True])
def test_half_window_partition_joins_to_msm(n, c, cuts, full):
    pts = M.gen_points(n, k0=5, step=3)
    sc = _full_scalars(n, n + c + 1) if full else M.gen_scalars(n, seed=n + c + 1)
    exp = closed_form(5, 3, sc)
    wm = M.window_count(c)
    rs = [(lo, hi, 2) for lo, hi in _ranges(2 * wm, cuts)]
    host = [M.compute_msm_partial(pts, sc, window_size=c, windows=r) for r in rs]
    assert M.combine_partials(np.stack(host)) == exp, rs
    dp, ds = _dev(pts), _dev(sc)
    dev = [M.compute_msm_device_partial(dp, ds, n, window_size=c, windows=r) for r in rs]
    assert M.combine_partials(np.stack(dev)) == exp, rs
    # whole windows in half units (even edges): the whole MSM (affine; the projective form depends
    # on the order the atomics place a bucket's entries in)
    assert M.combine_partials(M.compute_msm_partial(pts, sc, window_size=c, windows=(0, 2 * wm, 2)).reshape(1, 32)) == exp


def test_pipelined_half_window_split():
    """The rank/device split's share: 2^17-point shards x the two half-window ranges of c = 15
    (msm_amd.dist.split_part), pipelined K MSMs per share, joined per MSM."""
    from msm_amd.dist import split_part

    n, K, world = 1 << 18, 5, 4
    pts = M.gen_points(n, k0=2, step=5)
    scs = [M.gen_scalars(n, seed=1200 + j) for j in range(K)]
    exps = [closed_form(2, 5, s) for s in scs]
    parts = []
    for rank in range(world):
        lo, hi, win, c = split_part(n, rank, world, "2x2")
        assert win is not None and len(win) == 3
        dp = _dev(pts[lo:hi])
        dss = [_dev(s[lo:hi]) for s in scs]
        parts.append(M.compute_msm_many_device_partial([dp] * K, dss, hi - lo, window_size=c, windows=win))
    assert M.combine_partials_many(np.stack(parts)) == exps


@pytest.mark.parametrize("rng", [(0, 37, 2), (5, 5, 2), (7, 3, 2), (0, 2, 3)])
def test_bad_half_window_ranges_rejected(rng):
    pts, sc = M.gen_points(64), M.gen_scalars(64)
    if rng[2] == 3:
        with pytest.raises(ValueError):
            M.compute_msm_partial(pts, sc, window_size=15, windows=rng)
        return
    with pytest.raises(M.MsmError) as e:
        M.compute_msm_partial(pts, sc, window_size=15, windows=rng)  # 2 * 18 = 36 half windows at c = 15
    assert e.value.code == -1
