"""GPU parity of libmsm's launch paths added for host-resident inputs, shared base vectors
(prover batch), caller-stream ordering, serial launches and the captured-graph cache.

Every expected value is the closed form sum s_i (k_i G) = ((sum s_i k_i) mod r) G, which the
survey pinned to the Aleo-wasm oracle at 2^12..2^20 (tests/golden/msm_vectors.json); comparisons
are bit-exact.
"""
import os

import numpy as np
import pytest

import msm_amd as M
from _closed_form import as_xy, closed_form

pytestmark = pytest.mark.gpu


def _dev(a):
    import torch

    return torch.from_numpy(np.ascontiguousarray(a).view(np.int32)).cuda()


def test_host_entry_ragged_pieces():
    # msm_compute uploads points in 65536-point pieces, each prepared as it lands: three pieces,
    # the last one partial and not a multiple of the preparation workgroup
    n = 2 * 65536 + 77
    pts = M.gen_points(n, k0=5, step=3)
    sc = M.gen_scalars(n, seed=31)
    exp = closed_form(5, 3, sc)
    assert M.compute_msm_wire(pts, sc) == exp
    assert M.compute_msm_wire(pts, sc, window_size=13) == exp
    # an exact multiple of the piece
    n2 = 65536
    assert M.compute_msm_wire(pts[:n2], sc[:n2]) == closed_form(5, 3, sc[:n2])


@pytest.mark.parametrize("n", [2 * (1 << 17), 3 * (1 << 17), 3 * (1 << 17) + 2, (1 << 19) + 7])
def test_host_entry_split_into_slices(n):
    # (2^18: the one-launch path, just below the split) msm_compute from host arrays at n >= 3 x 2^17 runs G point-slices through the pipelined entry
    # (slice g+1 uploads while slice g computes) and joins the partials; n not a multiple of G
    # leaves the last slice short, padded on the device (identity points, zero scalars)
    pts = M.gen_points(n, k0=3, step=5)
    sc = M.gen_scalars(n, seed=41 + n % 7)
    exp = closed_form(3, 5, sc)
    assert M.compute_msm_wire(pts, sc) == exp
    part = M.compute_msm_partial(pts, sc)
    assert M.combine_partials(np.asarray(part, dtype=np.uint32).reshape(1, 32)) == exp


@pytest.mark.parametrize("first", [3, None])
def test_host_split_projective_points(first):
    # the split host path with projective points (z != 1, normalised by k_prepare_points) in one
    # launch's slices and in the short, device-padded last slice; z = 0 in another launch is still
    # rejected.  first=None: slice 0 of launch 0 is affine, so it goes up packed as x|y before
    # slice 1's z != 1 makes the launch repack both as x|y|z and send them again
    from oracle import oracle as O

    n = (1 << 19) + 5  # four slices in two launches, the last one short
    pts = M.gen_points(n, k0=9, step=7)
    sc = M.gen_scalars(n, seed=77)
    exp = closed_form(9, 7, sc)
    # projective points in launch 0 (slices 0 and 1) and at the end of the short last slice
    zs = [((1 << 17) + 11, 12345678901), (n - 1, O.P - 2)] + ([(first, 2)] if first is not None else [])
    for i, z in zs:
        x, y, t = (O.be_words_to_int(pts[i, 8 * j: 8 * j + 8]) for j in range(3))
        for j, v in enumerate((x * z % O.P, y * z % O.P, t * z % O.P, z)):
            pts[i, 8 * j: 8 * j + 8] = O.int_to_be_words(v)
    assert M.compute_msm_wire(pts, sc) == exp
    pts[(1 << 18) + 20, 24:32] = 0  # launch 1
    with pytest.raises(M.MsmError) as e:
        M.compute_msm_wire(pts, sc)
    assert e.value.code == -4
    # affine again: the same result
    assert M.compute_msm_wire(M.gen_points(n, k0=9, step=7), sc) == exp


def test_host_lone_pieces_mixed_formats():
    # the lone host path (n < 3 x 2^17) packs each 2^16-point piece on its own: x|y for the affine
    # pieces, x|y|z for a piece with some z != 1, each prepared in its format; t >= p anywhere is
    # still MSM_ERR_COORD_RANGE, and the next call is clean
    from oracle import oracle as O

    n = (1 << 17) + 777  # pieces 0, 1 full, piece 2 short
    pts = M.gen_points(n, k0=6, step=11)
    sc = M.gen_scalars(n, seed=19)
    exp = closed_form(6, 11, sc)
    for i, z in (((1 << 16) + 3, 99), (n - 1, O.P - 5)):  # pieces 1 and 2 projective, piece 0 affine
        x, y, t = (O.be_words_to_int(pts[i, 8 * j: 8 * j + 8]) for j in range(3))
        for j, v in enumerate((x * z % O.P, y * z % O.P, t * z % O.P, z)):
            pts[i, 8 * j: 8 * j + 8] = O.int_to_be_words(v)
    assert M.compute_msm_wire(pts, sc) == exp
    bad = pts.copy()
    bad[5, 16:24] = O.int_to_be_words(O.P)  # t = p in the affine piece
    with pytest.raises(M.MsmError) as e:
        M.compute_msm_wire(bad, sc)
    assert e.value.code == -3  # MSM_ERR_COORD_RANGE
    assert M.compute_msm_wire(pts, sc) == exp


@pytest.mark.parametrize("n", [1000, (1 << 19) + 5])
def test_t_is_checked_but_not_used(n):
    """Every entry derives d t from the affine x and y (the oracle reads only (x, y)): a record with
    an inconsistent t < p gives the same result, and t >= p is still MSM_ERR_COORD_RANGE -- on
    the device-resident entry and from host arrays, where the split path (n >= 3 x 2^17) uploads
    only x|y (packed by the library's threads) and checks t on the host."""
    pts = M.gen_points(n, k0=4, step=9)
    sc = M.gen_scalars(n, seed=5 + n % 3)
    exp = closed_form(4, 9, sc)
    bad_t = pts.copy()
    for i in (0, n // 2, n - 1):
        bad_t[i, 16:24] = np.uint32(0x01234567) ^ np.arange(8, dtype=np.uint32)  # t < p, not x y
    assert M.compute_msm_wire(bad_t, sc) == exp
    assert M.compute_msm_device(_dev(bad_t), _dev(sc), n) == exp
    # the host batch API packs the same way: three MSMs in one call, the bad t in the second
    many = M.compute_msm_many([pts, bad_t, pts], [sc, sc, sc], n)
    assert all(tuple(as_xy(r)) == tuple(exp) for r in many)
    over = pts.copy()
    over[n - 2, 16:24] = 0xFFFFFFFF  # t >= p
    for fn in (lambda: M.compute_msm_wire(over, sc), lambda: M.compute_msm_device(_dev(over), _dev(sc), n),
               lambda: M.compute_msm_many([pts, over, pts], [sc, sc, sc], n)):
        with pytest.raises(M.MsmError) as e:
            fn()
        assert e.value.code == -3
    assert M.compute_msm_wire(pts, sc) == exp  # recovers
    assert tuple(as_xy(M.compute_msm_many([pts], [sc], n)[0])) == tuple(exp)


def test_host_many_distinct():
    cases = []
    for j, n in enumerate((3000, 3000, 3000, 3000, 3000)):
        pts = M.gen_points(n, k0=2 + j, step=1 + j)
        sc = M.gen_scalars(n, seed=400 + j)
        cases.append((pts, sc, closed_form(2 + j, 1 + j, sc)))
    order = [0, 1, 2, 3, 4, 1, 0]
    out = M.compute_msm_many([cases[i][0] for i in order], [cases[i][1] for i in order], 3000)
    for r, i in zip(out, order):
        assert as_xy(r) == cases[i][2], i


def test_host_many_large_pieces():
    n = (1 << 17) + 5
    pts = [M.gen_points(n, k0=1 + j, step=2) for j in range(3)]
    scs = [M.gen_scalars(n, seed=500 + j) for j in range(3)]
    out = M.compute_msm_many(pts, scs, n)
    for j in range(3):
        assert as_xy(out[j]) == closed_form(1 + j, 2, scs[j])


def test_shared_base_vector_host_and_device():
    # the prover-batch entries: one base vector, prepared once per call, many scalar vectors
    n = 20000
    pts = M.gen_points(n, k0=7, step=5)
    scs = [M.gen_scalars(n, seed=600 + j) for j in range(7)]
    exps = [closed_form(7, 5, s) for s in scs]
    out = M.compute_msm_shared(pts, scs)
    for r, e in zip(out, exps):
        assert as_xy(r) == e
    d_pts = _dev(pts)
    d_scs = [_dev(s) for s in scs]
    out = M.compute_msm_shared_device(d_pts, d_scs, n)
    for r, e in zip(out, exps):
        assert as_xy(r) == e
    # mixed with the distinct-base entry on the same slots (different point-record buffers,
    # different captured segments) and a single MSM in between
    out = M.compute_msm_many_device([d_pts] * 3, d_scs[:3], n)
    for r, e in zip(out, exps[:3]):
        assert as_xy(r) == e
    assert M.compute_msm_device(d_pts, d_scs[4], n) == exps[4]
    out = M.compute_msm_shared_device(d_pts, d_scs[::-1], n)
    for r, e in zip(out, exps[::-1]):
        assert as_xy(r) == e
    # a count of one, and a bad point fails the whole call
    out = M.compute_msm_shared_device(d_pts, d_scs[:1], n)
    assert as_xy(out[0]) == exps[0]
    bad = pts.copy()
    bad[123, 8:16] = 0xFFFFFFFF  # y >= p
    with pytest.raises(M.MsmError) as e:
        M.compute_msm_shared(bad, scs[:3])
    assert e.value.code == -3
    out = M.compute_msm_shared(pts, scs[:2])  # recovers
    assert as_xy(out[1]) == exps[1]


@pytest.mark.parametrize("n", [1 << 18])
def test_shared_prover_batch_shape(n):
    # BASELINE configs[4] per rank: MSMs of 2^18 points over one base vector, distinct seeds
    d_pts = _dev(M.gen_points(n))
    scs = [M.gen_scalars(n, seed=M.XORSHIFT_SEED + b) for b in range(8)]
    out = M.compute_msm_shared_device(d_pts, [_dev(s) for s in scs], n)
    for b in range(8):
        assert as_xy(out[b]) == closed_form(1, 1, scs[b]), b


def test_graph_cache_keyed_on_whole_plan():
    # above 2^20 a lone MSM and a pipelined pair both use one MSM per launch and
    # c = 16 but different reduction chunk lengths (L = 8 vs 16); a replayed graph of the other
    # plan would read the window terms at the wrong offsets.  Alternate the two, twice.
    n = (1 << 20) + 1
    pts = M.gen_points(n)
    scs = [M.gen_scalars(n, seed=700 + j) for j in range(2)]
    exps = [closed_form(1, 1, s) for s in scs]
    d_pts = _dev(pts)
    d_scs = [_dev(s) for s in scs]
    for _ in range(2):
        assert M.compute_msm_device(d_pts, d_scs[0], n) == exps[0]
        out = M.compute_msm_many_device([d_pts, d_pts], d_scs, n)
        assert [as_xy(r) for r in out] == exps


def test_caller_stream_ordering():
    # inputs produced by torch kernels still in flight on a side stream: passing that stream
    # (or leaving the default: torch's current stream) orders libmsm after them
    import torch

    n = 1 << 16
    pts = M.gen_points(n, k0=3, step=2)
    sc = M.gen_scalars(n, seed=801)
    exp = closed_form(3, 2, sc)
    host_p = torch.from_numpy(pts.view(np.int32)).pin_memory()
    host_s = torch.from_numpy(sc.view(np.int32)).pin_memory()
    side = torch.cuda.Stream()
    for _ in range(3):
        with torch.cuda.stream(side):
            d_p = torch.zeros_like(host_p, device="cuda")
            d_s = torch.zeros_like(host_s, device="cuda")
            # a long chain of small kernels before the real data lands
            for _ in range(200):
                d_p.add_(1)
            d_p.copy_(host_p, non_blocking=True)
            d_s.copy_(host_s, non_blocking=True)
            assert M.compute_msm_device(d_p, d_s, n) == exp  # torch's current stream = side
        with torch.cuda.stream(side):
            d_s.zero_()
            d_s.copy_(host_s, non_blocking=True)
        assert M.compute_msm_device(d_p, d_s, n, stream=side.cuda_stream) == exp
        with torch.cuda.stream(side):
            d_s.zero_()
            d_s.copy_(host_s, non_blocking=True)
        out = M.compute_msm_many_device([d_p] * 2, [d_s] * 2, n, stream=side.cuda_stream)
        assert [as_xy(r) for r in out] == [exp, exp]
    # the default (null) stream too
    d_p = torch.zeros_like(host_p, device="cuda")
    d_s = torch.zeros_like(host_s, device="cuda")
    d_p.copy_(host_p, non_blocking=True)
    d_s.copy_(host_s, non_blocking=True)
    assert M.compute_msm_device(d_p, d_s, n) == exp


def test_serial_flag_and_profile():
    n = 1 << 16
    d_pts = _dev(M.gen_points(n))
    scs = [M.gen_scalars(n, seed=900 + j) for j in range(5)]
    exps = [closed_form(1, 1, s) for s in scs]
    M.set_profiling(2)
    try:
        out = M.compute_msm_many_device([d_pts] * 5, [_dev(s) for s in scs], n, flags=M.MSM_FLAG_SERIAL)
        prof = M.last_profile()
    finally:
        M.set_profiling(False)
    assert [as_xy(r) for r in out] == exps
    # every launch is timed (k_accumulate between two events)
    # 2^16: four MSMs per launch by default, so the five MSMs take two launches (the last one
    # padded); an MSM_BATCH override (the alternative-configuration reruns) changes the count
    per = prof["msms_per_launch"]
    assert prof["profiled"] == -(-5 // per)
    if "MSM_BATCH" not in os.environ:
        assert per == 4
    assert 0 < prof["accumulate_sum"] / prof["profiled"] < 50.0


def test_eight_msms_per_launch_small_sizes():
    # up to 2^16 a count that fills eight-MSM launches runs eight per launch (padding MSMs of a
    # short last launch otherwise); every result bit-exact
    n = (1 << 16) - 3
    d_pts = _dev(M.gen_points(n, k0=3, step=2))
    scs = [M.gen_scalars(n, seed=1300 + j) for j in range(16)]
    exps = [closed_form(3, 2, s) for s in scs]
    M.set_profiling(2)
    try:
        out = M.compute_msm_many_device([d_pts] * 16, [_dev(s) for s in scs], n, flags=M.MSM_FLAG_SERIAL)
        prof = M.last_profile()
    finally:
        M.set_profiling(False)
    assert [as_xy(r) for r in out] == exps
    if "MSM_BATCH" not in os.environ:  # (an MSM_BATCH override sets the launch size itself)
        assert prof["msms_per_launch"] == 8 and prof["profiled"] == 2
    out = M.compute_msm_many([M.gen_points(n, k0=3, step=2)] * 13, scs[:13], n)  # 13 % 8 > 4: eight
    assert [as_xy(r) for r in out] == exps[:13]


@pytest.mark.parametrize("count,per", [(18, 8), (12, 4)])
def test_small_size_batch_choice(count, per):
    # up to 2^16, eight per launch whenever its launches (the padded last one included) cost less
    # than four per launch: 18 MSMs -> 3 launches of eight (2 real in the last), 12 -> 3 of four
    n = 1 << 16
    d_pts = _dev(M.gen_points(n))
    scs = [M.gen_scalars(n, seed=1500 + j) for j in range(count)]
    exps = [closed_form(1, 1, s) for s in scs]
    M.set_profiling(2)
    try:
        out = M.compute_msm_many_device([d_pts] * count, [_dev(s) for s in scs], n, flags=M.MSM_FLAG_SERIAL)
        prof = M.last_profile()
    finally:
        M.set_profiling(False)
    assert [as_xy(r) for r in out] == exps
    if "MSM_BATCH" not in os.environ:
        assert prof["msms_per_launch"] == per and prof["profiled"] == -(-count // per)


def test_beyond_2_20_all_entries():
    # 2^21 + 17 points: one MSM per launch in the pipelined plan, L = 8 reduction for a lone MSM,
    # the host path as 16 slices, the last short and padded; device, pipelined and host entries agree with
    # the closed form
    n = (1 << 21) + 17
    pts = M.gen_points(n, k0=11, step=7)
    scs = [M.gen_scalars(n, seed=77 + j) for j in range(3)]
    exps = [closed_form(11, 7, s) for s in scs]
    d_pts = _dev(pts)
    d_sc = [_dev(s) for s in scs]
    import torch

    torch.cuda.synchronize()
    assert M.compute_msm_device(d_pts, d_sc[0], n) == exps[0]
    out = M.compute_msm_many_device([d_pts] * 3, d_sc, n)
    assert [as_xy(r) for r in out] == exps
    assert M.compute_msm_wire(pts, scs[1]) == exps[1]
