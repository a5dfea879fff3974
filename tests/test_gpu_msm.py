"""Parity of libmsm's HIP path against the oracle (run on an MI355X: pytest -m gpu).

Integer work: every comparison is bit-exact.
"""
import numpy as np
import pytest

import msm_amd as M
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _case_inputs(case):
    ks = [int(k) for k in case["ks"]]
    ss = [int(s, 16) for s in case["scalars"]]
    pts = O.affine_to_wire([O.scalar_mul(O.G, k % O.R_ORDER) for k in ks])
    return pts, O.ints_to_be_words(ss), (int(case["x"]), int(case["y"]))


def _le_words(vals):
    return np.array([[(v >> (32 * i)) & 0xFFFFFFFF for i in range(8)] for v in vals], dtype=np.uint32)


def _from_le(row):
    return sum(int(w) << (32 * i) for i, w in enumerate(row))


def test_device_present():
    assert M.device_count() >= 1


def test_field_ops_random():
    rng = np.random.default_rng(7)
    n = 4096
    a = [int.from_bytes(rng.bytes(32), "little") % O.P for _ in range(n)]
    b = [int.from_bytes(rng.bytes(32), "little") % O.P for _ in range(n)]
    a[:4] = [0, 1, O.P - 1, O.P - 1]
    b[:4] = [0, O.P - 1, O.P - 1, 1]
    A, B = _le_words(a), _le_words(b)
    mul = M._test_field_op(0, A, B)
    add = M._test_field_op(1, A, B)
    sub = M._test_field_op(2, A, B)
    k2d = M._test_field_op(3, A, B)  # fe_mul_2d: 2d * a, the point add's small-constant multiply
    for i in range(n):
        assert _from_le(mul[i]) == a[i] * b[i] % O.P
        assert _from_le(add[i]) == (a[i] + b[i]) % O.P
        assert _from_le(sub[i]) == (a[i] - b[i]) % O.P
        assert _from_le(k2d[i]) == 6042 * a[i] % O.P


def test_signed_difference_multiply():
    """fe_mul_sd (pt_madd's products of signed differences) on the device: (a - b)(b - a) and
    (a - b)(a + b) mod p for random operands and the edge values, bit-exact against Python."""
    rng = np.random.default_rng(23)
    a = [int.from_bytes(rng.bytes(32), "little") % O.P for _ in range(4096)]
    b = [int.from_bytes(rng.bytes(32), "little") % O.P for _ in range(4096)]
    edge = [0, 1, 2, O.P - 1, O.P - 2, (O.P - 1) // 2, 1 << 252]
    for x in edge:
        for y in edge:
            a.append(x)
            b.append(y)
    A, B = _le_words(a), _le_words(b)
    neg_sq = M._test_field_op(4, A, B)
    diff_sq = M._test_field_op(5, A, B)
    for i in range(len(a)):
        assert _from_le(neg_sq[i]) == -(a[i] - b[i]) ** 2 % O.P, i
        assert _from_le(diff_sq[i]) == (a[i] * a[i] - b[i] * b[i]) % O.P, i


def test_point_ops_vs_oracle(golden):
    rng = np.random.default_rng(3)
    ks = [int(rng.integers(1, 2**62)) for _ in range(64)]
    ps = [O.scalar_mul(O.G, k) for k in ks]
    qs = [O.scalar_mul(O.G, k * 3 + 1) for k in ks]
    qs[0] = ps[0]            # doubling through the unified add
    qs[1] = O.IDENTITY       # identity operand
    qs[2] = O.aff_neg(ps[2])  # P + (-P) = identity
    for x, _, _ in golden["kats"]["add_points_x"]["cases"][:2]:
        ps.append(O.point_from_x(int(x)))
        qs.append(O.point_from_x(int(x)))
    P_ = np.concatenate([_le_words([p[0] for p in ps]), _le_words([p[1] for p in ps])], axis=1)
    Q_ = np.concatenate([_le_words([q[0] for q in qs]), _le_words([q[1] for q in qs])], axis=1)
    for op in (0, 1, 2, 3):  # 3: quad-cooperative add (pt_add_quad)
        out = M._test_point_op(op, P_, Q_)
        for i in range(len(ps)):
            X, Y, T, Z = (_from_le(out[i, 8 * j: 8 * j + 8]) for j in range(4))
            zi = O.inv(Z)
            got = (X * zi % O.P, Y * zi % O.P)
            exp = O.aff_add(ps[i], ps[i]) if op == 2 else O.aff_add(ps[i], qs[i])
            assert got == exp, (op, i)
            assert X * Y % O.P == T * Z % O.P  # extended-coordinate invariant


def test_small_vectors_default_window(golden):
    for case in golden["msm"]["small"]:
        pts, sc, exp = _case_inputs(case)
        assert M.compute_msm_wire(pts, sc) == exp, case["name"]


@pytest.mark.parametrize("window", [4, 5, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 20])
def test_small_vectors_all_windows(golden, window):
    for case in golden["msm"]["small"]:
        if case["n"] > 600 and window < 8:
            continue
        pts, sc, exp = _case_inputs(case)
        assert M.compute_msm_wire(pts, sc, window_size=window) == exp, (case["name"], window)


@pytest.mark.parametrize("run_length", [1, 2, 3, 7, 32, 100, 1000])
def test_run_lengths(golden, run_length):
    # run boundaries inside / across buckets; K = 1 makes every bucket straddle runs
    for name in ("all_equal_scalars", "all_equal_points", "random_mod_p_1000", "repeated_digit_blocks"):
        case = next(c for c in golden["msm"]["small"] if c["name"] == name)
        pts, sc, exp = _case_inputs(case)
        assert M.compute_msm_wire(pts, sc, window_size=12, run_length=run_length) == exp, (name, run_length)


def test_empty_and_zero():
    assert M.compute_msm_wire(np.zeros((0, 32), np.uint32), np.zeros((0, 8), np.uint32)) == (0, 1)
    pts = O.gen_points(10)
    assert M.compute_msm_wire(pts, np.zeros((10, 8), np.uint32)) == (0, 1)


def test_length_mismatch_zips_to_shorter():
    pts = O.gen_points(12)
    ss = O.xorshift_scalars(9)
    assert M.compute_msm_wire(pts, O.ints_to_be_words(ss)) == O.closed_form_msm(range(1, 10), ss)


def test_bigint_and_u32_inputs_agree():
    n = 33
    pts = O.gen_points(n, k0=5, step=3)
    ss = O.xorshift_scalars(n, seed=99)
    exp = O.closed_form_msm([5 + 3 * i for i in range(n)], ss)
    big = [{k: O.be_words_to_int(pts[i, 8 * j: 8 * j + 8]) for j, k in enumerate("xytz")} for i in range(n)]
    assert M.compute_msm(big, ss) == exp
    u32 = [{k: pts[i, 8 * j: 8 * j + 8] for j, k in enumerate("xytz")} for i in range(n)]
    assert M.compute_msm(u32, [O.ints_to_be_words([s])[0] for s in ss]) == exp


def test_projective_inputs_z_not_one():
    n = 40
    rng = np.random.default_rng(5)
    ks = list(range(7, 7 + n))
    ss = [int(rng.integers(1, 2**63)) for _ in range(n)]
    pts = np.zeros((n, 32), np.uint32)
    for i, k in enumerate(ks):
        x, y = O.scalar_mul(O.G, k)
        z = int(rng.integers(2, 2**62)) if i % 3 else 1
        X, Y = x * z % O.P, y * z % O.P
        T = x * y % O.P * z % O.P
        for j, v in enumerate((X, Y, T, z)):
            pts[i, 8 * j: 8 * j + 8] = O.int_to_be_words(v)
    assert M.compute_msm_wire(pts, O.ints_to_be_words(ss)) == O.closed_form_msm(ks, ss)


def test_coordinate_out_of_range_rejected():
    pts = O.gen_points(4)
    pts[2, 8:16] = O.int_to_be_words(O.P + 1)
    with pytest.raises(M.MsmError) as e:
        M.compute_msm_wire(pts, O.ints_to_be_words([1, 2, 3, 4]))
    assert e.value.code == -3


def test_z_zero_rejected():
    pts = O.gen_points(4)
    pts[1, 24:32] = 0
    with pytest.raises(M.MsmError) as e:
        M.compute_msm_wire(pts, O.ints_to_be_words([1, 2, 3, 4]))
    assert e.value.code == -4


def test_unsupported_window():
    pts = O.gen_points(4)
    with pytest.raises(M.MsmError) as e:
        M.compute_msm_wire(pts, O.ints_to_be_words([1, 2, 3, 4]), window_size=21)
    assert e.value.code == -2


def test_non_subgroup_points_full_scalar_semantics():
    # The reference's Rust path multiplies by the full 256-bit scalar (no reduction mod r); for
    # points outside the r-torsion subgroup only the C restatement of lib.rs can check that.
    n = 300
    rng = np.random.default_rng(11)
    pts = []
    x = 5
    while len(pts) < n:
        x += 1
        x2 = x * x % O.P
        y = O.sqrt_mod((O.EDWARDS_A * x2 - 1) * O.inv(O.EDWARDS_D * x2 - 1))
        if y is not None:
            pts.append((x, y))
    wire = O.affine_to_wire(pts)
    sc = O.ints_to_be_words([int.from_bytes(rng.bytes(32), "big") for _ in range(n)])
    assert M.compute_msm_wire(wire, sc) == O.msm(wire, sc, window=12, threads=4)


@pytest.mark.parametrize("logn", [12, 16])
def test_survey_rows(golden, logn):
    row = {r["n"]: r for r in golden["msm"]["survey"]}[1 << logn]
    pts = O.gen_points(1 << logn)
    sc = O.xorshift_scalars_np(1 << logn)
    exp = (int(row["x"]), int(row["y"]))
    assert M.compute_msm_wire(pts, sc) == exp
    assert M.compute_msm_wire(pts, sc, window_size=16) == exp  # BASELINE config 2 (c = 16)


@pytest.mark.parametrize("logn", [17, 18, 19, 20])
def test_closed_form_rows_pipelined(golden, logn):
    # the bench's sizes through the pipelined entry (two MSMs per launch, throughput window; at
    # 2^20 also the 16-bucket reduction chunks of the pipelined plan)
    torch = pytest.importorskip("torch")
    row = {r["n"]: r for r in golden["msm"]["closed_form"] + golden["msm"]["survey"]}[1 << logn]
    n = row["n"]
    d_pts = torch.from_numpy(M.gen_points(n).view(np.int32)).cuda()
    d_sc = torch.from_numpy(M.gen_scalars(n).view(np.int32)).cuda()
    out = M.compute_msm_many_device([d_pts] * 3, [d_sc] * 3, n)
    for r in out:
        assert (O.be_words_to_int(r[:8]), O.be_words_to_int(r[8:])) == (int(row["x"]), int(row["y"]))


def test_many_device_skewed_2_20():
    # the pipelined 2^20 plan (16-bucket reduction chunks) under bucket skew: giant buckets drive
    # the chain / lead / cross-workgroup joins that feed k_bucket_reduce_1
    torch = pytest.importorskip("torch")
    n = 1 << 20
    d_pts = torch.from_numpy(M.gen_points(n).view(np.int32)).cuda()
    s = 0x0DEADBEEF1234567_89ABCDEF0FEDCBA9_8765432112345678_9ABCDEF011223344 % O.P
    vals = [s, 3 * s % O.P, (1 << 190) + 12345]
    eq = np.tile(O.ints_to_be_words([s]), (n, 1))
    few = np.tile(O.ints_to_be_words(vals), (n // 3 + 1, 1))[:n]
    exp_eq = O.scalar_mul(O.G, s * (n * (n + 1) // 2) % O.R_ORDER)
    exp_few = O.scalar_mul(O.G, sum(v * sum(range(j + 1, n + 1, 3)) for j, v in enumerate(vals)) % O.R_ORDER)
    d_eq = torch.from_numpy(eq.view(np.int32)).cuda()
    d_few = torch.from_numpy(np.ascontiguousarray(few).view(np.int32)).cuda()
    out = M.compute_msm_many_device([d_pts] * 4, [d_eq, d_few, d_few, d_eq], n)
    for r, exp in zip(out, (exp_eq, exp_few, exp_few, exp_eq)):
        assert (O.be_words_to_int(r[:8]), O.be_words_to_int(r[8:])) == exp


def test_survey_2_20(golden):
    row = {r["n"]: r for r in golden["msm"]["survey"]}[1 << 20]
    pts = O.gen_points(1 << 20)
    sc = O.xorshift_scalars_np(1 << 20)
    assert M.compute_msm_wire(pts, sc) == (int(row["x"]), int(row["y"]))


def test_c_oracle_agrees_at_2_16_random_full_scalars():
    n = 1 << 16
    rng = np.random.default_rng(2024)
    pts = O.gen_points(n, k0=987654321, step=12345)
    sc = rng.integers(0, 2**32, size=(n, 8), dtype=np.uint64).astype(np.uint32)
    assert M.compute_msm_wire(pts, sc, window_size=16) == O.msm(pts, sc, window=16, threads=16)


def test_partials_and_combine():
    n = 5000
    pts = O.gen_points(n, k0=3, step=7)
    ss = O.xorshift_scalars(n, seed=5)
    sc = O.ints_to_be_words(ss)
    exp = O.closed_form_msm([3 + 7 * i for i in range(n)], ss)
    parts = np.stack([M.compute_msm_partial(pts[a:b], sc[a:b]) for a, b in ((0, 1234), (1234, 4000), (4000, n))])
    assert M.combine_partials(parts) == exp


def test_device_resident_entry():
    torch = pytest.importorskip("torch")
    n = 3000
    pts = O.gen_points(n, k0=2, step=5)
    ss = O.xorshift_scalars(n, seed=8)
    exp = O.closed_form_msm([2 + 5 * i for i in range(n)], ss)
    dp = torch.from_numpy(pts.view(np.int32)).cuda()
    ds = torch.from_numpy(O.ints_to_be_words(ss).view(np.int32)).cuda()
    torch.cuda.synchronize()
    assert M.compute_msm_device(dp, ds, n) == exp
    stream = torch.cuda.current_stream().cuda_stream
    assert M.compute_msm_device(dp, ds, n, stream=stream) == exp
    out = M.compute_msm_batch_device(torch.cat([dp, dp]), torch.cat([ds, ds]), n, 2)
    for r in out:
        assert (O.be_words_to_int(r[:8]), O.be_words_to_int(r[8:])) == exp


# --- skewed scalars: buckets that hold many accumulation runs (the reference's tree schedule,
# gpu.ts:181-221, handles bucket-occupancy skew in O(log N) rounds; so must we) ---------------
@pytest.mark.parametrize("n,run_length", [(20000, 1), (20000, 4), (1 << 16, 0), (1 << 18, 0)])
def test_all_equal_scalars_giant_buckets(n, run_length):
    import time

    pts = O.gen_points(n, k0=11, step=1)
    s = 0x0DEADBEEF1234567_89ABCDEF0FEDCBA9_8765432112345678_9ABCDEF011223344 % O.P
    sc = O.ints_to_be_words([s] * n)
    exp = O.closed_form_msm(range(11, 11 + n), [s] * n)
    M.compute_msm_wire(pts, sc, run_length=run_length or None)  # warm (graph capture, allocation)
    t0 = time.perf_counter()
    got = M.compute_msm_wire(pts, sc, run_length=run_length or None)
    dt = time.perf_counter() - t0
    assert got == exp
    # one bucket per window holds every point: must stay logarithmic, not O(runs) serial adds
    assert dt < 0.05, f"skewed MSM took {dt * 1e3:.1f} ms"


def test_few_distinct_scalars():
    n = 50000
    rng = np.random.default_rng(7)
    vals = [int(v) for v in rng.integers(1, 2**62, size=3)]
    ss = [vals[i % 3] * (2**190 + 12345) % O.P for i in range(n)]
    pts = O.gen_points(n, k0=1000, step=3)
    exp = O.closed_form_msm([1000 + 3 * i for i in range(n)], ss)
    for K in (None, 2, 64):
        assert M.compute_msm_wire(pts, O.ints_to_be_words(ss), run_length=K) == exp, K


def test_small_scalars_sparse_windows():
    # only the lowest window is populated; all higher windows are empty
    n = 30000
    ss = [(i * 7919) % 60000 for i in range(n)]
    pts = O.gen_points(n, k0=5, step=2)
    exp = O.closed_form_msm([5 + 2 * i for i in range(n)], ss)
    assert M.compute_msm_wire(pts, O.ints_to_be_words(ss)) == exp
    assert M.compute_msm_wire(pts, O.ints_to_be_words(ss), window_size=16) == exp


def test_many_device_pipelined_distinct_inputs():
    # msm_compute_many_device keeps two MSMs in flight (device runs b+1 while the host finishes b);
    # every result must still be its own MSM's
    torch = pytest.importorskip("torch")
    n = 4096
    cases = []
    for j in range(5):
        pts = O.gen_points(n, k0=3 + j, step=2 + j)
        ss = O.xorshift_scalars(n, seed=100 + j)
        exp = O.closed_form_msm([3 + j + (2 + j) * i for i in range(n)], ss)
        cases.append((torch.from_numpy(pts.view(np.int32)).cuda(),
                      torch.from_numpy(O.ints_to_be_words(ss).view(np.int32)).cuda(), exp))
    torch.cuda.synchronize()
    order = [0, 1, 2, 3, 4, 2, 0, 4]
    out = M.compute_msm_many_device([cases[i][0] for i in order], [cases[i][1] for i in order], n)
    for r, i in zip(out, order):
        assert (O.be_words_to_int(r[:8]), O.be_words_to_int(r[8:])) == cases[i][2], i
    # interleaved with single calls (slot rotation) and a different size (re-plan, re-capture)
    assert M.compute_msm_device(cases[3][0], cases[3][1], n) == cases[3][2]
    small = M.compute_msm_many_device([cases[1][0]], [cases[1][1]], 100)
    assert (O.be_words_to_int(small[0][:8]), O.be_words_to_int(small[0][8:])) == \
        O.closed_form_msm([4 + 3 * i for i in range(100)], O.xorshift_scalars(100, seed=101))


@pytest.mark.parametrize("n,c", [(1 << 16, 14), (1 << 17, 15), ((7 << 16) - 1, 15), (7 << 16, 16)])
def test_many_device_throughput_window(n, c):
    # below 2^20 the pipelined entry picks a narrower window than a lone MSM (c = 14 at 2^16,
    # 15 at 2^17, 16 from 7/8 of 2^19: msm_host.hip pipelined_window); results must not depend on it
    torch = pytest.importorskip("torch")
    d_pts = torch.from_numpy(O.gen_points(n, k0=1, step=1).view(np.int32)).cuda()
    scs, exps = [], []
    for j in range(4):
        ss = O.xorshift_scalars(n, seed=700 + j)
        scs.append(torch.from_numpy(O.ints_to_be_words(ss).view(np.int32)).cuda())
        exps.append(O.closed_form_msm(range(1, n + 1), ss))
    torch.cuda.synchronize()
    M.set_profiling(2)  # records the plan of the bracketed (first) MSM
    try:
        out = M.compute_msm_many_device([d_pts] * 4, scs, n)
        prof = M.last_profile()
    finally:
        M.set_profiling(False)
    assert prof["window_bits"] == c
    for r, exp in zip(out, exps):
        assert (O.be_words_to_int(r[:8]), O.be_words_to_int(r[8:])) == exp
    assert M.compute_msm_device(d_pts, scs[0], n) == exps[0]  # lone MSM: c = 16


def test_many_device_odd_count_and_bad_member():
    # the pipelined entry launches MSMs two at a time: an odd count pads the last launch (its
    # extra result is dropped), and a bad input anywhere in a launch fails the call
    torch = pytest.importorskip("torch")
    n = 3000
    cases = []
    for j in range(3):
        pts = O.gen_points(n, k0=5 + j, step=1 + j)
        ss = O.xorshift_scalars(n, seed=900 + j)
        cases.append((torch.from_numpy(pts.view(np.int32)).cuda(),
                      torch.from_numpy(O.ints_to_be_words(ss).view(np.int32)).cuda(),
                      O.closed_form_msm([5 + j + (1 + j) * i for i in range(n)], ss)))
    torch.cuda.synchronize()
    out = M.compute_msm_many_device([c[0] for c in cases], [c[1] for c in cases], n)
    assert out.shape == (3, 16)
    for r, c in zip(out, cases):
        assert (O.be_words_to_int(r[:8]), O.be_words_to_int(r[8:])) == c[2]
    bad = O.gen_points(n, k0=5, step=1)
    bad[17, :8] = O.int_to_be_words(O.P + 3)  # x >= p
    d_bad = torch.from_numpy(bad.view(np.int32)).cuda()
    with pytest.raises(M.MsmError):
        M.compute_msm_many_device([cases[0][0], d_bad, cases[2][0]], [c[1] for c in cases], n)
    # the library recovers: the next call is correct
    out = M.compute_msm_many_device([cases[1][0]] * 2, [cases[1][1]] * 2, n)
    assert (O.be_words_to_int(out[1][:8]), O.be_words_to_int(out[1][8:])) == cases[1][2]


def test_unpacked_partition_entries():
    # coarse-binned entries carry their fine key in one u32 while the launch's points fit in
    # 2^(31 - fb) (msm_dev.h MsmDims::packed); c = 20 (fb = 11) with two MSMs of 2^19 + 3 points
    # per launch does not fit, so the two-array path runs
    torch = pytest.importorskip("torch")
    n = (1 << 19) + 3
    d_pts = torch.from_numpy(O.gen_points(n, k0=2, step=3).view(np.int32)).cuda()
    scs, exps = [], []
    for j in range(2):
        ss = O.xorshift_scalars(n, seed=1300 + j)
        scs.append(torch.from_numpy(O.ints_to_be_words(ss).view(np.int32)).cuda())
        exps.append(O.closed_form_msm(range(2, 2 + 3 * n, 3), ss))
    torch.cuda.synchronize()
    out = M.compute_msm_many_device([d_pts] * 2, scs, n, window_size=20)
    for r, exp in zip(out, exps):
        assert (O.be_words_to_int(r[:8]), O.be_words_to_int(r[8:])) == exp


def test_reference_format_test_case(tmp_path):
    # a case written in the reference's on-disk format (testCases.ts:34-52), z != 1 included
    from msm_amd import testdata as TD

    n = 3000
    quads, ks = [], [11 + 7 * i for i in range(n)]
    base = O.gen_points(n, k0=11, step=7)
    for i in range(n):
        x, y = O.be_words_to_int(base[i, :8]), O.be_words_to_int(base[i, 8:16])
        z = 1 + (i % 5)
        quads.append((x * z % O.P, y * z % O.P, x * y % O.P * z % O.P, z))
    ss = O.xorshift_scalars(n, seed=4242)
    pp, sp = str(tmp_path / "p.txt"), str(tmp_path / "s.txt")
    TD.write_test_case(pp, sp, quads, ss)
    pts, sc = TD.load_test_case(pp, sp)
    assert M.compute_msm_wire(pts, sc) == O.closed_form_msm(ks, ss)


def test_many_device_just_past_2p20():
    """Pipelined launches of two MSMs of 2^20 + 3 points (two per launch up to 2^21)."""
    torch = pytest.importorskip("torch")
    import msm_amd as M
    from _closed_form import closed_form

    n = (1 << 20) + 3
    d_pts = torch.from_numpy(M.gen_points(n, k0=2, step=3).view(np.int32)).cuda()
    scs = [M.gen_scalars(n, seed=900 + j) for j in range(3)]
    d_scs = [torch.from_numpy(s.view(np.int32)).cuda() for s in scs]
    torch.cuda.synchronize()
    out = M.compute_msm_many_device([d_pts] * 3, d_scs, n)
    for r, s in zip(out, scs):
        assert (O.be_words_to_int(r[:8]), O.be_words_to_int(r[8:])) == closed_form(2, 3, s)
