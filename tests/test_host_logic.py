"""Host-side marshalling and the TypeScript/JS surface (node), CPU only."""
import ctypes
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

import msm_amd as M
from oracle import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JS = os.path.join(ROOT, "webgpu-msm_amd", "js", "submission.mjs")
NODE = shutil.which("node")


def test_points_to_wire_forms_agree(golden):
    pts = O.gen_points(20, k0=4)
    as_int = [{k: O.be_words_to_int(pts[i, 8 * j: 8 * j + 8]) for j, k in enumerate("xytz")} for i in range(20)]
    as_tuple = [tuple(p[k] for k in "xytz") for p in as_int]
    as_u32 = [{k: pts[i, 8 * j: 8 * j + 8].copy() for j, k in enumerate("xytz")} for i in range(20)]
    for form in (as_int, as_tuple, as_u32, pts):
        assert np.array_equal(M.points_to_wire(form), pts)
    assert M.points_to_wire([]).shape == (0, 32)


def test_scalars_to_wire_limb_order(golden):
    cases = golden["kats"]["be_limbs"]["cases"]
    vals = [int(v) for v, _ in cases]
    w = M.scalars_to_wire(vals)
    assert w.tolist() == [words for _, words in cases]
    assert np.array_equal(M.scalars_to_wire([np.array(x, np.uint32) for _, x in cases]), w)
    with pytest.raises(ValueError):
        M.scalars_to_wire([1 << 256])
    assert M.wire_to_int(w[4]) == O.P


def _node(script):
    out = subprocess.run([NODE, "--input-type=module", "-e", script], capture_output=True, text=True, timeout=120,
                         cwd=os.path.dirname(JS))
    assert out.returncode == 0, out.stderr
    return out.stdout


@pytest.mark.skipif(NODE is None, reason="node not installed")
def test_js_surface_helpers(golden):
    cases = golden["kats"]["be_limbs"]["cases"]
    script = f"""
import * as m from {json.dumps(JS)};
const cases = {json.dumps(cases)};
const res = {{}};
res.limbs = cases.map(([v, w]) => m.u32ArrayToBigInts(new Uint32Array(w))[0].toString() === v);
res.best = [1<<16, 1<<20].map((n) => m.getBestWindowSize(n));
const sc = new Uint32Array([0x12345678, 0x9abcdef0, 1, 2, 3, 4, 5, 0xffffffff]);
res.split = Array.from(m.split_dynamic(13, sc));
console.log(JSON.stringify(res));
"""
    res = json.loads(_node(script))
    assert all(res["limbs"])
    assert res["best"] == [M.get_best_window_size(1 << 16), M.get_best_window_size(1 << 20)]
    sc = np.array([0x12345678, 0x9ABCDEF0, 1, 2, 3, 4, 5, 0xFFFFFFFF], np.uint32)
    assert res["split"] == O.split(13, sc).tolist()


@pytest.mark.skipif(NODE is None, reason="node not installed")
def test_js_point_add_affine(golden):
    a, b, exp = golden["kats"]["add_points_x"]["cases"][0]
    pa, pb = O.point_from_x(int(a)), O.point_from_x(int(b))
    wa = O.int_to_be_words(pa[0]) + O.int_to_be_words(pa[1])
    wb = O.int_to_be_words(pb[0]) + O.int_to_be_words(pb[1])
    script = f"""
import * as m from {json.dumps(JS)};
const r = m.point_add_affine(new Uint32Array({wa}), new Uint32Array({wb}));
console.log(m.u32ArrayToBigInts(r).map(String).join(","));
"""
    x, y = _node(script).strip().split(",")
    assert int(x) == int(exp) and (int(x), int(y)) == O.aff_add(pa, pb)


@pytest.mark.skipif(NODE is None, reason="node not installed")
def test_js_compute_msm_fails_loudly_without_device():
    if M.load().msm_init() == 0:
        pytest.skip("a GPU is present; covered by tests/test_gpu_js.py")
    script = f"""
import * as m from {json.dumps(JS)};
m.compute_msm([{{x: 1n, y: 2n, t: 2n, z: 1n}}], [3n]).then(
  () => console.log("resolved"), (e) => console.log("rejected " + e.code));
"""
    assert _node(script).strip() == "rejected -6"


def _red1_lane(Wm, nm, nhi, B, L, nchunks, gd):
    """Mirror of msm_kernels.hip red1_lane (k_bucket_reduce_1's lane -> (window, chunk) map)."""
    nmain = Wm - 1
    lc_hi = nchunks
    nfull = nhi if nhi else nmain
    lc_lo = (B // 2 + L - 1) // L if nhi else nchunks
    live = nfull * lc_hi + (nmain - nfull) * lc_lo
    if gd < nm * live:
        m, r = divmod(gd, live)
        if r < nfull * lc_hi:
            w, c = divmod(r, lc_hi)
        else:
            r2 = r - nfull * lc_hi
            w, c = nfull + r2 // lc_lo, r2 % lc_lo
        return m * Wm + w, c, True
    dead_lo = (nmain - nfull) * (nchunks - lc_lo)
    per = dead_lo + nchunks
    r0 = gd - nm * live
    if r0 >= nm * per:
        return None
    m, r = divmod(r0, per)
    if r < dead_lo:
        span = nchunks - lc_lo
        return m * Wm + nfull + r // span, lc_lo + r % span, False
    return m * Wm + nmain, r - dead_lo, False


def test_red1_lane_map_is_a_bijection_live_first():
    """Every (window, chunk) of a launch is reduced by exactly one k_bucket_reduce_1 lane, and the
    chunks a digit can reach come first (window geometry as make_plan builds it)."""
    for c in (4, 5, 8, 13, 14, 15, 16):
        wm = (254 + c - 1) // c
        q = 254 // wm
        nhi = 254 - q * wm
        cc = q + 1 if nhi else q
        B = 1 << (cc - 1)
        Wm = wm + 1
        for nm in ((1, 2) if c < 16 else (2,)):
            for L in ((4, 8, 9, 10, 12, 16) if c < 15 else (9, 16)):
                nchunks = (B + L - 1) // L
                seen, last_live = set(), True
                for gd in range(Wm * nm * nchunks):
                    w, ch, live = _red1_lane(Wm, nm, nhi, B, L, nchunks, gd)
                    assert 0 <= ch < nchunks and 0 <= w < Wm * nm
                    assert (w, ch) not in seen
                    seen.add((w, ch))
                    if live:
                        assert last_live, "live chunk after a dead one"
                    last_live = live
                    wl = w % Wm
                    bits = 3 if wl == Wm - 1 else (q + 1 if wl < nhi else q)
                    reach = 1 << (bits - 1)  # buckets a digit of this window can reach
                    if ch * L < reach and wl != Wm - 1:
                        assert live, (c, nm, L, w, ch)
                assert len(seen) == Wm * nm * nchunks
                assert _red1_lane(Wm, nm, nhi, B, L, nchunks, Wm * nm * nchunks) is None


def _shard(n, i, D):
    L = M.load()
    lo, hi = ctypes.c_size_t(), ctypes.c_size_t()
    assert L.msm_test_shard_range(n, i, D, ctypes.byref(lo), ctypes.byref(hi)) == 0
    return lo.value, hi.value


@pytest.mark.parametrize("n", [0, 1, 7, 1000, 1 << 20, (1 << 20) + 5])
def test_device_shards_partition_the_points(n):
    """The device-list split (msm_opts MSM_FLAG_DEVICES) is contiguous, covers [0, n), sizes
    differ by at most one, and agrees with the torch.distributed split (msm_amd.dist)."""
    from msm_amd.dist import shard_range
    for D in range(1, M.MSM_MAX_DEVICES + 1):
        spans = [_shard(n, i, D) for i in range(D)]
        assert spans[0][0] == 0 and spans[-1][1] == n
        assert all(spans[i][1] == spans[i + 1][0] for i in range(D - 1))
        sizes = [hi - lo for lo, hi in spans]
        assert max(sizes) - min(sizes) <= 1
        assert spans == [shard_range(n, i, D) for i in range(D)]


def test_device_shard_join_equals_whole_msm():
    """Shard partials (closed form per shard) joined by libmsm's host EC adds = the whole MSM."""
    from _closed_form import closed_form
    n = 1001
    sc = O.xorshift_scalars_np(n, seed=77)
    whole = closed_form(3, 5, sc)
    for D in (1, 2, 3, 8, 16):
        parts = np.zeros((D, 32), np.uint32)
        for i in range(D):
            lo, hi = _shard(n, i, D)
            x, y = closed_form(3 + 5 * lo, 5, sc[lo:hi]) if hi > lo else O.IDENTITY
            for j, v in enumerate((x, y, x * y % O.P, 1)):
                parts[i, 8 * j: 8 * j + 8] = O.int_to_be_words(v)
        assert M.combine_partials(parts) == whole


def _host_mont_words(v):
    m = v * (1 << 256) % O.P  # the host's Montgomery form (hostfield.h, R = 2^256), LE words
    return [(m >> (32 * q)) & 0xFFFFFFFF for q in range(8)]


@pytest.mark.parametrize("n", [1 << 12, 1 << 20])
def test_lone_msm_tail_threads_agree(n):
    """The window-parallel tail of a lone MSM (TailCrew: helper threads sum each window's terms,
    the caller runs the outer Horner) equals the one-thread Horner (which every GPU parity test
    checks end to end), identity terms included."""
    L = M.load()
    words = L.msm_test_tail_words(n)
    rng = np.random.default_rng(n)
    terms = np.zeros(words, np.uint32)
    pts = []
    for i in range(words // 32):
        if i % 7 == 3:  # an identity term (X = 0, Y = Z)
            x, y, z = 0, 1, 5
        else:
            x, y = O.scalar_mul(O.G, int(rng.integers(1, 1 << 40)))
            z = int(rng.integers(1, 1 << 40))
        pts.append((x, y))
        for j, v in enumerate((x * z % O.P, y * z % O.P, x * y % O.P * z % O.P, z)):
            terms[i * 32 + 8 * j: i * 32 + 8 * j + 8] = _host_mont_words(v)
    got = {}
    # helpers < 0: one persistent crew over 40 rounds, some armed and disarmed without terms (the
    # per-device crew of lone MSMs, including their error returns)
    for helpers in (0, 1, 3, -3, -1):
        out = (ctypes.c_uint32 * 16)()
        ms = ctypes.c_double()
        assert L.msm_test_tail(n, terms.ctypes.data, helpers, out, ctypes.byref(ms)) == 0, helpers
        got[helpers] = (M.wire_to_int(out[:8]), M.wire_to_int(out[8:]))
    assert got[0] == got[1] == got[3] == got[-3] == got[-1]


@pytest.mark.parametrize("n,k", [(1 << 12, 2), (1 << 17, 2), (1 << 16, 4), (1 << 12, 1)])
def test_batch_tail_matches_per_msm_horner(n, k):
    """The last launch's tails of a pipelined run (TailCrew::run_batch: the window sums of all k
    MSMs over the helpers, the outer Horners of MSMs 1.. taken by helpers) equal one horner_tail
    per MSM, for 1, 2 and 3 helpers (fewer helpers than MSMs: the caller runs the outer Horners no
    helper took), identity terms included."""
    L = M.load()
    words = L.msm_test_tail_words(n)
    rng = np.random.default_rng(n + k)
    terms = np.zeros(words * k, np.uint32)
    for i in range(words * k // 32):
        if i % 5 == 2:
            x, y, z = 0, 1, 3
        else:
            x, y = O.scalar_mul(O.G, int(rng.integers(1, 1 << 30)))
            z = int(rng.integers(1, 1 << 30))
        for j, v in enumerate((x * z % O.P, y * z % O.P, x * y % O.P * z % O.P, z)):
            terms[i * 32 + 8 * j: i * 32 + 8 * j + 8] = _host_mont_words(v)
    got = {}
    for helpers in (0, 1, 2, 3):
        out = (ctypes.c_uint32 * (16 * k))()
        ms = ctypes.c_double()
        assert L.msm_test_tail_batch(n, k, terms.ctypes.data, helpers, out, ctypes.byref(ms)) == 0, helpers
        got[helpers] = [(M.wire_to_int(out[16 * m: 16 * m + 8]), M.wire_to_int(out[16 * m + 8: 16 * m + 16]))
                        for m in range(k)]
    assert got[0] == got[1] == got[2] == got[3]
    assert len(set(got[0])) == k  # the MSMs' blocks differ: each Horner read its own block
    # the single-MSM entry on block 0 agrees
    out = (ctypes.c_uint32 * 16)()
    ms = ctypes.c_double()
    assert L.msm_test_tail(n, terms.ctypes.data, 3, out, ctypes.byref(ms)) == 0
    assert (M.wire_to_int(out[:8]), M.wire_to_int(out[8:])) == got[0][0]


def test_host_inverse_matches_fermat():
    """hostfield.h's binary-Euclid fq_inv (the affine conversion's inverse) equals a^(p-2) and
    a * a^-1 = 1 on 4,000 pseudo-random full-width and short values, 1 and p - 1, and maps 0 to 0
    (msm_test_host_timing mode 4 counts mismatches)."""
    L = M.load()
    bad = ctypes.c_double(-1)
    assert L.msm_test_host_timing(4, 4000, ctypes.byref(bad)) == 0
    assert bad.value == 0


def test_bench_refuses_more_gpus_than_visible():
    """bench.py --gpus N without torchrun measures N devices in one process; with fewer gfx950
    devices visible (none in the CPU container) it exits non-zero and prints no JSON line."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    import msm_amd as M

    n = len(M.device_ordinals())
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", str(max(n + 1, 2)), "--steps", "1",
                        "--no-extras", "--no-cpu-baseline"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode != 0
    assert "gfx950 device(s) visible" in r.stderr
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]


def _top_window_bucket_bound(n, c):
    """lambda + 5 sqrt(lambda) + 2 of the largest expected bucket of an n-point MSM at window width c
    (uniform scalars mod p; the top main window's digits stop at p >> offset), from the Python
    window layout, independently of libmsm's run_length_skew_floor."""
    import math

    wm = -(-254 // c)
    q, nhi = 254 // wm, 254 - (254 // wm) * wm
    lam = 0.0
    for w in range(wm):
        b = q + 1 if w < nhi else q
        vals = 1 << (b - 1)
        if w == wm - 1:
            off = w * q + min(w, nhi)
            vals = min(vals, (O.P >> off) + 1)
        lam = max(lam, n / vals)
    return lam + 5 * math.sqrt(lam) + 2


@pytest.mark.parametrize("n,nm,pipelined", [(1 << 20, 2, True), ((1 << 20) + 1, 2, True), (1 << 20, 1, False),
                                            ((1 << 20) + 1, 1, False), (1 << 21, 2, True), (1 << 21, 1, False),
                                            (5 << 18, 2, True), (3 << 18, 2, True), (1 << 18, 4, True),
                                            (1 << 17, 4, True), (1 << 16, 8, True), (1 << 19, 1, False),
                                            (4096, 1, False), (1000, 1, False)])
def test_run_length_clears_the_skew_joins(n, nm, pipelined):
    """The plan's run length K keeps every expected bucket under three whole runs (3 K + 2 entries:
    the skew joins' trigger in k_accumulate), so random scalars never take the second reduction;
    K is a multiple of 4 (16-B entry loads)."""
    pl = M.launch_plan(n, nm, pipelined)
    K = pl["run_length"]
    assert K % 4 == 0 and 16 <= K <= 4096
    assert 3 * K + 2 > _top_window_bucket_bound(n, pl["c"])
    assert K >= pl["skew_floor"]


def test_run_length_past_a_power_of_two():
    """The round-4 cliff: one point past 2^20 no longer shortens K (2^20 + 1 was 14% slower than
    2^20 at K = 44, the skew joins on every launch).  Pipelined launches keep K = 64; a lone MSM
    takes one round of K = 68 instead of two rounds; 2^20 itself and the small four-MSM launches
    (one round filled by a shorter K) are unchanged."""
    assert M.launch_plan(1 << 20, 2, True)["run_length"] == 64
    assert M.launch_plan((1 << 20) + 1, 2, True)["run_length"] == 64
    assert M.launch_plan(1 << 20, 1, False)["run_length"] == 64
    assert M.launch_plan((1 << 20) + 1, 1, False)["run_length"] == 68
    assert M.launch_plan(1 << 17, 4, True)["run_length"] == 36
    # an explicit run length is taken as given
    assert M.launch_plan((1 << 20) + 1, 2, True, run_length=44)["run_length"] == 44


@pytest.mark.parametrize("n", [0, 1, 7, 1000, 4099])
def test_host_packing_keeps_x_y_and_checks_t(n):
    """The packed uploads' host pass (pack_records, msm_test_pack; run on the library's own
    threads): x|y (16 words) or x|y|z (24 words) of every wire record, in order, whatever the
    share boundaries of the threads; `all z == 1` is exact (z has 8 words), and any t >= p is
    reported (t is checked on the host because it is not uploaded)."""
    rng = np.random.default_rng(n + 3)
    wire = np.zeros((n, 32), np.uint32)
    for i in range(n):
        for j in range(3):  # x, y, t < p
            wire[i, 8 * j: 8 * j + 8] = O.int_to_be_words(int(rng.integers(0, 1 << 62)) * 0x1f3 % O.P + j)
        wire[i, 24:32] = O.int_to_be_words(1)
    for xyz in (False, True):
        out, z1, tb = M.pack_points(wire, xyz=xyz)
        assert out.shape == (n, 24 if xyz else 16)
        assert np.array_equal(out[:, :16], wire[:, :16])
        if xyz:
            assert np.array_equal(out[:, 16:], wire[:, 24:32])
        assert z1 and not tb
    if n == 0:
        return
    k = n // 2
    w2 = wire.copy()
    w2[k, 24:32] = O.int_to_be_words(1 + (1 << 200))  # z != 1 only in a high word
    out, z1, tb = M.pack_points(w2, xyz=True)
    assert not z1 and not tb and np.array_equal(out[:, 16:], w2[:, 24:32])
    for tv, bad in ((O.P - 1, False), (O.P, True), ((1 << 256) - 1, True)):
        w3 = wire.copy()
        w3[n - 1, 16:24] = O.int_to_be_words(tv)
        _, z1, tb = M.pack_points(w3)
        assert z1 and tb == bad


def _red2_groups_model(T, U, nchunks, g, lg):
    """k_red2_groups' index algebra (msm_kernels.hip) over integers: the lg steps of in-place
    adds over the group's 2^lg chunks; returns (V, S, R_0..R_{lg-1})."""
    ch = 1 << lg
    A = [T[g * ch + i] if g * ch + i < nchunks else 0 for i in range(ch)]
    Bv = [U[g * ch + i] if g * ch + i < nchunks else 0 for i in range(ch)]
    for s in range(lg):
        lp = lg - 1 - s
        touched = set()
        for Q in range((2 + s) << lp):
            kind, i = Q >> lp, Q & ((1 << lp) - 1)
            arr = Bv if kind == 1 else A
            if kind < 2:
                dst = i << (s + 1)
                src = dst + (1 << s)
            else:
                j = kind - 2
                l = s - j - 1
                md = i << (l + 1)
                ms = md + (1 << l)
                dst, src = (2 * md + 1) << j, (2 * ms + 1) << j
            key = (kind == 1, dst), (kind == 1, src)
            assert not (set(key) & touched), "two tasks of one step share a point"
            touched |= set(key)
            arr[dst] += arr[src]
    return [Bv[0], A[0]] + [A[1 << k] for k in range(lg)]


@pytest.mark.parametrize("lg", [6, 7, 8])
@pytest.mark.parametrize("nchunks", [1, 5, 256, 300, 1821, 2048, 4096])
def test_red2_group_tree_terms(nchunks, lg):
    """k_red2_groups + k_red2_terms (the second bucket-reduction stage in two kernels, groups of
    2^lg chunks, MSM_RG_LOG) give terms with sum_v V_v + sum_k 2^k R_k (times L on the host) =
    sum_c U_c + sum_c c T_c, modelled over integers with the kernels' own index algebra (group
    trees in place, the R_k lists at indices whose lowest set bit is 2^k, the terms' group
    selection)."""
    rng = np.random.default_rng(nchunks)
    T = [int(x) for x in rng.integers(0, 1 << 40, nchunks)]
    U = [int(x) for x in rng.integers(0, 1 << 40, nchunks)]
    G = (nchunks + (1 << lg) - 1) >> lg
    grp = [_red2_groups_model(T, U, nchunks, g, lg) for g in range(G)]
    nv = 2 if nchunks >= 2 else 1
    cbits = 0
    while (1 << cbits) < nchunks:
        cbits += 1
    total = 0
    for term in range(nv + cbits):
        if term < nv:
            sl = (G + nv - 1) // nv
            g0 = min(G, term * sl)
            pts = [grp[g][0] for g in range(g0, min(G, g0 + sl))]
            total += sum(pts)
            continue
        k = term - nv
        if k < lg:
            pts = [grp[g][2 + k] for g in range(G)]
        else:
            kb = k - lg
            half = 1
            while 2 * half < G:
                half <<= 1
            gs = [((j >> kb) << (kb + 1)) | (1 << kb) | (j & ((1 << kb) - 1)) for j in range(half)]
            pts = [grp[g][1] for g in gs if g < G]
        total += (1 << k) * sum(pts)
    assert total == sum(U) + sum(c * t for c, t in enumerate(T))
