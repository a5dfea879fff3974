"""The exact reciprocal division of msm_kernels.hip (`div_by_inv`): floor(x / D) as
trunc((x + 0.5) * (1.0 / D)) in IEEE double precision, for any 32-bit x.  k_fine_sort divides by
the run length K (a bucket's first run, ceil(gs / K)) and k_bucket_reduce_1 by K * 256 (a bucket's
accumulation workgroup).  The device's v_cvt_f64_u32 / v_mul_f64 / v_cvt_u32_f64 are correctly
rounded IEEE operations, as numpy's float64 ones are, so this checks the kernels' arithmetic.
"""
import numpy as np

ACC_THREADS = 256


def div_by_inv(x, d):
    inv = np.float64(1.0) / np.float64(d)
    return ((x.astype(np.float64) + 0.5) * inv).astype(np.uint64)


def edge_values(d, rng):
    top = (1 << 32) - 1
    q = rng.integers(0, top // d + 1, size=4096, dtype=np.uint64)
    base = q * np.uint64(d)
    xs = [base, base - np.uint64(1), base + np.uint64(1), base + np.uint64(d - 1)]
    xs.append(np.array([0, 1, d - 1, d, d + 1, top, top - 1, top - (top % d)], dtype=np.uint64))
    xs.append(rng.integers(0, top, size=4096, dtype=np.uint64, endpoint=True))
    x = np.concatenate(xs)
    return x[(x <= top)]  # base - 1 wraps at q = 0


def test_div_by_inv_exact_for_run_lengths():
    rng = np.random.default_rng(11)
    for k in list(range(1, 257)) + [1000, 4096, 65535]:
        for d in (k, k * ACC_THREADS):
            x = edge_values(d, rng)
            assert np.array_equal(div_by_inv(x, d), x // np.uint64(d)), d


def test_first_run_of_bucket():
    # k_fine_sort: the runs starting inside [gs, ge) are r = ceil(gs / K) .. while r * K < ge
    rng = np.random.default_rng(12)
    for k in (20, 36, 52, 64, 68, 128):
        gs = rng.integers(0, (1 << 32) - k, size=20000, dtype=np.uint64)
        r0 = div_by_inv(gs + np.uint64(k - 1), k)
        assert np.array_equal(r0, (gs + np.uint64(k - 1)) // np.uint64(k))
        assert np.all(r0 * np.uint64(k) >= gs)
        pos = r0 > 0
        assert np.all((r0[pos] - np.uint64(1)) * np.uint64(k) < gs[pos])
