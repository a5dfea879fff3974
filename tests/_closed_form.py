"""Fast closed-form expected values for MSMs over P_i = k_i G (test infrastructure).

sum_i s_i (k_i G) = ((sum_i s_i k_i) mod r) G (the oracle's closed_form_msm, oracle/oracle.py),
with the inner sum done exactly in numpy: scalars split into 16-bit pieces so every dot product
stays below 2^64 for up to 2^21 terms of k < 2^21... and beyond by chunking.
"""
import numpy as np

from oracle import oracle as O


def scalar_dot(ks: np.ndarray, sc_be_words: np.ndarray) -> int:
    """sum_i k_i * s_i exactly; ks uint64 [n] (< 2^32), sc_be_words [n, 8] big-endian u32."""
    ks = np.asarray(ks, dtype=np.uint64)
    w = np.asarray(sc_be_words, dtype=np.uint32).reshape(-1, 8)
    assert ks.shape[0] == w.shape[0]
    total = 0
    step = 1 << 14  # k < 2^32, piece < 2^16: each product < 2^48, 2^14 of them < 2^62
    for lo in range(0, ks.shape[0], step):
        k = ks[lo:lo + step]
        blk = w[lo:lo + step].astype(np.uint64)
        for j in range(8):
            for h in range(2):
                piece = (blk[:, j] >> np.uint64(16 * h)) & np.uint64(0xFFFF)
                s = int(np.dot(k, piece))
                total += s << (32 * (7 - j) + 16 * h)
    return total


def closed_form(k0: int, step: int, sc_be_words: np.ndarray):
    """Expected affine MSM of P_i = (k0 + i step) G with the given scalars."""
    n = np.asarray(sc_be_words).reshape(-1, 8).shape[0]
    ks = k0 + step * np.arange(n, dtype=np.uint64)
    return O.scalar_mul(O.G, scalar_dot(ks, sc_be_words) % O.R_ORDER)


def as_xy(row):
    return O.be_words_to_int(row[:8]), O.be_words_to_int(row[8:16])
