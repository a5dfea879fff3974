"""ORACLE — test infrastructure only (the checker, never the product).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.

Two independent restatements of the reference's MSM semantics for Edwards-BLS12
(ark-ed-on-bls12-377; src/reference/params/AleoConstants.ts:2-5):

* ``liboracle.so`` (msm_oracle.c): the reference's own CPU Pippenger (src/submission/msm-wasm/
  src/lib.rs:24-121), group law of src/submission/wgsl/curve.wgsl:36-114, wire codec of
  bytes.rs:11-71, getPointFromX of src/reference/utils/FieldMath.ts:31-55.
* pure Python (this file): affine Edwards arithmetic and the closed form used by the survey to
  pin the Aleo-wasm oracle: with P_i = k_i G in the prime-order subgroup,
  sum_i s_i P_i = ((sum_i s_i k_i) mod r) G.

Both are pinned against the reference's known-answer vectors and the survey-recorded oracle
results (tests/golden/); see tests/test_oracle.py.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import Iterable, List, Optional, Sequence, Tuple

import numpy as np

# AleoConstants.ts:2-5 / FieldMath.ts:7-10
P = 8444461749428370424248824938781546531375899335154063827935233455917409239041
EDWARDS_A = P - 1
EDWARDS_D = 3021
R_ORDER = 2111115437357092606062206234695386632838870926408408195193685246394721360383

# The benchmark page's fixed point (src/ui/AllBenchmarks.tsx:111-119), in the r-torsion subgroup.
G = (
    2796670805570508460920584878396618987767121022598342527208237783066948667246,
    8134280397689638111748378379571739274369602049665521098046934931245960532166,
)
IDENTITY = (0, 1)

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")


# --------------------------------------------------------------------------------------------
# pure-Python field / curve (a = -1, d = 3021)
# --------------------------------------------------------------------------------------------
def inv(a: int) -> int:
    return pow(a % P, P - 2, P)


def on_curve(pt: Tuple[int, int]) -> bool:
    x, y = pt
    return (EDWARDS_A * x * x + y * y - 1 - EDWARDS_D * x * x * y * y) % P == 0


def aff_add(p1: Tuple[int, int], p2: Tuple[int, int]) -> Tuple[int, int]:
    """Affine twisted-Edwards addition (complete for this curve)."""
    x1, y1 = p1
    x2, y2 = p2
    t = EDWARDS_D * x1 * x2 * y1 * y2 % P
    x3 = (x1 * y2 + y1 * x2) * inv(1 + t) % P
    y3 = (y1 * y2 - EDWARDS_A * x1 * x2) * inv(1 - t) % P
    return (x3, y3)


def aff_neg(p: Tuple[int, int]) -> Tuple[int, int]:
    return ((-p[0]) % P, p[1])


def _ext_add(p, q):
    # extended coordinates, add-2008-hwcd (a = -1), unified
    X1, Y1, T1, Z1 = p
    X2, Y2, T2, Z2 = q
    A = X1 * X2 % P
    B = Y1 * Y2 % P
    C = EDWARDS_D * T1 * T2 % P
    D = Z1 * Z2 % P
    E = ((X1 + Y1) * (X2 + Y2) - A - B) % P
    F = (D - C) % P
    Gg = (D + C) % P
    H = (B + A) % P
    return (E * F % P, Gg * H % P, E * H % P, F * Gg % P)


def scalar_mul(pt: Tuple[int, int], k: int) -> Tuple[int, int]:
    """k * pt for any integer k >= 0 (double-and-add in extended coordinates)."""
    x, y = pt
    base = (x, y, x * y % P, 1)
    acc = (0, 1, 0, 1)
    for bit in bin(k)[2:] if k > 0 else "":
        acc = _ext_add(acc, acc)
        if bit == "1":
            acc = _ext_add(acc, base)
    X, Y, _, Z = acc
    zi = inv(Z)
    return (X * zi % P, Y * zi % P)


def sqrt_mod(a: int) -> Optional[int]:
    a %= P
    if a == 0:
        return 0
    if pow(a, (P - 1) // 2, P) != 1:
        return None
    q, s = P - 1, 0
    while q % 2 == 0:
        q //= 2
        s += 1
    z = 2
    while pow(z, (P - 1) // 2, P) == 1:
        z += 1
    m, c, t, r = s, pow(z, q, P), pow(a, q, P), pow(a, (q + 1) // 2, P)
    while t != 1:
        i, t2 = 0, t
        while t2 != 1:
            t2 = t2 * t2 % P
            i += 1
        b = pow(c, 1 << (m - i - 1), P)
        m, c, t, r = i, b * b % P, t * b * b % P, r * b % P
    return r


def point_from_x(x: int) -> Tuple[int, int]:
    """getPointFromX (FieldMath.ts:31-55): the y whose point lies in the r-torsion subgroup."""
    x2 = x * x % P
    y2 = (EDWARDS_A * x2 - 1) * inv(EDWARDS_D * x2 - 1) % P
    y = sqrt_mod(y2)
    if y is None:
        raise ValueError("x is not the x-coordinate of a curve point")
    if scalar_mul((x, y), R_ORDER) == IDENTITY:
        return (x, y)
    return (x, (-y) % P)


def closed_form_msm(ks: Sequence[int], ss: Sequence[int]) -> Tuple[int, int]:
    """sum s_i (k_i G) = ((sum s_i k_i) mod r) G."""
    acc = 0
    for k, s in zip(ks, ss):
        acc += k * s
    return scalar_mul(G, acc % R_ORDER)


# --------------------------------------------------------------------------------------------
# deterministic inputs (SURVEY.md §8c spec)
# --------------------------------------------------------------------------------------------
XORSHIFT_SEED = 0x9E3779B97F4A7C15


def xorshift_scalars(n: int, seed: int = XORSHIFT_SEED, mod: Optional[int] = P) -> List[int]:
    """xorshift64(13, 7, 17); 4 words per scalar, first word most significant; reduced mod p."""
    M = (1 << 64) - 1
    s = seed
    out = []
    for _ in range(n):
        v = 0
        for _ in range(4):
            s ^= (s << 13) & M
            s ^= s >> 7
            s ^= (s << 17) & M
            v = (v << 64) | s
        out.append(v % mod if mod else v)
    return out


def xorshift_scalars_np(n: int, seed: int = XORSHIFT_SEED) -> np.ndarray:
    """Vectorised-by-chunks variant of xorshift_scalars returning BE u32 [n, 8] (mod p)."""
    ints = xorshift_scalars(n, seed)
    return ints_to_be_words(ints)


# --------------------------------------------------------------------------------------------
# wire codec (bytes.rs:11-44, webgpu/utils.test.ts:4-41): 8 big-endian u32 words
# --------------------------------------------------------------------------------------------
def int_to_be_words(v: int) -> List[int]:
    return [(v >> (32 * (7 - i))) & 0xFFFFFFFF for i in range(8)]


def be_words_to_int(w: Iterable[int]) -> int:
    v = 0
    for x in w:
        v = (v << 32) | int(x)
    return v


def ints_to_be_words(vals: Sequence[int]) -> np.ndarray:
    n = len(vals)
    if n == 0:
        return np.zeros((0, 8), dtype=np.uint32)
    b = b"".join(int(v).to_bytes(32, "big") for v in vals)
    return np.frombuffer(b, dtype=">u4").astype(np.uint32).reshape(n, 8)


def be_words_to_ints(arr: np.ndarray) -> List[int]:
    a = np.ascontiguousarray(arr, dtype=np.uint32).reshape(-1, 8)
    raw = a.astype(">u4").tobytes()
    return [int.from_bytes(raw[32 * i: 32 * i + 32], "big") for i in range(a.shape[0])]


def affine_to_wire(pts: Sequence[Tuple[int, int]]) -> np.ndarray:
    """Affine points -> wire points [n, 32] (x|y|t|z, z = 1, t = x y)."""
    out = np.zeros((len(pts), 32), dtype=np.uint32)
    if not pts:
        return out
    out[:, 0:8] = ints_to_be_words([p[0] for p in pts])
    out[:, 8:16] = ints_to_be_words([p[1] for p in pts])
    out[:, 16:24] = ints_to_be_words([p[0] * p[1] % P for p in pts])
    out[:, 31] = 1
    return out


# --------------------------------------------------------------------------------------------
# C restatement (liboracle.so)
# --------------------------------------------------------------------------------------------
_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        u32p = np.ctypeslib.ndpointer(dtype=np.uint32, flags="C_CONTIGUOUS")
        u64p = np.ctypeslib.ndpointer(dtype=np.uint64, flags="C_CONTIGUOUS")
        L.oracle_msm.argtypes = [ctypes.c_uint32, u32p, u32p, ctypes.c_size_t, ctypes.c_int, u32p]
        L.oracle_msm.restype = ctypes.c_int
        L.oracle_field_op.argtypes = [ctypes.c_int, u64p, u64p, u64p]
        L.oracle_field_op.restype = ctypes.c_int
        for name in ("oracle_point_add", "oracle_point_add_affine"):
            getattr(L, name).argtypes = [u32p, u32p, u32p]
            getattr(L, name).restype = ctypes.c_int
        L.oracle_point_double.argtypes = [u32p, u32p]
        L.oracle_scalar_mul.argtypes = [u32p, u32p, u32p]
        L.oracle_on_curve.argtypes = [u32p]
        L.oracle_split.argtypes = [ctypes.c_uint32, u32p, ctypes.c_size_t, u32p]
        L.oracle_split_windows.argtypes = [ctypes.c_uint32]
        L.oracle_split_windows.restype = ctypes.c_uint32
        L.oracle_point_from_x.argtypes = [u32p, u32p]
        L.oracle_gen_points.argtypes = [u32p, u32p, ctypes.c_uint64, ctypes.c_size_t, u32p]
        _lib = L
    return _lib


def _u32(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.uint32)


def xy_words(pt: Tuple[int, int]) -> np.ndarray:
    return _u32(int_to_be_words(pt[0]) + int_to_be_words(pt[1]))


def words_xy(w: np.ndarray) -> Tuple[int, int]:
    return (be_words_to_int(w[:8]), be_words_to_int(w[8:16]))


def msm(points_be: np.ndarray, scalars_be: np.ndarray, window: int = 16, threads: int = 1) -> Tuple[int, int]:
    """msm_end_to_end (lib.rs:106-121) on wire inputs; returns affine (x, y) ints."""
    pts = _u32(points_be).reshape(-1, 32)
    sc = _u32(scalars_be).reshape(-1, 8)
    n = min(pts.shape[0], sc.shape[0])
    out = np.zeros(16, dtype=np.uint32)
    rc = lib().oracle_msm(window, _u32(sc[:n]).reshape(-1), _u32(pts[:n]).reshape(-1), n, threads, out)
    if rc != 0:
        raise ValueError(f"oracle_msm failed: {rc}")
    return words_xy(out)


def split(window: int, scalars_be: np.ndarray) -> np.ndarray:
    sc = _u32(scalars_be).reshape(-1, 8)
    nw = lib().oracle_split_windows(window)
    out = np.zeros(nw * sc.shape[0], dtype=np.uint32)
    lib().oracle_split(window, sc.reshape(-1), sc.shape[0], out)
    return out


def c_point_add(a: Tuple[int, int], b: Tuple[int, int]) -> Tuple[int, int]:
    out = np.zeros(16, dtype=np.uint32)
    lib().oracle_point_add(xy_words(a), xy_words(b), out)
    return words_xy(out)


def c_point_double(a: Tuple[int, int]) -> Tuple[int, int]:
    out = np.zeros(16, dtype=np.uint32)
    lib().oracle_point_double(xy_words(a), out)
    return words_xy(out)


def c_scalar_mul(a: Tuple[int, int], k: int) -> Tuple[int, int]:
    out = np.zeros(16, dtype=np.uint32)
    lib().oracle_scalar_mul(xy_words(a), _u32(int_to_be_words(k)), out)
    return words_xy(out)


def c_point_from_x(x: int) -> int:
    out = np.zeros(8, dtype=np.uint32)
    rc = lib().oracle_point_from_x(_u32(int_to_be_words(x)), out)
    if rc != 0:
        raise ValueError("not an x-coordinate")
    return be_words_to_int(out)


def c_field_op(op: int, a: int, b: int = 0) -> int:
    def limbs(v):
        return np.array([(v >> (64 * i)) & ((1 << 64) - 1) for i in range(4)], dtype=np.uint64)

    out = np.zeros(4, dtype=np.uint64)
    rc = lib().oracle_field_op(op, limbs(a), limbs(b), out)
    if rc != 0:
        raise ValueError("operand out of range")
    return sum(int(out[i]) << (64 * i) for i in range(4))


def gen_points(n: int, k0: int = 1, step: int = 1, base: Tuple[int, int] = G) -> np.ndarray:
    """Wire points [n, 32] for (k0 + i*step) * base, i = 0..n-1 (z = 1, t = x y)."""
    out = np.zeros((max(n, 1), 32), dtype=np.uint32)
    if n:
        lib().oracle_gen_points(xy_words(base), _u32(int_to_be_words(k0)), step, n, out.reshape(-1))
    return out[:n]
