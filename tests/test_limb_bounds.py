"""Static limb-bound proof for the device field/curve code (webgpu-msm_amd/csrc/fp29.cuh, ec.cuh).

The 29-bit-limb lazy Montgomery multiply accumulates up to 18 partial products per 64-bit column
with no carry handling, and the curve formulas feed unnormalised sums/differences into it.  A
column overflow would be a silent, data-dependent wrong answer that random tests hit almost
never, so this test walks every formula in the kernels with per-limb worst-case bounds (interval
arithmetic on the limb maxima) and asserts:

  * every fe_mul column stays < 2^64 (products + reduction terms + incoming carry);
  * every fe_mul operand pair keeps a*b < p * 2^261, so the lazy result is < 2p (no final
    subtraction needed);
  * fe_sub / fe_neg never produce a negative limb (K8P dominates the subtrahend limb-wise);
  * pt_madd's signed differences (fe_sub_s) keep every fe_mul_sd column register inside int64
    (per-limb intervals, with the centring offsets SD_OFF58) and its biased result in [0, 2p).

It mirrors the kernels by hand; test_mirrored_sources_unchanged pins a digest of every mirrored
function body, so an edit to fp29.cuh / ec.cuh fails until the model here is re-reviewed.
"""
P = 8444461749428370424248824938781546531375899335154063827935233455917409239041
NL, LB = 9, 29
MASK = (1 << LB) - 1
R = 1 << 261
P29 = [(P >> (LB * i)) & MASK for i in range(NL)]
K8P29 = [536870920, 610271231, 536871443, 661646591, 939568340, 880373981, 718018184, 1050291364, 9788201]
K5P29 = [536870917, 851181567, 536871243, 681964575, 654339076, 550233738, 717196821, 991976422, 6117625]


class B:
    """Worst-case limb maxima + value maximum of a field element."""

    def __init__(self, limbs, value):
        self.l = list(limbs)
        self.v = value

    @staticmethod
    def normalised(value):
        top = value >> (LB * (NL - 1))
        return B([MASK] * (NL - 1) + [top], value)


N_MUL = B.normalised(2 * P)  # fe_mul output: normalised, value < 2p


def value_of(limbs):
    return sum(x << (LB * i) for i, x in enumerate(limbs))


WIDE_ALL, WIDE_GH, WIDE_EH, WIDE_EF = 0xFF, 0xE7, 0xBF, 0xEF  # fp29.cuh: steps with a 32-bit digit


def seed(wide: int, k: int) -> int:
    """fp29.cuh fe_mul_seed: register offset of column k (2^32 - 1 on the reduction columns, -7
    after a narrow step)."""
    return ((1 << 32) - 1 if k <= NL - 1 else 0) - (7 if k >= 1 and not (wide >> (k - 1)) & 1 else 0)


def digit_max(wide: int, i: int) -> int:
    return (1 << 32) - 1 if i < NL - 1 and (wide >> i) & 1 else (1 << LB) - 1


def fe_mul(a: B, b: B, wide: int = WIDE_ALL) -> B:
    # the digits add sum_i m_i 2^(29 i) p to the product before the division by R
    extra = sum(digit_max(wide, i) << (LB * i) for i in range(NL)) * P
    assert a.v * b.v + extra < 2 * P * R, "lazy Montgomery output would exceed 2p"
    cols = [0] * (2 * NL)
    for i in range(NL):
        for j in range(NL):
            cols[i + j] += a.l[i] * b.l[j]
    carry = 0
    for k in range(2 * NL):
        red = sum(digit_max(wide, i) * P29[k - i] for i in range(NL) if 1 <= k - i < NL)
        # the register: true column (products + reduction terms + incoming carry) + its seed
        col = cols[k] + red + carry
        assert col + max(0, seed(wide, k)) < 1 << 64, f"column {k} may reach {col / 2**64:.3f} * 2^64"
        # carry out: (column + digit) / 2^29 on the reduction columns, column >> 29 above
        carry = (col + digit_max(wide, k)) >> LB if k < NL else col >> LB
    return N_MUL


def fe_mul_exact(a, b, wide: int = WIDE_ALL):
    """Bit-exact model of fp29.cuh fe_mul_w<wide> on limb lists (64-bit register wrap checked):
    returns the 9 output limbs."""
    M64 = (1 << 64) - 1
    c = [0] * (2 * NL)
    for k in range(NL + 1):
        c[k] = seed(wide, k) & M64
    for i in range(NL):
        for j in range(NL):
            c[i + j] = (c[i + j] + a[i] * b[j]) & M64
    for i in range(NL):
        lo = c[i] & 0xFFFFFFFF
        if i < NL - 1 and (wide >> i) & 1:
            m = ~lo & 0xFFFFFFFF
            c[i + 1] = (c[i + 1] + 8 * (c[i] >> 32)) & M64
        else:
            m = ~lo & MASK
            c[i + 1] = (c[i + 1] + (c[i] >> LB)) & M64
        for j in range(1, NL):
            c[i + j] = (c[i + j] + m * P29[j]) & M64
    r = [0] * NL
    for k in range(NL, 2 * NL - 1):
        c[k + 1] = (c[k + 1] + (c[k] >> LB)) & M64
        r[k - NL] = c[k] & MASK
    r[NL - 1] = c[2 * NL - 1] & 0xFFFFFFFF
    return r


K2D_INT, MU2D = 6042, (1 << 284) // P


def fe_mul_2d_exact(v: int):
    """Bit-exact model of fp29.cuh fe_mul_2d on the normalised representation of v (< 2^254):
    returns (limbs, value)."""
    a = [(v >> (LB * i)) & MASK for i in range(NL - 1)] + [v >> (LB * (NL - 1))]
    r, c = [0] * NL, 0
    for i in range(NL - 1):
        c = a[i] * K2D_INT + c
        assert c < 1 << 64
        r[i] = c & MASK
        c >>= LB
    c = a[NL - 1] * K2D_INT + c
    assert c >> 20 < 1 << 32
    q = ((c >> 20) * MU2D) >> 32
    d = 0
    for i in range(NL - 1):
        d += r[i] - q * P29[i]
        assert -(1 << 63) <= d < 1 << 63
        r[i] = d & MASK
        d >>= LB  # Python's >> is arithmetic, like the int64 shift
    r[NL - 1] = d + c - q * P29[NL - 1]
    assert 0 <= r[NL - 1] < 1 << 32
    return r, value_of(r)


KD_INT, MU272 = 3021, (1 << 272) // P


def fe_mul_d_exact(v: int):
    """Bit-exact model of fp29.cuh fe_mul_d on the normalised representation of v (< 2^254):
    returns (limbs, value)."""
    a = [(v >> (LB * i)) & MASK for i in range(NL - 1)] + [v >> (LB * (NL - 1))]
    r, c = [0] * NL, 0
    for i in range(NL - 1):
        c = a[i] * KD_INT + c
        assert c < 1 << 64
        r[i] = c & MASK
        c >>= LB
    c = a[NL - 1] * KD_INT + c
    assert c < 1 << 34
    q = ((c >> 8) * MU272) >> 32
    assert q < 1 << 32
    d = 0
    for i in range(NL - 1):
        d += r[i] - q * P29[i]
        assert -(1 << 63) <= d < 1 << 63
        r[i] = d & MASK
        d >>= LB
    r[NL - 1] = d + c - q * P29[NL - 1]
    assert 0 <= r[NL - 1] < 1 << 32
    return r, value_of(r)


def fe_mul_2d(a: B) -> B:
    assert all(x <= MASK for x in a.l[:NL - 1]) and a.v < 1 << 254
    return B.normalised(3 * P)


def fe_add(a: B, b: B) -> B:
    return B([x + y for x, y in zip(a.l, b.l)], a.v + b.v)


def fe_sub_u(a: B, b: B) -> B:
    for i in range(NL):
        assert K8P29[i] >= b.l[i], "fe_sub: negative limb possible"
    assert b.v < 8 * P
    return B([x + k for x, k in zip(a.l, K8P29)], a.v + 8 * P)


def fe_sub_v(a: B, b: B) -> B:
    """a + 5p - b (fp29.cuh fe_sub_v): b must be an fe_mul output (normalised, < 2p)."""
    for i in range(NL):
        assert K5P29[i] >= b.l[i], "fe_sub_v: negative limb possible"
    assert b.v <= 2 * P  # B.v is an exclusive bound
    return B([x + k for x, k in zip(a.l, K5P29)], a.v + 5 * P)


def fe_norm(a: B) -> B:
    return B.normalised(a.v)


def fe_sub(a: B, b: B) -> B:
    for i in range(NL - 1):
        assert a.l[i] < 1 << 30
    return fe_norm(fe_sub_u(a, b))


def fe_neg_v(b: B) -> B:  # kt_neg_if's unnormalised 5p - kt
    for i in range(NL):
        assert K5P29[i] >= b.l[i]
    assert b.v <= 2 * P  # B.v is an exclusive bound
    return B(list(K5P29), 5 * P)


# point coordinates are always fe_mul outputs (or the identity's normalised constants)
PT = dict(X=N_MUL, Y=N_MUL, T=N_MUL, Z=N_MUL)
ONE29 = 536870474 + (276299775 << 29)  # value of Montgomery one is < p; covered by N_MUL


# ---- signed differences (fp29.cuh fe_sub_s / fe_mul_sd, pt_madd) ----------------------------------
DELTA_SD_LOG = 26  # fp29.cuh: the bias DELTA_SD p 2^232 added through the seeds of columns 8..16
SD_OFF58 = [-1, -3, -3, -5, -9, -9, -12, -14, -14, -12, -11, -9, -6, -5, -2, -1, -1, 0]  # fp29.cuh: O_k / 2^58


def sd_seed(wide: int, k: int) -> int:
    """fp29.cuh fe_mul_sd_seed as a signed integer: register offset + bias + O_k - O_(k-1) / 2^29."""
    bias = (P29[k - (NL - 1)] << DELTA_SD_LOG) if NL - 1 <= k < 2 * NL - 1 else 0
    return (seed(wide, k) if k <= NL else 0) + bias + (SD_OFF58[k] << 58) - ((SD_OFF58[k - 1] << 29) if k >= 1 else 0)


class SB:
    """Interval bounds of a field element with signed limbs: per-limb [lo, hi] and value [vlo, vhi]
    (all inclusive)."""

    def __init__(self, lo, hi, vlo, vhi):
        self.lo, self.hi, self.vlo, self.vhi = list(lo), list(hi), vlo, vhi

    @staticmethod
    def of(b: B) -> "SB":  # an unsigned form (exclusive value bound b.v)
        return SB([0] * NL, list(b.l), 0, b.v - 1)


def sb_add(a: SB, b: SB) -> SB:
    return SB([x + y for x, y in zip(a.lo, b.lo)], [x + y for x, y in zip(a.hi, b.hi)], a.vlo + b.vlo, a.vhi + b.vhi)


def fe_sub_s(a: SB, b: SB) -> SB:
    return SB([x - y for x, y in zip(a.lo, b.hi)], [x - y for x, y in zip(a.hi, b.lo)], a.vlo - b.vhi, a.vhi - b.vlo)


def _ival_mul(a0, a1, b0, b1):
    c = (a0 * b0, a0 * b1, a1 * b0, a1 * b1)
    return min(c), max(c)


def fe_mul_sd(a: SB, b: SB, wide: int = WIDE_ALL) -> B:
    """fp29.cuh fe_mul_sd: signed 32x32 products, signed carries, result biased by DELTA_SD p / 2^29.
    Asserts every operand limb fits an int32, every column register fits an int64, and the result
    lies in [0, 2p) -- i.e. it is an ordinary fe_mul output (N_MUL)."""
    for x in a.lo + b.lo:
        assert x >= -(1 << 31)
    for x in a.hi + b.hi:
        assert x < 1 << 31
    delta = 1 << DELTA_SD_LOG
    bias = [delta * P29[k - (NL - 1)] if NL - 1 <= k < 2 * NL - 1 else 0 for k in range(2 * NL)]
    lo, hi = [0] * (2 * NL), [0] * (2 * NL)
    for i in range(NL):
        for j in range(NL):
            x0, x1 = _ival_mul(a.lo[i], a.hi[i], b.lo[j], b.hi[j])
            lo[i + j] += x0
            hi[i + j] += x1
    clo = chi = 0
    for k in range(2 * NL):
        red = sum(digit_max(wide, i) * P29[k - i] for i in range(NL) if 1 <= k - i < NL)
        col_lo = lo[k] + bias[k] + clo
        col_hi = hi[k] + bias[k] + red + chi
        off = seed(wide, k) if k <= NL else 0  # register offset (2^32 - 1, -7), then the centring offset O_k
        o = SD_OFF58[k] << 58
        assert -(1 << 63) <= col_lo + min(0, off) + o and col_hi + max(0, off) + o < 1 << 63, \
            f"column {k} leaves int64"
        if k < NL:  # (column + digit) / 2^29, floor
            clo, chi = col_lo >> LB, (col_hi + digit_max(wide, k)) >> LB
        else:
            clo, chi = col_lo >> LB, col_hi >> LB
    t0, t1 = _ival_mul(a.vlo, a.vhi, b.vlo, b.vhi)
    extra = sum(digit_max(wide, i) << (LB * i) for i in range(NL)) * P
    X = delta * P << (LB * (NL - 1))
    assert t0 + X >= 0, "fe_mul_sd result may be negative"
    assert t1 + X + extra < 2 * P * R, "fe_mul_sd result may reach 2p"
    return N_MUL


def test_madd_bounds():
    # halved record from k_prepare_points: ymx = fe_sub (normalised), ypx = fe_add_n, kt = fe_mul
    ymx = fe_sub(N_MUL, N_MUL)
    ypx = fe_norm(fe_add(N_MUL, N_MUL))
    kt = N_MUL
    for neg in (False, True):
        # the gather swaps the halves of a negated point (load_pre_signed); kt_neg_if negates d t
        q_ymx, q_ypx = (ypx, ymx) if neg else (ymx, ypx)
        q_kt = fe_neg_v(kt) if neg else kt
        X = Y = T = Z = SB.of(N_MUL)
        A = fe_mul_sd(fe_sub_s(Y, X), SB.of(q_ymx))
        Bv = fe_mul(fe_add(N_MUL, N_MUL), q_ypx)
        C = fe_mul(N_MUL, q_kt)
        E = fe_sub_s(SB.of(Bv), SB.of(A))
        F = fe_sub_s(Z, SB.of(C))
        G = fe_add(N_MUL, C)
        H = fe_add(Bv, A)
        fe_mul_sd(E, F)
        fe_mul(G, H)
        fe_mul_sd(E, SB.of(H))
        fe_mul_sd(F, SB.of(G))


def fe_mul_sd_exact(a, b, wide: int = WIDE_ALL):
    """Bit-exact model of fp29.cuh fe_mul_sd on limb lists (signed limbs; 64-bit two's-complement
    registers, wrap checked against the true integers): returns the 9 output limbs."""
    M64 = (1 << 64) - 1

    def s64(x):
        x &= M64
        return x - (1 << 64) if x >> 63 else x

    def s32(x):
        x &= 0xFFFFFFFF
        return x - (1 << 32) if x >> 31 else x

    c = [sd_seed(wide, k) for k in range(2 * NL)]  # the registers, as signed integers
    for i in range(NL):
        for j in range(NL):
            c[i + j] += s32(a[i]) * s32(b[j])
    for i in range(NL):
        assert -(1 << 63) <= c[i] < 1 << 63
        lo = c[i] & 0xFFFFFFFF
        if i < NL - 1 and (wide >> i) & 1:
            m = ~lo & 0xFFFFFFFF
            c[i + 1] += 8 * s32(c[i] >> 32)
        else:
            m = ~lo & MASK
            c[i + 1] += c[i] >> LB
        for j in range(1, NL):
            c[i + j] += m * P29[j]
    r = [0] * NL
    for k in range(NL, 2 * NL - 1):
        assert -(1 << 63) <= c[k] < 1 << 63
        c[k + 1] += c[k] >> LB
        r[k - NL] = c[k] & MASK
    assert 0 <= c[2 * NL - 1] < 1 << 32
    r[NL - 1] = c[2 * NL - 1]
    return [x & 0xFFFFFFFF for x in r]


def test_sd_offsets_match_header():
    src = open(os.path.join(_CSRC, "fp29.cuh")).read()
    m = re.search(r"SD_OFF58\[2 \* NL\] = \{([^}]*)\}", src)
    assert [int(x) for x in m.group(1).split(",")] == SD_OFF58
    assert int(re.search(r"DELTA_SD_LOG = (\d+);", src).group(1)) == DELTA_SD_LOG


def test_fe_mul_sd_exact_model():
    """fe_mul_sd is a b R^-1 mod p with a normalised result < 2p, for signed differences of fe_mul
    outputs against the unsigned forms pt_madd feeds it, random and at the interval corners."""
    import random
    rnd = random.Random(17)
    Rinv = pow(R, -1, P)

    def limbs(v):
        return [(v >> (LB * i)) & MASK for i in range(NL - 1)] + [v >> (LB * (NL - 1))]

    def diff(x, y):  # fe_sub_s on limbs (two's complement words)
        return [(p - q) & 0xFFFFFFFF for p, q in zip(limbs(x), limbs(y))]

    def sval(l):
        return sum((x - (1 << 32) if x >> 31 else x) << (LB * i) for i, x in enumerate(l))

    top = [MASK] * (NL - 1)
    cases = []
    for _ in range(2000):
        x, y, z, w = (rnd.randrange(2 * P) for _ in range(4))
        u = rnd.randrange(10 * P)
        cases.append((diff(x, y), limbs(u)))                      # A = (Y - X) ymx
        cases.append((diff(x, y), diff(z, w)))                    # X3 = E F
        cases.append((diff(x, y), limbs(z + w)))                  # T3 = E H, Z3 = F G (sums of two)
    # limb extremes: 0 - max and max - 0 in every limb, against maximal unsigned operands
    mx = top + [(2 * P - 1) >> (LB * (NL - 1))]
    neg = [(-x) & 0xFFFFFFFF for x in mx]
    s_max = [2 * x for x in mx]
    for a in (mx, neg):
        for b in (mx, neg, s_max):
            cases.append((a, b))
    for a, b in cases:
        r = fe_mul_sd_exact(a, b)
        v = value_of(r)
        assert v % P == sval(a) * sval(b) * Rinv % P
        assert 0 <= v < 2 * P and all(x <= MASK for x in r[:NL - 1])


def test_halved_record_is_the_same_point():
    """pt_madd with the halved record ((y-x)/2, (y+x)/2, d t) and D = Z1 returns the textbook
    add-2008-hwcd-3 sum (2d, D = 2 Z1) scaled by 1/4: the same projective point."""
    import random
    rnd = random.Random(3)
    d = 3021
    inv2 = pow(2, -1, P)
    for _ in range(50):
        X1, Y1, Z1 = (rnd.randrange(1, P) for _ in range(3))
        T1 = X1 * Y1 * pow(Z1, -1, P) % P
        x2, y2 = rnd.randrange(1, P), rnd.randrange(1, P)
        t2 = x2 * y2 % P
        # textbook
        A = (Y1 - X1) * (y2 - x2); Bv = (Y1 + X1) * (y2 + x2); C = T1 * 2 * d * t2; D = 2 * Z1
        E, F, G, H = Bv - A, D - C, D + C, Bv + A
        ref = [v % P for v in (E * F, G * H, E * H, F * G)]
        # halved record, D = Z1
        A = (Y1 - X1) * (y2 - x2) * inv2; Bv = (Y1 + X1) * (y2 + x2) * inv2; C = T1 * d * t2; D = Z1
        E, F, G, H = Bv - A, D - C, D + C, Bv + A
        got = [v % P for v in (E * F, G * H, E * H, F * G)]
        assert all(g * 4 % P == r for g, r in zip(got, ref))


def padd_operands():
    """pt_add_quad's operands (U-form differences, as before pt_add moved to the V form)."""
    p = q = PT
    A = fe_mul(fe_sub_u(p["Y"], p["X"]), fe_sub(q["Y"], q["X"]))
    Bv = fe_mul(fe_add(p["Y"], p["X"]), fe_add(q["Y"], q["X"]))
    C = fe_mul_2d(fe_mul(p["T"], q["T"]))
    D0 = fe_mul(p["Z"], q["Z"])
    D = fe_add(D0, D0)
    E = fe_sub_u(Bv, A)
    F = fe_sub(D, C)
    G = fe_add(D, C)
    H = fe_add(Bv, A)
    return E, F, G, H


def test_padd_bounds():
    p = q = PT
    A = fe_mul(fe_sub_v(p["Y"], p["X"]), fe_sub_v(q["Y"], q["X"]), WIDE_EF)
    Bv = fe_mul(fe_add(p["Y"], p["X"]), fe_add(q["Y"], q["X"]))
    C = fe_mul_2d(fe_mul(p["T"], q["T"]))
    D0 = fe_mul(p["Z"], q["Z"])
    D = fe_add(D0, D0)
    E = fe_sub_v(Bv, A)
    F = fe_sub(D, C)
    G = fe_add(D, C)
    H = fe_add(Bv, A)
    fe_mul(E, F)
    fe_mul(G, H, WIDE_GH)
    fe_mul(E, H)
    fe_mul(F, G)


def test_mul_2d_exact_and_bounded():
    import random
    rnd = random.Random(11)
    vals = [0, 1, P - 1, P, 2 * P - 1, (1 << 254) - 1, (1 << 253), (1 << 252) - 1]
    vals += [rnd.randrange(0, 2 * P) for _ in range(20000)] + [rnd.randrange(0, 1 << 254) for _ in range(5000)]
    # values straddling every Barrett boundary q p of 6042 v
    for q in range(0, 6042 * 2, 97):
        for dv in (-2, -1, 0, 1):
            x = (q * P) // K2D_INT + dv
            if 0 <= x < 1 << 254:
                vals.append(x)
    for v in vals:
        limbs, r = fe_mul_2d_exact(v)
        assert r % P == (K2D_INT * v) % P
        assert 0 <= r < 3 * P
        assert all(x <= MASK for x in limbs[:NL - 1])


def test_mul_d_exact_and_below_2p():
    # k_prepare_points: d t = fe_mul_d(fe_mul(x + x, y + y)); the result must be normalised and
    # < 2p like an fe_mul output (pt_madd's C and kt_neg_if's 5p - kt rely on it)
    import random
    rnd = random.Random(12)
    vals = [0, 1, P - 1, P, 2 * P - 1, (1 << 254) - 1, (1 << 253), (1 << 252) - 1]
    vals += [rnd.randrange(0, 2 * P) for _ in range(20000)] + [rnd.randrange(0, 1 << 254) for _ in range(5000)]
    for q in range(0, KD_INT * 2 + 2, 7):  # every Barrett boundary q p of 3021 v, both sides
        for dv in (-2, -1, 0, 1):
            x = (q * P) // KD_INT + dv
            if 0 <= x < 1 << 254:
                vals.append(x)
    for v in vals:
        limbs, r = fe_mul_d_exact(v)
        assert r % P == (KD_INT * v) % P
        assert 0 <= r < 2 * P, (v, r)
        assert all(x <= MASK for x in limbs[:NL - 1])
    # the multiply before it: two doubled fe_mul outputs (S form, value < 4p) meet in fe_mul
    x2 = fe_add(B.normalised(2 * P - 1), B.normalised(2 * P - 1))
    fe_mul(x2, x2)


def test_quad_add_bounds():
    # pt_add_quad: round 1 A | B | T1T2 | Z1Z2 on the four lanes, C = fe_mul_2d(T1T2) on lane 2,
    # then EF | GH | EH | FG -- the same operands as pt_add, through one multiply whose wide steps
    # suit all four (WIDE_GH & WIDE_EH)
    E, F, G, H = padd_operands()
    for a, b in ((E, F), (G, H), (E, H), (F, G)):
        fe_mul(a, b, WIDE_GH & WIDE_EH)


def test_wide_masks_are_maximal():
    """The masks in fp29.cuh are the widest the column budget allows for their operand forms."""
    N = N_MUL
    G, H, E, V = fe_add(fe_add(N, N), N), fe_add(N, N), fe_sub_u(N, N), fe_sub_v(N, N)
    for (a, b), mask in (((G, H), WIDE_GH), ((E, H), WIDE_EH), ((V, V), WIDE_EF)):
        fe_mul(a, b, mask)
        for extra in range(8):
            if not (mask >> extra) & 1:
                try:
                    fe_mul(a, b, mask | 1 << extra)
                except AssertionError:
                    continue
                raise AssertionError(f"mask {mask:#x} could also widen step {extra}")


def test_fe_mul_exact_model():
    """Bit-exact model of fe_mul_w: a b R^-1 mod p, normalised limbs, value < 2p -- random
    operands and operands at the limb maxima of each call site's forms."""
    import random
    rnd = random.Random(5)
    Rinv = pow(R, -1, P)

    def limbs_of(v):
        return [(v >> (LB * i)) & MASK for i in range(NL - 1)] + [v >> (LB * (NL - 1))]

    cases = []
    for _ in range(3000):
        cases.append((limbs_of(rnd.randrange(2 * P)), limbs_of(rnd.randrange(2 * P)), rnd.choice(
            (WIDE_ALL, WIDE_GH, WIDE_EH, WIDE_EF, WIDE_GH & WIDE_EH, 0))))
    # unnormalised operands at their forms' maxima (value = sum of limbs 2^(29 i), kept < 2^257)
    top = (1 << 257) >> (LB * (NL - 1))
    s_max = [(1 << 30) - 1] * (NL - 1) + [top // 2]
    g_max = [3 * (1 << 29) // 2] * (NL - 1) + [top // 4]
    u_max = [x + k - 1 for x, k in zip([0] * NL, K8P29)]
    v_max = [MASK + k for k in K5P29[:NL - 1]] + [((2 * P) >> (LB * (NL - 1))) + K5P29[NL - 1]]
    for a, b, w in ((g_max, s_max, WIDE_GH), (u_max, s_max, WIDE_EH), (s_max, s_max, WIDE_ALL),
                    (v_max, v_max, WIDE_EF), (v_max, s_max, WIDE_ALL)):
        cases.append((a, b, w))
    for a, b, w in cases:
        r = fe_mul_exact(a, b, w)
        v = value_of(r)
        assert v % P == value_of(a) * value_of(b) * Rinv % P
        assert v < 2 * P and all(x <= MASK for x in r[:NL - 1])


def test_pdbl_bounds():
    p = PT
    A = fe_mul(p["X"], p["X"])
    Bv = fe_mul(p["Y"], p["Y"])
    Z2 = fe_mul(p["Z"], p["Z"])
    C = fe_norm(fe_add(Z2, Z2))
    S = fe_mul(fe_add(p["X"], p["Y"]), fe_add(p["X"], p["Y"]))
    E = fe_sub(fe_sub(S, A), Bv)
    G = fe_sub(Bv, A)
    F = fe_sub(G, C)
    AB = fe_norm(fe_add(A, Bv))
    H = fe_norm(fe_sub_u(B([0] * NL, 0), AB))
    fe_mul(E, F)
    fe_mul(G, H)
    fe_mul(E, H)
    fe_mul(F, G)


def test_model_matches_header_constants():
    assert value_of(K8P29) == 8 * P
    assert all(k >= MASK for k in K8P29[:8])
    assert value_of(K5P29) == 5 * P
    assert all(k >= MASK for k in K5P29[:8]) and K5P29[8] >= (2 * P - 1) >> (LB * 8)
    assert P29 == [1, 277610496, 66, 351141280, 452990362, 110046747, 358187729, 198395284, 1223525]


# --- the proof above mirrors these device functions by hand.  Their normalised source text is
# pinned here, so editing any of them fails this test until the mirrored formulas (and this
# table) are re-reviewed.  Regenerate a digest with _body_digest(<file>, <name>).
import hashlib  # noqa: E402
import os  # noqa: E402
import re  # noqa: E402

_CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "webgpu-msm_amd", "csrc")
REVIEWED = {
    ("fp29.cuh", "mad64"): "b50540a0d8a64ede",
    ("fp29.cuh", "seeded"): "d5de263bcd90d0e8",
    ("fp29.cuh", "fe_mul"): "cb1d67f3d0051cb5",
    ("fp29.cuh", "fe_mul_w"): "9fc551211780fac2",
    ("fp29.cuh", "fe_mul_seed"): "d98e5e7e34126a6e",
    ("fp29.cuh", "fe_norm"): "37b756e7bd4474d2",
    ("fp29.cuh", "fe_add"): "d14b6a137a6ff34d",
    ("fp29.cuh", "fe_add_n"): "bdf7dd24032e38f7",
    ("fp29.cuh", "fe_dbl_n"): "07019b3ba4e2775f",
    ("fp29.cuh", "fe_sub"): "ea72835f159885cc",
    ("fp29.cuh", "fe_sub_u"): "3dba987a0530b5b5",
    ("fp29.cuh", "fe_neg"): "a754b1a94a6b8415",
    ("fp29.cuh", "fe_mul_2d"): "b9f5c6afdcbc7ff4",
    ("fp29.cuh", "fe_mul_d"): "be44d19d0395d3fb",
    ("fp29.cuh", "P29"): "b4babf5a3c9d7331",
    ("fp29.cuh", "K8P29"): "13315f5ba6ec470d",
    ("fp29.cuh", "K5P29"): "f3dc542f8a39d740",
    ("fp29.cuh", "fe_sub_v"): "b95cf1f871e652b6",
    ("fp29.cuh", "fe_sub_s"): "2394a6c588a7e363",
    ("fp29.cuh", "smad64"): "f570120e573dc55c",
    ("fp29.cuh", "SD_OFF58"): "c88a1438ac9f5b80",
    ("fp29.cuh", "fe_mul_sd_seed"): "d2395c468f273ed7",
    ("fp29.cuh", "opaque_v"): "9936fb9d6abd51ca",
    ("fp29.cuh", "fe_mul_sd"): "1524d4c9c2554e87",
    ("ec.cuh", "pt_madd"): "940afc2112f7fd6f",
    ("ec.cuh", "pt_add"): "1449f0a88822c610",
    ("ec.cuh", "pt_dbl"): "784353f9934ef437",
    ("ec.cuh", "kt_neg_if"): "19c79f3cf45dee09",
    ("ec.cuh", "pt_add_quad"): "875eba21c1f11e82",
}


def _body(fname, name):
    src = open(os.path.join(_CSRC, fname)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"//[^\n]*", "", src)
    m = re.search(r"[^\n;{}]*\b" + re.escape(name) + r"\b\s*(\[[^\]]*\])?\s*(\([^)]*\))?\s*(=\s*)?\{", src)
    assert m, f"{name} not found in {fname}"
    i, depth = m.end() - 1, 0
    for j in range(i, len(src)):
        depth += {"{": 1, "}": -1}.get(src[j], 0)
        if depth == 0:
            return " ".join((src[m.start():j + 1]).split())
    raise AssertionError(f"unbalanced braces after {name} in {fname}")


def _body_digest(fname, name):
    return hashlib.sha256(_body(fname, name).encode()).hexdigest()[:16]


def test_mirrored_sources_unchanged():
    changed = {f"{f}:{n}": _body_digest(f, n) for (f, n), d in REVIEWED.items() if _body_digest(f, n) != d}
    assert not changed, ("device code mirrored by this proof changed -- re-check the formulas above, then update "
                         f"REVIEWED with: {changed}")


def test_wide_mask_constants_match_header():
    src = open(os.path.join(_CSRC, "fp29.cuh")).read()
    got = {k: int(v, 16) for k, v in re.findall(r"constexpr uint32_t (WIDE_[A-Z]+) = (0x[0-9A-Fa-f]+)u;", src)}
    assert got == {"WIDE_ALL": WIDE_ALL, "WIDE_GH": WIDE_GH, "WIDE_EH": WIDE_EH, "WIDE_EF": WIDE_EF}
