// Base-field arithmetic for Edwards-BLS12 on gfx950: Fq with
//   p = 8444461749428370424248824938781546531375899335154063827935233455917409239041 (253 bits)
// (reference: src/reference/params/AleoConstants.ts:2, src/submission/wgsl/field_modulus.wgsl:7-10).
//
// Representation ("fe"): 9 unsaturated limbs of 29 bits held in u32 VGPRs, Montgomery form with
// R = 2^261.  Why not 8x32: on gfx950 v_mad_u64_u32 issues at ~4 cycles/wave but every 32-bit
// CIOS step also needs carry adds (v_addc + VCC hazards); with 29-bit limbs a 9x9 product
// accumulates up to 18 partial products per 64-bit column with no carry handling at all, so
// the whole multiply is 153 independent v_mad_u64_u32 plus a short carry pass.  Measured
// (tools/ubench/fmul_bench.hip, MI355X): 168 Gmul/s chip-wide vs 104 Gmul/s for 8x32 CIOS.
//
// Laziness: R = 2^261 >> p, so the Montgomery product of any a, b < 2^257 (~16p) is < 2p and
// needs no final subtraction.  Additions are limb-wise with no carry; subtractions add a
// redundant multiple of p whose limbs dominate any normalised limb, then renormalise.
// Limb forms: "N" = normalised (limbs < 2^29), "S" = sum of two N (limbs < 2^30), "U" = an
// unnormalised difference over 8p (limbs < 1.48 * 2^30), "V" = one over 5p (limbs < 1.43 * 2^30,
// fe_sub_v).  Each 64-bit column holds up to 9 limb products
// plus the reduction products (fe_mul_w: up to 2^32 * p_j), so which operand forms may meet is
// decided per call site by tests/test_limb_bounds.py (every column < 2^64, worst case over the
// per-limb maxima).  Values entering fe_mul stay < 2^257.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace msm {

constexpr int NL = 9;
constexpr uint32_t LBITS = 29;
constexpr uint32_t LMASK = (1u << 29) - 1;

struct fe {
  uint32_t v[NL];
};

// p in 29-bit limbs (little-endian).  p ≡ 1 (mod 2^29) so -p^-1 mod 2^29 = 2^29-1: the
// Montgomery quotient digit is m = (-t) mod 2^29 and m*p_0 = m (no multiply).
__device__ constexpr uint32_t P29[NL] = {1u, 277610496u, 66u, 351141280u, 452990362u,
                                         110046747u, 358187729u, 198395284u, 1223525u};
// R^2 mod p (to enter Montgomery form from a standard-form integer).
__device__ constexpr uint32_t R2_29[NL] = {102099907u, 496719628u, 421467643u, 16176098u, 367912240u,
                                           263044200u, 69768239u, 111235120u, 824440u};
// R mod p = Montgomery form of 1.
__device__ constexpr uint32_t ONE29[NL] = {536870474u, 276299775u, 536841777u, 282071103u, 232458597u,
                                           117906524u, 416951824u, 75953059u, 966800u};
// The point records hold the precomputed affine point halved, ((y-x)/2, (y+x)/2, d*t) (ec.cuh
// pt_madd), built straight from standard-form coordinates with these:
// R^2/2 mod p: fe_mul(a_std, R2H_29) = Montgomery form of a/2.
__device__ constexpr uint32_t R2H_29[NL] = {51049954u, 118729606u, 210733855u, 183658689u, 142015845u,
                                            186545474u, 213977984u, 423250658u, 1023982u};
// R/2 mod p: Montgomery form of 1/2.
__device__ constexpr uint32_t HALF29[NL] = {536870693u, 406585343u, 536856344u, 409471007u, 116229298u,
                                            58953262u, 476911368u, 37976529u, 483400u};
// d*R^2 mod p: fe_mul(t_std, KD_R2_29) = Montgomery form of d*t (d = 3021).
__device__ constexpr uint32_t KD_R2_29[NL] = {279913524u, 423508698u, 332684583u, 15420509u, 112057194u,
                                              17618952u, 475123559u, 489499438u, 759738u};
// d*R mod p: Montgomery form of d.
__device__ constexpr uint32_t KD29[NL] = {535545327u, 246677503u, 448696855u, 3926111u, 291341u,
                                          98484521u, 353554619u, 160914044u, 148170u};
// 2^256 mod p (standard form): fe_mul(a_mont, R256_29) = a * 2^256 mod p, i.e. the host's
// 4x64-bit Montgomery representation (hostfield.h, R = 2^256) of a.
__device__ constexpr uint32_t R256_29[NL] = {536870899u, 149159935u, 536870047u, 267001567u, 16705317u,
                                             180005014u, 175397728u, 105215859u, 871386u};
// 8p in a redundant form with limbs 0..7 >= 2^29-1, so (a + K8P - b) never goes negative limb-wise
// for normalised b.
__device__ constexpr uint32_t K8P29[NL] = {536870920u, 610271231u, 536871443u, 661646591u, 939568340u,
                                           880373981u, 718018184u, 1050291364u, 9788201u};
// 5p in a redundant form with limbs 0..7 >= 2^29-1 and limb 8 above the top limb of any value
// < 2p, so (a + K5P - b) never goes negative limb-wise for b an fe_mul output: pt_madd's
// differences (the "V" form, fe_sub_v), whose small limbs let them meet each other in a multiply.
__device__ constexpr uint32_t K5P29[NL] = {536870917u, 851181567u, 536871243u, 681964575u, 654339076u,
                                           550233738u, 717196821u, 991976422u, 6117625u};

__device__ __forceinline__ uint64_t mad64(uint32_t a, uint32_t b, uint64_t c) {
  return (uint64_t)a * b + c;
}

// Pins a seeded product: an empty asm on the result keeps LLVM from reassociating the seed out
// of the multiply-add (it would otherwise add it separately, one 64-bit add per column).
__device__ __forceinline__ uint64_t seeded(uint64_t x) {
  asm("" : "+v"(x));
  return x;
}

__device__ __forceinline__ void fe_set(fe& r, const uint32_t* c) {
#pragma unroll
  for (int i = 0; i < NL; i++) r.v[i] = c[i];
}
__device__ __forceinline__ fe fe_const(const uint32_t* c) {
  fe r;
  fe_set(r, c);
  return r;
}
__device__ __forceinline__ fe fe_zero() {
  fe r;
#pragma unroll
  for (int i = 0; i < NL; i++) r.v[i] = 0;
  return r;
}
__device__ __forceinline__ fe fe_one() { return fe_const(ONE29); }

// Montgomery product a*b*2^-261 mod p (result normalised, value < 2p when a,b < 2^257).
//
// Reduction digits (p = 1 mod 2^29, so m * p_0 = m).  Every reduction column k = 0..8 is seeded
// with 2^32 - 1, so its register holds s_k = c_k + 2^32 - 1 (c_k = the true column, >= 0).  Step
// k is one of two kinds (bit k of WIDE):
//  * wide (k <= 7): a full 32-bit digit m_k = ~lo(s_k) (one v_not).  Then c_k + m_k = 2^32 hi(s_k)
//    exactly, i.e. the column is zero to 32 bits and its carry into column k+1 (units of 2^29) is
//    8 hi(s_k): ONE v_mad_u64_u32 (hi, 8, s_{k+1}) -- no 64-bit shift and add.
//  * narrow: m_k = ~lo(s_k) mod 2^29 = 2^29 - 1 - ((c_k - 1) mod 2^29) zeroes the column to 29
//    bits; its carry is (s_k >> 29) - 7, added as s_k >> 29 (64-bit shift + add) with the -7
//    pre-seeded into column k+1.  The last step (k = 8) is always narrow: the digits' share of
//    the result is sum_k m_k 2^(29k) p / 2^261, so a 32-bit m_8 would add up to 8p, while 32-bit
//    digits below it add at most 2^-26 p -- the result stays < 2p.
// A 32-bit digit makes its reduction products 8x larger, so the columns near the middle only fit
// 64 bits for the narrower operand forms: WIDE_ALL for N/S/U/V x N operands, S x S and V x S,
// fewer wide steps for the V x V products (pt_madd's E F, pt_add's A) and for the products with
// an S operand against a 1.5-form or U one (tests/test_limb_bounds.py proves every call site's
// columns < 2^64).
#ifndef MSM_NARROW_DIGITS  // A/B builds only: -DMSM_NARROW_DIGITS gives every step a 29-bit digit
constexpr uint32_t WIDE_ALL = 0xFFu;  // steps 0..7 wide
constexpr uint32_t WIDE_GH = 0xE7u;   // steps 0, 1, 2, 5, 6, 7: G (< 1.5 * 2^30 limbs) x H (S)
constexpr uint32_t WIDE_EH = 0xBFu;   // steps 0..5, 7:          E (U) x H (S) (pt_add_quad)
constexpr uint32_t WIDE_EF = 0xEFu;   // steps 0..3, 5..7:       pt_madd's E (V) x F (V)
#else
constexpr uint32_t WIDE_ALL = 0u, WIDE_GH = 0u, WIDE_EH = 0u, WIDE_EF = 0u;
#endif

__host__ __device__ constexpr uint64_t fe_mul_seed(uint32_t wide, int k) {
  // column k's register offset: 2^32 - 1 for the reduction columns, minus 7 after a narrow step
  return (k <= NL - 1 ? 0xFFFFFFFFull : 0ull) - ((k >= 1 && !((wide >> (k - 1)) & 1u)) ? 7ull : 0ull);
}

// An opaque 32-bit value held in an SGPR: the multiplier of the wide steps' carry product, so
// LLVM keeps 8 hi(s) + s' one v_mad_u64_u32 instead of rewriting it as shifts and masks.
__device__ __forceinline__ uint32_t opaque_s(uint32_t v) {
  asm("" : "+s"(v));
  return v;
}

template <uint32_t WIDE>
__device__ __forceinline__ fe fe_mul_w(const fe& a, const fe& b) {
  uint64_t c[2 * NL];
  const uint32_t eight = opaque_s(8u);
  // Each column is one chain of multiply-adds starting from its seed.  Every link is pinned
  // (seeded): LLVM's reassociation would otherwise sum the products first and add the seed (or
  // the carry) with a separate 64-bit add.
#pragma unroll
  for (int k = 0; k < NL; k++) c[k] = seeded(mad64(a.v[0], b.v[k], fe_mul_seed(WIDE, k)));
  c[NL] = seeded(mad64(a.v[1], b.v[NL - 1], fe_mul_seed(WIDE, NL)));
#pragma unroll
  for (int k = NL + 1; k < 2 * NL; k++) c[k] = 0;
#pragma unroll
  for (int i = 1; i < NL; i++)
#pragma unroll
    for (int j = 0; j < NL; j++) {
      if (i == 1 && j == NL - 1) continue;  // issued above as a seeded product
      c[i + j] = i + j > NL ? mad64(a.v[i], b.v[j], c[i + j]) : seeded(mad64(a.v[i], b.v[j], c[i + j]));
    }
#pragma unroll
  for (int i = 0; i < NL; i++) {
    const uint32_t lo = (uint32_t)c[i];
    uint32_t m;
    if (i < NL - 1 && ((WIDE >> i) & 1u)) {
      m = ~lo;
      c[i + 1] = seeded(mad64((uint32_t)(c[i] >> 32), eight, c[i + 1]));
    } else {
      m = ~lo & LMASK;
      c[i + 1] += c[i] >> LBITS;
    }
#pragma unroll
    for (int j = 1; j < NL; j++) c[i + j] = mad64(m, P29[j], c[i + j]);
  }
  fe r;
#pragma unroll
  for (int k = NL; k < 2 * NL - 1; k++) {
    c[k + 1] += c[k] >> LBITS;
    r.v[k - NL] = (uint32_t)c[k] & LMASK;
  }
  r.v[NL - 1] = (uint32_t)c[2 * NL - 1];
  return r;
}

// ---- signed differences (pt_madd) -------------------------------------------------------------
// pt_madd's differences are plain limb-wise subtractions with no redundant multiple of p: their
// limbs are two's-complement integers (|limb| < 2^29 for normalised operands, the top limb
// signed), legal only as fe_mul_sd operands.  That saves the 5p offset's nine additions per
// difference.  fe_mul_sd multiplies them with signed 32 x 32 -> 64 products (v_mad_i64_i32, the
// same issue rate as the unsigned ones), takes its carries as arithmetic shifts, and keeps its
// result non-negative by a bias: DELTA_SD p 2^232 joins the product through the seeds of columns
// 8..16 (free: they start multiply-add chains), raising the result by DELTA_SD p / 2^29 = p / 8,
// more than the most negative |a b| / 2^261 of its call sites.  The result is then an ordinary
// fe_mul output (normalised, value in [0, 2p)).  tests/test_limb_bounds.py (fe_mul_sd) proves every
// column register within int64 and the result range, per call site.
__device__ __forceinline__ fe fe_sub_s(const fe& a, const fe& b) {
  fe r;
#pragma unroll
  for (int i = 0; i < NL; i++) r.v[i] = a.v[i] - b.v[i];
  return r;
}

constexpr uint32_t DELTA_SD_LOG = 26;  // DELTA_SD = 2^26

__device__ __forceinline__ uint64_t smad64(uint32_t a, uint32_t b, uint64_t c) {
  return (uint64_t)((int64_t)(int32_t)a * (int64_t)(int32_t)b) + c;
}

// With signed products a column's true range is lopsided (the reduction terms are non-negative
// and reach ~1.3 * 2^63 in the middle columns), so every column register also carries an offset
// O_k = SD_OFF58[k] * 2^58 that centres its range in int64.  O_k is a multiple of 2^32, so the
// low word (the reduction digit) is untouched and the carry out grows by exactly O_k / 2^29,
// which the next column's seed takes back.
__device__ constexpr int8_t SD_OFF58[2 * NL] = {-1, -3, -3, -5, -9, -9, -12, -14, -14, -12, -11, -9, -6, -5, -2, -1, -1, 0};

__device__ constexpr uint64_t fe_mul_sd_seed(uint32_t wide, int k, uint32_t p_k8) {
  // fe_mul_seed's register offset, the bias DELTA_SD p_(k-8) on columns 8..16, and the centring
  // offset O_k less the previous column's O_(k-1) / 2^29 (its carry's excess)
  return (k <= NL ? fe_mul_seed(wide, k) : 0ull) + ((k >= NL - 1 && k < 2 * NL - 1) ? (uint64_t)p_k8 << DELTA_SD_LOG : 0ull) +
         (uint64_t)((int64_t)SD_OFF58[k] * (1ll << 58)) -
         (k >= 1 ? (uint64_t)((int64_t)SD_OFF58[k - 1] * (1ll << 29)) : 0ull);
}

// a b 2^-261 mod p with a signed (fe_sub_s) and b signed too (SB) or an unsigned form < 2^31.
__device__ __forceinline__ uint32_t opaque_v(uint32_t v) {
  asm("" : "+v"(v));
  return v;
}

template <uint32_t WIDE, bool SB>
__device__ __forceinline__ fe fe_mul_sd(const fe& a_in, const fe& b_in) {
  // Operands through an empty asm: LLVM otherwise proves some limbs non-negative (masked) and
  // lowers their sign-extended products as unsigned products plus sign corrections.
  fe a, b;
#pragma unroll
  for (int i = 0; i < NL; i++) {
    a.v[i] = opaque_v(a_in.v[i]);
    b.v[i] = opaque_v(b_in.v[i]);
  }
  uint64_t c[2 * NL];
  const uint32_t eight = opaque_s(8u);
#define MSM_SD_SEED(k) fe_mul_sd_seed(WIDE, (k), (k) >= NL - 1 && (k) < 2 * NL - 1 ? P29[(k) - (NL - 1)] : 0u)
#pragma unroll
  for (int k = 0; k < NL; k++) c[k] = seeded(smad64(a.v[0], b.v[k], MSM_SD_SEED(k)));
  c[NL] = seeded(smad64(a.v[1], b.v[NL - 1], MSM_SD_SEED(NL)));
#pragma unroll
  for (int k = NL + 1; k < 2 * NL; k++) c[k] = MSM_SD_SEED(k);
#undef MSM_SD_SEED
#pragma unroll
  for (int i = 1; i < NL; i++)
#pragma unroll
    for (int j = 0; j < NL; j++) {
      if (i == 1 && j == NL - 1) continue;  // issued above as a seeded product
      c[i + j] = seeded(smad64(a.v[i], b.v[j], c[i + j]));
    }
#pragma unroll
  for (int i = 0; i < NL; i++) {
    const uint32_t lo = (uint32_t)c[i];
    uint32_t m;
    if (i < NL - 1 && ((WIDE >> i) & 1u)) {
      m = ~lo;
      c[i + 1] = seeded(smad64((uint32_t)(c[i] >> 32), eight, c[i + 1]));  // 8 * (signed high word)
    } else {
      m = ~lo & LMASK;
      c[i + 1] += (uint64_t)((int64_t)c[i] >> LBITS);
    }
#pragma unroll
    for (int j = 1; j < NL; j++) c[i + j] = mad64(m, P29[j], c[i + j]);
  }
  fe r;
#pragma unroll
  for (int k = NL; k < 2 * NL - 1; k++) {
    c[k + 1] += (uint64_t)((int64_t)c[k] >> LBITS);
    r.v[k - NL] = (uint32_t)c[k] & LMASK;
  }
  r.v[NL - 1] = (uint32_t)c[2 * NL - 1];
  return r;
}

// Every operand pair but the S x (1.5 | U) products named above: all eight low digits wide.
__device__ __forceinline__ fe fe_mul(const fe& a, const fe& b) { return fe_mul_w<WIDE_ALL>(a, b); }

__device__ __forceinline__ fe fe_sqr(const fe& a) { return fe_mul(a, a); }

// 2d * a = 6042 a (mod p), lazily: add-2008-hwcd-3's "k * (T1 T2)" without a full multiply.  The
// Montgomery form commutes with an integer factor, so the limbs are simply scaled (one 42-bit
// product per limb, carried), then v = 6042 a < 2^267 is reduced by q p with a Barrett digit from
// its top bits: q0 = floor(v / 2^252) < 2^15, q = floor(q0 * MU2D / 2^32) with
// MU2D = floor(2^284 / p), so 0 <= v - q p < 2.86 p (q never exceeds floor(v / p)).
// Requires a normalised with value < 2^254 (any fe_mul output); returns normalised, value < 3p.
// ~50 VALU instructions instead of fe_mul's ~190.  tests/test_limb_bounds.py re-derives the bounds.
constexpr uint32_t K2D_INT = 6042;
constexpr uint32_t MU2D = 3680838779u;  // floor(2^284 / p)
__device__ __forceinline__ fe fe_mul_2d(const fe& a) {
  fe r;
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < NL - 1; i++) {
    c = mad64(a.v[i], K2D_INT, c);
    r.v[i] = (uint32_t)c & LMASK;
    c >>= LBITS;
  }
  c = mad64(a.v[NL - 1], K2D_INT, c);  // limb 8 of v (bits 232..), < 2^36
  const uint32_t q = __umulhi((uint32_t)(c >> 20), MU2D);
  int64_t d = 0;
#pragma unroll
  for (int i = 0; i < NL - 1; i++) {
    d += (int64_t)r.v[i] - (int64_t)q * (int64_t)P29[i];
    r.v[i] = (uint32_t)d & LMASK;
    d >>= LBITS;  // arithmetic: borrows propagate
  }
  r.v[NL - 1] = (uint32_t)(d + (int64_t)c - (int64_t)q * (int64_t)P29[NL - 1]);
  return r;
}

// d * a = 3021 a (mod p) with the result below 2p (the bound of an fe_mul output), for
// k_prepare_points' d t = d x y (one fe_mul fewer than multiplying by the Montgomery form of d).
// Limbs scaled as in fe_mul_2d, then v = 3021 a < 2^266 (a < 2^254) is reduced by q p with
// q = floor(floor(v / 2^240) * MU272 / 2^32), MU272 = floor(2^272 / p): the two truncations
// cost less than 0.06 of a unit, so q is floor(v / p) or one less and 0 <= v - q p < 2p.
// Requires a normalised; returns normalised.  tests/test_limb_bounds.py models it bit-exactly.
constexpr uint32_t KD_INT = 3021;
constexpr uint32_t MU272 = 898642u;  // floor(2^272 / p)
__device__ __forceinline__ fe fe_mul_d(const fe& a) {
  fe r;
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < NL - 1; i++) {
    c = mad64(a.v[i], KD_INT, c);
    r.v[i] = (uint32_t)c & LMASK;
    c >>= LBITS;
  }
  c = mad64(a.v[NL - 1], KD_INT, c);  // v = c 2^232 + (limbs 0..7), c < 2^34
  const uint32_t q = (uint32_t)(((c >> 8) * (uint64_t)MU272) >> 32);
  int64_t d = 0;
#pragma unroll
  for (int i = 0; i < NL - 1; i++) {
    d += (int64_t)r.v[i] - (int64_t)q * (int64_t)P29[i];
    r.v[i] = (uint32_t)d & LMASK;
    d >>= LBITS;  // arithmetic: borrows propagate
  }
  r.v[NL - 1] = (uint32_t)(d + (int64_t)c - (int64_t)q * (int64_t)P29[NL - 1]);
  return r;
}

// Carry-propagate so limbs 0..7 are < 2^29 (value unchanged).
__device__ __forceinline__ void fe_norm(fe& a) {
#pragma unroll
  for (int i = 0; i < NL - 1; i++) {
    a.v[i + 1] += a.v[i] >> LBITS;
    a.v[i] &= LMASK;
  }
}

// Lazy add: limb-wise, no carry (N+N -> S).
__device__ __forceinline__ fe fe_add(const fe& a, const fe& b) {
  fe r;
#pragma unroll
  for (int i = 0; i < NL; i++) r.v[i] = a.v[i] + b.v[i];
  return r;
}
// a + b, normalised.
__device__ __forceinline__ fe fe_add_n(const fe& a, const fe& b) {
  fe r = fe_add(a, b);
  fe_norm(r);
  return r;
}
// a + a, normalised.
__device__ __forceinline__ fe fe_dbl_n(const fe& a) {
  fe r;
#pragma unroll
  for (int i = 0; i < NL; i++) r.v[i] = a.v[i] << 1;
  fe_norm(r);
  return r;
}
// a - b + 8p, normalised.  Requires b normalised with value < 8p; a limbs < 2^30.
__device__ __forceinline__ fe fe_sub(const fe& a, const fe& b) {
  fe r;
#pragma unroll
  for (int i = 0; i < NL; i++) r.v[i] = a.v[i] + K8P29[i] - b.v[i];
  fe_norm(r);
  return r;
}
// a - b + 8p without renormalisation ("U": limbs < 1.48 * 2^30).  Legal as one fe_mul operand
// against an N or S operand (column bound 0.95 * 2^64), never U*U.
__device__ __forceinline__ fe fe_sub_u(const fe& a, const fe& b) {
  fe r;
#pragma unroll
  for (int i = 0; i < NL; i++) r.v[i] = a.v[i] + K8P29[i] - b.v[i];
  return r;
}
// a - b + 5p without renormalisation ("V": limbs < 2^29 + K5P's).  Requires b an fe_mul output
// (normalised, value < 2p) and a normalised.
__device__ __forceinline__ fe fe_sub_v(const fe& a, const fe& b) {
  fe r;
#pragma unroll
  for (int i = 0; i < NL; i++) r.v[i] = a.v[i] + K5P29[i] - b.v[i];
  return r;
}
// -b (= 8p - b), normalised.
__device__ __forceinline__ fe fe_neg(const fe& b) {
  fe r;
#pragma unroll
  for (int i = 0; i < NL; i++) r.v[i] = K8P29[i] - b.v[i];
  fe_norm(r);
  return r;
}
// Branch-free select: c ? b : a.
__device__ __forceinline__ fe fe_sel(bool c, const fe& a, const fe& b) {
  fe r;
#pragma unroll
  for (int i = 0; i < NL; i++) r.v[i] = c ? b.v[i] : a.v[i];
  return r;
}

// Standard-form little-endian 8x32 word integer (< 2^256) -> 29-bit limbs (not Montgomery).
__device__ __forceinline__ fe fe_from_words_le(const uint32_t w[8]) {
  fe r;
#pragma unroll
  for (int i = 0; i < NL; i++) {
    const int bit = 29 * i, wi = bit >> 5, sh = bit & 31;
    uint32_t lo = w[wi] >> sh;
    uint32_t hi = (sh > 3 && wi + 1 < 8) ? (w[wi + 1] << (32 - sh)) : 0u;
    r.v[i] = (lo | hi) & LMASK;
  }
  return r;
}

// Normalised limbs (value < 2^261) -> little-endian 8x32 words (value must be < 2^256).
__device__ __forceinline__ void fe_to_words_le(const fe& a, uint32_t w[8]) {
#pragma unroll
  for (int k = 0; k < 8; k++) w[k] = 0;
#pragma unroll
  for (int i = 0; i < NL; i++) {
    const int bit = 29 * i, wi = bit >> 5, sh = bit & 31;
    w[wi] |= a.v[i] << sh;
    if (sh > 3 && wi + 1 < 8) w[wi + 1] |= a.v[i] >> (32 - sh);
  }
}

// Compare normalised limbs (value < 2^261) against p: returns true if a >= p.
__device__ __forceinline__ bool fe_geq_p(const fe& a) {
  bool gt = false, eq = true;
#pragma unroll
  for (int i = NL - 1; i >= 0; i--) {
    bool g = a.v[i] > P29[i], l = a.v[i] < P29[i];
    gt = gt || (eq && g);
    eq = eq && !g && !l;
  }
  return gt || eq;
}

// a - p for normalised a >= p (result normalised; borrows handled limb-wise).
__device__ __forceinline__ fe fe_sub_p(const fe& a) {
  fe r;
  int32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < NL; i++) {
    int64_t t = (int64_t)a.v[i] - P29[i] + borrow;
    borrow = t < 0 ? -1 : 0;
    r.v[i] = (uint32_t)(t + (t < 0 ? (1ll << 29) : 0));
  }
  return r;
}

// Montgomery form -> canonical standard form in [0, p) as normalised limbs.
__device__ __forceinline__ fe fe_to_std(const fe& a) {
  fe one = fe_zero();
  one.v[0] = 1;
  fe r = fe_mul(a, one);  // value <= p
  fe_norm(r);
  if (fe_geq_p(r)) r = fe_sub_p(r);
  return r;
}

// Device Montgomery form -> canonical host Montgomery form (a * 2^256 mod p, in [0, p)).
__device__ __forceinline__ fe fe_to_host_mont(const fe& a) {
  fe r = fe_mul(a, fe_const(R256_29));  // value < p + small: one conditional subtraction
  fe_norm(r);
  if (fe_geq_p(r)) r = fe_sub_p(r);
  return r;
}

// Standard-form words (< 2^256) -> Montgomery form (normalised, < 2p).
__device__ __forceinline__ fe fe_to_mont(const fe& std_limbs) { return fe_mul(std_limbs, fe_const(R2_29)); }

// Check a standard-form 256-bit value (LE words) is < p.
__device__ __forceinline__ bool words_lt_p(const uint32_t w[8]) {
  const uint32_t PW[8] = {0x00000001u, 0x0a118000u, 0xd0000001u, 0x59aa76feu,
                          0x5c37b001u, 0x60b44d1eu, 0x9a2ca556u, 0x12ab655eu};
  // w < p iff w - p borrows: one subtract-with-borrow per word (v_sub_co / v_subb_co)
  unsigned int b = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) (void)__builtin_subc(w[i], PW[i], b, &b);
  return b != 0;
}

// Inverse by Fermat (a^(p-2)); only used on the rare z != 1 input path.
__device__ inline fe fe_inv(const fe& a) {
  // p - 2 as little-endian words
  const uint32_t E[8] = {0xffffffffu, 0x0a117fffu, 0xd0000001u, 0x59aa76feu,
                         0x5c37b001u, 0x60b44d1eu, 0x9a2ca556u, 0x12ab655eu};
  fe r = fe_one();
  for (int wi = 7; wi >= 0; wi--) {
    for (int b = 31; b >= 0; b--) {
      r = fe_sqr(r);
      if ((E[wi] >> b) & 1u) r = fe_mul(r, a);
    }
  }
  return r;
}

}  // namespace msm
