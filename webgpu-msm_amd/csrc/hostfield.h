// Host-side Fq / Edwards arithmetic for the serial tail of the MSM (window Horner, affine
// conversion, shard combine).  4 x 64-bit Montgomery limbs, R = 2^256.  The device uses a
// different representation (9 x 29-bit, R = 2^261, fp29.cuh); the two only meet through
// canonical standard-form integers.
//
// Replaces the reference's arkworks calls in reduce_last / point_add_affine
// (src/submission/msm-wasm/src/lib.rs:88-104, 240-253) and write_fq (bytes.rs:33-44).
#pragma once
#include <stdint.h>
#include <string.h>
#include <x86intrin.h>

namespace msmh {

typedef unsigned __int128 u128;

struct Fq {
  uint64_t l[4];  // Montgomery form, little-endian limbs, value in [0, p)
};

static const uint64_t P[4] = {0x0a11800000000001ULL, 0x59aa76fed0000001ULL, 0x60b44d1e5c37b001ULL,
                              0x12ab655e9a2ca556ULL};
static const uint64_t NP = 0x0a117fffffffffffULL;  // -p^-1 mod 2^64
static const uint64_t RMODP[4] = {0x7d1c7ffffffffff3ULL, 0x7257f50f6ffffff2ULL, 0x16d81575512c0feeULL,
                                  0x0d4bda322bbb9a9dULL};
static const uint64_t R2MODP[4] = {0x25d577bab861857bULL, 0xcc2c27b58860591fULL, 0xa7cc008fe5dc8593ULL,
                                   0x011fdae7eff1c939ULL};
static const uint64_t K2D_M[4] = {0x967e7ffffffebc5fULL, 0x87a7a94f2ffeafa4ULL, 0xb14e318dbde89b04ULL,
                                  0x014ee2fab55008a9ULL};  // 2d * R mod p

static inline bool geq_p(const uint64_t a[4]) {
  for (int i = 3; i >= 0; i--) {
    if (a[i] > P[i]) return true;
    if (a[i] < P[i]) return false;
  }
  return true;
}
static inline void sub_p(uint64_t a[4]) {
  u128 borrow = 0;
  for (int i = 0; i < 4; i++) {
    u128 t = (u128)a[i] - P[i] - borrow;
    a[i] = (uint64_t)t;
    borrow = (t >> 64) ? 1 : 0;
  }
}

// CIOS Montgomery multiply with explicit add-with-carry chains (adc/adcx under -madx); about
// 1.7x faster than the u128-accumulator form under clang.  Inputs < p, output < p.
typedef unsigned long long ull;
static inline ull mul_lohi(ull a, ull b, ull* hi) {
  u128 r = (u128)a * b;
  *hi = (ull)(r >> 64);
  return (ull)r;
}
static inline Fq fq_mul(const Fq& a, const Fq& b) {
  const ull b0 = b.l[0], b1 = b.l[1], b2 = b.l[2], b3 = b.l[3];
  ull t0 = 0, t1 = 0, t2 = 0, t3 = 0, t4 = 0;
  for (int i = 0; i < 4; i++) {
    const ull ai = a.l[i];
    ull h0, h1, h2, h3;
    const ull l0 = mul_lohi(ai, b0, &h0), l1 = mul_lohi(ai, b1, &h1);
    const ull l2 = mul_lohi(ai, b2, &h2), l3 = mul_lohi(ai, b3, &h3);
    unsigned char c = 0;
    c = _addcarry_u64(c, t0, l0, &t0);
    c = _addcarry_u64(c, t1, l1, &t1);
    c = _addcarry_u64(c, t2, l2, &t2);
    c = _addcarry_u64(c, t3, l3, &t3);
    c = _addcarry_u64(c, t4, 0, &t4);
    ull t5 = c;
    c = _addcarry_u64(0, t1, h0, &t1);
    c = _addcarry_u64(c, t2, h1, &t2);
    c = _addcarry_u64(c, t3, h2, &t3);
    c = _addcarry_u64(c, t4, h3, &t4);
    t5 += c;
    const ull m = t0 * NP;
    const ull m0 = mul_lohi(m, P[0], &h0), m1 = mul_lohi(m, P[1], &h1);
    const ull m2 = mul_lohi(m, P[2], &h2), m3 = mul_lohi(m, P[3], &h3);
    ull drop;
    c = _addcarry_u64(0, t0, m0, &drop);
    c = _addcarry_u64(c, t1, m1, &t0);
    c = _addcarry_u64(c, t2, m2, &t1);
    c = _addcarry_u64(c, t3, m3, &t2);
    c = _addcarry_u64(c, t4, 0, &t3);
    t5 += c;
    c = _addcarry_u64(0, t0, h0, &t0);
    c = _addcarry_u64(c, t1, h1, &t1);
    c = _addcarry_u64(c, t2, h2, &t2);
    c = _addcarry_u64(c, t3, h3, &t3);
    t4 = t5 + c;
  }
  // a, b < p < 2^253: the CIOS result is < 2p < 2^254, so t4 == 0 and one subtraction suffices
  ull d0, d1, d2, d3;
  unsigned char br = _subborrow_u64(0, t0, P[0], &d0);
  br = _subborrow_u64(br, t1, P[1], &d1);
  br = _subborrow_u64(br, t2, P[2], &d2);
  br = _subborrow_u64(br, t3, P[3], &d3);
  Fq r;
  if (br) {
    r.l[0] = t0, r.l[1] = t1, r.l[2] = t2, r.l[3] = t3;
  } else {
    r.l[0] = d0, r.l[1] = d1, r.l[2] = d2, r.l[3] = d3;
  }
  return r;
}
// N independent products r[k] = a[k] b[k], the same CIOS steps interleaved across the N so the
// core overlaps their carry chains (a lone fq_mul is one long dependent chain: a doubling's
// four squarings and three products measured as ~9 multiply latencies done one after another).
template <int N>
static inline void fq_mul_n(Fq* r, const Fq* a, const Fq* b) {
  ull t0[N], t1[N], t2[N], t3[N], t4[N];
#pragma GCC unroll 4
  for (int k = 0; k < N; k++) t0[k] = t1[k] = t2[k] = t3[k] = t4[k] = 0;
#pragma GCC unroll 4
  for (int i = 0; i < 4; i++) {
#pragma GCC unroll 4
    for (int k = 0; k < N; k++) {
      const ull ai = a[k].l[i];
      ull h0, h1, h2, h3;
      const ull l0 = mul_lohi(ai, b[k].l[0], &h0), l1 = mul_lohi(ai, b[k].l[1], &h1);
      const ull l2 = mul_lohi(ai, b[k].l[2], &h2), l3 = mul_lohi(ai, b[k].l[3], &h3);
      unsigned char c = 0;
      c = _addcarry_u64(c, t0[k], l0, &t0[k]);
      c = _addcarry_u64(c, t1[k], l1, &t1[k]);
      c = _addcarry_u64(c, t2[k], l2, &t2[k]);
      c = _addcarry_u64(c, t3[k], l3, &t3[k]);
      c = _addcarry_u64(c, t4[k], 0, &t4[k]);
      ull t5 = c;
      c = _addcarry_u64(0, t1[k], h0, &t1[k]);
      c = _addcarry_u64(c, t2[k], h1, &t2[k]);
      c = _addcarry_u64(c, t3[k], h2, &t3[k]);
      c = _addcarry_u64(c, t4[k], h3, &t4[k]);
      t5 += c;
      const ull m = t0[k] * NP;
      const ull m0 = mul_lohi(m, P[0], &h0), m1 = mul_lohi(m, P[1], &h1);
      const ull m2 = mul_lohi(m, P[2], &h2), m3 = mul_lohi(m, P[3], &h3);
      ull drop;
      c = _addcarry_u64(0, t0[k], m0, &drop);
      c = _addcarry_u64(c, t1[k], m1, &t0[k]);
      c = _addcarry_u64(c, t2[k], m2, &t1[k]);
      c = _addcarry_u64(c, t3[k], m3, &t2[k]);
      c = _addcarry_u64(c, t4[k], 0, &t3[k]);
      t5 += c;
      c = _addcarry_u64(0, t0[k], h0, &t0[k]);
      c = _addcarry_u64(c, t1[k], h1, &t1[k]);
      c = _addcarry_u64(c, t2[k], h2, &t2[k]);
      c = _addcarry_u64(c, t3[k], h3, &t3[k]);
      t4[k] = t5 + c;
    }
  }
#pragma GCC unroll 4
  for (int k = 0; k < N; k++) {
    ull d0, d1, d2, d3;
    unsigned char br = _subborrow_u64(0, t0[k], P[0], &d0);
    br = _subborrow_u64(br, t1[k], P[1], &d1);
    br = _subborrow_u64(br, t2[k], P[2], &d2);
    br = _subborrow_u64(br, t3[k], P[3], &d3);
    if (br) {
      r[k].l[0] = t0[k], r[k].l[1] = t1[k], r[k].l[2] = t2[k], r[k].l[3] = t3[k];
    } else {
      r[k].l[0] = d0, r[k].l[1] = d1, r[k].l[2] = d2, r[k].l[3] = d3;
    }
  }
}
// Branch-free (a data-dependent branch per add mispredicts half the time on random values).
static inline Fq fq_add(const Fq& a, const Fq& b) {
  ull s0, s1, s2, s3, d0, d1, d2, d3;
  unsigned char c = _addcarry_u64(0, a.l[0], b.l[0], &s0);  // p < 2^253: no carry out
  c = _addcarry_u64(c, a.l[1], b.l[1], &s1);
  c = _addcarry_u64(c, a.l[2], b.l[2], &s2);
  _addcarry_u64(c, a.l[3], b.l[3], &s3);
  unsigned char br = _subborrow_u64(0, s0, P[0], &d0);
  br = _subborrow_u64(br, s1, P[1], &d1);
  br = _subborrow_u64(br, s2, P[2], &d2);
  br = _subborrow_u64(br, s3, P[3], &d3);
  const ull keep = 0ull - (ull)br;  // all ones when a + b < p
  return Fq{{(s0 & keep) | (d0 & ~keep), (s1 & keep) | (d1 & ~keep), (s2 & keep) | (d2 & ~keep),
             (s3 & keep) | (d3 & ~keep)}};
}
static inline Fq fq_sub(const Fq& a, const Fq& b) {
  ull d0, d1, d2, d3;
  unsigned char br = _subborrow_u64(0, a.l[0], b.l[0], &d0);
  br = _subborrow_u64(br, a.l[1], b.l[1], &d1);
  br = _subborrow_u64(br, a.l[2], b.l[2], &d2);
  br = _subborrow_u64(br, a.l[3], b.l[3], &d3);
  const ull m = 0ull - (ull)br;  // add p back when a < b
  ull r0, r1, r2, r3;
  unsigned char c = _addcarry_u64(0, d0, P[0] & m, &r0);
  c = _addcarry_u64(c, d1, P[1] & m, &r1);
  c = _addcarry_u64(c, d2, P[2] & m, &r2);
  _addcarry_u64(c, d3, P[3] & m, &r3);
  return Fq{{r0, r1, r2, r3}};
}
static inline Fq fq_zero() { return Fq{{0, 0, 0, 0}}; }
static inline Fq fq_one() { return Fq{{RMODP[0], RMODP[1], RMODP[2], RMODP[3]}}; }
static inline bool fq_is_zero(const Fq& a) { return !(a.l[0] | a.l[1] | a.l[2] | a.l[3]); }
static inline bool fq_eq(const Fq& a, const Fq& b) { return !memcmp(a.l, b.l, 32); }

// standard-form little-endian 64-bit limbs (< p) <-> Montgomery
static inline Fq fq_from_std(const uint64_t s[4]) {
  Fq a;
  memcpy(a.l, s, 32);
  return fq_mul(a, Fq{{R2MODP[0], R2MODP[1], R2MODP[2], R2MODP[3]}});
}
static inline void fq_to_std(const Fq& a, uint64_t s[4]) {
  Fq one = {{1, 0, 0, 0}};
  Fq r = fq_mul(a, one);
  memcpy(s, r.l, 32);
}
static inline Fq fq_pow(const Fq& a, const uint64_t e[4]) {
  Fq r = fq_one();
  for (int i = 3; i >= 0; i--)
    for (int b = 63; b >= 0; b--) {
      r = fq_mul(r, r);
      if ((e[i] >> b) & 1) r = fq_mul(r, a);
    }
  return r;
}
static inline Fq fq_inv_pow(const Fq& a) {
  const uint64_t E[4] = {0x0a117fffffffffffULL, 0x59aa76fed0000001ULL, 0x60b44d1e5c37b001ULL,
                         0x12ab655e9a2ca556ULL};  // p - 2
  return fq_pow(a, E);
}

static const uint64_t R3MODP[4] = {0x6a4295c90f65454cULL, 0x624d23ffae271699ULL, 0xb1e55ef6f1c9d713ULL,
                                   0x0601dfa555c48ddaULL};  // R^3 mod p
// x <- x / 2^k mod p for x < p, 1 <= k <= 63: add the multiple of p that clears the low k bits
// (m = x * (-p^-1) mod 2^k), shift; (x + m p) / 2^k < 2p, so one conditional subtraction.
static inline void div2k_mod(uint64_t x[4], int k) {
  const ull m = (x[0] * NP) & ((1ull << k) - 1);
  ull t[5];
  u128 acc = 0;
  for (int i = 0; i < 4; i++) {
    acc += (u128)m * P[i] + x[i];
    t[i] = (ull)acc;
    acc >>= 64;
  }
  t[4] = (ull)acc;
  for (int i = 0; i < 4; i++) x[i] = (t[i] >> k) | (t[i + 1] << (64 - k));
  if (geq_p(x)) sub_p(x);
}
// u >>= ctz(u) (u odd afterwards, u != 0); x <- x / 2^ctz(u) mod p alongside.
static inline void strip_twos(ull u[4], uint64_t x[4]) {
  while (!(u[0] & 1)) {
    const int k = u[0] ? __builtin_ctzll(u[0]) : 63;
    for (int i = 0; i < 3; i++) u[i] = (u[i] >> k) | (u[i + 1] << (64 - k));
    u[3] >>= k;
    div2k_mod(x, k);
  }
}
static inline bool u4_is_one(const ull u[4]) { return u[0] == 1 && !(u[1] | u[2] | u[3]); }
static inline bool u4_geq(const ull a[4], const ull b[4]) {
  for (int i = 3; i >= 0; i--)
    if (a[i] != b[i]) return a[i] > b[i];
  return true;
}
static inline void u4_sub(ull a[4], const ull b[4]) {
  unsigned char br = _subborrow_u64(0, a[0], b[0], &a[0]);
  br = _subborrow_u64(br, a[1], b[1], &a[1]);
  br = _subborrow_u64(br, a[2], b[2], &a[2]);
  _subborrow_u64(br, a[3], b[3], &a[3]);
}
// Inverse by the binary extended Euclidean algorithm on the Montgomery representative a' = aR:
// invariants x1 a' = u, x2 a' = v (mod p) with u, v odd; the smaller is subtracted from the larger
// and its factors of two stripped (several bits per step through div2k_mod).  x = a'^-1 when u
// or v reaches 1, and x R^3 / R = a^-1 R is the Montgomery form of the inverse.  Variable time
// (nothing here is secret); ~4x faster than a^(p-2) (253 dependent squarings).  0 -> 0.
static inline Fq fq_inv(const Fq& a) {
  if (!(a.l[0] | a.l[1] | a.l[2] | a.l[3])) return a;
  ull u[4] = {a.l[0], a.l[1], a.l[2], a.l[3]}, v[4] = {P[0], P[1], P[2], P[3]};
  Fq x1 = {{1, 0, 0, 0}}, x2 = {{0, 0, 0, 0}};
  strip_twos(u, x1.l);
  const Fq r3 = {{R3MODP[0], R3MODP[1], R3MODP[2], R3MODP[3]}};
  for (;;) {
    if (u4_is_one(u)) return fq_mul(x1, r3);
    if (u4_geq(u, v)) {
      u4_sub(u, v);
      x1 = fq_sub(x1, x2);
      strip_twos(u, x1.l);
    } else {
      u4_sub(v, u);
      x2 = fq_sub(x2, x1);
      strip_twos(v, x2.l);
      if (u4_is_one(v)) return fq_mul(x2, r3);
    }
  }
}

// 8 big-endian u32 words (bytes.rs layout) <-> standard limbs
static inline void be_words_to_std(const uint32_t* w, uint64_t s[4]) {
  for (int i = 0; i < 4; i++) s[i] = ((uint64_t)w[6 - 2 * i] << 32) | w[7 - 2 * i];
}
static inline void std_to_be_words(const uint64_t s[4], uint32_t* w) {
  for (int i = 0; i < 4; i++) {
    w[7 - 2 * i] = (uint32_t)s[i];
    w[6 - 2 * i] = (uint32_t)(s[i] >> 32);
  }
}
static inline bool std_lt_p(const uint64_t s[4]) { return !geq_p(s); }

// ------------------------------------------------------------------------------------------
// Extended twisted Edwards points, a = -1, k = 2d (add-2008-hwcd-3 / dbl-2008-hwcd).
// ------------------------------------------------------------------------------------------
struct Pt {
  Fq X, Y, T, Z;
};
static inline Pt pt_identity() { return Pt{fq_zero(), fq_one(), fq_zero(), fq_one()}; }

// p + q; with want_t = false the result's T is left stale (fine when a doubling comes next:
// dbl-2008-hwcd never reads T).
static inline Pt pt_add(const Pt& p, const Pt& q, bool want_t = true) {
  const Fq a1[4] = {fq_sub(p.Y, p.X), fq_add(p.Y, p.X), p.T, p.Z};
  const Fq b1[4] = {fq_sub(q.Y, q.X), fq_add(q.Y, q.X), q.T, q.Z};
  Fq m1[4];
  fq_mul_n<4>(m1, a1, b1);  // A, B, T1 T2, Z1 Z2
  const Fq& A = m1[0];
  const Fq& B = m1[1];
  const Fq C = fq_mul(m1[2], Fq{{K2D_M[0], K2D_M[1], K2D_M[2], K2D_M[3]}});
  const Fq D = fq_add(m1[3], m1[3]);
  const Fq E = fq_sub(B, A), F = fq_sub(D, C), G = fq_add(D, C), H = fq_add(B, A);
  const Fq a2[4] = {E, G, F, E}, b2[4] = {F, H, G, H};
  Fq m2[4];
  if (want_t) {
    fq_mul_n<4>(m2, a2, b2);
  } else {
    fq_mul_n<3>(m2, a2, b2);
    m2[3] = fq_zero();
  }
  return Pt{m2[0], m2[1], m2[3], m2[2]};
}
static inline Pt pt_dbl(const Pt& p) {
  Fq A = fq_mul(p.X, p.X);
  Fq B = fq_mul(p.Y, p.Y);
  Fq C = fq_mul(p.Z, p.Z);
  C = fq_add(C, C);
  Fq S = fq_add(p.X, p.Y);
  S = fq_mul(S, S);
  Fq E = fq_sub(fq_sub(S, A), B);
  Fq G = fq_sub(B, A);
  Fq F = fq_sub(G, C);
  Fq H = fq_sub(fq_zero(), fq_add(A, B));
  return Pt{fq_mul(E, F), fq_mul(G, H), fq_mul(E, H), fq_mul(F, G)};
}
// 2^k * p.  dbl-2008-hwcd never reads T, so every doubling but the last skips T3 = E*H.  The
// four squarings, then the output products, run as interleaved batches (fq_mul_n).
static inline Pt pt_dbl_n(Pt p, int k) {
  for (int i = 0; i < k; i++) {
    const Fq S0 = fq_add(p.X, p.Y);
    const Fq in[4] = {p.X, p.Y, p.Z, S0};
    Fq sq[4];
    fq_mul_n<4>(sq, in, in);
    const Fq &A = sq[0], &B = sq[1], &S = sq[3];
    const Fq C = fq_add(sq[2], sq[2]);
    const Fq E = fq_sub(fq_sub(S, A), B);
    const Fq G = fq_sub(B, A);
    const Fq F = fq_sub(G, C);
    const Fq H = fq_sub(fq_zero(), fq_add(A, B));
    const Fq ma[4] = {E, G, F, E}, mb[4] = {F, H, G, H};
    Fq out[4];
    if (i == k - 1) {
      fq_mul_n<4>(out, ma, mb);
      p.T = out[3];
    } else {
      fq_mul_n<3>(out, ma, mb);
    }
    p.X = out[0];
    p.Y = out[1];
    p.Z = out[2];
  }
  return p;
}
// affine (x, y) in standard form; identity -> (0, 1)
static inline void pt_to_affine_std(const Pt& p, uint64_t x[4], uint64_t y[4]) {
  Fq zi = fq_inv(p.Z);
  fq_to_std(fq_mul(p.X, zi), x);
  fq_to_std(fq_mul(p.Y, zi), y);
}
static inline Pt pt_from_affine_std(const uint64_t x[4], const uint64_t y[4]) {
  Pt r;
  r.X = fq_from_std(x);
  r.Y = fq_from_std(y);
  r.T = fq_mul(r.X, r.Y);
  r.Z = fq_one();
  return r;
}

}  // namespace msmh
