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
static inline Fq fq_add(const Fq& a, const Fq& b) {
  Fq r;
  u128 c = 0;
  for (int i = 0; i < 4; i++) {
    c += (u128)a.l[i] + b.l[i];
    r.l[i] = (uint64_t)c;
    c >>= 64;
  }
  if (geq_p(r.l)) sub_p(r.l);  // p < 2^253: no carry out
  return r;
}
static inline Fq fq_sub(const Fq& a, const Fq& b) {
  Fq r;
  u128 borrow = 0;
  for (int i = 0; i < 4; i++) {
    u128 t = (u128)a.l[i] - b.l[i] - borrow;
    r.l[i] = (uint64_t)t;
    borrow = (t >> 64) ? 1 : 0;
  }
  if (borrow) {
    u128 c = 0;
    for (int i = 0; i < 4; i++) {
      c += (u128)r.l[i] + P[i];
      r.l[i] = (uint64_t)c;
      c >>= 64;
    }
  }
  return r;
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
static inline Fq fq_inv(const Fq& a) {
  const uint64_t E[4] = {0x0a117fffffffffffULL, 0x59aa76fed0000001ULL, 0x60b44d1e5c37b001ULL,
                         0x12ab655e9a2ca556ULL};  // p - 2
  return fq_pow(a, E);
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
  Fq A = fq_mul(fq_sub(p.Y, p.X), fq_sub(q.Y, q.X));
  Fq B = fq_mul(fq_add(p.Y, p.X), fq_add(q.Y, q.X));
  Fq C = fq_mul(fq_mul(p.T, q.T), Fq{{K2D_M[0], K2D_M[1], K2D_M[2], K2D_M[3]}});
  Fq D = fq_mul(p.Z, q.Z);
  D = fq_add(D, D);
  Fq E = fq_sub(B, A), F = fq_sub(D, C), G = fq_add(D, C), H = fq_add(B, A);
  return Pt{fq_mul(E, F), fq_mul(G, H), want_t ? fq_mul(E, H) : fq_zero(), fq_mul(F, G)};
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
// 2^k * p.  dbl-2008-hwcd never reads T, so every doubling but the last skips T3 = E*H.
static inline Pt pt_dbl_n(Pt p, int k) {
  for (int i = 0; i < k; i++) {
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
    p.X = fq_mul(E, F);
    p.Y = fq_mul(G, H);
    p.Z = fq_mul(F, G);
    if (i == k - 1) p.T = fq_mul(E, H);
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
