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

static inline Fq fq_mul(const Fq& a, const Fq& b) {
  uint64_t t[6] = {0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 4; i++) {
    u128 c = 0;
    for (int j = 0; j < 4; j++) {
      c += (u128)a.l[i] * b.l[j] + t[j];
      t[j] = (uint64_t)c;
      c >>= 64;
    }
    u128 s = (u128)t[4] + (uint64_t)c;
    t[4] = (uint64_t)s;
    t[5] = (uint64_t)(s >> 64);
    uint64_t m = t[0] * NP;
    c = (u128)m * P[0] + t[0];
    c >>= 64;
    for (int j = 1; j < 4; j++) {
      c += (u128)m * P[j] + t[j];
      t[j - 1] = (uint64_t)c;
      c >>= 64;
    }
    s = (u128)t[4] + (uint64_t)c;
    t[3] = (uint64_t)s;
    t[4] = t[5] + (uint64_t)(s >> 64);
  }
  Fq r;
  memcpy(r.l, t, 32);
  if (t[4] || geq_p(r.l)) sub_p(r.l);
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

static inline Pt pt_add(const Pt& p, const Pt& q) {
  Fq A = fq_mul(fq_sub(p.Y, p.X), fq_sub(q.Y, q.X));
  Fq B = fq_mul(fq_add(p.Y, p.X), fq_add(q.Y, q.X));
  Fq C = fq_mul(fq_mul(p.T, q.T), Fq{{K2D_M[0], K2D_M[1], K2D_M[2], K2D_M[3]}});
  Fq D = fq_mul(p.Z, q.Z);
  D = fq_add(D, D);
  Fq E = fq_sub(B, A), F = fq_sub(D, C), G = fq_add(D, C), H = fq_add(B, A);
  return Pt{fq_mul(E, F), fq_mul(G, H), fq_mul(E, H), fq_mul(F, G)};
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
