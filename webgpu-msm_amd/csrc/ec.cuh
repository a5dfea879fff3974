// Twisted Edwards "Edwards-BLS12" (ark-ed-on-bls12-377): -x^2 + y^2 = 1 + d x^2 y^2, d = 3021
// (reference: src/submission/wgsl/curve.wgsl:1-63, src/reference/params/AleoConstants.ts:3-4).
//
// Extended coordinates (X:Y:T:Z), x = X/Z, y = Y/Z, T = XY/Z.  a = -1 is a square and d a
// non-square mod p, so the unified add-2008-hwcd-3 formulas below are complete: one branch-free
// path covers P+Q, P+P and the identity (0:1:0:1).  The reference's add_points
// (curve.wgsl:36-63) computes the same group law with 9 multiplies; here:
//   * madd (mixed, Q in precomputed affine form (y-x, y+x, 2d*t), z = 1): 7M — the bucket hot loop;
//   * padd (projective + projective): 9M;
//   * pdbl (dbl-2008-hwcd): 4M + 4S.
#pragma once
#include "fp29.cuh"

namespace msm {

struct xyzt {
  fe X, Y, T, Z;
};
// Precomputed affine point: (y - x, y + x, 2d*t).  Negation swaps the first two and negates kt.
struct pre {
  fe ymx, ypx, kt;
};

__device__ __forceinline__ xyzt pt_identity() {
  xyzt r;
  r.X = fe_zero();
  r.Y = fe_one();
  r.T = fe_zero();
  r.Z = fe_one();
  return r;
}

// acc + q (q affine precomputed).  add-2008-hwcd-3 with Z2 = 1, k = 2d.  All outputs normalised.
__device__ __forceinline__ xyzt pt_madd(const xyzt& p, const pre& q) {
  fe A = fe_mul(fe_sub_u(p.Y, p.X), q.ymx);  // U*N
  fe B = fe_mul(fe_add(p.Y, p.X), q.ypx);    // S*N
  fe C = fe_mul(p.T, q.kt);                  // N*N (or N*U for a negated q, pre_neg_if)
  fe D = fe_add(p.Z, p.Z);                   // 2N: limbs < 2^30, left unnormalised
  fe E = fe_sub_u(B, A);                     // U (meets F: N and H: S only)
  fe F = fe_sub(D, C);                       // N
  fe G = fe_add(D, C);                       // 2N + N: limbs < 1.5 * 2^30 (meets H: S and F: N only)
  fe H = fe_add(B, A);                       // S
  xyzt r;
  r.X = fe_mul(E, F);
  r.Y = fe_mul(G, H);
  r.T = fe_mul(E, H);
  r.Z = fe_mul(F, G);
  return r;
}

// p + q, both extended projective.  add-2008-hwcd-3, k = 2d: 9M.
__device__ __forceinline__ xyzt pt_add(const xyzt& p, const xyzt& q) {
  fe A = fe_mul(fe_sub_u(p.Y, p.X), fe_sub(q.Y, q.X));  // U*N
  fe B = fe_mul(fe_add(p.Y, p.X), fe_add(q.Y, q.X));  // S*S
  fe C = fe_mul(fe_mul(p.T, q.T), fe_const(K2D29));
  fe D = fe_mul(p.Z, q.Z);
  D = fe_add(D, D);  // 2N, unnormalised (see pt_madd)
  fe E = fe_sub_u(B, A);
  fe F = fe_sub(D, C);
  fe G = fe_add(D, C);
  fe H = fe_add(B, A);
  xyzt r;
  r.X = fe_mul(E, F);
  r.Y = fe_mul(G, H);
  r.T = fe_mul(E, H);
  r.Z = fe_mul(F, G);
  return r;
}

// 2p.  dbl-2008-hwcd with a = -1: A = X^2, B = Y^2, C = 2Z^2, D = -A, E = (X+Y)^2 - A - B,
// G = D + B, F = G - C, H = D - B; X3 = EF, Y3 = GH, T3 = EH, Z3 = FG.
__device__ __forceinline__ xyzt pt_dbl(const xyzt& p) {
  fe A = fe_sqr(p.X);
  fe B = fe_sqr(p.Y);
  fe C = fe_dbl_n(fe_sqr(p.Z));
  fe S = fe_sqr(fe_add(p.X, p.Y));
  fe E = fe_sub(fe_sub(S, A), B);
  fe G = fe_sub(B, A);  // D + B = B - A
  fe F = fe_sub(G, C);
  fe H = fe_neg(fe_add_n(A, B));
  xyzt r;
  r.X = fe_mul(E, F);
  r.Y = fe_mul(G, H);
  r.T = fe_mul(E, H);
  r.Z = fe_mul(F, G);
  return r;
}

__device__ __forceinline__ xyzt pt_neg(const xyzt& p) {
  xyzt r = p;
  r.X = fe_neg(p.X);
  r.T = fe_neg(p.T);
  return r;
}

// -q = (-x, y): swap (y - x, y + x) and negate 2dt.  The negated kt = 8p - kt is left
// unnormalised (U form, limbs < 2^30), legal as pt_madd's C = T * kt operand (N * U).
__device__ __forceinline__ pre pre_neg_if(const pre& q, bool neg) {
  pre r;
  r.ymx = fe_sel(neg, q.ymx, q.ypx);
  r.ypx = fe_sel(neg, q.ypx, q.ymx);
#pragma unroll
  for (int i = 0; i < NL; i++) r.kt.v[i] = neg ? K8P29[i] - q.kt.v[i] : q.kt.v[i];
  return r;
}

__device__ __forceinline__ xyzt pt_sel(bool c, const xyzt& a, const xyzt& b) {
  xyzt r;
  r.X = fe_sel(c, a.X, b.X);
  r.Y = fe_sel(c, a.Y, b.Y);
  r.T = fe_sel(c, a.T, b.T);
  r.Z = fe_sel(c, a.Z, b.Z);
  return r;
}

}  // namespace msm
