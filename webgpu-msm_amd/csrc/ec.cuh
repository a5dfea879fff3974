// Twisted Edwards "Edwards-BLS12" (ark-ed-on-bls12-377): -x^2 + y^2 = 1 + d x^2 y^2, d = 3021
// (reference: src/submission/wgsl/curve.wgsl:1-63, src/reference/params/AleoConstants.ts:3-4).
//
// Extended coordinates (X:Y:T:Z), x = X/Z, y = Y/Z, T = XY/Z.  a = -1 is a square and d a
// non-square mod p, so the unified add-2008-hwcd-3 formulas below are complete: one branch-free
// path covers P+Q, P+P and the identity (0:1:0:1).  The reference's add_points
// (curve.wgsl:36-63) computes the same group law with 9 multiplies; here:
//   * madd (mixed, Q in halved precomputed affine form ((y-x)/2, (y+x)/2, d*t), z = 1): 7M — the
//     bucket hot loop;
//   * padd (projective + projective): 9M;
//   * pdbl (dbl-2008-hwcd): 4M + 4S.
#pragma once
#include "fp29.cuh"

namespace msm {

struct xyzt {
  fe X, Y, T, Z;
};
// Precomputed affine point, halved: ((y - x)/2, (y + x)/2, d*t) (pt_madd).  Negation swaps the
// first two and negates kt.
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

// acc + q (q a halved precomputed affine point, below).  add-2008-hwcd-3 with Z2 = 1, k = 2d.
// The record holds ((y-x)/2, (y+x)/2, d*t): A, B and C come out halved, so D = 2 Z1 / 2 = Z1 needs
// no doubling, and (X3:Y3:T3:Z3) is the sum with every coordinate scaled by 1/4 -- the same
// projective point.  Differences are signed (fe_sub_s) and meet fe_mul_sd; all outputs normalised.
__device__ __forceinline__ xyzt pt_madd(const xyzt& p, const pre& q) {
  fe A = fe_mul_sd<WIDE_ALL, false>(fe_sub_s(p.Y, p.X), q.ymx);  // signed x N
  fe B = fe_mul(fe_add(p.Y, p.X), q.ypx);                         // S x N
  fe C = fe_mul(p.T, q.kt);  // N x N (or N x V for a negated q, kt_neg_if)
  fe E = fe_sub_s(B, A);     // signed
  fe F = fe_sub_s(p.Z, C);   // signed
  fe G = fe_add(p.Z, C);     // S
  fe H = fe_add(B, A);       // S
  xyzt r;
  r.X = fe_mul_sd<WIDE_ALL, true>(E, F);   // signed x signed
  r.Y = fe_mul(G, H);                      // S x S
  r.T = fe_mul_sd<WIDE_ALL, false>(E, H);  // signed x S
  r.Z = fe_mul_sd<WIDE_ALL, false>(F, G);  // signed x S
  return r;
}

// p + q, both extended projective.  add-2008-hwcd-3, k = 2d: 9M (the k multiply is fe_mul_2d).
__device__ __forceinline__ xyzt pt_add(const xyzt& p, const xyzt& q) {
  fe A = fe_mul_w<WIDE_EF>(fe_sub_v(p.Y, p.X), fe_sub_v(q.Y, q.X));  // V*V
  fe B = fe_mul(fe_add(p.Y, p.X), fe_add(q.Y, q.X));  // S*S
  fe C = fe_mul_2d(fe_mul(p.T, q.T));  // k = 2d = 6042: scaled, not multiplied (value < 3p)
  fe D = fe_mul(p.Z, q.Z);
  D = fe_add(D, D);  // 2N, unnormalised
  fe E = fe_sub_v(B, A);  // V
  fe F = fe_sub(D, C);    // N
  fe G = fe_add(D, C);    // 2N + N: limbs < 1.5 * 2^30 (meets H: S and F: N only)
  fe H = fe_add(B, A);    // S
  xyzt r;
  r.X = fe_mul(E, F);             // V x N
  r.Y = fe_mul_w<WIDE_GH>(G, H);  // 1.5-form x S: fewer 32-bit reduction digits (fp29.cuh)
  r.T = fe_mul(E, H);             // V x S
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

// d*t of -q = (-x, y) is -d*t: 5p - kt, left unnormalised (V form), legal as pt_madd's
// C = T * kt operand (N * V).  (The other half of the negation, swapping (y-x)/2 and (y+x)/2,
// is done by the record gather: msm_kernels.hip load_pre_signed.)
__device__ __forceinline__ fe kt_neg_if(const fe& kt, bool neg) {
  fe r;
#pragma unroll
  for (int i = 0; i < NL; i++) r.v[i] = neg ? K5P29[i] - kt.v[i] : kt.v[i];
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

// ---- quad-cooperative addition (latency-bound reductions) -------------------------------------
// Lane q = lane & 3 of each group of 4 lanes holds coordinate q (0 X, 1 Y, 2 T, 3 Z) of P in `p`
// and of Q in `r`; every lane gets its coordinate of P + Q.  Same add-2008-hwcd-3 formula as
// pt_add, but its multiplies run as rounds of one multiply per lane (A | B | T1T2 | Z1Z2, then
// C = 2d T1T2 by fe_mul_2d on lane 2, then EF | GH | EH | FG), operands exchanged with DPP quad
// permutes.  Two multiply latencies (plus a small scaling) instead of nine: for reduction trees
// whose levels are too narrow to fill the machine.
template <int K>
__device__ __forceinline__ fe fe_quad_bcast(const fe& a) {
  fe r;
#pragma unroll
  for (int i = 0; i < NL; i++) r.v[i] = (uint32_t)__builtin_amdgcn_mov_dpp((int)a.v[i], K * 0x55, 0xF, 0xF, false);
  return r;
}
__device__ __forceinline__ fe pt_add_quad(const fe& p, const fe& r) {
  const uint32_t q = threadIdx.x & 3;
  const fe X1 = fe_quad_bcast<0>(p), Y1 = fe_quad_bcast<1>(p);
  const fe X2 = fe_quad_bcast<0>(r), Y2 = fe_quad_bcast<1>(r);
  const fe s1 = fe_sub_u(Y1, X1), a1 = fe_add(Y1, X1);  // U, S
  const fe s2 = fe_sub(Y2, X2), a2 = fe_add(Y2, X2);    // N, S
  fe a = fe_sel(q == 0, fe_sel(q == 1, p, a1), s1);
  fe b = fe_sel(q == 0, fe_sel(q == 1, r, a2), s2);
  const fe m = fe_mul(a, b);  // lane 0: A, 1: B, 2: T1 T2, 3: Z1 Z2
  const fe m2 = q == 2 ? fe_mul_2d(m) : m;  // lane 2: C = 2d T1 T2
  const fe A = fe_quad_bcast<0>(m2), B = fe_quad_bcast<1>(m2);
  const fe C = fe_quad_bcast<2>(m2), D0 = fe_quad_bcast<3>(m2);
  const fe D = fe_add(D0, D0);
  const fe E = fe_sub_u(B, A), F = fe_sub(D, C), G = fe_add(D, C), H = fe_add(B, A);
  const fe a3 = fe_sel(q == 0 || q == 2, fe_sel(q == 1, F, G), E);  // E F | G H | E H | F G
  const fe b3 = fe_sel(q == 0, fe_sel(q == 3, H, G), F);
  return fe_mul_w<WIDE_GH & WIDE_EH>(a3, b3);  // one multiply serves E F, G H, E H and F G
}

}  // namespace msm
