// Host CPU Pippenger: msm_compute_cpu, the reference's CPU-only path (cpuWorkRatio = 1,
// submission.ts:96-115 -> msm_end_to_end, msm-wasm/src/lib.rs:24-44, 106-121), multithreaded.
//
// It is an explicit entry of its own, never a fallback: the GPU entries fail with
// MSM_ERR_NO_DEVICE when no gfx950 is present.  Same wire formats and semantics as the GPU path
// (full 256-bit scalars, points x|y|t|z with z != 1 normalised, identity (0, 1)).
//
// Algorithm: signed c-bit digits (as the device's k_recode_hist), 2^(c-1) buckets per window.
// Work items are (window, slice of points): each thread accumulates its slice into a private
// bucket table with 7-multiplication mixed adds against precomputed affine records
// (y - x, y + x, 2d t), reduces that table to the item's window sum (running sums), and the
// items' window sums are added; a Horner pass over the windows finishes (reduce_last,
// lib.rs:88-104).  Field arithmetic: hostfield.h (4 x 64-bit Montgomery, adx chains).
#pragma once
#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "msm_util.h"

#include "hostfield.h"

namespace msmh {

struct PreAff {  // precomputed affine point for the mixed add
  Fq ymx, ypx, kt;
};

// acc + q (q affine, precomputed; neg: add -q = (-x, y): swap ymx/ypx and negate kt).  7M.
static inline void pt_madd_pre(Pt& p, const PreAff& q, bool neg) {
  const Fq& qa = neg ? q.ypx : q.ymx;
  const Fq& qb = neg ? q.ymx : q.ypx;
  Fq A = fq_mul(fq_sub(p.Y, p.X), qa);
  Fq B = fq_mul(fq_add(p.Y, p.X), qb);
  Fq C = fq_mul(p.T, q.kt);
  if (neg) C = fq_sub(fq_zero(), C);
  Fq D = fq_add(p.Z, p.Z);
  Fq E = fq_sub(B, A), F = fq_sub(D, C), G = fq_add(D, C), H = fq_add(B, A);
  p = Pt{fq_mul(E, F), fq_mul(G, H), fq_mul(E, H), fq_mul(F, G)};
}

// Signed digit of window w (width c): digit = bits + carry_in, folded into (-2^(c-1), 2^(c-1)].
static inline int32_t cpu_digit(const uint64_t s[4], uint32_t c, uint32_t w, uint32_t& carry) {
  const uint32_t bit = c * w;
  uint64_t v = 0;
  if (bit < 256) {
    const uint32_t li = bit / 64, sh = bit % 64;
    v = s[li] >> sh;
    if (sh && li + 1 < 4) v |= s[li + 1] << (64 - sh);
    v &= (1ull << c) - 1;
  }
  v += carry;
  const uint64_t half = 1ull << (c - 1);
  if (v > half) {
    carry = 1;
    return (int32_t)((int64_t)v - (int64_t)(2 * half));
  }
  carry = 0;
  return (int32_t)v;
}

// Convert wire points to precomputed affine records (z != 1 normalised by batch inversion).
static inline int cpu_prepare(const uint32_t* pts_be, size_t lo, size_t hi, PreAff* out) {
  const Fq k2d{{K2D_M[0], K2D_M[1], K2D_M[2], K2D_M[3]}};
  std::vector<size_t> proj;
  std::vector<Pt> raw;
  for (size_t i = lo; i < hi; i++) {
    const uint32_t* w = pts_be + 32 * i;
    uint64_t s[4][4];
    for (int f = 0; f < 4; f++) {
      be_words_to_std(w + 8 * f, s[f]);
      if (!std_lt_p(s[f])) return MSM_ERR_COORD_RANGE;
    }
    const bool z_one = s[3][0] == 1 && !s[3][1] && !s[3][2] && !s[3][3];
    const bool z_zero = !(s[3][0] | s[3][1] | s[3][2] | s[3][3]);
    if (z_zero) return MSM_ERR_BAD_POINT;
    Pt p{fq_from_std(s[0]), fq_from_std(s[1]), fq_from_std(s[2]), fq_from_std(s[3])};
    if (!z_one) {
      proj.push_back(i);
      raw.push_back(p);
      continue;
    }
    out[i - lo] = PreAff{fq_sub(p.Y, p.X), fq_add(p.Y, p.X), fq_mul(p.T, k2d)};
  }
  if (!proj.empty()) {  // Montgomery's trick: one inversion for all the projective inputs
    std::vector<Fq> pref(proj.size());
    Fq acc = fq_one();
    for (size_t j = 0; j < proj.size(); j++) {
      pref[j] = acc;
      acc = fq_mul(acc, raw[j].Z);
    }
    Fq inv = fq_inv(acc);
    for (size_t j = proj.size(); j-- > 0;) {
      const Fq zi = fq_mul(inv, pref[j]);
      inv = fq_mul(inv, raw[j].Z);
      const Fq x = fq_mul(raw[j].X, zi), y = fq_mul(raw[j].Y, zi), t = fq_mul(raw[j].T, zi);
      out[proj[j] - lo] = PreAff{fq_sub(y, x), fq_add(y, x), fq_mul(t, k2d)};
    }
  }
  return MSM_OK;
}

static inline int cpu_msm(const uint32_t* points_be, const uint32_t* scalars_be, size_t n, uint32_t c,
                          int n_threads, uint32_t out_xy_be[16]) {
  auto emit = [&](const Pt& r) {
    uint64_t x[4], y[4];
    pt_to_affine_std(r, x, y);
    std_to_be_words(x, out_xy_be);
    std_to_be_words(y, out_xy_be + 8);
  };
  if (n == 0) {
    emit(pt_identity());
    return MSM_OK;
  }
  unsigned T = n_threads > 0 ? (unsigned)n_threads : host_threads();
  T = (unsigned)std::min<size_t>(T, std::max<size_t>(1, n / 256));
  if (c == 0) {  // ~16 points per bucket of one (window, slice) item, 4..16 bits
    const size_t per_slice = n / std::max<size_t>(1, (3 * T) / 18);
    c = 4;
    while (c < 16 && ((size_t)1 << (c + 3)) <= per_slice) c++;
  }
  if (c < 4 || c > 20) return MSM_ERR_UNSUPPORTED_WINDOW;
  const uint32_t W = (256 + c - 1) / c + 1;  // + the final carry
  const uint32_t B = 1u << (c - 1);
  // 1) records and scalars, split over the threads
  std::vector<PreAff> pre(n);
  std::vector<int32_t> dig((size_t)W * n);  // window-major signed digits
  std::atomic<int> err{MSM_OK};
  auto par = [&](auto&& fn) {
    std::vector<std::thread> ts;
    for (unsigned t = 0; t < T; t++) ts.emplace_back(fn, t);
    for (auto& th : ts) th.join();
  };
  par([&](unsigned t) {
    const size_t lo = n * t / T, hi = n * (t + 1) / T;
    int rc = cpu_prepare(points_be, lo, hi, pre.data() + lo);
    if (rc != MSM_OK) err.store(rc);
    for (size_t i = lo; i < hi; i++) {
      uint64_t s4[4];
      be_words_to_std(scalars_be + 8 * i, s4);
      uint32_t carry = 0;
      for (uint32_t w = 0; w < W; w++) dig[(size_t)w * n + i] = cpu_digit(s4, c, w, carry);
    }
  });
  if (err.load() != MSM_OK) return err.load();
  // 2) (window, slice) items: enough of them to keep every thread busy to the end
  const uint32_t S = (uint32_t)std::max<size_t>(1, std::min<size_t>((3 * T + W - 1) / W, n / 1024 + 1));
  std::vector<Pt> part((size_t)W * S, pt_identity());
  std::atomic<uint32_t> next{0};
  par([&](unsigned) {
    std::vector<Pt> bk(B);
    std::vector<uint8_t> live(B);
    for (;;) {
      const uint32_t item = next.fetch_add(1);
      if (item >= W * S) break;
      const uint32_t w = item / S, sl = item % S;
      const size_t lo = n * sl / S, hi = n * (sl + 1) / S;
      std::fill(live.begin(), live.end(), 0);
      for (size_t i = lo; i < hi; i++) {
        const int32_t d = dig[(size_t)w * n + i];
        if (!d) continue;
        const uint32_t b = (uint32_t)(d < 0 ? -d : d) - 1;
        if (!live[b]) {
          bk[b] = pt_identity();
          live[b] = 1;
        }
        pt_madd_pre(bk[b], pre[i], d < 0);
      }
      // sum_b (b + 1) B_b by running sums from the top bucket (bucket_sum_cpu, lib.rs:46-56)
      Pt run = pt_identity(), acc = pt_identity();
      bool any = false;
      for (uint32_t b = B; b-- > 0;) {
        if (live[b]) {
          run = any ? pt_add(run, bk[b]) : bk[b];
          any = true;
        }
        if (any) acc = pt_add(acc, run);
      }
      part[item] = acc;
    }
  });
  // 3) window sums, then Horner from the top window (reduce_last, lib.rs:88-104)
  Pt r = pt_identity();
  for (uint32_t w = W; w-- > 0;) {
    if (w + 1 < W) r = pt_dbl_n(r, (int)c);
    for (uint32_t s = 0; s < S; s++) r = pt_add(r, part[(size_t)w * S + s]);
  }
  emit(r);
  return MSM_OK;
}

}  // namespace msmh
