// Pippenger MSM kernels for MI355X (gfx950).  Replaces the reference's GPU intra-bucket
// reduction (src/submission/gpu.ts:36-285 + wgsl/entry_padd_idx.wgsl:23-46) and its Rust
// split / inter-bucket reduce (src/submission/msm-wasm/src/lib.rs:46-133) with one on-device
// pipeline:
//
//   k_prepare_points   wire points (BE x|y|t|z, 128 B) -> precomputed affine (y-x, y+x, 2dt) in
//                      29-bit Montgomery limbs, 128 B records (one cache line each)
//   k_recode_count     signed c-bit digits per scalar (window-carry recoding, |d| <= 2^(c-1)),
//                      LDS histogram of (window, coarse bucket range)
//   k_coarse_scan      exclusive scan of the coarse histogram (one workgroup)
//   k_coarse_scatter   digits -> coarse bins (per-WG reservation, write runs stay contiguous)
//   k_fine_sort        one WG per coarse bin: LDS counting sort by bucket -> globally sorted
//                      (entry, bucket key) list + per-bucket counts
//   k_accumulate       fixed-length runs of the sorted list, one lane per run: mixed adds, whole
//                      buckets written directly, run-boundary pieces written as head/tail partials
//   k_fixup            joins head/tail partials of buckets that straddle runs
//   k_bucket_reduce_1  per (window, chunk of L buckets): running sums -> U_c = sum (i+1) B, T_c = sum B
//   k_bucket_reduce_2  per (window, term): plain sums R_{w,V} = sum_c U_c, R_{w,k} = sum_{c: bit k} T_c,
//                      converted to canonical standard form for the host Horner
//
// Digit semantics differ from the reference's (unsigned, MSB-first, lib.rs:58-84 + msm-macro) on
// purpose: only the final affine (x, y) is the parity contract, and signed digits halve the
// bucket count.
#include "ec.cuh"
#include "msm_dev.h"

namespace msm {

// ---------------------------------------------------------------------------------------------
// point preparation
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void load_be_words(const uint32_t* src, uint32_t le[8]) {
  uint4 a = reinterpret_cast<const uint4*>(src)[0];
  uint4 b = reinterpret_cast<const uint4*>(src)[1];
  // big-endian word order: src[0] is the most significant 32 bits (bytes.rs:11-20)
  le[7] = a.x; le[6] = a.y; le[5] = a.z; le[4] = a.w;
  le[3] = b.x; le[2] = b.y; le[1] = b.z; le[0] = b.w;
}

__device__ __forceinline__ void store_fe(uint32_t* dst, const fe& a) {
#pragma unroll
  for (int i = 0; i < NL; i++) dst[i] = a.v[i];
}
__device__ __forceinline__ fe load_fe(const uint32_t* src) {
  fe r;
#pragma unroll
  for (int i = 0; i < NL; i++) r.v[i] = src[i];
  return r;
}

extern "C" __global__ void __launch_bounds__(256) k_prepare_points(const uint32_t* __restrict__ wire,
                                                                   uint32_t* __restrict__ pts, uint32_t n,
                                                                   uint32_t* __restrict__ err) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t* src = wire + (size_t)i * 32;
  uint32_t xw[8], yw[8], tw[8], zw[8];
  load_be_words(src, xw);
  load_be_words(src + 8, yw);
  load_be_words(src + 16, tw);
  load_be_words(src + 24, zw);
  bool ok = words_lt_p(xw) && words_lt_p(yw) && words_lt_p(tw) && words_lt_p(zw);
  if (!ok) atomicOr(err, MSM_DEV_ERR_COORD_RANGE);
  bool z_one = zw[0] == 1u;
  bool z_zero = zw[0] == 0u;
#pragma unroll
  for (int k = 1; k < 8; k++) {
    z_one = z_one && zw[k] == 0u;
    z_zero = z_zero && zw[k] == 0u;
  }
  if (z_zero) atomicOr(err, MSM_DEV_ERR_BAD_POINT);
  fe x = fe_to_mont(fe_from_words_le(xw));
  fe y = fe_to_mont(fe_from_words_le(yw));
  fe kt;
  if (z_one) {
    kt = fe_mul(fe_from_words_le(tw), fe_const(K2D_R2_29));
  } else {
    // Projective input (z != 1, README.md:92 allows it): normalise to affine with one inversion.
    fe zi = fe_inv(fe_to_mont(fe_from_words_le(zw)));
    fe t = fe_mul(fe_to_mont(fe_from_words_le(tw)), zi);
    x = fe_mul(x, zi);
    y = fe_mul(y, zi);
    kt = fe_mul(t, fe_const(K2D29));
  }
  fe ymx = fe_sub(y, x);
  fe ypx = fe_add_n(y, x);
  uint32_t rec[32];
#pragma unroll
  for (int k = 0; k < NL; k++) {
    rec[k] = ymx.v[k];
    rec[NL + k] = ypx.v[k];
    rec[2 * NL + k] = kt.v[k];
  }
#pragma unroll
  for (int k = 3 * NL; k < 32; k++) rec[k] = 0;
  uint4* dst = reinterpret_cast<uint4*>(pts + (size_t)i * 32);
#pragma unroll
  for (int k = 0; k < 8; k++) dst[k] = make_uint4(rec[4 * k], rec[4 * k + 1], rec[4 * k + 2], rec[4 * k + 3]);
}

__device__ __forceinline__ pre load_pre(const uint32_t* __restrict__ pts, uint32_t idx) {
  const uint4* src = reinterpret_cast<const uint4*>(pts + (size_t)idx * 32);
  uint32_t rec[28];
#pragma unroll
  for (int k = 0; k < 7; k++) {
    uint4 v = src[k];
    rec[4 * k] = v.x; rec[4 * k + 1] = v.y; rec[4 * k + 2] = v.z; rec[4 * k + 3] = v.w;
  }
  pre q;
#pragma unroll
  for (int k = 0; k < NL; k++) {
    q.ymx.v[k] = rec[k];
    q.ypx.v[k] = rec[NL + k];
    q.kt.v[k] = rec[2 * NL + k];
  }
  return q;
}

// ---------------------------------------------------------------------------------------------
// scalar recoding
// ---------------------------------------------------------------------------------------------
// Raw c-bit window w of a 256-bit little-endian scalar (bits beyond 255 read as zero).
__device__ __forceinline__ uint32_t window_bits(const uint32_t s[8], uint32_t lo_bit, uint32_t c) {
  uint32_t wi = lo_bit >> 5, sh = lo_bit & 31;
  uint32_t lo = wi < 8 ? (s[wi] >> sh) : 0u;
  uint32_t hi = (sh != 0 && wi + 1 < 8) ? (s[wi + 1] << (32 - sh)) : 0u;
  return (lo | hi) & ((1u << c) - 1u);
}

// Signed recoding of one scalar.  Calls f(window, digit) for every window, digit in
// [-(2^(c-1)-1), 2^(c-1)]; sum_w digit_w 2^(c w) == scalar exactly (W = ceil(257/c) windows).
template <typename F>
__device__ __forceinline__ void recode(const uint32_t s[8], const MsmDims& d, F&& f) {
  uint32_t carry = 0;
  for (uint32_t w = 0; w < d.W; w++) {
    uint32_t v = window_bits(s, w * d.c, d.c) + carry;
    int32_t digit;
    if (v > d.B) {
      digit = (int32_t)v - (int32_t)(2 * d.B);
      carry = 1;
    } else {
      digit = (int32_t)v;
      carry = 0;
    }
    f(w, digit);
  }
}

__device__ __forceinline__ void load_scalar(const uint32_t* __restrict__ scalars, uint32_t i, uint32_t s[8]) {
  load_be_words(scalars + (size_t)i * 8, s);
}

extern "C" __global__ void __launch_bounds__(256) k_recode_count(const uint32_t* __restrict__ scalars, MsmDims d,
                                                                 uint32_t* __restrict__ coarse_count) {
  extern __shared__ uint32_t lds_hist[];
  for (uint32_t b = threadIdx.x; b < d.nbins; b += blockDim.x) lds_hist[b] = 0;
  __syncthreads();
  const uint32_t base = blockIdx.x * (blockDim.x * d.spt);
  for (uint32_t k = 0; k < d.spt; k++) {
    uint32_t i = base + k * blockDim.x + threadIdx.x;
    if (i >= d.n) break;
    uint32_t s[8];
    load_scalar(scalars, i, s);
    recode(s, d, [&](uint32_t w, int32_t digit) {
      if (digit != 0) {
        uint32_t b = (uint32_t)(digit < 0 ? -digit : digit) - 1u;
        atomicAdd(&lds_hist[w * d.nbc + (b >> d.fb)], 1u);
      }
    });
  }
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < d.nbins; b += blockDim.x) {
    uint32_t h = lds_hist[b];
    if (h) atomicAdd(&coarse_count[b], h);
  }
}

// Exclusive scan of coarse_count[0..nbins) into coarse_base[0..nbins] (coarse_base[nbins] = total);
// coarse_cursor gets a copy of the bases.  One workgroup of 1024 threads.
extern "C" __global__ void __launch_bounds__(1024) k_coarse_scan(const uint32_t* __restrict__ coarse_count,
                                                                 uint32_t* __restrict__ coarse_base,
                                                                 uint32_t* __restrict__ coarse_cursor, uint32_t nbins) {
  __shared__ uint32_t part[1024];
  const uint32_t per = (nbins + 1023) / 1024;
  const uint32_t lo = threadIdx.x * per;
  uint32_t sum = 0;
  for (uint32_t k = 0; k < per; k++)
    if (lo + k < nbins) sum += coarse_count[lo + k];
  part[threadIdx.x] = sum;
  __syncthreads();
  for (uint32_t off = 1; off < 1024; off <<= 1) {
    uint32_t v = threadIdx.x >= off ? part[threadIdx.x - off] : 0u;
    __syncthreads();
    part[threadIdx.x] += v;
    __syncthreads();
  }
  uint32_t run = part[threadIdx.x] - sum;  // exclusive prefix
  for (uint32_t k = 0; k < per; k++) {
    if (lo + k < nbins) {
      coarse_base[lo + k] = run;
      coarse_cursor[lo + k] = run;
      run += coarse_count[lo + k];
    }
  }
  if (threadIdx.x == 1023) coarse_base[nbins] = part[1023];
}

extern "C" __global__ void __launch_bounds__(256) k_coarse_scatter(const uint32_t* __restrict__ scalars, MsmDims d,
                                                                   uint32_t* __restrict__ coarse_cursor,
                                                                   uint32_t* __restrict__ part_entry,
                                                                   uint16_t* __restrict__ part_fine) {
  extern __shared__ uint32_t lds_hist[];
  for (uint32_t b = threadIdx.x; b < d.nbins; b += blockDim.x) lds_hist[b] = 0;
  __syncthreads();
  const uint32_t base = blockIdx.x * (blockDim.x * d.spt);
  for (uint32_t k = 0; k < d.spt; k++) {
    uint32_t i = base + k * blockDim.x + threadIdx.x;
    if (i >= d.n) break;
    uint32_t s[8];
    load_scalar(scalars, i, s);
    recode(s, d, [&](uint32_t w, int32_t digit) {
      if (digit != 0) {
        uint32_t b = (uint32_t)(digit < 0 ? -digit : digit) - 1u;
        atomicAdd(&lds_hist[w * d.nbc + (b >> d.fb)], 1u);
      }
    });
  }
  __syncthreads();
  // reserve this workgroup's slice of every coarse bin it touches
  for (uint32_t b = threadIdx.x; b < d.nbins; b += blockDim.x) {
    uint32_t h = lds_hist[b];
    lds_hist[b] = h ? atomicAdd(&coarse_cursor[b], h) : 0u;
  }
  __syncthreads();
  const uint32_t fmask = (1u << d.fb) - 1u;
  for (uint32_t k = 0; k < d.spt; k++) {
    uint32_t i = base + k * blockDim.x + threadIdx.x;
    if (i >= d.n) break;
    uint32_t s[8];
    load_scalar(scalars, i, s);
    recode(s, d, [&](uint32_t w, int32_t digit) {
      if (digit != 0) {
        uint32_t b = (uint32_t)(digit < 0 ? -digit : digit) - 1u;
        uint32_t pos = atomicAdd(&lds_hist[w * d.nbc + (b >> d.fb)], 1u);
        part_entry[pos] = (i << 1) | (digit < 0 ? 1u : 0u);
        part_fine[pos] = (uint16_t)(b & fmask);
      }
    });
  }
}

// One workgroup per coarse bin: counting sort of the bin's entries by fine bucket.
extern "C" __global__ void __launch_bounds__(256) k_fine_sort(const uint32_t* __restrict__ part_entry,
                                                              const uint16_t* __restrict__ part_fine,
                                                              const uint32_t* __restrict__ coarse_base, MsmDims d,
                                                              uint32_t* __restrict__ sorted_entry,
                                                              uint32_t* __restrict__ sorted_key,
                                                              uint32_t* __restrict__ bucket_count) {
  __shared__ uint32_t cnt[512];
  __shared__ uint32_t scan_tmp[256];
  const uint32_t bin = blockIdx.x;
  const uint32_t nf = 1u << d.fb;
  const uint32_t base = coarse_base[bin];
  const uint32_t m = coarse_base[bin + 1] - base;
  const uint32_t w = bin / d.nbc, cb = bin % d.nbc;
  const uint32_t key0 = w * d.B + (cb << d.fb);
  for (uint32_t f = threadIdx.x; f < nf; f += blockDim.x) cnt[f] = 0;
  __syncthreads();
  for (uint32_t e = threadIdx.x; e < m; e += blockDim.x) atomicAdd(&cnt[part_fine[base + e]], 1u);
  __syncthreads();
  // exclusive scan of cnt[0..nf) (nf <= 512: two values per thread)
  uint32_t c0 = 0, c1 = 0;
  const uint32_t f0 = 2 * threadIdx.x, f1 = 2 * threadIdx.x + 1;
  if (f0 < nf) c0 = cnt[f0];
  if (f1 < nf) c1 = cnt[f1];
  scan_tmp[threadIdx.x] = c0 + c1;
  __syncthreads();
  for (uint32_t off = 1; off < 256; off <<= 1) {
    uint32_t v = threadIdx.x >= off ? scan_tmp[threadIdx.x - off] : 0u;
    __syncthreads();
    scan_tmp[threadIdx.x] += v;
    __syncthreads();
  }
  uint32_t ex = scan_tmp[threadIdx.x] - (c0 + c1);
  __syncthreads();
  if (f0 < nf) {
    bucket_count[key0 + f0] = c0;
    cnt[f0] = ex;
  }
  if (f1 < nf) {
    bucket_count[key0 + f1] = c1;
    cnt[f1] = ex + c0;
  }
  __syncthreads();
  for (uint32_t e = threadIdx.x; e < m; e += blockDim.x) {
    uint32_t f = part_fine[base + e];
    uint32_t pos = base + atomicAdd(&cnt[f], 1u);
    sorted_entry[pos] = part_entry[base + e];
    sorted_key[pos] = key0 + f;
  }
}

// ---------------------------------------------------------------------------------------------
// bucket accumulation
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void store_pt(uint32_t* __restrict__ dst, const xyzt& p) {
  uint32_t rec[36];
#pragma unroll
  for (int k = 0; k < NL; k++) {
    rec[k] = p.X.v[k];
    rec[NL + k] = p.Y.v[k];
    rec[2 * NL + k] = p.T.v[k];
    rec[3 * NL + k] = p.Z.v[k];
  }
  uint4* d4 = reinterpret_cast<uint4*>(dst);
#pragma unroll
  for (int k = 0; k < 9; k++) d4[k] = make_uint4(rec[4 * k], rec[4 * k + 1], rec[4 * k + 2], rec[4 * k + 3]);
}
__device__ __forceinline__ xyzt load_pt(const uint32_t* __restrict__ src) {
  uint32_t rec[36];
  const uint4* s4 = reinterpret_cast<const uint4*>(src);
#pragma unroll
  for (int k = 0; k < 9; k++) {
    uint4 v = s4[k];
    rec[4 * k] = v.x; rec[4 * k + 1] = v.y; rec[4 * k + 2] = v.z; rec[4 * k + 3] = v.w;
  }
  xyzt p;
#pragma unroll
  for (int k = 0; k < NL; k++) {
    p.X.v[k] = rec[k];
    p.Y.v[k] = rec[NL + k];
    p.T.v[k] = rec[2 * NL + k];
    p.Z.v[k] = rec[3 * NL + k];
  }
  return p;
}

// Write one finished segment of the sorted list.  Whole buckets go straight to the bucket table;
// a segment cut by the run start (head) or run end (tail) goes to the run's partial slots.
__device__ __forceinline__ void flush_segment(const xyzt& acc, uint32_t key, bool is_head, bool is_tail, uint32_t t,
                                              uint32_t* __restrict__ buckets, uint32_t* __restrict__ run_head,
                                              uint32_t* __restrict__ run_tail, uint32_t* __restrict__ head_key,
                                              uint32_t* __restrict__ tail_key) {
  if (is_head) {
    store_pt(run_head + (size_t)t * PT_WORDS, acc);
    head_key[t] = key | (is_tail ? KEY_PASS : 0u);
  } else if (is_tail) {
    store_pt(run_tail + (size_t)t * PT_WORDS, acc);
    tail_key[t] = key;
  } else {
    store_pt(buckets + (size_t)key * PT_WORDS, acc);
  }
}

extern "C" __global__ void __launch_bounds__(256) k_accumulate(const uint32_t* __restrict__ pts,
                                                               const uint32_t* __restrict__ sorted_entry,
                                                               const uint32_t* __restrict__ sorted_key,
                                                               const uint32_t* __restrict__ total_ptr, uint32_t K,
                                                               uint32_t* __restrict__ buckets,
                                                               uint32_t* __restrict__ run_head,
                                                               uint32_t* __restrict__ run_tail,
                                                               uint32_t* __restrict__ head_key,
                                                               uint32_t* __restrict__ tail_key) {
  const uint32_t M = *total_ptr;
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t s = t * K;
  if (s >= M) return;
  const uint32_t e = min(s + K, M);
  head_key[t] = KEY_INVALID;
  tail_key[t] = KEY_INVALID;
  uint32_t cur = sorted_key[s];
  const bool started_before = s > 0 && sorted_key[s - 1] == cur;
  bool seg_first = true;
  xyzt acc = pt_identity();
  for (uint32_t pos = s; pos < e; pos++) {
    uint32_t k = sorted_key[pos];
    if (k != cur) {
      flush_segment(acc, cur, seg_first && started_before, false, t, buckets, run_head, run_tail, head_key, tail_key);
      acc = pt_identity();
      cur = k;
      seg_first = false;
    }
    uint32_t ent = sorted_entry[pos];
    pre q = pre_neg_if(load_pre(pts, ent >> 1), (ent & 1u) != 0);
    acc = pt_madd(acc, q);
  }
  const bool cont = e < M && sorted_key[e] == cur;
  flush_segment(acc, cur, seg_first && started_before, cont, t, buckets, run_head, run_tail, head_key, tail_key);
}

// Joins a bucket cut across runs: tail partial of run t + head partials of runs t+1.. (pass-through
// runs continue the chain).
extern "C" __global__ void __launch_bounds__(256) k_fixup(const uint32_t* __restrict__ total_ptr, uint32_t K,
                                                          const uint32_t* __restrict__ run_head,
                                                          const uint32_t* __restrict__ run_tail,
                                                          const uint32_t* __restrict__ head_key,
                                                          const uint32_t* __restrict__ tail_key,
                                                          uint32_t* __restrict__ buckets) {
  const uint32_t M = *total_ptr;
  const uint32_t nruns = (M + K - 1) / K;
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nruns) return;
  const uint32_t key = tail_key[t];
  if (key == KEY_INVALID) return;
  xyzt acc = load_pt(run_tail + (size_t)t * PT_WORDS);
  for (uint32_t u = t + 1; u < nruns; u++) {
    acc = pt_add(acc, load_pt(run_head + (size_t)u * PT_WORDS));
    const uint32_t hk = head_key[u];
    if (hk == KEY_INVALID || !(hk & KEY_PASS)) break;
  }
  store_pt(buckets + (size_t)key * PT_WORDS, acc);
}

// ---------------------------------------------------------------------------------------------
// bucket reduction:  G_w = sum_{b} (b+1) B_{w,b}
//   chunk c (L buckets): U_c = sum_i (i+1) B_{cL+i}, T_c = sum_i B_{cL+i}   (running sums)
//   G_w = sum_c U_c + L * sum_c c T_c = R_{w,V} + sum_k 2^(lgL+k) R_{w,k},  R_{w,k} = sum_{c: bit k} T_c
// ---------------------------------------------------------------------------------------------
extern "C" __global__ void __launch_bounds__(256) k_bucket_reduce_1(const uint32_t* __restrict__ buckets,
                                                                    const uint32_t* __restrict__ bucket_count, MsmDims d,
                                                                    uint32_t L, uint32_t* __restrict__ out_U,
                                                                    uint32_t* __restrict__ out_T) {
  const uint32_t nchunks = d.B / L;
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= d.W * nchunks) return;
  const uint32_t w = g / nchunks, c = g % nchunks;
  const uint32_t key0 = w * d.B + c * L;
  xyzt carry = pt_identity(), acc = pt_identity();
  bool carry_live = false, acc_live = false;
  for (int i = (int)L - 1; i >= 0; i--) {
    if (bucket_count[key0 + i]) {
      xyzt b = load_pt(buckets + (size_t)(key0 + i) * PT_WORDS);
      carry = carry_live ? pt_add(carry, b) : b;
      carry_live = true;
    }
    if (carry_live) {
      acc = acc_live ? pt_add(acc, carry) : carry;
      acc_live = true;
    }
  }
  store_pt(out_U + (size_t)g * PT_WORDS, acc);
  store_pt(out_T + (size_t)g * PT_WORDS, carry);
}

// One workgroup per (window, term).  term 0: R_V = sum_c U_c; term 1+k: R_k = sum_{c: bit k of c} T_c.
// Output: X, Y, T, Z in canonical standard form (8 LE words each) for the host.
constexpr int RED2_THREADS = 256;
extern "C" __global__ void __launch_bounds__(RED2_THREADS) k_bucket_reduce_2(const uint32_t* __restrict__ in_U,
                                                                             const uint32_t* __restrict__ in_T,
                                                                             uint32_t nchunks, uint32_t nterms,
                                                                             uint32_t* __restrict__ out_std) {
  __shared__ uint32_t sh[RED2_THREADS / 2][PT_WORDS];
  const uint32_t w = blockIdx.x / nterms, term = blockIdx.x % nterms;
  const uint32_t* src = term == 0 ? in_U : in_T;
  const uint32_t kbit = term - 1;
  xyzt acc = pt_identity();
  bool live = false;
  // the terms this thread owns: chunks c = tid, tid + 256, ... with (term==0 || bit k of c set)
  for (uint32_t c = threadIdx.x; c < nchunks; c += RED2_THREADS) {
    if (term != 0 && !((c >> kbit) & 1u)) continue;
    xyzt p = load_pt(src + ((size_t)w * nchunks + c) * PT_WORDS);
    acc = live ? pt_add(acc, p) : p;
    live = true;
  }
  // tree reduce through LDS: upper half hands its point to the lower half each round
  for (uint32_t half = RED2_THREADS / 2; half >= 1; half >>= 1) {
    if (threadIdx.x >= half && threadIdx.x < 2 * half) store_pt(sh[threadIdx.x - half], acc);
    __syncthreads();
    if (threadIdx.x < half) acc = pt_add(acc, load_pt(sh[threadIdx.x]));
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    uint32_t* o = out_std + (size_t)blockIdx.x * 32;
    fe c4[4] = {fe_to_std(acc.X), fe_to_std(acc.Y), fe_to_std(acc.T), fe_to_std(acc.Z)};
#pragma unroll
    for (int q = 0; q < 4; q++) fe_to_words_le(c4[q], o + 8 * q);
  }
}

// Small utility kernels used by tests: batch field ops / point ops on canonical inputs.
// op 0: field mul, 1: add, 2: sub; inputs LE standard words [n][8] x2, output [n][8].
extern "C" __global__ void k_test_field(const uint32_t* __restrict__ a, const uint32_t* __restrict__ b,
                                        uint32_t* __restrict__ out, uint32_t n, uint32_t op) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t aw[8], bw[8], ow[8];
#pragma unroll
  for (int k = 0; k < 8; k++) {
    aw[k] = a[(size_t)i * 8 + k];
    bw[k] = b[(size_t)i * 8 + k];
  }
  fe x = fe_to_mont(fe_from_words_le(aw)), y = fe_to_mont(fe_from_words_le(bw));
  fe r = op == 0 ? fe_mul(x, y) : op == 1 ? fe_add_n(x, y) : fe_sub(x, y);
  fe_to_words_le(fe_to_std(r), ow);
#pragma unroll
  for (int k = 0; k < 8; k++) out[(size_t)i * 8 + k] = ow[k];
}

// op 0: P + Q via pt_add, 1: P + Q via pt_madd (Q affine from its x,y), 2: 2P via pt_dbl.
// Inputs: affine points as LE words [n][16] (x, y); output affine-projective X,Y,T,Z std LE words [n][32].
template <int OP>
__global__ void k_test_point(const uint32_t* __restrict__ p, const uint32_t* __restrict__ q,
                             uint32_t* __restrict__ out, uint32_t n) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t w[4][8];
#pragma unroll
  for (int k = 0; k < 8; k++) {
    w[0][k] = p[(size_t)i * 16 + k];
    w[1][k] = p[(size_t)i * 16 + 8 + k];
    w[2][k] = q[(size_t)i * 16 + k];
    w[3][k] = q[(size_t)i * 16 + 8 + k];
  }
  xyzt P;
  P.X = fe_to_mont(fe_from_words_le(w[0]));
  P.Y = fe_to_mont(fe_from_words_le(w[1]));
  P.T = fe_mul(P.X, P.Y);
  P.Z = fe_one();
  xyzt Q;
  Q.X = fe_to_mont(fe_from_words_le(w[2]));
  Q.Y = fe_to_mont(fe_from_words_le(w[3]));
  Q.T = fe_mul(Q.X, Q.Y);
  Q.Z = fe_one();
  xyzt R;
  if constexpr (OP == 0) {
    R = pt_add(P, Q);
  } else if constexpr (OP == 1) {
    pre qq;
    qq.ymx = fe_sub(Q.Y, Q.X);
    qq.ypx = fe_add_n(Q.Y, Q.X);
    qq.kt = fe_mul(Q.T, fe_const(K2D29));
    R = pt_madd(P, qq);
  } else {
    R = pt_dbl(P);
  }
  fe c4[4] = {fe_to_std(R.X), fe_to_std(R.Y), fe_to_std(R.T), fe_to_std(R.Z)};
  uint32_t ow[8];
#pragma unroll
  for (int qd = 0; qd < 4; qd++) {
    fe_to_words_le(c4[qd], ow);
#pragma unroll
    for (int k = 0; k < 8; k++) out[(size_t)i * 32 + qd * 8 + k] = ow[k];
  }
}

}  // namespace msm
