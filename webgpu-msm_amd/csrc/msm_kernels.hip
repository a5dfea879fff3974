// Pippenger MSM kernels for MI355X (gfx950).  Replaces the reference's GPU intra-bucket
// reduction (src/submission/gpu.ts:36-285 + wgsl/entry_padd_idx.wgsl:23-46) and its Rust
// split / inter-bucket reduce (src/submission/msm-wasm/src/lib.rs:46-133) with one on-device
// pipeline:
//
//   k_prepare_points   wire points (BE x|y|t|z, 128 B) -> halved precomputed affine records
//                      ((y-x)/2, (y+x)/2, d t) in 29-bit Montgomery limbs, 128 B (one cache line)
//   k_recode_hist      signed c-bit digits per scalar (window-carry recoding, |d| <= 2^(c-1)),
//                      written window-major (= first sort level: one contiguous array per window),
//                      with the coarse-bin totals (LDS histogram, flushed with global atomics)
//   k_part_scatter     digits -> coarse bins (each chunk reserves and writes one contiguous slice
//                      per bin)
//   k_fine_sort        per coarse bin: LDS counting sort by bucket -> (entry, bucket key) lists
//   k_accumulate       fixed-length runs per lane over the sorted list (mixed adds), whole buckets
//                      written directly, buckets cut by run boundaries joined through LDS
//                      (segmented scan for long chains)
//   k_lead_scan        chains bucket continuations that run through whole workgroups (skew only)
//   k_bucket_reduce_1  per (window, chunk of L buckets): running sums -> U_c = sum (i+1) B, T_c = sum B
//   k_red2_groups      per (window, group of 128 chunks): V_g = sum U_c, S_g = sum T_c and the
//                      group's low bit terms R_{g,k}, in LDS (quad-cooperative adds)
//   k_red2_terms       per (window, term): R_{w,V} = sum V_g, R_{w,k} = sum_g R_{g,k} or
//                      sum_{g: bit k-7} S_g, in the host's Montgomery form for the host Horner
//   k_bucket_reduce_2  the same terms straight from every chunk's U_c / T_c (windows of more than
//                      64 groups, or MSM_RED2_TREE=0)
//
// Digit semantics differ from the reference's (unsigned, MSB-first, lib.rs:58-84 + msm-macro) on
// purpose: only the final affine (x, y) is the parity contract, and signed digits halve the
// bucket count.
#include "ec.cuh"
#include "msm_dev.h"


namespace msm {

// Phase probe (tuning builds only, -DMSM_PHASE_PROBE=1): thread 0 of each workgroup of the sort
// kernels stamps the shader clock at its phase boundaries into g_probe[kernel][workgroup][slot]
// (slots 8 and 9: the 100 MHz real-time clock at slots 0 and 7); msm_test_probe_dump writes the
// last launch's stamps to a file (tools/phase_probe.py reads them).
#ifdef MSM_PHASE_PROBE
constexpr uint32_t PROBE_WG = 16384, PROBE_SLOTS = 10;
__device__ uint64_t g_probe[4][PROBE_WG][PROBE_SLOTS];
#define PROBE(k, wg, s)                                                                   \
  do {                                                                                   \
    if (threadIdx.x == 0 && (wg) < PROBE_WG) {                                           \
      g_probe[k][wg][s] = __builtin_readcyclecounter();                                  \
      if ((s) == 0 || (s) == 7) g_probe[k][wg][8 + ((s) == 7)] = __builtin_amdgcn_s_memrealtime(); \
    }                                                                                    \
  } while (0)
#define PROBE_WAIT_VM() asm volatile("s_waitcnt vmcnt(0)" ::: "memory")
#else
#define PROBE(k, wg, s) \
  do {                  \
  } while (0)
#define PROBE_WAIT_VM() \
  do {                  \
  } while (0)
#endif

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

// One workgroup = PP_THREADS points.  Wire records and output records (128 B each) move between
// HBM and LDS with fully coalesced 16-B accesses (a wave covers 1 KiB contiguous per
// instruction); each lane then works on its own point out of LDS.  The 16-B slots of a record are
// XOR-swizzled by the record index so the per-lane 128-B-strided LDS reads and writes are free of
// bank conflicts.  With `nt` the records are written with nontemporal stores: the host sets it
// when a launch's records outgrow the 256 MiB Infinity Cache, where the regular write-back stores
// only evict lines that the gather in k_accumulate will not find there anyway (measured -11% on
// this kernel at 2 x 2^20 points; smaller launches keep their records cache-resident).
#ifndef MSM_PP_THREADS
#define MSM_PP_THREADS 256
#endif
constexpr uint32_t PP_THREADS = MSM_PP_THREADS;
static_assert(PP_THREADS * 8 <= (1u << 16), "k_prepare_points' multiply-high slot division");
typedef uint32_t pp_v4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint32_t pp_slot(uint32_t rec, uint32_t q) { return rec * 8 + (q ^ (rec & 7)); }

// Input point formats (`fmt`): PT_FMT_WIRE the reference's 128-B x|y|t|z records; the compact
// forms of host uploads (run_host_split) leave t out -- PT_FMT_XYZ 96 B x|y|z, PT_FMT_XY 64 B x|y
// with z = 1 -- and the record's d t is derived from x and y (the oracle's own semantics: Aleo's
// msm reads affine (x, y)).
constexpr uint32_t PT_FMT_WIRE = 0, PT_FMT_XY = 1, PT_FMT_XYZ = 2;
__host__ __device__ constexpr uint32_t pt_fmt_slots(uint32_t fmt) {  // 16-B slots per input point
  return fmt == PT_FMT_XY ? 4u : fmt == PT_FMT_XYZ ? 6u : 8u;
}

// blockIdx.y = MSM of the batch: its wire points come from wires.p[y], its records go to
// pts[y n ..).
extern "C" __global__ void __launch_bounds__(PP_THREADS) k_prepare_points(BatchPtrs wires,
                                                                          uint32_t* __restrict__ pts, uint32_t n,
                                                                          uint32_t* __restrict__ err, uint32_t nt,
                                                                          uint32_t fmt) {
  __shared__ uint4 st[PP_THREADS * 8];
  const uint32_t S = pt_fmt_slots(fmt);
  // g / S for the wave-uniform S in {4, 6, 8} as one multiply-high (exact for g < 2^16; the
  // generic unsigned division it replaces cost ~12 VALU per slot)
  const uint32_t s_inv = S == 8 ? (1u << 29) : S == 4 ? (1u << 30) : 0x2AAAAAABu;
  const uint32_t p0 = blockIdx.x * PP_THREADS;
  const uint32_t np = min(PP_THREADS, n - p0);
  const uint4* src = reinterpret_cast<const uint4*>(wires.p[blockIdx.y]) + (size_t)p0 * S;
  pts += (size_t)blockIdx.y * n * PRE_WORDS;
#pragma unroll
  for (uint32_t j = 0; j < 8; j++) {
    const uint32_t g = j * PP_THREADS + threadIdx.x;  // 16-B slot within the block's records
    const uint32_t rec = __umulhi(g, s_inv);
    if (g < np * S) st[pp_slot(rec, g - rec * S)] = src[g];
  }
  __syncthreads();
  const uint32_t i = threadIdx.x;
  const bool live = i < np;
  const bool has_t = fmt == PT_FMT_WIRE, has_z = fmt != PT_FMT_XY;  // t: range check only
  uint32_t xw[8], yw[8], tw[8], zw[8];
#pragma unroll
  for (int k = 0; k < 8; k++) xw[k] = yw[k] = tw[k] = zw[k] = 0;
  zw[0] = 1;
  if (live) {
    uint4 v[8];
#pragma unroll
    for (uint32_t q = 0; q < 8; q++) v[q] = q < S ? st[pp_slot(i, q)] : make_uint4(0u, 0u, 0u, 0u);
    // big-endian word order: word 0 is the most significant 32 bits (bytes.rs:11-20); the
    // compact forms hold x, y (and z) in that order
    uint32_t* dsts[4] = {xw, yw, has_t ? tw : zw, zw};
#pragma unroll
    for (int f = 0; f < 4; f++) {
      if (f == 3 && !has_t) break;   // x|y|z: z was the third field
      if (f == 2 && !has_z) break;   // x|y
      const uint4 a = v[2 * f], b = v[2 * f + 1];
      uint32_t* le = dsts[f];
      le[7] = a.x; le[6] = a.y; le[5] = a.z; le[4] = a.w;
      le[3] = b.x; le[2] = b.y; le[1] = b.z; le[0] = b.w;
    }
  }
  __syncthreads();
  bool ok = words_lt_p(xw) && words_lt_p(yw) && words_lt_p(tw) && words_lt_p(zw);
  if (live && !ok) atomicOr(err, MSM_DEV_ERR_COORD_RANGE);
  bool z_one = zw[0] == 1u;
  bool z_zero = zw[0] == 0u;
#pragma unroll
  for (int k = 1; k < 8; k++) {
    z_one = z_one && zw[k] == 0u;
    z_zero = z_zero && zw[k] == 0u;
  }
  if (live && z_zero) atomicOr(err, MSM_DEV_ERR_BAD_POINT);
  // the halved record (ec.cuh pt_madd): x/2, y/2 and d*t in Montgomery form
  // d t is derived from the affine x and y in every format: the input t is range-checked above
  // but not used, so a record's result depends on (x, y, z) alone, as the oracle's does (Aleo's
  // msm reads affine points), whichever entry and upload form carried it
  fe x, y;
  if (z_one) {
    x = fe_mul(fe_from_words_le(xw), fe_const(R2H_29));
    y = fe_mul(fe_from_words_le(yw), fe_const(R2H_29));
  } else {
    // Projective input (z != 1, README.md:92 allows it): normalise to affine with one inversion.
    fe zi = fe_inv(fe_to_mont(fe_from_words_le(zw)));
    fe zh = fe_mul(zi, fe_const(HALF29));
    x = fe_mul(fe_to_mont(fe_from_words_le(xw)), zh);
    y = fe_mul(fe_to_mont(fe_from_words_le(yw)), zh);
  }
  // d x y: (2 (x/2)) (2 (y/2)) = x y in Montgomery form (S x S operands), then d by limb scaling
  const fe kt = fe_mul_d(fe_mul(fe_add(x, x), fe_add(y, y)));
  fe ymx = fe_sub(y, x);
  fe ypx = fe_add_n(y, x);
  uint32_t rec[32];  // layout: msm_dev.h PRE_WORDS
#pragma unroll
  for (int k = 0; k < 32; k++) rec[k] = 0;
#pragma unroll
  for (int k = 0; k < NL; k++) {
    rec[k] = ymx.v[k];
    rec[PRE_HALF + k] = ypx.v[k];
  }
#pragma unroll
  for (int k = 0; k < NL - 1; k++) rec[PRE_KT + k] = kt.v[k];
  // each half also carries d*t's top limb and the OTHER half's top limb: the half read first
  // supplies both, so the half read second needs only its eight low limbs (seven loads in all)
  rec[NL] = rec[PRE_HALF + NL] = kt.v[NL - 1];
  rec[NL + 1] = ypx.v[NL - 1];
  rec[PRE_HALF + NL + 1] = ymx.v[NL - 1];
#pragma unroll
  for (uint32_t q = 0; q < 8; q++)
    st[pp_slot(i, q)] = make_uint4(rec[4 * q], rec[4 * q + 1], rec[4 * q + 2], rec[4 * q + 3]);
  __syncthreads();
  uint4* dst = reinterpret_cast<uint4*>(pts) + (size_t)p0 * 8;
#pragma unroll
  for (uint32_t j = 0; j < 8; j++) {
    const uint32_t g = j * PP_THREADS + threadIdx.x;
    if (g < np * 8) {
      const uint4 v = st[pp_slot(g >> 3, g & 7)];
      if (nt) {
        const pp_v4 w = {v.x, v.y, v.z, v.w};
        __builtin_nontemporal_store(w, reinterpret_cast<pp_v4*>(dst + g));
      } else {
        dst[g] = v;
      }
    }
  }
}

// Pads a short host-input slice on the device (run_host_split with n not a multiple of its slice
// count): `count` points set to the identity (x, y, t, z) = (0, 1, 0, 1) -- in the input format
// `fmt` of the slice's point buffer (wire records, or the compact x|y|z of a compact upload) --
// and `count` scalars set to 0, so the padding contributes no bucket entry.  16-B stores, one
// per thread.
extern "C" __global__ void __launch_bounds__(256) k_pad_identity(uint32_t* __restrict__ wire_pts,
                                                                   uint32_t* __restrict__ wire_sc, uint32_t count,
                                                                   uint32_t fmt) {
  const uint32_t S = pt_fmt_slots(fmt);
  const uint32_t g = blockIdx.x * 256 + threadIdx.x;  // 16-B slot: S per point, then 2 per scalar
  if (g < count * S) {
    // BE words: the least significant word of y (slot 3), and of z (the point's last slot) unless
    // the format has no z
    const uint32_t q = g % S;
    const bool one = q == 3 || (fmt != PT_FMT_XY && q == S - 1);
    reinterpret_cast<uint4*>(wire_pts)[g] = make_uint4(0u, 0u, 0u, one ? 1u : 0u);
  } else if (g < count * (S + 2)) {
    reinterpret_cast<uint4*>(wire_sc)[g - count * S] = make_uint4(0u, 0u, 0u, 0u);
  }
}

// Gathers the record of sorted entry `ent` (point index << 1 | sign) as the point it adds:
// a negated point's (y-x)/2 and (y+x)/2 swap by reading the record's halves in the other order
// (msm_dev.h PRE_WORDS), and its d*t is negated (kt_neg_if).
__device__ __forceinline__ pre load_pre_signed(const uint32_t* __restrict__ pts, uint32_t ent) {
  const uint32_t sgn = ent & 1u;
  const bool neg = sgn != 0;
  // byte offsets: record (ent >> 1) * 128 = (ent & ~1) * 64; halves at 48 sgn and 48 (1 - sgn)
  const char* rec = reinterpret_cast<const char*>(pts) + ((size_t)(ent & ~1u) << 6);
  const uint32_t o0 = sgn * (PRE_HALF * 4);
  const uint32_t* h0 = reinterpret_cast<const uint32_t*>(rec + o0);
  const uint32_t* h1 = reinterpret_cast<const uint32_t*>(rec + (o0 ^ (PRE_HALF * 4)));
  const uint4 a0 = reinterpret_cast<const uint4*>(h0)[0], a1 = reinterpret_cast<const uint4*>(h0)[1];
  const uint4 a2 = reinterpret_cast<const uint4*>(h0)[2];  // top limb, d*t's top limb, the other half's top limb
  const uint4 b0 = reinterpret_cast<const uint4*>(h1)[0], b1 = reinterpret_cast<const uint4*>(h1)[1];
  const uint32_t b2 = a2.z;
  const uint4 c0 = reinterpret_cast<const uint4*>(rec + PRE_KT * 4)[0];
  const uint4 c1 = reinterpret_cast<const uint4*>(rec + PRE_KT * 4)[1];
  const uint32_t av[NL] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w, a2.x};
  const uint32_t bv[NL] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w, b2};
  const uint32_t kv[NL] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w, a2.y};
  pre q;
#pragma unroll
  for (int k = 0; k < NL; k++) {
    q.ymx.v[k] = av[k];
    q.ypx.v[k] = bv[k];
    q.kt.v[k] = kv[k];
  }
  q.kt = kt_neg_if(q.kt, neg);
  return q;
}

// ---------------------------------------------------------------------------------------------
// scalar recoding
// ---------------------------------------------------------------------------------------------
// Signed recoding of one scalar (little-endian words, consumed in place).  Calls f(window,
// digit) for every window, digit in [-(2^(b-1)-1), 2^(b-1)] for a window of b bits (win_bits);
// sum_w digit_w 2^win_off(w) == scalar exactly.  The scalar is shifted down b bits per window
// with v_alignbit so no register array is ever indexed dynamically (that would spill it to
// scratch).
template <typename F>
__device__ __forceinline__ void recode(uint32_t s[8], const MsmDims& d, F&& f) {
  uint32_t carry = 0;
  // carries only climb: a window range's digits need the windows below it, never those above
  // (a lower share of a windows split stops at its top window)
  const uint32_t wend = d.w0 + d.Wr;
  for (uint32_t w = 0; w < wend; w++) {
    const uint32_t b = win_bits(d, w);
    const uint32_t half = 1u << (b - 1);
    const uint32_t v = (s[0] & ((1u << b) - 1u)) + carry;
#pragma unroll
    for (int q = 0; q < 7; q++) s[q] = __builtin_amdgcn_alignbit(s[q + 1], s[q], b);
    s[7] >>= b;
    int32_t digit;
    if (v > half) {
      digit = (int32_t)v - (int32_t)(2 * half);
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

// Wave-level inclusive scan of one u32 per lane (64 lanes, all active) by DPP: four row shifts
// scan each 16-lane row, two row broadcasts carry the rows' totals across.  No LDS round trips
// (the ds_bpermute form took ~0.5 us of latency per scan, a tenth of a k_fine_sort workgroup's life).
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);  // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);  // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);  // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);  // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return x;
}
// Exclusive scan of one u32 per lane; `total` = the wave sum.
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v, uint32_t& total) {
  const uint32_t x = wave_incl_scan(v);
  total = (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
  return x - v;
}

// Exclusive scan of cnt[0..nf) in LDS by the first wave of the workgroup.  256 counters (the
// scatter's bins, the wide fine sorts) go as one 16-B vector per lane and 128 as one 8-B vector;
// other multiples of 256 as runs of vectors read twice (a register array would cost the calling
// kernels their occupancy); other counts take the scalar loop.
__device__ __forceinline__ void lds_excl_scan_wave0(uint32_t* cnt, uint32_t nf) {
  if (threadIdx.x >= 64) return;
  const uint32_t lane = threadIdx.x;
  if (nf == 256) {
    uint4* c4 = reinterpret_cast<uint4*>(cnt) + lane;
    const uint4 v = *c4;
    uint32_t tot;
    const uint32_t run = wave_excl_scan(v.x + v.y + v.z + v.w, tot);
    *c4 = make_uint4(run, run + v.x, run + v.x + v.y, run + v.x + v.y + v.z);
    return;
  }
  if ((nf & 255u) == 0) {
    const uint32_t n4 = nf / 256;  // uint4s per lane
    uint4* c4 = reinterpret_cast<uint4*>(cnt) + lane * n4;
    uint32_t local = 0;
    for (uint32_t k = 0; k < n4; k++) {
      const uint4 v = c4[k];
      local += v.x + v.y + v.z + v.w;
    }
    uint32_t tot;
    uint32_t run = wave_excl_scan(local, tot);
    for (uint32_t k = 0; k < n4; k++) {
      const uint4 v = c4[k];
      c4[k] = make_uint4(run, run + v.x, run + v.x + v.y, run + v.x + v.y + v.z);
      run += v.x + v.y + v.z + v.w;
    }
    return;
  }
  if (nf == 128) {
    uint2* c2 = reinterpret_cast<uint2*>(cnt) + lane;
    const uint2 v = *c2;
    uint32_t tot;
    const uint32_t run = wave_excl_scan(v.x + v.y, tot);
    *c2 = make_uint2(run, run + v.x);
    return;
  }
  const uint32_t per = (nf + 63) / 64;
  const uint32_t lo = lane * per;
  uint32_t local = 0;
  for (uint32_t k = 0; k < per; k++)
    if (lo + k < nf) local += cnt[lo + k];
  uint32_t tot;
  uint32_t run = wave_excl_scan(local, tot);
  for (uint32_t k = 0; k < per; k++) {
    if (lo + k < nf) {
      const uint32_t c = cnt[lo + k];
      cnt[lo + k] = run;
      run += c;
    }
  }
}

// Fine bits of MSM window `wm`: every window keeps nbc coarse bins over its OWN buckets, so a
// window narrower than the widest (the balanced 15-bit windows at c = 16, the 13-bit ones at
// c = 14, the 3-bit overflow window) sorts fb - (c - b) fine bits per bin and its bins are as full
// as the others'.  (With one fb for all, half of such a window's bins held all its entries --
// 8,192 per bin at 2^20, past k_fine_sort's LDS staging -- and took the slow unstaged path.)
__device__ __forceinline__ uint32_t win_fb(const MsmDims& d, uint32_t wm) {
  const uint32_t drop = d.c - win_bits(d, wm);
  return d.fb > drop ? d.fb - drop : 0u;
}
// The same for window w of a launch's batch (w in [0, W): MSM w / Wr, local window w % Wr).
__device__ __forceinline__ uint32_t batch_win_fb(const MsmDims& d, uint32_t w) { return win_fb(d, d.w0 + w % d.Wr); }

// Digit codes, window-major digits[w][i]: bucket b = |d| - 1 plus a sign bit, or ZERO.
//   c <= 16: uint16_t, sign = bit 15, ZERO = 0xffff (b = 0x7fff with the sign set would be
//            d = -2^15, which signed recoding never produces)
//   c >  16: uint32_t, sign = bit 31, ZERO = 0xffffffff
template <typename T>
struct DigitCode;
template <>
struct DigitCode<uint16_t> {
  static constexpr uint32_t ZERO = 0xffffu, SIGN = 0x8000u, MAG = 0x7fffu, SHIFT = 15;
};
template <>
struct DigitCode<uint32_t> {
  static constexpr uint32_t ZERO = 0xffffffffu, SIGN = 0x80000000u, MAG = 0x7fffffffu, SHIFT = 31;
};

// Pass 0+1 (fused): each workgroup recodes RC_SPAN scalars into window-major digit codes (the
// window-major layout is the first sort level for free: each window is one contiguous array) and
// builds, in LDS, their histogram over every window's nbc coarse bins, flushed with global
// atomics into the bin totals colsum[w][bin] (kept zeroed between MSMs by k_fine_sort).  Digits
// are read back only once, by k_part_scatter.
#ifndef MSM_PT_THREADS
#define MSM_PT_THREADS 1024
#endif
#ifndef MSM_PS_R
#define MSM_PS_R 16
#endif
constexpr uint32_t PT_THREADS = MSM_PT_THREADS;
constexpr uint32_t PS_R = MSM_PS_R;  // digits per lane (ch = PT_THREADS * PS_R)
#ifndef MSM_RC_THREADS
#define MSM_RC_THREADS 1024
#endif
constexpr uint32_t RC_THREADS = MSM_RC_THREADS;
#ifndef MSM_RC_SPAN
#define MSM_RC_SPAN 4096
#endif
constexpr uint32_t RC_SPAN = MSM_RC_SPAN;  // scalars per recode workgroup
// Signed recoding with the window geometry fixed at compile time (the common widths: q = 15,
// nhi = 14 is c = 16; 14/16 c = 15; 13/7 c = 14; 12/14 c = 13).  Adding the constant
// C = sum_w (2^(b_w - 1) - 1) 2^off_w to the scalar makes every window independent: digit_w =
// bits_w(s + C) - (2^(b_w - 1) - 1) is exactly the carry recoding of `recode` (a window's bits plus
// the carry v give v when v <= 2^(b-1), else v - 2^b with a carry out -- the same as
// (v + 2^(b-1) - 1) mod 2^b - (2^(b-1) - 1) and the add's own carry), and the overflow window is
// t's bits 254 and up, the add's carry out included (<= 4, never negative).  So each window is one
// funnel shift of two known words and a mask: no 256-bit shift per window and no per-window scalar
// bookkeeping (the generic loop issued more scalar than vector instructions).
template <uint32_t Q, uint32_t NHI>
struct FixedGeo {
  static constexpr uint32_t WMAIN = (MAIN_BITS - NHI) / Q;
  static constexpr uint32_t bits(uint32_t w) { return w < NHI ? Q + 1 : Q; }
  static constexpr uint32_t off(uint32_t w) { return w * Q + (w < NHI ? w : NHI); }
  struct Words {
    uint32_t v[8];
  };
  static constexpr Words bias() {
    Words c{};
    for (uint32_t w = 0; w < WMAIN; w++) {
      const uint64_t h = (1ull << (bits(w) - 1)) - 1ull;  // < 2^16, spans at most two words
      const uint32_t o = off(w), k = o / 32, sh = o % 32;
      const uint64_t lo = (uint64_t)c.v[k] + ((h << sh) & 0xffffffffull);
      c.v[k] = (uint32_t)lo;
      uint64_t carry = (lo >> 32) + ((h << sh) >> 32);
      for (uint32_t j = k + 1; j < 8 && carry; j++) {
        const uint64_t x = (uint64_t)c.v[j] + carry;
        c.v[j] = (uint32_t)x;
        carry = x >> 32;
      }
    }
    return c;
  }
};

// The recode's LDS histogram [Wr][nbc] into the bin totals colsum[w][bin] (global atomics), and
// the windows' totals (LDS words after the histogram, summed per wave when a wave's 64 bins lie in
// one window) into wtot[w] = colsum[nbins + w]: k_part_scatter takes a window's first slot from
// the totals of the windows below it.  colsum and wtot are zeroed again by k_fine_sort.
__device__ __forceinline__ void flush_hist(uint32_t* lds_hist, const MsmDims& d, uint32_t w0,
                                           uint32_t* __restrict__ colsum) {
  const uint32_t nh = d.Wr * d.nbc, lg = __builtin_ctz(d.nbc);
  uint32_t* wt = lds_hist + nh;
  for (uint32_t b = threadIdx.x; b < nh; b += RC_THREADS) {
    const uint32_t v = lds_hist[b];
    if (v) atomicAdd(&colsum[w0 * d.nbc + b], v);
    if (d.nbc >= 64) {
      const uint32_t t = wave_incl_scan(v);
      if ((threadIdx.x & 63) == 63 && t) atomicAdd(&wt[b >> lg], t);
    } else if (v) {
      atomicAdd(&wt[b >> lg], v);
    }
  }
  __syncthreads();
  if (threadIdx.x < d.Wr && wt[threadIdx.x]) atomicAdd(&colsum[d.nbins + w0 + threadIdx.x], wt[threadIdx.x]);
}

// Pass 0+1 (fused), blockIdx.y = MSM of the batch: scalars from scalar_sets.p[y], digits into its
// windows [y Wr, (y+1) Wr).  Carries only climb, so windows below the launch's range [d.w0, d.w0 +
// d.Wr) are recoded for their carries (the generic loop stops at the range's top); only the range
// is written and counted.  The generic form (`recode`) serves any geometry.
template <typename T>
__global__ void __launch_bounds__(RC_THREADS) k_recode_hist(BatchPtrs scalar_sets, MsmDims d,
                                                            T* __restrict__ digits, uint32_t* __restrict__ colsum) {
  extern __shared__ uint32_t lds_hist[];  // [Wr][nbc]
  const uint32_t* __restrict__ scalars = scalar_sets.p[blockIdx.y];
  const uint32_t lo = blockIdx.x * RC_SPAN, hi = min(d.n, lo + RC_SPAN);
  const uint32_t w0 = blockIdx.y * d.Wr;
  const uint32_t nh = d.Wr * d.nbc;
  [[maybe_unused]] const uint32_t pwg = blockIdx.y * gridDim.x + blockIdx.x;
  PROBE(0, pwg, 0);
  for (uint32_t b = threadIdx.x; b < nh + d.Wr; b += RC_THREADS) lds_hist[b] = 0;  // + the window totals
  __syncthreads();
  PROBE(0, pwg, 1);
  // (loading all of a lane's scalars before recoding any measured slower: 43 vs 37 us per
  // two-MSM 2^20 launch)
  for (uint32_t i = lo + threadIdx.x; i < hi; i += RC_THREADS) {
    uint32_t s[8];
    load_scalar(scalars, i, s);
    recode(s, d, [&](uint32_t wa, int32_t digit) {
      const uint32_t w = wa - d.w0;  // local window (wraps to >= Wr below the range)
      if (w >= d.Wr) return;
      uint32_t code = DigitCode<T>::ZERO;
      if (digit != 0) {
        const uint32_t mag = (uint32_t)(digit < 0 ? -digit : digit) - 1u;
        // half windows at the range's ends: a bucket outside the kept half is another share's
        const uint32_t hb = 1u << (win_bits(d, wa) - 2);
        if ((w == 0 && d.half_lo && mag < hb) || (w + 1 == d.Wr && d.half_hi && mag >= hb)) {
          digits[(size_t)(w0 + w) * d.n + i] = (T)code;
          return;
        }
        code = mag | (digit < 0 ? DigitCode<T>::SIGN : 0u);
        atomicAdd(&lds_hist[w * d.nbc + (mag >> win_fb(d, wa))], 1u);
      }
      digits[(size_t)(w0 + w) * d.n + i] = (T)code;
    });
  }
  __syncthreads();
  PROBE(0, pwg, 2);
  flush_hist(lds_hist, d, w0, colsum);
  PROBE(0, pwg, 7);
}

// The same with the geometry fixed at compile time (FixedGeo above) and 16-bit codes.  FULL: the
// launch covers every window (no range, no half windows), so nothing per window is uniform but
// the two fine-bit counts; else each window checks the range.  Row and histogram addresses advance
// by a stride per window kept in the range.
// (__launch_bounds__ with 8 waves per SIMD: two workgroups per CU need <= 80 SGPRs, which the
// unrolled windows' constants otherwise exceed -- one workgroup per CU took 37 against 31 us.)
template <uint32_t Q, uint32_t NHI, bool FULL>
__global__ void __launch_bounds__(RC_THREADS, 8) k_recode_fixed(BatchPtrs scalar_sets, MsmDims d,
                                                             uint16_t* __restrict__ digits,
                                                             uint32_t* __restrict__ colsum) {
  using G = FixedGeo<Q, NHI>;
  using DC = DigitCode<uint16_t>;
  static_assert(G::off(G::WMAIN) == MAIN_BITS, "main windows cover bits [0, 254)");
  constexpr typename G::Words C = G::bias();
  extern __shared__ uint32_t lds_hist[];  // [Wr][nbc]
  const uint32_t* __restrict__ scalars = scalar_sets.p[blockIdx.y];
  const uint32_t lo = blockIdx.x * RC_SPAN, hi = min(d.n, lo + RC_SPAN);
  const uint32_t w0 = blockIdx.y * d.Wr;
  const uint32_t nh = d.Wr * d.nbc;
  [[maybe_unused]] const uint32_t pwg = blockIdx.y * gridDim.x + blockIdx.x;
  PROBE(0, pwg, 0);
  for (uint32_t b = threadIdx.x; b < nh + d.Wr; b += RC_THREADS) lds_hist[b] = 0;  // + the window totals
  // fine bits of the wide (Q + 1) windows, the narrow (Q) ones and the overflow window (win_fb)
  const uint32_t fb_w = d.fb - (d.c - (NHI ? Q + 1 : Q));
  const uint32_t fb_n = d.fb > d.c - Q ? d.fb - (d.c - Q) : 0u;
  const uint32_t fb_o = d.fb > d.c - OVF_BITS ? d.fb - (d.c - OVF_BITS) : 0u;
  const uint32_t wlo = d.w0, whi = d.w0 + d.Wr;
  __syncthreads();
  PROBE(0, pwg, 1);
  // Each lane recodes two adjacent scalars: their loads are one 64-B run, and a window's two
  // codes go out as one 4-B store (when n is even, so that every row stays 4-B aligned).
  const bool pair_store = (d.n & 1u) == 0;
  for (uint32_t i = lo + 2 * threadIdx.x; i < hi; i += 2 * RC_THREADS) {
    const bool two = i + 1 < hi;
    uint32_t t0[8], t1[8], cy0 = 0, cy1 = 0;
    {
      uint32_t s0[8], s1[8];
      load_scalar(scalars, i, s0);
      if (two)
        load_scalar(scalars, i + 1, s1);
      else
#pragma unroll
        for (int k = 0; k < 8; k++) s1[k] = 0;
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const uint64_t x0 = (uint64_t)s0[k] + C.v[k] + cy0;
        const uint64_t x1 = (uint64_t)s1[k] + C.v[k] + cy1;
        t0[k] = (uint32_t)x0;
        t1[k] = (uint32_t)x1;
        cy0 = (uint32_t)(x0 >> 32);
        cy1 = (uint32_t)(x1 >> 32);
      }
    }
    uint16_t* row = digits + (size_t)w0 * d.n + i;
    uint32_t* h = lds_hist;
#pragma unroll
    for (uint32_t wa = 0; wa <= G::WMAIN; wa++) {
      if (!FULL && (wa < wlo || wa >= whi)) continue;
      int32_t dg[2];
      uint32_t fbits, hb;
      if (wa < G::WMAIN) {
        const uint32_t o = G::off(wa), b = G::bits(wa), k = o / 32, sh = o % 32;
        const uint32_t x0 = (sh + b <= 32 ? t0[k] >> sh : __builtin_amdgcn_alignbit(t0[k + 1], t0[k], sh)) & ((1u << b) - 1u);
        const uint32_t x1 = (sh + b <= 32 ? t1[k] >> sh : __builtin_amdgcn_alignbit(t1[k + 1], t1[k], sh)) & ((1u << b) - 1u);
        dg[0] = (int32_t)x0 - (int32_t)((1u << (b - 1)) - 1u);
        dg[1] = (int32_t)x1 - (int32_t)((1u << (b - 1)) - 1u);
        fbits = b == Q + 1 ? fb_w : fb_n;
        hb = 1u << (b - 2);
      } else {
        dg[0] = (int32_t)((t0[7] >> 30) | (cy0 << 2));
        dg[1] = (int32_t)((t1[7] >> 30) | (cy1 << 2));
        fbits = fb_o;
        hb = 1u << (OVF_BITS - 2);
      }
      uint32_t code[2];
#pragma unroll
      for (int q = 0; q < 2; q++) {
        const int32_t digit = dg[q];
        const uint32_t mag = (uint32_t)(digit < 0 ? -digit : digit) - 1u;
        bool live = digit != 0 && (q == 0 || two);
        if (!FULL) {
          // half windows at the range's ends: a bucket outside the kept half is another share's
          if (wa == wlo && d.half_lo) live = live && mag >= hb;
          if (wa + 1 == whi && d.half_hi) live = live && mag < hb;
        }
        // every lane adds (0 for a zero digit): no divergent branch around the LDS atomic
        atomicAdd(&h[live ? mag >> fbits : 0u], live ? 1u : 0u);
        code[q] = live ? mag | (digit < 0 ? DC::SIGN : 0u) : DC::ZERO;
      }
      if (pair_store && two) {
        *reinterpret_cast<uint32_t*>(row) = code[0] | code[1] << 16;
      } else {
        row[0] = (uint16_t)code[0];
        if (two) row[1] = (uint16_t)code[1];
      }
      row += d.n;
      h += d.nbc;
    }
  }
  __syncthreads();
  PROBE(0, pwg, 2);
  flush_hist(lds_hist, d, w0, colsum);
  PROBE(0, pwg, 7);
}

// k_fine_sort geometry
#ifndef MSM_FS_THREADS
#define MSM_FS_THREADS 512
#endif
// Bins staged in LDS: up to FS_CAP entries.  A bin averages ~4K entries, but the top window of
// scalars reduced mod r (< 0.58 * 2^253, as any prover's are) fills only 58% of its buckets, so
// its bins hold ~7K: 8,192 keeps them on the staged path (at 6,144 they took the unstaged one and
// were the kernel's stragglers, ~25 us each).
#ifndef MSM_FS_CAP
#define MSM_FS_CAP 8192
#endif
constexpr uint32_t FS_THREADS = MSM_FS_THREADS;
constexpr uint32_t FS_R = MSM_FS_CAP / FS_THREADS;
constexpr uint32_t FS_CAP = FS_THREADS * FS_R;  // (512 threads: -12% vs 256 at 6,144, measured)
constexpr uint32_t FS_MAXF = 2048;

// Pass 2: each (window, chunk) workgroup moves its digits into its own contiguous slice of every
// coarse bin.  The chunk is counting-sorted by bin inside LDS -- the LDS atomic that counts an
// entry also returns its rank inside its bin, so every entry is placed without a second atomic
// -- and each bin's slice is reserved with one global atomic on the bin's cursor (bin_cur, counted
// from zero; the slices' order inside a bin is immaterial: the bucket sums commute).  The
// staged chunk is then streamed out so that consecutive lanes write consecutive addresses of a
// slice (>= 64 entries per slice by construction of ch).  (Writing each entry straight from
// registers to its slice, with no LDS staging, measured 59 -> 153 us per two-MSM 2^20 launch; the
// same in k_fine_sort 96 -> 168 us.)
//
// Staging keeps 4 B per entry for 16-bit codes: code << PS_POS | position in the chunk (ch = 2^PS_POS),
// 64 KiB, so two workgroups share a CU; 32-bit codes (c > 16) stage (code, position) pairs.
constexpr uint32_t PS_POS = __builtin_ctz(PT_THREADS * PS_R);  // bits of a position in a chunk
template <typename T>
struct PartStage;
template <>
struct PartStage<uint16_t> {
  using V = uint32_t;
  static __device__ __forceinline__ V pack(uint32_t code, uint32_t li) { return code << PS_POS | li; }
  static __device__ __forceinline__ uint32_t code(V v) { return v >> PS_POS; }
  static __device__ __forceinline__ uint32_t pos(V v) { return v & ((1u << PS_POS) - 1u); }
};
template <>
struct PartStage<uint32_t> {
  using V = uint2;
  static __device__ __forceinline__ V pack(uint32_t code, uint32_t li) { return make_uint2(code, li); }
  static __device__ __forceinline__ uint32_t code(V v) { return v.x; }
  static __device__ __forceinline__ uint32_t pos(V v) { return v.y; }
};
static_assert(PT_THREADS * PS_R == (1u << PS_POS) && PS_POS <= 16, "PartStage<uint16_t> packs code and position in 32 bits");

template <typename T>
__global__ void __launch_bounds__(PT_THREADS) k_part_scatter(const T* __restrict__ digits, MsmDims d,
                                                             uint32_t* __restrict__ colsum,
                                                             uint32_t* __restrict__ bin_cur,
                                                             uint32_t* __restrict__ bin_base,
                                                             uint32_t* __restrict__ part_entry,
                                                             uint16_t* __restrict__ part_fine) {
  using S = PartStage<T>;
  __shared__ typename S::V st[PT_THREADS * PS_R];
  __shared__ uint32_t m_live;
  __shared__ uint32_t wpart[PT_THREADS / 64];
  // [nbc] count -> local start, [nbc] global slice start - local start, [nbc] bin start in window
  extern __shared__ uint4 dyn4[];
  uint32_t* lcnt = reinterpret_cast<uint32_t*>(dyn4);
  uint32_t* gdel = lcnt + d.nbc;
  uint32_t* bscan = gdel + d.nbc;
  const uint32_t w = blockIdx.y, ck = blockIdx.x;
  const uint32_t fbw = batch_win_fb(d, w);
  const uint32_t pbase = d.shared ? 0u : (w / d.Wr) * d.n;  // first point record of this window's MSM
  const T* dw = digits + (size_t)w * d.n;
  const uint32_t lo = ck * d.ch, hi = min(d.n, lo + d.ch);
  [[maybe_unused]] const uint32_t pwg = blockIdx.y * gridDim.x + blockIdx.x;
  PROBE(1, pwg, 0);
  // 16-bit codes carry their rank in the bin in their upper half (one register per digit: the
  // workgroup stays within 64 VGPRs, two per CU); 32-bit codes keep it apart
  constexpr bool PACK = sizeof(T) == 2;
  uint32_t code[PS_R], rank[PACK ? 1 : PS_R];
#pragma unroll
  for (uint32_t r = 0; r < PS_R; r++) {
    const uint32_t i = lo + r * PT_THREADS + threadIdx.x;
    code[r] = i < hi ? (uint32_t)dw[i] : DigitCode<T>::ZERO;
  }
  // Beside the digit loads: the window's bin totals (scanned below into the bins' starts inside
  // the window) and the sum of the lower windows' totals (the window's first slot) -- what a
  // separate one-workgroup scan kernel computed before (k_bin_scan, ~10 us per launch).
  // nbc <= 256 <= PT_THREADS (make_plan): one bin per thread.
  const bool bin_lane = threadIdx.x < d.nbc;
  const uint32_t tot_b = bin_lane ? colsum[w * d.nbc + threadIdx.x] : 0u;
  const uint32_t* wtot = colsum + d.nbins;
  uint32_t lower = 0;
  for (uint32_t v = threadIdx.x; v < w; v += PT_THREADS) lower += wtot[v];
  lower = wave_incl_scan(lower);
  if ((threadIdx.x & 63) == 63) wpart[threadIdx.x >> 6] = lower;
  if (bin_lane) {
    lcnt[threadIdx.x] = 0;
    bscan[threadIdx.x] = tot_b;
  }
  PROBE_WAIT_VM();
  PROBE(1, pwg, 1);
  __syncthreads();
#pragma unroll
  for (uint32_t r = 0; r < PS_R; r++) {
    if (code[r] != DigitCode<T>::ZERO) {
      const uint32_t rk = atomicAdd(&lcnt[(code[r] & DigitCode<T>::MAG) >> fbw], 1u);
      if constexpr (PACK)
        code[r] |= rk << 16;
      else
        rank[r] = rk;
    }
  }
  lds_excl_scan_wave0(bscan, d.nbc);
  __syncthreads();
  PROBE(1, pwg, 2);
  // each bin's slice is reserved with one global atomic on the bin's cursor (zero-based; its
  // latency overlaps the local scan)
  const uint32_t cb = bin_lane ? lcnt[threadIdx.x] : 0u;
  const uint32_t g = cb ? atomicAdd(&bin_cur[w * d.nbc + threadIdx.x], cb) : 0u;
  if (threadIdx.x == d.nbc - 1) m_live = cb;
  uint32_t wbase = 0;
#pragma unroll
  for (uint32_t k = 0; k < PT_THREADS / 64; k++) wbase += wpart[k];
  __syncthreads();
  PROBE(1, pwg, 3);
  lds_excl_scan_wave0(lcnt, d.nbc);
  __syncthreads();
  PROBE(1, pwg, 4);
  if (bin_lane) {
    const uint32_t start = wbase + bscan[threadIdx.x];  // the bin's first slot in the sorted order
    gdel[threadIdx.x] = start + g - lcnt[threadIdx.x];  // entry j of bin b goes to j + gdel[b]
    if (ck == 0) {
      bin_base[w * d.nbc + threadIdx.x] = start;
      if (w + 1 == d.W && threadIdx.x == d.nbc - 1) bin_base[d.nbins] = start + tot_b;
    }
  }
#pragma unroll
  for (uint32_t r = 0; r < PS_R; r++) {
    const uint32_t cd = PACK ? code[r] & 0xffffu : code[r];
    if (cd != DigitCode<T>::ZERO)
      st[lcnt[(cd & DigitCode<T>::MAG) >> fbw] + (PACK ? code[r] >> 16 : rank[PACK ? 0 : r])] =
          S::pack(cd, r * PT_THREADS + threadIdx.x);
  }
  __syncthreads();
  PROBE(1, pwg, 5);
  const uint32_t m = lcnt[d.nbc - 1] + m_live;  // live digits of the chunk
  const uint32_t fmask = (1u << fbw) - 1u;
  for (uint32_t j = threadIdx.x; j < m; j += PT_THREADS) {
    const typename S::V v = st[j];
    const uint32_t cd = S::code(v);
    const uint32_t b = cd & DigitCode<T>::MAG;
    const uint32_t fine = b & fmask;
    const uint32_t ent = ((pbase + lo + S::pos(v)) << 1) | (cd >> DigitCode<T>::SHIFT);
    const uint32_t dst = j + gdel[b >> fbw];
    // packed: the fine key in the low d.fb bits (a narrower window's fbw <= d.fb of them used)
    part_entry[dst] = d.packed ? (ent << d.fb) | fine : ent;
    if (!d.packed) part_fine[dst] = (uint16_t)fine;
  }
  PROBE(1, pwg, 6);
  PROBE(1, pwg, 7);
}

// Pass 3: one workgroup per coarse bin, counting sort by fine bucket (<= FS_MAXF per bin).  A bin
// of at most FS_CAP entries is sorted inside LDS and streamed out coalesced.  Besides the sorted
// entry list it writes the bucket boundaries the accumulation walks: bucket_start[key] (global
// position of bucket `key`'s first entry; bucket_start[W*B] = bucket_start[W*B+1] = total) and
// run_key[r] = the bucket holding position r*K (the first entry of accumulation run r).  A window
// narrower than the widest has fewer buckets than B (win_fb): the bins' workgroups also set its
// keys past them, each a share, to the window's end.
//
// A bigger bin (skewed scalars: one giant bucket, or few distinct digits) is sorted by its own
// workgroup in register tiles: a counting pass that collapses runs of equal keys per lane before
// touching LDS (a bin that is one giant bucket costs one atomic per lane, not per entry), then a
// placement pass in which the lanes of a wave holding the same key find each other by ballots over
// the key's bits and their leader reserves all their slots with one atomic -- so equal keys never
// serialise on one LDS address, and they are written coalesced.  (This replaced k_big_place, a
// tile-parallel kernel of its own that cost a launch, ~5 us, on every MSM for the skewed inputs'
// sake.)

// One coarse-binned entry: its fine key (bucket within the bin) and the sorted-list entry
// (idx << 1 | sign), from the packed word or the two arrays (MsmDims::packed).
__device__ __forceinline__ void part_load(const uint32_t* __restrict__ pe, const uint16_t* __restrict__ pf,
                                          const MsmDims& d, uint32_t i, uint32_t& fine, uint32_t& entry) {
  const uint32_t v = pe[i];
  if (d.packed) {
    fine = v & ((1u << d.fb) - 1u);
    entry = v >> d.fb;
  } else {
    fine = pf[i];
    entry = v;
  }
}

// floor(x / D) for a runtime, wave-uniform D, given inv = 1.0 / D: (x + 0.5) / D is at least
// 0.5 / D away from an integer, and the two roundings (inv, the product) err by < 2^-20 / D for any
// 32-bit x, so the truncation is exact.  Three VALU against the ~14 of an unsigned division.
__device__ __forceinline__ uint32_t div_by_inv(uint32_t x, double inv) {
  return (uint32_t)(((double)x + 0.5) * inv);
}

__device__ __forceinline__ void count_runs(uint32_t* cnt, uint32_t& last, uint32_t& run, uint32_t key) {
  if (key == last) {
    run++;
  } else {
    if (run) atomicAdd(&cnt[last], run);
    last = key;
    run = 1;
  }
}

// Lanes of the wave whose `key` (fbits bits) equals this lane's, among the lanes in `live`.
__device__ __forceinline__ uint64_t key_peers(uint32_t key, uint32_t fbits, uint64_t live) {
  uint64_t peers = live;
  for (uint32_t b = 0; b < fbits; b++) {
    const uint64_t set = __ballot((key >> b) & 1u);
    peers &= ((key >> b) & 1u) ? set : ~set;
  }
  return peers;
}

// MSM_FS_MINW: minimum waves per SIMD asked of the compiler.  8 = four workgroups per CU (<= 64
// VGPRs, a few spilled in the unstaged path): 57 against 63 us per two-MSM 2^20 launch at 76 VGPRs
// (three workgroups per CU).
#ifndef MSM_FS_MINW
#define MSM_FS_MINW 8
#endif
#if MSM_FS_MINW > 0
#define FS_BOUNDS __launch_bounds__(FS_THREADS, MSM_FS_MINW)
#else
#define FS_BOUNDS __launch_bounds__(FS_THREADS)
#endif
extern "C" __global__ void FS_BOUNDS k_fine_sort(const uint32_t* __restrict__ part_entry,
                                                                     const uint16_t* __restrict__ part_fine,
                                                                     const uint32_t* __restrict__ bin_base, MsmDims d,
                                                                     uint32_t K, uint32_t* __restrict__ sorted_entry,
                                                                     uint32_t* __restrict__ bucket_start,
                                                                     uint32_t* __restrict__ run_key,
                                                                     uint32_t* __restrict__ colsum,
                                                                     uint32_t* __restrict__ bin_cur) {
  __shared__ __attribute__((aligned(16))) uint32_t cnt[FS_MAXF];
  __shared__ uint32_t st_entry[FS_CAP];
  const uint32_t bin = blockIdx.x;
  PROBE(2, bin, 0);
  const uint32_t w = bin / d.nbc, cb = bin % d.nbc;
  const uint32_t fbw = batch_win_fb(d, w);
  const uint32_t nf = 1u << fbw;
  const uint32_t base = bin_base[bin];
  const uint32_t m = bin_base[bin + 1] - base;
  const uint32_t key0 = w * d.B + (cb << fbw);
  for (uint32_t f = threadIdx.x; f < nf; f += FS_THREADS) cnt[f] = 0;
  if (threadIdx.x == 0) {
    // the bin's total, cursor and window total are consumed (k_part_scatter): zero for the next MSM
    colsum[bin] = 0;
    bin_cur[bin] = 0;
    if (cb == 0) colsum[d.nbins + w] = 0;
  }
  if (bin + 1 == gridDim.x && threadIdx.x == 0) {
    bucket_start[d.W * d.B] = base + m;
    bucket_start[d.W * d.B + 1] = base + m;
  }
  {
    // a narrower window's keys past its buckets: empty, all at the window's end
    const uint32_t k1 = d.nbc << fbw;
    if (k1 < d.B) {
      const uint32_t span = (d.B - k1) / d.nbc, wend = bin_base[(w + 1) * d.nbc];
      for (uint32_t f = threadIdx.x; f < span; f += FS_THREADS) bucket_start[w * d.B + k1 + cb * span + f] = wend;
    }
  }
  __syncthreads();
  PROBE(2, bin, 1);
  const bool staged = m <= FS_CAP;
  const uint32_t fmask = (1u << d.fb) - 1u;  // the packed word's fine field (fbw <= d.fb bits used)
  // fk: fine key (< 2^11) of a staged entry, later | its rank in its bucket << 16 (< FS_CAP)
  uint32_t fk[FS_R], en[FS_R];
  if (staged) {
    // every load issued before any is used; the packed/unpacked choice is uniform
    if (d.packed) {
#pragma unroll
      for (uint32_t r = 0; r < FS_R; r++) {
        const uint32_t e = r * FS_THREADS + threadIdx.x;
        en[r] = e < m ? part_entry[base + e] : 0u;
      }
#pragma unroll
      for (uint32_t r = 0; r < FS_R; r++) {
        const uint32_t e = r * FS_THREADS + threadIdx.x;
        fk[r] = e < m ? en[r] & fmask : 0xffffu;
        en[r] >>= d.fb;
      }
      PROBE_WAIT_VM();
      PROBE(2, bin, 2);
    } else {
#pragma unroll
      for (uint32_t r = 0; r < FS_R; r++) {
        const uint32_t e = r * FS_THREADS + threadIdx.x;
        fk[r] = e < m ? part_fine[base + e] : 0xffffu;
        en[r] = e < m ? part_entry[base + e] : 0u;
      }
    }
#pragma unroll
    for (uint32_t r = 0; r < FS_R; r++)
      if (fk[r] != 0xffffu) fk[r] |= atomicAdd(&cnt[fk[r]], 1u) << 16;
  } else {
    // register tiles of FS_R keys per lane (independent loads in flight); runs of equal keys
    // are collapsed before the LDS atomic
    uint32_t last = 0, run = 0;
    for (uint32_t t0 = 0; t0 < m; t0 += FS_CAP) {
#pragma unroll
      for (uint32_t r = 0; r < FS_R; r++) {
        const uint32_t e = t0 + r * FS_THREADS + threadIdx.x;
        uint32_t en_unused;
        fk[r] = 0xffffu;
        if (e < m) part_load(part_entry, part_fine, d, base + e, fk[r], en_unused);
      }
#pragma unroll
      for (uint32_t r = 0; r < FS_R; r++)
        if (fk[r] != 0xffffu) count_runs(cnt, last, run, fk[r]);
    }
    if (run) atomicAdd(&cnt[last], run);
  }
  __syncthreads();
  PROBE(2, bin, 3);
  // per-bucket counts -> exclusive offsets; boundaries and run starts go out with them (a bucket
  // ends where the next one starts)
  lds_excl_scan_wave0(cnt, nf);
  const double kinv = 1.0 / (double)K;  // div_by_inv: the bucket's first run, ceil(gs / K)
  __syncthreads();
  PROBE(2, bin, 4);
#pragma unroll
  for (uint32_t q = 0; q < FS_MAXF / FS_THREADS; q++) {
    const uint32_t f = q * FS_THREADS + threadIdx.x;
    if (f < nf) {
      const uint32_t gs = base + cnt[f];
      const uint32_t ge = base + (f + 1 < nf ? cnt[f + 1] : m);
      bucket_start[key0 + f] = gs;
      const uint32_t r0 = div_by_inv(gs + K - 1, kinv);
      for (uint32_t r = r0; r * K < ge; r++) run_key[r] = key0 + f;
    }
  }
  __syncthreads();
  PROBE(2, bin, 5);
  if (!staged) {
    // placement: a wave's lanes with equal keys take consecutive slots of their bucket, reserved
    // by the lowest of them with one LDS atomic
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t below = (1ull << lane) - 1ull;
    for (uint32_t t0 = 0; t0 < m; t0 += FS_CAP) {
#pragma unroll
      for (uint32_t r = 0; r < FS_R; r++) {
        const uint32_t e = t0 + r * FS_THREADS + threadIdx.x;
        fk[r] = 0u;
        en[r] = 0u;
        if (e < m) part_load(part_entry, part_fine, d, base + e, fk[r], en[r]);
      }
#pragma unroll
      for (uint32_t r = 0; r < FS_R; r++) {
        const bool live = t0 + r * FS_THREADS + threadIdx.x < m;
        const uint64_t peers = key_peers(fk[r], fbw, __ballot(live));
        const uint32_t leader = (uint32_t)__builtin_ctzll(peers | (1ull << 63));
        uint32_t slot = 0;
        if (live && lane == leader) slot = atomicAdd(&cnt[fk[r]], (uint32_t)__popcll(peers));
        slot = (uint32_t)__shfl((int)slot, (int)leader, 64);
        if (live) sorted_entry[base + slot + (uint32_t)__popcll(peers & below)] = en[r];
      }
    }
    PROBE(2, bin, 6);
    PROBE(2, bin, 7);
    return;
  }
#pragma unroll
  for (uint32_t r = 0; r < FS_R; r++)
    if (fk[r] != 0xffffu) st_entry[cnt[fk[r] & 0xffffu] + (fk[r] >> 16)] = en[r];
  __syncthreads();
  PROBE(2, bin, 6);
  for (uint32_t j = threadIdx.x; j < m; j += FS_THREADS) sorted_entry[base + j] = st_entry[j];
  PROBE(2, bin, 7);
}

#ifdef MSM_GAP_KERNEL
// tuning builds: a no-op launch between the sort and the accumulation
extern "C" __global__ void k_gap(uint32_t* __restrict__ p) {
  if (p == nullptr && threadIdx.x == 1234567) p[0] = 0;
}
#endif

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

__device__ __forceinline__ void store_fe_lds(uint32_t* dst, const fe& a) {
#pragma unroll
  for (int k = 0; k < NL; k++) dst[k] = a.v[k];
}
__device__ __forceinline__ fe load_fe_lds(const uint32_t* src) {
  fe a;
#pragma unroll
  for (int k = 0; k < NL; k++) a.v[k] = src[k];
  return a;
}
__device__ __forceinline__ void store_pt_lds(uint32_t* dst, const xyzt& p) {
#pragma unroll
  for (int k = 0; k < NL; k++) {
    dst[k] = p.X.v[k];
    dst[NL + k] = p.Y.v[k];
    dst[2 * NL + k] = p.T.v[k];
    dst[3 * NL + k] = p.Z.v[k];
  }
}
__device__ __forceinline__ xyzt load_pt_lds(const uint32_t* src) {
  xyzt p;
#pragma unroll
  for (int k = 0; k < NL; k++) {
    p.X.v[k] = src[k];
    p.Y.v[k] = src[NL + k];
    p.T.v[k] = src[2 * NL + k];
    p.Z.v[k] = src[3 * NL + k];
  }
  return p;
}

// First bucket key k > cur whose end bucket_start[k + 1] lies past pos, given that bucket cur is
// empty (bucket_start[cur + 1] == pos).  bucket_start is non-decreasing and ends with the total
// (> pos), so an exponential search then a binary search find it in O(log gap) loads: a window
// narrower than the bucket table, or a stretch of empty windows (small or structured scalars),
// would otherwise cost one dependent load per empty bucket.
__device__ __forceinline__ uint32_t next_nonempty(const uint32_t* __restrict__ bucket_start, uint32_t cur, uint32_t pos,
                                               uint32_t nkeys) {
  uint32_t lo = cur, step = 1;  // bucket lo is empty
  uint32_t hi = cur + 1;        // bucket nkeys - 1 ends at the total (> pos): the search stops there
  while (bucket_start[hi + 1] == pos) {
    lo = hi;
    step <<= 1;
    hi = min(cur + step, nkeys - 1);
  }
  // bucket lo empty, bucket hi ends past pos: the answer is in (lo, hi]
  while (hi - lo > 1) {
    const uint32_t mid = lo + (hi - lo) / 2;
    if (bucket_start[mid + 1] == pos) lo = mid;
    else hi = mid;
  }
  return hi;
}

// Bucket accumulation over the sorted list.  Lane = run of K consecutive entries (perfect load
// balance whatever the bucket sizes).  Inside a run, whole buckets are written straight to the
// bucket table; bucket boundaries come from bucket_start (one load per bucket, issued a bucket
// ahead), the run's first bucket from run_key.
//
// A bucket cut by run boundaries is joined without a second pass over HBM.  Every run's leading
// piece (head: the entries of a bucket begun in an earlier run) is staged in LDS, flagged
// "pass" when the whole run lies inside that bucket and the bucket continues.  After one barrier
// the run where the bucket begins adds its trailing piece (tail) to the head of the next run.
// A workgroup with a pass-through run (skewed scalars: a bucket holding several runs) instead
// stages its heads and tails in HBM and leaves the joins to k_chain_join, which collapses the
// chains with a logarithmic segmented scan; that keeps this kernel's register budget (and
// occupancy) set by the main loop.
//
// A chain reaching the end of workgroup g continues in workgroup g+1's lane-0 chain ("lead"):
// the tail owner stores its part in the bucket table and cross_key[g] names the bucket;
// k_bucket_reduce_1 adds lead_val[g+1] to it, after k_lead_scan has chained leads that
// themselves run through whole workgroups.
#ifndef MSM_ACC_VEC
#define MSM_ACC_VEC 1
#endif
// Progress-ordered wave priority.  A SIMD's VALU issue goes by wave priority, then age, so of the
// four equal runs sharing a SIMD the oldest finished first and the youngest last (an 8-GPU share,
// one round of workgroups: 186 / 294 / 407 / 510 us by dispatch order, tools/phase_probe.py), and
// the last ~30% of the launch ran with one to three waves per SIMD.  Each wave therefore lowers
// its priority as it passes each quarter of its run (3, 2, 1, 0): a wave ahead of its partners
// yields to them, and the four finish within the last quarter's age order (share: 371 / 400 /
// 428 / 453 us).  A lone 2^20 MSM's accumulation 744 -> 717 us (latency 1.074 -> 1.045 ms);
// pipelined launches and the 8-GPU shares within noise (sessions t15, t16).
#ifndef MSM_ACC_PRIO
#define MSM_ACC_PRIO 1
#endif
constexpr uint32_t ACC_THREADS = 256;
// One workgroup-sized tile of the accumulation: runs [wg ACC_THREADS, (wg + 1) ACC_THREADS).
__device__ __forceinline__ void acc_tile(uint32_t wg, uint32_t (*sh_head)[PT_WORDS], uint32_t* sh_hkey,
                                         const uint32_t* __restrict__ pts,
                                         const uint32_t* __restrict__ sorted_entry,
                                         const uint32_t* __restrict__ bucket_start,
                                         const uint32_t* __restrict__ run_key,
                                         const uint32_t* __restrict__ total_ptr, uint32_t K,
                                         uint32_t nkeys,
                                         uint32_t* __restrict__ buckets,
                                         uint32_t* __restrict__ lead_val,
                                         uint32_t* __restrict__ lead_open,
                                         uint32_t* __restrict__ cross_key,
                                         uint32_t* __restrict__ skew_list,
                                         uint32_t* __restrict__ g_head,
                                         uint32_t* __restrict__ g_hkey,
                                         uint32_t* __restrict__ g_tkey) {
  const uint32_t M = *total_ptr;
  const uint32_t lt = threadIdx.x;
  const uint32_t t = wg * ACC_THREADS + lt;
  const uint32_t s = t * K;
  sh_hkey[lt] = KEY_INVALID;
  xyzt acc = pt_identity();
  uint32_t cur = KEY_INVALID;
  bool has_tail = false, cont = false;
  if (s < M) {
    const uint32_t e = min(s + K, M);
    cur = run_key[t];
    const bool started_before = bucket_start[cur] < s;
    uint32_t bend = bucket_start[cur + 1];   // end of bucket `cur`
    uint32_t bnext = bucket_start[cur + 2];  // end of the bucket after it (prefetched)
    bool seg_first = true;
#if MSM_ACC_VEC
    // sorted entries four at a time (one 16-B load per lane every fourth step: the lanes walk
    // runs K entries apart, so scalar loads cost one cache-line request per lane per step)
    const bool vec = (K & 3u) == 0;  // run starts (t K) are then 16-B aligned
    uint4 eb = make_uint4(0u, 0u, 0u, 0u);
#endif
#if MSM_ACC_PRIO
    // (levels at 70 / 84 / 95% of the run instead, so that the age order left inside the last
    // level decides only its last 5%: pipelined 2^20 +7%, session t16)
    const uint32_t q1 = K >> 2, q2 = K >> 1, q3 = q1 + q2;
#endif
    for (uint32_t pos = s; pos < e; pos++) {
#if MSM_ACC_PRIO
      {
        const uint32_t q = __builtin_amdgcn_readfirstlane(pos - s);  // uniform: every run is K long
        if (q == q1) __builtin_amdgcn_s_setprio(2);
        else if (q == q2) __builtin_amdgcn_s_setprio(1);
        else if (q == q3) __builtin_amdgcn_s_setprio(0);
      }
#endif
#if MSM_ACC_VEC
      const uint32_t jq = (pos - s) & 3u;  // uniform across the lanes still in the loop
      if (vec && jq == 0) eb = *reinterpret_cast<const uint4*>(sorted_entry + pos);
#endif
      if (pos == bend) {
        if (seg_first && started_before) {
          store_pt_lds(sh_head[lt], acc);
          sh_hkey[lt] = cur;
        } else {
          store_pt(buckets + (size_t)cur * PT_WORDS, acc);
        }
        // advance to the next non-empty bucket (a run of empty ones is skipped by galloping)
        cur++;
        bend = bnext;
        bnext = bucket_start[cur + 2];
        if (bend == pos) {
          cur = next_nonempty(bucket_start, cur, pos, nkeys);
          bend = bucket_start[cur + 1];
          bnext = bucket_start[cur + 2];
        }
        acc = pt_identity();
        seg_first = false;
      }
#if MSM_ACC_VEC
      const uint32_t ent = !vec ? sorted_entry[pos] : jq == 0 ? eb.x : jq == 1 ? eb.y : jq == 2 ? eb.z : eb.w;
#else
      const uint32_t ent = sorted_entry[pos];
#endif
      const pre q = load_pre_signed(pts, ent);
      acc = pt_madd(acc, q);
    }
    cont = bend > e;  // bucket `cur` continues into the next run
    if (seg_first && started_before) {  // the whole run belongs to a bucket begun earlier
      store_pt_lds(sh_head[lt], acc);
      sh_hkey[lt] = cur | (cont ? KEY_PASS : 0u);
    } else if (cont) {
      has_tail = true;  // acc = tail piece of bucket `cur`
    } else {
      store_pt(buckets + (size_t)cur * PT_WORDS, acc);
    }
  }
  // the last live run of the workgroup says whether a bucket leaves the workgroup
  const uint32_t nruns = (M + K - 1) / K;
  const uint32_t last = min(ACC_THREADS, nruns - min(nruns, wg * ACC_THREADS)) - 1;
  if (lt == last) cross_key[wg] = cont ? cur : KEY_INVALID;
  __syncthreads();
  // Chains of heads: a run whose head is "pass" continues into the next run.  Runs of three or
  // more pass heads in a row (buckets of ~200+ entries: skewed scalars), and a lead chain that
  // leaves the workgroup, are deferred to k_chain_join's logarithmic scan; otherwise every chain
  // has at most two pass heads and is joined right here with at most three adds.  (The top
  // window of canonical scalars holds ~110 entries per bucket, so two-pass chains are common.)
  const uint32_t hk = sh_hkey[lt];
  auto is_pass = [&](uint32_t r) {
    const uint32_t k = sh_hkey[r];
    return k != KEY_INVALID && (k & KEY_PASS) != 0;
  };
  const bool my_pass = hk != KEY_INVALID && (hk & KEY_PASS);
  const bool nxt_pass = lt < last && is_pass(lt + 1);
  const bool nxt2_pass = lt + 1 < last && is_pass(lt + 2);
  if (__syncthreads_or((my_pass && nxt_pass && nxt2_pass) ||
                       (lt == 0 && my_pass && (last == 0 || (nxt_pass && last == 1))))) {
    // skewed workgroup: stage heads and tail pieces for k_chain_join
    if (s < M) {
      g_hkey[t] = hk;
      if (hk != KEY_INVALID) store_pt(g_head + (size_t)t * PT_WORDS, load_pt_lds(sh_head[lt]));
      g_tkey[t] = has_tail ? cur : KEY_INVALID;
      if (has_tail) store_pt(buckets + (size_t)cur * PT_WORDS, acc);
    }
    if (lt == 0) skew_list[1 + atomicAdd(&skew_list[0], 1u)] = wg;
    return;
  }
  // Lane 0's head is the end of the previous workgroup's crossing bucket: the workgroup's lead.
  // If it is pass-through (a bucket spanning run 0 whole), the bucket ends in run 1 or 2 (not
  // past the workgroup here), and lane 0 joins those heads into the lead.
  const bool lead_join = lt == 0 && my_pass;
  if (lt == 0) {
    lead_open[wg] = 0u;
    if (s < M && hk != KEY_INVALID && !lead_join)
      store_pt(lead_val + (size_t)wg * PT_WORDS, load_pt_lds(sh_head[0]));
  }
  if (has_tail || lead_join) {
    // a tail's bucket continues in run lt+1 (and lt+2, lt+3 while those are pass-through), unless
    // it leaves the workgroup: then k_bucket_reduce_1 adds the next workgroup's lead
    // (cross_key).  (Straight-line adds: the same in a loop costs ~50 more VGPRs and occupancy.)
    const uint32_t nwalk =
        lead_join ? 1u + (nxt_pass ? 1u : 0u)
                  : (lt < last ? 1u + ((nxt_pass && lt + 1 < last) ? 1u + ((nxt2_pass && lt + 2 < last) ? 1u : 0u) : 0u)
                               : 0u);
    if (lead_join) acc = load_pt_lds(sh_head[0]);
    if (nwalk) acc = pt_add(acc, load_pt_lds(sh_head[lt + 1]));
    if (nwalk > 1) acc = pt_add(acc, load_pt_lds(sh_head[lt + 2]));
    if (nwalk > 2) acc = pt_add(acc, load_pt_lds(sh_head[lt + 3]));
    store_pt(lead_join ? lead_val + (size_t)wg * PT_WORDS : buckets + (size_t)cur * PT_WORDS, acc);
  }
}

// The kernel: one tile per workgroup.  (A persistent grid of 2-3 workgroups per CU striding over
// the tiles, to leave CU room for the other launch's kernels, measured no faster: DESIGN.md §4.1.)
extern "C" __global__ void __launch_bounds__(ACC_THREADS) k_accumulate(const uint32_t* __restrict__ pts,
                                         const uint32_t* __restrict__ sorted_entry,
                                         const uint32_t* __restrict__ bucket_start,
                                         const uint32_t* __restrict__ run_key,
                                         const uint32_t* __restrict__ total_ptr, uint32_t K,
                                         uint32_t nkeys,
                                         uint32_t* __restrict__ buckets,
                                         uint32_t* __restrict__ lead_val,
                                         uint32_t* __restrict__ lead_open,
                                         uint32_t* __restrict__ cross_key,
                                         uint32_t* __restrict__ skew_list,
                                         uint32_t* __restrict__ g_head,
                                         uint32_t* __restrict__ g_hkey,
                                         uint32_t* __restrict__ g_tkey) {
  __shared__ uint32_t sh_head[ACC_THREADS][PT_WORDS];
  __shared__ uint32_t sh_hkey[ACC_THREADS];
  PROBE(3, blockIdx.x, 0);
#if MSM_ACC_PRIO
  __builtin_amdgcn_s_setprio(3);
#endif
  acc_tile(blockIdx.x, sh_head, sh_hkey, pts, sorted_entry, bucket_start, run_key, total_ptr, K, nkeys, buckets,
           lead_val, lead_open, cross_key, skew_list, g_head, g_hkey, g_tkey);
  PROBE(3, blockIdx.x, 7);
}

// Joins for workgroups that k_accumulate found to hold a pass-through run (skewed scalars).
// Segmented suffix scan over the workgroup's heads by pointer jumping: after it, head r holds
// h_r + h_{r+1} + ... to the end of r's chain (or the workgroup's end), and its pass bit says
// whether the chain leaves the workgroup; log2(256) steps of one point add.  Then every tail
// owner adds the chain that follows it, and lane 0 publishes the workgroup's lead.
constexpr uint32_t CJ_GRID = 256;  // k_chain_join workgroups (they loop over the skewed list)
extern "C" __global__ void __launch_bounds__(ACC_THREADS) k_chain_join(const uint32_t* __restrict__ skew_list,
                                         const uint32_t* __restrict__ total_ptr,
                                         uint32_t K,
                                         const uint32_t* __restrict__ g_head,
                                         const uint32_t* __restrict__ g_hkey,
                                         const uint32_t* __restrict__ g_tkey,
                                         uint32_t* __restrict__ buckets,
                                         uint32_t* __restrict__ lead_val,
                                         uint32_t* __restrict__ lead_open,
                                         uint32_t* __restrict__ lead_flag) {
  const uint32_t nskew = skew_list[0];
  if (blockIdx.x >= nskew) return;
  const uint32_t M = *total_ptr;
  const uint32_t nruns = (M + K - 1) / K;
  __shared__ uint32_t sh_head[ACC_THREADS][PT_WORDS];
  __shared__ uint32_t sh_hkey[ACC_THREADS];
  const uint32_t lt = threadIdx.x;
  for (uint32_t li = blockIdx.x; li < nskew; li += gridDim.x) {
  const uint32_t wg = skew_list[1 + li];
  const uint32_t t = wg * ACC_THREADS + lt;
  const bool live = t < nruns;
  const uint32_t hk = live ? g_hkey[t] : KEY_INVALID;
  sh_hkey[lt] = hk;
  xyzt v = pt_identity();
  if (hk != KEY_INVALID) {
    v = load_pt(g_head + (size_t)t * PT_WORDS);
    store_pt_lds(sh_head[lt], v);
  }
  bool open = hk != KEY_INVALID && (hk & KEY_PASS);
  __syncthreads();
  for (uint32_t d = 1; d < ACC_THREADS; d <<= 1) {
    const bool take = open && lt + d < ACC_THREADS;
    xyzt nv;
    bool nopen = false;
    if (take) {
      nv = load_pt_lds(sh_head[lt + d]);
      nopen = (sh_hkey[lt + d] & KEY_PASS) != 0;
    }
    __syncthreads();
    if (take) {
      v = pt_add(v, nv);
      open = nopen;
      store_pt_lds(sh_head[lt], v);
      sh_hkey[lt] = (sh_hkey[lt] & ~KEY_PASS) | (open ? KEY_PASS : 0u);
    }
    __syncthreads();
  }
  if (lt == 0) {
    const uint32_t h0 = sh_hkey[0];
    const bool has_head = h0 != KEY_INVALID;
    const bool lopen = has_head && (h0 & KEY_PASS);
    if (has_head) store_pt(lead_val + (size_t)wg * PT_WORDS, load_pt_lds(sh_head[0]));
    lead_open[wg] = lopen ? 1u : 0u;
    if (lopen) atomicOr(lead_flag, 1u);
  }
  const uint32_t tk = live ? g_tkey[t] : KEY_INVALID;
  if (tk != KEY_INVALID) {
    xyzt acc = load_pt(buckets + (size_t)tk * PT_WORDS);
    if (lt + 1 < ACC_THREADS) acc = pt_add(acc, load_pt_lds(sh_head[lt + 1]));
    store_pt(buckets + (size_t)tk * PT_WORDS, acc);
  }
  __syncthreads();  // LDS reused by the next listed workgroup
  }
}

// Chains leads that run through whole workgroups (a bucket spanning three or more workgroups):
// segmented suffix scan lead_val[g] <- lead_val[g] + lead_val[g+1] + ... while lead_open.  One
// workgroup walks the leads from the end in tiles of LS_THREADS; a no-op unless k_accumulate saw
// an open lead.
constexpr uint32_t LS_THREADS = 512;
extern "C" __global__ void __launch_bounds__(LS_THREADS) k_lead_scan(uint32_t* __restrict__ lead_val,
                                                                     const uint32_t* __restrict__ lead_open,
                                                                     const uint32_t* __restrict__ lead_flag,
                                                                     const uint32_t* __restrict__ total_ptr,
                                                                     uint32_t K) {
  if (*lead_flag == 0) return;
  __shared__ uint32_t sv[LS_THREADS][PT_WORDS];
  __shared__ uint32_t so[LS_THREADS];
  const uint32_t M = *total_ptr;
  const uint32_t nruns = (M + K - 1) / K;
  const uint32_t nwg = (nruns + ACC_THREADS - 1) / ACC_THREADS;
  const uint32_t i = threadIdx.x;
  const uint32_t ntiles = (nwg + LS_THREADS - 1) / LS_THREADS;
  for (int tile = (int)ntiles - 1; tile >= 0; tile--) {
    const uint32_t g = (uint32_t)tile * LS_THREADS + i;
    // every lead an open lead can reach is valid (an open chain enters the next workgroup's
    // lane 0); other slots may hold stale data and are never absorbed
    bool open = g < nwg && lead_open[g] != 0;
    xyzt v = g < nwg ? load_pt(lead_val + (size_t)g * PT_WORDS) : pt_identity();
    store_pt_lds(sv[i], v);
    so[i] = open ? 1u : 0u;
    __syncthreads();
    for (uint32_t d = 1; d < LS_THREADS; d <<= 1) {
      const bool take = open && i + d < LS_THREADS && g + d < nwg;
      xyzt nv;
      bool nopen = false;
      if (take) {
        nv = load_pt_lds(sv[i + d]);
        nopen = so[i + d] != 0;
      }
      __syncthreads();
      if (take) {
        v = pt_add(v, nv);
        open = nopen;
        store_pt_lds(sv[i], v);
        so[i] = open ? 1u : 0u;
      }
      __syncthreads();
    }
    // still open at the tile's end: absorb the (final) value of the next tile's first lead
    const uint32_t gn = (uint32_t)(tile + 1) * LS_THREADS;
    if (open && gn < nwg) v = pt_add(v, load_pt(lead_val + (size_t)gn * PT_WORDS));
    __syncthreads();
    if (g < nwg && lead_open[g] != 0) store_pt(lead_val + (size_t)g * PT_WORDS, v);
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------------
// bucket reduction:  G_w = sum_{b} (b+1) B_{w,b}
//   chunk c (L buckets): U_c = sum_i (i+1) B_{cL+i}, T_c = sum_i B_{cL+i}   (running sums)
//   G_w = sum_c U_c + L * sum_c c T_c = R_{w,V} + sum_k L 2^k R_{w,k},  R_{w,k} = sum_{c: bit k} T_c
// L need not be a power of two: the host Horner places R_{w,k} once per set bit of L.
// ---------------------------------------------------------------------------------------------
// L = buckets per k_bucket_reduce_1 lane.  Each lane's running sums are a chain of ~2L dependent
// adds and one wave per SIMD already keeps its VALU ~82% busy, so the kernel takes ~one chain per
// SIMD -- as long as the live lanes fit in one wave per SIMD.  The host picks the smallest L
// (of RED1_LS) for which they do (bucket_reduce_L): at c = 15 two MSMs have 540,672 live buckets,
// so L = 8 would need 1,056 waves on 1,024 SIMDs (two chains on some) and L = 9 needs 939.
#ifndef MSM_RED1_THREADS
#define MSM_RED1_THREADS 256
#endif
constexpr uint32_t RED1_THREADS = MSM_RED1_THREADS;

// Chunks of a window that a digit can reach (its "live" chunks; the others hold no entry): a main
// window of the table's full width fills every chunk, a (q)-bit window in a (q+1)-bit table its
// lower half, and the overflow window (|digit| <= 4, buckets 0..3) is counted dead altogether (it
// is empty for canonical scalars).  `a` is the window's index in its MSM.
__host__ __device__ __forceinline__ uint32_t red1_live_chunks(const MsmDims& d, uint32_t L, uint32_t nchunks,
                                                              uint32_t a) {
  if (a + 1 == d.Wm) return 0;
  if (d.nhi == 0 || a < d.nhi) return nchunks;
  return (d.B / 2 + L - 1) / L;
}

// Lane -> (window, chunk) of k_bucket_reduce_1.  Live chunks of every MSM's windows come first, so
// real work is whole waves at the front of the grid; then the dead ones (empty unless the scalars
// are non-canonical), which exit early.
__device__ __forceinline__ bool red1_lane(const MsmDims& d, uint32_t L, uint32_t nchunks, uint32_t gd, uint32_t& w,
                                          uint32_t& c) {
  uint32_t live = 0;  // per MSM
  for (uint32_t l = 0; l < d.Wr; l++) live += red1_live_chunks(d, L, nchunks, d.w0 + l);
  const uint32_t dead = d.Wr * nchunks - live;
  uint32_t r, m;
  bool in_live;
  if (gd < d.nm * live) {
    m = gd / live;
    r = gd % live;
    in_live = true;
  } else {
    const uint32_t r0 = gd - d.nm * live;
    if (r0 >= d.nm * dead) return false;
    m = r0 / dead;
    r = r0 % dead;
    in_live = false;
  }
  for (uint32_t l = 0; l < d.Wr; l++) {
    const uint32_t lc = red1_live_chunks(d, L, nchunks, d.w0 + l);
    const uint32_t span = in_live ? lc : nchunks - lc;
    if (r < span) {
      w = m * d.Wr + l;
      c = in_live ? r : lc + r;
      return true;
    }
    r -= span;
  }
  return false;
}

// Running sums of chunk c of window w (one lane): U = sum_i (i+1) B_i and T = sum_i B_i over the
// chunk's buckets, i counted within the chunk.
template <uint32_t RL>
__device__ __forceinline__ void red1_chunk(const uint32_t* __restrict__ buckets, const uint32_t* __restrict__ bucket_start,
                                           const MsmDims& d, uint32_t K, uint32_t w, uint32_t c,
                                           const uint32_t* __restrict__ cross_key, const uint32_t* __restrict__ lead_val,
                                           xyzt& U, xyzt& T) {
  const uint32_t key0 = w * d.B + c * RL;
  const uint32_t nb = min(RL, d.B - c * RL);  // buckets of this chunk inside the window (last chunk: fewer)
  // bucket metadata up front (independent loads): which buckets are non-empty, and which left
  // their accumulation workgroup and need the continuation from lead_val
  uint32_t bs[RL + 1];
#pragma unroll
  for (uint32_t i = 0; i <= RL; i++) bs[i] = i <= nb ? bucket_start[key0 + i] : 0u;
  uint32_t live = 0, cross = 0;
  const double ginv = 1.0 / ((double)K * ACC_THREADS);  // (bs / K) / ACC_THREADS = bs / (K ACC_THREADS)
#pragma unroll
  for (uint32_t i = 0; i < RL; i++) {
    if (i < nb && bs[i + 1] != bs[i]) {
      live |= 1u << i;
      if (cross_key[div_by_inv(bs[i], ginv)] == key0 + i) cross |= 1u << i;
    }
  }
  if (!live) {  // whole chunk empty (e.g. the windows above the scalars' top bit)
    U = T = pt_identity();
    return;
  }
  xyzt carry = pt_identity(), acc = pt_identity();
  bool carry_live = false, acc_live = false;
  // running sums from the top bucket down; the next live bucket's load is issued before the
  // current bucket's adds.  (Software-pipelining the two adds of a step -- both read the previous
  // carry -- measured 159 -> 184 us at 2^17: the compiler keeps 242 VGPRs and serialises them.)
  int i = 31 - __builtin_clz(live);
  xyzt nb_pt = load_pt(buckets + (size_t)(key0 + i) * PT_WORDS);
#pragma unroll 1
  for (; i >= 0; i--) {
    if ((live >> i) & 1u) {
      xyzt b = nb_pt;
      const uint32_t below = live & ((1u << i) - 1u);
      if (below) nb_pt = load_pt(buckets + (size_t)(key0 + 31 - __builtin_clz(below)) * PT_WORDS);
      if ((cross >> i) & 1u) {  // rare: reload the bucket's start rather than index bs[] dynamically
        const uint32_t g0 = (bucket_start[key0 + i] / K) / ACC_THREADS;
        b = pt_add(b, load_pt(lead_val + (size_t)(g0 + 1) * PT_WORDS));
      }
      carry = carry_live ? pt_add(carry, b) : b;
      carry_live = true;
    }
    if (carry_live) {
      acc = acc_live ? pt_add(acc, carry) : carry;
      acc_live = true;
    }
  }
  U = acc;
  T = carry;
}

template <uint32_t RL>
__global__ void __launch_bounds__(RED1_THREADS) k_bucket_reduce_1(const uint32_t* __restrict__ buckets,
                                                         const uint32_t* __restrict__ bucket_start, MsmDims d,
                                                         uint32_t K, uint32_t nchunks,
                                                         const uint32_t* __restrict__ cross_key,
                                                         const uint32_t* __restrict__ lead_val,
                                                         uint32_t* __restrict__ out_U, uint32_t* __restrict__ out_T) {
  uint32_t w, c;
  if (!red1_lane(d, RL, nchunks, blockIdx.x * blockDim.x + threadIdx.x, w, c)) return;
  const uint32_t g = w * nchunks + c;
  xyzt U, T;
  red1_chunk<RL>(buckets, bucket_start, d, K, w, c, cross_key, lead_val, U, T);
  store_pt(out_U + (size_t)g * PT_WORDS, U);
  store_pt(out_T + (size_t)g * PT_WORDS, T);
}

// The same running sums on lane pairs (MSM_RED1_PAIRS=1; measured no faster, kept off): a chunk's two chains run on two
// lanes in lock step -- the even lane the bucket chain T (carry += B_i, top bucket down), the odd
// lane the weighted chain U (acc += the carry after the even lane's previous step, taken with a
// DPP quad permute) -- so every lane holds one running point instead of two plus the prefetched
// bucket: half the registers (more waves per SIMD to hide the adds' latency) for L + 1 steps of
// one add instead of 2L adds.  Identity adds (empty buckets, the chains' ends) are harmless: the
// formulas are complete.
__device__ __forceinline__ fe fe_from_even(const fe& a) {
  fe r;
#pragma unroll
  for (int i = 0; i < NL; i++) r.v[i] = (uint32_t)__builtin_amdgcn_mov_dpp((int)a.v[i], 0xA0, 0xF, 0xF, false);
  return r;
}

#ifndef MSM_RED1P_WAVES
#define MSM_RED1P_WAVES 3  // waves per SIMD asked of the compiler (4: <= 128 VGPRs, 17 spilled)
#endif
template <uint32_t RL>
__global__ void __launch_bounds__(RED1_THREADS, MSM_RED1P_WAVES) k_bucket_reduce_1p(const uint32_t* __restrict__ buckets,
                                                          const uint32_t* __restrict__ bucket_start, MsmDims d,
                                                          uint32_t K, uint32_t nchunks,
                                                          const uint32_t* __restrict__ cross_key,
                                                          const uint32_t* __restrict__ lead_val,
                                                          uint32_t* __restrict__ out_U, uint32_t* __restrict__ out_T) {
  const bool u_lane = (threadIdx.x & 1u) != 0;
  uint32_t w, c;
  // both lanes of a pair map to the same chunk, so a pair leaves (or stays) together
  if (!red1_lane(d, RL, nchunks, (blockIdx.x * blockDim.x + threadIdx.x) >> 1, w, c)) return;
  const uint32_t g = w * nchunks + c;
  const uint32_t key0 = w * d.B + c * RL;
  const uint32_t nb = min(RL, d.B - c * RL);
  uint32_t live = 0, cross = 0;
  {
    uint32_t bs[RL + 1];
#pragma unroll
    for (uint32_t i = 0; i <= RL; i++) bs[i] = i <= nb ? bucket_start[key0 + i] : 0u;
#pragma unroll
    for (uint32_t i = 0; i < RL; i++) {
      if (i < nb && bs[i + 1] != bs[i]) {
        live |= 1u << i;
        if (!u_lane && cross_key[(bs[i] / K) / ACC_THREADS] == key0 + i) cross |= 1u << i;
      }
    }
  }
  uint32_t* out = (u_lane ? out_U : out_T) + (size_t)g * PT_WORDS;
  if (!live) {  // whole chunk empty (e.g. the windows above the scalars' top bit)
    store_pt(out, pt_identity());
    return;
  }
  const int top = 31 - __builtin_clz(live);
  xyzt run = pt_identity();
#pragma unroll 1
  for (int i = top; i >= -1; i--) {
    // the odd lane's operand: its even lane's carry as it stands before this step's add
    xyzt q;
    q.X = fe_from_even(run.X);
    q.Y = fe_from_even(run.Y);
    q.T = fe_from_even(run.T);
    q.Z = fe_from_even(run.Z);
    if (u_lane) {
      // q as permuted (identity at the first step: the even lane's carry starts there)
    } else if (i >= 0 && ((live >> i) & 1u)) {
      q = load_pt(buckets + (size_t)(key0 + i) * PT_WORDS);
      if ((cross >> i) & 1u) {  // rare: the bucket continues past its accumulation workgroup
        const uint32_t g0 = (bucket_start[key0 + i] / K) / ACC_THREADS;
        q = pt_add(q, load_pt(lead_val + (size_t)(g0 + 1) * PT_WORDS));
      }
    } else {
      q = pt_identity();
    }
    run = pt_add(run, q);
  }
  store_pt(out, run);
}

// One workgroup per (window, term).  Terms 0..nv-1: R_{V,v} = sum of U_c over the v-th slice of
// chunks; term nv+k: R_k = sum_{c: bit k of c} T_c.  Every workgroup sums at most
// pow2ceil(nchunks)/2 points.
// Output: X, Y, T, Z in the host's Montgomery form (a * 2^256 mod p, 8 LE words each), written
// straight into coherent pinned host memory (no readback copy), so the host Horner
// (hostfield.h) uses them without conversion.  Block 0 also forwards the error flags, the entry
// count and whether the joins of skewed buckets are still due.
#ifndef MSM_RED2_THREADS
#define MSM_RED2_THREADS 512
#endif
constexpr int RED2_THREADS = MSM_RED2_THREADS;
#ifndef MSM_RED2_QUAD
#define MSM_RED2_QUAD 256
#endif
constexpr uint32_t RED2_QUAD = MSM_RED2_QUAD;  // tree levels below this many points use quad-cooperative adds
extern "C" __global__ void __launch_bounds__(RED2_THREADS) k_bucket_reduce_2(const uint32_t* __restrict__ in_U,
                                                                             const uint32_t* __restrict__ in_T,
                                                                             uint32_t nchunks, uint32_t nv,
                                                                             uint32_t nterms,
                                                                             uint32_t* __restrict__ err,
                                                                             uint32_t* __restrict__ lead_flag,
                                                                             uint32_t* __restrict__ skew_list,
                                                                             const uint32_t* __restrict__ total,
                                                                             uint32_t final_pass,
                                                                             const uint32_t* __restrict__ bucket_start,
                                                                             uint32_t B,
                                                                             uint32_t* __restrict__ out_host) {
  __shared__ uint32_t sh[RED2_THREADS / 2][PT_WORDS];
  const uint32_t w = blockIdx.x / nterms, term = blockIdx.x % nterms;
  // a window without entries (the overflow window of canonical scalars, a window range's empty
  // windows) has identity terms: skip its loads and latency-bound tree
  const bool empty = bucket_start[(size_t)w * B] == bucket_start[(size_t)(w + 1) * B];
  if (empty) {
    if (threadIdx.x == 0) store_pt_lds(sh[0], pt_identity());
    __syncthreads();
  } else {
    const bool vterm = term < nv;
    const uint32_t* src = vterm ? in_U : in_T;
    const uint32_t kbit = term - nv;
    // A V slice is ceil(nchunks/nv) consecutive chunks; a bit term enumerates its j-th chunk with
    // bit k set directly (j < pow2ceil(nchunks)/2, chunks past the end skipped), so every lane
    // loads about the same number of points (a stride-and-skip loop over all chunks would give half
    // the lanes all the work for k < 10).
    const uint32_t vslice = (nchunks + nv - 1) / nv;
    uint32_t half_n = 1;
    while (2 * half_n < nchunks) half_n <<= 1;
    xyzt acc = pt_identity();
    bool live = false;
    for (uint32_t j = threadIdx.x; j < (vterm ? vslice : half_n); j += RED2_THREADS) {
      const uint32_t c = vterm ? term * vslice + j : (((j >> kbit) << (kbit + 1)) | (1u << kbit) | (j & ((1u << kbit) - 1u)));
      if (c >= nchunks) continue;
      xyzt p = load_pt(src + ((size_t)w * nchunks + c) * PT_WORDS);
      acc = live ? pt_add(acc, p) : p;
      live = true;
    }
    // tree reduce through LDS: upper half hands its point to the lower half each round.  The wide
    // levels add one point per lane; from RED2_QUAD points down, each add is spread over a quad of
    // lanes (pt_add_quad: 3 multiply latencies instead of 9) since those levels are latency-bound.
    for (uint32_t half = RED2_THREADS / 2; half >= RED2_QUAD; half >>= 1) {
      if (threadIdx.x >= half && threadIdx.x < 2 * half) store_pt_lds(sh[threadIdx.x - half], acc);
      __syncthreads();
      if (threadIdx.x < half) acc = pt_add(acc, load_pt_lds(sh[threadIdx.x]));
      __syncthreads();
    }
    if (threadIdx.x < RED2_QUAD) store_pt_lds(sh[threadIdx.x], acc);
    __syncthreads();
    {
      const uint32_t j = threadIdx.x >> 2, q = threadIdx.x & 3;
      for (uint32_t half = RED2_QUAD / 2; half >= 1; half >>= 1) {
        const bool act = j < half;  // uniform across a quad
        fe res;
        if (act) res = pt_add_quad(load_fe_lds(&sh[j][q * NL]), load_fe_lds(&sh[j + half][q * NL]));
        __syncthreads();
        if (act) store_fe_lds(&sh[j][q * NL], res);
        __syncthreads();
      }
    }
  }
  if (threadIdx.x < 4) {  // one lane per coordinate (X, Y, T, Z): the conversions run side by side
    const uint32_t q = threadIdx.x;
    uint32_t* o = out_host + (size_t)blockIdx.x * 32 + 8 * q;
    uint32_t wd[8];
    fe_to_words_le(fe_to_host_mont(load_fe_lds(&sh[0][q * NL])), wd);
#pragma unroll
    for (int k = 0; k < 8; k++) o[k] = wd[k];
  }
  if (threadIdx.x == 0) {
    if (blockIdx.x == 0) {
      // Without the joins in the sequence (final_pass 0), skewed buckets make the terms invalid:
      // the host then runs the joins and this reduction again (msm_host.hip PART_JOIN), so the
      // skew flags stay set for them.
      const size_t tail = (size_t)gridDim.x * 32;
      const bool skew = skew_list[0] != 0 || *lead_flag != 0;
      out_host[tail] = *err;
      out_host[tail + 1] = *total;
      out_host[tail + 2] = (skew && !final_pass) ? 1u : 0u;
      *err = 0;  // flags start the next MSM cleared (no memset node in the graph)
      if (final_pass || !skew) {
        *lead_flag = 0;
        skew_list[0] = 0;
      }
    }
    __threadfence_system();
  }
}

// ---- bucket reduction, second stage in two kernels (k_red2_groups + k_red2_terms) ------------
// k_bucket_reduce_2 sums, per window, every chunk's U_c once and its T_c once per set bit of c
// (~6.5 adds per chunk at 2,048 chunks), in trees whose wide levels make it VALU-bound.  Here
// the chunks of a window go in groups of RG_CH = 2^RG_LOG: k_red2_groups reduces a group in LDS
// to 2 + RG_LOG points,
//   V_g = sum U_c,  S_g = sum T_c,  R_{g,k} = sum_{c: bit k of (c - RG_CH g)} T_c  (k < RG_LOG),
// with ~3 adds per chunk: one tree over U, one over T whose odd operands at level j are exactly
// R_{g,j}'s points (kept in place, lowest set bit of the index = 2^j), and the R trees run in
// the same steps as the main trees (RG_LOG steps of <= 2 RG_CH quad-cooperative adds).
// k_red2_terms then forms the same terms as k_bucket_reduce_2 from <= 64 group points each:
//   V slices = sum V_g,  R_k = sum_g R_{g,k} (k < RG_LOG),  R_k = sum_{g: bit k-RG_LOG of g} S_g,
// since sum_c c T_c = sum_g (RG_CH g S_g + sum_k 2^k R_{g,k}).
#ifndef MSM_RG_LOG
#define MSM_RG_LOG 7
#endif
constexpr uint32_t RG_LOG = MSM_RG_LOG;      // log2 chunks per group
constexpr uint32_t RG_CH = 1u << RG_LOG;     // chunks per group
constexpr uint32_t RG_OUT = 2 + RG_LOG;      // points per group: V, S, R_0..R_{RG_LOG-1}
constexpr uint32_t RG_MAXG = 64;             // groups per window k_red2_terms takes
#ifndef MSM_RED2_SYSFENCE
#define MSM_RED2_SYSFENCE 0
#endif

// Coordinate q (0 X, 1 Y, 2 T, 3 Z) of the identity (0, 1, 0, 1).
__device__ __forceinline__ fe identity_coord(uint32_t q) { return fe_sel((q & 1u) != 0, fe_zero(), fe_one()); }
__device__ __forceinline__ fe load_fe_g(const uint32_t* __restrict__ src) {
  fe a;
#pragma unroll
  for (int k = 0; k < NL; k++) a.v[k] = src[k];
  return a;
}

// The RG_LOG steps of one group's reduction over its chunk points in LDS (T in shA, U in shB):
// leaves V at shB[0], S at shA[0] and R_k at shA[2^k].  Quad Q of the block's quads takes tasks
// Q, Q + nquads, ... of each step (no task of a step reads another's destination).
__device__ __forceinline__ void red2_tree_steps(uint32_t (*shA)[PT_WORDS], uint32_t (*shB)[PT_WORDS]) {
  const uint32_t q = threadIdx.x & 3, nquads = blockDim.x >> 2;
#pragma unroll 1
  for (uint32_t s = 0; s < RG_LOG; s++) {
    const uint32_t lp = RG_LOG - 1 - s;  // log2 of the pairs per list at this step
    const uint32_t ntask = (2 + s) << lp;
#pragma unroll 1
    for (uint32_t Q = threadIdx.x >> 2; Q < ntask; Q += nquads) {
      const uint32_t kind = Q >> lp, i = Q & ((1u << lp) - 1u);
      uint32_t(*arr)[PT_WORDS] = kind == 1 ? shB : shA;
      uint32_t dst, srcx;
      if (kind < 2) {  // the T and U trees: pairs (i 2^(s+1), i 2^(s+1) + 2^s)
        dst = i << (s + 1);
        srcx = dst + (1u << s);
      } else {  // R_j's tree, level s - j - 1, over its list at indices (2 m + 1) 2^j
        const uint32_t j = kind - 2, l = s - j - 1;
        const uint32_t md = i << (l + 1), ms = md + (1u << l);
        dst = (2 * md + 1) << j;
        srcx = (2 * ms + 1) << j;
      }
      const fe r = pt_add_quad(load_fe_lds(&arr[dst][q * NL]), load_fe_lds(&arr[srcx][q * NL]));
      store_fe_lds(&arr[dst][q * NL], r);  // no other task of this step reads dst or srcx
    }
    __syncthreads();
  }
}

// One group's reduction (k_red2_groups): chunks g RG_CH .. of window w from in_U / in_T into
// shA (T) / shB (U), then the steps.  Every thread of the block takes part (4 RG_CH threads,
// quad Q = chunk).
__device__ __forceinline__ void red2_group_tree(const uint32_t* __restrict__ in_U, const uint32_t* __restrict__ in_T,
                                                uint32_t nchunks, uint32_t w, uint32_t g,
                                                uint32_t (*shA)[PT_WORDS], uint32_t (*shB)[PT_WORDS]) {
  const uint32_t Q = threadIdx.x >> 2, q = threadIdx.x & 3;
  const uint32_t c = g * RG_CH + Q;
  fe u, t;
  if (c < nchunks) {
    const size_t off = ((size_t)w * nchunks + c) * PT_WORDS + q * NL;
    u = load_fe_g(in_U + off);
    t = load_fe_g(in_T + off);
  } else {
    u = t = identity_coord(q);
  }
  store_fe_lds(&shB[Q][q * NL], u);
  store_fe_lds(&shA[Q][q * NL], t);
  __syncthreads();
  red2_tree_steps(shA, shB);
}

// Group point idx (0 V, 1 S, 2 + k R_k) of the tree left in shA / shB.
__device__ __forceinline__ const uint32_t* red2_group_point(uint32_t (*shA)[PT_WORDS], uint32_t (*shB)[PT_WORDS],
                                                            uint32_t idx) {
  return idx == 0 ? shB[0] : idx == 1 ? shA[0] : shA[1u << (idx - 2)];
}

// Which group points make term `term` of a window: point idx of groups g0 + j (or, for the bit
// terms past RG_LOG, of the j-th group with bit kbit set), j < npts.
struct Red2Term {
  uint32_t idx, g0, g1, kbit, npts;
  bool bitsel;
};
__device__ __forceinline__ Red2Term red2_term(uint32_t term, uint32_t nv, uint32_t ngroups) {
  Red2Term r{0, 0, 0, 0, 0, false};
  if (term < nv) {
    const uint32_t sl = (ngroups + nv - 1) / nv;
    r.g0 = min(ngroups, term * sl);
    r.g1 = min(ngroups, r.g0 + sl);
    r.npts = r.g1 - r.g0;
  } else if (term - nv < RG_LOG) {
    r.idx = 2 + (term - nv);
    r.g1 = ngroups;
    r.npts = ngroups;
  } else {
    r.idx = 1;
    r.kbit = term - nv - RG_LOG;
    r.bitsel = true;
    r.npts = 1;  // g = ((j >> kbit) << (kbit + 1)) | (1 << kbit) | (j & (2^kbit - 1)), j < pow2ceil(ngroups) / 2
    while (2 * r.npts < ngroups) r.npts <<= 1;
  }
  return r;
}
__device__ __forceinline__ uint32_t red2_term_group(const Red2Term& t, uint32_t j) {
  return t.bitsel ? (((j >> t.kbit) << (t.kbit + 1)) | (1u << t.kbit) | (j & ((1u << t.kbit) - 1u))) : t.g0 + j;
}

// Block 0 of k_red2_terms: the MSM's flags beside the terms (as k_bucket_reduce_2).
__device__ __forceinline__ void red2_flags(uint32_t nwindows_terms, uint32_t* __restrict__ err,
                                           uint32_t* __restrict__ lead_flag, uint32_t* __restrict__ skew_list,
                                           const uint32_t* __restrict__ total, uint32_t final_pass,
                                           uint32_t* __restrict__ out_host) {
  const size_t tail = (size_t)nwindows_terms * 32;
  const bool skew = skew_list[0] != 0 || *lead_flag != 0;
  out_host[tail] = *err;
  out_host[tail + 1] = *total;
  out_host[tail + 2] = (skew && !final_pass) ? 1u : 0u;
  *err = 0;
  if (final_pass || !skew) {
    *lead_flag = 0;
    skew_list[0] = 0;
  }
}

extern "C" __global__ void __launch_bounds__(4 * RG_CH) k_red2_groups(const uint32_t* __restrict__ in_U,
                                                                     const uint32_t* __restrict__ in_T,
                                                                     uint32_t nchunks, uint32_t ngroups,
                                                                     const uint32_t* __restrict__ bucket_start,
                                                                     uint32_t B, uint32_t* __restrict__ out) {
  __shared__ uint32_t shA[RG_CH][PT_WORDS];  // T, then its partial sums and the R lists in place
  __shared__ uint32_t shB[RG_CH][PT_WORDS];  // U
  const uint32_t w = blockIdx.x / ngroups, g = blockIdx.x % ngroups;
  if (bucket_start[(size_t)w * B] == bucket_start[(size_t)(w + 1) * B]) return;  // empty window: unread
  red2_group_tree(in_U, in_T, nchunks, w, g, shA, shB);
  const uint32_t Q = threadIdx.x >> 2, q = threadIdx.x & 3;
  if (Q < RG_OUT) {
    const fe v = load_fe_lds(red2_group_point(shA, shB, Q) + q * NL);
    uint32_t* o = out + (((size_t)w * ngroups + g) * RG_OUT + Q) * PT_WORDS + q * NL;
#pragma unroll
    for (int k = 0; k < NL; k++) o[k] = v.v[k];
  }
}

// The first stage and the group trees in one launch (MSM_RED_FOLD=1; measured slower, kept off:
// the tree runs at the first stage's occupancy, two 226-VGPR waves per group): a workgroup of RG_CH
// lanes takes one group of RG_CH consecutive chunks of a window -- each lane its chunk's running
// sums (red1_chunk), straight into LDS, then the group's tree (red2_tree_steps, 32 quads) -- and
// writes the group's V, S and R_0..R_{RG_LOG-1}: the chunk sums never go to memory and the second
// launch of the stage (k_red2_groups) is gone.  Live groups first (red1_group), then the dead ones
// (chunks a canonical scalar's digit cannot reach); a group without entries writes identities, and
// an empty window's groups are not read.
__device__ __forceinline__ bool red1_group(const MsmDims& d, uint32_t L, uint32_t nchunks, uint32_t G, uint32_t gd,
                                           uint32_t& w, uint32_t& g, bool& live) {
  uint32_t lg = 0;  // live groups per MSM
  for (uint32_t l = 0; l < d.Wr; l++) lg += (red1_live_chunks(d, L, nchunks, d.w0 + l) + RG_CH - 1) / RG_CH;
  const uint32_t dg = d.Wr * G - lg;
  uint32_t r, m;
  if (gd < d.nm * lg) {
    m = gd / lg;
    r = gd % lg;
    live = true;
  } else {
    const uint32_t r0 = gd - d.nm * lg;
    if (r0 >= d.nm * dg) return false;
    m = r0 / dg;
    r = r0 % dg;
    live = false;
  }
  for (uint32_t l = 0; l < d.Wr; l++) {
    const uint32_t lgl = (red1_live_chunks(d, L, nchunks, d.w0 + l) + RG_CH - 1) / RG_CH;
    const uint32_t span = live ? lgl : G - lgl;
    if (r < span) {
      w = m * d.Wr + l;
      g = live ? r : lgl + r;
      return true;
    }
    r -= span;
  }
  return false;
}

template <uint32_t RL>
__global__ void __launch_bounds__(RG_CH) k_bucket_reduce_1g(const uint32_t* __restrict__ buckets,
                                                          const uint32_t* __restrict__ bucket_start, MsmDims d,
                                                          uint32_t K, uint32_t nchunks, uint32_t ngroups,
                                                          const uint32_t* __restrict__ cross_key,
                                                          const uint32_t* __restrict__ lead_val,
                                                          uint32_t* __restrict__ out) {
  __shared__ uint32_t shA[RG_CH][PT_WORDS];  // T
  __shared__ uint32_t shB[RG_CH][PT_WORDS];  // U
  uint32_t w, g;
  bool live;  // (order only: a dead group with entries is reduced like any other)
  if (!red1_group(d, RL, nchunks, ngroups, blockIdx.x, w, g, live)) return;
  if (bucket_start[(size_t)w * d.B] == bucket_start[(size_t)(w + 1) * d.B]) return;  // empty window: unread
  uint32_t* o = out + ((size_t)w * ngroups + g) * RG_OUT * PT_WORDS;
  // a group without entries (the dead groups, unless the scalars are non-canonical) is identities
  const uint32_t kb0 = w * d.B + min(d.B, g * RG_CH * RL), kb1 = w * d.B + min(d.B, (g + 1) * RG_CH * RL);
  if (bucket_start[kb0] == bucket_start[kb1]) {
    for (uint32_t k = threadIdx.x; k < RG_OUT * 4; k += RG_CH) {
      const fe id = identity_coord(k & 3);
#pragma unroll
      for (int j = 0; j < NL; j++) o[(k >> 2) * PT_WORDS + (k & 3) * NL + j] = id.v[j];
    }
    return;
  }
  const uint32_t c = g * RG_CH + threadIdx.x;
  xyzt U = pt_identity(), T = pt_identity();
  if (c < nchunks) red1_chunk<RL>(buckets, bucket_start, d, K, w, c, cross_key, lead_val, U, T);
  store_pt_lds(shB[threadIdx.x], U);
  store_pt_lds(shA[threadIdx.x], T);
  __syncthreads();
  red2_tree_steps(shA, shB);
  const uint32_t Q = threadIdx.x >> 2, q = threadIdx.x & 3;
  if (Q < RG_OUT) {
    const fe v = load_fe_lds(red2_group_point(shA, shB, Q) + q * NL);
#pragma unroll
    for (int k = 0; k < NL; k++) o[Q * PT_WORDS + q * NL + k] = v.v[k];
  }
}

extern "C" __global__ void __launch_bounds__(4 * RG_MAXG) k_red2_terms(const uint32_t* __restrict__ grp,
                                                                      uint32_t ngroups, uint32_t nv,
                                                                      uint32_t nterms, uint32_t* __restrict__ err,
                                                                      uint32_t* __restrict__ lead_flag,
                                                                      uint32_t* __restrict__ skew_list,
                                                                      const uint32_t* __restrict__ total,
                                                                      uint32_t final_pass,
                                                                      const uint32_t* __restrict__ bucket_start,
                                                                      uint32_t B, uint32_t* __restrict__ out_host) {
  __shared__ uint32_t sh[RG_MAXG][PT_WORDS];
  const uint32_t w = blockIdx.x / nterms, term = blockIdx.x % nterms;
  const uint32_t Q = threadIdx.x >> 2, q = threadIdx.x & 3;
  const bool empty = bucket_start[(size_t)w * B] == bucket_start[(size_t)(w + 1) * B];
  const Red2Term rt = red2_term(term, nv, ngroups);
  fe v = identity_coord(q);
  if (!empty && Q < rt.npts) {
    const uint32_t g = red2_term_group(rt, Q);
    if (g < ngroups) v = load_fe_g(grp + (((size_t)w * ngroups + g) * RG_OUT + rt.idx) * PT_WORDS + q * NL);
  }
  store_fe_lds(&sh[Q][q * NL], v);
  __syncthreads();
  uint32_t half = 1;
  while (2 * half < rt.npts) half <<= 1;
  if (empty || rt.npts <= 1) half = 0;
#pragma unroll 1
  for (; half >= 1; half >>= 1) {
    if (Q < half) {
      const fe r = pt_add_quad(load_fe_lds(&sh[Q][q * NL]), load_fe_lds(&sh[Q + half][q * NL]));
      store_fe_lds(&sh[Q][q * NL], r);
    }
    __syncthreads();
  }
  if (threadIdx.x < 4) {  // as k_bucket_reduce_2: host Montgomery form, straight into pinned memory
    uint32_t* o = out_host + (size_t)blockIdx.x * 32 + 8 * q;
    uint32_t wd[8];
    fe_to_words_le(fe_to_host_mont(load_fe_lds(&sh[0][q * NL])), wd);
#pragma unroll
    for (int k = 0; k < 8; k++) o[k] = wd[k];
  }
#if MSM_RED2_SYSFENCE
  if (threadIdx.x == 0) {
    if (blockIdx.x == 0) red2_flags(gridDim.x, err, lead_flag, skew_list, total, final_pass, out_host);
    __threadfence_system();
  }
#else
  // no system-scope fence per workgroup: the host reads the terms only after the launch's event,
  // whose completion makes the kernel's writes to pinned memory visible
  if (threadIdx.x == 0 && blockIdx.x == 0) red2_flags(gridDim.x, err, lead_flag, skew_list, total, final_pass, out_host);
#endif
}

// Small utility kernels used by tests: batch field ops / point ops on canonical inputs.
// op 0: field mul, 1: add, 2: sub, 3: 2d * a (fe_mul_2d); inputs LE standard words [n][8] x2, output [n][8].
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
  // ops 4, 5: pt_madd's signed-difference multiply, (x - y)(y - x) and (x - y)(x + y)
  fe r = op == 0   ? fe_mul(x, y)
         : op == 1 ? fe_add_n(x, y)
         : op == 2 ? fe_sub(x, y)
         : op == 3 ? fe_mul_2d(x)
         : op == 4 ? fe_mul_sd<WIDE_ALL, true>(fe_sub_s(x, y), fe_sub_s(y, x))
                   : fe_mul_sd<WIDE_ALL, false>(fe_sub_s(x, y), fe_add(x, y));
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
    pre qq;  // halved, as k_prepare_points writes it
    qq.ymx = fe_mul(fe_sub(Q.Y, Q.X), fe_const(HALF29));
    qq.ypx = fe_mul(fe_add_n(Q.Y, Q.X), fe_const(HALF29));
    qq.kt = fe_mul(Q.T, fe_const(KD29));
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

// Quad-cooperative add check: pair i is handled by lanes 4i..4i+3.  Inputs as k_test_point
// (affine LE words), output X,Y,T,Z std LE words [n][32].
extern "C" __global__ void k_test_quad(const uint32_t* __restrict__ p, const uint32_t* __restrict__ q,
                                       uint32_t* __restrict__ out, uint32_t n) {
  const uint32_t i = (blockIdx.x * blockDim.x + threadIdx.x) >> 2, c = threadIdx.x & 3;
  const bool live = i < n;
  const uint32_t ii = live ? i : 0;
  uint32_t w[4][8];
#pragma unroll
  for (int k = 0; k < 8; k++) {
    w[0][k] = p[(size_t)ii * 16 + k];
    w[1][k] = p[(size_t)ii * 16 + 8 + k];
    w[2][k] = q[(size_t)ii * 16 + k];
    w[3][k] = q[(size_t)ii * 16 + 8 + k];
  }
  const fe px = fe_to_mont(fe_from_words_le(w[0])), py = fe_to_mont(fe_from_words_le(w[1]));
  const fe qx = fe_to_mont(fe_from_words_le(w[2])), qy = fe_to_mont(fe_from_words_le(w[3]));
  const fe pc[4] = {px, py, fe_mul(px, py), fe_one()};
  const fe qc[4] = {qx, qy, fe_mul(qx, qy), fe_one()};
  fe a = pc[0], b = qc[0];
#pragma unroll
  for (uint32_t k = 1; k < 4; k++) {
    a = fe_sel(c == k, a, pc[k]);
    b = fe_sel(c == k, b, qc[k]);
  }
  const fe r = pt_add_quad(a, b);
  uint32_t ow[8];
  fe_to_words_le(fe_to_std(r), ow);
  if (live) {
#pragma unroll
    for (int k = 0; k < 8; k++) out[(size_t)i * 32 + c * 8 + k] = ow[k];
  }
}

}  // namespace msm
