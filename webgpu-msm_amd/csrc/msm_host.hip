// libmsm host driver: C ABI (include/msm.h), device workspaces, launch sequence, host tail.
//
// The reference's host orchestration this replaces:
//   compute_msm            src/submission/submission.ts:25-157   -> msm_compute / msm_compute_device
//   getBestWindowSize      submission.ts:18-23                    -> msm_best_window
//   gpuIntraBucketReduction src/submission/gpu.ts:36-285          -> k_prepare_points .. k_fixup
//   split_dynamic          msm-wasm/src/lib.rs:196-202            -> msm_split (host) / k_recode_* (device)
//   inter_bucket_reduce    lib.rs:46-56, 123-133                  -> k_bucket_reduce_1/2
//   reduce_last            lib.rs:88-104                          -> horner_tail (host)
//   point_add_affine       lib.rs:240-253                         -> msm_point_add_affine
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "../../include/msm.h"
#include "hostfield.h"
#include "msm_util.h"
#include "msm_kernels.hip"

using namespace msm;
using namespace msmh;

namespace {

#define HIPCHECK(expr)                                                                         \
  do {                                                                                         \
    hipError_t _e = (expr);                                                                    \
    if (_e != hipSuccess) {                                                                    \
      fprintf(stderr, "libmsm: HIP error %s at %s:%d\n", hipGetErrorString(_e), __FILE__, __LINE__); \
      return _e == hipErrorOutOfMemory ? MSM_ERR_OOM : MSM_ERR_HIP;                            \
    }                                                                                          \
  } while (0)

enum Phase {
  PH_START = 0,
  PH_PREPARE,
  PH_RECODE,
  PH_SCAN,
  PH_SCATTER,
  PH_FINE,
  PH_ACCUM,
  PH_FIXUP,
  PH_RED1,
  PH_RED2,
  PH_READBACK,
  PH_COUNT
};

uint64_t g_alloc_gen = 0;  // bumped on every (re)allocation: captured graphs hold raw pointers

struct Buf {
  void* p = nullptr;
  size_t cap = 0;
  int ensure(size_t bytes) {
    if (bytes <= cap) return MSM_OK;
    g_alloc_gen++;
    if (p) hipFree(p);
    p = nullptr;
    cap = 0;
    size_t want = std::max<size_t>(bytes, 256);
    if (hipMalloc(&p, want) != hipSuccess) {
      p = nullptr;
      return MSM_ERR_OOM;
    }
    cap = want;
    return MSM_OK;
  }
  template <typename T>
  T* as() const {
    return reinterpret_cast<T*>(p);
  }
  void release() {
    if (p) hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

struct HostBuf {
  void* p = nullptr;
  size_t cap = 0;
  int ensure(size_t bytes) {
    if (bytes <= cap) return MSM_OK;
    g_alloc_gen++;
    if (p) hipHostFree(p);
    p = nullptr;
    cap = 0;
    // pinned, host-cacheable memory; k_bucket_reduce_2 writes its results straight into it and
    // publishes them with __threadfence_system() (a coherent/uncached mapping would make the
    // host Horner's reads ~4x slower)
    if (hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) {
      p = nullptr;
      return MSM_ERR_OOM;
    }
    cap = bytes;
    return MSM_OK;
  }
  void release() {
    if (p) hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
};

struct Plan {
  MsmDims d;
  uint32_t K;       // run length
  uint32_t L;       // bucket-reduce chunk length
  uint32_t lgL;
  uint32_t nchunks; // B / L
  uint32_t nv;      // V-slices: R_V = sum_c U_c is split into nv equal partial sums
  uint32_t nterms;  // nv + log2(nchunks)
  size_t Mmax;      // W * n upper bound on sorted entries
  size_t runs_max;
};

// Device workspace of one MSM (all sizes from Plan; grown on demand, never shrunk).
struct Workspace {
  Buf pts, err, digits, hist_rows, rel, colsum, bin_base;
  Buf part_entry, part_fine, sorted_entry, bucket_start, run_key, buckets, big_tiles, cursor;
  Buf lead_val, lead_open, cross_key, lead_flag, skew_list, g_head, g_hkey, g_tkey, red_U, red_T;
  void release() {
    Buf* bufs[] = {&pts, &err, &digits, &hist_rows, &rel, &colsum, &bin_base, &part_entry, &part_fine,
                   &sorted_entry, &bucket_start, &run_key, &buckets, &big_tiles, &cursor, &lead_val, &lead_open, &cross_key,
                   &lead_flag, &skew_list, &g_head, &g_hkey, &g_tkey, &red_U, &red_T};
    for (Buf* b : bufs) b->release();
  }
};

// One in-flight MSM: its own stream, device workspace, result buffer, captured graphs and events.
// Several slots let msm_compute_many_device keep MSMs b+1.. on the device while MSM b is still
// there (the latency-bound tails of one overlap the others' kernels) and while the host
// finishes MSM b (window Horner).
struct Slot {
  hipStream_t stream = nullptr;
  Workspace ws;
  HostBuf h_out;  // k_bucket_reduce_2 writes the window terms, err and total here
  void* h_out_dev = nullptr;
  struct GraphKey {
    size_t n;
    uint32_t c, K, nm;
    int prof;
    uint64_t gen;
    bool operator==(const GraphKey& o) const {
      return n == o.n && c == o.c && K == o.K && nm == o.nm && prof == o.prof && gen == o.gen;
    }
  } gkey{};
  hipGraph_t graph[3] = {nullptr, nullptr, nullptr};
  hipGraphExec_t gexec[3] = {nullptr, nullptr, nullptr};  // whole MSM, or pre / - / post
  // the two kernel nodes (in graph[0]) that take the MSM's input buffers: repointed per launch
  hipGraphNode_t n_prep = nullptr, n_recode = nullptr;
  hipKernelNodeParams p_prep{}, p_recode{};
  BatchPtrs g_pts{}, g_sc{};  // inputs the instantiated graph currently reads
  hipEvent_t ev_start = nullptr, ev_acc0 = nullptr, ev_acc1 = nullptr, ev_end = nullptr, ev_done = nullptr;
  Plan pl{};
  bool bracketed = false;
};
constexpr int NSLOT = 4;  // at most this many MSMs in flight (one HIP stream each)
constexpr uint32_t PROF_EVERY = 4;

struct DevCtx {
  int device = -1;
  int n_cu = 256;
  std::mutex mu;
  Buf wire_points, wire_scalars;  // staging for host-resident inputs (msm_compute)
  Slot slot[NSLOT];
  uint32_t prof_seq = 0;
  hipEvent_t ev[PH_COUNT] = {};  // per-phase events (profiling mode 1)
  int profiling = 0;  // 0 off, 1 every phase (eager launches), 2 k_accumulate only (graph-friendly)
  // The launch sequence of each slot is captured once into HIP graphs and replayed: one
  // hipGraphLaunch instead of ~16 enqueues per MSM.
  bool graphs_ok = true;
  msm_profile_t last{};
};

std::mutex g_mu;
std::vector<DevCtx*> g_ctx;
int g_profiling = 0;
int g_ndev = -1;

int probe_devices() {
  if (g_ndev >= 0) return g_ndev;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
  int good = 0;
  for (int i = 0; i < n; i++) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, i) == hipSuccess && strncmp(prop.gcnArchName, "gfx950", 6) == 0) good++;
  }
  g_ndev = good == n ? n : good;
  return g_ndev;
}

int get_ctx(int device, DevCtx** out) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (probe_devices() <= 0) return MSM_ERR_NO_DEVICE;
  if (device < 0) {
    if (hipGetDevice(&device) != hipSuccess) return MSM_ERR_HIP;
  }
  if (device >= g_ndev) return MSM_ERR_INVALID_ARG;
  if ((int)g_ctx.size() < g_ndev) g_ctx.resize(g_ndev, nullptr);
  if (!g_ctx[device]) {
    DevCtx* c = new DevCtx();
    c->device = device;
    int prev = 0;
    hipGetDevice(&prev);
    if (hipSetDevice(device) != hipSuccess) {
      delete c;
      return MSM_ERR_HIP;
    }
    for (Slot& sl : c->slot) {
      if (hipStreamCreateWithFlags(&sl.stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        hipSetDevice(prev);
        return MSM_ERR_HIP;
      }
    }
    for (int i = 0; i < PH_COUNT; i++) hipEventCreate(&c->ev[i]);
    for (Slot& sl : c->slot) {
      hipEventCreate(&sl.ev_start);
      hipEventCreate(&sl.ev_acc0);
      hipEventCreate(&sl.ev_acc1);
      hipEventCreate(&sl.ev_end);
      hipEventCreateWithFlags(&sl.ev_done, hipEventDisableTiming);
    }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
      c->n_cu = prop.multiProcessorCount;
    hipSetDevice(prev);
    g_ctx[device] = c;
  }
  g_ctx[device]->profiling = g_profiling;
  *out = g_ctx[device];
  return MSM_OK;
}

uint32_t ilog2(uint32_t v) {
  uint32_t r = 0;
  while ((1u << (r + 1)) <= v) r++;
  return r;
}

// Window width for MSMs kept in flight by the pipelined entries (whole-job throughput rather
// than one MSM's latency): there the bucket reduction's work, not its latency, is what counts,
// so sub-2^20 sizes prefer narrower windows.  Measured on MI355X (tools/window_sweep.sh): c = 14
// at 2^16, 15 at 2^17..2^19 (-16% at 2^17 vs c = 16), 16 from 2^20.
uint32_t pipelined_window(size_t n) {
  if (n >= (1u << 20)) return 16;
  if (n >= (1u << 17)) return 15;
  if (n >= (1u << 15)) return 14;
  return msm_best_window(n);
}

int make_plan(size_t n, const msm_opts* o, int n_cu, Plan* pl, bool pipelined = false, uint32_t nm = 1) {
  uint32_t c = (o && o->window_bits) ? o->window_bits : pipelined ? pipelined_window(n) : msm_best_window(n);
  if (c < 4 || c > 20) return MSM_ERR_UNSUPPORTED_WINDOW;
  if (n >= (1ull << 30)) return MSM_ERR_INVALID_ARG;
  MsmDims d;
  d.n = (uint32_t)n;
  d.c = c;
  // balanced main windows of at most c bits over MAIN_BITS, plus the overflow window
  const uint32_t wm = (MAIN_BITS + c - 1) / c;
  d.q = MAIN_BITS / wm;
  d.nhi = MAIN_BITS - d.q * wm;
  d.Wm = wm + 1;
  d.nm = nm;
  d.W = d.Wm * nm;
  d.c = d.nhi ? d.q + 1 : d.q;
  d.B = 1u << (d.c - 1);
  // Coarse bins: aim at ~4K entries per bin (half the LDS staging capacity of k_fine_sort) with at
  // most FS_MAXF buckets per bin.  Partition chunks hold >= 64 entries per bin slice.
  uint32_t nbc = 1;
  while (nbc < d.B && nbc < 256 && (size_t)nbc * 4096 < n) nbc <<= 1;
  while (nbc < d.B && (d.B / nbc) > FS_MAXF) nbc <<= 1;
  d.nbc = nbc;
  d.fb = ilog2(d.B / nbc);
  d.packed = ((uint64_t)nm * n) <= (1ull << (31 - d.fb)) ? 1u : 0u;
  d.nbins = d.W * d.nbc;
  d.ch = PT_THREADS * PS_R;  // 16384 digits per partition chunk (>= 64 per bin slice while nbc <= 256)
  d.nch = (uint32_t)((n + d.ch - 1) / d.ch);
  pl->d = d;
  // Run length: long enough to amortise the per-run head/tail joins, short enough to leave
  // ~4 waves per SIMD (262144 lanes) of accumulation work.
  uint32_t kauto = 64;
  while (kauto > 16 && (size_t)d.W * n / kauto < 262144) kauto >>= 1;
  pl->K = (o && o->run_length) ? o->run_length : kauto;
  if (pl->K < 1 || pl->K > 4096) return MSM_ERR_INVALID_ARG;
  static const uint32_t l_env = getenv("MSM_RED_L") ? (uint32_t)atoi(getenv("MSM_RED_L")) : 0u;
  // Buckets per k_bucket_reduce_1 lane.  L = 16 halves k_bucket_reduce_2's bit-term work but
  // doubles the running-sum chain: a throughput win only for the wide pipelined windows (2^20:
  // -1.5% per MSM; single-MSM latency +50 us at 2^18-2^19).  tools/l_sweep.sh; MSM_RED_L overrides.
  pl->L = (l_env == 4 || l_env == 8 || (l_env == 16 && d.B >= 32)) ? l_env
          : (pipelined && d.B >= (1u << 15)) ? 16u : 8u;
  pl->lgL = ilog2(pl->L);
  pl->nchunks = d.B / pl->L;
  // every k_bucket_reduce_2 workgroup sums at most nchunks/2 points (the R_k terms' size)
  pl->nv = pl->nchunks >= 2 ? 2 : 1;
  pl->nterms = pl->nv + ilog2(pl->nchunks);
  pl->Mmax = (size_t)d.W * n;
  pl->runs_max = (pl->Mmax + pl->K - 1) / pl->K + 1;
  if (pl->Mmax >= (1ull << 31)) return MSM_ERR_INVALID_ARG;
  return MSM_OK;
}

int ensure_workspace(DevCtx* c, const Plan& pl, int si) {
  Slot& sl0 = c->slot[si];
  Workspace& w = sl0.ws;
  const MsmDims& d = pl.d;
  const size_t nb = (size_t)d.W * d.B;
  int rc;
  const uint64_t gen0 = g_alloc_gen;
#define ENS(buf, bytes) \
  if ((rc = w.buf.ensure(bytes)) != MSM_OK) return rc
  ENS(pts, (size_t)d.nm * d.n * PRE_WORDS * 4);
  ENS(err, 16);
  ENS(digits, (size_t)d.W * d.n * 4);
  ENS(hist_rows, (size_t)d.nch * d.nbins * 4);
  ENS(rel, (size_t)d.nch * d.nbins * 4);
  ENS(colsum, (size_t)d.nbins * 4);
  ENS(bin_base, ((size_t)d.nbins + 1) * 4);
  ENS(part_entry, pl.Mmax * 4);
  ENS(part_fine, pl.Mmax * 2);
  ENS(sorted_entry, pl.Mmax * 4 + 16);  // + a 16-B tail for k_accumulate's vector entry loads
  ENS(bucket_start, (nb + 2) * 4);
  ENS(run_key, pl.runs_max * 4);
  ENS(big_tiles, (pl.Mmax / FS_CAP + d.nbins + 1) * 8 + 8);
  ENS(cursor, nb * 4);
  ENS(buckets, nb * PT_WORDS * 4);
  const size_t nwg = pl.runs_max / ACC_THREADS + 2;
  ENS(lead_val, nwg * PT_WORDS * 4);
  ENS(lead_open, nwg * 4);
  ENS(cross_key, nwg * 4);
  ENS(lead_flag, 16);
  ENS(skew_list, (nwg + 1) * 4);
  ENS(g_head, pl.runs_max * PT_WORDS * 4);  // touched only by skewed workgroups
  ENS(g_hkey, pl.runs_max * 4);
  ENS(g_tkey, pl.runs_max * 4);
  ENS(red_U, (size_t)d.W * pl.nchunks * PT_WORDS * 4);
  ENS(red_T, (size_t)d.W * pl.nchunks * PT_WORDS * 4);
#undef ENS
  if (g_alloc_gen != gen0) {
    // err, lead_flag and hist_rows are kept all-zero between MSMs by the kernels themselves
    // (k_bucket_reduce_2 clears the flags, k_part_scatter the histogram rows it consumed), so a
    // replayed graph needs no memset nodes; fresh allocations start that invariant here.
    hipStream_t st = sl0.stream;
    if (hipMemsetAsync(w.err.p, 0, w.err.cap, st) != hipSuccess ||
        hipMemsetAsync(w.lead_flag.p, 0, w.lead_flag.cap, st) != hipSuccess ||
        hipMemsetAsync(w.skew_list.p, 0, 4, st) != hipSuccess ||
        hipMemsetAsync(w.hist_rows.p, 0, w.hist_rows.cap, st) != hipSuccess || hipStreamSynchronize(st) != hipSuccess)
      return MSM_ERR_HIP;
  }
  const size_t hbytes = (size_t)d.W * pl.nterms * 32 * 4 + 64;
  if (hbytes > sl0.h_out.cap || !sl0.h_out_dev) {
    if ((rc = sl0.h_out.ensure(hbytes)) != MSM_OK) return rc;
    if (hipHostGetDevicePointer(&sl0.h_out_dev, sl0.h_out.p, 0) != hipSuccess) return MSM_ERR_HIP;
  }
  return MSM_OK;
}

inline unsigned grid_for(size_t threads, unsigned block) { return (unsigned)((threads + block - 1) / block); }

// Enqueue (parts of) the device pipeline on `s`; the reduced per-window terms land in c->h_out.
// PART_PRE: memsets, point preparation and the sort; PART_ACC: bucket accumulation;
// PART_POST: fixup and bucket reduction.
constexpr int PART_PRE = 1, PART_ACC = 2, PART_POST = 4, PART_ALL = 7;
int enqueue_msm(DevCtx* c, const Plan& pl, const BatchPtrs& d_points, const BatchPtrs& d_scalars, int si,
                hipStream_t s, int parts = PART_ALL) {
  const MsmDims& d = pl.d;
  Slot& sl = c->slot[si];
  Workspace& w = sl.ws;
  const bool prof = c->profiling == 1;
  auto mark = [&](int ph) {
    if (prof) hipEventRecord(c->ev[ph], s);
  };
  const uint32_t* total = w.bin_base.as<uint32_t>() + d.nbins;
  const unsigned rgrid = grid_for(pl.runs_max, ACC_THREADS);
  if (parts & PART_PRE) {
  mark(PH_START);
  hipLaunchKernelGGL(k_prepare_points, dim3(grid_for(d.n, PP_THREADS), d.nm), dim3(PP_THREADS), 0, s, d_points, w.pts.as<uint32_t>(), d.n,
                     w.err.as<uint32_t>());
  mark(PH_PREPARE);
  const size_t hist_lds = (size_t)d.Wm * d.nbc * 4;
  const unsigned rc_grid = grid_for(d.n, RC_SPAN);
  if (d.c <= 16) {
    hipLaunchKernelGGL(k_recode_hist<uint16_t>, dim3(rc_grid, d.nm), dim3(RC_THREADS), hist_lds, s, d_scalars, d,
                       w.digits.as<uint16_t>(), w.hist_rows.as<uint32_t>());
  } else {
    hipLaunchKernelGGL(k_recode_hist<uint32_t>, dim3(rc_grid, d.nm), dim3(RC_THREADS), hist_lds, s, d_scalars, d,
                       w.digits.as<uint32_t>(), w.hist_rows.as<uint32_t>());
  }
  mark(PH_RECODE);
  hipLaunchKernelGGL(k_part_colscan, dim3(grid_for(d.nbc, 64), d.W), dim3(1024), 0, s, w.hist_rows.as<uint32_t>(), d,
                     w.rel.as<uint32_t>(), w.colsum.as<uint32_t>());
  hipLaunchKernelGGL(k_bin_scan, dim3(1), dim3(1024), 0, s, w.colsum.as<uint32_t>(), w.bin_base.as<uint32_t>(),
                     d.nbins, w.big_tiles.as<uint32_t>());
  mark(PH_SCAN);
  if (d.c <= 16) {
    hipLaunchKernelGGL(k_part_scatter<uint16_t>, dim3(d.nch, d.W), dim3(PT_THREADS), (size_t)d.nbc * 12, s,
                       w.digits.as<uint16_t>(), d, w.hist_rows.as<uint32_t>(), w.rel.as<uint32_t>(),
                       w.bin_base.as<uint32_t>(), w.part_entry.as<uint32_t>(), w.part_fine.as<uint16_t>());
  } else {
    hipLaunchKernelGGL(k_part_scatter<uint32_t>, dim3(d.nch, d.W), dim3(PT_THREADS), (size_t)d.nbc * 12, s,
                       w.digits.as<uint32_t>(), d, w.hist_rows.as<uint32_t>(), w.rel.as<uint32_t>(),
                       w.bin_base.as<uint32_t>(), w.part_entry.as<uint32_t>(), w.part_fine.as<uint16_t>());
  }
  mark(PH_SCATTER);
  hipLaunchKernelGGL(k_fine_sort, dim3(d.nbins), dim3(FS_THREADS), 0, s, w.part_entry.as<uint32_t>(),
                     w.part_fine.as<uint16_t>(), w.bin_base.as<uint32_t>(), d, pl.K, w.sorted_entry.as<uint32_t>(),
                     w.bucket_start.as<uint32_t>(), w.run_key.as<uint32_t>(), w.cursor.as<uint32_t>());
  hipLaunchKernelGGL(k_big_place, dim3(BP_GRID), dim3(FS_THREADS), 0, s, w.part_entry.as<uint32_t>(),
                     w.part_fine.as<uint16_t>(), w.bin_base.as<uint32_t>(), d, w.big_tiles.as<uint32_t>(),
                     w.cursor.as<uint32_t>(), w.sorted_entry.as<uint32_t>());
  mark(PH_FINE);
  }
  if (parts & PART_ACC) {
  hipLaunchKernelGGL(k_accumulate, dim3(rgrid), dim3(ACC_THREADS), 0, s, w.pts.as<uint32_t>(),
                     w.sorted_entry.as<uint32_t>(), w.bucket_start.as<uint32_t>(), w.run_key.as<uint32_t>(), total,
                     pl.K, d.W * d.B, w.buckets.as<uint32_t>(), w.lead_val.as<uint32_t>(), w.lead_open.as<uint32_t>(),
                     w.cross_key.as<uint32_t>(), w.skew_list.as<uint32_t>(), w.g_head.as<uint32_t>(),
                     w.g_hkey.as<uint32_t>(), w.g_tkey.as<uint32_t>());
  mark(PH_ACCUM);
  }
  if (parts & PART_POST) {
  hipLaunchKernelGGL(k_chain_join, dim3(CJ_GRID), dim3(ACC_THREADS), 0, s, w.skew_list.as<uint32_t>(), total, pl.K,
                     w.g_head.as<uint32_t>(), w.g_hkey.as<uint32_t>(), w.g_tkey.as<uint32_t>(),
                     w.buckets.as<uint32_t>(), w.lead_val.as<uint32_t>(), w.lead_open.as<uint32_t>(),
                     w.lead_flag.as<uint32_t>());
  hipLaunchKernelGGL(k_lead_scan, dim3(1), dim3(LS_THREADS), 0, s, w.lead_val.as<uint32_t>(),
                     w.lead_open.as<uint32_t>(), w.lead_flag.as<uint32_t>(), total, pl.K);
  mark(PH_FIXUP);
  hipLaunchKernelGGL(pl.L == 4 ? k_bucket_reduce_1<4> : pl.L == 16 ? k_bucket_reduce_1<16> : k_bucket_reduce_1<8>,
                     dim3(grid_for((size_t)d.W * pl.nchunks, RED1_THREADS)), dim3(RED1_THREADS), 0, s, w.buckets.as<uint32_t>(),
                     w.bucket_start.as<uint32_t>(), d, pl.K, w.cross_key.as<uint32_t>(), w.lead_val.as<uint32_t>(),
                     w.red_U.as<uint32_t>(), w.red_T.as<uint32_t>());
  mark(PH_RED1);
  hipLaunchKernelGGL(k_bucket_reduce_2, dim3(d.W * pl.nterms), dim3(RED2_THREADS), 0, s, w.red_U.as<uint32_t>(),
                     w.red_T.as<uint32_t>(), pl.nchunks, pl.nv, pl.nterms, w.err.as<uint32_t>(),
                     w.lead_flag.as<uint32_t>(), w.skew_list.as<uint32_t>(), total,
                     reinterpret_cast<uint32_t*>(sl.h_out_dev));
  mark(PH_RED2);
  mark(PH_READBACK);
  }
  HIPCHECK(hipGetLastError());
  return MSM_OK;
}

// Host tail: MSM = sum_w 2^(c w) [ sum_v R_{w,v} + sum_k 2^(lgL + k) R_{w,k} ]  (Horner over bit
// positions).  Follows reduce_last (lib.rs:88-104) in role: doublings between windows, then
// into_affine.  The device already emitted the terms in this file's Montgomery form
// (fe_to_host_mont).  Runs of doublings skip T (pt_dbl_proj) except the one feeding an add.
Pt horner_tail(const Plan& pl, const uint32_t* terms, uint32_t m = 0) {
  const MsmDims& d = pl.d;
  terms += (size_t)m * d.Wm * pl.nterms * 32;  // MSM m's windows
  // terms in descending bit position: windows from the top, inside a window R_k from the top
  // down to the V slices (position 0)
  std::vector<uint32_t> pos, idx;
  pos.reserve((size_t)d.Wm * pl.nterms);
  idx.reserve((size_t)d.Wm * pl.nterms);
  for (int w = (int)d.Wm - 1; w >= 0; w--)
    for (int t = (int)pl.nterms - 1; t >= 0; t--) {
      const uint32_t i = (uint32_t)w * pl.nterms + (uint32_t)t;
      const uint32_t* o = terms + (size_t)i * 32;
      Fq X;
      memcpy(X.l, o, 32);
      if (fq_is_zero(X) && !memcmp(o + 8, o + 24, 32)) continue;  // identity: X = 0, Y = Z
      pos.push_back(win_off(d, (uint32_t)w) + ((uint32_t)t < pl.nv ? 0u : pl.lgL + ((uint32_t)t - pl.nv)));
      idx.push_back(i);
    }
  Pt acc = pt_identity();
  if (pos.empty()) return acc;
  for (size_t j = 0; j < pos.size(); j++) {
    const uint32_t* o = terms + (size_t)idx[j] * 32;
    Pt p;
    memcpy(p.X.l, o, 32);
    memcpy(p.Y.l, o + 8, 32);
    memcpy(p.T.l, o + 16, 32);
    memcpy(p.Z.l, o + 24, 32);
    // T of the sum is needed when another add follows at the same position, and for the final
    // result (msm_compute_partial returns X|Y|T|Z); a doubling next never reads it
    const bool want_t = j + 1 == pos.size() || pos[j + 1] == pos[j];
    acc = j == 0 ? p : pt_add(acc, p, want_t);
    const uint32_t next = j + 1 < pos.size() ? pos[j + 1] : 0u;
    if (pos[j] > next) acc = pt_dbl_n(acc, (int)(pos[j] - next));
  }
  return acc;
}

void pt_to_be_affine(const Pt& p, uint32_t out[16]) {
  uint64_t x[4], y[4];
  pt_to_affine_std(p, x, y);
  std_to_be_words(x, out);
  std_to_be_words(y, out + 8);
}
void pt_to_be_xyzt(const Pt& p, uint32_t out[32]) {
  uint64_t s[4];
  const Fq* f[4] = {&p.X, &p.Y, &p.T, &p.Z};
  for (int i = 0; i < 4; i++) {
    fq_to_std(*f[i], s);
    std_to_be_words(s, out + 8 * i);
  }
}
int pt_from_be_xyzt(const uint32_t in[32], Pt* p) {
  uint64_t s[4];
  Fq* f[4] = {&p->X, &p->Y, &p->T, &p->Z};
  for (int i = 0; i < 4; i++) {
    be_words_to_std(in + 8 * i, s);
    if (!std_lt_p(s)) return MSM_ERR_COORD_RANGE;
    *f[i] = fq_from_std(s);
  }
  return MSM_OK;
}

using clk = std::chrono::steady_clock;

bool graphs_enabled() {
  static const bool on = !getenv("MSM_NO_GRAPH");
  return on;
}

void drop_graphs(Slot& sl) {
  for (int i = 0; i < 3; i++) {
    if (sl.gexec[i]) hipGraphExecDestroy(sl.gexec[i]);
    if (sl.graph[i]) hipGraphDestroy(sl.graph[i]);
    sl.gexec[i] = nullptr;
    sl.graph[i] = nullptr;
  }
  sl.n_prep = sl.n_recode = nullptr;
  sl.g_pts = sl.g_sc = BatchPtrs{};
}

int capture(DevCtx* c, const Plan& pl, const BatchPtrs& d_points, const BatchPtrs& d_scalars, int si, hipStream_t s,
            int parts, hipGraph_t* gout, hipGraphExec_t* out) {
  hipGraph_t g = nullptr;
  if (hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal) != hipSuccess) return MSM_ERR_HIP;
  int rc = enqueue_msm(c, pl, d_points, d_scalars, si, s, parts);
  hipError_t e = hipStreamEndCapture(s, &g);
  if (rc != MSM_OK || e != hipSuccess || !g) {
    if (g) hipGraphDestroy(g);
    (void)hipGetLastError();
    return MSM_ERR_HIP;
  }
  e = hipGraphInstantiate(out, g, nullptr, nullptr, 0);
  if (e != hipSuccess) {
    hipGraphDestroy(g);
    *out = nullptr;
    (void)hipGetLastError();
    return MSM_ERR_HIP;
  }
  *gout = g;
  return MSM_OK;
}

// Find the input-reading kernel nodes of slot graph 0 so later launches can repoint them.
int find_input_nodes(Slot& sl) {
  size_t num = 0;
  if (hipGraphGetNodes(sl.graph[0], nullptr, &num) != hipSuccess || num == 0) return MSM_ERR_HIP;
  std::vector<hipGraphNode_t> nodes(num);
  if (hipGraphGetNodes(sl.graph[0], nodes.data(), &num) != hipSuccess) return MSM_ERR_HIP;
  const void* f_prep = reinterpret_cast<const void*>(&k_prepare_points);
  const void* f_rc16 = reinterpret_cast<const void*>(&k_recode_hist<uint16_t>);
  const void* f_rc32 = reinterpret_cast<const void*>(&k_recode_hist<uint32_t>);
  for (hipGraphNode_t nd : nodes) {
    hipGraphNodeType ty;
    if (hipGraphNodeGetType(nd, &ty) != hipSuccess || ty != hipGraphNodeTypeKernel) continue;
    hipKernelNodeParams kp{};
    if (hipGraphKernelNodeGetParams(nd, &kp) != hipSuccess) continue;
    if (kp.func == f_prep) {
      sl.n_prep = nd;
      sl.p_prep = kp;
    } else if (kp.func == f_rc16 || kp.func == f_rc32) {
      sl.n_recode = nd;
      sl.p_recode = kp;
    }
  }
  return sl.n_prep && sl.n_recode ? MSM_OK : MSM_ERR_HIP;
}

// Point the instantiated slot graph at new input buffers (kernel-node argument update, no
// re-capture).
int repoint_inputs(DevCtx* c, const Plan& pl, Slot& sl, const BatchPtrs& d_points, const BatchPtrs& d_scalars) {
  const MsmDims& d = pl.d;
  Workspace& w = sl.ws;
  BatchPtrs wire = d_points;
  uint32_t* ptsb = w.pts.as<uint32_t>();
  uint32_t n = d.n;
  uint32_t* err = w.err.as<uint32_t>();
  void* a_prep[] = {&wire, &ptsb, &n, &err};
  hipKernelNodeParams kp = sl.p_prep;
  kp.kernelParams = a_prep;
  kp.extra = nullptr;
  if (hipGraphExecKernelNodeSetParams(sl.gexec[0], sl.n_prep, &kp) != hipSuccess) return MSM_ERR_HIP;
  BatchPtrs scal = d_scalars;
  MsmDims dd = d;
  void* digits = w.digits.p;
  uint32_t* hist = w.hist_rows.as<uint32_t>();
  void* a_rc[] = {&scal, &dd, &digits, &hist};
  hipKernelNodeParams kr = sl.p_recode;
  kr.kernelParams = a_rc;
  kr.extra = nullptr;
  if (hipGraphExecKernelNodeSetParams(sl.gexec[0], sl.n_recode, &kr) != hipSuccess) return MSM_ERR_HIP;
  sl.g_pts = d_points;
  sl.g_sc = d_scalars;
  return MSM_OK;
}

// Enqueue one MSM in slot `si`.  The launch sequence of each slot is captured into HIP graphs and
// replayed (one hipGraphLaunch instead of ~14 enqueues); new input buffers only repoint two
// kernel nodes.  Profiling mode 1 launches eagerly with an event between every phase; mode 2
// brackets an eager k_accumulate launch with events, between two graphs (pre / post).  Captures
// only on the library's own stream (a caller's stream may be capturing or in use).
bool same_ptrs(const BatchPtrs& a, const BatchPtrs& b) { return memcmp(&a, &b, sizeof(BatchPtrs)) == 0; }

int launch_msm(DevCtx* c, const Plan& pl, const BatchPtrs& d_points, const BatchPtrs& d_scalars, int si, hipStream_t s,
               bool own_stream, bool bracket) {
  Slot& sl = c->slot[si];
  const int prof = bracket ? 2 : 0;
  const bool graphs = own_stream && c->graphs_ok && graphs_enabled() && c->profiling != 1;
  if (graphs) {
    Slot::GraphKey key{(size_t)pl.d.n, pl.d.c, pl.K, pl.d.nm, prof, g_alloc_gen};
    if (!(sl.gexec[0] && key == sl.gkey)) {
      drop_graphs(sl);
      int rc;
      if (prof == 2) {
        rc = capture(c, pl, d_points, d_scalars, si, s, PART_PRE, &sl.graph[0], &sl.gexec[0]);
        if (rc == MSM_OK) rc = capture(c, pl, d_points, d_scalars, si, s, PART_POST, &sl.graph[2], &sl.gexec[2]);
      } else {
        rc = capture(c, pl, d_points, d_scalars, si, s, PART_ALL, &sl.graph[0], &sl.gexec[0]);
      }
      if (rc == MSM_OK) rc = find_input_nodes(sl);
      if (rc != MSM_OK) {
        drop_graphs(sl);
        c->graphs_ok = false;  // capture unsupported here: stay eager
      } else {
        sl.gkey = key;
        sl.g_pts = d_points;
        sl.g_sc = d_scalars;
      }
    }
    if (c->graphs_ok && (!same_ptrs(sl.g_pts, d_points) || !same_ptrs(sl.g_sc, d_scalars)) &&
        repoint_inputs(c, pl, sl, d_points, d_scalars) != MSM_OK) {
      drop_graphs(sl);
      (void)hipGetLastError();
      c->graphs_ok = false;
    }
  }
  const bool use_graphs = graphs && c->graphs_ok;
  if (prof == 2) {
    HIPCHECK(hipEventRecord(sl.ev_start, s));
    if (use_graphs) {
      HIPCHECK(hipGraphLaunch(sl.gexec[0], s));
    } else if (int rc = enqueue_msm(c, pl, d_points, d_scalars, si, s, PART_PRE)) {
      return rc;
    }
    // k_accumulate itself is launched eagerly between its two events: a graph launch there would
    // put the graph's own launch latency inside the measured bracket
    HIPCHECK(hipEventRecord(sl.ev_acc0, s));
    if (int rc = enqueue_msm(c, pl, d_points, d_scalars, si, s, PART_ACC)) return rc;
    HIPCHECK(hipEventRecord(sl.ev_acc1, s));
    if (use_graphs) {
      HIPCHECK(hipGraphLaunch(sl.gexec[2], s));
    } else if (int rc = enqueue_msm(c, pl, d_points, d_scalars, si, s, PART_POST)) {
      return rc;
    }
    HIPCHECK(hipEventRecord(sl.ev_end, s));
    return MSM_OK;
  }
  if (use_graphs) {
    HIPCHECK(hipGraphLaunch(sl.gexec[0], s));
    return MSM_OK;
  }
  return enqueue_msm(c, pl, d_points, d_scalars, si, s, PART_ALL);
}

// Start one MSM (device-resident inputs) in slot `si`; returns once it is enqueued.
int submit_msm(DevCtx* c, const Plan& pl, const BatchPtrs& d_points, const BatchPtrs& d_scalars, int si,
               hipStream_t s) {
  Slot& sl = c->slot[si];
  sl.pl = pl;
  // profiling mode 2 brackets k_accumulate with events on every PROF_EVERY-th MSM only (each
  // bracket costs ~20 us of launch gaps); the mean over those is the reported duration
  sl.bracketed = c->profiling == 2 && (c->prof_seq++ % PROF_EVERY) == 0;
  int rc = launch_msm(c, pl, d_points, d_scalars, si, s, s == sl.stream, sl.bracketed);
  if (rc != MSM_OK) return rc;
  HIPCHECK(hipEventRecord(sl.ev_done, s));
  return MSM_OK;
}

// Wait for the MSM in slot `si` (spinning briefly: the result is usually due within a couple of
// milliseconds, and a blocking wait adds a wake-up latency) and take its window terms.  With
// `terms` the terms are copied out, so the slot can take its next MSM before the host tail runs
// (finish_terms); otherwise the host tail runs here, on the pinned buffer.
int finish_msm(DevCtx* c, int si, Pt* result, std::vector<uint32_t>* terms = nullptr) {
  Slot& sl = c->slot[si];
  const Plan& pl = sl.pl;
  const auto spin_until = clk::now() + std::chrono::milliseconds(50);
  hipError_t q;
  while ((q = hipEventQuery(sl.ev_done)) == hipErrorNotReady && clk::now() < spin_until) _mm_pause();
  if (q == hipErrorNotReady) q = hipEventSynchronize(sl.ev_done);
  HIPCHECK(q);
  const size_t outb = (size_t)pl.d.W * pl.nterms * 32 * 4;
  const uint32_t* h = reinterpret_cast<const uint32_t*>(sl.h_out.p);
  uint32_t err = h[outb / 4];
  uint32_t total = h[outb / 4 + 1];
  if (err & MSM_DEV_ERR_COORD_RANGE) return MSM_ERR_COORD_RANGE;
  if (err & MSM_DEV_ERR_BAD_POINT) return MSM_ERR_BAD_POINT;
  auto t0 = clk::now();
  if (terms)
    terms->assign(h, h + outb / 4);
  else
    *result = horner_tail(pl, h);
  auto t1 = clk::now();
  if (c->profiling == 1 || (c->profiling == 2 && sl.bracketed)) {
    float ms[PH_COUNT] = {};
    msm_profile_t& P = c->last;
    if (c->profiling == 1) {
      for (int i = 1; i < PH_COUNT; i++) hipEventElapsedTime(&ms[i], c->ev[i - 1], c->ev[i]);
      hipEventElapsedTime(&P.device_total, c->ev[PH_START], c->ev[PH_READBACK]);
    } else {
      hipEventElapsedTime(&ms[PH_ACCUM], sl.ev_acc0, sl.ev_acc1);
      hipEventElapsedTime(&P.device_total, sl.ev_start, sl.ev_end);
    }
    P.prepare_points = ms[PH_PREPARE];
    P.recode_count = ms[PH_RECODE];
    P.coarse_scan = ms[PH_SCAN];
    P.coarse_scatter = ms[PH_SCATTER];
    P.fine_sort = ms[PH_FINE];
    P.accumulate = ms[PH_ACCUM];
    P.fixup = ms[PH_FIXUP];
    P.bucket_reduce_1 = ms[PH_RED1];
    P.bucket_reduce_2 = ms[PH_RED2];
    P.readback = ms[PH_READBACK];
    P.host_tail = std::chrono::duration<float, std::milli>(t1 - t0).count();
    P.entries = total;
    P.window_bits = pl.d.c;
    P.windows = pl.d.Wm;
    P.run_length = pl.K;
    P.chunk_len = pl.L;
    P.accumulate_sum += P.accumulate;
    P.device_total_sum += P.device_total;
    P.profiled++;
  }
  return MSM_OK;
}

// Run one MSM with device inputs; result as a projective host point.
int run_device(DevCtx* c, const uint32_t* d_points, const uint32_t* d_scalars, size_t n, const msm_opts* o,
               hipStream_t user_stream, Pt* result) {
  if (n == 0) {
    *result = pt_identity();
    return MSM_OK;
  }
  Plan pl;
  int rc = make_plan(n, o, c->n_cu, &pl);
  if (rc != MSM_OK) return rc;
  const int si = 0;  // a lone MSM always uses slot 0 (the other workspaces only for pipelining)
  if ((rc = ensure_workspace(c, pl, si)) != MSM_OK) return rc;
  hipStream_t s = user_stream ? user_stream : c->slot[si].stream;
  BatchPtrs bp{}, bs{};
  for (uint32_t m = 0; m < MSM_MAX_BATCH; m++) {
    bp.p[m] = d_points;
    bs.p[m] = d_scalars;
  }
  if ((rc = submit_msm(c, pl, bp, bs, si, s)) != MSM_OK) return rc;
  return finish_msm(c, si, result);
}

// MSMs kept in flight by the pipelined entries.  Small MSMs are latency-bound (their reduction
// and sort kernels leave most of the chip idle), so several run side by side; MSM_SLOTS
// overrides (1 = everything in order on one stream: clean per-kernel profiles).
int pipeline_slots(size_t n) {
  static const int env = getenv("MSM_SLOTS") ? atoi(getenv("MSM_SLOTS")) : 0;
  if (env >= 1) return std::min(env, NSLOT);
  (void)n;
  return 3;  // measured best at 2^16..2^20 (4 streams contend for the hardware queues)
}

// MSMs per launch (batch) for the pipelined entries: the latency-bound kernels (reduction trees,
// scans, small sorts) of two MSMs fill the machine together.  Measured on MI355X
// (tools/batch_sweep.sh, ms per MSM, batch 1 -> 2): 2^16 0.218 -> 0.162, 2^17 0.273 -> 0.247,
// 2^18 0.420 -> 0.381, 2^19 0.679 -> 0.638, 2^20 1.162 -> 1.136; 4 is no better than 2.
// MSM_BATCH overrides (1..MSM_MAX_BATCH).
uint32_t pipeline_batch(size_t n, size_t count) {
  static const int env = getenv("MSM_BATCH") ? atoi(getenv("MSM_BATCH")) : 0;
  uint32_t nm = env >= 1 ? (uint32_t)std::min(env, (int)MSM_MAX_BATCH) : (n <= (1u << 20) ? 2u : 1u);
  return (uint32_t)std::max<size_t>(1, std::min<size_t>(nm, count));
}

// `count` MSMs of n points each, pipelined over pipeline_slots(n) slots, each with its own stream
// and workspace, in launches of pipeline_batch MSMs (the last batch is padded by repeating its
// last MSM, whose extra results are dropped): later batches are enqueued before the host
// finishes batch j, so the host tail (window Horner) of one overlaps the device work of the
// next, and the batches' kernels may overlap on the device (the latency-bound reduction of one
// beside another's sort and accumulation).  With a caller-supplied stream everything runs in
// order on it.  Results go out affine (16 words each) or, with `projective`, as X|Y|T|Z
// partials (32 words).
int run_many(DevCtx* c, const uint32_t* const* d_points, const uint32_t* const* d_scalars, size_t n, size_t count,
             const msm_opts* o, hipStream_t user_stream, uint32_t* out_be, bool projective) {
  auto emit = [&](const Pt& r, size_t b) {
    if (projective)
      pt_to_be_xyzt(r, out_be + 32 * b);
    else
      pt_to_be_affine(r, out_be + 16 * b);
  };
  if (n == 0) {
    for (size_t b = 0; b < count; b++) emit(pt_identity(), b);
    return MSM_OK;
  }
  for (size_t b = 0; b < count; b++)
    if (!d_points[b] || !d_scalars[b]) return MSM_ERR_INVALID_ARG;
  const uint32_t nm = pipeline_batch(n, count);
  const size_t nbatch = (count + nm - 1) / nm;
  Plan pl;
  int rc = make_plan(n, o, c->n_cu, &pl, count > 1, nm);
  if (rc != MSM_OK) return rc;
  const int nslot = nbatch > 1 ? (int)std::min<size_t>(nbatch, (size_t)pipeline_slots(n)) : 1;
  for (int si = 0; si < nslot; si++)
    if ((rc = ensure_workspace(c, pl, si)) != MSM_OK) return rc;
  auto stream_of = [&](int si) { return user_stream ? user_stream : c->slot[si].stream; };
  // Batch j goes to slot j % nslot.  Its previous occupant, batch j - nslot, is waited for and
  // its window terms copied out just before; the host tail (window Horner) of batch j - nslot
  // runs after j is enqueued, so the device holds nslot batches while the host works
  // (otherwise batches that finish together leave the device idle for a Horner each).
  std::vector<uint32_t> terms;
  auto fail = [&](int code) {
    for (int k = 0; k < nslot; k++) hipStreamSynchronize(stream_of(k));
    return code;
  };
  for (size_t j = 0; j < nbatch + nslot; j++) {
    const bool have = j >= (size_t)nslot;
    const size_t f = have ? j - nslot : 0;
    if (have && (rc = finish_msm(c, (int)(f % nslot), nullptr, &terms)) != MSM_OK) return fail(rc);
    if (j < nbatch) {
      BatchPtrs bp{}, bs{};
      for (uint32_t m = 0; m < MSM_MAX_BATCH; m++) {
        const size_t b = std::min(j * nm + std::min<uint32_t>(m, nm - 1), count - 1);
        bp.p[m] = d_points[b];
        bs.p[m] = d_scalars[b];
      }
      const int si = (int)(j % nslot);
      if ((rc = submit_msm(c, pl, bp, bs, si, stream_of(si))) != MSM_OK) return fail(rc);
    }
    if (have)
      for (uint32_t m = 0; m < nm && f * nm + m < count; m++) emit(horner_tail(pl, terms.data(), m), f * nm + m);
  }
  return MSM_OK;
}

int with_device(const msm_opts* o, DevCtx** c) {
  int dev = o ? o->device : -1;
  return get_ctx(dev, c);
}

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    hipGetDevice(&prev);
    if (prev != dev) hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur;
    hipGetDevice(&cur);
    if (prev >= 0 && cur != prev) hipSetDevice(prev);
  }
};

int run_host(const uint32_t* points_be, const uint32_t* scalars_be, size_t n, const msm_opts* opts, Pt* result) {
  DevCtx* c;
  int rc = with_device(opts, &c);
  if (rc != MSM_OK) return rc;
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  if (n == 0) {
    *result = pt_identity();
    return MSM_OK;
  }
  if ((rc = c->wire_points.ensure(n * 128)) != MSM_OK) return rc;
  if ((rc = c->wire_scalars.ensure(n * 32)) != MSM_OK) return rc;
  HIPCHECK(hipMemcpyAsync(c->wire_points.p, points_be, n * 128, hipMemcpyHostToDevice, c->slot[0].stream));
  HIPCHECK(hipMemcpyAsync(c->wire_scalars.p, scalars_be, n * 32, hipMemcpyHostToDevice, c->slot[0].stream));
  return run_device(c, c->wire_points.as<uint32_t>(), c->wire_scalars.as<uint32_t>(), n, opts, nullptr, result);
}

}  // namespace

extern "C" {

int msm_init(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  return probe_devices() > 0 ? MSM_OK : MSM_ERR_NO_DEVICE;
}

void msm_shutdown(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  for (DevCtx* c : g_ctx) {
    if (!c) continue;
    std::lock_guard<std::mutex> lk2(c->mu);
    int prev = 0;
    hipGetDevice(&prev);
    hipSetDevice(c->device);
    for (Slot& sl : c->slot) hipStreamSynchronize(sl.stream);
    c->wire_points.release();
    c->wire_scalars.release();
    for (Slot& sl : c->slot) {
      sl.ws.release();
      drop_graphs(sl);
      sl.h_out.release();
      sl.h_out_dev = nullptr;
      for (hipEvent_t e : {sl.ev_start, sl.ev_acc0, sl.ev_acc1, sl.ev_end, sl.ev_done})
        if (e) hipEventDestroy(e);
    }
    for (int i = 0; i < PH_COUNT; i++) hipEventDestroy(c->ev[i]);
    for (Slot& sl : c->slot) hipStreamDestroy(sl.stream);
    hipSetDevice(prev);
  }
  for (DevCtx*& c : g_ctx) {
    delete c;
    c = nullptr;
  }
}

int msm_device_count(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  return probe_devices();
}

const char* msm_strerror(int code) {
  switch (code) {
    case MSM_OK: return "ok";
    case MSM_ERR_INVALID_ARG: return "invalid argument";
    case MSM_ERR_UNSUPPORTED_WINDOW: return "unsupported window size";
    case MSM_ERR_COORD_RANGE: return "coordinate not in [0, p)";
    case MSM_ERR_BAD_POINT: return "invalid point (z == 0)";
    case MSM_ERR_HIP: return "HIP runtime error";
    case MSM_ERR_NO_DEVICE: return "no gfx950 (MI355X) device available";
    case MSM_ERR_OOM: return "device out of memory";
    default: return "unknown error";
  }
}

uint32_t msm_best_window(size_t n) {
  // Measured on MI355X (tools/window_sweep.sh, balanced windows): c = 16 is fastest from 2^16 to
  // 2^20 -- the bucket reduction is latency-bound, so its cost hardly grows with 2^c, while
  // every extra window adds n entries and narrow windows make dense, chained buckets.  Below
  // that, keep ~8+ entries per bucket; the bucket tables (W * 2^(c-1) points) shrink with c.
  if (n >= (1u << 15)) return 16;
  uint32_t c = 8;
  while (c < 16 && (size_t)(1u << (c + 3)) <= n) c++;
  return c;
}

int msm_compute(const uint32_t* points_be, const uint32_t* scalars_be, size_t n, const msm_opts* opts,
                uint32_t out_xy_be[16]) {
  if ((!points_be || !scalars_be) && n) return MSM_ERR_INVALID_ARG;
  if (!out_xy_be) return MSM_ERR_INVALID_ARG;
  Pt r;
  int rc = run_host(points_be, scalars_be, n, opts, &r);
  if (rc != MSM_OK) return rc;
  pt_to_be_affine(r, out_xy_be);
  return MSM_OK;
}

int msm_compute_partial(const uint32_t* points_be, const uint32_t* scalars_be, size_t n, const msm_opts* opts,
                        uint32_t out_xyzt_be[32]) {
  if ((!points_be || !scalars_be) && n) return MSM_ERR_INVALID_ARG;
  if (!out_xyzt_be) return MSM_ERR_INVALID_ARG;
  Pt r;
  int rc = run_host(points_be, scalars_be, n, opts, &r);
  if (rc != MSM_OK) return rc;
  pt_to_be_xyzt(r, out_xyzt_be);
  return MSM_OK;
}

static int device_entry(const uint32_t* d_points_be, const uint32_t* d_scalars_be, size_t n, const msm_opts* opts,
                        void* hip_stream, Pt* r) {
  if ((!d_points_be || !d_scalars_be) && n) return MSM_ERR_INVALID_ARG;
  DevCtx* c;
  int rc = with_device(opts, &c);
  if (rc != MSM_OK) return rc;
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  return run_device(c, d_points_be, d_scalars_be, n, opts, (hipStream_t)hip_stream, r);
}

int msm_compute_device(const uint32_t* d_points_be, const uint32_t* d_scalars_be, size_t n, const msm_opts* opts,
                       void* hip_stream, uint32_t out_xy_be[16]) {
  if (!out_xy_be) return MSM_ERR_INVALID_ARG;
  Pt r;
  int rc = device_entry(d_points_be, d_scalars_be, n, opts, hip_stream, &r);
  if (rc != MSM_OK) return rc;
  pt_to_be_affine(r, out_xy_be);
  return MSM_OK;
}

int msm_compute_device_partial(const uint32_t* d_points_be, const uint32_t* d_scalars_be, size_t n,
                               const msm_opts* opts, void* hip_stream, uint32_t out_xyzt_be[32]) {
  if (!out_xyzt_be) return MSM_ERR_INVALID_ARG;
  Pt r;
  int rc = device_entry(d_points_be, d_scalars_be, n, opts, hip_stream, &r);
  if (rc != MSM_OK) return rc;
  pt_to_be_xyzt(r, out_xyzt_be);
  return MSM_OK;
}

int msm_compute_many_device(const uint32_t* const* d_points_be, const uint32_t* const* d_scalars_be, size_t n,
                            size_t count, const msm_opts* opts, void* hip_stream, uint32_t* out_xy_be) {
  if (!out_xy_be || ((!d_points_be || !d_scalars_be) && count)) return MSM_ERR_INVALID_ARG;
  if (count == 0) return MSM_OK;
  DevCtx* c;
  int rc = with_device(opts, &c);
  if (rc != MSM_OK) return rc;
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  return run_many(c, d_points_be, d_scalars_be, n, count, opts, (hipStream_t)hip_stream, out_xy_be, false);
}

int msm_compute_many_device_partial(const uint32_t* const* d_points_be, const uint32_t* const* d_scalars_be,
                                    size_t n, size_t count, const msm_opts* opts, void* hip_stream,
                                    uint32_t* out_xyzt_be) {
  if (!out_xyzt_be || ((!d_points_be || !d_scalars_be) && count)) return MSM_ERR_INVALID_ARG;
  if (count == 0) return MSM_OK;
  DevCtx* c;
  int rc = with_device(opts, &c);
  if (rc != MSM_OK) return rc;
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  return run_many(c, d_points_be, d_scalars_be, n, count, opts, (hipStream_t)hip_stream, out_xyzt_be, true);
}

int msm_compute_batch_device(const uint32_t* d_points_be, const uint32_t* d_scalars_be, size_t n, size_t count,
                             const msm_opts* opts, void* hip_stream, uint32_t* out_xy_be) {
  if (!out_xy_be || ((!d_points_be || !d_scalars_be) && n && count)) return MSM_ERR_INVALID_ARG;
  std::vector<const uint32_t*> pp(count), ss(count);
  for (size_t b = 0; b < count; b++) {
    pp[b] = d_points_be + b * n * 32;
    ss[b] = d_scalars_be + b * n * 8;
  }
  return msm_compute_many_device(pp.data(), ss.data(), n, count, opts, hip_stream, out_xy_be);
}

int msm_combine_partials(const uint32_t* partials_xyzt_be, size_t count, uint32_t out_xy_be[16]) {
  if ((!partials_xyzt_be && count) || !out_xy_be) return MSM_ERR_INVALID_ARG;
  Pt acc = pt_identity();
  for (size_t i = 0; i < count; i++) {
    Pt p;
    int rc = pt_from_be_xyzt(partials_xyzt_be + 32 * i, &p);
    if (rc != MSM_OK) return rc;
    if (fq_is_zero(p.Z)) return MSM_ERR_BAD_POINT;
    acc = pt_add(acc, p);
  }
  pt_to_be_affine(acc, out_xy_be);
  return MSM_OK;
}

int msm_point_add_affine(const uint32_t a_xy_be[16], const uint32_t b_xy_be[16], uint32_t out_xy_be[16]) {
  if (!a_xy_be || !b_xy_be || !out_xy_be) return MSM_ERR_INVALID_ARG;
  uint64_t ax[4], ay[4], bx[4], by[4];
  be_words_to_std(a_xy_be, ax);
  be_words_to_std(a_xy_be + 8, ay);
  be_words_to_std(b_xy_be, bx);
  be_words_to_std(b_xy_be + 8, by);
  if (!std_lt_p(ax) || !std_lt_p(ay) || !std_lt_p(bx) || !std_lt_p(by)) return MSM_ERR_COORD_RANGE;
  Pt r = pt_add(pt_from_affine_std(ax, ay), pt_from_affine_std(bx, by));
  pt_to_be_affine(r, out_xy_be);
  return MSM_OK;
}

uint32_t msm_split_windows(uint32_t window_bits) {
  if (window_bits == 0 || window_bits > 32) return 0;
  return (256 + window_bits - 1) / window_bits;
}

int msm_split(uint32_t c, const uint32_t* scalars_be, size_t n, uint32_t* out) {
  // Reference semantics (msm-macro/src/lib.rs:90-176): window i (0 = least significant) takes bits
  // [c*i, c*i + c) of the big-endian u32[8] scalar; output index j = n_windows - 1 - i (MSB first).
  if (c == 0 || c > 31) return MSM_ERR_UNSUPPORTED_WINDOW;
  if ((!scalars_be || !out) && n) return MSM_ERR_INVALID_ARG;
  const uint32_t nw = msm_split_windows(c);
  for (size_t s = 0; s < n; s++) {
    const uint32_t* be = scalars_be + 8 * s;
    for (uint32_t i = 0; i < nw; i++) {
      uint32_t bit = c * i, v = 0;
      for (uint32_t b = 0; b < c && bit + b < 256; b++) {
        uint32_t pos = bit + b;
        uint32_t word = be[7 - pos / 32];
        v |= ((word >> (pos % 32)) & 1u) << b;
      }
      out[(size_t)(nw - 1 - i) * n + s] = v;
    }
  }
  return MSM_OK;
}

int msm_set_profiling(int enable) {
  std::lock_guard<std::mutex> lk(g_mu);
  g_profiling = enable < 0 ? 0 : enable > 2 ? 1 : enable;
  for (DevCtx* c : g_ctx)
    if (c) {
      c->profiling = g_profiling;
      c->last.accumulate_sum = c->last.device_total_sum = 0;
      c->last.profiled = 0;
      c->prof_seq = 0;
    }
  return MSM_OK;
}

int msm_last_profile(msm_profile_t* out) {
  if (!out) return MSM_ERR_INVALID_ARG;
  DevCtx* c;
  int rc = get_ctx(-1, &c);
  if (rc != MSM_OK) return rc;
  std::lock_guard<std::mutex> lk(c->mu);
  *out = c->last;
  return MSM_OK;
}

int msm_gen_points(const uint32_t g_xy_be[16], uint64_t k0, uint64_t step, size_t n, uint32_t* points_be) {
  if (!g_xy_be || (!points_be && n)) return MSM_ERR_INVALID_ARG;
  uint64_t gx[4], gy[4];
  be_words_to_std(g_xy_be, gx);
  be_words_to_std(g_xy_be + 8, gy);
  if (!std_lt_p(gx) || !std_lt_p(gy)) return MSM_ERR_COORD_RANGE;
  gen_points(pt_from_affine_std(gx, gy), k0, step, n, points_be);
  return MSM_OK;
}

int msm_gen_scalars(uint64_t seed, size_t n, uint32_t* scalars_be) {
  if (!scalars_be && n) return MSM_ERR_INVALID_ARG;
  gen_scalars(seed, n, scalars_be);
  return MSM_OK;
}

// ---- test hooks (not in msm.h): batch field / point ops on the device, canonical LE words ----
int msm_test_field_op(uint32_t op, const uint32_t* a, const uint32_t* b, uint32_t* out, size_t n) {
  DevCtx* c;
  int rc = get_ctx(-1, &c);
  if (rc != MSM_OK) return rc;
  std::lock_guard<std::mutex> lk(c->mu);
  uint32_t *da, *db, *dout;
  HIPCHECK(hipMalloc(&da, n * 32 + 32));
  HIPCHECK(hipMalloc(&db, n * 32 + 32));
  HIPCHECK(hipMalloc(&dout, n * 32 + 32));
  HIPCHECK(hipMemcpy(da, a, n * 32, hipMemcpyHostToDevice));
  HIPCHECK(hipMemcpy(db, b, n * 32, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_test_field, dim3(grid_for(n, 256)), dim3(256), 0, 0, da, db, dout, (uint32_t)n, op);
  HIPCHECK(hipGetLastError());
  HIPCHECK(hipMemcpy(out, dout, n * 32, hipMemcpyDeviceToHost));
  hipFree(da);
  hipFree(db);
  hipFree(dout);
  return MSM_OK;
}

int msm_test_point_op(uint32_t op, const uint32_t* p, const uint32_t* q, uint32_t* out, size_t n) {
  DevCtx* c;
  int rc = get_ctx(-1, &c);
  if (rc != MSM_OK) return rc;
  std::lock_guard<std::mutex> lk(c->mu);
  uint32_t *dp, *dq, *dout;
  HIPCHECK(hipMalloc(&dp, n * 64 + 64));
  HIPCHECK(hipMalloc(&dq, n * 64 + 64));
  HIPCHECK(hipMalloc(&dout, n * 128 + 128));
  HIPCHECK(hipMemcpy(dp, p, n * 64, hipMemcpyHostToDevice));
  HIPCHECK(hipMemcpy(dq, q, n * 64, hipMemcpyHostToDevice));
  if (op == 3)
    hipLaunchKernelGGL(k_test_quad, dim3(grid_for(4 * n, 256)), dim3(256), 0, 0, dp, dq, dout, (uint32_t)n);
  else if (op == 0)
    hipLaunchKernelGGL(k_test_point<0>, dim3(grid_for(n, 256)), dim3(256), 0, 0, dp, dq, dout, (uint32_t)n);
  else if (op == 1)
    hipLaunchKernelGGL(k_test_point<1>, dim3(grid_for(n, 256)), dim3(256), 0, 0, dp, dq, dout, (uint32_t)n);
  else
    hipLaunchKernelGGL(k_test_point<2>, dim3(grid_for(n, 256)), dim3(256), 0, 0, dp, dq, dout, (uint32_t)n);
  HIPCHECK(hipGetLastError());
  HIPCHECK(hipMemcpy(out, dout, n * 128, hipMemcpyDeviceToHost));
  hipFree(dp);
  hipFree(dq);
  hipFree(dout);
  return MSM_OK;
}

}  // extern "C"
