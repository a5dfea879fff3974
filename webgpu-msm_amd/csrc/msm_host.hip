// libmsm host driver: C ABI (include/msm.h), device workspaces, launch sequence, host tail.
//
// The reference's host orchestration this replaces:
//   compute_msm            src/submission/submission.ts:25-157   -> msm_compute / msm_compute_device
//   getBestWindowSize      submission.ts:18-23                    -> msm_best_window
//   gpuIntraBucketReduction src/submission/gpu.ts:36-285          -> k_prepare_points .. k_lead_scan
//     (its staging ring, gpu.ts:146-155 / 244-271)                -> the packed pinned ring (PinRing,
//                                                                    PackPool) and the uploader thread
//   split_dynamic          msm-wasm/src/lib.rs:196-202            -> msm_split (host) / k_recode_* (device)
//   inter_bucket_reduce    lib.rs:46-56, 123-133                  -> k_bucket_reduce_1, k_red2_groups / _terms
//   reduce_last            lib.rs:88-104                          -> horner_tail (host)
//   point_add_affine       lib.rs:240-253                         -> msm_point_add_affine
//   msm_end_to_end         lib.rs:24-44, 106-121                  -> msm_compute_cpu (msm_cpu.h)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include <immintrin.h>

#include "../../include/msm.h"
#include "hostfield.h"
#include "msm_cpu.h"
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

// Bumped on every (re)allocation anywhere: captured graphs hold raw pointers, so a graph is
// replayed only while the generation it was captured under is current.
std::atomic<uint64_t> g_alloc_gen{0};

struct Buf {
  void* p = nullptr;
  size_t cap = 0;
  int ensure(size_t bytes) {
    if (bytes <= cap) return MSM_OK;
    g_alloc_gen.fetch_add(1);
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
    g_alloc_gen.fetch_add(1);
    if (p) hipHostFree(p);
    p = nullptr;
    cap = 0;
    // pinned, host-cacheable memory; k_red2_terms (or k_bucket_reduce_2) writes its results
    // straight into it, visible to the host once the launch's event completes (a coherent /
    // uncached mapping would make the host Horner's reads ~4x slower)
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
  uint32_t L;       // bucket-reduce chunk length (any of RED1_LS; not necessarily a power of two)
  uint32_t nchunks; // ceil(B / L)
  uint32_t nv;      // V-slices: R_V = sum_c U_c is split into nv equal partial sums
  uint32_t nterms;  // nv + bits of the largest chunk index
  size_t Mmax;      // W * n upper bound on sorted entries
  size_t runs_max;
  uint32_t pfmt;    // input point format of k_prepare_points (PT_FMT_*: wire records or a compact upload)
};

// Every field that shapes a launch (grids, buffer offsets, the h_out layout): a captured graph is
// replayed only for an identical plan.
bool plan_eq(const Plan& a, const Plan& b) {
  const MsmDims &x = a.d, &y = b.d;
  return x.n == y.n && x.c == y.c && x.B == y.B && x.W == y.W && x.Wm == y.Wm && x.w0 == y.w0 && x.Wr == y.Wr &&
         x.half_lo == y.half_lo && x.half_hi == y.half_hi &&
         x.nm == y.nm && x.q == y.q &&
         x.nhi == y.nhi && x.fb == y.fb && x.nbc == y.nbc && x.nbins == y.nbins && x.ch == y.ch && x.nch == y.nch &&
         x.packed == y.packed && x.shared == y.shared && a.K == b.K && a.L == b.L &&
         a.nchunks == b.nchunks && a.nv == b.nv && a.nterms == b.nterms && a.Mmax == b.Mmax &&
         a.runs_max == b.runs_max && a.pfmt == b.pfmt;
}

// Device workspace of one MSM (all sizes from Plan; grown on demand, never shrunk).
struct Workspace {
  Buf pts, err, digits, colsum, bin_base, bin_cur;
  Buf part_entry, part_fine, sorted_entry, bucket_start, run_key, buckets;
  Buf lead_val, lead_open, cross_key, lead_flag, skew_list, g_head, g_hkey, g_tkey, red_U, red_T;
  Buf wire_pts, wire_sc;  // device copies of host-resident inputs (msm_compute*, host entries)
  Buf red_G;               // k_red2_groups' points per (window, group of RG_CH chunks)
#ifdef MSM_DUMMY_ALLOC
  Buf dummy_tiles, dummy_cursor;  // tuning builds: the round-5 allocation layout
#endif
  void release() {
    Buf* bufs[] = {&pts, &err, &digits, &colsum, &bin_base, &bin_cur, &part_entry, &part_fine,
                   &sorted_entry, &bucket_start, &run_key, &buckets, &lead_val, &lead_open, &cross_key,
                   &lead_flag, &skew_list, &g_head, &g_hkey, &g_tkey, &red_U, &red_T, &wire_pts, &wire_sc, &red_G};
    for (Buf* b : bufs) b->release();
  }
};

// Launch-sequence parts.  PREP: wire points -> precomputed records; SORT: scalar recoding and the
// bucket sort; ACC: bucket accumulation; POST: the bucket reduction; JOIN: the joins of skewed
// buckets (k_chain_join, k_lead_scan).  The regular sequence (PART_ALL) leaves JOIN out: with
// unskewed scalars both kernels would do nothing, yet each costs ~5 us of the critical path.
// k_accumulate flags skew, k_bucket_reduce_2 reports it with the terms, and finish_msm then runs
// JOIN + POST again on the slot (the order of the original sequence; nothing they read was
// changed by the first reduction).
constexpr int PART_PREP = 1, PART_SORT = 2, PART_ACC = 4, PART_POST = 8, PART_ALL = 15, PART_JOIN = 16;

// One captured graph of a slot: a contiguous part of the launch sequence for one plan.
struct Segment {
  Plan pl{};
  int parts = 0;
  const uint32_t* pts_buf = nullptr;  // the point-record buffer the captured kernels use
  int acc_events = 0;                 // event-record nodes: 2 around k_accumulate, 1 after it only
  bool fork = false;                  // the preparation forked beside the sort (slot_forks)
  uint64_t gen = 0;
  uint64_t used = 0;
  hipGraph_t graph = nullptr;
  hipGraphExec_t exec = nullptr;
  // the kernel nodes that take the MSM's input buffers: repointed per launch
  hipGraphNode_t n_prep = nullptr, n_recode = nullptr;
  hipKernelNodeParams p_prep{}, p_recode{};
  BatchPtrs in_pts{}, in_sc{};
  void drop() {
    if (exec) hipGraphExecDestroy(exec);
    if (graph) hipGraphDestroy(graph);
    exec = nullptr;
    graph = nullptr;
    n_prep = n_recode = nullptr;
    parts = 0;
  }
};
constexpr int NSEG = 6;

// One in-flight launch (one or a batch of MSMs): its own stream, device workspace, result buffer,
// captured graph segments and events.  Several slots let the pipelined entries keep launches
// j+1.. on the device while launch j is still there (the latency-bound tails of one overlap the
// others' kernels) and while the host finishes launch j (window Horner).
struct Slot {
  hipStream_t stream = nullptr;
  // k_prepare_points forks onto aux (ev_fork) and rejoins before the accumulation (ev_join): the
  // point preparation (HBM streaming) runs beside the bucket sort (the scalars' kernels)
  hipStream_t aux = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  Workspace ws;
  HostBuf h_out;  // k_bucket_reduce_2 writes the window terms, err and total here
  void* h_out_dev = nullptr;
  Segment seg[NSEG];
  uint64_t seg_clock = 0;
  hipEvent_t ev_start = nullptr, ev_acc0 = nullptr, ev_acc1 = nullptr, ev_end = nullptr, ev_done = nullptr;
  hipEvent_t ev_in = nullptr;  // inputs of the slot's next launch are in place (uploads, caller's stream)
  hipEvent_t ev_sc = nullptr;  // the scalars of the slot's next launch are in place (host uploads)
  Plan pl{};
  bool acc_timed = false;
  bool stagger = false;  // this slot's pipelined launches are staggered (stagger_launches)
  bool pipelined = false;  // a launch of a pipelined run (another launch in flight beside it)
};
constexpr int NSLOT = 4;      // at most this many launches in flight (one HIP stream each)
constexpr int NCHUNK_EV = 8;  // events marking uploaded point chunks

class TailCrew;
class HornerPool;
class PackPool;

// Pinned staging buffers of the packed host upload (run_host_split with host_pack()): the
// library's own threads write compacted points (and the scalars) into them, the copy engine
// reads them (a DMA from pinned memory needs no staging by the runtime), each buffer reused once
// the copy out of it has completed (ev).
constexpr int NPIN = 3;
struct PinRing {
  HostBuf buf[NPIN];
  hipEvent_t ev[NPIN] = {};
  bool used[NPIN] = {};
};

// What the launch plans take from the device: compute units, and k_accumulate's waves per SIMD
// (the occupancy query at context creation; run_length_for fills whole rounds of them).  The test
// hooks plan for the defaults, so their plans do not depend on which device was used first.
struct DevShape {
  int n_cu = 256;
  int acc_waves = 4;
};

struct DevCtx {
  int device = -1;
  DevShape shape;
  std::mutex mu;
  Slot slot[NSLOT];
  hipStream_t copy_stream = nullptr;  // host->device uploads (overlap the slots' kernels)
  hipEvent_t ev_chunk[NCHUNK_EV] = {};
  hipEvent_t ev_user = nullptr;  // recorded on a caller's stream: the library's streams wait on it
  hipEvent_t ev_shared = nullptr;
  Buf shared_pts;  // point records of a shared base vector (msm_compute_shared*)
  Buf host_sc;     // all the scalars of a split host-input MSM (run_host_split), uploaded first
  Buf host_pts;    // and all its points, slice by slice (no slot buffer reused within the call)
  PinRing pin;     // pinned staging of the packed host upload
  PackPool* packer = nullptr;  // its packing threads (persistent, created on first use)
  hipEvent_t ev[PH_COUNT] = {};  // per-phase events (profiling mode 1)
  int profiling = 0;  // 0 off, 1 every phase (eager launches), 2 k_accumulate + device total per launch
  // The launch sequence of each slot is captured into HIP graphs and replayed: one
  // hipGraphLaunch instead of ~14 enqueues per launch.
  bool graphs_ok = true;
  bool graph_events_ok = true;  // event-record nodes can be added to captured graphs here
  hipEvent_t ev_base = nullptr;  // per-call time origin of the accumulation intervals (profiling 2)
  std::vector<std::pair<float, float>> acc_ivals;
  msm_profile_t last{};
  TailCrew* crew = nullptr;  // a lone MSM's host-tail helpers (persistent, created on first use)
  HornerPool* pool = nullptr;  // the pipelined entries' host tails, off the launching thread
  // per-launch upload events of a host-input pipelined run (launch j: up_ev[2 j] its scalars,
  // up_ev[2 j + 1] all its inputs), grown on demand
  std::vector<hipEvent_t> up_ev;
};

std::mutex g_mu;
std::vector<DevCtx*> g_ctx;   // indexed by HIP ordinal
std::vector<int> g_gfx950;    // HIP ordinals of the gfx950 devices
int g_nhip = -1;              // HIP devices visible (any architecture)
std::atomic<int> g_profiling{0};  // read by calls on other devices' threads

int probe_devices() {
  if (g_nhip >= 0) return (int)g_gfx950.size();
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
  g_nhip = n;
  for (int i = 0; i < n; i++) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, i) == hipSuccess && strncmp(prop.gcnArchName, "gfx950", 6) == 0)
      g_gfx950.push_back(i);
  }
  return (int)g_gfx950.size();
}

bool is_gfx950(int device) { return std::find(g_gfx950.begin(), g_gfx950.end(), device) != g_gfx950.end(); }

int get_ctx(int device, DevCtx** out) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (probe_devices() <= 0) return MSM_ERR_NO_DEVICE;
  if (device < 0) {
    if (hipGetDevice(&device) != hipSuccess) return MSM_ERR_HIP;
  }
  // opts.device is a HIP ordinal; only gfx950 ordinals are accepted (a mixed node keeps its
  // numbering)
  if (device >= g_nhip || !is_gfx950(device)) return MSM_ERR_INVALID_ARG;
  if ((int)g_ctx.size() < g_nhip) g_ctx.resize(g_nhip, nullptr);
  if (!g_ctx[device]) {
    DevCtx* c = new DevCtx();
    c->device = device;
    int prev = 0;
    hipGetDevice(&prev);
    if (hipSetDevice(device) != hipSuccess) {
      delete c;
      return MSM_ERR_HIP;
    }
    // Streams in this order because the runtime deals them round-robin over its hardware queues
    // (GPU_MAX_HW_QUEUES, 4 by default) and two streams on one queue run in order: the slots'
    // streams first, so the launches in flight never share a queue (three slots for host inputs
    // beside the copy stream), then the aux streams of the preparation fork.
    bool ok = hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking) == hipSuccess;
    for (Slot& sl : c->slot) ok = ok && hipStreamCreateWithFlags(&sl.stream, hipStreamNonBlocking) == hipSuccess;
    for (Slot& sl : c->slot) ok = ok && hipStreamCreateWithFlags(&sl.aux, hipStreamNonBlocking) == hipSuccess;
    auto ev = [&](hipEvent_t* e, bool timed) {
      ok = ok && (timed ? hipEventCreate(e) : hipEventCreateWithFlags(e, hipEventDisableTiming)) == hipSuccess;
    };
    for (int i = 0; i < PH_COUNT; i++) ev(&c->ev[i], true);
    for (int i = 0; i < NCHUNK_EV; i++) ev(&c->ev_chunk[i], false);
    ev(&c->ev_user, false);
    ev(&c->ev_shared, false);
    ev(&c->ev_base, true);
    for (Slot& sl : c->slot) {
      ev(&sl.ev_start, true);
      ev(&sl.ev_acc0, true);
      ev(&sl.ev_acc1, true);
      ev(&sl.ev_end, true);
      ev(&sl.ev_done, false);
      ev(&sl.ev_in, false);
      ev(&sl.ev_sc, false);
      ev(&sl.ev_fork, false);
      ev(&sl.ev_join, false);
    }
    if (!ok) {  // no context without its streams and events (a null event would fail every call later)
      delete c;
      hipSetDevice(prev);
      return MSM_ERR_HIP;
    }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
      c->shape.n_cu = prop.multiProcessorCount;
    int acc_blocks = 0;  // k_accumulate workgroups per CU -> waves per SIMD (run_length_for)
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&acc_blocks, reinterpret_cast<const void*>(&k_accumulate),
                                                     ACC_THREADS, 0) == hipSuccess &&
        acc_blocks > 0)
      c->shape.acc_waves = std::max(1, acc_blocks * (int)(ACC_THREADS / 64) / 4);
    hipSetDevice(prev);
    g_ctx[device] = c;
  }
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
// so sub-2^20 sizes prefer narrower windows.  Measured on MI355X (tools/window_sweep.sh; round 2
// re-check with the current launch plan, profiles/r2ab_window_ab.jsonl): c = 14 at 2^16, 15 at
// 2^17..2^18, 16 from 2^19 (2^19: 0.584-0.592 vs 0.604-0.614 ms at c = 15).
uint32_t pipelined_window(size_t n) {
  // c = 16 from 7/8 of 2^19: 2^19 - 1 points ran 0.571-0.576 ms at c = 16 against 0.619-0.621 at
  // c = 15, 3/4 of 2^19 0.451-0.454 at c = 15 against 0.457-0.469 (tools/window_boundary_probe.sh)
  if (n >= (7u << 16)) return 16;
  if (n >= (1u << 17)) return 15;
  if (n >= (1u << 15)) return 14;
  return msm_best_window(n);
}

// Chunk lengths k_bucket_reduce_1 is instantiated for.
constexpr uint32_t RED1_LS[] = {8, 9, 10, 12, 16, 17, 20};

// Buckets per k_bucket_reduce_1 lane: the shortest chain (L) for which the live lanes of every
// MSM's main windows fit in one wave per SIMD (see msm_kernels.hip); 16 if none does.  Measured
// (profiles/r2i_ks17*): c = 15 with two MSMs per launch ran L = 8 as 1,056 waves -- two chains on
// some SIMDs, 140 us -- where L = 9 fits.  Chains past 16 serve the four-MSM launches of small
// sizes (2^17: L = 17, 994 waves).  MSM_RED_L overrides (any of RED1_LS, or 4).
uint32_t bucket_reduce_L(const MsmDims& d, const DevShape& sh) {
  const int n_cu = sh.n_cu;
  static const uint32_t l_env = getenv("MSM_RED_L") ? (uint32_t)atoi(getenv("MSM_RED_L")) : 0u;
  if (l_env == 4) return 4;
  for (uint32_t L : RED1_LS)
    if (l_env == L) return L;
  const uint64_t simds = 4ull * (uint64_t)(n_cu > 0 ? n_cu : 256);
  for (uint32_t L : RED1_LS) {
    const uint32_t nchunks = (d.B + L - 1) / L;
    uint64_t lanes = 0;
    for (uint32_t l = 0; l < d.Wr; l++) lanes += red1_live_chunks(d, L, nchunks, d.w0 + l);
    lanes *= d.nm;
    if ((lanes + 63) / 64 <= simds) return L;
  }
  return 16;
}

// The shortest run length that keeps random scalars off the skew joins.  A bucket that holds
// three whole runs (3 K + 2 entries or more) sends its workgroup to k_chain_join, and the launch
// through a second reduction (~0.25 ms at 2^20: DESIGN.md §2.4).  The largest buckets are the top
// main window's: its digits only reach p >> offset (p < 2^253; 9,551 values at c = 16), so at 2^20
// they hold ~110 entries each, against 32-64 in the other windows.  K is sized for the largest
// expected bucket of the launch's range, lambda + 5 sqrt(lambda) + 2 entries (Poisson, uniform
// scalars mod p).  This is what made 2^20 + 1 points 14% slower than 2^20 (round 4): K = 44 there,
// so a top-window bucket of ~134+ entries (one in ~10^4) held three runs in every launch.
uint32_t run_length_skew_floor(const MsmDims& d) {
  double lam_max = 0;
  for (uint32_t l = 0; l < d.Wr; l++) {
    const uint32_t w = d.w0 + l;
    if (w + 1 >= d.Wm) continue;  // the overflow window: empty for canonical scalars
    double vals = (double)(1u << (win_bits(d, w) - 1));
    if (w + 2 == d.Wm) {  // the top main window: digits below (p >> off) + 1
      const uint32_t off = win_off(d, w);
      const double top = off >= 192 ? (double)(P[3] >> (off - 192)) + 1.0 : vals;
      vals = std::min(vals, top);
    }
    lam_max = std::max(lam_max, (double)d.n / vals);
  }
  const double maxb = lam_max + 5.0 * std::sqrt(lam_max) + 2.0;
  const uint32_t k = (uint32_t)std::floor((maxb - 2.0) / 3.0) + 1;  // 3 K + 2 > maxb
  return (k + 3) & ~3u;
}

// Run length K (entries per k_accumulate lane, a multiple of 4 for the 16-B entry loads): the
// accumulation holds sh.acc_waves waves per SIMD (4: VGPR- and LDS-bound, from the runtime's
// occupancy query for the device), so its lanes run in rounds of that many x 4 x CUs waves.
// - A launch under one round at K = 64 takes the smallest K that fills the round (2^17, four MSMs:
//   K = 36, 3,868 waves, where K = 32 needed 4,352: a 6% second round that runs on few SIMDs).
// - Pipelined launches past one round take the K of whole rounds (2^20, two MSMs: K = 64, two
//   rounds) unless that K is under the skew floor: then K = 64 (or the floor), and the next
//   launch's kernels fill whatever a short last round leaves idle.  2^20 + 1 points, two MSMs:
//   1.030 ms per MSM at K = 64 against 1.062 at K = 68 (two rounds) and 1.170 at the balanced
//   K = 44 (skew joins) (profiles/r5/run_length.jsonl).
// - A lone MSM past one round (its latency counts, and nothing fills its tail) takes the K up to
//   128 whose whole rounds cost least (rounds x K): 2^20 + 1 points run one round of K = 68.
// K never drops below run_length_skew_floor.  (Upper bound of the entries: every main-window
// digit nonzero.)
uint32_t run_length_for(const MsmDims& d, const DevShape& sh, bool pipelined) {
  // main windows of the launch's range (the overflow window holds no entry for canonical scalars)
  const uint64_t nmain = d.Wr - ((d.w0 + d.Wr == d.Wm) ? 1u : 0u);
  const uint64_t m = (uint64_t)d.nm * std::max<uint64_t>(1, nmain) * d.n;
  const uint64_t round_lanes =
      64ull * (uint64_t)std::max(1, sh.acc_waves) * 4 * (uint64_t)(sh.n_cu > 0 ? sh.n_cu : 256);
  const uint64_t kfloor = std::max<uint64_t>(16, run_length_skew_floor(d));
  const uint64_t r64 = std::max<uint64_t>(1, (m + 64 * round_lanes - 1) / (64 * round_lanes));
  uint64_t K;
  if (r64 == 1) {
    K = (m + round_lanes - 1) / round_lanes;  // one round
  } else if (pipelined) {
    // whole rounds of a shorter K where that clears the skew floor (2^18, four MSMs: K = 36,
    // 0.332-0.337 ms per MSM against 0.340-0.342 at K = 64), else K = 64
    K = (m + r64 * round_lanes - 1) / (r64 * round_lanes);
    K = (K + 3) & ~3ull;
    if (K < kfloor) K = std::max<uint64_t>(64, kfloor);
  } else {
    uint64_t best = ~0ull;
    K = 64;
    for (uint64_t k = 16; k <= 128; k += 4) {
      if (k < kfloor) continue;
      const uint64_t cost = (m + k * round_lanes - 1) / (k * round_lanes) * k;
      if (cost < best) best = cost, K = k;
    }
  }
  K = (K + 3) & ~3ull;
  return (uint32_t)std::min<uint64_t>(4096, std::max<uint64_t>(kfloor, K));
}

int finish_plan(const MsmDims& d, const msm_opts* o, const DevShape& sh, Plan* pl, bool pipelined = false);

int make_plan(size_t n, const msm_opts* o, const DevShape& sh, Plan* pl, bool pipelined = false, uint32_t nm = 1,
              bool shared = false) {
  *pl = Plan{};
  uint32_t c = (o && o->window_bits) ? o->window_bits : pipelined ? pipelined_window(n) : msm_best_window(n);
  if (c < 4 || c > 20) return MSM_ERR_UNSUPPORTED_WINDOW;
  if (n >= (1ull << 30)) return MSM_ERR_INVALID_ARG;
  MsmDims d{};
  d.n = (uint32_t)n;
  d.c = c;
  // balanced main windows of at most c bits over MAIN_BITS, plus the overflow window
  const uint32_t wm = (MAIN_BITS + c - 1) / c;
  d.q = MAIN_BITS / wm;
  d.nhi = MAIN_BITS - d.q * wm;
  d.Wm = wm + 1;
  d.nm = nm;
  d.w0 = 0;
  d.Wr = d.Wm;
  d.half_lo = d.half_hi = 0;
  if (o && (o->flags & MSM_FLAG_WINDOWS)) {
    // a window range needs an explicit width, so that every caller's ranges cut the same windows
    const uint32_t units = (o->flags & MSM_FLAG_HALF_WINDOWS) ? 2u : 1u;
    if (!o->window_bits || o->window_lo >= o->window_hi || o->window_hi > units * d.Wm) return MSM_ERR_INVALID_ARG;
    d.w0 = o->window_lo / units;
    d.Wr = (o->window_hi + units - 1) / units - d.w0;
    if (units == 2) {
      d.half_lo = o->window_lo & 1u;  // starts at window w0's upper half
      d.half_hi = o->window_hi & 1u;  // ends after window w0 + Wr - 1's lower half
    }
  }
  d.W = d.Wr * nm;
  d.c = d.nhi ? d.q + 1 : d.q;
  d.B = 1u << (d.c - 1);
  // Coarse bins: aim at ~4K entries per bin (half the LDS staging capacity of k_fine_sort) with at
  // most FS_MAXF buckets per bin.  Partition chunks hold >= 64 entries per bin slice.
  uint32_t nbc = 1;
  while (nbc < d.B && nbc < 256 && (size_t)nbc * 4096 < n) nbc <<= 1;
  while (nbc < d.B && (d.B / nbc) > FS_MAXF) nbc <<= 1;
  d.nbc = nbc;
  d.fb = ilog2(d.B / nbc);
  d.shared = shared ? 1u : 0u;
  const uint64_t npts = shared ? n : (uint64_t)nm * n;  // point records the entries index
  d.packed = npts <= (1ull << (31 - d.fb)) ? 1u : 0u;
  d.nbins = d.W * d.nbc;
  d.ch = PT_THREADS * PS_R;  // 16384 digits per partition chunk (>= 64 per bin slice while nbc <= 256)
  d.nch = (uint32_t)((n + d.ch - 1) / d.ch);
  return finish_plan(d, o, sh, pl, pipelined);
}

// The launch-shape fields that follow from the geometry d.
int finish_plan(const MsmDims& d, const msm_opts* o, const DevShape& sh, Plan* pl, bool pipelined) {
  const size_t n = d.n;
  pl->d = d;
  pl->K = (o && o->run_length) ? o->run_length : run_length_for(d, sh, pipelined);
  if (pl->K < 1 || pl->K > 4096) return MSM_ERR_INVALID_ARG;
  pl->L = bucket_reduce_L(d, sh);
  pl->nchunks = (d.B + pl->L - 1) / pl->L;
  // every k_bucket_reduce_2 workgroup sums at most pow2ceil(nchunks)/2 points (the R_k terms' size)
  pl->nv = pl->nchunks >= 2 ? 2 : 1;
  uint32_t cbits = 0;
  while ((1u << cbits) < pl->nchunks) cbits++;
  pl->nterms = pl->nv + cbits;
  pl->Mmax = (size_t)d.W * n;
  pl->runs_max = (pl->Mmax + pl->K - 1) / pl->K + 1;
  if (pl->Mmax >= (1ull << 31)) return MSM_ERR_INVALID_ARG;
  return MSM_OK;
}

// The first bucket-reduction stage and the second's group trees in one launch (k_bucket_reduce_1g,
// MSM_RED_FOLD=1, where the tree form of the second stage applies; default k_bucket_reduce_1 then
// k_red2_groups).  Measured slower: 287 against 157 + 31 us per two-MSM 2^20 launch -- a group's
// tree then runs on two waves of 226-VGPR lanes (the first stage's occupancy) instead of eight
// light ones.
bool red_fold() {
  static const bool on = getenv("MSM_RED_FOLD") && atoi(getenv("MSM_RED_FOLD")) != 0;
  return on;
}

// The first bucket-reduction stage on lane pairs (k_bucket_reduce_1p, MSM_RED1_PAIRS=1; default one
// lane per chunk, k_bucket_reduce_1).  Measured equal: 159-162 against 160 us per two-MSM 2^20
// launch at three or four waves per SIMD, 154 at L = 8 but with the second stage then 51 against
// 31 us -- the chains' adds are issue-bound, not latency-bound.
bool red1_pairs() {
  static const bool on = getenv("MSM_RED1_PAIRS") && atoi(getenv("MSM_RED1_PAIRS")) != 0;
  return on;
}

// The second bucket-reduction stage as k_red2_groups + k_red2_terms (default; MSM_RED2_TREE=0:
// k_bucket_reduce_2), for windows of at most RG_MAXG groups of RG_CH chunks (k_bucket_reduce_2
// past that).  Single stream, 2^20, two MSMs per launch: 50 against 58 us.
uint32_t red2_groups(const Plan& pl) { return (pl.nchunks + RG_CH - 1) / RG_CH; }
bool red2_tree(const Plan& pl) {
  static const bool on = !(getenv("MSM_RED2_TREE") && atoi(getenv("MSM_RED2_TREE")) == 0);
  return on && red2_groups(pl) <= RG_MAXG;
}

int ensure_workspace(DevCtx* c, const Plan& pl, int si) {
  Slot& sl0 = c->slot[si];
  Workspace& w = sl0.ws;
  const MsmDims& d = pl.d;
  const size_t nb = (size_t)d.W * d.B;
  int rc;
  const uint64_t gen0 = g_alloc_gen.load();
#define ENS(buf, bytes) \
  if ((rc = w.buf.ensure(bytes)) != MSM_OK) return rc
  ENS(pts, (size_t)(d.shared ? 1 : d.nm) * d.n * PRE_WORDS * 4);
  ENS(err, 16);
  ENS(digits, (size_t)d.W * d.n * 4);
  ENS(colsum, ((size_t)d.nbins + d.W) * 4);  // bin totals, then window totals
  ENS(bin_base, ((size_t)d.nbins + 1) * 4);
  ENS(bin_cur, (size_t)d.nbins * 4);
  ENS(part_entry, pl.Mmax * 4);
  ENS(part_fine, pl.Mmax * 2);
  ENS(sorted_entry, pl.Mmax * 4 + 16);  // + a 16-B tail for k_accumulate's vector entry loads
  ENS(bucket_start, (nb + 2) * 4);
  ENS(run_key, pl.runs_max * 4);
#ifdef MSM_DUMMY_ALLOC
  ENS(dummy_tiles, (pl.Mmax / FS_CAP + d.nbins + 1) * 8 + 8);
  ENS(dummy_cursor, nb * 4);
#endif
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
  if (red2_tree(pl)) ENS(red_G, (size_t)d.W * red2_groups(pl) * RG_OUT * PT_WORDS * 4);
#undef ENS
  if (g_alloc_gen.load() != gen0) {
    // err, lead_flag, colsum and bin_cur are kept all-zero between MSMs by the kernels themselves
    // (k_bucket_reduce_2 clears the flags, k_fine_sort the bin totals and cursors), so a
    // replayed graph needs no memset nodes; fresh allocations start that invariant here.
    hipStream_t st = sl0.stream;
    if (hipMemsetAsync(w.err.p, 0, w.err.cap, st) != hipSuccess ||
        hipMemsetAsync(w.lead_flag.p, 0, w.lead_flag.cap, st) != hipSuccess ||
        hipMemsetAsync(w.skew_list.p, 0, 4, st) != hipSuccess ||
        hipMemsetAsync(w.colsum.p, 0, w.colsum.cap, st) != hipSuccess ||
        hipMemsetAsync(w.bin_cur.p, 0, w.bin_cur.cap, st) != hipSuccess || hipStreamSynchronize(st) != hipSuccess)
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

// Whether a launch sequence holding both the point preparation and the sort runs the two side by
// side (MSM_FORK_PREP=0 keeps them in order on one stream, for A/B runs).
bool fork_prepare() {
  static const bool on = !(getenv("MSM_FORK_PREP") && atoi(getenv("MSM_FORK_PREP")) == 0);
  return on;
}
// The same for the launches of a pipelined run (MSM_FORK_PREP_PIPE=1; default off).  There the fork
// measured slower: 2^20 at 20 steps 1.010 against 1.044 ms per MSM, three interleaved rounds each
// (and 1.022 against 1.035 in another session, profiles/r5/pipeline_ab.jsonl) -- a captured graph's
// forked branch runs on a hardware queue of the runtime's choosing, which the other slot's launch
// may be using (kernel traces show both slots' kernels on the same queues).
bool fork_prepare_pipelined() {
  static const bool on = getenv("MSM_FORK_PREP_PIPE") && atoi(getenv("MSM_FORK_PREP_PIPE")) != 0;
  return on;
}
bool slot_forks(const Slot& sl) { return sl.pipelined ? fork_prepare() && fork_prepare_pipelined() : fork_prepare(); }

// Whether k_prepare_points writes `records` point records with nontemporal stores: only when they
// outgrow the Infinity Cache (>= 128 MiB, i.e. 2^20 records; MSM_PP_NT=0/1 forces it).
uint32_t prep_nt(size_t records) {
  static const int forced = getenv("MSM_PP_NT") ? atoi(getenv("MSM_PP_NT")) : -1;
  if (forced >= 0) return forced ? 1u : 0u;
  return records * 128 >= (size_t(1) << 27) ? 1u : 0u;
}

// k_prepare_points over `cnt` points of one wire buffer into `pts_out` (one MSM, or one uploaded
// chunk of it); `nt` from prep_nt of the whole record buffer.
void launch_prepare(const uint32_t* wire, uint32_t* pts_out, uint32_t cnt, uint32_t* err, uint32_t nt,
                    hipStream_t s, uint32_t fmt = PT_FMT_WIRE) {
  BatchPtrs bp{};
  bp.p[0] = wire;
  hipLaunchKernelGGL(k_prepare_points, dim3(grid_for(cnt, PP_THREADS), 1), dim3(PP_THREADS), 0, s, bp, pts_out, cnt,
                     err, nt, fmt);
}

// The scalar recoding: the fixed-geometry kernel for the common window widths (c = 13..16,
// recode_fixed), the generic loop for the others (MSM_RECODE_FIXED=0 forces it everywhere).
bool recode_fixed_on() {
  static const bool on = !(getenv("MSM_RECODE_FIXED") && atoi(getenv("MSM_RECODE_FIXED")) == 0);
  return on;
}
template <uint32_t Q, uint32_t NHI>
void launch_recode_fixed(const MsmDims& d, const BatchPtrs& sc, void* digits, uint32_t* colsum, hipStream_t s) {
  const bool full = d.w0 == 0 && d.Wr == d.Wm && !d.half_lo && !d.half_hi;
  const dim3 grid(grid_for(d.n, RC_SPAN), d.nm);
  const size_t lds = ((size_t)d.Wr * d.nbc + d.Wr) * 4;
  if (full)
    hipLaunchKernelGGL((k_recode_fixed<Q, NHI, true>), grid, dim3(RC_THREADS), lds, s, sc, d,
                       static_cast<uint16_t*>(digits), colsum);
  else
    hipLaunchKernelGGL((k_recode_fixed<Q, NHI, false>), grid, dim3(RC_THREADS), lds, s, sc, d,
                       static_cast<uint16_t*>(digits), colsum);
}
void launch_recode(const MsmDims& d, const BatchPtrs& sc, void* digits, uint32_t* colsum, hipStream_t s) {
  const dim3 grid(grid_for(d.n, RC_SPAN), d.nm);
  const size_t lds = ((size_t)d.Wr * d.nbc + d.Wr) * 4;  // histogram + window totals
  if (d.c > 16) {
    hipLaunchKernelGGL(k_recode_hist<uint32_t>, grid, dim3(RC_THREADS), lds, s, sc, d, static_cast<uint32_t*>(digits),
                       colsum);
    return;
  }
  if (recode_fixed_on()) {
    if (d.q == 15 && d.nhi == 14) return launch_recode_fixed<15, 14>(d, sc, digits, colsum, s);
    if (d.q == 14 && d.nhi == 16) return launch_recode_fixed<14, 16>(d, sc, digits, colsum, s);
    if (d.q == 13 && d.nhi == 7) return launch_recode_fixed<13, 7>(d, sc, digits, colsum, s);
    if (d.q == 12 && d.nhi == 14) return launch_recode_fixed<12, 14>(d, sc, digits, colsum, s);
  }
  hipLaunchKernelGGL(k_recode_hist<uint16_t>, grid, dim3(RC_THREADS), lds, s, sc, d, static_cast<uint16_t*>(digits),
                     colsum);
}
bool is_recode_kernel(const void* f) {
  const void* ks[] = {reinterpret_cast<const void*>(&k_recode_hist<uint32_t>),
                      reinterpret_cast<const void*>(&k_recode_hist<uint16_t>),
                      reinterpret_cast<const void*>(&k_recode_fixed<15, 14, true>),
                      reinterpret_cast<const void*>(&k_recode_fixed<15, 14, false>),
                      reinterpret_cast<const void*>(&k_recode_fixed<14, 16, true>),
                      reinterpret_cast<const void*>(&k_recode_fixed<14, 16, false>),
                      reinterpret_cast<const void*>(&k_recode_fixed<13, 7, true>),
                      reinterpret_cast<const void*>(&k_recode_fixed<13, 7, false>),
                      reinterpret_cast<const void*>(&k_recode_fixed<12, 14, true>),
                      reinterpret_cast<const void*>(&k_recode_fixed<12, 14, false>)};
  for (const void* k : ks)
    if (f == k) return true;
  return false;
}

// Enqueue parts of the device pipeline on `s`; the reduced per-window terms land in the slot's
// h_out.  `pts` is the point-record buffer (the slot's own, or a shared base vector's).
// With `acc_events` (eager launches only), k_accumulate runs between the slot's ev_acc0 / ev_acc1
// (2), or is followed by ev_acc1 alone (1);
// captured graphs get the same events as record nodes (add_acc_event_nodes).
int enqueue_msm(DevCtx* c, const Plan& pl, const BatchPtrs& d_points, const BatchPtrs& d_scalars, int si,
                hipStream_t s, int parts, uint32_t* pts, int acc_events = 0) {
  const MsmDims& d = pl.d;
  Slot& sl = c->slot[si];
  Workspace& w = sl.ws;
  const bool prof = c->profiling == 1;
  auto mark = [&](int ph) {
    if (prof) hipEventRecord(c->ev[ph], s);
  };
  const uint32_t* total = w.bin_base.as<uint32_t>() + d.nbins;
  const unsigned rgrid = grid_for(pl.runs_max, ACC_THREADS);
  // The preparation reads only the points and the sort only the scalars: with both in this
  // sequence the preparation forks onto the slot's aux stream (a parallel branch of the captured
  // graph) and rejoins before the accumulation, so a lone MSM's sort no longer waits behind it.
  // (Profiling mode 1 keeps them in order, one event between every phase.)
  const bool fork = (parts & PART_PREP) && (parts & PART_SORT) && !prof && slot_forks(sl);
  auto prepare = [&](hipStream_t ps) {
    hipLaunchKernelGGL(k_prepare_points, dim3(grid_for(d.n, PP_THREADS), d.shared ? 1 : d.nm), dim3(PP_THREADS), 0, ps,
                       d_points, pts, d.n, w.err.as<uint32_t>(), prep_nt((size_t)(d.shared ? 1 : d.nm) * d.n), pl.pfmt);
  };
  if (parts & PART_PREP) {
    mark(PH_START);
    hipStream_t ps = s;
    if (fork) {
      HIPCHECK(hipEventRecord(sl.ev_fork, s));
      HIPCHECK(hipStreamWaitEvent(sl.aux, sl.ev_fork, 0));
      ps = sl.aux;
    }
    prepare(ps);
    if (fork) HIPCHECK(hipEventRecord(sl.ev_join, sl.aux));
    mark(PH_PREPARE);
  }
  if (parts & PART_SORT) {
    if (!(parts & PART_PREP)) {
      mark(PH_START);
      mark(PH_PREPARE);
    }
    launch_recode(d, d_scalars, w.digits.p, w.colsum.as<uint32_t>(), s);
    mark(PH_RECODE);
    mark(PH_SCAN);
    if (d.c <= 16) {
      hipLaunchKernelGGL(k_part_scatter<uint16_t>, dim3(d.nch, d.W), dim3(PT_THREADS), (size_t)d.nbc * 12, s,
                         w.digits.as<uint16_t>(), d, w.colsum.as<uint32_t>(), w.bin_cur.as<uint32_t>(),
                         w.bin_base.as<uint32_t>(), w.part_entry.as<uint32_t>(),
                         w.part_fine.as<uint16_t>());
    } else {
      hipLaunchKernelGGL(k_part_scatter<uint32_t>, dim3(d.nch, d.W), dim3(PT_THREADS), (size_t)d.nbc * 12, s,
                         w.digits.as<uint32_t>(), d, w.colsum.as<uint32_t>(), w.bin_cur.as<uint32_t>(),
                         w.bin_base.as<uint32_t>(), w.part_entry.as<uint32_t>(),
                         w.part_fine.as<uint16_t>());
    }
    mark(PH_SCATTER);
    hipLaunchKernelGGL(k_fine_sort, dim3(d.nbins), dim3(FS_THREADS), 0, s, w.part_entry.as<uint32_t>(),
                       w.part_fine.as<uint16_t>(), w.bin_base.as<uint32_t>(), d, pl.K, w.sorted_entry.as<uint32_t>(),
                       w.bucket_start.as<uint32_t>(), w.run_key.as<uint32_t>(), w.colsum.as<uint32_t>(),
                       w.bin_cur.as<uint32_t>());
#ifdef MSM_GAP_KERNEL
    hipLaunchKernelGGL(k_gap, dim3(MSM_GAP_KERNEL), dim3(64), 0, s, w.err.as<uint32_t>());
#endif
    mark(PH_FINE);
  }
  if (fork) HIPCHECK(hipStreamWaitEvent(s, sl.ev_join, 0));
  if ((parts & PART_ACC) && acc_events == 2) HIPCHECK(hipEventRecord(sl.ev_acc0, s));
  if (parts & PART_ACC) {
    hipLaunchKernelGGL(k_accumulate, dim3(rgrid), dim3(ACC_THREADS), 0, s, pts, w.sorted_entry.as<uint32_t>(),
                       w.bucket_start.as<uint32_t>(), w.run_key.as<uint32_t>(), total, pl.K, d.W * d.B,
                       w.buckets.as<uint32_t>(), w.lead_val.as<uint32_t>(), w.lead_open.as<uint32_t>(),
                       w.cross_key.as<uint32_t>(), w.skew_list.as<uint32_t>(), w.g_head.as<uint32_t>(),
                       w.g_hkey.as<uint32_t>(), w.g_tkey.as<uint32_t>());
    mark(PH_ACCUM);
  }
  if ((parts & PART_ACC) && acc_events) HIPCHECK(hipEventRecord(sl.ev_acc1, s));
  // profiling mode 1 keeps the joins in line (its per-phase timings include them)
  const bool joins = (parts & PART_JOIN) || prof;
  if ((parts & PART_POST) && joins) {
    hipLaunchKernelGGL(k_chain_join, dim3(CJ_GRID), dim3(ACC_THREADS), 0, s, w.skew_list.as<uint32_t>(), total, pl.K,
                       w.g_head.as<uint32_t>(), w.g_hkey.as<uint32_t>(), w.g_tkey.as<uint32_t>(),
                       w.buckets.as<uint32_t>(), w.lead_val.as<uint32_t>(), w.lead_open.as<uint32_t>(),
                       w.lead_flag.as<uint32_t>());
    hipLaunchKernelGGL(k_lead_scan, dim3(1), dim3(LS_THREADS), 0, s, w.lead_val.as<uint32_t>(),
                       w.lead_open.as<uint32_t>(), w.lead_flag.as<uint32_t>(), total, pl.K);
  }
  if (parts & PART_POST) {
    mark(PH_FIXUP);
    const bool fold = red_fold() && red2_tree(pl);
    if (fold) {
      const uint32_t G = red2_groups(pl);
      auto red1g = pl.L == 4    ? k_bucket_reduce_1g<4>
                   : pl.L == 9  ? k_bucket_reduce_1g<9>
                   : pl.L == 10 ? k_bucket_reduce_1g<10>
                   : pl.L == 12 ? k_bucket_reduce_1g<12>
                   : pl.L == 16 ? k_bucket_reduce_1g<16>
                   : pl.L == 17 ? k_bucket_reduce_1g<17>
                   : pl.L == 20 ? k_bucket_reduce_1g<20>
                                : k_bucket_reduce_1g<8>;
      hipLaunchKernelGGL(red1g, dim3(d.W * G), dim3(RG_CH), 0, s, w.buckets.as<uint32_t>(),
                         w.bucket_start.as<uint32_t>(), d, pl.K, pl.nchunks, G, w.cross_key.as<uint32_t>(),
                         w.lead_val.as<uint32_t>(), w.red_G.as<uint32_t>());
    }
    const bool pairs = red1_pairs();
    auto red1 = pl.L == 4    ? (pairs ? k_bucket_reduce_1p<4> : k_bucket_reduce_1<4>)
                : pl.L == 9  ? (pairs ? k_bucket_reduce_1p<9> : k_bucket_reduce_1<9>)
                : pl.L == 10 ? (pairs ? k_bucket_reduce_1p<10> : k_bucket_reduce_1<10>)
                : pl.L == 12 ? (pairs ? k_bucket_reduce_1p<12> : k_bucket_reduce_1<12>)
                : pl.L == 16 ? (pairs ? k_bucket_reduce_1p<16> : k_bucket_reduce_1<16>)
                : pl.L == 17 ? (pairs ? k_bucket_reduce_1p<17> : k_bucket_reduce_1<17>)
                : pl.L == 20 ? (pairs ? k_bucket_reduce_1p<20> : k_bucket_reduce_1<20>)
                             : (pairs ? k_bucket_reduce_1p<8> : k_bucket_reduce_1<8>);
    if (!fold)
    hipLaunchKernelGGL(red1, dim3(grid_for((size_t)d.W * pl.nchunks * (pairs ? 2 : 1), RED1_THREADS)), dim3(RED1_THREADS), 0, s,
                       w.buckets.as<uint32_t>(), w.bucket_start.as<uint32_t>(), d, pl.K, pl.nchunks,
                       w.cross_key.as<uint32_t>(), w.lead_val.as<uint32_t>(), w.red_U.as<uint32_t>(),
                       w.red_T.as<uint32_t>());
    mark(PH_RED1);
    if (red2_tree(pl)) {
      const uint32_t G = red2_groups(pl);
      if (!fold)
        hipLaunchKernelGGL(k_red2_groups, dim3(d.W * G), dim3(4 * RG_CH), 0, s, w.red_U.as<uint32_t>(),
                           w.red_T.as<uint32_t>(), pl.nchunks, G, w.bucket_start.as<uint32_t>(), d.B,
                           w.red_G.as<uint32_t>());
      // one lane quad per group point of the widest term (a wave at least): 2^16 pipelined
      // 0.117-0.120 against 0.125-0.131 ms per MSM with 64 quads throughout
      uint32_t gp = 16;
      while (gp < G) gp <<= 1;
      hipLaunchKernelGGL(k_red2_terms, dim3(d.W * pl.nterms), dim3(4 * gp), 0, s,
                         w.red_G.as<uint32_t>(), G,
                         pl.nv, pl.nterms, w.err.as<uint32_t>(), w.lead_flag.as<uint32_t>(),
                         w.skew_list.as<uint32_t>(), total, joins ? 1u : 0u, w.bucket_start.as<uint32_t>(), d.B,
                         reinterpret_cast<uint32_t*>(sl.h_out_dev));
    } else {
      hipLaunchKernelGGL(k_bucket_reduce_2, dim3(d.W * pl.nterms), dim3(RED2_THREADS), 0, s, w.red_U.as<uint32_t>(),
                         w.red_T.as<uint32_t>(), pl.nchunks, pl.nv, pl.nterms, w.err.as<uint32_t>(),
                         w.lead_flag.as<uint32_t>(), w.skew_list.as<uint32_t>(), total, joins ? 1u : 0u,
                         w.bucket_start.as<uint32_t>(), d.B, reinterpret_cast<uint32_t*>(sl.h_out_dev));
    }
    mark(PH_RED2);
    mark(PH_READBACK);
  }
  HIPCHECK(hipGetLastError());
  return MSM_OK;
}

// Host tail: MSM = sum_w 2^(c w) [ sum_v R_{w,v} + sum_k L 2^k R_{w,k} ]  (Horner over bit
// positions).  Follows reduce_last (lib.rs:88-104) in role: doublings between windows, then
// into_affine.  The device already emitted the terms in this file's Montgomery form
// (fe_to_host_mont).  Runs of doublings skip T (pt_dbl_proj) except the one feeding an add.

Pt term_at(const uint32_t* o) {
  Pt p;
  memcpy(p.X.l, o, 32);
  memcpy(p.Y.l, o + 8, 32);
  memcpy(p.T.l, o + 16, 32);
  memcpy(p.Z.l, o + 24, 32);
  return p;
}

// (bit position - base, term) pairs of the launch's local windows [w0, w1) of MSM terms block
// `terms` (local window l is window d.w0 + l of the MSM): V slices at the window's offset, R_k once
// per set bit b of L at offset + k + b; identity terms skipped.
void collect_terms(const Plan& pl, const uint32_t* terms, uint32_t w0, uint32_t w1, uint32_t base,
                   std::vector<std::pair<uint32_t, const uint32_t*>>* at) {
  const MsmDims& d = pl.d;
  for (uint32_t w = w0; w < w1; w++)
    for (uint32_t t = 0; t < pl.nterms; t++) {
      const uint32_t* o = terms + (size_t)(w * pl.nterms + t) * 32;
      Fq X;
      memcpy(X.l, o, 32);
      if (fq_is_zero(X) && !memcmp(o + 8, o + 24, 32)) continue;  // identity: X = 0, Y = Z
      const uint32_t off = win_off(d, d.w0 + w) - base;
      if (t < pl.nv) {
        at->emplace_back(off, o);
      } else {
        for (uint32_t b = 0; (pl.L >> b) != 0; b++)
          if ((pl.L >> b) & 1u) at->emplace_back(off + (t - pl.nv) + b, o);
      }
    }
}

// sum_j 2^(pos_j) P_j by Horner in descending position; get(j) gives P_j.
template <typename Get>
Pt horner_run(std::vector<std::pair<uint32_t, const uint32_t*>>& at, Get&& get) {
  std::stable_sort(at.begin(), at.end(), [](const auto& x, const auto& y) { return x.first > y.first; });
  Pt acc = pt_identity();
  for (size_t j = 0; j < at.size(); j++) {
    const Pt p = get(at[j].second);
    // T of the sum is needed when another add follows at the same position, and for the final
    // result (msm_compute_partial returns X|Y|T|Z); a doubling next never reads it
    const bool want_t = j + 1 == at.size() || at[j + 1].first == at[j].first;
    acc = j == 0 ? p : pt_add(acc, p, want_t);
    const uint32_t next = j + 1 < at.size() ? at[j + 1].first : 0u;
    if (at[j].first > next) acc = pt_dbl_n(acc, (int)(at[j].first - next));
  }
  return acc;
}

Pt horner_tail(const Plan& pl, const uint32_t* terms, uint32_t m = 0) {
  const MsmDims& d = pl.d;
  terms += (size_t)m * d.Wr * pl.nterms * 32;  // MSM m's windows
  std::vector<std::pair<uint32_t, const uint32_t*>> at;
  at.reserve((size_t)d.Wr * pl.nterms * 2);
  collect_terms(pl, terms, 0, d.Wr, 0, &at);
  return horner_run(at, term_at);
}

// The tail of a lone MSM (its latency, not a pipeline's throughput, is what counts), spread over
// helper threads started right after the launch, while the device works (thread start-up before
// the launch measured +15 us of latency; after it, it overlaps the device; they spin, yielding,
// until the terms land).  The helpers compute the window sums
// W_w = sum 2^(pos - off_w) term top window first, while the calling thread runs the outer Horner
// MSM = sum_w 2^(off_w) W_w, taking each W_w as it becomes ready: ~254 doublings and ~W adds on the
// critical path instead of ~254 doublings and ~W * nterms adds.  MSM_TAIL_THREADS sets the helper
// count (default 3; 0 = the one-thread horner_tail).
// The library's host threads are sized from the process's CPU budget (host_threads(): the
// hardware threads capped by the cgroup quota -- 16 on the GPU boxes, whose nproc says 256), shared
// among the devices of the running call (a device list runs one host thread per device, and each
// device context keeps its own pools): per device b = max(2, budget / devices); packing threads
// (the caller included) b / 2 up to 8, lone-MSM tail helpers b / 4 up to 3, pipelined-tail threads
// b / 8 up to 2, plus one uploader during a host-array call.  At one device on a 16-CPU quota that
// is the measured 8 / 3 / 2; a call over 8 devices gets 1 / 0 / 0 per device, so
// its 7 device threads and 8 uploaders stay within the quota.  The MSM_*_THREADS variables fix a
// count instead.
thread_local int t_call_devices = 1;  // devices of the call running on this thread (for_each_device)
int per_device_budget() { return std::max(2, (int)host_threads() / std::max(1, t_call_devices)); }
int env_threads(const char* name, int lo, int hi) {
  const char* e = getenv(name);
  return e ? std::max(lo, std::min(hi, atoi(e))) : -1;
}
int tail_helpers() {
  static const int env = env_threads("MSM_TAIL_THREADS", 0, 16);
  return env >= 0 ? env : std::min(3, per_device_budget() / 4);
}

class TailCrew {
 public:
  // The helpers are started once (per device context) and sleep between MSMs; arm() wakes them
  // right after a launch so they spin (yielding) while the device works, and run() hands them the
  // terms.  disarm() sends them back to sleep when no terms will come (an error return).
  explicit TailCrew(int helpers) {
    for (int i = 0; i < helpers; i++) th_.emplace_back([this] { work(); });
  }
  ~TailCrew() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      quit_.store(true);
    }
    cv_.notify_all();
    for (std::thread& t : th_) t.join();
  }
  bool active() const { return !th_.empty(); }
  int helpers() const { return (int)th_.size(); }
  void arm() {
    if (th_.empty()) return;
    wait_idle();  // the previous round is over (run() and disarm() wait for it too)
    {
      std::lock_guard<std::mutex> lk(mu_);
      idle_.store(0);
      armed_.store(true);
      gen_++;
    }
    cv_.notify_all();
  }
  void disarm() {
    armed_.store(false);
    wait_idle();
  }
  // The terms are on the host: the helpers start on the window sums, the caller on the outer
  // Horner, taking each window sum as it becomes ready (and computing one itself when none is).
  Pt run(const Plan& pl, const uint32_t* terms) {
    Pt r;
    run_batch(pl, terms, 1, &r);
    return r;
  }
  // The same for the k MSMs of one launch (terms block m at m * Wr * nterms * 32 words): the window
  // sums of all k, top windows first, over every thread; the outer Horner of MSM 0 on the caller,
  // those of MSMs 1.. on the first helpers free (the caller runs any no helper took).
  void run_batch(const Plan& pl, const uint32_t* terms, uint32_t k, Pt* out) {
    pl_ = &pl;
    terms_ = terms;
    k_ = k;
    out_ = out;
    const uint32_t n = k * pl.d.Wr;
    sums_.assign(n, pt_identity());
    ready_.reset(new std::atomic<int>[n]);
    for (uint32_t i = 0; i < n; i++) ready_[i].store(0);
    odone_.reset(new std::atomic<int>[k]);
    for (uint32_t m = 0; m < k; m++) odone_[m].store(0);
    next_.store(0);
    next_outer_.store(1);
    go_.store(true, std::memory_order_release);
    out[0] = outer(0);
    for (uint32_t m; (m = next_outer_.fetch_add(1)) < k;) {
      out[m] = outer(m);
      odone_[m].store(1, std::memory_order_release);
    }
    for (uint32_t m = 1; m < k; m++)
      while (!odone_[m].load(std::memory_order_acquire))
        if (!take_one()) _mm_pause();
    // every helper is out of this job before its state is reset by the next one
    armed_.store(false);
    wait_idle();
    go_.store(false);
  }

 private:
  void wait_idle() {
    while (idle_.load(std::memory_order_acquire) < (int)th_.size()) _mm_pause();
  }
  // MSM m = sum_w 2^(off_w) W_w by Horner over its windows, top first, each window sum taken as it
  // becomes ready (computing others meanwhile).
  Pt outer(uint32_t m) {
    const Plan& pl = *pl_;
    const uint32_t Wr = pl.d.Wr, w0 = pl.d.w0;  // local window w is window w0 + w of the MSM
    Pt acc = pt_identity();
    bool any = false;
    for (uint32_t kk = 0; kk < Wr; kk++) {
      const uint32_t w = Wr - 1 - kk;
      while (!ready_[m * Wr + w].load(std::memory_order_acquire))
        if (!take_one()) _mm_pause();
      const Pt& p = sums_[m * Wr + w];
      const bool ident = fq_is_zero(p.X) && fq_eq(p.Y, p.Z);
      if (!ident) acc = any ? pt_add(acc, p) : p;
      any = any || !ident;
      const uint32_t next = w ? win_off(pl.d, w0 + w - 1) : 0u;
      if (any && win_off(pl.d, w0 + w) > next) acc = pt_dbl_n(acc, (int)(win_off(pl.d, w0 + w) - next));
    }
    return acc;
  }
  // One window sum, top windows (of every MSM) first; false when none is left.
  bool take_one() {
    const uint32_t Wr = pl_->d.Wr;
    const uint32_t job = next_.fetch_add(1);
    if (job >= k_ * Wr) return false;
    const uint32_t m = job % k_, w = Wr - 1 - job / k_;
    std::vector<std::pair<uint32_t, const uint32_t*>> at;
    collect_terms(*pl_, terms_ + (size_t)m * Wr * pl_->nterms * 32, w, w + 1, win_off(pl_->d, pl_->d.w0 + w), &at);
    sums_[m * Wr + w] = horner_run(at, term_at);
    ready_[m * Wr + w].store(1, std::memory_order_release);
    return true;
  }
  void work() {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return quit_.load() || gen_ != seen; });
        if (quit_.load()) return;
        seen = gen_;
      }
      // armed: spin (a long device wait: stay cheap) until the terms are posted or the call ends
      uint64_t spins = 0;
      while (!go_.load(std::memory_order_acquire) && armed_.load() && !quit_.load()) {
        if (++spins > 4096) std::this_thread::yield();
        else _mm_pause();
      }
      if (go_.load(std::memory_order_acquire)) {
        for (uint32_t m; (m = next_outer_.fetch_add(1)) < k_;) {
          out_[m] = outer(m);
          odone_[m].store(1, std::memory_order_release);
        }
        while (take_one()) {
        }
      }
      idle_.fetch_add(1, std::memory_order_release);
    }
  }
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_;
  uint64_t gen_ = 0;
  std::atomic<bool> go_{false}, armed_{false}, quit_{false};
  std::atomic<int> idle_{1 << 30};  // helpers done with the current round (all idle at start)
  std::atomic<uint32_t> next_{0}, next_outer_{1};
  const Plan* pl_ = nullptr;
  const uint32_t* terms_ = nullptr;
  uint32_t k_ = 1;
  Pt* out_ = nullptr;
  std::vector<Pt> sums_;
  std::unique_ptr<std::atomic<int>[]> ready_, odone_;
};

// Host tails of a pipelined run's launches (all but the last, whose tails are the run's drain and
// go over the TailCrew), on persistent worker threads: the launching thread only waits for a
// launch, copies its terms and enqueues the next one.  With the tails on the launching thread, a
// slot whose launch finished while that thread was busy with another launch's Horner waited for
// it: a kernel trace of the 2^20 bench showed one slot's next launch 300 us behind the other's
// while the device ran only that other's sort (profiles/r5/pipeline_gap.txt).
class HornerPool {
 public:
  explicit HornerPool(int threads) {
    for (int i = 0; i < threads; i++) th_.emplace_back([this] { work(); });
  }
  ~HornerPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      quit_ = true;
    }
    cv_.notify_all();
    for (std::thread& t : th_) t.join();
  }
  void push(std::function<void()> fn) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      q_.push_back(std::move(fn));
      pending_++;
    }
    cv_.notify_one();
  }
  int size() const { return (int)th_.size(); }
  // every job pushed so far has run
  void wait_all() {
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [&] { return pending_ == 0; });
  }

 private:
  void work() {
    for (;;) {
      std::function<void()> fn;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return quit_ || !q_.empty(); });
        if (q_.empty()) return;  // quit with nothing left
        fn = std::move(q_.front());
        q_.pop_front();
      }
      fn();
      {
        std::lock_guard<std::mutex> lk(mu_);
        if (--pending_ == 0) done_cv_.notify_all();
      }
    }
  }
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  std::deque<std::function<void()>> q_;
  int pending_ = 0;
  bool quit_ = false;
};

// The packed host upload's threads: run(fn) calls fn(k, K) on K threads (the caller is k = 0) and
// returns when all are done.  Workers sleep on a condition variable between jobs; the caller spins
// (pausing) until they are done.
class PackPool {
 public:
  explicit PackPool(int threads) : k_(std::max(1, threads)) {
    for (int i = 1; i < k_; i++) th_.emplace_back([this, i] { work(i); });
  }
  ~PackPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      quit_ = true;
      gen_++;
    }
    cv_.notify_all();
    for (std::thread& t : th_) t.join();
  }
  int size() const { return k_; }
  void run(const std::function<void(int, int)>& fn) {
    fn_ = &fn;
    done_.store(0);
    {
      std::lock_guard<std::mutex> lk(mu_);
      gen_++;
    }
    cv_.notify_all();
    fn(0, k_);
    while (done_.load(std::memory_order_acquire) < k_ - 1) _mm_pause();
  }

 private:
  void work(int i) {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
        if (quit_) return;
      }
      (*fn_)(i, k_);
      done_.fetch_add(1, std::memory_order_release);
    }
  }
  int k_;
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_;
  uint64_t gen_ = 0;
  bool quit_ = false;
  const std::function<void(int, int)>* fn_ = nullptr;
  std::atomic<int> done_{0};
};

// Whether run_host_split packs its points (MSM_HOST_PACK, default on): the library's threads copy
// only x|y of every 128-B record (or x|y|z when some point of a launch has z != 1) into pinned
// staging, and t is derived from x and y on the device -- half the PCIe bytes of the points.
// pack_range uses AVX2 stores: a host without AVX2 uploads unpacked instead of faulting.
bool host_pack() {
  static const bool on =
      !(getenv("MSM_HOST_PACK") && atoi(getenv("MSM_HOST_PACK")) == 0) && __builtin_cpu_supports("avx2");
  return on;
}
int pack_threads() {
  static const int env = env_threads("MSM_HOST_PACK_THREADS", 1, 32);
  return env >= 0 ? env : std::max(1, std::min(8, per_device_budget() / 2));
}

// t < p for a coordinate in BE words (t is not uploaded by the packed path, so its range is
// checked here: the reference panics on any coordinate >= p, bytes.rs:19).
inline bool be_lt_p(const uint32_t* w) {
  static const uint32_t PBE[8] = {0x12ab655eu, 0x9a2ca556u, 0x60b44d1eu, 0x5c37b001u,
                                  0x59aa76feu, 0xd0000001u, 0x0a118000u, 0x00000001u};
  for (int k = 0; k < 8; k++)
    if (w[k] != PBE[k]) return w[k] < PBE[k];
  return false;
}

// One thread's share of pack_records: records [lo, hi).  32-B loads from the caller's array and
// nontemporal 32-B stores into the pinned staging (no read-for-ownership of the lines written;
// the staging is only read again by the copy engine; cached stores measured the same,
// profiles/r5/e2e_pack.jsonl).  dst is 32-B aligned (a pinned buffer at a
// multiple of 64 B).
__attribute__((target("avx2"))) void pack_range(uint32_t* dst, const uint32_t* src, size_t lo, size_t hi, uint32_t fmt,
                                                bool* z_other, bool* t_bad) {
  const size_t pw = pt_fmt_slots(fmt) * 4;
  bool zo = false, bad = false;
  for (size_t i = lo; i < hi; i++) {
    const uint32_t* r = src + i * 32;
    __m256i* d = reinterpret_cast<__m256i*>(dst + i * pw);
    _mm256_stream_si256(d, _mm256_loadu_si256(reinterpret_cast<const __m256i*>(r)));
    _mm256_stream_si256(d + 1, _mm256_loadu_si256(reinterpret_cast<const __m256i*>(r + 8)));
    if (fmt == PT_FMT_XYZ) _mm256_stream_si256(d + 2, _mm256_loadu_si256(reinterpret_cast<const __m256i*>(r + 24)));
    zo = zo || r[31] != 1u || (r[24] | r[25] | r[26] | r[27] | r[28] | r[29] | r[30]) != 0u;
    bad = bad || (r[16] >= 0x12ab655eu && !be_lt_p(r + 16));
  }
  _mm_sfence();
  *z_other = zo;
  *t_bad = bad;
}

// Pack cnt wire records (x|y|t|z, 32 BE words) into dst in format fmt (PT_FMT_XY: x|y, 16 words;
// PT_FMT_XYZ: x|y|z, 24 words) over the pool; returns whether every z is 1 (XY is then exact)
// and sets *t_bad when some t >= p.
bool pack_records(PackPool& pool, uint32_t* dst, const uint32_t* src, size_t cnt, uint32_t fmt, bool* t_bad) {
  std::atomic<bool> z_other{false}, tb{false};
  pool.run([&](int k, int K) {
    const size_t lo = cnt * k / K, hi = cnt * (k + 1) / K;
    bool zo = false, bad = false;
    pack_range(dst, src, lo, hi, fmt, &zo, &bad);
    if (zo) z_other.store(true, std::memory_order_relaxed);
    if (bad) tb.store(true, std::memory_order_relaxed);
  });
  if (tb.load()) *t_bad = true;
  return !z_other.load();
}

// Plain parallel copy into pinned staging (the packed path's scalars).
void pack_copy(PackPool& pool, void* dst, const void* src, size_t bytes) {
  pool.run([&](int k, int K) {
    const size_t lo = (bytes * k / K) & ~size_t(63), hi = k + 1 == K ? bytes : (bytes * (k + 1) / K) & ~size_t(63);
    if (hi > lo) memcpy(static_cast<char*>(dst) + lo, static_cast<const char*>(src) + lo, hi - lo);
  });
}

// The next staging buffer of the ring, at least `bytes` long, once the copy out of it is done.
int pin_take(DevCtx* c, int k, size_t bytes, void** out) {
  PinRing& r = c->pin;
  if (!r.ev[k] && hipEventCreateWithFlags(&r.ev[k], hipEventDisableTiming) != hipSuccess) return MSM_ERR_HIP;
  if (r.used[k] && hipEventSynchronize(r.ev[k]) != hipSuccess) return MSM_ERR_HIP;
  r.used[k] = false;
  if (int rc = r.buf[k].ensure(bytes)) return rc;
  *out = r.buf[k].p;
  return MSM_OK;
}
// The copy out of buffer k is enqueued on `s`: it is reusable once that completes.
int pin_give(DevCtx* c, int k, hipStream_t s) {
  if (hipEventRecord(c->pin.ev[k], s) != hipSuccess) return MSM_ERR_HIP;
  c->pin.used[k] = true;
  return MSM_OK;
}

// Every staging buffer of the ring at `bytes` before a packed call enqueues anything (a growth
// bumps the allocation generation).  False -- the call then uploads unpacked -- for buffers over
// 512 MiB (a launch of more than ~2^22 points: that much pinned memory per buffer costs more to
// allocate than packing saves) or when the pinned allocation fails.
size_t pin_max_bytes() {  // MSM_PIN_MAX_MB overrides (tests force the fallback with a small cap)
  static const long mb = getenv("MSM_PIN_MAX_MB") ? atol(getenv("MSM_PIN_MAX_MB")) : 512;
  static const size_t v = mb >= 0 && mb < (1l << 30) ? (size_t)mb << 20 : size_t(512) << 20;
  return v;
}
bool pin_ring_ready(DevCtx* c, size_t bytes) {
  if (bytes > pin_max_bytes()) return false;
  for (int k = 0; k < NPIN; k++) {
    void* b;
    if (pin_take(c, k, bytes, &b) != MSM_OK) {
      (void)hipGetLastError();
      return false;
    }
  }
  return true;
}

// Worker threads of the pool (MSM_HORNER_THREADS; 0 = the launching thread runs the tails itself).
int horner_threads() {
  static const int env = env_threads("MSM_HORNER_THREADS", 0, 16);
  return env >= 0 ? env : std::min(2, per_device_budget() / 8);
}

// A device context's pools at the sizes above for the running call (re-created when the call's
// share differs from the one they were made for; calls on a context hold its mutex).
PackPool* ctx_packer(DevCtx* c) {
  const int k = pack_threads();
  if (!c->packer || c->packer->size() != k) {
    delete c->packer;
    c->packer = new PackPool(k);
  }
  return c->packer;
}
TailCrew* ctx_crew(DevCtx* c) {
  const int h = tail_helpers();
  if (!c->crew || c->crew->helpers() != h) {
    delete c->crew;
    c->crew = new TailCrew(h);
  }
  return c->crew;
}
// Pools the CPU test hooks start (msm_test_pack, msm_test_pools), stopped by msm_shutdown too.
struct TestPools {
  PackPool* packer = nullptr;
  TailCrew* crew = nullptr;
  HornerPool* pool = nullptr;
  void stop() {
    delete packer;
    delete crew;
    delete pool;
    packer = nullptr;
    crew = nullptr;
    pool = nullptr;
  }
};
std::mutex g_test_mu;
TestPools g_test_pools;

HornerPool* ctx_pool(DevCtx* c) {
  const int h = horner_threads();
  if (h == 0) return nullptr;
  if (!c->pool || c->pool->size() != h) {
    delete c->pool;
    c->pool = new HornerPool(h);
  }
  return c->pool;
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

// Bracket the captured k_accumulate node with event-record nodes (the slot's ev_acc0 / ev_acc1):
// every replay of the graph then times the accumulation, with no extra launches.
int add_acc_event_nodes(hipGraph_t g, Slot& sl, bool both) {
  size_t num = 0;
  if (hipGraphGetNodes(g, nullptr, &num) != hipSuccess || num == 0) return MSM_ERR_HIP;
  std::vector<hipGraphNode_t> nodes(num);
  if (hipGraphGetNodes(g, nodes.data(), &num) != hipSuccess) return MSM_ERR_HIP;
  const void* f_acc = reinterpret_cast<const void*>(&k_accumulate);
  hipGraphNode_t acc = nullptr;
  for (hipGraphNode_t nd : nodes) {
    hipGraphNodeType ty;
    hipKernelNodeParams kp{};
    if (hipGraphNodeGetType(nd, &ty) == hipSuccess && ty == hipGraphNodeTypeKernel &&
        hipGraphKernelNodeGetParams(nd, &kp) == hipSuccess && kp.func == f_acc)
      acc = nd;
  }
  if (!acc) return MSM_ERR_HIP;
  size_t nd = 0, nx = 0;
  if (hipGraphNodeGetDependencies(acc, nullptr, &nd) != hipSuccess ||
      hipGraphNodeGetDependentNodes(acc, nullptr, &nx) != hipSuccess)
    return MSM_ERR_HIP;
  std::vector<hipGraphNode_t> deps(nd), outs(nx);
  if ((nd && hipGraphNodeGetDependencies(acc, deps.data(), &nd) != hipSuccess) ||
      (nx && hipGraphNodeGetDependentNodes(acc, outs.data(), &nx) != hipSuccess))
    return MSM_ERR_HIP;
  hipGraphNode_t r0 = nullptr, r1 = nullptr;
  if (both) {
    for (hipGraphNode_t d : deps)
      if (hipGraphRemoveDependencies(g, &d, &acc, 1) != hipSuccess) return MSM_ERR_HIP;
    if (hipGraphAddEventRecordNode(&r0, g, deps.data(), deps.size(), sl.ev_acc0) != hipSuccess ||
        hipGraphAddDependencies(g, &r0, &acc, 1) != hipSuccess)
      return MSM_ERR_HIP;
  }
  for (hipGraphNode_t o : outs)
    if (hipGraphRemoveDependencies(g, &acc, &o, 1) != hipSuccess) return MSM_ERR_HIP;
  if (hipGraphAddEventRecordNode(&r1, g, &acc, 1, sl.ev_acc1) != hipSuccess) return MSM_ERR_HIP;
  for (hipGraphNode_t o : outs)
    if (hipGraphAddDependencies(g, &r1, &o, 1) != hipSuccess) return MSM_ERR_HIP;
  return MSM_OK;
}

int capture(DevCtx* c, const Plan& pl, const BatchPtrs& d_points, const BatchPtrs& d_scalars, int si, hipStream_t s,
            int parts, uint32_t* pts, int acc_events, hipGraph_t* gout, hipGraphExec_t* out) {
  hipGraph_t g = nullptr;
  if (hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal) != hipSuccess) return MSM_ERR_HIP;
  int rc = enqueue_msm(c, pl, d_points, d_scalars, si, s, parts, pts);
  hipError_t e = hipStreamEndCapture(s, &g);
  if (rc != MSM_OK || e != hipSuccess || !g) {
    if (g) hipGraphDestroy(g);
    (void)hipGetLastError();
    return MSM_ERR_HIP;
  }
  if (acc_events && (parts & PART_ACC) && add_acc_event_nodes(g, c->slot[si], acc_events == 2) != MSM_OK) {
    hipGraphDestroy(g);
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

// Find the input-reading kernel nodes of a segment so later launches can repoint them.
int find_input_nodes(Segment& sg) {
  size_t num = 0;
  if (hipGraphGetNodes(sg.graph, nullptr, &num) != hipSuccess || num == 0) return MSM_ERR_HIP;
  std::vector<hipGraphNode_t> nodes(num);
  if (hipGraphGetNodes(sg.graph, nodes.data(), &num) != hipSuccess) return MSM_ERR_HIP;
  const void* f_prep = reinterpret_cast<const void*>(&k_prepare_points);
  for (hipGraphNode_t nd : nodes) {
    hipGraphNodeType ty;
    if (hipGraphNodeGetType(nd, &ty) != hipSuccess || ty != hipGraphNodeTypeKernel) continue;
    hipKernelNodeParams kp{};
    if (hipGraphKernelNodeGetParams(nd, &kp) != hipSuccess) continue;
    if (kp.func == f_prep) {
      sg.n_prep = nd;
      sg.p_prep = kp;
    } else if (is_recode_kernel(kp.func)) {
      sg.n_recode = nd;
      sg.p_recode = kp;
    }
  }
  const bool ok = (!(sg.parts & PART_PREP) || sg.n_prep) && (!(sg.parts & PART_SORT) || sg.n_recode);
  return ok ? MSM_OK : MSM_ERR_HIP;
}

bool same_ptrs(const BatchPtrs& a, const BatchPtrs& b) { return memcmp(&a, &b, sizeof(BatchPtrs)) == 0; }

// Point an instantiated segment at new input buffers (kernel-node argument update, no
// re-capture).
int repoint_inputs(const Plan& pl, Slot& sl, Segment& sg, const BatchPtrs& d_points, const BatchPtrs& d_scalars) {
  const MsmDims& d = pl.d;
  Workspace& w = sl.ws;
  if (sg.n_prep && !same_ptrs(sg.in_pts, d_points)) {
    BatchPtrs wire = d_points;
    uint32_t* ptsb = const_cast<uint32_t*>(sg.pts_buf);
    uint32_t n = d.n;
    uint32_t* err = w.err.as<uint32_t>();
    uint32_t nt = prep_nt((size_t)(d.shared ? 1 : d.nm) * d.n);
    uint32_t fmt = pl.pfmt;
    void* a_prep[] = {&wire, &ptsb, &n, &err, &nt, &fmt};
    hipKernelNodeParams kp = sg.p_prep;
    kp.kernelParams = a_prep;
    kp.extra = nullptr;
    if (hipGraphExecKernelNodeSetParams(sg.exec, sg.n_prep, &kp) != hipSuccess) return MSM_ERR_HIP;
    sg.in_pts = d_points;
  }
  if (sg.n_recode && !same_ptrs(sg.in_sc, d_scalars)) {
    BatchPtrs scal = d_scalars;
    MsmDims dd = d;
    void* digits = w.digits.p;
    uint32_t* hist = w.colsum.as<uint32_t>();
    void* a_rc[] = {&scal, &dd, &digits, &hist};
    hipKernelNodeParams kr = sg.p_recode;
    kr.kernelParams = a_rc;
    kr.extra = nullptr;
    if (hipGraphExecKernelNodeSetParams(sg.exec, sg.n_recode, &kr) != hipSuccess) return MSM_ERR_HIP;
    sg.in_sc = d_scalars;
  }
  return MSM_OK;
}

// The cached graph of `parts` for this plan (captured on first use, least recently used segment
// evicted), repointed at the launch's inputs; nullptr when graphs are unavailable.
Segment* get_segment(DevCtx* c, const Plan& pl, const BatchPtrs& d_points, const BatchPtrs& d_scalars, int si,
                     int parts, uint32_t* pts, int acc_events) {
  Slot& sl = c->slot[si];
  const uint64_t gen = g_alloc_gen.load();
  Segment* hit = nullptr;
  for (Segment& sg : sl.seg)
    if (sg.exec && sg.parts == parts && sg.pts_buf == pts && sg.acc_events == acc_events && sg.gen == gen &&
        sg.fork == slot_forks(sl) && plan_eq(sg.pl, pl))
      hit = &sg;
  if (!hit) {
    Segment* victim = &sl.seg[0];
    for (Segment& sg : sl.seg) {
      if (!sg.exec || sg.gen != gen) {
        victim = &sg;
        break;
      }
      if (sg.used < victim->used) victim = &sg;
    }
    victim->drop();
    victim->pl = pl;
    victim->parts = parts;
    victim->pts_buf = pts;
    victim->acc_events = acc_events;
    victim->fork = slot_forks(sl);
    victim->gen = gen;
    int rc = capture(c, pl, d_points, d_scalars, si, sl.stream, parts, pts, acc_events, &victim->graph,
                     &victim->exec);
    if (rc == MSM_OK) rc = find_input_nodes(*victim);
    if (rc != MSM_OK) {
      victim->drop();
      // event-record nodes unsupported: time k_accumulate eagerly between graph segments;
      // otherwise capture itself is unsupported here: stay eager
      if (acc_events) c->graph_events_ok = false;
      else c->graphs_ok = false;
      return nullptr;
    }
    victim->in_pts = d_points;
    victim->in_sc = d_scalars;
    hit = victim;
  }
  if (repoint_inputs(pl, sl, *hit, d_points, d_scalars) != MSM_OK) {
    hit->drop();
    (void)hipGetLastError();
    c->graphs_ok = false;
    return nullptr;
  }
  hit->used = ++sl.seg_clock;
  return hit;
}

// Enqueue `parts` of one launch in slot `si` (on the slot's stream) by replaying the captured
// graph of those parts; k_accumulate runs between the slot's two timing events on every launch
// (event-record nodes inside the graph), so the production path is the timed one.  Where the
// runtime cannot capture event records, the accumulation is launched eagerly between a graph of
// the parts before it and one of the parts after it.  Profiling mode 1 launches everything
// eagerly with an event between every phase.
int launch_on(DevCtx* c, const Plan& pl, const BatchPtrs& d_points, const BatchPtrs& d_scalars, int si, int parts,
              uint32_t* pts, hipStream_t s) {
  // k_accumulate's bracketing events only when profiling mode 2 reads them: each event-record
  // node adds ~6 us to the launch sequence's critical path (profiles/r3/latency_timeline.txt)
  // (a staggered slot's graphs also record ev_acc1 after k_accumulate: the next launch waits on it)
  const int acc = (parts & PART_ACC) == 0 ? 0 : c->profiling == 2 ? 2 : c->slot[si].stagger ? 1 : 0;
  if (parts & PART_ACC) c->slot[si].acc_timed = acc == 2;
  if (c->profiling == 1) {
    c->slot[si].acc_timed = false;
    if (int rc = enqueue_msm(c, pl, d_points, d_scalars, si, s, parts, pts)) return rc;
  } else if (c->graphs_ok && graphs_enabled()) {
    Segment* sg = (!acc || c->graph_events_ok) ? get_segment(c, pl, d_points, d_scalars, si, parts, pts, acc) : nullptr;
    if (sg) {
      HIPCHECK(hipGraphLaunch(sg->exec, s));
    } else {
      auto run = [&](int p) -> int {
        if (!p) return MSM_OK;
        Segment* g = c->graphs_ok ? get_segment(c, pl, d_points, d_scalars, si, p, pts, false) : nullptr;
        if (g) {
          HIPCHECK(hipGraphLaunch(g->exec, s));
          return MSM_OK;
        }
        return enqueue_msm(c, pl, d_points, d_scalars, si, s, p, pts);
      };
      if (int rc = run(parts & (PART_PREP | PART_SORT))) return rc;
      if (parts & PART_ACC)
        if (int rc = enqueue_msm(c, pl, d_points, d_scalars, si, s, PART_ACC, pts, acc)) return rc;
      if (int rc = run(parts & (PART_POST | PART_JOIN))) return rc;
    }
  } else if (int rc = enqueue_msm(c, pl, d_points, d_scalars, si, s, parts, pts, acc)) {
    return rc;
  }
  return MSM_OK;
}

int launch_parts(DevCtx* c, const Plan& pl, const BatchPtrs& d_points, const BatchPtrs& d_scalars, int si,
                 int parts, uint32_t* pts) {
  Slot& sl = c->slot[si];
  hipStream_t s = sl.stream;
  if (c->profiling && (parts & (PART_PREP | PART_SORT))) HIPCHECK(hipEventRecord(sl.ev_start, s));
  if (int rc = launch_on(c, pl, d_points, d_scalars, si, parts, pts, s)) return rc;
  if (parts & PART_POST) {
    if (c->profiling) HIPCHECK(hipEventRecord(sl.ev_end, s));
    HIPCHECK(hipEventRecord(sl.ev_done, s));
  }
  return MSM_OK;
}


// Wait for the launch in slot `si` (spinning briefly: the result is usually due within a couple of
// milliseconds, and a blocking wait adds a wake-up latency) and check its flags; its window terms
// are then in the slot's h_out.  Skewed scalars: the sequence ran without the bucket joins
// (PART_JOIN), so they and the reduction run again here (the slot's stream is idle: its next launch
// is enqueued afterwards).
int wait_slot(DevCtx* c, int si, uint32_t* total_out = nullptr) {
  Slot& sl = c->slot[si];
  const Plan& pl = sl.pl;
  const auto spin_until = clk::now() + std::chrono::milliseconds(50);
  hipError_t q;
  while ((q = hipEventQuery(sl.ev_done)) == hipErrorNotReady && clk::now() < spin_until) _mm_pause();
  if (q == hipErrorNotReady) q = hipEventSynchronize(sl.ev_done);
  HIPCHECK(q);
  const size_t outb = (size_t)pl.d.W * pl.nterms * 32 * 4;
  const uint32_t* h = reinterpret_cast<const uint32_t*>(sl.h_out.p);
  const uint32_t err = h[outb / 4];
  if (total_out) *total_out = h[outb / 4 + 1];
  if (h[outb / 4 + 2]) {
    // only the second k_bucket_reduce_2 clears the skew list and the lead flag: if the re-run
    // cannot be enqueued or does not complete, clear them here, or the slot's next MSM would append
    // to a stale skew list and rejoin stale workgroups without any error
    int rc = enqueue_msm(c, pl, BatchPtrs{}, BatchPtrs{}, si, sl.stream, PART_JOIN | PART_POST, nullptr);
    if (rc == MSM_OK && (hipEventRecord(sl.ev_done, sl.stream) != hipSuccess ||
                         hipEventSynchronize(sl.ev_done) != hipSuccess))
      rc = MSM_ERR_HIP;
    if (rc != MSM_OK) {
      (void)hipGetLastError();
      hipMemsetAsync(sl.ws.skew_list.p, 0, 4, sl.stream);
      hipMemsetAsync(sl.ws.lead_flag.p, 0, sl.ws.lead_flag.cap, sl.stream);
      hipStreamSynchronize(sl.stream);
      return rc;
    }
  }
  if (err & MSM_DEV_ERR_COORD_RANGE) return MSM_ERR_COORD_RANGE;
  if (err & MSM_DEV_ERR_BAD_POINT) return MSM_ERR_BAD_POINT;
  return MSM_OK;
}

int finish_msm(DevCtx* c, int si, Pt* result, std::vector<uint32_t>* terms = nullptr, TailCrew* crew = nullptr) {
  Slot& sl = c->slot[si];
  const Plan& pl = sl.pl;
  uint32_t total = 0;
  if (int rc = wait_slot(c, si, &total)) return rc;
  const size_t outb = (size_t)pl.d.W * pl.nterms * 32 * 4;
  const uint32_t* h = reinterpret_cast<const uint32_t*>(sl.h_out.p);
  auto t0 = clk::now();
  if (terms)
    terms->assign(h, h + outb / 4);
  else if (crew && crew->active())
    *result = crew->run(pl, h);
  else
    *result = horner_tail(pl, h);
  auto t1 = clk::now();
  if (c->profiling == 1 || (c->profiling == 2 && sl.acc_timed)) {
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
    P.windows = pl.d.Wr;
    P.run_length = pl.K;
    P.chunk_len = pl.L;
    P.msms_per_launch = pl.d.nm;
    P.accumulate_sum += P.accumulate;
    P.device_total_sum += P.device_total;
    P.profiled++;
    if (c->profiling == 2) {
      float a = 0, b = 0;
      if (hipEventElapsedTime(&a, c->ev_base, sl.ev_acc0) == hipSuccess &&
          hipEventElapsedTime(&b, c->ev_base, sl.ev_acc1) == hipSuccess)
        c->acc_ivals.emplace_back(a, b);
    }
  }
  return MSM_OK;
}

// Profiling mode 2: the call's accumulation intervals start from ev_base; at the end their union
// (wall time with at least one k_accumulate in flight) is added to accumulate_union_sum.  With
// several launches in flight accumulations may overlap each other, so the union, not the sum of
// brackets, is the kernel's share of the device time.
void begin_call(DevCtx* c) {
  c->acc_ivals.clear();
  if (c->profiling == 2) hipEventRecord(c->ev_base, c->slot[0].stream);
}
void end_call(DevCtx* c) {
  if (c->profiling != 2 || c->acc_ivals.empty()) return;
  std::sort(c->acc_ivals.begin(), c->acc_ivals.end());
  double total = 0, lo = c->acc_ivals[0].first, hi = c->acc_ivals[0].second;
  for (const auto& iv : c->acc_ivals) {
    if (iv.first > hi) {
      total += hi - lo;
      lo = iv.first;
      hi = iv.second;
    } else {
      hi = std::max<double>(hi, iv.second);
    }
  }
  total += hi - lo;
  c->last.accumulate_union_sum += total;
  c->acc_ivals.clear();
}

BatchPtrs splat(const uint32_t* p) {
  BatchPtrs b{};
  for (uint32_t m = 0; m < MSM_MAX_BATCH; m++) b.p[m] = p;
  return b;
}

// The caller's stream (if any) -> every slot stream about to be used waits for its work so far.
int order_after_user(DevCtx* c, hipStream_t user, int nslot) {
  if (!user) return MSM_OK;
  HIPCHECK(hipEventRecord(c->ev_user, user == (hipStream_t)MSM_STREAM_NULL ? nullptr : user));
  for (int si = 0; si < nslot; si++) HIPCHECK(hipStreamWaitEvent(c->slot[si].stream, c->ev_user, 0));
  return MSM_OK;
}

// The host tail of a lone MSM in slot `si`, over the device context's persistent helpers: armed
// right after the launch (they spin while the device works), handed the terms when they land.
int finish_lone(DevCtx* c, int si, Pt* result) {
  TailCrew* crew = ctx_crew(c);
  crew->arm();
  const int rc = finish_msm(c, si, result, nullptr, crew);
  if (rc != MSM_OK) crew->disarm();  // no terms will come
  return rc;
}

// Run one MSM with device inputs; result as a projective host point.
int run_device(DevCtx* c, const uint32_t* d_points, const uint32_t* d_scalars, size_t n, const msm_opts* o,
               hipStream_t user_stream, Pt* result) {
  if (n == 0) {
    *result = pt_identity();
    return MSM_OK;
  }
  Plan pl;
  int rc = make_plan(n, o, c->shape, &pl);
  if (rc != MSM_OK) return rc;
  const int si = 0;  // a lone MSM always uses slot 0 (the other workspaces only for pipelining)
  c->slot[si].pipelined = false;
  c->slot[si].stagger = false;
  if ((rc = ensure_workspace(c, pl, si)) != MSM_OK) return rc;
  if ((rc = order_after_user(c, user_stream, 1)) != MSM_OK) return rc;
  c->slot[si].pl = pl;
  if ((rc = launch_parts(c, pl, splat(d_points), splat(d_scalars), si, PART_ALL, c->slot[si].ws.pts.as<uint32_t>())))
    return rc;
  return finish_lone(c, si, result);
}

// Host -> device copy of one input array on the copy stream, in pieces of `piece` bytes; after
// each piece `on_piece(off, bytes)` may hand the uploaded range to the device (an event on the
// copy stream marks it).  hipMemcpyAsync stages pageable memory itself at the PCIe rate
// (tools/ubench/h2d_bench.cpp: 56 GB/s pageable or pinned), so no extra host copy is made.
template <typename F>
int upload(DevCtx* c, void* dst, const void* src, size_t bytes, size_t piece, F&& on_piece) {
  for (size_t off = 0; off < bytes; off += piece) {
    const size_t b = std::min(piece, bytes - off);
    HIPCHECK(hipMemcpyAsync(static_cast<char*>(dst) + off, static_cast<const char*>(src) + off, b,
                            hipMemcpyHostToDevice, c->copy_stream));
    if (int rc = on_piece(off, b)) return rc;
  }
  return MSM_OK;
}

constexpr size_t UPLOAD_PTS_PIECE = 65536;  // points per uploaded piece (8 MiB; a multiple of PP_THREADS)

// Upload n host points into `wire` and prepare them into `pts` piece by piece on stream `s`: the
// preparation of piece k overlaps the upload of piece k+1 (the reference's staging ring,
// gpu.ts:146-155, without its 128 MiB cap).
int upload_points(DevCtx* c, const uint32_t* points_be, size_t n, uint32_t* wire, uint32_t* pts, uint32_t* err,
                  hipStream_t s) {
  int k = 0;
  return upload(c, wire, points_be, n * 128, UPLOAD_PTS_PIECE * 128, [&](size_t off, size_t b) -> int {
    hipEvent_t e = c->ev_chunk[k++ % NCHUNK_EV];
    HIPCHECK(hipEventRecord(e, c->copy_stream));
    HIPCHECK(hipStreamWaitEvent(s, e, 0));
    const size_t p0 = off / 128;
    launch_prepare(wire + p0 * 32, pts + p0 * PRE_WORDS, (uint32_t)(b / 128), err, prep_nt(n), s);
    HIPCHECK(hipGetLastError());
    return MSM_OK;
  });
}

// Upload a scalar vector into `wire` and make stream `s` wait for it.
int upload_scalars(DevCtx* c, const uint32_t* scalars_be, size_t n, uint32_t* wire, hipStream_t s, hipEvent_t e) {
  int rc = upload(c, wire, scalars_be, n * 32, n * 32, [](size_t, size_t) { return MSM_OK; });
  if (rc != MSM_OK) return rc;
  HIPCHECK(hipEventRecord(e, c->copy_stream));
  HIPCHECK(hipStreamWaitEvent(s, e, 0));
  return MSM_OK;
}

// One MSM of host-resident inputs: the scalars go up first and the bucket sort starts on them
// while the points upload piece by piece, each piece prepared as it lands; accumulation starts
// after the last piece.  The end-to-end time is then ~ PCIe transfer + the post-upload tail.
int run_host(DevCtx* c, const uint32_t* points_be, const uint32_t* scalars_be, size_t n, const msm_opts* o,
             Pt* result) {
  if (n == 0) {
    *result = pt_identity();
    return MSM_OK;
  }
  Plan pl;
  int rc = make_plan(n, o, c->shape, &pl);
  if (rc != MSM_OK) return rc;
  const int si = 0;
  Slot& sl = c->slot[si];
  sl.pipelined = false;
  sl.stagger = false;
  Workspace& w = sl.ws;
  if ((rc = ensure_workspace(c, pl, si)) != MSM_OK) return rc;
  if ((rc = w.wire_pts.ensure(n * 128)) != MSM_OK || (rc = w.wire_sc.ensure(n * 32)) != MSM_OK) return rc;
  sl.pl = pl;
  uint32_t* pts = w.pts.as<uint32_t>();
  const BatchPtrs bp = splat(w.wire_pts.as<uint32_t>()), bs = splat(w.wire_sc.as<uint32_t>());
  // once an upload is queued, an error return first waits for it: the copies read the caller's
  // arrays, which msm.h promises are not read after the call returns
  auto fail = [&](int code) {
    hipStreamSynchronize(c->copy_stream);
    hipStreamSynchronize(sl.stream);
    return code;
  };
  bool t_bad = false;  // some t >= p, checked on the host (t is not uploaded): reported once the
                       // MSM has run, so the device's flags end cleared as after any call
  if (host_pack() && pin_ring_ready(c, std::min(n, UPLOAD_PTS_PIECE) * 96)) {
    // packed (as the split, §2.6): the scalars through the pinned ring, then each 8 MiB piece of
    // points as x|y (x|y|z for a piece with some z != 1), prepared in its own format as it lands
    ctx_packer(c);
    int k = 0;
    uint32_t* wsc = w.wire_sc.as<uint32_t>();
    for (size_t off = 0; off < n; off += UPLOAD_PTS_PIECE, k++) {
      const size_t cnt = std::min(UPLOAD_PTS_PIECE, n - off);
      void* buf;
      if ((rc = pin_take(c, k % NPIN, cnt * 32, &buf)) != MSM_OK) return fail(rc);
      pack_copy(*c->packer, buf, scalars_be + off * 8, cnt * 32);
      if (hipMemcpyAsync(wsc + off * 8, buf, cnt * 32, hipMemcpyHostToDevice, c->copy_stream) != hipSuccess)
        return fail(MSM_ERR_HIP);
      if ((rc = pin_give(c, k % NPIN, c->copy_stream)) != MSM_OK) return fail(rc);
    }
    if (hipEventRecord(sl.ev_in, c->copy_stream) != hipSuccess || hipStreamWaitEvent(sl.stream, sl.ev_in, 0) != hipSuccess)
      return fail(MSM_ERR_HIP);
    if ((rc = launch_parts(c, pl, bp, bs, si, PART_SORT, pts)) != MSM_OK) return fail(rc);
    bool tb = false;
    uint32_t* wp = w.wire_pts.as<uint32_t>();
    for (size_t p0 = 0; p0 < n; p0 += UPLOAD_PTS_PIECE, k++) {
      const size_t cnt = std::min(UPLOAD_PTS_PIECE, n - p0);
      void* buf;
      if ((rc = pin_take(c, k % NPIN, cnt * 96, &buf)) != MSM_OK) return fail(rc);
      uint32_t fmt = PT_FMT_XY;
      if (!pack_records(*c->packer, static_cast<uint32_t*>(buf), points_be + p0 * 32, cnt, PT_FMT_XY, &tb)) {
        fmt = PT_FMT_XYZ;
        pack_records(*c->packer, static_cast<uint32_t*>(buf), points_be + p0 * 32, cnt, PT_FMT_XYZ, &tb);
      }
      const size_t pw = pt_fmt_slots(fmt) * 4;
      if (hipMemcpyAsync(wp + p0 * 24, buf, cnt * pw * 4, hipMemcpyHostToDevice, c->copy_stream) != hipSuccess)
        return fail(MSM_ERR_HIP);
      if ((rc = pin_give(c, k % NPIN, c->copy_stream)) != MSM_OK) return fail(rc);
      hipEvent_t e = c->ev_chunk[k % NCHUNK_EV];
      if (hipEventRecord(e, c->copy_stream) != hipSuccess || hipStreamWaitEvent(sl.stream, e, 0) != hipSuccess)
        return fail(MSM_ERR_HIP);
      launch_prepare(wp + p0 * 24, pts + p0 * PRE_WORDS, (uint32_t)cnt, w.err.as<uint32_t>(), prep_nt(n), sl.stream, fmt);
      if (hipGetLastError() != hipSuccess) return fail(MSM_ERR_HIP);
    }
    t_bad = tb;
  } else {
    if ((rc = upload_scalars(c, scalars_be, n, w.wire_sc.as<uint32_t>(), sl.stream, sl.ev_in)) != MSM_OK)
      return fail(rc);
    if ((rc = launch_parts(c, pl, bp, bs, si, PART_SORT, pts)) != MSM_OK) return fail(rc);
    if ((rc = upload_points(c, points_be, n, w.wire_pts.as<uint32_t>(), pts, w.err.as<uint32_t>(), sl.stream)) !=
        MSM_OK)
      return fail(rc);
  }
  if ((rc = launch_parts(c, pl, bp, bs, si, PART_ACC | PART_POST, pts)) != MSM_OK) return fail(rc);
  rc = finish_lone(c, si, result);
  return rc == MSM_OK && t_bad ? MSM_ERR_COORD_RANGE : rc;
}

// MSMs kept in flight by the pipelined entries.  Small MSMs are latency-bound (their reduction
// and sort kernels leave most of the chip idle), so several run side by side; MSM_SLOTS
// overrides (1 = everything in order on one stream: clean per-kernel profiles), and so does the
// MSM_FLAG_SERIAL option flag.
int pipeline_slots(size_t n, const msm_opts* o) {
  if (o && (o->flags & MSM_FLAG_SERIAL)) return 1;
  static const int env = getenv("MSM_SLOTS") ? atoi(getenv("MSM_SLOTS")) : 0;
  if (env >= 1) return std::min(env, NSLOT);
  (void)n;
  // Two launches in flight.  Round 1 measured three best (one or two MSMs per launch); with two
  // to four MSMs per launch and the one-wave-per-SIMD reduction, two beat three at every size
  // (profiles/r2s_slots_ab.jsonl, ms per MSM, 50 steps: 2^16 0.137 vs 0.145-0.175, 2^17
  // 0.210-0.236 vs 0.219-0.222, 2^18 0.354-0.358 vs 0.374, 2^20 1.083-1.114 vs 1.095-1.128).
  return 2;
}

// MSMs per launch (batch) for the pipelined entries: the latency-bound kernels (reduction trees,
// scans, small sorts) of two MSMs fill the machine together.  Measured on MI355X
// (tools/batch_sweep.sh, ms per MSM, batch 1 -> 2): 2^16 0.218 -> 0.162, 2^17 0.273 -> 0.247,
// 2^18 0.420 -> 0.381, 2^19 0.679 -> 0.638, 2^20 1.162 -> 1.136.  Four per launch up to 2^18,
// measured once the reduction kept one wave per SIMD and two launches are in flight
// (profiles/r2mn_*, r2y_*): 2^17 0.268 -> 0.248, 2^18 0.363 -> 0.347 ms per MSM; 2^19 +1.5%,
// 2^20 +4.5% (kept at two).  Eight up to 2^16: a four-MSM 2^16 launch costs ~0.64 ms of pipeline
// time and an eight-MSM one ~1.04 (profiles/r3/batch_sizes.txt: 0.13 against 0.16 ms per MSM over
// 50 MSMs, the last launch padded; 2^17 and 2^18 are 2-13% slower with eight), so eight is taken
// whenever its launches, padded last one included, cost less: ceil(count/8) * 13 < ceil(count/4) * 8.
// Two also above 2^20, up to 2^21: 2^21 measured 2.31-2.33 ms per MSM with two against 2.36-2.43
// with one, and one extra point past 2^20 cost 17% with one per launch
// (1.194 against 1.023 ms, profiles/r4/pipelined_sizes.jsonl).  MSM_BATCH overrides (1..MSM_MAX_BATCH).
uint32_t pipeline_batch(size_t n, size_t count) {
  static const int env = getenv("MSM_BATCH") ? atoi(getenv("MSM_BATCH")) : 0;
  uint32_t nm = env >= 1 ? (uint32_t)std::min(env, (int)MSM_MAX_BATCH)
                         : (n <= (1u << 18) ? 4u : n <= (1u << 21) ? 2u : 1u);
  if (env < 1 && n <= (1u << 16) && count >= 8 && (count + 7) / 8 * 13 < (count + 3) / 4 * 8) nm = 8;
  return (uint32_t)std::max<size_t>(1, std::min<size_t>(nm, count));
}

// Whether a host-input pipelined run starts its last launch's sort before that launch's points
// upload (MSM_HOST_SORT_EARLY=0 disables, for A/B runs).
bool host_sort_early() {
  static const bool on = !(getenv("MSM_HOST_SORT_EARLY") && atoi(getenv("MSM_HOST_SORT_EARLY")) == 0);
  return on;
}

// Staggered pipelined launches (default; MSM_STAGGER=0 turns them off): launch j's preparation and
// sort wait for launch j-1's accumulation -- the stream waits on the previous slot's ev_acc1,
// recorded by an event node right after k_accumulate inside that launch's graph -- so they run
// beside j-1's bucket reduction (one wave per SIMD, no LDS) instead of being dispatched into the
// accumulation that holds every CU.  Unstaggered, the two slots drifted into running their
// accumulations side by side and their sorts and reductions side by side (kernel traces t11,
// t19); staggered, 2^20 pipelined 0.966-0.973 against 0.985-1.013 ms per MSM (sessions t20-t23,
// DESIGN.md §4.1).  Device-resident inputs only: host-input launches are paced by their uploads.
// (MSM_STAGGER=2 staggers host-input launches too, for A/B runs.)
int stagger_launches() {
  static const int v = getenv("MSM_STAGGER") ? atoi(getenv("MSM_STAGGER")) : 1;
  return v < 0 ? 0 : v > 2 ? 2 : v;
}

// Where the inputs of one pipelined run come from.
struct ManyInputs {
  enum Kind { DEVICE, HOST } kind = DEVICE;
  const uint32_t* const* points = nullptr;  // per MSM (ignored when shared_points is set)
  const uint32_t* const* scalars = nullptr;
  const uint32_t* shared_points = nullptr;  // one base vector for every MSM (prover batch)
  uint32_t batch = 0;                        // MSMs per launch (0: pipeline_batch's choice)
  const size_t* lens = nullptr;  // host inputs: real points per MSM (<= n; the rest is padded on
                                 // the device with identity points and zero scalars); null: all n
  const uint32_t* const* dev_points = nullptr;  // host inputs: per MSM, the device buffer (n points,
                                                // its own, never reused in the call) their points are
                                                // uploaded into instead of the slot's wire buffer
  bool packed = false;  // host points packed by the library's threads into pinned staging (x|y, or
                        // x|y|z for a launch with some z != 1) and copied into dev_points (24 words
                        // of room per point) or the slots' wire buffers; the launch's
                        // k_prepare_points reads that format
  const uint32_t* const* dev_scalars = nullptr;  // host inputs whose scalars are already on the
                                                 // device (n + padding words per MSM): no scalar upload
};

// `count` MSMs of n points each, pipelined over pipeline_slots slots, each with its own stream and
// workspace, in launches of pipeline_batch MSMs (the last launch is padded by repeating its last
// MSM, whose extra results are dropped): later launches are enqueued before the host finishes
// launch j, so the host tail (window Horner) of one overlaps the device work of the next, and
// the launches' kernels overlap on the device (the latency-bound reduction of one beside
// another's sort and accumulation).  Host inputs are uploaded on the copy stream into the
// slot's wire buffers, overlapping the other slots' kernels.  A shared base vector is prepared
// once, before the first launch, and every launch reads its records.  Results go out affine (16
// words each) or, with `projective`, as X|Y|T|Z partials (32 words).
int run_many(DevCtx* c, const ManyInputs& in, size_t n, size_t count, const msm_opts* o, hipStream_t user_stream,
             uint32_t* out_be, bool projective, Pt* out_pts = nullptr) {
  auto emit = [&](const Pt& r, size_t b) {
    if (out_pts)
      out_pts[b] = r;
    else if (projective)
      pt_to_be_xyzt(r, out_be + 32 * b);
    else
      pt_to_be_affine(r, out_be + 16 * b);
  };
  if (n == 0) {
    for (size_t b = 0; b < count; b++) emit(pt_identity(), b);
    return MSM_OK;
  }
  const bool shared = in.shared_points != nullptr;
  const bool host = in.kind == ManyInputs::HOST;
  for (size_t b = 0; b < count; b++)
    if ((!shared && !in.points[b]) || !in.scalars[b]) return MSM_ERR_INVALID_ARG;
  // the batch's BatchPtrs hold MSM_MAX_BATCH entries: never more MSMs per launch than that
  const uint32_t nm = (uint32_t)std::min<size_t>(
      in.batch ? std::min<size_t>(in.batch, count) : pipeline_batch(n, count), MSM_MAX_BATCH);
  const size_t nbatch = (count + nm - 1) / nm;
  Plan pl;
  int rc = make_plan(n, o, c->shape, &pl, count > 1, nm, shared);
  if (rc != MSM_OK) return rc;
  // host inputs: one more launch in flight, so its upload queues behind the running ones
  // (2^20 msm_compute 4.21 -> 4.05 ms with three, profiles/r2t_*; device inputs are best with two)
  const int want = pipeline_slots(n, o) + (host && !(o && (o->flags & MSM_FLAG_SERIAL)) && !getenv("MSM_SLOTS") ? 1 : 0);
  const int nslot = nbatch > 1 ? (int)std::min<size_t>(nbatch, (size_t)std::min(want, NSLOT)) : 1;
  for (int si = 0; si < nslot; si++) {
    c->slot[si].pipelined = nslot > 1;
    if ((rc = ensure_workspace(c, pl, si)) != MSM_OK) return rc;
    if (host) {
      Workspace& w = c->slot[si].ws;
      if ((!shared && (rc = w.wire_pts.ensure((size_t)nm * n * 128)) != MSM_OK) ||
          (rc = w.wire_sc.ensure((size_t)nm * n * 32)) != MSM_OK)
        return rc;
    }
  }
  if ((rc = order_after_user(c, user_stream, nslot)) != MSM_OK) return rc;
  auto fail0 = [&](int code) {  // before the uploader starts
    hipStreamSynchronize(c->copy_stream);
    for (int k = 0; k < nslot; k++) hipStreamSynchronize(c->slot[k].stream);
    return code;
  };
  uint32_t* pts_shared = nullptr;
  if (shared) {
    // the base vector's records, prepared once on slot 0's stream; the other slots wait for them
    if ((rc = c->shared_pts.ensure(n * PRE_WORDS * 4)) != MSM_OK) return rc;
    pts_shared = c->shared_pts.as<uint32_t>();
    Slot& s0 = c->slot[0];
    if (host) {
      if ((rc = s0.ws.wire_pts.ensure(n * 128)) != MSM_OK) return rc;
      rc = upload_points(c, in.shared_points, n, s0.ws.wire_pts.as<uint32_t>(), pts_shared, s0.ws.err.as<uint32_t>(),
                         s0.stream);
      if (rc != MSM_OK) return fail0(rc);
    } else {
      launch_prepare(in.shared_points, pts_shared, (uint32_t)n, s0.ws.err.as<uint32_t>(), prep_nt(n), s0.stream);
      if (hipGetLastError() != hipSuccess) return fail0(MSM_ERR_HIP);
    }
    if (hipEventRecord(c->ev_shared, s0.stream) != hipSuccess) return fail0(MSM_ERR_HIP);
    for (int si = 1; si < nslot; si++)
      if (hipStreamWaitEvent(c->slot[si].stream, c->ev_shared, 0) != hipSuccess) return fail0(MSM_ERR_HIP);
  }
  // The inputs of launch j (per-MSM pointers, or the slot's wire buffers for host inputs) and the
  // number of real (not padding) MSMs in it.
  auto launch_inputs = [&](size_t j, BatchPtrs* bp, BatchPtrs* bs) -> uint32_t {
    Slot& sl = c->slot[j % nslot];
    const uint32_t nreal = (uint32_t)std::min<size_t>(nm, count - j * nm);
    *bp = BatchPtrs{};
    *bs = BatchPtrs{};
    for (uint32_t m = 0; m < MSM_MAX_BATCH; m++) {
      const size_t b = std::min(j * nm + std::min<uint32_t>(m, nm - 1), count - 1);
      bp->p[m] = shared ? in.shared_points : in.points[b];
      bs->p[m] = in.scalars[b];
      if (host) {  // padding MSMs of a short last launch read the last real MSM's wire buffers
        const uint32_t mr = std::min<uint32_t>(m, nreal - 1);
        bs->p[m] = in.dev_scalars ? in.dev_scalars[j * nm + mr] : sl.ws.wire_sc.as<uint32_t>() + (size_t)mr * n * 8;
        if (!shared)
          bp->p[m] = in.dev_points ? in.dev_points[j * nm + mr] : sl.ws.wire_pts.as<uint32_t>() + (size_t)mr * n * 32;
      }
    }
    return nreal;
  };
  // Host inputs of launch j into its slot's wire buffers, on the copy stream: the scalars, the
  // device padding of short MSMs, an event on the scalars (up_ev[2 j]), the points, an event on all
  // of them (up_ev[2 j + 1]).  MSMs whose host arrays are adjacent (the slices of run_host_split) go up in one
  // copy per array: each pageable hipMemcpyAsync costs ~20 us of copy-engine idle time between
  // transfers.  The padding MSMs of a short last launch upload nothing; a short MSM (in.lens) goes
  // up alone and its tail is padded on the device.
  const bool packed = host && in.packed && !shared && pin_ring_ready(c, (size_t)nm * n * 128);
  // run_host_split sized its own point buffers (in.dev_points) for packed records: no unpacked
  // fallback into them (it checked the ring itself; only a failure since then lands here)
  if (host && in.packed && !shared && !packed && in.dev_points) return MSM_ERR_HIP;
  std::vector<uint32_t> launch_fmt(nbatch, PT_FMT_WIRE);  // the packed launches' point formats
  std::atomic<bool> t_bad{false};                         // a packed t >= p (MSM_ERR_COORD_RANGE)
  if (packed) ctx_packer(c);
  auto upload_launch = [&](size_t j, const std::function<void()>& scalars_done) -> int {
    BatchPtrs bp, bs;
    const uint32_t nreal = launch_inputs(j, &bp, &bs);
    auto len_of = [&](size_t b) { return in.lens ? std::min(in.lens[b], n) : n; };
    if (packed) {
      // the launch's scalars, then its points, through pinned staging buffer j % NPIN (points at
      // [0, 24 nm n) words, scalars after them): the scalars first, each slice's into its
      // dev_scalars region, so the sort can start; the points as x|y if every z is 1, else x|y|z,
      // one copy per slice into its dev_points region; a short slice's padding in that format
      const int k = (int)(j % NPIN);
      void* buf;
      if (int rc = pin_take(c, k, (size_t)nm * n * 128, &buf)) return rc;
      uint32_t* pb = static_cast<uint32_t*>(buf);
      uint32_t* psc = pb + (size_t)nm * n * 24;
      for (uint32_t m = 0; m < nreal; m++) {
        const size_t b = j * nm + m, len = len_of(b);
        if (!len) continue;
        pack_copy(*c->packer, psc + (size_t)m * n * 8, in.scalars[b], len * 32);
        if (hipMemcpyAsync(const_cast<uint32_t*>(bs.p[m]), psc + (size_t)m * n * 8, len * 32, hipMemcpyHostToDevice,
                           c->copy_stream) != hipSuccess)
          return MSM_ERR_HIP;
        // a short slice's scalar tail is zero before the sort may start (k_pad_identity below
        // pads its points)
        if (len < n && hipMemsetAsync(const_cast<uint32_t*>(bs.p[m]) + len * 8, 0, (n - len) * 32, c->copy_stream) !=
                           hipSuccess)
          return MSM_ERR_HIP;
      }
      HIPCHECK(hipEventRecord(c->up_ev[2 * j], c->copy_stream));
      scalars_done();
      // each slice's x|y goes up as soon as it is packed; a z != 1 anywhere in the launch repacks
      // every slice as x|y|z and sends it again over the same regions (stream order)
      uint32_t fmt = PT_FMT_XY;
      bool tb = false;
      auto send = [&](uint32_t m) -> bool {
        const size_t len = len_of(j * nm + m), pw = pt_fmt_slots(fmt) * 4;
        return !len || hipMemcpyAsync(const_cast<uint32_t*>(bp.p[m]), pb + (size_t)m * n * pw, len * pw * 4,
                                      hipMemcpyHostToDevice, c->copy_stream) == hipSuccess;
      };
      for (uint32_t m = 0; m < nreal && fmt == PT_FMT_XY; m++) {
        if (!pack_records(*c->packer, pb + (size_t)m * n * 16, in.points[j * nm + m], len_of(j * nm + m), PT_FMT_XY,
                          &tb))
          fmt = PT_FMT_XYZ;
        else if (!send(m))
          return MSM_ERR_HIP;
      }
      if (fmt == PT_FMT_XYZ)
        for (uint32_t m = 0; m < nreal; m++) {
          const size_t b = j * nm + m;
          pack_records(*c->packer, pb + (size_t)m * n * 24, in.points[b], len_of(b), PT_FMT_XYZ, &tb);
          if (!send(m)) return MSM_ERR_HIP;
        }
      if (tb) t_bad.store(true);
      for (uint32_t m = 0; m < nreal; m++) {
        const size_t len = len_of(j * nm + m);
        if (len < n) {
          hipLaunchKernelGGL(k_pad_identity, dim3(grid_for((n - len) * (pt_fmt_slots(fmt) + 2), 256)), dim3(256), 0,
                             c->copy_stream, const_cast<uint32_t*>(bp.p[m]) + len * pt_fmt_slots(fmt) * 4,
                             const_cast<uint32_t*>(bs.p[m]) + len * 8, (uint32_t)(n - len), fmt);
          if (hipGetLastError() != hipSuccess) return MSM_ERR_HIP;
        }
      }
      if (int rc = pin_give(c, k, c->copy_stream)) return rc;
      launch_fmt[j] = fmt;
      HIPCHECK(hipEventRecord(c->up_ev[2 * j + 1], c->copy_stream));
      return MSM_OK;
    }
    auto up = [&](const uint32_t* const* src, const BatchPtrs& dst, size_t per) -> bool {
      for (uint32_t m0 = 0; m0 < nreal;) {
        const size_t b0 = std::min(j * nm + m0, count - 1);
        const uint32_t* h0 = src[b0];
        uint32_t m1 = m0 + 1;
        if (len_of(b0) == n)
          while (m1 < nreal && len_of(j * nm + m1) == n && src[j * nm + m1] == h0 + (size_t)(m1 - m0) * n * per) m1++;
        const size_t words = (m1 - m0 == 1 ? len_of(b0) : (size_t)(m1 - m0) * n) * per;
        if (words && hipMemcpyAsync(const_cast<uint32_t*>(dst.p[m0]), h0, words * 4, hipMemcpyHostToDevice,
                                    c->copy_stream) != hipSuccess)
          return false;
        m0 = m1;
      }
      return true;
    };
    if (!in.dev_scalars && !up(in.scalars, bs, 8)) return MSM_ERR_HIP;
    for (uint32_t m = 0; m < nreal && !shared; m++) {
      const size_t len = len_of(std::min(j * nm + m, count - 1));
      if (len < n) {
        hipLaunchKernelGGL(k_pad_identity, dim3(grid_for((n - len) * 10, 256)), dim3(256), 0, c->copy_stream,
                           const_cast<uint32_t*>(bp.p[m]) + len * 32, const_cast<uint32_t*>(bs.p[m]) + len * 8,
                           (uint32_t)(n - len), PT_FMT_WIRE);
        if (hipGetLastError() != hipSuccess) return MSM_ERR_HIP;
      }
    }
    HIPCHECK(hipEventRecord(c->up_ev[2 * j], c->copy_stream));
    scalars_done();
    if (!shared && !up(in.points, bp, 32)) return MSM_ERR_HIP;
    HIPCHECK(hipEventRecord(c->up_ev[2 * j + 1], c->copy_stream));
    return MSM_OK;
  };
  // With host inputs and more than one launch, a helper thread (the uploader) issues every
  // launch's copies back to back while this thread enqueues the launches and runs the host tails:
  // a pageable hipMemcpyAsync returns only once its data is staged, so copies issued from the
  // launching thread left the copy engine idle for every graph launch and host tail between them
  // (~120 us per launch, profiles/r4/e2e_timeline_before.txt).  A slot's wire buffers are rewritten
  // only after its previous launch is done with them: the copy stream waits for that launch's
  // ev_done, recorded once this thread has enqueued it (`enqueued`).
  const bool uploader = host && nbatch > 1;
  // Inputs uploaded into buffers of their own (dev_points / dev_scalars, never reused within the
  // call) need no wait for a slot's previous launch: the copies then run back to back.
  const bool own_buffers = (shared || in.dev_points) && in.dev_scalars;
  if (host) {
    while (c->up_ev.size() < 2 * nbatch) {
      hipEvent_t e;
      if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return MSM_ERR_HIP;
      c->up_ev.push_back(e);
    }
  }
  std::atomic<size_t> sc_ready{0}, up_ready{0}, enqueued{0};
  std::atomic<int> up_rc{MSM_OK};
  std::atomic<bool> up_stop{false};
  std::thread up_th;
  auto wait_for = [&](std::atomic<size_t>& v, size_t want) -> bool {  // false: the uploader failed
    for (uint32_t spins = 0; v.load(std::memory_order_acquire) < want; spins++) {
      if (up_rc.load() != MSM_OK) return false;
      if (spins > 256) std::this_thread::yield();
      else _mm_pause();
    }
    return true;
  };
  auto stop_uploader = [&] {
    up_stop.store(true);
    if (up_th.joinable()) up_th.join();
  };
  // the device context's tail helpers take the last launch's host tails (armed once it is enqueued)
  TailCrew* crew = tail_helpers() > 0 ? ctx_crew(c) : nullptr;
  bool crew_armed = false;
  // and the pool the earlier launches' tails (their terms copied out per launch)
  HornerPool* pool = ctx_pool(c);
  std::vector<std::vector<uint32_t>> launch_terms(pool ? nbatch : 0);
  auto fail = [&](int code) {
    if (crew_armed) crew->disarm();  // no terms will come
    crew_armed = false;
    if (pool) pool->wait_all();  // its jobs read launch_terms
    stop_uploader();
    hipStreamSynchronize(c->copy_stream);
    for (int k = 0; k < nslot; k++) hipStreamSynchronize(c->slot[k].stream);
    return code;
  };
  if (uploader) {
    up_th = std::thread([&] {
      hipSetDevice(c->device);
      for (size_t j = 0; j < nbatch && !up_stop.load(); j++) {
        int urc = MSM_OK;
        if (j >= (size_t)nslot && !own_buffers) {
          // launch j - nslot (the slot's previous one) must have been enqueued before its
          // ev_done can be waited for
          while (enqueued.load(std::memory_order_acquire) < j - nslot + 1 && !up_stop.load()) std::this_thread::yield();
          if (up_stop.load()) break;
          if (hipStreamWaitEvent(c->copy_stream, c->slot[j % nslot].ev_done, 0) != hipSuccess) urc = MSM_ERR_HIP;
        }
        if (urc == MSM_OK) urc = upload_launch(j, [&] { sc_ready.store(j + 1, std::memory_order_release); });
        if (urc != MSM_OK) {
          up_rc.store(urc);
          break;
        }
        up_ready.store(j + 1, std::memory_order_release);
      }
    });
  }
  // Launch j goes to slot j % nslot.  Its previous occupant, launch j - nslot, is waited for and
  // its window terms copied out just before; the host tail (window Horner) of launch j - nslot
  // runs after j is enqueued, so the device holds nslot launches while the host works
  // (otherwise launches that finish together leave the device idle for a Horner each).
  std::vector<uint32_t> terms;
  const bool stagger = nslot > 1 && c->profiling != 1 && stagger_launches() > (host ? 1 : 0);
  for (int si = 0; si < NSLOT; si++) c->slot[si].stagger = stagger && si < nslot;
  for (size_t j = 0; j < nbatch + nslot; j++) {
    const bool have = j >= (size_t)nslot;
    const size_t f = have ? j - nslot : 0;
    // the last launch's terms stay in `terms` (its tails run here, over the crew); the pool's jobs
    // read their launch's own copy
    std::vector<uint32_t>* tdst = pool && have && f + 1 < nbatch ? &launch_terms[f] : &terms;
    if (have && (rc = finish_msm(c, (int)(f % nslot), nullptr, tdst)) != MSM_OK) return fail(rc);
    if (j < nbatch) {
      const int si = (int)(j % nslot);
      Slot& sl = c->slot[si];
      BatchPtrs bp, bs;
      launch_inputs(j, &bp, &bs);
      const int parts = shared ? (PART_SORT | PART_ACC | PART_POST) : PART_ALL;
      uint32_t* pts = shared ? pts_shared : sl.ws.pts.as<uint32_t>();
      // The last launch's bucket sort starts on its scalars while its points upload: the sort then
      // leaves the call's tail (earlier launches overlap the next uploads anyway).
      const bool sort_early = host && !shared && j + 1 == nbatch && nbatch > 1 && host_sort_early();
      if (host) {
        if (!uploader && (rc = upload_launch(j, [] {})) != MSM_OK) return fail(rc);
        if (sort_early) {
          if (uploader && !wait_for(sc_ready, j + 1)) return fail(up_rc.load());
          if (hipStreamWaitEvent(sl.stream, c->up_ev[2 * j], 0) != hipSuccess) return fail(MSM_ERR_HIP);
          sl.pl = pl;
          if ((rc = launch_parts(c, pl, bp, bs, si, PART_SORT, pts)) != MSM_OK) return fail(rc);
        }
        if (uploader && !wait_for(up_ready, j + 1)) return fail(up_rc.load());
        if (hipStreamWaitEvent(sl.stream, c->up_ev[2 * j + 1], 0) != hipSuccess) return fail(MSM_ERR_HIP);
      }
      Plan plj = pl;
      plj.pfmt = packed ? launch_fmt[j] : PT_FMT_WIRE;  // set by the uploader before up_ready
      sl.pl = plj;
      const int lp = sort_early ? parts & ~PART_SORT : parts;
      // staggered: launch j's preparation and sort after launch j-1's accumulation
      if (stagger && j > 0 && hipStreamWaitEvent(sl.stream, c->slot[(j - 1) % nslot].ev_acc1, 0) != hipSuccess)
        return fail(MSM_ERR_HIP);
      if ((rc = launch_parts(c, plj, bp, bs, si, lp, pts)) != MSM_OK) return fail(rc);
      enqueued.store(j + 1, std::memory_order_release);
      if (crew && j + 1 == nbatch) {
        crew->arm();  // spins while the device runs the last launch
        crew_armed = true;
      }
    }
    if (have) {
      const uint32_t k = (uint32_t)std::min<size_t>(nm, count - f * nm);
      Pt res[MSM_MAX_BATCH];
      if (pool && f + 1 < nbatch) {
        // off this thread: the next launch's enqueue must not wait for these tails
        const uint32_t* tp = launch_terms[f].data();
        for (uint32_t m = 0; m < k; m++)
          pool->push([&, tp, f, m] { emit(horner_tail(pl, tp, m), f * nm + m); });
        continue;
      }
      if (crew_armed && f + 1 == nbatch) {
        // the last launch's tails are the pipeline's drain, on the critical path of the call: their
        // window sums over the device context's helpers, the k outer Horners side by side
        crew->run_batch(pl, terms.data(), k, res);
        crew_armed = false;
      } else {
        // earlier launches' tails overlap the device's next launches: one host thread per MSM
        std::thread th[MSM_MAX_BATCH];
        for (uint32_t m = 1; m < k; m++) th[m] = std::thread([&, m] { res[m] = horner_tail(pl, terms.data(), m); });
        res[0] = horner_tail(pl, terms.data(), 0);
        for (uint32_t m = 1; m < k; m++) th[m].join();
      }
      for (uint32_t m = 0; m < k; m++) emit(res[m], f * nm + m);
    }
  }
  if (pool) pool->wait_all();
  stop_uploader();  // its last copies were waited for by the last launch
  return t_bad.load() ? MSM_ERR_COORD_RANGE : MSM_OK;
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

// Lock the device context of `opts` and run `fn(ctx)` with its device current.
template <typename F>
int on_device(const msm_opts* opts, F&& fn) {
  DevCtx* c;
  int rc = with_device(opts, &c);
  if (rc != MSM_OK) return rc;
  std::lock_guard<std::mutex> lk(c->mu);
  DeviceGuard g(c->device);
  c->profiling = g_profiling.load();
  begin_call(c);
  rc = fn(c);
  end_call(c);
  return rc;
}

// Host-input points per slice of a split MSM (run_host_split), and MSMs per launch there.
size_t host_piece() {
  static const int lg = getenv("MSM_HOST_PIECE_LOG") ? atoi(getenv("MSM_HOST_PIECE_LOG")) : 17;
  static const size_t v = (size_t)1 << (lg >= 10 && lg <= 24 ? lg : 17);
  return v;
}
uint32_t host_batch() {  // two slices per launch: measured best for 2^17 slices
  static const int env = getenv("MSM_HOST_NM") ? atoi(getenv("MSM_HOST_NM")) : 2;
  return (uint32_t)std::min(std::max(env, 1), (int)MSM_MAX_BATCH);
}

// One large MSM of host-resident inputs as G point-slices (G <= 16, slices of ~2^17 points):
// MSM = sum_g MSM(slice g), the reference's own shard/join identity (submission.ts:116-154,
// lib.rs:240-253) inside one GPU.  The slices go through the pipelined entry: slice g+1 uploads
// on the copy stream while slice g runs, so the PCIe transfer -- the bulk of a host-input MSM --
// overlaps all the compute but the last launch's; the partials are joined with G - 1 adds.  When
// G does not divide n the last slice is short: it is padded on the device (identity points, zero
// scalars) rather than run as a separate remainder MSM after the others.
// Whether the split uploads all the scalars in one copy before the first launch's points
// (MSM_HOST_SC_FIRST=0: per launch, beside its points): one copy instead of one per launch, so
// fewer ~20-us gaps between copies, and every launch's sort can start as soon as it is enqueued.
bool host_scalars_first() {
  static const bool on = !(getenv("MSM_HOST_SC_FIRST") && atoi(getenv("MSM_HOST_SC_FIRST")) == 0);
  return on;
}

// Points per slice of the split's last launch (MSM_HOST_TAIL_LOG; 0 = none): round 4 measured
// such tails slower (one more launch, and the copies waited for slots); re-measured with the
// call's own upload buffers.
size_t host_tail() {
  static const int lg = getenv("MSM_HOST_TAIL_LOG") ? atoi(getenv("MSM_HOST_TAIL_LOG")) : 0;
  static const size_t v = lg > 0 && lg <= 24 ? (size_t)1 << lg : 0;
  return v;
}

bool host_own_points() {
  static const bool on = !(getenv("MSM_HOST_OWN_PTS") && atoi(getenv("MSM_HOST_OWN_PTS")) == 0);
  return on;
}

int run_host_split(DevCtx* c, const uint32_t* points_be, const uint32_t* scalars_be, size_t n, const msm_opts* o,
                   Pt* result) {
  // G <= 16 balanced slices of s points, a whole number of launches of nmb slices (every slice
  // is an MSM of s points to the pipelined entry; in.lens: a short slice is padded on the device
  // with identity points and zero scalars, which add no bucket entries).  (Short tail slices for
  // the last launch -- its compute is what is left after the last upload -- measured slower: one
  // more launch costs more than the shorter tail saves)
  // With MSM_HOST_TAIL_LOG = k the last launch instead holds nmb short slices of 2^k points (the
  // body then n - nmb 2^k points in Gb balanced slices): its compute after the last upload shrinks.
  const uint32_t nmb = host_batch();
  size_t t = host_tail();
  if (t * nmb * 8 > n) t = 0;  // small MSMs: no tail launch
  size_t body, Gb, s;
  for (;;) {
    body = n - t * nmb;
    Gb = std::max<size_t>(1, std::min<size_t>(16, body / host_piece()));
    Gb = (Gb + nmb - 1) / nmb * nmb;
    s = (body + Gb - 1) / Gb;
    // every slice runs as an MSM of s points (run_many sizes its buffers and clamps lengths by s):
    // a tail slice longer than a body slice would lose points, so then there is no tail launch
    if (t <= s) break;
    t = 0;
  }
  std::vector<size_t> offs, lens;
  for (size_t g = 0; g < Gb; g++) {
    offs.push_back(std::min(g * s, body));
    lens.push_back(g * s < body ? std::min(s, body - g * s) : 0);  // 0 only for tiny MSM_HOST_PIECE_LOG overrides
  }
  for (size_t g = 0; t && g < nmb; g++) {
    offs.push_back(body + g * t);
    lens.push_back(t);
  }
  const size_t G = offs.size();
  std::vector<const uint32_t*> pp(G), ss(G);
  for (size_t g = 0; g < G; g++) {
    pp[g] = points_be + offs[g] * 32;
    ss[g] = scalars_be + offs[g] * 8;
  }
  ManyInputs in;
  in.kind = ManyInputs::HOST;
  in.points = pp.data();
  in.scalars = ss.data();
  in.batch = nmb;
  in.lens = lens.data();
  std::vector<const uint32_t*> dsc(G);
  const bool pack =
      host_scalars_first() && host_own_points() && host_pack() && pin_ring_ready(c, (size_t)nmb * s * 128);
  if (pack) {
    // packed: every launch's scalars and points go up through the pinned ring from the uploader,
    // scalars first (run_many), into these device regions (slice g at g s)
    if (int rc = c->host_sc.ensure(G * s * 32)) return rc;
    ctx_packer(c);
    for (size_t g = 0; g < G; g++) dsc[g] = c->host_sc.as<uint32_t>() + g * s * 8;
    in.dev_scalars = dsc.data();
  } else if (host_scalars_first()) {
    // slice g's scalars at g s in one device buffer (s words each, the tail of a short slice is
    // its device padding): the run of full slices at the front goes up in one copy, every other
    // slice in its own
    if (int rc = c->host_sc.ensure(G * s * 32)) return rc;
    uint32_t* base = c->host_sc.as<uint32_t>();
    for (size_t g = 0; g < G;) {
      size_t h = g + 1;
      if (lens[g] == s)
        while (h < G && lens[h] == s && offs[h] == offs[g] + (h - g) * s) h++;
      const size_t words = (h - g == 1 ? lens[g] : (h - g) * s) * 8;
      if (words && hipMemcpyAsync(base + g * s * 8, scalars_be + offs[g] * 8, words * 4, hipMemcpyHostToDevice,
                                  c->copy_stream) != hipSuccess) {
        hipStreamSynchronize(c->copy_stream);
        return MSM_ERR_HIP;
      }
      g = h;
    }
    for (size_t g = 0; g < G; g++) dsc[g] = base + g * s * 8;
    in.dev_scalars = dsc.data();
  }
  // the points into a buffer of the call's own as well (slice g at g s, with room for its device
  // padding): the uploader then never waits for a slot's previous launch before a copy, so the
  // copy engine runs the whole upload back to back (MSM_HOST_OWN_PTS=0: the slots' wire buffers)
  std::vector<const uint32_t*> dpt(G);
  if (host_scalars_first() && host_own_points()) {
    // packed: room for the widest packed form, x|y|z (24 words per point)
    const size_t pw = pack ? 24 : 32;
    if (int rc = c->host_pts.ensure(G * s * pw * 4)) {
      hipStreamSynchronize(c->copy_stream);  // the scalar copy reads the caller's array
      return rc;
    }
    for (size_t g = 0; g < G; g++) dpt[g] = c->host_pts.as<uint32_t>() + g * s * pw;
    in.dev_points = dpt.data();
    in.packed = pack;
  }
  // The slices' window: that of a 2^17 slice (c = 15) whatever their length.  n not a multiple of
  // 2^18 makes slices a little short of 2^17 (2^20 - 524 points: 131,007), where pipelined_window
  // would pick c = 14 -- two more windows' sort and accumulation for a 2% shorter slice
  // (msm_compute 4.3-4.4 against 3.7 ms; tools/e2e_align_probe.py).
  // field by field: a caller built against the original 16-byte msm_opts owns no fields past
  // `flags`, and the later ones are read only under the flags that announce them (msm.h)
  msm_opts oc;
  memset(&oc, 0, sizeof(oc));
  if (o) {
    oc.window_bits = o->window_bits;
    oc.run_length = o->run_length;
    oc.device = o->device;
    oc.flags = o->flags;
    if (o->flags & MSM_FLAG_DEVICES) {
      oc.devices = o->devices;
      oc.n_devices = o->n_devices;
    }
    if (o->flags & MSM_FLAG_WINDOWS) {
      oc.window_lo = o->window_lo;
      oc.window_hi = o->window_hi;
    }
  }
  if (!oc.window_bits) oc.window_bits = pipelined_window(std::max(s, host_piece()));
  std::vector<Pt> part(G, pt_identity());
  int rc = run_many(c, in, s, G, &oc, nullptr, nullptr, true, part.data());
  if (rc != MSM_OK) {
    hipStreamSynchronize(c->copy_stream);  // the scalar copy reads the caller's array
    return rc;
  }
  Pt acc = part[0];
  for (size_t g = 1; g < G; g++) acc = pt_add(acc, part[g]);
  *result = acc;
  return MSM_OK;
}

int host_entry(const uint32_t* points_be, const uint32_t* scalars_be, size_t n, const msm_opts* opts, Pt* r) {
  if ((!points_be || !scalars_be) && n) return MSM_ERR_INVALID_ARG;
  static const bool split_off = getenv("MSM_HOST_SPLIT") && atoi(getenv("MSM_HOST_SPLIT")) == 0;
  return on_device(opts, [&](DevCtx* c) {
    // the split from 3 slices' worth: at 2^18 and 2.5 x 2^17 points one launch with its points in
    // 8 MiB pieces measured 5-10% faster, from 3 x 2^17 the split (tools/e2e_size_probe.py)
    if (!split_off && n >= 3 * host_piece())
      return run_host_split(c, points_be, scalars_be, n, opts, r);
    return run_host(c, points_be, scalars_be, n, opts, r);
  });
}

int device_entry(const uint32_t* d_points_be, const uint32_t* d_scalars_be, size_t n, const msm_opts* opts,
                 void* hip_stream, Pt* r) {
  if ((!d_points_be || !d_scalars_be) && n) return MSM_ERR_INVALID_ARG;
  return on_device(opts, [&](DevCtx* c) {
    return run_device(c, d_points_be, d_scalars_be, n, opts, (hipStream_t)hip_stream, r);
  });
}

int many_entry(const ManyInputs& in, size_t n, size_t count, const msm_opts* opts, void* hip_stream, uint32_t* out,
               bool projective) {
  if (!out || (!in.scalars && count) || (!in.points && !in.shared_points && count)) return MSM_ERR_INVALID_ARG;
  if (count == 0) return MSM_OK;
  return on_device(opts, [&](DevCtx* c) {
    return run_many(c, in, n, count, opts, (hipStream_t)hip_stream, out, projective);
  });
}

// ---- several devices in one call (msm_opts.flags & MSM_FLAG_DEVICES, include/msm.h) ----------
// The reference's one sharding precedent is inside compute_msm: the point vector split between
// the CPU and the GPU worker (submission.ts:116-154, gpu_worker.ts:9-18) and the two partials
// joined with point_add_affine (lib.rs:240-253).  Here the split is over gfx950 devices, one
// host thread each, and the join is projective (one EC add per shard, one inversion at the end).

bool devices_listed(const msm_opts* o) { return o && (o->flags & MSM_FLAG_DEVICES); }

// The listed ordinals, checked for shape (non-null, 1..MSM_MAX_DEVICES entries, non-negative,
// distinct) before any device is touched, then for being gfx950 devices.
int device_list(const msm_opts* o, std::vector<int>* devs) {
  devs->clear();
  if (!o->devices || o->n_devices == 0 || o->n_devices > MSM_MAX_DEVICES) return MSM_ERR_INVALID_ARG;
  for (uint32_t i = 0; i < o->n_devices; i++) {
    const int d = o->devices[i];
    if (d < 0 || std::find(devs->begin(), devs->end(), d) != devs->end()) return MSM_ERR_INVALID_ARG;
    devs->push_back(d);
  }
  for (int d : *devs) {
    DevCtx* c;
    if (int rc = get_ctx(d, &c)) return rc;
  }
  return MSM_OK;
}

// One listed device's single-device options (a window range carried over).
msm_opts opts_on(const msm_opts* o, int device) {
  msm_opts r{};
  r.window_bits = o->window_bits;
  r.run_length = o->run_length;
  r.flags = o->flags & ~MSM_FLAG_DEVICES;
  r.device = device;
  if (o->flags & MSM_FLAG_WINDOWS) {
    r.window_lo = o->window_lo;
    r.window_hi = o->window_hi;
  }
  return r;
}

// Contiguous shard i of D over n items: [n i / D, n (i+1) / D) (sizes differ by at most one).
void shard_range(size_t n, size_t i, size_t D, size_t* lo, size_t* hi) {
  *lo = n * i / D;
  *hi = n * (i + 1) / D;
}

// fn(i) for every listed device, device i on its own host thread (device 0 on the caller's); the
// first error in list order is returned once all have finished.
template <typename F>
int for_each_device(size_t D, F&& fn) {
  std::vector<int> rc(D, MSM_OK);
  std::vector<std::thread> th;
  for (size_t i = 1; i < D; i++)
    th.emplace_back([&, i] {
      t_call_devices = (int)D;
      rc[i] = fn(i);
    });
  const int own = t_call_devices;
  t_call_devices = (int)D;
  rc[0] = fn(0);
  t_call_devices = own;
  for (std::thread& t : th) t.join();
  for (int r : rc)
    if (r != MSM_OK) return r;
  return MSM_OK;
}

Pt join_partials(const std::vector<Pt>& part) {
  Pt acc = part[0];
  for (size_t i = 1; i < part.size(); i++) acc = pt_add(acc, part[i]);
  return acc;
}

// msm_compute / msm_compute_partial: each listed device uploads and reduces its own shard.
// (`devs` may repeat a device only through the test hook msm_test_sharded: its shards then run
// one after another on that device.)
int sharded_host(const uint32_t* points_be, const uint32_t* scalars_be, size_t n, const msm_opts* opts,
                 const std::vector<int>& devs, Pt* r) {
  const size_t D = devs.size();
  std::vector<Pt> part(D, pt_identity());
  int rc = for_each_device(D, [&](size_t i) {
    size_t lo, hi;
    shard_range(n, i, D, &lo, &hi);
    const msm_opts od = opts_on(opts, devs[i]);
    return host_entry(points_be + lo * 32, scalars_be + lo * 8, hi - lo, &od, &part[i]);
  });
  if (rc != MSM_OK) return rc;
  *r = join_partials(part);
  return MSM_OK;
}

int multi_host_entry(const uint32_t* points_be, const uint32_t* scalars_be, size_t n, const msm_opts* opts, Pt* r) {
  if (!devices_listed(opts)) return host_entry(points_be, scalars_be, n, opts, r);
  if ((!points_be || !scalars_be) && n) return MSM_ERR_INVALID_ARG;
  std::vector<int> devs;
  if (int rc = device_list(opts, &devs)) return rc;
  return sharded_host(points_be, scalars_be, n, opts, devs, r);
}

// Peer access of the current device `dev` to `owner`'s memory, enabled once per ordered pair, so
// the peer copies of peer_shard run device to device over xGMI (without it the runtime may stage
// them through host memory).  "Already enabled" (another library in the process, e.g. RCCL, did it)
// counts as enabled; a pair without peer support is remembered and left to the runtime's staged
// copies.  Returns 1 when enabled, 0 otherwise (msm_test_peer_state).
std::mutex g_peer_mu;
std::vector<int8_t> g_peer;  // [g_nhip * g_nhip]: 0 untried, 1 enabled, -1 unavailable

int enable_peer(int dev, int owner) {
  if (dev == owner) return 1;
  std::lock_guard<std::mutex> lk(g_peer_mu);
  if (g_nhip <= 0 || dev >= g_nhip || owner >= g_nhip) return 0;
  if (g_peer.size() != (size_t)g_nhip * g_nhip) g_peer.assign((size_t)g_nhip * g_nhip, 0);
  int8_t& st = g_peer[(size_t)dev * g_nhip + owner];
  if (st == 0) {
    int can = 0;
    st = -1;
    if (hipDeviceCanAccessPeer(&can, dev, owner) == hipSuccess && can) {
      const hipError_t e = hipDeviceEnablePeerAccess(owner, 0);
      if (e == hipSuccess || e == hipErrorPeerAccessAlreadyEnabled) st = 1;
    }
    (void)hipGetLastError();  // a refused enable leaves no sticky error for the next call
  }
  return st > 0 ? 1 : 0;
}

// One shard of device-resident inputs that live on another device: copied over xGMI (a peer copy
// on the slot's stream, peer access enabled first) into this device's wire buffers, then reduced
// here.
int peer_shard(int owner, const uint32_t* d_points, const uint32_t* d_scalars, size_t cnt, const msm_opts* od,
               Pt* r) {
  return on_device(od, [&](DevCtx* c) -> int {
    if (cnt == 0) {
      *r = msmh::pt_identity();
      return MSM_OK;
    }
    enable_peer(c->device, owner);
    Slot& sl = c->slot[0];
    Workspace& w = sl.ws;
    int rc;
    if ((rc = w.wire_pts.ensure(cnt * 128)) != MSM_OK || (rc = w.wire_sc.ensure(cnt * 32)) != MSM_OK) return rc;
    HIPCHECK(hipMemcpyPeerAsync(w.wire_pts.p, c->device, d_points, owner, cnt * 128, sl.stream));
    HIPCHECK(hipMemcpyPeerAsync(w.wire_sc.p, c->device, d_scalars, owner, cnt * 32, sl.stream));
    rc = run_device(c, w.wire_pts.as<uint32_t>(), w.wire_sc.as<uint32_t>(), cnt, od, nullptr, r);
    if (rc != MSM_OK) hipStreamSynchronize(sl.stream);  // the copies read the caller's buffers
    return rc;
  });
}

// msm_compute_device / msm_compute_device_partial: the inputs live on one listed device (the
// owner), which reduces its shard in place; every other listed device copies its shard over.
// (Through msm_test_sharded a device may be listed again: its later shards take the copy path.)
int sharded_device(const uint32_t* d_points_be, const uint32_t* d_scalars_be, size_t n, const msm_opts* opts,
                   void* hip_stream, const std::vector<int>& devs, Pt* r) {
  int owner = devs[0];
  if (n) {
    hipPointerAttribute_t ap{}, as{};
    if (hipPointerGetAttributes(&ap, d_points_be) != hipSuccess ||
        hipPointerGetAttributes(&as, d_scalars_be) != hipSuccess) {
      (void)hipGetLastError();
      return MSM_ERR_INVALID_ARG;
    }
    owner = ap.device;
    if (as.device != owner || std::find(devs.begin(), devs.end(), owner) == devs.end()) return MSM_ERR_INVALID_ARG;
  }
  if (hip_stream && n) {
    // the peer copies start on other devices' streams: the inputs' producers finish first
    DeviceGuard g(owner);
    HIPCHECK(hipStreamSynchronize(hip_stream == MSM_STREAM_NULL ? nullptr : (hipStream_t)hip_stream));
  }
  const size_t D = devs.size();
  const size_t own = (size_t)(std::find(devs.begin(), devs.end(), owner) - devs.begin());
  std::vector<Pt> part(D, pt_identity());
  int rc = for_each_device(D, [&](size_t i) {
    size_t lo, hi;
    shard_range(n, i, D, &lo, &hi);
    const msm_opts od = opts_on(opts, devs[i]);
    if (i == own)
      return device_entry(d_points_be + lo * 32, d_scalars_be + lo * 8, hi - lo, &od, nullptr, &part[i]);
    return peer_shard(owner, d_points_be + lo * 32, d_scalars_be + lo * 8, hi - lo, &od, &part[i]);
  });
  if (rc != MSM_OK) return rc;
  *r = join_partials(part);
  return MSM_OK;
}

int multi_device_entry(const uint32_t* d_points_be, const uint32_t* d_scalars_be, size_t n, const msm_opts* opts,
                       void* hip_stream, Pt* r) {
  if (!devices_listed(opts)) return device_entry(d_points_be, d_scalars_be, n, opts, hip_stream, r);
  if ((!d_points_be || !d_scalars_be) && n) return MSM_ERR_INVALID_ARG;
  std::vector<int> devs;
  if (int rc = device_list(opts, &devs)) return rc;
  return sharded_device(d_points_be, d_scalars_be, n, opts, hip_stream, devs, r);
}

// msm_compute_many / msm_compute_shared: a contiguous block of the MSMs per listed device
// (whole MSMs, nothing to join).  Device batches take one device.
int multi_many_entry(const ManyInputs& in, size_t n, size_t count, const msm_opts* opts, void* hip_stream,
                     uint32_t* out, bool projective) {
  if (!devices_listed(opts)) return many_entry(in, n, count, opts, hip_stream, out, projective);
  if (in.kind != ManyInputs::HOST) return MSM_ERR_INVALID_ARG;
  if (!out || (!in.scalars && count) || (!in.points && !in.shared_points && count)) return MSM_ERR_INVALID_ARG;
  std::vector<int> devs;
  if (int rc = device_list(opts, &devs)) return rc;
  const size_t D = devs.size();
  return for_each_device(D, [&](size_t i) -> int {
    size_t b0, b1;
    shard_range(count, i, D, &b0, &b1);
    if (b0 == b1) return MSM_OK;
    ManyInputs sub = in;
    if (in.points) sub.points = in.points + b0;
    sub.scalars = in.scalars + b0;
    const msm_opts od = opts_on(opts, devs[i]);
    return many_entry(sub, n, b1 - b0, &od, nullptr, out + b0 * (projective ? 32 : 16), projective);
  });
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
    hipStreamSynchronize(c->copy_stream);
    for (Slot& sl : c->slot) hipStreamSynchronize(sl.stream);
    c->shared_pts.release();
    c->host_sc.release();
    c->host_pts.release();
    for (Slot& sl : c->slot) {
      sl.ws.release();
      for (Segment& sg : sl.seg) sg.drop();
      sl.h_out.release();
      sl.h_out_dev = nullptr;
      for (hipEvent_t e : {sl.ev_start, sl.ev_acc0, sl.ev_acc1, sl.ev_end, sl.ev_done, sl.ev_in, sl.ev_sc, sl.ev_fork,
                          sl.ev_join})
        if (e) hipEventDestroy(e);
    }
    for (int i = 0; i < PH_COUNT; i++) hipEventDestroy(c->ev[i]);
    for (int i = 0; i < NCHUNK_EV; i++) hipEventDestroy(c->ev_chunk[i]);
    hipEventDestroy(c->ev_user);
    hipEventDestroy(c->ev_shared);
    hipEventDestroy(c->ev_base);
    for (Slot& sl : c->slot) {
      hipStreamDestroy(sl.stream);
      hipStreamDestroy(sl.aux);
    }
    hipStreamDestroy(c->copy_stream);
    delete c->crew;
    c->crew = nullptr;
    delete c->pool;
    c->pool = nullptr;
    delete c->packer;
    c->packer = nullptr;
    for (int k = 0; k < NPIN; k++) {
      c->pin.buf[k].release();
      if (c->pin.ev[k]) hipEventDestroy(c->pin.ev[k]);
      c->pin.ev[k] = nullptr;
      c->pin.used[k] = false;
    }
    for (hipEvent_t e : c->up_ev) hipEventDestroy(e);
    c->up_ev.clear();
    hipSetDevice(prev);
  }
  for (DevCtx*& c : g_ctx) {
    delete c;
    c = nullptr;
  }
  std::lock_guard<std::mutex> lk3(g_test_mu);
  g_test_pools.stop();
}

int msm_device_count(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  return probe_devices();
}

int msm_device_ordinal(int index) {
  std::lock_guard<std::mutex> lk(g_mu);
  const int n = probe_devices();
  return index >= 0 && index < n ? g_gfx950[index] : -1;
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
  if (!out_xy_be) return MSM_ERR_INVALID_ARG;
  Pt r;
  int rc = multi_host_entry(points_be, scalars_be, n, opts, &r);
  if (rc != MSM_OK) return rc;
  pt_to_be_affine(r, out_xy_be);
  return MSM_OK;
}

// CPU/GPU co-compute (submission.ts:94-154): the host Pippenger (msm_cpu.h) takes points
// [0, share) on a thread of its own while the device path runs [share, n) as msm_compute, and the
// two affine results join with one EC add (point_add_affine, lib.rs:240-253).
int msm_compute_cocompute(const uint32_t* points_be, const uint32_t* scalars_be, size_t n, const msm_opts* opts,
                          double cpu_work_ratio, int cpu_threads, uint32_t out_xy_be[16]) {
  if (!out_xy_be || ((!points_be || !scalars_be) && n) || !(cpu_work_ratio >= 0.0)) return MSM_ERR_INVALID_ARG;
  // a window range has no CPU counterpart (the host Pippenger computes every window): joining a
  // range's GPU share with a whole CPU share would be silently wrong
  if (opts && (opts->flags & MSM_FLAG_WINDOWS)) return MSM_ERR_INVALID_ARG;
  // cpuShare = floor(cpuWorkRatio * n) (submission.ts:98); >= n is the reference's CPU-only branch
  const double share_d = cpu_work_ratio * (double)n;
  const size_t share = share_d >= (double)n ? n : (size_t)share_d;
  if (share == 0) return msm_compute(points_be, scalars_be, n, opts, out_xy_be);
  int rc = msm_init();  // a device entry all the same: no gfx950, no result (the CPU-only entry is msm_compute_cpu)
  if (rc != MSM_OK) return rc;
  uint32_t cpu_xy[16];
  int cpu_rc = MSM_OK;
  std::thread cpu([&] { cpu_rc = cpu_msm(points_be, scalars_be, share, 0, cpu_threads, cpu_xy); });
  Pt r = pt_identity();
  if (share < n) rc = multi_host_entry(points_be + 32 * share, scalars_be + 8 * share, n - share, opts, &r);
  cpu.join();
  if (rc != MSM_OK) return rc;
  if (cpu_rc != MSM_OK) return cpu_rc;
  uint64_t x[4], y[4];
  be_words_to_std(cpu_xy, x);
  be_words_to_std(cpu_xy + 8, y);
  r = pt_add(r, pt_from_affine_std(x, y));
  pt_to_be_affine(r, out_xy_be);
  return MSM_OK;
}

int msm_compute_partial(const uint32_t* points_be, const uint32_t* scalars_be, size_t n, const msm_opts* opts,
                        uint32_t out_xyzt_be[32]) {
  if (!out_xyzt_be) return MSM_ERR_INVALID_ARG;
  Pt r;
  int rc = multi_host_entry(points_be, scalars_be, n, opts, &r);
  if (rc != MSM_OK) return rc;
  pt_to_be_xyzt(r, out_xyzt_be);
  return MSM_OK;
}

int msm_compute_device(const uint32_t* d_points_be, const uint32_t* d_scalars_be, size_t n, const msm_opts* opts,
                       void* hip_stream, uint32_t out_xy_be[16]) {
  if (!out_xy_be) return MSM_ERR_INVALID_ARG;
  Pt r;
  int rc = multi_device_entry(d_points_be, d_scalars_be, n, opts, hip_stream, &r);
  if (rc != MSM_OK) return rc;
  pt_to_be_affine(r, out_xy_be);
  return MSM_OK;
}

int msm_compute_device_partial(const uint32_t* d_points_be, const uint32_t* d_scalars_be, size_t n,
                               const msm_opts* opts, void* hip_stream, uint32_t out_xyzt_be[32]) {
  if (!out_xyzt_be) return MSM_ERR_INVALID_ARG;
  Pt r;
  int rc = multi_device_entry(d_points_be, d_scalars_be, n, opts, hip_stream, &r);
  if (rc != MSM_OK) return rc;
  pt_to_be_xyzt(r, out_xyzt_be);
  return MSM_OK;
}

int msm_compute_many_device(const uint32_t* const* d_points_be, const uint32_t* const* d_scalars_be, size_t n,
                            size_t count, const msm_opts* opts, void* hip_stream, uint32_t* out_xy_be) {
  ManyInputs in;
  in.points = d_points_be;
  in.scalars = d_scalars_be;
  return multi_many_entry(in, n, count, opts, hip_stream, out_xy_be, false);
}

int msm_compute_many_device_partial(const uint32_t* const* d_points_be, const uint32_t* const* d_scalars_be,
                                    size_t n, size_t count, const msm_opts* opts, void* hip_stream,
                                    uint32_t* out_xyzt_be) {
  ManyInputs in;
  in.points = d_points_be;
  in.scalars = d_scalars_be;
  return multi_many_entry(in, n, count, opts, hip_stream, out_xyzt_be, true);
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

int msm_compute_shared_device(const uint32_t* d_points_be, const uint32_t* const* d_scalars_be, size_t n,
                              size_t count, const msm_opts* opts, void* hip_stream, uint32_t* out_xy_be) {
  if (!d_points_be && n && count) return MSM_ERR_INVALID_ARG;
  ManyInputs in;
  in.shared_points = d_points_be;
  in.scalars = d_scalars_be;
  if (!n) in.points = d_scalars_be;  // n = 0: identities, no input is read
  return multi_many_entry(in, n, count, opts, hip_stream, out_xy_be, false);
}

int msm_compute_many(const uint32_t* const* points_be, const uint32_t* const* scalars_be, size_t n, size_t count,
                     const msm_opts* opts, uint32_t* out_xy_be) {
  ManyInputs in;
  in.kind = ManyInputs::HOST;
  in.points = points_be;
  in.scalars = scalars_be;
  in.packed = host_pack();  // x|y (x|y|z) through the pinned ring into the slots' wire buffers
  return multi_many_entry(in, n, count, opts, nullptr, out_xy_be, false);
}

int msm_compute_shared(const uint32_t* points_be, const uint32_t* const* scalars_be, size_t n, size_t count,
                       const msm_opts* opts, uint32_t* out_xy_be) {
  if (!points_be && n && count) return MSM_ERR_INVALID_ARG;
  ManyInputs in;
  in.kind = ManyInputs::HOST;
  in.shared_points = points_be;
  in.scalars = scalars_be;
  if (!n) in.points = scalars_be;
  return multi_many_entry(in, n, count, opts, nullptr, out_xy_be, false);
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

int msm_combine_partials_many(const uint32_t* partials_xyzt_be, size_t world, size_t count, uint32_t* out_xy_be) {
  if ((!partials_xyzt_be && world && count) || (!out_xy_be && count)) return MSM_ERR_INVALID_ARG;
  std::vector<Pt> acc(count, pt_identity());
  for (size_t k = 0; k < count; k++)
    for (size_t w = 0; w < world; w++) {
      Pt p;
      int rc = pt_from_be_xyzt(partials_xyzt_be + 32 * (w * count + k), &p);
      if (rc != MSM_OK) return rc;
      if (fq_is_zero(p.Z)) return MSM_ERR_BAD_POINT;
      acc[k] = w == 0 ? p : pt_add(acc[k], p);
    }
  if (!count) return MSM_OK;
  // Montgomery's trick: one inversion of the product of every Z, then each Z^-1 from prefix
  // products (complete formulas: a sum of valid points never has Z = 0)
  std::vector<Fq> pre(count);
  pre[0] = acc[0].Z;
  for (size_t k = 1; k < count; k++) pre[k] = fq_mul(pre[k - 1], acc[k].Z);
  Fq inv = fq_inv(pre[count - 1]);
  for (size_t k = count; k-- > 0;) {
    const Fq zi = k ? fq_mul(inv, pre[k - 1]) : inv;
    if (k) inv = fq_mul(inv, acc[k].Z);
    uint64_t x[4], y[4];
    fq_to_std(fq_mul(acc[k].X, zi), x);
    fq_to_std(fq_mul(acc[k].Y, zi), y);
    std_to_be_words(x, out_xy_be + 16 * k);
    std_to_be_words(y, out_xy_be + 16 * k + 8);
  }
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

uint32_t msm_window_count(uint32_t window_bits) {
  if (window_bits < 4 || window_bits > 20) return 0;
  return (MAIN_BITS + window_bits - 1) / window_bits + 1;  // balanced main windows + the overflow window
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

int msm_compute_cpu(const uint32_t* points_be, const uint32_t* scalars_be, size_t n, uint32_t window_bits,
                    int n_threads, uint32_t out_xy_be[16]) {
  if (!out_xy_be || ((!points_be || !scalars_be) && n)) return MSM_ERR_INVALID_ARG;
  return cpu_msm(points_be, scalars_be, n, window_bits, n_threads, out_xy_be);
}

int msm_set_profiling(int enable) {
  std::lock_guard<std::mutex> lk(g_mu);
  g_profiling.store(enable < 0 ? 0 : enable > 2 ? 1 : enable);
  for (DevCtx* c : g_ctx)
    if (c) {
      std::lock_guard<std::mutex> lk2(c->mu);  // a call in flight on another thread finishes first
      c->profiling = g_profiling.load();
      c->last.accumulate_sum = c->last.device_total_sum = c->last.accumulate_union_sum = 0;
      c->last.profiled = 0;
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

// ---- test hooks (not in msm.h) ----
// The device-list shard split (tests/test_host_logic.py checks it against msm_amd.dist).
int msm_test_shard_range(size_t n, size_t i, size_t D, size_t* lo, size_t* hi) {
  if (!lo || !hi || D == 0 || i >= D) return MSM_ERR_INVALID_ARG;
  shard_range(n, i, D, lo, hi);
  return MSM_OK;
}

// The sharded paths with a list that may repeat a device (the one-GPU box has no second device):
// mode 0 = msm_compute (host inputs), 1 = msm_compute_device; affine result.
int msm_test_sharded(int mode, const uint32_t* points, const uint32_t* scalars, size_t n, const msm_opts* opts,
                     const int32_t* devices, uint32_t n_devices, void* hip_stream, uint32_t out_xy_be[16]) {
  if (!opts || !devices || !n_devices || n_devices > MSM_MAX_DEVICES || !out_xy_be) return MSM_ERR_INVALID_ARG;
  std::vector<int> devs(devices, devices + n_devices);
  for (int d : devs) {
    DevCtx* c;
    if (int rc = get_ctx(d, &c)) return rc;
  }
  Pt r;
  const int rc = mode == 0 ? sharded_host(points, scalars, n, opts, devs, &r)
                           : sharded_device(points, scalars, n, opts, hip_stream, devs, &r);
  if (rc != MSM_OK) return rc;
  pt_to_be_affine(r, out_xy_be);
  return MSM_OK;
}

// Peer access of device `dev` to `owner` (enabled on first use, as peer_shard does): 1 enabled
// (or dev == owner), 0 unavailable, MSM_ERR_INVALID_ARG for a non-gfx950 ordinal.
int msm_test_peer_state(int dev, int owner) {
  DevCtx *a, *b;
  if (get_ctx(dev, &a) != MSM_OK || get_ctx(owner, &b) != MSM_OK) return MSM_ERR_INVALID_ARG;
  DeviceGuard g(dev);
  return enable_peer(dev, owner);
}

// The host tail of a lone MSM of n points (auto plan) on caller-supplied window terms (host
// Montgomery X|Y|T|Z words, the layout k_bucket_reduce_2 writes): helpers = 0 runs horner_tail,
// otherwise the TailCrew.  Affine result; *ms = the tail's wall time.
// helpers < 0: one crew of -helpers threads over 40 rounds (the persistent crew of a device
// context), every third round armed and disarmed without terms first (an error return); the
// result of the last round, MSM_ERR_INVALID_ARG if any round disagrees with the first.
int msm_test_tail(size_t n, const uint32_t* terms, int helpers, uint32_t out_xy_be[16], double* ms) {
  Plan pl;
  if (int rc = make_plan(n, nullptr, DevShape{}, &pl)) return rc;
  const int rounds = helpers < 0 ? 40 : 1;
  TailCrew crew(helpers < 0 ? -helpers : helpers);
  Pt first{}, r{};
  bool same = true;
  const auto t0 = clk::now();
  for (int k = 0; k < rounds; k++) {
    if (helpers < 0 && k % 3 == 1) {
      crew.arm();
      crew.disarm();
    }
    crew.arm();
    r = helpers ? crew.run(pl, terms) : horner_tail(pl, terms);
    crew.disarm();
    if (k == 0) first = r;
    same = same && fq_eq(fq_mul(r.X, first.Z), fq_mul(first.X, r.Z)) && fq_eq(fq_mul(r.Y, first.Z), fq_mul(first.Y, r.Z));
  }
  *ms = std::chrono::duration<double, std::milli>(clk::now() - t0).count() / rounds;
  pt_to_be_affine(r, out_xy_be);
  return same ? MSM_OK : MSM_ERR_INVALID_ARG;
}

// Host field / curve timings (ns per operation, dependent chains): what 0 = fq_mul, 1 = one
// doubling of pt_dbl_n, 2 = pt_add, 3 = fq_inv.  For sizing the host tail.
int msm_test_host_timing(int what, size_t iters, double* ns) {
  if (!ns || iters == 0 || what < 0 || what > 4) return MSM_ERR_INVALID_ARG;
  if (what == 4) {  // self-check: binary-Euclid fq_inv against a^(p-2) on iters pseudo-random a
    uint64_t st = 0x9E3779B97F4A7C15ull, bad = 0;
    for (size_t i = 0; i < iters; i++) {
      uint64_t s[4];
      for (int j = 0; j < 4; j++) {
        st = st * 6364136223846793005ull + 1442695040888963407ull;
        s[j] = st ^ (st >> 29);
      }
      s[3] &= (i & 1) ? 0x0fffffffffffffffull : 0x000000000000ffffull;  // full-width and short
      if (i == 0) s[0] = 1, s[1] = s[2] = s[3] = 0;
      if (i == 1) s[0] = P[0] - 1, s[1] = P[1], s[2] = P[2], s[3] = P[3];
      const Fq a = fq_from_std(s);
      const Fq x = fq_inv(a);
      bad += !fq_eq(x, fq_inv_pow(a)) || !fq_eq(fq_mul(x, a), fq_one());
    }
    bad += !fq_is_zero(fq_inv(fq_zero()));
    *ns = (double)bad;
    return MSM_OK;
  }
  Pt p = pt_identity();
  p.X = fq_one();
  p.Y = fq_add(fq_one(), fq_one());
  p.T = fq_add(p.Y, fq_one());
  p.Z = fq_add(p.T, fq_one());
  Fq a = p.Z;
  const auto t0 = clk::now();
  for (size_t i = 0; i < iters; i++) {
    if (what == 0) a = fq_mul(a, a);
    else if (what == 1) p = pt_dbl_n(p, 1);
    else if (what == 2) p = pt_add(p, p);
    else a = fq_inv(a);
  }
  *ns = std::chrono::duration<double, std::nano>(clk::now() - t0).count() / (double)iters;
  volatile uint64_t sink = a.l[0] ^ p.X.l[0];
  (void)sink;
  return MSM_OK;
}

// The number of window-term words msm_test_tail reads for n points.
// msm_test_tail over k MSMs' terms at once (k blocks of msm_test_tail_words(n) words), as the last
// launch of a pipelined run finishes: helpers > 0 runs TailCrew::run_batch on a crew of that many
// threads, helpers = 0 one horner_tail per MSM.  out_xy_be: k affine results (16 words each).
int msm_test_tail_batch(size_t n, uint32_t k, const uint32_t* terms, int helpers, uint32_t* out_xy_be, double* ms) {
  if (!terms || !out_xy_be || !ms || k < 1 || k > MSM_MAX_BATCH || helpers < 0) return MSM_ERR_INVALID_ARG;
  Plan pl;
  if (int rc = make_plan(n, nullptr, DevShape{}, &pl)) return rc;
  TailCrew crew(helpers);
  Pt r[MSM_MAX_BATCH];
  const auto t0 = clk::now();
  if (helpers) {
    crew.arm();
    crew.run_batch(pl, terms, k, r);
  } else {
    for (uint32_t m = 0; m < k; m++) r[m] = horner_tail(pl, terms, m);
  }
  *ms = std::chrono::duration<double, std::milli>(clk::now() - t0).count();
  for (uint32_t m = 0; m < k; m++) pt_to_be_affine(r[m], out_xy_be + 16 * m);
  return MSM_OK;
}

// The launch plan make_plan builds for n points, nm MSMs per launch, pipelined or lone, with
// `opts` (window width / range; may be null): out = {c (widest window), windows in the launch per
// MSM (Wr), run length K, reduction chunk L, MSMs per launch, coarse bins per window, skew floor
// of K}, for the default device shape (256 CUs, 4 accumulation waves per SIMD).
int msm_test_plan(size_t n, uint32_t nm, int pipelined, const msm_opts* opts, uint32_t out[7]) {
  if (!out || nm < 1 || nm > MSM_MAX_BATCH) return MSM_ERR_INVALID_ARG;
  Plan pl;
  if (int rc = make_plan(n, opts, DevShape{}, &pl, pipelined != 0, nm)) return rc;
  const uint32_t v[7] = {pl.d.c, pl.d.Wr, pl.K, pl.L, pl.d.nm, pl.d.nbc, run_length_skew_floor(pl.d)};
  memcpy(out, v, sizeof(v));
  return MSM_OK;
}

// The host packing of the packed uploads (pack_records over a pool of MSM_HOST_PACK_THREADS):
// n wire records -> out (16 words per point for fmt 1 = x|y, 24 for fmt 2 = x|y|z); *all_z_one =
// whether every z is 1, *t_bad = whether some t >= p.  Host code only (no device needed).
// The host thread pools a call over `ndev` devices runs per device context (CPU test hook,
// no device needed): out[0] the CPU budget (host_threads: hardware threads capped by the cgroup
// quota), out[1..3] packing threads (the caller included), lone-MSM tail helpers and pipelined-tail
// threads per device, out[4] the threads the library adds for the whole call -- per device its
// packing workers, helpers, tail threads and one uploader, plus a host thread per device but the
// first.  With `run` the three pools are started at those sizes (replacing the previous set), given
// one job each, and left parked until the next call or msm_shutdown.
int msm_test_pools(int ndev, int run, int* out) {
  if (ndev < 1 || ndev > 64 || !out) return MSM_ERR_INVALID_ARG;
  const int own = t_call_devices;
  t_call_devices = ndev;
  const int pk = pack_threads(), th = tail_helpers(), hn = horner_threads();
  t_call_devices = own;
  out[0] = (int)host_threads();
  out[1] = pk;
  out[2] = th;
  out[3] = hn;
  out[4] = ndev * ((pk - 1) + th + hn + 1) + (ndev - 1);
  if (!run) return MSM_OK;
  std::lock_guard<std::mutex> lk(g_test_mu);
  g_test_pools.stop();
  g_test_pools.packer = new PackPool(pk);
  g_test_pools.crew = new TailCrew(th);
  g_test_pools.pool = hn ? new HornerPool(hn) : nullptr;
  std::atomic<int> hits{0};
  g_test_pools.packer->run([&](int, int) { hits.fetch_add(1); });
  if (g_test_pools.pool) {
    for (int i = 0; i < 2 * hn; i++) g_test_pools.pool->push([&] { hits.fetch_add(1); });
    g_test_pools.pool->wait_all();
  }
  g_test_pools.crew->arm();  // the helpers wake and spin, then go back to sleep
  g_test_pools.crew->disarm();
  return hits.load() == pk + 2 * hn ? MSM_OK : MSM_ERR_HIP;
}

int msm_test_pack(const uint32_t* wire, size_t n, uint32_t fmt, uint32_t* out, int* all_z_one, int* t_bad) {
  if ((!wire || !out) && n) return MSM_ERR_INVALID_ARG;
  if (fmt != PT_FMT_XY && fmt != PT_FMT_XYZ) return MSM_ERR_INVALID_ARG;
  std::lock_guard<std::mutex> lk(g_test_mu);
  PackPool*& pool = g_test_pools.packer;
  if (!pool) pool = new PackPool(pack_threads());
  const size_t bytes = n * pt_fmt_slots(fmt) * 16;
  void* tmp = aligned_alloc(64, (bytes + 63) / 64 * 64 + 64);  // the nontemporal stores want 32-B alignment
  if (!tmp) return MSM_ERR_OOM;
  bool tb = false;
  const bool z1 = pack_records(*pool, static_cast<uint32_t*>(tmp), wire, n, fmt, &tb);
  memcpy(out, tmp, bytes);
  free(tmp);
  if (all_z_one) *all_z_one = z1 ? 1 : 0;
  if (t_bad) *t_bad = tb ? 1 : 0;
  return MSM_OK;
}

size_t msm_test_tail_words(size_t n) {
  Plan pl;
  if (make_plan(n, nullptr, DevShape{}, &pl)) return 0;
  return (size_t)pl.d.W * pl.nterms * 32;
}

// Batch field / point ops on the device, canonical LE words.
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

#ifdef MSM_PHASE_PROBE
// Tuning builds only: writes the sort kernels' phase stamps of the last launch (g_probe) to `path`.
int msm_test_probe_dump(const char* path) {
  static std::vector<uint64_t> buf(sizeof(g_probe) / 8);
  if (hipDeviceSynchronize() != hipSuccess) return MSM_ERR_HIP;
  if (hipMemcpyFromSymbol(buf.data(), HIP_SYMBOL(g_probe), sizeof(g_probe), 0, hipMemcpyDeviceToHost) != hipSuccess)
    return MSM_ERR_HIP;
  FILE* f = fopen(path, "wb");
  if (!f) return MSM_ERR_INVALID_ARG;
  fwrite(buf.data(), 8, buf.size(), f);
  fclose(f);
  return MSM_OK;
}
#endif

}  // extern "C"
