/*
 * libmsm — MI355X (gfx950) multi-scalar multiplication over Edwards-BLS12
 * (ark-ed-on-bls12-377: -x^2 + y^2 = 1 + 3021 x^2 y^2 over the 253-bit BLS12-377 scalar field).
 *
 * C ABI that replaces the compute path under the reference's
 *   compute_msm(baseAffinePoints, scalars) -> Promise<{x, y}>      src/submission/submission.ts:25-157
 * i.e. the WebGPU intra-bucket reduction + Rust/wasm split / bucket-sum / window combine.
 * Plain pointers and sizes only; every entry point is re-entrant (calls on one device serialise).
 *
 * Wire formats (identical to the reference's, src/submission/consts.ts:1-4, bytes.rs:11-71):
 *   field element : 8 x uint32, BIG-endian word order (index 0 = most significant), standard form
 *   point         : x | y | t | z  = 32 x uint32 = 128 B   (t = x*y/z, z usually 1); every
 *                   coordinate must be < p (MSM_ERR_COORD_RANGE otherwise), but the MSM itself
 *                   uses only x, y and z -- d t is recomputed from the affine x y, as the oracle
 *                   (Aleo's msm over affine points) does, so an inconsistent t does not change it
 *   scalar        : 8 x uint32 big-endian = full 256-bit integer (not reduced mod r)
 *   result        : x | y affine = 16 x uint32; identity = (0, 1)
 */
#ifndef MSM_MI355X_H
#define MSM_MI355X_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Return codes.  The reference panics where these are returned (cited). */
#define MSM_OK 0
#define MSM_ERR_INVALID_ARG (-1)        /* null pointer / bad option                          */
#define MSM_ERR_UNSUPPORTED_WINDOW (-2) /* lib.rs:200,208,223,231 `Unsupported window size`  */
#define MSM_ERR_COORD_RANGE (-3)        /* bytes.rs:19 Fq::from_bigint(..).unwrap() (coord >= p) */
#define MSM_ERR_BAD_POINT (-4)          /* z == 0 (not a projective point)                    */
#define MSM_ERR_HIP (-5)                /* HIP runtime failure                                */
#define MSM_ERR_NO_DEVICE (-6)          /* no gfx950 device visible: there is no CPU fallback */
#define MSM_ERR_OOM (-7)                /* device allocation failed                           */

/* hip_stream argument of the *_device entries: order after the null (legacy default) stream,
 * e.g. torch's default stream (whose handle is 0, i.e. indistinguishable from "no stream"). */
#define MSM_STREAM_NULL ((void*)1)

/* msm_opts.flags */
#define MSM_FLAG_SERIAL 1u  /* pipelined entries: one launch in flight at a time (no overlap)     */
#define MSM_FLAG_DEVICES 2u /* the device-list fields (devices, n_devices) are set: see below     */
#define MSM_FLAG_WINDOWS 4u /* the window-range fields (window_lo, window_hi) are set: see below  */
#define MSM_FLAG_HALF_WINDOWS 8u /* with MSM_FLAG_WINDOWS: window_lo / window_hi count half windows */

#define MSM_MAX_DEVICES 16

/* Options.  The struct is versioned by its flags: the first four fields are the original
 * (16-byte) layout, and a caller that never sets MSM_FLAG_DEVICES may pass that shorter struct --
 * the library reads `devices` / `n_devices` only when the flag is set.
 *
 * Device list (MSM_FLAG_DEVICES; SURVEY.md §8b's "device mask, n_gpus"): the MSM runs on the
 * `n_devices` listed gfx950 HIP ordinals (distinct, 1..MSM_MAX_DEVICES; `device` is ignored).  It
 * generalises the reference's only sharding precedent, the CPU/GPU split inside one compute_msm
 * call (submission.ts:116-154 + gpu_worker.ts:9-18, joined by point_add_affine lib.rs:240-253):
 *   - msm_compute / msm_compute_partial: the point vector is cut into n_devices contiguous shards
 *     (shard d = [n d / D, n (d+1) / D)), each device uploads and reduces its own shard on its own
 *     host thread (its own PCIe link), and the shards' partials are joined with one EC add each;
 *   - msm_compute_device / msm_compute_device_partial: the inputs live on one device (where the
 *     pointers were allocated, which must be listed); the other listed devices copy their shard
 *     from it over xGMI (peer copies) and reduce it, and the partials are joined the same way;
 *   - msm_compute_many / msm_compute_shared (host batches): each device takes a contiguous block
 *     of the `count` MSMs (no join: whole MSMs per device, the prover-batch replicas).
 * The result is the same group element whatever the list (tests/test_gpu_multidev.py).  A
 * repeated, negative or non-gfx950 ordinal, an empty list or more than MSM_MAX_DEVICES entries
 * give MSM_ERR_INVALID_ARG; the list is checked before any work is enqueued. */
typedef struct msm_opts {
  uint32_t window_bits; /* 0 = auto (msm_best_window); else 4..20. Replaces ?windowSize (submission.ts:29-33) */
  uint32_t run_length;  /* sorted-list entries per accumulation lane; 0 = auto                     */
  int32_t device;       /* HIP device ordinal (a gfx950 one), -1 = the calling thread's current device */
  uint32_t flags;       /* MSM_FLAG_* (0 = defaults)                                              */
  /* --- read only when flags & MSM_FLAG_DEVICES --- */
  const int32_t* devices; /* n_devices HIP ordinals                                                */
  uint32_t n_devices;
  uint32_t reserved; /* 0 */
  /* --- read only when flags & MSM_FLAG_WINDOWS --- */
  uint32_t window_lo, window_hi; /* the MSM's windows [window_lo, window_hi) only (below)             */
} msm_opts;

/* Window range (MSM_FLAG_WINDOWS): with an explicit window_bits c, the scalars are recoded into
 * msm_window_count(c) signed-digit windows (counted from the least significant; the last is the
 * overflow window for bits 254..255 and the carry) and only windows [window_lo, window_hi) are
 * sorted, accumulated and reduced: the result is sum over those windows w of 2^(offset w) G_w.
 * The ranges of a partition of [0, msm_window_count(c)) sum (as group elements) to the whole MSM,
 * so the window ranges are a second way to shard one MSM over devices besides the point vector:
 * every device then reads all n points and scalars but does 1/D of the bucket work and of the
 * reduction.  Meant for the *_partial entries (the affine entries return the
 * range's sum in affine form, which joins by msm_point_add_affine); window_bits 0, an empty range
 * or one past the last window give MSM_ERR_INVALID_ARG, and so does the flag on
 * msm_compute_cocompute (its host share always covers every window).
 * msm_profile_t.windows reports the launch's range (its window count), not the MSM's layout:
 * msm_window_count(window_bits) gives that.
 * With MSM_FLAG_HALF_WINDOWS the range is counted in half windows, [0, 2 msm_window_count(c)):
 * half window 2w is window w's buckets of the lower half of its digit magnitudes, 2w + 1 the upper
 * half, so a range may start or end in the middle of a window (an odd number of windows can be
 * cut into equal shares). */
uint32_t msm_window_count(uint32_t window_bits);

/* Per-phase device times (ms) of the most recent MSM on the calling thread's device when
 * profiling is enabled (hipEvents on the library's stream). */
typedef struct msm_profile_t {
  float prepare_points, recode_count, coarse_scan, coarse_scatter, fine_sort;
  float accumulate, fixup, bucket_reduce_1, bucket_reduce_2, readback;
  float device_total; /* first kernel start -> readback end */
  float host_tail;    /* host Horner + affine conversion (wall) */
  uint64_t entries;   /* nonzero digits sorted (= accumulation adds) */
  uint32_t window_bits, windows, run_length, chunk_len;
  double accumulate_sum; /* sum of `accumulate` over every launch profiled since msm_set_profiling */
  double device_total_sum;
  uint32_t profiled;     /* number of launches in those sums */
  uint32_t msms_per_launch; /* MSMs one launch (and one k_accumulate) covers */
  double accumulate_union_sum; /* wall time with >= 1 k_accumulate in flight, summed over the calls
                                  since msm_set_profiling (launches in flight may overlap) */
} msm_profile_t;

/* Library lifetime.  msm_init replaces the wasm init()/initThreadPool (submission.ts:89-93);
 * it probes the devices and fails with MSM_ERR_NO_DEVICE when no gfx950 is present. */
int msm_init(void);
void msm_shutdown(void);
/* Number of gfx950 devices visible, and the HIP ordinal of the index-th of them (0-based; -1 when
 * out of range).  On a node that mixes GPU types the gfx950 ordinals need not be contiguous, so
 * callers mapping a rank or a list index to opts.device / opts.devices should go through it. */
int msm_device_count(void);
int msm_device_ordinal(int index);
const char* msm_strerror(int code);

/* getBestWindowSize (submission.ts:18-23), re-tuned for signed digits on MI355X. */
uint32_t msm_best_window(size_t n);

/* compute_msm: host-resident inputs, result on the host.  n = 0 gives the identity (0, 1),
 * like the oracle's empty `Address.msm`.  Uploads overlap compute (generalises the reference's
 * staging ring, gpu.ts:146-155 / 244-271): from n = 3 * 2^17 the MSM runs as point slices of ~2^17
 * through the pipelined launches, slice g+1 uploading on a copy stream while slice g computes,
 * and the slices' partials are joined (the shard/join identity of submission.ts:116-154); there
 * the library's threads pack x|y of every point (x|y|z for a launch with some z != 1) into pinned
 * staging -- half the PCIe bytes -- and check every t < p on the host; smaller MSMs upload the
 * scalars first (the bucket sort starts on them) and the points in 2^16-point pieces, packed the
 * same way per piece, each prepared as it lands.  The packing runs on a pool of
 * MSM_HOST_PACK_THREADS (default 8) threads per device context, created on first use and parked
 * between calls, plus three pinned staging buffers per context (up to 32 MiB each at 2^20).  The
 * caller keeps ownership of the arrays; they are not read after the call returns. */
int msm_compute(const uint32_t* points_be, const uint32_t* scalars_be, size_t n, const msm_opts* opts,
                uint32_t out_xy_be[16]);

/* compute_msm with the reference's CPU/GPU co-compute (?cpuWorkRatio, submission.ts:94-154):
 * share = floor(cpu_work_ratio * n) points [0, share) run on the library's host Pippenger
 * (msm_compute_cpu's, cpu_threads threads, <= 0 as there, its own window) on a
 * thread of their own while points [share, n) run as msm_compute(opts) on the GPU(s); the two
 * results join with one EC add (point_add_affine, lib.rs:240-253).  cpu_work_ratio 0 (or a share
 * that floors to 0) is msm_compute; a share >= n is the reference's CPU-only branch.  Still a device
 * entry: MSM_ERR_NO_DEVICE without a gfx950.  A negative or NaN ratio gives MSM_ERR_INVALID_ARG.
 * The result equals msm_compute's for every ratio; on MI355X any share > ~0.1% delays it (the host
 * runs a 2^20 MSM ~800x slower than one GPU), so this exists for interface parity. */
int msm_compute_cocompute(const uint32_t* points_be, const uint32_t* scalars_be, size_t n, const msm_opts* opts,
                          double cpu_work_ratio, int cpu_threads, uint32_t out_xy_be[16]);

/* Same with inputs already in device memory (device pointers, wire layout).  `hip_stream` may be
 * NULL or a hipStream_t: the library's streams then wait for the work enqueued on it so far (the
 * inputs it produces), and the call returns when the result is on the host.  With NULL the
 * caller must have completed the inputs' producers (e.g. torch.cuda.synchronize()).  The same
 * holds for every *_device entry below. */
int msm_compute_device(const uint32_t* d_points_be, const uint32_t* d_scalars_be, size_t n, const msm_opts* opts,
                       void* hip_stream, uint32_t out_xy_be[16]);

/* Shard entry for multi-GPU / co-compute: the shard's MSM as a projective point
 * X|Y|T|Z (32 big-endian words, standard form) so shards join with one EC add each
 * (generalises the cpu/gpu co-compute join, submission.ts:116-154 + lib.rs:240-253). */
int msm_compute_device_partial(const uint32_t* d_points_be, const uint32_t* d_scalars_be, size_t n,
                               const msm_opts* opts, void* hip_stream, uint32_t out_xyzt_be[32]);
int msm_compute_partial(const uint32_t* points_be, const uint32_t* scalars_be, size_t n, const msm_opts* opts,
                        uint32_t out_xyzt_be[32]);
/* Sum `count` projective partials and return the affine result. */
int msm_combine_partials(const uint32_t* partials_xyzt_be, size_t count, uint32_t out_xy_be[16]);
/* The multi-GPU join of a batch: partials [world][count][32] (as one all_gather over `world`
 * ranks returns them); result k = sum over ranks of partial [w][k], affine, [count][16].  One
 * field inversion for the whole batch (Montgomery's trick) instead of one per MSM. */
int msm_combine_partials_many(const uint32_t* partials_xyzt_be, size_t world, size_t count, uint32_t* out_xy_be);

/* Batch of `count` independent MSMs of equal size n, inputs contiguous ([count][n][32] points,
 * [count][n][8] scalars), all device-resident; results [count][16].  Prover-batch shape. */
int msm_compute_batch_device(const uint32_t* d_points_be, const uint32_t* d_scalars_be, size_t n, size_t count,
                             const msm_opts* opts, void* hip_stream, uint32_t* out_xy_be);

/* `count` independent MSMs of n points each, inputs given by per-MSM device pointers; results
 * [count][16].  Pipelined: launches of 2-4 MSMs stay on the device while the host finishes earlier ones
 * (window Horner), so throughput exceeds 1 / latency.  With window_bits = 0 the window is tuned
 * for throughput, which below 2^20 points is narrower than msm_best_window's (same results).
 * msm_compute_batch_device is this with contiguous inputs. */
int msm_compute_many_device(const uint32_t* const* d_points_be, const uint32_t* const* d_scalars_be, size_t n,
                            size_t count, const msm_opts* opts, void* hip_stream, uint32_t* out_xy_be);
/* Same, each result as a projective X|Y|T|Z partial ([count][32] words) for a later
 * msm_combine_partials: the pipelined shard entry of a multi-GPU batch. */
int msm_compute_many_device_partial(const uint32_t* const* d_points_be, const uint32_t* const* d_scalars_be,
                                    size_t n, size_t count, const msm_opts* opts, void* hip_stream,
                                    uint32_t* out_xyzt_be);

/* Prover batch: `count` independent MSMs over ONE base vector (d_points_be, [n][32]) with their own
 * scalar vectors d_scalars_be[b] ([n][8] each); results [count][16].  The base vector is prepared
 * once per call (k_prepare_points) and every MSM reads its records; otherwise as
 * msm_compute_many_device.  BASELINE configs[4] (64 x 2^18). */
int msm_compute_shared_device(const uint32_t* d_points_be, const uint32_t* const* d_scalars_be, size_t n,
                              size_t count, const msm_opts* opts, void* hip_stream, uint32_t* out_xy_be);

/* Host-resident batches (the streaming API of SURVEY.md §8f2).  msm_compute_many: `count`
 * independent MSMs, per-MSM host arrays; msm_compute_shared: one host base vector, per-MSM host
 * scalar vectors.  Inputs are uploaded on a copy stream into the in-flight launch slots while the
 * other slots compute (the base vector of msm_compute_shared once, piece by piece, prepared as it
 * lands); msm_compute_many packs x|y of every point as msm_compute does (t checked on the host,
 * MSM_ERR_COORD_RANGE for t >= p).  Results [count][16].  Footprint: msm_compute_many's packing
 * keeps three pinned host buffers of one launch's points and scalars (nm * n * 128 B each: nm = 2
 * MSMs per launch up to 2^21 points, 4 up to 2^18, 8 up to 2^16 -- e.g. 3 x 256 MiB at 2^20) until
 * msm_shutdown; a launch needing more than 512 MiB per buffer (MSM_PIN_MAX_MB) uploads unpacked. */
int msm_compute_many(const uint32_t* const* points_be, const uint32_t* const* scalars_be, size_t n, size_t count,
                     const msm_opts* opts, uint32_t* out_xy_be);
int msm_compute_shared(const uint32_t* points_be, const uint32_t* const* scalars_be, size_t n, size_t count,
                       const msm_opts* opts, uint32_t* out_xy_be);

/* The reference's CPU-only path (cpuWorkRatio = 1: submission.ts:96-115 -> msm_end_to_end,
 * lib.rs:24-44, 106-121) as the library's own multithreaded host Pippenger: signed c-bit digits,
 * 7M mixed adds into per-thread bucket tables.  window_bits 0 = auto, n_threads <= 0 = all
 * hardware threads the process may run (capped by a cgroup CPU quota).  An explicit entry, never a fallback for the GPU entries. */
int msm_compute_cpu(const uint32_t* points_be, const uint32_t* scalars_be, size_t n, uint32_t window_bits,
                    int n_threads, uint32_t out_xy_be[16]);

/* point_add_affine (lib.rs:240-253): affine a + b -> affine, 16 words each. */
int msm_point_add_affine(const uint32_t a_xy_be[16], const uint32_t b_xy_be[16], uint32_t out_xy_be[16]);

/* split_dynamic (lib.rs:196-202, msm-macro lib.rs:73-177): the reference's own unsigned digit
 * split, out[w*n + i] = c-bit window w of scalar i with w = 0 the MOST significant window,
 * n_windows = ceil(256 / c).  Host-side; kept for interface parity and tests. */
int msm_split(uint32_t window_bits, const uint32_t* scalars_be, size_t n, uint32_t* out);
uint32_t msm_split_windows(uint32_t window_bits);

/* Synthetic-input utilities (the benchmark page's generators, src/ui/AllBenchmarks.tsx:107-140 and
 * src/reference/webgpu/utils.ts:81-100), host-side and multithreaded:
 *   points_be[i] = (k0 + i*step) * G for the affine base G (16 BE words), wire layout, z = 1;
 *   scalars_be[i] = 4 xorshift64(13,7,17) words (first = most significant) reduced mod p. */
int msm_gen_points(const uint32_t g_xy_be[16], uint64_t k0, uint64_t step, size_t n, uint32_t* points_be);
int msm_gen_scalars(uint64_t seed, size_t n, uint32_t* scalars_be);

/* Profiling.  enable = 0: off; 1: hipEvents between every phase (launches go eagerly, no graph
 * replay); 2: k_accumulate's duration and the device total of every launch (the production path:
 * k_accumulate always runs between two events).  msm_last_profile reports the calling thread's
 * device. */
int msm_set_profiling(int enable);
int msm_last_profile(msm_profile_t* out);

#ifdef __cplusplus
}
#endif

#endif /* MSM_MI355X_H */
