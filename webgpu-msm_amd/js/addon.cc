// Node N-API addon: the thin FFI between the reference's TypeScript surface
// (compute_msm, src/submission/submission.ts:25-157) and libmsm's C ABI (include/msm.h).
//
// Exports (all compute is asynchronous through napi_async_work, resolving a Promise, because
// compute_msm is async in the reference):
//   computeMsmU32(points: Uint32Array(32n), scalars: Uint32Array(8n), windowSize, devices?)
//       -> Promise<Uint32Array(16)>
//   computeMsmBigInt(points: {x,y,t,z: bigint}[], scalars: bigint[], windowSize, devices?)
//       -> Promise<Uint32Array(16)>
//       BigInt -> big-endian u32 marshalling happens natively (napi_get_value_bigint_words),
//       replacing convert_worker.ts:8-57 and the 8-worker fan-out of submission.ts:47-74.
//   `devices` (an array of HIP ordinals) shards the MSM over those gfx950 devices in this one call
//   (msm_opts MSM_FLAG_DEVICES: one host thread and PCIe link per device, partials joined with one
//   EC add each -- the reference's CPU/GPU split of submission.ts:116-154 generalised).
//
// Input ownership while the promise is pending (the worker thread reads the inputs): typed arrays
// over a SharedArrayBuffer -- what the reference's own compute_msm allocates
// (submission.ts:35-39) and what submission.mjs's flattenU32 builds -- cannot be detached, so they
// are read in place (a reference keeps them alive; writing them before the promise settles races
// with the upload).  Typed arrays over a plain ArrayBuffer could be detached (transferred) by the
// caller while the job runs, freeing the memory under the worker, so they are copied first.
//   pointAddAffine(a: Uint32Array(16), b: Uint32Array(16)) -> Uint32Array(16)      (lib.rs:240-253)
//   split(windowSize, scalars: Uint32Array(8n)) -> Uint32Array(W*n)                 (lib.rs:196-202)
//   bestWindowSize(n) -> number                                                     (submission.ts:18-23)
//   init() -> number (0 ok), deviceCount() -> number, deviceOrdinals() -> number[],
//   strerror(code) -> string
#include <node_api.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "msm.h"

namespace {

#define NAPI_OK(call)                                              \
  do {                                                             \
    if ((call) != napi_ok) {                                       \
      napi_throw_error(env, nullptr, "N-API call failed: " #call); \
      return nullptr;                                              \
    }                                                              \
  } while (0)

// Staging for the copies of plain-ArrayBuffer inputs: one buffer pair kept between calls (its pages
// stay mapped: a fresh 160 MB allocation per 2^20 call spent ~60 ms in first-touch page faults),
// lent to one job at a time; a concurrent job gets its own and frees it when done.  The cached pair
// is kept only up to MSM_NODE_STAGING_CACHE_MB (default 256 MiB: a 2^20 MSM's 160 MiB); a larger
// one is freed after its job.  SharedArrayBuffer inputs need no staging at all.
struct Staging {
  std::vector<uint32_t> points, scalars;
  size_t bytes() const { return (points.capacity() + scalars.capacity()) * 4; }
};
std::mutex g_stage_mu;
Staging* g_stage = nullptr;  // the idle cached pair, or null while lent out

size_t staging_cache_cap() {
  static const size_t cap = (getenv("MSM_NODE_STAGING_CACHE_MB") ? (size_t)atol(getenv("MSM_NODE_STAGING_CACHE_MB"))
                                                                  : (size_t)256) << 20;
  return cap;
}

Staging* take_staging() {
  std::lock_guard<std::mutex> lk(g_stage_mu);
  Staging* s = g_stage ? g_stage : new Staging();
  g_stage = nullptr;
  return s;
}
void give_staging(Staging* s) {
  std::lock_guard<std::mutex> lk(g_stage_mu);
  if (!g_stage && s->bytes() <= staging_cache_cap()) {
    g_stage = s;
  } else {
    delete s;
  }
}

// dst[0..n) = src[0..n) over a few threads (one thread copies ~10 GB/s)
void copy_words(uint32_t* dst, const uint32_t* src, size_t n) {
  const size_t parts = n >= (1u << 20) ? 8 : 1;
  std::vector<std::thread> th;
  const size_t per = (n + parts - 1) / parts;
  for (size_t k = 1; k < parts; k++) {
    const size_t lo = std::min(n, k * per), hi = std::min(n, lo + per);
    th.emplace_back([=] { memcpy(dst + lo, src + lo, (hi - lo) * 4); });
  }
  memcpy(dst, src, std::min(n, per) * 4);
  for (auto& t : th) t.join();
}

struct Job {
  napi_async_work work = nullptr;
  napi_deferred deferred = nullptr;
  // marshalled BigInt inputs (computeMsmBigInt)
  std::vector<uint32_t> points, scalars;
  // the copy of plain-ArrayBuffer typed arrays (computeMsmU32), returned to the cache when done
  Staging* stage = nullptr;
  // computeMsmU32 over SharedArrayBuffers: the caller's arrays, held by references until the job
  // completes and read in place by msm_compute
  napi_ref ref_points = nullptr, ref_scalars = nullptr;
  const uint32_t* p_points = nullptr;
  const uint32_t* p_scalars = nullptr;
  size_t n = 0;
  uint32_t window = 0;
  std::vector<int32_t> devices;  // empty: the current device
  double cpu_work_ratio = 0;     // > 0: CPU/GPU co-compute (msm_compute_cocompute)
  uint32_t out[16] = {0};
  int rc = 0;
};

void execute(napi_env, void* data) {
  Job* j = static_cast<Job*>(data);
  msm_opts o;
  memset(&o, 0, sizeof(o));
  o.window_bits = j->window;
  o.device = -1;
  if (!j->devices.empty()) {
    o.flags |= MSM_FLAG_DEVICES;
    o.devices = j->devices.data();
    o.n_devices = (uint32_t)j->devices.size();
  }
  const uint32_t* pts = j->p_points ? j->p_points : j->stage ? j->stage->points.data() : j->points.data();
  const uint32_t* sc = j->p_scalars ? j->p_scalars : j->stage ? j->stage->scalars.data() : j->scalars.data();
  j->rc = j->cpu_work_ratio != 0 ? msm_compute_cocompute(pts, sc, j->n, &o, j->cpu_work_ratio, 0, j->out)
                                  : msm_compute(pts, sc, j->n, &o, j->out);
}

void complete(napi_env env, napi_status, void* data) {
  Job* j = static_cast<Job*>(data);
  if (j->rc == MSM_OK) {
    napi_value ab, arr;
    void* buf;
    napi_create_arraybuffer(env, 64, &buf, &ab);
    memcpy(buf, j->out, 64);
    napi_create_typedarray(env, napi_uint32_array, 16, ab, 0, &arr);
    napi_resolve_deferred(env, j->deferred, arr);
  } else {
    napi_value msg, code, err;
    std::string m = std::string("libmsm: ") + msm_strerror(j->rc);
    napi_create_string_utf8(env, m.c_str(), m.size(), &msg);
    napi_create_int32(env, j->rc, &code);
    napi_create_error(env, nullptr, msg, &err);
    napi_set_named_property(env, err, "code", code);
    napi_reject_deferred(env, j->deferred, err);
  }
  if (j->ref_points) napi_delete_reference(env, j->ref_points);
  if (j->ref_scalars) napi_delete_reference(env, j->ref_scalars);
  if (j->stage) give_staging(j->stage);
  napi_delete_async_work(env, j->work);
  delete j;
}

napi_value start_job(napi_env env, Job* j) {
  napi_value promise, name;
  NAPI_OK(napi_create_promise(env, &j->deferred, &promise));
  NAPI_OK(napi_create_string_utf8(env, "msm_compute", NAPI_AUTO_LENGTH, &name));
  NAPI_OK(napi_create_async_work(env, nullptr, name, execute, complete, j, &j->work));
  NAPI_OK(napi_queue_async_work(env, j->work));
  return promise;
}

bool get_u32_array(napi_env env, napi_value v, const uint32_t** data, size_t* len, bool* shared = nullptr) {
  bool is_ta = false;
  if (napi_is_typedarray(env, v, &is_ta) != napi_ok || !is_ta) return false;
  napi_typedarray_type t;
  void* d;
  napi_value ab;
  size_t off;
  if (napi_get_typedarray_info(env, v, &t, len, &d, &ab, &off) != napi_ok || t != napi_uint32_array) return false;
  *data = static_cast<const uint32_t*>(d);
  if (shared) {  // napi_is_arraybuffer is false for a SharedArrayBuffer
    bool plain = true;
    if (napi_is_arraybuffer(env, ab, &plain) != napi_ok) return false;
    *shared = !plain;
  }
  return true;
}

// Optional device list: an array of HIP ordinals (undefined / null: none).  false on a bad value.
bool get_devices(napi_env env, size_t argc, napi_value* argv, size_t at, std::vector<int32_t>* out) {
  out->clear();
  if (argc <= at) return true;
  napi_valuetype vt;
  if (napi_typeof(env, argv[at], &vt) != napi_ok) return false;
  if (vt == napi_undefined || vt == napi_null) return true;
  bool arr = false;
  if (napi_is_array(env, argv[at], &arr) != napi_ok || !arr) return false;
  uint32_t len = 0;
  if (napi_get_array_length(env, argv[at], &len) != napi_ok) return false;
  for (uint32_t i = 0; i < len; i++) {
    napi_value e;
    int32_t d;
    if (napi_get_element(env, argv[at], i, &e) != napi_ok || napi_get_value_int32(env, e, &d) != napi_ok) return false;
    out->push_back(d);
  }
  return true;  // shape and ordinals are checked by libmsm (msm_opts, MSM_ERR_INVALID_ARG)
}

// Optional cpuWorkRatio (submission.ts:95-98): a number >= 0 (undefined / null: 0).  false on a bad value.
bool get_ratio(napi_env env, size_t argc, napi_value* argv, size_t at, double* out) {
  *out = 0;
  if (argc <= at) return true;
  napi_valuetype vt;
  if (napi_typeof(env, argv[at], &vt) != napi_ok) return false;
  if (vt == napi_undefined || vt == napi_null) return true;
  if (vt != napi_number || napi_get_value_double(env, argv[at], out) != napi_ok) return false;
  return *out >= 0;  // NaN and negatives rejected here (libmsm rejects them too)
}

uint32_t get_window(napi_env env, napi_value v) {
  napi_valuetype t;
  if (napi_typeof(env, v, &t) != napi_ok || t != napi_number) return 0;
  uint32_t w = 0;
  napi_get_value_uint32(env, v, &w);
  return w;
}

napi_value ComputeMsmU32(napi_env env, napi_callback_info info) {
  size_t argc = 5;
  napi_value argv[5];
  NAPI_OK(napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  const uint32_t *pts, *sc;
  size_t plen, slen;
  bool pshared = false, sshared = false;
  std::vector<int32_t> devs;
  double ratio = 0;
  if (argc < 2 || !get_u32_array(env, argv[0], &pts, &plen, &pshared) ||
      !get_u32_array(env, argv[1], &sc, &slen, &sshared) || !get_devices(env, argc, argv, 3, &devs) ||
      !get_ratio(env, argc, argv, 4, &ratio)) {
    napi_throw_type_error(env, nullptr,
                          "computeMsmU32(points: Uint32Array, scalars: Uint32Array, windowSize?, devices?: number[], "
                          "cpuWorkRatio?: number >= 0)");
    return nullptr;
  }
  Job* j = new Job();
  j->n = std::min(plen / 32, slen / 8);
  j->devices = std::move(devs);
  j->cpu_work_ratio = ratio;
  if (pshared && sshared) {
    j->p_points = pts;
    j->p_scalars = sc;
    if (napi_create_reference(env, argv[0], 1, &j->ref_points) != napi_ok ||
        napi_create_reference(env, argv[1], 1, &j->ref_scalars) != napi_ok) {
      if (j->ref_points) napi_delete_reference(env, j->ref_points);
      delete j;
      napi_throw_error(env, nullptr, "cannot reference the input arrays");
      return nullptr;
    }
  } else {  // detachable memory: the worker reads a copy
    j->stage = take_staging();
    if (j->stage->points.size() < j->n * 32) j->stage->points.resize(j->n * 32);
    if (j->stage->scalars.size() < j->n * 8) j->stage->scalars.resize(j->n * 8);
    copy_words(j->stage->points.data(), pts, j->n * 32);
    copy_words(j->stage->scalars.data(), sc, j->n * 8);
  }
  j->window = argc > 2 ? get_window(env, argv[2]) : 0;
  return start_job(env, j);
}

// bigint -> 8 big-endian u32 words; false if negative or wider than 256 bits
bool bigint_be(napi_env env, napi_value v, uint32_t* out8) {
  int sign = 0;
  size_t wc = 4;
  uint64_t words[4] = {0, 0, 0, 0};
  if (napi_get_value_bigint_words(env, v, &sign, &wc, words) != napi_ok) return false;
  if (sign || wc > 4) return false;
  for (int i = 0; i < 4; i++) {
    out8[7 - 2 * i] = (uint32_t)words[i];
    out8[6 - 2 * i] = (uint32_t)(words[i] >> 32);
  }
  return true;
}

napi_value ComputeMsmBigInt(napi_env env, napi_callback_info info) {
  size_t argc = 5;
  napi_value argv[5];
  NAPI_OK(napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  bool ap = false, as = false;
  if (argc < 2 || napi_is_array(env, argv[0], &ap) != napi_ok || !ap || napi_is_array(env, argv[1], &as) != napi_ok ||
      !as) {
    napi_throw_type_error(env, nullptr, "computeMsmBigInt(points: BigIntPoint[], scalars: bigint[], windowSize?)");
    return nullptr;
  }
  uint32_t np_ = 0, ns = 0;
  NAPI_OK(napi_get_array_length(env, argv[0], &np_));
  NAPI_OK(napi_get_array_length(env, argv[1], &ns));
  Job* j = new Job();
  if (!get_devices(env, argc, argv, 3, &j->devices) || !get_ratio(env, argc, argv, 4, &j->cpu_work_ratio)) {
    delete j;
    napi_throw_type_error(env, nullptr, "devices must be an array of device ordinals, cpuWorkRatio a number >= 0");
    return nullptr;
  }
  j->n = std::min(np_, ns);
  j->points.resize(j->n * 32);
  j->scalars.resize(j->n * 8);
  // The four property keys are made once per call (napi_get_named_property would create and
  // intern a string per coordinate: 4 n of them), and the element handles live in one handle
  // scope per block of points, so the handle stack stays small instead of growing by ~6 n handles.
  static const char* names[4] = {"x", "y", "t", "z"};
  napi_value keys[4];
  for (int k = 0; k < 4; k++)
    if (napi_create_string_utf8(env, names[k], 1, &keys[k]) != napi_ok) {
      delete j;
      napi_throw_error(env, nullptr, "cannot create the coordinate keys");
      return nullptr;
    }
  constexpr uint32_t BLOCK = 1024;
  const char* bad = nullptr;  // the error of the first bad element, thrown after its scope closes
  for (uint32_t i0 = 0; i0 < j->n && !bad; i0 += BLOCK) {
    napi_handle_scope scope;
    if (napi_open_handle_scope(env, &scope) != napi_ok) {
      bad = "bad input element";
      break;
    }
    const uint32_t i1 = std::min<uint32_t>(j->n, i0 + BLOCK);
    for (uint32_t i = i0; i < i1 && !bad; i++) {
      napi_value p, s;
      if (napi_get_element(env, argv[0], i, &p) != napi_ok || napi_get_element(env, argv[1], i, &s) != napi_ok) {
        bad = "bad input element";
        break;
      }
      for (int k = 0; k < 4 && !bad; k++) {
        napi_value c;
        if (napi_get_property(env, p, keys[k], &c) != napi_ok || !bigint_be(env, c, &j->points[i * 32 + 8 * k]))
          bad = "point coordinate must be a bigint in [0, 2^256)";
      }
      if (!bad && !bigint_be(env, s, &j->scalars[i * 8])) bad = "scalar must be a bigint in [0, 2^256)";
    }
    napi_close_handle_scope(env, scope);
  }
  if (bad) {
    delete j;
    bool pending = false;
    napi_is_exception_pending(env, &pending);  // a throwing getter: keep its exception
    if (!pending) {
      if (bad[0] == 'b') napi_throw_error(env, nullptr, bad);
      else napi_throw_range_error(env, nullptr, bad);
    }
    return nullptr;
  }
  j->window = argc > 2 ? get_window(env, argv[2]) : 0;
  return start_job(env, j);
}

napi_value make_u32(napi_env env, const uint32_t* src, size_t n) {
  napi_value ab, arr;
  void* buf;
  NAPI_OK(napi_create_arraybuffer(env, n * 4, &buf, &ab));
  if (n) memcpy(buf, src, n * 4);
  NAPI_OK(napi_create_typedarray(env, napi_uint32_array, n, ab, 0, &arr));
  return arr;
}

napi_value throw_rc(napi_env env, int rc) {
  std::string m = std::string("libmsm: ") + msm_strerror(rc);
  napi_throw_error(env, std::to_string(rc).c_str(), m.c_str());
  return nullptr;
}

napi_value PointAddAffine(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  NAPI_OK(napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  const uint32_t *a, *b;
  size_t la, lb;
  if (argc < 2 || !get_u32_array(env, argv[0], &a, &la) || !get_u32_array(env, argv[1], &b, &lb) || la != 16 ||
      lb != 16) {
    napi_throw_type_error(env, nullptr, "pointAddAffine(a: Uint32Array(16), b: Uint32Array(16))");
    return nullptr;
  }
  uint32_t out[16];
  int rc = msm_point_add_affine(a, b, out);
  if (rc != MSM_OK) return throw_rc(env, rc);
  return make_u32(env, out, 16);
}

napi_value Split(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  NAPI_OK(napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  const uint32_t* sc;
  size_t len;
  uint32_t c = argc > 0 ? get_window(env, argv[0]) : 0;
  if (argc < 2 || !get_u32_array(env, argv[1], &sc, &len)) {
    napi_throw_type_error(env, nullptr, "split(windowSize, scalars: Uint32Array)");
    return nullptr;
  }
  size_t n = len / 8;
  uint32_t nw = msm_split_windows(c);
  std::vector<uint32_t> out((size_t)nw * n + 1);
  int rc = msm_split(c, sc, n, out.data());
  if (rc != MSM_OK) return throw_rc(env, rc);
  return make_u32(env, out.data(), (size_t)nw * n);
}

// flattenU32(points, scalars, pointWords, scalarWords): U32ArrayPoint[] / Uint32Array[] into flat
// wire buffers (x|y|t|z BE words per point, submission.ts:75-86), natively: per point one property
// read per coordinate (keys made once) and one typed-array lookup, then a 32-B copy.  The A/B
// against the JS loop (flattenU32 in submission.mjs) is tools/node_flatten_ab.mjs.
napi_value FlattenU32(napi_env env, napi_callback_info info) {
  size_t argc = 4;
  napi_value argv[4];
  NAPI_OK(napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  if (argc < 4) {
    napi_throw_type_error(env, nullptr, "flattenU32(points, scalars, pointWords, scalarWords)");
    return nullptr;
  }
  uint32_t np_ = 0, ns = 0;
  NAPI_OK(napi_get_array_length(env, argv[0], &np_));
  NAPI_OK(napi_get_array_length(env, argv[1], &ns));
  const uint32_t n = std::min(np_, ns);
  const uint32_t *pwc = nullptr, *swc = nullptr;
  size_t plen = 0, slen = 0;
  if (!get_u32_array(env, argv[2], &pwc, &plen) || !get_u32_array(env, argv[3], &swc, &slen) ||
      plen < (size_t)n * 32 || slen < (size_t)n * 8) {
    napi_throw_type_error(env, nullptr, "pointWords / scalarWords must be Uint32Arrays of n x 32 / n x 8 words");
    return nullptr;
  }
  uint32_t* pw = const_cast<uint32_t*>(pwc);  // the caller's output buffers
  uint32_t* sw = const_cast<uint32_t*>(swc);
  static const char* names[4] = {"x", "y", "t", "z"};
  napi_value keys[4];
  for (int k = 0; k < 4; k++) NAPI_OK(napi_create_string_utf8(env, names[k], 1, &keys[k]));
  constexpr uint32_t BLOCK = 1024;
  const char* bad = nullptr;
  for (uint32_t i0 = 0; i0 < n && !bad; i0 += BLOCK) {
    napi_handle_scope scope;
    if (napi_open_handle_scope(env, &scope) != napi_ok) {
      bad = "bad input element";
      break;
    }
    const uint32_t i1 = std::min<uint32_t>(n, i0 + BLOCK);
    for (uint32_t i = i0; i < i1 && !bad; i++) {
      napi_value p, s;
      const uint32_t* src;
      size_t len;
      if (napi_get_element(env, argv[0], i, &p) != napi_ok || napi_get_element(env, argv[1], i, &s) != napi_ok) {
        bad = "bad input element";
        break;
      }
      for (int k = 0; k < 4 && !bad; k++) {
        napi_value c;
        if (napi_get_property(env, p, keys[k], &c) != napi_ok || !get_u32_array(env, c, &src, &len) || len < 8)
          bad = "point coordinates must be Uint32Arrays of 8 words";
        else
          memcpy(pw + (size_t)i * 32 + 8 * k, src, 32);
      }
      if (!bad) {
        if (!get_u32_array(env, s, &src, &len) || len < 8)
          bad = "scalars must be Uint32Arrays of 8 words";
        else
          memcpy(sw + (size_t)i * 8, src, 32);
      }
    }
    napi_close_handle_scope(env, scope);
  }
  if (bad) {
    bool pending = false;
    napi_is_exception_pending(env, &pending);
    if (!pending) napi_throw_type_error(env, nullptr, bad);
    return nullptr;
  }
  napi_value r;
  NAPI_OK(napi_create_uint32(env, n, &r));
  return r;
}

napi_value BestWindowSize(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  NAPI_OK(napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  double n = 0;
  if (argc > 0) napi_get_value_double(env, argv[0], &n);
  napi_value r;
  NAPI_OK(napi_create_uint32(env, msm_best_window((size_t)n), &r));
  return r;
}

napi_value Init(napi_env env, napi_callback_info) {
  napi_value r;
  NAPI_OK(napi_create_int32(env, msm_init(), &r));
  return r;
}

napi_value DeviceCount(napi_env env, napi_callback_info) {
  napi_value r;
  NAPI_OK(napi_create_int32(env, msm_device_count(), &r));
  return r;
}

// HIP ordinals of the gfx950 devices (the values a `devices` list takes).
napi_value DeviceOrdinals(napi_env env, napi_callback_info) {
  napi_value arr;
  const int n = msm_device_count();
  NAPI_OK(napi_create_array_with_length(env, n > 0 ? n : 0, &arr));
  for (int i = 0; i < n; i++) {
    napi_value v;
    NAPI_OK(napi_create_int32(env, msm_device_ordinal(i), &v));
    NAPI_OK(napi_set_element(env, arr, i, v));
  }
  return arr;
}

napi_value StrError(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  NAPI_OK(napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
  int32_t code = 0;
  if (argc > 0) napi_get_value_int32(env, argv[0], &code);
  napi_value r;
  NAPI_OK(napi_create_string_utf8(env, msm_strerror(code), NAPI_AUTO_LENGTH, &r));
  return r;
}

// Explicit teardown when the last environment that loaded the addon is torn down (process exit
// of the main thread, or the last worker): the library's streams, buffers and parked pool threads
// are released and joined then, not left to the shared objects' finalizers.  (A call in flight
// holds its device context, which msm_shutdown waits for.)
std::atomic<int> g_envs{0};
void CleanupEnv(void*) {
  if (g_envs.fetch_sub(1) == 1) msm_shutdown();
}

napi_value ModuleInit(napi_env env, napi_value exports) {
  if (napi_add_env_cleanup_hook(env, CleanupEnv, nullptr) == napi_ok) g_envs.fetch_add(1);
  napi_property_descriptor props[] = {
      {"computeMsmU32", nullptr, ComputeMsmU32, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
      {"computeMsmBigInt", nullptr, ComputeMsmBigInt, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
      {"pointAddAffine", nullptr, PointAddAffine, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
      {"split", nullptr, Split, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
      {"flattenU32", nullptr, FlattenU32, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
      {"bestWindowSize", nullptr, BestWindowSize, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
      {"init", nullptr, Init, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
      {"deviceCount", nullptr, DeviceCount, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
      {"deviceOrdinals", nullptr, DeviceOrdinals, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
      {"strerror", nullptr, StrError, nullptr, nullptr, nullptr, napi_enumerable, nullptr},
  };
  napi_define_properties(env, exports, sizeof(props) / sizeof(props[0]), props);
  return exports;
}

}  // namespace

NAPI_MODULE(NODE_GYP_MODULE_NAME, ModuleInit)
