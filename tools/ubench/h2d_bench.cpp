// Host->device upload microbenchmark (MI355X box): picks the host-input staging strategy of
// msm_compute.  Prints one JSON line per measurement.
//   hipcc -O2 -std=c++17 --offload-arch=gfx950 -o h2d_bench h2d_bench.cpp -lpthread
#include <hip/hip_runtime.h>
#include <sys/mman.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

using clk = std::chrono::steady_clock;
static double ms_since(clk::time_point t0) { return std::chrono::duration<double, std::milli>(clk::now() - t0).count(); }

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e));        \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

static void par_copy(char* dst, const char* src, size_t bytes, int th) {
  if (th <= 1) {
    memcpy(dst, src, bytes);
    return;
  }
  std::vector<std::thread> ts;
  size_t per = (bytes + th - 1) / th;
  per = (per + 4095) & ~size_t(4095);
  for (int t = 0; t < th; t++) {
    size_t lo = std::min(bytes, t * per), hi = std::min(bytes, lo + per);
    ts.emplace_back([=] { memcpy(dst + lo, src + lo, hi - lo); });
  }
  for (auto& t : ts) t.join();
}

// persistent pool: workers spin on a generation counter while a call is active
struct Pool {
  int n;
  std::vector<std::thread> ts;
  std::atomic<uint64_t> gen{0};
  std::atomic<int> done{0};
  std::atomic<bool> quit{false};
  char* dst = nullptr;
  const char* src = nullptr;
  size_t bytes = 0;
  explicit Pool(int n_) : n(n_) {
    for (int i = 1; i < n; i++)
      ts.emplace_back([this, i] {
        uint64_t seen = 0;
        while (!quit.load()) {
          uint64_t g = gen.load(std::memory_order_acquire);
          if (g == seen) {
            __builtin_ia32_pause();
            continue;
          }
          seen = g;
          part(i);
          done.fetch_add(1, std::memory_order_release);
        }
      });
  }
  void part(int i) {
    size_t per = ((bytes + n - 1) / n + 4095) & ~size_t(4095);
    size_t lo = std::min(bytes, i * per), hi = std::min(bytes, lo + per);
    if (hi > lo) memcpy(dst + lo, src + lo, hi - lo);
  }
  void copy(char* d, const char* s, size_t b) {
    dst = d;
    src = s;
    bytes = b;
    done.store(0);
    gen.fetch_add(1, std::memory_order_release);
    part(0);
    while (done.load(std::memory_order_acquire) < n - 1) __builtin_ia32_pause();
  }
  ~Pool() {
    quit = true;
    for (auto& t : ts) t.join();
  }
};

int main(int argc, char** argv) {
  const size_t MB = 1 << 20;
  const size_t total = (argc > 1 ? atoi(argv[1]) : 160) * MB;
  char* host = (char*)aligned_alloc(4096, total);
  for (size_t i = 0; i < total; i += 8) *(uint64_t*)(host + i) = i * 0x9E3779B97F4A7C15ull;
  void* dev;
  CK(hipMalloc(&dev, total));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  auto rep = [&](const char* what, double ms, const char* extra = "") {
    printf("{\"what\": \"%s\", \"ms\": %.3f, \"GBps\": %.1f%s}\n", what, ms, total / ms / 1e6, extra);
    fflush(stdout);
  };
  // pageable
  for (int r = 0; r < 3; r++) {
    auto t0 = clk::now();
    CK(hipMemcpyAsync(dev, host, total, hipMemcpyHostToDevice, s));
    CK(hipStreamSynchronize(s));
    if (r == 2) rep("pageable_memcpy", ms_since(t0));
  }
  // pageable sources by page type: the copy engine's rate depends on how the source is mapped
  // (numpy's large arrays are transparent-huge-page backed; a Node SharedArrayBuffer need not be)
  for (int kind = 0; kind < 4; kind++) {
    static const char* names[4] = {"src_thp_madvise", "src_nohugepage", "src_mmap_shared", "src_mmap_private"};
    char* src = nullptr;
    if (kind < 2) {
      src = (char*)aligned_alloc(2 * MB, total);
      madvise(src, total, kind == 0 ? MADV_HUGEPAGE : MADV_NOHUGEPAGE);
    } else {
      void* m = mmap(nullptr, total, PROT_READ | PROT_WRITE, (kind == 2 ? MAP_SHARED : MAP_PRIVATE) | MAP_ANONYMOUS, -1, 0);
      if (m == MAP_FAILED) continue;
      src = (char*)m;
    }
    memcpy(src, host, total);
    double best = 1e9;
    for (int r = 0; r < 4; r++) {
      auto t0 = clk::now();
      CK(hipMemcpyAsync(dev, src, total, hipMemcpyHostToDevice, s));
      CK(hipStreamSynchronize(s));
      if (r) best = std::min(best, ms_since(t0));
    }
    rep(names[kind], best);
    if (kind < 2) free(src);
    else munmap(src, total);
  }
  // pageable source in pieces (the host-input split's copies): one stream, or alternating over two
  // streams (whether a second copy queue hides the ~20 us gap between consecutive copies)
  {
    hipStream_t s2;
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    for (int pieces : {8, 10, 16}) {
      for (int streams : {1, 2}) {
        double best = 1e9;
        for (int r = 0; r < 3; r++) {
          const size_t per = total / pieces;
          auto t0 = clk::now();
          for (int k = 0; k < pieces; k++)
            CK(hipMemcpyAsync((char*)dev + k * per, host + k * per, per, hipMemcpyHostToDevice,
                              (streams == 2 && (k & 1)) ? s2 : s));
          CK(hipStreamSynchronize(s));
          CK(hipStreamSynchronize(s2));
          best = std::min(best, ms_since(t0));
        }
        char ex[96];
        snprintf(ex, sizeof ex, ", \"pieces\": %d, \"streams\": %d", pieces, streams);
        rep("pageable_pieces", best, ex);
      }
    }
    CK(hipStreamDestroy(s2));
  }
  // strided: only part of every 128-B point record (x|y = 64 B and z = 32 B of x|y|t|z: t
  // derived on the device) by 2D copies from the pageable array -- payload GB/s against the whole
  // 128-B records' contiguous copy
  for (int variant = 0; variant < 3; variant++) {
    const size_t pts = total / 128;
    double best = 1e9;
    for (int r = 0; r < 3; r++) {
      auto t0 = clk::now();
      if (variant == 0) {  // x|y only
        CK(hipMemcpy2DAsync(dev, 64, host, 128, 64, pts, hipMemcpyHostToDevice, s));
      } else if (variant == 1) {  // x|y and z: two 2D copies into two device arrays
        CK(hipMemcpy2DAsync(dev, 64, host, 128, 64, pts, hipMemcpyHostToDevice, s));
        CK(hipMemcpy2DAsync((char*)dev + pts * 64, 32, host + 96, 128, 32, pts, hipMemcpyHostToDevice, s));
      } else {  // x|y|t (96 B) in one 2D copy
        CK(hipMemcpy2DAsync(dev, 96, host, 128, 96, pts, hipMemcpyHostToDevice, s));
      }
      CK(hipStreamSynchronize(s));
      best = std::min(best, ms_since(t0));
    }
    static const char* names[3] = {"strided_xy", "strided_xy_and_z", "strided_xyt"};
    const size_t payload = variant == 0 ? pts * 64 : pts * 96;
    char ex[128];
    snprintf(ex, sizeof ex, ", \"payload_GBps\": %.1f, \"payload_MiB\": %zu", payload / best / 1e6, payload / MB);
    rep(names[variant], best, ex);
  }
  // pinned source
  char* pin;
  auto tp = clk::now();
  CK(hipHostMalloc((void**)&pin, total, hipHostMallocDefault));
  rep("hipHostMalloc_alloc", ms_since(tp));
  memcpy(pin, host, total);
  for (int r = 0; r < 3; r++) {
    auto t0 = clk::now();
    CK(hipMemcpyAsync(dev, pin, total, hipMemcpyHostToDevice, s));
    CK(hipStreamSynchronize(s));
    if (r == 2) rep("pinned_memcpy", ms_since(t0));
  }
  // register in place
  for (int r = 0; r < 2; r++) {
    auto t0 = clk::now();
    CK(hipHostRegister(host, total, hipHostRegisterDefault));
    double reg = ms_since(t0);
    auto t1 = clk::now();
    CK(hipMemcpyAsync(dev, host, total, hipMemcpyHostToDevice, s));
    CK(hipStreamSynchronize(s));
    double cp = ms_since(t1);
    auto t2 = clk::now();
    CK(hipHostUnregister(host));
    double unreg = ms_since(t2);
    char ex[128];
    snprintf(ex, sizeof ex, ", \"register_ms\": %.3f, \"copy_ms\": %.3f, \"unregister_ms\": %.3f", reg, cp, unreg);
    if (r == 1) rep("host_register_copy", reg + cp + unreg, ex);
  }
  // register a FRESH buffer each time (first-touch pages, never registered before): the cost a
  // caller's new arrays would pay
  for (int r = 0; r < 3; r++) {
    char* fresh = (char*)aligned_alloc(4096, total);
    memcpy(fresh, host, total);
    auto t0 = clk::now();
    CK(hipHostRegister(fresh, total, hipHostRegisterDefault));
    double reg = ms_since(t0);
    auto t1 = clk::now();
    CK(hipMemcpyAsync(dev, fresh, total, hipMemcpyHostToDevice, s));
    CK(hipStreamSynchronize(s));
    double cp = ms_since(t1);
    auto t2 = clk::now();
    CK(hipHostUnregister(fresh));
    double unreg = ms_since(t2);
    char ex[128];
    snprintf(ex, sizeof ex, ", \"register_ms\": %.3f, \"copy_ms\": %.3f, \"unregister_ms\": %.3f", reg, cp, unreg);
    rep("fresh_register_copy", reg + cp + unreg, ex);
    free(fresh);
  }
  // host memcpy pageable -> pinned, T threads
  for (int th : {1, 4, 8, 16, 32}) {
    Pool pool(th);
    pool.copy(pin, host, total);
    auto t0 = clk::now();
    pool.copy(pin, host, total);
    char ex[64];
    snprintf(ex, sizeof ex, ", \"threads\": %d", th);
    rep("host_memcpy_to_pinned", ms_since(t0), ex);
  }
  // staged ring: pool memcpy into pinned chunk k, async DMA, overlap
  for (int th : {8, 16}) {
    Pool pool(th);
    for (size_t chunk : {2 * MB, 4 * MB, 8 * MB, 16 * MB}) {
      const int NST = 4;
      hipEvent_t ev[NST];
      for (int k = 0; k < NST; k++) CK(hipEventCreateWithFlags(&ev[k], hipEventDisableTiming));
      double best = 1e9;
      for (int r = 0; r < 3; r++) {
        auto t0 = clk::now();
        int k = 0;
        bool used[NST] = {};
        for (size_t off = 0; off < total; off += chunk, k = (k + 1) % NST) {
          size_t b = std::min(chunk, total - off);
          if (used[k]) CK(hipEventSynchronize(ev[k]));
          pool.copy(pin + k * chunk, host + off, b);
          CK(hipMemcpyAsync((char*)dev + off, pin + k * chunk, b, hipMemcpyHostToDevice, s));
          CK(hipEventRecord(ev[k], s));
          used[k] = true;
        }
        CK(hipStreamSynchronize(s));
        best = std::min(best, ms_since(t0));
      }
      char ex[96];
      snprintf(ex, sizeof ex, ", \"threads\": %d, \"chunk_MiB\": %zu", th, chunk / MB);
      rep("staged_ring", best, ex);
      for (int k = 0; k < NST; k++) hipEventDestroy(ev[k]);
    }
  }
  // packed ring: pool threads copy only x|y (64 of every 128 B) -- or x|y|z (96) -- of the
  // pageable records into pinned chunks, each chunk DMAed while the next is packed: the compact
  // host upload (t is derived on the device; z only when some point has z != 1)
  for (int keep : {64, 96}) {
    for (int th : {4, 8, 16}) {
      Pool pool(th);
      const size_t pts = total / 128;
      for (size_t chunk_pts : {size_t(1) << 17, size_t(1) << 18}) {
        const int NST = 3;
        hipEvent_t ev[NST];
        for (int k = 0; k < NST; k++) CK(hipEventCreateWithFlags(&ev[k], hipEventDisableTiming));
        double best = 1e9;
        for (int r = 0; r < 3; r++) {
          auto t0 = clk::now();
          bool used[NST] = {};
          int k = 0;
          for (size_t p0 = 0; p0 < pts; p0 += chunk_pts, k = (k + 1) % NST) {
            const size_t np = std::min(chunk_pts, pts - p0);
            if (used[k]) CK(hipEventSynchronize(ev[k]));
            char* dst = pin + k * chunk_pts * keep;
            const char* srcp = host + p0 * 128;
            // strided pack across the pool's threads
            std::atomic<int> done{0};
            auto work = [&](size_t lo, size_t hi) {
              for (size_t i = lo; i < hi; i++) {
                memcpy(dst + i * keep, srcp + i * 128, 64);
                if (keep == 96) memcpy(dst + i * keep + 64, srcp + i * 128 + 96, 32);
              }
            };
            std::vector<std::thread> ts;
            const size_t per = (np + th - 1) / th;
            for (int t = 1; t < th; t++) ts.emplace_back(work, std::min(np, t * per), std::min(np, (t + 1) * per));
            work(0, std::min(np, per));
            for (auto& t : ts) t.join();
            (void)done;
            CK(hipMemcpyAsync((char*)dev + p0 * keep, dst, np * keep, hipMemcpyHostToDevice, s));
            CK(hipEventRecord(ev[k], s));
            used[k] = true;
          }
          CK(hipStreamSynchronize(s));
          best = std::min(best, ms_since(t0));
        }
        char ex[160];
        snprintf(ex, sizeof ex, ", \"keep_B\": %d, \"threads\": %d, \"chunk_points\": %zu, \"records_per_ms\": %.0f",
                 keep, th, chunk_pts, pts / best);
        rep("packed_ring", best, ex);
        for (int q = 0; q < NST; q++) hipEventDestroy(ev[q]);
      }
    }
  }
  // pinned source, chunked DMA (the pinned-input fast path)
  for (size_t chunk : {4 * MB, 16 * MB}) {
    auto t0 = clk::now();
    for (size_t off = 0; off < total; off += chunk)
      CK(hipMemcpyAsync((char*)dev + off, pin + off, std::min(chunk, total - off), hipMemcpyHostToDevice, s));
    CK(hipStreamSynchronize(s));
    char ex[64];
    snprintf(ex, sizeof ex, ", \"chunk_MiB\": %zu", chunk / MB);
    rep("pinned_chunked", ms_since(t0), ex);
  }
  hipHostFree(pin);
  hipFree(dev);
  free(host);
  return 0;
}
