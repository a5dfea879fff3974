// Synthetic-input generators (host, multithreaded): msm_gen_points / msm_gen_scalars.
// Mirrors the benchmark page's input generation (src/ui/AllBenchmarks.tsx:107-140, fixed base
// point; src/reference/webgpu/utils.ts:81-100, scalars uniform mod p) with a deterministic
// spec: P_i = (k0 + i step) G, scalars from xorshift64.
#pragma once
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "hostfield.h"

namespace msmh {

static inline Pt pt_mul_u64(const Pt& p, uint64_t k) {
  Pt r = pt_identity();
  for (int b = 63; b >= 0; b--) {
    r = pt_dbl(r);
    if ((k >> b) & 1) r = pt_add(r, p);
  }
  return r;
}

static inline void gen_points_range(const Pt& g, uint64_t k0, uint64_t step, size_t lo, size_t hi, uint32_t* out) {
  if (lo >= hi) return;
  Pt cur = pt_mul_u64(g, k0 + lo * step);  // k fits u64 for any realistic n
  Pt stp = pt_mul_u64(g, step);
  const size_t BLK = 512;
  std::vector<Pt> blk(BLK);
  std::vector<Fq> pref(BLK);
  for (size_t base = lo; base < hi; base += BLK) {
    size_t m = std::min(BLK, hi - base);
    for (size_t i = 0; i < m; i++) {
      blk[i] = cur;
      cur = pt_add(cur, stp);
    }
    Fq acc = fq_one();
    for (size_t i = 0; i < m; i++) {
      pref[i] = acc;
      acc = fq_mul(acc, blk[i].Z);
    }
    Fq inv = fq_inv(acc);
    for (size_t ii = m; ii-- > 0;) {
      Fq zi = fq_mul(inv, pref[ii]);
      inv = fq_mul(inv, blk[ii].Z);
      Fq xa = fq_mul(blk[ii].X, zi), ya = fq_mul(blk[ii].Y, zi);
      uint64_t x[4], y[4], t[4], one[4] = {1, 0, 0, 0};
      fq_to_std(xa, x);
      fq_to_std(ya, y);
      fq_to_std(fq_mul(xa, ya), t);
      uint32_t* o = out + 32 * (base + ii);
      std_to_be_words(x, o);
      std_to_be_words(y, o + 8);
      std_to_be_words(t, o + 16);
      std_to_be_words(one, o + 24);
    }
  }
}

// Threads the host can run at once: the hardware threads, capped by a cgroup-v2 CPU quota
// (/sys/fs/cgroup/cpu.max = "quota period"): a container reports the whole machine's threads
// (256 on an MI355X node) while its quota may allow 16, and 256 threads on 16 CPUs thrash.
static inline unsigned host_threads() {
  static const unsigned t = [] {
    unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
      char quota[32] = {0};
      unsigned long long period = 0;
      if (fscanf(f, "%31s %llu", quota, &period) == 2 && strcmp(quota, "max") != 0 && period > 0)
        hw = (unsigned)std::min<unsigned long long>(hw, std::max(1ull, strtoull(quota, nullptr, 10) / period));
      fclose(f);
    }
    return hw;
  }();
  return t;
}

static inline void gen_points(const Pt& g, uint64_t k0, uint64_t step, size_t n, uint32_t* out) {
  unsigned th = std::max(1u, std::min(64u, host_threads()));
  if (n < 4096) th = 1;
  std::vector<std::thread> ts;
  size_t per = (n + th - 1) / th;
  for (unsigned t = 0; t < th; t++) {
    size_t lo = t * per, hi = std::min(n, lo + per);
    ts.emplace_back(gen_points_range, g, k0, step, lo, hi, out);
  }
  for (auto& t : ts) t.join();
}

static inline void gen_scalars(uint64_t seed, size_t n, uint32_t* out) {
  uint64_t s = seed;
  for (size_t i = 0; i < n; i++) {
    uint64_t w[4];
    for (int j = 0; j < 4; j++) {
      s ^= s << 13;
      s ^= s >> 7;
      s ^= s << 17;
      w[j] = s;  // w[0] most significant
    }
    uint64_t v[4] = {w[3], w[2], w[1], w[0]};  // little-endian limbs
    // reduce mod p: v < 2^256 < 14 p
    while (!std_lt_p(v)) {
      unsigned __int128 br = 0;
      for (int k = 0; k < 4; k++) {
        unsigned __int128 t = (unsigned __int128)v[k] - P[k] - br;
        v[k] = (uint64_t)t;
        br = (t >> 64) ? 1 : 0;
      }
    }
    std_to_be_words(v, out + 8 * i);
  }
}

}  // namespace msmh
