// What LDS bank conflicts cost the sort's counting atomics (gfx950).  Tuning tool, not part of
// the product.
//
// Every workgroup (1024 threads, as k_recode_hist / k_part_scatter; 512 as k_fine_sort) keeps a
// histogram of NB counters in LDS and has each lane do R returning atomicAdd's on it per round
// -- the sort's "count and take a rank" step -- with keys drawn three ways:
//   random    xorshift keys, as random scalars give the sort (the conflicts PMC counts)
//   spread    key = (lane + 64 r) mod NB: the 64 lanes of a wave on 64 distinct banks
//   same      every lane of the wave on one counter (the skewed-scalar worst case)
// and reports ns per wave-level atomic per CU (32 waves per CU, all resident) and the implied
// time of the sort's atomics per two-MSM 2^20 launch (33.5M entries; k_recode_hist and
// k_part_scatter count each entry once into 256 coarse bins, k_fine_sort once into 128 fine ones).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define CHECK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP error %s at %d\n",hipGetErrorString(e),__LINE__); exit(1);}}while(0)

constexpr int R = 16;
constexpr int ROUNDS = 256;

template <int NB, int MODE>
__global__ void __launch_bounds__(1024) k_hist(uint32_t* out, uint32_t seed) {
  __shared__ uint32_t cnt[NB];
  for (int b = threadIdx.x; b < NB; b += blockDim.x) cnt[b] = 0;
  __syncthreads();
  uint32_t x = (threadIdx.x + 1) * 2654435761u ^ seed ^ (blockIdx.x * 40503u);
  const uint32_t lane = threadIdx.x & 63;
  uint32_t acc = 0;
  for (int it = 0; it < ROUNDS; it++) {
    uint32_t key[R];
#pragma unroll
    for (int r = 0; r < R; r++) {
      if (MODE == 0) {
        x ^= x << 13;
        x ^= x >> 17;
        x ^= x << 5;
        key[r] = x % NB;
      } else if (MODE == 1) {
        key[r] = (lane + 64u * (uint32_t)(r + it)) % NB;
      } else {
        key[r] = (uint32_t)(r + it) % NB;
      }
    }
#pragma unroll
    for (int r = 0; r < R; r++) acc += atomicAdd(&cnt[key[r]], 1u);
  }
  __syncthreads();
  if (acc == 0xdeadbeef) out[0] = acc;  // keep the returned ranks live
  if (threadIdx.x < NB) atomicAdd(&out[1 + threadIdx.x % 64], cnt[threadIdx.x]);
}

template <int NB, int MODE>
double run(int threads, int cus, uint32_t* d_out) {
  const int per_cu = 2048 / threads;  // 32 waves per CU: every workgroup resident
  const int grid = per_cu * cus;
  hipLaunchKernelGGL((k_hist<NB, MODE>), dim3(grid), dim3(threads), 0, 0, d_out, 1u);
  CHECK(hipDeviceSynchronize());
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  CHECK(hipEventRecord(a));
  const int reps = 5;
  for (int i = 0; i < reps; i++) hipLaunchKernelGGL((k_hist<NB, MODE>), dim3(grid), dim3(threads), 0, 0, d_out, 7u + i);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  const double wave_atomics_per_cu = (double)reps * per_cu * (threads / 64) * ROUNDS * R;
  return ms * 1e6 / wave_atomics_per_cu;  // ns per wave-level atomic per CU
}

int main() {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  uint32_t* d_out;
  CHECK(hipMalloc(&d_out, 4096));
  const char* names[3] = {"random", "spread", "same"};
  const double entries = 33554432.0;  // one two-MSM 2^20 launch, 16 windows
  for (int wg : {1024, 512}) {
    double ns256[3] = {run<256, 0>(wg, cus, d_out), run<256, 1>(wg, cus, d_out), run<256, 2>(wg, cus, d_out)};
    double ns128[3] = {run<128, 0>(wg, cus, d_out), run<128, 1>(wg, cus, d_out), run<128, 2>(wg, cus, d_out)};
    for (int m = 0; m < 3; m++) {
      // the sort's atomics of one launch spread over every CU at this rate
      const double us256 = entries / 64.0 / cus * ns256[m] / 1e3;
      const double us128 = entries / 64.0 / cus * ns128[m] / 1e3;
      printf("{\"workgroup\": %d, \"keys\": \"%s\", \"ns_per_wave_atomic_per_cu_256_bins\": %.3f, "
             "\"ns_per_wave_atomic_per_cu_128_bins\": %.3f, \"launch_atomics_us_256_bins\": %.2f, "
             "\"launch_atomics_us_128_bins\": %.2f, \"cus\": %d}\n",
             wg, names[m], ns256[m], ns128[m], us256, us128, cus);
    }
  }
  CHECK(hipFree(d_out));
  return 0;
}
