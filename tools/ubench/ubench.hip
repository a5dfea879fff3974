// Instruction-rate microbenchmarks for gfx950 integer wide-arithmetic building blocks.
// Each kernel runs ITER iterations of U independent instruction chains per lane so that
// throughput (not latency) bounds it; the host prints wave-instructions per CU per cycle.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#define CHECK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP error %s at %d\n",hipGetErrorString(e),__LINE__); exit(1);}}while(0)

constexpr int ITER = 2048;

__global__ void k_mad64(uint32_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x ^ seed, b = a * 7 + 1;
  uint64_t acc[8];
  for (int u = 0; u < 8; u++) acc[u] = a + u;
  for (int it = 0; it < ITER; it++) {
#pragma unroll
    for (int u = 0; u < 8; u++)
      asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0" : "+v"(acc[u]) : "v"(a), "v"(b) : "s0", "s1");
  }
  uint64_t s = 0; for (int u = 0; u < 8; u++) s += acc[u];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s ^ (uint32_t)(s >> 32);
}
__global__ void k_mulhi(uint32_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x ^ seed, b = a * 7 + 1;
  uint32_t acc[8];
  for (int u = 0; u < 8; u++) acc[u] = a + u;
  for (int it = 0; it < ITER; it++) {
#pragma unroll
    for (int u = 0; u < 8; u++)
      asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(acc[u]) : "v"(b));
  }
  uint32_t s = 0; for (int u = 0; u < 8; u++) s += acc[u];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_mullo(uint32_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x ^ seed, b = a * 7 + 1;
  uint32_t acc[8];
  for (int u = 0; u < 8; u++) acc[u] = a + u;
  for (int it = 0; it < ITER; it++) {
#pragma unroll
    for (int u = 0; u < 8; u++)
      asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(acc[u]) : "v"(b));
  }
  uint32_t s = 0; for (int u = 0; u < 8; u++) s += acc[u];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_addc(uint32_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x ^ seed;
  uint32_t acc[8];
  for (int u = 0; u < 8; u++) acc[u] = a + u;
  for (int it = 0; it < ITER; it++) {
#pragma unroll
    for (int u = 0; u < 8; u++)
      asm volatile("v_addc_co_u32 %0, s[0:1], %0, %1, s[2:3]" : "+v"(acc[u]) : "v"(a) : "s0", "s1");
  }
  uint32_t s = 0; for (int u = 0; u < 8; u++) s += acc[u];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_add(uint32_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x ^ seed;
  uint32_t acc[8];
  for (int u = 0; u < 8; u++) acc[u] = a + u;
  for (int it = 0; it < ITER; it++) {
#pragma unroll
    for (int u = 0; u < 8; u++)
      asm volatile("v_add_u32 %0, %0, %1" : "+v"(acc[u]) : "v"(a));
  }
  uint32_t s = 0; for (int u = 0; u < 8; u++) s += acc[u];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_lshladd64(uint32_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x ^ seed;
  uint64_t b = a * 3ull;
  uint64_t acc[8];
  for (int u = 0; u < 8; u++) acc[u] = a + u;
  for (int it = 0; it < ITER; it++) {
#pragma unroll
    for (int u = 0; u < 8; u++)
      asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(acc[u]) : "v"(b));
  }
  uint64_t s = 0; for (int u = 0; u < 8; u++) s += acc[u];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s;
}
__global__ void k_mad24(uint32_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x ^ seed, b = a * 7 + 1;
  uint32_t acc[8];
  for (int u = 0; u < 8; u++) acc[u] = a + u;
  for (int it = 0; it < ITER; it++) {
#pragma unroll
    for (int u = 0; u < 8; u++)
      asm volatile("v_mad_u32_u24 %0, %1, %2, %0" : "+v"(acc[u]) : "v"(a), "v"(b));
  }
  uint32_t s = 0; for (int u = 0; u < 8; u++) s += acc[u];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_fma64(uint32_t* out, uint32_t seed) {
  double a = (threadIdx.x ^ seed) * 1e-3, b = 1.0000001;
  double acc[8];
  for (int u = 0; u < 8; u++) acc[u] = a + u;
  for (int it = 0; it < ITER; it++) {
#pragma unroll
    for (int u = 0; u < 8; u++)
      asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(acc[u]) : "v"(b), "v"(a));
  }
  double s = 0; for (int u = 0; u < 8; u++) s += acc[u];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(s);
}
// latency: one dependent chain
__global__ void k_mad64_lat(uint32_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x ^ seed, b = a * 7 + 1;
  uint64_t acc = a;
  for (int it = 0; it < ITER * 8; it++)
    asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b) : "s0", "s1");
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)acc;
}

typedef void (*kfn)(uint32_t*, uint32_t);
int main() {
  hipDeviceProp_t prop; CHECK(hipGetDeviceProperties(&prop, 0));
  int cus = prop.multiProcessorCount; int clk_khz = prop.clockRate;
  printf("device %s CUs %d clock %d MHz\n", prop.gcnArchName, cus, clk_khz / 1000);
  uint32_t* out; CHECK(hipMalloc(&out, 64ull << 20));
  struct { const char* name; kfn f; } ks[] = {
    {"v_mad_u64_u32", k_mad64}, {"v_mul_hi_u32", k_mulhi}, {"v_mul_lo_u32", k_mullo},
    {"v_addc_co_u32", k_addc}, {"v_add_u32", k_add}, {"v_lshl_add_u64", k_lshladd64},
    {"v_mad_u32_u24", k_mad24}, {"v_fma_f64", k_fma64}};
  hipEvent_t e0, e1; CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  for (int wavesPerSimd : {1, 2, 4, 8}) {
    int block = 256; int grid = cus * wavesPerSimd;  // 4 waves per block = 1 per SIMD
    for (auto& k : ks) {
      hipLaunchKernelGGL(k.f, dim3(grid), dim3(block), 0, 0, out, 1u);
      CHECK(hipDeviceSynchronize());
      CHECK(hipEventRecord(e0));
      for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k.f, dim3(grid), dim3(block), 0, 0, out, 1u);
      CHECK(hipEventRecord(e1)); CHECK(hipEventSynchronize(e1));
      float ms; CHECK(hipEventElapsedTime(&ms, e0, e1)); ms /= 5;
      double winstr = (double)grid * (block / 64) * ITER * 8;  // wave-instructions
      double per_cu_per_ns = winstr / cus / (ms * 1e6);
      double lane_ops = winstr * 64 / (ms * 1e-3);
      printf("waves/SIMD %d  %-16s %8.3f ms  %.3f wave-instr/CU/ns  (%.1f cyc/wave-instr/SIMD @2.4GHz)  %.2f Tlane-op/s\n",
             wavesPerSimd, k.name, ms, per_cu_per_ns, 4.0 * 2.4 / per_cu_per_ns, lane_ops / 1e12);
    }
  }
  {
    int grid = cus; int block = 64;
    hipLaunchKernelGGL(k_mad64_lat, dim3(grid), dim3(block), 0, 0, out, 1u);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_mad64_lat, dim3(grid), dim3(block), 0, 0, out, 1u);
    CHECK(hipEventRecord(e1)); CHECK(hipEventSynchronize(e1));
    float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
    printf("mad64 dependent-chain latency: %.2f ns per instr (%.1f cycles @2.4GHz)\n", ms * 1e6 / (ITER * 8), ms * 1e6 / (ITER * 8) * 2.4);
  }
  return 0;
}
