// Issue-rate microbenchmark for the VALU instructions fe_mul is built from (gfx950).
// Each kernel runs ITER x 16 independent instances of one instruction per lane (8 chains), at
// 8 waves/SIMD; reports cycles per wave-instruction relative to v_add_u32 (full rate = 4 cycles
// per 64-lane wave on a 16-lane SIMD).  Tuning tool, not part of the product.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define CHECK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP error %s at %d\n",hipGetErrorString(e),__LINE__); exit(1);}}while(0)
constexpr int ITER = 2048;

#define REP8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

template <int OP>
__global__ void __launch_bounds__(256) krate(uint32_t* out, uint32_t seed) {
  uint32_t a0 = threadIdx.x ^ seed, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 11, a5 = a0 * 13, a6 = a0 * 17, a7 = a0 * 19;
  uint32_t b0 = a0 + 1, b1 = a1 + 1, b2 = a2 + 1, b3 = a3 + 1, b4 = a4 + 1, b5 = a5 + 1, b6 = a6 + 1, b7 = a7 + 1;
  uint64_t c0 = a0, c1 = a1, c2 = a2, c3 = a3, c4 = a4, c5 = a5, c6 = a6, c7 = a7;
  uint32_t k = seed | 1;
  const uint64_t mask = 0x5555555555555555ull ^ seed;
  uint64_t sc0 = 0, sc1 = 0, sc2 = 0, sc3 = 0, sc4 = 0, sc5 = 0, sc6 = 0, sc7 = 0;  // live carry-outs
  for (int it = 0; it < ITER; it++) {
#pragma unroll
    for (int u = 0; u < 2; u++) {
      if constexpr (OP == 0) {
#define X(i) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a##i) : "v"(k));
        REP8(X)
#undef X
      } else if constexpr (OP == 1) {
// one carry-out SGPR pair per chain: a shared vcc would serialise the chains (WAW on vcc)
#define X(i) asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(c##i), "=s"(sc##i) : "v"(a##i), "v"(k));
        REP8(X)
#undef X
      } else if constexpr (OP == 2) {
#define X(i) asm volatile("v_lshrrev_b64 %0, 29, %0" : "+v"(c##i));
        REP8(X)
#undef X
      } else if constexpr (OP == 3) {
#define X(i) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(c##i) : "v"(c0));
        REP8(X)
#undef X
      } else if constexpr (OP == 4) {
#define X(i) asm volatile("v_and_b32 %0, 0x1fffffff, %0" : "+v"(a##i));
        REP8(X)
#undef X
      } else if constexpr (OP == 5) {
#define X(i) asm volatile("v_mad_i64_i32 %0, %1, %2, %3, %0" : "+v"(c##i), "=s"(sc##i) : "v"(a##i), "v"(k));
        REP8(X)
#undef X
      } else if constexpr (OP == 6) {
#define X(i) asm volatile("v_alignbit_b32 %0, %1, %0, 29" : "+v"(a##i) : "v"(k));
        REP8(X)
#undef X
      } else if constexpr (OP == 7) {
#define X(i) asm volatile("v_add_co_u32 %0, vcc, %0, %2\n v_addc_co_u32 %1, vcc, %1, 0, vcc" : "+v"(a##i), "+v"(b##i) : "v"(k) : "vcc");
        REP8(X)
#undef X
      } else if constexpr (OP == 8) {
#define X(i) asm volatile("v_cndmask_b32 %0, %0, %1, %2" : "+v"(a##i) : "v"(k), "s"(mask));
        REP8(X)
#undef X
      } else if constexpr (OP == 9) {
#define X(i) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a##i) : "v"(k));
        REP8(X)
#undef X
      } else if constexpr (OP == 10) {
#define X(i) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a##i) : "v"(k));
        REP8(X)
#undef X
      } else if constexpr (OP == 11) {
#define X(i) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a##i) : "v"(k));
        REP8(X)
#undef X
      } else if constexpr (OP == 12) {
#define X(i) asm volatile("v_fma_f64 %0, %0, %1, %0" : "+v"(c##i) : "v"(c0));
        REP8(X)
#undef X
      } else if constexpr (OP == 13) {
#define X(i) asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(a##i) : "v"(k));
        REP8(X)
#undef X
      } else if constexpr (OP == 14) {
#define X(i) asm volatile("v_bfe_u32 %0, %0, 3, 29" : "+v"(a##i));
        REP8(X)
#undef X
      } else if constexpr (OP == 15) {
#define X(i) asm volatile("v_mov_b64 %0, %1" : "=v"(c##i) : "v"(c##i));
        REP8(X)
#undef X
      }
    }
  }
  uint32_t s = b0 ^ b1 ^ b2 ^ b3 ^ b4 ^ b5 ^ b6 ^ b7 ^ a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ k;
  s ^= (uint32_t)(c0 ^ c1 ^ c2 ^ c3 ^ c4 ^ c5 ^ c6 ^ c7) ^ (uint32_t)((c0 ^ c7) >> 32);
  s ^= (uint32_t)(sc0 ^ sc1 ^ sc2 ^ sc3 ^ sc4 ^ sc5 ^ sc6 ^ sc7);
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int OP>
float run(int grid, uint32_t* out) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(krate<OP>, dim3(grid), dim3(256), 0, 0, out, 12345u);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0));
  for (int r = 0; r < 5; r++) hipLaunchKernelGGL(krate<OP>, dim3(grid), dim3(256), 0, 0, out, 12345u + r);
  CHECK(hipEventRecord(e1)); CHECK(hipEventSynchronize(e1));
  float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
  return ms / 5;
}

int main() {
  hipDeviceProp_t prop; CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const int grid = cus * 8;  // 8 WG of 4 waves per CU = 8 waves/SIMD
  uint32_t* out; CHECK(hipMalloc(&out, (size_t)grid * 256 * 4));
  const char* names[] = {"v_add_u32", "v_mad_u64_u32", "v_lshrrev_b64", "v_lshl_add_u64", "v_and_b32",
                         "v_mad_i64_i32", "v_alignbit_b32", "v_add_co+v_addc (pair)", "v_cndmask_b32", "v_mul_hi_u32",
                         "v_mul_lo_u32", "v_pk_add_u16", "v_fma_f64", "v_add3_u32", "v_bfe_u32", "v_mov_b64"};
  float t[16];
  t[0] = run<0>(grid, out); t[1] = run<1>(grid, out); t[2] = run<2>(grid, out); t[3] = run<3>(grid, out);
  t[4] = run<4>(grid, out); t[5] = run<5>(grid, out); t[6] = run<6>(grid, out); t[7] = run<7>(grid, out);
  t[8] = run<8>(grid, out); t[9] = run<9>(grid, out); t[10] = run<10>(grid, out); t[11] = run<11>(grid, out);
  t[12] = run<12>(grid, out); t[13] = run<13>(grid, out); t[14] = run<14>(grid, out); t[15] = run<15>(grid, out);
  const double insts = (double)grid * 4 * ITER * 16;  // wave-instructions
  // SIMD-cycles per wave-instruction at the rated clock (gfx950: a SIMD issues a 32-bit VALU
  // wave64 instruction over 2 cycles, MI355X_MICROARCH.md "Wave scheduling")
  const double simd_cycles = (double)cus * 4 * 2.4e9;
  printf("{\"CUs\": %d, \"clock_kHz\": %d, \"rates\": {", cus, prop.clockRate);
  for (int i = 0; i < 16; i++)
    printf("%s\"%s\": {\"ms\": %.4f, \"cycles_per_wave_inst\": %.2f, \"G_wave_inst_per_s\": %.1f}", i ? ", " : "",
           names[i], t[i], simd_cycles * t[i] * 1e-3 / insts, insts / t[i] / 1e6);
  printf("}}\n");
  return 0;
}
