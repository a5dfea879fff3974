// Does VGPR bank placement set the issue rate of v_mad_u64_u32 on gfx950?  (Tuning probe for
// DESIGN.md §8 item 1; not part of the product.)  Each kernel runs ITER x 8 independent
// multiply-adds per lane on explicitly named registers (VGPR bank = register index mod 4):
//   mode 0: accumulators v[16:17].. (banks 0,1), factors in banks 2 and 3   -> no two operands share a bank
//   mode 1: accumulators in banks 0,1, both factors in bank 2               -> factor/factor conflict
//   mode 2: accumulators in banks 2,3 (v[18:19]..), factors in banks 2, 3  -> factor/accumulator conflicts
//   mode 3: mode 0 with v_mad_i64_i32
// Prints cycles per wave64 instruction at the nominal clock, like isa_rates.hip.
//   hipcc -O2 --offload-arch=gfx950 -o mad_banks mad_banks.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
constexpr int ITER = 4096;

#define CLOB "v2", "v3", "v6", "v7", "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23", "v24", "v25", \
             "v26", "v27", "v28", "v29", "v30", "v31", "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", \
             "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "s20", "s21"

template <int MODE>
__global__ void __launch_bounds__(256) kmad(uint32_t* out, uint32_t seed) {
  uint32_t x = threadIdx.x ^ seed;
  asm volatile(
      "v_mov_b32 v2, %0\n v_add_u32 v3, 7, %0\n v_add_u32 v6, 9, %0\n v_mov_b32 v7, 11\n"
      "v_mov_b32 v16, %0\n v_mov_b32 v17, 0\n v_mov_b32 v18, %0\n v_mov_b32 v19, 0\n"
      "v_mov_b32 v20, %0\n v_mov_b32 v21, 0\n v_mov_b32 v22, %0\n v_mov_b32 v23, 0\n"
      "v_mov_b32 v24, %0\n v_mov_b32 v25, 0\n v_mov_b32 v26, %0\n v_mov_b32 v27, 0\n"
      "v_mov_b32 v28, %0\n v_mov_b32 v29, 0\n v_mov_b32 v30, %0\n v_mov_b32 v31, 0\n"
      "v_mov_b32 v32, %0\n v_mov_b32 v33, 0\n v_mov_b32 v34, %0\n v_mov_b32 v35, 0\n"
      "v_mov_b32 v36, %0\n v_mov_b32 v37, 0\n v_mov_b32 v38, %0\n v_mov_b32 v39, 0\n"
      "v_mov_b32 v40, %0\n v_mov_b32 v41, 0\n v_mov_b32 v42, %0\n v_mov_b32 v43, 0\n"
      "v_mov_b32 v44, %0\n v_mov_b32 v45, 0\n v_mov_b32 v46, %0\n v_mov_b32 v47, 0\n"
      :
      : "v"(x)
      : CLOB);
  for (int it = 0; it < ITER; it++) {
    if constexpr (MODE == 0) {  // acc banks {0,1}; factors v2 (bank 2), v3 (bank 3)
      asm volatile(
          "v_mad_u64_u32 v[16:17], s[20:21], v2, v3, v[16:17]\n v_mad_u64_u32 v[20:21], s[20:21], v2, v3, v[20:21]\n"
          "v_mad_u64_u32 v[24:25], s[20:21], v2, v3, v[24:25]\n v_mad_u64_u32 v[28:29], s[20:21], v2, v3, v[28:29]\n"
          "v_mad_u64_u32 v[32:33], s[20:21], v2, v3, v[32:33]\n v_mad_u64_u32 v[36:37], s[20:21], v2, v3, v[36:37]\n"
          "v_mad_u64_u32 v[40:41], s[20:21], v2, v3, v[40:41]\n v_mad_u64_u32 v[44:45], s[20:21], v2, v3, v[44:45]\n" ::
              : CLOB);
    } else if constexpr (MODE == 1) {  // both factors in bank 2 (v2, v6)
      asm volatile(
          "v_mad_u64_u32 v[16:17], s[20:21], v2, v6, v[16:17]\n v_mad_u64_u32 v[20:21], s[20:21], v2, v6, v[20:21]\n"
          "v_mad_u64_u32 v[24:25], s[20:21], v2, v6, v[24:25]\n v_mad_u64_u32 v[28:29], s[20:21], v2, v6, v[28:29]\n"
          "v_mad_u64_u32 v[32:33], s[20:21], v2, v6, v[32:33]\n v_mad_u64_u32 v[36:37], s[20:21], v2, v6, v[36:37]\n"
          "v_mad_u64_u32 v[40:41], s[20:21], v2, v6, v[40:41]\n v_mad_u64_u32 v[44:45], s[20:21], v2, v6, v[44:45]\n" ::
              : CLOB);
    } else if constexpr (MODE == 2) {  // accumulators in banks {2,3}: v[18:19].. with factors v2, v3
      asm volatile(
          "v_mad_u64_u32 v[18:19], s[20:21], v2, v3, v[18:19]\n v_mad_u64_u32 v[22:23], s[20:21], v2, v3, v[22:23]\n"
          "v_mad_u64_u32 v[26:27], s[20:21], v2, v3, v[26:27]\n v_mad_u64_u32 v[30:31], s[20:21], v2, v3, v[30:31]\n"
          "v_mad_u64_u32 v[34:35], s[20:21], v2, v3, v[34:35]\n v_mad_u64_u32 v[38:39], s[20:21], v2, v3, v[38:39]\n"
          "v_mad_u64_u32 v[42:43], s[20:21], v2, v3, v[42:43]\n v_mad_u64_u32 v[46:47], s[20:21], v2, v3, v[46:47]\n" ::
              : CLOB);
    } else {  // mode 0 placement, signed multiply
      asm volatile(
          "v_mad_i64_i32 v[16:17], s[20:21], v2, v3, v[16:17]\n v_mad_i64_i32 v[20:21], s[20:21], v2, v3, v[20:21]\n"
          "v_mad_i64_i32 v[24:25], s[20:21], v2, v3, v[24:25]\n v_mad_i64_i32 v[28:29], s[20:21], v2, v3, v[28:29]\n"
          "v_mad_i64_i32 v[32:33], s[20:21], v2, v3, v[32:33]\n v_mad_i64_i32 v[36:37], s[20:21], v2, v3, v[36:37]\n"
          "v_mad_i64_i32 v[40:41], s[20:21], v2, v3, v[40:41]\n v_mad_i64_i32 v[44:45], s[20:21], v2, v3, v[44:45]\n" ::
              : CLOB);
    }
  }
  uint32_t r;
  asm volatile(
      "v_xor_b32 %0, v16, v18\n v_xor_b32 %0, %0, v20\n v_xor_b32 %0, %0, v22\n v_xor_b32 %0, %0, v24\n"
      "v_xor_b32 %0, %0, v26\n v_xor_b32 %0, %0, v28\n v_xor_b32 %0, %0, v30\n v_xor_b32 %0, %0, v32\n"
      "v_xor_b32 %0, %0, v34\n v_xor_b32 %0, %0, v36\n v_xor_b32 %0, %0, v38\n v_xor_b32 %0, %0, v40\n"
      "v_xor_b32 %0, %0, v42\n v_xor_b32 %0, %0, v44\n v_xor_b32 %0, %0, v46\n"
      : "=v"(r)::CLOB);
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <int MODE>
float run(uint32_t* d, int blocks) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  hipLaunchKernelGGL(kmad<MODE>, dim3(blocks), dim3(256), 0, 0, d, 1u);  // warm-up
  CHECK(hipEventRecord(a));
  hipLaunchKernelGGL(kmad<MODE>, dim3(blocks), dim3(256), 0, 0, d, 2u);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms;
  CHECK(hipEventElapsedTime(&ms, a, b));
  return ms;
}

int main() {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  const int blocks = cus * 8;  // 8 workgroups of 4 waves per CU = 8 waves per SIMD
  uint32_t* d;
  CHECK(hipMalloc(&d, (size_t)blocks * 256 * 4));
  const double wave_inst = (double)blocks * 4 * ITER * 8;  // wave64 instructions
  const double simds = cus * 4.0, clk = 2.4e9;
  const char* names[] = {"u64 acc{0,1} f{2,3}", "u64 acc{0,1} f{2,2}", "u64 acc{2,3} f{2,3}", "i64 acc{0,1} f{2,3}"};
  float ms[4] = {run<0>(d, blocks), run<1>(d, blocks), run<2>(d, blocks), run<3>(d, blocks)};
  printf("{");
  for (int m = 0; m < 4; m++)
    printf("%s\"%s\": {\"ms\": %.4f, \"cycles_per_wave_inst\": %.2f}", m ? ", " : "", names[m], ms[m],
           ms[m] * 1e-3 * clk * simds / wave_inst);
  printf("}\n");
  hipFree(d);
  return 0;
}
