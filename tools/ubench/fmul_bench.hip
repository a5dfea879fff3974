// Field-multiply throughput: 8x32-bit CIOS (compiler) vs 9x29-bit lazy Montgomery (R=2^261).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define CHECK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP error %s at %d\n",hipGetErrorString(e),__LINE__); exit(1);}}while(0)
constexpr int ITER = 256;
__device__ __forceinline__ uint64_t mad(uint32_t a, uint32_t b, uint64_t c){ return (uint64_t)a*b + c; }

__device__ __forceinline__ void mul32(const uint32_t* a, const uint32_t* b, uint32_t* o) {
  const uint32_t P[8]={0x1,0xa118000,0xd0000001,0x59aa76fe,0x5c37b001,0x60b44d1e,0x9a2ca556,0x12ab655e};
  uint32_t t[9];
  #pragma unroll
  for(int j=0;j<9;j++) t[j]=0;
  #pragma unroll
  for(int ii=0;ii<8;ii++){
    uint64_t c=0;
    #pragma unroll
    for(int j=0;j<8;j++){ uint64_t s=mad(a[ii],b[j],(uint64_t)t[j]+c); t[j]=(uint32_t)s; c=s>>32; }
    uint32_t t8 = t[8] + (uint32_t)c;
    uint32_t m = -t[0];
    c = (t[0]!=0);
    #pragma unroll
    for(int j=1;j<8;j++){ uint64_t s=mad(m,P[j],(uint64_t)t[j]+c); t[j-1]=(uint32_t)s; c=s>>32; }
    uint64_t s = (uint64_t)t8 + c; t[7]=(uint32_t)s; t[8]=(uint32_t)(s>>32);
  }
  #pragma unroll
  for(int j=0;j<8;j++) o[j]=t[j];
}

__device__ __forceinline__ void mul29(const uint32_t* a, const uint32_t* b, uint32_t* o) {
  const uint32_t P[9]={1u, 277610496u, 66u, 351141280u, 452990362u, 110046747u, 358187729u, 198395284u, 1223525u};
  const uint32_t MASK = (1u<<29)-1;
  uint64_t c[18];
  #pragma unroll
  for(int k=0;k<18;k++) c[k]=0;
  #pragma unroll
  for(int i=0;i<9;i++)
    #pragma unroll
    for(int j=0;j<9;j++) c[i+j]=mad(a[i],b[j],c[i+j]);
  #pragma unroll
  for(int i=0;i<9;i++){
    uint32_t m = (0u - (uint32_t)c[i]) & MASK;
    c[i] += m;
    c[i+1] += c[i] >> 29;
    #pragma unroll
    for(int j=1;j<9;j++) c[i+j]=mad(m,P[j],c[i+j]);
  }
  #pragma unroll
  for(int k=9;k<17;k++){ c[k+1] += c[k]>>29; o[k-9]=(uint32_t)c[k] & MASK; }
  o[8]=(uint32_t)c[17];
}

template<int V>
__global__ void kbench(const uint32_t* in, uint32_t* out) {
  int tid = blockIdx.x*blockDim.x+threadIdx.x;
  constexpr int L = (V==0)?8:9;
  uint32_t x[L], y[L], z[L];
  #pragma unroll
  for(int j=0;j<L;j++){ x[j]=in[(tid*L+j)&1023] & 0x0fffffff; y[j]=in[(tid*L+j+7)&1023]&0x0fffffff; z[j]=x[j]^y[j];}
  for(int it=0; it<ITER; it++){
    // two independent chains for ILP
    if constexpr (V==0){ mul32(x,y,x); mul32(z,y,z);} else { mul29(x,y,x); mul29(z,y,z);}  
  }
  uint32_t s=0;
  #pragma unroll
  for(int j=0;j<L;j++) s+=x[j]^z[j];
  out[tid]=s;
}

int main(){
  hipDeviceProp_t prop; CHECK(hipGetDeviceProperties(&prop, 0));
  int cus = prop.multiProcessorCount;
  uint32_t *in, *out; CHECK(hipMalloc(&in, 4096)); CHECK(hipMalloc(&out, 64<<20));
  uint32_t h[1024]; for(int i=0;i<1024;i++) h[i]=i*2654435761u; CHECK(hipMemcpy(in,h,4096,hipMemcpyHostToDevice));
  hipEvent_t e0,e1; CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  for(int wps: {1,2,4,8}){
    int block=256, grid=cus*wps;
    for(int v=0; v<2; v++){
      auto f = v==0 ? kbench<0> : kbench<1>;
      hipLaunchKernelGGL(f, dim3(grid), dim3(block), 0, 0, in, out); CHECK(hipDeviceSynchronize());
      CHECK(hipEventRecord(e0));
      for(int r=0;r<3;r++) hipLaunchKernelGGL(f, dim3(grid), dim3(block), 0, 0, in, out);
      CHECK(hipEventRecord(e1)); CHECK(hipEventSynchronize(e1));
      float ms; CHECK(hipEventElapsedTime(&ms,e0,e1)); ms/=3;
      double muls = (double)grid*block*ITER*2;
      printf("waves/SIMD %d %s: %.3f ms  %.2f Gmul/s  (%.0f cycles per wave-mul per SIMD)\n", wps, v==0?"mont32-CIOS":"mont29-lazy", ms, muls/ms/1e6,
        (ms*1e-3*2.4e9) / (muls/64.0 / (cus*4)));
    }
  }
  return 0;
}
