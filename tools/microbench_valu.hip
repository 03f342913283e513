// Microbenchmark of the gfx950 VALU instructions a big-integer Montgomery
// product can be built from.  Measures issue throughput (8 independent chains
// per lane) and dependent latency (1 chain) for each instruction, chip-wide.
// Output: one line per instruction: wave-instructions/cycle/CU and lane-ops/s.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

#define CHECK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP error %s @%d\n",hipGetErrorString(e),__LINE__); exit(1);} }while(0)

#define REP8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

// ---- mad_u64_u32 -----------------------------------------------------------
template<int CH>
__global__ void __launch_bounds__(256) k_mad64(uint64_t* out, uint32_t s, int iters){
  uint64_t acc[8]; uint64_t cc[8]={0}; uint32_t x = threadIdx.x + s, y = threadIdx.x * 3 + s;
  #pragma unroll
  for(int c=0;c<8;c++) acc[c] = c + threadIdx.x;
  for(int it=0; it<iters; it++){
    #pragma unroll
    for(int u=0;u<16;u++){
      #pragma unroll
      for(int c=0;c<CH;c++)
        asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc[c]), "=s"(cc[c]) : "v"(x), "v"(y));
    }
  }
  uint64_t r=0;
  #pragma unroll
  for(int c=0;c<CH;c++) r+=acc[c]+cc[c];
  out[blockIdx.x*blockDim.x+threadIdx.x]=r;
}
// ---- mul_lo_u32 -------------------------------------------------------------
template<int CH>
__global__ void __launch_bounds__(256) k_mullo(uint64_t* out, uint32_t s, int iters){
  uint32_t acc[8]; uint32_t y = threadIdx.x * 3 + s;
  #pragma unroll
  for(int c=0;c<8;c++) acc[c] = c + threadIdx.x;
  for(int it=0; it<iters; it++){
    #pragma unroll
    for(int u=0;u<16;u++){
      #pragma unroll
      for(int c=0;c<CH;c++)
        asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(acc[c]) : "v"(y));
    }
  }
  uint64_t r=0;
  #pragma unroll
  for(int c=0;c<CH;c++) r+=acc[c];
  out[blockIdx.x*blockDim.x+threadIdx.x]=r;
}
template<int CH>
__global__ void __launch_bounds__(256) k_mulhi(uint64_t* out, uint32_t s, int iters){
  uint32_t acc[8]; uint32_t y = threadIdx.x * 3 + s;
  #pragma unroll
  for(int c=0;c<8;c++) acc[c] = c + threadIdx.x;
  for(int it=0; it<iters; it++){
    #pragma unroll
    for(int u=0;u<16;u++){
      #pragma unroll
      for(int c=0;c<CH;c++)
        asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(acc[c]) : "v"(y));
    }
  }
  uint64_t r=0;
  #pragma unroll
  for(int c=0;c<CH;c++) r+=acc[c];
  out[blockIdx.x*blockDim.x+threadIdx.x]=r;
}
// ---- add_co / addc ----------------------------------------------------------
template<int CH>
__global__ void __launch_bounds__(256) k_addc(uint64_t* out, uint32_t s, int iters){
  uint32_t acc[8]; uint64_t cc[8]={0}; uint32_t y = threadIdx.x * 3 + s;
  #pragma unroll
  for(int c=0;c<8;c++) acc[c] = c + threadIdx.x;
  for(int it=0; it<iters; it++){
    #pragma unroll
    for(int u=0;u<16;u++){
      #pragma unroll
      for(int c=0;c<CH;c++)
        asm volatile("v_addc_co_u32 %0, %1, %0, %2, %1" : "+v"(acc[c]), "+s"(cc[c]) : "v"(y));
    }
  }
  uint64_t r=0;
  #pragma unroll
  for(int c=0;c<CH;c++) r+=acc[c];
  out[blockIdx.x*blockDim.x+threadIdx.x]=r;
}
template<int CH>
__global__ void __launch_bounds__(256) k_add32(uint64_t* out, uint32_t s, int iters){
  uint32_t acc[8]; uint32_t y = threadIdx.x * 3 + s;
  #pragma unroll
  for(int c=0;c<8;c++) acc[c] = c + threadIdx.x;
  for(int it=0; it<iters; it++){
    #pragma unroll
    for(int u=0;u<16;u++){
      #pragma unroll
      for(int c=0;c<CH;c++)
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(acc[c]) : "v"(y));
    }
  }
  uint64_t r=0;
  #pragma unroll
  for(int c=0;c<CH;c++) r+=acc[c];
  out[blockIdx.x*blockDim.x+threadIdx.x]=r;
}
// ---- lshl_add_u64 (64-bit add) ----------------------------------------------
template<int CH>
__global__ void __launch_bounds__(256) k_add64(uint64_t* out, uint32_t s, int iters){
  uint64_t acc[8]; uint64_t y = threadIdx.x * 3 + s;
  #pragma unroll
  for(int c=0;c<8;c++) acc[c] = c + threadIdx.x;
  for(int it=0; it<iters; it++){
    #pragma unroll
    for(int u=0;u<16;u++){
      #pragma unroll
      for(int c=0;c<CH;c++)
        asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(acc[c]) : "v"(y));
    }
  }
  uint64_t r=0;
  #pragma unroll
  for(int c=0;c<CH;c++) r+=acc[c];
  out[blockIdx.x*blockDim.x+threadIdx.x]=r;
}
// ---- fma_f64 ----------------------------------------------------------------
template<int CH>
__global__ void __launch_bounds__(256) k_fma64(uint64_t* out, uint32_t s, int iters){
  double acc[8]; double x = 1.0000001 + threadIdx.x*1e-9, y = 0.999999 + s*1e-12;
  #pragma unroll
  for(int c=0;c<8;c++) acc[c] = c + threadIdx.x;
  for(int it=0; it<iters; it++){
    #pragma unroll
    for(int u=0;u<16;u++){
      #pragma unroll
      for(int c=0;c<CH;c++)
        asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(acc[c]) : "v"(x), "v"(y));
    }
  }
  double r=0;
  #pragma unroll
  for(int c=0;c<CH;c++) r+=acc[c];
  out[blockIdx.x*blockDim.x+threadIdx.x]=(uint64_t)r;
}
// ---- mad_u32_u24 / mul_hi_u32_u24 ------------------------------------------
template<int CH>
__global__ void __launch_bounds__(256) k_mad24(uint64_t* out, uint32_t s, int iters){
  uint32_t acc[8]; uint32_t x = threadIdx.x + s, y = threadIdx.x * 3 + s;
  #pragma unroll
  for(int c=0;c<8;c++) acc[c] = c + threadIdx.x;
  for(int it=0; it<iters; it++){
    #pragma unroll
    for(int u=0;u<16;u++){
      #pragma unroll
      for(int c=0;c<CH;c++)
        asm volatile("v_mad_u32_u24 %0, %1, %2, %0" : "+v"(acc[c]) : "v"(x), "v"(y));
    }
  }
  uint64_t r=0;
  #pragma unroll
  for(int c=0;c<CH;c++) r+=acc[c];
  out[blockIdx.x*blockDim.x+threadIdx.x]=r;
}
// ---- v_pk_fma_f32 / v_fma_f32 ------------------------------------------------
template<int CH>
__global__ void __launch_bounds__(256) k_fma32(uint64_t* out, uint32_t s, int iters){
  float acc[8]; float x = 1.0000001f + threadIdx.x*1e-9f, y = 0.999999f + s*1e-12f;
  #pragma unroll
  for(int c=0;c<8;c++) acc[c] = c + threadIdx.x;
  for(int it=0; it<iters; it++){
    #pragma unroll
    for(int u=0;u<16;u++){
      #pragma unroll
      for(int c=0;c<CH;c++)
        asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(acc[c]) : "v"(x), "v"(y));
    }
  }
  float r=0;
  #pragma unroll
  for(int c=0;c<CH;c++) r+=acc[c];
  out[blockIdx.x*blockDim.x+threadIdx.x]=(uint64_t)r;
}

typedef void (*kfn)(uint64_t*, uint32_t, int);

static void run(const char* name, kfn f, int chains, int blocks_per_cu, uint64_t* d){
  int cus = 256; hipDeviceProp_t p; CHECK(hipGetDeviceProperties(&p,0)); cus = p.multiProcessorCount;
  int blocks = cus*blocks_per_cu, iters = 4096;
  hipLaunchKernelGGL(f, dim3(blocks), dim3(256), 0, 0, d, 1u, 16);
  CHECK(hipDeviceSynchronize());
  hipEvent_t a,b; CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
  CHECK(hipEventRecord(a,0));
  hipLaunchKernelGGL(f, dim3(blocks), dim3(256), 0, 0, d, 1u, iters);
  CHECK(hipEventRecord(b,0)); CHECK(hipEventSynchronize(b));
  float ms; CHECK(hipEventElapsedTime(&ms,a,b));
  double wave_instr = (double)blocks*4 /*waves*/ * iters * 16 * chains;
  double lane_ops = wave_instr*64;
  double clk = 2.4e9;
  printf("%-14s chains=%d blk/CU=%d  %.3f ms  lane-ops/s=%.3e  wave-instr/clk/CU(@2.4GHz)=%.3f  cycles/wave-instr/SIMD=%.2f\n",
         name, chains, blocks_per_cu, ms, lane_ops/(ms*1e-3), wave_instr/(ms*1e-3)/clk/cus,
         4.0/(wave_instr/(ms*1e-3)/clk/cus));
}

int main(){
  uint64_t* d; CHECK(hipMalloc(&d, 256*8*256*8*8));
  for(int bpc : {2, 4}){
    run("mad_u64_u32", k_mad64<8>, 8, bpc, d);
    run("mul_lo_u32", k_mullo<8>, 8, bpc, d);
    run("mul_hi_u32", k_mulhi<8>, 8, bpc, d);
    run("addc_co_u32", k_addc<8>, 8, bpc, d);
    run("add_u32", k_add32<8>, 8, bpc, d);
    run("lshl_add_u64", k_add64<8>, 8, bpc, d);
    run("fma_f64", k_fma64<8>, 8, bpc, d);
    run("fma_f32", k_fma32<8>, 8, bpc, d);
    run("mad_u32_u24", k_mad24<8>, 8, bpc, d);
  }
  // latency: one chain, one wave per SIMD
  run("mad_u64 lat", k_mad64<1>, 1, 1, d);
  run("mul_lo lat", k_mullo<1>, 1, 1, d);
  run("addc lat", k_addc<1>, 1, 1, d);
  run("lshl_add64 lat", k_add64<1>, 1, 1, d);
  run("fma_f64 lat", k_fma64<1>, 1, 1, d);
  return 0;
}
