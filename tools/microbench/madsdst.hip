// Does the carry-out register limit a wave's v_mad_u64_u32 issue rate?  The N-adic engine
// writes every multiply's (unused) carry-out to vcc; a wave alone issues one every 8.8
// cycles (madpeak.hip) while four waves per SIMD reach 3.2.  Same loop as madpeak.hip
// (16 independent 64-bit accumulators per lane), carry-out to
//   mode 0: vcc for every multiply (as the engine)
//   mode 1: 16 distinct SGPR pairs, one per accumulator
//   mode 2: as mode 1, every other multiply taking its multiplicand from an SGPR (the
//           engine's q*N_k rows read N_k from SGPRs)
// Prints cycles per wave-instruction (s_memtime) per mode and waves per SIMD.
//   hipcc --offload-arch=gfx950 -O3 tools/microbench/madsdst.hip -o tools/microbench/madsdst
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define NACC 16
#define INNER 64
#define CHK(x)                                                              \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));               \
      exit(1);                                                              \
    }                                                                       \
  } while (0)

#define MAD_SS(c, LO, HI)                                                                   \
  asm volatile("v_mad_u64_u32 %0, s[" #LO ":" #HI "], %1, %2, %0" : "+v"(acc[c]) : "v"(a + c), "s"(sb) \
               : "s" #LO, "s" #HI)
#define MAD_S(c, LO, HI)                                                                    \
  asm volatile("v_mad_u64_u32 %0, s[" #LO ":" #HI "], %1, %2, %0" : "+v"(acc[c]) : "v"(a + c), "v"(b) \
               : "s" #LO, "s" #HI)

template <int MODE>
__global__ void k_mad(uint64_t* out, uint64_t* cyc, uint32_t s, int iters) {
  uint32_t a = threadIdx.x + s, b = blockIdx.x * 7 + s;
  const uint32_t sb = __builtin_amdgcn_readfirstlane(b) + 3u;
  uint64_t acc[NACC];
#pragma unroll
  for (int c = 0; c < NACC; ++c) acc[c] = c + a;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < INNER / NACC; ++j) {
      if (MODE == 0) {
#pragma unroll
        for (int c = 0; c < NACC; ++c)
          asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc[c]) : "v"(a + c), "v"(b) : "vcc");
      } else if (MODE == 2) {
        MAD_S(0, 40, 41); MAD_SS(1, 42, 43); MAD_S(2, 44, 45); MAD_SS(3, 46, 47);
        MAD_S(4, 48, 49); MAD_SS(5, 50, 51); MAD_S(6, 52, 53); MAD_SS(7, 54, 55);
        MAD_S(8, 56, 57); MAD_SS(9, 58, 59); MAD_S(10, 60, 61); MAD_SS(11, 62, 63);
        MAD_S(12, 64, 65); MAD_SS(13, 66, 67); MAD_S(14, 68, 69); MAD_SS(15, 70, 71);
      } else {
        MAD_S(0, 40, 41); MAD_S(1, 42, 43); MAD_S(2, 44, 45); MAD_S(3, 46, 47);
        MAD_S(4, 48, 49); MAD_S(5, 50, 51); MAD_S(6, 52, 53); MAD_S(7, 54, 55);
        MAD_S(8, 56, 57); MAD_S(9, 58, 59); MAD_S(10, 60, 61); MAD_S(11, 62, 63);
        MAD_S(12, 64, 65); MAD_S(13, 66, 67); MAD_S(14, 68, 69); MAD_S(15, 70, 71);
      }
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  uint64_t x = 0;
#pragma unroll
  for (int c = 0; c < NACC; ++c) x ^= acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
  if (threadIdx.x % 64 == 0) cyc[(blockIdx.x * blockDim.x + threadIdx.x) / 64] = t1 - t0;
}

template <int MODE>
void run(int cus, int iters) {
  for (int waves = 1; waves <= 4; waves *= 2) {
    const int blocks = cus * waves, threads = 256;
    uint64_t *d, *c;
    CHK(hipMalloc(&d, sizeof(uint64_t) * blocks * threads));
    CHK(hipMalloc(&c, sizeof(uint64_t) * blocks * threads / 64));
    hipLaunchKernelGGL(k_mad<MODE>, dim3(blocks), dim3(threads), 0, 0, d, c, 1u, 100);
    CHK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    CHK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_mad<MODE>, dim3(blocks), dim3(threads), 0, 0, d, c, 1u, iters);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    float ms;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    const int nw = blocks * threads / 64;
    uint64_t* h = (uint64_t*)malloc(sizeof(uint64_t) * nw);
    CHK(hipMemcpy(h, c, sizeof(uint64_t) * nw, hipMemcpyDeviceToHost));
    double avg = 0;
    for (int i = 0; i < nw; ++i) avg += (double)h[i];
    avg /= nw;
    const double instr = (double)iters * INNER;
    const double lane_ops = (double)blocks * threads * instr;
    printf("{\"mode\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.3f, \"cyc_per_wave_instr\": %.3f, "
           "\"clock_GHz\": %.3f, \"T_lane_mad_s\": %.2f}\n",
           MODE == 0 ? "vcc" : MODE == 1 ? "sgpr-pairs" : "sgpr-pairs+sgpr-src", waves, ms, avg / instr, avg / (ms * 1e-3) / 1e9,
           lane_ops / (ms * 1e-3) / 1e12);
    CHK(hipFree(d));
    CHK(hipFree(c));
    CHK(hipEventDestroy(e0));
    CHK(hipEventDestroy(e1));
    free(h);
  }
}

int main(int argc, char** argv) {
  hipDeviceProp_t p;
  CHK(hipGetDeviceProperties(&p, 0));
  const int iters = argc > 1 ? atoi(argv[1]) : 20000;
  run<0>(p.multiProcessorCount, iters);
  run<1>(p.multiProcessorCount, iters);
  run<2>(p.multiProcessorCount, iters);
  return 0;
}
