// v_mad_u64_u32 peak issue rate on gfx950, measured in shader clocks (s_memtime) per
// wave so the result does not depend on an assumed clock: 16 independent 64-bit
// accumulators per lane (no dependency stalls), carry-out to vcc (as in the Montgomery
// engine), `waves` waves per SIMD.  Prints cycles per wave-instruction and the chip-wide
// lane-op rate at the measured clock.
//   hipcc --offload-arch=gfx950 -O3 tools/microbench/madpeak.hip -o tools/microbench/madpeak
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define NACC 16
#define INNER 64

__global__ void k_mad(uint64_t* out, uint64_t* cyc, uint32_t s, int iters) {
  uint32_t a = threadIdx.x + s, b = blockIdx.x * 7 + s;
  uint64_t acc[NACC];
#pragma unroll
  for (int c = 0; c < NACC; ++c) acc[c] = c + a;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < INNER / NACC; ++j) {
#pragma unroll
      for (int c = 0; c < NACC; ++c)
        asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc[c]) : "v"(a + c), "v"(b) : "vcc");
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  uint64_t x = 0;
#pragma unroll
  for (int c = 0; c < NACC; ++c) x ^= acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
  if (threadIdx.x % 64 == 0) cyc[(blockIdx.x * blockDim.x + threadIdx.x) / 64] = t1 - t0;
}

int main(int argc, char** argv) {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  const int iters = argc > 1 ? atoi(argv[1]) : 20000;
  for (int waves = 1; waves <= 4; waves *= 2) {
    // one workgroup of 256 threads = one wave per SIMD; `waves` workgroups per CU
    const int blocks = cus * waves, threads = 256;
    uint64_t *d, *c;
    hipMalloc(&d, sizeof(uint64_t) * blocks * threads);
    hipMalloc(&c, sizeof(uint64_t) * blocks * threads / 64);
    hipLaunchKernelGGL(k_mad, dim3(blocks), dim3(threads), 0, 0, d, c, 1u, 100);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_mad, dim3(blocks), dim3(threads), 0, 0, d, c, 1u, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const int nw = blocks * threads / 64;
    uint64_t* h = (uint64_t*)malloc(sizeof(uint64_t) * nw);
    hipMemcpy(h, c, sizeof(uint64_t) * nw, hipMemcpyDeviceToHost);
    double avg = 0;
    for (int i = 0; i < nw; ++i) avg += (double)h[i];
    avg /= nw;
    const double instr = (double)iters * INNER;               // per wave
    const double lane_ops = (double)blocks * threads * instr;  // chip
    // s_memtime ticks at the shader clock; the wall clock gives the effective clock
    printf("{\"waves_per_simd\": %d, \"ms\": %.3f, \"cyc_per_wave_instr\": %.3f, \"clock_GHz\": %.3f, "
           "\"T_lane_mad_s\": %.2f}\n",
           waves, ms, avg / instr, avg / (ms * 1e-3) / 1e9, lane_ops / (ms * 1e-3) / 1e12);
    hipFree(d);
    hipFree(c);
    free(h);
  }
  return 0;
}
