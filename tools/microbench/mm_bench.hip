// Montgomery-product microbenchmark: assembly engine (fbm_mont_asm.hpp) vs the C++
// mont_mul<74> (fbm_mont.hpp).  Both compute the identical lazy product, so the results of
// a chain of squarings / multiplies must agree bit for bit; the timing shows the
// instruction-cache effect of the 90 KB unrolled C++ product.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/microbench/mm_bench.hip -o tools/microbench/mm_bench
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <random>
#include <vector>

#include "../../fedbiomed_amd/csrc/fbm_mont.hpp"
#include "../../fedbiomed_amd/csrc/fbm_mont_asm.hpp"

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

typedef __attribute__((address_space(3))) uint32_t lds_u32;
constexpr int NL = FBM_NL;

// io: blocked columns [block][limb][256]; b: same layout (multiplier for odd steps)
__global__ void __launch_bounds__(256, 1) k_cpp(uint32_t* io, const uint32_t* bm, MontCtx c, int reps) {
  __shared__ uint32_t lds_a[NL * 256];
  const int tid = threadIdx.x;
  uint32_t* g = io + (uint64_t)blockIdx.x * NL * 256 + tid;
  const uint32_t* gb = bm + (uint64_t)blockIdx.x * NL * 256 + tid;
  uint32_t* lds = lds_a + tid;
  uint32_t acc[NL];
  col_load(g, acc);
#pragma unroll 1
  for (int r = 0; r < reps; ++r) {
    r = __builtin_amdgcn_readfirstlane(r);
    asm volatile("" : "+s"(r));
    if (r & 1) {  // acc <- acc * b
      lds_store_col(lds, 256, acc);
      col_load(gb, acc);
    } else {      // acc <- acc^2
      lds_store_col(lds, 256, acc);
    }
    mont_mul(acc, lds, 256, c);
  }
  col_store(g, acc);
}

__global__ void __launch_bounds__(256, 2) k_asm(uint32_t* io, const uint32_t* bm, const uint32_t* M, uint32_t mp,
                                                int reps) {
  __shared__ uint32_t lds_a[(NL + 1) * 256];
  const int tid = threadIdx.x;
  const uint32_t off = (uint32_t)(uintptr_t)((lds_u32*)lds_a + tid);
  uint32_t* g = io + (uint64_t)blockIdx.x * NL * 256 + tid;
  for (int k = 0; k < NL; ++k) lds_a[k * 256 + tid] = g[k * 256];
  const uint32_t boff = (uint32_t)(((uint64_t)blockIdx.x * NL * 256 + tid) * 4);
#pragma unroll 1
  for (int r = 0; r < reps; ++r) {
    if (r & 1)
      fbm_mm_glb(off, bm, boff, M, mp);
    else
      fbm_mm_lds(off, off, M, mp);
  }
  asm volatile("" : "+v"(g));
  for (int k = 0; k < NL; ++k) g[k * 256] = lds_a[k * 256 + tid];
}

int main(int argc, char** argv) {
  const int blocks = argc > 1 ? atoi(argv[1]) : 512;
  const int reps = argc > 2 ? atoi(argv[2]) : 64;
  std::mt19937_64 rng(12345);
  // random odd 2046-bit modulus M in 28-bit limbs
  MontCtx c;
  memset(&c, 0, sizeof(c));
  for (int k = 0; k < NL; ++k) c.M[k] = (uint32_t)rng() & FBM_LMASK;
  c.M[0] |= 1u;
  c.M[NL - 1] = 0u;
  c.M[NL - 2] = (c.M[NL - 2] & 0x3FFFFu) | 0x20000u;  // top at bit 2044-ish
  // mp = -M^{-1} mod 2^28 (Newton)
  uint32_t inv = 1;
  for (int i = 0; i < 5; ++i) inv = inv * (2u - c.M[0] * inv);
  c.mp = (0u - inv) & FBM_LMASK;
  const size_t words = (size_t)blocks * NL * 256;
  std::vector<uint32_t> h(words), hb(words);
  for (size_t i = 0; i < words; ++i) {
    const int k = (int)((i / 256) % NL);
    const bool top = k >= NL - 2;
    h[i] = top ? 0u : ((uint32_t)rng() & FBM_LMASK);
    hb[i] = top ? 0u : ((uint32_t)rng() & FBM_LMASK);
  }
  uint32_t *d1, *d2, *db, *dM;
  CK(hipMalloc(&d1, words * 4));
  CK(hipMalloc(&d2, words * 4));
  CK(hipMalloc(&db, words * 4));
  CK(hipMalloc(&dM, 128 * 4));
  std::vector<uint32_t> Mw(128, 0);
  memcpy(Mw.data(), c.M, sizeof(c.M));
  CK(hipMemcpy(dM, Mw.data(), 128 * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d1, h.data(), words * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d2, h.data(), words * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(db, hb.data(), words * 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1, e2;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventCreate(&e2));
  // warm-up launches (one rep) then the timed ones
  hipLaunchKernelGGL(k_cpp, dim3(blocks), dim3(256), 0, 0, d1, db, c, 0);
  hipLaunchKernelGGL(k_asm, dim3(blocks), dim3(256), 0, 0, d2, db, dM, c.mp, 0);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  hipLaunchKernelGGL(k_cpp, dim3(blocks), dim3(256), 0, 0, d1, db, c, reps);
  CK(hipEventRecord(e1));
  hipLaunchKernelGGL(k_asm, dim3(blocks), dim3(256), 0, 0, d2, db, dM, c.mp, reps);
  CK(hipEventRecord(e2));
  CK(hipDeviceSynchronize());
  float t_cpp = 0, t_asm = 0;
  CK(hipEventElapsedTime(&t_cpp, e0, e1));
  CK(hipEventElapsedTime(&t_asm, e1, e2));
  std::vector<uint32_t> r1(words), r2(words);
  CK(hipMemcpy(r1.data(), d1, words * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(r2.data(), d2, words * 4, hipMemcpyDeviceToHost));
  size_t diff = 0, first = (size_t)-1;
  for (size_t i = 0; i < words; ++i)
    if (r1[i] != r2[i]) {
      if (first == (size_t)-1) first = i;
      ++diff;
    }
  const double mm = (double)blocks * 256 * reps;
  const double mads = mm * 74 * 148;
  printf("{\"blocks\": %d, \"reps\": %d, \"cpp_ms\": %.3f, \"asm_ms\": %.3f, \"cpp_Mmontmul_s\": %.1f, "
         "\"asm_Mmontmul_s\": %.1f, \"asm_Tmad_s\": %.2f, \"mismatch_words\": %zu, \"first_mismatch\": %lld}\n",
         blocks, reps, t_cpp, t_asm, mm / t_cpp / 1e3, mm / t_asm / 1e3, mads / t_asm / 1e9, diff,
         (long long)(first == (size_t)-1 ? -1 : (long long)first));
  return diff ? 2 : 0;
}
