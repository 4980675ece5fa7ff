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
// mode 0: alternate squaring / multiply by bm;  mode 1: squarings only
__global__ void __launch_bounds__(256, 1) k_cpp(uint32_t* io, const uint32_t* bm, MontCtx c, int reps, int mode) {
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
    if ((r & 1) && mode == 0) {  // acc <- acc * b
      lds_store_col(lds, 256, acc);
      col_load(gb, acc);
    } else {      // acc <- acc^2
      lds_store_col(lds, 256, acc);
    }
    mont_mul(acc, lds, 256, c);
  }
  col_store(g, acc);
}

// use_sq: squarings through fbm_sq_lds (else the general product with b == a)
__global__ void __launch_bounds__(256, 2) k_asm(uint32_t* io, const uint32_t* bm, const uint32_t* M, uint32_t mp,
                                                int reps, int mode, int use_sq) {
  __shared__ uint32_t lds_a[(NL + 1) * 256];
  const int tid = threadIdx.x;
  const uint32_t off = (uint32_t)(uintptr_t)((lds_u32*)lds_a + tid);
  uint32_t* g = io + (uint64_t)blockIdx.x * NL * 256 + tid;
  for (int k = 0; k < NL; ++k) lds_a[k * 256 + tid] = g[k * 256];
  const uint32_t boff = (uint32_t)(((uint64_t)blockIdx.x * NL * 256 + tid) * 4);
#pragma unroll 1
  for (int r = 0; r < reps; ++r) {
    if ((r & 1) && mode == 0)
      fbm_mm_glb(off, bm, boff, M, mp);
    else if (use_sq)
      fbm_sq_lds(off, M, mp);
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
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  uint32_t* d3;
  CK(hipMalloc(&d3, words * 4));
  int bad = 0;
  for (int mode = 0; mode < 2; ++mode) {
    float t[3];
    std::vector<uint32_t> r[3];
    uint32_t* dd[3] = {d1, d2, d3};
    for (int v = 0; v < 3; ++v) {
      CK(hipMemcpy(dd[v], h.data(), words * 4, hipMemcpyHostToDevice));
      if (v == 0) hipLaunchKernelGGL(k_cpp, dim3(blocks), dim3(256), 0, 0, dd[v], db, c, 0, mode);
      else hipLaunchKernelGGL(k_asm, dim3(blocks), dim3(256), 0, 0, dd[v], db, dM, c.mp, 0, mode, v == 2);
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0));
      if (v == 0) hipLaunchKernelGGL(k_cpp, dim3(blocks), dim3(256), 0, 0, dd[v], db, c, reps, mode);
      else hipLaunchKernelGGL(k_asm, dim3(blocks), dim3(256), 0, 0, dd[v], db, dM, c.mp, reps, mode, v == 2);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&t[v], e0, e1));
      r[v].resize(words);
      CK(hipMemcpy(r[v].data(), dd[v], words * 4, hipMemcpyDeviceToHost));
    }
    size_t diff1 = 0, diff2 = 0;
    for (size_t i = 0; i < words; ++i) {
      diff1 += r[0][i] != r[1][i];
      diff2 += r[0][i] != r[2][i];
    }
    bad |= (diff1 || diff2);
    const double mm = (double)blocks * 256 * reps;
    printf("{\"mode\": \"%s\", \"blocks\": %d, \"reps\": %d, \"cpp_ms\": %.3f, \"asm_ms\": %.3f, "
           "\"asm_sq_ms\": %.3f, \"cpp_Gprod_s\": %.3f, \"asm_Gprod_s\": %.3f, \"asm_sq_Gprod_s\": %.3f, "
           "\"asm_Tmad_s\": %.2f, \"mismatch_asm\": %zu, \"mismatch_asm_sq\": %zu}\n",
           mode ? "square-only" : "square/multiply", blocks, reps, t[0], t[1], t[2], mm / t[0] / 1e6,
           mm / t[1] / 1e6, mm / t[2] / 1e6, mm * 74 * 148 / t[1] / 1e9, diff1, diff2);
  }
  return bad ? 2 : 0;
}
