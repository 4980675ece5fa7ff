// Checks the lane maps of v_mfma_i32_32x32x32_i8 on gfx950 with exact integer data (asymmetric A and B):
//   A: lane l holds A[row l&31][k = kmap(l>>5, j)], j = 0..15 (16 int8 in 4 VGPRs)
//   B: lane l holds B[k = kmap(l>>5, j)][col l&31]
//   C: lane l, register r holds C[row (r&3) + 8(r>>2) + 4(l>>5)][col l&31]
// for two candidate k maps (16h + j, and two K=16 halves 8h + j / 16 + 8h + j - 8).  Prints one line each.
// Build: hipcc --offload-arch=gfx950 -O3 mfma_i8_map.hip -o mfma_i8_map
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

__device__ __host__ inline int kmap(int variant, int h, int j) {
  return variant == 0 ? 16 * h + j : (j < 8 ? 8 * h + j : 16 + 8 * h + (j - 8));
}

__global__ void probe(const int8_t* A, const int8_t* B, int* C, int variant) {
  const int l = threadIdx.x, r = l & 31, h = l >> 5;
  int8_t a[16], b[16];
  for (int j = 0; j < 16; ++j) {
    a[j] = A[r * 32 + kmap(variant, h, j)];
    b[j] = B[kmap(variant, h, j) * 32 + r];
  }
  v4i av, bv;
  __builtin_memcpy(&av, a, 16);
  __builtin_memcpy(&bv, b, 16);
  v16i c = {0};
  c = __builtin_amdgcn_mfma_i32_32x32x32_i8(av, bv, c, 0, 0, 0);
  for (int reg = 0; reg < 16; ++reg) C[((reg & 3) + 8 * (reg >> 2) + 4 * h) * 32 + r] = c[reg];
}

int main() {
  int8_t hA[1024], hB[1024];
  int ref[1024], hC[1024];
  srand(12345);
  for (int i = 0; i < 1024; ++i) {
    hA[i] = (int8_t)(rand() % 256 - 128);
    hB[i] = (int8_t)((rand() % 251) - 120);
  }
  for (int i = 0; i < 32; ++i)
    for (int j = 0; j < 32; ++j) {
      int s = 0;
      for (int k = 0; k < 32; ++k) s += (int)hA[i * 32 + k] * (int)hB[k * 32 + j];
      ref[i * 32 + j] = s;
    }
  int8_t *dA, *dB;
  int* dC;
  hipMalloc(&dA, 1024);
  hipMalloc(&dB, 1024);
  hipMalloc(&dC, 4096);
  hipMemcpy(dA, hA, 1024, hipMemcpyHostToDevice);
  hipMemcpy(dB, hB, 1024, hipMemcpyHostToDevice);
  for (int v = 0; v < 2; ++v) {
    hipMemset(dC, 0, 4096);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dA, dB, dC, v);
    hipMemcpy(hC, dC, 4096, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 1024; ++i) bad += hC[i] != ref[i];
    printf("{\"kmap\": \"%s\", \"mismatches\": %d, \"C00\": %d, \"ref00\": %d}\n",
           v == 0 ? "16h+j" : "8h+j|16+8h+j-8", bad, hC[0], ref[0]);
  }
  return 0;
}
