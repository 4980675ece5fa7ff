// Pricing kernel (round-5 VERDICT item 3): one Montgomery reduction t = (T + m N) / R with the two
// products by the fixed modulus on int8 MFMA, every conversion on the VALU, one lane per ciphertext
// (the one-lane engine's layout), no LDS:
//   T (2088 bits, 72 limbs of 29 bits, as the VALU engine holds a square) -> the 149 low 7-bit digits of
//   T mod R (R = 128^149 = 2^1043 >= 2^19 N) -> m = T N' mod R as v_mfma_i32_32x32x32_i8 against Toeplitz
//   blocks of N' (15 MFMAs per 32 ciphertexts) -> the i32 columns normalised to balanced digits in
//   [-64, 63] by a carry chain (m_bal, the unique balanced representative of T N' mod R) -> m_bal N as 20
//   MFMAs against Toeplitz blocks of N (only the output blocks that reach the high half) -> the carry out
//   of the low half from its top columns, the high columns accumulated into 29-bit limbs, + (T >> 1043)
//   + N (so t = (T + (m_bal + R) N) / R > 0) -> t normalised to 37 limbs.
// The MFMA operands need each ciphertext's digits in two lanes (B: lane l = ciphertext l & 31, k-half
// l >> 5) and give each ciphertext's output columns in two lanes (C: rows by lane half): one
// v_permlane32_swap per register moves them between that layout and the one-lane layout.
// Every iteration feeds t back as T = t + H 2^1044 (H a per-ciphertext constant < 2^1021), so a launch
// runs `iters` dependent reductions in registers; tools/microbench/mfma_redc_check.py builds the inputs
// and constants, replays the chain with Python integers and checks every output limb.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 mfma_redc.hip -o mfma_redc
// Run:   ./mfma_redc <in.bin> <out.bin> <iters> <reps>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

constexpr int ND = 149;      // 7-bit digits of R = 2^1043
constexpr int NL = 36;       // 29-bit limbs of T's low part / of t
constexpr uint32_t M29 = (1u << 29) - 1;

// (new vdst, new vsrc) of v_permlane32_swap: lanes 32-63 of vdst <-> lanes 0-31 of vsrc
__device__ __forceinline__ void pswap(uint32_t& x, uint32_t& y) {
  auto r = __builtin_amdgcn_permlane32_swap(x, y, false, false);
  x = r[0];
  y = r[1];
}

// 28 bits of the limb array starting at bit 28 w, spread into four bytes of 7 bits
template <int W>
__device__ __forceinline__ uint32_t digits4(const uint32_t* tl) {
  constexpr int b = 28 * W, L = b / 29, o = b % 29;
  constexpr int need = (W == 37) ? 7 : 28;  // digit 148 alone in the last word
  uint32_t x = tl[L] >> o;
  if constexpr (o + need > 29) x |= tl[L + 1] << (29 - o);
  x &= (W == 37) ? 0x7Fu : 0x0FFFFFFFu;  // digit 148 is the last below R
  x = x + (x & 0xFFFFFF80u);               // digits 1..3 up by one bit
  x = x + (x & 0xFFFF8000u);               // digits 2..3 up by one more
  x = x + (x & 0xFF800000u);               // digit 3 up by one more
  return x;
}

template <int W>
__device__ __forceinline__ void all_digits(const uint32_t* tl, uint32_t* tw) {
  if constexpr (W < 38) {
    tw[W] = digits4<W>(tl);
    all_digits<W + 1>(tl, tw);
  }
}

__global__ void __launch_bounds__(256, 2) redc_kernel(const uint32_t* __restrict__ Tin, const uint32_t* __restrict__ Hin,
                                                   const v4i* __restrict__ Anp, const v4i* __restrict__ An,
                                                   const uint32_t* __restrict__ Nl, uint32_t* __restrict__ out,
                                                   uint32_t n, int iters) {
  const uint32_t ct = blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63;
  // the Toeplitz blocks' A fragments (N' offsets 0..4, N offsets 0..5) in LDS: one ds_read_b128 per MFMA
  // pair instead of 44 resident VGPRs
  __shared__ v4i sA[11][64];
  for (int e = threadIdx.x; e < 11 * 64; e += blockDim.x) sA[e / 64][e % 64] = e < 5 * 64 ? Anp[e] : An[e - 5 * 64];
  __syncthreads();
  uint32_t tl[NL];
#pragma unroll
  for (int L = 0; L < NL; ++L) tl[L] = Tin[(size_t)L * n + ct];
  uint32_t top = 0;
  for (int it = 0; it < iters; ++it) {
    // ---- T mod R -> digits; fragments for both 32-ciphertext groups ----
    uint32_t tw[40];
    all_digits<0>(tl, tw);
    tw[38] = tw[39] = 0;
#pragma unroll
    for (int kb = 0; kb < 5; ++kb)
#pragma unroll
      for (int q = 0; q < 4; ++q) pswap(tw[8 * kb + q], tw[8 * kb + 4 + q]);
    // (tw[8kb + 0..3] = group 0's B fragment of K-block kb, tw[8kb + 4..7] = group 1's)
    const double tfrac = (double)(tl[35] & 0x0FFFFFFFu) * 0x1p-28 + (double)tl[34] * 0x1p-57 +
                         (double)tl[33] * 0x1p-86;
    const uint32_t tbit = (tl[35] >> 28) + (top << 1);  // T >> 1043 below 2^1044 (t's own top limb)

    // ---- m = T N' mod R, balanced digits ----
    uint32_t mw[40];
    int32_t c = 0;
#pragma unroll
    for (int mb = 0; mb < 5; ++mb) {
      v16i a0 = {0}, a1 = {0};
#pragma unroll
      for (int kb = 0; kb <= mb; ++kb) {
        const v4i b0 = {(int)tw[8 * kb], (int)tw[8 * kb + 1], (int)tw[8 * kb + 2], (int)tw[8 * kb + 3]};
        const v4i b1 = {(int)tw[8 * kb + 4], (int)tw[8 * kb + 5], (int)tw[8 * kb + 6], (int)tw[8 * kb + 7]};
        const v4i A = sA[mb - kb][lane];
        a0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(A, b0, a0, 0, 0, 0);
        a1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(A, b1, a1, 0, 0, 0);
      }
      uint32_t X[16], Y[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        X[r] = (uint32_t)a0[r];
        Y[r] = (uint32_t)a1[r];
        pswap(X[r], Y[r]);  // X: this lane's ciphertext, rows of half 0; Y: rows of half 1
      }
#pragma unroll
      for (int rho = 0; rho < 32; ++rho) {
        const int i = 32 * mb + rho;
        if (i < ND) {
          const int reg = (rho & 3) + 4 * (rho >> 3);
          const int32_t col = (int32_t)((rho & 4) ? Y[reg] : X[reg]);
          const int32_t tt = col + c + 64;
          c = tt >> 7;
          const uint32_t d = (uint32_t)((tt & 127) - 64) & 0xFFu;
          if ((i & 3) == 0)
            mw[i >> 2] = d;
          else
            mw[i >> 2] |= d << (8 * (i & 3));
        }
      }
    }
    mw[37] &= 0xFFu;  // digit 148 is the last
    mw[38] = mw[39] = 0;
#pragma unroll
    for (int kb = 0; kb < 5; ++kb)
#pragma unroll
      for (int q = 0; q < 4; ++q) pswap(mw[8 * kb + q], mw[8 * kb + 4 + q]);

    // ---- P = m_bal N: the blocks reaching column 141 and up ----
    int64_t acc[NL];
#pragma unroll
    for (int L = 0; L < NL; ++L) acc[L] = (int64_t)Nl[L] + 2 * (int64_t)Hin[(size_t)L * n + ct];
    double est = tfrac;
#pragma unroll
    for (int mb = 4; mb < 10; ++mb) {
      v16i a0 = {0}, a1 = {0};
#pragma unroll
      for (int kb = 0; kb < 5; ++kb) {
        const int d = mb - kb;
        if (d < 0 || d > 5) continue;
        const v4i b0 = {(int)mw[8 * kb], (int)mw[8 * kb + 1], (int)mw[8 * kb + 2], (int)mw[8 * kb + 3]};
        const v4i b1 = {(int)mw[8 * kb + 4], (int)mw[8 * kb + 5], (int)mw[8 * kb + 6], (int)mw[8 * kb + 7]};
        const v4i A = sA[5 + d][lane];
        a0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(A, b0, a0, 0, 0, 0);
        a1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(A, b1, a1, 0, 0, 0);
      }
      uint32_t X[16], Y[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        X[r] = (uint32_t)a0[r];
        Y[r] = (uint32_t)a1[r];
        pswap(X[r], Y[r]);
      }
#pragma unroll
      for (int rho = 0; rho < 32; ++rho) {
        const int j = 32 * mb + rho;
        const int reg = (rho & 3) + 4 * (rho >> 3);
        const int32_t col = (int32_t)((rho & 4) ? Y[reg] : X[reg]);
        if (j >= 141 && j < ND) est += (double)col * __builtin_ldexp(1.0, 7 * (j - ND));
        if (j >= ND && j < 296) {
          const int bit = 7 * (j - ND), Lt = bit / 29, s = bit % 29;
          acc[Lt] += (int64_t)col * (int64_t)(1ll << s);
        }
      }
    }
    acc[0] += (int64_t)__builtin_rint(est) + (int64_t)tbit;
    // ---- normalise: t = 36 limbs + top ----
    int64_t cy = 0;
#pragma unroll
    for (int L = 0; L < NL; ++L) {
      const int64_t v = acc[L] + cy;
      tl[L] = (uint32_t)v & M29;
      cy = v >> 29;
    }
    top = (uint32_t)cy;
  }
#pragma unroll
  for (int L = 0; L < NL; ++L) out[(size_t)L * n + ct] = tl[L];
  out[(size_t)NL * n + ct] = top;
}

__global__ void swap_probe(uint32_t* o) {
  uint32_t x = threadIdx.x, y = 100 + threadIdx.x;
  pswap(x, y);
  o[threadIdx.x] = x;
  o[64 + threadIdx.x] = y;
}

int main(int argc, char** argv) {
  if (argc < 5) {
    fprintf(stderr, "usage: mfma_redc in.bin out.bin iters reps\n");
    return 1;
  }
  const int iters = atoi(argv[3]), reps = atoi(argv[4]);
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 1;
  uint32_t n;
  if (fread(&n, 4, 1, f) != 1) return 1;
  if (n % 256) {
    fprintf(stderr, "n must be a multiple of 256\n");
    return 1;
  }
  std::vector<uint32_t> T((size_t)NL * n), H((size_t)NL * n), Nl(NL);
  std::vector<v4i> Anp(5 * 64), An(6 * 64);
  size_t got = fread(T.data(), 4, T.size(), f) + fread(H.data(), 4, H.size(), f) + fread(Nl.data(), 4, NL, f) +
               fread(Anp.data(), 16, Anp.size(), f) + fread(An.data(), 16, An.size(), f);
  fclose(f);
  if (got != T.size() + H.size() + NL + Anp.size() + An.size()) {
    fprintf(stderr, "short input\n");
    return 1;
  }
  uint32_t *dT, *dH, *dN, *dO, *dP;
  v4i *dAnp, *dAn;
  CK(hipMalloc(&dT, T.size() * 4));
  CK(hipMalloc(&dH, H.size() * 4));
  CK(hipMalloc(&dN, NL * 4));
  CK(hipMalloc(&dO, (size_t)(NL + 1) * n * 4));
  CK(hipMalloc(&dAnp, Anp.size() * 16));
  CK(hipMalloc(&dAn, An.size() * 16));
  CK(hipMalloc(&dP, 128 * 4));
  CK(hipMemcpy(dT, T.data(), T.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dH, H.data(), H.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dN, Nl.data(), NL * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dAnp, Anp.data(), Anp.size() * 16, hipMemcpyHostToDevice));
  CK(hipMemcpy(dAn, An.data(), An.size() * 16, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(swap_probe, dim3(1), dim3(64), 0, 0, dP);
  uint32_t probe[128];
  CK(hipMemcpy(probe, dP, 512, hipMemcpyDeviceToHost));
  printf("{\"permlane32_swap\": {\"x_lane0\": %u, \"x_lane32\": %u, \"y_lane0\": %u, \"y_lane32\": %u}}\n", probe[0],
         probe[32], probe[64], probe[96]);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<float> ts;
  for (int r = 0; r <= reps; ++r) {
    CK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(redc_kernel, dim3(n / 256), dim3(256), 0, 0, dT, dH, dAnp, dAn, dN, dO, n, iters);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (r) ts.push_back(ms);
  }
  CK(hipGetLastError());
  std::sort(ts.begin(), ts.end());
  std::vector<uint32_t> O((size_t)(NL + 1) * n);
  CK(hipMemcpy(O.data(), dO, O.size() * 4, hipMemcpyDeviceToHost));
  FILE* g = fopen(argv[2], "wb");
  fwrite(O.data(), 4, O.size(), g);
  fclose(g);
  printf("{\"n_ct\": %u, \"iters\": %d, \"ms_median\": %.4f, \"ms_min\": %.4f, \"us_per_redc_per_131072_ct\": %.4f}\n", n,
         iters, ts[ts.size() / 2], ts[0], 1000.0 * ts[ts.size() / 2] / iters / (n / 131072.0));
  return 0;
}
