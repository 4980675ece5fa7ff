// Integer / FP64 VALU issue-rate microbenchmark for the JL Montgomery engine design
// (which multiply primitive should carry the 2048-bit modmul on gfx950?).
// Each kernel runs 8 independent dependency chains per lane, ITER iterations; the
// host reports per-instruction throughput in Gop/s (lane-ops) for the whole chip.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define ITER 4096
#define CH 8

__global__ void k_mad64(uint64_t* out, uint32_t s) {
  uint32_t a = threadIdx.x + s, b = blockIdx.x * 7 + s;
  uint64_t acc[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = c + a;
  for (int i = 0; i < ITER; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      uint64_t r, cc;
      asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(r), "=s"(cc) : "v"(a + c), "v"(b), "v"(acc[c]));
      acc[c] = r;
    }
  }
  uint64_t x = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) x ^= acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

__global__ void k_mullo(uint64_t* out, uint32_t s) {
  uint32_t a = threadIdx.x + s, b = blockIdx.x * 7 + s;
  uint32_t acc[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = c + a;
  for (int i = 0; i < ITER; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      uint32_t r;
      asm volatile("v_mul_lo_u32 %0, %1, %2" : "=v"(r) : "v"(acc[c]), "v"(b));
      acc[c] = r;
    }
  }
  uint64_t x = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) x ^= acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

__global__ void k_mulhi(uint64_t* out, uint32_t s) {
  uint32_t a = threadIdx.x + s, b = blockIdx.x * 7 + s;
  uint32_t acc[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = c + a;
  for (int i = 0; i < ITER; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      uint32_t r;
      asm volatile("v_mul_hi_u32 %0, %1, %2" : "=v"(r) : "v"(acc[c]), "v"(b));
      acc[c] = r;
    }
  }
  uint64_t x = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) x ^= acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

__global__ void k_addc(uint64_t* out, uint32_t s) {
  uint32_t a = threadIdx.x + s;
  uint32_t acc[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = c + a;
  for (int i = 0; i < ITER; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      uint32_t r;
      asm volatile("v_add_co_u32 %0, vcc, %1, %2" : "=v"(r) : "v"(acc[c]), "v"(a) : "vcc");
      acc[c] = r;
    }
  }
  uint64_t x = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) x ^= acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

__global__ void k_add3(uint64_t* out, uint32_t s) {
  uint32_t a = threadIdx.x + s;
  uint32_t acc[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = c + a;
  for (int i = 0; i < ITER; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      uint32_t r;
      asm volatile("v_add3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(acc[c]), "v"(a), "v"(s));
      acc[c] = r;
    }
  }
  uint64_t x = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) x ^= acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

__global__ void k_fma64(uint64_t* out, uint32_t s) {
  double a = threadIdx.x * 1e-3 + s, b = 0.999999;
  double acc[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = c + a;
  for (int i = 0; i < ITER; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      double r;
      asm volatile("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(acc[c]), "v"(b), "v"(a));
      acc[c] = r;
    }
  }
  double x = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) x += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)x;
}

__global__ void k_mul24(uint64_t* out, uint32_t s) {
  uint32_t a = threadIdx.x + s, b = blockIdx.x * 7 + s;
  uint32_t acc[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = c + a;
  for (int i = 0; i < ITER; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      uint32_t r;
      asm volatile("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(r) : "v"(acc[c]), "v"(b), "v"(a));
      acc[c] = r;
    }
  }
  uint64_t x = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) x ^= acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

#define K32(NAME, ASM)                                                                  \
  __global__ void NAME(uint64_t* out, uint32_t s) {                                     \
    uint32_t a = threadIdx.x + s;                                                       \
    uint32_t acc[CH];                                                                   \
    _Pragma("unroll") for (int c = 0; c < CH; ++c) acc[c] = c + a;                      \
    for (int i = 0; i < ITER; ++i) {                                                    \
      _Pragma("unroll") for (int c = 0; c < CH; ++c) {                                  \
        uint32_t r;                                                                     \
        asm volatile(ASM : "=v"(r) : "v"(acc[c]), "v"(a));                              \
        acc[c] = r;                                                                     \
      }                                                                                 \
    }                                                                                   \
    uint64_t x = 0;                                                                     \
    _Pragma("unroll") for (int c = 0; c < CH; ++c) x ^= acc[c];                         \
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;                                     \
  }
K32(k_add32, "v_add_u32 %0, %1, %2")
K32(k_xor32, "v_xor_b32 %0, %1, %2")
K32(k_align, "v_alignbit_b32 %0, %1, %1, 16")
K32(k_perm, "v_perm_b32 %0, %1, %1, %2")
K32(k_lshlor, "v_lshl_or_b32 %0, %1, 7, %2")
K32(k_xad, "v_xad_u32 %0, %1, %2, %1")
K32(k_bfi, "v_pk_add_u16 %0, %1, %2")

// 64-bit shift / shift-add (the carry retire of the Montgomery rows)
#define K64(NAME, ASM)                                                                  \
  __global__ void NAME(uint64_t* out, uint32_t s) {                                     \
    uint64_t a = threadIdx.x + s;                                                       \
    uint64_t acc[CH];                                                                   \
    _Pragma("unroll") for (int c = 0; c < CH; ++c) acc[c] = c + a;                      \
    for (int i = 0; i < ITER; ++i) {                                                    \
      _Pragma("unroll") for (int c = 0; c < CH; ++c) {                                  \
        uint64_t r;                                                                     \
        asm volatile(ASM : "=v"(r) : "v"(acc[c]), "v"(a));                              \
        acc[c] = r;                                                                     \
      }                                                                                 \
    }                                                                                   \
    uint64_t x = 0;                                                                     \
    _Pragma("unroll") for (int c = 0; c < CH; ++c) x ^= acc[c];                         \
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;                                     \
  }
K64(k_lshr64, "v_lshrrev_b64 %0, 28, %1")
K64(k_lshladd64, "v_lshl_add_u64 %0, %1, 0, %2")

// ChaCha20 double-rounds as the LOM kernel runs them (ITER/64 blocks per lane); ops counted
// as 976 per block (the kernel's add/xor/rotate count).
#include "../../fedbiomed_amd/csrc/fbm_common.hpp"
#define CHACHA_BLOCKS (ITER / 16)
__global__ void k_chacha(uint64_t* out, uint32_t s) {
  uint32_t key[8];
  for (int w = 0; w < 8; ++w) key[w] = threadIdx.x * 31u + w + s;
  uint32_t x = 0;
  for (int b = 0; b < CHACHA_BLOCKS; ++b) {
    uint32_t ks[16];
    fbm_chacha20_block(key, (uint64_t)blockIdx.x * 1000 + b, s, x, ks);
    for (int w = 0; w < 16; ++w) x ^= ks[w];
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

// SDWA form of a VOP2 op (is it issued at the VOP2 rate?  measured: no, 4.2 cycles)
K32(k_xorsdwa, "v_xor_b32_sdwa %0, %1, %2 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0")

// (The grouped-issue ChaCha20 rounds -- the four quarter-rounds side by side as groups of four
// independent same-type instructions -- measured 3.58 cycles per op against 4.05 for the
// compiler's schedule, with an identical keystream; they now live in fbm_common.hpp, which
// k_chacha above uses.)

#define DR_NOP0 \
  "v_add_u32 %0, %0, %4\n" \
  "v_add_u32 %1, %1, %5\n" \
  "v_add_u32 %2, %2, %6\n" \
  "v_add_u32 %3, %3, %7\n" \
  "s_nop 0\n" \
  "v_xor_b32 %12, %12, %0\n" \
  "v_xor_b32 %13, %13, %1\n" \
  "v_xor_b32 %14, %14, %2\n" \
  "v_xor_b32 %15, %15, %3\n" \
  "s_nop 0\n" \
  "v_alignbit_b32 %12, %12, %12, 16\n" \
  "v_alignbit_b32 %13, %13, %13, 16\n" \
  "v_alignbit_b32 %14, %14, %14, 16\n" \
  "v_alignbit_b32 %15, %15, %15, 16\n" \
  "s_nop 0\n" \
  "v_add_u32 %8, %8, %12\n" \
  "v_add_u32 %9, %9, %13\n" \
  "v_add_u32 %10, %10, %14\n" \
  "v_add_u32 %11, %11, %15\n" \
  "s_nop 0\n" \
  "v_xor_b32 %4, %4, %8\n" \
  "v_xor_b32 %5, %5, %9\n" \
  "v_xor_b32 %6, %6, %10\n" \
  "v_xor_b32 %7, %7, %11\n" \
  "s_nop 0\n" \
  "v_alignbit_b32 %4, %4, %4, 20\n" \
  "v_alignbit_b32 %5, %5, %5, 20\n" \
  "v_alignbit_b32 %6, %6, %6, 20\n" \
  "v_alignbit_b32 %7, %7, %7, 20\n" \
  "s_nop 0\n" \
  "v_add_u32 %0, %0, %4\n" \
  "v_add_u32 %1, %1, %5\n" \
  "v_add_u32 %2, %2, %6\n" \
  "v_add_u32 %3, %3, %7\n" \
  "s_nop 0\n" \
  "v_xor_b32 %12, %12, %0\n" \
  "v_xor_b32 %13, %13, %1\n" \
  "v_xor_b32 %14, %14, %2\n" \
  "v_xor_b32 %15, %15, %3\n" \
  "s_nop 0\n" \
  "v_alignbit_b32 %12, %12, %12, 24\n" \
  "v_alignbit_b32 %13, %13, %13, 24\n" \
  "v_alignbit_b32 %14, %14, %14, 24\n" \
  "v_alignbit_b32 %15, %15, %15, 24\n" \
  "s_nop 0\n" \
  "v_add_u32 %8, %8, %12\n" \
  "v_add_u32 %9, %9, %13\n" \
  "v_add_u32 %10, %10, %14\n" \
  "v_add_u32 %11, %11, %15\n" \
  "s_nop 0\n" \
  "v_xor_b32 %4, %4, %8\n" \
  "v_xor_b32 %5, %5, %9\n" \
  "v_xor_b32 %6, %6, %10\n" \
  "v_xor_b32 %7, %7, %11\n" \
  "s_nop 0\n" \
  "v_alignbit_b32 %4, %4, %4, 25\n" \
  "v_alignbit_b32 %5, %5, %5, 25\n" \
  "v_alignbit_b32 %6, %6, %6, 25\n" \
  "v_alignbit_b32 %7, %7, %7, 25\n" \
  "s_nop 0\n" \
  "v_add_u32 %0, %0, %5\n" \
  "v_add_u32 %1, %1, %6\n" \
  "v_add_u32 %2, %2, %7\n" \
  "v_add_u32 %3, %3, %4\n" \
  "s_nop 0\n" \
  "v_xor_b32 %15, %15, %0\n" \
  "v_xor_b32 %12, %12, %1\n" \
  "v_xor_b32 %13, %13, %2\n" \
  "v_xor_b32 %14, %14, %3\n" \
  "s_nop 0\n" \
  "v_alignbit_b32 %15, %15, %15, 16\n" \
  "v_alignbit_b32 %12, %12, %12, 16\n" \
  "v_alignbit_b32 %13, %13, %13, 16\n" \
  "v_alignbit_b32 %14, %14, %14, 16\n" \
  "s_nop 0\n" \
  "v_add_u32 %10, %10, %15\n" \
  "v_add_u32 %11, %11, %12\n" \
  "v_add_u32 %8, %8, %13\n" \
  "v_add_u32 %9, %9, %14\n" \
  "s_nop 0\n" \
  "v_xor_b32 %5, %5, %10\n" \
  "v_xor_b32 %6, %6, %11\n" \
  "v_xor_b32 %7, %7, %8\n" \
  "v_xor_b32 %4, %4, %9\n" \
  "s_nop 0\n" \
  "v_alignbit_b32 %5, %5, %5, 20\n" \
  "v_alignbit_b32 %6, %6, %6, 20\n" \
  "v_alignbit_b32 %7, %7, %7, 20\n" \
  "v_alignbit_b32 %4, %4, %4, 20\n" \
  "s_nop 0\n" \
  "v_add_u32 %0, %0, %5\n" \
  "v_add_u32 %1, %1, %6\n" \
  "v_add_u32 %2, %2, %7\n" \
  "v_add_u32 %3, %3, %4\n" \
  "s_nop 0\n" \
  "v_xor_b32 %15, %15, %0\n" \
  "v_xor_b32 %12, %12, %1\n" \
  "v_xor_b32 %13, %13, %2\n" \
  "v_xor_b32 %14, %14, %3\n" \
  "s_nop 0\n" \
  "v_alignbit_b32 %15, %15, %15, 24\n" \
  "v_alignbit_b32 %12, %12, %12, 24\n" \
  "v_alignbit_b32 %13, %13, %13, 24\n" \
  "v_alignbit_b32 %14, %14, %14, 24\n" \
  "s_nop 0\n" \
  "v_add_u32 %10, %10, %15\n" \
  "v_add_u32 %11, %11, %12\n" \
  "v_add_u32 %8, %8, %13\n" \
  "v_add_u32 %9, %9, %14\n" \
  "s_nop 0\n" \
  "v_xor_b32 %5, %5, %10\n" \
  "v_xor_b32 %6, %6, %11\n" \
  "v_xor_b32 %7, %7, %8\n" \
  "v_xor_b32 %4, %4, %9\n" \
  "s_nop 0\n" \
  "v_alignbit_b32 %5, %5, %5, 25\n" \
  "v_alignbit_b32 %6, %6, %6, 25\n" \
  "v_alignbit_b32 %7, %7, %7, 25\n" \
  "v_alignbit_b32 %4, %4, %4, 25\n" \
  "s_nop 0\n"

#define DR_NOP1 \
  "v_add_u32 %0, %0, %4\n" \
  "v_add_u32 %1, %1, %5\n" \
  "v_add_u32 %2, %2, %6\n" \
  "v_add_u32 %3, %3, %7\n" \
  "s_nop 1\n" \
  "v_xor_b32 %12, %12, %0\n" \
  "v_xor_b32 %13, %13, %1\n" \
  "v_xor_b32 %14, %14, %2\n" \
  "v_xor_b32 %15, %15, %3\n" \
  "s_nop 1\n" \
  "v_alignbit_b32 %12, %12, %12, 16\n" \
  "v_alignbit_b32 %13, %13, %13, 16\n" \
  "v_alignbit_b32 %14, %14, %14, 16\n" \
  "v_alignbit_b32 %15, %15, %15, 16\n" \
  "s_nop 1\n" \
  "v_add_u32 %8, %8, %12\n" \
  "v_add_u32 %9, %9, %13\n" \
  "v_add_u32 %10, %10, %14\n" \
  "v_add_u32 %11, %11, %15\n" \
  "s_nop 1\n" \
  "v_xor_b32 %4, %4, %8\n" \
  "v_xor_b32 %5, %5, %9\n" \
  "v_xor_b32 %6, %6, %10\n" \
  "v_xor_b32 %7, %7, %11\n" \
  "s_nop 1\n" \
  "v_alignbit_b32 %4, %4, %4, 20\n" \
  "v_alignbit_b32 %5, %5, %5, 20\n" \
  "v_alignbit_b32 %6, %6, %6, 20\n" \
  "v_alignbit_b32 %7, %7, %7, 20\n" \
  "s_nop 1\n" \
  "v_add_u32 %0, %0, %4\n" \
  "v_add_u32 %1, %1, %5\n" \
  "v_add_u32 %2, %2, %6\n" \
  "v_add_u32 %3, %3, %7\n" \
  "s_nop 1\n" \
  "v_xor_b32 %12, %12, %0\n" \
  "v_xor_b32 %13, %13, %1\n" \
  "v_xor_b32 %14, %14, %2\n" \
  "v_xor_b32 %15, %15, %3\n" \
  "s_nop 1\n" \
  "v_alignbit_b32 %12, %12, %12, 24\n" \
  "v_alignbit_b32 %13, %13, %13, 24\n" \
  "v_alignbit_b32 %14, %14, %14, 24\n" \
  "v_alignbit_b32 %15, %15, %15, 24\n" \
  "s_nop 1\n" \
  "v_add_u32 %8, %8, %12\n" \
  "v_add_u32 %9, %9, %13\n" \
  "v_add_u32 %10, %10, %14\n" \
  "v_add_u32 %11, %11, %15\n" \
  "s_nop 1\n" \
  "v_xor_b32 %4, %4, %8\n" \
  "v_xor_b32 %5, %5, %9\n" \
  "v_xor_b32 %6, %6, %10\n" \
  "v_xor_b32 %7, %7, %11\n" \
  "s_nop 1\n" \
  "v_alignbit_b32 %4, %4, %4, 25\n" \
  "v_alignbit_b32 %5, %5, %5, 25\n" \
  "v_alignbit_b32 %6, %6, %6, 25\n" \
  "v_alignbit_b32 %7, %7, %7, 25\n" \
  "s_nop 1\n" \
  "v_add_u32 %0, %0, %5\n" \
  "v_add_u32 %1, %1, %6\n" \
  "v_add_u32 %2, %2, %7\n" \
  "v_add_u32 %3, %3, %4\n" \
  "s_nop 1\n" \
  "v_xor_b32 %15, %15, %0\n" \
  "v_xor_b32 %12, %12, %1\n" \
  "v_xor_b32 %13, %13, %2\n" \
  "v_xor_b32 %14, %14, %3\n" \
  "s_nop 1\n" \
  "v_alignbit_b32 %15, %15, %15, 16\n" \
  "v_alignbit_b32 %12, %12, %12, 16\n" \
  "v_alignbit_b32 %13, %13, %13, 16\n" \
  "v_alignbit_b32 %14, %14, %14, 16\n" \
  "s_nop 1\n" \
  "v_add_u32 %10, %10, %15\n" \
  "v_add_u32 %11, %11, %12\n" \
  "v_add_u32 %8, %8, %13\n" \
  "v_add_u32 %9, %9, %14\n" \
  "s_nop 1\n" \
  "v_xor_b32 %5, %5, %10\n" \
  "v_xor_b32 %6, %6, %11\n" \
  "v_xor_b32 %7, %7, %8\n" \
  "v_xor_b32 %4, %4, %9\n" \
  "s_nop 1\n" \
  "v_alignbit_b32 %5, %5, %5, 20\n" \
  "v_alignbit_b32 %6, %6, %6, 20\n" \
  "v_alignbit_b32 %7, %7, %7, 20\n" \
  "v_alignbit_b32 %4, %4, %4, 20\n" \
  "s_nop 1\n" \
  "v_add_u32 %0, %0, %5\n" \
  "v_add_u32 %1, %1, %6\n" \
  "v_add_u32 %2, %2, %7\n" \
  "v_add_u32 %3, %3, %4\n" \
  "s_nop 1\n" \
  "v_xor_b32 %15, %15, %0\n" \
  "v_xor_b32 %12, %12, %1\n" \
  "v_xor_b32 %13, %13, %2\n" \
  "v_xor_b32 %14, %14, %3\n" \
  "s_nop 1\n" \
  "v_alignbit_b32 %15, %15, %15, 24\n" \
  "v_alignbit_b32 %12, %12, %12, 24\n" \
  "v_alignbit_b32 %13, %13, %13, 24\n" \
  "v_alignbit_b32 %14, %14, %14, 24\n" \
  "s_nop 1\n" \
  "v_add_u32 %10, %10, %15\n" \
  "v_add_u32 %11, %11, %12\n" \
  "v_add_u32 %8, %8, %13\n" \
  "v_add_u32 %9, %9, %14\n" \
  "s_nop 1\n" \
  "v_xor_b32 %5, %5, %10\n" \
  "v_xor_b32 %6, %6, %11\n" \
  "v_xor_b32 %7, %7, %8\n" \
  "v_xor_b32 %4, %4, %9\n" \
  "s_nop 1\n" \
  "v_alignbit_b32 %5, %5, %5, 25\n" \
  "v_alignbit_b32 %6, %6, %6, 25\n" \
  "v_alignbit_b32 %7, %7, %7, 25\n" \
  "v_alignbit_b32 %4, %4, %4, 25\n" \
  "s_nop 1\n"

#define DR_SETPRIO \
  "v_add_u32 %0, %0, %4\n" \
  "v_add_u32 %1, %1, %5\n" \
  "v_add_u32 %2, %2, %6\n" \
  "v_add_u32 %3, %3, %7\n" \
  "v_xor_b32 %12, %12, %0\n" \
  "v_xor_b32 %13, %13, %1\n" \
  "v_xor_b32 %14, %14, %2\n" \
  "v_xor_b32 %15, %15, %3\n" \
  "v_alignbit_b32 %12, %12, %12, 16\n" \
  "v_alignbit_b32 %13, %13, %13, 16\n" \
  "v_alignbit_b32 %14, %14, %14, 16\n" \
  "v_alignbit_b32 %15, %15, %15, 16\n" \
  "v_add_u32 %8, %8, %12\n" \
  "v_add_u32 %9, %9, %13\n" \
  "v_add_u32 %10, %10, %14\n" \
  "v_add_u32 %11, %11, %15\n" \
  "v_xor_b32 %4, %4, %8\n" \
  "v_xor_b32 %5, %5, %9\n" \
  "v_xor_b32 %6, %6, %10\n" \
  "v_xor_b32 %7, %7, %11\n" \
  "v_alignbit_b32 %4, %4, %4, 20\n" \
  "v_alignbit_b32 %5, %5, %5, 20\n" \
  "v_alignbit_b32 %6, %6, %6, 20\n" \
  "v_alignbit_b32 %7, %7, %7, 20\n" \
  "v_add_u32 %0, %0, %4\n" \
  "v_add_u32 %1, %1, %5\n" \
  "v_add_u32 %2, %2, %6\n" \
  "v_add_u32 %3, %3, %7\n" \
  "v_xor_b32 %12, %12, %0\n" \
  "v_xor_b32 %13, %13, %1\n" \
  "v_xor_b32 %14, %14, %2\n" \
  "v_xor_b32 %15, %15, %3\n" \
  "v_alignbit_b32 %12, %12, %12, 24\n" \
  "v_alignbit_b32 %13, %13, %13, 24\n" \
  "v_alignbit_b32 %14, %14, %14, 24\n" \
  "v_alignbit_b32 %15, %15, %15, 24\n" \
  "v_add_u32 %8, %8, %12\n" \
  "v_add_u32 %9, %9, %13\n" \
  "v_add_u32 %10, %10, %14\n" \
  "v_add_u32 %11, %11, %15\n" \
  "v_xor_b32 %4, %4, %8\n" \
  "v_xor_b32 %5, %5, %9\n" \
  "v_xor_b32 %6, %6, %10\n" \
  "v_xor_b32 %7, %7, %11\n" \
  "v_alignbit_b32 %4, %4, %4, 25\n" \
  "v_alignbit_b32 %5, %5, %5, 25\n" \
  "v_alignbit_b32 %6, %6, %6, 25\n" \
  "v_alignbit_b32 %7, %7, %7, 25\n" \
  "v_add_u32 %0, %0, %5\n" \
  "v_add_u32 %1, %1, %6\n" \
  "v_add_u32 %2, %2, %7\n" \
  "v_add_u32 %3, %3, %4\n" \
  "v_xor_b32 %15, %15, %0\n" \
  "v_xor_b32 %12, %12, %1\n" \
  "v_xor_b32 %13, %13, %2\n" \
  "v_xor_b32 %14, %14, %3\n" \
  "v_alignbit_b32 %15, %15, %15, 16\n" \
  "v_alignbit_b32 %12, %12, %12, 16\n" \
  "v_alignbit_b32 %13, %13, %13, 16\n" \
  "v_alignbit_b32 %14, %14, %14, 16\n" \
  "v_add_u32 %10, %10, %15\n" \
  "v_add_u32 %11, %11, %12\n" \
  "v_add_u32 %8, %8, %13\n" \
  "v_add_u32 %9, %9, %14\n" \
  "v_xor_b32 %5, %5, %10\n" \
  "v_xor_b32 %6, %6, %11\n" \
  "v_xor_b32 %7, %7, %8\n" \
  "v_xor_b32 %4, %4, %9\n" \
  "v_alignbit_b32 %5, %5, %5, 20\n" \
  "v_alignbit_b32 %6, %6, %6, 20\n" \
  "v_alignbit_b32 %7, %7, %7, 20\n" \
  "v_alignbit_b32 %4, %4, %4, 20\n" \
  "v_add_u32 %0, %0, %5\n" \
  "v_add_u32 %1, %1, %6\n" \
  "v_add_u32 %2, %2, %7\n" \
  "v_add_u32 %3, %3, %4\n" \
  "v_xor_b32 %15, %15, %0\n" \
  "v_xor_b32 %12, %12, %1\n" \
  "v_xor_b32 %13, %13, %2\n" \
  "v_xor_b32 %14, %14, %3\n" \
  "v_alignbit_b32 %15, %15, %15, 24\n" \
  "v_alignbit_b32 %12, %12, %12, 24\n" \
  "v_alignbit_b32 %13, %13, %13, 24\n" \
  "v_alignbit_b32 %14, %14, %14, 24\n" \
  "v_add_u32 %10, %10, %15\n" \
  "v_add_u32 %11, %11, %12\n" \
  "v_add_u32 %8, %8, %13\n" \
  "v_add_u32 %9, %9, %14\n" \
  "v_xor_b32 %5, %5, %10\n" \
  "v_xor_b32 %6, %6, %11\n" \
  "v_xor_b32 %7, %7, %8\n" \
  "v_xor_b32 %4, %4, %9\n" \
  "v_alignbit_b32 %5, %5, %5, 25\n" \
  "v_alignbit_b32 %6, %6, %6, 25\n" \
  "v_alignbit_b32 %7, %7, %7, 25\n" \
  "v_alignbit_b32 %4, %4, %4, 25\n"

#define DR(STR, x)                                                                               \
  asm volatile(STR : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]),      \
               "+v"(x[6]), "+v"(x[7]), "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]),            \
               "+v"(x[12]), "+v"(x[13]), "+v"(x[14]), "+v"(x[15]))
#define CHACHA_VARIANT(KNAME, STR)                                                               \
  __global__ void KNAME(uint64_t* out, uint32_t s) {                                             \
    uint32_t key[8];                                                                             \
    for (int w = 0; w < 8; ++w) key[w] = threadIdx.x * 31u + w + s;                              \
    uint32_t acc = 0;                                                                            \
    for (int b = 0; b < CHACHA_BLOCKS; ++b) {                                                    \
      uint64_t ctr = (uint64_t)blockIdx.x * 1000 + b;                                            \
      uint32_t x[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u, key[0], key[1],       \
                        key[2], key[3], key[4], key[5], key[6], key[7], (uint32_t)ctr,           \
                        (uint32_t)(ctr >> 32), s, acc};                                          \
      _Pragma("unroll") for (int r = 0; r < 10; ++r) DR(STR, x);                                 \
      uint32_t ks[16] = {x[0] + 0x61707865u, x[1] + 0x3320646eu, x[2] + 0x79622d32u,             \
                         x[3] + 0x6b206574u, x[4] + key[0], x[5] + key[1], x[6] + key[2],        \
                         x[7] + key[3], x[8] + key[4], x[9] + key[5], x[10] + key[6],            \
                         x[11] + key[7], x[12] + (uint32_t)ctr, x[13] + (uint32_t)(ctr >> 32),   \
                         x[14] + s, x[15] + acc};                                                \
      for (int w = 0; w < 16; ++w) acc ^= ks[w];                                                 \
    }                                                                                            \
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;                                            \
  }
#define DR_PAIR \
  "v_add_u32 %0, %0, %4\n" \
  "v_add_u32 %1, %1, %5\n" \
  "s_nop 0\n" \
  "v_add_u32 %2, %2, %6\n" \
  "v_add_u32 %3, %3, %7\n" \
  "s_nop 0\n" \
  "v_xor_b32 %12, %12, %0\n" \
  "v_xor_b32 %13, %13, %1\n" \
  "s_nop 0\n" \
  "v_xor_b32 %14, %14, %2\n" \
  "v_xor_b32 %15, %15, %3\n" \
  "s_nop 0\n" \
  "v_alignbit_b32 %12, %12, %12, 16\n" \
  "v_alignbit_b32 %13, %13, %13, 16\n" \
  "s_nop 0\n" \
  "v_alignbit_b32 %14, %14, %14, 16\n" \
  "v_alignbit_b32 %15, %15, %15, 16\n" \
  "s_nop 0\n" \
  "v_add_u32 %8, %8, %12\n" \
  "v_add_u32 %9, %9, %13\n" \
  "s_nop 0\n" \
  "v_add_u32 %10, %10, %14\n" \
  "v_add_u32 %11, %11, %15\n" \
  "s_nop 0\n" \
  "v_xor_b32 %4, %4, %8\n" \
  "v_xor_b32 %5, %5, %9\n" \
  "s_nop 0\n" \
  "v_xor_b32 %6, %6, %10\n" \
  "v_xor_b32 %7, %7, %11\n" \
  "s_nop 0\n" \
  "v_alignbit_b32 %4, %4, %4, 20\n" \
  "v_alignbit_b32 %5, %5, %5, 20\n" \
  "s_nop 0\n" \
  "v_alignbit_b32 %6, %6, %6, 20\n" \
  "v_alignbit_b32 %7, %7, %7, 20\n" \
  "s_nop 0\n" \
  "v_add_u32 %0, %0, %4\n" \
  "v_add_u32 %1, %1, %5\n" \
  "s_nop 0\n" \
  "v_add_u32 %2, %2, %6\n" \
  "v_add_u32 %3, %3, %7\n" \
  "s_nop 0\n" \
  "v_xor_b32 %12, %12, %0\n" \
  "v_xor_b32 %13, %13, %1\n" \
  "s_nop 0\n" \
  "v_xor_b32 %14, %14, %2\n" \
  "v_xor_b32 %15, %15, %3\n" \
  "s_nop 0\n" \
  "v_alignbit_b32 %12, %12, %12, 24\n" \
  "v_alignbit_b32 %13, %13, %13, 24\n" \
  "s_nop 0\n" \
  "v_alignbit_b32 %14, %14, %14, 24\n" \
  "v_alignbit_b32 %15, %15, %15, 24\n" \
  "s_nop 0\n" \
  "v_add_u32 %8, %8, %12\n" \
  "v_add_u32 %9, %9, %13\n" \
  "s_nop 0\n" \
  "v_add_u32 %10, %10, %14\n" \
  "v_add_u32 %11, %11, %15\n" \
  "s_nop 0\n" \
  "v_xor_b32 %4, %4, %8\n" \
  "v_xor_b32 %5, %5, %9\n" \
  "s_nop 0\n" \
  "v_xor_b32 %6, %6, %10\n" \
  "v_xor_b32 %7, %7, %11\n" \
  "s_nop 0\n" \
  "v_alignbit_b32 %4, %4, %4, 25\n" \
  "v_alignbit_b32 %5, %5, %5, 25\n" \
  "s_nop 0\n" \
  "v_alignbit_b32 %6, %6, %6, 25\n" \
  "v_alignbit_b32 %7, %7, %7, 25\n" \
  "s_nop 0\n" \
  "v_add_u32 %0, %0, %5\n" \
  "v_add_u32 %1, %1, %6\n" \
  "s_nop 0\n" \
  "v_add_u32 %2, %2, %7\n" \
  "v_add_u32 %3, %3, %4\n" \
  "s_nop 0\n" \
  "v_xor_b32 %15, %15, %0\n" \
  "v_xor_b32 %12, %12, %1\n" \
  "s_nop 0\n" \
  "v_xor_b32 %13, %13, %2\n" \
  "v_xor_b32 %14, %14, %3\n" \
  "s_nop 0\n" \
  "v_alignbit_b32 %15, %15, %15, 16\n" \
  "v_alignbit_b32 %12, %12, %12, 16\n" \
  "s_nop 0\n" \
  "v_alignbit_b32 %13, %13, %13, 16\n" \
  "v_alignbit_b32 %14, %14, %14, 16\n" \
  "s_nop 0\n" \
  "v_add_u32 %10, %10, %15\n" \
  "v_add_u32 %11, %11, %12\n" \
  "s_nop 0\n" \
  "v_add_u32 %8, %8, %13\n" \
  "v_add_u32 %9, %9, %14\n" \
  "s_nop 0\n" \
  "v_xor_b32 %5, %5, %10\n" \
  "v_xor_b32 %6, %6, %11\n" \
  "s_nop 0\n" \
  "v_xor_b32 %7, %7, %8\n" \
  "v_xor_b32 %4, %4, %9\n" \
  "s_nop 0\n" \
  "v_alignbit_b32 %5, %5, %5, 20\n" \
  "v_alignbit_b32 %6, %6, %6, 20\n" \
  "s_nop 0\n" \
  "v_alignbit_b32 %7, %7, %7, 20\n" \
  "v_alignbit_b32 %4, %4, %4, 20\n" \
  "s_nop 0\n" \
  "v_add_u32 %0, %0, %5\n" \
  "v_add_u32 %1, %1, %6\n" \
  "s_nop 0\n" \
  "v_add_u32 %2, %2, %7\n" \
  "v_add_u32 %3, %3, %4\n" \
  "s_nop 0\n" \
  "v_xor_b32 %15, %15, %0\n" \
  "v_xor_b32 %12, %12, %1\n" \
  "s_nop 0\n" \
  "v_xor_b32 %13, %13, %2\n" \
  "v_xor_b32 %14, %14, %3\n" \
  "s_nop 0\n" \
  "v_alignbit_b32 %15, %15, %15, 24\n" \
  "v_alignbit_b32 %12, %12, %12, 24\n" \
  "s_nop 0\n" \
  "v_alignbit_b32 %13, %13, %13, 24\n" \
  "v_alignbit_b32 %14, %14, %14, 24\n" \
  "s_nop 0\n" \
  "v_add_u32 %10, %10, %15\n" \
  "v_add_u32 %11, %11, %12\n" \
  "s_nop 0\n" \
  "v_add_u32 %8, %8, %13\n" \
  "v_add_u32 %9, %9, %14\n" \
  "s_nop 0\n" \
  "v_xor_b32 %5, %5, %10\n" \
  "v_xor_b32 %6, %6, %11\n" \
  "s_nop 0\n" \
  "v_xor_b32 %7, %7, %8\n" \
  "v_xor_b32 %4, %4, %9\n" \
  "s_nop 0\n" \
  "v_alignbit_b32 %5, %5, %5, 25\n" \
  "v_alignbit_b32 %6, %6, %6, 25\n" \
  "s_nop 0\n" \
  "v_alignbit_b32 %7, %7, %7, 25\n" \
  "v_alignbit_b32 %4, %4, %4, 25\n" \
  "s_nop 0\n"

#define DR_VOP2 \
  "v_add_u32 %0, %0, %4\n" \
  "v_add_u32 %1, %1, %5\n" \
  "v_add_u32 %2, %2, %6\n" \
  "v_add_u32 %3, %3, %7\n" \
  "s_nop 0\n" \
  "v_xor_b32 %12, %12, %0\n" \
  "v_xor_b32 %13, %13, %1\n" \
  "v_xor_b32 %14, %14, %2\n" \
  "v_xor_b32 %15, %15, %3\n" \
  "s_nop 0\n" \
  "v_alignbit_b32 %12, %12, %12, 16\n" \
  "v_alignbit_b32 %13, %13, %13, 16\n" \
  "v_alignbit_b32 %14, %14, %14, 16\n" \
  "v_alignbit_b32 %15, %15, %15, 16\n" \
  "v_add_u32 %8, %8, %12\n" \
  "v_add_u32 %9, %9, %13\n" \
  "v_add_u32 %10, %10, %14\n" \
  "v_add_u32 %11, %11, %15\n" \
  "s_nop 0\n" \
  "v_xor_b32 %4, %4, %8\n" \
  "v_xor_b32 %5, %5, %9\n" \
  "v_xor_b32 %6, %6, %10\n" \
  "v_xor_b32 %7, %7, %11\n" \
  "s_nop 0\n" \
  "v_alignbit_b32 %4, %4, %4, 20\n" \
  "v_alignbit_b32 %5, %5, %5, 20\n" \
  "v_alignbit_b32 %6, %6, %6, 20\n" \
  "v_alignbit_b32 %7, %7, %7, 20\n" \
  "v_add_u32 %0, %0, %4\n" \
  "v_add_u32 %1, %1, %5\n" \
  "v_add_u32 %2, %2, %6\n" \
  "v_add_u32 %3, %3, %7\n" \
  "s_nop 0\n" \
  "v_xor_b32 %12, %12, %0\n" \
  "v_xor_b32 %13, %13, %1\n" \
  "v_xor_b32 %14, %14, %2\n" \
  "v_xor_b32 %15, %15, %3\n" \
  "s_nop 0\n" \
  "v_alignbit_b32 %12, %12, %12, 24\n" \
  "v_alignbit_b32 %13, %13, %13, 24\n" \
  "v_alignbit_b32 %14, %14, %14, 24\n" \
  "v_alignbit_b32 %15, %15, %15, 24\n" \
  "v_add_u32 %8, %8, %12\n" \
  "v_add_u32 %9, %9, %13\n" \
  "v_add_u32 %10, %10, %14\n" \
  "v_add_u32 %11, %11, %15\n" \
  "s_nop 0\n" \
  "v_xor_b32 %4, %4, %8\n" \
  "v_xor_b32 %5, %5, %9\n" \
  "v_xor_b32 %6, %6, %10\n" \
  "v_xor_b32 %7, %7, %11\n" \
  "s_nop 0\n" \
  "v_alignbit_b32 %4, %4, %4, 25\n" \
  "v_alignbit_b32 %5, %5, %5, 25\n" \
  "v_alignbit_b32 %6, %6, %6, 25\n" \
  "v_alignbit_b32 %7, %7, %7, 25\n" \
  "v_add_u32 %0, %0, %5\n" \
  "v_add_u32 %1, %1, %6\n" \
  "v_add_u32 %2, %2, %7\n" \
  "v_add_u32 %3, %3, %4\n" \
  "s_nop 0\n" \
  "v_xor_b32 %15, %15, %0\n" \
  "v_xor_b32 %12, %12, %1\n" \
  "v_xor_b32 %13, %13, %2\n" \
  "v_xor_b32 %14, %14, %3\n" \
  "s_nop 0\n" \
  "v_alignbit_b32 %15, %15, %15, 16\n" \
  "v_alignbit_b32 %12, %12, %12, 16\n" \
  "v_alignbit_b32 %13, %13, %13, 16\n" \
  "v_alignbit_b32 %14, %14, %14, 16\n" \
  "v_add_u32 %10, %10, %15\n" \
  "v_add_u32 %11, %11, %12\n" \
  "v_add_u32 %8, %8, %13\n" \
  "v_add_u32 %9, %9, %14\n" \
  "s_nop 0\n" \
  "v_xor_b32 %5, %5, %10\n" \
  "v_xor_b32 %6, %6, %11\n" \
  "v_xor_b32 %7, %7, %8\n" \
  "v_xor_b32 %4, %4, %9\n" \
  "s_nop 0\n" \
  "v_alignbit_b32 %5, %5, %5, 20\n" \
  "v_alignbit_b32 %6, %6, %6, 20\n" \
  "v_alignbit_b32 %7, %7, %7, 20\n" \
  "v_alignbit_b32 %4, %4, %4, 20\n" \
  "v_add_u32 %0, %0, %5\n" \
  "v_add_u32 %1, %1, %6\n" \
  "v_add_u32 %2, %2, %7\n" \
  "v_add_u32 %3, %3, %4\n" \
  "s_nop 0\n" \
  "v_xor_b32 %15, %15, %0\n" \
  "v_xor_b32 %12, %12, %1\n" \
  "v_xor_b32 %13, %13, %2\n" \
  "v_xor_b32 %14, %14, %3\n" \
  "s_nop 0\n" \
  "v_alignbit_b32 %15, %15, %15, 24\n" \
  "v_alignbit_b32 %12, %12, %12, 24\n" \
  "v_alignbit_b32 %13, %13, %13, 24\n" \
  "v_alignbit_b32 %14, %14, %14, 24\n" \
  "v_add_u32 %10, %10, %15\n" \
  "v_add_u32 %11, %11, %12\n" \
  "v_add_u32 %8, %8, %13\n" \
  "v_add_u32 %9, %9, %14\n" \
  "s_nop 0\n" \
  "v_xor_b32 %5, %5, %10\n" \
  "v_xor_b32 %6, %6, %11\n" \
  "v_xor_b32 %7, %7, %8\n" \
  "v_xor_b32 %4, %4, %9\n" \
  "s_nop 0\n" \
  "v_alignbit_b32 %5, %5, %5, 25\n" \
  "v_alignbit_b32 %6, %6, %6, 25\n" \
  "v_alignbit_b32 %7, %7, %7, 25\n" \
  "v_alignbit_b32 %4, %4, %4, 25\n"

#define DR_ROT \
  "v_add_u32 %0, %0, %4\n" \
  "v_add_u32 %1, %1, %5\n" \
  "v_add_u32 %2, %2, %6\n" \
  "v_add_u32 %3, %3, %7\n" \
  "v_xor_b32 %12, %12, %0\n" \
  "v_xor_b32 %13, %13, %1\n" \
  "v_xor_b32 %14, %14, %2\n" \
  "v_xor_b32 %15, %15, %3\n" \
  "v_alignbit_b32 %12, %12, %12, 16\n" \
  "v_alignbit_b32 %13, %13, %13, 16\n" \
  "v_alignbit_b32 %14, %14, %14, 16\n" \
  "v_alignbit_b32 %15, %15, %15, 16\n" \
  "s_nop 0\n" \
  "v_add_u32 %8, %8, %12\n" \
  "v_add_u32 %9, %9, %13\n" \
  "v_add_u32 %10, %10, %14\n" \
  "v_add_u32 %11, %11, %15\n" \
  "v_xor_b32 %4, %4, %8\n" \
  "v_xor_b32 %5, %5, %9\n" \
  "v_xor_b32 %6, %6, %10\n" \
  "v_xor_b32 %7, %7, %11\n" \
  "v_alignbit_b32 %4, %4, %4, 20\n" \
  "v_alignbit_b32 %5, %5, %5, 20\n" \
  "v_alignbit_b32 %6, %6, %6, 20\n" \
  "v_alignbit_b32 %7, %7, %7, 20\n" \
  "s_nop 0\n" \
  "v_add_u32 %0, %0, %4\n" \
  "v_add_u32 %1, %1, %5\n" \
  "v_add_u32 %2, %2, %6\n" \
  "v_add_u32 %3, %3, %7\n" \
  "v_xor_b32 %12, %12, %0\n" \
  "v_xor_b32 %13, %13, %1\n" \
  "v_xor_b32 %14, %14, %2\n" \
  "v_xor_b32 %15, %15, %3\n" \
  "v_alignbit_b32 %12, %12, %12, 24\n" \
  "v_alignbit_b32 %13, %13, %13, 24\n" \
  "v_alignbit_b32 %14, %14, %14, 24\n" \
  "v_alignbit_b32 %15, %15, %15, 24\n" \
  "s_nop 0\n" \
  "v_add_u32 %8, %8, %12\n" \
  "v_add_u32 %9, %9, %13\n" \
  "v_add_u32 %10, %10, %14\n" \
  "v_add_u32 %11, %11, %15\n" \
  "v_xor_b32 %4, %4, %8\n" \
  "v_xor_b32 %5, %5, %9\n" \
  "v_xor_b32 %6, %6, %10\n" \
  "v_xor_b32 %7, %7, %11\n" \
  "v_alignbit_b32 %4, %4, %4, 25\n" \
  "v_alignbit_b32 %5, %5, %5, 25\n" \
  "v_alignbit_b32 %6, %6, %6, 25\n" \
  "v_alignbit_b32 %7, %7, %7, 25\n" \
  "s_nop 0\n" \
  "v_add_u32 %0, %0, %5\n" \
  "v_add_u32 %1, %1, %6\n" \
  "v_add_u32 %2, %2, %7\n" \
  "v_add_u32 %3, %3, %4\n" \
  "v_xor_b32 %15, %15, %0\n" \
  "v_xor_b32 %12, %12, %1\n" \
  "v_xor_b32 %13, %13, %2\n" \
  "v_xor_b32 %14, %14, %3\n" \
  "v_alignbit_b32 %15, %15, %15, 16\n" \
  "v_alignbit_b32 %12, %12, %12, 16\n" \
  "v_alignbit_b32 %13, %13, %13, 16\n" \
  "v_alignbit_b32 %14, %14, %14, 16\n" \
  "s_nop 0\n" \
  "v_add_u32 %10, %10, %15\n" \
  "v_add_u32 %11, %11, %12\n" \
  "v_add_u32 %8, %8, %13\n" \
  "v_add_u32 %9, %9, %14\n" \
  "v_xor_b32 %5, %5, %10\n" \
  "v_xor_b32 %6, %6, %11\n" \
  "v_xor_b32 %7, %7, %8\n" \
  "v_xor_b32 %4, %4, %9\n" \
  "v_alignbit_b32 %5, %5, %5, 20\n" \
  "v_alignbit_b32 %6, %6, %6, 20\n" \
  "v_alignbit_b32 %7, %7, %7, 20\n" \
  "v_alignbit_b32 %4, %4, %4, 20\n" \
  "s_nop 0\n" \
  "v_add_u32 %0, %0, %5\n" \
  "v_add_u32 %1, %1, %6\n" \
  "v_add_u32 %2, %2, %7\n" \
  "v_add_u32 %3, %3, %4\n" \
  "v_xor_b32 %15, %15, %0\n" \
  "v_xor_b32 %12, %12, %1\n" \
  "v_xor_b32 %13, %13, %2\n" \
  "v_xor_b32 %14, %14, %3\n" \
  "v_alignbit_b32 %15, %15, %15, 24\n" \
  "v_alignbit_b32 %12, %12, %12, 24\n" \
  "v_alignbit_b32 %13, %13, %13, 24\n" \
  "v_alignbit_b32 %14, %14, %14, 24\n" \
  "s_nop 0\n" \
  "v_add_u32 %10, %10, %15\n" \
  "v_add_u32 %11, %11, %12\n" \
  "v_add_u32 %8, %8, %13\n" \
  "v_add_u32 %9, %9, %14\n" \
  "v_xor_b32 %5, %5, %10\n" \
  "v_xor_b32 %6, %6, %11\n" \
  "v_xor_b32 %7, %7, %8\n" \
  "v_xor_b32 %4, %4, %9\n" \
  "v_alignbit_b32 %5, %5, %5, 25\n" \
  "v_alignbit_b32 %6, %6, %6, 25\n" \
  "v_alignbit_b32 %7, %7, %7, 25\n" \
  "v_alignbit_b32 %4, %4, %4, 25\n" \
  "s_nop 0\n"

CHACHA_VARIANT(k_cc_nop0, DR_NOP0)
CHACHA_VARIANT(k_cc_pair, DR_PAIR)
CHACHA_VARIANT(k_cc_vop2, DR_VOP2)
CHACHA_VARIANT(k_cc_rot, DR_ROT)
CHACHA_VARIANT(k_cc_nop1, DR_NOP1)
CHACHA_VARIANT(k_cc_plain, DR_SETPRIO)

typedef void (*kfn)(uint64_t*, uint32_t);

int main() {
  const int blocks = 256 * 8, threads = 256;
  uint64_t* d;
  hipMalloc(&d, sizeof(uint64_t) * blocks * threads);
  struct { const char* name; kfn f; } ks[] = {
      {"v_mad_u64_u32", k_mad64}, {"v_mul_lo_u32", k_mullo}, {"v_mul_hi_u32", k_mulhi},
      {"v_add_co_u32", k_addc},   {"v_add3_u32", k_add3},    {"v_fma_f64", k_fma64},
      {"v_mad_u32_u24", k_mul24}, {"v_add_u32", k_add32}, {"v_xor_b32", k_xor32},
      {"v_alignbit_b32", k_align}, {"v_perm_b32", k_perm}, {"v_lshl_or_b32", k_lshlor}, {"v_xad_u32", k_xad}, {"v_pk_add_u16", k_bfi},
      {"v_lshrrev_b64", k_lshr64}, {"v_lshl_add_u64", k_lshladd64}, {"v_xor_b32_sdwa", k_xorsdwa}, {"chacha20 (976/blk)", k_chacha},
      {"cc groups+nop0", k_cc_nop0}, {"cc groups+nop1", k_cc_nop1}, {"cc groups", k_cc_plain},
      {"cc nop per pair", k_cc_pair}, {"cc nop after vop2", k_cc_vop2}, {"cc nop after rot", k_cc_rot}};
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (auto& k : ks) {
    hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, d, 1u);
    hipDeviceSynchronize();
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
      hipEventRecord(e0);
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, d, 1u);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (ms < best) best = ms;
    }
    double ops = (double)blocks * threads * ITER * CH;
    if (k.f == k_chacha || k.f == k_cc_nop0 || k.f == k_cc_nop1 || k.f == k_cc_plain || k.f == k_cc_pair ||
        k.f == k_cc_vop2 || k.f == k_cc_rot) ops = (double)blocks * threads * CHACHA_BLOCKS * 976.0;
    printf("%-16s %8.3f ms  %8.1f G lane-ops/s  (%.2f cyc/wave-instr @2.4GHz/1024 SIMDs)\n", k.name, best,
           ops / best / 1e6, (1024.0 * 2.4e9) / (ops / 64.0 / (best * 1e-3)));
  }
  {  // the variants must agree with each other (same keystream schedule)
    const size_t cnt = (size_t)blocks * threads;
    std::vector<uint64_t> h[3];
    kfn fs[3] = {k_cc_nop0, k_cc_nop1, k_cc_plain};
    for (int i = 0; i < 3; ++i) {
      hipLaunchKernelGGL(fs[i], dim3(blocks), dim3(threads), 0, 0, d, 3u);
      hipDeviceSynchronize();
      h[i].resize(cnt);
      hipMemcpy(h[i].data(), d, sizeof(uint64_t) * cnt, hipMemcpyDeviceToHost);
    }
    printf("variants agree: %s\n", (h[0] == h[1] && h[1] == h[2]) ? "yes" : "NO");
  }
  return 0;
}
