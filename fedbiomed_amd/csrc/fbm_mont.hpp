// fedbiomed_amd -- Montgomery arithmetic for gfx950 (one lane = one residue).
//
// Replaces GMP's mpz_powm / mpz mult-mod that the reference reaches through gmpy2
// (fedbiomed/common/secagg/_jls.py:60-73 powmod, :353-374 ciphertext product,
//  :494-502 encrypt, :547-558 decrypt).
//
// Representation: radix 2^28.  Modulus N^2 (<= 2048 bits): NL = 74 limbs, R = 2^2072.
// Modulus N (<= 1024 bits, used for the inverse mod N): NL = 37 limbs, R = 2^1036.
// Why 28-bit limbs: on gfx950 `v_mad_u64_u32` issues at ~full VALU rate (measured,
// tools/microbench/intrate.hip).  A 28x28-bit product is < 2^56, so a 64-bit column
// accumulator absorbs >= 256 of them without overflow: every multiply-accumulate of the
// Montgomery product is ONE `v_mad_u64_u32` with no carry chain (32-bit-limb CIOS needs
// mad + add_co + addc per limb product).  Carries are resolved once per product.
//
// Per-lane state of one product: NL-1 64-bit accumulators + the B operand in VGPRs; the
// A operand is consumed one limb per row from a per-lane LDS column (ds_read_b32,
// conflict-free [limb][lane] layout); the modulus limbs are uniform (scalar loads).
#pragma once
#include "fbm_common.hpp"

#define FBM_NL 74
#define FBM_NLN 37
#define FBM_LB 28
#define FBM_LMASK 0x0FFFFFFFu

template <int NL>
struct MontCtxT {
  uint32_t M[NL];    // modulus limbs (radix 2^28), M odd
  uint32_t R2[NL];   // R^2 mod M
  uint32_t mp;       // -M^{-1} mod 2^28
  uint32_t pad;
};
typedef MontCtxT<FBM_NL> MontCtx;
typedef MontCtxT<FBM_NLN> MontCtxN;

// Pointer laundering.  Hot kernels run a loop around one ~90 KB Montgomery product; any
// loop-invariant address or uniform constant the optimiser hoists out of that loop stays
// live across the product and pushes it over 256 VGPRs.  Passing the base through an
// empty asm makes every use re-derive it locally (a few scalar/vector adds).
template <typename T>
__device__ __forceinline__ T* launder_v(T* p) {
  asm volatile("" : "+v"(p));
  return p;
}
template <typename T>
__device__ __forceinline__ const T* launder_s(const T* p) {
  asm volatile("" : "+s"(p));
  return p;
}

// b <- b - M if b >= M  (b < 2M, normalised limbs): full reduction of a lazy result
template <int NL>
__device__ __forceinline__ void mont_csub(uint32_t (&b)[NL], const uint32_t* M) {
  int32_t borrow = 0;
#pragma unroll
  for (int k = 0; k < NL; ++k) {
    const int32_t v = (int32_t)b[k] - (int32_t)M[k] + borrow;
    borrow = v >> FBM_LB;  // 0 or -1
  }
  if (borrow == 0) {
    borrow = 0;
#pragma unroll
    for (int k = 0; k < NL; ++k) {
      const int32_t v = (int32_t)b[k] - (int32_t)M[k] + borrow;
      b[k] = (uint32_t)v & FBM_LMASK;
      borrow = v >> FBM_LB;
    }
  }
}

// -------------------------------------------------------------------------------------
// Montgomery product  b <- a * b * R^{-1}  (lazy: result < 2M, NOT fully reduced)
//   requires a*b < R*M;  with R >= 2^24 * M (R = 2^2072 vs M < 2^2048, R_N = 2^1036 vs
//   N < 2^1024) any a, b < 2^k*M with small k qualify, so operands may stay in [0, 2M)
//   for whole exponentiations and only the final result is reduced (mont_csub).
//   a: limb i at lds[i * ls] (per-lane LDS column)
//
// The row loop is FULLY unrolled on purpose: with a runtime row loop the 64-bit
// accumulator window shifts by one column per row, and LLVM cannot coalesce the
// loop-carried copies (it doubles the accumulator registers and spills).  Unrolled, the
// shift is pure renaming: 146 + 74 + ~25 VGPRs, no spills.  The modulus pointer is
// laundered per row so the 74 uniform limbs are re-read with scalar loads instead of
// being hoisted into (and spilling out of) the SGPR file.
// -------------------------------------------------------------------------------------
template <int NL>
__device__ __forceinline__ void mont_mul(uint32_t (&b)[NL], const uint32_t* lds, int ls, const MontCtxT<NL>& c) {
  uint64_t A[NL - 1];
#pragma unroll
  for (int j = 0; j < NL - 1; ++j) A[j] = 0;
#pragma clang loop unroll(full)
  for (int i = 0; i < NL; ++i) {
    const uint32_t* M = launder_s(c.M);
    const uint32_t ai = lds[i * ls];
    uint64_t a0 = A[0] + (uint64_t)ai * b[0];
    const uint32_t m = ((uint32_t)a0 * c.mp) & FBM_LMASK;
    a0 += (uint64_t)m * M[0];
    const uint64_t carry = a0 >> FBM_LB;
#pragma unroll
    for (int j = 1; j < NL - 1; ++j) A[j - 1] = A[j] + (uint64_t)ai * b[j] + (uint64_t)m * M[j];
    A[NL - 2] = (uint64_t)ai * b[NL - 1] + (uint64_t)m * M[NL - 1];
    A[0] += carry;
  }
  // normalise: t = sum A[k] 2^(28k) < 2M
  uint64_t carry = 0;
#pragma unroll
  for (int k = 0; k < NL - 1; ++k) {
    const uint64_t v = A[k] + carry;
    b[k] = (uint32_t)v & FBM_LMASK;
    carry = v >> FBM_LB;
  }
  b[NL - 1] = (uint32_t)carry;
}

// blocked limb-major layout for per-lane 28-bit residues: lane l of workgroup g owns
// limb k at base[(g * NL + k) * 256 + l]  (constant 1 KB stride between limbs)
template <int NL>
__device__ __forceinline__ void col_store(uint32_t* p, const uint32_t (&v)[NL]) {
  p = launder_v(p);
#pragma unroll
  for (int k = 0; k < NL; ++k) p[k * 256] = v[k];
}
template <int NL>
__device__ __forceinline__ void col_load(const uint32_t* p, uint32_t (&v)[NL]) {
  p = launder_v(p);
#pragma unroll
  for (int k = 0; k < NL; ++k) v[k] = p[k * 256];
}

template <int NL>
__device__ __forceinline__ void lds_store_col(uint32_t* lds, int ls, const uint32_t (&v)[NL]) {
#pragma unroll
  for (int k = 0; k < NL; ++k) lds[k * ls] = v[k];
}
template <int NL>
__device__ __forceinline__ void lds_load_col(const uint32_t* lds, int ls, uint32_t (&v)[NL]) {
#pragma unroll
  for (int k = 0; k < NL; ++k) v[k] = lds[k * ls];
}
template <int NL>
__device__ __forceinline__ void lds_store_uniform(uint32_t* lds, int ls, const uint32_t* u) {
  u = launder_s(u);
#pragma unroll
  for (int k = 0; k < NL; ++k) lds[k * ls] = u[k];
}
template <int NL>
__device__ __forceinline__ void lds_store_one(uint32_t* lds, int ls) {
#pragma unroll
  for (int k = 0; k < NL; ++k) lds[k * ls] = k == 0 ? 1u : 0u;
}

// -------------------------------------------------------------------------------------
// radix conversion  (32-bit little-endian limbs  <->  28-bit limbs)
// -------------------------------------------------------------------------------------
template <int N32, int NL>
__device__ __forceinline__ void to28(const uint32_t (&w)[N32], uint32_t (&o)[NL]) {
#pragma unroll
  for (int k = 0; k < NL; ++k) {
    const int bit = k * FBM_LB;
    const int wi = bit >> 5, sh = bit & 31;
    const uint64_t lo = (wi < N32) ? w[wi] : 0u;
    const uint64_t hi = (wi + 1 < N32) ? w[wi + 1] : 0u;
    o[k] = (uint32_t)(((hi << 32) | lo) >> sh) & FBM_LMASK;
  }
}

template <int NL, int N32>
__device__ __forceinline__ void from28(const uint32_t (&o)[NL], uint32_t (&w)[N32]) {
#pragma unroll
  for (int i = 0; i < N32; ++i) {
    const int bit = i * 32;
    const int k = bit / FBM_LB, sh = bit % FBM_LB;
    uint64_t v = 0;
    v |= (uint64_t)((k < NL) ? o[k] : 0u) >> sh;
    v |= (uint64_t)((k + 1 < NL) ? o[k + 1] : 0u) << (FBM_LB - sh);
    v |= (uint64_t)((k + 2 < NL) ? o[k + 2] : 0u) << (2 * FBM_LB - sh);
    w[i] = (uint32_t)v;
  }
}
