// fedbiomed_amd -- additive secret sharing of vectors for gfx950.
//
//   ass_split_kernel        AdditiveSecret.split / _shares_int  (secagg/_additive_ss.py:40-98)
//   ass_reconstruct_kernel  AdditiveShares.reconstruct          (secagg/_additive_ss.py:252-267)
//
// Per element v (64-bit): n_shares-1 shares uniform in [0, 2^b] (random.randint(0, 2**b) is
// inclusive; b = bit length of |v| unless given), the last share = v - sum(others).  Shares can
// reach -(P-1)*2^64, so they are int128 (lo, hi) pairs, share-major: shares[(s*n + i)*2 + {0,1}].
// The reference draws from Python's MT19937; only the invariants are part of the contract
// (SURVEY §8 a18): sum == secret exactly, first P-1 shares in [0, 2^b].  Randomness here:
// ChaCha20(seed, counter = global element index * blocks_per_element + j), 128 bits per share,
// Lemire multiply-high onto the 2^b + 1 values (statistical distance <= 2^-63).
#include "fbm_internal.hpp"

namespace fbm {

struct AssParams {
  uint32_t key[8];     // ChaCha20 key (seed)
  uint32_t n14, n15;   // nonce words
  uint64_t elem_offset;
  int n_shares;
  int bit_length;      // < 0: per-element bit length of |v|
  int is_signed;       // secret dtype int64 (else uint64)
  int pad;
};

__device__ __forceinline__ unsigned __int128 lemire_0_2b(unsigned __int128 x, int b) {
  // floor(x * (2^b + 1) / 2^128) for 0 <= b <= 64: uniform-ish in [0, 2^b]
  const unsigned __int128 hi = b ? (x >> (128 - b)) : (unsigned __int128)0;  // (x << b) >> 128
  const unsigned __int128 lo = x << b;                                         // (x << b) mod 2^128
  const unsigned __int128 s = lo + x;
  return hi + (s < lo ? 1 : 0);
}

__global__ void __launch_bounds__(256) ass_split_kernel(const uint64_t* __restrict__ secret, uint64_t n, AssParams p,
                                                        int64_t* __restrict__ shares) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t raw = secret[i];
  // value as int128 and its bit length (Python int.bit_length of |v|)
  __int128 v;
  uint64_t mag;
  if (p.is_signed) {
    const int64_t s = (int64_t)raw;
    v = s;
    mag = s < 0 ? (uint64_t)0 - raw : raw;
  } else {
    v = (__int128)(unsigned __int128)raw;
    mag = raw;
  }
  const int b = p.bit_length >= 0 ? p.bit_length : (mag ? 64 - __builtin_clzll(mag) : 0);
  const int bpe = (p.n_shares - 1 + 3) / 4;  // ChaCha blocks per element (4 shares per block)
  const uint64_t ctr0 = (p.elem_offset + i) * (uint64_t)bpe;
  __int128 sum = 0;
  uint32_t ks[16];
  for (int s = 0; s < p.n_shares - 1; ++s) {
    if ((s & 3) == 0) fbm_chacha20_block(p.key, ctr0 + (uint64_t)(s >> 2), p.n14, p.n15, ks);
    const int w = (s & 3) * 4;
    const unsigned __int128 x = ((unsigned __int128)(((uint64_t)ks[w + 3] << 32) | ks[w + 2]) << 64) |
                                (((uint64_t)ks[w + 1] << 32) | ks[w]);
    const unsigned __int128 r = lemire_0_2b(x, b);
    sum += (__int128)r;
    int64_t* o = shares + ((uint64_t)s * n + i) * 2;
    o[0] = (int64_t)(uint64_t)r;
    o[1] = (int64_t)(uint64_t)(r >> 64);
  }
  const __int128 last = v - sum;
  int64_t* o = shares + ((uint64_t)(p.n_shares - 1) * n + i) * 2;
  o[0] = (int64_t)(uint64_t)(unsigned __int128)last;
  o[1] = (int64_t)(uint64_t)((unsigned __int128)last >> 64);
}

// exact column sum of int128 shares (two's complement; exact while |sum| < 2^127)
__global__ void __launch_bounds__(256) ass_reconstruct_kernel(const int64_t* __restrict__ shares, int n_shares,
                                                              uint64_t n, int64_t* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  unsigned __int128 acc = 0;
  for (int s = 0; s < n_shares; ++s) {
    const longlong2 v = *reinterpret_cast<const longlong2*>(shares + ((uint64_t)s * n + i) * 2);
    acc += ((unsigned __int128)(uint64_t)v.y << 64) | (uint64_t)v.x;
  }
  *reinterpret_cast<longlong2*>(out + i * 2) = make_longlong2((int64_t)(uint64_t)acc, (int64_t)(uint64_t)(acc >> 64));
}

int launch_ass_split(const uint64_t* secret, uint64_t n, const uint32_t* key, uint32_t n14, uint32_t n15,
                     uint64_t elem_offset, int n_shares, int bit_length, int is_signed, int64_t* shares,
                     hipStream_t s) {
  if (n == 0) return FBM_OK;
  AssParams p;
  for (int w = 0; w < 8; ++w) p.key[w] = key[w];
  p.n14 = n14;
  p.n15 = n15;
  p.elem_offset = elem_offset;
  p.n_shares = n_shares;
  p.bit_length = bit_length;
  p.is_signed = is_signed;
  p.pad = 0;
  hipLaunchKernelGGL(ass_split_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, secret, n, p, shares);
  return check_launch("ass_split_kernel");
}

int launch_ass_reconstruct(const int64_t* shares, int n_shares, uint64_t n, int64_t* out, hipStream_t s) {
  if (n == 0) return FBM_OK;
  hipLaunchKernelGGL(ass_reconstruct_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, shares, n_shares,
                     n, out);
  return check_launch("ass_reconstruct_kernel");
}

}  // namespace fbm
