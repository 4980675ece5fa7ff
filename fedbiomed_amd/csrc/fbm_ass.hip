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

// ------------------------------------------------------------------------------------------
// Wide path: secrets of any size (the reference's scalar use is the 2040-bit JL user key,
// node/secagg/_secagg_setups.py:248-268; researcher/secagg/_secagg_context.py:380).
// Values are two's-complement u32 limbs, limb-major: word (s*L + k)*n + i (share s, limb k,
// element i), so a wave's access to one limb is coalesced.  Share draw r uniform on [0, 2^b]:
// x = first b+64 bits of the share's ChaCha20 stream (LE words), r = (x >> 64) + carry,
// carry = [x mod 2^64 + (x >> b) >= 2^64] -- that is floor(x (2^b + 1) / 2^(b+64)), the
// multiply-high (Lemire) map of the 128-bit path above, for any b.
struct AssWide {
  uint32_t key[8];
  uint32_t n14, n15;
  uint64_t elem_offset;
  int n_shares;
  int bit_length;  // < 0: bit length of |v| per element
  int l_in, l_out; // limbs of a secret / of a share
  int blocks;      // ChaCha20 blocks per share draw (ceil((b_max + 64) / 512))
};

// word w (w < 16*blocks) of the draw stream of (element e, share s); one block is cached
struct AssStream {
  uint32_t ks[16];
  uint64_t cur;
  __device__ __forceinline__ uint32_t word(const AssWide& p, uint64_t base, int w) {
    const uint64_t blk = base + (uint64_t)(w >> 4);
    if (blk != cur) {
      fbm_chacha20_block(p.key, blk, p.n14, p.n15, ks);
      cur = blk;
    }
    return ks[w & 15];
  }
};

__global__ void __launch_bounds__(256) ass_split_wide_kernel(const uint32_t* __restrict__ secret, uint64_t n,
                                                             AssWide p, uint32_t* __restrict__ shares) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int L = p.l_out;
  auto sec = [&](int k) -> uint32_t {  // sign-extended secret limb k
    if (k < p.l_in) return secret[(uint64_t)k * n + i];
    return (secret[(uint64_t)(p.l_in - 1) * n + i] >> 31) ? 0xffffffffu : 0u;
  };
  const bool neg = sec(p.l_in - 1) >> 31;
  int b = p.bit_length;
  if (b < 0) {  // bit length of |v|: of v for v >= 0, of ~v + 1 otherwise
    b = 0;
    uint32_t carry = 1;
    for (int k = 0; k < p.l_in; ++k) {
      uint32_t w = sec(k);
      if (neg) {
        const uint64_t t = (uint64_t)(~w) + carry;
        w = (uint32_t)t;
        carry = (uint32_t)(t >> 32);
      }
      if (w) b = 32 * k + 32 - __builtin_clz(w);
    }
  }
  uint32_t* last = shares + (uint64_t)(p.n_shares - 1) * L * n;  // running v - sum(shares)
  for (int k = 0; k < L; ++k) last[(uint64_t)k * n + i] = sec(k);
  const int xw = (b + 64 + 31) / 32;  // words of x
  const uint32_t topmask = ((b + 64) & 31) ? ((1u << ((b + 64) & 31)) - 1u) : 0xffffffffu;
  for (int sh = 0; sh < p.n_shares - 1; ++sh) {
    const uint64_t base = ((p.elem_offset + i) * (uint64_t)(p.n_shares - 1) + (uint64_t)sh) * (uint64_t)p.blocks;
    AssStream st;
    st.cur = ~0ull;
    auto xword = [&](int w) -> uint32_t {
      if (w >= xw) return 0u;
      const uint32_t v = st.word(p, base, w);
      return w == xw - 1 ? (v & topmask) : v;
    };
    // q = x >> b (64 bits: x has b + 64 bits)
    const int wq = b >> 5, sq = b & 31;
    const unsigned __int128 v96 = ((unsigned __int128)xword(wq + 2) << 64) |
                                  ((unsigned __int128)xword(wq + 1) << 32) | (unsigned __int128)xword(wq);
    const uint64_t q = (uint64_t)(v96 >> sq);
    const uint64_t xl = (uint64_t)xword(0) | ((uint64_t)xword(1) << 32);
    uint32_t carry = (xl + q < xl) ? 1u : 0u;
    // r = (x >> 64) + carry; share limb k = word k + 2; last -= r
    uint32_t* out = shares + (uint64_t)sh * L * n;
    uint32_t borrow = 0;
    for (int k = 0; k < L; ++k) {
      const uint64_t rk = (uint64_t)xword(k + 2) + carry;
      const uint32_t r = (uint32_t)rk;
      carry = (uint32_t)(rk >> 32);
      out[(uint64_t)k * n + i] = r;
      const uint64_t l = (uint64_t)last[(uint64_t)k * n + i] - r - borrow;
      last[(uint64_t)k * n + i] = (uint32_t)l;
      borrow = (uint32_t)(l >> 63);
    }
  }
}

// exact column sum of P two's-complement L-limb values (result L limbs, wraps mod 2^(32L):
// the caller sizes L so the true sum fits)
__global__ void __launch_bounds__(256) ass_reconstruct_wide_kernel(const uint32_t* __restrict__ shares,
                                                                   int n_shares, int L, uint64_t n,
                                                                   uint32_t* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t carry = 0;  // signed carry into limb k, kept as a two's-complement 64-bit value
  for (int k = 0; k < L; ++k) {
    int64_t acc = (int64_t)carry;
    for (int s = 0; s < n_shares; ++s) acc += (int64_t)(uint64_t)shares[((uint64_t)s * L + k) * n + i];
    out[(uint64_t)k * n + i] = (uint32_t)(uint64_t)acc;
    carry = (uint64_t)(acc >> 32);  // arithmetic shift: limbs are unsigned digits, carry may be 0..P
  }
}

int launch_ass_split_wide(const uint32_t* secret, uint64_t n, int l_in, const uint32_t* key, uint32_t n14,
                          uint32_t n15, uint64_t elem_offset, int n_shares, int bit_length, int l_out,
                          uint32_t* shares, hipStream_t s) {
  if (n == 0) return FBM_OK;
  AssWide p;
  for (int w = 0; w < 8; ++w) p.key[w] = key[w];
  p.n14 = n14;
  p.n15 = n15;
  p.elem_offset = elem_offset;
  p.n_shares = n_shares;
  p.bit_length = bit_length;
  p.l_in = l_in;
  p.l_out = l_out;
  const int bmax = bit_length >= 0 ? bit_length : 32 * l_in;
  p.blocks = (bmax + 64 + 511) / 512;
  hipLaunchKernelGGL(ass_split_wide_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, secret, n, p,
                     shares);
  return check_launch("ass_split_wide_kernel");
}

int launch_ass_reconstruct_wide(const uint32_t* shares, int n_shares, int l, uint64_t n, uint32_t* out,
                                hipStream_t s) {
  if (n == 0) return FBM_OK;
  hipLaunchKernelGGL(ass_reconstruct_wide_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, shares,
                     n_shares, l, n, out);
  return check_launch("ass_reconstruct_wide_kernel");
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

// Wave-split reconstruct (round 5) for a compile-time share count S: W waves per workgroup, one tile of 64
// elements; wave w loads shares w, w + W, ... (16-byte nontemporal loads), the W partial int128 sums meet in
// LDS and the 64 results leave through the workgroup's first wave.  The lom_aggregate_ws_kernel form
// (fbm_lom.hip), for config 5's 16-share reconstruct.
#ifndef FBM_ASS_WS
#define FBM_ASS_WS 1  // 0: ass_reconstruct_kernel for every share count (A/B base)
#endif
template <int W, int S>
__global__ void __launch_bounds__(64 * W) ass_reconstruct_ws_kernel(const int64_t* __restrict__ shares, uint64_t n,
                                                                    int64_t* __restrict__ out) {
  static_assert(S % W == 0, "shares per wave");
  __shared__ unsigned __int128 part[W][64];
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const uint64_t i = (uint64_t)blockIdx.x * 64 + l;
  typedef long long ll2 __attribute__((ext_vector_type(2)));
  unsigned __int128 acc = 0;
  if (i < n) {
    ll2 v[S / W];
#pragma unroll
    for (int k = 0; k < S / W; ++k)
      v[k] = __builtin_nontemporal_load(reinterpret_cast<const ll2*>(shares + ((uint64_t)(w + W * k) * n + i) * 2));
#pragma unroll
    for (int k = 0; k < S / W; ++k) acc += ((unsigned __int128)(uint64_t)v[k].y << 64) | (uint64_t)v[k].x;
  }
  part[w][l] = acc;
  __syncthreads();
  if (w == 0 && i < n) {
#pragma unroll
    for (int q = 1; q < W; ++q) acc += part[q][l];
    const ll2 r = {(long long)(uint64_t)acc, (long long)(uint64_t)(acc >> 64)};
    __builtin_nontemporal_store(r, reinterpret_cast<ll2*>(out + i * 2));
  }
}

int launch_ass_reconstruct(const int64_t* shares, int n_shares, uint64_t n, int64_t* out, hipStream_t s) {
  if (n == 0) return FBM_OK;
  if (FBM_ASS_WS && n_shares == 16) {
    hipLaunchKernelGGL((ass_reconstruct_ws_kernel<8, 16>), dim3((unsigned)((n + 63) / 64)), dim3(512), 0, s, shares, n,
                       out);
    return check_launch("ass_reconstruct_ws_kernel");
  }
  hipLaunchKernelGGL(ass_reconstruct_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, shares, n_shares,
                     n, out);
  return check_launch("ass_reconstruct_kernel");
}

}  // namespace fbm
