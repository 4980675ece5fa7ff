// fedbiomed_amd -- Joye-Libert kernels for gfx950.
//
// Encrypt (one party):  pack -> nude -> fdh -> exp(ENC)
//   jl_pack_kernel   quantize + weight + VES.encode     (_secagg_utils.py:82-119,
//                    _secagg_crypter.py:252-276, _jls.py:118-144,169-176)
//   jl_nude_kernel   N*pt + 1 as N-adic digits (1, pt)     (_jls.py:494-496)
//   jl_fdh_kernel    FDH.H(t_k), t_k = (k<<512)|tau       (_jls.py:451-467,727-762)
//   jl_exp_kernel    H^sk mod N^2 (GMP mpz_powm via gmpy2, _jls.py:60-73,500-501) and
//                    the final product with nude           (_jls.py:502)
// Encrypt with its factor computed ahead (fbm_jl_encrypt_factor):  pack -> encf
//   jl_encf_kernel   (N*pt + 1) * F mod N^2, F = H^sk from the aggregate's factor kernels
// Aggregate:  fdh -> exp(DEC, digits out) -> inv -> lift -> prod -> decode
//   jl_exp_kernel    H^|sk0| mod N^2 as N-adic digits     (_jls.py:550-551)
//   jl_inv_modn_kernel, jl_lift_kernel
//                    (H^|sk0|)^-1 mod N^2 (gmpy2.powmod with b<0 inverts; _jls.py:550-551)
//   jl_prod_kernel   v = prod_u c_u * factor mod N^2, x = (v-1)//N   (_jls.py:353-374,
//                    691-693, 553-558)
//   jl_decode_kernel VES.decode + _apply_average + reverse_quantize
//                    (_jls.py:146-192, _secagg_crypter.py:233-249, _secagg_utils.py:152-187)
//
// HBM layouts: 32-bit-limb integers are row-major [ct][words] (pt: 32 words, H / E / inv /
// ciphertexts: 64 words = int.to_bytes(256,'little')); 28-bit-limb residues (nude, X) and
// the per-lane exponent tables are limb-major [limb][lane] so a wave's accesses coalesce.
#include <stdlib.h>
#include <string.h>

#include <atomic>

#include "fbm_internal.hpp"
#include "fbm_mont_asm.hpp"
#include "fbm_nadic_asm.hpp"
#include "fbm_quad_asm.hpp"
#include "fbm_tri_asm.hpp"
#include "fbm_safegcd.hpp"

namespace fbm {

#define FBM_BLOCK 256

// ------------------------------------------------------------------------------------
// pack: one work-item per 32-bit limb of a packed plaintext
// ------------------------------------------------------------------------------------
// XT = float/double: quantise (crypter path);  XT = uint64_t: raw integers (JoyeLibert.protect)
template <typename XT>
__device__ __forceinline__ uint64_t jl_input(const XT* x, uint64_t i, const QuantParams& qp, bool& clipped) {
  const double v = (double)x[i];
  clipped |= fbm_outside_clip(v, qp);
  return fbm_quantize(v, qp);
}
template <>
__device__ __forceinline__ uint64_t jl_input<uint64_t>(const uint64_t* x, uint64_t i, const QuantParams&, bool&) {
  return x[i];
}

template <typename XT>
__global__ void __launch_bounds__(256) jl_pack_kernel(const XT* __restrict__ x, uint64_t n, QuantParams qp,
                                                      uint64_t weight, int es, int cr, uint64_t n_ct,
                                                      uint32_t* __restrict__ pt, uint32_t* __restrict__ stats) {
  const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t ct = gid >> 5;
  const int L = (int)(gid & 31);
  bool clipped = false;
  if (ct >= n_ct) {
    flag_if_any(false, stats, FBM_WARN_CLIPPED);
    return;
  }
  const uint64_t first = ct * (uint64_t)cr;
  const int cnt = (n - first) >= (uint64_t)cr ? cr : (int)(n - first);
  const int lo_bit = 32 * L;
  uint32_t w = 0;
  if ((int64_t)weight >= 0) {
    int j0 = lo_bit / es, j1 = (lo_bit + 31) / es;
    if (j1 > cnt - 1) j1 = cnt - 1;
    for (int j = j0; j <= j1; ++j) {
      const uint64_t q = jl_input<XT>(x, first + j, qp, clipped);
      const unsigned __int128 v = (unsigned __int128)q * weight;
      const int sh = es * j - lo_bit;
      w |= sh >= 0 ? (uint32_t)(v << sh) : (uint32_t)(v >> (-sh));
    }
  } else {
    // Negative weight (the reference accepts it: _secagg_crypter.py:106-112 only bounds its bit
    // length).  VES._batch ORs the slots (_jls.py:169-176): in two's complement the first
    // non-zero slot v_j* = q_j* w < 0 has all bits above its own set, so the packing is exactly
    // v_j* << (es j*) (0 if every q is 0).  Here pt = |v_j*| << (es j*); jl_nude_kernel makes the
    // digit of N*pt + 1 from it with the sign (kernel argument).
    const uint64_t aw = 0ull - weight;
    uint64_t qs = 0;
    int js = -1;
    for (int j = 0; j < cnt; ++j) {
      const uint64_t q = jl_input<XT>(x, first + j, qp, clipped);
      if (js < 0 && q != 0) {
        js = j;
        qs = q;
      }
    }
    if (js >= 0) {
      const unsigned __int128 v = (unsigned __int128)qs * aw;
      const int sh = es * js - lo_bit;
      w = sh >= 0 ? (sh < 32 ? (uint32_t)(v << sh) : 0u) : (-sh < 128 ? (uint32_t)(v >> (-sh)) : 0u);
    }
  }
  pt[ct * 32 + L] = w;
  flag_if_any(clipped, stats, FBM_WARN_CLIPPED);
}

// VES.encode of raw integers (JoyeLibert.protect / VES.encode on int lists, _jls.py:118-144,
// 169-176): values are (lo, hi) uint64 pairs, v < 2^128, ORed into slot j at bit es*j with the
// reference's OR semantics also for a value wider than its slot (its high bits land in the
// next slots).  Slot j reaches limb L (bits [32L, 32L+32)) iff es*j < 32L + 32 and
// es*j + 128 > 32L.  A bit at or above 2^1024 (only possible for a value wider than its slot
// in the last slots) flags FBM_ERR_PT_WIDE: outside the 1024-bit plaintext the device keeps.
__global__ void __launch_bounds__(256) jl_pack_wide_kernel(const uint64_t* __restrict__ x, uint64_t n, int es,
                                                           int cr, uint64_t n_ct, uint32_t* __restrict__ pt,
                                                           uint32_t* __restrict__ stats) {
  const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t ct = gid >> 5;
  const int L = (int)(gid & 31);
  if (ct >= n_ct) return;
  const uint64_t first = ct * (uint64_t)cr;
  const int cnt = (n - first) >= (uint64_t)cr ? cr : (int)(n - first);
  const int lo_bit = 32 * L;
  int j0 = lo_bit >= 128 ? (lo_bit - 128) / es + 1 : 0;
  int j1 = (lo_bit + 31) / es;
  if (j1 > cnt - 1) j1 = cnt - 1;
  uint32_t w = 0;
  for (int j = j0; j <= j1; ++j) {
    const unsigned __int128 v = ((unsigned __int128)x[2 * (first + j) + 1] << 64) | x[2 * (first + j)];
    const int sh = es * j - lo_bit;
    w |= sh >= 0 ? (uint32_t)(v << sh) : (uint32_t)(v >> (-sh));
  }
  pt[ct * 32 + L] = w;
  if (L == 31) {  // bits past 2^1024: slots with es*j + 128 > 1024
    bool wide = false;
    for (int j = 0; j < cnt; ++j) {
      if (es * j + 128 <= 1024) continue;
      const unsigned __int128 v = ((unsigned __int128)x[2 * (first + j) + 1] << 64) | x[2 * (first + j)];
      const int room = 1024 - es * j;  // bits of v that stay below 2^1024
      wide |= room <= 0 ? v != 0 : (v >> room) != 0;
    }
    if (wide) atomicOr(stats + FBM_STAT_ERRFLAGS, FBM_ERR_PT_WIDE);
  }
}

// VES objects of any shape (round 4; _jls.py:118-192 for element sizes above 100 bits, plaintexts wider
// than 1024 bits, values of any width): values as wv-word little-endian rows, plaintexts as pw-word rows.
// Bits [off, off + 32) of a w-word number (off may be negative: the number shifted up by -off).
__device__ __forceinline__ uint32_t bits32_at(const uint32_t* v, int w, int off) {
  if (off < 0) return -off < 32 && w > 0 ? v[0] << (-off) : 0u;
  const int i = off >> 5, b = off & 31;
  const uint32_t lo = i < w ? v[i] : 0u;
  const uint32_t hi = b && i + 1 < w ? v[i + 1] : 0u;
  return b ? (lo >> b) | (hi << (32 - b)) : lo;
}
// the same for a two's-complement value of w words: past its top word the sign bit repeats (Python's ints)
__device__ __forceinline__ uint32_t bits32_at_signed(const uint32_t* v, int w, int off) {
  const uint32_t ext = (v[w - 1] >> 31) ? ~0u : 0u;
  if (off < 0) return -off < 32 ? v[0] << (-off) : 0u;
  const int i = off >> 5, b = off & 31;
  const uint32_t lo = i < w ? v[i] : ext;
  const uint32_t hi = i + 1 < w ? v[i + 1] : ext;
  return b ? (lo >> b) | (hi << (32 - b)) : lo;
}
// encode: one thread per plaintext word; slot j's value ORed in at bit es j, its bits past the slot into
// the next slots (the reference's a |= v << es j).  sgn: the values are two's complement (ABI 4): a
// negative one's sign extends to the plaintext's top word, whose top bit then marks the plaintext negative
// (Python's OR of a negative int), and every lower slot can reach word L.
__global__ void __launch_bounds__(256) ves_pack_kernel(const uint32_t* __restrict__ x, uint64_t n, int wv, int es,
                                                       int cr, int pw, int sgn, uint64_t n_ct,
                                                       uint32_t* __restrict__ pt) {
  const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t ct = gid / (uint64_t)pw;
  const int L = (int)(gid % (uint64_t)pw);
  if (ct >= n_ct) return;
  const uint64_t first = ct * (uint64_t)cr;
  const int cnt = (n - first) >= (uint64_t)cr ? cr : (int)(n - first);
  const int64_t lo_bit = 32ll * L;
  int64_t j0 = !sgn && lo_bit - 32ll * wv + 1 > 0 ? (lo_bit - 32ll * wv + 1 + es - 1) / es : 0;
  int64_t j1 = (lo_bit + 31) / es;
  if (j1 > cnt - 1) j1 = cnt - 1;
  uint32_t w = 0;
  if (sgn) {
    for (int64_t j = j0; j <= j1; ++j)
      w |= bits32_at_signed(x + (first + j) * (uint64_t)wv, wv, (int)(lo_bit - es * j));
  } else {
    for (int64_t j = j0; j <= j1; ++j) w |= bits32_at(x + (first + j) * (uint64_t)wv, wv, (int)(lo_bit - es * j));
  }
  pt[ct * (uint64_t)pw + L] = w;
}
// decode: one thread per output word; value o = slot o % cr of plaintext o / cr, masked to es bits
__global__ void __launch_bounds__(256) ves_unpack_kernel(const uint32_t* __restrict__ pt, int pw, int es, int cr,
                                                         uint64_t n_out, int ow, uint32_t* __restrict__ vals) {
  const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t o = gid / (uint64_t)ow;
  const int w = (int)(gid % (uint64_t)ow);
  if (o >= n_out) return;
  const uint64_t ct = o / (uint64_t)cr;
  const int slot = (int)(o % (uint64_t)cr);
  uint32_t v = bits32_at(pt + ct * (uint64_t)pw, pw, es * slot + 32 * w);
  const int left = es - 32 * w;  // bits of the value in this word
  if (left < 32) v = left <= 0 ? 0u : v & ((1u << left) - 1u);
  vals[o * (uint64_t)ow + w] = v;
}

#define FBM_QMASK ((1u << FBM_QA_LB) - 1u)  // the 29-bit engines' limb mask

// radix changes between the shared final step's 28-bit limbs and the engines' 29-bit limbs
// (both normalised: every limb below its radix)
__device__ __forceinline__ void relimb_29_28(const uint32_t (&x)[FBM_QA_L], uint32_t (&o)[FBM_NLN]) {
#pragma unroll
  for (int j = 0; j < FBM_NLN; ++j) {
    const int bit = j * FBM_LB, k = bit / FBM_QA_LB, off = bit % FBM_QA_LB;
    const uint64_t v = ((uint64_t)(k + 1 < FBM_QA_L ? x[k + 1] : 0u) << FBM_QA_LB) | (k < FBM_QA_L ? x[k] : 0u);
    o[j] = (uint32_t)(v >> off) & FBM_LMASK;
  }
}
__device__ __forceinline__ void relimb_28_29(const uint32_t* x, uint32_t* o) {  // FBM_NLN -> FBM_QA_L limbs
#pragma unroll
  for (int k = 0; k < FBM_QA_L; ++k) {
    const int bit = k * FBM_QA_LB, j = bit / FBM_LB, off = bit % FBM_LB;
    const uint64_t v = ((uint64_t)(j + 1 < FBM_NLN ? x[j + 1] : 0u) << FBM_LB) | (j < FBM_NLN ? x[j] : 0u);
    o[k] = (uint32_t)(v >> off) & FBM_QMASK;
  }
}

// ------------------------------------------------------------------------------------
// nude = N*pt + 1 as the N-adic digit pair (1, pt)  ->  digit 1 only (digit 0 is the constant 1,
// which the engines take as immediates: fbm_na_mm_nude), [limb][ct] 29-bit limbs in the engines' B
// layout: rows 0..35, 256-ciphertext blocks FBM_NUDE_ROWS rows apart (the last operand of the
// exponentiation's encrypt, read in place by jl_exp_kernel; pt < 2^1036 < R is a valid one-off digit)
// ------------------------------------------------------------------------------------
// negative != 0 (a negative weight, see jl_pack_kernel): pt holds |pt| and N*pt + 1 is
// (1, M - |pt|) with M = N * 2^(1036 - bits(N)) = 0 (mod N): 2^1035 <= M < R, so the digit is
// non-negative and below R for every |pt| < 2^1024.
static_assert(FBM_NUDE_ROWS == FBM_NUDE_D1 + FBM_QA_L, "jl_nude_kernel stores digit 1's 29-bit limbs");
__global__ void __launch_bounds__(256) jl_nude_kernel(const uint32_t* __restrict__ pt, uint64_t n_ct, JlParams jp,
                                                      int negative, uint32_t* __restrict__ nude) {
  const uint64_t ct = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (ct >= n_ct) return;
  uint32_t p32[32];
  const uint4* src = reinterpret_cast<const uint4*>(pt + ct * 32);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint4 v = src[i];
    p32[4 * i] = v.x; p32[4 * i + 1] = v.y; p32[4 * i + 2] = v.z; p32[4 * i + 3] = v.w;
  }
  uint32_t p28[FBM_NLN];
  to28<32, FBM_NLN>(p32, p28);
  if (negative) {
    int32_t br = 0;
#pragma unroll
    for (int k = 0; k < FBM_NLN; ++k) {
      const int32_t v = (int32_t)jp.mneg[k] - (int32_t)p28[k] + br;
      p28[k] = (uint32_t)v & FBM_LMASK;
      br = v >> FBM_LB;
    }
  }
  // N*pt + 1 in N-adic digits is (1, pt): no arithmetic, only the layout of the
  // exponentiation's B operand (blocked column, 29-bit limbs of digit 1; 144 bytes per ciphertext)
  uint32_t p29[FBM_QA_L];
  relimb_28_29(p28, p29);
  uint32_t* dst = launder_v(nude + (ct >> 8) * (FBM_NUDE_ROWS * 256) + (ct & 255));
#ifdef FBM_NUDE_BOTH_DIGITS
#pragma unroll
  for (int k = 0; k < FBM_QA_L; ++k) dst[k * 256] = k == 0 ? 1u : 0u;
#endif
#pragma unroll
  for (int k = 0; k < FBM_QA_L; ++k) dst[(FBM_NUDE_D1 + k) * 256] = p29[k];
}

// ------------------------------------------------------------------------------------
// FDH
// ------------------------------------------------------------------------------------
// gcd(u, N) == 1 for u < 2^(32 W) (W limbs: 64 for the crypter's FDH, 120 for FDH objects of up to
// 4096 bits), N odd (<= 1024 bits).  Binary GCD, bounded.
template <int W>
__device__ bool gcd_is_one_w(uint32_t (&u)[W], const uint32_t* N32, uint32_t& err) {
  uint32_t v[W];
#pragma unroll
  for (int i = 0; i < W; ++i) v[i] = i < 32 ? N32[i] : 0u;
  uint32_t any = 0;
#pragma unroll
  for (int i = 0; i < W; ++i) any |= u[i];
  if (any) {
    int it = 0;
    for (; it < 20000; ++it) {
      // strip factors of two from u (N is odd, so they never divide the gcd)
      while (u[0] == 0u) {
#pragma unroll
        for (int i = 0; i < W - 1; ++i) u[i] = u[i + 1];
        u[W - 1] = 0u;
      }
      const int s = __builtin_ctz(u[0]);
      if (s) {
#pragma unroll
        for (int i = 0; i < W - 1; ++i) u[i] = (u[i] >> s) | (u[i + 1] << (32 - s));
        u[W - 1] >>= s;
      }
      int cmp = 0;
#pragma unroll
      for (int i = W - 1; i >= 0; --i)
        if (cmp == 0) cmp = (u[i] > v[i]) - (u[i] < v[i]);
      if (cmp == 0) break;
      if (cmp < 0) {
#pragma unroll
        for (int i = 0; i < W; ++i) {
          const uint32_t t = u[i];
          u[i] = v[i];
          v[i] = t;
        }
      }
      uint32_t br = 0;  // u -= v (u > v, both odd: result even and nonzero)
#pragma unroll
      for (int i = 0; i < W; ++i) {
        const uint64_t d = (uint64_t)u[i] - v[i] - br;
        u[i] = (uint32_t)d;
        br = (uint32_t)(d >> 63);
      }
    }
    if (it >= 20000) err |= FBM_ERR_ITER_CAP;
  }
  uint32_t rest = 0;
#pragma unroll
  for (int i = 1; i < W; ++i) rest |= v[i];
  return v[0] == 1u && rest == 0;
}

__device__ bool gcd_is_one(uint32_t (&u)[64], const uint32_t* N32, uint32_t& err) { return gcd_is_one_w<64>(u, N32, err); }

// gcd(r, N) == 1 for a one-digest r (8 limbs), N odd: the common case, far less work than
// the 64-limb binary gcd above.  Factors of two of r do not divide N, so they are stripped
// (v = r' odd); then t = N * 2^-1024 mod v by a word-serial Montgomery reduction of N by v
// (2^-1024 is a unit mod the odd v, so gcd(t, v) = gcd(N, v); 32 rows of 8 multiply-adds
// instead of 1024 shift-subtract steps of a bitwise N mod v), and a binary gcd of (t, v) on 8
// limbs.  r == 0 -> gcd = N >= 3 -> false (as the reference's math.gcd).  __host__ too: unit
// tested on the host through fbm_test_fdh_gcd (include/fbm_secagg.h).
__host__ __device__ inline bool gcd_is_one_r8(const uint32_t (&r)[8], const uint32_t* N32, uint32_t& err) {
  uint32_t v[8];
  uint32_t any = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    v[i] = r[i];
    any |= r[i];
  }
  if (!any) return false;
  while (v[0] == 0u) {
#pragma unroll
    for (int i = 0; i < 7; ++i) v[i] = v[i + 1];
    v[7] = 0u;
  }
  {
    const int sh = __builtin_ctz(v[0]);
    if (sh) {
#pragma unroll
      for (int i = 0; i < 7; ++i) v[i] = (v[i] >> sh) | (v[i + 1] << (32 - sh));
      v[7] >>= sh;
    }
  }
  // t = REDC_v(N) = (N + M v) / 2^1024 <= v  (M < 2^1024; N < 2^1024): a window of 8 words
  // plus a 64-bit top word slides over N one word per row.
  uint32_t vinv = v[0];  // Newton: v^-1 mod 2^32 (v odd)
#pragma unroll
  for (int i = 0; i < 5; ++i) vinv *= 2u - v[0] * vinv;
  const uint32_t vp = 0u - vinv;
  uint32_t w[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) w[i] = N32[i];
  uint64_t top = N32[8];
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    const uint32_t m = w[0] * vp;
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint64_t x = (uint64_t)w[j] + (uint64_t)m * v[j] + c;
      w[j] = (uint32_t)x;
      c = x >> 32;
    }
    top += c;  // w[0] is now 0: shift the window by one word
#pragma unroll
    for (int j = 0; j < 7; ++j) w[j] = w[j + 1];
    w[7] = (uint32_t)top;
    top = (top >> 32) + (i + 9 < 32 ? N32[i + 9] : 0u);
  }
  uint32_t t[8];  // t <= v < 2^256: the top word is 0
#pragma unroll
  for (int i = 0; i < 8; ++i) t[i] = w[i];
  // binary gcd(t, v), v odd
  uint32_t u[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) u[i] = t[i];
  int it = 0;
  for (; it < 4096; ++it) {
    uint32_t nz = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) nz |= u[i];
    if (!nz) break;
    while (u[0] == 0u) {
#pragma unroll
      for (int i = 0; i < 7; ++i) u[i] = u[i + 1];
      u[7] = 0u;
    }
    const int sh = __builtin_ctz(u[0]);
    if (sh) {
#pragma unroll
      for (int i = 0; i < 7; ++i) u[i] = (u[i] >> sh) | (u[i + 1] << (32 - sh));
      u[7] >>= sh;
    }
    int cmp = 0;
#pragma unroll
    for (int i = 7; i >= 0; --i)
      if (cmp == 0) cmp = (u[i] > v[i]) - (u[i] < v[i]);
    if (cmp < 0) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const uint32_t x = u[i];
        u[i] = v[i];
        v[i] = x;
      }
    }
    uint32_t br = 0;  // u -= v (both odd, u >= v)
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const uint64_t x = (uint64_t)u[i] - v[i] - br;
      u[i] = (uint32_t)x;
      br = (uint32_t)(x >> 63);
    }
  }
  if (it >= 4096) err |= FBM_ERR_ITER_CAP;
  uint32_t rest = 0;
#pragma unroll
  for (int i = 1; i < 8; ++i) rest |= v[i];
  return v[0] == 1u && rest == 0u;
}

// FDH.H(t_k): message = t.to_bytes(1024,'big') || counter (1 byte), t = (k << 512) | tau.  Blocks
// 0..13 hold the round's bits 1024..8191 (the same for every k < 2^64: a midstate from the host), block
// 14 its bits 512..1023 OR k, block 15 its bits 0..511,
// block 16 the counter byte + padding (length 8200 bits).  While gcd(r, N^2) != 1 the
// counter is bumped and r grows by one digest (r = D1 || D2 || ...).  r is tested with 1..7
// digests only: once 8 digests (256 bytes = bits_size // 8) are in, the reference's inner
// loop (_jls.py:746-755) never breaks again and counter.to_bytes(1) overflows at 256 -- its
// OverflowError, whatever gcd the 8-digest r would have.
//
// Two kernels: jl_fdh_kernel takes the first digest, which every ciphertext of a real biprime keeps
// (its gcd on 8 words, gcd_is_one_r8), in few registers; a ciphertext whose first digest is not coprime
// (small or even moduli) is marked in word 63 of its H row -- never nonzero in an r of at most 7 digests --
// and jl_fdh_retry_kernel redoes it with r of up to 7 digests (the 64-word gcd).  One kernel holding both
// paths took 256 VGPRs and ran one wave per SIMD.
__device__ __forceinline__ void fdh_state_after_t(const JlParams& jp, uint64_t k, uint32_t (&st)[8]) {
  uint32_t W[16];
#pragma unroll
  for (int i = 0; i < 8; ++i) st[i] = jp.mid[i];
#pragma unroll
  for (int i = 0; i < 16; ++i) W[i] = jp.tau14_w[i];  // block 14: the round's bits 512..1023, OR k
  W[14] |= (uint32_t)(k >> 32);
  W[15] |= (uint32_t)k;
  fbm_sha256_compress(st, W);
#pragma unroll
  for (int i = 0; i < 16; ++i) W[i] = jp.tau_w[i];  // block 15: the round's bits 0..511
  fbm_sha256_compress(st, W);
}
__device__ __forceinline__ void fdh_digest(const uint32_t (&st)[8], uint32_t c, uint32_t (&d)[8]) {
  uint32_t W[16];
#pragma unroll
  for (int i = 0; i < 8; ++i) d[i] = st[i];
#pragma unroll
  for (int i = 0; i < 16; ++i) W[i] = 0u;
  W[0] = (c << 24) | (0x80u << 16);
  W[15] = 8200u;
  fbm_sha256_compress(d, W);
}
constexpr uint32_t FBM_FDH_RETRY = ~0u;  // word 63 of an H row: the first digest was not coprime

__global__ void __launch_bounds__(256) jl_fdh_kernel(uint64_t n_ct, JlParams jp, uint32_t* __restrict__ H,
                                                     uint32_t* __restrict__ stats, uint32_t* __restrict__ Hc) {
  const uint64_t kl = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (kl >= n_ct) return;
  uint32_t err = 0, st[8], d[8], r8[8];
  fdh_state_after_t(jp, kl + jp.ct_offset, st);
  fdh_digest(st, 1u, d);
#pragma unroll
  for (int i = 0; i < 8; ++i) r8[i] = d[7 - i];  // r = D1 as 8 little-endian limbs
  const bool ok = !(jp.fdh_even && !(r8[0] & 1u)) && gcd_is_one_r8(r8, jp.N32, err);  // even 2^s N: r odd too
  if (err) atomicOr(stats + FBM_STAT_ERRFLAGS, err);
  uint4* o = reinterpret_cast<uint4*>(H + kl * 64);
  if (!ok) {  // the retry kernel writes the whole row (and the compact row's sentinel stays)
    if (Hc) {
      uint4* c = reinterpret_cast<uint4*>(Hc + kl * 8);
      c[0] = c[1] = make_uint4(~0u, ~0u, ~0u, ~0u);
    }
    o[15] = make_uint4(0u, 0u, 0u, FBM_FDH_RETRY);
    return;
  }
  if (Hc) {  // compact: 32 bytes per ciphertext, the whole row only behind the sentinel
    uint32_t ones = ~0u;
#pragma unroll
    for (int i = 0; i < 8; ++i) ones &= r8[i];
    const bool full = ones == ~0u;  // (a one-digest r of all ones takes the sentinel)
    uint4* c = reinterpret_cast<uint4*>(Hc + kl * 8);
    c[0] = full ? make_uint4(~0u, ~0u, ~0u, ~0u) : make_uint4(r8[0], r8[1], r8[2], r8[3]);
    c[1] = full ? make_uint4(~0u, ~0u, ~0u, ~0u) : make_uint4(r8[4], r8[5], r8[6], r8[7]);
    if (!full) return;
  }
  o[0] = make_uint4(r8[0], r8[1], r8[2], r8[3]);
  o[1] = make_uint4(r8[4], r8[5], r8[6], r8[7]);
#pragma unroll
  for (int i = 2; i < 16; ++i) o[i] = make_uint4(0u, 0u, 0u, 0u);
}

// The ciphertexts jl_fdh_kernel marked: r of 2 .. 7 digests (_jls.py:746-762), the whole H row.
// With compact rows only a sentinel row can be marked (the H rows behind other compact rows are not
// written by this call: their word 63 is not looked at).
__global__ void __launch_bounds__(64) jl_fdh_retry_kernel(uint64_t n_ct, JlParams jp, uint32_t* __restrict__ H,
                                                          uint32_t* __restrict__ stats, const uint32_t* __restrict__ Hc) {
  const uint64_t kl = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (kl >= n_ct) return;
  if (Hc) {
    const uint4 a = reinterpret_cast<const uint4*>(Hc + kl * 8)[0];
    if ((a.x & a.y & a.z & a.w) != ~0u) return;
  }
  if (H[kl * 64 + 63] != FBM_FDH_RETRY) return;
  uint32_t err = 0, st[8];
  fdh_state_after_t(jp, kl + jp.ct_offset, st);
  uint32_t r[64];
#pragma unroll
  for (int i = 0; i < 64; ++i) r[i] = 0u;
  bool ok = false;
  for (uint32_t c = 1; c <= 7 && !ok; ++c) {
    uint32_t d[8];
    fdh_digest(st, c, d);
#pragma unroll
    for (int i = 63; i >= 8; --i) r[i] = r[i - 8];
#pragma unroll
    for (int i = 0; i < 8; ++i) r[i] = d[7 - i];
    if (jp.fdh_even && !(r[0] & 1u)) {  // an even modulus 2^s N: gcd = 1 needs r odd too
      ok = false;
    } else if (c == 1) {  // one digest: r = d (8 limbs)
      uint32_t r8[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) r8[i] = r[i];
      ok = gcd_is_one_r8(r8, jp.N32, err);
    } else {       // retries (only reachable for moduli with small factors)
      uint32_t u[64];
#pragma unroll
      for (int i = 0; i < 64; ++i) u[i] = r[i];
      ok = gcd_is_one(u, jp.N32, err);
    }
  }
  if (!ok) err |= FBM_ERR_FDH_OVERFLOW;
  if (err) atomicOr(stats + FBM_STAT_ERRFLAGS, err);
  uint4* o = reinterpret_cast<uint4*>(H + kl * 64);
#pragma unroll
  for (int i = 0; i < 16; ++i) o[i] = make_uint4(r[4 * i], r[4 * i + 1], r[4 * i + 2], r[4 * i + 3]);
}

// ciphertext ct's H row (64 words) from the compact rows Hc (launch_jl_fdh) or, behind the sentinel / with
// no compact rows, from H
__device__ __forceinline__ void load_h(const uint32_t* H, const uint32_t* Hc, uint64_t ct, uint32_t (&h)[64]) {
  if (Hc) {  // (uniform)
    const uint4* c = reinterpret_cast<const uint4*>(Hc + ct * 8);
    const uint4 a = c[0], b = c[1];
    const bool full = (a.x & a.y & a.z & a.w & b.x & b.y & b.z & b.w) == ~0u;
    h[0] = a.x; h[1] = a.y; h[2] = a.z; h[3] = a.w; h[4] = b.x; h[5] = b.y; h[6] = b.z; h[7] = b.w;
#pragma unroll
    for (int i = 8; i < 64; ++i) h[i] = 0u;
    if (__any(full)) {  // wave-uniform (FDH retries: small moduli only): whole rows behind the sentinel
      const uint4* s = reinterpret_cast<const uint4*>(H + ct * 64);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const uint4 v = s[i];
        h[4 * i] = full ? v.x : h[4 * i];
        h[4 * i + 1] = full ? v.y : h[4 * i + 1];
        h[4 * i + 2] = full ? v.z : h[4 * i + 2];
        h[4 * i + 3] = full ? v.w : h[4 * i + 3];
      }
    }
    return;
  }
  const uint4* s = reinterpret_cast<const uint4*>(H + ct * 64);
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const uint4 v = s[i];
    h[4 * i] = v.x; h[4 * i + 1] = v.y; h[4 * i + 2] = v.z; h[4 * i + 3] = v.w;
  }
}

// FDH.H of any bits_size (_jls.py:742-762), for FDH objects other than the crypter's FDH(2048, N^2): the
// message is t.to_bytes(L, 'big') || counter (L = bits_size // 2 bytes), r the digests so far
// concatenated (r = D1 || D2 || ...), at most kmax of them -- the reference's inner loop stops breaking
// once r holds bits_size // 8 bytes and its counter byte then overflows.  One lane per t: the blocks of
// t bytes alone are hashed once, the one or two tail blocks (t's last bytes, the counter, the padding and
// the length) per counter.  r is kept to 15 digests (120 words: every r an FDH of up to 4096 bits can
// take); a bits_size that would let the reference try a 16th reports FBM_ERR_FDH_WIDE instead of guessing.
struct FdhModArg {
  uint32_t n32[32];  // the modulus's odd part (of M or of sqrt(M)), 32 limbs
  int even;          // M even: a coprime r must be odd as well
};
__device__ __forceinline__ uint32_t fdh_msg_byte(const uint32_t* t, int L, int i) {  // byte i of t.to_bytes(L)
  const int j = L - 1 - i;
  return (t[j >> 2] >> (8 * (j & 3))) & 0xFFu;
}
// SHA-256 state after the F blocks made of t's bytes alone (shared by every counter)
__device__ __noinline__ void fdh_msg_prefix(const uint32_t* tr, int L, int F, uint32_t (&st)[8]) {
  uint32_t W[16];
  fbm_sha256_init(st);
#pragma unroll 1
  for (int b = 0; b < F; ++b) {
#pragma unroll 1
    for (int j = 0; j < 16; ++j) {
      uint32_t w = 0;
      for (int q = 0; q < 4; ++q) w = (w << 8) | fdh_msg_byte(tr, L, 64 * b + 4 * j + q);
      W[j] = w;
    }
    fbm_sha256_compress(st, W);
  }
}
// digest of counter c: the prefix state, then the tail blocks (t's last bytes, c, 0x80, the 64-bit length)
__device__ __noinline__ void fdh_msg_digest(const uint32_t (&st)[8], const uint32_t* tr, int L, int F, int rem, int nb,
                                            uint64_t len_bits, int c, uint32_t (&d)[8]) {
  uint32_t W[16];
#pragma unroll
  for (int i = 0; i < 8; ++i) d[i] = st[i];
#pragma unroll 1
  for (int b = 0; b < nb; ++b) {
#pragma unroll 1
    for (int j = 0; j < 16; ++j) {
      uint32_t w = 0;
      for (int q = 0; q < 4; ++q) {
        const int p = 64 * b + 4 * j + q;
        uint32_t v = 0;
        if (p < rem) v = fdh_msg_byte(tr, L, 64 * F + p);
        else if (p == rem) v = (uint32_t)c;
        else if (p == rem + 1) v = 0x80u;
        else if (p >= 64 * nb - 8) v = (uint32_t)(len_bits >> (8 * (64 * nb - 1 - p))) & 0xFFu;
        w = (w << 8) | v;
      }
      W[j] = w;
    }
    fbm_sha256_compress(d, W);
  }
}
__global__ void __launch_bounds__(64) jl_fdh_msg_kernel(uint64_t n, const uint32_t* __restrict__ t, int tw, int L,
                                                        int kmax, FdhModArg m, uint32_t* __restrict__ H,
                                                        uint32_t* __restrict__ stats) {
  const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const uint32_t* tr = t + k * (uint64_t)tw;
  uint32_t st[8];
  const int F = L / 64;                          // blocks of t bytes only: the same for every counter
  fdh_msg_prefix(tr, L, F, st);
  const int rem = L - 64 * F;                    // t bytes left for the tail
  const int nb = (rem + 1 + 1 + 8 + 63) / 64;    // + counter, 0x80, 64-bit length: 1 or 2 blocks
  const uint64_t len_bits = 8ull * (uint64_t)(L + 1);
  uint32_t r[FBM_FDH_MSG_WORDS];
#pragma unroll
  for (int i = 0; i < FBM_FDH_MSG_WORDS; ++i) r[i] = 0u;
  uint32_t err = 0;
  bool ok = false;
  const int kuse = kmax < FBM_FDH_MSG_DIGESTS ? kmax : FBM_FDH_MSG_DIGESTS;
#pragma unroll 1
  for (int c = 1; c <= kuse && !ok; ++c) {
    uint32_t d[8];
    fdh_msg_digest(st, tr, L, F, rem, nb, len_bits, c, d);
#pragma unroll 1
    for (int i = FBM_FDH_MSG_WORDS - 1; i >= 8; --i) r[i] = r[i - 8];
#pragma unroll
    for (int i = 0; i < 8; ++i) r[i] = d[7 - i];
    if (m.even && !(r[0] & 1u)) {
      ok = false;
    } else if (c == 1) {
      uint32_t r8[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) r8[i] = r[i];
      ok = gcd_is_one_r8(r8, m.n32, err);
    } else {
      uint32_t u[FBM_FDH_MSG_WORDS];
#pragma unroll 1
      for (int i = 0; i < FBM_FDH_MSG_WORDS; ++i) u[i] = r[i];
      ok = gcd_is_one_w<FBM_FDH_MSG_WORDS>(u, m.n32, err);
    }
  }
  if (!ok) err |= FBM_ERR_FDH_OVERFLOW;  // (kmax <= FBM_FDH_MSG_DIGESTS here: wider FDHs take the wide kernel)
  uint32_t* o = H + k * FBM_FDH_MSG_ROW;
#pragma unroll 1
  for (int i = 0; i < FBM_FDH_MSG_ROW; ++i) o[i] = i < FBM_FDH_MSG_WORDS ? r[i] : 0u;
  if (err) atomicOr(stats + FBM_STAT_ERRFLAGS, err);
}

// FDH.H of bits_size > 4096 (round 5): r may need 16 .. 255 digests (the counter byte caps it at 255), too
// wide for registers.  Each digest goes to the output row as it is made (block c - 1, digest order; the
// blocks are reversed into r's little-endian word order at the end), and coprimality is decided on
// y = r R mod m (R = 2^1024, m the modulus's odd part, a unit factor that leaves gcd(r, m) alone), kept as
// r grows: y <- y 2^256 + D R = mont(y, K1) + mont(D, K2), K1 = 2^256 R, K2 = R^2 (mod m), then a 32-word
// binary gcd of (y, m).  An even M also needs r odd: the last digest's low bit.
struct FdhWideArg {
  uint32_t m[32], k1[32], k2[32];
  uint32_t mp;  // -m^-1 mod 2^32
  int even;
};
// a b R^-1 mod m, a < R, b < m: CIOS over 32 words, result < m
__device__ __noinline__ void fdh_mont32(const uint32_t (&a)[32], const uint32_t* b, const FdhWideArg& w,
                                        uint32_t (&o)[32]) {
  uint32_t t[34];
#pragma unroll
  for (int j = 0; j < 34; ++j) t[j] = 0u;
#pragma unroll 1
  for (int i = 0; i < 32; ++i) {
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < 32; ++j) {
      const uint64_t v = (uint64_t)a[j] * b[i] + t[j] + c;
      t[j] = (uint32_t)v;
      c = v >> 32;
    }
    uint64_t v = (uint64_t)t[32] + c;
    t[32] = (uint32_t)v;
    t[33] = (uint32_t)(v >> 32);
    const uint32_t q = t[0] * w.mp;
    c = ((uint64_t)q * w.m[0] + t[0]) >> 32;
#pragma unroll
    for (int j = 1; j < 32; ++j) {
      const uint64_t x = (uint64_t)q * w.m[j] + t[j] + c;
      t[j - 1] = (uint32_t)x;
      c = x >> 32;
    }
    v = (uint64_t)t[32] + c;
    t[31] = (uint32_t)v;
    t[32] = t[33] + (uint32_t)(v >> 32);
  }
  // t < 2m: subtract m once if t >= m
  uint32_t s[32], br = 0;
#pragma unroll
  for (int j = 0; j < 32; ++j) {
    const uint64_t d = (uint64_t)t[j] - w.m[j] - br;
    s[j] = (uint32_t)d;
    br = (uint32_t)(d >> 63);
  }
  const bool ge = t[32] || !br;
#pragma unroll
  for (int j = 0; j < 32; ++j) o[j] = ge ? s[j] : t[j];
}

__global__ void __launch_bounds__(64) jl_fdh_msg_wide_kernel(uint64_t n, const uint32_t* __restrict__ t, int tw, int L,
                                                             int kmax, FdhWideArg w, uint32_t* __restrict__ H, int hw,
                                                             uint32_t* __restrict__ stats) {
  const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const uint32_t* tr = t + k * (uint64_t)tw;
  uint32_t st[8];
  const int F = L / 64;
  fdh_msg_prefix(tr, L, F, st);
  const int rem = L - 64 * F;
  const int nb = (rem + 1 + 1 + 8 + 63) / 64;
  const uint64_t len_bits = 8ull * (uint64_t)(L + 1);
  const int kuse = kmax < 255 ? kmax : 255;  // counter.to_bytes(1) overflows at 256
  uint32_t* o = H + k * (uint64_t)hw;
  uint32_t y[32], err = 0;
#pragma unroll
  for (int i = 0; i < 32; ++i) y[i] = 0u;
  bool ok = false;
  int c = 0;
#pragma unroll 1
  while (!ok && c < kuse) {
    ++c;
    uint32_t d[8];
    fdh_msg_digest(st, tr, L, F, rem, nb, len_bits, c, d);
    uint32_t D[32], a[32], b[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) D[i] = i < 8 ? d[7 - i] : 0u;
#pragma unroll
    for (int i = 0; i < 8; ++i) o[8 * (c - 1) + i] = D[i];
    fdh_mont32(y, w.k1, w, a);  // y 2^256
    fdh_mont32(D, w.k2, w, b);  // D R
    uint32_t s[32], br = 0;
    uint64_t cy = 0;
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      const uint64_t v = (uint64_t)a[i] + b[i] + cy;
      y[i] = (uint32_t)v;
      cy = v >> 32;
    }
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      const uint64_t v = (uint64_t)y[i] - w.m[i] - br;
      s[i] = (uint32_t)v;
      br = (uint32_t)(v >> 63);
    }
    const bool ge = cy || !br;
#pragma unroll
    for (int i = 0; i < 32; ++i) y[i] = ge ? s[i] : y[i];
    if (w.even && !(D[0] & 1u)) continue;
    uint32_t u[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) u[i] = y[i];
    ok = gcd_is_one_w<32>(u, w.m, err);
  }
  if (!ok) err |= FBM_ERR_FDH_OVERFLOW;
  // r = D_1 || ... || D_c: D_c is the least significant block -- reverse the blocks written in digest order
#pragma unroll 1
  for (int j = 0; j < c / 2; ++j)
#pragma unroll 1
    for (int i = 0; i < 8; ++i) {
      const uint32_t x = o[8 * j + i];
      o[8 * j + i] = o[8 * (c - 1 - j) + i];
      o[8 * (c - 1 - j) + i] = x;
    }
#pragma unroll 1
  for (int i = 8 * c; i < hw; ++i) o[i] = 0u;
  if (err) atomicOr(stats + FBM_STAT_ERRFLAGS, err);
}

// ------------------------------------------------------------------------------------
// exponentiation engine
// ------------------------------------------------------------------------------------
// per-lane exponent table: workgroup-blocked, entry e / limb k at tb[(e * NL + k) * 256]
__device__ __forceinline__ void tbl_store(uint32_t* tb, int e, const uint32_t (&v)[FBM_NL]) {
  col_store(tb + e * (FBM_NL * 256), v);
}
__device__ __forceinline__ void tbl_load(const uint32_t* tb, int e, uint32_t (&v)[FBM_NL]) {
  col_load(tb + e * (FBM_NL * 256), v);
}
__device__ __forceinline__ void load_row64(const uint32_t* p, uint32_t (&w)[64]) {
  const uint4* s = reinterpret_cast<const uint4*>(launder_v(p));
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const uint4 v = s[i];
    w[4 * i] = v.x; w[4 * i + 1] = v.y; w[4 * i + 2] = v.z; w[4 * i + 3] = v.w;
  }
}
__device__ __forceinline__ void load_row32(const uint4* s, uint32_t (&w)[32]) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint4 v = s[i];
    w[4 * i] = v.x; w[4 * i + 1] = v.y; w[4 * i + 2] = v.z; w[4 * i + 3] = v.w;
  }
}
__device__ __forceinline__ void store_row64(uint32_t* p, const uint32_t (&w)[64]) {
  uint4* o = reinterpret_cast<uint4*>(launder_v(p));
#pragma unroll
  for (int i = 0; i < 16; ++i) o[i] = make_uint4(w[4 * i], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]);
}

// ------------------------------------------------------------------------------------
// The two hot kernels below run on the assembly Montgomery product (fbm_mont_asm.hpp):
// the running residue lives in the lane's LDS column (75 limb rows, 2 workgroups/CU =
// 2 waves/SIMD), B operands come from that column (squaring) or from workgroup-blocked
// global columns (table entries, nude, scratch, broadcast constants).  Everything around
// the products is wave-uniform.
// ------------------------------------------------------------------------------------
typedef __attribute__((address_space(3))) uint32_t lds_u32;
__device__ __forceinline__ uint32_t lds_addr(uint32_t* p) { return (uint32_t)(uintptr_t)(lds_u32*)p; }

// LDS column <-> workgroup-blocked global column (limb stride 256 words)
__device__ __forceinline__ void lds_to_glb(const uint32_t* lds, uint32_t* g) {
  uint32_t v[FBM_NL];
  lds_load_col(lds, FBM_BLOCK, v);
  col_store(g, v);
}
__device__ __forceinline__ void glb_to_lds(const uint32_t* g, uint32_t* lds) {
  uint32_t v[FBM_NL];
  col_load(g, v);
  lds_store_col(lds, FBM_BLOCK, v);
}

// x <- x - n if x >= n (28-bit limbs, branch-free); returns whether it subtracted
template <int L>
__device__ __forceinline__ uint32_t csub28(uint32_t (&x)[L], const uint32_t (&n)[L]) {
  uint32_t d[L];
  int32_t br = 0;
#pragma unroll
  for (int k = 0; k < L; ++k) {
    const int32_t v = (int32_t)x[k] - (int32_t)n[k] + br;
    d[k] = (uint32_t)v & FBM_LMASK;
    br = v >> FBM_LB;
  }
  const uint32_t ge = br == 0;
#pragma unroll
  for (int k = 0; k < L; ++k) x[k] = ge ? d[k] : x[k];
  return ge;
}

// N-adic result (t, s) in the lane's LDS column (t < N + 1, s < 2N: the last product of
// the exponentiation has a (1, .) operand) -> the canonical residue V = t + s N < N^2,
// 64 words, or (nadic_out) its reduced digits (V mod N | V div N), 32 words each.
// NK: the engine's constants block (N limbs at words 0..9, 16..42).
__device__ __forceinline__ void na_final_digits(uint32_t (&t)[FBM_NLN], uint32_t (&sd)[FBM_NLN], const uint32_t* NK,
                                                uint32_t (&w)[64], int nadic_out = 0) {
  const uint32_t* nk = launder_s(NK);
  uint32_t n[FBM_NLN];
#pragma unroll
  for (int j = 0; j < FBM_NLN; ++j) n[j] = j < 10 ? nk[j] : nk[6 + j];
  // t + s N = (t mod N) + N (s + [t >= N])  ->  reduce s + carry mod N
  uint32_t cy = csub28(t, n);
  cy += csub28(t, n);  // (a second one only matters for digits >= 2N: none here, kept cheap)
#pragma unroll
  for (int k = 0; k < FBM_NLN; ++k) {
    const uint32_t v = sd[k] + cy;
    sd[k] = v & FBM_LMASK;
    cy = v >> FBM_LB;
  }
  csub28(sd, n);
  csub28(sd, n);
  csub28(sd, n);
  if (nadic_out) {  // the digits themselves (the inverse's input: no division by N needed)
    uint32_t d0[32], d1[32];
    from28<FBM_NLN, 32>(t, d0);
    from28<FBM_NLN, 32>(sd, d1);
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      w[i] = d0[i];
      w[32 + i] = d1[i];
    }
    return;
  }
  // V = t + s N by columns (each < 37 products < 2^56 + t limb + carry)
  uint32_t v28[FBM_NL];
  uint64_t carry = 0;
#pragma unroll
  for (int k = 0; k < FBM_NL; ++k) {
    uint64_t acc = carry + (k < FBM_NLN ? t[k] : 0u);
#pragma unroll
    for (int i = (k < FBM_NLN ? 0 : k - FBM_NLN + 1); i <= (k < FBM_NLN ? k : FBM_NLN - 1); ++i)
      acc += (uint64_t)n[i] * sd[k - i];
    v28[k] = (uint32_t)acc & FBM_LMASK;
    carry = acc >> FBM_LB;
  }
  from28<FBM_NL, 64>(v28, w);
}


// a 64-word (2048-bit) row -> its 72 29-bit limbs (h_lo, h_hi): h = h_lo + h_hi 2^1044
__device__ __forceinline__ void to29_row64(const uint32_t (&w)[64], uint32_t (&o)[2 * FBM_QA_L]) {
#pragma unroll
  for (int k = 0; k < 2 * FBM_QA_L; ++k) {
    const int bit = k * FBM_QA_LB, wi = bit >> 5, sh = bit & 31;
    const uint64_t v = ((uint64_t)(wi + 1 < 64 ? w[wi + 1] : 0u) << 32) | (wi < 64 ? w[wi] : 0u);
    o[k] = (uint32_t)(v >> sh) & FBM_QMASK;
  }
}

// the one-lane engine's result (normalised 29-bit digits in the lane's LDS column) -> na_final_digits
__device__ __forceinline__ void na_final(const uint32_t* lds, const uint32_t* NK, uint32_t (&w)[64], int nadic_out) {
  uint32_t t29[FBM_QA_L], s29[FBM_QA_L];
#pragma unroll
  for (int k = 0; k < FBM_QA_L; ++k) {
    t29[k] = lds[k * FBM_BLOCK];
    s29[k] = lds[(FBM_QA_L + k) * FBM_BLOCK];
  }
  uint32_t t[FBM_NLN], sd[FBM_NLN];
  relimb_29_28(t29, t);
  relimb_29_28(s29, sd);
  na_final_digits(t, sd, NK, w, nadic_out);
}

// mode 0 (ENC): out[ct] = nude[ct] * H[ct]^key  mod N^2          (ciphertext)
// mode 1 (DEC): out[ct] = H[ct]^key mod N^2 (plain)                (for the inverse)
// | FBM_EXP_OUT_NADIC: out rows hold the result's digits (v mod N, v div N) (jl_lift_kernel)
// N-adic engine (fbm_nadic_asm.hpp): a residue is the digit pair (x0, x1), X = x0 + x1 N,
// 72 limbs = 2 x 36 of 29 bits in the same blocked columns (entries keep the 74-row stride).  Sliding window (width FBM_WIN,
// FBM_TABLE odd powers) over the device copy of the host-built schedule.  Per-lane table:
// FBM_TENTRIES blocked columns (the last = h / h^2 scratch).
//   a = R^2 (uniform, N-adic digits), b = (h, 0)  -> h*R              -> table[0]
//   a = h*R,  squared                              -> h^2*R            -> table[16]
//   a = h^(2t-1)*R, b = table[16]                  -> h^(2t+1)*R       -> table[t], t = 1..15
//   a = table[first], then per op: nsq squarings, one product with table[idx]
//   a = acc,  b = nude = (1, pt) | 1 = (1, 0)      -> c | h^key (digits) -> t + s N -> out
// h < R = 2^1044 (one FDH digest: always, for a 1024-bit N) IS the digit pair (h, 0); a wider h
// (FDH retries, small moduli) enters as h_lo R + h_hi R^2 (one more product, that wave only).
// Lanes past n_ct (last chunk) redo the last ciphertext and store nothing.
//
// BATCH: one launch over several SEGMENTS (the exponentiations of several parties' encrypts and
// the decryption factor, same biprime; JlExpSeg table in device memory): the chunks of all
// segments are pulled from one counter, so the launch packs the chip's rounds whatever the
// segments' sizes.  A chunk never spans two segments.  A segment's fields are re-read from the
// table (scalar values) where they are used rather than held across the products, as the plain
// kernel's arguments are.
template <typename T>
__device__ __forceinline__ T uniform_val(T v) {  // a wave-uniform value as a scalar (SGPR) value
  if constexpr (sizeof(T) == 8) {
    uint64_t u;
    __builtin_memcpy(&u, &v, 8);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)u);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(u >> 32));
    u = ((uint64_t)hi << 32) | (uint64_t)lo;  // (readfirstlane returns int: no sign extension)
    __builtin_memcpy(&v, &u, 8);
    return v;
  } else {
    return (T)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
  }
}

template <bool BATCH>
__global__ void __launch_bounds__(FBM_BLOCK, 2) jl_exp_kernel(const uint32_t* __restrict__ H_a, uint64_t n_ct_a,
                                                             uint32_t* __restrict__ cst, uint32_t np,
                                                             const uint32_t* __restrict__ ops_a, int n_ops_a,
                                                             int first_a, int mode_a, int key_is_zero_a,
                                                             int sbits_a, const uint32_t* __restrict__ nude_a,
                                                             uint32_t* __restrict__ table,
                                                             uint32_t* __restrict__ out_a,
                                                             const JlExpSeg* __restrict__ segs, int nseg,
                                                             uint32_t total_chunks, uint32_t* __restrict__ ctr,
                                                             const uint32_t* __restrict__ Hc_a) {
  __shared__ uint32_t lds_a[(FBM_NL + 1) * FBM_BLOCK];
  __shared__ uint32_t chunk_s;
  const int tid = threadIdx.x;
  uint32_t* lds = lds_a + tid;
  const uint32_t aoff = lds_addr(lds);
  const uint32_t* NK = cst + FBM_CST_NA29;
  // LDS row FBM_NL (no product touches it; the chunk loop's first barrier orders the writes before
  // any read): words 0..71 the short-base product's initial s pairs (D'_j, 0), D'_j = D_j + (2^29 - 1)
  // [j < 9] + [j == 0] (fbm_na_ms_reg: the rows' 2^29 - 1 - q_i folded in); words 72..143 the square's
  // (2^29 - 1 + P'_j, 0) (fbm_na_sq_lds)
  const uint32_t doff = lds_addr(lds_a + FBM_NL * FBM_BLOCK);
  const uint32_t koff = doff + 72u * 4u;
  if (tid < 72) {
    uint32_t v = launder_s(cst)[FBM_CST_QD + tid];
    if (!(tid & 1)) v += ((tid >> 1) < FBM_NA_SHORT_LIMBS ? FBM_QMASK : 0u) + (tid == 0 ? 1u : 0u);
    lds_a[FBM_NL * FBM_BLOCK + tid] = v;
  } else if (tid < 144) {
    lds_a[FBM_NL * FBM_BLOCK + tid] = launder_s(cst)[FBM_CST_QP + tid - 72];
  }
  constexpr int NA = FBM_NA_LIMBS;
  static_assert(NA == FBM_QA_L && FBM_NA_LIMB_BITS == FBM_QA_LB && 2 * NA <= FBM_NL, "one-lane engine limbs");
  // byte offset of this lane's table entry 0 (entries FBM_NL*256 words apart)
  const uint32_t tb0 = (uint32_t)(((uint64_t)blockIdx.x * FBM_TENTRIES * FBM_NL * FBM_BLOCK + tid) * 4);
  const uint32_t tstride = FBM_NL * FBM_BLOCK * 4;
  const uint32_t n_chunks = BATCH ? total_chunks : (uint32_t)((n_ct_a + FBM_BLOCK - 1) / FBM_BLOCK);
  uint32_t* counter = BATCH ? ctr : cst + FBM_CST_CTR;
  // Persistent workgroups pull 256-ciphertext chunks from a counter (zeroed by
  // jl_setup_kernel / before the batch launch): a workgroup leaves as soon as the chunks run
  // out, so the tail of one launch leaves CUs free for a concurrent launch on another stream
  // (the parties' encrypts), instead of every workgroup idling through a partial last round.
#pragma unroll 1
  for (;;) {
    if (tid == 0) chunk_s = atomicAdd(counter, 1u);
    __syncthreads();
    const uint32_t chunk = __builtin_amdgcn_readfirstlane(chunk_s);
    __syncthreads();
    if (chunk >= n_chunks) break;
    int si = 0;
    if (BATCH) {
#pragma unroll 1
      for (int i = 1; i < nseg; ++i)
        if (chunk >= uniform_val(segs[i].chunk0)) si = i;
      si = __builtin_amdgcn_readfirstlane(si);
    }
#define SEG(f, a) (BATCH ? uniform_val(launder_s(segs)[si].f) : a)
    const uint64_t n_ct = SEG(n_ct, n_ct_a);
    const uint64_t ct_raw = (uint64_t)(chunk - (BATCH ? uniform_val(segs[si].chunk0) : 0u)) * FBM_BLOCK + tid;
    const bool valid = ct_raw < n_ct;
    const uint64_t ct = valid ? ct_raw : n_ct - 1;
    bool wide = false, shortp = false;
    const int sbits = SEG(sbits, sbits_a);
    uint32_t hs[FBM_NA_SHORT_LIMBS];  // the short path's h: its 9 limbs, in registers for the whole chain
    {  // h -> 29-bit limbs -> (table path) scratch entry 16
      uint32_t h[64];
      if (SEG(key_is_zero, key_is_zero_a)) {
#pragma unroll
        for (int i = 0; i < 64; ++i) h[i] = i == 0 ? 1u : 0u;
      } else {
#ifdef FBM_EXP_FULL_H_LOAD  // (A/B variant: the round-3 whole-row load)
        load_row64(SEG(H, H_a) + ct * 64, h);
#else
        load_h(SEG(H, H_a), SEG(Hc, Hc_a), ct, h);
#endif
      }
      uint32_t h29[2 * NA];
      {  // h = h_lo + h_hi R: the 72-limb decomposition is (h_lo, h_hi)
        to29_row64(h, h29);
        uint32_t hi = 0, mid = 0;
#pragma unroll
        for (int k = NA; k < 2 * NA; ++k) hi |= h29[k];
#pragma unroll
        for (int k = FBM_NA_SHORT_LIMBS; k < NA; ++k) mid |= h29[k];
        wide = hi != 0u;
        // the short path (binary chain, short-base products): every lane's h below 2^261 -- one
        // FDH digest, always for a 1024-bit N -- and a schedule for it (sbits >= 0: N > 2^262, key != 0)
        shortp = sbits >= 0 && !SEG(key_is_zero, key_is_zero_a) && !__any(wide || mid != 0u);
#pragma unroll
        for (int k = 0; k < FBM_NA_SHORT_LIMBS; ++k) hs[k] = h29[k];
        if (shortp) lds_store_col(lds, FBM_BLOCK, h29);  // A = (h, 0), raw (no Montgomery form)
        if (wide) {  // FDH retries (small moduli only): h_hi R^2 = (h_hi, 0) * R^3 R^-1 -> entry 1
#pragma unroll
          for (int k = 0; k < NA; ++k) {
            h29[k] = h29[NA + k];
            h29[NA + k] = 0u;
          }
        }
      }
      if (!shortp) col_store(table + (tb0 + FBM_TSCRATCH * tstride) / 4, h29);
    }
    if (shortp) {
      // left-to-right binary over |key| below its top bit: a squaring per bit, a short-base
      // product (x h 2^-261) per 1 bit, then C = 2^f R^2 (host-built, ops buffer) turns the
      // chain's h^|key| 2^-f into h^|key| R -- 1 305 multiplies per 1 bit instead of a window
      // table's 31 + ~293 general products of 6 584 and its per-lane table traffic
      const uint32_t* kw = SEG(ops, ops_a) + FBM_OPS_KW;
      uint32_t w = 0;
#pragma unroll 1
      for (int j = sbits - 1; j >= 0; --j) {
        if (j == sbits - 1 || (j & 31) == 31)  // one exponent word per 32 bits, loaded ahead of the squaring
          w = __builtin_amdgcn_readfirstlane(launder_s(kw)[j >> 5]);
        fbm_na_sq_lds(aoff, koff, NK, np);
        if ((w >> (j & 31)) & 1u) fbm_na_ms_reg(aoff, hs, doff, NK, np);
      }
      // x C: the chain stays the LDS operand, C (uniform) is the B operand read from its broadcast
      // column in the ops buffer (limb k at word k * 256, every lane the same address)
      fbm_na_mm_glb(aoff, SEG(ops, ops_a) + FBM_OPS_CBC, 0u, NK, np);
    } else {
#ifndef FBM_EXP_SHORT_ONLY  // (a measurement variant: the launch's code without the table path)
    if (__any(wide)) {  // wave-uniform: lanes with a narrow h multiply 0 and add nothing
      lds_store_uniform<2 * NA>(lds, FBM_BLOCK, cst + FBM_CST_QR3);
      fbm_na_mm_glb(aoff, table, tb0 + FBM_TSCRATCH * tstride, NK, np);  // h_hi*R^2 (wide lanes)
      lds_to_glb(lds, table + (tb0 + tstride) / 4);
      uint32_t h[64];
#ifdef FBM_EXP_FULL_H_LOAD  // (A/B variant: the round-3 whole-row load)
      load_row64(SEG(H, H_a) + ct * 64, h);
#else
      load_h(SEG(H, H_a), SEG(Hc, Hc_a), ct, h);
#endif
      uint32_t h29[2 * NA];
      to29_row64(h, h29);
#pragma unroll
      for (int k = NA; k < 2 * NA; ++k) h29[k] = 0u;  // (h_lo, 0)
      col_store(table + (tb0 + FBM_TSCRATCH * tstride) / 4, h29);
    }
    lds_store_uniform<2 * NA>(lds, FBM_BLOCK, cst + FBM_CST_QR2);
    fbm_na_mm_glb(aoff, table, tb0 + FBM_TSCRATCH * tstride, NK, np);  // h*R (narrow) | h_lo*R (wide)
    if (__any(wide)) {  // h R = h_lo R + h_hi R^2: digit-wise sum (< 6N + 2, fine as an operand)
      uint32_t a[2 * NA], b[2 * NA];
      lds_load_col(lds, FBM_BLOCK, a);
      col_load(table + (tb0 + tstride) / 4, b);
#pragma unroll
      for (int d = 0; d < 2; ++d) {
        uint32_t c = 0;
#pragma unroll
        for (int k = 0; k < NA; ++k) {
          const uint32_t v = a[d * NA + k] + (wide ? b[d * NA + k] : 0u) + c;
          a[d * NA + k] = k + 1 < NA ? v & FBM_QMASK : v;  // the top limb keeps the digit's excess
          c = v >> FBM_QA_LB;
        }
      }
      lds_store_col(lds, FBM_BLOCK, a);
    }
    if (!SEG(key_is_zero, key_is_zero_a)) {
      lds_to_glb(lds, table + tb0 / 4);
      fbm_na_sq_lds_looped(aoff, NK, np);  // h^2*R
      lds_to_glb(lds, table + (tb0 + FBM_TSCRATCH * tstride) / 4);
      glb_to_lds(table + tb0 / 4, lds);
#pragma unroll 1
      for (int t = 1; t < FBM_TABLE; ++t) {
        fbm_na_mm_glb(aoff, table, tb0 + FBM_TSCRATCH * tstride, NK, np);
        lds_to_glb(lds, table + (tb0 + (uint32_t)t * tstride) / 4);
      }
      glb_to_lds(table + (tb0 + (uint32_t)SEG(first, first_a) * tstride) / 4, lds);
      const int n_ops = SEG(n_ops, n_ops_a);
#pragma unroll 1
      for (int k = 0; k < n_ops; ++k) {
        const uint32_t op = __builtin_amdgcn_readfirstlane(SEG(ops, ops_a)[k]);
        const int nsq = (int)(op >> FBM_OP_SHIFT);
        const int idx = (int)(op & ((1u << FBM_OP_SHIFT) - 1u)) - 1;
#pragma unroll 1
        for (int q = 0; q < nsq; ++q) fbm_na_sq_lds_looped(aoff, NK, np);
        if (idx >= 0) fbm_na_mm_glb(aoff, table, tb0 + (uint32_t)idx * tstride, NK, np);
      }
    }
#endif
    }  // (table path)
    const int mode = SEG(mode, mode_a);
    if ((mode & FBM_EXP_DEC) == 0) {  // x nude = (1, pt): jl_nude_kernel's 29-bit blocked column, read in place
      // (a chunk is one 256-ciphertext block: its base is uniform, the lane's offset is tid)
      const uint32_t* nb = SEG(nude, nude_a) + uniform_val((uint64_t)(ct >> 8)) * (FBM_NUDE_ROWS * 256);
#ifdef FBM_NUDE_BOTH_DIGITS
      fbm_na_mm_glb(aoff, nb, (uint32_t)(ct & 255) * 4u, NK, np);
#else
      fbm_na_mm_nude(aoff, nb, (uint32_t)(ct & 255) * 4u, NK, np);
#endif
    } else {
      fbm_na_mm_glb(aoff, cst + FBM_CST_ONE, 0u, NK, np);
    }
    uint32_t w[64];
    na_final(lds, cst + FBM_CST_NK, w, mode & FBM_EXP_OUT_NADIC);
    if (valid) store_row64(SEG(out, out_a) + ct * 64, w);
#undef SEG
  }
}

// ------------------------------------------------------------------------------------
// The same exponentiation on the lane-GROUP engines (tools/gen_quad_asm.py): G lanes per
// ciphertext, 29-bit limbs (36 per digit, R = 2^1044), lane l owning limbs M l .. M l + M - 1
// of both digits (M = 36 / G), for launches that hold fewer ciphertexts than the chip has
// resident lanes (one party's 1M elements, the aggregate of a 1/8 stripe): the G x lanes fill
// the chip and a ciphertext's exponentiation takes a fraction of a lane's time.  Same residues
// at every step (the Montgomery form uses R = 2^1044 instead of 2^1036), the same canonical
// results (tests/test_quad_asm.py; the -m gpu tests through every engine).
//   QUAD   (G = 4, fbm_quad_asm.hpp): 16 ciphertexts per wave, DPP quad_perm exchanges.
//   TRIPLE (G = 3, fbm_tri_asm.hpp): 21 ciphertexts per wave (lanes 0..62) + a dummy lane 63
//          with an all-zero column (the wave-shift neighbour of lane 62), ds_bpermute broadcasts.
//   workgroup: 256 lanes = 4 waves; LDS column of ciphertext c: limb k of digit d at word
//   (36 d + k) * ROWW + c (2 spare rows: the last row's prefetch); per-lane tables: entry e,
//   limb row j (b0: j = r, b1: j = M + r) at word (slot * FBM_TENTRIES + e) * ENTRY + j * 256 + tid.
// ------------------------------------------------------------------------------------
#define FBM_QBLOCK 256
#ifndef FBM_GROUP_WAVES  // resident group-engine waves per SIMD (= workgroups per CU): the VGPR budget
#define FBM_GROUP_WAVES 3
#endif

// limb k (lb bits at bit lb k) of a little-endian number of `nw` words in global memory
__device__ __forceinline__ uint32_t glb_limb(const uint32_t* p, int nw, int k, int lb) {
  const int bit = k * lb, wi = bit >> 5, sh = bit & 31;
  const uint64_t lo = wi < nw ? p[wi] : 0u;
  const uint64_t hi = wi + 1 < nw ? p[wi + 1] : 0u;
  return (uint32_t)(((hi << 32) | lo) >> sh) & ((1u << lb) - 1u);
}

template <int G>
struct GroupEng;
template <>
struct GroupEng<4> {
  static constexpr int M = FBM_QA_LIMBS, ROWW = FBM_QA_ROWW, CT_WAVE = 16, CT_WG = 64;
  __device__ static void lane_map(int tid, int& c, int& l, bool& dummy) {
    c = tid >> 2;
    l = tid & 3;
    dummy = false;
  }
  __device__ static uint32_t group_mask(uint64_t bal, int tid) { return (uint32_t)((bal >> ((tid & 63) & ~3)) & 0xFull); }
  __device__ static void mm(uint32_t ac, uint32_t al, const uint32_t* bb, uint32_t boff, const uint32_t* QK, uint32_t np,
                            const uint32_t (&n)[M], uint32_t e0, uint32_t) {
    fbm_qa_mm_glb(ac, al, bb, boff, QK, np, n, e0);
  }
  __device__ static void sq(uint32_t ac, uint32_t al, const uint32_t* QK, uint32_t np, const uint32_t (&n)[M],
                            uint32_t e0, uint32_t) {
    fbm_qa_sq_lds(ac, al, QK, np, n, e0);
  }
  __device__ static void sq_looped(uint32_t ac, uint32_t al, const uint32_t* QK, uint32_t np, const uint32_t (&n)[M],
                                   uint32_t e0, uint32_t) {
    fbm_qa_sq_lds_looped(ac, al, QK, np, n, e0);
  }
  __device__ static void ms(uint32_t ac, uint32_t al, uint32_t dl, uint32_t np, const uint32_t (&n)[M], uint32_t e0,
                            uint32_t) {
    fbm_qa_ms_lds(ac, al, dl, np, n, e0);
  }
};
template <>
struct GroupEng<3> {
  static constexpr int M = FBM_TA_LIMBS, ROWW = FBM_TA_ROWW, CT_WAVE = 21, CT_WG = 84;
  __device__ static void lane_map(int tid, int& c, int& l, bool& dummy) {
    const int w = tid >> 6, j = tid & 63;
    dummy = j == 63;
    c = dummy ? CT_WG : CT_WAVE * w + j / 3;  // the 4 dummy lanes share the zero column CT_WG
    l = dummy ? 0 : j % 3;
  }
  __device__ static uint32_t group_mask(uint64_t bal, int tid) {
    const int j = tid & 63;
    return (uint32_t)((bal >> (3 * (j / 3))) & 0x7ull);
  }
  __device__ static void mm(uint32_t ac, uint32_t al, const uint32_t* bb, uint32_t boff, const uint32_t* QK, uint32_t np,
                            const uint32_t (&n)[M], uint32_t e0, uint32_t bp) {
    fbm_ta_mm_glb(ac, al, bb, boff, QK, np, n, e0, bp);
  }
  __device__ static void sq(uint32_t ac, uint32_t al, const uint32_t* QK, uint32_t np, const uint32_t (&n)[M],
                            uint32_t e0, uint32_t bp) {
    fbm_ta_sq_lds(ac, al, QK, np, n, e0, bp);
  }
  __device__ static void sq_looped(uint32_t ac, uint32_t al, const uint32_t* QK, uint32_t np, const uint32_t (&n)[M],
                                   uint32_t e0, uint32_t bp) {
    fbm_ta_sq_lds_looped(ac, al, QK, np, n, e0, bp);
  }
  __device__ static void ms(uint32_t ac, uint32_t al, uint32_t dl, uint32_t np, const uint32_t (&n)[M], uint32_t e0,
                            uint32_t bp) {
    fbm_ta_ms_lds(ac, al, dl, np, n, e0, bp);
  }
};

// the lane's slice of a digit pair held as 72 uniform 29-bit limbs (R^2, R^3 digits) -> LDS
template <int M, int ROWW>
__device__ __forceinline__ void qa_lds_store_uniform(uint32_t* col, int l, const uint32_t* u) {
  u = launder_s(u);
#pragma unroll
  for (int d = 0; d < 2; ++d)
#pragma unroll
    for (int r = 0; r < M; ++r) {
      const int k = M * l + r;
      col[(d * FBM_QA_D1 + k) * ROWW] = u[d * FBM_QA_L + k];
    }
}
// lane slice LDS <-> table entry (p = entry base + tid)
template <int M, int ROWW>
__device__ __forceinline__ void qa_lds_to_tbl(const uint32_t* col, int l, uint32_t* p) {
  uint32_t v[2 * M];
#pragma unroll
  for (int d = 0; d < 2; ++d)
#pragma unroll
    for (int r = 0; r < M; ++r) v[d * M + r] = col[(d * FBM_QA_D1 + M * l + r) * ROWW];
  col_store<2 * M>(p, v);
}
template <int M, int ROWW>
__device__ __forceinline__ void qa_tbl_to_lds(const uint32_t* p, uint32_t* col, int l) {
  uint32_t v[2 * M];
  col_load<2 * M>(p, v);
#pragma unroll
  for (int d = 0; d < 2; ++d)
#pragma unroll
    for (int r = 0; r < M; ++r) col[(d * FBM_QA_D1 + M * l + r) * ROWW] = v[d * M + r];
}
// lane 0 of the group: carry-normalise both digits of the column in place (lazy limbs from
// a digit-wise sum; the engine's own outputs need no pass)
template <int ROWW>
__device__ __forceinline__ void qa_normalise_column(uint32_t* col) {
#pragma unroll 1
  for (int d = 0; d < 2; ++d) {
    uint32_t c = 0;
#pragma unroll 1
    for (int k = 0; k < FBM_QA_L; ++k) {
      const uint32_t v = col[(d * FBM_QA_D1 + k) * ROWW] + c;
      col[(d * FBM_QA_D1 + k) * ROWW] = v & FBM_QMASK;
      c = v >> FBM_QA_LB;
    }
  }
}

template <int G>
__global__ void __launch_bounds__(FBM_QBLOCK, FBM_GROUP_WAVES) jl_expg_kernel(const uint32_t* __restrict__ H, uint64_t n_ct,
                                                               uint32_t* __restrict__ cst, uint32_t np29,
                                                               const uint32_t* __restrict__ ops, int n_ops,
                                                               int first, int mode, int key_is_zero, int sbits,
                                                               const uint32_t* __restrict__ nude,
                                                               uint32_t* __restrict__ table,
                                                               uint32_t* __restrict__ out,
                                                               const uint32_t* __restrict__ Hc) {
  using E = GroupEng<G>;
  constexpr int M = E::M, ROWW = E::ROWW;
  constexpr uint32_t ENTRY = 2 * M * 256;  // words of one table entry
  // column rows: the two digits, two spare rows, the short path's h limbs (FBM_QA_HROW ..) and their
  // prefetch row; the pairs (D_j, 0) of the short product, then 12 zero pairs (the dummy lane's)
  constexpr int ROWS = FBM_QA_HROW + FBM_NA_SHORT_LIMBS + 1;
  static_assert(FBM_QA_HROW == FBM_TA_HROW && FBM_QA_HROW == 2 * FBM_QA_D1 + 2, "column rows");
  __shared__ uint32_t lds_q[ROWS * ROWW];
  __shared__ uint32_t lds_d[96];
  __shared__ uint32_t chunk_s;
  const int tid = threadIdx.x;
  int c, l;
  bool dummy;
  E::lane_map(tid, c, l, dummy);
  uint32_t* col = lds_q + c;
  const uint32_t ac = lds_addr(col);
  const uint32_t al = ac + (uint32_t)(M * l * ROWW * 4);
  const uint32_t* QK = cst + FBM_CST_QK;
  uint32_t n[M];
#pragma unroll
  for (int r = 0; r < M; ++r) n[r] = dummy ? 0u : cst[FBM_CST_QNP + M * l + r];
  const uint32_t e0 = (l == 0 && !dummy) ? 1u : 0u;
  // ds_bpermute source of the quotient digits: the group's lane 0 (the dummy: itself)
  const uint32_t bp = (uint32_t)(4 * (dummy ? (tid & 63) : (tid & 63) - l));
  if (dummy) {  // the dummy column stays all-zero: its lanes multiply nothing but zeros
#pragma unroll 1
    for (int k = 0; k < ROWS; ++k) col[k * ROWW] = 0u;
  }
  if (tid < 96) lds_d[tid] = tid < 72 ? launder_s(cst)[FBM_CST_QD + tid] : 0u;  // (ordered by the loop's barrier)
  const uint32_t dl = lds_addr(lds_d) + 8u * (uint32_t)(dummy ? FBM_QA_L : M * l);
  // byte offset of this lane's word in table entry 0 of this workgroup's slot
  const uint32_t tb0 = (uint32_t)(((uint64_t)blockIdx.x * FBM_TENTRIES * ENTRY + tid) * 4);
  const uint32_t tstride = ENTRY * 4;
  const uint32_t n_chunks = (uint32_t)((n_ct + E::CT_WG - 1) / E::CT_WG);
#pragma unroll 1
  for (;;) {
    if (tid == 0) chunk_s = atomicAdd(cst + FBM_CST_CTR, 1u);
    __syncthreads();
    const uint32_t chunk = __builtin_amdgcn_readfirstlane(chunk_s);
    __syncthreads();
    if (chunk >= n_chunks) break;
    const uint64_t ct_raw = (uint64_t)chunk * E::CT_WG + c;
    const bool valid = !dummy && ct_raw < n_ct;
    const uint64_t ct = ct_raw < n_ct ? ct_raw : n_ct - 1;
    uint32_t* scratch = table + (tb0 + FBM_TSCRATCH * tstride) / 4;
    bool wide = false, shortp = false;
    {  // h -> the lane's 29-bit limbs of (h mod R, h div R) -> scratch
      uint32_t h18[2 * M];
      // the compact row (8 words, launch_jl_fdh) unless it holds the sentinel (or there is none): the whole row
      const uint32_t* hr = H + ct * 64;
      int hw = 64;
      if (Hc) {
        const uint4* c = reinterpret_cast<const uint4*>(Hc + ct * 8);
        const uint4 a = c[0], b = c[1];
        if ((a.x & a.y & a.z & a.w & b.x & b.y & b.z & b.w) != ~0u) {
          hr = Hc + ct * 8;
          hw = 8;
        }
      }
#pragma unroll
      for (int r = 0; r < M; ++r) {
        const int k = M * l + r;
        uint32_t lo = 0, hi = 0;
        if (dummy) {
        } else if (key_is_zero) {
          lo = k == 0 ? 1u : 0u;
        } else {
          lo = glb_limb(hr, hw, k, FBM_QA_LB);
          hi = glb_limb(hr, hw, FBM_QA_L + k, FBM_QA_LB);
        }
        h18[r] = lo;
        h18[M + r] = hi;
      }
      {
        uint32_t any = 0, mid = 0;
#pragma unroll
        for (int r = 0; r < M; ++r) {
          any |= h18[M + r];
          if (M * l + r >= FBM_NA_SHORT_LIMBS) mid |= h18[r];
        }
        // the short path (as jl_exp_kernel's): every h of the wave below 2^261 and a schedule for it
        shortp = sbits >= 0 && !key_is_zero && !__any(any != 0u || mid != 0u);
        if (shortp) {  // A = (h, 0) raw; h's limbs 0 .. KS (the last: 0, the prefetch row) -> rows HROW ..
#pragma unroll
          for (int r = 0; r < M; ++r) {
            const int k = M * l + r;
            col[k * ROWW] = h18[r];
            col[(FBM_QA_D1 + k) * ROWW] = 0u;
            if (k <= FBM_NA_SHORT_LIMBS) col[(FBM_QA_HROW + k) * ROWW] = h18[r];
          }
        }
        // wide is a property of the ciphertext, not of the lane's slice: OR over the group
        wide = E::group_mask(__ballot(any != 0u), tid) != 0u;
        if (!shortp && __any(wide)) {  // FDH retries (small moduli): h_hi R^2 = (h_hi, 0) * R^3 R^-1 -> entry 1
          uint32_t w18[2 * M];
#pragma unroll
          for (int r = 0; r < M; ++r) {
            w18[r] = h18[M + r];
            w18[M + r] = 0u;
            h18[M + r] = 0u;  // (h_lo, 0) for the main product below
          }
          col_store<2 * M>(scratch, w18);
          if (!dummy) qa_lds_store_uniform<M, ROWW>(col, l, cst + FBM_CST_QR3);
          E::mm(ac, al, table, tb0 + FBM_TSCRATCH * tstride, QK, np29, n, e0, bp);
          qa_lds_to_tbl<M, ROWW>(col, l, table + (tb0 + tstride) / 4);
        }
      }
      if (!shortp) col_store<2 * M>(scratch, h18);
    }
    if (shortp) {  // binary chain with short-base products, then C (jl_exp_kernel's short path)
      const uint32_t* kw = ops + FBM_OPS_KW;
      uint32_t w = 0;
#pragma unroll 1
      for (int j = sbits - 1; j >= 0; --j) {
        if (j == sbits - 1 || (j & 31) == 31) w = __builtin_amdgcn_readfirstlane(launder_s(kw)[j >> 5]);
        E::sq(ac, al, QK, np29, n, e0, bp);
        if ((w >> (j & 31)) & 1u) E::ms(ac, al, dl, np29, n, e0, bp);
      }
      qa_lds_to_tbl<M, ROWW>(col, l, table + tb0 / 4);
      if (!dummy) qa_lds_store_uniform<M, ROWW>(col, l, ops + FBM_OPS_CORR);
      E::mm(ac, al, table, tb0, QK, np29, n, e0, bp);
    } else {
    if (!dummy) qa_lds_store_uniform<M, ROWW>(col, l, cst + FBM_CST_QR2);
    E::mm(ac, al, table, tb0 + FBM_TSCRATCH * tstride, QK, np29, n, e0, bp);  // h R | h_lo R
    if (__any(wide)) {  // h R = h_lo R + h_hi R^2 (digit-wise, then carries)
      uint32_t b18[2 * M];
      col_load<2 * M>(table + (tb0 + tstride) / 4, b18);
#pragma unroll
      for (int d = 0; d < 2; ++d)
#pragma unroll
        for (int r = 0; r < M; ++r) col[(d * FBM_QA_D1 + M * l + r) * ROWW] += wide ? b18[d * M + r] : 0u;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // a group never straddles two waves
      if (l == 0 && !dummy) qa_normalise_column<ROWW>(col);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    if (!key_is_zero) {
      qa_lds_to_tbl<M, ROWW>(col, l, table + tb0 / 4);
      E::sq_looped(ac, al, QK, np29, n, e0, bp);  // h^2 R (table path: the looped square, cold code)
      qa_lds_to_tbl<M, ROWW>(col, l, scratch);
      qa_tbl_to_lds<M, ROWW>(table + tb0 / 4, col, l);
#pragma unroll 1
      for (int t = 1; t < FBM_TABLE; ++t) {
        E::mm(ac, al, table, tb0 + FBM_TSCRATCH * tstride, QK, np29, n, e0, bp);
        qa_lds_to_tbl<M, ROWW>(col, l, table + (tb0 + (uint32_t)t * tstride) / 4);
      }
      qa_tbl_to_lds<M, ROWW>(table + (tb0 + (uint32_t)first * tstride) / 4, col, l);
#pragma unroll 1
      for (int k = 0; k < n_ops; ++k) {
        const uint32_t op = __builtin_amdgcn_readfirstlane(ops[k]);
        const int nsq = (int)(op >> FBM_OP_SHIFT);
        const int idx = (int)(op & ((1u << FBM_OP_SHIFT) - 1u)) - 1;
#pragma unroll 1
        for (int q = 0; q < nsq; ++q) E::sq_looped(ac, al, QK, np29, n, e0, bp);
        if (idx >= 0) E::mm(ac, al, table, tb0 + (uint32_t)idx * tstride, QK, np29, n, e0, bp);
      }
    }
    }  // (table path)
    {  // last operand: nude = (1, pt) (encrypt; jl_nude_kernel's 29-bit rows, the lane's slice) or 1
      uint32_t b18[2 * M];
      const uint32_t* nb = nude + (ct >> 8) * (FBM_NUDE_ROWS * 256) + (ct & 255);
#pragma unroll
      for (int d = 0; d < 2; ++d)
#pragma unroll
        for (int r = 0; r < M; ++r) {
          const int k = M * l + r;
          uint32_t v = 0;
          if (dummy) {
          } else if ((mode & FBM_EXP_DEC) == 0) {
            v = d == 0 ? (k == 0 ? 1u : 0u) : nb[(FBM_NUDE_D1 + k) * 256];  // (1, pt): jl_nude_kernel's rows of pt
          } else {
            v = (d == 0 && k == 0) ? 1u : 0u;
          }
          b18[d * M + r] = v;
        }
      col_store<2 * M>(scratch, b18);
    }
    E::mm(ac, al, table, tb0 + FBM_TSCRATCH * tstride, QK, np29, n, e0, bp);
    if (l == 0 && !dummy) {  // t + s N -> the canonical residue (lane 0 of the group, from the LDS column)
      uint32_t t29[FBM_QA_L], s29[FBM_QA_L];
      uint32_t ct0 = 0, cs0 = 0;
#pragma unroll
      for (int k = 0; k < FBM_QA_L; ++k) {  // the engine's lazy limbs -> normalised 29-bit limbs
        const uint32_t vt = col[k * ROWW] + ct0;
        const uint32_t vs = col[(FBM_QA_D1 + k) * ROWW] + cs0;
        t29[k] = vt & FBM_QMASK;
        s29[k] = vs & FBM_QMASK;
        ct0 = vt >> FBM_QA_LB;
        cs0 = vs >> FBM_QA_LB;
      }
      uint32_t t[FBM_NLN], sd[FBM_NLN];  // re-limbed to 28 bits for the shared final step
#pragma unroll
      for (int j = 0; j < FBM_NLN; ++j) {
        const int bit = j * FBM_LB, k = bit / FBM_QA_LB, off = bit % FBM_QA_LB;
        const uint64_t tw = ((uint64_t)(k + 1 < FBM_QA_L ? t29[k + 1] : 0u) << FBM_QA_LB) | (k < FBM_QA_L ? t29[k] : 0u);
        const uint64_t sw = ((uint64_t)(k + 1 < FBM_QA_L ? s29[k + 1] : 0u) << FBM_QA_LB) | (k < FBM_QA_L ? s29[k] : 0u);
        t[j] = (uint32_t)(tw >> off) & FBM_LMASK;
        sd[j] = (uint32_t)(sw >> off) & FBM_LMASK;
      }
      uint32_t w[64];
      na_final_digits(t, sd, cst + FBM_CST_NK, w, mode & FBM_EXP_OUT_NADIC);
      if (valid) store_row64(out + ct * 64, w);
    }
  }
}

// ------------------------------------------------------------------------------------
// (v - 1) div N for v < N^2 (64 words, v >= 1 for any unit: D = v - 1 on entry) -> x (32
// words).  Exact whenever the keys are consistent (v = 1 + N x mod N^2): x = D N^-1 mod
// 2^1024, accepted iff x N == D.  Otherwise (a wrong server key: the reference still returns
// floor((v-1)/N), _jls.py:553-558) binary long division.
// ------------------------------------------------------------------------------------
__device__ __forceinline__ void mullo1024(const uint32_t (&d)[32], const uint32_t* m, uint32_t (&q)[32]) {
  // q = d * m mod 2^1024, product scanning over 32-bit words (3-word column sums)
  uint64_t lo = 0, hi = 0;
#pragma clang loop unroll(full)
  for (int k = 0; k < 32; ++k) {
#pragma clang loop unroll(full)
    for (int i = 0; i <= k; ++i) {
      const uint64_t p = (uint64_t)d[i] * m[k - i];
      lo += (uint32_t)p;
      hi += (p >> 32);
    }
    q[k] = (uint32_t)lo;
    const uint64_t c = (lo >> 32) + hi;
    lo = c & 0xffffffffull;
    hi = c >> 32;
  }
}

// r = a * b (32 x 32 words -> 64), product scanning like mullo1024 (fully unrolled: a
// row-by-row form gets re-rolled by the optimiser into a loop over a scratch array)
__device__ __forceinline__ void mul1024(const uint32_t (&a)[32], const uint32_t* b, uint32_t (&r)[64]) {
  uint64_t lo = 0, hi = 0;
#pragma clang loop unroll(full)
  for (int k = 0; k < 63; ++k) {
#pragma clang loop unroll(full)
    for (int i = (k < 32 ? 0 : k - 31); i <= (k < 32 ? k : 31); ++i) {
      const uint64_t p = (uint64_t)a[i] * b[k - i];
      lo += (uint32_t)p;
      hi += (p >> 32);
    }
    r[k] = (uint32_t)lo;
    const uint64_t c = (lo >> 32) + hi;
    lo = c & 0xffffffffull;
    hi = c >> 32;
  }
  r[63] = (uint32_t)lo;
}

// binary long division (the fallback of the exact-division check)
__device__ __forceinline__ void div_by_n_slow(uint32_t (&D)[64], const JlParams& jp, uint32_t (&q)[32]) {
  uint32_t r[33];
#pragma unroll
  for (int i = 0; i < 32; ++i) q[i] = 0u;
#pragma unroll
  for (int i = 0; i < 33; ++i) r[i] = 0u;
  int top = 0;
#pragma unroll
  for (int i = 0; i < 64; ++i)
    if (D[i]) top = i;
  const int nbits = 32 * (top + 1);
#pragma unroll 1
  for (int s = top; s < 63; ++s) {  // left-align the significant words
#pragma unroll
    for (int i = 63; i > 0; --i) D[i] = D[i - 1];
    D[0] = 0u;
  }
#pragma unroll 1
  for (int b = 0; b < nbits; ++b) {
    const uint32_t bit = D[63] >> 31;
#pragma unroll
    for (int i = 63; i > 0; --i) D[i] = (D[i] << 1) | (D[i - 1] >> 31);
    D[0] <<= 1;
#pragma unroll
    for (int i = 32; i > 0; --i) r[i] = (r[i] << 1) | (r[i - 1] >> 31);
    r[0] = (r[0] << 1) | bit;
#pragma unroll
    for (int i = 31; i > 0; --i) q[i] = (q[i] << 1) | (q[i - 1] >> 31);
    q[0] <<= 1;
    uint32_t t[33];
    uint32_t br = 0;
#pragma unroll
    for (int i = 0; i < 33; ++i) {
      const uint64_t d = (uint64_t)r[i] - (i < 32 ? jp.N32[i] : 0u) - br;
      t[i] = (uint32_t)d;
      br = (uint32_t)(d >> 63);
    }
    if (!br) {
#pragma unroll
      for (int i = 0; i < 33; ++i) r[i] = t[i];
      q[0] |= 1u;
    }
  }
}

// D in the lane's LDS column (64 words, stride FBM_BLOCK): the fast path holds only D's low half, then q and
// the running column sums, in registers -- q N's low half equals D's by construction of q, so only the high half
// is compared, each word read from LDS as its column completes.  D's 64 registers kept live across the check
// (round 6's first form) cost the two-waves-per-SIMD jl_prod_kernel 308 bytes of scratch per lane.
__device__ __forceinline__ void div_by_n_lds(const uint32_t* ldsD, const JlParams& jp, uint32_t (&q)[32]) {
  {
    uint32_t dl[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) dl[i] = ldsD[i * FBM_BLOCK];
    mullo1024(dl, jp.Ninv32, q);
  }
  uint64_t lo = 0, hi = 0;
  uint32_t diff = 0;
#pragma clang loop unroll(full)
  for (int k = 0; k < 63; ++k) {
#pragma clang loop unroll(full)
    for (int i = (k < 32 ? 0 : k - 31); i <= (k < 32 ? k : 31); ++i) {
      const uint64_t p = (uint64_t)q[i] * jp.N32[k - i];
      lo += (uint32_t)p;
      hi += (p >> 32);
    }
    if (k >= 32) diff |= (uint32_t)lo ^ ldsD[k * FBM_BLOCK];
    const uint64_t c = (lo >> 32) + hi;
    lo = c & 0xffffffffull;
    hi = c >> 32;
  }
  diff |= (uint32_t)lo ^ ldsD[63 * FBM_BLOCK];
  if (diff == 0) return;
  uint32_t D[64];
#pragma unroll
  for (int i = 0; i < 64; ++i) D[i] = ldsD[i * FBM_BLOCK];
  div_by_n_slow(D, jp, q);
}


// ------------------------------------------------------------------------------------
// aggregate (_jls.py:353-374 product, :547-558 decrypt), one lane per ciphertext:
//   v = prod_u c_u * F mod N^2,  x = (v - 1) div N   -> xout [ct][32]
// Montgomery products mod M = N^2 on the assembly engine (fbm_mont_asm.hpp), a = the running
// product in the lane's LDS column, b = the next operand read by the product straight from its
// 64-word row (fbm_mm_row: sixteen 16-byte loads, the 28-bit limbs made in B's registers):
//   a = R^(P+1) mod M (uniform, cst[FBM_CST_RK]),  b = c_0   -> c_0 R^P
//   b = c_u, u = 1 .. P-1, then b = F                        -> each drops one R -> v (lazy)
// P + 1 products, no Montgomery-form round trips; any c_u < 2^2048 qualifies (a b < R M).
// One LDS column per lane: 76.8 KB per workgroup, two waves per SIMD, no scratch (the exact division
// checks against D parked in the same column: div_by_n_lds).
// ------------------------------------------------------------------------------------
// factor == nullptr: the bare product (EncryptedNumber sums, _jls.py:353-374): a starts from
// R^P, P products, and the canonical v goes to xout [ct][64] (no decryption).
// History: the operand staged as a 28-bit column in a second LDS column (153.6 KB,
// one wave per SIMD: 1.60 ms at 10M x 8, now 1.35); a global scratch column before that (3x the HBM traffic).
__global__ void __launch_bounds__(FBM_BLOCK, 2) jl_prod_kernel(const uint32_t* __restrict__ cts, int n_parties,
                                                              uint64_t n_ct, const uint32_t* __restrict__ cst,
                                                              JlParams jp, const uint32_t* __restrict__ factor,
                                                              uint32_t* __restrict__ xout) {
  __shared__ uint32_t lds_a[(FBM_NL + 1) * FBM_BLOCK];
  const int tid = threadIdx.x;
  uint32_t* lds = lds_a + tid;
  const uint32_t aoff = lds_addr(lds);
  const uint32_t* M = cst + FBM_CST_M;
  const uint64_t ct_raw = (uint64_t)blockIdx.x * FBM_BLOCK + tid;
  const bool valid = ct_raw < n_ct;  // (an early return here measured 15 % slower)
  const uint64_t ct = valid ? ct_raw : n_ct - 1;
  lds_store_uniform<FBM_NL>(lds, FBM_BLOCK, cst + FBM_CST_RK);
  const int n_ops = n_parties + (factor ? 1 : 0);
#pragma unroll 1
  for (int u = 0; u < n_ops; ++u) {
    const uint32_t* row = u < n_parties ? cts + ((uint64_t)u * n_ct + ct) * 64 : factor + ct * 64;
    fbm_mm_row(aoff, row, M, jp.mc.mp);
  }
  uint32_t D[64];
  {
    uint32_t v[FBM_NL];
    lds_load_col(lds, FBM_BLOCK, v);
    mont_csub(v, jp.mc.M);
    from28<FBM_NL, 64>(v, D);
  }
  if (!factor) {
    if (valid) store_row64(xout + ct * 64, D);
    return;
  }
  uint32_t br = 1;  // D = v - 1
#pragma unroll
  for (int i = 0; i < 64; ++i) {
    const uint64_t d = (uint64_t)D[i] - br;
    D[i] = (uint32_t)d;
    br = (uint32_t)(d >> 63);
  }
  uint32_t x[32];
  if (br) {  // v == 0 (a ciphertext = 0 mod N^2): ((0 - 1) // N) mod N = N - 1 in Python
    uint32_t b = 1;
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      const uint64_t d = (uint64_t)jp.N32[i] - b;
      x[i] = (uint32_t)d;
      b = (uint32_t)(d >> 63);
    }
  } else {
    lds_store_col<64>(lds, FBM_BLOCK, D);  // (the column is free: the product is in D)
    div_by_n_lds(lds, jp, x);
  }
  if (valid) {
    uint4* o = reinterpret_cast<uint4*>(xout + ct * 32);
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = make_uint4(x[4 * i], x[4 * i + 1], x[4 * i + 2], x[4 * i + 3]);
  }
}

// ------------------------------------------------------------------------------------
// encrypt with its factor computed ahead (fbm_jl_encrypt_factor, UserKey.encrypt, _jls.py:473-505):
//   c = (N pt + 1) F mod N^2,  F = H(t_k)^sk mod N^2 (jl_factor: the decryption factor's
// kernels with the party's key, run before the plaintext exists), the exponentiation's encrypt
// bit for bit.  Two Montgomery products mod M = N^2 from a = R^2 (jl_rk_kernel), as jl_prod_kernel:
//   b = N pt + 1 (formed in registers: pt < 2^1024, N < 2^1024, so b < 2^2048 qualifies)  -> R b
//   b = F                                                                           -> b F mod M
// A negative weight (pt = |pt|, see jl_pack_kernel) encrypts 1 - N |pt|: b = N |pt| - 1, and
// the product is negated mod M at the end ((1 - N |pt|) F = -(N |pt| - 1) F); |pt| = 0 is 1.
// ------------------------------------------------------------------------------------
// Round 6: b = N pt + 1 is staged in the lane's own output row (rewritten at the end) and both products read
// their operand rows with fbm_mm_row, as jl_prod_kernel: one LDS column per lane, two waves per SIMD.  A lane
// past n_ct reads the factor row of ciphertext n_ct - 1 (read-only) instead, and stores nothing.
__global__ void __launch_bounds__(FBM_BLOCK, 2) jl_encf_kernel(const uint32_t* __restrict__ pt, uint64_t n_ct,
                                                              const uint32_t* __restrict__ cst, JlParams jp,
                                                              int negative, const uint32_t* __restrict__ factor,
                                                              uint32_t* __restrict__ out) {
  __shared__ uint32_t lds_a[(FBM_NL + 1) * FBM_BLOCK];
  const int tid = threadIdx.x;
  uint32_t* lds = lds_a + tid;
  const uint32_t aoff = lds_addr(lds);
  const uint32_t* M = cst + FBM_CST_M;
  const uint64_t ct_raw = (uint64_t)blockIdx.x * FBM_BLOCK + tid;
  const bool valid = ct_raw < n_ct;  // no early return: every lane runs the products
  const uint64_t ct = valid ? ct_raw : n_ct - 1;
  lds_store_uniform<FBM_NL>(lds, FBM_BLOCK, cst + FBM_CST_RK);
  bool neg;
  {
    uint32_t p[32];
    load_row32(reinterpret_cast<const uint4*>(pt + ct * 32), p);
    uint32_t any = 0;
#pragma unroll
    for (int i = 0; i < 32; ++i) any |= p[i];
    neg = negative && any;
    // b = N p' + A, product-scanned into the output row four words at a time (no 64-word b in registers):
    // p' = pt, A = 1 -> N pt + 1 < 2^2048; a negative weight p' = |pt| - 1, A = N - 1 -> N |pt| - 1
    uint32_t br = neg ? 1u : 0u;
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      const uint64_t d = (uint64_t)p[i] - br;
      p[i] = (uint32_t)d;
      br = (uint32_t)(d >> 63);
    }
    uint4* o = reinterpret_cast<uint4*>(out + ct * 64);
    uint64_t lo = neg ? (uint64_t)(jp.N32[0] - 1u) : 1u, hi = 0;
    uint32_t w[4];
#pragma clang loop unroll(full)
    for (int k = 0; k < 63; ++k) {
      if (k > 0 && k < 32) lo += neg ? jp.N32[k] : 0u;
#pragma clang loop unroll(full)
      for (int i = (k < 32 ? 0 : k - 31); i <= (k < 32 ? k : 31); ++i) {
        const uint64_t m = (uint64_t)p[i] * jp.N32[k - i];
        lo += (uint32_t)m;
        hi += (m >> 32);
      }
      w[k & 3] = (uint32_t)lo;
      const uint64_t c = (lo >> 32) + hi;
      lo = c & 0xffffffffull;
      hi = c >> 32;
      if ((k & 3) == 3 && valid) o[k >> 2] = make_uint4(w[0], w[1], w[2], w[3]);
    }
    w[3] = (uint32_t)lo;
    if (valid) {
      o[15] = make_uint4(w[0], w[1], w[2], w[3]);
      __builtin_amdgcn_s_waitcnt(0);  // (vmcnt 0: the stores done before the product loads the row)
    }
  }
  fbm_mm_row(aoff, valid ? out + ct * 64 : factor + ct * 64, M, jp.mc.mp);  // a = R b
  fbm_mm_row(aoff, factor + ct * 64, M, jp.mc.mp);                         // a = b F (lazy)
  uint32_t v[FBM_NL], D[64];
  lds_load_col(lds, FBM_BLOCK, v);
  mont_csub(v, jp.mc.M);
  uint32_t nz = 0;
#pragma unroll
  for (int k = 0; k < FBM_NL; ++k) nz |= v[k];
  if (neg && nz) {  // M - v, v in (0, M)
    int32_t br = 0;
#pragma unroll
    for (int k = 0; k < FBM_NL; ++k) {
      const int32_t d = (int32_t)jp.mc.M[k] - (int32_t)v[k] + br;
      v[k] = (uint32_t)d & FBM_LMASK;
      br = d >> FBM_LB;
    }
  }
  from28<FBM_NL, 64>(v, D);
  if (valid) store_row64(out + ct * 64, D);
}

// ------------------------------------------------------------------------------------
// inverse mod N^2 from N-adic digits: y = e0^-1 mod N (Bernstein-Yang divsteps), then
// one N-adic lift step (jl_lift_kernel).  e = H^|sk0| mod N^2 (the factor) or H (a
// negative-key encrypt).
// ------------------------------------------------------------------------------------
template <int W>
__device__ __forceinline__ void shr1(uint32_t (&a)[W], uint32_t top) {
#pragma unroll
  for (int i = 0; i < W - 1; ++i) a[i] = (a[i] >> 1) | (a[i + 1] << 31);
  a[W - 1] = (a[W - 1] >> 1) | (top << 31);
}
template <int W>
__device__ __forceinline__ uint32_t add_into(uint32_t (&a)[W], const uint32_t* b) {
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < W; ++i) {
    const uint64_t s = (uint64_t)a[i] + b[i] + c;
    a[i] = (uint32_t)s;
    c = (uint32_t)(s >> 32);
  }
  return c;
}
template <int W>
__device__ __forceinline__ uint32_t sub_from(uint32_t (&a)[W], const uint32_t (&b)[W]) {
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < W; ++i) {
    const uint64_t d = (uint64_t)a[i] - b[i] - br;
    a[i] = (uint32_t)d;
    br = (uint32_t)(d >> 63);
  }
  return br;
}

// y = e0^-1 mod N -> Y [ct][32], e0 = words 0..31 of src row ct (stride src_stride words),
// by Bernstein-Yang divsteps (fbm_safegcd.hpp): branch-free batches of 30 divsteps; the loop
// leaves when every lane of the wave is done (a finished lane is a fixed point of further
// batches).
__global__ void __launch_bounds__(FBM_BLOCK) jl_inv_modn_kernel(uint64_t n_ct, JlParams jp,
                                                               const uint32_t* __restrict__ src, int src_stride,
                                                               uint32_t* __restrict__ Y,
                                                               uint32_t* __restrict__ stats) {
  const uint64_t ct_raw = (uint64_t)blockIdx.x * FBM_BLOCK + threadIdx.x;
  const uint64_t ct = ct_raw < n_ct ? ct_raw : n_ct - 1;  // all lanes take part in the vote
  uint32_t err = 0;
  uint32_t x1[32];
  {
    uint32_t u[32];
    const uint4* yi = reinterpret_cast<const uint4*>(src + ct * (uint64_t)src_stride);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const uint4 v = yi[i];
      u[4 * i] = v.x; u[4 * i + 1] = v.y; u[4 * i + 2] = v.z; u[4 * i + 3] = v.w;
    }
    FbmInvState st;
    fbm_modinv_init(st, u, jp.n30);
    for (int b = 0; b < FBM_INV_MAX_BATCHES; ++b) {
      if (__all(fbm_s30_is_zero(st.g))) break;
      fbm_modinv_batch(st, jp.n30);
    }
    if (!fbm_s30_is_zero(st.g)) {
      err |= FBM_ERR_ITER_CAP;
    } else if (!fbm_modinv_finish(st, jp.n30, x1)) {
      err |= FBM_ERR_NOT_INVERTIBLE;
    }
  }
  if (ct_raw < n_ct) {
    uint4* yo = reinterpret_cast<uint4*>(Y + ct * 32);
#pragma unroll
    for (int i = 0; i < 8; ++i) yo[i] = make_uint4(x1[4 * i], x1[4 * i + 1], x1[4 * i + 2], x1[4 * i + 3]);
    if (err) atomicOr(stats + FBM_STAT_ERRFLAGS, err);
  }
}

// E^-1 mod N^2 from E = e0 + e1 N (digits < N, Ed [ct][64] = e0 | e1) and y = e0^-1 mod N:
// e0 y = 1 + a N with a < N, so E y = 1 + N (a + e1 y) mod N^2 and
//   E^-1 = y (1 - N (a + e1 y)) = y + N v,   v = -y (a + e1 y) mod N.
// a = (e0 y - 1) N^-1 mod 2^1024 from the low halves alone (a < N); v by three Montgomery
// products mod N (37 limbs, R_N = 2^1036): Y' = y R_N, u = e1 y, w = (a + u) y.
// With nude (a negative-key encrypt: c = (N pt + 1) H^key = nude * (H^|key|)^-1, nude = the
// digits (1, p) of jl_nude_kernel): c = y + N ((v + p y) mod N), one more product.
// out [ct][64] canonical.  out may alias Ed: each lane reads its row before writing it.
__global__ void __launch_bounds__(FBM_BLOCK, 2) jl_lift_kernel(uint64_t n_ct, JlParams jp,
                                                              const uint32_t* __restrict__ cst, const uint32_t* Ed,
                                                              const uint32_t* __restrict__ Y,
                                                              const uint32_t* __restrict__ nude, uint32_t* out) {
  const MontCtxN& mn = *reinterpret_cast<const MontCtxN*>(cst + FBM_CST_MN);
  __shared__ uint32_t lds_a[FBM_NLN * FBM_BLOCK];
  const int tid = threadIdx.x;
  uint32_t* lds = lds_a + tid;
  const int ls = FBM_BLOCK;
  const uint64_t ct0 = (uint64_t)blockIdx.x * FBM_BLOCK;
  const uint64_t ct = ct0 + tid < n_ct ? ct0 + tid : n_ct - 1;  // no early return: barriers below
  // y, e0 and a are (re)loaded / formed where they are used: nothing 1024-bit stays live across
  // the Montgomery products (no scratch spills; the rows are L2-resident re-reads)
  const uint4* yi = reinterpret_cast<const uint4*>(Y + ct * 32);
  uint32_t acc[FBM_NLN];
  {
    uint32_t y[32], y28[FBM_NLN];
    load_row32(yi, y);
    to28<32, FBM_NLN>(y, y28);
    lds_store_col(lds, ls, y28);
  }
#pragma unroll
  for (int k = 0; k < FBM_NLN; ++k) acc[k] = mn.R2[k];
  mont_mul(acc, lds, ls, mn);  // Y' = y R_N (lazy < 2N)
  lds_store_col(lds, ls, acc);
  {
    uint32_t e1[32];
    load_row32(reinterpret_cast<const uint4*>(Ed + ct * 64 + 32), e1);
    to28<32, FBM_NLN>(e1, acc);
  }
  mont_mul(acc, lds, ls, mn);  // u = e1 y (lazy < 2N)
  {
    uint32_t e0[32], y[32], p[32], a[32];
    load_row32(reinterpret_cast<const uint4*>(Ed + ct * 64), e0);
    load_row32(yi, y);
    mullo1024(e0, y, p);
    uint32_t br = 1;  // p = e0 y - 1 (mod 2^1024)
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      const uint64_t d = (uint64_t)p[i] - br;
      p[i] = (uint32_t)d;
      br = (uint32_t)(d >> 63);
    }
    mullo1024(p, jp.Ninv32, a);
    uint32_t a28[FBM_NLN];
    to28<32, FBM_NLN>(a, a28);
    uint32_t c = 0;
#pragma unroll
    for (int k = 0; k < FBM_NLN; ++k) {  // a + u < 3N
      const uint32_t v = acc[k] + a28[k] + c;
      acc[k] = v & FBM_LMASK;
      c = v >> FBM_LB;
    }
  }
  mont_mul(acc, lds, ls, mn);  // w = (a + u) y (lazy < 2N)
  mont_csub(acc, mn.M);
  {  // v = N - w, then N -> 0
    int32_t br = 0;
#pragma unroll
    for (int k = 0; k < FBM_NLN; ++k) {
      const int32_t d = (int32_t)mn.M[k] - (int32_t)acc[k] + br;
      acc[k] = (uint32_t)d & FBM_LMASK;
      br = d >> FBM_LB;
    }
    mont_csub(acc, mn.M);
  }
  if (nude) {  // v <- (v + p y) mod N; p < 2^1036 = R_N, Y' < 2N: p Y' R_N^-1 < 3N
    uint32_t p28[FBM_NLN], p29[FBM_QA_L];
    const uint32_t* nb = nude + (ct >> 8) * (FBM_NUDE_ROWS * 256) + (ct & 255);
#pragma unroll
    for (int k = 0; k < FBM_QA_L; ++k) p29[k] = nb[(FBM_NUDE_D1 + k) * 256];  // jl_nude_kernel's 29-bit digit 1
    relimb_29_28(p29, p28);
    mont_mul(p28, lds, ls, mn);  // p y
    uint32_t c = 0;
#pragma unroll
    for (int k = 0; k < FBM_NLN; ++k) {  // < 4N
      const uint32_t t = acc[k] + p28[k] + c;
      acc[k] = t & FBM_LMASK;
      c = t >> FBM_LB;
    }
    uint32_t n[FBM_NLN];
#pragma unroll
    for (int k = 0; k < FBM_NLN; ++k) n[k] = mn.M[k];
    csub28(acc, n);
    csub28(acc, n);
    csub28(acc, n);
  }
  uint32_t v[32];
  from28<FBM_NLN, 32>(acc, v);
  uint32_t f[64];  // y + N v < N^2
  mul1024(v, jp.N32, f);
  uint32_t y[32];
  load_row32(yi, y);
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 64; ++i) {
    const uint64_t t = (uint64_t)f[i] + (i < 32 ? y[i] : 0u) + c;
    f[i] = (uint32_t)t;
    c = (uint32_t)(t >> 32);
  }
  // The workgroup's rows are one contiguous range of out: staged through LDS in two halves
  // (128 B of every row, padded stride 33 words), each 128-B line is written whole by eight
  // consecutive work-items -- per-lane 16-B row stores left partial lines to the L2, written
  // back up to 3x over at the full vector (tools/pmc_agg.sh).  Every lane has read its Ed row
  // (out may alias it) before the first barrier.
  const uint64_t rows = n_ct - ct0 < FBM_BLOCK ? n_ct - ct0 : FBM_BLOCK;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 32; ++i) lds_a[tid * 33 + i] = f[32 * h + i];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int q = k * FBM_BLOCK + tid;  // 16-B chunk q: row q / 8, chunk q % 8 of its half
      const int r = q >> 3, c4 = (q & 7) * 4;
      if ((uint64_t)r < rows) {
        const uint32_t* src = lds_a + r * 33 + c4;
        *reinterpret_cast<uint4*>(out + (ct0 + r) * 64 + 32 * h + c4) = make_uint4(src[0], src[1], src[2], src[3]);
      }
    }
  }
}

// ------------------------------------------------------------------------------------
// decode + average + dequantise: one work-item per output element
// ------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) jl_decode_kernel(const uint32_t* __restrict__ xs, int es, int cr,
                                                        uint64_t n_out, uint64_t total_weight, double neg_c,
                                                        double step, double* __restrict__ out,
                                                        uint64_t* __restrict__ sums, uint32_t* __restrict__ stats) {
  const uint64_t o = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= n_out) return;
  const uint64_t k = o / (uint64_t)cr;
  const int j = (int)(o - k * (uint64_t)cr);
  const int bit = es * j;
  const uint32_t* x = xs + k * 32;
  unsigned __int128 v = 0;
  const int w0 = bit >> 5, sh = bit & 31;
#pragma unroll
  for (int t = 0; t < 5; ++t) {
    const int w = w0 + t;
    const uint32_t word = (w < 32) ? x[w] : 0u;
    const int pos = 32 * t - sh;
    if (pos >= 0) {
      if (pos < 128) v |= (unsigned __int128)word << pos;
    } else {
      v |= (unsigned __int128)(word >> (-pos));
    }
  }
  if (es < 128) v &= (((unsigned __int128)1) << es) - 1;
  if (sums) {
    sums[2 * o] = (uint64_t)v;
    sums[2 * o + 1] = (uint64_t)(v >> 64);
  }
  if (!out) return;
  const double a = fbm_true_div_u128(v, total_weight);
  if (a >= 18446744073709551616.0) {  // reverse_quantize guard (only when dequantising)
    atomicOr(stats + FBM_STAT_ERRFLAGS, FBM_ERR_DEQUANT_RANGE);
    out[o] = 0.0;
    return;
  }
  out[o] = fbm_dequantize(a, neg_c, step);
}

// ------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------
// CU count of the calling thread's current device, cached per device (a process may drive
// several devices from several threads; 0 = not yet queried, written once per device).
#define FBM_MAX_DEVICES 64
static std::atomic<int> g_num_cu[FBM_MAX_DEVICES];

int device_num_cu() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0) dev = 0;
  if (dev >= FBM_MAX_DEVICES) dev = FBM_MAX_DEVICES - 1;
  int n = g_num_cu[dev].load(std::memory_order_relaxed);
  if (n <= 0) {
    hipDeviceProp_t prop;
    n = (hipGetDeviceProperties(&prop, dev) == hipSuccess) ? prop.multiProcessorCount : 0;
    if (n <= 0) n = 256;
    g_num_cu[dev].store(n, std::memory_order_relaxed);
  }
  return n;
}

uint64_t jl_table_slots() {
  // two workgroups of FBM_BLOCK lanes per CU: 2 waves/SIMD (244 VGPRs per lane in the
  // assembly product; 2 x 75 KB LDS columns per CU)
  return (uint64_t)device_num_cu() * 2 * FBM_BLOCK;
}

static inline dim3 grid1(uint64_t items, unsigned block) { return dim3((unsigned)((items + block - 1) / block)); }

int launch_jl_pack(const void* x, int x_dtype, uint64_t n, const QuantParams& qp, uint64_t weight, int es, int cr,
                   uint64_t n_ct, uint32_t* pt, uint32_t* stats, hipStream_t s) {
  if (n_ct == 0) return FBM_OK;
  if (x_dtype == FBM_F32)
    hipLaunchKernelGGL(jl_pack_kernel<float>, grid1(n_ct * 32, 256), dim3(256), 0, s, (const float*)x, n, qp, weight,
                       es, cr, n_ct, pt, stats);
  else if (x_dtype == FBM_F64)
    hipLaunchKernelGGL(jl_pack_kernel<double>, grid1(n_ct * 32, 256), dim3(256), 0, s, (const double*)x, n, qp,
                       weight, es, cr, n_ct, pt, stats);
  else if (x_dtype == FBM_U128)
    hipLaunchKernelGGL(jl_pack_wide_kernel, grid1(n_ct * 32, 256), dim3(256), 0, s, (const uint64_t*)x, n, es, cr,
                       n_ct, pt, stats);
  else
    hipLaunchKernelGGL(jl_pack_kernel<uint64_t>, grid1(n_ct * 32, 256), dim3(256), 0, s, (const uint64_t*)x, n, qp,
                       weight, es, cr, n_ct, pt, stats);
  return check_launch("jl_pack_kernel");
}

int launch_jl_nude(const uint32_t* pt, uint64_t n_ct, const JlParams& jp, int negative, uint32_t* nude,
                   hipStream_t s) {
  if (n_ct == 0) return FBM_OK;
  hipLaunchKernelGGL(jl_nude_kernel, grid1(n_ct, 256), dim3(256), 0, s, pt, n_ct, jp, negative, nude);
  return check_launch("jl_nude_kernel");
}

int launch_ves_pack(const uint32_t* x, uint64_t n, int wv, int es, int cr, int pw, int sgn, uint32_t* pt,
                    hipStream_t s) {
  const uint64_t n_ct = (n + (uint64_t)cr - 1) / (uint64_t)cr;
  if (n_ct == 0) return FBM_OK;
  hipLaunchKernelGGL(ves_pack_kernel, grid1(n_ct * (uint64_t)pw, 256), dim3(256), 0, s, x, n, wv, es, cr, pw, sgn, n_ct,
                     pt);
  return check_launch("ves_pack_kernel");
}

int launch_ves_unpack(const uint32_t* pt, int pw, int es, int cr, uint64_t n_out, int ow, uint32_t* vals,
                      hipStream_t s) {
  if (n_out == 0) return FBM_OK;
  hipLaunchKernelGGL(ves_unpack_kernel, grid1(n_out * (uint64_t)ow, 256), dim3(256), 0, s, pt, pw, es, cr, n_out, ow,
                     vals);
  return check_launch("ves_unpack_kernel");
}

int launch_jl_fdh_msg_wide(uint64_t n, const uint32_t* t, int tw, int msg_bytes, int kmax, const uint32_t* m32,
                           const uint32_t* k1, const uint32_t* k2, uint32_t mp, int even, uint32_t* H, int hw,
                           uint32_t* stats, hipStream_t s) {
  if (n == 0) return FBM_OK;
  FdhWideArg w;
  memcpy(w.m, m32, sizeof(w.m));
  memcpy(w.k1, k1, sizeof(w.k1));
  memcpy(w.k2, k2, sizeof(w.k2));
  w.mp = mp;
  w.even = even;
  hipLaunchKernelGGL(jl_fdh_msg_wide_kernel, grid1(n, 64), dim3(64), 0, s, n, t, tw, msg_bytes, kmax, w, H, hw, stats);
  return check_launch("jl_fdh_msg_wide_kernel");
}

int launch_jl_fdh_msg(uint64_t n, const uint32_t* t, int tw, int msg_bytes, int kmax, const uint32_t* n32, int even,
                      uint32_t* H, uint32_t* stats, hipStream_t s) {
  if (n == 0) return FBM_OK;
  FdhModArg m;
  memcpy(m.n32, n32, sizeof(m.n32));
  m.even = even;
  hipLaunchKernelGGL(jl_fdh_msg_kernel, grid1(n, 64), dim3(64), 0, s, n, t, tw, msg_bytes, kmax, m, H, stats);
  return check_launch("jl_fdh_msg_kernel");
}

int launch_jl_fdh(uint64_t n_ct, const JlParams& jp, uint32_t* H, uint32_t* stats, hipStream_t s, uint32_t* Hc) {
  if (n_ct == 0) return FBM_OK;
  hipLaunchKernelGGL(jl_fdh_kernel, grid1(n_ct, 256), dim3(256), 0, s, n_ct, jp, H, stats, Hc);
  int rc = check_launch("jl_fdh_kernel");
  if (rc) return rc;
  hipLaunchKernelGGL(jl_fdh_retry_kernel, grid1(n_ct, 64), dim3(64), 0, s, n_ct, jp, H, stats, (const uint32_t*)Hc);
  return check_launch("jl_fdh_retry_kernel");
}

// Per-call device constants: the schedule travels as a kernel argument (copied by the
// runtime at launch, so the host struct may die immediately) and is spilled to device
// memory for the exp kernel, which indexes it dynamically; M and R^2 for the scalar
// loads of the assembly product; broadcast columns of 1 and R^2 (limb k at word k*256,
// read by every lane at offset 0).
__global__ void jl_setup_kernel(JlSched sc, MontCtx mc, MontCtxN mn, NadicCtx na, QuadCtx qa,
                                uint32_t* __restrict__ ops, uint32_t* __restrict__ cst) {
  const int t = threadIdx.x;
  if (t < 128)  // MontCtxN image: M[37] R2[37] mp pad
    cst[FBM_CST_MN + t] = t < FBM_NLN ? mn.M[t] : t < 2 * FBM_NLN ? mn.R2[t - FBM_NLN] : t == 2 * FBM_NLN ? mn.mp : 0u;
  for (int i = t; i < sc.n_ops; i += blockDim.x) ops[i] = sc.op[i];
  if (t < 128) {
    cst[FBM_CST_M + t] = t < FBM_NL ? mc.M[t] : 0u;
    cst[FBM_CST_R2 + t] = t < FBM_NL ? mc.R2[t] : 0u;
    cst[FBM_CST_NK + t] = t < 80 ? na.nk[t] : 0u;
    cst[FBM_CST_NA29 + t] = t < 80 ? na.nk29[t] : 0u;
  }
  if (t < 64) {  // group engines: K'_i and N's 29-bit limbs
    cst[FBM_CST_QK + t] = t < FBM_QA_L ? qa.kp[t] : 0u;
    cst[FBM_CST_QNP + t] = t < FBM_QA_L ? qa.n[t] : 0u;
  }
  if (t < 128) {
    cst[FBM_CST_QR2 + t] = t < 2 * FBM_QA_L ? qa.r2[t] : 0u;
    cst[FBM_CST_QR3 + t] = t < 2 * FBM_QA_L ? qa.r3[t] : 0u;
    cst[FBM_CST_QP + t] = t < 2 * FBM_QA_L && !(t & 1) ? qa.sqp[t >> 1] : 0u;
  }
  for (int i = t; i < FBM_NL * 256; i += blockDim.x) {
    const int k = i >> 8, l = i & 255;
    cst[FBM_CST_ONE + i] = (l == 0 && k == 0) ? 1u : 0u;
  }
}

// the short path's per-call words: |key| and C into the ops buffer, the pairs (D_j, 0) into the
// constants block
__global__ void jl_short_setup_kernel(JlShort sh, uint32_t* __restrict__ ops, uint32_t* __restrict__ cst) {
  const int t = threadIdx.x;
  if (t < 64) ops[FBM_OPS_KW + t] = sh.kw[t];
  if (t < 72) ops[FBM_OPS_CORR + t] = sh.corr[t];
  if (t < 72) ops[FBM_OPS_CBC + t * 256] = sh.corr[t];  // C's broadcast column (the one-lane engine's B)
  if (t < 72) cst[FBM_CST_QD + t] = (t & 1) ? 0u : sh.d[t >> 1];
}

int launch_jl_setup(const JlParams& jp, const JlSched& sc, uint32_t* ops, uint32_t* cst, hipStream_t s,
                    const JlShort* sh) {
  hipLaunchKernelGGL(jl_setup_kernel, dim3(1), dim3(256), 0, s, sc, jp.mc, jp.mn, jp.na, jp.qa, ops, cst);
  int rc = check_launch("jl_setup_kernel");
  if (rc || !sh) return rc;
  hipLaunchKernelGGL(jl_short_setup_kernel, dim3(1), dim3(128), 0, s, *sh, ops, cst);
  return check_launch("jl_short_setup_kernel");
}

// ---- exponentiation engine choice ------------------------------------------------------
// FBM_ENGINE_SINGLE: one lane per ciphertext (throughput: every lane busy, 2 waves/SIMD);
// FBM_ENGINE_QUAD / FBM_ENGINE_TRIPLE: four / three lanes per ciphertext (latency: launches
// below about two thirds of the chip's lane count).  FBM_ENGINE_AUTO picks the engine of least
// modelled time.  A group engine's launch time is set by its busiest SIMD: with w waves' worth
// of work on it (w = workgroups per CU, each workgroup's 4 waves on the CU's 4 SIMDs; beyond
// FBM_GROUP_WAVES resident workgroups the persistent ones loop) it takes about A + B w -- A the
// part of a lone wave's time another wave cannot fill, B a wave's issue time.  Refit on MI355X
// after round 3's cyclic-band square and carry rotation (tools/exp_probe.py, 2043-bit exponent,
// profiles/r3_engine_sweep_cyc.jsonl): triple 13.4 / 23.7 / 33.7 / 44.9 / 54.7 ms at w = 1 … 5
// (A = 3.2, B = 10.3), quad 9.9 / 17.8 / 26.1 / 33.7 / 48.3 at w = 1 / 2 / 3 / 4 / 6 (A = 2.5,
// B = 7.8).  The one-lane engine: 31.7 ms up to one wave per SIMD, 56 ms for a launch of one round
// of two, 50 ms per round of longer launches.  (A build with 4 resident group waves per SIMD,
// -DFBM_GROUP_WAVES=4, measured no faster at w = 4: the issue is already saturated at 3.)
// The policy is per THREAD (round 6): a caller that picks an engine for its launches (the test build's
// fbm_jl_set_engine, include/fbm_secagg_test.h) changes nothing for the process's other threads.  The
// product library never sets it: every launch takes the cost model's engine (FBM_ENGINE_AUTO).
static thread_local int t_engine = FBM_ENGINE_AUTO;

int jl_engine_policy() { return t_engine; }

int jl_engine_set(int mode) {
  const int prev = t_engine;
  t_engine = mode;
  return prev;
}

#define FBM_GROUP_WGS_PER_CU FBM_GROUP_WAVES
static uint64_t group_wgs_max() { return (uint64_t)device_num_cu() * FBM_GROUP_WGS_PER_CU; }
static int group_ct_per_wg(int engine) { return engine == FBM_ENGINE_TRIPLE ? 84 : 64; }

// modelled launch time (ms) of n_ct ciphertexts on one engine (relative ranking only); refit on the
// short path (profiles/r3_engine_sweep_short.jsonl): triple 12.3 / 23.1 / 33.0 / 42.9 / 52.7 ms at
// w = 1 … 5, quad 9.4 / 17.1 / 24.8 / 32.5 / 46.6 at w = 1 / 2 / 3 / 4 / 6; the one-lane engine with its
// unrolled square (profiles/r3_unroll_ab.jsonl) 27.2 (lone waves), 49 (one round of two), then ~45.5 per
// round (a tail of at most half a round: ~23)
static double engine_model_ms(int engine, uint64_t n_ct) {
  const uint64_t ncu = (uint64_t)device_num_cu();
  if (engine == FBM_ENGINE_SINGLE) {
    const uint64_t lanes = ncu * 2 * FBM_BLOCK;
    if (n_ct <= lanes / 2) return 27.2;
    if (n_ct <= lanes) return 49.0;
    const uint64_t part = n_ct % lanes;
    return 45.5 * (double)(n_ct / lanes) + (part == 0 ? 0.0 : part <= lanes / 2 ? 23.0 : 45.5);
  }
  const uint64_t wgs = (n_ct + group_ct_per_wg(engine) - 1) / group_ct_per_wg(engine);
  const uint64_t w = (wgs + ncu - 1) / ncu;
  const double A = engine == FBM_ENGINE_TRIPLE ? 2.2 : 1.7, B = engine == FBM_ENGINE_TRIPLE ? 10.1 : 7.7;
  return A + B * (double)w;
}

int jl_engine_for(uint64_t n_ct) {
  const int e = jl_engine_policy();
  if (e != FBM_ENGINE_AUTO) return e;
  int best = FBM_ENGINE_SINGLE;
  double tb = engine_model_ms(FBM_ENGINE_SINGLE, n_ct);
  for (int g : {FBM_ENGINE_QUAD, FBM_ENGINE_TRIPLE}) {
    const double t = engine_model_ms(g, n_ct);
    if (t < tb) {
      tb = t;
      best = g;
    }
  }
  return best;
}

uint64_t jl_table_bytes(uint64_t n_ct) {
  const uint64_t cap = jl_table_slots();
  uint64_t g = ((n_ct + 255) / 256) * 256;
  uint64_t need = (g < cap ? g : cap) * FBM_TENTRIES * FBM_NL * 4;
  for (int e : {FBM_ENGINE_QUAD, FBM_ENGINE_TRIPLE}) {
    uint64_t w = (n_ct + group_ct_per_wg(e) - 1) / group_ct_per_wg(e);
    if (w > group_wgs_max()) w = group_wgs_max();
    const uint64_t m = e == FBM_ENGINE_TRIPLE ? FBM_TA_LIMBS : FBM_QA_LIMBS;
    const uint64_t b = w * FBM_TENTRIES * 2 * m * 256 * 4;
    if (b > need) need = b;
  }
  return need;
}

// ---- batched one-lane exponentiations (fbm_jl_batch_begin / _flush, include/fbm_secagg.h) ----
struct JlBatchState {
  bool active = false;
  bool accept = false;  // set by the phase-2 entry points only (jl_batch_accept): other calls launch
  JlExpBatch bt;
  const uint32_t* cst = nullptr;  // the first segment's constants block (all segments: same N), or
                                  // the first short-path segment's (short_cst)
  bool short_cst = false;
  uint32_t n32[32];
  uint32_t np = 0;
};
static thread_local JlBatchState g_batch;

bool jl_batch_active() { return g_batch.active; }

int jl_batch_begin() {
  if (g_batch.active) {
    set_error("fbm_jl_batch_begin: a batch is already open on this thread");
    return FBM_E_ARG;
  }
  memset(&g_batch.bt, 0, sizeof(g_batch.bt));
  g_batch.cst = nullptr;
  g_batch.short_cst = false;
  g_batch.active = true;
  return FBM_OK;
}

void jl_batch_abort() { g_batch.active = false; }

int jl_batch_count() { return g_batch.active ? g_batch.bt.nseg : 0; }

bool jl_batch_accept(bool on) {
  const bool prev = g_batch.accept;
  g_batch.accept = on;
  return prev;
}

static int jl_batch_record(const uint32_t* H, uint64_t n_ct, const JlParams& jp, const JlSched& sc, int mode,
                           const uint32_t* nude, const uint32_t* ops, const uint32_t* cst, uint32_t* out,
                           const uint32_t* Hc) {
  JlExpBatch& bt = g_batch.bt;
  if (n_ct == 0) return FBM_OK;
  if (bt.nseg >= FBM_EXP_MAXSEG) {
    set_error("a JL exponentiation batch holds at most %d calls", FBM_EXP_MAXSEG);
    return FBM_E_UNSUPPORTED;
  }
  if (bt.nseg == 0) {
    g_batch.cst = cst;
    memcpy(g_batch.n32, jp.N32, sizeof(g_batch.n32));
    g_batch.np = jp.qa.np;
  } else if (memcmp(g_batch.n32, jp.N32, sizeof(g_batch.n32)) != 0) {
    set_error("every call of a JL exponentiation batch must use the same biprime");
    return FBM_E_ARG;
  }
  // the launch reads the short product's pairs (D_j, 0) -- a function of N alone -- from one
  // constants block: the first segment's whose setup wrote them (a short-path schedule), not
  // merely the first segment's (that call may have run with the short path off)
  if (sc.sbits >= 0 && !g_batch.short_cst) {
    g_batch.short_cst = true;
    g_batch.cst = cst;
  }
  const uint64_t chunks = (n_ct + FBM_BLOCK - 1) / FBM_BLOCK;
  if ((uint64_t)bt.total_chunks + chunks > 0xFFFFFFFFull) {
    set_error("JL exponentiation batch too large");
    return FBM_E_UNSUPPORTED;
  }
  bt.seg[bt.nseg++] =
      JlExpSeg{H, Hc, nude, out, ops, n_ct, bt.total_chunks, sc.n_ops, sc.first, mode, jp.key_is_zero, sc.sbits};
  bt.total_chunks += (uint32_t)chunks;
  return FBM_OK;
}

uint64_t jl_batch_workspace() { return 256 + 4096 + jl_table_slots() * (uint64_t)FBM_TENTRIES * FBM_NL * 4; }

// the batch's segment table into device memory (a kernel argument -> the batch workspace) and
// the chunk counter zeroed
__global__ void jl_batch_desc_kernel(JlExpBatch bt, JlExpSeg* __restrict__ segs, uint32_t* __restrict__ ctr) {
  const int t = threadIdx.x;
  if (t < bt.nseg) segs[t] = bt.seg[t];
  if (t == 0) ctr[0] = 0u;
}

int launch_jl_exp(const uint32_t* H, uint64_t n_ct, const JlParams& jp, const JlSched& sc, int mode,
                  const uint32_t* nude, uint32_t* table, uint64_t table_slots, const uint32_t* ops,
                  const uint32_t* cst, uint32_t* out, hipStream_t s, const uint32_t* Hc) {
  if (n_ct == 0) return FBM_OK;
  if (g_batch.active && g_batch.accept) return jl_batch_record(H, n_ct, jp, sc, mode, nude, ops, cst, out, Hc);
  const int eng = jl_engine_for(n_ct);
  if (eng == FBM_ENGINE_QUAD || eng == FBM_ENGINE_TRIPLE) {
    uint64_t g = (n_ct + group_ct_per_wg(eng) - 1) / group_ct_per_wg(eng);
    // Workgroups launched per CU (each pulls chunks until none are left).  Up to four chunks per CU, two
    // resident workgroups finish first: the aggregate's 1/4 stripe (83 334 ciphertexts) 43.0 -> 40.8 ms,
    // 64 512 ciphertexts 33.7 -> 31.1 (triple) and 32.9 -> 30.6 (quad); past that three (100 000: 51.8
    // against 60.3) -- profiles/r5bm_group_wgs.jsonl.  FBM_GROUP_WGS = 1..3 overrides (A/B).
#ifdef FBM_AB_KNOBS  // A/B builds only (python -m fedbiomed_amd._build --out ... -DFBM_AB_KNOBS)
    static const uint64_t wgs_env = getenv("FBM_GROUP_WGS") ? (uint64_t)atoi(getenv("FBM_GROUP_WGS")) : 0u;
#else
    constexpr uint64_t wgs_env = 0u;
#endif
    const uint64_t ncu = (uint64_t)device_num_cu();
    const uint64_t wgs_cu = wgs_env >= 1 && wgs_env <= FBM_GROUP_WGS_PER_CU ? wgs_env : g <= 4 * ncu ? 2u : 3u;
    if (g > ncu * wgs_cu) g = ncu * wgs_cu;
    // probe knob (A/B of workgroup placement): extra dynamic LDS per workgroup, e.g. enough to hold a
    // group launch to two workgroups per CU
#ifdef FBM_AB_KNOBS
    static const unsigned glds_pad = getenv("FBM_GROUP_LDS_PAD") ? (unsigned)atoi(getenv("FBM_GROUP_LDS_PAD")) : 0u;
#else
    constexpr unsigned glds_pad = 0u;
#endif
    if (eng == FBM_ENGINE_QUAD) {
      hipLaunchKernelGGL(jl_expg_kernel<4>, dim3((unsigned)g), dim3(FBM_QBLOCK), glds_pad, s, H, n_ct, (uint32_t*)cst,
                         jp.qa.np, ops, sc.n_ops, sc.first, mode, jp.key_is_zero, sc.sbits, nude, table, out, Hc);
      return check_launch("jl_expq_kernel");
    }
    hipLaunchKernelGGL(jl_expg_kernel<3>, dim3((unsigned)g), dim3(FBM_QBLOCK), glds_pad, s, H, n_ct, (uint32_t*)cst,
                       jp.qa.np, ops, sc.n_ops, sc.first, mode, jp.key_is_zero, sc.sbits, nude, table, out, Hc);
    return check_launch("jl_expt_kernel");
  }
  uint64_t g = (n_ct + FBM_BLOCK - 1) / FBM_BLOCK;
  const uint64_t gmax = table_slots / FBM_BLOCK;
  if (g > gmax) g = gmax;
  // probe knob (tools/mixed_probe.py): extra dynamic LDS per workgroup, e.g. enough to hold the
  // one-lane engine to one workgroup per CU
#ifdef FBM_AB_KNOBS
  static const unsigned lds_pad = getenv("FBM_EXP_LDS_PAD") ? (unsigned)atoi(getenv("FBM_EXP_LDS_PAD")) : 0u;
#else
  constexpr unsigned lds_pad = 0u;
#endif
  hipLaunchKernelGGL(jl_exp_kernel<false>, dim3((unsigned)g), dim3(FBM_BLOCK), lds_pad, s, H, n_ct, (uint32_t*)cst, jp.qa.np,
                     ops, sc.n_ops, sc.first, mode, jp.key_is_zero, sc.sbits, nude, table, out, (const JlExpSeg*)nullptr,
                     0, 0u, (uint32_t*)nullptr, Hc);
  return check_launch("jl_exp_kernel");
}

int jl_batch_flush(void* workspace, uint64_t ws_bytes, hipStream_t s) {
  if (!g_batch.active) {
    set_error("fbm_jl_batch_flush: no open batch on this thread");
    return FBM_E_ARG;
  }
  g_batch.active = false;
  const JlExpBatch& bt = g_batch.bt;
  if (bt.nseg == 0) return FBM_OK;
  if (!workspace || ws_bytes < jl_batch_workspace()) {
    set_error("fbm_jl_batch_flush: workspace of %llu bytes needed", (unsigned long long)jl_batch_workspace());
    return FBM_E_ARG;
  }
  // workspace: counter (word 0) | segment table (at 256) | exponent tables (at 256 + 4 KB)
  uint32_t* ctr = (uint32_t*)workspace;
  JlExpSeg* segs = (JlExpSeg*)((uint8_t*)workspace + 256);
  uint32_t* table = (uint32_t*)((uint8_t*)workspace + 256 + 4096);
  hipLaunchKernelGGL(jl_batch_desc_kernel, dim3(1), dim3(64), 0, s, bt, segs, ctr);
  int rc = check_launch("jl_batch_desc_kernel");
  if (rc) return rc;
  uint64_t g = bt.total_chunks;
  const uint64_t gmax = jl_table_slots() / FBM_BLOCK;
  if (g > gmax) g = gmax;
  hipLaunchKernelGGL(jl_exp_kernel<true>, dim3((unsigned)g), dim3(FBM_BLOCK), 0, s, (const uint32_t*)nullptr, (uint64_t)0,
                     (uint32_t*)g_batch.cst, g_batch.np, (const uint32_t*)nullptr, 0, 0, 0, 0, -1, (const uint32_t*)nullptr,
                     table, (uint32_t*)nullptr, (const JlExpSeg*)segs, bt.nseg, bt.total_chunks, ctr, (const uint32_t*)nullptr);
  return check_launch("jl_exp_kernel (batch)");
}

int launch_jl_encf(const uint32_t* pt, uint64_t n_ct, const JlParams& jp, const uint32_t* cst, int negative,
                   const uint32_t* factor, uint32_t* out, hipStream_t s) {
  if (n_ct == 0) return FBM_OK;
  hipLaunchKernelGGL(jl_encf_kernel, grid1(n_ct, FBM_BLOCK), dim3(FBM_BLOCK), 0, s, pt, n_ct, cst, jp, negative, factor,
                     out);
  return check_launch("jl_encf_kernel");
}

int launch_jl_prod(const uint32_t* cts, int n_parties, uint64_t n_ct, const JlParams& jp, const uint32_t* cst,
                   const uint32_t* factor, uint32_t* xout, hipStream_t s) {
  if (n_ct == 0) return FBM_OK;
  hipLaunchKernelGGL(jl_prod_kernel, grid1(n_ct, FBM_BLOCK), dim3(FBM_BLOCK), 0, s, cts, n_parties, n_ct, cst, jp,
                     factor, xout);
  return check_launch("jl_prod_kernel");
}

__global__ void jl_rk_kernel(JlRk rk, uint32_t* __restrict__ cst) {
  const int t = threadIdx.x;
  if (t < 128) cst[FBM_CST_RK + t] = t < FBM_NL ? rk.w[t] : 0u;
}

int launch_jl_rk(const JlRk& rk, uint32_t* cst, hipStream_t s) {
  hipLaunchKernelGGL(jl_rk_kernel, dim3(1), dim3(128), 0, s, rk, cst);
  return check_launch("jl_rk_kernel");
}

int launch_jl_inv(uint64_t n_ct, const JlParams& jp, const uint32_t* cst, const uint32_t* Ed, uint32_t* Y,
                  const uint32_t* nude, uint32_t* out, uint32_t* stats, hipStream_t s) {
  if (n_ct == 0) return FBM_OK;
  hipLaunchKernelGGL(jl_inv_modn_kernel, grid1(n_ct, FBM_BLOCK), dim3(FBM_BLOCK), 0, s, n_ct, jp, Ed, 64, Y, stats);
  int rc = check_launch("jl_inv_modn_kernel");
  if (rc) return rc;
  hipLaunchKernelGGL(jl_lift_kernel, grid1(n_ct, FBM_BLOCK), dim3(FBM_BLOCK), 0, s, n_ct, jp, cst, Ed, Y, nude, out);
  return check_launch("jl_lift_kernel");
}

// host test hook (fbm_test_fdh_gcd, include/fbm_secagg.h): the device's one-digest gcd test
int host_gcd_is_one_r8(const uint32_t* r8, const uint32_t* n32, uint32_t* err) {
  uint32_t r[8];
  for (int i = 0; i < 8; ++i) r[i] = r8[i];
  uint32_t e = 0;
  const bool ok = gcd_is_one_r8(r, n32, e);
  *err = e;
  return ok ? 1 : 0;
}

int launch_jl_decode(const uint32_t* xs, int es, int cr, uint64_t n_out, uint64_t total_weight, double neg_c,
                     double step, double* out, uint64_t* sums, uint32_t* stats, hipStream_t s) {
  if (n_out == 0) return FBM_OK;
  hipLaunchKernelGGL(jl_decode_kernel, grid1(n_out, 256), dim3(256), 0, s, xs, es, cr, n_out, total_weight, neg_c,
                     step, out, sums, stats);
  return check_launch("jl_decode_kernel");
}

// multiply / divide of the reference's secagg utils (_secagg_utils.py:122-149: [e * k], [e / k]) on
// (lo, hi) uint64 pairs v < 2^128:
//   op 0: v * k, k < 2^64 -> (w0, w1, w2) uint64 words of the exact product (< 2^192; the host
//         applies the sign of a negative weight)
//   op 1: v / k, 1 <= k < 2^64, Python's int/int true division (correctly rounded float64)
//   op 2: v / kd, kd = the float64 whose bits k holds: Python's int / float (float(v), correctly
//         rounded, then the IEEE division)
//   op 3: -(v / k), the int/int division by a negative divisor -k
__global__ void __launch_bounds__(256) int_ops_kernel(const uint64_t* __restrict__ x, uint64_t n, uint64_t k, int op,
                                                      uint64_t* __restrict__ prod, double* __restrict__ quot,
                                                      uint32_t* __restrict__ stats) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t lo = x[2 * i], hi = x[2 * i + 1];
  const unsigned __int128 v = ((unsigned __int128)hi << 64) | lo;
  if (op == 1 || op == 3) {
    const double q = fbm_true_div_u128(v, k);
    quot[i] = op == 3 ? -q : q;
    return;
  }
  if (op == 2) {
    double kd;
    memcpy(&kd, &k, sizeof(kd));
    quot[i] = fbm_true_div_u128(v, 1) / kd;  // float(v) (round to nearest even), then one division
    return;
  }
  const unsigned __int128 pl = (unsigned __int128)lo * k, ph = (unsigned __int128)hi * k;
  const unsigned __int128 mid = (pl >> 64) + (uint64_t)ph;
  prod[3 * i] = (uint64_t)pl;
  prod[3 * i + 1] = (uint64_t)mid;
  prod[3 * i + 2] = (uint64_t)(ph >> 64) + (uint64_t)(mid >> 64);
}

// v / k for an integer k >= 2^64 (utils.divide with a wide divisor, _secagg_utils.py:137-149): Python's
// correctly rounded int / int true division (round half to even, subnormal results rounded once) of
// v < 2^128.  q = floor(v 2^s / k) with s chosen so q has 55 or 56 bits, by 56 steps of restoring long
// division on the divisor's limbs (at most 38 words: a divisor of more than 1 204 bits makes every
// quotient round to 0 -- the host passes zero_all); then round q at the result's ulp.
struct KBig {
  uint32_t w[40];  // |k|, little-endian words (bits <= 1204)
  int words, bits, negative, zero_all;
};
// one value (__host__ too: the CPU suite checks it against Python's division through fbm_test_true_div_big)
__host__ __device__ inline double true_div_big(uint64_t lo, uint64_t hi, const KBig& kb) {
  const double sign = kb.negative ? -1.0 : 1.0;
  const int la = hi ? 128 - __builtin_clzll(hi) : (lo ? 64 - __builtin_clzll(lo) : 0);
  if (la == 0 || kb.zero_all || kb.bits - la >= 1076)  // v / k < 2^-1075: rounds to (signed) zero
    return sign * 0.0;
  constexpr int W = 42;  // the divisor (<= 1 204 bits) shifted left by at most 9, plus a spare word
  uint32_t a[4] = {(uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32)};
  const int s = 55 - (la - kb.bits);  // q = floor(v 2^s / k) in [2^54, 2^56); s >= -9 (v < 2^128 <= k 2^64)
  // B = k << max(-s, 0); the numerator X = v << max(s, 0), consumed a bit at a time from bit 55 down
  uint32_t B[W], Y[W];
  const int bs = s < 0 ? -s : 0, xs = s > 0 ? s : 0;
  for (int j = 0; j < W; ++j) {
    const int src = j;  // B[j] = (k << bs) word j
    const uint32_t cur = src < kb.words ? kb.w[src] : 0u;
    const uint32_t prev = src - 1 >= 0 && src - 1 < kb.words ? kb.w[src - 1] : 0u;
    B[j] = bs ? (cur << bs) | (prev >> (32 - bs)) : cur;
  }
  // Y = X >> 56 = v << (xs - 56) (or v >> (56 - xs)), word by word
  for (int j = 0; j < W; ++j) {
    const int sh = xs - 56;  // bit shift of v into Y
    uint32_t w = 0;
    for (int b = 0; b < 32; ++b) {  // bit (32 j + b) of Y = bit (32 j + b - sh) of v
      const int vb = 32 * j + b - sh;
      if (vb >= 0 && vb < 128 && ((a[vb >> 5] >> (vb & 31)) & 1u)) w |= 1u << b;
    }
    Y[j] = w;
  }
  uint64_t q = 0;
  for (int t = 55; t >= 0; --t) {
    uint32_t carry = 0;  // Y = 2 Y + bit t of X
    for (int j = 0; j < W; ++j) {
      const uint32_t nc = Y[j] >> 31;
      Y[j] = (Y[j] << 1) | carry;
      carry = nc;
    }
    const int vb = t - xs;
    if (vb >= 0 && vb < 128 && ((a[vb >> 5] >> (vb & 31)) & 1u)) Y[0] |= 1u;
    int cmp = 0;
    for (int j = W - 1; j >= 0 && cmp == 0; --j) cmp = (Y[j] > B[j]) - (Y[j] < B[j]);
    if (cmp >= 0) {
      uint32_t br = 0;
      for (int j = 0; j < W; ++j) {
        const uint64_t d = (uint64_t)Y[j] - B[j] - br;
        Y[j] = (uint32_t)d;
        br = (uint32_t)(d >> 63);
      }
      q |= 1ull << t;
    }
  }
  uint32_t rem = 0;
  for (int j = 0; j < W; ++j) rem |= Y[j];
  const int lq = 64 - __builtin_clzll(q);
  const int E = lq - 1 - s;                       // floor(log2(v / k))
  const int ulp = (E < -1022 ? -1022 : E) - 52;  // the result's ulp: 2^ulp
  const int drop = ulp + s;                       // low bits of q below the ulp (>= 2)
  uint64_t m = drop >= 64 ? 0ull : q >> drop;
  const uint64_t rbit = drop - 1 >= 64 ? 0ull : (q >> (drop - 1)) & 1ull;
  const bool sticky = rem != 0u || (drop - 1 >= 64 ? q != 0ull : (q & ((1ull << (drop - 1)) - 1ull)) != 0ull);
  if (rbit && (sticky || (m & 1ull))) ++m;
#ifdef __HIP_DEVICE_COMPILE__
  return sign * ldexp((double)m, ulp);
#else
  return sign * __builtin_ldexp((double)m, ulp);
#endif
}

__global__ void __launch_bounds__(256) int_true_div_big_kernel(const uint64_t* __restrict__ x, uint64_t n, KBig kb,
                                                               double* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = true_div_big(x[2 * i], x[2 * i + 1], kb);
}

static KBig kbig_of(const uint32_t* k, int k_words, int negative) {
  KBig kb;
  memset(&kb, 0, sizeof(kb));
  kb.negative = negative;
  int bits = 0;
  for (int i = k_words - 1; i >= 0; --i)
    if (k[i]) {
      bits = 32 * i + 32 - __builtin_clz(k[i]);
      break;
    }
  if (bits > 40 * 32 - 32) {  // > 1 248 bits: every quotient of a v < 2^128 is below 2^-1120
    kb.zero_all = 1;
  } else {
    kb.words = (bits + 31) / 32;
    for (int i = 0; i < kb.words; ++i) kb.w[i] = k[i];
    kb.bits = bits;
  }
  return kb;
}

int launch_int_true_div_big(const uint64_t* x, uint64_t n, const uint32_t* k, int k_words, int negative, double* out,
                            hipStream_t s) {
  if (n == 0) return FBM_OK;
  const KBig kb = kbig_of(k, k_words, negative);
  hipLaunchKernelGGL(int_true_div_big_kernel, grid1(n, 256), dim3(256), 0, s, x, n, kb, out);
  return check_launch("int_true_div_big_kernel");
}

void host_true_div_big(const uint64_t* x, uint64_t n, const uint32_t* k, int k_words, int negative, double* out) {
  const KBig kb = kbig_of(k, k_words, negative);
  for (uint64_t i = 0; i < n; ++i) out[i] = true_div_big(x[2 * i], x[2 * i + 1], kb);
}

int launch_int_ops(const uint64_t* x, uint64_t n, uint64_t k, int op, uint64_t* prod, double* quot, uint32_t* stats,
                   hipStream_t s) {
  if (n == 0) return FBM_OK;
  hipLaunchKernelGGL(int_ops_kernel, grid1(n, 256), dim3(256), 0, s, x, n, k, op, prod, quot, stats);
  return check_launch("int_ops_kernel");
}

}  // namespace fbm
