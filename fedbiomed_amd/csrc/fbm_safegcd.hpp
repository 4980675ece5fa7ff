// fedbiomed_amd -- modular inverse mod an odd N < 2^1024 by Bernstein-Yang divsteps
// ("Fast constant-time gcd computation and modular inversion", 2019), for the server-key
// inverse of ServerKey.decrypt (reference fedbiomed/common/secagg/_jls.py:550-551: gmpy2
// powmod with a negative exponent inverts first).
//
// Why: a per-lane binary extended Euclid branches on the data (lanes of a wave take
// different paths every iteration) and needs four 1024-bit arrays in flight; divsteps are
// branch-free, and 30 of them at a time run on one 32-bit word, leaving only a 2x2 matrix
// product on the full-width numbers per batch.
//
// Representation: signed 30-bit limbs, value = sum l[i] 2^(30 i), l[0..33] in [0, 2^30),
// l[34] signed (35 limbs = 1050 bits).  Invariants (x the input, all mod N):
//   d*x == f,  e*x == g;   f odd;   start f = N, g = x, d = 0, e = 1, delta = 1.
// Each batch: 30 divsteps on the low words give T = [u v; q r] with
//   [f'; g'] = T [f; g] / 2^30   (exact),   [d'; e'] = (T [d; e] + [md; me] N) / 2^30
// where md, me make the division exact (md = -(u d0 + v e0) / N mod 2^30) and start from
// (u if d < 0) + (v if e < 0), which keeps d, e within (-2N, N).  When g == 0, f = +-gcd;
// gcd == 1 gives x^-1 = +-d mod N.  __host__ __device__: the same code is unit-tested on the
// host through fbm_test_modinv (include/fbm_secagg.h).
#pragma once
#include <stdint.h>

#define FBM_S30 35
#define FBM_M30 0x3FFFFFFF
// batches of 30 divsteps: the constant-time bound for 1024-bit operands is
// ceil((49 * 1024 + 57) / 17) = 2955 divsteps = 99 batches
#define FBM_INV_MAX_BATCHES 100

struct FbmN30 {
  int32_t n[FBM_S30];  // N in signed-30 limbs (all non-negative)
  uint32_t ninv;       // N^-1 mod 2^30
};

__host__ __device__ inline void fbm_to_s30(const uint32_t* w32, int nw, int32_t (&o)[FBM_S30]) {
  #pragma unroll
  for (int i = 0; i < FBM_S30; ++i) {
    const int bit = 30 * i;
    const int wi = bit >> 5, sh = bit & 31;
    const uint64_t lo = (wi < nw) ? w32[wi] : 0u;
    const uint64_t hi = (wi + 1 < nw) ? w32[wi + 1] : 0u;
    o[i] = (int32_t)((((hi << 32) | lo) >> sh) & FBM_M30);
  }
}

// non-negative value < 2^1024 in signed-30 limbs (normalised) -> 32 little-endian words
__host__ __device__ inline void fbm_from_s30(const int32_t (&a)[FBM_S30], uint32_t* w32) {
  #pragma unroll
  for (int i = 0; i < 32; ++i) {
    const int bit = 32 * i;
    const int k = bit / 30, sh = bit % 30;
    uint64_t v = (uint64_t)(uint32_t)a[k] >> sh;
    if (k + 1 < FBM_S30) v |= (uint64_t)(uint32_t)a[k + 1] << (30 - sh);
    if (k + 2 < FBM_S30) v |= (uint64_t)(uint32_t)a[k + 2] << (60 - sh);
    w32[i] = (uint32_t)v;
  }
}

// 30 divsteps on the low words; returns the new delta, writes T
__host__ __device__ inline int32_t fbm_divsteps30(int32_t delta, uint32_t f, uint32_t g, int32_t& tu, int32_t& tv,
                                                  int32_t& tq, int32_t& tr) {
  uint32_t u = 1, v = 0, q = 0, r = 1;
  #pragma unroll
  for (int i = 0; i < 30; ++i) {
    // swap when delta > 0 and g odd: (f, g) <- (g, -f), (u, v, q, r) <- (q, r, -u, -v), delta <- -delta
    const uint32_t odd = 0u - (g & 1u);
    const uint32_t sw = odd & (delta > 0 ? 0xFFFFFFFFu : 0u);
    delta = (int32_t)(((uint32_t)delta ^ sw) - sw);
    const uint32_t nf = f ^ ((f ^ g) & sw);
    const uint32_t ng = (g & ~sw) | ((0u - f) & sw);
    const uint32_t nu = u ^ ((u ^ q) & sw), nv = v ^ ((v ^ r) & sw);
    const uint32_t nq = (q & ~sw) | ((0u - u) & sw), nr = (r & ~sw) | ((0u - v) & sw);
    f = nf;
    g = ng;
    u = nu;
    v = nv;
    q = nq;
    r = nr;
    // g odd: g <- (g + f)/2, (q, r) += (u, v);  always: (u, v) <<= 1, delta += 1
    g = (g + (f & odd)) >> 1;
    q += u & odd;
    r += v & odd;
    u <<= 1;
    v <<= 1;
    delta += 1;
  }
  tu = (int32_t)u;
  tv = (int32_t)v;
  tq = (int32_t)q;
  tr = (int32_t)r;
  return delta;
}

__host__ __device__ inline void fbm_update_fg(int32_t (&f)[FBM_S30], int32_t (&g)[FBM_S30], int32_t u, int32_t v,
                                              int32_t q, int32_t r) {
  int64_t cf = (int64_t)u * f[0] + (int64_t)v * g[0];
  int64_t cg = (int64_t)q * f[0] + (int64_t)r * g[0];
  cf >>= 30;
  cg >>= 30;
  #pragma unroll
  for (int i = 1; i < FBM_S30; ++i) {
    cf += (int64_t)u * f[i] + (int64_t)v * g[i];
    cg += (int64_t)q * f[i] + (int64_t)r * g[i];
    f[i - 1] = (int32_t)(cf & FBM_M30);
    g[i - 1] = (int32_t)(cg & FBM_M30);
    cf >>= 30;
    cg >>= 30;
  }
  f[FBM_S30 - 1] = (int32_t)cf;
  g[FBM_S30 - 1] = (int32_t)cg;
}

__host__ __device__ inline void fbm_update_de(int32_t (&d)[FBM_S30], int32_t (&e)[FBM_S30], int32_t u, int32_t v,
                                              int32_t q, int32_t r, const FbmN30& N) {
  const int32_t sd = d[FBM_S30 - 1] >> 31, se = e[FBM_S30 - 1] >> 31;  // -1 if negative
  int32_t md = (u & sd) + (v & se);
  int32_t me = (q & sd) + (r & se);
  int64_t cd = (int64_t)u * d[0] + (int64_t)v * e[0];
  int64_t ce = (int64_t)q * d[0] + (int64_t)r * e[0];
  md -= (int32_t)((N.ninv * (uint32_t)cd + (uint32_t)md) & FBM_M30);
  me -= (int32_t)((N.ninv * (uint32_t)ce + (uint32_t)me) & FBM_M30);
  cd += (int64_t)N.n[0] * md;
  ce += (int64_t)N.n[0] * me;
  cd >>= 30;
  ce >>= 30;
  #pragma unroll
  for (int i = 1; i < FBM_S30; ++i) {
    cd += (int64_t)u * d[i] + (int64_t)v * e[i] + (int64_t)N.n[i] * md;
    ce += (int64_t)q * d[i] + (int64_t)r * e[i] + (int64_t)N.n[i] * me;
    d[i - 1] = (int32_t)(cd & FBM_M30);
    e[i - 1] = (int32_t)(ce & FBM_M30);
    cd >>= 30;
    ce >>= 30;
  }
  d[FBM_S30 - 1] = (int32_t)cd;
  e[FBM_S30 - 1] = (int32_t)ce;
}

__host__ __device__ inline bool fbm_s30_is_zero(const int32_t (&a)[FBM_S30]) {
  int32_t acc = 0;
  #pragma unroll
  for (int i = 0; i < FBM_S30; ++i) acc |= a[i];
  return acc == 0;
}

// a <- a + s * N  (s in {-1, 0, 1}), renormalising the limbs
__host__ __device__ inline void fbm_s30_add_n(int32_t (&a)[FBM_S30], int32_t s, const FbmN30& N) {
  int64_t c = 0;
  #pragma unroll
  for (int i = 0; i < FBM_S30 - 1; ++i) {
    c += (int64_t)a[i] + (int64_t)s * N.n[i];
    a[i] = (int32_t)(c & FBM_M30);
    c >>= 30;
  }
  a[FBM_S30 - 1] = (int32_t)(c + a[FBM_S30 - 1] + (int64_t)s * N.n[FBM_S30 - 1]);
}

// a <- -a (normalised)
__host__ __device__ inline void fbm_s30_neg(int32_t (&a)[FBM_S30]) {
  int64_t c = 0;
  #pragma unroll
  for (int i = 0; i < FBM_S30 - 1; ++i) {
    c -= a[i];
    a[i] = (int32_t)(c & FBM_M30);
    c >>= 30;
  }
  a[FBM_S30 - 1] = (int32_t)(c - a[FBM_S30 - 1]);
}

// compare a (normalised, non-negative) with N: a >= N
__host__ __device__ inline bool fbm_s30_ge_n(const int32_t (&a)[FBM_S30], const FbmN30& N) {
  int cmp = 0;
  #pragma unroll
  for (int i = FBM_S30 - 1; i >= 0; --i)
    if (cmp == 0) cmp = (a[i] > N.n[i]) - (a[i] < N.n[i]);
  return cmp >= 0;
}

// One lane's state; `fbm_modinv_batch` advances it by one batch.
struct FbmInvState {
  int32_t f[FBM_S30], g[FBM_S30], d[FBM_S30], e[FBM_S30];
  int32_t delta;
};

__host__ __device__ inline void fbm_modinv_init(FbmInvState& s, const uint32_t* x32, const FbmN30& N) {
  #pragma unroll
  for (int i = 0; i < FBM_S30; ++i) {
    s.f[i] = N.n[i];
    s.d[i] = 0;
    s.e[i] = i == 0 ? 1 : 0;
  }
  fbm_to_s30(x32, 32, s.g);
  s.delta = 1;
}

__host__ __device__ inline void fbm_modinv_batch(FbmInvState& s, const FbmN30& N) {
  int32_t u, v, q, r;
  s.delta = fbm_divsteps30(s.delta, (uint32_t)s.f[0], (uint32_t)s.g[0], u, v, q, r);
  fbm_update_de(s.d, s.e, u, v, q, r, N);
  fbm_update_fg(s.f, s.g, u, v, q, r);
}

// After g == 0: out = x^-1 mod N (32 words); returns false if gcd(x, N) != 1.
__host__ __device__ inline bool fbm_modinv_finish(FbmInvState& s, const FbmN30& N, uint32_t* out32) {
  // f = +-1 ?
  const int32_t sf = s.f[FBM_S30 - 1] >> 31;
  int32_t rest = 0;
  #pragma unroll
  for (int i = 1; i < FBM_S30 - 1; ++i) rest |= s.f[i];
  const bool pos_one = s.f[0] == 1 && rest == 0 && s.f[FBM_S30 - 1] == 0;
  // -1 in normalised signed-30: low limbs all 2^30 - 1, top limb -1
  int32_t all = FBM_M30;
  #pragma unroll
  for (int i = 0; i < FBM_S30 - 1; ++i) all &= s.f[i];
  const bool neg_one = sf == -1 && all == FBM_M30 && s.f[FBM_S30 - 1] == -1;
  if (!pos_one && !neg_one) return false;
  if (neg_one) fbm_s30_neg(s.d);
  // d in about (-2N, 2N): bring into [0, N)
  #pragma unroll
  for (int k = 0; k < 4; ++k)
    if (s.d[FBM_S30 - 1] < 0) fbm_s30_add_n(s.d, 1, N);
  #pragma unroll
  for (int k = 0; k < 4; ++k)
    if (fbm_s30_ge_n(s.d, N)) fbm_s30_add_n(s.d, -1, N);
  fbm_from_s30(s.d, out32);
  return true;
}

// host-side helper for the parameters
__host__ inline void fbm_n30_setup(const uint32_t* n32, FbmN30& N) {
  fbm_to_s30(n32, 32, N.n);
  uint32_t inv = 1;  // Newton: inv = N^-1 mod 2^32
  #pragma unroll
  for (int i = 0; i < 5; ++i) inv *= 2u - n32[0] * inv;
  N.ninv = inv & FBM_M30;
}
