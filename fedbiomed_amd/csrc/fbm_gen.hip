// fedbiomed_amd -- the generic Joye-Libert engine for gfx950: any biprime N, even ones included.
//
// The fast engines of fbm_jl.hip are Montgomery products, which need an odd modulus.  The
// reference computes with any N -- gmpy2's powmod / invert and Python integers (_jls.py:37-73,
// 473-505, 520-562) -- and two of its caller tests pass even biprimes
// (tests/test_node_secagg.py:207-221, N = 1156; tests/test_secure_aggregation.py:193-233,
// N = 1234).  Every JL entry point of the C-ABI sends an even N here (fbm_capi.hip), and, under
// FBM_ENGINE_GENERIC, an odd one as well, which cross-checks the fast engines bit for bit.
//
//   jl_gen_exp_kernel      H^key mod N^2 (gmpy2.powmod; key < 0: the inverse of H^|key|), times
//                          (N pt + 1) mod N^2 for an encrypt                 (_jls.py:494-502, 550)
//   jl_gen_combine_kernel  prod_u c_u (* the server key's factor) mod N^2 (EncryptedNumber sums,
//                          _jls.py:353-374, 691-693); decrypt: ((v - 1) // N) mod N with Python's
//                          floor division (v = 0 gives N - 1)                (_jls.py:552-558)
//
// Arithmetic: 32-bit limbs, column-wise (Comba) products into a 96-bit accumulator, Barrett
// reduction (HAC 14.42: any modulus; also gives the quotient of the decryption), and the inverse
// modulo N^2 = 2^e m2 (m2 = m^2, m the odd part of N) by CRT of a binary inversion modulo m2
// (Guide to ECC, Alg. 2.22) and a Newton inversion modulo 2^e.  One lane per ciphertext; a lane's
// working numbers are LDS columns (word i at lds[i * 64 + lane]: a wave's access is one
// conflict-free LDS row) and the modulus constants are uniform (scalar loads from the call's
// constants block).  A correctness path: real biprimes are odd (a product of two large primes)
// and run on the fast engines; even ones are the reference tests' small moduli.
#include <vector>

#include "fbm_internal.hpp"

namespace fbm {

#define GEN_W 64  // lanes per workgroup: the LDS column stride
// per-lane LDS words: HB (base / scratch) | AC (accumulator) | T (products) | Q (Barrett
// scratch) | E (extra); every region has room for one word past its widest number
#define GEN_HB 0
#define GEN_AC 66
#define GEN_T 132
#define GEN_Q 264
#define GEN_E 396
#define GEN_WORDS 462
#define GEN_INV_CAP 40000  // binary inversion: <= 2 (bits(u) + bits(m2)) <= 8192 steps

static_assert(sizeof(GenCtx) % 4 == 0, "GenCtx is copied word by word");
static_assert(sizeof(GenCtx) <= FBM_CST_WORDS * 4, "GenCtx fits the call's constants block");

struct Col {  // one lane's number in LDS
  uint32_t* p;
  __host__ __device__ __forceinline__ uint32_t& operator[](int i) const { return p[i * GEN_W]; }
  __host__ __device__ __forceinline__ Col at(int i) const { return Col{p + i * GEN_W}; }
};
struct Glb {  // a uniform constant (device memory, scalar loads)
  const uint32_t* p;
  __host__ __device__ __forceinline__ uint32_t operator[](int i) const { return p[i]; }
};

__host__ __device__ __forceinline__ void g_zero(Col a, int n) {
  for (int i = 0; i < n; ++i) a[i] = 0u;
}
template <class S>
__host__ __device__ __forceinline__ void g_copy(Col d, S s, int n) {
  for (int i = 0; i < n; ++i) d[i] = s[i];
}
__host__ __device__ __forceinline__ bool g_is_zero(Col a, int n) {
  uint32_t o = 0;
  for (int i = 0; i < n; ++i) o |= a[i];
  return o == 0u;
}
__host__ __device__ __forceinline__ bool g_is_one(Col a, int n) {
  uint32_t o = a[0] ^ 1u;
  for (int i = 1; i < n; ++i) o |= a[i];
  return o == 0u;
}

// r[0, nr) = (a[0, na) * b[0, nb)) mod 2^(32 nr); r overlaps neither a nor b, except that it
// may write below where it reads: column c is stored after every word it reads
template <class A, class B>
__host__ __device__ void g_mul(Col r, A a, int na, B b, int nb, int nr) {
  uint64_t lo = 0;
  uint32_t hi = 0;
  for (int c = 0; c < nr; ++c) {
    const int i0 = c < nb ? 0 : c - nb + 1;
    const int i1 = c < na ? c : na - 1;
#pragma unroll 4
    for (int i = i0; i <= i1; ++i) {
      const uint64_t p = (uint64_t)a[i] * b[c - i];
      lo += p;
      hi += lo < p ? 1u : 0u;
    }
    r[c] = (uint32_t)lo;
    lo = (lo >> 32) | ((uint64_t)hi << 32);
    hi = 0;
  }
}

// a >= b ?
template <class B>
__host__ __device__ bool g_ge(Col a, int na, B b, int nb) {
  for (int i = (na > nb ? na : nb) - 1; i >= 0; --i) {
    const uint32_t x = i < na ? a[i] : 0u, y = i < nb ? b[i] : 0u;
    if (x != y) return x > y;
  }
  return true;
}

// a -= b mod 2^(32 na); returns the borrow out
template <class B>
__host__ __device__ uint32_t g_sub(Col a, int na, B b, int nb) {
  uint32_t br = 0;
  for (int i = 0; i < na; ++i) {
    const uint64_t d = (uint64_t)a[i] - (i < nb ? b[i] : 0u) - br;
    a[i] = (uint32_t)d;
    br = (uint32_t)(d >> 63);
  }
  return br;
}

template <class B>
__host__ __device__ void g_add(Col a, int na, B b, int nb) {
  uint64_t c = 0;
  for (int i = 0; i < na; ++i) {
    c += (uint64_t)a[i] + (i < nb ? b[i] : 0u);
    a[i] = (uint32_t)c;
    c >>= 32;
  }
}

// Barrett (HAC 14.42): R[0, k] = X mod m and, if want_q, QO[0, k] = X div m, for X[0, 2k) (any
// value below 2^(64k)), m of k words (top word non-zero), mu = floor(2^(64k) / m), read as k + 2
// words (k + 1 unless m is exactly 2^(32(k-1)): then mu = 2^(32(k+1))).  Q: scratch of 2k + 3
// words.  R may be X itself (its words are read before written).
__host__ __device__ uint32_t g_barrett(Col X, int k, Glb m, Glb mu, Col Q, Col R, Col QO, bool want_q) {
  g_mul(Q, X.at(k - 1), k + 1, mu, k + 2, 2 * k + 3);  // q2 = q1 mu, q1 = X div 2^(32(k-1))
  g_mul(Q, Q.at(k + 1), k + 1, m, k, k + 1);           // (q3 m) mod 2^(32(k+1)), q3 = q2 div 2^(32(k+1))
  uint32_t br = 0;                                     // r = X - q3 m  (0 <= r < 3m)
  for (int i = 0; i <= k; ++i) {
    const uint64_t d = (uint64_t)X[i] - Q[i] - br;
    R[i] = (uint32_t)d;
    br = (uint32_t)(d >> 63);
  }
  uint32_t corr = 0;
  while (corr < 3 && g_ge(R, k + 1, m, k)) {
    g_sub(R, k + 1, m, k);
    ++corr;
  }
  if (want_q) {
    uint64_t c = corr;
    for (int i = 0; i <= k; ++i) {
      c += Q[k + 1 + i];
      QO[i] = (uint32_t)c;
      c >>= 32;
    }
  }
  return corr < 3 ? 0u : FBM_ERR_ITER_CAP;
}

// R[0, k) = x[0, nx) mod m for a row x in device memory (any length): word-serial chunks of k
// words, r <- (r 2^(32c) + chunk) mod m; T: 2k words, Q: 2k + 3 words of scratch
__host__ __device__ uint32_t g_reduce_row(const uint32_t* x, int nx, int k, Glb m, Glb mu, Col T, Col Q, Col R) {
  while (nx > 0 && x[nx - 1] == 0u) --nx;
  g_zero(R, k + 1);
  uint32_t err = 0;
  int i = nx;
  while (i > 0) {
    const int c = i < k ? i : k;
    for (int j = 0; j < c; ++j) T[j] = x[i - c + j];
    for (int j = 0; j < k; ++j) T[c + j] = R[j];
    for (int j = c + k; j < 2 * k; ++j) T[j] = 0u;
    err |= g_barrett(T, k, m, mu, Q, R, R, false);
    i -= c;
  }
  return err;
}

// A = A B mod m (k words; A has room for k + 1)
__host__ __device__ uint32_t g_modmul(Col A, Col B, int k, Glb m, Glb mu, Col T, Col Q) {
  g_mul(T, A, k, B, k, 2 * k);
  return g_barrett(T, k, m, mu, Q, A, A, false);
}

// x = x / 2 mod p (p odd, x < p, w words with room for x + p)
__host__ __device__ void g_halve_mod(Col x, int w, Glb p, int kp) {
  if (x[0] & 1u) g_add(x, w, p, kp);
  for (int i = 0; i < w; ++i) x[i] = (x[i] >> 1) | (i + 1 < w ? x[i + 1] << 31 : 0u);
}

__host__ __device__ void g_shr1(Col x, int w) {
  for (int i = 0; i < w; ++i) x[i] = (x[i] >> 1) | (i + 1 < w ? x[i + 1] << 31 : 0u);
}

// x = x - y mod p (x, y < p)
__host__ __device__ void g_sub_mod(Col x, Col y, int w, Glb p, int kp) {
  if (g_sub(x, w, y, w)) g_add(x, w, p, kp);
}

// A = A^-1 mod M, M = 2^e m2: CRT of A^-1 mod m2 (binary inversion) and A^-1 mod 2^e (Newton).
// HB, T, Q, E: scratch.  Returns error flags (not invertible: gmpy2's ZeroDivisionError).
__host__ __device__ uint32_t g_inverse(Col A, const GenCtx* __restrict__ g, Col HB, Col T, Col Q, Col E) {
  const int kM = g->kM, km2 = g->km2, e = g->e;
  const Glb m2{g->m2};
  uint32_t err = 0;
  g_zero(HB, kM + 1);  // a = A^-1 mod m2 (0 when m2 = 1)
  if (!(km2 == 1 && g->m2[0] == 1u)) {
    const int w = kM + 1;
    Col u = T, v = T.at(66), x1 = Q, x2 = Q.at(66);
    g_copy(u, A, kM);
    u[kM] = 0u;
    g_zero(v, w);
    g_copy(v, m2, km2);
    g_zero(x1, w);
    x1[0] = 1u;
    g_zero(x2, w);
    for (int it = 0;; ++it) {
      if (it >= GEN_INV_CAP) {
        err |= FBM_ERR_ITER_CAP;
        break;
      }
      if (g_is_zero(u, w) || g_is_zero(v, w)) {  // gcd(A, m2) > 1
        err |= FBM_ERR_NOT_INVERTIBLE;
        break;
      }
      if (g_is_one(u, w)) {
        g_copy(HB, x1, km2);
        break;
      }
      if (g_is_one(v, w)) {
        g_copy(HB, x2, km2);
        break;
      }
      while (!(u[0] & 1u)) {
        g_shr1(u, w);
        g_halve_mod(x1, w, m2, km2);
      }
      while (!(v[0] & 1u)) {
        g_shr1(v, w);
        g_halve_mod(x2, w, m2, km2);
      }
      if (g_ge(u, w, v, w)) {
        g_sub(u, w, v, w);
        g_sub_mod(x1, x2, w, m2, km2);
      } else {
        g_sub(v, w, u, w);
        g_sub_mod(x2, x1, w, m2, km2);
      }
    }
  }
  if (e == 0) {  // odd N: M = m2
    g_copy(A, HB, kM);
    return err;
  }
  // b2 = A^-1 mod 2^(32W) by Newton (A odd: a unit mod 2^e) -> E
  const int W = (e + 31) >> 5;
  const uint32_t a0 = A[0];
  if (!(a0 & 1u)) return err | FBM_ERR_NOT_INVERTIBLE;
  uint32_t y = a0;  // 3 bits, then 6, 12, 24, 48
  for (int i = 0; i < 4; ++i) y *= 2u - a0 * y;
  g_zero(E, W);
  E[0] = y;
  for (int prec = 32; prec < 32 * W; prec *= 2) {
    Col t1 = T, t2 = T.at(66);
    g_mul(t1, A, kM < W ? kM : W, E, W, W);  // t1 = A y
    uint64_t c = 3;                           // t1 = 2 - t1 = ~t1 + 3
    for (int i = 0; i < W; ++i) {
      c += (uint32_t)~t1[i];
      t1[i] = (uint32_t)c;
      c >>= 32;
    }
    g_mul(t2, E, W, t1, W, W);  // y = y (2 - A y)
    g_copy(E, t2, W);
  }
  // t = ((b2 - a) m2^-1) mod 2^e;  A = a + m2 t  (< M)
  uint32_t br = 0;
  for (int i = 0; i < W; ++i) {
    const uint64_t d = (uint64_t)E[i] - (i < km2 ? HB[i] : 0u) - br;
    T[i] = (uint32_t)d;
    br = (uint32_t)(d >> 63);
  }
  g_mul(Q, T, W, Glb{g->m2inv}, W, W);
  if (e & 31) Q[W - 1] &= (1u << (e & 31)) - 1u;
  g_mul(T, Q, W, m2, km2, kM);
  g_copy(A, T, kM);
  g_add(A, kM, HB, km2);
  return err;
}

__host__ __device__ __forceinline__ void g_store_row(uint32_t* dst, Col a, int k, int words) {
  for (int i = 0; i < words; ++i) dst[i] = i < k ? a[i] : 0u;
}

// one ciphertext of jl_gen_exp_kernel: out = H^key mod M (times (N pt + 1) mod M when pt); col =
// this lane's LDS column base (stride GEN_W).  Returns FBM_ERR_* flags.  __host__ too: the test
// hook fbm_test_gen_exp runs it on the CPU.
__host__ __device__ uint32_t gen_exp_lane(const uint32_t* Hrow, const uint32_t* ptrow, int negative,
                                          const GenCtx* __restrict__ g, uint32_t* col, uint32_t* outrow) {
  const Col base{col};
  const Col HB = base.at(GEN_HB), AC = base.at(GEN_AC), T = base.at(GEN_T), Q = base.at(GEN_Q), E = base.at(GEN_E);
  const int kM = g->kM, kN = g->kN;
  const Glb M{g->M}, muM{g->muM};
  uint32_t err = g_reduce_row(Hrow, 64, kM, M, muM, T, Q, HB);  // h = H mod M
  // AC = h^|key| mod M: left-to-right binary (1 mod M for a zero key, gmpy2's powmod(h, 0, M))
  g_zero(AC, kM + 1);
  AC[0] = (kM == 1 && M[0] == 1u) ? 0u : 1u;  // h^0 mod 1 = 0
  for (int b = g->key_bits - 1; b >= 0; --b) {
    err |= g_modmul(AC, AC, kM, M, muM, T, Q);
    if ((g->key[b >> 5] >> (b & 31)) & 1u) err |= g_modmul(AC, HB, kM, M, muM, T, Q);
  }
  if (g->key_negative && g->key_bits > 0) err |= g_inverse(AC, g, HB, T, Q, E);
  if (ptrow) {  // (N pt + 1) mod M = N (pt mod N) + 1; a negative packing -|pt|: N ((-|pt|) mod N) + 1
    const Glb Nc{g->N};
    err |= g_reduce_row(ptrow, 32, kN, Nc, Glb{g->muN}, T, Q, E);
    if (negative && !g_is_zero(E, kN)) {
      for (int i = 0; i < kN; ++i) Q[i] = E[i];
      g_copy(E, Nc, kN);
      g_sub(E, kN, Q, kN);
    }
    g_mul(T, E, kN, Nc, kN, 2 * kN);
    g_zero(HB, kM + 1);
    g_copy(HB, T, kM);  // N (pt mod N) + 1 < M: the words past kM are zero
    uint64_t c = 1;
    for (int i = 0; i < kM && c; ++i) {
      c += HB[i];
      HB[i] = (uint32_t)c;
      c >>= 32;
    }
    err |= g_modmul(AC, HB, kM, M, muM, T, Q);
  }
  g_store_row(outrow, AC, kM, 64);
  return err;
}

// one ciphertext of jl_gen_combine_kernel: v = prod_u c_u (* factor) mod M (party u's row at
// cts + u * stride), out = v (FBM_GEN_PRODUCT, 64 words) or ((v - 1) // N) mod N (32 words)
__host__ __device__ uint32_t gen_combine_lane(const uint32_t* cts, int n_parties, uint64_t stride,
                                              const uint32_t* frow, const GenCtx* __restrict__ g, int mode,
                                              uint32_t* col, uint32_t* outrow) {
  const Col base{col};
  const Col HB = base.at(GEN_HB), AC = base.at(GEN_AC), T = base.at(GEN_T), Q = base.at(GEN_Q), E = base.at(GEN_E);
  const int kM = g->kM, kN = g->kN;
  const Glb M{g->M}, muM{g->muM};
  // operands of any size below 2^2048 are reduced first (the reference multiplies Python ints)
  uint32_t err = g_reduce_row(cts, 64, kM, M, muM, T, Q, AC);
  for (int u = 1; u < n_parties; ++u) {
    err |= g_reduce_row(cts + (uint64_t)u * stride, 64, kM, M, muM, T, Q, HB);
    err |= g_modmul(AC, HB, kM, M, muM, T, Q);
  }
  if (frow) {
    err |= g_reduce_row(frow, 64, kM, M, muM, T, Q, HB);
    err |= g_modmul(AC, HB, kM, M, muM, T, Q);
  }
  if (mode == FBM_GEN_PRODUCT) {
    g_store_row(outrow, AC, kM, 64);
    return err;
  }
  const Glb Nc{g->N};
  if (g_is_zero(AC, kM)) {  // (0 - 1) // N = -1, mod N: N - 1
    g_copy(HB, Nc, kN);
    uint32_t br = 1;
    for (int i = 0; i < kN; ++i) {
      const uint64_t d = (uint64_t)HB[i] - br;
      HB[i] = (uint32_t)d;
      br = (uint32_t)(d >> 63);
    }
  } else {  // (v - 1) // N < N (v < N^2): Barrett's quotient
    uint32_t br = 1;
    for (int i = 0; i < kM; ++i) {
      const uint64_t d = (uint64_t)AC[i] - br;
      AC[i] = (uint32_t)d;
      br = (uint32_t)(d >> 63);
    }
    g_zero(T, 2 * kN);
    g_copy(T, AC, kM);
    err |= g_barrett(T, kN, Nc, Glb{g->muN}, Q, E, HB, true);
  }
  g_store_row(outrow, HB, kN, 32);
  return err;
}

__global__ void __launch_bounds__(GEN_W) jl_gen_exp_kernel(const uint32_t* __restrict__ H,
                                                           const uint32_t* __restrict__ pt, int negative,
                                                           uint64_t n_ct, const GenCtx* __restrict__ g,
                                                           uint32_t* __restrict__ out, uint32_t* __restrict__ stats) {
  __shared__ uint32_t lds[GEN_WORDS * GEN_W];
  const uint64_t ct = (uint64_t)blockIdx.x * GEN_W + threadIdx.x;
  if (ct >= n_ct) return;
  const uint32_t err = gen_exp_lane(H + ct * 64, pt ? pt + ct * 32 : nullptr, negative, g, lds + threadIdx.x,
                                    out + ct * 64);
  if (err && stats) atomicOr(stats + FBM_STAT_ERRFLAGS, err);
}

__global__ void __launch_bounds__(GEN_W) jl_gen_combine_kernel(const uint32_t* __restrict__ cts, int n_parties,
                                                               uint64_t n_ct, const uint32_t* __restrict__ factor,
                                                               const GenCtx* __restrict__ g, int mode,
                                                               uint32_t* __restrict__ out,
                                                               uint32_t* __restrict__ stats) {
  __shared__ uint32_t lds[GEN_WORDS * GEN_W];
  const uint64_t ct = (uint64_t)blockIdx.x * GEN_W + threadIdx.x;
  if (ct >= n_ct) return;
  const uint32_t err = gen_combine_lane(cts + ct * 64, n_parties, n_ct * 64, factor ? factor + ct * 64 : nullptr, g,
                                        mode, lds + threadIdx.x, out + ct * (mode == FBM_GEN_PRODUCT ? 64 : 32));
  if (err && stats) atomicOr(stats + FBM_STAT_ERRFLAGS, err);
}

__global__ void jl_gen_setup_kernel(GenCtx g, uint32_t* __restrict__ dst) {
  const uint32_t* src = reinterpret_cast<const uint32_t*>(&g);
  for (int i = threadIdx.x; i < (int)(sizeof(GenCtx) / 4); i += blockDim.x) dst[i] = src[i];
}

int launch_jl_gen_setup(const GenCtx& g, uint32_t* cst, hipStream_t s) {
  hipLaunchKernelGGL(jl_gen_setup_kernel, dim3(1), dim3(256), 0, s, g, cst);
  return check_launch("jl_gen_setup_kernel");
}

int launch_jl_gen_exp(const uint32_t* H, const uint32_t* pt, int negative, uint64_t n_ct, const uint32_t* cst,
                      uint32_t* out, uint32_t* stats, hipStream_t s) {
  if (n_ct == 0) return FBM_OK;
  hipLaunchKernelGGL(jl_gen_exp_kernel, dim3((unsigned)((n_ct + GEN_W - 1) / GEN_W)), dim3(GEN_W), 0, s, H, pt,
                     negative, n_ct, (const GenCtx*)cst, out, stats);
  return check_launch("jl_gen_exp_kernel");
}

int launch_jl_gen_combine(const uint32_t* cts, int n_parties, uint64_t n_ct, const uint32_t* factor,
                          const uint32_t* cst, int mode, uint32_t* out, uint32_t* stats, hipStream_t s) {
  if (n_ct == 0) return FBM_OK;
  hipLaunchKernelGGL(jl_gen_combine_kernel, dim3((unsigned)((n_ct + GEN_W - 1) / GEN_W)), dim3(GEN_W), 0, s, cts,
                     n_parties, n_ct, factor, (const GenCtx*)cst, mode, out, stats);
  return check_launch("jl_gen_combine_kernel");
}

// host test hooks (fbm_test_gen_exp / fbm_test_gen_combine, fbm_capi.hip): one lane on the CPU
uint32_t host_gen_exp(const uint32_t* Hrow, const uint32_t* ptrow, int negative, const GenCtx& g, uint32_t* out) {
  std::vector<uint32_t> col((size_t)GEN_WORDS * GEN_W, 0u);
  return gen_exp_lane(Hrow, ptrow, negative, &g, col.data(), out);
}

uint32_t host_gen_combine(const uint32_t* cts, int n_parties, const uint32_t* frow, const GenCtx& g, int mode,
                          uint32_t* out) {
  std::vector<uint32_t> col((size_t)GEN_WORDS * GEN_W, 0u);
  return gen_combine_lane(cts, n_parties, 64, frow, &g, mode, col.data(), out);
}

}  // namespace fbm
