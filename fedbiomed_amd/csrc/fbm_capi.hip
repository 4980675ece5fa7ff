// fedbiomed_amd -- C ABI (include/fbm_secagg.h): argument validation, per-call uniform
// parameter setup (Montgomery constants, SHA-256 midstate, sliding-window schedule,
// ChaCha20 IV words) and kernel launches.  All device memory belongs to the caller.
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <atomic>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "fbm_internal.hpp"
#include "fbm_nadic_asm.hpp"
#include "fbm_quad_asm.hpp"
#include "fbm_tri_asm.hpp"
#include "fbm_safegcd.hpp"
#ifdef FBM_TEST_HOOKS
#include "../../include/fbm_secagg_test.h"
#endif

namespace fbm {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s launch failed: %s", what, hipGetErrorString(e));
    return FBM_E_HIP;
  }
  return FBM_OK;
}

static int zero_stats(uint32_t* stats, hipStream_t s) {
  if (!stats) {
    set_error("stats buffer is required");
    return FBM_E_ARG;
  }
  hipError_t e = hipMemsetAsync(stats, 0, FBM_STATS_WORDS * sizeof(uint32_t), s);
  if (e != hipSuccess) {
    set_error("hipMemsetAsync(stats): %s", hipGetErrorString(e));
    return FBM_E_HIP;
  }
  return FBM_OK;
}

static int quant_params(double clip, double two_clip, double target_f, uint64_t target_m1, QuantParams& qp) {
  if (!(clip > 0.0) || !(two_clip > 0.0) || !(target_f >= 1.0)) {
    set_error("invalid quantisation parameters (clip=%g, target=%g)", clip, target_f);
    return FBM_E_ARG;
  }
  qp.c = clip;
  qp.two_c = two_clip;
  qp.tf = target_f;
  qp.tm1 = target_m1;
  return FBM_OK;
}

// ---------------------------------------------------------------------------------------
// host big-integer helpers (tiny, per call)
// ---------------------------------------------------------------------------------------
typedef std::vector<uint32_t> Big;  // little-endian 32-bit limbs

static int big_bits(const Big& a) {
  for (int i = (int)a.size() - 1; i >= 0; --i)
    if (a[i]) return 32 * i + 32 - __builtin_clz(a[i]);
  return 0;
}

static Big big_mul(const Big& a, const Big& b) {
  Big r(a.size() + b.size(), 0u);
  for (size_t i = 0; i < a.size(); ++i) {
    uint64_t c = 0;
    for (size_t j = 0; j < b.size(); ++j) {
      const uint64_t t = (uint64_t)a[i] * b[j] + r[i + j] + c;
      r[i + j] = (uint32_t)t;
      c = t >> 32;
    }
    r[i + b.size()] = (uint32_t)c;
  }
  return r;
}

static int big_cmp(const Big& a, const Big& b) {
  const size_t n = a.size() > b.size() ? a.size() : b.size();
  for (size_t k = n; k-- > 0;) {
    const uint32_t x = k < a.size() ? a[k] : 0u, y = k < b.size() ? b[k] : 0u;
    if (x != y) return x > y ? 1 : -1;
  }
  return 0;
}

static void big_sub_inplace(Big& a, const Big& b) {  // a >= b
  int64_t br = 0;
  for (size_t k = 0; k < a.size(); ++k) {
    const int64_t d = (int64_t)a[k] - (int64_t)(k < b.size() ? b[k] : 0u) + br;
    a[k] = (uint32_t)d;
    br = d < 0 ? -1 : 0;
  }
}

// 2^e mod m by repeated doubling (m odd, > 1)
static Big big_pow2_mod(int e, const Big& m) {
  Big x(m.size() + 1, 0u);
  x[0] = 1u;
  for (int i = 0; i < e; ++i) {
    uint32_t c = 0;
    for (size_t k = 0; k < x.size(); ++k) {
      const uint32_t nc = x[k] >> 31;
      x[k] = (x[k] << 1) | c;
      c = nc;
    }
    if (big_cmp(x, m) >= 0) big_sub_inplace(x, m);
  }
  return x;
}

// a b 2^-32n mod m (CIOS over n = m.size() 32-bit words; m odd, a, b < m)
static Big host_mont(const Big& a, const Big& b, const Big& m, uint32_t mi) {
  const size_t n = m.size();
  std::vector<uint32_t> t(n + 2, 0u);
  for (size_t i = 0; i < n; ++i) {
    uint64_t c = 0;
    for (size_t j = 0; j < n; ++j) {
      const uint64_t v = (uint64_t)a[j] * b[i] + t[j] + c;
      t[j] = (uint32_t)v;
      c = v >> 32;
    }
    uint64_t v = (uint64_t)t[n] + c;
    t[n] = (uint32_t)v;
    t[n + 1] = (uint32_t)(v >> 32);
    const uint32_t q = t[0] * mi;
    c = ((uint64_t)q * m[0] + t[0]) >> 32;
    for (size_t j = 1; j < n; ++j) {
      const uint64_t w = (uint64_t)q * m[j] + t[j] + c;
      t[j - 1] = (uint32_t)w;
      c = w >> 32;
    }
    v = (uint64_t)t[n] + c;
    t[n - 1] = (uint32_t)v;
    t[n] = t[n + 1] + (uint32_t)(v >> 32);
  }
  Big r(t.begin(), t.begin() + n + 1);
  if (big_cmp(r, m) >= 0) big_sub_inplace(r, m);
  r.resize(n);
  return r;
}

// 2^e mod m (m odd, > 1, top word nonzero or not): left-to-right, Montgomery squarings and
// plain modular doublings -- log2(e) products instead of e doublings (big_pow2_mod)
static Big big_pow2_mod_mont(uint64_t e, Big m) {
  while (m.size() > 1 && m.back() == 0u) m.pop_back();
  const size_t n = m.size();
  uint32_t inv = m[0];  // Newton: m^-1 mod 2^32
  for (int i = 0; i < 5; ++i) inv *= 2u - m[0] * inv;
  const uint32_t mi = 0u - inv;
  Big x = big_pow2_mod((int)(32 * n), m);  // 1 in Montgomery form
  x.resize(n);
  auto dbl = [&](Big& y) {
    Big z(y.begin(), y.end());
    z.push_back(0u);
    uint32_t c = 0;
    for (size_t k = 0; k < z.size(); ++k) {
      const uint32_t nc = z[k] >> 31;
      z[k] = (z[k] << 1) | c;
      c = nc;
    }
    if (big_cmp(z, m) >= 0) big_sub_inplace(z, m);
    z.resize(n);
    y = z;
  };
  for (int b = 63; b >= 0; --b) {
    x = host_mont(x, x, m, mi);
    if ((e >> b) & 1u) dbl(x);
  }
  Big one(n, 0u);
  one[0] = 1u;
  return host_mont(x, one, m, mi);
}

static void to_limbs_host(const Big& a, uint32_t* o, int nl, int lb) {
  for (int k = 0; k < nl; ++k) {
    const int bit = k * lb, wi = bit >> 5, sh = bit & 31;
    const uint64_t lo = wi < (int)a.size() ? a[wi] : 0u;
    const uint64_t hi = wi + 1 < (int)a.size() ? a[wi + 1] : 0u;
    o[k] = (uint32_t)(((hi << 32) | lo) >> sh) & ((1u << lb) - 1u);
  }
}

static void to28_host(const Big& a, uint32_t* o, int nl) { to_limbs_host(a, o, nl, FBM_LB); }

template <int NL>
static void build_mont(const Big& m, MontCtxT<NL>& c) {
  to28_host(m, c.M, NL);
  const Big R2 = big_pow2_mod(2 * NL * FBM_LB, m);
  to28_host(R2, c.R2, NL);
  uint32_t inv = m[0];  // Newton: inv = m^-1 mod 2^32
  for (int i = 0; i < 5; ++i) inv *= 2u - m[0] * inv;
  c.mp = (0u - inv) & FBM_LMASK;
}

// (q, r) = (a div m, a mod m) by binary long division (host, per call; a < 2^2080, m odd)
static void big_divmod(const Big& a, const Big& m, Big& q, Big& r) {
  const int nb = big_bits(a);
  q.assign(a.size(), 0u);
  r.assign(m.size() + 1, 0u);
  for (int i = nb - 1; i >= 0; --i) {
    uint32_t c = (a[i >> 5] >> (i & 31)) & 1u;
    for (size_t k = 0; k < r.size(); ++k) {
      const uint32_t nc = r[k] >> 31;
      r[k] = (r[k] << 1) | c;
      c = nc;
    }
    if (big_cmp(r, m) >= 0) {
      big_sub_inplace(r, m);
      q[i >> 5] |= 1u << (i & 31);
    }
  }
}


// Constants of the quad engine (tools/gen_quad_asm.py): 29-bit limbs, R = 2^(36*29) = 2^1044.
static void build_quad(const Big& N, const Big& M, QuadCtx& qa) {
  memset(&qa, 0, sizeof(qa));
  const int LB = FBM_QA_LB, L = FBM_QA_L;
  Big Rm = big_pow2_mod(L * LB, N);  // R mod N
  Big K(N.size() + 1, 0u);
  K[0] = 1u;
  if (big_cmp(Rm, K) > 0) {  // K = N + 1 - Rm
    Big t(N.begin(), N.end());
    t.push_back(0u);
    uint64_t c = 1;
    for (size_t k = 0; k < t.size(); ++k) {
      c += t[k];
      t[k] = (uint32_t)c;
      c >>= 32;
    }
    big_sub_inplace(t, Rm);
    K = t;
  } else {
    K.assign(1, 0u);
  }
  uint32_t k29[FBM_QA_L];
  to_limbs_host(K, k29, L, LB);
  for (int j = 0; j < L; ++j) qa.kp[j] = ((1u << LB) - 1u) + k29[j];
  {  // the one-lane square's initial s window: 2^29 - 1 + P'_j, P' = (K - E) mod N (fbm_nadic_asm.hpp)
    Big E(40, 0u);
    for (int c = 0; c < 64; ++c)
      if ((FBM_NA_SQ_ONE_MASK >> c) & 1ull) {
        const int bit = 32 + LB * c;
        E[bit >> 5] |= 1u << (bit & 31);
      }
    Big q, r;
    big_divmod(E, N, q, r);  // E mod N
    Big P(K.begin(), K.end());
    P.resize(N.size() + 1, 0u);
    if (big_cmp(P, r) < 0) {  // P' = K - r (+ N)
      uint64_t c = 0;
      for (size_t k = 0; k < P.size(); ++k) {
        c += (uint64_t)P[k] + (k < N.size() ? N[k] : 0u);
        P[k] = (uint32_t)c;
        c >>= 32;
      }
    }
    big_sub_inplace(P, r);
    uint32_t p29[FBM_QA_L];
    to_limbs_host(P, p29, L, LB);
    for (int j = 0; j < L; ++j) qa.sqp[j] = ((1u << LB) - 1u) + p29[j];
  }
  to_limbs_host(N, qa.n, L, LB);
  for (int e = 2; e <= 3; ++e) {
    const Big u = big_pow2_mod(e * L * LB, M);
    Big q, r;
    big_divmod(u, N, q, r);
    uint32_t* dst = e == 2 ? qa.r2 : qa.r3;
    to_limbs_host(r, dst, L, LB);
    to_limbs_host(q, dst + L, L, LB);
  }
  uint32_t inv = N[0];  // Newton: N^-1 mod 2^32
  for (int i = 0; i < 5; ++i) inv *= 2u - N[0] * inv;
  qa.np = (0u - inv) & ((1u << LB) - 1u);
}

// Constants of the one-lane N-adic engine (tools/gen_nadic_asm.py): the group engines' 29-bit
// N and K'_i (the same R = 2^1044) in the layout of its scalar loads, and N's 28-bit limbs
// for the final step shared by all N-adic engines (na_final_digits).
static void build_nadic(const MontCtxN& mn, const QuadCtx& qa, NadicCtx& na) {
  static_assert(FBM_NA_LIMBS == FBM_QA_L && FBM_NA_LIMB_BITS == FBM_QA_LB, "one R for all N-adic engines");
  memset(&na, 0, sizeof(na));
  for (int j = 0; j < FBM_NLN; ++j) na.nk[j < 10 ? j : 6 + j] = mn.M[j];
  for (int j = 0; j < FBM_QA_L; ++j) na.nk29[j < 10 ? j : 6 + j] = qa.n[j];
  for (int j = 0; j < FBM_QA_L; ++j) na.nk29[42 + j] = qa.kp[j];
}

// SHA-256 midstate over the 14 leading blocks of t.to_bytes(1024,'big') (FDH.H), t = (k << 512) | tau:
// bytes 0..895 = t's bits 1024..8191 = tau's words 32..255 (k < 2^64 never reaches them).  Block b's
// SHA word j is t's little-endian word 255 - 16 b - j.  All-zero for a round below 2^1024.
static void fdh_midstate(uint32_t mid[8], const uint32_t* tau = nullptr) {
  static uint32_t zero_mid[8];
  static std::once_flag once;
  std::call_once(once, [] {
    uint32_t st[8], W[16];
    fbm_sha256_init(st);
    memset(W, 0, sizeof(W));
    for (int b = 0; b < 14; ++b) fbm_sha256_compress(st, W);
    memcpy(zero_mid, st, sizeof(st));
  });
  bool hi = false;
  for (int i = 32; tau && i < FBM_TAU_LIMBS; ++i) hi |= tau[i] != 0u;
  if (!hi) {
    memcpy(mid, zero_mid, sizeof(zero_mid));
    return;
  }
  uint32_t st[8], W[16];
  fbm_sha256_init(st);
  for (int b = 0; b < 14; ++b) {
    for (int j = 0; j < 16; ++j) W[j] = tau[255 - 16 * b - j];
    fbm_sha256_compress(st, W);
  }
  memcpy(mid, st, sizeof(st));
}

// the round tau (FBM_TAU_LIMBS little-endian words, < 2^8192) -> FDH's message blocks: block 15 = tau's
// words 0..15, block 14 = words 16..31 (the kernel ORs k into its last two words), blocks 0..13 into the
// midstate -- t.to_bytes(1024, 'big') of t = (k << 512) | tau (_jls.py:451-467, 744-748) for any round
static void set_tau(JlParams& jp, const uint32_t* tau) {
  for (int i = 0; i < 16; ++i) jp.tau_w[i] = tau ? tau[15 - i] : 0u;
  for (int i = 0; i < 16; ++i) jp.tau14_w[i] = tau ? tau[31 - i] : 0u;
  fdh_midstate(jp.mid, tau);
}

static void big_trim(Big& a) {
  while (a.size() > 1 && a.back() == 0u) a.pop_back();
}

static int big_ctz(const Big& a) {
  for (size_t i = 0; i < a.size(); ++i)
    if (a[i]) return 32 * (int)i + __builtin_ctz(a[i]);
  return 0;
}

static Big big_shr(const Big& a, int s) {
  Big r(a.size(), 0u);
  const int w = s >> 5, b = s & 31;
  for (size_t i = 0; i + w < a.size(); ++i) {
    const uint64_t lo = a[i + w], hi = i + w + 1 < a.size() ? a[i + w + 1] : 0u;
    r[i] = (uint32_t)((((hi << 32) | lo) >> b));
  }
  big_trim(r);
  return r;
}

// a b mod 2^(32 n)
static Big big_mullo(const Big& a, const Big& b, size_t n) {
  Big r(n, 0u);
  for (size_t i = 0; i < n && i < a.size(); ++i) {
    uint64_t c = 0;
    for (size_t j = 0; i + j < n; ++j) {
      const uint64_t t = (uint64_t)a[i] * (j < b.size() ? b[j] : 0u) + r[i + j] + c;
      r[i + j] = (uint32_t)t;
      c = t >> 32;
    }
  }
  return r;
}

// FDH.H's parameters only (fbm_jl_fdh and the generic engine): the gcd modulus' odd part
// (>= 1; 1: every odd r is coprime) and whether r must be odd as well
static int fdh_params(const uint32_t* n_odd, int even, const uint32_t* tau, uint64_t ct_offset, JlParams& jp) {
  if (!(n_odd[0] & 1u)) {
    set_error("FDH: the gcd modulus' odd part must be odd");
    return FBM_E_ARG;
  }
  memset(&jp, 0, sizeof(jp));
  for (int i = 0; i < 32; ++i) jp.N32[i] = n_odd[i];
  jp.fdh_even = even ? 1 : 0;
  set_tau(jp, tau);
  jp.ct_offset = ct_offset;
  return FBM_OK;
}

// FDH(2048, N^2): gcd(r, N^2) == 1 iff r is coprime to N's odd part (and odd, for an even N)
static int fdh_params_for_biprime(const uint32_t* biprime, const uint32_t* tau, uint64_t ct_offset, JlParams& jp) {
  Big N(biprime, biprime + 32);
  const int s = big_ctz(N);
  Big m = big_shr(N, s);
  m.resize(32, 0u);
  return fdh_params(m.data(), s > 0, tau, ct_offset, jp);
}

// N = 1: the reference computes everything modulo N^2 = 1 (every ciphertext 0) and its decryption's
// invert(delta^2, N^2) raises; only the generic engine's Barrett products take a modulus of 1
static bool jl_is_one(const uint32_t* biprime) {
  if (biprime[0] != 1u) return false;
  for (int i = 1; i < 32; ++i)
    if (biprime[i]) return false;
  return true;
}

// the generic engine (fbm_gen.hip) takes every even N and N = 1, and every N under FBM_ENGINE_GENERIC
static bool jl_generic(const uint32_t* biprime) {
  return (biprime[0] & 1u) == 0u || jl_is_one(biprime) || jl_engine_policy() == FBM_ENGINE_GENERIC;
}

// the short path on (1) or off (0: every wave runs the window-table path) for this thread's calls; only the
// test build's fbm_jl_set_short changes it (include/fbm_secagg_test.h)
static thread_local int t_short_on = 1;

// The path a split call (fbm_jl_encrypt_phase / fbm_jl_decrypt_factor_phase) took at its phase 1
// -- generic or Montgomery engine, short path or not -- keyed by its workspace: the later phases
// read the constants phase 1 wrote, so they follow phase 1's choice even if the process-wide
// switches (the test build's fbm_jl_set_engine, fbm_jl_set_short) changed in between.  A later phase whose record is
// missing (phase 1 never ran on this workspace, or its record was evicted by FBM_PATH_RECS newer
// split calls) is refused with FBM_E_ARG: it would read constants laid out for a path it cannot know.
// fbm_jl_clear_caches leaves the records alone (they hold no key material).
struct JlPathRec {
  const void* ws;
  bool generic, short_on;
};
static constexpr size_t FBM_PATH_RECS = 4096;
static std::mutex g_path_mu;
static std::vector<JlPathRec> g_path_recs;  // most recent last, at most FBM_PATH_RECS

static int jl_path_for(const void* ws, int phase, int full, const uint32_t* biprime, bool& generic, bool& short_on) {
  if (!(phase & 1)) {
    std::lock_guard<std::mutex> lk(g_path_mu);
    for (size_t i = g_path_recs.size(); i-- > 0;)
      if (g_path_recs[i].ws == ws) {
        generic = g_path_recs[i].generic || (biprime[0] & 1u) == 0u || jl_is_one(biprime);
        short_on = g_path_recs[i].short_on;
        return FBM_OK;
      }
    set_error("phase %d of a split call on a workspace with no phase-1 record (run phase 1 on it first)", phase);
    return FBM_E_ARG;
  }
  generic = jl_generic(biprime);
  short_on = t_short_on != 0;
  if (phase != full) {
    std::lock_guard<std::mutex> lk(g_path_mu);
    for (size_t i = 0; i < g_path_recs.size(); ++i)
      if (g_path_recs[i].ws == ws) {
        g_path_recs.erase(g_path_recs.begin() + i);
        break;
      }
    if (g_path_recs.size() >= FBM_PATH_RECS) g_path_recs.erase(g_path_recs.begin());
    g_path_recs.push_back(JlPathRec{ws, generic, short_on});
  }
  return FBM_OK;
}

// GenCtx of (N, key): M = N^2, Barrett constants of M and N, M = 2^e m2 with m2 odd, m2^-1 mod 2^e
static int build_gen_ctx(const uint32_t* biprime, const uint32_t* key, int key_negative, GenCtx& g) {
  memset(&g, 0, sizeof(g));
  Big N(biprime, biprime + 32);
  big_trim(N);
  if (big_bits(N) < 1) {
    set_error("biprime must be >= 1");
    return FBM_E_UNSUPPORTED;
  }
  Big M = big_mul(N, N);
  big_trim(M);
  auto mu = [](const Big& m) {  // floor(2^(64 k) / m), k = words of m
    Big a(2 * m.size() + 1, 0u), q, r;
    a.back() = 1u;
    big_divmod(a, m, q, r);
    big_trim(q);
    return q;
  };
  const Big muM = mu(M), muN = mu(N);
  g.kM = (int)M.size();
  g.kN = (int)N.size();
  for (size_t i = 0; i < M.size(); ++i) g.M[i] = M[i];
  for (size_t i = 0; i < muM.size() && i < 68; ++i) g.muM[i] = muM[i];
  for (size_t i = 0; i < N.size(); ++i) g.N[i] = N[i];
  for (size_t i = 0; i < muN.size() && i < 36; ++i) g.muN[i] = muN[i];
  const int s = big_ctz(N);
  const Big m = big_shr(N, s);
  Big m2 = big_mul(m, m);
  big_trim(m2);
  g.km2 = (int)m2.size();
  g.e = 2 * s;
  for (size_t i = 0; i < m2.size(); ++i) g.m2[i] = m2[i];
  if (g.e > 0) {  // m2^-1 mod 2^e by Newton (m2 odd): y <- y (2 - m2 y), 32 -> 64 -> ... bits
    const size_t W = (size_t)((g.e + 31) / 32);
    uint32_t y0 = m2[0];
    for (int i = 0; i < 5; ++i) y0 *= 2u - m2[0] * y0;
    Big y(W, 0u);
    y[0] = y0;
    for (size_t prec = 32; prec < 32 * W; prec *= 2) {
      Big t = big_mullo(m2, y, W);
      uint64_t c = 3;  // 2 - t = ~t + 3 (mod 2^(32 W))
      for (size_t i = 0; i < W; ++i) {
        c += (uint32_t)~t[i];
        t[i] = (uint32_t)c;
        c >>= 32;
      }
      y = big_mullo(y, t, W);
    }
    if (g.e & 31) y[W - 1] &= (1u << (g.e & 31)) - 1u;
    for (size_t i = 0; i < W; ++i) g.m2inv[i] = y[i];
  }
  if (key) {
    Big K(key, key + 64);
    g.key_bits = big_bits(K);
    for (int i = 0; i < 64; ++i) g.key[i] = key[i];
    g.key_negative = key_negative ? 1 : 0;
  }
  return FBM_OK;
}

// The modulus-dependent part of JlParams (Montgomery / N-adic / group-engine constants, N^-1
// mod 2^1024, the FDH midstate): ~0.3 ms of host big-integer work per call, so it is built once
// per biprime and kept in a small process-wide cache (a round's encrypts and aggregate, and
// every round of an experiment, share one biprime).
static int build_jl_params_uncached(const uint32_t* biprime, int es, int cr, const uint32_t* tau, uint64_t ct_offset,
                                    JlParams& jp) {
  memset(&jp, 0, sizeof(jp));
  Big N(biprime, biprime + 32);
  const int nb = big_bits(N);
  if (nb < 2 || (N[0] & 1u) == 0u) {  // an even N takes the generic engine before this (jl_generic)
    set_error("biprime must be >= 2 (the Montgomery engines take an odd N >= 3); got %d bits, %s", nb,
              (N[0] & 1u) ? "odd" : "even");
    return FBM_E_UNSUPPORTED;
  }
  if (es < 1 || cr < 1 || es > 100 || (int64_t)es * cr > 1024) {
    set_error("invalid VES parameters es=%d cr=%d", es, cr);
    return FBM_E_ARG;
  }
  Big M = big_mul(N, N);  // 64 limbs
  while (M.size() > 64) M.pop_back();
  build_mont<FBM_NL>(M, jp.mc);
  build_mont<FBM_NLN>(N, jp.mn);
  build_quad(N, M, jp.qa);
  build_nadic(jp.mn, jp.qa, jp.na);
  for (int i = 0; i < 32; ++i) jp.N32[i] = biprime[i];
  {  // N^-1 mod 2^1024 by Newton: y <- y (2 - N y); y = N is correct to 3 bits for odd N
    uint32_t y[32], t[32];
    for (int i = 0; i < 32; ++i) y[i] = biprime[i];
    auto mullo = [](const uint32_t* a, const uint32_t* b, uint32_t* r) {  // r = a*b mod 2^1024
      uint32_t acc[32] = {0};
      for (int i = 0; i < 32; ++i) {
        uint64_t c = 0;
        for (int j = 0; i + j < 32; ++j) {
          const uint64_t v = (uint64_t)a[i] * b[j] + acc[i + j] + c;
          acc[i + j] = (uint32_t)v;
          c = v >> 32;
        }
      }
      memcpy(r, acc, sizeof(acc));
    };
    for (int it = 0; it < 9; ++it) {  // 3 -> 6 -> ... -> 1536 bits
      mullo(biprime, y, t);           // t = N y
      uint64_t br = 0;                // t = 2 - t  (mod 2^1024)
      for (int i = 0; i < 32; ++i) {
        const uint64_t d = (uint64_t)(i == 0 ? 2u : 0u) - t[i] - br;
        t[i] = (uint32_t)d;
        br = (d >> 63) & 1u;
      }
      mullo(y, t, y);
    }
    memcpy(jp.Ninv32, y, sizeof(y));
  }
  jp.n_bits = nb;
  {  // M = N << (1036 - nb): 0 mod N, in [2^1035, 2^1036) (negative-weight nude digit)
    Big m(N.begin(), N.end());
    m.resize(34, 0u);
    const int sh = FBM_NLN * FBM_LB - nb;
    for (int i = 0; i < sh; ++i) {
      uint32_t c = 0;
      for (size_t k = 0; k < m.size(); ++k) {
        const uint32_t nc = m[k] >> 31;
        m[k] = (m[k] << 1) | c;
        c = nc;
      }
    }
    to28_host(m, jp.mneg, FBM_NLN);
  }
  fbm_n30_setup(jp.N32, jp.n30);
  jp.es = es;
  jp.cr = cr;
  set_tau(jp, tau);
  jp.ct_offset = ct_offset;
  return FBM_OK;
}

struct JlParamsCacheEntry {
  uint32_t n32[32];
  JlParams jp;
};
static std::mutex g_jp_mu;
static std::vector<JlParamsCacheEntry> g_jp_cache;  // most recently used last, at most 8

static int build_jl_params(const uint32_t* biprime, int es, int cr, const uint32_t* tau, uint64_t ct_offset,
                           JlParams& jp) {
  if (es < 1 || cr < 1 || es > 100 || (int64_t)es * cr > 1024) {
    set_error("invalid VES parameters es=%d cr=%d", es, cr);
    return FBM_E_ARG;
  }
  {
    std::lock_guard<std::mutex> lk(g_jp_mu);
    for (size_t i = 0; i < g_jp_cache.size(); ++i) {
      if (memcmp(g_jp_cache[i].n32, biprime, sizeof(g_jp_cache[i].n32)) == 0) {
        JlParamsCacheEntry e = g_jp_cache[i];
        g_jp_cache.erase(g_jp_cache.begin() + i);
        g_jp_cache.push_back(e);
        jp = e.jp;
        jp.es = es;
        jp.cr = cr;
        set_tau(jp, tau);
        jp.ct_offset = ct_offset;
        jp.key_is_zero = 0;
        return FBM_OK;
      }
    }
  }
  const int rc = build_jl_params_uncached(biprime, es, cr, tau, ct_offset, jp);
  if (rc) return rc;
  JlParamsCacheEntry e;
  memcpy(e.n32, biprime, sizeof(e.n32));
  e.jp = jp;
  std::lock_guard<std::mutex> lk(g_jp_mu);
  if (g_jp_cache.size() >= 8) g_jp_cache.erase(g_jp_cache.begin());
  g_jp_cache.push_back(e);
  return FBM_OK;
}

// R^(P+1) mod N^2 in 28-bit limbs (the ciphertext product's first operand), cached per (N, P)
struct JlRkCacheEntry {
  uint32_t n32[32];
  int parties;
  JlRk rk;
};
static std::vector<JlRkCacheEntry> g_rk_cache;  // guarded by g_jp_mu, at most 16

static void jl_rk_for(const uint32_t* n32, int n_parties, JlRk& r) {
  {
    std::lock_guard<std::mutex> lk(g_jp_mu);
    for (const JlRkCacheEntry& e : g_rk_cache)
      if (e.parties == n_parties && memcmp(e.n32, n32, sizeof(e.n32)) == 0) {
        r = e.rk;
        return;
      }
  }
  Big M(n32, n32 + 32);
  M = big_mul(M, M);
  M.resize(64);
  const Big rk = big_pow2_mod_mont((uint64_t)(n_parties + 1) * FBM_NL * FBM_LB, M);
  memset(&r, 0, sizeof(r));
  to28_host(rk, r.w, FBM_NL);
  JlRkCacheEntry e;
  memcpy(e.n32, n32, sizeof(e.n32));
  e.parties = n_parties;
  e.rk = r;
  std::lock_guard<std::mutex> lk(g_jp_mu);
  if (g_rk_cache.size() >= 16) g_rk_cache.erase(g_rk_cache.begin());
  g_rk_cache.push_back(e);
}

// Left-to-right sliding window (width FBM_WIN) over |key|, odd-power table.
static int build_schedule(const uint32_t* key, JlSched& sc, int& is_zero) {
  memset(&sc, 0, sizeof(sc));
  sc.sbits = -1;  // (build_short)
  Big K(key, key + 64);
  const int nb = big_bits(K);
  is_zero = nb == 0;
  if (is_zero) return FBM_OK;
  auto bit = [&](int i) -> int { return (K[i >> 5] >> (i & 31)) & 1; };
  int i = nb - 1;
  int pending_sq = 0;
  bool first = true;
  while (i >= 0) {
    if (!bit(i)) {
      ++pending_sq;
      --i;
      continue;
    }
    int l = i - FBM_WIN + 1;
    if (l < 0) l = 0;
    while (!bit(l)) ++l;
    int val = 0;
    for (int j = i; j >= l; --j) val = (val << 1) | bit(j);
    const int width = i - l + 1;
    const int idx = (val - 1) / 2;
    if (first) {
      sc.first = idx;
      first = false;
    } else {
      int nsq = pending_sq + width;
      while (nsq > FBM_OP_MAXSQ) {
        if (sc.n_ops >= FBM_MAX_OPS) return FBM_E_ARG;
        sc.op[sc.n_ops++] = (uint16_t)(FBM_OP_MAXSQ << FBM_OP_SHIFT);
        nsq -= FBM_OP_MAXSQ;
      }
      if (sc.n_ops >= FBM_MAX_OPS) return FBM_E_ARG;
      sc.op[sc.n_ops++] = (uint16_t)((nsq << FBM_OP_SHIFT) | (idx + 1));
    }
    pending_sq = 0;
    i = l - 1;
  }
  while (pending_sq > 0) {
    const int nsq = pending_sq > FBM_OP_MAXSQ ? FBM_OP_MAXSQ : pending_sq;
    if (sc.n_ops >= FBM_MAX_OPS) return FBM_E_ARG;
    sc.op[sc.n_ops++] = (uint16_t)(nsq << FBM_OP_SHIFT);
    pending_sq -= nsq;
  }
  return FBM_OK;
}

// ---- the short path's constants (JlShort, fbm_internal.hpp) ------------------------------
// 2^E mod m for an odd m of at most 2048 bits and any E: left-to-right, Montgomery squarings
// (64-bit limbs) and modular doublings -- ~2 050 products for the ~2 050-bit E of a 2 040-bit key
static Big pow2_mod_big(const Big& E, Big m) {
  big_trim(m);
  const int n = (int)((m.size() + 1) / 2);
  uint64_t M[32] = {0};
  for (size_t i = 0; i < m.size(); ++i) M[i / 2] |= (uint64_t)m[i] << (32 * (i & 1));
  uint64_t inv = M[0];  // Newton: M^-1 mod 2^64
  for (int i = 0; i < 6; ++i) inv *= 2u - M[0] * inv;
  const uint64_t mi = 0u - inv;
  auto ge_sub = [&](uint64_t* a, uint64_t top) {  // a <- a - M if (top:a) >= M
    bool ge = top != 0;
    if (!ge) {
      ge = true;
      for (int k = n - 1; k >= 0; --k)
        if (a[k] != M[k]) {
          ge = a[k] > M[k];
          break;
        }
    }
    if (!ge) return;
    unsigned __int128 br = 0;
    for (int k = 0; k < n; ++k) {
      const unsigned __int128 d = (unsigned __int128)a[k] - M[k] - br;
      a[k] = (uint64_t)d;
      br = (d >> 64) & 1u;
    }
  };
  auto mul = [&](const uint64_t* a, const uint64_t* b, uint64_t* r) {  // a b 2^-64n mod M (CIOS)
    uint64_t t[34] = {0};
    for (int i = 0; i < n; ++i) {
      unsigned __int128 c = 0;
      for (int j = 0; j < n; ++j) {
        c += (unsigned __int128)a[j] * b[i] + t[j];
        t[j] = (uint64_t)c;
        c >>= 64;
      }
      c += t[n];
      t[n] = (uint64_t)c;
      t[n + 1] = (uint64_t)(c >> 64);
      const uint64_t q = t[0] * mi;
      c = ((unsigned __int128)q * M[0] + t[0]) >> 64;
      for (int j = 1; j < n; ++j) {
        c += (unsigned __int128)q * M[j] + t[j];
        t[j - 1] = (uint64_t)c;
        c >>= 64;
      }
      c += t[n];
      t[n - 1] = (uint64_t)c;
      t[n] = t[n + 1] + (uint64_t)(c >> 64);
    }
    ge_sub(t, t[n]);
    for (int k = 0; k < n; ++k) r[k] = t[k];
  };
  auto dbl = [&](uint64_t* a) {
    uint64_t c = 0;
    for (int k = 0; k < n; ++k) {
      const uint64_t nc = a[k] >> 63;
      a[k] = (a[k] << 1) | c;
      c = nc;
    }
    ge_sub(a, c);
  };
  uint64_t x[32] = {0};
  x[0] = 1;
  for (int i = 0; i < 64 * n; ++i) dbl(x);  // 1 in Montgomery form
  for (int b = big_bits(E) - 1; b >= 0; --b) {
    mul(x, x, x);
    if ((E[b >> 5] >> (b & 31)) & 1u) dbl(x);
  }
  uint64_t one[32] = {0};
  one[0] = 1;
  mul(x, one, x);
  Big r(2 * (size_t)n, 0u);
  for (int k = 0; k < n; ++k) {
    r[2 * k] = (uint32_t)x[k];
    r[2 * k + 1] = (uint32_t)(x[k] >> 32);
  }
  return r;
}

// The short path's constant C per (N, |key|), cached so a round's repeated calls skip the ~2 050
// host squarings.  An entry holds no key material: it is found by a SHA-256 digest of (N, |key|)
// and holds only C (a public function of the key, like the ciphertexts it is used for); entries
// are zeroed when evicted or cleared (fbm_jl_clear_caches).  The reference keeps nothing between
// calls (a fresh SecaggCrypter per call: fedbiomed/node/secagg/_secagg_round.py:142).
struct JlShortCacheEntry {
  uint32_t digest[8];  // SHA-256(N's 32 words || |key|'s 64 words, little-endian bytes)
  uint32_t corr[72];
};
static std::vector<JlShortCacheEntry> g_short_cache;  // guarded by g_jp_mu, at most 32

static void wipe(void* p, size_t n) {  // a zeroing the optimiser keeps
  volatile uint8_t* v = (volatile uint8_t*)p;
  while (n--) *v++ = 0;
}

// SHA-256 of a little-endian word message (host; the FDH kernel's compression function)
static void sha256_words(const uint32_t* w, int nw, uint32_t out[8]) {
  uint32_t st[8], W[16];
  fbm_sha256_init(st);
  const uint64_t nbytes = (uint64_t)nw * 4;
  const int nblocks = (int)((nbytes + 9 + 63) / 64);
  auto byte_at = [&](uint64_t i) -> uint32_t {
    if (i < nbytes) return (w[i / 4] >> (8 * (i % 4))) & 0xffu;  // little-endian words
    if (i == nbytes) return 0x80u;
    const uint64_t tail = (uint64_t)nblocks * 64 - i;  // the 8-byte big-endian bit length
    if (tail <= 8) return (uint32_t)(((nbytes * 8) >> (8 * (tail - 1))) & 0xffu);
    return 0u;
  };
  for (int b = 0; b < nblocks; ++b) {
    for (int j = 0; j < 16; ++j) {
      const uint64_t i = (uint64_t)b * 64 + 4 * j;
      W[j] = (byte_at(i) << 24) | (byte_at(i + 1) << 16) | (byte_at(i + 2) << 8) | byte_at(i + 3);
    }
    fbm_sha256_compress(st, W);
  }
  memcpy(out, st, sizeof(st));
  wipe(W, sizeof(W));
}

static void short_cache_clear() {
  std::lock_guard<std::mutex> lk(g_jp_mu);
  for (JlShortCacheEntry& e : g_short_cache) wipe(&e, sizeof(e));
  g_short_cache.clear();
}

// The short path (jl_exp_kernel): possible for N > 2^262 (D = N - 2^261 > the product's quotient
// m < 2^261); used with a nonzero key.  Returns whether N qualifies (then sh.d is valid and the
// constants block gets it); sets sc.sbits and sh.kw / sh.corr when the key does too.
static bool build_short(const uint32_t* biprime, const uint32_t* key, int is_zero, JlSched& sc, JlShort& sh,
                        bool short_on) {
  memset(&sh, 0, sizeof(sh));
  sc.sbits = -1;
  if (!short_on) return false;
  Big N(biprime, biprime + 32);
  big_trim(N);
  const int KSB = FBM_QA_LB * FBM_NA_SHORT_LIMBS;  // 261
  if (big_bits(N) < KSB + 2 || !(N[0] & 1u)) return false;
  {  // D = N - 2^261
    Big D(N.begin(), N.end());
    Big p(KSB / 32 + 1, 0u);
    p[KSB / 32] = 1u << (KSB % 32);
    big_sub_inplace(D, p);
    to_limbs_host(D, sh.d, FBM_QA_L, FBM_QA_LB);
  }
  if (is_zero) return true;
  Big K(key, key + 64);
  const int nb = big_bits(K);
  for (int i = 0; i < 64; ++i) sh.kw[i] = key[i];
  sc.sbits = nb - 1;
  uint32_t dg[8];
  {
    uint32_t msg[96];
    memcpy(msg, biprime, 32 * 4);
    memcpy(msg + 32, key, 64 * 4);
    sha256_words(msg, 96, dg);
    wipe(msg, sizeof(msg));
    std::lock_guard<std::mutex> lk(g_jp_mu);
    for (const JlShortCacheEntry& e : g_short_cache)
      if (memcmp(e.digest, dg, sizeof(dg)) == 0) {
        memcpy(sh.corr, e.corr, sizeof(sh.corr));
        return true;
      }
  }
  // E = L (2^s + 1) + 261 (|key| - 2^s), L = 1044, s = nb - 1: the chain leaves h^|key| 2^-(E - 2L)
  const int s = nb - 1;
  Big v(K.begin(), K.end());
  v[s >> 5] &= ~(1u << (s & 31));
  Big E(66, 0u);
  uint64_t c = 0;
  for (int i = 0; i < 64; ++i) {  // 261 v
    c += (uint64_t)v[i] * (uint64_t)KSB;
    E[i] = (uint32_t)c;
    c >>= 32;
  }
  E[64] = (uint32_t)c;
  auto add_at = [&](uint64_t val, int bit) {  // E += val << bit
    const int w = bit >> 5, sh2 = bit & 31;
    unsigned __int128 add = (unsigned __int128)val << sh2;
    uint64_t cy = 0;
    for (int i = w; i < (int)E.size(); ++i) {
      const uint64_t t = (uint64_t)E[i] + (uint64_t)(uint32_t)add + cy;
      E[i] = (uint32_t)t;
      cy = t >> 32;
      add >>= 32;
      if (!add && !cy) break;
    }
  };
  const int Lb = FBM_QA_L * FBM_QA_LB;  // 1044
  add_at((uint64_t)Lb, s);
  add_at((uint64_t)Lb, 0);
  Big M = big_mul(N, N);
  big_trim(M);
  const Big C = pow2_mod_big(E, M);
  Big q, r;
  big_divmod(C, N, q, r);
  to_limbs_host(r, sh.corr, FBM_QA_L, FBM_QA_LB);
  to_limbs_host(q, sh.corr + FBM_QA_L, FBM_QA_L, FBM_QA_LB);
  wipe(v.data(), v.size() * 4);  // (K, v, E: the key and its exponent -- not kept)
  wipe(K.data(), K.size() * 4);
  wipe(E.data(), E.size() * 4);
  JlShortCacheEntry e;
  memcpy(e.digest, dg, sizeof(dg));
  memcpy(e.corr, sh.corr, sizeof(e.corr));
  std::lock_guard<std::mutex> lk(g_jp_mu);
  if (g_short_cache.size() >= 32) {
    wipe(&g_short_cache.front(), sizeof(JlShortCacheEntry));
    g_short_cache.erase(g_short_cache.begin());
  }
  g_short_cache.push_back(e);
  wipe(&e, sizeof(e));
  return true;
}

static uint64_t table_slots_for(uint64_t n_ct) {
  const uint64_t cap = jl_table_slots();
  uint64_t g = ((n_ct + 255) / 256) * 256;
  return g < cap ? g : cap;
}

static uint64_t align256(uint64_t v) { return (v + 255) & ~255ull; }

// ---------------------------------------------------------------------------------------
// optional per-kernel event timer (test build only: fbm_prof_enable / fbm_prof_report,
// include/fbm_secagg_test.h): records a HIP event pair on the launch stream around each kernel
// launch; costs nothing when disabled.  The product library launches directly.
// ---------------------------------------------------------------------------------------
#ifdef FBM_TEST_HOOKS
struct ProfRec {
  const char* name;
  hipEvent_t a, b;
};
static std::mutex g_prof_mu;
static bool g_prof_on = false;
static std::vector<ProfRec> g_prof;
static std::map<std::string, std::pair<long, double>> g_prof_agg;

template <class F>
static int timed(const char* name, hipStream_t s, F f) {
  if (!g_prof_on) return f();
  ProfRec r{name, nullptr, nullptr};
  if (hipEventCreate(&r.a) != hipSuccess) return f();
  if (hipEventCreate(&r.b) != hipSuccess) {
    (void)hipEventDestroy(r.a);
    return f();
  }
  // Drain the stream first: a marker can otherwise complete while the previous kernel is
  // still running, and its interval would absorb that kernel's tail (measured: per-kernel
  // sums 2.3x the wall time).  Profiling mode therefore serialises host and device.
  // A failed drain or marker only loses this timing record, never the launch itself.
  if (hipStreamSynchronize(s) != hipSuccess || hipEventRecord(r.a, s) != hipSuccess) {
    (void)hipEventDestroy(r.a);
    (void)hipEventDestroy(r.b);
    return f();
  }
  const int rc = f();
  if (hipEventRecord(r.b, s) != hipSuccess) {
    (void)hipEventDestroy(r.a);
    (void)hipEventDestroy(r.b);
    return rc;
  }
  std::lock_guard<std::mutex> g(g_prof_mu);
  g_prof.push_back(r);
  return rc;
}
#else
template <class F>
static int timed(const char*, hipStream_t, F f) {
  return f();
}
#endif

static void fill_peers(LomPeers& pe, const uint8_t* nonce, uint64_t tau) {
  memset(&pe, 0, sizeof(pe));
  uint32_t iv[4];
  memcpy(iv, nonce, 16);
  pe.ctr0 = (uint64_t)iv[0] | ((uint64_t)iv[1] << 32);
  pe.n14 = iv[2];
  pe.n15 = iv[3];
  pe.tau = tau;
  uint8_t tb[16] = {0};
  for (int b = 0; b < 8; ++b) tb[15 - b] = (uint8_t)(tau >> (8 * b));
  memcpy(pe.tau_be, tb, 16);
}

}  // namespace fbm

using namespace fbm;

extern "C" {

int fbm_abi_version(void) { return FBM_ABI_VERSION; }

void fbm_jl_clear_caches(void) {
  short_cache_clear();  // the only one derived from a key (zeroed)
  {
    std::lock_guard<std::mutex> lk(g_jp_mu);
    g_jp_cache.clear();  // per-N public parameters
    g_rk_cache.clear();
  }
}

const char* fbm_last_error(void) { return g_err; }

int fbm_check_stats(const uint32_t* st, int lom_nodes, uint32_t* max_bits_out) {
  if (!st) return FBM_E_ARG;
  if (max_bits_out) *max_bits_out = st[FBM_STAT_MAXBITS];
  const uint32_t f = st[FBM_STAT_ERRFLAGS];
  if (f & FBM_ERR_FDH_OVERFLOW) {
    set_error("FDH: no r of 1..7 digests with gcd(r, N^2) == 1 (reference: OverflowError)");
    return FBM_E_FDH;
  }
  if (f & FBM_ERR_FDH_WIDE) {  // (no kernel reports it since round 5: r of up to 255 digests runs on the device)
    set_error("FDH: r wider than the device path's rows");
    return FBM_E_UNSUPPORTED;
  }
  if (f & FBM_ERR_NOT_INVERTIBLE) {
    set_error("invert() no inverse exists");
    return FBM_E_INVERSE;
  }
  if (f & FBM_ERR_ITER_CAP) {
    set_error("bounded device loop hit its iteration cap");
    return FBM_E_ITER;
  }
  if (f & FBM_ERR_PT_WIDE) {
    set_error("VES: a packed value spills past the 1024-bit plaintext (a value wider than its slot); "
              "outside the device path's domain");
    return FBM_E_UNSUPPORTED;
  }
  if (f & FBM_ERR_DEQUANT_RANGE) {
    set_error("Cannot reverse quantize, received values exceed maximum number");
    return FBM_E_RANGE;
  }
  if (lom_nodes > 0) {
    int node_bits = 0;
    while ((1ll << node_bits) < (long long)lom_nodes) ++node_bits;  // ceil(log2(P))
    if ((int)st[FBM_STAT_MAXBITS] >= 64 - node_bits) {
      set_error("Secure aggregation overflow detected: values need %u bits, %d available", st[FBM_STAT_MAXBITS],
                64 - node_bits);
      return FBM_E_OVERFLOW;
    }
  }
  if (f & FBM_ERR_ROUND_RANGE) {
    set_error("int too big to convert");
    return FBM_E_ROUND;
  }
  return FBM_OK;
}

int fbm_lom_protect(const void* x, int x_dtype, uint64_t n, double clip, double two_clip, double target_f,
                    uint64_t target_m1, uint64_t weight, const uint8_t* secrets, const int8_t* signs, int n_peers,
                    int raw_seeds, const uint8_t* nonce, uint64_t tau, uint64_t elem_offset, uint64_t* y,
                    uint32_t* stats, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  int rc = zero_stats(stats, s);
  if (rc) return rc;
  QuantParams qp;
  if ((rc = quant_params(clip, two_clip, target_f, target_m1, qp))) return rc;
  if (x_dtype != FBM_F32 && x_dtype != FBM_F64 && x_dtype != FBM_U64) {
    set_error("x_dtype must be FBM_F32, FBM_F64 or FBM_U64");
    return FBM_E_ARG;
  }
  if (n_peers < 0) {
    set_error("n_peers=%d < 0", n_peers);
    return FBM_E_ARG;
  }
  if ((n > 0 && ((!x && x_dtype != FBM_U64) || !y)) || !nonce || (n_peers > 0 && (!secrets || !signs))) {
    set_error("null pointer argument");
    return FBM_E_ARG;
  }
  // PRF.eval_vector guard (_lom.py:74-78), on global indices
  if ((elem_offset & 7ull) != 0) {
    set_error("elem_offset must be a multiple of 8 (ChaCha20 block aligned shard)");
    return FBM_E_ARG;
  }
  const uint64_t n_glob = elem_offset + n;
  if (n_glob < n || n_glob + 1000ull > (1ull << 61)) {
    set_error("Can not perform encryiton due to large input vector");
    return FBM_E_ARG;
  }
  // (i + tau).to_bytes(8, 'big') (_lom.py:81) past 2^64 is the reference's OverflowError, raised
  // after its overflow guard and only when there are peers (no PRF call without one): reported
  // through the status words in that order (fbm_check_stats), the counters wrapping meanwhile
  const int round_range = n_peers > 0 && n > 0 && tau > ~0ull - (n_glob - 1);
  // peers in groups of FBM_MAX_PEERS (the kernel-argument block): the first group with the
  // quantise/weight/overflow statistics, later groups accumulated in place
  for (int g0 = 0; g0 == 0 || g0 < n_peers; g0 += FBM_MAX_PEERS) {
    const int gn = n_peers - g0 < FBM_MAX_PEERS ? n_peers - g0 : FBM_MAX_PEERS;
    LomPeers pe;
    fill_peers(pe, nonce, tau);
    pe.n_peers = gn < 0 ? 0 : gn;
    pe.raw_seeds = raw_seeds;
    pe.elem_offset = elem_offset;
    pe.round_range = g0 == 0 ? round_range : 0;
    for (int p = 0; p < pe.n_peers; ++p) {
      memcpy(pe.secret[p], secrets + 32 * (g0 + p), 32);
      if (signs[g0 + p] >= 0) pe.add_bits |= 1ull << p;
    }
    if (g0 == 0)
      rc = timed("lom_protect", s, [&] { return launch_lom_protect(x, x_dtype, n, qp, weight, pe, y, stats, s); });
    else
      rc = timed("lom_protect", s, [&] { return launch_lom_mask_accumulate(n, pe, y, s); });
    if (rc) return rc;
  }
  return FBM_OK;
}

int fbm_prf_key(const uint8_t* secret, const uint8_t* nonce, uint64_t tau, uint8_t* seed_out, void* stream) {
  if (!secret || !nonce || !seed_out) {
    set_error("null pointer argument");
    return FBM_E_ARG;
  }
  LomPeers pe;
  fill_peers(pe, nonce, tau);
  pe.n_peers = 1;
  memcpy(pe.secret[0], secret, 32);
  return launch_prf_key(pe, (uint32_t*)seed_out, (hipStream_t)stream);
}

int fbm_dequantize(const uint64_t* u, uint64_t n, double neg_clip, double step, double* out, void* stream) {
  if (n > 0 && (!u || !out)) {
    set_error("null pointer argument");
    return FBM_E_ARG;
  }
  return launch_dequantize(u, n, neg_clip, step, out, (hipStream_t)stream);
}

int fbm_lom_aggregate(const uint64_t* y, int n_parties, uint64_t n, uint64_t total_weight, double neg_clip,
                      double step, double* out, uint64_t* sums, uint32_t* stats, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  int rc = zero_stats(stats, s);
  if (rc) return rc;
  if (n_parties < 1 || total_weight == 0 || (n > 0 && !y)) {
    set_error("invalid aggregate arguments (n_parties=%d, total_weight=%llu)", n_parties,
              (unsigned long long)total_weight);
    return FBM_E_ARG;
  }
  return timed("lom_aggregate", s, [&] { return launch_lom_aggregate(y, n_parties, n, total_weight, neg_clip, step, out, sums, stats, s); });
}

// ---- host-buffer LOM calls (small vectors): copy in, kernel, copy out, one stream synchronisation ----
// A 1 000-element list call is launch-bound; these fold its H2D copy, kernel, output and status copies
// and the wait into one C call (no device tensors made per call on the host side).

static int host_copy(void* dst, const void* src, uint64_t bytes, hipMemcpyKind kind, hipStream_t s, const char* what) {
  if (!bytes) return FBM_OK;
  hipError_t e = hipMemcpyAsync(dst, src, bytes, kind, s);
  if (e != hipSuccess) {
    set_error("hipMemcpyAsync(%s): %s", what, hipGetErrorString(e));
    return FBM_E_HIP;
  }
  return FBM_OK;
}

static int host_wait(hipStream_t s) {
  hipError_t e = hipStreamSynchronize(s);
  if (e != hipSuccess) {
    set_error("hipStreamSynchronize: %s", hipGetErrorString(e));
    return FBM_E_HIP;
  }
  return FBM_OK;
}

// workspace: input rows | output (n words) immediately followed by the status words, so that a caller
// whose host output and status words are adjacent too gets both back in one copy
uint64_t fbm_lom_host_workspace(uint64_t n, int n_parties) {
  const uint64_t rows = n_parties > 1 ? (uint64_t)n_parties : 1u;
  return align256(rows * n * 8) + align256(n * 8 + FBM_STATS_WORDS * 4);
}

static int host_copy_back(void* out_host, const void* out, uint64_t n, uint32_t* stats_host, const uint32_t* st,
                          hipStream_t s) {
  if ((uint8_t*)stats_host == (uint8_t*)out_host + n * 8)  // adjacent on the host as on the device: one copy
    return host_copy(out_host, out, n * 8 + FBM_STATS_WORDS * 4, hipMemcpyDeviceToHost, s, "output+stats");
  int rc = host_copy(out_host, out, n * 8, hipMemcpyDeviceToHost, s, "output");
  return rc ? rc : host_copy(stats_host, st, FBM_STATS_WORDS * 4, hipMemcpyDeviceToHost, s, "stats");
}

int fbm_lom_protect_host(const void* x_host, int x_dtype, uint64_t n, double clip, double two_clip, double target_f,
                         uint64_t target_m1, uint64_t weight, const uint8_t* secrets, const int8_t* signs, int n_peers,
                         int raw_seeds, const uint8_t* nonce, uint64_t tau, uint64_t elem_offset, uint64_t* y_host,
                         uint32_t* stats_host, void* workspace, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (!workspace || !stats_host || (n > 0 && (!x_host || !y_host))) {
    set_error("null pointer argument");
    return FBM_E_ARG;
  }
  if (x_dtype != FBM_F32 && x_dtype != FBM_F64 && x_dtype != FBM_U64) {
    set_error("x_dtype must be FBM_F32, FBM_F64 or FBM_U64");
    return FBM_E_ARG;
  }
  uint8_t* w = (uint8_t*)workspace;
  void* x = w;
  uint64_t* y = (uint64_t*)(w + align256(n * 8));
  uint32_t* st = (uint32_t*)(w + align256(n * 8) + n * 8);
  const uint64_t xb = n * (x_dtype == FBM_F32 ? 4u : 8u);
  int rc = host_copy(x, x_host, xb, hipMemcpyHostToDevice, s, "x");
  if (!rc) rc = fbm_lom_protect(x, x_dtype, n, clip, two_clip, target_f, target_m1, weight, secrets, signs, n_peers,
                                raw_seeds, nonce, tau, elem_offset, y, st, stream);
  if (!rc) rc = host_copy_back(y_host, y, n, stats_host, st, s);
  const int wrc = host_wait(s);  // (also after an error: nothing of this call left in flight on the buffers)
  return rc ? rc : wrc;
}

int fbm_lom_aggregate_host(const uint64_t* y_host, int n_parties, uint64_t n, uint64_t total_weight, double neg_clip,
                           double step, double* out_host, uint32_t* stats_host, void* workspace, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (!workspace || !stats_host || (n > 0 && (!y_host || !out_host))) {
    set_error("null pointer argument");
    return FBM_E_ARG;
  }
  if (n_parties < 1) {
    set_error("invalid aggregate arguments (n_parties=%d, total_weight=%llu)", n_parties,
              (unsigned long long)total_weight);
    return FBM_E_ARG;
  }
  uint8_t* w = (uint8_t*)workspace;
  const uint64_t yb = (uint64_t)n_parties * n * 8;
  uint64_t* y = (uint64_t*)w;
  double* out = (double*)(w + align256(yb));
  uint32_t* st = (uint32_t*)(w + align256(yb) + n * 8);
  int rc = host_copy(y, y_host, yb, hipMemcpyHostToDevice, s, "y");
  if (!rc) rc = fbm_lom_aggregate(y, n_parties, n, total_weight, neg_clip, step, out, nullptr, st, stream);
  if (!rc) rc = host_copy_back(out_host, out, n, stats_host, st, s);
  const int wrc = host_wait(s);
  return rc ? rc : wrc;
}

// FBM_COMPACT_H=0 (A/B builds with -DFBM_AB_KNOBS): whole 256-byte H rows for every engine, as before round 4
static bool jl_compact_h() {
#ifdef FBM_AB_KNOBS
  static const bool on = !(getenv("FBM_COMPACT_H") && !strcmp(getenv("FBM_COMPACT_H"), "0"));
  return on;
#else
  return true;
#endif
}

// encrypt workspace: ops | cst | pt [n_ct][32] | nude (blocked) | H [n_ct][64] | table |
//                    H^-1 [n_ct][64] + y [n_ct][32] (negative keys) | Hc [n_ct][8] (compact H rows)
uint64_t fbm_jl_encrypt_workspace(uint64_t n_ct) {
  const uint64_t slots = table_slots_for(n_ct);
  (void)slots;
  return align256(FBM_OPS_WORDS * 4) + align256(FBM_CST_WORDS * 4) + align256(n_ct * 32 * 4) +
         align256(((n_ct + 255) / 256) * 256 * FBM_NL * 4) + 2 * align256(n_ct * 64 * 4) + align256(n_ct * 32 * 4) +
         align256(jl_table_bytes(n_ct)) + align256(n_ct * 8 * 4);
}

uint64_t fbm_jl_aggregate_workspace(uint64_t n_ct) {
  const uint64_t slots = table_slots_for(n_ct);
  (void)slots;
  return align256(FBM_OPS_WORDS * 4) + align256(FBM_CST_WORDS * 4) + align256(((n_ct + 255) / 256) * 256 * FBM_NL * 4) +
         3 * align256(n_ct * 64 * 4) + align256(n_ct * 32 * 4) + align256(jl_table_bytes(n_ct)) + align256(n_ct * 8 * 4);
}

// phase bit 1: the prologue (status word, constants, pack, nude, FDH, and the inverse of H
// for a negative key); bit 2: the exponentiation.  Both phases rebuild the same host
// parameters from the same arguments and use the same workspace, so (1 then 2) == 3.
static int jl_encrypt_impl(const void* x, int x_dtype, uint64_t n, double clip, double two_clip, double target_f,
                           uint64_t target_m1, uint64_t weight, int es, int cr, const uint32_t* biprime,
                           const uint32_t* key, int key_negative, const uint32_t* tau, uint64_t ct_offset, uint32_t* ct_out,
                           void* workspace, uint32_t* stats, void* stream, int phase) {
  hipStream_t s = (hipStream_t)stream;
  int rc;
  if ((phase & 1) && (rc = zero_stats(stats, s))) return rc;
  QuantParams qp;
  if ((rc = quant_params(clip, two_clip, target_f, target_m1, qp))) return rc;
  if (x_dtype != FBM_F32 && x_dtype != FBM_F64 && x_dtype != FBM_U64 && x_dtype != FBM_U128 && x_dtype != FBM_PT) {
    set_error("x_dtype must be FBM_F32, FBM_F64, FBM_U64, FBM_U128 or FBM_PT");
    return FBM_E_ARG;
  }
  if ((x_dtype == FBM_U128 || x_dtype == FBM_PT) && weight != 1) {
    set_error("raw-integer / plaintext inputs take weight 1");
    return FBM_E_ARG;
  }
  if (x_dtype == FBM_PT && cr != 1) {
    set_error("plaintext input (FBM_PT) takes cr = 1");
    return FBM_E_ARG;
  }
  if (!biprime || !key) {
    set_error("null biprime/key");
    return FBM_E_ARG;
  }
  if (!tau) {  // the round is FDH's input: never defaulted (a NULL would silently mean round 0)
    set_error("null tau (the round's %d limbs)", FBM_TAU_LIMBS);
    return FBM_E_ARG;
  }
  if (n == 0) return FBM_OK;
  if (cr < 1) {
    set_error("invalid cr=%d", cr);
    return FBM_E_ARG;
  }
  const uint64_t n_ct = (n + (uint64_t)cr - 1) / (uint64_t)cr;
  if (n_ct > FBM_JL_MAX_CT) {
    set_error("%llu ciphertexts exceed FBM_JL_MAX_CT per call; split the range with ct_offset",
              (unsigned long long)n_ct);
    return FBM_E_UNSUPPORTED;
  }
  if (!x || !ct_out || !workspace) {
    set_error("null pointer argument");
    return FBM_E_ARG;
  }
  if ((int64_t)weight <= -(int64_t)(1 << 17)) {  // negative: the two's complement of a weight > -2^17
    set_error("negative weight %lld outside (-2^17, 0)", (long long)(int64_t)weight);
    return FBM_E_ARG;
  }
  bool generic, short_on;
  if ((rc = jl_path_for(workspace, phase, 3, biprime, generic, short_on))) return rc;
  if (generic) {  // any N (fbm_gen.hip): pack -> FDH -> H^key (N pt + 1) mod N^2
    if (es < 1 || es > 100 || (int64_t)es * cr > 1024) {
      set_error("invalid VES parameters es=%d cr=%d", es, cr);
      return FBM_E_ARG;
    }
    GenCtx g;
    JlParams fp;
    if ((rc = build_gen_ctx(biprime, key, key_negative, g)) || (rc = fdh_params_for_biprime(biprime, tau, ct_offset, fp)))
      return rc;
    uint8_t* ws = (uint8_t*)workspace;  // the encrypt workspace's cst | pt | (nude) | H
    uint32_t* cst = (uint32_t*)(ws + align256(FBM_OPS_WORDS * 4));
    uint32_t* pt = (uint32_t*)(ws + align256(FBM_OPS_WORDS * 4) + align256(FBM_CST_WORDS * 4));
    uint32_t* H = (uint32_t*)((uint8_t*)pt + align256(n_ct * 32 * 4) + align256(((n_ct + 255) / 256) * 256 * FBM_NL * 4));
    const uint32_t* ptp = x_dtype == FBM_PT ? (const uint32_t*)x : pt;
    if (phase & 1) {
      if ((rc = launch_jl_gen_setup(g, cst, s))) return rc;
      if (x_dtype != FBM_PT &&
          (rc = timed("jl_pack", s, [&] { return launch_jl_pack(x, x_dtype, n, qp, weight, es, cr, n_ct, pt, stats, s); })))
        return rc;
      if ((rc = timed("jl_fdh", s, [&] { return launch_jl_fdh(n_ct, fp, H, stats, s); }))) return rc;
    }
    if (!(phase & 2)) return FBM_OK;
    const int negw = (int64_t)weight < 0 ? 1 : 0;
    return timed("jl_gen_exp", s, [&] { return launch_jl_gen_exp(H, ptp, negw, n_ct, cst, ct_out, stats, s); });
  }
  JlParams jp;
  if ((rc = build_jl_params(biprime, es, cr, tau, ct_offset, jp))) return rc;
  JlSched sc;
  int is_zero = 0;
  if ((rc = build_schedule(key, sc, is_zero))) {
    set_error("exponent schedule overflow");
    return rc;
  }
  jp.key_is_zero = is_zero;
  JlShort sh;
  const bool shq = build_short(biprime, key, is_zero, sc, sh, short_on);
  const uint64_t slots = table_slots_for(n_ct);
  uint8_t* ws = (uint8_t*)workspace;
  uint32_t* ops = (uint32_t*)ws;
  uint64_t off = align256(FBM_OPS_WORDS * 4);
  uint32_t* cst = (uint32_t*)(ws + off);
  off += align256(FBM_CST_WORDS * 4);
  uint32_t* pt = (uint32_t*)(ws + off);
  off += align256(n_ct * 32 * 4);
  uint32_t* nude = (uint32_t*)(ws + off);
  off += align256(((n_ct + 255) / 256) * 256 * FBM_NL * 4);
  uint32_t* H = (uint32_t*)(ws + off);
  off += align256(n_ct * 64 * 4);
  uint32_t* table = (uint32_t*)(ws + off);
  off += align256(jl_table_bytes(n_ct));
  uint32_t* Hinv = (uint32_t*)(ws + off);  // negative keys only: H^|key| digits (after the table)
  off += align256(n_ct * 64 * 4);
  uint32_t* Y = (uint32_t*)(ws + off);
  off += align256(n_ct * 32 * 4);
  uint32_t* Hc = jl_compact_h() ? (uint32_t*)(ws + off) : nullptr;  // compact H rows: 32 B per ciphertext
  const bool inverse = key_negative && !is_zero;
  if (phase & 1) {
    if ((rc = timed("jl_setup", s, [&] { return launch_jl_setup(jp, sc, ops, cst, s, shq ? &sh : nullptr); })))
      return rc;
    if (x_dtype != FBM_PT &&
        (rc = timed("jl_pack", s, [&] { return launch_jl_pack(x, x_dtype, n, qp, weight, es, cr, n_ct, pt, stats, s); })))
      return rc;
    const uint32_t* ptp = x_dtype == FBM_PT ? (const uint32_t*)x : pt;  // UserKey.encrypt: packed already
    const int negw = (int64_t)weight < 0 ? 1 : 0;
    if ((rc = timed("jl_nude", s, [&] { return launch_jl_nude(ptp, n_ct, jp, negw, nude, s); }))) return rc;
    if (!is_zero && (rc = timed("jl_fdh", s, [&] { return launch_jl_fdh(n_ct, jp, H, stats, s, Hc); }))) return rc;
  }
  if (!(phase & 2)) return FBM_OK;
  if (inverse) {
    // gmpy2.powmod with a negative exponent (_jls.py:60-73) is (H^-1)^|key| = (H^|key|)^-1:
    // the power's N-adic digits (any H < 2^2048), then the lift inverts it and multiplies
    // by nude in the same pass
    if ((rc = timed("jl_exp", s, [&] {
           return launch_jl_exp(H, n_ct, jp, sc, FBM_EXP_DEC | FBM_EXP_OUT_NADIC, nullptr, table, slots, ops, cst, Hinv,
                                s, Hc);
         })))
      return rc;
    return timed("jl_inv", s, [&] { return launch_jl_inv(n_ct, jp, cst, Hinv, Y, nude, ct_out, stats, s); });
  }
  // a phase-2-only call inside an open batch (fbm_jl_batch_begin) is recorded, not launched
  // (and not timed: the batch's one launch is, at the flush)
  auto go = [&] { return launch_jl_exp(H, n_ct, jp, sc, 0, nude, table, slots, ops, cst, ct_out, s, Hc); };
  const bool rec = phase == 2 && jl_batch_active();
  const bool acc = jl_batch_accept(rec);
  rc = rec ? go() : timed("jl_exp", s, go);
  jl_batch_accept(acc);
  return rc;
}

int fbm_jl_encrypt(const void* x, int x_dtype, uint64_t n, double clip, double two_clip, double target_f,
                   uint64_t target_m1, uint64_t weight, int es, int cr, const uint32_t* biprime, const uint32_t* key,
                   int key_negative, const uint32_t* tau, uint64_t ct_offset, uint32_t* ct_out, void* workspace,
                   uint32_t* stats, void* stream) {
  return jl_encrypt_impl(x, x_dtype, n, clip, two_clip, target_f, target_m1, weight, es, cr, biprime, key,
                         key_negative, tau, ct_offset, ct_out, workspace, stats, stream, 3);
}

// The encrypt with its factor computed ahead: c_k = (N pt_k + 1) F_k mod N^2, F_k = H(t_k)^sk the
// decryption-factor kernels' output for the party's key (fbm_jl_decrypt_factor) -- fbm_jl_encrypt's
// ciphertexts bit for bit (the exponentiation's only input besides the plaintext is H(t_k)).  Any
// engine policy; the modulus must be odd and >= 3 (other moduli: fbm_jl_encrypt).
int fbm_jl_encrypt_factor(const void* x, int x_dtype, uint64_t n, double clip, double two_clip, double target_f,
                          uint64_t target_m1, uint64_t weight, int es, int cr, const uint32_t* biprime,
                          const uint32_t* factor, uint32_t* ct_out, void* workspace, uint32_t* stats, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  int rc = zero_stats(stats, s);
  if (rc) return rc;
  QuantParams qp;
  if ((rc = quant_params(clip, two_clip, target_f, target_m1, qp))) return rc;
  if (x_dtype != FBM_F32 && x_dtype != FBM_F64 && x_dtype != FBM_U64 && x_dtype != FBM_U128 && x_dtype != FBM_PT) {
    set_error("x_dtype must be FBM_F32, FBM_F64, FBM_U64, FBM_U128 or FBM_PT");
    return FBM_E_ARG;
  }
  if ((x_dtype == FBM_U128 || x_dtype == FBM_PT) && weight != 1) {
    set_error("raw-integer / plaintext inputs take weight 1");
    return FBM_E_ARG;
  }
  if (x_dtype == FBM_PT && cr != 1) {
    set_error("plaintext input (FBM_PT) takes cr = 1");
    return FBM_E_ARG;
  }
  if (!biprime) {
    set_error("null biprime");
    return FBM_E_ARG;
  }
  if (n == 0) return FBM_OK;
  if (cr < 1) {
    set_error("invalid cr=%d", cr);
    return FBM_E_ARG;
  }
  const uint64_t n_ct = (n + (uint64_t)cr - 1) / (uint64_t)cr;
  if (n_ct > FBM_JL_MAX_CT) {
    set_error("%llu ciphertexts exceed FBM_JL_MAX_CT per call; split the range with ct_offset",
              (unsigned long long)n_ct);
    return FBM_E_UNSUPPORTED;
  }
  if (!x || !factor || !ct_out || !workspace) {
    set_error("null pointer argument");
    return FBM_E_ARG;
  }
  {  // jl_encf_kernel stages N pt + 1 in the output rows before it reads the factor rows
    const uintptr_t o0 = (uintptr_t)ct_out, o1 = o0 + n_ct * 256, f0 = (uintptr_t)factor, f1 = f0 + n_ct * 256;
    if (o0 < f1 && f0 < o1) {
      set_error("fbm_jl_encrypt_factor: ct_out must not overlap factor");
      return FBM_E_ARG;
    }
  }
  if ((int64_t)weight <= -(int64_t)(1 << 17)) {
    set_error("negative weight %lld outside (-2^17, 0)", (long long)(int64_t)weight);
    return FBM_E_ARG;
  }
  if ((biprime[0] & 1u) == 0u || jl_is_one(biprime)) {
    set_error("fbm_jl_encrypt_factor takes an odd N >= 3 (fbm_jl_encrypt takes any N)");
    return FBM_E_UNSUPPORTED;
  }
  JlParams jp;
  if ((rc = build_jl_params(biprime, es, cr, nullptr, 0, jp))) return rc;
  JlSched none;
  memset(&none, 0, sizeof(none));
  uint8_t* ws = (uint8_t*)workspace;  // the encrypt workspace's ops | cst | pt
  uint32_t* ops = (uint32_t*)ws;
  uint32_t* cst = (uint32_t*)(ws + align256(FBM_OPS_WORDS * 4));
  uint32_t* pt = (uint32_t*)(ws + align256(FBM_OPS_WORDS * 4) + align256(FBM_CST_WORDS * 4));
  if ((rc = timed("jl_setup", s, [&] { return launch_jl_setup(jp, none, ops, cst, s); }))) return rc;
  {  // R^2 mod N^2: two products, each dropping one R
    JlRk r;
    jl_rk_for(jp.N32, 1, r);
    if ((rc = timed("jl_rk", s, [&] { return launch_jl_rk(r, cst, s); }))) return rc;
  }
  if (x_dtype != FBM_PT &&
      (rc = timed("jl_pack", s, [&] { return launch_jl_pack(x, x_dtype, n, qp, weight, es, cr, n_ct, pt, stats, s); })))
    return rc;
  const uint32_t* ptp = x_dtype == FBM_PT ? (const uint32_t*)x : pt;
  const int negw = (int64_t)weight < 0 ? 1 : 0;
  return timed("jl_encf", s, [&] { return launch_jl_encf(ptp, n_ct, jp, cst, negw, factor, ct_out, s); });
}

int fbm_jl_encrypt_phase(const void* x, int x_dtype, uint64_t n, double clip, double two_clip, double target_f,
                         uint64_t target_m1, uint64_t weight, int es, int cr, const uint32_t* biprime,
                         const uint32_t* key, int key_negative, const uint32_t* tau, uint64_t ct_offset, uint32_t* ct_out,
                         void* workspace, uint32_t* stats, void* stream, int phase) {
  if (phase < 1 || phase > 3) {
    set_error("fbm_jl_encrypt_phase: phase must be 1, 2 or 3");
    return FBM_E_ARG;
  }
  return jl_encrypt_impl(x, x_dtype, n, clip, two_clip, target_f, target_m1, weight, es, cr, biprime, key,
                         key_negative, tau, ct_offset, ct_out, workspace, stats, stream, phase);
}

// aggregate workspace: ops | cst | X (blocked) | H [n_ct][64] | E [n_ct][64] | F [n_ct][64] |
//                      xs [n_ct][32] | table    (fbm_jl_aggregate_workspace)
struct JlAggWs {
  uint32_t *ops, *cst, *X, *H, *E, *F, *xs, *table, *Hc;
  uint64_t slots;
};
static JlAggWs agg_ws(void* workspace, uint64_t n_ct) {
  JlAggWs w;
  uint8_t* ws = (uint8_t*)workspace;
  w.slots = table_slots_for(n_ct);
  uint64_t off = 0;
  w.ops = (uint32_t*)ws;
  off += align256(FBM_OPS_WORDS * 4);
  w.cst = (uint32_t*)(ws + off);
  off += align256(FBM_CST_WORDS * 4);
  w.X = (uint32_t*)(ws + off);
  off += align256(((n_ct + 255) / 256) * 256 * FBM_NL * 4);
  w.H = (uint32_t*)(ws + off);
  off += align256(n_ct * 64 * 4);
  w.E = (uint32_t*)(ws + off);
  off += align256(n_ct * 64 * 4);
  w.F = (uint32_t*)(ws + off);
  off += align256(n_ct * 64 * 4);
  w.xs = (uint32_t*)(ws + off);
  off += align256(n_ct * 32 * 4);
  w.table = (uint32_t*)(ws + off);
  off += align256(jl_table_bytes(n_ct));
  w.Hc = jl_compact_h() ? (uint32_t*)(ws + off) : nullptr;
  return w;
}

// ServerKey's factor H(t_k)^sk0 mod N^2 (inverse first for sk0 < 0): depends on the round,
// the ciphertext index and the key only -- not on the parties' ciphertexts.
// phase bits: 1 = constants + FDH, 2 = the exponentiation, 4 = the inverse (negative key)
static int jl_factor_impl(uint64_t n_ct, const uint32_t* biprime, const uint32_t* key, int key_negative, const uint32_t* tau,
                          uint64_t ct_offset, uint32_t* factor, const JlAggWs& w, uint32_t* stats, hipStream_t s,
                          int phase = 7) {
  JlParams jp;
  int rc;
  if (!tau) {
    set_error("null tau (the round's %d limbs)", FBM_TAU_LIMBS);
    return FBM_E_ARG;
  }
  bool generic, short_on;
  if ((rc = jl_path_for(w.ops, phase, 7, biprime, generic, short_on))) return rc;
  if (generic) {  // any N: FDH, then H^key mod N^2 with the inverse in the same kernel
    GenCtx g;
    if ((rc = build_gen_ctx(biprime, key, key_negative, g)) || (rc = fdh_params_for_biprime(biprime, tau, ct_offset, jp)))
      return rc;
    if (phase & 1) {
      if ((rc = launch_jl_gen_setup(g, w.cst, s))) return rc;
      if ((rc = timed("jl_fdh", s, [&] { return launch_jl_fdh(n_ct, jp, w.H, stats, s); }))) return rc;
    }
    if (phase & 2)
      return timed("jl_gen_exp", s, [&] { return launch_jl_gen_exp(w.H, nullptr, 0, n_ct, w.cst, factor, stats, s); });
    return FBM_OK;
  }
  if ((rc = build_jl_params(biprime, 1, 1, tau, ct_offset, jp))) return rc;
  JlSched sc;
  int is_zero = 0;
  if ((rc = build_schedule(key, sc, is_zero))) {
    set_error("exponent schedule overflow");
    return rc;
  }
  jp.key_is_zero = is_zero;
  JlShort sh;
  const bool shq = build_short(biprime, key, is_zero, sc, sh, short_on);
  const bool inv = key_negative && !is_zero;
  uint32_t* E = inv ? w.E : factor;
  if (phase & 1) {
    if ((rc = timed("jl_setup", s, [&] { return launch_jl_setup(jp, sc, w.ops, w.cst, s, shq ? &sh : nullptr); })))
      return rc;
    if (!is_zero && (rc = timed("jl_fdh", s, [&] { return launch_jl_fdh(n_ct, jp, w.H, stats, s, w.Hc); })))
      return rc;
  }
  if (phase & 2) {
    // the inverse starts from the power's N-adic digits (no division by N needed)
    auto go = [&] {
      return launch_jl_exp(w.H, n_ct, jp, sc, FBM_EXP_DEC | (inv ? FBM_EXP_OUT_NADIC : 0), nullptr, w.table, w.slots,
                           w.ops, w.cst, E, s, w.Hc);
    };
    const bool rec = phase == 2 && jl_batch_active();  // recorded (not launched, not timed) in an open batch
    const bool acc = jl_batch_accept(rec);
    rc = rec ? go() : timed("jl_exp", s, go);
    jl_batch_accept(acc);
    if (rc) return rc;
  }
  if ((phase & 4) && inv && jl_batch_active()) {
    set_error("the decryption factor's inverse needs its exponentiation: flush the open batch first");
    return FBM_E_ARG;
  }
  if ((phase & 4) && inv &&
      (rc = timed("jl_inv", s, [&] { return launch_jl_inv(n_ct, jp, w.cst, E, w.xs, nullptr, factor, stats, s); })))  // xs: y scratch
    return rc;
  return FBM_OK;
}

// v = prod_u c_u * factor mod N^2, x = (v-1)/N, decode + average + dequantise
// x_raw != NULL: ServerKey.decrypt's x to x_raw [n_ct][32] instead of decode/average/dequantise
static int jl_combine_impl(const uint32_t* cts, int n_parties, uint64_t n_ct, int es, int cr, uint64_t n_out,
                           const uint32_t* biprime, const uint32_t* factor, uint64_t total_weight, double neg_clip,
                           double step, double* out, uint64_t* sums, const JlAggWs& w, uint32_t* stats, hipStream_t s,
                           uint32_t* x_raw = nullptr) {
  JlParams jp;
  int rc;
  if (jl_is_one(biprime)) {  // the reference's invert(delta^2, N^2) has no nonzero result modulo 1
    set_error("invert() no inverse exists");
    return FBM_E_INVERSE;
  }
  if (jl_generic(biprime)) {  // any N: product, factor, ((v - 1) // N) mod N, then the decode
    if (es < 1 || cr < 1 || es > 100 || (int64_t)es * cr > 1024) {
      set_error("invalid VES parameters es=%d cr=%d", es, cr);
      return FBM_E_ARG;
    }
    GenCtx g;
    if ((rc = build_gen_ctx(biprime, nullptr, 0, g)) || (rc = launch_jl_gen_setup(g, w.cst, s))) return rc;
    uint32_t* xs = x_raw ? x_raw : w.xs;
    if ((rc = timed("jl_gen_combine", s, [&] {
           return launch_jl_gen_combine(cts, n_parties, n_ct, factor, w.cst, FBM_GEN_DECRYPT, xs, stats, s);
         })))
      return rc;
    if (x_raw) return FBM_OK;
    return timed("jl_decode", s, [&] {
      return launch_jl_decode(w.xs, es, cr, n_out, total_weight, neg_clip, step, out, sums, stats, s);
    });
  }
  if ((rc = build_jl_params(biprime, es, cr, nullptr, 0, jp))) return rc;
  JlSched none;
  memset(&none, 0, sizeof(none));
  if ((rc = timed("jl_setup", s, [&] { return launch_jl_setup(jp, none, w.ops, w.cst, s); }))) return rc;
  {  // R^(P+1) mod N^2: the product's uniform first operand (P + 1 products each drop one R)
    JlRk r;
    jl_rk_for(jp.N32, n_parties, r);
    if ((rc = timed("jl_rk", s, [&] { return launch_jl_rk(r, w.cst, s); }))) return rc;
  }
  uint32_t* xs = x_raw ? x_raw : w.xs;
  if ((rc = timed("jl_prod", s, [&] { return launch_jl_prod(cts, n_parties, n_ct, jp, w.cst, factor, xs, s); })))
    return rc;
  if (x_raw) return FBM_OK;
  return timed("jl_decode", s, [&] {
    return launch_jl_decode(w.xs, es, cr, n_out, total_weight, neg_clip, step, out, sums, stats, s);
  });
}

static int jl_agg_checks(int n_parties, uint64_t n_ct, const uint32_t* biprime, uint64_t total_weight) {
  if (n_parties < 1 || !biprime || total_weight == 0) {
    set_error("invalid aggregate arguments");
    return FBM_E_ARG;
  }
  if (n_ct > FBM_JL_MAX_CT) {
    set_error("%llu ciphertexts exceed FBM_JL_MAX_CT per call; split the range with ct_offset",
              (unsigned long long)n_ct);
    return FBM_E_UNSUPPORTED;
  }
  return FBM_OK;
}

int fbm_jl_aggregate(const uint32_t* cts, int n_parties, uint64_t n_ct, int es, int cr, uint64_t n_out,
                     const uint32_t* biprime, const uint32_t* key, int key_negative, const uint32_t* tau, uint64_t ct_offset,
                     uint64_t total_weight, double neg_clip, double step, double* out, uint64_t* sums,
                     void* workspace, uint32_t* stats, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  int rc = zero_stats(stats, s);
  if (rc) return rc;
  if ((rc = jl_agg_checks(n_parties, n_ct, biprime, total_weight))) return rc;
  if (!key) {
    set_error("null key");
    return FBM_E_ARG;
  }
  if (n_ct == 0) return FBM_OK;
  if (n_out > n_ct * (uint64_t)cr) n_out = n_ct * (uint64_t)cr;
  if (!cts || !workspace) {
    set_error("null pointer argument");
    return FBM_E_ARG;
  }
  const JlAggWs w = agg_ws(workspace, n_ct);
  if ((rc = jl_factor_impl(n_ct, biprime, key, key_negative, tau, ct_offset, w.F, w, stats, s))) return rc;
  return jl_combine_impl(cts, n_parties, n_ct, es, cr, n_out, biprime, w.F, total_weight, neg_clip, step, out, sums, w,
                         stats, s);
}

int fbm_jl_decrypt_factor(uint64_t n_ct, const uint32_t* biprime, const uint32_t* key, int key_negative, const uint32_t* tau,
                          uint64_t ct_offset, uint32_t* factor, void* workspace, uint32_t* stats, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  int rc = zero_stats(stats, s);
  if (rc) return rc;
  if ((rc = jl_agg_checks(1, n_ct, biprime, 1))) return rc;
  if (n_ct == 0) return FBM_OK;
  if (!key || !factor || !workspace) {
    set_error("null pointer argument");
    return FBM_E_ARG;
  }
  return jl_factor_impl(n_ct, biprime, key, key_negative, tau, ct_offset, factor, agg_ws(workspace, n_ct), stats, s);
}

int fbm_jl_decrypt_factor_phase(uint64_t n_ct, const uint32_t* biprime, const uint32_t* key, int key_negative,
                                const uint32_t* tau, uint64_t ct_offset, uint32_t* factor, void* workspace, uint32_t* stats,
                                void* stream, int phase) {
  hipStream_t s = (hipStream_t)stream;
  int rc;
  if (phase < 1 || phase > 7) {
    set_error("fbm_jl_decrypt_factor_phase: phase must be a non-empty subset of {1, 2, 4}");
    return FBM_E_ARG;
  }
  if ((phase & 1) && (rc = zero_stats(stats, s))) return rc;
  if ((rc = jl_agg_checks(1, n_ct, biprime, 1))) return rc;
  if (n_ct == 0) return FBM_OK;
  if (!key || !factor || !workspace) {
    set_error("null pointer argument");
    return FBM_E_ARG;
  }
  return jl_factor_impl(n_ct, biprime, key, key_negative, tau, ct_offset, factor, agg_ws(workspace, n_ct), stats, s,
                        phase);
}

int fbm_jl_aggregate_factor(const uint32_t* cts, int n_parties, uint64_t n_ct, int es, int cr, uint64_t n_out,
                            const uint32_t* biprime, const uint32_t* factor, uint64_t total_weight, double neg_clip,
                            double step, double* out, uint64_t* sums, void* workspace, uint32_t* stats, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  int rc = zero_stats(stats, s);
  if (rc) return rc;
  if ((rc = jl_agg_checks(n_parties, n_ct, biprime, total_weight))) return rc;
  if (n_ct == 0) return FBM_OK;
  if (n_out > n_ct * (uint64_t)cr) n_out = n_ct * (uint64_t)cr;
  if (!cts || !factor || !workspace) {
    set_error("null pointer argument");
    return FBM_E_ARG;
  }
  return jl_combine_impl(cts, n_parties, n_ct, es, cr, n_out, biprime, factor, total_weight, neg_clip, step, out, sums,
                         agg_ws(workspace, n_ct), stats, s);
}

// ---- the JoyeLibert object API (fedbiomed_amd/secagg/_jls.py) ----
int fbm_jl_pack(const void* x, int x_dtype, uint64_t n, int es, int cr, uint32_t* pt, uint32_t* stats, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  int rc = zero_stats(stats, s);
  if (rc) return rc;
  if (x_dtype != FBM_U128) {
    set_error("fbm_jl_pack takes FBM_U128 values");
    return FBM_E_ARG;
  }
  if (es < 1 || cr < 1 || (int64_t)es * cr > 1024) {
    set_error("invalid VES parameters es=%d cr=%d", es, cr);
    return FBM_E_ARG;
  }
  if (n == 0) return FBM_OK;
  if (!x || !pt) {
    set_error("null pointer argument");
    return FBM_E_ARG;
  }
  const uint64_t n_ct = (n + (uint64_t)cr - 1) / (uint64_t)cr;
  QuantParams qp{};
  return timed("jl_pack", s, [&] { return launch_jl_pack(x, x_dtype, n, qp, 1, es, cr, n_ct, pt, stats, s); });
}

int fbm_jl_unpack(const uint32_t* pt, uint64_t n_ct, int es, int cr, uint64_t n_out, uint64_t* vals, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (es < 1 || es > 128 || cr < 1 || (int64_t)es * cr > 1024) {
    set_error("invalid VES parameters es=%d cr=%d (device decode: es <= 128)", es, cr);
    return FBM_E_ARG;
  }
  if (n_out > n_ct * (uint64_t)cr) n_out = n_ct * (uint64_t)cr;
  if (n_out == 0) return FBM_OK;
  if (!pt || !vals) {
    set_error("null pointer argument");
    return FBM_E_ARG;
  }
  return timed("jl_decode", s, [&] { return launch_jl_decode(pt, es, cr, n_out, 1, 0.0, 1.0, nullptr, vals, nullptr, s); });
}

int fbm_jl_fdh(uint64_t n_ct, const uint32_t* modulus_odd, int modulus_even, const uint32_t* tau, uint64_t ct_offset,
               uint32_t* h, uint32_t* stats, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  int rc = zero_stats(stats, s);
  if (rc) return rc;
  if (!modulus_odd || !tau) {
    set_error("null modulus or tau");
    return FBM_E_ARG;
  }
  JlParams jp;
  if ((rc = fdh_params(modulus_odd, modulus_even, tau, ct_offset, jp))) return rc;
  if (n_ct == 0) return FBM_OK;
  if (!h) {
    set_error("null pointer argument");
    return FBM_E_ARG;
  }
  return timed("jl_fdh", s, [&] { return launch_jl_fdh(n_ct, jp, h, stats, s); });
}

int fbm_jl_fdh_msg(uint64_t n, const uint32_t* t, int t_words, int bits_size, const uint32_t* modulus_odd,
                   int modulus_even, uint32_t* h, int h_words, uint32_t* stats, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  int rc = zero_stats(stats, s);
  if (rc) return rc;
  if (!modulus_odd || bits_size < 0 || t_words < 0) {
    set_error("fbm_jl_fdh_msg: null modulus or negative size");
    return FBM_E_ARG;
  }
  const int msg_bytes = bits_size / 2;  // int(t).to_bytes(bits_size // 2, 'big')
  if ((int64_t)t_words * 4 < msg_bytes) {
    set_error("fbm_jl_fdh_msg: %d words hold no %d-byte message", t_words, msg_bytes);
    return FBM_E_ARG;
  }
  if (!(modulus_odd[0] & 1u)) {
    set_error("fbm_jl_fdh_msg: the modulus's odd part must be odd");
    return FBM_E_ARG;
  }
  // digests r may hold: the reference's inner loop breaks while r is shorter than bits_size // 8 bytes
  const int bytes = bits_size / 8;
  const int kmax = bytes >= 1 ? (bytes - 1) / 32 : 0;
  if (n == 0) return FBM_OK;
  if (kmax == 0) {  // a single digest is already bits_size // 8 bytes: the counter byte overflows at 256
    set_error("FDH of bits_size %d: r never shorter than bits_size // 8 bytes (reference: OverflowError)", bits_size);
    return FBM_E_FDH;
  }
  if (!t || !h) {
    set_error("null pointer argument");
    return FBM_E_ARG;
  }
  const int need = fbm_jl_fdh_msg_row_words(bits_size);
  if (h_words < need) {
    set_error("fbm_jl_fdh_msg: rows of %d words hold no r of bits_size %d (%d words)", h_words, bits_size, need);
    return FBM_E_ARG;
  }
  if (kmax <= FBM_FDH_MSG_DIGESTS) {
    if (h_words != FBM_FDH_MSG_ROW) {
      set_error("fbm_jl_fdh_msg: bits_size %d takes rows of %d words", bits_size, FBM_FDH_MSG_ROW);
      return FBM_E_ARG;
    }
    return timed("jl_fdh", s, [&] {
      return launch_jl_fdh_msg(n, t, t_words, msg_bytes, kmax, modulus_odd, modulus_even ? 1 : 0, h, stats, s);
    });
  }
  // r of up to 255 digests: the incremental Montgomery residue of the wide kernel (fbm_jl.hip)
  Big m(modulus_odd, modulus_odd + 32);
  uint32_t inv = m[0];  // Newton: m^-1 mod 2^32
  for (int i = 0; i < 5; ++i) inv *= 2u - m[0] * inv;
  Big k1 = big_pow2_mod(1024 + 256, m), k2 = big_pow2_mod(2048, m);
  k1.resize(32, 0u);
  k2.resize(32, 0u);
  return timed("jl_fdh", s, [&] {
    return launch_jl_fdh_msg_wide(n, t, t_words, msg_bytes, kmax, m.data(), k1.data(), k2.data(), 0u - inv,
                                  modulus_even ? 1 : 0, h, h_words, stats, s);
  });
}

int fbm_jl_fdh_msg_row_words(int bits_size) {
  const int bytes = bits_size / 8;
  int kmax = bytes >= 1 ? (bytes - 1) / 32 : 0;
  if (kmax > 255) kmax = 255;
  return kmax <= FBM_FDH_MSG_DIGESTS ? FBM_FDH_MSG_ROW : 8 * kmax;
}

int fbm_jl_product(const uint32_t* cts, int n_parties, uint64_t n_ct, const uint32_t* biprime, uint32_t* out,
                   void* workspace, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  int rc;
  if ((rc = jl_agg_checks(n_parties, n_ct, biprime, 1))) return rc;
  if (n_ct == 0) return FBM_OK;
  if (!cts || !out || !workspace) {
    set_error("null pointer argument");
    return FBM_E_ARG;
  }
  const JlAggWs w = agg_ws(workspace, n_ct);
  if (jl_generic(biprime)) {
    GenCtx g;
    if ((rc = build_gen_ctx(biprime, nullptr, 0, g)) || (rc = launch_jl_gen_setup(g, w.cst, s))) return rc;
    return timed("jl_gen_combine", s, [&] {
      return launch_jl_gen_combine(cts, n_parties, n_ct, nullptr, w.cst, FBM_GEN_PRODUCT, out, nullptr, s);
    });
  }
  JlParams jp;
  if ((rc = build_jl_params(biprime, 1, 1, nullptr, 0, jp))) return rc;
  JlSched none;
  memset(&none, 0, sizeof(none));
  if ((rc = timed("jl_setup", s, [&] { return launch_jl_setup(jp, none, w.ops, w.cst, s); }))) return rc;
  {  // R^P: P products, each dropping one R
    JlRk r;
    jl_rk_for(jp.N32, n_parties - 1, r);
    if ((rc = timed("jl_rk", s, [&] { return launch_jl_rk(r, w.cst, s); }))) return rc;
  }
  return timed("jl_prod", s, [&] { return launch_jl_prod(cts, n_parties, n_ct, jp, w.cst, nullptr, out, s); });
}

int fbm_jl_decrypt(const uint32_t* cts, int n_parties, uint64_t n_ct, const uint32_t* biprime, const uint32_t* key,
                   int key_negative, const uint32_t* tau, uint64_t ct_offset, uint32_t* x, void* workspace, uint32_t* stats,
                   void* stream) {
  hipStream_t s = (hipStream_t)stream;
  int rc = zero_stats(stats, s);
  if (rc) return rc;
  if ((rc = jl_agg_checks(n_parties, n_ct, biprime, 1))) return rc;
  if (!key) {
    set_error("null key");
    return FBM_E_ARG;
  }
  if (n_ct == 0) return FBM_OK;
  if (!cts || !x || !workspace) {
    set_error("null pointer argument");
    return FBM_E_ARG;
  }
  const JlAggWs w = agg_ws(workspace, n_ct);
  if ((rc = jl_factor_impl(n_ct, biprime, key, key_negative, tau, ct_offset, w.F, w, stats, s))) return rc;
  return jl_combine_impl(cts, n_parties, n_ct, 1, 1, 0, biprime, w.F, 1, 0.0, 1.0, nullptr, nullptr, w, stats, s, x);
}

// out[k] = nude_k * h[k]^key mod N^2 for caller-given bases (a PublicParam whose hashing function
// is not FBM's FDH): the encrypt's exponentiation without its FDH (nude = N pt + 1), or with
// pt == NULL the decryption factor's (the power alone).  Workspace: the encrypt's layout.
int fbm_jl_powmod(const uint32_t* h, const uint32_t* pt, uint64_t n_ct, const uint32_t* biprime, const uint32_t* key,
                  int key_negative, uint32_t* out, void* workspace, uint32_t* stats, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  int rc = zero_stats(stats, s);
  if (rc) return rc;
  if ((rc = jl_agg_checks(1, n_ct, biprime, 1))) return rc;
  if (!key) {
    set_error("null key");
    return FBM_E_ARG;
  }
  if (n_ct == 0) return FBM_OK;
  if (!h || !out || !workspace) {
    set_error("null pointer argument");
    return FBM_E_ARG;
  }
  uint8_t* ws = (uint8_t*)workspace;  // fbm_jl_encrypt_workspace: ops | cst | pt | nude | H | table | H^-1 | y
  uint32_t* ops = (uint32_t*)ws;
  uint64_t off = align256(FBM_OPS_WORDS * 4);
  uint32_t* cst = (uint32_t*)(ws + off);
  off += align256(FBM_CST_WORDS * 4) + align256(n_ct * 32 * 4);
  uint32_t* nude = (uint32_t*)(ws + off);
  off += align256(((n_ct + 255) / 256) * 256 * FBM_NL * 4) + align256(n_ct * 64 * 4);
  uint32_t* table = (uint32_t*)(ws + off);
  off += align256(jl_table_bytes(n_ct));
  uint32_t* Hinv = (uint32_t*)(ws + off);
  off += align256(n_ct * 64 * 4);
  uint32_t* Y = (uint32_t*)(ws + off);
  if (jl_generic(biprime)) {
    GenCtx g;
    if ((rc = build_gen_ctx(biprime, key, key_negative, g)) || (rc = launch_jl_gen_setup(g, cst, s))) return rc;
    return timed("jl_gen_exp", s, [&] { return launch_jl_gen_exp(h, pt, 0, n_ct, cst, out, stats, s); });
  }
  JlParams jp;
  if ((rc = build_jl_params(biprime, 1, 1, nullptr, 0, jp))) return rc;
  JlSched sc;
  int is_zero = 0;
  if ((rc = build_schedule(key, sc, is_zero))) {
    set_error("exponent schedule overflow");
    return rc;
  }
  jp.key_is_zero = is_zero;
  JlShort sh;
  const bool shq = build_short(biprime, key, is_zero, sc, sh, t_short_on != 0);
  const uint64_t slots = table_slots_for(n_ct);
  if ((rc = timed("jl_setup", s, [&] { return launch_jl_setup(jp, sc, ops, cst, s, shq ? &sh : nullptr); })))
    return rc;
  const int mode = pt ? 0 : FBM_EXP_DEC;
  if (pt && (rc = timed("jl_nude", s, [&] { return launch_jl_nude(pt, n_ct, jp, 0, nude, s); }))) return rc;
  if (key_negative && !is_zero) {  // powmod with a negative exponent: (h^|key|)^-1, then * nude
    if ((rc = timed("jl_exp", s, [&] {
           return launch_jl_exp(h, n_ct, jp, sc, FBM_EXP_DEC | FBM_EXP_OUT_NADIC, nullptr, table, slots, ops, cst, Hinv,
                                s);
         })))
      return rc;
    return timed("jl_inv", s, [&] { return launch_jl_inv(n_ct, jp, cst, Hinv, Y, pt ? nude : nullptr, out, stats, s); });
  }
  return timed("jl_exp", s, [&] {
    return launch_jl_exp(h, n_ct, jp, sc, mode, pt ? nude : nullptr, table, slots, ops, cst, out, s);
  });
}

// ServerKey.decrypt's last step with a caller-computed factor (fbm_jl_powmod, pt == NULL):
// x = ((prod_u cts[u] * factor mod N^2) - 1) // N mod N
int fbm_jl_decrypt_with(const uint32_t* cts, int n_parties, uint64_t n_ct, const uint32_t* biprime,
                        const uint32_t* factor, uint32_t* x, void* workspace, uint32_t* stats, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  int rc = zero_stats(stats, s);
  if (rc) return rc;
  if ((rc = jl_agg_checks(n_parties, n_ct, biprime, 1))) return rc;
  if (n_ct == 0) return FBM_OK;
  if (!cts || !factor || !x || !workspace) {
    set_error("null pointer argument");
    return FBM_E_ARG;
  }
  return jl_combine_impl(cts, n_parties, n_ct, 1, 1, 0, biprime, factor, 1, 0.0, 1.0, nullptr, nullptr,
                         agg_ws(workspace, n_ct), stats, s, x);
}

int fbm_int_ops(const uint64_t* x, uint64_t n, uint64_t k, int op, void* out, uint32_t* stats, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  int rc = zero_stats(stats, s);
  if (rc) return rc;
  if (op < 0 || op > 3 || ((op == 1 || op == 3) && k == 0)) {
    set_error("fbm_int_ops: op must be 0 (multiply), 1 / 3 (divide by k / -k, k >= 1) or 2 (divide by a float64)");
    return FBM_E_ARG;
  }
  if (n == 0) return FBM_OK;
  if (!x || !out) {
    set_error("null pointer argument");
    return FBM_E_ARG;
  }
  return timed("int_ops", s, [&] {
    return launch_int_ops(x, n, k, op, op == 0 ? (uint64_t*)out : nullptr, op != 0 ? (double*)out : nullptr, stats, s);
  });
}

int fbm_ves_pack(const uint32_t* x, uint64_t n, int wv, int es, int cr, int pw, int is_signed, uint32_t* pt,
                 void* stream) {
  if (wv < 1 || es < 1 || cr < 1 || pw < 1 || (int64_t)es * (cr - 1) + 32ll * wv > 32ll * pw) {
    set_error("fbm_ves_pack: bad shape (wv=%d es=%d cr=%d pw=%d)", wv, es, cr, pw);
    return FBM_E_ARG;
  }
  if (n > 0 && (!x || !pt)) {
    set_error("null pointer argument");
    return FBM_E_ARG;
  }
  return timed("ves_pack", (hipStream_t)stream,
               [&] { return launch_ves_pack(x, n, wv, es, cr, pw, is_signed ? 1 : 0, pt, (hipStream_t)stream); });
}

int fbm_ves_unpack(const uint32_t* pt, uint64_t n_ct, int pw, int es, int cr, uint64_t n_out, int ow, uint32_t* vals,
                   void* stream) {
  if (pw < 1 || es < 1 || cr < 1 || ow < (es + 31) / 32 || (int64_t)es * cr > 32ll * pw || n_out > n_ct * (uint64_t)cr) {
    set_error("fbm_ves_unpack: bad shape (pw=%d es=%d cr=%d ow=%d)", pw, es, cr, ow);
    return FBM_E_ARG;
  }
  if (n_out > 0 && (!pt || !vals)) {
    set_error("null pointer argument");
    return FBM_E_ARG;
  }
  return timed("ves_unpack", (hipStream_t)stream,
               [&] { return launch_ves_unpack(pt, pw, es, cr, n_out, ow, vals, (hipStream_t)stream); });
}

int fbm_int_true_div_big(const uint64_t* x, uint64_t n, const uint32_t* k, int k_words, int negative, double* out,
                         void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (!k || k_words < 1) {
    set_error("fbm_int_true_div_big: null or empty divisor");
    return FBM_E_ARG;
  }
  int nz = 0;
  for (int i = 0; i < k_words; ++i) nz |= k[i] != 0u;
  if (!nz) {
    set_error("division by zero");
    return FBM_E_ARG;
  }
  if (n == 0) return FBM_OK;
  if (!x || !out) {
    set_error("null pointer argument");
    return FBM_E_ARG;
  }
  return timed("int_ops", s, [&] { return launch_int_true_div_big(x, n, k, k_words, negative ? 1 : 0, out, s); });
}

int fbm_jl_batch_begin(void) { return jl_batch_begin(); }

void fbm_jl_batch_abort(void) { jl_batch_abort(); }

int fbm_jl_batch_count(void) { return jl_batch_count(); }

uint64_t fbm_jl_batch_workspace(void) { return jl_batch_workspace(); }

int fbm_jl_batch_flush(void* workspace, uint64_t workspace_bytes, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  return timed("jl_exp", s, [&] { return jl_batch_flush(workspace, workspace_bytes, s); });
}

int fbm_ass_split(const void* secret, int secret_dtype, uint64_t n, int n_shares, int bit_length,
                  const uint8_t* seed, const uint8_t* nonce, uint64_t elem_offset, int64_t* shares, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (n_shares < 1 || bit_length > 64 || !seed || !nonce || (secret_dtype != FBM_U64 && secret_dtype != FBM_I64)) {
    set_error("invalid additive-sharing arguments (n_shares >= 1, bit_length <= 64, 64-bit secrets)");
    return FBM_E_ARG;
  }
  if (n == 0) return FBM_OK;
  if (!secret || !shares) {
    set_error("null pointer argument");
    return FBM_E_ARG;
  }
  uint32_t key[8], nw[2];
  memcpy(key, seed, 32);
  memcpy(nw, nonce, 8);
  return timed("ass_split", s, [&] {
    return launch_ass_split((const uint64_t*)secret, n, key, nw[0], nw[1], elem_offset, n_shares, bit_length,
                            secret_dtype == FBM_I64, shares, s);
  });
}

int fbm_ass_reconstruct(const int64_t* shares, int n_shares, uint64_t n, int64_t* out, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (n_shares < 1) {
    set_error("n_shares must be >= 1");
    return FBM_E_ARG;
  }
  if (n == 0) return FBM_OK;
  if (!shares || !out) {
    set_error("null pointer argument");
    return FBM_E_ARG;
  }
  return timed("ass_reconstruct", s, [&] { return launch_ass_reconstruct(shares, n_shares, n, out, s); });
}

int fbm_ass_split_wide(const uint32_t* secret, uint64_t n, int l_in, int n_shares, int bit_length, int l_out,
                       const uint8_t* seed, const uint8_t* nonce, uint64_t elem_offset, uint32_t* shares,
                       void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const int bmax = bit_length >= 0 ? bit_length : 32 * l_in;
  int pbits = 0;
  while ((1ll << pbits) < (long long)n_shares) ++pbits;
  if (n_shares < 1 || l_in < 1 || l_in > 4096 || l_out < l_in || !seed || !nonce ||
      32ll * l_out < (long long)bmax + pbits + 2 || bmax > (1 << 20)) {
    set_error("invalid wide additive-sharing arguments (n_shares >= 1, 1 <= l_in <= l_out, "
              "32*l_out >= bits + ceil(log2 n_shares) + 2)");
    return FBM_E_ARG;
  }
  if (n == 0) return FBM_OK;
  if (!secret || !shares) {
    set_error("null pointer argument");
    return FBM_E_ARG;
  }
  uint32_t key[8], nw[2];
  memcpy(key, seed, 32);
  memcpy(nw, nonce, 8);
  return timed("ass_split_wide", s, [&] {
    return launch_ass_split_wide(secret, n, l_in, key, nw[0], nw[1], elem_offset, n_shares, bit_length, l_out,
                                 shares, s);
  });
}

int fbm_ass_reconstruct_wide(const uint32_t* shares, int n_shares, int l, uint64_t n, uint32_t* out, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (n_shares < 1 || l < 1) {
    set_error("n_shares and l must be >= 1");
    return FBM_E_ARG;
  }
  if (n == 0) return FBM_OK;
  if (!shares || !out) {
    set_error("null pointer argument");
    return FBM_E_ARG;
  }
  return timed("ass_reconstruct_wide", s,
               [&] { return launch_ass_reconstruct_wide(shares, n_shares, l, n, out, s); });
}

}  // extern "C"

// ---------------------------------------------------------------------------------------
// The test build's entry points (include/fbm_secagg_test.h; libfbm_secagg_test.so, compiled with
// -DFBM_TEST_HOOKS from this same file and linked with the same kernel objects): host runs of device
// routines, engine / short-path switches of the calling thread, engine and multiply counts, and the
// per-kernel event timer.  The product library (libfbm_secagg.so) exports none of them.
// ---------------------------------------------------------------------------------------
#ifdef FBM_TEST_HOOKS
extern "C" {

int fbm_jl_window(void) { return FBM_WIN; }
int fbm_jl_mads(int square) {  // 0: general product, 1: square, 2: short-base product
  return square == 2 ? FBM_NA_MADS_SHORT : square ? FBM_NA_MADS_SQR : FBM_NA_MADS_MUL;
}
int fbm_jl_quad_mads(int square) {
  return 4 * (square == 2 ? FBM_QA_MADS_SHORT : square ? FBM_QA_MADS_SQR : FBM_QA_MADS_MUL);
}
int fbm_jl_triple_mads(int square) {
  return 3 * (square == 2 ? FBM_TA_MADS_SHORT : square ? FBM_TA_MADS_SQR : FBM_TA_MADS_MUL);
}

int fbm_jl_set_engine(int mode) {
  if (mode != FBM_ENGINE_AUTO && mode != FBM_ENGINE_SINGLE && mode != FBM_ENGINE_GENERIC && mode != FBM_ENGINE_QUAD &&
      mode != FBM_ENGINE_TRIPLE) {
    set_error("fbm_jl_set_engine: mode must be 0 (auto), 1 (one lane per ciphertext), 2 (generic: any modulus), "
              "3 (three lanes) or 4 (four)");
    return FBM_E_ARG;
  }
  return jl_engine_set(mode);
}

int fbm_jl_engine_for(uint64_t n_ct) { return jl_engine_for(n_ct); }

int fbm_jl_set_short(int on) {
  const int prev = t_short_on;
  t_short_on = on ? 1 : 0;
  return prev;
}

int fbm_test_short_cache(uint32_t* out, int cap_words) {
  std::lock_guard<std::mutex> lk(g_jp_mu);
  const int per = (int)(sizeof(JlShortCacheEntry) / 4);
  const int n = (int)g_short_cache.size();
  if (out) {
    if (cap_words < n * per) {
      set_error("fbm_test_short_cache: %d words needed", n * per);
      return FBM_E_ARG;
    }
    for (int i = 0; i < n; ++i) memcpy(out + i * per, &g_short_cache[i], sizeof(JlShortCacheEntry));
  }
  return n * per;
}

int fbm_test_true_div_big(const uint64_t* x, uint64_t n, const uint32_t* k, int k_words, int negative, double* out) {
  if (!k || k_words < 1 || (n > 0 && (!x || !out))) {
    set_error("fbm_test_true_div_big: bad arguments");
    return FBM_E_ARG;
  }
  host_true_div_big(x, n, k, k_words, negative, out);
  return FBM_OK;
}

int fbm_test_fdh_gcd(const uint32_t* r8, const uint32_t* n32, uint32_t* err) {
  if (!r8 || !n32 || !err || !(n32[0] & 1u)) {
    set_error("fbm_test_fdh_gcd: null pointer or even modulus");
    return FBM_E_ARG;
  }
  return host_gcd_is_one_r8(r8, n32, err);
}

int fbm_test_gen_exp(const uint32_t* h, const uint32_t* pt, int negative, const uint32_t* biprime, const uint32_t* key,
                     int key_negative, uint32_t* out, uint32_t* err) {
  if (!h || !biprime || !key || !out || !err) {
    set_error("fbm_test_gen_exp: null pointer");
    return FBM_E_ARG;
  }
  GenCtx g;
  const int rc = build_gen_ctx(biprime, key, key_negative, g);
  if (rc) return rc;
  *err = host_gen_exp(h, pt, negative, g, out);
  return FBM_OK;
}

int fbm_test_gen_combine(const uint32_t* cts, int n_parties, const uint32_t* factor, const uint32_t* biprime,
                         int mode, uint32_t* out, uint32_t* err) {
  if (!cts || n_parties < 1 || !biprime || !out || !err || (mode != FBM_GEN_PRODUCT && mode != FBM_GEN_DECRYPT)) {
    set_error("fbm_test_gen_combine: bad arguments");
    return FBM_E_ARG;
  }
  GenCtx g;
  const int rc = build_gen_ctx(biprime, nullptr, 0, g);
  if (rc) return rc;
  *err = host_gen_combine(cts, n_parties, factor, g, mode, out);
  return FBM_OK;
}

int fbm_test_nadic_consts(const uint32_t* n32, uint32_t* nk, uint32_t* r2na, uint32_t* r3na, uint32_t* np) {
  if (!n32 || !nk || !r2na || !r3na || !np) {
    set_error("fbm_test_nadic_consts: null pointer");
    return FBM_E_ARG;
  }
  JlParams jp;
  uint32_t tau1[FBM_TAU_LIMBS] = {1u};
  int rc = build_jl_params(n32, 34, 30, tau1, 0, jp);
  if (rc) return rc;
  memcpy(nk, jp.na.nk29, sizeof(jp.na.nk29));
  memcpy(r2na, jp.qa.r2, sizeof(jp.qa.r2));
  memcpy(r3na, jp.qa.r3, sizeof(jp.qa.r3));
  *np = jp.qa.np;
  return FBM_OK;
}

int fbm_test_short_consts(const uint32_t* n32, const uint32_t* key, uint32_t* kw, uint32_t* corr, uint32_t* d) {
  if (!n32 || !key || !kw || !corr || !d) {
    set_error("fbm_test_short_consts: null pointer");
    return FBM_E_ARG;
  }
  JlSched sc;
  int is_zero = 0;
  int rc = build_schedule(key, sc, is_zero);
  if (rc) return rc;
  JlShort sh;
  const bool q = build_short(n32, key, is_zero, sc, sh, true);
  memcpy(kw, sh.kw, sizeof(sh.kw));
  memcpy(corr, sh.corr, sizeof(sh.corr));
  memcpy(d, sh.d, sizeof(sh.d));
  return q ? sc.sbits : -2;
}

int fbm_test_modinv(const uint32_t* x, const uint32_t* n, uint32_t* out, int* batches) {
  if (!x || !n || !out || !(n[0] & 1u)) {
    set_error("fbm_test_modinv: null pointer or even modulus");
    return FBM_E_ARG;
  }
  FbmN30 N;
  fbm_n30_setup(n, N);
  FbmInvState st;
  fbm_modinv_init(st, x, N);
  int b = 0;
  while (!fbm_s30_is_zero(st.g) && b < FBM_INV_MAX_BATCHES) {
    fbm_modinv_batch(st, N);
    ++b;
  }
  if (batches) *batches = b;
  if (!fbm_s30_is_zero(st.g)) {
    set_error("modular inverse did not converge");
    return FBM_E_ITER;
  }
  if (!fbm_modinv_finish(st, N, out)) {
    set_error("not invertible");
    return FBM_E_INVERSE;
  }
  return FBM_OK;
}

int fbm_test_lom_aggregate_kernel(int n_parties, uint64_t n, const void* y, char* buf, int len) {
  const int rc = lom_aggregate_kernel_name(n_parties, n, y, buf, len);
  if (rc) set_error("fbm_test_lom_aggregate_kernel: bad arguments or buffer too small");
  return rc;
}

int fbm_prof_enable(int on) {
  std::lock_guard<std::mutex> g(g_prof_mu);
  g_prof_on = on != 0;
  return FBM_OK;
}

// Synchronises the recorded events and writes "name count total_ms\n" lines (sorted by
// name) into buf; clears the records.  Returns the number of bytes needed.
int fbm_prof_report(char* buf, int len) {
  // Folds completed event pairs into g_prof_agg; the aggregate is only handed out (and
  // cleared) when buf can hold all of it, so a size query (buf == NULL) loses nothing.
  std::lock_guard<std::mutex> g(g_prof_mu);
  for (auto& r : g_prof) {
    float ms = 0.f;
    const bool ok = hipEventSynchronize(r.b) == hipSuccess && hipEventElapsedTime(&ms, r.a, r.b) == hipSuccess;
    if (ok) {
      auto& e = g_prof_agg[r.name];
      e.first += 1;
      e.second += ms;
    }
    (void)hipEventDestroy(r.a);
    (void)hipEventDestroy(r.b);
  }
  g_prof.clear();
  std::string out;
  for (auto& kv : g_prof_agg) {
    char line[160];
    snprintf(line, sizeof(line), "%s %ld %.6f\n", kv.first.c_str(), kv.second.first, kv.second.second);
    out += line;
  }
  const int need = (int)out.size() + 1;
  if (buf && len >= need) {
    memcpy(buf, out.c_str(), (size_t)need);
    g_prof_agg.clear();
  }
  return need;
}

}  // extern "C"
#endif  // FBM_TEST_HOOKS
