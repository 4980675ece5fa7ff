// fedbiomed_amd -- shared host/device primitives for the secure-aggregation hot path.
//
// Everything here is bit-exact restatement of what the reference computes in Python /
// OpenSSL / hashlib, written for gfx950 (and usable on the host for tiny setup work):
//   * fixed-point quantise          fedbiomed/common/utils/_secagg_utils.py:82-119
//   * dequantise                    fedbiomed/common/utils/_secagg_utils.py:152-187
//   * Python int/int true division  fedbiomed/common/secagg/_secagg_crypter.py:233-249
//   * ChaCha20 block (OpenSSL 64-bit counter)   fedbiomed/common/secagg/_lom.py:30-83
//   * SHA-256 compression           fedbiomed/common/secagg/_jls.py:747 (hashlib)
//
// Compiled with -ffp-contract=off: the FP64 sequences below must not be fused.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define FBM_HD __host__ __device__ __forceinline__

#pragma clang fp contract(off)

// ------------------------------------------------------------------------------------
// quantise / dequantise
// ------------------------------------------------------------------------------------
// q = uint64(min(T-1, (median(-c,x,c)+c)*T/(2c))).  Inside [-c,c] the reference's median
// is the float x and the arithmetic is RN(RN(RN(x+c)*RN(T))/RN(2c)); for x > c the median
// is the *int* c so the quotient is the exact int division T, rounded once (= RN(T));
// for x < -c it is 0.  NaN fails every comparison -> falls to the float path -> NaN ->
// min(T-1, NaN) returns T-1.  `min` compares int T-1 with the float exactly:
// qf >= T-1  <=>  floor(qf) >= T-1 (T-1 integral), and qf >= 2^64 > T-1 always.
struct QuantParams {
  double c;       // float(c)
  double two_c;   // float(2*c)
  double tf;      // float(T)      (RN of the Python int)
  uint64_t tm1;   // T - 1
};

FBM_HD uint64_t fbm_quantize(double x, const QuantParams& p) {
  double qf;
  if (x > p.c) {
    qf = p.tf;
  } else if (x < -p.c) {
    qf = 0.0;
  } else {
    double s = x + p.c;
    double m = s * p.tf;
    qf = m / p.two_c;
  }
  if (!(qf < 18446744073709551616.0)) return p.tm1;  // NaN or >= 2^64
  uint64_t qt = (uint64_t)qf;                        // truncation, qf in [0, 2^64)
  return qt < p.tm1 ? qt : p.tm1;
}

// _check_clipping_range (utils/_secagg_utils.py:189-204): x < -c or x > c (NaN: no)
FBM_HD bool fbm_outside_clip(double x, const QuantParams& p) { return x < -p.c || x > p.c; }

// Number of significant bits of the 128-bit value hi:lo (Python int.bit_length()).
FBM_HD uint32_t fbm_bitlen128(uint64_t hi, uint64_t lo) {
  if (hi) return 128u - (uint32_t)__builtin_clzll(hi);
  if (lo) return 64u - (uint32_t)__builtin_clzll(lo);
  return 0u;
}

// Python `a / b` for non-negative ints a (< 2^100) and b (1 <= b < 2^64): the correctly
// rounded (round-half-even) double of the exact quotient -- CPython's long_true_divide.
// Fast path when both operands are exact doubles (IEEE division is correctly rounded).
FBM_HD double fbm_true_div_u128(unsigned __int128 a, uint64_t b) {
  if (a == 0) return 0.0;
  if ((a >> 53) == 0 && (b >> 53) == 0) return (double)(uint64_t)a / (double)b;
  // bit lengths
  uint64_t ahi = (uint64_t)(a >> 64), alo = (uint64_t)a;
  int la = (int)fbm_bitlen128(ahi, alo);
  int lb = 64 - __builtin_clzll(b);
  // choose k so that q = floor(a*2^k / b) has 55 or 56 bits
  int k = 55 - (la - lb);
  unsigned __int128 A = a, B = b;
  if (k >= 0) A <<= k; else B <<= (-k);
  unsigned __int128 q = A / B;
  unsigned __int128 r = A - q * B;
  uint64_t q64 = (uint64_t)q;  // < 2^57
  int lq = 64 - __builtin_clzll(q64);
  int extra = lq - 53;         // 2 or 3
  uint64_t low = q64 & ((1ull << extra) - 1ull);
  uint64_t half = 1ull << (extra - 1);
  uint64_t m = q64 >> extra;
  bool sticky = (r != 0);
  if (low > half || (low == half && (sticky || (m & 1ull)))) m += 1ull;
  // value = m * 2^(extra - k)
  int e = extra - k;
  double d = (double)m;  // exact: m <= 2^53
#ifdef __HIP_DEVICE_COMPILE__
  return ldexp(d, e);
#else
  return __builtin_ldexp(d, e);
#endif
}

// reverse_quantize of one averaged value v (a float >= 0, < 2^64):
//   -c + step * double(uint64(trunc(v)))   (numpy: uint64 -> float64 RN, no FMA)
FBM_HD double fbm_dequantize(double v, double neg_c, double step) {
  uint64_t u = (uint64_t)v;
  double du = (double)u;
  double prod = step * du;
  return neg_c + prod;
}

// ------------------------------------------------------------------------------------
// ChaCha20 block (RFC 7539 rounds; OpenSSL's 16-byte IV = 64-bit LE counter || 8 B nonce)
// ------------------------------------------------------------------------------------
FBM_HD uint32_t fbm_rotl(uint32_t v, int n) { return (v << n) | (v >> (32 - n)); }

#define FBM_QR(a, b, c, d)                 \
  a += b; d ^= a; d = fbm_rotl(d, 16);     \
  c += d; b ^= c; b = fbm_rotl(b, 12);     \
  a += b; d ^= a; d = fbm_rotl(d, 8);      \
  c += d; b ^= c; b = fbm_rotl(b, 7);

#ifdef __HIP_DEVICE_COMPILE__
// Device rounds: the four quarter-rounds of a half-round issued side by side, as groups of
// four independent same-type instructions (add x4, xor x4, rotate x4, ...), with an s_nop
// after every add / xor group.  Measured on MI355X (tools/microbench/intrate.hip, identical
// keystreams): the compiler's own schedule of the QR chains runs at 4.08 cycles per
// ChaCha20 op; the groups alone at 4.07; groups separated by s_nop 0 at 3.53; an s_nop
// after the add/xor groups only at 3.46 (15 % faster).  gfx950 issues back-to-back
// independent VOP2 adds/xors at ~2.4 cycles per wave instruction (VOP3 v_alignbit_b32 at
// ~4.2), and the wait state lets the dependent group that follows issue without stalling
// the wave.  One asm statement per double round (the compiler cannot see hazards inside
// inline asm and would put its own s_nop between statements).  Operand k = state word x_k;
// v_alignbit_b32 d, d, d, n = rotr(d, n) = rotl(d, 32 - n).
#define FBM_CHACHA_DROUND_ASM \
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
#define FBM_CHACHA_DROUND(x)                                                                   \
  asm volatile(FBM_CHACHA_DROUND_ASM                                                            \
               : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), \
                 "+v"(x[7]), "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]),          \
                 "+v"(x[13]), "+v"(x[14]), "+v"(x[15]))
#endif

// key: 8 LE words; ctr: 64-bit block counter (words 12-13); n14,n15: IV words 2-3.
FBM_HD void fbm_chacha20_block(const uint32_t key[8], uint64_t ctr, uint32_t n14, uint32_t n15,
                               uint32_t out[16]) {
  const uint32_t s0 = 0x61707865u, s1 = 0x3320646eu, s2 = 0x79622d32u, s3 = 0x6b206574u;
#ifdef __HIP_DEVICE_COMPILE__
  uint32_t x[16] = {s0,     s1,     s2,     s3,     key[0],          key[1],                    key[2], key[3],
                    key[4], key[5], key[6], key[7], (uint32_t)ctr, (uint32_t)(ctr >> 32), n14,    n15};
#pragma unroll
  for (int r = 0; r < 10; ++r) FBM_CHACHA_DROUND(x);
  uint32_t x0 = x[0], x1 = x[1], x2 = x[2], x3 = x[3], x4 = x[4], x5 = x[5], x6 = x[6], x7 = x[7];
  uint32_t x8 = x[8], x9 = x[9], x10 = x[10], x11 = x[11], x12 = x[12], x13 = x[13], x14 = x[14], x15 = x[15];
#else
  uint32_t x0 = s0, x1 = s1, x2 = s2, x3 = s3;
  uint32_t x4 = key[0], x5 = key[1], x6 = key[2], x7 = key[3];
  uint32_t x8 = key[4], x9 = key[5], x10 = key[6], x11 = key[7];
  uint32_t x12 = (uint32_t)ctr, x13 = (uint32_t)(ctr >> 32), x14 = n14, x15 = n15;
  for (int r = 0; r < 10; ++r) {
    FBM_QR(x0, x4, x8, x12) FBM_QR(x1, x5, x9, x13) FBM_QR(x2, x6, x10, x14) FBM_QR(x3, x7, x11, x15)
    FBM_QR(x0, x5, x10, x15) FBM_QR(x1, x6, x11, x12) FBM_QR(x2, x7, x8, x13) FBM_QR(x3, x4, x9, x14)
  }
#endif
  out[0] = x0 + s0; out[1] = x1 + s1; out[2] = x2 + s2; out[3] = x3 + s3;
  out[4] = x4 + key[0]; out[5] = x5 + key[1]; out[6] = x6 + key[2]; out[7] = x7 + key[3];
  out[8] = x8 + key[4]; out[9] = x9 + key[5]; out[10] = x10 + key[6]; out[11] = x11 + key[7];
  out[12] = x12 + (uint32_t)ctr; out[13] = x13 + (uint32_t)(ctr >> 32); out[14] = x14 + n14; out[15] = x15 + n15;
}

FBM_HD uint64_t fbm_bswap64(uint64_t v) { return __builtin_bswap64(v); }

// ------------------------------------------------------------------------------------
// SHA-256 compression (FIPS 180-4); W holds the 16 big-endian message words of a block.
// ------------------------------------------------------------------------------------
FBM_HD uint32_t fbm_rotr(uint32_t v, int n) { return (v >> n) | (v << (32 - n)); }

#ifdef __HIP_DEVICE_COMPILE__
__constant__ static const uint32_t FBM_SHA_K[64] = {
#else
static const uint32_t FBM_SHA_K[64] = {
#endif
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};

FBM_HD void fbm_sha256_compress(uint32_t st[8], const uint32_t W0[16]) {
  uint32_t w[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) w[i] = W0[i];
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
  for (int i = 0; i < 64; ++i) {
    uint32_t wi;
    if (i < 16) {
      wi = w[i];
    } else {
      uint32_t w15 = w[(i - 15) & 15], w2 = w[(i - 2) & 15];
      uint32_t s0 = fbm_rotr(w15, 7) ^ fbm_rotr(w15, 18) ^ (w15 >> 3);
      uint32_t s1 = fbm_rotr(w2, 17) ^ fbm_rotr(w2, 19) ^ (w2 >> 10);
      wi = w[i & 15] + s0 + w[(i - 7) & 15] + s1;
      w[i & 15] = wi;
    }
    uint32_t S1 = fbm_rotr(e, 6) ^ fbm_rotr(e, 11) ^ fbm_rotr(e, 25);
    uint32_t ch = (e & f) ^ (~e & g);
    uint32_t t1 = h + S1 + ch + FBM_SHA_K[i] + wi;
    uint32_t S0 = fbm_rotr(a, 2) ^ fbm_rotr(a, 13) ^ fbm_rotr(a, 22);
    uint32_t maj = (a & b) ^ (a & c) ^ (b & c);
    uint32_t t2 = S0 + maj;
    h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

FBM_HD void fbm_sha256_init(uint32_t st[8]) {
  st[0] = 0x6a09e667u; st[1] = 0xbb67ae85u; st[2] = 0x3c6ef372u; st[3] = 0xa54ff53au;
  st[4] = 0x510e527fu; st[5] = 0x9b05688cu; st[6] = 0x1f83d9abu; st[7] = 0x5be0cd19u;
}
