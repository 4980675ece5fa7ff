// fedbiomed_amd -- internal declarations shared by the kernel files and the C-ABI.
#pragma once
#include "fbm_common.hpp"
#include "fbm_mont.hpp"
#include "fbm_safegcd.hpp"
#include "../../include/fbm_secagg.h"

#define FBM_MAX_PEERS 64

// stats words written by kernels (device u32[4], zeroed by the C-ABI before a launch)
#define FBM_STAT_MAXBITS 0   // max bit length of q*w (LOM overflow guard, _lom.py:133-150)
#define FBM_STAT_ERRFLAGS 1  // OR of FBM_ERR_* flags
#define FBM_STAT_COUNT 4

#define FBM_ERR_DEQUANT_RANGE 1u   // averaged value > 2^64-1 (reverse_quantize FB624)
#define FBM_ERR_FDH_OVERFLOW 2u    // no coprime r of 1..7 FDH digests (reference: OverflowError)
#define FBM_ERR_NOT_INVERTIBLE 4u  // server-key power not invertible mod N^2
#define FBM_ERR_ITER_CAP 8u        // a bounded data-dependent loop hit its cap
#define FBM_ERR_ROUND_RANGE 128u   // LOM: some i + tau reaches 2^64 with peers to mask with
#define FBM_ERR_PT_WIDE 32u        // VES: a packed value spills past the 1024-bit plaintext
#define FBM_ERR_FDH_WIDE 64u       // FDH of bits_size > 4096: no coprime r of 1..15 digests, and the
                                   // reference would go on to 16 or more (outside the device path's domain)
#define FBM_WARN_CLIPPED 16u       // not an error: some |x| > clipping range (the reference's
                                   // _check_clipping_range warning, _secagg_utils.py:189-204)

namespace fbm {

// wave-level OR of a per-lane warning/error condition into the stats flags (one atomic per wave)
__device__ __forceinline__ void flag_if_any(bool cond, uint32_t* stats, uint32_t bit) {
  if (__ballot(cond) && (threadIdx.x & 63) == 0) atomicOr(stats + FBM_STAT_ERRFLAGS, bit);
}

struct LomPeers {
  int n_peers;
  int raw_seeds;                 // 1: secret[] already are the per-round seeds (PRF.eval_vector)
  uint64_t ctr0;                 // nonce bytes 0-7 (LE) = 64-bit ChaCha20 block counter
  uint32_t n14, n15;             // nonce bytes 8-15 (LE words)
  uint64_t tau;                  // round
  uint64_t elem_offset;          // global index of x[0] (element-range shard; multiple of 8)
  uint32_t tau_be[4];            // tau.to_bytes(16, 'big') as LE words
  uint32_t secret[FBM_MAX_PEERS][8];
  uint64_t add_bits;             // bit p set: mask += vec (peer < node), clear: mask -= vec
  uint32_t round_range;          // 1: flag FBM_ERR_ROUND_RANGE (first peer group only)
};

int check_launch(const char* what);
void set_error(const char* fmt, ...);

int launch_lom_protect(const void* x, int x_dtype, uint64_t n, const QuantParams& qp, uint64_t weight,
                       const LomPeers& peers, uint64_t* y, uint32_t* stats, hipStream_t s);
int launch_lom_mask_accumulate(uint64_t n, const LomPeers& peers, uint64_t* y, hipStream_t s);
int launch_dequantize(const uint64_t* u, uint64_t n, double neg_c, double step, double* out, hipStream_t s);
int launch_prf_key(const LomPeers& peers, uint32_t* seed_out, hipStream_t s);
// the aggregate kernel's name (test build: fbm_test_lom_aggregate_kernel)
int lom_aggregate_kernel_name(int n_parties, uint64_t n, const void* y, char* buf, int len);
int launch_lom_aggregate(const uint64_t* y, int n_parties, uint64_t n, uint64_t total_weight, double neg_c,
                         double step, double* out, uint64_t* sums, uint32_t* stats, hipStream_t s);

// ---- Joye-Libert -------------------------------------------------------------------
// exponent schedule (host-computed sliding window, uniform across lanes)
#ifndef FBM_WIN
#define FBM_WIN 6  // A/B on MI355X: +1.7 % over 5 (325 vs 354 general products per ciphertext)
#endif
#define FBM_TABLE (1 << (FBM_WIN - 1))  // odd powers h^1, h^3, ..., h^(2^FBM_WIN - 1)
#define FBM_OP_SHIFT 6                  // op = nsq << 6 | (table index + 1); windows up to 6 bits
#define FBM_OP_MAXSQ 1023
#define FBM_MAX_OPS 512
#define FBM_TENTRIES (FBM_TABLE + 1)    // + one scratch column (h, then h^2)
#define FBM_TSCRATCH FBM_TABLE
// the per-call ops buffer: the sliding-window ops, then the short path's exponent words (|key|,
// 64 words) and its correction constant C (N-adic digits, 72 29-bit limbs; JlSched::corr)
#define FBM_OPS_KW FBM_MAX_OPS
#define FBM_OPS_CORR (FBM_MAX_OPS + 64)
// C's broadcast column: limb k at word FBM_OPS_CBC + 256 k (the one-lane engine reads it as a B operand
// with a zero lane offset: every lane the same address)
#define FBM_OPS_CBC (((FBM_MAX_OPS + 64 + 128) + 255) / 256 * 256)
#define FBM_OPS_WORDS (FBM_OPS_CBC + 72 * 256)

// per-call device constants (words): M, R^2 (74 limbs, padded to 128), the broadcast
// column 1 (limb k at word k*256) and R^(P+1) mod M (the aggregate's uniform first operand,
// written by jl_rk_kernel: P parties + the factor leave the product at the plain value)
// jl_nude_kernel's rows per 256-ciphertext block: digit 1 of (1, pt) only (fbm_na_mm_nude)
#ifdef FBM_NUDE_BOTH_DIGITS  // A/B variant: both digits stored (72 rows), as before round 4
#define FBM_NUDE_ROWS 72
#define FBM_NUDE_D1 36       // digit 1's first row
#else
#define FBM_NUDE_ROWS 36
#define FBM_NUDE_D1 0
#endif
#define FBM_CST_M 0
#define FBM_CST_CTR 120  // exp-kernel chunk counter (in M's padding; zeroed by jl_setup_kernel)
#define FBM_CST_R2 128
#define FBM_CST_ONE 256
#define FBM_CST_RK (256 + FBM_NL * 256)
// N's 28-bit limbs at words 0..9, 16..42 (the final step of every N-adic engine,
// na_final_digits), then the one-lane engine's (fbm_nadic_asm.hpp) 80-word constants block:
// N's 29-bit limbs and K'_i in the layout the assembly's scalar loads expect
#define FBM_CST_NK (FBM_CST_RK + 128)
#define FBM_CST_NA29 (FBM_CST_NK + 128)
// lane-group engines (fbm_quad_asm.hpp / fbm_tri_asm.hpp) and the one-lane engine, all 29-bit
// limbs with R = 2^1044: K'_i (36 words), N's limbs (limb k at word k), R^2 and R^3 mod N^2 as
// digit pairs (72 limbs each; the uniform A operand that brings h, or a wide h's high part,
// into Montgomery form)
#define FBM_CST_QK (FBM_CST_NA29 + 128)
#define FBM_CST_QNP (FBM_CST_QK + 64)
#define FBM_CST_QR2 (FBM_CST_QNP + 64)
#define FBM_CST_QR3 (FBM_CST_QR2 + 128)
// the MontCtxN image (M, R^2 mod N, mp: 76 words) for the mod-N products of jl_emodn /
// jl_lift, read through device memory (a laundered pointer into the by-value JlParams
// kernel argument would make the compiler copy all 3.3 KB of it to scratch per lane)
#define FBM_CST_MN (FBM_CST_QR3 + 128)
// the short-base product's pairs (D_j, 0), D = N - 2^(29 * 9) (72 words; JlShort::d)
#define FBM_CST_QD (FBM_CST_MN + 128)
// the one-lane square's initial s window (round 4, K' folded): pairs (2^29 - 1 + P'_j, 0),
// P' = (K - E) mod N (QuadCtx::sqp; FBM_NA_SQ_ONE_MASK in fbm_nadic_asm.hpp)
#define FBM_CST_QP (FBM_CST_QD + 128)
#define FBM_CST_WORDS (FBM_CST_QP + 128)

// sliding-window schedule, passed by value (kernarg segment -> scalar loads).
// op k (u16): (squarings before the multiply) << FBM_OP_SHIFT | (table index + 1, 0 = none)
// sbits: the SHORT path (below) takes bit length of |key| - 1 squarings; -1 = no short path.
struct JlSched {
  int n_ops;
  int first;       // table index of the leading window
  uint16_t op[FBM_MAX_OPS];
  int sbits;
};
// The SHORT path (one FDH digest h < 2^261, N > 2^262): left-to-right binary over |key| with the
// short-base product (fbm_na_ms_glb) -- kw = |key|'s words, corr = C = 2^(1044 (2^sbits + 1) +
// 261 (|key| - 2^sbits)) mod N^2 as N-adic digits (the constant whose product turns the chain's
// h^|key| 2^-f into h^|key| R), d = N - 2^261 (the short product's s-window start).  Written by
// jl_short_setup_kernel into the ops buffer (kw, corr) and the constants block (d).
struct JlShort {
  uint32_t kw[64];
  uint32_t corr[72];
  uint32_t d[36];
};

// N-adic constants.  nk: N's 28-bit limbs, words 0..9 = N_0..N_9, 16..42 = N_10..N_36 (the
// shared final step).  nk29 (tools/gen_nadic_asm.py, 29-bit limbs, R = 2^1044): words
// 0..9 = N_0..N_9, 16..41 = N_10..N_35, 42..77 = K'_i = (2^29 - 1) + K_i with K = (1 - R) mod N.
// R^2 / R^3 mod N^2 as 29-bit digit pairs: QuadCtx::r2 / r3 (the same R).
struct NadicCtx {
  uint32_t nk[80];
  uint32_t nk29[80];
};

// lane-group engine constants (tools/gen_quad_asm.py): 29-bit limbs, R = 2^1044
struct QuadCtx {
  uint32_t kp[36];   // K'_i = 2^29 - 1 + K_i, K = (1 - R) mod N
  uint32_t n[36];    // N
  uint32_t r2[72];   // R^2 mod N^2 = u0 + u1 N: u0 limbs, then u1 limbs
  uint32_t r3[72];   // R^3 mod N^2 likewise
  uint32_t np;       // -N^-1 mod 2^29
  uint32_t pad[3];
  uint32_t sqp[36];  // 2^29 - 1 + P'_j: the one-lane square's initial s window (FBM_CST_QP)
};

struct JlParams {
  MontCtx mc;                    // modulus M = N^2 (74 limbs)
  MontCtxN mn;                   // modulus N (37 limbs) -- inverse mod N, N*pt, N-adic np
  NadicCtx na;                   // N-adic engine constants (jl_exp_kernel)
  uint32_t N32[32];              // N, 32-bit limbs (<= 1024 bits)
  uint32_t Ninv32[32];           // N^-1 mod 2^1024 (exact divisions by N: jl_prod, jl_lift, jl_split)
  int n_bits;                    // bit length of N
  int es, cr;                    // VES slot size / slots per ciphertext
  uint32_t tau_w[16];            // the round's bits 0..511 as FDH's message block 15 (t's low 512 bits,
                                 // big-endian words: tau_w[15] = tau mod 2^32)
  uint32_t tau14_w[16];          // its bits 512..1023: block 14, into which the kernel ORs k (t = (k << 512) | tau)
  uint64_t ct_offset;            // global index of ciphertext 0 (element-range shard)
  uint32_t mid[8];               // SHA-256 state after message blocks 0..13 (the round's bits 1024..8191)
  FbmN30 n30;                    // N in signed-30 limbs + N^-1 mod 2^30 (modular inverse)
  int key_is_zero;
  int fdh_even;                  // FDH.H standalone: the modulus is even (r must be odd as well)
  uint32_t mneg[FBM_NLN];        // N * 2^(1036 - bits(N)) in 28-bit limbs (negative-weight packing)
  uint32_t pad2[3];
  QuadCtx qa;                    // quad exponentiation engine constants
};

int launch_jl_pack(const void* x, int x_dtype, uint64_t n, const QuantParams& qp, uint64_t weight, int es, int cr,
                   uint64_t n_ct, uint32_t* pt, uint32_t* stats, hipStream_t s);
// v / k (Python's int / int true division) for an integer |k| >= 2^64 given as k_words host limbs
int launch_int_true_div_big(const uint64_t* x, uint64_t n, const uint32_t* k, int k_words, int negative, double* out,
                            hipStream_t s);
void host_true_div_big(const uint64_t* x, uint64_t n, const uint32_t* k, int k_words, int negative, double* out);
int launch_int_ops(const uint64_t* x, uint64_t n, uint64_t k, int op, uint64_t* prod, double* quot, uint32_t* stats,
                   hipStream_t s);
int launch_jl_nude(const uint32_t* pt, uint64_t n_ct, const JlParams& jp, int negative, uint32_t* nude,
                   hipStream_t s);
// Hc != nullptr: the compact form the Montgomery engines read -- Hc[k] = r's 8 words when r is one digest
// (any real biprime), else the sentinel FBM_HC_FULL (8 words of ones) and the whole row in H[k]; Hc ==
// nullptr: every row whole in H (the generic engine, fbm_jl_fdh)
int launch_jl_fdh(uint64_t n_ct, const JlParams& jp, uint32_t* H, uint32_t* stats, hipStream_t s, uint32_t* Hc = nullptr);
// VES of any shape (fbm_ves_pack / fbm_ves_unpack)
int launch_ves_pack(const uint32_t* x, uint64_t n, int wv, int es, int cr, int pw, int sgn, uint32_t* pt,
                    hipStream_t s);
int launch_ves_unpack(const uint32_t* pt, int pw, int es, int cr, uint64_t n_out, int ow, uint32_t* vals, hipStream_t s);
// FDH.H of any bits_size: one lane per t (tw-word rows), message t.to_bytes(msg_bytes) || counter, r of at
// most kmax digests (fbm_jl_fdh_msg; r of up to FBM_FDH_MSG_DIGESTS digests, FBM_FDH_MSG_ROW-word rows)
#define FBM_FDH_MSG_DIGESTS 15
#define FBM_FDH_MSG_WORDS (8 * FBM_FDH_MSG_DIGESTS)
#define FBM_FDH_MSG_ROW 128
int launch_jl_fdh_msg_wide(uint64_t n, const uint32_t* t, int tw, int msg_bytes, int kmax, const uint32_t* m32,
                           const uint32_t* k1, const uint32_t* k2, uint32_t mp, int even, uint32_t* H, int hw,
                           uint32_t* stats, hipStream_t s);
int launch_jl_fdh_msg(uint64_t n, const uint32_t* t, int tw, int msg_bytes, int kmax, const uint32_t* n32, int even,
                      uint32_t* H, uint32_t* stats, hipStream_t s);
int launch_jl_setup(const JlParams& jp, const JlSched& sc, uint32_t* ops, uint32_t* cst, hipStream_t s,
                    const JlShort* sh = nullptr);
// one exponentiation launch over several calls' ciphertexts (jl_exp_kernel<true> segments)
#define FBM_EXP_MAXSEG 24
struct JlExpSeg {
  const uint32_t* H;
  const uint32_t* Hc;  // compact H rows (jl_fdh_kernel's 8 words per ciphertext; FBM_HC_FULL: read H), or nullptr
  const uint32_t* nude;
  uint32_t* out;
  const uint32_t* ops;
  uint64_t n_ct;
  uint32_t chunk0;  // first chunk of this segment in the launch's chunk sequence
  int n_ops, first, mode, key_is_zero;
  int sbits;        // JlSched::sbits (the short path's exponent bits - 1, or -1)
};
struct JlExpBatch {
  int nseg;
  uint32_t total_chunks;
  JlExpSeg seg[FBM_EXP_MAXSEG];
};
// batch mode (per thread): while a batch is open, the exponentiation of a phase-2-only call
// (jl_batch_accept(true) around it) is recorded instead of launched; flush launches them all
int jl_batch_begin();
void jl_batch_abort();
bool jl_batch_accept(bool on);
bool jl_batch_active();
int jl_batch_count();  // segments recorded in this thread's open batch (0 when none is open)
uint64_t jl_batch_workspace();
int jl_batch_flush(void* workspace, uint64_t ws_bytes, hipStream_t s);
// Hc: launch_jl_fdh's compact rows of the same ciphertexts (nullptr: H holds every row whole)
int launch_jl_exp(const uint32_t* H, uint64_t n_ct, const JlParams& jp, const JlSched& sc, int mode,
                  const uint32_t* nude, uint32_t* table, uint64_t table_slots, const uint32_t* ops,
                  const uint32_t* cst, uint32_t* out, hipStream_t s, const uint32_t* Hc = nullptr);
struct JlRk {  // R^(P+1) mod N^2, 28-bit limbs (jl_rk_kernel -> cst[FBM_CST_RK])
  uint32_t w[FBM_NL];
  uint32_t pad[2];
};
int launch_jl_rk(const JlRk& rk, uint32_t* cst, hipStream_t s);
// x_k = (prod_u c_u * F_k mod N^2 - 1) div N   (cst[FBM_CST_RK] = R^(P+1) mod N^2)
int launch_jl_encf(const uint32_t* pt, uint64_t n_ct, const JlParams& jp, const uint32_t* cst, int negative,
                   const uint32_t* factor, uint32_t* out, hipStream_t s);
int launch_jl_prod(const uint32_t* cts, int n_parties, uint64_t n_ct, const JlParams& jp, const uint32_t* cst,
                   const uint32_t* factor, uint32_t* xout, hipStream_t s);
#define FBM_EXP_DEC 1        // jl_exp mode bits: plain power (no nude product)
#define FBM_EXP_OUT_NADIC 4  // out rows are the result's N-adic digits (v mod N, v div N)
int host_gcd_is_one_r8(const uint32_t* r8, const uint32_t* n32, uint32_t* err);
// E^-1 mod N^2 (times nude when given: a negative-key encrypt) from E's N-adic digit rows
// Ed [ct][64] (e0 | e1): y = e0^-1 mod N into Y [ct][32], then the lift -> out [ct][64]
int launch_jl_inv(uint64_t n_ct, const JlParams& jp, const uint32_t* cst, const uint32_t* Ed, uint32_t* Y,
                  const uint32_t* nude, uint32_t* out, uint32_t* stats, hipStream_t s);
int launch_jl_decode(const uint32_t* xs, int es, int cr, uint64_t n_out, uint64_t total_weight, double neg_c,
                     double step, double* out, uint64_t* sums, uint32_t* stats, hipStream_t s);

// ---- the generic JL engine (fbm_gen.hip): any biprime N, even ones included ------------
// Constants of one (N, key), host-built (fbm_capi.hip build_gen_ctx), copied into the call's
// constants block by jl_gen_setup_kernel.  32-bit limbs, little-endian; M = N^2 = 2^e m2 with
// m2 odd; muX = floor(2^(64 kX) / X) (Barrett: kX + 1 words, or kX + 2 when X = 2^(32(kX-1)),
// zero-padded); m2inv = m2^-1 mod 2^e.
struct GenCtx {
  int kM, kN, km2, e;  // words of M, N, m2; e = 2 * (trailing zero bits of N)
  int key_bits, key_negative, pad0, pad1;
  uint32_t M[64];
  uint32_t muM[68];
  uint32_t N[32];
  uint32_t muN[36];
  uint32_t m2[64];
  uint32_t m2inv[64];
  uint32_t key[64];  // |key|
};
#define FBM_GEN_ENC 1       // jl_gen_exp: times (N pt + 1) mod N^2 (an encrypt)
#define FBM_GEN_PRODUCT 0   // jl_gen_combine: out = prod mod N^2 [ct][64]
#define FBM_GEN_DECRYPT 1   // jl_gen_combine: out = ((v - 1) // N) mod N [ct][32]
int launch_jl_gen_setup(const GenCtx& g, uint32_t* cst, hipStream_t s);
// out = H^key mod N^2 (the inverse of H^|key| for a negative key), times (N pt + 1) mod N^2
// when pt != NULL (pt [ct][32]: |pt| and the sign `negative` of a negative-weight packing)
int launch_jl_gen_exp(const uint32_t* H, const uint32_t* pt, int negative, uint64_t n_ct, const uint32_t* cst,
                      uint32_t* out, uint32_t* stats, hipStream_t s);
// v = prod_u cts[u] (* factor) mod N^2 -> out (FBM_GEN_PRODUCT) or ((v - 1) // N) mod N (FBM_GEN_DECRYPT)
int launch_jl_gen_combine(const uint32_t* cts, int n_parties, uint64_t n_ct, const uint32_t* factor,
                          const uint32_t* cst, int mode, uint32_t* out, uint32_t* stats, hipStream_t s);
// the same per-ciphertext work on the host, one ciphertext (test hooks; cts: n_parties rows of 64)
uint32_t host_gen_exp(const uint32_t* Hrow, const uint32_t* ptrow, int negative, const GenCtx& g, uint32_t* out);
uint32_t host_gen_combine(const uint32_t* cts, int n_parties, const uint32_t* frow, const GenCtx& g, int mode,
                          uint32_t* out);

int launch_ass_split(const uint64_t* secret, uint64_t n, const uint32_t* key, uint32_t n14, uint32_t n15,
                     uint64_t elem_offset, int n_shares, int bit_length, int is_signed, int64_t* shares,
                     hipStream_t s);
int launch_ass_reconstruct(const int64_t* shares, int n_shares, uint64_t n, int64_t* out, hipStream_t s);
int launch_ass_split_wide(const uint32_t* secret, uint64_t n, int l_in, const uint32_t* key, uint32_t n14,
                          uint32_t n15, uint64_t elem_offset, int n_shares, int bit_length, int l_out,
                          uint32_t* shares, hipStream_t s);
int launch_ass_reconstruct_wide(const uint32_t* shares, int n_shares, int l, uint64_t n, uint32_t* out,
                                hipStream_t s);

// table slots the encrypt/aggregate kernels need for a given grid
uint64_t jl_table_slots();
// exponentiation engine policy (fbm_jl_set_engine) and the table bytes both engines fit in
#define FBM_ENGINE_AUTO 0
#define FBM_ENGINE_SINGLE 1
#define FBM_ENGINE_GENERIC 2  // every modulus on the generic engine (fbm_gen.hip; odd N: a cross-check)
#define FBM_ENGINE_TRIPLE 3
#define FBM_ENGINE_QUAD 4
int jl_engine_policy();
int jl_engine_set(int mode);
int jl_engine_for(uint64_t n_ct);
uint64_t jl_table_bytes(uint64_t n_ct);
// compute units of the calling thread's current device (cached per device)
int device_num_cu();

}  // namespace fbm
