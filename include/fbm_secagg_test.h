/*
 * fbm_secagg_test.h -- the TEST build's extra entry points (libfbm_secagg_test.so).
 *
 * The test suite and bench.py load libfbm_secagg_test.so for these; it is compiled from the same
 * sources as libfbm_secagg.so (fedbiomed_amd/csrc/fbm_capi.hip with -DFBM_TEST_HOOKS, linked with the
 * same kernel objects), exports every function of fbm_secagg.h too, and adds:
 *   - host runs of device routines (fbm_test_*: no GPU needed),
 *   - the JL exponentiation engine and short-path switches of the CALLING THREAD (fbm_jl_set_engine,
 *     fbm_jl_set_short) and the engine a launch would take (fbm_jl_engine_for),
 *   - the engine's multiply counts (fbm_jl_mads, ...: the bench's VALU roofline),
 *   - the per-kernel HIP event timer (fbm_prof_*: the bench's live kernel durations).
 * No reference counterpart: the reference crypter has no such hooks.  The product library
 * (libfbm_secagg.so) exports none of these (tests/test_native_abi.py).
 */
#ifndef FBM_SECAGG_TEST_H
#define FBM_SECAGG_TEST_H

#include "fbm_secagg.h"

#ifdef __cplusplus
extern "C" {
#endif

/* host test hook (no GPU): fbm_int_true_div_big's per-value arithmetic on host arrays. */
int fbm_test_true_div_big(const uint64_t* x, uint64_t n, const uint32_t* k, int k_words, int negative, double* out);

/* Sliding-window width of the JL exponentiation's table path (odd-power table of 2^(w-1) entries;
 * the short path -- one FDH digest, N > 2^262: every 1024-bit biprime -- needs no table). */
int fbm_jl_window(void);
/* v_mad_u64_u32 per lane of one product of the JL exponentiation engine (N-adic Montgomery
 * product modulo N^2, fedbiomed_amd/csrc/fbm_nadic_asm.hpp): square = 0 a general product, 1 a
 * squaring, 2 the short path's short-base product (x h 2^-261); lets the bench count the
 * multiplies one ciphertext costs (its VALU roofline). */
int fbm_jl_mads(int square);
/* The same count for the quad / triple engines (4 / 3 lanes per ciphertext): v_mad_u64_u32
 * lane-ops per product summed over the lanes (fedbiomed_amd/csrc/fbm_quad_asm.hpp, fbm_tri_asm.hpp);
 * square = 2: the short-base product. */
int fbm_jl_quad_mads(int square);
int fbm_jl_triple_mads(int square);

/* Exponentiation engine policy of the CALLING THREAD for the JL entry points (encrypt, decryption
 * factor, aggregate): 0 = auto (the default: the engine of least modelled launch time for the
 * launch's ciphertext count -- lane groups of 4 or 3 below the chip's one-lane round, one lane
 * otherwise; fedbiomed_amd/csrc/fbm_jl.hip engine_model_ms), 1 = one lane per ciphertext
 * (throughput: several concurrent launches that fill the chip together), 3 / 4 = three / four
 * lanes per ciphertext (latency), 2 = the generic engine for every modulus (fbm_gen.hip: Barrett
 * products, any N; even N always take it -- under this policy odd N do too, a cross-check of the
 * Montgomery engines).  Results are bit-identical either way.  Returns the previous policy (or
 * FBM_E_ARG).  * fbm_jl_engine_for: the engine a launch of n_ct ciphertexts takes under the policy (1-4). */
int fbm_jl_set_engine(int mode);
int fbm_jl_engine_for(uint64_t n_ct);
/* The exponentiation's short path (a binary chain with the 9-row short-base product, taken for a
 * one-digest FDH h and N > 2^262: DESIGN.md 5.3) on (1, the default) or off (0: every wave runs the
 * sliding-window table path -- an A/B and test switch; results are bit-identical).  Returns the
 * previous setting. */
int fbm_jl_set_short(int on);

/* ---- host test hook (no GPU): the device modular-inverse routine (Bernstein-Yang divsteps,
 * fedbiomed_amd/csrc/fbm_safegcd.hpp) run on the host, for unit tests.
 * x, n, out: 32 little-endian words (n odd);  batches: number of 30-divstep batches used. */
int fbm_test_modinv(const uint32_t* x, const uint32_t* n, uint32_t* out, int* batches);
/* host test hook (no GPU): the FDH's one-digest coprimality test (fbm_jl.hip gcd_is_one_r8) --
 * r8: 8 words (a 256-bit digest), n32: 32 words (odd N).  Returns 1 if gcd(r, N) == 1, 0 if
 * not, a negative FBM_E_* code on bad arguments; *err receives device error flags. */
int fbm_test_fdh_gcd(const uint32_t* r8, const uint32_t* n32, uint32_t* err);
/* host test hooks (no GPU): one ciphertext of the generic engine (fedbiomed_amd/csrc/fbm_gen.hip)
 * run on the host, any N (1 <= N < 2^1024).  fbm_test_gen_exp: out (64 words) = h^key mod N^2 (the
 * inverse of h^|key| for key_negative), times (N pt + 1) mod N^2 when pt (32 words; `negative`:
 * pt holds |pt| of a negative packing) is not NULL; h: 64 words.  fbm_test_gen_combine: v =
 * prod of n_parties 64-word rows (cts, row-major) times factor (64 words, may be NULL) mod N^2;
 * mode 0: out = v (64 words), mode 1: out = ((v - 1) // N) mod N (32 words).  *err receives the
 * device error flags. */
int fbm_test_gen_exp(const uint32_t* h, const uint32_t* pt, int negative, const uint32_t* biprime, const uint32_t* key,
                     int key_negative, uint32_t* out, uint32_t* err);
int fbm_test_gen_combine(const uint32_t* cts, int n_parties, const uint32_t* factor, const uint32_t* biprime,
                         int mode, uint32_t* out, uint32_t* err);
/* host test hook (no GPU): the N-adic engine's per-modulus constants as the library builds
 * them -- nk: 80 words (29-bit N limbs, K'_i), r2na / r3na: 72 limbs (29-bit digits of R^2 /
 * R^3 mod N^2, R = 2^1044), np = -N^-1 mod 2^29. */
int fbm_test_nadic_consts(const uint32_t* n32, uint32_t* nk, uint32_t* r2na, uint32_t* r3na, uint32_t* np);
/* host test hook (no GPU): the short path's per-call words as the library builds them -- kw: |key|'s
 * 64 words, corr: 72 29-bit limbs (the N-adic digits of C = 2^(1044 (2^s + 1) + 261 (|key| - 2^s))
 * mod N^2), d: 36 limbs of N - 2^261.  Returns s = bit length of |key| - 1 (-1 for a zero key), or
 * -2 when N is outside the path's domain (N <= 2^262 or even). */
int fbm_test_short_consts(const uint32_t* n32, const uint32_t* key, uint32_t* kw, uint32_t* corr, uint32_t* d);
/* host test hook (no GPU): the raw words of the short path's cache entries (each: an 8-word digest
 * and 72 limbs of C); returns the word count (out == NULL: a size query), FBM_E_ARG if cap_words is
 * too small. */
int fbm_test_short_cache(uint32_t* out, int cap_words);

/* The LOM aggregate kernel fbm_lom_aggregate launches for n_parties rows of n elements at y (device
 * pointer; its alignment picks the form), as rocprofv3 names it without the "fbm::" namespace, e.g.
 * "lom_aggregate_ws_kernel<2, 4, 8>": the bench keys its committed HBM-traffic profile on it. */
int fbm_test_lom_aggregate_kernel(int n_parties, uint64_t n, const void* y, char* buf, int len);

/* ---- instrumentation -------------------------------------------------------------------
 * fbm_prof_enable(1) makes every entry point record a HIP event pair around each kernel
 * launch (on the caller's stream); fbm_prof_report() synchronises them and returns the
 * bytes needed for the "kernel count total_ms" lines; when len >= that, it writes them
 * into buf and clears the aggregate (buf == NULL is a non-destructive size query).       */
int fbm_prof_enable(int on);
int fbm_prof_report(char* buf, int len);

#ifdef __cplusplus
}
#endif
#endif /* FBM_SECAGG_TEST_H */
