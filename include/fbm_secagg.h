/*
 * fbm_secagg.h -- C ABI of the MI355X (gfx950) secure-aggregation crypter for Fed-BioMed.
 *
 * Drop-in boundary for the reference's Python crypter: these entry points are what the
 * bodies of `SecaggCrypter.encrypt/aggregate` and `SecaggLomCrypter.encrypt/aggregate`
 * (reference fedbiomed/common/secagg/_secagg_crypter.py:45,139,318,394) call, through
 * ctypes, instead of the pure-Python / gmpy2 / OpenSSL implementation.  The Python host
 * side (fedbiomed_amd/) keeps the reference's signatures, validation and exceptions.
 *
 * Conventions
 *  - every compute entry point is ASYNCHRONOUS on `stream` (a hipStream_t, NULL = default
 *    stream) and takes DEVICE pointers only; nothing is allocated inside the library.
 *  - `stats` is a caller-provided device buffer of FBM_STATS_WORDS uint32; the library
 *    zeroes it on `stream` and kernels record device-side conditions in it.  After the
 *    stream is synchronised the caller reads it back and maps it with fbm_check_stats().
 *  - big integers are little-endian arrays of uint32 limbs (== int.to_bytes(.., 'little')).
 *  - return value: FBM_OK or a negative FBM_E_* code; fbm_last_error() has the message
 *    (thread-local).
 *  - libfbm_secagg.so exports exactly the functions declared here (a linker version script made
 *    from this header; tests/test_native_abi.py checks `nm -D`).  The test suite's and the bench's
 *    hooks -- host runs of device routines, per-thread engine switches, the per-kernel event timer
 *    -- are declared in fbm_secagg_test.h and exported by libfbm_secagg_test.so only.
 */
#ifndef FBM_SECAGG_H
#define FBM_SECAGG_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FBM_ABI_VERSION 7 /* 7: the test, A/B and profiling hooks left this header for fbm_secagg_test.h (exported by
                             the test build only); 6: fbm_lom_*_host; 5: fbm_jl_encrypt_factor; 4: fbm_ves_pack takes is_signed; 3: the JL round is an 8192-bit value (FBM_TAU_LIMBS limbs);
                             2 took 16 limbs, 1 a uint64 */
/* The JL round `tau` of every JL entry point: a HOST pointer to FBM_TAU_LIMBS little-endian 32-bit
 * words, any round below 2^8192 -- FDH.H hashes t = (k << 512) | tau as t.to_bytes(1024, 'big')
 * (fedbiomed/common/secagg/_jls.py:451-467, 744-748), whose OverflowError past 2^8192 the Python layer
 * raises.  Never NULL (FBM_E_ARG). */
#define FBM_TAU_LIMBS 256

#define FBM_OK 0
#define FBM_E_ARG (-1)         /* bad argument (type/shape/range)            -> FB624      */
#define FBM_E_HIP (-2)         /* HIP runtime / launch failure                             */
#define FBM_E_RANGE (-3)       /* averaged value > 2^64-1 (reverse_quantize)  -> FB624      */
#define FBM_E_OVERFLOW (-4)    /* LOM overflow guard (_lom.py:133-150)        -> FB417      */
#define FBM_E_FDH (-5)         /* no coprime r of 1..7 FDH digests (_jls.py:742-760: OverflowError) */
#define FBM_E_INVERSE (-6)     /* H^|sk0| not invertible mod N^2 (gmpy2: ZeroDivisionError) */
#define FBM_E_ITER (-7)        /* a bounded data-dependent device loop hit its cap          */
#define FBM_E_UNSUPPORTED (-8) /* parameters outside the device path's domain (documented)  */
#define FBM_E_ROUND (-9)       /* LOM: some i + tau >= 2^64 (_lom.py:81: OverflowError), after FBM_E_OVERFLOW */

#define FBM_F32 0
#define FBM_F64 1
#define FBM_U64 2 /* raw integer input (LOM.protect / JoyeLibert.protect on ints); no quantisation */
#define FBM_I64 3 /* signed 64-bit integers (additive secret sharing)                           */
#define FBM_U128 4 /* raw integers < 2^128 as (lo, hi) uint64 pairs: JoyeLibert.protect / VES.encode */
#define FBM_PT 5   /* packed JL plaintexts, n x 32 uint32 limbs (UserKey.encrypt; cr = 1)          */

#define FBM_STATS_WORDS 4

int fbm_abi_version(void);
const char* fbm_last_error(void);

/* Map a stats block (already copied to host) to a status code.
 * lom_nodes > 0 applies the LOM overflow guard for that many nodes
 * (error iff max_bits >= 64 - ceil(log2(lom_nodes))).  max_bits_out may be NULL. */
int fbm_check_stats(const uint32_t* host_stats, int lom_nodes, uint32_t* max_bits_out);

/* ---- quantisation parameters (reference fedbiomed/common/utils/_secagg_utils.py:82-119)
 * clip      = float(c)          two_clip = float(2*c)
 * target_f  = float(T)          target_m1 = T - 1   (T <= 2^64)
 * weight    = multiplier applied after quantisation (1 = none), < 2^17            */

/* LOM encrypt of one party: quantise -> *weight -> + sum of +/- ChaCha20 pairwise masks.
 * Replaces SecaggLomCrypter.encrypt body (_secagg_crypter.py:318-392) = quantize +
 * _apply_weighting + LOM.protect (_lom.py:105-175) incl. PRF.eval_key/eval_vector (:30-83).
 *   x          device, n elements of dtype x_dtype (FBM_F32 / FBM_F64)
 *   secrets    HOST, n_peers x 32 bytes: the pairwise secrets of the peers (node order)
 *   signs      HOST, n_peers: +1 if peer_id < node_id (mask += PRF), -1 otherwise
 *   raw_seeds  0: secrets are pairwise secrets (seed = PRF.eval_key per round);
 *              1: secrets already are PRF seeds (PRF.eval_vector semantics)
 *   nonce      HOST, 16 bytes (str.encode(nonce).zfill(16)[:16])
 *   y          device, n uint64 (masked output)
 *   elem_offset global index of x[0] when the element range is sharded across devices
 *              (multiple of 8; 0 for a whole vector): PRF block counter and (i + tau) use
 *              global indices, so shards concatenate to the unsharded result.
 * With x_dtype == FBM_U64, x holds integers used as-is (x == NULL: zeros) and only the
 * weight multiplies them (weight 1 = LOM.protect semantics).
 * Status words (fbm_check_stats with lom_nodes = P): the overflow guard (FBM_E_OVERFLOW), then,
 * with n_peers > 0, some global i + tau >= 2^64 (FBM_E_ROUND: the reference's OverflowError from
 * (i + tau).to_bytes(8), _lom.py:81; the counters wrap meanwhile) -- the reference's order.    */
int fbm_lom_protect(const void* x, int x_dtype, uint64_t n, double clip, double two_clip, double target_f,
                    uint64_t target_m1, uint64_t weight, const uint8_t* secrets, const int8_t* signs, int n_peers,
                    int raw_seeds, const uint8_t* nonce, uint64_t tau, uint64_t elem_offset, uint64_t* y,
                    uint32_t* stats, void* stream);

/* PRF.eval_key (_lom.py:30-56): seed_out (device, 32 bytes) = ChaCha20(secret, nonce)
 * keystream[0:16] XOR tau.to_bytes(16,'big') || 16 zero bytes.   secret, nonce: HOST.   */
int fbm_prf_key(const uint8_t* secret, const uint8_t* nonce, uint64_t tau, uint8_t* seed_out, void* stream);

/* reverse_quantize (utils/_secagg_utils.py:152-187) of values already truncated to
 * uint64 (the reference's np.array(weights, dtype=uint64)): out = -c + step*double(u).   */
int fbm_dequantize(const uint64_t* u, uint64_t n, double neg_clip, double step, double* out, void* stream);

/* LOM aggregate: column sum mod 2^64 over n_parties rows, then the crypter's average and
 * dequantisation.  Replaces SecaggLomCrypter.aggregate (_secagg_crypter.py:394-455) =
 * LOM.aggregate (_lom.py:177-192) + _apply_average (:233-249) + reverse_quantize.
 *   y      device, n_parties x n uint64 (row-major, party-major)
 *   neg_clip = float(-c), step = (2c)/(T-1) as a Python float
 *   out    device, n float64 (may be NULL); sums device, n uint64 (may be NULL)           */
int fbm_lom_aggregate(const uint64_t* y, int n_parties, uint64_t n, uint64_t total_weight, double neg_clip,
                      double step, double* out, uint64_t* sums, uint32_t* stats, void* stream);

/* ---- LOM on host buffers (small vectors, e.g. BASELINE config 1's 1 000 elements) ----------------
 * The same computation as fbm_lom_protect / fbm_lom_aggregate with the operands in HOST memory
 * (pinned or not): the input copied to the device workspace, the kernel, the output and the status
 * words copied back, and the stream synchronised -- SYNCHRONOUS, unlike every other entry point: on
 * FBM_OK the host outputs are written.  Status words as the device calls' (fbm_check_stats on
 * stats_host).  A list call of 1 000 elements is launch-bound; this is its one-call form.
 *   workspace  device, fbm_lom_host_workspace(n, 1) bytes (protect) / (n, n_parties) (aggregate);
 *              one call at a time per workspace                                                    */
uint64_t fbm_lom_host_workspace(uint64_t n, int n_parties);
int fbm_lom_protect_host(const void* x_host, int x_dtype, uint64_t n, double clip, double two_clip, double target_f,
                         uint64_t target_m1, uint64_t weight, const uint8_t* secrets, const int8_t* signs, int n_peers,
                         int raw_seeds, const uint8_t* nonce, uint64_t tau, uint64_t elem_offset, uint64_t* y_host,
                         uint32_t* stats_host, void* workspace, void* stream);
int fbm_lom_aggregate_host(const uint64_t* y_host, int n_parties, uint64_t n, uint64_t total_weight, double neg_clip,
                           double step, double* out_host, uint32_t* stats_host, void* workspace, void* stream);

/* ---- Joye-Libert (reference fedbiomed/common/secagg/_jls.py) -------------------------
 * biprime: HOST, 32 limbs (N, 1 <= N < 2^1024; an odd N >= 3 runs on the Montgomery engines, an
 *          even one and N = 1 on the generic engine, fedbiomed_amd/csrc/fbm_gen.hip -- same results;
 *          at N = 1 every ciphertext is 0 and every decryption is FBM_E_INVERSE, the reference's
 *          invert(delta^2, N^2) modulo 1)
 * key:     HOST, 64 limbs |sk| (< 2^2048);  key_negative: sign of sk
 * es, cr:  VES slot bits / slots per ciphertext (JoyeLibert vector encoder, _jls.py:104-116)
 * tau:     HOST, FBM_TAU_LIMBS limbs: the round, < 2^8192 (t_k = (k << 512) | tau, FDH.H's input, _jls.py:451-467);
 *          n_ct = ceil(n / cr)
 * ct_offset: global index of ciphertext 0 (t_k = ((k + ct_offset) << 512) | tau) when the
 *          element range is sharded across devices on ciphertext boundaries; 0 otherwise.   */

/* largest n_ct one call accepts (the device addresses 28-bit-limb columns with 32-bit byte
 * offsets: n_ct * 296 B < 4 GiB); larger vectors are split by ct_offset (element-range
 * shards), which is also how they spread over GPUs.                                      */
#define FBM_JL_MAX_CT 14000000ull

/* bytes of device workspace fbm_jl_encrypt / fbm_jl_aggregate need */
uint64_t fbm_jl_encrypt_workspace(uint64_t n_ct);
uint64_t fbm_jl_aggregate_workspace(uint64_t n_ct);

/* JL encrypt of one party: quantise, weight, VES-pack, c_k = (N*pt_k+1) * H(t_k)^sk mod N^2.
 * Replaces SecaggCrypter.encrypt (_secagg_crypter.py:45-137) = quantize + _apply_weighting +
 * JoyeLibert.protect (_jls.py:593-644) + UserKey.encrypt (:473-505) + FDH.H (:727-762).
 *   weight: the int64 two's complement of the multiplier; a negative weight in (-2^17, 0)
 *           reproduces the reference's packing of negative products (VES._batch ORs the
 *           slots, _jls.py:169-176: pt = the first non-zero q*w shifted to its slot)
 *   ct_out: device, n_ct x 64 uint32 limbs                                                */
int fbm_jl_encrypt(const void* x, int x_dtype, uint64_t n, double clip, double two_clip, double target_f,
                   uint64_t target_m1, uint64_t weight, int es, int cr, const uint32_t* biprime,
                   const uint32_t* key, int key_negative, const uint32_t* tau, uint64_t ct_offset, uint32_t* ct_out,
                   void* workspace, uint32_t* stats, void* stream);
/* fbm_jl_encrypt in two phases on the same arguments and workspace: phase 1 = the prologue
 * kernels (pack, N*pt+1 digits, FDH, the inverse of H for a negative key), phase 2 = the
 * exponentiation, 3 = both (== fbm_jl_encrypt).  Lets a caller running several parties on one
 * device issue every prologue before the first exponentiation takes the whole chip.  Phase 2
 * follows the engine / short-path choice phase 1 made on the same workspace; phase 2 on a
 * workspace phase 1 never ran on (or one of more than 4 096 newer split calls ago) is FBM_E_ARG. */
int fbm_jl_encrypt_phase(const void* x, int x_dtype, uint64_t n, double clip, double two_clip, double target_f,
                         uint64_t target_m1, uint64_t weight, int es, int cr, const uint32_t* biprime,
                         const uint32_t* key, int key_negative, const uint32_t* tau, uint64_t ct_offset, uint32_t* ct_out,
                         void* workspace, uint32_t* stats, void* stream, int phase);

/* fbm_jl_encrypt with its factor computed ahead: c_k = (N pt_k + 1) F_k mod N^2, where F is
 * fbm_jl_decrypt_factor(n_ct, biprime, key, key_negative, tau, ct_offset, ...) for the PARTY's key --
 * H(t_k)^sk needs no plaintext, so a node can compute it while it trains.  Equal bit for bit to
 * fbm_jl_encrypt of the same key, round and ct_offset (UserKey.encrypt, _jls.py:473-505).
 *   factor: device, n_ct x 64 uint32 limbs;  workspace: fbm_jl_encrypt_workspace(n_ct) bytes.
 *   ct_out must not overlap factor (FBM_E_ARG) nor the input x: the kernel stages N pt + 1 in it.
 * An even N or N = 1 is FBM_E_UNSUPPORTED (fbm_jl_encrypt takes every N).                    */
int fbm_jl_encrypt_factor(const void* x, int x_dtype, uint64_t n, double clip, double two_clip, double target_f,
                          uint64_t target_m1, uint64_t weight, int es, int cr, const uint32_t* biprime,
                          const uint32_t* factor, uint32_t* ct_out, void* workspace, uint32_t* stats, void* stream);

/* JL aggregate: prod_u c_u * H(t_k)^sk0 mod N^2, x = ((v-1)//N) mod N, VES decode,
 * average, dequantise.  Replaces SecaggCrypter.aggregate (_secagg_crypter.py:139-230) =
 * JoyeLibert.aggregate (_jls.py:646-699) + ServerKey.decrypt (:520-562) + VES.decode +
 * _apply_average + reverse_quantize.
 *   cts:  device, n_parties x n_ct x 64 uint32 limbs (each < 2^2048)
 *   n_out = number of decoded values (the reference's num_expected_params rule applied)
 *   out:  device, n_out float64 (may be NULL)
 *   sums: device, n_out x 2 uint64 (lo, hi) decoded integer sums (may be NULL)            */
int fbm_jl_aggregate(const uint32_t* cts, int n_parties, uint64_t n_ct, int es, int cr, uint64_t n_out,
                     const uint32_t* biprime, const uint32_t* key, int key_negative, const uint32_t* tau,
                     uint64_t ct_offset, uint64_t total_weight, double neg_clip, double step, double* out, uint64_t* sums,
                     void* workspace, uint32_t* stats, void* stream);

/* The aggregate in two halves (fbm_jl_aggregate = factor, then combine, bit for bit):
 * fbm_jl_decrypt_factor: ServerKey.decrypt's H(t_k)^sk0 mod N^2 (_jls.py:520-562; inverse
 *   first for sk0 < 0) for ciphertexts [ct_offset, ct_offset + n_ct) of round tau --
 *   independent of the parties' ciphertexts, so a researcher can compute it while the
 *   nodes train/encrypt.  factor: device, n_ct x 64 u32 limbs.
 * fbm_jl_aggregate_factor: the ciphertext product (_jls.py:353-374,691-693), v = prod *
 *   factor, x = (v-1)/N, VES decode, average, dequantise -- as fbm_jl_aggregate.
 * Both take fbm_jl_aggregate_workspace(n_ct) bytes of workspace. */
int fbm_jl_decrypt_factor(uint64_t n_ct, const uint32_t* biprime, const uint32_t* key, int key_negative, const uint32_t* tau,
                          uint64_t ct_offset, uint32_t* factor, void* workspace, uint32_t* stats, void* stream);
/* fbm_jl_decrypt_factor in phases on the same arguments and workspace: bit 1 = constants and
 * FDH, bit 2 = the exponentiation, bit 4 = the inverse (negative key); 7 == fbm_jl_decrypt_factor.
 * Bits 2 and 4 without bit 1 need a phase-1 call on the same workspace first (else FBM_E_ARG). */
int fbm_jl_decrypt_factor_phase(uint64_t n_ct, const uint32_t* biprime, const uint32_t* key, int key_negative,
                                const uint32_t* tau, uint64_t ct_offset, uint32_t* factor, void* workspace, uint32_t* stats,
                                void* stream, int phase);
int fbm_jl_aggregate_factor(const uint32_t* cts, int n_parties, uint64_t n_ct, int es, int cr, uint64_t n_out,
                            const uint32_t* biprime, const uint32_t* factor, uint64_t total_weight, double neg_clip,
                            double step, double* out, uint64_t* sums, void* workspace, uint32_t* stats, void* stream);

/* ---- the JoyeLibert object API (reference _jls.py classes, fedbiomed_amd/secagg/_jls.py) ----
 * fbm_jl_encrypt also takes x_dtype FBM_U128 (JoyeLibert.protect: VES-packed raw integers,
 * weight 1) and FBM_PT (UserKey.encrypt, _jls.py:473-505: x = n plaintexts of 32 limbs, each
 * < 2^1024, cr = 1, n_ct = n).
 *
 * fbm_jl_pack: VES.encode (_jls.py:118-144,169-176) of n raw integers (FBM_U128: (lo, hi)
 *   pairs, < 2^128), slot j at bit es*j, cr slots per plaintext, the reference's OR packing
 *   (a value wider than its slot spills into the next slots).  pt: device, ceil(n/cr) x 32
 *   limbs.  A bit past 2^1024 is FBM_E_UNSUPPORTED at fbm_check_stats (the reference keeps it).
 * fbm_jl_unpack: VES.decode (_jls.py:146-192): value o = slot o % cr of plaintext o / cr,
 *   masked to es bits (es <= 128), as (lo, hi) uint64 pairs in vals [n_out x 2] (device).
 * fbm_jl_fdh: FBM's FDH.H (_jls.py:727-762) of t_k = ((k + ct_offset) << 512) | tau, k < n_ct,
 *   bits_size 2048, against a modulus M given as its odd part (32 limbs, odd, >= 1) and whether
 *   M is even (gcd(r, M) == 1 then also needs r odd); for M = N^2 pass N.  h: n_ct x 64 limbs.
 * fbm_jl_product: EncryptedNumber sums (_jls.py:308-374): out[k] = prod_u cts[u][k] mod N^2,
 *   canonical, n_ct x 64 limbs; workspace fbm_jl_aggregate_workspace(n_ct).
 * fbm_jl_decrypt: JoyeLibert.aggregate's product + ServerKey.decrypt (_jls.py:520-562) with
 *   delta = 1: x[k] = ((prod_u cts[u][k] * H(t_k)^key mod N^2) - 1) // N mod N, n_ct x 32
 *   limbs (no VES decode); workspace fbm_jl_aggregate_workspace(n_ct).                    */
int fbm_jl_pack(const void* x, int x_dtype, uint64_t n, int es, int cr, uint32_t* pt, uint32_t* stats, void* stream);
int fbm_jl_unpack(const uint32_t* pt, uint64_t n_ct, int es, int cr, uint64_t n_out, uint64_t* vals, void* stream);
int fbm_jl_fdh(uint64_t n_ct, const uint32_t* modulus_odd, int modulus_even, const uint32_t* tau, uint64_t ct_offset,
               uint32_t* h, uint32_t* stats, void* stream);
/* fbm_jl_fdh_msg: FDH(bits_size, M).H(t) for FDH objects of any bits_size (round 4; reference
 * _jls.py:742-762 -- the crypter's FDH(2048, N^2) takes fbm_jl_fdh): for each of n values t (device,
 * t_words little-endian 32-bit words each, t < 2^(8 (bits_size / 2)): the caller checks the
 * reference's to_bytes range), r = SHA256(t.to_bytes(bits_size / 2) || 1) || SHA256(... || 2) || ...
 * until gcd(r, M) == 1, at most min((bits_size / 8 - 1) / 32, 255) digests (FBM_E_FDH at fbm_check_stats
 * when none qualifies, or at once when bits_size < 264: the reference's counter byte overflows).  M as in
 * fbm_jl_fdh.  h: n rows of h_words limbs (device), h_words = fbm_jl_fdh_msg_row_words(bits_size): 128 up to
 * 15 digests (bits_size <= 4096), 8 per digest above (ABI 4: r of up to 255 digests). */
int fbm_jl_fdh_msg_row_words(int bits_size);
int fbm_jl_fdh_msg(uint64_t n, const uint32_t* t, int t_words, int bits_size, const uint32_t* modulus_odd,
                   int modulus_even, uint32_t* h, int h_words, uint32_t* stats, void* stream);
int fbm_jl_product(const uint32_t* cts, int n_parties, uint64_t n_ct, const uint32_t* biprime, uint32_t* out,
                   void* workspace, void* stream);
int fbm_jl_decrypt(const uint32_t* cts, int n_parties, uint64_t n_ct, const uint32_t* biprime, const uint32_t* key,
                   int key_negative, const uint32_t* tau, uint64_t ct_offset, uint32_t* x, void* workspace, uint32_t* stats,
                   void* stream);

/* Keys whose PublicParam hashes with a callable other than FBM's FDH(2048, N^2).H (BaseKey._populate_tau,
 * _jls.py:451-467, calls it per t on the host; the exponentiations stay on the device):
 * fbm_jl_powmod: out[k] = (N*pt[k] + 1) * h[k]^key mod N^2 (UserKey.encrypt, _jls.py:473-505), or with
 *   pt == NULL out[k] = h[k]^key mod N^2 (ServerKey.decrypt's powmod, :541-543).  h: device, n_ct x 64
 *   limbs (< 2^2048); pt: device, n_ct x 32 limbs (< 2^1024) or NULL; a negative key inverts first (a base
 *   with no inverse is FBM_E_INVERSE at fbm_check_stats); workspace fbm_jl_encrypt_workspace(n_ct).
 * fbm_jl_decrypt_with: x[k] = ((prod_u cts[u][k] * factor[k] mod N^2) - 1) // N mod N (:545-546) for a
 *   factor from fbm_jl_powmod (pt == NULL); n_ct x 32 limbs; workspace fbm_jl_aggregate_workspace(n_ct).
 *   (JoyeLibert.aggregate's VES decode on such a factor: fbm_jl_aggregate_factor.)                      */
int fbm_jl_powmod(const uint32_t* h, const uint32_t* pt, uint64_t n_ct, const uint32_t* biprime, const uint32_t* key,
                  int key_negative, uint32_t* out, void* workspace, uint32_t* stats, void* stream);
int fbm_jl_decrypt_with(const uint32_t* cts, int n_parties, uint64_t n_ct, const uint32_t* biprime,
                        const uint32_t* factor, uint32_t* x, void* workspace, uint32_t* stats, void* stream);

/* multiply / divide of the reference's secagg utils (fedbiomed/common/utils/_secagg_utils.py:122-149,
 * used by SecaggCrypter._apply_weighting / _apply_average, :233-276) on n integers v < 2^128 given as
 * (lo, hi) uint64 pairs in x (device):
 *   op 0: v * k (k < 2^64) into out as n x 3 uint64 words, the exact product (< 2^192); a negative
 *         multiplier is the caller's sign on the result;
 *   op 1: v / k (k >= 1) into out as float64, Python's correctly rounded int/int true division;
 *   op 2: v / kd with kd the float64 whose bit pattern k holds: Python's int / float (float(v)
 *         correctly rounded, then the IEEE division);
 *   op 3: v / (-k) (k >= 1): op 1 negated.                                                       */
int fbm_int_ops(const uint64_t* x, uint64_t n, uint64_t k, int op, void* out, uint32_t* stats, void* stream);
/* fbm_int_true_div_big (round 4): out[i] = x[i] / k (Python's int / int true division, correctly rounded,
 * subnormals included) for a divisor of any size -- |k| given as k_words HOST little-endian words,
 * negative its sign; x as in fbm_int_ops (device u128 pairs), out device float64. */
int fbm_int_true_div_big(const uint64_t* x, uint64_t n, const uint32_t* k, int k_words, int negative, double* out,
                         void* stream);
/* VES objects of any shape (round 4; reference _jls.py:118-192): fbm_ves_pack ORs value j of each group
 * of cr into its plaintext at bit es * j (values: n rows of wv little-endian words, device; bits past the
 * slot land in the next slots, as the reference's a |= v << es j; pt: ceil(n / cr) rows of pw words with
 * es (cr - 1) + 32 wv <= 32 pw); is_signed (ABI 4): the rows are two's complement and a negative value's
 * sign bit repeats up to the plaintext's top word (Python's OR of negative ints: the plaintext is then the
 * negative number pt - 2^(32 pw), its top bit set; keep 32 wv above every value's bit length for its sign);
 * fbm_ves_unpack writes value o = bits [es (o % cr), + es) of plaintext o / cr (pt: n_ct rows of pw words,
 * es cr <= 32 pw) as rows of ow >= ceil(es / 32) words. */
int fbm_ves_pack(const uint32_t* x, uint64_t n, int wv, int es, int cr, int pw, int is_signed, uint32_t* pt,
                 void* stream);
int fbm_ves_unpack(const uint32_t* pt, uint64_t n_ct, int pw, int es, int cr, uint64_t n_out, int ow, uint32_t* vals,
                   void* stream);

/* ---- additive secret sharing of vectors (reference fedbiomed/common/secagg/_additive_ss.py) ----
 * fbm_ass_split replaces AdditiveSecret.split / _shares_int (:40-98) for a list secret:
 * every element v (secret_dtype FBM_U64 or FBM_I64) gets n_shares-1 shares uniform in
 * [0, 2^b] (b = bit_length >= 0, or the bit length of |v| when bit_length < 0, as
 * random.randint(0, 2**b)) and a last share v - sum(others).
 *   shares   device, n_shares x n int128 as (lo, hi) int64 pairs, share-major
 *   seed     HOST, 32 bytes: ChaCha20 key; nonce HOST, 8 bytes (stream id)
 *   elem_offset  global index of secret[0] (element-range shards draw disjoint streams)
 * The reference's MT19937 stream is not reproduced: the contract is sum == v exactly and the
 * share ranges.
 * fbm_ass_reconstruct replaces AdditiveShares.reconstruct (:252-267): exact int128 column sum.
 */
int fbm_ass_split(const void* secret, int secret_dtype, uint64_t n, int n_shares, int bit_length,
                  const uint8_t* seed, const uint8_t* nonce, uint64_t elem_offset, int64_t* shares, void* stream);
int fbm_ass_reconstruct(const int64_t* shares, int n_shares, uint64_t n, int64_t* out, void* stream);

/* Wide additive sharing: secrets of any size, e.g. the 2040-bit JL user key the reference
 * splits at setup (node/secagg/_secagg_setups.py:248-268) and the server-key shares it sums
 * (researcher/secagg/_secagg_context.py:380-382).  Same contract as fbm_ass_split, with
 * two's-complement u32 limbs, limb-major (word k*n + i of element i):
 *   secret  device, l_in x n words;  shares device, n_shares x l_out x n words, where
 *   l_out >= words of (b + ceil(log2 n_shares) + 2) bits (the caller sizes it; b <= 32*l_in
 *   when bit_length < 0);  bit_length >= 0 overrides the per-element |v| bit length.
 * fbm_ass_reconstruct_wide: out (l x n words) = column sum mod 2^(32 l) of n_shares
 *   l-limb values -- exact when the caller's l holds the true sum. */
int fbm_ass_split_wide(const uint32_t* secret, uint64_t n, int l_in, int n_shares, int bit_length, int l_out,
                       const uint8_t* seed, const uint8_t* nonce, uint64_t elem_offset, uint32_t* shares,
                       void* stream);
int fbm_ass_reconstruct_wide(const uint32_t* shares, int n_shares, int l, uint64_t n, uint32_t* out, void* stream);

/* Drops the library's host-side caches: the short path's constant C per (N, |key|) -- kept under a
 * SHA-256 digest of (N, |key|), never the key itself, and zeroed here and on eviction -- and the
 * per-biprime public parameters.  The reference keeps nothing between calls (a fresh
 * SecaggCrypter per call, fedbiomed/node/secagg/_secagg_round.py:142); a caller that wants the
 * same can call this after each round.  Thread-safe; in-flight calls are unaffected (a split
 * call's record of its phase-1 path is kept: it holds no key material). */
void fbm_jl_clear_caches(void);

/* Batched exponentiation (one-lane engine), for callers that run several parties' encrypts and
 * the decryption factor on one device (simulation, the benchmark): between fbm_jl_batch_begin
 * and fbm_jl_batch_flush the calling thread's phase-2-only calls -- fbm_jl_encrypt_phase(..., 2)
 * with a non-negative key, fbm_jl_decrypt_factor_phase(..., 2) -- record their exponentiation
 * instead of launching it; the flush launches ONE kernel over all of them on `stream` (one chunk
 * counter: the chip's rounds pack whatever the parts' sizes and however streams map onto hardware
 * queues).  Calls on the generic engine (an even biprime) are not recorded: they launch at once,
 * on their own stream.  Every recorded call must use the same biprime; at most 24 calls; their prologues must
 * be complete on `stream` at the flush, and their outputs are valid after it.  Other calls made
 * while a batch is open launch as usual; a factor's inverse (phase 4) is refused until the flush.
 * workspace: fbm_jl_batch_workspace() bytes of device memory.  No reference counterpart: the
 * reference encrypts one party per call (fedbiomed/common/secagg/_secagg_crypter.py:45-137). */
int fbm_jl_batch_begin(void);
/* fbm_jl_batch_abort: drops the open batch -- the recorded exponentiations never run, so the calls'
 * outputs stay unwritten.  fbm_jl_batch_count: calls recorded in this thread's open batch (0 when
 * none is open; a call that launched at once, e.g. on the generic engine, is not counted). */
void fbm_jl_batch_abort(void);
int fbm_jl_batch_count(void);
uint64_t fbm_jl_batch_workspace(void);
int fbm_jl_batch_flush(void* workspace, uint64_t workspace_bytes, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* FBM_SECAGG_H */
