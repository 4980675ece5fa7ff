/* A plain C99 caller of the C ABI (include/fbm_secagg.h): what a maintainer binding the library from a
 * language other than Python (cgo, JNI, N-API, ...) would write, with nothing of fedbiomed_amd's Python
 * side in the loop.  It runs both crypters' device round trip -- every party's encrypt, then the
 * aggregate -- on device buffers it allocates itself with the HIP runtime, and writes the ciphertexts,
 * masked vectors and averages for tests/test_c_client.py to compare with the oracle and the Python API.
 * The Joye-Libert round also runs with every factor computed ahead (fbm_jl_decrypt_factor ->
 * fbm_jl_encrypt_factor / fbm_jl_aggregate_factor, ABI 5), and the LOM round again on host buffers
 * (fbm_lom_protect_host / fbm_lom_aggregate_host, ABI 6); both must give the same bytes.
 *
 *   fbm_c_roundtrip --abi          prints the ABI version (touches no device)
 *   fbm_c_roundtrip IN OUT         IN: the case (layout below, written by tests/test_c_client.py)
 *
 * IN, little-endian, in this order:
 *   char magic[8] "FBMCRT1"; u32 P, es, cr, pad; u64 n, n_out, target_m1, total_weight, lom_tau;
 *   f64 clip, two_clip, target_f, neg_clip, step;
 *   u32 biprime[32], jl_tau[FBM_TAU_LIMBS], server_key[64]; i32 server_key_negative, pad;
 *   per party: u64 weight; i32 key_negative, pad; u32 key[64];
 *   f32 x[P][n];
 *   u8 nonce[16]; per party: u8 secrets[P - 1][32]; i8 signs[P - 1]
 * OUT: u32 cts[P][n_ct][64]; f64 jl_avg[n_out]; u64 lom_y[P][n]; f64 lom_avg[n]
 * Exit status 0, or 1 with the library's message (fbm_last_error) on stderr.
 */
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "fbm_secagg.h"

static FILE* g_in;

static void die(const char* what, const char* detail) {
    fprintf(stderr, "fbm_c_roundtrip: %s: %s\n", what, detail ? detail : "");
    exit(1);
}

static void rd(void* dst, size_t bytes) {
    if (bytes && fread(dst, 1, bytes, g_in) != bytes) die("short input", NULL);
}

static void* xmalloc(size_t bytes) {
    void* p = malloc(bytes ? bytes : 1);
    if (!p) die("out of host memory", NULL);
    return p;
}

static void* dalloc(size_t bytes) {
    void* p = NULL;
    if (hipMalloc(&p, bytes ? bytes : 16) != hipSuccess) die("hipMalloc", NULL);
    return p;
}

static void hip_ok(hipError_t e, const char* what) {
    if (e != hipSuccess) die(what, hipGetErrorString(e));
}

static void fbm_ok(int rc, const char* what) {
    if (rc != FBM_OK) die(what, fbm_last_error());
}

/* the status words of a finished call: FBM_OK or die (lom_nodes > 0: the LOM overflow guard) */
static void stats_ok(const uint32_t* d_stats, int lom_nodes, const char* what) {
    uint32_t h[FBM_STATS_WORDS];
    hip_ok(hipMemcpy(h, d_stats, sizeof h, hipMemcpyDeviceToHost), "stats copy");
    fbm_ok(fbm_check_stats(h, lom_nodes, NULL), what);
}

int main(int argc, char** argv) {
    if (argc == 2 && strcmp(argv[1], "--abi") == 0) {
        printf("%d\n", fbm_abi_version());
        return fbm_abi_version() == FBM_ABI_VERSION ? 0 : 1;
    }
    if (argc != 3) die("usage", "fbm_c_roundtrip --abi | fbm_c_roundtrip IN OUT");
    if (fbm_abi_version() != FBM_ABI_VERSION) die("ABI", "the library is another ABI than this header");
    g_in = fopen(argv[1], "rb");
    if (!g_in) die("cannot open", argv[1]);

    char magic[8];
    uint32_t P, es, cr, pad;
    uint64_t n, n_out, target_m1, total_weight, lom_tau;
    double clip, two_clip, target_f, neg_clip, step;
    uint32_t biprime[32], jl_tau[FBM_TAU_LIMBS], server_key[64];
    int32_t sk_negative, pad32;
    rd(magic, 8);
    if (memcmp(magic, "FBMCRT1", 8) != 0) die("bad magic", argv[1]);
    rd(&P, 4), rd(&es, 4), rd(&cr, 4), rd(&pad, 4);
    rd(&n, 8), rd(&n_out, 8), rd(&target_m1, 8), rd(&total_weight, 8), rd(&lom_tau, 8);
    rd(&clip, 8), rd(&two_clip, 8), rd(&target_f, 8), rd(&neg_clip, 8), rd(&step, 8);
    rd(biprime, sizeof biprime), rd(jl_tau, sizeof jl_tau), rd(server_key, sizeof server_key);
    rd(&sk_negative, 4), rd(&pad32, 4);
    if (P < 2 || P > 64 || cr == 0 || n == 0 || n > (1u << 24)) die("case out of this client's range", NULL);

    uint64_t* weight = xmalloc(P * sizeof *weight);
    int32_t* key_negative = xmalloc(P * sizeof *key_negative);
    uint32_t* keys = xmalloc((size_t)P * 64 * 4);
    for (uint32_t p = 0; p < P; ++p) {
        rd(&weight[p], 8), rd(&key_negative[p], 4), rd(&pad32, 4);
        rd(keys + (size_t)p * 64, 64 * 4);
    }
    float* x = xmalloc((size_t)P * n * sizeof *x);
    rd(x, (size_t)P * n * sizeof *x);
    uint8_t nonce[16];
    rd(nonce, 16);
    const int n_peers = (int)P - 1;
    uint8_t* secrets = xmalloc((size_t)P * n_peers * 32);
    int8_t* signs = xmalloc((size_t)P * n_peers);
    for (uint32_t p = 0; p < P; ++p) {
        rd(secrets + (size_t)p * n_peers * 32, (size_t)n_peers * 32);
        rd(signs + (size_t)p * n_peers, (size_t)n_peers);
    }
    fclose(g_in);

    hipStream_t stream;
    hip_ok(hipStreamCreate(&stream), "hipStreamCreate");
    const uint64_t n_ct = (n + cr - 1) / cr;
    float* d_x = dalloc((size_t)P * n * sizeof *d_x);
    uint32_t* d_cts = dalloc((size_t)P * n_ct * 64 * 4);
    double* d_jl_avg = dalloc(n_out * sizeof(double));
    uint64_t* d_y = dalloc((size_t)P * n * 8);
    double* d_lom_avg = dalloc(n * sizeof(double));
    uint32_t* d_stats = dalloc(FBM_STATS_WORDS * 4);
    uint64_t ws_bytes = fbm_jl_encrypt_workspace(n_ct);
    if (fbm_jl_aggregate_workspace(n_ct) > ws_bytes) ws_bytes = fbm_jl_aggregate_workspace(n_ct);
    void* d_ws = dalloc(ws_bytes);
    hip_ok(hipMemcpyAsync(d_x, x, (size_t)P * n * sizeof *d_x, hipMemcpyHostToDevice, stream), "H2D");

    /* Joye-Libert: each party's encrypt into its row of the [P, n_ct, 64] block, then the aggregate */
    for (uint32_t p = 0; p < P; ++p) {
        fbm_ok(fbm_jl_encrypt(d_x + (size_t)p * n, FBM_F32, n, clip, two_clip, target_f, target_m1, weight[p],
                              (int)es, (int)cr, biprime, keys + (size_t)p * 64, key_negative[p], jl_tau, 0,
                              d_cts + (size_t)p * n_ct * 64, d_ws, d_stats, stream),
               "fbm_jl_encrypt");
        hip_ok(hipStreamSynchronize(stream), "sync");
        stats_ok(d_stats, 0, "fbm_jl_encrypt status");
    }
    fbm_ok(fbm_jl_aggregate(d_cts, (int)P, n_ct, (int)es, (int)cr, n_out, biprime, server_key, sk_negative, jl_tau, 0,
                            total_weight, neg_clip, step, d_jl_avg, NULL, d_ws, d_stats, stream),
           "fbm_jl_aggregate");
    hip_ok(hipStreamSynchronize(stream), "sync");
    stats_ok(d_stats, 0, "fbm_jl_aggregate status");

    /* the same round with every factor computed ahead (ABI 5): each party's H(t_k)^key by
     * fbm_jl_decrypt_factor with its own key, then fbm_jl_encrypt_factor; the server's by
     * fbm_jl_decrypt_factor, then fbm_jl_aggregate_factor -- the same bytes as above, or exit 1 */
    {
        uint32_t* d_f = dalloc((size_t)n_ct * 64 * 4);
        uint32_t* d_cts2 = dalloc((size_t)P * n_ct * 64 * 4);
        double* d_avg2 = dalloc(n_out * sizeof(double));
        const size_t ct_bytes = (size_t)P * n_ct * 64 * 4;
        for (uint32_t p = 0; p < P; ++p) {
            fbm_ok(fbm_jl_decrypt_factor(n_ct, biprime, keys + (size_t)p * 64, key_negative[p], jl_tau, 0, d_f, d_ws,
                                         d_stats, stream),
                   "fbm_jl_decrypt_factor (party key)");
            hip_ok(hipStreamSynchronize(stream), "sync");
            stats_ok(d_stats, 0, "fbm_jl_decrypt_factor status");
            fbm_ok(fbm_jl_encrypt_factor(d_x + (size_t)p * n, FBM_F32, n, clip, two_clip, target_f, target_m1, weight[p],
                                         (int)es, (int)cr, biprime, d_f, d_cts2 + (size_t)p * n_ct * 64, d_ws, d_stats,
                                         stream),
                   "fbm_jl_encrypt_factor");
            hip_ok(hipStreamSynchronize(stream), "sync");
            stats_ok(d_stats, 0, "fbm_jl_encrypt_factor status");
        }
        fbm_ok(fbm_jl_decrypt_factor(n_ct, biprime, server_key, sk_negative, jl_tau, 0, d_f, d_ws, d_stats, stream),
               "fbm_jl_decrypt_factor (server key)");
        hip_ok(hipStreamSynchronize(stream), "sync");
        stats_ok(d_stats, 0, "fbm_jl_decrypt_factor status");
        fbm_ok(fbm_jl_aggregate_factor(d_cts2, (int)P, n_ct, (int)es, (int)cr, n_out, biprime, d_f, total_weight,
                                       neg_clip, step, d_avg2, NULL, d_ws, d_stats, stream),
               "fbm_jl_aggregate_factor");
        hip_ok(hipStreamSynchronize(stream), "sync");
        stats_ok(d_stats, 0, "fbm_jl_aggregate_factor status");
        unsigned char* a = xmalloc(ct_bytes);
        unsigned char* b = xmalloc(ct_bytes);
        hip_ok(hipMemcpy(a, d_cts, ct_bytes, hipMemcpyDeviceToHost), "D2H");
        hip_ok(hipMemcpy(b, d_cts2, ct_bytes, hipMemcpyDeviceToHost), "D2H");
        if (memcmp(a, b, ct_bytes) != 0) die("factor ahead", "ciphertexts differ from fbm_jl_encrypt's");
        free(a), free(b);
        a = xmalloc(n_out * sizeof(double));
        b = xmalloc(n_out * sizeof(double));
        hip_ok(hipMemcpy(a, d_jl_avg, n_out * sizeof(double), hipMemcpyDeviceToHost), "D2H");
        hip_ok(hipMemcpy(b, d_avg2, n_out * sizeof(double), hipMemcpyDeviceToHost), "D2H");
        if (n_out && memcmp(a, b, n_out * sizeof(double)) != 0) die("factor ahead", "averages differ from fbm_jl_aggregate's");
        free(a), free(b);
        void* bufs[] = {d_f, d_cts2, d_avg2};
        for (size_t k = 0; k < 3; ++k) hip_ok(hipFree(bufs[k]), "hipFree");
    }

    /* LOM: each party's masked vector, then the column sums' average */
    for (uint32_t p = 0; p < P; ++p) {
        fbm_ok(fbm_lom_protect(d_x + (size_t)p * n, FBM_F32, n, clip, two_clip, target_f, target_m1, weight[p],
                               secrets + (size_t)p * n_peers * 32, signs + (size_t)p * n_peers, n_peers, 0, nonce,
                               lom_tau, 0, d_y + (size_t)p * n, d_stats, stream),
               "fbm_lom_protect");
        hip_ok(hipStreamSynchronize(stream), "sync");
        stats_ok(d_stats, (int)P, "fbm_lom_protect status");
    }
    fbm_ok(fbm_lom_aggregate(d_y, (int)P, n, total_weight, neg_clip, step, d_lom_avg, NULL, d_stats, stream),
           "fbm_lom_aggregate");
    hip_ok(hipStreamSynchronize(stream), "sync");
    stats_ok(d_stats, 0, "fbm_lom_aggregate status");

    /* the same LOM round on host buffers (ABI 6, synchronous): each party's fbm_lom_protect_host from its
     * host floats, then fbm_lom_aggregate_host of the host rows -- the same bytes as above, or exit 1 */
    {
        uint64_t wsb = fbm_lom_host_workspace(n, (int)P);
        void* d_hws = dalloc(wsb);
        uint64_t* y = xmalloc((size_t)P * n * 8);
        double* avg = xmalloc(n * sizeof(double));
        uint32_t st[FBM_STATS_WORDS];
        for (uint32_t p = 0; p < P; ++p) {
            fbm_ok(fbm_lom_protect_host(x + (size_t)p * n, FBM_F32, n, clip, two_clip, target_f, target_m1, weight[p],
                                        secrets + (size_t)p * n_peers * 32, signs + (size_t)p * n_peers, n_peers, 0,
                                        nonce, lom_tau, 0, y + (size_t)p * n, st, d_hws, stream),
                   "fbm_lom_protect_host");
            fbm_ok(fbm_check_stats(st, (int)P, NULL), "fbm_lom_protect_host status");
        }
        fbm_ok(fbm_lom_aggregate_host(y, (int)P, n, total_weight, neg_clip, step, avg, st, d_hws, stream),
               "fbm_lom_aggregate_host");
        fbm_ok(fbm_check_stats(st, 0, NULL), "fbm_lom_aggregate_host status");
        uint64_t* y_dev = xmalloc((size_t)P * n * 8);
        double* avg_dev = xmalloc(n * sizeof(double));
        hip_ok(hipMemcpy(y_dev, d_y, (size_t)P * n * 8, hipMemcpyDeviceToHost), "D2H");
        hip_ok(hipMemcpy(avg_dev, d_lom_avg, n * sizeof(double), hipMemcpyDeviceToHost), "D2H");
        if (memcmp(y, y_dev, (size_t)P * n * 8) != 0) die("host buffers", "masked vectors differ from fbm_lom_protect's");
        if (memcmp(avg, avg_dev, n * sizeof(double)) != 0) die("host buffers", "averages differ from fbm_lom_aggregate's");
        free(y), free(avg), free(y_dev), free(avg_dev);
        hip_ok(hipFree(d_hws), "hipFree");
    }

    FILE* out = fopen(argv[2], "wb");
    if (!out) die("cannot open", argv[2]);
    struct { const void* d; size_t bytes; } parts[4] = {
        {d_cts, (size_t)P * n_ct * 64 * 4}, {d_jl_avg, n_out * sizeof(double)},
        {d_y, (size_t)P * n * 8}, {d_lom_avg, n * sizeof(double)}};
    for (int k = 0; k < 4; ++k) {
        void* h = xmalloc(parts[k].bytes);
        hip_ok(hipMemcpy(h, parts[k].d, parts[k].bytes, hipMemcpyDeviceToHost), "D2H");
        if (parts[k].bytes && fwrite(h, 1, parts[k].bytes, out) != parts[k].bytes) die("short write", argv[2]);
        free(h);
    }
    fclose(out);
    void* dev_bufs[] = {d_x, d_cts, d_jl_avg, d_y, d_lom_avg, d_stats, d_ws};
    for (size_t k = 0; k < sizeof dev_bufs / sizeof dev_bufs[0]; ++k) hip_ok(hipFree(dev_bufs[k]), "hipFree");
    hip_ok(hipStreamDestroy(stream), "hipStreamDestroy");
    free(weight), free(key_negative), free(keys), free(x), free(secrets), free(signs);
    return 0;
}
