// fedbiomed_amd -- LOM (Low-Overhead Masking) kernels for gfx950.
//
//   lom_protect_kernel   = quantize (utils/_secagg_utils.py:82-119)
//                        + weighting (secagg/_secagg_crypter.py:252-276, :367-373)
//                        + PRF.eval_key per peer (secagg/_lom.py:30-56)
//                        + PRF.eval_vector + signed mask sum + add (secagg/_lom.py:58-83, :152-175)
//   lom_aggregate_kernel = LOM.aggregate u64 column sum (secagg/_lom.py:177-192)
//                        + _apply_average (secagg/_secagg_crypter.py:233-249)
//                        + reverse_quantize (utils/_secagg_utils.py:152-187)
//
// Layout in HBM: x (f32 or f64, n), y (u64, n) per party; aggregate input is a
// P x n row-major u64 matrix (party-major) -> out f64 n (+ optional u64 sums).
#include <cstdio>

#include "fbm_internal.hpp"

namespace fbm {

// One work-item = one ChaCha20 block = 8 consecutive elements (64 B of keystream per
// peer).  Peers are looped inside (uniform control flow); their 32-byte secrets arrive
// as kernel arguments and their per-round seeds (eval_key, one ChaCha20 block each) are
// derived once per workgroup into LDS.
// XT = float/double: quantise + weight (crypter path); XT = uint64_t: raw integer input
// (LOM.protect on a list of ints), x == nullptr means an all-zero input.
template <typename XT>
__device__ __forceinline__ uint64_t lom_input(const XT* x, uint64_t i, const QuantParams& qp, bool& clipped) {
  const double v = (double)x[i];
  clipped |= fbm_outside_clip(v, qp);
  return fbm_quantize(v, qp);
}
template <>
__device__ __forceinline__ uint64_t lom_input<uint64_t>(const uint64_t* x, uint64_t i, const QuantParams&, bool&) {
  return x ? x[i] : 0ull;
}

// Per-round peer seeds into LDS, one peer per thread: PRF.eval_key (_lom.py:30-56) =
// ChaCha20(secret, nonce) over tau.to_bytes(16,'big'), first 16 bytes of keystream XOR
// tau_be16, padded with 16 zero bytes -- or the seeds themselves when the caller has them.
__device__ __forceinline__ void lom_seeds_to_lds(const LomPeers& peers, uint32_t (*seeds)[8], int tid) {
  if (tid < peers.n_peers && peers.raw_seeds) {
#pragma unroll
    for (int w = 0; w < 8; ++w) seeds[tid][w] = peers.secret[tid][w];
  } else if (tid < peers.n_peers) {
    uint32_t ks[16];
    fbm_chacha20_block(peers.secret[tid], peers.ctr0, peers.n14, peers.n15, ks);
#pragma unroll
    for (int w = 0; w < 4; ++w) seeds[tid][w] = ks[w] ^ peers.tau_be[w];
#pragma unroll
    for (int w = 4; w < 8; ++w) seeds[tid][w] = 0u;
  }
}

#ifndef FBM_LOM_WG_PER_CU
// = the resident workgroups per CU of the 64-VGPR build (8 waves/SIMD); A/B on MI355X,
// 10M x 7 peers: 0.277 ms (99 VGPRs, 10 per CU) -> 0.250 (64 VGPRs: quantise after the peer
// loop) -> 0.242 (8 per CU).  0 = one work-item per block.
#define FBM_LOM_WG_PER_CU 8
#endif

// __launch_bounds__(256, 8): at most 64 VGPRs, 8 waves per SIMD (the ChaCha20 chains need the
// latency hiding; 65 VGPRs would cap the occupancy at 7)
template <typename XT>
__global__ void __launch_bounds__(256, 8) lom_protect_kernel(const XT* __restrict__ x, uint64_t n, QuantParams qp,
                                                          uint64_t weight, LomPeers peers,
                                                          uint64_t* __restrict__ y, uint32_t* __restrict__ stats) {
  __shared__ uint32_t seeds[FBM_MAX_PEERS][8];
  const int tid = threadIdx.x;
  lom_seeds_to_lds(peers, seeds, tid);
  __syncthreads();

  const uint64_t nblk = (n + 7) / 8;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  bool clipped = false;
  uint32_t maxbits = 0;
  // grid-stride over ChaCha20 blocks (a grid of FBM_LOM_WG_PER_CU workgroups per CU keeps
  // every wave resident for the whole launch: no ramp, no partial last round)
  for (uint64_t blk = (uint64_t)blockIdx.x * blockDim.x + tid; blk < nblk; blk += stride) {
    const uint64_t base = blk * 8;
    const int cnt = (n - base) >= 8 ? 8 : (int)(n - base);

    // masks (first: the quantised values are formed after the peer loop, so they do not
    // hold registers across the ChaCha20 blocks)
    uint64_t mask[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) mask[j] = 0;
    const uint64_t ctr = peers.ctr0 + (peers.elem_offset >> 3) + blk;  // global ChaCha20 block
    for (int p = 0; p < peers.n_peers; ++p) {
      uint32_t key[8];
#pragma unroll
      for (int w = 0; w < 8; ++w) key[w] = seeds[p][w];
      uint32_t ks[16];
      fbm_chacha20_block(key, ctr, peers.n14, peers.n15, ks);
      const bool add = (peers.add_bits >> p) & 1ull;  // scalar: no per-peer memory load
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint64_t idx = peers.elem_offset + base + (uint64_t)j + peers.tau;
        const uint64_t m = (((uint64_t)ks[2 * j + 1] << 32) | ks[2 * j]) ^ fbm_bswap64(idx);
        mask[j] = add ? mask[j] + m : mask[j] - m;
      }
    }

    // quantise + weight
    uint64_t val[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      uint64_t q = 0;
      if (j < cnt) q = lom_input<XT>(x, base + j, qp, clipped);
      const uint64_t lo = q * weight;
      const uint64_t hi = __umul64hi(q, weight);
      val[j] = lo;
      const uint32_t bl = fbm_bitlen128(hi, lo);
      maxbits = bl > maxbits ? bl : maxbits;
    }

    if (cnt == 8) {
      ulonglong2* yo = reinterpret_cast<ulonglong2*>(y + base);
#pragma unroll
      for (int j = 0; j < 4; ++j) yo[j] = make_ulonglong2(mask[2 * j] + val[2 * j], mask[2 * j + 1] + val[2 * j + 1]);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (j < cnt) y[base + j] = mask[j] + val[j];
    }
  }

  flag_if_any(clipped, stats, FBM_WARN_CLIPPED);
  if (peers.round_range && blockIdx.x == 0 && tid == 0) atomicOr(stats + FBM_STAT_ERRFLAGS, FBM_ERR_ROUND_RANGE);
  // wave-level max of the bit lengths, one atomic per wave
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const uint32_t o = __shfl_xor(maxbits, off, 64);
    maxbits = o > maxbits ? o : maxbits;
  }
  if ((tid & 63) == 0 && maxbits) atomicMax(stats + FBM_STAT_MAXBITS, maxbits);
}

// y += signed masks of a further group of peers (nodes with more than FBM_MAX_PEERS peers:
// the C-ABI runs lom_protect_kernel on the first group, then this kernel per later group).
// In place, no quantisation, no statistics; seeds are already per-round (eval_key done).
__global__ void __launch_bounds__(256) lom_mask_accumulate_kernel(uint64_t n, LomPeers peers, uint64_t* y) {
  __shared__ uint32_t seeds[FBM_MAX_PEERS][8];
  const int tid = threadIdx.x;
  lom_seeds_to_lds(peers, seeds, tid);
  __syncthreads();
  const uint64_t nblk = (n + 7) / 8;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t blk = (uint64_t)blockIdx.x * blockDim.x + tid; blk < nblk; blk += stride) {
    const uint64_t base = blk * 8;
    const int cnt = (n - base) >= 8 ? 8 : (int)(n - base);
    uint64_t mask[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) mask[j] = 0;
    const uint64_t ctr = peers.ctr0 + (peers.elem_offset >> 3) + blk;
    for (int p = 0; p < peers.n_peers; ++p) {
      uint32_t key[8];
#pragma unroll
      for (int w = 0; w < 8; ++w) key[w] = seeds[p][w];
      uint32_t ks[16];
      fbm_chacha20_block(key, ctr, peers.n14, peers.n15, ks);
      const bool add = (peers.add_bits >> p) & 1ull;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint64_t idx = peers.elem_offset + base + (uint64_t)j + peers.tau;
        const uint64_t m = (((uint64_t)ks[2 * j + 1] << 32) | ks[2 * j]) ^ fbm_bswap64(idx);
        mask[j] = add ? mask[j] + m : mask[j] - m;
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (j < cnt) y[base + j] += mask[j];
  }
}

int launch_lom_mask_accumulate(uint64_t n, const LomPeers& peers, uint64_t* y, hipStream_t s) {
  if (n == 0 || peers.n_peers == 0) return FBM_OK;
  const uint64_t nblk = (n + 7) / 8;
  uint64_t g = (nblk + 255) / 256;
  if (g > 256ull * FBM_LOM_WG_PER_CU) g = 256ull * FBM_LOM_WG_PER_CU;
  hipLaunchKernelGGL(lom_mask_accumulate_kernel, dim3((unsigned)g), dim3(256), 0, s, n, peers, y);
  return check_launch("lom_mask_accumulate_kernel");
}

// Column sum over P parties (mod 2^64) + Python-exact average + dequantise.
// EPT consecutive elements per work-item (EPT*8-byte loads per party row), grid-stride.
// PC > 0: party count known at compile time (every row load of a work-item is issued
// before the first add); PC == 0: runtime count.
#ifndef FBM_AGG_EPT
#define FBM_AGG_EPT 2
#endif
#ifndef FBM_AGG_WG_PER_CU
#define FBM_AGG_WG_PER_CU 0  // 0: one pass, no grid-stride (A/B: no measurable difference)
#endif

#ifndef FBM_AGG_NT
// 1: the masked rows are read with nontemporal loads (each byte is read exactly once; A/B on
// MI355X, 10M x 8 parties: 0.133 -> 0.115 ms, 5.4 -> 6.3 TB/s)
#define FBM_AGG_NT 1
#endif
__device__ __forceinline__ uint64_t agg_ld(const uint64_t* p) {
#if FBM_AGG_NT
  return __builtin_nontemporal_load(p);
#else
  return *p;
#endif
}

__device__ __forceinline__ double lom_avg_dequant(uint64_t s, uint64_t total_weight, double neg_c, double step,
                                                  uint32_t& err) {
  const double a = fbm_true_div_u128(s, total_weight);
  // reverse_quantize guard: value > 2^64-1 (float >= 2^64) -> FB624
  err |= (a >= 18446744073709551616.0) ? 1u : 0u;
  return fbm_dequantize(a >= 18446744073709551616.0 ? 0.0 : a, neg_c, step);
}

template <int EPT, int PC>
__global__ void __launch_bounds__(256) lom_aggregate_kernel(const uint64_t* __restrict__ y, int n_parties,
                                                            uint64_t n, uint64_t total_weight, double neg_c,
                                                            double step, double* __restrict__ out,
                                                            uint64_t* __restrict__ sums, uint32_t* __restrict__ stats) {
  const int P = PC > 0 ? PC : n_parties;
  const uint64_t ngrp = (n + EPT - 1) / EPT;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  // rows start (EPT*8)-byte aligned only when n is a multiple of EPT (and y is aligned)
  const bool vec = (n % EPT) == 0 && (reinterpret_cast<uintptr_t>(y) % (EPT * 8)) == 0;
  uint32_t err = 0;
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < ngrp; t += stride) {
    const uint64_t i = (uint64_t)EPT * t;
    uint64_t sm[EPT];
#pragma unroll
    for (int e = 0; e < EPT; ++e) sm[e] = 0;
    if (vec) {
#pragma unroll
      for (int p = 0; p < (PC > 0 ? PC : 1); ++p) {
        if (PC == 0) break;
        const uint64_t* row = static_cast<const uint64_t*>(__builtin_assume_aligned(y + (uint64_t)p * n + i, EPT * 8));
#pragma unroll
        for (int e = 0; e < EPT; ++e) sm[e] += agg_ld(row + e);
      }
      if (PC == 0) {
        for (int p = 0; p < P; ++p) {
          const uint64_t* row =
              static_cast<const uint64_t*>(__builtin_assume_aligned(y + (uint64_t)p * n + i, EPT * 8));
#pragma unroll
          for (int e = 0; e < EPT; ++e) sm[e] += agg_ld(row + e);
        }
      }
    } else {
      for (int p = 0; p < P; ++p)
#pragma unroll
        for (int e = 0; e < EPT; ++e)
          if (i + e < n) sm[e] += agg_ld(y + (uint64_t)p * n + i + e);
    }
    double o[EPT];
#pragma unroll
    for (int e = 0; e < EPT; ++e) o[e] = (i + e < n) ? lom_avg_dequant(sm[e], total_weight, neg_c, step, err) : 0.0;
    if (vec) {
      if (out) {
        double* od = static_cast<double*>(__builtin_assume_aligned(out + i, EPT * 8));
#pragma unroll
        for (int e = 0; e < EPT; ++e) od[e] = o[e];
      }
      if (sums) {
        uint64_t* sd = static_cast<uint64_t*>(__builtin_assume_aligned(sums + i, EPT * 8));
#pragma unroll
        for (int e = 0; e < EPT; ++e) sd[e] = sm[e];
      }
    } else {
#pragma unroll
      for (int e = 0; e < EPT; ++e) {
        if (i + e < n) {
          if (out) out[i + e] = o[e];
          if (sums) sums[i + e] = sm[e];
        }
      }
    }
  }
  if (err && out) atomicOr(stats + FBM_STAT_ERRFLAGS, FBM_ERR_DEQUANT_RANGE);
}

// Wave-split column sum (round 5) for a compile-time party count PC: a workgroup of W waves owns one
// tile of 64*EPT elements; wave w loads rows w, w + W, ... (PC / W rows of 16-byte nontemporal loads per
// lane), the W partial sums meet in LDS, and the epilogue (average, dequantise, nontemporal stores of the
// float64 output and the u64 sums) is spread over the workgroup's threads.  Against lom_aggregate_kernel
// (one thread loads all PC rows of its 2 elements) at config 5's 16 x 100M on one box: 6.05 -> 6.68 TB/s
// (tools/microbench/agg_variants.hip, profiles/r5c_agg_variants.jsonl): fewer rows per lane keep more
// waves resident with the same bytes in flight, and the epilogue's division no longer serialises wave 0.
// Needs n % EPT == 0 and 16-byte aligned rows (the launcher checks); the last tile is bounds-checked.
#ifndef FBM_AGG_WS
#define FBM_AGG_WS 1  // 0: every party count takes lom_aggregate_kernel (A/B base)
#endif
#ifndef FBM_AGG_WS_W8
#define FBM_AGG_WS_W8 4  // waves per workgroup at 8 parties (two rows per wave)
#endif
template <int EPT, int W, int PC>
__global__ void __launch_bounds__(64 * W) lom_aggregate_ws_kernel(const uint64_t* __restrict__ y, uint64_t n,
                                                                  uint64_t total_weight, double neg_c, double step,
                                                                  double* __restrict__ out,
                                                                  uint64_t* __restrict__ sums,
                                                                  uint32_t* __restrict__ stats) {
  static_assert(PC % W == 0, "rows per wave");
  constexpr int TILE = 64 * EPT, RPW = PC / W;
  __shared__ uint64_t part[W][TILE];
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const uint64_t base = (uint64_t)blockIdx.x * TILE;
  const uint64_t i = base + (uint64_t)l * EPT;
  uint64_t sm[EPT];
#pragma unroll
  for (int e = 0; e < EPT; ++e) sm[e] = 0;
  if (base + TILE <= n) {
    uint64_t v[RPW][EPT];
#pragma unroll
    for (int p = 0; p < RPW; ++p) {
      const uint64_t* row =
          static_cast<const uint64_t*>(__builtin_assume_aligned(y + (uint64_t)(w + W * p) * n + i, EPT * 8));
#pragma unroll
      for (int e = 0; e < EPT; ++e) v[p][e] = __builtin_nontemporal_load(row + e);
    }
#pragma unroll
    for (int p = 0; p < RPW; ++p)
#pragma unroll
      for (int e = 0; e < EPT; ++e) sm[e] += v[p][e];
  } else {
#pragma unroll
    for (int p = 0; p < RPW; ++p)
#pragma unroll
      for (int e = 0; e < EPT; ++e)
        if (i + e < n) sm[e] += __builtin_nontemporal_load(y + (uint64_t)(w + W * p) * n + i + e);
  }
#pragma unroll
  for (int e = 0; e < EPT; ++e) part[w][l * EPT + e] = sm[e];
  __syncthreads();
  uint32_t err = 0;
  for (int e = threadIdx.x; e < TILE; e += 64 * W) {
    if (base + e >= n) break;
    uint64_t s = 0;
#pragma unroll
    for (int q = 0; q < W; ++q) s += part[q][e];
    if (out) __builtin_nontemporal_store(lom_avg_dequant(s, total_weight, neg_c, step, err), out + base + e);
    if (sums) __builtin_nontemporal_store(s, sums + base + e);
  }
  if (err && out) atomicOr(stats + FBM_STAT_ERRFLAGS, FBM_ERR_DEQUANT_RANGE);
}

int launch_lom_protect(const void* x, int x_dtype, uint64_t n, const QuantParams& qp, uint64_t weight,
                       const LomPeers& peers, uint64_t* y, uint32_t* stats, hipStream_t s) {
  if (n == 0) return FBM_OK;
  const uint64_t nblk = (n + 7) / 8;
  uint64_t g = (nblk + 255) / 256;
  if (FBM_LOM_WG_PER_CU > 0 && g > 256ull * FBM_LOM_WG_PER_CU) g = 256ull * FBM_LOM_WG_PER_CU;
  const dim3 grid((unsigned)g), block(256);
  if (x_dtype == FBM_F32)
    hipLaunchKernelGGL(lom_protect_kernel<float>, grid, block, 0, s, (const float*)x, n, qp, weight, peers, y, stats);
  else if (x_dtype == FBM_F64)
    hipLaunchKernelGGL(lom_protect_kernel<double>, grid, block, 0, s, (const double*)x, n, qp, weight, peers, y, stats);
  else
    hipLaunchKernelGGL(lom_protect_kernel<uint64_t>, grid, block, 0, s, (const uint64_t*)x, n, qp, weight, peers, y,
                       stats);
  return check_launch("lom_protect_kernel");
}

// reverse_quantize of already-truncated values: -c + step * double(u)  (numpy order, no FMA)
__global__ void __launch_bounds__(256) dequantize_kernel(const uint64_t* __restrict__ u, uint64_t n, double neg_c,
                                                         double step, double* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double du = (double)u[i];
  const double prod = step * du;
  out[i] = neg_c + prod;
}

int launch_dequantize(const uint64_t* u, uint64_t n, double neg_c, double step, double* out, hipStream_t s) {
  if (n == 0) return FBM_OK;
  hipLaunchKernelGGL(dequantize_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, u, n, neg_c, step, out);
  return check_launch("dequantize_kernel");
}

// PRF.eval_key for one (secret, nonce, tau): 32-byte seed to device memory
__global__ void prf_key_kernel(LomPeers peers, uint32_t* __restrict__ seed_out) {
  if (threadIdx.x != 0) return;
  uint32_t ks[16];
  fbm_chacha20_block(peers.secret[0], peers.ctr0, peers.n14, peers.n15, ks);
#pragma unroll
  for (int w = 0; w < 4; ++w) seed_out[w] = ks[w] ^ peers.tau_be[w];
#pragma unroll
  for (int w = 4; w < 8; ++w) seed_out[w] = 0u;
}

int launch_prf_key(const LomPeers& peers, uint32_t* seed_out, hipStream_t s) {
  hipLaunchKernelGGL(prf_key_kernel, dim3(1), dim3(64), 0, s, peers, seed_out);
  return check_launch("prf_key_kernel");
}

// The column-sum kernel a launch of n_parties rows of n elements at y takes: the wave-split form for
// 8 and 16 parties on 16-byte aligned rows of an even length, the one-thread-per-EPT-elements form
// otherwise (PC = the compiled party count, 0 = any).  launch_lom_aggregate dispatches on it, and the
// test build names it (fbm_test_lom_aggregate_kernel): the bench keys its committed HBM-traffic
// profile on the kernel that ran.
static bool lom_agg_ws(int n_parties, uint64_t n, const uint64_t* y) {
  const bool aligned = (n % 2) == 0 && (reinterpret_cast<uintptr_t>(y) % 16) == 0;
  return FBM_AGG_WS && aligned && (n_parties == 16 || n_parties == 8);
}

int lom_aggregate_kernel_name(int n_parties, uint64_t n, const void* y, char* buf, int len) {
  if (n_parties < 1 || !buf || len < 1) return FBM_E_ARG;
  int w;
  if (lom_agg_ws(n_parties, n, (const uint64_t*)y))
    w = snprintf(buf, (size_t)len, "lom_aggregate_ws_kernel<2, %d, %d>", n_parties == 16 ? 8 : FBM_AGG_WS_W8, n_parties);
  else {
    const int pc = (n_parties == 2 || n_parties == 3 || n_parties == 4 || n_parties == 8 || n_parties == 16) ? n_parties : 0;
    w = snprintf(buf, (size_t)len, "lom_aggregate_kernel<%d, %d>", FBM_AGG_EPT, pc);
  }
  return w < len ? FBM_OK : FBM_E_ARG;
}

int launch_lom_aggregate(const uint64_t* y, int n_parties, uint64_t n, uint64_t total_weight, double neg_c, double step,
                         double* out, uint64_t* sums, uint32_t* stats, hipStream_t s) {
  if (n == 0) return FBM_OK;
  if (lom_agg_ws(n_parties, n, y)) {
    const dim3 grid((unsigned)((n + 127) / 128));
    if (n_parties == 16)
      hipLaunchKernelGGL((lom_aggregate_ws_kernel<2, 8, 16>), grid, dim3(512), 0, s, y, n, total_weight, neg_c, step,
                         out, sums, stats);
    else
      hipLaunchKernelGGL((lom_aggregate_ws_kernel<2, FBM_AGG_WS_W8, 8>), grid, dim3(64 * FBM_AGG_WS_W8), 0, s, y, n,
                         total_weight, neg_c, step, out, sums, stats);
    return check_launch("lom_aggregate_ws_kernel");
  }
  constexpr int EPT = FBM_AGG_EPT;
  const uint64_t ngrp = (n + EPT - 1) / EPT;
  uint64_t g = (ngrp + 255) / 256;
  const uint64_t gmax = 256ull * FBM_AGG_WG_PER_CU;  // 256 CUs, grid-stride beyond
  if (FBM_AGG_WG_PER_CU > 0 && g > gmax) g = gmax;
  const dim3 grid((unsigned)g), block(256);
#define FBM_AGG_CASE(PC)                                                                                          \
  case PC:                                                                                                        \
    hipLaunchKernelGGL((lom_aggregate_kernel<EPT, PC>), grid, block, 0, s, y, n_parties, n, total_weight, neg_c, \
                       step, out, sums, stats);                                                                   \
    break;
  switch (n_parties) {
    FBM_AGG_CASE(2) FBM_AGG_CASE(3) FBM_AGG_CASE(4) FBM_AGG_CASE(8) FBM_AGG_CASE(16)
    default:
      hipLaunchKernelGGL((lom_aggregate_kernel<EPT, 0>), grid, block, 0, s, y, n_parties, n, total_weight, neg_c,
                         step, out, sums, stats);
  }
#undef FBM_AGG_CASE
  return check_launch("lom_aggregate_kernel");
}

}  // namespace fbm
