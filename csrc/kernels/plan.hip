// Per-client local-round visit plans (reference client sampling: random.sample of num_data train rows,
// then DataLoader(shuffle=True) per epoch — src/RpcClient.py:97,166-172, client.py:75-111).
//
// order[c, e, i] = F_c(G_{c,e}(i)) for i < nd[c], 0 padding beyond:
//   F_c     keyed permutation of [0, n_train)  -> the client's subset is F_c([0, nd))
//   G_{c,e} keyed permutation of [0, nd[c])    -> the epoch's shuffle of that subset
// Both are 6-round balanced Feistel networks on the smallest even bit-width domain covering n, with
// cycle walking back into [0, n) (a bijection of [0, 2^k) restricted to [0, n) by walking the cycle).
// No sort, no host work: one launch builds the whole [C, E, maxnd] plan.  The integer math is
// mirrored bit-for-bit by attackfl_amd/fl/trainers.py:_feistel_plan (CPU branch); the helpers are
// __host__ __device__ so csrc/host/host_check.hip can run them under ASan/UBSan on the CPU.
#include <algorithm>
#include "common.h"
#include "kernels.h"

namespace {

__host__ __device__ __forceinline__ uint32_t pl_mix(uint32_t x) {
  x ^= x >> 16;
  x *= 0x85EBCA6Bu;
  x ^= x >> 13;
  x *= 0xC2B2AE35u;
  x ^= x >> 16;
  return x;
}

__host__ __device__ __forceinline__ uint32_t pl_feistel(uint32_t x, int half, uint32_t mask, uint32_t k0, uint32_t k1) {
  uint32_t L = x >> half, R = x & mask;
#pragma unroll
  for (int r = 0; r < 6; ++r) {
    const uint32_t F = pl_mix(R ^ k0 ^ (k1 + 0x9E3779B9u * (uint32_t)(r + 1))) & mask;
    const uint32_t nL = R;
    R = L ^ F;
    L = nL;
  }
  return (L << half) | R;
}

__host__ __device__ __forceinline__ uint32_t pl_perm(uint32_t x, uint32_t n, int half, uint32_t k0, uint32_t k1) {
  const uint32_t mask = (1u << half) - 1u;
  do {
    x = pl_feistel(x, half, mask, k0, k1);
  } while (x >= n);
  return x;
}

__host__ __device__ __forceinline__ int pl_half_bits(uint32_t n) {
  int k = 2;
  while ((1ull << k) < (unsigned long long)n) k += 2;
  return k / 2;
}

// subset keys (s0, s1) of a client seed and shuffle keys (e0, e1) of its epoch e
struct PlanKeys {
  uint32_t s0, s1, e0, e1;
};
__host__ __device__ __forceinline__ PlanKeys pl_keys(uint64_t s, int e) {
  const uint32_t lo = (uint32_t)s, hi = (uint32_t)(s >> 32);
  PlanKeys k;
  k.s0 = pl_mix(lo ^ 0x5BD1E995u);
  k.s1 = pl_mix(hi ^ 0x27D4EB2Fu);
  k.e0 = pl_mix(k.s0 ^ (0x165667B1u * (uint32_t)(e + 1)));
  k.e1 = pl_mix(k.s1 + 0xD3A2646Cu * (uint32_t)(e + 1));
  return k;
}

__global__ void __launch_bounds__(256) k_make_plan(const uint64_t* __restrict__ seeds, const int* __restrict__ nd,
                                                   int n_train, int E, int maxnd, int* __restrict__ order) {
  const int c = blockIdx.z, e = blockIdx.y;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= maxnd) return;
  const int n = nd[c];
  int* out = order + ((long)c * E + e) * maxnd;
  if (i >= n) {
    out[i] = 0;  // padding (never visited): a valid row index
    return;
  }
  const PlanKeys k = pl_keys(seeds[c], e);
  const uint32_t j = pl_perm((uint32_t)i, (uint32_t)n, pl_half_bits((uint32_t)n), k.e0, k.e1);
  out[i] = (int)pl_perm(j, (uint32_t)n_train, pl_half_bits((uint32_t)n_train), k.s0, k.s1);
}

// Per-step batch tables of a round (the layer-program and cnn2 trainers' step indexing, reference client.py:75-111:
// client c's s-th step is its s-th batch in (epoch, batch) order): idx [S, C, B] train-row index or -1,
// bsz [S, C] rows in the batch (0 past the client's last batch), ep [S, C] its epoch, nb [C] batches per epoch
// (the loss divisor).  The same launch zeroes the trainer's per-round words (zi [nzi] int32, zf [nzf] fp32), so
// the round boundary between two training launches is this one kernel instead of ~40 small tensor ops.
__global__ void __launch_bounds__(256) k_step_tables(const int* __restrict__ order, const int* __restrict__ nd, int C,
                                                     int E, int maxnd, int B, int S, int* __restrict__ idx,
                                                     int* __restrict__ bsz, int* __restrict__ ep, int* __restrict__ nb,
                                                     int* __restrict__ zi, long nzi, float* __restrict__ zf, long nzf) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i < (long)S * C * B) {
    const int b = (int)(i % B);
    const long sc = i / B;
    const int c = (int)(sc % C), s = (int)(sc / C);
    const int n = nd[c];
    const int nbc = max(1, (n + B - 1) / B);
    const bool valid = s < nbc * E;
    const int e = s / nbc, j = s - e * nbc;
    const int pos = j * B + b;
    const bool ok = valid && pos < n;
    idx[i] = ok ? order[((long)c * E + min(e, E - 1)) * maxnd + min(pos, maxnd - 1)] : -1;
    if (b == 0) {
      bsz[sc] = valid ? min(max(n - j * B, 0), B) : 0;
      ep[sc] = valid ? e : 0;
    }
  }
  if (i < C) nb[i] = max(1, (nd[i] + B - 1) / B);
  if (i < nzi) zi[i] = 0;
  if (i < nzf) zf[i] = 0.f;
}

}  // namespace

void afl_step_tables(const int* order, const int* nd, int C, int E, int maxnd, int B, int S, int* idx, int* bsz,
                     int* ep, int* nb, int* zi, long nzi, float* zf, long nzf, hipStream_t s) {
  const long n = std::max(std::max((long)S * C * B, (long)C), std::max(nzi, nzf));
  if (n <= 0) return;
  hipLaunchKernelGGL(k_step_tables, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, order, nd, C, E, maxnd, B, S,
                     idx, bsz, ep, nb, zi, nzi, zf, nzf);
}

void afl_make_plan(const uint64_t* seeds, const int* nd, int C, int n_train, int E, int maxnd, int* order,
                   hipStream_t s) {
  if (C <= 0 || E <= 0 || maxnd <= 0) return;
  hipLaunchKernelGGL(k_make_plan, dim3((maxnd + 255) / 256, E, C), dim3(256), 0, s, seeds, nd, n_train, E, maxnd,
                     order);
}
