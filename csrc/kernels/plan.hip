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

}  // namespace

void afl_make_plan(const uint64_t* seeds, const int* nd, int C, int n_train, int E, int maxnd, int* order,
                   hipStream_t s) {
  if (C <= 0 || E <= 0 || maxnd <= 0) return;
  hipLaunchKernelGGL(k_make_plan, dim3((maxnd + 255) / 256, E, C), dim3(256), 0, s, seeds, nd, n_train, E, maxnd,
                     order);
}
