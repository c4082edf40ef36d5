// Shared device helpers for the gfx950 kernels (wave64, 256-thread workgroups unless noted).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define AFL_WAVE 64

// ---------------------------------------------------------------------------------------------
// wave / block reductions (wave64: 6 xor-shuffle steps)
// ---------------------------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <typename T>
__device__ __forceinline__ T wave_max(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    T w = __shfl_xor(v, o, 64);
    v = v > w ? v : w;
  }
  return v;
}

template <typename T>
__device__ __forceinline__ T wave_min(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    T w = __shfl_xor(v, o, 64);
    v = v < w ? v : w;
  }
  return v;
}

// Block-wide sum; `scratch` must hold blockDim.x/64 elements. Result valid in every thread.
template <typename T>
__device__ __forceinline__ T block_sum(T v, T* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  T r = 0;
  for (int i = 0; i < nw; ++i) r += scratch[i];  // fixed order: deterministic
  return r;
}

// ---------------------------------------------------------------------------------------------
// counter-based RNG (SplitMix64-style finaliser on a 64-bit counter): stateless, any thread can
// regenerate any draw, so backward passes recompute dropout masks instead of storing them.
// ---------------------------------------------------------------------------------------------
__host__ __device__ __forceinline__ uint64_t afl_mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__host__ __device__ __forceinline__ uint32_t afl_hash32(uint32_t a, uint32_t b) {
  // 32-bit avalanche hash of (a, b) (lowbias32 finaliser); cheap enough for per-element dropout
  uint32_t x = a * 0x9E3779B1u ^ (b + 0x7F4A7C15u + (a << 6) + (a >> 2));
  x ^= x >> 16;
  x *= 0x21F0AAADu;
  x ^= x >> 15;
  x *= 0x735A2D97u;
  x ^= x >> 15;
  return x;
}

__device__ __forceinline__ float afl_uniform(uint64_t seed, uint64_t ctr) {
  return (float)(afl_mix64(seed ^ afl_mix64(ctr)) >> 40) * (1.0f / 16777216.0f);
}

// ---------------------------------------------------------------------------------------------
// launch helpers
// ---------------------------------------------------------------------------------------------
static inline int afl_cdiv(long a, long b) { return (int)((a + b - 1) / b); }

// ---------------------------------------------------------------------------------------------
// dropout keep-test shared by the layer kernels: one 32-bit hash of (step key, layer, row, column
// pair) gives the 16-bit uniforms of two adjacent columns; keep iff u16 >= round(p * 65536).
// Step key = afl_hash32(client seed, step).  Mirrored bit-exactly by ops/masks.py.
// ---------------------------------------------------------------------------------------------
__host__ __device__ __forceinline__ uint32_t afl_hash4(uint32_t key, uint32_t layer, uint32_t r, uint32_t c) {
  uint32_t x = key ^ (layer * 0x9E3779B9u) ^ (r * 0x85EBCA6Bu) ^ (c * 0xC2B2AE35u);
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}
__host__ __device__ __forceinline__ bool afl_keep(uint32_t key, uint32_t layer, uint32_t r, uint32_t c,
                                                  uint32_t thr16) {
  return ((afl_hash4(key, layer, r, c >> 1) >> ((c & 1u) << 4)) & 0xFFFFu) >= thr16;
}
