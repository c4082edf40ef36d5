// TransformerModel (ICU) parameter layout and shared device math for the fused kernels.
// Flat layout = state_dict order of reference src/Model.py:194-246 (47,693 fp32).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tf {

constexpr int D_V = 7, D_L = 16, HID = 64, FF = 6, ROW = 24;  // ROW = vitals|labs|label

// per-branch offsets relative to the branch start (Din = input dim)
struct BrOff {
  int dense_w, dense_b, inproj_w, inproj_b, out_w, out_b, ln1_w, ln1_b, ff0_w, ff0_b, ff3_w, ff3_b, ln2_w, ln2_b,
      bn_w, bn_b, size;
};

__host__ __device__ constexpr BrOff br_off(int din, int base) {
  BrOff o{};
  int p = base;
  o.dense_w = p; p += HID * din;
  o.dense_b = p; p += HID;
  o.inproj_w = p; p += 3 * HID * HID;
  o.inproj_b = p; p += 3 * HID;
  o.out_w = p; p += HID * HID;
  o.out_b = p; p += HID;
  o.ln1_w = p; p += HID;
  o.ln1_b = p; p += HID;
  o.ff0_w = p; p += FF * HID;
  o.ff0_b = p; p += FF;
  o.ff3_w = p; p += HID * FF;
  o.ff3_b = p; p += HID;
  o.ln2_w = p; p += HID;
  o.ln2_b = p; p += HID;
  o.bn_w = p; p += HID;
  o.bn_b = p; p += HID;
  o.size = p - base;
  return o;
}

constexpr BrOff OV = br_off(D_V, 0);
constexpr BrOff OL = br_off(D_L, OV.size);
constexpr int FC1_W = OV.size + OL.size;
constexpr int FC1_B = FC1_W + HID * 2 * HID;
constexpr int FC2_W = FC1_B + HID;
constexpr int FC2_B = FC2_W + 32 * HID;
constexpr int OUT_W = FC2_B + 32;
constexpr int OUT_B = OUT_W + 32;
constexpr int NPARAM = OUT_B + 1;
static_assert(NPARAM == 47693, "TransformerModel parameter count");

// ---------------------------------------------------------------------------------------------
// math helpers (fp32, branch-free).  GELU is the exact-erf form of F.gelu; erf comes from the
// Chebyshev erfc fit of Numerical Recipes (|relative error| < 1.2e-7), whose exp(-x^2/2) is shared
// with the Gaussian pdf of the GELU derivative.  LN eps 1e-5, biased variance.
// ---------------------------------------------------------------------------------------------
struct GeluPair {
  float cdf;  // Phi(x) = 0.5 (1 + erf(x / sqrt 2))
  float pdf;  // phi(x) = exp(-x^2 / 2) / sqrt(2 pi)
};
__device__ __forceinline__ GeluPair gelu_parts(float x) {
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(1.f + 0.5f * z);
  float p = 0.17087277f;
  p = fmaf(p, t, -0.82215223f);
  p = fmaf(p, t, 1.48851587f);
  p = fmaf(p, t, -1.13520398f);
  p = fmaf(p, t, 0.27886807f);
  p = fmaf(p, t, -0.18628806f);
  p = fmaf(p, t, 0.09678418f);
  p = fmaf(p, t, 0.37409196f);
  p = fmaf(p, t, 1.00002368f);
  p = fmaf(p, t, -1.26551223f);
  const float e = __expf(-z * z);                 // exp(-x^2/2)
  const float erfc_z = t * e * __expf(p);         // erfc(|x|/sqrt2)
  const float half_erfc = 0.5f * erfc_z;
  GeluPair g;
  g.cdf = x >= 0.f ? 1.f - half_erfc : half_erfc;
  g.pdf = 0.39894228040143268f * e;
  return g;
}
__device__ __forceinline__ float gelu(float x) { return x * gelu_parts(x).cdf; }
__device__ __forceinline__ float gelu_grad(float x) {
  const GeluPair g = gelu_parts(x);
  return fmaf(x, g.pdf, g.cdf);
}
// GELU and its derivative from one erf/exp evaluation (the forward keeps gelu' for the backward)
__device__ __forceinline__ float gelu_and_grad(float x, float& gp) {
  const GeluPair g = gelu_parts(x);
  gp = fmaf(x, g.pdf, g.cdf);
  return x * g.cdf;
}
__device__ __forceinline__ float sigmoidf_(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }

// dropout keep-test from a stateless hash of (step key, layer, row, column pair): one 32-bit hash
// gives the 16-bit uniforms of two adjacent columns (keep iff u16 >= p * 65536)
__device__ __forceinline__ uint32_t hash3(uint32_t key, uint32_t layer, uint32_t r, uint32_t c) {
  uint32_t x = key ^ (layer * 0x9E3779B9u) ^ (r * 0x85EBCA6Bu) ^ (c * 0xC2B2AE35u);
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}
__device__ __forceinline__ bool keep(uint32_t key, uint32_t layer, uint32_t r, uint32_t c, uint32_t thr16) {
  return ((hash3(key, layer, r, c >> 1) >> ((c & 1u) << 4)) & 0xFFFFu) >= thr16;
}
// keep() for columns c0 .. c0+N-1 (c0 even) as a bit mask (bit j = column c0 + j): computed once in the
// forward and reused by the backward instead of re-hashing
template <int N>
__device__ __forceinline__ uint32_t keep_bits(uint32_t key, uint32_t layer, uint32_t r, uint32_t c0, uint32_t thr16) {
  uint32_t m = 0;
#pragma unroll
  for (int j = 0; j < N; j += 2) {
    const uint32_t h = hash3(key, layer, r, (c0 + j) >> 1);
    m |= ((h & 0xFFFFu) >= thr16 ? 1u : 0u) << j;
    m |= ((h >> 16) >= thr16 ? 1u : 0u) << (j + 1);
  }
  return m;
}
__device__ __forceinline__ bool bit(uint32_t m, int j) { return (m >> j) & 1u; }

constexpr uint32_t THR_P01 = 6554u;    // round(0.1 * 2^16)
constexpr uint32_t THR_P03 = 19661u;   // round(0.3 * 2^16)
constexpr float INV_K01 = 1.f / 0.9f;
constexpr float INV_K03 = 1.f / 0.7f;

// layer ids for the dropout hash (branch-relative ids + 8 * branch)
enum : uint32_t { L_ATT = 0, L_D1 = 1, L_DF = 2, L_D2 = 3, L_HEAD = 16 };

}  // namespace tf
