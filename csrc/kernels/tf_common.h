// TransformerModel (ICU) parameter layout and shared device math for the fused kernels.
// Flat layout = state_dict order of reference src/Model.py:194-246 (47,693 fp32).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tf {

constexpr int D_V = 7, D_L = 16, HID = 64, FF = 6, ROW = 24;  // ROW = vitals|labs|label
constexpr int BR_SIZE_BASE = 17926;                           // branch params excluding dense.weight

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
// math helpers (fp32; exact-erf GELU like F.gelu default; LN eps 1e-5, biased variance)
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ float gelu(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_grad(float x) {
  const float cdf = 0.5f * (1.f + erff(x * 0.70710678118654752f));
  const float pdf = 0.39894228040143268f * __expf(-0.5f * x * x);
  return cdf + x * pdf;
}
__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + __expf(-x)); }

__device__ __forceinline__ unsigned short f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x7fffffu)) return (unsigned short)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (unsigned short)(u >> 16);
}
__device__ __forceinline__ float bf2f(unsigned short h) { return __uint_as_float(((uint32_t)h) << 16); }

// dropout keep-test from a stateless hash of (step key, layer, row, col)
__device__ __forceinline__ uint32_t hash3(uint32_t key, uint32_t layer, uint32_t r, uint32_t c) {
  uint32_t x = key ^ (layer * 0x9E3779B9u) ^ (r * 0x85EBCA6Bu) ^ (c * 0xC2B2AE35u);
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}
// keep with probability 1-p: threshold on 24 bits
__device__ __forceinline__ bool keep(uint32_t key, uint32_t layer, uint32_t r, uint32_t c, uint32_t thr24) {
  return (hash3(key, layer, r, c) >> 8) >= thr24;
}

constexpr uint32_t THR_P01 = 1677722u;   // round(0.1 * 2^24)
constexpr uint32_t THR_P03 = 5033165u;   // round(0.3 * 2^24)
constexpr float INV_K01 = 1.f / 0.9f;
constexpr float INV_K03 = 1.f / 0.7f;

// layer ids for the dropout hash (branch-relative ids + 8 * branch)
enum : uint32_t { L_ATT = 0, L_D1 = 1, L_DF = 2, L_D2 = 3, L_HEAD = 16 };

}  // namespace tf
