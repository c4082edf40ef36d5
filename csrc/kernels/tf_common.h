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
// math helpers (fp32, branch-free).  GELU is the exact-erf form of F.gelu; erfc comes from Abramowitz &
// Stegun 7.1.26 (|error of erf| <= 1.5e-7: a 5-term polynomial in t = 1/(1 + p z) times exp(-z^2)), whose
// exp(-x^2/2) is shared with the Gaussian pdf of the GELU derivative — one rcp and one exp per value.
// LN eps 1e-5, biased variance.
// ---------------------------------------------------------------------------------------------
// Instruction-lean form (the on-chip trainers are VALU-issue-bound and GELU is a fifth of a branch forward): the
// 1/2 of Phi and the pdf normalisation are folded into the constants — pdf = 2^(x^2 (-log2(e) / 2) + log2(1/sqrt(2 pi)))
// is ONE fma + exp2 of x^2, and erfc(|x|/sqrt2)/2 = t Q(t) pdf with Q = A&S's polynomial times sqrt(2 pi) / 2;
// t = 1/(1 + (p/sqrt2)|x|) is one fma whose |x| is a source modifier.
struct GeluPair {
  float cdf;  // Phi(x) = 0.5 (1 + erf(x / sqrt 2))
  float pdf;  // phi(x) = exp(-x^2 / 2) / sqrt(2 pi)
};
constexpr float AS_P = 0.3275911f, AS_A1 = 0.254829592f, AS_A2 = -0.284496736f, AS_A3 = 1.421413741f,
                AS_A4 = -1.453152027f, AS_A5 = 1.061405429f;
constexpr float G_PZ = (float)(0.3275911 * 0.70710678118654752);         // p / sqrt 2
constexpr float G_QK = 1.2533141373155003f;                                // sqrt(2 pi) / 2
constexpr float G_Q1 = (float)(0.254829592 * 1.2533141373155003), G_Q2 = (float)(-0.284496736 * 1.2533141373155003),
                G_Q3 = (float)(1.421413741 * 1.2533141373155003), G_Q4 = (float)(-1.453152027 * 1.2533141373155003),
                G_Q5 = (float)(1.061405429 * 1.2533141373155003);
constexpr float G_E2 = -0.72134752044448170f;    // -log2(e) / 2
constexpr float G_EL = -1.3257480647361593f;     // log2(1 / sqrt(2 pi))
__device__ __forceinline__ GeluPair gelu_parts(float x) {
  const float t = __builtin_amdgcn_rcpf(fmaf(fabsf(x), G_PZ, 1.f));
  GeluPair g;
  g.pdf = __builtin_amdgcn_exp2f(fmaf(x * x, G_E2, G_EL));
  float q = fmaf(G_Q5, t, G_Q4);
  q = fmaf(q, t, G_Q3);
  q = fmaf(q, t, G_Q2);
  q = fmaf(q, t, G_Q1);
  const float h = (q * t) * g.pdf;  // erfc(|x| / sqrt2) / 2
  g.cdf = x >= 0.f ? 1.f - h : h;
  return g;
}
// two values at once in packed FP32 (v_pk_fma / v_pk_mul: two lanes' worth of math per instruction);
// same formula as gelu_parts.  Returns gelu(x), sets gp = gelu'(x).
typedef float gf2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ gf2v gelu2(gf2v x, gf2v& gp) {
  const gf2v u = {fmaf(fabsf(x[0]), G_PZ, 1.f), fmaf(fabsf(x[1]), G_PZ, 1.f)};
  const gf2v t = {__builtin_amdgcn_rcpf(u[0]), __builtin_amdgcn_rcpf(u[1])};
  const gf2v e2 = (x * x) * G_E2 + G_EL;
  const gf2v pdf = {__builtin_amdgcn_exp2f(e2[0]), __builtin_amdgcn_exp2f(e2[1])};
  gf2v q = t * G_Q5 + G_Q4;
  q = q * t + G_Q3;
  q = q * t + G_Q2;
  q = q * t + G_Q1;
  const gf2v h = (q * t) * pdf;
  const gf2v cdf = {x[0] >= 0.f ? 1.f - h[0] : h[0], x[1] >= 0.f ? 1.f - h[1] : h[1]};
  gp = x * pdf + cdf;
  return x * cdf;
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
