// HAR TransformerClassifier encoder on bf16 activations (reference src/Model.py:418-458:
// Conv1d(1->64, k3) + PE stem, 2 post-norm nn.TransformerEncoderLayer (d 64, 4 heads x 16, FFN 256, ReLU,
// dropout 0.1), mean over L, MLP head).  The generic layer program kept every activation of the
// [C * B * 561, 64 .. 256] encoder in fp32 and ran LayerNorm / residual / dropout as separate passes over
// HBM (a 574k-row step moved ~10 GB); here a layer is five launches over bf16 rows:
//
//   k_har_qkv      x -> q | k | v (bf16, head-major [cb*H + h][3][Lp][16]: every attention workgroup reads
//                  one contiguous 36 KB block; q pre-scaled by log2(e) / sqrt(16), so a score is already in the
//                  log2 domain of the softmax's v_exp_f32)
//   k_har_attn_*   flash attention fwd / bwd on the head-major blocks (below)
//   k_har_post     ONE row pass: out_proj + dropout + residual + LN1 -> linear1 + ReLU + dropout -> linear2
//                  + dropout + residual + LN2; the 256-wide FFN activation never leaves registers (the
//                  backward recomputes it); saves the two normalised LN inputs (bf16), their rstd and the
//                  row's dropout keep bits (16 B per lane: the backward does no hashing)
//   k_har_post_bwd the matching backward row pass: LN2', FFN (recomputed), LN1', out_proj'; weight
//                  gradients accumulated per workgroup in MFMA accumulators over ~35 64-row blocks (the dW
//                  operands staged in XOR-swizzled LDS tiles, read with ds_read_b64_tr_b16), ordered
//                  per-workgroup partials reduced by k_har_reduce (deterministic, no atomics); also
//                  writes Delta = rowsum(dO o O) per head for the attention backward
//   k_har_qkv_bwd  dx = d(residual) + [dq dk dv] . W_in, d(in_proj) partials
//
// Row-pass layout (onchip.h "T layout"): a wave owns 16 rows; every GEMM is computed transposed,
// Y^T = W . X^T on v_mfma_f32_16x16x32_bf16, so lane (r, g) ends holding features 16t + 4g + i of row r —
// the B operand of the next GEMM when that weight's LDS image stores its K axis permuted (pcol).  A
// LayerNorm row sum is an in-lane sum plus two lane swaps.  Weights are staged once per workgroup (each
// workgroup serves one client's rows: grid = (blocks per client, clients)).
// Dropout masks: the row passes use the layer library's (afl_keep of (step key, layer id, row, column)); the
// attention probabilities use a row hash x column-pair hash mix (attn_mix, masks.keep_rc) that costs a
// fraction of a full hash per probability.  The layer program on CPU (ops/layers.py composites, attention
// scheme "rc") is the oracle of these kernels.
#include <type_traits>
#include "common.h"
#include "kernels.h"
#include "onchip.h"

using namespace oc;

namespace {

constexpr int D = 64, NH = 4, DH = 16, FF = 256;
constexpr int NW = 4, NTR = 64 * NW;  // backward row passes: 4 waves (one per SIMD), 64 rows per block
constexpr int NWF = 8, NTF = 64 * NWF;  // forward row passes: 8 waves (two per SIMD), 16 rows each
constexpr int NWP = 16, NTP = 64 * NWP;  // post-attention forward: 16 waves (four per SIMD; LDS allows one workgroup per CU)
#ifndef HAR_IMG_PAD
#define HAR_IMG_PAD 8
#endif
// weight-image row strides (bytes).  HAR_IMG_PAD=16 (32-byte padding) makes the fragment reads conflict-free in
// gfx950 banking (wfrag ds_read_b128: 4 -> 0 extra cycles per instruction, wtfrag tr_b16 4 / 6 -> 2;
// tools/dbg/lds_banks.py), but measured neutral here (3.381 vs 3.380 rounds/s, profiles/ab_r5_img_pad.log): these
// row passes are not bound by their image reads, unlike the on-chip trainers
constexpr int LDK64 = (64 + HAR_IMG_PAD) * 2, LDK256 = (256 + HAR_IMG_PAD) * 2;
// (the post backward's FFN-down image keeps the 8-element padding in any case: 16 more bytes per row do not fit)
constexpr int LDK256B = (256 + 8) * 2;
typedef unsigned short u16;
typedef __attribute__((address_space(1))) const u16 gcu16;

__device__ __forceinline__ uint32_t dkey(const AflDrop& d, int c) {
  return d.thr16 ? afl_hash32(d.seeds[c], (uint32_t)(d.stepctl ? *d.stepctl : 0)) : 0u;
}

// bf16 image [n][k'] of the fp32 row-major weight W [N][K]: k' = pcol(k) (PERM: K fed from T-layout
// registers) or k (natural: K fed from rows loaded straight from memory)
template <bool PERM>
__device__ void build_img(uchar* smem, int img, int ld, const float* __restrict__ W, int N, int K) {
  // 4 consecutive k per thread, one 8-byte LDS store (pcol keeps aligned groups of 4 together)
  const int K4 = K >> 2;
  for (int e = threadIdx.x; e < N * K4; e += blockDim.x) {
    const int n = e / K4, k = 4 * (e - n * K4);
    const float* w = W + (long)n * K + k;  // (dword loads: a client's parameter row need not be 16-byte aligned)
    *(LDS_AS u32x2v*)(smem + img + n * ld + (PERM ? pcol(k) : k) * 2) = u32x2v{pk2(w[0], w[1]), pk2(w[2], w[3])};
  }
}
__device__ void load_vec(uchar* smem, int off, const float* __restrict__ v, int n) {
  for (int e = threadIdx.x; e < n; e += blockDim.x) ldsf(smem, off)[e] = v[e];
}

// natural-order B fragment of k-step s: row r, features 32s + 8g .. +7 (one 16-byte load)
__device__ __forceinline__ s8v ldx8(const u16* __restrict__ rowp, int s, int g, bool ok) {
  if (!ok) return s8v{0, 0, 0, 0, 0, 0, 0, 0};
  return *(const s8v*)(rowp + 32 * s + 8 * g);
}
// T-layout 16 values (features 16t + 4g + i) of a bf16 row
__device__ __forceinline__ void ldt16(float (&x)[16], const u16* __restrict__ rowp, int g, bool ok) {
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    u32x2v u = ok ? *(const u32x2v*)(rowp + 16 * t + 4 * g) : u32x2v{0u, 0u};
    x[4 * t] = __uint_as_float(u[0] << 16);
    x[4 * t + 1] = __uint_as_float(u[0] & 0xFFFF0000u);
    x[4 * t + 2] = __uint_as_float(u[1] << 16);
    x[4 * t + 3] = __uint_as_float(u[1] & 0xFFFF0000u);
  }
}
__device__ __forceinline__ void stt16(u16* __restrict__ rowp, const float (&x)[16], int g) {
#pragma unroll
  for (int t = 0; t < 4; ++t)
    *(u32x2v*)(rowp + 16 * t + 4 * g) = u32x2v{pk2(x[4 * t], x[4 * t + 1]), pk2(x[4 * t + 2], x[4 * t + 3])};
}
// T-layout fp32 rows
__device__ __forceinline__ void ldt16f(float (&x)[16], const float* __restrict__ rowp, int g, bool ok) {
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const f4v v = ok ? *(const f4v*)(rowp + 16 * t + 4 * g) : Z4;
    x[4 * t] = v[0]; x[4 * t + 1] = v[1]; x[4 * t + 2] = v[2]; x[4 * t + 3] = v[3];
  }
}
__device__ __forceinline__ void stt16f(float* __restrict__ rowp, const float (&x)[16], int g) {
#pragma unroll
  for (int t = 0; t < 4; ++t) *(f4v*)(rowp + 16 * t + 4 * g) = f4v{x[4 * t], x[4 * t + 1], x[4 * t + 2], x[4 * t + 3]};
}

// keep bits (bit 4t + i) of features 16 (t0 + t) + 4g + i, t = 0..NT-1, of row r: afl_keep pairs
template <int NT>
__device__ __forceinline__ void keep_bits(uint32_t (&m)[(NT + 7) / 8], uint32_t key, uint32_t layer, uint32_t r, int g,
                                          uint32_t thr, int t0 = 0) {
#pragma unroll
  for (int w = 0; w < (NT + 7) / 8; ++w) m[w] = 0u;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint32_t x = afl_hash4(key, layer, r, (uint32_t)(8 * (t0 + t) + 2 * g + h));
      const uint32_t b = ((x & 0xFFFFu) >= thr ? 1u : 0u) | ((x >> 16) >= thr ? 2u : 0u);
      m[t >> 3] |= b << (4 * (t & 7) + 2 * h);
    }
}
// the FFN's 256 features: two words (tiles 0-7, 8-15)
__device__ __forceinline__ void ffn_bits(uint32_t (&m)[2], uint32_t key, uint32_t layer, uint32_t r, int g, uint32_t thr) {
  uint32_t lo[1], hi[1];
  keep_bits<8>(lo, key, layer, r, g, thr, 0);
  keep_bits<8>(hi, key, layer, r, g, thr, 8);
  m[0] = lo[0];
  m[1] = hi[0];
}
__device__ __forceinline__ float kf(float x, const uint32_t* m, int j, float inv) {
  return keepf(x, m[j >> 5], j & 31) * inv;
}

// =================================================================================== stem
// h0 [c][b*L + l][64] (bf16) = conv1d(x[c][b][:], k3, pad 1)[l] + bias + pe[l].  A block covers 32 rows, 8
// threads per row with 8 channels each (one 16-byte store); the conv weights and biases are staged in LDS once per
// block (the per-thread scattered parameter loads made this pass ~10x slower than its 73 MB of stores)
constexpr int STEM_ROWS = 32;
__global__ void __launch_bounds__(256) k_har_stem(const float* __restrict__ x, int B, int L, const float* __restrict__ params,
                                                  long P, int w_off, int b_off, int pe_off, u16* __restrict__ h) {
  __shared__ float wsb[64 * 4];  // [o][w0 w1 w2 b]
  const int c = blockIdx.y;
  const long R = (long)B * L;
  const float* pp = params + (long)c * P;
  if (threadIdx.x < 64) {
    const int o = threadIdx.x;
    wsb[4 * o] = pp[w_off + 3 * o];
    wsb[4 * o + 1] = pp[w_off + 3 * o + 1];
    wsb[4 * o + 2] = pp[w_off + 3 * o + 2];
    wsb[4 * o + 3] = pp[b_off + o];
  }
  __syncthreads();
  const long row = (long)blockIdx.x * STEM_ROWS + (threadIdx.x >> 3);
  const int o0 = (int)(threadIdx.x & 7) * 8;
  if (row >= R) return;
  const int l = (int)(row % L);
  const float* xr = x + (long)c * R + (row - l);
  const float xm = l >= 1 ? xr[l - 1] : 0.f, x0 = xr[l], xp = l + 1 < L ? xr[l + 1] : 0.f;
  const float* pe = pp + pe_off + l * 64 + o0;
  float v[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const f4v w = *(const f4v*)(wsb + 4 * (o0 + e));
    float s = w[3] + pe[e];  // (same operation order as the composite: bias + pe, then the taps)
    if (l >= 1) s += w[0] * xm;
    s += w[1] * x0;
    if (l + 1 < L) s += w[2] * xp;
    v[e] = s;
  }
  *(u32x4*)(h + ((long)c * R + row) * 64 + o0) = u32x4{pk2(v[0], v[1]), pk2(v[2], v[3]), pk2(v[4], v[5]), pk2(v[6], v[7])};
}

// mean over L of the last layer's rows -> pooled [c][b][64] fp32 (fixed-order sums): 32 row groups x 8 lanes of 8
// channels (16-byte loads, two rows per group in flight)
__global__ void __launch_bounds__(256) k_har_pool(const u16* __restrict__ y, int L, float* __restrict__ out) {
  __shared__ f4v part[32][16];
  const int cb = blockIdx.x, j8 = threadIdx.x & 7, rg = threadIdx.x >> 3;
  const u16* base = y + (long)cb * L * 64 + 8 * j8;
  f4v s0 = Z4, s1 = Z4;
  auto add = [&](u32x4 u) {
    s0[0] += __uint_as_float(u[0] << 16);
    s0[1] += __uint_as_float(u[0] & 0xFFFF0000u);
    s0[2] += __uint_as_float(u[1] << 16);
    s0[3] += __uint_as_float(u[1] & 0xFFFF0000u);
    s1[0] += __uint_as_float(u[2] << 16);
    s1[1] += __uint_as_float(u[2] & 0xFFFF0000u);
    s1[2] += __uint_as_float(u[3] << 16);
    s1[3] += __uint_as_float(u[3] & 0xFFFF0000u);
  };
  int l = rg;
  for (; l + 32 < L; l += 64) {
    const u32x4 a = *(const u32x4*)(base + (long)l * 64), b = *(const u32x4*)(base + (long)(l + 32) * 64);
    add(a);
    add(b);
  }
  if (l < L) add(*(const u32x4*)(base + (long)l * 64));
  part[rg][2 * j8] = s0;
  part[rg][2 * j8 + 1] = s1;
  __syncthreads();
  if (threadIdx.x < 16) {
    const int j4 = threadIdx.x;
    f4v t = part[0][j4];
    for (int k = 1; k < 32; ++k) t += part[k][j4];
    *(f4v*)(out + (long)cb * 64 + 4 * j4) = t * (1.f / (float)L);
  }
}

// =================================================================================== q | k | v
__global__ void __launch_bounds__(NTF) k_har_qkv(AflHarQkv a) {
  extern __shared__ __attribute__((aligned(16))) uchar smem[];
  constexpr int IMG = 0, VEC = 192 * LDK64;
  const int c = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4;
  const float* pp = a.params + (long)c * a.P;
  build_img<false>(smem, IMG, LDK64, pp + a.w_off, 192, 64);
  load_vec(smem, VEC, pp + a.b_off, 192);
  __syncthreads();
  const long R = (long)a.B * a.L;
  const int ntiles = (int)((R + 15) / 16);
  for (int t = blockIdx.x * NWF + wave; t < ntiles; t += gridDim.x * NWF) {
    const long r = 16L * t + (lane & 15);
    const bool ok = r < R;
    const u16* xr = a.x + ((long)c * R + (ok ? r : 0)) * 64;
    const s8v b0 = ldx8(xr, 0, g, ok), b1 = ldx8(xr, 1, g, ok);
    const int b = (int)(r / a.L), l = (int)(r - (long)b * a.L);
#pragma unroll
    for (int T = 0; T < 12; ++T) {
      f4v acc = mma(wfrag(smem + IMG, LDK64, T, 0, lane), b0, Z4);
      acc = mma(wfrag(smem + IMG, LDK64, T, 1, lane), b1, acc);
      const f4v bv = *(const LDS_AS f4v*)(smem + VEC + (16 * T + 4 * g) * 4);
      const float sc = T < 4 ? a.qscale : 1.f;
      const float v0 = (acc[0] + bv[0]) * sc, v1 = (acc[1] + bv[1]) * sc, v2 = (acc[2] + bv[2]) * sc,
                  v3 = (acc[3] + bv[3]) * sc;
      if (ok) {
        const int which = T >> 2, h = T & 3;
        u16* dst = a.qkv + ((((long)c * a.B + b) * NH + h) * 3 + which) * (long)a.Lp * DH + (long)l * DH + 4 * g;
        *(u32x2v*)dst = u32x2v{pk2(v0, v1), pk2(v2, v3)};
      }
    }
  }
}

// =================================================================================== post-attention pass
// LDS map (bytes): Wo (natural K) | W1 (pcol) | W2 (pcol, K 256) | fp32 vectors
constexpr int PF_WO = 0, PF_W1 = PF_WO + 64 * LDK64, PF_W2 = PF_W1 + 256 * LDK64, PF_VEC = PF_W2 + 64 * LDK256;
enum { V_BO = 0, V_G1 = 64, V_BE1 = 128, V_B1 = 192, V_B2 = 448, V_G2 = 512, V_BE2 = 576, V_N = 640 };
constexpr int PF_SMEM = PF_VEC + V_N * 4;

__device__ void post_vectors(uchar* smem, int vec, const float* pp, const AflHarLayerW& w) {
  load_vec(smem, vec + V_BO * 4, pp + w.ob, 64);
  load_vec(smem, vec + V_G1 * 4, pp + w.n1w, 64);
  load_vec(smem, vec + V_BE1 * 4, pp + w.n1b, 64);
  load_vec(smem, vec + V_B1 * 4, pp + w.l1b, 256);
  load_vec(smem, vec + V_B2 * 4, pp + w.l2b, 64);
  load_vec(smem, vec + V_G2 * 4, pp + w.n2w, 64);
  load_vec(smem, vec + V_BE2 * 4, pp + w.n2b, 64);
}

__global__ void __launch_bounds__(NTP) k_har_post(AflHarPost a) {
  extern __shared__ __attribute__((aligned(16))) uchar smem[];
  const int c = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4;
  const float* pp = a.params + (long)c * a.P;
  build_img<false>(smem, PF_WO, LDK64, pp + a.w.ow, 64, 64);
  build_img<true>(smem, PF_W1, LDK64, pp + a.w.l1w, 256, 64);
  build_img<true>(smem, PF_W2, LDK256, pp + a.w.l2w, 64, 256);
  post_vectors(smem, PF_VEC, pp, a.w);
  __syncthreads();
  const uchar* vec = smem + PF_VEC;
  const uint32_t k1 = dkey(a.d1, c), kf_ = dkey(a.df, c), k2 = dkey(a.d2, c);
  const long R = a.R;
  const int ntiles = (int)((R + 15) / 16);
  for (int t = blockIdx.x * NWP + wave; t < ntiles; t += gridDim.x * NWP) {
    const long r = 16L * t + (lane & 15);
    const bool ok = r < R;
    const long row = (long)c * R + (ok ? r : 0);
    // ---- a = Wo . o + bo, dropout1, residual, LayerNorm 1
    float s1[16];
    uint32_t m1[1] = {0xFFFFFFFFu};
    {
      const u16* orow = a.o + row * 64;
      const s8v o0 = ldx8(orow, 0, g, ok), o1 = ldx8(orow, 1, g, ok);
      float xres[16], bo[16];
      ldt16(xres, a.x + row * 64, g, ok);
      vec16(bo, vec + V_BO * 4, g);
      if (a.d1.thr16) keep_bits<4>(m1, k1, a.d1.layer, (uint32_t)r, g, a.d1.thr16);
      const float inv1 = a.d1.thr16 ? a.d1.inv_keep : 1.f;
#pragma unroll
      for (int T = 0; T < 4; ++T) {
        f4v acc = mma(wfrag(smem + PF_WO, LDK64, T, 0, lane), o0, Z4);
        acc = mma(wfrag(smem + PF_WO, LDK64, T, 1, lane), o1, acc);
#pragma unroll
        for (int i = 0; i < 4; ++i) s1[4 * T + i] = xres[4 * T + i] + kf(acc[i] + bo[4 * T + i], m1, 4 * T + i, inv1);
      }
    }
    const float rstd1 = ln_fwd2(s1);  // s1 := xhat1
    if (ok) {
      stt16(a.xh1 + row * 64, s1, g);
      if (g == 0) a.rs[row * 2] = rstd1;
    }
    float h1[16];
    {
      float gm[16], bt[16];
      vec16(gm, vec + V_G1 * 4, g);
      vec16(bt, vec + V_BE1 * 4, g);
      affine2(h1, s1, gm, bt);
    }
    // ---- FFN, two tiles at a time: f = dropout(relu(W1 . h1 + b1)) for features of tiles 2s, 2s + 1 is
    //      exactly linear2's B fragment of k-step s, consumed at once (the 256-wide activation is never
    //      materialised), then y = W2 . f + b2, dropout2, residual
    float s2[16];
    uint32_t mf[2] = {0xFFFFFFFFu, 0xFFFFFFFFu}, m2[1] = {0xFFFFFFFFu};
    {
      const s8v b0 = bfrag(h1, 0), b1 = bfrag(h1, 1);
      if (a.df.thr16) ffn_bits(mf, kf_, a.df.layer, (uint32_t)r, g, a.df.thr16);
      const float invf = a.df.thr16 ? a.df.inv_keep : 1.f;
      f4v acc2[4] = {Z4, Z4, Z4, Z4};
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        sb();
        float fp[8];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int T = 2 * s + u;
          f4v acc = mma(wfrag(smem + PF_W1, LDK64, T, 0, lane), b0, Z4);
          acc = mma(wfrag(smem + PF_W1, LDK64, T, 1, lane), b1, acc);
          const f4v bb = *(const LDS_AS f4v*)(vec + (V_B1 + 16 * T + 4 * g) * 4);
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float z = acc[i] + bb[i];
            fp[4 * u + i] = kf(z > 0.f ? z : 0.f, mf, 4 * T + i, invf);
          }
        }
        const s8v bf = pk8(fp[0], fp[1], fp[2], fp[3], fp[4], fp[5], fp[6], fp[7]);
#pragma unroll
        for (int T = 0; T < 4; ++T) acc2[T] = mma(wfrag(smem + PF_W2, LDK256, T, s, lane), bf, acc2[T]);
      }
      sb();
      float b2[16];
      vec16(b2, vec + V_B2 * 4, g);
      if (a.d2.thr16) keep_bits<4>(m2, k2, a.d2.layer, (uint32_t)r, g, a.d2.thr16);
      const float inv2 = a.d2.thr16 ? a.d2.inv_keep : 1.f;
#pragma unroll
      for (int T = 0; T < 4; ++T)
#pragma unroll
        for (int i = 0; i < 4; ++i) s2[4 * T + i] = h1[4 * T + i] + kf(acc2[T][i] + b2[4 * T + i], m2, 4 * T + i, inv2);
    }
    const float rstd2 = ln_fwd2(s2);
    if (ok && a.kbits)  // the keep bits for the backward (one 16-byte store per lane: no hashing there)
      *(u32x4*)(a.kbits + (row * 4 + g) * 4) = u32x4{(m1[0] & 0xFFFFu) | (m2[0] << 16), mf[0], mf[1], 0u};
    if (ok) {
      stt16(a.xh2 + row * 64, s2, g);
      if (g == 0) a.rs[row * 2 + 1] = rstd2;
      float gm[16], bt[16], y[16];
      vec16(gm, vec + V_G2 * 4, g);
      vec16(bt, vec + V_BE2 * 4, g);
      affine2(y, s2, gm, bt);
      stt16(a.y + row * 64, y, g);
    }
  }
}

// =================================================================================== attention
// One workgroup per (client, sample, head) over the head-major block [3][Lp][16] (q | k | v).
// K / V / Q / dO are staged as row-major [rows][16] bf16 images (32-byte rows); the 8-byte chunk p of row r
// sits at chunk p ^ ((r >> 2) & 3) (rch), so the 16 rows of one A-operand read (rows r0..r0+15, one chunk)
// spread over all banks in both the single and the compiler-paired read forms, while the transposed reads
// (4 consecutive rows x 4 chunks) only permute chunks within their rows.
// Transposed operands (V^T for O += V^T P^T, K^T for dQ, Q^T / dO^T for dK / dV) come straight from these
// row-major images through ds_read_b64_tr_b16: lane i of a 16-lane group gets column i of 4 rows whose
// order the lanes' addresses choose — the permuted key order of the score fragments — so no transposed
// copy is staged.  Scores stay in the log2 domain (one v_exp_f32 per probability; q carries log2(e) / 4).
constexpr float LOG2E = 1.4426950408889634f;
constexpr int AT_WAVES = 12, AT_NT = 64 * AT_WAVES;
typedef __bf16 bf8v __attribute__((ext_vector_type(8)));

__device__ __forceinline__ int rch(int r, int p) { return r * 32 + ((p ^ ((r >> 2) & 3)) << 3); }
__device__ __forceinline__ f4v mfma16(s4v a, s4v b, f4v c) { return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0); }
__device__ __forceinline__ f4v mfma32(s8v a, s8v b, f4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf8v, a), __builtin_bit_cast(bf8v, b), c, 0, 0, 0);
}
// One 8-byte fragment row.  The chunk swizzle p ^ ((r >> 2) & 3) keeps every access pattern of these images
// conflict-free: 16 consecutive rows of one chunk hit 16 distinct bank pairs mod 32 (the ds_read2st64_b64 /
// ds_read2_b64 the compiler pairs two such reads into: 16-lane groups, (a / 4) mod 32), two chunks of them 32
// distinct pairs mod 64 (ds_read_b64: 32-lane halves), and the transposed reads (4 rows x 4 chunks) permute the
// chunks within a row quad.  (Round 4 swizzled by row bit 3 only: rows r and r + 4 shared banks in the paired
// form, 3.63 / 1.97 conflict cycles per LDS instruction in dQ / the forward; forcing unpaired reads instead cost
// an address computation per read, -5 % HAR rounds/s.)
__device__ __forceinline__ s4v lds4(const uchar* img, int r, int p) { return *(const LDS_AS s4v*)(img + rch(r, p)); }
// transposed fragment: lane (q, p) of group g addresses row base(g) + q, chunk p -> column (lane & 15) of the 4 rows
__device__ __forceinline__ s8v trfrag(const uchar* img, int base0, int base1, int lane) {
  const int i = lane & 15;
  return cat44(tr16(img + rch(base0 + (i >> 2), i & 3)), tr16(img + rch(base1 + (i >> 2), i & 3)));
}
__device__ __forceinline__ s8v pack8f(const float* v) {
  return pk8(v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7]);
}
// rows [0, n) of a bf16 [n][16] source with row stride `stride` elements -> swizzled image (16 B per step)
__device__ void stage16(uchar* img, const u16* __restrict__ src, long stride, int n, int nvalid) {
  for (int e = threadIdx.x; e < 2 * n; e += blockDim.x) {
    const int r = e >> 1, hf = e & 1;
    const u32x4 v = r < nvalid ? *(const u32x4*)(src + (long)r * stride + 8 * hf) : u32x4{0u, 0u, 0u, 0u};
    // chunks 2 hf, 2 hf + 1 land at (2 hf) ^ sw, (2 hf + 1) ^ sw: one 16-byte pair, halves swapped when sw is odd
    const int sw = (r >> 2) & 3;
    const u32x4 w = (sw & 1) ? u32x4{v[2], v[3], v[0], v[1]} : v;
    *(LDS_AS u32x4*)(img + r * 32 + (((2 * hf) ^ (sw & 2)) << 3)) = w;
  }
}
__device__ __forceinline__ float max_x16_x32(float a) {
  auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(a), false, false);
  a = fmaxf(__uint_as_float(p[0]), __uint_as_float(p[1]));
  p = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(a), false, false);
  return fmaxf(__uint_as_float(p[0]), __uint_as_float(p[1]));
}
__device__ __forceinline__ float sum_x16_x32(float a) {
  auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(a), false, false);
  a = __uint_as_float(p[0]) + __uint_as_float(p[1]);
  p = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(a), false, false);
  return __uint_as_float(p[0]) + __uint_as_float(p[1]);
}
// Probability dropout (masks.keep_rc): a strong hash per row (attn_hr) and per column pair (attn_hc, an LDS
// table per workgroup) combined by xor and one multiply-xorshift round; 16 bits per column.  Only the forward
// hashes: it stores the flags as 64-bit ballot words (AflHarAttn::mask) that the backward kernels read back.
// Kept probabilities are NOT scaled here: 1/(1-p) is folded into O (forward), dV and dP (backward).
__device__ __forceinline__ uint32_t attn_hr(uint32_t key, uint32_t layer, uint32_t r) {
  return afl_hash4(key, layer, r, 0xFFFFFFFFu);
}
__device__ __forceinline__ uint32_t attn_hc(uint32_t key, uint32_t layer, uint32_t cp) {
  return afl_hash4(key ^ 0xA5A5A5A5u, layer, 0u, cp);
}
// One multiply-xorshift round (3 vector instructions per mix: xor, v_mul_lo_u32, xor with the high half):
// the draw is VALU-issue-bound and a second round measured as pure cost.  hr and hc are full-avalanche hashes;
// the product's carries break the xor structure of hr ^ hc (every output bit's four-corner parity is balanced,
// keep rate / halves / rectangles pinned by tests/test_programs.py).
__device__ __forceinline__ uint32_t attn_mix(uint32_t hr, uint32_t hc) {
  uint32_t x = (hr ^ hc) * 0x7FEB352Du;
  return x ^ (x >> 16);
}
// keep flags of keys kb .. kb+3 (kb even) of the row with hash hr: pairs kb/2, kb/2 + 1 from the LDS table
__device__ __forceinline__ void keep4(const LDS_AS uint32_t* HC, uint32_t hr, int kb, uint32_t thr, bool* k) {
  const u32x2v hc = *(const LDS_AS u32x2v*)(HC + (kb >> 1));
  const uint32_t x0 = attn_mix(hr, hc[0]), x1 = attn_mix(hr, hc[1]);
  k[0] = (x0 & 0xFFFFu) >= thr;
  k[1] = (x0 >> 16) >= thr;
  k[2] = (x1 & 0xFFFFu) >= thr;
  k[3] = (x1 >> 16) >= thr;
}
__device__ void fill_hc(LDS_AS uint32_t* HC, int npairs, uint32_t key, uint32_t layer) {
  for (int e = threadIdx.x; e < npairs; e += blockDim.x) HC[e] = attn_hc(key, layer, (uint32_t)e);
}

// lanes 2j / 2j + 1 of mw <- low / high half of keep word j (j = 0 .. 15), in two asm blocks of 16 writelanes
__device__ __forceinline__ void keep_words(uint32_t& mw, const uint32_t (&bl)[16], const uint32_t (&bh)[16]) {
  asm("s_nop 4\n\t" "v_writelane_b32 %0, %1, 0\n\t""v_writelane_b32 %0, %2, 1\n\t""v_writelane_b32 %0, %3, 2\n\t""v_writelane_b32 %0, %4, 3\n\t""v_writelane_b32 %0, %5, 4\n\t""v_writelane_b32 %0, %6, 5\n\t""v_writelane_b32 %0, %7, 6\n\t""v_writelane_b32 %0, %8, 7\n\t""v_writelane_b32 %0, %9, 8\n\t""v_writelane_b32 %0, %10, 9\n\t""v_writelane_b32 %0, %11, 10\n\t""v_writelane_b32 %0, %12, 11\n\t""v_writelane_b32 %0, %13, 12\n\t""v_writelane_b32 %0, %14, 13\n\t""v_writelane_b32 %0, %15, 14\n\t""v_writelane_b32 %0, %16, 15\n\t"
      : "+v"(mw)
      : "s"(bl[0]), "s"(bh[0]), "s"(bl[1]), "s"(bh[1]), "s"(bl[2]), "s"(bh[2]), "s"(bl[3]), "s"(bh[3]), "s"(bl[4]), "s"(bh[4]), "s"(bl[5]), "s"(bh[5]), "s"(bl[6]), "s"(bh[6]), "s"(bl[7]), "s"(bh[7]));
  asm("s_nop 4\n\t" "v_writelane_b32 %0, %1, 16\n\t""v_writelane_b32 %0, %2, 17\n\t""v_writelane_b32 %0, %3, 18\n\t""v_writelane_b32 %0, %4, 19\n\t""v_writelane_b32 %0, %5, 20\n\t""v_writelane_b32 %0, %6, 21\n\t""v_writelane_b32 %0, %7, 22\n\t""v_writelane_b32 %0, %8, 23\n\t""v_writelane_b32 %0, %9, 24\n\t""v_writelane_b32 %0, %10, 25\n\t""v_writelane_b32 %0, %11, 26\n\t""v_writelane_b32 %0, %12, 27\n\t""v_writelane_b32 %0, %13, 28\n\t""v_writelane_b32 %0, %14, 29\n\t""v_writelane_b32 %0, %15, 30\n\t""v_writelane_b32 %0, %16, 31\n\t"
      : "+v"(mw)
      : "s"(bl[8]), "s"(bh[8]), "s"(bl[9]), "s"(bh[9]), "s"(bl[10]), "s"(bh[10]), "s"(bl[11]), "s"(bh[11]), "s"(bl[12]), "s"(bh[12]), "s"(bl[13]), "s"(bh[13]), "s"(bl[14]), "s"(bh[14]), "s"(bl[15]), "s"(bh[15]));
}

template <bool DROP>
__global__ void __launch_bounds__(AT_NT) k_har_attn_fwd(AflHarAttn a) {
  extern __shared__ __attribute__((aligned(16))) uchar smem[];
  const int Lp = a.Lp, L = a.L;
  uchar* Ki = smem;
  uchar* Vi = smem + Lp * 32;
  LDS_AS uint32_t* HC = (LDS_AS uint32_t*)(smem + 2 * Lp * 32);
  const int cbh = blockIdx.x, h = cbh % NH, cb = cbh / NH, c = cb / a.B, b = cb - c * a.B;
  const u16* blk = a.qkv + (long)cbh * 3 * Lp * DH;
  const uint32_t key = DROP ? dkey(a.drop, c) : 0u;
  stage16(Ki, blk + (long)Lp * DH, DH, Lp, Lp);
  stage16(Vi, blk + 2L * Lp * DH, DH, Lp, Lp);
  if (DROP) fill_hc(HC, Lp / 2, key, a.drop.layer);
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, li = lane & 15;
  const uint32_t drow0 = (uint32_t)((b * NH + h) * L);
  const long orow0 = (long)c * a.B * L + (long)b * L;
  const int nkc = Lp >> 6;
  uint32_t* mrow = DROP ? (uint32_t*)(a.mask + (long)cbh * AFL_HAR_MASK_WORDS(Lp)) : nullptr;
  for (int q0 = wave * 16; q0 < Lp; q0 += 16 * AT_WAVES) {
    const int q = q0 + li;
    const s4v qf = *(const s4v*)(blk + (long)q * DH + 4 * g);
    const uint32_t hr = DROP ? attn_hr(key, a.drop.layer, drow0 + q) : 0u;
    float m = -INFINITY, l = 0.f;
    f4v o = Z4;
    // one 64-key chunk; only the last (partial) chunk masks keys >= L (peeled: no per-chunk compare/select)
    auto chunk = [&](int kt, auto tail) {
      float s[16];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const f4v st = mfma16(lds4(Ki, kt + 16 * t + li, g), qf, Z4);
#pragma unroll
        for (int e = 0; e < 4; ++e) s[4 * t + e] = st[e];  // (q carries 1/4 * log2 e: already log2-domain)
      }
      if constexpr (decltype(tail)::value) {
#pragma unroll
        for (int j = 0; j < 16; ++j)
          if (kt + 16 * (j >> 2) + 4 * g + (j & 3) >= L) s[j] = -INFINITY;
      }
      float mx = s[0];
#pragma unroll
      for (int j = 1; j < 16; ++j) mx = fmaxf(mx, s[j]);
      const float mn = fmaxf(m, max_x16_x32(mx));
      const float alpha = __builtin_amdgcn_exp2f(m - mn);
      // (pairs: v_pk_add_f32 for the shift and the row sum)
      float pd[16];
      of2v ps2 = of2v{0.f, 0.f};
      const of2v mn2 = of2v{mn, mn};
#pragma unroll
      for (int j = 0; j < 16; j += 2) {
        const of2v d = of2v{s[j], s[j + 1]} - mn2;
        pd[j] = __builtin_amdgcn_exp2f(d[0]);
        pd[j + 1] = __builtin_amdgcn_exp2f(d[1]);
        ps2 += of2v{pd[j], pd[j + 1]};
      }
      const float ps = ps2[0] + ps2[1];
      if (DROP) {
        // keep word (t, e) = ballot of the flags of keys kt + 16t + 4g + e over the wave (bit = lane): lanes 0..31
        // of mw collect the chunk's 16 words, stored for both backward kernels (no hashing there)
        uint32_t mw = 0u, bl[16], bh[16];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          bool k4[4];
          keep4(HC, hr, kt + 16 * t + 4 * g, a.drop.thr16, k4);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            pd[4 * t + e] = k4[e] ? pd[4 * t + e] : 0.f;
            const uint64_t bw = __builtin_amdgcn_ballot_w64(k4[e]);
            bl[4 * t + e] = (uint32_t)bw;
            bh[4 * t + e] = (uint32_t)(bw >> 32);
          }
        }
        // v_writelane reading an SGPR that a VALU compare has just written needs wait states the compiler does
        // not insert inside inline asm (measured: ~5 % of the low-half flags wrong without them): every ballot is
        // computed before the block, and the block opens with s_nop 4
        keep_words(mw, bl, bh);
        if (lane < 32) mrow[(long)((q0 >> 4) * nkc + (kt >> 6)) * 32 + lane] = mw;
      }
      l = l * alpha + sum_x16_x32(ps);
      m = mn;
      o *= alpha;
      o = mfma32(trfrag(Vi, kt + 4 * g, kt + 16 + 4 * g, lane), pack8f(pd), o);
      o = mfma32(trfrag(Vi, kt + 32 + 4 * g, kt + 48 + 4 * g, lane), pack8f(pd + 8), o);
    };
    int kt = 0;
    for (; kt + 64 <= L; kt += 64) chunk(kt, std::false_type{});
    if (kt < L) chunk(kt, std::true_type{});
    if (q < L) {
      const float inv = (DROP ? a.drop.inv_keep : 1.f) / l;
      *(u32x2v*)(a.o + (orow0 + q) * D + h * DH + 4 * g) = u32x2v{pk2(o[0] * inv, o[1] * inv), pk2(o[2] * inv, o[3] * inv)};
    }
    if (g == 0) a.lse2[(long)cbh * Lp + q] = q < L ? m + __log2f(l) : INFINITY;
  }
}

// ---- dK / dV: each wave owns 16 keys and sweeps the queries (32 per step) ----
// A lane holds one key (lane & 15) x 4 queries.  The dropout flags are the forward's keep words (no hashing
// in either backward kernel): one dword load per lane and query tile, one bit per element.
template <bool DROP>
__global__ void __launch_bounds__(AT_NT) k_har_attn_bwd_kv(AflHarAttn a) {
  extern __shared__ __attribute__((aligned(16))) uchar smem[];
  const int Lp = a.Lp, L = a.L;
  uchar* Qi = smem;
  uchar* Di = smem + Lp * 32;
  LDS_AS float* LS = (LDS_AS float*)(smem + 2 * Lp * 32);
  LDS_AS float* DL = LS + Lp;
  const int cbh = blockIdx.x, h = cbh % NH, cb = cbh / NH, c = cb / a.B, b = cb - c * a.B;
  const u16* blk = a.qkv + (long)cbh * 3 * Lp * DH;
  const long orow0 = (long)c * a.B * L + (long)b * L;
  stage16(Qi, blk, DH, Lp, Lp);
  stage16(Di, a.dout + orow0 * D + h * DH, D, Lp, L);
  for (int e = threadIdx.x; e < Lp; e += blockDim.x) {
    LS[e] = a.lse2[(long)cbh * Lp + e];
    DL[e] = e < L ? a.delta[(long)cbh * Lp + e] : 0.f;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, li = lane & 15;
  const float ik = DROP ? a.drop.inv_keep : 1.f;
  const long wq = (long)(Lp >> 6) * 16;  // keep words per query tile
  for (int k0 = wave * 16; k0 < Lp; k0 += 16 * AT_WAVES) {
    const int kk = k0 + li;
    const s4v kf = *(const s4v*)(blk + (long)(Lp + kk) * DH + 4 * g);
    const s4v vf = *(const s4v*)(blk + (long)(2 * Lp + kk) * DH + 4 * g);
    // the forward's keep word of key kk for query tile T: [T][kk >> 6][(kk >> 4) & 3][kk & 3]; the flags of
    // queries 16T + 4g + e sit at bits 16((kk >> 2) & 3) + 4g + e: one dword per (lane, tile), bit e of a nibble
    const int sh = 16 * ((kk >> 2) & 3) + 4 * g;
    const uint32_t* mw = DROP ? (const uint32_t*)(a.mask + (long)cbh * AFL_HAR_MASK_WORDS(Lp) + (kk >> 6) * 16 +
                                                  ((kk >> 4) & 3) * 4 + (kk & 3)) + (sh >> 5)
                              : nullptr;
    f4v dkT = Z4, dvT = Z4;
    // keep dwords of the two query tiles of a step, loaded one step ahead
    uint32_t wn[2] = {0xFFFFFFFFu, 0xFFFFFFFFu};
    if (DROP) {
      wn[0] = mw[0];
      wn[1] = mw[wq * 2];
    }
    for (int q0 = 0; q0 < L; q0 += 32) {
      float pdv[8], dsv[8];
      const uint32_t wc[2] = {wn[0], wn[1]};
      if (DROP && q0 + 32 < L) {
        wn[0] = mw[(long)((q0 + 32) >> 4) * wq * 2];
        wn[1] = mw[(long)((q0 + 48) >> 4) * wq * 2];
      }
#pragma unroll
      for (int qs = 0; qs < 2; ++qs) {
        const int qb = q0 + 16 * qs;
        const f4v s = mfma16(lds4(Qi, qb + li, g), kf, Z4);
        const f4v dp = mfma16(lds4(Di, qb + li, g), vf, Z4);
        const f4v l4 = *(const LDS_AS f4v*)(LS + qb + 4 * g);
        const f4v d4 = *(const LDS_AS f4v*)(DL + qb + 4 * g);
        const uint32_t wd = wc[qs];
#pragma unroll
        for (int e = 0; e < 4; e += 2) {
          // (keys >= L need no mask: a lane's values only reach its own key's dK / dV column, never stored)
          // (pairs: v_pk_add / v_pk_fma / v_pk_mul for the shift, dP - Delta and the product)
          const of2v sh2 = of2v{s[e], s[e + 1]} - of2v{l4[e], l4[e + 1]};
          const of2v p = of2v{__builtin_amdgcn_exp2f(sh2[0]), __builtin_amdgcn_exp2f(sh2[1])};
          // keep flag -> all-ones / zero word (sign-extended one-bit field)
          const uint32_t km0 = DROP ? (uint32_t)__builtin_amdgcn_sbfe((int)wd, (sh & 31) + e, 1) : 0xFFFFFFFFu;
          const uint32_t km1 = DROP ? (uint32_t)__builtin_amdgcn_sbfe((int)wd, (sh & 31) + e + 1, 1) : 0xFFFFFFFFu;
          pdv[4 * qs + e] = __uint_as_float(__float_as_uint(p[0]) & km0);  // (x 1/(1-p) on dV at the end)
          pdv[4 * qs + e + 1] = __uint_as_float(__float_as_uint(p[1]) & km1);
          const of2v dpm = of2v{__uint_as_float(__float_as_uint(dp[e]) & km0), __uint_as_float(__float_as_uint(dp[e + 1]) & km1)};
          const of2v ds = p * (dpm * of2v{ik, ik} - of2v{d4[e], d4[e + 1]});
          dsv[4 * qs + e] = ds[0];
          dsv[4 * qs + e + 1] = ds[1];
        }
      }
      // dV^T[d][key] += dO^T[d][q] Pd[q][key] ; dK^T[d][key] += Q_s^T[d][q] dS[q][key] (query order permuted)
      dvT = mfma32(trfrag(Di, q0 + 4 * g, q0 + 16 + 4 * g, lane), pack8f(pdv), dvT);
      dkT = mfma32(trfrag(Qi, q0 + 4 * g, q0 + 16 + 4 * g, lane), pack8f(dsv), dkT);
    }
    if (kk < L) {  // lane: d = 4g + e of key kk
      u16* dk = a.dqkv + ((long)cbh * 3 + 1) * Lp * DH + (long)kk * DH + 4 * g;
      u16* dv = a.dqkv + ((long)cbh * 3 + 2) * Lp * DH + (long)kk * DH + 4 * g;
      constexpr float iq = 1.f / LOG2E;  // dK = dS^T (q / 4) and the image holds q log2(e) / 4
      *(u32x2v*)dk = u32x2v{pk2(dkT[0] * iq, dkT[1] * iq), pk2(dkT[2] * iq, dkT[3] * iq)};
      *(u32x2v*)dv = u32x2v{pk2(dvT[0] * ik, dvT[1] * ik), pk2(dvT[2] * ik, dvT[3] * ik)};
    }
  }
}

// ---- dQ: each wave owns 16 queries and sweeps the keys (recomputing S and dP; no atomics) ----
// x where bit `lane` of the wave-uniform 64-bit keep word m is set, else 0 (one v_cndmask on an SGPR-pair mask).
// Not inline asm: the compiler's hazard recognizer does not pad an asm VALU that reads an MFMA result, and the
// v_cndmask read the dP accumulator a few cycles after its MFMA issued (garbage, NaN dQ in whole 16-row tiles,
// nondeterministically); inverse_ballot gives the same single instruction with the wait states inserted.
__device__ __forceinline__ float keep_sel(uint64_t m, float x) { return __builtin_amdgcn_inverse_ballot_w64(m) ? x : 0.f; }
template <bool DROP>
__global__ void __launch_bounds__(AT_NT) k_har_attn_bwd_dq(AflHarAttn a) {
  extern __shared__ __attribute__((aligned(16))) uchar smem[];
  const int Lp = a.Lp, L = a.L;
  uchar* Ki = smem;
  uchar* Vi = smem + Lp * 32;
  const int cbh = blockIdx.x, h = cbh % NH, cb = cbh / NH, c = cb / a.B, b = cb - c * a.B;
  const u16* blk = a.qkv + (long)cbh * 3 * Lp * DH;
  const long orow0 = (long)c * a.B * L + (long)b * L;
  stage16(Ki, blk + (long)Lp * DH, DH, Lp, Lp);
  stage16(Vi, blk + 2L * Lp * DH, DH, Lp, Lp);
  __syncthreads();
  const int lane = threadIdx.x & 63, g = lane >> 4, li = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const float ik = DROP ? a.drop.inv_keep : 1.f;
  const int nkc = Lp >> 6;
  const uint32_t* mblk = DROP ? (const uint32_t*)(a.mask + (long)cbh * AFL_HAR_MASK_WORDS(Lp)) : nullptr;
  for (int q0 = wave * 16; q0 < L; q0 += 16 * AT_WAVES) {
    const int q = q0 + li;
    const bool qok = q < L;
    const s4v qf = *(const s4v*)(blk + (long)q * DH + 4 * g);
    const s4v df = qok ? *(const s4v*)(a.dout + (orow0 + q) * D + h * DH + 4 * g) : s4v{0, 0, 0, 0};
    const float ls = a.lse2[(long)cbh * Lp + q];
    const float dl = qok ? a.delta[(long)cbh * Lp + q] : 0.f;
    // the forward's words of this query tile: element j of the 32-key step at kt is word 4((kt & 63) >> 4) + j of
    // chunk kt >> 6, bit = lane (same lane <-> (query, key) map as the forward)
    const uint32_t* mt = DROP ? mblk + (long)(q0 >> 4) * nkc * 32 : nullptr;
    f4v acc = Z4;
    auto step = [&](int kt, auto tail) {
      const f4v s0 = mfma16(lds4(Ki, kt + li, g), qf, Z4);
      const f4v s1 = mfma16(lds4(Ki, kt + 16 + li, g), qf, Z4);
      const f4v p0 = mfma16(lds4(Vi, kt + li, g), df, Z4);
      const f4v p1 = mfma16(lds4(Vi, kt + 16 + li, g), df, Z4);
      // the step's 8 keep words: wave-uniform vector loads made scalar with readfirstlane (a scalar s_load of
      // the same words read stale data from the scalar cache, which nothing invalidates between launches)
      uint64_t mw[8];
      if (DROP) {
        const uint32_t* w = mt + (kt >> 6) * 32 + ((kt & 63) >> 4) * 8;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint32_t lo = __builtin_amdgcn_readfirstlane(w[2 * j]), hi = __builtin_amdgcn_readfirstlane(w[2 * j + 1]);
          mw[j] = ((uint64_t)hi << 32) | lo;
        }
      }
      float ds[8];
      const of2v ls2 = of2v{ls, ls}, dl2 = of2v{dl, dl}, ik2 = of2v{ik, ik};
#pragma unroll
      for (int j = 0; j < 8; j += 2) {  // (pairs: v_pk_add / v_pk_fma / v_pk_mul)
        const of2v sv = j < 4 ? of2v{s0[j], s0[j + 1]} : of2v{s1[j - 4], s1[j - 3]};
        of2v dp = j < 4 ? of2v{p0[j], p0[j + 1]} : of2v{p1[j - 4], p1[j - 3]};
        if (DROP) dp = of2v{keep_sel(mw[j], dp[0]), keep_sel(mw[j + 1], dp[1])};
        const of2v sh2 = sv - ls2;
        of2v p = of2v{__builtin_amdgcn_exp2f(sh2[0]), __builtin_amdgcn_exp2f(sh2[1])};
        if constexpr (decltype(tail)::value) {  // keys >= L: last step only
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int kk = kt + (j + h < 4 ? 4 * g + j + h : 16 + 4 * g + j + h - 4);
            p[h] = kk < L ? p[h] : 0.f;
          }
        }
        const of2v d = p * (dp * ik2 - dl2);
        ds[j] = d[0];
        ds[j + 1] = d[1];
      }
      acc = mfma32(trfrag(Ki, kt + 4 * g, kt + 16 + 4 * g, lane), pack8f(ds), acc);
    };
    int kt = 0;
    for (; kt + 32 <= L; kt += 32) step(kt, std::false_type{});
    if (kt < L) step(kt, std::true_type{});
    if (qok) {  // d(q projection) = 1/4 d(q_s)
      u16* dq = a.dqkv + (long)cbh * 3 * Lp * DH + (long)q * DH + 4 * g;
      *(u32x2v*)dq = u32x2v{pk2(acc[0] * 0.25f, acc[1] * 0.25f), pk2(acc[2] * 0.25f, acc[3] * 0.25f)};
    }
  }
}

// =================================================================================== backward row passes
// dW operand tiles: [64 rows][64 bf16] XOR-swizzled (onchip.h t64), written 4 features per lane (st4) and read
// as MFMA operands with rows as K (tfrag, ds_read_b64_tr_b16).  A workgroup's 4 waves own fixed output
// tiles of every weight gradient and keep them in MFMA accumulators across all the row blocks the
// workgroup serves; the vector gradients (biases, LayerNorm) are per-lane column-sum registers.
constexpr int TILE = 64 * 128;
// LDS map of the post backward (bytes)
constexpr int PB_WO = 0, PB_W1 = PB_WO + 64 * LDK64, PB_W2 = PB_W1 + 256 * LDK64, PB_VEC = PB_W2 + 64 * LDK256B;
constexpr int PB_F = PB_VEC + V_N * 4;    // 4 tiles: f (dW2 operand), then d f (dW1 operand)
constexpr int PB_DF2 = PB_F + 4 * TILE;   // d f2
constexpr int PB_H1 = PB_DF2 + TILE;      // h1
constexpr int PB_DA = PB_H1 + TILE;       // d a (dropout1' of d s1)
constexpr int PB_O = PB_DA + TILE;        // attention output o
constexpr int PB_RED = PB_O + TILE;       // [4 waves][640] vector-gradient partials
constexpr int PB_SMEM = PB_RED + 4 * V_N * 4;
// gradient partial layout (floats): Wo | W1 | W2 | vectors in the V_* order
constexpr int G_WO = 0, G_W1 = 4096, G_W2 = G_W1 + 16384, G_VEC = G_W2 + 16384;
static_assert(G_VEC + V_N == AFL_HAR_POST_NG, "partial layout");

// per-lane column-sum accumulators: one feature per lane per 64-wide vector (colsum64 mapping)
__device__ __forceinline__ void csum_add(float& acc, const float (&x)[16], int lane) {
  float s;
  (void)colsum64(x, lane, s);
  acc += s;
}
__device__ __forceinline__ int csum_feature(int lane) {
  float x[16] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float s;
  return colsum64(x, lane, s);
}

__global__ void __launch_bounds__(NTR) k_har_post_bwd(AflHarPostB a) {
  extern __shared__ __attribute__((aligned(16))) uchar smem[];
  const int c = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6),
            g = lane >> 4, li = lane & 15;
  const float* pp = a.params + (long)c * a.P;
  build_img<true>(smem, PB_WO, LDK64, pp + a.w.ow, 64, 64);
  build_img<true>(smem, PB_W1, LDK64, pp + a.w.l1w, 256, 64);
  build_img<true>(smem, PB_W2, LDK256B, pp + a.w.l2w, 64, 256);
  post_vectors(smem, PB_VEC, pp, a.w);
  __syncthreads();
  const uchar* vec = smem + PB_VEC;
  const float inv1 = a.d1.thr16 ? a.d1.inv_keep : 1.f, invf = a.df.thr16 ? a.df.inv_keep : 1.f,
              inv2 = a.d2.thr16 ? a.d2.inv_keep : 1.f;
  const long R = a.R;
  const int nblk = (int)((R + 63) / 64);
  f4v aW2[16], aW1[16], aWo[4];
#pragma unroll
  for (int j = 0; j < 16; ++j) aW2[j] = aW1[j] = Z4;
#pragma unroll
  for (int j = 0; j < 4; ++j) aWo[j] = Z4;
  float cg2 = 0.f, cb2 = 0.f, cbf2 = 0.f, cbf[4] = {0.f, 0.f, 0.f, 0.f}, cg1 = 0.f, cb1 = 0.f, cbo = 0.f;
  const int rl = 16 * wave + li;  // this lane's row within a block
  // this lane's row inputs of one block; the NEXT block's are loaded while the current one computes
  struct In {
    f4v dy[4];
    u32x2v xh2[4], xh1[4], o[4];
    u32x4 kb;  // the forward's keep bits (all set without dropout)
    float rs1, rs2;
  };
  auto load = [&](int blk, In& in) {
    const long r = 64L * blk + rl;
    const bool ok = blk < nblk && r < R;
    const long row = (long)c * R + (ok ? r : 0);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      in.dy[t] = (ok && !a.dpool) ? *(const f4v*)(a.dy + row * 64 + 16 * t + 4 * g) : Z4;
      in.xh2[t] = ok ? *(const u32x2v*)(a.xh2 + row * 64 + 16 * t + 4 * g) : u32x2v{0u, 0u};
      in.xh1[t] = ok ? *(const u32x2v*)(a.xh1 + row * 64 + 16 * t + 4 * g) : u32x2v{0u, 0u};
      in.o[t] = ok ? *(const u32x2v*)(a.o + row * 64 + 16 * t + 4 * g) : u32x2v{0u, 0u};
    }
    in.kb = (ok && a.kbits) ? *(const u32x4*)(a.kbits + (row * 4 + g) * 4) : u32x4{~0u, ~0u, ~0u, ~0u};
    in.rs1 = ok ? a.rs[row * 2] : 0.f;
    in.rs2 = ok ? a.rs[row * 2 + 1] : 0.f;
  };
  auto unbf = [](float (&x)[16], const u32x2v (&u)[4]) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      x[4 * t] = __uint_as_float(u[t][0] << 16);
      x[4 * t + 1] = __uint_as_float(u[t][0] & 0xFFFF0000u);
      x[4 * t + 2] = __uint_as_float(u[t][1] << 16);
      x[4 * t + 3] = __uint_as_float(u[t][1] & 0xFFFF0000u);
    }
  };
  In cur;
  load(blockIdx.x, cur);
  for (int blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
    In nxt;
    load(blk + gridDim.x, nxt);
    // lane / wave made opaque per block: every LDS address is recomputed inside the iteration (hoisted out of
    // the loop, the per-lane swizzled addresses of all phases stayed live and spilled the accumulators)
    int ln_ = lane, wv_ = wave;
    opq(ln_, wv_);
    {
    const int lane = ln_, wave = wv_, g = ln_ >> 4, li = ln_ & 15, rl = 16 * wv_ + li;
    const long r = 64L * blk + rl;
    const bool ok = r < R;
    const long row = (long)c * R + (ok ? r : 0);
    // ---- LayerNorm 2 backward, dropout2'
    float dy[16], xh2[16], gm[16];
    if (a.dpool) {
      const int bb = (int)(r / a.L);
      const float* dp = a.dpool + ((long)c * a.B + (ok ? bb : 0)) * 64;
      const float il = 1.f / (float)a.L;
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) dy[4 * t + i] = ok ? dp[16 * t + 4 * g + i] * il : 0.f;
    } else {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        dy[4 * t] = cur.dy[t][0]; dy[4 * t + 1] = cur.dy[t][1]; dy[4 * t + 2] = cur.dy[t][2]; dy[4 * t + 3] = cur.dy[t][3];
      }
    }
    unbf(xh2, cur.xh2);
    const float rstd2 = cur.rs2;
    {
      float t2[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) t2[j] = dy[j] * xh2[j];
      csum_add(cg2, t2, lane);
      csum_add(cb2, dy, lane);
    }
    vec16(gm, vec + V_G2 * 4, g);
    float ds2[16];
    ln_bwd2(ds2, dy, xh2, rstd2, gm);
    float df2[16];
    {
      const uint32_t m2[1] = {cur.kb[0] >> 16};
#pragma unroll
      for (int j = 0; j < 16; ++j) df2[j] = kf(ds2[j], m2, j, inv2);
    }
    csum_add(cbf2, df2, lane);
    // ---- h1 and the FFN activation, recomputed; stage d f2 and f for dW2
    float xh1[16], h1[16];
    unbf(xh1, cur.xh1);
    const float rstd1 = cur.rs1;
    {
      float g1[16], b1[16];
      vec16(g1, vec + V_G1 * 4, g);
      vec16(b1, vec + V_BE1 * 4, g);
      affine2(h1, xh1, g1, b1);
    }
    const uint32_t mf[2] = {cur.kb[1], cur.kb[2]};
    uint32_t relu[2] = {0u, 0u};
    {
      const s8v b0 = bfrag(h1, 0), b1 = bfrag(h1, 1);
#pragma unroll
      for (int T = 0; T < 16; ++T) {
        if ((T & 3) == 0) sb();
        f4v acc = mma(wfrag(smem + PB_W1, LDK64, T, 0, lane), b0, Z4);
        acc = mma(wfrag(smem + PB_W1, LDK64, T, 1, lane), b1, acc);
        const f4v bb = *(const LDS_AS f4v*)(vec + (V_B1 + 16 * T + 4 * g) * 4);
        float fv[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float z = acc[i] + bb[i];
          const int j = 4 * T + i;
          if (z > 0.f) relu[j >> 5] |= 1u << (j & 31);
          fv[i] = kf(z > 0.f ? z : 0.f, mf, j, invf);
        }
        st4<TK64>(smem + PB_F + (T >> 2) * TILE, rl, 4 * (T & 3) + g, fv);
      }
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) st4<TK64>(smem + PB_DF2, rl, 4 * t + g, df2 + 4 * t);
    __syncthreads();
    {  // dW2^T [k: f feature tile j][n: output tile = wave]
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const s8v y = tfrag<TK64>(smem + PB_DF2, 32 * s, wave, lane);
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          if ((j & 3) == 0) sb();  // (bounds the operand reads in flight: all 32 hoisted would cost 128 VGPRs)
          aW2[j] = mma(tfrag<TK64>(smem + PB_F + (j >> 2) * TILE, 32 * s, j & 3, lane), y, aW2[j]);
        }
      }
    }
    __syncthreads();
    // ---- d f = W2^T . d f2 through dropout' and ReLU', four tiles at a time: staged for dW1, column-summed
    //      (bias), and consumed at once as the K-steps of d h1 = W1^T . d f (+ d s2 below)
    float dh1[16];
    {
      const s8v b0 = bfrag(df2, 0), b1 = bfrag(df2, 1);
      f4v accd[4] = {Z4, Z4, Z4, Z4};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        sb();
        float d16[16];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int T = 4 * q + u;
          f4v acc = mma(wtfrag<true>(smem + PB_W2, LDK256B, T, 0, lane), b0, Z4);
          acc = mma(wtfrag<true>(smem + PB_W2, LDK256B, T, 1, lane), b1, acc);
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int j = 4 * T + i;
            d16[4 * u + i] = keepf(kf(acc[i], mf, j, invf), relu[j >> 5], j & 31);
          }
          st4<TK64>(smem + PB_F + q * TILE, rl, 4 * u + g, d16 + 4 * u);
        }
        csum_add(cbf[q], d16, lane);
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          const s8v bf = pk8(d16[8 * hh], d16[8 * hh + 1], d16[8 * hh + 2], d16[8 * hh + 3], d16[8 * hh + 4],
                             d16[8 * hh + 5], d16[8 * hh + 6], d16[8 * hh + 7]);
#pragma unroll
          for (int T = 0; T < 4; ++T) accd[T] = mma(wtfrag<true>(smem + PB_W1, LDK64, T, 2 * q + hh, lane), bf, accd[T]);
        }
      }
      sb();
#pragma unroll
      for (int T = 0; T < 4; ++T)
#pragma unroll
        for (int i = 0; i < 4; ++i) dh1[4 * T + i] = accd[T][i] + ds2[4 * T + i];
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) st4<TK64>(smem + PB_H1, rl, 4 * t + g, h1 + 4 * t);
    __syncthreads();
    {  // dW1^T [k: h1 feature tile kt][n: f feature tile wave + 4 jn]
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        s8v x[4];
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) x[kt] = tfrag<TK64>(smem + PB_H1, 32 * s, kt, lane);
#pragma unroll
        for (int jn = 0; jn < 4; ++jn) {
          sb();
          const int tn = wave + 4 * jn;
          const s8v y = tfrag<TK64>(smem + PB_F + (tn >> 2) * TILE, 32 * s, tn & 3, lane);
#pragma unroll
          for (int kt = 0; kt < 4; ++kt) aW1[4 * jn + kt] = mma(x[kt], y, aW1[4 * jn + kt]);
        }
      }
    }
    {
      float t1[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) t1[j] = dh1[j] * xh1[j];
      csum_add(cg1, t1, lane);
      csum_add(cb1, dh1, lane);
    }
    float ds1[16], da[16], ov[16];
    vec16(gm, vec + V_G1 * 4, g);
    ln_bwd2(ds1, dh1, xh1, rstd1, gm);
    if (ok) stt16f(a.dres + row * 64, ds1, g);
    {
      const uint32_t m1[1] = {cur.kb[0]};
#pragma unroll
      for (int j = 0; j < 16; ++j) da[j] = kf(ds1[j], m1, j, inv1);
    }
    csum_add(cbo, da, lane);
    unbf(ov, cur.o);
    // (no barrier: DA / O are not read before the next one, and the previous block's dWo reads of them are
    // ordered by this block's first barrier)
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      st4<TK64>(smem + PB_DA, rl, 4 * t + g, da + 4 * t);
      st4<TK64>(smem + PB_O, rl, 4 * t + g, ov + 4 * t);
    }
    // ---- d o = Wo^T . d a (bf16), Delta = rowsum(d o o) per head
    {
      const s8v b0 = bfrag(da, 0), b1 = bfrag(da, 1);
      const int bb = (int)(r / a.L), ll = (int)(r - (long)bb * a.L);
#pragma unroll
      for (int T = 0; T < 4; ++T) {
        f4v acc = mma(wtfrag<true>(smem + PB_WO, LDK64, T, 0, lane), b0, Z4);
        acc = mma(wtfrag<true>(smem + PB_WO, LDK64, T, 1, lane), b1, acc);
        const uint32_t u0 = pk2(acc[0], acc[1]), u1 = pk2(acc[2], acc[3]);
        const float d0 = __uint_as_float(u0 << 16), d1 = __uint_as_float(u0 & 0xFFFF0000u),
                    d2 = __uint_as_float(u1 << 16), d3 = __uint_as_float(u1 & 0xFFFF0000u);
        const float dl = fk::rsum4(d0 * ov[4 * T] + d1 * ov[4 * T + 1] + d2 * ov[4 * T + 2] + d3 * ov[4 * T + 3]);
        if (ok) {
          *(u32x2v*)(a.dout + row * 64 + 16 * T + 4 * g) = u32x2v{u0, u1};
          if (g == 0) a.delta[(((long)c * a.B + bb) * NH + T) * a.Lp + ll] = dl;
        }
      }
    }
    __syncthreads();
    {  // dWo^T [k: o feature tile kt][n: a feature tile = wave]
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const s8v y = tfrag<TK64>(smem + PB_DA, 32 * s, wave, lane);
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) aWo[kt] = mma(tfrag<TK64>(smem + PB_O, 32 * s, kt, lane), y, aWo[kt]);
      }
    }
    }
    cur = nxt;
  }
  // ---- this workgroup's partials: dW tiles straight from the accumulators, vector sums in wave order
  float* ws = a.ws + ((long)c * gridDim.x + blockIdx.x) * AFL_HAR_POST_NG;
#pragma unroll
  for (int j = 0; j < 16; ++j)  // dW2^T tile (k tile j, n tile wave): element (k = 16j + 4g + e, n = 16 wave + li)
#pragma unroll
    for (int e = 0; e < 4; ++e) ws[G_W2 + (16 * wave + li) * 256 + 16 * j + 4 * g + e] = aW2[j][e];
#pragma unroll
  for (int jn = 0; jn < 4; ++jn)
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        ws[G_W1 + (16 * (wave + 4 * jn) + li) * 64 + 16 * kt + 4 * g + e] = aW1[4 * jn + kt][e];
#pragma unroll
  for (int kt = 0; kt < 4; ++kt)
#pragma unroll
    for (int e = 0; e < 4; ++e) ws[G_WO + (16 * wave + li) * 64 + 16 * kt + 4 * g + e] = aWo[kt][e];
  LDS_AS float* red = ldsf(smem, PB_RED) + wave * V_N;
  const int f = csum_feature(lane);
  red[V_BO + f] = cbo;
  red[V_G1 + f] = cg1;
  red[V_BE1 + f] = cb1;
#pragma unroll
  for (int q = 0; q < 4; ++q) red[V_B1 + 64 * q + f] = cbf[q];
  red[V_B2 + f] = cbf2;
  red[V_G2 + f] = cg2;
  red[V_BE2 + f] = cb2;
  __syncthreads();
  for (int e = tid; e < V_N; e += NTR) {
    const LDS_AS float* rr = ldsf(smem, PB_RED) + e;
    ws[G_VEC + e] = ((rr[0] + rr[V_N]) + rr[2 * V_N]) + rr[3 * V_N];
  }
}

// ---- q | k | v backward: dx = d(residual) + dqkv . W_in ; d(in_proj) partials ----
constexpr int QB_W = 0, QB_DQ = 192 * LDK64, QB_X = QB_DQ + 3 * TILE, QB_RED = QB_X + TILE;
constexpr int QB_SMEM = QB_RED + 4 * 192 * 4;
static_assert(QB_SMEM <= 160 * 1024 && PB_SMEM <= 160 * 1024 && PF_SMEM <= 160 * 1024, "HAR LDS budgets");

__global__ void __launch_bounds__(NTR) __attribute__((amdgpu_waves_per_eu(2, 2))) k_har_qkv_bwd(AflHarQkvB a) {
  extern __shared__ __attribute__((aligned(16))) uchar smem[];
  const int c = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, li = lane & 15;
  const float* pp = a.params + (long)c * a.P;
  build_img<true>(smem, QB_W, LDK64, pp + a.w_off, 192, 64);
  __syncthreads();
  const long R = (long)a.B * a.L;
  const int nblk = (int)((R + 63) / 64);
  f4v aW[12];
#pragma unroll
  for (int j = 0; j < 12; ++j) aW[j] = Z4;
  float cs[3] = {0.f, 0.f, 0.f};
  const int rl = 16 * wave + li;
  // this lane's inputs of one block; the NEXT block's are loaded while the current one computes (the pass is
  // latency-bound: a block's loads, two barriers and the dW MFMAs would otherwise run back to back)
  struct In {
    u32x2v dq[12], x[4];
    f4v dr[4];
  };
  auto load = [&](int blk, In& in) {
    const long r = 64L * blk + rl;
    const bool ok = blk < nblk && r < R;
    const long row = (long)c * R + (ok ? r : 0);
    const int bb = ok ? (int)(r / a.L) : 0, ll = ok ? (int)(r - (long)bb * a.L) : 0;
#pragma unroll
    for (int T = 0; T < 12; ++T) {
      const int which = T >> 2, h = T & 3;
      const u16* src = a.dqkv + ((((long)c * a.B + bb) * NH + h) * 3 + which) * (long)a.Lp * DH + (long)ll * DH + 4 * g;
      in.dq[T] = ok ? *(const u32x2v*)src : u32x2v{0u, 0u};
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      in.dr[t] = ok ? *(const f4v*)(a.dres + row * 64 + 16 * t + 4 * g) : Z4;
      in.x[t] = ok ? *(const u32x2v*)(a.x + row * 64 + 16 * t + 4 * g) : u32x2v{0u, 0u};
    }
  };
  In cur;
  load(blockIdx.x, cur);
  for (int blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
    In nxt;
    load(blk + gridDim.x, nxt);
    const long r = 64L * blk + rl;
    const bool ok = r < R;
    const long row = (long)c * R + (ok ? r : 0);
    float dq[48];
#pragma unroll
    for (int T = 0; T < 12; ++T) {
      const u32x2v u = cur.dq[T];
      dq[4 * T] = __uint_as_float(u[0] << 16);
      dq[4 * T + 1] = __uint_as_float(u[0] & 0xFFFF0000u);
      dq[4 * T + 2] = __uint_as_float(u[1] << 16);
      dq[4 * T + 3] = __uint_as_float(u[1] & 0xFFFF0000u);
      st4<TK64>(smem + QB_DQ + (T >> 2) * TILE, rl, 4 * (T & 3) + g, dq + 4 * T);
    }
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      float x16[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) x16[j] = dq[16 * q + j];
      csum_add(cs[q], x16, lane);
    }
    float dx[16], xv[16];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      dx[4 * t] = cur.dr[t][0]; dx[4 * t + 1] = cur.dr[t][1]; dx[4 * t + 2] = cur.dr[t][2]; dx[4 * t + 3] = cur.dr[t][3];
      xv[4 * t] = __uint_as_float(cur.x[t][0] << 16);
      xv[4 * t + 1] = __uint_as_float(cur.x[t][0] & 0xFFFF0000u);
      xv[4 * t + 2] = __uint_as_float(cur.x[t][1] << 16);
      xv[4 * t + 3] = __uint_as_float(cur.x[t][1] & 0xFFFF0000u);
    }
    {
      f4v acc[4] = {Z4, Z4, Z4, Z4};
#pragma unroll
      for (int s = 0; s < 6; ++s) {
        const s8v bf = bfrag(dq, s);
#pragma unroll
        for (int T = 0; T < 4; ++T) acc[T] = mma(wtfrag<true>(smem + QB_W, LDK64, T, s, lane), bf, acc[T]);
      }
#pragma unroll
      for (int T = 0; T < 4; ++T)
#pragma unroll
        for (int i = 0; i < 4; ++i) dx[4 * T + i] += acc[T][i];
    }
    if (ok) stt16f(a.dx + row * 64, dx, g);
#pragma unroll
    for (int t = 0; t < 4; ++t) st4<TK64>(smem + QB_X, rl, 4 * t + g, xv + 4 * t);
    __syncthreads();
#pragma unroll
    for (int s = 0; s < 2; ++s) {  // dW_in^T [k: x feature tile kt][n: qkv feature tile wave + 4 jn]
      s8v x[4];
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) x[kt] = tfrag<TK64>(smem + QB_X, 32 * s, kt, lane);
#pragma unroll
      for (int jn = 0; jn < 3; ++jn) {
        const int tn = wave + 4 * jn;
        const s8v y = tfrag<TK64>(smem + QB_DQ + (tn >> 2) * TILE, 32 * s, tn & 3, lane);
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) aW[4 * jn + kt] = mma(x[kt], y, aW[4 * jn + kt]);
      }
    }
    __syncthreads();
    cur = nxt;
  }
  float* ws = a.ws + ((long)c * gridDim.x + blockIdx.x) * AFL_HAR_QKV_NG;
#pragma unroll
  for (int jn = 0; jn < 3; ++jn)
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int e = 0; e < 4; ++e) ws[(16 * (wave + 4 * jn) + li) * 64 + 16 * kt + 4 * g + e] = aW[4 * jn + kt][e];
  LDS_AS float* red = ldsf(smem, QB_RED) + wave * 192;
  const int f = csum_feature(lane);
#pragma unroll
  for (int q = 0; q < 3; ++q) red[64 * q + f] = cs[q];
  __syncthreads();
  for (int e = tid; e < 192; e += NTR) {
    const LDS_AS float* rr = ldsf(smem, QB_RED) + e;
    ws[192 * 64 + e] = ((rr[0] + rr[192]) + rr[384]) + rr[576];
  }
}

// grads[c][param_off + e] = sum over g of ws[c][g][ws_off + e] (fixed order), per segment (ws_off, param_off, n)
__global__ void __launch_bounds__(256) k_har_reduce(const float* __restrict__ ws, int G, int n, const int* __restrict__ seg,
                                                    int nseg, float* __restrict__ grads, long P) {
  const int c = blockIdx.y;
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= n) return;
  int k = 0;
  while (k + 1 < nseg && e >= seg[3 * (k + 1)]) ++k;
  const int off = e - seg[3 * k];
  if (off >= seg[3 * k + 2]) return;
  const float* w = ws + (long)c * G * n + e;
  float s = 0.f;
  for (int i = 0; i < G; ++i) s += w[(long)i * n];
  grads[(long)c * P + seg[3 * k + 1] + off] = s;
}

}  // namespace

// =================================================================================== launchers
int afl_har_stem(const float* x, int C, int B, int L, const float* params, long P, int w_off, int b_off, int pe_off,
                 u16* h, hipStream_t s) {
  const long R = (long)B * L;
  hipLaunchKernelGGL(k_har_stem, dim3((unsigned)((R + STEM_ROWS - 1) / STEM_ROWS), C), dim3(256), 0, s, x, B, L, params, P,
                     w_off, b_off, pe_off, h);
  return (int)hipGetLastError();
}

int afl_har_pool(const u16* y, int C, int B, int L, float* out, hipStream_t s) {
  hipLaunchKernelGGL(k_har_pool, dim3(C * B), dim3(256), 0, s, y, L, out);
  return (int)hipGetLastError();
}

static int har_blocks(long R, int C = 1) {  // workgroups per client: about one per CU over all clients
  const long tiles = (R + 15) / 16;
  long g = (tiles + NWF - 1) / NWF;
  const long cap = 256 / (C > 0 ? C : 1);
  if (g > cap) g = cap;
  return (int)(g < 1 ? 1 : (g > 64 ? 64 : g));
}

int afl_har_qkv(const AflHarQkv& a, hipStream_t s) {
  if (a.Lp % 64 || a.Lp < a.L) return (int)hipErrorInvalidValue;
  const size_t lds = 192 * LDK64 + 192 * 4;
  hipLaunchKernelGGL(k_har_qkv, dim3(har_blocks((long)a.B * a.L, a.C), a.C), dim3(NTF), lds, s, a);
  return (int)hipGetLastError();
}

int afl_har_attn_fwd(const AflHarAttn& a, hipStream_t s) {
  if (a.Lp % 64 || a.Lp < a.L || a.Lp > 1024) return (int)hipErrorInvalidValue;
  if (a.drop.thr16 && !a.mask) return (int)hipErrorInvalidValue;
  const size_t lds = (size_t)a.Lp * 32 * 2 + (size_t)a.Lp * 2;  // K, V images + the column-pair hash table
  if (a.drop.thr16)
    hipLaunchKernelGGL(k_har_attn_fwd<true>, dim3(a.C * a.B * NH), dim3(AT_NT), lds, s, a);
  else
    hipLaunchKernelGGL(k_har_attn_fwd<false>, dim3(a.C * a.B * NH), dim3(AT_NT), lds, s, a);
  return (int)hipGetLastError();
}

int afl_har_attn_bwd(const AflHarAttn& a, hipStream_t s) {
  if (a.Lp % 64 || a.Lp < a.L || a.Lp > 1024) return (int)hipErrorInvalidValue;
  if (a.drop.thr16 && !a.mask) return (int)hipErrorInvalidValue;
  const size_t kv = (size_t)a.Lp * 32 * 2 + (size_t)a.Lp * 8, dq = (size_t)a.Lp * 32 * 2;
  const dim3 grid(a.C * a.B * NH);
  if (a.drop.thr16) {
    hipLaunchKernelGGL(k_har_attn_bwd_kv<true>, grid, dim3(AT_NT), kv, s, a);
    hipLaunchKernelGGL(k_har_attn_bwd_dq<true>, grid, dim3(AT_NT), dq, s, a);
  } else {
    hipLaunchKernelGGL(k_har_attn_bwd_kv<false>, grid, dim3(AT_NT), kv, s, a);
    hipLaunchKernelGGL(k_har_attn_bwd_dq<false>, grid, dim3(AT_NT), dq, s, a);
  }
  return (int)hipGetLastError();
}

int afl_har_blocks(long R) { return har_blocks(R); }

int afl_har_post_bwd(const AflHarPostB& a, int G, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute((const void*)k_har_post_bwd, hipFuncAttributeMaxDynamicSharedMemorySize, PB_SMEM) != hipSuccess)
      return -2;
    attr = true;
  }
  if (G < 1 || ((a.d1.thr16 || a.df.thr16 || a.d2.thr16) && !a.kbits)) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_har_post_bwd, dim3(G, a.C), dim3(NTR), PB_SMEM, s, a);
  return (int)hipGetLastError();
}

int afl_har_qkv_bwd(const AflHarQkvB& a, int G, hipStream_t s) {
  if (G < 1 || a.Lp % 64 || a.Lp < a.L) return (int)hipErrorInvalidValue;
  static bool attr = false;
  if (!attr) {  // (QB_SMEM passes 64 KB with HAR_IMG_PAD=16)
    if (hipFuncSetAttribute((const void*)k_har_qkv_bwd, hipFuncAttributeMaxDynamicSharedMemorySize, QB_SMEM) != hipSuccess)
      return -2;
    attr = true;
  }
  hipLaunchKernelGGL(k_har_qkv_bwd, dim3(G, a.C), dim3(NTR), QB_SMEM, s, a);
  return (int)hipGetLastError();
}

int afl_har_reduce(const float* ws, int C, int G, int n, const int* seg, int nseg, float* grads, long P, hipStream_t s) {
  hipLaunchKernelGGL(k_har_reduce, dim3((n + 255) / 256, C), dim3(256), 0, s, ws, G, n, seg, nseg, grads, P);
  return (int)hipGetLastError();
}

int afl_har_post(const AflHarPost& a, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute((const void*)k_har_post, hipFuncAttributeMaxDynamicSharedMemorySize, PF_SMEM) != hipSuccess)
      return -2;
    attr = true;
  }
  if ((a.d1.thr16 || a.df.thr16 || a.d2.thr16) && !a.kbits) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_har_post, dim3(har_blocks(a.R, a.C), a.C), dim3(NTP), PF_SMEM, s, a);
  return (int)hipGetLastError();
}
