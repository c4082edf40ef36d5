// Client-batched layer kernels for gfx950 — the native training/eval path of every model that has no
// whole-step fused trainer: CNNModel (reference src/Model.py:27-88), RNNModel (src/Model.py:91-163)
// and the HAR TransformerClassifier (src/Model.py:418-458).  The training step is a fixed sequence of
// these launches over all of a rank's clients at once ([C][rows][cols] tensors), captured once into a
// HIP graph and replayed per optimizer step (attackfl_amd/fl/programs.py); everything that varies per
// step (batch rows, batch size, epoch, dropout key, Adam step) is read from device memory.
//
//   k_bgemm       C (op)= epi(alpha * A.B^T) on v_mfma_f32_16x16x32_bf16 — 64x64 output tile per
//                 256-thread workgroup (4 waves x 32x32), fp32 operands converted to bf16 while staged
//                 into LDS, fp32 accumulate; fused epilogue: bias, activation (relu / erf-GELU),
//                 pre-activation copy, dropout (hash mask), activation-derivative multiply (backward),
//                 store / accumulate / atomic split-K accumulate.  Any strides: the same kernel runs
//                 X.W^T (forward), dY.W (input grad) and dY^T.X (weight grad).
//   k_colsum      bias gradients (column sums over rows)
//   k_im2col3 / k_col2im3     Conv1d(k=3, pad=1) as GEMM over channels-last activations (+relu')
//   k_pool4_*     AdaptiveAvgPool1d(4) (overlapping bins for L=7) + dropout, fwd/bwd (+relu')
//   k_ln_*        residual-add + dropout + LayerNorm(64) fused fwd/bwd (16 lanes per row)
//   k_gru_*       bidirectional GRU cell at seq_len 1 (h0 = 0 closed form), fwd/bwd
//   k_bce / k_ce  sigmoid-BCE / softmax-CE mean loss + gradient + NaN abort (client.py:95-103)
//   k_adam_clients   torch.optim.Adam over the [C][P] flat arena with per-client step counts
//   k_conv_pe_*, k_mean_rows_*   HAR stem (Conv1d(1->64) + positional encoding) and mean-pool over L
#include "common.h"
#include "kernels.h"

typedef short s8v __attribute__((ext_vector_type(8)));
typedef __bf16 bf8v __attribute__((ext_vector_type(8)));
typedef float f4v __attribute__((ext_vector_type(4)));
typedef float f2v __attribute__((ext_vector_type(2)));
typedef __bf16 b2v __attribute__((ext_vector_type(2)));
typedef unsigned int u4v __attribute__((ext_vector_type(4)));

namespace {

__device__ __forceinline__ uint32_t pk_bf2(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f2v){lo, hi}, b2v));
}

__device__ __forceinline__ float gelu_f(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_d(float x) {
  const float cdf = 0.5f * (1.f + erff(x * 0.70710678118654752f));
  return cdf + x * 0.39894228040143268f * __expf(-0.5f * x * x);
}
__device__ __forceinline__ float act_f(float v, int act) {
  return act == 1 ? (v < 0.f ? 0.f : v) : (act == 2 ? gelu_f(v) : v);  // relu keeps NaN, like torch
}
__device__ __forceinline__ float act_d(float g, int gact) {
  return gact == 1 ? (g > 0.f ? 1.f : 0.f) : (gact == 2 ? gelu_d(g) : 1.f);
}
__device__ __forceinline__ int cur_step(const int* stepctl) { return stepctl ? *stepctl : 0; }
__device__ __forceinline__ uint32_t drop_key(const AflDrop& d, int c) {
  return afl_hash32(d.seeds[c], (uint32_t)cur_step(d.stepctl));
}
__device__ __forceinline__ float drop_scale(const AflDrop& d, uint32_t key, uint32_t r, uint32_t col) {
  return afl_keep(key, d.layer, r, col, d.thr16) ? d.inv_keep : 0.f;
}

// ============================================================================ batched GEMM
constexpr int GT = 64, GK = 32, GLD = 40;  // output tile, k step, LDS row stride (bf16 elements)

// Each thread stages 8 consecutive-k elements of one row of the A tile and of the B tile.  AK / BK
// pick the thread->element map that keeps global reads coalesced: k-contiguous operands read 8
// consecutive k per thread, m-contiguous ones (transposed views) read consecutive m across lanes.
template <bool KC>
__device__ __forceinline__ void stage_load(const float* __restrict__ X, long sr, long sk, int rows, int r0, int k0,
                                           int ke, int tid, bool vec, float (&v)[8]) {
  const int r = KC ? r0 + (tid >> 2) : r0 + (tid & 63);
  const int k = KC ? k0 + (tid & 3) * 8 : k0 + (tid >> 6) * 8;
  const bool rok = r < rows;
  const float* p = X + (long)r * sr;
  if (KC && vec && rok && k + 8 <= ke) {  // 16-B aligned rows: two dwordx4 loads
    const f4v x0 = *(const f4v*)(p + k), x1 = *(const f4v*)(p + k + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[j] = x0[j];
      v[4 + j] = x1[j];
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (rok && k + j < ke) ? p[(long)(k + j) * sk] : 0.f;
}
template <bool KC>
__device__ __forceinline__ void stage_store(unsigned short* S, int tid, const float (&v)[8]) {
  const int r = KC ? (tid >> 2) : (tid & 63);
  const int k = KC ? (tid & 3) * 8 : (tid >> 6) * 8;
  u4v w;
  w[0] = pk_bf2(v[0], v[1]);
  w[1] = pk_bf2(v[2], v[3]);
  w[2] = pk_bf2(v[4], v[5]);
  w[3] = pk_bf2(v[6], v[7]);
  *(u4v*)(S + r * GLD + k) = w;
}
__device__ __forceinline__ s8v frag(const unsigned short* S, int r0, int lane) {
  return *(const s8v*)(S + (r0 + (lane & 15)) * GLD + 8 * (lane >> 4));
}

template <bool AK, bool BK>
__global__ void __launch_bounds__(256) k_bgemm(AflGemm g) {
  __shared__ __attribute__((aligned(16))) unsigned short As[GT * GLD];
  __shared__ __attribute__((aligned(16))) unsigned short Bs[GT * GLD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tiles_n = (g.N + GT - 1) / GT;
  const int m0 = (blockIdx.x / tiles_n) * GT, n0 = (blockIdx.x % tiles_n) * GT;
  const int c = blockIdx.z;
  const int kchunk = ((g.K + g.splitk - 1) / g.splitk + GK - 1) / GK * GK;
  const int kb = blockIdx.y * kchunk, ke = min(g.K, kb + kchunk);
  if (kb >= ke) return;
  const float* A = g.A + (long)c * g.sAc;
  const float* B = g.B + (long)c * g.sBc;

  f4v acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};
  const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;
  float ra[8], rb[8];
  stage_load<AK>(A, g.sAm, g.sAk, g.M, m0, kb, ke, tid, g.avec, ra);
  stage_load<BK>(B, g.sBn, g.sBk, g.N, n0, kb, ke, tid, g.bvec, rb);
  for (int k0 = kb; k0 < ke; k0 += GK) {
    stage_store<AK>(As, tid, ra);
    stage_store<BK>(Bs, tid, rb);
    __syncthreads();
    if (k0 + GK < ke) {  // next tile's global loads overlap this tile's MFMAs
      stage_load<AK>(A, g.sAm, g.sAk, g.M, m0, k0 + GK, ke, tid, g.avec, ra);
      stage_load<BK>(B, g.sBn, g.sBk, g.N, n0, k0 + GK, ke, tid, g.bvec, rb);
    }
    const s8v a0 = frag(As, wm, lane), a1 = frag(As, wm + 16, lane);
    const s8v b0 = frag(Bs, wn, lane), b1 = frag(Bs, wn + 16, lane);
    acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf8v, a0), __builtin_bit_cast(bf8v, b0),
                                                        acc[0][0], 0, 0, 0);
    acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf8v, a0), __builtin_bit_cast(bf8v, b1),
                                                        acc[0][1], 0, 0, 0);
    acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf8v, a1), __builtin_bit_cast(bf8v, b0),
                                                        acc[1][0], 0, 0, 0);
    acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf8v, a1), __builtin_bit_cast(bf8v, b1),
                                                        acc[1][1], 0, 0, 0);
    __syncthreads();
  }
  // epilogue: lane holds C[4*(lane>>4)+e][lane&15] of each 16x16 tile
  const bool dr = g.drop.thr16 != 0;
  const uint32_t key = dr ? drop_key(g.drop, c) : 0u;
  float* Cc = g.Cm + (long)c * g.sCc;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m0 + wm + 16 * i + 4 * (lane >> 4) + e;
        const int n = n0 + wn + 16 * j + (lane & 15);
        if (m >= g.M || n >= g.N) continue;
        float v = g.alpha * acc[i][j][e];
        if (g.bias) v += g.bias[(long)c * g.sbc + n];
        const long off = (long)m * g.sCm + (long)n * g.sCn;
        if (g.Z) g.Z[(long)c * g.sCc + off] = v;
        v = act_f(v, g.act);
        if (dr) v *= drop_scale(g.drop, key, m, n);
        if (g.G) v *= act_d(g.G[(long)c * g.sGc + (long)m * g.sGm + (long)n * g.sGn], g.gact);
        if (g.accum == 0)
          Cc[off] = v;
        else if (g.accum == 1)
          Cc[off] += v;
        else if (g.ws)  // deterministic split-K: this split's partial, summed in split order by k_split_sum
          g.ws[(((long)blockIdx.y * g.nC + c) * g.M + m) * g.N + n] = v;
        else
          atomicAdd(Cc + off, v);
      }
}

// sum of p[0], p[stride], ... p[(n-1) * stride] added strictly in index order (deterministic), with U loads in
// flight per batch: a plain loop issues one load, waits for it, adds, and so on (~L2 latency per partial)
template <int U>
__device__ __forceinline__ float ordered_sum(const float* __restrict__ p, long stride, int n) {
  float s = 0.f;
  int q = 0;
  for (; q + U <= n; q += U) {
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = p[(long)(q + u) * stride];
#pragma unroll
    for (int u = 0; u < U; ++u) s += v[u];
  }
  for (; q < n; ++q) s += p[(long)q * stride];
  return s;
}

// C[c][m][n] += sum over the first `ns` splits of ws[split][c][m][n], in split order (deterministic)
__global__ void __launch_bounds__(256) k_split_sum(const float* __restrict__ ws, int ns, int nC, int M, int N,
                                                   float* __restrict__ Cm, long sCc, long sCm, long sCn) {
  const long total = (long)nC * M * N;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int n = (int)(i % N);
    const long cm = i / N;
    const int m = (int)(cm % M), c = (int)(cm / M);
    Cm[(long)c * sCc + (long)m * sCm + (long)n * sCn] += ordered_sum<16>(ws + i, total, ns);
  }
}

// dst[c * sdc + j] += sum over p < np of ws[(p * nC + c) * ld + j]  (j < n), in p order: the deterministic
// second pass of every per-block partial sum below (block order fixed, whatever order the blocks ran in)
// (32 outputs per block, 8 partial groups per output: group g adds partials g, g + 8, ... in order, then the
// 8 group sums are added in group order — a fixed association, so still the same bits every run)
__global__ void __launch_bounds__(256) k_partial_sum(const float* __restrict__ ws, int np, int nC, int n, long ld,
                                                     float* __restrict__ dst, long sdc) {
  __shared__ float red[8][32];
  const long total = (long)nC * n;
  const int e = threadIdx.x & 31, gq = threadIdx.x >> 5;
  const long i = (long)blockIdx.x * 32 + e;
  const int c = (int)(i / n), j = (int)(i - (long)c * n);
  const int cnt = np > gq ? (np - gq + 7) / 8 : 0;  // partials gq, gq + 8, ...
  red[gq][e] = i < total ? ordered_sum<8>(ws + ((long)gq * nC + c) * ld + j, 8L * nC * ld, cnt) : 0.f;
  __syncthreads();
  if (gq == 0 && i < total) {
    float sum = red[0][e];
#pragma unroll
    for (int q = 1; q < 8; ++q) sum += red[q][e];
    dst[(long)c * sdc + j] += sum;
  }
}
void partial_sum(const float* ws, int np, int nC, int n, long ld, float* dst, long sdc, hipStream_t s) {
  const long total = (long)nC * n;
  hipLaunchKernelGGL(k_partial_sum, dim3((unsigned)((total + 31) / 32)), dim3(256), 0, s, ws, np, nC, n, ld, dst, sdc);
}

// ============================================================================ column sums
__global__ void __launch_bounds__(256) k_colsum(const float* __restrict__ Y, long sYc, long sYm, int M, int N,
                                                float* __restrict__ out, long sOc, float* __restrict__ ws) {
  __shared__ float red[4][64];
  const int c = blockIdx.z, col = blockIdx.x * 64 + (threadIdx.x & 63), rg = threadIdx.x >> 6;
  const int r0 = blockIdx.y * 256;
  float s = 0.f;
  if (col < N) {
    const float* p = Y + (long)c * sYc + col;
    for (int r = r0 + rg; r < min(M, r0 + 256); r += 4) s += p[(long)r * sYm];
  }
  red[rg][threadIdx.x & 63] = s;
  __syncthreads();
  if (rg == 0 && col < N) {
    s = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
    if (ws)
      ws[((long)blockIdx.y * gridDim.z + c) * N + col] = s;
    else
      atomicAdd(out + (long)c * sOc + col, s);
  }
}

// ============================================================================ batch gathers
__global__ void k_gather_icu(const float* __restrict__ rows, const int* __restrict__ idx, const int* stepctl, int C,
                             int B, int mask, float* __restrict__ vit, float* __restrict__ lab, float* __restrict__ y) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= C * B * 24) return;
  const int f = t % 24, cb = t / 24;
  const int r = idx[(long)cur_step(stepctl) * C * B + cb];
  float v = r >= 0 ? rows[(long)r * 24 + f] : 0.f;
  if (mask && f < 23 && v == -2.0f) v = 0.f;  // RNNModel masking (src/Model.py:121-122)
  if (f < 7)
    vit[(long)cb * 7 + f] = v;
  else if (f < 23)
    lab[(long)cb * 16 + f - 7] = v;
  else
    y[cb] = v;
}

__global__ void k_gather_har(const float* __restrict__ x, const long* __restrict__ y, int F,
                             const int* __restrict__ idx, const int* stepctl, int C, int B, float* __restrict__ ox,
                             long* __restrict__ oy) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long)C * B * F) return;
  const int f = (int)(t % F);
  const long cb = t / F;
  const int r = idx[(long)cur_step(stepctl) * C * B + cb];
  ox[t] = r >= 0 ? x[(long)r * F + f] : 0.f;
  if (f == 0) oy[cb] = r >= 0 ? y[r] : 0;
}

// ============================================================================ conv1d k=3 pad=1
__global__ void k_im2col3(const float* __restrict__ x, long sXc, long sXr, int C, int B, int L, int Cin,
                          float* __restrict__ out) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int K = 3 * Cin;
  if (t >= (long)C * B * L * K) return;
  const int k = (int)(t % K);
  const long row = (t / K) % ((long)B * L);
  const int c = (int)(t / ((long)K * B * L));
  const int ci = k / 3, j = k % 3;
  const int l = (int)(row % L) + j - 1;
  out[t] = (l >= 0 && l < L) ? x[(long)c * sXc + (row - (row % L) + l) * sXr + ci] : 0.f;
}

__global__ void k_col2im3(const float* __restrict__ dcols, int C, int B, int L, int Cin,
                          const float* __restrict__ relu_src, long sRc, long sRr, float* __restrict__ dx) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long)C * B * L * Cin) return;
  const int ci = (int)(t % Cin);
  const long row = (t / Cin) % ((long)B * L);
  const int c = (int)(t / ((long)Cin * B * L));
  const int l = (int)(row % L);
  const float* d = dcols + (long)c * B * L * 3 * Cin;
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int lo = l - j + 1;  // output position whose tap j reads input l
    if (lo >= 0 && lo < L) s += d[(row - l + lo) * 3 * Cin + ci * 3 + j];
  }
  if (relu_src && !(relu_src[(long)c * sRc + row * sRr + ci] > 0.f)) s = 0.f;
  dx[t] = s;
}

// ============================================================================ AdaptiveAvgPool1d(4)
__device__ __forceinline__ int bin_lo(int p, int L) { return (p * L) / 4; }
__device__ __forceinline__ int bin_hi(int p, int L) { return ((p + 1) * L + 3) / 4; }

__global__ void k_pool4_fwd(const float* __restrict__ h, int C, int B, int L, int Ch, float* __restrict__ out,
                            long sOc, long sOr, int col0, AflDrop d) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long)C * B * Ch * 4) return;
  const int p = (int)(t & 3), ch = (int)((t >> 2) % Ch);
  const int b = (int)((t / (4L * Ch)) % B), c = (int)(t / (4L * Ch * B));
  const int lo = bin_lo(p, L), hi = bin_hi(p, L);
  const float* src = h + ((long)c * B * L + (long)b * L) * Ch + ch;
  float s = 0.f;
  for (int l = lo; l < hi; ++l) s += src[(long)l * Ch];
  s /= (float)(hi - lo);
  const int col = col0 + ch * 4 + p;
  if (d.thr16) s *= drop_scale(d, drop_key(d, c), b, col);
  out[(long)c * sOc + (long)b * sOr + col] = s;
}

__global__ void k_pool4_bwd(const float* __restrict__ dout, long sOc, long sOr, int col0, const float* __restrict__ h,
                            int C, int B, int L, int Ch, float* __restrict__ dh, AflDrop d) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long)C * B * L * Ch) return;
  const int ch = (int)(t % Ch), l = (int)((t / Ch) % L);
  const int b = (int)((t / ((long)Ch * L)) % B), c = (int)(t / ((long)Ch * L * B));
  const uint32_t key = d.thr16 ? drop_key(d, c) : 0u;
  float s = 0.f;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int lo = bin_lo(p, L), hi = bin_hi(p, L);
    if (l >= lo && l < hi) {
      const int col = col0 + ch * 4 + p;
      float g = dout[(long)c * sOc + (long)b * sOr + col] / (float)(hi - lo);
      if (d.thr16) g *= drop_scale(d, key, b, col);
      s += g;
    }
  }
  if (!(h[t] > 0.f)) s = 0.f;  // relu' of the conv3 output
  dh[t] = s;
}

// ============================================================================ LayerNorm(64)
// 16 lanes per row, 4 columns per lane; 16 rows per 256-thread block (fwd).
__device__ __forceinline__ float sum16(float v) {
  v += __shfl_xor(v, 8, 64);
  v += __shfl_xor(v, 4, 64);
  v += __shfl_xor(v, 2, 64);
  v += __shfl_xor(v, 1, 64);
  return v;
}

// V4: every row pointer 16-B aligned (checked by the launcher) -> dwordx4 loads / stores per lane
template <bool V>
__device__ __forceinline__ void ld4f(const float* p, float (&v)[4]) {
  if constexpr (V) {
    const f4v t = *(const f4v*)p;
    v[0] = t[0]; v[1] = t[1]; v[2] = t[2]; v[3] = t[3];
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = p[j];
  }
}
template <bool V>
__device__ __forceinline__ void st4f(float* p, const float (&v)[4]) {
  if constexpr (V) {
    *(f4v*)p = f4v{v[0], v[1], v[2], v[3]};
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) p[j] = v[j];
  }
}

template <bool V4>
__global__ void __launch_bounds__(256) k_ln_fwd(AflLn l) {
  const int c = blockIdx.y;
  const int row = blockIdx.x * 16 + (threadIdx.x >> 4);
  if (row >= l.rows) return;
  const int c0 = (threadIdx.x & 15) * 4;
  const uint32_t ka = l.da.thr16 ? drop_key(l.da, c) : 0u;
  const uint32_t ko = l.dout.thr16 ? drop_key(l.dout, c) : 0u;
  float s[4];
  ld4f<V4>(l.x + (long)c * l.sXc + (long)row * l.sXr + c0, s);
  if (l.a) {
    float a[4];
    ld4f<V4>(l.a + (long)c * l.sAc + (long)row * l.sAr + c0, a);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (l.da.thr16) a[j] *= drop_scale(l.da, ka, row, c0 + j);
      s[j] += a[j];
    }
  }
  if (l.s) st4f<V4>(l.s + ((long)c * l.rows + row) * 64 + c0, s);
  const float mean = sum16(s[0] + s[1] + s[2] + s[3]) * (1.f / 64.f);
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) q += (s[j] - mean) * (s[j] - mean);
  const float rstd = rsqrtf(sum16(q) * (1.f / 64.f) + 1e-5f);
  const float* gm = l.gamma + (long)c * l.sPc;
  const float* bt = l.beta + (long)c * l.sPc;
  float y[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    y[j] = (s[j] - mean) * rstd * gm[c0 + j] + bt[c0 + j];
    if (l.dout.thr16) y[j] *= drop_scale(l.dout, ko, row, c0 + j);
  }
  st4f<V4>(l.y + (long)c * l.sYc + (long)row * l.sYr + c0, y);
  if ((threadIdx.x & 15) == 0) {
    float* st = l.stats + ((long)c * l.rows + row) * 2;
    st[0] = mean;
    st[1] = rstd;
  }
}

constexpr int LNB_ROWS = 256;  // rows per backward block (dgamma/dbeta partials -> 128 atomics)

template <bool V4>
__global__ void __launch_bounds__(256) k_ln_bwd(AflLnB l) {
  __shared__ float red[16][129];
  const int c = blockIdx.y, li = threadIdx.x & 15, rg = threadIdx.x >> 4;
  const int c0 = li * 4;
  const uint32_t ka = l.da_drop.thr16 ? drop_key(l.da_drop, c) : 0u;
  const uint32_t ko = l.dout.thr16 ? drop_key(l.dout, c) : 0u;
  const float* gm = l.gamma + (long)c * l.sPc;
  float gam[4], dg[4] = {0.f, 0.f, 0.f, 0.f}, db[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < 4; ++j) gam[j] = gm[c0 + j];
  const int rbeg = blockIdx.x * LNB_ROWS;
  for (int row = rbeg + rg; row < min(l.rows, rbeg + LNB_ROWS); row += 16) {
    const float* st = l.stats + ((long)c * l.rows + row) * 2;
    const float mean = st[0], rstd = st[1];
    float g[4], xh[4], sv[4], a1 = 0.f, a2 = 0.f;
    ld4f<V4>(l.dy + (long)c * l.sDc + (long)row * l.sDr + c0, g);
    ld4f<V4>(l.s + (long)c * l.sSc + (long)row * l.sSr + c0, sv);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (l.dout.thr16) g[j] *= drop_scale(l.dout, ko, row, c0 + j);
      xh[j] = (sv[j] - mean) * rstd;
      dg[j] += g[j] * xh[j];
      db[j] += g[j];
      const float dxh = g[j] * gam[j];
      a1 += dxh;
      a2 += dxh * xh[j];
    }
    a1 = sum16(a1) * (1.f / 64.f);
    a2 = sum16(a2) * (1.f / 64.f);
    float* dxp = l.dx + (long)c * l.sXc + (long)row * l.sXr + c0;
    float dx[4], dxo[4];
    if (l.dx_accum) ld4f<V4>(dxp, dxo);
#pragma unroll
    for (int j = 0; j < 4; ++j) dx[j] = rstd * (g[j] * gam[j] - a1 - xh[j] * a2);
    if (l.da) {
      float da[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) da[j] = l.da_drop.thr16 ? dx[j] * drop_scale(l.da_drop, ka, row, c0 + j) : dx[j];
      st4f<V4>(l.da + (long)c * l.sAc + (long)row * l.sAr + c0, da);
    }
    if (l.dx_accum) {
#pragma unroll
      for (int j = 0; j < 4; ++j) dx[j] += dxo[j];
    }
    st4f<V4>(dxp, dx);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    red[rg][c0 + j] = dg[j];
    red[rg][64 + c0 + j] = db[j];
  }
  __syncthreads();
  if (threadIdx.x < 128) {
    float s = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) s += red[r][threadIdx.x];
    if (l.ws) {
      l.ws[((long)blockIdx.x * l.nC + c) * 128 + threadIdx.x] = s;
    } else {
      float* dst = threadIdx.x < 64 ? l.dgamma + (long)c * l.sPc + threadIdx.x
                                    : l.dbeta + (long)c * l.sPc + threadIdx.x - 64;
      atomicAdd(dst, s);
    }
  }
}

// ============================================================================ GRU cell, seq_len 1, h0 = 0
// PyTorch gate order (r, z, n): r = s(gi_r + bhh_r), z = s(gi_z + bhh_z), n = tanh(gi_n + r * bhh_n),
// h = (1 - z) * n.  gi already holds x.W_ih^T + b_ih.  W_hh receives an exactly-zero gradient.
__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + __expf(-x)); }

__global__ void k_gru_fwd(const float* __restrict__ gi, const float* __restrict__ bhh, long sPc, int C, int B,
                          float* __restrict__ h, long sHc, long sHr, int col0) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= C * B * 32) return;
  const int j = t & 31, b = (t >> 5) % B, c = t / (32 * B);
  const float* g = gi + ((long)c * B + b) * 96;
  const float* bh = bhh + (long)c * sPc;
  const float r = sigm(g[j] + bh[j]);
  const float z = sigm(g[32 + j] + bh[32 + j]);
  const float n = tanhf(g[64 + j] + r * bh[64 + j]);
  h[(long)c * sHc + (long)b * sHr + col0 + j] = (1.f - z) * n;
}

__global__ void __launch_bounds__(256) k_gru_bwd(const float* __restrict__ dh, long sHc, long sHr, int col0,
                                                 const float* __restrict__ gi, const float* __restrict__ bhh, long sPc,
                                                 int B, float* __restrict__ dgi, float* __restrict__ dbih,
                                                 float* __restrict__ dbhh) {
  __shared__ float red[8][32][5];
  const int c = blockIdx.x, j = threadIdx.x & 31, rg = threadIdx.x >> 5;
  const float* bh = bhh + (long)c * sPc;
  const float bhr = bh[j], bhz = bh[32 + j], bhn = bh[64 + j];
  float sr = 0.f, sz = 0.f, sn = 0.f, snh = 0.f;
  for (int b = rg; b < B; b += 8) {
    const float* g = gi + ((long)c * B + b) * 96;
    const float r = sigm(g[j] + bhr);
    const float z = sigm(g[32 + j] + bhz);
    const float n = tanhf(g[64 + j] + r * bhn);
    const float d = dh[(long)c * sHc + (long)b * sHr + col0 + j];
    const float dan = d * (1.f - z) * (1.f - n * n);
    const float dar = dan * bhn * r * (1.f - r);
    const float daz = -d * n * z * (1.f - z);
    float* o = dgi + ((long)c * B + b) * 96;
    o[j] = dar;
    o[32 + j] = daz;
    o[64 + j] = dan;
    sr += dar;
    sz += daz;
    sn += dan;
    snh += dan * r;
  }
  red[rg][j][0] = sr;
  red[rg][j][1] = sz;
  red[rg][j][2] = sn;
  red[rg][j][3] = snh;
  __syncthreads();
  if (threadIdx.x < 32) {
    float a = 0.f, bz = 0.f, n = 0.f, nh = 0.f;
    for (int r = 0; r < 8; ++r) {
      a += red[r][j][0];
      bz += red[r][j][1];
      n += red[r][j][2];
      nh += red[r][j][3];
    }
    float* bi = dbih + (long)c * sPc;
    float* bhg = dbhh + (long)c * sPc;
    bi[j] = a;
    bi[32 + j] = bz;
    bi[64 + j] = n;
    bhg[j] = a;
    bhg[32 + j] = bz;
    bhg[64 + j] = nh;
  }
}

// ============================================================================ losses
// Per client: rows b < bsz of the current step are real; bsz < min_bs (size-1 batch skip A-21, or past
// the client's last batch) or a previous NaN -> no loss, zero gradient, no Adam update this step.
// stepctl = [step, min_bs, nan_abort]: min_bs 2 / nan_abort 1 are the ICU semantics (client.py:86-102);
// the reference's train_HAR (client.py:114-131) trains size-1 batches and never aborts (1 / 0).
__device__ __forceinline__ int step_min_bs(const int* stepctl) { return stepctl ? stepctl[1] : 2; }
__device__ __forceinline__ bool step_nan_abort(const int* stepctl) { return stepctl ? stepctl[2] != 0 : true; }
__device__ __forceinline__ bool step_active(const int* bsz, const int* stepctl, int C, int S, const int* failed,
                                            int c, int* bs_out) {
  const int s = cur_step(stepctl);
  const int bs = s < S ? bsz[(long)s * C + c] : 0;
  *bs_out = bs;
  return bs >= step_min_bs(stepctl) && bs >= 1 && failed[c] == 0;
}

__global__ void __launch_bounds__(256) k_bce(const float* __restrict__ z, const float* __restrict__ y,
                                             const int* bsz, const int* epoch, const int* nb, const int* stepctl,
                                             int C, int B, int S, int* failed, float* losses, int E,
                                             float* __restrict__ dz) {
  __shared__ float red[4];
  const int c = blockIdx.x;
  int bs;
  const bool act = step_active(bsz, stepctl, C, S, failed, c, &bs);
  float l = 0.f;
  for (int b = threadIdx.x; b < B; b += 256) {
    if (act && b < bs) {
      const float p = 1.f / (1.f + expf(-z[(long)c * B + b]));
      const float t = y[(long)c * B + b];
      l -= t * fmaxf(logf(p), -100.f) + (1.f - t) * fmaxf(log1pf(-p), -100.f);
      if (p != p) l = p;  // keep NaN (fmaxf would swallow it)
    }
  }
  l = wave_sum(l);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = l;
  __syncthreads();
  const float loss = (red[0] + red[1] + red[2] + red[3]) / (float)max(bs, 1);
  const bool abort = step_nan_abort(stepctl);
  const bool nan = act && abort && (loss != loss);
  for (int b = threadIdx.x; b < B; b += 256) {
    float g = 0.f;
    if (act && !nan && b < bs) {
      // torch: BCE'(p) = (p - t) / max(p (1 - p), 1e-12), times sigmoid'(z) = p (1 - p)
      const float p = 1.f / (1.f + expf(-z[(long)c * B + b]));
      const float w = p * (1.f - p);
      g = (p - y[(long)c * B + b]) / fmaxf(w, 1e-12f) * w / (float)bs;
    }
    dz[(long)c * B + b] = g;
  }
  if (threadIdx.x == 0 && act) {
    if (nan)
      failed[c] = 1;
    else
      losses[(long)c * E + epoch[(long)cur_step(stepctl) * C + c]] += loss / (float)nb[c];
  }
}

__global__ void __launch_bounds__(256) k_ce(const float* __restrict__ logits, const long* __restrict__ y, int K,
                                            const int* bsz, const int* epoch, const int* nb, const int* stepctl, int C,
                                            int B, int S, int* failed, float* losses, int E, float* __restrict__ dz) {
  __shared__ float red[4];
  const int c = blockIdx.x;
  int bs;
  const bool act = step_active(bsz, stepctl, C, S, failed, c, &bs);
  float l = 0.f;
  for (int b = threadIdx.x; b < B; b += 256) {
    if (act && b < bs) {
      const float* x = logits + ((long)c * B + b) * K;
      float mx = x[0];
      for (int k = 1; k < K; ++k) mx = fmaxf(mx, x[k]);
      float se = 0.f;
      for (int k = 0; k < K; ++k) se += expf(x[k] - mx);
      l += logf(se) + mx - x[y[(long)c * B + b]];
      if (x[0] != x[0]) l = x[0];
    }
  }
  l = wave_sum(l);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = l;
  __syncthreads();
  const float loss = (red[0] + red[1] + red[2] + red[3]) / (float)max(bs, 1);
  const bool abort = step_nan_abort(stepctl);
  const bool nan = act && abort && (loss != loss);  // without abort a NaN loss keeps training (NaN gradient)
  for (int b = threadIdx.x; b < B; b += 256) {
    const float* x = logits + ((long)c * B + b) * K;
    float* d = dz + ((long)c * B + b) * K;
    if (act && !nan && b < bs) {
      float mx = x[0];
      for (int k = 1; k < K; ++k) mx = fmaxf(mx, x[k]);
      float se = 0.f;
      for (int k = 0; k < K; ++k) se += expf(x[k] - mx);
      const long t = y[(long)c * B + b];
      for (int k = 0; k < K; ++k) d[k] = (expf(x[k] - mx) / se - (k == t ? 1.f : 0.f)) / (float)bs;
    } else {
      for (int k = 0; k < K; ++k) d[k] = 0.f;
    }
  }
  if (threadIdx.x == 0 && act) {
    if (nan)
      failed[c] = 1;
    else
      losses[(long)c * E + epoch[(long)cur_step(stepctl) * C + c]] += loss / (float)nb[c];
  }
}

// ============================================================================ optimizer
// One client row per grid.y.  Each thread owns 4 consecutive entries starting at a 16-B aligned address of
// the row (the row start c*P need not be aligned: thread 0 also takes the unaligned head, the last
// thread the tail), so the row streams as float4 whatever P is.  The per-element arithmetic is the
// scalar form's (same bits); the bias corrections are computed once per thread.
__device__ __forceinline__ void adam1(float& pi, float& mi, float& vi, float gi, float a, float sb) {
  const float mn = mi + 0.1f * (gi - mi);
  const float vn = 0.999f * vi + 0.001f * gi * gi;
  mi = mn;
  vi = vn;
  pi -= a * mn / (sqrtf(vn) / sb + 1e-8f);
}
__global__ void __launch_bounds__(256) k_adam_clients(float* __restrict__ p, float* __restrict__ g,
                                                      float* __restrict__ m, float* __restrict__ v, long P,
                                                      const int* tcount, const int* bsz, const int* stepctl, int C,
                                                      int S, const int* failed, float lr, long skip_lo, long skip_hi,
                                                      float sgd_lr, int zero_g) {
  const int c = blockIdx.y;
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long row = (long)c * P;
  const long head = (4 - (row & 3)) & 3;  // entries before the first 16-B aligned one (arena base aligned)
  const long i0 = head + 4 * t;            // this thread's aligned group
  int bs;
  if ((t > 0 && i0 >= P) || !step_active(bsz, stepctl, C, S, failed, c, &bs)) return;
  float a = 0.f, sb = 1.f;
  if (sgd_lr <= 0.f) {
    const float tt = (float)(tcount[c] + 1);
    const float bc1 = 1.f - powf(0.9f, tt), bc2 = 1.f - powf(0.999f, tt);
    a = lr / bc1;
    sb = sqrtf(bc2);
  }
  auto one = [&](long i) {  // scalar entry i of the row
    if (i >= skip_lo && i < skip_hi) return;  // buffers (e.g. the positional-encoding table)
    const long k = row + i;
    const float gi = g[k];
    if (zero_g) g[k] = 0.f;  // the next step accumulates into a zeroed arena without a fill launch
    if (sgd_lr > 0.f) {
      p[k] -= sgd_lr * gi;
      return;
    }
    float pi = p[k], mi = m[k], vi = v[k];
    adam1(pi, mi, vi, gi, a, sb);
    m[k] = mi;
    v[k] = vi;
    p[k] = pi;
  };
  if (t == 0)
    for (long i = 0; i < head && i < P; ++i) one(i);
  if (i0 + 4 > P) {  // tail
    for (long i = i0; i < P; ++i) one(i);
    return;
  }
  if (i0 + 4 <= skip_lo || i0 >= skip_hi) {
    const long k = row + i0;
    f4v g4 = *(const f4v*)(g + k), p4 = *(const f4v*)(p + k);
    if (zero_g) *(f4v*)(g + k) = f4v{0.f, 0.f, 0.f, 0.f};
    if (sgd_lr > 0.f) {
      *(f4v*)(p + k) = p4 - sgd_lr * g4;
      return;
    }
    f4v m4 = *(const f4v*)(m + k), v4 = *(const f4v*)(v + k);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float pe = p4[e], me = m4[e], ve = v4[e];
      adam1(pe, me, ve, g4[e], a, sb);
      p4[e] = pe;
      m4[e] = me;
      v4[e] = ve;
    }
    *(f4v*)(m + k) = m4;
    *(f4v*)(v + k) = v4;
    *(f4v*)(p + k) = p4;
  } else {
    for (long i = i0; i < i0 + 4; ++i) one(i);
  }
}

__global__ void k_step_end(int* stepctl, int* tcount, const int* bsz, const int* failed, int C, int S) {
  const int c = threadIdx.x;
  int bs;
  const bool act = c < C && step_active(bsz, stepctl, C, S, failed, c, &bs);
  __syncthreads();
  if (act) tcount[c] += 1;
  __syncthreads();
  if (threadIdx.x == 0) stepctl[0] += 1;
}

// ============================================================================ HAR stem and pooling
// h[c][b*L+l][o] = conv_b[o] + sum_j conv_w[o][j] x[c][b][l+j-1] + pe[l][o]   (src/Model.py:431-452)
// One thread per (row, 4 channels): 32-bit row / position arithmetic (the per-element 64-bit divisions
// of the first version dominated), float4 stores of h / loads of dh.
__global__ void __launch_bounds__(256) k_conv_pe_fwd(const float* __restrict__ x, int C, int B, int L,
                                                     const float* __restrict__ params, long P, int w_off, int b_off,
                                                     int pe_off, float* __restrict__ h) {
  const int c = blockIdx.y;
  const int nrows = B * L;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int row = t >> 4, o0 = (t & 15) * 4;
  if (row >= nrows) return;
  const int l = row % L;
  const float* pp = params + (long)c * P;
  const float* xr = x + (long)c * nrows + (row - l);
  const float xm = l >= 1 ? xr[l - 1] : 0.f, x0 = xr[l], xp = l + 1 < L ? xr[l + 1] : 0.f;
  f4v v;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int o = o0 + e;
    const float* w = pp + w_off + o * 3;
    float s = pp[b_off + o] + pp[pe_off + l * 64 + o];
    if (l >= 1) s += w[0] * xm;
    s += w[1] * x0;
    if (l + 1 < L) s += w[2] * xp;
    v[e] = s;
  }
  *(f4v*)(h + ((long)c * nrows + row) * 64 + o0) = v;
}

// conv weight / bias gradients: 16 row groups x 16 lanes of 4 channels per workgroup, 1024 rows per workgroup
__global__ void __launch_bounds__(256) k_conv_pe_bwd(const float* __restrict__ x, const float* __restrict__ dh,
                                                     int C, int B, int L, float* __restrict__ grads, long P,
                                                     int w_off, int b_off, float* __restrict__ ws) {
  __shared__ float red[16][64][4];
  const int c = blockIdx.y, o0 = (threadIdx.x & 15) * 4, rg = threadIdx.x >> 4;
  const int nrows = B * L, r0 = blockIdx.x * 1024;
  float a[4][4] = {};  // [channel][tap 0..2, bias]
  int row = r0 + rg, l = row % L;
  const float* xc = x + (long)c * nrows;
  const float* dc = dh + (long)c * nrows * 64 + o0;
  const int rend = min(nrows, r0 + 1024);
  // two rows (row, row + 16) per iteration: both gradient loads in flight before either is used
  for (; row < rend; row += 32) {
    int l2 = l + 16;
    while (l2 >= L) l2 -= L;
    const bool two = row + 16 < rend;
    const f4v d = *(const f4v*)(dc + (long)row * 64);
    const f4v d2 = two ? *(const f4v*)(dc + (long)(row + 16) * 64) : f4v{0.f, 0.f, 0.f, 0.f};
    const float* xr = xc + (row - l);
    const float xm = l >= 1 ? xr[l - 1] : 0.f, x0 = xr[l], xp = l + 1 < L ? xr[l + 1] : 0.f;
    const float* xr2 = xc + (row + 16 - l2);
    const float xm2 = two && l2 >= 1 ? xr2[l2 - 1] : 0.f, x02 = two ? xr2[l2] : 0.f,
                xp2 = two && l2 + 1 < L ? xr2[l2 + 1] : 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      a[e][0] += d[e] * xm;
      a[e][1] += d[e] * x0;
      a[e][2] += d[e] * xp;
      a[e][3] += d[e];
    }
    if (two) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        a[e][0] += d2[e] * xm2;
        a[e][1] += d2[e] * x02;
        a[e][2] += d2[e] * xp2;
        a[e][3] += d2[e];
      }
    }
    l = l2 + 16;
    while (l >= L) l -= L;
  }
#pragma unroll
  for (int e = 0; e < 4; ++e)
#pragma unroll
    for (int q = 0; q < 4; ++q) red[rg][o0 + e][q] = a[e][q];
  __syncthreads();
  {
    const int o = threadIdx.x >> 2, q = threadIdx.x & 3;  // 64 channels x 4 sums
    float s = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) s += red[r][o][q];
    if (ws) {  // [block][C][192 taps | 64 biases]
      ws[((long)blockIdx.x * C + c) * 256 + (q < 3 ? o * 3 + q : 192 + o)] = s;
    } else {
      float* gp = grads + (long)c * P;
      atomicAdd(gp + (q < 3 ? w_off + o * 3 + q : b_off + o), s);
    }
  }
}

// mean over L of h [C*B][L][64]: one workgroup per (client, sample), 16 row groups x 16 lanes of float4
__global__ void __launch_bounds__(256) k_mean_rows_fwd(const float* __restrict__ h, int L, float* __restrict__ out) {
  __shared__ f4v red[16][16];
  const long cb = blockIdx.x;  // c * B + b
  const int q = threadIdx.x & 15, rg = threadIdx.x >> 4;
  const float* src = h + cb * L * 64 + 4 * q;
  f4v s = f4v{0.f, 0.f, 0.f, 0.f};
  for (int l = rg; l < L; l += 16) s += *(const f4v*)(src + (long)l * 64);
  red[rg][q] = s;
  __syncthreads();
  if (rg == 0) {
    f4v t = red[0][q];
#pragma unroll
    for (int r = 1; r < 16; ++r) t += red[r][q];
    *(f4v*)(out + cb * 64 + 4 * q) = t / (float)L;
  }
}

// dh[c, b, l, :] = dout[c, b, :] / L (float4 per thread)
__global__ void k_mean_rows_bwd(const float* __restrict__ dout, long n4, int L, float* __restrict__ dh) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n4) return;
  const int q = (int)(t & 15);
  const long cb = (t >> 4) / L;
  *(f4v*)(dh + 4 * t) = *(const f4v*)(dout + cb * 64 + 4 * q) / (float)L;
}

inline int launched() { return (int)hipGetLastError(); }
inline unsigned nb256(long n) { return (unsigned)((n + 255) / 256); }


// ============================================================================ tall-skinny GEMM
// C[c][m][n] (op)= epi(alpha * A[c][m][:K] . B[c][n][:K]) for K = 32 KT <= 256, N = 16 NT <= 256 and any M
// (the HAR layers: 72k rows per client, d_model 64, FFN 256).  k_bgemm re-stages B per 64x64 tile and
// writes the output as 4-byte column strips; here
//   * the whole B operand (<= 32 KB bf16) is staged ONCE per workgroup, rows padded to K+8 (conflict-free
//     16-B fragment reads);
//   * each wave streams 16-row tiles of A from global memory straight into MFMA fragments (two dwordx4
//     per lane per 32-k step: no LDS, no barriers); for K = 64 (PF) it issues the NEXT tile's loads before
//     this tile's MFMAs, for larger K the registers are worth more as occupancy (measured, tools/gemm_bench.py);
//   * the fragment reads of B stay inside the tile loop (hoisted they cost 2x the VGPRs and half the
//     occupancy: 0.25 -> 0.16 ms for the HAR qkv projection when they were moved back);
//   * it computes D^T = B . A^T, so each lane ends up holding 4 consecutive n of one row m: bias, G and the
//     output move as float4, the dropout hash pairs (afl_keep) are shared by adjacent n.
// Persistent: a client's workgroups stride over its row tiles (grid = (blocks per client, C)).
constexpr int TS_NTH = 256;
constexpr int TS_WAVES = TS_NTH / 64;

template <int NT, int KT, bool PF, bool CS>
__global__ void __launch_bounds__(TS_NTH) k_tsgemm(AflGemm g) {
  constexpr int N = 16 * NT, K = 32 * KT, LDB = K + 8;
  extern __shared__ __attribute__((aligned(16))) unsigned short Bs[];  // [N][LDB] bf16, then bias [N] fp32
  float* bias_s = reinterpret_cast<float*>(Bs + N * LDB);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int c = blockIdx.y;
  if (tid < N) bias_s[tid] = g.bias ? g.bias[(long)c * g.sbc + tid] : 0.f;
  {
    const float* B = g.B + (long)c * g.sBc;
    if (g.sBk == 1) {
      for (int e = tid; e < N * K; e += TS_NTH) {
        const int n = e / K, k = e - n * K;
        Bs[n * LDB + k] = (unsigned short)(pk_bf2(B[(long)n * g.sBn + k], 0.f) & 0xFFFFu);
      }
    } else {  // transposed view (dY.W): n is the contiguous index
      for (int e = tid; e < N * K; e += TS_NTH) {
        const int k = e / N, n = e - k * N;
        Bs[n * LDB + k] = (unsigned short)(pk_bf2(B[(long)n * g.sBn + (long)k * g.sBk], 0.f) & 0xFFFFu);
      }
    }
  }
  __syncthreads();
  const float* A = g.A + (long)c * g.sAc;
  float* Cc = g.Cm + (long)c * g.sCc;
  const int M = g.M, ntile = (M + 15) / 16, j = lane & 15, q = lane >> 4;
  const int wstride = gridDim.x * TS_WAVES;
  const bool dr = g.drop.thr16 != 0;
  const uint32_t key = dr ? drop_key(g.drop, c) : 0u;
  f4v xa[KT][2], xn[KT][2];
  auto load = [&](int t, f4v (&x)[KT][2]) {
    const int m = 16 * t + j;
    const bool ok = m < M;
    const float* p = A + (long)(ok ? m : 0) * g.sAm + 8 * q;
#pragma unroll
    for (int kk = 0; kk < KT; ++kk) {
      x[kk][0] = ok ? *(const f4v*)(p + 32 * kk) : f4v{0.f, 0.f, 0.f, 0.f};
      x[kk][1] = ok ? *(const f4v*)(p + 32 * kk + 4) : f4v{0.f, 0.f, 0.f, 0.f};
    }
  };
  f4v cs[CS ? KT : 1][2];  // CS: this lane's running column sums of A (rows j of its tiles, k = 32 kk + 8 q ..)
#pragma unroll
  for (int kk = 0; kk < (CS ? KT : 1); ++kk) cs[kk][0] = cs[kk][1] = f4v{0.f, 0.f, 0.f, 0.f};
  int t = blockIdx.x * TS_WAVES + wave;
  if (PF && t < ntile) load(t, xa);
  for (; t < ntile; t += wstride) {
    if (PF) {
      if (t + wstride < ntile) load(t + wstride, xn);  // next tile's A in flight during this tile's work
    } else {
      load(t, xa);
    }
    if constexpr (CS) {  // rows past M were loaded as zeros
#pragma unroll
      for (int kk = 0; kk < KT; ++kk) {
        cs[kk][0] += xa[kk][0];
        cs[kk][1] += xa[kk][1];
      }
    }
    s8v bx[KT];
#pragma unroll
    for (int kk = 0; kk < KT; ++kk) {
      u4v w;
      w[0] = pk_bf2(xa[kk][0][0], xa[kk][0][1]);
      w[1] = pk_bf2(xa[kk][0][2], xa[kk][0][3]);
      w[2] = pk_bf2(xa[kk][1][0], xa[kk][1][1]);
      w[3] = pk_bf2(xa[kk][1][2], xa[kk][1][3]);
      bx[kk] = __builtin_bit_cast(s8v, w);
    }
    f4v acc[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[nt] = f4v{0.f, 0.f, 0.f, 0.f};
    int boff = (16 * 0 + j) * LDB + 8 * q;
    asm volatile("" : "+v"(boff));  // keep the fragment reads in the loop (hoisted, they cost occupancy)
#pragma unroll
    for (int kk = 0; kk < KT; ++kk)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const s8v wf = *(const s8v*)(Bs + boff + 16 * nt * LDB + 32 * kk);
        acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf8v, wf),
                                                          __builtin_bit_cast(bf8v, bx[kk]), acc[nt], 0, 0, 0);
      }
    // lane holds C[m][16 nt + 4 q + e], e = 0..3
    const int m = 16 * t + j;
    if (m < M) {
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const int n0 = 16 * nt + 4 * q;
        f4v v = acc[nt] * g.alpha;
        if (g.bias) v += *(const f4v*)(bias_s + n0);
        const long off = (long)m * g.sCm + n0;
        if (g.Z) *(f4v*)(g.Z + (long)c * g.sCc + off) = v;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float x = act_f(v[e], g.act);
          if (dr) x *= drop_scale(g.drop, key, m, n0 + e);
          v[e] = x;
        }
        if (g.G) {
          const f4v gv = *(const f4v*)(g.G + (long)c * g.sGc + (long)m * g.sGm + n0);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] *= act_d(gv[e], g.gact);
        }
        if (g.accum == 1) v += *(const f4v*)(Cc + off);
        *(f4v*)(Cc + off) = v;
      }
    }
    if (PF) {
#pragma unroll
      for (int kk = 0; kk < KT; ++kk) {
        xa[kk][0] = xn[kk][0];
        xa[kk][1] = xn[kk][1];
      }
    }
  }
  if constexpr (CS) {
    // reduce over the 16 lanes of a q group, then over the waves (LDS, reusing the B image), one atomic
    // per column and workgroup
#pragma unroll
    for (int kk = 0; kk < KT; ++kk)
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float x = cs[kk][h][e];
          x += __shfl_xor(x, 1, 64);
          x += __shfl_xor(x, 2, 64);
          x += __shfl_xor(x, 4, 64);
          x += __shfl_xor(x, 8, 64);
          cs[kk][h][e] = x;
        }
    __syncthreads();  // every wave is done reading the B image
    float* red = reinterpret_cast<float*>(Bs);  // [TS_WAVES][K]
    if (j == 0) {
#pragma unroll
      for (int kk = 0; kk < KT; ++kk)
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int e = 0; e < 4; ++e) red[wave * K + 32 * kk + 8 * q + 4 * h + e] = cs[kk][h][e];
    }
    __syncthreads();
    if (tid < K) {
      float x = 0.f;
#pragma unroll
      for (int w = 0; w < TS_WAVES; ++w) x += red[w * K + tid];
      if (g.ws_sum)  // ordered partials [block][C][K] (deterministic)
        g.ws_sum[((long)blockIdx.x * g.nC + c) * K + tid] = x;
      else
        atomicAdd(g.asum + (long)c * g.sasc + tid, x);
    }
  }
}

__host__ __forceinline__ bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

constexpr int TS_ASUM_PARTS = 128;  // blocks per client of a k_tsgemm with ordered column-sum partials

// shapes with a k_tsgemm instantiation; anything else (or misaligned / strided operands) takes k_bgemm
int tsgemm_try(const AflGemm& g, hipStream_t s) {
  if (g.accum == 2 || g.splitk > 1 || g.sAk != 1 || g.sCn != 1) return -1;
  if (!al16(g.A) || (g.sAm & 3) || (g.sAc & 3) || !al16(g.Cm) || (g.sCm & 3) || (g.sCc & 3)) return -1;
  if (g.Z && !al16(g.Z)) return -1;
  if (g.G && (g.sGn != 1 || !al16(g.G) || (g.sGm & 3) || (g.sGc & 3))) return -1;
  const void* fn = nullptr;
  const int key = g.N * 1024 + g.K;
#define TS_CASE(N_, K_)                                         \
  case N_ * 1024 + K_:                                          \
    fn = g.asum ? (const void*)k_tsgemm<N_ / 16, K_ / 32, (K_ <= 64), true>      \
                : (const void*)k_tsgemm<N_ / 16, K_ / 32, (K_ <= 64), false>;    \
    break;
  switch (key) {
    TS_CASE(64, 64)
    TS_CASE(128, 64)
    TS_CASE(192, 64)
    TS_CASE(256, 64)
    TS_CASE(64, 128)
    TS_CASE(64, 192)
    TS_CASE(64, 256)
    default:
      return -1;
  }
#undef TS_CASE
  const int ntile = (g.M + 15) / 16;
  // with ordered column-sum partials the block count per client must not depend on how many clients share
  // the launch (the partials' summation order would change with the packing)
  const int per_client = g.asum && g.ws_sum ? max(1, min((ntile + TS_WAVES - 1) / TS_WAVES, TS_ASUM_PARTS))
                                            : max(1, min((ntile + TS_WAVES - 1) / TS_WAVES, (4 * 256 + g.nC - 1) / g.nC));
  const size_t lds = (size_t)g.N * (g.K + 8) * 2 + (size_t)g.N * 4;
  AflGemm gg = g;
  void* args[] = {&gg};
  const int e = (int)hipLaunchKernel(fn, dim3(per_client, g.nC), dim3(TS_NTH), args, lds, s);
  if (e == 0 && g.asum && g.ws_sum) partial_sum(g.ws_sum, per_client, g.nC, g.K, g.K, g.asum, g.sasc, s);
  return e;
}

}  // namespace

// ============================================================================ host launchers
int afl_bgemm(const AflGemm& g, hipStream_t s) {
  if (g.M <= 0 || g.N <= 0 || g.K <= 0 || g.nC <= 0) return 0;
  if (g.splitk > 1 && g.accum != 2) return (int)hipErrorInvalidValue;
  if (!g.no_ts && g.asum && g.N >= 256 && g.sAk == 1) {
    // N = 256: the fused column sums' 16 extra VGPRs drop k_tsgemm<16, 2> to one wave per SIMD
    // (HAR FFN-down dX 0.41 -> 0.64 ms); a separate column-sum pass (~0.09 ms) is cheaper there
    const int e = afl_colsum(g.A, g.sAc, g.sAm, g.M, g.K, g.nC, g.asum, g.sasc, s, g.ws_sum);
    if (e) return e;
    AflGemm g2 = g;
    g2.asum = nullptr;
    return afl_bgemm(g2, s);
  }
  if (!g.no_ts && tsgemm_try(g, s) == 0) return launched();
  if (g.asum) {  // the 64x64-tile kernel re-reads A per column tile: column sums as a separate pass
    if (g.sAk != 1) return (int)hipErrorInvalidValue;
    const int e = afl_colsum(g.A, g.sAc, g.sAm, g.M, g.K, g.nC, g.asum, g.sasc, s, g.ws_sum);
    if (e) return e;
  }
  const int tiles = ((g.M + GT - 1) / GT) * ((g.N + GT - 1) / GT);
  dim3 grid(tiles, max(1, g.splitk), g.nC);
  const bool det = g.ws != nullptr && g.accum == 2 && g.splitk > 1;
  const int kchunk = ((g.K + g.splitk - 1) / g.splitk + GK - 1) / GK * GK;
  const int nsplit = (g.K + kchunk - 1) / kchunk;  // splits with a non-empty k range (every one of them
                                                   // writes its whole partial tile)
  AflGemm gg = g;  // 16-B aligned k-contiguous rows take the vector-load path
  gg.avec = g.sAk == 1 && g.sAm % 4 == 0 && g.sAc % 4 == 0 && ((uintptr_t)g.A & 15) == 0;
  gg.bvec = g.sBk == 1 && g.sBn % 4 == 0 && g.sBc % 4 == 0 && ((uintptr_t)g.B & 15) == 0;
  const bool ak = g.sAk == 1, bk = g.sBk == 1;
  if (ak && bk)
    hipLaunchKernelGGL((k_bgemm<true, true>), grid, dim3(256), 0, s, gg);
  else if (ak)
    hipLaunchKernelGGL((k_bgemm<true, false>), grid, dim3(256), 0, s, gg);
  else if (bk)
    hipLaunchKernelGGL((k_bgemm<false, true>), grid, dim3(256), 0, s, gg);
  else
    hipLaunchKernelGGL((k_bgemm<false, false>), grid, dim3(256), 0, s, gg);
  if (det) {
    const long total = (long)g.nC * g.M * g.N;
    const int nb = (int)std::min<long>(2048, (total + 255) / 256);
    hipLaunchKernelGGL(k_split_sum, dim3(nb), dim3(256), 0, s, (const float*)g.ws, nsplit, g.nC, g.M, g.N, g.Cm,
                       g.sCc, g.sCm, g.sCn);
  }
  return launched();
}

long afl_bgemm_asum_ws_floats(const AflGemm& g) {
  if (!g.asum || g.M <= 0 || g.K <= 0 || g.nC <= 0) return 0;
  return (long)std::max<long>((g.M + 255) / 256, TS_ASUM_PARTS) * g.nC * g.K;
}

long afl_colsum_ws_floats(int M, int N, int nC) { return (long)((M + 255) / 256) * nC * N; }

long afl_bgemm_ws_floats(const AflGemm& g) {
  if (g.accum != 2 || g.splitk <= 1 || g.M <= 0 || g.N <= 0 || g.K <= 0 || g.nC <= 0) return 0;
  const int kchunk = ((g.K + g.splitk - 1) / g.splitk + GK - 1) / GK * GK;
  return (long)((g.K + kchunk - 1) / kchunk) * g.nC * g.M * g.N;
}

int afl_colsum(const float* Y, long sYc, long sYm, int M, int N, int nC, float* out, long sOc, hipStream_t s,
               float* ws) {
  hipLaunchKernelGGL(k_colsum, dim3((N + 63) / 64, (M + 255) / 256, nC), dim3(256), 0, s, Y, sYc, sYm, M, N, out, sOc,
                     ws);
  if (ws) partial_sum(ws, (M + 255) / 256, nC, N, N, out, sOc, s);
  return launched();
}

int afl_gather_icu(const float* rows, const int* idx, const int* stepctl, int C, int B, int mask, float* vit,
                   float* lab, float* y, hipStream_t s) {
  hipLaunchKernelGGL(k_gather_icu, dim3(nb256((long)C * B * 24)), dim3(256), 0, s, rows, idx, stepctl, C, B, mask, vit,
                     lab, y);
  return launched();
}

int afl_gather_har(const float* x, const long* y, int F, const int* idx, const int* stepctl, int C, int B, float* ox,
                   long* oy, hipStream_t s) {
  hipLaunchKernelGGL(k_gather_har, dim3(nb256((long)C * B * F)), dim3(256), 0, s, x, y, F, idx, stepctl, C, B, ox, oy);
  return launched();
}

int afl_im2col3(const float* x, long sXc, long sXr, int C, int B, int L, int Cin, float* out, hipStream_t s) {
  hipLaunchKernelGGL(k_im2col3, dim3(nb256((long)C * B * L * 3 * Cin)), dim3(256), 0, s, x, sXc, sXr, C, B, L, Cin,
                     out);
  return launched();
}

int afl_col2im3(const float* dcols, int C, int B, int L, int Cin, const float* relu_src, long sRc, long sRr, float* dx,
                hipStream_t s) {
  hipLaunchKernelGGL(k_col2im3, dim3(nb256((long)C * B * L * Cin)), dim3(256), 0, s, dcols, C, B, L, Cin, relu_src,
                     sRc, sRr, dx);
  return launched();
}

int afl_pool4_fwd(const float* h, int C, int B, int L, int Ch, float* out, long sOc, long sOr, int col0, AflDrop d,
                  hipStream_t s) {
  hipLaunchKernelGGL(k_pool4_fwd, dim3(nb256((long)C * B * Ch * 4)), dim3(256), 0, s, h, C, B, L, Ch, out, sOc, sOr,
                     col0, d);
  return launched();
}

int afl_pool4_bwd(const float* dout, long sOc, long sOr, int col0, const float* h, int C, int B, int L, int Ch,
                  float* dh, AflDrop d, hipStream_t s) {
  hipLaunchKernelGGL(k_pool4_bwd, dim3(nb256((long)C * B * L * Ch)), dim3(256), 0, s, dout, sOc, sOr, col0, h, C, B, L,
                     Ch, dh, d);
  return launched();
}

inline bool rows16(const void* p, long sc, long sr) { return (((uintptr_t)p & 15) | (sc & 3) | (sr & 3)) == 0; }
int afl_ln_fwd(const AflLn& l, hipStream_t s) {
  const bool v4 = rows16(l.x, l.sXc, l.sXr) && (!l.a || rows16(l.a, l.sAc, l.sAr)) && (!l.s || rows16(l.s, 0, 0)) &&
                  rows16(l.y, l.sYc, l.sYr);
  if (v4)
    hipLaunchKernelGGL(k_ln_fwd<true>, dim3((l.rows + 15) / 16, l.nC), dim3(256), 0, s, l);
  else
    hipLaunchKernelGGL(k_ln_fwd<false>, dim3((l.rows + 15) / 16, l.nC), dim3(256), 0, s, l);
  return launched();
}

int afl_ln_bwd(const AflLnB& l, hipStream_t s) {
  const bool v4 = rows16(l.dy, l.sDc, l.sDr) && rows16(l.s, l.sSc, l.sSr) && rows16(l.dx, l.sXc, l.sXr) &&
                  (!l.da || rows16(l.da, l.sAc, l.sAr));
  const int np = (l.rows + LNB_ROWS - 1) / LNB_ROWS;
  if (v4)
    hipLaunchKernelGGL(k_ln_bwd<true>, dim3(np, l.nC), dim3(256), 0, s, l);
  else
    hipLaunchKernelGGL(k_ln_bwd<false>, dim3(np, l.nC), dim3(256), 0, s, l);
  if (l.ws) {  // gamma / beta gradients: the row blocks' partials in block order
    partial_sum(l.ws, np, l.nC, 64, 128, l.dgamma, l.sPc, s);
    partial_sum(l.ws + 64, np, l.nC, 64, 128, l.dbeta, l.sPc, s);
  }
  return launched();
}

long afl_ln_bwd_ws_floats(int rows, int nC) { return (long)((rows + LNB_ROWS - 1) / LNB_ROWS) * nC * 128; }

int afl_gru_fwd(const float* gi, const float* bhh, long sPc, int C, int B, float* h, long sHc, long sHr, int col0,
                hipStream_t s) {
  hipLaunchKernelGGL(k_gru_fwd, dim3(nb256((long)C * B * 32)), dim3(256), 0, s, gi, bhh, sPc, C, B, h, sHc, sHr, col0);
  return launched();
}

int afl_gru_bwd(const float* dh, long sHc, long sHr, int col0, const float* gi, const float* bhh, long sPc, int C,
                int B, float* dgi, float* dbih, float* dbhh, hipStream_t s) {
  hipLaunchKernelGGL(k_gru_bwd, dim3(C), dim3(256), 0, s, dh, sHc, sHr, col0, gi, bhh, sPc, B, dgi, dbih, dbhh);
  return launched();
}

int afl_bce(const float* z, const float* y, const int* bsz, const int* epoch, const int* nb, const int* stepctl, int C,
            int B, int S, int* failed, float* losses, int E, float* dz, hipStream_t s) {
  hipLaunchKernelGGL(k_bce, dim3(C), dim3(256), 0, s, z, y, bsz, epoch, nb, stepctl, C, B, S, failed, losses, E, dz);
  return launched();
}

int afl_ce(const float* logits, const long* y, int K, const int* bsz, const int* epoch, const int* nb,
           const int* stepctl, int C, int B, int S, int* failed, float* losses, int E, float* dz, hipStream_t s) {
  hipLaunchKernelGGL(k_ce, dim3(C), dim3(256), 0, s, logits, y, K, bsz, epoch, nb, stepctl, C, B, S, failed, losses, E,
                     dz);
  return launched();
}

int afl_adam_clients(float* p, float* g, float* m, float* v, long P, int C, const int* tcount, const int* bsz,
                     const int* stepctl, int S, const int* failed, float lr, long skip_lo, long skip_hi, float sgd_lr,
                     int zero_g, hipStream_t s) {
  if ((((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) != 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_adam_clients, dim3(nb256(P / 4 + 1), C), dim3(256), 0, s, p, g, m, v, P, tcount, bsz, stepctl, C,
                     S, failed, lr, skip_lo, skip_hi, sgd_lr, zero_g);
  return launched();
}

int afl_step_end(int* stepctl, int* tcount, const int* bsz, const int* failed, int C, int S, hipStream_t s) {
  if (C > 1024) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_step_end, dim3(1), dim3(max(64, (C + 63) / 64 * 64)), 0, s, stepctl, tcount, bsz, failed, C, S);
  return launched();
}

int afl_conv_pe_fwd(const float* x, int C, int B, int L, const float* params, long P, int w_off, int b_off, int pe_off,
                    float* h, hipStream_t s) {
  if (((uintptr_t)h & 15) != 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_conv_pe_fwd, dim3(nb256((long)B * L * 16), C), dim3(256), 0, s, x, C, B, L, params, P, w_off,
                     b_off, pe_off, h);
  return launched();
}

int afl_conv_pe_bwd(const float* x, const float* dh, int C, int B, int L, float* grads, long P, int w_off, int b_off,
                    hipStream_t s, float* ws) {
  if (((uintptr_t)dh & 15) != 0) return (int)hipErrorInvalidValue;
  const int np = (int)(((long)B * L + 1023) / 1024);
  hipLaunchKernelGGL(k_conv_pe_bwd, dim3((unsigned)np, C), dim3(256), 0, s, x, dh, C, B, L, grads, P, w_off, b_off, ws);
  if (ws) {  // the stem's tap / bias gradients: row blocks' partials in block order
    partial_sum(ws, np, C, 192, 256, grads + w_off, P, s);
    partial_sum(ws + 192, np, C, 64, 256, grads + b_off, P, s);
  }
  return launched();
}

long afl_conv_pe_bwd_ws_floats(int C, int B, int L) { return (((long)B * L + 1023) / 1024) * C * 256; }

int afl_mean_rows_fwd(const float* h, int C, int B, int L, float* out, hipStream_t s) {
  if ((((uintptr_t)h | (uintptr_t)out) & 15) != 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_mean_rows_fwd, dim3(C * B), dim3(256), 0, s, h, L, out);
  return launched();
}

int afl_mean_rows_bwd(const float* dout, int C, int B, int L, float* dh, hipStream_t s) {
  if ((((uintptr_t)dout | (uintptr_t)dh) & 15) != 0) return (int)hipErrorInvalidValue;
  const long n4 = (long)C * B * L * 16;
  hipLaunchKernelGGL(k_mean_rows_bwd, dim3(nb256(n4)), dim3(256), 0, s, dout, n4, L, dh);
  return launched();
}
