// Packed-hypernetwork kernels (server-side ``hyper`` mode; reference server.py:637-678).
//
// The hypernet's per-tensor heads are ONE row-major matrix W[P][H] (H = hidden = 100) plus b[P].
//   k_hyper_rows     : delta = W f + b - u   and   dfeat = W^T delta, in ONE pass over W
//                      (generate mode: out = W f + b)
//   k_hyper_adam     : Adam on W and b with grad(W) = s * delta (x) f, grad(b) = s * delta,
//                      computed on the fly: the P x H gradient is never materialised.
// W is streamed once per kernel (memory bound: 19.5 MB for TransformerModel heads).
#include "common.h"
#include "kernels.h"

constexpr int HR_ROWS = 64;   // rows per tile
constexpr int HR_HMAX = 128;  // max hidden size supported

__global__ void __launch_bounds__(256) k_hyper_rows(const float* __restrict__ W, const float* __restrict__ b,
                                                    const float* __restrict__ f, const float* __restrict__ u, long P,
                                                    int H, float* __restrict__ out, float* __restrict__ partial,
                                                    int pstride) {
  __shared__ float tile[HR_ROWS * HR_HMAX];
  __shared__ float fs[HR_HMAX];
  __shared__ float ds[HR_ROWS];
  __shared__ float sq[4];
  const int tid = threadIdx.x;
  float dsq = 0.f;  // sum of delta^2 over this thread's rows (pstride == H + 1)
  if (tid < H) fs[tid] = f[tid];
  float acc = 0.f;  // dfeat[tid] partial (tid < H)
  const long ntiles = (P + HR_ROWS - 1) / HR_ROWS;
  for (long t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const long r0 = t * HR_ROWS;
    const int nr = (int)min((long)HR_ROWS, P - r0);
    __syncthreads();
    const float* src = W + r0 * H;
    for (int i = tid; i < nr * H; i += blockDim.x) tile[i] = src[i];
    __syncthreads();
    // 4 threads per row
    const int r = tid >> 2, q = tid & 3;
    float s = 0.f;
    if (r < nr)
      for (int h = q; h < H; h += 4) s += tile[r * H + h] * fs[h];
    s += __shfl_xor(s, 1, 64);
    s += __shfl_xor(s, 2, 64);
    if (r < nr && q == 0) {
      float val = s + b[r0 + r];
      if (u) val -= u[r0 + r];
      out[r0 + r] = val;
      ds[r] = val;
      dsq += val * val;
    }
    __syncthreads();
    if (u && tid < H) {
      for (int rr = 0; rr < nr; ++rr) acc += tile[rr * H + tid] * ds[rr];
    }
  }
  if (u && tid < H) partial[(long)blockIdx.x * pstride + tid] = acc;
  if (u && pstride > H) {
    for (int o = 32; o > 0; o >>= 1) dsq += __shfl_xor(dsq, o, 64);
    if ((tid & 63) == 0) sq[tid >> 6] = dsq;
    __syncthreads();
    if (tid == 0) partial[(long)blockIdx.x * pstride + H] = (sq[0] + sq[1]) + (sq[2] + sq[3]);
  }
}

// float4 variant (H % 4 == 0, H <= 128, 16-B aligned W): no LDS staging.  A half-wave owns one row at a
// time (lane j holds columns 4j..4j+3 and the matching f in registers), dots reduce inside the half,
// each lane accumulates its 4 columns of W^T delta in registers; 4 rows per half in flight.
constexpr int HR4_NT = 1024;  // 16 waves: 4 per SIMD over the 256-block grid (the partials layout caps the grid)
constexpr int HR4_U = 4;
__global__ void __launch_bounds__(HR4_NT) k_hyper_rows4(const float* __restrict__ W, const float* __restrict__ b,
                                                        const float* __restrict__ f, const float* __restrict__ u,
                                                        long P, int H, float* __restrict__ out,
                                                        float* __restrict__ partial, int pstride) {
  __shared__ float red[HR4_NT / 64][HR_HMAX];
  __shared__ float sq[HR4_NT / 64];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int j = lane & 31, half = lane >> 5, H4 = H >> 2;
  const bool act = j < H4;
  const float4 fv = act ? reinterpret_cast<const float4*>(f)[j] : make_float4(0.f, 0.f, 0.f, 0.f);
  const float4* W4 = reinterpret_cast<const float4*>(W);
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  float dsq = 0.f;
  const long nslots = 2L * gridDim.x * (HR4_NT / 64);  // row slots per sweep
  const long slot = 2L * ((long)blockIdx.x * (HR4_NT / 64) + wv) + half;
  for (long r0 = slot; r0 < P; r0 += HR4_U * nslots) {
    float4 w[HR4_U];
#pragma unroll
    for (int q = 0; q < HR4_U; ++q) {
      const long r = r0 + q * nslots;
      w[q] = (act && r < P) ? W4[r * H4 + j] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int q = 0; q < HR4_U; ++q) {
      const long r = r0 + q * nslots;
      float d = w[q].x * fv.x + w[q].y * fv.y + w[q].z * fv.z + w[q].w * fv.w;
#pragma unroll
      for (int o = 16; o > 0; o >>= 1) d += __shfl_xor(d, o, 64);
      if (r < P) {
        float val = d + b[r];
        if (u) val -= u[r];
        if (j == 0) {
          out[r] = val;
          dsq += val * val;
        }
        acc.x += w[q].x * val;
        acc.y += w[q].y * val;
        acc.z += w[q].z * val;
        acc.w += w[q].w * val;
      }
    }
  }
  if (!u) return;
  acc.x += __shfl_xor(acc.x, 32, 64);
  acc.y += __shfl_xor(acc.y, 32, 64);
  acc.z += __shfl_xor(acc.z, 32, 64);
  acc.w += __shfl_xor(acc.w, 32, 64);
  if (half == 0 && act) {
    red[wv][4 * j] = acc.x;
    red[wv][4 * j + 1] = acc.y;
    red[wv][4 * j + 2] = acc.z;
    red[wv][4 * j + 3] = acc.w;
  }
  dsq = wave_sum(dsq);
  if (lane == 0) sq[wv] = dsq;
  __syncthreads();
  if (tid < H) {
    float a = 0.f;
#pragma unroll
    for (int k = 0; k < HR4_NT / 64; ++k) a += red[k][tid];
    partial[(long)blockIdx.x * pstride + tid] = a;
  }
  if (pstride > H && tid == 0) {
    float a = 0.f;
#pragma unroll
    for (int k = 0; k < HR4_NT / 64; ++k) a += sq[k];
    partial[(long)blockIdx.x * pstride + H] = a;
  }
}

__device__ __host__ inline bool hyper_rows4_ok(const float* W, const float* f, int H) {
  return (H & 3) == 0 && H <= HR_HMAX && (((uintptr_t)W | (uintptr_t)f) & 15) == 0;
}

__global__ void k_hyper_reduce(const float* __restrict__ partial, int nb, int H, float* __restrict__ dfeat) {
  int h = threadIdx.x;
  if (h >= H) return;
  double a = 0.0;
  for (int i = 0; i < nb; ++i) a += partial[(long)i * H + h];
  dfeat[h] = (float)a;
}

int afl_hyper_nblocks(long P) { return (int)min(256L, (P + HR_ROWS - 1) / HR_ROWS); }

void afl_hyper_rows(const float* W, const float* b, const float* f, const float* u, long P, int H, float* out,
                    float* partial, float* dfeat, hipStream_t s) {
  int nb = afl_hyper_nblocks(P);
  if (hyper_rows4_ok(W, f, H))
    hipLaunchKernelGGL(k_hyper_rows4, dim3(nb), dim3(HR4_NT), 0, s, W, b, f, u, P, H, out, partial, H);
  else
    hipLaunchKernelGGL(k_hyper_rows, dim3(nb), dim3(256), 0, s, W, b, f, u, P, H, out, partial, H);
  if (u) hipLaunchKernelGGL(k_hyper_reduce, dim3(1), dim3(128), 0, s, partial, nb, H, dfeat);
}

__global__ void __launch_bounds__(256) k_hyper_adam(float* __restrict__ W, float* __restrict__ bvec,
                                                    float* __restrict__ m, float* __restrict__ v,
                                                    const float* __restrict__ delta, const float* __restrict__ f,
                                                    long P, int H, float lr_bc1, float rsqrt_bc2, float b1, float b2,
                                                    float eps, float gs) {
  const long nW = P * H;
  const long total = nW + P;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    float g, p;
    if (i < nW) {
      long r = i / H;
      int h = (int)(i - r * H);
      g = gs * delta[r] * f[h];
      p = W[i];
    } else {
      g = gs * delta[i - nW];
      p = bvec[i - nW];
    }
    float mi = m[i] + (1.f - b1) * (g - m[i]);
    float vi = b2 * v[i] + (1.f - b2) * g * g;
    m[i] = mi;
    v[i] = vi;
    p -= lr_bc1 * mi / (sqrtf(vi) * rsqrt_bc2 + eps);
    if (i < nW) W[i] = p;
    else bvec[i - nW] = p;
  }
}

void afl_hyper_adam(float* W, float* bvec, float* m, float* v, const float* delta, const float* f, long P, int H,
                    int step, float lr, float b1, float b2, float eps, float gs, hipStream_t s) {
  double bc1 = 1.0 - pow((double)b1, step), bc2 = 1.0 - pow((double)b2, step);
  long total = P * H + P;
  int nb = (int)min(8192L, (total + 255) / 256);
  hipLaunchKernelGGL(k_hyper_adam, dim3(nb), dim3(256), 0, s, W, bvec, m, v, delta, f, P, H, (float)(lr / bc1),
                     (float)(1.0 / sqrt(bc2)), b1, b2, eps, gs);
}

// ------------------------------------------------------------------------------------------------
// Sync-free sequential server update: per selected client c_k, three launches and no host round trip
//   rows   : delta = W f + b - u,  partial W^T delta and |delta|^2 per block        (streams W once)
//   small  : one workgroup: reduce partials, recompute the MLP activations of c_k, back-propagate
//            into the embedding + MLP, global grad norm (head part in closed form:
//            |delta (x) f|^2 = |delta|^2 |f|^2), clip coefficient -> device scalar, Adam on the
//            embedding+MLP region, then the features f of c_{k+1} with the updated MLP
//   head   : Adam on W, b with grad = scale * delta (x) f computed on the fly (float4 streams)
// ------------------------------------------------------------------------------------------------
constexpr int HS_HMAX = 128;
constexpr int HS_LMAX = 8;
constexpr int HS_NT = 1024;          // threads of the small-net workgroup (16 waves)
constexpr int HS_SMEM = 28 * 1024;   // floats of embedding + MLP parameters staged in LDS (112 KB)
constexpr int HS_PF = 6;             // float4 moment chunks per thread held for the flat Adam (24 K floats)

// stage n floats (16-byte aligned source and destination when n4 mode) into LDS with every load of a thread in
// flight: clamped indices (a conditional load per slot made the compiler keep the batch in scratch and wait for
// each load in turn: 8 serial round trips per batch)
__device__ __forceinline__ void hs_stage(float* __restrict__ dst, const float* __restrict__ src, long n) {
  const int tid = threadIdx.x;
  if (n <= 0) return;
  if ((reinterpret_cast<uintptr_t>(src) & 15) == 0 && (n & 3) == 0) {
    const float4* s4 = reinterpret_cast<const float4*>(src);
    float4* d4 = reinterpret_cast<float4*>(dst);
    const long n4 = n / 4;
    for (long e0 = tid; e0 < n4; e0 += 8 * HS_NT) {
      float4 t[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const long e = e0 + q * HS_NT;
        t[q] = s4[e < n4 ? e : n4 - 1];
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const long e = e0 + q * HS_NT;
        if (e < n4) d4[e] = t[q];
      }
    }
  } else {
    for (long e0 = tid; e0 < n; e0 += 8 * HS_NT) {
      float t[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const long e = e0 + q * HS_NT;
        t[q] = src[e < n ? e : n - 1];
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const long e = e0 + q * HS_NT;
        if (e < n) dst[e] = t[q];
      }
    }
  }
}

// a list of client indices passed by value (the generation / feature kernels)
constexpr int HF_MAXC = 64;
struct HyClients {
  int c[HF_MAXC];
};

// relu that keeps NaN like torch.relu
__device__ __forceinline__ float hs_relu(float z) { return z < 0.f ? 0.f : z; }

// sum over the 8 lanes of an aligned lane group (all inside one wave)
__device__ __forceinline__ float hs_sum8(float x) {
  x += __shfl_xor(x, 1, 64);
  x += __shfl_xor(x, 2, 64);
  x += __shfl_xor(x, 4, 64);
  return x;
}

__device__ __forceinline__ float hs_wave_sum(float x) {
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
  return x;
}

// MLP forward of client c from the LDS copy (sm = the arena from d.emb on) -> acts[0..L]
// 8 lanes per output neuron.  sm holds the whole small region [d.emb, offW): embedding table and MLP (the
// embedding row came from global memory before, one load round trip per forward)
__device__ void hs_forward(const float* sm, const HySmallDesc& d, int c, float (*acts)[HS_HMAX]) {
  const int tid = threadIdx.x;
  if (tid < d.E) acts[0][tid] = sm[(long)c * d.E + tid];
  __syncthreads();
  const long base = d.emb;
  const int o = tid >> 3, sub = tid & 7;
  int din = d.E;
  for (int l = 0; l < d.L; ++l) {
    float acc = 0.f;
    if (o < d.H) {
      const float* w = sm + (d.w[l] - base) + (long)o * din;
      for (int k = sub; k < din; k += 8) acc = fmaf(w[k], acts[l][k], acc);
    }
    acc = hs_sum8(acc);
    if (o < d.H && sub == 0) {
      const float z = acc + sm[d.b[l] - base + o];
      acts[l + 1][o] = (l < d.L - 1) ? hs_relu(z) : z;
    }
    __syncthreads();
    din = d.H;
  }
}

// Adam on one element (gradient already scaled).  Every fused multiply-add is spelled out: the head update runs
// in three kernels (k_hyper_adam_v, k_hyper_adam_rows4, k_hyper_gen4) that must agree bitwise, which the
// compiler's own contraction choices do not promise across differently shaped kernels.
__device__ __forceinline__ float hs_adam(float p, float g, float& mm, float& vv, float lr_bc1, float rsqrt_bc2,
                                         float b1, float b2, float eps) {
#pragma clang fp contract(off)  // (g - mm must not absorb the caller's product that formed g)
  mm = __builtin_fmaf(1.f - b1, g - mm, mm);
  vv = __builtin_fmaf((1.f - b2) * g, g, b2 * vv);
  return p - (lr_bc1 * mm) / __builtin_fmaf(__builtin_sqrtf(vv), rsqrt_bc2, eps);
}

template <bool FLAT>
__global__ void __launch_bounds__(HS_NT) k_hyper_small(float* __restrict__ A, float* __restrict__ m,
                                                       float* __restrict__ v, const float* __restrict__ partial,
                                                       int nb, int ci, int cj, float* __restrict__ feat_j,
                                                       float* __restrict__ info, HySmallDesc d, long nsmall,
                                                       float clip, float lr_bc1, float rsqrt_bc2, float b1, float b2,
                                                       float eps, const int* __restrict__ enable, HyClients gen,
                                                       int ngen, float* __restrict__ gen_feat) {
  // enable (device word, optional): 0 = the round failed, leave the hypernetwork untouched (the engine enqueues
  // the update before it knows; FLEngine._early_launch).  gen / ngen: after the update, the MLP features of the
  // next generation's clients -> gen_feat [ngen, H] (from the untouched MLP when the update is disabled)
  const bool upd = enable == nullptr || *enable != 0;
  if (!upd && ngen == 0) return;
  __shared__ __attribute__((aligned(16))) float sm[HS_SMEM];
  __shared__ float acts[HS_LMAX + 1][HS_HMAX];
  __shared__ float dz[HS_LMAX][HS_HMAX];  // dL/d(output of layer l)
  __shared__ float gemb[HS_HMAX];
  __shared__ float red[HS_NT / 64][4];
  __shared__ float sc;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int H = d.H, L = d.L, E = d.E;
  const long base = d.emb;  // sm = [emb | mlp0.W | mlp0.b | ...] (nsmall floats)
  // the rows kernel's per-block partials (nb <= 256): 8 lanes per column, all 32 loads of a lane in flight and
  // issued ahead of the staging loads below (the two latencies overlap; summed in the same order as before)
  float pt[32];
  {
    const int c = tid >> 3, sub = tid & 7;
#pragma unroll
    for (int k = 0; k < 32; ++k) {
      const int bb = sub + 8 * k;
      pt[k] = (ci >= 0 && c <= H && bb < nb) ? partial[(long)bb * (H + 1) + c] : 0.f;
    }
  }
  // stage the embedding table and the MLP parameters (contiguous [emb, w_0 .. b_{L-1}]) in LDS
  hs_stage(sm, A + base, nsmall);
  // flat Adam over the whole small region (float4 chunks, every segment a multiple of 4 floats): the moments of
  // this thread's chunks are loaded ahead of the forward / backward passes (the per-segment loops waited for
  // seven load round trips after them)
  const long nemb = (long)d.n_nodes * E;
  const long n4s = nsmall / 4;
  constexpr bool flat = FLAT;  // (hs_flat_ok on the host)
  float4 pm[HS_PF], pv[HS_PF];
  if (ci >= 0 && upd) {
    // reduce the rows kernel's per-block partials: 8 lanes per column (W^T delta [H] and |delta|^2)
    {
      const int c = tid >> 3, sub = tid & 7;
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < 32; ++k) s += pt[k];  // (zeros past nb: adding +0.0 leaves every partial sum unchanged)
      s = hs_sum8(s);
      if (c <= H && sub == 0) {
        if (c < H) dz[L - 1][c] = s;
        else sc = s;  // |delta|^2 (sc is rewritten with the clip scale below)
      }
    }
    if (flat) {  // (after the partials are summed: their registers are free again)
      const float4* m4 = reinterpret_cast<const float4*>(m + base);
      const float4* v4 = reinterpret_cast<const float4*>(v + base);
#pragma unroll
      for (int i = 0; i < HS_PF; ++i) {
        const long c = tid + (long)i * HS_NT < n4s ? tid + (long)i * HS_NT : n4s - 1;  // (clamped: all in flight)
        pm[i] = m4[c];
        pv[i] = v4[c];
      }
    }
    hs_forward(sm, d, ci, acts);  // its barriers publish sm, dz[L-1] and sc
    const float dd = sc;
    for (int l = L - 1; l >= 0; --l) {
      const int din = l == 0 ? E : H;
      const int k = tid >> 3, sub = tid & 7;
      float da = 0.f;
      if (k < din) {
        const float* w = sm + (d.w[l] - base) + k;
        for (int o = sub; o < H; o += 8) da = fmaf(w[(long)o * din], dz[l][o], da);
      }
      da = hs_sum8(da);
      if (k < din && sub == 0) {
        if (l > 0) dz[l - 1][k] = acts[l][k] > 0.f ? da : 0.f;
        else gemb[k] = da;
      }
      __syncthreads();
    }
    // squared norms (wave 0): sum_l |dz_l|^2 (|a_l|^2 + 1) + |gemb|^2 ; |f|^2
    if (wv == 0) {
      float small = 0.f;
      for (int l = 0; l < L; ++l) {
        const int din = l == 0 ? E : H;
        float dzs = 0.f, as = 0.f;
        for (int k = lane; k < H; k += 64) dzs += dz[l][k] * dz[l][k];
        for (int k = lane; k < din; k += 64) as += acts[l][k] * acts[l][k];
        small += hs_wave_sum(dzs) * (hs_wave_sum(as) + 1.f);
      }
      float ff = 0.f, ge = 0.f;
      for (int k = lane; k < H; k += 64) ff += acts[L][k] * acts[L][k];
      for (int k = lane; k < E; k += 64) ge += gemb[k] * gemb[k];
      ff = hs_wave_sum(ff);
      ge = hs_wave_sum(ge);
      if (lane == 0) {
        const float total = sqrtf(dd * ff + dd + small + ge);
        float scale = 1.f;
        if (clip > 0.f) {
          const float coef = clip / (total + 1e-6f);
          if (coef < 1.f) scale = coef;
        }
        red[0][0] = scale;
        info[0] = total;
        info[1] = scale;
      }
    }
    __syncthreads();
    const float gs = red[0][0];
    if (flat) {
      // one float4 chunk of [emb | mlp0.W | mlp0.b | ...] per step: parameters from LDS, moments from the
      // registers loaded above; the global arena, the moments and the LDS copy (the next forward) written back
      float4* m4 = reinterpret_cast<float4*>(m + base);
      float4* v4 = reinterpret_cast<float4*>(v + base);
      float4* A4 = reinterpret_cast<float4*>(A + base);
      float4* s4 = reinterpret_cast<float4*>(sm);
#pragma unroll
      for (int i = 0; i < HS_PF; ++i) {
        const long c = tid + (long)i * HS_NT;
        if (c >= n4s) continue;
        const long x = 4 * c;
        float4 g;
        if (x < nemb) {  // embedding (zero-gradient rows still move: torch's dense Embedding grad)
          const int row = (int)(x / E), col = (int)(x - (long)row * E);
          g = row == ci ? make_float4(gs * gemb[col], gs * gemb[col + 1], gs * gemb[col + 2], gs * gemb[col + 3])
                        : make_float4(0.f, 0.f, 0.f, 0.f);
        } else {
          int l = 0;
          long ow = d.w[0] - base, ob = d.b[0] - base;
#pragma unroll
          for (int q = 1; q < HS_LMAX; ++q)  // (unrolled: no dynamic index into the by-value descriptor)
            if (q < L && x >= d.w[q] - base) {
              l = q;
              ow = d.w[q] - base;
              ob = d.b[q] - base;
            }
          if (x < ob) {  // W of layer l: row o, columns k..k+3 (din % 4 == 0)
            const int din = l == 0 ? E : H;
            const int o = (int)((x - ow) / din), k = (int)(x - ow - (long)o * din);
            const float go = gs * dz[l][o];
            g = make_float4(go * acts[l][k], go * acts[l][k + 1], go * acts[l][k + 2], go * acts[l][k + 3]);
          } else {  // bias of layer l
            const int o = (int)(x - ob);
            g = make_float4(gs * dz[l][o], gs * dz[l][o + 1], gs * dz[l][o + 2], gs * dz[l][o + 3]);
          }
        }
        float4 p = s4[c];
        p.x = hs_adam(p.x, g.x, pm[i].x, pv[i].x, lr_bc1, rsqrt_bc2, b1, b2, eps);
        p.y = hs_adam(p.y, g.y, pm[i].y, pv[i].y, lr_bc1, rsqrt_bc2, b1, b2, eps);
        p.z = hs_adam(p.z, g.z, pm[i].z, pv[i].z, lr_bc1, rsqrt_bc2, b1, b2, eps);
        p.w = hs_adam(p.w, g.w, pm[i].w, pv[i].w, lr_bc1, rsqrt_bc2, b1, b2, eps);
        m4[c] = pm[i];
        v4[c] = pv[i];
        A4[c] = p;
        s4[c] = p;
      }
      __syncthreads();  // the LDS copy updated for the next forward
    } else {
    // Adam over the embedding table (zero-gradient rows still move: torch's dense Embedding grad)
    for (long e = tid; e < nemb; e += HS_NT) {
      const int row = (int)(e / E), col = (int)(e - (long)row * E);
      float mm = m[d.emb + e], vv = v[d.emb + e];
      const float p = hs_adam(sm[e], row == ci ? gs * gemb[col] : 0.f, mm, vv, lr_bc1, rsqrt_bc2, b1, b2, eps);
      m[d.emb + e] = mm;
      v[d.emb + e] = vv;
      A[d.emb + e] = p;
      sm[e] = p;
    }
    // Adam over the MLP (params from LDS, moments streamed; the LDS copy is updated for the next forward)
    for (int l = 0; l < L; ++l) {
      const int din = l == 0 ? E : H;
      const long ow = d.w[l] - base, ob = d.b[l] - base;
      const long nw = (long)H * din;
      if (((d.w[l] | nw | din | ow) & 3) == 0) {  // float4 moments / params, 4 chunks in flight per thread
        const long n4 = nw / 4;
        float4* m4 = reinterpret_cast<float4*>(m + d.w[l]);
        float4* v4 = reinterpret_cast<float4*>(v + d.w[l]);
        float4* A4 = reinterpret_cast<float4*>(A + d.w[l]);
        float4* s4 = reinterpret_cast<float4*>(sm + ow);
        for (long e0 = tid; e0 < n4; e0 += 4 * HS_NT) {
          float4 mm[4], vv[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {  // (clamped: every load of the batch in flight, see hs_stage)
            const long e = e0 + q * HS_NT < n4 ? e0 + q * HS_NT : n4 - 1;
            mm[q] = m4[e];
            vv[q] = v4[e];
          }
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const long e4 = e0 + q * HS_NT;
            if (e4 >= n4) continue;
            const int o = (int)(4 * e4 / din), k = (int)(4 * e4 - (long)o * din);
            const float go = gs * dz[l][o];
            float4 p = s4[e4];
            p.x = hs_adam(p.x, go * acts[l][k], mm[q].x, vv[q].x, lr_bc1, rsqrt_bc2, b1, b2, eps);
            p.y = hs_adam(p.y, go * acts[l][k + 1], mm[q].y, vv[q].y, lr_bc1, rsqrt_bc2, b1, b2, eps);
            p.z = hs_adam(p.z, go * acts[l][k + 2], mm[q].z, vv[q].z, lr_bc1, rsqrt_bc2, b1, b2, eps);
            p.w = hs_adam(p.w, go * acts[l][k + 3], mm[q].w, vv[q].w, lr_bc1, rsqrt_bc2, b1, b2, eps);
            m4[e4] = mm[q];
            v4[e4] = vv[q];
            A4[e4] = p;
            s4[e4] = p;
          }
        }
      } else {
#pragma unroll 4
      for (long e = tid; e < nw; e += HS_NT) {
        const int o = (int)(e / din), k = (int)(e - (long)o * din);
        const long ge = d.w[l] + e;
        float mm = m[ge], vv = v[ge];
        const float p = hs_adam(sm[ow + e], gs * dz[l][o] * acts[l][k], mm, vv, lr_bc1, rsqrt_bc2, b1, b2, eps);
        m[ge] = mm;
        v[ge] = vv;
        A[ge] = p;
        sm[ow + e] = p;
      }
      }
      for (int o = tid; o < H; o += HS_NT) {
        const long ge = d.b[l] + o;
        float mm = m[ge], vv = v[ge];
        const float p = hs_adam(sm[ob + o], gs * dz[l][o], mm, vv, lr_bc1, rsqrt_bc2, b1, b2, eps);
        m[ge] = mm;
        v[ge] = vv;
        A[ge] = p;
        sm[ob + o] = p;
      }
    }
    __syncthreads();  // updated LDS embedding and MLP visible
    }
  }
  if (cj >= 0 && upd) {
    hs_forward(sm, d, cj, acts);
    if (tid < H) feat_j[tid] = acts[L][tid];
  }
  for (int k = 0; k < ngen; ++k) {
    hs_forward(sm, d, gen.c[k], acts);  // (its first barrier also orders the previous reads of acts)
    if (tid < H) gen_feat[(long)k * H + tid] = acts[L][tid];
  }
}

// Client k's head Adam (grad = (*gsp) * delta_k (x) f_k, as k_hyper_adam_v) FUSED with client k+1's rows
// pass (k_hyper_rows4) over the rows it has just updated: delta_n = W' f_n + b' - u_n, per-block partials of
// W'^T delta_n and |delta_n|^2.  One sweep over the [P, H] heads per client instead of two (the heads are
// 19.5 MB for TransformerModel; the rows pass needs the updated rows, which this thread holds in registers).
// Same row mapping as k_hyper_rows4, same partial layout (k_hyper_small reduces it), same arithmetic as the
// two kernels it replaces.
constexpr int HA_U = 2;  // rows per half-wave in flight (4 spilled at the 128-VGPR cap of 16-wave blocks)
__global__ void __launch_bounds__(HR4_NT) k_hyper_adam_rows4(float* __restrict__ W, float* __restrict__ b,
                                                             float* __restrict__ m, float* __restrict__ v,
                                                             const float* __restrict__ delta_k,
                                                             const float* __restrict__ f_k,
                                                             const float* __restrict__ gsp,
                                                             const float* __restrict__ f_n,
                                                             const float* __restrict__ u_n,
                                                             float* __restrict__ delta_n, float* __restrict__ partial,
                                                             long P, int H, float lr_bc1, float rsqrt_bc2, float b1,
                                                             float b2, float eps, const int* __restrict__ enable) {
  if (enable != nullptr && *enable == 0) return;
  __shared__ float red[HR4_NT / 64][HR_HMAX];
  __shared__ float sq[HR4_NT / 64];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int j = lane & 31, half = lane >> 5, H4 = H >> 2;
  const bool act = j < H4;
  const float4 fk = act ? reinterpret_cast<const float4*>(f_k)[j] : make_float4(0.f, 0.f, 0.f, 0.f);
  const float4 fn = act ? reinterpret_cast<const float4*>(f_n)[j] : make_float4(0.f, 0.f, 0.f, 0.f);
  const float gs = *gsp;
  float4* W4 = reinterpret_cast<float4*>(W);
  float4* m4 = reinterpret_cast<float4*>(m);
  float4* v4 = reinterpret_cast<float4*>(v);
  const long nW = P * H;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  float dsq = 0.f;
  const long nslots = 2L * gridDim.x * (HR4_NT / 64);
  const long slot = 2L * ((long)blockIdx.x * (HR4_NT / 64) + wv) + half;
  for (long r0 = slot; r0 < P; r0 += HA_U * nslots) {
    float4 w[HA_U], mm[HA_U], vv[HA_U];
#pragma unroll
    for (int q = 0; q < HA_U; ++q) {  // (clamped rows / columns: every load of the batch in flight, no scratch)
      const long r = r0 + q * nslots < P ? r0 + q * nslots : P - 1;
      const long e = r * H4 + (act ? j : 0);
      w[q] = W4[e];
      mm[q] = m4[e];
      vv[q] = v4[e];
    }
#pragma unroll
    for (int q = 0; q < HA_U; ++q) {
      const long r = r0 + q * nslots;
      const bool rv = r < P;  // (no early exit: the half-wave reduction below needs every lane of the half)
      const long rr = rv ? r : P - 1;
      if (!act) w[q] = make_float4(0.f, 0.f, 0.f, 0.f);
      const float dr = gs * delta_k[rr];
      {  // head Adam on this lane's 4 columns (k_hyper_adam_v)
        w[q].x = hs_adam(w[q].x, dr * fk.x, mm[q].x, vv[q].x, lr_bc1, rsqrt_bc2, b1, b2, eps);
        w[q].y = hs_adam(w[q].y, dr * fk.y, mm[q].y, vv[q].y, lr_bc1, rsqrt_bc2, b1, b2, eps);
        w[q].z = hs_adam(w[q].z, dr * fk.z, mm[q].z, vv[q].z, lr_bc1, rsqrt_bc2, b1, b2, eps);
        w[q].w = hs_adam(w[q].w, dr * fk.w, mm[q].w, vv[q].w, lr_bc1, rsqrt_bc2, b1, b2, eps);
        if (act && rv) {
          W4[r * H4 + j] = w[q];
          m4[r * H4 + j] = mm[q];
          v4[r * H4 + j] = vv[q];
        }
      }
      // bias Adam (every lane of the half computes it, lane 0 stores)
      float bm = m[nW + rr], bv = v[nW + rr];
      const float bn = hs_adam(b[rr], dr, bm, bv, lr_bc1, rsqrt_bc2, b1, b2, eps);
      // client k+1's rows pass on the updated row
      float d = w[q].x * fn.x + w[q].y * fn.y + w[q].z * fn.z + w[q].w * fn.w;
#pragma unroll
      for (int o = 16; o > 0; o >>= 1) d += __shfl_xor(d, o, 64);
      if (!rv) continue;
      float val = d + bn;
      val -= u_n[r];
      if (j == 0) {
        m[nW + r] = bm;
        v[nW + r] = bv;
        b[r] = bn;
        delta_n[r] = val;
        dsq += val * val;
      }
      acc.x += w[q].x * val;
      acc.y += w[q].y * val;
      acc.z += w[q].z * val;
      acc.w += w[q].w * val;
    }
  }
  acc.x += __shfl_xor(acc.x, 32, 64);
  acc.y += __shfl_xor(acc.y, 32, 64);
  acc.z += __shfl_xor(acc.z, 32, 64);
  acc.w += __shfl_xor(acc.w, 32, 64);
  if (half == 0 && act) {
    red[wv][4 * j] = acc.x;
    red[wv][4 * j + 1] = acc.y;
    red[wv][4 * j + 2] = acc.z;
    red[wv][4 * j + 3] = acc.w;
  }
  dsq = wave_sum(dsq);
  if (lane == 0) sq[wv] = dsq;
  __syncthreads();
  if (tid < H) {
    float a = 0.f;
#pragma unroll
    for (int k = 0; k < HR4_NT / 64; ++k) a += red[k][tid];
    partial[(long)blockIdx.x * (H + 1) + tid] = a;
  }
  if (tid == 0) {
    float a = 0.f;
#pragma unroll
    for (int k = 0; k < HR4_NT / 64; ++k) a += sq[k];
    partial[(long)blockIdx.x * (H + 1) + H] = a;
  }
}

// head Adam with grad = (*gsp) * delta (x) f ; float4 over W (H % 4 == 0, 16-B aligned), scalar over b
__global__ void __launch_bounds__(256) k_hyper_adam_v(float* __restrict__ W, float* __restrict__ bvec,
                                                      float* __restrict__ m, float* __restrict__ v,
                                                      const float* __restrict__ delta, const float* __restrict__ f,
                                                      long P, int H, float lr_bc1, float rsqrt_bc2, float b1,
                                                      float b2, float eps, const float* __restrict__ gsp,
                                                      const int* __restrict__ enable) {
  if (enable != nullptr && *enable == 0) return;
  __shared__ float fs[HS_HMAX];
  if (threadIdx.x < H) fs[threadIdx.x] = f[threadIdx.x];
  __syncthreads();
  const float gs = *gsp;
  const long nW4 = P * H / 4;
  const long stride = (long)gridDim.x * blockDim.x;
  float4* W4 = reinterpret_cast<float4*>(W);
  float4* m4 = reinterpret_cast<float4*>(m);
  float4* v4 = reinterpret_cast<float4*>(v);
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < nW4; i += stride) {
    const long e = 4 * i;
    const long r = e / H;
    const int h = (int)(e - r * H);
    const float dr = gs * delta[r];
    float4 p = W4[i], mm = m4[i], vv = v4[i];
    p.x = hs_adam(p.x, dr * fs[h], mm.x, vv.x, lr_bc1, rsqrt_bc2, b1, b2, eps);
    p.y = hs_adam(p.y, dr * fs[h + 1], mm.y, vv.y, lr_bc1, rsqrt_bc2, b1, b2, eps);
    p.z = hs_adam(p.z, dr * fs[h + 2], mm.z, vv.z, lr_bc1, rsqrt_bc2, b1, b2, eps);
    p.w = hs_adam(p.w, dr * fs[h + 3], mm.w, vv.w, lr_bc1, rsqrt_bc2, b1, b2, eps);
    W4[i] = p;
    m4[i] = mm;
    v4[i] = vv;
  }
  const long nW = P * H;
  for (long r = (long)blockIdx.x * blockDim.x + threadIdx.x; r < P; r += stride) {
    const float g = gs * delta[r];
    const long e = nW + r;
    float mi = m[e], vi = v[e];
    bvec[r] = hs_adam(bvec[r], g, mi, vi, lr_bc1, rsqrt_bc2, b1, b2, eps);
    m[e] = mi;
    v[e] = vi;
  }
}

// Generation W f_c + b for up to HG_MAXC clients in ONE sweep over the packed heads (was a library GEMM after
// the features launch), optionally FUSED with the last client's head Adam (ADAM: the row is updated in registers
// and the generation reads the updated row; the two-kernel sequence wrote and re-read the 39 MB heads of
// RNNModel).  Row mapping of k_hyper_rows4 (a half-wave per row, lane j owns columns 4j..4j+3).  The per-client
// dots of a row reduce as one transpose-reduction over the half-wave: 8 clients in 9 shuffles (a shuffle tree
// per client would be 40), lane j ends with the total of client (j >> 2) of its group of 8.  The fused and the
// plain kernel run the same arithmetic, so a START generated inside the update equals a later plain generation.
constexpr int HG_MAXC = 32;
template <bool ADAM>
__global__ void __launch_bounds__(HR4_NT) k_hyper_gen4(float* __restrict__ W, float* __restrict__ b,
                                                       float* __restrict__ m, float* __restrict__ v,
                                                       const float* __restrict__ delta_k,
                                                       const float* __restrict__ f_k, const float* __restrict__ gsp,
                                                       const float* __restrict__ gfeat, int ngen,
                                                       float* __restrict__ out, long P, int H, float lr_bc1,
                                                       float rsqrt_bc2, float b1, float b2, float eps,
                                                       const int* __restrict__ enable) {
  __shared__ float4 fs[HG_MAXC][HR_HMAX / 4];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int j = lane & 31, half = lane >> 5, H4 = H >> 2;
  const bool act = j < H4;
  const bool upd = ADAM && (enable == nullptr || *enable != 0);
  const int ng8 = (ngen + 7) & ~7;  // clients padded to groups of 8 (zero features)
  for (int e = tid; e < ng8 * (HR_HMAX / 4); e += HR4_NT) {
    const int c = e / (HR_HMAX / 4), q = e - c * (HR_HMAX / 4);
    fs[c][q] = (c < ngen && q < H4) ? reinterpret_cast<const float4*>(gfeat + (long)c * H)[q]
                                    : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  __syncthreads();
  float4 fk = make_float4(0.f, 0.f, 0.f, 0.f);
  float gs = 0.f;
  if (upd) {
    if (act) fk = reinterpret_cast<const float4*>(f_k)[j];
    gs = *gsp;
  }
  float4* W4 = reinterpret_cast<float4*>(W);
  float4* m4 = reinterpret_cast<float4*>(m);
  float4* v4 = reinterpret_cast<float4*>(v);
  const long nW = P * H;
  const long nslots = 2L * gridDim.x * (HR4_NT / 64);
  const long slot = 2L * ((long)blockIdx.x * (HR4_NT / 64) + wv) + half;
  const bool b4 = (j & 16) != 0, b3 = (j & 8) != 0, b2s = (j & 4) != 0;
  for (long r0 = slot; r0 < P; r0 += HR4_U * nslots) {
    float4 w[HR4_U], mm[HR4_U], vv[HR4_U];
#pragma unroll
    for (int q = 0; q < HR4_U; ++q) {  // (clamped rows: every load of the batch in flight)
      const long r = r0 + q * nslots < P ? r0 + q * nslots : P - 1;
      const long e = r * H4 + (act ? j : 0);
      w[q] = W4[e];
      if (upd) {
        mm[q] = m4[e];
        vv[q] = v4[e];
      }
    }
#pragma unroll
    for (int q = 0; q < HR4_U; ++q) {
      const long r = r0 + q * nslots;
      const bool rv = r < P;  // (no early exit: the half-wave reduction needs every lane of the half)
      const long rr = rv ? r : P - 1;
      if (!act) w[q] = make_float4(0.f, 0.f, 0.f, 0.f);
      float bn;
      if (upd) {
        const float dr = gs * delta_k[rr];
        // head Adam on this lane's 4 columns (k_hyper_adam_v's arithmetic)
        w[q].x = hs_adam(w[q].x, dr * fk.x, mm[q].x, vv[q].x, lr_bc1, rsqrt_bc2, b1, b2, eps);
        w[q].y = hs_adam(w[q].y, dr * fk.y, mm[q].y, vv[q].y, lr_bc1, rsqrt_bc2, b1, b2, eps);
        w[q].z = hs_adam(w[q].z, dr * fk.z, mm[q].z, vv[q].z, lr_bc1, rsqrt_bc2, b1, b2, eps);
        w[q].w = hs_adam(w[q].w, dr * fk.w, mm[q].w, vv[q].w, lr_bc1, rsqrt_bc2, b1, b2, eps);
        if (act && rv) {
          W4[r * H4 + j] = w[q];
          m4[r * H4 + j] = mm[q];
          v4[r * H4 + j] = vv[q];
        }
        float bm = m[nW + rr], bvv = v[nW + rr];
        bn = hs_adam(b[rr], dr, bm, bvv, lr_bc1, rsqrt_bc2, b1, b2, eps);
        if (rv && j == 0) {
          m[nW + r] = bm;
          v[nW + r] = bvv;
          b[r] = bn;
        }
      } else {
        bn = b[rr];
      }
      for (int c0 = 0; c0 < ng8; c0 += 8) {
        float dv[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          const float4 f = fs[c0 + c][j];
          dv[c] = __builtin_fmaf(w[q].w, f.w, __builtin_fmaf(w[q].z, f.z, __builtin_fmaf(w[q].y, f.y, w[q].x * f.x)));
        }
        // transpose-reduction: xor 16 halves the client set (bit 4 keeps the upper four), xor 8 and xor 4 again,
        // then xor 2 / xor 1 finish the sum over the lanes that share bits 4..2
        float d4[4], d2[2], d1;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const float keep = b4 ? dv[c + 4] : dv[c], send = b4 ? dv[c] : dv[c + 4];
          d4[c] = keep + __shfl_xor(send, 16, 64);
        }
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const float keep = b3 ? d4[c + 2] : d4[c], send = b3 ? d4[c] : d4[c + 2];
          d2[c] = keep + __shfl_xor(send, 8, 64);
        }
        {
          const float keep = b2s ? d2[1] : d2[0], send = b2s ? d2[0] : d2[1];
          d1 = keep + __shfl_xor(send, 4, 64);
        }
        d1 += __shfl_xor(d1, 2, 64);
        d1 += __shfl_xor(d1, 1, 64);
        // lane j holds client c0 + 4*b4 + 2*b3 + b2s
        const int c = c0 + (b4 ? 4 : 0) + (b3 ? 2 : 0) + (b2s ? 1 : 0);
        if (rv && (j & 3) == 0 && c < ngen) out[(long)c * P + r] = d1 + bn;
      }
    }
  }
}

void afl_hyper_generate(const float* A, const HySmallDesc& d, long offW, long offB, long P, const float* feat,
                        int n, float* out, hipStream_t s) {
  const int nb = afl_hyper_nblocks(P);
  float* W = const_cast<float*>(A) + offW;
  float* bv = const_cast<float*>(A) + offB;
  for (int c0 = 0; c0 < n; c0 += HG_MAXC) {
    const int m = n - c0 < HG_MAXC ? n - c0 : HG_MAXC;
    hipLaunchKernelGGL(k_hyper_gen4<false>, dim3(nb), dim3(HR4_NT), 0, s, W, bv, nullptr, nullptr, nullptr, nullptr,
                       nullptr, feat + (long)c0 * d.H, m, out + (long)c0 * P, P, d.H, 0.f, 0.f, 0.f, 0.f, 0.f,
                       nullptr);
  }
}

// the flat small-net Adam applies: float4 segments, and the moment chunks fit the per-thread registers
static bool hs_flat_ok(const HySmallDesc& d, long nsmall) {
  const long nemb = (long)d.n_nodes * d.E;
  return ((d.emb | nsmall | nemb | d.E) & 3) == 0 && nsmall / 4 <= (long)HS_PF * HS_NT;
}

void afl_hyper_server_update(float* A, float* m, float* v, const float* U, const long* urow, const int* clients,
                             int n, const HySmallDesc& d, long offW, long offB, long P, int step0, float lr,
                             float clip, float b1, float b2, float eps, float* delta, float* partial, float* feat,
                             float* info, const int* enable, const int* gen, int ngen, float* gen_feat,
                             float* gen_out, hipStream_t s) {
  // gen (optional, ngen <= HG_MAXC): the clients whose models the updated hypernetwork generates next; the last
  // client's small-net launch computes their features and the last head Adam writes gen_out [ngen, P]
  const int H = d.H;
  HyClients gl{};
  for (int k = 0; k < ngen; ++k) gl.c[k] = gen[k];
  const int nb = afl_hyper_nblocks(P);
  float* W = A + offW;
  float* bv = A + offB;
  const long nsmall = offW - d.emb;
  const auto small = hs_flat_ok(d, nsmall) ? k_hyper_small<true> : k_hyper_small<false>;
  hipLaunchKernelGGL(small, dim3(1), dim3(HS_NT), 0, s, A, m, v, partial, nb, -1, clients[0], feat, info, d,
                     nsmall, clip, 0.f, 0.f, b1, b2, eps, enable, gl, 0, gen_feat);
  const long nW4 = P * H / 4;
  const int nba = (int)min(4096L, (nW4 + 255) / 256);
  // the rows pass of client k + 1 rides in client k's head Adam (k_hyper_adam_rows4) when the heads are
  // float4-shaped; otherwise (and for the first client) it is its own launch.  delta: two [P] buffers.
#ifndef HYPER_NO_FUSE
  const bool fused = hyper_rows4_ok(W, feat, H) && ((uintptr_t)(m + offW) & 15) == 0 && ((uintptr_t)(v + offW) & 15) == 0;
#else
  const bool fused = false;  // A/B build
#endif
  for (int k = 0; k < n; ++k) {
    const int step = step0 + k + 1;
    const double bc1 = 1.0 - pow((double)b1, step), bc2 = 1.0 - pow((double)b2, step);
    const float lr_bc1 = (float)(lr / bc1), rbc2 = (float)(1.0 / sqrt(bc2));
    float* fk = feat + (k & 1) * HS_HMAX;
    float* fn = feat + ((k + 1) & 1) * HS_HMAX;
    float* dk = delta + (k & 1) * P;
    float* dn = delta + ((k + 1) & 1) * P;
    if (k == 0 || !fused) {
      if (hyper_rows4_ok(W, fk, H))
        hipLaunchKernelGGL(k_hyper_rows4, dim3(nb), dim3(HR4_NT), 0, s, W, bv, fk, U + urow[k] * P, P, H, dk,
                           partial, H + 1);
      else
        hipLaunchKernelGGL(k_hyper_rows, dim3(nb), dim3(256), 0, s, W, bv, fk, U + urow[k] * P, P, H, dk, partial,
                           H + 1);
    }
    const bool last = k + 1 == n;
    hipLaunchKernelGGL(small, dim3(1), dim3(HS_NT), 0, s, A, m, v, partial, nb, clients[k],
                       last ? -1 : clients[k + 1], fn, info + 2 * k, d, nsmall, clip, lr_bc1, rbc2, b1, b2, eps,
                       enable, gl, last ? ngen : 0, gen_feat);
    if (fused && !last)
      hipLaunchKernelGGL(k_hyper_adam_rows4, dim3(nb), dim3(HR4_NT), 0, s, W, bv, m + offW, v + offW, dk, fk,
                         info + 2 * k + 1, fn, U + urow[k + 1] * P, dn, partial, P, H, lr_bc1, rbc2, b1, b2, eps,
                         enable);
    else if (fused && ngen > 0)  // the last head Adam with the next generation in the same sweep
      hipLaunchKernelGGL(k_hyper_gen4<true>, dim3(nb), dim3(HR4_NT), 0, s, W, bv, m + offW, v + offW, dk, fk,
                         info + 2 * k + 1, gen_feat, ngen, gen_out, P, H, lr_bc1, rbc2, b1, b2, eps, enable);
    else
      hipLaunchKernelGGL(k_hyper_adam_v, dim3(nba), dim3(256), 0, s, W, bv, m + offW, v + offW, dk, fk, P, H,
                         lr_bc1, rbc2, b1, b2, eps, info + 2 * k + 1, enable);
  }
  if (ngen > 0 && !fused) afl_hyper_generate(A, d, offW, offB, P, gen_feat, ngen, gen_out, s);
}

// MLP features of up to HF_MAXC clients in ONE launch (the START / validation models of a round: one workgroup
// stages the embedding-MLP parameters once and runs hs_forward per client; was one k_hyper_small per client)
__global__ void __launch_bounds__(HS_NT) k_hyper_feat_many(const float* __restrict__ A, HySmallDesc d, long nsmall,
                                                           HyClients cl, int n, float* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) float sm[HS_SMEM];
  __shared__ float acts[HS_LMAX + 1][HS_HMAX];
  const int tid = threadIdx.x;
  hs_stage(sm, A + d.emb, nsmall);
  __syncthreads();
  for (int k = 0; k < n; ++k) {
    hs_forward(sm, d, cl.c[k], acts);  // (its first barrier also orders the previous client's reads of acts)
    if (tid < d.H) out[(long)k * d.H + tid] = acts[d.L][tid];
    __syncthreads();
  }
}

void afl_hyper_features(const float* A, const HySmallDesc& d, long offW, const int* clients, int n, float* out,
                        hipStream_t s) {
  for (int k0 = 0; k0 < n; k0 += HF_MAXC) {
    HyClients cl{};
    const int m = n - k0 < HF_MAXC ? n - k0 : HF_MAXC;
    for (int k = 0; k < m; ++k) cl.c[k] = clients[k0 + k];
    hipLaunchKernelGGL(k_hyper_feat_many, dim3(1), dim3(HS_NT), 0, s, A, d, offW - d.emb, cl, m, out + (long)k0 * d.H);
  }
}

long afl_hyper_small_capacity() { return HS_SMEM; }
