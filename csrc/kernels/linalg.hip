// Batched spectral norm sigma_max(X_b) for the reference's per-tensor attack distance
// (src/Utils.py:47 torch.linalg.norm(diff, ord=2) on 2-D tensors).
//
// One workgroup per matrix:
//   1. Gram A = X X^T or X^T X (the smaller side n <= 128), fp32 in LDS, padded to n8 = 8*ceil(n/8)
//   2. 12 normalised squarings A <- A*A / max|A*A| (= 4096 power iterations), 8x8 register tiles
//   3. v = the column of A^(4096) with the largest norm (spans the top eigenspace, exact even for a
//      repeated top eigenvalue), sigma^2 = Rayleigh quotient v^T G v / v^T v against the ORIGINAL
//      Gram (kept in global scratch), accumulated in fp64.
#include "common.h"
#include "kernels.h"

constexpr int SN_NMAX = 128;
constexpr int SN_SQUARINGS = 12;

// sigma_max of the r x c matrix x (row stride c) -> *out; g0 = n8*n8 floats of global scratch
__device__ __forceinline__ void spectral_one(const float* __restrict__ x, int r, int c, float* __restrict__ g0,
                                             double* __restrict__ out) {
  extern __shared__ float lds[];
  const bool rows = r <= c;  // Gram over the smaller side
  const int n = rows ? r : c;
  const int k = rows ? c : r;
  const int n8 = (n + 7) & ~7;
  const int ld = n8 + 4;  // padded row stride
  float* A = lds;
  float* B = lds + n8 * ld;
  __shared__ float red[4];
  __shared__ int sidx;
  const int tid = threadIdx.x;

  // ---- 1. Gram ----
  for (int e = tid; e < n8 * n8; e += blockDim.x) {
    int i = e / n8, j = e % n8;
    float s = 0.f;
    if (i < n && j < n && j >= i) {
      if (rows)
        for (int t = 0; t < k; ++t) s += x[(long)i * c + t] * x[(long)j * c + t];
      else
        for (int t = 0; t < k; ++t) s += x[(long)t * c + i] * x[(long)t * c + j];
    }
    if (j >= i) {
      A[i * ld + j] = s;
      A[j * ld + i] = s;
      g0[i * n8 + j] = s;
      g0[j * n8 + i] = s;
    }
  }
  __syncthreads();

  // ---- 2. normalised squarings: thread owns an 8x8 tile ----
  const int tiles = n8 / 8;
  for (int it = 0; it < SN_SQUARINGS; ++it) {
    float acc[8][8];
    const int ti = tid / tiles, tj = tid % tiles;
    const bool act = ti < tiles;
#pragma unroll
    for (int a = 0; a < 8; ++a)
#pragma unroll
      for (int bb = 0; bb < 8; ++bb) acc[a][bb] = 0.f;
    float mx = 0.f;
    if (act) {
      for (int kk = 0; kk < n8; ++kk) {
        float av[8], bv[8];
#pragma unroll
        for (int a = 0; a < 8; ++a) av[a] = A[kk * ld + ti * 8 + a];  // A symmetric: A[i][kk] = A[kk][i]
#pragma unroll
        for (int bb = 0; bb < 8; ++bb) bv[bb] = A[kk * ld + tj * 8 + bb];
#pragma unroll
        for (int a = 0; a < 8; ++a)
#pragma unroll
          for (int bb = 0; bb < 8; ++bb) acc[a][bb] += av[a] * bv[bb];
      }
#pragma unroll
      for (int a = 0; a < 8; ++a)
#pragma unroll
        for (int bb = 0; bb < 8; ++bb) {
          B[(ti * 8 + a) * ld + tj * 8 + bb] = acc[a][bb];
          mx = fmaxf(mx, fabsf(acc[a][bb]));
        }
    }
    mx = wave_max(mx);
    if ((tid & 63) == 0) red[tid >> 6] = mx;
    __syncthreads();
    mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    const float inv = mx > 0.f ? 1.f / mx : 0.f;
    for (int e = tid; e < n8 * n8; e += blockDim.x) {
      int i = e / n8, j = e % n8;
      A[i * ld + j] = B[i * ld + j] * inv;
    }
    __syncthreads();
  }

  // ---- 3. best column, Rayleigh quotient against G0 ----
  float best = -1.f;
  int bi = 0;
  for (int j = tid; j < n; j += blockDim.x) {
    float s = 0.f;
    for (int i = 0; i < n; ++i) s += A[i * ld + j] * A[i * ld + j];
    if (s > best) {
      best = s;
      bi = j;
    }
  }
  // argmax across the block (ties -> lowest index)
  for (int o = 32; o > 0; o >>= 1) {
    float ob = __shfl_xor(best, o, 64);
    int oi = __shfl_xor(bi, o, 64);
    if (ob > best || (ob == best && oi < bi)) {
      best = ob;
      bi = oi;
    }
  }
  __shared__ float wb[4];
  __shared__ int wi[4];
  if ((tid & 63) == 0) {
    wb[tid >> 6] = best;
    wi[tid >> 6] = bi;
  }
  __syncthreads();
  if (tid == 0) {
    float bb = wb[0];
    int ii = wi[0];
    for (int w = 1; w < 4; ++w)
      if (wb[w] > bb || (wb[w] == bb && wi[w] < ii)) {
        bb = wb[w];
        ii = wi[w];
      }
    sidx = ii;
  }
  __syncthreads();
  const int col = sidx;
  __shared__ double dred[2][4];
  double num = 0.0, den = 0.0;
  for (int i = tid; i < n; i += blockDim.x) {
    double vi = A[i * ld + col];
    double gv = 0.0;
    for (int j = 0; j < n; ++j) gv += (double)g0[i * n8 + j] * (double)A[j * ld + col];
    num += vi * gv;
    den += vi * vi;
  }
  num = wave_sum(num);
  den = wave_sum(den);
  if ((tid & 63) == 0) {
    dred[0][tid >> 6] = num;
    dred[1][tid >> 6] = den;
  }
  __syncthreads();
  if (tid == 0) {
    double nn = dred[0][0] + dred[0][1] + dred[0][2] + dred[0][3];
    double dd = dred[1][0] + dred[1][1] + dred[1][2] + dred[1][3];
    double lam = dd > 0 ? nn / dd : 0.0;
    *out = lam > 0 ? sqrt(lam) : 0.0;
  }
}

__global__ void __launch_bounds__(256) k_spectral(const float* __restrict__ X, int r, int c, float* __restrict__ G0,
                                                  double* __restrict__ out) {
  const int b = blockIdx.x;
  const int n = r <= c ? r : c;
  const int n8 = (n + 7) & ~7;
  spectral_one(X + (long)b * r * c, r, c, G0 + (long)b * n8 * n8, out + b);
}

// Ragged batch: every (row m, slot s) pair of D [M, P] in ONE launch, slot s = the r x c matrix at
// column offset tab[s].off of row m (all slots of a model at once instead of one launch per shape).
// tab[s] = {off, r, c, scratch offset}; scratch row stride = scr; out [M, S].
__global__ void __launch_bounds__(256) k_spectral_slots(const float* __restrict__ D, long P, const int4* __restrict__ tab,
                                                        int S, float* __restrict__ G0, long scr, double* __restrict__ out) {
  const int s = blockIdx.x, m = blockIdx.y;
  const int4 t = tab[s];
  spectral_one(D + (long)m * P + t.x, t.y, t.z, G0 + (long)m * scr + t.w, out + (long)m * S + s);
}

int afl_spectral_slots(const float* D, int M, long P, const int* tab, int S, int max_n, float* G0, long scr,
                       double* out, hipStream_t st) {
  if (max_n > SN_NMAX) return -1;
  int n8 = (max_n + 7) & ~7;
  size_t lds = (size_t)2 * n8 * (n8 + 4) * sizeof(float);
  if (lds > 64 * 1024)
    if (hipFuncSetAttribute((const void*)k_spectral_slots, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) !=
        hipSuccess)
      return -2;
  hipLaunchKernelGGL(k_spectral_slots, dim3(S, M), dim3(256), lds, st, D, P, (const int4*)tab, S, G0, scr, out);
  return 0;
}

int afl_spectral_scratch(int r, int c) {
  int n = r <= c ? r : c;
  int n8 = (n + 7) & ~7;
  return n8 * n8;
}

int afl_spectral(const float* X, int B, int r, int c, float* G0, double* out, hipStream_t s) {
  int n = r <= c ? r : c;
  if (n > SN_NMAX) return -1;
  int n8 = (n + 7) & ~7;
  size_t lds = (size_t)2 * n8 * (n8 + 4) * sizeof(float);
  if (lds > 64 * 1024)
    if (hipFuncSetAttribute((const void*)k_spectral, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) !=
        hipSuccess)
      return -2;
  hipLaunchKernelGGL(k_spectral, dim3(B), dim3(256), lds, s, X, r, c, G0, out);
  return 0;
}
