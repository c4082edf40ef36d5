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

// ------------------------------------------------------------------------------------------------
// Gram-form spectral norms for the bisection attacks (reference src/Utils.py:101-204: per-γ distances
// ||c(γ) - G_j||_2 summed over the 2-D tensors, c(γ) = mean - γ·dev).  With X_j = mean - G_j the slot
// matrix is M_j(γ) = X_j - γ D, and its Gram over the smaller side is
//     M M^T = X X^T - γ (X D^T + D X^T) + γ² D D^T,
// so the three n x n Grams are computed ONCE per attack (k_spec_grams, fp64 accumulation) and every γ of
// the bisection only forms A - γS + γ²C (fp64) and runs the squarings (k_spec_eval) — no pass over the
// [K, P] models and no materialised candidate rows per γ.  γ is read from device memory (the bisection
// keeps it there: no host synchronisation per step).  The pairwise distances use the same two kernels
// with D absent (γ = 0).
// Squarings: v_mfma_f64_16x16x4f64 on the fp32 LDS image (products and sums in fp64, the image rounded
// to fp32 between squarings like spectral_one), 12 normalised squarings, best column, Rayleigh quotient
// against the fp64 Gram.  Slots qualify when n = min(r, c) <= 64 and X and D fit in LDS.
constexpr int SG_NMAX = 64;
constexpr int SG_LD = 68;  // fp32 image row stride (bank spread for the MFMA operand reads)
typedef double sg_d4 __attribute__((ext_vector_type(4)));

template <bool DEV>
__global__ void __launch_bounds__(256) k_spec_grams(const float* __restrict__ X, long P, const float* __restrict__ dev,
                                                    const int4* __restrict__ tab, long sumq, double* __restrict__ arena) {
  extern __shared__ float sg_lds[];
  const int s = blockIdx.x, m = blockIdx.y, M = gridDim.y, tid = threadIdx.x;
  const int4 t = tab[s];
  const int r = t.y, c = t.z;
  const bool rows = r <= c;
  const int n = rows ? r : c, k = rows ? c : r, n16 = (n + 15) & ~15, kp = k + 1;
  float* xs = sg_lds;       // [n][k + 1]: xs[i * kp + u] = X(i, u) over the smaller side i
  float* ds = xs + n * kp;  // the same for D
  const float* x = X + (long)m * P + t.x;
  for (int e = tid; e < r * c; e += 256) {
    const int rr = e / c, cc = e - rr * c;
    const int i = rows ? rr : cc, u = rows ? cc : rr;
    xs[i * kp + u] = x[e];
    if (DEV) ds[i * kp + u] = dev[t.x + e];
  }
  __syncthreads();
  double* A = arena + (long)m * 2 * sumq + t.w;
  double* S = A + sumq;
  double* C = arena + (long)M * 2 * sumq + t.w;
  const bool doC = DEV && m == 0;
  for (int e = tid; e < n16 * n16; e += 256) {
    const int i = e / n16, l = e - i * n16;
    double a = 0.0, sx = 0.0, cc2 = 0.0;
    if (i < n && l < n) {
      const float* xi = xs + i * kp;
      const float* xl = xs + l * kp;
      if (DEV) {
        const float* di = ds + i * kp;
        const float* dl = ds + l * kp;
        for (int u = 0; u < k; ++u) {
          a = fma((double)xi[u], (double)xl[u], a);
          sx = fma((double)xi[u], (double)dl[u], sx);
          sx = fma((double)di[u], (double)xl[u], sx);
          if (doC) cc2 = fma((double)di[u], (double)dl[u], cc2);
        }
      } else {
        for (int u = 0; u < k; ++u) a = fma((double)xi[u], (double)xl[u], a);
      }
    }
    A[e] = a;
    if (DEV) {
      S[e] = sx;
      if (doC) C[e] = cc2;
    }
  }
}

__device__ __forceinline__ double sg_block_max(double v, double* red) {
  v = wave_max(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  return fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
}

// ---- the bisection's decision, fused (K-G5; reference loop src/Utils.py:118-130, 152-164, 190-202) ----
// Device state of one bisection (fp64): st[0] γ to try next, st[1] last accepted γ, st[2] last tried γ,
// st[4 + i] the γ tried at iteration i, st[20 + i] 1.0 if it was accepted.  One workgroup of 256 threads
// forms the K candidate distances at the current γ — row 0 is the candidate itself (A-7: distance 0), row j
// the closed-form vector slots sqrt(max(A - 2γB + γ²C, 0)) summed over Sv slots, plus the Gram-form
// spectral sums spec[(j - 1) S + s] of this launch — tests them (kind 0: max_j d_j < thr, Min-Max / Opt-Fang;
// 1: sum_j d_j² < thr, Min-Sum; a NaN distance rejects, as the torch comparison does) and moves γ by ±step/2.
constexpr int BS_TRIED = 4, BS_ACC = 20, BS_WORDS = 40;
__device__ void bisect_decide(const AflBisect& b, const double* spec, int S, int it, double step) {
  __shared__ double rs[4], rm[4];
  __shared__ int rn[4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const double g = b.st[0];
  double s2 = 0.0, mx = 0.0;
  int nan = 0;
  for (int j = tid; j < b.K; j += 256) {
    double d = 0.0;
    if (j > 0) {
      for (int v = 0; v < b.Sv; ++v) {
        const double q = (b.vA[(long)j * b.Sv + v] - 2.0 * g * b.vB[(long)j * b.Sv + v]) + g * g * b.vC[v];
        d += sqrt(q > 0.0 ? q : 0.0);
      }
      for (int v = 0; v < S; ++v)  // (written by the other workgroups of this launch: coherent loads)
        d += __builtin_bit_cast(double, __hip_atomic_load((const unsigned long long*)(spec + (long)(j - 1) * S + v),
                                                          __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    }
    nan |= d != d;
    s2 += d * d;
    mx = fmax(mx, d);
  }
  s2 = wave_sum(s2);
  mx = wave_max(mx);
  nan = (int)wave_max((double)nan);
  if (lane == 0) {
    rs[wave] = s2;
    rm[wave] = mx;
    rn[wave] = nan;
  }
  __syncthreads();
  if (tid == 0) {
    const double tot = (rs[0] + rs[1]) + (rs[2] + rs[3]);
    const double mxx = fmax(fmax(rm[0], rm[1]), fmax(rm[2], rm[3]));
    const bool bad = (rn[0] | rn[1] | rn[2] | rn[3]) != 0;
    const double thr = *b.thr;
    const bool acc = !bad && (b.kind == 1 ? tot < thr : mxx < thr);
    b.st[BS_TRIED + it] = g;
    b.st[BS_ACC + it] = acc ? 1.0 : 0.0;
    b.st[2] = g;
    if (acc) b.st[1] = g;
    b.st[0] = acc ? g + step / 2.0 : g - step / 2.0;
  }
  __syncthreads();
}

// every iteration in ONE launch (no spectral slots: flat distances, or vector-shaped tensors only)
__global__ void __launch_bounds__(256) k_bisect_vec(AflBisect b, int n_iter, double step0) {
  double step = step0;
  for (int it = 0; it < n_iter; ++it) {
    bisect_decide(b, nullptr, 0, it, step);
    step *= 0.5;
  }
}

template <bool BIS>
__global__ void __launch_bounds__(256) k_spec_eval(const double* __restrict__ arena, long sumq, const double* __restrict__ gamma,
                                                   const int4* __restrict__ tab, int S, double* __restrict__ out,
                                                   AflBisect bis, int it, double step) {
  __shared__ float F[2][SG_NMAX * SG_LD];
  __shared__ double red[4];
  __shared__ double dred[2][4];
  __shared__ float wb[4];
  __shared__ int wi[4];
  const int s = blockIdx.x, m = blockIdx.y, M = gridDim.y, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int4 t = tab[s];
  const int n = t.y <= t.z ? t.y : t.z, n16 = (n + 15) & ~15, T = n16 / 16;
  const double g = gamma ? *gamma : 0.0;
  const double* A = arena + (long)m * 2 * sumq + t.w;
  const double* Sg = A + sumq;
  const double* C = arena + (long)M * 2 * sumq + t.w;
  auto gram = [&](int e) -> double { return gamma ? (A[e] - g * Sg[e]) + (g * g) * C[e] : A[e]; };
  // ---- 1. G(γ), normalised, as the fp32 image
  double mx = 0.0;
  for (int e = tid; e < n16 * n16; e += 256) mx = fmax(mx, fabs(gram(e)));
  mx = sg_block_max(mx, red);
  double inv = mx > 0.0 ? 1.0 / mx : 0.0;
  for (int e = tid; e < n16 * n16; e += 256) {
    const int i = e / n16, l = e - i * n16;
    F[0][i * SG_LD + l] = (float)(gram(e) * inv);
  }
  __syncthreads();
  // ---- 2. normalised squarings on fp64 MFMA (wave w: output tiles w, w + 4, ...; f64 C/D layout
  //         acc[r] = C[(lane >> 4) + 4r][lane & 15], A operand [lane & 15][lane >> 4], B operand [lane >> 4][lane & 15])
  int cur = 0;
  for (int it = 0; it < SN_SQUARINGS; ++it) {
    sg_d4 acc[4];
    double lmx = 0.0;
    const float* Fc = F[cur];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      acc[q] = sg_d4{0.0, 0.0, 0.0, 0.0};
      const int p = wave + 4 * q;
      if (p < T * T) {
        const int ti = p / T, tj = p - ti * T;
        const float* arow = Fc + (ti * 16 + (lane & 15)) * SG_LD + (lane >> 4);
        const float* bcol = Fc + (lane >> 4) * SG_LD + tj * 16 + (lane & 15);
        for (int k0 = 0; k0 < n16; k0 += 4)
          acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64((double)arow[k0], (double)bcol[k0 * SG_LD], acc[q], 0, 0, 0);
#pragma unroll
        for (int r = 0; r < 4; ++r) lmx = fmax(lmx, fabs(acc[q][r]));
      }
    }
    mx = sg_block_max(lmx, red);
    inv = mx > 0.0 ? 1.0 / mx : 0.0;
    float* Fn = F[cur ^ 1];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int p = wave + 4 * q;
      if (p < T * T) {
        const int ti = p / T, tj = p - ti * T;
#pragma unroll
        for (int r = 0; r < 4; ++r) Fn[(ti * 16 + (lane >> 4) + 4 * r) * SG_LD + tj * 16 + (lane & 15)] = (float)(acc[q][r] * inv);
      }
    }
    __syncthreads();
    cur ^= 1;
  }
  const float* Fc = F[cur];
  // ---- 3. the column of largest norm (ties: lowest index)
  float best = -1.f;
  int bi = 0;
  for (int j = tid; j < n; j += 256) {
    float sum = 0.f;
    for (int i = 0; i < n; ++i) sum += Fc[i * SG_LD + j] * Fc[i * SG_LD + j];
    if (sum > best) {
      best = sum;
      bi = j;
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    const float ob = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (ob > best || (ob == best && oi < bi)) {
      best = ob;
      bi = oi;
    }
  }
  if (lane == 0) {
    wb[wave] = best;
    wi[wave] = bi;
  }
  __syncthreads();
  int col = wi[0];
  float bb = wb[0];
  for (int w = 1; w < 4; ++w)
    if (wb[w] > bb || (wb[w] == bb && wi[w] < col)) {
      bb = wb[w];
      col = wi[w];
    }
  // ---- 4. Rayleigh quotient v^T G v / v^T v against the fp64 Gram
  double num = 0.0, den = 0.0;
  for (int i = tid; i < n; i += 256) {
    const double vi = Fc[i * SG_LD + col];
    double gv = 0.0;
    for (int l = 0; l < n; ++l) gv = fma(gram(i * n16 + l), (double)Fc[l * SG_LD + col], gv);
    num = fma(vi, gv, num);
    den = fma(vi, vi, den);
  }
  num = wave_sum(num);
  den = wave_sum(den);
  if (lane == 0) {
    dred[0][wave] = num;
    dred[1][wave] = den;
  }
  __syncthreads();
  if (tid == 0) {
    const double nn = (dred[0][0] + dred[0][1]) + (dred[0][2] + dred[0][3]);
    const double dd = (dred[1][0] + dred[1][1]) + (dred[1][2] + dred[1][3]);
    const double lam = dd > 0.0 ? nn / dd : 0.0;
    const double val = lam > 0.0 ? sqrt(lam) : 0.0;
    if (!BIS) {
      out[(long)m * S + s] = val;
    } else {  // fan-in: publish (coherent store), count arrivals; the last workgroup decides this γ
      __hip_atomic_store((unsigned long long*)(out + (long)m * S + s), __builtin_bit_cast(unsigned long long, val),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned prev = __hip_atomic_fetch_add(bis.ctr, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
      wi[0] = prev == gridDim.x * gridDim.y - 1 ? 1 : 0;
    }
  }
  if (BIS) {
    __syncthreads();
    if (wi[0]) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      bisect_decide(bis, out, S, it, step);
      if (tid == 0) __hip_atomic_store(bis.ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // next launch
    }
  }
}

int afl_spec_grams(const float* X, int M, long P, const float* dev, const int* tab, int S, int max_lds_floats, long sumq,
                   double* arena, hipStream_t st) {
  const size_t lds = (size_t)max_lds_floats * sizeof(float);
  if (lds > 160 * 1024) return -1;
  const void* fn = dev ? (const void*)k_spec_grams<true> : (const void*)k_spec_grams<false>;
  if (lds > 64 * 1024 && hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
    return -2;
  if (dev)
    hipLaunchKernelGGL(k_spec_grams<true>, dim3(S, M), dim3(256), lds, st, X, P, dev, (const int4*)tab, sumq, arena);
  else
    hipLaunchKernelGGL(k_spec_grams<false>, dim3(S, M), dim3(256), lds, st, X, P, dev, (const int4*)tab, sumq, arena);
  return 0;
}

int afl_spec_eval(const double* arena, long sumq, int M, const double* gamma, const int* tab, int S, double* out,
                  hipStream_t st) {
  hipLaunchKernelGGL(k_spec_eval<false>, dim3(S, M), dim3(256), 0, st, arena, sumq, gamma, (const int4*)tab, S, out,
                     AflBisect{}, 0, 0.0);
  return 0;
}

int afl_spec_bisect(const double* arena, long sumq, int M, const int* tab, int S, double* out, const AflBisect* b, int it,
                    double step, hipStream_t st) {
  if (M <= 0 || S <= 0 || b->K != M + 1) return -1;
  hipLaunchKernelGGL(k_spec_eval<true>, dim3(S, M), dim3(256), 0, st, arena, sumq, b->st, (const int4*)tab, S, out, *b,
                     it, step);
  return 0;
}

int afl_bisect_vec(const AflBisect* b, int n_iter, double step0, hipStream_t st) {
  if (n_iter > 16) return -1;
  hipLaunchKernelGGL(k_bisect_vec, dim3(1), dim3(256), 0, st, *b, n_iter, step0);
  return 0;
}
