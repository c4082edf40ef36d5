// Aggregation / attack kernels on the gathered client-update matrix U[N, P] (fp32, row-major).
//
//   colstats        column mean / unbiased std (+ LIE candidate mean + z*std)      K-G2/K-G3
//   weighted_rows   out = sum_i w_i U_i (fp64 weights, fp64 accumulate)            K-G1 FedAvg
//   pair_sqdist     D2[i][j] = ||U_i - U_j||^2 (difference form, no cancellation)   K-G4b / Krum (K > 64)
//   gram_f64        the same from the centred Gram matrix on fp64 MFMA               K-G4b / Krum (K <= 64)
//   noise_philox    own + sigma * N(0,1) from Philox4x32-10 + Box-Muller             K-G10
//   seg_reduce      per-(row, state_dict tensor) partial sums over tiles             K-G4a / K-G5
//   coord_select    coordinate-wise lower median / trimmed mean (register sort)      K-G6
//   row_dots        <u,u>, <u,r>, <r,r> per row                                      K-G8
//   stoch_quant     ScionFL 1-bit stochastic quantisation                            K-G9
//   adam_flat       Adam over a flat arena (optional grad scale = clip coefficient)  K-O1
//
// Every reduction is two-pass with a fixed summation order (no float atomics), so results are
// bit-identical across ranks: the replicated server state on each rank stays in lock-step.
#include "common.h"
#include "kernels.h"

// ============================================================================ colstats
__global__ void __launch_bounds__(256) k_colstats(const float* __restrict__ G, int K, long P, float* __restrict__ mean,
                                                  float* __restrict__ stdv, float* __restrict__ out, float z, int mode) {
  long c = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= P) return;
  double s = 0.0;
  for (int k = 0; k < K; ++k) s += (double)G[(long)k * P + c];
  double m = s / K;
  double ss = 0.0;
  for (int k = 0; k < K; ++k) {
    double d = (double)G[(long)k * P + c] - m;
    ss += d * d;
  }
  float mf = (float)m;
  float sf = K > 1 ? (float)sqrt(ss / (K - 1)) : __int_as_float(0x7fc00000);
  mean[c] = mf;
  stdv[c] = sf;
  if (mode == 1) out[c] = mf + z * sf;
}

void afl_colstats(const float* G, int K, long P, float* mean, float* stdv, float* out, float z, int mode,
                  hipStream_t s) {
  hipLaunchKernelGGL(k_colstats, dim3(afl_cdiv(P, 256)), dim3(256), 0, s, G, K, P, mean, stdv, out, z, mode);
}

// ============================================================================ weighted rows
// ok (optional, int32 [N]): every entry > 0 -> the weighted sum, else out = fallback (FedAvg keeps the previous global
// model when a client failed: the early-launch aggregate, decided on the device in the same pass)
__global__ void __launch_bounds__(256) k_weighted_rows(const float* __restrict__ U, const double* __restrict__ w, int N,
                                                       long P, float* __restrict__ out, const int* __restrict__ ok,
                                                       const float* __restrict__ fallback) {
  long c = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= P) return;
  bool all_ok = true;
  if (ok != nullptr)
    for (int i = 0; i < N; ++i) all_ok = all_ok && ok[i] > 0;
  if (!all_ok) {
    out[c] = fallback[c];
    return;
  }
  double acc = 0.0;
  for (int i = 0; i < N; ++i) acc += w[i] * (double)U[(long)i * P + c];
  out[c] = (float)acc;
}

void afl_weighted_rows(const float* U, const double* w, int N, long P, float* out, hipStream_t s, const int* ok,
                       const float* fallback) {
  hipLaunchKernelGGL(k_weighted_rows, dim3(afl_cdiv(P, 256)), dim3(256), 0, s, U, w, N, P, out, ok, fallback);
}

// ============================================================================ pairwise sq-dist
// Block b stages a [K][CH] column chunk in LDS (row stride CH+1: conflict-free column reads),
// then threads loop over pairs; partial[b][pair] (fp64) is reduced by k_pair_reduce.
constexpr int PD_CH = 256;
__global__ void __launch_bounds__(256) k_pair_sqdist(const float* __restrict__ G, int K, long P,
                                                     double* __restrict__ partial) {
  extern __shared__ float lds[];  // K * (PD_CH + 1)
  const long c0 = (long)blockIdx.x * PD_CH;
  const int ncol = (int)min((long)PD_CH, P - c0);
  for (int k = 0; k < K; ++k)
    for (int j = threadIdx.x; j < PD_CH; j += blockDim.x)
      lds[k * (PD_CH + 1) + j] = j < ncol ? G[(long)k * P + c0 + j] : 0.f;
  __syncthreads();
  const int M = K * (K - 1) / 2;
  for (int pr = threadIdx.x; pr < M; pr += blockDim.x) {
    // pair index -> (i, j), i < j
    int i = 0, rem = pr;
    while (rem >= K - 1 - i) { rem -= K - 1 - i; ++i; }
    int j = i + 1 + rem;
    const float* a = lds + i * (PD_CH + 1);
    const float* b = lds + j * (PD_CH + 1);
    double acc = 0.0;
    for (int t = 0; t < ncol; ++t) {
      float d = a[t] - b[t];
      acc += (double)(d * d);
    }
    partial[(long)blockIdx.x * M + pr] = acc;
  }
}

__global__ void k_pair_reduce(const double* __restrict__ partial, int nb, int K, double* __restrict__ D) {
  const int M = K * (K - 1) / 2;
  int pr = blockIdx.x * blockDim.x + threadIdx.x;
  if (pr >= M) return;
  double acc = 0.0;
  for (int b = 0; b < nb; ++b) acc += partial[(long)b * M + pr];
  int i = 0, rem = pr;
  while (rem >= K - 1 - i) { rem -= K - 1 - i; ++i; }
  int j = i + 1 + rem;
  D[i * K + j] = acc;
  D[j * K + i] = acc;
}

int afl_pair_sqdist_nblocks(long P) { return afl_cdiv(P, PD_CH); }

void afl_pair_sqdist(const float* G, int K, long P, double* partial, double* D, hipStream_t s) {
  int nb = afl_cdiv(P, PD_CH);
  size_t lds = (size_t)K * (PD_CH + 1) * sizeof(float);
  hipLaunchKernelGGL(k_pair_sqdist, dim3(nb), dim3(256), lds, s, G, K, P, partial);
  int M = K * (K - 1) / 2;
  if (M > 0) hipLaunchKernelGGL(k_pair_reduce, dim3(afl_cdiv(M, 256)), dim3(256), 0, s, partial, nb, K, D);
}

// ============================================================================ pairwise via Gram (MFMA)
// D2[i][j] = ||G_i - G_j||^2 from the Gram matrix of the rows CENTRED on row 0 (X_i = G_i - G_0): the
// difference-form correction — model updates are close to each other, so ||G_i||^2 + ||G_j||^2 - 2<G_i,G_j>
// of the raw rows would cancel catastrophically, while the centred rows have norms of the order of the
// distances themselves.  The products run on v_mfma_f64_16x16x4_f64 (fp32 inputs widened to fp64: exact
// products, fp64 accumulation), so the result is as accurate as the fp64 difference loop above.
// K <= 64 (T <= 4 row tiles of 16).  Block b covers GR_CH columns; each of its 4 waves a quarter of them,
// 16 columns per step: lane l loads 4 consecutive columns of row (tile*16 + (l & 15)), column group l >> 4,
// and issues 4 MFMAs per tile pair (element q of the 4 = MFMA q's k = l >> 4: the 16 columns are summed in a
// fixed, data-independent order).  f64 C/D layout: acc[r] = C[(l >> 4) + 4r][l & 15].
constexpr int GR_CH = 1024;
typedef double d4v __attribute__((ext_vector_type(4)));

template <int T>
__global__ void __launch_bounds__(256) k_gram_f64(const float* __restrict__ G, int K, long P,
                                                  double* __restrict__ partial) {
  constexpr int NP = T * (T + 1) / 2;
  __shared__ double red[4][NP * 256];  // NP <= 10 tile pairs x 16 x 16
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r16 = lane & 15, grp = lane >> 4;
  d4v acc[NP];
#pragma unroll
  for (int p = 0; p < NP; ++p) acc[p] = d4v{0.0, 0.0, 0.0, 0.0};
  const long c_begin = (long)blockIdx.x * GR_CH + wave * (GR_CH / 4);
  for (int st = 0; st < GR_CH / 4 / 16; ++st) {
    const long c0 = c_begin + st * 16 + grp * 4;
    float x[T][4];
    float ctr[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) ctr[q] = c0 + q < P ? G[c0 + q] : 0.f;  // row 0 = the centre
#pragma unroll
    for (int t = 0; t < T; ++t) {
      const int row = t * 16 + r16;
#pragma unroll
      for (int q = 0; q < 4; ++q)
        x[t][q] = (row < K && c0 + q < P) ? G[(long)row * P + c0 + q] - ctr[q] : 0.f;
    }
    int p = 0;
#pragma unroll
    for (int ti = 0; ti < T; ++ti)
#pragma unroll
      for (int tj = ti; tj < T; ++tj, ++p)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          acc[p] = __builtin_amdgcn_mfma_f64_16x16x4f64((double)x[ti][q], (double)x[tj][q], acc[p], 0, 0, 0);
  }
  // fixed-order reduction over the 4 waves
#pragma unroll
  for (int p = 0; p < NP; ++p)
#pragma unroll
    for (int r = 0; r < 4; ++r) red[wave][p * 256 + (grp + 4 * r) * 16 + r16] = acc[p][r];
  __syncthreads();
  for (int e = threadIdx.x; e < NP * 256; e += 256)
    partial[(long)blockIdx.x * NP * 256 + e] = ((red[0][e] + red[1][e]) + red[2][e]) + red[3][e];
}

// sum the block partials in block order, then D2 = g_ii + g_jj - 2 g_ij (clamped at 0), symmetric, zero diagonal
__global__ void __launch_bounds__(256) k_gram_reduce(const double* __restrict__ partial, int nb, int K, int T,
                                                     double* __restrict__ gram, double* __restrict__ D) {
  const int NP = T * (T + 1) / 2;
  for (int e = threadIdx.x; e < NP * 256; e += 256) {
    double a = 0.0;
    for (int b = 0; b < nb; ++b) a += partial[(long)b * NP * 256 + e];
    // tile pair index -> (ti, tj)
    int p = e >> 8, ti = 0;
    while (p >= T - ti) { p -= T - ti; ++ti; }
    const int tj = ti + p;
    const int i = ti * 16 + ((e & 255) >> 4), j = tj * 16 + (e & 15);
    if (i < K && j < K) {
      gram[i * K + j] = a;
      gram[j * K + i] = a;
    }
  }
  __syncthreads();
  for (int e = threadIdx.x; e < K * K; e += 256) {
    const int i = e / K, j = e % K;
    const double d = i == j ? 0.0 : gram[i * K + i] + gram[j * K + j] - 2.0 * gram[i * K + j];
    D[e] = d > 0.0 ? d : 0.0;
  }
}

int afl_gram_partials(int K, long P) {
  const int T = (K + 15) / 16;
  return afl_cdiv(P, GR_CH) * T * (T + 1) / 2 * 256 + K * K;
}

int afl_pair_sqdist_gram(const float* G, int K, long P, double* partial, double* D, hipStream_t s) {
  if (K < 1 || K > 64) return (int)hipErrorInvalidValue;
  const int T = (K + 15) / 16, nb = afl_cdiv(P, GR_CH);
  switch (T) {
    case 1: hipLaunchKernelGGL(k_gram_f64<1>, dim3(nb), dim3(256), 0, s, G, K, P, partial); break;
    case 2: hipLaunchKernelGGL(k_gram_f64<2>, dim3(nb), dim3(256), 0, s, G, K, P, partial); break;
    case 3: hipLaunchKernelGGL(k_gram_f64<3>, dim3(nb), dim3(256), 0, s, G, K, P, partial); break;
    default: hipLaunchKernelGGL(k_gram_f64<4>, dim3(nb), dim3(256), 0, s, G, K, P, partial); break;
  }
  double* gram = partial + (long)nb * T * (T + 1) / 2 * 256;
  hipLaunchKernelGGL(k_gram_reduce, dim3(1), dim3(256), 0, s, partial, nb, K, T, gram, D);
  return (int)hipGetLastError();
}

// ============================================================================ Philox noise (Random attack)
// out = own + sigma * N(0, 1) (reference create_random_base_model, src/Utils.py:52-57).  Philox4x32-10
// (Salmon et al., SC'11) keyed by the 64-bit seed, counter = (element group, 0, 0, 0): one call gives 4
// uniforms for 4 consecutive elements, turned into normals by Box-Muller (2 pairs).  Stateless and
// deterministic: the same (seed, P) always yields the same noise, on any rank.  The Python mirror
// (ops/composite.py:philox_normal) reproduces the uniforms bit for bit.
__device__ __forceinline__ void philox_round(uint32_t& c0, uint32_t& c1, uint32_t& c2, uint32_t& c3, uint32_t k0,
                                             uint32_t k1) {
  const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
  const uint32_t h0 = (uint32_t)(p0 >> 32), l0 = (uint32_t)p0, h1 = (uint32_t)(p1 >> 32), l1 = (uint32_t)p1;
  const uint32_t n0 = h1 ^ c1 ^ k0, n2 = h0 ^ c3 ^ k1;
  c0 = n0;
  c1 = l1;
  c2 = n2;
  c3 = l0;
}

__global__ void __launch_bounds__(256) k_noise_philox(const float* __restrict__ own, float* __restrict__ out, long P,
                                                      float sigma, uint32_t k0, uint32_t k1) {
  const long g = (long)blockIdx.x * blockDim.x + threadIdx.x;  // element group of 4
  if (g * 4 >= P) return;
  uint32_t c0 = (uint32_t)g, c1 = (uint32_t)(g >> 32), c2 = 0, c3 = 0, a = k0, b = k1;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    philox_round(c0, c1, c2, c3, a, b);
    a += 0x9E3779B9u;
    b += 0xBB67AE85u;
  }
  // uniforms in (0, 1]: (x + 1) * 2^-32 in fp64 then Box-Muller in fp64 (no log(0); one rounding at the end)
  const double u0 = ((double)c0 + 1.0) * 2.3283064365386963e-10, u1 = ((double)c1 + 1.0) * 2.3283064365386963e-10;
  const double u2 = ((double)c2 + 1.0) * 2.3283064365386963e-10, u3 = ((double)c3 + 1.0) * 2.3283064365386963e-10;
  const double r0 = sqrt(-2.0 * log(u0)), r1 = sqrt(-2.0 * log(u2));
  const double t0 = 6.283185307179586 * u1, t1 = 6.283185307179586 * u3;
  const double z[4] = {r0 * cos(t0), r0 * sin(t0), r1 * cos(t1), r1 * sin(t1)};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const long i = g * 4 + q;
    if (i < P) out[i] = own[i] + sigma * (float)z[q];
  }
}

void afl_noise_philox(const float* own, float* out, long P, float sigma, uint64_t seed, hipStream_t s) {
  hipLaunchKernelGGL(k_noise_philox, dim3(afl_cdiv(afl_cdiv(P, 4), 256)), dim3(256), 0, s, own, out, P, sigma,
                     (uint32_t)seed, (uint32_t)(seed >> 32));
}

// ============================================================================ segmented reductions
// tiles[t] = (segment, start, end).  Pass 1: block (t, row) -> partial[t][row][q].  Pass 2:
// per (row, segment) sum of its tiles in order.
//   mode 0 (sqsum):   q0 = sum x^2                       X = diffs [M, P]
//   mode 1 (coeffs):  row < K: q0 = sum (m-g)^2, q1 = sum (m-g)*d ; row == K: q0 = sum d^2
__global__ void __launch_bounds__(256) k_seg_pass1(int mode, const float* __restrict__ X, long P, int rows,
                                                   const float* __restrict__ mean, const float* __restrict__ dev,
                                                   const int* __restrict__ tiles, double* __restrict__ partial) {
  __shared__ double scratch[8];
  const int t = blockIdx.x, r = blockIdx.y;
  const int st = tiles[3 * t + 1], en = tiles[3 * t + 2];
  double q0 = 0.0, q1 = 0.0;
  if (mode == 0) {
    const float* x = X + (long)r * P;
    for (int c = st + threadIdx.x; c < en; c += blockDim.x) {
      float v = x[c];
      q0 += (double)v * v;
    }
  } else if (r < rows - 1) {
    const float* g = X + (long)r * P;
    for (int c = st + threadIdx.x; c < en; c += blockDim.x) {
      double a = (double)mean[c] - (double)g[c];
      q0 += a * a;
      q1 += a * (double)dev[c];
    }
  } else {
    for (int c = st + threadIdx.x; c < en; c += blockDim.x) {
      double d = dev[c];
      q0 += d * d;
    }
  }
  q0 = block_sum(q0, scratch);
  q1 = block_sum(q1, scratch);
  if (threadIdx.x == 0) {
    partial[((long)t * rows + r) * 2 + 0] = q0;
    partial[((long)t * rows + r) * 2 + 1] = q1;
  }
}

__global__ void k_seg_pass2(const double* __restrict__ partial, const int* __restrict__ segf, int rows, int S,
                            double* __restrict__ out0, double* __restrict__ out1) {
  int id = blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= rows * S) return;
  int r = id / S, sg = id % S;
  double a = 0.0, b = 0.0;
  for (int t = segf[sg]; t < segf[sg + 1]; ++t) {
    a += partial[((long)t * rows + r) * 2 + 0];
    b += partial[((long)t * rows + r) * 2 + 1];
  }
  out0[(long)r * S + sg] = a;
  if (out1) out1[(long)r * S + sg] = b;
}

void afl_seg_reduce(int mode, const float* X, long P, int rows, const float* mean, const float* dev, const int* tiles,
                    int T, const int* segf, int S, double* partial, double* out0, double* out1, hipStream_t s) {
  hipLaunchKernelGGL(k_seg_pass1, dim3(T, rows), dim3(256), 0, s, mode, X, P, rows, mean, dev, tiles, partial);
  hipLaunchKernelGGL(k_seg_pass2, dim3(afl_cdiv((long)rows * S, 256)), dim3(256), 0, s, partial, segf, rows, S, out0,
                     out1);
}

// ============================================================================ coordinate select
// Each thread owns one column: N values in registers, odd-even transposition sort network with
// compile-time indices (NMAX template; padding +inf), then lower-median or trimmed mean.
template <int NMAX>
__global__ void __launch_bounds__(256) k_coord_select(const float* __restrict__ U, int N, long P, int mode, int trim,
                                                      float* __restrict__ out) {
  long c = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= P) return;
  float v[NMAX];
#pragma unroll
  for (int i = 0; i < NMAX; ++i) v[i] = i < N ? U[(long)i * P + c] : __int_as_float(0x7f800000);
#pragma unroll
  for (int r = 0; r < NMAX; ++r) {
#pragma unroll
    for (int i = (r & 1); i + 1 < NMAX; i += 2) {
      float a = v[i], b = v[i + 1];
      // NaN-aware: torch.sort/median place NaN last (treated as largest)
      bool sw = (a > b) || (a != a && b == b);
      v[i] = sw ? b : a;
      v[i + 1] = sw ? a : b;
    }
  }
  float r = 0.f;
  if (mode == 0) {
    const int mid = (N - 1) / 2;
#pragma unroll
    for (int i = 0; i < NMAX; ++i) r = (i == mid) ? v[i] : r;
  } else {
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < NMAX; ++i) acc += (i >= trim && i < N - trim) ? v[i] : 0.f;
    r = acc / (float)(N - 2 * trim);
  }
  out[c] = r;
}

void afl_coord_select(const float* U, int N, long P, int mode, int trim, float* out, hipStream_t s) {
  dim3 g(afl_cdiv(P, 256)), b(256);
  if (N <= 8) hipLaunchKernelGGL(k_coord_select<8>, g, b, 0, s, U, N, P, mode, trim, out);
  else if (N <= 16) hipLaunchKernelGGL(k_coord_select<16>, g, b, 0, s, U, N, P, mode, trim, out);
  else if (N <= 32) hipLaunchKernelGGL(k_coord_select<32>, g, b, 0, s, U, N, P, mode, trim, out);
  else hipLaunchKernelGGL(k_coord_select<64>, g, b, 0, s, U, N, P, mode, trim, out);
}

// ============================================================================ row dots
constexpr int RD_CH = 8192;
__global__ void __launch_bounds__(256) k_row_dots(const float* __restrict__ U, const float* __restrict__ ref, long P,
                                                  int mode, double* __restrict__ partial) {
  __shared__ double scratch[8];
  const int ch = blockIdx.x, r = blockIdx.y;
  const long st = (long)ch * RD_CH, en = min(P, st + RD_CH);
  const float* u = U + (long)r * P;
  double uu = 0, ur = 0, rr = 0;
  for (long c = st + threadIdx.x; c < en; c += blockDim.x) {
    double a = u[c];
    uu += a * a;
    if (mode) {
      double b = ref[c];
      ur += a * b;
      rr += b * b;
    }
  }
  uu = block_sum(uu, scratch);
  ur = block_sum(ur, scratch);
  rr = block_sum(rr, scratch);
  if (threadIdx.x == 0) {
    double* p = partial + ((long)r * gridDim.x + ch) * 3;
    p[0] = uu;
    p[1] = ur;
    p[2] = rr;
  }
}

__global__ void k_row_dots_reduce(const double* __restrict__ partial, int N, int nch, double* __restrict__ out) {
  int id = blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= N * 3) return;
  int r = id / 3, q = id % 3;
  double a = 0;
  for (int c = 0; c < nch; ++c) a += partial[((long)r * nch + c) * 3 + q];
  out[r * 3 + q] = a;
}

int afl_row_dots_nchunks(long P) { return afl_cdiv(P, RD_CH); }

void afl_row_dots(const float* U, const float* ref, int N, long P, int mode, double* partial, double* out,
                  hipStream_t s) {
  int nch = afl_cdiv(P, RD_CH);
  hipLaunchKernelGGL(k_row_dots, dim3(nch, N), dim3(256), 0, s, U, ref, P, mode, partial);
  hipLaunchKernelGGL(k_row_dots_reduce, dim3(afl_cdiv(N * 3, 256)), dim3(256), 0, s, partial, N, nch, out);
}

// ============================================================================ ScionFL quantisation
// Row min / max over SQ_NB chunks per row (one workgroup per row kept 8 CUs busy for 49 us at 8 x 47.7 k), the
// chunk partials reduced by the quantisation kernel's blocks themselves (min / max: any order gives the same
// values, so the bits are those of the one-pass form).
constexpr int SQ_NB = 32;
__global__ void __launch_bounds__(256) k_row_minmax(const float* __restrict__ U, long P, float* __restrict__ part) {
  __shared__ float smn[4], smx[4];
  const int r = blockIdx.y, b = blockIdx.x;
  const long c0 = P * b / SQ_NB, c1 = P * (b + 1) / SQ_NB;
  const float* u = U + (long)r * P;
  float mn = __int_as_float(0x7f800000), mx = -mn;
  for (long c = c0 + threadIdx.x; c < c1; c += blockDim.x) {
    const float a = u[c];
    mn = fminf(mn, a);
    mx = fmaxf(mx, a);
  }
  mn = wave_min(mn);
  mx = wave_max(mx);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) {
    smn[w] = mn;
    smx[w] = mx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < 4; ++i) {
      mn = fminf(mn, smn[i]);
      mx = fmaxf(mx, smx[i]);
    }
    part[((long)r * SQ_NB + b) * 2] = mn;
    part[((long)r * SQ_NB + b) * 2 + 1] = mx;
  }
}

__global__ void __launch_bounds__(256) k_stoch_quant(const float* __restrict__ U, long P, long total,
                                                     const float* __restrict__ part, float* __restrict__ smin,
                                                     float* __restrict__ smax, uint64_t seed,
                                                     float* __restrict__ sigma) {
  __shared__ float lo_s[2], hi_s[2];
  const long id0 = (long)blockIdx.x * blockDim.x;
  const long r0 = id0 / P;  // a block spans at most two rows (P >= 256) or several (P < 256: handled per row)
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (w < 2) {  // wave w reduces the partials of row r0 + w
    const long r = r0 + w;
    const long nrows = total / P;
    float mn = __int_as_float(0x7f800000), mx = -mn;
    if (r < nrows && lane < SQ_NB) {
      mn = part[(r * SQ_NB + lane) * 2];
      mx = part[(r * SQ_NB + lane) * 2 + 1];
    }
    mn = wave_min(mn);
    mx = wave_max(mx);
    if (lane == 0) {
      lo_s[w] = mn;
      hi_s[w] = mx;
    }
  }
  __syncthreads();
  const long id = id0 + threadIdx.x;
  if (id >= total) return;
  const long r = id / P;
  float lo, hi;
  if (r - r0 < 2) {
    lo = lo_s[r - r0];
    hi = hi_s[r - r0];
  } else {  // (rows shorter than a block: reduce this row's partials directly)
    lo = __int_as_float(0x7f800000);
    hi = -lo;
    for (int b = 0; b < SQ_NB; ++b) {
      lo = fminf(lo, part[(r * SQ_NB + b) * 2]);
      hi = fmaxf(hi, part[(r * SQ_NB + b) * 2 + 1]);
    }
  }
  if (id == r * P) {  // the row's first element publishes its min / max
    smin[r] = lo;
    smax[r] = hi;
  }
  const float p = (U[id] - lo) / (hi - lo + 1e-6f);
  sigma[id] = afl_uniform(seed, (uint64_t)id) < p ? 1.f : 0.f;
}

long afl_stoch_quant_ws(int N) { return (long)N * SQ_NB * 2; }

void afl_stoch_quant(const float* U, int N, long P, uint64_t seed, float* sigma, float* smin, float* smax,
                     float* ws, hipStream_t s) {
  hipLaunchKernelGGL(k_row_minmax, dim3(SQ_NB, N), dim3(256), 0, s, U, P, ws);
  const long total = (long)N * P;
  hipLaunchKernelGGL(k_stoch_quant, dim3(afl_cdiv(total, 256)), dim3(256), 0, s, U, P, total, ws, smin, smax, seed,
                     sigma);
}

// ============================================================================ Adam (flat)
// torch.optim.Adam (foreach=False) math: m <- m + (1-b1)(g-m); v <- b2 v + (1-b2) g^2;
// p <- p - (lr/bc1) * m / (sqrt(v)/sqrt(bc2) + eps).  `gscale` folds in a clip coefficient.
__global__ void __launch_bounds__(256) k_adam_flat(float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v, long n, float lr_bc1,
                                                   float rsqrt_bc2, float b1, float b2, float eps, float gscale) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float gi = g[i] * gscale;
  float mi = m[i] + (1.f - b1) * (gi - m[i]);
  float vi = b2 * v[i] + (1.f - b2) * gi * gi;
  m[i] = mi;
  v[i] = vi;
  p[i] -= lr_bc1 * mi / (sqrtf(vi) * rsqrt_bc2 + eps);
}

void afl_adam_flat(float* p, const float* g, float* m, float* v, long n, int step, float lr, float b1, float b2,
                   float eps, float gscale, hipStream_t s) {
  double bc1 = 1.0 - pow((double)b1, step), bc2 = 1.0 - pow((double)b2, step);
  hipLaunchKernelGGL(k_adam_flat, dim3(afl_cdiv(n, 256)), dim3(256), 0, s, p, g, m, v, n, (float)(lr / bc1),
                     (float)(1.0 / sqrt(bc2)), b1, b2, eps, gscale);
}

// ============================================================================ gmm_filter
// GMM gradient filter (reference server.py:352-370, src/Utils.py:257-323), all decisions on the device so the
// round needs no host round trip: input the centred Gram matrix G = Xc Xc^T [n][n] (fp64) of the client updates.
//   1. PCA scores in r dims (rank > 0: min(rank, 4, n); 0: max(1, min(4, n/2 - 1))): cyclic Jacobi eigen-decomposition of G (12 sweeps),
//      eigenvalues in descending order, Z = V_r sqrt(lambda_r), scaled by 1 / max |Z|;
//   2. rows ordered benign then malicious (train_gmm_model's vstack), a 2-component full-covariance GMM
//      (reg_covar 1e-6, tol 1e-3, <= 100 EM iterations, sklearn's M / E steps) initialised by a deterministic
//      k-means (centres: row 0 and the row farthest from it, 10 Lloyd iterations) — sklearn's k-means++ init
//      draws from an unseeded RNG in the reference, so any fixed init is one of its possible runs;
//   3. threshold = 3 x population std of the benign rows' Mahalanobis distances to component 0; a row is kept
//      when its distance to its most probable component is <= threshold.
// One wave: the Jacobi rotations are applied by lane k to row / column k, the E-step and the decisions run one lane
// per row, every sum stays on lane 0 in row order; agg.gmm_filter_ref in Python is the bit-level mirror.
constexpr int GMM_MAXN = 64, GMM_R = 4;

__device__ __host__ inline bool gmm_chol(const double (&S)[GMM_R][GMM_R], int r, double (&Lc)[GMM_R][GMM_R]) {
  for (int i = 0; i < r; ++i)
    for (int j = 0; j <= i; ++j) {
      double s = S[i][j];
      for (int k = 0; k < j; ++k) s -= Lc[i][k] * Lc[j][k];
      if (i == j) {
        if (!(s > 0.0)) return false;
        Lc[i][i] = sqrt(s);
      } else {
        Lc[i][j] = s / Lc[j][j];
      }
    }
  return true;
}
// squared Mahalanobis distance through the Cholesky factor (forward substitution)
__device__ __host__ inline double gmm_md2(const double (&Lc)[GMM_R][GMM_R], int r, const double* x, const double* mu) {
  double y[GMM_R], s = 0.0;
  for (int i = 0; i < r; ++i) {
    double v = x[i] - mu[i];
    for (int k = 0; k < i; ++k) v -= Lc[i][k] * y[k];
    y[i] = v / Lc[i][i];
    s += y[i] * y[i];
  }
  return s;
}

__global__ void __launch_bounds__(64) k_gmm_filter(const double* __restrict__ G, int n, const unsigned char* __restrict__ att,
                                                   unsigned char* __restrict__ keep, double* __restrict__ info, int rank) {
  __shared__ double A[GMM_MAXN * GMM_MAXN], V[GMM_MAXN * GMM_MAXN], Z[GMM_MAXN * GMM_R], X[GMM_MAXN * GMM_R];
  __shared__ double resp[GMM_MAXN * 2], ev[GMM_MAXN];
  __shared__ int ord[GMM_MAXN], evi[GMM_MAXN];
  for (int e = threadIdx.x; e < n * n; e += blockDim.x) {
    A[e] = G[e];
    V[e] = (e / n == e % n) ? 1.0 : 0.0;
  }
  __syncthreads();
  // ---- 1. Jacobi eigen-decomposition (cyclic sweeps, fixed count): every lane derives the rotation, lane k applies
  //      it to row / column k (the same element operations in the same order as the single-lane form and the host
  //      mirror; one lane walking the n^2 updates serially through LDS took ~0.6 ms for n = 8)
  const int k = threadIdx.x;
  for (int sweep = 0; sweep < 12; ++sweep)
    for (int p = 0; p < n - 1; ++p)
      for (int q = p + 1; q < n; ++q) {
        const double apq = A[p * n + q];
        if (fabs(apq) < 1e-300) continue;  // (uniform: every lane read the same word)
        const double th = (A[q * n + q] - A[p * n + p]) / (2.0 * apq);
        const double t = (th >= 0.0 ? 1.0 : -1.0) / (fabs(th) + sqrt(th * th + 1.0));
        const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
        __syncthreads();  // every lane has read A[p][p], A[q][q], A[p][q] before they change
        if (k < n) {  // columns p, q
          const double akp = A[k * n + p], akq = A[k * n + q];
          A[k * n + p] = c * akp - s * akq;
          A[k * n + q] = s * akp + c * akq;
        }
        __syncthreads();
        if (k < n) {  // rows p, q; eigenvectors
          const double apk = A[p * n + k], aqk = A[q * n + k];
          A[p * n + k] = c * apk - s * aqk;
          A[q * n + k] = s * apk + c * aqk;
          const double vkp = V[k * n + p], vkq = V[k * n + q];
          V[k * n + p] = c * vkp - s * vkq;
          V[k * n + q] = s * vkp + c * vkq;
        }
        __syncthreads();
      }
  // ---- the rest: one lane, except the E-step and the decisions (lane i = row i; the sums stay on lane 0 in row
  //      order, so every value equals the single-lane form's and the host mirror's)
  __shared__ double mu[2][GMM_R], w[2], cov[2][GMM_R][GMM_R], Lc[2][GMM_R][GMM_R], logdet[2], lse_row[GMM_MAXN];
  __shared__ int sh_r, sh_m, sh_nb, sh_K, sh_okc, sh_stop;
  __shared__ double sh_thr;
  if (k == 0) {
    for (int i = 0; i < n; ++i) {
      ev[i] = A[i * n + i];
      evi[i] = i;
    }
    for (int i = 1; i < n; ++i) {  // stable insertion sort, descending
      const double v = ev[i];
      const int ix = evi[i];
      int j = i - 1;
      while (j >= 0 && ev[j] < v) {
        ev[j + 1] = ev[j];
        evi[j + 1] = evi[j];
        --j;
      }
      ev[j + 1] = v;
      evi[j + 1] = ix;
    }
    const int r = rank > 0 ? min(min(rank, GMM_R), n) : max(1, min(GMM_R, n / 2 - 1));
    double zmax = 0.0;
    for (int i = 0; i < n; ++i)
      for (int kk = 0; kk < r; ++kk) {
        const double z = V[i * n + evi[kk]] * sqrt(fmax(ev[kk], 1e-30));
        Z[i * GMM_R + kk] = z;
        zmax = fmax(zmax, fabs(z));
      }
    zmax = fmax(zmax, 1e-30);
    int m = 0;
    for (int i = 0; i < n; ++i)
      if (!att[i]) ord[m++] = i;
    const int nb = m;
    for (int i = 0; i < n; ++i)
      if (att[i]) ord[m++] = i;
    for (int i = 0; i < n; ++i)
      for (int kk = 0; kk < r; ++kk) Z[i * GMM_R + kk] /= zmax;
    for (int i = 0; i < m; ++i)
      for (int kk = 0; kk < r; ++kk) X[i * GMM_R + kk] = Z[ord[i] * GMM_R + kk];
    const int K = m >= 2 ? 2 : 1;
    // ---- 2a. deterministic k-means initialisation
    for (int kk = 0; kk < r; ++kk) mu[0][kk] = mu[1][kk] = X[kk];
    if (K == 2) {
      int far = 0;
      double best = -1.0;
      for (int i = 0; i < m; ++i) {
        double d = 0.0;
        for (int kk = 0; kk < r; ++kk) d += (X[i * GMM_R + kk] - X[kk]) * (X[i * GMM_R + kk] - X[kk]);
        if (d > best) {
          best = d;
          far = i;
        }
      }
      for (int kk = 0; kk < r; ++kk) mu[1][kk] = X[far * GMM_R + kk];
      for (int it = 0; it < 10; ++it) {
        double sm[2][GMM_R] = {}, cnt[2] = {0.0, 0.0};
        for (int i = 0; i < m; ++i) {
          double d0 = 0.0, d1 = 0.0;
          for (int kk = 0; kk < r; ++kk) {
            d0 += (X[i * GMM_R + kk] - mu[0][kk]) * (X[i * GMM_R + kk] - mu[0][kk]);
            d1 += (X[i * GMM_R + kk] - mu[1][kk]) * (X[i * GMM_R + kk] - mu[1][kk]);
          }
          const int l = d1 < d0 ? 1 : 0;
          resp[i * 2 + 0] = l == 0 ? 1.0 : 0.0;
          resp[i * 2 + 1] = l == 1 ? 1.0 : 0.0;
          cnt[l] += 1.0;
          for (int kk = 0; kk < r; ++kk) sm[l][kk] += X[i * GMM_R + kk];
        }
        for (int c = 0; c < 2; ++c)
          if (cnt[c] > 0.0)
            for (int kk = 0; kk < r; ++kk) mu[c][kk] = sm[c][kk] / cnt[c];
      }
    } else {
      for (int i = 0; i < m; ++i) {
        resp[i * 2] = 1.0;
        resp[i * 2 + 1] = 0.0;
      }
    }
    sh_r = r;
    sh_m = m;
    sh_nb = nb;
    sh_K = K;
    sh_okc = 1;
  }
  __syncthreads();
  const int r = sh_r, m = sh_m, nb = sh_nb, K = sh_K;
  // ---- 2b. EM (sklearn GaussianMixture, covariance_type "full")
  const double eps10 = 10.0 * 2.220446049250313e-16, reg = 1e-6, LOG2PI = 1.8378770664093453;
  auto mstep = [&]() {  // (lane 0)
    double nks = 0.0;
    for (int c = 0; c < K; ++c) {
      double nk = eps10;
      for (int i = 0; i < m; ++i) nk += resp[i * 2 + c];
      for (int kk = 0; kk < r; ++kk) {
        double sv = 0.0;
        for (int i = 0; i < m; ++i) sv += resp[i * 2 + c] * X[i * GMM_R + kk];
        mu[c][kk] = sv / nk;
      }
      for (int a = 0; a < r; ++a)
        for (int b = 0; b < r; ++b) {
          double sv = 0.0;
          for (int i = 0; i < m; ++i)
            sv += resp[i * 2 + c] * (X[i * GMM_R + a] - mu[c][a]) * (X[i * GMM_R + b] - mu[c][b]);
          cov[c][a][b] = sv / nk + (a == b ? reg : 0.0);
        }
      w[c] = nk;
      nks += nk;
      sh_okc = sh_okc && gmm_chol(cov[c], r, Lc[c]);
      double ld = 0.0;
      for (int kk = 0; kk < r; ++kk) ld += log(Lc[c][kk][kk]);
      logdet[c] = 2.0 * ld;
    }
    for (int c = 0; c < K; ++c) w[c] /= nks;
  };
  auto wlogp = [&](const double* x, int c) {
    return log(w[c]) - 0.5 * (r * LOG2PI + gmm_md2(Lc[c], r, x, mu[c]) + logdet[c]);
  };
  if (k == 0) {
    mstep();
    sh_stop = sh_okc ? 0 : 1;
  }
  __syncthreads();
  double lb = -INFINITY;  // (lane 0's copy is the one that decides)
  for (int it = 0; it < 100 && !sh_stop; ++it) {
    if (k < m) {  // E-step, lane k = row k
      const double* x = X + k * GMM_R;
      double lp[2] = {wlogp(x, 0), K == 2 ? wlogp(x, 1) : -INFINITY};
      const double mx = fmax(lp[0], lp[1]);
      const double lse = mx + log(exp(lp[0] - mx) + exp(lp[1] - mx));
      lse_row[k] = lse;
      resp[k * 2] = exp(lp[0] - lse);
      resp[k * 2 + 1] = K == 2 ? exp(lp[1] - lse) : 0.0;
    }
    __syncthreads();
    if (k == 0) {
      const double prev = lb;
      double tot = 0.0;
      for (int i = 0; i < m; ++i) tot += lse_row[i];
      mstep();
      lb = tot / m;
      sh_stop = (!sh_okc || fabs(lb - prev) < 1e-3) ? 1 : 0;
    }
    __syncthreads();
  }
  // ---- 3. threshold and decisions
  if (k == 0) {
    double s1 = 0.0, s2 = 0.0;
    for (int i = 0; i < nb; ++i) s1 += sqrt(gmm_md2(Lc[0], r, X + i * GMM_R, mu[0]));
    const double meanb = nb ? s1 / nb : 0.0;
    for (int i = 0; i < nb; ++i) {
      const double d = sqrt(gmm_md2(Lc[0], r, X + i * GMM_R, mu[0])) - meanb;
      s2 += d * d;
    }
    sh_thr = nb ? 3.0 * sqrt(s2 / nb) : INFINITY;
  }
  __syncthreads();
  const double thr = sh_thr;
  const bool okc = sh_okc != 0;
  if (k < n) {  // lane k = client k
    const double* x = Z + k * GMM_R;
    const int c = (K == 2 && wlogp(x, 1) > wlogp(x, 0)) ? 1 : 0;
    const bool kp = okc && sqrt(gmm_md2(Lc[c], r, x, mu[c])) <= thr;
    keep[k] = kp ? 1 : 0;
    lse_row[k] = kp ? 1.0 : 0.0;
  }
  __syncthreads();
  if (k == 0) {
    int kept = 0;
    for (int i = 0; i < n; ++i) kept += lse_row[i] > 0.5 ? 1 : 0;
    info[0] = thr;
    info[1] = (double)kept;
    info[2] = okc ? 1.0 : 0.0;
  }
}

int afl_gmm_filter(const double* G, int n, const unsigned char* att, unsigned char* keep, double* info, int rank,
                   hipStream_t s) {
  if (n < 1 || n > GMM_MAXN || rank < 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_gmm_filter, dim3(1), dim3(64), 0, s, G, n, att, keep, info, rank);
  return (int)hipGetLastError();
}

// ============================================================================ top_pc
// First principal-component scores of n <= 64 rows from their centred Gram G = Xc Xc^T (fp64 [n][n]), the
// FLTracer PCA(1) (reference src/Utils.py:359-369): Jacobi eigen-decomposition on one wave (at most ``sweeps``
// sweeps, fewer once the off-diagonal mass is at fp64 rounding); z = v_max sqrt(lambda_max).  Parallel (round-robin) ordering: each step rotates m / 2 DISJOINT pairs at
// once (m = n rounded up to even; m - 1 steps cover every pair once per sweep), their (c, s) computed by one lane
// each, then one lane per (pair, row / column) applies them — 7 dependent steps per sweep at n = 8 instead of 28
// sequential rotations (the rotation's fp64 divide / square-root chain and three barriers were the kernel's whole
// time: 158 us per call).  (Repeated squaring of G, the round-4 form, let the second eigenvector leak in at
// (lambda_2 / lambda_1)^(2^squarings): 2 % at a 0.999 ratio, 66 % at 0.9999 — nearly iid updates.)
__global__ void __launch_bounds__(64) k_top_pc(const double* __restrict__ G, int n, int sweeps, double* __restrict__ z) {
  __shared__ double A[GMM_MAXN * GMM_MAXN], V[GMM_MAXN * GMM_MAXN];
  __shared__ double cs_c[GMM_MAXN / 2], cs_s[GMM_MAXN / 2];
  __shared__ int cs_p[GMM_MAXN / 2], cs_q[GMM_MAXN / 2];
  const int k = threadIdx.x;
  for (int e = k; e < n * n; e += blockDim.x) {
    A[e] = G[e];
    V[e] = (e / n == e % n) ? 1.0 : 0.0;
  }
  const int m = n + (n & 1);  // (an odd n pairs one index with the dummy index n each step: skipped)
  const int half = m / 2;
  __syncthreads();
  for (int sweep = 0; sweep < sweeps; ++sweep) {
    {  // converged to fp64 precision (off-diagonal mass <= 1e-32 of the diagonal's): the remaining rotations
       // would be identities up to rounding, so the sweep count is an upper bound (uniform decision)
      double off = 0.0, dia = 0.0;
      if (k < n) {
        dia = A[k * n + k] * A[k * n + k];
        for (int j = k + 1; j < n; ++j) off += A[k * n + j] * A[k * n + j];
      }
      for (int o = 32; o > 0; o >>= 1) {
        off += __shfl_xor(off, o, 64);
        dia += __shfl_xor(dia, o, 64);
      }
      if (off <= 1e-32 * dia) break;
    }
    for (int r = 0; r < m - 1; ++r) {
      if (k < half) {  // pair k of step r: (r, m - 1) and ((r + k) % (m - 1), (r - k + m - 1) % (m - 1))
        int p = k == 0 ? r : (r + k) % (m - 1);
        int q = k == 0 ? m - 1 : (r - k + m - 1) % (m - 1);
        if (p > q) {
          const int t = p;
          p = q;
          q = t;
        }
        double c = 1.0, sn = 0.0;
        if (q < n) {
          const double apq = A[p * n + q];
          if (fabs(apq) >= 1e-300) {
            const double th = (A[q * n + q] - A[p * n + p]) / (2.0 * apq);
            const double t = (th >= 0.0 ? 1.0 : -1.0) / (fabs(th) + sqrt(th * th + 1.0));
            c = 1.0 / sqrt(t * t + 1.0);
            sn = t * c;
          }
        }
        cs_p[k] = p;
        cs_q[k] = q < n ? q : p;  // (identity on the dummy pair: c = 1, s = 0 on column p alone)
        cs_c[k] = c;
        cs_s[k] = sn;
      }
      __syncthreads();
      // one lane per (pair t, row / column i): every pair's rotation applied at once (disjoint pairs)
      for (int e = k; e < half * n; e += 64) {  // columns p, q
        const int t = e / n, i = e - t * n;
        const int p = cs_p[t], q = cs_q[t];
        if (p == q) continue;
        const double c = cs_c[t], sn = cs_s[t];
        const double aip = A[i * n + p], aiq = A[i * n + q];
        const double vip = V[i * n + p], viq = V[i * n + q];
        A[i * n + p] = c * aip - sn * aiq;
        A[i * n + q] = sn * aip + c * aiq;
        V[i * n + p] = c * vip - sn * viq;
        V[i * n + q] = sn * vip + c * viq;
      }
      __syncthreads();
      for (int e = k; e < half * n; e += 64) {  // rows p, q
        const int t = e / n, i = e - t * n;
        const int p = cs_p[t], q = cs_q[t];
        if (p == q) continue;
        const double c = cs_c[t], sn = cs_s[t];
        const double api = A[p * n + i], aqi = A[q * n + i];
        A[p * n + i] = c * api - sn * aqi;
        A[q * n + i] = sn * api + c * aqi;
      }
      __syncthreads();
    }
  }
  int top = 0;
  for (int i = 1; i < n; ++i)
    if (A[i * n + i] > A[top * n + top]) top = i;
  if (k < n) z[k] = V[k * n + top] * sqrt(fmax(A[top * n + top], 0.0));
}

int afl_top_pc(const double* G, int n, int sweeps, double* z, hipStream_t s) {
  if (n < 1 || n > GMM_MAXN || sweeps < 1) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_top_pc, dim3(1), dim3(64), 0, s, G, n, sweeps, z);
  return (int)hipGetLastError();
}
