// ROC-AUC with sklearn's tie handling (one ROC point per distinct threshold, trapezoidal area), as the
// tie-corrected Mann-Whitney rank sum, which is the same number:
//   AUC = (sum over positives of avg_rank(score) - P(P+1)/2) / (P N)
// avg_rank of a tie group = (lo + 1 + hi) / 2 with lo / hi = lower / upper bound of the score in the
// ascending-sorted scores.  One thread per sample (two binary searches each), integer block sums with
// order-independent 64-bit atomics (deterministic), a one-thread finish.  Replaces a one-workgroup chunked
// scan over the sorted (score, label) pairs (~170 us for 80k samples; this is a few us after the sort).
#include "common.h"
#include "kernels.h"

constexpr int AUC_T = 256;

namespace {
__device__ __forceinline__ int lower_bound_f(const float* __restrict__ a, int n, float v) {
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (a[mid] < v) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}
__device__ __forceinline__ int upper_bound_f(const float* __restrict__ a, int n, float v) {
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (a[mid] <= v) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}
}  // namespace

// acc[0] += sum over positives of (lo + 1 + hi), acc[1] += #positives, acc[2] += #NaN scores
__global__ void __launch_bounds__(AUC_T) k_auc_terms(const float* __restrict__ sorted, const float* __restrict__ s,
                                                     const float* __restrict__ y, int n,
                                                     unsigned long long* __restrict__ acc) {
  __shared__ unsigned long long red[3][AUC_T / 64];
  const int i = blockIdx.x * AUC_T + threadIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  unsigned long long t = 0, p = 0, nn = 0;
  if (i < n) {
    const float v = s[i];
    if (v != v) nn = 1;
    else if (y[i] > 0.5f) {  // NaNs sort last, so the searches over finite v stay monotone
      p = 1;
      t = (unsigned long long)(lower_bound_f(sorted, n, v) + 1 + upper_bound_f(sorted, n, v));
    }
  }
  t = wave_sum(t);
  p = wave_sum(p);
  nn = wave_sum(nn);
  if (lane == 0) {
    red[0][w] = t;
    red[1][w] = p;
    red[2][w] = nn;
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    unsigned long long a = 0;
    for (int k = 0; k < AUC_T / 64; ++k) a += red[threadIdx.x][k];
    if (a) atomicAdd(acc + threadIdx.x, a);
  }
}

__global__ void k_auc_final(const unsigned long long* __restrict__ acc, int n, double* __restrict__ out) {
  const double P = (double)acc[1], N = (double)n - P;
  const double two_u = (double)acc[0] - P * (P + 1.0);  // exact: integers < 2^53
  out[0] = (P > 0 && N > 0) ? two_u / (2.0 * P * N) : __longlong_as_double(0x7ff8000000000000ll);
  out[1] = acc[2] ? 1.0 : 0.0;
}

// Small n (the validation set of one model, ~10k rows): count the (positive, negative) pairs directly,
// 2 * #(s_neg < s_pos) + #(s_neg == s_pos) = 2 U, no sort (the sort's ~10 rocprim launches cost more than
// the n^2 / 2 compares).  Grid (i blocks, j chunks); negatives' scores staged in LDS, positives staged as
// NaN (compares false).
constexpr int AUC_PJ = 1024;  // j chunk per workgroup
__global__ void __launch_bounds__(AUC_T) k_auc_pairs(const float* __restrict__ s, const float* __restrict__ y, int n,
                                                     unsigned long long* __restrict__ acc) {
  __shared__ float sj[AUC_PJ];
  __shared__ unsigned long long red[3][AUC_T / 64];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int j0 = blockIdx.y * AUC_PJ, jn = min(AUC_PJ, n - j0);
  for (int e = tid; e < jn; e += AUC_T) {
    const float v = s[j0 + e];
    sj[e] = y[j0 + e] > 0.5f ? __builtin_nanf("") : v;
  }
  __syncthreads();
  const int i = blockIdx.x * AUC_T + tid;
  unsigned long long t = 0, p = 0, nn = 0;
  if (i < n) {
    const float v = s[i];
    const bool pos = y[i] > 0.5f;
    if (blockIdx.y == 0) {
      p = pos ? 1 : 0;
      nn = v != v ? 1 : 0;
    }
    if (pos && v == v) {
      unsigned lt = 0, eq = 0;
#pragma unroll 8
      for (int e = 0; e < jn; ++e) {
        const float u = sj[e];
        lt += u < v ? 1u : 0u;
        eq += u == v ? 1u : 0u;
      }
      t = 2ull * lt + eq;
    }
  }
  t = wave_sum(t);
  p = wave_sum(p);
  nn = wave_sum(nn);
  if (lane == 0) {
    red[0][w] = t;
    red[1][w] = p;
    red[2][w] = nn;
  }
  __syncthreads();
  if (tid < 3) {
    unsigned long long a = 0;
    for (int k = 0; k < AUC_T / 64; ++k) a += red[tid][k];
    if (a) atomicAdd(acc + tid, a);
  }
}

__global__ void k_auc_final_pairs(const unsigned long long* __restrict__ acc, int n, double* __restrict__ out) {
  const double P = (double)acc[1], N = (double)n - P;
  out[0] = (P > 0 && N > 0) ? (double)acc[0] / (2.0 * P * N) : __longlong_as_double(0x7ff8000000000000ll);
  out[1] = acc[2] ? 1.0 : 0.0;
}

int afl_roc_auc_pairs_max() { return 32768; }

void afl_roc_auc_pairs(const float* s, const float* y, int n, unsigned long long* acc, double* out, hipStream_t st) {
  hipMemsetAsync(acc, 0, 3 * sizeof(unsigned long long), st);
  if (n > 0)
    hipLaunchKernelGGL(k_auc_pairs, dim3((n + AUC_T - 1) / AUC_T, (n + AUC_PJ - 1) / AUC_PJ), dim3(AUC_T), 0, st, s, y,
                       n, acc);
  hipLaunchKernelGGL(k_auc_final_pairs, dim3(1), dim3(1), 0, st, acc, n, out);
}

void afl_roc_auc(const float* sorted, const float* s, const float* y, int n, unsigned long long* acc, double* out,
                 hipStream_t st) {
  hipMemsetAsync(acc, 0, 3 * sizeof(unsigned long long), st);
  if (n > 0) hipLaunchKernelGGL(k_auc_terms, dim3((n + AUC_T - 1) / AUC_T), dim3(AUC_T), 0, st, sorted, s, y, n, acc);
  hipLaunchKernelGGL(k_auc_final, dim3(1), dim3(1), 0, st, acc, n, out);
}
