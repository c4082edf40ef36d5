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
                                                    int H, float* __restrict__ out, float* __restrict__ partial) {
  __shared__ float tile[HR_ROWS * HR_HMAX];
  __shared__ float fs[HR_HMAX];
  __shared__ float ds[HR_ROWS];
  const int tid = threadIdx.x;
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
    }
    __syncthreads();
    if (u && tid < H) {
      for (int rr = 0; rr < nr; ++rr) acc += tile[rr * H + tid] * ds[rr];
    }
  }
  if (u && tid < H) partial[(long)blockIdx.x * H + tid] = acc;
}

__global__ void k_hyper_reduce(const float* __restrict__ partial, int nb, int H, float* __restrict__ dfeat) {
  int h = threadIdx.x;
  if (h >= H) return;
  double a = 0.0;
  for (int i = 0; i < nb; ++i) a += partial[(long)i * H + h];
  dfeat[h] = (float)a;
}

int afl_hyper_nblocks(long P) { return (int)min(1024L, (P + HR_ROWS - 1) / HR_ROWS); }

void afl_hyper_rows(const float* W, const float* b, const float* f, const float* u, long P, int H, float* out,
                    float* partial, float* dfeat, hipStream_t s) {
  int nb = afl_hyper_nblocks(P);
  hipLaunchKernelGGL(k_hyper_rows, dim3(nb), dim3(256), 0, s, W, b, f, u, P, H, out, partial);
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
