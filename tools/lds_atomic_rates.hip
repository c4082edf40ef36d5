// Cost of the LDS accumulate forms the on-chip trainers can use for their cross-wave column sums (onchip.h
// lds_addq): every wave of a full chip (8 waves per 512-thread workgroup, one workgroup per CU) adds one value
// per lane into 64 slots of 8 bytes (the trainers' pattern: lane = feature), R times, timed with hipEvents.
// Forms: ds_add_f64, ds_add_u64, two ds_add_u32 (hi / lo words), one ds_add_f32, a plain ds_write_b32 to a
// per-wave slot.
//   hipcc --offload-arch=gfx950 -O3 tools/lds_atomic_rates.hip -o /tmp/lds_atomic_rates && /tmp/lds_atomic_rates
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int R = 4096;

template <int MODE>
__global__ void __launch_bounds__(512) k_acc(float* out, float c) {
  __shared__ __attribute__((aligned(16))) unsigned char s[8 * 64 * 8 + 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < 8 * 64 * 2; i += 512) ((unsigned*)s)[i] = 0u;
  __syncthreads();
  float v = c * (float)(lane + 1);
#pragma unroll 1
  for (int it = 0; it < R; ++it) {
    v = v * 1.0000001f;
    if (MODE == 0) {
      __hip_atomic_fetch_add((double*)s + lane, (double)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    } else if (MODE == 1) {
      const long long q = (long long)(int)__float_as_uint(v);
      __hip_atomic_fetch_add((long long*)s + lane, q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    } else if (MODE == 2) {
      const unsigned q = __float_as_uint(v);
      __hip_atomic_fetch_add((unsigned*)s + 2 * lane, q & 0xFFFFFFu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      __hip_atomic_fetch_add((unsigned*)s + 2 * lane + 1, q >> 24, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    } else if (MODE == 3) {
      __hip_atomic_fetch_add((float*)s + lane, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    } else {
      ((volatile float*)s)[w * 64 + lane] = v;
    }
  }
  __syncthreads();
  if (threadIdx.x < 64) out[blockIdx.x * 64 + threadIdx.x] = ((float*)s)[threadIdx.x] + v;
}

template <int MODE>
double run(float* out) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL(k_acc<MODE>, dim3(256), dim3(512), 0, 0, out, 1e-3f);
  hipEventRecord(a);
  for (int i = 0; i < 5; ++i) hipLaunchKernelGGL(k_acc<MODE>, dim3(256), dim3(512), 0, 0, out, 1e-3f);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0.f;
  hipEventElapsedTime(&ms, a, b);
  return ms / 5.0;
}

int main() {
  float* out;
  hipMalloc(&out, 256 * 64 * 4);
  const char* names[5] = {"ds_add_f64", "ds_add_u64", "2x ds_add_u32", "ds_add_f32", "ds_write_b32 (per-wave slot)"};
  double t[5] = {run<0>(out), run<1>(out), run<2>(out), run<3>(out), run<4>(out)};
  for (int m = 0; m < 5; ++m)
    printf("%-30s %8.3f ms  %7.1f cycles per wave-op per CU (2.4 GHz, 8 waves)\n", names[m], t[m],
           t[m] * 1e-3 * 2.4e9 / (8.0 * R));
  return 0;
}
