// Issue cost of single VALU instructions on gfx950: every lane of a full chip runs 8 independent chains
// of one instruction (inline asm, so the compiler cannot substitute another), timed with hipEvents.
// cycles/instr/SIMD = time * clock * SIMDs / wave-instructions.  Used to price the dropout-hash mixers
// (v_mul_lo_u32 vs v_mul_u32_u24 vs shift/xor) and packed fp32 math of the attention kernels.
//   hipcc --offload-arch=gfx950 -O3 tools/valu_rates.hip -o /tmp/valu_rates && /tmp/valu_rates
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int ITERS = 2048;

#define CHAIN8(OP)                                                                                 \
  _Pragma("unroll 1") for (int it = 0; it < ITERS; ++it) {                                          \
    OP(x0) OP(x1) OP(x2) OP(x3) OP(x4) OP(x5) OP(x6) OP(x7)                                         \
  }

#define K_BODY(NAME, OP)                                                                            \
  __global__ void __launch_bounds__(256) NAME(unsigned* out, unsigned c) {                           \
    unsigned x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5,     \
             x6 = x0 + 6, x7 = x0 + 7;                                                              \
    CHAIN8(OP)                                                                                      \
    out[blockIdx.x * 256 + threadIdx.x] = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7;                    \
  }

#define OP_MULLO(x) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x) : "v"(c));
#define OP_MUL24(x) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(x) : "v"(c));
#define OP_MULHI(x) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x) : "v"(c));
#define OP_XOR(x) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x) : "v"(c));
#define OP_LSHRXOR(x) asm volatile("v_lshrrev_b32 %0, 15, %0" : "+v"(x));
#define OP_XAD(x) asm volatile("v_xad_u32 %0, %0, %1, %0" : "+v"(x) : "v"(c));
#define OP_EXP(x) asm volatile("v_exp_f32 %0, %0" : "+v"(x));
#define OP_FMA(x) asm volatile("v_fma_f32 %0, %0, %1, %0" : "+v"(x) : "v"(c));
#define OP_BFE(x) asm volatile("v_bfe_u32 %0, %0, %1, 1" : "+v"(x) : "v"(c));
#define OP_CNDMASK(x) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x) : "v"(c));
#define OP_PERM(x) asm volatile("v_perm_b32 %0, %0, %1, %1" : "+v"(x) : "v"(c));
#define OP_ALIGNBIT(x) asm volatile("v_alignbit_b32 %0, %0, %0, 13" : "+v"(x));

K_BODY(k_mullo, OP_MULLO)
K_BODY(k_mul24, OP_MUL24)
K_BODY(k_mulhi, OP_MULHI)
K_BODY(k_xor, OP_XOR)
K_BODY(k_lshr, OP_LSHRXOR)
K_BODY(k_xad, OP_XAD)
K_BODY(k_exp, OP_EXP)
K_BODY(k_fma, OP_FMA)
K_BODY(k_bfe, OP_BFE)
K_BODY(k_cnd, OP_CNDMASK)
K_BODY(k_perm, OP_PERM)
K_BODY(k_align, OP_ALIGNBIT)

// packed fp32: 8 chains of v_pk_fma_f32 on register pairs
__global__ void __launch_bounds__(256) k_pkfma(unsigned* out, unsigned c) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  f2 x[8];
  for (int i = 0; i < 8; ++i) x[i] = f2{(float)threadIdx.x + i, (float)i};
  const f2 cc = f2{__uint_as_float(c), __uint_as_float(c)};
#pragma unroll 1
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_pk_fma_f32 %0, %0, %1, %0" : "+v"(x[i]) : "v"(cc));
  }
  float s = 0.f;
  for (int i = 0; i < 8; ++i) s += x[i][0] + x[i][1];
  out[blockIdx.x * 256 + threadIdx.x] = __float_as_uint(s);
}

int main() {
  int dev = 0, cus = 0, khz = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  hipDeviceGetAttribute(&khz, hipDeviceAttributeClockRate, dev);
  const int blocks = cus * 4 * 2;  // 2 waves per SIMD (4 waves per 256-thread block, 4 SIMDs per CU)
  unsigned* out;
  hipMalloc(&out, (size_t)blocks * 256 * 4);
  struct { const char* name; void (*k)(unsigned*, unsigned); } ks[] = {
      {"v_mul_lo_u32", k_mullo}, {"v_mul_u32_u24", k_mul24}, {"v_mul_hi_u32", k_mulhi}, {"v_xor_b32", k_xor},
      {"v_lshrrev_b32", k_lshr}, {"v_xad_u32", k_xad}, {"v_exp_f32", k_exp}, {"v_fma_f32", k_fma},
      {"v_bfe_u32", k_bfe}, {"v_cndmask_b32", k_cnd}, {"v_perm_b32", k_perm}, {"v_alignbit_b32", k_align},
      {"v_pk_fma_f32", k_pkfma}};
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  printf("CUs %d, clock %.0f MHz (nominal), %d blocks x 256 threads, %d x 8 instructions per lane\n", cus, khz / 1e3,
         blocks, ITERS);
  for (auto& k : ks) {
    hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, out, 0x9E3779B1u);
    hipDeviceSynchronize();
    hipEventRecord(a);
    for (int rep = 0; rep < 5; ++rep) hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, out, 0x9E3779B1u);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0.f;
    hipEventElapsedTime(&ms, a, b);
    const double waves = (double)blocks * 4, instr = waves * ITERS * 8 * 5;
    const double simd_cycles = ms * 1e-3 * khz * 1e3 * cus * 4;
    printf("%-16s %8.3f ms  %6.2f cycles per wave-instruction per SIMD\n", k.name, ms, simd_cycles / instr);
  }
  hipFree(out);
  return 0;
}
