// Flash attention for the HAR TransformerClassifier encoder (reference src/Model.py:435-458:
// nn.TransformerEncoderLayer(d_model 64, nhead 4) -> SDPA with head_dim 16, L = 561, attention
// dropout 0.1 in training).  The math path of the reference materialises [B*4, 561, 561] fp32
// probabilities (~645 MB per layer at B=128); here one 256-thread workgroup owns one
// (client, sample, head) and streams the whole sequence through LDS, never writing P.
//
// Layouts: qkv [C][B*L][192] fp32 (q | k | v, head h at columns 16h..16h+15 of each), O [C][B*L][64],
// lse [C*B*H][Lp] (Lp = L rounded up to 32).
//
// Forward (per wave: 16 queries, loop over 32-key tiles):
//   S^T[key][q] = K . Q^T on v_mfma_f32_16x16x16_bf16 (two 16-key subtiles) -> every lane holds 8
//   scores of ONE query (lane & 15), so the online-softmax max/sum need only two cross-lane steps
//   (xor 16, xor 32); the dropped probabilities already sit in the B-operand layout of
//   O^T[d][q] += V^T[d][key] . P^T[key][q] (v_mfma_f32_16x16x32_bf16, key order permuted to match),
//   and the running O^T of a query lives in the same lane as its softmax statistics (no shuffles).
// Backward (per wave: 16 keys, loop over 32-query tiles; FA2 recurrence with Delta = rowsum(dO o O)):
//   S, dP in [q][key] orientation (K, V fragments pinned in registers), dV += Pd^T dO and
//   dK += dS^T Q as 16x16x32 MFMAs straight from registers, dQ += dS K through a per-wave LDS
//   transpose of dS and LDS float atomics (summed over the 4 key-owning waves).
// Dropout: keep-mask = afl_keep(step key, layer, (b*H + h)*L + q, key) regenerated in backward.
#include "common.h"
#include "kernels.h"

typedef short s4v __attribute__((ext_vector_type(4)));
typedef short s8v __attribute__((ext_vector_type(8)));
typedef __bf16 bf4v __attribute__((ext_vector_type(4)));
typedef __bf16 bf8v __attribute__((ext_vector_type(8)));
typedef float f4v __attribute__((ext_vector_type(4)));
typedef float f2v __attribute__((ext_vector_type(2)));
typedef __bf16 b2v __attribute__((ext_vector_type(2)));

namespace {

constexpr int H = 4, DH = 16, DM = 64, QKV = 192;

__device__ __forceinline__ unsigned short bf(float x) { return __builtin_bit_cast(unsigned short, (__bf16)x); }
__device__ __forceinline__ f4v mfma16(s4v a, s4v b, f4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f4v mfma32(s8v a, s8v b, f4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf8v, a), __builtin_bit_cast(bf8v, b), c, 0, 0,
                                                 0);
}
__device__ __forceinline__ s4v ld4(const unsigned short* p) { return *(const s4v*)p; }
__device__ __forceinline__ s8v cat8(s4v a, s4v b) {
  s8v r;
  r[0] = a[0]; r[1] = a[1]; r[2] = a[2]; r[3] = a[3];
  r[4] = b[0]; r[5] = b[1]; r[6] = b[2]; r[7] = b[3];
  return r;
}
__device__ __forceinline__ s8v pack8(const float* v) {
  s8v r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (short)bf(v[j]);
  return r;
}

// ============================================================================ forward
__global__ void __launch_bounds__(256) k_attn_fwd(AflAttn a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int Lp = a.Lp, LDV = Lp + 8;
  unsigned short* Kl = (unsigned short*)smem;  // [Lp][16]
  unsigned short* Vt = Kl + Lp * DH;           // [16][LDV]
  const int bh = blockIdx.x, h = bh % H, b = (bh / H) % a.B, c = bh / (H * a.B);
  const long rowbase = ((long)c * a.B + b) * a.L;
  const float* src = a.qkv + rowbase * QKV;
  for (int t = threadIdx.x; t < Lp * DH; t += 256) {
    const int key = t >> 4, d = t & 15;
    const bool ok = key < a.L;
    Kl[t] = bf(ok ? src[(long)key * QKV + DM + h * DH + d] : 0.f);
    Vt[d * LDV + key] = bf(ok ? src[(long)key * QKV + 2 * DM + h * DH + d] : 0.f);
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, li = lane & 15;
  const bool dr = a.drop.thr16 != 0;
  const uint32_t key = dr ? afl_hash32(a.drop.seeds[c], (uint32_t)(a.drop.stepctl ? *a.drop.stepctl : 0)) : 0u;
  const uint32_t drow0 = (uint32_t)((b * H + h) * a.L);
  for (int q0 = wave * 16; q0 < Lp; q0 += 64) {
    const int q = q0 + li;
    s4v qf;
#pragma unroll
    for (int j = 0; j < 4; ++j) qf[j] = (short)bf(q < a.L ? src[(long)q * QKV + h * DH + 4 * g + j] : 0.f);
    float m = -INFINITY, l = 0.f;
    f4v o = f4v{0.f, 0.f, 0.f, 0.f};
    for (int kt = 0; kt < Lp; kt += 32) {
      f4v s0 = mfma16(ld4(Kl + (kt + li) * DH + 4 * g), qf, f4v{0.f, 0.f, 0.f, 0.f});
      f4v s1 = mfma16(ld4(Kl + (kt + 16 + li) * DH + 4 * g), qf, f4v{0.f, 0.f, 0.f, 0.f});
      float s[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        s[e] = (kt + 4 * g + e < a.L) ? s0[e] * a.scale : -INFINITY;
        s[4 + e] = (kt + 16 + 4 * g + e < a.L) ? s1[e] * a.scale : -INFINITY;
      }
      float mx = s[0];
#pragma unroll
      for (int j = 1; j < 8; ++j) mx = fmaxf(mx, s[j]);
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float mn = fmaxf(m, mx);
      const float alpha = __expf(m - mn);
      float ps = 0.f, pd[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float p = __expf(s[j] - mn);
        ps += p;
        const int kk = kt + (j < 4 ? 4 * g + j : 16 + 4 * g + j - 4);
        pd[j] = dr ? p * (afl_keep(key, a.drop.layer, drow0 + q, kk, a.drop.thr16) ? a.drop.inv_keep : 0.f) : p;
      }
      ps += __shfl_xor(ps, 16, 64);
      ps += __shfl_xor(ps, 32, 64);
      l = l * alpha + ps;
      m = mn;
      o *= alpha;
      const s8v vf = cat8(ld4(Vt + li * LDV + kt + 4 * g), ld4(Vt + li * LDV + kt + 16 + 4 * g));
      o = mfma32(vf, pack8(pd), o);
    }
    if (q < a.L) {
      const float inv = 1.f / l;
      float* dst = a.o + (rowbase + q) * DM + h * DH + 4 * g;
#pragma unroll
      for (int e = 0; e < 4; ++e) dst[e] = o[e] * inv;
    }
    if (g == 0) a.lse[(long)bh * Lp + q] = q < a.L ? m + __logf(l) : INFINITY;
  }
}

// ============================================================================ backward
__global__ void __launch_bounds__(256) k_attn_bwd(AflAttn a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int Lp = a.Lp, LDT = Lp + 8;
  unsigned short* Ql = (unsigned short*)smem;  // [Lp][16]
  unsigned short* Dl = Ql + Lp * DH;           // dO [Lp][16]
  unsigned short* Qt = Dl + Lp * DH;           // [16][LDT]
  unsigned short* Dt = Qt + DH * LDT;          // dO^T [16][LDT]
  float* LSE = (float*)(Dt + DH * LDT);        // [Lp]
  float* DEL = LSE + Lp;                       // [Lp]
  float* DQ = DEL + Lp;                        // [Lp][16] fp32 accumulators
  unsigned short* SS = (unsigned short*)(DQ + Lp * DH);  // per wave dS [32][16]
  const int bh = blockIdx.x, h = bh % H, b = (bh / H) % a.B, c = bh / (H * a.B);
  const long rowbase = ((long)c * a.B + b) * a.L;
  const float* src = a.qkv + rowbase * QKV;
  const float* dO = a.dout + rowbase * DM;
  const float* Oo = a.o + rowbase * DM;
  for (int t = threadIdx.x; t < Lp * DH; t += 256) {
    const int q = t >> 4, d = t & 15;
    const bool ok = q < a.L;
    const unsigned short qv = bf(ok ? src[(long)q * QKV + h * DH + d] : 0.f);
    const unsigned short dv = bf(ok ? dO[(long)q * DM + h * DH + d] : 0.f);
    Ql[t] = qv;
    Dl[t] = dv;
    Qt[d * LDT + q] = qv;
    Dt[d * LDT + q] = dv;
    DQ[t] = 0.f;
  }
  for (int q = threadIdx.x; q < Lp; q += 256) {
    float dl = 0.f;
    if (q < a.L) {
#pragma unroll
      for (int d = 0; d < DH; ++d) dl += dO[(long)q * DM + h * DH + d] * Oo[(long)q * DM + h * DH + d];
    }
    DEL[q] = dl;
    LSE[q] = a.lse[(long)bh * Lp + q];
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, li = lane & 15;
  unsigned short* ss = SS + wave * 32 * DH;
  const bool dr = a.drop.thr16 != 0;
  const uint32_t key = dr ? afl_hash32(a.drop.seeds[c], (uint32_t)(a.drop.stepctl ? *a.drop.stepctl : 0)) : 0u;
  const uint32_t drow0 = (uint32_t)((b * H + h) * a.L);
  for (int k0 = wave * 16; k0 < Lp; k0 += 64) {
    const int kk = k0 + li;  // this lane's key (column of S)
    const bool kok = kk < a.L;
    s4v kf, vf, kq;  // K[k][d], V[k][d] (B operands); K[k0+4g+j][li] (B operand of dQ)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      kf[j] = (short)bf(kok ? src[(long)kk * QKV + DM + h * DH + 4 * g + j] : 0.f);
      vf[j] = (short)bf(kok ? src[(long)kk * QKV + 2 * DM + h * DH + 4 * g + j] : 0.f);
      const int kr = k0 + 4 * g + j;
      kq[j] = (short)bf(kr < a.L ? src[(long)kr * QKV + DM + h * DH + li] : 0.f);
    }
    f4v dk = f4v{0.f, 0.f, 0.f, 0.f}, dv = f4v{0.f, 0.f, 0.f, 0.f};
    for (int q0 = 0; q0 < Lp; q0 += 32) {
      float pdv[8], dsv[8];
#pragma unroll
      for (int qs = 0; qs < 2; ++qs) {
        const int qb = q0 + 16 * qs;
        const f4v s = mfma16(ld4(Ql + (qb + li) * DH + 4 * g), kf, f4v{0.f, 0.f, 0.f, 0.f});
        const f4v dp = mfma16(ld4(Dl + (qb + li) * DH + 4 * g), vf, f4v{0.f, 0.f, 0.f, 0.f});
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int q = qb + 4 * g + e;
          const float p = kok ? __expf(s[e] * a.scale - LSE[q]) : 0.f;
          const float mk = dr ? (afl_keep(key, a.drop.layer, drow0 + q, kk, a.drop.thr16) ? a.drop.inv_keep : 0.f) : 1.f;
          pdv[4 * qs + e] = p * mk;
          dsv[4 * qs + e] = p * (dp[e] * mk - DEL[q]);
        }
      }
      // dV[k][d] += sum_q Pd[q][k] dO[q][d];  dK[k][d] += sum_q dS[q][k] Q[q][d]  (query order permuted)
      const s8v dof = cat8(ld4(Dt + li * LDT + q0 + 4 * g), ld4(Dt + li * LDT + q0 + 16 + 4 * g));
      const s8v qtf = cat8(ld4(Qt + li * LDT + q0 + 4 * g), ld4(Qt + li * LDT + q0 + 16 + 4 * g));
      dv = mfma32(pack8(pdv), dof, dv);
      dk = mfma32(pack8(dsv), qtf, dk);
      // dQ[q][d] += sum_k dS[q][k] K[k][d]: transpose dS through this wave's LDS scratch
#pragma unroll
      for (int j = 0; j < 8; ++j) ss[(16 * (j >> 2) + 4 * g + (j & 3)) * DH + li] = bf(dsv[j]);
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's writes visible to itself
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int qs = 0; qs < 2; ++qs) {
        const f4v dq = mfma16(ld4(ss + (16 * qs + li) * DH + 4 * g), kq, f4v{0.f, 0.f, 0.f, 0.f});
#pragma unroll
        for (int e = 0; e < 4; ++e) atomicAdd(DQ + (q0 + 16 * qs + 4 * g + e) * DH + li, dq[e] * a.scale);
      }
      __builtin_amdgcn_wave_barrier();
    }
    // lane holds dK/dV[k0 + 4g + e][li]
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int k = k0 + 4 * g + e;
      if (k < a.L) {
        float* dst = a.dqkv + (rowbase + k) * QKV + h * DH + li;
        dst[DM] = dk[e] * a.scale;
        dst[2 * DM] = dv[e];
      }
    }
  }
  __syncthreads();
  for (int t = threadIdx.x; t < a.L * DH; t += 256) {
    const int q = t >> 4, d = t & 15;
    a.dqkv[(rowbase + q) * QKV + h * DH + d] = DQ[t];
  }
}

}  // namespace

static int attn_lp(int L) { return (L + 31) / 32 * 32; }

int afl_attn_lp(int L) { return attn_lp(L); }

int afl_attn_fwd(const AflAttn& a, hipStream_t s) {
  if (a.Lp != attn_lp(a.L) || a.Lp > 1024) return (int)hipErrorInvalidValue;
  const size_t lds = (size_t)a.Lp * DH * 2 + (size_t)DH * (a.Lp + 8) * 2;
  hipLaunchKernelGGL(k_attn_fwd, dim3(a.C * a.B * H), dim3(256), lds, s, a);
  return (int)hipGetLastError();
}

static size_t bwd_lds(int Lp) {
  return (size_t)Lp * DH * 2 * 2 + (size_t)DH * (Lp + 8) * 2 * 2 + (size_t)Lp * 4 * 2 + (size_t)Lp * DH * 4 +
         4 * 32 * DH * 2;
}

int afl_attn_bwd(const AflAttn& a, hipStream_t s) {
  if (a.Lp != attn_lp(a.L) || a.Lp > 640) return (int)hipErrorInvalidValue;
  const size_t lds = bwd_lds(a.Lp);
  // raise the dynamic-LDS cap once, to the largest size this kernel can ask for (the first call
  // happens eagerly, before any graph capture, so the capture never sees this API)
  static int cap = 0;
  if (lds > 64 * 1024 && cap == 0) {
    const hipError_t e = hipFuncSetAttribute((const void*)k_attn_bwd, hipFuncAttributeMaxDynamicSharedMemorySize,
                                             (int)bwd_lds(640));
    if (e != hipSuccess) return (int)e;
    cap = 1;
  }
  hipLaunchKernelGGL(k_attn_bwd, dim3(a.C * a.B * H), dim3(256), lds, s, a);
  return (int)hipGetLastError();
}
