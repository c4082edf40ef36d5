// Flash attention for the HAR TransformerClassifier encoder (reference src/Model.py:435-458:
// nn.TransformerEncoderLayer(d_model 64, nhead 4) -> SDPA with head_dim 16, L = 561, attention
// dropout 0.1 in training).  The math path of the reference materialises [B*4, 561, 561] fp32
// probabilities (~645 MB per layer at B=128); here one 12-wave workgroup owns one
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
// Backward (FA2 recurrence with Delta = rowsum(dO o O)), two owner-computes kernels, no atomics:
//   k_attn_bwd_kv  each wave owns 16 keys and sweeps the queries: S, dP in [q][key] orientation (K, V
//                  fragments pinned in registers), dV += Pd^T dO and dK += dS^T Q as 16x16x32 MFMAs
//                  straight from registers; 12 waves share one ~80 KB LDS image (2 workgroups per CU).
//   k_attn_bwd_dq  each wave owns 16 queries and sweeps the keys (recomputing S, dP): dQ stays in
//                  registers.  (An LDS-atomic dQ reduction inside the kv kernel measured 5x slower:
//                  3.7 ms vs 0.75 ms for the kv sweep alone at C=8, B=64.)
// Dropout: keep-mask = afl_keep(step key, layer, (b*H + h)*L + q, key) regenerated in backward.
#include "common.h"
#include "kernels.h"

#define LDS_AS __attribute__((address_space(3)))
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
// [rows][16] bf16 images read as 4-column groups by 16 consecutive rows: rows with bit 3 set swap
// their column halves, so rows r and r+8 land on different banks (ds_read_b64: (a/4) mod 64)
__device__ __forceinline__ int swz(int r, int d) { return r * DH + (d ^ (((r >> 3) & 1) << 3)); }

// Dropout multipliers of the 8 keys a lane holds for one query row: keys kb0..kb0+3 and kb1..kb1+3
// (kb even).  Adjacent keys share one hash (afl_keep's column pairs): 4 hashes per 8 elements.
__device__ __forceinline__ void keep8(uint32_t key, uint32_t layer, uint32_t row, int kb0, int kb1, uint32_t thr,
                                      float ik, float (&mk)[8]) {
#pragma unroll
  for (int hf = 0; hf < 2; ++hf)
#pragma unroll
    for (int pr = 0; pr < 2; ++pr) {
      const uint32_t hsh = afl_hash4(key, layer, row, (uint32_t)(((hf ? kb1 : kb0) >> 1) + pr));
      mk[4 * hf + 2 * pr] = (hsh & 0xFFFFu) >= thr ? ik : 0.f;
      mk[4 * hf + 2 * pr + 1] = (hsh >> 16) >= thr ? ik : 0.f;
    }
}
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

// Loads of the staging helpers: quad (row = t >> 2, dims 4 (t & 3) .. +3) of two [rows][stride] sources
template <int NT, int NI>
__device__ __forceinline__ void load_quads(const float* __restrict__ s1, long st1, int off1, const float* __restrict__ s2,
                                           long st2, int off2, int nrows, int nvalid, f4v (&v1)[NI], f4v (&v2)[NI]) {
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int t = threadIdx.x + i * NT, row = t >> 2, qd = t & 3;
    const bool ok = row < nvalid && t < nrows * 4;
    v1[i] = ok ? *(const f4v*)(s1 + (long)row * st1 + off1 + 4 * qd) : f4v{0.f, 0.f, 0.f, 0.f};
    v2[i] = ok ? *(const f4v*)(s2 + (long)row * st2 + off2 + 4 * qd) : f4v{0.f, 0.f, 0.f, 0.f};
  }
}
__device__ __forceinline__ void put_quad(unsigned short* X, unsigned short* XT, int ldt, int row, int qd, f4v v) {
  s4v a;
#pragma unroll
  for (int j = 0; j < 4; ++j) a[j] = (short)bf(v[j]);
  if (X) *(s4v*)(X + swz(row, 4 * qd)) = a;
  if (XT) {
#pragma unroll
    for (int j = 0; j < 4; ++j) XT[(4 * qd + j) * ldt + row] = (unsigned short)a[j];
  }
}
constexpr int STAGE_MAXR = 1024 + 64;

// Stage rows [0, nrows) of two 16-wide head slices of a [rows][stride] fp32 matrix into LDS as bf16:
// X1 row-major swizzled ([row][16], swz) and X2 either row-major swizzled or transposed ([16][ldt]).
// Every thread issues ALL its 16-B global loads before the first LDS store (the naive per-element
// loop waited out one HBM latency per element: it dominated the kernels).
template <int NT, bool X2T>
__device__ __forceinline__ void stage2(const float* __restrict__ src, long stride, int off1, int off2, int nrows,
                                       int nvalid, unsigned short* X1, unsigned short* X2, int ldt) {
  constexpr int MAXR = 1024 + 64;
  constexpr int NI = (MAXR * 4 + NT - 1) / NT;
  f4v v1[NI], v2[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int t = threadIdx.x + i * NT, row = t >> 2, qd = t & 3;
    const bool ok = row < nvalid && t < nrows * 4;
    v1[i] = ok ? *(const f4v*)(src + (long)row * stride + off1 + 4 * qd) : f4v{0.f, 0.f, 0.f, 0.f};
    v2[i] = ok ? *(const f4v*)(src + (long)row * stride + off2 + 4 * qd) : f4v{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int t = threadIdx.x + i * NT, row = t >> 2, qd = t & 3;
    if (t < nrows * 4) {
      s4v a;
#pragma unroll
      for (int j = 0; j < 4; ++j) a[j] = (short)bf(v1[i][j]);
      *(s4v*)(X1 + swz(row, 4 * qd)) = a;
      if (X2T) {
#pragma unroll
        for (int j = 0; j < 4; ++j) X2[(4 * qd + j) * ldt + row] = bf(v2[i][j]);
      } else {
        s4v b;
#pragma unroll
        for (int j = 0; j < 4; ++j) b[j] = (short)bf(v2[i][j]);
        *(s4v*)(X2 + swz(row, 4 * qd)) = b;
      }
    }
  }
}

// ============================================================================ forward
constexpr int FW_WAVES = 12, FW_NT = 64 * FW_WAVES;
constexpr float LOG2E = 1.4426950408889634f, LN2 = 0.6931471805599453f;

// cross-lane max / sum over lanes l, l^16, l^32 with the gfx950 permlane swaps (no LDS round trip).
// permlane{16,32}_swap(a, a) returns {own value, partner value} in some order, so max / sum of the
// pair is exact.
__device__ __forceinline__ float max_x16_x32(float a) {
  auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(a), false, false);
  a = fmaxf(__uint_as_float(p[0]), __uint_as_float(p[1]));
  p = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(a), false, false);
  return fmaxf(__uint_as_float(p[0]), __uint_as_float(p[1]));
}
__device__ __forceinline__ float sum_x16_x32(float a) {
  auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(a), false, false);
  a = __uint_as_float(p[0]) + __uint_as_float(p[1]);
  p = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(a), false, false);
  return __uint_as_float(p[0]) + __uint_as_float(p[1]);
}
__device__ __forceinline__ float ex2(float x) { return __builtin_amdgcn_exp2f(x); }

// 64 keys per step: four 16-key S^T subtiles (lane: keys kt + 16 t + 4 g + e of query li), one
// max / sum reduction and one rescale per 64 keys, two O^T MFMAs (32 keys each).  Scores are kept in
// the log2 domain (scale * log2 e folded in) so every exponential is one v_exp_f32.
template <bool DROP>
__global__ void __launch_bounds__(FW_NT) k_attn_fwd(AflAttn a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int Lp = a.Lp, LDV = Lp + 8 + 32;  // +32: the last 64-key step may read one zero 32-key half
  unsigned short* Kl = (unsigned short*)smem;  // [Lp + 32][16]
  unsigned short* Vt = Kl + (Lp + 32) * DH;    // [16][LDV]
  const int bh = blockIdx.x, h = bh % H, b = (bh / H) % a.B, c = bh / (H * a.B);
  const long rowbase = ((long)c * a.B + b) * a.L;
  const float* src = a.qkv + rowbase * QKV;
  stage2<FW_NT, true>(src, QKV, DM + h * DH, 2 * DM + h * DH, Lp + 32, a.L, Kl, Vt, LDV);
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, li = lane & 15;
  const uint32_t key = DROP ? afl_hash32(a.drop.seeds[c], (uint32_t)(a.drop.stepctl ? *a.drop.stepctl : 0)) : 0u;
  const uint32_t drow0 = (uint32_t)((b * H + h) * a.L);
  const float sc2 = a.scale * LOG2E;
  for (int q0 = wave * 16; q0 < Lp; q0 += 16 * FW_WAVES) {
    const int q = q0 + li;
    s4v qf;
#pragma unroll
    for (int j = 0; j < 4; ++j) qf[j] = (short)bf(q < a.L ? src[(long)q * QKV + h * DH + 4 * g + j] : 0.f);
    float m = -INFINITY, l = 0.f;
    f4v o = f4v{0.f, 0.f, 0.f, 0.f};
    for (int kt = 0; kt < Lp; kt += 64) {
      float s[16];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const f4v st = mfma16(ld4(Kl + swz(kt + 16 * t + li, 4 * g)), qf, f4v{0.f, 0.f, 0.f, 0.f});
#pragma unroll
        for (int e = 0; e < 4; ++e) s[4 * t + e] = (kt + 16 * t + 4 * g + e < a.L) ? st[e] * sc2 : -INFINITY;
      }
      float mx = s[0];
#pragma unroll
      for (int j = 1; j < 16; ++j) mx = fmaxf(mx, s[j]);
      const float mn = fmaxf(m, max_x16_x32(mx));
      const float alpha = ex2(m - mn);
      float ps = 0.f, pd[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        pd[j] = ex2(s[j] - mn);
        ps += pd[j];
      }
      if (DROP) {
        float mk[16];
        keep8(key, a.drop.layer, drow0 + q, kt + 4 * g, kt + 16 + 4 * g, a.drop.thr16, a.drop.inv_keep, *(float(*)[8])mk);
        keep8(key, a.drop.layer, drow0 + q, kt + 32 + 4 * g, kt + 48 + 4 * g, a.drop.thr16, a.drop.inv_keep,
              *(float(*)[8])(mk + 8));
#pragma unroll
        for (int j = 0; j < 16; ++j) pd[j] *= mk[j];
      }
      l = l * alpha + sum_x16_x32(ps);
      m = mn;
      o *= alpha;
      const s8v v0 = cat8(ld4(Vt + li * LDV + kt + 4 * g), ld4(Vt + li * LDV + kt + 16 + 4 * g));
      const s8v v1 = cat8(ld4(Vt + li * LDV + kt + 32 + 4 * g), ld4(Vt + li * LDV + kt + 48 + 4 * g));
      o = mfma32(v0, pack8(pd), o);
      o = mfma32(v1, pack8(pd + 8), o);
    }
    if (q < a.L) {
      const float inv = 1.f / l;
      float* dst = a.o + (rowbase + q) * DM + h * DH + 4 * g;
#pragma unroll
      for (int e = 0; e < 4; ++e) dst[e] = o[e] * inv;
    }
    if (g == 0) a.lse[(long)bh * Lp + q] = q < a.L ? (m + __log2f(l)) * LN2 : INFINITY;
  }
}

// ============================================================================ backward
// ---- dK / dV: each wave owns 16 keys and sweeps every query ----
constexpr int BW_WAVES = 12, BW_NT = 64 * BW_WAVES;  // 12 waves share one ~80 KB LDS image (2 WGs per CU)

template <bool DROP>
__global__ void __launch_bounds__(BW_NT) k_attn_bwd_kv(AflAttn a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int Lp = a.Lp, LDT = Lp + 8;
  unsigned short* Ql = (unsigned short*)smem;  // [Lp][16] (swizzled)
  unsigned short* Dl = Ql + Lp * DH;           // dO [Lp][16] (swizzled)
  unsigned short* Qt = Dl + Lp * DH;           // [16][LDT]
  unsigned short* Dt = Qt + DH * LDT;          // dO^T [16][LDT]
  float* LSE = (float*)(Dt + DH * LDT);        // [Lp]
  float* DEL = LSE + Lp;                       // [Lp] Delta_q = dO_q . O_q
  const int bh = blockIdx.x, h = bh % H, b = (bh / H) % a.B, c = bh / (H * a.B);
  const long rowbase = ((long)c * a.B + b) * a.L;
  const float* src = a.qkv + rowbase * QKV;
  const float* dO = a.dout + rowbase * DM;
  const float* Oo = a.o + rowbase * DM;
  {  // Q, dO -> row-major + transposed images; Delta_q = dO_q . O_q; lse
    constexpr int NI = (STAGE_MAXR * 4 + BW_NT - 1) / BW_NT;
    f4v vq[NI], vd[NI];
    load_quads<BW_NT, NI>(src, QKV, h * DH, dO, DM, h * DH, Lp, a.L, vq, vd);
    float dl[NI];
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int t = threadIdx.x + i * BW_NT, row = t >> 2, qd = t & 3;
      f4v vo = f4v{0.f, 0.f, 0.f, 0.f};
      if (row < a.L && t < Lp * 4) vo = *(const f4v*)(Oo + (long)row * DM + h * DH + 4 * qd);
      dl[i] = vd[i][0] * vo[0] + vd[i][1] * vo[1] + vd[i][2] * vo[2] + vd[i][3] * vo[3];
    }
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int t = threadIdx.x + i * BW_NT, row = t >> 2, qd = t & 3;
      float d = dl[i];
      d += __shfl_xor(d, 1, 64);
      d += __shfl_xor(d, 2, 64);
      if (t < Lp * 4) {
        put_quad(Ql, Qt, LDT, row, qd, vq[i]);
        put_quad(Dl, Dt, LDT, row, qd, vd[i]);
        if (qd == 0) {
          DEL[row] = d;
          LSE[row] = a.lse[(long)bh * Lp + row];
        }
      }
    }
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, li = lane & 15;
  const uint32_t key = DROP ? afl_hash32(a.drop.seeds[c], (uint32_t)(a.drop.stepctl ? *a.drop.stepctl : 0)) : 0u;
  const uint32_t drow0 = (uint32_t)((b * H + h) * a.L);
  for (int k0 = wave * 16; k0 < Lp; k0 += 16 * BW_WAVES) {
    const int kk = k0 + li;  // this lane's key (column of S)
    const bool kok = kk < a.L;
    s4v kf, vf;  // K[k][d], V[k][d] (B operands)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      kf[j] = (short)bf(kok ? src[(long)kk * QKV + DM + h * DH + 4 * g + j] : 0.f);
      vf[j] = (short)bf(kok ? src[(long)kk * QKV + 2 * DM + h * DH + 4 * g + j] : 0.f);
    }
    f4v dk = f4v{0.f, 0.f, 0.f, 0.f}, dv = f4v{0.f, 0.f, 0.f, 0.f};
    for (int q0 = 0; q0 < Lp; q0 += 32) {
      float pdv[8], dsv[8];
#pragma unroll
      for (int qs = 0; qs < 2; ++qs) {
        const int qb = q0 + 16 * qs;
        const f4v s = mfma16(ld4(Ql + swz(qb + li, 4 * g)), kf, f4v{0.f, 0.f, 0.f, 0.f});
        const f4v dp = mfma16(ld4(Dl + swz(qb + li, 4 * g)), vf, f4v{0.f, 0.f, 0.f, 0.f});
        const f4v l4 = *(const f4v*)(LSE + qb + 4 * g);
        const f4v d4 = *(const f4v*)(DEL + qb + 4 * g);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float pe = __expf(s[e] * a.scale - l4[e]);
          const float p = kok ? pe : 0.f;
          float mk = 1.f;
          if (DROP) mk = afl_keep(key, a.drop.layer, drow0 + qb + 4 * g + e, kk, a.drop.thr16) ? a.drop.inv_keep : 0.f;
          pdv[4 * qs + e] = p * mk;
          dsv[4 * qs + e] = p * (dp[e] * mk - d4[e]);
        }
      }
      // dV[k][d] += sum_q Pd[q][k] dO[q][d];  dK[k][d] += sum_q dS[q][k] Q[q][d]  (query order permuted)
      const s8v dof = cat8(ld4(Dt + li * LDT + q0 + 4 * g), ld4(Dt + li * LDT + q0 + 16 + 4 * g));
      const s8v qtf = cat8(ld4(Qt + li * LDT + q0 + 4 * g), ld4(Qt + li * LDT + q0 + 16 + 4 * g));
      dv = mfma32(pack8(pdv), dof, dv);
      dk = mfma32(pack8(dsv), qtf, dk);
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
}

// ---- dQ: each wave owns 16 queries and sweeps every key (recomputes S and dP; no atomics) ----
//   S^T[key][q] = K.Q^T and dP^T[key][q] = V.dO^T (16x16x16, A from the [key][16] images), so the
//   lane holds 8 keys of ONE query — exactly the B-operand layout of dQ^T[d][q] += K^T[d][key] dS^T
//   (16x16x32, A from the transposed K image): dQ accumulates in registers.
constexpr int DQ_WAVES = 12, DQ_NT = 64 * DQ_WAVES;

template <bool DROP>
__global__ void __launch_bounds__(DQ_NT) k_attn_bwd_dq(AflAttn a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int Lp = a.Lp, LDT = Lp + 8;
  unsigned short* Kl = (unsigned short*)smem;  // [Lp][16] (swizzled)
  unsigned short* Vl = Kl + Lp * DH;           // [Lp][16] (swizzled)
  unsigned short* Kt = Vl + Lp * DH;           // [16][LDT]
  const int bh = blockIdx.x, h = bh % H, b = (bh / H) % a.B, c = bh / (H * a.B);
  const long rowbase = ((long)c * a.B + b) * a.L;
  const float* src = a.qkv + rowbase * QKV;
  const float* dO = a.dout + rowbase * DM;
  const float* Oo = a.o + rowbase * DM;
  {
    constexpr int NI = (STAGE_MAXR * 4 + DQ_NT - 1) / DQ_NT;
    f4v vk[NI], vv[NI];
    load_quads<DQ_NT, NI>(src, QKV, DM + h * DH, src, QKV, 2 * DM + h * DH, Lp, a.L, vk, vv);
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int t = threadIdx.x + i * DQ_NT, row = t >> 2, qd = t & 3;
      if (t < Lp * 4) {
        put_quad(Kl, Kt, LDT, row, qd, vk[i]);
        put_quad(Vl, nullptr, 0, row, qd, vv[i]);
      }
    }
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, li = lane & 15;
  const uint32_t key = DROP ? afl_hash32(a.drop.seeds[c], (uint32_t)(a.drop.stepctl ? *a.drop.stepctl : 0)) : 0u;
  const uint32_t drow0 = (uint32_t)((b * H + h) * a.L);
  for (int q0 = wave * 16; q0 < Lp; q0 += 16 * DQ_WAVES) {
    const int q = q0 + li;
    const bool qok = q < a.L;
    s4v qf, df;
    float dl = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float dov = qok ? dO[(long)q * DM + h * DH + 4 * g + j] : 0.f;
      qf[j] = (short)bf(qok ? src[(long)q * QKV + h * DH + 4 * g + j] : 0.f);
      df[j] = (short)bf(dov);
      dl += dov * (qok ? Oo[(long)q * DM + h * DH + 4 * g + j] : 0.f);
    }
    dl += __shfl_xor(dl, 16, 64);
    dl += __shfl_xor(dl, 32, 64);  // Delta_q = dO_q . O_q (fp32)
    const float lse = a.lse[(long)bh * Lp + q];
    f4v acc = f4v{0.f, 0.f, 0.f, 0.f};
    for (int kt = 0; kt < Lp; kt += 32) {
      const f4v s0 = mfma16(ld4(Kl + swz(kt + li, 4 * g)), qf, f4v{0.f, 0.f, 0.f, 0.f});
      const f4v s1 = mfma16(ld4(Kl + swz(kt + 16 + li, 4 * g)), qf, f4v{0.f, 0.f, 0.f, 0.f});
      const f4v p0 = mfma16(ld4(Vl + swz(kt + li, 4 * g)), df, f4v{0.f, 0.f, 0.f, 0.f});
      const f4v p1 = mfma16(ld4(Vl + swz(kt + 16 + li, 4 * g)), df, f4v{0.f, 0.f, 0.f, 0.f});
      float ds[8], mk[8];
      if (DROP) keep8(key, a.drop.layer, drow0 + q, kt + 4 * g, kt + 16 + 4 * g, a.drop.thr16, a.drop.inv_keep, mk);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int kk = kt + (j < 4 ? 4 * g + j : 16 + 4 * g + j - 4);
        const float sv = j < 4 ? s0[j] : s1[j - 4];
        const float dp = j < 4 ? p0[j] : p1[j - 4];
        const float pe = __expf(sv * a.scale - lse);
        const float p = kk < a.L ? pe : 0.f;
        ds[j] = p * (dp * (DROP ? mk[j] : 1.f) - dl);
      }
      const s8v kfr = cat8(ld4(Kt + li * LDT + kt + 4 * g), ld4(Kt + li * LDT + kt + 16 + 4 * g));
      acc = mfma32(kfr, pack8(ds), acc);
    }
    if (qok) {
      float* dst = a.dqkv + (rowbase + q) * QKV + h * DH + 4 * g;
#pragma unroll
      for (int e = 0; e < 4; ++e) dst[e] = acc[e] * a.scale;
    }
  }
}

}  // namespace

static int attn_lp(int L) { return (L + 31) / 32 * 32; }

int afl_attn_lp(int L) { return attn_lp(L); }

int afl_attn_fwd(const AflAttn& a, hipStream_t s) {
  if (a.Lp != attn_lp(a.L) || a.Lp > 1024) return (int)hipErrorInvalidValue;
  const size_t lds = (size_t)(a.Lp + 32) * DH * 2 + (size_t)DH * (a.Lp + 8 + 32) * 2;
  if (a.drop.thr16)
    hipLaunchKernelGGL(k_attn_fwd<true>, dim3(a.C * a.B * H), dim3(FW_NT), lds, s, a);
  else
    hipLaunchKernelGGL(k_attn_fwd<false>, dim3(a.C * a.B * H), dim3(FW_NT), lds, s, a);
  return (int)hipGetLastError();
}

static size_t kv_lds(int Lp) { return (size_t)Lp * DH * 2 * 2 + (size_t)DH * (Lp + 8) * 2 * 2 + (size_t)Lp * 4 * 2; }
static size_t dq_lds(int Lp) { return (size_t)Lp * DH * 2 * 2 + (size_t)DH * (Lp + 8) * 2; }

int afl_attn_bwd(const AflAttn& a, hipStream_t s) {
  if (a.Lp != attn_lp(a.L) || a.Lp > 1024) return (int)hipErrorInvalidValue;
  // raise the dynamic-LDS cap once (the first call happens eagerly, before any graph capture)
  static int cap = 0;
  if (cap == 0) {
    for (const void* f : {(const void*)k_attn_bwd_kv<true>, (const void*)k_attn_bwd_kv<false>}) {
      const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kv_lds(1024));
      if (e != hipSuccess) return (int)e;
    }
    for (const void* f : {(const void*)k_attn_bwd_dq<true>, (const void*)k_attn_bwd_dq<false>}) {
      const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)dq_lds(1024));
      if (e != hipSuccess) return (int)e;
    }
    cap = 1;
  }
  const dim3 grid(a.C * a.B * H);
  if (a.drop.thr16) {
    hipLaunchKernelGGL(k_attn_bwd_kv<true>, grid, dim3(BW_NT), kv_lds(a.Lp), s, a);
    hipLaunchKernelGGL(k_attn_bwd_dq<true>, grid, dim3(DQ_NT), dq_lds(a.Lp), s, a);
  } else {
    hipLaunchKernelGGL(k_attn_bwd_kv<false>, grid, dim3(BW_NT), kv_lds(a.Lp), s, a);
    hipLaunchKernelGGL(k_attn_bwd_dq<false>, grid, dim3(DQ_NT), dq_lds(a.Lp), s, a);
  }
  return (int)hipGetLastError();
}
