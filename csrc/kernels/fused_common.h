// Building blocks shared by the fused whole-step trainers (transformer.hip, rnn.hip): 512-thread
// workgroups of 8 waves x 16 rows, activations in LDS as bf16, GEMMs on v_mfma_f32_16x16x32_bf16,
// Adam fused into the dW epilogue, DPP / permlane row and column reductions, register LayerNorm,
// and the write-through cross-workgroup hand-off (cdna_hip_programming.md Guideline 16, R1).
// Everything that depends on a kernel's LDS map is templated on its context type CtxT<Layout>.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.h"

typedef short s8v __attribute__((ext_vector_type(8)));
typedef short s4v __attribute__((ext_vector_type(4)));
typedef __bf16 bf8v __attribute__((ext_vector_type(8)));
typedef float f4v __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
#define LDS_AS __attribute__((address_space(3)))
// Global-memory pointers carry address_space(1) explicitly: they pass through opaque asm at every phase
// barrier, and a generic pointer would demote every access to FLAT (which waits on vmcnt AND lgkmcnt).
#define GAS __attribute__((address_space(1)))
typedef GAS float gf;
typedef GAS unsigned short gu16;
typedef GAS int gi32;
typedef GAS uint32_t gu32;
typedef GAS unsigned long long gu64;


constexpr int NT = 512;  // threads per fused-trainer workgroup
constexpr int BM = 128;  // max rows per batch

namespace fk {

// bf16 round-to-nearest-even (hardware v_cvt_pk_bf16_f32, NaN preserving)
typedef float tf_f2v __attribute__((ext_vector_type(2)));
typedef __bf16 tf_b2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned short f2bf(float f) { return __builtin_bit_cast(unsigned short, (__bf16)f); }
__device__ __forceinline__ uint32_t pack_bf2(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((tf_f2v){lo, hi}, tf_b2v));
}
__device__ __forceinline__ float bf2f(unsigned short h) { return __uint_as_float(((uint32_t)h) << 16); }

struct AdamK {
  float lr_bc1, rsqrt_bc2;
  float sgd_lr;  // > 0: test mode, plain SGD p -= sgd_lr * g (exposes raw gradients to the tests)
};
constexpr float B1 = 0.9f, B2 = 0.999f, EPS = 1e-8f;

// Adam update given already-loaded state; returns the new parameter
__device__ __forceinline__ float adam_upd(float p, float& m, float& v, float g, AdamK k) {
  if (k.sgd_lr > 0.f) return p - k.sgd_lr * g;
  m = m + (1.f - B1) * (g - m);
  v = B2 * v + (1.f - B2) * g * g;
  return p - k.lr_bc1 * m * __builtin_amdgcn_rcpf(__builtin_sqrtf(v) * k.rsqrt_bc2 + EPS);
}
__device__ __forceinline__ float adam(gf* __restrict__ p, gf* __restrict__ m, gf* __restrict__ v, int idx, float g,
                                      AdamK k) {
  float pp = p[idx], mm = m[idx], vv = v[idx];
  pp = adam_upd(pp, mm, vv, g, k);
  p[idx] = pp;
  if (k.sgd_lr <= 0.f) {
    m[idx] = mm;
    v[idx] = vv;
  }
  return pp;
}

// Per-workgroup context of a fused trainer.  L supplies the LDS map: S_ACC / LDACC (fp32 GEMM output
// tile [128][LDACC]) and S_CS (column-sum partials [slots][8 waves][64]).
template <class L>
struct CtxT {
  static constexpr int LDACC = L::LDACC;
  unsigned char* smem;
  gf* P;     // master params of this client
  gf* M;
  gf* V;
  gu16* BF;  // bf16 weight copies
  gf* ws;
  int tid, lane, wave;
  int r, q;  // row-per-4-lanes layout: row, quarter

  // Phase barrier: LDS-only (global loads stay in flight, global stores are not drained), then make
  // every base value opaque so the compiler recomputes addresses per phase instead of keeping hundreds
  // of CSE'd pointers live across the whole step (which spills to scratch).
  __device__ __forceinline__ void bar() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    asm volatile("" : "+s"(P), "+s"(M), "+s"(V), "+s"(BF), "+s"(ws));
    asm volatile("" : "+v"(r), "+v"(q), "+v"(lane), "+v"(wave));
    bound();
  }
  // re-establish the value ranges the opaque asm hid, so index products select the full-rate
  // v_mul_u32_u24 instead of the quarter-rate v_mul_lo_u32
  __device__ __forceinline__ void bound() {
    r &= 127;
    q &= 3;
    lane &= 63;
    wave &= 7;
  }
  // Wave-local phase boundary: no s_barrier.  Valid where every LDS byte the next phase reads was
  // written by the SAME wave (row-per-wave layout: a wave's GEMM rows, elementwise rows and A-operand
  // rows coincide; a wave's LDS operations execute in order).  Keeps the opaque-address trick of bar().
  __device__ __forceinline__ void soft() {
    asm volatile("" : "+s"(P), "+s"(M), "+s"(V), "+s"(BF), "+s"(ws));
    asm volatile("" : "+v"(r), "+v"(q), "+v"(lane), "+v"(wave));
    bound();
  }
  // Full barrier (drains global stores: publishes Adam's writes to every wave)
  __device__ __forceinline__ void full_sync() {
    __syncthreads();
    asm volatile("" : "+s"(P), "+s"(M), "+s"(V), "+s"(BF), "+s"(ws));
    asm volatile("" : "+v"(r), "+v"(q), "+v"(lane), "+v"(wave));
    bound();
  }

  __device__ float* acc() const { return (float*)(smem + L::S_ACC); }
  __device__ unsigned short* u16(int off) const { return (unsigned short*)(smem + off); }
  __device__ float* cs(int v) const { return (float*)(smem + L::S_CS) + v * 8 * 64; }
  __device__ gf* wsf(long off) const { return ws + off; }
  // raw buffer descriptor over the (workgroup-uniform) workspace base, for 16-byte sc1 accesses
  __device__ __amdgpu_buffer_rsrc_t wrs() const {
    return __builtin_amdgcn_make_buffer_rsrc((void*)(float*)ws, 0, 0x7fffffff, 0x00020000);
  }
};

// ---------------------------------------------------------------- fragments
__device__ __forceinline__ s8v lds_row_frag(const unsigned short* base, int ld, int r0, int k0, int lane) {
  const unsigned short* p = base + (r0 + (lane & 15)) * ld + k0 + 8 * (lane >> 4);
  return *(const LDS_AS s8v*)p;
}
// A[m][k] = S[k][m] (S row-major [k rows][m cols]); two transposed 4x16 reads per 16-lane group
__device__ __forceinline__ s8v lds_col_frag(const unsigned short* S, int ld, int k0, int m0, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const unsigned short* a1 = S + (k0 + 8 * g + q) * ld + m0 + 4 * p;
  const unsigned short* a2 = a1 + 4 * ld;
  s4v r1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s4v*)a1);
  s4v r2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s4v*)a2);
  s8v r;
  r[0] = r1[0]; r[1] = r1[1]; r[2] = r1[2]; r[3] = r1[3];
  r[4] = r2[0]; r[5] = r2[1]; r[6] = r2[2]; r[7] = r2[3];
  return r;
}
__device__ __forceinline__ s8v glb_frag(const gu16* W, int ldk, int n0, int k0, int lane) {
  return *(const GAS s8v*)(W + (n0 + (lane & 15)) * ldk + k0 + 8 * (lane >> 4));
}
__device__ __forceinline__ f4v mfma(s8v a, s8v b, f4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf8v, a), __builtin_bit_cast(bf8v, b), c, 0, 0, 0);
}

// ACC[128][N] = A[128][K] (LDS bf16, ld lda) x W^T, W = global bf16 [N][K] row-major (eval path)
template <int N, int K, class CT>
__device__ __forceinline__ void gemm_xw(const CT& c, const unsigned short* A, int lda, const gu16* W) {
  constexpr int NTL = N / 16;
  f4v acc[NTL];
#pragma unroll
  for (int t = 0; t < NTL; ++t) acc[t] = f4v{0.f, 0.f, 0.f, 0.f};
  const int r0 = 16 * c.wave;
#pragma unroll
  for (int k0 = 0; k0 < K; k0 += 32) {
    s8v a = lds_row_frag(A, lda, r0, k0, c.lane);
#pragma unroll
    for (int t = 0; t < NTL; ++t) acc[t] = mfma(a, glb_frag(W, K, 16 * t, k0, c.lane), acc[t]);
  }
  float* out = c.acc();
#pragma unroll
  for (int t = 0; t < NTL; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) out[(r0 + 4 * (c.lane >> 4) + i) * CT::LDACC + 16 * t + (c.lane & 15)] = acc[t][i];
}

// ---- weight fragments prefetched into registers a phase ahead of their GEMM ----
template <int N, int K>
struct WFr {
  s8v f[N / 16][K / 32];
};
template <int N, int K>
__device__ __forceinline__ void wload(WFr<N, K>& w, const gu16* W, int lane) {
#pragma unroll
  for (int t = 0; t < N / 16; ++t)
#pragma unroll
    for (int kk = 0; kk < K / 32; ++kk) w.f[t][kk] = glb_frag(W, K, 16 * t, 32 * kk, lane);
}
template <int N, int K, class CT>
__device__ __forceinline__ void gemm_pf(const CT& c, const unsigned short* A, int lda, const WFr<N, K>& w) {
  constexpr int NTL = N / 16;
  f4v acc[NTL];
#pragma unroll
  for (int t = 0; t < NTL; ++t) acc[t] = f4v{0.f, 0.f, 0.f, 0.f};
  const int r0 = 16 * c.wave;
#pragma unroll
  for (int kk = 0; kk < K / 32; ++kk) {
    s8v a = lds_row_frag(A, lda, r0, 32 * kk, c.lane);
#pragma unroll
    for (int t = 0; t < NTL; ++t) acc[t] = mfma(a, w.f[t][kk], acc[t]);
  }
  float* out = c.acc();
#pragma unroll
  for (int t = 0; t < NTL; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) out[(r0 + 4 * (c.lane >> 4) + i) * CT::LDACC + 16 * t + (c.lane & 15)] = acc[t][i];
}

template <class CT>
__device__ __forceinline__ float cs_total(const CT& c, int v, int col);

// Matrix weight descriptor for the dW+Adam epilogue
struct MatW {
  int off;        // param offset of W[n][k]
  int n_real, k_real;
  int wf, wf_ld;  // bf16 WF [n][k] copy (ushort offset in BF region, row stride)
  int wt, wt_ld;  // bf16 WT [k][n] copy (-1 = none)
};

// dW[n][k] = sum_b DY[b][n] X[b][k] over 128 rows, then Adam on the real entries.  The Adam state
// (p, m, v) of each lane's 4 accumulator elements is loaded before the MFMAs so the global latency
// overlaps the tile's transposed LDS reads and matrix work.
// gfx9 counts loads and stores in ONE vmcnt queue, in issue order: a load issued behind a burst of
// Adam stores waits for their acknowledgements before its data can be used.  So every update below is
// split into a load part (issue it BEFORE the stores of earlier updates) and an apply part.
template <int TS>
struct DwSt {  // Adam state of up to TS of this wave's dW tiles (tile t = wave + 8j)
  float p[TS][4], m[TS][4], v[TS][4];
};
template <int MT, int NTL>
using DwS = DwSt<(MT * NTL + 7) / 8>;
template <int MT, int NTL, int TS, class CT>
__device__ __forceinline__ void dw_ld(const CT& c, MatW mw, DwSt<TS>& s) {
  constexpr int T = (MT * NTL + 7) / 8;
  static_assert(TS >= T, "state too small");
#pragma unroll
  for (int j = 0; j < T; ++j) {
    const int t = c.wave + 8 * j;
    if (t >= MT * NTL) break;
    const int mt = t / NTL, nt = t % NTL;
    const int kk = 16 * nt + (c.lane & 15);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int n = 16 * mt + 4 * (c.lane >> 4) + i;
      const bool ok = n < mw.n_real && kk < mw.k_real;
      const int idx = ok ? mw.off + n * mw.k_real + kk : mw.off;
      s.p[j][i] = c.P[idx];
      s.m[j][i] = c.M[idx];
      s.v[j][i] = c.V[idx];
    }
  }
}
// dW[n][k] = sum_b DY[b][n] X[b][k] over 128 rows (all tiles' MFMAs first), then Adam on the real entries
// img (optional): an LDS copy [n][img_ld] of the bf16 weight that also receives the updated values
template <int MT, int NTL, int TS, class CT>
__device__ __forceinline__ void dw_apply(const CT& c, const unsigned short* DY, int ldy, const unsigned short* X,
                                         int ldx, MatW mw, AdamK k, DwSt<TS>& s, unsigned short* img = nullptr,
                                         int img_ld = 0) {
  constexpr int T = (MT * NTL + 7) / 8;
  static_assert(TS >= T, "state too small");
  f4v acc[T];
#pragma unroll
  for (int j = 0; j < T; ++j) {
    const int t = c.wave + 8 * j;
    acc[j] = f4v{0.f, 0.f, 0.f, 0.f};
    if (t >= MT * NTL) break;
    const int mt = t / NTL, nt = t % NTL;
#pragma unroll
    for (int b0 = 0; b0 < BM; b0 += 32)
      acc[j] = mfma(lds_col_frag(DY, ldy, b0, 16 * mt, c.lane), lds_col_frag(X, ldx, b0, 16 * nt, c.lane), acc[j]);
  }
#pragma unroll
  for (int j = 0; j < T; ++j) {
    const int t = c.wave + 8 * j;
    if (t >= MT * NTL) break;
    const int mt = t / NTL, nt = t % NTL;
    const int kk = 16 * nt + (c.lane & 15);
    // the lane's 4 rows n0..n0+3 are 4 CONSECUTIVE elements of the transposed copy's row kk: one 8-byte
    // store instead of four scattered 2-byte ones (all-or-none real when n_real % 4 == 0)
    const int n0 = 16 * mt + 4 * (c.lane >> 4);
    const bool vec_t = mw.wt >= 0 && ((mw.n_real | mw.wt | mw.wt_ld) & 3) == 0;
    unsigned short hv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int n = n0 + i;
      hv[i] = 0;
      if (n < mw.n_real && kk < mw.k_real) {
        const int idx = mw.off + n * mw.k_real + kk;
        const float pn = adam_upd(s.p[j][i], s.m[j][i], s.v[j][i], acc[j][i], k);
        c.P[idx] = pn;
        if (k.sgd_lr <= 0.f) {
          c.M[idx] = s.m[j][i];
          c.V[idx] = s.v[j][i];
        }
        const unsigned short h = f2bf(pn);
        hv[i] = h;
        c.BF[mw.wf + n * mw.wf_ld + kk] = h;
        if (img) img[n * img_ld + kk] = h;
        if (mw.wt >= 0 && !vec_t) c.BF[mw.wt + kk * mw.wt_ld + n] = h;
      }
    }
    if (vec_t && n0 < mw.n_real && kk < mw.k_real)
      *(GAS u32x2*)(c.BF + mw.wt + kk * mw.wt_ld + n0) =
          u32x2{(uint32_t)hv[0] | ((uint32_t)hv[1] << 16), (uint32_t)hv[2] | ((uint32_t)hv[3] << 16)};
  }
}
template <int MT, int NTL, class CT>
__device__ __forceinline__ void gemm_dw_adam(const CT& c, const unsigned short* DY, int ldy, const unsigned short* X,
                                             int ldx, MatW mw, AdamK k) {
  DwS<MT, NTL> s;
  dw_ld<MT, NTL>(c, mw, s);
  dw_apply<MT, NTL>(c, DY, ldy, X, ldx, mw, k, s);
}

// Adam on up to 512 small-vector elements (biases, LayerNorm affine) in parallel: thread tid handles
// element tid of the concatenation of the listed vectors; gradient = column sum CS[v] over 8 waves.
// one parameter's Adam state, loaded ahead of the stores of earlier updates (see dw_ld)
struct AdamS {
  float p, m, v;
};
template <class CT>
__device__ __forceinline__ AdamS adam_ld(const CT& c, int idx) {
  return AdamS{c.P[idx], c.M[idx], c.V[idx]};
}
template <class CT>
__device__ __forceinline__ void adam_st(const CT& c, int idx, AdamS s, float g, AdamK k) {
  const float pn = adam_upd(s.p, s.m, s.v, g, k);
  c.P[idx] = pn;
  if (k.sgd_lr <= 0.f) {
    c.M[idx] = s.m;
    c.V[idx] = s.v;
  }
}
struct VecG {
  int off, n, csv;  // param offset, length, column-sum slot (-1: value supplied in `g0`)
  int cbase = 0;    // first column of the slot holding element 0
};
// Adam on vectors whose gradients are column sums: each thread owns at most one element of the list
template <int NV, class CT>
__device__ __forceinline__ AdamS adam_vecs_ld(const CT& c, const VecG (&vs)[NV]) {
  AdamS s{0.f, 0.f, 0.f};
  int e = c.tid;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    if (e >= 0 && e < vs[i].n) s = adam_ld(c, vs[i].off + e);
    e -= vs[i].n;
  }
  return s;
}
template <int NV, class CT>
__device__ __forceinline__ void adam_vecs_st(const CT& c, const VecG (&vs)[NV], AdamS s, AdamK k, float g0 = 0.f) {
  int e = c.tid;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    if (e >= 0 && e < vs[i].n) {
      const float g = vs[i].csv >= 0 ? cs_total(c, vs[i].csv, vs[i].cbase + e) : g0;
      adam_st(c, vs[i].off + e, s, g, k);
    }
    e -= vs[i].n;
  }
}
template <int NV, class CT>
__device__ __forceinline__ void adam_vecs(const CT& c, const VecG (&vs)[NV], AdamK k, float g0 = 0.f) {
  adam_vecs_st(c, vs, adam_vecs_ld(c, vs), k, g0);
}

// ---- cross-lane reductions without LDS ----
// Element layout: lane l of wave w owns row r = 16w + (l & 15) and quarter q = l >> 4 of that row.
// A column sum over the wave's 16 rows is a reduction over 16 consecutive lanes (DPP quad_perm,
// row_half_mirror, row_mirror / row_ror).  A row sum over the 4 quarters pairs lanes
// l, l^16, l^32: gfx950 v_permlane16_swap / v_permlane32_swap.
template <int CTRL>
__device__ __forceinline__ float dpp(float a) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(a), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float sum16lanes(float a) {
  a += dpp<0xB1>(a);   // quad_perm [1,0,3,2]
  a += dpp<0x4E>(a);   // quad_perm [2,3,0,1]
  a += dpp<0x141>(a);  // row_half_mirror
  a += dpp<0x140>(a);  // row_mirror
  return a;
}
__device__ __forceinline__ float xor16(float a) {
  auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(a), false, false);
  return __uint_as_float(p[0]) + __uint_as_float(p[1]) - a;  // = a[l ^ 16]
}
__device__ __forceinline__ float xor32(float a) {
  auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(a), false, false);
  return __uint_as_float(p[0]) + __uint_as_float(p[1]) - a;  // = a[l ^ 32]
}

// Column sums over a wave's 16 rows as a DPP reduce-SCATTER: each level pairs lane i with a partner
// that holds the same column set, keeps one half of the values and adds the partner's copy of that
// half, so W values take W-1 DPP adds (W/2 + W/4 + ...) instead of 4*W, and lane i ends up with
// the total of ONE column.  Split bits in order 2 (row_half_mirror, i <-> i^7: first level only),
// 0 (i^1), 1 (i^2), 3 (row_ror 8 = i^8); bits left over for W < 16 are summed in place.
template <int BIT>
__device__ __forceinline__ float dpp_pair(float a) {
  return dpp<BIT == 2 ? 0x141 : BIT == 0 ? 0xB1 : BIT == 1 ? 0x4E : 0x128>(a);
}
template <int N, int L>
__device__ __forceinline__ void rs_level(float* v, int i, int& j) {
  constexpr int BIT = L == 0 ? 2 : L == 1 ? 0 : L == 2 ? 1 : 3;
  constexpr int H = N / 2;
  const bool b = (i >> BIT) & 1;
  float keep[H], send[H];
#pragma unroll
  for (int k = 0; k < H; ++k) {
    keep[k] = b ? v[k + H] : v[k];
    send[k] = b ? v[k] : v[k + H];
  }
#pragma unroll
  for (int k = 0; k < H; ++k) v[k] = keep[k] + dpp_pair<BIT>(send[k]);
  j += b ? H : 0;
}
// W values of this lane's row -> cs(v)[wave*64 + base + column], summed over the wave's 16 rows
template <int W, class CT>
__device__ __forceinline__ void colsum_rs(const CT& c, int v, const float* x, int base) {
  static_assert(W == 4 || W == 8 || W == 16, "W");
  float s[W];
#pragma unroll
  for (int j = 0; j < W; ++j) s[j] = x[j];
  const int i = c.lane & 15;
  int j = 0;
  rs_level<W, 0>(s, i, j);
  rs_level<W / 2, 1>(s, i, j);
  if constexpr (W >= 8) rs_level<W / 4, 2>(s, i, j);
  if constexpr (W >= 16) rs_level<W / 8, 3>(s, i, j);
  int rest = 0;  // split bits not used at this width: plain pair sums
  if constexpr (W == 4) {
    s[0] += dpp_pair<1>(s[0]);
    rest |= 2;
  }
  if constexpr (W <= 8) {
    s[0] += dpp_pair<3>(s[0]);
    rest |= 8;
  }
  if ((i & rest) == 0) c.cs(v)[c.wave * 64 + base + j] = s[0];
}
// column partial sums of 16 values per lane (64-wide rows): CS[v][wave][q*16 + j]
template <class CT>
__device__ __forceinline__ void colsum16(const CT& c, int v, const float (&x)[16]) {
  colsum_rs<16>(c, v, x, (c.lane >> 4) * 16);
}
template <int W, class CT>
__device__ __forceinline__ void colsumW(const CT& c, int v, const float (&x)[W], int colbase) {
  colsum_rs<W>(c, v, x, colbase);
}
template <class CT>
__device__ __forceinline__ float cs_total(const CT& c, int v, int col) {
  asm volatile("" : "+v"(col));  // recompute the 8 addresses here: hoisted out of the step loop they spill
  float s = 0.f;
#pragma unroll
  for (int w = 0; w < 8; ++w) s += c.cs(v)[w * 64 + col];
  return s;
}

// row-wise sum over the 4 lanes (quarters) of a row: lanes l, l^16, l^32, l^48.  permlane16_swap(a, a)
// leaves this lane's and its l^16 partner's value in the two outputs (in either order), so their sum
// is the pair sum exactly; the same with permlane32_swap for l^32.
__device__ __forceinline__ float rsum4(float a) {
  auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(a), false, false);
  a = __uint_as_float(p[0]) + __uint_as_float(p[1]);
  auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(a), false, false);
  return __uint_as_float(q[0]) + __uint_as_float(q[1]);
}

// LayerNorm forward on 16 values/lane (64-wide row): returns xhat in place, rstd
__device__ __forceinline__ float ln_fwd(float (&x)[16]) {
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 16; ++j) s += x[j];
  const float mean = rsum4(s) * (1.f / 64.f);
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    x[j] -= mean;
    ss += x[j] * x[j];
  }
  const float var = rsum4(ss) * (1.f / 64.f);
  const float rstd = __builtin_amdgcn_rsqf(var + 1e-5f);
#pragma unroll
  for (int j = 0; j < 16; ++j) x[j] *= rstd;
  return rstd;
}
// LayerNorm backward: dy -> dx given xhat, rstd, gamma (per column, 16 values of this lane)
__device__ __forceinline__ void ln_bwd(float (&dx)[16], const float (&dy)[16], const float (&xh)[16], float rstd,
                                       const float (&gamma)[16]) {
  float a = 0.f, b = 0.f, g[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    g[j] = dy[j] * gamma[j];
    a += g[j];
    b += g[j] * xh[j];
  }
  a = rsum4(a) * (1.f / 64.f);
  b = rsum4(b) * (1.f / 64.f);
#pragma unroll
  for (int j = 0; j < 16; ++j) dx[j] = rstd * (g[j] - a - xh[j] * b);
}

__device__ __forceinline__ void load16(float (&x)[16], const gf* p) {
#pragma unroll
  for (int j = 0; j < 16; j += 4) {
    f4v v = *(const GAS f4v*)(p + j);
    x[j] = v[0]; x[j + 1] = v[1]; x[j + 2] = v[2]; x[j + 3] = v[3];
  }
}
__device__ __forceinline__ void load8(float (&x)[8], const gf* p) {
  f4v a = *(const GAS f4v*)p, b = *(const GAS f4v*)(p + 4);
  x[0] = a[0]; x[1] = a[1]; x[2] = a[2]; x[3] = a[3];
  x[4] = b[0]; x[5] = b[1]; x[6] = b[2]; x[7] = b[3];
}
__device__ __forceinline__ void store16(gf* p, const float (&x)[16]) {
#pragma unroll
  for (int j = 0; j < 16; j += 4) *(GAS f4v*)(p + j) = f4v{x[j], x[j + 1], x[j + 2], x[j + 3]};
}
typedef uint32_t u4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ s8v pack8bf(const float* x) {
  u4v u;
  u[0] = pack_bf2(x[0], x[1]);
  u[1] = pack_bf2(x[2], x[3]);
  u[2] = pack_bf2(x[4], x[5]);
  u[3] = pack_bf2(x[6], x[7]);
  return __builtin_bit_cast(s8v, u);
}
__device__ __forceinline__ void store16bf(unsigned short* p, const float (&x)[16]) {
  *(LDS_AS s8v*)p = pack8bf(x);
  *(LDS_AS s8v*)(p + 8) = pack8bf(x + 8);
}

// ---- cross-workgroup hand-off (branch-parallel mode; cdna_hip_programming.md Guideline 16, R1) ----
// payload: 16-byte write-through (sc1) stores; the storing wave drains (vmcnt 0), then ONE lane stores
// the flag.  Consumer: the wave polls the flag relaxed (bounded spin), then sc1 loads of the payload
// (never plain loads: there is no acquire).
// 16-byte write-through store / sc1 load at a BYTE offset from the workspace base (buffer_*_dwordx4
// sc1; a 16-B sc1 store costs what a plain one does, 8-B ones 2.7x per byte: MI355X_MICROARCH price list)
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
template <class CT>
__device__ __forceinline__ void st_wt16(const CT& c, int byte_off, u32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, c.wrs(), byte_off, 0, 16);
}
template <class CT>
__device__ __forceinline__ u32x4 ld_wt16(const CT& c, int byte_off) {
  return __builtin_amdgcn_raw_buffer_load_b128(c.wrs(), byte_off, 0, 16);
}
// A missing partner becomes an error, not a hang: ~2^24 polls of (load latency + s_sleep 1) is tens of
// seconds, orders of magnitude above any late co-resident dispatch (validation / checkpoint kernels on other
// streams run for milliseconds).  A time-based deadline (s_memrealtime every 1024 polls) measured 0.6 %
// slower on the TransformerModel headline (tools/ab_native.sh, same box, 2 x 2 runs: 94.07 vs 94.68
// rounds/s: the extra loop code moved the hot kernel's code placement), so the wait stays a poll count.
constexpr long XWG_MAX_SPINS = 1L << 24;
// Per-WAVE hand-off (row-per-wave layout: wave w produces and consumes rows 16w..16w+15 on both sides).
// The same R1 protocol with the wave as the storing unit: the wave's own sc1 payload stores, its own
// vmcnt(0) drain, then its lane 0 stores the wave's flag; the consumer wave polls its flag (all lanes one
// address: one request) and only then issues its sc1 payload loads.  No workgroup barrier on either
// side: a wave hands its rows over when IT is done instead of when the slowest wave is, and the consumer
// wave starts when ITS rows have landed.  Flags sit on 128-byte lines of their own.
template <class CT>
__device__ __forceinline__ void wave_publish(const CT& c, gu32* flag, uint32_t value) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (c.lane == 0) __hip_atomic_store(flag, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Per-wave hand-off flags of one client ([AFL_TF_SYNC_WORDS] zeroed words), each on a 128-byte line:
// group XF_VIT / XF_LAB: the branch output rows of wave w are ready (value = step); XF_BVIT / XF_BLAB:
// d(branch output) rows of wave w are ready (value = step << 1 | NaN abort); word XF_TMO: timeout
constexpr int XF_VIT = 0, XF_LAB = 1, XF_BVIT = 2, XF_BLAB = 3, XF_TMO = 4 * 8 * 32;
__device__ __forceinline__ gu32* xf(gu32* xflag, int group, int wave) { return xflag + (group * 8 + wave) * 32; }
// waits until (flag_a >> shift) >= want and (flag_b >> shift) >= want; returns flag_a's value
// (wave-uniform), or 0xFFFFFFFF on timeout (also raises *tmo)
template <class CT>
__device__ __forceinline__ uint32_t wave_wait(const CT& c, gu32* flag_a, gu32* flag_b, uint32_t want, int shift,
                                              gu32* tmo) {
  uint32_t v = 0;
  for (long spins = 0;; ++spins) {
    v = __builtin_amdgcn_readfirstlane(__hip_atomic_load(flag_a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    const uint32_t w = flag_b == flag_a
                           ? v
                           : __builtin_amdgcn_readfirstlane(__hip_atomic_load(flag_b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    if ((v >> shift) >= want && (w >> shift) >= want) break;
    if (spins > XWG_MAX_SPINS) {
      v = 0xFFFFFFFFu;
      if (c.lane == 0) __hip_atomic_store(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keeps the payload loads below the poll
  return v;
}

// write the bf16 copies of one matrix from the master params
template <class CT>
__device__ void init_copies(const CT& c, MatW mw) {
  for (int e = c.tid; e < mw.n_real * mw.k_real; e += NT) {
    const int n = e / mw.k_real, kk = e % mw.k_real;
    unsigned short h = f2bf(c.P[mw.off + e]);
    c.BF[mw.wf + n * mw.wf_ld + kk] = h;
    if (mw.wt >= 0) c.BF[mw.wt + kk * mw.wt_ld + n] = h;
  }
}


__device__ __forceinline__ int opaque(int v) {
  asm volatile("" : "+v"(v));
  return v;
}

// ACC row r, columns c0..c0+15 -> hand-off slot as bf16 (row stride 64; two write-through 16-byte
// stores).  The gradient crosses in bf16, the precision its consumer's GEMM operands have anyway:
// half the bytes on the step's critical hand-off.
template <class CT>
__device__ __forceinline__ void put_grad(const CT& c, long slot, int r, int c0) {
  const float* acc = c.acc() + r * CT::LDACC + c0;
  float x[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) x[j] = acc[j];
  const int bo = (int)slot * 4 + opaque(r * 64 + c0) * 2;
  st_wt16(c, bo, __builtin_bit_cast(u32x4, pack8bf(x)));
  st_wt16(c, bo + 16, __builtin_bit_cast(u32x4, pack8bf(x + 8)));
}
// 8 bf16 packed in a 16-byte granule -> fp32
__device__ __forceinline__ void unpack8bf(u32x4 v, float* x) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    x[2 * k] = __uint_as_float(v[k] << 16);
    x[2 * k + 1] = __uint_as_float(v[k] & 0xFFFF0000u);
  }
}



}  // namespace fk
