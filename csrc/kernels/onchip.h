// Shared device building blocks of the on-chip fused trainers (tf2.hip: TransformerModel, rnn2.hip:
// RNNModel).  Both keep a client's whole model on chip for a round: fp32 master weights in AGPRs (ar / aw),
// Adam moments in a per-workgroup global slab (mom_ld / mom_st), bf16 weight images in LDS read as MFMA A
// operands (wfrag forward, wtfrag transposed for d(input)), activations chained in registers in the
// "T layout" (lane (b, g) of wave w holds features 16t + 4g + i of batch row 16w + b), dW operands in
// XOR-swizzled LDS tiles read with ds_read_b64_tr_b16 (tfrag), per-wave cross-workgroup hand-offs through
// write-through buffer stores and flag words (publish / await).  See tf2.hip's header for the design.
#pragma once
#include "common.h"
#include "kernels.h"
#include "fused_common.h"

namespace oc {

typedef float of2v __attribute__((ext_vector_type(2)));
using fk::u32x4;
typedef unsigned int u32x2v __attribute__((ext_vector_type(2)));
typedef unsigned char uchar;

constexpr int NTH = 512;

// weight images: bf16 [rows][ld] with the K axis permuted (pcol); ld padded by 8 elements
constexpr int LD32 = 40 * 2, LD64 = 72 * 2, LD128 = 136 * 2;  // row strides in bytes

// ------------------------------------------------------------------------------ small helpers
// every LDS access goes through an address_space(3) pointer (a generic one would become FLAT, which
// counts in vmcnt too and breaks the hand-off's counted waits)
__device__ __forceinline__ LDS_AS float* ldsf(uchar* base, int byte_off) { return (LDS_AS float*)(base + byte_off); }
__device__ __forceinline__ LDS_AS uint32_t* ldsu(uchar* base, int byte_off) {
  return (LDS_AS uint32_t*)(base + byte_off);
}
__device__ __forceinline__ uint32_t pk2(float a, float b) { return fk::pack_bf2(a, b); }
__device__ __forceinline__ s8v pk8(float a0, float a1, float a2, float a3, float b0, float b1, float b2, float b3) {
  u32x4 u{pk2(a0, a1), pk2(a2, a3), pk2(b0, b1), pk2(b2, b3)};
  return __builtin_bit_cast(s8v, u);
}
// B fragment of k-step s from a T-layout register row (tiles 2s and 2s+1)
__device__ __forceinline__ s8v bfrag(const float* v, int s) {
  const float* a = v + 8 * s;
  return pk8(a[0], a[1], a[2], a[3], a[4], a[5], a[6], a[7]);
}
__device__ __forceinline__ s8v bfrag_lo(const float* v) {  // K = 16 padded to 32: second half zero
  return pk8(v[0], v[1], v[2], v[3], 0.f, 0.f, 0.f, 0.f);
}
__device__ __forceinline__ f4v mma(s8v a, s8v b, f4v c) { return fk::mfma(a, b, c); }
constexpr f4v Z4 = {0.f, 0.f, 0.f, 0.f};
// K <= 16 GEMMs (a branch's dense / ffn.3 input, ffn.0's 6 outputs, layer 1 of the GRU, the RNN head's fc2
// outputs): v_mfma_f32_16x16x16_bf16 with 4-element operands — lane group g supplies k = 4g .. 4g + 3 for both
// operands and the D layout is that of the 16x16x32 form, so the same T-layout chain works without the zero
// upper half (one MFMA pass less and no zero-filled operand registers)
__device__ __forceinline__ f4v mma16(s4v a, s4v b, f4v c) { return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0); }
__device__ __forceinline__ s4v bfrag4(const float* v) {
  return __builtin_bit_cast(s4v, u32x2v{pk2(v[0], v[1]), pk2(v[2], v[3])});
}

// permuted K position of weight column k: the 8 values lane group g of k-step s multiplies are
// columns {32s + 4g + i, 32s + 16 + 4g + i} (tiles 2s, 2s+1 of the T layout) -> stored contiguously
__host__ __device__ constexpr int pcol(int k) {
  return 32 * (k >> 5) + 8 * ((k >> 2) & 3) + 4 * ((k >> 4) & 1) + (k & 3);
}

// forward A fragment: W rows 16T + (lane & 15), permuted K chunk of k-step s (one ds_read_b128)
__device__ __forceinline__ s8v wfrag(const uchar* img, int ld, int T, int s, int lane) {
  return *(const LDS_AS s8v*)(img + (16 * T + (lane & 15)) * ld + (32 * s + 8 * (lane >> 4)) * 2);
}
// its K <= 16 form for mma16: the first 4 (pcol stores k = 4g .. 4g + 3 at 8g .. 8g + 3; one ds_read_b64)
__device__ __forceinline__ s4v wfrag4(const uchar* img, int ld, int T, int lane) {
  return *(const LDS_AS s4v*)(img + (16 * T + (lane & 15)) * ld + 16 * (lane >> 4));
}
__device__ __forceinline__ s4v tr16(const uchar* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s4v*)p);
}
__device__ __forceinline__ s8v cat44(s4v a, s4v b) {
  s8v r;
  r[0] = a[0]; r[1] = a[1]; r[2] = a[2]; r[3] = a[3];
  r[4] = b[0]; r[5] = b[1]; r[6] = b[2]; r[7] = b[3];
  return r;
}
// backward A fragment (d input = dY . W, computed as W^T . dY^T): lane (m, g) needs W[n][16T + m] for
// n = 32s + 16h + 4g + j (h = 0, 1; j = 0..3) -> two transposed reads of the same image.  Rows at or
// past `nrows` read as zero (hi == false drops the second half: images with <= 16 rows).
template <bool HI>
__device__ __forceinline__ s8v wtfrag(const uchar* img, int ld, int T, int s, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int col = 32 * (T >> 1) + 8 * p + 4 * (T & 1);
  const uchar* a = img + (32 * s + 4 * g + q) * ld + col * 2;
  s4v lo = tr16(a);
  s4v hi = {0, 0, 0, 0};
  if (HI) hi = tr16(a + 16 * ld);
  return cat44(lo, hi);
}

// the K <= 16 form of wtfrag<false> (images with <= 16 rows: the first transposed read only) for mma16
__device__ __forceinline__ s4v wtfrag4(const uchar* img, int ld, int T, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  return tr16(img + (4 * g + q) * ld + (32 * (T >> 1) + 8 * p + 4 * (T & 1)) * 2);
}

// XOR-swizzled activation tiles [128 rows][W bf16] (8-byte chunks); chosen so the T-layout row stores
// (16 rows x one chunk per instruction) and the dW transposed reads (rows 8g+q, 8g+q+4, chunks 4T+p)
// are conflict-free
__device__ __forceinline__ int sw64(int r) {
  return (r & 1) | (((r >> 2) & 1) << 1) | (((r >> 1) & 1) << 2) | (((r >> 3) & 1) << 3);
}
__device__ __forceinline__ int t64(int r, int c8) { return r * 128 + ((c8 ^ sw64(r)) << 3); }
__device__ __forceinline__ int sw128(int r) {
  return ((((r & 3) | (((r >> 3) & 1) << 2))) << 2) | ((r >> 2) & 1) | (((r >> 3) & 1) << 1);
}
__device__ __forceinline__ int t128(int r, int c8) { return r * 256 + ((c8 ^ sw128(r)) << 3); }
__device__ __forceinline__ int t32(int r, int c8) { return r * 64 + ((c8 ^ ((r >> 1) & 7)) << 3); }
__device__ __forceinline__ int t16(int r, int c8) {
  const int pr = r ^ (((r >> 3) & 1) << 2);
  return pr * 32 + ((c8 ^ ((pr >> 2) & 3)) << 3);
}
enum { TK16 = 0, TK32, TK64, TK128 };
template <int K>
__device__ __forceinline__ int toff(int r, int c8) {
  if constexpr (K == TK16) return t16(r, c8);
  else if constexpr (K == TK32) return t32(r, c8);
  else if constexpr (K == TK64) return t64(r, c8);
  else return t128(r, c8);
}
// 4 consecutive features (one 8-byte chunk) of a row
template <int K>
__device__ __forceinline__ void st4(uchar* tile, int r, int c8, const float* x) {
  *(LDS_AS u32x2v*)(tile + toff<K>(r, c8)) = u32x2v{pk2(x[0], x[1]), pk2(x[2], x[3])};
}
// dW operand fragment: lane (i, g) gets tile[r0 + 8g + j][16T + i], j = 0..7 (two transposed reads)
template <int K>
__device__ __forceinline__ s8v tfrag(const uchar* tile, int r0, int T, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int row = r0 + 8 * g + q;
  return cat44(tr16(tile + toff<K>(row, 4 * T + p)), tr16(tile + toff<K>(row + 4, 4 * T + p)));
}

// 16 fp32 of a T-layout row from an fp32 LDS vector (features 16t + 4g + i)
__device__ __forceinline__ void vec16(float (&x)[16], const uchar* vec, int g) {
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const f4v v = *(const LDS_AS f4v*)(vec + (16 * t + 4 * g) * 4);
    x[4 * t] = v[0]; x[4 * t + 1] = v[1]; x[4 * t + 2] = v[2]; x[4 * t + 3] = v[3];
  }
}
// The fp32 vectors sit past 64 KB of LDS, beyond a ds_read's 16-bit immediate offset: addressed from the
// vector base plus per-read constants the compiler materialises one v_add per read.  lane_vec() makes
// (vector base + this lane's 16 g bytes) ONE opaque VGPR per phase; vec16g reads at immediate offsets from it.
__device__ __forceinline__ const uchar* lane_vec(const uchar* vec, int g) {
  int o = 16 * g;
  asm volatile("" : "+v"(o));
  return vec + o;
}
__device__ __forceinline__ void vec16g(float (&x)[16], const uchar* vg) {
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const f4v v = *(const LDS_AS f4v*)(vg + 64 * t);
    x[4 * t] = v[0]; x[4 * t + 1] = v[1]; x[4 * t + 2] = v[2]; x[4 * t + 3] = v[3];
  }
}
__device__ __forceinline__ void vec8(float (&x)[8], const uchar* vec, int g) {  // 32-wide: tiles 0, 1
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const f4v v = *(const LDS_AS f4v*)(vec + (16 * t + 4 * g) * 4);
    x[4 * t] = v[0]; x[4 * t + 1] = v[1]; x[4 * t + 2] = v[2]; x[4 * t + 3] = v[3];
  }
}

// column sums over the wave's 16 rows of W values per lane (DPP reduce-scatter, fused_common.h): each
// lane ends with the sum of one feature; the caller sends it to a per-wave slot (head) or a fixed-point LDS
// accumulator (branches, below)
//
// Cross-wave accumulation that is bit-reproducible BY CONSTRUCTION: every fp32 partial is rounded to an integer
// number of quanta (quantum 2^-34) and the waves add these integers with fp64 LDS atomics.  With |partial| < 2^16
// an addend is an integer below 2^50 and any sum of at most 8 of them stays below 2^53, so every intermediate sum
// is exactly representable: the fp64 additions are exact, hence associative, and the result has the same bits
// whatever order the waves arrive in (unquantised fp64 partials were order-independent only while their exponents
// spanned fewer than ~29 bits).  A NaN / inf partial enters as NaN, which any order propagates: the non-finite
// result an fp32 sum would have given.  A FINITE partial with |v| >= 2^16 (a diverging client) saturates to
// +-(2^50 - 2^26) quanta (~ +-65536): the sum stays finite and order-independent, and that client keeps training
// like the fp32 reference would (with its column sum clipped to |partial| < 2^16 per wave).  Resolution 2^-34
// (~5.8e-11) absolute.
// Cost: rint + scale + convert + one select in front of the same ds_add_f64, straight-line (an int64 form with
// the conversion done in fp32 / int32 pieces lengthened each call's dependent chain by ~150 cycles: +0.4 us per
// TransformerModel step, measured; a poison flag through a uniform-address LDS atomic became a 64-iteration
// scalar loop).
constexpr float FX_SCALE = 17179869184.0f;  // 2^34
constexpr float FX_SAT = 1125899839733760.0f;  // 2^50 - 2^26: the largest fp32 below 2^50 quanta (8 of them < 2^53)
__device__ __forceinline__ void lds_addq(uchar* base, int idx, float v) {
#ifdef ONCHIP_FP64_COLSUM  // A/B variant (tools/ab_native.sh): the round-4 unquantised fp64 atomics
  __hip_atomic_fetch_add((LDS_AS double*)base + idx, (double)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  return;
#endif
  const float av = fabsf(v);
  float x = av < 65536.f ? __builtin_rintf(v * FX_SCALE)
          : av <= 3.402823466e38f ? __builtin_copysignf(FX_SAT, v) : __builtin_nanf("");
  asm volatile("" : "+v"(x));  // (select in fp32, then convert: one VGPR pair live, not a 64-bit NaN constant)
  __hip_atomic_fetch_add((LDS_AS double*)base + idx, (double)x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// the accumulated value of slot idx (read after the barrier that follows every add)
__device__ __forceinline__ float lds_getq(const uchar* base, int idx) {
#ifdef ONCHIP_FP64_COLSUM
  return (float)((const LDS_AS double*)base)[idx];
#endif
  return (float)(((const LDS_AS double*)base)[idx] * (1.0 / 17179869184.0));
}
// partner lane's value (bound_ctrl: 0 for a missing source, which none of these patterns has) in the
// form the backend's DPP combine folds into the consuming add
template <int BIT>
__device__ __forceinline__ float dppz(float a) {
  constexpr int C = BIT == 2 ? 0x141 : BIT == 0 ? 0xB1 : BIT == 1 ? 0x4E : 0x128;
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(a), C, 0xF, 0xF, true));
}
// one reduce-scatter level (fused_common.h rs_level, select-light form): both halves are summed with
// the partner's copy (the DPP move folds into the add) and ONE select keeps this lane's half
template <int N, int L>
__device__ __forceinline__ void rs_level2(float* v, int i, int& j) {
  constexpr int BIT = L == 0 ? 2 : L == 1 ? 0 : L == 2 ? 1 : 3;
  constexpr int H = N / 2;
  const bool b = (i >> BIT) & 1;
#pragma unroll
  for (int k = 0; k < H; ++k) {
    const float lo = v[k] + dppz<BIT>(v[k]), hi = v[k + H] + dppz<BIT>(v[k + H]);
    v[k] = b ? hi : lo;
  }
  j += b ? H : 0;
}
template <int W>
__device__ __forceinline__ int rs_slot(float (&s)[W], int i) {
  int j = 0;
  rs_level2<W, 0>(s, i, j);
  rs_level2<W / 2, 1>(s, i, j);
  if constexpr (W >= 8) rs_level2<W / 4, 2>(s, i, j);
  if constexpr (W >= 16) rs_level2<W / 8, 3>(s, i, j);
  if constexpr (W == 4) s[0] += fk::dpp_pair<1>(s[0]);
  if constexpr (W <= 8) s[0] += fk::dpp_pair<3>(s[0]);
  return j;
}
// 16 values (64 features, T layout) -> (feature of this lane, its column sum)
__device__ __forceinline__ int colsum64(const float (&x)[16], int lane, float& sum) {
  float s[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) s[j] = x[j];
  const int j = rs_slot<16>(s, lane & 15);
  sum = s[0];
  return 16 * (j >> 2) + 4 * (lane >> 4) + (j & 3);
}
// 8 values (32 features: tiles 0, 1); only lanes with (lane & 8) == 0 hold a sum (returns -1 otherwise)
__device__ __forceinline__ int colsum32(const float (&x)[8], int lane, float& sum) {
  float s[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] = x[j];
  const int i = lane & 15;
  const int j = rs_slot<8>(s, i);
  sum = s[0];
  return (i & 8) == 0 ? 16 * (j >> 2) + 4 * (lane >> 4) + (j & 3) : -1;
}

// ln p and ln(1 - p) of a sigmoid output for the BCE loss VALUE (reported per epoch, and its NaN test rides on the
// head's hand-off); the gradient does not use them.  v_log_f32 (log2) instead of the correctly rounded logf / log1pf
// expansions (dozens of instructions each on the head's critical path, and a spilled constant pair): ~1e-7
// absolute error per row; ln(1 - p) loses relative precision only where p < 2^-24, i.e. a term below 6e-8
__device__ __forceinline__ void bce_logs(float p, float& lg, float& lg1) {
  constexpr float LN2 = 0.69314718055994531f;
  lg = __builtin_amdgcn_logf(p) * LN2;
  lg1 = __builtin_amdgcn_logf(1.f - p) * LN2;
}

__device__ __forceinline__ bool mbit(uint32_t m, int j) { return (m >> j) & 1u; }
// x if bit j of m is set, else +0.0 (== bit ? x : 0.f bit for bit, NaN included): the bit becomes an
// all-ones / zero word with ONE signed bitfield extract and masks x with one AND — two VALU instructions
// instead of the test, compare and select
// (the extracted mask goes through an empty asm: otherwise the backend turns the pair back into a bit test, a
// compare and a v_cndmask — three instructions per element, measured in the tf2 forward's assembly)
__device__ __forceinline__ float keepf(float x, uint32_t m, int j) {
  int s = __builtin_amdgcn_sbfe((int)m, j, 1);
  asm("" : "+v"(s));
  return __uint_as_float(__float_as_uint(x) & (uint32_t)s);
}

// ------------------------------------------------------------------------ packed-FP32 row math
// The branch workgroups are VALU-issue-bound, so the LayerNorm / affine math runs two features per
// instruction (v_pk_add / v_pk_mul / v_pk_fma on float2 pairs of the 16 values a lane holds).
__device__ __forceinline__ of2v ld2(const float (&x)[16], int j) { return of2v{x[2 * j], x[2 * j + 1]}; }
__device__ __forceinline__ void st2(float (&x)[16], int j, of2v v) {
  x[2 * j] = v[0];
  x[2 * j + 1] = v[1];
}
// LayerNorm forward (biased variance, eps 1e-5) of a 64-wide row held as 16 values x 4 lanes: x -> xhat
__device__ __forceinline__ float ln_fwd2(float (&x)[16]) {
  of2v s = {0.f, 0.f};
#pragma unroll
  for (int j = 0; j < 8; ++j) s += ld2(x, j);
  const float mean = fk::rsum4(s[0] + s[1]) * (1.f / 64.f);
  of2v ss = {0.f, 0.f};
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const of2v d = ld2(x, j) - mean;
    st2(x, j, d);
    ss += d * d;
  }
  const float rstd = __builtin_amdgcn_rsqf(fk::rsum4(ss[0] + ss[1]) * (1.f / 64.f) + 1e-5f);
#pragma unroll
  for (int j = 0; j < 8; ++j) st2(x, j, ld2(x, j) * rstd);
  return rstd;
}
// LayerNorm backward: dx = rstd (g - mean(g) - xhat mean(g xhat)), g = dy gamma
__device__ __forceinline__ void ln_bwd2(float (&dx)[16], const float (&dy)[16], const float (&xh)[16], float rstd,
                                        const float (&gamma)[16]) {
  of2v a = {0.f, 0.f}, b = {0.f, 0.f}, g[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    g[j] = ld2(dy, j) * ld2(gamma, j);
    a += g[j];
    b += g[j] * ld2(xh, j);
  }
  const float am = fk::rsum4(a[0] + a[1]) * (1.f / 64.f), bm = fk::rsum4(b[0] + b[1]) * (1.f / 64.f);
#pragma unroll
  for (int j = 0; j < 8; ++j) st2(dx, j, (g[j] - am - ld2(xh, j) * bm) * rstd);
}
// y = x * gamma + beta
__device__ __forceinline__ void affine2(float (&y)[16], const float (&x)[16], const float (&gm)[16], const float (&bt)[16]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) st2(y, j, ld2(x, j) * ld2(gm, j) + ld2(bt, j));
}

// ------------------------------------------------------------------------------------------- Adam
// fp32 master weights live in ACCUMULATION registers (AGPRs) for the whole round: every access goes
// through v_accvgpr_read / v_accvgpr_write, so the register allocator gives them the AGPR class and the
// forward / backward working set keeps the architectural VGPRs (the two files share one 256-entry budget
// per lane at two waves per SIMD).  Their Adam moments m, v do NOT fit beside them: with p, m and v all in
// AGPRs the allocator spilled ~50 dwords of state to scratch, reloaded one dependent load at a time (~8 us
// of a 29 us step).  The moments therefore live in the workspace slab (WS_MOM) and every update phase
// issues all of its moment loads as one batch before the work that precedes the Adam arithmetic.
struct TS {  // one 16x16 weight-gradient tile's 4 elements of this lane
  float p[4];
};
struct VS {
  float p;
};
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(base, 0, 0x7fffffff, 0x00020000);
}
// moment slot s of this thread (sc1 loads: L2-served, never a stale L1 line of the previous step)
// A 16-byte vector-memory store reads its data VGPRs after issue: a VALU write to them in the next cycle can
// land in the stored data (measured: element 0 of a moment store taking the next instruction's value in some
// lanes -> a negative second moment -> NaN), and the backend does not insert the wait state.  Every b128 store
// helper below is followed by this pinned s_nop.
__device__ __forceinline__ void store_guard() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 1" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}
__device__ __forceinline__ f4v mom_ld(__amdgpu_buffer_rsrc_t rs, int s, int tid) {
  return __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(rs, (s * NTH + tid) * 16, 0, 16));
}
__device__ __forceinline__ void mom_st(__amdgpu_buffer_rsrc_t rs, int s, int tid, f4v v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rs, (s * NTH + tid) * 16, 0, 0);
  store_guard();
}
// same slab addressing with the (wave-uniform) slot part in the scalar offset: one per-lane address for
// every slot instead of one per slot (the compiler hoists those out of the step loop and keeps them live)
// (plain loads: the slab is private to the workgroup, written and read back on the same CU and XCD, so the
// L1 / L2 copies are the workgroup's own writes — sc1 would send every load past the L2)
__device__ __forceinline__ f4v slot_ld(__amdgpu_buffer_rsrc_t rs, int s, int tid16) {
  return __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(rs, tid16, s * NTH * 16, 0));
}
__device__ __forceinline__ void slot_st(__amdgpu_buffer_rsrc_t rs, int s, int tid16, f4v v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rs, tid16, s * NTH * 16, 0);
  store_guard();
}
#ifndef ONCHIP_NO_AGPR
__device__ __forceinline__ float ar(float a) {
  float r;
  asm("v_accvgpr_read_b32 %0, %1" : "=v"(r) : "a"(a));
  return r;
}
__device__ __forceinline__ float aw(float v) {
  float r;
  asm("v_accvgpr_write_b32 %0, %1" : "=a"(r) : "v"(v));
  return r;
}
#else  // state in architectural VGPRs (the allocator then has the whole 256-register budget for one class)
__device__ __forceinline__ float ar(float a) { return a; }
__device__ __forceinline__ float aw(float v) { return v; }
#endif
// Step constants.  Adam (torch.optim.Adam defaults): keep = 1, c1 = 1 - beta1, lr_bc1 = lr / (1 - beta1^t),
// rsqrt_bc2 = 1 / sqrt(1 - beta2^t), eps = 1e-8.  SGD test mode (raw gradients for the tests): keep = 0,
// c1 = 1, lr_bc1 = lr, rsqrt_bc2 = 0, eps = 1, so the same branch-free formula gives m = g, p -= lr g.
struct AdamK {
  float lr_bc1, rsqrt_bc2, keep, c1, eps;
};

// lr_bc1 / rsqrt_bc2 of step t come from the host-computed table a.kt (torch computes them in double on
// the host as well); a scalar load per step instead of double-precision division / sqrt on every wave
__device__ __forceinline__ AdamK adam_k(const AflTfTrainArgs& a, int step) {
  if (a.opt_mode == 1) return AdamK{a.lr, 0.f, 0.f, 1.f, 1.f};
  const float* k = a.kt + 2 * (step - 1);
  return AdamK{k[0], k[1], 1.f, 1.f - fk::B1, fk::EPS};
}
// one Adam step of an AGPR-resident weight with its moments m, v (VGPRs, updated in place); v_sqrt_f32
// (1 ulp) instead of the correctly rounded sqrt expansion: 4x fewer instructions on the update's chain
__device__ __forceinline__ float adam1(float& pa, float& m, float& v, float g, const AdamK& k) {
  float p = ar(pa);
  const float mk = m * k.keep;
  m = mk + k.c1 * (g - mk);
  v = fk::B2 * v + (1.f - fk::B2) * g * g;
  p -= k.lr_bc1 * m * __builtin_amdgcn_rcpf(__builtin_amdgcn_sqrtf(v) * k.rsqrt_bc2 + k.eps);
  pa = aw(p);
  return p;
}
// weight matrix W[n][k] (row-major in the flat params at `off`, n_real x k_real) and its LDS image
struct Mat {
  int off, n_real, k_real, img, ld;
};
// element (n, k) of this lane in tile (T = k tile, T' = n tile): n = 16T' + (lane & 15), k = 16T + 4g + i
__device__ __forceinline__ void tile_load(TS& s, const Mat& M, int T, int Tn, int lane, const float* P, uchar* smem) {
  const int n = 16 * Tn + (lane & 15), k0 = 16 * T + 4 * (lane >> 4);
  float h[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const bool ok = n < M.n_real && k0 + i < M.k_real;
    h[i] = ok ? P[M.off + n * M.k_real + k0 + i] : 0.f;
    s.p[i] = aw(h[i]);
  }
  if (n < 16 * ((M.n_real + 15) / 16))
    *(LDS_AS u32x2v*)(smem + M.img + n * M.ld + pcol(k0) * 2) = u32x2v{pk2(h[0], h[1]), pk2(h[2], h[3])};
}
__device__ __forceinline__ void tile_store(const TS& s, const Mat& M, int T, int Tn, int lane, float* P) {
  const int n = 16 * Tn + (lane & 15), k0 = 16 * T + 4 * (lane >> 4);
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (n < M.n_real && k0 + i < M.k_real) P[M.off + n * M.k_real + k0 + i] = ar(s.p[i]);
}
// Adam on the tile's real elements with gradient acc (= dW^T tile) and moments m, v, new bf16 values -> image
__device__ __forceinline__ void tile_adam(TS& s, f4v& m, f4v& v, const Mat& M, int T, int Tn, int lane, f4v acc,
                                          const AdamK& K, uchar* smem) {
  const int n = 16 * Tn + (lane & 15), k0 = 16 * T + 4 * (lane >> 4);
  float h[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const bool ok = n < M.n_real && k0 + i < M.k_real;
    float mi = m[i], vi = v[i];
    h[i] = ok ? adam1(s.p[i], mi, vi, acc[i], K) : 0.f;
    m[i] = mi;
    v[i] = vi;
  }
  if (n < 16 * ((M.n_real + 15) / 16))
    *(LDS_AS u32x2v*)(smem + M.img + n * M.ld + pcol(k0) * 2) = u32x2v{pk2(h[0], h[1]), pk2(h[2], h[3])};
}
// Adam on a PAIR of tiles in explicit stages (all weights read, packed m / v updates, all square roots, all
// reciprocals, all weights written): eight independent element chains in flight, so the transcendental
// latencies overlap (element by element the sqrt -> rcp -> fma chain serialised).  Tiles whose elements are
// all real (n_real / k_real multiples of 16 covering them): no per-element masks.
__device__ __forceinline__ void tile_adam_pair(TS& s0, TS& s1, f4v& m0, f4v& v0, f4v& m1, f4v& v1, const Mat& M, int T0,
                                               int T1, int Tn, int lane, f4v g0, f4v g1, const AdamK& K,
                                               uchar* smem) {
  float p[8], mm[8], vv[8], g[8];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    p[i] = ar(s0.p[i]);
    p[4 + i] = ar(s1.p[i]);
    mm[i] = m0[i]; mm[4 + i] = m1[i];
    vv[i] = v0[i]; vv[4 + i] = v1[i];
    g[i] = g0[i]; g[4 + i] = g1[i];
  }
  float den[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const float mk = mm[i] * K.keep;
    mm[i] = mk + K.c1 * (g[i] - mk);
    vv[i] = fk::B2 * vv[i] + (1.f - fk::B2) * g[i] * g[i];
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) den[i] = __builtin_amdgcn_sqrtf(vv[i]);
#pragma unroll
  for (int i = 0; i < 8; ++i) den[i] = __builtin_amdgcn_rcpf(den[i] * K.rsqrt_bc2 + K.eps);
#pragma unroll
  for (int i = 0; i < 8; ++i) p[i] -= K.lr_bc1 * mm[i] * den[i];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    s0.p[i] = aw(p[i]);
    s1.p[i] = aw(p[4 + i]);
    m0[i] = mm[i]; m1[i] = mm[4 + i];
    v0[i] = vv[i]; v1[i] = vv[4 + i];
  }
  const int n = 16 * Tn + (lane & 15), g4 = 4 * (lane >> 4);
  *(LDS_AS u32x2v*)(smem + M.img + n * M.ld + pcol(16 * T0 + g4) * 2) = u32x2v{pk2(p[0], p[1]), pk2(p[2], p[3])};
  *(LDS_AS u32x2v*)(smem + M.img + n * M.ld + pcol(16 * T1 + g4) * 2) = u32x2v{pk2(p[4], p[5]), pk2(p[6], p[7])};
}

// Adam on N independent entries in the same stages as tile_adam_pair (AGPR weights pa[], moments in place,
// gradients g[]); returns the new weights in pn[]
template <int N>
__device__ __forceinline__ void adam_staged(VS (&pa)[N], float (&m)[N], float (&v)[N], const float (&g)[N],
                                            float (&pn)[N], const AdamK& K) {
  float den[N];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    pn[i] = ar(pa[i].p);
    const float mk = m[i] * K.keep;
    m[i] = mk + K.c1 * (g[i] - mk);
    v[i] = fk::B2 * v[i] + (1.f - fk::B2) * g[i] * g[i];
  }
#pragma unroll
  for (int i = 0; i < N; ++i) den[i] = __builtin_amdgcn_sqrtf(v[i]);
#pragma unroll
  for (int i = 0; i < N; ++i) den[i] = __builtin_amdgcn_rcpf(den[i] * K.rsqrt_bc2 + K.eps);
#pragma unroll
  for (int i = 0; i < N; ++i) {
    pn[i] -= K.lr_bc1 * m[i] * den[i];
    pa[i].p = aw(pn[i]);
  }
}

// -------------------------------------------------------------------------- cross-workgroup hand-off
__device__ __forceinline__ void st_wt(__amdgpu_buffer_rsrc_t rs, int off, u32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, 16);  // sc1: write-through
  store_guard();
}
__device__ __forceinline__ u32x4 ld_wt(__amdgpu_buffer_rsrc_t rs, int off) {
  return __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 16);
}
__device__ __forceinline__ void publish(gu32* flag, uint32_t value, int lane) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (lane == 0) __hip_atomic_store(flag, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// waits until (*fa >> shift) >= want and (*fb >> shift) >= want; returns *fa, or 0xFFFFFFFF on timeout
__device__ __forceinline__ uint32_t await(gu32* fa, gu32* fb, uint32_t want, int shift, gu32* tmo, int lane) {
  uint32_t v = 0;
  for (long spins = 0;; ++spins) {
    v = __builtin_amdgcn_readfirstlane(__hip_atomic_load(fa, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    const uint32_t w =
        fb == fa ? v : __builtin_amdgcn_readfirstlane(__hip_atomic_load(fb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    if ((v >> shift) >= want && (w >> shift) >= want) break;
    if (spins > fk::XWG_MAX_SPINS) {
      v = 0xFFFFFFFFu;
      if (lane == 0) __hip_atomic_store(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // payload loads stay below the poll
  return v;
}
constexpr int XF_VIT = 0, XF_LAB = 1, XF_BVIT = 2, XF_BLAB = 3, XF_TMO = 4 * 8 * 32;

// ---- granule hand-off (cdna_hip_programming.md Guideline 16 R2: the data IS the flag) ----
// A wave hands its 64 lanes x 8 payload words over as {value, tag} granules: 4 write-through (sc1) 16-byte
// stores per lane, each carrying two granules (each 8-byte half lands untorn).  No drain, no flag store: the
// producer wave moves on at once, and the consumer's ONE sc1 sweep both detects and fetches the data (the
// flag form costs a drain on the producer plus a second dependent round trip on the consumer:
// MI355X_MICROARCH price list, handoff-1to1 vs handoff-flag).  Tags count steps within the launch (never 0),
// and the slots live in the per-call zeroed sync block, so a previous launch's granules never match.
// Slot (dir, src, wave): 4 KB = [k 0..3][lane] x 16 B — one store instruction writes 1 KB contiguously.
constexpr int GR_DIR_BYTES = 2 * 8 * 4096;
__device__ __forceinline__ int gr_off(int dir, int src, int wave, int lane) {
  return dir * GR_DIR_BYTES + (src * 8 + wave) * 4096 + lane * 16;
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t gr_rsrc(gu32* sync) { return rsrc((void*)(sync + AFL_TF_SYNC_WORDS)); }
#ifdef ONCHIP_R1_HANDOFF
// A/B variant (tools/ab_native.sh): the flag form (R1) on the same slots — 32 B of write-through payload per
// lane at the slot's start, the storing wave drains, lane 0 stores the tag into the slot's flag line
// (+2048); the consumer polls the flag(s), then issues its payload loads.
__device__ __forceinline__ void gr_put(__amdgpu_buffer_rsrc_t rg, int off, const u32x4 (&u)[2], uint32_t tag) {
  const int lane = threadIdx.x & 63, base = off - lane * 16;
  __builtin_amdgcn_raw_buffer_store_b128(u[0], rg, base + lane * 32, 0, 16);
  store_guard();
  __builtin_amdgcn_raw_buffer_store_b128(u[1], rg, base + lane * 32 + 16, 0, 16);
  store_guard();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (lane == 0) __builtin_amdgcn_raw_buffer_store_b32(tag, rg, base + 2048, 0, 16);
}
template <int S>
__device__ __forceinline__ uint32_t gr_get(__amdgpu_buffer_rsrc_t rg, const int (&off)[S], u32x4 (&out)[2 * S],
                                           uint32_t want, int shift, gu32* tmo, int lane) {
  uint32_t v = 0;
  for (long spins = 0;; ++spins) {
    bool ok = true;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const uint32_t f = __builtin_amdgcn_readfirstlane(
          __builtin_amdgcn_raw_buffer_load_b32(rg, off[s] - lane * 16 + 2048, 0, 16));
      if (s == 0) v = f;
      ok = ok && (f >> shift) == want;
    }
    if (ok) break;
    if (spins > fk::XWG_MAX_SPINS) {
      if (lane == 0) __hip_atomic_store(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return 0xFFFFFFFFu;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // payload loads stay below the poll
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const int base = off[s] - lane * 16;
    out[2 * s] = __builtin_amdgcn_raw_buffer_load_b128(rg, base + lane * 32, 0, 16);
    out[2 * s + 1] = __builtin_amdgcn_raw_buffer_load_b128(rg, base + lane * 32 + 16, 0, 16);
  }
  return v;
}
#else
__device__ __forceinline__ void gr_put(__amdgpu_buffer_rsrc_t rg, int off, const u32x4 (&u)[2], uint32_t tag) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int j = 2 * (k & 1);
    __builtin_amdgcn_raw_buffer_store_b128(u32x4{u[k >> 1][j], tag, u[k >> 1][j + 1], tag}, rg, off + k * 1024, 0, 16);
    store_guard();
  }
}
// sweeps the S slots at off[] until every granule's (tag >> shift) == want; returns the payload in out[2S]
// and the tag (wave-uniform), or 0xFFFFFFFF on timeout (also raises *tmo)
template <int S>
__device__ __forceinline__ uint32_t gr_get(__amdgpu_buffer_rsrc_t rg, const int (&off)[S], u32x4 (&out)[2 * S],
                                           uint32_t want, int shift, gu32* tmo, int lane) {
  for (long spins = 0;; ++spins) {
    u32x4 v[4 * S];
#pragma unroll
    for (int s = 0; s < S; ++s)
#pragma unroll
      for (int k = 0; k < 4; ++k) v[4 * s + k] = __builtin_amdgcn_raw_buffer_load_b128(rg, off[s] + k * 1024, 0, 16);
    bool ok = true;
#pragma unroll
    for (int i = 0; i < 4 * S; ++i) ok = ok && (v[i][1] >> shift) == want && (v[i][3] >> shift) == want;
    if (__builtin_amdgcn_ballot_w64(!ok) == 0) {
#pragma unroll
      for (int s = 0; s < S; ++s) {
        out[2 * s] = u32x4{v[4 * s][0], v[4 * s][2], v[4 * s + 1][0], v[4 * s + 1][2]};
        out[2 * s + 1] = u32x4{v[4 * s + 2][0], v[4 * s + 2][2], v[4 * s + 3][0], v[4 * s + 3][2]};
      }
      return __builtin_amdgcn_readfirstlane(v[0][1]);
    }
    if (spins > fk::XWG_MAX_SPINS) {
      if (lane == 0) __hip_atomic_store(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return 0xFFFFFFFFu;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}
#endif
__device__ __forceinline__ gu32* xf(gu32* base, int group, int wave) { return base + (group * 8 + wave) * 32; }

__device__ __forceinline__ void unpack16(const u32x4 (&u)[2], float (&x)[16]) {
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      x[8 * h + 2 * k] = __uint_as_float(u[h][k] << 16);
      x[8 * h + 2 * k + 1] = __uint_as_float(u[h][k] & 0xFFFF0000u);
    }
}
__device__ __forceinline__ void pack16(const float (&x)[16], u32x4 (&u)[2]) {
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int k = 0; k < 4; ++k) u[h][k] = pk2(x[8 * h + 2 * k], x[8 * h + 2 * k + 1]);
}

// Phase entry: make the lane / wave indices opaque so every LDS address of the phase is recomputed
// inside it.  Otherwise the compiler hoists the hundreds of per-lane swizzled addresses of the step out
// of the loop and keeps them live across all phases (spilling the optimizer state to scratch).
__device__ __forceinline__ void opq(int& lane, int& wave) {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" : "+v"(lane));
  asm volatile("" : "+s"(wave));
  lane &= 63;
  wave &= 7;
}
// sub-phase boundary inside a phase: the scheduler may not move instructions across it (keeps the next
// sub-phase's LDS loads from being hoisted into this one, which raises register pressure)
__device__ __forceinline__ void sb() { __builtin_amdgcn_sched_barrier(0); }

// barrier over LDS only (global loads stay in flight, stores are not drained)
__device__ __forceinline__ void lds_bar() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Intra-workgroup progress counters (monotone LDS words): a wave signals once its LDS stores AND reads before the
// signal have completed (so a waiter may overwrite what the signaller read); a waiter spins until the count
// reaches its target, then issues its LDS accesses (ordered after the count's read).  Lets the waves that are
// ahead start work that depends on every wave's progress without a full barrier.
__device__ __forceinline__ void lds_signal(uchar* smem, int off, int lane) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (lane == 0) __hip_atomic_fetch_add((LDS_AS uint32_t*)(smem + off), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// (bounded like the cross-workgroup hand-offs: false after XWG_MAX_SPINS, which the caller treats as a failed client
// — only a wave that never signals, i.e. a bug or a dead hand-off partner, gets there)
__device__ __forceinline__ bool lds_wait(const uchar* smem, int off, uint32_t target) {
  for (long spins = 0;; ++spins) {
    const uint32_t v = __builtin_amdgcn_readfirstlane(*(volatile const LDS_AS uint32_t*)(smem + off));
    if (v >= target) break;
    if (spins > fk::XWG_MAX_SPINS) return false;
    __builtin_amdgcn_s_sleep(1);
  }
  asm volatile("" ::: "memory");
  return true;
}

// --------------------------------------------------------------------------- batch walk (shared plan)
struct Walk {
  int e, b0;  // current epoch, batch start
};
// next non-skipped batch at or after (e, b0) (size-1 batches are skipped, client.py:86-87); false = done
__device__ __forceinline__ bool walk_valid(Walk& w, int nd, int BS, int E) {
  for (;;) {
    if (w.b0 >= nd) {
      ++w.e;
      w.b0 = 0;
      if (w.e >= E) return false;
      continue;
    }
    if (min(BS, nd - w.b0) == 1) {
      w.b0 += BS;
      continue;
    }
    return true;
  }
}

__device__ __forceinline__ uint32_t aru(float a) { return __float_as_uint(ar(a)); }
__device__ __forceinline__ float awu(uint32_t v) { return aw(__uint_as_float(v)); }

// bias gradient = column sums of a dY tile: the dW GEMM with an all-ones X fragment (every row of the
// 16x16 result equals the sums of the 16 columns of dY tile Tn)
// (as a plain constant the compiler hoists the quad out of a step loop as one invariant value, and under register
// pressure spills it and reloads it before every use: a loop that uses it materialises it per phase, opaque)
__device__ __forceinline__ s8v ones8() {
  const short o = (short)0x3F80;  // bf16 1.0
  return s8v{o, o, o, o, o, o, o, o};
}

}  // namespace oc
