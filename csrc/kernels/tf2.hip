// Fused TransformerModel/ICU local training, on-chip edition (reference training loop client.py:75-111,
// model src/Model.py:166-246).  ONE persistent launch trains every client of a rank for all its local
// epochs; each client runs on three co-resident 512-thread workgroups (head | vitals branch | labs
// branch) that hand activations and gradients to each other once per direction per step.
//
// What differs from transformer.hip: after the prologue NOTHING of a client's model lives in global
// memory.  Per workgroup:
//   * the head's fp32 master weights and the branches' compact entries (biases, LayerNorm, the small dense /
//     ffn weights) stay in REGISTERS (AGPRs) for the whole round; their Adam moments, and the branches'
//     64 x 64 v / out_proj blocks (weights AND moments), sit in a per-workgroup workspace slab that each
//     update phase loads ahead of its arithmetic (L2-resident; see br_update for why the blocks moved there);
//   * bf16 weight images (the MFMA operands) and an fp32 copy of the bias / LayerNorm vectors live in
//     LDS; Adam rewrites them in place;
//   * activations chain in registers: every GEMM is computed transposed, Y^T = W . X^T, so the
//     16x16x32 MFMA leaves lane (b, g) of wave w holding features 16t + 4g + i of batch row 16w + b
//     ("T layout") — exactly the B operand of the next GEMM once the weight image's K axis is stored in
//     the matching permuted order (pcol below).  The forward and the d(input) backward of a wave never
//     leave its registers and need no barrier; LayerNorm row sums are in-lane + two permlane swaps;
//   * the activations the weight gradients need (X and dY of every dW = dY^T X) are written to
//     XOR-swizzled LDS tiles as they are produced and read back with ds_read_b64_tr_b16; each wave starts
//     the weight-gradient work its inputs allow as soon as its own backward is done, tracked by LDS progress
//     counters instead of a barrier (br_update), so the waves that finish the backward first work while the
//     rest are still in theirs;
//   * the only global traffic in the step loop is the next batch's input rows (prefetched during the
//     hand-off wait) and the hand-offs themselves: per wave 2 KB of bf16 rows as {value, step tag}
//     granules in 16-byte write-through (sc1) stores, swept with sc1 loads until every tag matches — the
//     data is the flag (cdna_hip_programming.md Guideline 16 R2): no drain on the producer, one round trip
//     on the consumer.
// Numerics are those of transformer.hip: bf16 MFMA operands with fp32 accumulation, fp32 elementwise
// math, exact-erf GELU, hash dropout masks (tf_common.h), torch.optim.Adam with a fresh state per round.
#include "common.h"
#include "kernels.h"
#include "tf_common.h"
#include "fused_common.h"
#include "onchip.h"

using namespace tf;

namespace t2 {

using namespace oc;



// ----------------------------------------------------------------------------------- LDS maps (bytes)
// branch workgroup
// dense image compact (k unpermuted: the K <= 16 MFMA reads k = 4g .. 4g + 3 at byte 8g), which pays for 32-byte
// padding of the v / out_proj images (ds_read_b128 fragment reads conflict-free in gfx950 banking)
constexpr int LDDN = 24 * 2, LDVO = LD64 + 16;
constexpr int B_IMG_D = 0;                         // [64][32]  dense (K = din padded to 32)
constexpr int B_IMG_V = B_IMG_D + 64 * LDDN;       // [64][64]  in_proj rows 128..191 (v)
constexpr int B_IMG_O = B_IMG_V + 64 * LDVO;       // [64][64]  out_proj
constexpr int B_IMG_F1 = B_IMG_O + 64 * LDVO;      // [16][64]  ffn.0 (6 real rows)
constexpr int B_IMG_F2 = B_IMG_F1 + 16 * LD64;     // [64][32]  ffn.3 (6 real columns)
constexpr int B_H0 = B_IMG_F2 + 64 * LD32;         // tile64: h0 = gelu(dense)          (X of dWv)
constexpr int B_A = B_H0 + 16384;                  // tile64: a = att_dropout(v)         (X of dWo)
constexpr int B_X1N = B_A + 16384;                 // tile64: LN1 output                 (X of dWf1)
constexpr int B_DF3 = B_X1N + 16384;               // tile64: d(ffn.3 out)               (dY of dWf2)
constexpr int B_DO = B_DF3 + 16384;                // tile64: d(out_proj out)            (dY of dWo)
constexpr int B_DV = B_DO + 16384;                 // tile64: d(v)                       (dY of dWv)
constexpr int B_DZ0 = B_DV + 16384;                // tile64: d(dense pre-activation)    (dY of dWd)
constexpr int B_XIN = B_DZ0 + 16384;               // tile16: branch input               (X of dWd)
constexpr int B_F2 = B_XIN + 4096;                 // tile16: drop(gelu(ffn.0 out))      (X of dWf2)
constexpr int B_DF0 = B_F2 + 4096;                 // tile16: d(ffn.0 pre-activation)    (dY of dWf1)
constexpr int B_NVEC = 648;                        // 10 x 64 vectors + ffn.0 bias (8 slots, 6 real)
constexpr int B_VEC = B_DF0 + 4096;                // fp32 [648] bias / LayerNorm parameters
constexpr int B_CS = B_VEC + B_NVEC * 4;           // fp32 [648] their gradients (column sums)
// The LayerNorm gradient column sums (6 x 64, produced wave-locally during the backward) are summed over
// the 8 waves as integer quanta in fp64 LDS atomics (onchip.h lds_addq: exact) into DBL, which ALIASES CS
// (+ 480 bytes): the remaining CS entries are written only after the backward, and the sums are moved to
// their CS slots at the start of the update.  Integer addition makes the 8-way sum independent of the order
// the waves arrive in by construction, so a client's trajectory is bit-reproducible whatever launch or rank
// trains it (fp32 LDS atomics were not: ~1e-4 drift per round; fp64 ones only while the partials spanned
// < 2^29).
constexpr int B_NLN = 6 * 64;
constexpr int B_DBL = B_CS;                        // fp64 [384]: G1 B1 G2 B2 G3 B3
constexpr int B_DBL_BYTES = B_NLN * 8;
static_assert(B_DBL_BYTES >= B_NVEC * 4, "DBL covers CS");
constexpr int B_MISC = B_DBL + B_DBL_BYTES;        // u32 [8] per-wave abort words, then the progress counters
constexpr int B_CNT_A = B_MISC + 32;               // u32: waves past their out_proj backward (DO / DV stored, Wo read)
constexpr int B_CNT_B = B_MISC + 36;               // u32: waves past their whole backward (DZ0 stored, Wv read)
constexpr int B_CNT_C = B_MISC + 40;               // u32: waves past their ffn backward (DF3 / DF0 stored)
constexpr int B_TOTAL = B_MISC + 64;
// vector segments (x64 floats) of VEC / CS
enum { VS_DB = 0, VS_VB, VS_OB, VS_G1, VS_B1, VS_F2B, VS_G2, VS_B2, VS_G3, VS_B3 };
constexpr int VS_F1B = 640;  // ffn.0 bias (6 real)

// head workgroup
#ifndef TF2_HLD1
#define TF2_HLD1 (LD128 + 16)
#endif
#ifndef TF2_HLD2
#define TF2_HLD2 (LD64 + 16)
#endif
// head image row strides (bytes): rows padded by 16 elements (32 B), so the fragment reads are conflict-free in
// gfx950 banking (wfrag ds_read_b128 4 -> 0 extra cycles, wtfrag 4 / 6 -> 2; tools/dbg/lds_banks.py,
// profiles/ab_r5_img_pad.log); the head's LDS map has the room
constexpr int HLD1 = TF2_HLD1, HLD2 = TF2_HLD2;
constexpr int H_IMG_W1 = 0;                        // [64][128] fc1
constexpr int H_IMG_W2 = H_IMG_W1 + 64 * HLD1;     // [32][64]  fc2
constexpr int H_CAT = H_IMG_W2 + 32 * HLD2;        // tile128: cat(vitals, labs)     (X of dWf1)
constexpr int H_A1 = H_CAT + 32768;                // tile64:  drop(gelu(fc1))       (X of dWf2)
constexpr int H_DZ1 = H_A1 + 16384;                // tile64:  d(fc1 pre-activation) (dY of dWf1)
constexpr int H_DZ2 = H_DZ1 + 16384;               // tile32:  d(fc2 pre-activation) (dY of dWf2)
constexpr int H_NVEC = 132;                        // fc1.b 64 | fc2.b 32 | output.w 32 | output.b 1
constexpr int H_VEC = H_DZ2 + 8192;
constexpr int H_PART = H_VEC + H_NVEC * 4;         // fp32 [8 waves][132] per-wave column sums (their gradients)
constexpr int H_LOSS = H_PART + 8 * H_NVEC * 4;    // fp32 [8] per-wave loss partials, then u32 [8] their abort flags
constexpr int H_TOTAL = H_LOSS + 64;
enum { HV_B1 = 0, HV_B2 = 64, HV_WO = 96, HV_BO = 128 };

constexpr int SMEM_CORE = B_TOTAL > H_TOTAL ? B_TOTAL : H_TOTAL;
#ifdef TF2_STAMPS
constexpr int ST_OFF = SMEM_CORE, ST_N = 16;       // u64 [16] per-phase timers of the stamped workgroup
constexpr int SMEM = ST_OFF + ST_N * 8;
#else
constexpr int SMEM = SMEM_CORE;
#endif
static_assert(SMEM <= 160 * 1024, "LDS budget");

// ------------------------------------------------------------------- per-client workspace (bytes)
// (the hand-off payloads travel as tagged granules in the per-call zeroed sync block: onchip.h gr_put / gr_get)
// Head: Adam moments of its register-resident weights, slab [slot][thread] of float4 (MOM_SLOTS slots: m and v
// of the 4 fc1 tiles, then the remaining moments), loaded in one batch of sc1 loads ahead of the update phase and
// stored back after it.
// Branch: the compact entries' moments (CMP_SLOTS slots [slot][thread]), then the v / out_proj block UNITS: unit
// 2 w + u (u = 0 out_proj, 1 in_proj.v) is the 2 x 2 tile block (Ta, Tb) of wave w's index w4 = w & 3, stored as
// [unit][12][lane] float4 = m of its 4 tiles, v, then the fp32 master weights p — in memory, not registers, so
// whichever wave is free may update a block (see br_update).
constexpr int MOM_SLOTS = 11;
constexpr long WS_MOM = 0;
constexpr long MOM_WG_BYTES = (long)MOM_SLOTS * NTH * 16;
constexpr int CMP_SLOTS = 1;
constexpr long BR_UNITS = (long)CMP_SLOTS * NTH * 16;
// then the leaders' SMALL units: leader w4's dense / ffn.3 / ffn.0 weight tiles (4 elements per lane each), [w4][9]
// [lane] float4 = m of the three tiles, v, then p
constexpr long BR_SMALL = BR_UNITS + 8L * 12 * 64 * 16;
constexpr long BR_WG_BYTES = BR_SMALL + 4L * 9 * 64 * 16;
constexpr long WS_BYTES = WS_MOM + MOM_WG_BYTES + 2 * BR_WG_BYTES;  // head, vitals branch, labs branch

// branch LayerNorm column sums -> fp64 accumulator k of DBL (order G1 B1 G2 B2 G3 B3)
__device__ __forceinline__ void ln_colsum(uchar* smem, int k, const float (&x)[16], int lane) {
  float s;
  const int f = colsum64(x, lane, s);
  lds_addq(smem + B_DBL, 64 * k + f, s);
}
__host__ __device__ constexpr int ln_seg(int k) { return k < 2 ? VS_G1 + k : VS_G2 + (k - 2); }
static_assert(ln_seg(0) == VS_G1 && ln_seg(1) == VS_B1 && ln_seg(2) == VS_G2 && ln_seg(3) == VS_B2 &&
              ln_seg(4) == VS_G3 && ln_seg(5) == VS_B3, "DBL order");

// dropout keep bits of features 16t + 4g + i (bit 4t + i), hash pairs as tf::keep
__device__ __forceinline__ uint32_t mask16(uint32_t key, uint32_t layer, int r, int g, uint32_t thr) {
  uint32_t m = 0;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint32_t x = hash3(key, layer, (uint32_t)r, (uint32_t)(8 * t + 2 * g + h));
      m |= ((x & 0xFFFFu) >= thr ? 1u : 0u) << (4 * t + 2 * h);
      m |= ((x >> 16) >= thr ? 1u : 0u) << (4 * t + 2 * h + 1);
    }
  }
  return m;
}


// ------------------------------------------------------------------------ per-phase timers (diagnostics)
// Built only into the TF2_STAMPS instantiation (tf2_stamps.hip): s_memrealtime (100 MHz) deltas of
// lane 0 of ONE wave (stamps[62], default 0) of ONE workgroup (stamps[63]), summed over all steps in LDS,
// written out at the end.
// The production kernel gets the empty Stamp below (no code, no registers).
#ifdef TF2_STAMPS
// (the previous time stamp lives in LDS slot ST_N - 1 too: a register copy raised the kernel's register
// pressure enough to change its spills, i.e. the timings being measured)
struct Stamp {
  bool on = false;
  int who = 0;  // the stamping thread: lane 0 of wave stamps[62]
  uchar* smem = nullptr;
  __device__ __forceinline__ void operator()(int id, int tid) {
    if (!on) return;
    const uint64_t now = __builtin_amdgcn_s_memrealtime();
    if (tid == who) {
      LDS_AS uint64_t* t = (LDS_AS uint64_t*)(smem + ST_OFF);
      t[id] += now - t[ST_N - 1];
      t[ST_N - 1] = now;
    }
  }
};
#else
struct Stamp {
  __device__ __forceinline__ void operator()(int, int) {}
};
#endif

// Ablation switches of the diagnostic build (compile-time TF2_ABL bits, set through the AFL_TF2_ABL
// environment variable when building tf2_stamps.hip): skip one piece of work per step to price it
// (numerics are wrong then; timing only).  Always false in the production kernel.
enum { ABL_U3 = 1, ABL_UADAM = 2, ABL_UDW = 4, ABL_COLSUM = 8, ABL_HEADUPD = 16, ABL_U1 = 32 };
#if defined(TF2_STAMPS) && defined(TF2_ABL)
#define ABL(K, b) ((TF2_ABL & (b)) != 0)
#else
#define ABL(K, b) false
#endif



// Wave priorities: the two waves sharing a SIMD (w and w + 4) run the same critical chain, and the
// arbiter favours the older one, so waves 4-7 finished the forward 1.35 us after waves 0-3 (per-wave
// stamps) while waves 0-3 already hashed the NEXT step's dropout masks beside them.  Critical sections
// (forward, backward, update; the head's forward / backward) run at priority 2, the work that only has
// to be done before the next hand-off arrives (masks, prefetch, deferred head tiles) at 0.
#ifndef TF2_NO_PRIO
__device__ __forceinline__ void prio_hi() { __builtin_amdgcn_s_setprio(2); }
__device__ __forceinline__ void prio_lo() { __builtin_amdgcn_s_setprio(0); }
#else
__device__ __forceinline__ void prio_hi() {}
__device__ __forceinline__ void prio_lo() {}
#endif

// =============================================================================== branch workgroup
template <int BR>
struct BrK {
  static constexpr BrOff o = BR == 0 ? OV : OL;
  static constexpr int din = BR == 0 ? D_V : D_L;
  static constexpr int xoff = BR == 0 ? 0 : D_V;
  // (the dense, ffn.0 and ffn.3 weights are the leaders' small units: smu_elem gives their image positions)
  static constexpr Mat MV{o.inproj_w + 128 * 64, 64, 64, B_IMG_V, LDVO};
  static constexpr Mat MO{o.out_w, 64, 64, B_IMG_O, LDVO};
  // the v (lo) or out_proj block matrix, built from constants (a `lo ? MV : MO` lvalue select would
  // odr-use the static members and load them from memory, defeating the constant folding of n_real / k_real)
  static __device__ __forceinline__ Mat vo(bool lo) {
    return Mat{lo ? MV.off : MO.off, 64, 64, lo ? B_IMG_V : B_IMG_O, LDVO};
  }
  // VEC segment -> flat parameter offset
  static __device__ __forceinline__ int vec_param(int e) {
    if (e >= VS_F1B) return e - VS_F1B < FF ? o.ff0_b + (e - VS_F1B) : -1;
    const int s = e >> 6, i = e & 63;  // (a runtime-indexed array would live in scratch)
    const int b = s == 0 ? o.dense_b : s == 1 ? o.inproj_b + 128 : s == 2 ? o.out_b : s == 3 ? o.ln1_w
                : s == 4 ? o.ln1_b : s == 5 ? o.ff3_b : s == 6 ? o.ln2_w : s == 7 ? o.ln2_b : s == 8 ? o.bn_w : o.bn_b;
    return b + i;
  }
};

// values the backward needs from the forward, kept in registers (T layout).  The normalised LayerNorm
// outputs and gelu' are kept as bf16 pairs (the precision the backward's GEMM operands have anyway):
// fp32 copies of all four would not fit beside the optimizer state in the 256-register budget.
struct Saved {
  uint32_t xh1[8], xh2[8], gp[8];
  float rstd1, rstd2;
  uint32_t m1, m2, matt;
  float gk[4];  // drop'(.) * gelu'(ffn.0 out) of features 4g + i
};
__device__ __forceinline__ void save16(uint32_t (&d)[8], const float (&x)[16]) {
#pragma unroll
  for (int k = 0; k < 8; ++k) d[k] = pk2(x[2 * k], x[2 * k + 1]);
}
__device__ __forceinline__ void load16(float (&x)[16], const uint32_t (&d)[8]) {
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    x[2 * k] = __uint_as_float(d[k] << 16);
    x[2 * k + 1] = __uint_as_float(d[k] & 0xFFFF0000u);
  }
}

// Optimizer state of one branch lane (AGPR-resident, see ar/aw; the v / out_proj blocks' weights and moments live
// in the workspace units, see br_update):
//  * cmp: NCMP "compact" entries, the bias / LayerNorm vectors (VEC index e < 648): entry e belongs to thread
//    e % 512, slot e / 512.  (The dense, ffn.0 and ffn.3 weights were compact entries too, staged through LDS and
//    updated by every thread after the staging barrier; since round 6 the leaders update them as tiles in their
//    slack before barrier 1 — br_update, small units — and the compact pass is 2 entries per thread, not 5.)
constexpr int NCMP = 2;
struct BrState {
  VS cmp[NCMP];
  float dst[NCMP];  // AGPR: where compact entry h's new value goes (cmp_dst), fixed for the round
};
static_assert(B_NVEC <= NCMP * NTH, "compact entries");

// Every dropout keep-bit of a branch wave's forward for one step, packed into two words:
//   mk0 = m1 (out_proj dropout, 16 bits) | m2 (ffn.3 dropout) << 16;
//   mk1 = matt (attention dropout per head, 4 bits) | kf (ffn.0 dropout of features 4g + i) << 4.
// The branch computes the NEXT step's masks while it waits for the head (the wave is idle there) and
// parks them in two AGPRs, so the ~20 hashes per lane leave the forward's critical path.
template <int BR>
__device__ __forceinline__ void br_masks(uint32_t key, int r, int g, uint32_t& mk0, uint32_t& mk1) {
  const uint32_t ha = hash3(key, 8 * BR + L_ATT, r, 0), hb = hash3(key, 8 * BR + L_ATT, r, 1);
  const uint32_t matt = ((ha & 0xFFFFu) >= THR_P01 ? 1u : 0u) | ((ha >> 16) >= THR_P01 ? 2u : 0u) |
                        ((hb & 0xFFFFu) >= THR_P01 ? 4u : 0u) | ((hb >> 16) >= THR_P01 ? 8u : 0u);
  const uint32_t m1 = mask16(key, 8 * BR + L_D1, r, g, THR_P01), m2 = mask16(key, 8 * BR + L_D2, r, g, THR_P01);
  uint32_t kf = 0u;
  if (g < 2) {
    const uint32_t hd[2] = {hash3(key, 8 * BR + L_DF, r, 2 * g), hash3(key, 8 * BR + L_DF, r, 2 * g + 1)};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t u = (hd[i >> 1] >> ((i & 1) << 4)) & 0xFFFFu;
      kf |= (4 * g + i < FF && u >= THR_P01 ? 1u : 0u) << i;
    }
  }
  mk0 = m1 | (m2 << 16);
  mk1 = matt | (kf << 4);
}

template <int BR>
__device__ __forceinline__ void br_forward(uchar* smem, const float (&xin)[4], uint32_t mk0, uint32_t mk1, Saved& sv,
                                           u32x4 (&outp)[2], int lane, int wave) {
  using B = BrK<BR>;
  opq(lane, wave);
  const int g = lane >> 4, r = 16 * wave + (lane & 15);
  const uchar* vg = lane_vec(smem + B_VEC, g);  // (one lane base for every vector read of the phase)
  st4<TK16>(smem + B_XIN, r, g, xin);
  // ---- dense (K = din <= 16 padded to 32) + GELU
  float h0[16];
  sb();
  {
    const s4v bx = bfrag4(xin);
    f4v acc[4];
#pragma unroll
    for (int T = 0; T < 4; ++T)
      acc[T] = mma16(*(const LDS_AS s4v*)(smem + B_IMG_D + (16 * T + (lane & 15)) * LDDN + 8 * (lane >> 4)), bx, Z4);
    float bd[16], gp[16];
    vec16g(bd, vg + VS_DB * 256);
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int i = 0; i < 4; i += 2) {
        gf2v g2;
        const gf2v y = gelu2(gf2v{acc[t][i] + bd[4 * t + i], acc[t][i + 1] + bd[4 * t + i + 1]}, g2);
        h0[4 * t + i] = y[0];
        h0[4 * t + i + 1] = y[1];
        gp[4 * t + i] = g2[0];
        gp[4 * t + i + 1] = g2[1];
      }
    save16(sv.gp, gp);
#pragma unroll
    for (int t = 0; t < 4; ++t) st4<TK64>(smem + B_H0, r, 4 * t + g, h0 + 4 * t);
  }
  // ---- v projection, attention dropout per (row, head); at L = 1 softmax == 1, so attn = drop(v)
  float a[16];
  sb();
  {
    const s8v b0 = bfrag(h0, 0), b1 = bfrag(h0, 1);
    f4v acc[4];
#pragma unroll
    for (int T = 0; T < 4; ++T) {
      acc[T] = mma(wfrag(smem + B_IMG_V, LDVO, T, 0, lane), b0, Z4);
      acc[T] = mma(wfrag(smem + B_IMG_V, LDVO, T, 1, lane), b1, acc[T]);
    }
    sv.matt = mk1 & 0xFu;
    float bv[16];
    vec16g(bv, vg + VS_VB * 256);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const float m = keepf(INV_K01, sv.matt, t);
#pragma unroll
      for (int i = 0; i < 4; ++i) a[4 * t + i] = (acc[t][i] + bv[4 * t + i]) * m;
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) st4<TK64>(smem + B_A, r, 4 * t + g, a + 4 * t);
  }
  // ---- out projection, dropout, residual, LayerNorm 1
  float x1n[16];
  sb();
  {
    const s8v b0 = bfrag(a, 0), b1 = bfrag(a, 1);
    f4v acc[4];
#pragma unroll
    for (int T = 0; T < 4; ++T) {
      acc[T] = mma(wfrag(smem + B_IMG_O, LDVO, T, 0, lane), b0, Z4);
      acc[T] = mma(wfrag(smem + B_IMG_O, LDVO, T, 1, lane), b1, acc[T]);
    }
    sv.m1 = mk0 & 0xFFFFu;
    float bo[16];
    vec16g(bo, vg + VS_OB * 256);
    float x1[16];
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int j = 4 * t + i;
        x1[j] = h0[j] + keepf((acc[t][i] + bo[j]) * INV_K01, sv.m1, j);
      }
    sv.rstd1 = ln_fwd2(x1);
    save16(sv.xh1, x1);
    float gm[16], bt[16];
    vec16g(gm, vg + VS_G1 * 256);
    vec16g(bt, vg + VS_B1 * 256);
    affine2(x1n, x1, gm, bt);
#pragma unroll
    for (int t = 0; t < 4; ++t) st4<TK64>(smem + B_X1N, r, 4 * t + g, x1n + 4 * t);
  }
  // ---- ffn.0 (64 -> 6, one output tile) + GELU + dropout
  float f2v[4];
  sb();
  {
    f4v acc = mma(wfrag(smem + B_IMG_F1, LD64, 0, 0, lane), bfrag(x1n, 0), Z4);
    acc = mma(wfrag(smem + B_IMG_F1, LD64, 0, 1, lane), bfrag(x1n, 1), acc);
    const f4v bf = g < 2 ? *(const LDS_AS f4v*)(vg + VS_F1B * 4) : Z4;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float gp;
      const float gl = gelu_and_grad(acc[i] + bf[i], gp);
      f2v[i] = keepf(gl * INV_K01, mk1, 4 + i);
      sv.gk[i] = keepf(gp * INV_K01, mk1, 4 + i);
    }
    st4<TK16>(smem + B_F2, r, g, f2v);
  }
  // ---- ffn.3 (6 -> 64, K padded to 32), dropout, residual, LayerNorm 2, LayerNorm 3 (x_bn)
  sb();
  {
    const s4v bf = bfrag4(f2v);
    f4v acc[4];
#pragma unroll
    for (int T = 0; T < 4; ++T) acc[T] = mma16(wfrag4(smem + B_IMG_F2, LD32, T, lane), bf, Z4);
    sv.m2 = mk0 >> 16;
    float b3[16];
    vec16g(b3, vg + VS_F2B * 256);
    float x2[16];
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int j = 4 * t + i;
        x2[j] = x1n[j] + keepf((acc[t][i] + b3[j]) * INV_K01, sv.m2, j);
      }
    sv.rstd2 = ln_fwd2(x2);
    save16(sv.xh2, x2);
    float gm[16], bt[16];
    vec16g(gm, vg + VS_G2 * 256);
    vec16g(bt, vg + VS_B2 * 256);
    affine2(x2, x2, gm, bt);
    ln_fwd2(x2);
    vec16g(gm, vg + VS_G3 * 256);
    vec16g(bt, vg + VS_B3 * 256);
    affine2(x2, x2, gm, bt);
    pack16(x2, outp);
  }
}

// d(branch output) -> every activation gradient of the branch (wave-local), the dY tiles of the dW
// GEMMs and the column sums of the vector gradients
template <int BR>
__device__ __forceinline__ void br_backward(uchar* smem, const float (&dout)[16], const Saved& sv, const AdamK& K, int lane,
                                            int wave) {
  opq(lane, wave);
  const int g = lane >> 4, r = 16 * wave + (lane & 15);
  const uchar* vg = lane_vec(smem + B_VEC, g);
  float dr2[16];
  sb();
  {  // LayerNorm 3 and 2 backward (xh3 = LN(xh2 * gamma2 + beta2) recomputed: fewer saved registers)
    float gm[16], t[16], dx[16], xh[16], bt[16];
    load16(xh, sv.xh2);
    vec16g(gm, vg + VS_G2 * 256);
    vec16g(bt, vg + VS_B2 * 256);
    affine2(xh, xh, gm, bt);
    const float rstd3 = ln_fwd2(xh);
#pragma unroll
    for (int j = 0; j < 16; ++j) t[j] = dout[j] * xh[j];
    if (!ABL(K, ABL_COLSUM)) ln_colsum(smem, 4, t, lane);
    if (!ABL(K, ABL_COLSUM)) ln_colsum(smem, 5, dout, lane);
    vec16g(gm, vg + VS_G3 * 256);
    ln_bwd2(dx, dout, xh, rstd3, gm);
    load16(xh, sv.xh2);
#pragma unroll
    for (int j = 0; j < 16; ++j) t[j] = dx[j] * xh[j];
    if (!ABL(K, ABL_COLSUM)) ln_colsum(smem, 2, t, lane);
    if (!ABL(K, ABL_COLSUM)) ln_colsum(smem, 3, dx, lane);
    vec16g(gm, vg + VS_G2 * 256);
    ln_bwd2(dr2, dx, xh, sv.rstd2, gm);
  }
  float df0[4];
  sb();
  {  // d(ffn.3 out) -> ffn.3 backward (d f2) -> d(ffn.0 pre-activation)
    float d3[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) d3[j] = keepf(dr2[j] * INV_K01, sv.m2, j);
#pragma unroll
    for (int t = 0; t < 4; ++t) st4<TK64>(smem + B_DF3, r, 4 * t + g, d3 + 4 * t);
    f4v acc = mma(wtfrag<true>(smem + B_IMG_F2, LD32, 0, 0, lane), bfrag(d3, 0), Z4);
    acc = mma(wtfrag<true>(smem + B_IMG_F2, LD32, 0, 1, lane), bfrag(d3, 1), acc);
#pragma unroll
    for (int i = 0; i < 4; ++i) df0[i] = acc[i] * sv.gk[i];
    st4<TK16>(smem + B_DF0, r, g, df0);
  }
  lds_signal(smem, B_CNT_C, lane);  // DF3 / DF0 rows stored: the ffn weight tiles may be computed
  float dr1[16];
  sb();
  {  // ffn.0 backward (d x1n) + residual, LayerNorm 1 backward
    const s4v bd = bfrag4(df0);
    float dx[16];
#pragma unroll
    for (int T = 0; T < 4; ++T) {
      const f4v acc = mma16(wtfrag4(smem + B_IMG_F1, LD64, T, lane), bd, Z4);
#pragma unroll
      for (int i = 0; i < 4; ++i) dx[4 * T + i] = acc[i] + dr2[4 * T + i];
    }
    float t[16], gm[16], xh[16];
    load16(xh, sv.xh1);
#pragma unroll
    for (int j = 0; j < 16; ++j) t[j] = dx[j] * xh[j];
    if (!ABL(K, ABL_COLSUM)) ln_colsum(smem, 0, t, lane);
    if (!ABL(K, ABL_COLSUM)) ln_colsum(smem, 1, dx, lane);
    vec16g(gm, vg + VS_G1 * 256);
    ln_bwd2(dr1, dx, xh, sv.rstd1, gm);
  }
  float dv[16];
  sb();
  {  // out_proj backward: d a = d o . Wo ; d v = attention-dropout'(d a)
    float dO[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) dO[j] = keepf(dr1[j] * INV_K01, sv.m1, j);
#pragma unroll
    for (int t = 0; t < 4; ++t) st4<TK64>(smem + B_DO, r, 4 * t + g, dO + 4 * t);
    const s8v b0 = bfrag(dO, 0), b1 = bfrag(dO, 1);
#pragma unroll
    for (int T = 0; T < 4; ++T) {
      f4v acc = mma(wtfrag<true>(smem + B_IMG_O, LDVO, T, 0, lane), b0, Z4);
      acc = mma(wtfrag<true>(smem + B_IMG_O, LDVO, T, 1, lane), b1, acc);
      const float m = keepf(INV_K01, sv.matt, T);
#pragma unroll
      for (int i = 0; i < 4; ++i) dv[4 * T + i] = acc[i] * m;
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) st4<TK64>(smem + B_DV, r, 4 * t + g, dv + 4 * t);
  }
  lds_signal(smem, B_CNT_A, lane);  // DO / DV rows stored, out_proj image read: its block may be updated
  sb();
  {  // v backward: d h0 = d r1 + d v . Wv ; d z0 = d h0 * gelu'(z0)
    const s8v b0 = bfrag(dv, 0), b1 = bfrag(dv, 1);
    float dz[16], gp[16];
    load16(gp, sv.gp);
#pragma unroll
    for (int T = 0; T < 4; ++T) {
      f4v acc = mma(wtfrag<true>(smem + B_IMG_V, LDVO, T, 0, lane), b0, Z4);
      acc = mma(wtfrag<true>(smem + B_IMG_V, LDVO, T, 1, lane), b1, acc);
#pragma unroll
      for (int i = 0; i < 4; ++i) dz[4 * T + i] = (acc[i] + dr1[4 * T + i]) * gp[4 * T + i];
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) st4<TK64>(smem + B_DZ0, r, 4 * t + g, dz + 4 * t);
  }
  lds_signal(smem, B_CNT_B, lane);  // backward done: DZ0 rows stored, v image read, LayerNorm sums added
}


// compact entry e (< 648: a bias / LayerNorm vector element) of branch BR: flat parameter index (or -1)
template <int BR>
__device__ __forceinline__ int cmp_param(int e) {
  return e < B_NVEC ? BrK<BR>::vec_param(e) : -1;
}
// store descriptor of compact entry e for U3 (fp32 store into VEC); padding entries and entries past the end point
// at this lane's dummy word (DF0 tile) instead
template <int BR>
__device__ __forceinline__ uint32_t cmp_dst(int e, int lane) {
  const uint32_t dmy = B_DF0 + 768 + 4 * lane;
  return cmp_param<BR>(e) >= 0 ? (0x80000000u | (uint32_t)(B_VEC + 4 * e)) : (0x80000000u | dmy);
}

// ------------------------------------------------------------------------------ branch weight update
// Block units (workspace, see WS layout): wave index w4 = w & 3 names the 2 x 2 tile block (Ta = 2 (w4 & 1),
// Tb = 2 (w4 >> 1)) of the 64 x 64 out_proj (u = 0) or in_proj.v (u = 1) weight gradient; lane holds 4 elements
// per tile, tile t = 2a + b = (Ta + a, Tb + b): slots j = t (m), 4 + t (v), 8 + t (fp32 weight p).
__device__ __forceinline__ f4v unit_ld(__amdgpu_buffer_rsrc_t rm, int ui, int j, int lane) {
  return __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(rm, (int)BR_UNITS + ((ui * 12 + j) * 64 + lane) * 16,
                                                                        0, 16));
}
__device__ __forceinline__ void unit_st(__amdgpu_buffer_rsrc_t rm, int ui, int j, int lane, f4v v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rm, (int)BR_UNITS + ((ui * 12 + j) * 64 + lane) * 16,
                                         0, 0);
  store_guard();
}
// Adam on the 16 elements of a unit (p, m, v in U, gradients acc[a][b] of tile 2a + b), in explicit stages so the
// 16 independent sqrt -> rcp -> fma chains overlap
__device__ __forceinline__ void unit_adam(f4v (&U)[12], const f4v (&acc)[2][2], const AdamK& K) {
  float p[16], mm[16], vv[16], g[16], den[16];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      mm[4 * t + i] = U[t][i];
      vv[4 * t + i] = U[4 + t][i];
      p[4 * t + i] = U[8 + t][i];
      g[4 * t + i] = acc[t >> 1][t & 1][i];
    }
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const float mk = mm[e] * K.keep;
    mm[e] = mk + K.c1 * (g[e] - mk);
    vv[e] = fk::B2 * vv[e] + (1.f - fk::B2) * g[e] * g[e];
  }
#pragma unroll
  for (int e = 0; e < 16; ++e) den[e] = __builtin_amdgcn_sqrtf(vv[e]);
#pragma unroll
  for (int e = 0; e < 16; ++e) den[e] = __builtin_amdgcn_rcpf(den[e] * K.rsqrt_bc2 + K.eps);
#pragma unroll
  for (int e = 0; e < 16; ++e) p[e] -= K.lr_bc1 * mm[e] * den[e];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      U[t][i] = mm[4 * t + i];
      U[4 + t][i] = vv[4 * t + i];
      U[8 + t][i] = p[4 * t + i];
    }
}
// the unit's new bf16 weights into its image (rows n = 16 (Tb + b) + i16, permuted k chunk of tile Ta + a)
__device__ __forceinline__ void unit_img(uchar* smem, const Mat& M, int Ta, int Tb, int lane, const u32x2v (&w)[4]) {
  const int i16 = lane & 15, g4 = 4 * (lane >> 4);
#pragma unroll
  for (int t = 0; t < 4; ++t)
    *(LDS_AS u32x2v*)(smem + M.img + (16 * (Tb + (t & 1)) + i16) * M.ld + pcol(16 * (Ta + (t >> 1)) + g4) * 2) = w[t];
}
__device__ __forceinline__ void unit_pack(const f4v (&U)[12], u32x2v (&w)[4]) {
#pragma unroll
  for (int t = 0; t < 4; ++t) w[t] = u32x2v{pk2(U[8 + t][0], U[8 + t][1]), pk2(U[8 + t][2], U[8 + t][3])};
}
// dW^T of a unit over all 128 rows: acc[a][b] = X tile Ta + a  x  dY tile Tb + b; bias column sums of dY tiles
// Tb, Tb + 1 (the all-ones X fragment) when `bias`
__device__ __forceinline__ void unit_dw(const uchar* X, const uchar* DY, int Ta, int Tb, int lane, bool bias,
                                        f4v (&acc)[2][2], f4v (&bs)[2]) {
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = Z4;
  bs[0] = bs[1] = Z4;
  // (the all-ones operand from an opaque SGPR, materialised here: hoisted out of the step loop it is spilled)
  uint32_t o1 = 0x3F803F80u;
  asm volatile("" : "+s"(o1));
  const s8v one = __builtin_bit_cast(s8v, u32x4{o1, o1, o1, o1});
#pragma unroll  // (fully unrolled: the fragment reads of later k-steps overlap earlier MFMAs, +2.2 %)
  for (int s = 0; s < 4; ++s) {
    const s8v x0 = tfrag<TK64>(X, 32 * s, Ta, lane), x1 = tfrag<TK64>(X, 32 * s, Ta + 1, lane);
    const s8v y0 = tfrag<TK64>(DY, 32 * s, Tb, lane), y1 = tfrag<TK64>(DY, 32 * s, Tb + 1, lane);
    acc[0][0] = mma(x0, y0, acc[0][0]);
    acc[0][1] = mma(x0, y1, acc[0][1]);
    acc[1][0] = mma(x1, y0, acc[1][0]);
    acc[1][1] = mma(x1, y1, acc[1][1]);
    if (bias) {
      bs[0] = mma(one, y0, bs[0]);
      bs[1] = mma(one, y1, bs[1]);
    }
  }
}

// Small units: leader w4 owns its dense tile (k 0..15, n tile w4), ffn.3 tile (n tile w4, k 0..15) and ffn.0 k tile
// w4 (n 0..15) — the weight-gradient tiles it computes (lane element (k = 16 T + 4g + i, n = 16 Tn + i16)); tile s
// of the unit: 0 dense, 1 ffn.3, 2 ffn.0; slots s (m), 3 + s (v), 6 + s (p).  Padding elements (k >= din, ffn k >= 6,
// ffn.0 n >= 6) keep p = 0: their inputs / gradients are exactly zero, so Adam leaves them there.
__device__ __forceinline__ f4v smu_ld(__amdgpu_buffer_rsrc_t rm, int w4, int j, int lane) {
  return __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(rm, (int)BR_SMALL + ((w4 * 9 + j) * 64 + lane) * 16,
                                                                        0, 16));
}
__device__ __forceinline__ void smu_st(__amdgpu_buffer_rsrc_t rm, int w4, int j, int lane, f4v v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rm, (int)BR_SMALL + ((w4 * 9 + j) * 64 + lane) * 16,
                                         0, 0);
  store_guard();
}
// (flat parameter index, bf16 image byte offset) of element i of small tile s of leader w4's lane, or pi = -1
template <int BR>
__device__ __forceinline__ void smu_elem(int s, int w4, int lane, int i, int& pi, int& img) {
  using B = BrK<BR>;
  constexpr int din = BrK<BR>::din;
  const int g = lane >> 4, i16 = lane & 15;
  if (s == 0) {  // dense W[n][k], n = 16 w4 + i16, k = 4g + i; image compact, k unpermuted
    const int n = 16 * w4 + i16, k = 4 * g + i;
    pi = k < din ? B::o.dense_w + n * din + k : -1;
    img = B_IMG_D + n * LDDN + k * 2;
  } else if (s == 1) {  // ffn.3 W[n][k], n = 16 w4 + i16, k = 4g + i < 6
    const int n = 16 * w4 + i16, k = 4 * g + i;
    pi = k < FF ? B::o.ff3_w + n * FF + k : -1;
    img = B_IMG_F2 + n * LD32 + pcol(k) * 2;
  } else {  // ffn.0 W[n][k], n = i16 < 6, k = 16 w4 + 4g + i
    const int n = i16, k = 16 * w4 + 4 * g + i;
    pi = n < FF ? B::o.ff0_w + n * 64 + k : -1;
    img = B_IMG_F1 + n * LD64 + pcol(k) * 2;
  }
}
// Adam on the 12 elements of a small unit (S = {m0 m1 m2, v0 v1 v2, p0 p1 p2}), gradients g[3]; new bf16 images
__device__ __forceinline__ void smu_adam(f4v (&S)[9], const f4v (&gs)[3], const AdamK& K) {
  float p[12], mm[12], vv[12], g[12], den[12];
#pragma unroll
  for (int s = 0; s < 3; ++s)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      mm[4 * s + i] = S[s][i];
      vv[4 * s + i] = S[3 + s][i];
      p[4 * s + i] = S[6 + s][i];
      g[4 * s + i] = gs[s][i];
    }
#pragma unroll
  for (int e = 0; e < 12; ++e) {
    const float mk = mm[e] * K.keep;
    mm[e] = mk + K.c1 * (g[e] - mk);
    vv[e] = fk::B2 * vv[e] + (1.f - fk::B2) * g[e] * g[e];
  }
#pragma unroll
  for (int e = 0; e < 12; ++e) den[e] = __builtin_amdgcn_sqrtf(vv[e]);
#pragma unroll
  for (int e = 0; e < 12; ++e) den[e] = __builtin_amdgcn_rcpf(den[e] * K.rsqrt_bc2 + K.eps);
#pragma unroll
  for (int e = 0; e < 12; ++e) p[e] -= K.lr_bc1 * mm[e] * den[e];
#pragma unroll
  for (int s = 0; s < 3; ++s)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      S[s][i] = mm[4 * s + i];
      S[3 + s][i] = vv[4 * s + i];
      S[6 + s][i] = p[4 * s + i];
    }
}
// the small unit's new weights into the three images (4 consecutive (permuted) k per lane: one 8-byte store each)
template <int BR>
__device__ __forceinline__ void smu_img(uchar* smem, const f4v (&S)[9], int w4, int lane) {
#pragma unroll
  for (int s = 0; s < 3; ++s) {
    int pi, img;
    smu_elem<BR>(s, w4, lane, 0, pi, img);
    *(LDS_AS u32x2v*)(smem + img) = u32x2v{pk2(S[6 + s][0], S[6 + s][1]), pk2(S[6 + s][2], S[6 + s][3])};
  }
}

// Weight gradients + Adam for one step, started by each wave as soon as its own backward is done — no barrier
// between the backward and the weight-gradient work.  The waves of a SIMD pair run the same chain and the arbiter
// favours the older one, so waves 0-3 ("leaders") reach this point ~2.5 us before waves 4-7 ("laggards", the
// step's critical path).  Each wave starts what its inputs allow, tracked by progress counters (every wave signals
// them from its backward):
//   leaders   counter C (every wave's ffn.3 / ffn.0 dY rows): the ffn.3 tile w4 and ffn.0 k tile w4 weight
//             gradients and the ffn.3 / ffn.0 bias sums — work that used to follow the barrier, now done while
//             the laggards are still in their backward; then counter A (every wave's out_proj dY rows, the
//             out_proj image no longer read): their out_proj unit — dW over the 128 rows, Adam on the workspace
//             copy (p, m, v), image, bias sums; then counter B (every wave's dense dY rows): the dense tile w4
//             and its bias sums;
//   laggards  counter A (the v unit's dY rows): their in_proj.v unit, whose new bf16 weights wait for counter B (the
//             v image is read until the end of every wave's backward).
// The leaders then run Adam on their small unit (the dense / ffn.3 / ffn.0 tiles, workspace-resident like the
// blocks) and write its images — in their slack while the laggards finish the v block.  The bias sums are held in
// registers until barrier 1; then they and the LayerNorm sums (fixed-point accumulators DBL, aliasing CS) are
// stored; barrier 2; every thread runs Adam on its compact entries (U3: the 648 bias / LayerNorm elements, 2 per
// thread — 5 when the small weights were compact entries too: +3.6 %, profiles/ab_tf2_r6_update.log).  The abort decision
// (a NaN loss anywhere in the batch) is taken by every wave after counter A or B — every abort word is written
// before its wave signals — before anything is updated.  Returns false on abort.
// (Measured first: the leaders taking both units after counter A was 1 % slower — A is reached only ~0.2 us
// before B, so the leaders' two units became the tail; profiles/ab_tf2_r6_update.log.)
template <int BR>
__device__ __forceinline__ bool br_update(uchar* smem, BrState& st, const AdamK& K, int lane, int wave, int tid, int step,
                                          __amdgpu_buffer_rsrc_t rm, Stamp& stp, gu32* tmo) {
  using B = BrK<BR>;
  opq(lane, wave);
  asm volatile("" : "+v"(tid));
  const int w4 = wave & 3, g = lane >> 4, i16 = lane & 15;
  const bool lead = wave < 4;
  const uint32_t all = 8u * (uint32_t)step;
  LDS_AS uint32_t* abort_w = ldsu(smem, B_MISC);
  const int Ta = 2 * (w4 & 1), Tb = 2 * (w4 >> 1);
  const bool do_bias = (w4 & 1) == 0;  // one of the two units that read dY tiles Tb, Tb + 1
  f4v bsu[2];                          // the unit's bias sums (out_proj on leaders, v on laggards)
  f4v as = Z4, bd = Z4, a3 = Z4, af1 = Z4, b3 = Z4, b1 = Z4;  // leaders: dense / ffn.3 / ffn.0 tiles + bias sums
  const int ui = 2 * w4 + (lead ? 0 : 1);
  f4v U[12];
#pragma unroll
  for (int j = 0; j < 12; ++j) U[j] = unit_ld(rm, ui, j, lane);
  uint32_t o1 = 0x3F803F80u;  // (all-ones operand, opaque SGPR: see unit_dw)
  asm volatile("" : "+s"(o1));
  const s8v one = __builtin_bit_cast(s8v, u32x4{o1, o1, o1, o1});
  if (lead) {
    // the leaders' ffn tiles run below the laggards' backward on the same SIMD (priority 0: +1.9 % against 2,
    // +1.7 % at 1; profiles/ab_tf2_r6_update.log), the out_proj unit after A at the critical priority again
    prio_lo();
    if (!lds_wait(smem, B_CNT_C, all)) {
      if (lane == 0) __hip_atomic_store(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
#pragma unroll  // (fully unrolled: the fragment reads of later k-steps overlap earlier MFMAs, +2.2 %)
    for (int s = 0; s < (ABL(K, ABL_U1) ? 0 : 4); ++s) {
      const s8v y3 = tfrag<TK64>(smem + B_DF3, 32 * s, w4, lane), y1 = tfrag<TK16>(smem + B_DF0, 32 * s, 0, lane);
      a3 = mma(tfrag<TK16>(smem + B_F2, 32 * s, 0, lane), y3, a3);
      af1 = mma(tfrag<TK64>(smem + B_X1N, 32 * s, w4, lane), y1, af1);
      b3 = mma(one, y3, b3);
      if (wave == 0) b1 = mma(one, y1, b1);
    }
    if (!lds_wait(smem, B_CNT_A, all)) {
      if (lane == 0) __hip_atomic_store(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    prio_hi();
  } else {
    // (the v unit's operands are complete at A — only its image write waits for B, the end of every wave's
    // backward — so the laggards' weight-gradient MFMAs overlap the last laggard's v backward)
    if (!lds_wait(smem, B_CNT_A, all)) {
      if (lane == 0) __hip_atomic_store(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
  }
  {
    uint32_t any = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) any |= abort_w[i];
    if (any) return false;
  }
  stp(4, tid);
  {  // the unit: out_proj (leaders: X = a, dY = d o) or in_proj.v (laggards: X = h0, dY = d v)
    f4v acc[2][2];
    if (!ABL(K, ABL_UDW))
      unit_dw(smem + (lead ? B_A : B_H0), smem + (lead ? B_DO : B_DV), Ta, Tb, lane, do_bias, acc, bsu);
    if (!ABL(K, ABL_UADAM)) unit_adam(U, acc, K);
    u32x2v w[4];
    unit_pack(U, w);
    if (!lead && !lds_wait(smem, B_CNT_B, all)) {  // (the v image is read until the end of every wave's backward)
      if (lane == 0) __hip_atomic_store(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    unit_img(smem, B::vo(!lead), Ta, Tb, lane, w);
#pragma unroll
    for (int j = 0; j < 12; ++j) unit_st(rm, ui, j, lane, U[j]);
  }
  if (lead) {
    f4v S[9];  // the small unit (issued here: its loads overlap the wait for B and the dense MFMAs)
#pragma unroll
    for (int j = 0; j < 9; ++j) S[j] = smu_ld(rm, w4, j, lane);
    if (!lds_wait(smem, B_CNT_B, all)) {  // (the dense dY rows and the LayerNorm sums below are complete at B)
      if (lane == 0) __hip_atomic_store(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
#pragma unroll  // (fully unrolled: the fragment reads of later k-steps overlap earlier MFMAs, +2.2 %)
    for (int s = 0; s < (ABL(K, ABL_U1) ? 0 : 4); ++s) {
      const s8v yd = tfrag<TK64>(smem + B_DZ0, 32 * s, w4, lane);
      as = mma(tfrag<TK16>(smem + B_XIN, 32 * s, 0, lane), yd, as);
      bd = mma(one, yd, bd);
    }
    // Adam on the small unit (dense, ffn.3, ffn.0 tiles); their images are free: the dense one is read only by the
    // forward, the ffn ones by the backward before counters C / A
    const f4v gs3[3] = {as, a3, af1};
    if (!ABL(K, ABL_U3)) smu_adam(S, gs3, K);
    smu_img<BR>(smem, S, w4, lane);
#pragma unroll
    for (int j = 0; j < 9; ++j) smu_st(rm, w4, j, lane, S[j]);
  }
  // LayerNorm gradient sums out of the fp64 accumulators (complete: counter B; DBL aliases CS, written back below)
  const float lnsum = tid < B_NLN ? lds_getq(smem + B_DBL, tid) : 0.f;
  const f4v cmom = mom_ld(rm, 0, tid);  // compact entries' m0 m1 v0 v1
  stp(5, tid);
  prio_hi();
  lds_bar();
  {
    LDS_AS float* cs = ldsf(smem, B_CS);
    if (tid < B_NLN) cs[ln_seg(tid >> 6) * 64 + (tid & 63)] = lnsum;
    if (do_bias && g == 0) {
#pragma unroll
      for (int b = 0; b < 2; ++b) cs[(lead ? VS_OB : VS_VB) * 64 + 16 * (Tb + b) + i16] = bsu[b][0];
    }
    if (lead) {
      if (g == 0) {
        cs[VS_F2B * 64 + 16 * w4 + i16] = b3[0];
        cs[VS_DB * 64 + 16 * w4 + i16] = bd[0];
        if (wave == 0 && i16 < FF) cs[VS_F1B + i16] = b1[0];
      }
    }
  }
  lds_bar();
  stp(6, tid);
  // ---- U3: compact entries, branch-free: every entry reads its gradient (CS or GS), runs Adam and
  // makes three stores whose addresses come from its precomputed descriptor (cmp_dst): the real ones
  // land in VEC / CS (fp32) or a weight image (bf16), the others in per-lane dummy words of the DF0 tile
  // (dead until the next backward).  Entries past the end or padding compute on garbage that only
  // reaches the dummies.  (The divergent if / else version was ~1,200 instructions, 1.4 us per step.)
  if (tid < (B_DBL_BYTES - B_NVEC * 4) / 4) ldsf(smem, B_CS)[B_NVEC + tid] = 0.f;
  float mm[NCMP] = {cmom[0], cmom[1]}, vv[NCMP] = {cmom[2], cmom[3]};
  if (!ABL(K, ABL_U3)) {
    const int dmy = B_DF0 + 4 * (tid & 63);
    float gr[NCMP], pn[NCMP];
#pragma unroll
    for (int h = 0; h < NCMP; ++h) {
      const int e = tid + NTH * h;
      gr[h] = e < B_NVEC ? *(const LDS_AS float*)(smem + B_CS + 4 * e) : 0.f;  // (past the end: dummies only)
    }
    adam_staged<NCMP>(st.cmp, mm, vv, gr, pn, K);
#pragma unroll
    for (int h = 0; h < NCMP; ++h) {
      const int e = tid + NTH * h;
      const uint32_t d = aru(st.dst[h]);
      const bool vec = e < B_NVEC;
      const bool f32 = d >> 31;
      const int off = (int)(d & 0x7FFFFFFFu);
      *(LDS_AS float*)(smem + (vec ? B_CS + 4 * e : dmy)) = 0.f;
      *(LDS_AS float*)(smem + (f32 ? off : dmy + 256)) = pn[h];
      *(LDS_AS unsigned short*)(smem + (f32 ? dmy + 512 : off)) = fk::f2bf(pn[h]);
    }
  }
  mom_st(rm, 0, tid, f4v{mm[0], mm[1], vv[0], vv[1]});
  return true;
}

// fresh Adam state (torch.optim.Adam is re-created every round, client.py:78): zero moment slab
__device__ __forceinline__ void mom_zero(__amdgpu_buffer_rsrc_t rm, int tid) {
#pragma unroll
  for (int k = 0; k < MOM_SLOTS; ++k) mom_st(rm, k, tid, Z4);
}

template <int BR>
__device__ __forceinline__ void br_init(uchar* smem, BrState& st, const float* P, __amdgpu_buffer_rsrc_t rm, int lane,
                                        int wave, int tid) {
  using B = BrK<BR>;
#pragma unroll
  for (int k = 0; k < CMP_SLOTS; ++k) mom_st(rm, k, tid, Z4);
  {  // wave w: unit 2 (w & 3) + (w >> 2) (every unit once): p from the parameters -> workspace + bf16 image, m = v = 0
    const int w4 = wave & 3, u = wave >> 2, Ta = 2 * (w4 & 1), Tb = 2 * (w4 >> 1);
    const Mat M = B::vo(u == 1);
    const int i16 = lane & 15, g4 = 4 * (lane >> 4);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int n = 16 * (Tb + (t & 1)) + i16, k0 = 16 * (Ta + (t >> 1)) + g4;
      const float* src = P + M.off + n * M.k_real + k0;  // (a client's parameter row is not 16-byte aligned)
      const f4v p = {src[0], src[1], src[2], src[3]};
      unit_st(rm, 2 * w4 + u, t, lane, Z4);
      unit_st(rm, 2 * w4 + u, 4 + t, lane, Z4);
      unit_st(rm, 2 * w4 + u, 8 + t, lane, p);
      *(LDS_AS u32x2v*)(smem + M.img + n * M.ld + pcol(k0) * 2) = u32x2v{pk2(p[0], p[1]), pk2(p[2], p[3])};
    }
  }
  if (wave < 4) {  // leader w4's small unit: p from the parameters (0 for padding) -> workspace + images, m = v = 0
    f4v S[9];
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      S[s] = S[3 + s] = Z4;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        int pi, img;
        smu_elem<BR>(s, wave, lane, i, pi, img);
        S[6 + s][i] = pi >= 0 ? P[pi] : 0.f;
      }
    }
    smu_img<BR>(smem, S, wave, lane);
#pragma unroll
    for (int j = 0; j < 9; ++j) smu_st(rm, wave, j, lane, S[j]);
  }
#pragma unroll
  for (int h = 0; h < NCMP; ++h) {
    const int e = tid + NTH * h;
    float p0 = 0.f;
    if (e < B_NVEC) {
      const int pi = cmp_param<BR>(e);
      p0 = pi >= 0 ? P[pi] : 0.f;
      ldsf(smem, B_VEC)[e] = p0;
      ldsf(smem, B_CS)[e] = 0.f;
    }
    st.cmp[h] = VS{aw(p0)};
    st.dst[h] = awu(cmp_dst<BR>(e, lane));
  }
}

template <int BR>
__device__ __forceinline__ void br_fini(const BrState& st, float* P, __amdgpu_buffer_rsrc_t rm, int lane, int wave,
                                        int tid) {
  using B = BrK<BR>;
  {  // the units' weights (stored by the waves that updated them: wait for every store before reading back)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const int w4 = wave & 3, u = wave >> 2, Ta = 2 * (w4 & 1), Tb = 2 * (w4 >> 1);
    const Mat M = B::vo(u == 1);
    const int i16 = lane & 15, g4 = 4 * (lane >> 4);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int n = 16 * (Tb + (t & 1)) + i16, k0 = 16 * (Ta + (t >> 1)) + g4;
      const f4v p = unit_ld(rm, 2 * w4 + u, 8 + t, lane);
      float* dst = P + M.off + n * M.k_real + k0;
#pragma unroll
      for (int i = 0; i < 4; ++i) dst[i] = p[i];
      store_guard();  // (merged into one 16-byte store: the next unit's load must not be its very next instruction)
    }
  }
  if (wave < 4) {  // leader w4's small unit (its own stores)
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      const f4v p = smu_ld(rm, wave, 6 + s, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        int pi, img;
        smu_elem<BR>(s, wave, lane, i, pi, img);
        if (pi >= 0) P[pi] = p[i];
      }
      store_guard();
    }
  }
#pragma unroll
  for (int h = 0; h < NCMP; ++h) {
    const int e = tid + NTH * h;
    if (e < B_NVEC) {
      const int pi = cmp_param<BR>(e);
      if (pi >= 0) P[pi] = ar(st.cmp[h].p);
    }
  }
}

// this lane's 4 input features (4g + i) of row r of the batch starting at b0 of epoch e
template <int BR>
__device__ __forceinline__ void load_x(float (&x)[4], const AflTfTrainArgs& a, int cid, const Walk& w, int r, int g) {
  const int Bn = min(a.batch, a.nd[cid] - w.b0);
  const gi32* ord = (const gi32*)(a.order + ((long)cid * a.E + w.e) * a.maxnd);
  const bool valid = r < Bn;
  const int ridx = valid ? ord[w.b0 + r] : 0;
  const gf* row = (const gf*)a.rows + (long)ridx * ROW + BrK<BR>::xoff;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = 4 * g + i;
    x[i] = (valid && c < BrK<BR>::din) ? row[c] : 0.f;
  }
}

__device__ __forceinline__ void stamp_init(Stamp& stp, const AflTfTrainArgs& a, uchar* smem) {
#ifdef TF2_STAMPS
  stp.on = a.stamps && (long)blockIdx.x == (long)a.stamps[63];
  stp.who = a.stamps ? 64 * (int)(a.stamps[62] & 7) : 0;
  stp.smem = smem;
  if (threadIdx.x == 0) *(LDS_AS uint64_t*)(smem + ST_OFF + 8 * (ST_N - 1)) = __builtin_amdgcn_s_memrealtime();
#endif
  (void)stp; (void)a; (void)smem;
}
__device__ __forceinline__ void stamp_fini(Stamp& stp, const AflTfTrainArgs& a, uchar* smem, int tid) {
#ifdef TF2_STAMPS
  if (stp.on && tid == 0)
    for (int i = 0; i < ST_N - 1; ++i) a.stamps[i] = *(LDS_AS uint64_t*)(smem + ST_OFF + 8 * i);
#endif
  (void)stp; (void)a; (void)smem; (void)tid;
}

template <int BR>
__device__ __forceinline__ void branch_main(const AflTfTrainArgs& a, int cid, uchar* smem) {
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6), g = lane >> 4;
  float* P = a.params + (long)cid * NPARAM;
  uchar* ws = (uchar*)(a.ws + (long)cid * a.ws_stride);
  gu32* sync = (gu32*)(a.sync + (long)cid * AFL_TF2_SYNC_WORDS);
  const __amdgpu_buffer_rsrc_t rg = gr_rsrc(sync);  // granule hand-off slots
  for (int i = tid; i < SMEM / 4; i += NTH) ldsf(smem, 0)[i] = 0.f;
  __syncthreads();
  BrState st;
  const __amdgpu_buffer_rsrc_t rm = rsrc(ws + WS_MOM + MOM_WG_BYTES + BR * BR_WG_BYTES);  // this workgroup's units
  br_init<BR>(smem, st, P, rm, lane, wave, tid);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the units' first loads come from other waves' stores)
  __syncthreads();
  Stamp stp;
  stamp_init(stp, a, smem);

  const int nd = a.nd[cid], BS = a.batch, E = a.E;
  const uint32_t seed = a.seeds[cid];
  LDS_AS uint32_t* abort_w = ldsu(smem, B_MISC);
  int step = 0;
  bool failed = false;
  Walk w{0, 0};
  float xin[4];
  bool more = walk_valid(w, nd, BS, E);
  if (more) load_x<BR>(xin, a, cid, w, 16 * wave + (lane & 15), g);
  float mka0, mka1;  // the next forward's dropout masks (br_masks), parked in AGPRs
  {
    uint32_t m0, m1;
    br_masks<BR>(afl_hash32(seed, 1u), 16 * wave + (lane & 15), g, m0, m1);
    mka0 = awu(m0);
    mka1 = awu(m1);
  }
  while (more) {
    ++step;
    const AdamK K = adam_k(a, step);
    Saved sv;
    u32x4 outp[2];
    prio_hi();
    asm volatile(";MARK fwd");
#ifndef TF2_NO_FWD
    br_forward<BR>(smem, xin, aru(mka0), aru(mka1), sv, outp, lane, wave);
#else
    sv = Saved{}; outp[0] = u32x4{0,0,0,0}; outp[1] = outp[0];
#endif
    asm volatile(";MARK fwd_end");
    stp(0, tid);
    gr_put(rg, gr_off(0, BR, wave, lane), outp, (uint32_t)step);  // this wave's output rows -> head
    prio_lo();
    w.b0 += BS;  // prefetch the next batch's inputs while the head works
    more = walk_valid(w, nd, BS, E);
    if (more) load_x<BR>(xin, a, cid, w, 16 * wave + (lane & 15), g);
    {  // the next step's dropout masks, while the head works (this wave would only spin)
      uint32_t m0, m1;
      br_masks<BR>(afl_hash32(seed, (uint32_t)(step + 1)), 16 * wave + (lane & 15), g, m0, m1);
      mka0 = awu(m0);
      mka1 = awu(m1);
    }
    stp(1, tid);
    u32x4 du[2];
    const int go[1] = {gr_off(1, BR, wave, lane)};
    const uint32_t fv = gr_get<1>(rg, go, du, (uint32_t)step, 1, sync + XF_TMO, lane);  // d(out) of this wave's rows
    prio_hi();  // (the leaders' backward below the laggards' measured -0.5 %: profiles/ab_tf2_r6_update.log)
    stp(2, tid);
    if (fv == 0xFFFFFFFFu) {  // timed out: abort the step for every wave (they wait on this wave's progress)
      if (lane == 0) abort_w[wave] = 1u;
      lds_signal(smem, B_CNT_A, lane);
      lds_signal(smem, B_CNT_B, lane);
      failed = true;
      break;
    }
    float dout[16];
    unpack16(du, dout);
    if (lane == 0) abort_w[wave] = fv & 1u;
#ifndef TF2_NO_BWD
    asm volatile(";MARK bwd");
    br_backward<BR>(smem, dout, sv, K, lane, wave);
    asm volatile(";MARK bwd_end");
    stp(3, tid);
#else
    for (int j = 0; j < 16; ++j) asm volatile("" :: "v"(dout[j]));
    lds_signal(smem, B_CNT_A, lane);
    lds_signal(smem, B_CNT_B, lane);
#endif
    asm volatile(";MARK upd");
    // (false: the head saw a NaN loss somewhere in the batch — the client's round fails and this step's update is
    // not applied — or a wave stopped making progress)
    const bool upd_ok = br_update<BR>(smem, st, K, lane, wave, tid, step, rm, stp, sync + XF_TMO);
    asm volatile(";MARK upd_end");
    if (!upd_ok) {
      failed = true;
      break;
    }
    stp(7, tid);
    lds_bar();
    stp(8, tid);
  }
  (void)failed;
  stamp_fini(stp, a, smem, tid);
  br_fini<BR>(st, P, rm, lane, wave, tid);
}

// ================================================================================= head workgroup
constexpr Mat HW1{FC1_W, 64, 128, H_IMG_W1, HLD1};
constexpr Mat HW2{FC2_W, 32, 64, H_IMG_W2, HLD2};
__device__ __forceinline__ int hvec_param(int e) {
  return e < 64 ? FC1_B + e : e < 96 ? FC2_B + (e - 64) : e < 128 ? OUT_W + (e - 96) : e == 128 ? OUT_B : -1;
}
struct HdState {
  TS blk[4];  // fc1: k tiles 2(w&3)+{0,1} x n tiles 2(w>>2)+{0,1}
  TS t2;      // fc2: k tile w&3, n tile w>>2
  VS vec;
};

__device__ __forceinline__ void head_main(const AflTfTrainArgs& a, int cid, uchar* smem) {
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6), g = lane >> 4;
  const int r = 16 * wave + (lane & 15);
  float* P = a.params + (long)cid * NPARAM;
  uchar* ws = (uchar*)(a.ws + (long)cid * a.ws_stride);
  gu32* sync = (gu32*)(a.sync + (long)cid * AFL_TF2_SYNC_WORDS);
  const __amdgpu_buffer_rsrc_t rg = gr_rsrc(sync);  // granule hand-off slots
  for (int i = tid; i < SMEM / 4; i += NTH) ldsf(smem, 0)[i] = 0.f;
  __syncthreads();
  HdState st;
  Stamp stp;
  const __amdgpu_buffer_rsrc_t rm = rsrc(ws + WS_MOM);  // this workgroup's Adam moments
  mom_zero(rm, tid);
  {
    const int Ta = 2 * (wave & 3), Tb = 2 * (wave >> 2);
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int y = 0; y < 2; ++y) tile_load(st.blk[2 * x + y], HW1, Ta + x, Tb + y, lane, P, smem);
    tile_load(st.t2, HW2, wave & 3, wave >> 2, lane, P, smem);
    float p0 = 0.f;
    if (tid < H_NVEC) {
      const int pi = hvec_param(tid);
      p0 = pi >= 0 ? P[pi] : 0.f;
      ldsf(smem, H_VEC)[tid] = p0;
    }
    st.vec = VS{aw(p0)};
  }
  __syncthreads();
  stamp_init(stp, a, smem);

  const int nd = a.nd[cid], BS = a.batch, E = a.E;
  const int nb_total = (nd + BS - 1) / BS;
  const uint32_t seed = a.seeds[cid];
  const uchar* vec = smem + H_VEC;
  LDS_AS float* part = ldsf(smem, H_PART) + wave * H_NVEC;  // this wave's column sums
  LDS_AS float* lossw = ldsf(smem, H_LOSS);
  int step = 0;
  bool failed = false, timed_out = false;
  float epoch_loss = 0.f;
  Walk w{0, 0};
  int cur_e = 0;
  bool more = walk_valid(w, nd, BS, E);
  float lab = 0.f;
  auto load_lab = [&](const Walk& ww) {
    const int Bn = min(BS, nd - ww.b0);
    const gi32* ord = (const gi32*)(a.order + ((long)cid * E + ww.e) * a.maxnd);
    lab = r < Bn ? ((const gf*)a.rows)[(long)ord[ww.b0 + r] * ROW + ROW - 1] : 0.f;
  };
  if (more) load_lab(w);
  while (more) {
    // epoch boundaries crossed since the previous step (skipped batches included) close epoch losses
    while (cur_e < w.e) {
      if (tid == 0) a.losses[(long)cid * E + cur_e] = epoch_loss / (float)max(nb_total, 1);
      epoch_loss = 0.f;
      ++cur_e;
    }
    ++step;
    const AdamK K = adam_k(a, step);
    const uint32_t key = afl_hash32(seed, (uint32_t)step);
    const int Bn = min(BS, nd - w.b0);
    const bool valid = r < Bn;
    const float inv_bn = 1.f / (float)Bn;  // (before the wait: the division is off the critical path)
    // fc1 dropout mask before the wait (the wave would only spin there)
    const uint32_t mh = mask16(key, L_HEAD, r, g, THR_P03);
    sb();
    // ---- branch outputs of this wave's rows
    u32x4 cv[4];  // vitals rows (cv[0..1]) | labs rows (cv[2..3])
    const int go[2] = {gr_off(0, 0, wave, lane), gr_off(0, 1, wave, lane)};
    const uint32_t fv = gr_get<2>(rg, go, cv, (uint32_t)step, 0, sync + XF_TMO, lane);
    if (fv == 0xFFFFFFFFu) {
      timed_out = failed = true;
      break;
    }
    prio_hi();  // (head waves 0-3 below 4-7 measured -7 %: profiles/ab_tf2_r6_update.log)
    stp(10, tid);
    // (the dW operands of this step — cat, a1, dz1, dz2 tiles — and the head's column sums are written
    // only AFTER the d(cat) hand-off below: they are off the branches' critical path)
    // ---- fc1 + GELU + dropout(0.3)
    float a1[16], gk1[16];
    {
      f4v acc[4];
#pragma unroll
      for (int T = 0; T < 4; ++T) {
        acc[T] = Z4;
#pragma unroll
        for (int s = 0; s < 4; ++s)
          acc[T] = mma(wfrag(smem + H_IMG_W1, HLD1, T, s, lane), __builtin_bit_cast(s8v, cv[s]), acc[T]);
      }
      float b1[16];
      vec16(b1, vec + HV_B1 * 4, g);
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int i = 0; i < 4; i += 2) {
          const int j = 4 * t + i;
          gf2v gp;
          const gf2v gl = gelu2(gf2v{acc[t][i] + b1[j], acc[t][i + 1] + b1[j + 1]}, gp);
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            a1[j + h] = keepf(gl[h] * INV_K03, mh, j + h);
            gk1[j + h] = keepf(gp[h] * INV_K03, mh, j + h);
          }
        }
    }
    // ---- fc2 + GELU, output layer, sigmoid, BCE (log clamped at -100)
    float dz2[8], gw[8];
    float dy3 = 0.f, pl = 0.f;
    {
      const s8v b0 = bfrag(a1, 0), b1 = bfrag(a1, 1);
      f4v acc[2];
#pragma unroll
      for (int T = 0; T < 2; ++T) {
        acc[T] = mma(wfrag(smem + H_IMG_W2, HLD2, T, 0, lane), b0, Z4);
        acc[T] = mma(wfrag(smem + H_IMG_W2, HLD2, T, 1, lane), b1, acc[T]);
      }
      float b2[8], wo[8], g2[8], gp2[8];
      vec8(b2, vec + HV_B2 * 4, g);
      vec8(wo, vec + HV_WO * 4, g);
      float dot = 0.f;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int i = 0; i < 4; i += 2) {
          const int j = 4 * t + i;
          gf2v gp;
          const gf2v gl = gelu2(gf2v{acc[t][i] + b2[j], acc[t][i + 1] + b2[j + 1]}, gp);
          g2[j] = gl[0];
          g2[j + 1] = gl[1];
          gp2[j] = gp[0];
          gp2[j + 1] = gp[1];
          dot += g2[j] * wo[j];
          dot += g2[j + 1] * wo[j + 1];
        }
      const float y3 = fk::rsum4(dot) + *(const LDS_AS float*)(vec + HV_BO * 4);
      const float p = sigmoidf_(y3);
      if (valid) {
        // torch's BCELoss gradient (p - y) / max(p (1 - p), 1e-12) times the sigmoid's p (1 - p), as one factor
        // without a division (1 unless the sigmoid saturates; NaN propagates through the compare's false branch)
        const float pq = p * (1.f - p);
        dy3 = (p - lab) * (pq >= 1e-12f ? 1.f : pq * 1e12f) * inv_bn;
      }
      pl = p;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        dz2[j] = dy3 * wo[j] * gp2[j];
        gw[j] = dy3 * g2[j];
      }
    }
    // the NaN-loss abort rides on the hand-off tag: a row's loss is NaN exactly where its gradient factor dy3 is
    // not finite (p or the label NaN; labels are 0 / 1), so the flag needs no loss on the critical path — the loss
    // VALUE (logs, wave sum) is computed after the hand-off, and the head aborts on the same flags
    const uint32_t wave_nan = __builtin_amdgcn_ballot_w64(!(fabsf(dy3) <= 3.402823466e38f)) != 0 ? 1u : 0u;
    // ---- d a1 = dz2 . W2 -> d z1 = d a1 * drop'(.) * gelu'(z1)
    float dz1[16];
    {
      const s8v bz = bfrag(dz2, 0);
#pragma unroll
      for (int T = 0; T < 4; ++T) {
        const f4v acc = mma(wtfrag<true>(smem + H_IMG_W2, HLD2, T, 0, lane), bz, Z4);
#pragma unroll
        for (int i = 0; i < 4; ++i) dz1[4 * T + i] = acc[i] * gk1[4 * T + i];
      }
    }
    // ---- d cat = dz1 . W1, each half straight to its branch
    {
      const s8v b0 = bfrag(dz1, 0), b1 = bfrag(dz1, 1);
#pragma unroll
      for (int hb = 0; hb < 2; ++hb) {
        float d[16];
#pragma unroll
        for (int Tl = 0; Tl < 4; ++Tl) {
          const int T = 4 * hb + Tl;
          f4v acc = mma(wtfrag<true>(smem + H_IMG_W1, HLD1, T, 0, lane), b0, Z4);
          acc = mma(wtfrag<true>(smem + H_IMG_W1, HLD1, T, 1, lane), b1, acc);
#pragma unroll
          for (int i = 0; i < 4; ++i) d[4 * Tl + i] = acc[i];
        }
        u32x4 u[2];
        pack16(d, u);
        gr_put(rg, gr_off(1, hb, wave, lane), u, ((uint32_t)step << 1) | wave_nan);  // NaN abort rides on the tag
      }
    }
    prio_lo();
    {  // per-wave loss partial (each row counted once: lane group 0) and the abort flag, for the loss barrier
      float lrow = 0.f;
      if (valid) {
        // clamp like torch.clamp: NaN must propagate (fmaxf would swallow it)
        float lg, lg1;
        bce_logs(pl, lg, lg1);
        const float lp = lg < -100.f ? -100.f : lg, l1p = lg1 < -100.f ? -100.f : lg1;
        lrow = -(lab * lp + (1.f - lab) * l1p);
      }
      const float lsum = wave_sum(g == 0 ? lrow : 0.f);
      if (lane == 0) {
        lossw[wave] = lsum;
        lossw[8 + wave] = __uint_as_float(wave_nan);
      }
    }
    // ---- deferred: dW operand tiles and column sums of this wave's rows (read after the loss barrier)
    {
      sb();
#pragma unroll
      for (int t = 0; t < 8; ++t) {  // cat: tile t of the 8 = half (t & 1) of cv[t >> 1]
        const u32x4 u = cv[t >> 1];
        const u32x2v v = (t & 1) ? u32x2v{u[2], u[3]} : u32x2v{u[0], u[1]};
        *(LDS_AS u32x2v*)(smem + H_CAT + t128(r, 4 * t + g)) = v;
      }
#pragma unroll
      for (int t = 0; t < 4; ++t) st4<TK64>(smem + H_A1, r, 4 * t + g, a1 + 4 * t);
#pragma unroll
      for (int t = 0; t < 2; ++t) st4<TK32>(smem + H_DZ2, r, 4 * t + g, dz2 + 4 * t);
#pragma unroll
      for (int t = 0; t < 4; ++t) st4<TK64>(smem + H_DZ1, r, 4 * t + g, dz1 + 4 * t);
      float sb2, swo, sb1;
      const int f2 = colsum32(dz2, lane, sb2), fo = colsum32(gw, lane, swo);
      if (f2 >= 0) {
        part[HV_B2 + f2] = sb2;
        part[HV_WO + fo] = swo;
      }
      const int f1 = colsum64(dz1, lane, sb1);
      part[HV_B1 + f1] = sb1;
      const float dbo = wave_sum(g == 0 ? dy3 : 0.f);  // d output.bias
      if (lane == 0) part[HV_BO] = dbo;
    }
    stp(11, tid);
    // Adam moments of this step's update (after the hand-off drain, before the loss barrier)
    f4v hm[6], hv[6];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      hm[k] = mom_ld(rm, k, tid);
      hv[k] = mom_ld(rm, 4 + k, tid);
    }
    hm[4] = mom_ld(rm, 8, tid);
    hv[4] = mom_ld(rm, 9, tid);
    hm[5] = mom_ld(rm, 10, tid);
    // the next step's labels (after the hand-off stores: their drain above must not wait for these)
    Walk wn = w;
    wn.b0 += BS;
    more = walk_valid(wn, nd, BS, E);
    lds_bar();
    {
      float tot = 0.f;
      uint32_t any = 0;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        tot += lossw[i];
        any |= __float_as_uint(lossw[8 + i]);
      }
      const float loss = tot / (float)Bn;
      if (any) {  // a NaN loss (uniform across the workgroup; the branches abort on the same per-wave flags)
        failed = true;
        break;
      }
      epoch_loss += loss;
    }
    if (more) load_lab(wn);
    w = wn;
    stp(12, tid);
    // ---- weight gradients + Adam
    {
      const int Ta = 2 * (wave & 3), Tb = 2 * (wave >> 2);
      f4v acc[2][2] = {{Z4, Z4}, {Z4, Z4}};
      f4v a2 = Z4;
      const int T2 = wave & 3, Tn2 = wave >> 2;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const s8v x0 = tfrag<TK128>(smem + H_CAT, 32 * s, Ta, lane), x1 = tfrag<TK128>(smem + H_CAT, 32 * s, Ta + 1, lane);
        const s8v y0 = tfrag<TK64>(smem + H_DZ1, 32 * s, Tb, lane), y1 = tfrag<TK64>(smem + H_DZ1, 32 * s, Tb + 1, lane);
        acc[0][0] = mma(x0, y0, acc[0][0]);
        acc[0][1] = mma(x0, y1, acc[0][1]);
        acc[1][0] = mma(x1, y0, acc[1][0]);
        acc[1][1] = mma(x1, y1, acc[1][1]);
        a2 = mma(tfrag<TK64>(smem + H_A1, 32 * s, T2, lane), tfrag<TK32>(smem + H_DZ2, 32 * s, Tn2, lane), a2);
      }
#pragma unroll
      for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y)
          if (!ABL(K, ABL_HEADUPD))
            tile_adam(st.blk[2 * x + y], hm[2 * x + y], hv[2 * x + y], HW1, Ta + x, Tb + y, lane, acc[x][y], K, smem);
      if (!ABL(K, ABL_HEADUPD)) tile_adam(st.t2, hm[4], hv[4], HW2, T2, Tn2, lane, a2, K, smem);
      if (tid < H_NVEC) {
        // the 8 waves' partial sums in a fixed order: bit-reproducible whatever order the waves ran in
        const LDS_AS float* c = ldsf(smem, H_PART) + tid;
        float gsum = c[0];
#pragma unroll
        for (int w8 = 1; w8 < 8; ++w8) gsum += c[w8 * H_NVEC];
        float vm = hm[5][0], vvv = hm[5][1];
        if (hvec_param(tid) >= 0) ldsf(smem, H_VEC)[tid] = adam1(st.vec.p, vm, vvv, gsum, K);
        hm[5][0] = vm;
        hm[5][1] = vvv;
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        mom_st(rm, k, tid, hm[k]);
        mom_st(rm, 4 + k, tid, hv[k]);
      }
      mom_st(rm, 8, tid, hm[4]);
      mom_st(rm, 9, tid, hv[4]);
      mom_st(rm, 10, tid, hm[5]);
    }
    stp(13, tid);
    lds_bar();
    stp(14, tid);
  }
  stamp_fini(stp, a, smem, tid);
  if (!failed) {
    while (cur_e < E) {  // the last epoch (and trailing epochs that had no step)
      if (tid == 0) a.losses[(long)cid * E + cur_e] = epoch_loss / (float)max(nb_total, 1);
      epoch_loss = 0.f;
      ++cur_e;
    }
  }
  // parameters back (a failed client keeps its pre-step values: the failing step applied no update)
  {
    const int Ta = 2 * (wave & 3), Tb = 2 * (wave >> 2);
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int y = 0; y < 2; ++y) tile_store(st.blk[2 * x + y], HW1, Ta + x, Tb + y, lane, P);
    tile_store(st.t2, HW2, wave & 3, wave >> 2, lane, P);
    if (tid < H_NVEC && hvec_param(tid) >= 0) P[hvec_param(tid)] = ar(st.vec.p);
  }
  if (tid == 0) {
    const bool tmo = timed_out || __hip_atomic_load(sync + XF_TMO, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    a.ok[cid] = tmo ? -1 : (failed ? 0 : 1);
  }
}

}  // namespace t2

#ifdef TF2_STAMPS
#define K_TF2 k_tf2_train_stamped
#else
#define K_TF2 k_tf2_train
#endif
// 3 workgroups per client: blocks c (head), CP + c (vitals branch), 2 CP + c (labs branch).  Role-major block order
// with a block stride CP padded to a multiple of 8 when the grid still fits: a client's workgroups are blocks
// role * CP + cid, which the round-robin dispatch deals to ONE XCD (same-L2 hand-offs; speed only, never
// correctness); padding blocks (cid >= C) exit at once.
__global__ void __launch_bounds__(t2::NTH) K_TF2(AflTfTrainArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int cp = a.cpad > 0 ? a.cpad : a.C;
  const int role = blockIdx.x / cp, cid = blockIdx.x - role * cp;
  if (cid >= a.C) return;
#if defined(TF2_ROLE)
  if (TF2_ROLE == 0) t2::head_main(a, cid, smem);
  else if (TF2_ROLE == 1) t2::branch_main<0>(a, cid, smem);
  else t2::branch_main<1>(a, cid, smem);
  (void)role;
#else
  if (role == 0)
    t2::head_main(a, cid, smem);
  else if (role == 1)
    t2::branch_main<0>(a, cid, smem);
  else
    t2::branch_main<1>(a, cid, smem);
#endif
}

#ifndef TF2_STAMPS
// Determinism check of the cross-wave column-sum accumulator (onchip.h lds_addq), used by the tests: W waves
// each add their 64 partials (vals [W][64]) into 64 slots after a per-wave delay drawn from `seed` (so the
// arrival order changes from launch to launch); out [64] = the decoded sums.  mode 1: the unquantised fp64 LDS
// atomics the trainers used before (order-dependent once the partials span more than ~2^29).
__global__ void __launch_bounds__(1024) k_fxsum_test(const float* __restrict__ vals, int W, uint32_t seed, int mode,
                                                   float* __restrict__ out) {
  __shared__ double q[64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (threadIdx.x < 64) q[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t spins = afl_hash32(seed, (uint32_t)w) & 1023u;
  for (uint32_t i = 0; i < spins; ++i) __builtin_amdgcn_s_sleep(1);
  const float v = vals[w * 64 + lane];
  if (mode == 0)
    oc::lds_addq((oc::uchar*)q, lane, v);
  else
    __hip_atomic_fetch_add((LDS_AS double*)q + lane, (double)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  __syncthreads();
  if (threadIdx.x < 64)
    out[lane] = mode == 0 ? oc::lds_getq((const oc::uchar*)q, lane)
                          : (float)((LDS_AS double*)q)[lane];
}
int afl_fxsum_test(const float* vals, int W, uint32_t seed, int mode, float* out, hipStream_t s) {
  if (W < 1 || W > 8) return -1;  // (at most 8 partials per slot: onchip.h lds_addq)
  hipLaunchKernelGGL(k_fxsum_test, dim3(1), dim3(64 * W), 0, s, vals, W, seed, mode, out);
  return (int)hipGetLastError();
}
#endif

#ifdef TF2_STAMPS
int afl_tf2_train_stamped(const AflTfTrainArgs* a, hipStream_t s) {
#else
long afl_tf2_ws_floats() { return t2::WS_BYTES / 4; }

int afl_tf2_train(const AflTfTrainArgs* a, hipStream_t s) {
  if (a->stamps) return afl_tf2_train_stamped(a, s);
#endif
  if (a->batch > 128 || a->batch < 2 || !a->sync) return -1;
  if (!a->kt || a->kt_n < a->E * ((a->maxnd + a->batch - 1) / a->batch)) return -5;  // step table too short
  if (hipFuncSetAttribute((const void*)K_TF2, hipFuncAttributeMaxDynamicSharedMemorySize, t2::SMEM) != hipSuccess) return -2;
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return -3;
  const int wgs = 3;
  if (wgs * a->C > cus) return -4;  // the workgroups of a client spin on each other: all must be resident
  AflTfTrainArgs b = *a;
  b.cpad = (a->C + 7) / 8 * 8;
#ifdef TF2_NO_PAD  // A/B variant: the unpadded role-major grid
  b.cpad = a->C;
#endif
  if (wgs * b.cpad > cus) b.cpad = a->C;
  hipLaunchKernelGGL(K_TF2, dim3(wgs * b.cpad), dim3(t2::NTH), t2::SMEM, s, b);
  return 0;
}
