// Fused TransformerModel/ICU local training — ONE persistent launch trains every client of a rank
// for all its local epochs (reference training loop client.py:75-111, model src/Model.py:166-246).
//
// Grid = one 512-thread workgroup (8 waves) per client.  Per optimizer step (batch <= 128 rows):
//   forward  : 2 branches (dense->GELU -> L=1 MHA (== out_proj(dropout_head(v_proj))) -> +res LN ->
//              FFN(64->6->64, GELU) -> +res LN -> LN) -> head (128->64 GELU drop0.3 ->32 GELU ->1 sigmoid)
//   loss     : BCE (log clamped at -100); NaN -> client result False (client.py:100-102)
//   backward : hand-written VJPs of every op; weight gradients never leave the MFMA accumulators:
//              the dW GEMM epilogue applies Adam directly (torch.optim.Adam math, fresh per round)
//
// GEMMs run on v_mfma_f32_16x16x32_bf16 (bf16 operands, fp32 accumulate):
//   X.W^T and dY.W  : activation fragments from LDS (ds_read_b128), weight fragments from bf16
//                     copies in global memory (row and transposed layouts, rewritten by Adam),
//                     prefetched into registers one phase ahead
//   dW = dY^T.X     : both operands from LDS through the gfx950 transposed read ds_read_b64_tr_b16
// Elementwise work (bias, exact-erf GELU, dropout, residual, LayerNorm fwd/bwd, BCE) runs in fp32
// in a row-per-4-lanes layout between GEMM phases.  Master weights, Adam moments and activations
// saved for the backward pass live in a per-client global workspace (L2 resident); residuals that
// the same lane needs later (h0, x1, y1, dr2, dh0) stay in registers.
//
// The kernel is latency bound (one CU per client, ~50 dependent phases per step), so:
//   * phases are separated by raw LDS barriers (s_waitcnt lgkmcnt(0); s_barrier): global loads stay
//     in flight across them and global stores are not drained — every global value is re-read only by
//     the lane that wrote it within a step; one full __syncthreads() per step publishes Adam's writes;
//   * each phase issues all of its global loads before its first LDS access.
//
// Attention at seq_len 1: softmax over one key is exactly 1, so the output is
// out_proj(dropout(v_proj(x))) with the dropout mask per (row, head) (SDPA math path), and the
// q/k projections receive exactly zero gradient (softmax backward at L=1 is 0) — Adam leaves
// them unchanged, so they are skipped here bit-for-bit.
// Dropout masks come from a stateless hash of (client seed, step, layer, row, col), regenerated in
// backward; bitwise parity with torch's Philox stream is impossible by construction.
#include "common.h"
#include "kernels.h"
#include "tf_common.h"
#include "fused_common.h"

using namespace tf;
using namespace fk;

namespace {

// LDS map (bytes)
constexpr int LD64 = 72, LD32 = 40, LD128 = 136, LDACC = 68;
constexpr int S_ACC = 0;
constexpr int S_XIN = S_ACC + BM * LDACC * 4;     // 34816 ; XIN / DF0  [128][40] bf16
constexpr int S_TA = S_XIN + BM * LD32 * 2;       // 45056
constexpr int S_TB = S_TA + BM * LD64 * 2;        // 63488
constexpr int S_TC = S_TB + BM * LD64 * 2;        // 81920
constexpr int S_CAT = S_TC + BM * LD64 * 2;       // 100352 ; CAT [128][136] / TD [128][72]
constexpr int S_F2 = S_CAT + BM * LD128 * 2;      // 135168 ; F2 / T32 [128][40]
constexpr int S_CS = S_F2 + BM * LD32 * 2;        // 145408 ; CS fp32 [6][8][64]
constexpr int S_LAB = S_CS + 6 * 8 * 64 * 4;      // 157696
constexpr int S_DY3 = S_LAB + BM * 4;             // 158208
constexpr int S_RED = S_DY3 + BM * 4;             // 158720
constexpr int S_TOTAL = S_RED + 16 * 4;           // 158784
static_assert(S_TOTAL <= 160 * 1024, "LDS budget");
// Branch-only workgroups: bf16 image [64][LDW] of the dense weight inside the CAT region (past TD,
// which those workgroups never use as CAT).  The dWd Adam epilogue writes the updated weights here, so
// the next step's first GEMM reads them from LDS instead of waiting for the stores and a global reload.
constexpr int LDW = 40;
constexpr int S_WDI = S_CAT + BM * LD64 * 2;      // 118784
static_assert(S_WDI + 64 * LDW * 2 <= S_F2, "dense image fits behind TD");

// ---- workspace layout (float units) ----
constexpr long W_M = 0, W_V = NPARAM;
constexpr long W_BF = ((2L * NPARAM + 63) / 64) * 64;  // bf16 region (16-B aligned)
// bf16 weight copies (ushort offsets inside the bf16 region), per branch then head
struct BrW { int WFd, WFv, WTv, WFo, WTo, WF1, WT1, WF2, WT2; };
__host__ __device__ constexpr BrW brw(int base) {
  BrW w{};
  int p = base;
  w.WFd = p; p += 64 * 32;
  w.WFv = p; p += 64 * 64;
  w.WTv = p; p += 64 * 64;
  w.WFo = p; p += 64 * 64;
  w.WTo = p; p += 64 * 64;
  w.WF1 = p; p += 16 * 64;
  w.WT1 = p; p += 64 * 32;
  w.WF2 = p; p += 64 * 32;
  w.WT2 = p; p += 16 * 64;
  return w;
}
constexpr int BRW_SIZE = 64 * 32 + 4 * 64 * 64 + 16 * 64 + 64 * 32 + 64 * 32 + 16 * 64;  // 24576
constexpr BrW WBV = brw(0);
constexpr BrW WBL = brw(BRW_SIZE);
constexpr int WFF1 = 2 * BRW_SIZE, WTF1 = WFF1 + 64 * 128, WFF2 = WTF1 + 128 * 64, WTF2 = WFF2 + 32 * 64;
constexpr int BF_TOTAL = WTF2 + 64 * 32;  // ushorts
// saved activations (float offsets); every entry is written and re-read by the same lane
constexpr long W_ACT = ((W_BF + BF_TOTAL / 2 + 63) / 64) * 64;
struct BrS { long H0B, XH1, XH2, XH3, RS, F0, MK, GPD, F2S, AB; };
__host__ __device__ constexpr BrS brs(long base) {
  BrS s{};
  long p = base;
  s.H0B = p; p += BM * 64 / 2;  // bf16 h0
  s.XH1 = p; p += BM * 64;
  s.XH2 = p; p += BM * 64;
  s.XH3 = p; p += BM * 64;
  s.RS = p; p += BM * 4 * 4;     // per lane: rstd1, rstd2, rstd3, pad
  s.F0 = p; p += BM * 8;
  s.MK = p; p += BM * 16;        // per lane: dropout keep masks D1, DF, D2 (u32 bits), pad
  s.GPD = p; p += BM * 64;       // gelu'(z0) of the dense layer
  s.F2S = p; p += BM * 8;        // f2 = drop(gelu(f0)) (F0 holds drop'(.) * gelu'(f0))
  s.AB = p; p += BM * 64 / 2;    // bf16 a = head_dropout(v), the X operand of dWo
  return s;
}
constexpr long BRS_SIZE = BM * 32 + 3L * BM * 64 + BM * 16 + BM * 8 + BM * 16 + BM * 64 + BM * 8 + BM * 32;
constexpr BrS SV = brs(W_ACT);
constexpr BrS SL = brs(W_ACT + BRS_SIZE);
constexpr long W_DX3V = W_ACT + 2 * BRS_SIZE;
// branch-parallel mode hand-off slots (labs workgroup <-> vitals+head workgroup of one client)
constexpr long W_XF = W_DX3V + BM * 64;  // branch outputs, bf16 [2][128][64] (vitals, labs)
constexpr long W_XB = W_XF + 2 * BM * 32;  // d(branch outputs), bf16 [128][64] in fp32-sized slots [2][128][64]
constexpr long WS_FLOATS = W_XB + 2 * BM * 64;

struct TfLayout {
  static constexpr int S_ACC = ::S_ACC, LDACC = ::LDACC, S_CS = ::S_CS;
};
using Ctx = CtxT<TfLayout>;

template <int BR>
struct BrC {
  static constexpr BrOff o = BR == 0 ? OV : OL;
  static constexpr BrW w = BR == 0 ? WBV : WBL;
  static constexpr BrS s = BR == 0 ? SV : SL;
  static constexpr int din = BR == 0 ? D_V : D_L;
  static constexpr int xoff = BR == 0 ? 0 : D_V;
  static constexpr MatW dense{o.dense_w, 64, din, w.WFd, 32, -1, 0};
  static constexpr MatW vproj{o.inproj_w + 128 * 64, 64, 64, w.WFv, 64, w.WTv, 64};
  static constexpr MatW oproj{o.out_w, 64, 64, w.WFo, 64, w.WTo, 64};
  static constexpr MatW ff0{o.ff0_w, FF, 64, w.WF1, 64, w.WT1, 32};
  static constexpr MatW ff3{o.ff3_w, 64, FF, w.WF2, 32, w.WT2, 64};
};
constexpr MatW MFC1{FC1_W, 64, 128, WFF1, 128, WTF1, 64};
constexpr MatW MFC2{FC2_W, 32, 64, WFF2, 64, WTF2, 32};

// per-step, per-thread state (row-per-4-lanes layout)
struct St {
  bool valid;     // r < Bn
  int ridx;       // train row index
  int Bn;
  uint32_t key;   // dropout key of this step
  AdamK K;
  const gf* rows;
  float xin[2][8];  // this lane's 8 input columns of both branches (loaded at step start)
};

// per-phase wall-clock stamps (s_memrealtime, 100 MHz) of ONE workgroup (index in stamps[63]),
// accumulated over all steps; only when the caller passes a stamps buffer (diagnostics; one uniform
// branch per phase otherwise)
#define stamp_block ((unsigned)stamps[63])
#define STAMP(id)                                                                   \
  do {                                                                              \
    if (stamps && blockIdx.x == stamp_block && threadIdx.x == 0) {                 \
      uint64_t now_ = __builtin_amdgcn_s_memrealtime();                            \
      stamps[id] += now_ - t_prev;                                                  \
      t_prev = now_;                                                                \
    }                                                                               \
  } while (0)

#define BAR()          \
  do {                 \
    c.bar();           \
    r = c.r;           \
    q = c.q;           \
    c0 = q * 16;       \
  } while (0)
// wave-local boundary (Ctx::soft): the next phase reads only LDS rows this wave wrote
#define WBAR()         \
  do {                 \
    c.soft();          \
    r = c.r;           \
    q = c.q;           \
    c0 = q * 16;       \
  } while (0)

// inputs of one branch -> XIN (bf16, K padded to 32)
template <int BR>
__device__ __forceinline__ void put_x(const Ctx& c, const St& s) {
  unsigned short* XIN = c.u16(S_XIN);
  s8v v;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (short)f2bf(s.xin[BR][j]);
  *(LDS_AS s8v*)(XIN + c.r * LD32 + c.q * 8) = v;
}

// ============================================================== branch forward
// XCH: publish the branch output to the hand-off slot W_XF (write-through stores) instead of LDS CAT,
// each wave its own rows with its own flag xf(xflag, BR, wave) = pub_val; the backward's saved
// activations of the last phase are stored only after the flag, so the publish drain (vmcnt 0) waits
// for the payload, not for them too
template <int BR, bool XCH = false>
__device__ __forceinline__ void fwd_branch(Ctx& c, St& s, uint64_t* stamps, uint64_t& t_prev, gu32* xflag = nullptr,
                                           uint32_t pub_val = 0) {
  using B = BrC<BR>;
  unsigned short* XIN = c.u16(S_XIN);
  unsigned short* TA = c.u16(S_TA);
  unsigned short* TB = c.u16(S_TB);
  unsigned short* TC = c.u16(S_TC);
  unsigned short* CAT = c.u16(S_CAT);
  unsigned short* F2 = c.u16(S_F2);
  float* ACC = c.acc();
  int r = c.r, q = c.q, c0 = q * 16;
  // Parameter loads of each elementwise phase are issued BEFORE the workspace stores of the phases in
  // front of it (loads and stores share one vmcnt queue, so a load behind stores waits for their acks)
  WFr<64, 32> wd;
  if (XCH) {  // branch-only workgroup: the LDS image the last dWd epilogue wrote
#pragma unroll
    for (int t = 0; t < 4; ++t) wd.f[t][0] = lds_row_frag(c.u16(S_WDI), LDW, 16 * t, 0, c.lane);
  } else {
    wload(wd, c.BF + B::w.WFd, c.lane);
  }
  float bias[16], bias_v[16];
  load16(bias, c.P + B::o.dense_b + c0);
  load16(bias_v, c.P + B::o.inproj_b + 128 + c0);
  put_x<BR>(c, s);
  WBAR();
  gemm_pf<64, 32>(c, XIN, LD32, wd);
  WFr<64, 64> wv;
  wload(wv, c.BF + B::w.WFv, c.lane);
  float bias_o[16], g1[16], b1[16];
  load16(bias_o, c.P + B::o.out_b + c0);
  load16(g1, c.P + B::o.ln1_w + c0);
  load16(b1, c.P + B::o.ln1_b + c0);
  WBAR();
  STAMP(0);
  float h[16];  // h0 stays in registers until the residual (E3)
  {
    float gp[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) h[j] = gelu_and_grad(ACC[r * LDACC + c0 + j] + bias[j], gp[j]);
    store16bf(TA + r * LD64 + c0, h);
    store16(c.wsf(B::s.GPD) + opaque(r * 64 + c0), gp);
    gu16* hb = (gu16*)c.wsf(B::s.H0B) + opaque(r * 64 + c0);
    s8v a, b;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      a[j] = (short)f2bf(h[j]);
      b[j] = (short)f2bf(h[j + 8]);
    }
    *(GAS s8v*)hb = a;
    *(GAS s8v*)(hb + 8) = b;
  }
  WBAR();
  gemm_pf<64, 64>(c, TA, LD64, wv);
  WFr<64, 64> wo;
  wload(wo, c.BF + B::w.WFo, c.lane);
  WBAR();
  STAMP(1);
  {  // E2: a = head_dropout(v) (-> TB, and kept in the workspace for dWo)
    float x[16];
    const float m = keep(s.key, 8 * BR + L_ATT, r, q, THR_P01) ? INV_K01 : 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) x[j] = (ACC[r * LDACC + c0 + j] + bias_v[j]) * m;
    store16bf(TB + r * LD64 + c0, x);
    gu16* ab = (gu16*)c.wsf(B::s.AB) + opaque(r * 64 + c0);
    *(GAS s8v*)ab = pack8bf(x);
    *(GAS s8v*)(ab + 8) = pack8bf(x + 8);
  }
  float fb[8];
  load8(fb, c.P + B::o.ff0_b);  // 6 used (+2 beyond: next tensor, ignored)
  WBAR();
  gemm_pf<64, 64>(c, TB, LD64, wo);
  WFr<16, 64> w1;
  wload(w1, c.BF + B::w.WF1, c.lane);
  WBAR();
  STAMP(2);
  float x1[16];  // x1 stays in registers until the second residual (E5)
  {
    const int ro = opaque(r * 64 + c0);
    const uint32_t m1 = keep_bits<16>(s.key, 8 * BR + L_D1, r, c0, THR_P01);
    ((gu32*)c.wsf(B::s.MK))[opaque(r * 16 + q * 4) + 0] = m1;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const float o = ACC[r * LDACC + c0 + j] + bias_o[j];
      x1[j] = h[j] + (bit(m1, j) ? o * INV_K01 : 0.f);
    }
    const float rstd = ln_fwd(x1);
    store16(c.wsf(B::s.XH1) + ro, x1);
    c.wsf(B::s.RS)[opaque(r * 16 + q * 4) + 0] = rstd;
#pragma unroll
    for (int j = 0; j < 16; ++j) x1[j] = x1[j] * g1[j] + b1[j];
    store16bf(TC + r * LD64 + c0, x1);
  }
  WBAR();
  gemm_pf<16, 64>(c, TC, LD64, w1);
  WFr<64, 32> w2;
  wload(w2, c.BF + B::w.WF2, c.lane);
  WBAR();
  STAMP(3);
  float g2[16], bb2[16], g3[16], b3[16];
  load16(bias, c.P + B::o.ff3_b + c0);
  load16(g2, c.P + B::o.ln2_w + c0);
  load16(bb2, c.P + B::o.ln2_b + c0);
  load16(g3, c.P + B::o.bn_w + c0);
  load16(b3, c.P + B::o.bn_b + c0);
  {  // E4: f0 -> f2 (the FF <= 8 real columns live in quarter 0)
    static_assert(FF <= 8, "E4 keeps the ffn width in one quarter");
    s8v v;
    const uint32_t mf = q == 0 ? keep_bits<8>(s.key, 8 * BR + L_DF, r, 0, THR_P01) : 0u;
    float f0s[8], f2s[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float f2 = 0.f, f0 = 0.f;
      if (q == 0 && j < FF) {
        float gp;
        const float g = gelu_and_grad(ACC[r * LDACC + j] + fb[j], gp);
        const bool kp = bit(mf, j);
        f2 = kp ? g * INV_K01 : 0.f;
        f0 = kp ? gp * INV_K01 : 0.f;
      }
      f0s[j] = f0;
      f2s[j] = f2;
      v[j] = (short)f2bf(f2);
    }
    if (q == 0) {  // [128][8] rows, two 16-byte stores each (not FF scalar ones: fewer ops for the drain)
      gf* f0p = c.wsf(B::s.F0) + opaque(r * 8);
      gf* f2p = c.wsf(B::s.F2S) + opaque(r * 8);
      *(GAS f4v*)f0p = f4v{f0s[0], f0s[1], f0s[2], f0s[3]};
      *(GAS f4v*)(f0p + 4) = f4v{f0s[4], f0s[5], f0s[6], f0s[7]};
      *(GAS f4v*)f2p = f4v{f2s[0], f2s[1], f2s[2], f2s[3]};
      *(GAS f4v*)(f2p + 4) = f4v{f2s[4], f2s[5], f2s[6], f2s[7]};
    }
    *(LDS_AS s8v*)(F2 + r * LD32 + q * 8) = v;
  }
  WBAR();
  gemm_pf<64, 32>(c, F2, LD32, w2);
  WBAR();
  STAMP(4);
  {  // E5: r2 = x1 + drop(f3); LN2; LN3 -> CAT
    const int ro = opaque(r * 64 + c0);
    float x[16], xh2[16], xh3[16];
    const uint32_t m2 = keep_bits<16>(s.key, 8 * BR + L_D2, r, c0, THR_P01);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const float f3 = ACC[r * LDACC + c0 + j] + bias[j];
      xh2[j] = x1[j] + (bit(m2, j) ? f3 * INV_K01 : 0.f);
    }
    const float rstd2 = ln_fwd(xh2);
#pragma unroll
    for (int j = 0; j < 16; ++j) xh3[j] = xh2[j] * g2[j] + bb2[j];
    const float rstd3 = ln_fwd(xh3);
#pragma unroll
    for (int j = 0; j < 16; ++j) x[j] = xh3[j] * g3[j] + b3[j];
    if (XCH) {
      const int bo = (int)(W_XF + BR * BM * 32) * 4 + ro * 2;
      st_wt16(c, bo, __builtin_bit_cast(u32x4, pack8bf(x)));
      st_wt16(c, bo + 16, __builtin_bit_cast(u32x4, pack8bf(x + 8)));
      wave_publish(c, xf(xflag, BR, c.wave), pub_val);
    } else {
      store16bf(CAT + r * LD128 + BR * 64 + c0, x);
    }
    ((gu32*)c.wsf(B::s.MK))[opaque(r * 16 + q * 4) + 2] = m2;
    store16(c.wsf(B::s.XH2) + ro, xh2);
    store16(c.wsf(B::s.XH3) + ro, xh3);
    gf* rs = c.wsf(B::s.RS) + opaque(r * 16 + q * 4);
    rs[1] = rstd2;
    rs[2] = rstd3;
  }
  BAR();
  STAMP(5);
}

// ============================================================== branch backward
// Everything the first backward phase reads that does NOT depend on d(output): this lane's saved
// forward values, the LayerNorm affines, the W2 fragments.  A branch-only workgroup issues these loads
// BEFORE it waits for the head's gradient hand-off, so their latency overlaps the wait.
struct BwdPre {
  float xh3[16], xh2[16], gm3[16], gm2[16];
  float rstd2, rstd3;
  uint32_t m2;
  float gk[8], f2s[8];  // drop'(.) * gelu'(f0) and f2 of the forward
  WFr<16, 64> wt2;
  bool abort = false;  // DY == 2: this wave's d(output) flag carried the head's NaN abort
};
template <int BR>
__device__ __forceinline__ void bwd_prefetch(const Ctx& c, BwdPre& p) {
  using B = BrC<BR>;
  const int r = c.r, q = c.q, c0 = q * 16;
  const int ro = opaque(r * 64 + c0);
  wload(p.wt2, c.BF + B::w.WT2, c.lane);
  load16(p.xh3, c.wsf(B::s.XH3) + ro);
  load16(p.xh2, c.wsf(B::s.XH2) + ro);
  load16(p.gm3, c.P + B::o.bn_w + c0);
  load16(p.gm2, c.P + B::o.ln2_w + c0);
  const gf* rs = c.wsf(B::s.RS) + opaque(r * 16 + q * 4);
  p.rstd2 = rs[1];
  p.rstd3 = rs[2];
  p.m2 = ((const gu32*)c.wsf(B::s.MK))[opaque(r * 16 + q * 4) + 2];
  load8(p.gk, c.wsf(B::s.F0) + opaque(r * 8));
  load8(p.f2s, c.wsf(B::s.F2S) + opaque(r * 8));
}

// on entry: dx3 of this branch in ACC (DY == 0), the DX3V workspace (DY == 1) or the hand-off slot W_XB
// (DY == 2, branch-parallel mode, after the acquire); p from bwd_prefetch<BR>
// Returns true when the step is aborted (DY == 2: some wave's hand-off flag carried the head's NaN
// abort -- the head raises it per wave, from that wave's rows; the OR is taken at the first barrier,
// before anything is written outside LDS, so an aborted client keeps its pre-step parameters).
template <int BR, int DY>
__device__ __forceinline__ bool bwd_branch(Ctx& c, St& s, uint64_t* stamps, uint64_t& t_prev, const BwdPre& p) {
  using B = BrC<BR>;
  unsigned short* XIN = c.u16(S_XIN);  // also DF0
  unsigned short* TA = c.u16(S_TA);
  unsigned short* TB = c.u16(S_TB);
  unsigned short* TC = c.u16(S_TC);
  unsigned short* TD = c.u16(S_CAT);  // [128][72] alias of CAT (dead after dWf1)
  unsigned short* F2 = c.u16(S_F2);
  float* ACC = c.acc();
  int r = c.r, q = c.q, c0 = q * 16;
  const AdamK K = s.K;
  float dr2[16];  // residual gradient into x1, kept in registers until E12
  const WFr<16, 64>& wt2 = p.wt2;
  {  // E10: LN3 bwd, LN2 bwd, df3 ; colsums g3 (v0), b3 (v1), g2 (v2), be2 (v3), b2 (v4)
    const int ro = opaque(r * 64 + c0);
    float dy[16], dx[16], t[16];
    const float(&xh3)[16] = p.xh3;
    const float(&xh2)[16] = p.xh2;
    const float(&gm3)[16] = p.gm3;
    const float(&gm2)[16] = p.gm2;
    const float rstd2 = p.rstd2, rstd3 = p.rstd3;
    const uint32_t m2 = p.m2;
    if (DY == 0) {
#pragma unroll
      for (int j = 0; j < 16; ++j) dy[j] = ACC[r * LDACC + c0 + j];
    } else if (DY == 1) {
      load16(dy, c.wsf(W_DX3V) + ro);
    } else {  // hand-off slot written by the other workgroup: write-through granules, sc1 loads
      const int bo = (int)(W_XB + BR * BM * 64) * 4 + ro * 2;  // bf16 [128][64] (put_grad)
      unpack8bf(ld_wt16(c, bo), dy);
      unpack8bf(ld_wt16(c, bo + 16), dy + 8);
    }
    if (DY != 2) {  // same values as the bf16 hand-off of the branch-parallel launches
#pragma unroll
      for (int j = 0; j < 16; ++j) dy[j] = bf2f(f2bf(dy[j]));
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) t[j] = dy[j] * xh3[j];
    colsum16(c, 0, t);
    colsum16(c, 1, dy);
    ln_bwd(dx, dy, xh3, rstd3, gm3);
#pragma unroll
    for (int j = 0; j < 16; ++j) t[j] = dx[j] * xh2[j];
    colsum16(c, 2, t);
    colsum16(c, 3, dx);
    ln_bwd(dr2, dx, xh2, rstd2, gm2);
#pragma unroll
    for (int j = 0; j < 16; ++j) t[j] = bit(m2, j) ? dr2[j] * INV_K01 : 0.f;
    store16bf(TA + r * LD64 + c0, t);
    colsum16(c, 4, t);
  }
  const float(&gk)[8] = p.gk;  // drop'(.) * gelu'(f0) and f2 of the forward
  const float(&f2s)[8] = p.f2s;
  uint32_t* abort_w = (uint32_t*)(c.smem + S_RED) + 8;  // one word per wave (RED is head-only)
  if (DY == 2 && c.lane == 0) abort_w[c.wave] = p.abort ? 1u : 0u;
  BAR();
  if (DY == 2) {
    uint32_t any = 0;
#pragma unroll
    for (int w = 0; w < 8; ++w) any |= abort_w[w];
    if (any) return true;
  }
  STAMP(10);
  // A10 + G11 (df2 = df3 . W2).  Every phase below issues its global loads (Adam state, the next
  // GEMM's weights, saved activations) BEFORE its Adam stores: they share one vmcnt queue (dw_ld)
  const VecG v10[5] = {{B::o.bn_w, 64, 0}, {B::o.bn_b, 64, 1}, {B::o.ln2_w, 64, 2}, {B::o.ln2_b, 64, 3},
                       {B::o.ff3_b, 64, 4}};
  const AdamS s10 = adam_vecs_ld(c, v10);
  WFr<64, 32> wt1;
  wload(wt1, c.BF + B::w.WT1, c.lane);
  float xh1[16], gm1[16], bt1[16];  // for E12
  {
    const int ro = opaque(r * 64 + c0);
    load16(xh1, c.wsf(B::s.XH1) + ro);
    load16(gm1, c.P + B::o.ln1_w + c0);
    load16(bt1, c.P + B::o.ln1_b + c0);
  }
  const float rstd1 = c.wsf(B::s.RS)[opaque(r * 16 + q * 4)];
  const uint32_t m1 = ((const gu32*)c.wsf(B::s.MK))[opaque(r * 16 + q * 4) + 0];
  gemm_pf<16, 64>(c, TA, LD64, wt2);
  adam_vecs_st(c, v10, s10, K);
  WBAR();
  STAMP(11);
  {  // E11: df0 (-> DF0 = XIN region), f2 (-> F2); colsum b1 (v5)
    s8v vd, vf;
    float db[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int col = q * 8 + j;
      float d0 = 0.f, f2 = 0.f;
      if (col < FF) {
        d0 = ACC[r * LDACC + col] * gk[j];
        f2 = f2s[j];
      }
      db[j] = d0;
      vd[j] = (short)f2bf(d0);
      vf[j] = (short)f2bf(f2);
    }
    *(LDS_AS s8v*)(XIN + r * LD32 + q * 8) = vd;
    *(LDS_AS s8v*)(F2 + r * LD32 + q * 8) = vf;
    colsumW<8>(c, 5, db, q * 8);
  }
  BAR();
  STAMP(12);
  DwS<4, 1> s2;
  dw_ld<4, 1>(c, B::ff3, s2);
  AdamS sb1{};
  if (c.tid < FF) sb1 = adam_ld(c, B::o.ff0_b + c.tid);
  WFr<64, 64> wto;
  wload(wto, c.BF + B::w.WTo, c.lane);
  s8v h0a, h0b, aa, ab;  // for E13
  {
    const gu16* hb = (const gu16*)c.wsf(B::s.H0B) + opaque(r * 64 + c0);
    h0a = *(const GAS s8v*)hb;
    h0b = *(const GAS s8v*)(hb + 8);
    const gu16* abp = (const gu16*)c.wsf(B::s.AB) + opaque(r * 64 + c0);
    aa = *(const GAS s8v*)abp;
    ab = *(const GAS s8v*)(abp + 8);
  }
  gemm_pf<64, 32>(c, XIN, LD32, wt1);                 // dx1 = df0 . W1 (reads WT1 copy: before W1's Adam)
  dw_apply<4, 1>(c, TA, LD64, F2, LD32, B::ff3, K, s2);  // dW2 = df3^T f2
  if (c.tid < FF) adam_st(c, B::o.ff0_b + c.tid, sb1, cs_total(c, 5, c.tid), K);
  WBAR();
  STAMP(13);
  float dh0[16];  // residual gradient into h0, kept in registers until E15
  {  // E12: dx1 += dr2 ; LN1 bwd ; do ; x1 recompute ; colsums g1 (v0), be1 (v1), bo (v2)
    float dx[16], t[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) dx[j] = ACC[r * LDACC + c0 + j] + dr2[j];
#pragma unroll
    for (int j = 0; j < 16; ++j) t[j] = dx[j] * xh1[j];
    colsum16(c, 0, t);
    colsum16(c, 1, dx);
    ln_bwd(dh0, dx, xh1, rstd1, gm1);
#pragma unroll
    for (int j = 0; j < 16; ++j) t[j] = bit(m1, j) ? dh0[j] * INV_K01 : 0.f;
    store16bf(TB + r * LD64 + c0, t);
    colsum16(c, 2, t);
#pragma unroll
    for (int j = 0; j < 16; ++j) t[j] = xh1[j] * gm1[j] + bt1[j];
    store16bf(TC + r * LD64 + c0, t);
  }
  BAR();
  STAMP(14);
  DwS<1, 4> s1;
  dw_ld<1, 4>(c, B::ff0, s1);
  const VecG v14[3] = {{B::o.ln1_w, 64, 0}, {B::o.ln1_b, 64, 1}, {B::o.out_b, 64, 2}};
  const AdamS s14 = adam_vecs_ld(c, v14);
  WFr<64, 64> wtv;
  wload(wtv, c.BF + B::w.WTv, c.lane);
  gemm_pf<64, 64>(c, TB, LD64, wto);                      // da = do . Wo
  dw_apply<1, 4>(c, XIN, LD32, TC, LD64, B::ff0, K, s1);  // dW1 = df0^T x1
  adam_vecs_st(c, v14, s14, K);
  BAR();
  STAMP(15);
  {  // E13: dv (-> TC) ; h0 (-> TA) ; a (-> TD) ; colsum bv (v3)
    float d[16];
    const float m = keep(s.key, 8 * BR + L_ATT, r, q, THR_P01) ? INV_K01 : 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) d[j] = ACC[r * LDACC + c0 + j] * m;
    store16bf(TC + r * LD64 + c0, d);
    colsum16(c, 3, d);
    *(LDS_AS s8v*)(TA + r * LD64 + c0) = h0a;
    *(LDS_AS s8v*)(TA + r * LD64 + c0 + 8) = h0b;
    *(LDS_AS s8v*)(TD + r * LD64 + c0) = aa;
    *(LDS_AS s8v*)(TD + r * LD64 + c0 + 8) = ab;
  }
  BAR();
  STAMP(16);
  STAMP(17);
  DwS<4, 4> so;
  dw_ld<4, 4>(c, B::oproj, so);
  AdamS sbv{};
  if (c.tid < 64) sbv = adam_ld(c, B::o.inproj_b + 128 + c.tid);
  float gpd[16];  // gelu'(z0) of the forward
  load16(gpd, c.wsf(B::s.GPD) + opaque(r * 64 + c0));
  DwS<4, 4> sv;  // for dWv below
  dw_ld<4, 4>(c, B::vproj, sv);
  gemm_pf<64, 64>(c, TC, LD64, wtv);                          // dh0 part = dv . Wv
  dw_apply<4, 4>(c, TB, LD64, TD, LD64, B::oproj, K, so);  // dWo = do^T a
  if (c.tid < 64) adam_st(c, B::o.inproj_b + 128 + c.tid, sbv, cs_total(c, 3, c.tid), K);
  WBAR();
  STAMP(18);
  {  // E14: dh0 += ACC ; x for dWd
#pragma unroll
    for (int j = 0; j < 16; ++j) dh0[j] += ACC[r * LDACC + c0 + j];
    put_x<BR>(c, s);
  }
  WBAR();
  DwS<4, 1> sd;  // for dWd below
  dw_ld<4, 1>(c, B::dense, sd);
  AdamS sbd{};
  if (c.tid < 64) sbd = adam_ld(c, B::o.dense_b + c.tid);
  dw_apply<4, 4>(c, TC, LD64, TA, LD64, B::vproj, K, sv);  // dWv = dv^T h0
  BAR();
  STAMP(19);
  {  // E15: dz0 = dh0 * gelu'(z0) ; colsum bd (v4)
    float d[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) d[j] = dh0[j] * gpd[j];
    store16bf(TB + r * LD64 + c0, d);
    colsum16(c, 4, d);
  }
  BAR();
  // dWd = dz0^T x (branch-only workgroups also refresh the LDS image the next forward reads)
  dw_apply<4, 1>(c, TB, LD64, XIN, LD32, B::dense, K, sd, DY == 2 ? c.u16(S_WDI) : nullptr, LDW);
  if (c.tid < 64) adam_st(c, B::o.dense_b + c.tid, sbd, cs_total(c, 4, c.tid), K);
  BAR();
  STAMP(20);
  return false;
}

}  // namespace

template <int BR>
__device__ void init_copies_branch(const Ctx& c) {
  init_copies(c, BrC<BR>::dense);
  init_copies(c, BrC<BR>::vproj);
  init_copies(c, BrC<BR>::oproj);
  init_copies(c, BrC<BR>::ff0);
  init_copies(c, BrC<BR>::ff3);
}

__device__ void init_copies_all(const Ctx& c) {
  init_copies(c, BrC<0>::dense);
  init_copies(c, BrC<0>::vproj);
  init_copies(c, BrC<0>::oproj);
  init_copies(c, BrC<0>::ff0);
  init_copies(c, BrC<0>::ff3);
  init_copies(c, BrC<1>::dense);
  init_copies(c, BrC<1>::vproj);
  init_copies(c, BrC<1>::oproj);
  init_copies(c, BrC<1>::ff0);
  init_copies(c, BrC<1>::ff3);
  init_copies(c, MFC1);
  init_copies(c, MFC2);
}

// ROLE -1: the whole model in one workgroup per client.  Branch-parallel modes (co-resident
// workgroups per client exchanging activations / gradients every step through hand-off slots):
//   2 workgroups: ROLE 0 = vitals branch + head, ROLE 1 = labs branch;
//   3 workgroups: ROLE 2 = vitals branch, ROLE 1 = labs branch, ROLE 3 = head.
// Every wave of a branch-only workgroup publishes its output rows (flags XF_VIT / XF_LAB, one per
// wave) and waits for its rows of d(output) (XF_BVIT / XF_BLAB, which also carry the NaN abort); the
// head publishes the gradients BEFORE its own dWf1 update (and, in the 2-workgroup mode, before the
// vitals backward) so they overlap.
template <int ROLE>
__device__ __forceinline__ void train_body(const AflTfTrainArgs& a, int cid, unsigned char* smem) {
  constexpr bool DO0 = ROLE == -1 || ROLE == 0 || ROLE == 2;
  constexpr bool DO1 = ROLE == -1 || ROLE == 1;
  constexpr bool HEAD = ROLE == -1 || ROLE == 0 || ROLE == 3;
  constexpr int BONLY = ROLE == 1 ? 1 : (ROLE == 2 ? 0 : -1);  // branch of a branch-only workgroup
  Ctx c;
  c.smem = smem;
  c.P = (gf*)(a.params + (long)cid * NPARAM);
  c.ws = (gf*)(a.ws + (long)cid * a.ws_stride);
  c.M = c.ws + W_M;
  c.V = c.ws + W_V;
  c.BF = (gu16*)(c.ws + W_BF);
  c.tid = threadIdx.x;
  c.lane = threadIdx.x & 63;
  c.wave = threadIdx.x >> 6;
  c.r = 16 * (threadIdx.x >> 6) + (threadIdx.x & 15);  // row: 16 consecutive lanes per quarter
  c.q = (threadIdx.x >> 4) & 3;                         // quarter of the row (16 columns)
  const int tid = c.tid;
  uint64_t* stamps = a.stamps;
  uint64_t t_prev = 0;
  if (stamps && blockIdx.x == stamp_block && threadIdx.x == 0) t_prev = __builtin_amdgcn_s_memrealtime();

  // ---- init: zero Adam moments, bf16 weight copies (padding zeroed first), LDS ----
  {  // parameter / copy ranges owned by this workgroup: vitals, labs, head
    const int pr[4] = {0, OV.size, FC1_W, NPARAM};
    const int br[4] = {0, BRW_SIZE, 2 * BRW_SIZE, BF_TOTAL};
    const bool own[3] = {DO0, DO1, HEAD};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      if (!own[k]) continue;
      for (int i = pr[k] + tid; i < pr[k + 1]; i += NT) {
        c.M[i] = 0.f;
        c.V[i] = 0.f;
      }
      for (int i = br[k] + tid; i < br[k + 1]; i += NT) c.BF[i] = 0;
    }
  }
  for (int i = tid; i < S_TOTAL / 4; i += NT) ((float*)smem)[i] = 0.f;
  __syncthreads();
  if (DO0) init_copies_branch<0>(c);
  if (DO1) init_copies_branch<1>(c);
  if (HEAD) {
    init_copies(c, MFC1);
    init_copies(c, MFC2);
  }
  __syncthreads();
  if (BONLY >= 0) {  // the dense weight's LDS image (see S_WDI), from the bf16 copy just written
    constexpr int WFD = BrC<BONLY < 0 ? 0 : BONLY>::w.WFd;
    for (int i = tid; i < 64 * 32; i += NT) c.u16(S_WDI)[(i >> 5) * LDW + (i & 31)] = c.BF[WFD + i];
    __syncthreads();
  }
  gu32* xflag = (gu32*)(a.sync ? a.sync + (long)cid * AFL_TF_SYNC_WORDS : nullptr);  // XF_* words
  bool timed_out = false;

  const int nd = a.nd[cid];
  const int BS = a.batch;
  const int nb_total = (nd + BS - 1) / BS;
  const uint32_t seed = a.seeds[cid];
  double b1t = 1.0, b2t = 1.0;
  int step = 0;
  bool failed = false;
  float* LAB = (float*)(smem + S_LAB);
  float* DY3 = (float*)(smem + S_DY3);
  float* RED = (float*)(smem + S_RED);
  unsigned short* TA = c.u16(S_TA);
  unsigned short* TB = c.u16(S_TB);
  unsigned short* CAT = c.u16(S_CAT);
  unsigned short* F2 = c.u16(S_F2);
  float* ACC = c.acc();
  St s;
  s.rows = (const gf*)a.rows;
  int r = c.r, q = c.q, c0 = q * 16;
  bool have_next = false;  // inputs of the next step prefetched (branch-only workgroups)
  int ridx_next = 0;
  float xin_next[2][8];

  for (int e = 0; e < a.E && !failed; ++e) {
    const gi32* ord = (const gi32*)(a.order + ((long)cid * a.E + e) * a.maxnd);
    float epoch_loss = 0.f;
    for (int b0 = 0; b0 < nd; b0 += BS) {
      const int Bn = min(BS, nd - b0);
      if (Bn == 1) continue;  // reference skips size-1 batches (client.py:86-87)
      ++step;
      b1t *= (double)B1;
      b2t *= (double)B2;
      s.K = AdamK{(float)((double)a.lr / (1.0 - b1t)), (float)(1.0 / sqrt(1.0 - b2t)), a.opt_mode == 1 ? a.lr : 0.f};
      s.key = afl_hash32(seed, (uint32_t)step);
      s.Bn = Bn;
      r = c.r;
      q = c.q;
      s.valid = r < Bn;
      if (have_next) {  // a branch-only workgroup loaded this step's inputs while it waited for the head
        s.ridx = ridx_next;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          s.xin[0][j] = xin_next[0][j];
          s.xin[1][j] = xin_next[1][j];
        }
        have_next = false;
      } else {
        s.ridx = s.valid ? ord[b0 + r] : 0;
        // both branches' input columns and the label, loaded once per step
        const gf* row = s.rows + (long)s.ridx * ROW;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int col = q * 8 + j;
          s.xin[0][j] = (DO0 && s.valid && col < D_V) ? row[col] : 0.f;
          s.xin[1][j] = (DO1 && s.valid && col < D_L) ? row[D_V + col] : 0.f;
        }
        if (HEAD && q == 0) LAB[r] = s.valid ? row[ROW - 1] : 0.f;
      }
      const AdamK K = s.K;

      if (ROLE == -1 || ROLE == 0) fwd_branch<0>(c, s, stamps, t_prev);
      if (ROLE == -1) fwd_branch<1>(c, s, stamps, t_prev);
      if (BONLY >= 0) {  // branch-only workgroup: forward, hand-off, wait, backward
        fwd_branch<BONLY < 0 ? 0 : BONLY, true>(c, s, stamps, t_prev, xflag, (uint32_t)step);
        BwdPre pre;  // issued before the wait: the loads complete while the head works
        bwd_prefetch<BONLY < 0 ? 0 : BONLY>(c, pre);
        {  // the NEXT step's input rows too (two dependent loads: row index, then the row)
          int en = e, bn = b0 + BS;
          for (;;) {  // same walk as the loops: next batch, skipping size-1 batches
            if (bn >= nd) {
              ++en;
              bn = 0;
              if (en >= a.E) break;
              continue;
            }
            if (min(BS, nd - bn) == 1) {
              bn += BS;
              continue;
            }
            break;
          }
          if (en < a.E) {
            const gi32* ordn = (const gi32*)(a.order + ((long)cid * a.E + en) * a.maxnd);
            const bool vn = r < min(BS, nd - bn);
            ridx_next = vn ? ordn[bn + r] : 0;
            const gf* row = s.rows + (long)ridx_next * ROW;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              const int col = q * 8 + j;
              xin_next[0][j] = (DO0 && vn && col < D_V) ? row[col] : 0.f;
              xin_next[1][j] = (DO1 && vn && col < D_L) ? row[D_V + col] : 0.f;
            }
            have_next = true;
          }
        }
        gu32* fb = xf(xflag, BONLY == 1 ? XF_BLAB : XF_BVIT, c.wave);  // this wave's rows of d(output)
        const uint32_t v = wave_wait(c, fb, fb, (uint32_t)step, 1, xflag + XF_TMO);
        if (v == 0xFFFFFFFFu) {
          timed_out = true;
          failed = true;
          break;
        }
        pre.abort = (v & 1u) != 0;  // the head saw a NaN in this wave's rows
        STAMP(21);
        if (bwd_branch<BONLY < 0 ? 0 : BONLY, 2>(c, s, stamps, t_prev, pre)) {  // the client's round fails
          failed = true;
          break;
        }
        c.full_sync();
        continue;
      }
      // fc1 weight fragments and bias are issued BEFORE the wait for the branch outputs: their global
      // latency overlaps the wait instead of sitting on the critical path after it
      WFr<64, 128> wf1;
      wload(wf1, c.BF + WFF1, c.lane);
      WFr<32, 64> wf2;  // and the next two GEMMs' (small) fragments; the two dcat halves' are issued as
      wload(wf2, c.BF + WFF2, c.lane);  // soon as fc1 / fc2 free their registers, so no load of them
      WFr<64, 32> wtf2;                 // sits behind the gradient hand-off's drain
      wload(wtf2, c.BF + WTF2, c.lane);
      float bias[16];
      load16(bias, c.P + FC1_B + q * 16);
      if (ROLE == 0 || ROLE == 3) {  // branch outputs from the other workgroup(s) -> CAT
        // this wave's CAT rows: its own flags, no workgroup barrier
        const uint32_t v = wave_wait(c, xf(xflag, ROLE == 3 ? XF_VIT : XF_LAB, c.wave), xf(xflag, XF_LAB, c.wave),
                                     (uint32_t)step, 0, xflag + XF_TMO);
        if (v == 0xFFFFFFFFu) {
          timed_out = true;
          failed = true;
          break;
        }
#pragma unroll
        for (int br = ROLE == 3 ? 0 : 1; br < 2; ++br) {
          const int bo = (int)(W_XF + br * BM * 32) * 4 + opaque(r * 64 + c0) * 2;
          const u32x4 lo = ld_wt16(c, bo), hi = ld_wt16(c, bo + 16);
          *(LDS_AS s8v*)(CAT + r * LD128 + br * 64 + c0) = __builtin_bit_cast(s8v, lo);
          *(LDS_AS s8v*)(CAT + r * LD128 + br * 64 + c0 + 8) = __builtin_bit_cast(s8v, hi);
        }
        WBAR();
      }
      // =============================== head forward + loss ===============================
      gemm_pf<64, 128>(c, CAT, LD128, wf1);
      WFr<64, 64> wtf1a;
      wload(wtf1a, c.BF + WTF1, c.lane);
      WBAR();
      STAMP(6);
      float gk1[16];  // drop'(.) * gelu'(y1), kept in registers until E8
      {               // E6: y1 -> d1 = drop0.3(gelu(y1))
        float x[16];
        const uint32_t mh = keep_bits<16>(s.key, L_HEAD, r, c0, THR_P03);
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          float gp;
          const float g = gelu_and_grad(ACC[r * LDACC + c0 + j] + bias[j], gp);
          x[j] = bit(mh, j) ? g * INV_K03 : 0.f;
          gk1[j] = bit(mh, j) ? gp * INV_K03 : 0.f;
        }
        store16bf(TA + r * LD64 + c0, x);
      }
      float b2v[8], wov[8];
      load8(b2v, c.P + FC2_B + q * 8);
      load8(wov, c.P + OUT_W + q * 8);
      const float bout = c.P[OUT_B];
      WBAR();
      gemm_pf<32, 64>(c, TA, LD64, wf2);
      WFr<64, 64> wtf1b;
      wload(wtf1b, c.BF + WTF1 + 64 * 64, c.lane);
      WBAR();
      STAMP(7);
      uint32_t wave_nan = 0;  // this wave's rows produced a NaN loss term
      {  // E7: y2, g2, y3, sigmoid, BCE, dy3, dy2 ; colsums dWout (v0), dbf2 (v1)
        float gp2[8], g2[8], dot = 0.f;
        const int cc = q * 8;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          g2[j] = gelu_and_grad(ACC[r * LDACC + cc + j] + b2v[j], gp2[j]);
          dot += g2[j] * wov[j];
        }
        const float y3 = rsum4(dot) + bout;
        const float p = sigmoidf_(y3);
        const float lab = LAB[r];
        float lrow = 0.f, dy3 = 0.f;
        if (s.valid) {
          // clamp like torch.clamp: NaN must propagate (fmaxf would swallow it)
          const float lg = logf(p), lg1 = log1pf(-p);
          const float lp = lg < -100.f ? -100.f : lg, l1p = lg1 < -100.f ? -100.f : lg1;
          lrow = -(lab * lp + (1.f - lab) * l1p);
          const float pq = p * (1.f - p);
          dy3 = (p - lab) * (pq / fmaxf(pq, 1e-12f)) / (float)Bn;
        }
        if (q == 0) DY3[r] = dy3;
        float gw[8], dy2[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          gw[j] = dy3 * g2[j];
          dy2[j] = dy3 * wov[j] * gp2[j];
        }
        s8v v;
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = (short)f2bf(dy2[j]);
        *(LDS_AS s8v*)(F2 + r * LD32 + cc) = v;  // T32 aliases F2
        colsumW<8>(c, 0, gw, cc);
        colsumW<8>(c, 1, dy2, cc);
        float lsum = wave_sum(q == 0 ? lrow : 0.f);
        if (c.lane == 0) RED[c.wave] = lsum;
        wave_nan = __builtin_amdgcn_readfirstlane(lsum != lsum ? 1u : 0u);
      }
      // The 3-workgroup head takes the loss (and the NaN decision) only after the gradient hand-off:
      // every wave goes on with its own rows, flags its rows' NaN in its hand-off word, and the
      // branches OR those before they write anything (bwd_branch).  loss is NaN <=> some row's is.
      auto take_loss = [&]() {
        float tot = 0.f;
        for (int w = 0; w < 8; ++w) tot += RED[w];
        const float loss = tot / (float)Bn;
        if (loss != loss) failed = true;  // uniform across the workgroup
        else epoch_loss += loss;
      };
      if (ROLE != 3) {
        BAR();
        take_loss();
      }
      if (failed) {
        if (ROLE == 0 || ROLE == 3) {  // release them (every wave its rows' flags)
          if (ROLE == 3) wave_publish(c, xf(xflag, XF_BVIT, c.wave), ((uint32_t)step << 1) | 1u);
          wave_publish(c, xf(xflag, XF_BLAB, c.wave), ((uint32_t)step << 1) | 1u);
        }
        break;
      }
      // =============================== head backward ===============================
      // Adam of the output weights / fc2 bias (colsum slots 0, 1 and DY3) runs after the gradient
      // hand-off: nothing on the way to d(cat) reads them
      auto head_vec_adam = [&]() {
        float sm = 0.f;
        if (tid == 64)
          for (int i = 0; i < BM; ++i) sm += DY3[i];
        const VecG vs[3] = {{OUT_W, 32, 0}, {FC2_B, 32, 1}, {OUT_B, 1, -1}};
        adam_vecs(c, vs, K, sm);
      };
      gemm_pf<64, 32>(c, F2, LD32, wtf2);  // dd1 = dy2 . Wf2
      WBAR();
      STAMP(8);
      {  // E8: dy1 = drop'(dd1) * gelu'(y1) ; colsum dbf1 (v2)
        float d[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) d[j] = ACC[r * LDACC + c0 + j] * gk1[j];
        store16bf(TB + r * LD64 + c0, d);
        colsum16(c, 2, d);
      }
      WBAR();
      gemm_pf<64, 64>(c, TB, LD64, wtf1a);  // dcat[:, 0:64] = dy1 . Wf1[:, 0:64]
      if (ROLE == -1) {                     // one workgroup: dWf2 overlaps the dcat GEMMs
        head_vec_adam();
        gemm_dw_adam<2, 4>(c, F2, LD32, TA, LD64, MFC2, K);  // dWf2 = dy2^T d1
        if (tid < 64) adam(c.P, c.M, c.V, FC1_B + tid, cs_total(c, 2, tid), K);
      }
      WBAR();
      if (ROLE == 3) {  // vitals gradient -> its hand-off slot, released row-wave by row-wave
        put_grad(c, W_XB, r, c0);
        wave_publish(c, xf(xflag, XF_BVIT, c.wave), ((uint32_t)step << 1) | wave_nan);
      } else {
        float t[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) t[j] = ACC[r * LDACC + c0 + j];
        store16(c.wsf(W_DX3V) + opaque(r * 64 + c0), t);
      }
      WBAR();
      gemm_pf<64, 64>(c, TB, LD64, wtf1b);  // dcat[:, 64:128] (kept in ACC for the labs branch)
      if (ROLE == -1) BAR(); else WBAR();  // ROLE -1: dWf1 below reads every wave's TB rows
      if (ROLE == 0 || ROLE == 3) {  // hand the gradients over first: the head's own updates overlap
        put_grad(c, W_XB + BM * 64, r, c0);
        wave_publish(c, xf(xflag, XF_BLAB, c.wave), ((uint32_t)step << 1) | (ROLE == 3 ? wave_nan : 0u));
        BAR();  // the updates below read every wave's E8 column sums and TB rows
        if (ROLE == 3) {
          take_loss();
          if (failed) break;  // before any of the head's own updates
        }
        head_vec_adam();
        gemm_dw_adam<2, 4>(c, F2, LD32, TA, LD64, MFC2, K);  // dWf2 = dy2^T d1
        if (tid < 64) adam(c.P, c.M, c.V, FC1_B + tid, cs_total(c, 2, tid), K);
      }
      gemm_dw_adam<4, 8>(c, TB, LD64, CAT, LD128, MFC1, K);  // dWf1 = dy1^T cat
      BAR();
      STAMP(9);
      if (ROLE == -1) {
        BwdPre pre;
        bwd_prefetch<1>(c, pre);
        bwd_branch<1, 0>(c, s, stamps, t_prev, pre);
      }
      if (ROLE == -1 || ROLE == 0) {
        BwdPre pre;
        bwd_prefetch<0>(c, pre);
        bwd_branch<0, 1>(c, s, stamps, t_prev, pre);
      }
      // publish this step's Adam writes (bf16 weight copies, params) to every wave of the workgroup
      c.full_sync();
      r = c.r;
      q = c.q;
      c0 = q * 16;
    }
    if (HEAD && tid == 0) a.losses[(long)cid * a.E + e] = epoch_loss / (float)max(nb_total, 1);
  }
  if (HEAD && tid == 0) {
    const bool tmo =
        timed_out || (xflag && __hip_atomic_load(xflag + XF_TMO, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    a.ok[cid] = tmo ? -1 : (failed ? 0 : 1);
  }
}

__global__ void __launch_bounds__(NT) k_tf_train(AflTfTrainArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  train_body<-1>(a, blockIdx.x, smem);
}

// branch-parallel: workgroups 2c (vitals + head) and 2c+1 (labs) of client c
__global__ void __launch_bounds__(NT) k_tf_train_bp(AflTfTrainArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  if (blockIdx.x & 1)
    train_body<1>(a, blockIdx.x >> 1, smem);
  else
    train_body<0>(a, blockIdx.x >> 1, smem);
}

// branch-parallel, 3 workgroups per client: 3c (head), 3c+1 (vitals), 3c+2 (labs)
__global__ void __launch_bounds__(NT) k_tf_train_bp3(AflTfTrainArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int role = blockIdx.x % 3, cid = blockIdx.x / 3;
  if (role == 0)
    train_body<3>(a, cid, smem);
  else if (role == 1)
    train_body<2>(a, cid, smem);
  else
    train_body<1>(a, cid, smem);
}

// ================================================================================================
// eval forward: one 512-thread workgroup per 128-row tile of the test set (dropout off)
// ================================================================================================
namespace {
template <int BR>
__device__ __forceinline__ void eval_branch(const Ctx& c, const gu16* BF, const float* rows, bool valid,
                                            long ridx) {
  using B = BrC<BR>;
  const gf* P = c.P;
  const int r = 16 * c.wave + (c.lane & 15), q = c.lane >> 4, c0 = q * 16;
  unsigned short* XIN = c.u16(S_XIN);
  unsigned short* TA = c.u16(S_TA);
  unsigned short* TB = c.u16(S_TB);
  unsigned short* CAT = c.u16(S_CAT);
  unsigned short* F2 = c.u16(S_F2);
  float* ACC = c.acc();
  {
    s8v v;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int col = q * 8 + j;
      float x = (valid && col < B::din) ? rows[ridx * ROW + B::xoff + col] : 0.f;
      v[j] = (short)f2bf(x);
    }
    *(LDS_AS s8v*)(XIN + r * LD32 + q * 8) = v;
  }
  __syncthreads();
  gemm_xw<64, 32>(c, XIN, LD32, BF + B::w.WFd);
  __syncthreads();
  float h[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) h[j] = gelu(ACC[r * LDACC + c0 + j] + P[B::o.dense_b + c0 + j]);
  store16bf(TA + r * LD64 + c0, h);
  __syncthreads();
  gemm_xw<64, 64>(c, TA, LD64, BF + B::w.WFv);
  __syncthreads();
  {
    float x[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) x[j] = ACC[r * LDACC + c0 + j] + P[B::o.inproj_b + 128 + c0 + j];
    store16bf(TB + r * LD64 + c0, x);
  }
  __syncthreads();
  gemm_xw<64, 64>(c, TB, LD64, BF + B::w.WFo);
  __syncthreads();
  float x1[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) x1[j] = h[j] + ACC[r * LDACC + c0 + j] + P[B::o.out_b + c0 + j];
  ln_fwd(x1);
#pragma unroll
  for (int j = 0; j < 16; ++j) x1[j] = x1[j] * P[B::o.ln1_w + c0 + j] + P[B::o.ln1_b + c0 + j];
  store16bf(TA + r * LD64 + c0, x1);
  __syncthreads();
  gemm_xw<16, 64>(c, TA, LD64, BF + B::w.WF1);
  __syncthreads();
  {
    s8v v;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int col = q * 8 + j;
      v[j] = (short)f2bf(col < FF ? gelu(ACC[r * LDACC + col] + P[B::o.ff0_b + col]) : 0.f);
    }
    *(LDS_AS s8v*)(F2 + r * LD32 + q * 8) = v;
  }
  __syncthreads();
  gemm_xw<64, 32>(c, F2, LD32, BF + B::w.WF2);
  __syncthreads();
  {
    float x[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) x[j] = x1[j] + ACC[r * LDACC + c0 + j] + P[B::o.ff3_b + c0 + j];
    ln_fwd(x);
#pragma unroll
    for (int j = 0; j < 16; ++j) x[j] = x[j] * P[B::o.ln2_w + c0 + j] + P[B::o.ln2_b + c0 + j];
    ln_fwd(x);
#pragma unroll
    for (int j = 0; j < 16; ++j) x[j] = x[j] * P[B::o.bn_w + c0 + j] + P[B::o.bn_b + c0 + j];
    store16bf(CAT + r * LD128 + BR * 64 + c0, x);
  }
  __syncthreads();
}
}  // namespace

// blockIdx.y = model: params Pg + y * pstride, bf16 copies BFg + y * bfstride, scores out + y * n
__global__ void __launch_bounds__(NT) k_tf_eval(const float* __restrict__ Pg, long pstride,
                                                const unsigned short* __restrict__ BFg, long bfstride,
                                                const float* __restrict__ rows, int n, float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  Pg += blockIdx.y * pstride;
  BFg += blockIdx.y * bfstride;
  out += (long)blockIdx.y * n;
  Ctx c;
  c.smem = smem;
  c.tid = threadIdx.x;
  c.lane = threadIdx.x & 63;
  c.wave = threadIdx.x >> 6;
  c.P = (gf*)Pg;
  const gf* P = c.P;
  const gu16* BF = (const gu16*)BFg;
  const int r = 16 * c.wave + (c.lane & 15), q = c.lane >> 4;
  const int row0 = blockIdx.x * BM;
  const bool valid = row0 + r < n;
  const long ridx = valid ? row0 + r : 0;
  unsigned short* TA = c.u16(S_TA);
  unsigned short* CAT = c.u16(S_CAT);
  float* ACC = c.acc();
  eval_branch<0>(c, BF, rows, valid, ridx);
  eval_branch<1>(c, BF, rows, valid, ridx);
  gemm_xw<64, 128>(c, CAT, LD128, BF + WFF1);
  __syncthreads();
  {
    float x[16];
    const int c0 = q * 16;
#pragma unroll
    for (int j = 0; j < 16; ++j) x[j] = gelu(ACC[r * LDACC + c0 + j] + P[FC1_B + c0 + j]);
    store16bf(TA + r * LD64 + c0, x);
  }
  __syncthreads();
  gemm_xw<32, 64>(c, TA, LD64, BF + WFF2);
  __syncthreads();
  {
    float dot = 0.f;
    const int c0 = q * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) dot += gelu(ACC[r * LDACC + c0 + j] + P[FC2_B + c0 + j]) * P[OUT_W + c0 + j];
    const float y3 = rsum4(dot) + P[OUT_B];
    if (valid && q == 0) out[row0 + r] = sigmoidf_(y3);
  }
}

// bf16 weight copies for eval (same layout as the training workspace's BF region)
__device__ __forceinline__ void put_copy(const float* P, unsigned short* BF, MatW mw) {
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < mw.n_real * mw.k_real; e += gridDim.x * blockDim.x) {
    const int nn = e / mw.k_real, kk = e % mw.k_real;
    unsigned short h = f2bf(P[mw.off + e]);
    BF[mw.wf + nn * mw.wf_ld + kk] = h;
    if (mw.wt >= 0) BF[mw.wt + kk * mw.wt_ld + nn] = h;
  }
}
__global__ void k_tf_copies(const float* __restrict__ P, long pstride, unsigned short* __restrict__ BF,
                            long bfstride) {
  P += blockIdx.y * pstride;
  BF += blockIdx.y * bfstride;
  put_copy(P, BF, BrC<0>::dense);
  put_copy(P, BF, BrC<0>::vproj);
  put_copy(P, BF, BrC<0>::oproj);
  put_copy(P, BF, BrC<0>::ff0);
  put_copy(P, BF, BrC<0>::ff3);
  put_copy(P, BF, BrC<1>::dense);
  put_copy(P, BF, BrC<1>::vproj);
  put_copy(P, BF, BrC<1>::oproj);
  put_copy(P, BF, BrC<1>::ff0);
  put_copy(P, BF, BrC<1>::ff3);
  put_copy(P, BF, MFC1);
  put_copy(P, BF, MFC2);
}

long afl_tf_ws_floats() { return WS_FLOATS; }
int afl_tf_bf_ushorts() { return BF_TOTAL; }
int afl_tf_param_count() { return NPARAM; }

int afl_tf_train(const AflTfTrainArgs* a, hipStream_t s) {
  if (a->batch > BM || a->batch < 1) return -1;
  const int wgs = a->sync ? a->split : 1;  // workgroups per client
  if (wgs < 1 || wgs > 3) return -1;
  const void* fn = wgs == 3 ? (const void*)k_tf_train_bp3 : (wgs == 2 ? (const void*)k_tf_train_bp : (const void*)k_tf_train);
  if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, S_TOTAL) != hipSuccess) return -2;
  if (wgs > 1) {
    // the workgroups of a client spin on each other: every workgroup must be resident at once
    // (one 158 KB-LDS workgroup per CU); the caller zeroes the sync words before every launch
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return -3;
    if (wgs * a->C > cus) return -4;
    if (wgs == 3)
      hipLaunchKernelGGL(k_tf_train_bp3, dim3(3 * a->C), dim3(NT), S_TOTAL, s, *a);
    else
      hipLaunchKernelGGL(k_tf_train_bp, dim3(2 * a->C), dim3(NT), S_TOTAL, s, *a);
  } else {
    hipLaunchKernelGGL(k_tf_train, dim3(a->C), dim3(NT), S_TOTAL, s, *a);
  }
  return 0;
}

int afl_tf_eval_many(const float* params, long pstride, unsigned short* bf, long bfstride, int C, const float* rows,
                     int n, float* out, hipStream_t s) {
  if (C <= 0 || n <= 0) return 0;
  if (bfstride < BF_TOTAL) return -1;
  hipMemsetAsync(bf, 0, (size_t)bfstride * C * 2, s);
  hipLaunchKernelGGL(k_tf_copies, dim3(32, C), dim3(256), 0, s, params, pstride, bf, bfstride);
  if (hipFuncSetAttribute((const void*)k_tf_eval, hipFuncAttributeMaxDynamicSharedMemorySize, S_TOTAL) != hipSuccess)
    return -2;
  hipLaunchKernelGGL(k_tf_eval, dim3((n + BM - 1) / BM, C), dim3(NT), S_TOTAL, s, params, pstride,
                     (const unsigned short*)bf, bfstride, rows, n, out);
  return 0;
}

int afl_tf_eval_bf(const float* params, unsigned short* bf, const float* rows, int n, float* out, hipStream_t s) {
  return afl_tf_eval_many(params, 0, bf, BF_TOTAL, 1, rows, n, out, s);
}
