// Fused RNNModel/ICU local training — ONE launch trains every client of a rank for all its local
// epochs (reference model src/Model.py:91-163, training loop client.py:75-111).
//
// Each client runs on three co-resident 512-thread workgroups: the head (fc 128->32->16->1, BCE) and
// one per branch (vitals / labs: 3 stacked bidirectional GRU layers at seq_len 1, LayerNorm(64),
// dropout 0.3).  Per optimizer step the branch workgroups publish their outputs, the head runs its
// forward/backward and hands the branch gradients back before its own weight updates, and both branch
// backwards run concurrently (fused_common.h hand-off protocol, bounded spins).
//
// seq_len 1 with h0 = 0 makes every GRU direction a closed form of one input GEMM (PyTorch gate order
// r, z, n):  r = s(gi_r + b_hr), z = s(gi_z + b_hz), n = tanh(gi_n + r * b_hn), h = (1 - z) n,
// gi = x W_ih^T + b_ih.  W_hh multiplies h0 = 0: its gradient is exactly zero and Adam leaves it
// unchanged, so it is never touched.  GEMMs: v_mfma_f32_16x16x32_bf16 (input GEMMs from prefetched bf16
// weight fragments, dW = dY^T X from transposed LDS reads with Adam fused in the epilogue); gates,
// LayerNorm, loss in fp32 registers (row-per-4-lanes layout); the forward of a branch is row-local per
// wave and needs no workgroup barrier.
//
// Dropout masks use the layer-program convention (fl/programs.py, RNNProgram): key =
// hash(client seed, step index counted over every batch of the round, skipped size-1 batches
// included), layer id = branch, (row, column) of the 64-wide branch output — so the composite program
// on CPU is an exact-semantics oracle for this kernel.
#include "common.h"
#include "kernels.h"
#include "fused_common.h"
#include "rnn_common.h"

using namespace fk;

namespace {

using namespace rnl;

// ------------------------------------------------------------------------ bf16 weight copies (ushorts)
constexpr int BF_BR = 2 * G3 * 32 + 2 * 2 * (G3 * 64 + 64 * G3);  // 55296 per branch
__host__ __device__ constexpr int bf_wf(int br, int l, int d) {
  return br * BF_BR + (l == 1 ? d * G3 * 32 : 2 * G3 * 32 + (l - 2) * 2 * (2 * G3 * 64) + d * 2 * G3 * 64);
}
__host__ __device__ constexpr int bf_wt(int br, int l, int d) { return bf_wf(br, l, d) + G3 * 64; }  // l >= 2
constexpr int BF_HEAD = 2 * BF_BR;
constexpr int WF1 = BF_HEAD, WT1 = WF1 + 32 * 128, WF2 = WT1 + 128 * 32, WT2 = WF2 + 16 * 32;
constexpr int BF_TOTAL = WT2 + 32 * 32;
constexpr MatW MFC1{FC1_W, 32, 128, WF1, 128, WT1, 32};
constexpr MatW MFC2{FC2_W, 16, 32, WF2, 32, WT2, 32};

// ------------------------------------------------------------------------ workspace (floats)
constexpr long W_M = 0, W_V = NPARAM;
constexpr long W_BF = ((2L * NPARAM + 63) / 64) * 64;
constexpr long W_SAV = ((W_BF + BF_TOTAL / 2 + 63) / 64) * 64;
constexpr long SAV_RZN = 0, SAV_XH = 6L * BM * G3, SAV_RS = SAV_XH + BM * 64, SAV_BR = SAV_RS + BM;
constexpr long W_XF = W_SAV + 2 * SAV_BR;      // branch outputs bf16 [2][128][64]
constexpr long W_XB = W_XF + 2 * BM * 32;      // d(branch outputs) bf16 [128][64] in fp32-sized slots [2][128][64]
constexpr long WS_FLOATS = W_XB + 2 * BM * 64;

// ------------------------------------------------------------------------ LDS map (bytes)
constexpr int LDACC_R = 100, LDX = 40, LDH = 72, LDD = 104, LDC = 136;
constexpr int S_ACC = 0;
constexpr int S_CS = S_ACC + BM * LDACC_R * 4;  // 51200: column-sum partials [6][8][64]
constexpr int S_LAB = S_CS + 6 * 8 * 64 * 4;    // 63488
constexpr int S_DY3 = S_LAB + BM * 4;
constexpr int S_RED = S_DY3 + BM * 4;
constexpr int S_ROLE = S_RED + 16 * 4;          // 64576: role-specific region
// branch workgroup
constexpr int S_XIN = S_ROLE, S_H1 = S_XIN + BM * LDX * 2, S_H2 = S_H1 + BM * LDH * 2, S_DGI = S_H2 + BM * LDH * 2;
constexpr int S_BR_END = S_DGI + BM * LDD * 2;
// head workgroup
constexpr int S_CAT = S_ROLE, S_T1 = S_CAT + BM * LDC * 2, S_T1D = S_T1 + BM * LDX * 2, S_T2D = S_T1D + BM * LDX * 2;
constexpr int S_HD_END = S_T2D + BM * LDX * 2;
constexpr int S_TOTAL = S_BR_END > S_HD_END ? S_BR_END : S_HD_END;
static_assert(S_TOTAL <= 160 * 1024, "LDS budget");

struct RnLayout {
  static constexpr int S_ACC = ::S_ACC, LDACC = LDACC_R, S_CS = ::S_CS;
};
using Ctx = CtxT<RnLayout>;

constexpr uint32_t THR_P03 = 19661u;  // round(0.3 * 65536)
constexpr float INV_K03 = 1.f / 0.7f;

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + __expf(-x)); }
// torch.relu propagates NaN (fmaxf would swallow it and hide a diverged client from the NaN check)
__device__ __forceinline__ float relu_nan(float x) { return x < 0.f ? 0.f : x; }

__device__ __forceinline__ void store8bf(unsigned short* p, const float* x) { *(LDS_AS s8v*)p = pack8bf(x); }

// 8 fp32 at gf* -> 2 x float4 stores (and back)
__device__ __forceinline__ void st8(gf* p, const float* x) {
  *(GAS f4v*)p = f4v{x[0], x[1], x[2], x[3]};
  *(GAS f4v*)(p + 4) = f4v{x[4], x[5], x[6], x[7]};
}

// branch output y (16 values: columns q*8..+7 and 32+q*8..+7 of row r) -> hand-off slot (bf16)
__device__ __forceinline__ void put_out(const Ctx& c, long slot, int r, int q, const float* y) {
  const int bo = (int)slot * 4 + opaque(r * 64 + q * 8) * 2;
  st_wt16(c, bo, __builtin_bit_cast(u32x4, pack8bf(y)));
  st_wt16(c, bo + 64, __builtin_bit_cast(u32x4, pack8bf(y + 8)));  // +32 columns = 64 bytes
}

// ============================================================================ branch workgroup
template <int BR>
__device__ __forceinline__ void branch_body(const AflTfTrainArgs& a, int cid, unsigned char* smem) {
  using B = Br<BR>;
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
  c.r = 16 * c.wave + (c.lane & 15);
  c.q = c.lane >> 4;
  const int tid = c.tid;
  // init: Adam moments of this branch, its bf16 copies (padding zeroed first), LDS
  for (int i = B::base + tid; i < B::base + branch_size(B::din); i += NT) {
    c.M[i] = 0.f;
    c.V[i] = 0.f;
  }
  for (int i = BR * BF_BR + tid; i < (BR + 1) * BF_BR; i += NT) c.BF[i] = 0;
  for (int i = tid; i < S_TOTAL / 4; i += NT) ((float*)smem)[i] = 0.f;
  __syncthreads();
#pragma unroll
  for (int l = 1; l <= 3; ++l)
#pragma unroll
    for (int d = 0; d < 2; ++d)
      init_copies(c, MatW{B::wih(l, d), G3, B::kin(l), bf_wf(BR, l, d), l == 1 ? 32 : 64, l == 1 ? -1 : bf_wt(BR, l, d),
                          G3});
  __syncthreads();

  gu32* xflag = (gu32*)(a.sync + (long)cid * AFL_TF_SYNC_WORDS);  // per-wave XF_* flags (fused_common.h)
  unsigned short* XIN = c.u16(S_XIN);
  unsigned short* DGI = c.u16(S_DGI);
  float* ACC = c.acc();
  const gf* rows = (const gf*)a.rows;
  const gf* sav = c.wsf(W_SAV + BR * SAV_BR);
  const int nd = a.nd[cid];
  const int BS = a.batch;
  const int nb_total = (nd + BS - 1) / BS;
  const uint32_t seed = a.seeds[cid];
  double b1t = 1.0, b2t = 1.0;
  int step = 0;
  bool failed = false;
  int r = c.r, q = c.q;
  bool have_next = false;  // next step's inputs prefetched during the wait for the head
  float x_next[8];
  float grr[8], gzz[8], gnn[8], gbhn[8];  // saved r, z, n gates + b_hn of the next gate backward
  auto gate_prefetch = [&](int l, int d) {
    const gf* sv = sav + SAV_RZN + ((long)((l - 1) * 2 + d) * BM + opaque(c.r)) * G3 + c.q * 8;
    load8(grr, sv);
    load8(gzz, sv + HU);
    load8(gnn, sv + 2 * HU);
    load8(gbhn, c.P + B::bhh(l, d) + 2 * HU + c.q * 8);
  };

  for (int e = 0; e < a.E && !failed; ++e) {
    const gi32* ord = (const gi32*)(a.order + ((long)cid * a.E + e) * a.maxnd);
    for (int b0 = 0; b0 < nd; b0 += BS) {
      const int Bn = min(BS, nd - b0);
      if (Bn == 1) continue;
      ++step;
      b1t *= 0.9;
      b2t *= 0.999;
      const AdamK K{(float)((double)a.lr / (1.0 - b1t)), (float)(1.0 / sqrt(1.0 - b2t)), a.opt_mode == 1 ? a.lr : 0.f};
      const uint32_t key = afl_hash32(seed, (uint32_t)(e * nb_total + b0 / BS));
      r = c.r;
      q = c.q;
      {  // masked inputs (RNNModel maps -2.0 to 0) -> XIN (bf16, K padded to 32)
        float x[8];
        if (have_next) {  // loaded while this workgroup waited for the head's previous hand-off
#pragma unroll
          for (int j = 0; j < 8; ++j) x[j] = x_next[j];
          have_next = false;
        } else {
          const bool valid = r < Bn;
          const gf* row = rows + (long)(valid ? ord[b0 + r] : 0) * ROWW + (BR == 0 ? 0 : DV);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int col = q * 8 + j;
            float v = (valid && col < B::din) ? row[col] : 0.f;
            x[j] = v == -2.0f ? 0.f : v;
          }
        }
        store8bf(XIN + r * LDX + q * 8, x);
      }
      // ---------------- forward: 3 bidirectional GRU layers (row-local per wave) ----------------
      // The saved gates of each (layer, direction) are stored only after the NEXT one's weight and
      // bias loads are issued: loads and stores share one vmcnt queue, so loads behind the stores would
      // wait for their acknowledgements
      float h3[16];
      float sr[8], sz[8], sn[8];
      gf* ssv = nullptr;
#pragma unroll
      for (int l = 1; l <= 3; ++l) {
        const unsigned short* IN = l == 1 ? XIN : c.u16(l == 2 ? S_H1 : S_H2);
        unsigned short* HOUT = c.u16(l == 1 ? S_H1 : S_H2);  // (unused for l == 3)
#pragma unroll
        for (int d = 0; d < 2; ++d) {
          float bi[3][8], bh[3][8];
#pragma unroll
          for (int g = 0; g < 3; ++g) {
            load8(bi[g], c.P + B::bih(l, d) + g * HU + q * 8);
            load8(bh[g], c.P + B::bhh(l, d) + g * HU + q * 8);
          }
          if (l == 1) {
            WFr<96, 32> w;
            wload(w, c.BF + bf_wf(BR, l, d), c.lane);
            if (ssv) {
              st8(ssv, sr);
              st8(ssv + HU, sz);
              st8(ssv + 2 * HU, sn);
            }
            gemm_pf<96, 32>(c, IN, LDX, w);
          } else {
            WFr<96, 64> w;
            wload(w, c.BF + bf_wf(BR, l, d), c.lane);
            if (ssv) {
              st8(ssv, sr);
              st8(ssv + HU, sz);
              st8(ssv + 2 * HU, sn);
            }
            gemm_pf<96, 64>(c, IN, LDH, w);
          }
          float rr[8], zz[8], nn[8], h[8];
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const int j = q * 8 + i;
            rr[i] = sigm(ACC[r * LDACC_R + j] + bi[0][i] + bh[0][i]);
            zz[i] = sigm(ACC[r * LDACC_R + HU + j] + bi[1][i] + bh[1][i]);
            nn[i] = tanhf(ACC[r * LDACC_R + 2 * HU + j] + bi[2][i] + rr[i] * bh[2][i]);
            h[i] = (1.f - zz[i]) * nn[i];
          }
          ssv = (gf*)sav + SAV_RZN + ((long)((l - 1) * 2 + d) * BM + opaque(r)) * G3 + q * 8;
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            sr[i] = rr[i];
            sz[i] = zz[i];
            sn[i] = nn[i];
          }
          if (l < 3) {  // layer 1/2 outputs stay in LDS: next layer's input and its dW operand
            store8bf(HOUT + r * LDH + d * HU + q * 8, h);
          } else {
#pragma unroll
            for (int i = 0; i < 8; ++i) h3[d * 8 + i] = h[i];
          }
        }
      }
      // LayerNorm(64) + dropout 0.3 -> hand-off slot.  xhat, gamma, rstd and the dropout bits stay in
      // registers for the backward (nothing to reload or re-hash after the wait for the head)
      float lxh[16], lgm[16], lrstd;
      uint32_t lkeep = 0;
      {
        float bt[16];
        load8(*(float(*)[8])lgm, c.P + B::ln_w + q * 8);
        load8(*(float(*)[8])(lgm + 8), c.P + B::ln_w + HU + q * 8);
        load8(*(float(*)[8])bt, c.P + B::ln_b + q * 8);
        load8(*(float(*)[8])(bt + 8), c.P + B::ln_b + HU + q * 8);
        st8(ssv, sr);  // the last (layer, direction)'s saved gates
        st8(ssv + HU, sz);
        st8(ssv + 2 * HU, sn);
        lrstd = ln_fwd(h3);  // h3 -> xhat
        float y[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int col = (i < 8 ? 0 : HU) + q * 8 + (i & 7);
          const bool kp = afl_keep(key, BR, r, col, THR_P03);
          lkeep |= (kp ? 1u : 0u) << i;
          lxh[i] = h3[i];
          y[i] = (h3[i] * lgm[i] + bt[i]) * (kp ? INV_K03 : 0.f);
        }
        put_out(c, W_XF + BR * BM * 32, r, q, y);
      }
      wave_publish(c, xf(xflag, BR == 0 ? XF_VIT : XF_LAB, c.wave), (uint32_t)step);  // this wave's rows
      {  // the NEXT step's input row (two dependent loads) while the head works
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
          const gf* row = rows + (long)(vn ? ordn[bn + r] : 0) * ROWW + (BR == 0 ? 0 : DV);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int col = q * 8 + j;
            const float v = (vn && col < B::din) ? row[col] : 0.f;
            x_next[j] = v == -2.0f ? 0.f : v;
          }
          have_next = true;
        }
      }
      gate_prefetch(3, 0);  // the first gate backward's saved gates / bias, also before the wait
      gu32* fb = xf(xflag, BR == 0 ? XF_BVIT : XF_BLAB, c.wave);  // this wave's rows of d(output)
      const uint32_t v = wave_wait(c, fb, fb, (uint32_t)step, 1, xflag + XF_TMO);
      if (v == 0xFFFFFFFFu) {  // timeout
        failed = true;
        break;
      }
      // the head flags a NaN loss term per wave of rows; the OR is taken at the first barrier below,
      // before anything leaves LDS, so an aborted client keeps its pre-step parameters
      const uint32_t my_abort = v & 1u;
      // ---------------- backward ----------------
      float dh[16];
      {  // d(branch output) -> dropout' -> LayerNorm backward; colsums gamma (v0), beta (v1)
        const int bo = (int)(W_XB + BR * BM * 64) * 4 + opaque(r * 64 + q * 8) * 2;  // bf16 [128][64] (put_grad)
        float dy[16];
        unpack8bf(ld_wt16(c, bo), dy);            // columns q*8 .. +7
        unpack8bf(ld_wt16(c, bo + 64), dy + 8);   // columns 32 + q*8 .. +7
        const float(&xh)[16] = lxh;
        const float(&gm)[16] = lgm;
        const float rstd = lrstd;
        float t[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          dy[i] *= (lkeep >> i) & 1u ? INV_K03 : 0.f;
          t[i] = dy[i] * xh[i];
        }
        colsumW<8>(c, 0, *(const float(*)[8])t, q * 8);
        colsumW<8>(c, 0, *(const float(*)[8])(t + 8), HU + q * 8);
        colsumW<8>(c, 1, *(const float(*)[8])dy, q * 8);
        colsumW<8>(c, 1, *(const float(*)[8])(dy + 8), HU + q * 8);
        ln_bwd(dh, dy, xh, rstd, gm);
      }
      uint32_t* abort_w = (uint32_t*)(smem + S_RED) + 8;  // one word per wave (RED is head-only)
      if (c.lane == 0) abort_w[c.wave] = my_abort;
      __syncthreads();
      {
        uint32_t any = 0;
#pragma unroll
        for (int w = 0; w < 8; ++w) any |= abort_w[w];
        if (any) {  // the client's round fails
          failed = true;
          break;
        }
      }
      {
        const VecG vs[2] = {{B::ln_w, 64, 0}, {B::ln_b, 64, 1}};
        adam_vecs(c, vs, K);
      }
      WFr<64, 96> wdx;  // W_ih^T fragments of the dX GEMMs: the first one here, each next one right after
      wload(wdx, c.BF + bf_wt(BR, 3, 0), c.lane);  // the previous dX GEMM (before that matrix's Adam stores)
#pragma unroll
      for (int l = 3; l >= 1; --l) {
        const unsigned short* IN = l == 1 ? XIN : c.u16(l == 2 ? S_H1 : S_H2);
        float dsum[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) dsum[i] = 0.f;
#pragma unroll
        for (int d = 0; d < 2; ++d) {
          {  // gate backward for direction d: dgi (-> DGI), bias-gradient colsums v2 (r | z), v3 (n | n*r)
            // this (layer, direction)'s saved gates were loaded one iteration ahead (the first before
            // the wait for the head); issue the next one's loads now, behind this iteration's GEMMs
            float rr[8], zz[8], nn[8], bhn[8], dr[8], dz[8], dn[8], dnr[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) {
              rr[i] = grr[i];
              zz[i] = gzz[i];
              nn[i] = gnn[i];
              bhn[i] = gbhn[i];
            }
            {
              const int nl = d == 0 ? l : l - 1, ndr = d == 0 ? 1 : 0;
              if (nl >= 1) gate_prefetch(nl, ndr);
            }
#pragma unroll
            for (int i = 0; i < 8; ++i) {
              const float g = dh[d * 8 + i];
              const float pn = g * (1.f - zz[i]) * (1.f - nn[i] * nn[i]);  // d(pre-activation of n)
              const float pz = -g * nn[i] * zz[i] * (1.f - zz[i]);
              const float pr = pn * bhn[i] * rr[i] * (1.f - rr[i]);
              dr[i] = pr;
              dz[i] = pz;
              dn[i] = pn;
              dnr[i] = pn * rr[i];
            }
            store8bf(DGI + r * LDD + q * 8, dr);
            store8bf(DGI + r * LDD + HU + q * 8, dz);
            store8bf(DGI + r * LDD + 2 * HU + q * 8, dn);
            colsumW<8>(c, 2, dr, q * 8);
            colsumW<8>(c, 2, dz, HU + q * 8);
            colsumW<8>(c, 3, dn, q * 8);
            colsumW<8>(c, 3, dnr, HU + q * 8);
          }
          c.bar();
          r = c.r;
          q = c.q;
          if (l > 1) {  // d(layer input) += dgi . W_ih (transposed copy, before this matrix's Adam)
            gemm_pf<64, 96>(c, DGI, LDD, wdx);
            {
              const int nl = d == 0 ? l : l - 1, ndr = d == 0 ? 1 : 0;
              if (nl > 1) wload(wdx, c.BF + bf_wt(BR, nl, ndr), c.lane);
            }
#pragma unroll
            for (int i = 0; i < 8; ++i) {
              dsum[i] += ACC[r * LDACC_R + q * 8 + i];
              dsum[8 + i] += ACC[r * LDACC_R + HU + q * 8 + i];
            }
            c.bar();
            r = c.r;
            q = c.q;
          }
          // dW_ih = dgi^T x (Adam fused), then the two bias vectors
          const MatW mw{B::wih(l, d), G3, B::kin(l), bf_wf(BR, l, d), l == 1 ? 32 : 64, l == 1 ? -1 : bf_wt(BR, l, d),
                        G3};
          const VecG vs[4] = {{B::bih(l, d), 64, 2}, {B::bih(l, d) + 64, 32, 3}, {B::bhh(l, d), 64, 2},
                              {B::bhh(l, d) + 64, 32, 3, 32}};
          const AdamS sb = adam_vecs_ld(c, vs);  // the biases' state before the matrix's stores
          if (l == 1)
            gemm_dw_adam<6, 2>(c, DGI, LDD, IN, LDX, mw, K);
          else
            gemm_dw_adam<6, 4>(c, DGI, LDD, IN, LDH, mw, K);
          adam_vecs_st(c, vs, sb, K);
          c.bar();
          r = c.r;
          q = c.q;
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) dh[i] = dsum[i];
      }
      c.full_sync();  // publish this step's Adam writes (params, bf16 copies) to every wave
    }
  }
}

// ============================================================================ head workgroup
__device__ __forceinline__ void head_body(const AflTfTrainArgs& a, int cid, unsigned char* smem) {
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
  c.r = 16 * c.wave + (c.lane & 15);
  c.q = c.lane >> 4;
  const int tid = c.tid;
  for (int i = FC1_W + tid; i < NPARAM; i += NT) {
    c.M[i] = 0.f;
    c.V[i] = 0.f;
  }
  for (int i = BF_HEAD + tid; i < BF_TOTAL; i += NT) c.BF[i] = 0;
  for (int i = tid; i < S_TOTAL / 4; i += NT) ((float*)smem)[i] = 0.f;
  __syncthreads();
  init_copies(c, MFC1);
  init_copies(c, MFC2);
  __syncthreads();

  gu32* xflag = (gu32*)(a.sync + (long)cid * AFL_TF_SYNC_WORDS);  // per-wave XF_* flags (fused_common.h)
  unsigned short* CAT = c.u16(S_CAT);
  unsigned short* T1 = c.u16(S_T1);
  unsigned short* T1D = c.u16(S_T1D);
  unsigned short* T2D = c.u16(S_T2D);
  float* ACC = c.acc();
  float* LAB = (float*)(smem + S_LAB);
  float* DY3 = (float*)(smem + S_DY3);
  float* RED = (float*)(smem + S_RED);
  const gf* rows = (const gf*)a.rows;
  const int nd = a.nd[cid];
  const int BS = a.batch;
  const int nb_total = (nd + BS - 1) / BS;
  double b1t = 1.0, b2t = 1.0;
  int step = 0;
  bool failed = false, timed_out = false;
  int r = c.r, q = c.q;

  for (int e = 0; e < a.E && !failed; ++e) {
    const gi32* ord = (const gi32*)(a.order + ((long)cid * a.E + e) * a.maxnd);
    float epoch_loss = 0.f;
    for (int b0 = 0; b0 < nd; b0 += BS) {
      const int Bn = min(BS, nd - b0);
      if (Bn == 1) continue;
      ++step;
      b1t *= 0.9;
      b2t *= 0.999;
      const AdamK K{(float)((double)a.lr / (1.0 - b1t)), (float)(1.0 / sqrt(1.0 - b2t)), a.opt_mode == 1 ? a.lr : 0.f};
      r = c.r;
      q = c.q;
      const bool valid = r < Bn;
      if (q == 0) LAB[r] = valid ? rows[(long)ord[b0 + r] * ROWW + ROWW - 1] : 0.f;
      // weights and biases for the whole head forward, issued before the wait
      WFr<32, 128> w1;
      wload(w1, c.BF + WF1, c.lane);
      // every other GEMM's fragments of this step too (small): none is then loaded behind the
      // gradient hand-off's drain or on the way to it
      WFr<16, 32> w2;
      wload(w2, c.BF + WF2, c.lane);
      WFr<32, 32> wt2;
      wload(wt2, c.BF + WT2, c.lane);
      WFr<64, 32> wa, wb;
      wload(wa, c.BF + WT1, c.lane);
      wload(wb, c.BF + WT1 + 64 * 32, c.lane);
      float b1[8], b2[4], wo[4];
      load8(b1, c.P + FC1_B + q * 8);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        b2[i] = c.P[FC2_B + q * 4 + i];
        wo[i] = c.P[OUT_W + q * 4 + i];
      }
      const float bo = c.P[OUT_B];
      // this wave's CAT rows: its own flags, no workgroup barrier
      const uint32_t v = wave_wait(c, xf(xflag, XF_VIT, c.wave), xf(xflag, XF_LAB, c.wave), (uint32_t)step, 0,
                                   xflag + XF_TMO);
      if (v == 0xFFFFFFFFu) {
        timed_out = failed = true;
        break;
      }
#pragma unroll
      for (int br = 0; br < 2; ++br) {  // branch outputs -> CAT (this lane: 16 columns of its row)
        const int bo = (int)(W_XF + br * BM * 32) * 4 + opaque(r * 64 + q * 16) * 2;
        const u32x4 lo = ld_wt16(c, bo), hi = ld_wt16(c, bo + 16);
        *(LDS_AS s8v*)(CAT + r * LDC + br * 64 + q * 16) = __builtin_bit_cast(s8v, lo);
        *(LDS_AS s8v*)(CAT + r * LDC + br * 64 + q * 16 + 8) = __builtin_bit_cast(s8v, hi);
      }
      gemm_pf<32, 128>(c, CAT, LDC, w1);  // fc1 (row-local)
      float f1[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) f1[i] = relu_nan(ACC[r * LDACC_R + q * 8 + i] + b1[i]);
      store8bf(T1 + r * LDX + q * 8, f1);
      gemm_pf<16, 32>(c, T1, LDX, w2);  // fc2
      uint32_t wave_nan = 0;  // this wave's rows produced a NaN loss term
      {  // fc2 relu, output, sigmoid + BCE, d(out), d(fc2) ; colsums dW_out (v0), db2 (v1)
        float f2[4], dot = 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          f2[i] = relu_nan(ACC[r * LDACC_R + q * 4 + i] + b2[i]);
          dot += f2[i] * wo[i];
        }
        const float y3 = rsum4(dot) + bo;
        const float p = 1.f / (1.f + expf(-y3));
        const float lab = LAB[r];
        float lrow = 0.f, dy3 = 0.f;
        if (valid) {
          const float lg = logf(p), lg1 = log1pf(-p);
          const float lp = lg < -100.f ? -100.f : lg, l1p = lg1 < -100.f ? -100.f : lg1;
          lrow = -(lab * lp + (1.f - lab) * l1p);
          const float pq = p * (1.f - p);
          dy3 = (p - lab) * (pq / fmaxf(pq, 1e-12f)) / (float)Bn;
        }
        if (q == 0) DY3[r] = dy3;
        float gw[4], d2[8];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          gw[i] = dy3 * f2[i];
          d2[i] = f2[i] > 0.f ? dy3 * wo[i] : 0.f;
          d2[4 + i] = 0.f;
        }
        // T2D row: 16 real columns (4 per lane), columns 16..31 stay zero (K padding of the dX GEMM)
        *(LDS_AS s4v*)(T2D + r * LDX + q * 4) = __builtin_bit_cast(s4v, __builtin_bit_cast(u4v, pack8bf(d2)).xy);
        colsumW<4>(c, 0, gw, q * 4);
        colsumW<4>(c, 1, *(const float(*)[4])d2, q * 4);
        const float lsum = wave_sum(q == 0 ? lrow : 0.f);
        if (c.lane == 0) RED[c.wave] = lsum;
        wave_nan = __builtin_amdgcn_readfirstlane(lsum != lsum ? 1u : 0u);
      }
      // The loss (and the NaN decision) is taken only after the gradient hand-off: every wave goes on
      // with its own rows and flags its rows' NaN in its hand-off words; the branches OR those before
      // they write anything.  loss is NaN <=> some row's term is.
      gemm_pf<32, 32>(c, T2D, LDX, wt2);  // d(fc1 out) = d(fc2 out) . W2
      {
        float d1[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) d1[i] = f1[i] > 0.f ? ACC[r * LDACC_R + q * 8 + i] : 0.f;
        store8bf(T1D + r * LDX + q * 8, d1);
        colsumW<8>(c, 2, d1, q * 8);
      }
      gemm_pf<64, 32>(c, T1D, LDX, wa);  // d(vitals output) = d1 . W1[:, 0:64]
      put_grad(c, W_XB, r, q * 16);
      wave_publish(c, xf(xflag, XF_BVIT, c.wave), ((uint32_t)step << 1) | wave_nan);
      gemm_pf<64, 32>(c, T1D, LDX, wb);  // d(labs output)
      put_grad(c, W_XB + BM * 64, r, q * 16);
      wave_publish(c, xf(xflag, XF_BLAB, c.wave), ((uint32_t)step << 1) | wave_nan);
      c.bar();  // the updates below read every wave's rows and column sums
      r = c.r;
      q = c.q;
      {
        float tot = 0.f;
        for (int w = 0; w < 8; ++w) tot += RED[w];
        const float loss = tot / (float)Bn;
        if (loss != loss) failed = true;  // uniform: before any of the head's own updates
        else epoch_loss += loss;
      }
      if (failed) break;
      {  // output-layer / fc2-bias Adam (colsum slots 0, 1, DY3): off the way to the branch gradients
        float sm = 0.f;
        if (tid == 32)
          for (int i = 0; i < BM; ++i) sm += DY3[i];
        const VecG vs[3] = {{OUT_W, 16, 0}, {FC2_B, 16, 1}, {OUT_B, 1, -1}};
        adam_vecs(c, vs, K, sm);
      }
      gemm_dw_adam<1, 2>(c, T2D, LDX, T1, LDX, MFC2, K);    // dW2 = d2^T f1
      if (tid < 32) adam(c.P, c.M, c.V, FC1_B + tid, cs_total(c, 2, tid), K);
      gemm_dw_adam<2, 8>(c, T1D, LDX, CAT, LDC, MFC1, K);   // dW1 = d1^T cat
      c.full_sync();
      r = c.r;
      q = c.q;
    }
    if (tid == 0) a.losses[(long)cid * a.E + e] = epoch_loss / (float)max(nb_total, 1);
  }
  if (tid == 0) {
    const bool tmo = timed_out || __hip_atomic_load(xflag + XF_TMO, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    a.ok[cid] = tmo ? -1 : (failed ? 0 : 1);
  }
}

__global__ void __launch_bounds__(NT) k_rnn_train(AflTfTrainArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int role = blockIdx.x % 3, cid = blockIdx.x / 3;
  if (role == 0)
    head_body(a, cid, smem);
  else if (role == 1)
    branch_body<0>(a, cid, smem);
  else
    branch_body<1>(a, cid, smem);
}

}  // namespace

long afl_rnn_ws_floats() { return WS_FLOATS; }
int afl_rnn_param_count() { return NPARAM; }

int afl_rnn_train(const AflTfTrainArgs* a, hipStream_t s) {
  if (a->batch > BM || a->batch < 1 || !a->sync) return -1;
  if (hipFuncSetAttribute((const void*)k_rnn_train, hipFuncAttributeMaxDynamicSharedMemorySize, S_TOTAL) != hipSuccess)
    return -2;
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                                              hipSuccess)
    return -3;
  if (3 * a->C > cus) return -4;  // the three workgroups of every client spin on each other: all resident
  hipLaunchKernelGGL(k_rnn_train, dim3(3 * a->C), dim3(NT), S_TOTAL, s, *a);
  return 0;
}
