// Fused RNNModel/ICU local training, on-chip edition (reference model src/Model.py:91-163, training loop
// client.py:75-111).  One persistent launch trains every client of a rank for all its local epochs; each
// client runs on three co-resident 512-thread workgroups (head | vitals branch | labs branch) that hand
// activations and gradients to each other once per direction per step.  The design is tf2.hip's
// (onchip.h): after the prologue nothing of a client's model lives in global memory — fp32 master weights
// in AGPRs, bf16 weight images and fp32 bias / LayerNorm vectors in LDS, Adam moments in a per-workgroup
// slab loaded a phase ahead, activations chained in registers in the T layout.
//
// A branch is 3 stacked bidirectional GRU layers at seq_len 1 with h0 = 0, LayerNorm(64), dropout 0.3.
// With h0 = 0 every direction is a closed form of ONE input GEMM (PyTorch gate order r, z, n):
//     r = s(gi_r + b_hr),  z = s(gi_z + b_hz),  n = tanh(gi_n + r * b_hn),  h = (1 - z) n,  gi = W_ih x + b_ih,
// and W_hh (which multiplies h0 = 0) gets an exactly-zero gradient, so Adam leaves it untouched and it is
// never loaded.  Both directions of a layer are one 192-row "combined" gate matrix (row 96 d + 32 gate + j),
// so a layer is one T-layout GEMM of 12 output tiles whose direction-d half produces features 32 d + j of
// the layer output — already the B operand of the next layer.
//
// Per step, per branch workgroup:
//   forward (wave-local): 3 layers of MFMA + gates; the backward's per-feature factors
//     A = (1 - z)(1 - n^2), Bz = n z (1 - z), Cr = r (1 - r), r  are kept in registers as fp16 pairs
//     (relative precision 2^-11, and the factors themselves rather than r, z, n: (1 - n^2) from a rounded n
//     would lose all precision where the unit saturates);
//   LayerNorm + dropout -> hand-off to the head; the next batch's inputs and masks while the head works;
//   backward layer by layer: gate backward -> d(gate pre-activations) tile in LDS -> d(layer input)
//     through the transposed image (before that layer's Adam) -> barrier -> dW = dG^T X with Adam fused
//     (tile-owned weights) and bias sums (MFMA with an all-ones operand) -> barrier (the dG tile is reused);
//   the layer-1 weights are tile-owned as well (Adam fused into dW1, 12 tiles: waves 0-3 own two, 4-7 one);
//   the biases and LayerNorm vectors are "compact" entries (one element per thread slot) updated in one
//     branch-free pass at the end of the step.
// LDS is the binding budget (bf16 images 63 KB, h1 / h2 tiles 32 KB, one dG tile 48 KB), hence one dG tile
// and two barriers per layer.
//
// Dropout masks use the layer-program convention of rnn.hip / fl/programs.py (RNNProgram): key =
// hash(client seed, batch index counted over every batch of the round, skipped size-1 batches included),
// layer id = branch, (row, column) of the 64-wide branch output.
#include "onchip.h"
#include "rnn_common.h"

using namespace oc;

namespace r2 {

using namespace rnl;

constexpr uint32_t THR_P03 = 19661u;  // round(0.3 * 65536)
constexpr float INV_K03 = 1.f / 0.7f;
constexpr float LOG2E = 1.4426950408889634f;

// ----------------------------------------------------------------------------------- LDS maps (bytes)
// branch workgroup
constexpr int LDW1 = 24 * 2;                       // layer-1 image row stride: K = din <= 16 (unpermuted) + pad
#ifndef RNN2_LDW2
#define RNN2_LDW2 (LD64 + 16)
#endif
#ifndef RNN2_LDW3
#define RNN2_LDW3 (LD64 + 16)
#endif
// layer-2 / 3 image row strides (bytes): rows padded by 16 elements (32 B), so the gate GEMMs' fragment reads are
// conflict-free in gfx950 banking (wfrag ds_read_b128 4 -> 0 extra cycles per instruction, wtfrag 4 -> 2;
// tools/dbg/lds_banks.py): RNNModel +3.45 % (profiles/ab_r5_img_pad.log).  The room comes from the fp64 column-sum
// slots moving into the layer-1 image's row padding (dbl_slot).
constexpr int LDW2 = RNN2_LDW2, LDW3 = RNN2_LDW3;
__host__ __device__ constexpr int ldg(int l) { return l == 2 ? LDW2 : LDW3; }
constexpr int B_W1 = 0;                            // [192][24] layer 1 combined gate matrix
constexpr int B_W2 = B_W1 + 192 * LDW1;            // [192][72] layer 2 (K permuted, pcol)
constexpr int B_W3 = B_W2 + 192 * LDW2;            // [192][72] layer 3
constexpr int B_X2 = B_W3 + 192 * LDW3;            // tile64: h1 (X of dW2); after dW2: tile16 xin (X of dW1)
constexpr int B_X3 = B_X2 + 16384;                 // tile64: h2 (X of dW3)
constexpr int B_DG = B_X3 + 16384;                 // 3 x tile64: d(gate pre-activations) [128][192] of one layer
constexpr int B_NVEC = 1280;                       // 6 x (b_ih 96 | b_hh 96) in (layer, direction) order, LN w | b
constexpr int B_VEC = B_DG + 3 * 16384;            // fp32 [1280] bias / LayerNorm parameters
constexpr int B_CS = B_VEC + B_NVEC * 4;           // fp32 [1280] their gradients
// column sums produced wave-locally, accumulated as integer quanta in fp64 (onchip.h lds_addq: exact, so the
// 8-wave sums are independent of the wave order by construction, as tf2.hip): LN weight / bias (0..127), then
// per layer the d(b_hn) sums of both directions (128 + 64 (l - 1) + 32 d + j)
// The fp64 slots live in the layer-1 image's row padding (bytes 32..47 of each 48-byte row: the forward reads
// bytes 0..31 of a row, the dW1 update writes bytes 0..31 only), two slots per row (dbl_slot).
constexpr int B_NDBL = 128 + 3 * 64;
static_assert(B_NDBL <= 2 * 192 && LDW1 == 48, "fp64 column-sum slots fit the layer-1 image padding");
constexpr int B_MISC = B_CS + B_NVEC * 4;          // u32 [8] per-wave abort words (+ pad)
constexpr int B_TOTAL = B_MISC + 64;
constexpr int B_X1 = B_X2;
__device__ __forceinline__ uchar* dbl_slot(uchar* smem, int idx) { return smem + B_W1 + (idx >> 1) * LDW1 + 32 + 8 * (idx & 1); }
enum { VL_LNW = 1152, VL_LNB = 1216 };

// head workgroup
#ifndef RNN2_HPAD
#define RNN2_HPAD 0
#endif
// head image row strides (bytes): RNN2_HPAD=16 (32-byte padding, as tf2's head) measured neutral here (+0.07 %,
// profiles/ab_r5_img_pad.log)
constexpr int HLD1 = LD128 + RNN2_HPAD, HLD2 = LD32 + RNN2_HPAD;
constexpr int H_IMG_W1 = 0;                        // [32][128] fc1
constexpr int H_IMG_W2 = H_IMG_W1 + 32 * HLD1;     // [16][32]  fc2
constexpr int H_CAT = H_IMG_W2 + 16 * HLD2;        // tile128: cat(vitals, labs)     (X of dW1)
constexpr int H_A1 = H_CAT + 32768;                // tile32:  relu(fc1)              (X of dW2)
constexpr int H_DZ1 = H_A1 + 8192;                 // tile32:  d(fc1 pre-activation)  (dY of dW1)
constexpr int H_DZ2 = H_DZ1 + 8192;                // tile16:  d(fc2 pre-activation)  (dY of dW2)
constexpr int H_NVEC = 68;                         // fc1.b 32 | fc2.b 16 | output.w 16 | output.b 1 (| pad)
constexpr int H_VEC = H_DZ2 + 4096;
constexpr int H_PART = H_VEC + H_NVEC * 4;         // fp32 [8 waves][68] per-wave column sums
constexpr int H_LOSS = H_PART + 8 * H_NVEC * 4;    // fp32 [8] per-wave loss partials, then u32 [8] abort flags
constexpr int H_TOTAL = H_LOSS + 64;
enum { HV_B1 = 0, HV_B2 = 32, HV_WO = 48, HV_BO = 64, HV_N = 65 };

constexpr int SMEM_CORE = B_TOTAL > H_TOTAL ? B_TOTAL : H_TOTAL;
#ifdef RNN2_STAMPS
constexpr int ST_OFF = SMEM_CORE, ST_N = 16;       // u64 [16] per-phase timers of the stamped workgroup
constexpr int SMEM = ST_OFF + ST_N * 8;
#else
constexpr int SMEM = SMEM_CORE;
#endif
static_assert(SMEM <= 160 * 1024, "LDS budget");

// ------------------------------------------------------------------- per-client workspace (bytes)
// (hand-off payloads travel as tagged granules in the per-call zeroed sync block: onchip.h gr_put / gr_get)
// Adam moment slab per workgroup [slot][thread] of float4.  Branch: W3 tiles m 0-5 / v 6-11, W2 tiles m 12-17
// / v 18-23, compact entries m 24 / v 25, layer-1 tiles (m, v) 26-27 and 28-29.  Head: fc1 tiles m 0-1 / v 2-3, fc2 tile m 4 / v 5, vector 6.
constexpr int MOM_SLOTS = 30;
constexpr long WS_MOM = 0;
constexpr long MOM_WG_BYTES = (long)MOM_SLOTS * NTH * 16;
// saved backward factors of layers 1 and 2 (registers hold only layer 3's): per branch [layer][slot 0-7][thread]
// of 16 bytes, written during the forward, read back a phase ahead of each gate backward (L2-resident)
constexpr long WS_SAV = WS_MOM + 3 * MOM_WG_BYTES;
constexpr long SAV_BR_BYTES = 2L * 8 * NTH * 16;
constexpr long WS_BYTES = WS_SAV + 2 * SAV_BR_BYTES;

// ------------------------------------------------------------------------ per-phase timers (diagnostics)
#ifdef RNN2_STAMPS
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
// Wave priorities (as in tf2.hip): the critical chain at 2, the work that only has to finish before the next
// hand-off arrives (prefetch, masks, the head's deferred tiles) at 0.
#ifndef RNN2_NO_PRIO
__device__ __forceinline__ void prio_hi() { __builtin_amdgcn_s_setprio(2); }
__device__ __forceinline__ void prio_lo() { __builtin_amdgcn_s_setprio(0); }
#else
__device__ __forceinline__ void prio_hi() {}
__device__ __forceinline__ void prio_lo() {}
#endif
__device__ __forceinline__ void stamp_init(Stamp& stp, const AflTfTrainArgs& a, uchar* smem) {
#ifdef RNN2_STAMPS
  stp.on = a.stamps && (long)blockIdx.x == (long)a.stamps[63];
  stp.who = a.stamps ? 64 * (int)(a.stamps[62] & 7) : 0;
  stp.smem = smem;
  if (threadIdx.x == 0) *(LDS_AS uint64_t*)(smem + ST_OFF + 8 * (ST_N - 1)) = __builtin_amdgcn_s_memrealtime();
#endif
  (void)stp; (void)a; (void)smem;
}
__device__ __forceinline__ void stamp_fini(Stamp& stp, const AflTfTrainArgs& a, uchar* smem, int tid) {
#ifdef RNN2_STAMPS
  if (stp.on && tid == 0)
    for (int i = 0; i < ST_N - 1; ++i) a.stamps[i] = *(LDS_AS uint64_t*)(smem + ST_OFF + 8 * i);
#endif
  (void)stp; (void)a; (void)smem; (void)tid;
}

// Ablation switches of the diagnostic build (compile-time RNN2_ABL bits in the stamped build only, set through
// AFL_RNN2_ABL): skip one piece of work per step to price it (numerics are wrong then; timing only).
// ABL_HALF prices a row split of the branch (two workgroups of 64 rows, one wave per SIMD) without its exchanges:
// waves 4-7 skip every per-row and per-tile computation (still joining every barrier and hand-off), so waves 0-3
// run their rows' forward / backward and their dW tiles (half of the branch's, as an owned-half split would) alone
// on the SIMDs: the step time of that build bounds the split from below.
enum { ABL_TADAM = 1, ABL_BIAS = 2, ABL_MOM = 4, ABL_DWMMA = 8, ABL_HALF = 16 };
#if defined(RNN2_STAMPS) && defined(RNN2_ABL)
#define ABL(b) ((RNN2_ABL & (b)) != 0)
#else
#define ABL(b) false
#endif

// ------------------------------------------------------------------------------ gate math
typedef _Float16 h2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pkh(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(a, b));
}
__device__ __forceinline__ void unpkh(uint32_t u, float& a, float& b) {
  const h2v h = __builtin_bit_cast(h2v, u);
  a = (float)h[0];
  b = (float)h[1];
}
// two GRU units at h0 = 0 in packed FP32 (the branch is VALU-issue-bound; transcendentals stay scalar):
// returns h, saves each unit's backward factors (A, Bz) and (Cr, r) as fp16 pairs.  exp2 -> inf / 0 gives
// exactly 0 / 1 in the sigmoids and +-1 in tanh; NaN propagates.
__device__ __forceinline__ of2v exp2v(of2v x) { return of2v{__builtin_amdgcn_exp2f(x[0]), __builtin_amdgcn_exp2f(x[1])}; }
__device__ __forceinline__ of2v rcpv(of2v x) { return of2v{__builtin_amdgcn_rcpf(x[0]), __builtin_amdgcn_rcpf(x[1])}; }
__device__ __forceinline__ of2v gru_unit2(of2v ar, of2v az, of2v an, of2v bhn, uint32_t (&s0)[2], uint32_t (&s1)[2]) {
  const of2v r = rcpv(1.f + exp2v(ar * -LOG2E)), z = rcpv(1.f + exp2v(az * -LOG2E));
  const of2v e = exp2v((r * bhn + an) * (2.f * LOG2E));
  const of2v n = rcpv(1.f + e) * -2.f + 1.f;  // tanh
  const of2v omz = 1.f - z;
  const of2v A = omz * (n * -n + 1.f), Bz = n * z * omz, Cr = r * -r + r;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    s0[k] = pkh(A[k], Bz[k]);
    s1[k] = pkh(Cr[k], r[k]);
  }
  return omz * n;
}

// ------------------------------------------------------------------------------ branch workgroup
// One code path serves both branches (runtime branch index, wave-uniform): the vitals and labs branches differ
// only in din and their parameter offsets, and a single instantiation halves the kernel's code size.
constexpr int NC = (B_NVEC + NTH - 1) / NTH;   // compact slots per thread
// VEC segment of (layer l, direction d): b_ih at +0, b_hh at +96
__host__ __device__ constexpr int v0(int l, int d) { return ((l - 1) * 2 + d) * 192; }
struct RB {
  int base, din, xoff, N;
  __device__ __forceinline__ explicit RB(int br)
      : base(br ? BASE_L : BASE_V), din(br ? DL : DV), xoff(br ? DV : 0), N(B_NVEC) {}
  // flat offsets (rnn_common.h Br<>, with din at run time): W_ih of (layer l, direction d), b_ih, LN weight
  __device__ __forceinline__ int wih(int l, int d) const {
    return base + (l == 1 ? d * dir_block(din) : 2 * dir_block(din) + ((l - 2) * 2 + d) * dir_block(64));
  }
  __device__ __forceinline__ int bih(int l, int d) const { return wih(l, d) + G3 * (l == 1 ? din : 64) + G3 * HU; }
  __device__ __forceinline__ int ln_w() const { return base + 2 * dir_block(din) + 4 * dir_block(64); }
  // direction d's 96 x 64 block of the layer-l (2, 3) combined image
  __device__ __forceinline__ Mat mat(int l, int d) const {
    return Mat{wih(l, d), G3, 64, (l == 2 ? B_W2 : B_W3) + 96 * d * ldg(l), ldg(l)};
  }
  // compact entry -> flat parameter index
  __device__ __forceinline__ int cmp_param(int e) const {
    if (e < VL_LNW) {
      const int ld = e / 192, w = e - 192 * ld;               // (layer, direction) block, entry in it
      return bih(ld / 2 + 1, ld & 1) + w;                     // b_hh follows b_ih in the flat layout
    }
    return ln_w() + (e - VL_LNW);                             // ln_b follows ln_w
  }
  // layer-1 weight (row n of the combined [192][din] gate matrix, column k) -> flat parameter index
  __device__ __forceinline__ int w1_param(int n, int k) const { return wih(1, n / 96) + (n % 96) * din + k; }
};
static_assert(Br<1>::ln_b == Br<1>::ln_w + 64 && Br<0>::bhh(2, 1) == Br<0>::bih(2, 1) + G3, "contiguous vectors");

// values the backward needs from the forward (registers, through the hand-off wait)
struct Saved {
  uint32_t f3[32];    // layer 3, per feature 4 (2 d + t) + i: (A, Bz), (Cr, r) fp16 pairs (layers 1, 2: WS_SAV)
  uint32_t xh[8];     // LayerNorm xhat, bf16 pairs
  float rstd;
  uint32_t keep;      // dropout keep bits of the 16 output features
};
struct BrState {
  TS w3[6], w2[6];  // tiles of the layer-3 / layer-2 weight gradients (k tiles 2(w&1)+a, n tiles 3(w>>1)+b)
  TS l1[2];         // layer-1 tiles wave + 8 t (n rows 16 (wave + 8 t) + lane % 16, k = 4 (lane / 16) + i)
  VS cmp[NC];       // compact entries e = tid + 512 h
};

// dropout keep bits of the 16 T-layout output features 16t + 4g + i (bit 4t + i), rnn.hip's hash convention
__device__ __forceinline__ uint32_t out_mask(uint32_t key, uint32_t layer, int r, int g) {
  uint32_t m = 0;
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) m |= (afl_keep(key, layer, (uint32_t)r, (uint32_t)(16 * t + 4 * g + i), THR_P03) ? 1u : 0u)
                                     << (4 * t + i);
  return m;
}

// layer-1 A fragment (K = din <= 16, unpermuted): W[16T + (lane & 15)][4g .. 4g + 3], upper half zero
__device__ __forceinline__ s8v w1frag(const uchar* imgs, int T, int lane) {
  const s4v lo = *(const LDS_AS s4v*)(imgs + B_W1 + (16 * T + (lane & 15)) * LDW1 + 8 * (lane >> 4));
  return cat44(lo, s4v{0, 0, 0, 0});
}

// one bidirectional GRU layer of this wave's rows: x (B fragments) -> h (T layout), saved factors.
// imgs: the branch's three weight images (W1 at +B_W1, W2 at +B_W2, W3 at +B_W3); vec: its fp32 VEC block.
// (The forward-only eval kernel passes a scratch sv; the factor math is then dead code.)
template <int L>
__device__ __forceinline__ void gru_fwd(const uchar* imgs, const uchar* vec, const s8v* bx, float (&h)[16],
                                        uint32_t (&sv)[32], int lane) {
  const int g = lane >> 4;
  const uchar* img = imgs + (L == 2 ? B_W2 : B_W3);
  const uchar* vgl = lane_vec(vec, g);  // (this lane's vector base: immediate offsets for every bias read)
#pragma unroll
  for (int d = 0; d < 2; ++d) {
    f4v acc[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      const int T = 6 * d + k;
      if constexpr (L == 1) {  // K = din <= 16: the 16x16x16 form, no zero upper halves
        const s8v b = bx[0];
        acc[k] = mma16(*(const LDS_AS s4v*)(imgs + B_W1 + (16 * T + (lane & 15)) * LDW1 + 8 * (lane >> 4)),
                       s4v{b[0], b[1], b[2], b[3]}, Z4);
      } else {
        acc[k] = mma(wfrag(img, ldg(L), T, 0, lane), bx[0], Z4);
        acc[k] = mma(wfrag(img, ldg(L), T, 1, lane), bx[1], acc[k]);
      }
    }
    const uchar* vb = vgl + 4 * v0(L, d);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int o = 4 * (16 * t);
      const f4v bir = *(const LDS_AS f4v*)(vb + o), biz = *(const LDS_AS f4v*)(vb + 128 + o),
                bin = *(const LDS_AS f4v*)(vb + 256 + o), bhr = *(const LDS_AS f4v*)(vb + 384 + o),
                bhz = *(const LDS_AS f4v*)(vb + 512 + o), bhn = *(const LDS_AS f4v*)(vb + 640 + o);
#pragma unroll
      for (int i = 0; i < 4; i += 2) {
        const int f = 4 * (2 * d + t) + i;
        const of2v br = of2v{bir[i], bir[i + 1]} + of2v{bhr[i], bhr[i + 1]};
        const of2v bz = of2v{biz[i], biz[i + 1]} + of2v{bhz[i], bhz[i + 1]};
        uint32_t s0[2], s1[2];
        const of2v hv = gru_unit2(of2v{acc[t][i], acc[t][i + 1]} + br, of2v{acc[2 + t][i], acc[2 + t][i + 1]} + bz,
                                  of2v{acc[4 + t][i], acc[4 + t][i + 1]} + of2v{bin[i], bin[i + 1]},
                                  of2v{bhn[i], bhn[i + 1]}, s0, s1);
        h[f] = hv[0];
        h[f + 1] = hv[1];
        sv[2 * f] = s0[0];
        sv[2 * f + 1] = s1[0];
        sv[2 * f + 2] = s0[1];
        sv[2 * f + 3] = s1[1];
      }
    }
  }
}

// saved factors of layer L (1, 2) <-> the workspace (slot k of 8: features 4k .. 4k + 3... as 4 u32 each)
__device__ __forceinline__ void sav_st(__amdgpu_buffer_rsrc_t rsv, int L, int tid, const uint32_t (&sv)[32]) {
#pragma unroll
  for (int k = 0; k < 8; ++k)
  {
    __builtin_amdgcn_raw_buffer_store_b128(u32x4{sv[4 * k], sv[4 * k + 1], sv[4 * k + 2], sv[4 * k + 3]}, rsv, 16 * tid,
                                           ((L - 1) * 8 + k) * NTH * 16, 0);
    store_guard();
  }
}
__device__ __forceinline__ void sav_ld(__amdgpu_buffer_rsrc_t rsv, int L, int tid, uint32_t (&sv)[32]) {
  asm volatile("" : "+v"(tid));
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const u32x4 u = __builtin_amdgcn_raw_buffer_load_b128(rsv, 16 * tid, ((L - 1) * 8 + k) * NTH * 16, 0);
    sv[4 * k] = u[0];
    sv[4 * k + 1] = u[1];
    sv[4 * k + 2] = u[2];
    sv[4 * k + 3] = u[3];
  }
}

__device__ __forceinline__ void br_forward(uchar* smem, const float (&xin)[4], uint32_t keep, Saved& sv, u32x4 (&outp)[2],
                                           __amdgpu_buffer_rsrc_t rsv, int lane, int wave, int tid) {
  opq(lane, wave);
  const int g = lane >> 4, r = 16 * wave + (lane & 15);
  float h1[16], h2[16], h3[16];
  {
    const s8v bx[1] = {bfrag_lo(xin)};
    uint32_t s1[32];
    gru_fwd<1>(smem, smem + B_VEC, bx, h1, s1, lane);
    sav_st(rsv, 1, tid, s1);
  }
#pragma unroll
  for (int t = 0; t < 4; ++t) st4<TK64>(smem + B_X2, r, 4 * t + g, h1 + 4 * t);
  sb();
  {
    const s8v bx[2] = {bfrag(h1, 0), bfrag(h1, 1)};
    uint32_t s2[32];
    gru_fwd<2>(smem, smem + B_VEC, bx, h2, s2, lane);
    sav_st(rsv, 2, tid, s2);
  }
#pragma unroll
  for (int t = 0; t < 4; ++t) st4<TK64>(smem + B_X3, r, 4 * t + g, h2 + 4 * t);
  sb();
  {
    const s8v bx[2] = {bfrag(h2, 0), bfrag(h2, 1)};
    gru_fwd<3>(smem, smem + B_VEC, bx, h3, sv.f3, lane);
  }
  sb();
  // LayerNorm(64) + dropout 0.3
  sv.rstd = ln_fwd2(h3);
#pragma unroll
  for (int k = 0; k < 8; ++k) sv.xh[k] = pk2(h3[2 * k], h3[2 * k + 1]);
  float gm[16], bt[16];
  {
    const uchar* vgl = lane_vec(smem + B_VEC, g);
    vec16g(gm, vgl + 4 * VL_LNW);
    vec16g(bt, vgl + 4 * VL_LNB);
  }
  affine2(h3, h3, gm, bt);
  sv.keep = keep;
#pragma unroll
  for (int j = 0; j < 16; ++j) h3[j] = mbit(keep, j) ? h3[j] * INV_K03 : 0.f;
  pack16(h3, outp);
}

// gate backward of layer L, direction d: d(pre-activations) of this wave's rows -> dG tile (and registers),
// d(b_hn) terms dnr
template <int L>
__device__ __forceinline__ void gate_bwd(uchar* smem, const float (&dh)[16], const uint32_t (&sv)[32], int d, f4v (&dg)[6],
                                         float (&dnr)[16], int lane, int r) {
  const int g = lane >> 4;
  const uchar* vb = lane_vec(smem + B_VEC, g) + 4 * v0(L, d);
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const f4v bhn = *(const LDS_AS f4v*)(vb + 640 + 4 * (16 * t));
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int f = 4 * (2 * d + t) + i;
      float A, Bz, Cr, rr;
      unpkh(sv[2 * f], A, Bz);
      unpkh(sv[2 * f + 1], Cr, rr);
      const float gg = dh[f];
      const float dn = gg * A;
      dg[t][i] = dn * bhn[i] * Cr;   // r
      dg[2 + t][i] = -gg * Bz;       // z
      dg[4 + t][i] = dn;             // n
      dnr[f] = dn * rr;
    }
  }
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    const int T = 6 * d + k;
    float v[4] = {dg[k][0], dg[k][1], dg[k][2], dg[k][3]};
    st4<TK64>(smem + B_DG + (T >> 2) * 16384, r, 4 * (T & 3) + g, v);
  }
}

// d(b_hn) column sums of layer L (64 features: 32 d + j) -> fp64 accumulators
__device__ __forceinline__ void dnr_colsum(uchar* smem, int L, const float (&dnr)[16], int lane) {
  float s;
  const int f = colsum64(dnr, lane, s);
  lds_addq(dbl_slot(smem, 128 + 64 * (L - 1) + f), 0, s);
}

// backward of layer L (3 or 2) up to its d(input): dh (in) -> dG tile, dx (out)
template <int L>
__device__ __forceinline__ void layer_bwd(uchar* smem, const float (&dh)[16], const uint32_t (&sv)[32], float (&dx)[16],
                                          int lane, int wave) {
  opq(lane, wave);
  const int r = 16 * wave + (lane & 15);
  const uchar* img = smem + (L == 2 ? B_W2 : B_W3);
  f4v acc[4] = {Z4, Z4, Z4, Z4};
  float dnr[16];
#pragma unroll
  for (int d = 0; d < 2; ++d) {
    f4v dg[6];
    gate_bwd<L>(smem, dh, sv, d, dg, dnr, lane, r);
#pragma unroll
    for (int sl = 0; sl < 3; ++sl) {  // k-steps 3d + sl: gate rows 32 (3d + sl) .. + 31 = dG tiles 2 sl, 2 sl + 1
      const s8v b = pk8(dg[2 * sl][0], dg[2 * sl][1], dg[2 * sl][2], dg[2 * sl][3], dg[2 * sl + 1][0], dg[2 * sl + 1][1],
                        dg[2 * sl + 1][2], dg[2 * sl + 1][3]);
#pragma unroll
      for (int T = 0; T < 4; ++T) acc[T] = mma(wtfrag<true>(img, ldg(L), T, 3 * d + sl, lane), b, acc[T]);
    }
  }
  dnr_colsum(smem, L, dnr, lane);
#pragma unroll
  for (int T = 0; T < 4; ++T)
#pragma unroll
    for (int i = 0; i < 4; ++i) dx[4 * T + i] = acc[T][i];
}

// column sums of dG tile Tn (one per lane, i16 = feature) -> CS: b_ih, and b_hh for the r / z gates
__device__ __forceinline__ void bias_cs(uchar* smem, int L, int Tn, int i16, float s) {
  const int d = Tn >= 6 ? 1 : 0, w = 16 * (Tn - 6 * d) + i16;
  LDS_AS float* cs = ldsf(smem, B_CS) + v0(L, d);
  cs[w] = s;
  if (w < 64) cs[96 + w] = s;
}

// dW of layer L (3 or 2) = dG^T X with Adam on this wave's 6 tiles (k tiles Ta + a, n tiles Tn0 + b), one n
// tile at a time so only two accumulators and one tile pair's moments are live; the moments (moment slab
// slots mb .. mb + 11) are loaded at the phase start, behind the first n tile's MFMAs.  Then the bias sums.
// this wave's tile moments of layer L (slab slots mb .. mb + 11), issued ahead of the barrier before its dW phase
__device__ __forceinline__ void tile_mom_ld(__amdgpu_buffer_rsrc_t rm, int mb, int tid, f4v (&m)[6], f4v (&v)[6]) {
  asm volatile("" : "+v"(tid));
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    m[k] = ABL(ABL_MOM) ? Z4 : slot_ld(rm, mb + k, 16 * tid);
    v[k] = ABL(ABL_MOM) ? Z4 : slot_ld(rm, mb + 6 + k, 16 * tid);
  }
}
template <int L>
__device__ __forceinline__ void layer_dw(uchar* smem, const RB& R, TS (&wt)[6], f4v (&m)[6], f4v (&v)[6],
                                         __amdgpu_buffer_rsrc_t rm, int mb, const AdamK& K, int lane, int wave, int tid) {
  opq(lane, wave);
  asm volatile("" : "+v"(tid));
  const int i16 = lane & 15, g = lane >> 4;
  const uchar* X = smem + (L == 3 ? B_X3 : B_X2);
  const int Ta = 2 * (wave & 1), Tn0 = 3 * (wave >> 1), d = wave >> 2;
  const Mat M = R.mat(L, d);
  // bias sums of the three dG tiles this wave pair reads, MFMAs against an all-ones operand fused into the dW
  // loop (the dG fragment is already in registers): the even wave takes n tiles 0, 1, the odd wave tile 2
  const bool odd = (wave & 1) != 0;
#pragma unroll
  for (int b = 0; b < 3; ++b) {
    const int Tn = Tn0 + b;
    const uchar* DY = smem + B_DG + (Tn >> 2) * 16384;
    const bool bias = !ABL(ABL_BIAS) && (b == 2 ? odd : !odd);
    f4v acc0 = Z4, acc1 = Z4, bs = Z4;
    // (the all-ones operand materialised here, opaque: hoisted out of the step loop it was spilled and reloaded from
    // scratch before each of these MFMAs, 24 scratch round trips per dW phase.  Made opaque as a VGPR vector it was
    // still kept in an AGPR across the step and went through scratch once per step (a 16-byte reload in front of the
    // dW3 MFMAs); from an opaque SGPR the step loop has no scratch traffic at all)
    uint32_t o1 = 0x3F803F80u;  // bf16 1.0 pairs
    asm volatile("" : "+s"(o1));
    const s8v one = __builtin_bit_cast(s8v, u32x4{o1, o1, o1, o1});
    // fragments of k-step s + 1 issued before the MFMAs of k-step s (double-buffered)
    s8v y[2], x0[2], x1[2];
    y[0] = tfrag<TK64>(DY, 0, Tn & 3, lane);
    x0[0] = tfrag<TK64>(X, 0, Ta, lane);
    x1[0] = tfrag<TK64>(X, 0, Ta + 1, lane);
#pragma unroll
    for (int s = 0; s < (ABL(ABL_DWMMA) ? 0 : 4); ++s) {
      const int c = s & 1, n = c ^ 1;
      if (s < 3) {
        y[n] = tfrag<TK64>(DY, 32 * (s + 1), Tn & 3, lane);
        x0[n] = tfrag<TK64>(X, 32 * (s + 1), Ta, lane);
        x1[n] = tfrag<TK64>(X, 32 * (s + 1), Ta + 1, lane);
      }
      acc0 = mma(x0[c], y[c], acc0);
      acc1 = mma(x1[c], y[c], acc1);
      if (bias) bs = mma(one, y[c], bs);
    }
    if (bias && g == 0) bias_cs(smem, L, Tn, i16, bs[0]);
    if (!ABL(ABL_TADAM))  // (the 96 x 64 direction blocks are tile-exact: no element masks)
      tile_adam_pair(wt[b], wt[3 + b], m[b], v[b], m[3 + b], v[3 + b], M, Ta, Ta + 1, Tn - 6 * d, lane, acc0, acc1, K,
                     smem);
    if (!ABL(ABL_MOM)) {
      slot_st(rm, mb + b, 16 * tid, m[b]);
      slot_st(rm, mb + 6 + b, 16 * tid, v[b]);
      slot_st(rm, mb + 3 + b, 16 * tid, m[3 + b]);
      slot_st(rm, mb + 9 + b, 16 * tid, v[3 + b]);
    }
    sb();
  }
}

// layer 1: dW tiles with Adam fused (weights in AGPRs, moments in slots 26-29, bf16 -> the layer-1 image, whose
// bytes 0..31 of a row the backward does not read) and bias sums; the fp64 sums -> CS.  Columns k >= din are
// zero-gradient (their weights stay 0, the image's zero columns).
template <int NT>
__device__ __forceinline__ void l1_tiles(uchar* smem, BrState& st, f4v (&um)[4], const f4v (&acc)[2], int din,
                                         int wave, int lane, const AdamK& K) {
  constexpr int N = 4 * NT;
  const int g4 = 4 * (lane >> 4);
  float p[N], mm[N], vv[N], g[N], den[N];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      p[4 * t + i] = ar(st.l1[t].p[i]);
      mm[4 * t + i] = um[2 * t][i];
      vv[4 * t + i] = um[2 * t + 1][i];
      g[4 * t + i] = g4 + i < din ? acc[t][i] : 0.f;
    }
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const float mk = mm[i] * K.keep;
    mm[i] = mk + K.c1 * (g[i] - mk);
    vv[i] = fk::B2 * vv[i] + (1.f - fk::B2) * g[i] * g[i];
  }
#pragma unroll
  for (int i = 0; i < N; ++i) den[i] = __builtin_amdgcn_sqrtf(vv[i]);
#pragma unroll
  for (int i = 0; i < N; ++i) den[i] = __builtin_amdgcn_rcpf(den[i] * K.rsqrt_bc2 + K.eps);
#pragma unroll
  for (int i = 0; i < N; ++i) p[i] -= K.lr_bc1 * mm[i] * den[i];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      st.l1[t].p[i] = aw(p[4 * t + i]);
      um[2 * t][i] = mm[4 * t + i];
      um[2 * t + 1][i] = vv[4 * t + i];
    }
    const int n = 16 * (wave + 8 * t) + (lane & 15);
    *(LDS_AS u32x2v*)(smem + B_W1 + n * LDW1 + 2 * g4) =
        u32x2v{pk2(p[4 * t], p[4 * t + 1]), pk2(p[4 * t + 2], p[4 * t + 3])};
  }
}
__device__ __forceinline__ void layer1_mom_ld(__amdgpu_buffer_rsrc_t rm, int tid, f4v (&um)[4]) {
  asm volatile("" : "+v"(tid));
#pragma unroll
  for (int k = 0; k < 4; ++k) um[k] = slot_ld(rm, 26 + k, 16 * tid);
}
__device__ __forceinline__ void layer1_dw(uchar* smem, BrState& st, f4v (&um)[4], __amdgpu_buffer_rsrc_t rm, int din,
                                          const AdamK& K, int lane, int wave, int tid) {
  opq(lane, wave);
  const int i16 = lane & 15;
  const int nt = wave < 4 ? 2 : 1;
  f4v acc[2] = {Z4, Z4};
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    if (h == 1 && wave >= 4) break;
    const int Tn = wave + 8 * h;
    f4v bs = Z4;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const s8v y = tfrag<TK64>(smem + B_DG + (Tn >> 2) * 16384, 32 * s, Tn & 3, lane);
      acc[h] = mma(tfrag<TK16>(smem + B_X1, 32 * s, 0, lane), y, acc[h]);
      bs = mma(ones8(), y, bs);
    }
    if ((lane >> 4) == 0) bias_cs(smem, 1, Tn, i16, bs[0]);
  }
  if (!ABL(ABL_TADAM)) {
    if (nt == 2) l1_tiles<2>(smem, st, um, acc, din, wave, lane, K);
    else l1_tiles<1>(smem, st, um, acc, din, wave, lane, K);
  }
  if (!ABL(ABL_MOM)) {
    slot_st(rm, 26, 16 * tid, um[0]);
    slot_st(rm, 27, 16 * tid, um[1]);
    if (nt == 2) {
      slot_st(rm, 28, 16 * tid, um[2]);
      slot_st(rm, 29, 16 * tid, um[3]);
    }
  }
  if (tid < B_NDBL) {
    const float s = lds_getq(dbl_slot(smem, tid), 0);
    *(LDS_AS double*)dbl_slot(smem, tid) = 0.0;
    int e;
    if (tid < 128) {
      e = VL_LNW + tid;
    } else {
      const int k = tid - 128, l = k >> 6, f = k & 63;
      e = (2 * l + (f >> 5)) * 192 + 160 + (f & 31);
    }
    ldsf(smem, B_CS)[e] = s;
  }
}

// compact entries, branch-free (tf2.hip U3): gradient from CS, Adam, fp32 -> VEC (entries past the end write
// this lane's dummy word in the dG tile, dead while the compact entries are updated)
__device__ __forceinline__ void compact_mom_ld(__amdgpu_buffer_rsrc_t rm, int tid, f4v (&c)[2]) {
  asm volatile("" : "+v"(tid));
  c[0] = slot_ld(rm, 24, 16 * tid);
  c[1] = slot_ld(rm, 25, 16 * tid);
}
__device__ __forceinline__ void compact_update(uchar* smem, BrState& st, __amdgpu_buffer_rsrc_t rm, const f4v (&c)[2],
                                               const AdamK& K, int tid) {
  static_assert(NC <= 4, "compact moments fit one slot each");
  asm volatile("" : "+v"(tid));
  const int dmy = B_DG + 256 + 4 * (tid & 63);
  float gr[NC], mh[NC], vh[NC], pn[NC];
#pragma unroll
  for (int h = 0; h < NC; ++h) {
    const int e = tid + NTH * h;
    gr[h] = ldsf(smem, B_CS)[min(e, B_NVEC - 1)];  // (entries past the end: any finite value)
    mh[h] = c[0][h];
    vh[h] = c[1][h];
  }
  adam_staged<NC>(st.cmp, mh, vh, gr, pn, K);
#pragma unroll
  for (int h = 0; h < NC; ++h) {
    const int e = tid + NTH * h;
    *(LDS_AS float*)(smem + (e < B_NVEC ? B_VEC + 4 * e : dmy)) = pn[h];
  }
  f4v m4 = Z4, v4 = Z4;
#pragma unroll
  for (int h = 0; h < NC; ++h) {
    m4[h] = mh[h];
    v4[h] = vh[h];
  }
  slot_st(rm, 24, 16 * tid, m4);
  slot_st(rm, 25, 16 * tid, v4);
}

__device__ __forceinline__ void load_x(float (&x)[4], const AflTfTrainArgs& a, const RB& R, int cid, const Walk& w, int r,
                                       int g) {
  const int Bn = min(a.batch, a.nd[cid] - w.b0);
  const gi32* ord = (const gi32*)(a.order + ((long)cid * a.E + w.e) * a.maxnd);
  const bool valid = r < Bn;
  const int ridx = valid ? ord[w.b0 + r] : 0;
  const gf* row = (const gf*)a.rows + (long)ridx * ROWW + R.xoff;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = 4 * g + i;
    const float v = (valid && c < R.din) ? row[c] : 0.f;
    x[i] = v == -2.0f ? 0.f : v;  // RNNModel masks -2.0 to 0
  }
}

__device__ __forceinline__ void branch_main(const AflTfTrainArgs& a, int cid, uchar* smem, int BR) {
  const RB R(BR);
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6), g = lane >> 4;
  const int r = 16 * wave + (lane & 15);
  float* P = a.params + (long)cid * NPARAM;
  uchar* ws = (uchar*)(a.ws + (long)cid * a.ws_stride);
  gu32* sync = (gu32*)(a.sync + (long)cid * AFL_TF2_SYNC_WORDS);
  const __amdgpu_buffer_rsrc_t rg = gr_rsrc(sync);  // granule hand-off slots
  for (int i = tid; i < SMEM / 4; i += NTH) ldsf(smem, 0)[i] = 0.f;
  __syncthreads();
  BrState st;
  const __amdgpu_buffer_rsrc_t rm = rsrc(ws + WS_MOM + (BR + 1) * MOM_WG_BYTES);
  const __amdgpu_buffer_rsrc_t rsv = rsrc(ws + WS_SAV + BR * SAV_BR_BYTES);
#pragma unroll
  for (int k = 0; k < MOM_SLOTS; ++k) slot_st(rm, k, 16 * tid, Z4);
  {  // state: layer-2 / 3 tiles (AGPRs + images), compact entries (AGPRs + VEC / layer-1 image)
    const int Ta = 2 * (wave & 1), Tn0 = 3 * (wave >> 1), d = wave >> 2;
#pragma unroll
    for (int a2 = 0; a2 < 2; ++a2)
#pragma unroll
      for (int b = 0; b < 3; ++b) {
        tile_load(st.w3[3 * a2 + b], R.mat(3, d), Ta + a2, Tn0 + b - 6 * d, lane, P, smem);
        tile_load(st.w2[3 * a2 + b], R.mat(2, d), Ta + a2, Tn0 + b - 6 * d, lane, P, smem);
      }
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int n = 16 * (wave + 8 * t) + (lane & 15);
      float p0[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int k = 4 * g + i;
        p0[i] = (t == 0 || wave < 4) && k < R.din ? P[R.w1_param(n, k)] : 0.f;
        st.l1[t].p[i] = aw(p0[i]);
      }
      if (t == 0 || wave < 4)
        *(LDS_AS u32x2v*)(smem + B_W1 + n * LDW1 + 8 * g) = u32x2v{pk2(p0[0], p0[1]), pk2(p0[2], p0[3])};
    }
#pragma unroll
    for (int h = 0; h < NC; ++h) {
      const int e = tid + NTH * h;
      float p0 = 0.f;
      if (e < R.N) {
        p0 = P[R.cmp_param(e)];
        ldsf(smem, B_VEC)[e] = p0;
      }
      st.cmp[h] = VS{aw(p0)};
    }
  }
  __syncthreads();
  Stamp stp;
  stamp_init(stp, a, smem);

  const int nd = a.nd[cid], BS = a.batch, E = a.E;
  const int nb_total = (nd + BS - 1) / BS;
  const uint32_t seed = a.seeds[cid];
  LDS_AS uint32_t* abort_w = ldsu(smem, B_MISC);
  int step = 0;
  const bool half_idle = ABL(ABL_HALF) && wave >= 4;
  Walk w{0, 0};
  float xin[4];
  bool more = walk_valid(w, nd, BS, E);
  if (more) load_x(xin, a, R, cid, w, r, g);
  float mka = awu(more ? out_mask(afl_hash32(seed, (uint32_t)(w.e * nb_total + w.b0 / BS)), BR, r, g) : 0u);
  while (more) {
    ++step;
    const AdamK K = adam_k(a, step);
    Saved sv;
    u32x4 outp[2];
    prio_hi();
    asm volatile(";MARK fwd");
    if (!half_idle) br_forward(smem, xin, aru(mka), sv, outp, rsv, lane, wave, tid);
    if (half_idle) {  // (ablation build only: defined values for the skipped waves' hand-off rows, and zero X rows
                      // for the active waves' dW tiles: the h2 tile doubles as layer-1 gradient staging)
      outp[0] = outp[1] = u32x4{0u, 0u, 0u, 0u};
      sv.keep = 0u;
      const float zr[16] = {};
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        st4<TK64>(smem + B_X2, r, 4 * t + g, zr + 4 * t);
        st4<TK64>(smem + B_X3, r, 4 * t + g, zr + 4 * t);
      }
#pragma unroll
      for (int T = 0; T < 12; ++T) st4<TK64>(smem + B_DG + (T >> 2) * 16384, r, 4 * (T & 3) + g, zr);
    }
    const uint32_t xpk[2] = {pk2(xin[0], xin[1]), pk2(xin[2], xin[3])};  // xin -> X1 tile after dW2
    stp(0, tid);
    gr_put(rg, gr_off(0, BR, wave, lane), outp, (uint32_t)step);  // this wave's output rows -> head
    prio_lo();
    w.b0 += BS;  // the next batch's inputs and dropout masks while the head works
    more = walk_valid(w, nd, BS, E);
    if (more) {
      load_x(xin, a, R, cid, w, r, g);
      mka = awu(out_mask(afl_hash32(seed, (uint32_t)(w.e * nb_total + w.b0 / BS)), BR, r, g));
    }
    asm volatile(";MARK wait");
    stp(1, tid);
    u32x4 u[2];
    const int go[1] = {gr_off(1, BR, wave, lane)};
    const uint32_t fv = gr_get<1>(rg, go, u, (uint32_t)step, 1, sync + XF_TMO, lane);  // d(out) of this wave's rows
    prio_hi();
    stp(2, tid);
    if (fv == 0xFFFFFFFFu) break;
    float dh[16];
    if (half_idle)
#pragma unroll
      for (int j = 0; j < 16; ++j) dh[j] = 0.f;
    if (!half_idle) {  // d(branch output) -> dropout' -> LayerNorm backward; gamma / beta sums -> fixed point
      float dy[16], xh[16], t[16], gm[16];
      unpack16(u, dy);
#pragma unroll
      for (int j = 0; j < 16; ++j) dy[j] = mbit(sv.keep, j) ? dy[j] * INV_K03 : 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        xh[2 * k] = __uint_as_float(sv.xh[k] << 16);
        xh[2 * k + 1] = __uint_as_float(sv.xh[k] & 0xFFFF0000u);
      }
#pragma unroll
      for (int j = 0; j < 16; ++j) t[j] = dy[j] * xh[j];
      float s;
      int f = colsum64(t, lane, s);
      lds_addq(dbl_slot(smem, f), 0, s);
      f = colsum64(dy, lane, s);
      lds_addq(dbl_slot(smem, 64 + f), 0, s);
      vec16g(gm, lane_vec(smem + B_VEC, g) + 4 * VL_LNW);
      ln_bwd2(dh, dy, xh, sv.rstd, gm);
    }
    if (lane == 0) abort_w[wave] = fv & 1u;
    float dx[16];
    if (half_idle)
#pragma unroll
      for (int j = 0; j < 16; ++j) dx[j] = 0.f;
    asm volatile(";MARK bwd3");
    if (!half_idle) layer_bwd<3>(smem, dh, sv.f3, dx, lane, wave);
    stp(3, tid);
    f4v mm[6], vv[6];
    tile_mom_ld(rm, 0, tid, mm, vv);
    lds_bar();  // A3: every row's dG3 in LDS, every wave past its use of the W3 image
    {
      uint32_t any = 0;
#pragma unroll
      for (int i = 0; i < 8; ++i) any |= abort_w[i];
      if (any) break;  // the head saw a NaN loss: the round fails, this step's update is not applied
    }
    stp(4, tid);
    asm volatile(";MARK dw3");
    if (!half_idle) layer_dw<3>(smem, R, st.w3, mm, vv, rm, 0, K, lane, wave, tid);
    uint32_t sl[32];
    sav_ld(rsv, 2, tid, sl);
    lds_bar();  // B3: dG tile free
    stp(5, tid);
    asm volatile(";MARK bwd2");
    if (!half_idle) layer_bwd<2>(smem, dx, sl, dh, lane, wave);
    sav_ld(rsv, 1, tid, sl);
    tile_mom_ld(rm, 12, tid, mm, vv);
    lds_bar();  // A2
    stp(6, tid);
    asm volatile(";MARK dw2");
    if (!half_idle) layer_dw<2>(smem, R, st.w2, mm, vv, rm, 12, K, lane, wave, tid);
    lds_bar();  // B2: dG tile and the h1 tile free
    stp(7, tid);
    asm volatile(";MARK bwd1");
    if (!half_idle) {  // layer 1: gate backward only (no input gradient); xin -> X1 tile
      int ln = lane, wv = wave;
      opq(ln, wv);
      const int rr = 16 * wv + (ln & 15);
      f4v dg[6];
      float dnr[16];
      gate_bwd<1>(smem, dh, sl, 0, dg, dnr, ln, rr);
      gate_bwd<1>(smem, dh, sl, 1, dg, dnr, ln, rr);
      dnr_colsum(smem, 1, dnr, ln);
      *(LDS_AS u32x2v*)(smem + B_X1 + toff<TK16>(rr, ln >> 4)) = u32x2v{xpk[0], xpk[1]};
    }
    f4v um[4];
    layer1_mom_ld(rm, tid, um);
    lds_bar();  // A1
    stp(8, tid);
    asm volatile(";MARK dw1");
    if (!half_idle) layer1_dw(smem, st, um, rm, R.din, K, lane, wave, tid);
    f4v cmom[2];
    compact_mom_ld(rm, tid, cmom);
    lds_bar();  // C: every gradient of the compact entries in CS / GS
    stp(9, tid);
    asm volatile(";MARK u3");
    compact_update(smem, st, rm, cmom, K, tid);
    stp(10, tid);
    lds_bar();
    stp(11, tid);
  }
    asm volatile(";MARK fini");
  stamp_fini(stp, a, smem, tid);
  {  // parameters back (a failed client keeps its pre-step values: the failing step applied no update)
    const int Ta = 2 * (wave & 1), Tn0 = 3 * (wave >> 1), d = wave >> 2;
#pragma unroll
    for (int a2 = 0; a2 < 2; ++a2)
#pragma unroll
      for (int b = 0; b < 3; ++b) {
        tile_store(st.w3[3 * a2 + b], R.mat(3, d), Ta + a2, Tn0 + b - 6 * d, lane, P);
        tile_store(st.w2[3 * a2 + b], R.mat(2, d), Ta + a2, Tn0 + b - 6 * d, lane, P);
      }
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int n = 16 * (wave + 8 * t) + (lane & 15);
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if ((t == 0 || wave < 4) && 4 * g + i < R.din) P[R.w1_param(n, 4 * g + i)] = ar(st.l1[t].p[i]);
    }
#pragma unroll
    for (int h = 0; h < NC; ++h) {
      const int e = tid + NTH * h;
      if (e < R.N) P[R.cmp_param(e)] = ar(st.cmp[h].p);
    }
  }
}

// ================================================================================= head workgroup
constexpr Mat HW1{FC1_W, 32, 128, H_IMG_W1, HLD1};
constexpr Mat HW2{FC2_W, 16, 32, H_IMG_W2, HLD2};
__device__ __forceinline__ int hvec_param(int e) {
  return e < 32 ? FC1_B + e : e < 48 ? FC2_B + (e - 32) : e < 64 ? OUT_W + (e - 48) : e == 64 ? OUT_B : -1;
}
struct HdState {
  TS w1[2];  // fc1: k tile w, n tiles 0, 1
  TS w2;     // fc2: k tile w (waves 0, 1), n tile 0
  VS vec;
};
__device__ __forceinline__ float relu_nan(float x) { return x < 0.f ? 0.f : x; }  // NaN propagates like torch.relu

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
  const __amdgpu_buffer_rsrc_t rm = rsrc(ws + WS_MOM);
#pragma unroll
  for (int k = 0; k < 7; ++k) slot_st(rm, k, 16 * tid, Z4);
  {
#pragma unroll
    for (int b = 0; b < 2; ++b) tile_load(st.w1[b], HW1, wave, b, lane, P, smem);
    if (wave < 2) tile_load(st.w2, HW2, wave, 0, lane, P, smem);
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
  const uchar* vec = smem + H_VEC;
  LDS_AS float* part = ldsf(smem, H_PART) + wave * H_NVEC;
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
    lab = r < Bn ? ((const gf*)a.rows)[(long)ord[ww.b0 + r] * ROWW + ROWW - 1] : 0.f;
  };
  if (more) load_lab(w);
  while (more) {
    while (cur_e < w.e) {  // epoch boundaries crossed since the previous step close epoch losses
      if (tid == 0) a.losses[(long)cid * E + cur_e] = epoch_loss / (float)max(nb_total, 1);
      epoch_loss = 0.f;
      ++cur_e;
    }
    ++step;
    const AdamK K = adam_k(a, step);
    const int Bn = min(BS, nd - w.b0);
    const bool valid = r < Bn;
    const float inv_bn = 1.f / (float)Bn;  // (before the wait: the division is off the critical path)
    sb();
    u32x4 cv[4];  // vitals rows (cv[0..1]) | labs rows (cv[2..3])
    const int go[2] = {gr_off(0, 0, wave, lane), gr_off(0, 1, wave, lane)};
    const uint32_t fv = gr_get<2>(rg, go, cv, (uint32_t)step, 0, sync + XF_TMO, lane);
    if (fv == 0xFFFFFFFFu) {
      timed_out = failed = true;
      break;
    }
    prio_hi();
    stp(0, tid);
    // ---- fc1 + ReLU
    float z1[8], a1[8];
    {
      f4v acc[2];
#pragma unroll
      for (int T = 0; T < 2; ++T) {
        acc[T] = Z4;
#pragma unroll
        for (int s = 0; s < 4; ++s)
          acc[T] = mma(wfrag(smem + H_IMG_W1, HLD1, T, s, lane), __builtin_bit_cast(s8v, cv[s]), acc[T]);
      }
      float b1[8];
      vec8(b1, vec + HV_B1 * 4, g);
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          z1[4 * t + i] = acc[t][i] + b1[4 * t + i];
          a1[4 * t + i] = relu_nan(z1[4 * t + i]);
        }
    }
    // ---- fc2 + ReLU, output layer, sigmoid, BCE (log clamped at -100)
    float dz2[4], gw[4], f2[4];
    float dy3 = 0.f, pl = 0.f;
    {
      const f4v acc = mma(wfrag(smem + H_IMG_W2, HLD2, 0, 0, lane), bfrag(a1, 0), Z4);
      const f4v b2 = *(const LDS_AS f4v*)(vec + (HV_B2 + 4 * g) * 4), wo = *(const LDS_AS f4v*)(vec + (HV_WO + 4 * g) * 4);
      float dot = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        f2[i] = relu_nan(acc[i] + b2[i]);
        dot += f2[i] * wo[i];
      }
      const float y3 = fk::rsum4(dot) + *(const LDS_AS float*)(vec + HV_BO * 4);
      const float p = __builtin_amdgcn_rcpf(1.f + __expf(-y3));
      if (valid) {  // (torch's BCE gradient times the sigmoid's, without a division: tf2.hip head)
        const float pq = p * (1.f - p);
        dy3 = (p - lab) * (pq >= 1e-12f ? 1.f : pq * 1e12f) * inv_bn;
      }
      pl = p;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        dz2[i] = f2[i] > 0.f ? dy3 * wo[i] : 0.f;
        gw[i] = dy3 * f2[i];
      }
    }
    // NaN-loss abort flag from the gradient factor (NaN loss <=> non-finite dy3 for 0 / 1 labels, tf2.hip head);
    // the loss value is computed after the hand-off
    const uint32_t wave_nan = __builtin_amdgcn_ballot_w64(!(fabsf(dy3) <= 3.402823466e38f)) != 0 ? 1u : 0u;
    // ---- d a1 = dz2 . W2 -> d z1
    float dz1[8];
    {
      const s4v bz = bfrag4(dz2);
#pragma unroll
      for (int T = 0; T < 2; ++T) {
        const f4v acc = mma16(wtfrag4(smem + H_IMG_W2, HLD2, T, lane), bz, Z4);
#pragma unroll
        for (int i = 0; i < 4; ++i) dz1[4 * T + i] = z1[4 * T + i] > 0.f ? acc[i] : 0.f;
      }
    }
    // ---- d cat = dz1 . W1, each half straight to its branch
    {
      const s8v b0 = bfrag(dz1, 0);
#pragma unroll
      for (int hb = 0; hb < 2; ++hb) {
        float dd[16];
#pragma unroll
        for (int Tl = 0; Tl < 4; ++Tl) {
          const f4v acc = mma(wtfrag<true>(smem + H_IMG_W1, HLD1, 4 * hb + Tl, 0, lane), b0, Z4);
#pragma unroll
          for (int i = 0; i < 4; ++i) dd[4 * Tl + i] = acc[i];
        }
        u32x4 u[2];
        pack16(dd, u);
        gr_put(rg, gr_off(1, hb, wave, lane), u, ((uint32_t)step << 1) | wave_nan);  // NaN abort rides on the tag
      }
    }
    prio_lo();
    {  // per-wave loss partial (lane group 0: each row once) and the abort flag, for the loss barrier
      float lrow = 0.f;
      if (valid) {
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
    stp(1, tid);
    // ---- deferred: dW operand tiles and column sums of this wave's rows
    {
      sb();
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const u32x4 u = cv[t >> 1];
        const u32x2v v = (t & 1) ? u32x2v{u[2], u[3]} : u32x2v{u[0], u[1]};
        *(LDS_AS u32x2v*)(smem + H_CAT + t128(r, 4 * t + g)) = v;
      }
#pragma unroll
      for (int t = 0; t < 2; ++t) st4<TK32>(smem + H_A1, r, 4 * t + g, a1 + 4 * t);
#pragma unroll
      for (int t = 0; t < 2; ++t) st4<TK32>(smem + H_DZ1, r, 4 * t + g, dz1 + 4 * t);
      st4<TK16>(smem + H_DZ2, r, g, dz2);
      float sb1, sb2, swo;
      const int f1 = colsum32(dz1, lane, sb1);
      if (f1 >= 0) part[HV_B1 + f1] = sb1;
      const float z8[8] = {dz2[0], dz2[1], dz2[2], dz2[3], 0.f, 0.f, 0.f, 0.f};
      const float w8[8] = {gw[0], gw[1], gw[2], gw[3], 0.f, 0.f, 0.f, 0.f};
      const int f2i = colsum32(z8, lane, sb2), fo = colsum32(w8, lane, swo);
      if (f2i >= 0 && f2i < 16) {
        part[HV_B2 + f2i] = sb2;
        part[HV_WO + fo] = swo;
      }
      const float dbo = wave_sum(g == 0 ? dy3 : 0.f);
      if (lane == 0) part[HV_BO] = dbo;
    }
    f4v hm[3], hv[3], hvec;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      hm[k] = slot_ld(rm, k, 16 * tid);
      hv[k] = slot_ld(rm, 2 + k, 16 * tid);
    }
    hm[2] = slot_ld(rm, 4, 16 * tid);
    hv[2] = slot_ld(rm, 5, 16 * tid);
    hvec = slot_ld(rm, 6, 16 * tid);
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
      if (any) {  // (the same per-wave flags the branches abort on)
        failed = true;
        break;
      }
      epoch_loss += loss;
    }
    if (more) load_lab(wn);
    w = wn;
    stp(2, tid);
    // ---- weight gradients + Adam
    asm volatile(";MARK hd_upd");
    {
      f4v acc[2] = {Z4, Z4}, a2 = Z4;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const s8v x = tfrag<TK128>(smem + H_CAT, 32 * s, wave, lane);
        acc[0] = mma(x, tfrag<TK32>(smem + H_DZ1, 32 * s, 0, lane), acc[0]);
        acc[1] = mma(x, tfrag<TK32>(smem + H_DZ1, 32 * s, 1, lane), acc[1]);
        // fc2 tile (k tile wave & 1): every wave computes one (no branch among the MFMAs), waves 0, 1 own them
        a2 = mma(tfrag<TK32>(smem + H_A1, 32 * s, wave & 1, lane), tfrag<TK16>(smem + H_DZ2, 32 * s, 0, lane), a2);
      }
#ifdef RNN2_TRAP
      const f4v acc0 = acc[0], m0 = hm[0], v0 = hv[0];
      const float p0 = ar(st.w1[0].p[0]);
#endif
#pragma unroll
      for (int b = 0; b < 2; ++b) tile_adam(st.w1[b], hm[b], hv[b], HW1, wave, b, lane, acc[b], K, smem);
#ifdef RNN2_TRAP
      if (a.stamps && !__builtin_isfinite(ar(st.w1[0].p[0]))) {
        if (atomicCAS((unsigned long long*)a.stamps, 0ull, 1ull) == 0ull) {
          float* d = (float*)(a.stamps + 1);
          d[0] = cid; d[1] = step; d[2] = wave; d[3] = lane;
          d[4] = acc0[0]; d[5] = acc0[1]; d[6] = acc0[2]; d[7] = acc0[3];
          d[8] = m0[0]; d[9] = v0[0]; d[10] = p0; d[11] = hm[0][0]; d[12] = hv[0][0];
          d[13] = K.lr_bc1; d[14] = K.rsqrt_bc2; d[15] = K.keep; d[16] = K.c1; d[17] = K.eps;
        }
      }
#endif

      if (wave < 2) tile_adam(st.w2, hm[2], hv[2], HW2, wave, 0, lane, a2, K, smem);
      if (tid < HV_N) {  // the 8 waves' partial sums in a fixed order (bit-reproducible)
        const LDS_AS float* c = ldsf(smem, H_PART) + tid;
        float gsum = c[0];
#pragma unroll
        for (int w8 = 1; w8 < 8; ++w8) gsum += c[w8 * H_NVEC];
        float vm = hvec[0], vvv = hvec[1];
        ldsf(smem, H_VEC)[tid] = adam1(st.vec.p, vm, vvv, gsum, K);
        hvec[0] = vm;
        hvec[1] = vvv;
      }
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        slot_st(rm, k, 16 * tid, hm[k]);
        slot_st(rm, 2 + k, 16 * tid, hv[k]);
      }
      slot_st(rm, 4, 16 * tid, hm[2]);
      slot_st(rm, 5, 16 * tid, hv[2]);
      slot_st(rm, 6, 16 * tid, hvec);
    }
    asm volatile(";MARK hd_upd_end");
    stp(3, tid);
    lds_bar();
    stp(4, tid);
  }
  stamp_fini(stp, a, smem, tid);
  if (!failed) {
    while (cur_e < E) {
      if (tid == 0) a.losses[(long)cid * E + cur_e] = epoch_loss / (float)max(nb_total, 1);
      epoch_loss = 0.f;
      ++cur_e;
    }
  }
  {
#pragma unroll
    for (int b = 0; b < 2; ++b) tile_store(st.w1[b], HW1, wave, b, lane, P);
    if (wave < 2) tile_store(st.w2, HW2, wave, 0, lane, P);
    if (tid < HV_N) P[hvec_param(tid)] = ar(st.vec.p);
  }
  if (tid == 0) {
    const bool tmo = timed_out || __hip_atomic_load(sync + XF_TMO, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    a.ok[cid] = tmo ? -1 : (failed ? 0 : 1);
  }
}


#ifndef RNN2_STAMPS
// ============================================================================ forward-only evaluation
// C models over the same rows in ONE launch (validation: every client's generated model in hyper mode).
// Block (row tile of 128, model c): the fp32 parameters are converted once into the same bf16 images /
// fp32 vectors the trainer uses (both branches + head resident: 146 KB of LDS), then each wave runs its 16
// rows through both branches (GRU layers in the T layout, LayerNorm; eval mode: no dropout) and the head.
constexpr int E_BR = B_W3 + 192 * LDW3;          // one branch's images
constexpr int E_VEC = 2 * E_BR;                  // fp32 [2][1280]
constexpr int E_HW1 = E_VEC + 2 * B_NVEC * 4;    // fc1 image [32][LD128]
constexpr int E_HW2 = E_HW1 + 32 * LD128;        // fc2 image [16][LD32]
constexpr int E_HV = E_HW2 + 16 * LD32;          // fp32 [68] fc1.b | fc2.b | output.w | output.b
constexpr int E_SMEM = E_HV + H_NVEC * 4;
static_assert(E_SMEM <= 160 * 1024, "eval LDS budget");

__device__ __forceinline__ void st_bf(uchar* smem, int off, float v) { *(LDS_AS unsigned short*)(smem + off) = fk::f2bf(v); }

__global__ void __launch_bounds__(NTH) k_rnn2_eval(const float* __restrict__ params, long pstride,
                                                  const float* __restrict__ rows, int n, float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int c = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4;
  const float* P = params + (long)c * pstride;
#pragma unroll 1
  for (int br = 0; br < 2; ++br) {
    const RB R(br);
    uchar* imgs = smem + br * E_BR;
    for (int i = tid; i < 192 * 24; i += NTH) {  // layer 1, K = din (zero to the 24-element row stride)
      const int nn = i / 24, k = i - 24 * nn;
      st_bf(imgs, B_W1 + nn * LDW1 + 2 * k, k < R.din ? P[R.wih(1, nn / 96) + (nn % 96) * R.din + k] : 0.f);
    }
#pragma unroll 1
    for (int l = 2; l <= 3; ++l)
      for (int i = tid; i < 192 * 64; i += NTH) {
        const int nn = i >> 6, k = i & 63;
        st_bf(imgs, (l == 2 ? B_W2 : B_W3) + nn * ldg(l) + pcol(k) * 2, P[R.wih(l, nn / 96) + (nn % 96) * 64 + k]);
      }
    for (int e = tid; e < B_NVEC; e += NTH) ldsf(smem, E_VEC + br * B_NVEC * 4)[e] = P[R.cmp_param(e)];
  }
  for (int i = tid; i < 32 * 128; i += NTH) st_bf(smem, E_HW1 + (i >> 7) * LD128 + pcol(i & 127) * 2, P[FC1_W + i]);
  for (int i = tid; i < 16 * 32; i += NTH) st_bf(smem, E_HW2 + (i >> 5) * LD32 + pcol(i & 31) * 2, P[FC2_W + i]);
  if (tid < H_NVEC) ldsf(smem, E_HV)[tid] = tid < HV_N ? P[hvec_param(tid)] : 0.f;
  __syncthreads();

  const int r = blockIdx.x * 128 + 16 * wave + (lane & 15);
  const bool valid = r < n;
  float y[2][16];
#pragma unroll 1
  for (int br = 0; br < 2; ++br) {
    const RB R(br);
    const uchar* imgs = smem + br * E_BR;
    const uchar* vec = smem + E_VEC + br * B_NVEC * 4;
    float xin[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int col = 4 * g + i;
      const float v = (valid && col < R.din) ? rows[(long)r * ROWW + R.xoff + col] : 0.f;
      xin[i] = v == -2.0f ? 0.f : v;
    }
    float h1[16], h2[16], h3[16];
    uint32_t scratch[32];
    {
      const s8v bx[1] = {bfrag_lo(xin)};
      gru_fwd<1>(imgs, vec, bx, h1, scratch, lane);
    }
    {
      const s8v bx[2] = {bfrag(h1, 0), bfrag(h1, 1)};
      gru_fwd<2>(imgs, vec, bx, h2, scratch, lane);
    }
    {
      const s8v bx[2] = {bfrag(h2, 0), bfrag(h2, 1)};
      gru_fwd<3>(imgs, vec, bx, h3, scratch, lane);
    }
    ln_fwd2(h3);
    float gm[16], bt[16];
    vec16(gm, vec + 4 * VL_LNW, g);
    vec16(bt, vec + 4 * VL_LNB, g);
    affine2(h3, h3, gm, bt);
    if (br == 0) {
#pragma unroll
      for (int j = 0; j < 16; ++j) y[0][j] = h3[j];
    } else {
#pragma unroll
      for (int j = 0; j < 16; ++j) y[1][j] = h3[j];
    }
  }
  // head: fc1 (K = 128: vitals tiles 0-3, labs tiles 4-7) + ReLU, fc2 + ReLU, output, sigmoid
  f4v acc[2] = {Z4, Z4};
#pragma unroll
  for (int T = 0; T < 2; ++T)
#pragma unroll
    for (int s = 0; s < 4; ++s) acc[T] = mma(wfrag(smem + E_HW1, LD128, T, s, lane), bfrag(y[s >> 1], s & 1), acc[T]);
  float a1[8], b1[8];
  vec8(b1, smem + E_HV + HV_B1 * 4, g);
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) a1[4 * t + i] = relu_nan(acc[t][i] + b1[4 * t + i]);
  const f4v a2 = mma(wfrag(smem + E_HW2, LD32, 0, 0, lane), bfrag(a1, 0), Z4);
  const f4v b2 = *(const LDS_AS f4v*)(smem + E_HV + (HV_B2 + 4 * g) * 4), wo = *(const LDS_AS f4v*)(smem + E_HV + (HV_WO + 4 * g) * 4);
  float dot = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) dot += relu_nan(a2[i] + b2[i]) * wo[i];
  const float y3 = fk::rsum4(dot) + *(const LDS_AS float*)(smem + E_HV + HV_BO * 4);
  const float p = __builtin_amdgcn_rcpf(1.f + __expf(-y3));
  if (valid && g == 0) out[(long)c * n + r] = p;
}
#endif
}  // namespace r2

#ifdef RNN2_STAMPS
#define K_RNN2 k_rnn2_train_stamped
#else
#define K_RNN2 k_rnn2_train
#endif
// 3 workgroups per client: blocks c (head), C + c (vitals branch), 2C + c (labs branch)
__global__ void __launch_bounds__(oc::NTH) K_RNN2(AflTfTrainArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  // role-major block order: a client's workgroups are blocks cid, C + cid, 2C + cid, which the round-robin
  // dispatch deals to ONE XCD when C is a multiple of 8 (same-L2 hand-offs; speed only, never correctness)
  const int role = blockIdx.x / a.C, cid = blockIdx.x - role * a.C;
#if defined(RNN2_ROLE)  // register-pressure diagnostics: one role per build
  if (RNN2_ROLE == 0) r2::head_main(a, cid, smem);
  else if (RNN2_ROLE == 1) r2::branch_main(a, cid, smem, 0);
  else r2::branch_main(a, cid, smem, 1);
  (void)role;
#else
  if (role == 0)
    r2::head_main(a, cid, smem);
  else
    r2::branch_main(a, cid, smem, role - 1);  // one inlined copy for both branches
#endif
}

#ifdef RNN2_STAMPS
int afl_rnn2_train_stamped(const AflTfTrainArgs* a, hipStream_t s) {
#else
long afl_rnn2_ws_floats() { return r2::WS_BYTES / 4; }

int afl_rnn2_train(const AflTfTrainArgs* a, hipStream_t s) {
#ifndef RNN2_TRAP
  if (a->stamps) return afl_rnn2_train_stamped(a, s);
#endif
#endif
  if (a->batch > 128 || a->batch < 2 || !a->sync) return -1;
  if (!a->kt || a->kt_n < a->E * ((a->maxnd + a->batch - 1) / a->batch)) return -5;  // step table too short
  if (hipFuncSetAttribute((const void*)K_RNN2, hipFuncAttributeMaxDynamicSharedMemorySize, r2::SMEM) != hipSuccess)
    return -2;
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return -3;
  if (3 * a->C > cus) return -4;  // the workgroups of a client spin on each other: all must be resident
  hipLaunchKernelGGL(K_RNN2, dim3(3 * a->C), dim3(oc::NTH), r2::SMEM, s, *a);
  return 0;
}

#ifndef RNN2_STAMPS
// eval: out [C][n] = sigmoid outputs of C RNNModels (params [C][pstride]) over rows [n][24]
int afl_rnn2_eval(const float* params, long pstride, int C, const float* rows, int n, float* out, hipStream_t s) {
  if (C <= 0 || n <= 0) return 0;
  if (hipFuncSetAttribute((const void*)r2::k_rnn2_eval, hipFuncAttributeMaxDynamicSharedMemorySize, r2::E_SMEM) !=
      hipSuccess)
    return -2;
  hipLaunchKernelGGL(r2::k_rnn2_eval, dim3((n + 127) / 128, C), dim3(oc::NTH), r2::E_SMEM, s, params, pstride, rows, n,
                     out);
  return 0;
}
#endif
