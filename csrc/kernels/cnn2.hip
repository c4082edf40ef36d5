// CNNModel on-chip trainer: ONE launch trains every local client for its whole local round (all epochs,
// forward, backward, Adam) — the CNN counterpart of tf2.hip / rnn2.hip.  Reference model: src/Model.py:27-88
// (two Conv1d(1->32->64->128, k3, p1) + ReLU towers over vitals[7] / labs[16], AdaptiveAvgPool1d(4),
// Dropout(0.3), fc1 1024->128 -> fc2 64 -> fc3 32 -> output 1, sigmoid-BCE); trainer semantics
// client.py:66-112 (fresh Adam per round, size-1 batches skipped, NaN loss aborts the client).
//
// Replaces the per-step HIP-graph replay of ~14 launches (cnn.hip + layers.hip, ~160 us per step, a third
// of it launch floors) with a persistent cell of 25 workgroups per client, one per CU:
//
//   tower workgroups (8 vitals x 16 rows, 16 labs x 8 rows): the rows of a batch, both directions.
//     Activations live in LDS as bf16 in a "padded-row" layout — every sample's L positions framed by a
//     zero row on each side (L + 2 = 9 / 18 rows, 144 rows per workgroup in both towers) — so a k=3 conv is
//     three row-SHIFTED MFMA GEMMs (no im2col / col2im buffers): h_out = sum_j shift_{j-1}(h_in) . W_j^T,
//     d_in = sum_j shift_{1-j}(d_out) . W_j, dW_j = d_out^T . shift_{j-1}(h_in).  The pad rows make the
//     sample boundaries exact zeros.  The workgroup also computes its rows' fc1 pre-activation partial over
//     its tower's 512 concat features (z1p) and, in backward, its rows' d(concat) = d1 . W1.
//   the head workgroup: fc1 bias + ReLU on z1 = z1p_vitals + z1p_labs (fixed order), fc2 / fc3 / output,
//     BCE + NaN abort + epoch loss, the whole head backward (d1), Adam of fc2 / fc3 / output / fc1-bias
//     with p, m, v held in registers for the round.
//   ownership (ZeRO-style, all state in registers for the round): tower workgroup i owns 1/NTW of its
//     tower's conv parameters (output-channel blocks of 8) and a column block of fc1; it reduces the
//     tower's per-workgroup gradient partials for its block IN WORKGROUP ORDER (deterministic: no atomics),
//     runs Adam, and republishes the block as bf16 MFMA operand images in both orientations.
//
// Hand-offs (MI355X_MICROARCH.md, inter-workgroup visibility, table row 1): every handed-off byte is stored
// with 16-byte sc1 (write-through) stores and loaded with sc1 loads; each storing wave drains vmcnt, the
// workgroup barriers, one lane adds to an agent-scope counter; the consumer polls the counter with sc1
// loads (+ s_sleep) and barriers.  Per step: towers -> head (z1p), head -> towers (d1), tower group
// barrier after the partials, tower group barrier after the new images.  A client's 25 workgroups are
// blockIdx c, c + C, c + 2C, ... (one XCD at C = 8 under round-robin placement: speed only).  Every wait
// has a wall-clock deadline (s_memrealtime): a missing partner is an error, never a hang.
#include "common.h"
#include "kernels.h"

namespace {

typedef short s8v __attribute__((ext_vector_type(8)));
typedef short s4v __attribute__((ext_vector_type(4)));
typedef __bf16 bf8v __attribute__((ext_vector_type(8)));
typedef float f4v __attribute__((ext_vector_type(4)));
typedef float f2v __attribute__((ext_vector_type(2)));
typedef __bf16 b2v __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2v __attribute__((ext_vector_type(2)));
#define LDS_AS __attribute__((address_space(3)))
#define GAS __attribute__((address_space(1)))
typedef GAS uint32_t gu32;
typedef unsigned char uchar;

constexpr int NTH = 512;  // 8 waves
constexpr int NWG = 32;   // workgroups per client: 8 vitals + 16 labs towers + head + 7 fc1 owners
constexpr int WG_HEAD = 24, WG_FC1 = 25, NFC1 = 7;
constexpr long DEADLINE = 200000000L;  // s_memrealtime ticks (100 MHz): 2 s per wait

__device__ __forceinline__ f4v mfma(s8v a, s8v b, f4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf8v, a), __builtin_bit_cast(bf8v, b), c, 0, 0, 0);
}
constexpr f4v Z4 = {0.f, 0.f, 0.f, 0.f};
__device__ __forceinline__ unsigned short bfu(float x) { return __builtin_bit_cast(unsigned short, (__bf16)x); }
__device__ __forceinline__ uint32_t pk2(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f2v){a, b}, b2v));
}
__device__ __forceinline__ float bff(unsigned short h) { return __uint_as_float(((uint32_t)h) << 16); }
__device__ __forceinline__ float relu(float v) { return v < 0.f ? 0.f : v; }  // keeps NaN like torch
__host__ __device__ constexpr int bin_lo(int p, int L) { return (p * L) / 4; }
__host__ __device__ constexpr int bin_hi(int p, int L) { return ((p + 1) * L + 3) / 4; }
__host__ __device__ constexpr float bin_rcp(int p, int L) { return 1.f / (float)(bin_hi(p, L) - bin_lo(p, L)); }

// ---- LDS fragments ----
// row-major [rows][ld] bf16: MFMA operand rows r0 + (lane & 15), k = k0 + 8 (lane >> 4) .. +7
__device__ __forceinline__ s8v rfrag(const uchar* S, int ld, int r0, int k0, int lane) {
  return *(const LDS_AS s8v*)(S + ((r0 + (lane & 15)) * ld + k0 + 8 * (lane >> 4)) * 2);
}
// transposed operand from a [k rows][m cols] bf16 image (ds_read_b64_tr_b16): A[m][k] = S[k][m]
__device__ __forceinline__ s8v cfrag(const uchar* S, int ld, int k0, int m0, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const uchar* a1 = S + ((k0 + 8 * g + q) * ld + m0 + 4 * p) * 2;
  const s4v r1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s4v*)a1);
  const s4v r2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s4v*)(a1 + 4 * ld * 2));
  s8v r;
  r[0] = r1[0]; r[1] = r1[1]; r[2] = r1[2]; r[3] = r1[3];
  r[4] = r2[0]; r[5] = r2[1]; r[6] = r2[2]; r[7] = r2[3];
  return r;
}
__device__ __forceinline__ LDS_AS unsigned short* lu16(uchar* S, int byte_off) {
  return (LDS_AS unsigned short*)(S + byte_off);
}
__device__ __forceinline__ LDS_AS float* lf(uchar* S, int byte_off) { return (LDS_AS float*)(S + byte_off); }

// ---- global hand-off memory: 16-byte sc1 (write-through) stores / sc1 loads through a buffer resource ----
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, 0x7fffffff, 0x00020000);
}
// a 16-byte vector-memory store reads its data VGPRs after issue: a VALU write to them in the next cycle can
// land in the stored data (onchip.h store_guard); every b128 store is followed by this pinned s_nop
__device__ __forceinline__ void sguard() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 1" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}
__device__ __forceinline__ void st16(__amdgpu_buffer_rsrc_t rs, int byte_off, u32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, rs, byte_off, 0, 16);
  sguard();
}
__device__ __forceinline__ void st16f(__amdgpu_buffer_rsrc_t rs, int byte_off, f4v v) {
  st16(rs, byte_off, __builtin_bit_cast(u32x4, v));
}
__device__ __forceinline__ u32x4 ld16(__amdgpu_buffer_rsrc_t rs, int byte_off) {
  return __builtin_amdgcn_raw_buffer_load_b128(rs, byte_off, 0, 16);
}
__device__ __forceinline__ f4v ld16f(__amdgpu_buffer_rsrc_t rs, int byte_off) {
  return __builtin_bit_cast(f4v, ld16(rs, byte_off));
}
__device__ __forceinline__ s8v ld16s(__amdgpu_buffer_rsrc_t rs, int byte_off) {
  return __builtin_bit_cast(s8v, ld16(rs, byte_off));
}
// Workgroup barrier over LDS only: waits for this wave's LDS operations, not for its outstanding global loads
// (__syncthreads() drains vmcnt too, which stalled every barrier behind the operand prefetches issued before it).
// Global data written by the workgroup is published only through arrive(), which drains explicitly.
__device__ __forceinline__ void lbar() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
// Phase entry: the lane / wave indices become opaque, so every per-lane address of a phase is computed inside
// it (otherwise the compiler hoists the hundreds of swizzled LDS / image addresses of the step out of the loop
// and keeps them live across all phases, spilling to scratch)
#define REOPQ()                                   \
  do {                                            \
    __builtin_amdgcn_sched_barrier(0);            \
    asm volatile("" : "+v"(lane));                \
    wave = __builtin_amdgcn_readfirstlane(wave);  \
    asm volatile("" : "+s"(wave));                \
    lane &= 63;                                   \
    wave &= 7;                                    \
    tid = wave * 64 + lane;                       \
    g = lane >> 4;                                \
    li = lane & 15;                               \
  } while (0)
#define SYNC()        \
  do {                \
    lbar();  \
    REOPQ();          \
  } while (0)
__device__ __forceinline__ void drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// ---- per-client workspace (bytes from the client's base) ----
// images: per tower [W2 3x64x32 | W3 3x128x64 | W2T 3x32x64 | W3T 3x64x128] bf16, then fc1 W1 [128][1024] and
// W1T [1024][128] bf16
constexpr int IM_W2 = 0, IM_W3 = 6144, IM_W2T = 30720, IM_W3T = 36864, IM_TOWER = 61440;  // ushorts
// fc1 images are double-buffered by step parity (the fc1 owners write step k + 1's while the towers read step k's)
constexpr int IM_W1 = 2 * IM_TOWER, IM_W1T = IM_W1 + 131072, IM_FC1PAR = 262144, IM_END = IM_W1 + 2 * IM_FC1PAR;
constexpr int WS_IMG = 0;
constexpr int WS_SMALL = WS_IMG + IM_END * 2;              // [2][320] fp32: conv1 W (96) | b1 (32) | b2 (64) | b3 (128)
constexpr int NSMALL = 320;
constexpr int WS_FEAT = WS_SMALL + 2 * NSMALL * 4;         // [2 parities][128][1024] bf16 concat features
constexpr int FEAT_PAR = 128 * 1024 * 2;
constexpr int WS_Z1P = WS_FEAT + 2 * FEAT_PAR;             // [2][128][128] fp32 fc1 partials per tower
constexpr int WS_D1 = WS_Z1P + 2 * 128 * 128 * 4;          // [128][128] bf16 d(fc1 pre-activation)
constexpr int WS_STAT = WS_D1 + 128 * 128 * 2;             // [8 waves] x 16 B: head status of the step
constexpr int PSZ = 24576 + 6144 + NSMALL;                 // one tower workgroup's gradient partial (floats)
// [3 taps][16 o-blocks][64 ci][8 o] | [3][8][32][8] | smalls: an owner's o-block is one contiguous 2 KB / 1 KB run per tap
constexpr int P_W3 = 0, P_W2 = 24576, P_SM = 24576 + 6144;
constexpr int WS_PART = WS_STAT + 128;                     // [24][PSZ] fp32 (vitals 0..7, labs 8..23)
constexpr int WS_MV = WS_PART + 24 * PSZ * 4;              // [25 workgroups][8 slots][512 threads] {m f4, v f4}
constexpr int MV_WG = 16 * 512 * 32;
constexpr long WS_BYTES = WS_MV + (long)NWG * MV_WG;
// counters per client: F (towers -> head), H (head -> towers), P0/P1 (partials), W0/W1 (images), TMO
// W1R: fc1 images of the next step published (7 arrivals per step)
// HW + w: head wave w published d1 rows 16 w .. 16 w + 15 (the towers of those rows wait on it alone)
// FW + w: the tower workgroups of head wave w's rows (1 vitals + 2 labs) published their z1 partials
constexpr int CT_H = 1, CT_P = 2, CT_W = 4, CT_TMO = 6, CT_W1R = 7, CT_HW = 8, CT_FW = 16, CT_N = 24;  // x 32 words

struct Ctx {
  const AflCnn2Args* a;
  int c, tid, lane, wave, role;
  uchar* smem;
  uchar* wsb;                  // client workspace base (generic pointer for the buffer resources)
  __amdgpu_buffer_rsrc_t rw;   // client workspace
  gu32* ctr;                   // client counters
};

// optional per-phase wall-clock stamps (s_memrealtime, 10 ns) of the first 64 active steps:
// stamps[c][role][step][16] (tools/cnn2_phases.py)
constexpr int ST_STEPS = 64;
__device__ __forceinline__ void stamp(const Ctx& x, int k, int slot) {
  if (x.a->stamps != nullptr && k < ST_STEPS && x.tid == 0)
    x.a->stamps[(((long)x.c * NWG + x.role) * ST_STEPS + k) * 16 + slot] = __builtin_amdgcn_s_memrealtime();
}

__device__ __forceinline__ void arrive(const Ctx& x, int which) {
  drain();
  __syncthreads();
  if (x.tid == 0) __hip_atomic_fetch_add(x.ctr + which * 32, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// true when the counter reached `target`; false (all threads) on the deadline
__device__ __forceinline__ bool wait_ge(const Ctx& x, int which, uint32_t target, int flag_off) {
  LDS_AS int* fl = (LDS_AS int*)(x.smem + flag_off);
  if (x.tid == 0) {
    int ok = 1;
    const long t0 = (long)__builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(x.ctr + which * 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      if ((long)__builtin_amdgcn_s_memrealtime() - t0 > DEADLINE) {
        ok = 0;
        __hip_atomic_store(x.ctr + CT_TMO * 32, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        x.a->failed[x.c] = 2;  // the host raises on 2 (a NaN loss is 1)
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    fl[0] = ok;
  }
  lbar();
  const int ok = fl[0];
  lbar();  // fl is rewritten by the next wait
  return ok != 0;
}

// one wave waits (lane 0 polls) until counter `which` reached `target`; false on the deadline.  The payload
// loads that follow stay below the poll (wavefront acquire fence, as onchip.h await).
__device__ __forceinline__ bool wait_wave(const Ctx& x, int which, uint32_t target) {
  int ok = 1;
  if ((threadIdx.x & 63) == 0) {
    const long t0 = (long)__builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(x.ctr + which * 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      if ((long)__builtin_amdgcn_s_memrealtime() - t0 > DEADLINE) {
        ok = 0;
        __hip_atomic_store(x.ctr + CT_TMO * 32, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        x.a->failed[x.c] = 2;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  ok = __builtin_amdgcn_readfirstlane(ok);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  return ok != 0;
}

// Adam moments of this thread's slot k (private to the thread: written and read back by it alone)
__device__ __forceinline__ int mv_off(const Ctx& x, int k) { return WS_MV + x.role * MV_WG + (k * 512 + x.tid) * 32; }
__device__ __forceinline__ void mv_ld(const Ctx& x, int k, f4v& m, f4v& v) {
  m = ld16f(x.rw, mv_off(x, k));
  v = ld16f(x.rw, mv_off(x, k) + 16);
}
__device__ __forceinline__ void mv_st(const Ctx& x, int k, f4v m, f4v v) {
  st16f(x.rw, mv_off(x, k), m);
  st16f(x.rw, mv_off(x, k) + 16, v);
}

// the reference Adam step (k_adam_clients / torch.optim.Adam defaults) with bias corrections a, sb of step t;
// sgd (the gradient-test mode, opt_mode 1): p - lr g, moments untouched — the step exposes the raw gradient
struct AdamT {
  float a, sb;
  int sgd;
};
__device__ __forceinline__ float adam1(float p, float& m, float& v, float g, const AdamT& k) {
  if (k.sgd) return p - k.a * g;
  m = m + 0.1f * (g - m);
  v = 0.999f * v + 0.001f * g * g;
  return p - k.a * m / (sqrtf(v) / k.sb + 1e-8f);
}
__device__ __forceinline__ AdamT adam_t(float lr, int t, int opt_mode) {
  const float tt = (float)t;
  if (opt_mode == 1) return AdamT{lr, 1.f, 1};
  return AdamT{lr / (1.f - powf(0.9f, tt)), sqrtf(1.f - powf(0.999f, tt)), 0};
}

// ============================================================================================ towers
template <int T>
struct TW {
  static constexpr int L = T == 0 ? 7 : 16, R = T == 0 ? 16 : 8, NTW = T == 0 ? 8 : 16, LP = L + 2;
  static constexpr int COL0 = T == 0 ? 0 : 512, XOFF = T == 0 ? 0 : 7, NC = T == 0 ? 64 : 32, FIRST = T == 0 ? 0 : 8;
  static constexpr int NS = T == 0 ? 2 : 1;  // owner chunk slots per thread (970 / 485 chunks per owner)
  static_assert(R * LP == 144, "144 padded rows per tower workgroup");
};
constexpr int NR = 162;  // LDS rows: padded row q at row q + 1; rows 0 and 145..161 stay zero
// activation row strides padded by 16 elements (32 B): the conv GEMMs' ds_read_b128 operand reads (rfrag) are then
// conflict-free in gfx950's 4 x 16-lane banking (8 extra bytes left 2-way conflicts on every read: 4 extra cycles
// per instruction, tools/dbg/lds_banks.py); the T-layout row stores get worse (4 -> 12 extra cycles) but are
// rarer: CNNModel +0.7-1.0 % (profiles/ab_r5_cnn_pad.log; the head's rows padded the same way measured neutral)
constexpr int LD1 = 48, LD2 = 80, LD3 = 144, LDF = 520, LDZ = 132, LDD = 136;
constexpr int O_H1 = 0;
constexpr int O_H2 = O_H1 + NR * LD1 * 2;
constexpr int O_H3 = O_H2 + NR * LD2 * 2;   // h3, then d(h3) in place
constexpr int O_DH2 = O_H3 + NR * LD3 * 2;
constexpr int O_XS = O_DH2 + NR * LD2 * 2;  // fp32 x per padded row
constexpr int O_FT = O_XS + 656;            // feat bf16 [16][520] | z1p staging f32 [16][132] ; dfeat f32 [16][516]
constexpr int O_ZS = O_FT + 16 * LDF * 2;
constexpr int O_D1R = O_FT + 16 * 516 * 4;  // own d1 rows bf16 [16][136]
constexpr int O_RED = O_D1R + 16 * LDD * 2; // reductions (8 KB)
constexpr int O_FLAG = O_RED + 10240;
constexpr int T_LDS = O_FLAG + 16;
static_assert(O_ZS + 16 * LDZ * 4 <= O_D1R, "z1p staging");
// owner-phase staging (dead activation regions after the backward)
// S3 / S2: [blk][tap][ci][8 o] (W^T pieces), S3B / S2B: [blk][tap][8 o][ci] (W pieces): both staged from registers
constexpr int O_S3B = 8192, O_S2B = O_S3B + 6144;
static_assert(O_S2B + 1536 <= O_XS, "owner staging");
constexpr int O_S3 = 0, O_S2 = 6144, O_D1F = 8192, O_FW = O_D1F + 128 * LDD * 2, O_SW = O_FW + 128 * 72 * 2;
static_assert(O_SW + 128 * 72 * 2 <= O_XS, "owner staging");
// reduction slots (floats from O_RED)
constexpr int R_DB2 = 0, R_DB3 = 128, R_C1 = 128 + 1024, R_SM = 128 + 1024 + 512;  // [8][16] | [8][128] | [8][16][4] | [320]
// dropout keep bytes [2 step parities][16 rows][64] (one byte = 8 concat columns), as floats: 2 x 256.  A step's
// bytes are hashed during the PREVIOUS step's wait for the head (idle time), not in the forward's pooling
constexpr int R_KEEP = R_SM + NSMALL;
static_assert((R_KEEP + 512) * 4 <= 10240, "reduction slots");

// relu(acc + b) on a valid row, exact 0 on a pad row: branch-free (the select form became exec-mask branches)
__device__ __forceinline__ u32x2v relu_pack4(f4v acc, f4v b, bool ok) {
  const uint32_t km = ok ? 0xFFFFFFFFu : 0u;
  float v[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) v[e] = __uint_as_float(__float_as_uint(relu(acc[e] + b[e])) & km);
  return u32x2v{pk2(v[0], v[1]), pk2(v[2], v[3])};
}
__device__ __forceinline__ bool valid_q(int q, int LP) {
  const int l = q % LP;
  return q < 144 && l != 0 && l != LP - 1;
}

// dropout keep bytes of step s (all rows of this tower workgroup) -> keep buffer `buf` (bit k of byte (r, cp) keeps
// concat column COL0 + 8 cp + k of row b0 + r: the layer-program hash convention, 16 bits per column pair)
template <int T>
__device__ __forceinline__ void keep_bytes(const AflCnn2Args& a, int c, int b0, int s, uchar* S, int buf, int tid) {
  using C = TW<T>;
  const uint32_t key = afl_hash32(a.seeds[c], (uint32_t)s);
  for (int e = tid; e < C::R * 64; e += NTH) {
    const int r = e >> 6, cp = e & 63;
    uint32_t kb = 0u;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t hsh = afl_hash4(key, (uint32_t)T, (uint32_t)(b0 + r), (uint32_t)((C::COL0 + 8 * cp) / 2 + k));
      kb |= ((hsh & 0xFFFFu) >= a.thr16 ? 1u : 0u) << (2 * k);
      kb |= ((hsh >> 16) >= a.thr16 ? 1u : 0u) << (2 * k + 1);
    }
    *(LDS_AS uchar*)(S + O_RED + (R_KEEP + 256 * buf) * 4 + r * 64 + cp) = (uchar)kb;
  }
}

template <int T>
struct TowerState {
  // owned conv chunks (4 elements each; moments in slab slots 0..NS-1)
  float p[TW<T>::NS][4];
};

// owned chunk u -> kind (0 none, 3 W3, 2 W2, 1 small), partial float offset, param element base (+ stride)
struct Chunk {
  int kind, poff, j, ci, o0, s0;
};
template <int T>
__device__ __forceinline__ Chunk chunk_of(int i, int cid) {
  Chunk k{0, 0, 0, 0, 0, 0};
  int lo;
  if (T == 0) {
    if (cid < 768) {
      const int bk = 2 * i + cid / 384;
      lo = cid % 384;
      k.kind = 3; k.j = lo / 128; k.ci = (lo % 128) >> 1; k.o0 = 8 * bk + 4 * (lo & 1);
    } else if (cid < 960) {
      lo = cid - 768;
      k.kind = 2; k.j = lo / 64; k.ci = (lo % 64) >> 1; k.o0 = 8 * i + 4 * (lo & 1);
    } else if (cid < 970) {  // 10 of the 80 small-vector chunks per owner
      k.kind = 1; k.s0 = 4 * (10 * i + cid - 960);
    }
  } else {
    // labs: W3 block i, half (ci 16 (i & 1) ..) of W2 block i >> 1, 5 of the 80 small-vector chunks
    if (cid < 384) {
      lo = cid;
      k.kind = 3; k.j = lo / 128; k.ci = (lo % 128) >> 1; k.o0 = 8 * i + 4 * (lo & 1);
    } else if (cid < 480) {
      lo = cid - 384;
      k.kind = 2; k.j = lo / 32; k.ci = 16 * (i & 1) + ((lo % 32) >> 1); k.o0 = 8 * (i >> 1) + 4 * (lo & 1);
    } else if (cid < 485) {
      k.kind = 1; k.s0 = 4 * (5 * i + cid - 480);
    }
  }
  if (k.kind == 3) k.poff = P_W3 + ((k.j * 16 + (k.o0 >> 3)) * 64 + k.ci) * 8 + (k.o0 & 7);
  if (k.kind == 2) k.poff = P_W2 + ((k.j * 8 + (k.o0 >> 3)) * 32 + k.ci) * 8 + (k.o0 & 7);
  if (k.kind == 1) k.poff = P_SM + k.s0;
  return k;
}
// arena index of element e of a chunk
template <int T>
__device__ __forceinline__ int elem_idx(const AflCnn2Args& a, const Chunk& k, int e) {
  const int* of = a.off + 6 * T;  // conv1 w, conv1 b, conv2 w, conv2 b, conv3 w, conv3 b
  if (k.kind == 3) return of[4] + ((k.o0 + e) * 64 + k.ci) * 3 + k.j;
  if (k.kind == 2) return of[2] + ((k.o0 + e) * 32 + k.ci) * 3 + k.j;
  const int s = k.s0 + e;
  if (s < 96) return of[0] + s;
  if (s < 128) return of[1] + s - 96;
  if (s < 192) return of[3] + s - 128;
  return of[5] + s - 192;
}

// publish the owned conv blocks (bf16 images in both orientations) and smalls (fp32) from the owner state
template <int T>
__device__ __forceinline__ void publish_conv(const Ctx& x, int i, const TowerState<T>& st) {
  using C = TW<T>;
  uchar* S = x.smem;
  const int tw = T * IM_TOWER;
  // stage: S3 [blk][j][ci][8 o], S2 [j][ci][8 o]
#pragma unroll
  for (int u = 0; u < C::NS; ++u) {
    const Chunk k = chunk_of<T>(i, x.tid + NTH * u);
    if (k.kind == 3) {
      const int blk = T == 0 ? ((k.o0 >> 3) - 2 * i) : 0;
      *(LDS_AS uint32_t*)(S + O_S3 + ((blk * 192 + k.j * 64 + k.ci) * 8 + (k.o0 & 7)) * 2) = pk2(st.p[u][0], st.p[u][1]);
      *(LDS_AS uint32_t*)(S + O_S3 + ((blk * 192 + k.j * 64 + k.ci) * 8 + (k.o0 & 7) + 2) * 2) = pk2(st.p[u][2], st.p[u][3]);
#pragma unroll
      for (int e = 0; e < 4; ++e)
        *lu16(S, O_S3B + (((blk * 3 + k.j) * 8 + (k.o0 & 7) + e) * 64 + k.ci) * 2) = bfu(st.p[u][e]);
    } else if (k.kind == 2) {
      *(LDS_AS uint32_t*)(S + O_S2 + ((k.j * 32 + k.ci) * 8 + (k.o0 & 7)) * 2) = pk2(st.p[u][0], st.p[u][1]);
      *(LDS_AS uint32_t*)(S + O_S2 + ((k.j * 32 + k.ci) * 8 + (k.o0 & 7) + 2) * 2) = pk2(st.p[u][2], st.p[u][3]);
#pragma unroll
      for (int e = 0; e < 4; ++e) *lu16(S, O_S2B + ((k.j * 8 + (k.o0 & 7) + e) * 32 + k.ci) * 2) = bfu(st.p[u][e]);
    } else if (k.kind == 1) {
      st16f(x.rw, WS_SMALL + (T * NSMALL + k.s0) * 4, f4v{st.p[u][0], st.p[u][1], st.p[u][2], st.p[u][3]});
    }
  }
  lbar();
  constexpr int NB3 = T == 0 ? 2 : 1;
  // W3T [j][ci][o]: one 16-B piece (8 o) per (blk, j, ci); W3 [j][o][ci]: 8 pieces (64 ci) per (blk, j, o)
  for (int e = x.tid; e < NB3 * 192 * 2; e += NTH) {
    const int blk = e / 384, r = e % 384;
    const int b3 = T == 0 ? 2 * i + blk : i;
    if (r < 192) {
      const int j = r / 64, ci = r % 64;
      const u32x4 v = *(const LDS_AS u32x4*)(S + O_S3 + (blk * 192 + j * 64 + ci) * 16);
      st16(x.rw, WS_IMG + (tw + IM_W3T + (j * 64 + ci) * 128 + 8 * b3) * 2, v);
    } else {
      const int q = r - 192, j = q / 64, o = (q % 64) >> 3, cc = q & 7;  // 8 o x 8 pieces per j
      st16(x.rw, WS_IMG + (tw + IM_W3 + (j * 128 + 8 * b3 + o) * 64 + 8 * cc) * 2,
           *(const LDS_AS u32x4*)(S + O_S3B + (((blk * 3 + j) * 8 + o) * 64 + 8 * cc) * 2));
    }
  }
  {
    // W2 block b2 (8 output channels), input channels ci0 .. ci0 + nci (labs owners hold half a block)
    const int b2 = T == 0 ? i : (i >> 1), ci0 = T == 0 ? 0 : 16 * (i & 1);
    constexpr int nci = T == 0 ? 32 : 16, npc = nci / 8;
    for (int e = x.tid; e < 3 * nci * 2; e += NTH) {
      if (e < 3 * nci) {
        const int j = e / nci, ci = ci0 + e % nci;
        const u32x4 v = *(const LDS_AS u32x4*)(S + O_S2 + (j * 32 + ci) * 16);
        st16(x.rw, WS_IMG + (tw + IM_W2T + (j * 32 + ci) * 64 + 8 * b2) * 2, v);
      } else {
        const int q = e - 3 * nci, j = q / (8 * npc), o = (q % (8 * npc)) / npc, cc = ci0 / 8 + q % npc;
        st16(x.rw, WS_IMG + (tw + IM_W2 + (j * 64 + 8 * b2 + o) * 32 + 8 * cc) * 2,
             *(const LDS_AS u32x4*)(S + O_S2B + ((j * 8 + o) * 32 + 8 * cc) * 2));
      }
    }
  }
}

template <int T>
__device__ __forceinline__ void tower(const Ctx& x, int i) {
  using C = TW<T>;
  const AflCnn2Args& a = *x.a;
  uchar* S = x.smem;
  int tid = x.tid, lane = x.lane, wave = x.wave, g = lane >> 4, li = lane & 15;
  const int c = x.c, B = a.B;
  const int b0 = i * C::R;
  float* P = a.params + (long)c * a.pstride;
  const int tw = T * IM_TOWER;
  const int pbase = WS_PART + (C::FIRST + i) * PSZ * 4;  // this workgroup's partial (bytes)
  TowerState<T> st;
  // ---------------------------------------------------------------- init: zero LDS, owned state, images
  for (int e = tid; e < T_LDS / 16; e += NTH) *(LDS_AS u32x4*)(S + 16 * e) = u32x4{0u, 0u, 0u, 0u};
#pragma unroll
  for (int u = 0; u < C::NS; ++u) {
    const Chunk k = chunk_of<T>(i, tid + NTH * u);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      st.p[u][e] = k.kind ? P[elem_idx<T>(a, k, e)] : 0.f;
    }
    mv_st(x, u, Z4, Z4);
  }
  lbar();
  publish_conv<T>(x, i, st);
  arrive(x, CT_W + T);
  lbar();
  // re-zero the staging the publishers used (rows 0.. of H1 / H2 / H3)
  for (int e = tid; e < O_XS / 16; e += NTH) *(LDS_AS u32x4*)(S + 16 * e) = u32x4{0u, 0u, 0u, 0u};

  const int min_bs = a.min_bs;
  // the next active step at or after s0 (a.S: none), and this thread's input value of a step (x rows of the
  // read-only table: prefetched one step ahead, during the backward)
  auto next_active = [&](int s0) -> int {
    int s2 = s0;
    for (; s2 < a.S; ++s2) {
      const int b2 = a.bsz[(long)s2 * a.C + c];
      if (b2 >= min_bs && b2 >= 1) break;
    }
    return s2;
  };
  auto load_x = [&](int s2) -> float {
    if (s2 >= a.S || tid >= C::R * C::L) return 0.f;
    const int r = tid / C::L, l = tid - r * C::L, b = b0 + r;
    const int row = b < B ? a.idx[((long)s2 * a.C + c) * B + b] : -1;
    return row >= 0 ? a.rows[(long)row * 24 + C::XOFF + l] : 0.f;
  };
  const int s_first = next_active(0);
  float xv_next = load_x(s_first);
  if (a.thr16 != 0 && s_first < a.S) keep_bytes<T>(a, c, b0, s_first, S, 0, tid);  // (behind the step's first barrier)
  int kact = 0;
  bool alive = true;
  for (int s = 0; s < a.S && alive; ++s) {
    const int bs = a.bsz[(long)s * a.C + c];
    if (bs < min_bs || bs < 1) continue;
    const float xv = xv_next;
    // this step's conv images; the fc1 owners' images are awaited only before their first use (conv3): with the
    // shorter tower backward the fc1 owners finish close to the step start (one poll for both: +1 us per step)
    if (!wait_ge(x, CT_W + T, (uint32_t)(C::NTW * (kact + 1)), O_FLAG)) break;
    REOPQ();
    stamp(x, kact, 0);
    // ------------------------------------------------------------------------------ forward
    // step inputs: x (prefetched), conv1 weights / biases (fp32 smalls)
    int xq = -1;
    if (tid < C::R * C::L) {
      const int r = tid / C::L, l = tid - r * C::L;
      xq = r * C::LP + 1 + l;
    }
    const int o1 = tid & 31;
    float w10, w11, w12, bb1;
    {
      // conv1 weight row o1 (3 floats at 3 o1) and bias: dword sc1 loads through the resource
      const int base = WS_SMALL + (T * NSMALL) * 4;
      w10 = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(x.rw, base + (3 * o1) * 4, 0, 16));
      w11 = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(x.rw, base + (3 * o1 + 1) * 4, 0, 16));
      w12 = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(x.rw, base + (3 * o1 + 2) * 4, 0, 16));
      bb1 = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(x.rw, base + (96 + o1) * 4, 0, 16));
    }
    // conv2 / conv3 B fragments (images) and biases
    const int nt2 = wave & 3, mp2 = wave >> 2;
    s8v w2f[3], w3f[6];
#pragma unroll
    for (int j = 0; j < 3; ++j) w2f[j] = ld16s(x.rw, WS_IMG + (tw + IM_W2 + (j * 64 + 16 * nt2 + li) * 32 + 8 * g) * 2);
#pragma unroll
    for (int k = 0; k < 6; ++k)
      w3f[k] = ld16s(x.rw, WS_IMG + (tw + IM_W3 + ((k >> 1) * 128 + 16 * wave + li) * 64 + 32 * (k & 1) + 8 * g) * 2);
    // (the conv GEMMs run transposed, D[o][q] = W . H^T: a lane ends with 4 consecutive channels of one position,
    // stored as one 8-byte LDS write; its 4 biases come as one 16-byte load)
    const f4v b2v = ld16f(x.rw, WS_SMALL + (T * NSMALL + 128 + 16 * nt2 + 4 * g) * 4);
    const f4v b3v = ld16f(x.rw, WS_SMALL + (T * NSMALL + 192 + 16 * wave + 4 * g) * 4);
    // boundary rows of the activation buffers back to zero (the owner phases stage through them)
    for (int e = tid; e < 18 * 4; e += NTH) {
      const int rr = e % 18, buf = e / 18;
      const int row = rr == 0 ? 0 : 144 + rr;
      const int off = buf == 0 ? O_H1 + row * LD1 * 2 : buf == 1 ? O_H2 + row * LD2 * 2 : buf == 2 ? O_H3 + row * LD3 * 2
                                                                                                   : O_DH2 + row * LD2 * 2;
      const int n16 = buf == 0 ? LD1 / 8 : buf == 2 ? LD3 / 8 : LD2 / 8;
      for (int k = 0; k < n16; ++k) *(LDS_AS u32x4*)(S + off + 16 * k) = u32x4{0u, 0u, 0u, 0u};
    }
    if (xq >= 0) *lf(S, O_XS + (xq + 1) * 4) = xv;
    SYNC();
    // conv1 (1 -> 32) on VALU -> H1 (bf16), pads exact zeros
#pragma unroll
    for (int u = 0; u < 9; ++u) {
      const int q = (tid >> 5) + 16 * u;
      float h = 0.f;
      if (valid_q(q, C::LP)) {
        const float xm = *lf(S, O_XS + q * 4), x0 = *lf(S, O_XS + (q + 1) * 4), xp = *lf(S, O_XS + (q + 2) * 4);
        h = relu(bb1 + w10 * xm + w11 * x0 + w12 * xp);
      }
      *lu16(S, O_H1 + ((q + 1) * LD1 + o1) * 2) = bfu(h);
    }
    SYNC();
#ifndef CNN2_DIAG2
    stamp(x, kact, 7);
#endif
    // conv2: H2[q][o] = relu(b2 + sum_j H1[q - 1 + j] . W2_j^T); wave: n-tile nt2, m-tiles mp2, mp2 + 2, ...
    // (two m-tiles per pass: independent accumulator chains interleave; a tile past 8 computes on zero rows and is
    // not stored)
    for (int mt0 = mp2; mt0 < 9; mt0 += 4) {
      f4v acc[2] = {Z4, Z4};
#pragma unroll
      for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int t = 0; t < 2; ++t) acc[t] = mfma(w2f[j], rfrag(S + O_H1, LD1, 16 * (mt0 + 2 * t) + j, 0, lane), acc[t]);
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int q = 16 * (mt0 + 2 * t) + li;
        if (mt0 + 2 * t < 9)
          *(LDS_AS u32x2v*)(S + O_H2 + ((q + 1) * LD2 + 16 * nt2 + 4 * g) * 2) = relu_pack4(acc[t], b2v, valid_q(q, C::LP));
      }
    }
    // fc1 B fragments (this tower's half of W1, n-tile = wave; the owners' images of this step), issued before
    // conv3: the 128 KB per workgroup take ~2.7 us to issue whatever phase they land in (every tower of every
    // client reads its half at once), and before conv3 they overlap its MFMA / LDS work (fwd 12.2 -> 11.5 us)
    const int par = kact & 1;
    if (!wait_ge(x, CT_W1R, (uint32_t)(NFC1 * (kact + 1)), O_FLAG)) break;
    s8v wf1[16];
#pragma unroll
    for (int k = 0; k < 16; ++k)
      wf1[k] = ld16s(x.rw, WS_IMG + (IM_W1 + par * IM_FC1PAR + (16 * wave + li) * 1024 + C::COL0 + 32 * k + 8 * g) * 2);
    SYNC();
    stamp(x, kact, 14);
    // conv3: wave = n-tile, all 9 m-tiles
    // (three m-tiles per pass, interleaved accumulator chains)
#pragma unroll
    for (int mt0 = 0; mt0 < 9; mt0 += 3) {
      f4v acc[3] = {Z4, Z4, Z4};
#pragma unroll
      for (int k = 0; k < 6; ++k)
#pragma unroll
        for (int t = 0; t < 3; ++t)
          acc[t] = mfma(w3f[k], rfrag(S + O_H2, LD2, 16 * (mt0 + t) + (k >> 1), 32 * (k & 1), lane), acc[t]);
#pragma unroll
      for (int t = 0; t < 3; ++t) {
        const int q = 16 * (mt0 + t) + li;
        *(LDS_AS u32x2v*)(S + O_H3 + ((q + 1) * LD3 + 16 * wave + 4 * g) * 2) = relu_pack4(acc[t], b3v, valid_q(q, C::LP));
      }
    }
    SYNC();
    stamp(x, kact, 8);
    // AdaptiveAvgPool1d(4) + dropout -> feat (LDS bf16 rows 0..15, zero past R) and the global concat.  Thread:
    // (row r, channel pair cp) = 8 concat columns 8 cp .. 8 cp + 7: the channel pair moves as one dword per
    // position, the bins are compile-time, the 8 keep bits (4 hashes) are kept as one LDS byte for the backward
    const bool dr = a.thr16 != 0;
#pragma unroll
    for (int it = 0; it < 16 * 64 / NTH; ++it) {
      const int e = tid + NTH * it, r = e >> 6, cp = e & 63;
      float f[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) f[k] = 0.f;
      if (r < C::R) {
        float h0[C::L], h1v[C::L];
#pragma unroll
        for (int l = 0; l < C::L; ++l) {
          const uint32_t w = *(const LDS_AS uint32_t*)(S + O_H3 + ((r * C::LP + 2 + l) * LD3 + 2 * cp) * 2);
          h0[l] = __uint_as_float(w << 16);
          h1v[l] = __uint_as_float(w & 0xFFFF0000u);
        }
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          float s0 = 0.f, s1 = 0.f;
#pragma unroll
          for (int l = bin_lo(p, C::L); l < bin_hi(p, C::L); ++l) {
            s0 += h0[l];
            s1 += h1v[l];
          }
          f[p] = s0 * bin_rcp(p, C::L);
          f[4 + p] = s1 * bin_rcp(p, C::L);
        }
        if (dr) {
          const uint32_t kb = *(const LDS_AS uchar*)(S + O_RED + (R_KEEP + 256 * par) * 4 + r * 64 + cp);
#pragma unroll
          for (int k = 0; k < 8; ++k) f[k] *= ((kb >> k) & 1u) ? a.inv_keep : 0.f;
        }
      }
      const u32x4 pkd = u32x4{pk2(f[0], f[1]), pk2(f[2], f[3]), pk2(f[4], f[5]), pk2(f[6], f[7])};
      *(LDS_AS u32x4*)(S + O_FT + (r * LDF + 8 * cp) * 2) = pkd;
      if (r < C::R) st16(x.rw, WS_FEAT + par * FEAT_PAR + ((b0 + r) * 1024 + C::COL0 + 8 * cp) * 2, pkd);
    }
    SYNC();
    stamp(x, kact, 9);
    // fc1 partial over this tower's 512 features: z1p[rows][n], wave = n-tile
    {
      f4v acc = Z4;
#pragma unroll
      for (int k = 0; k < 16; ++k) acc = mfma(rfrag(S + O_FT, LDF, 0, 32 * k, lane), wf1[k], acc);
#pragma unroll
      for (int e = 0; e < 4; ++e) *lf(S, O_ZS + ((4 * g + e) * LDZ + 16 * wave + li) * 4) = acc[e];
    }
    SYNC();
    for (int e = tid; e < C::R * 32; e += NTH) {
      const int r = e >> 5, pc = e & 31;
      const f4v v = *(const LDS_AS f4v*)(S + O_ZS + (r * LDZ + 4 * pc) * 4);
      st16f(x.rw, WS_Z1P + ((T * 128 + b0 + r) * 128 + 4 * pc) * 4, v);
    }
    arrive(x, CT_FW + (T == 0 ? i : (i >> 1)));  // (per head wave: it starts on its own rows' partials)
    REOPQ();
    stamp(x, kact, 1);
    const int s_next = next_active(s + 1);
    xv_next = load_x(s_next);
    // d(concat) B fragments (W1T, this tower's columns: n-tiles 4 w .. 4 w + 3) in flight during the wait
    s8v wt1[16];
#pragma unroll
    for (int k = 0; k < 16; ++k)
      wt1[k] = ld16s(x.rw, WS_IMG + (IM_W1T + par * IM_FC1PAR + (C::COL0 + 16 * (4 * wave + (k >> 2)) + li) * 128 +
                                    32 * (k & 3) + 8 * g) * 2);
    // the W3T / W2T fragments of the backward too, issued while the tower only waits for the head (their ~2 us
    // of issue landed in the d1 + dfeat and dh2 phases: tower backward 15.1 -> 13.0 us)
    const int nb2 = wave & 3, mpb = wave >> 2;
    s8v w3t[12];
#pragma unroll
    for (int k = 0; k < 12; ++k)
      w3t[k] = ld16s(x.rw, WS_IMG + (tw + IM_W3T + ((k >> 2) * 64 + 16 * nb2 + li) * 128 + 32 * (k & 3) + 8 * g) * 2);
    const int nb1 = wave & 1, mpa = wave >> 1;
    s8v w2t[6];
#pragma unroll
    for (int k = 0; k < 6; ++k)
      w2t[k] = ld16s(x.rw, WS_IMG + (tw + IM_W2T + ((k >> 1) * 32 + 16 * nb1 + li) * 64 + 32 * (k & 1) + 8 * g) * 2);
    // the next step's dropout keep bytes, hashed while the head works (the other parity's buffer; read after the
    // barriers of the wait below and of the next step)
    if (dr && s_next < a.S) keep_bytes<T>(a, c, b0, s_next, S, par ^ 1, tid);
    // ------------------------------------------------------------------------------ backward
    const int hw = T == 0 ? i : (i >> 1);  // the head wave that computes this workgroup's d1 rows
    if (!wait_ge(x, CT_HW + hw, (uint32_t)(kact + 1), O_FLAG)) break;
    REOPQ();
    stamp(x, kact, 2);
    {
      const u32x4 stt = ld16(x.rw, WS_STAT + 16 * hw);
      if (stt[0] != 0u) {  // NaN loss: the client's round ends here without an update (the head saw it too)
        alive = false;
        break;
      }
    }
    // own d1 rows -> LDS (rows >= R zero)
    if (tid < 16 * 16) {
      const int r = tid >> 4, pc = tid & 15;
      u32x4 v = u32x4{0u, 0u, 0u, 0u};
      if (r < C::R) v = ld16(x.rw, WS_D1 + ((b0 + r) * 128 + 8 * pc) * 2);
      *(LDS_AS u32x4*)(S + O_D1R + (r * LDD + 8 * pc) * 2) = v;
    }
    SYNC();
    // dfeat = d1 . W1[:, tower cols] -> f32 [16][516]
    {
      f4v acc[4] = {Z4, Z4, Z4, Z4};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const s8v af = rfrag(S + O_D1R, LDD, 0, 32 * k, lane);
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[t] = mfma(af, wt1[4 * t + k], acc[t]);
      }
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int e = 0; e < 4; ++e) *lf(S, O_FT + ((4 * g + e) * 516 + 16 * (4 * wave + t) + li) * 4) = acc[t][e];
    }
    SYNC();
    stamp(x, kact, 10);
    // dh3 = relu'(h3) * pool'(dropout'(dfeat)), in place over H3 (bf16).  Thread: (row r, channel pair cp) like the
    // forward pooling (keep byte from the forward, compile-time bins); conv3 bias partials per (row group, channel)
    float b0s = 0.f, b1s = 0.f;
    const int cp = tid & 63;
#pragma unroll
    for (int it = 0; it < C::R * 64 / NTH; ++it) {
      const int r = (tid >> 6) + 8 * it;
      const uint32_t kb = *(const LDS_AS uchar*)(S + O_RED + (R_KEEP + 256 * par) * 4 + r * 64 + cp);
      const f4v d0 = *(const LDS_AS f4v*)(S + O_FT + (r * 516 + 8 * cp) * 4);
      const f4v d1 = *(const LDS_AS f4v*)(S + O_FT + (r * 516 + 8 * cp + 4) * 4);
      float gq[8];
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        gq[p] = d0[p] * bin_rcp(p, C::L);
        gq[4 + p] = d1[p] * bin_rcp(p, C::L);
      }
      if (dr) {
#pragma unroll
        for (int k = 0; k < 8; ++k) gq[k] *= ((kb >> k) & 1u) ? a.inv_keep : 0.f;
      }
#pragma unroll
      for (int l = 0; l < C::L; ++l) {
        float v0 = 0.f, v1 = 0.f;
#pragma unroll
        for (int p = 0; p < 4; ++p)
          if (l >= bin_lo(p, C::L) && l < bin_hi(p, C::L)) {
            v0 += gq[p];
            v1 += gq[4 + p];
          }
        LDS_AS uint32_t* hp = (LDS_AS uint32_t*)(S + O_H3 + ((r * C::LP + 2 + l) * LD3 + 2 * cp) * 2);
        const uint32_t w = *hp;
        v0 = __uint_as_float(w << 16) > 0.f ? v0 : 0.f;
        v1 = __uint_as_float(w & 0xFFFF0000u) > 0.f ? v1 : 0.f;
        *hp = pk2(v0, v1);
        b0s += v0;
        b1s += v1;
      }
    }
    *(LDS_AS f2v*)(S + O_RED + (R_DB3 + (tid >> 6) * 128 + 2 * cp) * 4) = f2v{b0s, b1s};
    SYNC();
    stamp(x, kact, 11);
    // dh2 = relu'(h2) * sum_j shift_{1-j}(dh3) . W3_j  (K = 3 x 128): wave n-tile nb2, m-tiles mpb, mpb + 2, ..
    // (transposed: D[ci][q], 4 consecutive channels of one position per lane, 8-byte LDS accesses)
    {
      f4v cs = Z4;
      for (int mt0 = mpb; mt0 < 9; mt0 += 4) {
        f4v acc[2] = {Z4, Z4};
#pragma unroll
        for (int k = 0; k < 12; ++k)
#pragma unroll
          for (int t = 0; t < 2; ++t)
            acc[t] = mfma(w3t[k], rfrag(S + O_H3, LD3, 16 * (mt0 + 2 * t) + 2 - (k >> 2), 32 * (k & 3), lane), acc[t]);
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          if (mt0 + 2 * t >= 9) continue;
          const int q = 16 * (mt0 + 2 * t) + li;
          const u32x2v hw = *(const LDS_AS u32x2v*)(S + O_H2 + ((q + 1) * LD2 + 16 * nb2 + 4 * g) * 2);
          float v[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const uint32_t h = hw[e >> 1];
            v[e] = __uint_as_float((e & 1) ? (h & 0xFFFF0000u) : (h << 16)) > 0.f ? acc[t][e] : 0.f;
            cs[e] += v[e];
          }
          *(LDS_AS u32x2v*)(S + O_DH2 + ((q + 1) * LD2 + 16 * nb2 + 4 * g) * 2) = u32x2v{pk2(v[0], v[1]), pk2(v[2], v[3])};
        }
      }
#pragma unroll
      for (int o = 1; o <= 8; o <<= 1)
#pragma unroll
        for (int e = 0; e < 4; ++e) cs[e] += __shfl_xor(cs[e], o, 64);
      if (li == 0) *(LDS_AS f4v*)(S + O_RED + (R_DB2 + wave * 16 + 4 * g) * 4) = cs;
    }
    SYNC();
    stamp(x, kact, 12);
    // dh1 = relu'(h1) * sum_j shift_{1-j}(dh2) . W2_j (K = 3 x 64), straight into the conv1 gradients
    {
      f4v s0 = Z4, s1 = Z4, s2 = Z4, sb = Z4;  // per channel 4 g + e of the tile
      f4v accs[3] = {Z4, Z4, Z4};
#pragma unroll
      for (int k = 0; k < 6; ++k)
#pragma unroll
        for (int t = 0; t < 3; ++t)
          accs[t] = mfma(w2t[k], rfrag(S + O_DH2, LD2, 16 * (mpa + 4 * t) + 2 - (k >> 1), 32 * (k & 1), lane), accs[t]);
#pragma unroll
      for (int t = 0; t < 3; ++t) {
        const int mt = mpa + 4 * t;
        if (mt >= 9) continue;
        const f4v acc = accs[t];
        const int q = 16 * mt + li;
        const u32x2v hw = *(const LDS_AS u32x2v*)(S + O_H1 + ((q + 1) * LD1 + 16 * nb1 + 4 * g) * 2);
        const float xm = *lf(S, O_XS + q * 4), x0 = *lf(S, O_XS + (q + 1) * 4), xp = *lf(S, O_XS + (q + 2) * 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const uint32_t h = hw[e >> 1];
          const float d = __uint_as_float((e & 1) ? (h & 0xFFFF0000u) : (h << 16)) > 0.f ? acc[e] : 0.f;
          s0[e] += d * xm;
          s1[e] += d * x0;
          s2[e] += d * xp;
          sb[e] += d;
        }
      }
#pragma unroll
      for (int o = 1; o <= 8; o <<= 1)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          s0[e] += __shfl_xor(s0[e], o, 64);
          s1[e] += __shfl_xor(s1[e], o, 64);
          s2[e] += __shfl_xor(s2[e], o, 64);
          sb[e] += __shfl_xor(sb[e], o, 64);
        }
      if (li == 0)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          *(LDS_AS f4v*)(S + O_RED + (R_C1 + (wave * 16 + 4 * g + e) * 4) * 4) = f4v{s0[e], s1[e], s2[e], sb[e]};
    }
#ifdef CNN2_DIAG2  // sub-phases of the dh1 + dW phase (slot 15: dh1 done; slot 7: dW3 done)
    stamp(x, kact, 15);
#endif
    // dW3_j = dh3^T . shift_{j-1}(h2) (K = 160 rows: 144 + zero rows).  Wave: o-tiles 2 (w & 3) + {0, 1} x six of
    // the twelve (tap, ci-tile) blocks (w >> 2 picks the half): per k-step 2 + 6 transposed fragment reads for 12
    // MFMAs (was 1 + 12 with one o-tile per wave)
    {
      const int ob = 2 * (wave & 3), tb = 6 * (wave >> 2);
      f4v acc[2][6];
#pragma unroll
      for (int oi = 0; oi < 2; ++oi)
#pragma unroll
        for (int t = 0; t < 6; ++t) acc[oi][t] = Z4;
      for (int ks = 0; ks < 5; ++ks) {
        const s8v a0 = cfrag(S + O_H3 + LD3 * 2, LD3, 32 * ks, 16 * ob, lane);
        const s8v a1 = cfrag(S + O_H3 + LD3 * 2, LD3, 32 * ks, 16 * (ob + 1), lane);
#pragma unroll
        for (int t = 0; t < 6; ++t) {
          const int j = (tb + t) >> 2, ct = (tb + t) & 3;
          const s8v bf = cfrag(S + O_H2 + j * LD2 * 2, LD2, 32 * ks, 16 * ct, lane);
          acc[0][t] = mfma(a0, bf, acc[0][t]);
          acc[1][t] = mfma(a1, bf, acc[1][t]);
        }
      }
#pragma unroll
      for (int oi = 0; oi < 2; ++oi)
#pragma unroll
        for (int t = 0; t < 6; ++t) {
          const int j = (tb + t) >> 2, ci = 16 * ((tb + t) & 3) + li;
          st16f(x.rw, pbase + (P_W3 + ((j * 16 + 2 * (ob + oi) + (g >> 1)) * 64 + ci) * 8 + 4 * (g & 1)) * 4, acc[oi][t]);
        }
    }
#ifdef CNN2_DIAG2
    stamp(x, kact, 7);
#endif
    // dW2_j = dh2^T . shift_{j-1}(h1): wave -> o-tile (w & 3), ci-tile (w >> 2)
    {
      const int ot = wave & 3, ct = wave >> 2;
      f4v acc[3] = {Z4, Z4, Z4};
      for (int ks = 0; ks < 5; ++ks) {
        const s8v af = cfrag(S + O_DH2 + LD2 * 2, LD2, 32 * ks, 16 * ot, lane);
#pragma unroll
        for (int j = 0; j < 3; ++j) acc[j] = mfma(af, cfrag(S + O_H1 + j * LD1 * 2, LD1, 32 * ks, 16 * ct, lane), acc[j]);
      }
#pragma unroll
      for (int j = 0; j < 3; ++j)
        st16f(x.rw, pbase + (P_W2 + ((j * 8 + 2 * ot + (g >> 1)) * 32 + 16 * ct + li) * 8 + 4 * (g & 1)) * 4, acc[j]);
    }
    SYNC();
    stamp(x, kact, 13);
    // small partials: conv1 W [o][j] (96) | conv1 b (32) | conv2 b (64) | conv3 b (128), waves summed in order
    if (tid < NSMALL) {
      float v = 0.f;
      if (tid < 128) {
        const int o = tid < 96 ? tid / 3 : tid - 96, comp = tid < 96 ? tid % 3 : 3;
        const int nt = o >> 4;
        for (int w = nt; w < 8; w += 2) v += *lf(S, O_RED + (R_C1 + (w * 16 + (o & 15)) * 4 + comp) * 4);
      } else if (tid < 192) {
        const int o = tid - 128;
        v = *lf(S, O_RED + (R_DB2 + (o >> 4) * 16 + (o & 15)) * 4) + *lf(S, O_RED + (R_DB2 + ((o >> 4) + 4) * 16 + (o & 15)) * 4);
      } else {
        const int o = tid - 192;
#pragma unroll
        for (int rg = 0; rg < 8; ++rg) v += *lf(S, O_RED + (R_DB3 + 128 * rg + o) * 4);
      }
      *lf(S, O_RED + (R_SM + tid) * 4) = v;
    }
    SYNC();
    if (tid < NSMALL / 4) st16f(x.rw, pbase + (P_SM + 4 * tid) * 4, *(const LDS_AS f4v*)(S + O_RED + (R_SM + 4 * tid) * 4));
    arrive(x, CT_P + T);
    REOPQ();
    stamp(x, kact, 3);
    if (!wait_ge(x, CT_P + T, (uint32_t)(C::NTW * (kact + 1)), O_FLAG)) break;
    REOPQ();
    stamp(x, kact, 4);
    // ------------------------------------------------------------------ owner: conv blocks
    const AdamT ak = adam_t(a.lr, kact + 1, a.opt_mode);
    {
      f4v gsum[C::NS], mm[C::NS], vv[C::NS];
      Chunk ks[C::NS];
#pragma unroll
      for (int u = 0; u < C::NS; ++u) {
        ks[u] = chunk_of<T>(i, tid + NTH * u);
        gsum[u] = Z4;
        mv_ld(x, u, mm[u], vv[u]);
      }
      // every partial chunk of the owned slots in flight at once (owned-less slots read chunk 0 and drop it),
      // then summed in workgroup order
      f4v pv[C::NS][C::NTW];
#pragma unroll
      for (int u = 0; u < C::NS; ++u)
#pragma unroll
        for (int n = 0; n < C::NTW; ++n) pv[u][n] = ld16f(x.rw, WS_PART + ((C::FIRST + n) * PSZ + ks[u].poff) * 4);
#pragma unroll
      for (int u = 0; u < C::NS; ++u)
#pragma unroll
        for (int n = 0; n < C::NTW; ++n) gsum[u] += pv[u][n];
#ifdef CNN2_DIAG
      drain();
      stamp(x, kact, 15);
#endif
#pragma unroll
      for (int u = 0; u < C::NS; ++u) {
        if (ks[u].kind == 0) continue;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float me = mm[u][e], ve = vv[u][e];
          st.p[u][e] = adam1(st.p[u][e], me, ve, gsum[u][e], ak);
          mm[u][e] = me;
          vv[u][e] = ve;
        }
        mv_st(x, u, mm[u], vv[u]);
      }
    }
    publish_conv<T>(x, i, st);
    REOPQ();
    stamp(x, kact, 5);
    arrive(x, CT_W + T);
    stamp(x, kact, 6);
    ++kact;
  }
  // ---------------------------------------------------------------- round end: owned parameters -> arena
#pragma unroll
  for (int u = 0; u < C::NS; ++u) {
    const Chunk k = chunk_of<T>(i, tid + NTH * u);
    if (k.kind == 0) continue;
#pragma unroll
    for (int e = 0; e < 4; ++e) P[elem_idx<T>(a, k, e)] = st.p[u][e];
  }
}

// ============================================================================================== head
// LDS map (bytes)
constexpr int H_L1 = 136, H_L2 = 72, H_L3 = 40, H_F3 = 36;  // f3 rows 16-B aligned
constexpr int H_F1S = 0;
constexpr int H_W2S = H_F1S + 128 * H_L1 * 2;
constexpr int H_W3S = H_W2S + 64 * H_L1 * 2;
constexpr int H_F2S = H_W3S + 32 * H_L2 * 2;
constexpr int H_F3F = H_F2S + 128 * H_L2 * 2;
constexpr int H_D3S = H_F3F + 128 * H_F3 * 4;
constexpr int H_D2S = H_D3S + 128 * H_L3 * 2;
constexpr int H_DZ = H_D2S + 128 * H_L2 * 2;
constexpr int H_RED = H_DZ + 128 * 4;
constexpr int H_WO = H_RED + 8 * 4;
constexpr int H_RED3W = H_WO + 32 * 4;
constexpr int H_GBW = H_RED3W + 8 * 72 * 4;
constexpr int H_BIAS = H_GBW + 8 * 192 * 4;  // b1 [128] | b2 [64] | b3 [32] | bo [4]
constexpr int H_SUMS = H_BIAS + 228 * 4;      // gb2 [64] | gb3 [32] | gWo [32] | gbo [1] | gb1 [128]
constexpr int H_FLAG = H_SUMS + 260 * 4;
constexpr int H_LDS = H_FLAG + 16;
constexpr int LDS_TOTAL = T_LDS > H_LDS ? T_LDS : H_LDS;
static_assert(LDS_TOTAL <= 160 * 1024, "cnn2 LDS");

__device__ __forceinline__ float wsum(float x) {
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
  return x;
}

__device__ __forceinline__ void head(const Ctx& x) {
  const AflCnn2Args& a = *x.a;
  uchar* S = x.smem;
  int tid = x.tid, lane = x.lane, wave = x.wave, g = lane >> 4, li = lane & 15;
  const int c = x.c, B = a.B;
  float* P = a.params + (long)c * a.pstride;
  const int oW2 = a.off[14], ob2 = a.off[15], oW3 = a.off[16], ob3 = a.off[17], oWo = a.off[18], obo = a.off[19],
            ob1 = a.off[13];
  LDS_AS unsigned short* f1s = lu16(S, H_F1S);
  LDS_AS unsigned short* W2s = lu16(S, H_W2S);
  LDS_AS unsigned short* W3s = lu16(S, H_W3S);
  LDS_AS unsigned short* f2s = lu16(S, H_F2S);
  LDS_AS float* f3f = lf(S, H_F3F);
  LDS_AS unsigned short* d3s = lu16(S, H_D3S);
  LDS_AS unsigned short* d2s = lu16(S, H_D2S);
  LDS_AS float* dz = lf(S, H_DZ);
  LDS_AS float* red = lf(S, H_RED);
  LDS_AS float* wos = lf(S, H_WO);
  LDS_AS float* red3w = lf(S, H_RED3W);
  LDS_AS float* gbw = lf(S, H_GBW);
  LDS_AS float* bias = lf(S, H_BIAS);
  LDS_AS float* sums = lf(S, H_SUMS);
  // persistent Adam state: dW2 elements (o = 16 (w >> 1) + 4 g + e, i = 16 (4 (w & 1) + j) + li), dW3 elements
  // (o = 16 (w >> 2) + 4 g + e, i = 16 (w & 3) + li), one vector entry per thread < 257
  float p2[16], p3[4], pv = 0.f;  // moments in slab slots 0..3 (W2), 4 (W3), 5 (vector entry)
  const int o2b = 16 * (wave >> 1) + 4 * g, i2b = 16 * 4 * (wave & 1) + li;
  const int o3b = 16 * (wave >> 2) + 4 * g, i3 = 16 * (wave & 3) + li;
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      p2[4 * j + e] = P[oW2 + (o2b + e) * 128 + i2b + 16 * j];
    }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    p3[e] = P[oW3 + (o3b + e) * 64 + i3];
  }
  for (int k = 0; k < 6; ++k) mv_st(x, k, Z4, Z4);
  auto vidx = [&](int t) -> int {  // arena index of vector entry t
    return t < 64 ? ob2 + t : t < 96 ? ob3 + t - 64 : t < 128 ? oWo + t - 96 : t == 128 ? obo : ob1 + t - 129;
  };
  if (tid < 257) pv = P[vidx(tid)];
  // LDS images / vectors from the state
  auto put_state = [&]() {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) W2s[(o2b + e) * H_L1 + i2b + 16 * j] = bfu(p2[4 * j + e]);
#pragma unroll
    for (int e = 0; e < 4; ++e) W3s[(o3b + e) * H_L2 + i3] = bfu(p3[e]);
    if (tid < 257) {
      if (tid < 64) bias[128 + tid] = pv;
      else if (tid < 96) bias[192 + tid - 64] = pv;
      else if (tid < 128) wos[tid - 96] = pv;
      else if (tid == 128) bias[224] = pv;
      else bias[tid - 129] = pv;
    }
  };
  put_state();
  lbar();

  const int min_bs = a.min_bs;
  int kact = 0;
  bool nan_seen = false;  // the last finished step's batch loss was NaN (abort at the next step's start)
  for (int s = 0; s < a.S; ++s) {
    const int bs = a.bsz[(long)s * a.C + c];
    if (bs < min_bs || bs < 1) continue;
    const int ep = a.epoch[(long)s * a.C + c], nbc = a.nb[c];
    const int* idxs = a.idx + ((long)s * a.C + c) * B;
    // Every phase up to the d1 hand-off is ROW-LOCAL: wave w owns batch rows m0 = 16 w .. m0 + 15 from the z1 sum
    // to its d1 rows, so the critical path has ONE workgroup barrier (the batch loss, for the NaN abort); the
    // cross-row sums (bias / output-layer gradients, dW2, dW3) run after the hand-off, under the towers' backward.
    const int m0 = wave * 16;
    const int yb = min(m0 + li, B - 1);
    const int yrow = idxs[yb];
    const float yv = yrow >= 0 ? a.rows[(long)yrow * 24 + 23] : 0.f;
    if (nan_seen) {  // the previous step's loss was NaN: status only, the client's round ends (towers read it)
      if (tid == 0) {
        for (int w = 0; w < 8; ++w) st16(x.rw, WS_STAT + 16 * w, u32x4{1u, (uint32_t)s, 0u, 0u});
        a.failed[c] = 1;
      }
      arrive(x, CT_H);
      if (tid == 0)
        for (int w = 0; w < 8; ++w) __hip_atomic_fetch_add(x.ctr + (CT_HW + w) * 32, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      break;
    }
    if (!wait_wave(x, CT_FW + wave, 3u * (uint32_t)(kact + 1))) break;  // 1 vitals + 2 labs tower workgroups
    REOPQ();
    stamp(x, kact, 0);
    // z1 = z1p_vitals + z1p_labs (+ b1, ReLU) -> f1s rows of this wave; lane: row m0 + (lane >> 2), columns
    // 16 q + 4 (lane & 3) .. +3
    {
      const int b = m0 + (lane >> 2), i0 = 4 * (lane & 3);
      f4v za[8], zb[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        za[q] = ld16f(x.rw, WS_Z1P + (b * 128 + 16 * q + i0) * 4);
        zb[q] = ld16f(x.rw, WS_Z1P + ((128 + b) * 128 + 16 * q + i0) * 4);
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int i1 = 16 * q + i0;
        const f4v bb = *(const LDS_AS f4v*)(bias + i1);
        float v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = b < B ? relu((za[q][k] + zb[q][k]) + bb[k]) : 0.f;
        *(LDS_AS u32x2v*)(f1s + b * H_L1 + i1) = u32x2v{pk2(v[0], v[1]), pk2(v[2], v[3])};
      }
    }
    stamp(x, kact, 3);
    // fc2 (transposed, D[n][m] = W2 . f1^T: a lane ends with 4 consecutive features of one row)
    {
      f4v acc[4] = {Z4, Z4, Z4, Z4};
#pragma unroll
      for (int k0 = 0; k0 < 128; k0 += 32) {
        const s8v bf = rfrag(S + H_F1S, H_L1, m0, k0, lane);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = mfma(rfrag(S + H_W2S, H_L1, 16 * j, k0, lane), bf, acc[j]);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const f4v bv = *(const LDS_AS f4v*)(bias + 128 + 16 * j + 4 * g);
        *(LDS_AS u32x2v*)(f2s + (m0 + li) * H_L2 + 16 * j + 4 * g) =
            u32x2v{pk2(relu(acc[j][0] + bv[0]), relu(acc[j][1] + bv[1])), pk2(relu(acc[j][2] + bv[2]), relu(acc[j][3] + bv[3]))};
      }
    }
    // fc3 (transposed: one 16-byte store of 4 features per lane)
    {
      f4v acc[2] = {Z4, Z4};
#pragma unroll
      for (int k0 = 0; k0 < 64; k0 += 32) {
        const s8v bf = rfrag(S + H_F2S, H_L2, m0, k0, lane);
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[j] = mfma(rfrag(S + H_W3S, H_L2, 16 * j, k0, lane), bf, acc[j]);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const f4v bv = *(const LDS_AS f4v*)(bias + 192 + 16 * j + 4 * g);
        *(LDS_AS f4v*)(f3f + (m0 + li) * H_F3 + 16 * j + 4 * g) =
            f4v{relu(acc[j][0] + bv[0]), relu(acc[j][1] + bv[1]), relu(acc[j][2] + bv[2]), relu(acc[j][3] + bv[3])};
      }
    }
    stamp(x, kact, 4);
    // output logit (lane: row m0 + li, features 8 g .. 8 g + 7, summed over the 4 lane groups) + sigmoid-BCE
    // (k_bce arithmetic); d3 = dz wo^T * relu'(f3) for the same 8 features
    const int row = m0 + li;
    float gz = 0.f, lb = 0.f;
    {
      const f4v f0 = *(const LDS_AS f4v*)(f3f + row * H_F3 + 8 * g), f1 = *(const LDS_AS f4v*)(f3f + row * H_F3 + 8 * g + 4);
      const f4v w0 = *(const LDS_AS f4v*)(wos + 8 * g), w1 = *(const LDS_AS f4v*)(wos + 8 * g + 4);
      float acc = 0.f;
#pragma unroll
      for (int k = 0; k < 4; ++k) acc += f0[k] * w0[k];
#pragma unroll
      for (int k = 0; k < 4; ++k) acc += f1[k] * w1[k];
      acc += __shfl_xor(acc, 16, 64);
      acc += __shfl_xor(acc, 32, 64);
      const float zl = bias[224] + acc;
      if (row < bs) {
        const float p = 1.f / (1.f + expf(-zl));
        if (g == 0) {
          lb = -(yv * fmaxf(logf(p), -100.f) + (1.f - yv) * fmaxf(log1pf(-p), -100.f));
          if (p != p) lb = p;
        }
        const float w = p * (1.f - p);
        gz = (p - yv) / fmaxf(w, 1e-12f) * w / (float)bs;
      }
      if (g == 0) dz[row] = gz;
      const float f[8] = {f0[0], f0[1], f0[2], f0[3], f1[0], f1[1], f1[2], f1[3]};
      const float wv[8] = {w0[0], w0[1], w0[2], w0[3], w1[0], w1[1], w1[2], w1[3]};
      uint32_t d3[4];
#pragma unroll
      for (int k = 0; k < 4; ++k)
        d3[k] = pk2(f[2 * k] > 0.f ? gz * wv[2 * k] : 0.f, f[2 * k + 1] > 0.f ? gz * wv[2 * k + 1] : 0.f);
      *(LDS_AS u32x4*)(d3s + row * H_L3 + 8 * g) = u32x4{d3[0], d3[1], d3[2], d3[3]};
    }
    lb = wsum(lb);
    if (lane == 0) red[wave] = lb;
    stamp(x, kact, 5);
    // d2 = d3 . W3 * relu'(f2) (rows of this wave); gb2 partials per wave
    {
      const s8v af = rfrag(S + H_D3S, H_L3, m0, 0, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const f4v acc = mfma(af, cfrag(S + H_W3S, H_L2, 0, 16 * j, lane), Z4);
        const int n = 16 * j + li;
        float cs = 0.f;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int m = m0 + 4 * g + e;
          const unsigned short fb = f2s[m * H_L2 + n];
          const float v = (fb != 0 && !(fb & 0x8000)) ? acc[e] : 0.f;
          d2s[m * H_L2 + n] = bfu(v);
          cs += v;
        }
        cs += __shfl_xor(cs, 16, 64);
        cs += __shfl_xor(cs, 32, 64);
        if (lane < 16) gbw[wave * 192 + n] = cs;
      }
    }
    // d1^T = W2^T . d2^T * relu'(f1) (transposed: 4 consecutive features of one row per lane -> one 8-byte
    // write-through store each, no LDS staging), held until the batch loss is known
    uint32_t d1p[16];
    {
      const s8v b0 = rfrag(S + H_D2S, H_L2, m0, 0, lane), b1 = rfrag(S + H_D2S, H_L2, m0, 32, lane);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        f4v acc = mfma(cfrag(S + H_W2S, H_L1, 0, 16 * j, lane), b0, Z4);
        acc = mfma(cfrag(S + H_W2S, H_L1, 32, 16 * j, lane), b1, acc);
        const u32x2v fb = *(const LDS_AS u32x2v*)(f1s + row * H_L1 + 16 * j + 4 * g);
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const uint32_t h = (fb[e >> 1] >> (16 * (e & 1))) & 0xFFFFu;
          v[e] = (h != 0 && !(h & 0x8000u)) ? acc[e] : 0.f;
        }
        d1p[2 * j] = pk2(v[0], v[1]);
        d1p[2 * j + 1] = pk2(v[2], v[3]);
      }
    }
    // the d1 rows go out BEFORE the loss barrier (the write-through stores drain while the waves meet); the
    // towers read them only after this wave's counter, i.e. after the status word says the loss was not NaN
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      __builtin_amdgcn_raw_buffer_store_b64(u32x2v{d1p[2 * j], d1p[2 * j + 1]}, x.rw,
                                            WS_D1 + (row * 128 + 16 * j + 4 * g) * 2, 0, 16);
      sguard();
    }
    stamp(x, kact, 6);
    // per-wave hand-off with NO workgroup barrier: this wave's status slot, drained with its d1 rows, then its
    // counter — the tower workgroups of those rows start without waiting for the other waves.  The batch loss
    // (and its NaN test) is summed after the hand-off; a NaN step is caught at the next step's start, where
    // the abort goes out through the same status slots (the failed client's round is discarded either way:
    // the reference's client.py:100-102 abort, one step later on the device)
    if (lane == 0) st16(x.rw, WS_STAT + 16 * wave, u32x4{0u, (uint32_t)s, 0u, 0u});
    drain();
    stamp(x, kact, 8);
    if (lane == 0) __hip_atomic_fetch_add(x.ctr + (CT_HW + wave) * 32, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    arrive(x, CT_H);
    REOPQ();
    stamp(x, kact, 1);
    {
      const float loss = ((red[0] + red[1]) + (red[2] + red[3]) + ((red[4] + red[5]) + (red[6] + red[7]))) / (float)max(bs, 1);
      if (a.nan_abort && loss != loss) nan_seen = true;
      if (tid == 0) a.losses[(long)c * a.E + ep] += loss / (float)nbc;
    }
    // ---- off the critical path: gb1 (d1 again in the row-major layout for its column sums), output-layer /
    // fc3 / fc2 bias sums, dW3
    {
      const s8v a0 = rfrag(S + H_D2S, H_L2, m0, 0, lane), a1 = rfrag(S + H_D2S, H_L2, m0, 32, lane);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        f4v acc = mfma(a0, cfrag(S + H_W2S, H_L1, 0, 16 * j, lane), Z4);
        acc = mfma(a1, cfrag(S + H_W2S, H_L1, 32, 16 * j, lane), acc);
        const int n = 16 * j + li;
        float cs = 0.f;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int m = m0 + 4 * g + e;
          const unsigned short fb = f1s[m * H_L1 + n];
          cs += (fb != 0 && !(fb & 0x8000)) ? acc[e] : 0.f;
        }
        cs += __shfl_xor(cs, 16, 64);
        cs += __shfl_xor(cs, 32, 64);
        if (lane < 16) gbw[wave * 192 + 64 + n] = cs;
      }
    }
    SYNC();
    {
      const int j = tid & 31, r0 = 8 * (tid >> 5);
      float sa = 0.f, sw = 0.f, sz = 0.f;
#pragma unroll
      for (int bb = 0; bb < 8; ++bb) {
        const int b = r0 + bb;
        const float f = f3f[b * H_F3 + j], d = dz[b];
        sa += f > 0.f ? d : 0.f;
        sw += d * f;
        sz += d;
      }
      sa += __shfl_xor(sa, 32, 64);
      sw += __shfl_xor(sw, 32, 64);
      sz += __shfl_xor(sz, 32, 64);
      if (lane < 32) {
        red3w[wave * 72 + j] = sa;
        red3w[wave * 72 + 32 + j] = sw;
        if (j == 0) red3w[wave * 72 + 64] = sz;
      }
    }
    // dW3 [32 x 64] = d3^T f2 (registers until the Adam step)
    f4v g3;
    {
      const int o0 = (wave >> 2) * 16, ii0 = (wave & 3) * 16;
      g3 = Z4;
#pragma unroll
      for (int k0 = 0; k0 < 128; k0 += 32)
        g3 = mfma(cfrag(S + H_D3S, H_L3, k0, o0, lane), cfrag(S + H_F2S, H_L2, k0, ii0, lane), g3);
    }
    SYNC();
    if (tid < 32 || tid == 64) {
      float s0 = 0.f, s1 = 0.f;
#pragma unroll
      for (int w = 0; w < 8; ++w) {
        s0 += red3w[w * 72 + tid];
        if (tid < 32) s1 += red3w[w * 72 + 32 + tid];
      }
      if (tid < 32) {
        sums[64 + tid] = s0 * wos[tid];  // gb3
        sums[96 + tid] = s1;             // gWo
      } else {
        sums[128] = s0;                  // gbo
      }
    }
    if (tid < 64) {
      float sb = 0.f;
#pragma unroll
      for (int w = 0; w < 8; ++w) sb += gbw[w * 192 + tid];
      sums[tid] = sb;  // gb2
    }
    if (tid < 128) {
      float sb = 0.f;
#pragma unroll
      for (int w = 0; w < 8; ++w) sb += gbw[w * 192 + 64 + tid];
      sums[129 + tid] = sb;  // gb1
    }
    SYNC();
    // dW2 [64 x 128] = d2^T f1 (registers; after the d1 hand-off: off the critical path)
    f4v g2[4];
    {
      const int o0 = (wave >> 1) * 16, ib = (wave & 1) * 4;
#pragma unroll
      for (int j = 0; j < 4; ++j) g2[j] = Z4;
#pragma unroll
      for (int k0 = 0; k0 < 128; k0 += 32) {
        const s8v af = cfrag(S + H_D2S, H_L2, k0, o0, lane);
#pragma unroll
        for (int j = 0; j < 4; ++j) g2[j] = mfma(af, cfrag(S + H_F1S, H_L1, k0, 16 * (ib + j), lane), g2[j]);
      }
    }
    // Adam on the head parameters (off the critical path: the towers run their backward meanwhile)
    const AdamT ak = adam_t(a.lr, kact + 1, a.opt_mode);
    {
      f4v hm[6], hv[6];
#pragma unroll
      for (int k = 0; k < 6; ++k) mv_ld(x, k, hm[k], hv[k]);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float me = hm[j][e], ve = hv[j][e];
          p2[4 * j + e] = adam1(p2[4 * j + e], me, ve, g2[j][e], ak);
          hm[j][e] = me;
          hv[j][e] = ve;
        }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float me = hm[4][e], ve = hv[4][e];
        p3[e] = adam1(p3[e], me, ve, g3[e], ak);
        hm[4][e] = me;
        hv[4][e] = ve;
      }
      if (tid < 257) {
        // vector order of the state: b2 [64] | b3 [32] | Wo [32] | bo | b1 [128] == the sums layout
        float me = hm[5][0], ve = hv[5][0];
        pv = adam1(pv, me, ve, sums[tid], ak);
        hm[5][0] = me;
        hv[5][0] = ve;
      }
#pragma unroll
      for (int k = 0; k < 6; ++k) mv_st(x, k, hm[k], hv[k]);
    }
    SYNC();
    put_state();
    SYNC();
    stamp(x, kact, 2);
    ++kact;
  }
  if (nan_seen && tid == 0) a.failed[c] = 1;  // (a NaN loss on the round's last step)
  // round end: parameters -> arena
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) P[oW2 + (o2b + e) * 128 + i2b + 16 * j] = p2[4 * j + e];
#pragma unroll
  for (int e = 0; e < 4; ++e) P[oW3 + (o3b + e) * 64 + i3] = p3[e];
  if (tid < 257) P[vidx(tid)] = pv;
}

// ============================================================================================= fc1 owners
// Workgroup j (0..6) owns fc1 weight columns [144 j, 144 j + 16 nt) (nt = 9 column tiles, 10 for the last):
// dW1 = d1^T . feat over the batch rows (K = 128), Adam with the weights in registers (lane element (tile t, e) =
// (n = 16 w + 4 g + e, column 16 (9 j + t) + li)), and the block republished as bf16 W1 / W1T images of the
// NEXT step's parity.  Runs beside the towers' backward: off the step's critical path.
constexpr int F_LDF = 168;                          // feature block rows: up to 160 columns + 8
constexpr int F_D1 = 0, F_FW = 128 * LDD * 2, F_SW = F_FW + 128 * F_LDF * 2, F_FLAG = F_SW + 128 * F_LDF * 2;
static_assert(F_FLAG + 16 <= T_LDS, "fc1 owner LDS");

__device__ __forceinline__ void fc1_publish(const Ctx& x, int tid, int c0, int ntl, int par, const float (&p)[10][4]) {
  uchar* S = x.smem;
  const int lane = tid & 63, wave = tid >> 6, g = lane >> 4, li = lane & 15;
#pragma unroll
  for (int t = 0; t < 10; ++t)
    if (t < ntl)
#pragma unroll
      for (int e = 0; e < 4; ++e) *lu16(S, F_SW + ((16 * wave + 4 * g + e) * F_LDF + 16 * t + li) * 2) = bfu(p[t][e]);
  lbar();
  const int ncol = 16 * ntl, pr = ncol / 8;
  for (int e = tid; e < 128 * pr; e += NTH) {  // W1 [n][1024]: pr pieces of 8 columns per row
    const int n = e / pr, pc = e % pr;
    st16(x.rw, WS_IMG + (IM_W1 + par * IM_FC1PAR + n * 1024 + c0 + 8 * pc) * 2,
         *(const LDS_AS u32x4*)(S + F_SW + (n * F_LDF + 8 * pc) * 2));
  }
  for (int e = tid; e < ncol * 16; e += NTH) {  // W1T [1024][n]: 16 pieces of 8 n per column
    const int col = e >> 4, pc = e & 15;
    uint32_t w[4];
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      const unsigned short lo = *lu16(S, F_SW + ((8 * pc + 2 * h) * F_LDF + col) * 2);
      const unsigned short hi = *lu16(S, F_SW + ((8 * pc + 2 * h + 1) * F_LDF + col) * 2);
      w[h] = (uint32_t)lo | ((uint32_t)hi << 16);
    }
    st16(x.rw, WS_IMG + (IM_W1T + par * IM_FC1PAR + (c0 + col) * 128 + 8 * pc) * 2, u32x4{w[0], w[1], w[2], w[3]});
  }
}

__device__ __forceinline__ void fc1_owner(const Ctx& x, int j) {
  const AflCnn2Args& a = *x.a;
  uchar* S = x.smem;
  int tid = x.tid, lane = x.lane, wave = x.wave, g = lane >> 4, li = lane & 15;
  const int c = x.c;
  float* P = a.params + (long)c * a.pstride;
  const int ntl = j == NFC1 - 1 ? 10 : 9, c0 = 144 * j;
  float p[10][4];
#pragma unroll
  for (int t = 0; t < 10; ++t) {
#pragma unroll
    for (int e = 0; e < 4; ++e) p[t][e] = t < ntl ? P[a.off[12] + (16 * wave + 4 * g + e) * 1024 + c0 + 16 * t + li] : 0.f;
    mv_st(x, t, Z4, Z4);
  }
  fc1_publish(x, tid, c0, ntl, 0, p);
  arrive(x, CT_W1R);
  const int min_bs = a.min_bs;
  int kact = 0;
  for (int s = 0; s < a.S; ++s) {
    const int bs = a.bsz[(long)s * a.C + c];
    if (bs < min_bs || bs < 1) continue;
    const int par = kact & 1;
    if (!wait_ge(x, CT_H, (uint32_t)(kact + 1), F_FLAG)) break;
    REOPQ();
    stamp(x, kact, 0);
    if (ld16(x.rw, WS_STAT)[0] != 0u) break;  // NaN loss: the client's round ends without an update
    // d1 (all rows) and this block's feature columns -> LDS
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = tid + NTH * u, r = e >> 4, pc = e & 15;
      *(LDS_AS u32x4*)(S + F_D1 + (r * LDD + 8 * pc) * 2) = ld16(x.rw, WS_D1 + (r * 128 + 8 * pc) * 2);
    }
    const int pr = 2 * ntl;  // 16-B pieces per feature row
    for (int e = tid; e < 128 * pr; e += NTH) {
      const int r = e / pr, pc = e % pr;
      *(LDS_AS u32x4*)(S + F_FW + (r * F_LDF + 8 * pc) * 2) =
          ld16(x.rw, WS_FEAT + par * FEAT_PAR + (r * 1024 + c0 + 8 * pc) * 2);
    }
    f4v m[10], v[10];  // moments in flight during the staging barrier and the MFMAs (off the critical path)
#pragma unroll
    for (int t = 0; t < 10; ++t) mv_ld(x, t, m[t], v[t]);
    SYNC();
    f4v acc[10];
#pragma unroll
    for (int t = 0; t < 10; ++t) acc[t] = Z4;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const s8v af = cfrag(S + F_D1, LDD, 32 * ks, 16 * wave, lane);
#pragma unroll
      for (int t = 0; t < 10; ++t)
        if (t < ntl) acc[t] = mfma(af, cfrag(S + F_FW, F_LDF, 32 * ks, 16 * t, lane), acc[t]);
    }
    const AdamT ak = adam_t(a.lr, kact + 1, a.opt_mode);
#pragma unroll
    for (int t = 0; t < 10; ++t) {
      if (t >= ntl) continue;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float me = m[t][e], ve = v[t][e];
        p[t][e] = adam1(p[t][e], me, ve, acc[t][e], ak);
        m[t][e] = me;
        v[t][e] = ve;
      }
      mv_st(x, t, m[t], v[t]);
    }
    SYNC();
    fc1_publish(x, tid, c0, ntl, par ^ 1, p);
    arrive(x, CT_W1R);
    REOPQ();
    stamp(x, kact, 1);
    ++kact;
  }
#pragma unroll
  for (int t = 0; t < 10; ++t)
    if (t < ntl)
#pragma unroll
      for (int e = 0; e < 4; ++e) P[a.off[12] + (16 * wave + 4 * g + e) * 1024 + c0 + 16 * t + li] = p[t][e];
}

__global__ void __launch_bounds__(NTH) k_cnn2_train(AflCnn2Args a) {
  extern __shared__ __attribute__((aligned(16))) uchar smem_raw[];
  Ctx x;
  x.a = &a;
  x.c = blockIdx.x % a.C;
  const int role = blockIdx.x / a.C;
  x.tid = threadIdx.x;
  x.lane = threadIdx.x & 63;
  x.wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  x.role = role;
  x.smem = smem_raw;
  x.wsb = (uchar*)a.ws + (long)x.c * a.ws_stride;
  x.rw = rsrc(x.wsb);
  x.ctr = (gu32*)(a.ctr + (long)x.c * CT_N * 32);
#if defined(CNN2_ONLY_HEAD)
  head(x);
#elif defined(CNN2_ONLY_VIT)
  tower<0>(x, role);
#elif defined(CNN2_ONLY_LAB)
  tower<1>(x, role - 8);
#else
  if (role >= WG_FC1)
    fc1_owner(x, role - WG_FC1);
  else if (role == WG_HEAD)
    head(x);
  else if (role < 8)
    tower<0>(x, role);
  else
    tower<1>(x, role - 8);
#endif
}

// ============================================================================================== eval
// Forward-only CNNModel (eval mode: dropout off) of C models over rows [n][24] in ONE launch, grid (ceil(n / 16), C):
// the validation pass (src/Validation.py:19-68; the layer program spent ~1 ms per 4096 rows in k_cnn_fwd).  A workgroup
// takes 16 samples through both towers with the trainer's padded-row bf16 MFMA convolutions (the vitals tower as one
// 144-row pass, the labs tower as two 8-sample passes), fc1 / fc2 / fc3 on MFMA (bf16 operands, fp32 accumulation,
// as the trainer), the output unit in fp32.  Weights are read straight from the fp32 arena (bf16 fragments built in registers),
// so no image preparation launch is needed.
constexpr int E_H1 = 0, E_H2 = E_H1 + NR * LD1 * 2, E_H3 = E_H2 + NR * LD2 * 2, E_XS = E_H3 + NR * LD3 * 2;
constexpr int ELDF = 1032;                     // concat feature row stride (1024 + 8 bf16)
constexpr int E_FT = E_XS + 656;               // concat features bf16 [16][ELDF]
constexpr int E_A1 = E_FT + 16 * ELDF * 2;     // relu(fc1) bf16 [16][136] (fc2's MFMA operand)
constexpr int E_A2 = E_A1 + 16 * 136 * 2;      // relu(fc2) bf16 [16][72]
constexpr int E_A3 = E_A2 + 16 * 72 * 2;       // relu(fc3) fp32 [16][36]
constexpr int E_LDS = E_A3 + 16 * 36 * 4;
static_assert(E_LDS <= 160 * 1024 && (E_FT & 15) == 0 && (E_A1 & 15) == 0, "cnn2 eval LDS");

__device__ __forceinline__ s8v bf8(f4v lo, f4v hi) {
  return s8v{(short)bfu(lo[0]), (short)bfu(lo[1]), (short)bfu(lo[2]), (short)bfu(lo[3]),
             (short)bfu(hi[0]), (short)bfu(hi[1]), (short)bfu(hi[2]), (short)bfu(hi[3])};
}
// 8 elements at stride 3 (a conv weight column over 8 input channels of one tap) -> bf16 fragment
__device__ __forceinline__ s8v bf8s3(const float* p) {
  s8v r;
#pragma unroll
  for (int e = 0; e < 8; ++e) r[e] = (short)bfu(p[3 * e]);
  return r;
}

// one tower pass: samples s0 .. s0 + R - 1 (R = 16 vitals / 8 labs) -> feature rows fr0 .. fr0 + R - 1
template <int T>
__device__ __forceinline__ void eval_tower(const float* P, const int* of, const float* rows, int n, int s0, int fr0,
                                           uchar* S, int tid, int lane, int wave) {
  using C = TW<T>;
  const int g = lane >> 4, li = lane & 15;
  const float* cp1 = P + of[6 * T + 0];
  // x per padded row (XS index i holds padded row i - 1; pads and samples past n are zeros)
  for (int i = tid; i < 146; i += NTH) {
    const int q = i - 1;
    float v = 0.f;
    if (q >= 0 && valid_q(q, C::LP)) {
      const int smp = s0 + q / C::LP, l = q % C::LP - 1;
      if (smp < n) v = rows[(long)smp * 24 + C::XOFF + l];
    }
    *lf(S, E_XS + i * 4) = v;
  }
  const int o1 = tid & 31;
  const float w10 = cp1[3 * o1], w11 = cp1[3 * o1 + 1], w12 = cp1[3 * o1 + 2], bb1 = P[of[6 * T + 1] + o1];
  const int nt2 = wave & 3, mp2 = wave >> 2;
  s8v w2f[3], w3f[6];
#pragma unroll
  for (int j = 0; j < 3; ++j) w2f[j] = bf8s3(P + of[6 * T + 2] + ((16 * nt2 + li) * 32 + 8 * g) * 3 + j);
#pragma unroll
  for (int k = 0; k < 6; ++k)
    w3f[k] = bf8s3(P + of[6 * T + 4] + ((16 * wave + li) * 64 + 32 * (k & 1) + 8 * g) * 3 + (k >> 1));
  const f4v b2v = *(const f4v*)(P + of[6 * T + 3] + 16 * nt2 + 4 * g);
  const f4v b3v = *(const f4v*)(P + of[6 * T + 5] + 16 * wave + 4 * g);
  lbar();
  // conv1 (1 -> 32) on VALU -> H1 (bf16), pads exact zeros
#pragma unroll
  for (int u = 0; u < 9; ++u) {
    const int q = (tid >> 5) + 16 * u;
    float h = 0.f;
    if (valid_q(q, C::LP)) {
      const float xm = *lf(S, E_XS + q * 4), x0 = *lf(S, E_XS + (q + 1) * 4), xp = *lf(S, E_XS + (q + 2) * 4);
      h = relu(bb1 + w10 * xm + w11 * x0 + w12 * xp);
    }
    *lu16(S, E_H1 + ((q + 1) * LD1 + o1) * 2) = bfu(h);
  }
  lbar();
  // conv2 (transposed GEMM, as the trainer): wave n-tile nt2, m-tiles mp2, mp2 + 2, ...
  for (int mt0 = mp2; mt0 < 9; mt0 += 4) {
    f4v acc[2] = {Z4, Z4};
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
      for (int t = 0; t < 2; ++t) acc[t] = mfma(w2f[j], rfrag(S + E_H1, LD1, 16 * (mt0 + 2 * t) + j, 0, lane), acc[t]);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int q = 16 * (mt0 + 2 * t) + li;
      if (mt0 + 2 * t < 9)
        *(LDS_AS u32x2v*)(S + E_H2 + ((q + 1) * LD2 + 16 * nt2 + 4 * g) * 2) = relu_pack4(acc[t], b2v, valid_q(q, C::LP));
    }
  }
  lbar();
  // conv3: wave = n-tile, all 9 m-tiles
#pragma unroll
  for (int mt0 = 0; mt0 < 9; mt0 += 3) {
    f4v acc[3] = {Z4, Z4, Z4};
#pragma unroll
    for (int k = 0; k < 6; ++k)
#pragma unroll
      for (int t = 0; t < 3; ++t)
        acc[t] = mfma(w3f[k], rfrag(S + E_H2, LD2, 16 * (mt0 + t) + (k >> 1), 32 * (k & 1), lane), acc[t]);
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      const int q = 16 * (mt0 + t) + li;
      *(LDS_AS u32x2v*)(S + E_H3 + ((q + 1) * LD3 + 16 * wave + 4 * g) * 2) = relu_pack4(acc[t], b3v, valid_q(q, C::LP));
    }
  }
  lbar();
  // AdaptiveAvgPool1d(4) -> feature rows (concat column COL0 + 4 channel + bin)
#pragma unroll
  for (int it = 0; it < 16 * 64 / NTH; ++it) {
    const int e = tid + NTH * it, r = e >> 6, cp = e & 63;
    if (r < C::R) {
      float h0[C::L], h1v[C::L], f[8];
#pragma unroll
      for (int l = 0; l < C::L; ++l) {
        const uint32_t w = *(const LDS_AS uint32_t*)(S + E_H3 + ((r * C::LP + 2 + l) * LD3 + 2 * cp) * 2);
        h0[l] = __uint_as_float(w << 16);
        h1v[l] = __uint_as_float(w & 0xFFFF0000u);
      }
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        float a0 = 0.f, a1 = 0.f;
#pragma unroll
        for (int l = bin_lo(p, C::L); l < bin_hi(p, C::L); ++l) {
          a0 += h0[l];
          a1 += h1v[l];
        }
        f[p] = a0 * bin_rcp(p, C::L);
        f[4 + p] = a1 * bin_rcp(p, C::L);
      }
      *(LDS_AS u32x4*)(S + E_FT + ((fr0 + r) * ELDF + C::COL0 + 8 * cp) * 2) =
          u32x4{pk2(f[0], f[1]), pk2(f[2], f[3]), pk2(f[4], f[5]), pk2(f[6], f[7])};
    }
  }
  lbar();
}

struct AflCnn2Eval {
  const float* params;
  long pstride;
  int off[20];
  const float* rows;
  int n;
  float* out;  // [C][n]
};

__global__ void __launch_bounds__(NTH) k_cnn2_eval(AflCnn2Eval a) {
  extern __shared__ __attribute__((aligned(16))) uchar smem_raw[];
  uchar* S = smem_raw;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, li = lane & 15, c = blockIdx.y, s0 = blockIdx.x * 16;
  const float* P = a.params + (long)c * a.pstride;
  // zero the activation buffers once: their boundary rows are never written (exact zeros for every pass)
  for (int e = tid; e < E_XS / 16; e += NTH) *(LDS_AS u32x4*)(S + 16 * e) = u32x4{0u, 0u, 0u, 0u};
  lbar();
#if !defined(CNN2_EVAL_ABL) || !(CNN2_EVAL_ABL & 2)  // (timing ablation: no towers)
  eval_tower<0>(P, a.off, a.rows, a.n, s0, 0, S, tid, lane, wave);
  eval_tower<1>(P, a.off, a.rows, a.n, s0, 0, S, tid, lane, wave);
  eval_tower<1>(P, a.off, a.rows, a.n, s0 + 8, 8, S, tid, lane, wave);
#endif
  // fc1: z1[16 samples][128] = feat . W1^T, wave = n-tile; W1 rows 16 w + li converted to bf16 in registers
  {
    const float* W1 = P + a.off[12] + (long)(16 * wave + li) * 1024 + 8 * g;
    f4v acc = Z4;
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      s8v wf[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
#if defined(CNN2_EVAL_ABL) && (CNN2_EVAL_ABL & 1)  // (timing ablation: no W1 loads)
        wf[k] = s8v{(short)k, 1, 2, 3, 4, 5, 6, (short)kb};
#else
        const f4v lo = *(const f4v*)(W1 + 32 * (8 * kb + k)), hi = *(const f4v*)(W1 + 32 * (8 * kb + k) + 4);
        wf[k] = bf8(lo, hi);
#endif
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) acc = mfma(rfrag(S + E_FT, ELDF, 0, 32 * (8 * kb + k), lane), wf[k], acc);
    }
    const float b1 = P[a.off[13] + 16 * wave + li];
#pragma unroll
    for (int e = 0; e < 4; ++e) *lu16(S, E_A1 + ((4 * g + e) * 136 + 16 * wave + li) * 2) = bfu(relu(acc[e] + b1));
  }
  lbar();
  // fc2 (128 -> 64) + ReLU on MFMA (bf16 operands, as the trainer's head): waves 0-3, n-tile = wave
  if (wave < 4) {
    const float* W2 = P + a.off[14] + (16 * wave + li) * 128 + 8 * g;
    f4v acc = Z4;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      acc = mfma(rfrag(S + E_A1, 136, 0, 32 * k, lane), bf8(*(const f4v*)(W2 + 32 * k), *(const f4v*)(W2 + 32 * k + 4)), acc);
    const float b2 = P[a.off[15] + 16 * wave + li];
#pragma unroll
    for (int e = 0; e < 4; ++e) *lu16(S, E_A2 + ((4 * g + e) * 72 + 16 * wave + li) * 2) = bfu(relu(acc[e] + b2));
  }
  lbar();
  // fc3 (64 -> 32) + ReLU on MFMA: waves 0-1
  if (wave < 2) {
    const float* W3 = P + a.off[16] + (16 * wave + li) * 64 + 8 * g;
    f4v acc = Z4;
#pragma unroll
    for (int k = 0; k < 2; ++k)
      acc = mfma(rfrag(S + E_A2, 72, 0, 32 * k, lane), bf8(*(const f4v*)(W3 + 32 * k), *(const f4v*)(W3 + 32 * k + 4)), acc);
    const float b3 = P[a.off[17] + 16 * wave + li];
#pragma unroll
    for (int e = 0; e < 4; ++e) *lf(S, E_A3 + ((4 * g + e) * 36 + 16 * wave + li) * 4) = relu(acc[e] + b3);
  }
  lbar();
  // output (32 -> 1) + sigmoid: wave 0, lane (sample lane >> 2, quarter lane & 3)
  if (wave == 0) {
    const int r = lane >> 2, qt = lane & 3;
    float sv = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) sv += *lf(S, E_A3 + (r * 36 + 8 * qt + k) * 4) * P[a.off[18] + 8 * qt + k];
    sv += __shfl_xor(sv, 1, 64);
    sv += __shfl_xor(sv, 2, 64);
    const float z = sv + P[a.off[19]];
    if (qt == 0 && s0 + r < a.n) a.out[(long)c * a.n + s0 + r] = 1.f / (1.f + __expf(-z));
  }
  (void)g;
  (void)li;
}

}  // namespace

long afl_cnn2_ws_bytes() { return WS_BYTES; }
int afl_cnn2_ctr_words() { return CT_N * 32; }
int afl_cnn2_wgs_per_client() { return NWG; }

int afl_cnn2_train(const AflCnn2Args& a, hipStream_t s) {
  if (a.B < 2 || a.B > 128 || a.C < 1 || a.ws_stride < WS_BYTES || (a.ws_stride & 15)) return (int)hipErrorInvalidValue;
  static bool attr = false;
  if (!attr) {
    const hipError_t e =
        hipFuncSetAttribute((const void*)k_cnn2_train, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_TOTAL);
    if (e != hipSuccess) return (int)e;
    attr = true;
  }
  hipLaunchKernelGGL(k_cnn2_train, dim3(NWG * a.C), dim3(NTH), LDS_TOTAL, s, a);
  return (int)hipGetLastError();
}

// eval forward of C CNNModels (params [C][pstride], slot offsets off[20]) over rows [n][24] -> out [C][n]
int afl_cnn2_eval(const float* params, long pstride, const int* off, int C, const float* rows, int n, float* out,
                  hipStream_t s) {
  if (C <= 0 || n <= 0) return 0;
  static bool attr = false;
  if (!attr) {
    const hipError_t e = hipFuncSetAttribute((const void*)k_cnn2_eval, hipFuncAttributeMaxDynamicSharedMemorySize, E_LDS);
    if (e != hipSuccess) return (int)e;
    attr = true;
  }
  AflCnn2Eval a{};
  a.params = params;
  a.pstride = pstride;
  for (int k = 0; k < 20; ++k) a.off[k] = off[k];
  a.rows = rows;
  a.n = n;
  a.out = out;
  hipLaunchKernelGGL(k_cnn2_eval, dim3((n + 15) / 16, C), dim3(NTH), E_LDS, s, a);
  return (int)hipGetLastError();
}
