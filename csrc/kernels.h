// Host-side launchers of the gfx950 kernels (raw pointers + stream; no torch headers so the
// device translation units compile in seconds).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// agg.hip
void afl_colstats(const float* G, int K, long P, float* mean, float* stdv, float* out, float z, int mode,
                  hipStream_t s);
void afl_weighted_rows(const float* U, const double* w, int N, long P, float* out, hipStream_t s,
                       const int* ok = nullptr, const float* fallback = nullptr);
int afl_pair_sqdist_nblocks(long P);
void afl_pair_sqdist(const float* G, int K, long P, double* partial, double* D, hipStream_t s);
void afl_seg_reduce(int mode, const float* X, long P, int rows, const float* mean, const float* dev, const int* tiles,
                    int T, const int* segf, int S, double* partial, double* out0, double* out1, hipStream_t s);
void afl_coord_select(const float* U, int N, long P, int mode, int trim, float* out, hipStream_t s);
int afl_row_dots_nchunks(long P);
void afl_row_dots(const float* U, const float* ref, int N, long P, int mode, double* partial, double* out,
                  hipStream_t s);
long afl_stoch_quant_ws(int N);  // floats of workspace afl_stoch_quant needs
void afl_stoch_quant(const float* U, int N, long P, uint64_t seed, float* sigma, float* smin, float* smax,
                     float* ws, hipStream_t s);
void afl_adam_flat(float* p, const float* g, float* m, float* v, long n, int step, float lr, float b1, float b2,
                   float eps, float gscale, hipStream_t s);

// hyper.hip
int afl_hyper_nblocks(long P);
void afl_hyper_rows(const float* W, const float* b, const float* f, const float* u, long P, int H, float* out,
                    float* partial, float* dfeat, hipStream_t s);
void afl_hyper_adam(float* W, float* bvec, float* m, float* v, const float* delta, const float* f, long P, int H,
                    int step, float lr, float b1, float b2, float eps, float gs, hipStream_t s);
// arena offsets (floats) of the hypernet embedding + MLP (L layers, E -> H -> ... -> H)
struct HySmallDesc {
  long emb;
  long w[8];
  long b[8];
  int L, E, H, n_nodes;
};
void afl_hyper_server_update(float* A, float* m, float* v, const float* U, const long* urow, const int* clients,
                             int n, const HySmallDesc& d, long offW, long offB, long P, int step0, float lr,
                             float clip, float b1, float b2, float eps, float* delta, float* partial, float* feat,
                             float* info, const int* enable, const int* gen, int ngen, float* gen_feat,
                             float* gen_out, hipStream_t s);
// W f_c + b of n clients (feat [n, H]) -> out [n, P]: one sweep over the heads per 32 clients
void afl_hyper_generate(const float* A, const HySmallDesc& d, long offW, long offB, long P, const float* feat, int n,
                        float* out, hipStream_t s);
void afl_hyper_features(const float* A, const HySmallDesc& d, long offW, const int* clients, int n, float* out,
                        hipStream_t s);
long afl_hyper_small_capacity();  // max floats of embedding-MLP parameters the small-net kernel stages in LDS

// plan.hip
void afl_make_plan(const uint64_t* seeds, const int* nd, int C, int n_train, int E, int maxnd, int* order,
                   hipStream_t s);
void afl_step_tables(const int* order, const int* nd, int C, int E, int maxnd, int B, int S, int* idx, int* bsz,
                     int* ep, int* nb, int* zi, long nzi, float* zf, long nzf, hipStream_t s);

// linalg.hip
int afl_spectral_scratch(int r, int c);
int afl_spectral(const float* X, int B, int r, int c, float* G0, double* out, hipStream_t s);
// Gram-form spectral norms (linalg.hip): per (slot, row) fp64 Grams of X (and, with dev, X D^T + D X^T and
// D D^T) once; then sigma_max(X_m - γ D) per slot for a device-resident γ (null: γ = 0).  tab [S] int4 =
// {offset, r, c, arena offset}; arena = [M][2][sumq] + [sumq] doubles.
int afl_spec_grams(const float* X, int M, long P, const float* dev, const int* tab, int S, int max_lds_floats, long sumq,
                   double* arena, hipStream_t st);
// device-resident bisection state + inputs (linalg.hip bisect_decide)
struct AflBisect {
  double* st;            // [40] fp64 state (γ, γ_succ, last γ, tried[16], accepted[16])
  unsigned* ctr;         // arrival counter of a k_spec_eval<true> launch (zero before the first; self-resetting)
  const double* vA;      // [K, Sv] closed-form vector slots (A - 2γB + γ²C per slot), or null with Sv = 0
  const double* vB;      // [K, Sv]
  const double* vC;      // [Sv]
  const double* thr;     // device scalar threshold
  int Sv, K, kind;       // kind 0: max d < thr, 1: sum d² < thr
};
int afl_spec_bisect(const double* arena, long sumq, int M, const int* tab, int S, double* out, const AflBisect* b, int it,
                    double step, hipStream_t st);
int afl_bisect_vec(const AflBisect* b, int n_iter, double step0, hipStream_t st);
int afl_spec_eval(const double* arena, long sumq, int M, const double* gamma, const int* tab, int S, double* out,
                  hipStream_t st);
int afl_spectral_slots(const float* D, int M, long P, const int* tab, int S, int max_n, float* G0, long scr,
                       double* out, hipStream_t st);

// metrics.hip
int afl_roc_auc_pairs_max();
void afl_roc_auc_pairs(const float* s, const float* y, int n, unsigned long long* acc, double* out, hipStream_t st);
void afl_roc_auc(const float* sorted, const float* s, const float* y, int n, unsigned long long* acc, double* out,
                 hipStream_t st);

// transformer.hip (TransformerModel / ICU fused training + eval)
struct AflTfTrainArgs {
  float* params;          // [C, NPARAM] fp32, updated in place
  const float* rows;      // [Ntrain, 24]
  const int* order;       // [C, E, maxnd]
  const int* nd;          // [C]
  const uint32_t* seeds;  // [C]
  float* ws;              // [C, ws_stride] workspace
  long ws_stride;
  int* ok;                // [C]
  float* losses;          // [C, E]
  int C, E, maxnd, batch;
  float lr;
  int opt_mode;  // 0 = Adam (reference), 1 = SGD (test hook: exposes raw gradients)
  uint64_t* stamps;  // optional per-phase timers (AFL_TF_STAMPS builds), may be null
  uint32_t* sync;    // zeroed hand-off words (branch-parallel launches): [C][AFL_TF_SYNC_WORDS]
  int split;         // workgroups per client: 1, 2 (vitals+head | labs), 3 (head | vitals | labs)
  // tf2 only: per-step Adam constants [kt_n][2] = (lr / (1 - beta1^t), 1 / sqrt(1 - beta2^t)), t = 1..kt_n
  const float* kt;
  int kt_n;
  // on-chip trainers: block stride of the role-major grid (>= C; padded to a multiple of 8 when that still
  // fits, so a client's workgroups land on one XCD whatever C is); blocks with client index >= C exit
  int cpad;
};
int afl_tf_train(const AflTfTrainArgs* a, hipStream_t s);
int afl_tf_eval_bf(const float* params, unsigned short* bf, const float* rows, int n, float* out, hipStream_t s);
// C models (params + c * pstride) over the same rows in one launch pair; bf = C * bfstride ushorts of scratch
int afl_tf_eval_many(const float* params, long pstride, unsigned short* bf, long bfstride, int C, const float* rows,
                     int n, float* out, hipStream_t s);
long afl_tf_ws_floats();
constexpr int AFL_TF_SYNC_WORDS = 4 * 8 * 32 + 32;  // per-wave flags (128-B lines) + timeout word
// on-chip trainers (tf2 / rnn2): the flag words, then the granule hand-off slots (onchip.h gr_put / gr_get):
// 2 directions x 2 branches x 8 waves x 4 KB of {value, tag} granules, zeroed with the flags every call
constexpr int AFL_GR_WORDS = 2 * 2 * 8 * 1024;
constexpr int AFL_TF2_SYNC_WORDS = AFL_TF_SYNC_WORDS + AFL_GR_WORDS;
// tf2.hip (TransformerModel / ICU fused training, on-chip edition: weights, Adam state and activations
// in registers / LDS; 3 workgroups per client, sync words required)
int afl_tf2_train(const AflTfTrainArgs* a, hipStream_t s);
int afl_tf2_train_stamped(const AflTfTrainArgs* a, hipStream_t s);  // tf2_stamps.hip: per-phase timers
long afl_tf2_ws_floats();
// determinism check of the on-chip trainers' cross-wave column sums (tf2.hip k_fxsum_test; tests only)
int afl_fxsum_test(const float* vals, int W, uint32_t seed, int mode, float* out, hipStream_t s);
// rnn.hip (RNNModel / ICU fused training: 3 workgroups per client, sync words required)
int afl_rnn_train(const AflTfTrainArgs* a, hipStream_t s);
long afl_rnn_ws_floats();
// rnn2.hip (RNNModel on-chip trainer: 3 workgroups per client, model state on chip, Adam step table kt)
int afl_rnn2_train(const AflTfTrainArgs* a, hipStream_t s);
int afl_rnn2_train_stamped(const AflTfTrainArgs* a, hipStream_t s);
long afl_rnn2_ws_floats();
int afl_rnn2_eval(const float* params, long pstride, int C, const float* rows, int n, float* out, hipStream_t s);
int afl_rnn_param_count();
int afl_tf_bf_ushorts();
int afl_tf_param_count();

// ============================================================================================
// layers.hip — client-batched layer kernels: the native path of every model without a fused
// trainer (CNNModel, RNNModel, TransformerClassifier/HAR).  Tensors are [C clients][rows][cols]
// fp32 with explicit strides; GEMMs stage bf16 tiles in LDS and run v_mfma_f32_16x16x32_bf16.
// ============================================================================================
struct AflDrop {          // dropout site; thr16 == 0 disables it
  const uint32_t* seeds;  // [C] client seeds
  const int* stepctl;     // device step counter (null: step 0)
  uint32_t layer, thr16;
  float inv_keep;
};
struct AflGemm {
  // Cm[c][m][n] (op)= epi( alpha * sum_k A[c][m][k] * B[c][n][k] )
  const float* A;
  long sAc, sAm, sAk;
  const float* B;
  long sBc, sBn, sBk;
  float* Cm;
  long sCc, sCm, sCn;
  float* Z;            // optional copy of the pre-activation (Cm strides)
  const float* bias;   // optional bias[c * sbc + n]
  long sbc;
  const float* G;      // optional activation-derivative source: out *= act'(G[c][m][n])
  long sGc, sGm, sGn;
  int M, N, K, nC;
  int act;     // 0 none, 1 relu, 2 gelu(erf)
  int gact;    // 0 none, 1 relu' (G > 0), 2 gelu'(G)
  int accum;   // 0 store, 1 add (single writer), 2 atomic add (split-K)
  int splitk;
  float alpha;
  AflDrop drop;
  int avec, bvec;  // set by the launcher: operand rows 16-B aligned and k-contiguous
  int no_ts;       // 1: never take the tall-skinny path (tests compare the two kernels)
  float* asum;     // optional: asum[c * sasc + k] += sum_m A[c][m][k] (the bias gradient of a dX = dY.W GEMM)
  long sasc;
  float* ws;       // optional split-K workspace [splitk][C][M][N]: with it, accum 2 is DETERMINISTIC — each
                   // split stores its partial tile, a second pass adds the splits to C in split order
  float* ws_sum;   // optional workspace for the asum column sums (afl_bgemm_asum_ws_floats): ordered partials
};
int afl_bgemm(const AflGemm& g, hipStream_t s);
long afl_bgemm_ws_floats(const AflGemm& g);  // workspace the deterministic split-K path needs (0: none)
long afl_bgemm_asum_ws_floats(const AflGemm& g);  // workspace of the ordered asum partials (0: none)
long afl_colsum_ws_floats(int M, int N, int nC);

// cnn.hip: fused CNNModel towers (conv1-3 + pool + dropout) forward / backward, conv weight grads
struct AflCnnBranch {
  const float* x;                    // input [C][B*L] (one channel); client stride sXc
  long sXc;
  const float *W1, *b1, *W2, *b2, *W3, *b3;  // client-0 parameter views (client c at + c * sWc)
  float *h1, *h2, *h3;               // saved activations [C][B*L][32 | 64 | 128] (dense)
  float *dh1, *dh2, *dh3;            // backward outputs, same layout
  int L, R, ntiles, col0;            // R samples per workgroup tile (R * L <= 64)
  uint32_t layer;                    // dropout site id of the tower's concat slice
};
struct AflCnnTowers {
  AflCnnBranch br[2];
  long sWc;
  float* cat;                        // [C][B][1024] concat (forward output)
  const float* dcat;                 // its gradient (backward input), same strides
  long sCatc, sCatr;
  int C, B;
  AflDrop drop;                      // seeds / step / p (layer per branch)
  unsigned short* wimg;              // bf16 weight images (afl_cnn_wimg_ushorts(C)), built by the forward
  const float *W2h, *W3h;            // optional head fc2 / fc3 weights (client-0 views): images for k_cnn_head
};
long afl_cnn_wimg_ushorts(int C);
// cnn2.hip: CNNModel on-chip trainer (one launch per round; 25 workgroups per client, one per CU)
struct AflCnn2Args {
  float* params;         // [C][pstride] fp32 arena, trained in place
  long pstride;
  int off[20];           // CNNModel state_dict slot offsets (ParamLayout order)
  const float* rows;     // ICU table [N][24]
  const int* idx;        // [S][C][B] batch rows (-1 = padding)
  const int* bsz;        // [S][C]
  const int* epoch;      // [S][C]
  const int* nb;         // [C] batches per epoch (loss divisor)
  const uint32_t* seeds; // [C] dropout seeds (StepCtl)
  int S, C, B, E;
  uint32_t thr16;        // dropout threshold (0 = off), keep scale
  float inv_keep;
  int min_bs, nan_abort;
  float lr;
  int opt_mode;          // 0 Adam, 1 plain SGD p -= lr g (gradient tests)
  int* failed;           // [C] out: 1 = NaN loss
  float* losses;         // [C][E] accumulated epoch losses (zeroed by the caller)
  void* ws;              // [C][ws_stride] bytes workspace (afl_cnn2_ws_bytes)
  long ws_stride;
  uint32_t* ctr;         // [C][afl_cnn2_ctr_words] zeroed counters
  uint64_t* stamps;      // optional [C][25][64][16] per-phase s_memrealtime stamps (null: off)
};
long afl_cnn2_ws_bytes();
int afl_cnn2_ctr_words();
int afl_cnn2_wgs_per_client();
int afl_cnn2_train(const AflCnn2Args& a, hipStream_t s);
int afl_cnn2_eval(const float* params, long pstride, const int* off, int C, const float* rows, int n, float* out,
                  hipStream_t s);
int afl_cnn_towers_fwd(const AflCnnTowers& a, hipStream_t s);
int afl_cnn_towers_bwd(const AflCnnTowers& a, hipStream_t s);
struct AflConvDwJob {
  const float* dh;   // [C][B*L][Cout] dense
  const float* hp;   // [C][B*L][Cin] dense (conv input)
  float* gW;         // client-0 grad view [Cout][3*Cin] (client c at + c * sGc)
  float* gb;         // client-0 bias grad [Cout]
  int Cin, Cout, L, tile_base;
  long ws_off;       // this job's [Cout][3*Cin] + [Cout] block in a split's workspace slice
};
struct AflConvDw {
  AflConvDwJob job[6];
  int njobs, total_tiles, splitk, C, B;
  long sGc;
  float* ws;         // optional [splitk][C][ws_tot] workspace: deterministic split-K (partials, ordered sum)
  long ws_tot;
};
int afl_conv_dw(const AflConvDw& a, hipStream_t s);
struct AflCnnHead {
  float* f1;                         // [C][B][128] fc1 PRE-activation (bias + ReLU applied here, then zeroed)
  const float* b1;                   // fc1 bias (client-0 view)
  const unsigned short* wimg;        // head weight images of client 0 (built by the towers' forward)
  const float* y;                    // [C][B] labels
  const float *W2, *b2, *W3, *b3, *Wo, *bo;  // client-0 parameter views (+ c * sWc)
  long sWc;
  float *gW2, *gb2, *gW3, *gb3, *gWo, *gbo, *gb1;  // client-0 gradient views (+ c * sGc)
  long sGc;
  float* d1;                         // [C][B][128] d(fc1 pre-activation)
  float* z;                          // optional [C][B] logits
  const int *bsz, *epoch, *nb, *stepctl;
  int* failed;
  float* losses;
  int S, E, C, B;
};
int afl_cnn_head(const AflCnnHead& h, hipStream_t s);
// column sums; ws (optional, afl_colsum_ws_floats): per-row-block partials added in block order (deterministic)
int afl_colsum(const float* Y, long sYc, long sYm, int M, int N, int nC, float* out, long sOc, hipStream_t s,
               float* ws = nullptr);
int afl_gather_icu(const float* rows, const int* idx, const int* stepctl, int C, int B, int mask, float* vit,
                   float* lab, float* y, hipStream_t s);
int afl_gather_har(const float* x, const long* y, int F, const int* idx, const int* stepctl, int C, int B, float* ox,
                   long* oy, hipStream_t s);
int afl_im2col3(const float* x, long sXc, long sXr, int C, int B, int L, int Cin, float* out, hipStream_t s);
int afl_col2im3(const float* dcols, int C, int B, int L, int Cin, const float* relu_src, long sRc, long sRr, float* dx,
                hipStream_t s);
int afl_pool4_fwd(const float* h, int C, int B, int L, int Ch, float* out, long sOc, long sOr, int col0, AflDrop d,
                  hipStream_t s);
int afl_pool4_bwd(const float* dout, long sOc, long sOr, int col0, const float* h, int C, int B, int L, int Ch,
                  float* dh, AflDrop d, hipStream_t s);
struct AflLn {
  // y = LN(x + drop_a(a)) * gamma + beta, then y = drop_o(y); D = 64
  const float* x; long sXc, sXr;
  const float* a; long sAc, sAr;  // optional residual branch
  float* s;                       // optional stored pre-norm sum [C][rows][64] (dense)
  float* y; long sYc, sYr;
  float* stats;                   // [C][rows][2] mean, rstd
  const float* gamma; const float* beta; long sPc;  // params (+ client stride)
  int rows, nC;
  AflDrop da, dout;
};
int afl_ln_fwd(const AflLn& l, hipStream_t s);
struct AflLnB {
  const float* dy; long sDc, sDr;
  const float* s; long sSc, sSr;  // pre-norm input (dense [C][rows][64] when from AflLn.s)
  const float* stats;
  const float* gamma; long sPc;
  float* dx; long sXc, sXr; int dx_accum;  // d(pre-norm sum)
  float* da; long sAc, sAr;               // optional: drop_a'(dx) for the residual branch
  float* dgamma; float* dbeta;            // grad slots (+ sPc), accumulated
  int rows, nC;
  AflDrop da_drop, dout;
  float* ws;  // optional [row blocks][C][128] partials (afl_ln_bwd_ws_floats): ordered, deterministic sums
};
int afl_ln_bwd(const AflLnB& l, hipStream_t s);
long afl_ln_bwd_ws_floats(int rows, int nC);
int afl_gru_fwd(const float* gi, const float* bhh, long sPc, int C, int B, float* h, long sHc, long sHr, int col0,
                hipStream_t s);
int afl_gru_bwd(const float* dh, long sHc, long sHr, int col0, const float* gi, const float* bhh, long sPc, int C,
                int B, float* dgi, float* dbih, float* dbhh, hipStream_t s);
int afl_bce(const float* z, const float* y, const int* bsz, const int* epoch, const int* nb, const int* stepctl, int C,
            int B, int S, int* failed, float* losses, int E, float* dz, hipStream_t s);
int afl_ce(const float* logits, const long* y, int K, const int* bsz, const int* epoch, const int* nb,
           const int* stepctl, int C, int B, int S, int* failed, float* losses, int E, float* dz, hipStream_t s);
int afl_adam_clients(float* p, float* g, float* m, float* v, long P, int C, const int* tcount, const int* bsz,
                     const int* stepctl, int S, const int* failed, float lr, long skip_lo, long skip_hi, float sgd_lr,
                     int zero_g, hipStream_t s);
int afl_step_end(int* stepctl, int* tcount, const int* bsz, const int* failed, int C, int S, hipStream_t s);
int afl_conv_pe_fwd(const float* x, int C, int B, int L, const float* params, long P, int w_off, int b_off,
                    int pe_off, float* h, hipStream_t s);
int afl_conv_pe_bwd(const float* x, const float* dh, int C, int B, int L, float* grads, long P, int w_off, int b_off,
                    hipStream_t s, float* ws = nullptr);
long afl_conv_pe_bwd_ws_floats(int C, int B, int L);  // [row blocks][C][256] partials
int afl_mean_rows_fwd(const float* h, int C, int B, int L, float* out, hipStream_t s);
int afl_mean_rows_bwd(const float* dout, int C, int B, int L, float* dh, hipStream_t s);

// har.hip — HAR encoder on bf16 activations (row passes + head-major flash attention)
struct AflHarLayerW {  // flat-parameter offsets of one encoder layer
  int inw, inb, ow, ob, n1w, n1b, l1w, l1b, l2w, l2b, n2w, n2b;
};
struct AflHarQkv {
  const unsigned short* x;  // [C][R][64] bf16 layer input
  const float* params; long P; int w_off, b_off;
  unsigned short* qkv;      // [C*B*4][3][Lp][16] bf16, q scaled by qscale
  int C, B, L, Lp;
  float qscale;
};
struct AflHarPost {
  const unsigned short* o;  // [C][R][64] attention output
  const unsigned short* x;  // [C][R][64] layer input (residual)
  unsigned short* xh1;      // [C][R][64] saved normalised LN1 input
  unsigned short* xh2;      // [C][R][64] saved normalised LN2 input
  float* rs;                // [C][R][2] rstd1, rstd2
  unsigned short* y;        // [C][R][64] layer output
  const float* params; long P; AflHarLayerW w;
  int C; long R;
  AflDrop d1, df, d2;       // dropout1 (out_proj), FFN activation, dropout2 (linear2)
  unsigned* kbits;          // [C][R][4 g][4] keep bits of the row pass (dropout only, else null): word 0 = d1 (bits
                            // 0-15) | d2 (16-31), words 1-2 = the FFN's 64, word 3 unused; read back by the backward
};
struct AflHarPostB {
  const float* dy;          // [C][R][64] d(layer output) fp32 — or null with dpool set
  const float* dpool;       // [C][B][64] d(mean over L): dy[c][b*L + l] = dpool[c][b] / L (last layer)
  int B, L;
  const unsigned short* o;  // attention output (bf16)
  const unsigned short* xh1; const unsigned short* xh2; const float* rs;
  float* dres;              // [C][R][64] d(layer input) through the residual path (fp32)
  unsigned short* dout;     // [C][R][64] d(attention output) (bf16)
  float* delta;             // [C*B*4][Lp] rowsum(dO o O) per head
  int Lp;
  float* ws;                // [C][G][AFL_HAR_POST_NG] per-workgroup gradient partials
  const float* params; long P; AflHarLayerW w;
  int C; long R;
  AflDrop d1, df, d2;
  const unsigned* kbits;    // the forward's keep bits (AflHarPost::kbits); null = no dropout
};
struct AflHarQkvB {
  const unsigned short* dqkv;  // [C*B*4][3][Lp][16] d(q|k|v projection outputs) (bf16)
  const float* dres;           // [C][R][64]
  const unsigned short* x;     // [C][R][64] layer input
  float* dx;                   // [C][R][64] d(layer input) (fp32)
  float* ws;                   // [C][G][AFL_HAR_QKV_NG]
  const float* params; long P; int w_off;
  int C, B, L, Lp;
};
struct AflHarAttn {
  const unsigned short* qkv;   // [C*B*4][3][Lp][16] (q pre-scaled by 1/4)
  unsigned short* o;           // [C][B*L][64]
  float* lse2;                 // [C*B*4][Lp] log2-domain logsumexp of the scaled scores
  const unsigned short* dout;  // [C][B*L][64] (bwd)
  const float* delta;          // [C*B*4][Lp] (bwd)
  unsigned short* dqkv;        // [C*B*4][3][Lp][16] (bwd): d(q projection) (x 1/4 folded in), dk, dv
  unsigned long long* mask;    // [C*B*4][AFL_HAR_MASK_WORDS(Lp)] probability-dropout keep words: written by the
                               // forward, read by both backward kernels (dropout only)
  int C, B, L, Lp;
  AflDrop drop;
};
// keep words per (client, sample, head): [query tile Lp/16][key chunk Lp/64][t 4][e 4], bit = lane of the forward
#define AFL_HAR_MASK_WORDS(Lp) ((long)((Lp) / 16) * ((Lp) / 64) * 16)
#define AFL_HAR_KBITS_PER_ROW 16  // u32 words of AflHarPost::kbits per row
#define AFL_HAR_POST_NG (64 * 64 + 256 * 64 + 64 * 256 + 640)
#define AFL_HAR_QKV_NG (192 * 64 + 192)
int afl_har_stem(const float* x, int C, int B, int L, const float* params, long P, int w_off, int b_off, int pe_off,
                 unsigned short* h, hipStream_t s);
int afl_har_pool(const unsigned short* y, int C, int B, int L, float* out, hipStream_t s);
int afl_har_qkv(const AflHarQkv& a, hipStream_t s);
int afl_har_post(const AflHarPost& a, hipStream_t s);
int afl_har_post_bwd(const AflHarPostB& a, int G, hipStream_t s);
int afl_har_qkv_bwd(const AflHarQkvB& a, int G, hipStream_t s);
int afl_har_blocks(long R);
int afl_har_attn_fwd(const AflHarAttn& a, hipStream_t s);
int afl_har_attn_bwd(const AflHarAttn& a, hipStream_t s);
int afl_har_reduce(const float* ws, int C, int G, int n, const int* seg, int nseg, float* grads, long P, hipStream_t s);

// attention.hip — flash attention (HAR encoder: 4 heads x 16, L <= 640)
struct AflAttn {
  const float* qkv;   // [C][B*L][192]
  float* o;           // [C][B*L][64]  (fwd output; bwd input)
  float* lse;         // [C*B*4][Lp]
  const float* dout;  // [C][B*L][64]  (bwd)
  float* dqkv;        // [C][B*L][192] (bwd output)
  int C, B, L, Lp;
  float scale;
  AflDrop drop;
};
int afl_attn_lp(int L);
int afl_attn_fwd(const AflAttn& a, hipStream_t s);
int afl_attn_bwd(const AflAttn& a, hipStream_t s);

// agg.hip — Gram-form pairwise distances (fp64 MFMA, rows centred on row 0; K <= 64) and Philox noise
int afl_gram_partials(int K, long P);  // doubles of scratch afl_pair_sqdist_gram needs
int afl_pair_sqdist_gram(const float* G, int K, long P, double* partial, double* D, hipStream_t s);
// GMM gradient filter on the centred Gram matrix (agg.hip k_gmm_filter): keep[n] (0/1), info = {threshold, kept, ok}
int afl_gmm_filter(const double* G, int n, const unsigned char* att, unsigned char* keep, double* info, int rank,
                   hipStream_t s);
// FLTracer PCA(1) scores from the centred Gram [n][n] fp64 (n <= 64): Jacobi eigen-decomposition, z [n] fp64
int afl_top_pc(const double* G, int n, int sweeps, double* z, hipStream_t s);
void afl_noise_philox(const float* own, float* out, long P, float sigma, uint64_t seed, hipStream_t s);

// comm.hip — one-shot intra-node all-gather over IPC-mapped peer buffers (xGMI)
#define AFL_IPC_MAX_PEERS 16
#define AFL_IPC_FLAG_STRIDE 32  // uint32 per flag: one 128-byte line per (parity, sender)
struct AflIpcPeers {
  float* base[AFL_IPC_MAX_PEERS];  // every rank's receive buffer (own rank = local pointer)
  int world;
};
long afl_ipc_buffer_bytes(int world, long cap);
int afl_ipc_alloc(int world, long cap, float** base);
// stream-ordered: push + signal/wait; on a deadline miss (s_memrealtime ticks, 100 MHz) the wait sets bit r of
// *status (pinned host memory) for every sender r it did not hear from
int afl_ipc_all_gather(const float* src, long n, const AflIpcPeers& peers, int rank, long cap, uint32_t epoch,
                       int* status, uint64_t deadline_ticks, hipStream_t s);

// crc.hip — CRC-32 (IEEE 802.3, zlib's crc32) of a device buffer: the checkpoint writer's zip records.
// x2k[k] = x^(2^k) mod P (k < 48, zlib's reflected representation); *out must hold ~(0xFFFFFFFF (*) x^(8 nbytes))
// on entry (the launch XORs every chunk's shifted CRC into it, leaving the final CRC)
int afl_crc32(const void* data, long nbytes, const uint32_t* x2k, uint32_t* out, hipStream_t s);
