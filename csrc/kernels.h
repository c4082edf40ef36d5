// Host-side launchers of the gfx950 kernels (raw pointers + stream; no torch headers so the
// device translation units compile in seconds).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// agg.hip
void afl_colstats(const float* G, int K, long P, float* mean, float* stdv, float* out, float z, int mode,
                  hipStream_t s);
void afl_weighted_rows(const float* U, const double* w, int N, long P, float* out, hipStream_t s);
int afl_pair_sqdist_nblocks(long P);
void afl_pair_sqdist(const float* G, int K, long P, double* partial, double* D, hipStream_t s);
void afl_seg_reduce(int mode, const float* X, long P, int rows, const float* mean, const float* dev, const int* tiles,
                    int T, const int* segf, int S, double* partial, double* out0, double* out1, hipStream_t s);
void afl_coord_select(const float* U, int N, long P, int mode, int trim, float* out, hipStream_t s);
int afl_row_dots_nchunks(long P);
void afl_row_dots(const float* U, const float* ref, int N, long P, int mode, double* partial, double* out,
                  hipStream_t s);
void afl_stoch_quant(const float* U, int N, long P, uint64_t seed, float* sigma, float* smin, float* smax,
                     hipStream_t s);
void afl_adam_flat(float* p, const float* g, float* m, float* v, long n, int step, float lr, float b1, float b2,
                   float eps, float gscale, hipStream_t s);

// hyper.hip
int afl_hyper_nblocks(long P);
void afl_hyper_rows(const float* W, const float* b, const float* f, const float* u, long P, int H, float* out,
                    float* partial, float* dfeat, hipStream_t s);
void afl_hyper_adam(float* W, float* bvec, float* m, float* v, const float* delta, const float* f, long P, int H,
                    int step, float lr, float b1, float b2, float eps, float gs, hipStream_t s);

// linalg.hip
int afl_spectral_scratch(int r, int c);
int afl_spectral(const float* X, int B, int r, int c, float* G0, double* out, hipStream_t s);

// metrics.hip
void afl_roc_auc_sorted(const float* s, const float* y, int n, double* out, hipStream_t st);

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
};
int afl_tf_train(const AflTfTrainArgs* a, hipStream_t s);
int afl_tf_eval_bf(const float* params, unsigned short* bf, const float* rows, int n, float* out, hipStream_t s);
long afl_tf_ws_floats();
int afl_tf_bf_ushorts();
int afl_tf_param_count();
