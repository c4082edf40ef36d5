// torch bindings of the gfx950 kernels (attackfl_amd._C).  Host side only: shape checks, output
// allocation on the caching allocator, launch on the current HIP stream.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>

#include "kernels.h"

void afl_register_layers(pybind11::module& m);  // layers_bind.cpp
void afl_register_ipc(pybind11::module& m);     // comm/ipc.cpp
void afl_register_har(pybind11::module& m);     // har_bind.cpp

namespace {

hipStream_t cur() { return at::hip::getCurrentHIPStream().stream(); }

// surface launch-configuration errors at the call that caused them
// AFL_SYNC_CHECK=1: synchronise after every launch so an asynchronous fault is reported at the op
// that caused it (debug mode; the GPU counterpart of HIP_LAUNCH_BLOCKING for this extension)
bool sync_check() {
  static const bool on = [] {
    const char* e = getenv("AFL_SYNC_CHECK");
    return e && e[0] == '1';
  }();
  return on;
}
#define AFL_CHECK_LAUNCH()                                                              \
  do {                                                                                 \
    hipError_t e_ = hipGetLastError();                                                 \
    TORCH_CHECK(e_ == hipSuccess, "HIP launch failed: ", hipGetErrorString(e_));       \
    if (sync_check()) {                                                                \
      e_ = hipDeviceSynchronize();                                                     \
      TORCH_CHECK(e_ == hipSuccess, "HIP kernel failed: ", hipGetErrorString(e_));     \
    }                                                                                  \
  } while (0)

void check_dev(const torch::Tensor& t, const char* name, c10::ScalarType dt) {
  TORCH_CHECK(t.is_cuda(), name, " must be a device tensor");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
  TORCH_CHECK(t.scalar_type() == dt, name, " has dtype ", t.scalar_type(), ", expected ", dt);
}

std::vector<torch::Tensor> colstats(torch::Tensor G, int64_t mode, double z) {
  check_dev(G, "G", torch::kFloat32);
  TORCH_CHECK(G.dim() == 2 && G.size(0) >= 1, "G must be [K, P]");
  const int K = G.size(0);
  const long P = G.size(1);
  auto mean = torch::empty({P}, G.options());
  auto stdv = torch::empty({P}, G.options());
  auto out = mode == 1 ? torch::empty({P}, G.options()) : torch::empty({0}, G.options());
  afl_colstats(G.data_ptr<float>(), K, P, mean.data_ptr<float>(), stdv.data_ptr<float>(),
               mode == 1 ? out.data_ptr<float>() : nullptr, (float)z, (int)mode, cur());
  AFL_CHECK_LAUNCH();
  return {mean, stdv, out};
}

torch::Tensor pairwise_sqdist(torch::Tensor G) {
  check_dev(G, "G", torch::kFloat32);
  const int K = G.size(0);
  const long P = G.size(1);
  auto D = torch::zeros({K, K}, G.options().dtype(torch::kFloat64));
  if (K < 2) return D;
  TORCH_CHECK(K <= 128, "pairwise_sqdist supports K <= 128 rows");
  const int M = K * (K - 1) / 2;
  auto partial = torch::empty({(long)afl_pair_sqdist_nblocks(P) * M}, D.options());
  afl_pair_sqdist(G.data_ptr<float>(), K, P, partial.data_ptr<double>(), D.data_ptr<double>(), cur());
  AFL_CHECK_LAUNCH();
  return D;
}

// pairwise squared distances through the centred Gram matrix on fp64 MFMA (K <= 64)
torch::Tensor pairwise_sqdist_gram(torch::Tensor G) {
  check_dev(G, "G", torch::kFloat32);
  TORCH_CHECK(G.dim() == 2 && G.size(0) >= 1 && G.size(0) <= 64, "G must be [K <= 64, P]");
  const int K = G.size(0);
  const long P = G.size(1);
  auto D = torch::zeros({K, K}, G.options().dtype(torch::kFloat64));
  auto scratch = torch::empty({(long)afl_gram_partials(K, P)}, D.options());
  TORCH_CHECK(afl_pair_sqdist_gram(G.data_ptr<float>(), K, P, scratch.data_ptr<double>(), D.data_ptr<double>(),
                                   cur()) == 0, "gram launch failed");
  AFL_CHECK_LAUNCH();
  return D;
}

// GMM filter (agg.gmm): G = centred Gram [n, n] fp64, att [n] uint8 -> (keep [n] uint8, info [3] fp64)
std::vector<torch::Tensor> gmm_filter(torch::Tensor G, torch::Tensor att, int64_t rank) {
  check_dev(G, "G", torch::kFloat64);
  check_dev(att, "att", torch::kUInt8);
  const int64_t n = G.size(0);
  TORCH_CHECK(G.dim() == 2 && G.size(1) == n && att.numel() == n && n >= 1 && n <= 64, "gmm_filter: G [n, n], n <= 64");
  auto keep = torch::zeros({n}, att.options());
  auto info = torch::zeros({3}, G.options());
  TORCH_CHECK(afl_gmm_filter(G.data_ptr<double>(), (int)n, att.data_ptr<uint8_t>(), keep.data_ptr<uint8_t>(),
                             info.data_ptr<double>(), (int)rank, cur()) == 0, "gmm_filter launch failed");
  AFL_CHECK_LAUNCH();
  return {keep, info};
}

// cross-wave column-sum determinism check (tests): vals [W, 64] fp32 -> [64]
torch::Tensor fxsum_test(torch::Tensor vals, int64_t seed, int64_t mode) {
  check_dev(vals, "vals", torch::kFloat32);
  TORCH_CHECK(vals.dim() == 2 && vals.size(1) == 64 && vals.size(0) >= 1 && vals.size(0) <= 8, "vals [W <= 8, 64]");
  auto out = torch::empty({64}, vals.options());
  TORCH_CHECK(afl_fxsum_test(vals.data_ptr<float>(), (int)vals.size(0), (uint32_t)seed, (int)mode, out.data_ptr<float>(),
                             cur()) == 0, "fxsum_test launch failed");
  AFL_CHECK_LAUNCH();
  return out;
}

// FLTracer PCA(1) scores (agg.fltracer): G = centred Gram [n, n] fp64 -> z [n] fp64
torch::Tensor top_pc(torch::Tensor G, int64_t sweeps) {
  check_dev(G, "G", torch::kFloat64);
  const int64_t n = G.size(0);
  TORCH_CHECK(G.dim() == 2 && G.size(1) == n && n >= 1 && n <= 64, "top_pc: G [n, n], n <= 64");
  auto z = torch::empty({n}, G.options());
  TORCH_CHECK(afl_top_pc(G.data_ptr<double>(), (int)n, (int)sweeps, z.data_ptr<double>(), cur()) == 0,
              "top_pc launch failed");
  AFL_CHECK_LAUNCH();
  return z;
}

// Gram matrix of the rows centred on the MEAN row (PCA of the updates: agg.fltracer / agg.gmm), through the same
// fp64-MFMA pass (rows centred on row 0, H) followed by the double centring C = H - rowmean - colmean + mean
std::vector<torch::Tensor> gram_centred(torch::Tensor G) {
  check_dev(G, "G", torch::kFloat32);
  TORCH_CHECK(G.dim() == 2 && G.size(0) >= 1 && G.size(0) <= 64, "G must be [K <= 64, P]");
  const int K = G.size(0);
  const long P = G.size(1);
  auto D = torch::zeros({K, K}, G.options().dtype(torch::kFloat64));
  auto scratch = torch::empty({(long)afl_gram_partials(K, P)}, D.options());
  TORCH_CHECK(afl_pair_sqdist_gram(G.data_ptr<float>(), K, P, scratch.data_ptr<double>(), D.data_ptr<double>(),
                                   cur()) == 0, "gram launch failed");
  AFL_CHECK_LAUNCH();
  auto H = scratch.narrow(0, scratch.numel() - (long)K * K, (long)K * K).view({K, K});
  auto C = H - H.mean(0, true) - H.mean(1, true) + H.mean();
  return {C, D};
}

// own + sigma * N(0,1), Philox4x32-10 keyed by `seed` (Random attack)
torch::Tensor noise_philox(torch::Tensor own, double sigma, int64_t seed) {
  check_dev(own, "own", torch::kFloat32);
  auto out = torch::empty_like(own);
  if (own.numel() == 0) return out;
  afl_noise_philox(own.data_ptr<float>(), out.data_ptr<float>(), own.numel(), (float)sigma, (uint64_t)seed, cur());
  AFL_CHECK_LAUNCH();
  return out;
}

torch::Tensor segment_sqsum(torch::Tensor X, torch::Tensor tiles, torch::Tensor segf, int64_t S) {
  check_dev(X, "X", torch::kFloat32);
  check_dev(tiles, "tiles", torch::kInt32);
  check_dev(segf, "segf", torch::kInt32);
  const int rows = X.size(0);
  const long P = X.size(1);
  const int T = tiles.size(0);
  auto out = torch::empty({rows, S}, X.options().dtype(torch::kFloat64));
  auto partial = torch::empty({(long)T * rows * 2}, out.options());
  afl_seg_reduce(0, X.data_ptr<float>(), P, rows, nullptr, nullptr, tiles.data_ptr<int>(), T, segf.data_ptr<int>(),
                 (int)S, partial.data_ptr<double>(), out.data_ptr<double>(), nullptr, cur());
  AFL_CHECK_LAUNCH();
  return out;
}

std::vector<torch::Tensor> attack_coeffs(torch::Tensor G, torch::Tensor mean, torch::Tensor dev, torch::Tensor tiles,
                                         torch::Tensor segf, int64_t S) {
  check_dev(G, "G", torch::kFloat32);
  check_dev(mean, "mean", torch::kFloat32);
  check_dev(dev, "dev", torch::kFloat32);
  const int K = G.size(0);
  const long P = G.size(1);
  const int rows = K + 1;
  const int T = tiles.size(0);
  auto o0 = torch::empty({rows, S}, G.options().dtype(torch::kFloat64));
  auto o1 = torch::empty({rows, S}, o0.options());
  auto partial = torch::empty({(long)T * rows * 2}, o0.options());
  afl_seg_reduce(1, G.data_ptr<float>(), P, rows, mean.data_ptr<float>(), dev.data_ptr<float>(), tiles.data_ptr<int>(),
                 T, segf.data_ptr<int>(), (int)S, partial.data_ptr<double>(), o0.data_ptr<double>(),
                 o1.data_ptr<double>(), cur());
  AFL_CHECK_LAUNCH();
  return {o0.narrow(0, 0, K), o1.narrow(0, 0, K), o0[K]};
}

torch::Tensor spectral_norm(torch::Tensor X) {
  check_dev(X, "X", torch::kFloat32);
  TORCH_CHECK(X.dim() == 3, "X must be [B, r, c]");
  const int B = X.size(0), r = X.size(1), c = X.size(2);
  auto out = torch::empty({B}, X.options().dtype(torch::kFloat64));
  if (B == 0) return out;
  const int n = r <= c ? r : c;
  if (n > 128) {
    // rare (no model tensor has both dims > 128): exact batched SVD through the library
    return at::linalg_matrix_norm(X.to(torch::kFloat64), 2).contiguous();
  }
  auto scratch = torch::empty({(long)B * afl_spectral_scratch(r, c)}, X.options());
  TORCH_CHECK(afl_spectral(X.data_ptr<float>(), B, r, c, scratch.data_ptr<float>(), out.data_ptr<double>(), cur()) == 0,
              "spectral_norm launch failed");
  AFL_CHECK_LAUNCH();
  return out;
}

// D [M, P] fp32, tab [S, 4] int32 (off, r, c, scratch off; min(r, c) <= 128), scr = scratch per row -> [M, S] fp64
torch::Tensor spec_grams(torch::Tensor X, c10::optional<torch::Tensor> dev, torch::Tensor tab, int64_t max_lds_floats,
                         int64_t sumq) {
  check_dev(X, "X", torch::kFloat32);
  check_dev(tab, "tab", torch::kInt32);
  TORCH_CHECK(X.dim() == 2 && tab.dim() == 2 && tab.size(1) == 4, "spec_grams: bad shapes");
  const int M = X.size(0), S = tab.size(0);
  const float* dp = nullptr;
  if (dev.has_value() && dev->defined()) {
    check_dev(*dev, "dev", torch::kFloat32);
    TORCH_CHECK(dev->numel() == X.size(1), "spec_grams: dev must have P entries");
    dp = dev->data_ptr<float>();
  }
  auto arena = torch::empty({(2L * M + 1) * sumq}, X.options().dtype(torch::kFloat64));
  if (M == 0 || S == 0) return arena;
  TORCH_CHECK(afl_spec_grams(X.data_ptr<float>(), M, X.size(1), dp, tab.data_ptr<int>(), S, (int)max_lds_floats, sumq,
                             arena.data_ptr<double>(), cur()) == 0,
              "spec_grams launch failed");
  AFL_CHECK_LAUNCH();
  return arena;
}

torch::Tensor spec_eval(torch::Tensor arena, torch::Tensor tab, int64_t sumq, int64_t M, c10::optional<torch::Tensor> gamma) {
  check_dev(arena, "arena", torch::kFloat64);
  check_dev(tab, "tab", torch::kInt32);
  TORCH_CHECK(arena.numel() == (2 * M + 1) * sumq, "spec_eval: arena size");
  const int S = tab.size(0);
  const double* gp = nullptr;
  if (gamma.has_value() && gamma->defined()) {
    check_dev(*gamma, "gamma", torch::kFloat64);
    TORCH_CHECK(gamma->numel() == 1, "spec_eval: gamma must be a scalar");
    gp = gamma->data_ptr<double>();
  }
  auto out = torch::empty({M, S}, arena.options());
  if (M == 0 || S == 0) return out;
  TORCH_CHECK(afl_spec_eval(arena.data_ptr<double>(), sumq, (int)M, gp, tab.data_ptr<int>(), S, out.data_ptr<double>(),
                            cur()) == 0,
              "spec_eval launch failed");
  AFL_CHECK_LAUNCH();
  return out;
}

// fused bisection (linalg.hip): st [40] fp64, ctr [1] int32, vA/vB [K, Sv] + vC [Sv] fp64 (optional), thr [1] fp64
static AflBisect make_bisect(torch::Tensor st, c10::optional<torch::Tensor> ctr, c10::optional<torch::Tensor> vA,
                             c10::optional<torch::Tensor> vB, c10::optional<torch::Tensor> vC, torch::Tensor thr,
                             int64_t K, int64_t kind) {
  check_dev(st, "st", torch::kFloat64);
  check_dev(thr, "thr", torch::kFloat64);
  TORCH_CHECK(st.numel() >= 40 && thr.numel() == 1, "bisect: state [40], threshold scalar");
  AflBisect b{};
  b.st = st.data_ptr<double>();
  b.thr = thr.data_ptr<double>();
  b.K = (int)K;
  b.kind = (int)kind;
  if (ctr.has_value() && ctr->defined()) {
    check_dev(*ctr, "ctr", torch::kInt32);
    b.ctr = (unsigned*)ctr->data_ptr<int>();
  }
  if (vA.has_value() && vA->defined()) {
    check_dev(*vA, "vA", torch::kFloat64);
    check_dev(*vB, "vB", torch::kFloat64);
    check_dev(*vC, "vC", torch::kFloat64);
    TORCH_CHECK(vA->dim() == 2 && vA->size(0) == K && vB->sizes() == vA->sizes() && vC->numel() == vA->size(1) &&
                    vA->is_contiguous() && vB->is_contiguous() && vC->is_contiguous(),
                "bisect: vA/vB [K, Sv] and vC [Sv], contiguous");
    b.vA = vA->data_ptr<double>();
    b.vB = vB->data_ptr<double>();
    b.vC = vC->data_ptr<double>();
    b.Sv = (int)vA->size(1);
  }
  return b;
}

void bisect_vec(torch::Tensor st, torch::Tensor vA, torch::Tensor vB, torch::Tensor vC, torch::Tensor thr, int64_t K,
                int64_t kind, int64_t n_iter, double step0) {
  const AflBisect b = make_bisect(st, c10::nullopt, vA, vB, vC, thr, K, kind);
  TORCH_CHECK(afl_bisect_vec(&b, (int)n_iter, step0, cur()) == 0, "bisect_vec: at most 16 iterations");
  AFL_CHECK_LAUNCH();
}

torch::Tensor spec_bisect(torch::Tensor arena, torch::Tensor tab, int64_t sumq, int64_t M, torch::Tensor st,
                          torch::Tensor ctr, c10::optional<torch::Tensor> vA, c10::optional<torch::Tensor> vB,
                          c10::optional<torch::Tensor> vC, torch::Tensor thr, int64_t kind, int64_t it, double step) {
  check_dev(arena, "arena", torch::kFloat64);
  check_dev(tab, "tab", torch::kInt32);
  TORCH_CHECK(arena.numel() == (2 * M + 1) * sumq, "spec_bisect: arena size");
  TORCH_CHECK(it >= 0 && it < 16, "spec_bisect: iteration index");
  const AflBisect b = make_bisect(st, ctr, vA, vB, vC, thr, M + 1, kind);
  TORCH_CHECK(b.ctr != nullptr, "spec_bisect: arrival counter required");
  const int S = tab.size(0);
  auto out = torch::empty({M, S}, arena.options());
  TORCH_CHECK(afl_spec_bisect(arena.data_ptr<double>(), sumq, (int)M, tab.data_ptr<int>(), S, out.data_ptr<double>(),
                              &b, (int)it, step, cur()) == 0,
              "spec_bisect: needs M > 0 rows and S > 0 Gram slots");
  AFL_CHECK_LAUNCH();
  return out;
}

torch::Tensor spectral_norm_slots(torch::Tensor D, torch::Tensor tab, int64_t max_n, int64_t scr) {
  check_dev(D, "D", torch::kFloat32);
  check_dev(tab, "tab", torch::kInt32);
  TORCH_CHECK(D.dim() == 2 && tab.dim() == 2 && tab.size(1) == 4, "spectral_norm_slots: bad shapes");
  const int M = D.size(0), S = tab.size(0);
  auto out = torch::empty({M, S}, D.options().dtype(torch::kFloat64));
  if (M == 0 || S == 0) return out;
  auto scratch = torch::empty({(long)M * scr}, D.options());
  TORCH_CHECK(afl_spectral_slots(D.data_ptr<float>(), M, D.size(1), tab.data_ptr<int>(), S, (int)max_n,
                                 scratch.data_ptr<float>(), scr, out.data_ptr<double>(), cur()) == 0,
              "spectral_norm_slots launch failed");
  AFL_CHECK_LAUNCH();
  return out;
}

torch::Tensor weighted_rows(torch::Tensor U, torch::Tensor w, c10::optional<torch::Tensor> ok,
                            c10::optional<torch::Tensor> fallback) {
  check_dev(U, "U", torch::kFloat32);
  check_dev(w, "w", torch::kFloat64);
  const int N = U.size(0);
  const long P = U.size(1);
  TORCH_CHECK(w.numel() == N, "w must have N entries");
  TORCH_CHECK(ok.has_value() == fallback.has_value(), "weighted_rows: ok and fallback go together");
  const int* okp = nullptr;
  const float* fb = nullptr;
  if (ok.has_value()) {
    check_dev(*ok, "ok", torch::kInt32);
    check_dev(*fallback, "fallback", torch::kFloat32);
    TORCH_CHECK(ok->numel() == N && fallback->numel() == P, "weighted_rows: ok [N], fallback [P]");
    okp = ok->data_ptr<int>();
    fb = fallback->data_ptr<float>();
  }
  auto out = torch::empty({P}, U.options());
  afl_weighted_rows(U.data_ptr<float>(), w.data_ptr<double>(), N, P, out.data_ptr<float>(), cur(), okp, fb);
  AFL_CHECK_LAUNCH();
  return out;
}

torch::Tensor coord_select(torch::Tensor U, int64_t mode, int64_t trim) {
  check_dev(U, "U", torch::kFloat32);
  const int N = U.size(0);
  const long P = U.size(1);
  TORCH_CHECK(N >= 1 && N <= 64, "coord_select supports 1..64 rows");
  TORCH_CHECK(mode == 0 || 2 * trim < N, "trim too large");
  auto out = torch::empty({P}, U.options());
  afl_coord_select(U.data_ptr<float>(), N, P, (int)mode, (int)trim, out.data_ptr<float>(), cur());
  AFL_CHECK_LAUNCH();
  return out;
}

torch::Tensor row_dots(torch::Tensor U, torch::Tensor ref, int64_t mode) {
  check_dev(U, "U", torch::kFloat32);
  const int N = U.size(0);
  const long P = U.size(1);
  if (mode) {
    check_dev(ref, "ref", torch::kFloat32);
    TORCH_CHECK(ref.numel() == P, "ref must have P entries");
  }
  auto out = torch::empty({N, 3}, U.options().dtype(torch::kFloat64));
  auto partial = torch::empty({(long)N * afl_row_dots_nchunks(P) * 3}, out.options());
  afl_row_dots(U.data_ptr<float>(), mode ? ref.data_ptr<float>() : nullptr, N, P, (int)mode,
               partial.data_ptr<double>(), out.data_ptr<double>(), cur());
  AFL_CHECK_LAUNCH();
  return out;
}

std::vector<torch::Tensor> stoch_quant(torch::Tensor U, int64_t seed) {
  check_dev(U, "U", torch::kFloat32);
  const int N = U.size(0);
  const long P = U.size(1);
  auto sigma = torch::empty_like(U);
  auto smin = torch::empty({N}, U.options());
  auto smax = torch::empty({N}, U.options());
  auto ws = torch::empty({afl_stoch_quant_ws(N)}, U.options());
  afl_stoch_quant(U.data_ptr<float>(), N, P, (uint64_t)seed, sigma.data_ptr<float>(), smin.data_ptr<float>(),
                  smax.data_ptr<float>(), ws.data_ptr<float>(), cur());
  AFL_CHECK_LAUNCH();
  return {sigma, smin, smax};
}

void adam_flat(torch::Tensor p, torch::Tensor g, torch::Tensor m, torch::Tensor v, int64_t step, double lr, double b1,
               double b2, double eps, double scale) {
  for (auto* t : {&p, &g, &m, &v}) check_dev(*t, "adam tensor", torch::kFloat32);
  const long n = p.numel();
  TORCH_CHECK(g.numel() == n && m.numel() == n && v.numel() == n, "adam: size mismatch");
  afl_adam_flat(p.data_ptr<float>(), g.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(), n, (int)step,
                (float)lr, (float)b1, (float)b2, (float)eps, (float)scale, cur());
  AFL_CHECK_LAUNCH();
}

// [auc, any NaN score] (device doubles; one host read serves the NaN test and the metric)
torch::Tensor roc_auc_dev(torch::Tensor scores, torch::Tensor labels) {
  check_dev(scores, "scores", torch::kFloat32);
  check_dev(labels, "labels", torch::kFloat32);
  TORCH_CHECK(labels.numel() == scores.numel(), "roc_auc: scores / labels size mismatch");
  const int n = scores.numel();
  auto acc = torch::empty({3}, scores.options().dtype(torch::kInt64));
  auto out = torch::empty({2}, scores.options().dtype(torch::kFloat64));
  if (n <= afl_roc_auc_pairs_max()) {  // direct pair counts, no sort
    afl_roc_auc_pairs(scores.data_ptr<float>(), labels.data_ptr<float>(), n,
                      (unsigned long long*)acc.data_ptr<int64_t>(), out.data_ptr<double>(), cur());
    AFL_CHECK_LAUNCH();
    return out;
  }
  auto sorted = std::get<0>(scores.sort(/*stable=*/false, /*dim=*/0, /*descending=*/false)).contiguous();
  afl_roc_auc(sorted.data_ptr<float>(), scores.data_ptr<float>(), labels.data_ptr<float>(), n,
              (unsigned long long*)acc.data_ptr<int64_t>(), out.data_ptr<double>(), cur());
  AFL_CHECK_LAUNCH();
  return out;
}

double roc_auc(torch::Tensor scores, torch::Tensor labels) { return roc_auc_dev(scores, labels)[0].item<double>(); }

std::vector<torch::Tensor> hyper_delta_vjp(torch::Tensor W, torch::Tensor b, torch::Tensor f, torch::Tensor u) {
  check_dev(W, "W", torch::kFloat32);
  check_dev(b, "b", torch::kFloat32);
  check_dev(f, "f", torch::kFloat32);
  check_dev(u, "u", torch::kFloat32);
  const long P = W.size(0);
  const int H = W.size(1);
  TORCH_CHECK(H <= 128, "hidden size must be <= 128");
  auto delta = torch::empty({P}, W.options());
  auto dfeat = torch::empty({H}, W.options());
  auto partial = torch::empty({(long)afl_hyper_nblocks(P) * H}, W.options());
  afl_hyper_rows(W.data_ptr<float>(), b.data_ptr<float>(), f.data_ptr<float>(), u.data_ptr<float>(), P, H,
                 delta.data_ptr<float>(), partial.data_ptr<float>(), dfeat.data_ptr<float>(), cur());
  AFL_CHECK_LAUNCH();
  return {delta, dfeat};
}

torch::Tensor hyper_generate(torch::Tensor W, torch::Tensor b, torch::Tensor f) {
  check_dev(W, "W", torch::kFloat32);
  const long P = W.size(0);
  const int H = W.size(1);
  TORCH_CHECK(H <= 128, "hidden size must be <= 128");
  auto out = torch::empty({P}, W.options());
  afl_hyper_rows(W.data_ptr<float>(), b.data_ptr<float>(), f.data_ptr<float>(), nullptr, P, H, out.data_ptr<float>(),
                 nullptr, nullptr, cur());
  AFL_CHECK_LAUNCH();
  return out;
}

void hyper_adam_outer(torch::Tensor W, torch::Tensor b, torch::Tensor m, torch::Tensor v, torch::Tensor delta,
                      torch::Tensor f, int64_t step, double lr, double b1, double b2, double eps, double scale) {
  TORCH_CHECK(W.is_cuda() && W.is_contiguous(), "W");
  const long P = W.size(0);
  const int H = W.size(1);
  TORCH_CHECK(m.numel() >= P * H + P && v.numel() >= P * H + P, "moment buffers too small");
  afl_hyper_adam(W.data_ptr<float>(), b.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(),
                 delta.data_ptr<float>(), f.data_ptr<float>(), P, H, (int)step, (float)lr, (float)b1, (float)b2,
                 (float)eps, (float)scale, cur());
  AFL_CHECK_LAUNCH();
}

// layout = [emb, w_0, b_0, ..., w_{L-1}, b_{L-1}, L, E, H, n_nodes, offW, offB, P] (arena float offsets)
HySmallDesc hy_desc(const std::vector<int64_t>& lay, long& offW, long& offB, long& P) {
  HySmallDesc d{};
  TORCH_CHECK(lay.size() >= 8, "hyper layout too short");
  const int L = (int)lay[lay.size() - 7];
  TORCH_CHECK(L >= 1 && L <= 8 && (long)lay.size() == 1 + 2 * L + 7, "hyper layout: bad layer count");
  d.emb = lay[0];
  for (int l = 0; l < L; ++l) {
    d.w[l] = lay[1 + 2 * l];
    d.b[l] = lay[2 + 2 * l];
  }
  const size_t t = 1 + 2 * L;
  d.L = L;
  d.E = (int)lay[t + 1];
  d.H = (int)lay[t + 2];
  d.n_nodes = (int)lay[t + 3];
  offW = lay[t + 4];
  offB = lay[t + 5];
  P = lay[t + 6];
  TORCH_CHECK(d.E >= 1 && d.E <= 128 && d.H >= 1 && d.H <= 127, "hyper: embedding size must be <= 128, hidden <= 127");
  TORCH_CHECK(d.w[0] == d.emb + (long)d.n_nodes * d.E, "hyper: the embedding must precede the MLP in the arena");
  TORCH_CHECK(offW - d.emb <= afl_hyper_small_capacity(), "hyper: embedding + MLP too large for the small-net kernel");
  return d;
}

// Whole sequential hypernetwork server update of one round (every selected client in order), enqueued
// without a host synchronisation.  Returns {info [n, 2] = (grad norm, clip scale) per client, gen [ngen, P]}
// (device): gen = the models of the clients ``gen`` generated by the updated hypernetwork (by the unchanged one
// when ``enable`` is 0), produced inside the update's last launches (empty when no client is asked for).
std::vector<torch::Tensor> hyper_server_update(torch::Tensor arena, torch::Tensor m, torch::Tensor v, torch::Tensor U,
                                               std::vector<int64_t> urows, std::vector<int64_t> clients,
                                               std::vector<int64_t> lay, int64_t step0, double lr, double clip,
                                               double b1, double b2, double eps, c10::optional<torch::Tensor> enable,
                                               std::vector<int64_t> gen) {
  for (auto* t : {&arena, &m, &v, &U}) check_dev(*t, "hyper tensor", torch::kFloat32);
  const int* en = nullptr;
  if (enable.has_value() && enable->defined()) {
    check_dev(*enable, "enable", torch::kInt32);
    TORCH_CHECK(enable->numel() == 1, "hyper: enable must be one int32");
    en = enable->data_ptr<int>();
  }
  long offW, offB, P;
  HySmallDesc d = hy_desc(lay, offW, offB, P);
  const int n = (int)clients.size();
  TORCH_CHECK(n >= 1 && (int)urows.size() == n, "hyper: clients / rows mismatch");
  TORCH_CHECK(arena.numel() == offB + P && m.numel() == arena.numel() && v.numel() == arena.numel(), "hyper: arena");
  TORCH_CHECK(U.dim() == 2 && U.size(1) == P, "hyper: updates must be [rows, P]");
  TORCH_CHECK(d.H % 4 == 0 && offW % 4 == 0, "hyper: head block must be float4-aligned");
  for (int k = 0; k < n; ++k) {
    TORCH_CHECK(urows[k] >= 0 && urows[k] < U.size(0), "hyper: update row out of range");
    TORCH_CHECK(clients[k] >= 0 && clients[k] < d.n_nodes, "hyper: client index out of range");
  }
  const int ng = (int)gen.size();
  TORCH_CHECK(ng <= 32, "hyper: at most 32 generated clients per update");
  for (int k = 0; k < ng; ++k) TORCH_CHECK(gen[k] >= 0 && gen[k] < d.n_nodes, "hyper: generated client out of range");
  std::vector<int> cl(clients.begin(), clients.end());
  std::vector<int> gl(gen.begin(), gen.end());
  std::vector<long> ur(urows.begin(), urows.end());
  auto opt = arena.options();
  auto gfeat = torch::empty({std::max(ng, 1) * (long)d.H}, opt);
  auto gout = torch::empty({ng, P}, opt);
  auto delta = torch::empty({2 * P}, opt);  // (two: the fused head Adam reads client k's, writes client k+1's)
  auto partial = torch::empty({(long)afl_hyper_nblocks(P) * (d.H + 1)}, opt);
  auto feat = torch::empty({2 * 128}, opt);
  auto info = torch::empty({n, 2}, opt);
  afl_hyper_server_update(arena.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(), U.data_ptr<float>(),
                          ur.data(), cl.data(), n, d, offW, offB, P, (int)step0, (float)lr, (float)clip, (float)b1,
                          (float)b2, (float)eps, delta.data_ptr<float>(), partial.data_ptr<float>(),
                          feat.data_ptr<float>(), info.data_ptr<float>(), en, gl.data(), ng, gfeat.data_ptr<float>(),
                          gout.data_ptr<float>(), cur());
  AFL_CHECK_LAUNCH();
  return {info, gout};
}

// models of several clients generated by the hypernetwork (features launch + one sweep over the heads): [n, P]
torch::Tensor hyper_generate_many(torch::Tensor arena, std::vector<int64_t> clients, std::vector<int64_t> lay) {
  check_dev(arena, "arena", torch::kFloat32);
  long offW, offB, P;
  HySmallDesc d = hy_desc(lay, offW, offB, P);
  TORCH_CHECK(d.H % 4 == 0 && offW % 4 == 0 && arena.numel() == offB + P, "hyper: head block must be float4-aligned");
  const int n = (int)clients.size();
  for (int k = 0; k < n; ++k) TORCH_CHECK(clients[k] >= 0 && clients[k] < d.n_nodes, "hyper: client out of range");
  std::vector<int> cl(clients.begin(), clients.end());
  auto feat = torch::empty({n, d.H}, arena.options());
  auto out = torch::empty({n, P}, arena.options());
  if (n) {
    afl_hyper_features(arena.data_ptr<float>(), d, offW, cl.data(), n, feat.data_ptr<float>(), cur());
    afl_hyper_generate(arena.data_ptr<float>(), d, offW, offB, P, feat.data_ptr<float>(), n, out.data_ptr<float>(),
                       cur());
  }
  AFL_CHECK_LAUNCH();
  return out;
}

// hypernetwork features (embedding -> MLP output) of several clients -> [n, H]
torch::Tensor hyper_features(torch::Tensor arena, std::vector<int64_t> clients, std::vector<int64_t> lay) {
  check_dev(arena, "arena", torch::kFloat32);
  long offW, offB, P;
  HySmallDesc d = hy_desc(lay, offW, offB, P);
  const int n = (int)clients.size();
  for (int k = 0; k < n; ++k) TORCH_CHECK(clients[k] >= 0 && clients[k] < d.n_nodes, "hyper: client out of range");
  std::vector<int> cl(clients.begin(), clients.end());
  auto out = torch::empty({n, d.H}, arena.options());
  if (n) afl_hyper_features(arena.data_ptr<float>(), d, offW, cl.data(), n, out.data_ptr<float>(), cur());
  AFL_CHECK_LAUNCH();
  return out;
}

// per-step batch tables (idx [S, C, B], bsz [S, C], ep [S, C], nb [C]) from a visit plan, plus zeroed per-round
// words: zi int32 / zf fp32 tensors (any shape, contiguous) are zero-filled by the same launch (plan.hip)
std::vector<torch::Tensor> step_tables(torch::Tensor order, torch::Tensor nd, int64_t B, int64_t S,
                                       std::vector<torch::Tensor> zi, std::vector<torch::Tensor> zf) {
  check_dev(order, "order", torch::kInt32);
  check_dev(nd, "nd", torch::kInt32);
  TORCH_CHECK(order.dim() == 3 && nd.numel() == order.size(0), "step_tables: order [C, E, maxnd], nd [C]");
  TORCH_CHECK(B >= 1 && S >= 0, "step_tables: bad sizes");
  TORCH_CHECK(zi.size() <= 1 && zf.size() <= 1, "step_tables: at most one int32 and one fp32 tensor to zero");
  const int C = order.size(0), E = order.size(1), maxnd = order.size(2);
  auto idx = torch::empty({S, C, B}, order.options());
  auto bsz = torch::empty({S, C}, order.options());
  auto ep = torch::empty({S, C}, order.options());
  auto nb = torch::empty({C}, order.options());
  int* zip = nullptr;
  float* zfp = nullptr;
  long nzi = 0, nzf = 0;
  if (!zi.empty()) {
    check_dev(zi[0], "zi", torch::kInt32);
    zip = zi[0].data_ptr<int>();
    nzi = zi[0].numel();
  }
  if (!zf.empty()) {
    check_dev(zf[0], "zf", torch::kFloat32);
    zfp = zf[0].data_ptr<float>();
    nzf = zf[0].numel();
  }
  TORCH_CHECK(E >= 1 || S == 0, "step_tables: no epochs");
  afl_step_tables(order.data_ptr<int>(), nd.data_ptr<int>(), C, std::max(E, 1), std::max(maxnd, 1), (int)B, (int)S,
                  idx.data_ptr<int>(), bsz.data_ptr<int>(), ep.data_ptr<int>(), nb.data_ptr<int>(), zip, nzi, zfp, nzf,
                  cur());
  AFL_CHECK_LAUNCH();
  return {idx, bsz, ep, nb};
}

// [C, E, maxnd] int32 visit plan from per-client 64-bit seeds (plan.hip); padding is 0
torch::Tensor make_plan(torch::Tensor seeds, torch::Tensor nd, int64_t n_train, int64_t epochs, int64_t maxnd) {
  check_dev(seeds, "seeds", torch::kInt64);
  check_dev(nd, "nd", torch::kInt32);
  const int C = seeds.numel();
  TORCH_CHECK(nd.numel() == C, "make_plan: seeds / nd size mismatch");
  TORCH_CHECK(n_train >= 1 && n_train < (1L << 30) && maxnd >= 0 && maxnd <= n_train, "make_plan: bad sizes");
  auto order = torch::empty({C, epochs, maxnd}, nd.options());
  afl_make_plan((const uint64_t*)seeds.data_ptr<int64_t>(), nd.data_ptr<int>(), C, (int)n_train, (int)epochs,
                (int)maxnd, order.data_ptr<int>(), cur());
  AFL_CHECK_LAUNCH();
  return order;
}

// Fused whole-round trainers: kind 0 = TransformerModel (split 1 / 2 / 3 workgroups per client),
// kind 1 = RNNModel (always 3 workgroups per client).
std::vector<torch::Tensor> fused_train(int kind, torch::Tensor params, torch::Tensor rows, torch::Tensor order,
                                       torch::Tensor nd, torch::Tensor seeds, int64_t epochs, int64_t batch, double lr,
                                       int64_t opt_mode, c10::optional<torch::Tensor> stamps, int64_t split,
                                       c10::optional<torch::Tensor> kt = c10::nullopt) {
  check_dev(params, "params", torch::kFloat32);
  check_dev(rows, "rows", torch::kFloat32);
  check_dev(order, "order", torch::kInt32);
  check_dev(nd, "nd", torch::kInt32);
  check_dev(seeds, "seeds", torch::kInt32);
  const long P = kind == 0 ? afl_tf_param_count() : afl_rnn_param_count();
  TORCH_CHECK(params.dim() == 2 && params.size(1) == P, "params must be [C, ", P, "]");
  TORCH_CHECK(rows.dim() == 2 && rows.size(1) == 24, "rows must be [N, 24]");
  const int C = params.size(0);
  TORCH_CHECK(order.dim() == 3 && order.size(0) == C && order.size(1) == epochs, "order must be [C, E, maxnd]");
  TORCH_CHECK(batch >= 2 && batch <= 128, "fused trainer supports batch sizes 2..128");
  TORCH_CHECK(kind == 1 || (split >= 1 && split <= 4), "TransformerModel trainer split must be 1..4, got ", split);
  // split 4 = the on-chip trainers (tf2.hip / rnn2.hip: 3 workgroups per client, state in registers / LDS)
  const bool tf2 = kind == 0 && split == 4, rnn2 = kind == 1 && split == 4;
  const long wsf = tf2 ? afl_tf2_ws_floats() : rnn2 ? afl_rnn2_ws_floats() : kind == 0 ? afl_tf_ws_floats() : afl_rnn_ws_floats();
  const long stride = ((wsf + 63) / 64) * 64;
  auto ws = torch::empty({(long)C * stride}, params.options());
  const int split_eff = kind == 1 ? 3 : (int)std::max<int64_t>(1, split);  // (rnn2 / tf2: 3 workgroups per client)
  const long sync_words = split_eff > 1 ? (long)C * (tf2 || rnn2 ? AFL_TF2_SYNC_WORDS : AFL_TF_SYNC_WORDS) : 0;
  // ok [C] | losses [C, E] | the hand-off words (16-byte aligned): ONE zero fill per launch
  const long head = ((long)C + (long)C * epochs + 3) / 4 * 4;
  auto zero = torch::zeros({head + sync_words}, order.options());
  auto ok = zero.narrow(0, 0, C);
  auto losses = zero.narrow(0, C, (long)C * epochs).view(torch::kFloat32).view({(long)C, epochs});
  if (C == 0) return {ok, losses};
  AflTfTrainArgs a;
  a.params = params.data_ptr<float>();
  a.rows = rows.data_ptr<float>();
  a.order = order.data_ptr<int>();
  a.nd = nd.data_ptr<int>();
  a.seeds = (const uint32_t*)seeds.data_ptr<int>();
  a.ws = ws.data_ptr<float>();
  a.ws_stride = stride;
  a.ok = ok.data_ptr<int>();
  a.losses = losses.data_ptr<float>();
  a.C = C;
  a.E = (int)epochs;
  a.maxnd = order.size(2);
  a.batch = (int)batch;
  a.lr = (float)lr;
  a.opt_mode = (int)opt_mode;
  a.stamps = nullptr;
  if (stamps.has_value() && stamps->defined()) {
    TORCH_CHECK(stamps->is_cuda() && stamps->scalar_type() == torch::kInt64 && stamps->numel() >= 64,
                "stamps must be a device int64 tensor with >= 64 entries");
    a.stamps = (uint64_t*)stamps->data_ptr<int64_t>();
  }
  a.sync = nullptr;
  a.kt = nullptr;
  a.kt_n = 0;
  if (kt.has_value() && kt->defined()) {
    check_dev(*kt, "kt", torch::kFloat32);
    TORCH_CHECK(kt->dim() == 2 && kt->size(1) == 2, "kt must be [steps, 2]");
    a.kt = kt->data_ptr<float>();
    a.kt_n = (int)kt->size(0);
  }
  a.split = split_eff;
  a.cpad = 0;  // (the on-chip launchers pad the role-major block stride themselves)
  if (a.split > 1) a.sync = (uint32_t*)zero.data_ptr<int>() + head;  // branch-parallel: zeroed hand-off words
  const int rc = tf2 ? afl_tf2_train(&a, cur()) : rnn2 ? afl_rnn2_train(&a, cur())
                 : kind == 0 ? afl_tf_train(&a, cur()) : afl_rnn_train(&a, cur());
  TORCH_CHECK(rc != -4, "branch-parallel fused trainer needs split * C <= CUs (all workgroups resident at once): "
              "launch at most onchip_capacity() clients at a time (ops/transformer.py chunked; AFL_MAX_CLIENTS_PER_LAUNCH "
              "caps it)");
  TORCH_CHECK(rc != -5, "on-chip trainer: Adam step table (kt) missing or shorter than the round");
  TORCH_CHECK(rc == 0, "fused trainer launch failed (", rc, ")");
  AFL_CHECK_LAUNCH();
  return {ok, losses};
}

std::vector<torch::Tensor> tf_train(torch::Tensor params, torch::Tensor rows, torch::Tensor order, torch::Tensor nd,
                                    torch::Tensor seeds, int64_t epochs, int64_t batch, double lr,
                                    int64_t opt_mode, c10::optional<torch::Tensor> stamps, int64_t split,
                                    c10::optional<torch::Tensor> kt) {
  return fused_train(0, params, rows, order, nd, seeds, epochs, batch, lr, opt_mode, stamps, split, kt);
}

// split 3 = rnn.hip (global-workspace kernel), 4 = rnn2.hip (on-chip; needs the Adam step table kt)
std::vector<torch::Tensor> rnn_train(torch::Tensor params, torch::Tensor rows, torch::Tensor order, torch::Tensor nd,
                                     torch::Tensor seeds, int64_t epochs, int64_t batch, double lr, int64_t opt_mode,
                                     int64_t split, c10::optional<torch::Tensor> kt, c10::optional<torch::Tensor> stamps) {
  return fused_train(1, params, rows, order, nd, seeds, epochs, batch, lr, opt_mode, stamps, split, kt);
}

// eval forward of C RNNModels (params [C, P]) over the same rows -> [C, n]: ONE launch (rnn2.hip)
torch::Tensor rnn_eval_many(torch::Tensor params, torch::Tensor rows) {
  check_dev(params, "params", torch::kFloat32);
  check_dev(rows, "rows", torch::kFloat32);
  TORCH_CHECK(params.dim() == 2 && params.size(1) == afl_rnn_param_count(), "params must be [C, 97665]");
  TORCH_CHECK(rows.dim() == 2 && rows.size(1) == 24, "rows must be [N, 24]");
  const int C = params.size(0), n = rows.size(0);
  auto out = torch::empty({C, n}, rows.options());
  TORCH_CHECK(afl_rnn2_eval(params.data_ptr<float>(), params.stride(0), C, rows.data_ptr<float>(), n,
                            out.data_ptr<float>(), cur()) == 0, "rnn_eval launch failed");
  AFL_CHECK_LAUNCH();
  return out;
}

// eval forward of C TransformerModels (params [C, P]) over the same rows -> [C, n]; one call, 3 launches per
// model from C++ (the hyper validation scores every client's generated model)
torch::Tensor tf_eval_many(torch::Tensor params, torch::Tensor rows) {
  check_dev(params, "params", torch::kFloat32);
  check_dev(rows, "rows", torch::kFloat32);
  TORCH_CHECK(params.dim() == 2 && params.size(1) == afl_tf_param_count(), "params must be [C, 47693]");
  const int C = params.size(0), n = rows.size(0);
  auto out = torch::empty({C, n}, rows.options());
  const long bfs = ((long)afl_tf_bf_ushorts() + 63) / 64 * 64;  // per-model bf16 copies, 128-B aligned
  auto bf = torch::empty({(long)C * bfs / 2}, params.options());
  if (n == 0 || C == 0) return out;
  TORCH_CHECK(afl_tf_eval_many(params.data_ptr<float>(), params.stride(0), (unsigned short*)bf.data_ptr<float>(), bfs,
                               C, rows.data_ptr<float>(), n, out.data_ptr<float>(), cur()) == 0,
              "tf_eval launch failed");
  AFL_CHECK_LAUNCH();
  return out;
}

torch::Tensor tf_eval(torch::Tensor params, torch::Tensor rows) {
  check_dev(params, "params", torch::kFloat32);
  check_dev(rows, "rows", torch::kFloat32);
  TORCH_CHECK(params.numel() == afl_tf_param_count(), "params must have 47693 entries");
  const int n = rows.size(0);
  auto out = torch::empty({n}, rows.options());
  auto bf = torch::empty({(long)(afl_tf_bf_ushorts() + 1) / 2}, params.options());
  if (n == 0) return out;
  afl_tf_eval_bf(params.data_ptr<float>(), (unsigned short*)bf.data_ptr<float>(), rows.data_ptr<float>(), n,
                 out.data_ptr<float>(), cur());
  AFL_CHECK_LAUNCH();
  return out;
}

// ---- CRC-32 of a device buffer (crc.hip): host side computes the x^(8n) mod P fold constants ----
uint32_t crc_multmodp(uint32_t a, uint32_t b) {  // a (*) b mod P, reflected; a != 0
  uint32_t p = 0;
  for (uint32_t m = 1u << 31; m; m >>= 1) {
    if (a & m) {
      p ^= b;
      if ((a & (m - 1)) == 0) break;
    }
    b = (b & 1) ? (b >> 1) ^ 0xEDB88320u : b >> 1;
  }
  return p;
}

// zlib-compatible CRC-32 of the bytes of a contiguous device tensor -> int32 device tensor [1] (the CRC's bits)
torch::Tensor crc32(torch::Tensor data) {
  TORCH_CHECK(data.is_cuda() && data.is_contiguous(), "data must be a contiguous device tensor");
  const long nbytes = data.numel() * (long)data.element_size();
  TORCH_CHECK(nbytes > 0 && nbytes % 4 == 0, "crc32: byte count must be a positive multiple of 4");
  uint32_t x2k[48];
  uint32_t p = 1u << 30;  // x^1
  for (int k = 0; k < 48; ++k) {
    x2k[k] = p;  // x^(2^k)
    p = crc_multmodp(p, p);
  }
  uint32_t init = 0xFFFFFFFFu;  // the init register shifted through all nbytes: 0xFFFFFFFF (*) x^(8 nbytes)
  uint64_t e = (uint64_t)nbytes * 8;
  for (int k = 0; e; ++k, e >>= 1)
    if (e & 1) init = crc_multmodp(x2k[k], init);
  auto out = torch::full({1}, (int64_t)(int32_t)(~init), data.options().dtype(torch::kInt32));
  TORCH_CHECK(afl_crc32(data.data_ptr(), nbytes, x2k, (uint32_t*)out.data_ptr<int>(), cur()) == 0,
              "crc32 launch failed");
  AFL_CHECK_LAUNCH();
  return out;
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.def("crc32", &crc32);
  m.def("pairwise_sqdist_gram", &pairwise_sqdist_gram);
  m.def("noise_philox", &noise_philox);
  m.doc() = "attackfl_amd native gfx950 kernels";
  m.def("colstats", &colstats);
  m.def("pairwise_sqdist", &pairwise_sqdist);
  m.def("segment_sqsum", &segment_sqsum);
  m.def("attack_coeffs", &attack_coeffs);
  m.def("spectral_norm", &spectral_norm);
  m.def("spectral_norm_slots", &spectral_norm_slots);
  m.def("spec_grams", &spec_grams);
  m.def("spec_eval", &spec_eval);
  m.def("spec_bisect", &spec_bisect);
  m.def("bisect_vec", &bisect_vec);
  m.def("weighted_rows", &weighted_rows, pybind11::arg("U"), pybind11::arg("w"), pybind11::arg("ok") = pybind11::none(),
        pybind11::arg("fallback") = pybind11::none());
  m.def("coord_select", &coord_select);
  m.def("row_dots", &row_dots);
  m.def("gmm_filter", &gmm_filter, pybind11::arg("G"), pybind11::arg("att"), pybind11::arg("rank") = 0);
  m.def("top_pc", &top_pc);
  m.def("fxsum_test", &fxsum_test);
  m.def("gram_centred", &gram_centred);
  m.def("stoch_quant", &stoch_quant);
  m.def("adam_flat", &adam_flat);
  m.def("roc_auc", &roc_auc);
  m.def("roc_auc_dev", &roc_auc_dev);
  m.def("tf_eval_many", &tf_eval_many);
  m.def("hyper_delta_vjp", &hyper_delta_vjp);
  m.def("hyper_generate", &hyper_generate);
  m.def("hyper_adam_outer", &hyper_adam_outer);
  m.def("hyper_server_update", &hyper_server_update);
  m.def("make_plan", &make_plan);
  m.def("step_tables", &step_tables);
  m.def("hyper_features", &hyper_features);
  m.def("hyper_generate_many", &hyper_generate_many);
  m.def("hyper_small_capacity", &afl_hyper_small_capacity);
  m.def("tf_train", &tf_train, py::arg("params"), py::arg("rows"), py::arg("order"), py::arg("nd"),
        py::arg("seeds"), py::arg("epochs"), py::arg("batch"), py::arg("lr"), py::arg("opt_mode") = 0,
        py::arg("stamps") = py::none(), py::arg("split") = 1, py::arg("kt") = py::none());
  m.def("rnn_train", &rnn_train, py::arg("params"), py::arg("rows"), py::arg("order"), py::arg("nd"),
        py::arg("seeds"), py::arg("epochs"), py::arg("batch"), py::arg("lr"), py::arg("opt_mode") = 0,
        py::arg("split") = 3, py::arg("kt") = py::none(), py::arg("stamps") = py::none());
  m.def("rnn_param_count", &afl_rnn_param_count);
  m.def("rnn_eval_many", &rnn_eval_many, py::arg("params"), py::arg("rows"));
  m.def("tf_eval", &tf_eval);
  m.def("tf_param_count", &afl_tf_param_count);
  m.def("tf_ws_floats", &afl_tf_ws_floats);
  afl_register_layers(m);
  afl_register_ipc(m);
  afl_register_har(m);
}
