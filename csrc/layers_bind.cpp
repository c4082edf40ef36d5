// torch bindings of the client-batched layer kernels (layers.hip, attention.hip).
// Every op writes into caller-provided tensors (no allocation): the per-model step programs
// (attackfl_amd/fl/programs.py) preallocate their buffers once and capture the launch sequence in a
// HIP graph.  Strided operands are passed as 3-D views [C][rows][cols]; their strides go to the
// kernels unchanged (weights are views into the flat [C][P] parameter arena, transposes are free).
#include <map>
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>

#include <cmath>

#include "kernels.h"

namespace {

hipStream_t cur() { return at::hip::getCurrentHIPStream().stream(); }

void ok(int e, const char* what) {
  TORCH_CHECK(e == 0, what, " launch failed: ", hipGetErrorString((hipError_t)e));
  static const bool sync = [] {  // AFL_SYNC_CHECK=1: report asynchronous faults at the faulting op
    const char* v = getenv("AFL_SYNC_CHECK");
    return v && v[0] == '1';
  }();
  if (sync) {
    const hipError_t s = hipDeviceSynchronize();
    TORCH_CHECK(s == hipSuccess, what, " kernel failed: ", hipGetErrorString(s));
  }
}

void dev(const torch::Tensor& t, const char* n, c10::ScalarType dt = torch::kFloat32) {
  TORCH_CHECK(t.defined() && t.is_cuda(), n, " must be a device tensor");
  TORCH_CHECK(t.scalar_type() == dt, n, " has dtype ", t.scalar_type(), ", expected ", dt);
}
void dense(const torch::Tensor& t, const char* n, c10::ScalarType dt = torch::kFloat32) {
  dev(t, n, dt);
  TORCH_CHECK(t.is_contiguous(), n, " must be contiguous");
}
void view3(const torch::Tensor& t, const char* n) {
  dev(t, n);
  TORCH_CHECK(t.dim() == 3, n, " must be a 3-D [C, rows, cols] view");
}
const float* optp(const c10::optional<torch::Tensor>& t) {
  return (t.has_value() && t->defined()) ? t->data_ptr<float>() : nullptr;
}

AflDrop make_drop(const c10::optional<torch::Tensor>& seeds, const c10::optional<torch::Tensor>& stepctl,
                  int64_t layer, double p) {
  AflDrop d{};
  if (p <= 0.0) return d;
  TORCH_CHECK(seeds.has_value() && seeds->defined(), "dropout needs client seeds");
  dense(*seeds, "seeds", torch::kInt32);
  d.seeds = (const uint32_t*)seeds->data_ptr<int>();
  if (stepctl.has_value() && stepctl->defined()) {
    dense(*stepctl, "stepctl", torch::kInt32);
    d.stepctl = stepctl->data_ptr<int>();
  }
  d.layer = (uint32_t)layer;
  d.thr16 = (uint32_t)std::lround(p * 65536.0);
  d.inv_keep = (float)(1.0 / (1.0 - p));
  return d;
}

// C (op)= epi(alpha * A . B^T): A [C, M, K], B [C, N, K], C [C, M, N] (any strides)
void bgemm(torch::Tensor A, torch::Tensor B, torch::Tensor Cm, c10::optional<torch::Tensor> bias,
           c10::optional<torch::Tensor> Z, c10::optional<torch::Tensor> G, int64_t act, int64_t gact, int64_t accum,
           int64_t splitk, double alpha, c10::optional<torch::Tensor> seeds, c10::optional<torch::Tensor> stepctl,
           int64_t layer, double p, int64_t generic, c10::optional<torch::Tensor> asum) {
  view3(A, "A");
  view3(B, "B");
  view3(Cm, "C");
  const long nC = A.size(0), M = A.size(1), K = A.size(2), N = B.size(1);
  TORCH_CHECK(B.size(0) == nC && B.size(2) == K, "B must be [C, N, K]");
  TORCH_CHECK(Cm.size(0) == nC && Cm.size(1) == M && Cm.size(2) == N, "C must be [C, M, N]");
  AflGemm g{};
  g.A = A.data_ptr<float>();
  g.sAc = A.stride(0); g.sAm = A.stride(1); g.sAk = A.stride(2);
  g.B = B.data_ptr<float>();
  g.sBc = B.stride(0); g.sBn = B.stride(1); g.sBk = B.stride(2);
  g.Cm = Cm.data_ptr<float>();
  g.sCc = Cm.stride(0); g.sCm = Cm.stride(1); g.sCn = Cm.stride(2);
  if (bias.has_value() && bias->defined()) {
    dev(*bias, "bias");
    TORCH_CHECK(bias->dim() == 2 && bias->size(0) == nC && bias->size(1) == N && bias->stride(1) == 1,
                "bias must be a [C, N] view with unit column stride");
    g.bias = bias->data_ptr<float>();
    g.sbc = bias->stride(0);
  }
  if (Z.has_value() && Z->defined()) {
    view3(*Z, "Z");
    TORCH_CHECK(Z->sizes() == Cm.sizes() && Z->strides() == Cm.strides(), "Z must match C's shape and strides");
    g.Z = Z->data_ptr<float>();
  }
  if (G.has_value() && G->defined()) {
    view3(*G, "G");
    TORCH_CHECK(G->size(0) == nC && G->size(1) == M && G->size(2) == N, "G must be [C, M, N]");
    g.G = G->data_ptr<float>();
    g.sGc = G->stride(0); g.sGm = G->stride(1); g.sGn = G->stride(2);
  }
  g.M = M; g.N = N; g.K = K; g.nC = nC;
  g.act = act; g.gact = gact; g.accum = accum; g.splitk = std::max<int64_t>(1, splitk);
  g.alpha = (float)alpha;
  g.drop = make_drop(seeds, stepctl, layer, p);
  g.no_ts = generic ? 1 : 0;
  if (asum.has_value() && asum->defined()) {
    dev(*asum, "asum");
    TORCH_CHECK(asum->dim() == 2 && asum->size(0) == nC && asum->size(1) == K && asum->stride(1) == 1,
                "asum must be a [C, K] view with unit column stride");
    TORCH_CHECK(A.stride(2) == 1, "asum needs k-contiguous A rows");
    g.asum = asum->data_ptr<float>();
    g.sasc = asum->stride(0);
  }
  // split-K: deterministic (ordered partial sums) — the workspace lives in the caching allocator, stream-ordered
  // (inside a captured step it comes from the graph's private pool)
  torch::Tensor ws, ws_sum;
  const long nws = afl_bgemm_ws_floats(g);
  if (nws > 0) {
    ws = torch::empty({nws}, A.options());
    g.ws = ws.data_ptr<float>();
  }
  const long nsum = afl_bgemm_asum_ws_floats(g);  // the fused bias-gradient column sums: ordered partials
  if (nsum > 0) {
    ws_sum = torch::empty({nsum}, A.options());
    g.ws_sum = ws_sum.data_ptr<float>();
  }
  ok(afl_bgemm(g, cur()), "bgemm");
}

void colsum(torch::Tensor Y, torch::Tensor out) {
  view3(Y, "Y");
  dev(out, "out");
  TORCH_CHECK(Y.stride(2) == 1, "Y columns must be contiguous");
  TORCH_CHECK(out.dim() == 2 && out.size(0) == Y.size(0) && out.size(1) == Y.size(2) && out.stride(1) == 1,
              "out must be a [C, N] view");
  auto ws = torch::empty({afl_colsum_ws_floats(Y.size(1), Y.size(2), Y.size(0))}, Y.options());  // ordered partials
  ok(afl_colsum(Y.data_ptr<float>(), Y.stride(0), Y.stride(1), Y.size(1), Y.size(2), Y.size(0), out.data_ptr<float>(),
                out.stride(0), cur(), ws.data_ptr<float>()),
     "colsum");
}

void gather_icu(torch::Tensor rows, torch::Tensor idx, torch::Tensor stepctl, int64_t mask, torch::Tensor vit,
                torch::Tensor lab, torch::Tensor y) {
  dense(rows, "rows");
  dense(idx, "idx", torch::kInt32);
  dense(stepctl, "stepctl", torch::kInt32);
  dense(vit, "vit");
  dense(lab, "lab");
  dense(y, "y");
  TORCH_CHECK(rows.dim() == 2 && rows.size(1) == 24 && idx.dim() == 3, "rows [N, 24], idx [S, C, B]");
  const int C = idx.size(1), B = idx.size(2);
  TORCH_CHECK(vit.numel() == (long)C * B * 7 && lab.numel() == (long)C * B * 16 && y.numel() == (long)C * B,
              "output sizes");
  ok(afl_gather_icu(rows.data_ptr<float>(), idx.data_ptr<int>(), stepctl.data_ptr<int>(), C, B, (int)mask,
                    vit.data_ptr<float>(), lab.data_ptr<float>(), y.data_ptr<float>(), cur()),
     "gather_icu");
}

void gather_har(torch::Tensor x, torch::Tensor y, torch::Tensor idx, torch::Tensor stepctl, torch::Tensor ox,
                torch::Tensor oy) {
  dense(x, "x");
  dense(y, "y", torch::kInt64);
  dense(idx, "idx", torch::kInt32);
  dense(stepctl, "stepctl", torch::kInt32);
  dense(ox, "ox");
  dense(oy, "oy", torch::kInt64);
  const int C = idx.size(1), B = idx.size(2), F = x.size(1);
  TORCH_CHECK(ox.numel() == (long)C * B * F && oy.numel() == (long)C * B, "output sizes");
  ok(afl_gather_har(x.data_ptr<float>(), (const long*)y.data_ptr<int64_t>(), F, idx.data_ptr<int>(),
                    stepctl.data_ptr<int>(), C, B, ox.data_ptr<float>(), (long*)oy.data_ptr<int64_t>(), cur()),
     "gather_har");
}

void im2col3(torch::Tensor x, int64_t B, int64_t L, torch::Tensor out) {
  view3(x, "x");
  dense(out, "out");
  TORCH_CHECK(x.stride(2) == 1 && x.size(1) == B * L, "x must be [C, B*L, Cin] with contiguous channels");
  const int C = x.size(0), Cin = x.size(2);
  TORCH_CHECK(out.numel() == (long)C * B * L * 3 * Cin, "out must be [C, B*L, 3*Cin]");
  ok(afl_im2col3(x.data_ptr<float>(), x.stride(0), x.stride(1), C, B, L, Cin, out.data_ptr<float>(), cur()), "im2col3");
}

void col2im3(torch::Tensor dcols, int64_t B, int64_t L, int64_t Cin, c10::optional<torch::Tensor> relu_src,
             torch::Tensor dx) {
  dense(dcols, "dcols");
  dense(dx, "dx");
  const int C = dcols.size(0);
  TORCH_CHECK(dcols.numel() == (long)C * B * L * 3 * Cin && dx.numel() == (long)C * B * L * Cin, "sizes");
  long sRc = 0, sRr = 0;
  if (relu_src.has_value() && relu_src->defined()) {
    view3(*relu_src, "relu_src");
    TORCH_CHECK(relu_src->stride(2) == 1, "relu_src channels must be contiguous");
    sRc = relu_src->stride(0);
    sRr = relu_src->stride(1);
  }
  ok(afl_col2im3(dcols.data_ptr<float>(), C, B, L, Cin, optp(relu_src), sRc, sRr, dx.data_ptr<float>(), cur()),
     "col2im3");
}

void pool4_fwd(torch::Tensor h, int64_t B, int64_t L, torch::Tensor out, int64_t col0,
               c10::optional<torch::Tensor> seeds, c10::optional<torch::Tensor> stepctl, int64_t layer, double p) {
  dense(h, "h");
  view3(out, "out");
  TORCH_CHECK(out.stride(2) == 1, "out columns must be contiguous");
  const int C = h.size(0), Ch = h.size(-1);
  ok(afl_pool4_fwd(h.data_ptr<float>(), C, B, L, Ch, out.data_ptr<float>(), out.stride(0), out.stride(1), col0,
                   make_drop(seeds, stepctl, layer, p), cur()),
     "pool4_fwd");
}

void pool4_bwd(torch::Tensor dout, int64_t col0, torch::Tensor h, int64_t B, int64_t L, torch::Tensor dh,
               c10::optional<torch::Tensor> seeds, c10::optional<torch::Tensor> stepctl, int64_t layer, double p) {
  view3(dout, "dout");
  dense(h, "h");
  dense(dh, "dh");
  TORCH_CHECK(dout.stride(2) == 1, "dout columns must be contiguous");
  const int C = h.size(0), Ch = h.size(-1);
  ok(afl_pool4_bwd(dout.data_ptr<float>(), dout.stride(0), dout.stride(1), col0, h.data_ptr<float>(), C, B, L, Ch,
                   dh.data_ptr<float>(), make_drop(seeds, stepctl, layer, p), cur()),
     "pool4_bwd");
}

// ---- fused CNNModel towers (cnn.hip) ----
// t = [x, W1, b1, W2, b2, W3, b3, h1, h2, h3, dh1, dh2, dh3]; meta = [L, col0, layer]
AflCnnBranch cnn_branch(const std::vector<torch::Tensor>& t, const std::vector<int64_t>& meta, int64_t B,
                        long& sWc, bool bwd) {
  TORCH_CHECK(t.size() == 13 && meta.size() == 3, "cnn tower: 13 tensors and [L, col0, layer] expected");
  AflCnnBranch br{};
  const int L = (int)meta[0];
  TORCH_CHECK(L == 7 || L == 16, "cnn tower: the fused tower kernels are built for L = 7 (vitals) and 16 (labs)");
  const auto& x = t[0];
  dev(x, "x");
  const long C = x.size(0);
  TORCH_CHECK(x.dim() == 3 && x.size(1) == B && x.size(2) == L && x.stride(2) == 1 && x.stride(1) == L,
              "cnn tower: x must be [C, B, L] with contiguous samples");
  br.x = x.data_ptr<float>();
  br.sXc = x.stride(0);
  const int shp[6][2] = {{32, 3}, {32, 1}, {64, 96}, {64, 1}, {128, 192}, {128, 1}};
  const float* wp[6];
  for (int i = 0; i < 6; ++i) {
    const auto& w = t[1 + i];
    dev(w, "cnn weight");
    TORCH_CHECK(w.size(0) == C && w.stride(-1) == 1, "cnn weight: [C, ...] with contiguous rows");
    TORCH_CHECK(w.numel() == C * shp[i][0] * shp[i][1], "cnn weight: unexpected size");
    if (w.dim() == 3) TORCH_CHECK(w.stride(1) == w.size(2), "cnn weight rows must be dense");
    if (i == 0) sWc = C > 1 ? w.stride(0) : 0;
    TORCH_CHECK(C == 1 || w.stride(0) == sWc, "cnn weights must share the client stride (views of one arena)");
    wp[i] = w.data_ptr<float>();
  }
  br.W1 = wp[0]; br.b1 = wp[1]; br.W2 = wp[2]; br.b2 = wp[3]; br.W3 = wp[4]; br.b3 = wp[5];
  const int chs[3] = {32, 64, 128};
  float* hp[3];
  float* dp[3];
  for (int i = 0; i < 3; ++i) {
    dense(t[7 + i], "h");
    TORCH_CHECK(t[7 + i].numel() == C * B * L * chs[i], "cnn tower: h buffer size");
    hp[i] = t[7 + i].data_ptr<float>();
    dp[i] = nullptr;
    if (bwd) {
      dense(t[10 + i], "dh");
      TORCH_CHECK(t[10 + i].numel() == C * B * L * chs[i], "cnn tower: dh buffer size");
      dp[i] = t[10 + i].data_ptr<float>();
    }
  }
  br.h1 = hp[0]; br.h2 = hp[1]; br.h3 = hp[2];
  br.dh1 = dp[0]; br.dh2 = dp[1]; br.dh3 = dp[2];
  br.L = L;
  br.R = 64 / L;
  br.ntiles = (int)((B + br.R - 1) / br.R);
  br.col0 = (int)meta[1];
  br.layer = (uint32_t)meta[2];
  TORCH_CHECK(br.col0 >= 0 && br.col0 + 512 <= 1024, "cnn tower: concat slice out of range");
  return br;
}

AflCnnTowers cnn_towers(const std::vector<torch::Tensor>& t0, const std::vector<torch::Tensor>& t1,
                        const std::vector<int64_t>& m0, const std::vector<int64_t>& m1, int64_t B, torch::Tensor cat,
                        const c10::optional<torch::Tensor>& seeds, const c10::optional<torch::Tensor>& stepctl,
                        double p, bool bwd, torch::Tensor wimg) {
  AflCnnTowers a{};
  long s0 = 0, s1 = 0;
  a.br[0] = cnn_branch(t0, m0, B, s0, bwd);
  a.br[1] = cnn_branch(t1, m1, B, s1, bwd);
  TORCH_CHECK(s0 == s1, "both towers' weights must be views of one arena");
  a.sWc = s0;
  view3(cat, "cat");
  TORCH_CHECK(cat.size(1) == B && cat.size(2) == 1024 && cat.stride(2) == 1, "cat must be [C, B, 1024]");
  a.C = (int)t0[0].size(0);
  TORCH_CHECK(cat.size(0) == a.C && t1[0].size(0) == a.C, "client count mismatch");
  a.B = (int)B;
  a.cat = cat.data_ptr<float>();
  a.dcat = a.cat;
  a.sCatc = cat.stride(0);
  a.sCatr = cat.stride(1);
  a.drop = make_drop(seeds, stepctl, 0, p);
  dense(wimg, "wimg", torch::kInt16);
  TORCH_CHECK(wimg.numel() >= afl_cnn_wimg_ushorts(a.C), "cnn towers: weight-image buffer too small");
  a.wimg = (unsigned short*)wimg.data_ptr<int16_t>();
  return a;
}

void cnn_towers_fwd(std::vector<torch::Tensor> t0, std::vector<torch::Tensor> t1, std::vector<int64_t> m0,
                    std::vector<int64_t> m1, int64_t B, torch::Tensor cat, c10::optional<torch::Tensor> seeds,
                    c10::optional<torch::Tensor> stepctl, double p, torch::Tensor wimg, std::vector<torch::Tensor> head) {
  AflCnnTowers a = cnn_towers(t0, t1, m0, m1, B, cat, seeds, stepctl, p, false, wimg);
  a.W2h = a.W3h = nullptr;
  if (!head.empty()) {  // fc2 / fc3 weight views: their bf16 images feed k_cnn_head
    TORCH_CHECK(head.size() == 2, "cnn towers: head = [fc2.weight, fc3.weight]");
    const long hn[2] = {64 * 128, 32 * 64};
    for (int i = 0; i < 2; ++i) {
      dev(head[i], "head weight");
      TORCH_CHECK(head[i].dim() == 3 && head[i].size(0) == a.C && head[i].numel() == a.C * hn[i] &&
                      head[i].stride(2) == 1 && head[i].stride(1) == head[i].size(2) &&
                      (a.C == 1 || head[i].stride(0) == a.sWc),
                  "cnn towers: head weights must be [C, out, in] views of the same arena");
    }
    a.W2h = head[0].data_ptr<float>();
    a.W3h = head[1].data_ptr<float>();
  }
  ok(afl_cnn_towers_fwd(a, cur()), "cnn_towers_fwd");
}

void cnn_towers_bwd(std::vector<torch::Tensor> t0, std::vector<torch::Tensor> t1, std::vector<int64_t> m0,
                    std::vector<int64_t> m1, int64_t B, torch::Tensor dcat, c10::optional<torch::Tensor> seeds,
                    c10::optional<torch::Tensor> stepctl, double p, torch::Tensor wimg) {
  const AflCnnTowers a = cnn_towers(t0, t1, m0, m1, B, dcat, seeds, stepctl, p, true, wimg);
  ok(afl_cnn_towers_bwd(a, cur()), "cnn_towers_bwd");
}

// conv weight/bias grads: job k = (dh [C, B*L, Cout], hp [C, B*L, Cin], gW [C, Cout, 3*Cin] view, gb [C, Cout] view)
void conv_dw(std::vector<torch::Tensor> dh, std::vector<torch::Tensor> hp, std::vector<torch::Tensor> gW,
             std::vector<torch::Tensor> gb, std::vector<int64_t> L, int64_t B, int64_t splitk) {
  const size_t n = dh.size();
  TORCH_CHECK(n >= 1 && n <= 6 && hp.size() == n && gW.size() == n && gb.size() == n && L.size() == n,
              "conv_dw: 1..6 jobs");
  AflConvDw a{};
  a.njobs = (int)n;
  a.B = (int)B;
  a.splitk = (int)std::max<int64_t>(1, splitk);
  a.C = (int)dh[0].size(0);
  int tiles = 0;
  for (size_t k = 0; k < n; ++k) {
    dense(dh[k], "dh");
    dense(hp[k], "hp");
    view3(gW[k], "gW");
    dev(gb[k], "gb");
    const int Cout = (int)gW[k].size(1), K = (int)gW[k].size(2);
    TORCH_CHECK(K % 3 == 0, "conv_dw: gW must be [C, Cout, 3*Cin]");
    const int Cin = K / 3;
    TORCH_CHECK(gW[k].stride(2) == 1 && gW[k].stride(1) == K, "conv_dw: gW rows dense");
    TORCH_CHECK(dh[k].numel() == (long)a.C * B * L[k] * Cout && hp[k].numel() == (long)a.C * B * L[k] * Cin,
                "conv_dw: activation sizes");
    TORCH_CHECK(gb[k].size(0) == a.C && gb[k].size(-1) == Cout && gb[k].stride(-1) == 1, "conv_dw: gb [C, Cout]");
    if (k == 0) a.sGc = a.C > 1 ? gW[k].stride(0) : 0;
    TORCH_CHECK(a.C == 1 || (gW[k].stride(0) == a.sGc && gb[k].stride(0) == a.sGc),
                "conv_dw: grads must be views of one arena");
    AflConvDwJob& j = a.job[k];
    j.dh = dh[k].data_ptr<float>();
    j.hp = hp[k].data_ptr<float>();
    j.gW = gW[k].data_ptr<float>();
    j.gb = gb[k].data_ptr<float>();
    j.Cin = Cin;
    j.Cout = Cout;
    j.L = (int)L[k];
    j.tile_base = tiles;
    j.ws_off = a.ws_tot;
    a.ws_tot += (long)Cout * K + Cout;
    tiles += ((Cout + 63) / 64) * ((K + 63) / 64);
  }
  a.total_tiles = tiles;
  torch::Tensor ws;  // split-K partials: the weight gradients come out the same whatever order the splits ran in
  if (a.splitk > 1) {
    ws = torch::empty({(long)a.splitk * a.C * a.ws_tot}, dh[0].options());
    a.ws = ws.data_ptr<float>();
  }
  ok(afl_conv_dw(a, cur()), "conv_dw");
}

// CNNModel MLP head fc2 -> fc3 -> output + BCE + backward (cnn.hip:k_cnn_head)
// w = [W2, b2, W3, b3, Wo, bo] parameter views, g = [gW2, gb2, gW3, gb3, gWo, gbo, gb1] gradient views
void cnn_head(torch::Tensor f1, torch::Tensor y, std::vector<torch::Tensor> w, std::vector<torch::Tensor> g,
              torch::Tensor d1, c10::optional<torch::Tensor> z, torch::Tensor bsz, torch::Tensor epoch, torch::Tensor nb,
              torch::Tensor stepctl, torch::Tensor failed, torch::Tensor losses, torch::Tensor wimg) {
  dense(f1, "f1");
  dense(y, "y");
  dense(d1, "d1");
  TORCH_CHECK(w.size() == 7 && g.size() == 7, "cnn_head: 7 parameters and 7 gradients");
  const int C = f1.size(0), B = f1.size(1);
  TORCH_CHECK(f1.dim() == 3 && f1.size(2) == 128 && B <= 128, "cnn_head: f1 must be [C, B<=128, 128]");
  TORCH_CHECK(y.numel() == (long)C * B && d1.numel() == (long)C * B * 128, "cnn_head: y / d1 sizes");
  const long wn[7] = {64 * 128, 64, 32 * 64, 32, 32, 1, 128};
  const long gn[7] = {64 * 128, 64, 32 * 64, 32, 32, 1, 128};
  AflCnnHead h{};
  const float* wp[7];
  float* gp[7];
  for (int i = 0; i < 7; ++i) {
    dev(w[i], "head weight");
    TORCH_CHECK(w[i].size(0) == C && w[i].numel() == C * wn[i] && w[i].stride(-1) == 1, "cnn_head: weight view");
    if (i == 0) h.sWc = C > 1 ? w[i].stride(0) : 0;
    TORCH_CHECK(C == 1 || w[i].stride(0) == h.sWc, "cnn_head: weights must be views of one arena");
    wp[i] = w[i].data_ptr<float>();
  }
  for (int i = 0; i < 7; ++i) {
    dev(g[i], "head grad");
    TORCH_CHECK(g[i].size(0) == C && g[i].numel() == C * gn[i] && g[i].stride(-1) == 1, "cnn_head: grad view");
    if (i == 0) h.sGc = C > 1 ? g[i].stride(0) : 0;
    TORCH_CHECK(C == 1 || g[i].stride(0) == h.sGc, "cnn_head: grads must be views of one arena");
    gp[i] = g[i].data_ptr<float>();
  }
  for (int i : {0, 2}) TORCH_CHECK(w[i].dim() == 3 && w[i].stride(1) == w[i].size(2), "cnn_head: dense weight rows");
  h.f1 = f1.data_ptr<float>();  // read, then zeroed by the kernel
  h.y = y.data_ptr<float>();
  h.W2 = wp[0]; h.b2 = wp[1]; h.W3 = wp[2]; h.b3 = wp[3]; h.Wo = wp[4]; h.bo = wp[5]; h.b1 = wp[6];
  dense(wimg, "wimg", torch::kInt16);
  TORCH_CHECK(wimg.numel() >= afl_cnn_wimg_ushorts(C), "cnn_head: weight-image buffer too small");
  h.wimg = (const unsigned short*)wimg.data_ptr<int16_t>() + (afl_cnn_wimg_ushorts(C) - (long)C * (64 * 128 + 32 * 64));
  h.gW2 = gp[0]; h.gb2 = gp[1]; h.gW3 = gp[2]; h.gb3 = gp[3]; h.gWo = gp[4]; h.gbo = gp[5]; h.gb1 = gp[6];
  h.d1 = d1.data_ptr<float>();
  h.z = nullptr;
  if (z.has_value() && z->defined()) {
    dense(*z, "z");
    TORCH_CHECK(z->numel() == (long)C * B, "cnn_head: z size");
    h.z = z->data_ptr<float>();
  }
  dense(bsz, "bsz", torch::kInt32);
  dense(epoch, "epoch", torch::kInt32);
  dense(nb, "nb", torch::kInt32);
  dense(stepctl, "stepctl", torch::kInt32);
  dense(failed, "failed", torch::kInt32);
  dense(losses, "losses");
  TORCH_CHECK(bsz.dim() == 2 && bsz.size(1) == C, "cnn_head: bsz [S, C]");
  h.bsz = bsz.data_ptr<int>();
  h.epoch = epoch.data_ptr<int>();
  h.nb = nb.data_ptr<int>();
  h.stepctl = stepctl.data_ptr<int>();
  h.failed = failed.data_ptr<int>();
  h.losses = losses.data_ptr<float>();
  h.S = bsz.size(0);
  h.E = losses.size(1);
  h.C = C;
  h.B = B;
  ok(afl_cnn_head(h, cur()), "cnn_head");
}

void ln_fwd(torch::Tensor x, c10::optional<torch::Tensor> a, c10::optional<torch::Tensor> s, torch::Tensor y,
            torch::Tensor stats, torch::Tensor gamma, torch::Tensor beta, c10::optional<torch::Tensor> seeds,
            c10::optional<torch::Tensor> stepctl, int64_t layer_a, double p_a, int64_t layer_o, double p_o) {
  view3(x, "x");
  view3(y, "y");
  dense(stats, "stats");
  dev(gamma, "gamma");
  dev(beta, "beta");
  TORCH_CHECK(x.size(2) == 64 && x.stride(2) == 1 && y.stride(2) == 1, "LayerNorm rows of 64 contiguous columns");
  TORCH_CHECK(gamma.dim() == 2 && gamma.stride(1) == 1 && beta.stride(0) == gamma.stride(0), "gamma/beta [C, 64]");
  AflLn l{};
  l.x = x.data_ptr<float>(); l.sXc = x.stride(0); l.sXr = x.stride(1);
  if (a.has_value() && a->defined()) {
    view3(*a, "a");
    TORCH_CHECK(a->stride(2) == 1, "a columns must be contiguous");
    l.a = a->data_ptr<float>(); l.sAc = a->stride(0); l.sAr = a->stride(1);
  }
  if (s.has_value() && s->defined()) {
    dense(*s, "s");
    TORCH_CHECK(s->numel() == x.size(0) * x.size(1) * 64, "s must be [C, rows, 64]");
    l.s = s->data_ptr<float>();
  }
  l.y = y.data_ptr<float>(); l.sYc = y.stride(0); l.sYr = y.stride(1);
  l.stats = stats.data_ptr<float>();
  l.gamma = gamma.data_ptr<float>(); l.beta = beta.data_ptr<float>(); l.sPc = gamma.stride(0);
  l.rows = x.size(1); l.nC = x.size(0);
  l.da = make_drop(seeds, stepctl, layer_a, p_a);
  l.dout = make_drop(seeds, stepctl, layer_o, p_o);
  ok(afl_ln_fwd(l, cur()), "ln_fwd");
}

void ln_bwd(torch::Tensor dy, torch::Tensor s, torch::Tensor stats, torch::Tensor gamma, torch::Tensor dx,
            int64_t dx_accum, c10::optional<torch::Tensor> da, torch::Tensor dgamma, torch::Tensor dbeta,
            c10::optional<torch::Tensor> seeds, c10::optional<torch::Tensor> stepctl, int64_t layer_a, double p_a,
            int64_t layer_o, double p_o) {
  view3(dy, "dy");
  view3(s, "s");
  view3(dx, "dx");
  dense(stats, "stats");
  TORCH_CHECK(dy.stride(2) == 1 && s.stride(2) == 1 && dx.stride(2) == 1, "contiguous columns");
  TORCH_CHECK(dgamma.stride(0) == gamma.stride(0) && dbeta.stride(0) == gamma.stride(0), "param/grad strides");
  AflLnB l{};
  l.dy = dy.data_ptr<float>(); l.sDc = dy.stride(0); l.sDr = dy.stride(1);
  l.s = s.data_ptr<float>(); l.sSc = s.stride(0); l.sSr = s.stride(1);
  l.stats = stats.data_ptr<float>();
  l.gamma = gamma.data_ptr<float>(); l.sPc = gamma.stride(0);
  l.dx = dx.data_ptr<float>(); l.sXc = dx.stride(0); l.sXr = dx.stride(1); l.dx_accum = (int)dx_accum;
  if (da.has_value() && da->defined()) {
    view3(*da, "da");
    l.da = da->data_ptr<float>(); l.sAc = da->stride(0); l.sAr = da->stride(1);
  }
  l.dgamma = dgamma.data_ptr<float>(); l.dbeta = dbeta.data_ptr<float>();
  l.rows = dy.size(1); l.nC = dy.size(0);
  l.da_drop = make_drop(seeds, stepctl, layer_a, p_a);
  l.dout = make_drop(seeds, stepctl, layer_o, p_o);
  auto ws = torch::empty({afl_ln_bwd_ws_floats(l.rows, l.nC)}, dy.options());  // gamma / beta: ordered partials
  l.ws = ws.data_ptr<float>();
  ok(afl_ln_bwd(l, cur()), "ln_bwd");
}

void gru_fwd(torch::Tensor gi, torch::Tensor bhh, torch::Tensor h, int64_t col0) {
  dense(gi, "gi");
  dev(bhh, "bhh");
  view3(h, "h");
  const int C = gi.size(0), B = gi.size(1);
  TORCH_CHECK(gi.size(2) == 96 && bhh.stride(1) == 1 && h.stride(2) == 1, "gru shapes");
  ok(afl_gru_fwd(gi.data_ptr<float>(), bhh.data_ptr<float>(), bhh.stride(0), C, B, h.data_ptr<float>(), h.stride(0),
                 h.stride(1), col0, cur()),
     "gru_fwd");
}

void gru_bwd(torch::Tensor dh, int64_t col0, torch::Tensor gi, torch::Tensor bhh, torch::Tensor dgi,
             torch::Tensor dbih, torch::Tensor dbhh) {
  view3(dh, "dh");
  dense(gi, "gi");
  dense(dgi, "dgi");
  TORCH_CHECK(dbih.stride(0) == bhh.stride(0) && dbhh.stride(0) == bhh.stride(0), "grad strides");
  const int C = gi.size(0), B = gi.size(1);
  ok(afl_gru_bwd(dh.data_ptr<float>(), dh.stride(0), dh.stride(1), col0, gi.data_ptr<float>(), bhh.data_ptr<float>(),
                 bhh.stride(0), C, B, dgi.data_ptr<float>(), dbih.data_ptr<float>(), dbhh.data_ptr<float>(), cur()),
     "gru_bwd");
}

void bce(torch::Tensor z, torch::Tensor y, torch::Tensor bsz, torch::Tensor epoch, torch::Tensor nb,
         torch::Tensor stepctl, torch::Tensor failed, torch::Tensor losses, torch::Tensor dz) {
  dense(z, "z");
  dense(y, "y");
  dense(bsz, "bsz", torch::kInt32);
  dense(epoch, "epoch", torch::kInt32);
  dense(nb, "nb", torch::kInt32);
  dense(stepctl, "stepctl", torch::kInt32);
  dense(failed, "failed", torch::kInt32);
  dense(losses, "losses");
  dense(dz, "dz");
  const int S = bsz.size(0), C = bsz.size(1), B = z.numel() / C;
  ok(afl_bce(z.data_ptr<float>(), y.data_ptr<float>(), bsz.data_ptr<int>(), epoch.data_ptr<int>(), nb.data_ptr<int>(),
             stepctl.data_ptr<int>(), C, B, S, failed.data_ptr<int>(), losses.data_ptr<float>(), losses.size(1),
             dz.data_ptr<float>(), cur()),
     "bce");
}

void ce(torch::Tensor logits, torch::Tensor y, torch::Tensor bsz, torch::Tensor epoch, torch::Tensor nb,
        torch::Tensor stepctl, torch::Tensor failed, torch::Tensor losses, torch::Tensor dz) {
  dense(logits, "logits");
  dense(y, "y", torch::kInt64);
  dense(bsz, "bsz", torch::kInt32);
  dense(epoch, "epoch", torch::kInt32);
  dense(nb, "nb", torch::kInt32);
  dense(stepctl, "stepctl", torch::kInt32);
  dense(failed, "failed", torch::kInt32);
  dense(losses, "losses");
  dense(dz, "dz");
  const int S = bsz.size(0), C = bsz.size(1), K = logits.size(-1), B = logits.numel() / ((long)C * K);
  ok(afl_ce(logits.data_ptr<float>(), (const long*)y.data_ptr<int64_t>(), K, bsz.data_ptr<int>(), epoch.data_ptr<int>(),
            nb.data_ptr<int>(), stepctl.data_ptr<int>(), C, B, S, failed.data_ptr<int>(), losses.data_ptr<float>(),
            losses.size(1), dz.data_ptr<float>(), cur()),
     "ce");
}

void adam_clients(torch::Tensor p, torch::Tensor g, torch::Tensor m, torch::Tensor v, torch::Tensor tcount,
                  torch::Tensor bsz, torch::Tensor stepctl, torch::Tensor failed, double lr, int64_t skip_lo,
                  int64_t skip_hi, double sgd_lr, int64_t zero_grads) {
  dense(p, "p");
  dense(g, "g");
  dense(m, "m");
  dense(v, "v");
  dense(tcount, "tcount", torch::kInt32);
  dense(bsz, "bsz", torch::kInt32);
  const int C = p.size(0), S = bsz.size(0);
  ok(afl_adam_clients(p.data_ptr<float>(), g.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(), p.size(1), C,
                      tcount.data_ptr<int>(), bsz.data_ptr<int>(), stepctl.data_ptr<int>(), S,
                      failed.data_ptr<int>(), (float)lr, skip_lo, skip_hi, (float)sgd_lr, (int)zero_grads, cur()),
     "adam_clients");
}

void step_end(torch::Tensor stepctl, torch::Tensor tcount, torch::Tensor bsz, torch::Tensor failed) {
  dense(stepctl, "stepctl", torch::kInt32);
  dense(tcount, "tcount", torch::kInt32);
  ok(afl_step_end(stepctl.data_ptr<int>(), tcount.data_ptr<int>(), bsz.data_ptr<int>(), failed.data_ptr<int>(),
                  bsz.size(1), bsz.size(0), cur()),
     "step_end");
}

void conv_pe_fwd(torch::Tensor x, torch::Tensor params, int64_t w_off, int64_t b_off, int64_t pe_off, torch::Tensor h) {
  dense(x, "x");
  dense(params, "params");
  dense(h, "h");
  const int C = x.size(0), B = x.size(1), L = x.size(2);
  ok(afl_conv_pe_fwd(x.data_ptr<float>(), C, B, L, params.data_ptr<float>(), params.size(1), w_off, b_off, pe_off,
                     h.data_ptr<float>(), cur()),
     "conv_pe_fwd");
}

void conv_pe_bwd(torch::Tensor x, torch::Tensor dh, torch::Tensor grads, int64_t w_off, int64_t b_off) {
  dense(x, "x");
  dense(dh, "dh");
  dense(grads, "grads");
  const int C = x.size(0), B = x.size(1), L = x.size(2);
  auto ws = torch::empty({afl_conv_pe_bwd_ws_floats(C, B, L)}, x.options());  // ordered partials
  ok(afl_conv_pe_bwd(x.data_ptr<float>(), dh.data_ptr<float>(), C, B, L, grads.data_ptr<float>(), grads.size(1), w_off,
                     b_off, cur(), ws.data_ptr<float>()),
     "conv_pe_bwd");
}

void mean_rows_fwd(torch::Tensor h, int64_t B, int64_t L, torch::Tensor out) {
  dense(h, "h");
  dense(out, "out");
  ok(afl_mean_rows_fwd(h.data_ptr<float>(), h.size(0), B, L, out.data_ptr<float>(), cur()), "mean_rows_fwd");
}

void mean_rows_bwd(torch::Tensor dout, int64_t B, int64_t L, torch::Tensor dh) {
  dense(dout, "dout");
  dense(dh, "dh");
  ok(afl_mean_rows_bwd(dout.data_ptr<float>(), dout.size(0), B, L, dh.data_ptr<float>(), cur()), "mean_rows_bwd");
}

AflAttn attn_args(torch::Tensor qkv, torch::Tensor o, torch::Tensor lse, int64_t B, int64_t L,
                  c10::optional<torch::Tensor> seeds, c10::optional<torch::Tensor> stepctl, int64_t layer, double p) {
  dense(qkv, "qkv");
  dense(o, "o");
  dense(lse, "lse");
  AflAttn a{};
  a.C = qkv.size(0);
  a.B = B;
  a.L = L;
  a.Lp = afl_attn_lp(L);
  TORCH_CHECK(qkv.numel() == (long)a.C * B * L * 192 && o.numel() == (long)a.C * B * L * 64, "qkv/o sizes");
  TORCH_CHECK(lse.numel() == (long)a.C * B * 4 * a.Lp, "lse must hold C*B*4*Lp floats");
  a.qkv = qkv.data_ptr<float>();
  a.o = o.data_ptr<float>();
  a.lse = lse.data_ptr<float>();
  a.scale = 0.25f;  // 1 / sqrt(head_dim 16)
  a.drop = make_drop(seeds, stepctl, layer, p);
  return a;
}

void attn_fwd(torch::Tensor qkv, torch::Tensor o, torch::Tensor lse, int64_t B, int64_t L,
              c10::optional<torch::Tensor> seeds, c10::optional<torch::Tensor> stepctl, int64_t layer, double p) {
  AflAttn a = attn_args(qkv, o, lse, B, L, seeds, stepctl, layer, p);
  ok(afl_attn_fwd(a, cur()), "attn_fwd");
}

void attn_bwd(torch::Tensor qkv, torch::Tensor o, torch::Tensor lse, torch::Tensor dout, torch::Tensor dqkv, int64_t B,
              int64_t L, c10::optional<torch::Tensor> seeds, c10::optional<torch::Tensor> stepctl, int64_t layer,
              double p) {
  AflAttn a = attn_args(qkv, o, lse, B, L, seeds, stepctl, layer, p);
  dense(dout, "dout");
  dense(dqkv, "dqkv");
  a.dout = dout.data_ptr<float>();
  a.dqkv = dqkv.data_ptr<float>();
  ok(afl_attn_bwd(a, cur()), "attn_bwd");
}

// CNNModel on-chip trainer (cnn2.hip): one launch trains every client of params [C, P] for the whole round
// over the step tables of fl/programs.py:step_tables; ws / ctr from cnn2_ws_bytes / cnn2_ctr_words (ctr zeroed)
void cnn2_train(torch::Tensor params, std::vector<int64_t> offs, torch::Tensor rows, torch::Tensor idx, torch::Tensor bsz,
                torch::Tensor epoch, torch::Tensor nb, torch::Tensor seeds, double p, int64_t min_bs, bool nan_abort,
                double lr, torch::Tensor failed, torch::Tensor losses, torch::Tensor ws, torch::Tensor ctr,
                c10::optional<torch::Tensor> stamps, int64_t opt_mode) {
  dense(params, "params");
  dense(rows, "rows");
  dense(idx, "idx", torch::kInt32);
  dense(bsz, "bsz", torch::kInt32);
  dense(epoch, "epoch", torch::kInt32);
  dense(nb, "nb", torch::kInt32);
  dense(seeds, "seeds", torch::kInt32);
  dense(failed, "failed", torch::kInt32);
  dense(losses, "losses");
  dense(ws, "ws", torch::kUInt8);
  dense(ctr, "ctr", torch::kInt32);
  TORCH_CHECK(offs.size() == 20, "cnn2_train: 20 CNNModel slot offsets");
  TORCH_CHECK(params.dim() == 2 && rows.dim() == 2 && rows.size(1) == 24, "cnn2_train: params [C, P], rows [N, 24]");
  const int C = (int)params.size(0);
  TORCH_CHECK(idx.dim() == 3 && idx.size(1) == C && bsz.dim() == 2 && bsz.size(1) == C && epoch.sizes() == bsz.sizes(),
              "cnn2_train: step tables [S, C, B] / [S, C]");
  const int S = (int)idx.size(0), B = (int)idx.size(2);
  TORCH_CHECK(bsz.size(0) == S && nb.numel() == C && seeds.numel() == C && failed.numel() == C && losses.dim() == 2 &&
                  losses.size(0) == C, "cnn2_train: per-client sizes");
  TORCH_CHECK(ws.numel() >= (int64_t)C * afl_cnn2_ws_bytes() && ctr.numel() >= (int64_t)C * afl_cnn2_ctr_words(),
              "cnn2_train: workspace too small");
  AflCnn2Args a{};
  a.params = params.data_ptr<float>();
  a.pstride = params.size(1);
  for (int k = 0; k < 20; ++k) {
    TORCH_CHECK(offs[k] >= 0 && offs[k] < a.pstride, "cnn2_train: slot offset out of range");
    a.off[k] = (int)offs[k];
  }
  a.rows = rows.data_ptr<float>();
  a.idx = idx.data_ptr<int>();
  a.bsz = bsz.data_ptr<int>();
  a.epoch = epoch.data_ptr<int>();
  a.nb = nb.data_ptr<int>();
  a.seeds = (const uint32_t*)seeds.data_ptr<int>();
  a.S = S;
  a.C = C;
  a.B = B;
  a.E = (int)losses.size(1);
  a.thr16 = p > 0.0 ? (uint32_t)std::lround(p * 65536.0) : 0u;
  a.inv_keep = p > 0.0 ? (float)(1.0 / (1.0 - p)) : 1.f;
  a.min_bs = (int)min_bs;
  a.nan_abort = nan_abort ? 1 : 0;
  a.lr = (float)lr;
  TORCH_CHECK(opt_mode == 0 || opt_mode == 1, "cnn2_train: opt_mode 0 (Adam) or 1 (SGD)");
  a.opt_mode = (int)opt_mode;
  a.failed = failed.data_ptr<int>();
  a.losses = losses.data_ptr<float>();
  a.ws = ws.data_ptr();
  a.ws_stride = afl_cnn2_ws_bytes();
  a.ctr = (uint32_t*)ctr.data_ptr<int>();
  if (stamps.has_value() && stamps->defined()) {
    dense(*stamps, "stamps", torch::kInt64);
    TORCH_CHECK(stamps->numel() >= (int64_t)C * afl_cnn2_wgs_per_client() * 64 * 16, "cnn2_train: stamps too small");
    a.stamps = (uint64_t*)stamps->data_ptr<int64_t>();
  }
  ok(afl_cnn2_train(a, cur()), "cnn2_train");
}

// eval forward of C CNNModels (params [C, P], 20 slot offsets) over rows [n, 24] -> sigmoid outputs [C, n]: ONE launch
torch::Tensor cnn2_eval(torch::Tensor params, std::vector<int64_t> offs, torch::Tensor rows) {
  dense(params, "params");
  dense(rows, "rows");
  TORCH_CHECK(offs.size() == 20, "cnn2_eval: 20 CNNModel slot offsets");
  TORCH_CHECK(params.dim() == 2 && rows.dim() == 2 && rows.size(1) == 24, "cnn2_eval: params [C, P], rows [N, 24]");
  int off[20];
  // every slot's extent (the kernel reads whole weight matrices from each offset)
  static const int64_t numel[20] = {96, 32, 6144, 64, 24576, 128, 96, 32, 6144, 64, 24576, 128,
                                    131072, 128, 8192, 64, 2048, 32, 32, 1};
  for (int k = 0; k < 20; ++k) {
    TORCH_CHECK(offs[k] >= 0 && offs[k] + numel[k] <= params.size(1), "cnn2_eval: slot offset out of range");
    off[k] = (int)offs[k];
  }
  // the kernel reads these slots (conv biases, fc weights) as 16-byte vectors: 4-float aligned offsets, and a row
  // stride and base that keep them aligned for every model (an odd stride such as CNNModel's 203649 is padded)
  for (int k : {3, 5, 9, 11, 12, 14, 16}) TORCH_CHECK(off[k] % 4 == 0, "cnn2_eval: slot offset not 4-float aligned");
  // One model with an aligned base needs no padding (the stride is never used).  Otherwise the rows are copied
  // into a padded buffer cached per (device, stream) across calls (validation, prefetch and hyper evaluations of every
  // client reuse it: no allocation or zero fill on the round boundary; the padding columns are never read).
  torch::Tensor p = params;
  const bool aligned = (reinterpret_cast<uintptr_t>(p.data_ptr<float>()) & 15) == 0;
  if (!(aligned && (p.size(0) == 1 || p.size(1) % 4 == 0))) {
    // keyed by stream: calls on one stream are ordered, so the buffer is free again when the next copy runs
    static std::map<std::pair<int, hipStream_t>, torch::Tensor> cache;
    const int64_t Pp = (p.size(1) + 3) / 4 * 4;
    torch::Tensor& buf = cache[{(int)p.get_device(), cur()}];
    if (!buf.defined() || buf.size(0) < p.size(0) || buf.size(1) != Pp)
      buf = torch::empty({std::max<int64_t>(p.size(0), buf.defined() ? buf.size(0) : 0), Pp}, p.options());
    p = buf.narrow(0, 0, params.size(0));
    p.narrow(1, 0, params.size(1)).copy_(params);
  }
  const int C = (int)p.size(0), n = (int)rows.size(0);
  auto out = torch::empty({C, n}, rows.options());
  ok(afl_cnn2_eval(p.data_ptr<float>(), p.size(1), off, C, rows.data_ptr<float>(), n, out.data_ptr<float>(), cur()),
     "cnn2_eval");
  return out;
}

}  // namespace

void afl_register_layers(pybind11::module& m) {
  namespace py = pybind11;
  const auto none = py::none();
  m.def("bgemm", &bgemm, py::arg("A"), py::arg("B"), py::arg("C"), py::arg("bias") = none, py::arg("Z") = none,
        py::arg("G") = none, py::arg("act") = 0, py::arg("gact") = 0, py::arg("accum") = 0, py::arg("splitk") = 1,
        py::arg("alpha") = 1.0, py::arg("seeds") = none, py::arg("stepctl") = none, py::arg("layer") = 0,
        py::arg("p") = 0.0, py::arg("generic") = 0, py::arg("asum") = none);
  m.def("colsum", &colsum);
  m.def("gather_icu", &gather_icu);
  m.def("gather_har", &gather_har);
  m.def("im2col3", &im2col3);
  m.def("col2im3", &col2im3);
  m.def("pool4_fwd", &pool4_fwd);
  m.def("cnn_towers_fwd", &cnn_towers_fwd);
  m.def("cnn_towers_bwd", &cnn_towers_bwd);
  m.def("conv_dw", &conv_dw);
  m.def("cnn_head", &cnn_head);
  m.def("cnn_wimg_size", &afl_cnn_wimg_ushorts);
  m.def("cnn2_train", &cnn2_train, py::arg("params"), py::arg("offs"), py::arg("rows"), py::arg("idx"), py::arg("bsz"),
        py::arg("epoch"), py::arg("nb"), py::arg("seeds"), py::arg("p"), py::arg("min_bs"), py::arg("nan_abort"),
        py::arg("lr"), py::arg("failed"), py::arg("losses"), py::arg("ws"), py::arg("ctr"), py::arg("stamps") = none,
        py::arg("opt_mode") = 0);
  m.def("cnn2_eval", &cnn2_eval, py::arg("params"), py::arg("offs"), py::arg("rows"));
  m.def("cnn2_ws_bytes", &afl_cnn2_ws_bytes);
  m.def("cnn2_ctr_words", &afl_cnn2_ctr_words);
  m.def("cnn2_wgs_per_client", &afl_cnn2_wgs_per_client);
  m.def("pool4_bwd", &pool4_bwd);
  m.def("ln_fwd", &ln_fwd);
  m.def("ln_bwd", &ln_bwd);
  m.def("gru_fwd", &gru_fwd);
  m.def("gru_bwd", &gru_bwd);
  m.def("bce", &bce);
  m.def("ce", &ce);
  m.def("adam_clients", &adam_clients);
  m.def("step_end", &step_end);
  m.def("conv_pe_fwd", &conv_pe_fwd);
  m.def("conv_pe_bwd", &conv_pe_bwd);
  m.def("mean_rows_fwd", &mean_rows_fwd);
  m.def("mean_rows_bwd", &mean_rows_bwd);
  m.def("attn_fwd", &attn_fwd);
  m.def("attn_bwd", &attn_bwd);
  m.def("attn_lp", &afl_attn_lp);
}
