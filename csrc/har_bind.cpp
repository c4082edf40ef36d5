#include <cstdlib>
// torch bindings of the bf16 HAR encoder kernels (kernels/har.hip).  Every op writes into caller-provided
// tensors: bf16 activations are torch.bfloat16 tensors, gradients / statistics fp32.  The HAR layer
// program (attackfl_amd/fl/programs.py HARProgram, device path) preallocates them once and captures the
// step in a HIP graph.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>

#include <cmath>
#include <vector>

#include "kernels.h"

namespace {

hipStream_t cur() { return at::hip::getCurrentHIPStream().stream(); }

void ok(int e, const char* what) { TORCH_CHECK(e == 0, what, " launch failed: ", hipGetErrorString((hipError_t)e)); }

void dense(const torch::Tensor& t, const char* n, c10::ScalarType dt) {
  TORCH_CHECK(t.defined() && t.is_cuda(), n, " must be a device tensor");
  TORCH_CHECK(t.scalar_type() == dt, n, " has dtype ", t.scalar_type(), ", expected ", dt);
  TORCH_CHECK(t.is_contiguous(), n, " must be contiguous");
}
unsigned short* bf(const torch::Tensor& t, const char* n) {
  dense(t, n, torch::kBFloat16);
  return (unsigned short*)t.data_ptr();
}
float* f32(const torch::Tensor& t, const char* n) {
  dense(t, n, torch::kFloat32);
  return t.data_ptr<float>();
}

AflDrop drop(const c10::optional<torch::Tensor>& seeds, const c10::optional<torch::Tensor>& stepctl, int64_t layer,
             double p) {
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

AflHarLayerW layer_w(const std::vector<int64_t>& w) {
  TORCH_CHECK(w.size() == 12, "layer offsets: 12 entries");
  return AflHarLayerW{(int)w[0], (int)w[1], (int)w[2], (int)w[3], (int)w[4],  (int)w[5],
                      (int)w[6], (int)w[7], (int)w[8], (int)w[9], (int)w[10], (int)w[11]};
}

// rows of a [C, R, 64] activation
void rows64(const torch::Tensor& t, int64_t C, int64_t R, const char* n) {
  TORCH_CHECK(t.dim() == 3 && t.size(0) == C && t.size(1) == R && t.size(2) == 64, n, " must be [C, B*L, 64]");
}
void headmajor(const torch::Tensor& t, int64_t C, int64_t B, int64_t Lp, const char* n) {
  TORCH_CHECK(t.dim() == 4 && t.size(0) == C * B * 4 && t.size(1) == 3 && t.size(2) == Lp && t.size(3) == 16, n,
              " must be [C*B*4, 3, Lp, 16]");
}

void har_stem(torch::Tensor x, torch::Tensor params, int64_t w_off, int64_t b_off, int64_t pe_off, torch::Tensor h) {
  const float* xp = f32(x, "x");
  TORCH_CHECK(x.dim() == 3, "x must be [C, B, L]");
  const int64_t C = x.size(0), B = x.size(1), L = x.size(2);
  rows64(h, C, B * L, "h");
  ok(afl_har_stem(xp, (int)C, (int)B, (int)L, f32(params, "params"), params.size(1), (int)w_off, (int)b_off, (int)pe_off,
                  bf(h, "h"), cur()),
     "har_stem");
}

void har_pool(torch::Tensor y, int64_t B, int64_t L, torch::Tensor out) {
  const int64_t C = out.size(0);
  rows64(y, C, B * L, "y");
  TORCH_CHECK(out.dim() == 3 && out.size(1) == B && out.size(2) == 64, "out must be [C, B, 64]");
  ok(afl_har_pool(bf(y, "y"), (int)C, (int)B, (int)L, f32(out, "out"), cur()), "har_pool");
}

void har_qkv(torch::Tensor x, torch::Tensor params, int64_t w_off, int64_t b_off, torch::Tensor qkv, int64_t B,
             int64_t L, double qscale) {
  const int64_t C = params.size(0), Lp = qkv.size(2);
  rows64(x, C, B * L, "x");
  headmajor(qkv, C, B, Lp, "qkv");
  AflHarQkv a{bf(x, "x"), f32(params, "params"), params.size(1), (int)w_off, (int)b_off, bf(qkv, "qkv"),
              (int)C, (int)B, (int)L, (int)Lp, (float)qscale};
  ok(afl_har_qkv(a, cur()), "har_qkv");
}

// row-pass keep bits (written by har_post, read by har_post_bwd): int32 [C, R, AFL_HAR_KBITS_PER_ROW], dropout only
unsigned* kbits_of(const c10::optional<torch::Tensor>& kb, int64_t C, int64_t R, bool drop) {
  if (!drop) return nullptr;
  TORCH_CHECK(kb.has_value() && kb->defined(), "row-pass dropout needs the keep-bit buffer");
  TORCH_CHECK(kb->is_cuda() && kb->scalar_type() == torch::kInt32 && kb->is_contiguous(), "kbits: int32 cuda");
  TORCH_CHECK(kb->numel() == C * R * AFL_HAR_KBITS_PER_ROW, "kbits must be [C, R, ", AFL_HAR_KBITS_PER_ROW, "]");
  return (unsigned*)kb->data_ptr<int32_t>();
}

void har_post(torch::Tensor o, torch::Tensor x, torch::Tensor xh1, torch::Tensor xh2, torch::Tensor rs, torch::Tensor y,
              torch::Tensor params, std::vector<int64_t> w, c10::optional<torch::Tensor> seeds,
              c10::optional<torch::Tensor> stepctl, int64_t layer, double p, c10::optional<torch::Tensor> kbits) {
  const int64_t C = params.size(0), R = o.size(1);
  for (auto* t : {&o, &x, &xh1, &xh2, &y}) rows64(*t, C, R, "activation");
  TORCH_CHECK(rs.numel() == C * R * 2, "rs must be [C, R, 2]");
  AflHarPost a{};
  a.o = bf(o, "o");
  a.x = bf(x, "x");
  a.xh1 = bf(xh1, "xh1");
  a.xh2 = bf(xh2, "xh2");
  a.rs = f32(rs, "rs");
  a.y = bf(y, "y");
  a.params = f32(params, "params");
  a.P = params.size(1);
  a.w = layer_w(w);
  a.C = (int)C;
  a.R = R;
  a.d1 = drop(seeds, stepctl, layer + 1, p);
  a.df = drop(seeds, stepctl, layer + 2, p);
  a.d2 = drop(seeds, stepctl, layer + 3, p);
  a.kbits = kbits_of(kbits, C, R, a.d1.thr16 || a.df.thr16 || a.d2.thr16);
  ok(afl_har_post(a, cur()), "har_post");
}

AflHarAttn attn_args(torch::Tensor qkv, torch::Tensor lse2, int64_t B, int64_t L, c10::optional<torch::Tensor> seeds,
                     c10::optional<torch::Tensor> stepctl, int64_t layer, double p) {
  const int64_t Lp = qkv.size(2), C = qkv.size(0) / (4 * B);
  headmajor(qkv, C, B, Lp, "qkv");
  TORCH_CHECK(lse2.numel() == C * B * 4 * Lp, "lse2 must be [C*B*4, Lp]");
  AflHarAttn a{};
  a.qkv = bf(qkv, "qkv");
  a.lse2 = f32(lse2, "lse2");
  a.C = (int)C;
  a.B = (int)B;
  a.L = (int)L;
  a.Lp = (int)Lp;
  a.drop = drop(seeds, stepctl, layer, p);
  return a;
}

// dropout keep words (written by the forward, read by the backward): int64 [C*B*4, AFL_HAR_MASK_WORDS(Lp)]
void attn_mask(AflHarAttn& a, const c10::optional<torch::Tensor>& mask) {
  if (!a.drop.thr16) return;
  TORCH_CHECK(mask.has_value() && mask->defined(), "attention dropout needs the keep-word buffer");
  TORCH_CHECK(mask->is_cuda() && mask->scalar_type() == torch::kInt64 && mask->is_contiguous(), "mask: int64 cuda");
  TORCH_CHECK(mask->numel() == (int64_t)a.C * a.B * 4 * AFL_HAR_MASK_WORDS(a.Lp), "mask must be [C*B*4, ",
              AFL_HAR_MASK_WORDS(a.Lp), "]");
  a.mask = (unsigned long long*)mask->data_ptr<int64_t>();
}

void har_attn_fwd(torch::Tensor qkv, torch::Tensor o, torch::Tensor lse2, int64_t B, int64_t L,
                  c10::optional<torch::Tensor> seeds, c10::optional<torch::Tensor> stepctl, int64_t layer, double p,
                  c10::optional<torch::Tensor> mask) {
  AflHarAttn a = attn_args(qkv, lse2, B, L, seeds, stepctl, layer, p);
  attn_mask(a, mask);
  rows64(o, a.C, B * L, "o");
  a.o = bf(o, "o");
  ok(afl_har_attn_fwd(a, cur()), "har_attn_fwd");
}

void har_attn_bwd(torch::Tensor qkv, torch::Tensor lse2, torch::Tensor dout, torch::Tensor delta, torch::Tensor dqkv,
                  int64_t B, int64_t L, c10::optional<torch::Tensor> seeds, c10::optional<torch::Tensor> stepctl,
                  int64_t layer, double p, c10::optional<torch::Tensor> mask) {
  AflHarAttn a = attn_args(qkv, lse2, B, L, seeds, stepctl, layer, p);
  attn_mask(a, mask);
  rows64(dout, a.C, B * L, "dout");
  headmajor(dqkv, a.C, B, a.Lp, "dqkv");
  TORCH_CHECK(delta.numel() == (int64_t)a.C * B * 4 * a.Lp, "delta must be [C*B*4, Lp]");
  a.dout = bf(dout, "dout");
  a.delta = f32(delta, "delta");
  a.dqkv = bf(dqkv, "dqkv");
  ok(afl_har_attn_bwd(a, cur()), "har_attn_bwd");
}

void har_post_bwd(c10::optional<torch::Tensor> dy, c10::optional<torch::Tensor> dpool, int64_t B, int64_t L,
                  torch::Tensor o, torch::Tensor xh1, torch::Tensor xh2, torch::Tensor rs, torch::Tensor dres,
                  torch::Tensor dout, torch::Tensor delta, torch::Tensor ws, torch::Tensor params, std::vector<int64_t> w,
                  c10::optional<torch::Tensor> seeds, c10::optional<torch::Tensor> stepctl, int64_t layer, double p,
                  int64_t G, c10::optional<torch::Tensor> kbits) {
  const int64_t C = params.size(0), R = B * L;
  for (auto* t : {&o, &xh1, &xh2, &dout}) rows64(*t, C, R, "activation");
  rows64(dres, C, R, "dres");
  AflHarPostB a{};
  if (dpool.has_value() && dpool->defined()) {
    TORCH_CHECK(dpool->numel() == C * B * 64, "dpool must be [C, B, 64]");
    a.dpool = f32(*dpool, "dpool");
  } else {
    TORCH_CHECK(dy.has_value() && dy->defined(), "har_post_bwd needs dy or dpool");
    rows64(*dy, C, R, "dy");
    a.dy = f32(*dy, "dy");
  }
  a.B = (int)B;
  a.L = (int)L;
  a.o = bf(o, "o");
  a.xh1 = bf(xh1, "xh1");
  a.xh2 = bf(xh2, "xh2");
  a.rs = f32(rs, "rs");
  TORCH_CHECK(rs.numel() == C * R * 2, "rs must be [C, R, 2]");
  a.dres = f32(dres, "dres");
  a.dout = bf(dout, "dout");
  a.delta = f32(delta, "delta");
  a.Lp = (int)(delta.numel() / (C * B * 4));
  TORCH_CHECK(delta.numel() == C * B * 4 * (int64_t)a.Lp && a.Lp >= L, "delta must be [C*B*4, Lp]");
  TORCH_CHECK(ws.numel() >= C * G * (int64_t)AFL_HAR_POST_NG, "ws too small");
  a.ws = f32(ws, "ws");
  a.params = f32(params, "params");
  a.P = params.size(1);
  a.w = layer_w(w);
  a.C = (int)C;
  a.R = R;
  a.d1 = drop(seeds, stepctl, layer + 1, p);
  a.df = drop(seeds, stepctl, layer + 2, p);
  a.d2 = drop(seeds, stepctl, layer + 3, p);
  a.kbits = kbits_of(kbits, C, R, a.d1.thr16 || a.df.thr16 || a.d2.thr16);
  ok(afl_har_post_bwd(a, (int)G, cur()), "har_post_bwd");
}

void har_qkv_bwd(torch::Tensor dqkv, torch::Tensor dres, torch::Tensor x, torch::Tensor dx, torch::Tensor ws,
                 torch::Tensor params, int64_t w_off, int64_t B, int64_t L, int64_t G) {
  const int64_t C = params.size(0), R = B * L, Lp = dqkv.size(2);
  headmajor(dqkv, C, B, Lp, "dqkv");
  rows64(dres, C, R, "dres");
  rows64(x, C, R, "x");
  rows64(dx, C, R, "dx");
  TORCH_CHECK(ws.numel() >= C * G * (int64_t)AFL_HAR_QKV_NG, "ws too small");
  AflHarQkvB a{bf(dqkv, "dqkv"), f32(dres, "dres"), bf(x, "x"), f32(dx, "dx"), f32(ws, "ws"), f32(params, "params"),
               params.size(1), (int)w_off, (int)C, (int)B, (int)L, (int)Lp};
  ok(afl_har_qkv_bwd(a, (int)G, cur()), "har_qkv_bwd");
}

void har_reduce(torch::Tensor ws, int64_t G, int64_t n, torch::Tensor seg, torch::Tensor grads) {
  dense(seg, "seg", torch::kInt32);
  TORCH_CHECK(seg.dim() == 2 && seg.size(1) == 3, "seg must be [nseg, 3]");
  const int64_t C = grads.size(0);
  TORCH_CHECK(ws.numel() >= C * G * n, "ws too small");
  ok(afl_har_reduce(f32(ws, "ws"), (int)C, (int)G, (int)n, seg.data_ptr<int>(), (int)seg.size(0), f32(grads, "grads"),
                    grads.size(1), cur()),
     "har_reduce");
}

}  // namespace

void afl_register_har(pybind11::module& m) {
  namespace py = pybind11;
  m.def("har_stem", &har_stem);
  m.def("har_pool", &har_pool);
  m.def("har_qkv", &har_qkv);
  m.def("har_post", &har_post, py::arg("o"), py::arg("x"), py::arg("xh1"), py::arg("xh2"), py::arg("rs"), py::arg("y"),
        py::arg("params"), py::arg("w"), py::arg("seeds"), py::arg("stepctl"), py::arg("layer"), py::arg("p"),
        py::arg("kbits") = py::none());
  m.attr("har_kbits_per_row") = py::int_(AFL_HAR_KBITS_PER_ROW);
  m.def("har_attn_fwd", &har_attn_fwd, py::arg("qkv"), py::arg("o"), py::arg("lse2"), py::arg("B"), py::arg("L"),
        py::arg("seeds"), py::arg("stepctl"), py::arg("layer"), py::arg("p"), py::arg("mask") = py::none());
  m.def("har_attn_bwd", &har_attn_bwd, py::arg("qkv"), py::arg("lse2"), py::arg("dout"), py::arg("delta"),
        py::arg("dqkv"), py::arg("B"), py::arg("L"), py::arg("seeds"), py::arg("stepctl"), py::arg("layer"),
        py::arg("p"), py::arg("mask") = py::none());
  m.def("har_mask_words", [](int64_t Lp) { return (int64_t)AFL_HAR_MASK_WORDS(Lp); });
  m.def("har_post_bwd", &har_post_bwd, py::arg("dy"), py::arg("dpool"), py::arg("B"), py::arg("L"), py::arg("o"),
        py::arg("xh1"), py::arg("xh2"), py::arg("rs"), py::arg("dres"), py::arg("dout"), py::arg("delta"), py::arg("ws"),
        py::arg("params"), py::arg("w"), py::arg("seeds"), py::arg("stepctl"), py::arg("layer"), py::arg("p"),
        py::arg("G"), py::arg("kbits") = py::none());
  m.def("har_qkv_bwd", &har_qkv_bwd);
  m.def("har_reduce", &har_reduce);
  m.def("har_blocks", [](int64_t R) { return afl_har_blocks(R); });
  m.attr("har_post_ng") = py::int_(AFL_HAR_POST_NG);
  m.attr("har_qkv_ng") = py::int_(AFL_HAR_QKV_NG);
}
