// RNNModel (ICU) flat parameter layout shared by the fused trainers (rnn.hip, rnn2.hip): state_dict order
// of reference src/Model.py:91-118 (97,665 fp32).  Per branch: 3 bidirectional GRU layers (per direction
// W_ih [96][kin], W_hh [96][32], b_ih [96], b_hh [96], gate order r z n), LayerNorm(64) weight | bias; then
// fc1 (128 -> 32), fc2 (32 -> 16), output (16 -> 1).
#pragma once
#include <hip/hip_runtime.h>

namespace rnl {

constexpr int HU = 32, G3 = 96, ROWW = 24, DV = 7, DL = 16;
__host__ __device__ constexpr int dir_block(int k) { return G3 * k + G3 * HU + 2 * G3; }
__host__ __device__ constexpr int branch_size(int din) { return 2 * dir_block(din) + 4 * dir_block(64) + 128; }
constexpr int BASE_V = 0, BASE_L = branch_size(DV);
constexpr int FC1_W = BASE_L + branch_size(DL);
constexpr int FC1_B = FC1_W + 32 * 128, FC2_W = FC1_B + 32, FC2_B = FC2_W + 16 * 32, OUT_W = FC2_B + 16,
              OUT_B = OUT_W + 16, NPARAM = OUT_B + 1;
static_assert(NPARAM == 97665, "RNNModel parameter count");

template <int BR>
struct Br {
  static constexpr int base = BR == 0 ? BASE_V : BASE_L;
  static constexpr int din = BR == 0 ? DV : DL;
  static constexpr int kin(int l) { return l == 1 ? din : 64; }
  // offset of layer l (1..3), direction d (0, 1): W_ih [96][kin], W_hh [96][32], b_ih [96], b_hh [96]
  static constexpr int dir_off(int l, int d) {
    return base + (l == 1 ? d * dir_block(din) : 2 * dir_block(din) + ((l - 2) * 2 + d) * dir_block(64));
  }
  static constexpr int wih(int l, int d) { return dir_off(l, d); }
  static constexpr int bih(int l, int d) { return dir_off(l, d) + G3 * kin(l) + G3 * HU; }
  static constexpr int bhh(int l, int d) { return bih(l, d) + G3; }
  static constexpr int ln_w = base + 2 * dir_block(din) + 4 * dir_block(64);
  static constexpr int ln_b = ln_w + 64;
};
static_assert(Br<1>::ln_b + 64 == FC1_W, "branch layout");

}  // namespace rnl
