// Host-side checker for the integer math the GPU kernels share with their Python mirrors, built with
// AddressSanitizer + UndefinedBehaviorSanitizer on the host half only (the reference has
// no sanitizer coverage; GPU ASan is not available on this pool, so the sanitised build runs on CPU):
//
//   hipcc --offload-arch=gfx950 -O1 -g -fno-omit-frame-pointer -I csrc \
//         -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined host_check.hip -o host_check
//
// (tools/host_sanitize.sh does exactly this; tests/test_host_sanitize.py builds and runs it.)
//
// Modes (all output on stdout, exit status != 0 on any failed invariant):
//   plan <n_train> <epochs> <seed>:<nd> ...    visit plan of every client (plan.hip:k_make_plan on the
//                                              host), one line per (client, epoch); also checks that each
//                                              row is duplicate-free, in range, and that every epoch of a
//                                              client visits the same subset
//   mask <key> <layer> <rows> <cols> <p>       dropout keep bits of common.h:afl_keep, one row per line
//   hash <a> <b>                               common.h:afl_hash32 (the per-step dropout key)
//   selftest                                   bijection sweep of pl_perm over many domain sizes / keys
// The Python side compares the printed values bit-for-bit with attackfl_amd/fl/trainers.py and
// attackfl_amd/ops/masks.py, which themselves are the CPU oracles of the GPU kernels.
#include "../kernels/plan.hip"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace {

int fail(const char* what, long a = 0, long b = 0) {
  std::fprintf(stderr, "host_check: FAILED %s (%ld, %ld)\n", what, a, b);
  return 1;
}

// the subset-then-shuffle plan of one client, exactly as k_make_plan computes row (c, e)
void plan_row(uint64_t seed, int nd, int n_train, int e, std::vector<int>& out) {
  out.resize(nd);
  const PlanKeys k = pl_keys(seed, e);
  const int hn = pl_half_bits((uint32_t)nd), ht = pl_half_bits((uint32_t)n_train);
  for (int i = 0; i < nd; ++i) {
    const uint32_t j = pl_perm((uint32_t)i, (uint32_t)nd, hn, k.e0, k.e1);
    out[i] = (int)pl_perm(j, (uint32_t)n_train, ht, k.s0, k.s1);
  }
}

int run_plan(int argc, char** argv) {
  if (argc < 4) return fail("usage: plan <n_train> <epochs> <seed>:<nd> ...");
  const int n_train = std::atoi(argv[2]), E = std::atoi(argv[3]);
  if (n_train <= 0 || E <= 0) return fail("bad n_train / epochs", n_train, E);
  std::vector<int> row;
  std::vector<unsigned char> seen(n_train), subset(n_train);
  for (int a = 4; a < argc; ++a) {
    const char* colon = std::strchr(argv[a], ':');
    if (!colon) return fail("client spec must be seed:nd", a);
    const uint64_t seed = std::strtoull(argv[a], nullptr, 10);
    const int nd = std::atoi(colon + 1);
    if (nd <= 0 || nd > n_train) return fail("nd out of range", nd, n_train);
    std::fill(subset.begin(), subset.end(), 0);
    for (int e = 0; e < E; ++e) {
      plan_row(seed, nd, n_train, e, row);
      std::fill(seen.begin(), seen.end(), 0);
      for (int i = 0; i < nd; ++i) {
        const int v = row[i];
        if (v < 0 || v >= n_train) return fail("row index out of range", v, n_train);
        if (seen[v]++) return fail("duplicate row in an epoch", v, e);
        if (e == 0)
          subset[v] = 1;
        else if (!subset[v])
          return fail("epoch visits a row outside the client's subset", v, e);
        std::printf(i ? " %d" : "%d", v);
      }
      std::printf("\n");
    }
  }
  return 0;
}

int run_mask(int argc, char** argv) {
  if (argc != 7) return fail("usage: mask <key> <layer> <rows> <cols> <p>");
  const uint32_t key = (uint32_t)std::strtoul(argv[2], nullptr, 10), layer = (uint32_t)std::atoi(argv[3]);
  const int rows = std::atoi(argv[4]), cols = std::atoi(argv[5]);
  const double p = std::atof(argv[6]);
  if (rows <= 0 || cols <= 0 || !(p >= 0.0 && p < 1.0)) return fail("bad mask shape / p", rows, cols);
  const uint32_t thr = (uint32_t)std::lround(p * 65536.0);
  std::string line((size_t)cols, '0');
  for (int r = 0; r < rows; ++r) {
    for (int c = 0; c < cols; ++c) line[c] = afl_keep(key, layer, (uint32_t)r, (uint32_t)c, thr) ? '1' : '0';
    std::printf("%s\n", line.c_str());
  }
  return 0;
}

int run_selftest() {
  // pl_perm must be a bijection of [0, n) for every n and key: walk a spread of sizes incl. the
  // powers of two and their neighbours (cycle-walking edge cases) and the ICU/HAR table sizes
  std::vector<uint32_t> sizes = {1, 2, 3, 4, 5, 7, 8, 9, 15, 16, 17, 63, 64, 65, 255, 256, 257, 1000, 4095, 4096,
                                 4097, 12000, 15000, 65535, 65536, 65537, 98765, 262145};
  std::vector<unsigned char> seen;
  long checked = 0;
  for (uint32_t n : sizes) {
    const int h = pl_half_bits(n);
    if ((1ull << (2 * h)) < n || (h > 1 && (1ull << (2 * h - 2)) >= n)) return fail("pl_half_bits", n, h);
    for (uint64_t seed : {0ull, 1ull, 0x123456789ABCDEFull, ~0ull}) {
      const PlanKeys k = pl_keys(seed, (int)(seed & 7));
      seen.assign(n, 0);
      for (uint32_t i = 0; i < n; ++i) {
        const uint32_t v = pl_perm(i, n, h, k.s0, k.e1);
        if (v >= n) return fail("pl_perm out of range", (long)v, (long)n);
        if (seen[v]++) return fail("pl_perm not injective", (long)v, (long)n);
      }
      checked += n;
    }
  }
  // afl_keep: the 16-bit halves of one hash must give two independent-looking columns; check the
  // empirical keep rate for p in {0.1, 0.5} over a 512 x 512 grid is within 1% of 1 - p
  for (double p : {0.1, 0.5}) {
    const uint32_t thr = (uint32_t)std::lround(p * 65536.0);
    long kept = 0;
    for (uint32_t r = 0; r < 512; ++r)
      for (uint32_t c = 0; c < 512; ++c) kept += afl_keep(afl_hash32(7u, 3u), 2u, r, c, thr);
    const double rate = (double)kept / (512.0 * 512.0);
    if (std::fabs(rate - (1.0 - p)) > 0.01) return fail("afl_keep rate", (long)(rate * 1e6), (long)(p * 1e6));
  }
  std::printf("selftest ok: %ld permutation points\n", checked);
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) return fail("usage: host_check plan|mask|hash|selftest ...");
  const std::string mode = argv[1];
  if (mode == "plan") return run_plan(argc, argv);
  if (mode == "mask") return run_mask(argc, argv);
  if (mode == "hash") {
    if (argc != 4) return fail("usage: hash <a> <b>");
    std::printf("%u\n", afl_hash32((uint32_t)std::strtoul(argv[2], nullptr, 10),
                                   (uint32_t)std::strtoul(argv[3], nullptr, 10)));
    return 0;
  }
  if (mode == "selftest") return run_selftest();
  return fail("unknown mode");
}
