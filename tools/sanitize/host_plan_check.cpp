// Host-side launch planning of the rtseg HIP kernels under AddressSanitizer + UBSan (CPU only):
// every tile / slab / workspace planner the bindings call before a launch is swept over the
// zoo's shape space and checked for overflow, UB and internally consistent results, and the
// FastDiv magic numbers used in every index decomposition are checked against exact division.
// Built and run by tools/sanitize/run.sh (tests/test_sanitizers_cpu.py); the kernels themselves
// are compiled host-only here (no device code, no GPU needed).
#include <cstdio>
#include <cstdlib>
#include <random>

#include "rtseg_common.h"
#include "rtseg_launch.h"

using namespace rtseg;

static int failures = 0;
#define CHECK(cond, ...)                         \
  do {                                           \
    if (!(cond)) {                               \
      std::fprintf(stderr, "FAIL %s: ", #cond);  \
      std::fprintf(stderr, __VA_ARGS__);         \
      std::fprintf(stderr, "\n");                \
      ++failures;                                \
    }                                            \
  } while (0)

static uint32_t fastdiv_host(const FastDiv& f, uint32_t n) {  // == FastDiv::div on the device
  const uint64_t t = (static_cast<uint64_t>(n) * f.m) >> 32;
  return static_cast<uint32_t>((t + n) >> f.s);
}

static void check_fastdiv() {
  std::mt19937 rng(1234);
  const uint32_t ds[] = {1, 2, 3, 5, 7, 19, 32, 33, 64, 96, 100, 127, 128, 255, 256, 257, 1000, 1023, 1024, 1025,
                         2047, 2048, 4095, 65535, 65536, 1u << 20, (1u << 20) + 1, 1u << 31};
  for (uint32_t d : ds) {
    const FastDiv f = FastDiv::make(d);
    for (int i = 0; i < 20000; ++i) {
      uint32_t n = i < 4096 ? static_cast<uint32_t>(i) : rng() >> (rng() % 32);
      if (i % 1000 == 999) n = 0x7fffffffu - static_cast<uint32_t>(i);
      CHECK(fastdiv_host(f, n) == n / d, "d=%u n=%u got %u", d, n, fastdiv_host(f, n));
    }
  }
}

static ConvGeom geom(int n, int cin, int h, int w, int cout, int k, int s, int d) {
  ConvGeom g{};
  g.n = n; g.cin = cin; g.h = h; g.w_in = w; g.cout = cout;
  g.kh = g.kw = k; g.sh = g.sw = s; g.dh = g.dw = d; g.ph = g.pw = (k - 1) / 2 * d;
  g.ho = (h + 2 * g.ph - d * (k - 1) - 1) / s + 1;
  g.wo = (w + 2 * g.pw - d * (k - 1) - 1) / s + 1;
  return g;
}

static void check_conv_plans() {
  const int cs[] = {32, 64, 96, 128, 192, 256, 512, 1024};
  const int hw[][2] = {{256, 512}, {128, 256}, {64, 128}, {32, 64}, {16, 32}, {7, 9}, {1, 1}};
  for (int n : {1, 2, 32})
    for (int cin : cs)
      for (int cout : cs)
        for (auto& s : hw)
          for (int k : {1, 3})
            for (int st : {1, 2}) {
              const ConvGeom g = geom(n, cin, s[0], s[1], cout, k, st, 1);
              if (g.ho <= 0 || g.wo <= 0) continue;
              for (int mode = 0; mode < 3; ++mode) {
                if (!conv_igemm_supported(g, mode)) continue;
                if (mode == 0) CHECK(conv_igemm_slabs(g) > 0, "fwd slabs n=%d cin=%d cout=%d", n, cin, cout);
                if (mode == 2) {
                  const int64_t ws = conv_igemm_wgrad_ws_elems(g);
                  CHECK(ws >= static_cast<int64_t>(cout) * cin * k * k, "wgrad ws %lld", static_cast<long long>(ws));
                }
              }
              for (int mode = 0; mode < 2; ++mode)
                if (conv_halo_supported(g, mode) && mode == 0) CHECK(conv_halo_slabs(g) > 0, "halo slabs");
            }
}

static void check_bn_plans() {
  for (int dtype : {kF32, kBF16, kF16})
    for (int C = 1; C <= 2048; C += (C < 64 ? 1 : 37)) {
      const int v = bn_vec_width(dtype, C);
      if (v == 0) continue;
      CHECK(C % v == 0 && C / v <= 256, "bn vec C=%d v=%d", C, v);
      for (int64_t M : {int64_t{1}, int64_t{2}, int64_t{255}, int64_t{65536}, int64_t{32} * 256 * 512}) {
        const int G = bn_partial_grid(M, C, dtype);
        // odd C (flat, phase-stationary kernels): a multiple of C blocks, at most one C past 1024
        const bool flat = dtype != kF16 && C >= 3 && (C & 1) && v == 1;
        if (flat) {
          CHECK(G >= C && G % C == 0 && G < 1024 + C, "bn flat grid M=%lld C=%d G=%d", static_cast<long long>(M), C, G);
        } else {
          CHECK(G >= 1 && G <= 2048, "bn grid M=%lld C=%d G=%d", static_cast<long long>(M), C, G);  // RTSEG_BN_REDUCE_CAP default
        }
      }
    }
}

static void check_misc_plans() {
  for (int dtype : {kF32, kBF16})
    for (int C : {1, 3, 8, 16, 19, 24, 64, 96, 128, 384, 1024}) {
      const int v = gate_vec_width(dtype, C);
      CHECK(v == 0 || C % v == 0, "gate vec C=%d v=%d", C, v);
      CHECK(dw_vec(dtype, C) >= 0, "dw vec");
    }
  for (int64_t hw : {int64_t{1}, int64_t{64}, int64_t{4096}, int64_t{1} << 21})
    for (int n : {1, 8, 32}) CHECK(gate_channel_blocks(hw, n) >= 1, "gate blocks");
  for (int ch : {1, 7, 512, 1024})
    for (int cw : {1, 9, 1024, 2048}) {
      const int b = augment_stat_blocks(ch, cw);
      CHECK(b >= 1 && b <= 64, "aug blocks %d", b);
    }
  // PReLU weight-gradient plans cover every row / plane exactly once
  for (int C : {1, 3, 16, 19, 64, 100, 256, 4096})
    for (int64_t M : {int64_t{1}, int64_t{7}, int64_t{4096}, int64_t{32} * 128 * 256}) {
      ActArgs a{};
      a.C = C;
      a.n = M * C;
      a.inner = 1;
      ActPreluPlan p = act_prelu_plan(a);
      CHECK(!p.planes && p.blocks >= 1 && p.rows_per_block * p.blocks >= M &&
                p.rows_per_block * (p.blocks - 1) < M && p.tx >= 1 && p.tx <= 64,
            "prelu rows C=%d M=%lld", C, static_cast<long long>(M));
      if (C > 1) {
        a.inner = 4096;
        a.n = int64_t{8} * C * 4096;
        p = act_prelu_plan(a);
        CHECK(p.planes && p.slices >= 1 && p.blocks == 8 * C * p.slices, "prelu planes C=%d", C);
      }
    }
  for (int n : {1, 4}) CHECK(detail_loss_blocks(n, 1024, 2048) >= 1, "detail blocks");
  CHECK(kd_partial_blocks(int64_t{32} * 1024 * 2048) >= 1, "kd blocks");
}

int main() {
  check_fastdiv();
  check_conv_plans();
  check_bn_plans();
  check_misc_plans();
  if (failures) {
    std::fprintf(stderr, "%d check(s) failed\n", failures);
    return 1;
  }
  std::printf("host planning checks passed\n");
  return 0;
}
