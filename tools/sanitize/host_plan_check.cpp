// Host-side sanitizer harness (AddressSanitizer + UndefinedBehaviorSanitizer; SURVEY §5 race /
// fault detection). GPU ASan / XNACK runs are not available on the MI355X pool, so the host logic
// of the kernel library is checked here on the CPU: the launch planners that size split-K / slab
// workspaces, BatchNorm-statistics slab rows and persistent grids, and the autotuner's candidate
// lists — for every conv geometry of the model zoo census at the batch sizes the framework runs,
// and for every candidate (tile config, split) the autotuner could pick. No kernel is launched;
// without a GPU the device queries fall back to the MI355X defaults (256 CUs).
//
// Build + run: tools/sanitize/run.sh (tests/test_sanitize_cpu.py drives it).
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <utility>
#include <vector>

namespace pca {
int64_t conv_fwd_ws_floats(int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride, int pad,
                           int groups, int Ho, int Wo, bool has_bias);
int64_t conv_dgrad_ws_floats(int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride,
                             int pad, int groups, int Ho, int Wo);
int conv_fwd_stat_rows(int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride, int pad,
                       int groups, int Ho, int Wo, bool has_bias);
int conv_dgrad_bn_rows(int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride, int pad,
                       int groups, int Ho, int Wo);
int64_t conv_wgrad_ws_floats(int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride,
                             int pad, int groups, int Ho, int Wo);
std::vector<std::pair<int, int>> conv_tune_candidates(int kind, int N, int H, int W, int Cin,
                                                      int Cout, int KH, int KW, int stride,
                                                      int pad, int groups, int Ho, int Wo);
std::vector<std::pair<int, int>> wgrad_tune_candidates(int N, int H, int W, int Cin, int Cout,
                                                       int KH, int KW, int stride, int pad,
                                                       int groups);
void conv_set_trial(int cfg, int split);
void wgrad_set_trial(int cfg, int split);
}  // namespace pca

struct Shape {
  int Cin, Cout, H, k, s, p, g;
};

// conv census of the zoo: ResNet / VGG / MobileNetV2 / EfficientNet / RegNet /
// ResNeXt / DPN shapes (+ depthwise / grouped / odd widths the planners must reject cleanly)
static const Shape kShapes[] = {
    {8, 64, 32, 3, 1, 1, 1},     {64, 64, 32, 3, 1, 1, 1},    {64, 128, 32, 3, 2, 1, 1},
    {64, 128, 32, 1, 2, 0, 1},   {128, 128, 16, 3, 1, 1, 1},  {128, 256, 16, 3, 2, 1, 1},
    {256, 256, 8, 3, 1, 1, 1},   {256, 512, 8, 3, 2, 1, 1},   {512, 512, 4, 3, 1, 1, 1},
    {128, 256, 16, 1, 2, 0, 1},  {256, 512, 8, 1, 2, 0, 1},   {16, 96, 32, 1, 1, 0, 1},
    {96, 24, 32, 1, 1, 0, 1},    {24, 144, 32, 1, 1, 0, 1},   {144, 144, 32, 3, 1, 1, 144},
    {160, 960, 4, 1, 1, 0, 1},   {320, 1280, 4, 1, 1, 0, 1},  {1152, 192, 2, 1, 1, 0, 1},
    {672, 672, 4, 5, 1, 2, 672}, {232, 232, 4, 3, 2, 1, 8},   {128, 128, 8, 3, 1, 1, 32},
    {96, 96, 16, 3, 1, 1, 3},    {3, 64, 32, 3, 1, 1, 1},     {6, 16, 14, 5, 1, 0, 1},
    {512, 10, 1, 1, 1, 0, 1},    {48, 48, 8, 3, 1, 1, 1},
};

static int g_fail = 0;
#define CHECK(cond, ...)                                   \
  do {                                                     \
    if (!(cond)) {                                         \
      std::fprintf(stderr, "CHECK failed: " #cond " : "); \
      std::fprintf(stderr, __VA_ARGS__);                   \
      std::fprintf(stderr, "\n");                          \
      ++g_fail;                                            \
    }                                                      \
  } while (0)

int main() {
  long checks = 0;
  for (int N : {1, 7, 16, 128, 256, 1024}) {
    for (const Shape& sh : kShapes) {
      const int Ho = (sh.H + 2 * sh.p - sh.k) / sh.s + 1;
      if (Ho <= 0) continue;
      const int args[] = {N, sh.H, sh.H, sh.Cin, sh.Cout, sh.k, sh.k, sh.s, sh.p, sh.g, Ho, Ho};
      (void)args;
      const bool mfma_ok = (sh.Cin / sh.g) % 8 == 0 && (sh.Cout / sh.g) % 8 == 0;
      if (!mfma_ok) continue;   // the Python layer routes these to padded / direct kernels
      for (int kind = 0; kind < 2; ++kind) {
        auto cands = pca::conv_tune_candidates(kind, N, sh.H, sh.H, sh.Cin, sh.Cout, sh.k, sh.k,
                                               sh.s, sh.p, sh.g, Ho, Ho);
        cands.push_back({-1, -1});   // the heuristic / tuned path
        for (const auto& c : cands) {
          pca::conv_set_trial(c.first, c.second);
          if (kind == 0) {
            const int64_t ws = pca::conv_fwd_ws_floats(N, sh.H, sh.H, sh.Cin, sh.Cout, sh.k, sh.k,
                                                       sh.s, sh.p, sh.g, Ho, Ho, false);
            const int rows = pca::conv_fwd_stat_rows(N, sh.H, sh.H, sh.Cin, sh.Cout, sh.k, sh.k,
                                                     sh.s, sh.p, sh.g, Ho, Ho, false);
            CHECK(ws >= 0 && ws <= (int64_t)8 * N * Ho * Ho * sh.Cout, "fwd ws %lld N=%d cfg=%d",
                  (long long)ws, N, c.first);
            CHECK(rows >= 1 && rows <= 4096, "fwd stat rows %d N=%d cfg=%d", rows, N, c.first);
          } else {
            const int64_t ws = pca::conv_dgrad_ws_floats(N, sh.H, sh.H, sh.Cin, sh.Cout, sh.k,
                                                         sh.k, sh.s, sh.p, sh.g, Ho, Ho);
            const int rows = pca::conv_dgrad_bn_rows(N, sh.H, sh.H, sh.Cin, sh.Cout, sh.k, sh.k,
                                                     sh.s, sh.p, sh.g, Ho, Ho);
            CHECK(ws >= 0 && ws <= (int64_t)8 * N * sh.H * sh.H * sh.Cin, "dgrad ws %lld cfg=%d",
                  (long long)ws, c.first);
            CHECK(rows >= 0 && rows <= 8192, "dgrad bn rows %d cfg=%d", rows, c.first);
          }
          checks += 2;
        }
        pca::conv_set_trial(-1, -1);
      }
      auto wc = pca::wgrad_tune_candidates(N, sh.H, sh.H, sh.Cin, sh.Cout, sh.k, sh.k, sh.s, sh.p,
                                           sh.g);
      wc.push_back({-1, -1});
      for (const auto& c : wc) {
        pca::wgrad_set_trial(c.first, c.second);
        const int64_t ws = pca::conv_wgrad_ws_floats(N, sh.H, sh.H, sh.Cin, sh.Cout, sh.k, sh.k,
                                                     sh.s, sh.p, sh.g, Ho, Ho);
        const int64_t dw = (int64_t)sh.Cout * sh.k * sh.k * (sh.Cin / sh.g);
        // a slab holds at most (pixel splits) x dW; splits never exceed the pixel count
        CHECK(ws >= 0 && ws <= dw * ((int64_t)N * Ho * Ho + 1), "wgrad ws %lld cfg=%d split=%d",
              (long long)ws, c.first, c.second);
        ++checks;
      }
      pca::wgrad_set_trial(-1, -1);
    }
  }
  std::printf("host plan checks: %ld, failures: %d\n", checks, g_fail);
  return g_fail ? 1 : 0;
}
