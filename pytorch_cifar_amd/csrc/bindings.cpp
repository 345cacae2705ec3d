// Python bindings of the gfx950 kernel library (module pytorch_cifar_amd._C).
//
// Every entry point validates dtype/layout/shape on the host before launching (a mis-shaped
// launch of a hand-written kernel can fault the whole GPU), allocates outputs through the
// PyTorch caching allocator and enqueues on the current HIP stream, so all ops are
// hipGraph-capturable (no host syncs, no hipMalloc inside).
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>
#include <torch/extension.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

extern "C" const char pca_src_digest[];  // build/srcdigest.cpp, written by _build.py

typedef __bf16 bf16;

namespace pca {
// conv_mfma.hip
void conv_fwd_launch(const bf16*, const bf16*, const float*, bf16*, float*, int, int, int, int, int,
                     int, int, int, int, int, int, int, hipStream_t, float* ws);
int64_t conv_fwd_ws_floats(int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride,
                           int pad, int groups, int Ho, int Wo, bool has_bias);
int64_t conv_dgrad_ws_floats(int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride,
                             int pad, int groups, int Ho, int Wo);
bool conv_needs_tune(int kind, int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride,
                     int pad, int groups, int Ho, int Wo, bool has_bias);
std::vector<std::pair<int, int>> conv_tune_candidates(int kind, int N, int H, int W, int Cin,
                                                      int Cout, int KH, int KW, int stride,
                                                      int pad, int groups, int Ho, int Wo);
void conv_set_trial(int cfg, int split);
void conv_record_tuned(int kind, int N, int H, int W, int Cin, int Cout, int KH, int KW,
                       int stride, int pad, int groups, int Ho, int Wo, int cfg, int split);
int conv_tuned_count();
void conv_clear_tuned();
bool wgrad_needs_tune(int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride, int pad,
                      int groups);
std::vector<std::pair<int, int>> wgrad_tune_candidates(int N, int H, int W, int Cin, int Cout,
                                                       int KH, int KW, int stride, int pad,
                                                       int groups);
void wgrad_set_trial(int cfg, int split);
void wgrad_record_tuned(int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride, int pad,
                        int groups, int cfg, int split);
int wgrad_tuned_count();
void wgrad_clear_tuned();
std::vector<std::vector<int>> tune_export();
void c64_set_prof(int64_t* p);
int c64_grid_size(int N, int H);
void conv_c64_set_xf(const float* xf, uint8_t* mask);
bool conv_c64_applicable(int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride,
                         int pad, int groups);
void set_halo_xf(const float* xf);
int64_t wgrad_halo_ws_floats(int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride,
                             int pad, int groups);
void set_bn_dbias(float* p);
bool winograd_applicable(int N, int H, int W, int Ci, int Co);
int winograd_stat_rows(int N, int H, int W);
void winograd_filter_launch(const float* w, int Co, int Ci, bf16* U, hipStream_t st);
void winograd_fwd_launch(const bf16* x, const bf16* U, bf16* y, float* stats, int N, int H, int W,
                         int Ci, int Co, hipStream_t st);
void copy_rows_launch(const bf16* src, int lds, bf16* dst, int ldd, int P, int C, hipStream_t st,
                      const bf16* add = nullptr, int lda = 0);
// batchnorm.hip: row strides of the next BN launches' tensors (0 = dense; common.h BnLd)
struct BnLd {
  int y, out, dout, dx, dx_acc;
};
BnLd bn_ld();
void set_bn_ld(const BnLd& ld);
int c64_version(int v);
int tune_import(const std::vector<std::vector<int>>& rows);
int conv_fwd_stat_rows(int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride, int pad,
                       int groups, int Ho, int Wo, bool has_bias);
void set_conv_tile(int kind, int idx);
void conv_dgrad_launch(const bf16*, const bf16*, bf16*, int, int, int, int, int, int, int, int,
                       int, int, int, int, hipStream_t, const bf16* addend, float* ws,
                       const bf16* bn_y = nullptr, const uint8_t* bn_mask = nullptr,
                       const float* bn_aux = nullptr, float* bn_part = nullptr);
int conv_dgrad_bn_rows(int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride, int pad,
                       int groups, int Ho, int Wo);
void conv_set_bn_dual(const bf16* y2, const float* aux2);
void conv_set_bn_ldy(int ld);
void conv_set_addend_s2c(int on);
bool conv_dgrad_s2c_ok(int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride, int pad,
                       int groups, int Ho, int Wo);
void s2c_expand_launch(const bf16* in, bf16* out, int N, int Hc, int Wc, int C, hipStream_t st);
void conv_wgrad_launch(const bf16* x, const bf16* dy, float* dw, float* ws, int N, int H, int W,
                       int Cin, int Cout, int KH, int KW, int stride, int pad, int groups, int Ho,
                       int Wo, hipStream_t st);
int64_t conv_wgrad_ws_floats(int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride,
                             int pad, int groups, int Ho, int Wo);
// batchnorm.hip
int bn_row_blocks(int M, int C);
int bn_rows_max_c();
void wgrad_defer_scope(bool on);
int wgrad_deferred_count();
void wgrad_flush_launch(hipStream_t st);
void set_wgrad_piggy(bool on);
void wgrad_truncate_pending(int n);
int64_t conv_nk_min_m(int64_t v);
void bn_stats_launch(const bf16*, int, int, float*, int, hipStream_t, float* krow = nullptr);
void bn_stats_copy_launch(const bf16* x, int ldx, int M, int C, bf16* dst, int ldd, float* acc,
                          int ldc, int R, int P, float* krow, hipStream_t st);
int colsum_launch(const float*, int, int, float*, hipStream_t);
void bias_grad_fold_launch(const float*, int, int, int, float*, hipStream_t);
void bn_finalize_launch(const float*, int, int, double, const float*, const float*, float*, float*,
                        int64_t*, float, float, int, int, float*, hipStream_t,
                        const float* kin = nullptr, float* pilot_out = nullptr,
                        float* zero = nullptr, int zero_n = 0, int ld = 0);
void bn_apply_launch(const bf16*, const float*, int, size_t, const bf16*, const bf16*,
                     const float*, int, bf16*, uint8_t*, hipStream_t);
void bn_bwd_reduce_launch(const bf16*, const bf16*, const uint8_t*, const bf16*, const float*,
                          const bf16*, const float*, int, int, int, float*, int, hipStream_t);
void bn_bwd_finalize_launch(const float*, int, int, int, float, const float*, const float*,
                            const float*, const float*, int, float*, float*, float*, float*,
                            float*, int, hipStream_t, float* zero1 = nullptr, int zero1_n = 0,
                            float* zero2 = nullptr, int zero2_n = 0);
void bn_bwd_apply_launch(const bf16*, const bf16*, const uint8_t*, const bf16*, const float*,
                         const float*, int, int, size_t, bf16*, bf16*, const bf16*, bf16*,
                         hipStream_t);
int stat_shards();
void set_stat_shards(int shards);
const float* stat_shift();
void set_stat_shift(const float* k);
bool bn_apply_acc_launch(const bf16* y, int C, int M, float count, float* acc, int R,
                         const float* gamma, const float* beta, float* rmean, float* rvar,
                         int64_t* nbt, float momentum, float eps, float* aux, float* acc2, int R2,
                         const float* gamma2, const float* beta2, float* rmean2, float* rvar2,
                         int64_t* nbt2, float momentum2, float eps2, float* aux2, const bf16* res,
                         const bf16* y2, int act, bf16* out, uint8_t* mask, float* zero,
                         int zero_n, hipStream_t st, bool shifted = false, float* pilot = nullptr,
                         bool shifted2 = false, float* pilot2 = nullptr, int acc_off = 0, int acc_ld = 0);
bool bn_bwd_apply_acc_launch(const bf16* dout, const uint8_t* mask, const bf16* y, int C, int M,
                             float count, float* acc, int R, const float* aux, const float* gamma,
                             float* dgamma, float* dbeta, const float* aux2, const float* gamma2,
                             float* dgamma2, float* dbeta2, int act, bf16* dy, bf16* dres,
                             const bf16* y2, bf16* dy2, float* zero, int zero_n, float* zero2,
                             int zero2_n, hipStream_t st);
// stem.hip
bool stem_wgrad_supported(int N, int H, int W, int Cs, int Ci, int Co);
int stem_wgrad_slab_rows(int N, int H);
void stem_wgrad_launch(const bf16* x, const bf16* dy, int N, int H, int Co, float* slab, float* out,
                       hipStream_t st);
// misc.hip
void nchw_to_nhwc_launch(const float*, int, int, int, int, bf16*, hipStream_t);
void nhwc_to_nchw_launch(const bf16*, int, int, int, int, float*, hipStream_t);
void augment_launch(const uint8_t*, const int64_t*, const int32_t*, int, int, int, int,
                    const float*, const float*, bf16*, const int64_t*, int64_t*, hipStream_t);
void gap_fwd_launch(const bf16*, int, int, int, float*, hipStream_t);
void gap_bwd_launch(const float*, int, int, int, bf16*, hipStream_t);
bool head_supported(int C, int K);
bool se_mlp_supported(int C, int R);
void se_mlp_fwd_launch(const float*, int, int, int, const float*, const float*, const float*,
                       const float*, int, float*, float*, hipStream_t);
void se_mlp_bwd_launch(const float*, const float*, const float*, int, int, int, const float*,
                       const float*, int, float*, float*, float*, float*, float*, float*,
                       hipStream_t);
void se_ds_launch(const bf16*, const bf16*, const float*, int, int, int, float*, hipStream_t);
void se_dx_launch(const bf16*, const float*, const float*, int, int, int, bf16*, hipStream_t);
bool head_batch_supported(int N, int K);
void head_fwd_launch(const bf16*, int, int, int, const float*, const float*, int, float*, float*,
                     float, int64_t*, uint8_t*, hipStream_t);
void head_bwd_launch(const float*, const float*, const float*, int, int, int, int, bf16*, float*,
                     float*, float, const uint8_t*, hipStream_t, const bf16* bn_y,
                     const uint8_t* bn_mask, const float* bn_aux, float* bn_acc, int bn_R);
void dropout_fwd_launch(const void*, bool, size_t, int64_t, float, int64_t*, uint8_t*, void*,
                        hipStream_t);
void dropout_bwd_launch(const void*, bool, size_t, int64_t, float, const uint8_t*, void*,
                        hipStream_t);
void avgpool_fwd_launch(const bf16*, int, int, int, int, int, int, int, int, int, bf16*, hipStream_t);
void avgpool_bwd_launch(const bf16*, int, int, int, int, int, int, int, int, int, bf16*, hipStream_t);
void maxpool_fwd_launch(const bf16*, int, int, int, int, int, int, int, int, int, bf16*, uint8_t*,
                        hipStream_t);
void maxpool_bwd_launch(const bf16*, const uint8_t*, int, int, int, int, int, int, int, int, int,
                        bf16*, hipStream_t);
void ce_fused_launch(const float*, const int64_t*, int, int, float*, float*, double*, hipStream_t);
void scale_by_scalar_launch(const float*, const float*, size_t, float*, hipStream_t);
void sgd_launch(const int64_t*, int, float* const*, const float* const*, float* const*,
                bf16* const*, const float*, float, float, float, float, int, int, hipStream_t,
                int zero_grad);
void sgd_prep_launch(const int64_t*, int, float* const*, const float* const*, float* const*,
                     const float*, float, float, float, float, int, int, const int64_t*,
                     const int64_t*, int, const int64_t*, hipStream_t, int zero_grad);
void se_scale_fwd_launch(const bf16*, const float*, int, int, int, bf16*, hipStream_t);
bool se_fused_supported(int C, int R);
void se_fwd_fused_launch(const bf16*, int, int, int, int, const float*, const float*,
                         const float*, const float*, int, float*, float*, float*, hipStream_t);
void se_bwd_data_launch(const bf16*, const bf16*, const float*, int, int, int, int, const float*,
                        const float*, const float*, int, float*, float*, float*, hipStream_t);
void se_mlp_bwd_param_launch(const float*, const float*, const float*, const float*, int, int,
                             int, int, float*, float*, float*, float*, hipStream_t);
struct CatArgs {
  const bf16* src[8];
  bf16* dst[8];
  int off[9];
  int k;
};
void cat_nhwc_launch(const CatArgs&, bf16*, int, bool, hipStream_t);
void interleave2_launch(bf16*, bf16*, bf16*, int, int, bool, hipStream_t, bf16* = nullptr,
                        int ldh = 0);
void chan_remap_launch(const void*, void*, bool, bool, const int*, const int*, int, int, int, int,
                       hipStream_t, bool = false);
void dpn_merge_fwd_launch(const bf16*, const bf16*, int, int, int, int, bf16*, hipStream_t);
void dpn_merge_bwd_launch(const bf16*, const bf16*, int, int, int, int, bf16*, bf16*, hipStream_t);
void se_scale_bwd_launch(const bf16*, const bf16*, const float*, int, int, int, bf16*, float*,
                         hipStream_t);
void act_fwd_launch(const bf16*, size_t, int, bf16*, hipStream_t);
void act_bwd_launch(const bf16*, const bf16*, size_t, int, bf16*, hipStream_t);
void add_act_launch(const bf16*, const bf16*, size_t, int, bf16*, hipStream_t);
void weight_prep_launch(const float*, int, int, int, int, bf16*, bf16*, hipStream_t);
void weight_prep_multi_launch(const int64_t* desc, const int64_t* chunks, int nchunks,
                              hipStream_t st);
// dwconv.hip
void dw_fwd_launch(const bf16*, const float*, int, int, int, int, int, int, int, int, int, int, int,
                   bf16*, hipStream_t);
void dw_dgrad_launch(const bf16*, const float*, int, int, int, int, int, int, int, int, int, int,
                     int, bf16*, hipStream_t);
int dw_wgrad_partials(int, int, int);
bool dw_in_supported(int N, int H, int W, int C, int Ho, int Wo, int Co, int KH, int KW, int s,
                     int p, int act);
void dw_fwd_in_launch(const bf16* x, const float* wT, int N, int H, int W, int C, int Ho, int Wo,
                      int Co, int KH, int KW, int s, int p, const float* isc, const float* ish,
                      int act, bf16* y, hipStream_t st);
void dw_wgrad_in_launch(const bf16* x, const bf16* dy, int N, int H, int W, int C, int Ho, int Wo,
                        int Co, int KH, int KW, int s, int p, const float* isc, const float* ish,
                        int act, float* partial, int chunks, int accum, float* dw,
                        hipStream_t st);
bool dw_fwd_stats_launch(const bf16*, const float*, int, int, int, int, int, int, int, int, int,
                         int, int, bf16*, float*, int, hipStream_t);
bool dw_dgrad_bn_launch(const bf16*, const float*, int, int, int, int, int, int, int, int, int,
                        int, int, bf16*, const bf16*, const uint8_t*, const float*, int, float*,
                        int, hipStream_t);
void dw_wgrad_launch(const bf16*, const bf16*, int, int, int, int, int, int, int, int, int, int,
                     int, float*, int, int, float*, hipStream_t);
// conv_direct.hip
void direct_fwd_launch(const bf16*, const float*, const float*, int, int, int, int, int, int, int,
                       int, int, int, int, int, bf16*, hipStream_t);
void direct_dgrad_launch(const bf16*, const float*, int, int, int, int, int, int, int, int, int,
                         int, int, int, bf16*, hipStream_t);
int direct_wgrad_splits(int, int, int, int);
void direct_wgrad_launch(const bf16*, const bf16*, int, int, int, int, int, int, int, int, int,
                         int, int, int, int, float*, int, float*, hipStream_t);
// comm.cpp
void register_comm(py::module& m);
void set_deterministic_conv(bool on);
bool deterministic_conv();
}  // namespace pca

using at::Tensor;
using c10::optional;

namespace {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

template <typename T>
T* ptr(const Tensor& t) {
  return reinterpret_cast<T*>(t.data_ptr());
}
template <typename T>
T* optr(const optional<Tensor>& t) {
  return (t.has_value() && t->defined()) ? reinterpret_cast<T*>(t->data_ptr()) : nullptr;
}

void check_bf16(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == at::kBFloat16, name, " must be bf16");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous (NHWC)");
}
// NHWC bf16 [N,H,W,C] whose pixels may be strided rows (a channel slice of a wider concat slab:
// stride(3) = 1, stride(2) = ld >= C, outer strides dense over ld): returns ld (C when dense)
int rows_ld(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == at::kBFloat16, name, " must be bf16");
  const int C = t.size(-1);
  if (t.is_contiguous()) return C;
  TORCH_CHECK(t.dim() == 4 && t.stride(3) == 1 && t.stride(2) >= C && C % 8 == 0 &&
                  t.stride(1) == t.size(2) * t.stride(2) && t.stride(0) == t.size(1) * t.stride(1),
              name, " must be contiguous NHWC or a row-strided channel slice with C % 8 == 0");
  return (int)t.stride(2);
}

// rows_ld without the C % 8 condition: a BatchNorm input that is the channel prefix of a
// zero-padded conv output (rows of a multiple of 8), read by the vector kernels with a row stride
int rows_ld_bn(const Tensor& t, const char* name) {
  const int C = t.size(-1);
  if (t.is_contiguous() || C % 8 == 0) return rows_ld(t, name);
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kBFloat16, name, " must be bf16 on the GPU");
  TORCH_CHECK(t.dim() == 4 && t.stride(3) == 1 && t.stride(2) > C && t.stride(2) % 8 == 0 &&
                  t.stride(1) == t.size(2) * t.stride(2) && t.stride(0) == t.size(1) * t.stride(1),
              name, " must be contiguous NHWC or the channel prefix of rows padded to a multiple of 8");
  return (int)t.stride(2);
}

// dst <- src for NHWC [N,H,W,C] tensors of the same shape, either of them row-strided (a channel
// slice of a concat slab), C % 8 == 0
void copy_rows(const Tensor& src, const Tensor& dst) {
  const int ls = rows_ld(src, "src"), ld = rows_ld(dst, "dst");
  TORCH_CHECK(src.sizes() == dst.sizes() && src.dim() == 4, "copy_rows: shape mismatch");
  const int C = src.size(3);
  TORCH_CHECK(C % 8 == 0, "copy_rows needs C % 8 == 0");
  pca::copy_rows_launch(ptr<bf16>(src), ls, ptr<bf16>(dst), ld, (int)(src.numel() / C), C, cur_stream());
}

// dst <- src (NHWC rows, either row-strided) and src's per-channel centred sums (K = row 0) added
// into channels [acc_off, acc_off + C) of a [R][2][acc_ld] + K-row fp32 cache (zeroed by the
// caller before the first producer of a step)
static int acc_reduce_blocks(int M, int C, int R);
constexpr int kAccDepth = 16;
void bn_stats_copy(const Tensor& src, const Tensor& dst, const Tensor& acc, int acc_off, int acc_ld,
                   int R) {
  const int ls = rows_ld(src, "src"), ld = rows_ld(dst, "dst");
  TORCH_CHECK(src.sizes() == dst.sizes() && src.dim() == 4, "bn_stats_copy: shape mismatch");
  const int C = src.size(3);
  TORCH_CHECK(C % 8 == 0, "bn_stats_copy needs C % 8 == 0");
  TORCH_CHECK(acc.is_cuda() && acc.scalar_type() == at::kFloat && acc.is_contiguous(),
              "acc must be contiguous fp32 on the GPU");
  TORCH_CHECK(R >= 1 && acc_off >= 0 && acc_off + C <= acc_ld &&
                  acc.numel() >= (int64_t)R * 2 * acc_ld + acc_ld,
              "bn_stats_copy: acc must be [R][2][acc_ld] + K row");
  const int M = (int)(src.numel() / C);
  float* a = ptr<float>(acc);
  // (up to 4 x kAccDepth workgroups per shard row: the copy's bytes need the wider grid, and
  // each workgroup adds only 2 x C sums at its end)
  const int P = std::max(1, std::min({2 * pca::bn_row_blocks(M, C), 4 * kAccDepth * R, 1024}));
  pca::bn_stats_copy_launch(ptr<bf16>(src), ls, M, C, ptr<bf16>(dst), ld, a + acc_off, acc_ld, R,
                            P, a + (size_t)R * 2 * acc_ld + acc_off, cur_stream());
}

// t <- 0 on the current stream (the runtime's fill: a memset node under hipGraph capture)
void zero_(const Tensor& t) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "zero_: contiguous GPU tensor");
  TORCH_CHECK(hipMemsetAsync(t.data_ptr(), 0, t.numel() * t.element_size(), cur_stream()) ==
                  hipSuccess, "zero_: fill failed");
}

// dst <- src + add (NHWC rows; every operand dense or row-strided)
void add_rows(const Tensor& src, const Tensor& add, const Tensor& dst) {
  const int ls = rows_ld(src, "src"), la = rows_ld(add, "add"), ld = rows_ld(dst, "dst");
  TORCH_CHECK(src.sizes() == dst.sizes() && add.sizes() == dst.sizes() && src.dim() == 4,
              "add_rows: shape mismatch");
  const int C = src.size(3);
  TORCH_CHECK(C % 8 == 0, "add_rows needs C % 8 == 0");
  pca::copy_rows_launch(ptr<bf16>(src), ls, ptr<bf16>(dst), ld, (int)(src.numel() / C), C,
                        cur_stream(), ptr<bf16>(add), la);
}

// RAII: the row strides (0 = dense) the BatchNorm launches in scope read / write with
struct BnLdScope {
  pca::BnLd prev;
  explicit BnLdScope(int C, int y, int out, int dout = 0, int dx = 0, bool dx_acc = false)
      : prev(pca::bn_ld()) {
    pca::BnLd ld{y == C ? 0 : y, out == C ? 0 : out, dout == C ? 0 : dout, dx == C ? 0 : dx,
                 dx_acc ? 1 : 0};
    pca::set_bn_ld(ld);
  }
  ~BnLdScope() { pca::set_bn_ld(prev); }
};

void check_f32(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == at::kFloat, name, " must be fp32");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}

int out_dim(int in, int k, int s, int p) { return (in + 2 * p - k) / s + 1; }

// ------------------------------------------------------------------------------ conv
// Autotuning of the MFMA conv tile / split-K choice per geometry (cudnn.benchmark analogue,
// reference main.py:75). On by default; PCA_CONV_AUTOTUNE=0 or conv_autotune(False) disables.
static bool g_autotune = [] {
  const char* e = std::getenv("PCA_CONV_AUTOTUNE");
  return !(e && e[0] == '0');
}();

static bool stream_capturing(hipStream_t st) {
  hipStreamCaptureStatus s = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &s) != hipSuccess) return true;   // be conservative
  return s != hipStreamCaptureStatusNone;
}

// mean time (ms) of `reps` launches after one warm-up launch, HIP events on stream st
template <class F>
static float time_launches(F&& f, hipStream_t st, int reps) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  f();
  hipEventRecord(a, st);
  for (int i = 0; i < reps; ++i) f();
  hipEventRecord(b, st);
  hipEventSynchronize(b);
  float ms = 0.f;
  hipEventElapsedTime(&ms, a, b);
  hipEventDestroy(a);
  hipEventDestroy(b);
  return ms / reps;
}

// PCA_TUNE_LOG=1: print every autotune trial (tools/gpu sweeps read it from stderr)
static bool tune_log() {
  static const bool on = [] {
    const char* e = std::getenv("PCA_TUNE_LOG");
    return e && e[0] == '1';
  }();
  return on;
}

// time every candidate (cfg, split) of a conv geometry and record the fastest. `run` launches
// the conv once with the trial selection active, allocating its own scratch outputs.
template <class F>
static void autotune_conv(int kind, int N, int H, int W, int Cin, int Cout, int KH, int KW,
                          int stride, int pad, int groups, int Ho, int Wo, F&& run,
                          bool need_bn_fuse = false) {
  auto cands = pca::conv_tune_candidates(kind, N, H, W, Cin, Cout, KH, KW, stride, pad, groups,
                                         Ho, Wo);
  if (need_bn_fuse) {
    // a dgrad that should carry the producer BN's backward reduce: candidates that cannot fuse
    // it (the phased kernel) would leave a separate reduce + finalize + apply behind, which their
    // trial does not time — keep them only when no candidate can fuse
    std::vector<std::pair<int, int>> fusable;
    for (const auto& c : cands) {
      pca::conv_set_trial(c.first, c.second);
      if (pca::conv_dgrad_bn_rows(N, H, W, Cin, Cout, KH, KW, stride, pad, groups, Ho, Wo) > 0)
        fusable.push_back(c);
    }
    pca::conv_set_trial(-1, -1);
    if (!fusable.empty()) cands.swap(fusable);
  }
  if (cands.empty()) return;
  const hipStream_t st = cur_stream();
  float best = 1e30f;
  std::pair<int, int> pick = cands.front();
  for (const auto& c : cands) {
    pca::conv_set_trial(c.first, c.second);
    const float t = time_launches(run, st, 3);
    if (tune_log())
      fprintf(stderr, "[tune] %s N=%d H=%d W=%d Cin=%d Cout=%d k=%dx%d s=%d g=%d bnfuse=%d cfg=%d split=%d %.1f us\n",
              kind == 0 ? "fwd" : "dgrad", N, H, W, Cin, Cout, KH, KW, stride, groups, (int)need_bn_fuse,
              c.first, c.second, t * 1e3f);
    if (t < best) {
      best = t;
      pick = c;
    }
  }
  pca::conv_set_trial(-1, -1);
  pca::conv_record_tuned(kind, N, H, W, Cin, Cout, KH, KW, stride, pad, groups, Ho, Wo,
                         pick.first, pick.second);
}

// RAII: the BN partial-sum form of the producer launches in scope (0 = slab rows)
struct ShardScope {
  int prev;
  explicit ShardScope(int s) : prev(pca::stat_shards()) { pca::set_stat_shards(s); }
  ~ShardScope() { pca::set_stat_shards(prev); }
};

// zero-at-rest accumulator [R][NS][C] for the sharded BN partial sums
void check_acc(const Tensor& acc, int R, int NS, int C) {
  check_f32(acc, "stat accumulator");
  TORCH_CHECK(R >= 1 && acc.numel() >= (int64_t)R * NS * C, "stat accumulator must hold R*NS*C floats");
}

// RAII: the shift K (pilot mean) the producer launches in scope subtract from their BN sums
struct ShiftScope {
  const float* prev;
  explicit ShiftScope(const float* k) : prev(pca::stat_shift()) { pca::set_stat_shift(k); }
  ~ShiftScope() { pca::set_stat_shift(prev); }
};

// The BatchNorm+ReLU producing a conv's input applied on that conv's operand loads (the layer-1
// c64 forward and the halo wgrad): x is the PRE-BN y, xf the BN's aux [mean|istd|scale|shift][C].
bool conv_xf_supported(const Tensor& x, const Tensor& wb, int stride, int pad, int groups) {
  if (x.dim() != 4 || wb.dim() != 4) return false;
  const int N = x.size(0), H = x.size(1), W = x.size(2), Cin = x.size(3);
  const int Cout = wb.size(0), KH = wb.size(1), KW = wb.size(2);
  return pca::conv_c64_applicable(N, H, W, Cin, Cout, KH, KW, stride, pad, groups) &&
         pca::c64_version(-1) == 2 &&
         pca::wgrad_halo_ws_floats(N, H, W, Cin, Cout, KH, KW, stride, pad, groups) >= 0;
}

struct XfScope {
  bool fwd, on;
  XfScope(bool f, const float* xf, uint8_t* mask) : fwd(f), on(xf != nullptr) {
    if (!on) return;
    if (fwd) pca::conv_c64_set_xf(xf, mask);
    else pca::set_halo_xf(xf);
  }
  ~XfScope() {
    if (!on) return;
    if (fwd) pca::conv_c64_set_xf(nullptr, nullptr);
    else pca::set_halo_xf(nullptr);
  }
};

static const float* check_xf(const optional<Tensor>& xf, int C) {
  if (!(xf.has_value() && xf->defined())) return nullptr;
  check_f32(*xf, "xf (BN aux)");
  TORCH_CHECK(xf->numel() >= 4 * C, "xf: BN aux [mean|istd|scale|shift][C]");
  return ptr<float>(*xf) + 2 * C;
}

std::vector<Tensor> conv_fwd(const Tensor& x, const Tensor& wb, const optional<Tensor>& bias,
                             int stride, int pad, int groups, bool want_stats,
                             const optional<Tensor>& stat_acc, int acc_rows,
                             const optional<Tensor>& stat_shift,
                             const optional<Tensor>& xf = c10::nullopt,
                             const optional<Tensor>& xf_mask = c10::nullopt) {
  check_bf16(x, "x");
  check_bf16(wb, "weight");
  TORCH_CHECK(x.dim() == 4 && wb.dim() == 4, "conv_fwd expects x[N,H,W,C], w[Cout,KH,KW,Cin/G]");
  const int N = x.size(0), H = x.size(1), W = x.size(2), Cin = x.size(3);
  const int Cout = wb.size(0), KH = wb.size(1), KW = wb.size(2), Cg = wb.size(3);
  TORCH_CHECK(groups >= 1 && Cin % groups == 0 && Cout % groups == 0, "bad groups");
  TORCH_CHECK(Cg == Cin / groups, "weight Cin/G mismatch");
  TORCH_CHECK(Cg % 8 == 0 && (Cout / groups) % 8 == 0,
              "MFMA conv path needs Cin/G and Cout/G multiples of 8");
  const int Ho = out_dim(H, KH, stride, pad), Wo = out_dim(W, KW, stride, pad);
  TORCH_CHECK(Ho > 0 && Wo > 0, "empty conv output");
  const bool has_bias0 = bias.has_value() && bias->defined();
  const float* xfp = check_xf(xf, Cin);
  uint8_t* xmask = nullptr;
  if (xfp) {
    TORCH_CHECK(conv_xf_supported(x, wb, stride, pad, groups) && !has_bias0 && want_stats,
                "conv_fwd xf: only the layer-1 c64 forward (no bias, with statistics)");
    TORCH_CHECK(xf_mask.has_value() && xf_mask->defined() && xf_mask->is_contiguous() &&
                    xf_mask->scalar_type() == at::kByte && xf_mask->numel() * 8 == x.numel(),
                "xf_mask: one bit per input element");
    xmask = xf_mask->data_ptr<uint8_t>();
  }
  if (g_autotune && !stream_capturing(cur_stream()) &&
      pca::conv_needs_tune(0, N, H, W, Cin, Cout, KH, KW, stride, pad, groups, Ho, Wo, has_bias0)) {
    autotune_conv(0, N, H, W, Cin, Cout, KH, KW, stride, pad, groups, Ho, Wo, [&] {
      auto yt = at::empty({N, Ho, Wo, Cout}, x.options());
      Tensor stt, wst;
      if (want_stats) {
        const int gm = pca::conv_fwd_stat_rows(N, H, W, Cin, Cout, KH, KW, stride, pad, groups, Ho, Wo,
                                               has_bias0);
        stt = at::empty({gm, 2, Cout}, x.options().dtype(at::kFloat));
      }
      const int64_t n = pca::conv_fwd_ws_floats(N, H, W, Cin, Cout, KH, KW, stride, pad, groups,
                                                Ho, Wo, has_bias0);
      if (n > 0) wst = at::empty({n}, x.options().dtype(at::kFloat));
      pca::conv_fwd_launch(ptr<bf16>(x), ptr<bf16>(wb), optr<float>(bias), ptr<bf16>(yt),
                           want_stats ? ptr<float>(stt) : nullptr, N, H, W, Cin, Cout, KH, KW,
                           stride, pad, groups, Ho, Wo, cur_stream(),
                           n > 0 ? ptr<float>(wst) : nullptr);
    });
  }
  auto y = at::empty({N, Ho, Wo, Cout}, x.options());
  Tensor stats;
  const bool use_acc = want_stats && stat_acc.has_value() && stat_acc->defined();
  if (use_acc) {
    check_acc(*stat_acc, acc_rows, 2, Cout);
    stats = *stat_acc;
  } else if (want_stats) {
    const int gm = pca::conv_fwd_stat_rows(N, H, W, Cin, Cout, KH, KW, stride, pad, groups, Ho, Wo,
                                               has_bias0);
    stats = at::empty({gm, 2, Cout}, x.options().dtype(at::kFloat));
  }
  ShardScope shards(use_acc ? acc_rows : 0);
  const bool shift = want_stats && stat_shift.has_value() && stat_shift->defined();
  if (shift) {
    check_f32(*stat_shift, "stat_shift");
    TORCH_CHECK(stat_shift->numel() == Cout, "stat_shift [Cout]");
    if (use_acc)
      TORCH_CHECK(stats.numel() >= (int64_t)acc_rows * 2 * Cout + Cout,
                  "shifted accumulator needs its K row");
  }
  ShiftScope shift_scope(shift ? ptr<float>(*stat_shift) : nullptr);
  if (bias.has_value() && bias->defined()) {
    check_f32(*bias, "bias");
    TORCH_CHECK(bias->numel() == Cout, "bias size");
  }
  const bool has_bias = bias.has_value() && bias->defined();
  const int64_t wsn = pca::conv_fwd_ws_floats(N, H, W, Cin, Cout, KH, KW, stride, pad, groups, Ho,
                                              Wo, has_bias);
  Tensor ws;
  if (wsn > 0) ws = at::empty({wsn}, x.options().dtype(at::kFloat));
  XfScope xf_scope(true, xfp, xmask);
  pca::conv_fwd_launch(ptr<bf16>(x), ptr<bf16>(wb), optr<float>(bias), ptr<bf16>(y),
                       want_stats ? ptr<float>(stats) : nullptr, N, H, W, Cin, Cout, KH, KW,
                       stride, pad, groups, Ho, Wo, cur_stream(),
                       wsn > 0 ? ptr<float>(ws) : nullptr);
  return {y, stats};
}

// dgrad; with (bn_y, bn_mask, bn_aux) also the fused backward reduce of the BatchNorm+ReLU that
// produced the conv input: returns {dx, partial [rows][2][Cin]} (partial empty when the selected
// kernel cannot fuse it, e.g. the phased 256-row kernel; the caller then reduces separately)
std::vector<Tensor> conv_dgrad_impl(const Tensor& dy, const Tensor& wt, int H, int W, int stride,
                                    int pad, int groups, const optional<Tensor>& addend,
                                    const optional<Tensor>& bn_y, const optional<Tensor>& bn_mask,
                                    const optional<Tensor>& bn_aux,
                                    const optional<Tensor>& bn_acc = c10::nullopt,
                                    int acc_rows = 0,
                                    const optional<Tensor>& bn_y2 = c10::nullopt,
                                    const optional<Tensor>& bn_aux2 = c10::nullopt,
                                    bool addend_s2c = false) {
  check_bf16(dy, "dy");
  check_bf16(wt, "wt");
  const int N = dy.size(0), Ho = dy.size(1), Wo = dy.size(2), Cout = dy.size(3);
  const int Cin = wt.size(0), KH = wt.size(1), KW = wt.size(2), Cog = wt.size(3);
  TORCH_CHECK(Cog * groups == Cout, "wt Cout/G mismatch");
  TORCH_CHECK(Cog % 8 == 0 && (Cin / groups) % 8 == 0, "MFMA dgrad needs multiples of 8");
  TORCH_CHECK(out_dim(H, KH, stride, pad) == Ho && out_dim(W, KW, stride, pad) == Wo,
              "dgrad geometry mismatch");
  const bf16* add = nullptr;
  Tensor add_full;   // a compact stride-2 addend expanded, where the selected kernel needs it whole
  if (addend.has_value() && addend->defined()) {
    check_bf16(*addend, "addend");
    if (addend_s2c) {
      // [N][H/2][W/2][Cin]: the dX of a 1x1 stride-2 conv of the same input (even-even pixels)
      TORCH_CHECK(stride == 2 && H % 2 == 0 && W % 2 == 0 && addend->is_contiguous() &&
                      addend->numel() == (int64_t)N * (H / 2) * (W / 2) * Cin,
                  "compact stride-2 addend must be [N][H/2][W/2][Cin]");
      // (expanded lazily below: for tuning trials, or when the selected kernel needs it whole)
    } else {
      TORCH_CHECK(addend->numel() == (int64_t)N * H * W * Cin && addend->is_contiguous(),
                  "addend must match dx (NHWC)");
      add = ptr<bf16>(*addend);
    }
  }
  const bool want_bn = bn_y.has_value() && bn_y->defined();
  int bn_ldy = 0;   // y a row-strided channel slice (a DenseNet BatchNorm's slab suffix)
  if (want_bn) {
    if (bn_y->is_contiguous()) {
      check_bf16(*bn_y, "bn_y");
    } else {
      TORCH_CHECK(bn_y->dim() == 4 && bn_y->size(-1) == Cin, "bn_y must be NHWC [N,H,W,Cin]");
      bn_ldy = rows_ld(*bn_y, "bn_y");
      TORCH_CHECK(!(bn_y2.has_value() && bn_y2->defined()), "row-strided bn_y: single BN only");
    }
    TORCH_CHECK(bn_y->numel() == (int64_t)N * H * W * Cin, "bn_y must match dx (NHWC)");
    TORCH_CHECK(bn_mask.has_value() && bn_mask->defined() && bn_mask->is_contiguous() &&
                    bn_mask->scalar_type() == at::kByte && bn_mask->numel() * 8 == bn_y->numel(),
                "bn_mask: one bit per element");
    TORCH_CHECK(bn_aux.has_value() && bn_aux->defined(), "bn_aux required");
    check_f32(*bn_aux, "bn_aux");
    TORCH_CHECK(bn_aux->numel() >= 2 * Cin, "bn_aux [mean|istd|...][C]");
  }
  // dual BN (projection-shortcut block tail): third sum dz * xhat2, accumulator mode only
  const bool dual = want_bn && bn_y2.has_value() && bn_y2->defined() && bn_acc.has_value() &&
                    bn_acc->defined();
  if (dual) {
    check_bf16(*bn_y2, "bn_y2");
    TORCH_CHECK(bn_y2->numel() == bn_y->numel(), "bn_y2 must match dx (NHWC)");
    TORCH_CHECK(bn_aux2.has_value() && bn_aux2->defined(), "bn_aux2 required");
    check_f32(*bn_aux2, "bn_aux2");
    TORCH_CHECK(bn_aux2->numel() >= 2 * Cin, "bn_aux2 [mean|istd|...][C]");
  }
  const int NS = dual ? 3 : 2;
  struct LdyScope {
    bool on;
    explicit LdyScope(int ld) : on(ld != 0) {
      if (on) pca::conv_set_bn_ldy(ld);
    }
    ~LdyScope() {
      if (on) pca::conv_set_bn_ldy(0);
    }
  } ldy_scope(bn_ldy);
  struct DualScope {
    bool on;
    DualScope(bool d, const bf16* y2, const float* a2) : on(d) {
      if (on) pca::conv_set_bn_dual(y2, a2);
    }
    ~DualScope() {
      if (on) pca::conv_set_bn_dual(nullptr, nullptr);
    }
  } dual_scope(dual, dual ? ptr<bf16>(*bn_y2) : nullptr, dual ? ptr<float>(*bn_aux2) : nullptr);
  auto expand_s2c = [&]() {
    if (!add_full.defined()) {
      add_full = at::empty({N, H, W, Cin}, dy.options());
      pca::s2c_expand_launch(ptr<bf16>(*addend), ptr<bf16>(add_full), N, H / 2, W / 2, Cin,
                             cur_stream());
    }
    return ptr<bf16>(add_full);
  };
  const bool s2c = addend_s2c && addend.has_value() && addend->defined();
  if (g_autotune && !stream_capturing(cur_stream()) &&
      pca::conv_needs_tune(1, N, H, W, Cin, Cout, KH, KW, stride, pad, groups, Ho, Wo, false)) {
    if (s2c) add = expand_s2c();   // (trials run with the whole addend)
    // trials run the call as issued: with the fused BN-backward reduce when it is requested
    // (its epilogue traffic decides between candidates that tie on the plain dgrad)
    autotune_conv(1, N, H, W, Cin, Cout, KH, KW, stride, pad, groups, Ho, Wo, [&] {
      auto dxt = at::empty({N, H, W, Cin}, dy.options());
      Tensor wst, pt;
      const int64_t n = pca::conv_dgrad_ws_floats(N, H, W, Cin, Cout, KH, KW, stride, pad, groups,
                                                  Ho, Wo);
      if (n > 0) wst = at::empty({n}, dy.options().dtype(at::kFloat));
      const int r = want_bn ? pca::conv_dgrad_bn_rows(N, H, W, Cin, Cout, KH, KW, stride, pad,
                                                      groups, Ho, Wo)
                            : 0;
      if (r > 0) pt = at::empty({r, NS, Cin}, dy.options().dtype(at::kFloat));
      pca::conv_dgrad_launch(ptr<bf16>(dy), ptr<bf16>(wt), ptr<bf16>(dxt), N, H, W, Cin, Cout, KH,
                             KW, stride, pad, groups, Ho, Wo, cur_stream(), add,
                             n > 0 ? ptr<float>(wst) : nullptr,
                             r > 0 ? ptr<bf16>(*bn_y) : nullptr,
                             r > 0 ? bn_mask->data_ptr<uint8_t>() : nullptr,
                             r > 0 ? ptr<float>(*bn_aux) : nullptr, r > 0 ? ptr<float>(pt) : nullptr);
    }, want_bn);
  }
  auto dx = at::empty({N, H, W, Cin}, dy.options());
  const int64_t wsn = pca::conv_dgrad_ws_floats(N, H, W, Cin, Cout, KH, KW, stride, pad, groups,
                                                Ho, Wo);
  Tensor ws;
  if (wsn > 0) ws = at::empty({wsn}, dy.options().dtype(at::kFloat));
  Tensor part;
  const int rows = want_bn ? pca::conv_dgrad_bn_rows(N, H, W, Cin, Cout, KH, KW, stride, pad,
                                                     groups, Ho, Wo)
                           : 0;
  const bool use_acc = rows > 0 && bn_acc.has_value() && bn_acc->defined();
  if (use_acc) {
    check_acc(*bn_acc, acc_rows, NS, Cin);
    part = *bn_acc;
  } else if (rows > 0) {
    part = at::empty({rows, 2, Cin}, dy.options().dtype(at::kFloat));
  }
  ShardScope shards(use_acc ? acc_rows : 0);
  // the kernel the (tuned) selection runs adds a compact addend itself when it can
  struct S2cScope {
    bool on;
    explicit S2cScope(bool o) : on(o) {
      if (on) pca::conv_set_addend_s2c(1);
    }
    ~S2cScope() {
      if (on) pca::conv_set_addend_s2c(0);
    }
  } s2c_scope(s2c && pca::conv_dgrad_s2c_ok(N, H, W, Cin, Cout, KH, KW, stride, pad, groups, Ho,
                                            Wo));
  if (s2c) add = s2c_scope.on ? ptr<bf16>(*addend) : expand_s2c();
  pca::conv_dgrad_launch(ptr<bf16>(dy), ptr<bf16>(wt), ptr<bf16>(dx), N, H, W, Cin, Cout, KH, KW,
                         stride, pad, groups, Ho, Wo, cur_stream(), add,
                         wsn > 0 ? ptr<float>(ws) : nullptr,
                         rows > 0 ? ptr<bf16>(*bn_y) : nullptr,
                         rows > 0 ? bn_mask->data_ptr<uint8_t>() : nullptr,
                         rows > 0 ? ptr<float>(*bn_aux) : nullptr,
                         rows > 0 ? ptr<float>(part) : nullptr);
  if (rows == 0) part = at::empty({0}, dy.options().dtype(at::kFloat));
  return {dx, part};
}

Tensor conv_dgrad(const Tensor& dy, const Tensor& wt, int H, int W, int stride, int pad,
                  int groups, const optional<Tensor>& addend, bool addend_s2c) {
  return conv_dgrad_impl(dy, wt, H, W, stride, pad, groups, addend, c10::nullopt, c10::nullopt,
                         c10::nullopt, c10::nullopt, 0, c10::nullopt, c10::nullopt, addend_s2c)[0];
}

// dw: fp32 [Cout, KH, KW, Cin/G] (zeroed here)
// wgrad autotune under the piggybacked reductions (PCA_TUNE_PIGGY=1): a candidate's slab reduce
// is charged at this fraction of its standalone launch
constexpr float kPiggyWeight = 0.5f;
static bool tune_piggy() {
  static const bool on = [] {
    const char* e = getenv("PCA_TUNE_PIGGY");
    return e && e[0] == '1';
  }();
  return on;
}

// slab workspaces of deferred reductions: alive until wgrad_flush launched their reduce
static std::vector<Tensor> g_deferred_ws;

// defer: a split-K slab reduction is recorded (one batched launch at wgrad_flush) instead of
// launched; only for `out` = the gradient buffer the caller flushes before anyone reads it
Tensor conv_wgrad(const Tensor& x, const Tensor& dy, int KH, int KW, int stride, int pad,
                  int groups, const optional<Tensor>& out, bool defer,
                  const optional<Tensor>& xf = c10::nullopt) {
  check_bf16(x, "x");
  check_bf16(dy, "dy");
  const int N = x.size(0), H = x.size(1), W = x.size(2), Cin = x.size(3);
  const float* xfp = check_xf(xf, Cin);
  if (xfp)
    TORCH_CHECK(pca::wgrad_halo_ws_floats(N, H, W, Cin, dy.size(3), KH, KW, stride, pad, groups) >= 0,
                "conv_wgrad xf: only the halo (3x3 / stride-1) wgrad transforms its X operand");
  const int Ho = dy.size(1), Wo = dy.size(2), Cout = dy.size(3);
  TORCH_CHECK(dy.size(0) == N, "batch mismatch");
  TORCH_CHECK(out_dim(H, KH, stride, pad) == Ho && out_dim(W, KW, stride, pad) == Wo,
              "wgrad geometry mismatch");
  TORCH_CHECK((Cin / groups) % 8 == 0 && (Cout / groups) % 8 == 0, "MFMA wgrad needs multiples of 8");
  // fp32 atomics accumulate into `out` (a .grad buffer in physical order) when given.
  Tensor dw;
  if (out.has_value() && out->defined()) {
    check_f32(*out, "dw out");
    TORCH_CHECK(out->dim() == 4 && out->size(0) == Cout && out->size(1) == KH &&
                    out->size(2) == KW && out->size(3) == Cin / groups,
                "dw out shape");
    dw = *out;
  } else {
    // (zeroed by the runtime's fill on this stream, not an at::native kernel)
    dw = at::empty({Cout, KH, KW, Cin / groups}, x.options().dtype(at::kFloat));
    TORCH_CHECK(hipMemsetAsync(dw.data_ptr(), 0, dw.numel() * sizeof(float), cur_stream()) ==
                    hipSuccess, "conv_wgrad: zero fill failed");
  }
  if (g_autotune && !stream_capturing(cur_stream()) &&
      pca::wgrad_needs_tune(N, H, W, Cin, Cout, KH, KW, stride, pad, groups)) {
    // trials accumulate into a scratch gradient (never the real one)
    auto dwt = at::empty({Cout, KH, KW, Cin / groups}, x.options().dtype(at::kFloat));
    auto cands = pca::wgrad_tune_candidates(N, H, W, Cin, Cout, KH, KW, stride, pad, groups);
    float best = 1e30f;
    std::pair<int, int> pick = cands.front();
    for (const auto& c : cands) {
      pca::wgrad_set_trial(c.first, c.second);
      const int64_t n = pca::conv_wgrad_ws_floats(N, H, W, Cin, Cout, KH, KW, stride, pad, groups, Ho, Wo);
      Tensor wst;
      if (n > 0) wst = at::empty({n}, x.options().dtype(at::kFloat));
      float t = time_launches([&] {
        pca::conv_wgrad_launch(ptr<bf16>(x), ptr<bf16>(dy), ptr<float>(dwt),
                               n > 0 ? ptr<float>(wst) : nullptr, N, H, W, Cin, Cout, KH, KW,
                               stride, pad, groups, Ho, Wo, cur_stream());
      }, cur_stream(), 3);
      if (n > 0 && tune_piggy()) {
        // the production step runs this candidate's slab reduce inside the next BatchNorm-backward
        // launch (ops/functional.py PCA_WGRAD_DEFER=piggy), beside a pass it is independent of:
        // charge the reduce at kPiggyWeight of its standalone time
        const int keep = pca::wgrad_deferred_count();
        const float tw = time_launches([&] {
          pca::wgrad_defer_scope(true);
          pca::conv_wgrad_launch(ptr<bf16>(x), ptr<bf16>(dy), ptr<float>(dwt), ptr<float>(wst), N,
                                 H, W, Cin, Cout, KH, KW, stride, pad, groups, Ho, Wo, cur_stream());
          pca::wgrad_defer_scope(false);
          pca::wgrad_truncate_pending(keep);
        }, cur_stream(), 3);
        if (tw < t) t = tw + kPiggyWeight * (t - tw);
      }
      if (tune_log())
        fprintf(stderr, "[tune] wgrad N=%d H=%d W=%d Cin=%d Cout=%d k=%dx%d s=%d g=%d cfg=%d split=%d %.1f us\n",
                N, H, W, Cin, Cout, KH, KW, stride, groups, c.first, c.second, t * 1e3f);
      if (t < best) {
        best = t;
        pick = c;
      }
    }
    pca::wgrad_set_trial(-1, -1);
    pca::wgrad_record_tuned(N, H, W, Cin, Cout, KH, KW, stride, pad, groups, pick.first, pick.second);
  }
  // (after tuning: the trials time the plain selection; the X transform forces a halo config)
  XfScope xf_scope(false, xfp, nullptr);
  // slab workspace of the wide kernel (partial tiles, reduced into dw in a fixed order)
  const int64_t wsn = pca::conv_wgrad_ws_floats(N, H, W, Cin, Cout, KH, KW, stride, pad, groups, Ho, Wo);
  Tensor ws;
  if (wsn > 0) ws = at::empty({wsn}, x.options().dtype(at::kFloat));
  defer = defer && wsn > 0 && out.has_value() && out->defined();
  const int pend = pca::wgrad_deferred_count();
  if (defer) pca::wgrad_defer_scope(true);
  pca::conv_wgrad_launch(ptr<bf16>(x), ptr<bf16>(dy), ptr<float>(dw), wsn > 0 ? ptr<float>(ws) : nullptr,
                         N, H, W, Cin, Cout, KH, KW, stride, pad, groups, Ho, Wo, cur_stream());
  if (defer) {
    pca::wgrad_defer_scope(false);
    if (pca::wgrad_deferred_count() > pend) g_deferred_ws.push_back(ws);
  }
  return dw;
}

// pending wgrad slab reductions ride along in the next fused BatchNorm-backward launch
void wgrad_piggy(bool on) { pca::set_wgrad_piggy(on); }

// every deferred slab reduction in one launch (per 20) on the current stream; returns how many
int wgrad_flush() {
  const int n = pca::wgrad_deferred_count();
  if (n) pca::wgrad_flush_launch(cur_stream());
  g_deferred_ws.clear();   // (stream-ordered: later reuse of the slabs runs after the reduce)
  return n;
}

// w fp32 [Cout, KH, KW, Cin/G] contiguous -> (bf16 same layout, bf16 [Cin, KH, KW, Cout/G])
std::vector<Tensor> weight_prep(const Tensor& w, int groups, bool want_t) {
  check_f32(w, "w");
  const int Cout = w.size(0), KH = w.size(1), KW = w.size(2), Cg = w.size(3);
  auto wb = at::empty(w.sizes(), w.options().dtype(at::kBFloat16));
  Tensor wt;
  if (want_t) wt = at::empty({Cg * groups, KH, KW, Cout / groups}, wb.options());
  pca::weight_prep_launch(ptr<float>(w), groups, Cout / groups, KH * KW, Cg, ptr<bf16>(wb),
                          want_t ? ptr<bf16>(wt) : nullptr, cur_stream());
  return {wb, wt};
}

// batched weight_prep over a descriptor table (see misc.hip weight_prep_multi_kernel)
void weight_prep_multi(const Tensor& desc, const Tensor& chunks) {
  TORCH_CHECK(desc.is_cuda() && desc.scalar_type() == at::kLong && desc.dim() == 2 &&
                  desc.size(1) == 8, "desc must be a [n,8] int64 GPU tensor");
  TORCH_CHECK(chunks.is_cuda() && chunks.scalar_type() == at::kLong && chunks.dim() == 2 &&
                  chunks.size(1) == 4, "chunks must be a [m,4] int64 GPU tensor");
  pca::weight_prep_multi_launch(desc.data_ptr<int64_t>(), chunks.data_ptr<int64_t>(),
                                (int)chunks.size(0), cur_stream());
}

// ------------------------------------------------------------------------------- BN
Tensor bn_stats(const Tensor& x) {
  const int ldx = rows_ld(x, "x");
  const int C = x.size(-1);
  const int M = x.numel() / C;
  const int P = pca::bn_row_blocks(M, C);
  auto partial = at::empty({P, 2, C}, x.options().dtype(at::kFloat));
  BnLdScope lds(C, ldx, C);
  pca::bn_stats_launch(ptr<bf16>(x), M, C, ptr<float>(partial), P, cur_stream());
  return partial;
}

// centered form (robust variance): sums of x - K with K = x's first row, K returned alongside
// -> {partial [P][2][C], K [C]} (the finalize's kin)
std::vector<Tensor> bn_stats_centered(const Tensor& x) {
  const int ldx = rows_ld(x, "x");
  const int C = x.size(-1);
  BnLdScope lds(C, ldx, C);
  const int M = x.numel() / C;
  const int P = pca::bn_row_blocks(M, C);
  auto buf = at::empty({(int64_t)P * 2 * C + C}, x.options().dtype(at::kFloat));
  float* k = ptr<float>(buf) + (size_t)P * 2 * C;
  pca::bn_stats_launch(ptr<bf16>(x), M, C, ptr<float>(buf), P, cur_stream(), k);
  return {buf.narrow(0, 0, (int64_t)P * 2 * C).view({P, 2, C}), buf.narrow(0, (int64_t)P * 2 * C, C)};
}

// Reduce-kernel grid when it adds into an R-row sharded accumulator: at most kAccDepth
// workgroups per shard row, so the same-address fp32 atomics stay shallow (deeper queues — 1024
// blocks into 16 rows — cost more than the finalize launch they remove).

static int acc_reduce_blocks(int M, int C, int R) {
  return std::max(1, std::min(pca::bn_row_blocks(M, C), kAccDepth * R));
}
// tensors up to this size use the accumulator form for a separate statistics / backward-reduce
// pass (small per-GPU batches: EfficientNet-B0 at bs128), larger ones keep slab rows + finalize
// largest tensor (elements) whose statistics / backward sums a separate pass adds into an
// accumulator (PCA_BN_ACC_MAX_ELEMS; larger ones take the slab + finalize path)
static int64_t acc_max_elems() {
  static const int64_t v = [] {
    const char* e = getenv("PCA_BN_ACC_MAX_ELEMS");
    return e ? (int64_t)atoll(e) : (int64_t)0;   // measured: the slab path is faster
  }();
  return v;
}

// per-channel (sum, sumsq) of a bare tensor added into a zeroed sharded accumulator [R][2][C];
// returns false (nothing launched) when the tensor is too large for the accumulator form
bool bn_stats_acc(const Tensor& x, const Tensor& acc, int R) {
  const int ldx = rows_ld(x, "x");
  const int C = x.size(-1);
  BnLdScope lds(C, ldx, C);
  const int M = x.numel() / C;
  check_acc(acc, R, 2, C);
  if ((int64_t)M * C > acc_max_elems()) return false;
  ShardScope shards(R);
  pca::bn_stats_launch(ptr<bf16>(x), M, C, ptr<float>(acc), acc_reduce_blocks(M, C, R), cur_stream());
  return true;
}

// conv bias gradient: per-channel sum of dY [.., C] (bf16), added into `accum` (fp32 [C], e.g.
// the bias's gradient-arena view) when given, else returned as a new tensor
Tensor bias_grad(const Tensor& dy, const optional<Tensor>& accum) {
  check_bf16(dy, "dy");
  const int C = dy.size(-1);
  const int M = dy.numel() / C;
  const int P = pca::bn_row_blocks(M, C);
  auto partial = at::empty({P, 2, C}, dy.options().dtype(at::kFloat));
  pca::bn_stats_launch(ptr<bf16>(dy), M, C, ptr<float>(partial), P, cur_stream());
  const bool acc = accum.has_value() && accum->defined();
  Tensor db = acc ? *accum : at::empty({C}, dy.options().dtype(at::kFloat));
  if (acc)
    TORCH_CHECK(db.scalar_type() == at::kFloat && db.is_contiguous() && db.numel() == C,
                "bias_grad: accum must be contiguous fp32 [C]");
  pca::bias_grad_fold_launch(ptr<float>(partial), P, C, acc ? 1 : 0, ptr<float>(db), cur_stream());
  return db;
}

// partial [R, 2, C] (or undefined in eval) -> aux [4, C] = {mean, invstd, scale, shift}
// kin: the shift K the producer subtracted from its sums (pilot / centred stats), or none;
// pilot_out: receives the batch mean (may be kin itself)
Tensor bn_finalize(const optional<Tensor>& partial, double count, const optional<Tensor>& gamma,
                   const optional<Tensor>& beta, const Tensor& rmean, const Tensor& rvar,
                   const optional<Tensor>& nbt, double momentum, double eps, bool training,
                   bool update_running, const optional<Tensor>& kin,
                   const optional<Tensor>& pilot_out, const optional<Tensor>& zero) {
  const int C = rmean.numel();
  auto aux = at::empty({4, C}, rmean.options());
  const float* stat = nullptr;
  int R = 0;
  Tensor folded;
  int ld = C;
  if (training) {
    TORCH_CHECK(partial.has_value(), "training BN needs statistics");
    const Tensor& p = *partial;
    TORCH_CHECK(p.is_cuda() && p.scalar_type() == at::kFloat, "partial must be fp32 on the GPU");
    TORCH_CHECK(p.size(-1) == C, "stat channel mismatch");
    if (!p.is_contiguous()) {
      // the channel prefix of zero-padded statistics [R][2][ld] (a padded conv's slab rows)
      TORCH_CHECK(p.dim() == 3 && p.size(1) == 2 && p.stride(2) == 1 && p.stride(1) >= C &&
                      p.stride(0) == 2 * p.stride(1),
                  "partial: contiguous, or the channel prefix of [R][2][ld] rows");
      ld = (int)p.stride(1);
    }
    R = p.size(0);
    stat = p.data_ptr<float>();
    if (R > 1024) {  // finalize folds up to 1024 partial rows in one pass
      folded = at::empty({64, 2, ld}, p.options());
      R = pca::colsum_launch(stat, R, 2 * ld, ptr<float>(folded), cur_stream());
      stat = ptr<float>(folded);
    }
  }
  if (kin.has_value() && kin->defined()) {
    check_f32(*kin, "kin");
    TORCH_CHECK(kin->numel() == C, "kin [C]");
  }
  if (pilot_out.has_value() && pilot_out->defined()) {
    check_f32(*pilot_out, "pilot_out");
    TORCH_CHECK(pilot_out->numel() == C, "pilot_out [C]");
  }
  pca::bn_finalize_launch(stat, R, C, count, optr<float>(gamma), optr<float>(beta),
                          ptr<float>(rmean), ptr<float>(rvar), optr<int64_t>(nbt), (float)momentum,
                          (float)eps, training ? 1 : 0, update_running ? 1 : 0, ptr<float>(aux),
                          cur_stream(), training ? optr<float>(kin) : nullptr,
                          training ? optr<float>(pilot_out) : nullptr, optr<float>(zero),
                          (zero.has_value() && zero->defined()) ? (int)zero->numel() : 0, ld);
  return aux;
}

// out: optional destination (a row-strided channel slice of a concat slab), else a new tensor
// (a strided odd-width y goes to the vector kernels only without residual / second BN; with
// them it is made dense first)
static bool bn_odd_strided(const Tensor& y) { return !y.is_contiguous() && y.size(-1) % 8 != 0; }

std::vector<Tensor> bn_apply_impl(const Tensor& y, const Tensor& aux, const optional<Tensor>& res,
                                  const optional<Tensor>& y2, const optional<Tensor>& aux2, int act,
                                  bool want_mask, const optional<Tensor>& out_opt);
std::vector<Tensor> bn_apply(const Tensor& y, const Tensor& aux, const optional<Tensor>& res,
                             const optional<Tensor>& y2, const optional<Tensor>& aux2, int act,
                             bool want_mask, const optional<Tensor>& out_opt) {
  const bool extra = (res.has_value() && res->defined()) || (y2.has_value() && y2->defined()) ||
                     (out_opt.has_value() && out_opt->defined());
  if (bn_odd_strided(y) && extra) return bn_apply_impl(y.contiguous(), aux, res, y2, aux2, act, want_mask, out_opt);
  return bn_apply_impl(y, aux, res, y2, aux2, act, want_mask, out_opt);
}

std::vector<Tensor> bn_apply_impl(const Tensor& y, const Tensor& aux, const optional<Tensor>& res,
                                  const optional<Tensor>& y2, const optional<Tensor>& aux2, int act,
                                  bool want_mask, const optional<Tensor>& out_opt) {
  const int ldy = rows_ld_bn(y, "y");
  const int C = y.size(-1);
  TORCH_CHECK(aux.size(1) == C, "aux channel mismatch");
  if (res.has_value() && res->defined()) {
    check_bf16(*res, "res");
    TORCH_CHECK(res->sizes() == y.sizes(), "residual shape mismatch");
  }
  if (y2.has_value() && y2->defined()) {
    check_bf16(*y2, "y2");
    TORCH_CHECK(y2->sizes() == y.sizes(), "second BN input shape mismatch");
  }
  Tensor out;
  int ldo = C;
  if (out_opt.has_value() && out_opt->defined()) {
    out = *out_opt;
    ldo = rows_ld(out, "out");
    TORCH_CHECK(out.sizes() == y.sizes(), "out shape mismatch");
  } else {
    out = at::empty(y.sizes(), y.options());
  }
  // ReLU sign bits (1 byte / 8 channels) for the backward, when C allows the 8-wide path
  Tensor mask;
  if (want_mask && act == 1 && C % 8 == 0)
    mask = at::empty({(int64_t)(y.numel() / 8)}, y.options().dtype(at::kByte));
  BnLdScope lds(C, ldy, ldo);
  pca::bn_apply_launch(ptr<bf16>(y), ptr<float>(aux), C, y.numel(), optr<bf16>(res), optr<bf16>(y2),
                       optr<float>(aux2), act, ptr<bf16>(out),
                       mask.defined() ? mask.data_ptr<uint8_t>() : nullptr, cur_stream());
  return {out, mask};
}

// Training BN(+act, +residual | +second BN) whose batch sums sit in sharded accumulators (the
// producing convs added them): finalize folded into the apply kernel. `zero` (this BN's backward
// accumulator, or none) is cleared by the kernel's block 0. Returns {out, mask, aux, aux2}.
// Falls back to finalize + apply (+ memset of `zero`) where the fused row kernel does not apply.
std::vector<Tensor> bn_apply_acc(const Tensor& y, const Tensor& acc, int R, double count,
                                 const optional<Tensor>& gamma, const optional<Tensor>& beta,
                                 const Tensor& rmean, const Tensor& rvar,
                                 const optional<Tensor>& nbt, double momentum, double eps,
                                 const optional<Tensor>& res, const optional<Tensor>& y2,
                                 const optional<Tensor>& acc2, int R2,
                                 const optional<Tensor>& gamma2, const optional<Tensor>& beta2,
                                 const optional<Tensor>& rmean2, const optional<Tensor>& rvar2,
                                 const optional<Tensor>& nbt2, double momentum2, double eps2,
                                 int act, bool want_mask, const optional<Tensor>& zero,
                                 bool shifted, const optional<Tensor>& pilot, bool shifted2,
                                 const optional<Tensor>& pilot2, const optional<Tensor>& out_opt,
                                 int acc_off, int acc_ld) {
  const int ldy = rows_ld(y, "y");
  const int C = y.size(-1);
  const int M = y.numel() / C;
  if (acc_ld > 0) {
    // channels [acc_off, acc_off + C) of a wider [R][2][acc_ld] accumulator + its K row (a
    // DenseNet slab's statistics cache): fused form only, single BN
    check_f32(acc, "acc");
    TORCH_CHECK(acc_off >= 0 && acc_off + C <= acc_ld && shifted &&
                    acc.numel() >= (int64_t)R * 2 * acc_ld + acc_ld,
                "acc view: [R][2][acc_ld] + K row, channels [acc_off, acc_off + C)");
    TORCH_CHECK(!(y2.has_value() && y2->defined()), "acc view: single BN only");
  } else {
    check_acc(acc, R, 2, C);
  }
  // shifted accumulators carry the producers' K row after the sums; the pilots get the means
  TORCH_CHECK(acc_ld > 0 || !shifted || acc.numel() >= (int64_t)R * 2 * C + C,
              "shifted accumulator needs its K row");
  for (const auto* pt : {&pilot, &pilot2})
    if (pt->has_value() && (*pt)->defined()) {
      check_f32(**pt, "pilot");
      TORCH_CHECK((*pt)->numel() == C, "pilot [C]");
    }
  const bool dual = y2.has_value() && y2->defined();
  if (dual) {
    check_bf16(*y2, "y2");
    TORCH_CHECK(y2->sizes() == y.sizes(), "second BN input shape mismatch");
    TORCH_CHECK(acc2.has_value() && acc2->defined() && rmean2.has_value() && rvar2.has_value(),
                "dual BN needs the second accumulator and running stats");
    check_acc(*acc2, R2, 2, C);
    TORCH_CHECK(!shifted2 || acc2->numel() >= (int64_t)R2 * 2 * C + C,
                "shifted accumulator needs its K row");
  }
  if (res.has_value() && res->defined()) {
    check_bf16(*res, "res");
    TORCH_CHECK(res->sizes() == y.sizes(), "residual shape mismatch");
  }
  auto fopt = y.options().dtype(at::kFloat);
  Tensor out;
  int ldo = C;
  if (out_opt.has_value() && out_opt->defined()) {
    out = *out_opt;
    ldo = rows_ld(out, "out");
    TORCH_CHECK(out.sizes() == y.sizes(), "out shape mismatch");
  } else {
    out = at::empty(y.sizes(), y.options());
  }
  Tensor mask;
  if (want_mask && act == 1 && C % 8 == 0)
    mask = at::empty({(int64_t)(y.numel() / 8)}, y.options().dtype(at::kByte));
  auto aux = at::empty({4, C}, fopt);
  BnLdScope lds(C, ldy, ldo);
  const float* k1 = shifted ? ptr<float>(acc) + (size_t)R * 2 * C : nullptr;
  const float* k2 = (dual && shifted2) ? ptr<float>(*acc2) + (size_t)R2 * 2 * C : nullptr;
  Tensor aux2;
  if (dual) aux2 = at::empty({4, C}, fopt);
  const auto st = cur_stream();
  const bool has_zero = zero.has_value() && zero->defined();
  if (has_zero) check_f32(*zero, "zero");
  const bool fused = pca::bn_apply_acc_launch(
      ptr<bf16>(y), C, M, (float)count, ptr<float>(acc), R, optr<float>(gamma), optr<float>(beta),
      ptr<float>(rmean), ptr<float>(rvar), optr<int64_t>(nbt), (float)momentum, (float)eps,
      ptr<float>(aux), dual ? ptr<float>(*acc2) : nullptr, R2, optr<float>(gamma2),
      optr<float>(beta2), optr<float>(rmean2), optr<float>(rvar2), optr<int64_t>(nbt2),
      (float)momentum2, (float)eps2, dual ? ptr<float>(aux2) : nullptr, optr<bf16>(res),
      optr<bf16>(y2), act, ptr<bf16>(out), mask.defined() ? mask.data_ptr<uint8_t>() : nullptr,
      has_zero ? ptr<float>(*zero) : nullptr, has_zero ? (int)zero->numel() : 0, st, shifted,
      optr<float>(pilot), shifted2, optr<float>(pilot2), acc_off, acc_ld);
  TORCH_CHECK(fused || acc_ld == 0, "acc view needs the fused row kernels");
  if (!fused) {
    pca::bn_finalize_launch(ptr<float>(acc), R, C, count, optr<float>(gamma), optr<float>(beta),
                            ptr<float>(rmean), ptr<float>(rvar), optr<int64_t>(nbt),
                            (float)momentum, (float)eps, 1, 1, ptr<float>(aux), st, k1,
                            optr<float>(pilot));
    if (dual)
      pca::bn_finalize_launch(ptr<float>(*acc2), R2, C, count, optr<float>(gamma2),
                              optr<float>(beta2), ptr<float>(*rmean2), ptr<float>(*rvar2),
                              optr<int64_t>(nbt2), (float)momentum2, (float)eps2, 1, 1,
                              ptr<float>(aux2), st, k2, optr<float>(pilot2));
    if (has_zero) zero->zero_();
    pca::bn_apply_launch(ptr<bf16>(y), ptr<float>(aux), C, y.numel(), optr<bf16>(res),
                         optr<bf16>(y2), dual ? ptr<float>(aux2) : nullptr, act, ptr<bf16>(out),
                         mask.defined() ? mask.data_ptr<uint8_t>() : nullptr, st);
  }
  return {out, mask, aux, aux2};
}

// Full BN backward: returns {dy, dres, dy2, dgamma, dbeta, dgamma2, dbeta2}
std::vector<Tensor> bn_backward_impl(const Tensor& dout, const optional<Tensor>& out,
                                     const optional<Tensor>& mask, const Tensor& y,
                                     const Tensor& aux, const optional<Tensor>& gamma,
                                     const optional<Tensor>& y2, const optional<Tensor>& aux2,
                                     const optional<Tensor>& gamma2, int act, bool training,
                                     bool need_dres, const optional<Tensor>& dgamma_acc,
                                     const optional<Tensor>& dbeta_acc,
                                     const optional<Tensor>& dgamma2_acc,
                                     const optional<Tensor>& dbeta2_acc,
                                     const optional<Tensor>& partial_in,
                                     const optional<Tensor>& acc_in, int acc_rows, bool acc_filled,
                                     const optional<Tensor>& zero1, const optional<Tensor>& zero2,
                                     const optional<Tensor>& dx_out, bool dx_acc);
std::vector<Tensor> bn_backward(const Tensor& dout, const optional<Tensor>& out,
                                const optional<Tensor>& mask, const Tensor& y,
                                const Tensor& aux, const optional<Tensor>& gamma,
                                const optional<Tensor>& y2, const optional<Tensor>& aux2,
                                const optional<Tensor>& gamma2, int act, bool training,
                                bool need_dres, const optional<Tensor>& dgamma_acc,
                                const optional<Tensor>& dbeta_acc,
                                const optional<Tensor>& dgamma2_acc,
                                const optional<Tensor>& dbeta2_acc,
                                const optional<Tensor>& partial_in,
                                const optional<Tensor>& acc_in, int acc_rows, bool acc_filled,
                                const optional<Tensor>& zero1, const optional<Tensor>& zero2,
                                const optional<Tensor>& dx_out, bool dx_acc,
                                const optional<Tensor>& dbias_acc) {
  // dbias_acc: the bias gradient of the conv that feeds only this BN, added by the finalize
  float* dbias = nullptr;
  if (dbias_acc.has_value() && dbias_acc->defined() && training) {
    check_f32(*dbias_acc, "dbias_acc");
    TORCH_CHECK(dbias_acc->numel() == y.size(-1), "dbias_acc size");
    dbias = ptr<float>(*dbias_acc);
  }
  struct DbiasScope {
    explicit DbiasScope(float* p) { pca::set_bn_dbias(p); }
    ~DbiasScope() { pca::set_bn_dbias(nullptr); }
  } dbias_scope(dbias);
  const bool extra = need_dres || (y2.has_value() && y2->defined()) ||
                     (dx_out.has_value() && dx_out->defined());
  const Tensor yd = bn_odd_strided(y) && extra ? y.contiguous() : y;
  return bn_backward_impl(dout, out, mask, yd, aux, gamma, y2, aux2, gamma2, act, training,
                          need_dres, dgamma_acc, dbeta_acc, dgamma2_acc, dbeta2_acc, partial_in,
                          acc_in, acc_rows, acc_filled, zero1, zero2, dx_out, dx_acc);
}

std::vector<Tensor> bn_backward_impl(const Tensor& dout, const optional<Tensor>& out,
                                const optional<Tensor>& mask, const Tensor& y,
                                const Tensor& aux, const optional<Tensor>& gamma,
                                const optional<Tensor>& y2, const optional<Tensor>& aux2,
                                const optional<Tensor>& gamma2, int act, bool training,
                                bool need_dres, const optional<Tensor>& dgamma_acc,
                                const optional<Tensor>& dbeta_acc,
                                const optional<Tensor>& dgamma2_acc,
                                const optional<Tensor>& dbeta2_acc,
                                const optional<Tensor>& partial_in,
                                const optional<Tensor>& acc_in, int acc_rows, bool acc_filled,
                                const optional<Tensor>& zero1, const optional<Tensor>& zero2,
                                const optional<Tensor>& dx_out, bool dx_acc) {
  // dout / y may be row-strided channel slices of concat slabs; dx_out (optional) receives dy
  // (added into it with dx_acc), else dy is a new tensor
  const int ldd = rows_ld(dout, "dout");
  const int ldy = rows_ld_bn(y, "y");
  const int C = y.size(-1);
  TORCH_CHECK(dout.sizes() == y.sizes(), "dout shape mismatch");
  int ldx = C;
  const bool has_dx = dx_out.has_value() && dx_out->defined();
  if (has_dx) {
    ldx = rows_ld(*dx_out, "dx_out");
    TORCH_CHECK(dx_out->sizes() == y.sizes(), "dx_out shape mismatch");
  }
  TORCH_CHECK(has_dx || !dx_acc, "dx_acc needs dx_out");
  // y the prefix of zero-padded rows (C % 8 != 0): dy comes back in the same padded layout, its
  // padding zeroed by the kernel — the padded conv's dY, with no pad pass
  const bool pad_dy = !has_dx && ldy != C && C % 8 != 0;
  if (pad_dy) ldx = ldy;
  BnLdScope lds(C, ldy, C, ldd, ldx, dx_acc);
  auto new_dy = [&]() {
    if (has_dx) return *dx_out;
    if (pad_dy)
      return at::empty({y.size(0), y.size(1), y.size(2), (int64_t)ldy}, y.options()).narrow(3, 0, C);
    return at::empty(y.sizes(), y.options());
  };
  const int M = y.numel() / C;
  const bool dual = y2.has_value() && y2->defined();
  const int NS = dual ? 3 : 2;
  const bool has_mask = mask.has_value() && mask->defined();
  if (act == 1)
    TORCH_CHECK((out.has_value() && out->defined()) || (has_mask && C % 8 == 0),
                "relu backward needs the output or its sign mask");
  const uint8_t* mk = has_mask ? mask->data_ptr<uint8_t>() : nullptr;
  auto st = cur_stream();
  auto fopt = y.options().dtype(at::kFloat);
  // Parameter gradients are accumulated straight into the caller's .grad buffers when given
  // (the flat gradient arena); otherwise fresh tensors are returned.
  auto pick = [&](const optional<Tensor>& acc) {
    if (acc.has_value() && acc->defined()) {
      check_f32(*acc, "grad accumulator");
      TORCH_CHECK(acc->numel() == C, "grad accumulator size");
      return *acc;
    }
    return at::zeros({C}, fopt);
  };
  if (training && acc_in.has_value() && acc_in->defined()) {
    // sharded accumulator path: sums from the consumer conv's dgrad epilogue (acc_filled) or
    // from the reduce kernel below, folded by the fused apply kernel (which re-zeroes it)
    const Tensor& acc = *acc_in;
    check_acc(acc, acc_rows, NS, C);
    const bool z1 = zero1.has_value() && zero1->defined();
    const bool z2 = zero2.has_value() && zero2->defined();
    if (z1) check_f32(*zero1, "zero1");
    if (z2) check_f32(*zero2, "zero2");
    float* zp1 = z1 ? ptr<float>(*zero1) : nullptr;
    float* zp2 = z2 ? ptr<float>(*zero2) : nullptr;
    const int zn1 = z1 ? (int)zero1->numel() : 0, zn2 = z2 ? (int)zero2->numel() : 0;
    if (!acc_filled && (int64_t)M * C <= acc_max_elems()) {
      // no dgrad epilogue delivered the sums: a separate reduce pass over dout, adding into the
      // accumulator from a grid of at most kAccDepth blocks per shard row
      ShardScope shards(acc_rows);
      pca::bn_bwd_reduce_launch(ptr<bf16>(dout), optr<bf16>(out), mk, ptr<bf16>(y), ptr<float>(aux),
                                optr<bf16>(y2), optr<float>(aux2), act, M, C, ptr<float>(acc),
                                acc_reduce_blocks(M, C, acc_rows), st);
      acc_filled = true;
    }
    if (!acc_filled) {
      // large tensor, no dgrad epilogue delivered the sums: its ~1024 reduce blocks would
      // serialise on the accumulator's few shard rows (same-address atomics), so this case keeps
      // ordered slab rows + the finalize kernel (whose block 0 clears the forward accumulators)
      // and the accumulator stays untouched.
      const int P = pca::bn_row_blocks(M, C);
      auto partial = at::empty({P, NS, C}, fopt);
      pca::bn_bwd_reduce_launch(ptr<bf16>(dout), optr<bf16>(out), mk, ptr<bf16>(y), ptr<float>(aux),
                                optr<bf16>(y2), optr<float>(aux2), act, M, C, ptr<float>(partial),
                                P, st);
      const float* stat = ptr<float>(partial);
      int R = P;
      Tensor folded;
      if (R > 1024) {
        folded = at::empty({64, NS, C}, fopt);
        R = pca::colsum_launch(stat, R, NS * C, ptr<float>(folded), st);
        stat = ptr<float>(folded);
      }
      auto dgamma = pick(dgamma_acc), dbeta = pick(dbeta_acc);
      Tensor dgamma2, dbeta2;
      if (dual) {
        dgamma2 = pick(dgamma2_acc);
        dbeta2 = pick(dbeta2_acc);
      }
      auto coef = at::empty({dual ? 6 : 3, C}, fopt);
      pca::bn_bwd_finalize_launch(stat, R, NS, C, (float)M, ptr<float>(aux), optr<float>(gamma),
                                  optr<float>(aux2), optr<float>(gamma2), 1, ptr<float>(dgamma),
                                  ptr<float>(dbeta), dual ? ptr<float>(dgamma2) : nullptr,
                                  dual ? ptr<float>(dbeta2) : nullptr, ptr<float>(coef), 1, st,
                                  zp1, zn1, zp2, zn2);
      auto dy = new_dy();
      Tensor dres, dy2;
      if (need_dres) dres = at::empty(y.sizes(), y.options());
      if (dual) dy2 = at::empty(y.sizes(), y.options());
      pca::bn_bwd_apply_launch(ptr<bf16>(dout), optr<bf16>(out), mk, ptr<bf16>(y), ptr<float>(aux),
                               ptr<float>(coef), act, C, y.numel(), ptr<bf16>(dy),
                               need_dres ? ptr<bf16>(dres) : nullptr, optr<bf16>(y2),
                               dual ? ptr<bf16>(dy2) : nullptr, st);
      return {dy, dres, dy2, dgamma, dbeta, dgamma2, dbeta2};
    }
    auto dgamma = pick(dgamma_acc), dbeta = pick(dbeta_acc);
    Tensor dgamma2, dbeta2;
    if (dual) {
      dgamma2 = pick(dgamma2_acc);
      dbeta2 = pick(dbeta2_acc);
    }
    auto dy = new_dy();
    Tensor dres, dy2;
    if (need_dres) dres = at::empty(y.sizes(), y.options());
    if (dual) dy2 = at::empty(y.sizes(), y.options());
    const int pend = pca::wgrad_deferred_count();
    const bool fused = pca::bn_bwd_apply_acc_launch(
        ptr<bf16>(dout), mk, ptr<bf16>(y), C, M, (float)M, ptr<float>(acc), acc_rows,
        ptr<float>(aux), optr<float>(gamma), ptr<float>(dgamma), ptr<float>(dbeta),
        optr<float>(aux2), optr<float>(gamma2), dual ? ptr<float>(dgamma2) : nullptr,
        dual ? ptr<float>(dbeta2) : nullptr, act, ptr<bf16>(dy),
        need_dres ? ptr<bf16>(dres) : nullptr, optr<bf16>(y2), dual ? ptr<bf16>(dy2) : nullptr,
        zp1, zn1, zp2, zn2, st);
    // (the launch took the pending wgrad slab reductions along: their workspaces may be reused
    // by later allocations, which are stream-ordered after it)
    if (pend && pca::wgrad_deferred_count() == 0) g_deferred_ws.clear();
    if (!fused) {
      auto coef = at::empty({dual ? 6 : 3, C}, fopt);
      pca::bn_bwd_finalize_launch(ptr<float>(acc), acc_rows, NS, C, (float)M, ptr<float>(aux),
                                  optr<float>(gamma), optr<float>(aux2), optr<float>(gamma2), 1,
                                  ptr<float>(dgamma), ptr<float>(dbeta),
                                  dual ? ptr<float>(dgamma2) : nullptr,
                                  dual ? ptr<float>(dbeta2) : nullptr, ptr<float>(coef), 1, st,
                                  zp1, zn1, zp2, zn2);
      pca::bn_bwd_apply_launch(ptr<bf16>(dout), optr<bf16>(out), mk, ptr<bf16>(y), ptr<float>(aux),
                               ptr<float>(coef), act, C, y.numel(), ptr<bf16>(dy),
                               need_dres ? ptr<bf16>(dres) : nullptr, optr<bf16>(y2),
                               dual ? ptr<bf16>(dy2) : nullptr, st);
    }
    return {dy, dres, dy2, dgamma, dbeta, dgamma2, dbeta2};
  }
  Tensor partial;
  int R;
  if (partial_in.has_value() && partial_in->defined() && partial_in->numel() > 0) {
    // (sum dz, sum dz*xhat) already reduced by the producing conv's dgrad epilogue
    check_f32(*partial_in, "partial_in");
    TORCH_CHECK(!dual && partial_in->dim() == 3 && partial_in->size(1) == 2 &&
                    partial_in->size(2) == C, "partial_in must be [R][2][C] (single BN)");
    partial = *partial_in;
    R = partial.size(0);
  } else {
    const int P = pca::bn_row_blocks(M, C);
    partial = at::empty({P, NS, C}, fopt);
    pca::bn_bwd_reduce_launch(ptr<bf16>(dout), optr<bf16>(out), mk, ptr<bf16>(y), ptr<float>(aux),
                              optr<bf16>(y2), optr<float>(aux2), act, M, C, ptr<float>(partial), P,
                              st);
    R = P;
  }
  const float* stat = ptr<float>(partial);
  Tensor folded;
  if (R > 1024) {
    folded = at::empty({64, NS, C}, fopt);
    R = pca::colsum_launch(stat, R, NS * C, ptr<float>(folded), st);
    stat = ptr<float>(folded);
  }
  auto dgamma = pick(dgamma_acc), dbeta = pick(dbeta_acc);
  Tensor dgamma2, dbeta2;
  if (dual) {
    dgamma2 = pick(dgamma2_acc);
    dbeta2 = pick(dbeta2_acc);
  }
  auto coef = at::empty({dual ? 6 : 3, C}, fopt);
  // (the finalize's block 0 also clears the forward accumulators this BN consumed, if any)
  const bool nz1 = zero1.has_value() && zero1->defined();
  const bool nz2 = zero2.has_value() && zero2->defined();
  if (nz1) check_f32(*zero1, "zero1");
  if (nz2) check_f32(*zero2, "zero2");
  pca::bn_bwd_finalize_launch(stat, R, NS, C, (float)M, ptr<float>(aux), optr<float>(gamma),
                              optr<float>(aux2), optr<float>(gamma2), training ? 1 : 0,
                              ptr<float>(dgamma), ptr<float>(dbeta),
                              dual ? ptr<float>(dgamma2) : nullptr,
                              dual ? ptr<float>(dbeta2) : nullptr, ptr<float>(coef), 1, st,
                              nz1 ? ptr<float>(*zero1) : nullptr, nz1 ? (int)zero1->numel() : 0,
                              nz2 ? ptr<float>(*zero2) : nullptr, nz2 ? (int)zero2->numel() : 0);
  auto dy = new_dy();
  Tensor dres, dy2;
  if (need_dres) dres = at::empty(y.sizes(), y.options());
  if (dual) dy2 = at::empty(y.sizes(), y.options());
  pca::bn_bwd_apply_launch(ptr<bf16>(dout), optr<bf16>(out), mk, ptr<bf16>(y), ptr<float>(aux),
                           ptr<float>(coef), act, C, y.numel(), ptr<bf16>(dy),
                           need_dres ? ptr<bf16>(dres) : nullptr, optr<bf16>(y2),
                           dual ? ptr<bf16>(dy2) : nullptr, st);
  return {dy, dres, dy2, dgamma, dbeta, dgamma2, dbeta2};
}

// ---- fused Winograd F(2x2,3x3) forward (csrc/winograd.hip) ----
// w: fp32 [Co][3][3][Ci] (the physical channels_last master) -> U bf16 [16][Co][Ci]
Tensor winograd_filter(const Tensor& w) {
  check_f32(w, "w");
  TORCH_CHECK(w.dim() == 4 && w.size(1) == 3 && w.size(2) == 3, "w must be [Co][3][3][Ci]");
  const int Co = w.size(0), Ci = w.size(3);
  auto U = at::empty({16, Co, Ci}, w.options().dtype(at::kBFloat16));
  pca::winograd_filter_launch(ptr<float>(w), Co, Ci, ptr<bf16>(U), cur_stream());
  return U;
}

// x NHWC bf16, U [16][Co][Ci] -> (y NHWC bf16, BN partial sums [rows][2][Co] or empty)
std::vector<Tensor> winograd_fwd(const Tensor& x, const Tensor& U, bool want_stats) {
  check_bf16(x, "x");
  check_bf16(U, "U");
  TORCH_CHECK(x.dim() == 4 && U.dim() == 3 && U.size(0) == 16 && U.size(2) == x.size(3),
              "winograd_fwd: x [N,H,W,Ci], U [16,Co,Ci]");
  const int N = x.size(0), H = x.size(1), W = x.size(2), Ci = x.size(3), Co = U.size(1);
  TORCH_CHECK(pca::winograd_applicable(N, H, W, Ci, Co),
              "winograd_fwd: needs even H, W, Ci % 32 == 0, Co % 64 == 0");
  auto y = at::empty({N, H, W, Co}, x.options());
  Tensor st = want_stats ? at::empty({pca::winograd_stat_rows(N, H, W), 2, Co},
                                     x.options().dtype(at::kFloat))
                         : at::empty({0}, x.options().dtype(at::kFloat));
  pca::winograd_fwd_launch(ptr<bf16>(x), ptr<bf16>(U), ptr<bf16>(y),
                           want_stats ? ptr<float>(st) : nullptr, N, H, W, Ci, Co, cur_stream());
  return {y, st};
}

// ------------------------------------------------------------------------------ misc
Tensor nchw_to_nhwc(const Tensor& x, int Cp) {
  check_f32(x, "x");
  const int N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  TORCH_CHECK(Cp >= C, "pad channels");
  auto y = at::empty({N, H, W, Cp}, x.options().dtype(at::kBFloat16));
  pca::nchw_to_nhwc_launch(ptr<float>(x), N, C, H * W, Cp, ptr<bf16>(y), cur_stream());
  return y;
}

Tensor nhwc_to_nchw(const Tensor& y, int C) {
  check_bf16(y, "y");
  const int N = y.size(0), H = y.size(1), W = y.size(2), Cp = y.size(3);
  auto x = at::empty({N, C, H, W}, y.options().dtype(at::kFloat));
  pca::nhwc_to_nchw_launch(ptr<bf16>(y), N, C, H * W, Cp, ptr<float>(x), cur_stream());
  return x;
}

Tensor augment(const Tensor& data, const Tensor& idx, const Tensor& rnd, int pad,
               std::vector<double> mean, std::vector<double> std) {
  TORCH_CHECK(data.is_cuda() && data.scalar_type() == at::kByte && data.dim() == 4 &&
                  data.size(3) == 3 && data.is_contiguous(),
              "data must be uint8 [N,H,W,3] on GPU");
  TORCH_CHECK(idx.scalar_type() == at::kLong && rnd.scalar_type() == at::kInt, "idx/rnd dtypes");
  TORCH_CHECK(idx.numel() == rnd.numel(), "idx/rnd size");
  TORCH_CHECK(mean.size() == 3 && std.size() == 3, "mean/std");
  const int B = idx.numel(), H = data.size(1), W = data.size(2);
  auto out = at::empty({B, H, W, 8}, data.options().dtype(at::kBFloat16));
  float m[3] = {(float)mean[0], (float)mean[1], (float)mean[2]};
  float s[3] = {(float)std[0], (float)std[1], (float)std[2]};
  pca::augment_launch(ptr<uint8_t>(data), ptr<int64_t>(idx), ptr<int32_t>(rnd), B, H, W, pad, m, s,
                      ptr<bf16>(out), nullptr, nullptr, cur_stream());
  return out;
}

// stem 3x3 conv weight gradient added into `out` (the fp32 gradient, physical [Co][3][3][3]) from
// the 8-channel padded input x [N,H,W,8] and dy [N,H,W,Co]; False when the shape is not the
// stem's (the caller then takes the generic padded wgrad)
bool stem_wgrad(const Tensor& x, const Tensor& dy, int64_t stride, int64_t padding, Tensor out) {
  if (!(x.is_cuda() && dy.is_cuda() && out.is_cuda() && x.dim() == 4 && dy.dim() == 4 &&
        out.dim() == 4 && x.scalar_type() == at::kBFloat16 && dy.scalar_type() == at::kBFloat16 &&
        out.scalar_type() == at::kFloat && x.is_contiguous() && dy.is_contiguous() &&
        out.is_contiguous() && stride == 1 && padding == 1))
    return false;
  const int N = x.size(0), H = x.size(1), W = x.size(2), Cs = x.size(3), Co = dy.size(3);
  if (dy.size(0) != N || dy.size(1) != H || dy.size(2) != W) return false;
  if (out.size(0) != Co || out.size(1) != 3 || out.size(2) != 3) return false;
  if (!pca::stem_wgrad_supported(N, H, W, Cs, (int)out.size(3), Co)) return false;
  auto slab = at::empty({pca::stem_wgrad_slab_rows(N, H), Co * 27}, out.options());
  pca::stem_wgrad_launch(ptr<bf16>(x), ptr<bf16>(dy), N, H, Co, ptr<float>(slab), ptr<float>(out),
                         cur_stream());
  return true;
}

// packed[b] = sample | word << 32 (word: the augmentation draw, see augment_kernel) ->
// (NHWC8 bf16 images, int64 targets gathered from labels) in one launch
std::vector<Tensor> augment_packed(const Tensor& data, const Tensor& labels, const Tensor& packed,
                                   int pad, std::vector<double> mean, std::vector<double> std) {
  TORCH_CHECK(data.is_cuda() && data.scalar_type() == at::kByte && data.dim() == 4 &&
                  data.size(3) == 3 && data.is_contiguous(),
              "data must be uint8 [N,H,W,3] on GPU");
  TORCH_CHECK(packed.scalar_type() == at::kLong && packed.is_contiguous() && packed.is_cuda(),
              "packed must be contiguous int64 on GPU");
  TORCH_CHECK(labels.scalar_type() == at::kLong && labels.is_contiguous() &&
                  labels.numel() == data.size(0),
              "labels must be int64 [N]");
  TORCH_CHECK(mean.size() == 3 && std.size() == 3, "mean/std");
  const int B = packed.numel(), H = data.size(1), W = data.size(2);
  auto out = at::empty({B, H, W, 8}, data.options().dtype(at::kBFloat16));
  auto targets = at::empty({B}, labels.options());
  float m[3] = {(float)mean[0], (float)mean[1], (float)mean[2]};
  float s[3] = {(float)std[0], (float)std[1], (float)std[2]};
  pca::augment_launch(ptr<uint8_t>(data), ptr<int64_t>(packed), nullptr, B, H, W, pad, m, s,
                      ptr<bf16>(out), ptr<int64_t>(labels), ptr<int64_t>(targets), cur_stream());
  return {out, targets};
}

// fused classifier head: x [N,H,W,C] bf16 -> (logits [N,K] fp32, pooled [N,C] fp32)
// rng state of the dropout kernels: int64[3] {seed, step, tickets} on the device (misc.hip)
static void check_rng(const Tensor& rng) {
  TORCH_CHECK(rng.is_cuda() && rng.scalar_type() == at::kLong && rng.numel() == 3 &&
                  rng.is_contiguous(),
              "dropout rng state must be a contiguous int64[3] device tensor {seed, step, 0}");
}

std::vector<Tensor> head_fwd(const Tensor& x, const Tensor& w, const optional<Tensor>& b,
                             double p, const optional<Tensor>& rng) {
  check_bf16(x, "x");
  check_f32(w, "weight");
  const int N = x.size(0), HW = x.size(1) * x.size(2), C = x.size(3);
  const int K = w.size(0);
  TORCH_CHECK(w.dim() == 2 && w.size(1) == C, "weight must be [K, C]");
  TORCH_CHECK(pca::head_supported(C, K) && pca::head_batch_supported(N, K),
              "fused head needs C % 8 == 0, K <= 16 and N * K <= 12288");
  if (b.has_value() && b->defined()) {
    check_f32(*b, "bias");
    TORCH_CHECK(b->numel() == K, "bias size");
  }
  auto fopt = x.options().dtype(at::kFloat);
  auto logits = at::empty({N, K}, fopt);
  auto pooled = at::empty({N, C}, fopt);
  TORCH_CHECK(p >= 0.0 && p < 1.0, "dropout p must be in [0, 1)");
  Tensor dmask;
  if (p > 0.0) {
    TORCH_CHECK(rng.has_value() && rng->defined(), "dropout needs its rng state");
    check_rng(*rng);
    dmask = at::empty({N, C}, x.options().dtype(at::kByte));
  }
  pca::head_fwd_launch(ptr<bf16>(x), N, HW, C, ptr<float>(w), optr<float>(b), K, ptr<float>(pooled),
                       ptr<float>(logits), (float)p, p > 0.0 ? ptr<int64_t>(*rng) : nullptr,
                       p > 0.0 ? ptr<uint8_t>(dmask) : nullptr, cur_stream());
  return {logits, pooled, dmask};
}

// generic dropout / drop-connect on a contiguous bf16 or fp32 tensor: one keep byte per unit of
// `unit_len` consecutive elements (1 = elementwise dropout; C*H*W = per-sample drop-connect)
std::vector<Tensor> dropout_fwd(const Tensor& x, double p, int64_t unit_len, const Tensor& rng) {
  TORCH_CHECK(x.is_cuda() && x.is_contiguous() &&
                  (x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kFloat),
              "dropout: contiguous bf16 / fp32 device tensor");
  TORCH_CHECK(p > 0.0 && p < 1.0 && unit_len >= 1 && x.numel() % unit_len == 0, "dropout args");
  check_rng(rng);
  auto y = at::empty_like(x);
  auto mask = at::empty({x.numel() / unit_len}, x.options().dtype(at::kByte));
  if (x.numel())
    pca::dropout_fwd_launch(x.data_ptr(), x.scalar_type() == at::kBFloat16, x.numel(), unit_len,
                            (float)p, ptr<int64_t>(rng), ptr<uint8_t>(mask), y.data_ptr(), cur_stream());
  return {y, mask};
}

Tensor dropout_bwd(const Tensor& dy, const Tensor& mask, double p, int64_t unit_len) {
  TORCH_CHECK(dy.is_cuda() && dy.is_contiguous() &&
                  (dy.scalar_type() == at::kBFloat16 || dy.scalar_type() == at::kFloat),
              "dropout grad: contiguous bf16 / fp32 device tensor");
  TORCH_CHECK(mask.scalar_type() == at::kByte && mask.numel() * unit_len == dy.numel(), "mask");
  auto dx = at::empty_like(dy);
  if (dy.numel())
    pca::dropout_bwd_launch(dy.data_ptr(), dy.scalar_type() == at::kBFloat16, dy.numel(), unit_len,
                            (float)p, ptr<uint8_t>(mask), dx.data_ptr(), cur_stream());
  return dx;
}

// backward of head_fwd: returns {dx [N,H,W,C] bf16, dw [K,C], db [K]}; dw / db are added into
// the given accumulators (gradient-arena views) when present, else fresh zero-based tensors
std::vector<Tensor> head_bwd(const Tensor& dl, const Tensor& w, const Tensor& pooled, int H, int W,
                             const optional<Tensor>& dw_acc, const optional<Tensor>& db_acc,
                             bool want_db, double p, const optional<Tensor>& dmask,
                             const optional<Tensor>& bn_y = c10::nullopt,
                             const optional<Tensor>& bn_mask = c10::nullopt,
                             const optional<Tensor>& bn_aux = c10::nullopt,
                             const optional<Tensor>& bn_acc = c10::nullopt, int acc_rows = 0) {
  check_f32(dl, "dlogits");
  check_f32(w, "weight");
  check_f32(pooled, "pooled");
  const int N = dl.size(0), K = dl.size(1), C = w.size(1);
  TORCH_CHECK(pooled.size(0) == N && pooled.size(1) == C && w.size(0) == K, "head shapes");
  auto fopt = dl.options();
  auto dx = at::empty({N, H, W, C}, dl.options().dtype(at::kBFloat16));
  Tensor dw = (dw_acc.has_value() && dw_acc->defined()) ? *dw_acc : at::zeros({K, C}, fopt);
  Tensor db;
  if (want_db) db = (db_acc.has_value() && db_acc->defined()) ? *db_acc : at::zeros({K}, fopt);
  TORCH_CHECK(dw.is_contiguous() && dw.numel() == (int64_t)K * C, "dw accumulator");
  if (db.defined()) TORCH_CHECK(db.is_contiguous() && db.numel() == K, "db accumulator");
  const bool drop = dmask.has_value() && dmask->defined();
  if (drop)
    TORCH_CHECK(dmask->scalar_type() == at::kByte && dmask->numel() == (int64_t)N * C && p > 0.0 &&
                    p < 1.0,
                "dropout mask [N, C] uint8 and p in (0, 1)");
  // fused backward sums of the BN(+ReLU) that produced the pooled features (see head_bwd_kernel)
  const bool bnf = bn_acc.has_value() && bn_acc->defined();
  if (bnf) {
    TORCH_CHECK(C % 8 == 0 && 256 % (C / 8) == 0, "head_bwd BN fusion: 256 % (C/8) == 0");
    check_bf16(*bn_y, "bn_y");
    TORCH_CHECK(bn_y->numel() == (int64_t)N * H * W * C, "bn_y must match dx");
    TORCH_CHECK(bn_mask.has_value() && bn_mask->defined() && bn_mask->scalar_type() == at::kByte &&
                    bn_mask->numel() * 8 == bn_y->numel(), "bn_mask: one bit per element");
    check_f32(*bn_aux, "bn_aux");
    TORCH_CHECK(bn_aux->numel() >= 2 * C, "bn_aux [mean|istd|...][C]");
    check_acc(*bn_acc, acc_rows, 2, C);
  }
  pca::head_bwd_launch(ptr<float>(dl), ptr<float>(w), ptr<float>(pooled), N, H * W, C, K,
                       ptr<bf16>(dx), ptr<float>(dw), db.defined() ? ptr<float>(db) : nullptr,
                       (float)p, drop ? ptr<uint8_t>(*dmask) : nullptr, cur_stream(),
                       bnf ? ptr<bf16>(*bn_y) : nullptr, bnf ? bn_mask->data_ptr<uint8_t>() : nullptr,
                       bnf ? ptr<float>(*bn_aux) : nullptr, bnf ? ptr<float>(*bn_acc) : nullptr,
                       bnf ? acc_rows : 0);
  return {dx, dw, db};
}

// whole squeeze-excite block on NHWC x [N,H,W,C]: pool -> s = W2 act(W1 p + b1) + b2 ->
// out = x * sigmoid(s). w1 [R, C(,1,1)], w2 [C, R(,1,1)] fp32. Returns {out, pooled, hpre, s}.
static void check_se(const Tensor& x, const Tensor& w1, const Tensor& w2, int& R) {
  const int C = x.size(3);
  R = w1.size(0);
  check_f32(w1, "w1");
  check_f32(w2, "w2");
  TORCH_CHECK(w1.is_contiguous() && w2.is_contiguous() && w1.numel() == (int64_t)R * C &&
                  w2.numel() == (int64_t)R * C && w2.size(0) == C,
              "squeeze-excite weights must be [R, C] and [C, R]");
  TORCH_CHECK(pca::se_mlp_supported(C, R), "squeeze-excite MLP: C % 8 == 0, C <= 2048, R <= 192");
}

// One-block-per-sample pool + MLP forward and ds + MLP-data backward (misc.hip se_*_fused: 2
// launches forward, 3 backward instead of 4 and 5), taken when the caller passes W2^T (ops/
// functional.py does under PCA_SE_FUSED=1). Off by default there: the per-sample blocks serialise
// the MLP latency — EfficientNet-B0 bs128 3.99 vs 3.87 ms, bs1024 9.12 vs 8.31 ms (round 6).
static int g_se_fused = -1;   // -1: PCA_SE_FUSED decides; 0 / 1 set by se_fused_mode (A/B)
static bool se_fused(int C, int R) {
  static const bool on = [] {
    const char* e = getenv("PCA_SE_FUSED");
    return !(e && e[0] == '0');
  }();
  return (g_se_fused < 0 ? on : g_se_fused == 1) && pca::se_fused_supported(C, R);
}
int se_fused_mode(int m) {
  const int prev = g_se_fused;
  g_se_fused = m;
  return prev;
}

// w2t: W2 transposed [R][C] fp32 (the fused kernels read it coalesced); without it the split
// kernels run
static const float* check_w2t(const optional<Tensor>& w2t, int R, int C) {
  if (!(w2t.has_value() && w2t->defined())) return nullptr;
  check_f32(*w2t, "w2t");
  TORCH_CHECK(w2t->is_contiguous() && w2t->numel() == (int64_t)R * C, "w2t must be [R][C]");
  return ptr<float>(*w2t);
}

std::vector<Tensor> se_forward(const Tensor& x, const Tensor& w1, const optional<Tensor>& b1,
                               const Tensor& w2, const optional<Tensor>& b2, int act,
                               const optional<Tensor>& w2t = c10::nullopt) {
  check_bf16(x, "x");
  int R;
  check_se(x, w1, w2, R);
  const float* w2tp = check_w2t(w2t, R, x.size(3));
  const int N = x.size(0), HW = x.size(1) * x.size(2), C = x.size(3);
  TORCH_CHECK(act == 1 || act == 2, "squeeze-excite act: relu (1) / swish (2)");
  if (b1.has_value() && b1->defined()) TORCH_CHECK(b1->numel() == R, "b1");
  if (b2.has_value() && b2->defined()) TORCH_CHECK(b2->numel() == C, "b2");
  auto fopt = x.options().dtype(at::kFloat);
  auto pooled = at::empty({N, C}, fopt);
  auto hpre = at::empty({N, R}, fopt);
  auto s = at::empty({N, C}, fopt);
  auto out = at::empty_like(x);
  auto st = cur_stream();
  if (w2tp && se_fused(C, R)) {
    pca::se_fwd_fused_launch(ptr<bf16>(x), N, HW, C, R, ptr<float>(w1), optr<float>(b1),
                             w2tp, optr<float>(b2), act, ptr<float>(pooled),
                             ptr<float>(hpre), ptr<float>(s), st);
  } else {
    pca::gap_fwd_launch(ptr<bf16>(x), N, HW, C, ptr<float>(pooled), st);
    pca::se_mlp_fwd_launch(ptr<float>(pooled), N, C, R, ptr<float>(w1), optr<float>(b1),
                           ptr<float>(w2), optr<float>(b2), act, ptr<float>(hpre), ptr<float>(s),
                           st);
  }
  pca::se_scale_fwd_launch(ptr<bf16>(x), ptr<float>(s), N, HW, C, ptr<bf16>(out), st);
  return {out, pooled, hpre, s};
}

// backward of se_forward: returns {dx, dw1, db1, dw2, db2}; parameter gradients are added into
// the given accumulators (gradient-arena views) when present, else into fresh zero tensors
// (db* undefined when want_b* is false)
std::vector<Tensor> se_backward(const Tensor& dout, const Tensor& x, const Tensor& pooled,
                                const Tensor& hpre, const Tensor& s, const Tensor& w1,
                                const Tensor& w2, int act, const optional<Tensor>& dw1_acc,
                                const optional<Tensor>& db1_acc, const optional<Tensor>& dw2_acc,
                                const optional<Tensor>& db2_acc, bool want_b1, bool want_b2,
                                const optional<Tensor>& w2t = c10::nullopt) {
  check_bf16(dout, "dout");
  check_bf16(x, "x");
  int R;
  check_se(x, w1, w2, R);
  const float* w2tp = check_w2t(w2t, R, x.size(3));
  const int N = x.size(0), HW = x.size(1) * x.size(2), C = x.size(3);
  TORCH_CHECK(dout.sizes() == x.sizes(), "dout shape");
  TORCH_CHECK(pooled.numel() == (int64_t)N * C && s.numel() == (int64_t)N * C &&
                  hpre.numel() == (int64_t)N * R,
              "saved squeeze-excite tensors");
  auto fopt = x.options().dtype(at::kFloat);
  auto pick = [&](const optional<Tensor>& a, int64_t n, bool want) {
    if (!want) return Tensor();
    Tensor t = (a.has_value() && a->defined()) ? *a : at::zeros({n}, fopt);
    TORCH_CHECK(t.is_contiguous() && t.numel() == n && t.scalar_type() == at::kFloat,
                "squeeze-excite gradient accumulator");
    return t;
  };
  Tensor dw1 = pick(dw1_acc, (int64_t)R * C, true), dw2 = pick(dw2_acc, (int64_t)R * C, true);
  Tensor db1 = pick(db1_acc, R, want_b1), db2 = pick(db2_acc, C, want_b2);
  auto ds = at::empty({N, C}, fopt);
  auto dp = at::empty({N, C}, fopt);
  auto dz = at::empty({N, R}, fopt);
  auto dx = at::empty_like(x);
  auto st = cur_stream();
  if (w2tp && se_fused(C, R)) {
    pca::se_bwd_data_launch(ptr<bf16>(dout), ptr<bf16>(x), ptr<float>(s), N, HW, C, R,
                            ptr<float>(w1), w2tp, ptr<float>(hpre), act, ptr<float>(ds),
                            ptr<float>(dz), ptr<float>(dp), st);
    pca::se_mlp_bwd_param_launch(ptr<float>(ds), ptr<float>(dz), ptr<float>(hpre),
                                 ptr<float>(pooled), N, C, R, act, ptr<float>(dw1),
                                 db1.defined() ? ptr<float>(db1) : nullptr, ptr<float>(dw2),
                                 db2.defined() ? ptr<float>(db2) : nullptr, st);
  } else {
    pca::se_ds_launch(ptr<bf16>(dout), ptr<bf16>(x), ptr<float>(s), N, HW, C, ptr<float>(ds), st);
    pca::se_mlp_bwd_launch(ptr<float>(ds), ptr<float>(hpre), ptr<float>(pooled), N, C, R,
                           ptr<float>(w1), ptr<float>(w2), act, ptr<float>(dz), ptr<float>(dp),
                           ptr<float>(dw1), db1.defined() ? ptr<float>(db1) : nullptr,
                           ptr<float>(dw2), db2.defined() ? ptr<float>(db2) : nullptr, st);
  }
  pca::se_dx_launch(ptr<bf16>(dout), ptr<float>(s), ptr<float>(dp), N, HW, C, ptr<bf16>(dx), st);
  return {dx, dw1, db1, dw2, db2};
}

Tensor gap_fwd(const Tensor& x) {
  check_bf16(x, "x");
  const int N = x.size(0), HW = x.size(1) * x.size(2), C = x.size(3);
  auto y = at::empty({N, C}, x.options().dtype(at::kFloat));
  pca::gap_fwd_launch(ptr<bf16>(x), N, HW, C, ptr<float>(y), cur_stream());
  return y;
}

Tensor gap_bwd(const Tensor& dy, int H, int W) {
  check_f32(dy, "dy");
  const int N = dy.size(0), C = dy.size(1);
  auto dx = at::empty({N, H, W, C}, dy.options().dtype(at::kBFloat16));
  pca::gap_bwd_launch(ptr<float>(dy), N, H * W, C, ptr<bf16>(dx), cur_stream());
  return dx;
}

Tensor avgpool_fwd(const Tensor& x, int k, int s, int p) {
  check_bf16(x, "x");
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  const int Ho = out_dim(H, k, s, p), Wo = out_dim(W, k, s, p);
  auto y = at::empty({N, Ho, Wo, C}, x.options());
  pca::avgpool_fwd_launch(ptr<bf16>(x), N, H, W, C, Ho, Wo, k, s, p, ptr<bf16>(y), cur_stream());
  return y;
}

Tensor avgpool_bwd(const Tensor& dy, int H, int W, int k, int s, int p) {
  check_bf16(dy, "dy");
  const int N = dy.size(0), Ho = dy.size(1), Wo = dy.size(2), C = dy.size(3);
  auto dx = at::empty({N, H, W, C}, dy.options());
  pca::avgpool_bwd_launch(ptr<bf16>(dy), N, H, W, C, Ho, Wo, k, s, p, ptr<bf16>(dx), cur_stream());
  return dx;
}

std::vector<Tensor> maxpool_fwd(const Tensor& x, int k, int s, int p) {
  check_bf16(x, "x");
  TORCH_CHECK(k * k <= 255, "maxpool window too large");
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  const int Ho = out_dim(H, k, s, p), Wo = out_dim(W, k, s, p);
  auto y = at::empty({N, Ho, Wo, C}, x.options());
  auto arg = at::empty({N, Ho, Wo, C}, x.options().dtype(at::kByte));
  pca::maxpool_fwd_launch(ptr<bf16>(x), N, H, W, C, Ho, Wo, k, s, p, ptr<bf16>(y), ptr<uint8_t>(arg),
                          cur_stream());
  return {y, arg};
}

Tensor maxpool_bwd(const Tensor& dy, const Tensor& arg, int H, int W, int k, int s, int p) {
  check_bf16(dy, "dy");
  const int N = dy.size(0), Ho = dy.size(1), Wo = dy.size(2), C = dy.size(3);
  auto dx = at::empty({N, H, W, C}, dy.options());
  pca::maxpool_bwd_launch(ptr<bf16>(dy), ptr<uint8_t>(arg), N, H, W, C, Ho, Wo, k, s, p,
                          ptr<bf16>(dx), cur_stream());
  return dx;
}

std::vector<Tensor> ce_fused(const Tensor& logits, const Tensor& tgt,
                             const optional<Tensor>& metrics, bool want_grad) {
  check_f32(logits, "logits");
  TORCH_CHECK(tgt.scalar_type() == at::kLong && tgt.is_cuda(), "targets int64 on GPU");
  const int N = logits.size(0), K = logits.size(1);
  TORCH_CHECK(tgt.numel() == N, "target count");
  if (metrics.has_value() && metrics->defined())
    TORCH_CHECK(metrics->scalar_type() == at::kDouble && metrics->numel() >= 3, "metrics buffer");
  auto loss = at::empty({}, logits.options());
  Tensor dl;
  if (want_grad) dl = at::empty_like(logits);
  pca::ce_fused_launch(ptr<float>(logits), ptr<int64_t>(tgt), N, K, ptr<float>(loss),
                       want_grad ? ptr<float>(dl) : nullptr, optr<double>(metrics), cur_stream());
  return {loss, dl};
}

Tensor scale_by_scalar(const Tensor& g, const Tensor& s) {
  check_f32(g, "g");
  auto out = at::empty_like(g);
  pca::scale_by_scalar_launch(ptr<float>(g), ptr<float>(s), g.numel(), ptr<float>(out),
                              cur_stream());
  return out;
}

// ptr tables are int64 GPU tensors holding device addresses; chunks [n,3] int64 on GPU
void sgd_step(const Tensor& chunks, const Tensor& pptr, const Tensor& gptr, const Tensor& bptr,
              const optional<Tensor>& sptr, const Tensor& lr, double momentum, double dampening,
              double wd, double grad_scale, bool nesterov, bool first, bool zero_grad) {
  TORCH_CHECK(chunks.is_cuda() && chunks.scalar_type() == at::kLong, "chunks");
  TORCH_CHECK(lr.is_cuda() && lr.scalar_type() == at::kFloat, "lr must be a GPU fp32 scalar");
  pca::sgd_launch(ptr<int64_t>(chunks), chunks.size(0), ptr<float* const>(pptr),
                  ptr<const float* const>(gptr), ptr<float* const>(bptr),
                  sptr.has_value() && sptr->defined() ? ptr<bf16* const>(*sptr) : nullptr,
                  ptr<float>(lr), (float)momentum, (float)dampening, (float)wd, (float)grad_scale,
                  nesterov ? 1 : 0, first ? 1 : 0, cur_stream(), zero_grad ? 1 : 0);
}

// optimizer step + bf16 operand refresh in one launch: `chunks` (SGD chunks of the arena ranges
// no conv operand is built from) + `pchunks` (WeightPrepPlan chunks over `desc`, whose masters
// are updated in place; gm[t] = {grad, momentum} of desc tensor t)
void sgd_prep_step(const Tensor& chunks, const Tensor& pptr, const Tensor& gptr, const Tensor& bptr,
                   const Tensor& lr, double momentum, double dampening, double wd,
                   double grad_scale, bool nesterov, bool first, const Tensor& desc,
                   const Tensor& pchunks, const Tensor& gm, bool zero_grad) {
  for (const Tensor* t : {&chunks, &pptr, &gptr, &bptr, &desc, &pchunks, &gm})
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kLong && t->is_contiguous(),
                "sgd_prep_step tables: contiguous int64 on the GPU");
  TORCH_CHECK(chunks.numel() == 0 || (chunks.dim() == 2 && chunks.size(1) == 3), "chunks [n][3]");
  TORCH_CHECK(pchunks.dim() == 2 && pchunks.size(1) == 4, "pchunks [n][4]");
  TORCH_CHECK(desc.dim() == 2 && desc.size(1) == 8 && gm.numel() == 2 * desc.size(0),
              "desc [t][8], gm [t][2]");
  check_f32(lr, "lr");
  pca::sgd_prep_launch(chunks.numel() ? ptr<int64_t>(chunks) : nullptr,
                       chunks.numel() ? (int)chunks.size(0) : 0, ptr<float* const>(pptr),
                       ptr<const float* const>(gptr), ptr<float* const>(bptr), ptr<float>(lr),
                       (float)momentum, (float)dampening, (float)wd, (float)grad_scale,
                       nesterov ? 1 : 0, first ? 1 : 0, ptr<int64_t>(desc), ptr<int64_t>(pchunks),
                       (int)pchunks.size(0), ptr<int64_t>(gm), cur_stream(), zero_grad ? 1 : 0);
}

Tensor se_scale_fwd(const Tensor& x, const Tensor& s) {
  check_bf16(x, "x");
  check_f32(s, "s");
  const int N = x.size(0), HW = x.size(1) * x.size(2), C = x.size(3);
  TORCH_CHECK(s.numel() == (int64_t)N * C, "excitation shape");
  auto out = at::empty_like(x);
  pca::se_scale_fwd_launch(ptr<bf16>(x), ptr<float>(s), N, HW, C, ptr<bf16>(out), cur_stream());
  return out;
}

std::vector<Tensor> se_scale_bwd(const Tensor& dout, const Tensor& x, const Tensor& s) {
  check_bf16(dout, "dout");
  check_bf16(x, "x");
  check_f32(s, "s");
  const int N = x.size(0), HW = x.size(1) * x.size(2), C = x.size(3);
  auto dx = at::empty_like(x);
  auto ds = at::empty({N, C}, s.options());
  pca::se_scale_bwd_launch(ptr<bf16>(dout), ptr<bf16>(x), ptr<float>(s), N, HW, C, ptr<bf16>(dx),
                           ptr<float>(ds), cur_stream());
  return {dx, ds};
}

// channel concat of NHWC bf16 tensors [N,H,W,C_i] (<= 8 pieces) -> [N,H,W,sum C_i]
Tensor cat_nhwc(const std::vector<Tensor>& xs) {
  TORCH_CHECK(!xs.empty() && xs.size() <= 8, "cat_nhwc: 1..8 inputs");
  pca::CatArgs a{};
  a.k = (int)xs.size();
  a.off[0] = 0;
  for (int j = 0; j < a.k; ++j) {
    check_bf16(xs[j], "x");
    TORCH_CHECK(xs[j].dim() == 4 && xs[j].size(0) == xs[0].size(0) && xs[j].size(1) == xs[0].size(1) &&
                    xs[j].size(2) == xs[0].size(2), "cat_nhwc: pixel mismatch");
    a.src[j] = ptr<bf16>(xs[j]);
    a.off[j + 1] = a.off[j] + (int)xs[j].size(3);
  }
  const int P = xs[0].size(0) * xs[0].size(1) * xs[0].size(2);
  auto out = at::empty({xs[0].size(0), xs[0].size(1), xs[0].size(2), a.off[a.k]}, xs[0].options());
  pca::cat_nhwc_launch(a, ptr<bf16>(out), P, false, cur_stream());
  return out;
}

// inverse: [N,H,W,sum C_i] -> pieces of widths `sizes`
std::vector<Tensor> split_nhwc(const Tensor& whole, const std::vector<int64_t>& sizes) {
  check_bf16(whole, "whole");
  TORCH_CHECK(!sizes.empty() && sizes.size() <= 8, "split_nhwc: 1..8 pieces");
  pca::CatArgs a{};
  a.k = (int)sizes.size();
  a.off[0] = 0;
  std::vector<Tensor> outs;
  for (int j = 0; j < a.k; ++j) {
    outs.push_back(at::empty({whole.size(0), whole.size(1), whole.size(2), sizes[j]}, whole.options()));
    a.dst[j] = ptr<bf16>(outs.back());
    a.off[j + 1] = a.off[j] + (int)sizes[j];
  }
  TORCH_CHECK(a.off[a.k] == whole.size(3), "split_nhwc: widths must sum to the channel count");
  const int P = whole.size(0) * whole.size(1) * whole.size(2);
  pca::cat_nhwc_launch(a, ptr<bf16>(whole), P, true, cur_stream());
  return outs;
}

// channel remap (group pad / unpad / shuffle and their adjoints): x viewed as [rows, Cin]
// (Cin = last dim), out [Q, J] with Q = rmap.numel() * K (outer row map) or rows; `acc` (fp32)
// is added into instead of allocating the output.
Tensor chan_remap(const Tensor& x, const Tensor& cmap, const optional<Tensor>& rmap, int64_t K,
                  const optional<Tensor>& acc, bool clear_src) {
  TORCH_CHECK(x.is_cuda() && x.is_contiguous(), "chan_remap: contiguous GPU input");
  const bool fp32 = x.scalar_type() == at::kFloat;
  TORCH_CHECK(fp32 || x.scalar_type() == at::kBFloat16, "chan_remap: bf16 or fp32");
  TORCH_CHECK(!clear_src || fp32, "chan_remap: clear_src is for fp32 gradient buffers");
  TORCH_CHECK(cmap.scalar_type() == at::kInt && cmap.is_cuda() && cmap.dim() == 1, "chan_remap: int32 cmap");
  const int64_t Cin = x.size(-1);
  const int64_t rows = Cin ? x.numel() / Cin : 0;
  const int* rm = optr<int>(rmap);
  int64_t Q = rows;
  if (rm) {
    TORCH_CHECK(rmap->scalar_type() == at::kInt && rmap->is_cuda(), "chan_remap: int32 rmap");
    TORCH_CHECK(K >= 1 && rows % K == 0, "chan_remap: rows must be a multiple of K");
    Q = rmap->numel() * K;
  }
  const int64_t J = cmap.numel();
  TORCH_CHECK(Q < (int64_t)1 << 31 && J > 0, "chan_remap: size");
  Tensor out;
  if (acc.has_value() && acc->defined()) {
    TORCH_CHECK(acc->scalar_type() == x.scalar_type() && acc->is_contiguous() && acc->numel() == Q * J,
                "chan_remap: accumulator of Q*J elements, the input's dtype");
    out = *acc;
  } else {
    out = at::empty({Q, J}, x.options());
  }
  if (Q > 0)
    pca::chan_remap_launch(x.data_ptr(), out.data_ptr(), fp32, acc.has_value() && acc->defined(),
                           ptr<int>(cmap), rm, (int)Q, (int)(rm ? K : 1), (int)Cin, (int)J, cur_stream(),
                           clear_src);
  return out;
}

// shuffle(cat[a, b], 2) for equal widths: a, b [N,H,W,C] -> [N,H,W,2C] interleaved; and back
Tensor interleave2(const Tensor& a, const Tensor& b) {
  check_bf16(a, "a");
  check_bf16(b, "b");
  TORCH_CHECK(a.sizes() == b.sizes() && a.dim() == 4, "interleave2: equal NHWC shapes");
  const int P = a.size(0) * a.size(1) * a.size(2), C = a.size(3);
  auto y = at::empty({a.size(0), a.size(1), a.size(2), 2 * C}, a.options());
  pca::interleave2_launch(ptr<bf16>(a), ptr<bf16>(b), ptr<bf16>(y), P, C, false, cur_stream());
  return y;
}

std::vector<Tensor> deinterleave2(const Tensor& y) {
  check_bf16(y, "y");
  TORCH_CHECK(y.dim() == 4 && y.size(3) % 2 == 0, "deinterleave2: even channel count");
  const int P = y.size(0) * y.size(1) * y.size(2), C = y.size(3) / 2;
  auto a = at::empty({y.size(0), y.size(1), y.size(2), C}, y.options());
  auto b = at::empty_like(a);
  pca::interleave2_launch(ptr<bf16>(a), ptr<bf16>(b), const_cast<bf16*>(ptr<bf16>(y)), P, C, true,
                          cur_stream());
  return {a, b};
}

// split(shuffle(cat[a, b], 2)) into its channel halves [lo, hi] (each [N,H,W,C]) in one pass:
// the ShuffleNetV2 join feeding the next block's SplitBlock; and its backward from [dlo, dhi]
static void check_halves(const Tensor& a, const Tensor& b, const char* what) {
  check_bf16(a, "a");
  check_bf16(b, "b");
  TORCH_CHECK(a.sizes() == b.sizes() && a.dim() == 4 && a.size(3) % 2 == 0, what,
              ": equal NHWC shapes with an even channel count");
}
// pad_hi > C: hi is returned as the channel prefix of a [N,H,W,pad_hi] buffer whose padding
// channels the kernel zeroes (a zero-padded conv input read in place)
std::vector<Tensor> interleave2_split(const Tensor& a, const Tensor& b, int64_t pad_hi) {
  check_halves(a, b, "interleave2_split");
  const int P = a.size(0) * a.size(1) * a.size(2), C = a.size(3);
  const int ldh = pad_hi > C ? (int)pad_hi : C;
  TORCH_CHECK(ldh == C || ldh % 8 == 0, "interleave2_split: padded width must be a multiple of 8");
  auto lo = at::empty_like(a);
  auto hib = at::empty({a.size(0), a.size(1), a.size(2), ldh}, a.options());
  pca::interleave2_launch(ptr<bf16>(a), ptr<bf16>(b), ptr<bf16>(lo), P, C, false, cur_stream(),
                          ptr<bf16>(hib), ldh);
  return {lo, ldh == C ? hib : hib.narrow(3, 0, C)};
}
std::vector<Tensor> deinterleave2_split(const Tensor& lo, const Tensor& hi) {
  check_bf16(lo, "lo");
  TORCH_CHECK(hi.is_cuda() && hi.scalar_type() == at::kBFloat16, "hi: bf16 GPU tensor");
  TORCH_CHECK(lo.is_contiguous() && lo.dim() == 4 && lo.size(3) % 2 == 0 && hi.sizes() == lo.sizes(),
              "deinterleave2_split: equal NHWC shapes with an even channel count");
  const int P = lo.size(0) * lo.size(1) * lo.size(2), C = lo.size(3);
  // hi: dense, or the channel prefix of wider rows (a padded conv input's gradient)
  const int64_t ldh = hi.stride(2);
  TORCH_CHECK(hi.stride(3) == 1 && ldh >= C && hi.stride(1) == hi.size(2) * ldh &&
                  hi.stride(0) == hi.size(1) * hi.stride(1),
              "deinterleave2_split: hi must be dense or row-strided NHWC");
  auto a = at::empty_like(lo), b = at::empty_like(lo);
  pca::interleave2_launch(ptr<bf16>(a), ptr<bf16>(b), const_cast<bf16*>(ptr<bf16>(lo)), P, C, true,
                          cur_stream(), ptr<bf16>(hi), (int)ldh);
  return {a, b};
}

// DPN dual-path merge: x [N,H,W,Cx], o [N,H,W,Co] NHWC bf16 -> relu(cat[x[:d]+o[:d], x[d:], o[d:]])
Tensor dpn_merge_fwd(const Tensor& x, const Tensor& o, int d) {
  check_bf16(x, "x");
  check_bf16(o, "o");
  const int Cx = x.size(3), Co = o.size(3);
  TORCH_CHECK(x.size(0) == o.size(0) && x.size(1) == o.size(1) && x.size(2) == o.size(2), "dpn_merge: pixel mismatch");
  TORCH_CHECK(d % 8 == 0 && Cx % 8 == 0 && Co % 8 == 0 && d <= Cx && d <= Co, "dpn_merge: channels must be multiples of 8");
  const int P = x.size(0) * x.size(1) * x.size(2);
  auto y = at::empty({x.size(0), x.size(1), x.size(2), Cx + Co - d}, x.options());
  pca::dpn_merge_fwd_launch(ptr<bf16>(x), ptr<bf16>(o), P, Cx, Co, d, ptr<bf16>(y), cur_stream());
  return y;
}

std::vector<Tensor> dpn_merge_bwd(const Tensor& dy, const Tensor& y, int Cx, int Co, int d) {
  check_bf16(dy, "dy");
  check_bf16(y, "y");
  TORCH_CHECK(dy.sizes() == y.sizes() && y.size(3) == Cx + Co - d, "dpn_merge_bwd: shape");
  const int P = y.size(0) * y.size(1) * y.size(2);
  auto dx = at::empty({y.size(0), y.size(1), y.size(2), Cx}, y.options());
  auto dout = at::empty({y.size(0), y.size(1), y.size(2), Co}, y.options());
  pca::dpn_merge_bwd_launch(ptr<bf16>(dy), ptr<bf16>(y), P, Cx, Co, d, ptr<bf16>(dx),
                            ptr<bf16>(dout), cur_stream());
  return {dx, dout};
}

Tensor act_fwd(const Tensor& x, int act) {
  check_bf16(x, "x");
  auto y = at::empty_like(x);
  pca::act_fwd_launch(ptr<bf16>(x), x.numel(), act, ptr<bf16>(y), cur_stream());
  return y;
}

Tensor act_bwd(const Tensor& dy, const Tensor& x, int act) {
  check_bf16(dy, "dy");
  check_bf16(x, "x");
  auto dx = at::empty_like(x);
  pca::act_bwd_launch(ptr<bf16>(dy), ptr<bf16>(x), x.numel(), act, ptr<bf16>(dx), cur_stream());
  return dx;
}

Tensor add_act(const Tensor& a, const Tensor& b, int act) {
  check_bf16(a, "a");
  check_bf16(b, "b");
  TORCH_CHECK(a.sizes() == b.sizes(), "add shape mismatch");
  auto y = at::empty_like(a);
  pca::add_act_launch(ptr<bf16>(a), ptr<bf16>(b), a.numel(), act, ptr<bf16>(y), cur_stream());
  return y;
}

// ---------------------------------------------------------------------------- dwconv
// wT fp32 [KH*KW, Cout]
Tensor dw_fwd(const Tensor& x, const Tensor& wT, int KH, int KW, int stride, int pad) {
  check_bf16(x, "x");
  check_f32(wT, "wT");
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  const int Co = wT.size(1);
  TORCH_CHECK(wT.size(0) == KH * KW && Co % C == 0, "depthwise weight shape");
  const int Ho = out_dim(H, KH, stride, pad), Wo = out_dim(W, KW, stride, pad);
  auto y = at::empty({N, Ho, Wo, Co}, x.options());
  pca::dw_fwd_launch(ptr<bf16>(x), ptr<float>(wT), N, H, W, C, Ho, Wo, Co, KH, KW, stride, pad,
                     ptr<bf16>(y), cur_stream());
  return y;
}

Tensor dw_dgrad(const Tensor& dy, const Tensor& wT, int H, int W, int C, int KH, int KW, int stride,
                int pad) {
  check_bf16(dy, "dy");
  check_f32(wT, "wT");
  const int N = dy.size(0), Ho = dy.size(1), Wo = dy.size(2), Co = dy.size(3);
  TORCH_CHECK(out_dim(H, KH, stride, pad) == Ho && out_dim(W, KW, stride, pad) == Wo, "geometry");
  auto dx = at::empty({N, H, W, C}, dy.options());
  pca::dw_dgrad_launch(ptr<bf16>(dy), ptr<float>(wT), N, H, W, C, Ho, Wo, Co, KH, KW, stride, pad,
                       ptr<bf16>(dx), cur_stream());
  return dx;
}

// forward + the consumer BN's statistics added into its zeroed sharded accumulator
// [rows][2][Co]; returns {y, flag} with flag = 1 when the fused kernel ran (else nothing added)
std::vector<Tensor> dw_fwd_stats(const Tensor& x, const Tensor& wT, int KH, int KW, int stride,
                                 int pad, const Tensor& acc, int acc_rows) {
  check_bf16(x, "x");
  check_f32(wT, "wT");
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  const int Co = wT.size(1);
  TORCH_CHECK(wT.size(0) == KH * KW, "wT [KH*KW][Co]");
  const int Ho = out_dim(H, KH, stride, pad), Wo = out_dim(W, KW, stride, pad);
  check_acc(acc, acc_rows, 2, Co);
  auto y = at::empty({N, Ho, Wo, Co}, x.options());
  const bool ok = pca::dw_fwd_stats_launch(ptr<bf16>(x), ptr<float>(wT), N, H, W, C, Ho, Wo, Co,
                                           KH, KW, stride, pad, ptr<bf16>(y), ptr<float>(acc),
                                           acc_rows, cur_stream());
  if (!ok)
    pca::dw_fwd_launch(ptr<bf16>(x), ptr<float>(wT), N, H, W, C, Ho, Wo, Co, KH, KW, stride, pad,
                       ptr<bf16>(y), cur_stream());
  return {y, at::full({1}, ok ? 1 : 0, x.options().dtype(at::kInt).device(at::kCPU))};
}

// dgrad + the backward reduce of the BN(+act) that produced x, added into that BN's zeroed
// backward accumulator [rows][2][C] (act 1: ReLU via the 1-bit mask, 2: swish via aux rows
// scale | shift); returns {dx, flag}
std::vector<Tensor> dw_dgrad_bn(const Tensor& dy, const Tensor& wT, int H, int W, int C, int KH,
                                int KW, int stride, int pad, const Tensor& bn_y,
                                const optional<Tensor>& bn_mask, const Tensor& bn_aux, int act,
                                const Tensor& acc, int acc_rows) {
  check_bf16(dy, "dy");
  check_f32(wT, "wT");
  check_bf16(bn_y, "bn_y");
  check_f32(bn_aux, "bn_aux");
  const int N = dy.size(0), Ho = dy.size(1), Wo = dy.size(2), Co = dy.size(3);
  TORCH_CHECK(out_dim(H, KH, stride, pad) == Ho && out_dim(W, KW, stride, pad) == Wo, "geometry");
  TORCH_CHECK(bn_y.numel() == (int64_t)N * H * W * C && bn_y.is_contiguous(), "bn_y must match dx");
  TORCH_CHECK(bn_aux.numel() >= (act == 2 ? 4 : 2) * C, "bn_aux [mean|istd|scale|shift][C]");
  const bool has_mask = bn_mask.has_value() && bn_mask->defined();
  if (has_mask)
    TORCH_CHECK(bn_mask->scalar_type() == at::kByte && bn_mask->numel() * 8 == bn_y.numel(),
                "bn_mask: one bit per element");
  check_acc(acc, acc_rows, 2, C);
  auto dx = at::empty({N, H, W, C}, dy.options());
  const bool ok = pca::dw_dgrad_bn_launch(
      ptr<bf16>(dy), ptr<float>(wT), N, H, W, C, Ho, Wo, Co, KH, KW, stride, pad, ptr<bf16>(dx),
      ptr<bf16>(bn_y), has_mask ? bn_mask->data_ptr<uint8_t>() : nullptr, ptr<float>(bn_aux), act,
      ptr<float>(acc), acc_rows, cur_stream());
  if (!ok)
    pca::dw_dgrad_launch(ptr<bf16>(dy), ptr<float>(wT), N, H, W, C, Ho, Wo, Co, KH, KW, stride, pad,
                         ptr<bf16>(dx), cur_stream());
  return {dx, at::full({1}, ok ? 1 : 0, dy.options().dtype(at::kInt).device(at::kCPU))};
}

// ---- depthwise with the producer BN(+act) applied on the input loads (the BN output is never
// written): y = the BN input, aux = its [mean | istd | scale | shift] rows, act 1 relu / 2 swish
bool dw_in_supported_t(const Tensor& y, int Co, int KH, int KW, int stride, int pad, int act) {
  const int N = y.size(0), H = y.size(1), W = y.size(2), C = y.size(3);
  return pca::dw_in_supported(N, H, W, C, out_dim(H, KH, stride, pad), out_dim(W, KW, stride, pad),
                              Co, KH, KW, stride, pad, act);
}

Tensor dw_fwd_in(const Tensor& y, const Tensor& wT, int KH, int KW, int stride, int pad,
                 const Tensor& aux, int act) {
  check_bf16(y, "y");
  check_f32(wT, "wT");
  check_f32(aux, "aux");
  const int N = y.size(0), H = y.size(1), W = y.size(2), C = y.size(3);
  const int Co = wT.size(1);
  TORCH_CHECK(wT.size(0) == KH * KW && Co == C, "depthwise (multiplier 1) weight shape");
  TORCH_CHECK(aux.numel() >= 4 * C, "aux [mean|istd|scale|shift][C]");
  const int Ho = out_dim(H, KH, stride, pad), Wo = out_dim(W, KW, stride, pad);
  TORCH_CHECK(pca::dw_in_supported(N, H, W, C, Ho, Wo, Co, KH, KW, stride, pad, act),
              "dw_fwd_in: unsupported geometry / activation");
  auto out = at::empty({N, Ho, Wo, Co}, y.options());
  const float* a = ptr<float>(aux);
  pca::dw_fwd_in_launch(ptr<bf16>(y), ptr<float>(wT), N, H, W, C, Ho, Wo, Co, KH, KW, stride, pad,
                        a + 2 * C, a + 3 * C, act, ptr<bf16>(out), cur_stream());
  return out;
}

Tensor dw_wgrad_in(const Tensor& y, const Tensor& dy, int KH, int KW, int stride, int pad,
                   const Tensor& aux, int act, const optional<Tensor>& accum) {
  check_bf16(y, "y");
  check_bf16(dy, "dy");
  check_f32(aux, "aux");
  const int N = y.size(0), H = y.size(1), W = y.size(2), C = y.size(3);
  const int Ho = dy.size(1), Wo = dy.size(2), Co = dy.size(3);
  TORCH_CHECK(out_dim(H, KH, stride, pad) == Ho && out_dim(W, KW, stride, pad) == Wo, "geometry");
  TORCH_CHECK(pca::dw_in_supported(N, H, W, C, Ho, Wo, Co, KH, KW, stride, pad, act),
              "dw_wgrad_in: unsupported geometry / activation");
  TORCH_CHECK(aux.numel() >= 4 * C, "aux [mean|istd|scale|shift][C]");
  const int chunks = pca::dw_wgrad_partials(N, Ho, Wo);
  auto fopt = y.options().dtype(at::kFloat);
  auto partial = at::empty({chunks, KH * KW, Co}, fopt);
  const bool acc = accum.has_value() && accum->defined();
  Tensor dw = acc ? *accum : at::empty({Co, KH * KW}, fopt);
  if (acc)
    TORCH_CHECK(dw.scalar_type() == at::kFloat && dw.is_contiguous() && dw.numel() == (int64_t)Co * KH * KW,
                "dw_wgrad_in: accum must be a contiguous fp32 [Co*KH*KW] tensor");
  const float* a = ptr<float>(aux);
  pca::dw_wgrad_in_launch(ptr<bf16>(y), ptr<bf16>(dy), N, H, W, C, Ho, Wo, Co, KH, KW, stride, pad,
                          a + 2 * C, a + 3 * C, act, ptr<float>(partial), chunks, acc ? 1 : 0,
                          ptr<float>(dw), cur_stream());
  return dw;
}

// returns dw fp32 [Cout, KH*KW]
// dW [Co, KH*KW] fp32; with `accum` given (fp32, Co*KH*KW contiguous, e.g. the parameter's view
// of the gradient arena) the result is added into it by the final reduce and `accum` returned
Tensor dw_wgrad(const Tensor& x, const Tensor& dy, int KH, int KW, int stride, int pad,
                const optional<Tensor>& accum) {
  check_bf16(x, "x");
  check_bf16(dy, "dy");
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  const int Ho = dy.size(1), Wo = dy.size(2), Co = dy.size(3);
  TORCH_CHECK(out_dim(H, KH, stride, pad) == Ho && out_dim(W, KW, stride, pad) == Wo, "geometry");
  const int chunks = pca::dw_wgrad_partials(N, Ho, Wo);
  auto fopt = x.options().dtype(at::kFloat);
  auto partial = at::empty({chunks, KH * KW, Co}, fopt);
  Tensor dw;
  if (accum.has_value() && accum->defined()) {
    dw = *accum;
    TORCH_CHECK(dw.scalar_type() == at::kFloat && dw.is_contiguous() && dw.numel() == (int64_t)Co * KH * KW &&
                    dw.device() == x.device(),
                "dw_wgrad: accum must be a contiguous fp32 [Co*KH*KW] tensor on the input's device");
  } else {
    dw = at::empty({Co, KH * KW}, fopt);
  }
  pca::dw_wgrad_launch(ptr<bf16>(x), ptr<bf16>(dy), N, H, W, C, Ho, Wo, Co, KH, KW, stride, pad,
                       ptr<float>(partial), chunks, accum.has_value() && accum->defined() ? 1 : 0,
                       ptr<float>(dw), cur_stream());
  return dw;
}

// ------------------------------------------------------------------------- direct conv
// w fp32 [Cout, KH, KW, Cin/G] contiguous (physical layout of the channels_last parameter)
Tensor direct_fwd(const Tensor& x, const Tensor& w, const optional<Tensor>& bias, int stride,
                  int pad, int groups) {
  check_bf16(x, "x");
  check_f32(w, "w");
  const int N = x.size(0), H = x.size(1), W = x.size(2), Cin = x.size(3);
  const int Cout = w.size(0), KH = w.size(1), KW = w.size(2);
  TORCH_CHECK(w.size(3) * groups == Cin && Cout % groups == 0, "direct conv weight shape");
  const int Ho = out_dim(H, KH, stride, pad), Wo = out_dim(W, KW, stride, pad);
  TORCH_CHECK(Ho > 0 && Wo > 0, "empty conv output");
  auto y = at::empty({N, Ho, Wo, Cout}, x.options());
  pca::direct_fwd_launch(ptr<bf16>(x), ptr<float>(w), optr<float>(bias), N, H, W, Cin, Ho, Wo, Cout,
                         KH, KW, stride, pad, groups, ptr<bf16>(y), cur_stream());
  return y;
}

Tensor direct_dgrad(const Tensor& dy, const Tensor& w, int H, int W, int stride, int pad,
                    int groups) {
  check_bf16(dy, "dy");
  check_f32(w, "w");
  const int N = dy.size(0), Ho = dy.size(1), Wo = dy.size(2), Cout = dy.size(3);
  const int KH = w.size(1), KW = w.size(2), Cin = w.size(3) * groups;
  TORCH_CHECK(w.size(0) == Cout, "direct dgrad weight shape");
  TORCH_CHECK(out_dim(H, KH, stride, pad) == Ho && out_dim(W, KW, stride, pad) == Wo, "geometry");
  auto dx = at::empty({N, H, W, Cin}, dy.options());
  pca::direct_dgrad_launch(ptr<bf16>(dy), ptr<float>(w), N, H, W, Cin, Ho, Wo, Cout, KH, KW, stride,
                           pad, groups, ptr<bf16>(dx), cur_stream());
  return dx;
}

// returns fp32 [Cout*KH*KW*Cin/G + (bias ? Cout : 0)]
Tensor direct_wgrad(const Tensor& x, const Tensor& dy, int KH, int KW, int stride, int pad,
                    int groups, bool with_bias) {
  check_bf16(x, "x");
  check_bf16(dy, "dy");
  const int N = x.size(0), H = x.size(1), W = x.size(2), Cin = x.size(3);
  const int Ho = dy.size(1), Wo = dy.size(2), Cout = dy.size(3);
  TORCH_CHECK(out_dim(H, KH, stride, pad) == Ho && out_dim(W, KW, stride, pad) == Wo, "geometry");
  const int tot = Cout * KH * KW * (Cin / groups) + (with_bias ? Cout : 0);
  const int splits = pca::direct_wgrad_splits(N, Ho, Wo, tot);
  auto fopt = x.options().dtype(at::kFloat);
  auto partial = at::empty({splits, tot}, fopt);
  auto out = at::empty({tot}, fopt);
  pca::direct_wgrad_launch(ptr<bf16>(x), ptr<bf16>(dy), N, H, W, Cin, Ho, Wo, Cout, KH, KW, stride,
                           pad, groups, with_bias ? 1 : 0, ptr<float>(partial), splits,
                           ptr<float>(out), cur_stream());
  return out;
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "pytorch_cifar_amd gfx950 kernels";
  m.def("set_deterministic", &pca::set_deterministic_conv,
        "weight gradients reduced through ordered slab rows (no fp32 atomics): bitwise-reproducible");
  m.def("deterministic", &pca::deterministic_conv);
  m.def("last_error", []() {
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? std::string() : std::string(hipGetErrorString(e));
  }, "hipGetLastError() of this thread as a string ('' = no error); clears it");
  m.def("conv_fwd", &conv_fwd, py::arg("x"), py::arg("wb"), py::arg("bias"), py::arg("stride"),
        py::arg("pad"), py::arg("groups"), py::arg("want_stats"), py::arg("stat_acc") = py::none(),
        py::arg("acc_rows") = 0, py::arg("stat_shift") = py::none(), py::arg("xf") = py::none(),
        py::arg("xf_mask") = py::none(),
        "xf (BN aux [mean|istd|scale|shift][Cin]) + xf_mask: x is the pre-BN y and relu(BN(y)) is "
        "applied on the loads (layer-1 c64 forward only), its 1-bit ReLU mask written to xf_mask");
  m.def("conv_xf_supported", &conv_xf_supported, py::arg("x"), py::arg("wb"), py::arg("stride"),
        py::arg("pad"), py::arg("groups"),
        "can conv_fwd / conv_wgrad apply the producing BN+ReLU on their operand loads here?");
  m.def("conv_dgrad", &conv_dgrad, py::arg("dy"), py::arg("wt"), py::arg("H"), py::arg("W"),
        py::arg("stride"), py::arg("pad"), py::arg("groups"), py::arg("addend") = py::none(),
        py::arg("addend_s2c") = false);
  m.def("conv_dgrad_bn", &conv_dgrad_impl, py::arg("dy"), py::arg("wt"), py::arg("H"),
        py::arg("W"), py::arg("stride"), py::arg("pad"), py::arg("groups"), py::arg("addend"),
        py::arg("bn_y"), py::arg("bn_mask"), py::arg("bn_aux"), py::arg("bn_acc") = py::none(),
        py::arg("acc_rows") = 0, py::arg("bn_y2") = py::none(), py::arg("bn_aux2") = py::none(),
        py::arg("addend_s2c") = false,
        "dgrad + fused backward reduce of the producing BN+ReLU -> (dx, partial[rows][2][C]); "
        "with bn_y2 / bn_aux2 (dual BN, accumulator mode) the accumulator gets [R][3][C] sums");
  m.def("conv_wgrad", &conv_wgrad, py::arg("x"), py::arg("dy"), py::arg("KH"), py::arg("KW"),
        py::arg("stride"), py::arg("pad"), py::arg("groups"), py::arg("out"),
        py::arg("defer") = false, py::arg("xf") = py::none());
  m.def("wgrad_piggy", &wgrad_piggy, "pending wgrad slab reductions ride along in the next fused BN-backward launch");
  m.def("wgrad_flush", &wgrad_flush,
        "launch every deferred weight-gradient slab reduction (one batched kernel); returns count");
  m.def("wgrad_deferred", &pca::wgrad_deferred_count, "pending deferred slab reductions");
  m.def("conv_autotune", [](bool on) { g_autotune = on; }, "enable/disable conv tile autotuning");
  m.def("conv_autotune_enabled", []() { return g_autotune; });
  m.def("c64_set_prof", [](const optional<Tensor>& t) {
    if (t.has_value() && t->defined()) {
      TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kLong && t->is_contiguous(), "int64 device tensor");
      pca::c64_set_prof(t->data_ptr<int64_t>());
    } else {
      pca::c64_set_prof(nullptr);
    }
  }, "diagnostics: record c64 per-wave tile stamps into t ([grid][4][16][4] int64) or stop");
  m.def("c64_grid_size", &pca::c64_grid_size);
  m.def("c64_version", &pca::c64_version,
        "layer-1 c64 kernel version (2: 16x16x32 MFMA, 3: 32x32x16 plane layout); v < 0 only "
        "queries; returns the previous version");
  m.def("tune_export", &pca::tune_export, "autotuned conv / wgrad choices as int rows");
  // bump when a kernel candidate set or a cfg numbering changes: shipped tune tables
  // (engine/tuning.py) made for another set are then ignored
  m.def("tune_version", []() { return 5; }, "version of the autotuner's candidate sets");
  m.def("tune_import", &pca::tune_import, "restore rows from tune_export (returns rows taken)");
  m.def("src_digest", []() { return std::string(pca_src_digest); },
        "sha256 of the csrc sources this library was built from (_build.source_digest)");
  m.def("conv_trial", [](int kind, int cfg, int split) {
    if (kind == 0) pca::conv_set_trial(cfg, split);
    else pca::wgrad_set_trial(cfg, split);
  }, "force an autotune candidate (kind 0 fwd/dgrad, 1 wgrad); (-1, -1) clears");
  m.def("wgrad_candidates", &pca::wgrad_tune_candidates);
  m.def("igemm_candidates", &pca::conv_tune_candidates);
  m.def("conv_tuned_count", []() { return pca::conv_tuned_count() + pca::wgrad_tuned_count(); });
  m.def("conv_clear_tuned", []() {
    pca::conv_clear_tuned();
    pca::wgrad_clear_tuned();
  });
  m.def("set_conv_tile", &pca::set_conv_tile, "override tile config (kind 0: fwd/dgrad, 1: wgrad; -1 = heuristic)");
  m.def("weight_prep", &weight_prep);
  m.def("weight_prep_multi", &weight_prep_multi);
  m.def("bn_stats", &bn_stats);
  m.def("bn_stats_centered", &bn_stats_centered,
        "BN sums of x - x[0] (robust variance) -> (partial [P][2][C], K [C])");
  m.def("bn_acc_max_elems", &acc_max_elems,
        "largest tensor whose BN sums a separate pass adds into an accumulator");
  m.def("bn_stats_acc", &bn_stats_acc, "BN sums of a bare tensor into a sharded accumulator");
  m.def("bn_rows_max_c", &pca::bn_rows_max_c,
        "widest C of the row-tiled BN kernels (0: disabled); row-strided BN operands need them");
  m.def("bias_grad", &bias_grad, py::arg("dy"), py::arg("accum") = py::none());
  m.def("bn_finalize", &bn_finalize, py::arg("partial"), py::arg("count"), py::arg("gamma"),
        py::arg("beta"), py::arg("rmean"), py::arg("rvar"), py::arg("nbt"), py::arg("momentum"),
        py::arg("eps"), py::arg("training"), py::arg("update_running"), py::arg("kin") = py::none(),
        py::arg("pilot_out") = py::none(), py::arg("zero") = py::none());
  m.def("bn_apply", &bn_apply, py::arg("y"), py::arg("aux"), py::arg("res"), py::arg("y2"),
        py::arg("aux2"), py::arg("act"), py::arg("want_mask"), py::arg("out") = py::none());
  m.def("bn_backward", &bn_backward, py::arg("dout"), py::arg("out"), py::arg("mask"), py::arg("y"),
        py::arg("aux"), py::arg("gamma"), py::arg("y2"), py::arg("aux2"), py::arg("gamma2"),
        py::arg("act"), py::arg("training"), py::arg("need_dres"), py::arg("dgamma_acc"),
        py::arg("dbeta_acc"), py::arg("dgamma2_acc"), py::arg("dbeta2_acc"),
        py::arg("partial_in") = py::none(), py::arg("acc") = py::none(), py::arg("acc_rows") = 0,
        py::arg("acc_filled") = false, py::arg("zero1") = py::none(),
        py::arg("zero2") = py::none(), py::arg("dx_out") = py::none(), py::arg("dx_acc") = false,
        py::arg("dbias_acc") = py::none());
  m.def("bn_apply_acc", &bn_apply_acc, py::arg("y"), py::arg("acc"), py::arg("R"),
        py::arg("count"), py::arg("gamma"), py::arg("beta"), py::arg("rmean"), py::arg("rvar"),
        py::arg("nbt"), py::arg("momentum"), py::arg("eps"), py::arg("res"), py::arg("y2"),
        py::arg("acc2"), py::arg("R2"), py::arg("gamma2"), py::arg("beta2"), py::arg("rmean2"),
        py::arg("rvar2"), py::arg("nbt2"), py::arg("momentum2"), py::arg("eps2"), py::arg("act"),
        py::arg("want_mask"), py::arg("zero") = py::none(), py::arg("shifted") = false,
        py::arg("pilot") = py::none(), py::arg("shifted2") = false, py::arg("pilot2") = py::none(),
        py::arg("out") = py::none(), py::arg("acc_off") = 0, py::arg("acc_ld") = 0,
        "training BN(+act/+res/+BN2) with the finalize folded in from sharded accumulators");
  m.def("conv_nk_min_m", [](int64_t v) { return pca::conv_nk_min_m(v); }, py::arg("v") = -1,
        "pixel count from which 1x1 narrow-K forwards take conv1x1_nk (returns the previous)");
  m.def("zero_", &zero_, "t <- 0 (runtime fill on the current stream)");
  m.def("bn_stats_copy", &bn_stats_copy, py::arg("src"), py::arg("dst"), py::arg("acc"),
        py::arg("acc_off"), py::arg("acc_ld"), py::arg("R"),
        "dst <- src (NHWC rows) with the channels' centred sums added into a wider sharded cache");
  m.def("nchw_to_nhwc", &nchw_to_nhwc);
  m.def("copy_rows", &copy_rows, "dst <- src for NHWC tensors, either a row-strided channel slice");
  m.def("winograd_filter", &winograd_filter, "U = G g G^T: fp32 [Co][3][3][Ci] -> bf16 [16][Co][Ci]");
  m.def("winograd_fwd", &winograd_fwd, py::arg("x"), py::arg("U"), py::arg("want_stats") = false,
        "fused Winograd F(2x2,3x3) 3x3/s1/p1 forward -> (y, BN partial sums [rows][2][Co])");
  m.def("winograd_applicable", &pca::winograd_applicable);
  m.def("add_rows", &add_rows, "dst <- src + add for NHWC tensors (each dense or row-strided)");
  m.def("nhwc_to_nchw", &nhwc_to_nchw);
  m.def("augment", &augment);
  m.def("augment_packed", &augment_packed);
  m.def("stem_wgrad", &stem_wgrad);
  m.def("gap_fwd", &gap_fwd);
  m.def("se_supported", &pca::se_mlp_supported, "fused squeeze-excite path for (C, R)?");
  m.def("se_forward", &se_forward, py::arg("x"), py::arg("w1"), py::arg("b1"), py::arg("w2"),
        py::arg("b2"), py::arg("act"), py::arg("w2t") = py::none(),
        "squeeze-excite: pool + MLP + sigmoid scale (NHWC bf16); with w2t ([R][C]) the fused kernels");
  m.def("se_backward", &se_backward, py::arg("dout"), py::arg("x"), py::arg("pooled"),
        py::arg("hpre"), py::arg("s"), py::arg("w1"), py::arg("w2"), py::arg("act"),
        py::arg("dw1_acc"), py::arg("db1_acc"), py::arg("dw2_acc"), py::arg("db2_acc"),
        py::arg("want_b1"), py::arg("want_b2"), py::arg("w2t") = py::none());
  m.def("se_fused_mode", &se_fused_mode, py::arg("mode"),
        "squeeze-excite kernels: 1 fused (2 + 3 launches), 0 split, -1 PCA_SE_FUSED; returns previous");
  m.def("head_fwd", &head_fwd, py::arg("x"), py::arg("w"), py::arg("b"), py::arg("p") = 0.0,
        py::arg("rng") = py::none(),
        "fused global-average-pool [+ Philox dropout] + Linear -> (logits, pooled, keep mask)");
  m.def("head_bwd", &head_bwd, py::arg("dl"), py::arg("w"), py::arg("pooled"), py::arg("H"),
        py::arg("W"), py::arg("dw_acc") = py::none(), py::arg("db_acc") = py::none(),
        py::arg("want_db") = true, py::arg("p") = 0.0, py::arg("dmask") = py::none(),
        py::arg("bn_y") = py::none(), py::arg("bn_mask") = py::none(), py::arg("bn_aux") = py::none(),
        py::arg("bn_acc") = py::none(), py::arg("acc_rows") = 0);
  m.def("dropout_fwd", &dropout_fwd, "Philox dropout / drop-connect -> (y, keep mask per unit)");
  m.def("dropout_bwd", &dropout_bwd, "dropout / drop-connect gradient from the keep mask");
  m.def("head_supported", [](int N, int C, int K) {
    return pca::head_supported(C, K) && pca::head_batch_supported(N, K);
  });
  m.def("gap_bwd", &gap_bwd);
  m.def("avgpool_fwd", &avgpool_fwd);
  m.def("avgpool_bwd", &avgpool_bwd);
  m.def("maxpool_fwd", &maxpool_fwd);
  m.def("maxpool_bwd", &maxpool_bwd);
  m.def("ce_fused", &ce_fused);
  m.def("scale_by_scalar", &scale_by_scalar);
  m.def("dw_fwd_stats", &dw_fwd_stats);
  m.def("dw_dgrad_bn", &dw_dgrad_bn);
  m.def("sgd_step", &sgd_step, py::arg("chunks"), py::arg("pptr"), py::arg("gptr"), py::arg("bptr"),
        py::arg("sptr"), py::arg("lr"), py::arg("momentum"), py::arg("dampening"), py::arg("wd"),
        py::arg("grad_scale"), py::arg("nesterov"), py::arg("first"), py::arg("zero_grad") = false);
  m.def("sgd_prep_step", &sgd_prep_step, py::arg("chunks"), py::arg("pptr"), py::arg("gptr"),
        py::arg("bptr"), py::arg("lr"), py::arg("momentum"), py::arg("dampening"), py::arg("wd"),
        py::arg("grad_scale"), py::arg("nesterov"), py::arg("first"), py::arg("desc"),
        py::arg("pchunks"), py::arg("gm"), py::arg("zero_grad") = false);
  m.def("se_scale_fwd", &se_scale_fwd);
  m.def("se_scale_bwd", &se_scale_bwd);
  m.def("dpn_merge_fwd", &dpn_merge_fwd);
  m.def("cat_nhwc", &cat_nhwc);
  m.def("interleave2", &interleave2);
  m.def("chan_remap", &chan_remap, py::arg("x"), py::arg("cmap"), py::arg("rmap") = py::none(),
        py::arg("K") = 1, py::arg("acc") = py::none(), py::arg("clear_src") = false);
  m.def("deinterleave2", &deinterleave2);
  m.def("interleave2_split", &interleave2_split, py::arg("a"), py::arg("b"), py::arg("pad_hi") = 0);
  m.def("deinterleave2_split", &deinterleave2_split);
  m.def("split_nhwc", &split_nhwc);
  m.def("dpn_merge_bwd", &dpn_merge_bwd);
  m.def("act_fwd", &act_fwd);
  m.def("act_bwd", &act_bwd);
  m.def("add_act", &add_act);
  m.def("dw_fwd", &dw_fwd);
  m.def("dw_in_supported", &dw_in_supported_t);
  m.def("dw_fwd_in", &dw_fwd_in, "depthwise conv of act(BN(y)) with the BN applied on the loads");
  m.def("dw_wgrad_in", &dw_wgrad_in, py::arg("y"), py::arg("dy"), py::arg("KH"), py::arg("KW"),
        py::arg("stride"), py::arg("pad"), py::arg("aux"), py::arg("act"),
        py::arg("accum") = py::none());
  m.def("dw_dgrad", &dw_dgrad);
  m.def("dw_wgrad", &dw_wgrad, py::arg("x"), py::arg("dy"), py::arg("KH"), py::arg("KW"),
        py::arg("stride"), py::arg("pad"), py::arg("accum") = py::none());
  m.def("direct_fwd", &direct_fwd);
  m.def("direct_dgrad", &direct_dgrad);
  m.def("direct_wgrad", &direct_wgrad);
  pca::register_comm(m);
}
