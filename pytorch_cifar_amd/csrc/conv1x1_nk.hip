// Narrow-K 1x1 convolution forward: the expand convs of the inverted-residual blocks (reference
// models/mobilenetv2.py:25-35 conv1, models/efficientnet.py:63-71 expand conv; K = 16 / 24 / 32 /
// 40 input channels, Cout = 6K output channels).
//
// With one 64-deep K step per tile the generic implicit GEMM is a serial chain per tile (operand
// DMA -> MFMA -> LDS epilogue -> stores) and lands at ~2.8x the bytes floor on these shapes
// (MobileNetV2 bs1024 24->144: 166-170 us for 352 MB). Here the whole weight matrix sits in LDS
// once per workgroup, each wave walks 16-pixel groups with the next group's input fragment in
// flight, and the MFMA is issued as W x X^T: lane (r, kq) holds pixel r's K-chunk kq as the B
// operand and gets back four consecutive output channels of pixel r, stored straight from
// registers (8 bytes per lane, every pixel row written whole by the wave) — no LDS round trip,
// no barrier in the pixel loop. BatchNorm statistics (shifted sums, common.h stat_shift) of the
// stored bf16 values accumulate in registers and leave once per workgroup (stat_out).
#include "mfma_util.h"

#include <algorithm>
#include <cstdlib>

namespace pca {

int stat_shards();
const float* stat_shift();

// The same GEMM shape is the data gradient of a narrow-output 1x1 conv (the inverted-residual
// project conv, Cout = K: dX[M][CO] = dY[M][K] . W^T with W^T = its [CO][K] dgrad operand). DGRAD
// replaces the statistics epilogue by the dgrad one: the residual addend, and the fused backward
// reduce of the BatchNorm(+ReLU) that produced the conv input (sums of dz = dX * relu'(mask) and
// dz * (y - mean), istd applied at the flush: the igemm dgrad epilogue's slab-row / sharded form).
struct NkBn {
  const bf16* addend;
  const bf16* y;            // that BN's input (its mean | istd in aux)
  const uint8_t* mask;      // its 1-bit ReLU mask (all ones for a BN without activation)
  const float* aux;
  float* part;              // [rows][2][CO] slab rows, or the sharded accumulator
};

template <int KS, int CT, bool STG, bool DGRAD>
__global__ __launch_bounds__(256) void conv1x1_nk_kernel(const bf16* __restrict__ x,
                                                         const bf16* __restrict__ w,
                                                         bf16* __restrict__ y, int M, int K,
                                                         float* __restrict__ stats, int shards,
                                                         const float* __restrict__ kshift,
                                                         NkBn bn) {
  constexpr int CO = CT * 16;
  constexpr int KP = KS * 32;   // zero-padded reduction width (MFMA K steps of 32)
  __shared__ __attribute__((aligned(16))) bf16 ws[CO * KP];
  __shared__ float kks[CO];     // forward: the statistics shift; dgrad: the BN mean
  __shared__ float kis[DGRAD ? CO : 1];   // dgrad: the BN istd
  __shared__ float red[4][2][CO];
  // STG: each wave's 16 x CO output tile is staged in a private LDS region and leaves as whole
  // contiguous 16-byte row pieces (the direct form stores 8 bytes per lane, 32 bytes per pixel
  // row piece per instruction)
  __shared__ __attribute__((aligned(16))) bf16 stg[STG ? 4 * 16 * CO : 8];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  for (int i = tid; i < CO * (KP / 8); i += 256) {
    const int co = i / (KP / 8), kc = (i % (KP / 8)) * 8;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (kc < K) v = *reinterpret_cast<const uint4*>(w + (size_t)co * K + kc);
    *reinterpret_cast<uint4*>(ws + co * KP + kc) = v;
  }
  const bool fuse = DGRAD && bn.part != nullptr;
  if constexpr (DGRAD) {
    for (int c = tid; c < CO; c += 256) {
      kks[c] = fuse ? bn.aux[c] : 0.f;
      kis[c] = fuse ? bn.aux[CO + c] : 0.f;
    }
  } else {
    for (int c = tid; c < CO; c += 256) kks[c] = kshift ? kshift[c] : 0.f;
  }
  __syncthreads();

  const int r = lane & 15, kq = lane >> 4;
  float s[CT][4], q[CT][4];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct)
#pragma unroll
    for (int j = 0; j < 4; ++j) s[ct][j] = q[ct][j] = 0.f;
  const bool want = DGRAD ? fuse : stats != nullptr;

  const int ngroups = (M + 15) >> 4;
  const int gstride = gridDim.x * 4;
  auto load_b = [&](int g, bf16x8* b) {
    const int px = g * 16 + r;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int kc = ks * 32 + kq * 8;
      if (px < M && kc < K) {
        b[ks] = *reinterpret_cast<const bf16x8*>(x + (size_t)px * K + kc);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) b[ks][e] = (bf16)0.f;
      }
    }
  };
  int g = blockIdx.x * 4 + wid;
  bf16x8 bcur[KS], bnext[KS];
  if (g < ngroups) load_b(g, bcur);
  for (; g < ngroups; g += gstride) {
    const int gn = g + gstride;
    if (gn < ngroups) load_b(gn, bnext);   // the next group's operand in flight
    const int px = g * 16 + r;
    const bool pok = px < M;
    bf16* yrow = y + (size_t)px * CO + kq * 4;
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(ws + (ct * 16 + r) * KP + ks * 32 + kq * 8);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bcur[ks], acc, 0, 0, 0);
      }
      // D[row = channel ct*16 + 4kq + j][col = pixel r]: four consecutive channels of pixel r
      const size_t eo = (size_t)px * CO + ct * 16 + kq * 4;   // (element offset, pixel r)
      if constexpr (DGRAD) {
        if (bn.addend && pok) {
          const uint2 av = *reinterpret_cast<const uint2*>(bn.addend + eo);
          acc[0] += __uint_as_float(av.x << 16);
          acc[1] += __uint_as_float(av.x & 0xffff0000u);
          acc[2] += __uint_as_float(av.y << 16);
          acc[3] += __uint_as_float(av.y & 0xffff0000u);
        }
      }
      const uint32_t lo = pack2(acc[0], acc[1]), hi = pack2(acc[2], acc[3]);
      if constexpr (STG)
        *reinterpret_cast<uint2*>(stg + wid * 16 * CO + r * CO + ct * 16 + kq * 4) = make_uint2(lo, hi);
      else if (pok)
        *reinterpret_cast<uint2*>(yrow + ct * 16) = make_uint2(lo, hi);
      if (want && pok) {
        const float f[4] = {__uint_as_float(lo << 16), __uint_as_float(lo & 0xffff0000u),
                            __uint_as_float(hi << 16), __uint_as_float(hi & 0xffff0000u)};
        if constexpr (DGRAD) {
          // dz = dX * relu'(mask) of the stored dX; sums of dz and dz * (y - mean)
          const uint2 yv = *reinterpret_cast<const uint2*>(bn.y + eo);
          const float yy[4] = {__uint_as_float(yv.x << 16), __uint_as_float(yv.x & 0xffff0000u),
                               __uint_as_float(yv.y << 16), __uint_as_float(yv.y & 0xffff0000u)};
          const uint32_t mb = (uint32_t)bn.mask[eo >> 3] >> (eo & 7);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float dz = ((mb >> j) & 1u) ? f[j] : 0.f;
            s[ct][j] += dz;
            q[ct][j] = fmaf(dz, yy[j] - kks[ct * 16 + kq * 4 + j], q[ct][j]);
          }
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float d = f[j] - kks[ct * 16 + kq * 4 + j];   // the stored value, shifted
            s[ct][j] += d;
            q[ct][j] = fmaf(d, d, q[ct][j]);
          }
        }
      }
    }
    if constexpr (STG) {
      // (wave-private region: this wave's LDS writes complete before its reads, in order)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      const int npx = min(16, M - g * 16);
      const int nchunk = npx * CO / 8;
      const uint4* src = reinterpret_cast<const uint4*>(stg + wid * 16 * CO);
      uint4* dst = reinterpret_cast<uint4*>(y + (size_t)g * 16 * CO);
      for (int i = lane; i < nchunk; i += 64) dst[i] = src[i];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // (reads done before the next writes)
    }
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) bcur[ks] = bnext[ks];
  }
  if (!want) return;
  // the 16 pixel lanes of each channel quad, then the four waves, then one row per workgroup
#pragma unroll
  for (int ct = 0; ct < CT; ++ct)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float a = s[ct][j], b = q[ct][j];
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        a += __shfl_xor(a, o, 64);
        b += __shfl_xor(b, o, 64);
      }
      if (r == 0) {
        red[wid][0][ct * 16 + kq * 4 + j] = a;
        red[wid][1][ct * 16 + kq * 4 + j] = b;
      }
    }
  __syncthreads();
  float* out = DGRAD ? bn.part : stats;
  for (int c = tid; c < CO; c += 256) {
    const float q2 = red[0][1][c] + red[1][1][c] + red[2][1][c] + red[3][1][c];
    stat_out(out, blockIdx.x, shards, 2 * CO, c,
             red[0][0][c] + red[1][0][c] + red[2][0][c] + red[3][0][c]);
    stat_out(out, blockIdx.x, shards, 2 * CO, CO + c, DGRAD ? q2 * kis[c] : q2);
  }
  if constexpr (!DGRAD) stat_krow(stats, shards, 2 * CO, kshift, CO);
}

static int nk_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    hipDeviceProp_t p;
    if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&p, dev) == hipSuccess)
      n = p.multiProcessorCount;
    if (n <= 0) n = 256;
  }
  return n;
}

static int64_t g_nk_min_m = -1;
static int64_t nk_min_m() {
  if (g_nk_min_m < 0) {
    const char* e = getenv("PCA_NK_MIN_M");
    g_nk_min_m = e ? (int64_t)atoll(e) : (int64_t)16 * 4 * 8 * 4 * 256;
  }
  return g_nk_min_m;
}
// (tests: the threshold below which the implicit GEMM keeps these shapes; returns the old one)
int64_t conv_nk_min_m(int64_t v) {
  const int64_t old = nk_min_m();
  if (v >= 0) g_nk_min_m = v;
  return old;
}

bool conv1x1_nk_applicable(int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride,
                           int pad, int groups) {
  static const bool on = [] {
    const char* e = getenv("PCA_CONV_NK");
    return !(e && e[0] == '0');
  }();
  // large pixel counts only: every wave should walk >= 8 pixel groups, or the per-workgroup
  // weight staging is not amortized (measured, tools/nk_bench.py: the 16x16 MobileNetV2 / the
  // bs128 shapes run as fast or faster on the implicit GEMM)
  const int64_t min_m = nk_min_m();
  const int ct = Cout / 16;
  const int64_t M = (int64_t)N * H * W;
  return on && N > 0 && KH == 1 && KW == 1 && stride == 1 && pad == 0 && groups == 1 &&
         Cin % 8 == 0 && Cin >= 8 && Cin <= 64 && Cout % 16 == 0 &&
         (ct == 6 || ct == 9 || ct == 12 || ct == 15) && M >= min_m && M < (1 << 30);
}

// workgroups (= BN statistics slab rows): four 16-pixel groups per round, at most four rounds of
// workgroups per CU
int conv1x1_nk_stat_rows(int N, int H, int W) {
  const int64_t groups = ((int64_t)N * H * W + 15) / 16;
  return (int)std::max<int64_t>(1, std::min<int64_t>((groups + 3) / 4, std::min(4 * nk_cus(), 1024)));
}

template <bool DGRAD>
static void nk_dispatch(const bf16* x, const bf16* w, bf16* y, float* stats, int M, int K, int CO,
                        int grid, int sh, const float* k, const NkBn& b, bool stg, hipStream_t st) {
  const int ks = K <= 32 ? 1 : 2;
#define PCA_NK(KS_, CT_)                                                                          \
  if (ks == KS_ && CO == CT_ * 16) {                                                             \
    if (stg)                                                                                      \
      hipLaunchKernelGGL((conv1x1_nk_kernel<KS_, CT_, true, DGRAD>), dim3(grid), dim3(256), 0, st, \
                         x, w, y, M, K, stats, sh, k, b);                                         \
    else                                                                                          \
      hipLaunchKernelGGL((conv1x1_nk_kernel<KS_, CT_, false, DGRAD>), dim3(grid), dim3(256), 0,   \
                         st, x, w, y, M, K, stats, sh, k, b);                                     \
    return;                                                                                       \
  }
  PCA_NK(1, 6) PCA_NK(1, 9) PCA_NK(1, 12) PCA_NK(1, 15)
  PCA_NK(2, 6) PCA_NK(2, 9) PCA_NK(2, 12) PCA_NK(2, 15)
#undef PCA_NK
}

// x [M][Cin] bf16, w [Cout][Cin] bf16 -> y [M][Cout] bf16; stats: slab rows
// [conv1x1_nk_stat_rows][2][Cout] (shards 0) or the sharded accumulator (stat_shards() > 0)
void conv1x1_nk_launch(const bf16* x, const bf16* w, bf16* y, float* stats, int N, int H, int W,
                       int Cin, int Cout, hipStream_t st) {
  const int M = N * H * W;
  const int grid = conv1x1_nk_stat_rows(N, H, W);
  const int sh = stat_shards();
  const float* k = stats ? stat_shift() : nullptr;
  static const bool stg = [] {
    const char* e = getenv("PCA_NK_STG");
    return !(e && e[0] == '0');
  }();
  nk_dispatch<false>(x, w, y, stats, M, Cin, Cout, grid, sh, k, NkBn{}, stg, st);
}

// dX [M][Cin] = dY [M][Cout] . W^T of a 1x1 / stride-1 conv with Cout <= 64 (wt = its [Cin][Cout]
// dgrad operand): the narrow-K form with the dgrad epilogue (conv_dgrad_launch)
void conv1x1_nk_dgrad_launch(const bf16* dy, const bf16* wt, bf16* dx, int N, int H, int W,
                             int Cin, int Cout, const bf16* addend, const bf16* bn_y,
                             const uint8_t* bn_mask, const float* bn_aux, float* bn_part,
                             hipStream_t st) {
  const int M = N * H * W;
  const int grid = conv1x1_nk_stat_rows(N, H, W);
  static const bool stg = [] {
    const char* e = getenv("PCA_NK_STG");
    return !(e && e[0] == '0');
  }();
  NkBn b{addend, bn_y, bn_mask, bn_aux, bn_part};
  nk_dispatch<true>(dy, wt, dx, nullptr, M, Cout, Cin, grid, stat_shards(), nullptr, b, stg, st);
}

}  // namespace pca
