// Skinny 1x1 convolutions: the pointwise convs of the inverted-residual blocks, where one side of
// the GEMM is narrow (reference models/mobilenetv2.py:25-35, models/efficientnet.py:63-80;
// SURVEY §2.8 K4):
//   narrow K  — the expand conv, K = 16..64 input channels -> Cout = 6K (96..240);
//   narrow N  — the project conv, K = 33..256 -> Cout = 8..64.
//
// With one or a few 64-deep K steps per tile the generic implicit GEMM is a serial chain per tile
// (operand DMA -> MFMA -> LDS epilogue -> stores) and lands at 2-3x the bytes floor on these
// shapes (MobileNetV2 bs1024 24->144: 166-176 us for 352 MB). Here the whole (zero-padded) weight
// matrix sits in LDS once per workgroup, each wave walks 16-pixel groups with the next group's
// input fragments in flight, and the MFMA is issued as W x X^T: lane (r, kq) holds pixel r's
// K-chunks kq as the B operand and gets back four consecutive output channels of pixel r. The
// wave's 16-pixel output tile goes through a wave-private LDS region and leaves as contiguous
// 16-byte row pieces (no workgroup barrier in the pixel loop; the direct 8-byte-per-lane stores
// measured slower, tools/nk_bench.py). BatchNorm statistics (shifted sums, common.h stat_shift)
// of the stored bf16 values accumulate in registers and leave once per workgroup (stat_out).
//
// The same GEMM shapes are the data gradients of the transposed convs (dX[M][Co] = dY[M][K] . W^T
// with the conv's [Co][K] dgrad operand): DGRAD replaces the statistics epilogue by the dgrad
// one — the residual addend, and the fused backward reduce of the BatchNorm(+ReLU) that produced
// the conv input (sums of dz = dX * relu'(mask) and dz * (y - mean), istd applied at the flush:
// the igemm dgrad epilogue's slab-row / sharded form).
#include "mfma_util.h"

#include <algorithm>
#include <cstdlib>

namespace pca {

int stat_shards();
const float* stat_shift();

struct NkBn {
  const bf16* addend;
  const bf16* y;            // that BN's input (its mean | istd in aux)
  const uint8_t* mask;      // its 1-bit ReLU mask (all ones for a BN without activation)
  const float* aux;
  float* part;              // [rows][2][Co] slab rows, or the sharded accumulator
};

// KS: MFMA K steps of 32 (K <= 32 KS, zero padded); CT: 16-channel output tiles (Co <= 16 CT,
// Co % 8 == 0: a lane's four channels are all real or all padding)
template <int KS, int CT, bool DGRAD>
__global__ __launch_bounds__(256) void conv1x1_nk_kernel(const bf16* __restrict__ x,
                                                         const bf16* __restrict__ w,
                                                         bf16* __restrict__ y, int M, int K, int Co,
                                                         float* __restrict__ stats, int shards,
                                                         const float* __restrict__ kshift,
                                                         NkBn bn) {
  constexpr int CP = CT * 16;   // padded output channels
  constexpr int KP = KS * 32;   // padded reduction width
  __shared__ __attribute__((aligned(16))) bf16 ws[CP * KP];
  __shared__ float kks[CP];     // forward: the statistics shift; dgrad: the BN mean
  __shared__ float kis[DGRAD ? CP : 1];   // dgrad: the BN istd
  __shared__ float red[4][2][CP];
  __shared__ __attribute__((aligned(16))) bf16 stg[4 * 16 * CP];   // wave-private output tiles
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  for (int i = tid; i < CP * (KP / 8); i += 256) {
    const int co = i / (KP / 8), kc = (i % (KP / 8)) * 8;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (co < Co && kc < K) v = *reinterpret_cast<const uint4*>(w + (size_t)co * K + kc);
    *reinterpret_cast<uint4*>(ws + co * KP + kc) = v;
  }
  const bool fuse = DGRAD && bn.part != nullptr;
  for (int c = tid; c < CP; c += 256) {
    if constexpr (DGRAD) {
      kks[c] = fuse && c < Co ? bn.aux[c] : 0.f;
      kis[c] = fuse && c < Co ? bn.aux[Co + c] : 0.f;
    } else {
      kks[c] = kshift && c < Co ? kshift[c] : 0.f;
    }
  }
  __syncthreads();

  const int r = lane & 15, kq = lane >> 4;
  float s[CT][4], q[CT][4];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct)
#pragma unroll
    for (int j = 0; j < 4; ++j) s[ct][j] = q[ct][j] = 0.f;
  const bool want = DGRAD ? fuse : stats != nullptr;
  bf16* stile = stg + wid * 16 * CP;   // this wave's tile, row pitch Co (= the global rows)

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
    if (gn < ngroups) load_b(gn, bnext);   // the next group's operands in flight
    const int px = g * 16 + r;
    const bool pok = px < M;
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      if (ct * 16 >= Co) continue;         // (wave-uniform: a tile of padding channels)
      const int cb = ct * 16 + kq * 4;     // this lane's four channels
      const bool cok = cb < Co;            // (the last tile may be half padding)
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(ws + (ct * 16 + r) * KP + ks * 32 + kq * 8);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bcur[ks], acc, 0, 0, 0);
      }
      // D[row = channel cb + j][col = pixel r]
      const size_t eo = (size_t)px * Co + cb;   // element offset of (pixel r, channel cb)
      if constexpr (DGRAD) {
        if (bn.addend && pok && cok) {
          const uint2 av = *reinterpret_cast<const uint2*>(bn.addend + eo);
          acc[0] += __uint_as_float(av.x << 16);
          acc[1] += __uint_as_float(av.x & 0xffff0000u);
          acc[2] += __uint_as_float(av.y << 16);
          acc[3] += __uint_as_float(av.y & 0xffff0000u);
        }
      }
      const uint32_t lo = pack2(acc[0], acc[1]), hi = pack2(acc[2], acc[3]);
      if (cok) *reinterpret_cast<uint2*>(stile + r * Co + cb) = make_uint2(lo, hi);
      if (want && pok && cok) {
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
            q[ct][j] = fmaf(dz, yy[j] - kks[cb + j], q[ct][j]);
          }
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float d = f[j] - kks[cb + j];   // the stored value, shifted
            s[ct][j] += d;
            q[ct][j] = fmaf(d, d, q[ct][j]);
          }
        }
      }
    }
    // the wave's tile (rows of Co channels) is contiguous in y: whole 16-byte pieces
    // (wave-private region: this wave's LDS writes complete before its reads, in order)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const int npx = min(16, M - g * 16);
    const int nchunk = npx * Co / 8;
    const uint4* src = reinterpret_cast<const uint4*>(stile);
    uint4* dst = reinterpret_cast<uint4*>(y + (size_t)g * 16 * Co);
    for (int i = lane; i < nchunk; i += 64) dst[i] = src[i];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // (reads done before the next writes)
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
  for (int c = tid; c < Co; c += 256) {
    const float q2 = red[0][1][c] + red[1][1][c] + red[2][1][c] + red[3][1][c];
    stat_out(out, blockIdx.x, shards, 2 * Co, c,
             red[0][0][c] + red[1][0][c] + red[2][0][c] + red[3][0][c]);
    stat_out(out, blockIdx.x, shards, 2 * Co, Co + c, DGRAD ? q2 * kis[c] : q2);
  }
  if constexpr (!DGRAD) stat_krow(stats, shards, 2 * Co, kshift, Co);
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

// (KS, CT) of a K -> Co GEMM the kernel is instantiated for, or false
static bool nk_shape(int K, int Co, int* ks, int* ct) {
  static const bool narrow_n = [] {
    const char* e = getenv("PCA_NK_NARROW_N");
    return !(e && e[0] == '0');
  }();
  if (K % 8 || Co % 8 || K < 8) return false;
  *ks = (K + 31) / 32;
  *ct = (Co + 15) / 16;
  if (K <= 64 && Co % 16 == 0 && (*ct == 6 || *ct == 9 || *ct == 12 || *ct == 15)) return true;   // narrow K
  return narrow_n && K <= 256 && Co <= 64 && *ks >= 2;   // narrow N
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
  const int64_t M = (int64_t)N * H * W;
  int ks, ct;
  return on && N > 0 && KH == 1 && KW == 1 && stride == 1 && pad == 0 && groups == 1 &&
         nk_shape(Cin, Cout, &ks, &ct) && M >= min_m && M < (1 << 30);
}

// workgroups (= BN statistics slab rows): four 16-pixel groups per round, at most four rounds of
// workgroups per CU
int conv1x1_nk_stat_rows(int N, int H, int W) {
  const int64_t groups = ((int64_t)N * H * W + 15) / 16;
  return (int)std::max<int64_t>(1, std::min<int64_t>((groups + 3) / 4, std::min(4 * nk_cus(), 1024)));
}

template <bool DGRAD>
static void nk_dispatch(const bf16* x, const bf16* w, bf16* y, float* stats, int M, int K, int Co,
                        int grid, int sh, const float* k, const NkBn& b, hipStream_t st) {
  int ks = 0, ct = 0;
  if (!nk_shape(K, Co, &ks, &ct)) return;
#define PCA_NK(KS_, CT_)                                                                         \
  if (ks == KS_ && ct == CT_) {                                                                 \
    hipLaunchKernelGGL((conv1x1_nk_kernel<KS_, CT_, DGRAD>), dim3(grid), dim3(256), 0, st, x, w, \
                       y, M, K, Co, stats, sh, k, b);                                            \
    return;                                                                                      \
  }
  PCA_NK(1, 6) PCA_NK(1, 9) PCA_NK(1, 12) PCA_NK(1, 15)
  PCA_NK(2, 6) PCA_NK(2, 9) PCA_NK(2, 12) PCA_NK(2, 15)
  PCA_NK(2, 1) PCA_NK(2, 2) PCA_NK(2, 3) PCA_NK(2, 4)
  PCA_NK(3, 1) PCA_NK(3, 2) PCA_NK(3, 3) PCA_NK(3, 4)
  PCA_NK(4, 1) PCA_NK(4, 2) PCA_NK(4, 3) PCA_NK(4, 4)
  PCA_NK(5, 1) PCA_NK(5, 2) PCA_NK(5, 3) PCA_NK(5, 4)
  PCA_NK(6, 1) PCA_NK(6, 2) PCA_NK(6, 3) PCA_NK(6, 4)
  PCA_NK(7, 1) PCA_NK(7, 2) PCA_NK(7, 3) PCA_NK(7, 4)
  PCA_NK(8, 1) PCA_NK(8, 2) PCA_NK(8, 3) PCA_NK(8, 4)
#undef PCA_NK
}

// x [M][Cin] bf16, w [Cout][Cin] bf16 -> y [M][Cout] bf16; stats: slab rows
// [conv1x1_nk_stat_rows][2][Cout] (shards 0) or the sharded accumulator (stat_shards() > 0)
void conv1x1_nk_launch(const bf16* x, const bf16* w, bf16* y, float* stats, int N, int H, int W,
                       int Cin, int Cout, hipStream_t st) {
  const int M = N * H * W;
  nk_dispatch<false>(x, w, y, stats, M, Cin, Cout, conv1x1_nk_stat_rows(N, H, W), stat_shards(),
                     stats ? stat_shift() : nullptr, NkBn{}, st);
}

// dX [M][Cin] = dY [M][Cout] . W^T of a 1x1 / stride-1 conv whose transposed GEMM is skinny (wt =
// its [Cin][Cout] dgrad operand): the dgrad epilogue form (conv_dgrad_launch)
void conv1x1_nk_dgrad_launch(const bf16* dy, const bf16* wt, bf16* dx, int N, int H, int W,
                             int Cin, int Cout, const bf16* addend, const bf16* bn_y,
                             const uint8_t* bn_mask, const float* bn_aux, float* bn_part,
                             hipStream_t st) {
  const int M = N * H * W;
  NkBn b{addend, bn_y, bn_mask, bn_aux, bn_part};
  nk_dispatch<true>(dy, wt, dx, nullptr, M, Cout, Cin, conv1x1_nk_stat_rows(N, H, W),
                    stat_shards(), nullptr, b, st);
}

}  // namespace pca
