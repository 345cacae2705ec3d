// Pooling fast paths (NHWC bf16, C % 8 == 0): rolling-row 3x3 / stride-1 / pad-1 max pool and
// window == stride average pool. The generic kernels (misc.hip) handle every other geometry.
//
// GoogLeNet's Inception pool branch (reference models/googlenet.py:41-45: MaxPool2d(3, stride=1,
// padding=1) in all nine Inceptions) is the zoo's heaviest pool: the generic 8-wide kernels
// re-read all nine window taps per output (forward) and nine (dy, argmax) pairs per input
// (backward) with runtime divisions per tap, 1.75 ms of a 14.4 ms bs256 step. Here one thread
// owns 8 channels of one image column and walks its rows: the forward loads each new input row
// once (3 horizontal taps, neighbours' loads hit L1) and keeps the last three row maxima in
// registers; the backward loads each output row's (dy, argmax) once and scatters it into the
// three input rows it feeds, emitting an input row once its last contributor has been seen.
// Ties and NaNs resolve exactly as the generic kernel (first maximum in (kh, kw) scan order, a
// NaN wins), so the argmax bytes — and the backward — are the same.
//
// Average pool with k == s, p == 0 (DenseNet transitions, densenet.py:31-32; the 2x2 / 4x4
// pools): one thread per 8 channels of one OUTPUT pixel; backward writes its k*k input pixels.
#include "common.h"

#include <algorithm>

namespace pca {

struct Pool3Geom {
  int N, H, W, G;   // G = C / 8
};

// max over the three taps of one input row at columns w-1, w, w+1 (kw order, generic tie rule)
__device__ __forceinline__ void row_max3(const bf16* row, int w, int W, int C, float* m,
                                         uint32_t* a) {
#pragma unroll
  for (int v = 0; v < 8; ++v) {
    m[v] = -INFINITY;
    a[v] = 0;
  }
#pragma unroll
  for (int kw = 0; kw < 3; ++kw) {
    const int iw = w - 1 + kw;
    if ((unsigned)iw >= (unsigned)W) continue;
    float f[8];
    unpack8(*reinterpret_cast<const uint4*>(row + (size_t)iw * C), f);
#pragma unroll
    for (int v = 0; v < 8; ++v)
      if (f[v] > m[v] || f[v] != f[v]) {
        m[v] = f[v];
        a[v] = kw;
      }
  }
}

// A thread walks a strip of kStrip rows (more threads in flight than whole columns: the first
// version, one thread per column, ran GoogLeNet's 32x32 pools latency-bound; a strip re-reads
// one halo row on each side).
constexpr int kStrip = 8;

__global__ __launch_bounds__(256) void maxpool3s1_fwd_kernel(const bf16* __restrict__ x,
                                                             Pool3Geom g, bf16* __restrict__ y,
                                                             uint8_t* __restrict__ arg) {
  const int strips = (g.H + kStrip - 1) / kStrip;
  const int total = g.N * strips * g.W * g.G;
  const int C = g.G * 8;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int gi = i % g.G;
    int q = i / g.G;
    const int w = q % g.W;
    q /= g.W;
    const int sidx = q % strips;
    const int n = q / strips;
    const int r0 = sidx * kStrip, r1 = min(r0 + kStrip, g.H);
    const bf16* xn = x + (size_t)n * g.H * g.W * C + gi * 8;
    const size_t ybase = ((size_t)n * g.H * g.W + w) * C + gi * 8;
    // row maxima of input rows oh-1 (p), oh (c), oh+1 (n) for the current output row oh
    float mp[8], mc[8], mn[8];
    uint32_t ap[8], ac[8], an[8];
    if (r0 > 0) {
      row_max3(xn + (size_t)(r0 - 1) * g.W * C, w, g.W, C, mp, ap);
    } else {
#pragma unroll
      for (int v = 0; v < 8; ++v) {
        mp[v] = -INFINITY;
        ap[v] = 0;
      }
    }
    row_max3(xn + (size_t)r0 * g.W * C, w, g.W, C, mc, ac);
    for (int oh = r0; oh < r1; ++oh) {
      if (oh + 1 < g.H) {
        row_max3(xn + (size_t)(oh + 1) * g.W * C, w, g.W, C, mn, an);
      } else {
#pragma unroll
        for (int v = 0; v < 8; ++v) {
          mn[v] = -INFINITY;
          an[v] = 0;
        }
      }
      float best[8];
      uint32_t bi[8];
      const bool top = oh > 0, bot = oh + 1 < g.H;
#pragma unroll
      for (int v = 0; v < 8; ++v) {
        best[v] = -INFINITY;
        bi[v] = 0;
        if (top && (mp[v] > best[v] || mp[v] != mp[v])) {
          best[v] = mp[v];
          bi[v] = ap[v];
        }
        if (mc[v] > best[v] || mc[v] != mc[v]) {
          best[v] = mc[v];
          bi[v] = 3 + ac[v];
        }
        if (bot && (mn[v] > best[v] || mn[v] != mn[v])) {
          best[v] = mn[v];
          bi[v] = 6 + an[v];
        }
      }
      const size_t o = ybase + (size_t)oh * g.W * C;
      *reinterpret_cast<uint4*>(y + o) = pack8(best);
      *reinterpret_cast<uint2*>(arg + o) =
          make_uint2(bi[0] | (bi[1] << 8) | (bi[2] << 16) | (bi[3] << 24),
                     bi[4] | (bi[5] << 8) | (bi[6] << 16) | (bi[7] << 24));
#pragma unroll
      for (int v = 0; v < 8; ++v) {
        mp[v] = mc[v];
        ap[v] = ac[v];
        mc[v] = mn[v];
        ac[v] = an[v];
      }
    }
  }
}

// Contribution of output row oh (columns w+1, w, w-1 = taps kw 0, 1, 2 as seen from input column
// w) to input row oh - 1 + kh, for kh = 0, 1, 2: part[kh][v] = sum over kw of dy where the
// output's argmax byte is kh*3 + kw (summed in kw order, as the generic kernel does).
__device__ __forceinline__ void out_row_parts(const bf16* dyr, const uint8_t* ar, int w, int W,
                                              int C, float (*part)[8]) {
#pragma unroll
  for (int kh = 0; kh < 3; ++kh)
#pragma unroll
    for (int v = 0; v < 8; ++v) part[kh][v] = 0.f;
#pragma unroll
  for (int kw = 0; kw < 3; ++kw) {
    const int ow = w + 1 - kw;
    if ((unsigned)ow >= (unsigned)W) continue;
    const uint2 a = *reinterpret_cast<const uint2*>(ar + (size_t)ow * C);
    float f[8];
    unpack8(*reinterpret_cast<const uint4*>(dyr + (size_t)ow * C), f);
#pragma unroll
    for (int v = 0; v < 8; ++v) {
      const uint32_t av = ((v < 4 ? a.x : a.y) >> ((v & 3) * 8)) & 0xffu;
#pragma unroll
      for (int kh = 0; kh < 3; ++kh)
        if (av == (uint32_t)(kh * 3 + kw)) part[kh][v] += f[v];
    }
  }
}

__global__ __launch_bounds__(256) void maxpool3s1_bwd_kernel(const bf16* __restrict__ dy,
                                                             const uint8_t* __restrict__ arg,
                                                             Pool3Geom g, bf16* __restrict__ dx) {
  const int strips = (g.H + kStrip - 1) / kStrip;
  const int total = g.N * strips * g.W * g.G;
  const int C = g.G * 8;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int gi = i % g.G;
    int q = i / g.G;
    const int w = q % g.W;
    q /= g.W;
    const int sidx = q % strips;
    const int n = q / strips;
    const int r0 = sidx * kStrip, r1 = min(r0 + kStrip, g.H);
    const size_t nb = (size_t)n * g.H * g.W * C + gi * 8;
    const size_t xo = nb + (size_t)w * C;
    // Output row oh feeds input row oh - 1 + kh with its kh part. Input row ih is summed in the
    // generic kernel's order kh 0 (output row ih + 1), kh 1 (row ih), kh 2 (row ih - 1), so it is
    // complete once row ih + 1 has been read: h1 / h2 hold the kh 1 / kh 2 parts of the row
    // being completed, n2 the kh 2 part of the row after it. The strip's input rows [r0, r1)
    // read output rows r0 - 1 .. r1.
    float h1[8], h2[8], n2[8];
#pragma unroll
    for (int v = 0; v < 8; ++v) h1[v] = h2[v] = n2[v] = 0.f;
    const int o0 = max(r0 - 1, 0), o1 = min(r1, g.H - 1);
    for (int oh = o0; oh <= o1; ++oh) {
      float part[3][8];
      out_row_parts(dy + nb + (size_t)oh * g.W * C, arg + nb + (size_t)oh * g.W * C, w, g.W, C,
                    part);
      if (oh - 1 >= r0) {
        float s[8];
#pragma unroll
        for (int v = 0; v < 8; ++v) s[v] = ((0.f + part[0][v]) + h1[v]) + h2[v];
        *reinterpret_cast<uint4*>(dx + xo + (size_t)(oh - 1) * g.W * C) = pack8(s);
      }
#pragma unroll
      for (int v = 0; v < 8; ++v) {
        h1[v] = part[1][v];
        h2[v] = n2[v];
        n2[v] = part[2][v];
      }
    }
    if (r1 == g.H) {   // the last row has no kh 0 contributor
      float s[8];
#pragma unroll
      for (int v = 0; v < 8; ++v) s[v] = (0.f + h1[v]) + h2[v];
      *reinterpret_cast<uint4*>(dx + xo + (size_t)(g.H - 1) * g.W * C) = pack8(s);
    }
  }
}

void maxpool3s1_fwd_launch(const bf16* x, int N, int H, int W, int C, bf16* y, uint8_t* arg,
                           hipStream_t st) {
  const Pool3Geom g{N, H, W, C / 8};
  const int total = N * ((H + kStrip - 1) / kStrip) * W * (C / 8);
  const int blocks = std::min((total + 255) / 256, 16384);
  hipLaunchKernelGGL(maxpool3s1_fwd_kernel, dim3(blocks), dim3(256), 0, st, x, g, y, arg);
}

void maxpool3s1_bwd_launch(const bf16* dy, const uint8_t* arg, int N, int H, int W, int C, bf16* dx,
                           hipStream_t st) {
  const Pool3Geom g{N, H, W, C / 8};
  const int total = N * ((H + kStrip - 1) / kStrip) * W * (C / 8);
  const int blocks = std::min((total + 255) / 256, 16384);
  hipLaunchKernelGGL(maxpool3s1_bwd_kernel, dim3(blocks), dim3(256), 0, st, dy, arg, g, dx);
}

// ---- average pool, window == stride, no padding (every zoo avg pool) ----
template <int K>
__global__ __launch_bounds__(256) void avgpool_ks_fwd_kernel(const bf16* __restrict__ x, int N,
                                                             int H, int W, int G,
                                                             bf16* __restrict__ y) {
  const int Ho = H / K, Wo = W / K, C = G * 8;
  const int total = N * Ho * Wo * G;
  const float inv = 1.f / (K * K);
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int gi = i % G;
    int q = i / G;
    const int ow = q % Wo;
    q /= Wo;
    const int oh = q % Ho;
    const int n = q / Ho;
    const bf16* xp = x + (((size_t)n * H + oh * K) * W + ow * K) * C + gi * 8;
    float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kh = 0; kh < K; ++kh)
#pragma unroll
      for (int kw = 0; kw < K; ++kw) {
        float f[8];
        unpack8(*reinterpret_cast<const uint4*>(xp + ((size_t)kh * W + kw) * C), f);
#pragma unroll
        for (int v = 0; v < 8; ++v) s[v] += f[v];
      }
#pragma unroll
    for (int v = 0; v < 8; ++v) s[v] *= inv;
    *reinterpret_cast<uint4*>(y + (size_t)i * 8) = pack8(s);
  }
}

template <int K>
__global__ __launch_bounds__(256) void avgpool_ks_bwd_kernel(const bf16* __restrict__ dy, int N,
                                                             int H, int W, int G,
                                                             bf16* __restrict__ dx) {
  const int Ho = H / K, Wo = W / K, C = G * 8;
  const int total = N * Ho * Wo * G;
  const float inv = 1.f / (K * K);
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int gi = i % G;
    int q = i / G;
    const int ow = q % Wo;
    q /= Wo;
    const int oh = q % Ho;
    const int n = q / Ho;
    float f[8];
    unpack8(*reinterpret_cast<const uint4*>(dy + (size_t)i * 8), f);
#pragma unroll
    for (int v = 0; v < 8; ++v) f[v] = (0.f + f[v]) * inv;   // (the generic kernel's sum, then scale)
    const uint4 o = pack8(f);
    bf16* xp = dx + (((size_t)n * H + oh * K) * W + ow * K) * C + gi * 8;
#pragma unroll
    for (int kh = 0; kh < K; ++kh)
#pragma unroll
      for (int kw = 0; kw < K; ++kw) *reinterpret_cast<uint4*>(xp + ((size_t)kh * W + kw) * C) = o;
  }
}

// returns false when the geometry is not a fast-path one (caller runs the generic kernel)
bool avgpool_ks_launch(bool bwd, const bf16* in, int N, int H, int W, int C, int k, int s, int p,
                       bf16* out, hipStream_t st) {
  if (C % 8 || k != s || p != 0 || H % k || W % k) return false;
  if ((size_t)N * H * W * C >= (size_t)INT32_MAX) return false;
  const int total = N * (H / k) * (W / k) * (C / 8);
  const int blocks = std::max(1, std::min((total + 255) / 256, 16384));
#define PCA_AVG(KK)                                                                              \
  case KK:                                                                                       \
    if (bwd)                                                                                     \
      hipLaunchKernelGGL(avgpool_ks_bwd_kernel<KK>, dim3(blocks), dim3(256), 0, st, in, N, H, W, \
                         C / 8, out);                                                            \
    else                                                                                         \
      hipLaunchKernelGGL(avgpool_ks_fwd_kernel<KK>, dim3(blocks), dim3(256), 0, st, in, N, H, W, \
                         C / 8, out);                                                            \
    return true;
  switch (k) {
    PCA_AVG(2)
    PCA_AVG(4)
    PCA_AVG(8)
    default:
      return false;
  }
#undef PCA_AVG
}

}  // namespace pca
