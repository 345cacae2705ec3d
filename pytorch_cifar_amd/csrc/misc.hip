// Memory-bound kernels around the conv/BN core, NHWC bf16 activations, fp32 parameters.
//
//   layout      : NCHW fp32 model input -> NHWC bf16 (channel-padded) and back      (K26)
//   augment     : GPU-resident uint8 CIFAR images -> random crop(pad 4) + flip +
//                 normalize -> NHWC bf16 (main.py:30-35 / main_dist.py:93-97)       (K25)
//   pooling     : global average (head + SE squeeze), kxk avg, kxk max (+ saved argmax)
//                 (resnet.py:127, googlenet.py:42/68/79, lenet.py:16)               (K15/K16)
//   cross-entropy: log-softmax + NLL + dlogits + argmax/correct in one kernel
//                 (main.py:103,108-110)                                              (K18/K19)
//   sgd         : one multi-tensor launch, momentum 0.9 / wd 5e-4 semantics of
//                 torch.optim.SGD (main.py:87-88)                                    (K20)
//   se / swish  : squeeze-excite channel scaling and standalone activations          (K13/K14)
//   eltwise     : residual add(+act) for the non-fused paths, act backward
#include "common.h"

#include <algorithm>
#include <cstdlib>

#include <type_traits>

namespace pca {

static int grid_cap(size_t work, int per_block = 256, int cap = 8192) {
  size_t b = (work + per_block - 1) / per_block;
  if (b < 1) b = 1;
  return (int)(b < (size_t)cap ? b : cap);
}

// ------------------------------------------------------------------------------ layout
__global__ void nchw_to_nhwc_kernel(const float* __restrict__ x, int N, int C, int HW, int Cp,
                                    bf16* __restrict__ y) {
  const size_t total = (size_t)N * HW * Cp;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % Cp);
    const size_t p = i / Cp;
    const int hw = (int)(p % HW);
    const int n = (int)(p / HW);
    y[i] = c < C ? f2bf(x[((size_t)n * C + c) * HW + hw]) : f2bf(0.f);
  }
}

__global__ void nhwc_to_nchw_kernel(const bf16* __restrict__ y, int N, int C, int HW, int Cp,
                                    float* __restrict__ x) {
  const size_t total = (size_t)N * C * HW;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    const int hw = (int)(i % HW);
    const size_t q = i / HW;
    const int c = (int)(q % C);
    const int n = (int)(q / C);
    x[i] = bf2f(y[((size_t)n * HW + hw) * Cp + c]);
  }
}

// ----------------------------------------------------------------------------- augment
// One thread per output pixel: gathers 3 uint8 channels, writes 8 bf16 (16 B, C padded to 8).
// Packed form (rnd == nullptr): idx[b] = sample | word << 32, drawn once per epoch by the loader,
// so a training step needs no RNG launches; the thread of pixel 0 also gathers targets[b].
__global__ void augment_kernel(const uint8_t* __restrict__ data, const int64_t* __restrict__ idx,
                               const int32_t* __restrict__ rnd, int B, int H, int W, int pad,
                               float m0, float m1, float m2, float is0, float is1, float is2,
                               bf16* __restrict__ out, const int64_t* __restrict__ labels,
                               int64_t* __restrict__ targets) {
  const int total = B * H * W;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int b = i / (H * W);
    const int hw = i % (H * W);
    const int h = hw / W, w = hw % W;
    // augmentation word k drawn uniformly in [0, span^2 * 2): dy = k % span,
    // dx = (k / span) % span, flip = k / span^2 (span = 2 * pad + 1) -> exactly uniform offsets
    const int64_t e = idx[b];
    const int r = rnd ? rnd[b] : (int)(e >> 32);
    const int64_t sample = rnd ? e : (e & 0xffffffffll);
    if (targets && hw == 0) targets[b] = labels[sample];
    const int span = 2 * pad + 1;
    const int dy = r % span;
    const int dx = (r / span) % span;
    const bool flip = (r / (span * span)) & 1;
    const int sh = h + dy - pad;
    const int sw0 = flip ? (W - 1 - w) : w;
    const int sw = sw0 + dx - pad;
    float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    // torchvision RandomCrop(padding) zero-pads the uint8 image, so a padded pixel is 0 before
    // ToTensor/Normalize: (0 - mean) / std.
    float px[3] = {0.f, 0.f, 0.f};
    if (sh >= 0 && sh < H && sw >= 0 && sw < W) {
      const uint8_t* src = data + (((size_t)sample * H + sh) * W + sw) * 3;
      px[0] = src[0] * (1.f / 255.f);
      px[1] = src[1] * (1.f / 255.f);
      px[2] = src[2] * (1.f / 255.f);
    }
    v[0] = (px[0] - m0) * is0;
    v[1] = (px[1] - m1) * is1;
    v[2] = (px[2] - m2) * is2;
    *reinterpret_cast<uint4*>(out + (size_t)i * 8) = pack8(v);
  }
}

// ------------------------------------------------------------------------------ pooling
// Global average over HW: x[N][HW][C] bf16 -> y[N][C] fp32. One block per (n, 256-channel tile).
__global__ void gap_fwd_kernel(const bf16* __restrict__ x, int HW, int C, float* __restrict__ y) {
  const int n = blockIdx.y;
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const bf16* p = x + (size_t)n * HW * C + c;
  float s = 0.f;
  for (int i = 0; i < HW; ++i) s += bf2f(p[(size_t)i * C]);
  y[(size_t)n * C + c] = s / HW;
}

__global__ void gap_bwd_kernel(const float* __restrict__ dy, int N, int HW, int C,
                               bf16* __restrict__ dx) {
  const size_t total = (size_t)N * HW * C;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const int n = (int)(i / ((size_t)HW * C));
    dx[i] = f2bf(dy[(size_t)n * C + c] / HW);
  }
}

// k x k pooling (avg: count_include_pad semantics of F.avg_pool2d; max: -inf padding)
struct PoolGeom {
  int N, H, W, C, Ho, Wo, k, s, p;
};

__global__ void avgpool_fwd_kernel(const bf16* __restrict__ x, PoolGeom g, bf16* __restrict__ y) {
  const size_t total = (size_t)g.N * g.Ho * g.Wo * g.C;
  const float inv = 1.f / (g.k * g.k);
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % g.C);
    size_t q = i / g.C;
    const int ow = (int)(q % g.Wo);
    q /= g.Wo;
    const int oh = (int)(q % g.Ho);
    const int n = (int)(q / g.Ho);
    float s = 0.f;
    for (int kh = 0; kh < g.k; ++kh) {
      const int ih = oh * g.s - g.p + kh;
      if (ih < 0 || ih >= g.H) continue;
      for (int kw = 0; kw < g.k; ++kw) {
        const int iw = ow * g.s - g.p + kw;
        if (iw < 0 || iw >= g.W) continue;
        s += bf2f(x[(((size_t)n * g.H + ih) * g.W + iw) * g.C + c]);
      }
    }
    y[i] = f2bf(s * inv);
  }
}

__global__ void avgpool_bwd_kernel(const bf16* __restrict__ dy, PoolGeom g, bf16* __restrict__ dx) {
  const size_t total = (size_t)g.N * g.H * g.W * g.C;
  const float inv = 1.f / (g.k * g.k);
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % g.C);
    size_t q = i / g.C;
    const int iw = (int)(q % g.W);
    q /= g.W;
    const int ih = (int)(q % g.H);
    const int n = (int)(q / g.H);
    float s = 0.f;
    for (int kh = 0; kh < g.k; ++kh) {
      const int t = ih + g.p - kh;
      if (t < 0 || t % g.s) continue;
      const int oh = t / g.s;
      if (oh >= g.Ho) continue;
      for (int kw = 0; kw < g.k; ++kw) {
        const int u = iw + g.p - kw;
        if (u < 0 || u % g.s) continue;
        const int ow = u / g.s;
        if (ow >= g.Wo) continue;
        s += bf2f(dy[(((size_t)n * g.Ho + oh) * g.Wo + ow) * g.C + c]);
      }
    }
    dx[i] = f2bf(s * inv);
  }
}

__global__ void maxpool_fwd_kernel(const bf16* __restrict__ x, PoolGeom g, bf16* __restrict__ y,
                                   uint8_t* __restrict__ arg) {
  const size_t total = (size_t)g.N * g.Ho * g.Wo * g.C;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % g.C);
    size_t q = i / g.C;
    const int ow = (int)(q % g.Wo);
    q /= g.Wo;
    const int oh = (int)(q % g.Ho);
    const int n = (int)(q / g.Ho);
    float best = -INFINITY;
    int bi = 0;
    for (int kh = 0; kh < g.k; ++kh) {
      const int ih = oh * g.s - g.p + kh;
      if (ih < 0 || ih >= g.H) continue;
      for (int kw = 0; kw < g.k; ++kw) {
        const int iw = ow * g.s - g.p + kw;
        if (iw < 0 || iw >= g.W) continue;
        const float v = bf2f(x[(((size_t)n * g.H + ih) * g.W + iw) * g.C + c]);
        if (v > best || (v != v)) {
          best = v;
          bi = kh * g.k + kw;
        }
      }
    }
    y[i] = f2bf(best);
    arg[i] = (uint8_t)bi;
  }
}

__global__ void maxpool_bwd_kernel(const bf16* __restrict__ dy, const uint8_t* __restrict__ arg,
                                   PoolGeom g, bf16* __restrict__ dx) {
  const size_t total = (size_t)g.N * g.H * g.W * g.C;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % g.C);
    size_t q = i / g.C;
    const int iw = (int)(q % g.W);
    q /= g.W;
    const int ih = (int)(q % g.H);
    const int n = (int)(q / g.H);
    float s = 0.f;
    for (int kh = 0; kh < g.k; ++kh) {
      const int t = ih + g.p - kh;
      if (t < 0 || t % g.s) continue;
      const int oh = t / g.s;
      if (oh >= g.Ho) continue;
      for (int kw = 0; kw < g.k; ++kw) {
        const int u = iw + g.p - kw;
        if (u < 0 || u % g.s) continue;
        const int ow = u / g.s;
        if (ow >= g.Wo) continue;
        const size_t o = (((size_t)n * g.Ho + oh) * g.Wo + ow) * g.C + c;
        if (arg[o] == kh * g.k + kw) s += bf2f(dy[o]);
      }
    }
    dx[i] = f2bf(s);
  }
}

// 8-channel vectorized max pool (C % 8 == 0): one thread per 8 channels of one output (fwd) or
// input (bwd) pixel, 16-byte data and 8-byte argmax accesses, 32-bit indexing. The scalar
// kernels above (one 2-byte element per thread, 64-bit div/mod) ran GoogLeNet's 3x3/s1
// inception pools at ~15 % of HBM bandwidth (9 of its 23 ms/step at bs256).
__global__ __launch_bounds__(256) void maxpool_fwd8_kernel(const bf16* __restrict__ x, PoolGeom g,
                                                           bf16* __restrict__ y,
                                                           uint8_t* __restrict__ arg) {
  const int G = g.C >> 3;
  const int total = g.N * g.Ho * g.Wo * G;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int gi = i % G;
    int q = i / G;
    const int ow = q % g.Wo;
    q /= g.Wo;
    const int oh = q % g.Ho;
    const int n = q / g.Ho;
    float best[8];
    uint32_t bi[8];
#pragma unroll
    for (int v = 0; v < 8; ++v) {
      best[v] = -INFINITY;
      bi[v] = 0;
    }
    const bf16* xn = x + (size_t)n * g.H * g.W * g.C + gi * 8;
    for (int kh = 0; kh < g.k; ++kh) {
      const int ih = oh * g.s - g.p + kh;
      if ((unsigned)ih >= (unsigned)g.H) continue;
      for (int kw = 0; kw < g.k; ++kw) {
        const int iw = ow * g.s - g.p + kw;
        if ((unsigned)iw >= (unsigned)g.W) continue;
        float f[8];
        unpack8(*reinterpret_cast<const uint4*>(xn + (ih * g.W + iw) * g.C), f);
        const uint32_t t = kh * g.k + kw;
#pragma unroll
        for (int v = 0; v < 8; ++v)
          if (f[v] > best[v] || f[v] != f[v]) {
            best[v] = f[v];
            bi[v] = t;
          }
      }
    }
    *reinterpret_cast<uint4*>(y + (size_t)i * 8) = pack8(best);
    *reinterpret_cast<uint2*>(arg + (size_t)i * 8) =
        make_uint2(bi[0] | (bi[1] << 8) | (bi[2] << 16) | (bi[3] << 24),
                   bi[4] | (bi[5] << 8) | (bi[6] << 16) | (bi[7] << 24));
  }
}

__global__ __launch_bounds__(256) void maxpool_bwd8_kernel(const bf16* __restrict__ dy,
                                                           const uint8_t* __restrict__ arg,
                                                           PoolGeom g, bf16* __restrict__ dx) {
  const int G = g.C >> 3;
  const int total = g.N * g.H * g.W * G;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int gi = i % G;
    int q = i / G;
    const int iw = q % g.W;
    q /= g.W;
    const int ih = q % g.H;
    const int n = q / g.H;
    float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const size_t nb = (size_t)n * g.Ho * g.Wo;
    for (int kh = 0; kh < g.k; ++kh) {
      const int t = ih + g.p - kh;
      if (t < 0) continue;
      const int oh = t / g.s;
      if (oh * g.s != t || oh >= g.Ho) continue;
      for (int kw = 0; kw < g.k; ++kw) {
        const int u = iw + g.p - kw;
        if (u < 0) continue;
        const int ow = u / g.s;
        if (ow * g.s != u || ow >= g.Wo) continue;
        const size_t o = ((nb + oh * g.Wo + ow) * g.C) + gi * 8;
        const uint2 a = *reinterpret_cast<const uint2*>(arg + o);
        const uint32_t tap = kh * g.k + kw;
        float f[8];
        unpack8(*reinterpret_cast<const uint4*>(dy + o), f);
#pragma unroll
        for (int v = 0; v < 8; ++v) {
          const uint32_t av = ((v < 4 ? a.x : a.y) >> ((v & 3) * 8)) & 0xffu;
          if (av == tap) s[v] += f[v];
        }
      }
    }
    *reinterpret_cast<uint4*>(dx + (size_t)i * 8) = pack8(s);
  }
}

// ---- DPN dual-path merge (dpn.py:29-31): y = relu(cat[x[:d] + o[:d], x[d:], o[d:]]) in one
// pass over 8-channel groups (d, Cx, Co % 8 == 0), replacing two channel-slice copies, the
// add, two ReLUs and the concatenation; backward routes relu'(y) * dy to dX / dO the same way.
__global__ __launch_bounds__(256) void dpn_merge_fwd_kernel(const bf16* __restrict__ x,
                                                            const bf16* __restrict__ o, int P,
                                                            int Cx, int Co, int d,
                                                            bf16* __restrict__ y) {
  const int Ct = Cx + Co - d, G = Ct >> 3;
  const int total = P * G;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int gi = i % G, p = i / G;
    const int j = gi * 8;
    float a[8];
    if (j < d) {
      float b[8];
      unpack8(*reinterpret_cast<const uint4*>(x + (size_t)p * Cx + j), a);
      unpack8(*reinterpret_cast<const uint4*>(o + (size_t)p * Co + j), b);
#pragma unroll
      for (int v = 0; v < 8; ++v) a[v] += b[v];
    } else if (j < Cx) {
      unpack8(*reinterpret_cast<const uint4*>(x + (size_t)p * Cx + j), a);
    } else {
      unpack8(*reinterpret_cast<const uint4*>(o + (size_t)p * Co + j - Cx + d), a);
    }
#pragma unroll
    for (int v = 0; v < 8; ++v) a[v] = fmaxf(a[v], 0.f);
    *reinterpret_cast<uint4*>(y + (size_t)i * 8) = pack8(a);
  }
}

__global__ __launch_bounds__(256) void dpn_merge_bwd_kernel(const bf16* __restrict__ dy,
                                                            const bf16* __restrict__ y, int P,
                                                            int Cx, int Co, int d,
                                                            bf16* __restrict__ dx,
                                                            bf16* __restrict__ dout) {
  const int Ct = Cx + Co - d, G = Ct >> 3;
  const int total = P * G;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int gi = i % G, p = i / G;
    const int j = gi * 8;
    float g[8], yy[8];
    unpack8(*reinterpret_cast<const uint4*>(dy + (size_t)i * 8), g);
    unpack8(*reinterpret_cast<const uint4*>(y + (size_t)i * 8), yy);
#pragma unroll
    for (int v = 0; v < 8; ++v) g[v] = yy[v] > 0.f ? g[v] : 0.f;
    const uint4 gv = pack8(g);
    if (j < Cx) *reinterpret_cast<uint4*>(dx + (size_t)p * Cx + j) = gv;
    if (j < d) *reinterpret_cast<uint4*>(dout + (size_t)p * Co + j) = gv;
    else if (j >= Cx) *reinterpret_cast<uint4*>(dout + (size_t)p * Co + j - Cx + d) = gv;
  }
}

void dpn_merge_fwd_launch(const bf16* x, const bf16* o, int P, int Cx, int Co, int d, bf16* y,
                          hipStream_t st) {
  hipLaunchKernelGGL(dpn_merge_fwd_kernel, dim3(grid_cap((size_t)P * (Cx + Co - d) / 8)), dim3(256),
                     0, st, x, o, P, Cx, Co, d, y);
}

void dpn_merge_bwd_launch(const bf16* dy, const bf16* y, int P, int Cx, int Co, int d, bf16* dx,
                          bf16* dout, hipStream_t st) {
  hipLaunchKernelGGL(dpn_merge_bwd_kernel, dim3(grid_cap((size_t)P * (Cx + Co - d) / 8)), dim3(256),
                     0, st, dy, y, P, Cx, Co, d, dx, dout);
}

// ---- channel concatenation of NHWC tensors (DenseNet / DLA / GoogLeNet / DPN joins) and its
// inverse split (the backward): out[p][off_i + c] <-> in_i[p][c], one launch for all pieces,
// V-channel vectors (the widest that divides every width); SPLIT scatters out -> pieces.
struct CatArgs {
  const bf16* src[8];
  bf16* dst[8];
  int off[9];   // prefix channel offsets, off[k] = total
  int k;
};

template <int V, bool SPLIT>
__global__ __launch_bounds__(256) void cat_nhwc_kernel(CatArgs a, bf16* __restrict__ whole, int P) {
  const int Ct = a.off[a.k], G = Ct / V;
  const int total = P * G;
  using T = typename std::conditional<V == 8, uint4, typename std::conditional<V == 4, uint2,
            typename std::conditional<V == 2, uint32_t, uint16_t>::type>::type>::type;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int gi = i % G, p = i / G;
    const int c = gi * V;
    int j = 0;
#pragma unroll 1
    while (j + 1 < a.k && c >= a.off[j + 1]) ++j;
    const int w = a.off[j + 1] - a.off[j];
    const size_t piece = (size_t)p * w + (c - a.off[j]);
    T* wh = reinterpret_cast<T*>(whole + (size_t)p * Ct + c);
    if constexpr (SPLIT) *reinterpret_cast<T*>(a.dst[j] + piece) = *wh;
    else *wh = *reinterpret_cast<const T*>(a.src[j] + piece);
  }
}

void cat_nhwc_launch(const CatArgs& a, bf16* whole, int P, bool split, hipStream_t st) {
  int g = 0;
  for (int j = 0; j < a.k; ++j) g |= (a.off[j + 1] - a.off[j]);
  const int V = (g & 7) == 0 ? 8 : (g & 3) == 0 ? 4 : (g & 1) == 0 ? 2 : 1;
  const dim3 grid(grid_cap((size_t)P * a.off[a.k] / V)), block(256);
#define PCA_CAT(VV)                                                                           \
  if (V == VV) {                                                                              \
    if (split) hipLaunchKernelGGL((cat_nhwc_kernel<VV, true>), grid, block, 0, st, a, whole, P); \
    else hipLaunchKernelGGL((cat_nhwc_kernel<VV, false>), grid, block, 0, st, a, whole, P);      \
    return;                                                                                   \
  }
  PCA_CAT(8) PCA_CAT(4) PCA_CAT(2) PCA_CAT(1)
#undef PCA_CAT
}

// ---- row copy between NHWC matrices with their own row strides (zero-copy concatenation: a
// producer's output into its channel slice of a slab, a slab slice's gradient out to a dense
// tensor): dst[p * ldd + c] = src[p * lds + c], c < C (C % 8 == 0), 16-byte vectors
// out[n][2i+a][2j+b][c] = (a == b == 0) ? in[n][i][j][c] : 0 — a compact stride-2 dgrad
// addend expanded for a kernel that cannot add it per parity class (16-byte vectors, C % 8 == 0)
__global__ __launch_bounds__(256) void s2c_expand_kernel(const bf16* __restrict__ in,
                                                         bf16* __restrict__ out, int Hc, int Wc,
                                                         int C8, int64_t total) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int c = (int)(i % C8);
    int64_t q = i / C8;
    const int x = (int)(q % (2 * Wc));
    q /= 2 * Wc;
    const int y = (int)(q % (2 * Hc));
    const int64_t n = q / (2 * Hc);
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (!(x & 1) && !(y & 1))
      v = reinterpret_cast<const uint4*>(in)[((n * Hc + (y >> 1)) * Wc + (x >> 1)) * C8 + c];
    reinterpret_cast<uint4*>(out)[i] = v;
  }
}

void s2c_expand_launch(const bf16* in, bf16* out, int N, int Hc, int Wc, int C, hipStream_t st) {
  const int64_t total = (int64_t)N * 4 * Hc * Wc * (C / 8);
  hipLaunchKernelGGL(s2c_expand_kernel, dim3((unsigned)std::min<int64_t>(cdiv64(total, 256), 8192)),
                     dim3(256), 0, st, in, out, Hc, Wc, C / 8, total);
}

// dst <- src [+ add] over NHWC rows of C channels, each operand with its own row stride (a concat
// slab slice or a dense tensor). With `add` it is the gradient junction of a slab slice that also
// fed a dense copy (DLA / SimpleDLA trees): the two gradients summed in fp32, rounded once — the
// arithmetic of the autograd bf16 add it replaces.
template <bool ADD>
__global__ __launch_bounds__(256) void copy_rows_kernel(const bf16* __restrict__ src, int lds,
                                                        bf16* __restrict__ dst, int ldd, int P,
                                                        int C, const bf16* __restrict__ add,
                                                        int lda) {
  const int G = C / 8;
  const size_t total = (size_t)P * G;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (size_t)gridDim.x * 256) {
    const size_t p = i / G, c = (i - p * G) * 8;
    uint4 v = *reinterpret_cast<const uint4*>(src + p * lds + c);
    if constexpr (ADD) {
      float a[8], b[8];
      unpack8(v, a);
      unpack8(*reinterpret_cast<const uint4*>(add + p * lda + c), b);
#pragma unroll
      for (int k = 0; k < 8; ++k) a[k] += b[k];
      v = pack8(a);
    }
    *reinterpret_cast<uint4*>(dst + p * ldd + c) = v;
  }
}

void copy_rows_launch(const bf16* src, int lds, bf16* dst, int ldd, int P, int C, hipStream_t st,
                      const bf16* add, int lda) {
  if (add)
    hipLaunchKernelGGL(copy_rows_kernel<true>, dim3(grid_cap((size_t)P * C / 8)), dim3(256), 0, st,
                       src, lds, dst, ldd, P, C, add, lda);
  else
    hipLaunchKernelGGL(copy_rows_kernel<false>, dim3(grid_cap((size_t)P * C / 8)), dim3(256), 0, st,
                       src, lds, dst, ldd, P, C, nullptr, 0);
}

// ---- ShuffleNetV2 join: shuffle(cat[a, b], groups=2) with equal widths C is the channel
// interleave y[p][2i] = a[p][i], y[p][2i+1] = b[p][i] (shufflenetv2.py:49/73, ShuffleBlock
// 10-19); one vectorized pass instead of a concat and a transposing copy. INV de-interleaves
// (the backward).
// word-level interleave of two bf16 pairs: (a0 a1), (b0 b1) -> (a0 b0), (a1 b1) and back
__device__ __forceinline__ void il_words(uint32_t ua, uint32_t ub, uint32_t& lo, uint32_t& hi) {
  lo = (ua & 0xffffu) | (ub << 16);
  hi = (ua >> 16) | (ub & 0xffff0000u);
}

// SPLIT: y is held as its two channel halves, y = [N,H,W,C] channels [0, C) and y1 = [C, 2C)
// (the next ShuffleNetV2 block's SplitBlock halves, shufflenetv2.py:22-29, so the split is never
// a pass of its own); needs C % (2V) == 0 so that no 2V-channel group straddles the halves.
// ldh: row stride of the y1 half (>= C): the next block's branch input held zero-padded to a
// multiple of 8 channels (the forward writes the padding zeros), so its odd-width 1x1 conv reads
// it in place instead of a pad pass (shufflenetv2.py:41 conv1 on the 58-channel half).
template <int V, bool INV, bool SPLIT = false>
__global__ __launch_bounds__(256) void interleave2_kernel(bf16* __restrict__ a, bf16* __restrict__ b,
                                                          bf16* __restrict__ y0, int P, int C,
                                                          bf16* __restrict__ y1 = nullptr,
                                                          int ldh = 0) {
  const int G = C / V;
  const int total = P * G;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int gi = i % G, p = i / G;
    const size_t ia = (size_t)p * C + gi * V;         // element index in a / b
    size_t iy = (size_t)p * 2 * C + gi * 2 * V;       // element index in y
    bf16* y = y0;
    if constexpr (SPLIT) {
      const int k = gi * 2 * V;                       // channel in the joined [0, 2C)
      iy = k < C ? (size_t)p * C + k : (size_t)p * ldh + (k - C);
      if (k >= C) y = y1;
      if constexpr (!INV) {
        if (gi == G - 1)                              // (the row's last group: its padding)
          for (int c = C; c < ldh; ++c) y1[(size_t)p * ldh + c] = bf16(0.f);
      }
    }
    if constexpr (V == 4) {
      if constexpr (!INV) {
        const uint2 va = *reinterpret_cast<const uint2*>(a + ia);
        const uint2 vb = *reinterpret_cast<const uint2*>(b + ia);
        uint4 o;
        il_words(va.x, vb.x, o.x, o.y);
        il_words(va.y, vb.y, o.z, o.w);
        *reinterpret_cast<uint4*>(y + iy) = o;
      } else {
        const uint4 o = *reinterpret_cast<const uint4*>(y + iy);
        uint2 va, vb;
        il_words(o.x, o.y, va.x, vb.x);   // the same word shuffle is its own inverse
        il_words(o.z, o.w, va.y, vb.y);
        *reinterpret_cast<uint2*>(a + ia) = va;
        *reinterpret_cast<uint2*>(b + ia) = vb;
      }
    } else if constexpr (V == 2) {
      if constexpr (!INV) {
        uint2 o;
        il_words(*reinterpret_cast<const uint32_t*>(a + ia), *reinterpret_cast<const uint32_t*>(b + ia),
                 o.x, o.y);
        *reinterpret_cast<uint2*>(y + iy) = o;
      } else {
        const uint2 o = *reinterpret_cast<const uint2*>(y + iy);
        uint32_t ua, ub;
        il_words(o.x, o.y, ua, ub);
        *reinterpret_cast<uint32_t*>(a + ia) = ua;
        *reinterpret_cast<uint32_t*>(b + ia) = ub;
      }
    } else {
      if constexpr (!INV) {
        y[iy] = a[ia];
        y[iy + 1] = b[ia];
      } else {
        a[ia] = y[iy];
        b[ia] = y[iy + 1];
      }
    }
  }
}

// y1 != nullptr: the joined tensor as two halves (y = channels [0, C), y1 = [C, 2C) with row
// stride ldh >= C, 0 = C)
void interleave2_launch(bf16* a, bf16* b, bf16* y, int P, int C, bool inverse, hipStream_t st,
                        bf16* y1, int ldh) {
  if (ldh <= 0) ldh = C;
  const int V = y1 ? (C % 8 == 0 ? 4 : C % 4 == 0 ? 2 : 1) : (C % 4 == 0 ? 4 : C % 2 == 0 ? 2 : 1);
  const dim3 grid(grid_cap((size_t)P * C / V)), block(256);
#define PCA_IL(VV)                                                                                  \
  if (V == VV) {                                                                                    \
    if (y1 && inverse)                                                                              \
      hipLaunchKernelGGL((interleave2_kernel<VV, true, true>), grid, block, 0, st, a, b, y, P, C, y1, ldh); \
    else if (y1)                                                                                    \
      hipLaunchKernelGGL((interleave2_kernel<VV, false, true>), grid, block, 0, st, a, b, y, P, C, y1, ldh); \
    else if (inverse)                                                                               \
      hipLaunchKernelGGL((interleave2_kernel<VV, true>), grid, block, 0, st, a, b, y, P, C, nullptr, 0); \
    else                                                                                            \
      hipLaunchKernelGGL((interleave2_kernel<VV, false>), grid, block, 0, st, a, b, y, P, C, nullptr, 0); \
    return;                                                                                         \
  }
  PCA_IL(4) PCA_IL(2) PCA_IL(1)
#undef PCA_IL
}

// ----------------------------------------------------------------------- cross-entropy
// logits[N][K] fp32, targets int64. One 256-thread block, deterministic reductions.
// Writes loss (mean), dlogits = (softmax - onehot) / N, and accumulates
// metrics[0] += sum loss, metrics[1] += correct, metrics[2] += N (fp64 accumulator).
// One block of up to 1024 threads (one sample per thread up to bs1024). For K <= kCeRegK the
// logits row is loaded once into registers with clamped, all-issued loads (the row loop of the
// first version re-read it three times as a dependent chain: 19 us at bs1024); wave sums + one
// LDS pass reduce the loss and the correct count.
constexpr int kCeRegK = 16;
__global__ __launch_bounds__(1024) void ce_fused_kernel(const float* __restrict__ logits,
                                                        const int64_t* __restrict__ tgt, int N,
                                                        int K, float* __restrict__ loss,
                                                        float* __restrict__ dlogits,
                                                        double* __restrict__ metrics) {
  __shared__ float sl[16];
  __shared__ int sc[16];
  float lsum = 0.f;
  int corr = 0;
  const float invN = 1.f / N;
  for (int n = threadIdx.x; n < N; n += blockDim.x) {
    const float* row = logits + (size_t)n * K;
    const int64_t t64 = tgt[n];
    // a label outside [0, K) poisons this sample's loss and gradient with NaN (the trainer's
    // non-finite-loss guard then stops the run, as F.cross_entropy would raise) instead of
    // silently training on a wrong logit or reading past the row
    const bool bad = t64 < 0 || t64 >= K;
    const int t = bad ? 0 : (int)t64;
    if (bad) {
      lsum += __builtin_nanf("");
      if (dlogits)
        for (int k = 0; k < K; ++k) dlogits[(size_t)n * K + k] = __builtin_nanf("");
      continue;
    }
    if (K <= kCeRegK) {
      float v[kCeRegK];
#pragma unroll
      for (int k = 0; k < kCeRegK; ++k) v[k] = row[min(k, K - 1)];
      float mx = v[0];
      int am = 0;
#pragma unroll
      for (int k = 1; k < kCeRegK; ++k)
        if (k < K && v[k] > mx) {
          mx = v[k];
          am = k;
        }
      float se = 0.f;
#pragma unroll
      for (int k = 0; k < kCeRegK; ++k) se += k < K ? __expf(v[k] - mx) : 0.f;
      const float lse = mx + __logf(se);
      float vt = v[0];
#pragma unroll
      for (int k = 1; k < kCeRegK; ++k) vt = k == t ? v[k] : vt;
      lsum += lse - vt;
      corr += (am == t);
      if (dlogits) {
#pragma unroll
        for (int k = 0; k < kCeRegK; ++k)
          if (k < K) dlogits[(size_t)n * K + k] = (__expf(v[k] - lse) - (k == t ? 1.f : 0.f)) * invN;
      }
      continue;
    }
    float mx = -INFINITY;
    int am = 0;
    for (int k = 0; k < K; ++k) {
      const float v = row[k];
      if (v > mx) {
        mx = v;
        am = k;
      }
    }
    float se = 0.f;
    for (int k = 0; k < K; ++k) se += __expf(row[k] - mx);
    const float lse = mx + __logf(se);
    lsum += lse - row[t];
    corr += (am == t);
    if (dlogits) {
      for (int k = 0; k < K; ++k) {
        const float p = __expf(row[k] - lse);
        dlogits[(size_t)n * K + k] = (p - (k == t ? 1.f : 0.f)) * invN;
      }
    }
  }
  lsum = wave_sum(lsum);
  corr = wave_sum(corr);
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63, nw = blockDim.x >> 6;
  if (lane == 0) {
    sl[wid] = lsum;
    sc[wid] = corr;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float a = 0.f;
    int c = 0;
    for (int w = 0; w < nw; ++w) {   // fixed order: deterministic
      a += sl[w];
      c += sc[w];
    }
    loss[0] = a / N;
    if (metrics) {
      metrics[0] += (double)a / N;
      metrics[1] += (double)c;
      metrics[2] += (double)N;
    }
  }
}

__global__ void scale_by_scalar_kernel(const float* __restrict__ g, const float* __restrict__ s,
                                       size_t n, float* __restrict__ out) {
  const float v = s[0];
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    out[i] = g[i] * v;
}

// ---------------------------------------------------------------------------------- SGD
// Multi-tensor SGD with momentum/weight decay/nesterov/dampening (torch.optim.SGD semantics).
// `meta` holds per-chunk {tensor index, start, end}; ptrs holds param/grad/buf pointers.
struct SgdArgs {
  const int64_t* chunks;   // [nchunks][3]
  float* const* params;
  const float* const* grads;
  float* const* bufs;
  bf16* const* shadows;    // optional bf16 copies (nullptr entries allowed)
  const float* lr;         // device scalar (graph-capture friendly)
  float momentum, dampening, wd, grad_scale;
  int nesterov, first;
  int zero_grad;           // clear each gradient after reading it (the next step's zero_grad)
};

// one element of the update with explicit FMAs, shared by every SGD path (the plain chunks and
// the fused update + prep) so that all of them round identically
__device__ __forceinline__ float sgd_elem(float pv, float gv, float& bv, float lr, float momentum,
                                          float dampening, float wd, float grad_scale, int nesterov,
                                          int first) {
  float d = gv * grad_scale;
  if (wd != 0.f) d = __builtin_fmaf(wd, pv, d);
  if (momentum != 0.f) {
    bv = first ? d : __builtin_fmaf(momentum, bv, (1.f - dampening) * d);
    d = nesterov ? __builtin_fmaf(momentum, bv, d) : bv;
  }
  return __builtin_fmaf(-lr, d, pv);
}

__device__ __forceinline__ void sgd_chunk(const SgdArgs& a, int blk) {
  const int64_t* ch = a.chunks + (size_t)blk * 3;
  const int t = (int)ch[0];
  const int64_t s = ch[1], e = ch[2];
  float* p = a.params[t];
  const float* g = a.grads[t];
  float* b = a.bufs[t];
  bf16* sh = a.shadows ? a.shadows[t] : nullptr;
  const float lr = a.lr[0];
  if (((s | e) & 3) == 0 && !sh && g && ((reinterpret_cast<uintptr_t>(p) | reinterpret_cast<uintptr_t>(g) |
                                          reinterpret_cast<uintptr_t>(b)) & 15) == 0) {
    // float4 path: 16-byte loads/stores of param, grad and momentum (the whole arena)
    float4* p4 = reinterpret_cast<float4*>(p);
    const float4* g4 = reinterpret_cast<const float4*>(g);
    float4* b4 = reinterpret_cast<float4*>(b);
    for (int64_t i = s / 4 + threadIdx.x; i < e / 4; i += 256) {
      const float4 gv = g4[i], pv = p4[i];
      float pf[4] = {pv.x, pv.y, pv.z, pv.w}, gf[4] = {gv.x, gv.y, gv.z, gv.w}, bf[4] = {0.f, 0.f, 0.f, 0.f};
      if (a.momentum != 0.f && !a.first) {
        const float4 bv = b4[i];
        bf[0] = bv.x; bf[1] = bv.y; bf[2] = bv.z; bf[3] = bv.w;
      }
#pragma unroll
      for (int k = 0; k < 4; ++k)
        pf[k] = sgd_elem(pf[k], gf[k], bf[k], lr, a.momentum, a.dampening, a.wd, a.grad_scale,
                         a.nesterov, a.first);
      if (a.momentum != 0.f) b4[i] = make_float4(bf[0], bf[1], bf[2], bf[3]);
      p4[i] = make_float4(pf[0], pf[1], pf[2], pf[3]);
      if (a.zero_grad) const_cast<float4*>(g4)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    return;
  }
  for (int64_t i = s + threadIdx.x; i < e; i += 256) {
    float bv = (a.momentum != 0.f && !a.first) ? b[i] : 0.f;
    const float np = sgd_elem(p[i], g ? g[i] : 0.f, bv, lr, a.momentum, a.dampening, a.wd,
                              a.grad_scale, a.nesterov, a.first);
    if (a.momentum != 0.f) b[i] = bv;
    p[i] = np;
    if (a.zero_grad && g) const_cast<float*>(g)[i] = 0.f;
    if (sh) sh[i] = f2bf(np);
  }
}

__global__ __launch_bounds__(256) void sgd_kernel(SgdArgs a) { sgd_chunk(a, blockIdx.x); }

// The SGD update of one element for the fused update + weight-prep launch (same arithmetic as
// sgd_chunk): reads grad / momentum at index i of the tensor's arena views, writes the new master
// and momentum, returns the new master for the bf16 operand copies.
struct SgdUpd {
  const int64_t* gm;       // [tensors][2] {grad, momentum} pointers parallel to the prep desc
  const float* lr;
  float momentum, dampening, wd, grad_scale;
  int nesterov, first, zero_grad;
};

__device__ __forceinline__ float sgd_upd(const SgdUpd& u, float lr, float* w, const float* g,
                                         float* m, int i) {
  float bv = (u.momentum != 0.f && !u.first) ? m[i] : 0.f;
  const float np = sgd_elem(w[i], g[i], bv, lr, u.momentum, u.dampening, u.wd, u.grad_scale,
                            u.nesterov, u.first);
  if (u.momentum != 0.f) m[i] = bv;
  w[i] = np;
  if (u.zero_grad) const_cast<float*>(g)[i] = 0.f;
  return np;
}

// -------------------------------------------------------------------------- SE / acts
// out[n,hw,c] = x[n,hw,c] * sigmoid(s[n,c])   (s = pre-sigmoid excitation logits, fp32)
__global__ void se_scale_fwd_kernel(const bf16* __restrict__ x, const float* __restrict__ s,
                                    int N, int HW, int C, bf16* __restrict__ out) {
  const size_t total = (size_t)N * HW * C;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const int n = (int)(i / ((size_t)HW * C));
    out[i] = f2bf(bf2f(x[i]) * sigmoidf_(s[(size_t)n * C + c]));
  }
}

// dx = dout * sig(s);  ds[n,c] = sum_hw dout*x * sig'(s). One block per (n, 64-channel tile).
__global__ __launch_bounds__(256) void se_scale_bwd_kernel(const bf16* __restrict__ dout,
                                                           const bf16* __restrict__ x,
                                                           const float* __restrict__ s, int N,
                                                           int HW, int C, bf16* __restrict__ dx,
                                                           float* __restrict__ ds) {
  __shared__ float red[4][64];
  const int n = blockIdx.y;
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int r = threadIdx.x >> 6;
  float acc = 0.f;
  if (c < C) {
    const float sg = sigmoidf_(s[(size_t)n * C + c]);
    for (int hw = r; hw < HW; hw += 4) {
      const size_t i = ((size_t)n * HW + hw) * C + c;
      const float d = bf2f(dout[i]);
      dx[i] = f2bf(d * sg);
      acc += d * bf2f(x[i]);
    }
    acc *= sg * (1.f - sg);
  }
  red[r][threadIdx.x & 63] = acc;
  __syncthreads();
  if (r == 0 && c < C)
    ds[(size_t)n * C + c] = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] +
                            red[3][threadIdx.x];
}

// ---- vectorized (8-channel, 16-byte) global pooling / squeeze-excite scaling, C % 8 == 0 and
// C <= 2048: one block per image, thread t owns channel group t % G and walks the pixels
// hw = t / G, + RW, ... (RW = 256 / G pixel lanes), lanes reduced through LDS in a fixed order.
// The scalar kernels above (2-byte accesses, 64-bit index math, one pixel chain per thread) run
// the EfficientNet-B0 squeeze-excite path at a fraction of HBM bandwidth.
__global__ __launch_bounds__(256) void gap_fwd8_kernel(const bf16* __restrict__ x, int HW, int C,
                                                       float* __restrict__ y) {
  __shared__ float red[256 * 8];
  const int G = C >> 3, RW = 256 / G;
  const int t = threadIdx.x, gi = t % G, r = t / G, n = blockIdx.x;
  float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (r < RW) {
    const bf16* p = x + (size_t)n * HW * C + gi * 8;
    for (int hw = r; hw < HW; hw += RW) {
      float f[8];
      unpack8(*reinterpret_cast<const uint4*>(p + (size_t)hw * C), f);
#pragma unroll
      for (int v = 0; v < 8; ++v) a[v] += f[v];
    }
  }
#pragma unroll
  for (int v = 0; v < 8; ++v) red[t * 8 + v] = a[v];
  __syncthreads();
  if (t < G) {
    const float inv = 1.f / HW;
#pragma unroll
    for (int v = 0; v < 8; ++v) {
      float s = 0.f;
      for (int j = 0; j < RW; ++j) s += red[(j * G + t) * 8 + v];
      y[(size_t)n * C + t * 8 + v] = s * inv;
    }
  }
}

__global__ __launch_bounds__(256) void gap_bwd8_kernel(const float* __restrict__ dy, int N, int HW,
                                                       int C, bf16* __restrict__ dx) {
  const int G = C >> 3;
  const int total = N * HW * G;
  const float inv = 1.f / HW;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int gi = i % G, n = i / (HW * G);
    const float4 a = *reinterpret_cast<const float4*>(dy + (size_t)n * C + gi * 8);
    const float4 b = *reinterpret_cast<const float4*>(dy + (size_t)n * C + gi * 8 + 4);
    const float f[8] = {a.x * inv, a.y * inv, a.z * inv, a.w * inv,
                        b.x * inv, b.y * inv, b.z * inv, b.w * inv};
    *reinterpret_cast<uint4*>(dx + (size_t)i * 8) = pack8(f);
  }
}

__global__ __launch_bounds__(256) void se_scale_fwd8_kernel(const bf16* __restrict__ x,
                                                            const float* __restrict__ s, int N,
                                                            int HW, int C, bf16* __restrict__ out) {
  const int G = C >> 3;
  const int total = N * HW * G;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int gi = i % G, n = i / (HW * G);
    const float* sp = s + (size_t)n * C + gi * 8;
    float f[8];
    unpack8(*reinterpret_cast<const uint4*>(x + (size_t)i * 8), f);
#pragma unroll
    for (int v = 0; v < 8; ++v) f[v] *= sigmoidf_(sp[v]);
    *reinterpret_cast<uint4*>(out + (size_t)i * 8) = pack8(f);
  }
}

// dx = dout * sig(s); ds[n,c] = sum_hw dout*x * sig'(s); one block per image (DX = false: ds
// only, dx is written later by se_dx8_kernel together with the squeeze path's gradient)
template <bool DX>
__global__ __launch_bounds__(256) void se_scale_bwd8_kernel(const bf16* __restrict__ dout,
                                                            const bf16* __restrict__ x,
                                                            const float* __restrict__ s, int HW,
                                                            int C, bf16* __restrict__ dx,
                                                            float* __restrict__ ds) {
  __shared__ float red[256 * 8];
  const int G = C >> 3, RW = 256 / G;
  const int t = threadIdx.x, gi = t % G, r = t / G, n = blockIdx.x;
  float sg[8], a[8];
#pragma unroll
  for (int v = 0; v < 8; ++v) {
    a[v] = 0.f;
    sg[v] = r < RW ? sigmoidf_(s[(size_t)n * C + gi * 8 + v]) : 0.f;
  }
  if (r < RW) {
    const size_t base = (size_t)n * HW * C + gi * 8;
    for (int hw = r; hw < HW; hw += RW) {
      const size_t e = base + (size_t)hw * C;
      float d[8], xv[8], o[8];
      unpack8(*reinterpret_cast<const uint4*>(dout + e), d);
      unpack8(*reinterpret_cast<const uint4*>(x + e), xv);
#pragma unroll
      for (int v = 0; v < 8; ++v) {
        o[v] = d[v] * sg[v];
        a[v] += d[v] * xv[v];
      }
      if (DX) *reinterpret_cast<uint4*>(dx + e) = pack8(o);
    }
  }
#pragma unroll
  for (int v = 0; v < 8; ++v) red[t * 8 + v] = a[v];
  __syncthreads();
  if (t < G) {
#pragma unroll
    for (int v = 0; v < 8; ++v) {
      float acc = 0.f;
      for (int j = 0; j < RW; ++j) acc += red[(j * G + t) * 8 + v];
      ds[(size_t)n * C + t * 8 + v] = acc * sg[v] * (1.f - sg[v]);
    }
  }
}

// ---- squeeze-excite MLP on the pooled [N, C] fp32 vector (efficientnet.py:26-36, senet.py:
// 59-66, regnet.py:15-24): s = W2 act(W1 p + b1) + b2, W1 [R][C], W2 [C][R] (the 1x1 convs'
// fp32 masters). Four small kernels replace the library GEMM / GEMV / elementwise chain (5
// launches forward, 8 backward): two "row" dot kernels (a wave per 8 samples x 4 outputs, lanes
// across the C reduction) and two "column" kernels (a thread per channel x 8 samples, the short
// R reduction serial), so even a 128-sample batch spreads over many waves with short
// dependency chains — a staged-tile variant with one block per 8 samples ran 10-200 us per call.
constexpr int kSeNB = 8;        // samples per wave / thread
constexpr int kSeRC = 4;        // row outputs per wave

__device__ __forceinline__ float se_act(float v, int act) {
  return act == ACT_RELU ? fmaxf(v, 0.f) : v * sigmoidf_(v);
}
__device__ __forceinline__ float se_act_grad(float v, int act) {
  return act == ACT_RELU ? (v > 0.f ? 1.f : 0.f) : act_grad(v, ACT_SWISH);
}

// out[n][r] = sum_c a[n][c] W(r, c) with W(r, c) = w[r*C + c] (WT = false, W1) or w[c*R + r]
// (WT = true, W2).  Forward (BWD = false): out = hpre = sum + b1[r].  Backward: out = dz =
// sum * act'(hpre[n][r]).  One block per (8-sample group, 4 outputs): its 4 waves split the C
// reduction (two channels per lane in flight), then combine through LDS.
template <bool WT, bool BWD>
__global__ __launch_bounds__(256) void se_rowdot_kernel(const float* __restrict__ a, int N, int C,
                                                        int R, const float* __restrict__ w,
                                                        const float* __restrict__ b1,
                                                        const float* __restrict__ hpre, int act,
                                                        float* __restrict__ out) {
  __shared__ float part[4][kSeNB * kSeRC];
  const int lane = threadIdx.x & 63, wv_id = threadIdx.x >> 6;
  const int rgroups = cdiv(R, kSeRC);
  const int n0 = (blockIdx.x / rgroups) * kSeNB, r0 = (blockIdx.x % rgroups) * kSeRC;
  float acc[kSeNB][kSeRC];
#pragma unroll
  for (int i = 0; i < kSeNB; ++i)
#pragma unroll
    for (int j = 0; j < kSeRC; ++j) acc[i][j] = 0.f;
  int rr[kSeRC], nn[kSeNB];
#pragma unroll
  for (int j = 0; j < kSeRC; ++j) rr[j] = min(r0 + j, R - 1);   // clamped: computed, not stored
#pragma unroll
  for (int i = 0; i < kSeNB; ++i) nn[i] = min(n0 + i, N - 1);
  for (int c0 = wv_id * 64 + lane; c0 < C; c0 += 512) {
    const int c1 = min(c0 + 256, C - 1);
    const float keep = c0 + 256 < C ? 1.f : 0.f;       // second channel of the pair, if any
    float wv[2][kSeRC], av[2][kSeNB];
#pragma unroll
    for (int j = 0; j < kSeRC; ++j) {
      wv[0][j] = WT ? w[(size_t)c0 * R + rr[j]] : w[(size_t)rr[j] * C + c0];
      wv[1][j] = (WT ? w[(size_t)c1 * R + rr[j]] : w[(size_t)rr[j] * C + c1]) * keep;
    }
#pragma unroll
    for (int i = 0; i < kSeNB; ++i) {
      av[0][i] = a[(size_t)nn[i] * C + c0];
      av[1][i] = a[(size_t)nn[i] * C + c1];
    }
#pragma unroll
    for (int i = 0; i < kSeNB; ++i)
#pragma unroll
      for (int j = 0; j < kSeRC; ++j) acc[i][j] += av[0][i] * wv[0][j] + av[1][i] * wv[1][j];
  }
#pragma unroll
  for (int i = 0; i < kSeNB; ++i)
#pragma unroll
    for (int j = 0; j < kSeRC; ++j) {
      const float v = wave_sum(acc[i][j]);
      if (lane == 0) part[wv_id][i * kSeRC + j] = v;
    }
  __syncthreads();
  if (threadIdx.x < kSeNB * kSeRC) {
    const int i = threadIdx.x / kSeRC, j = threadIdx.x % kSeRC, n = n0 + i, r = r0 + j;
    const float v = part[0][threadIdx.x] + part[1][threadIdx.x] + part[2][threadIdx.x] +
                    part[3][threadIdx.x];
    if (n < N && r < R) {
      const size_t o = (size_t)n * R + r;
      out[o] = BWD ? v * se_act_grad(hpre[o], act) : v + (b1 ? b1[r] : 0.f);
    }
  }
}

// out[n][c] = bias[c] + sum_r h(n, r) W(r, c), h = act(hin) (ACTIN) or hin; W(r, c) =
// w[c*R + r] (WT = true, W2) or w[r*C + c] (WT = false, W1).  Thread -> (channel, 8 samples);
// the block's 8 x R input rows are staged in LDS (R <= 256).
template <bool WT, bool ACTIN>
__global__ __launch_bounds__(256) void se_coldot_kernel(const float* __restrict__ hin, int N, int C,
                                                        int R, const float* __restrict__ w,
                                                        const float* __restrict__ bias, int act,
                                                        float* __restrict__ out) {
  __shared__ float hs[kSeNB * 256];
  const int n0 = blockIdx.y * kSeNB, c = blockIdx.x * 256 + threadIdx.x;
  for (int i = threadIdx.x; i < kSeNB * R; i += 256) {
    const int n = n0 + i / R;
    const float v = n < N ? hin[(size_t)n0 * R + i] : 0.f;
    hs[i] = ACTIN ? se_act(v, act) : v;
  }
  __syncthreads();
  if (c >= C) return;
  float acc[kSeNB];
  const float b = bias ? bias[c] : 0.f;
#pragma unroll
  for (int i = 0; i < kSeNB; ++i) acc[i] = b;
  for (int r = 0; r < R; ++r) {
    const float wv = WT ? w[(size_t)c * R + r] : w[(size_t)r * C + c];
#pragma unroll
    for (int i = 0; i < kSeNB; ++i) acc[i] += hs[i * R + r] * wv;
  }
#pragma unroll
  for (int i = 0; i < kSeNB; ++i)
    if (n0 + i < N) out[(size_t)(n0 + i) * C + c] = acc[i];
}

// backward, parameter part, added into the gradient buffers with fp32 atomics:
//   dW2[c][r] += sum_n ds[n][c] h[n][r], db2[c] += sum_n ds[n][c],
//   dW1[r][c] += sum_n dz[n][r] p[n][c], db1[r] += sum_n dz[n][r].
// Grid (C / 32 channel tiles, sample chunks); each block walks its chunk 32 samples at a time.
// LDS: dsT[32][32] | pT[32][32] | hs[32][R] | dzs[32][R]
constexpr int kSeWC = 32, kSeWN = 32;
template <int J>   // J >= outputs per thread = 2 * 32 * R / 256
__global__ __launch_bounds__(256) void se_mlp_bwd_param_kernel(
    const float* __restrict__ ds, const float* __restrict__ dz, const float* __restrict__ hpre,
    const float* __restrict__ pooled, int N, int C, int R, int act, int chunk,
    float* __restrict__ dw1, float* __restrict__ db1, float* __restrict__ dw2,
    float* __restrict__ db2) {
  extern __shared__ float sm[];
  float* dsT = sm;
  float* pT = dsT + kSeWN * kSeWC;
  float* hs = pT + kSeWN * kSeWC;
  float* dzs = hs + kSeWN * R;
  const int t = threadIdx.x, c0 = blockIdx.x * kSeWC;
  const int tc = min(kSeWC, C - c0);
  const int nbeg = blockIdx.y * chunk, nend = min(N, nbeg + chunk);
  const int nout = 2 * kSeWC * R;
  const bool do_b1 = blockIdx.x == 0 && db1 != nullptr;
  float acc[J];
#pragma unroll
  for (int j = 0; j < J; ++j) acc[j] = 0.f;
  float bacc = 0.f;
  for (int nb0 = nbeg; nb0 < nend; nb0 += kSeWN) {
    const int nn = min(kSeWN, nend - nb0);
    __syncthreads();
    for (int i = t; i < kSeWN * kSeWC; i += 256) {
      const int n = i / kSeWC, cc = i % kSeWC;
      const bool ok = n < nn && cc < tc;
      dsT[i] = ok ? ds[(size_t)(nb0 + n) * C + c0 + cc] : 0.f;
      pT[i] = ok ? pooled[(size_t)(nb0 + n) * C + c0 + cc] : 0.f;
    }
    for (int i = t; i < kSeWN * R; i += 256) {
      const int n = i / R;
      const bool ok = n < nn;
      hs[i] = ok ? se_act(hpre[(size_t)nb0 * R + i], act) : 0.f;
      dzs[i] = ok ? dz[(size_t)nb0 * R + i] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int o = t + 256 * j;
      if (o < nout) {
        float a = 0.f;
        if (o < kSeWC * R) {            // dW2[c0 + cc][r]
          const int cc = o / R, r = o % R;
          for (int n = 0; n < kSeWN; ++n) a += dsT[n * kSeWC + cc] * hs[n * R + r];
        } else {                        // dW1[r][c0 + cc]
          const int o2 = o - kSeWC * R, r = o2 / kSeWC, cc = o2 % kSeWC;
          for (int n = 0; n < kSeWN; ++n) a += dzs[n * R + r] * pT[n * kSeWC + cc];
        }
        acc[j] += a;
      }
    }
    if (t < kSeWC) {
      for (int n = 0; n < kSeWN; ++n) bacc += dsT[n * kSeWC + t];
    } else if (do_b1 && t - kSeWC < R) {
      for (int n = 0; n < kSeWN; ++n) bacc += dzs[n * R + t - kSeWC];
    }
  }
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int o = t + 256 * j;
    if (o < nout) {
      if (o < kSeWC * R) {
        const int cc = o / R, r = o % R;
        if (cc < tc) atomicAdd(dw2 + (size_t)(c0 + cc) * R + r, acc[j]);
      } else {
        const int o2 = o - kSeWC * R, r = o2 / kSeWC, cc = o2 % kSeWC;
        if (cc < tc) atomicAdd(dw1 + (size_t)r * C + c0 + cc, acc[j]);
      }
    }
  }
  if (t < tc && db2) atomicAdd(db2 + c0 + t, bacc);
  else if (do_b1 && t >= kSeWC && t - kSeWC < R) atomicAdd(db1 + t - kSeWC, bacc);
}

// ---- squeeze-excite in few launches (efficientnet.py:26-36, senet.py:59-66): one block per NB
// samples does everything that reduces over a sample — forward: pool + both MLP layers
// (se_fwd_fused_kernel; + se_scale_fwd = 2 launches); backward: the excitation reduce ds and
// the MLP data path dz, dp (se_bwd_data_kernel; + the parameter kernel + se_dx = 3 launches).
// The MLP weights stream through each block once per NB samples; NB grows with the batch so
// large batches do not multiply the weight traffic (NB = 1 at the 8-GPU shard's 128 samples).
// LDS: vec [NB][C] (pooled / ds) | h [NB][R] | red [256 * 8]
constexpr int kSeFusedMaxC = 2048, kSeFusedMaxR = 192;

template <int NB>
__device__ __forceinline__ void se_pool8(const bf16* __restrict__ x, const bf16* __restrict__ dout,
                                         const float* __restrict__ s, int HW, int C, int n,
                                         float* red, float* outv) {
  // outv[c] = mean_hw x (dout == nullptr) or sum_hw dout*x * sig'(s) (excitation gradient)
  const int G = C >> 3, RW = 256 / G;
  const int t = threadIdx.x, gi = t % G, r = t / G;
  float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (r < RW) {
    const size_t base = (size_t)n * HW * C + gi * 8;
    for (int hw = r; hw < HW; hw += RW) {
      float f[8];
      unpack8(*reinterpret_cast<const uint4*>(x + base + (size_t)hw * C), f);
      if (dout) {
        float d[8];
        unpack8(*reinterpret_cast<const uint4*>(dout + base + (size_t)hw * C), d);
#pragma unroll
        for (int v = 0; v < 8; ++v) a[v] += d[v] * f[v];
      } else {
#pragma unroll
        for (int v = 0; v < 8; ++v) a[v] += f[v];
      }
    }
  }
#pragma unroll
  for (int v = 0; v < 8; ++v) red[t * 8 + v] = a[v];
  __syncthreads();
  if (t < G) {
#pragma unroll
    for (int v = 0; v < 8; ++v) {
      float acc = 0.f;
      for (int j = 0; j < RW; ++j) acc += red[(j * G + t) * 8 + v];
      if (dout) {
        const float sg = sigmoidf_(s[(size_t)n * C + t * 8 + v]);
        outv[t * 8 + v] = acc * sg * (1.f - sg);
      } else {
        outv[t * 8 + v] = acc / HW;
      }
    }
  }
  __syncthreads();
}

// w2t: W2 transposed, [R][C] (the weight-prep plan's fp32 copy, ops/functional.py _dw_weight):
// the layer-2 / dh reductions read it coalesced (W2's [C][R] rows put consecutive lanes 4R bytes
// apart: 64 cache lines per load instruction, the fused path's bottleneck at C = 1152, R = 48)
template <int NB>
__global__ __launch_bounds__(256) void se_fwd_fused_kernel(
    const bf16* __restrict__ x, int N, int HW, int C, int R, const float* __restrict__ w1,
    const float* __restrict__ b1, const float* __restrict__ w2t, const float* __restrict__ b2,
    int act, float* __restrict__ pooled, float* __restrict__ hpre, float* __restrict__ s) {
  extern __shared__ float sm[];
  float* vec = sm;                       // [NB][C]
  float* h = vec + NB * C;               // [NB][R]
  float* red = h + NB * R;               // [256 * 8]
  const int n0 = blockIdx.x * NB;
  const int nb = min(NB, N - n0);
  for (int k = 0; k < nb; ++k) se_pool8<NB>(x, nullptr, nullptr, HW, C, n0 + k, red, vec + k * C);
  for (int i = threadIdx.x; i < nb * C; i += 256) pooled[(size_t)n0 * C + i] = vec[i];
  // layer 1: each wave owns 8 output rows at a time, lanes across C (coalesced W1 rows): the 8
  // row loads per channel are independent (a wave per single row serialised 12+ load-latency
  // rounds per block at R = 48)
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int r0 = wv * 8; r0 < R; r0 += 32) {
    float a[NB][8];
#pragma unroll
    for (int k = 0; k < NB; ++k)
#pragma unroll
      for (int j = 0; j < 8; ++j) a[k][j] = 0.f;
    for (int c = lane; c < C; c += 64) {
      float pv[NB];
#pragma unroll
      for (int k = 0; k < NB; ++k) pv[k] = vec[k * C + c];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float w = r0 + j < R ? w1[(size_t)(r0 + j) * C + c] : 0.f;
#pragma unroll
        for (int k = 0; k < NB; ++k) a[k][j] += w * pv[k];
      }
    }
#pragma unroll
    for (int k = 0; k < NB; ++k)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int r = r0 + j;
        const float v = wave_sum(a[k][j]) + ((b1 && r < R) ? b1[r] : 0.f);
        if (lane == 0 && k < nb && r < R) {
          hpre[(size_t)(n0 + k) * R + r] = v;
          h[k * R + r] = se_act(v, act);
        }
      }
  }
  __syncthreads();
  // layer 2: a thread per channel against the block's h rows (W2^T rows: coalesced)
  for (int c = threadIdx.x; c < C; c += 256) {
    float a[NB];
#pragma unroll
    for (int k = 0; k < NB; ++k) a[k] = b2 ? b2[c] : 0.f;
#pragma unroll 8
    for (int r = 0; r < R; ++r) {
      const float w = w2t[(size_t)r * C + c];
#pragma unroll
      for (int k = 0; k < NB; ++k) a[k] += w * h[k * R + r];
    }
#pragma unroll
    for (int k = 0; k < NB; ++k)
      if (k < nb) s[(size_t)(n0 + k) * C + c] = a[k];
  }
}

template <int NB>
__global__ __launch_bounds__(256) void se_bwd_data_kernel(
    const bf16* __restrict__ dout, const bf16* __restrict__ x, const float* __restrict__ s,
    int N, int HW, int C, int R, const float* __restrict__ w1, const float* __restrict__ w2t,
    const float* __restrict__ hpre, int act, float* __restrict__ ds, float* __restrict__ dz,
    float* __restrict__ dp) {
  extern __shared__ float sm[];
  float* vec = sm;                       // [NB][C] ds
  float* h = vec + NB * C;               // [NB][R] dz
  float* red = h + NB * R;               // [256 * 8]
  const int n0 = blockIdx.x * NB;
  const int nb = min(NB, N - n0);
  for (int k = 0; k < nb; ++k) se_pool8<NB>(x, dout, s, HW, C, n0 + k, red, vec + k * C);
  for (int i = threadIdx.x; i < nb * C; i += 256) ds[(size_t)n0 * C + i] = vec[i];
  // dh[r] = sum_c ds[c] W2[c][r] = sum_c ds[c] W2^T[r][c]: each wave owns 8 rows at a time,
  // lanes across C (coalesced W2^T rows, 8 independent loads per channel), one wave sum per row
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int r0 = wv * 8; r0 < R; r0 += 32) {
    float p[NB][8];
#pragma unroll
    for (int k = 0; k < NB; ++k)
#pragma unroll
      for (int j = 0; j < 8; ++j) p[k][j] = 0.f;
    for (int c = lane; c < C; c += 64) {
      float dv[NB];
#pragma unroll
      for (int k = 0; k < NB; ++k) dv[k] = vec[k * C + c];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float w = r0 + j < R ? w2t[(size_t)(r0 + j) * C + c] : 0.f;
#pragma unroll
        for (int k = 0; k < NB; ++k) p[k][j] += w * dv[k];
      }
    }
#pragma unroll
    for (int k = 0; k < NB; ++k)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int r = r0 + j;
        const float v = wave_sum(p[k][j]);
        if (lane == 0 && k < nb && r < R) {
          const size_t o = (size_t)(n0 + k) * R + r;
          const float d = v * se_act_grad(hpre[o], act);
          dz[o] = d;
          h[k * R + r] = d;
        }
      }
  }
  __syncthreads();
  // dp[c] = sum_r W1[r][c] dz[r] (threads over c: coalesced W1 rows)
  for (int c = threadIdx.x; c < C; c += 256) {
    float a[NB];
#pragma unroll
    for (int k = 0; k < NB; ++k) a[k] = 0.f;
    for (int r = 0; r < R; ++r) {
      const float w = w1[(size_t)r * C + c];
#pragma unroll
      for (int k = 0; k < NB; ++k) a[k] += w * h[k * R + r];
    }
#pragma unroll
    for (int k = 0; k < NB; ++k)
      if (k < nb) dp[(size_t)(n0 + k) * C + c] = a[k];
  }
}

// dx = dout * sig(s) + dp / HW   (excitation path + broadcast squeeze-path gradient)
__global__ __launch_bounds__(256) void se_dx8_kernel(const bf16* __restrict__ dout,
                                                     const float* __restrict__ s,
                                                     const float* __restrict__ dp, int N, int HW,
                                                     int C, bf16* __restrict__ dx) {
  const int G = C >> 3;
  const int total = N * HW * G;
  const float inv = 1.f / HW;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int gi = i % G, n = i / (HW * G);
    const size_t sc = (size_t)n * C + gi * 8;
    float d[8];
    unpack8(*reinterpret_cast<const uint4*>(dout + (size_t)i * 8), d);
#pragma unroll
    for (int v = 0; v < 8; ++v) d[v] = d[v] * sigmoidf_(s[sc + v]) + dp[sc + v] * inv;
    *reinterpret_cast<uint4*>(dx + (size_t)i * 8) = pack8(d);
  }
}

__global__ void act_fwd_kernel(const bf16* __restrict__ x, size_t n, int act, bf16* __restrict__ y) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    y[i] = f2bf(apply_act(bf2f(x[i]), act));
}

__global__ void act_bwd_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ x, size_t n,
                               int act, bf16* __restrict__ dx) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    dx[i] = f2bf(bf2f(dy[i]) * act_grad(bf2f(x[i]), act));
}

// out = act(a + b), vectorized by 8 when possible
__global__ void add_act_kernel(const bf16* __restrict__ a, const bf16* __restrict__ b, size_t n,
                               int act, bf16* __restrict__ y) {
  const size_t nv = n / 8;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv;
       i += (size_t)gridDim.x * blockDim.x) {
    float fa[8], fb[8];
    unpack8(reinterpret_cast<const uint4*>(a)[i], fa);
    unpack8(reinterpret_cast<const uint4*>(b)[i], fb);
#pragma unroll
    for (int k = 0; k < 8; ++k) fa[k] = apply_act(fa[k] + fb[k], act);
    reinterpret_cast<uint4*>(y)[i] = pack8(fa);
  }
  for (size_t i = nv * 8 + (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    y[i] = f2bf(apply_act(bf2f(a[i]) + bf2f(b[i]), act));
}

// fp32 -> bf16 cast (weights) and the dgrad weight transpose
// w [G][Cn][T][Cr] -> wt [G][Cr][T][Cn]
__global__ void weight_prep_kernel(const float* __restrict__ w, int G, int Cn, int T, int Cr,
                                   bf16* __restrict__ wb, bf16* __restrict__ wt) {
  const size_t total = (size_t)G * Cn * T * Cr;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    const int ci = (int)(i % Cr);
    size_t q = i / Cr;
    const int t = (int)(q % T);
    q /= T;
    const int co = (int)(q % Cn);
    const int g = (int)(q / Cn);
    const bf16 v = f2bf(w[i]);
    if (wb) wb[i] = v;
    if (wt) wt[(((size_t)g * Cr + ci) * T + t) * Cn + co] = v;
  }
}

// Multi-tensor weight preparation: one launch converts every MFMA conv weight of a model
// (fp32 master [G*Cn][T][Cr], physical channels_last order) into its bf16 forward operand (same
// layout) and its bf16 transposed dgrad operand [G*Cr][T][Cn]. desc[t] = {w, wb, wt, G, Cn, T,
// Cr, numel}; chunks[b] = {t, a, b, pass}:
//   pass 0: elements [a, b) of the forward layout, 8 per thread (16-byte stores);
//   pass 1: 64x64 (co, ci) transpose tile number a of one (group, tap), staged through LDS so
//           both the fp32 reads (along ci) and the bf16 writes (along co) are coalesced;
//   pass 2: depthwise weight [Cn][T] -> fp32 tap-major copy [T][Cn] (desc wb = the copy) for
//           output channels [a, b), the layout the depthwise kernels read 8 channels at a time;
//   pass 3: rows [a, b) of a channel-padded forward copy (desc numel slot = padded width);
//   pass 4: pass 1 that also writes the forward copy of the tile's elements (one read of the
//           master feeds both operands; the plan then issues no pass-0 chunks for the weight);
//   pass 5: pass 4 for a per-group zero-padded operand (odd-width grouped / narrow convs): the
//           operands are [G*Cn][T][Cr] with Cn, Cr the padded widths, the master [G*mCn][T][mCr]
//           with desc numel slot = mCn << 32 | mCr; padded positions read nothing (each master
//           element is still read, and in the fused optimizer updated, exactly once);
//   pass 6: pass 4 for a block-diagonal super-group operand (narrow groups run as one group of
//           S = P x Cg channels): operand [G'*Cn][T][S], master [G'*Cn][T][Cg] with numel slot =
//           cout_g << 32 | Cg; output row r belongs to original group r / cout_g, whose Cg
//           channels sit at [lg*Cg, (lg+1)*Cg) of the S, lg = (r / cout_g) % P (zeros elsewhere).
// All index math is 32-bit and per block / per 8 elements (64-bit div/mod per element made the
// first version of this kernel 10x slower than its bandwidth).
// UPD: the fused optimizer form — every master element is read exactly once by the chunk plan,
// so it is SGD-updated there (sgd_upd) and the bf16 operands are written from the new value: the
// next forward finds its operands current and the separate prep pass (a full re-read of the
// masters right after the optimizer wrote them) is gone.
template <bool UPD>
__device__ __forceinline__ void prep_chunk(const int64_t* __restrict__ desc,
                                           const int64_t* __restrict__ ch, const SgdUpd& u,
                                           float (*tile)[65]) {
  const int64_t* d = desc + ch[0] * 8;
  float* const w = reinterpret_cast<float*>(d[0]);
  const int Cn = (int)d[4], T = (int)d[5], Cr = (int)d[6];
  const int tid = threadIdx.x;
  const float* ug = UPD ? reinterpret_cast<const float*>(u.gm[ch[0] * 2]) : nullptr;
  float* um = UPD ? reinterpret_cast<float*>(u.gm[ch[0] * 2 + 1]) : nullptr;
  const float lr = UPD ? u.lr[0] : 0.f;
  auto ld = [&](int i) -> float {
    if constexpr (UPD) return sgd_upd(u, lr, w, ug, um, i);
    else return w[i];
  };
  if (ch[3] == 2) {
    float* wtf = reinterpret_cast<float*>(d[1]);
    const int c0 = (int)ch[1], nc = (int)ch[2] - c0;
    for (int k = tid; k < nc * T; k += 256) {
      const int co = c0 + k / T, tap = k % T;
      wtf[tap * Cn + co] = ld(co * T + tap);
    }
    return;
  }
  if (ch[3] == 3) {
    // channel-padded bf16 copy (stem convs on 8-channel padded RGB): rows [r0, r1) of
    // [Cout*T][Cr] -> [Cout*T][Cp] with zeros in channels Cr..Cp-1 (Cp = desc[7])
    bf16* wb = reinterpret_cast<bf16*>(d[1]);
    const int Cp = (int)d[7], r0 = (int)ch[1], nr = (int)ch[2] - r0;
    for (int k = tid; k < nr * Cp; k += 256) {
      const int r = r0 + k / Cp, c = k % Cp;
      wb[r * Cp + c] = f2bf(c < Cr ? ld(r * Cr + c) : 0.f);
    }
    return;
  }
  if (ch[3] == 0) {
    bf16* wb = reinterpret_cast<bf16*>(d[1]);
    const int s0 = (int)ch[1], s1 = (int)ch[2];
    for (int i = s0 + tid * 8; i < s1; i += 256 * 8) {
      float f[8];
      if constexpr (UPD) {
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = ld(i + j);
      } else {
        const float4 v0 = *reinterpret_cast<const float4*>(w + i);
        const float4 v1 = *reinterpret_cast<const float4*>(w + i + 4);
        f[0] = v0.x; f[1] = v0.y; f[2] = v0.z; f[3] = v0.w;
        f[4] = v1.x; f[5] = v1.y; f[6] = v1.z; f[7] = v1.w;
      }
      *reinterpret_cast<uint4*>(wb + i) = pack8(f);
    }
    return;
  }
  bf16* wt = reinterpret_cast<bf16*>(d[2]);
  bf16* wbt = ch[3] >= 4 ? reinterpret_cast<bf16*>(d[1]) : nullptr;   // pass 4/5: + forward copy
  const int mCn = ch[3] >= 5 ? (int)(d[7] >> 32) : Cn;               // master widths
  const int mCr = ch[3] >= 5 ? (int)(d[7] & 0xffffffff) : Cr;
  const int nco = (Cn + 63) >> 6, nci = (Cr + 63) >> 6;
  int q = (int)ch[1];
  const int ci_t = q % nci;
  q /= nci;
  const int co_t = q % nco;
  q /= nco;
  const int tap = q % T;
  const int g = q / T;
  const int co0 = co_t * 64, ci0 = ci_t * 64;
  for (int k = tid; k < 64 * 64; k += 256) {
    const int r = k >> 6, c = k & 63;               // r: co, c: ci (contiguous in w)
    const int co = co0 + r, ci = ci0 + c;
    if (ch[3] == 6) {   // block diagonal: mCn = cout_g, mCr = Cg
      const int row = g * Cn + co, lg = (row / mCn) % (Cr / mCr), c_lo = lg * mCr;
      tile[r][c] = (co < Cn && ci >= c_lo && ci < c_lo + mCr)
                       ? ld((row * T + tap) * mCr + ci - c_lo) : 0.f;
    } else {
      tile[r][c] = (co < mCn && ci < mCr) ? ld(((g * mCn + co) * T + tap) * mCr + ci) : 0.f;
    }
  }
  __syncthreads();
  if (wbt) {   // forward copy of the tile: 8 consecutive ci per thread, 16-byte stores
    for (int k = tid; k < 64 * 8; k += 256) {
      const int r = k >> 3, c8 = (k & 7) * 8;
      const int co = co0 + r, ci = ci0 + c8;
      if (co < Cn && ci < Cr) {
        float f[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = tile[r][c8 + j];
        *reinterpret_cast<uint4*>(wbt + ((g * Cn + co) * T + tap) * Cr + ci) = pack8(f);
      }
    }
  }
  if (Cn % 8 == 0) {   // transposed copy: 8 consecutive co per thread, 16-byte stores
    for (int k = tid; k < 64 * 8; k += 256) {
      const int r = k >> 3, c8 = (k & 7) * 8;       // r: ci, c8: first co (contiguous in wt)
      const int ci = ci0 + r, co = co0 + c8;
      if (ci < Cr && co < Cn) {
        float f[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = tile[c8 + j][r];
        *reinterpret_cast<uint4*>(wt + ((g * Cr + ci) * T + tap) * Cn + co) = pack8(f);
      }
    }
    return;
  }
  for (int k = tid; k < 64 * 64; k += 256) {
    const int r = k >> 6, c = k & 63;               // r: ci, c: co (contiguous in wt)
    const int ci = ci0 + r, co = co0 + c;
    if (ci < Cr && co < Cn) wt[((g * Cr + ci) * T + tap) * Cn + co] = f2bf(tile[c][r]);
  }
}

__global__ __launch_bounds__(256) void weight_prep_multi_kernel(const int64_t* __restrict__ desc,
                                                                const int64_t* __restrict__ chunks) {
  __shared__ float tile[64][65];
  prep_chunk<false>(desc, chunks + (size_t)blockIdx.x * 4, SgdUpd{}, tile);
}

// One launch for the whole optimizer step: blocks [0, nsgd) run the plain SGD chunks (every
// arena range that no conv operand is built from), the rest the fused update + prep chunks.
__global__ __launch_bounds__(256) void sgd_prep_kernel(SgdArgs a, int nsgd,
                                                       const int64_t* __restrict__ desc,
                                                       const int64_t* __restrict__ chunks,
                                                       SgdUpd u) {
  __shared__ float tile[64][65];
  if ((int)blockIdx.x < nsgd) {
    sgd_chunk(a, blockIdx.x);
    return;
  }
  prep_chunk<true>(desc, chunks + (size_t)(blockIdx.x - nsgd) * 4, u, tile);
}

// ================================================================================ host
void weight_prep_multi_launch(const int64_t* desc, const int64_t* chunks, int nchunks,
                              hipStream_t st) {
  if (nchunks > 0)
    hipLaunchKernelGGL(weight_prep_multi_kernel, dim3(nchunks), dim3(256), 0, st, desc, chunks);
}
void nchw_to_nhwc_launch(const float* x, int N, int C, int HW, int Cp, bf16* y, hipStream_t st) {
  hipLaunchKernelGGL(nchw_to_nhwc_kernel, dim3(grid_cap((size_t)N * HW * Cp)), dim3(256), 0, st, x,
                     N, C, HW, Cp, y);
}
void nhwc_to_nchw_launch(const bf16* y, int N, int C, int HW, int Cp, float* x, hipStream_t st) {
  hipLaunchKernelGGL(nhwc_to_nchw_kernel, dim3(grid_cap((size_t)N * HW * C)), dim3(256), 0, st, y,
                     N, C, HW, Cp, x);
}
void augment_launch(const uint8_t* data, const int64_t* idx, const int32_t* rnd, int B, int H,
                    int W, int pad, const float* mean, const float* std, bf16* out,
                    const int64_t* labels, int64_t* targets, hipStream_t st) {
  hipLaunchKernelGGL(augment_kernel, dim3(grid_cap((size_t)B * H * W)), dim3(256), 0, st, data, idx,
                     rnd, B, H, W, pad, mean[0], mean[1], mean[2], 1.f / std[0], 1.f / std[1],
                     1.f / std[2], out, labels, targets);
}
static bool vec8_ok(int C) { return C % 8 == 0 && C <= 2048; }

// ------------------------------------------------------------------------- dropout (Philox)
// Counter-based RNG: Philox4x32-10 (Salmon et al., SC'11) keyed by a 64-bit seed, counter =
// (element/unit index lo, hi, step lo, step hi). `rng` is a device int64[3] {seed, step, tickets}:
// every block reads `step` first, then takes a ticket; the block drawing the last ticket advances
// `step` and resets the tickets (vector atomics), so each launch — eager or a hipGraph replay —
// draws fresh masks with no host involvement, and every block saw the same step.
__device__ __forceinline__ uint4 philox4x32_10(uint4 c, uint2 k) {
  constexpr uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t hi0 = __umulhi(M0, c.x), lo0 = M0 * c.x;
    const uint32_t hi1 = __umulhi(M1, c.z), lo1 = M1 * c.z;
    c = make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
    k.x += W0;
    k.y += W1;
  }
  return c;
}

// keep decision of unit u at `step` (probability 1 - p)
__device__ __forceinline__ bool drop_keep(uint64_t seed, uint64_t step, uint64_t u, float p) {
  const uint4 r = philox4x32_10(make_uint4((uint32_t)u, (uint32_t)(u >> 32), (uint32_t)step,
                                           (uint32_t)(step >> 32)),
                                make_uint2((uint32_t)seed, (uint32_t)(seed >> 32)));
  return (float)(r.x >> 8) * (1.f / 16777216.f) >= p;
}

// last block of the launch advances the step (see above); call after the block's last read of
// rng[1], from every thread (contains a barrier)
__device__ __forceinline__ void drop_advance(int64_t* rng) {
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    unsigned long long* r = reinterpret_cast<unsigned long long*>(rng);
    const unsigned long long t = atomicAdd(r + 2, 1ull);
    if (t == (unsigned long long)gridDim.x - 1) {
      atomicAdd(r + 1, 1ull);
      atomicExch(r + 2, 0ull);
    }
  }
}

// y = x * keep(unit(i)) / (1 - p); unit(i) = i / unit_len (1: dropout, C*H*W: drop-connect);
// mask[unit] = keep (written by the thread that owns the unit's first element)
template <typename T>
__global__ __launch_bounds__(256) void dropout_fwd_kernel(const T* __restrict__ x, size_t n,
                                                          int64_t unit_len, float p,
                                                          int64_t* __restrict__ rng,
                                                          uint8_t* __restrict__ mask,
                                                          T* __restrict__ y) {
  const uint64_t seed = (uint64_t)rng[0], step = (uint64_t)rng[1];
  const float scale = 1.f / (1.f - p);
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    const uint64_t u = i / (uint64_t)unit_len;
    const bool keep = drop_keep(seed, step, u, p);
    if (i % (uint64_t)unit_len == 0) mask[u] = keep;
    y[i] = (T)(keep ? (float)x[i] * scale : 0.f);
  }
  drop_advance(rng);
}

template <typename T>
__global__ __launch_bounds__(256) void dropout_bwd_kernel(const T* __restrict__ dy, size_t n,
                                                          int64_t unit_len, float p,
                                                          const uint8_t* __restrict__ mask,
                                                          T* __restrict__ dx) {
  const float scale = 1.f / (1.f - p);
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    dx[i] = (T)(mask[i / (uint64_t)unit_len] ? (float)dy[i] * scale : 0.f);
}

void dropout_fwd_launch(const void* x, bool bf, size_t n, int64_t unit_len, float p, int64_t* rng,
                        uint8_t* mask, void* y, hipStream_t st) {
  const dim3 grid(std::min<size_t>(cdiv64((int64_t)n, 256), 2048)), block(256);
  if (bf)
    hipLaunchKernelGGL(dropout_fwd_kernel<bf16>, grid, block, 0, st, (const bf16*)x, n, unit_len,
                       p, rng, mask, (bf16*)y);
  else
    hipLaunchKernelGGL(dropout_fwd_kernel<float>, grid, block, 0, st, (const float*)x, n, unit_len,
                       p, rng, mask, (float*)y);
}

void dropout_bwd_launch(const void* dy, bool bf, size_t n, int64_t unit_len, float p,
                        const uint8_t* mask, void* dx, hipStream_t st) {
  const dim3 grid(std::min<size_t>(cdiv64((int64_t)n, 256), 2048)), block(256);
  if (bf)
    hipLaunchKernelGGL(dropout_bwd_kernel<bf16>, grid, block, 0, st, (const bf16*)dy, n, unit_len,
                       p, mask, (bf16*)dx);
  else
    hipLaunchKernelGGL(dropout_bwd_kernel<float>, grid, block, 0, st, (const float*)dy, n, unit_len,
                       p, mask, (float*)dx);
}

// ------------------------------------------------------------------- classifier head
// Global average pool + Linear, fused (every zoo head: resnet.py:127-130 avg_pool2d(4) -> view ->
// linear, mobilenetv2.py:74, efficientnet.py:145 ...). The reference runs a pooling kernel, a
// cuBLAS addmm and, in backward, two GEMMs, a bias reduction, two AccumulateGrad adds and the
// pooling backward; here the forward is one kernel and the backward one kernel.
//   forward : block n pools x[n] (8-channel vectors, HW rows split over row lanes, LDS fold) and
//             computes logits[n][k] = pooled . W[k] + b[k] (one wave per k, wave reduction);
//             pooled is kept for dW.
//   backward: blocks 0..N-1 write dx[n][hw][c] = sum_k dl[n][k] W[k][c] / HW; the other blocks
//             each own 64 weight columns x 64 samples and add their share of
//             dW[k][c] += sum_n dl[n][k] pooled[n][c] with fp32 atomics (deterministic mode uses the
//             unfused path); the first of them also adds db[k] += sum_n dl[n][k].
// Loops over the K classes are unrolled to kHeadMaxK with clamped (always issued) loads and a
// zero multiplier past K: a load guarded by k < K would make the compiler branch around it and
// wait for each one in turn (the first version spent 15-27 us on these latency chains).
constexpr int kHeadMaxK = 16;
constexpr int kHeadSamples = 64;   // samples per weight-gradient block

__global__ __launch_bounds__(256) void head_fwd_kernel(const bf16* __restrict__ x, int HW, int C,
                                                       const float* __restrict__ w,
                                                       const float* __restrict__ b, int K,
                                                       float* __restrict__ pooled,
                                                       float* __restrict__ logits, float p,
                                                       int64_t* __restrict__ rng,
                                                       uint8_t* __restrict__ dmask) {
  // p > 0: training-mode dropout on the pooled features before the Linear (efficientnet.py:147-
  // 149): pooled holds the dropped, 1/(1-p)-scaled features (the weight gradient's operand) and
  // dmask the keep bytes (the input gradient's)
  extern __shared__ float hs[];                  // [RL][C] row-lane partials; [4][K] wave sums
  const int n = blockIdx.x, tid = threadIdx.x;
  const int CG = C >> 3;
  const int RL = CG >= 256 ? 1 : 256 / CG;       // row lanes
  const bf16* xn = x + (size_t)n * HW * C;
  for (int g0 = 0; g0 < CG; g0 += 256) {
    const int g = g0 + tid % (CG >= 256 ? 256 : CG), rl = CG >= 256 ? 0 : tid / CG;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (rl < RL && g < CG) {
#pragma unroll 4
      for (int hw = rl; hw < HW; hw += RL) {
        float f[8];
        unpack8(*reinterpret_cast<const uint4*>(xn + (size_t)hw * C + g * 8), f);
#pragma unroll
        for (int v = 0; v < 8; ++v) acc[v] += f[v];
      }
#pragma unroll
      for (int v = 0; v < 8; ++v) hs[rl * C + g * 8 + v] = acc[v];
    }
  }
  __syncthreads();
  // every thread: pooled channels c = tid, tid + 256, ... and the partial dot products of all K
  // classes over them (K independent weight loads per channel), then one block reduction per k
  const float inv = 1.f / HW;
  const bool drop = p > 0.f;
  const uint64_t seed = drop ? (uint64_t)rng[0] : 0, step = drop ? (uint64_t)rng[1] : 0;
  const float dscale = drop ? 1.f / (1.f - p) : 1.f;
  float part[kHeadMaxK];
#pragma unroll
  for (int k = 0; k < kHeadMaxK; ++k) part[k] = 0.f;
  for (int c = tid; c < C; c += 256) {
    float t = 0.f;
    for (int r = 0; r < RL; ++r) t += hs[r * C + c];
    t *= inv;
    if (drop) {
      const bool keep = drop_keep(seed, step, (uint64_t)n * C + c, p);
      dmask[(size_t)n * C + c] = keep;
      t = keep ? t * dscale : 0.f;
    }
    pooled[(size_t)n * C + c] = t;
#pragma unroll
    for (int k = 0; k < kHeadMaxK; ++k) {
      const float wk = w[(size_t)min(k, K - 1) * C + c];
      part[k] += (k < K ? t : 0.f) * wk;
    }
  }
  __syncthreads();                               // hs is reused for the wave sums below
  const int lane = tid & 63, wv = tid >> 6;
#pragma unroll
  for (int k = 0; k < kHeadMaxK; ++k) {
    const float t = wave_sum(part[k]);
    if (lane == 0) hs[wv * kHeadMaxK + k] = t;
  }
  __syncthreads();
  if (tid < K) {
    const float t = hs[tid] + hs[kHeadMaxK + tid] + hs[2 * kHeadMaxK + tid] + hs[3 * kHeadMaxK + tid];
    logits[(size_t)n * K + tid] = t + (b ? b[tid] : 0.f);
  }
  if (drop) drop_advance(rng);
}

// Optional fused backward reduce of the BatchNorm(+ReLU) that produced the pooled features
// (ResNet / PreAct block tails): the per-sample blocks also add sum dz and sum dz * xhat of
// dz = dX * relu'(mask) into that BN's sharded accumulator (one launch fewer for its reduce and
// one for its finalize). Needs 256 % (C / 8) == 0 (a thread's channel group is fixed).
struct HeadBnFuse {
  const bf16* y;
  const uint8_t* mask;
  const float* aux;   // [mean | istd | ...][C]
  float* acc;         // [R][2][C]
  int R;
  int spb;            // samples per block of the fused path: (N / spb) / R same-address atomics
};

__global__ __launch_bounds__(256) void head_bwd_kernel(const float* __restrict__ dl,
                                                       const float* __restrict__ w,
                                                       const float* __restrict__ pooled, int N,
                                                       int HW, int C, int K,
                                                       bf16* __restrict__ dx,
                                                       float* __restrict__ dw,
                                                       float* __restrict__ db, float p,
                                                       const uint8_t* __restrict__ dmask,
                                                       HeadBnFuse bf) {
  extern __shared__ float hs[];
  const int tid = threadIdx.x;
  // sample blocks: one sample each, or bf.spb samples each in the fused-BN form (their sums are
  // accumulated in registers and added once per block: at bs1024 one block per sample put 256
  // same-address atomics on every accumulator shard)
  const int spb = bf.acc ? bf.spb : 1;
  const int NB = (N + spb - 1) / spb;
  if ((int)blockIdx.x < NB) {
    // (dropout: the pooled-feature gradient passes kept features scaled by 1/(1-p))
    const float inv = 1.f / HW * (dmask ? 1.f / (1.f - p) : 1.f);
    const int CG = C >> 3;
    // fused BN-backward sums: this thread's channel group g = tid % CG is fixed (256 % CG == 0)
    const int g = tid % CG;
    float mean[8], istd[8], s1[8], s2[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      mean[q] = bf.acc ? bf.aux[g * 8 + q] : 0.f;
      istd[q] = bf.acc ? bf.aux[C + g * 8 + q] : 0.f;
      s1[q] = s2[q] = 0.f;
    }
    const int nb0 = blockIdx.x * spb, nb1 = min(N, nb0 + spb);
    for (int n = nb0; n < nb1; ++n) {
      float d[kHeadMaxK];
#pragma unroll
      for (int k = 0; k < kHeadMaxK; ++k) {
        const float v = dl[(size_t)n * K + min(k, K - 1)];
        d[k] = k < K ? v * inv : 0.f;
      }
      for (int c = tid; c < C; c += 256) {
        float t = 0.f;
#pragma unroll
        for (int k = 0; k < kHeadMaxK; ++k) t += d[k] * w[(size_t)min(k, K - 1) * C + c];
        hs[c] = (dmask && !dmask[(size_t)n * C + c]) ? 0.f : t;
      }
      __syncthreads();
      bf16* dxn = dx + (size_t)n * HW * C;
      if (!bf.acc) {
        for (int i = tid; i < HW * CG; i += 256) {
          const int gi = i % CG;
          *reinterpret_cast<uint4*>(dxn + (size_t)i * 8) = pack8(hs + gi * 8);
        }
        return;
      }
      const uint4 v = pack8(hs + g * 8);   // every pixel of the sample carries the same dX row
      float f[8];
      unpack8(v, f);
      const size_t base = (size_t)n * HW * C;
      for (int i = tid; i < HW * CG; i += 256) {
        const size_t o = base + (size_t)i * 8;
        *reinterpret_cast<uint4*>(dx + o) = v;
        float yy[8];
        unpack8(*reinterpret_cast<const uint4*>(bf.y + o), yy);
        const uint8_t m = bf.mask[o >> 3];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const float dz = ((m >> q) & 1u) ? f[q] : 0.f;
          s1[q] += dz;
          s2[q] += dz * (yy[q] - mean[q]) * istd[q];
        }
      }
      __syncthreads();                   // hs (this sample's dX row) is no longer read
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      hs[tid * 16 + q] = s1[q];
      hs[tid * 16 + 8 + q] = s2[q];
    }
    __syncthreads();
    if (tid < CG) {
      float a[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) a[q] = 0.f;
      for (int j = tid; j < 256; j += CG)
#pragma unroll
        for (int q = 0; q < 16; ++q) a[q] += hs[j * 16 + q];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        stat_out(bf.acc, blockIdx.x, bf.R, 2 * C, tid * 8 + q, a[q]);
        stat_out(bf.acc, blockIdx.x, bf.R, 2 * C, C + tid * 8 + q, a[8 + q]);
      }
    }
    return;
  }
  // weight / bias gradient: block (j, q) = 64 columns x kHeadSamples samples, 4 sample lanes
  const int jq = blockIdx.x - NB;
  const int ncb = cdiv(C, 64);
  const int j = jq % ncb, q = jq / ncb;
  const int cl = tid & 63, nl = tid >> 6;
  const int c = j * 64 + cl;
  const int n0 = q * kHeadSamples, n1 = min(N, n0 + kHeadSamples);
  float* red = hs;                                // [kHeadMaxK][4][64]
  float acc[kHeadMaxK];
#pragma unroll
  for (int k = 0; k < kHeadMaxK; ++k) acc[k] = 0.f;
  if (c < C) {
#pragma unroll 4
    for (int n = n0 + nl; n < n1; n += 4) {
      const float p = pooled[(size_t)n * C + c];
#pragma unroll
      for (int k = 0; k < kHeadMaxK; ++k) acc[k] += dl[(size_t)n * K + min(k, K - 1)] * p;
    }
  }
#pragma unroll
  for (int k = 0; k < kHeadMaxK; ++k) red[(k * 4 + nl) * 64 + cl] = acc[k];
  __syncthreads();
  if (nl == 0 && c < C) {
    for (int k = 0; k < K; ++k) {
      const float t = red[(k * 4 + 0) * 64 + cl] + red[(k * 4 + 1) * 64 + cl] +
                      red[(k * 4 + 2) * 64 + cl] + red[(k * 4 + 3) * 64 + cl];
      atomicAdd(dw + (size_t)k * C + c, t);
    }
  }
  if (jq == 0 && db && nl == 1) {       // one wave: db[k] += sum_n dl[n][k]
    // all classes per sample at once (clamped loads, zero weight past K) and independent wave
    // reductions: a per-class loop of load chains + reductions was the kernel's critical path
    float t[kHeadMaxK];
#pragma unroll
    for (int k = 0; k < kHeadMaxK; ++k) t[k] = 0.f;
#pragma unroll 2
    for (int n = cl; n < N; n += 64)
#pragma unroll
      for (int k = 0; k < kHeadMaxK; ++k) t[k] += dl[(size_t)n * K + min(k, K - 1)];
#pragma unroll
    for (int k = 0; k < kHeadMaxK; ++k) t[k] = wave_sum(t[k]);
    if (cl == 0)
      for (int k = 0; k < K; ++k) db[k] += t[k];
  }
}

bool head_supported(int C, int K) { return C % 8 == 0 && C <= 4096 && K >= 1 && K <= kHeadMaxK; }
bool head_batch_supported(int N, int K) { return N >= 1 && K >= 1; }

void head_fwd_launch(const bf16* x, int N, int HW, int C, const float* w, const float* b, int K,
                     float* pooled, float* logits, float p, int64_t* rng, uint8_t* dmask,
                     hipStream_t st) {
  const int CG = C >> 3;
  const int RL = CG >= 256 ? 1 : 256 / CG;
  const size_t lds = std::max<size_t>((size_t)RL * C, 4 * kHeadMaxK) * sizeof(float);
  hipLaunchKernelGGL(head_fwd_kernel, dim3(N), dim3(256), lds, st, x, HW, C, w, b, K, pooled,
                     logits, p, rng, dmask);
}

void head_bwd_launch(const float* dl, const float* w, const float* pooled, int N, int HW, int C,
                     int K, bf16* dx, float* dw, float* db, float p, const uint8_t* dmask,
                     hipStream_t st, const bf16* bn_y, const uint8_t* bn_mask, const float* bn_aux,
                     float* bn_acc, int bn_R) {
  // fused BN sums: at most 64 sample blocks per accumulator shard row
  const int spb = bn_acc ? std::max(1, cdiv(N, 64 * std::max(1, bn_R))) : 1;
  HeadBnFuse bf{bn_y, bn_mask, bn_aux, bn_acc, bn_R, spb};
  size_t lds = std::max<size_t>((size_t)C, (size_t)kHeadMaxK * 4 * 64) * sizeof(float);
  if (bn_acc) lds = std::max<size_t>(lds, 256 * 16 * sizeof(float));
  const int wblocks = cdiv(C, 64) * cdiv(N, kHeadSamples);
  hipLaunchKernelGGL(head_bwd_kernel, dim3(cdiv(N, spb) + wblocks), dim3(256), lds, st, dl, w,
                     pooled, N, HW, C, K, dx, dw, db, p, dmask, bf);
}

void gap_fwd_launch(const bf16* x, int N, int HW, int C, float* y, hipStream_t st) {
  if (vec8_ok(C)) {
    hipLaunchKernelGGL(gap_fwd8_kernel, dim3(N), dim3(256), 0, st, x, HW, C, y);
    return;
  }
  hipLaunchKernelGGL(gap_fwd_kernel, dim3(cdiv(C, 64), N), dim3(64), 0, st, x, HW, C, y);
}
void gap_bwd_launch(const float* dy, int N, int HW, int C, bf16* dx, hipStream_t st) {
  if (vec8_ok(C)) {
    hipLaunchKernelGGL(gap_bwd8_kernel, dim3(grid_cap((size_t)N * HW * C / 8)), dim3(256), 0, st,
                       dy, N, HW, C, dx);
    return;
  }
  hipLaunchKernelGGL(gap_bwd_kernel, dim3(grid_cap((size_t)N * HW * C)), dim3(256), 0, st, dy, N, HW,
                     C, dx);
}
static PoolGeom pg(int N, int H, int W, int C, int Ho, int Wo, int k, int s, int p) {
  PoolGeom g{N, H, W, C, Ho, Wo, k, s, p};
  return g;
}
// pool.hip fast paths (PCA_POOL_FAST=0: the generic kernels below for every geometry)
bool avgpool_ks_launch(bool bwd, const bf16* in, int N, int H, int W, int C, int k, int s, int p,
                       bf16* out, hipStream_t st);
void maxpool3s1_fwd_launch(const bf16* x, int N, int H, int W, int C, bf16* y, uint8_t* arg,
                           hipStream_t st);
void maxpool3s1_bwd_launch(const bf16* dy, const uint8_t* arg, int N, int H, int W, int C, bf16* dx,
                           hipStream_t st);
static bool pool_fast() {
  static const bool on = [] {
    const char* e = getenv("PCA_POOL_FAST");
    return !(e && e[0] == '0');
  }();
  return on;
}
static bool maxpool3s1_ok(int N, int H, int W, int C, int k, int s, int p) {
  return pool_fast() && k == 3 && s == 1 && p == 1 && C % 8 == 0 &&
         (size_t)N * H * W * C < (size_t)INT32_MAX;
}

void avgpool_fwd_launch(const bf16* x, int N, int H, int W, int C, int Ho, int Wo, int k, int s,
                        int p, bf16* y, hipStream_t st) {
  if (pool_fast() && avgpool_ks_launch(false, x, N, H, W, C, k, s, p, y, st)) return;
  hipLaunchKernelGGL(avgpool_fwd_kernel, dim3(grid_cap((size_t)N * Ho * Wo * C)), dim3(256), 0, st,
                     x, pg(N, H, W, C, Ho, Wo, k, s, p), y);
}
void avgpool_bwd_launch(const bf16* dy, int N, int H, int W, int C, int Ho, int Wo, int k, int s,
                        int p, bf16* dx, hipStream_t st) {
  if (pool_fast() && avgpool_ks_launch(true, dy, N, H, W, C, k, s, p, dx, st)) return;
  hipLaunchKernelGGL(avgpool_bwd_kernel, dim3(grid_cap((size_t)N * H * W * C)), dim3(256), 0, st, dy,
                     pg(N, H, W, C, Ho, Wo, k, s, p), dx);
}
static bool pool8_ok(int N, int H, int W, int C) {
  return C % 8 == 0 && (size_t)N * H * W * (C / 8) < (size_t)INT32_MAX;
}
void maxpool_fwd_launch(const bf16* x, int N, int H, int W, int C, int Ho, int Wo, int k, int s,
                        int p, bf16* y, uint8_t* arg, hipStream_t st) {
  if (maxpool3s1_ok(N, H, W, C, k, s, p)) {
    maxpool3s1_fwd_launch(x, N, H, W, C, y, arg, st);
    return;
  }
  if (k * k <= 256 && pool8_ok(N, H, W, C) && pool8_ok(N, Ho, Wo, C)) {
    hipLaunchKernelGGL(maxpool_fwd8_kernel, dim3(grid_cap((size_t)N * Ho * Wo * C / 8)), dim3(256), 0,
                       st, x, pg(N, H, W, C, Ho, Wo, k, s, p), y, arg);
    return;
  }
  hipLaunchKernelGGL(maxpool_fwd_kernel, dim3(grid_cap((size_t)N * Ho * Wo * C)), dim3(256), 0, st,
                     x, pg(N, H, W, C, Ho, Wo, k, s, p), y, arg);
}
void maxpool_bwd_launch(const bf16* dy, const uint8_t* arg, int N, int H, int W, int C, int Ho,
                        int Wo, int k, int s, int p, bf16* dx, hipStream_t st) {
  if (maxpool3s1_ok(N, H, W, C, k, s, p)) {
    maxpool3s1_bwd_launch(dy, arg, N, H, W, C, dx, st);
    return;
  }
  if (k * k <= 256 && pool8_ok(N, H, W, C) && pool8_ok(N, Ho, Wo, C)) {
    hipLaunchKernelGGL(maxpool_bwd8_kernel, dim3(grid_cap((size_t)N * H * W * C / 8)), dim3(256), 0,
                       st, dy, arg, pg(N, H, W, C, Ho, Wo, k, s, p), dx);
    return;
  }
  hipLaunchKernelGGL(maxpool_bwd_kernel, dim3(grid_cap((size_t)N * H * W * C)), dim3(256), 0, st, dy,
                     arg, pg(N, H, W, C, Ho, Wo, k, s, p), dx);
}
void ce_fused_launch(const float* logits, const int64_t* tgt, int N, int K, float* loss,
                     float* dlogits, double* metrics, hipStream_t st) {
  const int threads = std::min(1024, std::max(64, (N + 63) / 64 * 64));
  hipLaunchKernelGGL(ce_fused_kernel, dim3(1), dim3(threads), 0, st, logits, tgt, N, K, loss, dlogits,
                     metrics);
}
void scale_by_scalar_launch(const float* g, const float* s, size_t n, float* out, hipStream_t st) {
  hipLaunchKernelGGL(scale_by_scalar_kernel, dim3(grid_cap(n)), dim3(256), 0, st, g, s, n, out);
}
void sgd_launch(const int64_t* chunks, int nchunks, float* const* params, const float* const* grads,
                float* const* bufs, bf16* const* shadows, const float* lr, float momentum,
                float dampening, float wd, float grad_scale, int nesterov, int first,
                hipStream_t st, int zero_grad) {
  SgdArgs a{chunks, params, grads, bufs, shadows, lr, momentum, dampening, wd, grad_scale,
            nesterov, first, zero_grad};
  hipLaunchKernelGGL(sgd_kernel, dim3(nchunks), dim3(256), 0, st, a);
}
void sgd_prep_launch(const int64_t* chunks, int nchunks, float* const* params,
                     const float* const* grads, float* const* bufs, const float* lr, float momentum,
                     float dampening, float wd, float grad_scale, int nesterov, int first,
                     const int64_t* desc, const int64_t* pchunks, int npchunks, const int64_t* gm,
                     hipStream_t st, int zero_grad) {
  SgdArgs a{chunks, params, grads, bufs, nullptr, lr, momentum, dampening, wd, grad_scale,
            nesterov, first, zero_grad};
  SgdUpd u{gm, lr, momentum, dampening, wd, grad_scale, nesterov, first, zero_grad};
  if (nchunks + npchunks > 0)
    hipLaunchKernelGGL(sgd_prep_kernel, dim3(nchunks + npchunks), dim3(256), 0, st, a, nchunks, desc,
                       pchunks, u);
}
void se_scale_fwd_launch(const bf16* x, const float* s, int N, int HW, int C, bf16* out,
                         hipStream_t st) {
  if (vec8_ok(C)) {
    hipLaunchKernelGGL(se_scale_fwd8_kernel, dim3(grid_cap((size_t)N * HW * C / 8)), dim3(256), 0,
                       st, x, s, N, HW, C, out);
    return;
  }
  hipLaunchKernelGGL(se_scale_fwd_kernel, dim3(grid_cap((size_t)N * HW * C)), dim3(256), 0, st, x, s,
                     N, HW, C, out);
}
void se_scale_bwd_launch(const bf16* dout, const bf16* x, const float* s, int N, int HW, int C,
                         bf16* dx, float* ds, hipStream_t st) {
  if (vec8_ok(C)) {
    hipLaunchKernelGGL(se_scale_bwd8_kernel<true>, dim3(N), dim3(256), 0, st, dout, x, s, HW, C, dx, ds);
    return;
  }
  hipLaunchKernelGGL(se_scale_bwd_kernel, dim3(cdiv(C, 64), N), dim3(256), 0, st, dout, x, s, N, HW,
                     C, dx, ds);
}
static size_t se_param_lds_bytes(int R) {
  return sizeof(float) * (2 * kSeWN * kSeWC + 2 * (size_t)kSeWN * R);
}
// (64 KB of static LDS per block for the parameter kernel; R <= 192 keeps its per-thread
// outputs within 64 registers and the column kernels' staged rows within 8 x 256 floats)
bool se_mlp_supported(int C, int R) {
  return C % 8 == 0 && C <= 2048 && R >= 1 && R <= 192 && se_param_lds_bytes(R) <= 65536;
}
static dim3 se_row_grid(int N, int R) { return dim3(cdiv(N, kSeNB) * cdiv(R, kSeRC)); }
static dim3 se_col_grid(int N, int C) { return dim3(cdiv(C, 256), cdiv(N, kSeNB)); }
// the parameter part of se_mlp_bwd_launch alone (dz from se_bwd_data_kernel)
void se_mlp_bwd_param_launch(const float* ds, const float* dz, const float* hpre,
                             const float* pooled, int N, int C, int R, int act, float* dw1,
                             float* db1, float* dw2, float* db2, hipStream_t st);
void se_mlp_fwd_launch(const float* pooled, int N, int C, int R, const float* w1, const float* b1,
                       const float* w2, const float* b2, int act, float* hpre, float* s,
                       hipStream_t st) {
  hipLaunchKernelGGL((se_rowdot_kernel<false, false>), se_row_grid(N, R), dim3(256), 0, st, pooled,
                     N, C, R, w1, b1, nullptr, act, hpre);
  hipLaunchKernelGGL((se_coldot_kernel<true, true>), se_col_grid(N, C), dim3(256), 0, st, hpre, N,
                     C, R, w2, b2, act, s);
}
void se_mlp_bwd_launch(const float* ds, const float* hpre, const float* pooled, int N, int C,
                       int R, const float* w1, const float* w2, int act, float* dz, float* dp,
                       float* dw1, float* db1, float* dw2, float* db2, hipStream_t st) {
  hipLaunchKernelGGL((se_rowdot_kernel<true, true>), se_row_grid(N, R), dim3(256), 0, st, ds, N, C,
                     R, w2, nullptr, hpre, act, dz);
  hipLaunchKernelGGL((se_coldot_kernel<false, false>), se_col_grid(N, C), dim3(256), 0, st, dz, N,
                     C, R, w1, nullptr, act, dp);
  se_mlp_bwd_param_launch(ds, dz, hpre, pooled, N, C, R, act, dw1, db1, dw2, db2, st);
}
void se_mlp_bwd_param_launch(const float* ds, const float* dz, const float* hpre,
                             const float* pooled, int N, int C, int R, int act, float* dw1,
                             float* db1, float* dw2, float* db2, hipStream_t st) {
  // ~2 blocks per CU: split the samples into chunks over the channel tiles
  const int ct = cdiv(C, kSeWC);
  const int nchunks = std::max(1, std::min(cdiv(N, kSeWN), 512 / ct));
  const int chunk = cdiv(cdiv(N, nchunks), kSeWN) * kSeWN;
  const size_t lds = se_param_lds_bytes(R);
  const dim3 grid(ct, cdiv(N, chunk));
  const int need = cdiv(2 * kSeWC * R, 256);
#define PCA_SE_PARAM(J)                                                                        \
  hipLaunchKernelGGL(se_mlp_bwd_param_kernel<J>, grid, dim3(256), lds, st, ds, dz, hpre, pooled, \
                     N, C, R, act, chunk, dw1, db1, dw2, db2)
  if (need <= 4) PCA_SE_PARAM(4);
  else if (need <= 8) PCA_SE_PARAM(8);
  else if (need <= 16) PCA_SE_PARAM(16);
  else if (need <= 32) PCA_SE_PARAM(32);
  else PCA_SE_PARAM(64);
#undef PCA_SE_PARAM
}
static int se_fused_nb(int N) { return N >= 1024 ? 4 : N >= 512 ? 2 : 1; }
static size_t se_fused_lds(int NB, int C, int R) {
  return ((size_t)NB * C + (size_t)NB * R + 256 * 8) * sizeof(float);
}
bool se_fused_supported(int C, int R) {
  return C % 8 == 0 && C <= kSeFusedMaxC && R >= 1 && R <= kSeFusedMaxR &&
         se_fused_lds(4, C, R) <= 64 * 1024;
}
void se_fwd_fused_launch(const bf16* x, int N, int HW, int C, int R, const float* w1,
                         const float* b1, const float* w2t, const float* b2, int act, float* pooled,
                         float* hpre, float* s, hipStream_t st) {
  const int NB = se_fused_nb(N);
  const dim3 grid(cdiv(N, NB)), block(256);
  const size_t lds = se_fused_lds(NB, C, R);
  if (NB == 4)
    hipLaunchKernelGGL(se_fwd_fused_kernel<4>, grid, block, lds, st, x, N, HW, C, R, w1, b1, w2t, b2, act, pooled, hpre, s);
  else if (NB == 2)
    hipLaunchKernelGGL(se_fwd_fused_kernel<2>, grid, block, lds, st, x, N, HW, C, R, w1, b1, w2t, b2, act, pooled, hpre, s);
  else
    hipLaunchKernelGGL(se_fwd_fused_kernel<1>, grid, block, lds, st, x, N, HW, C, R, w1, b1, w2t, b2, act, pooled, hpre, s);
}
void se_bwd_data_launch(const bf16* dout, const bf16* x, const float* s, int N, int HW, int C,
                        int R, const float* w1, const float* w2t, const float* hpre, int act,
                        float* ds, float* dz, float* dp, hipStream_t st) {
  const int NB = se_fused_nb(N);
  const dim3 grid(cdiv(N, NB)), block(256);
  const size_t lds = se_fused_lds(NB, C, R);
  if (NB == 4)
    hipLaunchKernelGGL(se_bwd_data_kernel<4>, grid, block, lds, st, dout, x, s, N, HW, C, R, w1, w2t, hpre, act, ds, dz, dp);
  else if (NB == 2)
    hipLaunchKernelGGL(se_bwd_data_kernel<2>, grid, block, lds, st, dout, x, s, N, HW, C, R, w1, w2t, hpre, act, ds, dz, dp);
  else
    hipLaunchKernelGGL(se_bwd_data_kernel<1>, grid, block, lds, st, dout, x, s, N, HW, C, R, w1, w2t, hpre, act, ds, dz, dp);
}

void se_ds_launch(const bf16* dout, const bf16* x, const float* s, int N, int HW, int C, float* ds,
                  hipStream_t st) {
  hipLaunchKernelGGL(se_scale_bwd8_kernel<false>, dim3(N), dim3(256), 0, st, dout, x, s, HW, C,
                     nullptr, ds);
}
void se_dx_launch(const bf16* dout, const float* s, const float* dp, int N, int HW, int C, bf16* dx,
                  hipStream_t st) {
  hipLaunchKernelGGL(se_dx8_kernel, dim3(grid_cap((size_t)N * HW * C / 8)), dim3(256), 0, st, dout,
                     s, dp, N, HW, C, dx);
}
void act_fwd_launch(const bf16* x, size_t n, int act, bf16* y, hipStream_t st) {
  hipLaunchKernelGGL(act_fwd_kernel, dim3(grid_cap(n)), dim3(256), 0, st, x, n, act, y);
}
void act_bwd_launch(const bf16* dy, const bf16* x, size_t n, int act, bf16* dx, hipStream_t st) {
  hipLaunchKernelGGL(act_bwd_kernel, dim3(grid_cap(n)), dim3(256), 0, st, dy, x, n, act, dx);
}
void add_act_launch(const bf16* a, const bf16* b, size_t n, int act, bf16* y, hipStream_t st) {
  hipLaunchKernelGGL(add_act_kernel, dim3(grid_cap(n / 8 + 1)), dim3(256), 0, st, a, b, n, act, y);
}
void weight_prep_launch(const float* w, int G, int Cn, int T, int Cr, bf16* wb, bf16* wt,
                        hipStream_t st) {
  hipLaunchKernelGGL(weight_prep_kernel, dim3(grid_cap((size_t)G * Cn * T * Cr)), dim3(256), 0, st, w,
                     G, Cn, T, Cr, wb, wt);
}

// ---- channel remap (K22): out[q][j] = in[src(q)][cmap[j]], 0 where a map entry is -1.
// src(q) = q, or rmap[q / K] * K + q % K with an outer row map (conv weights [Cout][KH*KW][Cg]:
// K = KH*KW). One kernel covers the per-group zero padding of odd-width grouped convs (input,
// weight, bias) and its inverse slice (output, BN statistics), ShuffleNet's channel shuffle
// (shufflenet.py:10-19), and every backward of those — the adjoint of an injective remap is the
// remap with the inverse maps. ACC adds into `out` (fp32 parameter gradients in the arena).
// The channel map is staged in LDS once per block; each thread writes V consecutive output
// channels with one vector store (the gathered reads hit the same input row, L1/L2-resident).
// CLR zeroes every input element it reads (an injective map reads each at most once): a
// persistent padded weight-gradient buffer is handed back clean for the next accumulation.
template <typename T, int V, bool ACC, bool CLR = false>
__global__ __launch_bounds__(256) void chan_remap_kernel(T* __restrict__ in, T* __restrict__ out,
                                                         const int* __restrict__ cmap,
                                                         const int* __restrict__ rmap, int Q, int K,
                                                         int Cin, int J, int map_in_lds) {
  extern __shared__ int smap[];
  const int* mp = cmap;
  if (map_in_lds) {
    for (int j = threadIdx.x; j < J; j += blockDim.x) smap[j] = cmap[j];
    __syncthreads();
    mp = smap;
  }
  struct alignas(sizeof(T) * V) Vec { T v[V]; };
  const int G = J / V;
  const int64_t total = (int64_t)Q * G;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int q = (int)(i / G), gi = (int)(i - (int64_t)q * G);
    int64_t srow = q;
    if (rmap) {
      const int r = q / K;
      const int s = rmap[r];
      srow = s < 0 ? -1 : (int64_t)s * K + (q - r * K);
    }
    T* row = in + srow * Cin;
    Vec o;
#pragma unroll
    for (int u = 0; u < V; ++u) {
      const int c = mp[gi * V + u];
      o.v[u] = (srow >= 0 && c >= 0) ? row[c] : T(0.f);
      if constexpr (CLR) {
        if (srow >= 0 && c >= 0) row[c] = T(0.f);
      }
    }
    Vec* dst = reinterpret_cast<Vec*>(out + (int64_t)q * J + gi * V);
    if constexpr (ACC) {
      Vec a = *dst;
#pragma unroll
      for (int u = 0; u < V; ++u) a.v[u] = a.v[u] + o.v[u];
      *dst = a;
    } else {
      *dst = o;
    }
  }
}

// Row-staged form for activations (no row map): a block loads RB whole input rows into LDS with
// 16-byte (or the widest dividing) loads, then writes RB output rows gathering from LDS — every
// global access coalesced and vectorized (the per-element gather above issues V scalar loads
// per output vector: slower than a stock pad on DPN / RegNet's padded groups).
// ACC (bf16 activations): out += the remapped rows, summed in fp32 (a gradient junction: the
// unpad of a zero-padded conv's dX adding the other consumer's gradient in the same pass)
template <typename T, int VIN, int V, bool ACC = false>
__global__ __launch_bounds__(256) void chan_remap_rows_kernel(const T* __restrict__ in,
                                                              T* __restrict__ out,
                                                              const int* __restrict__ cmap, int Q,
                                                              int Cin, int J, int RB) {
  extern __shared__ __attribute__((aligned(16))) char rsm[];
  int* smap = reinterpret_cast<int*>(rsm);
  T* rows = reinterpret_cast<T*>(rsm + ((J * (int)sizeof(int) + 15) & ~15));
  for (int j = threadIdx.x; j < J; j += blockDim.x) smap[j] = cmap[j];
  struct alignas(sizeof(T) * VIN) VecI { T v[VIN]; };
  struct alignas(sizeof(T) * V) VecO { T v[V]; };
  const int ci = Cin / VIN, jo = J / V;
  for (int r0 = blockIdx.x * RB; r0 < Q; r0 += gridDim.x * RB) {
    const int nr = min(RB, Q - r0);
    __syncthreads();   // (map staged / previous rows consumed)
    const VecI* src = reinterpret_cast<const VecI*>(in + (int64_t)r0 * Cin);
    VecI* dst = reinterpret_cast<VecI*>(rows);
    for (int i = threadIdx.x; i < nr * ci; i += blockDim.x) dst[i] = src[i];
    __syncthreads();
    VecO* o = reinterpret_cast<VecO*>(out + (int64_t)r0 * J);
    for (int i = threadIdx.x; i < nr * jo; i += blockDim.x) {
      const int r = i / jo, gi = i - r * jo;
      VecO v;
#pragma unroll
      for (int u = 0; u < V; ++u) {
        const int c = smap[gi * V + u];
        v.v[u] = c >= 0 ? rows[r * Cin + c] : T(0.f);
      }
      if constexpr (ACC) {
        const VecO a = o[i];
#pragma unroll
        for (int u = 0; u < V; ++u) v.v[u] = T((float)a.v[u] + (float)v.v[u]);
      }
      o[i] = v;
    }
  }
}

template <typename T, bool ACC = false>
static bool chan_remap_rows(const T* in, T* out, const int* cmap, int Q, int Cin, int J,
                            hipStream_t st) {
  constexpr int VMAX = 16 / sizeof(T);
  int vin = VMAX, v = VMAX;
  while (vin > 1 && (Cin % vin)) vin >>= 1;
  while (v > 1 && (J % v)) v >>= 1;
  const size_t map_bytes = ((size_t)J * sizeof(int) + 15) & ~(size_t)15;
  const size_t row_bytes = (size_t)Cin * sizeof(T);
  if (map_bytes + row_bytes > 48 * 1024) return false;
  int RB = (int)((48 * 1024 - map_bytes) / row_bytes);
  RB = std::max(1, std::min(RB, 64));
  const size_t lds = map_bytes + (size_t)RB * row_bytes;
  const int blocks = (int)std::min<int64_t>(cdiv64(Q, RB), 4096);
#define PCA_RR(VI, VO)                                                                       \
  if (vin == VI && v == VO) {                                                                \
    hipLaunchKernelGGL((chan_remap_rows_kernel<T, VI, VO, ACC>), dim3(blocks), dim3(256), lds, st, \
                       in, out, cmap, Q, Cin, J, RB);                                        \
    return true;                                                                             \
  }
  if constexpr (VMAX == 8) {
    PCA_RR(8, 8) PCA_RR(8, 4) PCA_RR(8, 2) PCA_RR(8, 1) PCA_RR(4, 8) PCA_RR(2, 8) PCA_RR(1, 8)
  }
  PCA_RR(4, 4) PCA_RR(4, 2) PCA_RR(4, 1) PCA_RR(2, 4) PCA_RR(2, 2) PCA_RR(2, 1) PCA_RR(1, 4)
  PCA_RR(1, 2) PCA_RR(1, 1)
#undef PCA_RR
  return false;
}

template <typename T, bool ACC, bool CLR = false>
static void chan_remap_dispatch(T* in, T* out, const int* cmap, const int* rmap, int Q, int K,
                                int Cin, int J, hipStream_t st) {
  if constexpr (!ACC && !CLR) {
    if (!rmap && chan_remap_rows<T>(in, out, cmap, Q, Cin, J, st)) return;
  }
  if constexpr (ACC && !CLR && sizeof(T) == 2) {
    if (!rmap && chan_remap_rows<T, true>(in, out, cmap, Q, Cin, J, st)) return;
  }
  constexpr int VMAX = 16 / sizeof(T);
  int V = VMAX;
  while (V > 1 && (J % V)) V >>= 1;
  const int lds_ok = J <= 16384 ? 1 : 0;
  const size_t lds = lds_ok ? (size_t)J * sizeof(int) : 0;
  const dim3 grid(grid_cap((size_t)Q * (J / V))), block(256);
#define PCA_REMAP(VV)                                                                           \
  if (V == VV) {                                                                                \
    hipLaunchKernelGGL((chan_remap_kernel<T, VV, ACC, CLR>), grid, block, lds, st, in, out, cmap, rmap, \
                       Q, K, Cin, J, lds_ok);                                                   \
    return;                                                                                     \
  }
  if constexpr (VMAX >= 8) { PCA_REMAP(8) }
  PCA_REMAP(4) PCA_REMAP(2) PCA_REMAP(1)
#undef PCA_REMAP
}

void chan_remap_launch(const void* in, void* out, bool fp32, bool accumulate, const int* cmap,
                       const int* rmap, int Q, int K, int Cin, int J, hipStream_t st,
                       bool clear_src) {
  // (the kernels take a mutable source for the clearing form; the others only read it)
  if (fp32) {
    float* i = const_cast<float*>(static_cast<const float*>(in));
    if (accumulate && clear_src)
      chan_remap_dispatch<float, true, true>(i, (float*)out, cmap, rmap, Q, K, Cin, J, st);
    else if (accumulate)
      chan_remap_dispatch<float, true>(i, (float*)out, cmap, rmap, Q, K, Cin, J, st);
    else if (clear_src)
      chan_remap_dispatch<float, false, true>(i, (float*)out, cmap, rmap, Q, K, Cin, J, st);
    else
      chan_remap_dispatch<float, false>(i, (float*)out, cmap, rmap, Q, K, Cin, J, st);
  } else if (accumulate) {
    chan_remap_dispatch<bf16, true>(const_cast<bf16*>(static_cast<const bf16*>(in)), (bf16*)out,
                                    cmap, rmap, Q, K, Cin, J, st);
  } else {
    chan_remap_dispatch<bf16, false>(const_cast<bf16*>(static_cast<const bf16*>(in)), (bf16*)out,
                                     cmap, rmap, Q, K, Cin, J, st);
  }
}

}  // namespace pca
