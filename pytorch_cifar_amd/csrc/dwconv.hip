// Depthwise convolution (groups == Cin, channel multiplier m = Cout/Cin), NHWC bf16.
//
// Replaces the cuDNN depthwise kernels of the mobile zoo: mobilenet.py:15,
// mobilenetv2.py:20, efficientnet.py:70-76 (k3/k5), shufflenetv2.py:40/63/73, pnasnet.py:14-17
// (k3/k5/k7, multiplier 2 at stride 2). Bandwidth-bound: one thread owns 8 channels of one
// output pixel (16-byte vectors); the k*k taps are re-read from L1/L2.
//
// Weights arrive transposed as fp32 wT[tap][Cout] so the 8 channel weights of a tap are two
// float4 loads. wgrad is a deterministic per-(pixel-chunk, tap) slab reduction.
#include "common.h"

#include <algorithm>
#include <cstdlib>

namespace pca {

struct DwGeom {
  int N, H, W, C, Ho, Wo, Co, KH, KW, s, p, mult;
};

template <int VEC>
__global__ __launch_bounds__(256) void dw_fwd_kernel(const bf16* __restrict__ x,
                                                     const float* __restrict__ wT, DwGeom g,
                                                     bf16* __restrict__ y) {
  const int G = g.Co / VEC;
  const size_t total = (size_t)g.N * g.Ho * g.Wo * G;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    const int gi = (int)(i % G);
    size_t q = i / G;
    const int ow = (int)(q % g.Wo);
    q /= g.Wo;
    const int oh = (int)(q % g.Ho);
    const int n = (int)(q / g.Ho);
    const int co = gi * VEC;
    float acc[VEC];
#pragma unroll
    for (int v = 0; v < VEC; ++v) acc[v] = 0.f;
    for (int kh = 0; kh < g.KH; ++kh) {
      const int ih = oh * g.s - g.p + kh;
      if (ih < 0 || ih >= g.H) continue;
      for (int kw = 0; kw < g.KW; ++kw) {
        const int iw = ow * g.s - g.p + kw;
        if (iw < 0 || iw >= g.W) continue;
        const float* wr = wT + (size_t)(kh * g.KW + kw) * g.Co + co;
        const bf16* xr = x + (((size_t)n * g.H + ih) * g.W + iw) * g.C;
        if constexpr (VEC == 8) {
          float f[8];
          unpack8(*reinterpret_cast<const uint4*>(xr + co), f);
          const float4 w0 = *reinterpret_cast<const float4*>(wr);
          const float4 w1 = *reinterpret_cast<const float4*>(wr + 4);
          acc[0] += f[0] * w0.x; acc[1] += f[1] * w0.y; acc[2] += f[2] * w0.z; acc[3] += f[3] * w0.w;
          acc[4] += f[4] * w1.x; acc[5] += f[5] * w1.y; acc[6] += f[6] * w1.z; acc[7] += f[7] * w1.w;
        } else {
          acc[0] += bf2f(xr[co / g.mult]) * wr[0];
        }
      }
    }
    bf16* yr = y + (((size_t)n * g.Ho + oh) * g.Wo + ow) * g.Co + co;
    if constexpr (VEC == 8) {
      *reinterpret_cast<uint4*>(yr) = pack8(acc);
    } else {
      yr[0] = f2bf(acc[0]);
    }
  }
}

// dx[n,ih,iw,c] = sum_{j<mult} sum_taps dy[n,oh,ow,c*mult+j] * w[c*mult+j][tap]
template <int VEC>
__global__ __launch_bounds__(256) void dw_dgrad_kernel(const bf16* __restrict__ dy,
                                                       const float* __restrict__ wT, DwGeom g,
                                                       bf16* __restrict__ dx) {
  const int G = g.C / VEC;
  const size_t total = (size_t)g.N * g.H * g.W * G;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    const int gi = (int)(i % G);
    size_t q = i / G;
    const int iw = (int)(q % g.W);
    q /= g.W;
    const int ih = (int)(q % g.H);
    const int n = (int)(q / g.H);
    const int c = gi * VEC;
    float acc[VEC];
#pragma unroll
    for (int v = 0; v < VEC; ++v) acc[v] = 0.f;
    for (int kh = 0; kh < g.KH; ++kh) {
      const int t = ih + g.p - kh;
      if (t < 0) continue;
      const int oh = t / g.s;
      if (oh * g.s != t || oh >= g.Ho) continue;
      for (int kw = 0; kw < g.KW; ++kw) {
        const int u = iw + g.p - kw;
        if (u < 0) continue;
        const int ow = u / g.s;
        if (ow * g.s != u || ow >= g.Wo) continue;
        const float* wr = wT + (size_t)(kh * g.KW + kw) * g.Co;
        const bf16* dr = dy + (((size_t)n * g.Ho + oh) * g.Wo + ow) * g.Co;
        if constexpr (VEC == 8) {
          float f[8];
          unpack8(*reinterpret_cast<const uint4*>(dr + c), f);
          const float4 w0 = *reinterpret_cast<const float4*>(wr + c);
          const float4 w1 = *reinterpret_cast<const float4*>(wr + c + 4);
          acc[0] += f[0] * w0.x; acc[1] += f[1] * w0.y; acc[2] += f[2] * w0.z; acc[3] += f[3] * w0.w;
          acc[4] += f[4] * w1.x; acc[5] += f[5] * w1.y; acc[6] += f[6] * w1.z; acc[7] += f[7] * w1.w;
        } else {
          for (int j = 0; j < g.mult; ++j) {
            const int co = c * g.mult + j;
            acc[0] += bf2f(dr[co]) * wr[co];
          }
        }
      }
    }
    bf16* xr = dx + (((size_t)n * g.H + ih) * g.W + iw) * g.C + c;
    if constexpr (VEC == 8) {
      *reinterpret_cast<uint4*>(xr) = pack8(acc);
    } else {
      xr[0] = f2bf(acc[0]);
    }
  }
}

// partial[chunk][tap][Co] = sum over the chunk's output pixels of dy * x(shifted by tap)
template <int VEC>
__global__ __launch_bounds__(256) void dw_wgrad_kernel(const bf16* __restrict__ x,
                                                       const bf16* __restrict__ dy, DwGeom g,
                                                       int rows_per_block,
                                                       float* __restrict__ partial) {
  __shared__ float red[256 * VEC];
  const int tap = blockIdx.y;
  const int kh = tap / g.KW, kw = tap % g.KW;
  const int G = g.Co / VEC;
  const int TPR = G < 256 ? G : 256;
  const int RPP = 256 / TPR;
  const int t = threadIdx.x;
  const int gx = t % TPR, ry = t / TPR;
  const int P = g.N * g.Ho * g.Wo;
  const int r0 = blockIdx.x * rows_per_block, r1 = min(P, r0 + rows_per_block);
  for (int gbase = 0; gbase < G; gbase += TPR) {
    const int gi = gbase + gx;
    const int co = gi * VEC;
    float acc[VEC];
#pragma unroll
    for (int v = 0; v < VEC; ++v) acc[v] = 0.f;
    if (ry < RPP && gi < G) {
      for (int r = r0 + ry; r < r1; r += RPP) {
        const int ow = r % g.Wo;
        const int q = r / g.Wo;
        const int oh = q % g.Ho, n = q / g.Ho;
        const int ih = oh * g.s - g.p + kh, iw = ow * g.s - g.p + kw;
        if (ih < 0 || ih >= g.H || iw < 0 || iw >= g.W) continue;
        const bf16* xr = x + (((size_t)n * g.H + ih) * g.W + iw) * g.C;
        const bf16* dr = dy + (size_t)r * g.Co + co;
        if constexpr (VEC == 8) {
          float fx[8], fd[8];
          unpack8(*reinterpret_cast<const uint4*>(xr + co), fx);
          unpack8(*reinterpret_cast<const uint4*>(dr), fd);
#pragma unroll
          for (int v = 0; v < 8; ++v) acc[v] += fx[v] * fd[v];
        } else {
          acc[0] += bf2f(xr[co / g.mult]) * bf2f(dr[0]);
        }
      }
    }
#pragma unroll
    for (int v = 0; v < VEC; ++v) red[t * VEC + v] = acc[v];
    __syncthreads();
    if (ry == 0 && gi < G) {
      for (int k = 1; k < RPP; ++k)
#pragma unroll
        for (int v = 0; v < VEC; ++v) acc[v] += red[(k * TPR + gx) * VEC + v];
      float* prow = partial + ((size_t)blockIdx.x * g.KH * g.KW + tap) * g.Co + co;
#pragma unroll
      for (int v = 0; v < VEC; ++v) prow[v] = acc[v];
    }
    __syncthreads();
  }
}

// dw[co][tap] = sum_r partial[r][tap][co]
__global__ void dw_wgrad_final_kernel(const float* __restrict__ partial, int R, int T, int Co,
                                      float* __restrict__ dw) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= T * Co) return;
  const int co = i % Co, tap = i / Co;
  float s = 0.f;
  for (int r = 0; r < R; ++r) s += partial[((size_t)r * T + tap) * Co + co];
  dw[(size_t)co * T + tap] = s;
}

// ---------------------------------------------------------------------------------------
// k3 / k5 depthwise fast paths (multiplier 1, stride 1 or 2, "same" padding K/2) — the
// MobileNet / MobileNetV2 / ShuffleNetV2 / EfficientNet-B0 (k3 and k5, efficientnet.py:70-76)
// shapes. The generic kernels above re-load every weight and every tap from L1/L2 per output
// vector, with 64-bit index math per element, and the generic wgrad runs one block per tap
// (dY re-read K*K times): 2.5-15x off their bandwidth roofline (profiles/). Here a thread owns
// V channels of one output column strip (RPT rows):
//   * the K input rows of the KxK window roll down the strip as raw bf16 vectors, so each output
//     row loads K new vectors (stride 1) or 2K (stride 2) instead of K*K;
//   * fwd / stride-1 dgrad keep the K*K x V fp32 weights in registers (the stride-1 dgrad is the
//     same correlation with mirrored taps and pad K-1-p);
//   * wgrad accumulates all K*K taps x V channels in registers across every strip the thread
//     walks (dY read once), then the threads sharing a channel group are reduced through LDS,
//     one tap at a time, into one deterministic partial row per block.
// V = 8 (16-byte vectors) at K = 3; V = 4 (8-byte vectors) at K = 5 and V = 2 (4-byte) at K = 7,
// so that the K*K x V weights (or accumulators) plus the K*K-vector window stay in registers.
// ---------------------------------------------------------------------------------------
template <int V> struct DwVec;
template <> struct DwVec<8> { using T = uint4; };
template <> struct DwVec<4> { using T = uint2; };
template <> struct DwVec<2> { using T = uint32_t; };

template <int V>
__device__ __forceinline__ typename DwVec<V>::T dw_zero() {
  if constexpr (V == 8) return make_uint4(0u, 0u, 0u, 0u);
  else if constexpr (V == 4) return make_uint2(0u, 0u);
  else return 0u;
}

template <int V>
__device__ __forceinline__ void dw_unpack(const typename DwVec<V>::T& u, float* f) {
  if constexpr (V == 8) {
    unpack8(u, f);
  } else if constexpr (V == 2) {
    f[0] = __uint_as_float(u << 16);
    f[1] = __uint_as_float(u & 0xffff0000u);
  } else {
    f[0] = __uint_as_float(u.x << 16);
    f[1] = __uint_as_float(u.x & 0xffff0000u);
    f[2] = __uint_as_float(u.y << 16);
    f[3] = __uint_as_float(u.y & 0xffff0000u);
  }
}

template <int V>
__device__ __forceinline__ typename DwVec<V>::T dw_pack(const float* f) {
  if constexpr (V == 8) return pack8(f);
  else if constexpr (V == 4) return make_uint2(pack2(f[0], f[1]), pack2(f[2], f[3]));
  else return pack2(f[0], f[1]);
}

// Input transform (IN != 0): the kernel's input is the PRE-BatchNorm tensor y of the BN(+act)
// that feeds this depthwise conv, and every loaded vector becomes act(y * scale + shift) — the
// BN's output, rounded to bf16 exactly as its apply pass would store it — before it enters the
// window; zero padding stays zero. The BN's output tensor is never written or read again
// (mobilenetv2.py:31-35 conv1 -> bn1 -> relu -> conv2, efficientnet.py:96-98 with swish).
template <int V, int IN>
__device__ __forceinline__ typename DwVec<V>::T dw_in(const typename DwVec<V>::T& u,
                                                      const float* sc, const float* sh) {
  if constexpr (IN == 0) {
    return u;
  } else {
    float f[V];
    dw_unpack<V>(u, f);
#pragma unroll
    for (int v = 0; v < V; ++v) f[v] = apply_act(f[v] * sc[v] + sh[v], IN);
    return dw_pack<V>(f);
  }
}

// per-thread scale / shift of its V channels (IN != 0)
template <int V, int IN>
__device__ __forceinline__ void dw_in_coef(const float* isc, const float* ish, int c, float* sc,
                                           float* sh) {
#pragma unroll
  for (int v = 0; v < V; ++v) {
    sc[v] = IN ? isc[c + v] : 1.f;
    sh[v] = IN ? ish[c + v] : 0.f;
  }
}

// the K vectors (kw = 0..K-1) of input row ih starting at column iw0 (zeros outside the image)
template <int K, int V, int IN = 0>
__device__ __forceinline__ void dwk_load_row(const bf16* xn, const DwGeom& g, int ih, int iw0,
                                             typename DwVec<V>::T* r, const float* sc = nullptr,
                                             const float* sh = nullptr) {
  using T = typename DwVec<V>::T;
  const bool rok = (unsigned)ih < (unsigned)g.H;
#pragma unroll
  for (int kw = 0; kw < K; ++kw) {
    const int iw = iw0 + kw;
    r[kw] = (rok && (unsigned)iw < (unsigned)g.W)
                ? dw_in<V, IN>(*reinterpret_cast<const T*>(xn + ((size_t)ih * g.W + iw) * g.C), sc, sh)
                : dw_zero<V>();
  }
}

// advance the window by S input rows: rows S..K-1 move up, rows K-S..K-1 are reloaded
template <int K, int S, typename T>
__device__ __forceinline__ void dwk_roll(T (&win)[K][K]) {
#pragma unroll
  for (int k = 0; k + S < K; ++k)
#pragma unroll
    for (int kw = 0; kw < K; ++kw) win[k][kw] = win[k + S][kw];
}

template <int K, int S, int V, bool FLIP, int IN = 0>
__global__ __launch_bounds__(256) void dwk_fwd_kernel(const bf16* __restrict__ x,
                                                      const float* __restrict__ wT, DwGeom g,
                                                      int rpt, bf16* __restrict__ y,
                                                      const float* __restrict__ isc = nullptr,
                                                      const float* __restrict__ ish = nullptr) {
  using T = typename DwVec<V>::T;
  constexpr int KK = K * K;
  const int G = g.C / V;
  const int nstrip = (g.Ho + rpt - 1) / rpt;
  const int total = g.N * nstrip * g.Wo * G;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int gi = i % G;
    int q = i / G;
    const int ow = q % g.Wo;
    q /= g.Wo;
    const int strip = q % nstrip;
    const int n = q / nstrip;
    const int c = gi * V;
    float w[KK][V];
#pragma unroll
    for (int t = 0; t < KK; ++t) {
      const int src = FLIP ? KK - 1 - t : t;
      if constexpr (V == 2) {
        const float2 wv = *reinterpret_cast<const float2*>(wT + src * g.Co + c);
        w[t][0] = wv.x; w[t][1] = wv.y;
      } else {
#pragma unroll
        for (int v4 = 0; v4 < V; v4 += 4) {
          const float4 wv = *reinterpret_cast<const float4*>(wT + src * g.Co + c + v4);
          w[t][v4] = wv.x; w[t][v4 + 1] = wv.y; w[t][v4 + 2] = wv.z; w[t][v4 + 3] = wv.w;
        }
      }
    }
    const bf16* xn = x + (size_t)n * g.H * g.W * g.C + c;
    const int oh0 = strip * rpt, oh1 = min(g.Ho, oh0 + rpt);
    const int iw0 = ow * S - g.p;
    float isv[V], ihv[V];
    dw_in_coef<V, IN>(isc, ish, c, isv, ihv);
    T win[K][K];
#pragma unroll
    for (int k = 0; k < K - S; ++k)
      dwk_load_row<K, V, IN>(xn, g, oh0 * S - g.p + k, iw0, win[k], isv, ihv);
    bf16* yr = y + (((size_t)n * g.Ho + oh0) * g.Wo + ow) * g.Co + c;
    for (int oh = oh0; oh < oh1; ++oh) {
      const int ih0 = oh * S - g.p;
#pragma unroll
      for (int k = K - S; k < K; ++k) dwk_load_row<K, V, IN>(xn, g, ih0 + k, iw0, win[k], isv, ihv);
      float acc[V];
#pragma unroll
      for (int v = 0; v < V; ++v) acc[v] = 0.f;
#pragma unroll
      for (int kh = 0; kh < K; ++kh)
#pragma unroll
        for (int kw = 0; kw < K; ++kw) {
          float f[V];
          dw_unpack<V>(win[kh][kw], f);
#pragma unroll
          for (int v = 0; v < V; ++v) acc[v] += f[v] * w[kh * K + kw][v];
        }
      *reinterpret_cast<T*>(yr) = dw_pack<V>(acc);
      yr += (size_t)g.Wo * g.Co;
      dwk_roll<K, S>(win);
    }
  }
}

// partial[block.x][tap][Co]: block (x, y) owns channel groups [y*GB, y*GB + GB) (GB <= 256);
// thread t owns group y*GB + t % GB and walks the column strips item = x*W + t/GB (+ gridDim.x*W
// ...), W = 256 / GB workers per group
template <int K, int S, int V, int IN = 0>
__global__ __launch_bounds__(256) void dwk_wgrad_kernel(const bf16* __restrict__ x,
                                                        const bf16* __restrict__ dy, DwGeom g,
                                                        int rpt, int GB,
                                                        float* __restrict__ partial,
                                                        const float* __restrict__ isc = nullptr,
                                                        const float* __restrict__ ish = nullptr) {
  using T = typename DwVec<V>::T;
  constexpr int KK = K * K;
  __shared__ float red[256 * V];
  const int G = g.Co / V;
  const int gb0 = blockIdx.y * GB;
  const int Gl = min(GB, G - gb0);
  const int W = 256 / GB;
  const int t = threadIdx.x;
  const int gl = t % GB, wk = t / GB;
  const int c = (gb0 + gl) * V;
  const int nstrip = (g.Ho + rpt - 1) / rpt;
  const int items = g.N * nstrip * g.Wo;
  float acc[KK][V];
#pragma unroll
  for (int k = 0; k < KK; ++k)
#pragma unroll
    for (int v = 0; v < V; ++v) acc[k][v] = 0.f;
  if (wk < W && gl < Gl) {
    for (int item = blockIdx.x * W + wk; item < items; item += gridDim.x * W) {
      const int ow = item % g.Wo;
      const int q = item / g.Wo;
      const int strip = q % nstrip, n = q / nstrip;
      const bf16* xn = x + (size_t)n * g.H * g.W * g.C + c;
      const int oh0 = strip * rpt, oh1 = min(g.Ho, oh0 + rpt);
      const int iw0 = ow * S - g.p;
      float isv[V], ihv[V];
      dw_in_coef<V, IN>(isc, ish, c, isv, ihv);
      T win[K][K];
#pragma unroll
      for (int k = 0; k < K - S; ++k)
        dwk_load_row<K, V, IN>(xn, g, oh0 * S - g.p + k, iw0, win[k], isv, ihv);
      const bf16* dr = dy + (((size_t)n * g.Ho + oh0) * g.Wo + ow) * g.Co + c;
      for (int oh = oh0; oh < oh1; ++oh) {
        const int ih0 = oh * S - g.p;
#pragma unroll
        for (int k = K - S; k < K; ++k) dwk_load_row<K, V, IN>(xn, g, ih0 + k, iw0, win[k], isv, ihv);
        float d[V];
        dw_unpack<V>(*reinterpret_cast<const T*>(dr), d);
        dr += (size_t)g.Wo * g.Co;
#pragma unroll
        for (int kh = 0; kh < K; ++kh)
#pragma unroll
          for (int kw = 0; kw < K; ++kw) {
            float f[V];
            dw_unpack<V>(win[kh][kw], f);
#pragma unroll
            for (int v = 0; v < V; ++v) acc[kh * K + kw][v] += f[v] * d[v];
          }
        dwk_roll<K, S>(win);
      }
    }
  }
  float* prow = partial + (size_t)blockIdx.x * KK * g.Co;
#pragma unroll
  for (int k = 0; k < KK; ++k) {
#pragma unroll
    for (int v = 0; v < V; ++v) red[t * V + v] = acc[k][v];
    __syncthreads();
    if (t < Gl) {
      float s[V];
#pragma unroll
      for (int v = 0; v < V; ++v) s[v] = red[t * V + v];
      for (int j = 1; j < W; ++j)
#pragma unroll
        for (int v = 0; v < V; ++v) s[v] += red[(j * GB + t) * V + v];
      float* o = prow + (size_t)k * g.Co + (gb0 + t) * V;
      if constexpr (V == 2) {
        *reinterpret_cast<float2*>(o) = make_float2(s[0], s[1]);
      } else {
#pragma unroll
        for (int v4 = 0; v4 < V / 4; ++v4)
          reinterpret_cast<float4*>(o)[v4] =
              make_float4(s[4 * v4], s[4 * v4 + 1], s[4 * v4 + 2], s[4 * v4 + 3]);
      }
    }
    __syncthreads();
  }
}

// stride-2 dgrad (multiplier 1, C % 8 == 0): dx[ih, iw] only meets the taps kh = (ih + p) & 1
// (+2 ...) — the output rows oh = (ih + p - kh) / 2 are exact — so each thread walks just those
// (<= ceil(K/2)^2) taps of its 8 channels with 32-bit indexing, instead of testing all K*K taps
// for divisibility with 64-bit math as the generic kernel does.
template <int K>
__global__ __launch_bounds__(256) void dwk_dgrad_s2_kernel(const bf16* __restrict__ dy,
                                                           const float* __restrict__ wT, DwGeom g,
                                                           bf16* __restrict__ dx) {
  const int G = g.C >> 3;
  const int total = g.N * g.H * g.W * G;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int gi = i % G;
    int q = i / G;
    const int iw = q % g.W;
    q /= g.W;
    const int ih = q % g.H;
    const int n = q / g.H;
    const int c = gi * 8;
    float acc[8];
#pragma unroll
    for (int v = 0; v < 8; ++v) acc[v] = 0.f;
    const int kh0 = (ih + g.p) & 1, kw0 = (iw + g.p) & 1;
    const bf16* dyn = dy + (size_t)n * g.Ho * g.Wo * g.Co + c;
#pragma unroll
    for (int th = 0; th < (K + 1) / 2; ++th) {
      const int kh = kh0 + 2 * th;
      const int oh = (ih + g.p - kh) >> 1;
      if (kh >= K || (unsigned)oh >= (unsigned)g.Ho) continue;
#pragma unroll
      for (int tw = 0; tw < (K + 1) / 2; ++tw) {
        const int kw = kw0 + 2 * tw;
        const int ow = (iw + g.p - kw) >> 1;
        if (kw >= K || (unsigned)ow >= (unsigned)g.Wo) continue;
        float f[8];
        unpack8(*reinterpret_cast<const uint4*>(dyn + (oh * g.Wo + ow) * g.Co), f);
        const float* wr = wT + (kh * K + kw) * g.Co + c;
        const float4 w0 = *reinterpret_cast<const float4*>(wr);
        const float4 w1 = *reinterpret_cast<const float4*>(wr + 4);
        acc[0] += f[0] * w0.x; acc[1] += f[1] * w0.y; acc[2] += f[2] * w0.z; acc[3] += f[3] * w0.w;
        acc[4] += f[4] * w1.x; acc[5] += f[5] * w1.y; acc[6] += f[6] * w1.z; acc[7] += f[7] * w1.w;
      }
    }
    *reinterpret_cast<uint4*>(dx + (size_t)i * 8) = pack8(acc);
  }
}

// dw[co][tap] = sum_r partial[r][tap][co]: 32 columns x 8 row lanes per block, lanes added in
// a fixed order (deterministic)
__global__ __launch_bounds__(256) void dw_wgrad_final4_kernel(const float* __restrict__ partial,
                                                              int R, int T, int Co,
                                                              float* __restrict__ dw, int accum) {
  __shared__ float red[8][32];
  const int cl = threadIdx.x & 31, l = threadIdx.x >> 5;
  const int idx = blockIdx.x * 32 + cl;
  const int n = T * Co;
  float s = 0.f;
  if (idx < n) {
#pragma unroll 4
    for (int r = l; r < R; r += 8) s += partial[(size_t)r * n + idx];
  }
  red[l][cl] = s;
  __syncthreads();
  if (l == 0 && idx < n) {
    float o = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) o += red[k][cl];
    const int tap = idx / Co, co = idx - tap * Co;
    float* d = dw + (size_t)co * T + tap;
    *d = accum ? *d + o : o;   // accum: straight into the gradient arena (no separate add)
  }
}

// ---------------------------------------------------------------------------------------
// Fused BatchNorm epilogues (k3 / k5, stride 1 or 2, 8-channel vectors).
//   MODE 1 (forward): per-channel (sum, sumsq) of the output — the statistics of the BN that
//          consumes it, so that BN runs no separate statistics + finalize passes;
//   MODE 2 / 3 (dgrad): the backward reduce of the BN(+act) that produced this conv's input —
//          sum dz and sum dz * xhat, dz = dX * relu'(1-bit mask) (2) or dX * swish'(z),
//          z = y * scale + shift (3) — so that BN's backward runs no reduce + finalize passes.
// Channel-tiled mapping: a block owns CT (<= 8) channel groups of 8 and a share of the pixel
// strips, so its flush into the sharded accumulator is 2 x 64 columns (the plain kernels' mapping
// put every channel in every block: 2C atomics per block, ~16 MB of atomics per launch at
// MobileNetV2 bs1024 and 1.1-1.7x the plain time).
// ---------------------------------------------------------------------------------------
struct DwEpi {
  int mode;
  float* part;            // accumulator [shards][2][C]
  int shards;
  const bf16* y;          // dgrad modes: the BN input
  const uint8_t* mask;    // mode 2
  const float* aux;       // [mean | istd | scale | shift][C]
};

template <int MODE>
__device__ __forceinline__ void dw_epi_acc(const float* acc, const uint4& packed, const uint4& yv,
                                           uint32_t mb, const float* ax, float* s1, float* s2) {
  // ax: LDS [4][8] of this thread's channels (mean, istd, scale, shift)
  if constexpr (MODE == 1) {
#pragma unroll
    for (int v = 0; v < 8; ++v) {
      s1[v] += acc[v];
      s2[v] += acc[v] * acc[v];
    }
  } else {
    float f[8], yy[8];
    unpack8(packed, f);
    unpack8(yv, yy);
#pragma unroll
    for (int v = 0; v < 8; ++v) {
      float dz;
      if constexpr (MODE == 2) dz = ((mb >> v) & 1u) ? f[v] : 0.f;
      else dz = f[v] * act_grad(yy[v] * ax[16 + v] + ax[24 + v], ACT_SWISH);
      s1[v] += dz;
      s2[v] += dz * (yy[v] - ax[v]) * ax[8 + v];
    }
  }
}

// block tile geometry: CT groups x (256 / CT) workers
struct DwTile {
  int ct, ntile, gl, wk, nwk, g0, part, parts;
  __device__ DwTile(int G) {
    ct = G < 8 ? G : 8;
    ntile = (G + ct - 1) / ct;
    gl = threadIdx.x % ct;
    wk = threadIdx.x / ct;
    nwk = 256 / ct;
    const int tile = blockIdx.x % ntile;
    g0 = tile * ct;
    part = blockIdx.x / ntile;
    parts = gridDim.x / ntile;
  }
};

// LDS: aux [CT*8][4 rows interleaved per channel group] then the flush sums [2][CT*8]
template <int MODE>
__device__ __forceinline__ void dw_epi_setup(const DwEpi& e, const DwTile& t, int G, int C,
                                             float* ax_s, float* red) {
  const int nch = t.ct * 8;
  for (int k = threadIdx.x; k < 2 * nch; k += 256) red[k] = 0.f;
  if constexpr (MODE >= 2) {
    for (int k = threadIdx.x; k < t.ct * 32; k += 256) {
      const int gl = k / 32, r = (k / 8) % 4, v = k % 8;
      const int c = (t.g0 + gl) * 8 + v;
      ax_s[k] = (t.g0 + gl < G) ? e.aux[r * C + c] : 0.f;
    }
  }
  __syncthreads();
}

__device__ __forceinline__ void dw_epi_flush2(const DwEpi& e, const DwTile& t, bool has, int C,
                                              const float* s1, const float* s2, float* red) {
  const int nch = t.ct * 8;
  if (has) {
#pragma unroll
    for (int v = 0; v < 8; ++v) {
      atomicAdd(red + t.gl * 8 + v, s1[v]);
      atomicAdd(red + nch + t.gl * 8 + v, s2[v]);
    }
  }
  __syncthreads();
  for (int k = threadIdx.x; k < 2 * nch; k += 256) {
    const int half = k / nch, cc = k % nch;
    const int c = t.g0 * 8 + cc;
    if (c < C) stat_out(e.part, blockIdx.x, e.shards, 2 * C, half * C + c, red[k]);
  }
}

template <int K, int S, bool FLIP, int MODE>
__global__ __launch_bounds__(256) void dwk_epi_kernel(const bf16* __restrict__ x,
                                                      const float* __restrict__ wT, DwGeom g,
                                                      int rpt, bf16* __restrict__ y, DwEpi e) {
  constexpr int KK = K * K;
  constexpr int V = 8;
  using T = uint4;
  __shared__ float ax_s[8 * 32];
  __shared__ float red[2 * 64];
  const int G = g.C / V;
  const DwTile t(G);
  dw_epi_setup<MODE>(e, t, G, g.Co, ax_s, red);
  const int gi = t.g0 + t.gl;
  const bool active = t.wk < t.nwk && gi < G;
  const int c = gi * V;
  const int nstrip = (g.Ho + rpt - 1) / rpt;
  const int items = g.N * nstrip * g.Wo;
  float s1[8], s2[8];
#pragma unroll
  for (int v = 0; v < 8; ++v) s1[v] = s2[v] = 0.f;
  if (active) {
    float w[KK][V];
#pragma unroll
    for (int tp = 0; tp < KK; ++tp) {
      const int src = FLIP ? KK - 1 - tp : tp;
#pragma unroll
      for (int v4 = 0; v4 < V; v4 += 4) {
        const float4 wv = *reinterpret_cast<const float4*>(wT + src * g.Co + c + v4);
        w[tp][v4] = wv.x; w[tp][v4 + 1] = wv.y; w[tp][v4 + 2] = wv.z; w[tp][v4 + 3] = wv.w;
      }
    }
    const float* ax = ax_s + t.gl * 32;
    for (int j = t.part * t.nwk + t.wk; j < items; j += t.parts * t.nwk) {
      const int ow = j % g.Wo;
      const int q = j / g.Wo;
      const int strip = q % nstrip;
      const int n = q / nstrip;
      const bf16* xn = x + (size_t)n * g.H * g.W * g.C + c;
      const int oh0 = strip * rpt, oh1 = min(g.Ho, oh0 + rpt);
      const int iw0 = ow * S - g.p;
      T win[K][K];
#pragma unroll
      for (int k = 0; k < K - S; ++k) dwk_load_row<K, V>(xn, g, oh0 * S - g.p + k, iw0, win[k]);
      bf16* yr = y + (((size_t)n * g.Ho + oh0) * g.Wo + ow) * g.Co + c;
#pragma unroll 1
      for (int oh = oh0; oh < oh1; ++oh) {
        const int ih0 = oh * S - g.p;
#pragma unroll
        for (int k = K - S; k < K; ++k) dwk_load_row<K, V>(xn, g, ih0 + k, iw0, win[k]);
        const size_t o = (size_t)(yr - y);
        uint4 yv = make_uint4(0u, 0u, 0u, 0u);
        uint32_t mb = 0;
        if constexpr (MODE >= 2) yv = *reinterpret_cast<const uint4*>(e.y + o);
        if constexpr (MODE == 2) mb = e.mask[o >> 3];
        float acc[V];
#pragma unroll
        for (int v = 0; v < V; ++v) acc[v] = 0.f;
#pragma unroll
        for (int kh = 0; kh < K; ++kh)
#pragma unroll
          for (int kw = 0; kw < K; ++kw) {
            float f[V];
            dw_unpack<V>(win[kh][kw], f);
#pragma unroll
            for (int v = 0; v < V; ++v) acc[v] += f[v] * w[kh * K + kw][v];
          }
        const uint4 packed = pack8(acc);
        *reinterpret_cast<uint4*>(yr) = packed;
        dw_epi_acc<MODE>(acc, packed, yv, mb, ax, s1, s2);
        yr += (size_t)g.Wo * g.Co;
        dwk_roll<K, S>(win);
      }
    }
  }
  dw_epi_flush2(e, t, active, g.Co, s1, s2, red);
}

// stride-2 dgrad (the parity-exact tap walk of dwk_dgrad_s2_kernel) with MODE 2 / 3
template <int K, int MODE>
__global__ __launch_bounds__(256) void dwk_epi_s2_kernel(const bf16* __restrict__ dy,
                                                         const float* __restrict__ wT, DwGeom g,
                                                         bf16* __restrict__ dx, DwEpi e) {
  __shared__ float ax_s[8 * 32];
  __shared__ float red[2 * 64];
  const int G = g.C >> 3;
  const DwTile t(G);
  dw_epi_setup<MODE>(e, t, G, g.C, ax_s, red);
  const int gi = t.g0 + t.gl;
  const bool active = t.wk < t.nwk && gi < G;
  const int c = gi * 8;
  const int items = g.N * g.H * g.W;
  float s1[8], s2[8];
#pragma unroll
  for (int v = 0; v < 8; ++v) s1[v] = s2[v] = 0.f;
  if (active) {
    const float* ax = ax_s + t.gl * 32;
    for (int j = t.part * t.nwk + t.wk; j < items; j += t.parts * t.nwk) {
      const int iw = j % g.W;
      const int q = j / g.W;
      const int ih = q % g.H;
      const int n = q / g.H;
      const size_t o = (size_t)j * g.C + c;
      uint4 yv = *reinterpret_cast<const uint4*>(e.y + o);
      uint32_t mb = 0;
      if constexpr (MODE == 2) mb = e.mask[o >> 3];
      float acc[8];
#pragma unroll
      for (int v = 0; v < 8; ++v) acc[v] = 0.f;
      const int kh0 = (ih + g.p) & 1, kw0 = (iw + g.p) & 1;
      const bf16* dyn = dy + (size_t)n * g.Ho * g.Wo * g.Co + c;
#pragma unroll
      for (int th = 0; th < (K + 1) / 2; ++th) {
        const int kh = kh0 + 2 * th;
        const int oh = (ih + g.p - kh) >> 1;
        if (kh >= K || (unsigned)oh >= (unsigned)g.Ho) continue;
#pragma unroll
        for (int tw = 0; tw < (K + 1) / 2; ++tw) {
          const int kw = kw0 + 2 * tw;
          const int ow = (iw + g.p - kw) >> 1;
          if (kw >= K || (unsigned)ow >= (unsigned)g.Wo) continue;
          float f[8];
          unpack8(*reinterpret_cast<const uint4*>(dyn + (oh * g.Wo + ow) * g.Co), f);
          const float* wr = wT + (kh * K + kw) * g.Co + c;
          const float4 w0 = *reinterpret_cast<const float4*>(wr);
          const float4 w1 = *reinterpret_cast<const float4*>(wr + 4);
          acc[0] += f[0] * w0.x; acc[1] += f[1] * w0.y; acc[2] += f[2] * w0.z; acc[3] += f[3] * w0.w;
          acc[4] += f[4] * w1.x; acc[5] += f[5] * w1.y; acc[6] += f[6] * w1.z; acc[7] += f[7] * w1.w;
        }
      }
      const uint4 packed = pack8(acc);
      *reinterpret_cast<uint4*>(dx + o) = packed;
      dw_epi_acc<MODE>(acc, packed, yv, mb, ax, s1, s2);
    }
  }
  dw_epi_flush2(e, t, active, g.C, s1, s2, red);
}

// ================================================================================ host
static DwGeom dwg(int N, int H, int W, int C, int Ho, int Wo, int Co, int KH, int KW, int s, int p) {
  DwGeom g{N, H, W, C, Ho, Wo, Co, KH, KW, s, p, Co / C};
  return g;
}
static int gcap(size_t work) {
  size_t b = (work + 255) / 256;
  return (int)(b < 8192 ? (b ? b : 1) : 8192);
}

// K of the fast path (3 or 5) this geometry takes, 0 = generic kernels
static int dwk_kind(const DwGeom& g) {
  static const bool off = [] {
    const char* e = getenv("PCA_DW3");
    return e && e[0] == '0';
  }();
  if (off || g.mult != 1 || g.KH != g.KW || (g.s != 1 && g.s != 2)) return 0;
  if (g.C % 2) return 0;
  if (g.KH == 3 && g.p == 1) return 3;
  if (g.KH == 5 && g.p == 2) return 5;
  if (g.KH == 7 && g.p == 3) return 7;   // PNASNet SepConv k7 (pnasnet.py:14-17)
  return 0;
}

// channels per thread: the widest vector C allows, capped per K by the register budget
// (ShuffleNetV2's 58/116/232-channel branches take V = 2 / 4 at k3)
static int dwk_vec(int kind, int C) {
  const int vmax = kind == 3 ? 8 : kind == 5 ? 4 : 2;
  if (vmax >= 8 && C % 8 == 0) return 8;
  if (vmax >= 4 && C % 4 == 0) return 4;
  return 2;
}

static int dwk_rpt(int Ho) { return Ho < 8 ? Ho : 8; }

template <int K, int V, int IN = 0>
static void dwk_fwd_t(const bf16* x, const float* wT, const DwGeom& g, bool flip, bf16* y,
                      hipStream_t st, const float* isc = nullptr, const float* ish = nullptr) {
  const int rpt = dwk_rpt(g.Ho);
  const size_t work = (size_t)g.N * cdiv(g.Ho, rpt) * g.Wo * (g.C / V);
  const dim3 grid(gcap(work)), block(256);
  if (g.s == 1) {
    if (flip) hipLaunchKernelGGL((dwk_fwd_kernel<K, 1, V, true>), grid, block, 0, st, x, wT, g, rpt, y, nullptr, nullptr);
    else hipLaunchKernelGGL((dwk_fwd_kernel<K, 1, V, false, IN>), grid, block, 0, st, x, wT, g, rpt, y, isc, ish);
  } else {
    hipLaunchKernelGGL((dwk_fwd_kernel<K, 2, V, false, IN>), grid, block, 0, st, x, wT, g, rpt, y, isc, ish);
  }
}

template <int IN = 0>
static void dwk_fwd(int kind, const bf16* x, const float* wT, const DwGeom& g, bool flip, bf16* y,
                    hipStream_t st, const float* isc = nullptr, const float* ish = nullptr) {
  const int v = dwk_vec(kind, g.C);
  if (kind == 3) {
    if (v == 8) dwk_fwd_t<3, 8, IN>(x, wT, g, flip, y, st, isc, ish);
    else if (v == 4) dwk_fwd_t<3, 4, IN>(x, wT, g, flip, y, st, isc, ish);
    else dwk_fwd_t<3, 2, IN>(x, wT, g, flip, y, st, isc, ish);
  } else if (kind == 5) {
    if (v == 4) dwk_fwd_t<5, 4, IN>(x, wT, g, flip, y, st, isc, ish);
    else dwk_fwd_t<5, 2, IN>(x, wT, g, flip, y, st, isc, ish);
  } else {
    dwk_fwd_t<7, 2, IN>(x, wT, g, flip, y, st, isc, ish);
  }
}

template <int K, int V, int IN = 0>
static void dwk_wgrad_t(const bf16* x, const bf16* dy, const DwGeom& g, int chunks,
                        float* partial, hipStream_t st, const float* isc = nullptr,
                        const float* ish = nullptr) {
  const int G = g.Co / V;
  const int ny = cdiv(G, 256);
  const int GB = cdiv(G, ny);
  const int rpt = dwk_rpt(g.Ho);
  const dim3 grid(chunks, ny), block(256);
  if (g.s == 1)
    hipLaunchKernelGGL((dwk_wgrad_kernel<K, 1, V, IN>), grid, block, 0, st, x, dy, g, rpt, GB, partial, isc, ish);
  else
    hipLaunchKernelGGL((dwk_wgrad_kernel<K, 2, V, IN>), grid, block, 0, st, x, dy, g, rpt, GB, partial, isc, ish);
}

// k3 with 8-channel groups
static bool dw_epi_ok(const DwGeom& g) {
  // (k5 x 8 channels holds 200 weight registers: one wave per SIMD — k5 keeps the plain passes)
  return dwk_kind(g) == 3 && g.C % 8 == 0 && g.mult == 1;
}

// blocks: channel tiles x pixel parts, ~2048 in all (2 x 64 accumulator adds each)
static int dw_epi_blocks(int G, int items) {
  const int ct = G < 8 ? G : 8;
  const int ntile = cdiv(G, ct);
  const int nwk = 256 / ct;
  int parts = std::max(1, std::min(cdiv(items, nwk), cdiv(2048, ntile)));
  return ntile * parts;
}

template <int MODE>
static void dw_epi_launch(int kind, bool flip, const bf16* x, const float* wT, const DwGeom& g,
                          bf16* y, const DwEpi& e, hipStream_t st) {
  const int rpt = dwk_rpt(g.Ho);
  const int items = g.N * cdiv(g.Ho, rpt) * g.Wo;
  const dim3 grid(dw_epi_blocks(g.C / 8, items)), block(256);
#define PCA_DWE(K, S, F) \
  hipLaunchKernelGGL((dwk_epi_kernel<K, S, F, MODE>), grid, block, 0, st, x, wT, g, rpt, y, e)
  (void)kind;   // k3 only (dw_epi_ok)
  if (g.s == 2) PCA_DWE(3, 2, false);
  else if (flip) PCA_DWE(3, 1, true);
  else PCA_DWE(3, 1, false);
#undef PCA_DWE
}

// forward with the consumer BN's statistics fused (mode 1); false: not launched
bool dw_fwd_stats_launch(const bf16* x, const float* wT, int N, int H, int W, int C, int Ho,
                         int Wo, int Co, int KH, int KW, int s, int p, bf16* y, float* acc,
                         int shards, hipStream_t st) {
  DwGeom g = dwg(N, H, W, C, Ho, Wo, Co, KH, KW, s, p);
  if (!dw_epi_ok(g) || shards <= 0) return false;
  const DwEpi e{1, acc, shards, nullptr, nullptr, nullptr};
  dw_epi_launch<1>(dwk_kind(g), false, x, wT, g, y, e, st);
  return true;
}

// dgrad with the producer BN's backward reduce fused (act 1: ReLU through the 1-bit mask, 2:
// swish from y and aux); false: not launched
bool dw_dgrad_bn_launch(const bf16* dy, const float* wT, int N, int H, int W, int C, int Ho,
                        int Wo, int Co, int KH, int KW, int s, int p, bf16* dx, const bf16* bn_y,
                        const uint8_t* bn_mask, const float* bn_aux, int act, float* acc,
                        int shards, hipStream_t st) {
  DwGeom g = dwg(N, H, W, C, Ho, Wo, Co, KH, KW, s, p);
  if (!dw_epi_ok(g) || shards <= 0 || (act != 1 && act != 2) || (act == 1 && !bn_mask))
    return false;
  const DwEpi e{act == 1 ? 2 : 3, acc, shards, bn_y, bn_mask, bn_aux};
  const int kind = dwk_kind(g);
  if (s == 1) {
    const DwGeom gd = dwg(N, Ho, Wo, Co, H, W, C, KH, KW, 1, KH - 1 - p);
    if (act == 1) dw_epi_launch<2>(kind, true, dy, wT, gd, dx, e, st);
    else dw_epi_launch<3>(kind, true, dy, wT, gd, dx, e, st);
    return true;
  }
  const dim3 grid(dw_epi_blocks(C / 8, N * H * W)), block(256);
  (void)kind;
  if (act == 1) hipLaunchKernelGGL((dwk_epi_s2_kernel<3, 2>), grid, block, 0, st, dy, wT, g, dx, e);
  else hipLaunchKernelGGL((dwk_epi_s2_kernel<3, 3>), grid, block, 0, st, dy, wT, g, dx, e);
  return true;
}

// ---- depthwise conv with the producer BN(+act) applied on its input loads (IN transform) ----
// supported: the k3 / k5 / k7 fast paths, multiplier 1 (the mobile zoo's depthwise convs)
bool dw_in_supported(int N, int H, int W, int C, int Ho, int Wo, int Co, int KH, int KW, int s,
                     int p, int act) {
  DwGeom g = dwg(N, H, W, C, Ho, Wo, Co, KH, KW, s, p);
  return dwk_kind(g) != 0 && g.mult == 1 && (act == ACT_RELU || act == ACT_SWISH);
}

// x is the BN input y; isc / ish = that BN's scale / shift rows (aux rows 2 and 3)
void dw_fwd_in_launch(const bf16* x, const float* wT, int N, int H, int W, int C, int Ho, int Wo,
                      int Co, int KH, int KW, int s, int p, const float* isc, const float* ish,
                      int act, bf16* y, hipStream_t st) {
  DwGeom g = dwg(N, H, W, C, Ho, Wo, Co, KH, KW, s, p);
  const int kind = dwk_kind(g);
  if (act == ACT_SWISH) dwk_fwd<ACT_SWISH>(kind, x, wT, g, false, y, st, isc, ish);
  else dwk_fwd<ACT_RELU>(kind, x, wT, g, false, y, st, isc, ish);
}

void dw_wgrad_in_launch(const bf16* x, const bf16* dy, int N, int H, int W, int C, int Ho, int Wo,
                        int Co, int KH, int KW, int s, int p, const float* isc, const float* ish,
                        int act, float* partial, int chunks, int accum, float* dw,
                        hipStream_t st) {
  DwGeom g = dwg(N, H, W, C, Ho, Wo, Co, KH, KW, s, p);
  const int kind = dwk_kind(g);
  const int T = KH * KW;
  const int v = dwk_vec(kind, Co);
#define PCA_DWIN(K_, V_)                                                                  \
  do {                                                                                    \
    if (act == ACT_SWISH) dwk_wgrad_t<K_, V_, ACT_SWISH>(x, dy, g, chunks, partial, st, isc, ish); \
    else dwk_wgrad_t<K_, V_, ACT_RELU>(x, dy, g, chunks, partial, st, isc, ish);          \
  } while (0)
  if (kind == 3 && v == 8) PCA_DWIN(3, 8);
  else if (kind == 3 && v == 4) PCA_DWIN(3, 4);
  else if (kind == 3) PCA_DWIN(3, 2);
  else if (kind == 5 && v == 4) PCA_DWIN(5, 4);
  else if (kind == 5) PCA_DWIN(5, 2);
  else PCA_DWIN(7, 2);
#undef PCA_DWIN
  hipLaunchKernelGGL(dw_wgrad_final4_kernel, dim3(cdiv(T * Co, 32)), dim3(256), 0, st, partial,
                     chunks, T, Co, dw, accum);
}

void dw_fwd_launch(const bf16* x, const float* wT, int N, int H, int W, int C, int Ho, int Wo,
                   int Co, int KH, int KW, int s, int p, bf16* y, hipStream_t st) {
  DwGeom g = dwg(N, H, W, C, Ho, Wo, Co, KH, KW, s, p);
  if (const int kind = dwk_kind(g)) return dwk_fwd(kind, x, wT, g, false, y, st);
  if (g.mult == 1 && C % 8 == 0)
    hipLaunchKernelGGL(dw_fwd_kernel<8>, dim3(gcap((size_t)N * Ho * Wo * Co / 8)), dim3(256), 0, st,
                       x, wT, g, y);
  else
    hipLaunchKernelGGL(dw_fwd_kernel<1>, dim3(gcap((size_t)N * Ho * Wo * Co)), dim3(256), 0, st, x,
                       wT, g, y);
}

void dw_dgrad_launch(const bf16* dy, const float* wT, int N, int H, int W, int C, int Ho, int Wo,
                     int Co, int KH, int KW, int s, int p, bf16* dx, hipStream_t st) {
  DwGeom g = dwg(N, H, W, C, Ho, Wo, Co, KH, KW, s, p);
  const int kind = dwk_kind(g);
  if (kind && s == 1) {
    // stride-1 dgrad = forward correlation of dY with the mirrored taps (pad K-1-p)
    const DwGeom gd = dwg(N, Ho, Wo, Co, H, W, C, KH, KW, 1, KH - 1 - p);
    return dwk_fwd(kind, dy, wT, gd, true, dx, st);
  }
  if (kind && C % 8 == 0) {   // stride 2: parity-exact taps
    const dim3 grid(gcap((size_t)N * H * W * C / 8)), block(256);
    if (kind == 3) hipLaunchKernelGGL(dwk_dgrad_s2_kernel<3>, grid, block, 0, st, dy, wT, g, dx);
    else if (kind == 5) hipLaunchKernelGGL(dwk_dgrad_s2_kernel<5>, grid, block, 0, st, dy, wT, g, dx);
    else hipLaunchKernelGGL(dwk_dgrad_s2_kernel<7>, grid, block, 0, st, dy, wT, g, dx);
    return;
  }
  if (g.mult == 1 && C % 8 == 0)
    hipLaunchKernelGGL(dw_dgrad_kernel<8>, dim3(gcap((size_t)N * H * W * C / 8)), dim3(256), 0, st,
                       dy, wT, g, dx);
  else
    hipLaunchKernelGGL(dw_dgrad_kernel<1>, dim3(gcap((size_t)N * H * W * C)), dim3(256), 0, st, dy,
                       wT, g, dx);
}

// partial rows = grid.x of the wgrad kernels: one per 256 output pixels, but at least 256 (one
// block per CU) so the small late-stage maps (EfficientNet 2x2 / 4x4: P = 4-16K) still fill the
// chip, and at most 1024 (the final reduce reads rows x taps x Co floats)
int dw_wgrad_partials(int N, int Ho, int Wo) {
  const int P = N * Ho * Wo;
  int chunks = std::max(cdiv(P, 256), std::min(256, P));
  return chunks > 1024 ? 1024 : chunks;
}

void dw_wgrad_launch(const bf16* x, const bf16* dy, int N, int H, int W, int C, int Ho, int Wo,
                     int Co, int KH, int KW, int s, int p, float* partial, int chunks,
                     int accum, float* dw, hipStream_t st) {
  DwGeom g = dwg(N, H, W, C, Ho, Wo, Co, KH, KW, s, p);
  const int P = N * Ho * Wo;
  const int rows = cdiv(P, chunks);
  const int T = KH * KW;
  if (const int kind = dwk_kind(g)) {
    // chunks = partial rows = blocks (grid.x) of the strip-walking kernel
    static const int vcap = [] {   // debug knob: cap the wgrad vector width (register budget A/B)
      const char* e = getenv("PCA_DWK_WGRAD_V");
      return e ? atoi(e) : 8;
    }();
    int v = dwk_vec(kind, Co);
    while (v > vcap && v > 2) v >>= 1;
    if (kind == 3 && v == 8) dwk_wgrad_t<3, 8>(x, dy, g, chunks, partial, st);
    else if (kind == 3 && v == 4) dwk_wgrad_t<3, 4>(x, dy, g, chunks, partial, st);
    else if (kind == 3) dwk_wgrad_t<3, 2>(x, dy, g, chunks, partial, st);
    else if (kind == 5 && v == 4) dwk_wgrad_t<5, 4>(x, dy, g, chunks, partial, st);
    else if (kind == 5) dwk_wgrad_t<5, 2>(x, dy, g, chunks, partial, st);
    else dwk_wgrad_t<7, 2>(x, dy, g, chunks, partial, st);
    hipLaunchKernelGGL(dw_wgrad_final4_kernel, dim3(cdiv(T * Co, 32)), dim3(256), 0, st, partial,
                       chunks, T, Co, dw, accum);
    return;
  }
  if (g.mult == 1 && Co % 8 == 0)
    hipLaunchKernelGGL(dw_wgrad_kernel<8>, dim3(chunks, T), dim3(256), 0, st, x, dy, g, rows,
                       partial);
  else
    hipLaunchKernelGGL(dw_wgrad_kernel<1>, dim3(chunks, T), dim3(256), 0, st, x, dy, g, rows,
                       partial);
  hipLaunchKernelGGL(dw_wgrad_final4_kernel, dim3(cdiv(T * Co, 32)), dim3(256), 0, st, partial,
                     chunks, T, Co, dw, accum);
}

}  // namespace pca
