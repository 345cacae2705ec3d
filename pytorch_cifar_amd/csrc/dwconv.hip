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

// ================================================================================ host
static DwGeom dwg(int N, int H, int W, int C, int Ho, int Wo, int Co, int KH, int KW, int s, int p) {
  DwGeom g{N, H, W, C, Ho, Wo, Co, KH, KW, s, p, Co / C};
  return g;
}
static int gcap(size_t work) {
  size_t b = (work + 255) / 256;
  return (int)(b < 8192 ? (b ? b : 1) : 8192);
}

void dw_fwd_launch(const bf16* x, const float* wT, int N, int H, int W, int C, int Ho, int Wo,
                   int Co, int KH, int KW, int s, int p, bf16* y, hipStream_t st) {
  DwGeom g = dwg(N, H, W, C, Ho, Wo, Co, KH, KW, s, p);
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
  if (g.mult == 1 && C % 8 == 0)
    hipLaunchKernelGGL(dw_dgrad_kernel<8>, dim3(gcap((size_t)N * H * W * C / 8)), dim3(256), 0, st,
                       dy, wT, g, dx);
  else
    hipLaunchKernelGGL(dw_dgrad_kernel<1>, dim3(gcap((size_t)N * H * W * C)), dim3(256), 0, st, dy,
                       wT, g, dx);
}

int dw_wgrad_partials(int N, int Ho, int Wo) {
  const int P = N * Ho * Wo;
  int chunks = cdiv(P, 256);
  return chunks > 256 ? 256 : chunks;
}

void dw_wgrad_launch(const bf16* x, const bf16* dy, int N, int H, int W, int C, int Ho, int Wo,
                     int Co, int KH, int KW, int s, int p, float* partial, int chunks,
                     float* partial2, float* dw, hipStream_t st) {
  DwGeom g = dwg(N, H, W, C, Ho, Wo, Co, KH, KW, s, p);
  const int P = N * Ho * Wo;
  const int rows = cdiv(P, chunks);
  const int T = KH * KW;
  if (g.mult == 1 && Co % 8 == 0)
    hipLaunchKernelGGL(dw_wgrad_kernel<8>, dim3(chunks, T), dim3(256), 0, st, x, dy, g, rows,
                       partial);
  else
    hipLaunchKernelGGL(dw_wgrad_kernel<1>, dim3(chunks, T), dim3(256), 0, st, x, dy, g, rows,
                       partial);
  hipLaunchKernelGGL(dw_wgrad_final_kernel, dim3(cdiv(T * Co, 256)), dim3(256), 0, st, partial,
                     chunks, T, Co, dw);
  (void)partial2;
}

}  // namespace pca
