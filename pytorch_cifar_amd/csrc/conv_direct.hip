// Generic direct convolution (any Cin/G, Cout/G, kernel, stride, padding), NHWC bf16 in/out,
// fp32 accumulation. SURVEY §2.8 K7: covers what the MFMA implicit-GEMM path cannot tile —
// LeNet's 3->6->16 5x5 convs (lenet.py:8-9), DPN's groups=32 with Cin/G = 3..24 (dpn.py:15),
// ResNeXt29_32x4d Cin/G = 4 (resnext.py:19), PNASNet-A's 44-channel cells, ShuffleNet's 50/25
// channel bottlenecks and densenet_cifar's growth-12 layers.
//
// fwd  : one thread per output element, loops taps x Cin/G.
// dgrad: one thread per input element, gathers the (tap, co) pairs that read it.
// wgrad: grid (weight-element tiles, pixel splits) -> partial slab -> deterministic fold.
#include "common.h"

namespace pca {

struct DirGeom {
  int N, H, W, Cin, Ho, Wo, Cout, KH, KW, s, p, G, cin_g, cout_g;
};

__global__ __launch_bounds__(256) void direct_fwd_kernel(const bf16* __restrict__ x,
                                                         const float* __restrict__ w,
                                                         const float* __restrict__ bias, DirGeom g,
                                                         bf16* __restrict__ y) {
  const size_t total = (size_t)g.N * g.Ho * g.Wo * g.Cout;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    const int co = (int)(i % g.Cout);
    size_t q = i / g.Cout;
    const int ow = (int)(q % g.Wo);
    q /= g.Wo;
    const int oh = (int)(q % g.Ho);
    const int n = (int)(q / g.Ho);
    const int grp = co / g.cout_g;
    float acc = bias ? bias[co] : 0.f;
    const float* wr = w + (size_t)co * g.KH * g.KW * g.cin_g;  // [co][kh][kw][ci]
    for (int kh = 0; kh < g.KH; ++kh) {
      const int ih = oh * g.s - g.p + kh;
      if (ih < 0 || ih >= g.H) continue;
      for (int kw = 0; kw < g.KW; ++kw) {
        const int iw = ow * g.s - g.p + kw;
        if (iw < 0 || iw >= g.W) continue;
        const bf16* xr = x + (((size_t)n * g.H + ih) * g.W + iw) * g.Cin + grp * g.cin_g;
        const float* wt = wr + (kh * g.KW + kw) * g.cin_g;
        for (int ci = 0; ci < g.cin_g; ++ci) acc += bf2f(xr[ci]) * wt[ci];
      }
    }
    y[i] = f2bf(acc);
  }
}

__global__ __launch_bounds__(256) void direct_dgrad_kernel(const bf16* __restrict__ dy,
                                                           const float* __restrict__ w, DirGeom g,
                                                           bf16* __restrict__ dx) {
  const size_t total = (size_t)g.N * g.H * g.W * g.Cin;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    const int ci = (int)(i % g.Cin);
    size_t q = i / g.Cin;
    const int iw = (int)(q % g.W);
    q /= g.W;
    const int ih = (int)(q % g.H);
    const int n = (int)(q / g.H);
    const int grp = ci / g.cin_g, cil = ci % g.cin_g;
    float acc = 0.f;
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
        const bf16* dr = dy + (((size_t)n * g.Ho + oh) * g.Wo + ow) * g.Cout + grp * g.cout_g;
        const float* wt = w + (size_t)grp * g.cout_g * g.KH * g.KW * g.cin_g +
                          (kh * g.KW + kw) * g.cin_g + cil;
        const size_t wstride = (size_t)g.KH * g.KW * g.cin_g;
        for (int co = 0; co < g.cout_g; ++co) acc += bf2f(dr[co]) * wt[co * wstride];
      }
    }
    dx[i] = f2bf(acc);
  }
}

// partial[split][Wel] with Wel = Cout*KH*KW*cin_g in [co][kh][kw][ci] order; bias grads in the
// trailing Cout entries (sum of dy).
__global__ __launch_bounds__(256) void direct_wgrad_kernel(const bf16* __restrict__ x,
                                                           const bf16* __restrict__ dy, DirGeom g,
                                                           int chunk, int with_bias,
                                                           float* __restrict__ partial) {
  const int Wel = g.Cout * g.KH * g.KW * g.cin_g;
  const int tot = Wel + (with_bias ? g.Cout : 0);
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= tot) return;
  const int P = g.N * g.Ho * g.Wo;
  const int p0 = blockIdx.y * chunk, p1 = min(P, p0 + chunk);
  float acc = 0.f;
  if (e < Wel) {
    const int ci = e % g.cin_g;
    int q = e / g.cin_g;
    const int kw = q % g.KW;
    q /= g.KW;
    const int kh = q % g.KH;
    const int co = q / g.KH;
    const int grp = co / g.cout_g;
    for (int pix = p0; pix < p1; ++pix) {
      const int ow = pix % g.Wo;
      const int r = pix / g.Wo;
      const int oh = r % g.Ho, n = r / g.Ho;
      const int ih = oh * g.s - g.p + kh, iw = ow * g.s - g.p + kw;
      if (ih < 0 || ih >= g.H || iw < 0 || iw >= g.W) continue;
      acc += bf2f(dy[(size_t)pix * g.Cout + co]) *
             bf2f(x[(((size_t)n * g.H + ih) * g.W + iw) * g.Cin + grp * g.cin_g + ci]);
    }
  } else {
    const int co = e - Wel;
    for (int pix = p0; pix < p1; ++pix) acc += bf2f(dy[(size_t)pix * g.Cout + co]);
  }
  partial[(size_t)blockIdx.y * tot + e] = acc;
}

__global__ void fold_rows_kernel(const float* __restrict__ partial, int R, int L,
                                 float* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= L) return;
  float s = 0.f;
  for (int r = 0; r < R; ++r) s += partial[(size_t)r * L + i];
  out[i] = s;
}

static DirGeom dg(int N, int H, int W, int Cin, int Ho, int Wo, int Cout, int KH, int KW, int s,
                  int p, int G) {
  DirGeom g{N, H, W, Cin, Ho, Wo, Cout, KH, KW, s, p, G, Cin / G, Cout / G};
  return g;
}
static int gcap2(size_t work) {
  size_t b = (work + 255) / 256;
  return (int)(b < 16384 ? (b ? b : 1) : 16384);
}

void direct_fwd_launch(const bf16* x, const float* w, const float* bias, int N, int H, int W,
                       int Cin, int Ho, int Wo, int Cout, int KH, int KW, int s, int p, int G,
                       bf16* y, hipStream_t st) {
  DirGeom g = dg(N, H, W, Cin, Ho, Wo, Cout, KH, KW, s, p, G);
  hipLaunchKernelGGL(direct_fwd_kernel, dim3(gcap2((size_t)N * Ho * Wo * Cout)), dim3(256), 0, st,
                     x, w, bias, g, y);
}

void direct_dgrad_launch(const bf16* dy, const float* w, int N, int H, int W, int Cin, int Ho,
                         int Wo, int Cout, int KH, int KW, int s, int p, int G, bf16* dx,
                         hipStream_t st) {
  DirGeom g = dg(N, H, W, Cin, Ho, Wo, Cout, KH, KW, s, p, G);
  hipLaunchKernelGGL(direct_dgrad_kernel, dim3(gcap2((size_t)N * H * W * Cin)), dim3(256), 0, st,
                     dy, w, g, dx);
}

int direct_wgrad_splits(int N, int Ho, int Wo, int welems) {
  const int P = N * Ho * Wo;
  const int wblocks = cdiv(welems, 256);
  int splits = cdiv(2048, wblocks);
  splits = splits < 1 ? 1 : splits;
  const int maxs = cdiv(P, 64);
  return splits > maxs ? maxs : splits;
}

// dw out: [Cout*KH*KW*cin_g (+Cout bias)] fp32
void direct_wgrad_launch(const bf16* x, const bf16* dy, int N, int H, int W, int Cin, int Ho,
                         int Wo, int Cout, int KH, int KW, int s, int p, int G, int with_bias,
                         float* partial, int splits, float* out, hipStream_t st) {
  DirGeom g = dg(N, H, W, Cin, Ho, Wo, Cout, KH, KW, s, p, G);
  const int tot = Cout * KH * KW * (Cin / G) + (with_bias ? Cout : 0);
  const int P = N * Ho * Wo;
  const int chunk = cdiv(P, splits);
  hipLaunchKernelGGL(direct_wgrad_kernel, dim3(cdiv(tot, 256), splits), dim3(256), 0, st, x, dy, g,
                     chunk, with_bias, partial);
  hipLaunchKernelGGL(fold_rows_kernel, dim3(cdiv(tot, 256)), dim3(256), 0, st, partial, splits, tot,
                     out);
}

}  // namespace pca
