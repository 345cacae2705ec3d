// Fused Winograd F(2x2, 3x3) forward convolution (3x3 / stride 1 / pad 1, NHWC bf16) on gfx950
// MFMA — the "implicit-GEMM / Winograd" alternative of the BASELINE north star for the ResNet
// 3x3 convs (reference models/resnet.py:23-27), layers 2-4 (C = 128 / 256 / 512).
//
//   V = B^T d B (4x4 input patch d of each 2x2 output tile, per input channel)
//   U = G g G^T (per (co, ci); winograd_filter_kernel, [16][Co][Ci] bf16)
//   M[p] = V[p] U[p]   p = 0..15: 16 GEMMs of [tiles x Ci] x [Ci x Co]  (2.25x fewer MACs)
//   Y = A^T M A (2x2 outputs per tile)
//
// One workgroup = 32 output tiles x 64 output channels, 4 waves. Per K-step of 32 input channels
// every thread loads one tile's 4x4 patch of 4 channels (16 x 8-byte loads, zeros outside the
// image), transforms it in registers and writes the 16 points to LDS (the A operands of the 16
// GEMMs, shared by the 4 waves); the next K-step's patch is loaded into registers while this
// step's MFMAs run. Wave w owns output channels [16w, 16w + 16) for ALL 16 points and both
// 16-tile halves: 16 x 2 mfma_f32_16x16x32_bf16 per K-step, B fragments (U) straight from global
// / L2 as 16-byte rows. Because a lane's accumulators hold all 16 points of the same (tile, co),
// the output transform runs in registers, followed by the BatchNorm-statistics epilogue (per-
// channel sum / sum of squares, the conv_fwd partial-row layout) and the bf16 stores.
//
// Numerics: V and U are rounded to bf16 (the MFMA operands), M accumulates in fp32; the
// transforms add ~2x the direct conv's rounding error (tests/test_winograd.py pins the bound).
#include "common.h"

#include <algorithm>

namespace pca {

constexpr int kWgTiles = 32;   // output 2x2 tiles per workgroup (GEMM rows)
constexpr int kWgCo = 64;      // output channels per workgroup (4 waves x 16)
constexpr int kWgK = 32;       // input channels per K-step (one MFMA K)
constexpr int kWgLd = 40;      // LDS pitch of a V row in bf16 (32 channels + 8: conflict-free reads)

struct WgGeom {
  int N, H, W, Ci, Co;
  int TH, TW, tiles;           // H / 2, W / 2, N * TH * TW
};

// U[p][co][ci] = (G g G^T)[p] for the fp32 master w[co][kh][kw][ci] (physical channels_last)
__global__ __launch_bounds__(256) void winograd_filter_kernel(const float* __restrict__ w, int Co,
                                                              int Ci, bf16* __restrict__ U) {
  const int total = Co * Ci;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int co = i / Ci, ci = i - co * Ci;
    float g[3][3];
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
      for (int b = 0; b < 3; ++b) g[a][b] = w[((size_t)co * 9 + a * 3 + b) * Ci + ci];
    // t = G g  (4 x 3)
    float t[4][3];
#pragma unroll
    for (int b = 0; b < 3; ++b) {
      t[0][b] = g[0][b];
      t[1][b] = 0.5f * (g[0][b] + g[1][b] + g[2][b]);
      t[2][b] = 0.5f * (g[0][b] - g[1][b] + g[2][b]);
      t[3][b] = g[2][b];
    }
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const float u0 = t[a][0];
      const float u1 = 0.5f * (t[a][0] + t[a][1] + t[a][2]);
      const float u2 = 0.5f * (t[a][0] - t[a][1] + t[a][2]);
      const float u3 = t[a][2];
      const size_t o = (size_t)co * Ci + ci;
      const size_t ps = (size_t)Co * Ci;
      U[(a * 4 + 0) * ps + o] = f2bf(u0);
      U[(a * 4 + 1) * ps + o] = f2bf(u1);
      U[(a * 4 + 2) * ps + o] = f2bf(u2);
      U[(a * 4 + 3) * ps + o] = f2bf(u3);
    }
  }
}

__device__ __forceinline__ void unpack4(const uint2& u, float* f) {
  f[0] = __uint_as_float(u.x << 16);
  f[1] = __uint_as_float(u.x & 0xffff0000u);
  f[2] = __uint_as_float(u.y << 16);
  f[3] = __uint_as_float(u.y & 0xffff0000u);
}

__global__ __launch_bounds__(256) void winograd_fwd_kernel(const bf16* __restrict__ X,
                                                           const bf16* __restrict__ U,
                                                           bf16* __restrict__ Y,
                                                           float* __restrict__ stats, WgGeom g) {
  __shared__ __attribute__((aligned(16))) bf16 Vs[16 * kWgTiles * kWgLd];   // 40 KiB
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tile0 = blockIdx.x * kWgTiles;
  const int co0 = blockIdx.y * kWgCo + wave * 16;

  // ---- transform role: tile t, channels [4 cg, 4 cg + 4) of the K-step ----
  const int t = tid >> 3, cg = tid & 7;
  const int T = tile0 + t;
  const bool tok = T < g.tiles;
  int n = 0, th = 0, tw = 0;
  if (tok) {
    const int per = g.TH * g.TW;
    n = T / per;
    const int r = T - n * per;
    th = r / g.TW;
    tw = r - th * g.TW;
  }
  // patch origin (2 th - 1, 2 tw - 1); bit i*4+j of `valid`: pixel (i, j) inside the image
  const bf16* xb = X + ((size_t)(n * g.H + 2 * th - 1) * g.W + 2 * tw - 1) * g.Ci + cg * 4;
  uint32_t valid = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int h = 2 * th - 1 + i, w = 2 * tw - 1 + j;
      if (tok && (unsigned)h < (unsigned)g.H && (unsigned)w < (unsigned)g.W) valid |= 1u << (i * 4 + j);
    }
  const int rowp = g.W * g.Ci;
  uint2 d[16];
  auto load_patch = [&](int ci0) {
#pragma unroll
    for (int k = 0; k < 16; ++k)
      d[k] = (valid >> k) & 1u
                 ? *reinterpret_cast<const uint2*>(xb + (k >> 2) * rowp + (k & 3) * g.Ci + ci0)
                 : make_uint2(0u, 0u);
  };

  // ---- MFMA role ----
  f32x4 acc[16][2];
#pragma unroll
  for (int p = 0; p < 16; ++p)
#pragma unroll
    for (int h = 0; h < 2; ++h) acc[p][h] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int co_l = co0 + (lane & 15);
  const int kq = 8 * (lane >> 4);
  const size_t ups = (size_t)g.Co * g.Ci;
  const bf16* ub = U + (size_t)co_l * g.Ci + kq;

  load_patch(0);
  for (int ci0 = 0; ci0 < g.Ci; ci0 += kWgK) {
    // input transform V = B^T d B (4 channels), into LDS as bf16
    {
      float v[16][4];
#pragma unroll
      for (int k = 0; k < 16; ++k) unpack4(d[k], v[k]);
      float r[16][4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int c = 0; c < 4; ++c) {   // columns: B^T along i
          const float d0 = v[0 * 4 + j][c], d1 = v[1 * 4 + j][c], d2 = v[2 * 4 + j][c], d3 = v[3 * 4 + j][c];
          r[0 * 4 + j][c] = d0 - d2;
          r[1 * 4 + j][c] = d1 + d2;
          r[2 * 4 + j][c] = d2 - d1;
          r[3 * 4 + j][c] = d1 - d3;
        }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float o[4][4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {   // rows: B along j
          const float e0 = r[i * 4 + 0][c], e1 = r[i * 4 + 1][c], e2 = r[i * 4 + 2][c], e3 = r[i * 4 + 3][c];
          o[0][c] = e0 - e2;
          o[1][c] = e1 + e2;
          o[2][c] = e2 - e1;
          o[3][c] = e1 - e3;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int p = i * 4 + j;
          uint2 pk;
          pk.x = pack2(o[j][0], o[j][1]);
          pk.y = pack2(o[j][2], o[j][3]);
          *reinterpret_cast<uint2*>(Vs + (p * kWgTiles + t) * kWgLd + cg * 4) = pk;
        }
      }
    }
    __syncthreads();
    if (ci0 + kWgK < g.Ci) load_patch(ci0 + kWgK);   // next K-step's patch, under the MFMAs
#pragma unroll
    for (int p = 0; p < 16; ++p) {
      const bf16x8 b = *reinterpret_cast<const bf16x8*>(ub + p * ups + ci0);
      const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(Vs + (p * kWgTiles + (lane & 15)) * kWgLd + kq);
      const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(Vs + (p * kWgTiles + 16 + (lane & 15)) * kWgLd + kq);
      acc[p][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b, acc[p][0], 0, 0, 0);
      acc[p][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, b, acc[p][1], 0, 0, 0);
    }
    __syncthreads();
  }

  // ---- output transform Y = A^T M A per (tile, co) in registers + BN statistics ----
  float ssum = 0.f, ssq = 0.f;
  const bool cok = co_l < g.Co;
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int Tt = tile0 + h * 16 + (lane >> 4) * 4 + r;
      if (Tt >= g.tiles || !cok) continue;
      float s0[4], s1[4];
#pragma unroll
      for (int nu = 0; nu < 4; ++nu) {
        const float m0 = acc[0 * 4 + nu][h][r], m1 = acc[1 * 4 + nu][h][r];
        const float m2 = acc[2 * 4 + nu][h][r], m3 = acc[3 * 4 + nu][h][r];
        s0[nu] = m0 + m1 + m2;
        s1[nu] = m1 - m2 - m3;
      }
      const float y00 = s0[0] + s0[1] + s0[2], y01 = s0[1] - s0[2] - s0[3];
      const float y10 = s1[0] + s1[1] + s1[2], y11 = s1[1] - s1[2] - s1[3];
      const int per = g.TH * g.TW;
      const int nn = Tt / per;
      const int rr = Tt - nn * per;
      const int oh = 2 * (rr / g.TW), ow = 2 * (rr % g.TW);
      bf16* yb = Y + (((size_t)nn * g.H + oh) * g.W + ow) * g.Co + co_l;
      yb[0] = f2bf(y00);
      yb[g.Co] = f2bf(y01);
      yb[(size_t)g.W * g.Co] = f2bf(y10);
      yb[(size_t)g.W * g.Co + g.Co] = f2bf(y11);
      ssum += (y00 + y01) + (y10 + y11);
      ssq += (y00 * y00 + y01 * y01) + (y10 * y10 + y11 * y11);
    }
  if (stats) {
    // lanes l, l+16, l+32, l+48 hold the same channel: fold, then one row per workgroup
    ssum += __shfl_xor(ssum, 16, 64);
    ssq += __shfl_xor(ssq, 16, 64);
    ssum += __shfl_xor(ssum, 32, 64);
    ssq += __shfl_xor(ssq, 32, 64);
    if (lane < 16 && cok) {
      stats[((size_t)blockIdx.x * 2 + 0) * g.Co + co_l] = ssum;
      stats[((size_t)blockIdx.x * 2 + 1) * g.Co + co_l] = ssq;
    }
  }
}

bool winograd_applicable(int N, int H, int W, int Ci, int Co) {
  return N > 0 && H % 2 == 0 && W % 2 == 0 && Ci % kWgK == 0 && Co % kWgCo == 0 &&
         (size_t)N * H * W * std::max(Ci, Co) < (size_t)INT32_MAX;
}

int winograd_stat_rows(int N, int H, int W) {
  return (N * (H / 2) * (W / 2) + kWgTiles - 1) / kWgTiles;
}

void winograd_filter_launch(const float* w, int Co, int Ci, bf16* U, hipStream_t st) {
  const int blocks = std::min((Co * Ci + 255) / 256, 4096);
  hipLaunchKernelGGL(winograd_filter_kernel, dim3(blocks), dim3(256), 0, st, w, Co, Ci, U);
}

void winograd_fwd_launch(const bf16* x, const bf16* U, bf16* y, float* stats, int N, int H, int W,
                         int Ci, int Co, hipStream_t st) {
  WgGeom g{N, H, W, Ci, Co, H / 2, W / 2, N * (H / 2) * (W / 2)};
  const dim3 grid((g.tiles + kWgTiles - 1) / kWgTiles, Co / kWgCo);
  hipLaunchKernelGGL(winograd_fwd_kernel, grid, dim3(256), 0, st, x, U, y, stats, g);
}

}  // namespace pca
