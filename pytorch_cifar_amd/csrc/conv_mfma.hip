// Implicit-GEMM convolution on CDNA4 matrix cores (v_mfma_f32_16x16x32_bf16), NHWC bf16.
//
// Replaces the implicit cuDNN kernels behind the reference's nn.Conv2d (SURVEY §2.8 K1-K5:
// models/resnet.py:23-27, 33-34, 61-67; models/regnet.py:37; models/resnext.py:19 ...).
//
//   forward : Y[m, co]      = sum_{tap, ci} X[gather(m, tap), ci] * W[co, tap, ci]
//             GEMM  M = N*OH*OW pixels, N = Cout/G, K = KH*KW*Cin/G
//             epilogue optionally emits per-channel (sum, sumsq) partials of Y for the
//             training-mode BatchNorm that always follows (one slab row per M-tile).
//   dgrad   : dX[m, ci]     = sum_{tap, co} dY[scatter(m, tap), co] * W[co, tap, ci]
//             same kernel, A = dY, B = W transposed to [Cin][tap][Cout/G]; the gather
//             inverts the stride (taps whose (ih + pad - kh) is not a multiple of the
//             stride read zero).
//   wgrad   : dW[co, tap, ci] = sum_p dY[p, co] * X[gather(p, tap), ci]
//             GEMM with K = pixels (huge): split-K over pixel ranges, both operands staged
//             [pixel][channel] in LDS and read transposed with ds_read_b64_tr_b16, fp32
//             atomics into the (zeroed) fp32 gradient.
//
// Tiles are sized for CIFAR shapes (32x32 and smaller maps): 256-thread workgroups = 4 waves
// of 64 lanes, register-staged double-buffered LDS (one barrier per K-step), XOR-swizzled
// 16-byte chunks so the ds_read_b128 fragment reads are conflict-free.
#include "common.h"

#include <algorithm>

namespace pca {

// Exact unsigned division by a runtime constant (n < 2^31): q = (umulhi(n, m) + n) >> s.
struct FastDiv {
  uint32_t d, m, s;
};

static inline FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  f.d = d;
  uint32_t s = 0;
  while ((1ull << s) < d) ++s;
  f.s = s;
  f.m = (uint32_t)(((1ull << 32) * ((1ull << s) - d)) / d + 1);
  return f;
}

__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
  const uint64_t t = (uint64_t)__umulhi(n, f.m) + n;
  return (uint32_t)(t >> f.s);
}

struct ConvGeom {
  int N;                // batch
  int Hs, Ws, Cs;       // gathered (A-side) tensor dims, NHWC; Cs = its total channels
  int Ho, Wo, Co;       // produced tensor dims; Co = its total channels
  int KH, KW, stride, pad;
  int groups;
  int Cr;               // reduction channels per group (A side)
  int Cn;               // produced channels per group (GEMM N)
  int M;                // N*Ho*Wo
  int Ktot;             // KH*KW*Cr
  FastDiv fd_hw, fd_w, fd_cr8, fd_kw, fd_s;
};

// 16-byte chunk swizzle for an LDS row of RB bytes, used by the fragment (row) reads.
template <int RB>
__device__ __forceinline__ int row_swz(int r) {
  if constexpr (RB >= 128) return r & 7;
  else return (r >> 1) & 3;
}

// ---------------------------------------------------------------------------------------
// forward / dgrad implicit GEMM
// ---------------------------------------------------------------------------------------
template <int BM, int BN, int WM, int WN, bool DGRAD, bool STATS>
__global__ __launch_bounds__(256, 2) void conv_igemm_kernel(const bf16* __restrict__ A,
                                                            const bf16* __restrict__ B,
                                                            bf16* __restrict__ Y,
                                                            float* __restrict__ stats,
                                                            const float* __restrict__ bias,
                                                            const ConvGeom g) {
  constexpr int BK = 64;            // bf16 elements of K per stage (= 128 B rows)
  constexpr int NT = 256;
  constexpr int GR = BK / 8;        // 16-byte granules per row
  constexpr int RPI = NT / GR;      // rows covered per load pass (32)
  constexpr int A_IT = BM / RPI;
  constexpr int B_IT = BN / RPI;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  constexpr int STAGE = A_BYTES + B_BYTES;
  static_assert(WM * WN == 4, "4 waves");
  static_assert(A_IT >= 1 && B_IT >= 1, "tile too small");

  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int grp = blockIdx.z;
  const int m0 = blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;
  const int cg = tid & (GR - 1);
  const int rb = tid / GR;

  // Per-thread A rows: decompose the produced pixel index once.
  int a_n[A_IT], a_h[A_IT], a_w[A_IT];
  bool a_ok[A_IT];
#pragma unroll
  for (int i = 0; i < A_IT; ++i) {
    const int r = m0 + rb + i * RPI;
    a_ok[i] = r < g.M;
    const uint32_t rr = a_ok[i] ? r : 0;
    const uint32_t n = fdiv(rr, g.fd_hw);
    const uint32_t rem = rr - n * (g.Ho * g.Wo);
    const uint32_t h = fdiv(rem, g.fd_w);
    a_n[i] = n;
    a_h[i] = h;
    a_w[i] = rem - h * g.Wo;
  }

  const int KT = cdiv(g.Ktot, BK);
  uint4 ra[A_IT], rbv[B_IT];
  const uint4 zero4 = make_uint4(0, 0, 0, 0);
  const size_t a_cbase = (size_t)grp * g.Cr;
  const size_t b_rbase = (size_t)grp * g.Cn;

  auto load_tiles = [&](int kt) {
    const int kg = kt * GR + cg;          // global 8-channel granule index along K
    const bool kok = kg * 8 < g.Ktot;
    const int tap = kok ? (int)fdiv(kg, g.fd_cr8) : 0;
    const int c8 = kg - tap * (g.Cr >> 3);
    const int kh = (int)fdiv(tap, g.fd_kw);
    const int kw = tap - kh * g.KW;
#pragma unroll
    for (int i = 0; i < A_IT; ++i) {
      int sh, sw;
      bool ok = a_ok[i] && kok;
      if constexpr (!DGRAD) {
        sh = a_h[i] * g.stride - g.pad + kh;
        sw = a_w[i] * g.stride - g.pad + kw;
      } else {
        const int nh = a_h[i] + g.pad - kh, nw = a_w[i] + g.pad - kw;
        if (g.stride == 1) {
          sh = nh;
          sw = nw;
        } else {
          sh = (nh >= 0) ? (int)fdiv(nh, g.fd_s) : -1;
          sw = (nw >= 0) ? (int)fdiv(nw, g.fd_s) : -1;
          ok = ok && (sh * g.stride == nh) && (sw * g.stride == nw);
        }
      }
      ok = ok && sh >= 0 && sh < g.Hs && sw >= 0 && sw < g.Ws;
      if (ok) {
        const size_t off = (((size_t)a_n[i] * g.Hs + sh) * g.Ws + sw) * g.Cs + a_cbase + c8 * 8;
        ra[i] = *reinterpret_cast<const uint4*>(A + off);
      } else {
        ra[i] = zero4;
      }
    }
#pragma unroll
    for (int i = 0; i < B_IT; ++i) {
      const int br = n0 + rb + i * RPI;
      if (kok && br < g.Cn) {
        rbv[i] = *reinterpret_cast<const uint4*>(B + (b_rbase + br) * g.Ktot + (size_t)kg * 8);
      } else {
        rbv[i] = zero4;
      }
    }
  };

  auto store_tiles = [&](int buf) {
    char* As = smem + buf * STAGE;
    char* Bs = As + A_BYTES;
#pragma unroll
    for (int i = 0; i < A_IT; ++i) {
      const int r = rb + i * RPI;
      *reinterpret_cast<uint4*>(As + r * (BK * 2) + ((cg ^ row_swz<BK * 2>(r)) << 4)) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < B_IT; ++i) {
      const int r = rb + i * RPI;
      *reinterpret_cast<uint4*>(Bs + r * (BK * 2) + ((cg ^ row_swz<BK * 2>(r)) << 4)) = rbv[i];
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int buf) {
    const char* As = smem + buf * STAGE;
    const char* Bs = As + A_BYTES;
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      bf16x8 af[TM], bfv[TN];
      const int gsel = kk * 4 + (lane >> 4);
#pragma unroll
      for (int mi = 0; mi < TM; ++mi) {
        const int r = wm * WTM + mi * 16 + (lane & 15);
        af[mi] = *reinterpret_cast<const bf16x8*>(As + r * (BK * 2) + ((gsel ^ row_swz<BK * 2>(r)) << 4));
      }
#pragma unroll
      for (int ni = 0; ni < TN; ++ni) {
        const int r = wn * WTN + ni * 16 + (lane & 15);
        bfv[ni] = *reinterpret_cast<const bf16x8*>(Bs + r * (BK * 2) + ((gsel ^ row_swz<BK * 2>(r)) << 4));
      }
#pragma unroll
      for (int mi = 0; mi < TM; ++mi)
#pragma unroll
        for (int ni = 0; ni < TN; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mi], bfv[ni], acc[mi][ni], 0, 0, 0);
    }
  };

  load_tiles(0);
  store_tiles(0);
  __syncthreads();
  for (int kt = 0; kt < KT; ++kt) {
    const bool more = kt + 1 < KT;
    if (more) load_tiles(kt + 1);
    compute(kt & 1);
    if (more) store_tiles((kt + 1) & 1);
    __syncthreads();
  }

  // ---- epilogue: bias, per-channel BN partials, then bf16 tile through LDS for 16-B stores ----
  if (bias) {
#pragma unroll
    for (int ni = 0; ni < TN; ++ni) {
      const int c = n0 + wn * WTN + ni * 16 + (lane & 15);
      const float b = c < g.Cn ? bias[grp * g.Cn + c] : 0.f;
#pragma unroll
      for (int mi = 0; mi < TM; ++mi) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int r = m0 + wm * WTM + mi * 16 + (lane >> 4) * 4 + j;
          if (r < g.M) acc[mi][ni][j] += b;
        }
      }
    }
  }
  if constexpr (STATS) {
    float* red = reinterpret_cast<float*>(smem);  // [WM][BN][2]
#pragma unroll
    for (int ni = 0; ni < TN; ++ni) {
      float s = 0.f, q = 0.f;
#pragma unroll
      for (int mi = 0; mi < TM; ++mi)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float v = acc[mi][ni][j];
          s += v;
          q += v * v;
        }
      s += __shfl_xor(s, 16, 64);
      s += __shfl_xor(s, 32, 64);
      q += __shfl_xor(q, 16, 64);
      q += __shfl_xor(q, 32, 64);
      if (lane < 16) {
        const int c = wn * WTN + ni * 16 + lane;
        red[(wm * BN + c) * 2 + 0] = s;
        red[(wm * BN + c) * 2 + 1] = q;
      }
    }
    __syncthreads();
    if (tid < BN) {
      float s = 0.f, q = 0.f;
#pragma unroll
      for (int w = 0; w < WM; ++w) {
        s += red[(w * BN + tid) * 2 + 0];
        q += red[(w * BN + tid) * 2 + 1];
      }
      const int c = n0 + tid;
      if (c < g.Cn) {
        float* srow = stats + (size_t)blockIdx.x * 2 * g.Co;
        srow[grp * g.Cn + c] = s;
        srow[g.Co + grp * g.Cn + c] = q;
      }
    }
    __syncthreads();
  }

  constexpr int CST = BN + 8;  // padded bf16 row stride of the C tile
  bf16* Cs = reinterpret_cast<bf16*>(smem);
#pragma unroll
  for (int mi = 0; mi < TM; ++mi)
#pragma unroll
    for (int ni = 0; ni < TN; ++ni)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int r = wm * WTM + mi * 16 + (lane >> 4) * 4 + j;
        const int c = wn * WTN + ni * 16 + (lane & 15);
        Cs[r * CST + c] = f2bf(acc[mi][ni][j]);
      }
  __syncthreads();
  constexpr int CG = BN / 8;
  for (int idx = tid; idx < BM * CG; idx += NT) {
    const int r = idx / CG, c8 = idx % CG;
    const int gm = m0 + r, gc = n0 + c8 * 8;
    if (gm < g.M && gc < g.Cn) {
      const uint4 v = *reinterpret_cast<const uint4*>(Cs + r * CST + c8 * 8);
      *reinterpret_cast<uint4*>(Y + (size_t)gm * g.Co + (size_t)grp * g.Cn + gc) = v;
    }
  }
}

// ---------------------------------------------------------------------------------------
// wgrad: split-K GEMM over pixels with transposed LDS reads
// ---------------------------------------------------------------------------------------
// LDS image of a [BKP pixel][COLS channel] tile: 16-byte chunk c of pixel-row r lives at
// r*RB + 16*(c ^ tr_swz(r)). The XOR spreads the 8 rows one ds_read_b64_tr_b16 half-wave
// touches (rows k0..k0+3 and k0+8..k0+11) over all 64 banks.
template <int RB>
__device__ __forceinline__ int tr_swz(int r) {
  if constexpr (RB == 256) return 2 * ((r & 3) | (((r >> 3) & 1) << 2));
  else if constexpr (RB == 128) return 2 * (((r >> 1) & 1) | (((r >> 3) & 1) << 1));
  else return 2 * ((r >> 3) & 1);
}

struct WgradGeom {
  int N, H, W, Cx;       // input X dims (NHWC), Cx total channels
  int Ho, Wo, Cy;        // dY dims, Cy total channels
  int KH, KW, stride, pad;
  int groups;
  int cin_g, cout_g;
  int P;                 // N*Ho*Wo
  int Ktot;              // KH*KW*cin_g (GEMM N)
  int chunk;             // pixels per split
  int splits;
  FastDiv fd_hw, fd_w, fd_cin8;
};

template <int COLS>
__device__ __forceinline__ bf16x8 tr_frag(const char* base, int k0, int c0, int lane) {
  constexpr int RB = COLS * 2;
  const int li = lane & 15;
  const int q = li >> 2, p = li & 3;
  const int col = c0 + 4 * p;
  bf16x8 out;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int r = k0 + 8 * (lane >> 4) + 4 * h + q;
    const int chunk = col >> 3;
    const int byte = r * RB + ((chunk ^ tr_swz<RB>(r)) << 4) + ((col & 7) << 1);
    typedef __attribute__((address_space(3))) i16x4 lds_i16x4;
    i16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(base + byte));
#pragma unroll
    for (int e = 0; e < 4; ++e) out[4 * h + e] = __builtin_bit_cast(bf16, v[e]);
  }
  return out;
}

template <int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(256, 2) void conv_wgrad_kernel(const bf16* __restrict__ X,
                                                            const bf16* __restrict__ DY,
                                                            float* __restrict__ DW,
                                                            const WgradGeom g) {
  constexpr int BKP = 64;   // pixels per stage
  constexpr int NT = 256;
  constexpr int AGR = BM / 8, BGR = BN / 8;
  constexpr int A_IT = BKP * AGR / NT, B_IT = BKP * BGR / NT;
  constexpr int A_BYTES = BKP * BM * 2, B_BYTES = BKP * BN * 2;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  static_assert(A_IT >= 1 && B_IT >= 1, "tile");
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int split = blockIdx.z % g.splits;
  const int grp = blockIdx.z / g.splits;
  const int m0 = blockIdx.x * BM;   // output channel (within group)
  const int n0 = blockIdx.y * BN;   // (tap, ci) column
  const int p_begin = split * g.chunk;
  const int p_end = min(g.P, p_begin + g.chunk);

  // A loads: [pixel][co] granules; thread covers fixed channel granule, rows step NT/AGR.
  const int a_cg = tid % AGR, a_r0 = tid / AGR;
  constexpr int A_RS = NT / AGR;
  const int a_co = m0 + a_cg * 8;
  const bool a_cok = a_co < g.cout_g;
  // B loads: fixed column granule -> (tap, ci8).
  const int b_cg = tid % BGR, b_r0 = tid / BGR;
  constexpr int B_RS = NT / BGR;
  const int b_col = n0 + b_cg * 8;
  const bool b_cok = b_col < g.Ktot;
  const int b_tap = b_cok ? (int)fdiv(b_col >> 3, g.fd_cin8) : 0;
  const int b_c8 = (b_col >> 3) - b_tap * (g.cin_g >> 3);
  const int b_kh = b_tap / g.KW, b_kw = b_tap - b_kh * g.KW;

  uint4 ra[A_IT], rbv[B_IT];
  const uint4 zero4 = make_uint4(0, 0, 0, 0);

  auto load_tiles = [&](int pbase) {
#pragma unroll
    for (int i = 0; i < A_IT; ++i) {
      const int p = pbase + a_r0 + i * A_RS;
      if (a_cok && p < p_end)
        ra[i] = *reinterpret_cast<const uint4*>(DY + (size_t)p * g.Cy + (size_t)grp * g.cout_g + a_co);
      else
        ra[i] = zero4;
    }
#pragma unroll
    for (int i = 0; i < B_IT; ++i) {
      const int p = pbase + b_r0 + i * B_RS;
      bool ok = b_cok && p < p_end;
      const uint32_t pp = ok ? p : 0;
      const uint32_t n = fdiv(pp, g.fd_hw);
      const uint32_t rem = pp - n * (g.Ho * g.Wo);
      const uint32_t oh = fdiv(rem, g.fd_w);
      const uint32_t ow = rem - oh * g.Wo;
      const int ih = (int)oh * g.stride - g.pad + b_kh;
      const int iw = (int)ow * g.stride - g.pad + b_kw;
      ok = ok && ih >= 0 && ih < g.H && iw >= 0 && iw < g.W;
      if (ok)
        rbv[i] = *reinterpret_cast<const uint4*>(
            X + (((size_t)n * g.H + ih) * g.W + iw) * g.Cx + (size_t)grp * g.cin_g + b_c8 * 8);
      else
        rbv[i] = zero4;
    }
  };
  auto store_tiles = [&](int buf) {
    char* As = smem + buf * STAGE;
    char* Bs = As + A_BYTES;
#pragma unroll
    for (int i = 0; i < A_IT; ++i) {
      const int r = a_r0 + i * A_RS;
      *reinterpret_cast<uint4*>(As + r * (BM * 2) + ((a_cg ^ tr_swz<BM * 2>(r)) << 4)) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < B_IT; ++i) {
      const int r = b_r0 + i * B_RS;
      *reinterpret_cast<uint4*>(Bs + r * (BN * 2) + ((b_cg ^ tr_swz<BN * 2>(r)) << 4)) = rbv[i];
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int buf) {
    const char* As = smem + buf * STAGE;
    const char* Bs = As + A_BYTES;
#pragma unroll
    for (int kk = 0; kk < BKP / 32; ++kk) {
      bf16x8 af[TM], bfv[TN];
#pragma unroll
      for (int mi = 0; mi < TM; ++mi) af[mi] = tr_frag<BM>(As, kk * 32, wm * WTM + mi * 16, lane);
#pragma unroll
      for (int ni = 0; ni < TN; ++ni) bfv[ni] = tr_frag<BN>(Bs, kk * 32, wn * WTN + ni * 16, lane);
#pragma unroll
      for (int mi = 0; mi < TM; ++mi)
#pragma unroll
        for (int ni = 0; ni < TN; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mi], bfv[ni], acc[mi][ni], 0, 0, 0);
    }
  };

  if (p_begin < p_end) {
    load_tiles(p_begin);
    store_tiles(0);
    __syncthreads();
    int buf = 0;
    for (int pb = p_begin; pb < p_end; pb += BKP) {
      const bool more = pb + BKP < p_end;
      if (more) load_tiles(pb + BKP);
      compute(buf);
      if (more) store_tiles(buf ^ 1);
      __syncthreads();
      buf ^= 1;
    }
  }

  // fp32 atomics into DW[grp*cout_g + m][Ktot]
#pragma unroll
  for (int mi = 0; mi < TM; ++mi)
#pragma unroll
    for (int ni = 0; ni < TN; ++ni)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = m0 + wm * WTM + mi * 16 + (lane >> 4) * 4 + j;
        const int n = n0 + wn * WTN + ni * 16 + (lane & 15);
        if (m < g.cout_g && n < g.Ktot)
          atomicAdd(DW + ((size_t)grp * g.cout_g + m) * g.Ktot + n, acc[mi][ni][j]);
      }
}

}  // namespace pca

// ---------------------------------------------------------------------------------------
// host launchers
// ---------------------------------------------------------------------------------------
namespace pca {

static ConvGeom make_geom(int N, int Hs, int Ws, int Cs, int Ho, int Wo, int Co, int KH, int KW,
                          int stride, int pad, int groups, int Cr, int Cn) {
  ConvGeom g;
  g.N = N; g.Hs = Hs; g.Ws = Ws; g.Cs = Cs;
  g.Ho = Ho; g.Wo = Wo; g.Co = Co;
  g.KH = KH; g.KW = KW; g.stride = stride; g.pad = pad;
  g.groups = groups; g.Cr = Cr; g.Cn = Cn;
  g.M = N * Ho * Wo;
  g.Ktot = KH * KW * Cr;
  g.fd_hw = make_fastdiv(Ho * Wo);
  g.fd_w = make_fastdiv(Wo);
  g.fd_cr8 = make_fastdiv(Cr / 8);
  g.fd_kw = make_fastdiv(KW);
  g.fd_s = make_fastdiv(stride);
  return g;
}

template <int BM, int BN, int WM, int WN, bool DGRAD>
static void launch_igemm(const bf16* A, const bf16* B, bf16* Y, float* stats, const float* bias,
                         const ConvGeom& g, hipStream_t st) {
  dim3 grid(cdiv(g.M, BM), cdiv(g.Cn, BN), g.groups);
  if (stats)
    hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, DGRAD, true>), grid, dim3(256), 0, st,
                       A, B, Y, stats, bias, g);
  else
    hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, DGRAD, false>), grid, dim3(256), 0, st,
                       A, B, Y, stats, bias, g);
}

// Tile choice keyed on the GEMM N (channels per group) and M.
template <bool DGRAD>
static int igemm_dispatch(const bf16* A, const bf16* B, bf16* Y, float* stats, const float* bias,
                          const ConvGeom& g, hipStream_t st) {
  if (g.Cn > 64) {
    launch_igemm<128, 128, 2, 2, DGRAD>(A, B, Y, stats, bias, g, st);
  } else if (g.Cn > 32) {
    launch_igemm<128, 64, 2, 2, DGRAD>(A, B, Y, stats, bias, g, st);
  } else {
    launch_igemm<128, 32, 4, 1, DGRAD>(A, B, Y, stats, bias, g, st);
  }
  return 128;
}

int conv_fwd_bm() { return 128; }

void conv_fwd_launch(const bf16* x, const bf16* w, const float* bias, bf16* y, float* stats, int N, int H, int W,
                     int Cin, int Cout, int KH, int KW, int stride, int pad, int groups, int Ho,
                     int Wo, hipStream_t st) {
  ConvGeom g = make_geom(N, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, groups, Cin / groups,
                         Cout / groups);
  igemm_dispatch<false>(x, w, y, stats, bias, g, st);
}

// dx = conv^T(dy, W); wt is W transposed to [Cin][KH][KW][Cout/G].
void conv_dgrad_launch(const bf16* dy, const bf16* wt, bf16* dx, int N, int H, int W, int Cin,
                       int Cout, int KH, int KW, int stride, int pad, int groups, int Ho, int Wo,
                       hipStream_t st) {
  ConvGeom g = make_geom(N, Ho, Wo, Cout, H, W, Cin, KH, KW, stride, pad, groups, Cout / groups,
                         Cin / groups);
  igemm_dispatch<true>(dy, wt, dx, nullptr, nullptr, g, st);
}

template <int BM, int BN, int WM, int WN>
static void launch_wgrad(const bf16* x, const bf16* dy, float* dw, WgradGeom g, hipStream_t st,
                         int target_blocks) {
  const int tiles = cdiv(g.cout_g, BM) * cdiv(g.Ktot, BN) * g.groups;
  int splits = cdiv(target_blocks, tiles);
  const int min_chunk = 512;
  splits = std::max(1, std::min(splits, cdiv(g.P, min_chunk)));
  int chunk = cdiv(g.P, splits);
  chunk = cdiv(chunk, 64) * 64;
  splits = cdiv(g.P, chunk);
  g.chunk = chunk;
  g.splits = splits;
  dim3 grid(cdiv(g.cout_g, BM), cdiv(g.Ktot, BN), splits * g.groups);
  hipLaunchKernelGGL((conv_wgrad_kernel<BM, BN, WM, WN>), grid, dim3(256), 0, st, x, dy, dw, g);
}

void conv_wgrad_launch(const bf16* x, const bf16* dy, float* dw, int N, int H, int W, int Cin,
                       int Cout, int KH, int KW, int stride, int pad, int groups, int Ho, int Wo,
                       hipStream_t st) {
  WgradGeom g;
  g.N = N; g.H = H; g.W = W; g.Cx = Cin;
  g.Ho = Ho; g.Wo = Wo; g.Cy = Cout;
  g.KH = KH; g.KW = KW; g.stride = stride; g.pad = pad;
  g.groups = groups; g.cin_g = Cin / groups; g.cout_g = Cout / groups;
  g.P = N * Ho * Wo;
  g.Ktot = KH * KW * g.cin_g;
  g.fd_hw = make_fastdiv(Ho * Wo);
  g.fd_w = make_fastdiv(Wo);
  g.fd_cin8 = make_fastdiv(g.cin_g / 8);
  const int target = 1024;
  if (g.cout_g > 64 && g.Ktot > 64)
    launch_wgrad<128, 128, 2, 2>(x, dy, dw, g, st, target);
  else if (g.cout_g > 32)
    launch_wgrad<64, 128, 2, 2>(x, dy, dw, g, st, target);
  else
    launch_wgrad<32, 128, 1, 4>(x, dy, dw, g, st, target);
}

}  // namespace pca
