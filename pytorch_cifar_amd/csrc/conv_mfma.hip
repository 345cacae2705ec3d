// Implicit-GEMM convolution on CDNA4 matrix cores (v_mfma_f32_16x16x32_bf16), NHWC bf16.
//
// Replaces the implicit cuDNN kernels behind the reference's nn.Conv2d (SURVEY §2.8 K1-K5:
// models/resnet.py:23-27, 33-34, 61-67; models/regnet.py:37; models/resnext.py:19 ...).
//
//   forward : Y[m, co]      = sum_{tap, ci} X[gather(m, tap), ci] * W[co, tap, ci]
//             GEMM  M = N*OH*OW pixels, N = Cout/G, K = KH*KW*Cin/G
//             epilogue: optional bias, per-channel (sum, sumsq) partials of Y for the
//             training-mode BatchNorm that always follows (one slab row per workgroup).
//   dgrad   : dX[m, ci]     = sum_{tap, co} dY[scatter(m, tap), co] * W[co, tap, ci]
//             same kernel, A = dY, B = W transposed to [Cin][tap][Cout/G]; the gather
//             inverts the stride (taps whose (ih + pad - kh) is not a multiple of the
//             stride read zero).
//   wgrad   : dW[co, tap, ci] = sum_p dY[p, co] * X[gather(p, tap), ci]
//             GEMM with K = pixels (huge): split-K over pixel ranges, both operands staged
//             [pixel][channel] in LDS and read transposed with ds_read_b64_tr_b16, fp32
//             atomics into the gradient (which lives in the flat gradient arena).
//
// Memory pipeline (cdna_hip_programming.md §5 "Pipelining across barriers"): operands are
// staged with LDS-DMA (buffer_load ... lds, 16 B per lane, 1 KiB per wave instruction) into a
// STAGES-deep LDS ring. Out-of-range rows (conv zero padding, M/N/K tails) use an offset past
// the buffer descriptor's size, which the hardware returns as zeros — no branches, no masks.
// Each K-step: counted `s_waitcnt vmcnt(N)` for the oldest stage only, one raw s_barrier,
// issue the stage STAGES-1 ahead, then ds_read + MFMA on the landed stage. No register
// staging (the previous register-staged version spilled its staging arrays to scratch).
// The XOR swizzle of each LDS row is applied on the DMA *source* address (the DMA writes
// lane-linearly) and on the fragment read address (rule 21: both sides or neither).
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

typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, bytes, 0x00020000);
}

// one 16-byte-per-lane LDS-DMA (1 KiB per wave instruction at lds_base + 16*lane)
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rs, char* lds_base, uint32_t voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)lds_base, 16, (int)voff, 0, 0, 0);
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

constexpr uint32_t kOOB = 0x80000000u;  // byte offset past any descriptor range -> zeros

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
  uint32_t a_bytes, b_bytes;
  FastDiv fd_hw, fd_w, fd_cr8, fd_kw, fd_s;
};

// ---------------------------------------------------------------------------------------
// forward / dgrad implicit GEMM
// ---------------------------------------------------------------------------------------
// MODE 0: forward; 1: dgrad (generic gather, any stride); 2: dgrad of a stride-2 conv split
// into its 4 output parity classes (blockIdx.z = group*4 + class): class (ph, pw) only meets
// the taps kh = (ph+pad)&1 (+2...), so no MFMA work is spent on the 3/4 of taps that a strided
// transposed convolution would multiply by zero.
template <int BM, int BN, int WM, int WN, int STAGES, int MODE, bool STATS>
__global__ __launch_bounds__(256) void conv_igemm_kernel(const bf16* __restrict__ A,
                                                         const bf16* __restrict__ B,
                                                         bf16* __restrict__ Y,
                                                         float* __restrict__ stats,
                                                         const float* __restrict__ bias,
                                                         const ConvGeom g) {
  constexpr int BK = 64;                 // K elements per stage: 128-byte LDS rows
  constexpr int RB = BK * 2;
  constexpr int A_BYTES = BM * RB, B_BYTES = BN * RB;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int A_PW = BM / 32;          // DMA instructions (8 rows each) per wave per stage
  constexpr int B_PW = BN / 32;
  constexpr int LPS = A_PW + B_PW;       // loads per stage per lane
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int CST = BN + 8;            // padded bf16 row stride of the staged C tile
  static_assert(WM * WN == 4, "4 waves");
  static_assert(BM % 32 == 0 && BN % 32 == 0, "tile");
  static_assert(STAGES >= 2, "stages");
  static_assert(BM * CST * 2 <= STAGES * STAGE, "C tile must fit the LDS ring");

  __shared__ __attribute__((aligned(16))) char smem[STAGES * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  constexpr bool DGRAD = MODE != 0;
  constexpr bool PARITY = MODE == 2;
  const int grp = PARITY ? (blockIdx.z >> 2) : blockIdx.z;
  const int cls = PARITY ? (blockIdx.z & 3) : 0;
  const int ph = cls >> 1, pw = cls & 1;
  // tap sets: kh = kh0 + tstep*t for t < nth (all taps unless PARITY)
  const int tstep = PARITY ? 2 : 1;
  const int kh0 = PARITY ? ((ph + g.pad) & 1) : 0;
  const int kw0 = PARITY ? ((pw + g.pad) & 1) : 0;
  const int nth = PARITY ? ((g.KH - kh0 + 1) >> 1) : g.KH;
  const int ntw = PARITY ? ((g.KW - kw0 + 1) >> 1) : g.KW;
  const int Kcls = nth * ntw * g.Cr;
  // produced-pixel grid this block walks: the full output, or one parity class of it
  const int rows_h = PARITY ? (g.Ho >> 1) : g.Ho;
  const int rows_w = PARITY ? (g.Wo >> 1) : g.Wo;
  const int Mrows = g.N * rows_h * rows_w;
  const int n0 = blockIdx.y * BN;
  const int mtiles = cdiv(Mrows, BM);
  const int kfull = g.KH * g.KW * g.Cr;   // row length of the B matrix

  const __amdgpu_buffer_rsrc_t rsA = make_rsrc(A, g.a_bytes);
  const __amdgpu_buffer_rsrc_t rsB = make_rsrc(B, g.b_bytes);

  // DMA lane geometry: lane -> (row l>>3 of an 8-row group, physical chunk l&7); it fetches
  // logical chunk (l&7) ^ (row&7) so that the row-swizzled LDS image is written linearly.
  const int lrow = lane >> 3;
  const int lchunk = (lane & 7) ^ lrow;
  const int crg = g.Cr >> 3;
  const int KT = cdiv(Kcls, BK);

  // per-lane BatchNorm partial sums, accumulated over every tile this workgroup owns
  float st_s[TN], st_q[TN];
#pragma unroll
  for (int ni = 0; ni < TN; ++ni) st_s[ni] = st_q[ni] = 0.f;

  // Persistent over M tiles (grid.x <= mtiles): amortises the per-block set-up and bounds the
  // BN statistics slab at grid.x rows.
  for (int tile = blockIdx.x; tile < mtiles; tile += gridDim.x) {
    const int m0 = tile * BM;
    int a_n[A_PW], a_h[A_PW], a_w[A_PW];
#pragma unroll
    for (int i = 0; i < A_PW; ++i) {
      const int r = m0 + (wid * A_PW + i) * 8 + lrow;
      const uint32_t rr = r < Mrows ? r : 0;
      const uint32_t n = fdiv(rr, g.fd_hw);
      const uint32_t rem = rr - n * (rows_h * rows_w);
      const uint32_t h = fdiv(rem, g.fd_w);
      a_n[i] = r < Mrows ? (int)n : -1;
      a_h[i] = PARITY ? (int)(2 * h + ph) : (int)h;
      a_w[i] = PARITY ? (int)(2 * (rem - h * rows_w) + pw) : (int)(rem - h * rows_w);
    }

    auto issue = [&](int kt, int buf) {
      char* As = smem + buf * STAGE;
      char* Bs = As + A_BYTES;
      const int kg = kt * 8 + lchunk;                  // 8-channel granule along K
      const bool kok = kg * 8 < Kcls;
      const int tap = kok ? (int)fdiv(kg, g.fd_cr8) : 0;
      const int c8 = kg - tap * crg;
      int kh, kw;
      if constexpr (PARITY) {
        const int th = tap / ntw;
        kh = kh0 + 2 * th;
        kw = kw0 + 2 * (tap - th * ntw);
      } else {
        kh = (int)fdiv(tap, g.fd_kw);
        kw = tap - kh * g.KW;
      }
      const int kcol = (kh * g.KW + kw) * g.Cr + c8 * 8;   // element column in the B row
#pragma unroll
      for (int i = 0; i < A_PW; ++i) {
        int sh, sw;
        bool ok = kok && a_n[i] >= 0;
        if constexpr (!DGRAD) {
          sh = a_h[i] * g.stride - g.pad + kh;
          sw = a_w[i] * g.stride - g.pad + kw;
        } else if constexpr (PARITY) {
          // (ih + pad - kh) is even by the choice of taps: exact halving, no masking
          sh = (a_h[i] + g.pad - kh) >> 1;
          sw = (a_w[i] + g.pad - kw) >> 1;
        } else {
          const int nh = a_h[i] + g.pad - kh, nw = a_w[i] + g.pad - kw;
          sh = (nh >= 0) ? (int)fdiv(nh, g.fd_s) : -1;
          sw = (nw >= 0) ? (int)fdiv(nw, g.fd_s) : -1;
          ok = ok && (sh * g.stride == nh) && (sw * g.stride == nw);
        }
        ok = ok && sh >= 0 && sh < g.Hs && sw >= 0 && sw < g.Ws;
        const uint32_t off =
            ok ? (uint32_t)(((((a_n[i] * g.Hs + sh) * g.Ws + sw) * g.Cs) + grp * g.Cr + c8 * 8) * 2)
               : kOOB;
        dma16(rsA, As + (wid * A_PW + i) * 1024, off);
      }
#pragma unroll
      for (int i = 0; i < B_PW; ++i) {
        const int br = n0 + (wid * B_PW + i) * 8 + lrow;
        const bool ok = kok && br < g.Cn;
        const uint32_t off = ok ? (uint32_t)((((grp * g.Cn + br) * kfull) + kcol) * 2) : kOOB;
        dma16(rsB, Bs + (wid * B_PW + i) * 1024, off);
      }
    };

    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
    for (int s = 0; s < STAGES - 1; ++s) issue(s, s);

    for (int kt = 0; kt < KT; ++kt) {
      wait_vmcnt<(STAGES - 2) * LPS>();
      raw_barrier();
      issue(kt + STAGES - 1, (kt + STAGES - 1) % STAGES);   // past-the-end stages load zeros
      const char* As = smem + (kt % STAGES) * STAGE;
      const char* Bs = As + A_BYTES;
#pragma unroll
      for (int kk = 0; kk < BK / 32; ++kk) {
        bf16x8 af[TM], bfv[TN];
        const int gsel = kk * 4 + (lane >> 4);
#pragma unroll
        for (int mi = 0; mi < TM; ++mi) {
          const int r = wm * WTM + mi * 16 + (lane & 15);
          af[mi] = *reinterpret_cast<const bf16x8*>(As + r * RB + ((gsel ^ (r & 7)) << 4));
        }
#pragma unroll
        for (int ni = 0; ni < TN; ++ni) {
          const int r = wn * WTN + ni * 16 + (lane & 15);
          bfv[ni] = *reinterpret_cast<const bf16x8*>(Bs + r * RB + ((gsel ^ (r & 7)) << 4));
        }
#pragma unroll
        for (int mi = 0; mi < TM; ++mi)
#pragma unroll
          for (int ni = 0; ni < TN; ++ni)
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mi], bfv[ni], acc[mi][ni], 0, 0, 0);
      }
    }
    wait_vmcnt<0>();
    __syncthreads();

    // ---- epilogue: bias, BN partials, bf16 tile through LDS for 16-byte row stores ----
    if (bias) {
#pragma unroll
      for (int ni = 0; ni < TN; ++ni) {
        const int c = n0 + wn * WTN + ni * 16 + (lane & 15);
        const float b = c < g.Cn ? bias[grp * g.Cn + c] : 0.f;
#pragma unroll
        for (int mi = 0; mi < TM; ++mi)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int r = m0 + wm * WTM + mi * 16 + (lane >> 4) * 4 + j;
            if (r < Mrows) acc[mi][ni][j] += b;
          }
      }
    }
    if constexpr (STATS) {
#pragma unroll
      for (int ni = 0; ni < TN; ++ni)
#pragma unroll
        for (int mi = 0; mi < TM; ++mi)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float v = acc[mi][ni][j];   // rows past M are exact zeros (zero-filled A)
            st_s[ni] += v;
            st_q[ni] += v * v;
          }
    }
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
#pragma unroll
    for (int it = 0; it < (BM * CG) / 256; ++it) {
      const int idx = tid + it * 256;
      const int r = idx / CG, c8 = idx % CG;
      const int gm = m0 + r, gc = n0 + c8 * 8;
      if (gm < Mrows && gc < g.Cn) {
        size_t pix = gm;
        if constexpr (PARITY) {
          const uint32_t n = fdiv(gm, g.fd_hw);
          const uint32_t rem = gm - n * (rows_h * rows_w);
          const uint32_t h = fdiv(rem, g.fd_w);
          const uint32_t w = rem - h * rows_w;
          pix = ((size_t)n * g.Ho + 2 * h + ph) * g.Wo + 2 * w + pw;
        }
        const uint4 v = *reinterpret_cast<const uint4*>(Cs + r * CST + c8 * 8);
        *reinterpret_cast<uint4*>(Y + pix * g.Co + (size_t)grp * g.Cn + gc) = v;
      }
    }
    __syncthreads();   // the C tile aliases the ring the next tile's prologue refills
  }

  if constexpr (STATS) {
    float* red = reinterpret_cast<float*>(smem);  // [WM][BN][2]
#pragma unroll
    for (int ni = 0; ni < TN; ++ni) {
      float s = st_s[ni], q = st_q[ni];
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
  uint32_t x_bytes, dy_bytes;
  FastDiv fd_hw, fd_w, fd_cin8;
};

template <int COLS>
__device__ __forceinline__ bf16x8 tr_frag(const char* base, int k0, int c0, int lane) {
  constexpr int RB = COLS * 2;
  typedef __attribute__((address_space(3))) i16x4 lds_i16x4;
  typedef short i16x8 __attribute__((ext_vector_type(8)));
  const int li = lane & 15;
  const int q = li >> 2, p = li & 3;
  const int col = c0 + 4 * p;
  const int chunk = col >> 3;
  const int r0 = k0 + 8 * (lane >> 4) + q;
  const int r1 = r0 + 4;
  const int b0 = r0 * RB + ((chunk ^ tr_swz<RB>(r0)) << 4) + ((col & 7) << 1);
  const int b1 = r1 * RB + ((chunk ^ tr_swz<RB>(r1)) << 4) + ((col & 7) << 1);
  const i16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(base + b0));
  const i16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(base + b1));
  const i16x8 v = __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, v);
}

template <int BM, int BN, int WM, int WN, int STAGES>
__global__ __launch_bounds__(256) void conv_wgrad_kernel(const bf16* __restrict__ X,
                                                         const bf16* __restrict__ DY,
                                                         float* __restrict__ DW,
                                                         const WgradGeom g) {
  constexpr int BKP = 64;                     // pixels per stage
  constexpr int RA = BM * 2, RBB = BN * 2;    // LDS row bytes
  constexpr int A_BYTES = BKP * RA, B_BYTES = BKP * RBB;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int A_INS = A_BYTES / 1024, B_INS = B_BYTES / 1024;   // DMA instructions per stage
  constexpr int A_PW = A_INS / 4, B_PW = B_INS / 4;
  constexpr int LPS = A_PW + B_PW;
  constexpr int A_RPI = 1024 / RA, B_RPI = 1024 / RBB;            // rows per instruction
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  static_assert(A_PW >= 1 && B_PW >= 1, "tile");
  __shared__ __attribute__((aligned(16))) char smem[STAGES * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int split = blockIdx.z % g.splits;
  const int grp = blockIdx.z / g.splits;
  const int m0 = blockIdx.x * BM;   // output channel (within group)
  const int n0 = blockIdx.y * BN;   // (tap, ci) column
  const int p_begin = split * g.chunk;
  const int p_end = min(g.P, p_begin + g.chunk);

  const __amdgpu_buffer_rsrc_t rsX = make_rsrc(X, g.x_bytes);
  const __amdgpu_buffer_rsrc_t rsD = make_rsrc(DY, g.dy_bytes);

  // lane -> (row within the instruction's rows, physical 16-byte chunk of that row)
  constexpr int ACH = RA / 16, BCH = RBB / 16;
  const int a_lrow = lane / ACH, a_pch = lane % ACH;
  const int b_lrow = lane / BCH, b_pch = lane % BCH;

  auto issue = [&](int pbase, int buf) {
    char* As = smem + buf * STAGE;
    char* Bs = As + A_BYTES;
#pragma unroll
    for (int i = 0; i < A_PW; ++i) {
      const int r = (wid * A_PW + i) * A_RPI + a_lrow;
      const int lch = a_pch ^ tr_swz<RA>(r);
      const int p = pbase + r;
      const int co = m0 + lch * 8;
      const bool ok = p < p_end && co < g.cout_g;
      const uint32_t off = ok ? (uint32_t)((p * g.Cy + grp * g.cout_g + co) * 2) : kOOB;
      dma16(rsD, As + (wid * A_PW + i) * 1024, off);
    }
#pragma unroll
    for (int i = 0; i < B_PW; ++i) {
      const int r = (wid * B_PW + i) * B_RPI + b_lrow;
      const int lch = b_pch ^ tr_swz<RBB>(r);
      const int col = n0 + lch * 8;
      const int p = pbase + r;
      bool ok = p < p_end && col < g.Ktot;
      const uint32_t pp = ok ? p : 0;
      const uint32_t n = fdiv(pp, g.fd_hw);
      const uint32_t rem = pp - n * (g.Ho * g.Wo);
      const uint32_t oh = fdiv(rem, g.fd_w);
      const uint32_t ow = rem - oh * g.Wo;
      const int gran = ok ? (col >> 3) : 0;
      const int tap = (int)fdiv(gran, g.fd_cin8);
      const int c8 = gran - tap * (g.cin_g >> 3);
      const int kh = tap / g.KW, kw = tap - (tap / g.KW) * g.KW;
      const int ih = (int)oh * g.stride - g.pad + kh;
      const int iw = (int)ow * g.stride - g.pad + kw;
      ok = ok && ih >= 0 && ih < g.H && iw >= 0 && iw < g.W;
      const uint32_t off =
          ok ? (uint32_t)(((((int)n * g.H + ih) * g.W + iw) * g.Cx + grp * g.cin_g + c8 * 8) * 2)
             : kOOB;
      dma16(rsX, Bs + (wid * B_PW + i) * 1024, off);
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int KT = p_end > p_begin ? cdiv(p_end - p_begin, BKP) : 0;
#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s) issue(p_begin + s * BKP, s);
  for (int kt = 0; kt < KT; ++kt) {
    wait_vmcnt<(STAGES - 2) * LPS>();
    raw_barrier();
    issue(p_begin + (kt + STAGES - 1) * BKP, (kt + STAGES - 1) % STAGES);
    const char* As = smem + (kt % STAGES) * STAGE;
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
  }
  wait_vmcnt<0>();

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

// ---------------------------------------------------------------------------------------
// host launchers
// ---------------------------------------------------------------------------------------
static ConvGeom make_geom(int N, int Hs, int Ws, int Cs, int Ho, int Wo, int Co, int KH, int KW,
                          int stride, int pad, int groups, int Cr, int Cn) {
  ConvGeom g;
  g.N = N; g.Hs = Hs; g.Ws = Ws; g.Cs = Cs;
  g.Ho = Ho; g.Wo = Wo; g.Co = Co;
  g.KH = KH; g.KW = KW; g.stride = stride; g.pad = pad;
  g.groups = groups; g.Cr = Cr; g.Cn = Cn;
  g.M = N * Ho * Wo;
  g.Ktot = KH * KW * Cr;
  g.a_bytes = (uint32_t)((size_t)N * Hs * Ws * Cs * 2);
  g.b_bytes = (uint32_t)((size_t)groups * Cn * g.Ktot * 2);
  g.fd_hw = make_fastdiv(Ho * Wo);
  g.fd_w = make_fastdiv(Wo);
  g.fd_cr8 = make_fastdiv(Cr / 8);
  g.fd_kw = make_fastdiv(KW);
  g.fd_s = make_fastdiv(stride);
  return g;
}

// persistent grid: at most kMaxTilesX workgroups along M (also the BN slab row count)
constexpr int kMaxTilesX = 1024;
static int igemm_grid_x(int M, int BM) { return std::min(cdiv(M, BM), kMaxTilesX); }

template <int BM, int BN, int WM, int WN, int ST, int MODE>
static void launch_igemm(const bf16* A, const bf16* B, bf16* Y, float* stats, const float* bias,
                         const ConvGeom& g, hipStream_t st) {
  const int rows = MODE == 2 ? g.N * (g.Ho / 2) * (g.Wo / 2) : g.M;
  dim3 grid(igemm_grid_x(rows, BM), cdiv(g.Cn, BN), g.groups * (MODE == 2 ? 4 : 1));
  if (stats)
    hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, ST, MODE, true>), grid, dim3(256), 0, st,
                       A, B, Y, stats, bias, g);
  else
    hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, ST, MODE, false>), grid, dim3(256), 0, st,
                       A, B, Y, stats, bias, g);
}

// Tile configurations. The heuristic picks by GEMM N (channels per group); a process-wide
// override (set_conv_tile) lets tools/bench_conv.py sweep them on the GPU.
static int g_igemm_override = -1;
static int g_wgrad_override = -1;

void set_conv_tile(int kind, int idx) {
  if (kind == 0) g_igemm_override = idx;
  else g_wgrad_override = idx;
}

static int igemm_select(const ConvGeom& g) {
  if (g_igemm_override >= 0) return g_igemm_override;
  // measured on MI355X (tools/bench_conv.py, profiles/conv_sweep_r1.md): two-stage rings at
  // 2-3 workgroups/CU beat deeper rings at one workgroup/CU on every ResNet-18 shape.
  if (g.Cn > 64) return 3;
  if (g.Cn > 32) return 4;
  return 8;
}

static int igemm_bm(int cfg) { return cfg == 6 || cfg == 7 ? 256 : 128; }

template <int MODE>
static void igemm_dispatch(const bf16* A, const bf16* B, bf16* Y, float* stats, const float* bias,
                           const ConvGeom& g, hipStream_t st) {
  switch (igemm_select(g)) {
    case 0: launch_igemm<128, 128, 2, 2, 3, MODE>(A, B, Y, stats, bias, g, st); break;
    case 1: launch_igemm<128, 64, 2, 2, 4, MODE>(A, B, Y, stats, bias, g, st); break;
    case 2: launch_igemm<128, 32, 4, 1, 4, MODE>(A, B, Y, stats, bias, g, st); break;
    case 3: launch_igemm<128, 128, 2, 2, 2, MODE>(A, B, Y, stats, bias, g, st); break;
    case 4: launch_igemm<128, 64, 2, 2, 2, MODE>(A, B, Y, stats, bias, g, st); break;
    case 5: launch_igemm<128, 64, 4, 1, 3, MODE>(A, B, Y, stats, bias, g, st); break;
    case 6: launch_igemm<256, 64, 4, 1, 3, MODE>(A, B, Y, stats, bias, g, st); break;
    case 7: launch_igemm<256, 128, 2, 2, 2, MODE>(A, B, Y, stats, bias, g, st); break;
    case 8: launch_igemm<128, 32, 4, 1, 2, MODE>(A, B, Y, stats, bias, g, st); break;
    default: launch_igemm<128, 128, 2, 2, 3, MODE>(A, B, Y, stats, bias, g, st); break;
  }
}

// number of BN-statistics slab rows the forward launch will write (= grid.x)
int conv_fwd_stat_rows(int M, int Cout, int groups) {
  ConvGeom g;
  g.Cn = Cout / groups;
  g.M = M;
  return igemm_grid_x(M, igemm_bm(igemm_select(g)));
}

void conv_fwd_launch(const bf16* x, const bf16* w, const float* bias, bf16* y, float* stats, int N,
                     int H, int W, int Cin, int Cout, int KH, int KW, int stride, int pad,
                     int groups, int Ho, int Wo, hipStream_t st) {
  ConvGeom g = make_geom(N, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, groups, Cin / groups,
                         Cout / groups);
  igemm_dispatch<0>(x, w, y, stats, bias, g, st);
}

// dx = conv^T(dy, W); wt is W transposed to [Cin][KH][KW][Cout/G].
void conv_dgrad_launch(const bf16* dy, const bf16* wt, bf16* dx, int N, int H, int W, int Cin,
                       int Cout, int KH, int KW, int stride, int pad, int groups, int Ho, int Wo,
                       hipStream_t st) {
  ConvGeom g = make_geom(N, Ho, Wo, Cout, H, W, Cin, KH, KW, stride, pad, groups, Cout / groups,
                         Cin / groups);
  if (stride == 2 && H % 2 == 0 && W % 2 == 0 && Ho == H / 2 && Wo == W / 2) {
    // parity-class decomposition: rows are one class's (H/2) x (W/2) pixels
    g.fd_hw = make_fastdiv((H / 2) * (W / 2));
    g.fd_w = make_fastdiv(W / 2);
    igemm_dispatch<2>(dy, wt, dx, nullptr, nullptr, g, st);
  } else {
    igemm_dispatch<1>(dy, wt, dx, nullptr, nullptr, g, st);
  }
}

template <int BM, int BN, int WM, int WN, int ST>
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
  hipLaunchKernelGGL((conv_wgrad_kernel<BM, BN, WM, WN, ST>), grid, dim3(256), 0, st, x, dy, dw, g);
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
  g.x_bytes = (uint32_t)((size_t)N * H * W * Cin * 2);
  g.dy_bytes = (uint32_t)((size_t)N * Ho * Wo * Cout * 2);
  g.fd_hw = make_fastdiv(Ho * Wo);
  g.fd_w = make_fastdiv(Wo);
  g.fd_cin8 = make_fastdiv(g.cin_g / 8);
  const int target = 1024;
  int cfg = g_wgrad_override;
  if (cfg < 0) cfg = (g.cout_g > 64 && g.Ktot > 64) ? 3 : (g.cout_g > 32 ? 6 : 7);
  switch (cfg) {
    case 0: launch_wgrad<128, 128, 2, 2, 3>(x, dy, dw, g, st, target); break;
    case 1: launch_wgrad<64, 128, 2, 2, 3>(x, dy, dw, g, st, target); break;
    case 2: launch_wgrad<32, 128, 1, 4, 3>(x, dy, dw, g, st, target); break;
    case 3: launch_wgrad<128, 128, 2, 2, 2>(x, dy, dw, g, st, target); break;
    case 4: launch_wgrad<128, 128, 2, 2, 3>(x, dy, dw, g, st, 2048); break;
    case 5: launch_wgrad<128, 128, 2, 2, 3>(x, dy, dw, g, st, 512); break;
    case 6: launch_wgrad<64, 128, 2, 2, 2>(x, dy, dw, g, st, target); break;
    case 7: launch_wgrad<32, 128, 1, 4, 2>(x, dy, dw, g, st, target); break;
    default: launch_wgrad<128, 128, 2, 2, 3>(x, dy, dw, g, st, target); break;
  }
}

}  // namespace pca
