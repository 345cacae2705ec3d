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
#include "mfma_util.h"

#include <algorithm>
#include <map>
#include <type_traits>
#include <vector>

#ifndef PCA_IGEMM_DMA_SPREAD
#define PCA_IGEMM_DMA_SPREAD 0
#endif
// rows per thread whose epilogue operands are loaded together (store-loop chunk). 1: the
// operands of a row go out together (the per-operand waits are gone); 2 and 4 hold more rows'
// operands at once and spilled the 256x128 dgrad (2 and 4: 7 and 38 VGPRs), measured slower.
#ifndef PCA_IGEMM_EU
#define PCA_IGEMM_EU 1
#endif
// 1: software-pipelined epilogue store loop (next row's operands in flight), 0: chunked EU rows
#ifndef PCA_IGEMM_EPF
#define PCA_IGEMM_EPF 1
#endif

namespace pca {

bool deterministic_conv();   // conv_halo.hip
int wgrad_split_force();     // conv_halo.hip
void set_wgrad_split(int splits);

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
  int ksplit;           // split-K factor (1 = off): grid.z = ksplit * groups * classes
  float* ws;            // split-K fp32 partials [ksplit][N*Ho*Wo][Co]
  int mode;             // 0 fwd, 1 dgrad, 2 parity dgrad (autotune cache key)
  int ilv;              // register-pipelined K loop in the >= 3-stage configs (PCA_IGEMM_ILV)
  // dgrad only: fused backward reduce of the BatchNorm(+ReLU) that produced this conv's input
  // (bn_part != nullptr): per-channel sums of dz = dX * relu'(mask) and dz * xhat into slab rows
  const bf16* bn_y;     // that BN's input y
  const uint8_t* bn_mask;
  const float* bn_aux;  // [mean | istd | ...][Co]
  float* bn_part;       // [rows][NS][Co]
  // dual BN (projection-shortcut block tail act(BN(y) + BN2(y2))): the third sum dz * xhat2
  // (accumulator mode only; NS = 3)
  const bf16* bn_y2;
  const float* bn_aux2;
  int shards;           // BN partial sums (stats / bn_part): 0 = slab rows, >0 = sharded atomics
  const float* kshift;  // forward stats: per-channel shift K (common.h stat_shift), or nullptr
  // parity dgrad (MODE 2): the addend is COMPACT — [N][H/2][W/2][Co], the dX of a 1x1 stride-2
  // conv reading the same input (ResNet projection shortcut), nonzero only at the even-even
  // pixels: parity class 0 adds it at its own row index, the other classes add nothing
  int addend_s2c;
  // fused BN reduce: row stride of bn_y (0 = dense, Co) — a DenseNet BatchNorm reads a channel
  // suffix of its block's concat slab in place (ops/functional.py DenseSlab)
  int bn_ldy;
};

// dz = dX * relu'(y), accumulated as (sum dz, sum dz * xhat) for 8 channels
__device__ __forceinline__ void bn_fuse_acc(const uint4& v, const bf16* y, uint8_t m,
                                            const float* mean, const float* istd, float* s1,
                                            float* s2) {
  float f[8], yy[8];
  unpack8(v, f);
  unpack8(*reinterpret_cast<const uint4*>(y), yy);
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const float dz = ((m >> q) & 1u) ? f[q] : 0.f;
    s1[q] += dz;
    s2[q] += dz * (yy[q] - mean[q]) * istd[q];
  }
}

// the same with y already in registers (the batched store loop of the igemm epilogue); s2
// collects sum dz * (y - mean) — the per-channel istd is applied once at the flush
__device__ __forceinline__ void bn_fuse_acc_v(const uint4& v, const uint4& yv, uint8_t m,
                                              const float* mean, float* s1, float* s2) {
  float f[8], yy[8];
  unpack8(v, f);
  unpack8(yv, yy);
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const float dz = relu_bit(f[q], m, q);
    s1[q] += dz;
    s2[q] = fmaf(dz, yy[q] - mean[q], s2[q]);
  }
}

// dual-BN third sum, sum dz * (y2 - mean2) (x istd2 at the flush)
__device__ __forceinline__ void bn_fuse_acc3_v(const uint4& v, const uint4& y2v, uint8_t m,
                                               const float* m2, float* s3) {
  float f[8], yy[8];
  unpack8(v, f);
  unpack8(y2v, yy);
#pragma unroll
  for (int q = 0; q < 8; ++q) s3[q] = fmaf(relu_bit(f[q], m, q), yy[q] - m2[q], s3[q]);
}

// dual-BN third sum from mean2 / istd2 already in LDS or registers (m2, i2: this vector's 8
// channels)
__device__ __forceinline__ void bn_fuse_acc3s(const uint4& v, const bf16* y2, uint8_t m,
                                              const float* m2, const float* i2, float* s3) {
  float f[8], yy[8];
  unpack8(v, f);
  unpack8(*reinterpret_cast<const uint4*>(y2), yy);
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const float dz = ((m >> q) & 1u) ? f[q] : 0.f;
    s3[q] += dz * (yy[q] - m2[q]) * i2[q];
  }
}

// block reduction of NSUM per-thread 8-channel sums v[NSUM*8] of channel group c8 = tid % CG
// (CG | 64) into slab row `row`, sums s0 .. s0+NSUM-1 of a row of NS sums per channel (row stride
// NS * Co); channel base ch0 of group 0. The lanes of a wave that share a group (lane % CG) are
// folded by a butterfly first, so LDS holds one row per wave ([NW][NSUM*8][CG]) and each output
// is an NW-term sum by its own thread (the per-thread planar form left CG threads summing
// NT/CG rows each while the block waited).
template <int NT, int CG, int NSUM>
__device__ __forceinline__ void bn_flush_block(float* red, float* v, int ch0, int cvalid, int Co,
                                               float* part, int row, int shards, int NS, int s0) {
  constexpr int NW = NT / 64, NV = NSUM * 8;
  static_assert(CG >= 1 && CG <= 64 && (64 % CG) == 0, "channel groups per wave");
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int x = CG; x < 64; x <<= 1) v[i] += __shfl_xor(v[i], x, 64);
  if (lane < CG) {
#pragma unroll
    for (int i = 0; i < NV; ++i) red[(w * NV + i) * CG + lane] = v[i];
  }
  __syncthreads();
  for (int j = tid; j < NV * CG; j += NT) {   // j = i * CG + c8
    const int i = j / CG, c = (j % CG) * 8 + (i & 7);
    if (c < cvalid) {
      float a = 0.f;
#pragma unroll
      for (int ww = 0; ww < NW; ++ww) a += red[ww * NV * CG + j];
      stat_out(part, row, shards, (size_t)NS * Co, (s0 + (i >> 3)) * Co + ch0 + c, a);
    }
  }
}

// ---------------------------------------------------------------------------------------
// forward / dgrad implicit GEMM
// ---------------------------------------------------------------------------------------
// MODE 0: forward; 1: dgrad (generic gather, any stride); 2: dgrad of a stride-2 conv split
// into its 4 output parity classes (blockIdx.z = group*4 + class): class (ph, pw) only meets
// the taps kh = (ph+pad)&1 (+2...), so no MFMA work is spent on the 3/4 of taps that a strided
// transposed convolution would multiply by zero.
template <int BM, int BN, int WM, int WN, int STAGES, int MODE, bool STATS, bool SPLITK = false>
__global__ __launch_bounds__(WM * WN * 64) void conv_igemm_kernel(const bf16* __restrict__ A,
                                                                  const bf16* __restrict__ B,
                                                                  bf16* __restrict__ Y,
                                                                  float* __restrict__ stats,
                                                                  const float* __restrict__ bias,
                                                                  const bf16* __restrict__ addend,
                                                                  const ConvGeom g) {
  constexpr int NW = WM * WN, NT = NW * 64;
  constexpr int BK = 64;                 // K elements per stage: 128-byte LDS rows
  constexpr int RB = BK * 2;
  constexpr int A_BYTES = BM * RB, B_BYTES = BN * RB;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int A_PW = BM / (8 * NW);    // DMA instructions (8 rows each) per wave per stage
  constexpr int B_PW = BN / (8 * NW);
  constexpr int LPS = A_PW + B_PW;       // loads per stage per lane
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int CST = BN + 8;            // padded bf16 row stride of the staged C tile
  static_assert(NW == 4 || NW == 8, "4 or 8 waves");
  static_assert(A_PW >= 1 && B_PW >= 1 && BM % (8 * NW) == 0 && BN % (8 * NW) == 0, "tile");
  static_assert(STAGES >= 2, "stages");
  static_assert(BM * CST * 2 <= STAGES * STAGE, "C tile must fit the LDS ring");
  static_assert((BM * (BN / 8)) % NT == 0, "epilogue store loop");

  // (one LDS array — a second __shared__ object can cost a vmcnt(0) per K-step; dgrad: its tail
  // holds the dual BN's mean2 | istd2 of this block's channels, read by the epilogue)
  constexpr int AUX2_OFF = STAGES * STAGE;
  // (only where the tail costs no workgroup per CU: 160 KiB / LDS unchanged)
  constexpr bool AUX2_LDS = MODE != 0 && STAGES * STAGE + 2 * BN * 4 <= 160 * 1024 &&
                            (160 * 1024) / (STAGES * STAGE + 2 * BN * 4) == (160 * 1024) / (STAGES * STAGE);
  __shared__ __attribute__((aligned(16))) char smem[STAGES * STAGE + (AUX2_LDS ? 2 * BN * 4 : 0)];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  constexpr bool DGRAD = MODE != 0;
  constexpr bool PARITY = MODE == 2;
  // split-K: blockIdx.z = split * (groups * classes) + (group, class)
  const int gzb = g.groups * (PARITY ? 4 : 1);
  const int zb = SPLITK ? (int)(blockIdx.z % gzb) : (int)blockIdx.z;
  const int split = SPLITK ? (int)(blockIdx.z / gzb) : 0;
  const int grp = PARITY ? (zb >> 2) : zb;
  const int cls = PARITY ? (zb & 3) : 0;
  const int ph = cls >> 1, pw = cls & 1;
  // tap sets: kh = kh0 + tstep*t for t < nth (all taps unless PARITY)
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
  const int KT_all = cdiv(Kcls, BK);
  // this block's K-step range [kt_begin, KT)
  const int kper = SPLITK ? cdiv(KT_all, g.ksplit) : KT_all;
  const int kt_begin = SPLITK ? min(KT_all, split * kper) : 0;
  const int KT = SPLITK ? min(KT_all, kt_begin + kper) : KT_all;

  // Fast path: every K-step lies inside ONE tap (Cr % 64 == 0) and the gathered pixel is
  // (row base + scalar tap offset) — true for the forward, the stride-1 dgrad and every parity
  // class. The tap walk is then pure SALU and each DMA costs a few VALU ops (bounds + offset).
  const bool fast = (g.Cr % BK == 0) && (MODE != 1 || g.stride == 1);
  const int ksub = g.Cr / BK;              // K-steps per tap (fast path)

  // per-lane B row byte offsets (tap-independent part), fixed for the whole kernel
  int b_off[B_PW];
#pragma unroll
  for (int i = 0; i < B_PW; ++i) {
    const int br = n0 + (wid * B_PW + i) * 8 + lrow;
    b_off[i] = br < g.Cn ? ((grp * g.Cn + br) * kfull + lchunk * 8) * 2 : -1;
  }

  // per-lane BatchNorm partial sums, accumulated over every tile this workgroup owns
  float st_s[TN], st_q[TN];
#pragma unroll
  for (int ni = 0; ni < TN; ++ni) st_s[ni] = st_q[ni] = 0.f;
  int n_pad = 0;   // padding rows past M summed by this block (shifted statistics)

  // fused BN-backward reduce (dgrad): this thread's store-loop channel group is fixed
  constexpr int CG_ = BN / 8;
  static_assert(NT % CG_ == 0, "store loop channel group must be per-thread constant");
  const bool bnf = DGRAD && !SPLITK && g.bn_part != nullptr;
  float bs1[8], bs2[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) bs1[q] = bs2[q] = 0.f;
  // this thread's BN mean / istd: (re)loaded per tile at the epilogue (L2-resident), so their 16
  // registers are not held across the K loop
  auto load_bn_aux = [&](float* bmean, float* bistd) {
#pragma unroll
    for (int q = 0; q < 8; ++q) bmean[q] = bistd[q] = 0.f;
    if (bnf) {
      const int gc = n0 + (tid % CG_) * 8;
      if (gc < g.Cn) {
        const int ch = grp * g.Cn + gc;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          bmean[q] = g.bn_aux[ch + q];
          bistd[q] = g.bn_aux[g.Co + ch + q];
        }
      }
    }
  };
  if constexpr (AUX2_LDS) {
    if (bnf && g.bn_y2 != nullptr) {   // (block-uniform) the dual BN's mean2 | istd2 into LDS
      float* aux2s = reinterpret_cast<float*>(smem + AUX2_OFF);
      for (int i = tid; i < 2 * BN; i += NT) {
        const int c = n0 + (i % BN);
        aux2s[i] = c < g.Cn ? g.bn_aux2[(i >= BN ? g.Co : 0) + grp * g.Cn + c] : 0.f;
      }
      __syncthreads();
    }
  }

  // Persistent over M tiles (grid.x <= mtiles): amortises the per-block set-up and bounds the
  // BN statistics slab at grid.x rows.
  for (int tile = blockIdx.x; tile < mtiles; tile += gridDim.x) {
    const int m0 = tile * BM;
    int a_n[A_PW], a_h[A_PW], a_w[A_PW];
    int f_h[A_PW], f_w[A_PW], f_off[A_PW];   // fast path: gather base row/col and byte offset
#pragma unroll
    for (int i = 0; i < A_PW; ++i) {
      const int r = m0 + (wid * A_PW + i) * 8 + lrow;
      const uint32_t rr = r < Mrows ? r : 0;
      const uint32_t n = fdiv(rr, g.fd_hw);
      const uint32_t rem = rr - n * (rows_h * rows_w);
      const uint32_t h = fdiv(rem, g.fd_w);
      const uint32_t w = rem - h * rows_w;
      a_n[i] = r < Mrows ? (int)n : -1;
      a_h[i] = PARITY ? (int)(2 * h + ph) : (int)h;
      a_w[i] = PARITY ? (int)(2 * w + pw) : (int)w;
      int bh, bw;
      if constexpr (!DGRAD) {
        bh = (int)h * g.stride - g.pad;
        bw = (int)w * g.stride - g.pad;
      } else if constexpr (PARITY) {
        bh = (int)h + ((ph + g.pad - kh0) >> 1);
        bw = (int)w + ((pw + g.pad - kw0) >> 1);
      } else {
        bh = (int)h + g.pad;
        bw = (int)w + g.pad;
      }
      f_off[i] = ((((int)n * g.Hs + bh) * g.Ws + bw) * g.Cs + grp * g.Cr + lchunk * 8) * 2;
      if (r >= Mrows) bh = -(1 << 20);      // fails every bounds test (n = 0: no overflow)
      f_h[i] = bh;
      f_w[i] = bw;
    }

    // fast-path tap cursor (uniform): K-step kt = (tap, sub) with tap = (th, tw)
    int cur_sub = 0, cur_th = 0, cur_tw = 0, cur_kt = kt_begin;
    if (SPLITK && fast && kt_begin > 0) {
      const int tap0 = kt_begin / ksub;
      cur_sub = kt_begin - tap0 * ksub;
      cur_th = tap0 / ntw;
      cur_tw = tap0 - cur_th * ntw;
    }

    auto issue = [&](int kt, int buf) {
      char* As = smem + buf * STAGE;
      char* Bs = As + A_BYTES;
      if (fast) {
        const bool kok = cur_kt < KT;
        int dh, dw, kh, kw;
        if constexpr (!DGRAD) {
          dh = cur_th; dw = cur_tw; kh = cur_th; kw = cur_tw;
        } else if constexpr (PARITY) {
          dh = -cur_th; dw = -cur_tw; kh = kh0 + 2 * cur_th; kw = kw0 + 2 * cur_tw;
        } else {
          dh = -cur_th; dw = -cur_tw; kh = cur_th; kw = cur_tw;
        }
        const int a_delta = ((dh * g.Ws + dw) * g.Cs + cur_sub * BK) * 2;
        const int b_delta = ((kh * g.KW + kw) * g.Cr + cur_sub * BK) * 2;
#pragma unroll
        for (int i = 0; i < A_PW; ++i) {
          const bool ok = kok & ((uint32_t)(f_h[i] + dh) < (uint32_t)g.Hs) &
                          ((uint32_t)(f_w[i] + dw) < (uint32_t)g.Ws);
          dma16(rsA, As + (wid * A_PW + i) * 1024, ok ? (uint32_t)(f_off[i] + a_delta) : kOOB);
        }
#pragma unroll
        for (int i = 0; i < B_PW; ++i) {
          const bool ok = kok & (b_off[i] >= 0);
          dma16(rsB, Bs + (wid * B_PW + i) * 1024, ok ? (uint32_t)(b_off[i] + b_delta) : kOOB);
        }
        // advance the cursor
        ++cur_kt;
        if (++cur_sub == ksub) {
          cur_sub = 0;
          if (++cur_tw == ntw) {
            cur_tw = 0;
            ++cur_th;
          }
        }
        return;
      }
      const int kg = kt * 8 + lchunk;                  // 8-channel granule along K
      const bool kok = kg * 8 < Kcls && kt < KT;
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
    for (int s = 0; s < STAGES - 1; ++s) issue(kt_begin + s, s);

    if (STAGES >= 3 && g.ilv) {
      // Register-pipelined K loop (>= 3 LDS stages): the fragments of half-step kk = 1 are read
      // while the kk = 0 MFMAs run, and those of the NEXT K-step's kk = 0 while the kk = 1 MFMAs
      // run, one ds_read per MFMA (sched_group_barrier) — the LDS read latency leaves the
      // critical path instead of sitting between the barrier and the first MFMA of every step.
      // The barrier moves to mid-step: it publishes the next stage (landed by the counted vmcnt
      // wait) and, with each wave's own reads of the current stage drained (lgkmcnt(0)), frees
      // the current stage for the DMA issued at the top of the following step.
      constexpr int NF = TM + TN;
      bf16x8 af[2][TM], bfv[2][TN];
      auto frag = [&](int slot, int kk, int j) {
        const char* As = smem + slot * STAGE;
        const char* Bs = As + A_BYTES;
        const int gsel = kk * 4 + (lane >> 4);
        if (j < TN) {
          const int r = wn * WTN + j * 16 + (lane & 15);
          bfv[kk][j] = *reinterpret_cast<const bf16x8*>(Bs + r * RB + ((gsel ^ (r & 7)) << 4));
        } else {
          const int r = wm * WTM + (j - TN) * 16 + (lane & 15);
          af[kk][j - TN] = *reinterpret_cast<const bf16x8*>(As + r * RB + ((gsel ^ (r & 7)) << 4));
        }
      };
      // one MFMA, one ds_read, ... then the remaining MFMAs (or reads)
      auto ilv_pattern = [&]() {
        constexpr int PAIRS = NF < TM * TN ? NF : TM * TN;
#pragma unroll
        for (int i = 0; i < PAIRS; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // one MFMA
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // one ds_read
        }
        if constexpr (TM * TN > PAIRS) __builtin_amdgcn_sched_group_barrier(0x008, TM * TN - PAIRS, 0);
        if constexpr (NF > PAIRS) __builtin_amdgcn_sched_group_barrier(0x100, NF - PAIRS, 0);
      };
      wait_vmcnt<(STAGES - 2) * LPS>();
      raw_barrier();
#pragma unroll
      for (int j = 0; j < NF; ++j) frag(0, 0, j);
      for (int kt = kt_begin; kt < KT; ++kt) {
        const int rel = kt - kt_begin;
        const int slot = rel % STAGES;
        __builtin_amdgcn_sched_barrier(0);
        issue(kt + STAGES - 1, (rel + STAGES - 1) % STAGES);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < NF; ++j) frag(slot, 1, j);
#pragma unroll
        for (int mi = 0; mi < TM; ++mi)
#pragma unroll
          for (int ni = 0; ni < TN; ++ni)
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[0][mi], bfv[0][ni], acc[mi][ni], 0, 0, 0);
        ilv_pattern();
        __builtin_amdgcn_sched_barrier(0);
        wait_vmcnt<(STAGES - 2) * LPS>();   // stage kt+1 landed (this wave's pieces)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        raw_barrier();
        const bool more = kt + 1 < KT;
        if (more) {
          const int nslot = (rel + 1) % STAGES;
#pragma unroll
          for (int j = 0; j < NF; ++j) frag(nslot, 0, j);
        }
#pragma unroll
        for (int mi = 0; mi < TM; ++mi)
#pragma unroll
          for (int ni = 0; ni < TN; ++ni)
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[1][mi], bfv[1][ni], acc[mi][ni], 0, 0, 0);
        if (more) {
          ilv_pattern();
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    } else
    for (int kt = kt_begin; kt < KT; ++kt) {
      const int rel = kt - kt_begin;
      wait_vmcnt<(STAGES - 2) * LPS>();
      raw_barrier();
      // PCA_IGEMM_DMA_SPREAD=1 (build-time: as a runtime branch it cost the 128x128 forward its
      // second workgroup per CU): the next stage's DMA pieces go out after the first quarter of
      // this step's MFMAs instead of before its fragment reads (their issue cycles then overlap
      // the matrix pipe)
      // PCA_IGEMM_DMA_SPREAD=2: issued after this step's fragment reads, before its MFMAs (the
      // reads' LDS latency then runs under the DMA issue)
      constexpr bool dspread = PCA_IGEMM_DMA_SPREAD == 1;
      constexpr bool dafter = PCA_IGEMM_DMA_SPREAD == 2;
      if constexpr (!dspread && !dafter) issue(kt + STAGES - 1, (rel + STAGES - 1) % STAGES);   // past-the-end stages load zeros
      const char* As = smem + (rel % STAGES) * STAGE;
      const char* Bs = As + A_BYTES;
      // all fragments of the K-step are read up front into distinct registers (the compiler
      // otherwise sinks each A read next to its MFMAs and waits lgkmcnt(0) per fragment);
      // the waits then retire them in issue order while the MFMAs run
      bf16x8 af[BK / 32][TM], bfv[BK / 32][TN];
#pragma unroll
      for (int kk = 0; kk < BK / 32; ++kk) {
        const int gsel = kk * 4 + (lane >> 4);
#pragma unroll
        for (int ni = 0; ni < TN; ++ni) {
          const int r = wn * WTN + ni * 16 + (lane & 15);
          bfv[kk][ni] = *reinterpret_cast<const bf16x8*>(Bs + r * RB + ((gsel ^ (r & 7)) << 4));
        }
#pragma unroll
        for (int mi = 0; mi < TM; ++mi) {
          const int r = wm * WTM + mi * 16 + (lane & 15);
          af[kk][mi] = *reinterpret_cast<const bf16x8*>(As + r * RB + ((gsel ^ (r & 7)) << 4));
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (dafter) {
        issue(kt + STAGES - 1, (rel + STAGES - 1) % STAGES);
        __builtin_amdgcn_sched_barrier(0);
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int kk = 0; kk < BK / 32; ++kk)
#pragma unroll
        for (int mi = 0; mi < TM; ++mi)
#pragma unroll
          for (int ni = 0; ni < TN; ++ni) {
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[kk][mi], bfv[kk][ni], acc[mi][ni], 0, 0, 0);
            constexpr int NMF = (BK / 32) * TM * TN;
            if constexpr (dspread) if ((kk * TM + mi) * TN + ni == (NMF / 4 > 0 ? NMF / 4 - 1 : 0)) {
              __builtin_amdgcn_sched_barrier(0);
              issue(kt + STAGES - 1, (rel + STAGES - 1) % STAGES);
              __builtin_amdgcn_sched_barrier(0);
            }
          }
      __builtin_amdgcn_s_setprio(0);
    }
    wait_vmcnt<0>();
    __syncthreads();

    if constexpr (SPLITK) {
      // fp32 partial tile straight from the accumulators (16 lanes = 64 contiguous bytes);
      // bias / addend / BN statistics / bf16 conversion happen in splitk_reduce_kernel
      float* wsp = g.ws + (size_t)split * g.N * g.Ho * g.Wo * g.Co;
#pragma unroll
      for (int mi = 0; mi < TM; ++mi)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int gm = m0 + wm * WTM + mi * 16 + (lane >> 4) * 4 + j;
          if (gm >= Mrows) continue;
          size_t pix = gm;
          if constexpr (PARITY) {
            const uint32_t n = fdiv(gm, g.fd_hw);
            const uint32_t rem = gm - n * (rows_h * rows_w);
            const uint32_t h = fdiv(rem, g.fd_w);
            const uint32_t w = rem - h * rows_w;
            pix = ((size_t)n * g.Ho + 2 * h + ph) * g.Wo + 2 * w + pw;
          }
#pragma unroll
          for (int ni = 0; ni < TN; ++ni) {
            const int c = n0 + wn * WTN + ni * 16 + (lane & 15);
            if (c < g.Cn) wsp[pix * g.Co + (size_t)grp * g.Cn + c] = acc[mi][ni][j];
          }
        }
      continue;   // no LDS reuse before the next tile's prologue: the ring was drained above
    }

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
      // shifted sums (robust variance): d = v - K[c] (K = 0 unshifted). Rows past M are exact
      // zeros (zero-filled A, no bias) and add -K / K^2 each: taken back once per block (n_pad)
      // instead of a per-row mask (the masks cost the 128x128 forward its second wave per SIMD)
#pragma unroll
      for (int ni = 0; ni < TN; ++ni) {
        const int c = n0 + wn * WTN + ni * 16 + (lane & 15);
        const float kc = (g.kshift && c < g.Cn) ? g.kshift[grp * g.Cn + c] : 0.f;
#pragma unroll
        for (int mi = 0; mi < TM; ++mi)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float d = acc[mi][ni][j] - kc;
            st_s[ni] += d;
            st_q[ni] += d * d;
          }
      }
      n_pad += max(0, m0 + BM - Mrows);
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
    float bmean[8], bistd[8];
    load_bn_aux(bmean, bistd);
    constexpr int CG = BN / 8;
    float bs3[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) bs3[q] = 0.f;
    const bool dual = bnf && g.bn_y2 != nullptr;
    // Store loop in chunks of EU rows per thread: every global operand of a chunk (addend, y,
    // mask, y2) is loaded before any is used, so a chunk costs one memory round trip instead of
    // one per row and operand (the per-row guarded form waited vmcnt(0) up to 3x per row:
    // addend, then y + mask, then y2).
    // Rows past M / channels past Cn load from offset 0 (always valid) and are never stored.
    constexpr int EIT = (BM * CG) / NT;
    constexpr int EU = EIT >= PCA_IGEMM_EU ? PCA_IGEMM_EU : EIT;
    static_assert(EIT % EU == 0, "store loop chunks");
    const int c8 = tid % CG;   // (NT % CG == 0: fixed per thread)
    const int gc = n0 + c8 * 8;
#if PCA_IGEMM_EPF
    // Software-pipelined store loop: row it+1's global operands (addend, y, mask, y2) are in
    // flight while row it is combined and stored, so the tile's epilogue costs about one memory
    // round trip instead of EIT of them (the one-workgroup-per-CU 256x128 dgrad otherwise idles
    // its matrix cores for EIT latencies per tile). Two rows' operands live: 18 VGPRs.
    // (a compact stride-2 addend exists for parity class 0 only)
    const bool add_on = addend != nullptr && (!PARITY || !g.addend_s2c || cls == 0);
    struct EOp {
      size_t o;
      bool ok;
      uint4 av, yv, y2v;
      uint8_t mk;
    };
    auto eload = [&](int it, EOp& e) {
      const int gm = m0 + (tid + it * NT) / CG;
      e.ok = gm < Mrows && gc < g.Cn;
      size_t pix = gm;
      if constexpr (PARITY) {
        const uint32_t n = fdiv(gm, g.fd_hw);
        const uint32_t rem = gm - n * (rows_h * rows_w);
        const uint32_t h = fdiv(rem, g.fd_w);
        const uint32_t w = rem - h * rows_w;
        pix = ((size_t)n * g.Ho + 2 * h + ph) * g.Wo + 2 * w + pw;
      }
      e.o = e.ok ? pix * g.Co + (size_t)grp * g.Cn + gc : 0;
      if (add_on) {
        const size_t oa = (PARITY && g.addend_s2c) ? (e.ok ? (size_t)gm * g.Co + (size_t)grp * g.Cn + gc : 0) : e.o;
        e.av = *reinterpret_cast<const uint4*>(addend + oa);
      }
      if (bnf) {
        const size_t yo = g.bn_ldy ? (e.ok ? pix * g.bn_ldy + (size_t)grp * g.Cn + gc : 0) : e.o;
        e.yv = *reinterpret_cast<const uint4*>(g.bn_y + yo);
        e.mk = g.bn_mask[e.o >> 3];
      }
      if (dual) e.y2v = *reinterpret_cast<const uint4*>(g.bn_y2 + e.o);
    };
    auto eproc = [&](int it, const EOp& e) {
      const int r = (tid + it * NT) / CG;
      uint4 v = *reinterpret_cast<const uint4*>(Cs + r * CST + c8 * 8);
      if (add_on) {
        float a[8], b[8];
        unpack8(v, a);
        unpack8(e.av, b);
#pragma unroll
        for (int q = 0; q < 8; ++q) a[q] += b[q];
        v = pack8(a);
      }
      const uint8_t m = e.ok ? e.mk : 0;
      if (bnf) bn_fuse_acc_v(v, e.yv, m, bmean, bs1, bs2);
      if (dual) {
        if constexpr (AUX2_LDS) {
          const float* aux2s = reinterpret_cast<const float*>(smem + AUX2_OFF) + c8 * 8;
          bn_fuse_acc3_v(v, e.y2v, m, aux2s, bs3);
        } else {
          const float* a2 = g.bn_aux2 + grp * g.Cn + gc;
          bn_fuse_acc3_v(v, e.y2v, m, a2, bs3);
        }
      }
      if (e.ok) *reinterpret_cast<uint4*>(Y + e.o) = v;
    };
    (void)EU;
    EOp e0, e1;
    eload(0, e0);
#pragma unroll 1
    for (int it = 0; it < EIT; it += 2) {
      const bool has1 = it + 1 < EIT;
      if (has1) eload(it + 1, e1);
      eproc(it, e0);
      if (has1) {
        if (it + 2 < EIT) eload(it + 2, e0);
        eproc(it + 1, e1);
      }
    }
#else
#pragma unroll 1
    for (int it0 = 0; it0 < EIT; it0 += EU) {
      size_t o[EU], yo[EU];
      bool ok[EU];
      uint4 av[EU], yv[EU], y2v[EU];
      uint8_t mk[EU];
#pragma unroll
      for (int u = 0; u < EU; ++u) {
        const int gm = m0 + (tid + (it0 + u) * NT) / CG;
        ok[u] = gm < Mrows && gc < g.Cn;
        size_t pix = gm;
        if constexpr (PARITY) {
          const uint32_t n = fdiv(gm, g.fd_hw);
          const uint32_t rem = gm - n * (rows_h * rows_w);
          const uint32_t h = fdiv(rem, g.fd_w);
          const uint32_t w = rem - h * rows_w;
          pix = ((size_t)n * g.Ho + 2 * h + ph) * g.Wo + 2 * w + pw;
        }
        o[u] = ok[u] ? pix * g.Co + (size_t)grp * g.Cn + gc : 0;
        yo[u] = g.bn_ldy ? (ok[u] ? pix * g.bn_ldy + (size_t)grp * g.Cn + gc : 0) : o[u];
      }
      const bool add_on = addend != nullptr && (!PARITY || !g.addend_s2c || cls == 0);
      if (add_on) {
#pragma unroll
        for (int u = 0; u < EU; ++u) {
          const int gm = m0 + (tid + (it0 + u) * NT) / CG;
          const size_t oa = (PARITY && g.addend_s2c) ? (ok[u] ? (size_t)gm * g.Co + (size_t)grp * g.Cn + gc : 0) : o[u];
          av[u] = *reinterpret_cast<const uint4*>(addend + oa);
        }
      }
      if (bnf) {
#pragma unroll
        for (int u = 0; u < EU; ++u) {
          yv[u] = *reinterpret_cast<const uint4*>(g.bn_y + yo[u]);
          mk[u] = g.bn_mask[o[u] >> 3];
        }
      }
      if (dual) {
#pragma unroll
        for (int u = 0; u < EU; ++u) y2v[u] = *reinterpret_cast<const uint4*>(g.bn_y2 + o[u]);
      }
#pragma unroll
      for (int u = 0; u < EU; ++u) {
        const int r = (tid + (it0 + u) * NT) / CG;
        uint4 v = *reinterpret_cast<const uint4*>(Cs + r * CST + c8 * 8);
        if (add_on) {
          // fused gradient accumulation (dgrad): dX = conv^T(dY) + the other branch's dX
          float a[8], b[8];
          unpack8(v, a);
          unpack8(av[u], b);
#pragma unroll
          for (int q = 0; q < 8; ++q) a[q] += b[q];
          v = pack8(a);
        }
        const uint8_t m = ok[u] ? mk[u] : 0;   // (masked-off rows add nothing to the sums)
        if (bnf) bn_fuse_acc_v(v, yv[u], m, bmean, bs1, bs2);
        if (dual) {
          if constexpr (AUX2_LDS) {
            const float* aux2s = reinterpret_cast<const float*>(smem + AUX2_OFF) + c8 * 8;
            bn_fuse_acc3_v(v, y2v[u], m, aux2s, bs3);
          } else {   // (configs whose LDS would cost occupancy: from global, L1-cached)
            const float* a2 = g.bn_aux2 + grp * g.Cn + gc;
            bn_fuse_acc3_v(v, y2v[u], m, a2, bs3);
          }
        }
        if (ok[u]) *reinterpret_cast<uint4*>(Y + o[u]) = v;
      }
    }
#endif
    __syncthreads();   // the C tile aliases the ring the next tile's prologue refills
    if constexpr (DGRAD && !SPLITK) {
      if (dual) {   // (epilogue-local: no accumulator registers live across the K loop)
        // sum dz * (y2 - mean2) -> dz * xhat2: istd2 of this thread's 8 channels
        // (the LDS aux2 tail is overwritten by the flush's reduction only after this read)
        if (gc < g.Cn) {
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            float i2;
            if constexpr (AUX2_LDS) i2 = reinterpret_cast<const float*>(smem + AUX2_OFF)[BN + c8 * 8 + q];
            else i2 = g.bn_aux2[g.Co + grp * g.Cn + gc + q];
            bs3[q] *= i2;
          }
        }
        bn_flush_block<NT, CG_, 1>(reinterpret_cast<float*>(smem), bs3, grp * g.Cn + n0,
                                   g.Cn - n0, g.Co, g.bn_part, (int)blockIdx.x, g.shards, 3, 2);
        __syncthreads();
      }
    }
  }

  if constexpr (DGRAD && !SPLITK) {
    if (bnf) {   // slab row per (M-walker, parity class); channels of this block's N tile
      const int row = PARITY ? (int)blockIdx.x * 4 + cls : (int)blockIdx.x;
      float bmean[8], bistd[8];
      load_bn_aux(bmean, bistd);   // (sum dz * (y - mean) -> sum dz * xhat)
      float v[16];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        v[q] = bs1[q];
        v[8 + q] = bs2[q] * bistd[q];
      }
      bn_flush_block<NT, CG_, 2>(reinterpret_cast<float*>(smem), v, grp * g.Cn + n0, g.Cn - n0,
                                 g.Co, g.bn_part, row, g.shards, g.bn_y2 ? 3 : 2, 0);
    }
  }
  if constexpr (STATS && !SPLITK) {
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
        if (g.kshift && n_pad) {   // the padding rows' (0 - K) terms
          const float kc = g.kshift[grp * g.Cn + c];
          s += (float)n_pad * kc;
          q -= (float)n_pad * kc * kc;
        }
        stat_out(stats, blockIdx.x, g.shards, 2 * g.Co, grp * g.Cn + c, s);
        stat_out(stats, blockIdx.x, g.shards, 2 * g.Co, g.Co + grp * g.Cn + c, q);
      }
    }
    stat_krow(stats, g.shards, 2 * g.Co, g.kshift, g.Co);
  }
}

// ---------------------------------------------------------------------------------------
// phased 256-row implicit GEMM (large-M forward and stride-1 dgrad), after the structure of
// cdna_hip_programming.md §5 "The 256² 8-phase template": 8 waves (2 M x 4 N, 512 threads),
// BK = 64, two LDS K-tile buffers, 4 phases per K-tile. Each phase = {counted vmcnt (never 0 in
// the loop), one raw barrier, LDS-DMA of one quarter ("part") of the NEXT K-tile, this phase's
// fragment reads, the MFMAs of one quadrant of the wave's 128 x BN/4 output}. Parts are staged in
// the order they are first read (A rows of M-quadrant 0, B rows of N-quadrant 0, B N-quadrant 1,
// A M-quadrant 1), so every part is read >= 2 phases after it was issued and loads stay in
// flight across barriers; the structure the 2-stage kernel above lacks (it waits vmcnt(0) +
// barrier once per K-step, which caps it near ~0.9 PF/s, §5 'The step-3 structure').
// Fast path only: Cr % 64 == 0 (every K-step inside one tap), forward or stride-1 dgrad.
// ---------------------------------------------------------------------------------------
template <int BN, int WAVES, int MODE, bool STATS>
__global__ __launch_bounds__(WAVES * 64) void conv_igemm_ph_kernel(const bf16* __restrict__ A,
                                                            const bf16* __restrict__ B,
                                                            bf16* __restrict__ Y,
                                                            float* __restrict__ stats,
                                                            const float* __restrict__ bias,
                                                            const bf16* __restrict__ addend,
                                                            const ConvGeom g) {
  static_assert(MODE == 0 || MODE == 1, "forward or stride-1 dgrad");
  constexpr int BM = 256, BK = 64, RB = 128;
  constexpr int NT = WAVES * 64;
  constexpr int A_BYTES = BM * RB, B_BYTES = BN * RB, BUF = A_BYTES + B_BYTES;
  constexpr int WAVES_N = WAVES / 2;  // waves are 2 (M) x WAVES_N (N); each owns 128 x WTN
  constexpr int WTN = BN / WAVES_N;
  constexpr int TN = WTN / 16;        // N-fragments per wave
  constexpr int QN = TN / 2;          // N-fragments per N-quadrant
  constexpr int GA = 16 / WAVES;      // DMA instructions per wave for an A part (128 rows)
  constexpr int GB = BN / 16 / WAVES; // ... for a B part (BN/2 rows)
  static_assert(BN == 128 || BN == 256, "BN");
  static_assert(WAVES == 4 || WAVES == 8, "waves");
  static_assert(GB >= 1 && QN >= 1, "tile");
  static_assert(BM * BN * 2 <= 2 * BUF, "C tile must fit the LDS ring");
  constexpr bool DGRAD = MODE != 0;

  __shared__ __attribute__((aligned(16))) char smem[2 * BUF];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WAVES_N, wn = wid % WAVES_N;
  const int grp = blockIdx.z;
  const int n0 = blockIdx.y * BN;
  const int Mrows = g.M;
  const int mtiles = cdiv(Mrows, BM);
  const int kfull = g.KH * g.KW * g.Cr;
  const int ksub = g.Cr / BK;
  const int KT = g.KH * g.KW * ksub;

  const __amdgpu_buffer_rsrc_t rsA = make_rsrc(A, g.a_bytes);
  const __amdgpu_buffer_rsrc_t rsB = make_rsrc(B, g.b_bytes);
  const int lrow = lane >> 3;
  const int lchunk = (lane & 7) ^ lrow;   // swizzle on the DMA source (rows are 8-aligned)

  // A DMA slots: q (M-quadrant) x i (instruction): 8-row group j = 2*wid + i of the quadrant
  // covers rows (j >> 3) * 128 + q * 64 + (j & 7) * 8 + [0, 8)
  auto a_row0 = [&](int q, int i) {
    const int j = GA * wid + i;
    return (j >> 3) * 128 + q * 64 + (j & 7) * 8;
  };
  // B DMA slots: q (N-quadrant) x i: group j = GB*wid + i, wn' = j / (BN/64), k = j % (BN/64)
  auto b_row0 = [&](int q, int i) {
    const int j = GB * wid + i;
    return (j / TN) * WTN + q * (WTN / 2) + (j % TN) * 8;
  };

  int b_off[2][GB];
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int i = 0; i < GB; ++i) {
      const int br = n0 + b_row0(q, i) + lrow;
      b_off[q][i] = br < g.Cn ? ((grp * g.Cn + br) * kfull + lchunk * 8) * 2 : -1;
    }

  float st_s[TN], st_q[TN];
#pragma unroll
  for (int ni = 0; ni < TN; ++ni) st_s[ni] = st_q[ni] = 0.f;

  for (int tile = blockIdx.x; tile < mtiles; tile += gridDim.x) {
    const int m0 = tile * BM;
    int f_h[2][GA], f_w[2][GA], f_off[2][GA];
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int i = 0; i < GA; ++i) {
        const int r = m0 + a_row0(q, i) + lrow;
        const uint32_t rr = r < Mrows ? r : 0;
        const uint32_t n = fdiv(rr, g.fd_hw);
        const uint32_t rem = rr - n * (g.Ho * g.Wo);
        const uint32_t h = fdiv(rem, g.fd_w);
        const uint32_t w = rem - h * g.Wo;
        int bh, bw;
        if constexpr (!DGRAD) {
          bh = (int)h * g.stride - g.pad;
          bw = (int)w * g.stride - g.pad;
        } else {
          bh = (int)h + g.pad;
          bw = (int)w + g.pad;
        }
        f_off[q][i] = ((((int)n * g.Hs + bh) * g.Ws + bw) * g.Cs + grp * g.Cr + lchunk * 8) * 2;
        if (r >= Mrows) bh = -(1 << 20);
        f_h[q][i] = bh;
        f_w[q][i] = bw;
      }

    // staging cursor: K-tile kt = (tap (th, tw), sub)
    int s_kt = 0, s_sub = 0, s_th = 0, s_tw = 0;
    int a_delta = 0, b_delta = 0, s_dh = 0, s_dw = 0;
    bool s_ok = false;
    auto cursor = [&]() {   // deltas of the K-tile at the cursor
      s_ok = s_kt < KT;
      if constexpr (!DGRAD) {
        s_dh = s_th;
        s_dw = s_tw;
      } else {
        s_dh = -s_th;
        s_dw = -s_tw;
      }
      a_delta = ((s_dh * g.Ws + s_dw) * g.Cs + s_sub * BK) * 2;
      b_delta = ((s_th * g.KW + s_tw) * g.Cr + s_sub * BK) * 2;
    };
    auto advance = [&]() {
      ++s_kt;
      if (++s_sub == ksub) {
        s_sub = 0;
        if (++s_tw == g.KW) {
          s_tw = 0;
          ++s_th;
        }
      }
      cursor();
    };
    // part p of the cursor's K-tile into buffer `buf`: 0 = A quadrant 0, 1 = B quadrant 0,
    // 2 = B quadrant 1, 3 = A quadrant 1
    // (compile-time part / quadrant indices: std::integral_constant arguments, so every
    // accumulator index is a constant after inlining and acc stays in registers)
    auto stage = [&](auto pc, int buf) {
      constexpr int p = decltype(pc)::value;
      char* As = smem + buf * BUF;
      char* Bs = As + A_BYTES;
      if constexpr (p == 0 || p == 3) {
        constexpr int q = p == 0 ? 0 : 1;
#pragma unroll
        for (int i = 0; i < GA; ++i) {
          // bitwise, not short-circuit: && becomes exec-mask branches around each DMA
          const bool ok = s_ok & ((uint32_t)(f_h[q][i] + s_dh) < (uint32_t)g.Hs) &
                          ((uint32_t)(f_w[q][i] + s_dw) < (uint32_t)g.Ws);
          dma16(rsA, As + a_row0(q, i) * RB, ok ? (uint32_t)(f_off[q][i] + a_delta) : kOOB);
        }
      } else {
        constexpr int q = p - 1;
#pragma unroll
        for (int i = 0; i < GB; ++i) {
          const bool ok = s_ok & (b_off[q][i] >= 0);
          dma16(rsB, Bs + b_row0(q, i) * RB, ok ? (uint32_t)(b_off[q][i] + b_delta) : kOOB);
        }
      }
    };

    f32x4 acc[8][TN];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // prologue: K-tile 0 -> buffer 0, parts in read order
    cursor();
    stage(std::integral_constant<int, 0>{}, 0);
    stage(std::integral_constant<int, 1>{}, 0);
    stage(std::integral_constant<int, 2>{}, 0);
    stage(std::integral_constant<int, 3>{}, 0);
    advance();

    bf16x8 fa[2][4], fb[2][QN];
    // fragment rows are (multiple of 16) + (lane & 15), so their swizzle (row & 7) is lane & 7:
    // one per-lane base per operand and kk, everything else is an immediate offset
    const int a_lane = (wm * 128 + (lane & 15)) * RB;
    const int b_lane = (wn * WTN + (lane & 15)) * RB;
    const int swz0 = ((0 + (lane >> 4)) ^ (lane & 7)) << 4;
    const int swz1 = ((4 + (lane >> 4)) ^ (lane & 7)) << 4;
    auto read_a = [&](const char* As, auto qc) {
      constexpr int q = decltype(qc)::value;
      const char* p0 = As + a_lane + swz0 + q * 64 * RB;
      const char* p1 = As + a_lane + swz1 + q * 64 * RB;
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) {
        fa[0][mi] = *reinterpret_cast<const bf16x8*>(p0 + mi * 16 * RB);
        fa[1][mi] = *reinterpret_cast<const bf16x8*>(p1 + mi * 16 * RB);
      }
    };
    auto read_b = [&](const char* Bs, auto qc) {
      constexpr int q = decltype(qc)::value;
      const char* p0 = Bs + b_lane + swz0 + q * (WTN / 2) * RB;
      const char* p1 = Bs + b_lane + swz1 + q * (WTN / 2) * RB;
#pragma unroll
      for (int ni = 0; ni < QN; ++ni) {
        fb[0][ni] = *reinterpret_cast<const bf16x8*>(p0 + ni * 16 * RB);
        fb[1][ni] = *reinterpret_cast<const bf16x8*>(p1 + ni * 16 * RB);
      }
    };
    auto mma = [&](auto qmc, auto qnc) {
      constexpr int qm = decltype(qmc)::value, qn = decltype(qnc)::value;
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
          for (int ni = 0; ni < QN; ++ni)
            acc[qm * 4 + mi][qn * QN + ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                fa[kk][mi], fb[kk][ni], acc[qm * 4 + mi][qn * QN + ni], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    };

    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using I3 = std::integral_constant<int, 3>;
    for (int kt = 0; kt < KT; ++kt) {
      const int cur = kt & 1, nxt = cur ^ 1;
      const char* As = smem + cur * BUF;
      const char* Bs = As + A_BYTES;
      // phase 0: needs parts 0, 1 of kt (parts 2, 3 may stay in flight)
      wait_vmcnt<GB + GA>();
      raw_barrier();
      stage(I0{}, nxt);
      read_a(As, I0{});
      read_b(Bs, I0{});
      mma(I0{}, I0{});
      // phase 1: needs part 2 of kt (part 3 of kt, part 0 of kt+1 in flight)
      wait_vmcnt<2 * GA>();
      raw_barrier();
      stage(I1{}, nxt);
      read_b(Bs, I1{});
      mma(I0{}, I1{});
      // phase 2: needs part 3 of kt (parts 0, 1 of kt+1 in flight)
      wait_vmcnt<GA + GB>();
      raw_barrier();
      stage(I2{}, nxt);
      read_a(As, I1{});
      mma(I1{}, I1{});
      // phase 3: A quadrant 1 stays in registers, B quadrant 0 is re-read (landed since phase 0;
      // its buffer is not restaged before the next K-tile's phase 1, after two barriers)
      stage(I3{}, nxt);
      advance();
      read_b(Bs, I0{});
      mma(I1{}, I0{});
    }
    wait_vmcnt<0>();
    __syncthreads();

    // ---- epilogue: bias, BN partials, bf16 tile through LDS (XOR-swizzled 16-B chunks) ----
    if (bias) {
#pragma unroll
      for (int ni = 0; ni < TN; ++ni) {
        const int c = n0 + wn * WTN + ni * 16 + (lane & 15);
        const float bv = c < g.Cn ? bias[grp * g.Cn + c] : 0.f;
#pragma unroll
        for (int mi = 0; mi < 8; ++mi)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int r = m0 + wm * 128 + mi * 16 + (lane >> 4) * 4 + j;
            if (r < Mrows) acc[mi][ni][j] += bv;
          }
      }
    }
    if constexpr (STATS) {
#pragma unroll
      for (int ni = 0; ni < TN; ++ni) {
        const int c = n0 + wn * WTN + ni * 16 + (lane & 15);
        const float kc = (g.kshift && c < g.Cn) ? g.kshift[grp * g.Cn + c] : 0.f;
#pragma unroll
        for (int mi = 0; mi < 8; ++mi)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            // rows past M are exact zeros (zero-filled A): unshifted they add nothing, shifted
            // they must not add -K
            const int r = m0 + wm * 128 + mi * 16 + (lane >> 4) * 4 + j;
            const float d = r < Mrows ? acc[mi][ni][j] - kc : 0.f;
            st_s[ni] += d;
            st_q[ni] += d * d;
          }
      }
    }
    constexpr int CRB = BN * 2;   // bytes per staged C row
#pragma unroll
    for (int mi = 0; mi < 8; ++mi)
#pragma unroll
      for (int ni = 0; ni < TN; ++ni)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int r = wm * 128 + mi * 16 + (lane >> 4) * 4 + j;
          const int c = wn * WTN + ni * 16 + (lane & 15);
          *reinterpret_cast<bf16*>(smem + r * CRB + ((((c >> 3) ^ (r & 7))) << 4) + (c & 7) * 2) =
              f2bf(acc[mi][ni][j]);
        }
    __syncthreads();
    constexpr int CG = BN / 8;
#pragma unroll
    for (int it = 0; it < (BM * CG) / NT; ++it) {
      const int idx = tid + it * NT;
      const int r = idx / CG, c8 = idx % CG;
      const int gm = m0 + r, gc = n0 + c8 * 8;
      if (gm < Mrows && gc < g.Cn) {
        uint4 v = *reinterpret_cast<const uint4*>(smem + r * CRB + ((c8 ^ (r & 7)) << 4));
        const size_t o = (size_t)gm * g.Co + (size_t)grp * g.Cn + gc;
        if (addend) {
          float a[8], b[8];
          unpack8(v, a);
          unpack8(*reinterpret_cast<const uint4*>(addend + o), b);
#pragma unroll
          for (int q = 0; q < 8; ++q) a[q] += b[q];
          v = pack8(a);
        }
        *reinterpret_cast<uint4*>(Y + o) = v;
      }
    }
    __syncthreads();   // the C tile aliases the ring the next tile's prologue refills
  }

  if constexpr (STATS) {
    float* red = reinterpret_cast<float*>(smem);  // [2 wm][BN][2]
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
      const float s = red[tid * 2 + 0] + red[(BN + tid) * 2 + 0];
      const float q = red[tid * 2 + 1] + red[(BN + tid) * 2 + 1];
      const int c = n0 + tid;
      if (c < g.Cn) {
        stat_out(stats, blockIdx.x, g.shards, 2 * g.Co, grp * g.Cn + c, s);
        stat_out(stats, blockIdx.x, g.shards, 2 * g.Co, g.Co + grp * g.Cn + c, q);
      }
    }
    stat_krow(stats, g.shards, 2 * g.Co, g.kshift, g.Co);
  }
}

// ---------------------------------------------------------------------------------------
// wgrad: split-K GEMM over pixels with transposed LDS reads
// ---------------------------------------------------------------------------------------
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
  int atomic;            // wide kernel: 1 = fp32 atomics into dW, 0 = slab rows + reduce
  uint32_t x_bytes, dy_bytes;
  FastDiv fd_hw, fd_w, fd_cin8;
};

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
        if (m < g.cout_g && n < g.Ktot) {
          const size_t idx = ((size_t)grp * g.cout_g + m) * g.Ktot + n;
          if (g.atomic) {
            if (g.splits == 1) DW[idx] += acc[mi][ni][j];   // sole writer: plain read-modify-write
            else atomicAdd(DW + idx, acc[mi][ni][j]);
          } else {
            DW[(size_t)split * g.groups * g.cout_g * g.Ktot + idx] = acc[mi][ni][j];
          }
        }
      }
}

// ---------------------------------------------------------------------------------------
// wide wgrad: all taps of a 64-channel block per workgroup, blocked LDS images, slab output
// ---------------------------------------------------------------------------------------
// For Cin/G % 64 == 0 the GEMM column axis (tap, ci) splits into 64-column blocks that each lie
// inside ONE tap, so a block's gather is a scalar tap offset on a per-pixel base: the per-DMA
// cost is a bounds test and an add. Both operands are staged as blocked images
// [64-channel block][KP pixels][128 B] (the RB = 128 swizzle of tr_frag), so one workgroup can
// own a wide column tile (up to 9 blocks = all 9 taps of 64 channels) and x / dY are read from
// memory once per column tile instead of once per 128 columns. Each workgroup walks a contiguous
// pixel range and writes its fp32 partial tile to a slab row; a reduce kernel then adds the slab
// rows into dW in a fixed order (deterministic, no atomics).
template <int MB, int NB, int WM, int WN>
__global__ __launch_bounds__(WM * WN * 64) void conv_wgrad_wide_kernel(const bf16* __restrict__ X,
                                                                       const bf16* __restrict__ DY,
                                                                       float* __restrict__ slab,
                                                                       const WgradGeom g) {
  constexpr int NW = WM * WN;
  constexpr int KP = 32;                         // pixels per stage (one MFMA K step)
  constexpr int BLK = KP * 128;                  // bytes of one 64-channel block image
  constexpr int NOPS = MB + NB;                  // operand blocks per stage
  constexpr int STAGE = NOPS * BLK;
  constexpr int BM = MB * 64, BN = NB * 64;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int OPW = (NOPS + NW - 1) / NW;      // operand blocks per wave (last may be idle)
  static_assert(WTM % 16 == 0 && WTN % 16 == 0, "wave tile");
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int split = blockIdx.z % g.splits;
  const int grp = blockIdx.z / g.splits;
  const int m0 = blockIdx.x * BM;                // output channel (within group)
  const int n0 = blockIdx.y * BN;                // (tap, ci) column
  const int p_begin = split * g.chunk;
  const int p_end = min(g.P, p_begin + g.chunk);

  const __amdgpu_buffer_rsrc_t rsX = make_rsrc(X, g.x_bytes);
  const __amdgpu_buffer_rsrc_t rsD = make_rsrc(DY, g.dy_bytes);

  // lane -> (row (l>>3) + 8i of the stage, logical 16-byte chunk) for the 4 row groups
  int lch[KP / 8];
#pragma unroll
  for (int i = 0; i < KP / 8; ++i) lch[i] = ((lane & 7) ^ tr_swz<128>(8 * i + (lane >> 3))) * 16;

  // scalar per-operand-block gather parameters (this wave's blocks only)
  int o_kind[OPW], o_col[OPW], o_dh[OPW], o_dw[OPW];
#pragma unroll
  for (int j = 0; j < OPW; ++j) {
    const int o = wid + NW * j;
    o_kind[j] = o < NOPS ? (o < MB ? 0 : 1) : 2;
    o_col[j] = 0; o_dh[j] = 0; o_dw[j] = 0;
    if (o < MB) {
      const int co = m0 + 64 * o;
      o_kind[j] = co < g.cout_g ? 0 : 2;
      o_col[j] = (grp * g.cout_g + co) * 2;
    } else if (o < NOPS) {
      const int col = n0 + 64 * (o - MB);
      if (col >= g.Ktot) {
        o_kind[j] = 2;
      } else {
        const int tap = col / g.cin_g, ci = col - tap * g.cin_g;
        const int kh = tap / g.KW, kw = tap - kh * g.KW;
        o_dh[j] = kh;
        o_dw[j] = kw;
        o_col[j] = ((kh * g.W + kw) * g.Cx + grp * g.cin_g + ci) * 2;
      }
    }
  }

  auto issue = [&](int pbase, int buf) {
    char* S = smem + buf * STAGE;
    int ih0[KP / 8], iw0[KP / 8], xo[KP / 8], dyo[KP / 8];
    bool pv[KP / 8];
#pragma unroll
    for (int i = 0; i < KP / 8; ++i) {
      const int p = pbase + 8 * i + (lane >> 3);
      pv[i] = p < p_end;
      const uint32_t pp = pv[i] ? p : 0;
      const uint32_t n = fdiv(pp, g.fd_hw);
      const uint32_t rem = pp - n * (g.Ho * g.Wo);
      const uint32_t oh = fdiv(rem, g.fd_w);
      const uint32_t ow = rem - oh * g.Wo;
      ih0[i] = (int)oh * g.stride - g.pad;
      iw0[i] = (int)ow * g.stride - g.pad;
      xo[i] = ((((int)n * g.H + ih0[i]) * g.W + iw0[i]) * g.Cx) * 2 + lch[i];
      dyo[i] = (int)pp * g.Cy * 2 + lch[i];
    }
#pragma unroll
    for (int j = 0; j < OPW; ++j) {
      const int o = wid + NW * j;
      if (o_kind[j] == 2) {
        if (o < NOPS) {   // column / channel tail: keep the block's image zero
#pragma unroll
          for (int i = 0; i < KP / 8; ++i) dma16(rsX, S + o * BLK + i * 1024, kOOB);
        }
        continue;
      }
#pragma unroll
      for (int i = 0; i < KP / 8; ++i) {
        uint32_t off;
        if (o_kind[j] == 0) {
          off = pv[i] ? (uint32_t)(dyo[i] + o_col[j]) : kOOB;
          dma16(rsD, S + o * BLK + i * 1024, off);
        } else {
          const bool ok = pv[i] && (uint32_t)(ih0[i] + o_dh[j]) < (uint32_t)g.H &&
                          (uint32_t)(iw0[i] + o_dw[j]) < (uint32_t)g.W;
          off = ok ? (uint32_t)(xo[i] + o_col[j]) : kOOB;
          dma16(rsX, S + o * BLK + i * 1024, off);
        }
      }
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int KT = p_end > p_begin ? cdiv(p_end - p_begin, KP) : 0;
  issue(p_begin, 0);
  for (int kt = 0; kt < KT; ++kt) {
    wait_vmcnt<0>();
    raw_barrier();
    if (kt + 1 < KT) issue(p_begin + (kt + 1) * KP, (kt + 1) & 1);
    const char* S = smem + (kt & 1) * STAGE;
    bf16x8 af[TM];
#pragma unroll
    for (int mi = 0; mi < TM; ++mi) {
      const int m = wm * WTM + mi * 16;
      af[mi] = tr_frag<64>(S + (m >> 6) * BLK, 0, m & 63, lane);
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ni = 0; ni < TN; ++ni) {
      const int n = wn * WTN + ni * 16;
      const bf16x8 bfv = tr_frag<64>(S + (MB + (n >> 6)) * BLK, 0, n & 63, lane);
#pragma unroll
      for (int mi = 0; mi < TM; ++mi)
        acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mi], bfv, acc[mi][ni], 0, 0, 0);
    }
    __builtin_amdgcn_s_setprio(0);
  }

  // partial tile -> slab row (split), layout [splits][groups*cout_g][Ktot]
  float* out = slab + (size_t)split * g.groups * g.cout_g * g.Ktot;
#pragma unroll
  for (int mi = 0; mi < TM; ++mi)
#pragma unroll
    for (int ni = 0; ni < TN; ++ni)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = m0 + wm * WTM + mi * 16 + (lane >> 4) * 4 + j;
        const int n = n0 + wn * WTN + ni * 16 + (lane & 15);
        if (m < g.cout_g && n < g.Ktot) {
          const size_t idx = ((size_t)grp * g.cout_g + m) * g.Ktot + n;
          if (g.atomic) {
            if (g.splits == 1) slab[idx] += acc[mi][ni][j];
            else atomicAdd(slab + idx, acc[mi][ni][j]);
          } else {
            out[idx] = acc[mi][ni][j];
          }
        }
      }
}

// dW[i] += sum_s slab[s][i], fixed summation order (float4 lanes)
__global__ __launch_bounds__(256) void wgrad_slab_reduce_kernel(const float* __restrict__ slab,
                                                                float* __restrict__ dw, int splits,
                                                                int64_t n4) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  const float4* s4 = reinterpret_cast<const float4*>(slab);
  float4 a = reinterpret_cast<float4*>(dw)[i];
  for (int s = 0; s < splits; ++s) {
    const float4 v = s4[(int64_t)s * n4 + i];
    a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
  }
  reinterpret_cast<float4*>(dw)[i] = a;
}

// ---------------------------------------------------------------------------------------
// split-K reduction: sum the fp32 partials in a fixed order (deterministic), add bias or the
// fused dgrad addend, store bf16 and emit one BN-statistics slab row per block (the same slab
// format the igemm epilogue writes, so bn_finalize is unchanged).
// ---------------------------------------------------------------------------------------
template <bool STATS>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ ws, int S,
                                                           int M, int Co, int rows_per_block,
                                                           const float* __restrict__ bias,
                                                           const bf16* __restrict__ addend,
                                                           bf16* __restrict__ Y,
                                                           float* __restrict__ stats,
                                                           const bf16* __restrict__ bn_y,
                                                           const uint8_t* __restrict__ bn_mask,
                                                           const float* __restrict__ bn_aux,
                                                           float* __restrict__ bn_part,
                                                           int shards,
                                                           const bf16* __restrict__ bn_y2,
                                                           const float* __restrict__ bn_aux2,
                                                           const float* __restrict__ kshift,
                                                           int bn_ldy) {
  __shared__ float red[3 * 2048];
  const int NSB = bn_y2 ? 3 : 2;      // fused BN sums per channel (3: dual BN)
  const int CG = Co >> 3;             // 8-channel groups per row (Co <= 2048: CG <= 256)
  const int RP = 256 / CG;            // rows per pass
  const int tid = threadIdx.x;
  const int cg = tid % CG, rr = tid / CG;
  const bool active = rr < RP;
  float sm[8], sq[8], b[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) sm[q] = sq[q] = 0.f;
#pragma unroll
  for (int q = 0; q < 8; ++q) b[q] = bias ? bias[cg * 8 + q] : 0.f;
  // (forward statistics and the dgrad's fused BN reduce never meet in one launch: the STATS
  // variant drops the reduce's registers)
  float* const bnp = STATS ? nullptr : bn_part;
  float kk[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) kk[q] = (STATS && kshift && active) ? kshift[cg * 8 + q] : 0.f;
  const int r0 = blockIdx.x * rows_per_block;
  const int r1 = min(M, r0 + rows_per_block);
  const size_t plane = (size_t)M * Co;
  float bs1[8], bs2[8], bs3[8], bmean[8], bistd[8], bmean2[8], bistd2[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    bs1[q] = bs2[q] = bs3[q] = 0.f;
    bmean[q] = bnp && active ? bn_aux[cg * 8 + q] : 0.f;
    bistd[q] = bnp && active ? bn_aux[Co + cg * 8 + q] : 0.f;
    bmean2[q] = bnp && bn_y2 && active ? bn_aux2[cg * 8 + q] : 0.f;
    bistd2[q] = bnp && bn_y2 && active ? bn_aux2[Co + cg * 8 + q] : 0.f;
  }
  if (active) {
    for (int r = r0 + rr; r < r1; r += RP) {
      const size_t o = (size_t)r * Co + cg * 8;
      float a[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) a[q] = b[q];
      // up to 8 partial planes' loads in flight before the first add (a runtime-S loop issued
      // them one round trip at a time); the adds keep the plane order, so the sum is unchanged
      for (int k0 = 0; k0 < S; k0 += 8) {
        float4 v0[8], v1[8];
#pragma unroll
        for (int k = 0; k < 8; ++k)
          if (k0 + k < S) {
            v0[k] = *reinterpret_cast<const float4*>(ws + (k0 + k) * plane + o);
            v1[k] = *reinterpret_cast<const float4*>(ws + (k0 + k) * plane + o + 4);
          }
#pragma unroll
        for (int k = 0; k < 8; ++k)
          if (k0 + k < S) {
            a[0] += v0[k].x; a[1] += v0[k].y; a[2] += v0[k].z; a[3] += v0[k].w;
            a[4] += v1[k].x; a[5] += v1[k].y; a[6] += v1[k].z; a[7] += v1[k].w;
          }
      }
      if constexpr (STATS) {
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const float d = a[q] - kk[q];   // shifted sums (kk = 0 unshifted)
          sm[q] += d;
          sq[q] += d * d;
        }
      }
      if (addend) {
        float d[8];
        unpack8(*reinterpret_cast<const uint4*>(addend + o), d);
#pragma unroll
        for (int q = 0; q < 8; ++q) a[q] += d[q];
      }
      const uint4 pv = pack8(a);
      if (bnp) bn_fuse_acc(pv, bn_y + (bn_ldy ? (size_t)r * bn_ldy + cg * 8 : o), bn_mask[o >> 3],
                           bmean, bistd, bs1, bs2);
      if (bnp && bn_y2) bn_fuse_acc3s(pv, bn_y2 + o, bn_mask[o >> 3], bmean2, bistd2, bs3);
      *reinterpret_cast<uint4*>(Y + o) = pv;
    }
  }
  // block reductions below: planes [sum][RP x Co] written as float4 pairs (consecutive lanes,
  // consecutive 32-byte runs) and read with consecutive lanes on consecutive channels — the
  // interleaved [row][channel][sum] layout was 12-19 extra LDS cycles per access
  constexpr int PL = 2048;   // RP * Co = 256 / CG * 8 * CG
  auto put8 = [&](int plane, const float* v) {
    float4* d = reinterpret_cast<float4*>(red + plane * PL + rr * Co + cg * 8);
    d[0] = make_float4(v[0], v[1], v[2], v[3]);
    d[1] = make_float4(v[4], v[5], v[6], v[7]);
  };
  if (bnp) {   // fused BN-backward reduce: one slab row per block (rows = gridDim.x)
    __syncthreads();
    if (active) {
      put8(0, bs1);
      put8(1, bs2);
      put8(2, bs3);
    }
    __syncthreads();
    for (int c = tid; c < Co; c += 256) {
      float s0 = 0.f, q0 = 0.f, t0 = 0.f;
      for (int k = 0; k < RP; ++k) {
        s0 += red[k * Co + c];
        q0 += red[PL + k * Co + c];
        t0 += red[2 * PL + k * Co + c];
      }
      stat_out(bnp, blockIdx.x, shards, NSB * Co, c, s0);
      stat_out(bnp, blockIdx.x, shards, NSB * Co, Co + c, q0);
      if (NSB == 3) stat_out(bnp, blockIdx.x, shards, NSB * Co, 2 * Co + c, t0);
    }
    return;
  }
  if constexpr (STATS) {
    if (active) {
      put8(0, sm);
      put8(1, sq);
    }
    __syncthreads();
    for (int c = tid; c < Co; c += 256) {
      float s0 = 0.f, q0 = 0.f;
      for (int k = 0; k < RP; ++k) {
        s0 += red[k * Co + c];
        q0 += red[PL + k * Co + c];
      }
      stat_out(stats, blockIdx.x, shards, 2 * Co, c, s0);
      stat_out(stats, blockIdx.x, shards, 2 * Co, Co + c, q0);
    }
    stat_krow(stats, shards, 2 * Co, kshift, Co);
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
  g.ksplit = 1;
  g.ws = nullptr;
  g.mode = 0;
  static const int ilv = [] {
    const char* e = getenv("PCA_IGEMM_ILV");
    return e && e[0] == '1' ? 1 : 0;
  }();
  g.ilv = ilv;
  g.bn_y = nullptr;
  g.bn_mask = nullptr;
  g.bn_aux = nullptr;
  g.bn_part = nullptr;
  g.bn_y2 = nullptr;
  g.bn_aux2 = nullptr;
  g.shards = stat_shards();
  g.kshift = stat_shift();
  g.addend_s2c = 0;
  g.bn_ldy = 0;
  return g;
}

// Persistent grid. grid.x (M-tile walkers, also the BN-statistics slab row count, <= 1024) is
// sized so that grid.x * grid.y * grid.z fills exactly the resident workgroup slots of the chip
// (occupancy x CUs): a grid of 1024 walkers over 768 slots would run a second, one-third-full
// round of blocks (measured: the 64-channel layers lost ~25% to that tail).
constexpr int kMaxTilesX = 1024;

static int num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    if (n <= 0) n = 256;
  }
  return n;
}

template <int BM, int BN, int WM, int WN, int ST, int MODE>
static int igemm_occupancy() {
  static int occ = 0;
  if (occ == 0) {
occ = std::min(
        blocks_per_cu((const void*)conv_igemm_kernel<BM, BN, WM, WN, ST, MODE, true>, WM * WN * 64, "igemm"),
        blocks_per_cu((const void*)conv_igemm_kernel<BM, BN, WM, WN, ST, MODE, false>, WM * WN * 64, "igemm"));
  }
  return occ;
}

static int persistent_grid_x(int mtiles, int gyz, int occ) {
  const int slots = occ * num_cus();
  int gx = std::max(1, slots / std::max(1, gyz));
  gx = std::min({gx, mtiles, kMaxTilesX});
  const int per = cdiv(mtiles, gx);   // equalise tiles per walker
  return cdiv(mtiles, per);
}

template <int MODE>
static int igemm_rows(const ConvGeom& g) {
  return MODE == 2 ? g.N * (g.Ho / 2) * (g.Wo / 2) : g.M;
}

// process-wide overrides (set_conv_tile) used by tools/bench_conv.py sweeps and the tests
static int g_igemm_override = -1;
static int g_wgrad_override = -1;
static int g_weff_cfg = -1;    // wgrad config resolved by wgrad_resolve() for the current geometry

// ---- autotuning (the analogue of the reference's cudnn.benchmark = True, main.py:75) ----
// The first eager call of each conv geometry times a candidate set of (tile config, split-K)
// pairs with HIP events (bindings.cpp drives it, outside stream capture) and caches the
// fastest; later calls and hipGraph captures use the cached choice.
struct TuneKey {
  int v[13];
  bool operator<(const TuneKey& o) const { return std::lexicographical_compare(v, v + 13, o.v, o.v + 13); }
};
static std::map<TuneKey, std::pair<int, int>> g_tuned;   // key -> (cfg, split)
static int g_trial_cfg = -1, g_trial_split = -1;

// Dual-BN request of the next dgrad launch(es) (bindings scope it around one call): the fused
// reduce also adds dz * xhat2 of the projection-shortcut BN (y2, aux2) — generic igemm / split-K
// stride-1 dgrads into a sharded accumulator only.
static const bf16* g_dual_y2 = nullptr;
static const float* g_dual_aux2 = nullptr;

// A dual-BN dgrad is tuned apart from the plain one of the same geometry (bit 3 of the mode
// field): the halo kernel cannot carry the third sum, so where it wins the plain dgrad it must
// not be picked for the dual call too (that left a separate reduce + finalize + apply behind,
// 70-126 us per projection block at bs1024)
static TuneKey tune_key(const ConvGeom& g) {
  const int mode = g.mode + (g.mode != 0 && g_dual_y2 ? 8 : 0);
  return TuneKey{{mode, g.N, g.Hs, g.Ws, g.Cs, g.Ho, g.Wo, g.Co, g.KH, g.KW, g.stride, g.pad,
                  g.groups}};
}

static const std::pair<int, int>* tuned_choice(const ConvGeom& g) {
  auto it = g_tuned.find(tune_key(g));
  return it == g_tuned.end() ? nullptr : &it->second;
}

// Split-K (small-M layers: a per-GPU batch of 128 gives layer-4 M = 2048, i.e. 64 tiles of
// 128x128 for 256 CUs). When the output tiles fill less than half the resident slots, the K
// loop is split S ways (each split keeps >= 4 K-steps), partials go to an fp32 workspace and
// splitk_reduce_kernel finishes the epilogue. set_conv_tile(2, S) forces S (sweeps).
static int g_splitk_override = -1;
constexpr int kMaxSplitCo = 2048;

template <int MODE>
static int igemm_ksteps(const ConvGeom& g) {
  const int taps = MODE == 2 ? cdiv(g.KH, 2) * cdiv(g.KW, 2) : g.KH * g.KW;
  return cdiv(taps * g.Cr, 64);
}

template <int BM, int BN, int WM, int WN, int ST, int MODE>
static int igemm_ksplit_t(const ConvGeom& g) {
  if (g.Co % 8 != 0 || g.Co > kMaxSplitCo) return 1;
  const int KT = igemm_ksteps<MODE>(g);
  if (g_splitk_override >= 1) return std::max(1, std::min(g_splitk_override, KT));
  if (g_splitk_override == 0) return 1;
  if (g_trial_split >= 1) return std::max(1, std::min(g_trial_split, KT));
  if (g_igemm_override < 0 && g_trial_cfg < 0) {
    if (const auto* t = tuned_choice(g)) return std::max(1, std::min(t->second, KT));
  }
  const int gzb = g.groups * (MODE == 2 ? 4 : 1);
  const int tiles = cdiv(igemm_rows<MODE>(g), BM) * cdiv(g.Cn, BN) * gzb;
  const int slots = igemm_occupancy<BM, BN, WM, WN, ST, MODE>() * num_cus();
  // split only when the tiles leave most CUs idle: the fp32 partial round trip costs
  // ~S*M*Co*8 bytes of HBM traffic (measured: a 2-way split of 128->128 @16x16, bs128, lost 45%)
  if (2 * tiles > num_cus()) return 1;
  const int S = std::min({slots / tiles, KT / 4, 8});
  return S >= 2 ? S : 1;
}

static int splitk_reduce_grid(int M, int Co, int* rows_per_block) {
  // every block adds its BN sums into the R shard rows of the accumulator at the end: the grid
  // cap also bounds those same-address atomics (PCA_SPLITK_RED_CAP blocks; default one per CU —
  // same-box A/B vs two per CU: bs128 equal, bs256 -0.3 %, bs512 -0.5 %)
  static const int cap = [] {
    const char* e = getenv("PCA_SPLITK_RED_CAP");
    const int v = e ? atoi(e) : 0;
    return v > 0 ? v : 0;
  }();
  const int RP = 256 / (Co / 8);
  int gx = std::min(cdiv(M, RP), cap > 0 ? cap : num_cus());
  const int rpb = cdiv(M, gx);
  *rows_per_block = rpb;
  return cdiv(M, rpb);
}

template <int BM, int BN, int WM, int WN, int ST, int MODE>
static int igemm_grid_x_t(const ConvGeom& g) {
  const int S = igemm_ksplit_t<BM, BN, WM, WN, ST, MODE>(g);
  if (S > 1) {   // stats rows come from the reduce kernel
    int rpb;
    return splitk_reduce_grid(g.N * g.Ho * g.Wo, g.Co, &rpb);
  }
  const int gyz = cdiv(g.Cn, BN) * g.groups * (MODE == 2 ? 4 : 1);
  return persistent_grid_x(cdiv(igemm_rows<MODE>(g), BM), gyz, igemm_occupancy<BM, BN, WM, WN, ST, MODE>());
}

template <int BM, int BN, int WM, int WN, int ST, int MODE>
static int64_t igemm_ws_floats_t(const ConvGeom& g) {
  const int S = igemm_ksplit_t<BM, BN, WM, WN, ST, MODE>(g);
  return S > 1 ? (int64_t)S * g.N * g.Ho * g.Wo * g.Co : 0;
}

template <int BM, int BN, int WM, int WN, int ST, int MODE>
static void launch_igemm(const bf16* A, const bf16* B, bf16* Y, float* stats, const float* bias,
                         const ConvGeom& g0, hipStream_t st, const bf16* addend = nullptr,
                         float* ws = nullptr) {
  const int S = ws ? igemm_ksplit_t<BM, BN, WM, WN, ST, MODE>(g0) : 1;
  if (S > 1) {
    ConvGeom g = g0;
    g.ksplit = S;
    g.ws = ws;
    const int gzb = g.groups * (MODE == 2 ? 4 : 1);
    dim3 grid(cdiv(igemm_rows<MODE>(g), BM), cdiv(g.Cn, BN), gzb * S);
    hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, ST, MODE, false, true>), grid,
                       dim3(WM * WN * 64), 0, st, A, B, Y, nullptr, nullptr, nullptr, g);
    const int M = g.N * g.Ho * g.Wo;
    int rpb;
    const int gx = splitk_reduce_grid(M, g.Co, &rpb);
    if (g.addend_s2c) addend = nullptr;   // (tuning trials only: bindings expand it for real calls)
    if (stats)
      hipLaunchKernelGGL(splitk_reduce_kernel<true>, dim3(gx), dim3(256), 0, st, ws, S, M, g.Co,
                         rpb, bias, addend, Y, stats, g.bn_y, g.bn_mask, g.bn_aux, g.bn_part, g.shards, g.bn_y2, g.bn_aux2,
                         g.kshift, 0);
    else
      hipLaunchKernelGGL(splitk_reduce_kernel<false>, dim3(gx), dim3(256), 0, st, ws, S, M, g.Co,
                         rpb, bias, addend, Y, stats, g.bn_y, g.bn_mask, g.bn_aux, g.bn_part, g.shards, g.bn_y2, g.bn_aux2,
                         nullptr, g.bn_ldy);
    return;
  }
  const ConvGeom& g = g0;
  dim3 grid(igemm_grid_x_t<BM, BN, WM, WN, ST, MODE>(g), cdiv(g.Cn, BN),
            g.groups * (MODE == 2 ? 4 : 1));
  if (stats)
    hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, ST, MODE, true>), grid,
                       dim3(WM * WN * 64), 0, st, A, B, Y, stats, bias, addend, g);
  else
    hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, WM, WN, ST, MODE, false>), grid,
                       dim3(WM * WN * 64), 0, st, A, B, Y, stats, bias, addend, g);
}

// Tile configurations. The heuristic picks by GEMM N (channels per group); a process-wide
// override (set_conv_tile) lets tools/bench_conv.py sweep them on the GPU.

void set_conv_tile(int kind, int idx) {
  if (kind == 0) g_igemm_override = idx;
  else if (kind == 1) g_wgrad_override = idx;
  else g_splitk_override = idx;
}

static int igemm_select(const ConvGeom& g) {
  if (g_igemm_override >= 0) return g_igemm_override;
  if (g_trial_cfg >= 0) return g_trial_cfg;
  if (const auto* t = tuned_choice(g)) return t->first;
  // measured on MI355X (tools/bench_conv.py, profiles/conv_census_r1.md)
  if (g.Cn > 64) return 3;
  if (g.Cn > 32) return 4;
  return 8;
}

// X(cfg, BM, BN, WM, WN, STAGES)
#define PCA_IGEMM_CFGS(X)            \
  X(0, 128, 128, 2, 2, 3)            \
  X(1, 128, 64, 2, 2, 4)             \
  X(2, 128, 32, 4, 1, 4)             \
  X(3, 128, 128, 2, 2, 2)            \
  X(4, 128, 64, 2, 2, 2)             \
  X(5, 128, 64, 4, 1, 3)             \
  X(6, 256, 64, 4, 1, 3)             \
  X(7, 256, 128, 2, 2, 2)            \
  X(8, 128, 32, 4, 1, 2)             \
  X(9, 256, 128, 4, 2, 3)            \
  X(10, 256, 64, 4, 2, 3)            \
  X(11, 256, 64, 4, 2, 4)            \
  X(12, 256, 128, 4, 2, 2)           \
  X(13, 512, 64, 8, 1, 2)            \
  X(14, 128, 128, 2, 4, 3)           \
  X(15, 128, 64, 4, 2, 4)            \
  X(16, 64, 128, 1, 4, 3)            \
  X(17, 64, 64, 2, 2, 3)             \
  X(18, 64, 64, 1, 4, 4)

// ---- phased 256-row kernel: cfg 20 (BN 256, 8 waves), 21 (BN 128, 8 waves),
//      22 (BN 256, 4 waves: 128x128 per wave, 1 wave/SIMD), 23 (BN 128, 4 waves) ----
static bool ph_eligible(const ConvGeom& g, int mode) {
  return g.Cr % 64 == 0 && (mode == 0 || (mode == 1 && g.stride == 1));
}

template <int BN, int WAVES, int MODE>
static int ph_occupancy() {
  static int occ = 0;
  if (occ == 0)
    occ = std::min(
        blocks_per_cu((const void*)conv_igemm_ph_kernel<BN, WAVES, MODE, true>, WAVES * 64, "igemm_ph"),
        blocks_per_cu((const void*)conv_igemm_ph_kernel<BN, WAVES, MODE, false>, WAVES * 64, "igemm_ph"));
  return occ;
}

template <int BN, int WAVES, int MODE>
static int ph_grid_x(const ConvGeom& g) {
  return persistent_grid_x(cdiv(g.M, 256), cdiv(g.Cn, BN) * g.groups, ph_occupancy<BN, WAVES, MODE>());
}

template <int BN, int WAVES, int MODE>
static void launch_ph(const bf16* A, const bf16* B, bf16* Y, float* stats, const float* bias,
                      const ConvGeom& g, hipStream_t st, const bf16* addend) {
  dim3 grid(ph_grid_x<BN, WAVES, MODE>(g), cdiv(g.Cn, BN), g.groups);
  if (stats)
    hipLaunchKernelGGL((conv_igemm_ph_kernel<BN, WAVES, MODE, true>), grid, dim3(WAVES * 64), 0, st,
                       A, B, Y, stats, bias, addend, g);
  else
    hipLaunchKernelGGL((conv_igemm_ph_kernel<BN, WAVES, MODE, false>), grid, dim3(WAVES * 64), 0, st,
                       A, B, Y, stats, bias, addend, g);
}

// ---- halo-staged 3x3 kernel (conv3x3_hx.hip): cfg 30, forward and stride-1 dgrad ----
constexpr int kHxCfg = 30;
bool conv_hx_applicable(int N, int H, int W, int CA, int CO, int KH, int KW, int stride, int pad,
                        int groups);
int conv_hx_launch(const bf16* a, const bf16* b, bf16* y, float* stats, const bf16* addend,
                   const float* bias, int N, int H, int CA, int CO, int mode, hipStream_t st,
                   const bf16* bn_y, const uint8_t* bn_mask, const float* bn_aux, float* bn_part,
                   bool launch, const bf16* bn_y2 = nullptr, const float* bn_aux2 = nullptr);
bool conv_hx_s2_applicable(int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride,
                           int pad, int groups, int Ho, int Wo);
bool conv_hx_dual();
void conv_hx_set_addend_s2c(int on);
void conv_hx_s2_weights(const bf16* wt, int Cin, int Cout, bf16* w2, hipStream_t st);
// (for a dgrad geometry g: Hs/Ws/Cs = dY, Ho/Wo/Co = dX)
static bool hx_ok(const ConvGeom& g, int mode) {
  if (mode == 2)
    return conv_hx_s2_applicable(g.N, g.Ho, g.Wo, g.Co, g.Cs, g.KH, g.KW, g.stride, g.pad, g.groups,
                                 g.Hs, g.Ws);
  return (mode == 0 || mode == 1) && g.Ho == g.Hs && g.Wo == g.Ws &&
         conv_hx_applicable(g.N, g.Hs, g.Ws, g.Cs, g.Co, g.KH, g.KW, g.stride, g.pad, g.groups);
}
// stride-2 dgrad: bf16 2x2 class weights live in the launch workspace (in floats)
static int64_t hx_s2_ws_floats(const ConvGeom& g) { return (int64_t)16 * g.Co * g.Cs / 2; }
static int igemm_select(const ConvGeom& g);
template <int MODE>
static bool use_hx(const ConvGeom& g) {
  return igemm_select(g) == kHxCfg && hx_ok(g, MODE);
}
template <int MODE>
static int hx_grid(const ConvGeom& g) {
  return conv_hx_launch(nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, g.N, g.Hs, g.Cs,
                        MODE == 2 ? 4 * g.Co : g.Co, MODE, nullptr, nullptr, nullptr, nullptr, nullptr,
                        false);
}

// cfg of the phased kernel to use for this launch, or -1 (generic tile configs)
template <int MODE>
static int ph_cfg(const ConvGeom& g) {
  if constexpr (MODE == 2) {
    return -1;
  } else {
    const int c = igemm_select(g);
    return (c >= 20 && c <= 23) && ph_eligible(g, MODE) ? c : -1;
  }
}

template <int MODE>
static bool ph_launch(int pc, const bf16* A, const bf16* B, bf16* Y, float* stats,
                      const float* bias, const ConvGeom& g, hipStream_t st, const bf16* addend) {
  if constexpr (MODE == 2) {
    return false;
  } else {
    switch (pc) {
      case 20: launch_ph<256, 8, MODE>(A, B, Y, stats, bias, g, st, addend); return true;
      case 21: launch_ph<128, 8, MODE>(A, B, Y, stats, bias, g, st, addend); return true;
      case 22: launch_ph<256, 4, MODE>(A, B, Y, stats, bias, g, st, addend); return true;
      case 23: launch_ph<128, 4, MODE>(A, B, Y, stats, bias, g, st, addend); return true;
      default: return false;
    }
  }
}

template <int MODE>
static int ph_grid(int pc, const ConvGeom& g) {
  if constexpr (MODE == 2) {
    return 0;
  } else {
    switch (pc) {
      case 20: return ph_grid_x<256, 8, MODE>(g);
      case 21: return ph_grid_x<128, 8, MODE>(g);
      case 22: return ph_grid_x<256, 4, MODE>(g);
      case 23: return ph_grid_x<128, 4, MODE>(g);
      default: return 0;
    }
  }
}

template <int MODE>
static void igemm_dispatch(const bf16* A, const bf16* B, bf16* Y, float* stats, const float* bias,
                           const ConvGeom& g, hipStream_t st, const bf16* addend = nullptr,
                           float* ws = nullptr) {
  if (ph_launch<MODE>(ph_cfg<MODE>(g), A, B, Y, stats, bias, g, st, addend)) return;
  if (use_hx<MODE>(g)) {
    const bf16* Bw = B;
    if constexpr (MODE == 2) {   // the 2x2 class weights, into the workspace
      bf16* w2 = reinterpret_cast<bf16*>(ws);
      conv_hx_s2_weights(B, g.Co, g.Cs, w2, st);
      Bw = w2;
    }
    conv_hx_set_addend_s2c(MODE == 2 ? g.addend_s2c : 0);
    conv_hx_launch(A, Bw, Y, stats, addend, bias, g.N, g.Hs, g.Cs, MODE == 2 ? 4 * g.Co : g.Co,
                   MODE, st, g.bn_y, g.bn_mask, g.bn_aux, g.bn_part, true, g.bn_y2, g.bn_aux2);
    conv_hx_set_addend_s2c(0);
    return;
  }
  switch (igemm_select(g)) {
#define PCA_CASE(C, BM, BN, WM, WN, ST) \
    case C: launch_igemm<BM, BN, WM, WN, ST, MODE>(A, B, Y, stats, bias, g, st, addend, ws); break;
    PCA_IGEMM_CFGS(PCA_CASE)
#undef PCA_CASE
    default: launch_igemm<128, 128, 2, 2, 2, MODE>(A, B, Y, stats, bias, g, st, addend, ws); break;
  }
}

template <int MODE>
static int64_t igemm_ws_floats(const ConvGeom& g) {
  if (ph_cfg<MODE>(g) >= 0) return 0;   // no split-K in the phased kernel
  if (use_hx<MODE>(g)) return MODE == 2 ? hx_s2_ws_floats(g) : 0;
  switch (igemm_select(g)) {
#define PCA_CASE(C, BM, BN, WM, WN, ST) \
    case C: return igemm_ws_floats_t<BM, BN, WM, WN, ST, MODE>(g);
    PCA_IGEMM_CFGS(PCA_CASE)
#undef PCA_CASE
    default: return igemm_ws_floats_t<128, 128, 2, 2, 2, MODE>(g);
  }
}

template <int MODE>
static int igemm_grid_x(const ConvGeom& g) {
  if (const int pc = ph_cfg<MODE>(g); pc >= 0) return ph_grid<MODE>(pc, g);
  if (use_hx<MODE>(g)) return hx_grid<MODE>(g);
  switch (igemm_select(g)) {
#define PCA_CASE(C, BM, BN, WM, WN, ST) \
    case C: return igemm_grid_x_t<BM, BN, WM, WN, ST, MODE>(g);
    PCA_IGEMM_CFGS(PCA_CASE)
#undef PCA_CASE
    default: return igemm_grid_x_t<128, 128, 2, 2, 2, MODE>(g);
  }
}

// number of BN-statistics slab rows the forward launch will write (= grid.x)
// ResNet layer-1 specialisation (conv3x3_c64.hip)
// stem.hip: 3x3 forward on the 8-channel padded RGB input
bool conv_stem_applicable(int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride,
                          int pad, int groups);
int conv_stem_stat_rows(int N, int H);
void conv_stem_fwd_launch(const bf16* x, const bf16* w, const float* bias, bf16* y, float* stats,
                          int N, int H, int Cout, hipStream_t st);

bool conv_c64_applicable(int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride,
                         int pad, int groups);
int conv_c64_stat_rows(int N, int H);
bool conv_c64_xf_active();
void conv_c64_launch(const bf16* a, const bf16* w, bf16* y, float* stats, const bf16* addend,
                     int N, int H, bool dgrad, hipStream_t st, const bf16* bn_y = nullptr,
                     const uint8_t* bn_mask = nullptr, const float* bn_aux = nullptr,
                     float* bn_part = nullptr);

// split-K workspace (floats) the forward / dgrad launch of this geometry will need (0 = none)
int64_t conv_fwd_ws_floats(int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride,
                           int pad, int groups, int Ho, int Wo, bool has_bias) {
  if (g_igemm_override < 0 && !has_bias &&
      conv_c64_applicable(N, H, W, Cin, Cout, KH, KW, stride, pad, groups))
    return 0;
  if (g_igemm_override < 0 && conv_stem_applicable(N, H, W, Cin, Cout, KH, KW, stride, pad, groups))
    return 0;
  ConvGeom g = make_geom(N, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, groups, Cin / groups,
                         Cout / groups);
  return igemm_ws_floats<0>(g);
}

// geometry of a dgrad launch (mode 1 generic / 2 parity classes)
static ConvGeom dgrad_geom(int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride,
                           int pad, int groups, int Ho, int Wo);

static bool dgrad_parity(int H, int W, int stride, int Ho, int Wo) {
  return stride == 2 && H % 2 == 0 && W % 2 == 0 && Ho == H / 2 && Wo == W / 2;
}

// compact stride-2 addend (ConvGeom::addend_s2c) of the next dgrad launches (bindings scope it)
static int g_addend_s2c = 0;
void conv_set_addend_s2c(int on) { g_addend_s2c = on; }

// can the dgrad this geometry selects take a compact stride-2 addend? (parity class 0 adds it:
// the halo stride-2 kernel and the unsplit parity igemm; c64 / split-K / generic gather cannot)
bool conv_dgrad_s2c_ok(int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride, int pad,
                       int groups, int Ho, int Wo) {
  if (g_igemm_override < 0 && conv_c64_applicable(N, H, W, Cin, Cout, KH, KW, stride, pad, groups))
    return false;
  const ConvGeom g = dgrad_geom(N, H, W, Cin, Cout, KH, KW, stride, pad, groups, Ho, Wo);
  if (g.mode != 2 || ph_cfg<2>(g) >= 0) return false;
  if (use_hx<2>(g)) return true;
  return igemm_ws_floats<2>(g) == 0;
}

int64_t conv_dgrad_ws_floats(int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride,
                             int pad, int groups, int Ho, int Wo) {
  if (g_igemm_override < 0 && conv_c64_applicable(N, H, W, Cin, Cout, KH, KW, stride, pad, groups))
    return 0;
  const ConvGeom g = dgrad_geom(N, H, W, Cin, Cout, KH, KW, stride, pad, groups, Ho, Wo);
  return g.mode == 2 ? igemm_ws_floats<2>(g) : igemm_ws_floats<1>(g);
}

static ConvGeom dgrad_geom(int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride,
                           int pad, int groups, int Ho, int Wo) {
  ConvGeom g = make_geom(N, Ho, Wo, Cout, H, W, Cin, KH, KW, stride, pad, groups, Cout / groups,
                         Cin / groups);
  g.mode = 1;
  if (dgrad_parity(H, W, stride, Ho, Wo)) {
    // parity-class decomposition: rows are one class's (H/2) x (W/2) pixels
    g.mode = 2;
    g.fd_hw = make_fastdiv((H / 2) * (W / 2));
    g.fd_w = make_fastdiv(W / 2);
  }
  return g;
}

// Row stride of the fused BN reduce's y for the next dgrad launch(es) (0 = dense; bindings scope it
// around one call): generic igemm / split-K stride-1 dgrads only
static int g_bn_ldy = 0;
void conv_set_bn_ldy(int ld) { g_bn_ldy = ld; }

bool conv1x1_nk_applicable(int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride,
                           int pad, int groups);
int conv1x1_nk_stat_rows(int N, int H, int W);
void conv1x1_nk_launch(const bf16* x, const bf16* w, bf16* y, float* stats, int N, int H, int W,
                       int Cin, int Cout, hipStream_t st);
void conv1x1_nk_dgrad_launch(const bf16* dy, const bf16* wt, bf16* dx, int N, int H, int W,
                             int Cin, int Cout, const bf16* addend, const bf16* bn_y,
                             const uint8_t* bn_mask, const float* bn_aux, float* bn_part,
                             hipStream_t st);
// the data gradient of a 1x1 conv with a narrow output (Cout <= 64) is the narrow-K GEMM
static bool nk_dgrad_applicable(int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride,
                                int pad, int groups);

void conv_set_bn_dual(const bf16* y2, const float* aux2) {
  g_dual_y2 = y2;
  g_dual_aux2 = aux2;
}

// slab rows the fused BN-backward reduce of this dgrad launch writes (its grid / reduce grid),
// or 0 when the selected kernel cannot fuse it (the phased 256-row kernel; with a dual-BN request
// every kernel but the generic igemm / split-K stride-1 dgrad)
int conv_dgrad_bn_rows(int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride, int pad,
                       int groups, int Ho, int Wo) {
  const bool dual = g_dual_y2 != nullptr;
  // the layer-1 c64 kernel prefetches the fused reduce's y / mask (and the residual addend) at
  // tile start so they hide under its MFMA loop (read in its one-workgroup-per-CU epilogue they
  // cost +116 us per call at bs1024); PCA_C64_BN_FUSE=0 keeps the separate reduce for layer 1
  static const bool c64_fuse = [] {
    const char* e = getenv("PCA_C64_BN_FUSE");
    return !(e && e[0] == '0');
  }();
  if (g_igemm_override < 0 && conv_c64_applicable(N, H, W, Cin, Cout, KH, KW, stride, pad, groups))
    return c64_fuse && !dual && !g_bn_ldy ? conv_c64_stat_rows(N, H) : 0;
  const ConvGeom g = dgrad_geom(N, H, W, Cin, Cout, KH, KW, stride, pad, groups, Ho, Wo);
  if (g.Co % 8 != 0) return 0;
  // a row-strided y: the generic igemm / split-K stride-1 dgrads only
  if (g_bn_ldy && (dual || g.mode != 1 || ph_cfg<1>(g) >= 0 || use_hx<1>(g))) return 0;
  if (!dual && !g_bn_ldy && g_igemm_override < 0 &&
      nk_dgrad_applicable(N, H, W, Cin, Cout, KH, KW, stride, pad, groups))
    return conv1x1_nk_stat_rows(N, H, W);
  if (dual && (g.mode != 1 || ph_cfg<1>(g) >= 0 || (use_hx<1>(g) && !conv_hx_dual()))) return 0;
  if (g.mode == 2) {
    if (use_hx<2>(g)) return hx_grid<2>(g);   // one slab row per (tile group, class-channel block)
    if (igemm_ws_floats<2>(g) > 0) {
      int rpb;
      return splitk_reduce_grid(g.N * g.Ho * g.Wo, g.Co, &rpb);
    }
    return igemm_grid_x<2>(g) * 4;
  }
  if (ph_cfg<1>(g) >= 0) return 0;
  if (igemm_ws_floats<1>(g) > 0) {
    int rpb;
    return splitk_reduce_grid(g.N * g.Ho * g.Wo, g.Co, &rpb);
  }
  return igemm_grid_x<1>(g);
}

// ---- autotune API (bindings.cpp) ----
// kind 0: forward, 1: dgrad. Returns false when the geometry is not autotunable (c64 path,
// an explicit override is active) or is already tuned.
static bool tunable(const ConvGeom& g, bool c64) {
  return !c64 && g_igemm_override < 0 && g_splitk_override < 0 && g_trial_cfg < 0 &&
         !deterministic_conv() &&
         !tuned_choice(g);
}

bool conv_needs_tune(int kind, int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride,
                     int pad, int groups, int Ho, int Wo, bool has_bias) {
  const bool c64 = conv_c64_applicable(N, H, W, Cin, Cout, KH, KW, stride, pad, groups) &&
                   !(kind == 0 && has_bias);
  if (kind == 0) {
    ConvGeom g = make_geom(N, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, groups, Cin / groups,
                           Cout / groups);
    return tunable(g, c64 || conv_stem_applicable(N, H, W, Cin, Cout, KH, KW, stride, pad, groups) ||
                          (!has_bias && conv1x1_nk_applicable(N, H, W, Cin, Cout, KH, KW, stride,
                                                              pad, groups)));
  }
  return tunable(dgrad_geom(N, H, W, Cin, Cout, KH, KW, stride, pad, groups, Ho, Wo),
                 c64 || nk_dgrad_applicable(N, H, W, Cin, Cout, KH, KW, stride, pad, groups));
}

static bool nk_dgrad_applicable(int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride,
                                int pad, int groups) {
  static const bool on = [] {
    const char* e = getenv("PCA_CONV_NK_DGRAD");
    return !(e && e[0] == '0');
  }();
  return on && conv1x1_nk_applicable(N, H, W, Cout, Cin, KH, KW, stride, pad, groups);
}

// candidate (cfg, split) list for a geometry: tile shapes from 64x64 to 128x128, split-K 1..8
std::vector<std::pair<int, int>> conv_tune_candidates(int kind, int N, int H, int W, int Cin,
                                                      int Cout, int KH, int KW, int stride,
                                                      int pad, int groups, int Ho, int Wo) {
  ConvGeom g = kind == 0 ? make_geom(N, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, groups,
                                     Cin / groups, Cout / groups)
                         : dgrad_geom(N, H, W, Cin, Cout, KH, KW, stride, pad, groups, Ho, Wo);
  const int taps = g.mode == 2 ? cdiv(KH, 2) * cdiv(KW, 2) : KH * KW;
  const int KT = cdiv(taps * g.Cr, 64);
  const bool can_split = g.Co % 8 == 0 && g.Co <= kMaxSplitCo;
  std::vector<std::pair<int, int>> c;
  // every compiled tile config: BN in {32, 64, 128}, BM in {64, 128, 256, 512}, 4 or 8 waves,
  // 2-4 stages (the 8-wave / 256-row tiles win on large-M shapes, the 64-row ones at small M)
  static const int cfgs[] = {3, 0, 4, 1, 16, 17, 18, 5, 6, 7, 9, 10, 11, 12, 13, 14, 15, 2, 8};
  static const int bn_of[] = {128, 64, 32, 128, 64, 64, 64, 128, 32, 128, 64, 64, 128, 64, 128, 64, 128, 64, 64};
  if (ph_eligible(g, g.mode) && g.M >= 256 * 64) {   // phased 256-row kernel: large M only
    // cfg 20 (BN 256, 8 waves) spills at 2 waves/SIMD (256 registers) and cfg 22 (BN 256, 4
    // waves) past 512: not candidates
    // (cfg 23, the 4-wave form, measured 30-40 % slower everywhere: one wave per SIMD cannot
    // cover the DMA / LDS latency; not a candidate)
    if (g.Cn >= 128) c.emplace_back(21, 1);
  }
  if (hx_ok(g, g.mode)) c.emplace_back(kHxCfg, 1);   // halo-staged 3x3 (conv3x3_hx.hip; the
                                                      // stride-2 dgrad as its 2x2 class form)
  for (int cfg : cfgs) {
    if (bn_of[cfg] >= 128 && g.Cn <= 64) continue;   // 128-wide N tiles on <= 64 channels
    if (bn_of[cfg] <= 32 && g.Cn > 64) continue;     // 32-wide N tiles on wide layers
    for (int sp : {1, 2, 4, 8}) {
      if (sp > 1 && (!can_split || KT / sp < 2)) continue;
      c.emplace_back(cfg, sp);
    }
  }
  return c;
}

void conv_set_trial(int cfg, int split) {
  g_trial_cfg = cfg;
  g_trial_split = split;
}

void conv_record_tuned(int kind, int N, int H, int W, int Cin, int Cout, int KH, int KW,
                       int stride, int pad, int groups, int Ho, int Wo, int cfg, int split) {
  ConvGeom g = kind == 0 ? make_geom(N, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, groups,
                                     Cin / groups, Cout / groups)
                         : dgrad_geom(N, H, W, Cin, Cout, KH, KW, stride, pad, groups, Ho, Wo);
  g_tuned[tune_key(g)] = {cfg, split};
}

int conv_tuned_count() { return (int)g_tuned.size(); }
void conv_clear_tuned() { g_tuned.clear(); }

// (must pick the kernel conv_fwd_launch picks: a biased 64->64 layer-1-shaped conv — VGG16/19's
// second conv — runs on the igemm, whose statistics grid is larger than the c64 kernel's)
int conv_fwd_stat_rows(int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride, int pad,
                       int groups, int Ho, int Wo, bool has_bias) {
  if (g_igemm_override < 0 && !has_bias &&
      conv_c64_applicable(N, H, W, Cin, Cout, KH, KW, stride, pad, groups))
    return conv_c64_stat_rows(N, H);
  if (g_igemm_override < 0 && conv_stem_applicable(N, H, W, Cin, Cout, KH, KW, stride, pad, groups))
    return conv_stem_stat_rows(N, H);
  if (g_igemm_override < 0 && !has_bias &&
      conv1x1_nk_applicable(N, H, W, Cin, Cout, KH, KW, stride, pad, groups))
    return conv1x1_nk_stat_rows(N, H, W);
  ConvGeom g = make_geom(N, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, groups, Cin / groups,
                         Cout / groups);
  return igemm_grid_x<0>(g);
}

void conv_fwd_launch(const bf16* x, const bf16* w, const float* bias, bf16* y, float* stats, int N,
                     int H, int W, int Cin, int Cout, int KH, int KW, int stride, int pad,
                     int groups, int Ho, int Wo, hipStream_t st, float* ws) {
  if (g_igemm_override < 0 && bias == nullptr &&
      conv_c64_applicable(N, H, W, Cin, Cout, KH, KW, stride, pad, groups)) {
    conv_c64_launch(x, w, y, stats, nullptr, N, H, false, st);
    return;
  }
  if (conv_c64_xf_active()) {
    fprintf(stderr, "[pca] conv input transform: only the c64 forward applies it\n");
    abort();
  }
  if (g_igemm_override < 0 && conv_stem_applicable(N, H, W, Cin, Cout, KH, KW, stride, pad, groups)) {
    conv_stem_fwd_launch(x, w, bias, y, stats, N, H, Cout, st);
    return;
  }
  if (g_igemm_override < 0 && bias == nullptr &&
      conv1x1_nk_applicable(N, H, W, Cin, Cout, KH, KW, stride, pad, groups)) {
    conv1x1_nk_launch(x, w, y, stats, N, H, W, Cin, Cout, st);
    return;
  }
  ConvGeom g = make_geom(N, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, groups, Cin / groups,
                         Cout / groups);
  igemm_dispatch<0>(x, w, y, stats, bias, g, st, nullptr, ws);
}

// dx = conv^T(dy, W); wt is W transposed to [Cin][KH][KW][Cout/G].
void conv_dgrad_launch(const bf16* dy, const bf16* wt, bf16* dx, int N, int H, int W, int Cin,
                       int Cout, int KH, int KW, int stride, int pad, int groups, int Ho, int Wo,
                       hipStream_t st, const bf16* addend, float* ws, const bf16* bn_y,
                       const uint8_t* bn_mask, const float* bn_aux, float* bn_part) {
  if (g_igemm_override < 0 && conv_c64_applicable(N, H, W, Cin, Cout, KH, KW, stride, pad, groups)) {
    conv_c64_launch(dy, wt, dx, nullptr, addend, N, H, true, st, bn_y, bn_mask, bn_aux, bn_part);
    return;
  }
  if (g_igemm_override < 0 && !g_bn_ldy && !(bn_part && g_dual_y2) &&
      nk_dgrad_applicable(N, H, W, Cin, Cout, KH, KW, stride, pad, groups)) {
    conv1x1_nk_dgrad_launch(dy, wt, dx, N, H, W, Cin, Cout, addend, bn_y, bn_mask, bn_aux, bn_part,
                            st);
    return;
  }
  ConvGeom g = dgrad_geom(N, H, W, Cin, Cout, KH, KW, stride, pad, groups, Ho, Wo);
  g.bn_y = bn_y;
  g.bn_mask = bn_mask;
  g.bn_aux = bn_aux;
  g.bn_part = bn_part;
  g.addend_s2c = g.mode == 2 ? g_addend_s2c : 0;
  g.bn_ldy = bn_y ? g_bn_ldy : 0;
  if (bn_part && g_dual_y2 && g.mode == 1 && ph_cfg<1>(g) < 0 && (!use_hx<1>(g) || conv_hx_dual())) {
    g.bn_y2 = g_dual_y2;
    g.bn_aux2 = g_dual_aux2;
  }
  if (g.mode == 2) {
    igemm_dispatch<2>(dy, wt, dx, nullptr, nullptr, g, st, addend, ws);
  } else {
    igemm_dispatch<1>(dy, wt, dx, nullptr, nullptr, g, st, addend, ws);
  }
}

void set_deterministic_conv(bool on);
bool deterministic_conv();
void slab_reduce_launch(float* ws, float* dw, int splits, int64_t n, hipStream_t st);
int64_t slab_ws_floats(int splits, int64_t n);

// split-K plan of the generic wgrad kernel; returns the slab size (0 = atomics)
template <int BM, int BN>
static int64_t splitk_plan(WgradGeom& g, int target_blocks) {
  const int tiles = cdiv(g.cout_g, BM) * cdiv(g.Ktot, BN) * g.groups;
  int splits = cdiv(target_blocks, tiles);
  const int min_chunk = 512;
  splits = std::max(1, std::min(splits, cdiv(g.P, min_chunk)));
  if (wgrad_split_force() >= 1) splits = std::min(wgrad_split_force(), std::max(1, cdiv(g.P, 64)));
  int chunk = cdiv(g.P, splits);
  chunk = cdiv(chunk, 64) * 64;
  splits = cdiv(g.P, chunk);
  g.chunk = chunk;
  g.splits = splits;
  g.atomic = deterministic_conv() ? 0 : 1;
  return g.atomic ? 0 : slab_ws_floats(splits, (int64_t)g.groups * g.cout_g * g.Ktot);
}

template <int BM, int BN, int WM, int WN, int ST>
static void launch_wgrad(const bf16* x, const bf16* dy, float* dw, float* ws, WgradGeom g,
                         hipStream_t st, int target_blocks) {
  splitk_plan<BM, BN>(g, target_blocks);
  dim3 grid(cdiv(g.cout_g, BM), cdiv(g.Ktot, BN), g.splits * g.groups);
  hipLaunchKernelGGL((conv_wgrad_kernel<BM, BN, WM, WN, ST>), grid, dim3(256), 0, st, x, dy,
                     g.atomic ? dw : ws, g);
  if (!g.atomic) slab_reduce_launch(ws, dw, g.splits, (int64_t)g.groups * g.cout_g * g.Ktot, st);
}

// wide-kernel configurations: X(cfg, MB, NB, WM, WN)  (tile = 64*MB cout x 64*NB columns)
#define PCA_WIDE_CFGS(X) \
  X(16, 1, 9, 1, 4)      \
  X(17, 2, 9, 2, 4)      \
  X(18, 2, 4, 2, 2)      \
  X(19, 1, 4, 1, 4)      \
  X(20, 2, 8, 2, 4)      \
  X(21, 4, 4, 4, 2)

template <int MB, int NB, int WM, int WN>
static int wide_occupancy() {
  static int occ = 0;
  if (occ == 0) {
occ = blocks_per_cu((const void*)conv_wgrad_wide_kernel<MB, NB, WM, WN>, WM * WN * 64, "wgrad_wide");
  }
  return occ;
}

static WgradGeom wgrad_geom(int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride,
                            int pad, int groups, int Ho, int Wo) {
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
  g.chunk = 0; g.splits = 1; g.atomic = 1;
  return g;
}

static int wgrad_select(const WgradGeom& g) {
  const bool wide_ok = g.cin_g % 64 == 0 && g.cout_g % 64 == 0;
  int cfg = g_weff_cfg >= 32 ? -1 : g_weff_cfg;
  if (cfg >= 16 && !wide_ok) cfg = -1;
  if (cfg < 0) {
    // measured (tools/bench_conv.py): the wide kernel only pays with all 9 taps in a tile and
    // a stride of 1; strided / 1x1 wgrad stays on the split-K kernel
    if (wide_ok && g.Ktot >= 9 * 64 && g.stride == 1) cfg = g.cout_g <= 64 ? 16 : 18;
    else cfg = (g.cout_g > 64 && g.Ktot > 64) ? 3 : (g.cout_g > 32 ? 6 : 7);
  }
  return cfg;
}

// plan a wide launch: fills chunk/splits/atomic, returns the slab size in floats (0 = atomics)
template <int MB, int NB, int WM, int WN>
static int64_t wide_plan(WgradGeom& g) {
  const int tiles = cdiv(g.cout_g, 64 * MB) * cdiv(g.Ktot, 64 * NB) * g.groups;
  const int slots = wide_occupancy<MB, NB, WM, WN>() * num_cus();
  int splits = std::max(1, slots / tiles);
  splits = std::min(splits, std::max(1, cdiv(g.P, 256)));
  const int forced = wgrad_split_force();
  if (forced >= 1) splits = std::min(forced, std::max(1, cdiv(g.P, 32)));
  if (forced <= -2) splits = std::min(-forced, std::max(1, cdiv(g.P, 32)));   // slab, fixed count
  int chunk = cdiv(cdiv(g.P, splits), 32) * 32;
  splits = cdiv(g.P, chunk);
  g.chunk = chunk;
  g.splits = splits;
  // few partials per output: atomics; many: slab rows + one ordered reduce
  g.atomic = (!deterministic_conv() && (forced >= 1 || (forced == -1 && splits <= 8))) ? 1 : 0;
  return g.atomic ? 0 : slab_ws_floats(splits, (int64_t)g.groups * g.cout_g * g.Ktot);
}

template <int MB, int NB, int WM, int WN>
static void launch_wide(const bf16* x, const bf16* dy, float* dw, float* ws, WgradGeom g,
                        hipStream_t st) {
  const int64_t slab = wide_plan<MB, NB, WM, WN>(g);
  dim3 grid(cdiv(g.cout_g, 64 * MB), cdiv(g.Ktot, 64 * NB), g.splits * g.groups);
  hipLaunchKernelGGL((conv_wgrad_wide_kernel<MB, NB, WM, WN>), grid, dim3(WM * WN * 64), 0, st, x,
                     dy, g.atomic ? dw : ws, g);
  if (!g.atomic) slab_reduce_launch(ws, dw, g.splits, (int64_t)g.groups * g.cout_g * g.Ktot, st);
  (void)slab;
}

// halo-staged 3x3/s1 wgrad (conv_halo.hip); selected by default where it applies, or forced
// with set_conv_tile(1, 32 + halo cfg)
int64_t wgrad_halo_ws_floats(int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride,
                             int pad, int groups);
void wgrad_halo_launch(const bf16* x, const bf16* dy, float* dw, float* ws, int N, int H, int W,
                       int Cin, int Cout, int groups, hipStream_t st);
void set_halo_cfg(int cfg);
bool halo_xf_active();

// wgrad autotuning: (cfg, split) per geometry; cfg >= 32 = halo config cfg-32, 16..21 = wide,
// 0..7 = generic split-K; split -1 = occupancy-derived plan
static std::map<TuneKey, std::pair<int, int>> g_wtuned;
static int g_wtrial_cfg = -1, g_wtrial_split = -1;

static TuneKey wgrad_key(int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride,
                         int pad, int groups) {
  return TuneKey{{10, N, H, W, Cin, 0, 0, Cout, KH, KW, stride, pad, groups}};
}

static void wgrad_resolve(int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride,
                          int pad, int groups) {
  int cfg = g_wgrad_override, split = -1;
  if (cfg < 0 && g_wtrial_cfg >= 0) {
    cfg = g_wtrial_cfg;
    split = g_wtrial_split;
  } else if (cfg < 0) {
    auto it = g_wtuned.find(wgrad_key(N, H, W, Cin, Cout, KH, KW, stride, pad, groups));
    if (it != g_wtuned.end() && !deterministic_conv()) {
      cfg = it->second.first;
      split = it->second.second;
    }
  }
  // an X input transform (the BN applied on the operand loads) exists only in the halo kernel
  if (halo_xf_active() && cfg >= 0 && cfg < 32) {
    cfg = -1;
    split = -1;
  }
  g_weff_cfg = cfg;
  set_wgrad_split(split);
}

static bool use_halo() { return g_weff_cfg < 0 || g_weff_cfg >= 32; }

// workspace (floats) conv_wgrad_launch will need for this geometry under the current selection
int64_t conv_wgrad_ws_floats(int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride,
                             int pad, int groups, int Ho, int Wo) {
  wgrad_resolve(N, H, W, Cin, Cout, KH, KW, stride, pad, groups);
  if (use_halo()) {
    set_halo_cfg(g_weff_cfg >= 32 ? g_weff_cfg - 32 : -1);
    const int64_t h = wgrad_halo_ws_floats(N, H, W, Cin, Cout, KH, KW, stride, pad, groups);
    if (h >= 0) return h;
  }
  WgradGeom g = wgrad_geom(N, H, W, Cin, Cout, KH, KW, stride, pad, groups, Ho, Wo);
  const int target = 1024;
  switch (wgrad_select(g)) {
    case 4: return splitk_plan<128, 128>(g, 2048);
    case 5: return splitk_plan<128, 128>(g, 512);
    case 0: case 3: return splitk_plan<128, 128>(g, target);
    case 1: case 6: return splitk_plan<64, 128>(g, target);
    case 2: case 7: return splitk_plan<32, 128>(g, target);
#define PCA_CASE(C, MB, NB, WM, WN) \
    case C: return wide_plan<MB, NB, WM, WN>(g);
    PCA_WIDE_CFGS(PCA_CASE)
#undef PCA_CASE
    default: return splitk_plan<128, 128>(g, target);
  }
}

void conv_wgrad_launch(const bf16* x, const bf16* dy, float* dw, float* ws, int N, int H, int W,
                       int Cin, int Cout, int KH, int KW, int stride, int pad, int groups, int Ho,
                       int Wo, hipStream_t st) {
  wgrad_resolve(N, H, W, Cin, Cout, KH, KW, stride, pad, groups);
  if (use_halo()) {
    set_halo_cfg(g_weff_cfg >= 32 ? g_weff_cfg - 32 : -1);
    if (wgrad_halo_ws_floats(N, H, W, Cin, Cout, KH, KW, stride, pad, groups) >= 0) {
      wgrad_halo_launch(x, dy, dw, ws, N, H, W, Cin, Cout, groups, st);
      return;
    }
  }
  if (halo_xf_active()) {
    fprintf(stderr, "[pca] wgrad X transform: the halo kernel does not apply to this geometry\n");
    abort();
  }
  WgradGeom g = wgrad_geom(N, H, W, Cin, Cout, KH, KW, stride, pad, groups, Ho, Wo);
  const int target = 1024;
  switch (wgrad_select(g)) {
    case 0: launch_wgrad<128, 128, 2, 2, 3>(x, dy, dw, ws, g, st, target); break;
    case 1: launch_wgrad<64, 128, 2, 2, 3>(x, dy, dw, ws, g, st, target); break;
    case 2: launch_wgrad<32, 128, 1, 4, 3>(x, dy, dw, ws, g, st, target); break;
    case 3: launch_wgrad<128, 128, 2, 2, 2>(x, dy, dw, ws, g, st, target); break;
    case 4: launch_wgrad<128, 128, 2, 2, 3>(x, dy, dw, ws, g, st, 2048); break;
    case 5: launch_wgrad<128, 128, 2, 2, 3>(x, dy, dw, ws, g, st, 512); break;
    case 6: launch_wgrad<64, 128, 2, 2, 2>(x, dy, dw, ws, g, st, target); break;
    case 7: launch_wgrad<32, 128, 1, 4, 2>(x, dy, dw, ws, g, st, target); break;
#define PCA_CASE(C, MB, NB, WM, WN) \
    case C: launch_wide<MB, NB, WM, WN>(x, dy, dw, ws, g, st); break;
    PCA_WIDE_CFGS(PCA_CASE)
#undef PCA_CASE
    default: launch_wgrad<128, 128, 2, 2, 3>(x, dy, dw, ws, g, st, target); break;
  }
}

// ---- wgrad autotune API (bindings.cpp) ----
bool wgrad_needs_tune(int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride, int pad,
                      int groups) {
  if (g_wgrad_override >= 0 || g_wtrial_cfg >= 0 || deterministic_conv()) return false;
  return g_wtuned.find(wgrad_key(N, H, W, Cin, Cout, KH, KW, stride, pad, groups)) == g_wtuned.end();
}

std::vector<std::pair<int, int>> wgrad_tune_candidates(int N, int H, int W, int Cin, int Cout,
                                                       int KH, int KW, int stride, int pad,
                                                       int groups) {
  std::vector<int> cfgs;
  const bool halo = wgrad_halo_ws_floats(N, H, W, Cin, Cout, KH, KW, stride, pad, groups) >= 0;
  // (42-46: the 4-6 stage halo configs; PCA_HALO_DEEP=0 leaves them out of the search)
  static const bool deep = [] {
    const char* e = getenv("PCA_HALO_DEEP");
    return !(e && e[0] == '0');
  }();
  if (halo) cfgs.insert(cfgs.end(), {32, 33, 34, 35, 36, 37, 38, 39, 40, 41});
  if (halo && deep) cfgs.insert(cfgs.end(), {42, 43, 44, 45, 46});
  const int cin_g = Cin / groups, cout_g = Cout / groups;
  if (cin_g % 64 == 0 && cout_g % 64 == 0) cfgs.insert(cfgs.end(), {16, 17, 18, 19, 20, 21});
  cfgs.insert(cfgs.end(), {0, 1, 2, 3, 6, 7});
  const int64_t P = (int64_t)N * ((H + 2 * pad - KH) / stride + 1) * ((W + 2 * pad - KW) / stride + 1);
  std::vector<std::pair<int, int>> c;
  for (int cfg : cfgs)
    for (int sp : {-1, 1, 2, 4, 8, 16, 32, 64, -2, -4, -8, -16, -32, -64, -128}) {
      if (sp > 1 && P / sp < 256) continue;
      if (sp <= -2 && (cfg < 16 || P / -sp < 256)) continue;   // slab counts: halo / wide only
      c.emplace_back(cfg, sp);
    }
  return c;
}

void wgrad_set_trial(int cfg, int split) {
  g_wtrial_cfg = cfg;
  g_wtrial_split = split;
}

void wgrad_record_tuned(int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride, int pad,
                        int groups, int cfg, int split) {
  g_wtuned[wgrad_key(N, H, W, Cin, Cout, KH, KW, stride, pad, groups)] = {cfg, split};
}

int wgrad_tuned_count() { return (int)g_wtuned.size(); }
void wgrad_clear_tuned() { g_wtuned.clear(); }

// ---- tuning cache (PCA_TUNE_CACHE, _native.py): rows {table, key[13], cfg, split} ----
std::vector<std::vector<int>> tune_export() {
  std::vector<std::vector<int>> rows;
  int table = 0;
  for (const auto* m : {&g_tuned, &g_wtuned}) {
    for (const auto& kv : *m) {
      std::vector<int> r{table};
      r.insert(r.end(), kv.first.v, kv.first.v + 13);
      r.push_back(kv.second.first);
      r.push_back(kv.second.second);
      rows.push_back(std::move(r));
    }
    ++table;
  }
  return rows;
}

int tune_import(const std::vector<std::vector<int>>& rows) {
  int n = 0;
  for (const auto& r : rows) {
    if (r.size() != 16 || (r[0] != 0 && r[0] != 1)) continue;
    TuneKey k;
    std::copy(r.begin() + 1, r.begin() + 14, k.v);
    (r[0] == 0 ? g_tuned : g_wtuned)[k] = {r[14], r[15]};
    ++n;
  }
  return n;
}

}  // namespace pca
