// Stem-conv weight gradient: 3x3, stride 1, pad 1, 3 input channels (RGB padded to 8 in the
// NHWC input the augmentation kernel writes), 32-wide images — the first conv of every CIFAR
// zoo model (resnet.py:102, vgg.py:33 first layer, mobilenetv2.py:58, efficientnet.py:136,
// regnet.py:84, dla.py:91 ...; reference executes it as cuDNN wgrad).
//
// As a GEMM it is dW[co][tap*3+ci] = sum_p dy[p][co] * x[p + tap][ci]: M = Cout, N = 27,
// K = N*H*W pixels (131072 at bs128, 1M at bs1024). The generic split-K wgrad spends most of its
// time on the 8-wide padded channel dimension and a full-size fp32 output per split; here:
//   * one workgroup walks 8-row image chunks (256 pixels = 8 MFMA K-steps of 32);
//   * the dy chunk is staged TRANSPOSED in LDS ([co][pixel], pixel pairs written as dwords so a
//     wave's stores hit 64 distinct banks), the x chunk as three column-shifted copies
//     xs[dw][ci][row][col] = x[row-1][col+dw-1][ci] so every B fragment (8 consecutive pixels of
//     one (tap, ci) column) is one aligned 16-byte LDS read;
//   * v_mfma_f32_16x16x32_bf16 accumulates Cout x 32 (27 used) per wave over its rows; the four
//     waves fold through LDS once per workgroup into one fp32 slab row of Cout*27 floats;
//   * stem_wgrad_reduce_kernel sums the slab rows in a fixed order and ADDS the result into the
//     fp32 gradient (physical [Cout][3][3][3]) — deterministic, no atomics, no padded copy.
#include "common.h"

#include <algorithm>
#include <cstdlib>

namespace pca {
namespace {
constexpr int kSW = 32;            // image width
constexpr int kSR = 8;             // output rows per chunk
constexpr int kSP = kSR * kSW;     // pixels per chunk
constexpr int kSPS = kSP + 8;      // bf16 row pitch of the transposed dy image (528 B: 16-lane
                                   // ds_read_b128 row reads land 4 banks apart, conflict-free)
constexpr int kSCI = 3;            // real input channels
constexpr int kSCS = 8;            // channel pitch of the padded NHWC input
constexpr int kSGrid = 512;        // workgroups (slab rows)
}  // namespace

template <int CO>
__global__ __launch_bounds__(256) void stem_wgrad_kernel(const bf16* __restrict__ x,
                                                         const bf16* __restrict__ dy, int N, int H,
                                                         float* __restrict__ slab) {
  constexpr int MT = CO / 16;
  constexpr int NO = 9 * kSCI;               // outputs per output channel (27)
  constexpr int NT = (NO + 15) / 16;         // N tiles (2)
  constexpr int XR = kSR + 2;                // x rows incl. the halo
  constexpr int DY_BYTES = CO * kSPS * 2;
  constexpr int RED_BYTES = 4 * CO * NT * 16 * 4;
  constexpr int U_BYTES = DY_BYTES > RED_BYTES ? DY_BYTES : RED_BYTES;
  __shared__ __attribute__((aligned(16))) char smem[U_BYTES];
  __shared__ __attribute__((aligned(16))) bf16 xs[3 * kSCI * XR * kSW];
  bf16* dyT = reinterpret_cast<bf16*>(smem);

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int cpi = H / kSR;                   // chunks per image
  const int chunks = N * cpi;

  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // B-fragment column of this lane: n = nt*16 + (lane & 15) -> (tap, ci); n >= 27 reads zeros
  int b_off[NT];
  bool b_ok[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int n = nt * 16 + (lane & 15);
    b_ok[nt] = n < NO;
    const int tap = b_ok[nt] ? n / kSCI : 0, ci = b_ok[nt] ? n % kSCI : 0;
    const int dh = tap / 3, dw = tap % 3;
    b_off[nt] = ((dw * kSCI + ci) * XR + dh) * kSW + 8 * (lane >> 4);
  }

  // Global loads of the next chunk are issued into registers before the current chunk's MFMAs
  // (software pipeline: with 2 workgroups per CU the loads would otherwise sit exposed between
  // the two barriers of every chunk).
  constexpr int CG = CO / 8;
  constexpr int DY_IT = (kSP / 2) * CG / 256;             // dy pixel-pair items per thread
  constexpr int X_ITEMS = 3 * XR * (kSW / 2);
  constexpr int X_IT = (X_ITEMS + 255) / 256;             // x items per thread
  static_assert((kSP / 2) * CG % 256 == 0, "dy items");
  uint4 ra[DY_IT], rb[DY_IT], xa[X_IT], xb[X_IT];
  auto load = [&](int ck) {
    const int n = ck / cpi, h0 = (ck - n * cpi) * kSR;
    const bf16* dyc = dy + (size_t)(n * H + h0) * kSW * CO;
#pragma unroll
    for (int i = 0; i < DY_IT; ++i) {
      const int e = tid + 256 * i;
      const int cg = e % CG, pp = e / CG;   // CG lanes read one pixel's channels: coalesced
      ra[i] = *reinterpret_cast<const uint4*>(dyc + (size_t)(2 * pp) * CO + cg * 8);
      rb[i] = *reinterpret_cast<const uint4*>(dyc + (size_t)(2 * pp + 1) * CO + cg * 8);
    }
#pragma unroll
    for (int i = 0; i < X_IT; ++i) {
      const int e = tid + 256 * i;
      const int cp = e % (kSW / 2);
      const int t = e / (kSW / 2);
      const int r = t % XR, dw = t / XR;
      const int hh = h0 - 1 + r;
      xa[i] = make_uint4(0, 0, 0, 0);
      xb[i] = make_uint4(0, 0, 0, 0);
      if (e < X_ITEMS && hh >= 0 && hh < H) {
        const int s0 = 2 * cp + dw - 1, s1 = s0 + 1;
        const bf16* row = x + (size_t)(n * H + hh) * kSW * kSCS;
        if (s0 >= 0) xa[i] = *reinterpret_cast<const uint4*>(row + s0 * kSCS);
        if (s1 < kSW) xb[i] = *reinterpret_cast<const uint4*>(row + s1 * kSCS);
      }
    }
  };
  if ((int)blockIdx.x < chunks) load(blockIdx.x);

  for (int ck = blockIdx.x; ck < chunks; ck += gridDim.x) {
    // dy chunk -> dyT[co][pixel] (pixel pairs as dwords). The 16-byte chunk (8 pixels) of row co
    // sits at chunk index (pixel / 8) ^ ((co / 8) & 7): the CG lanes of one pixel pair write 8
    // rows 8 apart, which the swizzle spreads over distinct banks (a plain pitch cannot also keep
    // the 16-row fragment reads conflict-free)
#pragma unroll
    for (int i = 0; i < DY_IT; ++i) {
      const int e = tid + 256 * i;
      const int cg = e % CG, pp = e / CG;
      const int col = ((((pp >> 2) ^ (cg & 7)) << 2) | (pp & 3)) * 2;   // swizzled pixel index
      const uint32_t aw[4] = {ra[i].x, ra[i].y, ra[i].z, ra[i].w};
      const uint32_t bw[4] = {rb[i].x, rb[i].y, rb[i].z, rb[i].w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t lo = (aw[q] & 0xffffu) | (bw[q] << 16);
        const uint32_t hi = (aw[q] >> 16) | (bw[q] & 0xffff0000u);
        *reinterpret_cast<uint32_t*>(dyT + (cg * 8 + 2 * q) * kSPS + col) = lo;
        *reinterpret_cast<uint32_t*>(dyT + (cg * 8 + 2 * q + 1) * kSPS + col) = hi;
      }
    }
    // x rows h0-1 .. h0+kSR, three column shifts xs[dw][ci][r][c] = x[h0-1+r][c+dw-1][ci]
#pragma unroll
    for (int i = 0; i < X_IT; ++i) {
      const int e = tid + 256 * i;
      if (e < X_ITEMS) {
        const int cp = e % (kSW / 2);
        const int t = e / (kSW / 2);
        const int r = t % XR, dw = t / XR;
        const uint32_t aw[2] = {xa[i].x, xa[i].y}, bw[2] = {xb[i].x, xb[i].y};
#pragma unroll
        for (int ci = 0; ci < kSCI; ++ci) {
          const uint32_t av = (ci & 1) ? (aw[ci >> 1] >> 16) : (aw[ci >> 1] & 0xffffu);
          const uint32_t bv = (ci & 1) ? (bw[ci >> 1] & 0xffff0000u) : (bw[ci >> 1] << 16);
          *reinterpret_cast<uint32_t*>(xs + ((dw * kSCI + ci) * XR + r) * kSW + 2 * cp) = av | bv;
        }
      }
    }
    __syncthreads();
    if (ck + (int)gridDim.x < chunks) load(ck + gridDim.x);
    // wave wid: chunk rows wid and wid + 4 (one 32-pixel K-step each)
#pragma unroll
    for (int r = wid; r < kSR; r += 4) {
      bf16x8 bfr[NT];
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(xs + b_off[nt] + r * kSW);
        bfr[nt] = b_ok[nt] ? v : bf16x8{};
      }
      const int kc = r * (kSW / 8) + (lane >> 4);   // 8-pixel chunk of this lane's K slice
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int co = mt * 16 + (lane & 15);
        const bf16x8 a =
            *reinterpret_cast<const bf16x8*>(dyT + co * kSPS + ((kc ^ ((co >> 3) & 7)) << 3));
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bfr[nt], acc[mt][nt], 0, 0, 0);
      }
    }
    __syncthreads();
  }

  // fold the four waves, one slab row per workgroup
  float* red = reinterpret_cast<float*>(smem);   // [4][CO][NT*16]
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int co = mt * 16 + 4 * (lane >> 4) + j, nn = nt * 16 + (lane & 15);
        red[(wid * CO + co) * (NT * 16) + nn] = acc[mt][nt][j];
      }
  __syncthreads();
  float* row = slab + (size_t)blockIdx.x * CO * NO;
  for (int e = tid; e < CO * NO; e += 256) {
    const int co = e / NO, nn = e - co * NO;
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) s += red[(w * CO + co) * (NT * 16) + nn];
    row[e] = s;
  }
}

// out[o] += sum_b slab[b][o], b in a fixed order: 8 outputs x 32 partial lanes per workgroup,
// each lane with 4 independent partial sums (loads in flight instead of one dependent chain).
__global__ __launch_bounds__(256) void stem_wgrad_reduce_kernel(const float* __restrict__ slab,
                                                                int nb, int total,
                                                                float* __restrict__ out) {
  __shared__ float part[32][9];
  const int c = threadIdx.x & 7, s = threadIdx.x >> 3;
  const int o = blockIdx.x * 8 + c;
  float v0 = 0.f, v1 = 0.f, v2 = 0.f, v3 = 0.f;
  if (o < total) {
    int b = s;
    for (; b + 96 < nb; b += 128) {
      v0 += slab[(size_t)b * total + o];
      v1 += slab[(size_t)(b + 32) * total + o];
      v2 += slab[(size_t)(b + 64) * total + o];
      v3 += slab[(size_t)(b + 96) * total + o];
    }
    for (; b < nb; b += 32) v0 += slab[(size_t)b * total + o];
  }
  part[s][c] = (v0 + v1) + (v2 + v3);
  __syncthreads();
  if (threadIdx.x < 8 && o < total) {
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < 32; ++q) t += part[q][c];
    out[o] += t;
  }
}

// ---------------------------------------------------------------------------------------
// Stem forward: y[p][co] = sum_{tap, ci < 8} x[p + tap][ci] * W[co][tap][ci] on the 8-channel
// padded NHWC input (the batched weight prep pads W's channels with zeros). The generic igemm
// runs this as K = 72 over two 64-wide K-steps with a per-granule gather. Here:
//   * a workgroup walks 8-row chunks (256 pixels); the chunk's halo (10 x 34 pixels x 16 B)
//     is staged once in LDS with zero borders;
//   * the MFMA K axis is (tap, 8 channels): one K-step of v_mfma_f32_16x16x32_bf16 covers four
//     taps, so every A fragment is ONE aligned 16-byte LDS read (the lane's pixel shifted by its
//     tap) and every B fragment one 16-byte weight row; three K-steps cover the nine taps
//     (slots 9-11 are zero), the weight fragments stay in registers for the whole kernel;
//   * wave w owns chunk rows 2w, 2w+1 (64 pixels x Cout); the bf16 tile goes out through LDS as
//     16-byte coalesced row stores; the BatchNorm partial sums (sum, sumsq of the fp32 outputs)
//     accumulate over all the workgroup's chunks and leave once (stat_out: slab row or sharded
//     accumulator, like every conv epilogue).
// ---------------------------------------------------------------------------------------
namespace {
constexpr int kFW2 = kSW + 2;            // halo row pitch (pixels)
constexpr int kFHP = (kSR + 2) * kFW2;   // halo pixels per chunk (340)
constexpr int kFGrid = 512;
}  // namespace

// (two blocks per CU: the CO = 64 variant otherwise took 218 + 64 registers, one wave per SIMD)
template <int CO>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void stem_fwd_kernel(const bf16* __restrict__ x,
                                                       const bf16* __restrict__ w,
                                                       const float* __restrict__ bias,
                                                       bf16* __restrict__ y, int N, int H,
                                                       float* __restrict__ stats, int shards,
                                                       const float* __restrict__ kshift) {
  constexpr int NT = CO / 16;
  constexpr int CST = CO + 8;                      // staged C row pitch (bf16)
  __shared__ __attribute__((aligned(16))) bf16 halo[kFHP * kSCS];
  __shared__ __attribute__((aligned(16))) bf16 ct[kSP * CST];
  __shared__ float red[4][2][CO];
  __shared__ float kks[CO];                        // statistics shift K (LDS: no live registers)

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int cpi = H / kSR, chunks = N * cpi;

  // weight fragments: B[k = (tap, ci)][n = co]; lane: co = nt*16 + lane%16, tap = 4*ks + lane/16
  bf16x8 bw[3][NT];
#pragma unroll
  for (int ks = 0; ks < 3; ++ks)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int tap = 4 * ks + (lane >> 4), co = nt * 16 + (lane & 15);
      bw[ks][nt] = tap < 9 ? *reinterpret_cast<const bf16x8*>(w + ((size_t)co * 9 + tap) * kSCS)
                           : bf16x8{};
    }
  float bb[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) bb[nt] = bias ? bias[nt * 16 + (lane & 15)] : 0.f;
  // A-fragment tap offsets (halo pixels) of this lane for the three K-steps
  int toff[3];
  bool tok[3];
#pragma unroll
  for (int ks = 0; ks < 3; ++ks) {
    const int tap = 4 * ks + (lane >> 4);
    tok[ks] = tap < 9;
    toff[ks] = tok[ks] ? (tap / 3) * kFW2 + tap % 3 : 0;
  }
  float st_s[NT], st_q[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) st_s[nt] = st_q[nt] = 0.f;
  for (int c = tid; c < CO; c += 256) kks[c] = kshift ? kshift[c] : 0.f;   // (first barrier below)

  // halo of a chunk: rows h0-1 .. h0+8, cols -1 .. 32, zeros outside the image; loaded into
  // registers one chunk ahead (issued before the current chunk's MFMAs and epilogue)
  constexpr int HI = (kFHP + 255) / 256;
  uint4 hv[HI];
  auto load = [&](int ck) {
    const int n = ck / cpi, h0 = (ck - n * cpi) * kSR;
#pragma unroll
    for (int i = 0; i < HI; ++i) {
      const int e = tid + 256 * i;
      const int r = e / kFW2, c = e - r * kFW2;
      const int hh = h0 - 1 + r, ww = c - 1;
      hv[i] = make_uint4(0, 0, 0, 0);
      if (e < kFHP && hh >= 0 && hh < H && ww >= 0 && ww < kSW)
        hv[i] = *reinterpret_cast<const uint4*>(x + ((size_t)(n * H + hh) * kSW + ww) * kSCS);
    }
  };
  if ((int)blockIdx.x < chunks) load(blockIdx.x);

  for (int ck = blockIdx.x; ck < chunks; ck += gridDim.x) {
    const int n = ck / cpi, h0 = (ck - n * cpi) * kSR;
#pragma unroll
    for (int i = 0; i < HI; ++i) {
      const int e = tid + 256 * i;
      if (e < kFHP) *reinterpret_cast<uint4*>(halo + e * kSCS) = hv[i];
    }
    __syncthreads();
    if (ck + (int)gridDim.x < chunks) load(ck + gridDim.x);
    f32x4 acc[4][NT];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      const int p = wid * 64 + mt * 16 + (lane & 15);          // chunk pixel of the A row
      const int base = (p >> 5) * kFW2 + (p & 31);             // its halo pixel at tap (0, 0)
#pragma unroll
      for (int ks = 0; ks < 3; ++ks) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(halo + (base + toff[ks]) * kSCS);
        const bf16x8 av = tok[ks] ? a : bf16x8{};
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bw[ks][nt], acc[mt][nt], 0, 0, 0);
      }
    }
    // epilogue: bias, statistics, bf16 tile through LDS
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float v = acc[mt][nt][j] + bb[nt];
          const float d = v - kks[nt * 16 + (lane & 15)];   // shifted sums (K = 0 unshifted)
          st_s[nt] += d;
          st_q[nt] += d * d;
          const int p = wid * 64 + mt * 16 + 4 * (lane >> 4) + j;
          ct[p * CST + nt * 16 + (lane & 15)] = f2bf(v);
        }
    __syncthreads();
    bf16* yc = y + (size_t)(n * H + h0) * kSW * CO;
    constexpr int CG = CO / 8;
    for (int e = tid; e < kSP * CG; e += 256) {
      const int p = e / CG, c8 = e - p * CG;
      *reinterpret_cast<uint4*>(yc + (size_t)p * CO + c8 * 8) =
          *reinterpret_cast<const uint4*>(ct + p * CST + c8 * 8);
    }
    // (the next chunk's halo writes do not touch ct; its barrier orders these reads before the
    // next epilogue's ct writes)
  }
  if (stats) {
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      float s1 = st_s[nt], s2 = st_q[nt];
      s1 += __shfl_xor(s1, 16, 64);
      s1 += __shfl_xor(s1, 32, 64);
      s2 += __shfl_xor(s2, 16, 64);
      s2 += __shfl_xor(s2, 32, 64);
      if (lane < 16) {
        red[wid][0][nt * 16 + lane] = s1;
        red[wid][1][nt * 16 + lane] = s2;
      }
    }
    __syncthreads();
    if (tid < 2 * CO) {
      const int k = tid / CO, c = tid - k * CO;
      const float v = red[0][k][c] + red[1][k][c] + red[2][k][c] + red[3][k][c];
      stat_out(stats, blockIdx.x, shards, 2 * CO, k * CO + c, v);
    }
    stat_krow(stats, shards, 2 * CO, kshift, CO);
  }
}

bool conv_stem_applicable(int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride,
                          int pad, int groups) {
  static const bool on = [] {
    const char* e = getenv("PCA_STEM_FWD");
    return !(e && e[0] == '0');
  }();
  return on && N > 0 && Cin == kSCS && KH == 3 && KW == 3 && stride == 1 && pad == 1 &&
         groups == 1 && W == kSW && H % kSR == 0 && (Cout == 16 || Cout == 32 || Cout == 64);
}

int conv_stem_stat_rows(int N, int H) { return std::min(kFGrid, N * (H / kSR)); }

// x [N][H][32][8] bf16, w [Cout][3][3][8] bf16, y [N][H][32][Cout] bf16; stats: slab rows
// [conv_stem_stat_rows][2][Cout] (shards 0) or the sharded accumulator (stat_shards() > 0)
void conv_stem_fwd_launch(const bf16* x, const bf16* w, const float* bias, bf16* y, float* stats,
                          int N, int H, int Cout, hipStream_t st) {
  const int grid = conv_stem_stat_rows(N, H), sh = stat_shards();
  const float* k = stats ? stat_shift() : nullptr;
  switch (Cout) {
    case 16: hipLaunchKernelGGL(stem_fwd_kernel<16>, dim3(grid), dim3(256), 0, st, x, w, bias, y, N, H, stats, sh, k); break;
    case 32: hipLaunchKernelGGL(stem_fwd_kernel<32>, dim3(grid), dim3(256), 0, st, x, w, bias, y, N, H, stats, sh, k); break;
    default: hipLaunchKernelGGL(stem_fwd_kernel<64>, dim3(grid), dim3(256), 0, st, x, w, bias, y, N, H, stats, sh, k); break;
  }
}

bool stem_wgrad_supported(int N, int H, int W, int Cs, int Ci, int Co) {
  return N > 0 && W == kSW && H % kSR == 0 && Cs == kSCS && Ci == kSCI &&
         (Co == 16 || Co == 32 || Co == 64);
}

int stem_wgrad_slab_rows(int N, int H) { return std::min(kSGrid, N * (H / kSR)); }

// x [N][H][32][8] bf16, dy [N][H][32][Co] bf16, slab [rows][Co*27] fp32, out [Co][3][3][3] fp32
void stem_wgrad_launch(const bf16* x, const bf16* dy, int N, int H, int Co, float* slab,
                       float* out, hipStream_t st) {
  const int rows = stem_wgrad_slab_rows(N, H);
  switch (Co) {
    case 16: hipLaunchKernelGGL(stem_wgrad_kernel<16>, dim3(rows), dim3(256), 0, st, x, dy, N, H, slab); break;
    case 32: hipLaunchKernelGGL(stem_wgrad_kernel<32>, dim3(rows), dim3(256), 0, st, x, dy, N, H, slab); break;
    default: hipLaunchKernelGGL(stem_wgrad_kernel<64>, dim3(rows), dim3(256), 0, st, x, dy, N, H, slab); break;
  }
  const int total = Co * 9 * kSCI;
  hipLaunchKernelGGL(stem_wgrad_reduce_kernel, dim3(cdiv(total, 8)), dim3(256), 0, st, slab, rows,
                     total, out);
}

}  // namespace pca
