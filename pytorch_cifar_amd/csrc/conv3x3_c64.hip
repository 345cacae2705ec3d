// 3x3 / stride-1 / pad-1 convolution with 64 input and 64 output channels on 32-wide images —
// the ResNet layer-1 shape (reference models/resnet.py:23-27 via nn.Conv2d(64, 64, 3, 1, 1) on
// 32x32 CIFAR maps; SURVEY §2.8 K1/K2, App. C: 27 % of ResNet-18's MACs), forward and dgrad.
//
// The generic implicit GEMM (conv_mfma.hip) is weak here: GEMM N = 64 caps its tile at 128x64,
// every K-step re-gathers the tap-shifted input through the texture path (9x the bytes of the
// input), and the weights are re-staged per tile. This kernel is laid out for the shape instead:
//   * the whole 64 x 576 weight matrix (72 KiB) is staged ONCE per persistent workgroup into
//     LDS (XOR-swizzled 16-byte chunks: conflict-free fragment reads) and stays resident,
//     each of the 4 waves owns 64 pixels x all 64 output channels,
//   * a 256-pixel tile (8 image rows) is staged ONCE into LDS as its halo (10 x 34 pixels x
//     128 B, LDS-DMA, XOR-swizzled 16-byte chunks), and the 9 taps are read from it at row
//     offsets kh*34 + kw (72 + 2 x 43 KiB = the whole 160 KiB LDS: one workgroup per CU),
//   * the halo of tile t+1 streams in (double buffer) while tile t computes; one wait per tile,
//   * epilogue: per-channel BatchNorm sum/sumsq partials (forward), the fused residual-gradient
//     addend (dgrad), bf16 tile staged through LDS for 16-byte coalesced stores.
// dgrad is the same kernel on dY with the transposed weights read at the mirrored tap (8 - tap).
#include "mfma_util.h"

namespace pca {

struct C64Geom {
  int N, H;        // images, rows (W == 32)
  int tiles;       // N * H / 8
  uint32_t a_bytes;
  // dgrad: fused backward reduce of the BN(+ReLU) that produced the conv input (see
  // conv_mfma.hip ConvGeom::bn_*); bn_part = nullptr disables it
  const bf16* bn_y;
  const uint8_t* bn_mask;
  const float* bn_aux;
  float* bn_part;   // [gridDim.x][2][64]
  int shards;       // stats / bn_part: 0 = slab rows, >0 = sharded atomic accumulator
};

namespace c64 {
constexpr int W = 32, W2 = 34, ROWS = 8;
constexpr int TILE = ROWS * W;                  // 256 output pixels
constexpr int HROWS = (ROWS + 2) * W2;          // 340 halo pixels
constexpr int HI = (HROWS + 7) / 8;             // 43 LDS-DMA instructions (1 KiB each)
constexpr int HBYTES = HI * 1024;
constexpr int NW = 4;                           // waves: 4 x (64 pixels, 64 channels)
constexpr int SLOTS = (HI + NW - 1) / NW;       // DMA instructions per wave per tile
constexpr int CST = 64 + 8;                     // staged C row stride (bf16)
constexpr int BBYTES = 64 * 576 * 2;           // resident weights
constexpr int BI = BBYTES / 1024;               // 72 DMA instructions
static_assert(TILE * CST * 2 <= HBYTES, "C tile must fit a halo buffer");
static_assert(BBYTES + 2 * HBYTES <= 160 * 1024, "LDS budget");
}  // namespace c64

template <bool DGRAD, bool STATS>
__global__ __launch_bounds__(256)
void conv3x3_c64_kernel(const bf16* __restrict__ A, const bf16* __restrict__ Wm,
                        bf16* __restrict__ Y, float* __restrict__ stats,
                        const bf16* __restrict__ addend, const C64Geom g) {
  using namespace c64;
  __shared__ __attribute__((aligned(16))) char smem[BBYTES + 2 * HBYTES];
  char* const Bs = smem + 2 * HBYTES;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid;                            // 64 pixels (2 image rows) x 64 channels
  const int tiles_per_img = g.H / ROWS;
  const __amdgpu_buffer_rsrc_t rsA = make_rsrc(A, g.a_bytes);

  // ---- DMA slots: halo rows hr = 8*i + (lane>>3), fixed (j, c) per lane and slot ----
  int s_jc[SLOTS], s_ch[SLOTS];
#pragma unroll
  for (int k = 0; k < SLOTS; ++k) {
    const int i = wid + NW * k;
    const int hr = 8 * i + (lane >> 3);
    const int j = hr / W2, c = hr - j * W2;
    s_jc[k] = (hr < HROWS) ? ((j << 8) | c) : -1;
    s_ch[k] = ((lane & 7) ^ (hr & 7)) << 4;       // logical chunk fetched into physical (lane&7)
  }
  auto issue = [&](int t, int buf) {
    const int n = t / tiles_per_img, h0 = (t - n * tiles_per_img) * ROWS;
    char* S = smem + buf * HBYTES;
#pragma unroll
    for (int k = 0; k < SLOTS; ++k) {
      const int i = wid + NW * k;
      if (i >= HI) continue;                       // wave-uniform
      uint32_t off = kOOB;
      if (s_jc[k] >= 0) {
        const int ih = h0 + (s_jc[k] >> 8) - 1, iw = (s_jc[k] & 0xff) - 1;
        if ((uint32_t)ih < (uint32_t)g.H && (uint32_t)iw < (uint32_t)W)
          off = (uint32_t)((((n * g.H + ih) * W + iw) * 64) * 2 + s_ch[k]);
      }
      dma16(rsA, S + i * 1024, off);
    }
  };

  if (blockIdx.x < g.tiles) issue(blockIdx.x, 0);

  // ---- weights -> LDS once: row n (output channel), 72 chunks of 8 K-values; physical chunk
  // pc holds logical chunk (pc & ~7) | ((pc ^ n) & 7). K order = (tap, input channel). ----
  {
    const __amdgpu_buffer_rsrc_t rsW = make_rsrc(Wm, BBYTES);
    for (int i = wid; i < BI; i += NW) {
      const int q = i * 64 + lane;
      const int n = q / 72, pc = q - n * 72;
      const int lc = (pc & ~7) | ((pc ^ n) & 7);
      const int tap = lc >> 3, c8 = lc & 7;
      const int src_tap = DGRAD ? 8 - tap : tap;
      dma16(rsW, Bs + i * 1024, (uint32_t)((n * 576 + src_tap * 64 + c8 * 8) * 2));
    }
  }

  // per-lane halo row of tap (0,0) for each A fragment: pixel (2*wm + (mi>>1), (mi&1)*16 + l&15)
  int rbase[4];
#pragma unroll
  for (int mi = 0; mi < 4; ++mi) rbase[mi] = (2 * wm + (mi >> 1)) * W2 + (mi & 1) * 16 + (lane & 15);
  const int kq = lane >> 4;                      // 8-channel chunk within a 32-channel half

  float st_s[4] = {0.f, 0.f, 0.f, 0.f}, st_q[4] = {0.f, 0.f, 0.f, 0.f};
  // fused BN-backward reduce (dgrad): this thread's store-loop channel group is tid & 7
  const bool bnf = DGRAD && g.bn_part != nullptr;
  float bs1[8], bs2[8], bmean[8], bistd[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    bs1[q] = bs2[q] = 0.f;
    bmean[q] = bnf ? g.bn_aux[(tid & 7) * 8 + q] : 0.f;
    bistd[q] = bnf ? g.bn_aux[64 + (tid & 7) * 8 + q] : 0.f;
  }

  constexpr int STORES = (TILE * 8) / 256;      // global stores per thread per tile
  wait_vmcnt<0>();                                // weights + first halo
  int it = 0;
  for (int t = blockIdx.x; t < g.tiles; t += gridDim.x, ++it) {
    const int buf = it & 1;
    // this tile's halo landed; the previous tile's output stores (issued after it, retired in
    // order) may stay in flight
    wait_vmcnt<STORES>();
    raw_barrier();
    if (t + (int)gridDim.x < g.tiles) issue(t + gridDim.x, buf ^ 1);
    const char* S = smem + buf * HBYTES;

    // epilogue operands of this tile (residual-gradient addend; BN input y + ReLU mask of the
    // fused backward reduce) are loaded now, so their latency hides under the 18 MFMA steps
    // instead of sitting in the epilogue of a one-workgroup-per-CU kernel
    uint4 pre_a[STORES], pre_y[STORES];
    uint32_t pre_m[STORES];
    {
      const int pn = t / tiles_per_img, ph0 = (t - pn * tiles_per_img) * ROWS;
      const size_t ppix0 = ((size_t)pn * g.H + ph0) * W;
#pragma unroll
      for (int q = 0; q < STORES; ++q) {
        const int idx = tid + q * 256;
        const size_t o = (ppix0 + (idx >> 3)) * 64 + (idx & 7) * 8;
        if (addend) pre_a[q] = *reinterpret_cast<const uint4*>(addend + o);
        if (bnf) {
          pre_y[q] = *reinterpret_cast<const uint4*>(g.bn_y + o);
          pre_m[q] = g.bn_mask[o >> 3];
        }
      }
    }

    f32x4 acc[4][4];
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = f32x4{0.f, 0.f, 0.f, 0.f};

    // K loop with the fragments of step s+1 read while step s's 16 MFMAs run (one wave per
    // SIMD: the LDS latency has to hide behind this wave's own MFMAs)
    auto load_step = [&](int s, bf16x8* af, bf16x8* bv) {
      const int tap = s >> 1, kh = tap / 3, kw = tap % 3;
      const int chunk = (s & 1) * 4 + kq;
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) {
        const int R = rbase[mi] + kh * W2 + kw;
        af[mi] = *reinterpret_cast<const bf16x8*>(S + R * 128 + ((chunk ^ (R & 7)) << 4));
      }
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const int n = ni * 16 + (lane & 15);
        const int lc = s * 4 + kq;
        const int pc = (lc & ~7) | ((lc ^ n) & 7);
        bv[ni] = *reinterpret_cast<const bf16x8*>(Bs + n * 1152 + pc * 16);
      }
    };
    bf16x8 fa[2][4], fb[2][4];
    load_step(0, fa[0], fb[0]);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 18; ++s) {
      const int cur = s & 1;
      if (s + 1 < 18) load_step(s + 1, fa[cur ^ 1], fb[cur ^ 1]);
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[cur][mi], fb[cur][ni], acc[mi][ni], 0, 0, 0);
    }
    __builtin_amdgcn_s_setprio(0);

    // ---- epilogue ----
    if constexpr (STATS) {
#pragma unroll
      for (int ni = 0; ni < 4; ++ni)
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float v = acc[mi][ni][j];
            st_s[ni] += v;
            st_q[ni] += v * v;
          }
    }
    raw_barrier();                                // every wave is done reading this halo
    bf16* Cs = reinterpret_cast<bf16*>(smem + buf * HBYTES);
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int p = wm * 64 + mi * 16 + (lane >> 4) * 4 + j;
          const int c = ni * 16 + (lane & 15);
          Cs[p * CST + c] = f2bf(acc[mi][ni][j]);
        }
    __syncthreads();
    const int n = t / tiles_per_img, h0 = (t - n * tiles_per_img) * ROWS;
    const size_t pix0 = ((size_t)n * g.H + h0) * W;
#pragma unroll
    for (int q = 0; q < (TILE * 8) / 256; ++q) {
      const int idx = tid + q * 256;
      const int p = idx >> 3, c8 = idx & 7;
      uint4 v = *reinterpret_cast<const uint4*>(Cs + p * CST + c8 * 8);
      const size_t o = (pix0 + p) * 64 + c8 * 8;
      if (addend) {
        float a[8], b[8];
        unpack8(v, a);
        unpack8(pre_a[q], b);
#pragma unroll
        for (int e = 0; e < 8; ++e) a[e] += b[e];
        v = pack8(a);
      }
      if (bnf) {
        float f[8], yy[8];
        unpack8(v, f);
        unpack8(pre_y[q], yy);
        const uint32_t m = pre_m[q];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float dz = ((m >> e) & 1u) ? f[e] : 0.f;
          bs1[e] += dz;
          bs2[e] += dz * (yy[e] - bmean[e]) * bistd[e];
        }
      }
      *reinterpret_cast<uint4*>(Y + o) = v;
    }
  }

  if constexpr (STATS) {
    wait_vmcnt<0>();
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem);  // [4 wm][64][2]
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      float s = st_s[ni], q = st_q[ni];
      s += __shfl_xor(s, 16, 64);
      s += __shfl_xor(s, 32, 64);
      q += __shfl_xor(q, 16, 64);
      q += __shfl_xor(q, 32, 64);
      if (lane < 16) {
        const int c = ni * 16 + lane;
        red[(wm * 64 + c) * 2 + 0] = s;
        red[(wm * 64 + c) * 2 + 1] = q;
      }
    }
    __syncthreads();
    if (tid < 64) {
      float s = 0.f, q = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        s += red[(w * 64 + tid) * 2 + 0];
        q += red[(w * 64 + tid) * 2 + 1];
      }
      stat_out(stats, blockIdx.x, g.shards, 128, tid, s);
      stat_out(stats, blockIdx.x, g.shards, 128, 64 + tid, q);
    }
  } else {
    wait_vmcnt<0>();
    if (bnf) {
      __syncthreads();
      float* red = reinterpret_cast<float*>(smem);  // [256][16]
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        red[tid * 16 + q] = bs1[q];
        red[tid * 16 + 8 + q] = bs2[q];
      }
      __syncthreads();
      if (tid < 8) {
        float a[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) a[q] = 0.f;
        for (int j = tid; j < 256; j += 8)
#pragma unroll
          for (int q = 0; q < 16; ++q) a[q] += red[j * 16 + q];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          stat_out(g.bn_part, blockIdx.x, g.shards, 128, tid * 8 + q, a[q]);
          stat_out(g.bn_part, blockIdx.x, g.shards, 128, 64 + tid * 8 + q, a[8 + q]);
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------------------
static int c64_grid(int tiles) {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
  }
  const int per = cdiv(tiles, cus);             // one persistent workgroup per CU
  return cdiv(tiles, per);
}

// shape gate (the caller falls back to the generic implicit GEMM otherwise)
bool conv_c64_applicable(int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride,
                         int pad, int groups) {
  static const bool off = [] {
    const char* e = getenv("PCA_CONV_C64");
    return e && e[0] == '0';
  }();
  return !off && Cin == 64 && Cout == 64 && KH == 3 && KW == 3 && stride == 1 && pad == 1 &&
         groups == 1 && W == 32 && H % 8 == 0 && N > 0;
}

int conv_c64_stat_rows(int N, int H) { return c64_grid(N * H / 8); }

void conv_c64_launch(const bf16* a, const bf16* w, bf16* y, float* stats, const bf16* addend,
                     int N, int H, bool dgrad, hipStream_t st, const bf16* bn_y,
                     const uint8_t* bn_mask, const float* bn_aux, float* bn_part) {
  C64Geom g;
  g.N = N;
  g.H = H;
  g.tiles = N * H / 8;
  g.a_bytes = (uint32_t)((size_t)N * H * 32 * 64 * 2);
  g.bn_y = bn_y;
  g.bn_mask = bn_mask;
  g.bn_aux = bn_aux;
  g.bn_part = dgrad ? bn_part : nullptr;
  g.shards = stat_shards();
  const dim3 grid(c64_grid(g.tiles)), block(256);
  if (dgrad)
    hipLaunchKernelGGL((conv3x3_c64_kernel<true, false>), grid, block, 0, st, a, w, y, nullptr,
                       addend, g);
  else if (stats)
    hipLaunchKernelGGL((conv3x3_c64_kernel<false, true>), grid, block, 0, st, a, w, y, stats,
                       addend, g);
  else
    hipLaunchKernelGGL((conv3x3_c64_kernel<false, false>), grid, block, 0, st, a, w, y, nullptr,
                       addend, g);
}

}  // namespace pca
