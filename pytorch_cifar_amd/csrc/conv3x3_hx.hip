// Halo-staged implicit GEMM for the 3x3 / stride-1 / pad-1 convolutions of ResNet layers 2-4
// (reference models/resnet.py:23-27, 61-64 on 16x16 / 8x8 / 4x4 maps with 128-512 channels;
// SURVEY §2.8 K1/K2), forward and stride-1 dgrad.
//
// Why a separate kernel: in the generic implicit GEMM (conv_mfma.hip) every K-step re-gathers a
// tap-shifted copy of the input tile through LDS-DMA, so a 128x128 tile moves 32 KiB (32 DMA
// pieces) per 128x128x64 MACs. An LDS-DMA piece costs ~60-185 issue cycles of its wave, and at
// that rate the DMA issue, not the matrix core, bounds the kernel (~30-35 % MFMA busy,
// profiles/pmc_top10_r3.md). Here a workgroup owns whole images (BM = 128 / 256 pixels) and, per
// 64-channel input chunk, stages the images' zero-padded halo ONCE ((W+2)^2 rows per image); the
// nine taps read it at row offsets kh*(W+2) + kw. Per K-step only the weight tile (BN rows x
// 128 B) is staged: ~2.3x fewer DMA pieces per MAC than the 256x128 generic tile.
//
// Layout (cf. conv3x3_c64.hip, the 64-channel layer-1 version with resident weights):
//   * WM x WN waves, each 64 pixels x 64 output channels (4 x 4 16x16x32 MFMA tiles);
//   * the MFMA is issued as W x X^T with the weight rows staged in a permuted channel order, so a
//     lane's accumulators are 16 consecutive channels of one pixel: epilogue stores (bf16, and
//     the fused dgrad addend / BatchNorm-backward sums) go straight from registers;
//   * K loop = chunk (64 input channels) x tap (9) x half (32 channels); the weight tile of the
//     next tap and the halo of the next chunk (or of the next tile's first chunk) stream in while
//     the current one computes: one barrier + counted vmcnt per tap, weight ring of 2, halo ring
//     of 2;
//   * dgrad: the same kernel on dY with the transposed weights read at the mirrored tap 8 - t.
#include "mfma_util.h"

namespace pca {

struct HxGeom {
  int N;            // images
  int CA;           // channels of the gathered tensor (x: Cin, dgrad: dY's Cout)
  int CO;           // channels produced (forward: Cout, dgrad: Cin; stride-2 dgrad: 4 x Cin)
  int COUT;         // channels of the output tensor (CO, or Cin for the stride-2 dgrad)
  int KC;           // 64-channel chunks of CA
  int tiles;        // N * H * W / BM
  uint32_t a_bytes, b_bytes;
  int shards;       // stats / bn_part: 0 = slab rows, >0 = sharded atomic accumulator
  int add_s2c;      // stride-2 dgrad: compact [N][H/2][W/2][Cin] addend for class 0 only
  // dgrad: fused backward reduce of the BN(+ReLU) that produced this conv's input (bn_part != 0)
  const bf16* bn_y;
  const uint8_t* bn_mask;
  const float* bn_aux;
  float* bn_part;
  // MODE 3 (stride-1 dgrad of a projection-shortcut block tail act(BN(y) + BN2(y2))): the third
  // sum dz * xhat2 (accumulator rows of 3 sums)
  const bf16* bn_y2;
  const float* bn_aux2;
  const float* kshift;   // forward stats: per-channel shift K (common.h stat_shift), or nullptr
};

// dgrad: prefetch the fused BN reduce's y during the last tap (true) or load it at the epilogue
// (false: 36 fewer registers live across the MFMA loop; the 8-wave dgrads spilled with it)
#ifndef PCA_HX_PREFETCH_Y
#define PCA_HX_PREFETCH_Y 0
#endif
constexpr bool kHxPrefetchY = PCA_HX_PREFETCH_Y != 0;
#ifndef PCA_HX_DMA_AFTER_READ
#define PCA_HX_DMA_AFTER_READ 0
#endif
constexpr bool kHxDmaAfterRead = PCA_HX_DMA_AFTER_READ != 0;   // (forward only: the dgrad spills more)
// MODE 3 (dual-BN third sum) is compiled out: its 48 per-lane sums spill the 8-wave variants
// (180+ registers); the dual-BN block-tail dgrads stay on the generic igemm
constexpr bool kHxDual = false;
bool conv_hx_dual() { return kHxDual; }

__device__ __forceinline__ int hx_perm(int n) { return ((n >> 2) & 3) * 16 + (n >> 4) * 4 + (n & 3); }

template <int W, int IMGS, int WM, int WN, int TAPS = 9>
struct HxShape {
  static constexpr int NW = WM * WN;
  static constexpr int BM = WM * 64, BN = WN * 64;
  static constexpr int W2 = W + 2;
  static constexpr int IMG_ROWS = W2 * W2;
  static constexpr int HROWS = IMGS * IMG_ROWS;
  static constexpr int HI = (HROWS + 7) / 8;          // halo DMA pieces per chunk
  static constexpr int HBYTES = HI * 1024;
  static constexpr int HS = (HI + NW - 1) / NW;       // halo pieces per wave per chunk
  static constexpr int BPC = BN / 8;                  // weight pieces per tap
  static constexpr int BS = BPC / NW;                 // ... per wave
  static constexpr int BBYTES = BN * 128;
  static constexpr int LDS = 2 * HBYTES + 2 * BBYTES + 1024 + BN * 16;
  static_assert(IMGS * W * W == BM, "a tile is whole images");
  static_assert(BPC % NW == 0, "weight pieces split evenly over the waves");
  // halo piece k is issued during tap k % (TAPS-1) (the last tap stages the next chunk's weights)
  static constexpr int pieces_at(int tap) {
    return tap >= TAPS - 1 ? 0 : (HS - tap + TAPS - 2) / (TAPS - 1);
  }
  static_assert(HS <= 3 * (TAPS - 1), "at most three halo pieces per tap");
  static_assert(LDS <= 160 * 1024, "LDS budget");
};

// MODE 0: forward (3x3 taps); 1: stride-1 dgrad (mirrored taps, fused dgrad epilogue); 3: MODE 1
// whose fused BN-backward reduce also sums dz * xhat2 of a dual-BN block tail;
// 2: stride-2 dgrad as a 2x2 convolution over dY producing the four output parity classes as
// 4 x Cin channels (weights pre-arranged by hx_s2_weight_kernel, zero where a class does not meet
// a tap), written depth-to-space: class (ph, pw) of dY pixel (y, x) is dX pixel (2y+ph, 2x+pw).
// No zero-inserted MACs and no per-class launches (the generic parity-class kernel ran 1-4 taps
// per tile and was epilogue-bound: 205 us for ResNet-18's layer-2 downsample at bs1024).
template <int W, int IMGS, int WM, int WN, int MODE, bool STATS>
__global__ __launch_bounds__(WM * WN * 64)
void conv3x3_hx_kernel(const bf16* __restrict__ A, const bf16* __restrict__ Bw,
                       bf16* __restrict__ Y, float* __restrict__ stats,
                       const bf16* __restrict__ addend, const float* __restrict__ bias,
                       const HxGeom g) {
  constexpr bool DGRAD = MODE != 0;
  constexpr bool D2S = MODE == 2;
  constexpr bool DUAL = MODE == 3;
  constexpr int KS = D2S ? 2 : 3, TAPS = KS * KS;
  using SH = HxShape<W, IMGS, WM, WN, TAPS>;
  constexpr int NW = SH::NW, BM = SH::BM, BN = SH::BN, W2 = SH::W2;
  constexpr int HB = SH::HBYTES, BB = SH::BBYTES;
  __shared__ __attribute__((aligned(16))) char smem[SH::LDS];
  char* const Hs = smem;                       // [2][HBYTES] halo ring
  char* const Bs = smem + 2 * HB;              // [2][BBYTES] weight ring
  char* const dummy = smem + 2 * HB + 2 * BB;  // landing place of padding DMA slots
  // dgrad: BN mean | istd [| 2]; forward statistics: the shift K of the block's channels
  float* const auxs = reinterpret_cast<float*>(dummy + 1024);

  typedef __attribute__((address_space(3))) const char lds_char;
  typedef __attribute__((address_space(3))) const bf16x8 lds_bf16x8;
  lds_char* const lds_base = (lds_char*)smem;   // fragment reads through explicit LDS pointers

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int q = lane >> 4, kq = lane >> 4;
  const int nb0 = blockIdx.y * BN;             // first produced channel of this workgroup
  const int KA = TAPS * g.CA;                  // weight row length (elements)
  const __amdgpu_buffer_rsrc_t rsA = make_rsrc(A, g.a_bytes);
  const __amdgpu_buffer_rsrc_t rsB = make_rsrc(Bw, g.b_bytes);

  // ---- halo DMA slots: halo row hr = 8*i + (lane>>3) of piece i = wid + NW*k ----
  int s_px[SH::HS], s_ch[SH::HS];
#pragma unroll
  for (int k = 0; k < SH::HS; ++k) {
    const int i = wid + NW * k;
    const int hr = 8 * i + (lane >> 3);
    const int img = hr / SH::IMG_ROWS, rem = hr - img * SH::IMG_ROWS;
    const int jr = rem / W2, c = rem - jr * W2;
    // packed (img, ih + 1, iw + 1) of the source pixel, -1 for padding rows
    s_px[k] = (i < SH::HI && hr < SH::HROWS) ? ((img << 16) | (jr << 8) | c) : -1;
    s_ch[k] = ((lane & 7) ^ (hr & 7)) << 4;    // logical chunk fetched into physical (lane&7)
  }
  // halo piece k of chunk `ch` of tile `t` into ring slot `hb`
  auto halo_piece = [&](int t, int ch, int hb, int k) {
    const int i = wid + NW * k;
    const int sp = s_px[k];
    const int n = t * IMGS + (sp >> 16);
    const int ih = ((sp >> 8) & 0xff) - 1, iw = (sp & 0xff) - 1;
    const bool ok = (sp >= 0) & (n < g.N) & ((uint32_t)ih < (uint32_t)W) & ((uint32_t)iw < (uint32_t)W);
    const uint32_t off = ok ? (uint32_t)(((((n * W + ih) * W + iw) * g.CA) + ch * 64) * 2 + s_ch[k]) : kOOB;
    dma16(rsA, smem + (i < SH::HI ? hb * HB + i * 1024 : 2 * HB + 2 * BB), off);
  };
  // weight tile of (tap, chunk) into ring slot `bb`: LDS row r = 64-channel block r/64 of this
  // workgroup, channel hx_perm(r % 64) within it; 16-byte chunks XOR-swizzled by (r & 7)
  int b_row[SH::BS];
#pragma unroll
  for (int k = 0; k < SH::BS; ++k) {
    const int r = 8 * (wid + NW * k) + (lane >> 3);
    const int ch = nb0 + (r & ~63) + hx_perm(r & 63);
    b_row[k] = (ch * KA + (((lane & 7) ^ (r & 7)) << 3)) * 2;
  }
  auto b_tile = [&](int tap, int ch, int bb) {
    const int src_tap = (MODE == 1 || MODE == 3) ? 8 - tap : tap;
    const int delta = (src_tap * g.CA + ch * 64) * 2;
#pragma unroll
    for (int k = 0; k < SH::BS; ++k)
      dma16(rsB, Bs + bb * BB + (wid + NW * k) * 1024, (uint32_t)(b_row[k] + delta));
  };

  // ---- fragment addressing ----
  // A (pixels): tile pixel p = wm*64 + mi*16 + (lane&15) -> halo row of tap (0,0)
  int rb[4];
#pragma unroll
  for (int mi = 0; mi < 4; ++mi) {
    const int p = wm * 64 + mi * 16 + (lane & 15);
    const int img = p / (W * W), r = p - img * (W * W);
    rb[mi] = img * SH::IMG_ROWS + (r / W) * W2 + (r % W);
  }
  // B (weights): LDS row wn*64 + ni*16 + (lane&15)
  int boff[4];
#pragma unroll
  for (int ni = 0; ni < 4; ++ni) {
    const int nn = wn * 64 + ni * 16 + (lane & 15);
    boff[ni] = nn * 128 + ((kq ^ (nn & 7)) << 4);
  }

  // per-lane BatchNorm sums of channels nb0 + wn*64 + q*16 + e (forward stats / dgrad reduce)
  const bool bnf = DGRAD && g.bn_part != nullptr;
  // per-lane sums of its 16 channels, accumulated over every tile (forward statistics / dgrad
  // fused BN-backward reduce; MODE 3 a third one)
  float s1[16], s2[16], s3[DUAL ? 16 : 1];
#pragma unroll
  for (int e = 0; e < 16; ++e) s1[e] = s2[e] = 0.f;
#pragma unroll
  for (int e = 0; e < (DUAL ? 16 : 1); ++e) s3[e] = 0.f;
  const int ch_lane = nb0 + wn * 64 + q * 16;  // first of this lane's 16 produced channels
  if constexpr (STATS) {   // (in LDS, not 16 registers live across the MFMA loop: those spilled)
    for (int i = tid; i < BN; i += NW * 64) auxs[i] = g.kshift ? g.kshift[nb0 + i] : 0.f;
    __syncthreads();
  }
  // its output-tensor channel (depth-to-space: class ch / COUT, channel ch % COUT)
  const int co_lane = D2S ? ch_lane % g.COUT : ch_lane;
  const int cls_lane = D2S ? ch_lane / g.COUT : 0;
  // (a compact stride-2 addend belongs to parity class 0: the even-even output pixels)
  const bool add_on = addend != nullptr && (!D2S || !g.add_s2c || cls_lane == 0);
  if (bnf) {   // the block's BN mean / istd once into LDS (read per element in the epilogue)
    for (int i = tid; i < 2 * BN; i += NW * 64)
      auxs[i] = g.bn_aux[(i >= BN ? g.COUT : 0) + (nb0 + (i % BN)) % g.COUT];
    if constexpr (DUAL)
      for (int i = tid; i < 2 * BN; i += NW * 64)
        auxs[2 * BN + i] = g.bn_aux2[(i >= BN ? g.COUT : 0) + (nb0 + (i % BN)) % g.COUT];
    __syncthreads();
  }
  // output pixel of tile pixel p (the dY-resolution pixel for D2S, shifted to its class)
  auto out_pix = [&](int t, int p) -> size_t {
    if constexpr (!D2S) {
      return (size_t)t * BM + p;
    } else {
      const int img = t * IMGS + p / (W * W), r = p % (W * W);
      const int y = r / W, x = r % W;
      return ((size_t)img * (2 * W) + 2 * y + (cls_lane >> 1)) * (2 * W) + 2 * x + (cls_lane & 1);
    }
  };

  constexpr int STORES = 8;                    // global stores per lane per tile
  // prologue: first tile's chunk-0 halo and tap-0 weights
  if ((int)blockIdx.x < g.tiles) {
#pragma unroll
    for (int k = 0; k < SH::HS; ++k) halo_piece(blockIdx.x, 0, 0, k);
    b_tile(0, 0, 0);
  }
  wait_vmcnt<0>();

  int hc = 0;   // global chunk counter (halo ring slot = hc & 1)
  int bc = 0;   // global tap counter (weight ring slot = bc & 1)
  for (int t = blockIdx.x; t < g.tiles; t += gridDim.x) {
    const int tn = t + (int)gridDim.x;
    f32x4 acc[4][4];
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = f32x4{0.f, 0.f, 0.f, 0.f};
    uint4 pre_a[4][2], pre_y[4][2];
    uint32_t pre_m[4];

    for (int ch = 0; ch < g.KC; ++ch, ++hc) {
      const bool last_chunk = ch + 1 == g.KC;
      // what streams in during this chunk: the next chunk's halo (or the next tile's first)
      const int h_t = last_chunk ? tn : t, h_ch = last_chunk ? 0 : ch + 1;
      const int Soff = (hc & 1) * HB;          // this chunk's halo slot (byte offset in smem)
      // (a runtime tap loop: unrolled, the 9 taps' fragment offsets were hoisted as loop
      // invariants and pushed the 8-wave variants past 256 registers into spills)
#pragma unroll 1
      for (int tap = 0; tap < TAPS; ++tap, ++bc) {
        // weights of this tap were issued one tap ago; after them came at most one halo piece,
        // or, at a tile's first tap, the previous tile's epilogue stores (may stay in flight)
        if (tap == 0) {
          if (ch == 0) wait_vmcnt<STORES>();
          else wait_vmcnt<0>();
        } else {
          switch (SH::pieces_at(tap - 1)) {   // wave-uniform
            case 0: wait_vmcnt<0>(); break;
            case 1: wait_vmcnt<1>(); break;
            case 2: wait_vmcnt<2>(); break;
            default: wait_vmcnt<3>(); break;
          }
        }
        raw_barrier();
        // next tap's weights (past the last tile: harmless re-load of real rows), then this tap's
        // halo pieces of the next chunk (the vmcnt waits above count on that order)
        auto tap_dma = [&]() {
          if (tap < TAPS - 1) b_tile(tap + 1, ch, (bc + 1) & 1);
          else b_tile(0, last_chunk ? 0 : ch + 1, (bc + 1) & 1);
#pragma unroll
          for (int k = 0; k < SH::HS; ++k)
            if (k % (TAPS - 1) == tap) halo_piece(h_t, h_ch, (hc + 1) & 1, k);   // wave-uniform
        };
        constexpr bool dma_after = kHxDmaAfterRead && MODE == 0;
        if constexpr (!dma_after) tap_dma();
        if constexpr (DGRAD) {
          if (last_chunk && tap == TAPS - 1) {
            // epilogue operands (residual-gradient addend; BN input y + ReLU mask), read
            // behind this tap's MFMAs
#pragma unroll
            for (int mi = 0; mi < 4; ++mi) {
              const size_t o = out_pix(t, wm * 64 + mi * 16 + (lane & 15)) * g.COUT + co_lane;
              if (add_on) {
                const size_t oa = (D2S && g.add_s2c)
                                      ? ((size_t)t * BM + wm * 64 + mi * 16 + (lane & 15)) * g.COUT + co_lane
                                      : o;
                pre_a[mi][0] = *reinterpret_cast<const uint4*>(addend + oa);
                pre_a[mi][1] = *reinterpret_cast<const uint4*>(addend + oa + 8);
              }
              if (bnf) {
                if constexpr (kHxPrefetchY) {
                  pre_y[mi][0] = *reinterpret_cast<const uint4*>(g.bn_y + o);
                  pre_y[mi][1] = *reinterpret_cast<const uint4*>(g.bn_y + o + 8);
                }
                pre_m[mi] = *reinterpret_cast<const uint16_t*>(g.bn_mask + (o >> 3));
              }
            }
          }
        }
        const int Boff = 2 * HB + (bc & 1) * BB; // this tap's weight slot
        // tap (kh, kw) reads halo row offset kh*(W+2) + kw; the 2x2 stride-2 dgrad taps are the
        // dY pixels (y, x) .. (y+1, x+1): halo offsets 1..2
        const int toff = KS == 3 ? (tap / 3) * W2 + (tap % 3) : (1 + tap / 2) * W2 + 1 + (tap % 2);
        auto load_half = [&](int h, bf16x8* fa, bf16x8* fb) {
#pragma unroll
          for (int mi = 0; mi < 4; ++mi) {
            const int R = rb[mi] + toff;
            const int o = Soff + R * 128 + ((((h << 2) | kq) ^ (R & 7)) << 4);
            fa[mi] = *reinterpret_cast<const lds_bf16x8*>(lds_base + o);
          }
#pragma unroll
          for (int ni = 0; ni < 4; ++ni)
            fb[ni] = *reinterpret_cast<const lds_bf16x8*>(lds_base + Boff + (boff[ni] ^ (h << 6)));
        };
        auto mfma_half = [&](const bf16x8* fa, const bf16x8* fb) {
#pragma unroll
          for (int mi = 0; mi < 4; ++mi)
#pragma unroll
            for (int ni = 0; ni < 4; ++ni)
              acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[ni], fa[mi], acc[mi][ni], 0, 0, 0);
        };
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          bf16x8 fa[4], fb[4];
          load_half(h, fa, fb);
          if constexpr (dma_after) {
            // (build-time PCA_HX_DMA_AFTER_READ: the first half's fragment reads go out before the
            // tap's DMA pieces, whose issue cycles then cover the reads' LDS latency)
            if (h == 0) {
              __builtin_amdgcn_sched_barrier(0);
              tap_dma();
              __builtin_amdgcn_sched_barrier(0);
            }
          }
          mfma_half(fa, fb);
        }
      }
    }

    // ---- epilogue: lane holds channels ch_lane + [0,16) of tile pixel wm*64 + mi*16 + lane&15 ----
    if constexpr (DGRAD && !kHxPrefetchY) {
      // the BN input y of the fused reduce, loaded now for all four rows at once (prefetched
      // during the last tap it held 32 more registers across the MFMA loop: 256 + spills)
      if (bnf) {
#pragma unroll
        for (int mi = 0; mi < 4; ++mi) {
          const size_t o = out_pix(t, wm * 64 + mi * 16 + (lane & 15)) * g.COUT + co_lane;
          pre_y[mi][0] = *reinterpret_cast<const uint4*>(g.bn_y + o);
          pre_y[mi][1] = *reinterpret_cast<const uint4*>(g.bn_y + o + 8);
        }
      }
    }
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
      float v[16];
#pragma unroll
      for (int e = 0; e < 16; ++e) v[e] = acc[mi][e >> 2][e & 3];
      if (bias) {
#pragma unroll
        for (int e = 0; e < 16; ++e) v[e] += bias[ch_lane + e];
      }
      if constexpr (STATS) {
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const float d = v[e] - auxs[ch_lane - nb0 + e];   // shifted sums (K = 0 unshifted)
          s1[e] += d;
          s2[e] += d * d;
        }
      }
      if constexpr (DGRAD) {
        if (add_on) {   // dX = conv^T(dY) + addend in fp32, rounded to bf16 once
          float b2[16];
          unpack8(pre_a[mi][0], b2);
          unpack8(pre_a[mi][1], b2 + 8);
#pragma unroll
          for (int e = 0; e < 16; ++e) v[e] += b2[e];
        }
      }
      uint4 o0 = pack8(v), o1 = pack8(v + 8);
      if constexpr (DGRAD) {
        if (bnf) {
          float f[16], yy[16];
          unpack8(o0, f);
          unpack8(o1, f + 8);
          unpack8(pre_y[mi][0], yy);
          unpack8(pre_y[mi][1], yy + 8);
          const uint32_t m = pre_m[mi];
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const float dz = relu_bit(f[e], m, e);
            s1[e] += dz;
            const int c = ch_lane - nb0 + e;
            s2[e] = fmaf(dz, yy[e] - auxs[c], s2[e]);   // (x istd at the flush; aux of c % COUT)
          }
          if constexpr (DUAL) {   // (y2 read here: no prefetch registers for it)
            const size_t o = out_pix(t, wm * 64 + mi * 16 + (lane & 15)) * g.COUT + co_lane;
            unpack8(*reinterpret_cast<const uint4*>(g.bn_y2 + o), yy);
            unpack8(*reinterpret_cast<const uint4*>(g.bn_y2 + o + 8), yy + 8);
#pragma unroll
            for (int e = 0; e < 16; ++e) {
              const float dz = relu_bit(f[e], m, e);
              const int c = ch_lane - nb0 + e;
              s3[e] = fmaf(dz, yy[e] - auxs[2 * BN + c], s3[e]);   // (x istd2 at the flush)
            }
          }
        }
      }
      bf16* dst = Y + out_pix(t, wm * 64 + mi * 16 + (lane & 15)) * g.COUT + co_lane;
      *reinterpret_cast<uint4*>(dst) = o0;
      *reinterpret_cast<uint4*>(dst + 8) = o1;
    }
  }

  // ---- per-block channel sums: the 16 lanes of a group share channels; WM waves per column ----
  if constexpr (DGRAD) {
    if (bnf) {   // sums of dz * (y - mean) -> dz * xhat (istd of channel c, istd2 for the dual)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int c = ch_lane - nb0 + e;
        s2[e] *= auxs[BN + c];
        if constexpr (DUAL) s3[e] *= auxs[3 * BN + c];
      }
    }
  }
  if (STATS || bnf) {
    constexpr int NSR = DUAL ? 3 : 2;             // sums per channel
#pragma unroll
    for (int e = 0; e < 16; ++e) {
#pragma unroll
      for (int x = 1; x < 16; x <<= 1) {
        s1[e] += __shfl_xor(s1[e], x, 64);
        s2[e] += __shfl_xor(s2[e], x, 64);
        if constexpr (DUAL) s3[e] += __shfl_xor(s3[e], x, 64);
      }
    }
    wait_vmcnt<0>();
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem);  // [WM][BN][NSR]
    if ((lane & 15) == 0) {
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        red[(wm * BN + wn * 64 + q * 16 + e) * NSR + 0] = s1[e];
        red[(wm * BN + wn * 64 + q * 16 + e) * NSR + 1] = s2[e];
        if constexpr (DUAL) red[(wm * BN + wn * 64 + q * 16 + e) * NSR + 2] = s3[e];
      }
    }
    __syncthreads();
    // output channel c of this block gathers its produced channels c, c + COUT, ... (the
    // parity classes of the stride-2 dgrad); slab row per (M walker, N block) for D2S
    const int nco = D2S ? (BN < g.COUT ? BN : g.COUT) : BN;
    if (tid < nco) {
      float a = 0.f, b = 0.f, d3 = 0.f;
      for (int j = tid; j < BN; j += (D2S ? g.COUT : BN)) {
#pragma unroll
        for (int w = 0; w < WM; ++w) {   // fixed order: deterministic per block
          a += red[(w * BN + j) * NSR + 0];
          b += red[(w * BN + j) * NSR + 1];
          if constexpr (DUAL) d3 += red[(w * BN + j) * NSR + 2];
        }
      }
      float* dst = STATS ? stats : g.bn_part;
      // (D2S: the N blocks that share columns — one per class when COUT >= BN — get rows of
      // their own; together the rows of one M walker cover every column)
      const int cb = D2S && g.COUT > BN ? g.COUT / BN : 1;
      const int row = D2S ? (int)(blockIdx.x * (gridDim.y / cb) + blockIdx.y / cb) : (int)blockIdx.x;
      const int col = (nb0 + tid) % g.COUT;
      stat_out(dst, row, g.shards, NSR * g.COUT, col, a);
      stat_out(dst, row, g.shards, NSR * g.COUT, g.COUT + col, b);
      if constexpr (DUAL) stat_out(dst, row, g.shards, NSR * g.COUT, 2 * g.COUT + col, d3);
    }
    if constexpr (STATS) stat_krow(stats, g.shards, 2 * g.COUT, g.kshift, g.COUT);
  }
}

// ---------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------
int stat_shards();
const float* stat_shift();

static int hx_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    if (n <= 0) n = 256;
  }
  return n;
}

// shape gate: 3x3 s1 p1, square 16 / 8 / 4 maps, channel counts multiples of 128
bool conv_hx_applicable(int N, int H, int W, int CA, int CO, int KH, int KW, int stride, int pad,
                        int groups) {
  static const bool off = [] {
    const char* e = getenv("PCA_CONV_HX");
    return e && e[0] == '0';
  }();
  if (off || KH != 3 || KW != 3 || stride != 1 || pad != 1 || groups != 1 || H != W) return false;
  if (CA % 64 || CO % 128) return false;
  const int bm = W == 4 ? 128 : 256;
  return (W == 16 || W == 8 || W == 4) && (N * H * W) % bm == 0;
}

template <int W, int IMGS, int WM, int WN, int MODE, bool STATS>
static int hx_occ() {
  static int occ = 0;
  if (occ == 0)
    occ = blocks_per_cu((const void*)conv3x3_hx_kernel<W, IMGS, WM, WN, MODE, STATS>, WM * WN * 64,
                        "conv3x3_hx");
  return occ;
}

template <int W, int IMGS, int WM, int WN, int MODE>
static int hx_grid_x(const HxGeom& g, int nblocks) {
  const int slots = hx_occ<W, IMGS, WM, WN, MODE, MODE == 0>() * hx_cus();
  int gx = std::max(1, slots / std::max(1, nblocks));
  gx = std::min(gx, g.tiles);
  const int per = cdiv(g.tiles, gx);
  return cdiv(g.tiles, per);
}

// returns the BN-sum slab rows the launch writes (grid.x; MODE 2: grid.x x the N blocks per column)
template <int W, int IMGS, int WM, int WN, int MODE>
static int hx_run(const bf16* a, const bf16* b, bf16* y, float* stats, const bf16* addend,
                  const float* bias, const HxGeom& g, hipStream_t st, bool launch) {
  constexpr int BN = WN * 64;
  const int nblocks = g.CO / BN;
  const int gx = hx_grid_x<W, IMGS, WM, WN, MODE>(g, nblocks);
  if (launch) {
    const dim3 grid(gx, nblocks), block(WM * WN * 64);
    if (kHxDual && MODE == 1 && g.bn_part && g.bn_y2)
      hipLaunchKernelGGL((conv3x3_hx_kernel<W, IMGS, WM, WN, kHxDual ? 3 : 1, false>), grid, block,
                         0, st, a, b, y, nullptr, addend, nullptr, g);
    else if (MODE != 0)
      hipLaunchKernelGGL((conv3x3_hx_kernel<W, IMGS, WM, WN, MODE, false>), grid, block, 0, st, a, b,
                         y, nullptr, addend, nullptr, g);
    else if (stats)
      hipLaunchKernelGGL((conv3x3_hx_kernel<W, IMGS, WM, WN, 0, true>), grid, block, 0, st, a, b, y,
                         stats, nullptr, bias, g);
    else
      hipLaunchKernelGGL((conv3x3_hx_kernel<W, IMGS, WM, WN, 0, false>), grid, block, 0, st, a, b, y,
                         nullptr, nullptr, bias, g);
  }
  return MODE == 2 ? gx * nblocks / (g.COUT > BN ? g.COUT / BN : 1) : gx;
}

template <int MODE>
static int hx_dispatch(const bf16* a, const bf16* b, bf16* y, float* stats, const bf16* addend,
                       const float* bias, HxGeom& g, int H, hipStream_t st, bool launch) {
  switch (H) {
    case 16: g.tiles = g.N; return hx_run<16, 1, 4, 2, MODE>(a, b, y, stats, addend, bias, g, st, launch);
    case 8: g.tiles = g.N / 4; return hx_run<8, 4, 4, 2, MODE>(a, b, y, stats, addend, bias, g, st, launch);
    default: g.tiles = g.N / 8; return hx_run<4, 8, 2, 2, MODE>(a, b, y, stats, addend, bias, g, st, launch);
  }
}

// launch (or, with launch = false, only size: returns the BN-statistics slab rows).
// dgrad: H is the produced (= dY) map size; mode 2 (stride-2 dgrad) takes H = the dY map size and
// b = the 2x2 class weights from conv_hx_s2_weights (CO = 4 x Cin).
static int g_hx_add_s2c = 0;
void conv_hx_set_addend_s2c(int on) { g_hx_add_s2c = on; }

int conv_hx_launch(const bf16* a, const bf16* b, bf16* y, float* stats, const bf16* addend,
                   const float* bias, int N, int H, int CA, int CO, int mode, hipStream_t st,
                   const bf16* bn_y, const uint8_t* bn_mask, const float* bn_aux, float* bn_part,
                   bool launch, const bf16* bn_y2, const float* bn_aux2) {
  HxGeom g;
  g.N = N;
  g.CA = CA;
  g.CO = CO;
  g.COUT = mode == 2 ? CO / 4 : CO;
  g.KC = CA / 64;
  g.a_bytes = (uint32_t)((size_t)N * H * H * CA * 2);
  g.b_bytes = (uint32_t)((size_t)CO * (mode == 2 ? 4 : 9) * CA * 2);
  g.shards = stat_shards();
  g.bn_y = bn_y;
  g.bn_mask = bn_mask;
  g.bn_aux = bn_aux;
  g.bn_part = mode != 0 ? bn_part : nullptr;
  g.bn_y2 = mode == 1 && bn_part ? bn_y2 : nullptr;   // (accumulator mode: rows of 3 sums)
  g.bn_aux2 = g.bn_y2 ? bn_aux2 : nullptr;
  g.kshift = mode == 0 && stats ? stat_shift() : nullptr;
  g.add_s2c = mode == 2 ? g_hx_add_s2c : 0;
  if (mode == 0) return hx_dispatch<0>(a, b, y, stats, addend, bias, g, H, st, launch);
  if (mode == 1) return hx_dispatch<1>(a, b, y, stats, addend, bias, g, H, st, launch);
  return hx_dispatch<2>(a, b, y, stats, addend, bias, g, H, st, launch);
}

// stride-2 dgrad applicability: 3x3 / stride 2 / pad 1 forward conv with H = 2 * Ho, dY maps of
// 16 / 8 / 4, Cout % 64 (the gathered dY chunks), 4 * Cin % 128 (the produced class channels),
// Cin % 128 past 128 (a 128-channel N block then stays inside one class)
bool conv_hx_s2_applicable(int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride,
                           int pad, int groups, int Ho, int Wo) {
  static const bool off = [] {
    const char* e = getenv("PCA_CONV_HX");
    return e && e[0] == '0';
  }();
  if (off || KH != 3 || KW != 3 || stride != 2 || pad != 1 || groups != 1 || H != W) return false;
  if (Ho != Wo || H != 2 * Ho || (Ho != 16 && Ho != 8 && Ho != 4)) return false;
  if (Cout % 64 || (4 * Cin) % 128 || (Cin > 128 && Cin % 128)) return false;
  const int bm = Ho == 4 ? 128 : 256;
  return (N * Ho * Ho) % bm == 0;
}

// 2x2 class weights of the stride-2 dgrad from the transposed 3x3 weights wt[Cin][3][3][Cout]:
//   w2[(ph*2 + pw)*Cin + ci][a*2 + b][co] = wt[ci][ph + 1 - 2a][pw + 1 - 2b][co]  (0 if out of range)
// (dX pixel (2y+ph, 2x+pw) meets dY pixel (y+a, x+b) through tap (ph+1-2a, pw+1-2b))
__global__ __launch_bounds__(256) void hx_s2_weight_kernel(const bf16* __restrict__ wt, int Cin,
                                                           int Cout, bf16* __restrict__ w2) {
  const int c8 = Cout / 8;
  const int total = 4 * Cin * 4 * c8;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int cc = i % c8, t = (i / c8) % 4, z = i / (c8 * 4);
    const int cls = z / Cin, ci = z % Cin;
    const int kh = (cls >> 1) + 1 - 2 * (t >> 1), kw = (cls & 1) + 1 - 2 * (t & 1);
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (kh >= 0 && kh < 3 && kw >= 0 && kw < 3)
      v = *reinterpret_cast<const uint4*>(wt + (((size_t)ci * 3 + kh) * 3 + kw) * Cout + cc * 8);
    *reinterpret_cast<uint4*>(w2 + ((size_t)z * 4 + t) * Cout + cc * 8) = v;
  }
}

void conv_hx_s2_weights(const bf16* wt, int Cin, int Cout, bf16* w2, hipStream_t st) {
  const int total = 4 * Cin * 4 * (Cout / 8);
  hipLaunchKernelGGL(hx_s2_weight_kernel, dim3(std::min(cdiv(total, 256), 1024)), dim3(256), 0, st, wt,
                     Cin, Cout, w2);
}

}  // namespace pca
