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

#include <cstdlib>

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
  int64_t* prof;    // diagnostics: per-wave shader-clock stamps (c64_set_prof), else nullptr
  const float* kshift;   // forward stats: per-channel shift K (common.h stat_shift), or nullptr
  // forward input transform (the BatchNorm+ReLU that produced the input, applied on the halo
  // instead of by its own pass): x = relu(a * xf[c] + xf[64 + c]) (BN scale | shift = aux rows
  // 2-3) and its 1-bit ReLU mask of every tile interior into xf_mask (conv3x3_c64_kernel<.., XF>)
  const float* xf;
  uint8_t* xf_mask;
};

namespace c64 {
constexpr int W = 32, W2 = 34, ROWS = 8;
constexpr int TILE = ROWS * W;                  // 256 output pixels
constexpr int HROWS = (ROWS + 2) * W2;          // 340 halo pixels
constexpr int HI = (HROWS + 7) / 8;             // 43 LDS-DMA instructions (1 KiB each)
constexpr int HBYTES = HI * 1024;
constexpr int NW = 4;                           // waves: 4 x (64 pixels, 64 channels)
constexpr int SLOTS = (HI + NW - 1) / NW;       // DMA instructions per wave per tile
constexpr int BBYTES = 64 * 576 * 2;           // resident weights
constexpr int BI = BBYTES / 1024;               // 72 DMA instructions
static_assert(BBYTES + 2 * HBYTES <= 160 * 1024, "LDS budget");
}  // namespace c64

// Output layout trick (no LDS round trip in the epilogue): the MFMA is issued as
// D = W x X^T, so a lane's accumulators hold CHANNELS of one pixel instead of pixels of one
// channel. The weight rows are staged in LDS in a permuted channel order, perm(n) =
// ((n >> 2) & 3) * 16 + (n >> 4) * 4 + (n & 3), which makes lane l (q = l >> 4) of every 16x16
// tile ni hold output channels q*16 + ni*4 + [0, 4): over the 4 tiles, 16 consecutive channels of
// pixel (l & 15) — two 16-byte global stores straight from the accumulators. (The previous
// epilogue staged the bf16 tile through LDS with 64 two-byte writes per lane and two barriers.)
// The next tile's halo DMA is issued one 1 KiB piece per K-step inside the MFMA loop (an LDS-DMA
// piece costs ~60-185 issue cycles; issued back-to-back at tile start with one wave per SIMD
// they idled the matrix core).
__device__ __forceinline__ int c64_perm(int n) { return ((n >> 2) & 3) * 16 + (n >> 4) * 4 + (n & 3); }

// XF (forward only): the input is the PRE-BatchNorm y of the previous conv; every halo piece is
// transformed in LDS right after it lands (x = relu(y * scale + shift) with the BN apply pass's
// exact arithmetic; the zero padding stays zero) and the tile interior's ReLU mask is written for
// the BN backward — the BN's own apply pass (read y, write x + mask) disappears.
template <bool DGRAD, bool STATS, bool PROF = false, bool XF = false>
__global__ __launch_bounds__(256)
void conv3x3_c64_kernel(const bf16* __restrict__ A, const bf16* __restrict__ Wm,
                        bf16* __restrict__ Y, float* __restrict__ stats,
                        const bf16* __restrict__ addend, const C64Geom g) {
  using namespace c64;
  static_assert(!(XF && DGRAD), "input transform: forward only");
  // (XF: + the transform's scale | shift and the statistics shift K, LDS-resident: the kernel runs
  // at the 512-register limit)
  __shared__ __attribute__((aligned(16))) char smem[BBYTES + 2 * HBYTES + 1024 + (XF ? 768 : 0)];
  char* const Bs = smem + 2 * HBYTES;
  float* const xfs = reinterpret_cast<float*>(smem + BBYTES + 2 * HBYTES + 1024);   // [sc|sh][64]

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid;                            // 64 pixels (2 image rows) x 64 channels
  const int q = lane >> 4;                       // this lane's 16-channel group
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
  // branch-free (selects only, so it does not split the K-step's scheduling region): slots past
  // the halo (i >= HI) write their zeros into a 1 KiB dummy area behind the weights
  auto issue_piece = [&](int n, int h0, int buf, int k) {
    const int i = wid + NW * k;
    const int ih = h0 + (s_jc[k] >> 8) - 1, iw = (s_jc[k] & 0xff) - 1;
    const bool ok = (s_jc[k] >= 0) & ((uint32_t)ih < (uint32_t)g.H) & ((uint32_t)iw < (uint32_t)W);
    const uint32_t off = ok ? (uint32_t)((((n * g.H + ih) * W + iw) * 64) * 2 + s_ch[k]) : kOOB;
    dma16(rsA, i < HI ? smem + buf * HBYTES + i * 1024 : smem + 2 * HBYTES + BBYTES, off);
  };

  if (blockIdx.x < g.tiles) {
    const int n0 = blockIdx.x / tiles_per_img;
#pragma unroll
    for (int k = 0; k < SLOTS; ++k) issue_piece(n0, (blockIdx.x - n0 * tiles_per_img) * ROWS, 0, k);
  }

  // ---- weights -> LDS once: LDS row n holds output channel perm(n); 72 chunks of 8 K-values;
  // physical chunk pc holds logical chunk (pc & ~7) | ((pc ^ n) & 7). K order = (tap, input
  // channel). ----
  {
    const __amdgpu_buffer_rsrc_t rsW = make_rsrc(Wm, BBYTES);
    for (int i = wid; i < BI; i += NW) {
      const int qq = i * 64 + lane;
      const int n = qq / 72, pc = qq - n * 72;
      const int lc = (pc & ~7) | ((pc ^ n) & 7);
      const int tap = lc >> 3, c8 = lc & 7;
      const int src_tap = DGRAD ? 8 - tap : tap;
      dma16(rsW, Bs + i * 1024, (uint32_t)((c64_perm(n) * 576 + src_tap * 64 + c8 * 8) * 2));
    }
  }

  // per-lane fragment byte offsets (even 32-channel half): halo row R of tap (kh, kw) for pixel
  // (2*wm + (mi>>1), (mi&1)*16 + l&15) with its XOR-swizzled 16-byte chunk; weight row nn
  const int kq = lane >> 4;                      // 8-channel chunk within a 32-channel half
  // (fragment mi | 1 is 16 halo rows after mi & ~1: same swizzle key, +2048 bytes)
  int aoff[9][2], boff[4];
#pragma unroll
  for (int tap = 0; tap < 9; ++tap)
#pragma unroll
    for (int mh = 0; mh < 2; ++mh) {
      const int R = (2 * wm + mh + tap / 3) * W2 + (lane & 15) + tap % 3;
      aoff[tap][mh] = R * 128 + ((kq ^ (R & 7)) << 4);
    }
#pragma unroll
  for (int ni = 0; ni < 4; ++ni) {
    const int nn = ni * 16 + (lane & 15);
    boff[ni] = nn * 1152 + ((kq ^ (nn & 7)) << 4);
  }

  // per-lane BatchNorm sums of channels q*16 + e, accumulated over every tile (forward; shifted
  // by kk = the consumer BN's pilot mean when given)
  float st_s[16], st_q[16], kk[XF ? 1 : 16];
  float* const kks = xfs + 128;                   // XF: K in LDS [64]
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    st_s[e] = st_q[e] = 0.f;
    if constexpr (!XF) kk[e] = (STATS && g.kshift) ? g.kshift[q * 16 + e] : 0.f;
  }
  // fused BN-backward reduce (dgrad): sums of dz and dz * xhat of channels q*16 + e
  const bool bnf = DGRAD && g.bn_part != nullptr;
  float bs1[16], bs2[16], bmean[16], bistd[16];
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    bs1[e] = bs2[e] = 0.f;
    bmean[e] = bnf ? g.bn_aux[q * 16 + e] : 0.f;
    bistd[e] = bnf ? g.bn_aux[64 + q * 16 + e] : 0.f;
  }

  // Deferred epilogue: tile t's accumulators are stored (and reduced into the BN sums) during
  // K-steps 11, 13, 15, 17 of tile t+1, one 16-pixel fragment row per step, in the MFMA
  // shadow (one wave per SIMD: run after the K loop it idled the matrix core for ~1.8k cycles
  // per tile). Two accumulator sets alternate between tiles (the tile loop is unrolled by two).
  // Its dgrad operands (residual addend, BN input y, ReLU mask) are loaded at step 0.
  constexpr int STORES = 8;                      // global stores per lane per tile (4 px x 2)
  uint4 pre_a[4][2], pre_y[4][2];
  uint32_t pre_m[4];
  auto pre_load = [&](size_t pix0p) {
    if constexpr (DGRAD) {
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) {
        const size_t o = (pix0p + wm * 64 + mi * 16 + (lane & 15)) * 64 + q * 16;
        if (addend) {
          pre_a[mi][0] = *reinterpret_cast<const uint4*>(addend + o);
          pre_a[mi][1] = *reinterpret_cast<const uint4*>(addend + o + 8);
        }
        if (bnf) {
          pre_y[mi][0] = *reinterpret_cast<const uint4*>(g.bn_y + o);
          pre_y[mi][1] = *reinterpret_cast<const uint4*>(g.bn_y + o + 8);
          pre_m[mi] = *reinterpret_cast<const uint16_t*>(g.bn_mask + (o >> 3));
        }
      }
    }
  };
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  auto epi_part = [&](f32x4 (&A)[4][4], int mi, size_t pix0p) {
    // lane holds channels q*16 + [0,16) of pixel wm*64 + mi*16 + (lane&15)
    float v[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) v[e] = A[mi][e >> 2][e & 3];
    if constexpr (STATS) {
      // scalar: these run beside the next tile's MFMAs, where packed f32 ops cost more issue
      // than two scalar ones (MI355X_MICROARCH.md cycle constants), and the vectorized form
      // needed register-pair moves; the empty asm keeps the SLP vectorizer from re-pairing them
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        float d = v[e] - (XF ? kks[q * 16 + e] : kk[e]);
        asm volatile("" : "+v"(d));
        st_s[e] += d;
        st_q[e] = fmaf(d, d, st_q[e]);
      }
    }
    if constexpr (DGRAD) {
      if (addend) {   // dX = conv^T(dY) + addend in fp32, rounded to bf16 once
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
          bs1[e] += dz;
          bs2[e] = fmaf(dz, yy[e] - bmean[e], bs2[e]);   // (x istd at the flush)
        }
      }
    }
    bf16* dst = Y + (pix0p + wm * 64 + mi * 16 + (lane & 15)) * 64 + q * 16;
    *reinterpret_cast<uint4*>(dst) = o0;
    *reinterpret_cast<uint4*>(dst + 8) = o1;
  };

  // XF: this wave's own halo pieces of tile t (they landed: counted wait above) are transformed
  // in place before the tile barrier publishes them, relu(y * scale + shift) with the BN apply
  // pass's arithmetic. A lane's 16-byte pieces all hold the same logical 8-channel chunk
  // ((lane & 7) ^ (hr & 7) with hr & 7 == lane >> 3). Pieces of padding pixels (DMA'd as zeros)
  // stay zero; interior pixels also get their mask byte (bit v = channel c8*8 + v > 0), exactly
  // as the BN apply pass writes it. One piece at a time with its scale / shift re-read from LDS:
  // the kernel runs at the 512-register limit (every variant that kept more live — the pieces
  // of a group, the coefficients across pieces, the transform inside the K loop — spilled and
  // ran 1.5-3.5x slower than this one).
  auto xform_tile = [&](int t, int buf) {
    const int c8 = (lane & 7) ^ (lane >> 3);
    const int n = t / tiles_per_img, h0 = (t - n * tiles_per_img) * ROWS;
#pragma unroll
    for (int k = 0; k < SLOTS; ++k) {
      __builtin_amdgcn_sched_barrier(0);
      const int i = wid + NW * k;
      if (i >= HI) continue;                      // (wave-uniform)
      const int jr = s_jc[k] >> 8, c = s_jc[k] & 0xff;
      const int ih = h0 + jr - 1, iw = c - 1;
      if (s_jc[k] < 0 || (uint32_t)ih >= (uint32_t)g.H || (uint32_t)iw >= (uint32_t)W) continue;
      uint4* p = reinterpret_cast<uint4*>(smem + buf * HBYTES + i * 1024 + lane * 16);
      float f[8], sc[8], sh[8];
      unpack8(*p, f);
#pragma unroll
      for (int v = 0; v < 8; ++v) {
        sc[v] = xfs[c8 * 8 + v];
        sh[v] = xfs[64 + c8 * 8 + v];
      }
      uint32_t b = 0;
#pragma unroll
      for (int v = 0; v < 8; ++v) {
        float a = f[v] * sc[v] + sh[v];
        a = apply_act(a, ACT_RELU);
        b |= (a > 0.f ? 1u : 0u) << v;
        f[v] = a;
      }
      *p = pack8(f);
      if (jr >= 1 && jr <= ROWS)
        g.xf_mask[((size_t)(n * g.H + ih) * W + iw) * 8 + c8] = (uint8_t)b;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  };

  // (dgrad keeps the epilogue after its K loop: its fused addend / BN-reduce operands and sums
  // with a second accumulator set exceed the 512 registers)
  constexpr bool DEFER = !DGRAD;
  auto pix0_of = [&](int t) {
    const int n = t / tiles_per_img, h0 = (t - n * tiles_per_img) * ROWS;
    return ((size_t)n * g.H + h0) * W;
  };
  auto tile_body = [&](int t, int it, f32x4 (&Acc)[4][4], f32x4 (&Prev)[4][4], bool have_prev,
                       size_t pix0p) {
    const int buf = it & 1;
    // this tile's halo landed (every piece was issued before the previous tile's 8 deferred
    // stores, which may stay in flight)
    wait_vmcnt<STORES>();
    if constexpr (XF) xform_tile(t, buf);
    raw_barrier();
    int64_t* pst = nullptr;
    if constexpr (PROF) {
      pst = g.prof + ((size_t)(blockIdx.x * 4 + wid) * 16 + (it & 15)) * 4;
      const int64_t t0 = (int64_t)__builtin_amdgcn_s_memtime();
      if (lane == 0) pst[0] = t0;
    }
    const char* S = smem + buf * HBYTES;
    const int tn = t + (int)gridDim.x;
    const int nn_img = tn / tiles_per_img, nn_h0 = (tn - nn_img * tiles_per_img) * ROWS;
    if (DEFER && have_prev) pre_load(pix0p);
    if (!DEFER) pre_load(pix0_of(t));

#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) Acc[mi][ni] = f32x4{0.f, 0.f, 0.f, 0.f};

    // K loop: step s = (tap s>>1, 32-channel half s&1). The fragments of step s+1 (separate
    // registers) are read while step s's 16 MFMAs run, interleaved one ds_read per MFMA
    // (sched_group_barrier): with one wave per SIMD, reads issued as a block after the MFMAs
    // cost their full issue time every step. Addresses are precomputed per (tap, fragment); the
    // odd half flips bit 6 (chunk ^ 4) and the tap adds 128 B to the weight row offset.
    auto load_step = [&](int st, bf16x8* af, bf16x8* bv) {
      const int tap = st >> 1, hx = (st & 1) << 6;
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
        af[mi] = *reinterpret_cast<const bf16x8*>(S + (aoff[tap][mi >> 1] ^ hx) + (mi & 1) * 2048);
#pragma unroll
      for (int ni = 0; ni < 4; ++ni)
        bv[ni] = *reinterpret_cast<const bf16x8*>(Bs + (boff[ni] ^ hx) + tap * 128);
    };
    bf16x8 fa[2][4], fb[2][4];
    load_step(0, fa[0], fb[0]);
#pragma unroll
    for (int st = 0; st < 18; ++st) {
      const int cur = st & 1;
      // one scheduling region per step: {DMA piece, reads of step st+1, MFMAs of step st}
      __builtin_amdgcn_sched_barrier(0);
      // (past the last tile the offsets fall outside the input: the pieces land zeros)
      if (st < SLOTS) issue_piece(nn_img, nn_h0, buf ^ 1, st);
      if (st + 1 < 18) load_step(st + 1, fa[cur ^ 1], fb[cur ^ 1]);
      // (no s_setprio here: it is a scheduling boundary and would keep the reads out of the
      // MFMA region; with one wave per SIMD priority has nothing to arbitrate)
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni)
          Acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[cur][ni], fa[cur][mi], Acc[mi][ni], 0, 0, 0);
      if (st + 1 < 18) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // one MFMA
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // one ds_read
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
      if (DEFER && st >= 11 && (st & 1) && have_prev) epi_part(Prev, (st - 11) >> 1, pix0p);
    }
    if constexpr (!DEFER) {
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) epi_part(Acc, mi, pix0_of(t));
    }
    if constexpr (PROF) {
      const int64_t t1 = (int64_t)__builtin_amdgcn_s_memtime();
      if (lane == 0) pst[1] = t1;
      if (lane == 0) pst[2] = t1;
    }
  };
  f32x4 accA[4][4], accB[4][4];
  if constexpr (XF) {
    if (tid < 128) xfs[tid] = g.xf[tid];
    else if (tid < 192) kks[tid - 128] = g.kshift ? g.kshift[tid - 128] : 0.f;
    __syncthreads();
  }
  wait_vmcnt<0>();                                // weights + first halo
  {
    int t = blockIdx.x, it = 0;
    bool have_prev = false;
    size_t pix0p = 0;
    while (t < g.tiles) {
      tile_body(t, it, accA, accB, have_prev, pix0p);
      have_prev = true;
      pix0p = pix0_of(t);
      t += gridDim.x;
      ++it;
      if (t >= g.tiles) {                         // last tile: its epilogue now
        if constexpr (DEFER) {
          pre_load(pix0p);
#pragma unroll
          for (int mi = 0; mi < 4; ++mi) epi_part(accA, mi, pix0p);
        }
        break;
      }
      if constexpr (DEFER) {
        tile_body(t, it, accB, accA, have_prev, pix0p);
      } else {
        tile_body(t, it, accA, accB, have_prev, pix0p);
      }
      pix0p = pix0_of(t);
      t += gridDim.x;
      ++it;
      if (t >= g.tiles) {
        if constexpr (DEFER) {
          pre_load(pix0p);
#pragma unroll
          for (int mi = 0; mi < 4; ++mi) epi_part(accB, mi, pix0p);
        }
        break;
      }
    }
  }

  // ---- per-block channel sums: lanes of one 16-lane group share channels q*16 + e ----
  if constexpr (DGRAD) {
#pragma unroll
    for (int e = 0; e < 16; ++e) bs2[e] *= bistd[e];   // sum dz*(y - mean) -> sum dz*xhat
  }
  if (STATS || bnf) {
    float* s1 = STATS ? st_s : bs1;
    float* s2 = STATS ? st_q : bs2;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
#pragma unroll
      for (int x = 1; x < 16; x <<= 1) {
        s1[e] += __shfl_xor(s1[e], x, 64);
        s2[e] += __shfl_xor(s2[e], x, 64);
      }
    }
    wait_vmcnt<0>();
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem);  // [4 waves][64 ch][2]
    if ((lane & 15) == 0) {
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        red[(wm * 64 + q * 16 + e) * 2 + 0] = s1[e];
        red[(wm * 64 + q * 16 + e) * 2 + 1] = s2[e];
      }
    }
    __syncthreads();
    if (tid < 64) {
      float a = 0.f, b = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) {   // fixed order: deterministic per block
        a += red[(w * 64 + tid) * 2 + 0];
        b += red[(w * 64 + tid) * 2 + 1];
      }
      float* dst = STATS ? stats : g.bn_part;
      stat_out(dst, blockIdx.x, g.shards, 128, tid, a);
      stat_out(dst, blockIdx.x, g.shards, 128, 64 + tid, b);
    }
    if constexpr (STATS) stat_krow(stats, g.shards, 128, g.kshift, 64);
  }
}

// round-2 version (LDS-staged epilogue, halo DMA issued at tile start): PCA_C64_V=1 (A/B)
template <bool DGRAD, bool STATS>
__global__ __launch_bounds__(256)
void conv3x3_c64_v1_kernel(const bf16* __restrict__ A, const bf16* __restrict__ Wm,
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

  constexpr int STORES = (TILE * 8) / 256;
  constexpr int CST = 64 + 8;      // global stores per thread per tile
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
      for (int ni = 0; ni < 4; ++ni) {
        const float kc = g.kshift ? g.kshift[ni * 16 + (lane & 15)] : 0.f;
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float v = acc[mi][ni][j] - kc;
            st_s[ni] += v;
            st_q[ni] += v * v;
          }
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
    stat_krow(stats, g.shards, 128, g.kshift, 64);
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
// Versions 3 / 4 (opt-in, PCA_C64_V): the same tile plan on v_mfma_f32_32x32x16_bf16.
//
// Why: with one wave per SIMD every non-MFMA instruction of the wave (fragment reads, halo DMA
// pieces, the deferred epilogue's BN sums / packs / stores) has to issue in the MFMA shadow. A
// 16x16x32 MFMA runs 16 cycles and blocks vector issue for 8 of them (8 free cycles per MFMA);
// a 32x32x16 runs 32 and blocks 8 (24 free) at the same MACs per cycle
// (MI355X_MICROARCH.md, vector-instruction issue cost row). The fragment bytes per MAC are the
// same (a 64x64 wave tile reads 2 A + 2 B fragments per 16-deep K step for 4 MFMAs).
//   * D[channel][pixel] = W x X^T per 32x32 tile: lane l holds pixel (l & 31) of its tile and,
//     with the weight rows staged in the permuted order perm32, output channels
//     32*ct + 16*(l >> 5) + [0, 16) — two 16-byte stores per (pixel tile, channel tile);
//   * a wave owns two output rows (pixel tiles pt = one 32-wide image row each) x 64 channels;
//   * LDS "planes": the halo and the weights are stored as 16-channel (32-byte) planes, one per
//     16-deep K step, so a K step moves a fragment read by an immediate offset (an XOR-swizzled
//     128-byte row layout needs a separate address register per K step: the compiler hoisted
//     144 of them and the forward spilled). A 32x32x16 operand read touches 16 consecutive rows per
//     ds_read_b128 lane group; with 32-byte rows and the two 16-byte halves swapped on rows with
//     bit 3 set, those 16 rows cover all 64 banks once.
namespace c64w {
constexpr int HP = 11;                           // 1 KiB DMA pieces per halo plane (340 rows x 32 B)
constexpr int HPB = HP * 1024;                   // bytes per halo plane
constexpr int HB = 4 * HPB;                      // one halo buffer: 4 planes (64 channels)
constexpr int HI = 4 * HP;                       // 44 pieces per tile: 11 per wave
constexpr int SLOTS = HI / c64::NW;
static_assert(c64::BBYTES + 2 * HB <= 160 * 1024, "LDS budget");
// LDS weight row r (within a 32-row tile) holds output channel perm32(r): accumulator register
// e of lane half h is D row (e & 3) + 8 (e >> 2) + 4 h -> channel 16 h + e
__device__ __forceinline__ int perm32(int r) { return ((r >> 2) & 1) * 16 + (r >> 3) * 4 + (r & 3); }
__device__ __forceinline__ int swz(int r) { return (r >> 3) & 1; }
}  // namespace c64w

// HPLANE: halo as 16-channel planes (true) or as 128-byte pixel rows with the 16-byte chunks
// XOR-swizzled by (row >> 1) & 7 (false: each DMA piece moves 8 whole 128-byte lines; a K step
// is then an XOR of the fragment offset, recomputed per tile instead of hoisted)
template <bool DGRAD, bool STATS, bool HPLANE = true>
__global__ __launch_bounds__(256)
void conv3x3_c64w_kernel(const bf16* __restrict__ A, const bf16* __restrict__ Wm,
                         bf16* __restrict__ Y, float* __restrict__ stats,
                         const bf16* __restrict__ addend, const C64Geom g) {
  using c64::W;
  using c64::W2;
  using c64::ROWS;
  using c64::HROWS;
  using c64::NW;
  using c64::BBYTES;
  using c64::BI;
  using namespace c64w;
  __shared__ __attribute__((aligned(16))) char smem[2 * HB + BBYTES];
  char* const Bs = smem + 2 * HB;
  typedef __attribute__((address_space(3))) const char lds_char;
  typedef __attribute__((address_space(3))) const bf16x8 lds_bf16x8;
  lds_char* const lds_base = (lds_char*)smem;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid;                            // output rows 2*wm + pt of the 8-row tile
  const int h = lane >> 5;                       // 8-channel half of a K step / 16-channel group
  const int px = lane & 31;                      // x of the lane's pixel
  const int tiles_per_img = g.H / ROWS;
  const __amdgpu_buffer_rsrc_t rsA = make_rsrc(A, g.a_bytes);

  // ---- halo DMA piece k of a wave: piece i = wid + NW*k = (plane i / HP, rows 32*(i % HP) + l/2),
  // lane half (l & 1) fetching the 8 channels 16*plane + 8*((l & 1) ^ swz(row)) ----
  auto issue_piece = [&](int n, int h0, int buf, int k) {
    const int i = wid + NW * k;
    int R, ch;
    if constexpr (HPLANE) {
      const int plane = i / HP;
      R = (i - plane * HP) * 32 + (lane >> 1);
      ch = 16 * plane + 8 * ((lane & 1) ^ swz(R));
    } else {
      R = 8 * i + (lane >> 3);
      ch = 8 * ((lane & 7) ^ ((R >> 1) & 7));
    }
    const int j = R / W2, c = R - j * W2;
    const int ih = h0 + j - 1, iw = c - 1;
    const bool ok = (R < HROWS) & ((uint32_t)ih < (uint32_t)g.H) & ((uint32_t)iw < (uint32_t)W);
    const uint32_t off = ok ? (uint32_t)((((n * g.H + ih) * W + iw) * 64 + ch) * 2) : kOOB;
    dma16(rsA, smem + buf * HB + i * 1024, off);
  };
  if (blockIdx.x < g.tiles) {
    const int n0 = blockIdx.x / tiles_per_img;
#pragma unroll
    for (int k = 0; k < SLOTS; ++k) issue_piece(n0, (blockIdx.x - n0 * tiles_per_img) * ROWS, 0, k);
  }
  // ---- resident weights: plane P = tap*4 + k (2 KiB) holds the K values tap*64 + 16k + [0,16)
  // of LDS row n = 32*ct + r (channel 32*ct + perm32(r)), halves swapped on rows with swz(n) ----
  {
    const __amdgpu_buffer_rsrc_t rsW = make_rsrc(Wm, BBYTES);
    for (int i = wid; i < BI; i += NW) {
      const int P = i >> 1, n = (i & 1) * 32 + (lane >> 1);
      const int tap = P >> 2, k = P & 3;
      const int src_tap = DGRAD ? 8 - tap : tap;
      const int ch = (n & 32) + perm32(n & 31);
      const int kv = src_tap * 64 + 16 * k + 8 * ((lane & 1) ^ swz(n));
      dma16(rsW, Bs + i * 1024, (uint32_t)((ch * 576 + kv) * 2));
    }
  }

  // fragment byte offsets within a plane: halo row R of tap (kh, kw) for (pt, px); weight row n
  int aoff[9][2], boff[2];
#pragma unroll
  for (int tap = 0; tap < 9; ++tap)
#pragma unroll
    for (int pt = 0; pt < 2; ++pt) {
      const int R = (2 * wm + pt + tap / 3) * W2 + px + tap % 3;
      aoff[tap][pt] = HPLANE ? R * 32 + ((h ^ swz(R)) << 4) : R * 128 + ((h ^ ((R >> 1) & 7)) << 4);
    }
#pragma unroll
  for (int ct = 0; ct < 2; ++ct) {
    const int n = ct * 32 + px;
    boff[ct] = n * 32 + ((h ^ swz(n)) << 4);
  }

  // per-lane BN sums. dgrad (fused BN-backward reduce): channels 32*ct + 16*h + e, kk = that BN's
  // mean. Forward statistics (shifted by kk = K): lanes 2j and 2j+1 hold the same channels of
  // different pixels, so each half-part folds the pair with one DPP swap and lane parity o keeps
  // channels 32*ct + 16*h + 8*eh + 4*o + e (e < 4): 16 channels, index ct*8 + eh*4 + e — 48 fewer
  // registers than 32 channels of sums + shifts, which spilled the two-accumulator forward.
  const bool bnf = DGRAD && g.bn_part != nullptr;
  const int odd = lane & 1;
  constexpr int NS = DGRAD ? 32 : 16;
  float st_s[NS], st_q[NS], kk[NS];
  float bistd[DGRAD ? 32 : 1];
  auto sum_ch = [&](int i) {   // channel of sum slot i
    return DGRAD ? 32 * (i >> 4) + 16 * h + (i & 15) : 32 * (i >> 3) + 16 * h + 8 * ((i >> 2) & 1) + 4 * odd + (i & 3);
  };
#pragma unroll
  for (int i = 0; i < NS; ++i) {
    const int c = sum_ch(i);
    st_s[i] = st_q[i] = 0.f;
    kk[i] = (STATS && g.kshift) ? g.kshift[c] : (bnf ? g.bn_aux[c] : 0.f);
    if constexpr (DGRAD) bistd[i] = bnf ? g.bn_aux[64 + c] : 0.f;
  }

  constexpr int STORES = 8;                      // global stores per lane per tile
  uint4 pre_a[2][2][2], pre_y[2][2][2];
  uint32_t pre_m[2][2];
  auto pix_of = [&](size_t pix0p, int pt) { return pix0p + (size_t)(2 * wm + pt) * W + px; };
  auto pre_load = [&](size_t pix0p) {
    if constexpr (DGRAD) {
#pragma unroll
      for (int pt = 0; pt < 2; ++pt)
#pragma unroll
        for (int ct = 0; ct < 2; ++ct) {
          const size_t o = pix_of(pix0p, pt) * 64 + 32 * ct + 16 * h;
          if (addend) {
            pre_a[pt][ct][0] = *reinterpret_cast<const uint4*>(addend + o);
            pre_a[pt][ct][1] = *reinterpret_cast<const uint4*>(addend + o + 8);
          }
          if (bnf) {
            pre_y[pt][ct][0] = *reinterpret_cast<const uint4*>(g.bn_y + o);
            pre_y[pt][ct][1] = *reinterpret_cast<const uint4*>(g.bn_y + o + 8);
            pre_m[pt][ct] = *reinterpret_cast<const uint16_t*>(g.bn_mask + (o >> 3));
          }
        }
    }
  };
  // one 8-channel half-part q = (pt, ct, eh) of a finished tile
  auto epi_part = [&](f32x16 (&Acc)[2][2], int q, size_t pix0p) {
    const int pt = q >> 2, ct = (q >> 1) & 1, eh = q & 1;
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = Acc[pt][ct][eh * 8 + e];
    if constexpr (STATS) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float keep = odd ? v[4 + e] : v[e];
        const float send = odd ? v[e] : v[4 + e];
        // quad_perm [1,0,3,2]: the partner lane's value
        const float recv = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(send), 0xB1, 0xF, 0xF, true));
        const int i = ct * 8 + eh * 4 + e;
        const float d1 = keep - kk[i], d2 = recv - kk[i];
        st_s[i] += d1 + d2;
        st_q[i] += d1 * d1 + d2 * d2;
      }
    }
    if constexpr (DGRAD) {
      if (addend) {   // dX = conv^T(dY) + addend in fp32, rounded to bf16 once
        float b2[8];
        unpack8(pre_a[pt][ct][eh], b2);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += b2[e];
      }
    }
    uint4 o = pack8(v);
    if constexpr (DGRAD) {
      if (bnf) {
        float f[8], yy[8];
        unpack8(o, f);
        unpack8(pre_y[pt][ct][eh], yy);
        const uint32_t m = pre_m[pt][ct] >> (8 * eh);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int i = ct * 16 + eh * 8 + e;
          const float dz = ((m >> e) & 1u) ? f[e] : 0.f;
          st_s[i] += dz;
          st_q[i] += dz * (yy[e] - kk[i]) * bistd[i];
        }
      }
    }
    *reinterpret_cast<uint4*>(Y + pix_of(pix0p, pt) * 64 + 32 * ct + 16 * h + 8 * eh) = o;
  };

  constexpr bool DEFER = !DGRAD;
  auto pix0_of = [&](int t) {
    const int n = t / tiles_per_img, h0 = (t - n * tiles_per_img) * ROWS;
    return ((size_t)n * g.H + h0) * W;
  };
  auto tile_body = [&](int t, int it, f32x16 (&Acc)[2][2], f32x16 (&Prev)[2][2], bool have_prev,
                       size_t pix0p) {
    const int buf = it & 1;
    wait_vmcnt<STORES>();                        // this tile's halo (the previous stores may fly)
    raw_barrier();
    lds_char* const Sb = lds_base + buf * HB;
    lds_char* const Wb = lds_base + 2 * HB;
    const int tn = t + (int)gridDim.x;
    const int nn_img = tn / tiles_per_img, nn_h0 = (tn - nn_img * tiles_per_img) * ROWS;
    if (DEFER && have_prev) pre_load(pix0p);
    if (!DEFER) pre_load(pix0_of(t));
#pragma unroll
    for (int pt = 0; pt < 2; ++pt)
#pragma unroll
      for (int ct = 0; ct < 2; ++ct)
#pragma unroll
        for (int e = 0; e < 16; ++e) Acc[pt][ct][e] = 0.f;
    // step st = (tap st >> 1, K steps 2 (st & 1) + kk2): 8 MFMAs; the next step's 8 fragments
    // are read in their shadow, one ds_read per MFMA (plane = immediate offset)
    int ao[9][2];   // (HPLANE = false: laundered per tile so the per-step XORs stay in the loop)
#pragma unroll
    for (int tap = 0; tap < 9; ++tap)
#pragma unroll
      for (int pt = 0; pt < 2; ++pt) {
        ao[tap][pt] = aoff[tap][pt];
        if constexpr (!HPLANE) asm volatile("" : "+v"(ao[tap][pt]));
      }
    auto load_step = [&](int st, bf16x8 (&xa)[2][2], bf16x8 (&wb)[2][2]) {
      const int tap = st >> 1;
#pragma unroll
      for (int kk2 = 0; kk2 < 2; ++kk2) {
        const int k = (st & 1) * 2 + kk2;
#pragma unroll
        for (int pt = 0; pt < 2; ++pt)
          xa[kk2][pt] = *reinterpret_cast<const lds_bf16x8*>(
              HPLANE ? Sb + k * HPB + ao[tap][pt] : Sb + (ao[tap][pt] ^ (k << 5)));
#pragma unroll
        for (int ct = 0; ct < 2; ++ct)
          wb[kk2][ct] = *reinterpret_cast<const lds_bf16x8*>(Wb + (tap * 4 + k) * 2048 + boff[ct]);
      }
    };
    bf16x8 fx[2][2][2], fw[2][2][2];
    load_step(0, fx[0], fw[0]);
#pragma unroll
    for (int st = 0; st < 18; ++st) {
      const int cur = st & 1;
      __builtin_amdgcn_sched_barrier(0);
      if (st < SLOTS) issue_piece(nn_img, nn_h0, buf ^ 1, st);
      if (st + 1 < 18) load_step(st + 1, fx[cur ^ 1], fw[cur ^ 1]);
#pragma unroll
      for (int kk2 = 0; kk2 < 2; ++kk2)
#pragma unroll
        for (int pt = 0; pt < 2; ++pt)
#pragma unroll
          for (int ct = 0; ct < 2; ++ct)
            Acc[pt][ct] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fw[cur][kk2][ct], fx[cur][kk2][pt],
                                                                 Acc[pt][ct], 0, 0, 0);
      if (st + 1 < 18) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // one MFMA
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // one ds_read
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      if (DEFER && st >= 10 && have_prev) epi_part(Prev, st - 10, pix0p);
    }
    if constexpr (!DEFER) {
#pragma unroll
      for (int q = 0; q < 8; ++q) epi_part(Acc, q, pix0_of(t));
    }
  };
  f32x16 accA[2][2], accB[2][2];
  wait_vmcnt<0>();                                // weights + first halo
  {
    int t = blockIdx.x, it = 0;
    bool have_prev = false;
    size_t pix0p = 0;
    while (t < g.tiles) {
      tile_body(t, it, accA, accB, have_prev, pix0p);
      have_prev = true;
      pix0p = pix0_of(t);
      t += gridDim.x;
      ++it;
      if (t >= g.tiles) {
        if constexpr (DEFER) {
          pre_load(pix0p);
#pragma unroll
          for (int q = 0; q < 8; ++q) epi_part(accA, q, pix0p);
        }
        break;
      }
      if constexpr (DEFER) {
        tile_body(t, it, accB, accA, have_prev, pix0p);
      } else {
        tile_body(t, it, accA, accB, have_prev, pix0p);
      }
      pix0p = pix0_of(t);
      t += gridDim.x;
      ++it;
      if (t >= g.tiles) {
        if constexpr (DEFER) {
          pre_load(pix0p);
#pragma unroll
          for (int q = 0; q < 8; ++q) epi_part(accB, q, pix0p);
        }
        break;
      }
    }
  }

  // ---- per-block channel sums: lanes with the same h (and, forward, the same parity) share
  // their sum slots' channels ----
  if (STATS || bnf) {
#pragma unroll
    for (int i = 0; i < NS; ++i)
#pragma unroll
      for (int x = DGRAD ? 1 : 2; x < 32; x <<= 1) {
        st_s[i] += __shfl_xor(st_s[i], x, 64);
        st_q[i] += __shfl_xor(st_q[i], x, 64);
      }
    wait_vmcnt<0>();
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem);  // [4 waves][64 ch][2]
    if (px < (DGRAD ? 1 : 2)) {
#pragma unroll
      for (int i = 0; i < NS; ++i) {
        red[(wm * 64 + sum_ch(i)) * 2 + 0] = st_s[i];
        red[(wm * 64 + sum_ch(i)) * 2 + 1] = st_q[i];
      }
    }
    __syncthreads();
    if (tid < 64) {
      float a = 0.f, b = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) {   // fixed order: deterministic per block
        a += red[(w * 64 + tid) * 2 + 0];
        b += red[(w * 64 + tid) * 2 + 1];
      }
      float* dst = STATS ? stats : g.bn_part;
      stat_out(dst, blockIdx.x, g.shards, 128, tid, a);
      stat_out(dst, blockIdx.x, g.shards, 128, 64 + tid, b);
    }
    if constexpr (STATS) stat_krow(stats, g.shards, 128, g.kshift, 64);
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
// diagnostics: when set, launches record per-wave tile stamps [grid][4][16][4] (int64) here
static int64_t* g_c64_prof = nullptr;
void c64_set_prof(int64_t* p) { g_c64_prof = p; }
int c64_grid_size(int N, int H) { return c64_grid(N * H / 8); }

// kernel version: PCA_C64_V (default 2; 3 / 4 are the 32x32x16 variants, measured slower:
// README round 5), or set at run time (tests compare the versions)
static int g_c64_ver = [] {
  const char* e = getenv("PCA_C64_V");
  return e ? atoi(e) : 2;
}();
int c64_version(int v) {
  const int prev = g_c64_ver;
  if (v >= 1 && v <= 4) g_c64_ver = v;
  return prev;
}

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

// forward input transform of the next conv_c64_launch(es) (bindings.cpp conv_fwd xf=...):
// scale | shift [2][64] and the ReLU-mask destination, or nullptr
static const float* g_c64_xf = nullptr;
static uint8_t* g_c64_xf_mask = nullptr;
void conv_c64_set_xf(const float* xf, uint8_t* mask) {
  g_c64_xf = xf;
  g_c64_xf_mask = mask;
}
bool conv_c64_xf_active() { return g_c64_xf != nullptr; }

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
  g.kshift = (!dgrad && stats) ? stat_shift() : nullptr;
  g.prof = nullptr;
  g.xf = dgrad ? nullptr : g_c64_xf;
  g.xf_mask = dgrad ? nullptr : g_c64_xf_mask;
  const dim3 grid(c64_grid(g.tiles)), block(256);
  if (g.xf) {
    if (!stats || !g.xf_mask) {
      fprintf(stderr, "[pca] c64 input transform needs the statistics form and a mask\n");
      abort();
    }
    hipLaunchKernelGGL((conv3x3_c64_kernel<false, true, false, true>), grid, block, 0, st, a, w, y,
                       stats, addend, g);
    return;
  }
  const int ver = c64_version(-1);
  g.prof = g_c64_prof;
  if (g.prof) {
    if (dgrad)
      hipLaunchKernelGGL((conv3x3_c64_kernel<true, false, true>), grid, block, 0, st, a, w, y, nullptr,
                         addend, g);
    else
      hipLaunchKernelGGL((conv3x3_c64_kernel<false, true, true>), grid, block, 0, st, a, w, y, stats,
                         addend, g);
    return;
  }
  if (ver == 1) {
    if (dgrad)
      hipLaunchKernelGGL((conv3x3_c64_v1_kernel<true, false>), grid, block, 0, st, a, w, y, nullptr,
                         addend, g);
    else if (stats)
      hipLaunchKernelGGL((conv3x3_c64_v1_kernel<false, true>), grid, block, 0, st, a, w, y, stats,
                         addend, g);
    else
      hipLaunchKernelGGL((conv3x3_c64_v1_kernel<false, false>), grid, block, 0, st, a, w, y, nullptr,
                         addend, g);
    return;
  }
  if (ver == 3) {
    if (dgrad)
      hipLaunchKernelGGL((conv3x3_c64w_kernel<true, false>), grid, block, 0, st, a, w, y, nullptr,
                         addend, g);
    else if (stats)
      hipLaunchKernelGGL((conv3x3_c64w_kernel<false, true>), grid, block, 0, st, a, w, y, stats,
                         addend, g);
    else
      hipLaunchKernelGGL((conv3x3_c64w_kernel<false, false>), grid, block, 0, st, a, w, y, nullptr,
                         addend, g);
    return;
  }
  if (ver == 4) {
    if (dgrad)
      hipLaunchKernelGGL((conv3x3_c64w_kernel<true, false, false>), grid, block, 0, st, a, w, y,
                         nullptr, addend, g);
    else if (stats)
      hipLaunchKernelGGL((conv3x3_c64w_kernel<false, true, false>), grid, block, 0, st, a, w, y,
                         stats, addend, g);
    else
      hipLaunchKernelGGL((conv3x3_c64w_kernel<false, false, false>), grid, block, 0, st, a, w, y,
                         nullptr, addend, g);
    return;
  }
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
