// Halo-staged weight gradient of 3x3 / stride-1 / pad-1 convolutions (the ResNet BasicBlock and
// Bottleneck 3x3 convs: reference models/resnet.py:23-27, 61-64 -> SURVEY §2.8 K3).
//
//   dW[co, (kh,kw), ci] = sum_p dY[p, co] * X[p + (kh-1, kw-1), ci]
//
// The generic wgrad gathers the X operand once per tap: nine tap-shifted copies of the same
// pixels pass through the texture path for every 64-channel block, and the kernel ends up bound
// by DMA issue and latency, not by the matrix cores. Here a stage is KP = 32 output pixels made
// of whole image rows (or whole images when W*H < 32) and the X operand is staged ONCE per stage
// as the rows' halo: (rows+2) x (W+2) pixels x 64 channels, zero-padded by the descriptor.
// The nine tap operands are then read out of that one LDS image at row offsets
// kh*(W+2) + kw with ds_read_b64_tr_b16 — 17 KiB of LDS-DMA per stage instead of 40 KiB.
//
// One workgroup owns a [64*MB output channels] x [9 taps x 64 input channels] tile (all taps of
// one 64-channel input block), walks a contiguous range of pixels, and writes its fp32 partial
// tile to a slab row (or adds it atomically when only a few workgroups share a tile). The slab
// rows are reduced into the gradient in a fixed order (deterministic).
#include "mfma_util.h"
#include "slab_reduce.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

namespace pca {

struct HaloGeom {
  int N, H, W;
  int Cx, Cy;             // channels of X and dY (all groups)
  int groups, cin_g, cout_g;
  int P;                  // N*H*W output pixels
  int Ktot;               // 9 * cin_g
  int RS, IMGS;           // image rows per image slot of a stage, image slots per stage
  int HR;                 // halo rows per stage = IMGS * (RS+2) * (W+2)
  int HI;                 // halo DMA instructions per stage = ceil(HR / 8)
  int chunk, splits, atomic;
  int ablate;             // diagnostics (PCA_HALO_ABLATE): 1 = no DMA, 2 = no MFMA phase, 4 = no epilogue
  int xcd;                // XCD-aware block order (PCA_HALO_XCD=1; default: dispatch order)
  int ilv;                // next stage's DMA pieces issued between this stage's MFMAs (PCA_HALO_ILV=0: off)
  // X input transform (X is the PRE-BatchNorm y; the conv consumed relu(BN(y)), applied on its
  // loads — conv3x3_c64.hip XF): x = relu(y * xf[c] + xf[Cx + c]) (BN scale | shift rows), or null
  const float* xf;
  uint32_t x_bytes, dy_bytes;
  FastDiv fd_hw, fd_w;
};

// transposed fragment from explicit LDS rows (row r0 for k-rows 0..3 of the lane's quad, r1 for
// 4..7) of a [row][64 channel] image with the RB = 128 swizzle
__device__ __forceinline__ bf16x8 tr_frag_rows(const char* base, int r0, int r1, int c0, int lane) {
  typedef __attribute__((address_space(3))) i16x4 lds_i16x4;
  typedef short i16x8 __attribute__((ext_vector_type(8)));
  const int p = lane & 3;
  const int col = c0 + 4 * p;
  const int chunk = col >> 3;
  const int b0 = r0 * 128 + ((chunk ^ tr_swz<128>(r0)) << 4) + ((col & 7) << 1);
  const int b1 = r1 * 128 + ((chunk ^ tr_swz<128>(r1)) << 4) + ((col & 7) << 1);
  const i16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(base + b0));
  const i16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(base + b1));
  const i16x8 v = __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, v);
}


// Compile-time stage geometry for a square W x W image (W | KP): a stage is KP output pixels =
// RS rows of IMGS images; the halo is IMGS x (RS+2) x W2P rows (row pitch W2P = W+2 rounded up to
// a multiple of 8 so that a kh*W2P row shift only flips bit 3 of the XOR swizzle key). A stage
// is KP / 32 MFMA K-steps deep: KP = 64 / 128 amortise the per-stage barrier, counted wait and
// DMA issue over 2 / 4 steps (KP = 32 left one 16x16x32 MFMA row per wave between barriers, the
// reason the bs128 shapes ran at 15 % of a CU's matrix rate).
template <int W, int KP = 32>
struct HaloShape {
  static constexpr int RS = (KP / W) <= W ? KP / W : W;
  static constexpr int IMGS = (KP / W) <= W ? 1 : (KP / W) / W;
  static constexpr int W2P = ((W + 2) + 7) / 8 * 8;
  static constexpr int HR = IMGS * (RS + 2) * W2P;
  static constexpr int HI = (HR + 7) / 8;        // halo DMA instructions per stage
  static constexpr int HBYTES = HI * 1024;
  static_assert(IMGS * RS * W == KP, "a stage must be whole rows / whole images");
};

template <int W, int MB, int KP>
constexpr int halo_stage_bytes() {
  return HaloShape<W, KP>::HBYTES + MB * KP * 128 + 1024;
}
constexpr int kHaloXfBytes = 512;   // the X transform's scale | shift of the 64-channel block
template <int W, int MB, int KP, int ST = 3>
constexpr bool halo_fits() {
  return ST * halo_stage_bytes<W, MB, KP>() + kHaloXfBytes <= 160 * 1024;
}

// ST = LDS stages in the ring (ST - 1 stages in flight): the small-image shapes of the 8-GPU
// shard (layer 4 at bs128: 96 tiles, 32 short stages per tile, DMA-latency bound with 2 stages in
// flight) take 6 stages of 32 pixels instead of 3 of 64.
template <int W, int MB, int WM, int WN, int KP, int TG = 9, int ST = 3, bool XF = false>
__global__ __launch_bounds__(WM * WN * 64) __attribute__((amdgpu_waves_per_eu(2, 2))) void wgrad_halo_kernel(const bf16* __restrict__ X,
                                                                  const bf16* __restrict__ DY,
                                                                  float* __restrict__ out,
                                                                  const HaloGeom g) {
  using SH = HaloShape<W, KP>;
  constexpr int NW = WM * WN;
  constexpr int KS = KP / 32;                    // MFMA K-steps per stage
  constexpr int DYI = KP / 8;                    // DMA instructions per 64-channel dY block
  constexpr int STAGES = ST;
  static_assert(ST >= 3, "stages");
  constexpr int A_OFF = SH::HBYTES;              // dY blocks follow the halo image
  constexpr int J_OFF = A_OFF + MB * KP * 128;   // junk KiB for the padding DMA slots
  constexpr int STAGE = J_OFF + 1024;
  // TG = 3: a workgroup owns one kernel row (3 taps) of the output tile, so the grid has 3x the
  // tiles and needs 3x fewer pixel splits to fill the chip (slab traffic / 3; none at all when
  // the tiles alone fill it, e.g. ResNet layer 4 on the 8-GPU shard)
  static_assert(TG == 9 || TG == 3, "taps per workgroup");
  constexpr int BM = MB * 64, BN = TG * 64;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int T = SH::HI + DYI * MB;           // real DMA instructions per stage
  constexpr int SLOTS = (T + NW - 1) / NW;       // every wave issues exactly SLOTS per stage
  constexpr int W2P = SH::W2P;
  static_assert(WTM % 16 == 0 && WTN % 16 == 0, "wave tile");
  static_assert(32 % W == 0, "image width");
  __shared__ __attribute__((aligned(16))) char smem[STAGES * STAGE + (XF ? kHaloXfBytes : 0)];
  float* const xfs = reinterpret_cast<float*>(smem + STAGES * STAGE);   // [sc | sh][64]

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  // XCD-aware block order: consecutive workgroups go to consecutive XCDs, so the tiles of one
  // pixel split (which stage the same X halo and dY rows) were spread over all eight L2s. The
  // remap gives each XCD a contiguous range of the (split, tile) order: one split's tiles share
  // an L2, and the staged pixels are fetched beyond it once per XCD instead of once per tile.
  const int gxy = gridDim.x * gridDim.y;
  int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
  if (g.xcd) {
    const int q = xcd_remap(bx + gridDim.x * (by + gridDim.y * bz), gxy * gridDim.z);
    bx = q % gridDim.x;
    by = (q / gridDim.x) % gridDim.y;
    bz = q / gxy;
  }
  const int split = bz % g.splits;
  const int grp = bz / g.splits;
  const int m0 = bx * BM;                      // output channel tile (within group)
  const int cinb = g.cin_g / 64;
  const int cib = by % cinb;                   // 64-channel input block
  const int tap0 = TG == 9 ? 0 : (by / cinb) * 3;   // first tap of this row
  const int p_begin = split * g.chunk;
  const int p_end = min(g.P, p_begin + g.chunk);

  const __amdgpu_buffer_rsrc_t rsX = make_rsrc(X, g.x_bytes);
  const __amdgpu_buffer_rsrc_t rsD = make_rsrc(DY, g.dy_bytes);

  // ---- per-lane DMA slots (fixed for the kernel) ----
  // halo slot: packed (row ok, image slot, halo row j, halo col c) + swizzled chunk byte offset
  // dY slot:   stage pixel r + (swizzled chunk + channel) byte offset
  int s_a[SLOTS], s_b[SLOTS];
#pragma unroll
  for (int j = 0; j < SLOTS; ++j) {
    const int t = wid + NW * j;
    const int row8 = lane >> 3;
    if (t < SH::HI) {
      const int hr = 8 * t + row8;
      const int img = hr / ((SH::RS + 2) * W2P);
      const int rem = hr - img * ((SH::RS + 2) * W2P);
      const int jr = rem / W2P, c = rem - jr * W2P;
      const bool ok = hr < SH::HR && c < W + 2;
      s_a[j] = (ok << 24) | (img << 16) | (jr << 8) | c;
      s_b[j] = (((lane & 7) ^ tr_swz<128>(hr)) << 4) + (grp * g.cin_g + cib * 64) * 2;
    } else if (t < T) {
      const int q = t - SH::HI;
      const int r = 8 * (q % DYI) + row8;
      s_a[j] = r;
      s_b[j] = (((lane & 7) ^ tr_swz<128>(r)) << 4) + (grp * g.cout_g + m0 + 64 * (q / DYI)) * 2;
    } else {
      s_a[j] = 0;
      s_b[j] = 0;
    }
  }

  // DMA slot j of the stage starting at pixel pbase into ring buffer buf
  auto issue_slot = [&](int pbase, int buf, int j) {
    if (g.ablate & 1) return;
    char* S = smem + buf * STAGE;
    const bool live = pbase < p_end;
    // first image / row of the stage (W power of two: shifts)
    const int n0 = pbase / (W * W);
    const int h0 = (pbase / W) % W;
    {
      const int t = wid + NW * j;                // wave-uniform slot kind
      uint32_t off = kOOB;
      if (t < SH::HI) {
        const int n = n0 + ((s_a[j] >> 16) & 0xff);
        const int ih = h0 + ((s_a[j] >> 8) & 0xff) - 1;
        const int iw = (s_a[j] & 0xff) - 1;
        const bool ok = live && (s_a[j] >> 24) && n < g.N && (uint32_t)ih < (uint32_t)W &&
                        (uint32_t)iw < (uint32_t)W;
        if (ok) off = (uint32_t)((((n * W + ih) * W + iw) * g.Cx) * 2 + s_b[j]);
        dma16(rsX, S + t * 1024, off);
      } else if (t < T) {
        const int q = t - SH::HI;
        const int p = pbase + s_a[j];
        if (live && p < p_end) off = (uint32_t)(p * g.Cy * 2 + s_b[j]);
        dma16(rsD, S + A_OFF + (q / DYI) * KP * 128 + (q % DYI) * 1024, off);
      } else {
        dma16(rsD, S + J_OFF, kOOB);              // keeps vmcnt per wave uniform
      }
    }
  };
  auto issue = [&](int pbase, int buf) {
#pragma unroll
    for (int j = 0; j < SLOTS; ++j) issue_slot(pbase, buf, j);
  };

  // X transform of this wave's own halo pieces of the stage at pbase (they landed: the counted
  // wait), in place before the stage barrier publishes them; padding pieces (DMA'd zeros) stay
  // zero. Arithmetic as the BN apply pass (batchnorm.hip bn_apply_rows_body).
  auto xform_stage = [&](int pbase, int buf) {
    const char* S = smem + buf * STAGE;
    const int n0 = pbase / (W * W);
    const int h0 = (pbase / W) % W;
#pragma unroll
    for (int j = 0; j < SLOTS; ++j) {
      const int t = wid + NW * j;                // (wave-uniform)
      if (t >= SH::HI) continue;
      const int n = n0 + ((s_a[j] >> 16) & 0xff);
      const int ih = h0 + ((s_a[j] >> 8) & 0xff) - 1;
      const int iw = (s_a[j] & 0xff) - 1;
      const bool ok = pbase < p_end && (s_a[j] >> 24) && n < g.N && (uint32_t)ih < (uint32_t)W &&
                      (uint32_t)iw < (uint32_t)W;
      if (!ok) continue;
      const int c0 = ((s_b[j] >> 1) & 63) & ~7;  // chunk of the 64-channel block (8 channels)
      uint4* p = reinterpret_cast<uint4*>(const_cast<char*>(S) + t * 1024 + lane * 16);
      float f[8];
      unpack8(*p, f);
#pragma unroll
      for (int v = 0; v < 8; ++v) f[v] = apply_act(f[v] * xfs[c0 + v] + xfs[64 + c0 + v], ACT_RELU);
      *p = pack8(f);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  };
  if constexpr (XF) {   // this workgroup's 64 input channels' scale | shift
    const int cb = grp * g.cin_g + cib * 64;
    for (int i = tid; i < 128; i += NW * 64) xfs[i] = g.xf[(i < 64 ? 0 : g.Cx - 64) + cb + i];
    __syncthreads();
  }

  // ---- per-lane B-fragment addressing: halo rows of this lane's two pixel rows ----
  // B frag (tap kh,kw; columns c0..c0+15 of the 64-channel block) for the lane lives at
  //   row R = prow + kh*W2P + kw,  byte = R*128 + ((c0/8 ^ swz(R)) << 4) + L
  // and swz(R) = swz(prow + kw) ^ (kh*W2P/8 odd ? 4 : 0) because W2P % 8 == 0. K-step ks of a
  // stage covers the stage pixels 32*ks .. 32*ks + 31.
  int rbase[KS][2], swk[KS][2][3];
  {
    const int q = (lane & 15) >> 2, pq = lane & 3;
    const int L = ((pq >> 1) << 4) + ((pq & 1) << 3);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int r = 32 * ks + 8 * (lane >> 4) + q + 4 * h;
        const int img = r / (SH::RS * W), rr = r - img * (SH::RS * W);
        const int jj = rr / W, ow = rr - jj * W;
        const int prow = img * (SH::RS + 2) * W2P + jj * W2P + ow;
        rbase[ks][h] = prow * 128 + L;
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) swk[ks][h][kw] = tr_swz<128>(prow + kw) << 4;
      }
  }

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  typedef __attribute__((address_space(3))) i16x4 lds_i16x4;
  typedef short i16x8 __attribute__((ext_vector_type(8)));
  const int KT = p_end > p_begin ? cdiv(p_end - p_begin, KP) : 0;
#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s) issue(p_begin + s * KP, s);
  for (int kt = 0; kt < KT; ++kt) {
    wait_vmcnt<(STAGES - 2) * SLOTS>();   // stage kt landed (the STAGES - 2 after it may not have)
    if constexpr (XF) xform_stage(p_begin + kt * KP, kt % STAGES);
    raw_barrier();
    const int pnext = p_begin + (kt + STAGES - 1) * KP, bnext = (kt + STAGES - 1) % STAGES;
    // the next stage's pieces: all at once here, or (g.ilv, wave-uniform) spread over this
    // stage's MFMAs — issued as a block they kept the matrix pipe idle (the DMA-only and MFMA-only
    // ablations of this kernel added up instead of overlapping)
    if (!g.ilv || (g.ablate & 2)) issue(pnext, bnext);
    if (g.ablate & 2) continue;
    const char* S = smem + (kt % STAGES) * STAGE;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      bf16x8 af[TM];
#pragma unroll
      for (int mi = 0; mi < TM; ++mi) {
        const int m = wm * WTM + mi * 16;
        af[mi] = tr_frag<64>(S + A_OFF + (m >> 6) * KP * 128, 32 * ks, m & 63, lane);
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int ni = 0; ni < TN; ++ni) {
        const int n = wn * WTN + ni * 16;
        const int tap = tap0 + (n >> 6), kh = tap / 3, kw = tap % 3;
        const int c0 = n & 63;
        const int cx = ((c0 >> 3) ^ (((kh * W2P / 8) & 1) ? 4 : 0)) << 4;
        const int rsh = (kh * W2P + kw) * 128;
        const i16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (lds_i16x4*)(S + rbase[ks][0] + rsh + (cx ^ swk[ks][0][kw])));
        const i16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (lds_i16x4*)(S + rbase[ks][1] + rsh + (cx ^ swk[ks][1][kw])));
        const bf16x8 bfv = __builtin_bit_cast(bf16x8, (i16x8)__builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
        for (int mi = 0; mi < TM; ++mi)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mi], bfv, acc[mi][ni], 0, 0, 0);
        if (g.ilv) {
          // slot j after MFMA group (ks, ni) = j * KS * TN / SLOTS (compile-time after unrolling)
#pragma unroll
          for (int j = 0; j < SLOTS; ++j)
            if (ks * TN + ni == (j * KS * TN) / SLOTS) issue_slot(pnext, bnext, j);
        }
      }
      __builtin_amdgcn_s_setprio(0);
    }
  }
  wait_vmcnt<0>();
  if (g.ablate & 4) return;

  if (!g.atomic) {
    // slab row in accumulator order: each (wave, mi, ni) fragment is one 1 KiB dwordx4 store of
    // 64 lanes x float4, instead of 4 dword stores of 4 x 64-byte row pieces each (the scattered
    // store tail alone took ~18 us of the ~25 us kernel on the bs128 shard: 256 blocks x 147 KB).
    // halo_slab_reduce_kernel maps the order back to dW[co][tap][ci].
    const int tiles = gridDim.x * gridDim.y * g.groups;
    const int tile = (grp * gridDim.x + bx) * gridDim.y + by;
    float4* dst4 = reinterpret_cast<float4*>(out) + (size_t)(split * tiles + tile) * (BM * BN / 4);
#pragma unroll
    for (int mi = 0; mi < TM; ++mi)
#pragma unroll
      for (int ni = 0; ni < TN; ++ni)
        dst4[((wid * TM + mi) * TN + ni) * 64 + lane] =
            make_float4(acc[mi][ni][0], acc[mi][ni][1], acc[mi][ni][2], acc[mi][ni][3]);
    return;
  }
#pragma unroll
  for (int mi = 0; mi < TM; ++mi)
#pragma unroll
    for (int ni = 0; ni < TN; ++ni) {
      const int n = wn * WTN + ni * 16 + (lane & 15);
      const int col = (tap0 + (n >> 6)) * g.cin_g + cib * 64 + (n & 63);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = m0 + wm * WTM + mi * 16 + (lane >> 4) * 4 + j;
        if (m < g.cout_g) {
          const size_t idx = ((size_t)grp * g.cout_g + m) * g.Ktot + col;
          if (g.splits == 1) out[idx] += acc[mi][ni][j];   // sole writer
          else atomicAdd(out + idx, acc[mi][ni][j]);
        }
      }
    }
}

// dW += sum_s slab[s] in a fixed order: a block owns 64 float4 slots; its L = blockDim/64 split
// lanes sum slab rows s = l, l+L, ... (4 loads in flight), the L partials are added in lane order,
// and the slot is scattered back to dW[co][tap][ci] (its 4 rows).
__global__ __launch_bounds__(1024) void halo_slab_reduce_kernel(const float4* __restrict__ slab,
                                                                float* __restrict__ dw, int splits,
                                                                int64_t n4, HaloSlabMap mp) {
  __shared__ float4 red[16][64];
  const int c = threadIdx.x & 63, l = threadIdx.x >> 6, L = blockDim.x >> 6;
  const int64_t q = (int64_t)blockIdx.x * 64 + c;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  if (q < n4) {
    int s = l;
    for (; s + 3 * L < splits; s += 4 * L) {
      const float4 v0 = slab[(int64_t)s * n4 + q];
      const float4 v1 = slab[(int64_t)(s + L) * n4 + q];
      const float4 v2 = slab[(int64_t)(s + 2 * L) * n4 + q];
      const float4 v3 = slab[(int64_t)(s + 3 * L) * n4 + q];
      a.x += v0.x; a.y += v0.y; a.z += v0.z; a.w += v0.w;
      a.x += v1.x; a.y += v1.y; a.z += v1.z; a.w += v1.w;
      a.x += v2.x; a.y += v2.y; a.z += v2.z; a.w += v2.w;
      a.x += v3.x; a.y += v3.y; a.z += v3.z; a.w += v3.w;
    }
    for (; s < splits; s += L) {
      const float4 v = slab[(int64_t)s * n4 + q];
      a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
  }
  red[l][c] = a;
  __syncthreads();
  if (l != 0 || q >= n4) return;
  for (int k = 1; k < L; ++k) {
    const float4 v = red[k][c];
    a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
  }
  const int per_tile = mp.BM * mp.BN / 4;
  const int tile = (int)(q / per_tile);
  int r = (int)(q - (int64_t)tile * per_tile);
  const int lane = r & 63;
  r >>= 6;
  const int ni = r % mp.TN;
  r /= mp.TN;
  const int mi = r % mp.TM;
  const int wid = r / mp.TM;
  const int wm = wid / mp.WN, wn = wid - wm * mp.WN;
  const int by = tile % mp.tiles_y;
  const int bx = (tile / mp.tiles_y) % mp.tiles_x;
  const int grp = tile / (mp.tiles_y * mp.tiles_x);
  const int n = wn * mp.WTN + ni * 16 + (lane & 15);
  const int cinb = mp.cin_g / 64;
  const int tap0 = mp.TG == 9 ? 0 : (by / cinb) * 3;
  const int col = (tap0 + (n >> 6)) * mp.cin_g + (by % cinb) * 64 + (n & 63);
  const int mb = bx * mp.BM + wm * mp.WTM + mi * 16 + (lane >> 4) * 4;
  const float v[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (mb + j < mp.cout_g) dw[((size_t)grp * mp.cout_g + mb + j) * mp.Ktot + col] += v[j];
}

// Slab reduction in a fixed order, one kernel: a block owns 64 float4 columns; its L =
// blockDim/64 thread lanes per column sum the slab rows s = l, l+L, ... (4 loads in flight) and
// the L lane partials are added in lane order (deterministic) before dW += sum.
__global__ __launch_bounds__(1024) void slab_reduce_kernel(const float4* __restrict__ slab,
                                                           float4* __restrict__ dw, int splits,
                                                           int64_t n4) {
  __shared__ float4 red[16][64];
  const int c = threadIdx.x & 63, l = threadIdx.x >> 6, L = blockDim.x >> 6;
  const int64_t i = (int64_t)blockIdx.x * 64 + c;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i < n4) {
    int s = l;
    for (; s + 3 * L < splits; s += 4 * L) {
      const float4 v0 = slab[(int64_t)s * n4 + i];
      const float4 v1 = slab[(int64_t)(s + L) * n4 + i];
      const float4 v2 = slab[(int64_t)(s + 2 * L) * n4 + i];
      const float4 v3 = slab[(int64_t)(s + 3 * L) * n4 + i];
      a.x += v0.x; a.y += v0.y; a.z += v0.z; a.w += v0.w;
      a.x += v1.x; a.y += v1.y; a.z += v1.z; a.w += v1.w;
      a.x += v2.x; a.y += v2.y; a.z += v2.z; a.w += v2.w;
      a.x += v3.x; a.y += v3.y; a.z += v3.z; a.w += v3.w;
    }
    for (; s < splits; s += L) {
      const float4 v = slab[(int64_t)s * n4 + i];
      a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
  }
  red[l][c] = a;
  __syncthreads();
  if (l == 0 && i < n4) {
    float4 o = dw[i];
    for (int k = 0; k < L; ++k) {
      const float4 v = red[k][c];
      o.x += v.x; o.y += v.y; o.z += v.z; o.w += v.w;
    }
    dw[i] = o;
  }
}

__global__ __launch_bounds__(1024) void slab_reduce_multi_kernel(SlabRedBatch b) {
  __shared__ float4 red[16][64];
  slab_reduce_multi_body<16>(b, (int)blockIdx.x, red);
}

// ---------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------
static bool g_defer_on = false;            // set around a production wgrad launch (bindings)
static std::vector<SlabRedDesc> g_deferred;

void wgrad_defer_scope(bool on) { g_defer_on = on; }
// drop the reductions recorded after the first n (tuning trials on scratch gradients; the real
// pending ones of the backward pass in progress stay)
void wgrad_truncate_pending(int n) {
  if ((size_t)n < g_deferred.size()) g_deferred.resize(n);
}
int wgrad_deferred_count() { return (int)g_deferred.size(); }

static int split_lanes(int splits) {
  int L = 1;   // split lanes per column: a power of two <= min(16, splits)
  while (L < 16 && 2 * L <= splits) L *= 2;
  return L;
}

static bool defer_reduce(const float* ws, float* dw, int splits, int64_t n4, const HaloSlabMap* mp) {
  if (!g_defer_on) return false;
  SlabRedDesc d{};
  d.slab = reinterpret_cast<const float4*>(ws);
  d.dw = dw;
  d.n4 = n4;
  d.splits = splits;
  d.L = split_lanes(splits);
  d.halo = mp ? 1 : 0;
  if (mp) d.mp = *mp;
  g_deferred.push_back(d);
  return true;
}

// Launch every pending reduction (in recording order, kSlabRedMax per launch) and forget them.
void wgrad_flush_launch(hipStream_t st) {
  size_t i = 0;
  while (i < g_deferred.size()) {
    SlabRedBatch b{};
    int blocks = 0;
    for (; i < g_deferred.size() && b.n < kSlabRedMax; ++i) {
      SlabRedDesc d = g_deferred[i];
      d.block0 = blocks;
      blocks += (int)cdiv64(d.n4, 64);
      b.d[b.n++] = d;
    }
    hipLaunchKernelGGL(slab_reduce_multi_kernel, dim3((unsigned)blocks), dim3(1024), 0, st, b);
  }
  g_deferred.clear();
}

// Hand every pending reduction (at most kSlabRedMax, else none) to a launch that runs them as
// extra 64-column workgroups (the next BatchNorm-backward kernel): returns those workgroups, 0 =
// nothing taken.
int wgrad_take_pending(SlabRedBatch* b) {
  if (g_deferred.empty() || g_deferred.size() > (size_t)kSlabRedMax) return 0;
  int blocks = 0;
  b->n = 0;
  for (const SlabRedDesc& d0 : g_deferred) {
    SlabRedDesc d = d0;
    d.block0 = blocks;
    blocks += (int)cdiv64(d.n4, 64);
    b->d[b->n++] = d;
  }
  g_deferred.clear();
  return blocks;
}

static int halo_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    if (n <= 0) n = 256;
  }
  return n;
}

// X(cfg, MB, WM, WN, KP, TG, ST)
#define PCA_HALO_CFGS(X)       \
  X(0, 1, 1, 4, 32, 9, 3)      \
  X(1, 2, 2, 4, 32, 9, 3)      \
  X(2, 1, 2, 4, 32, 9, 3)      \
  X(3, 1, 2, 4, 64, 9, 3)      \
  X(4, 2, 2, 4, 64, 9, 3)      \
  X(5, 1, 2, 4, 128, 9, 3)     \
  X(6, 1, 1, 4, 64, 9, 3)      \
  X(7, 1, 2, 4, 64, 3, 3)      \
  X(8, 1, 1, 4, 64, 3, 3)      \
  X(9, 2, 2, 4, 64, 3, 3)      \
  X(10, 2, 2, 4, 32, 3, 6)     \
  X(11, 1, 2, 4, 32, 3, 6)     \
  X(12, 1, 1, 4, 32, 3, 6)     \
  X(13, 1, 2, 4, 32, 9, 6)     \
  X(14, 2, 2, 4, 64, 3, 4)
constexpr int kHaloCfgs = 15;

template <int W, int MB, int WM, int WN, int KP, int TG, int ST>
static int halo_occupancy() {
  static int occ = 0;
  if (occ == 0) {
    occ = blocks_per_cu((const void*)wgrad_halo_kernel<W, MB, WM, WN, KP, TG, ST>, WM * WN * 64,
                        "wgrad_halo");
  }
  return occ;
}

static int g_halo_override = -1;
void set_halo_cfg(int cfg) { g_halo_override = cfg; }

// X transform of the next halo wgrad launch(es) (bindings.cpp conv_wgrad xf=...), or nullptr
static const float* g_halo_xf = nullptr;
void set_halo_xf(const float* xf) { g_halo_xf = xf; }
bool halo_xf_active() { return g_halo_xf != nullptr; }

// Deterministic mode: every weight gradient is reduced through slab rows in a fixed order
// (no fp32 atomics), so repeated runs are bitwise identical.
static bool g_deterministic = false;
void set_deterministic_conv(bool on) { g_deterministic = on; }
bool deterministic_conv() { return g_deterministic; }

// Forced split-K plan for the wgrad kernels (autotuner trials / tuned choices): splits >= 1
// replaces the occupancy-derived split count and forces fp32 atomics (non-deterministic mode);
// splits <= -2 fixes the count at -splits with deterministic slab rows (autotune candidates that
// trade parallelism against slab traffic, which does not shrink with the batch).
static int g_wsplit = -1;
void set_wgrad_split(int splits) { g_wsplit = splits; }
int wgrad_split_force() { return g_deterministic ? -1 : g_wsplit; }

// dW[i] += sum_s slab[s][i] over `splits` rows of n floats (fixed order); the workspace must
// hold slab_ws_floats(splits, n) floats.
void slab_reduce_launch(float* ws, float* dw, int splits, int64_t n, hipStream_t st) {
  const int64_t n4 = n / 4;
  if (defer_reduce(ws, dw, splits, n4, nullptr)) return;
  const int L = split_lanes(splits);
  hipLaunchKernelGGL(slab_reduce_kernel, dim3((unsigned)cdiv64(n4, 64)), dim3(64 * L), 0, st,
                     reinterpret_cast<const float4*>(ws), reinterpret_cast<float4*>(dw), splits, n4);
}

int64_t slab_ws_floats(int splits, int64_t n) { return (int64_t)splits * n; }

// Is the halo kernel applicable? 3x3 s1 p1, 64-channel blocks, whole rows (or images) per stage.
static bool halo_geom(HaloGeom& g, int N, int H, int W, int Cin, int Cout, int groups) {
  g.N = N; g.H = H; g.W = W; g.Cx = Cin; g.Cy = Cout;
  g.groups = groups; g.cin_g = Cin / groups; g.cout_g = Cout / groups;
  g.P = N * H * W;
  g.Ktot = 9 * g.cin_g;
  if (g.cin_g % 64 || g.cout_g % 64) return false;
  if (H != W || (W != 4 && W != 8 && W != 16 && W != 32)) return false;
  g.x_bytes = (uint32_t)((size_t)N * H * W * Cin * 2);
  g.dy_bytes = (uint32_t)((size_t)N * H * W * Cout * 2);
  g.fd_hw = make_fastdiv(H * W);
  g.fd_w = make_fastdiv(W);
  static const int abl = [] {
    const char* e = getenv("PCA_HALO_ABLATE");
    return e ? atoi(e) : 0;
  }();
  g.ablate = abl;
  // (measured neutral on the ResNet-18 wgrad shapes at bs1024 and bs128: off by default)
  static const int xcd = [] {
    const char* e = getenv("PCA_HALO_XCD");
    return e && e[0] == '1' ? 1 : 0;
  }();
  g.xcd = xcd;
  // (default on: ResNet-18 3x3 wgrads 4-8 % faster per call, step 6.49 -> 6.41 ms at bs1024 and
  // 1.885 -> 1.86 ms at bs128, same box; PCA_HALO_ILV=0 issues each stage's pieces as a block)
  static const int ilv = [] {
    const char* e = getenv("PCA_HALO_ILV");
    return e && e[0] == '0' ? 0 : 1;
  }();
  g.ilv = ilv;
  g.xf = g_halo_xf;
  return true;
}

static int halo_select(const HaloGeom& g) {
  if (g_halo_override >= 0) return g_halo_override;
  return g.cout_g <= 64 ? 0 : 1;
}

template <int W, int MB, int WM, int WN, int KP, int TG, int ST>
static int64_t halo_plan(HaloGeom& g) {
  const int tiles = cdiv(g.cout_g, 64 * MB) * (g.cin_g / 64) * (9 / TG) * g.groups;
  const int slots = halo_occupancy<W, MB, WM, WN, KP, TG, ST>() * halo_cus();
  int splits = std::max(1, slots / tiles);
  splits = std::min(splits, std::max(1, cdiv(g.P, 256)));
  const int forced = wgrad_split_force();
  if (forced >= 1) splits = std::min(forced, std::max(1, cdiv(g.P, 32)));
  if (forced <= -2) splits = std::min(-forced, std::max(1, cdiv(g.P, 32)));   // slab, fixed count
  int chunk = cdiv(cdiv(g.P, splits), KP) * KP;
  splits = cdiv(g.P, chunk);
  g.chunk = chunk;
  g.splits = splits;
  g.atomic = (splits == 1 || (!g_deterministic && forced >= 1) ||
              (!g_deterministic && forced == -1 && splits <= 4)) ? 1 : 0;
  static const bool verbose = getenv("PCA_CONV_VERBOSE") != nullptr;
  if (verbose)
    fprintf(stderr, "[pca] halo wgrad W=%d MB=%d waves=%d KP=%d: occ=%d cus=%d tiles=%d splits=%d chunk=%d atomic=%d\n",
            W, MB, WM * WN, KP, halo_occupancy<W, MB, WM, WN, KP, TG, ST>(), halo_cus(), tiles, splits,
            chunk, g.atomic);
  if (g.atomic) return 0;
  return slab_ws_floats(splits, (int64_t)tiles * (64 * MB) * (TG * 64));
}

template <int W, int MB, int WM, int WN, int KP, int TG, int ST>
static void launch_halo(const bf16* x, const bf16* dy, float* dw, float* ws, HaloGeom g,
                        hipStream_t st) {
  halo_plan<W, MB, WM, WN, KP, TG, ST>(g);
  dim3 grid(cdiv(g.cout_g, 64 * MB), (g.cin_g / 64) * (9 / TG), g.splits * g.groups);
  if (g.xf) {
    // (the X transform is instantiated for the 32-wide layer-1 images only: conv_xf_supported)
    if constexpr (W == 32) {
      hipLaunchKernelGGL((wgrad_halo_kernel<W, MB, WM, WN, KP, TG, ST, true>), grid,
                         dim3(WM * WN * 64), 0, st, x, dy, g.atomic ? dw : ws, g);
    } else {
      fprintf(stderr, "[pca] halo wgrad X transform: W=%d not instantiated\n", W);
      abort();
    }
  } else {
    hipLaunchKernelGGL((wgrad_halo_kernel<W, MB, WM, WN, KP, TG, ST>), grid, dim3(WM * WN * 64), 0,
                       st, x, dy, g.atomic ? dw : ws, g);
  }
  if (g.atomic) return;
  constexpr int BM = 64 * MB, BN = TG * 64;
  HaloSlabMap mp;
  mp.BM = BM;
  mp.BN = BN;
  mp.WN = WN;
  mp.WTM = BM / WM;
  mp.WTN = BN / WN;
  mp.TM = mp.WTM / 16;
  mp.TN = mp.WTN / 16;
  mp.tiles_x = (int)grid.x;
  mp.tiles_y = (int)grid.y;
  mp.cout_g = g.cout_g;
  mp.cin_g = g.cin_g;
  mp.Ktot = g.Ktot;
  mp.TG = TG;
  const int64_t n4 = (int64_t)grid.x * grid.y * g.groups * (BM * BN / 4);
  if (defer_reduce(ws, dw, g.splits, n4, &mp)) return;
  const int L = split_lanes(g.splits);   // split lanes per slot
  hipLaunchKernelGGL(halo_slab_reduce_kernel, dim3((unsigned)cdiv64(n4, 64)), dim3(64 * L), 0, st,
                     reinterpret_cast<const float4*>(ws), dw, g.splits, n4, mp);
}

// One dispatcher for planning (ws == nullptr && plan_only) and launching.
template <int W>
static int64_t halo_dispatch_w(const bf16* x, const bf16* dy, float* dw, float* ws, HaloGeom& g,
                               hipStream_t st, bool plan_only) {
  switch (halo_select(g)) {
#define PCA_CASE(C, MB, WM, WN, KP, TG, ST)                              \
    case C:                                                              \
      if constexpr (halo_fits<W, MB, KP, ST>()) {                        \
        if (plan_only) return halo_plan<W, MB, WM, WN, KP, TG, ST>(g);   \
        launch_halo<W, MB, WM, WN, KP, TG, ST>(x, dy, dw, ws, g, st);    \
        return 0;                                                        \
      }                                                                  \
      break;
    PCA_HALO_CFGS(PCA_CASE)
#undef PCA_CASE
    default:
      break;
  }
  // (a configuration whose LDS stages do not fit this image width falls back to cfg 0)
  if (plan_only) return halo_plan<W, 1, 1, 4, 32, 9, 3>(g);
  launch_halo<W, 1, 1, 4, 32, 9, 3>(x, dy, dw, ws, g, st);
  return 0;
}

static int64_t halo_dispatch(const bf16* x, const bf16* dy, float* dw, float* ws, HaloGeom& g,
                             hipStream_t st, bool plan_only) {
  switch (g.W) {
    case 4: return halo_dispatch_w<4>(x, dy, dw, ws, g, st, plan_only);
    case 8: return halo_dispatch_w<8>(x, dy, dw, ws, g, st, plan_only);
    case 16: return halo_dispatch_w<16>(x, dy, dw, ws, g, st, plan_only);
    default: return halo_dispatch_w<32>(x, dy, dw, ws, g, st, plan_only);
  }
}

// workspace floats for the halo wgrad, or -1 when the halo kernel does not apply
int64_t wgrad_halo_ws_floats(int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride,
                             int pad, int groups) {
  if (KH != 3 || KW != 3 || stride != 1 || pad != 1) return -1;
  HaloGeom g;
  if (!halo_geom(g, N, H, W, Cin, Cout, groups)) return -1;
  return halo_dispatch(nullptr, nullptr, nullptr, nullptr, g, nullptr, true);
}

void wgrad_halo_launch(const bf16* x, const bf16* dy, float* dw, float* ws, int N, int H, int W,
                       int Cin, int Cout, int groups, hipStream_t st) {
  HaloGeom g;
  halo_geom(g, N, H, W, Cin, Cout, groups);
  halo_dispatch(x, dy, dw, ws, g, st, false);
}

}  // namespace pca
