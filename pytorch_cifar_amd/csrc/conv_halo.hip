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

#include <algorithm>

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

template <int N>
__device__ __forceinline__ void wait_vmcnt_rt(int n) {
  // counted wait with a wave-uniform runtime count (n <= N)
  if constexpr (N > 0) {
    if (n >= N) {
      wait_vmcnt<N>();
      return;
    }
    wait_vmcnt_rt<N - 1>(n);
  } else {
    wait_vmcnt<0>();
  }
}

constexpr int kHaloMaxHI = 13;                 // W = 32: 3 x 34 = 102 halo rows
constexpr int kHaloBytes = kHaloMaxHI * 1024;

template <int MB, int WM, int WN>
__global__ __launch_bounds__(WM * WN * 64) void wgrad_halo_kernel(const bf16* __restrict__ X,
                                                                  const bf16* __restrict__ DY,
                                                                  float* __restrict__ out,
                                                                  const HaloGeom g) {
  constexpr int NW = WM * WN;
  constexpr int KP = 32;
  constexpr int STAGES = 3;
  constexpr int A_OFF = kHaloBytes;             // dY blocks follow the halo image
  constexpr int STAGE = kHaloBytes + MB * KP * 128;
  constexpr int BM = MB * 64, BN = 9 * 64;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int TMAX = kHaloMaxHI + 4 * MB;     // DMA instructions per stage (upper bound)
  constexpr int SLOTS = (TMAX + NW - 1) / NW;   // per wave
  static_assert(WTM % 16 == 0 && WTN % 16 == 0, "wave tile");
  __shared__ __attribute__((aligned(16))) char smem[STAGES * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int split = blockIdx.z % g.splits;
  const int grp = blockIdx.z / g.splits;
  const int m0 = blockIdx.x * BM;              // output channel tile (within group)
  const int cib = blockIdx.y;                  // 64-channel input block
  const int p_begin = split * g.chunk;
  const int p_end = min(g.P, p_begin + g.chunk);
  const int W2 = g.W + 2;

  const __amdgpu_buffer_rsrc_t rsX = make_rsrc(X, g.x_bytes);
  const __amdgpu_buffer_rsrc_t rsD = make_rsrc(DY, g.dy_bytes);

  // ---- per-lane DMA slots (fixed for the kernel): kind 0 = halo row group, 1 = dY rows ----
  const int T = g.HI + 4 * MB;
  int s_kind[SLOTS], s_a[SLOTS], s_b[SLOTS], s_lds[SLOTS];
#pragma unroll
  for (int j = 0; j < SLOTS; ++j) {
    const int t = wid + NW * j;
    const int row8 = lane >> 3;
    s_kind[j] = 2;
    s_a[j] = 0;
    s_b[j] = 0;
    s_lds[j] = 0;
    if (t < g.HI) {
      const int hr = 8 * t + row8;               // halo row
      const int per_img = (g.RS + 2) * W2;
      const int img = hr / per_img;
      const int rem = hr - img * per_img;
      const int jr = rem / W2;
      const int c = rem - jr * W2;
      s_kind[j] = 0;                             // (wave-uniform: one DMA per slot)
      // packed (row-valid, image slot, halo row, halo col); halo (jr, c) = input
      // (h0 + jr - 1, c - 1); rows past the halo (the last instruction's tail) load zeros
      s_a[j] = ((hr < g.HR) << 24) | (img << 16) | (jr << 8) | c;
      s_b[j] = (((lane & 7) ^ tr_swz<128>(hr)) << 4);
      s_lds[j] = t * 1024;
    } else if (t < T) {
      const int q = t - g.HI;                    // dY instruction: block q>>2, row group q&3
      const int r = 8 * (q & 3) + row8;          // stage pixel
      s_kind[j] = 1;
      s_a[j] = r;
      s_b[j] = (((lane & 7) ^ tr_swz<128>(r)) << 4) + (grp * g.cout_g + m0 + 64 * (q >> 2)) * 2;
      s_lds[j] = A_OFF + (q >> 2) * KP * 128 + (q & 3) * 1024;
    }
  }
  // loads this wave issues per stage (wave-uniform)
  const int my_loads = (T - wid + NW - 1) / NW;

  auto issue = [&](int pbase, int buf) {
    char* S = smem + buf * STAGE;
    const bool live = pbase < p_end;
    // stage geometry (uniform): first image and first row of the stage
    const uint32_t pp = live ? (uint32_t)pbase : 0u;
    const int n0 = (int)fdiv(pp, g.fd_hw);
    const int h0 = (int)fdiv(pp - (uint32_t)n0 * (uint32_t)(g.H * g.W), g.fd_w);
#pragma unroll
    for (int j = 0; j < SLOTS; ++j) {
      const int kind = s_kind[j];
      if (kind == 2) continue;
      uint32_t off = kOOB;
      if (kind == 0) {
        const int n = n0 + ((s_a[j] >> 16) & 0xff);
        const int ih = h0 + ((s_a[j] >> 8) & 0xff) - 1;
        const int iw = (s_a[j] & 0xff) - 1;
        const bool ok = live && (s_a[j] >> 24) && n < g.N && (uint32_t)ih < (uint32_t)g.H &&
                        (uint32_t)iw < (uint32_t)g.W;
        if (ok)
          off = (uint32_t)((((n * g.H + ih) * g.W + iw) * g.Cx + grp * g.cin_g + cib * 64) * 2 + s_b[j]);
        dma16(rsX, S + s_lds[j], off);
      } else {
        const int p = pbase + s_a[j];
        if (live && p < p_end) off = (uint32_t)(p * g.Cy * 2 + s_b[j]);
        dma16(rsD, S + s_lds[j], off);
      }
    }
  };

  // per-lane halo rows of the pixels this lane's B fragments cover (tap (0,0))
  int prow0, prow1;
  {
    const int q = (lane & 15) >> 2;
    const int r0 = 8 * (lane >> 4) + q, r1 = r0 + 4;
    const int rsw = g.RS * g.W;
    auto hrow = [&](int r) {
      const int img = r / rsw, rr = r - img * rsw;
      const int j = rr / g.W, ow = rr - j * g.W;
      return img * (g.RS + 2) * W2 + j * W2 + ow;
    };
    prow0 = hrow(r0);
    prow1 = hrow(r1);
  }

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int KT = p_end > p_begin ? cdiv(p_end - p_begin, KP) : 0;
  issue(p_begin, 0);
  issue(p_begin + KP, 1);
  for (int kt = 0; kt < KT; ++kt) {
    wait_vmcnt_rt<8>(my_loads);     // stage kt landed (stage kt+1 may still be in flight)
    raw_barrier();
    issue(p_begin + (kt + 2) * KP, (kt + 2) % STAGES);
    const char* S = smem + (kt % STAGES) * STAGE;
    bf16x8 af[TM];
#pragma unroll
    for (int mi = 0; mi < TM; ++mi) {
      const int m = wm * WTM + mi * 16;
      af[mi] = tr_frag<64>(S + A_OFF + (m >> 6) * KP * 128, 0, m & 63, lane);
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ni = 0; ni < TN; ++ni) {
      const int n = wn * WTN + ni * 16;
      const int tap = n >> 6;
      const int toff = (tap / 3) * W2 + (tap % 3);
      const bf16x8 bfv = tr_frag_rows(S, prow0 + toff, prow1 + toff, n & 63, lane);
#pragma unroll
      for (int mi = 0; mi < TM; ++mi)
        acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mi], bfv, acc[mi][ni], 0, 0, 0);
    }
    __builtin_amdgcn_s_setprio(0);
  }
  wait_vmcnt<0>();

  float* dst = g.atomic ? out : out + (size_t)split * g.groups * g.cout_g * g.Ktot;
#pragma unroll
  for (int mi = 0; mi < TM; ++mi)
#pragma unroll
    for (int ni = 0; ni < TN; ++ni) {
      const int n = wn * WTN + ni * 16 + (lane & 15);
      const int col = (n >> 6) * g.cin_g + cib * 64 + (n & 63);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = m0 + wm * WTM + mi * 16 + (lane >> 4) * 4 + j;
        if (m < g.cout_g) {
          const size_t idx = ((size_t)grp * g.cout_g + m) * g.Ktot + col;
          if (g.atomic) atomicAdd(dst + idx, acc[mi][ni][j]);
          else dst[idx] = acc[mi][ni][j];
        }
      }
    }
}

// Slab reduction in a fixed order: stage 1 sums groups of <= 16 slab rows into part[g];
// stage 2 adds the parts (in order) into dW.
__global__ __launch_bounds__(256) void slab_partial_kernel(const float4* __restrict__ slab,
                                                           float4* __restrict__ part, int splits,
                                                           int per, int64_t n4) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  const int s0 = blockIdx.y * per, s1 = min(splits, s0 + per);
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int s = s0; s < s1; ++s) {
    const float4 v = slab[(int64_t)s * n4 + i];
    a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
  }
  part[(int64_t)blockIdx.y * n4 + i] = a;
}

__global__ __launch_bounds__(256) void slab_final_kernel(const float4* __restrict__ part,
                                                         float4* __restrict__ dw, int nparts,
                                                         int64_t n4) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  float4 a = dw[i];
  for (int s = 0; s < nparts; ++s) {
    const float4 v = part[(int64_t)s * n4 + i];
    a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
  }
  dw[i] = a;
}

// ---------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------
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

// X(cfg, MB, WM, WN)
#define PCA_HALO_CFGS(X) \
  X(0, 1, 1, 4)          \
  X(1, 2, 2, 4)          \
  X(2, 1, 2, 4)

template <int MB, int WM, int WN>
static int halo_occupancy() {
  static int occ = 0;
  if (occ == 0) {
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void*)wgrad_halo_kernel<MB, WM, WN>,
                                                 WM * WN * 64, 0);
    occ = std::max(1, occ);
  }
  return occ;
}

static int g_halo_override = -1;
void set_halo_cfg(int cfg) { g_halo_override = cfg; }

// Is the halo kernel applicable? 3x3 s1 p1, 64-channel blocks, whole rows (or images) per stage.
static bool halo_geom(HaloGeom& g, int N, int H, int W, int Cin, int Cout, int groups) {
  g.N = N; g.H = H; g.W = W; g.Cx = Cin; g.Cy = Cout;
  g.groups = groups; g.cin_g = Cin / groups; g.cout_g = Cout / groups;
  g.P = N * H * W;
  g.Ktot = 9 * g.cin_g;
  if (g.cin_g % 64 || g.cout_g % 64 || 32 % W) return false;
  const int rows = 32 / W;                    // image rows per stage
  if (rows <= H) {
    if (H % rows) return false;
    g.RS = rows; g.IMGS = 1;
  } else {
    if (rows % H) return false;
    g.RS = H; g.IMGS = rows / H;
  }
  g.HR = g.IMGS * (g.RS + 2) * (W + 2);
  g.HI = cdiv(g.HR, 8);
  if (g.HI > kHaloMaxHI) return false;
  g.x_bytes = (uint32_t)((size_t)N * H * W * Cin * 2);
  g.dy_bytes = (uint32_t)((size_t)N * H * W * Cout * 2);
  g.fd_hw = make_fastdiv(H * W);
  g.fd_w = make_fastdiv(W);
  return true;
}

static int halo_select(const HaloGeom& g) {
  if (g_halo_override >= 0) return g_halo_override;
  return g.cout_g <= 64 ? 0 : 1;
}

template <int MB, int WM, int WN>
static int64_t halo_plan(HaloGeom& g) {
  const int tiles = cdiv(g.cout_g, 64 * MB) * (g.cin_g / 64) * g.groups;
  const int slots = halo_occupancy<MB, WM, WN>() * halo_cus();
  int splits = std::max(1, slots / tiles);
  splits = std::min(splits, std::max(1, cdiv(g.P, 256)));
  int chunk = cdiv(cdiv(g.P, splits), 32) * 32;
  splits = cdiv(g.P, chunk);
  g.chunk = chunk;
  g.splits = splits;
  g.atomic = splits <= 4 ? 1 : 0;
  if (g.atomic) return 0;
  const int64_t n = (int64_t)g.groups * g.cout_g * g.Ktot;
  const int nparts = cdiv(splits, 16);
  return (int64_t)splits * n + (int64_t)nparts * n;   // slab rows + partial sums
}

static int64_t halo_plan_any(HaloGeom& g) {
  switch (halo_select(g)) {
#define PCA_CASE(C, MB, WM, WN) \
    case C: return halo_plan<MB, WM, WN>(g);
    PCA_HALO_CFGS(PCA_CASE)
#undef PCA_CASE
    default: return halo_plan<1, 1, 4>(g);
  }
}

// workspace floats for the halo wgrad, or -1 when the halo kernel does not apply
int64_t wgrad_halo_ws_floats(int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride,
                             int pad, int groups) {
  if (KH != 3 || KW != 3 || stride != 1 || pad != 1) return -1;
  HaloGeom g;
  if (!halo_geom(g, N, H, W, Cin, Cout, groups)) return -1;
  return halo_plan_any(g);
}

template <int MB, int WM, int WN>
static void launch_halo(const bf16* x, const bf16* dy, float* dw, float* ws, HaloGeom g,
                        hipStream_t st) {
  halo_plan<MB, WM, WN>(g);
  dim3 grid(cdiv(g.cout_g, 64 * MB), g.cin_g / 64, g.splits * g.groups);
  hipLaunchKernelGGL((wgrad_halo_kernel<MB, WM, WN>), grid, dim3(WM * WN * 64), 0, st, x, dy,
                     g.atomic ? dw : ws, g);
  if (!g.atomic) {
    const int64_t n = (int64_t)g.groups * g.cout_g * g.Ktot;
    const int64_t n4 = n / 4;
    const int per = 16, nparts = cdiv(g.splits, per);
    float* part = ws + (int64_t)g.splits * n;
    const unsigned gx = (unsigned)cdiv64(n4, 256);
    hipLaunchKernelGGL(slab_partial_kernel, dim3(gx, nparts), dim3(256), 0, st,
                       reinterpret_cast<const float4*>(ws), reinterpret_cast<float4*>(part),
                       g.splits, per, n4);
    hipLaunchKernelGGL(slab_final_kernel, dim3(gx), dim3(256), 0, st,
                       reinterpret_cast<const float4*>(part), reinterpret_cast<float4*>(dw), nparts,
                       n4);
  }
}

void wgrad_halo_launch(const bf16* x, const bf16* dy, float* dw, float* ws, int N, int H, int W,
                       int Cin, int Cout, int groups, hipStream_t st) {
  HaloGeom g;
  halo_geom(g, N, H, W, Cin, Cout, groups);
  switch (halo_select(g)) {
#define PCA_CASE(C, MB, WM, WN) \
    case C: launch_halo<MB, WM, WN>(x, dy, dw, ws, g, st); break;
    PCA_HALO_CFGS(PCA_CASE)
#undef PCA_CASE
    default: launch_halo<1, 1, 4>(x, dy, dw, ws, g, st); break;
  }
}

}  // namespace pca
