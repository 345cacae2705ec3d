// Training/eval BatchNorm2d with fused activation and residual on NHWC bf16 activations.
//
// Replaces cuDNN BN + F.relu + the in-place residual add of the reference blocks
// (models/resnet.py:47-51 `relu(bn2(conv2(out)) + shortcut(x))`,
// efficientnet.py:96-103 swish(bn(...)), mobilenetv2.py:33-36).
//
// Forward:  stats partials (from the conv epilogue, or bn_stats_kernel for a bare tensor)
//           -> colsum (stage-1 fold) -> bn_finalize (mean/invstd/scale/shift + running stats)
//           -> bn_apply: out = act(y*scale + shift [+ res | + y2*scale2 + shift2]).
// Backward: bn_bwd_reduce (sum dz, sum dz*xhat [, sum dz*xhat2]) -> colsum -> bn_bwd_finalize
//           (dgamma, dbeta, per-channel affine coefficients) -> bn_bwd_apply
//           dy = a*dz + b*y + d  (dz = dout * act'(z), the residual gradient is dz itself).
// Every reduction is a deterministic slab fold (no float atomics).
#include "common.h"
#include "slab_reduce.h"

#include <cstdlib>

namespace pca {

static int g_stat_shards = 0;
int stat_shards() { return g_stat_shards; }
void set_stat_shards(int shards) { g_stat_shards = shards; }
static const float* g_stat_shift = nullptr;
const float* stat_shift() { return g_stat_shift; }
void set_stat_shift(const float* k) { g_stat_shift = k; }

// Row strides (elements between consecutive NHWC pixels) of the tensors the next BN launch
// touches, 0 = dense (the channel count): a channel slice of a wider concat slab is a row-strided
// [M][C] matrix, so concatenation can be zero-copy (producers write their slice, consumers read a
// channel range; models/densenet.py, googlenet.py, dla*.py). Set by the host bindings around a
// launch (like stat_shards); only the row-tiled kernels (C % 8 == 0) take strides.
//   y: BN input, out: forward output, dout: backward input gradient, dx: backward output
//   (dx_acc: the backward adds into dx instead of overwriting it)
static BnLd g_bn_ld{};
BnLd bn_ld() { return g_bn_ld; }
void set_bn_ld(const BnLd& ld) { g_bn_ld = ld; }
static bool bn_ld_dense() {
  return g_bn_ld.y == 0 && g_bn_ld.out == 0 && g_bn_ld.dout == 0 && g_bn_ld.dx == 0 && !g_bn_ld.dx_acc;
}
__host__ __device__ __forceinline__ int ld_or(int ld, int C) { return ld ? ld : C; }

// Row-parallel geometry for an [M][C] NHWC matrix: TPR threads cover a row's granules
// (VEC channels each), RPP rows are processed per pass by one 256-thread block.
struct RowPar {
  int C, G, TPR, RPP;
};

static inline RowPar make_rowpar(int C, int vec) {
  RowPar r;
  r.C = C;
  r.G = (C + vec - 1) / vec;
  r.TPR = r.G < 256 ? r.G : 256;
  r.RPP = 256 / r.TPR;
  return r;
}

// VEC = 8 / 4 / 2 / 1 channels per access (16 / 8 / 4 / 2 bytes): the widest that divides C, so
// odd-width nets (ShuffleNet 58/116/232, PNASNet 44, densenet growth 12) are not scalar
template <int VEC>
__device__ __forceinline__ void load_vec(const bf16* p, float* f) {
  if constexpr (VEC == 8) {
    unpack8(*reinterpret_cast<const uint4*>(p), f);
  } else if constexpr (VEC == 4) {
    const uint2 u = *reinterpret_cast<const uint2*>(p);
    f[0] = __uint_as_float(u.x << 16);
    f[1] = __uint_as_float(u.x & 0xffff0000u);
    f[2] = __uint_as_float(u.y << 16);
    f[3] = __uint_as_float(u.y & 0xffff0000u);
  } else if constexpr (VEC == 2) {
    const uint32_t u = *reinterpret_cast<const uint32_t*>(p);
    f[0] = __uint_as_float(u << 16);
    f[1] = __uint_as_float(u & 0xffff0000u);
  } else {
    f[0] = bf2f(*p);
  }
}

template <int VEC>
__device__ __forceinline__ void store_vec(bf16* p, const float* f) {
  if constexpr (VEC == 8) {
    *reinterpret_cast<uint4*>(p) = pack8(f);
  } else if constexpr (VEC == 4) {
    *reinterpret_cast<uint2*>(p) = make_uint2(pack2(f[0], f[1]), pack2(f[2], f[3]));
  } else if constexpr (VEC == 2) {
    *reinterpret_cast<uint32_t*>(p) = pack2(f[0], f[1]);
  } else {
    *p = f2bf(f[0]);
  }
}

// ---- per-channel sum / sumsq partials of a bare tensor: partial[P][2][C] ----
// centered (krow != nullptr): sums of x - K with K[c] = x[0][c] (the first row: a value within a
// few standard deviations of the channel mean, the same for every block), K published in krow
// for the finalize / fold (robust variance, see common.h stat_shift)
template <int VEC>
__global__ __launch_bounds__(256) void bn_stats_kernel(const bf16* __restrict__ x, int M,
                                                       RowPar rp, int rows_per_block,
                                                       float* __restrict__ partial, int shards,
                                                       float* __restrict__ krow, int ldx, int ldc,
                                                       bf16* __restrict__ dst, int ldd) {
  __shared__ float red[256 * VEC * 2];
  const int t = threadIdx.x;
  const int gx = t % rp.TPR, ry = t / rp.TPR;
  const int r0 = blockIdx.x * rows_per_block;
  const int r1 = min(M, r0 + rows_per_block);
  if (krow && blockIdx.x == 0)
    for (int c = t; c < rp.C; c += 256) krow[c] = bf2f(x[c]);
  for (int gbase = 0; gbase < rp.G; gbase += rp.TPR) {
    const int gi = gbase + gx;
    float s[VEC], q[VEC], k[VEC];
#pragma unroll
    for (int v = 0; v < VEC; ++v) s[v] = q[v] = k[v] = 0.f;
    if (krow && gi < rp.G) load_vec<VEC>(x + gi * VEC, k);
    if (ry < rp.RPP && gi < rp.G) {
      // 4 rows in flight per thread (the rows are independent loads; one at a time left these
      // small-grid reductions latency bound: ~12 us for 1 MB)
      int r = r0 + ry;
      for (; r + 3 * rp.RPP < r1; r += 4 * rp.RPP) {
        float f[4][VEC];
#pragma unroll
        for (int u = 0; u < 4; ++u) load_vec<VEC>(x + (size_t)(r + u * rp.RPP) * ldx + gi * VEC, f[u]);
        if (dst) {   // (bf16 -> fp32 -> bf16: exact)
#pragma unroll
          for (int u = 0; u < 4; ++u) store_vec<VEC>(dst + (size_t)(r + u * rp.RPP) * ldd + gi * VEC, f[u]);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int v = 0; v < VEC; ++v) {
            const float d = f[u][v] - k[v];
            s[v] += d;
            q[v] += d * d;
          }
      }
      for (; r < r1; r += rp.RPP) {
        float f[VEC];
        load_vec<VEC>(x + (size_t)r * ldx + gi * VEC, f);
        if (dst) store_vec<VEC>(dst + (size_t)r * ldd + gi * VEC, f);
#pragma unroll
        for (int v = 0; v < VEC; ++v) {
          const float d = f[v] - k[v];
          s[v] += d;
          q[v] += d * d;
        }
      }
    }
#pragma unroll
    for (int v = 0; v < VEC; ++v) {
      red[(t * VEC + v) * 2] = s[v];
      red[(t * VEC + v) * 2 + 1] = q[v];
    }
    __syncthreads();
    if (ry == 0 && gi < rp.G) {
      for (int k = 1; k < rp.RPP; ++k) {
        const int tt = k * rp.TPR + gx;
#pragma unroll
        for (int v = 0; v < VEC; ++v) {
          s[v] += red[(tt * VEC + v) * 2];
          q[v] += red[(tt * VEC + v) * 2 + 1];
        }
      }
#pragma unroll
      for (int v = 0; v < VEC; ++v) {
        const int c = gi * VEC + v;
        if (c < rp.C) {
          stat_out(partial, blockIdx.x, shards, 2 * ldc, c, s[v]);
          stat_out(partial, blockIdx.x, shards, 2 * ldc, ldc + c, q[v]);
        }
      }
    }
    __syncthreads();
  }
}

// ---- stage-1 fold: in[R][L] -> out[R2][L], out row j sums rows [j*chunk, (j+1)*chunk) ----
__global__ __launch_bounds__(256) void colsum_kernel(const float* __restrict__ in, int R, int L,
                                                     int chunk, float* __restrict__ out) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= L) return;
  const int r0 = blockIdx.y * chunk, r1 = min(R, r0 + chunk);
  float s = 0.f;
  for (int r = r0; r < r1; ++r) s += in[(size_t)r * L + c];
  out[(size_t)blockIdx.y * L + c] = s;
}

// ---- bias gradient: db[c] (+)= sum_r stat[r][0][c] (the per-channel sums of dY from the
// bn_stats partials), 64 channels x 16 row lanes per block, lanes added in a fixed order; written
// straight into the gradient arena (no separate reduce + accumulate-add launches)
__global__ __launch_bounds__(1024) void bias_grad_fold_kernel(const float* __restrict__ stat,
                                                              int R, int C, int accumulate,
                                                              float* __restrict__ db) {
  __shared__ float red[16][64];
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  float s = 0.f;
  if (c < C)
    for (int r = rl; r < R; r += 16) s += stat[(size_t)r * 2 * C + c];
  red[rl][cl] = s;
  __syncthreads();
  if (rl == 0 && c < C) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) t += red[k][cl];
    db[c] = accumulate ? db[c] + t : t;
  }
}

void bias_grad_fold_launch(const float* stat, int R, int C, int accumulate, float* db,
                           hipStream_t st) {
  hipLaunchKernelGGL(bias_grad_fold_kernel, dim3(cdiv(C, 64)), dim3(1024), 0, st, stat, R, C,
                     accumulate, db);
}

// ---- forward finalize: stat[R][2][C] -> aux[4][C] = {mean, invstd, scale, shift} ----
// One 1024-thread block per 64 channels: 16 row-lanes fold the R (<= 1024) partial rows in
// parallel (coalesced 256-byte row segments), then lane-row 0 combines them in fp64.
// kin: the shift K[c] the producer subtracted (its K row / the pilot it read; nullptr = 0);
// pilot_out: receives the batch mean (the next step's K; may alias kin — one thread per channel
// reads K before writing the mean)
__global__ __launch_bounds__(1024) void bn_finalize_kernel(
    const float* __restrict__ stat, int R, int C, double count, const float* __restrict__ gamma,
    const float* __restrict__ beta, float* __restrict__ rmean, float* __restrict__ rvar,
    int64_t* __restrict__ nbt, float momentum, float eps, int training, int update_running,
    float* __restrict__ aux, const float* kin, float* pilot_out, float* zero, int zero_n, int ld) {
  // (stat rows [R][2][ld], ld >= C: a zero-padded conv's statistics are read in place, its
  // padding channels skipped)
  __shared__ float red[16][64][2];
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  // block 0 clears this BN's backward accumulator (its consumer dgrad refills it later in the
  // step; no memset launch on the separate-statistics path)
  if (zero && blockIdx.x == 0)
    for (int i = threadIdx.x; i < zero_n; i += blockDim.x) zero[i] = 0.f;
  if (blockIdx.x == 0 && threadIdx.x == 0 && update_running && nbt) nbt[0] += 1;
  float s = 0.f, q = 0.f;
  if (training && c < C) {
#pragma unroll 4
    for (int r = rl; r < R; r += 16) {
      s += stat[(size_t)r * 2 * ld + c];
      q += stat[(size_t)r * 2 * ld + ld + c];
    }
  }
  red[rl][cl][0] = s;
  red[rl][cl][1] = q;
  __syncthreads();
  if (rl != 0 || c >= C) return;
  float mean, var;
  if (training) {
    double ds = 0.0, dq = 0.0;
    for (int k = 0; k < 16; ++k) {
      ds += red[k][cl][0];
      dq += red[k][cl][1];
    }
    const double m = ds / count;          // mean of x - K
    double v = dq / count - m * m;
    if (v < 0.0) v = 0.0;
    mean = (float)(m + (kin ? (double)kin[c] : 0.0));
    var = (float)v;
    if (pilot_out) pilot_out[c] = mean;
    if (update_running) {
      const double unb = count > 1.0 ? v * count / (count - 1.0) : v;
      rmean[c] = (1.f - momentum) * rmean[c] + momentum * mean;
      rvar[c] = (1.f - momentum) * rvar[c] + momentum * (float)unb;
    }
  } else {
    mean = rmean[c];
    var = rvar[c];
  }
  const float invstd = rsqrtf(var + eps);
  const float g = gamma ? gamma[c] : 1.f;
  const float b = beta ? beta[c] : 0.f;
  aux[c] = mean;
  aux[C + c] = invstd;
  aux[2 * C + c] = g * invstd;
  aux[3 * C + c] = b - mean * g * invstd;
}

// ---- apply: out = act(y*scale + shift [+ res] [+ y2*scale2 + shift2]) ----
template <int VEC>
__global__ __launch_bounds__(256) void bn_apply_kernel(const bf16* __restrict__ y,
                                                       const float* __restrict__ aux, int C,
                                                       size_t total, const bf16* __restrict__ res,
                                                       const bf16* __restrict__ y2,
                                                       const float* __restrict__ aux2, int act,
                                                       bf16* __restrict__ out,
                                                       uint8_t* __restrict__ mask, int ldy) {
  // (ldy > C: y is the channel prefix of wider rows — a zero-padded conv's output read in place)
  const size_t nvec = total / VEC;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < nvec; i += (size_t)gridDim.x * 256) {
    const size_t e = i * VEC;
    const int c0 = (int)(e % C);
    const size_t ey = ldy == C ? e : (e / C) * ldy + c0;
    float f[VEC];
    load_vec<VEC>(y + ey, f);
#pragma unroll
    for (int v = 0; v < VEC; ++v) f[v] = f[v] * aux[2 * C + c0 + v] + aux[3 * C + c0 + v];
    if (res) {
      float r[VEC];
      load_vec<VEC>(res + e, r);
#pragma unroll
      for (int v = 0; v < VEC; ++v) f[v] += r[v];
    }
    if (y2) {
      float r[VEC];
      load_vec<VEC>(y2 + e, r);
#pragma unroll
      for (int v = 0; v < VEC; ++v) f[v] += r[v] * aux2[2 * C + c0 + v] + aux2[3 * C + c0 + v];
    }
#pragma unroll
    for (int v = 0; v < VEC; ++v) f[v] = apply_act(f[v], act);
    store_vec<VEC>(out + e, f);
    if constexpr (VEC == 8) {
      // ReLU mask as bits (1 byte per 8 channels): the backward reads T/16 bytes instead of the
      // bf16 output (T), which it only needs for the sign
      if (mask) {
        uint32_t b = 0;
#pragma unroll
        for (int v = 0; v < 8; ++v) b |= (f[v] > 0.f ? 1u : 0u) << v;
        mask[i] = (uint8_t)b;
      }
    }
  }
}

// dz from the incoming gradient: relu uses the saved output as mask; swish/sigmoid recompute z.
// (e: element offset in the dense [M][C] indexing of out / mask; ed, ey: of dout, y)
template <int VEC>
__device__ __forceinline__ void compute_dz(const bf16* dout, const bf16* out, const uint8_t* mask,
                                           const bf16* y, const float* aux, int C, int c0, size_t e,
                                           int act, float* dz, size_t ed, size_t ey) {
  load_vec<VEC>(dout + ed, dz);
  if (act == ACT_RELU && VEC == 8 && mask) {
    const uint32_t b = mask[e >> 3];
#pragma unroll
    for (int v = 0; v < VEC; ++v) dz[v] = ((b >> v) & 1u) ? dz[v] : 0.f;
  } else if (act == ACT_RELU) {
    float o[VEC];
    load_vec<VEC>(out + e, o);
#pragma unroll
    for (int v = 0; v < VEC; ++v) dz[v] = o[v] > 0.f ? dz[v] : 0.f;
  } else if (act != ACT_NONE) {
    float yy[VEC];
    load_vec<VEC>(y + ey, yy);
#pragma unroll
    for (int v = 0; v < VEC; ++v) {
      const float z = yy[v] * aux[2 * C + c0 + v] + aux[3 * C + c0 + v];
      dz[v] *= act_grad(z, act);
    }
  }
}

// ---- backward reduce: partial[P][NS][C] with sums of dz, dz*xhat, (dz*xhat2) ----
// Fast path body (8 channels, single BN; masked ReLU / swish / no act): kBwdRows rows of one
// thread from clamped (unconditional) loads issued before the per-channel constants, rows past
// r1 weighted 0. Straight-line loads matter on the small late-stage tensors, where each thread
// sees only a few rows: a guarded / loop-carried chain of them (and branchy per-element loads
// of the constants) left the kernel latency-bound at ~10 us whatever the size.
constexpr int kBwdRows = 4;
// RA: activation derivative recomputed from y and aux scale | shift (0 none, ACT_SWISH,
// ACT_RELU_Y)
template <bool MASK, int RA>
__device__ __forceinline__ void bwd_reduce_rows(const bf16* __restrict__ dout,
                                                const bf16* __restrict__ y,
                                                const uint8_t* __restrict__ mask,
                                                const float* __restrict__ aux, int C, int c0, int r,
                                                int r1, int rpp, float (&acc)[2][8], int ldd,
                                                int ldy) {
  uint4 dr[kBwdRows], yr[kBwdRows];
  uint32_t mr[kBwdRows];
  float wgt[kBwdRows];
#pragma unroll
  for (int k = 0; k < kBwdRows; ++k) {
    const int rk = r + k * rpp;
    wgt[k] = rk < r1 ? 1.f : 0.f;
    const size_t rr = (size_t)min(rk, r1 - 1);
    const size_t e = rr * C + c0;
    dr[k] = *reinterpret_cast<const uint4*>(dout + rr * ldd + c0);
    yr[k] = *reinterpret_cast<const uint4*>(y + rr * ldy + c0);
    mr[k] = MASK ? mask[e >> 3] : 0xffu;
  }
  // aux = [mean | istd | scale | shift] x C (scale / shift: the BN affine as used by the act)
  float mean[8], istd[8], sc[8], sh[8];
  const float4* a4 = reinterpret_cast<const float4*>(aux + c0);
  const int q = C >> 2;
  const float4 m0 = a4[0], m1 = a4[1], i0 = a4[q], i1 = a4[q + 1];
  mean[0] = m0.x; mean[1] = m0.y; mean[2] = m0.z; mean[3] = m0.w;
  mean[4] = m1.x; mean[5] = m1.y; mean[6] = m1.z; mean[7] = m1.w;
  istd[0] = i0.x; istd[1] = i0.y; istd[2] = i0.z; istd[3] = i0.w;
  istd[4] = i1.x; istd[5] = i1.y; istd[6] = i1.z; istd[7] = i1.w;
  if constexpr (RA != 0) {
    const float4 s0 = a4[2 * q], s1 = a4[2 * q + 1], h0 = a4[3 * q], h1 = a4[3 * q + 1];
    sc[0] = s0.x; sc[1] = s0.y; sc[2] = s0.z; sc[3] = s0.w;
    sc[4] = s1.x; sc[5] = s1.y; sc[6] = s1.z; sc[7] = s1.w;
    sh[0] = h0.x; sh[1] = h0.y; sh[2] = h0.z; sh[3] = h0.w;
    sh[4] = h1.x; sh[5] = h1.y; sh[6] = h1.z; sh[7] = h1.w;
  }
#pragma unroll
  for (int k = 0; k < kBwdRows; ++k) {
    float dz[8], yy[8];
    unpack8(dr[k], dz);
    unpack8(yr[k], yy);
#pragma unroll
    for (int v = 0; v < 8; ++v) {
      float a = ((mr[k] >> v) & 1u) ? dz[v] * wgt[k] : 0.f;
      if constexpr (RA != 0) a *= act_grad(yy[v] * sc[v] + sh[v], RA);
      acc[0][v] += a;
      acc[1][v] += a * (yy[v] - mean[v]) * istd[v];
    }
  }
}

template <int VEC, int NS>
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(
    const bf16* __restrict__ dout, const bf16* __restrict__ out, const uint8_t* __restrict__ mask,
    const bf16* __restrict__ y, const float* __restrict__ aux, const bf16* __restrict__ y2,
    const float* __restrict__ aux2, int act, int M, RowPar rp, int rows_per_block,
    float* __restrict__ partial, int shards, int ldd, int ldy) {
  __shared__ float red[256 * VEC * NS];
  const int t = threadIdx.x;
  const int gx = t % rp.TPR, ry = t / rp.TPR;
  const int C = rp.C;
  const int r0 = blockIdx.x * rows_per_block;
  const int r1 = min(M, r0 + rows_per_block);
  for (int gbase = 0; gbase < rp.G; gbase += rp.TPR) {
    const int gi = gbase + gx;
    const int c0 = gi * VEC;
    float acc[NS][VEC];
#pragma unroll
    for (int k = 0; k < NS; ++k)
#pragma unroll
      for (int v = 0; v < VEC; ++v) acc[k][v] = 0.f;
    if (ry < rp.RPP && gi < rp.G) {
      float mean[VEC], istd[VEC], mean2[VEC], istd2[VEC];
#pragma unroll
      for (int v = 0; v < VEC; ++v) {
        mean[v] = aux[c0 + v];
        istd[v] = aux[C + c0 + v];
        if (NS == 3) {
          mean2[v] = aux2[c0 + v];
          istd2[v] = aux2[C + c0 + v];
        }
      }
      int r = r0 + ry;
      if constexpr (VEC == 8 && NS == 2) {
        // masked-ReLU / no-act / swish fast path (bwd_reduce_rows)
        if (mask)
          for (; r < r1; r += kBwdRows * rp.RPP)
            bwd_reduce_rows<true, 0>(dout, y, mask, aux, C, c0, r, r1, rp.RPP, acc, ldd, ldy);
        else if (act == ACT_SWISH)
          for (; r < r1; r += kBwdRows * rp.RPP)
            bwd_reduce_rows<false, ACT_SWISH>(dout, y, mask, aux, C, c0, r, r1, rp.RPP, acc, ldd, ldy);
        else if (act == ACT_RELU_Y)
          for (; r < r1; r += kBwdRows * rp.RPP)
            bwd_reduce_rows<false, ACT_RELU_Y>(dout, y, mask, aux, C, c0, r, r1, rp.RPP, acc, ldd, ldy);
        else if (act == ACT_NONE)
          for (; r < r1; r += kBwdRows * rp.RPP)
            bwd_reduce_rows<false, 0>(dout, y, mask, aux, C, c0, r, r1, rp.RPP, acc, ldd, ldy);
      }
      for (; r < r1; r += rp.RPP) {
        const size_t e = (size_t)r * C + c0;
        float dz[VEC], yy[VEC];
        compute_dz<VEC>(dout, out, mask, y, aux, C, c0, e, act, dz, (size_t)r * ldd + c0,
                        (size_t)r * ldy + c0);
        load_vec<VEC>(y + (size_t)r * ldy + c0, yy);
#pragma unroll
        for (int v = 0; v < VEC; ++v) {
          acc[0][v] += dz[v];
          acc[1][v] += dz[v] * (yy[v] - mean[v]) * istd[v];
        }
        if constexpr (NS == 3) {
          float y2v[VEC];
          load_vec<VEC>(y2 + e, y2v);
#pragma unroll
          for (int v = 0; v < VEC; ++v) acc[2][v] += dz[v] * (y2v[v] - mean2[v]) * istd2[v];
        }
      }
    }
#pragma unroll
    for (int k = 0; k < NS; ++k)
#pragma unroll
      for (int v = 0; v < VEC; ++v) red[(t * VEC + v) * NS + k] = acc[k][v];
    __syncthreads();
    if (ry == 0 && gi < rp.G) {
      for (int j = 1; j < rp.RPP; ++j) {
        const int tt = j * rp.TPR + gx;
#pragma unroll
        for (int k = 0; k < NS; ++k)
#pragma unroll
          for (int v = 0; v < VEC; ++v) acc[k][v] += red[(tt * VEC + v) * NS + k];
      }
#pragma unroll
      for (int k = 0; k < NS; ++k)
#pragma unroll
        for (int v = 0; v < VEC; ++v) {
          const int c = c0 + v;
          if (c < C) stat_out(partial, blockIdx.x, shards, NS * C, k * C + c, acc[k][v]);
        }
    }
    __syncthreads();
  }
}

// ---- backward finalize: stat[R][NS][C] -> dgamma/dbeta (+ second BN) and coef[3|6][C] ----
template <int NS>
__global__ __launch_bounds__(1024) void bn_bwd_finalize_kernel(
    const float* __restrict__ stat, int R, int C, float count, const float* __restrict__ aux,
    const float* __restrict__ gamma, const float* __restrict__ aux2,
    const float* __restrict__ gamma2, int training, float* __restrict__ dgamma,
    float* __restrict__ dbeta, float* __restrict__ dgamma2, float* __restrict__ dbeta2,
    float* __restrict__ coef, int accumulate, float* __restrict__ zero1, int zero1_n,
    float* __restrict__ zero2, int zero2_n, float* __restrict__ dbias) {
  __shared__ float red[16][64][3];
  // block 0 also clears the forward accumulators this BN consumed (sharded-sum mode)
  if (blockIdx.x == 0) {
    if (zero1)
      for (int i = threadIdx.x; i < zero1_n; i += blockDim.x) zero1[i] = 0.f;
    if (zero2)
      for (int i = threadIdx.x; i < zero2_n; i += blockDim.x) zero2[i] = 0.f;
  }
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  float acc[3] = {0.f, 0.f, 0.f};
  if (c < C) {
#pragma unroll 4
    for (int r = rl; r < R; r += 16)
#pragma unroll
      for (int k = 0; k < NS; ++k) acc[k] += stat[((size_t)r * NS + k) * C + c];
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) red[rl][cl][k] = acc[k];
  __syncthreads();
  if (rl != 0 || c >= C) return;
  double sd[3] = {0.0, 0.0, 0.0};
  for (int j = 0; j < 16; ++j)
    for (int k = 0; k < 3; ++k) sd[k] += red[j][cl][k];
  const float db = (float)sd[0];
  for (int b = 0; b < (NS == 3 ? 2 : 1); ++b) {
    const float* ax = b == 0 ? aux : aux2;
    const float* gm = b == 0 ? gamma : gamma2;
    const float dg = (float)sd[1 + b];
    const float mean = ax[c], istd = ax[C + c];
    const float g = gm ? gm[c] : 1.f;
    float A, Bc, D;
    if (training) {
      A = g * istd;
      Bc = -g * istd * istd * dg / count;
      D = -g * istd * db / count + g * istd * istd * mean * dg / count;
    } else {
      A = g * istd;
      Bc = 0.f;
      D = 0.f;
    }
    float* cf = coef + (size_t)b * 3 * C;
    cf[c] = A;
    cf[C + c] = Bc;
    cf[2 * C + c] = D;
    float* dgo = b == 0 ? dgamma : dgamma2;
    float* dbo = b == 0 ? dbeta : dbeta2;
    if (dgo) dgo[c] = accumulate ? dgo[c] + dg : dg;
    if (dbo) dbo[c] = accumulate ? dbo[c] + db : db;
    // bias of the conv feeding this BN (its only consumer): sum_m dY = A*sum dz + B*sum y + D*M
    if (dbias && b == 0) dbias[c] += A * db + Bc * (count * mean) + D * count;
  }
}

// ---- backward apply: dy = a*dz + b*y + d ; dres = dz ; dy2 = a2*dz + b2*y2 + d2 ----
template <int VEC>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(
    const bf16* __restrict__ dout, const bf16* __restrict__ out, const uint8_t* __restrict__ mask,
    const bf16* __restrict__ y, const float* __restrict__ aux, const float* __restrict__ coef,
    int act, int C, size_t total,
    bf16* __restrict__ dy, bf16* __restrict__ dres, const bf16* __restrict__ y2,
    bf16* __restrict__ dy2, int ldy, int ldx) {
  // ldy / ldx > C: y read from, and dy written into, the channel prefix of wider rows; dy's
  // padding channels are written as zeros (the gradient of a zero-padded conv's output, handed
  // to that conv without a pad pass)
  const size_t nvec = total / VEC;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < nvec; i += (size_t)gridDim.x * 256) {
    const size_t e = i * VEC;
    const int c0 = (int)(e % C);
    const size_t row = e / C;
    const size_t ey = ldy == C ? e : row * ldy + c0, ex = ldx == C ? e : row * ldx + c0;
    float dz[VEC], yy[VEC], o[VEC];
    compute_dz<VEC>(dout, out, mask, y, aux, C, c0, e, act, dz, e, ey);
    load_vec<VEC>(y + ey, yy);
#pragma unroll
    for (int v = 0; v < VEC; ++v) o[v] = coef[c0 + v] * dz[v] + coef[C + c0 + v] * yy[v] + coef[2 * C + c0 + v];
    store_vec<VEC>(dy + ex, o);
    if (ldx > C && c0 + VEC == C)
      for (int c = C; c < ldx; ++c) dy[row * ldx + c] = bf16(0.f);
    if (dres) store_vec<VEC>(dres + e, dz);
    if (dy2) {
      load_vec<VEC>(y2 + e, yy);
      const float* cf = coef + 3 * C;
#pragma unroll
      for (int v = 0; v < VEC; ++v) o[v] = cf[c0 + v] * dz[v] + cf[C + c0 + v] * yy[v] + cf[2 * C + c0 + v];
      store_vec<VEC>(dy2 + e, o);
    }
  }
}

// ---- row-tiled fast paths (C % 8 == 0, C <= 2048) ----
// Thread t owns the 8-channel group g = t % TPR for every row it visits, so the per-channel
// coefficients live in registers for the whole kernel (the generic grid-stride kernels re-load
// them per vector); consecutive threads still read consecutive 16-byte chunks of NHWC rows.
// Each iteration handles kRowsInFlight rows per thread: every load of the iteration is issued
// before any use, from clamped (always valid) row indices, and only the stores are predicated —
// a conditional load would make the compiler branch around it and drain vmcnt per row, which
// capped these kernels at ~2.5-2.9 TB/s (layer-1 shapes, bs1024).
// `scale`/`shift` (and `scale2`/`shift2`) point at [C] coefficient vectors in global memory
// (aux rows 2 and 3) or in LDS (the fused-finalize kernels below).
constexpr int kRowsInFlight = 4;

template <bool RES, bool DUAL, int ACT>
__device__ __forceinline__ void bn_apply_rows_body(
    const bf16* __restrict__ y, const float* scale, const float* shift, int C, int M,
    const bf16* __restrict__ res, const bf16* __restrict__ y2, const float* scale2,
    const float* shift2, bf16* __restrict__ out, uint8_t* __restrict__ mask, BnLd ld) {
  const int ldy = ld_or(ld.y, C), ldo = ld_or(ld.out, C);
  constexpr int U = kRowsInFlight;
  const int TPR = C >> 3, RPB = 256 / TPR;
  const int g = threadIdx.x % TPR, ro = threadIdx.x / TPR;
  if (ro >= RPB) return;
  const int c0 = g * 8;
  float sc[8], sh[8], sc2[8], sh2[8];
#pragma unroll
  for (int v = 0; v < 8; ++v) {
    sc[v] = scale[c0 + v];
    sh[v] = shift[c0 + v];
    if constexpr (DUAL) {
      sc2[v] = scale2[c0 + v];
      sh2[v] = shift2[c0 + v];
    }
  }
  const int rstep = gridDim.x * RPB;
  for (int r0 = blockIdx.x * RPB + ro; r0 < M; r0 += U * rstep) {
    uint4 vy[U], vt[U];
    size_t e[U];
    int rr[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int r = min(r0 + u * rstep, M - 1);
      rr[u] = r;
      e[u] = (size_t)r * C + c0;
      vy[u] = *reinterpret_cast<const uint4*>(y + (size_t)r * ldy + c0);
      if constexpr (RES) vt[u] = *reinterpret_cast<const uint4*>(res + e[u]);
      if constexpr (DUAL) vt[u] = *reinterpret_cast<const uint4*>(y2 + e[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float f[8], t[8];
      unpack8(vy[u], f);
      if constexpr (RES || DUAL) unpack8(vt[u], t);
      uint32_t b = 0;
#pragma unroll
      for (int v = 0; v < 8; ++v) {
        float a = f[v] * sc[v] + sh[v];
        if constexpr (RES) a += t[v];
        if constexpr (DUAL) a += t[v] * sc2[v] + sh2[v];
        a = apply_act(a, ACT);
        b |= (a > 0.f ? 1u : 0u) << v;
        f[v] = a;
      }
      if (r0 + u * rstep < M) {
        *reinterpret_cast<uint4*>(out + (size_t)rr[u] * ldo + c0) = pack8(f);
        if (mask) mask[e[u] >> 3] = (uint8_t)b;
      }
    }
  }
}

template <bool RES, bool DUAL, int ACT>
__global__ __launch_bounds__(256) void bn_apply_rows_kernel(
    const bf16* __restrict__ y, const float* __restrict__ aux, int C, int M,
    const bf16* __restrict__ res, const bf16* __restrict__ y2, const float* __restrict__ aux2,
    bf16* __restrict__ out, uint8_t* __restrict__ mask, BnLd ld) {
  bn_apply_rows_body<RES, DUAL, ACT>(y, aux + 2 * C, aux + 3 * C, C, M, res, y2,
                                     DUAL ? aux2 + 2 * C : nullptr, DUAL ? aux2 + 3 * C : nullptr,
                                     out, mask, ld);
}

// KIND: 0 = no activation, 1 = ReLU through the 1-bit mask, 2 = swish (z recomputed from y),
// 3 = ReLU with the sign recomputed from y (ACT_RELU_Y)
// `coef` = [3|6][C] affine coefficients in global memory or LDS (fused-finalize kernel below)
template <bool RES, bool DUAL, int KIND>
__device__ __forceinline__ void bn_bwd_apply_rows_body(
    const bf16* __restrict__ dout, const uint8_t* __restrict__ mask, const bf16* __restrict__ y,
    const float* coef, int C, int M, bf16* __restrict__ dy, bf16* __restrict__ dres,
    const bf16* __restrict__ y2, bf16* __restrict__ dy2, const float* __restrict__ aux, BnLd ld,
    int nblk) {
  constexpr bool MASK = KIND == 1;
  const int ldd = ld_or(ld.dout, C), ldy = ld_or(ld.y, C), ldx = ld_or(ld.dx, C);
  constexpr int U = kRowsInFlight;
  const int TPR = C >> 3, RPB = 256 / TPR;
  const int g = threadIdx.x % TPR, ro = threadIdx.x / TPR;
  if (ro >= RPB) return;
  const int c0 = g * 8;
  float ca[8], cb[8], cd[8], ca2[8], cb2[8], cd2[8], zs[8], zb[8];
#pragma unroll
  for (int v = 0; v < 8; ++v) {
    if constexpr (KIND == 2 || KIND == 3) {
      zs[v] = aux[2 * C + c0 + v];
      zb[v] = aux[3 * C + c0 + v];
    }
    ca[v] = coef[c0 + v];
    cb[v] = coef[C + c0 + v];
    cd[v] = coef[2 * C + c0 + v];
    if constexpr (DUAL) {
      ca2[v] = coef[3 * C + c0 + v];
      cb2[v] = coef[4 * C + c0 + v];
      cd2[v] = coef[5 * C + c0 + v];
    }
  }
  const int rstep = nblk * RPB;   // (nblk: the workgroups of this pass; gridDim.x unless the
                                  // launch also carries slab-reduce workgroups)
  for (int r0 = blockIdx.x * RPB + ro; r0 < M; r0 += U * rstep) {
    uint4 vd[U], vy[U], v2[U], vx[U];
    uint32_t vm[U];
    size_t e[U];
    int rr[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int r = min(r0 + u * rstep, M - 1);
      rr[u] = r;
      e[u] = (size_t)r * C + c0;
      vd[u] = *reinterpret_cast<const uint4*>(dout + (size_t)r * ldd + c0);
      vy[u] = *reinterpret_cast<const uint4*>(y + (size_t)r * ldy + c0);
      if (ld.dx_acc) vx[u] = *reinterpret_cast<const uint4*>(dy + (size_t)r * ldx + c0);
      if constexpr (MASK) vm[u] = mask[e[u] >> 3];
      if constexpr (DUAL) v2[u] = *reinterpret_cast<const uint4*>(y2 + e[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float dz[8], yy[8], o[8];
      unpack8(vd[u], dz);
      unpack8(vy[u], yy);
      if constexpr (MASK) {
#pragma unroll
        for (int v = 0; v < 8; ++v) dz[v] = ((vm[u] >> v) & 1u) ? dz[v] : 0.f;
      }
      if constexpr (KIND == 2 || KIND == 3) {
#pragma unroll
        for (int v = 0; v < 8; ++v)
          dz[v] *= act_grad(yy[v] * zs[v] + zb[v], KIND == 2 ? ACT_SWISH : ACT_RELU_Y);
      }
#pragma unroll
      for (int v = 0; v < 8; ++v) o[v] = ca[v] * dz[v] + cb[v] * yy[v] + cd[v];
      if (ld.dx_acc) {   // (concat slab: the other readers' gradients are already there)
        float xa[8];
        unpack8(vx[u], xa);
#pragma unroll
        for (int v = 0; v < 8; ++v) o[v] += xa[v];
      }
      const bool live = r0 + u * rstep < M;
      if (live) *reinterpret_cast<uint4*>(dy + (size_t)rr[u] * ldx + c0) = pack8(o);
      if constexpr (RES) {
        if (live) *reinterpret_cast<uint4*>(dres + e[u]) = pack8(dz);
      }
      if constexpr (DUAL) {
        unpack8(v2[u], yy);
#pragma unroll
        for (int v = 0; v < 8; ++v) o[v] = ca2[v] * dz[v] + cb2[v] * yy[v] + cd2[v];
        if (live) *reinterpret_cast<uint4*>(dy2 + e[u]) = pack8(o);
      }
    }
  }
}

template <bool RES, bool DUAL, int KIND>
__global__ __launch_bounds__(256) void bn_bwd_apply_rows_kernel(
    const bf16* __restrict__ dout, const uint8_t* __restrict__ mask, const bf16* __restrict__ y,
    const float* __restrict__ coef, int C, int M, bf16* __restrict__ dy, bf16* __restrict__ dres,
    const bf16* __restrict__ y2, bf16* __restrict__ dy2, const float* __restrict__ aux, BnLd ld) {
  bn_bwd_apply_rows_body<RES, DUAL, KIND>(dout, mask, y, coef, C, M, dy, dres, y2, dy2, aux, ld,
                                          gridDim.x);
}

// ---- fused finalize + apply (sharded accumulators, no finalize launch) ----
// The producer (conv epilogue / dgrad epilogue / reduce kernel) added its per-channel partial
// sums into acc[R][NS][C] (stat_out with shards = R). Every block of the consumer folds the R
// shard rows of all C channels into LDS coefficients (R*NS*C <= 4096 floats for C >= 64,
// L2-resident), block 0 also publishes aux / running stats / parameter gradients, then the body
// runs exactly as the unfused kernel. Re-zeroing: each BN's accumulators are zeroed by the OTHER
// pass of the same BN — the forward kernel's block 0 clears the backward accumulator (its
// producer, the dgrad epilogue, runs later in the step) and the backward kernel's block 0 clears
// the forward accumulator(s) (consumed earlier in the step, refilled next step). No ticket, no
// memset launch, stable addresses for hipGraph replay.
struct BnFin {
  float* acc;            // [R][NS][C] this kernel folds
  int R;
  float count;           // elements per channel (N*H*W)
  const float* gamma;
  const float* beta;
  float* rmean;          // running stats (forward, may be null)
  float* rvar;
  int64_t* nbt;
  float momentum, eps;
  float* aux;            // forward out: [4][C] mean, invstd, scale, shift (block 0)
  const float* aux_in;   // backward in: the forward's [mean | invstd] rows
  float* dgamma;         // backward out (block 0, accumulated; may be null)
  float* dbeta;
  float* zero;           // block 0 zeroes [zero, zero + zero_n) (the other pass's accumulator)
  int zero_n;
  const float* krow;     // forward: the shift K the producers subtracted (acc K row), or nullptr
  float* pilot;          // forward: block 0 writes the batch mean here (the next step's K)
  float* dbias;          // backward: += sum_m dY (bias gradient of the conv feeding this BN)
  int ldc;               // forward: row pitch of acc (0 = C; a channel suffix of a wider cache)
};

// The fold of the R shard rows is spread over the block: TPC lanes (consecutive threads, a
// power of two <= R) share a channel, each loads every TPC-th row (independent loads, unrolled),
// and the lanes combine with shuffles; 256 / TPC channels per pass.
__device__ __forceinline__ int fin_tpc(int C, int R) {
  int t = 1;
  while (t * 2 <= R && t * 2 * C <= 256) t *= 2;
  return t;
}

template <int NS_>
__device__ __forceinline__ void fin_fold(const float* acc, int R, int NS, int C, int c, int j,
                                         int tpc, bool ok, float* sum) {
#pragma unroll
  for (int k = 0; k < NS_; ++k) sum[k] = 0.f;
  if (ok) {
#pragma unroll 8
    for (int r = j; r < R; r += tpc)
#pragma unroll
      for (int k = 0; k < NS_; ++k) sum[k] += acc[((size_t)r * NS + k) * C + c];
  }
  for (int o = 1; o < tpc; o <<= 1)
#pragma unroll
    for (int k = 0; k < NS_; ++k) sum[k] += __shfl_xor(sum[k], o, 64);
}

__device__ __forceinline__ void bn_fin_forward(const BnFin& f, int C, float* sc, float* sh) {
  const int tpc = fin_tpc(C, f.R), cpp = blockDim.x / tpc;
  const int j = threadIdx.x % tpc;
  for (int cb = 0; cb < C; cb += cpp) {
    const int c = cb + threadIdx.x / tpc;
    float sum[2];
    fin_fold<2>(f.acc, f.R, 2, f.ldc ? f.ldc : C, c, j, tpc, c < C, sum);
    if (j != 0 || c >= C) continue;
    const double m = (double)sum[0] / f.count;     // mean of x - K (shifted sums)
    double v = (double)sum[1] / f.count - m * m;
    if (v < 0.0) v = 0.0;
    const float mean = (float)(m + (f.krow ? (double)f.krow[c] : 0.0));
    const float istd = rsqrtf((float)v + f.eps);
    const float gm = f.gamma ? f.gamma[c] : 1.f;
    const float bt = f.beta ? f.beta[c] : 0.f;
    sc[c] = gm * istd;
    sh[c] = bt - mean * gm * istd;
    if (blockIdx.x == 0) {
      f.aux[c] = mean;
      f.aux[C + c] = istd;
      f.aux[2 * C + c] = gm * istd;
      f.aux[3 * C + c] = bt - mean * gm * istd;
      if (f.pilot) f.pilot[c] = mean;   // (the other blocks read K from the K row, not here)
      if (f.rmean) {
        const double unb = f.count > 1.f ? v * f.count / (f.count - 1.0) : v;
        f.rmean[c] = (1.f - f.momentum) * f.rmean[c] + f.momentum * mean;
        f.rvar[c] = (1.f - f.momentum) * f.rvar[c] + f.momentum * (float)unb;
      }
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0 && f.nbt) f.nbt[0] += 1;
}

// training-mode BN backward coefficients: dy = A*dz + B*y + D (per channel); sums = {dz, dz*xhat
// [, dz*xhat2]}; BN k (0 or 1) uses sums 0 and 1 + k
template <int NS>
__device__ __forceinline__ void bn_fin_backward(const BnFin& f, const BnFin& f2, int C,
                                                float* cf) {
  const int tpc = fin_tpc(C, f.R), cpp = blockDim.x / tpc;
  const int j = threadIdx.x % tpc;
  for (int cb = 0; cb < C; cb += cpp) {
    const int c = cb + threadIdx.x / tpc;
    float sum[NS];
    fin_fold<NS>(f.acc, f.R, NS, C, c, j, tpc, c < C, sum);
    if (j != 0 || c >= C) continue;
#pragma unroll
    for (int k = 0; k < NS - 1; ++k) {
      const BnFin& b = k == 0 ? f : f2;
      const float mean = b.aux_in[c], istd = b.aux_in[C + c];
      const float gm = b.gamma ? b.gamma[c] : 1.f;
      const float dg = sum[1 + k], db = sum[0];
      float* o = cf + (size_t)k * 3 * C;
      o[c] = gm * istd;
      o[C + c] = -gm * istd * istd * dg / f.count;
      o[2 * C + c] = -gm * istd * db / f.count + gm * istd * istd * mean * dg / f.count;
      if (blockIdx.x == 0) {
        if (b.dgamma) b.dgamma[c] += dg;
        if (b.dbeta) b.dbeta[c] += db;
        if (k == 0 && f.dbias)
          f.dbias[c] += o[c] * db + o[C + c] * (f.count * mean) + o[2 * C + c] * f.count;
      }
    }
  }
}

__device__ __forceinline__ void bn_fin_zero(const BnFin& f) {
  if (blockIdx.x == 0 && f.zero)
    for (int i = threadIdx.x; i < f.zero_n; i += blockDim.x) f.zero[i] = 0.f;
}

template <bool RES, bool DUAL, int ACT>
__global__ __launch_bounds__(256) void bn_apply_acc_rows_kernel(
    const bf16* __restrict__ y, BnFin f, BnFin f2, int C, int M, const bf16* __restrict__ res,
    const bf16* __restrict__ y2, bf16* __restrict__ out, uint8_t* __restrict__ mask, BnLd ld) {
  extern __shared__ float lds[];   // [sc | sh | sc2 | sh2][C]
  bn_fin_forward(f, C, lds, lds + C);
  if constexpr (DUAL) bn_fin_forward(f2, C, lds + 2 * C, lds + 3 * C);
  bn_fin_zero(f);
  __syncthreads();
  bn_apply_rows_body<RES, DUAL, ACT>(y, lds, lds + C, C, M, res, y2, lds + 2 * C, lds + 3 * C,
                                     out, mask, ld);
}

template <bool RES, bool DUAL, int KIND>
__global__ __launch_bounds__(256) void bn_bwd_apply_acc_rows_kernel(
    const bf16* __restrict__ dout, const uint8_t* __restrict__ mask, const bf16* __restrict__ y,
    BnFin f, BnFin f2, int C, int M, bf16* __restrict__ dy, bf16* __restrict__ dres,
    const bf16* __restrict__ y2, bf16* __restrict__ dy2, const float* __restrict__ aux, BnLd ld) {
  extern __shared__ float lds[];   // coef [3|6][C]
  constexpr int NS = DUAL ? 3 : 2;
  bn_fin_backward<NS>(f, f2, C, lds);
  bn_fin_zero(f);
  bn_fin_zero(f2);
  __syncthreads();
  bn_bwd_apply_rows_body<RES, DUAL, KIND>(dout, mask, y, lds, C, M, dy, dres, y2, dy2, aux, ld,
                                          gridDim.x);
}

// The same with the pending weight-gradient slab reductions of the preceding wgrads riding along
// as extra workgroups [napply, gridDim.x) (conv_halo.hip wgrad_take_pending): on the small
// per-rank shard each reduce was a ~10 us latency-bound launch of its own between the wgrad and
// this kernel; here it runs beside the BatchNorm pass it is independent of (the slab was just
// written: L2 / MALL resident, unlike the end-of-pass batch of PCA_WGRAD_DEFER=1).
template <bool RES, bool DUAL, int KIND>
__global__ __launch_bounds__(256) void bn_bwd_apply_acc_rows_red_kernel(
    const bf16* __restrict__ dout, const uint8_t* __restrict__ mask, const bf16* __restrict__ y,
    BnFin f, BnFin f2, int C, int M, bf16* __restrict__ dy, bf16* __restrict__ dres,
    const bf16* __restrict__ y2, bf16* __restrict__ dy2, const float* __restrict__ aux, BnLd ld,
    int napply, SlabRedBatch rb) {
  if ((int)blockIdx.x >= napply) {   // (block-uniform: a reduce workgroup)
    __shared__ float4 red[4][64];
    slab_reduce_multi_body<4>(rb, (int)blockIdx.x - napply, red);
    return;
  }
  extern __shared__ float lds[];   // coef [3|6][C]
  constexpr int NS = DUAL ? 3 : 2;
  bn_fin_backward<NS>(f, f2, C, lds);
  bn_fin_zero(f);
  bn_fin_zero(f2);
  __syncthreads();
  bn_bwd_apply_rows_body<RES, DUAL, KIND>(dout, mask, y, lds, C, M, dy, dres, y2, dy2, aux, ld,
                                          napply);
}

int wgrad_take_pending(SlabRedBatch* b);
static bool g_wgrad_piggy = false;
void set_wgrad_piggy(bool on) { g_wgrad_piggy = on; }

static bool rows_enabled() {
  static const bool on = [] {
    const char* e = getenv("PCA_BN_ROWS");
    return !(e && e[0] == '0');
  }();
  return on;
}

static int rows_grid(int M, int C) {
  // every block first folds the R x 2 x C accumulator rows (16 KiB): the cap bounds that prologue
  // traffic and latency against the streaming passes' need for resident waves (PCA_BN_ROWS_CAP)
  static const int cap = [] {
    const char* e = getenv("PCA_BN_ROWS_CAP");
    const int v = e ? atoi(e) : 0;
    return v > 0 ? v : 512;   // measured: 512 -0.6 % vs 2048 at bs1024, equal at bs128
  }();
  const int RPB = 256 / (C >> 3);
  int b = cdiv(M, RPB * kRowsInFlight);
  return b < cap ? (b ? b : 1) : cap;
}

// =========================================== host ========================================

static int grid_for(size_t nvec) {
  size_t b = (nvec + 255) / 256;
  return (int)(b < 4096 ? (b ? b : 1) : 4096);
}

static int bn_vec(int C) { return C % 8 == 0 ? 8 : C % 4 == 0 ? 4 : C % 2 == 0 ? 2 : 1; }

// Widest C the row-tiled kernels take (0 when PCA_BN_ROWS=0). Row-strided BN operands (concat
// slab slices and suffixes, zero-padded conv prefixes) need these kernels: callers that would hand
// such operands to a wider BN keep dense tensors instead (ops/functional.py ChannelSlab/DenseSlab).
int bn_rows_max_c() { return rows_enabled() ? 2048 : 0; }

int bn_row_blocks(int M, int C) {
  const int vec = bn_vec(C);
  RowPar rp = make_rowpar(C, vec);
  int P = cdiv(M, rp.RPP * 8);
  if (P > 1024) P = 1024;
  if (P < 1) P = 1;
  return P;
}

void bn_stats_launch(const bf16* x, int M, int C, float* partial, int P, hipStream_t st,
                     float* krow) {
  const int rows = cdiv(M, P);
  switch (bn_vec(C)) {
#define PCA_STATS(V)                                                                              \
  case V: {                                                                                       \
    RowPar rp = make_rowpar(C, V);                                                                \
    hipLaunchKernelGGL(bn_stats_kernel<V>, dim3(P), dim3(256), 0, st, x, M, rp, rows, partial, g_stat_shards, krow, ld_or(g_bn_ld.y, C), C, (bf16*)nullptr, 0); \
    break;                                                                                        \
  }
    PCA_STATS(8) PCA_STATS(4) PCA_STATS(2) PCA_STATS(1)
#undef PCA_STATS
  }
}

// Copy + statistics in one pass (DenseNet's concat slab, ops/functional.py DenseSlab): dst rows
// (row stride ldd) <- x rows (ldx), and the channels' centred sums (K = row 0) added into R shard
// rows of a wider [R][2][ldc] accumulator (acc points at this tensor's first channel) whose K row
// starts at krow. The slab caches every channel's batch sums as it is produced, so each dense
// layer's BatchNorm folds its suffix of the cache instead of re-reducing the whole suffix.
void bn_stats_copy_launch(const bf16* x, int ldx, int M, int C, bf16* dst, int ldd, float* acc,
                          int ldc, int R, int P, float* krow, hipStream_t st) {
  const int rows = cdiv(M, P);
  switch (bn_vec(C)) {
#define PCA_STATS(V)                                                                              \
  case V: {                                                                                       \
    RowPar rp = make_rowpar(C, V);                                                                \
    hipLaunchKernelGGL(bn_stats_kernel<V>, dim3(P), dim3(256), 0, st, x, M, rp, rows, acc, R, krow, ldx, ldc, dst, ldd); \
    break;                                                                                        \
  }
    PCA_STATS(8) PCA_STATS(4) PCA_STATS(2) PCA_STATS(1)
#undef PCA_STATS
  }
}

// Fold R rows of width L down to <= 64 rows (stage 1); returns rows in the output buffer.
int colsum_launch(const float* in, int R, int L, float* out, hipStream_t st) {
  if (R <= 64) return 0;
  const int R2 = 64;
  const int chunk = cdiv(R, R2);
  const int r2 = cdiv(R, chunk);
  hipLaunchKernelGGL(colsum_kernel, dim3(cdiv(L, 256), r2), dim3(256), 0, st, in, R, L, chunk, out);
  return r2;
}

void bn_finalize_launch(const float* stat, int R, int C, double count, const float* gamma,
                        const float* beta, float* rmean, float* rvar, int64_t* nbt,
                        float momentum, float eps, int training, int update_running, float* aux,
                        hipStream_t st, const float* kin, float* pilot_out, float* zero,
                        int zero_n, int ld) {
  hipLaunchKernelGGL(bn_finalize_kernel, dim3(cdiv(C, 64)), dim3(1024), 0, st, stat, R, C, count,
                     gamma, beta, rmean, rvar, nbt, momentum, eps, training, update_running, aux,
                     kin, pilot_out, zero, zero_n, ld > 0 ? ld : C);
}

void bn_apply_launch(const bf16* y, const float* aux, int C, size_t total, const bf16* res,
                     const bf16* y2, const float* aux2, int act, bf16* out, uint8_t* mask,
                     hipStream_t st) {
  if (rows_enabled() && C % 8 == 0 && C <= 2048 &&
      (act == ACT_RELU || act == ACT_NONE || (act == ACT_SWISH && !res && !y2)) && !(res && y2)) {
    const int M = (int)(total / C);
    const dim3 gr(rows_grid(M, C)), bl(256);
#define PCA_APPLY(R, D, A) \
    hipLaunchKernelGGL((bn_apply_rows_kernel<R, D, A>), gr, bl, 0, st, y, aux, C, M, res, y2, aux2, out, mask, g_bn_ld)
    if (act == ACT_SWISH) {
      PCA_APPLY(false, false, ACT_SWISH);
    } else if (act == ACT_RELU) {
      if (res) PCA_APPLY(true, false, ACT_RELU);
      else if (y2) PCA_APPLY(false, true, ACT_RELU);
      else PCA_APPLY(false, false, ACT_RELU);
    } else {
      if (res) PCA_APPLY(true, false, ACT_NONE);
      else if (y2) PCA_APPLY(false, true, ACT_NONE);
      else PCA_APPLY(false, false, ACT_NONE);
    }
#undef PCA_APPLY
    return;
  }
  // (the vector kernels take a row-strided input y only: a zero-padded conv's output prefix)
  if (g_bn_ld.out || g_bn_ld.dout || g_bn_ld.dx || g_bn_ld.dx_acc || (g_bn_ld.y && (res || y2))) {
    fprintf(stderr, "pca: strided BatchNorm apply needs the row-tiled kernel (C %% 8 == 0)\n");
    abort();
  }
  const int ldy = ld_or(g_bn_ld.y, C);
  switch (bn_vec(C)) {
    case 8:
      hipLaunchKernelGGL(bn_apply_kernel<8>, dim3(grid_for(total / 8)), dim3(256), 0, st, y, aux, C,
                         total, res, y2, aux2, act, out, mask, ldy);
      break;
#define PCA_APPLY_V(V)                                                                             \
  case V:                                                                                          \
    hipLaunchKernelGGL(bn_apply_kernel<V>, dim3(grid_for(total / V)), dim3(256), 0, st, y, aux, C, \
                       total, res, y2, aux2, act, out, (uint8_t*)nullptr, ldy);                    \
    break;
    PCA_APPLY_V(4) PCA_APPLY_V(2) PCA_APPLY_V(1)
#undef PCA_APPLY_V
  }
}

void bn_bwd_reduce_launch(const bf16* dout, const bf16* out, const uint8_t* mask, const bf16* y,
                          const float* aux,
                          const bf16* y2, const float* aux2, int act, int M, int C,
                          float* partial, int P, hipStream_t st) {
  const int rows = cdiv(M, P);
  switch (bn_vec(C)) {
#define PCA_RED(V)                                                                                 \
  case V: {                                                                                        \
    RowPar rp = make_rowpar(C, V);                                                                 \
    if (y2)                                                                                        \
      hipLaunchKernelGGL((bn_bwd_reduce_kernel<V, 3>), dim3(P), dim3(256), 0, st, dout, out, mask, \
                         y, aux, y2, aux2, act, M, rp, rows, partial, g_stat_shards,               \
                         ld_or(g_bn_ld.dout, C), ld_or(g_bn_ld.y, C));                             \
    else                                                                                           \
      hipLaunchKernelGGL((bn_bwd_reduce_kernel<V, 2>), dim3(P), dim3(256), 0, st, dout, out, mask, \
                         y, aux, y2, aux2, act, M, rp, rows, partial, g_stat_shards,               \
                         ld_or(g_bn_ld.dout, C), ld_or(g_bn_ld.y, C));                             \
    break;                                                                                         \
  }
    PCA_RED(8) PCA_RED(4) PCA_RED(2) PCA_RED(1)
#undef PCA_RED
  }
}

// Bias gradient of the conv whose output this BN alone consumes (googlenet.py / vgg.py
// Conv2d(bias=True) -> BatchNorm2d): added by the next BN-backward launches' finalize from the
// per-channel sums they already hold — sum_m dY = A * sum dz + B * sum y + D * M with
// sum y = M * mean — instead of a column-sum pass over dY (exactly 0 in exact arithmetic for a
// training-mode BN; bindings scope it per call).
static float* g_bn_dbias = nullptr;
void set_bn_dbias(float* p) { g_bn_dbias = p; }

void bn_bwd_finalize_launch(const float* stat, int R, int NS, int C, float count,
                            const float* aux, const float* gamma, const float* aux2,
                            const float* gamma2, int training, float* dgamma, float* dbeta,
                            float* dgamma2, float* dbeta2, float* coef, int accumulate,
                            hipStream_t st, float* zero1, int zero1_n, float* zero2,
                            int zero2_n) {
  if (NS == 3)
    hipLaunchKernelGGL(bn_bwd_finalize_kernel<3>, dim3(cdiv(C, 64)), dim3(1024), 0, st, stat, R, C,
                       count, aux, gamma, aux2, gamma2, training, dgamma, dbeta, dgamma2, dbeta2,
                       coef, accumulate, zero1, zero1_n, zero2, zero2_n, g_bn_dbias);
  else
    hipLaunchKernelGGL(bn_bwd_finalize_kernel<2>, dim3(cdiv(C, 64)), dim3(1024), 0, st, stat, R, C,
                       count, aux, gamma, aux2, gamma2, training, dgamma, dbeta, dgamma2, dbeta2,
                       coef, accumulate, zero1, zero1_n, zero2, zero2_n, g_bn_dbias);
}

void bn_bwd_apply_launch(const bf16* dout, const bf16* out, const uint8_t* mask, const bf16* y,
                         const float* aux, const float* coef, int act, int C, size_t total,
                         bf16* dy, bf16* dres, const bf16* y2, bf16* dy2, hipStream_t st) {
  const bool masked = act == ACT_RELU && mask != nullptr;
  const bool swish = act == ACT_SWISH && !dres && !y2;
  const bool relu_y = act == ACT_RELU_Y && !dres && !y2;
  if (rows_enabled() && C % 8 == 0 && C <= 2048 && (masked || act == ACT_NONE || swish || relu_y)) {
    const int M = (int)(total / C);
    const dim3 gr(rows_grid(M, C)), bl(256);
#define PCA_BWD(R, D, K) \
    hipLaunchKernelGGL((bn_bwd_apply_rows_kernel<R, D, K>), gr, bl, 0, st, dout, mask, y, coef, C, M, dy, dres, y2, dy2, aux, g_bn_ld)
    if (masked) {
      if (dres && y2) PCA_BWD(true, true, 1);
      else if (dres) PCA_BWD(true, false, 1);
      else if (y2) PCA_BWD(false, true, 1);
      else PCA_BWD(false, false, 1);
    } else if (swish) {
      PCA_BWD(false, false, 2);
    } else if (relu_y) {
      PCA_BWD(false, false, 3);
    } else {
      if (dres && y2) PCA_BWD(true, true, 0);
      else if (dres) PCA_BWD(true, false, 0);
      else if (y2) PCA_BWD(false, true, 0);
      else PCA_BWD(false, false, 0);
    }
#undef PCA_BWD
    return;
  }
  // (the vector kernels take a row-strided y and dy only — a zero-padded conv's output prefix
  // and its gradient, whose padding they zero)
  if (g_bn_ld.out || g_bn_ld.dout || g_bn_ld.dx_acc ||
      ((g_bn_ld.y || g_bn_ld.dx) && (dres || y2 || dy2))) {
    fprintf(stderr, "pca: strided BatchNorm backward needs the row-tiled kernel (C %% 8 == 0)\n");
    abort();
  }
  const int ldy = ld_or(g_bn_ld.y, C), ldx = ld_or(g_bn_ld.dx, C);
  switch (bn_vec(C)) {
    case 8:
      hipLaunchKernelGGL(bn_bwd_apply_kernel<8>, dim3(grid_for(total / 8)), dim3(256), 0, st, dout,
                         out, mask, y, aux, coef, act, C, total, dy, dres, y2, dy2, ldy, ldx);
      break;
#define PCA_BWD_V(V)                                                                              \
  case V:                                                                                         \
    hipLaunchKernelGGL(bn_bwd_apply_kernel<V>, dim3(grid_for(total / V)), dim3(256), 0, st, dout, \
                       out, (const uint8_t*)nullptr, y, aux, coef, act, C, total, dy, dres, y2,   \
                       dy2, ldy, ldx);                                                            \
    break;
    PCA_BWD_V(4) PCA_BWD_V(2) PCA_BWD_V(1)
#undef PCA_BWD_V
  }
}

// ---- fused finalize + apply launchers (sharded accumulators); false = not eligible ----
static int acc_rows_grid(int M, int C) { return rows_grid(M, C); }

bool bn_apply_acc_launch(const bf16* y, int C, int M, float count, float* acc, int R,
                         const float* gamma, const float* beta, float* rmean, float* rvar,
                         int64_t* nbt, float momentum, float eps, float* aux, float* acc2, int R2,
                         const float* gamma2, const float* beta2, float* rmean2, float* rvar2,
                         int64_t* nbt2, float momentum2, float eps2, float* aux2, const bf16* res,
                         const bf16* y2, int act, bf16* out, uint8_t* mask, float* zero,
                         int zero_n, hipStream_t st, bool shifted, float* pilot, bool shifted2,
                         float* pilot2, int acc_off, int acc_ld) {
  if (!(rows_enabled() && C % 8 == 0 && C <= 2048 &&
        (act == ACT_RELU || act == ACT_NONE || (act == ACT_SWISH && !res && !y2)) && !(res && y2)))
    return false;
  // K rows of shifted accumulators follow their [R][2][C] sums
  BnFin f{acc, R, count, gamma, beta, rmean, rvar, nbt, momentum, eps, aux, nullptr, nullptr, nullptr,
          zero, zero_n, shifted ? acc + (size_t)R * 2 * C : nullptr, pilot};
  if (acc_ld > 0) {   // channels [acc_off, acc_off + C) of a [R][2][acc_ld] accumulator + K row
    f.acc = acc + acc_off;
    f.ldc = acc_ld;
    f.krow = shifted ? acc + (size_t)R * 2 * acc_ld + acc_off : nullptr;
  }
  BnFin f2{acc2, R2, count, gamma2, beta2, rmean2, rvar2, nbt2, momentum2, eps2, aux2, nullptr,
           nullptr, nullptr, nullptr, 0, (shifted2 && acc2) ? acc2 + (size_t)R2 * 2 * C : nullptr,
           pilot2};
  const dim3 gr(acc_rows_grid(M, C)), bl(256);
  const size_t lds = (size_t)(y2 ? 4 : 2) * C * sizeof(float);
#define PCA_APPLY(R_, D, A) \
  hipLaunchKernelGGL((bn_apply_acc_rows_kernel<R_, D, A>), gr, bl, lds, st, y, f, f2, C, M, res, y2, out, mask, g_bn_ld)
  if (act == ACT_SWISH) {
    PCA_APPLY(false, false, ACT_SWISH);
  } else if (act == ACT_RELU) {
    if (res) PCA_APPLY(true, false, ACT_RELU);
    else if (y2) PCA_APPLY(false, true, ACT_RELU);
    else PCA_APPLY(false, false, ACT_RELU);
  } else {
    if (res) PCA_APPLY(true, false, ACT_NONE);
    else if (y2) PCA_APPLY(false, true, ACT_NONE);
    else PCA_APPLY(false, false, ACT_NONE);
  }
#undef PCA_APPLY
  return true;
}

bool bn_bwd_apply_acc_launch(const bf16* dout, const uint8_t* mask, const bf16* y, int C, int M,
                             float count, float* acc, int R, const float* aux, const float* gamma,
                             float* dgamma, float* dbeta, const float* aux2, const float* gamma2,
                             float* dgamma2, float* dbeta2, int act, bf16* dy, bf16* dres,
                             const bf16* y2, bf16* dy2, float* zero, int zero_n, float* zero2,
                             int zero2_n, hipStream_t st) {
  const bool masked = act == ACT_RELU && mask != nullptr;
  const bool swish = act == ACT_SWISH && !dres && !y2;
  if (!(rows_enabled() && C % 8 == 0 && C <= 2048 && (masked || act == ACT_NONE || swish)))
    return false;
  BnFin f{acc, R, count, gamma, nullptr, nullptr, nullptr, nullptr, 0.f, 0.f, nullptr, aux, dgamma,
          dbeta, zero, zero_n};
  f.dbias = g_bn_dbias;
  BnFin f2{acc, R, count, gamma2, nullptr, nullptr, nullptr, nullptr, 0.f, 0.f, nullptr, aux2,
           dgamma2, dbeta2, zero2, zero2_n};
  const dim3 gr(acc_rows_grid(M, C)), bl(256);
  const size_t lds = (size_t)(y2 ? 6 : 3) * C * sizeof(float);
  SlabRedBatch rb{};
  const int nred = g_wgrad_piggy ? wgrad_take_pending(&rb) : 0;
#define PCA_BWD(R_, D, K)                                                                             \
  do {                                                                                                \
    if (nred)                                                                                         \
      hipLaunchKernelGGL((bn_bwd_apply_acc_rows_red_kernel<R_, D, K>), dim3(gr.x + nred), bl, lds,   \
                         st, dout, mask, y, f, f2, C, M, dy, dres, y2, dy2, aux, g_bn_ld,            \
                         (int)gr.x, rb);                                                              \
    else                                                                                              \
      hipLaunchKernelGGL((bn_bwd_apply_acc_rows_kernel<R_, D, K>), gr, bl, lds, st, dout, mask, y,   \
                         f, f2, C, M, dy, dres, y2, dy2, aux, g_bn_ld);                               \
  } while (0)
  if (masked) {
    if (dres && y2) PCA_BWD(true, true, 1);
    else if (dres) PCA_BWD(true, false, 1);
    else if (y2) PCA_BWD(false, true, 1);
    else PCA_BWD(false, false, 1);
  } else if (swish) {
    PCA_BWD(false, false, 2);
  } else {
    if (dres && y2) PCA_BWD(true, true, 0);
    else if (dres) PCA_BWD(true, false, 0);
    else if (y2) PCA_BWD(false, true, 0);
    else PCA_BWD(false, false, 0);
  }
#undef PCA_BWD
  return true;
}

}  // namespace pca
