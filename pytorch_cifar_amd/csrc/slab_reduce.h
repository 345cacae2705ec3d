// Batched split-K weight-gradient slab reductions (conv_halo.hip: deferred reduces; batchnorm.hip:
// reduces riding along in the next BatchNorm-backward launch).
#pragma once

#include "common.h"

namespace pca {

// Geometry of the accumulator-order slab rows written by wgrad_halo_kernel (per tile:
// [wave][mi][ni][lane] float4 = rows m..m+3 of one column).
struct HaloSlabMap {
  int TM, TN, WN, WTM, WTN, BM, BN;
  int tiles_x, tiles_y;   // grid.x (output-channel tiles), grid.y (input blocks x tap rows)
  int cout_g, cin_g, Ktot;
  int TG;                 // taps per tile (9, or 3 = one kernel row)
};

// ---- deferred slab reductions: every pending wgrad slab of a backward pass in ONE launch ----
// A weight gradient written as split-K slab rows needs a reduce launch; on the bs128 shard those
// are ~10 us latency-bound launches each (ResNet-18: 12 per step, 117 us). With deferral on, the
// wgrad launch records its reduction here instead, and the owner of the gradient (the end of the
// backward pass, or a DDP bucket about to be all-reduced) flushes every pending one at once.
// Each descriptor keeps its own L (split lanes per column) and fixed summation order, so the
// result is bitwise the one of the per-conv reduce kernels.
struct SlabRedDesc {
  const float4* slab;
  float* dw;
  int64_t n4;
  int splits, L;           // slab rows; split lanes per column (power of two <= 16)
  int halo;                // 1: accumulator-order rows mapped back through mp
  int block0;              // first block of this descriptor in the batched grid
  HaloSlabMap mp;
};
constexpr int kSlabRedMax = 20;   // descriptors per launch (kernel-argument bytes: ~2 KiB)
struct SlabRedBatch {
  SlabRedDesc d[kSlabRedMax];
  int n;
};

// One workgroup of a batched slab reduction: block `blk` of the batch's grid, LMAX = blockDim / 64
// split lanes at most (a descriptor's L is capped to it: the 256-thread form inside the BatchNorm
// backward kernel sums in another fixed order than the 1024-thread launches, still deterministic)
template <int LMAX>
__device__ __forceinline__ void slab_reduce_multi_body(const SlabRedBatch& b, int blk,
                                                       float4 (*red)[64]) {
  int k = 0;
  while (k + 1 < b.n && blk >= b.d[k + 1].block0) ++k;
  const SlabRedDesc& d = b.d[k];
  const int c = threadIdx.x & 63, l = threadIdx.x >> 6, L = d.L < LMAX ? d.L : LMAX;
  const int64_t q = (int64_t)(blk - d.block0) * 64 + c;
  const int64_t n4 = d.n4;
  const int splits = d.splits;
  const float4* __restrict__ slab = d.slab;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  if (q < n4 && l < L) {
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
  if (!d.halo) {   // (slab_reduce_kernel's order: dw first, then the lane partials)
    float4* dw4 = reinterpret_cast<float4*>(d.dw);
    float4 o = dw4[q];
    for (int j = 0; j < L; ++j) {
      const float4 v = red[j][c];
      o.x += v.x; o.y += v.y; o.z += v.z; o.w += v.w;
    }
    dw4[q] = o;
    return;
  }
  for (int j = 1; j < L; ++j) {
    const float4 v = red[j][c];
    a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
  }
  const HaloSlabMap& mp = d.mp;
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
    if (mb + j < mp.cout_g) d.dw[((size_t)grp * mp.cout_g + mb + j) * mp.Ktot + col] += v[j];
}


}  // namespace pca
