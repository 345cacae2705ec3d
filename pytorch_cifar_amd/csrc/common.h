// Shared device helpers for the gfx950 (CDNA4 / MI355X) kernels of pytorch_cifar_amd.
//
// Conventions used by every kernel in csrc/:
//   * activations are NHWC bf16 ("channels-last"), one contiguous [N*H*W][C] matrix;
//   * parameters are fp32 masters whose *physical* layout is [Cout][KH][KW][Cin/G]
//     (torch.channels_last strides on the reference [Cout,Cin,KH,KW] shape), so a conv
//     weight is already the K-contiguous GEMM operand the MFMA B-fragment wants;
//   * all reductions accumulate in fp32; per-block partials are written to slabs and folded by
//     a finalize kernel (deterministic mode), or added into small sharded accumulators that the
//     consumer folds in its prologue (default; see stat_out below).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pca {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kWave = 64;  // CDNA wavefront width

__device__ __forceinline__ float bf2f(bf16 v) { return static_cast<float>(v); }
__device__ __forceinline__ bf16 f2bf(float v) { return static_cast<bf16>(v); }

// 16-byte vector of 8 bf16 as raw bits (for loads/stores/LDS traffic).
struct alignas(16) U128 {
  uint32_t x, y, z, w;
};

__device__ __forceinline__ void unpack8(const uint4& u, float* f) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}

// one v_cvt_pk_bf16_f32 (round to nearest even, NaN kept) per pair: converting the two floats
// separately and or-ing the halves let the SLP vectorizer pair elements across calls and emit
// and / shift / or_sdwa fix-ups (6 VALU per 4 values in the conv epilogues instead of 2)
__device__ __forceinline__ uint32_t pack2(float a, float b) {
  typedef float f32x2_t __attribute__((ext_vector_type(2)));
  typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
  const bf16x2_t h = __builtin_convertvector((f32x2_t){a, b}, bf16x2_t);
  return __builtin_bit_cast(uint32_t, h);
}

__device__ __forceinline__ uint4 pack8(const float* f) {
  uint4 u;
  u.x = pack2(f[0], f[1]);
  u.y = pack2(f[2], f[3]);
  u.z = pack2(f[4], f[5]);
  u.w = pack2(f[6], f[7]);
  return u;
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <typename T>
__device__ __forceinline__ T wave_max(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

__host__ __device__ __forceinline__ int cdiv(int a, int b) { return (a + b - 1) / b; }
__host__ __device__ __forceinline__ int64_t cdiv64(int64_t a, int64_t b) { return (a + b - 1) / b; }

// XCD-aware remap of a linear workgroup id (cdna_hip_programming.md §5, "XCD swizzle must be
// bijective"): blocks b and b+8 share an XCD, so give each XCD a contiguous chunk of tiles.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int q = nwg / 8, r = nwg % 8, x = orig % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + orig / 8;
}

// BatchNorm partial sums leave a producer kernel in one of two forms:
//   shards == 0: slab row `row` of [rows][rowlen] (deterministic; folded by a finalize kernel),
//   shards  > 0: an fp32 atomic add into accumulator row `row % shards` of [shards][rowlen].
// The consuming BN kernel folds the sharded accumulator while normalizing (no finalize launch);
// the other pass of the same BN re-zeroes it (batchnorm.hip, "fused finalize + apply").
__device__ __forceinline__ void stat_out(float* base, int row, int shards, size_t rowlen, int col,
                                         float v) {
  if (shards > 0)
    atomicAdd(base + (size_t)(row % shards) * rowlen + col, v);
  else
    base[(size_t)row * rowlen + col] = v;
}

// Row strides of the BatchNorm kernels' tensors (batchnorm.hip set_bn_ld; 0 = dense [M][C]):
// y input, out forward output, dout / dx backward input / output (dx_acc: add into dx)
// f where bit `bit` of the ReLU mask m is set, else +0: the bit is sign-extended into an
// all-ones / zero word and ANDed with f's bits (v_bfe_i32 + v_and: one op fewer than a compare +
// select per element in the fused BN-backward reduces)
__device__ __forceinline__ float relu_bit(float f, uint32_t m, int bit) {
  const int keep = ((int)(m << (31 - bit))) >> 31;
  return __int_as_float(__float_as_int(f) & keep);
}

struct BnLd {
  int y, out, dout, dx, dx_acc;
};
BnLd bn_ld();
void set_bn_ld(const BnLd& ld);

// Process-wide shard count the next producer launch writes with (0 = slab rows); set by the
// host bindings around a launch (batchnorm.hip).
int stat_shards();
void set_stat_shards(int shards);

// Shifted BatchNorm forward sums (robust variance). A producer of forward statistics sums
// d = v - K[c] and d*d, where K is the consuming BN's pilot mean (its previous batch mean): the
// fold's E[d^2] - E[d]^2 then has no catastrophic cancellation once K is near the batch mean
// (fp32 E[x^2] - E[x]^2 loses (mean/std)^2 * eps of the variance). K comes from stat_shift() (set
// by the bindings around a launch, like stat_shards; nullptr = unshifted, K = 0). With a sharded
// accumulator the producer also publishes the K it used in the accumulator's K row
// base[shards * rowlen + c] (every block stores the same values; block 0 does), which is what
// the fold reads — the fold's block 0 may overwrite the pilot itself while other blocks fold.
const float* stat_shift();
void set_stat_shift(const float* k);

__device__ __forceinline__ float shift_of(const float* k, int c) { return k ? k[c] : 0.f; }

__device__ __forceinline__ void stat_krow(float* base, int shards, size_t rowlen, const float* k,
                                          int C) {
  if (k && shards > 0 && blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0)
    for (int c = threadIdx.x; c < C; c += blockDim.x) base[(size_t)shards * rowlen + c] = k[c];
}

// ACT_RELU_Y: ReLU whose backward recomputes the sign from the BN input (z = y*scale + shift)
// instead of a stored mask / output — the BN output of a depthwise consumer that applies the BN
// on its loads (dwconv.hip "input transform") is never written
enum Act : int { ACT_NONE = 0, ACT_RELU = 1, ACT_SWISH = 2, ACT_SIGMOID = 3, ACT_RELU_Y = 4 };

__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + __expf(-x)); }

__device__ __forceinline__ float apply_act(float v, int act) {
  if (act == ACT_RELU || act == ACT_RELU_Y) return fmaxf(v, 0.f);
  if (act == ACT_SWISH) return v * sigmoidf_(v);
  if (act == ACT_SIGMOID) return sigmoidf_(v);
  return v;
}

// d act(z)/dz evaluated from the pre-activation z.
__device__ __forceinline__ float act_grad(float z, int act) {
  if (act == ACT_RELU || act == ACT_RELU_Y) return z > 0.f ? 1.f : 0.f;
  if (act == ACT_SWISH) {
    const float s = sigmoidf_(z);
    return s * (1.f + z * (1.f - s));
  }
  if (act == ACT_SIGMOID) {
    const float s = sigmoidf_(z);
    return s * (1.f - s);
  }
  return 1.f;
}

}  // namespace pca
