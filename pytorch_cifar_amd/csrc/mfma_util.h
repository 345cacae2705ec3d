// Device helpers shared by the MFMA convolution kernels (conv_mfma.hip, conv_halo.hip):
// exact division by runtime constants, buffer descriptors + LDS-DMA, counted waits, raw
// barriers and the transposed (ds_read_b64_tr_b16) fragment reads of [k][col] LDS images.
#pragma once
#include "common.h"

#include <algorithm>

#include <cstdio>
#include <cstdlib>

namespace pca {

// Resident workgroups per CU of a kernel on gfx950 (160 KiB LDS, 512 VGPR+AGPR per lane per SIMD,
// 8 waves per SIMD), from the code object's attributes. hipOccupancyMaxActiveBlocksPerMultiprocessor
// is not used: on this stack it reported 1 block/CU for every kernel with > 32 KiB of LDS, which
// sized the persistent grids for a quarter of the machine.
inline int blocks_per_cu(const void* fn, int threads, const char* name) {
  hipFuncAttributes a{};
  (void)hipFuncGetAttributes(&a, fn);
  const int waves = (threads + 63) / 64;                 // per block
  const int wps = (waves + 3) / 4;                       // waves per SIMD per block
  int regs = a.numRegs > 0 ? a.numRegs : 256;
  regs = (regs + 7) / 8 * 8;
  int by_regs = std::max(1, 512 / regs);                 // waves per SIMD
  by_regs = std::min(by_regs, 8) / wps;
  const int lds = (int)a.sharedSizeBytes;
  const int by_lds = lds > 0 ? (160 * 1024) / lds : 32;
  int occ = std::max(1, std::min({by_regs, by_lds, 32 / waves}));
  int api = 0;
  (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&api, fn, threads, 0);
  static const bool verbose = getenv("PCA_CONV_VERBOSE") != nullptr;
  if (verbose)
    fprintf(stderr, "[pca] occupancy %s: regs=%d lds=%d threads=%d -> %d blocks/CU (hip api %d)\n",
            name, a.numRegs, lds, threads, occ, api);
  return occ;
}

// Exact unsigned division by a runtime constant (n < 2^31): q = (umulhi(n, m) + n) >> s.
struct FastDiv {
  uint32_t d, m, s;
};

static inline FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  f.d = d;
  uint32_t s = 0;
  while ((1ull << s) < d) ++s;
  f.s = s;
  f.m = (uint32_t)(((1ull << 32) * ((1ull << s) - d)) / d + 1);
  return f;
}

__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
  const uint64_t t = (uint64_t)__umulhi(n, f.m) + n;
  return (uint32_t)(t >> f.s);
}

typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, bytes, 0x00020000);
}

// one 16-byte-per-lane LDS-DMA (1 KiB per wave instruction at lds_base + 16*lane).
// Issued from inline asm (M0 saved/set/restored inside the statement, cdna_hip_programming.md
// §5.7) so the compiler does not see an LDS write in flight: with the builtin, hipcc (ROCm 7.2)
// emits `s_waitcnt vmcnt(0)` before every ds_read_b64_tr_b16 that follows a DMA issue, which
// drained the whole prefetch pipeline each K-step of the transposed-read (wgrad) kernels.
// Completion is ordered by the kernels' own counted vmcnt waits + barriers.
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rs, char* lds_base, uint32_t voff) {
  typedef __attribute__((address_space(3))) char lds_char;
  const uint32_t lds = __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(lds_char*)lds_base);
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %1\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %2, %3, 0 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "s"(lds), "v"(voff), "s"(rs)
      : "memory");
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int N>
__device__ __forceinline__ void wait_vmcnt_rt(int n) {
  // counted wait with a wave-uniform runtime count (n <= N; folds to one wait for a constant n)
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

__device__ __forceinline__ void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

constexpr uint32_t kOOB = 0x80000000u;  // byte offset past any descriptor range -> zeros

// LDS image of a [BKP pixel][COLS channel] tile: 16-byte chunk c of pixel-row r lives at
// r*RB + 16*(c ^ tr_swz(r)). The XOR spreads the 8 rows one ds_read_b64_tr_b16 half-wave
// touches (rows k0..k0+3 and k0+8..k0+11) over all 64 banks.
template <int RB>
__device__ __forceinline__ int tr_swz(int r) {
  if constexpr (RB == 256) return 2 * ((r & 3) | (((r >> 3) & 1) << 2));
  else if constexpr (RB == 128) return 2 * (((r >> 1) & 1) | (((r >> 3) & 1) << 1));
  else return 2 * ((r >> 3) & 1);
}

template <int COLS>
__device__ __forceinline__ bf16x8 tr_frag(const char* base, int k0, int c0, int lane) {
  constexpr int RB = COLS * 2;
  typedef __attribute__((address_space(3))) i16x4 lds_i16x4;
  typedef short i16x8 __attribute__((ext_vector_type(8)));
  const int li = lane & 15;
  const int q = li >> 2, p = li & 3;
  const int col = c0 + 4 * p;
  const int chunk = col >> 3;
  const int r0 = k0 + 8 * (lane >> 4) + q;
  const int r1 = r0 + 4;
  const int b0 = r0 * RB + ((chunk ^ tr_swz<RB>(r0)) << 4) + ((col & 7) << 1);
  const int b1 = r1 * RB + ((chunk ^ tr_swz<RB>(r1)) << 4) + ((col & 7) << 1);
  const i16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(base + b0));
  const i16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(base + b1));
  const i16x8 v = __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, v);
}

}  // namespace pca
