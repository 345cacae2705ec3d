// Probe: per-CU store throughput of a split-K epilogue. B blocks of 512 threads each write a
// contiguous region of KB KiB with float4 stores (a partial-tile slab row), nothing else.
// Prints us per launch for (blocks, KiB per block) so that the time can be split into a
// chip-wide (total bytes) and a per-CU (bytes per block) term.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(512) void store_probe(float4* out, int per_block4, int nt) {
  if (nt == 2) {   // halo-epilogue layout: each wave writes its own contiguous per_block/8 region
    float4* dw = out + (size_t)blockIdx.x * per_block4 + (threadIdx.x >> 6) * (per_block4 / 8);
    const float v = (float)threadIdx.x;
    for (int i = threadIdx.x & 63; i < per_block4 / 8; i += 64) dw[i] = make_float4(v, v, v, v);
    return;
  }
  float4* dst = out + (size_t)blockIdx.x * per_block4;
  const float v = (float)threadIdx.x;
  for (int i = threadIdx.x; i < per_block4; i += 512) {
    if (nt)
      { typedef float f4v __attribute__((ext_vector_type(4))); f4v x = {v, v, v, v}; __builtin_nontemporal_store(x, reinterpret_cast<f4v*>(dst + i)); }
    else
      dst[i] = make_float4(v, v, v, v);
  }
}

int main() {
  float4* d;
  hipMalloc(&d, (size_t)512 * 1024 * 1024);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int blocks[] = {256, 512};
  const int kbs[] = {16, 48, 96, 147, 294};
  for (int nt = 0; nt < 3; nt += 2)
    for (int B : blocks)
      for (int kb : kbs) {
        const int per4 = kb * 1024 / 16;
        if ((size_t)B * kb * 1024 > (size_t)512 * 1024 * 1024) continue;
        for (int w = 0; w < 3; ++w) store_probe<<<B, 512>>>(d, per4, nt);
        hipEventRecord(a);
        for (int it = 0; it < 20; ++it) store_probe<<<B, 512>>>(d, per4, nt);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        const double us = ms * 1e3 / 20;
        printf("nt=%d blocks=%5d KiB/block=%4d total=%7.1f MB  %7.2f us  %6.2f TB/s\n", nt, B, kb,
               B * kb / 1024.0, us, B * kb * 1024.0 / us / 1e6);
      }
  return 0;
}
