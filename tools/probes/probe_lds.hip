// Probe: semantics of ds_read_b64_tr_b16 and buffer_load ... lds (OOB zero fill) on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef short s4 __attribute__((ext_vector_type(4)));

__global__ void tr_probe(short* out) {
  __shared__ __attribute__((aligned(16))) short lds[64 * 64];
  for (int i = threadIdx.x; i < 64 * 64; i += 64) lds[i] = i;  // value = row*64 + col (64-col rows)
  __syncthreads();
  const int l = threadIdx.x, li = l & 15, q = li >> 2, p = li & 3, G = l >> 4;
  // group G: block rows 4G..4G+3, cols 0..15; lane 4q+p supplies &lds[row q][col 4p]
  const int row = 4 * G + q, col = 4 * p;
  s4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4*)(lds + row * 64 + col));
  for (int e = 0; e < 4; ++e) out[l * 4 + e] = v[e];
}

__global__ void dma_probe(const int* src, int nbytes, int* out) {
  __shared__ __attribute__((aligned(16))) int lds[1024];
  for (int i = threadIdx.x; i < 1024; i += 64) lds[i] = -1;
  __syncthreads();
  __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)src, 0, nbytes, 0x00020000);
  // lane l fetches 16B from byte offset (63-l)*16; lanes >= 48 get an out-of-range offset
  int voff = (threadIdx.x >= 48) ? 0x7ffffff0 : (63 - threadIdx.x) * 16;
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)lds, 16, voff, 0, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  for (int i = threadIdx.x; i < 256; i += 64) out[i] = lds[i];
}

int main() {
  short* d; hipMalloc(&d, 64 * 4 * 2);
  tr_probe<<<1, 64>>>(d);
  short h[256]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  int bad = 0;
  for (int l = 0; l < 64; ++l) {
    const int G = l >> 4, i = l & 15;
    for (int e = 0; e < 4; ++e) {
      int expect = (4 * G + e) * 64 + i;  // column i of row (4G+e)
      if (h[l * 4 + e] != expect) ++bad;
    }
  }
  printf("tr16: lane0 = %d %d %d %d ; lane1 = %d %d %d %d ; lane17 = %d %d %d %d ; mismatches vs 'lane i gets col i rows 0..3' = %d\n",
         h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7], h[68], h[69], h[70], h[71], bad);
  int *s, *o; hipMalloc(&s, 1024 * 4); hipMalloc(&o, 256 * 4);
  int hs[1024]; for (int i = 0; i < 1024; ++i) hs[i] = i; hipMemcpy(s, hs, sizeof(hs), hipMemcpyHostToDevice);
  dma_probe<<<1, 64>>>(s, 1024 * 4, o);
  int ho[256]; hipMemcpy(ho, o, sizeof(ho), hipMemcpyDeviceToHost);
  int bad2 = 0;
  for (int l = 0; l < 64; ++l) for (int e = 0; e < 4; ++e) {
    int expect = (l >= 48) ? 0 : (63 - l) * 4 + e;
    if (ho[l * 4 + e] != expect) ++bad2;
  }
  printf("dma: lds[0..3]=%d %d %d %d lds[48*4]=%d mismatches=%d\n", ho[0], ho[1], ho[2], ho[3], ho[192], bad2);
  return (bad || bad2) ? 1 : 0;
}
