// Probe: unaligned 16-byte LDS reads/writes (ds_read_b128 / ds_write_b128 at
// byte offsets) give the same bytes as byte-wise access
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef __attribute__((address_space(3))) uint8_t l_u8;
__device__ __forceinline__ uint4 lld16(const l_u8* p) { uint4 v; __builtin_memcpy(&v, p, 16); return v; }
__device__ __forceinline__ void lst16(l_u8* p, uint4 v) { __builtin_memcpy(p, &v, 16); }
__global__ void k(uint32_t* bad, uint32_t* sample) {
  __shared__ __attribute__((aligned(16))) uint8_t buf[8192];
  l_u8* b = (l_u8*)buf;
  const uint32_t l = threadIdx.x;
  for (uint32_t i = l; i < 8192; i += 64) b[i] = (uint8_t)(i * 7 + 3);
  __syncthreads();
  uint32_t nbad = 0;
  // unaligned reads
  for (uint32_t o = l; o < 4096; o += 64) {
    uint4 v = lld16(b + o);
    uint32_t w[4] = {v.x, v.y, v.z, v.w};
    for (int k2 = 0; k2 < 16; k2++) if (((w[k2 >> 2] >> (8 * (k2 & 3))) & 255) != (uint8_t)((o + k2) * 7 + 3)) nbad++;
  }
  __syncthreads();
  // unaligned writes: lane l writes 16 bytes at 4096 + 17*l
  uint4 v = make_uint4(0x03020100u + l * 0x10101010u, 0x07060504u, 0x0b0a0908u, 0x0f0e0d0cu);
  lst16(b + 4096 + 17 * l, v);
  __syncthreads();
  for (int k2 = 0; k2 < 16; k2++) {
    uint32_t w[4] = {v.x, v.y, v.z, v.w};
    if (b[4096 + 17 * l + k2] != ((w[k2 >> 2] >> (8 * (k2 & 3))) & 255)) nbad++;
  }
  atomicAdd(bad, nbad);
  if (l == 0) { uint4 s = lld16(b + 5); sample[0] = s.x; sample[1] = s.y; }
}
int main() {
  uint32_t *d; hipMalloc(&d, 64); hipMemset(d, 0, 64);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, d + 4);
  uint32_t h[8]; hipMemcpy(h, d, 32, hipMemcpyDeviceToHost);
  printf("lds unaligned b128 mismatches: %u (sample %08x %08x)\n", h[0], h[4], h[5]);
  return h[0] != 0;
}
