// Microbenchmark: per-lane streaming copies at various strides vs a
// wave-cooperative copy (diagnostic for the lane decode engine)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef __attribute__((address_space(1))) uint8_t g_u8;
__device__ __forceinline__ uint4 gld16(const uint8_t* p) { uint4 v; __builtin_memcpy(&v, (const g_u8*)p, 16); return v; }
__device__ __forceinline__ void gst16(uint8_t* p, uint4 v) { __builtin_memcpy((g_u8*)p, &v, 16); }
// each lane copies len bytes at src + l*stride -> dst + l*stride, starting at rotation rot*l
__global__ void k_lane(const uint8_t* src, uint8_t* dst, uint64_t stride, uint32_t len, uint32_t nl, uint32_t rot) {
  const uint32_t l = blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= nl) return;
  const uint8_t* s = src + (uint64_t)l * stride;
  uint8_t* d = dst + (uint64_t)l * stride;
  const uint32_t r0 = (rot * l) % len & ~63u;
  for (uint32_t c = 0; c < len; c += 64) {
    uint32_t o = c + r0; if (o >= len) o -= len;
    uint4 a = gld16(s + o), b = gld16(s + o + 16), e = gld16(s + o + 32), f = gld16(s + o + 48);
    gst16(d + o, a); gst16(d + o + 16, b); gst16(d + o + 32, e); gst16(d + o + 48, f);
  }
}
// each wave copies its 64 lanes' regions cooperatively (1 KiB per step)
__global__ void k_wave(const uint8_t* src, uint8_t* dst, uint64_t stride, uint32_t len, uint32_t nl) {
  const uint32_t w0 = (blockIdx.x * blockDim.x + threadIdx.x) & ~63u, ln = threadIdx.x & 63;
  for (uint32_t k = 0; k < 64 && w0 + k < nl; k++) {
    const uint8_t* s = src + (uint64_t)(w0 + k) * stride;
    uint8_t* d = dst + (uint64_t)(w0 + k) * stride;
    for (uint32_t c = 16 * ln; c < len; c += 1024) gst16(d + c, gld16(s + c));
  }
}
int main() {
  const uint32_t nl = 100000, len = 65536;
  uint64_t strides[3] = {65536, 65536 + 4352, 65536 * 2};
  uint8_t *a, *b;
  const size_t bytes = (size_t)nl * 65536 * 2 + (1 << 20);
  if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, bytes) != hipSuccess) { printf("alloc failed\n"); return 1; }
  hipMemset(a, 1, bytes); hipMemset(b, 0, bytes);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int si = 0; si < 3; si++) for (int rot = 0; rot < 2; rot++) {
    for (int rep = 0; rep < 2; rep++) {
      hipEventRecord(e0);
      hipLaunchKernelGGL(k_lane, dim3((nl + 255) / 256), dim3(256), 0, 0, a, b, strides[si], len, nl, rot ? 1088u : 0u);
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      if (rep) printf("lane stride %llu rot %d: %.2f ms  %.1f GB/s (read+write)\n", (unsigned long long)strides[si], rot, ms, 2.0 * nl * len / ms / 1e6);
    }
  }
  for (int si = 0; si < 3; si++) for (int rep = 0; rep < 2; rep++) {
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_wave, dim3((nl + 255) / 256), dim3(256), 0, 0, a, b, strides[si], len, nl);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    if (rep) printf("wave stride %llu: %.2f ms  %.1f GB/s\n", (unsigned long long)strides[si], ms, 2.0 * nl * len / ms / 1e6);
  }
  return 0;
}
