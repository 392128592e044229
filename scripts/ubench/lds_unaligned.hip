// Check: unaligned ds_write_b32 / ds_read_b32 in LDS (byte addresses not multiple of 4)
// and time a per-lane unaligned write stream (lanes ~41 bytes apart, 12 writes each).
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_check(uint32_t* out) {
  __shared__ uint8_t buf[4096];
  const int t = threadIdx.x;
  for (int i = t; i < 4096; i += 256) buf[i] = 0xEE;
  __syncthreads();
  // lane t writes 0xA0B0C0D0 + t at byte address 5 + 13*t (unaligned for most t)
  uint32_t v = 0xA0B0C0D0u + t;
  uint32_t addr = 5 + 13 * t;
  asm volatile("ds_write_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" :: "v"(addr), "v"(v) : "memory");
  __syncthreads();
  uint32_t r;
  asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(addr) : "memory");
  // reconstruct from bytes
  const uint32_t b = buf[addr] | (buf[addr + 1] << 8) | (buf[addr + 2] << 16) | (buf[addr + 3] << 24);
  out[3 * t] = v;
  out[3 * t + 1] = r;
  out[3 * t + 2] = b;
}

__global__ __launch_bounds__(512) void k_stream(uint32_t* sink, int iters, int aligned) {
  __shared__ uint8_t buf[512 * 48 + 64];
  const int t = threadIdx.x;
  uint32_t pos = t * 41 + 3;
  uint32_t acc = 0;
  for (int it = 0; it < iters; ++it) {
    uint32_t p = pos;
#pragma unroll
    for (int j = 0; j < 12; ++j) {
      const uint32_t a = aligned ? (p & ~3u) : p;
      asm volatile("ds_write_b32 %0, %1" :: "v"(a), "v"(p) : "memory");
      p += 3;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    acc += buf[(pos + it) % (512 * 41)];
  }
  if (acc == 0x12345) sink[0] = acc;
}

int main() {
  uint32_t* d;
  hipMalloc(&d, 1 << 20);
  k_check<<<1, 256>>>(d);
  uint32_t h[768];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  int bad = 0;
  for (int t = 0; t < 256; ++t)
    if (h[3 * t] != h[3 * t + 1] || h[3 * t] != h[3 * t + 2]) {
      if (bad < 4) printf("t=%d wrote %08x read %08x bytes %08x\n", t, h[3 * t], h[3 * t + 1], h[3 * t + 2]);
      ++bad;
    }
  printf("unaligned ds_write/read_b32: %s (%d mismatches)\n", bad ? "BROKEN" : "ok", bad);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int al = 1; al >= 0; --al) {
    k_stream<<<1024, 512>>>(d, 100, al);
    hipEventRecord(e0);
    k_stream<<<1024, 512>>>(d, 1000, al);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double writes = 1024.0 * 512 * 1000 * 12 / 64;  // wave-instructions
    printf("%s writes: %.3f ms, %.2f cycles/wave-instr/CU at 2.4GHz\n", al ? "aligned  " : "unaligned", ms,
           ms * 1e-3 * 2.4e9 * 256 / writes);
  }
  printf("status %s\n", hipGetErrorString(hipDeviceSynchronize()));
  return 0;
}
