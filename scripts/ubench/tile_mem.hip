// Microbenchmark: the memory pattern of the tile kernel alone (no decode, no LDS),
// to find the ceiling of its persistent structure.  Persistent grid of 512-thread
// workgroups, 2 per CU, static round-robin over tiles of 1536 segments (3 per lane):
// per iteration a workgroup loads tile t's 16-byte segment words (+ the look-ahead
// dword and the gap dword per segment: F & 1), and stores tile t-LAG's 16-byte words to
// the output (as the copy-out does).  Prefetch distance PF tiles (register sets).
// F & 2: nontemporal loads and stores; F & 4: one workgroup barrier per iteration.
// 1.01 GB in, 1.01 GB out, like cfg4.  Prints us per pass and GB/s (read + write).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

constexpr int TB = 512, U = 3;
typedef unsigned int v4u __attribute__((ext_vector_type(4)));

template <int F, int PF>
__global__ __launch_bounds__(TB) void tile_mem(const uint4* __restrict__ pay, const uint32_t* __restrict__ gaps,
                                              uint4* __restrict__ out, uint32_t ntiles, uint32_t* sink) {
  const int tid = threadIdx.x;
  uint4 w[PF][U];
  uint32_t x[PF][U];
  auto load = [&](int s, uint32_t t) {
    const uint32_t b = (t < ntiles ? t : ntiles - 1) * (uint32_t)(U * TB) + tid;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t sc = b + u * TB;
      if (F & 2) {
        const v4u q = __builtin_nontemporal_load((const v4u*)(pay + sc));
        w[s][u] = make_uint4(q.x, q.y, q.z, q.w);
      } else {
        w[s][u] = pay[sc];
      }
      x[s][u] = 0;
      if (F & 1) x[s][u] = ((const uint32_t*)pay)[4ull * sc + 4] ^ gaps[sc >> 3];
    }
  };
  uint32_t t = blockIdx.x;
#pragma unroll
  for (int s = 0; s < PF; ++s) load(s, t + s * gridDim.x);
  uint32_t acc = 0;
  for (; t < ntiles; t += gridDim.x) {
    uint4 v[U];
    uint32_t y = 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      v[u] = w[0][u];
      y ^= x[0][u];
    }
#pragma unroll
    for (int s = 0; s + 1 < PF; ++s)
#pragma unroll
      for (int u = 0; u < U; ++u) {
        w[s][u] = w[s + 1][u];
        x[s][u] = x[s + 1][u];
      }
    load(PF - 1, t + PF * gridDim.x);
    const uint32_t b = t * (uint32_t)(U * TB) + tid;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      v[u].x ^= y;
      if (F & 2) __builtin_nontemporal_store(v4u{v[u].x, v[u].y, v[u].z, v[u].w}, (v4u*)(out + b + u * TB));
      else out[b + u * TB] = v[u];
    }
    if (F & 4) __syncthreads();
    acc += y;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

int main(int argc, char** argv) {
  const uint64_t nseg = 63281250;  // cfg4: 1.0125 GB of payload
  const uint32_t ntiles = (uint32_t)((nseg + U * TB - 1) / (U * TB));
  const uint64_t n16 = (uint64_t)ntiles * U * TB + 16;
  uint4 *a, *b;
  uint32_t *g, *sink;
  if (hipMalloc(&a, n16 * 16) || hipMalloc(&b, n16 * 16) || hipMalloc(&g, n16 / 2 + 64) || hipMalloc(&sink, 64)) {
    printf("alloc failed\n");
    return 1;
  }
  hipMemset(a, 1, n16 * 16);
  hipMemset(g, 3, n16 / 2 + 64);
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const double bytes = 2.0 * (double)ntiles * U * TB * 16;
  auto run = [&](const char* name, auto kern, unsigned grid) {
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(kern, dim3(grid), dim3(TB), 0, 0, a, g, b, ntiles, sink);
    hipEventRecord(e0);
    for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(kern, dim3(grid), dim3(TB), 0, 0, a, g, b, ntiles, sink);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= 10;
    printf("%-40s grid %4u %8.1f us %7.0f GB/s\n", name, grid, ms * 1e3, bytes / (ms * 1e-3) / 1e9);
  };
  const unsigned g2 = 2 * ncu;
  run("x4 only, PF1", tile_mem<0, 1>, g2);
  run("x4+dwords, PF1", tile_mem<1, 1>, g2);
  run("x4+dwords, PF1, barrier", tile_mem<5, 1>, g2);
  run("x4+dwords, PF1, nt", tile_mem<3, 1>, g2);
  run("x4+dwords, PF2", tile_mem<1, 2>, g2);
  run("x4+dwords, PF2, barrier", tile_mem<5, 2>, g2);
  run("x4+dwords, PF2, nt", tile_mem<3, 2>, g2);
  run("x4+dwords, PF3", tile_mem<1, 3>, g2);
  run("x4 only, PF2", tile_mem<0, 2>, g2);
  run("x4+dwords, PF1, 4 WG/CU", tile_mem<1, 1>, 4 * ncu);
  run("x4+dwords, PF2, 4 WG/CU", tile_mem<1, 2>, 4 * ncu);
  printf("status %s\n", hipGetErrorString(hipDeviceSynchronize()));
  return 0;
}
