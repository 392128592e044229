// Microbenchmark: what a streaming copy reaches on this MI355X, to size the yardstick
// (gh_bw_copy) and the decode's memory bound.  1 GiB -> 1 GiB (2 GiB moved) unless
// argv[1] gives MiB per side.  Variants: loads per lane in flight (U), nontemporal or
// plain, workgroups per CU, workgroup size.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

template <int U, bool NT, int TB>
__global__ __launch_bounds__(TB) void copyk(v4u* __restrict__ dst, const v4u* __restrict__ src, uint64_t n16) {
  const uint64_t stride = (uint64_t)gridDim.x * TB;
  uint64_t i = (uint64_t)blockIdx.x * TB + threadIdx.x;
  for (; i + (U - 1) * stride < n16; i += U * stride) {
    v4u v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = NT ? __builtin_nontemporal_load(src + i + u * stride) : src[i + u * stride];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (NT) __builtin_nontemporal_store(v[u], dst + i + u * stride);
      else dst[i + u * stride] = v[u];
    }
  }
  for (; i < n16; i += stride) dst[i] = src[i];
}

// Block-contiguous: each workgroup copies one contiguous chunk (like a tile kernel).
template <int U, int TB>
__global__ __launch_bounds__(TB) void copy_chunks(v4u* __restrict__ dst, const v4u* __restrict__ src, uint64_t n16,
                                                  uint64_t per_block) {
  const uint64_t b0 = (uint64_t)blockIdx.x * per_block, b1 = b0 + per_block < n16 ? b0 + per_block : n16;
  for (uint64_t i = b0 + threadIdx.x; i < b1; i += (uint64_t)U * TB) {
    v4u v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = (i + u * TB < b1) ? src[i + u * TB] : v4u{0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i + u * TB < b1) dst[i + u * TB] = v[u];
  }
}

int main(int argc, char** argv) {
  const uint64_t mib = argc > 1 ? strtoull(argv[1], nullptr, 10) : 1024;
  const uint64_t bytes = mib << 20, n16 = bytes / 16;
  v4u *a, *b;
  if (hipMalloc(&a, bytes) || hipMalloc(&b, bytes)) { printf("alloc failed\n"); return 1; }
  hipMemset(a, 1, bytes);
  hipMemset(b, 2, bytes);
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto run = [&](const char* name, auto launch) {
    for (int i = 0; i < 3; ++i) launch();
    hipEventRecord(e0);
    for (int i = 0; i < 10; ++i) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= 10;
    printf("%-44s %8.1f us  %7.0f GB/s (read+write)\n", name, ms * 1e3, 2.0 * bytes / (ms * 1e-3) / 1e9);
  };
#define GRID(k, TB) dim3((unsigned)(ncu * (k)))
#define RUN(U, NT, TB, K)                                                                                   \
  run(#U " nt=" #NT " tb=" #TB " wg/cu=" #K,                                                                \
      [&] { hipLaunchKernelGGL((copyk<U, NT, TB>), GRID(K, TB), dim3(TB), 0, 0, b, a, n16); })
  RUN(4, true, 256, 8);
  RUN(4, false, 256, 8);
  RUN(1, false, 256, 8);
  RUN(2, false, 256, 8);
  RUN(8, false, 256, 8);
  RUN(4, false, 256, 4);
  RUN(4, false, 256, 16);
  RUN(4, false, 512, 2);
  RUN(4, false, 512, 4);
  RUN(4, false, 1024, 2);
  RUN(8, false, 512, 4);
  RUN(4, true, 512, 4);
  for (unsigned k : {2u, 4u, 8u}) {
    const uint64_t blocks = (uint64_t)ncu * 64 * k;
    const uint64_t per = (n16 + blocks - 1) / blocks;
    char nm[64];
    snprintf(nm, sizeof nm, "chunks 512thr U4 blocks=%llu", (unsigned long long)blocks);
    run(nm, [&] { hipLaunchKernelGGL((copy_chunks<4, 512>), dim3((unsigned)blocks), dim3(512), 0, 0, b, a, n16, per); });
  }
  printf("status %s\n", hipGetErrorString(hipDeviceSynchronize()));
  return 0;
}
