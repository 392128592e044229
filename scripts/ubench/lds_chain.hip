// Microbenchmark: dependent LDS table-lookup chains (the decode loop's skeleton).
// Each lane runs U independent chains; each step = one ds_read_b32 from a 2^K-entry
// table + EXTRA dependent VALU ops.  MODE 0: random index (hash of the state),
// MODE 1: conflict-free index (lane-distinct bank) but still data-dependent.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

template <int U, int MODE, int EXTRA>
__global__ __launch_bounds__(256) void chain(int K, int steps, uint32_t* out) {
  extern __shared__ uint32_t tab[];
  const uint32_t n = 1u << K;
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) tab[i] = (i * 2654435761u) ^ (i >> 3);
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  uint32_t x[U], idx[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    x[u] = (blockIdx.x * 256 + threadIdx.x) * 0x9E3779B1u + u * 0x85EBCA6Bu;
    idx[u] = x[u] >> (32 - K);
  }
  for (int s = 0; s < steps; ++s) {
    uint32_t e[U];
#pragma unroll
    for (int u = 0; u < U; ++u) e[u] = tab[idx[u]];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      uint32_t v = x[u] + e[u];
#pragma unroll
      for (int k = 0; k < EXTRA; ++k) v = __builtin_amdgcn_alignbit(v, x[u], e[u] + k);
      x[u] = v;
      if (MODE == 0) idx[u] = v >> (32 - K);
      else idx[u] = ((v & 0) + lane + 64 * (s & 3)) & (n - 1);
    }
  }
  uint32_t acc = 0;
#pragma unroll
  for (int u = 0; u < U; ++u) acc ^= x[u];
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

template <int U, int MODE, int EXTRA>
void run(int K, int blocks_per_cu, int ncu, uint32_t* d_out) {
  const int steps = 4096;
  const int grid = blocks_per_cu * ncu;
  size_t lds = (size_t(4) << K);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL((chain<U, MODE, EXTRA>), dim3(grid), dim3(256), lds, 0, K, 16, d_out);
  hipEventRecord(a);
  hipLaunchKernelGGL((chain<U, MODE, EXTRA>), dim3(grid), dim3(256), lds, 0, K, steps, d_out);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  // lookups per SIMD per cycle at 2.4 GHz
  const double lookups = double(grid) * 256 * U * steps;
  const double cyc = ms * 1e-3 * 2.4e9;
  printf("U=%d MODE=%d EXTRA=%2d K=%2d wg/cu=%d waves/simd=%d: %.3f ms  %.2f wave-lookups/CU/kcyc  %.1f cyc per wave-step per SIMD\n",
         U, MODE, EXTRA, K, blocks_per_cu, blocks_per_cu, ms, lookups / 64 / ncu / cyc * 1000,
         cyc / (lookups / 64 / ncu / 4));
  hipEventDestroy(a);
  hipEventDestroy(b);
}

int main() {
  int ncu;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  uint32_t* d_out;
  hipMalloc(&d_out, 8 * 256 * ncu * 4);
  for (int K : {9, 12})
    for (int wg : {1, 2, 4, 8}) {
      run<1, 0, 8>(K, wg, ncu, d_out);
      run<2, 0, 8>(K, wg, ncu, d_out);
      run<4, 0, 8>(K, wg, ncu, d_out);
      run<2, 1, 8>(K, wg, ncu, d_out);
      run<4, 1, 8>(K, wg, ncu, d_out);
      run<2, 0, 0>(K, wg, ncu, d_out);
      run<4, 0, 0>(K, wg, ncu, d_out);
      run<4, 1, 0>(K, wg, ncu, d_out);
    }
  return 0;
}
