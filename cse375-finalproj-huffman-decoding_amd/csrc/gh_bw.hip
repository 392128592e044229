// gh_bw.hip — the streaming-copy yardstick the decode's roofline is quoted against
// (BASELINE.md §3 "GPU metric": the fraction of a measured streaming copy on the same
// box, next to the 8 TB/s figure).  Diagnostic entry point; not on the decode path.
//
// One pass reads `bytes` and writes `bytes` with 16-byte lanes, four loads in flight
// per lane, a grid of 8 workgroups of 256 threads per CU (persistent, grid-stride).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>

#include "gh_internal.hpp"

namespace gh {
namespace {

#define GH_HIP(expr)                                                              \
  do {                                                                            \
    hipError_t e_ = (expr);                                                       \
    if (e_ != hipSuccess)                                                         \
      return fail(GH_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));   \
  } while (0)

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
constexpr int BW_TB = 256;
constexpr int BW_UNROLL = 4;

__global__ __launch_bounds__(BW_TB) void gh_bw_copy_kernel(v4u* __restrict__ dst,
                                                            const v4u* __restrict__ src, uint64_t n16) {
  const uint64_t stride = (uint64_t)gridDim.x * BW_TB;
  uint64_t i = (uint64_t)blockIdx.x * BW_TB + threadIdx.x;
  for (; i + (BW_UNROLL - 1) * stride < n16; i += BW_UNROLL * stride) {
    v4u v[BW_UNROLL];
#pragma unroll
    for (int u = 0; u < BW_UNROLL; ++u) v[u] = __builtin_nontemporal_load(src + i + u * stride);
#pragma unroll
    for (int u = 0; u < BW_UNROLL; ++u) __builtin_nontemporal_store(v[u], dst + i + u * stride);
  }
  for (; i < n16; i += stride) __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}

}  // namespace
}  // namespace gh

using namespace gh;

extern "C" int gh_bw_copy(void* dst, const void* src, uint64_t bytes, void* hip_stream, int reps,
                          float* ms_avg) {
  if (!dst || !src || (bytes & 15) || ((uintptr_t)dst & 15) || ((uintptr_t)src & 15))
    return fail(GH_E_ARG, "gh_bw_copy: null or non-16-byte-aligned buffer or size");
  if (reps < 1) reps = 1;
  hipStream_t st = (hipStream_t)hip_stream;
  int dev = 0, ncu = 0;
  GH_HIP(hipGetDevice(&dev));
  GH_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  const uint64_t n16 = bytes / 16;
  const uint32_t grid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)ncu * 8, (n16 + BW_TB - 1) / BW_TB));
  hipEvent_t e0, e1;
  GH_HIP(hipEventCreate(&e0));
  GH_HIP(hipEventCreate(&e1));
  hipLaunchKernelGGL(gh_bw_copy_kernel, dim3(grid), dim3(BW_TB), 0, st, (v4u*)dst, (const v4u*)src, n16);
  GH_HIP(hipEventRecord(e0, st));
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL(gh_bw_copy_kernel, dim3(grid), dim3(BW_TB), 0, st, (v4u*)dst, (const v4u*)src, n16);
  GH_HIP(hipEventRecord(e1, st));
  GH_HIP(hipGetLastError());
  GH_HIP(hipEventSynchronize(e1));
  float ms = 0;
  GH_HIP(hipEventElapsedTime(&ms, e0, e1));
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  if (ms_avg) *ms_avg = ms / reps;
  return GH_OK;
}
