// gh_bw.hip — the streaming-copy yardstick the decode's roofline is quoted against
// (BASELINE.md §3 "GPU metric": the fraction of a measured streaming copy on the same
// box, next to the 8 TB/s figure).  Diagnostic entry point; not on the decode path.
//
// One pass reads `bytes` and writes `bytes` with 16-byte lanes: workgroup b copies the
// contiguous chunk [b*CH, (b+1)*CH) (CH = 8 KiB, four loads in flight per lane).  This
// chunked form measured fastest of the copies tried on MI355X (scripts/ubench/copy_bw.hip:
// 6.1 TB/s read+write at 1 GiB, against 4.4-4.9 for persistent grid-stride loops).
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
constexpr int BW_TB = 512;
constexpr int BW_UNROLL = 4;

constexpr uint64_t BW_CHUNK16 = 512;  // 16-byte units per workgroup (8 KiB)

__global__ __launch_bounds__(BW_TB) void gh_bw_copy_kernel(v4u* __restrict__ dst, const v4u* __restrict__ src,
                                                            uint64_t n16) {
  const uint64_t b0 = (uint64_t)blockIdx.x * BW_CHUNK16;
  const uint64_t b1 = b0 + BW_CHUNK16 < n16 ? b0 + BW_CHUNK16 : n16;
  for (uint64_t i = b0 + threadIdx.x; i < b1; i += (uint64_t)BW_UNROLL * BW_TB) {
    v4u v[BW_UNROLL];
#pragma unroll
    for (int u = 0; u < BW_UNROLL; ++u) v[u] = (i + u * BW_TB < b1) ? src[i + u * BW_TB] : v4u{0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < BW_UNROLL; ++u)
      if (i + u * BW_TB < b1) dst[i + u * BW_TB] = v[u];
  }
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
  const uint64_t n16 = bytes / 16;
  const uint64_t nb = std::max<uint64_t>(1, (n16 + BW_CHUNK16 - 1) / BW_CHUNK16);
  if (nb > 0x7fffffffull) return fail(GH_E_ARG, "gh_bw_copy: size too large");
  const uint32_t grid = (uint32_t)nb;
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
