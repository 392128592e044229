// Microbenchmark: output write patterns for the decode kernel.  Each lane owns a
// variable-length byte record (n in [nlo, nhi], records packed back to back, as the
// per-segment outputs of the decoder are).  Modes:
//   0  coalesced 16-byte stores of the same total bytes (reference rate)
//   1  floor(n/4) unaligned dword stores + (n&3) byte stores per lane
//   2  same, but every record padded to a multiple of 4 bytes (aligned dwords)
//   3  unaligned dword stores in DESCENDING order incl. the partial last word
//      (the partial word's spill is overwritten by the next lane's first word)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

__device__ __forceinline__ uint32_t hash(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}

template <int MODE>
__global__ __launch_bounds__(256) void k_store(uint8_t* out, uint64_t nrec, int nlo, int nhi) {
  const uint64_t rec = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const int lane = threadIdx.x & 63;
  // record length and in-wave exclusive prefix
  const uint32_t span = (uint32_t)(nhi - nlo + 1);
  uint32_t n = rec < nrec ? nlo + hash((uint32_t)rec) % span : 0;
  if (MODE == 2) n = (n + 3) & ~3u;
  uint32_t incl = n;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t t = __shfl_up(incl, d, 64);
    if (lane >= d) incl += t;
  }
  const uint64_t wave0 = (rec - lane) * (uint64_t)((nlo + nhi + (MODE == 2 ? 3 : 0)) / 2 + 2);
  const uint64_t a = wave0 + incl - n;
  uint32_t ow[8];
#pragma unroll
  for (int m = 0; m < 8; ++m) ow[m] = hash((uint32_t)rec * 8 + m);
  if (MODE == 1 || MODE == 2) {
#pragma unroll
    for (int m = 0; m < 8; ++m)
      if (4 * m + 4 <= (int)n) *(uint32_t*)(out + a + 4 * m) = ow[m];
    const uint32_t full = n & ~3u;
    uint32_t last = 0;
#pragma unroll
    for (int m = 0; m < 8; ++m) last = (4 * m == (int)full) ? ow[m] : last;
#pragma unroll
    for (int b = 0; b < 3; ++b)
      if (full + b < n) out[a + full + b] = (uint8_t)(last >> (8 * b));
  } else if (MODE == 3) {
#pragma unroll
    for (int m = 7; m >= 0; --m)
      if (4 * m < (int)n) *(uint32_t*)(out + a + 4 * m) = ow[m];
  }
}

__global__ __launch_bounds__(256) void k_copy(uint4* out, uint64_t n16) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n16) out[i] = make_uint4((uint32_t)i, 1, 2, 3);
}

int main(int argc, char** argv) {
  const int nlo = argc > 1 ? atoi(argv[1]) : 14;
  const int nhi = argc > 2 ? atoi(argv[2]) : 19;
  const uint64_t nrec = 61363584ull;  // cfg4 segments
  const uint64_t bytes = nrec * (uint64_t)(nhi + 8);
  uint8_t* out;
  hipMalloc(&out, bytes + 4096);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const uint64_t avg = nrec * (uint64_t)(nlo + nhi) / 2;
  auto run = [&](const char* name, auto launch) {
    for (int i = 0; i < 3; ++i) launch();
    hipEventRecord(e0);
    for (int i = 0; i < 10; ++i) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= 10;
    printf("%-28s %8.1f us  %7.1f GB/s written (avg record %d B)\n", name, ms * 1e3, avg / (ms * 1e-3) / 1e9,
           (nlo + nhi) / 2);
  };
  const unsigned grid = (unsigned)((nrec + 255) / 256);
  run("coalesced uint4", [&] { k_copy<<<(unsigned)((avg / 16 + 255) / 256), 256>>>((uint4*)out, avg / 16); });
  run("unaligned dword + bytes", [&] { k_store<1><<<grid, 256>>>(out, nrec, nlo, nhi); });
  run("aligned dword + bytes", [&] { k_store<2><<<grid, 256>>>(out, nrec, nlo, nhi); });
  run("unaligned dword descending", [&] { k_store<3><<<grid, 256>>>(out, nrec, nlo, nhi); });
  hipError_t err = hipDeviceSynchronize();
  printf("status %s\n", hipGetErrorString(err));
  return 0;
}
