// Microbenchmark: the tile kernel's skeleton built up feature by feature.
// Persistent 512-thread workgroups stream tiles of 1024 segments (uint4 + dword
// look-ahead + gap dword per segment, 2 segments per lane, register prefetch one
// tile ahead, one barrier per tile).  Feature bits (template F):
//   1  output: stage 16 B per segment in LDS, copy the previous tile out with
//      16-byte stores (double-buffered staging)
//   2  decode-like compute: STEPS dependent LDS lookups per segment chain, 2 chains
//   4  look-back: publish a granule per tile, 2 granule loads per lane per tile
//   8  wave scan + tile sums through LDS
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

template <int F, int STEPS>
__global__ __launch_bounds__(512) void skel(const uint32_t* payload, const uint32_t* gaps,
                                            uint4* out, unsigned long long* gran, uint32_t ntiles,
                                            uint32_t nseg, uint32_t* sink) {
  __shared__ uint4 stg[2][1024 + 4];
  __shared__ uint32_t lut[2048];
  __shared__ uint32_t wsum[2][16];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  for (int i = tid; i < 2048; i += 512) lut[i] = (i * 2654435761u) >> 7;
  __syncthreads();
  uint4 w[2];
  uint32_t w4[2], gw[2];
  auto load = [&](uint32_t t) {
    const uint32_t seg0 = min(t, ntiles - 1) * 1024u + tid;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const uint32_t sc = min(seg0 + u * 512u, nseg - 1);
      w[u] = *(const uint4*)(payload + 4ull * sc);
      w4[u] = payload[4ull * sc + 4];
      gw[u] = gaps[sc >> 3];
    }
  };
  uint32_t t = blockIdx.x;
  load(t);
  uint32_t acc = 0, par = 0, tprev = 0xFFFFFFFFu;
  for (; t < ntiles || tprev < ntiles; t += gridDim.x, par ^= 1) {
    const bool have = t < ntiles;
    uint4 v[2] = {w[0], w[1]};
    uint32_t g0 = gw[0] ^ w4[0], g1 = gw[1] ^ w4[1];
    unsigned long long ga = 0, gb = 0;
    if (F & 4) {
      const bool hp = tprev < ntiles;
      const long long pa = (long long)tprev - 1 - tid, pb = pa - 512;
      ga = __hip_atomic_load(&gran[(hp && pa > 0) ? pa : 0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      gb = __hip_atomic_load(&gran[(hp && pb > 0) ? pb : 0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    load(t + gridDim.x);
    if (F & 2) {
      uint32_t x0 = v[0].x ^ g0, x1 = v[1].x ^ g1;
#pragma unroll
      for (int s = 0; s < STEPS; ++s) {
        x0 = lut[(x0 >> 9) & 2047] + v[0].y;
        x1 = lut[(x1 >> 9) & 2047] + v[1].y;
      }
      v[0].z ^= x0;
      v[1].z ^= x1;
    }
    uint32_t tot = 1024;
    if (F & 8) {
      uint32_t c = (v[0].w & 7) + 14, incl = c;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(incl, d, 64);
        if (lane >= d) incl += y;
      }
      if (lane == 63) wsum[par][wid] = incl;
    }
    if (F & 4) acc += (uint32_t)(ga ^ gb);
    __syncthreads();
    if (F & 8) {
      tot = 0;
#pragma unroll
      for (int q = 0; q < 8; ++q) tot += wsum[par][q];
    }
    if ((F & 4) && tid == 0 && have)
      __hip_atomic_store(&gran[t], (unsigned long long)tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (F & 1) {
      if (tprev < ntiles) {  // copy the previous tile out
#pragma unroll
        for (int u = 0; u < 2; ++u) out[(unsigned long long)tprev * 1024 + u * 512 + tid] = stg[par ^ 1][u * 512 + tid];
      }
      if (have) {
        stg[par][tid] = v[0];
        stg[par][512 + tid] = v[1];
      }
    } else {
      acc += v[0].x + v[1].y + v[0].z + v[1].z;
    }
    tprev = have ? t : 0xFFFFFFFFu;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

int main() {
  const uint32_t nseg = 61363584u;  // cfg4
  const uint32_t ntiles = (nseg + 1023) / 1024;
  uint32_t *payload, *gaps, *sink;
  uint4* out;
  unsigned long long* gran;
  hipMalloc(&payload, 4ull * (4ull * nseg + 16));
  hipMalloc(&gaps, 4ull * (nseg / 8 + 16));
  hipMalloc(&out, 16ull * ntiles * 1024);
  hipMalloc(&gran, 8ull * ntiles);
  hipMalloc(&sink, 64);
  hipMemset(payload, 1, 4ull * (4ull * nseg + 16));
  hipMemset(gaps, 2, 4ull * (nseg / 8 + 16));
  hipMemset(gran, 0, 8ull * ntiles);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto run = [&](const char* name, auto kern, unsigned grid) {
    for (int i = 0; i < 3; ++i) kern<<<grid, 512>>>(payload, gaps, out, gran, ntiles, nseg, sink);
    hipEventRecord(e0);
    for (int i = 0; i < 10; ++i) kern<<<grid, 512>>>(payload, gaps, out, gran, ntiles, nseg, sink);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= 10;
    printf("%-40s grid %4u %8.1f us\n", name, grid, ms * 1e3);
  };
  for (unsigned grid : {512u}) {
    run("base (loads+barrier)", skel<0, 21>, grid);
    run("+scan", skel<8, 21>, grid);
    run("+output", skel<1, 21>, grid);
    run("+output +scan", skel<9, 21>, grid);
    run("+output +scan +lookback", skel<13, 21>, grid);
    run("+decode21", skel<2, 21>, grid);
    run("+decode21 +output", skel<3, 21>, grid);
    run("+decode21 +output +scan +lookback", skel<15, 21>, grid);
    run("+decode10 +output +scan +lookback", skel<15, 10>, grid);
    run("+decode40 +output +scan +lookback", skel<15, 40>, grid);
  }
  printf("status %s\n", hipGetErrorString(hipDeviceSynchronize()));
  return 0;
}
