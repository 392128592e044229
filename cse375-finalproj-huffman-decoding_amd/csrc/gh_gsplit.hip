// Grouped single-symbol split decode ("gsplit"), included by gh_decode.hip after the
// tile kernel (it reuses its decode loop and staging helpers).
//
// For the codes of the tile kernel's grouped path (complete, every codeword within
// the LUT width, minlen >= 4): two kernels and no inter-workgroup waiting, instead of
// the tile kernel's per-round prefixes (whose polls, waiting for the slowest
// workgroup of a round, measured about a sixth of that kernel's time).
//
//   gh_gs_count_kernel  decodes every segment of a workgroup's contiguous tile range
//                       counting codewords (the reference rule: codewords starting
//                       before the segment end, decoder.cu:529-569) and writes the
//                       range's total; no per-segment output.
//   gh_gs_write_kernel  offsets its range by the totals before it, decodes each tile
//                       again into registers (decode_tile_grouped), scans the counts,
//                       stages the bytes in LDS at the output's 16-byte alignment
//                       (aligned dword stores, then the 1-3 head bytes of each
//                       segment) and copies the tile out with aligned 16-byte stores.
//
// Count and write ranges nest (count grid = count_per x write grid).  Reference
// counterpart: gpu_dec_l1_l2's count / scan / decode passes (decoder.cu:529-728).

constexpr int TB_GS = 256;  // workgroup size of both kernels
constexpr int U_GS = 2;     // segments per thread (lock-step chains)

struct GsParams {
  const uint32_t* payload;       // local segment j owns words [4j, 4j+4); +1 look-ahead, zero padded
  const uint32_t* gaps;          // nibble gap_nib0 + j - 1: start of segment j >= 1
  const uint32_t* lut;           // 2^K u32 {len | sym << 24}
  unsigned long long* wg_tot;    // symbols per count-kernel workgroup range
  uint8_t* out;
  unsigned int* status;
  unsigned long long* total;
  unsigned long long out_cap;
  uint32_t nseg, ntiles, gap_nib0, first_start, kbits, lgr, lut_bytes, stage_bytes, count_per;
};

template <int U, int TBK>
__device__ __forceinline__ void gs_load(const GsParams& p, uint32_t tile, int tid, uint4 (&w)[U],
                                        uint32_t (&w4)[U], uint32_t (&ga)[U]) {
  const uint32_t t = min(tile, p.ntiles - 1);
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint32_t seg = t * (uint32_t)(U * TBK) + (uint32_t)(u * TBK + tid);
    const uint32_t sc = min(seg, p.nseg - 1);
    w[u] = *(const uint4*)(p.payload + 4ull * sc);
    w4[u] = p.payload[4ull * sc + 4];
    ga[u] = p.gaps[(p.gap_nib0 + (sc ? sc - 1u : 0u)) >> 3];
  }
}

// LUT to LDS, replicated 2^lgr times (dword i of LDS = entry i >> lgr); returns the
// e-window shift S and sets the address mask and this lane's replica offset.
template <int TBK>
__device__ __forceinline__ uint32_t gs_setup(const GsParams& p, uint8_t* smem, int tid, uint32_t& amask,
                                             uint32_t& laneoff) {
  uint32_t* sl = (uint32_t*)smem;
  for (uint32_t i = tid; i < p.lut_bytes / 4; i += TBK) sl[i] = p.lut[i >> p.lgr];
  amask = ((1u << p.kbits) - 1u) << (2u + p.lgr);
  laneoff = ((uint32_t)(tid & 63) & ((1u << p.lgr) - 1u)) << 2;
  return 30u - p.kbits - p.lgr;
}

template <int U, int TBK>
__device__ __forceinline__ void gs_windows(const GsParams& p, uint32_t t, int tid, const uint4 (&w)[U],
                                           const uint32_t (&w4)[U], const uint32_t (&ga)[U], uint32_t S,
                                           uint32_t (&e)[U][5], int (&start)[U], bool (&act)[U]) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint32_t seg = t * (uint32_t)(U * TBK) + (uint32_t)(u * TBK + tid);
    act[u] = seg < p.nseg;
    start[u] = seg == 0 ? (int)p.first_start : (int)ms_nib(ga[u], p.gap_nib0 + seg - 1u);
    make_ewin(w[u], w4[u], start[u], S, e[u]);
  }
}

template <int U, int TBK, int G>
__global__ __launch_bounds__(TBK) void gh_gs_count_kernel(const GsParams p) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int tid = threadIdx.x;
  uint32_t amask, laneoff;
  const uint32_t S = gs_setup<TBK>(p, smem, tid, amask, laneoff);
  const uint32_t t0 = (uint32_t)(((unsigned long long)blockIdx.x * p.ntiles) / gridDim.x);
  const uint32_t t1 = (uint32_t)(((unsigned long long)(blockIdx.x + 1) * p.ntiles) / gridDim.x);
  uint4 w[U];
  uint32_t w4[U], ga[U];
  if (t0 < t1) gs_load<U, TBK>(p, t0, tid, w, w4, ga);
  if (tid == 0 && (uint32_t)(size_t)(const __attribute__((address_space(3))) uint8_t*)smem != 0u)
    atomicOr(p.status, (unsigned)GH_ST_LAYOUT);
  __syncthreads();
  unsigned long long wg_total = 0;
  for (uint32_t t = t0; t < t1; ++t) {
    uint32_t e[U][5], cnt[U];
    int start[U];
    bool act[U];
    gs_windows<U, TBK>(p, t, tid, w, w4, ga, S, e, start, act);
    if (t + 1 < t1) gs_load<U, TBK>(p, t + 1, tid, w, w4, ga);  // prefetch
    uint32_t ow[U][OW];
    decode_tile_grouped<G, U, 0, void (*)(), false>(e, start, act, ow, cnt, amask, laneoff, []() {});
#pragma unroll
    for (int u = 0; u < U; ++u) wg_total += cnt[u];  // inactive segments count 0
  }
  wg_total = wave_sum_u64(wg_total);
  __syncthreads();
  unsigned long long* s_red = (unsigned long long*)smem;
  if ((tid & 63) == 0) s_red[tid >> 6] = wg_total;
  __syncthreads();
  if (tid == 0) {
    unsigned long long s = 0;
    for (int q = 0; q < TBK / 64; ++q) s += s_red[q];
    p.wg_tot[blockIdx.x] = s;
  }
}

template <int U, int TBK, int G>
__global__ __launch_bounds__(TBK) void gh_gs_write_kernel(const GsParams p) {
  constexpr int NWAVE = TBK / 64;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  uint8_t* s_stage = smem + p.lut_bytes;
  uint32_t* s_wsum = (uint32_t*)(s_stage + p.stage_bytes);                     // [U][NWAVE]
  unsigned long long* s_base = (unsigned long long*)(s_wsum + U * NWAVE + 2);  // [NWAVE]
  uint32_t amask, laneoff;
  const uint32_t S = gs_setup<TBK>(p, smem, tid, amask, laneoff);
  const uint32_t t0 = (uint32_t)(((unsigned long long)blockIdx.x * p.ntiles) / gridDim.x);
  const uint32_t t1 = (uint32_t)(((unsigned long long)(blockIdx.x + 1) * p.ntiles) / gridDim.x);
  uint4 w[U];
  uint32_t w4[U], ga[U];
  if (t0 < t1) gs_load<U, TBK>(p, t0, tid, w, w4, ga);
  {  // output offset of this range: the count totals of the ranges before it
    unsigned long long b = 0;
    const uint32_t nb = blockIdx.x * p.count_per;
    for (uint32_t i = tid; i < nb; i += TBK) b += p.wg_tot[i];
    b = wave_sum_u64(b);
    if (lane == 0) s_base[wid] = b;
  }
  if (tid == 0 && (uint32_t)(size_t)(const __attribute__((address_space(3))) uint8_t*)smem != 0u)
    atomicOr(p.status, (unsigned)GH_ST_LAYOUT);
  __syncthreads();
  unsigned long long goff = 0;
#pragma unroll
  for (int q = 0; q < NWAVE; ++q) goff += s_base[q];
  const uint32_t stage0 = p.lut_bytes;  // absolute LDS address of the staging buffer
  for (uint32_t t = t0; t < t1; ++t) {
    uint32_t e[U][5], cnt[U];
    int start[U];
    bool act[U];
    gs_windows<U, TBK>(p, t, tid, w, w4, ga, S, e, start, act);
    if (t + 1 < t1) gs_load<U, TBK>(p, t + 1, tid, w, w4, ga);  // prefetch
    uint32_t ow[U][OW];
    decode_tile_grouped<G, U, 0, void (*)(), true>(e, start, act, ow, cnt, amask, laneoff, []() {});
    uint32_t bpos[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t incl = wave_incl_scan(cnt[u], lane);
      if (lane == 63) s_wsum[u * NWAVE + wid] = incl;
      bpos[u] = incl - cnt[u];
    }
    __syncthreads();  // wave sums; the previous tile's copy-out is done
    uint32_t ttot = 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      uint32_t add = ttot;
#pragma unroll
      for (int q = 0; q < NWAVE; ++q) {
        const uint32_t x = s_wsum[u * NWAVE + q];
        add += (q < wid) ? x : 0u;
        ttot += x;
      }
      bpos[u] += add;
    }
    // staging byte 16 + lb + i = tile byte i: staging chunk c <-> output bytes
    // [goff - lb - 16 + 16c, +16), aligned 16-byte copies
    const uint32_t lb = (uint32_t)(goff & 15);
    uint32_t nb[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      nb[u] = 0;
      if (cnt[u]) nb[u] = stage_aligned_p1(ow[u], cnt[u], stage0 + 16u + lb + bpos[u]);
    }
    __syncthreads();  // phase 1 done: every segment's tail dword is in place
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (nb[u]) stage_head(stage0 + 16u + lb + bpos[u], ow[u][0], nb[u]);
    __syncthreads();  // tile staged
    const unsigned long long a0 = goff - lb;
    const unsigned long long oend = min(goff + ttot, p.out_cap);
    const uint32_t nz = (16u + lb + ttot + 15u) >> 4;
    const uint4* st4 = (const uint4*)s_stage;
    constexpr int CO = 4;
    for (uint32_t c0 = 1u + tid; c0 < nz; c0 += CO * TBK) {
      uint4 d[CO];
#pragma unroll
      for (int i = 0; i < CO; ++i) d[i] = st4[min(c0 + (uint32_t)i * TBK, nz - 1u)];
#pragma unroll
      for (int i = 0; i < CO; ++i) {
        const uint32_t c = c0 + (uint32_t)i * TBK;
        const unsigned long long gs = a0 - 16 + 16ull * c;
        if (c >= nz || gs >= oend) continue;
        if (gs >= goff && gs + 16 <= oend) {
          *(uint4*)(p.out + gs) = d[i];
        } else {
          const uint32_t wv[4] = {d[i].x, d[i].y, d[i].z, d[i].w};
#pragma unroll
          for (int k = 0; k < 16; ++k) {
            const unsigned long long ga2 = gs + k;
            if (ga2 >= goff && ga2 < oend) p.out[ga2] = (uint8_t)(wv[k >> 2] >> (8 * (k & 3)));
          }
        }
      }
    }
    goff += ttot;
  }
  if (blockIdx.x == gridDim.x - 1 && tid == 0) *p.total = goff;
}
