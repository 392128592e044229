// Wave-tile decode ("wtile"), included by gh_decode.hip after the tile kernel (whose
// e-window decode, aligned staging and fixed-count copy-out helpers it uses).
//
// One persistent kernel, one decode pass, and no workgroup barrier after the LUT copy.
// The unit of work is a wave tile: 64 x U consecutive segments (lane l owns segments
// 64u + l of the tile).  A workgroup of NW waves takes NW consecutive wave tiles per
// iteration (one "WG tile"); workgroup b takes WG tiles b, b + G, b + 2G, ... (static
// round robin over the G resident workgroups), so iteration k of every workgroup is
// round k.  Per iteration, each wave alone:
//
//   1. decodes its tile from registers (words loaded one iteration earlier) into
//      per-lane symbol words (single-symbol LUT on pre-shifted windows, grouped
//      window shifts: decode_tile_grouped);
//   2. scans the segment counts with DPP, writes its total to an LDS ring slot and
//      bumps the slot's arrival counter; the wave that arrives last sums the NW
//      totals and publishes the WG tile's aggregate granule (no wave waits here);
//   3. (one wave per round) leads round k-1: loads the G aggregates of that round,
//      scans them and publishes each WG tile's within-round prefix and the next
//      round's offset R[k] = R[k-1] + round total;
//   4. copies its tile of iteration k-2 out of its own LDS staging buffer with
//      16-byte stores, at R[k-2] + the WG tile's prefix + the totals of the earlier
//      waves of the WG tile (LDS ring, iteration k-2); the next tile's words are
//      loaded just before those stores (fixed store count: vmcnt(N), not vmcnt(0));
//   5. stages this tile into the buffer just emptied: aligned dwords, then the head
//      bytes of each segment — one wave's LDS operations complete in order, so the
//      two phases need no barrier.
//
// Every hand-off has an iteration of slack; a wave waits only when a prefix two
// rounds old is still missing.  Reference counterpart: gpu_dec_l1_l2
// (decoder.cu:454-730): count (:529-569), scan + decoupled look-back (:571-653),
// decode and write (:655-728); its atomic ticket (:494-499) is a static round robin
// here (a waiting wave never holds an unstarted tile of an earlier round).

#ifndef GH_WT_DEFAULT
#define GH_WT_DEFAULT 0  // wave-tile kernel by default for grouped codes (else the tile kernel)
#endif
#ifndef GH_WT_NW
#define GH_WT_NW 8  // waves per workgroup
#endif
constexpr int WT_NW = GH_WT_NW;
constexpr int WT_TB = 64 * WT_NW;
constexpr int WT_U = 2;           // segments per lane per tile
constexpr int WT_RING = 8;        // iterations of wave totals kept in LDS (see the ring note)
#ifndef GH_WT_PF
#define GH_WT_PF 2                // iterations between a tile's loads and its decode (1 or 2)
#endif
constexpr uint32_t WT_PF = GH_WT_PF;
#ifndef GH_WT_NS
#define GH_WT_NS 2                // 16-byte stores per lane per copy-out (the rest loops)
#endif
#ifndef GH_WT_ABLATE
#define GH_WT_ABLATE 0  // diagnostic variants only (results wrong): 1 no copy-out, 2 no prefix wait, 4 no staging, 8 no decode
#endif
constexpr unsigned long long WT_SPIN_TICKS = 400000000ull;  // 4 s of the 100 MHz clock

#ifdef GH_STAMPS
#define WT_STAMP_DECL unsigned long long wst_acc[8] = {}; unsigned long long wst_last = __builtin_amdgcn_s_memtime();
#define WT_STAMP(i) do { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); wst_acc[i] += t_ - wst_last; wst_last = t_; } while (0)
#define WT_STAMP_FLUSH do { if (lane == 0 && p.stamps) { for (int i_ = 0; i_ < 8; ++i_) p.stamps[((size_t)blockIdx.x * NW + wid) * 16 + i_] = wst_acc[i_]; } } while (0)
#else
#define WT_STAMP_DECL
#define WT_STAMP(i) do {} while (0)
#define WT_STAMP_FLUSH do {} while (0)
#endif

struct WtParams {
  const uint32_t* payload;       // local segment j owns words [4j, 4j+4); +1 look-ahead, zero padded
  const uint32_t* gaps;          // nibble gap_nib0 + j - 1 = start of local segment j >= 1
  const uint32_t* lut;           // 2^K u32 {len | sym << 24}
  uint8_t* out;
  unsigned int* agg;             // per WG tile: epoch << 16 | its symbol count (<= 32768)
  unsigned int* status;
  unsigned long long* total;
  uint4* junk;                   // 16 bytes per thread of the grid: padding stores with nothing to duplicate
  unsigned long long out_cap;
  unsigned int nseg, ntiles, ntw;  // segments, WG tiles, wave tiles with segments
  unsigned int gap_nib0, first_start, kbits, lgr;
  unsigned int epoch;            // 1 .. 0xFFFF (granules carry it in their high half)
  unsigned int lut_bytes;        // LUT bytes in LDS (replicated 4 << (K + lgr))
  unsigned int stage_bytes;      // one staging buffer of one wave
  unsigned long long* stamps;    // diagnostic build only (GH_STAMPS): per-wave phase cycles
};

// LDS after the LUT and the staging: per ring slot (iteration mod WT_RING) the NW wave
// totals, the NW partial window sums, the WG tile's prefix (u64 as two words) and its
// tag, and two arrival counters.
template <int NW>
inline size_t wt_lds_bytes(size_t lut_bytes, size_t stage_bytes) {
  return lut_bytes + (size_t)NW * 2 * stage_bytes + 4 * WT_RING * (2 * NW + 5) + 16;
}

__device__ __forceinline__ bool wt_ok(const WtParams& p, uint32_t v) { return (v >> 16) == p.epoch; }

// Poll an aggregate until it carries this launch's epoch.  Bounded by wall time (a
// persistent kernel sharing the GPU with another kernel may wait for its not-yet-
// resident workgroups: a delay, not a fault); after a timeout every poll returns at once.
__device__ __forceinline__ uint32_t wt_poll(const WtParams& p, unsigned int* g) {
  if (__hip_atomic_load(p.status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & GH_ST_TIMEOUT)
    return p.epoch << 16;
  const unsigned long long t0 = wall_clock64();
  for (;;) {
    const uint32_t v = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (wt_ok(p, v)) return v;
    if (wall_clock64() - t0 > WT_SPIN_TICKS) {
      atomicOr(p.status, (unsigned)GH_ST_TIMEOUT);
      return p.epoch << 16;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

// Prefixes without a leader.  WG tile j = kG + b (iteration k of workgroup b) starts at
//   P(j) = P(j - G) + T(j - G) + sum of the aggregates of WG tiles (j - G, j)
// (P(j - G), T(j - G): the same workgroup's previous tile, held in LDS).  At the top of
// iteration k every wave loads its share of the G - 1 aggregates for P of iteration
// k-1 (one u32 per lane, published during iterations k-2 and k-1); after its decode it
// sums them with DPP, and the last of the NW waves to arrive adds the partial sums and
// writes P(k-1) to the LDS ring.  The copy-out of iteration k+1 reads it there.  No
// workgroup waits on another's prefix, only on other workgroups' aggregates, which
// are published right after each decode.
//
// LDS ring slots are reused every WT_RING iterations: waves of a workgroup stay within
// two iterations of each other (a wave's copy-out of iteration k needs P(k-2), written
// once every wave has finished the window step of iteration k-1), so 8 slots are ample.
template <int NW, int GRP, int NS, int LPW>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(4, 4)))
void gh_wtile_kernel(const WtParams p) {
  constexpr int U = WT_U;
  constexpr int TBW = 64 * NW;
  constexpr uint32_t R = WT_RING;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  uint32_t* ring = (uint32_t*)(smem + p.lut_bytes + (size_t)NW * 2 * p.stage_bytes);
  volatile uint32_t* s_wt = ring;                   // [R][NW] wave totals
  volatile uint32_t* s_ps = ring + R * NW;          // [R][NW] partial window sums
  volatile uint32_t* s_pk = ring + 2 * R * NW;      // [R][2] WG tile prefix (lo, hi)
  volatile uint32_t* s_tag = ring + 2 * R * NW + 2 * R;  // [R] iteration whose prefix the slot holds
  uint32_t* s_arr = ring + 2 * R * NW + 3 * R;      // [2][R] arrival counters (totals, windows)
  {  // LUT to LDS, replicated: dword i of LDS = entry i >> lgr
    const uint32_t nd = p.lut_bytes >> 2;
    uint32_t* sl = (uint32_t*)smem;
    for (uint32_t i = tid; i < nd; i += TBW) sl[i] = p.lut[i >> p.lgr];
    if (tid < (int)R) s_tag[tid] = 0xFFFFFFFFu;
    if (tid < 2 * (int)R) s_arr[tid] = 0;
  }
  if (tid == 0 && (uint32_t)(size_t)(const __attribute__((address_space(3))) uint8_t*)smem != 0u)
    atomicOr(p.status, (unsigned)GH_ST_LAYOUT);
  __syncthreads();  // the only barrier

  const uint32_t S = 30u - p.kbits - p.lgr;
  const uint32_t amask = ((1u << p.kbits) - 1u) << (2u + p.lgr);
  const uint32_t laneoff = ((uint32_t)lane & ((1u << p.lgr) - 1u)) << 2;
  const uint32_t G = gridDim.x, vb = blockIdx.x;  // host: G <= ntiles, G - 1 <= 64 * NW * LPW
  const uint32_t last_k = (p.ntiles - 1u - vb) / G;
  const uint32_t stg0 = p.lut_bytes + (uint32_t)wid * 2u * p.stage_bytes;  // absolute LDS address
  uint4* junk = p.junk + (size_t)blockIdx.x * TBW + tid;
  const uint32_t ezero = p.epoch << 16;

  // a tile's words: loaded WT_PF iterations before its decode (register sets A, B)
  struct Words {
    uint4 w[U];
    uint32_t w4[U], gw[U];
  };
  auto load = [&](uint32_t k, Words& r) {
    const uint32_t t = min(k * G + vb, p.ntiles - 1u) * (uint32_t)NW + (uint32_t)wid;  // wave tile
    const uint32_t seg0 = t * (uint32_t)(64 * U) + (uint32_t)lane;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t sc = min(seg0 + (uint32_t)(64 * u), p.nseg - 1u);
      r.w[u] = *(const uint4*)(p.payload + 4ull * sc);
      r.w4[u] = p.payload[4ull * sc + 4];
      r.gw[u] = p.gaps[(p.gap_nib0 + (sc ? sc - 1u : 0u)) >> 3];
    }
  };
  uint32_t tot1 = 0, tot2 = 0;  // this wave's totals of iterations k-1, k-2
  WT_STAMP_DECL
  auto iter = [&](uint32_t k, Words& cur) {
    const bool have_cur = k <= last_k;
    const bool have2 = k >= 2;
    const uint32_t j = k * G + vb;                        // WG tile of this iteration
    const uint32_t t = j * (uint32_t)NW + (uint32_t)wid;  // wave tile
    const uint32_t slot = k % R;
    // window of P(k-1): WG tiles [lo, jp), jp = (k-1)G + b
    const bool do_pref = k >= 1 && k - 1u <= last_k;
    const uint32_t jp = j - G, lo = jp >= G ? jp - G + 1u : 0u;
    uint32_t wv[LPW];
#pragma unroll
    for (int q = 0; q < LPW; ++q) {
      const uint32_t i = lo + (uint32_t)((q * NW + wid) * 64 + lane);
      wv[q] = (do_pref && i < jp) ? __hip_atomic_load(&p.agg[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                  : ezero;
    }
    // ---- 1. decode ------------------------------------------------------------
    uint32_t ow[U][OW], cnt[U];
    {
      int start[U];
      bool act[U];
      uint32_t e[U][5];
      const uint32_t seg0 = t * (uint32_t)(64 * U) + (uint32_t)lane;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t seg = seg0 + (uint32_t)(64 * u);
        act[u] = have_cur && seg < p.nseg;
        const uint32_t nib = (p.gap_nib0 + seg - 1u) & 7u;
        start[u] = seg == 0 ? (int)p.first_start : (int)((cur.gw[u] >> (4 * nib)) & 15u);
        make_ewin(cur.w[u], cur.w4[u], start[u], S, e[u]);
      }
      auto nothing = [&]() {};
      if (have_cur && (GH_WT_ABLATE & 8)) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          cnt[u] = act[u] ? 16u : 0u;
#pragma unroll
          for (int m = 0; m < OW; ++m) ow[u][m] = m < 5 ? e[u][m] : 0u;
        }
      } else if (have_cur) {
        decode_tile_grouped<GRP, U, 1000>(e, start, act, ow, cnt, amask, laneoff, nothing);
      } else {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          cnt[u] = 0;
#pragma unroll
          for (int m = 0; m < OW; ++m) ow[u][m] = 0;
        }
      }
    }
    WT_STAMP(0);
    // ---- 2. scan; wave total to the LDS ring; the last arriver publishes -------
    uint32_t lpos[U], wtot = 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t incl = wave_incl_scan(cnt[u], lane);
      lpos[u] = wtot + incl - cnt[u];
      wtot += (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    }
    if (have_cur && lane == 0) {
      s_wt[slot * NW + wid] = wtot;
      const uint32_t old = __hip_atomic_fetch_add(&s_arr[slot], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
      if (old % NW == NW - 1) {
        uint32_t sum = 0;
#pragma unroll
        for (int q = 0; q < NW; ++q) sum += s_wt[slot * NW + q];
        __hip_atomic_store(&p.agg[j], ezero | sum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    WT_STAMP(1);
    // ---- 3. window sum; the last arriver writes P(k-1) --------------------------
    if (do_pref) {
      bool ready = true;
#pragma unroll
      for (int q = 0; q < LPW; ++q) ready &= wt_ok(p, wv[q]);
      if (!__all(ready)) {
#pragma unroll
        for (int q = 0; q < LPW; ++q)
          if (!wt_ok(p, wv[q])) wv[q] = wt_poll(p, &p.agg[lo + (uint32_t)((q * NW + wid) * 64 + lane)]);
      }
      uint32_t ws = 0;
#pragma unroll
      for (int q = 0; q < LPW; ++q) ws += wv[q] & 0xFFFFu;
      ws = (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan(ws, lane), 63);  // < 2^32
      if (lane == 0) {
        s_ps[slot * NW + wid] = ws;
        const uint32_t old = __hip_atomic_fetch_add(&s_arr[R + slot], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (old % NW == NW - 1) {
          unsigned long long pk = 0;
          if (k >= 2) {
            const uint32_t s2 = (k - 2u) % R;
            pk = ((unsigned long long)s_pk[2 * s2 + 1] << 32) | s_pk[2 * s2];
#pragma unroll
            for (int q = 0; q < NW; ++q) pk += s_wt[s2 * NW + q];
          }
#pragma unroll
          for (int q = 0; q < NW; ++q) pk += s_ps[slot * NW + q];
          const uint32_t s1 = (k - 1u) % R;
          s_pk[2 * s1] = (uint32_t)pk;
          s_pk[2 * s1 + 1] = (uint32_t)(pk >> 32);
          s_tag[s1] = k - 1u;
        }
      }
    }
    WT_STAMP(2);
    // ---- 4. copy out the tile of iteration k-2 ---------------------------------
    const uint32_t buf = stg0 + (k & 1u) * p.stage_bytes;
    if (have2) {
      unsigned long long goff = 0;
      if ((GH_WT_ABLATE & 2) && lane == 0) {
        goff = (unsigned long long)(j - 2u * G) * NW * 2048ull + wid * 2048ull;
      } else if (lane == 0) {
        const uint32_t s2 = (k - 2u) % R;
        if (s_tag[s2] != k - 2u) {  // written once every wave of the WG did iteration k-1's window step
          const unsigned long long t0 = wall_clock64();
          while (s_tag[s2] != k - 2u) {
            if (wall_clock64() - t0 > WT_SPIN_TICKS) {
              atomicOr(p.status, (unsigned)GH_ST_TIMEOUT);
              break;
            }
            __builtin_amdgcn_s_sleep(1);
          }
        }
        goff = ((unsigned long long)s_pk[2 * s2 + 1] << 32) | s_pk[2 * s2];
#pragma unroll
        for (int q = 0; q < NW - 1; ++q)
          if (q < wid) goff += s_wt[s2 * NW + q];
        if ((j - 2u * G) * (uint32_t)NW + (uint32_t)wid == p.ntw - 1u) *p.total = goff + tot2;
      }
      goff = rfl_u64(goff);
      WT_STAMP(3);
      const uint32_t n2 =
          goff >= p.out_cap ? 0u : (uint32_t)min<unsigned long long>(tot2, p.out_cap - goff);
      if constexpr (WT_PF == 1) load(k + 1u, cur);  // the next tile's words, before this copy-out's stores
      if (!(GH_WT_ABLATE & 1)) copy_out_tile_fixed<64, NS>(p.out, buf, goff, n2, lane, junk);
    } else if constexpr (WT_PF == 1) {
      load(k + 1u, cur);
    }
    WT_STAMP(4);
    // ---- 5. stage this tile (the buffer just emptied) ---------------------------
    if (have_cur && !(GH_WT_ABLATE & 4)) {
      const uint32_t sbase = buf + STAGE_PAD;
      uint32_t nb[U];
#pragma unroll
      for (int u = 0; u < U; ++u) nb[u] = cnt[u] ? stage_aligned_p1(ow[u], cnt[u], sbase + lpos[u]) : 0u;
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (nb[u]) stage_head(sbase + lpos[u], ow[u][0], nb[u]);
    }
    WT_STAMP(5);
    // two iterations ahead: the tile after next, issued once this tile is staged (the
    // other register set is in flight meanwhile)
    if constexpr (WT_PF == 2) load(k + 2u, cur);
    tot2 = tot1;
    tot1 = wtot;
    WT_STAMP(6);
  };
  Words A, B;
  load(0, A);
  if constexpr (WT_PF == 1) {
    for (uint32_t k = 0; k <= last_k + 2u; ++k) iter(k, A);
  } else {
    load(1, B);
    for (uint32_t k = 0; k <= last_k + 2u; k += 2) {
      iter(k, A);
      if (k + 1u <= last_k + 2u) iter(k + 1u, B);
    }
  }
  WT_STAMP_FLUSH;
}
