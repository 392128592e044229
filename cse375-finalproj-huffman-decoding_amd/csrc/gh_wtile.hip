// Wave-tile decode ("wtile"), included by gh_decode.hip after the tile kernel (whose
// e-window decode, aligned staging and fixed-count copy-out helpers it uses) and after
// gh_msplit.hip (count-LUT helpers).
//
// One persistent kernel, no workgroup barrier after the LUT copy, and no wave waiting
// on another's prefix in steady state.  The unit of work is a wave tile: 64 x U
// consecutive segments (lane l owns segments 64u + l of the tile).  A workgroup of NW
// waves takes NW consecutive wave tiles per iteration (one "WG tile"); workgroup b takes
// WG tiles b, b + G, b + 2G, ... (static round robin over the G resident workgroups).
//
// The reference counts a tile, scans, and decodes it again (decoder.cu:529-728).  Here
// the count runs WT_L iterations AHEAD of the decode, so a tile's aggregate is
// published long before anyone needs it, and a tile is written out as soon as it is
// decoded (one staging buffer per wave, no lag to cover).  In iteration k each wave:
//
//   1. counts its wave tile of iteration k + L (words loaded one iteration earlier):
//      codeword ends per segment with the wave split's end-mask LUT (one v_bcnt per
//      lookup of up to 13 bits); the wave total goes to an LDS ring slot, and the last
//      of the NW waves to arrive publishes the WG tile's aggregate (u32, epoch-tagged);
//   2. sums its share of the G - 1 aggregates between the workgroup's tiles of
//      iterations k and k+1 (loaded at the top of the iteration; published L - 1
//      iterations ago), and the last arriver writes the WG tile prefix
//         P(k+1) = P(k) + T(k) + sum
//      to the LDS ring (P(k), T(k): the same workgroup's previous tile);
//   3. decodes its wave tile of iteration k (single-symbol LUT on pre-shifted windows,
//      grouped window shifts: decode_tile_grouped), scans the segment counts with DPP,
//      stages the bytes in its LDS buffer (aligned dwords, then each segment's head
//      bytes: one wave's LDS operations complete in order, so no barrier) and copies
//      them out with 16-byte stores at P(k) + the earlier waves' counted totals.
//
// A workgroup waits only when another workgroup's count is L - 1 iterations behind.
// The decode re-reads the payload the count read L iterations earlier: L x G x 32 KiB
// of traffic lies between, far inside the 256 MiB Infinity Cache, so HBM sees the
// payload once.  Reference counterpart: gpu_dec_l1_l2 (decoder.cu:454-730) — count
// (:529-569), scan + decoupled look-back (:571-653), decode and write (:655-728).

#ifndef GH_WT_DEFAULT
#define GH_WT_DEFAULT 0  // wave-tile kernel by default for grouped codes (else the tile kernel)
#endif
#ifndef GH_WT_NW
#define GH_WT_NW 8  // waves per workgroup
#endif
constexpr int WT_NW = GH_WT_NW;
constexpr int WT_TB = 64 * WT_NW;
constexpr int WT_U = 2;           // segments per lane per tile
constexpr int WT_RING = 16;       // LDS ring slots (iterations)
#ifndef GH_WT_L
#define GH_WT_L 2                 // iterations the count runs ahead of the decode (>= 1, <= 4)
#endif
constexpr int WT_L = GH_WT_L;
#ifndef GH_WT_ABLATE
#define GH_WT_ABLATE 0  // diagnostic variants only (results wrong): 1 no copy-out, 4 no staging, 8 no decode, 16 no count
#endif
#ifndef GH_WT_PRIO
#define GH_WT_PRIO 0  // alternate s_setprio between the two workgroup slots of a CU
#endif
#ifndef GH_WT_SCOPE
#define GH_WT_SCOPE __HIP_MEMORY_SCOPE_AGENT  // scope of the aggregate stores and loads
#endif
constexpr unsigned long long WT_SPIN_TICKS = 400000000ull;  // 4 s of the 100 MHz clock

#ifdef GH_STAMPS
#define WT_STAMP_DECL unsigned long long wst_acc[8] = {}; unsigned long long wst_last = __builtin_amdgcn_s_memtime();
#define WT_STAMP(i) do { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); wst_acc[i] += t_ - wst_last; wst_last = t_; } while (0)
#define WT_COUNT(i) do { wst_acc[i] += 1; } while (0)
#define WT_STAMP_FLUSH do { if (lane == 0 && p.stamps) { for (int i_ = 0; i_ < 8; ++i_) p.stamps[((size_t)blockIdx.x * NW + wid) * 16 + i_] = wst_acc[i_]; } } while (0)
#else
#define WT_STAMP_DECL
#define WT_STAMP(i) do {} while (0)
#define WT_COUNT(i) do {} while (0)
#define WT_STAMP_FLUSH do {} while (0)
#endif

struct WtParams {
  const uint32_t* payload;       // local segment j owns words [4j, 4j+4); +1 look-ahead, zero padded
  const uint32_t* gaps;          // nibble gap_nib0 + j - 1 = start of local segment j >= 1; + j its end
  const uint32_t* lut;           // decode: 2^K u32 {len | sym << 24}
  const uint32_t* lutc;          // count: 2^Kc u32 {b | end mask << 16}
  uint8_t* out;
  unsigned int* agg;             // per WG tile: epoch << 16 | its symbol count (<= 32768)
  unsigned int* status;
  unsigned long long* total;
  uint4* junk;                   // 16 bytes per thread of the grid: padding stores with nothing to duplicate
  unsigned long long out_cap;
  unsigned int nseg, ntiles, ntw;  // segments, WG tiles, wave tiles with segments
  unsigned int gap_nib0, first_start, kbits, kcbits, lgr;
  unsigned int last_end;         // != 0: end bit of local segment nseg-1 (the stream's last)
  unsigned int epoch;            // 1 .. 0xFFFF (aggregates carry it in their high half)
  unsigned int lut_bytes;        // decode LUT bytes in LDS (replicated 4 << (K + lgr))
  unsigned int lutc_bytes;       // count LUT bytes in LDS (4 << Kc)
  unsigned int stage_bytes;      // one wave's staging buffer
  unsigned long long* stamps;    // diagnostic build only (GH_STAMPS): per-wave phase cycles
};

// LDS after the two LUTs and the staging: per ring slot (iteration mod WT_RING) the NW
// counted wave totals, the NW partial window sums, the WG tile's prefix (two words), its
// tag, and two arrival counters.
template <int NW>
inline size_t wt_lds_bytes(size_t lut_bytes, size_t lutc_bytes, size_t stage_bytes) {
  return lut_bytes + lutc_bytes + (size_t)NW * stage_bytes + 4 * WT_RING * (2 * NW + 5) + 16;
}

// LDS ring accesses at absolute LDS byte addresses (the kernel's LDS starts at 0).  Inline
// asm: through a volatile generic pointer the compiler emits flat accesses, each followed
// by vmcnt(0) — a wait for every outstanding global load and store of the wave.
__device__ __forceinline__ uint32_t wt_ld(uint32_t a) {
  uint32_t v;
  asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a) : "memory");
  return v;
}
__device__ __forceinline__ void wt_st(uint32_t a, uint32_t v) {
  asm volatile("ds_write_b32 %0, %1" ::"v"(a), "v"(v) : "memory");
}
__device__ __forceinline__ uint32_t wt_add(uint32_t a, uint32_t v) {
  uint32_t r;
  asm volatile("ds_add_rtn_u32 %0, %1, %2\n\ts_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(a), "v"(v) : "memory");
  return r;
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
    const uint32_t v = __hip_atomic_load(g, __ATOMIC_RELAXED, GH_WT_SCOPE);
    if (wt_ok(p, v)) return v;
    if (wall_clock64() - t0 > WT_SPIN_TICKS) {
      atomicOr(p.status, (unsigned)GH_ST_TIMEOUT);
      return p.epoch << 16;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

// Ring slots are reused every WT_RING iterations.  The waves of a workgroup stay within
// about one iteration of each other (a wave's copy-out of iteration k needs P(k), written
// once every wave has finished the window step of iteration k-1), and a slot is last
// read L + 1 iterations after it is written, so 8 slots suffice for L <= 4.
// NS: 16-byte stores per lane per copy-out, enough for the worst-case wave tile (the
// host picks 4 or 5 from the code's shortest codeword), so the store count is fixed.
template <int NW, int GRP, int GC, int NS, int LPW>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(4, 8)))
void gh_wtile_kernel(const WtParams p) {
  constexpr int U = WT_U;
  constexpr int TBW = 64 * NW;
  constexpr uint32_t R = WT_RING;
  constexpr int L = WT_L;
  static_assert(L >= 1 && L + 3 <= (int)R, "ring too small for the count-ahead distance");
  static_assert(NW * 64 * U * 32 <= 65535, "WG tile total must fit the aggregate's 16 bits");
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  // ring (absolute LDS byte addresses): counted wave totals [R][NW], partial window sums
  // [R][NW], WG tile prefixes [R][2] (lo, hi), tags [R], arrival counters [2][R]
  const uint32_t a_ct = p.lut_bytes + p.lutc_bytes + (uint32_t)NW * p.stage_bytes;
  const uint32_t a_ps = a_ct + 4u * R * NW, a_pk = a_ps + 4u * R * NW, a_tag = a_pk + 8u * R,
                 a_arr = a_tag + 4u * R;
  {  // LUTs to LDS: decode replicated (dword i = entry i >> lgr), count as is
    uint32_t* sl = (uint32_t*)smem;
    for (uint32_t i = tid; i < (p.lut_bytes >> 2); i += TBW) sl[i] = p.lut[i >> p.lgr];
    uint32_t* sc = (uint32_t*)(smem + p.lut_bytes);
    for (uint32_t i = tid; i < (p.lutc_bytes >> 2); i += TBW) sc[i] = p.lutc[i];
    if (tid < (int)R) wt_st(a_tag + 4u * tid, 0xFFFFFFFFu);
    if (tid < 2 * (int)R) wt_st(a_arr + 4u * tid, 0u);
  }
  if (tid == 0 && (uint32_t)(size_t)(const __attribute__((address_space(3))) uint8_t*)smem != 0u)
    atomicOr(p.status, (unsigned)GH_ST_LAYOUT);
  __syncthreads();  // the only barrier

  const uint32_t S = 30u - p.kbits - p.lgr;
  const uint32_t amask = ((1u << p.kbits) - 1u) << (2u + p.lgr);
  const uint32_t laneoff = ((uint32_t)lane & ((1u << p.lgr) - 1u)) << 2;
  const uint32_t csh = 30u - p.kcbits;                   // count LUT: index bits -> byte offset
  const uint32_t cmask = ((1u << p.kcbits) - 1u) << 2;
  const uint32_t cbase = p.lut_bytes;                    // absolute LDS address of the count LUT
  const uint32_t G = gridDim.x, vb = blockIdx.x;         // host: G <= ntiles, G - 1 <= 64 * NW * LPW
  const int last_k = (int)((p.ntiles - 1u - vb) / G);
  const uint32_t buf = p.lut_bytes + p.lutc_bytes + (uint32_t)wid * p.stage_bytes;  // absolute LDS address
  uint4* junk = p.junk + (size_t)blockIdx.x * TBW + tid;
  const uint32_t ezero = p.epoch << 16;
  auto wave_tile = [&](int k) { return min((uint32_t)k * G + vb, p.ntiles - 1u) * (uint32_t)NW + (uint32_t)wid; };

  // a tile's words and gap words; loaded one iteration before they are used
  struct CWords {  // count pass: start and end nibbles
    uint4 w[U];
    uint32_t w4[U], ga[U], gb[U];
  };
  struct DWords {  // decode pass: start nibble
    uint4 w[U];
    uint32_t w4[U], gw[U];
  };
  auto load_c = [&](int k, CWords& r) {
    const uint32_t seg0 = wave_tile(k) * (uint32_t)(64 * U) + (uint32_t)lane;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t sc = min(seg0 + (uint32_t)(64 * u), p.nseg - 1u);
      r.w[u] = *(const uint4*)(p.payload + 4ull * sc);
      r.w4[u] = p.payload[4ull * sc + 4];
      r.ga[u] = p.gaps[(p.gap_nib0 + (sc ? sc - 1u : 0u)) >> 3];
      r.gb[u] = p.gaps[(p.gap_nib0 + sc) >> 3];
    }
  };
  auto load_d = [&](int k, DWords& r) {
    const uint32_t seg0 = wave_tile(k) * (uint32_t)(64 * U) + (uint32_t)lane;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t sc = min(seg0 + (uint32_t)(64 * u), p.nseg - 1u);
      r.w[u] = *(const uint4*)(p.payload + 4ull * sc);
      r.w4[u] = p.payload[4ull * sc + 4];
      r.gw[u] = p.gaps[(p.gap_nib0 + (sc ? sc - 1u : 0u)) >> 3];
    }
  };
  // Every iteration issues the same global operations, unconditionally (clamped
  // addresses, stores to junk slots when there is nothing to write): one window load,
  // the next count tile's loads, one aggregate store, the next decode tile's loads and
  // NS + 1 copy-out stores.  Loads and stores share the in-order vmcnt counter, so a
  // fixed sequence lets the compiler wait for a prefetch with vmcnt(N) instead of
  // vmcnt(0) (which would wait for every store still in flight).
  uint32_t* const agg_junk = (uint32_t*)junk;
  uint32_t bad = 0;                 // counted and decoded totals differ (corrupted stream)
  unsigned long long total = ~0ull;  // lane 0 of the wave holding the last wave tile
  // two register sets each, alternating by iteration parity (the loop is unrolled by
  // two), so a prefetch lands in the registers its consumer reads: no copies at the
  // loop's back edge, whose moves would each wait for the load in flight
  CWords cwA, cwB;
  DWords dwA, dwB;
  load_c(0, cwA);
  load_d(-L, dwA);
  WT_STAMP_DECL
  // count of iteration k + L, the window of P(k + 1)
  auto count_step = [&](int k, CWords& cw, CWords& cwn) {
#if GH_WT_PRIO
    // the second workgroup dispatched to a CU loses every issue-arbitration tie to the
    // first (age order): alternate the two slots' priority by iteration
    if ((((uint32_t)(k + 64) + (vb >= (G >> 1) ? 1u : 0u)) & 1u) != 0u) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
#endif
    const bool do_pref = k + 1 >= 0 && k + 1 <= last_k;
    const uint32_t jn = (uint32_t)(k + 1) * G + vb, lo = jn >= G ? jn - G + 1u : 0u;
    uint32_t wv[LPW];
#pragma unroll
    for (int q = 0; q < LPW; ++q) {
      const uint32_t i = lo + (uint32_t)((q * NW + wid) * 64 + lane);
      const uint32_t v = __hip_atomic_load(&p.agg[do_pref && i < jn ? i : 0u], __ATOMIC_RELAXED, GH_WT_SCOPE);
      wv[q] = (do_pref && i < jn) ? v : ezero;
    }
    const int kc = k + L;
    const bool have_c = kc <= last_k;
    const uint32_t seg0 = wave_tile(kc) * (uint32_t)(64 * U) + (uint32_t)lane;
    Win v[U];
    int Rb[U];
    uint32_t cnt[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t seg = seg0 + (uint32_t)(64 * u);
      const bool act = have_c && seg < p.nseg;
      const int start = seg == 0 ? (int)p.first_start : (int)ms_nib(cw.ga[u], p.gap_nib0 + seg - 1u);
      const int E = (p.last_end && seg == p.nseg - 1u) ? (int)p.last_end
                                                       : 128 + (int)ms_nib(cw.gb[u], p.gap_nib0 + seg);
      v[u] = make_win(cw.w[u], cw.w4[u], start);
      Rb[u] = act ? E - start : 0;
      cnt[u] = 0;
    }
    load_c(kc + 1, cwn);  // the next count tile's words (clamped; always issued)
    if (!(GH_WT_ABLATE & 16)) {
      for (int g = 0; g < 160; ++g) {
        uint32_t rm[U], q[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          rm[u] = ms_rmask(Rb[u]);
          q[u] = 32u;
        }
#pragma unroll
        for (int j = 0; j < GC; ++j) {
          uint32_t e[U];
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const uint32_t x = j == 0 ? v[u].d0 : __builtin_amdgcn_alignbit(v[u].d0, v[u].d1, q[u]);
            asm volatile("ds_read_b32 %0, %1" : "=v"(e[u]) : "v"(((x >> csh) & cmask) + cbase) : "memory");
          }
          lds_wait_all(e);
#pragma unroll
          for (int u = 0; u < U; ++u) {
            uint32_t m;
            asm("v_and_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD"
                : "=v"(m) : "v"(e[u]), "v"(rm[u]));
            cnt[u] = __builtin_popcount(m) + cnt[u];
            asm("v_ashrrev_i32 %0, %1, %0" : "+v"(rm[u]) : "v"(e[u]));
            q[u] -= e[u];
          }
        }
        bool more = false;
#pragma unroll
        for (int u = 0; u < U; ++u) {
          ms_shift(v[u], q[u]);  // consumed = 32 - (q & 0xFFFF): v_alignbit reads q & 31
          Rb[u] -= 32 - (int)(q[u] & 0xFFFFu);
          more |= Rb[u] > 0;
        }
        if (!__any(more)) break;
      }
    } else {
#pragma unroll
      for (int u = 0; u < U; ++u) cnt[u] = Rb[u] > 0 ? 16u : 0u;
    }
    uint32_t ctot = 0;
#pragma unroll
    for (int u = 0; u < U; ++u) ctot += cnt[u];
    ctot = (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan(ctot, lane), 63);
    // wave total to the ring; the last of the NW waves publishes the WG tile's aggregate
    // (every wave stores: the others to their junk slot)
    uint32_t* adst = agg_junk;
    uint32_t aval = 0;
    if (lane == 0 && have_c) {
      const uint32_t slot = (uint32_t)kc % R;
      wt_st(a_ct + 4u * (slot * NW + wid), ctot);
      const uint32_t old = wt_add(a_arr + 4u * slot, 1u);
      if (old % NW == NW - 1) {
#pragma unroll
        for (int q = 0; q < NW; ++q) aval += wt_ld(a_ct + 4u * (slot * NW + q));
        aval |= ezero;
        adst = &p.agg[(uint32_t)kc * G + vb];
      }
    }
    __hip_atomic_store(lane == 0 ? adst : agg_junk, aval, __ATOMIC_RELAXED, GH_WT_SCOPE);
    WT_STAMP(0);
    // window sum; the last arriver writes P(k+1) to the ring
    if (do_pref) {
      bool ready = true;
#pragma unroll
      for (int q = 0; q < LPW; ++q) ready &= wt_ok(p, wv[q]);
      if (!__all(ready)) {
        WT_COUNT(6);
#ifdef GH_STAMPS
        // diagnostics: poll rounds (one sc1 load each) until every window value is fresh
        for (int rounds = 0; rounds < 100000; ++rounds) {
          bool all = true;
#pragma unroll
          for (int q = 0; q < LPW; ++q)
            if (!wt_ok(p, wv[q])) {
              wv[q] = __hip_atomic_load(&p.agg[lo + (uint32_t)((q * NW + wid) * 64 + lane)], __ATOMIC_RELAXED,
                                        GH_WT_SCOPE);
              all = false;
            }
          if (__all(all)) break;
          WT_COUNT(7);
        }
#else
#pragma unroll
        for (int q = 0; q < LPW; ++q)
          if (!wt_ok(p, wv[q])) wv[q] = wt_poll(p, &p.agg[lo + (uint32_t)((q * NW + wid) * 64 + lane)]);
#endif
      }
      uint32_t ws = 0;
#pragma unroll
      for (int q = 0; q < LPW; ++q) ws += wv[q] & 0xFFFFu;
      ws = (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan(ws, lane), 63);  // < 2^32
      if (lane == 0) {
        const uint32_t slot = (uint32_t)(k + 1) % R;
        wt_st(a_ps + 4u * (slot * NW + wid), ws);
        const uint32_t old = wt_add(a_arr + 4u * (R + slot), 1u);
        if (old % NW == NW - 1) {
          unsigned long long pk = 0;
          if (k >= 0) {  // P(k) + T(k)
            const uint32_t s0 = (uint32_t)k % R;
            pk = ((unsigned long long)wt_ld(a_pk + 8u * s0 + 4u) << 32) | wt_ld(a_pk + 8u * s0);
#pragma unroll
            for (int q = 0; q < NW; ++q) pk += wt_ld(a_ct + 4u * (s0 * NW + q));
          }
#pragma unroll
          for (int q = 0; q < NW; ++q) pk += wt_ld(a_ps + 4u * (slot * NW + q));
          wt_st(a_pk + 8u * slot, (uint32_t)pk);
          wt_st(a_pk + 8u * slot + 4u, (uint32_t)(pk >> 32));
          wt_st(a_tag + 4u * slot, (uint32_t)(k + 1));  // after the value: one wave's LDS ops complete in order
        }
      }
    }
    WT_STAMP(1);
  };
  // decode, stage and copy out the wave tile of iteration k
  auto decode_step = [&](int k, DWords& dw, DWords& dwn) {
    const bool have_d = k >= 0;
    const uint32_t t = wave_tile(k < 0 ? 0 : k);
    uint32_t ow[U][OW], cnt[U];
    {
      int start[U];
      bool act[U];
      uint32_t e[U][5];
      const uint32_t seg0 = t * (uint32_t)(64 * U) + (uint32_t)lane;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t seg = seg0 + (uint32_t)(64 * u);
        act[u] = have_d && seg < p.nseg;
        const uint32_t nib = (p.gap_nib0 + seg - 1u) & 7u;
        start[u] = seg == 0 ? (int)p.first_start : (int)((dw.gw[u] >> (4 * nib)) & 15u);
        make_ewin(dw.w[u], dw.w4[u], start[u], S, e[u]);
      }
      load_d(k + 1, dwn);  // the next decode tile's words (clamped; the count read them: cache hits)
      auto nothing = [&]() {};
      if (GH_WT_ABLATE & 8) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          cnt[u] = act[u] ? 16u : 0u;
#pragma unroll
          for (int m = 0; m < OW; ++m) ow[u][m] = m < 5 ? e[u][m] : 0u;
        }
      } else {
        decode_tile_grouped<GRP, U, 1000>(e, start, act, ow, cnt, amask, laneoff, nothing);
      }
    }
    WT_STAMP(2);
    uint32_t lpos[U], wtot = 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t incl = wave_incl_scan(cnt[u], lane);
      lpos[u] = wtot + incl - cnt[u];
      wtot += (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    }
    unsigned long long goff = ~0ull;  // k < 0: past out_cap, nothing written
    if (lane == 0 && have_d) {
      const uint32_t s0 = (uint32_t)k % R;
      if (wt_ld(a_tag + 4u * s0) != (uint32_t)k) {  // written once every wave did the window step of k-1
        const unsigned long long t0 = wall_clock64();
        while (wt_ld(a_tag + 4u * s0) != (uint32_t)k) {
          if (wall_clock64() - t0 > WT_SPIN_TICKS) {
            bad |= GH_ST_TIMEOUT;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
      }
      goff = ((unsigned long long)wt_ld(a_pk + 8u * s0 + 4u) << 32) | wt_ld(a_pk + 8u * s0);
#pragma unroll
      for (int q = 0; q < NW - 1; ++q)
        if (q < wid) goff += wt_ld(a_ct + 4u * (s0 * NW + q));
      if (wt_ld(a_ct + 4u * (s0 * NW + wid)) != wtot) bad |= GH_ST_BADCODE;
      if (t == p.ntw - 1u) total = goff + wtot;
    }
    goff = rfl_u64(goff);
    WT_STAMP(3);
    if (!(GH_WT_ABLATE & 4)) {
      const uint32_t sbase = buf + STAGE_PAD;
      uint32_t nb[U];
#pragma unroll
      for (int u = 0; u < U; ++u) nb[u] = cnt[u] ? stage_aligned_p1(ow[u], cnt[u], sbase + lpos[u]) : 0u;
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (nb[u]) stage_head(sbase + lpos[u], ow[u][0], nb[u]);
    }
    WT_STAMP(4);
    const uint32_t n = goff >= p.out_cap ? 0u : (uint32_t)min<unsigned long long>(wtot, p.out_cap - goff);
    if (!(GH_WT_ABLATE & 1)) copy_out_tile_fixed<64, NS, false>(p.out, buf, goff, n, lane, junk);
    WT_STAMP(5);
  };
  // One loop from k = -L: iterations k < 0 count only (their decode step runs on no
  // segment and stores to junk slots), so every iteration issues the same operations.
  for (int k = -L; k <= last_k; k += 2) {
    count_step(k, cwA, cwB);
    decode_step(k, dwA, dwB);
    if (k + 1 > last_k) break;
    count_step(k + 1, cwB, cwA);
    decode_step(k + 1, dwB, dwA);
  }
  // rare outcomes, reported once (a conditional atomic inside the loop would break the
  // fixed operation sequence above)
  if (lane == 0 && bad) atomicOr(p.status, bad);
  if (lane == 0 && total != ~0ull) *p.total = total;
  WT_STAMP_FLUSH;
}
