// Two-pass tile kernel: the decode of short-codeword codes (complete, 1 <= len <= 16,
// multi-symbol lookups worth >= 1.5 codewords, e.g. BASELINE's r = 0.9 data; codewords
// longer than the tables through a canonical fallback), included by
// gh_decode.hip after gh_tile.hip (whose round leader, prefix granules, copy-out and LDS
// helpers it shares).  Reference counterpart: gpu_dec_l1_l2 (decoder/src/decoder.cu:
// 454-730) — its count pass (:529-569), decoupled look-back (:571-653) and decode pass
// (:655-728) — with the payload read from HBM ONCE: the two passes run over the same
// register-resident words, one tile apart.
//
// A segment of these codes holds up to 64 codewords (128 with a 1-bit codeword: 11-bit
// tables then, 8.5 KB regions, and a copy-out in two parts, NP = 2), too many to keep as bytes in
// registers (the single-pass tile kernel's way), so a tile is decoded twice from its
// words, with one table of up to four codewords per lookup,
//   entry = {symbols (bytes 0..3), b | n << 8 | startmask << 16}
// (b = their bits, n = their number, startmask bit s = a codeword starts at window bit
// s).  Iteration k of a decoding workgroup (1024 threads, U = 2 segments per lane,
// wave-contiguous segments as in gh_tile.hip):
//
//   count tile k:  per lookup, cnt += popcount(startmask & rm), rm = the window bits
//                  still before the segment end (the reference's rule: a codeword is
//                  kept iff it starts before bit 128), rm >>= b;
//   load tile k+1's words; wave scans of the counts; the last wave to arrive publishes
//                  tile k's aggregate (as in gh_tile.hip);
//   write tile k-1 (its windows, offsets and counts held in registers since iteration
//                  k-1) into the wave's LDS region at its local offsets: each lookup's
//                  four bytes with one unaligned ds_write_b32;
//   read the prefix of tile k-1 (published during the last iteration) and copy the
//                  wave's piece out with the fixed-count 16-byte stores of gh_tile.hip.
//
// Write overruns: a lookup's four bytes past its n symbols are zeros, and the lookup that
// reaches a segment's end writes up to three bytes past it, over the next segment's first
// bytes, which that segment (another lane, in lock-step) wrote earlier; a finished
// segment's lane goes on writing (no branch) at its end, i.e. over the next segment's
// first four bytes.  So every segment keeps its first four bytes in a register (from its
// first four lookups: each holds at least one codeword) and stores them again after the
// wave's last lookup (a wave's LDS operations complete in order).  A segment has at least
// floor(113 / 12) = 9 codewords, so these head stores never overlap.
//
// The prefix of tile k-1 is needed one iteration after its aggregate left (the count
// pass is the first thing an iteration does, the prefix wait the last), with one staging
// region per wave.  Round 4's single-read attempt (gh_ftile.hip, removed) counted with a
// second table and ORed each lookup into a staging buffer that its own copy-out waited
// on: two LUTs left LDS for one buffer per workgroup, and it ran 0.77 ms on cfg3.

#ifndef GH_MTILE_TB
#define GH_MTILE_TB 1024
#endif
constexpr int MT_TB = GH_MTILE_TB;  // threads per workgroup
constexpr int MT_U = 2;             // segments per lane
#ifndef GH_MT_ABLATE
#define GH_MT_ABLATE 0  // diagnostic builds only, bits: 1 no count pass (40 symbols per segment),
                        // 2 no write pass, 4 no prefix wait (fake offsets); output wrong
#endif
#ifndef GH_MT_LAG
#define GH_MT_LAG 2  // a tile is written and copied out LAG iterations after its count pass
#endif
constexpr int MT_LAG = GH_MT_LAG;
#ifndef GH_MT_CLUT
#define GH_MT_CLUT 1  // the count pass reads its own u32 table (all codewords of the window,
                      // 4 << K bytes after the write table) instead of the write table's high words
#endif
#ifndef GH_MT_WOR
#define GH_MT_WOR 2  // write pass: 1 ORs into zeroed staging (two aligned ds_or_b32 per lookup,
                     // the copy-out re-zeroes), 2 the same with the bytes gathered into
                     // aligned dwords first (one ds_or_b32 per lookup), 0 unaligned
                     // ds_write_b32 + head restore
#endif
#ifndef GH_MT_NOFB
#define GH_MT_NOFB 0  // experiment: no chain-by-chain path
#endif
constexpr int MT_GMAX = 80;         // lookup groups per segment, at most (>= 1 codeword and >= 1 bit per lookup,
                                    // GL = 2: <= 64 groups to cover 128 codewords / bits)

// Advance a 5-word e-window by 32 - (q & 31) bits.
__device__ __forceinline__ void win_shift5(uint32_t (&e)[5], uint32_t q) {
  e[0] = __builtin_amdgcn_alignbit(e[0], e[1], q);
  e[1] = __builtin_amdgcn_alignbit(e[1], e[2], q);
  e[2] = __builtin_amdgcn_alignbit(e[2], e[3], q);
  e[3] = __builtin_amdgcn_alignbit(e[3], e[4], q);
  e[4] = __builtin_amdgcn_alignbit(e[4], 0u, q);
}

// Codes longer than the tables (FB): a codeword longer than the table width has no entry
// (b = 0 / n = 0); its 16 bits are taken from the e-window (S bits below the lookup
// position) and decoded canonically from the LDS tables (gh_wsplit.hip's ws_canon;
// codes here are complete, so every pattern decodes).
struct MtFb {
  const uint32_t* s_fb;
  uint32_t lo, hi;  // lengths searched: table width + 1 .. maxlen
};
__device__ __forceinline__ uint32_t mt_canon(const MtFb& fb, uint32_t x, uint32_t y, uint32_t S) {
  uint32_t bad = 0;
  return ws_canon(fb.s_fb, __builtin_amdgcn_alignbit(x, y, 32u - S) >> 16, fb.lo, fb.hi, bad);  // (sym << 8) | len
}

// LDS: LUT (8 << K bytes), one staging region per wave, the per-tile wave totals /
// offsets / arrival counters / prefixes (TILE_SLOTS tiles), leader wave totals.
inline size_t mtile_lds_bytes(size_t lut_bytes, size_t stage_bytes) {
  constexpr size_t NW = MT_TB / 64;
  return lut_bytes + NW * stage_bytes + TILE_SLOTS * (2 * NW + 1) * 4 + TILE_SLOTS * 12 + 4 * NW + 32;
}

// Count pass of U segments per lane on e-windows (S = 29 - K, u64 entries): codewords
// that start before the segment end, R = 128 - start bits away.  GL lookups per window
// shift (GL * K <= 24 bits: rm, recomputed per group from R, covers the group's starts).
template <int U, int GL, bool FB = false, int SH = 0>
__device__ __forceinline__ void mt_count(uint32_t (&e)[U][5], const int (&R0)[U], uint32_t (&cnt)[U], uint32_t amask,
                                         uint32_t cbase, const MtFb& fb = MtFb{}, uint32_t Sc = 0) {
  int R[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    R[u] = R0[u];
    cnt[u] = 0;
  }
  for (int g = 0; g < MT_GMAX; ++g) {
    uint32_t rm[U], q[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      rm[u] = __builtin_amdgcn_ubfe(0xFFFFFFFFu, 0, (uint32_t)min(max(R[u], 0), 31));  // (1 << R) - 1
      q[u] = 32u;
    }
#pragma unroll
    for (int j = 0; j < GL; ++j) {
      uint32_t hi[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t x = j == 0 ? e[u][0] : __builtin_amdgcn_alignbit(e[u][0], e[u][1], q[u]);
        hi[u] = lds_u32_nowait(((x >> SH) & amask) | cbase);  // the count entry (or the write entry's high word)
      }
      lds_wait(hi);
      if constexpr (FB) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if ((hi[u] & 31u) == 0u) {  // a codeword longer than the table: one codeword, start bit 0
            const uint32_t x = j == 0 ? e[u][0] : __builtin_amdgcn_alignbit(e[u][0], e[u][1], q[u]);
            const uint32_t y = j == 0 ? e[u][1] : __builtin_amdgcn_alignbit(e[u][1], e[u][2], q[u]);
            hi[u] = (mt_canon(fb, x, y, Sc) & 31u) | (1u << 16);
          }
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        uint32_t m;
        asm("v_and_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD"
            : "=v"(m) : "v"(hi[u]), "v"(rm[u]));
        cnt[u] = __builtin_popcount(m) + cnt[u];
        asm("v_lshrrev_b32 %0, %1, %0" : "+v"(rm[u]) : "v"(hi[u]));  // rm >>= b (low 5 bits)
        q[u] -= hi[u];  // low 5 bits: 32 - bits consumed in the group (b <= 12, GL * 12 < 32)
      }
    }
    bool more = false;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      win_shift5(e[u], q[u]);
      R[u] += (int)(q[u] & 31u) - 32;
      more |= R[u] > 0;
    }
    if (!__any(more)) break;
  }
}

// Write pass: the n[u] codewords of each segment to LDS bytes [o[u], o[u] + n[u]) (then
// the head stores, above).  A chain with n = 0 writes nothing.
template <int U, int GL, bool FB = false, int SH = 0>
__device__ __forceinline__ void mt_write(uint32_t (&e)[U][5], const uint32_t (&o)[U], const uint32_t (&n)[U],
                                         uint32_t amask, uint32_t wbase, const MtFb& fb = MtFb{}, uint32_t Sw = 0) {
  uint32_t ptr[U], end[U], head[U];
  uint32_t alo[U], ahi[U], fill[U], dptr[U];  // (GH_MT_WOR 2) pending bytes, their count, dword address
  int rem[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    ptr[u] = o[u];
    end[u] = o[u] + n[u];
    head[u] = 0;
    alo[u] = 0;
    ahi[u] = 0;
    fill[u] = o[u] & 3u;
    dptr[u] = o[u] & ~3u;
    rem[u] = (int)n[u];
  }
  auto group = [&](auto first) {
    constexpr int L0 = decltype(first)::value;  // index of the group's first lookup (< 4: head bytes), or 4
    uint32_t q[U];
#pragma unroll
    for (int u = 0; u < U; ++u) q[u] = 32u;
#pragma unroll
    for (int j = 0; j < GL; ++j) {
      uint2 ent[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t x = j == 0 ? e[u][0] : __builtin_amdgcn_alignbit(e[u][0], e[u][1], q[u]);
        ent[u] = lds_u64_nowait(((x >> SH) & amask) | wbase);
      }
      lds_wait(ent);
      if constexpr (FB) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if ((ent[u].y & 0x700u) == 0u) {  // n = 0: a codeword longer than the table
            const uint32_t x = j == 0 ? e[u][0] : __builtin_amdgcn_alignbit(e[u][0], e[u][1], q[u]);
            const uint32_t y = j == 0 ? e[u][1] : __builtin_amdgcn_alignbit(e[u][1], e[u][2], q[u]);
            const uint32_t r = mt_canon(fb, x, y, Sw);
            ent[u] = make_uint2(r >> 8, (r & 31u) | (1u << 8));
          }
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (GH_MT_WOR == 2) {
          // gather into the pending dword (bytes [fill, fill + n)), OR it at its aligned
          // address (again as it fills up: ORing the same bytes twice is harmless), move on
          // once it is complete; a finished segment ORs zero
          const bool on = rem[u] > 0;
          const unsigned long long d = (unsigned long long)(on ? ent[u].x : 0u) << (fill[u] << 3);
          alo[u] |= (uint32_t)d;
          ahi[u] |= (uint32_t)(d >> 32);
          asm volatile("ds_or_b32 %0, %1" ::"v"(dptr[u]), "v"(alo[u]) : "memory");
          const uint32_t nn = on ? __builtin_amdgcn_ubfe(ent[u].y, 8, 3) : 0u;
          rem[u] -= (int)nn;
          fill[u] += nn;
          const bool adv = fill[u] >= 4u;
          dptr[u] += adv ? 4u : 0u;
          alo[u] = adv ? ahi[u] : alo[u];
          ahi[u] = adv ? 0u : ahi[u];
          fill[u] -= adv ? 4u : 0u;
        } else if (GH_MT_WOR) {
          // OR the four bytes into the two aligned dwords they span (zeroed staging; a
          // finished segment ORs zero at its end)
          const bool on = ptr[u] < end[u];
          const uint32_t a = on ? ptr[u] : end[u];
          const unsigned long long d = (unsigned long long)(on ? ent[u].x : 0u) << ((a & 3u) << 3);
          asm volatile("ds_or_b32 %0, %1\n\tds_or_b32 %0, %2 offset:4" ::"v"(a & ~3u), "v"((uint32_t)d),
                       "v"((uint32_t)(d >> 32)) : "memory");
        } else {
          // unaligned (gfx950 LDS runs in unaligned mode); a finished segment keeps
          // writing at its end, over the next segment's head (restored below)
          lds_st32(min(ptr[u], end[u]), ent[u].x);
        }
        if (GH_MT_WOR) {
        } else if (L0 + j == 0) {  // (constants once unrolled)
          head[u] = ent[u].x;
        } else if (L0 + j < 4) {
          const uint32_t pos = ptr[u] - o[u];  // bytes so far (>= L0 + j)
          head[u] = pos < 4u ? head[u] | (ent[u].x << (8u * pos)) : head[u];
        }
        ptr[u] = add_n(ptr[u], ent[u].y);
        q[u] -= ent[u].y;
      }
    }
    bool more = false;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      win_shift5(e[u], q[u]);
      more |= GH_MT_WOR == 2 ? rem[u] > 0 : ptr[u] < end[u];
    }
    return more;
  };
  // the first groups carry the head bytes (static lookup indices), the rest loop
  bool more = group(std::integral_constant<int, 0>{});
  if (GL < 4) more = group(std::integral_constant<int, GL>{}) || more;  // lookups GL.. 2GL-1 >= 3
  if (__any(more)) {
    for (int g = 0; g < MT_GMAX; ++g) {
      if (!__any(group(std::integral_constant<int, 4>{}))) break;
    }
  }
  // every lane's lookups are done: the head bytes over the previous segment's overrun
  // and end writes (in wave order: after them); (GH_MT_WOR 2) the pending dword a last
  // lookup moved past
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if (!GH_MT_WOR && n[u]) lds_st32(o[u], head[u]);
    if (GH_MT_WOR == 2) asm volatile("ds_or_b32 %0, %1" ::"v"(dptr[u]), "v"(alo[u]) : "memory");
  }
}

// Zero the staging a write pass ORed into: piece bytes [0, n) and the last lookups'
// overrun (the last lookup ORs two dwords: < 8 bytes past), i.e. region chunks [1, ce).  LDS operations
// of a wave complete in order: after the copy-out's reads.
__device__ __forceinline__ void mt_zero(uint32_t region, uint32_t n, int lane) {
  const uint32_t ce = (STAGE_PAD + n + 8u + 15u) >> 4;
  for (uint32_t c = 1u + (uint32_t)lane; c < ce; c += 64u)
    asm volatile("ds_write_b128 %0, %1" ::"v"(region + 16u * c), "v"(tile_v4u{0, 0, 0, 0}) : "memory");
}

template <int TB, int GL, int NS, bool FB = false, int NP = 1>
__global__ __launch_bounds__(TB) __attribute__((amdgpu_waves_per_eu(4, 4))) void gh_mtile_kernel(const TileParams p) {
  constexpr int U = MT_U;
  constexpr int NW = TB / 64;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t stage_lds = p.lut_bytes;                                  // [NW] regions
  uint32_t* s_tot = (uint32_t*)(smem + p.lut_bytes + NW * p.stage_bytes);  // [SLOTS][NW] wave totals
  uint32_t* s_off = s_tot + TILE_SLOTS * NW;                               // [SLOTS][NW] wave offsets
  uint32_t* s_cnt = s_off + TILE_SLOTS * NW;                               // [SLOTS] arrivals
  unsigned long long* s_pfx = (unsigned long long*)(s_cnt + TILE_SLOTS);  // [SLOTS] prefixes
  uint32_t* s_ptile = (uint32_t*)(s_pfx + TILE_SLOTS);                     // [SLOTS] their tiles
  uint32_t* s_lead = s_ptile + TILE_SLOTS;                                 // [NW] (leader)
  const uint32_t cnt_lds = (uint32_t)((uint8_t*)s_cnt - smem);
  const uint32_t ptile_lds = (uint32_t)((uint8_t*)s_ptile - smem);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const uint32_t D = gridDim.x - 1;
  if (blockIdx.x == 0) {
    tile_round_leader<TB>(p, D, s_lead, tid, lane, wid);
    return;
  }
  {  // LUT to LDS (u64 entries, one copy); zeroed staging regions
    const uint4* g = (const uint4*)p.lut;
    uint4* s4 = (uint4*)smem;
    for (uint32_t i = tid; i < p.lut_bytes / 16; i += TB) s4[i] = g[i];
    for (uint32_t i = tid; i < NW * p.stage_bytes / 16; i += TB) s4[p.lut_bytes / 16 + i] = make_uint4(0, 0, 0, 0);
    if (tid < TILE_SLOTS) {
      s_cnt[tid] = 0;
      s_ptile[tid] = 0xFFFFFFFFu;
    }
  }
  // (FB, NP = 2: 11-bit tables on windows of S = 17, the lookups shifted down: a window
  // holds segment bits start - S .. start - S + 159, and a 16-bit codeword at bit 127
  // ends at bit 142, so S <= 17 for the fallback to see all its bits)
  constexpr int WSH = (FB && NP == 2) ? 1 : 0, CSH = (FB && NP == 2) ? 2 : 0;
  const uint32_t S = 29u - p.kbits - WSH;                  // write pass: u64 entries
  const uint32_t amask = ((1u << p.kbits) - 1u) << 3;
  // count pass: its own u32 table of width Kc (GH_MT_CLUT), the larger of the two
  // tables first so that each base ORs into its table's addresses; or the write table's
  // high words
  const uint32_t Kc = GH_MT_CLUT ? p.kbits_c : p.kbits;
  // (the count table in 2^lgr copies, lane l reading copy l mod 2^lgr: lgr = 0 by default)
  const uint32_t Sc = GH_MT_CLUT ? 30u - Kc - CSH - p.lgr : S;
  const uint32_t amask_c = GH_MT_CLUT ? ((1u << Kc) - 1u) << (2u + p.lgr) : amask;
  const uint32_t cbytes = 4u << (Kc + p.lgr);
  const bool cfirst = GH_MT_CLUT && cbytes > (8u << p.kbits);
  const uint32_t cbase = (!GH_MT_CLUT ? 4u : cfirst ? 0u : 8u << p.kbits) | (((uint32_t)lane & ((1u << p.lgr) - 1u)) << 2);
  const uint32_t wbase = cfirst ? cbytes : 0u;
  // (FB) the canonical tables: the last FB_BYTES of the LUT area
  const MtFb fb{(const uint32_t*)(smem + p.lut_bytes - (FB ? FB_BYTES : 0)), p.kbits + 1u, p.fb_hi};
  check_lds_base(smem, p.status);
  const uint32_t G = D, b = blockIdx.x - 1;
  const uint32_t nseg = (uint32_t)p.nseg;
  constexpr uint32_t NONE = 0xFFFFFFFFu;
  __syncthreads();  // the LUT and the counters (the last barrier of a decoding workgroup)
  const uint32_t last_tile_k = b < p.ntiles ? (p.ntiles - 1 - b) / G : NONE;
  uint32_t cur = b, nxt = b + G;
  const uint32_t lseg = (uint32_t)(wid * 64 * U + lane);
  uint4 w[U];
  uint32_t w4[U], gw[U];
  auto load = [&](uint32_t t) {
    const uint32_t seg0 = min(t, p.ntiles - 1) * (uint32_t)(U * TB) + lseg;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t sc = min(seg0 + (uint32_t)(64 * u), nseg - 1);
      // nontemporal: read once (and not merged with the look-ahead dword into an
      // overlapping load, which left register copies and a vmcnt wait at the loop's back edge)
      const tile_v4u v = __builtin_nontemporal_load((const tile_v4u*)(p.payload + 4ull * sc));
      w[u] = make_uint4(v.x, v.y, v.z, v.w);
      w4[u] = p.payload[4ull * sc + 4];
      gw[u] = p.gaps[(p.gap_nib0 + (sc ? sc - 1u : 0u)) >> 3];
    }
  };
  load(cur);
  {  // as many stores after these loads as every iteration issues after its prefetch
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(p.out, 0, 0x7FFFFFF0, 0x00020000);
#pragma unroll
    for (int i = 0; i < NS * NP; ++i) __builtin_amdgcn_raw_buffer_store_b128(tile_v4u{0, 0, 0, 0}, rs, (int)(OOB_OFF + 16u * (uint32_t)i), 0, 2);  // (distinct: not merged)
#pragma unroll
    for (int i = 0; i < NP; ++i) __builtin_amdgcn_raw_buffer_store_b8((uint8_t)0, rs, (int)(OOB_OFF + 16u * (uint32_t)i), 0, 2);
  }
  if (cur >= p.ntiles) cur = NONE;
  // tiles k-1 .. k-LAG, held for their write pass: e-windows, the segments' offsets in
  // the wave's piece and counts, the piece's length
  constexpr int L = MT_LAG;
  uint32_t th[L], he[L][U][5], hpos[L][U], hcnt[L][U], htot[L];
#pragma unroll
  for (int i2 = 0; i2 < L; ++i2) {
    th[i2] = NONE;
    htot[i2] = 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      hpos[i2][u] = 0;
      hcnt[i2][u] = 0;
#pragma unroll
      for (int i = 0; i < 5; ++i) he[i2][u][i] = 0;
    }
  }
  uint32_t rank = 0;
  const uint32_t region = stage_lds + (uint32_t)wid * p.stage_bytes;
  const uint32_t piece_cap = p.stage_bytes - (uint32_t)(STAGE_PAD + 8);
  for (uint32_t k = 0;; ++k) {
    const bool have_cur = cur < p.ntiles;
    const uint32_t t2 = th[L - 1];  // the tile written and copied out this iteration
    const bool have2 = t2 < p.ntiles;
    bool pending = have_cur;
#pragma unroll
    for (int i2 = 0; i2 < L; ++i2) pending |= th[i2] < p.ntiles;
    if (!pending) break;
    if (last_tile_k != NONE && k > last_tile_k + L + 3) {  // cannot happen; never hang the GPU
      if (lane == 0) atomicOr(p.status, (unsigned)GH_ST_TIMEOUT);
      break;
    }
    const uint32_t slot = k % TILE_SLOTS, slot2 = (k + TILE_SLOTS - L) % TILE_SLOTS;
    if (rank >= 3) __builtin_amdgcn_s_setprio(3);
    else if (rank == 2) __builtin_amdgcn_s_setprio(2);
    else if (rank == 1) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
    unsigned long long* const pf2 = &p.prefix[have2 ? t2 : 0u];
    const unsigned long long gp0 = __hip_atomic_load(pf2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // ---- count pass over tile k ---------------------------------------------------------
    const uint32_t seg0 = cur * (uint32_t)(U * TB) + lseg;
    uint32_t e[U][5], ce[U][5], cnt[U];
    {
      int R[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t seg = seg0 + (uint32_t)(64 * u);
        const bool act = have_cur && seg < nseg;
        const int start = seg == 0 ? (int)p.first_start : (int)gap_nib(gw[u], p.gap_nib0 + seg - 1u);
        R[u] = act ? 128 - start : 0;
        make_ewin(w[u], w4[u], start, S, ce[u]);  // held for the write pass
        if (GH_MT_CLUT) {
          make_ewin(w[u], w4[u], start, Sc, e[u]);
        } else {
#pragma unroll
          for (int i = 0; i < 5; ++i) e[u][i] = ce[u][i];
        }
      }
      if (GH_MT_ABLATE & 1) {
#pragma unroll
        for (int u = 0; u < U; ++u) cnt[u] = R[u] > 0 ? 40u : 0u;
      } else {
        mt_count<U, GL, FB, CSH>(e, R, cnt, amask_c, cbase, fb, Sc);
      }
    }
    const unsigned long long gp = __hip_atomic_load(pf2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    load(nxt);
    // ---- wave scans, arrival at tile k (gh_tile.hip) -------------------------------------
    uint32_t bpos[U], wave_tot = 0;
#pragma unroll
    for (int u = 0; u < U; ++u) bpos[u] = wave_incl_scan(cnt[u]);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t ct = (uint32_t)__builtin_amdgcn_readlane((int)bpos[u], 63);
      bpos[u] += wave_tot - cnt[u];
      wave_tot += ct;
    }
    if (have_cur) {
      uint32_t old = 0;
      if (lane == 0) {
        s_tot[slot * NW + wid] = wave_tot;
        asm volatile("ds_add_rtn_u32 %0, %1, %2\n\ts_waitcnt lgkmcnt(0)" : "=v"(old) : "v"(cnt_lds + 4u * slot), "v"(1u)
                     : "memory");
      }
      const uint32_t arr = (uint32_t)__builtin_amdgcn_readfirstlane((int)old);
      rank = (4u * arr) / NW;
      if (arr == NW - 1) {
        const uint32_t x = lane < NW ? s_tot[slot * NW + lane] : 0u;
        const uint32_t xi = wave_incl_scan(x);
        if (lane < NW) s_off[slot * NW + lane] = xi - x;
        const uint32_t tile_total = (uint32_t)__builtin_amdgcn_readlane((int)xi, NW - 1);
        if (lane == 0) {
          s_cnt[slot] = 0;
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          __hip_atomic_store(&p.granules[cur], granule(p.epoch, 1, tile_total), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    }
    // ---- write pass of tile k-1 into the wave's region (local offsets: no prefix needed)
    const uint32_t wtot = htot[L - 1];
    const bool fits = GH_MT_NOFB ? true : wtot <= piece_cap;
    if (have2 && fits && !(GH_MT_ABLATE & 2)) {
      uint32_t o[U];
#pragma unroll
      for (int u = 0; u < U; ++u) o[u] = region + STAGE_PAD + hpos[L - 1][u];
      mt_write<U, GL, FB, WSH>(he[L - 1], o, hcnt[L - 1], amask, wbase, fb, S);
    }
    // ---- the prefix of tile k-1 -> this wave's piece's output offset (gh_tile.hip) --------
    unsigned long long goff = 0;
    uint32_t n2 = 0;
    bool got = true;
    if (have2 && (GH_MT_ABLATE & 4)) {
      goff = ((unsigned long long)t2 * (U * TB * 40) + (uint32_t)wid * (U * 64 * 40)) % (p.out_cap - (U * TB * 64));
      n2 = (uint32_t)min<unsigned long long>(wtot, p.out_cap - goff);
    } else if (have2) {
      unsigned long long g = rfl_u64(gp0);
      if (!granule_ok(p, g, 2)) {
        g = rfl_u64(gp);
        if (!granule_ok(p, g, 2)) {
          if (wid == 0 && lane == 0) atomicAdd(p.stats, 1ull);
          unsigned long long t0w = 0;
          for (uint32_t spins = 1;; ++spins) {
            if (lds_ld_u32(ptile_lds + 4u * slot2) == t2) {
              asm volatile("" ::: "memory");
              g = s_pfx[slot2];
              break;
            }
            g = rfl_u64(__hip_atomic_load(pf2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            if (granule_ok(p, g, 2)) {
              if (lane == 0) {
                s_pfx[slot2] = g;
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                lds_st_u32(ptile_lds + 4u * slot2, t2);
              }
              break;
            }
            if ((spins & 63u) == 0u) {
              if (__hip_atomic_load(p.status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & GH_ST_TIMEOUT) break;
              const unsigned long long t = wall_clock64();
              if (t0w == 0) {
                t0w = t;
              } else if (t - t0w > 400000000ull) {
                if (lane == 0) atomicOr(p.status, (unsigned)GH_ST_TIMEOUT);
                break;
              }
            }
            __builtin_amdgcn_s_sleep(1);
          }
          got = granule_ok(p, g, 2);
        }
      }
      asm volatile("" ::: "memory");
      goff = (g & GRAN_VMASK) + s_off[slot2 * NW + wid];
      if (wid == NW - 1 && t2 == p.ntiles - 1 && got && lane == 0) *p.total = goff + wtot;
      n2 = (!got || goff >= p.out_cap) ? 0u : (uint32_t)min<unsigned long long>(wtot, p.out_cap - goff);
    }
    // ---- copy-out ---------------------------------------------------------------------------
    if (fits) {
#pragma unroll
      for (int part = 0; part < NP; ++part) {  // (NP parts of 64 * NS chunks: pieces of up to 8 KB)
        tile_v4u cv[NS];
        uint32_t cb;
        copy_out_piece<NS, false>(p.out, region, goff, n2, lane, cv, cb, 64u * NS * (uint32_t)part);  // fixed store count
      }
      if (GH_MT_WOR) mt_zero(region, wtot, lane);
    } else {
      // a piece larger than the region (data whose shortest codewords cluster): one chain
      // at a time (a chain's worst case fits), then drain (rare path)
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t c0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)hpos[L - 1][u]);  // chain u's first byte
        const uint32_t ct = (u + 1 < U ? (uint32_t)__builtin_amdgcn_readfirstlane((int)hpos[L - 1][u + 1 < U ? u + 1 : u])
                                       : wtot) - c0;
        uint32_t o[U], nn[U];
#pragma unroll
        for (int v = 0; v < U; ++v) {
          // the other chains write nothing of theirs: their (branch-free) stores go to
          // the region's pad, before piece byte 0
          o[v] = v == u ? region + STAGE_PAD + (hpos[L - 1][v] - c0) : region;
          nn[v] = v == u ? hcnt[L - 1][v] : 0u;
        }
        uint32_t ew[U][5];
#pragma unroll
        for (int v = 0; v < U; ++v)
#pragma unroll
          for (int i = 0; i < 5; ++i) ew[v][i] = he[L - 1][v][i];
        mt_write<U, GL, FB, WSH>(ew, o, nn, amask, wbase, fb, S);
        const unsigned long long gu = goff + c0;
        const uint32_t nu = (!got || gu >= p.out_cap) ? 0u : (uint32_t)min<unsigned long long>(ct, p.out_cap - gu);
#pragma unroll
        for (int part = 0; part < NP; ++part) {
          tile_v4u cv[NS];
          uint32_t cb;
          copy_out_piece<NS, false>(p.out, region, gu, nu, lane, cv, cb, 64u * NS * (uint32_t)part);
        }
        if (GH_MT_WOR) mt_zero(region, ct, lane);
      }
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    }
    // ---- hold tile k for its write pass -----------------------------------------------------
#pragma unroll
    for (int i2 = L - 1; i2 > 0; --i2) {
      th[i2] = th[i2 - 1];
      htot[i2] = htot[i2 - 1];
#pragma unroll
      for (int u = 0; u < U; ++u) {
#pragma unroll
        for (int i = 0; i < 5; ++i) he[i2][u][i] = he[i2 - 1][u][i];
        hpos[i2][u] = hpos[i2 - 1][u];
        hcnt[i2][u] = hcnt[i2 - 1][u];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int i = 0; i < 5; ++i) he[0][u][i] = ce[u][i];
      hpos[0][u] = bpos[u];
      hcnt[0][u] = cnt[u];
    }
    htot[0] = have_cur ? wave_tot : 0u;
    th[0] = have_cur ? cur : NONE;
    cur = nxt < p.ntiles ? nxt : NONE;
    nxt += G;
  }
}
