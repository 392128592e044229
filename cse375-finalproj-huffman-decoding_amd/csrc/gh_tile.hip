// Tile kernel: the decode of grouped codes (complete, 3 <= len <= 12, e.g. BASELINE's
// r = 0.1 and r = 0.5 data), included by gh_decode.hip.  Reference counterpart:
// gpu_dec_l1_l2 (decoder/src/decoder.cu:454-730) — its per-segment count (:529-569),
// decoupled look-back (:571-653) and second decode that writes the bytes (:655-728) — as
// ONE decode pass per segment in one persistent kernel.
//
// 1024-thread workgroups (16 waves), U segments per lane, a tile = U * 1024 consecutive
// segments; wave w of a workgroup owns the 64 * U consecutive segments [64Uw, 64U(w+1))
// of its tile, lane l the segments 64Uw + Ul .. 64Uw + Ul + U - 1 (lane-major,
// GH_TILE_LMAJ; chain u of lane l is segment 64Uw + Ul + u).  Workgroup 0 is the round
// leader; the D = grid - 1 others decode: workgroup b takes tiles b, b + D, b + 2D, ...
// (static round robin; grid <= 2048).  Iteration k of a decoding workgroup, every wave
// on its own (no workgroup barrier after the prologue):
//
//   decode tile k into registers (one codeword per lookup, G codewords per window shift;
//     a codeword is kept iff it starts before the segment end: the reference's rule)
//     - mid-decode: load the global prefix of tile k-LAG
//   copy tile k-LAG out of the wave's staging buffer (its prefix has had LAG-1 iterations
//     to arrive) with a fixed store count, reading aligned 16-byte LDS chunk pairs and
//     shifting them in registers; the next tile's loads are issued just before
//   wave scan of the counts -> the wave's total to LDS, an LDS arrival counter; the last
//     wave to arrive scans the 16 totals and publishes tile k's aggregate
//   stage tile k: every wave writes its own 64U segments into its own buffer; a tile
//     larger than staging waits for its prefix and stores its bytes from registers
//
// The leader takes the rounds (tiles rD .. rD + D - 1) in order: it waits for a round's
// aggregates, scans them and publishes every tile's global exclusive prefix.  The start
// of the next round stays in its registers, so the serial chain of round starts never
// crosses workgroups (rotating the leader role among the decoding workgroups made every
// round pay one cross-workgroup hand-off on that chain: 0.73 vs 0.70 ms on cfg4).
//
// Issue priority by arrival rank: the waves that arrived last at their previous tile gate
// the next aggregate, so they take priority 3, the first arrivals 0.
//
// Every alternative of the round-3/4 build knobs (copy-out interleaving, batched reads,
// early loads, ticket schedules, priority rotations, ...) measured slower and was removed
// (tile-kernel section).  Diagnostic builds only: GH_TILE_STAMPS, GH_TILE_ABLATE.

#ifndef GH_TILE_TB
#define GH_TILE_TB 1024
#endif
constexpr int TILE_TB = GH_TILE_TB;  // threads per workgroup
#ifndef GH_TILE_U
#define GH_TILE_U 3
#endif
constexpr int TILE_U = GH_TILE_U;  // segments per lane, codes of >= 4-bit codewords
constexpr int TILE_U3 = 2;    // segments per lane, codes with 3-bit codewords
constexpr int TILE_NS = 4;    // 16-byte stores per lane per copy-out (NS * 64 chunks cover a wave's piece)
constexpr int TILE_SCAP = 20; // staging bytes per segment, codes of >= 4-bit codewords
constexpr int TILE_MIDG = 2;  // decode group after which the prefix of tile k-LAG is loaded (again)
constexpr int STAGE_PAD = 16; // region byte STAGE_PAD + i = piece byte i
#ifndef GH_TILE_LAG
#define GH_TILE_LAG 2
#endif
constexpr int TILE_LAG = GH_TILE_LAG;  // a tile is copied out LAG iterations after it is decoded (LAG buffers)
constexpr int TILE_SLOTS = 16;  // per-tile wave totals / offsets / arrival counters / prefixes in LDS, by k mod 16
#ifndef GH_TILE_STAMPS
#define GH_TILE_STAMPS 0  // diagnostic builds only: per-phase s_memtime deltas of waves 0 and 4
#endif
#if GH_TILE_STAMPS
#define TSTAMP(i) (ts[i] = __builtin_amdgcn_s_memtime())
#else
#define TSTAMP(i) ((void)0)
#endif
#ifndef GH_TILE_CSUB
#define GH_TILE_CSUB 0  // the decode step's borrow count in C (the compiler's own hazard padding)
#endif
#ifndef GH_TILE_CLDS
#define GH_TILE_CLDS 0  // the decode's LUT reads as plain LDS loads (the compiler's own lgkmcnt waits)
#endif
#ifndef GH_TILE_LMAJ
#define GH_TILE_LMAJ 1  // lane-major segments: lane l of a wave decodes its segments U*l .. U*l + U - 1
#endif
#ifndef GH_TILE_POLLDIV
#define GH_TILE_POLLDIV 1  // a waiting wave re-polls the prefix granule every N-th spin (staggered by wave)
#endif
#ifndef GH_TILE_DYN
#define GH_TILE_DYN 0  // tiles by ticket (one counter per launch parity) and a frontier leader
#endif
constexpr int TILE_TAHEAD = 5;  // (GH_TILE_DYN) a tile index is posted this many iterations ahead
#ifndef GH_TILE_LATEP
#define GH_TILE_LATEP 0  // a third prefix load right before the prefetch (see the loop)
#endif
#ifndef GH_TILE_EPERM
#define GH_TILE_EPERM 0  // symbols placed into the output words as they are decoded (register peak)
#endif
#ifndef GH_TILE_HOLD
#define GH_TILE_HOLD 0  // a decoded tile is held in registers one iteration and staged the next:
                        // copy-out three iterations after the decode with two staging buffers
#endif
#ifndef GH_TILE_ALRD
#define GH_TILE_ALRD 1  // copy-out: aligned LDS reads realigned in registers (see copy_out_piece)
#endif
#ifndef GH_TILE_W2
#define GH_TILE_W2 0  // staging rounds in dword pairs (ds_write2_b32)
#endif
#ifndef GH_TILE_PF2
#define GH_TILE_PF2 0  // the tile after next prefetched (two register sets, the loop body unrolled twice)
#endif
#ifndef GH_TILE_ABLATE
#define GH_TILE_ABLATE 0  // diagnostic builds only (make variant), bits: 1 no decode, 2 no staging
                          // stores, 4 no prefix wait (a fake offset), 8 no copy-out, 16 even LUT
                          // entries only (no LUT bank conflicts), 32 pieces copied out to 16-byte
                          // aligned offsets (wrong output)
#endif
typedef unsigned int tile_v4u __attribute__((ext_vector_type(4)));
// 16-byte global store of the copy-out: streaming (the output is never re-read, so it
// should not displace the payload lines in L2; cfg4 0.574-0.579 vs 0.578-0.588 ms)
__device__ __forceinline__ void tile_st16(uint4* d, const uint4& v) {
  __builtin_nontemporal_store(tile_v4u{v.x, v.y, v.z, v.w}, (tile_v4u*)d);
}

struct TileParams {
  const uint32_t* payload;       // local segment j owns words [4j, 4j+4); +1 look-ahead, zero padded
  const uint32_t* gaps;          // gap words; nibble (gap_nib0 + j - 1) = start of local segment j>=1
  const uint32_t* lut;           // 2^K u32 {len | sym << 8 | len << 23}
  uint8_t* out;
  unsigned long long* granules;  // one per tile: its symbol count (flag 1)
  unsigned long long* prefix;    // one per tile: its global exclusive prefix (flag 2, by the leader)
  unsigned int* status;
  unsigned long long* total;
  unsigned long long* stats;     // poll counters (reported as slow_lookbacks)
  unsigned long long out_cap;
  unsigned long long nseg;
  unsigned int gap_nib0, first_start, ntiles, kbits, lgr, epoch;
  unsigned int lut_bytes;        // LUT bytes in LDS (replicated: 4 << (K + lgr))
  unsigned int idle_block;       // a block that exits at once (>= grid: none)
  unsigned int stage_bytes;      // one wave's staging region (16 + its piece + margin, a multiple of 16)
  unsigned int kbits_c;          // (gh_mtile.hip) the count table's width
  unsigned int fb_hi;            // (gh_mtile.hip, codes longer than the tables) the longest codeword
  unsigned int* tickets;         // (GH_TILE_DYN) tile counters by launch parity, 8 bytes apart
  uint4* stamps;                 // GH_TILE_STAMPS builds: [grid][2 waves][128 iterations][2] phase deltas
  unsigned long long* tstamps;   // GH_TILE_STAMPS builds: 100 MHz times: [ntiles] aggregate left, [ntiles]
                                 // prefix obtained by wave 0 (bit 63: polled), [rounds] round published
};

// LDS of the tile kernel: LUT, 2 x NW staging regions (one per wave and buffer), the
// per-tile wave totals, offsets and arrival counters (TILE_SLOTS tiles), leader wave totals.
// stage_bytes: one wave's region.
inline size_t tile_lds_bytes(size_t lut_bytes, size_t stage_bytes) {
  return lut_bytes + TILE_LAG * (TILE_TB / 64) * stage_bytes + TILE_SLOTS * (2 * (TILE_TB / 64) + 1) * 4 +
         TILE_SLOTS * 12 + 4 * (TILE_TB / 64) + 4 * TILE_SLOTS + 32;
}

// v_perm selector placing byte 1 of S0 (the symbol) at byte j, keeping S1's others.
__device__ __forceinline__ constexpr uint32_t perm_sel(int j) {
  return j == 0 ? 0x03020105u : j == 1 ? 0x03020500u : j == 2 ? 0x03050100u : 0x05020100u;
}

// e-window of a segment starting at bit `start` (0..15): e-stream bit 0 is segment
// bit start - S (bits before the segment read as 0); requires 16 <= S <= 31.  The
// lookup address of the codeword at window bit p is then
// alignbit(e0, e1, 32 - p) & (mask << (2 + lgr)) | lane_offset: two VALU ops.
__device__ __forceinline__ void make_ewin(uint4 w, uint32_t w4, int start, uint32_t S, uint32_t (&e)[5]) {
  const uint32_t r = S - (uint32_t)start;  // 1..31
  e[0] = __builtin_amdgcn_alignbit(0u, w.x, r);
  e[1] = __builtin_amdgcn_alignbit(w.x, w.y, r);
  e[2] = __builtin_amdgcn_alignbit(w.y, w.z, r);
  e[3] = __builtin_amdgcn_alignbit(w.z, w.w, r);
  e[4] = __builtin_amdgcn_alignbit(w.w, w4, r);
}

// Decode state of a segment, one register Q:
//   bits 0-7    32 - bits consumed in the current group (v_alignbit reads bits 0-4);
//   bits 8-22   symbol underflow room (the entries' symbol bytes are subtracted here);
//   bits 23-31  H = bits left before the segment end, minus 1 (9 bits).
// LUT entries are {len | sym << 8 | len << 23}, so Q -= entry advances both counters in
// one op, and its borrow is set exactly when H < len: at the codeword that reaches or
// crosses the segment end, the last one the reference keeps (it keeps a codeword iff it
// starts before the end).  The count is then the index of that codeword + 1 (one
// v_cndmask on the borrow).  Past it H has wrapped to >= 500 and stays above 127 (at most
// 32 x 12 more bits are subtracted), so no later codeword borrows; an inactive segment
// starts at H = 511.
constexpr uint32_t Q_SYMROOM = 0x7FFFu << 8;
constexpr uint32_t Q_LIVE = 128u << 23;  // Q below this: the next codeword is still kept
__device__ __forceinline__ uint32_t q_init(bool act, int start) {
  return ((act ? (uint32_t)(127 - start) : 511u) << 23) | Q_SYMROOM | 32u;
}

// Wait until at most N LDS operations of the wave are outstanding (they complete in
// order), tied to v so the compiler uses it only after the wait.
template <int N>
__device__ __forceinline__ void lds_wait_n(uint32_t& v) {
  static_assert(N >= 0 && N <= 3, "lgkmcnt 0..3");
  if constexpr (GH_TILE_CLDS) return;  // (the compiler's own waits for plain LDS loads)
  if constexpr (N == 0) asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v)::"memory");
  else if constexpr (N == 1) asm volatile("s_waitcnt lgkmcnt(1)" : "+v"(v)::"memory");
  else if constexpr (N == 2) asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(v)::"memory");
  else asm volatile("s_waitcnt lgkmcnt(3)" : "+v"(v)::"memory");
}

// Decode of U segments per lane on e-windows.  Each group decodes G codewords per chain
// from e0:e1 and then shifts the windows (G * maxlen <= 32, so the group's consumed bits
// fit Q's low byte).  Codeword j of a segment goes to byte j of ow (v_perm, static
// index); dead codewords go there too and are never staged.  `mid()` runs once, after
// group TILE_MIDG (NG > TILE_MIDG).  Returns the groups run (wave-uniform: the loop stops
// once no chain of the wave is live).  The chains' lookups roll: each chain waits only
// for its own read (a counted lgkmcnt: LDS reads of a wave complete in order) and issues
// its next one at once, so U reads stay in flight and a chain's step costs one LDS round
// trip plus its own few ops (round 5: cfg4 -0.7 %, cfg5 -2 % against the chains in
// lock-step, waiting for all U reads).  A chain shifts its window at its own group end;
// the early exit, after a group of every chain, drains the next group's U reads.
// Window trim: word k holds e-positions [C + 32k, +32) after a shift, C = the bits
// consumed so far >= (gi + 1) * G * MINL (no codeword is shorter than MINL bits).  A kept
// codeword starts before segment bit 128, e-position 127 - start + S, and its lookup reads
// K bits: nothing at e-position >= 157 - lgr - start is read for a kept codeword, so a
// word lying wholly at or above 157 is no longer shifted (its stale bits reach only such
// positions; dead codewords decode garbage, never counted).
template <int G, int U, int OW, int MINL, class Mid>
__device__ __forceinline__ int decode_tile_rolling(uint32_t (&e)[U][5], const int (&start)[U], const bool (&act)[U],
                                                   uint32_t (&ow)[U][OW], uint32_t (&cnt)[U], uint32_t amask,
                                                   uint32_t laneoff, Mid&& mid) {
  constexpr int S = 4 * OW;
  constexpr int NG = (S + G - 1) / G;
  // (four codewords per window shift: the deferred symbol placement kept too many entries
  // live and spilled; placed per group instead)
  constexpr int PLACE = GH_TILE_EPERM ? GH_TILE_EPERM : (G >= 4 ? 2 : 0);
  uint32_t q[U], ent[U];
#if GH_TILE_CLDS
  const __attribute__((address_space(3))) uint8_t* const lds0 = (const __attribute__((address_space(3))) uint8_t*)nullptr;
  auto lut_rd = [&](uint32_t a) -> uint32_t { return *(const __attribute__((address_space(3))) uint32_t*)(lds0 + a); };
#else
  auto lut_rd = [&](uint32_t a) -> uint32_t { return lds_u32_nowait(a); };
#endif
#pragma unroll
  for (int u = 0; u < U; ++u) {
    q[u] = q_init(act[u], start[u]);
    cnt[u] = 0;
#pragma unroll
    for (int k = 0; k < OW; ++k) asm volatile("" : "=v"(ow[u][k]));
  }
#pragma unroll
  for (int u = 0; u < U; ++u) ent[u] = lut_rd((e[u][0] & amask) | laneoff);
  int gdone = NG;
#pragma clang loop unroll(full)
  for (int gi = 0; gi < NG; ++gi) {
    const int CMIN = (gi + 1) * G * MINL;  // bits consumed by the end of this group, at least
    uint32_t qmin = 0xFFFFFFFFu;
#pragma clang loop unroll(full)
    for (int j = 0; j < G; ++j) {
      const int pos = gi * G + j;
      if (pos < S) {
        const bool gend = (j == G - 1) || (pos + 1 >= S);  // this chain's last codeword of the group
        const bool last = gend && gi + 1 >= NG;             // no read after it
#pragma clang loop unroll(full)
        for (int u = 0; u < U; ++u) {
          // outstanding: chains u.. of this codeword, and chains ..u-1's next reads
          if (last) {
            if constexpr (U == 3) {
              if (u == 0) lds_wait_n<2>(ent[u]);
              else if (u == 1) lds_wait_n<1>(ent[u]);
              else lds_wait_n<0>(ent[u]);
            } else if constexpr (U == 2) {
              if (u == 0) lds_wait_n<1>(ent[u]);
              else lds_wait_n<0>(ent[u]);
            } else {
              lds_wait_n<0>(ent[u]);
            }
          } else {
            lds_wait_n<U - 1>(ent[u]);
          }
#if GH_TILE_CSUB
          {
            uint32_t nq;
            const bool br = __builtin_sub_overflow(q[u], ent[u], &nq);
            q[u] = nq;
            cnt[u] = br ? (uint32_t)(pos + 1) : cnt[u];
          }
#else
          asm("v_sub_co_u32 %0, vcc, %0, %2\n\t"
              "v_cndmask_b32_e64 %1, %1, %3, vcc"
              : "+v"(q[u]), "+v"(cnt[u]) : "v"(ent[u]), "i"(pos + 1) : "vcc");
#endif
          ow[u][pos >> 2] = __builtin_amdgcn_perm(ent[u], ow[u][pos >> 2], perm_sel(pos & 3));
          // (GH_TILE_EPERM) place the symbol now: the compiler otherwise keeps every entry
          // live until the staging, ~60 VGPRs at the decode's peak
          if (PLACE == 1) asm volatile("" : "+v"(ow[u][pos >> 2]));
          if (!gend) {
            const uint32_t x = __builtin_amdgcn_alignbit(e[u][0], e[u][1], q[u]);
            ent[u] = lut_rd((x & amask) | laneoff);
          } else {
            // window shift (the trim of words no kept codeword reads: above)
            e[u][0] = __builtin_amdgcn_alignbit(e[u][0], e[u][1], q[u]);
            if (CMIN + 32 < 157) e[u][1] = __builtin_amdgcn_alignbit(e[u][1], e[u][2], q[u]);
            if (CMIN + 64 < 157) e[u][2] = __builtin_amdgcn_alignbit(e[u][2], e[u][3], q[u]);
            if (CMIN + 96 < 157) e[u][3] = __builtin_amdgcn_alignbit(e[u][3], e[u][4], q[u]);
            if (CMIN + 128 < 157) e[u][4] = __builtin_amdgcn_alignbit(e[u][4], 0u, q[u]);
            q[u] = (q[u] & 0xFFFFFF00u) | 32u;
            qmin = min(qmin, q[u]);
            if (!last) ent[u] = lut_rd((e[u][0] & amask) | laneoff);
          }
        }
      }
    }
    if (PLACE == 2) {  // this group's symbols placed by its end
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int w0 = (gi * G) >> 2, w1 = min(OW - 1, (gi * G + G - 1) >> 2);
#pragma unroll
        for (int wi = w0; wi <= w1; ++wi) asm volatile("" : "+v"(ow[u][wi]));
      }
    }
    if (gi == TILE_MIDG) mid();
    if (gi >= TILE_MIDG && gi + 1 < NG && !__any(qmin < Q_LIVE)) {
      // the next group's reads are in flight: drain them
#pragma unroll
      for (int u = 0; u < U; ++u) lds_wait_n<0>(ent[u]);
      gdone = gi + 1;
      break;
    }
  }
  return gdone;
}

// LDS store at an absolute byte address plus a constant offset (the instruction's
// offset field).
template <int OFF = 0>
__device__ __forceinline__ void lds_st32(uint32_t a, uint32_t v) {
  asm volatile("ds_write_b32 %0, %1 offset:%2" ::"v"(a), "v"(v), "i"(OFF) : "memory");
}
// A waited LDS read / write at an absolute byte address (hand-offs between waves).
__device__ __forceinline__ uint32_t lds_ld_u32(uint32_t a) {
  uint32_t v;
  asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a) : "memory");
  return v;
}
__device__ __forceinline__ void lds_st_u32(uint32_t a, uint32_t v) {
  asm volatile("ds_write_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" ::"v"(a), "v"(v) : "memory");
}
// ... with the offset 4m, m a constant of the unrolled caller (1..12)
__device__ __forceinline__ void lds_st32_m(uint32_t a, uint32_t v, int m) {
  switch (m) {
    case 1: lds_st32<4>(a, v); break;
    case 2: lds_st32<8>(a, v); break;
    case 3: lds_st32<12>(a, v); break;
    case 4: lds_st32<16>(a, v); break;
    case 5: lds_st32<20>(a, v); break;
    case 6: lds_st32<24>(a, v); break;
    case 7: lds_st32<28>(a, v); break;
    case 8: lds_st32<32>(a, v); break;
    case 9: lds_st32<36>(a, v); break;
    case 10: lds_st32<40>(a, v); break;
    case 11: lds_st32<44>(a, v); break;
    default: lds_st32<0>(a + 4u * (uint32_t)m, v); break;
  }
}
// Staging of one wave's 64U consecutive segments into the wave's own region (chain u lane
// l = segment 64u + l of the wave, n[u] bytes from ow[u] at LDS byte o[u]; the first one
// at the region's 16-byte aligned start), with no other wave involved.
//
// A segment's bytes are realigned to the dwords they fall in: with ap = o - base in 1..4
// (base = o rounded down to a dword, minus 4 when o is aligned), dword m >= 1 at base + 4m
// holds segment bytes [4m - ap, +4).  Rounds m = mmax .. 1 store dword m of every segment
// unconditionally, chain by chain: a dword past a segment's end holds garbage, but it lies
// in the next one or two segments of the wave, which store that address in a LATER round
// (their base is higher, so their m for it is lower; within a round a segment's dwords
// differ from the others').  LDS operations of a wave complete in order, so the last
// store to every address is the one of the last segment that starts before it: the right
// bytes, except in each segment's first dword (base, when ap < 4), which holds the
// previous segment's tail followed by garbage.  Each segment then reads that dword back
// and puts its head bytes over the garbage (read-modify-write, in order again).  Garbage
// past the wave's last segment lands in the region's margin.  (Rounds 2-4: aligned stores
// under exec masks, a second workgroup barrier and head bytes after it: ~36 VALU and ~21
// SALU per segment.)
template <int U, int OW>
__device__ __forceinline__ void stage_wave(const uint32_t (&ow)[U][OW], const uint32_t (&n)[U], const uint32_t (&o)[U],
                                           int mmax) {
  uint32_t base[U], sh[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint32_t ap = ((o[u] - 1u) & 3u) + 1u;
    base[u] = o[u] - ap;
    sh[u] = 4u - ap;  // v_alignbyte amount: dword m = bytes [4m - ap, +4) of the segment
  }
  auto dw = [&](int u, int m) { return __builtin_amdgcn_alignbyte(m < OW ? ow[u][m] : 0u, ow[u][m - 1], sh[u]); };
  if constexpr (GH_TILE_W2) {
    // dwords m and m - 1 of a segment in one ds_write2_b32 (rounds still descend; a
    // segment holds >= 8 bytes, so no store of one instruction lands on another's dword)
#pragma unroll
    for (int m = OW; m >= 1; m -= 2) {
      if (m - 1 >= 1) {
        if (m <= mmax) {
#pragma unroll
          for (int u = 0; u < U; ++u)
            asm volatile("ds_write2_b32 %0, %1, %2 offset0:%3 offset1:%4" ::"v"(base[u]), "v"(dw(u, m)),
                         "v"(dw(u, m - 1)), "i"(m), "i"(m - 1) : "memory");
        } else if (m - 1 <= mmax) {
#pragma unroll
          for (int u = 0; u < U; ++u) lds_st32_m(base[u], dw(u, m - 1), m - 1);
        }
      } else if (m <= mmax) {
#pragma unroll
        for (int u = 0; u < U; ++u) lds_st32_m(base[u], dw(u, m), m);
      }
    }
  } else {
#pragma unroll
    for (int m = OW; m >= 1; --m) {
      if (m > mmax) continue;  // wave-uniform: no segment of the wave reaches dword m
#pragma unroll
      for (int u = 0; u < U; ++u) lds_st32_m(base[u], dw(u, m), m);
    }
  }
  // head dwords: read back (the previous segment's tail + garbage), merge, store; the
  // reads are unconditional, the stores are not (a segment at an aligned offset, and the
  // empty segments past a shard's end, have no head dword)
  uint32_t rd[U];
#pragma unroll
  for (int u = 0; u < U; ++u) rd[u] = lds_u32_nowait(base[u]);
  lds_wait(rd);
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint32_t ap = o[u] - base[u];
    if (n[u] && ap < 4u) {
      const uint32_t ab = 8u * ap;  // the previous segment's bits in the dword
      lds_st32(base[u], (rd[u] & ((1u << ab) - 1u)) | (ow[u][0] << ab));
    }
  }
}

// Copy one wave's piece of a tile, staged at LDS byte stg + 16 + i = piece byte i, to
// out[goff, goff + n) (n already clamped at out_cap).  Output chunk c (16 bytes, aligned
// to the global address) is staging bytes [16c + 16 - lb, +16), lb = goff & 15: one
// unaligned ds_read_b128 (gfx950 LDS runs in unaligned mode).  Every lane issues exactly
// NS 16-byte buffer stores and one byte store (the partial head and tail chunks' bytes,
// one per lane): a lane with no chunk (byte) stores at an offset past the buffer's range,
// which the hardware drops, so no padding bytes reach memory and the store count is
// fixed.  gfx950 counts loads and stores in one in-order queue (vmcnt): with a fixed store
// count after the next tile's prefetch loads the compiler waits for those loads with a
// counted vmcnt instead of vmcnt(0), so a wave never waits for its copy-out's stores to
// be acknowledged.  The host sizes the regions so that NS * 64 chunks cover a piece.
constexpr uint32_t OOB_OFF = 0x80000000u;  // a buffer offset past every range: the store is dropped
// v, b: the data registers.  A caller that keeps them alive across its loop (as values
// carried from one copy-out to the next, "+v" below) keeps the register allocator from
// handing them to other values while the stores are in flight: the compiler waits for
// an outstanding store before its data registers are overwritten (vmcnt), so a reuse
// right after the copy-out stalled the next iteration on the stores.
template <int NS, bool PIN = true>
__device__ __forceinline__ void copy_out_piece(uint8_t* out, uint32_t stg, unsigned long long goff, uint32_t n,
                                               int lane, tile_v4u (&v)[NS], uint32_t& b, uint32_t c0 = 0) {
  // (c0: the first chunk of this call; a piece copied in parts, 64 * NS chunks each, has
  // its edge bytes stored by the part with c0 = 0)
  // goff and n are wave-uniform; said so explicitly, the buffer resource lives in SGPRs
  // (otherwise each store became a readfirstlane "waterfall" loop, and the compiler's
  // vmcnt counting across those loops fell back to short counts at the next iteration)
  goff = rfl_u64(goff);
  n = (uint32_t)__builtin_amdgcn_readfirstlane((int)n);
  const uint32_t lb = (uint32_t)(goff & 15);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out + (goff - lb), 0, 0x7FFFFFF0, 0x00020000);
  // (GH_TILE_ABLATE & 128, diagnostic: 16-byte aligned LDS reads, wrong bytes)
  const uint32_t src = (stg + 16u - ((GH_TILE_ABLATE & 128) ? 0u : lb)) & ((GH_TILE_ABLATE & 256) ? ~3u : ~0u);    // staging address of output chunk 0 (diagnostic 256: dword-aligned)
  const uint32_t cf = lb ? 1u : 0u;       // interior chunks [cf, ce)
  const uint32_t ce = n ? (lb + n) >> 4 : 0u;
  uint32_t off[NS];
#pragma unroll
  for (int i = 0; i < NS; ++i) {
    const uint32_t c = c0 + cf + (uint32_t)lane + 64u * (uint32_t)i;
    off[i] = c < ce ? 16u * c : OOB_OFF;
  }
  // edge bytes: the head chunk's [lb, min(16, lb + n)) when lb != 0, then the tail
  // chunk's [0, (lb + n) & 15) when it is another chunk; one byte per lane
  const uint32_t nh = (lb && n) ? min(16u, lb + n) - lb : 0u;
  const uint32_t tl = (lb + n) & 15u;
  const uint32_t nt = (n && tl && (ce > 0 || !lb)) ? tl : 0u;
  const uint32_t t = (uint32_t)lane;
  uint32_t k = OOB_OFF;
  if (c0 == 0u && !(GH_TILE_ABLATE & 64)) {  // (diagnostic 64: no edge bytes)
    if (t < nh) k = lb + t;
    else if (t < nh + nt) k = 16u * ce + (t - nh);
  }
  if constexpr (GH_TILE_ALRD) {
    // Output chunk c is staging bytes [src + 16c, +16): the last 16 - lb bytes of the
    // aligned chunk at stg + 16c and the first lb of the next.  Both aligned chunks are read
    // (an unaligned ds_read_b128 costs the copy-out several times its aligned pair: cfg4
    // window 0.53 vs 0.49 ms with the reads aligned, round 6) and shifted into place in
    // registers: output dword d = window bytes [s + 4d, +4) of P:Q, s = 16 - lb (lb = 0:
    // Q), a wave-uniform case on s >> 2 and v_alignbyte by s & 3.  Chunks go CG at a time
    // (registers), each group stored as soon as it is shifted; the store count is fixed.
    constexpr int CG = NS % 2 == 0 ? 2 : 1;
    const uint32_t sh = (16u - lb) & 15u, r = sh & 3u, m = lb ? sh >> 2 : 4u;
    if constexpr (GH_TILE_ALRD == 2) {
      // (variant) one aligned read per chunk: P_i = aligned chunk c_i of every lane (and
      // P_NS for lane 0), Q_i = the next lane's P_i (lane 63: P_{i+1} of lane 0) by DPP
      tile_v4u P[NS + 1];
#pragma unroll
      for (int i = 0; i <= NS; ++i) {
        const uint32_t c = c0 + cf + (uint32_t)lane + 64u * (uint32_t)i;
        const uint32_t a = stg + 16u * (c < ce + 1u ? c : cf);
        asm volatile("ds_read_b128 %0, %1" : "=v"(P[i]) : "v"(a) : "memory");
      }
      if (PIN) asm volatile("ds_read_u8 %0, %1" : "+v"(b) : "v"(src + (k == OOB_OFF ? 0u : k)) : "memory");
      else asm volatile("ds_read_u8 %0, %1" : "=v"(b) : "v"(src + (k == OOB_OFF ? 0u : k)) : "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int i = 0; i <= NS; ++i) asm volatile("" : "+v"(P[i]));
#pragma unroll
      for (int i = 0; i < NS; ++i) {
        tile_v4u Q;
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          const int nx = __builtin_amdgcn_update_dpp(0, (int)P[i + 1][d], 0x134, 0xf, 0xf, false);  // wave_rol:1
          Q[d] = (uint32_t)__builtin_amdgcn_update_dpp(nx, (int)P[i][d], 0x130, 0xf, 0xf, false);    // wave_shl:1
        }
        auto W = [&](int q) -> uint32_t { return q < 4 ? P[i][q] : Q[q - 4]; };
        switch (m) {
          case 0:
            for (int d = 0; d < 4; ++d) v[i][d] = __builtin_amdgcn_alignbyte(W(d + 1), W(d), r);
            break;
          case 1:
            for (int d = 0; d < 4; ++d) v[i][d] = __builtin_amdgcn_alignbyte(W(d + 2), W(d + 1), r);
            break;
          case 2:
            for (int d = 0; d < 4; ++d) v[i][d] = __builtin_amdgcn_alignbyte(W(d + 3), W(d + 2), r);
            break;
          case 3:
            for (int d = 0; d < 4; ++d) v[i][d] = __builtin_amdgcn_alignbyte(W(d + 4), W(d + 3), r);
            break;
          default:
            v[i] = Q;
            break;
        }
        __builtin_amdgcn_raw_buffer_store_b128(v[i], rs, (int)off[i], 0, 2);  // nt
      }
      if (PIN) asm volatile("" : "+v"(b));
      __builtin_amdgcn_raw_buffer_store_b8((uint8_t)b, rs, (int)k, 0, 2);
      return;
    }
#pragma unroll
    for (int g0 = 0; g0 < NS; g0 += CG) {
      tile_v4u pq[CG][2];
#pragma unroll
      for (int j = 0; j < CG; ++j) {
        const int i = g0 + j;
        const uint32_t c = c0 + cf + (uint32_t)lane + 64u * (uint32_t)i;
        const uint32_t a = stg + 16u * (c < ce ? c : cf);
        asm volatile("ds_read_b128 %0, %1" : "=v"(pq[j][0]) : "v"(a) : "memory");
        asm volatile("ds_read_b128 %0, %1 offset:16" : "=v"(pq[j][1]) : "v"(a) : "memory");
      }
      if (g0 + CG >= NS) {  // the edge byte with the last group
        if (PIN) asm volatile("ds_read_u8 %0, %1" : "+v"(b) : "v"(src + (k == OOB_OFF ? 0u : k)) : "memory");
        else asm volatile("ds_read_u8 %0, %1" : "=v"(b) : "v"(src + (k == OOB_OFF ? 0u : k)) : "memory");
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int j = 0; j < CG; ++j) asm volatile("" : "+v"(pq[j][0]), "+v"(pq[j][1]));  // (after the wait)
      auto shift = [&](auto mc) {
        constexpr int M = decltype(mc)::value;
#pragma unroll
        for (int j = 0; j < CG; ++j) {
          if constexpr (M == 4) {
            v[g0 + j] = pq[j][1];
          } else {
            auto W = [&](int q) -> uint32_t { return q < 4 ? pq[j][0][q] : pq[j][1][q - 4]; };
#pragma unroll
            for (int d = 0; d < 4; ++d) v[g0 + j][d] = __builtin_amdgcn_alignbyte(W(M + d + 1), W(M + d), r);
          }
        }
      };
      switch (m) {
        case 0: shift(std::integral_constant<int, 0>{}); break;
        case 1: shift(std::integral_constant<int, 1>{}); break;
        case 2: shift(std::integral_constant<int, 2>{}); break;
        case 3: shift(std::integral_constant<int, 3>{}); break;
        default: shift(std::integral_constant<int, 4>{}); break;
      }
#pragma unroll
      for (int j = 0; j < CG; ++j) __builtin_amdgcn_raw_buffer_store_b128(v[g0 + j], rs, (int)off[g0 + j], 0, 2);  // nt
    }
    if (PIN) asm volatile("" : "+v"(b));
    __builtin_amdgcn_raw_buffer_store_b8((uint8_t)b, rs, (int)k, 0, 2);
    return;
  }
#pragma unroll
  for (int i = 0; i < NS; ++i) {
    const uint32_t c = c0 + cf + (uint32_t)lane + 64u * (uint32_t)i;
    if (PIN) asm volatile("ds_read_b128 %0, %1" : "+v"(v[i]) : "v"(src + 16u * (c < ce ? c : cf)) : "memory");
    else asm volatile("ds_read_b128 %0, %1" : "=v"(v[i]) : "v"(src + 16u * (c < ce ? c : cf)) : "memory");
  }
  if (PIN) asm volatile("ds_read_u8 %0, %1" : "+v"(b) : "v"(src + (k == OOB_OFF ? 0u : k)) : "memory");
  else asm volatile("ds_read_u8 %0, %1" : "=v"(b) : "v"(src + (k == OOB_OFF ? 0u : k)) : "memory");
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(b)::"memory");
#pragma unroll
  for (int i = 0; i < NS; ++i) asm volatile("" : "+v"(v[i]));  // (after the wait: asm volatile order)
#pragma unroll
  for (int i = 0; i < NS; ++i) __builtin_amdgcn_raw_buffer_store_b128(v[i], rs, (int)off[i], 0, 2);  // nt
  __builtin_amdgcn_raw_buffer_store_b8((uint8_t)b, rs, (int)k, 0, 2);
}

// A segment's n bytes (ow, byte 0 first) stored to out[o, o + n), clamped at cap: the
// path of a tile too large for staging (byte stores; rare).
template <int OW>
__device__ __forceinline__ void store_direct(uint8_t* out, unsigned long long cap, unsigned long long o,
                                             const uint32_t (&ow)[OW], uint32_t n) {
#pragma unroll
  for (int i = 0; i < 4 * OW; ++i)
    if ((uint32_t)i < n && o + (uint32_t)i < cap) out[o + (uint32_t)i] = (uint8_t)(ow[i >> 2] >> (8 * (i & 3)));
}

__device__ __forceinline__ bool granule_ok(const TileParams& p, unsigned long long v, uint32_t flag) {
  return (uint32_t)(v >> 40) == p.epoch && (uint32_t)((v >> 38) & 3u) == flag;
}

// Poll a granule until it carries this launch's epoch with the wanted flag.  Bounded by
// wall time, 4 s of the 100 MHz clock: a persistent grid that shares the GPU with
// another kernel (another stream or process) waits for its not-yet-resident workgroups
// until that kernel's workgroups retire — a delay, not a fault.  After a timeout every
// later poll returns at once (the decode then fails with GH_E_HIP).  The clock and the
// status word are read only every 64th poll: a poll's load sits in the CU's memory
// queue behind its streaming traffic (microseconds), and the hand-off chain pays every
// extra round trip.
__device__ __forceinline__ unsigned long long poll_granule(const TileParams& p, unsigned long long* g,
                                                           uint32_t flag) {
  unsigned long long t0 = 0;
  for (uint32_t spins = 1;; ++spins) {
    const unsigned long long v = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (granule_ok(p, v, flag)) return v;
    if ((spins & 63u) == 0u) {
      if (__hip_atomic_load(p.status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & GH_ST_TIMEOUT) return 0;
      const unsigned long long t = wall_clock64();
      if (t0 == 0) {
        t0 = t;
      } else if (t - t0 > 400000000ull) {
        atomicOr(p.status, (unsigned)GH_ST_TIMEOUT);
        return 0;
      }
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

// The round leader (workgroup 0): for every round r of D decoding workgroups' tiles, wait
// for the round's aggregates (thread t takes the A = ceil(D / TB) <= LEAD_A consecutive
// tiles t*A .. t*A + A - 1 of the round), scan them and publish each tile's global
// exclusive prefix; R, the start of the round, stays in a register.  (Spreading the rounds
// over the leader's waves, the next rounds' aggregates loaded ahead, measured slower:
// 0.74 vs 0.71 ms in round 3 with eight rounds in flight, 0.615 vs 0.586 ms in round 5
// with two.)
constexpr int LEAD_A = 4;
template <int TB>
__device__ __forceinline__ void tile_round_leader(const TileParams& p, uint32_t D, uint32_t* s_lead, int tid,
                                                  int lane, int wid) {
  const uint32_t A = (D + TB - 1) / TB;  // <= LEAD_A (the host caps the grid)
  const uint32_t nr = (p.ntiles + D - 1) / D;
  unsigned long long R = 0;
  for (uint32_t r = 0; r < nr; ++r) {
    const uint32_t t0 = r * D, n = min(D, p.ntiles - t0);
    uint32_t v[LEAD_A], sum = 0;
#pragma unroll
    for (int i = 0; i < LEAD_A; ++i) {
      const uint32_t j = (uint32_t)tid * A + (uint32_t)i;
      v[i] = 0;
      if ((uint32_t)i < A && j < n) {
        unsigned long long g = __hip_atomic_load(&p.granules[t0 + j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (!granule_ok(p, g, 1)) {
          atomicAdd(p.stats + 1, 1ull);
          g = poll_granule(p, &p.granules[t0 + j], 1);
        }
        v[i] = (uint32_t)(g & GRAN_VMASK);  // a tile holds < 2^32 symbols
      }
      sum += v[i];
    }
    const uint32_t incl = wave_incl_scan(sum);
    if (lane == 63) s_lead[wid] = incl;
    __syncthreads();
    unsigned long long before = 0, total = 0;
#pragma unroll
    for (int q = 0; q < TB / 64; ++q) {
      const uint32_t x = s_lead[q];
      before += (q < wid) ? x : 0u;
      total += x;
    }
    unsigned long long run = R + before + incl - sum;
#pragma unroll
    for (int i = 0; i < LEAD_A; ++i) {
      const uint32_t j = (uint32_t)tid * A + (uint32_t)i;
      if ((uint32_t)i < A && j < n)
        __hip_atomic_store(&p.prefix[t0 + j], granule(p.epoch, 2, run), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      run += v[i];
    }
    R += total;
#if GH_TILE_STAMPS
    if (tid == 0) p.tstamps[2 * p.ntiles + r] = __builtin_amdgcn_s_memrealtime();  // round r published
#endif
    __syncthreads();
  }
}

// (GH_TILE_DYN) The frontier leader: tiles are handed out by ticket, so a round of D
// consecutive tiles may hold a tile whose workgroup waits on another tile of that round;
// instead each tile's prefix is published as soon as every tile before it has published
// its aggregate (a workgroup waits only on tiles older than every tile it holds, so no
// wait cycle exists).  Per pass, thread i looks at tile F + i: the leading run of
// aggregates already in is scanned and published, F moves past it.  Bounded like
// poll_granule (4 s of the 100 MHz clock without progress).
template <int TB>
__device__ __forceinline__ void tile_frontier_leader(const TileParams& p, uint32_t* s_w, int tid, int lane, int wid) {
  constexpr int NW = TB / 64;
  uint32_t F = 0;
  unsigned long long R = 0, t0 = 0;
  uint32_t* const s_first = s_w;       // [2][NW] first tile not in, per wave (double-buffered by pass)
  uint32_t* const s_sum = s_w + 2 * NW;  // [2][NW] wave sums
  for (uint32_t pass = 0; F < p.ntiles; ++pass) {
    const uint32_t t = F + (uint32_t)tid, pb = (pass & 1u) * NW;
    bool in = false;
    uint32_t v = 0;
    if (t < p.ntiles) {
      const unsigned long long g = __hip_atomic_load(&p.granules[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      in = granule_ok(p, g, 1);
      v = (uint32_t)(g & GRAN_VMASK);
    }
    const unsigned long long out = __ballot(!in);
    if (lane == 0) s_first[pb + wid] = out ? (uint32_t)__builtin_ctzll(out) : 64u;
    __syncthreads();
    uint32_t m = (uint32_t)TB;
#pragma unroll
    for (int q = NW - 1; q >= 0; --q) {
      const uint32_t f = s_first[pb + q];
      m = f < 64u ? 64u * (uint32_t)q + f : m;
    }
    const uint32_t vv = (uint32_t)tid < m ? v : 0u;
    const uint32_t incl = wave_incl_scan(vv);
    if (lane == 63) s_sum[pb + wid] = incl;
    __syncthreads();
    unsigned long long before = 0, total = 0;
#pragma unroll
    for (int q = 0; q < NW; ++q) {
      const uint32_t x = s_sum[pb + q];
      before += (q < wid) ? x : 0u;
      total += x;
    }
    if ((uint32_t)tid < m) {
      __hip_atomic_store(&p.prefix[t], granule(p.epoch, 2, R + before + incl - vv), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
#if GH_TILE_STAMPS
      p.tstamps[2 * p.ntiles + t] = __builtin_amdgcn_s_memrealtime();  // tile t's prefix published
#endif
    }
    R += total;
    F += m;
    if (m == 0u) {
      if (tid == 0) atomicAdd(p.stats + 1, 1ull);
      if ((pass & 63u) == 0u) {  // no progress: bounded (every thread reads the same clock)
        if (__hip_atomic_load(p.status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & GH_ST_TIMEOUT) return;
        const unsigned long long tw = wall_clock64();
        if (t0 == 0) {
          t0 = tw;
        } else if (tw - t0 > 400000000ull) {
          if (tid == 0) atomicOr(p.status, (unsigned)GH_ST_TIMEOUT);
          return;
        }
      }
      __builtin_amdgcn_s_sleep(2);
    } else {
      t0 = 0;
    }
  }
}

// TB threads, U segments per lane, GRP codewords per window shift, OW output words per
// segment, codewords of at least MINL bits.  Compiled for 4 waves per SIMD (128 VGPRs):
// one 1024-thread workgroup per CU, which its LUT copies and staging buffers (~157 KB of
// LDS) fill.
//
// The waves of a decoding workgroup run without a workgroup barrier: each stages its own
// segments into its own LDS region and copies its own piece out.  The tile's aggregate
// is published by the wave that arrives last at it (an LDS counter per tile slot), which
// also writes every wave's offset in the tile; a wave reads the offsets of tile k-2 only
// after its global prefix has arrived, which the aggregate (so every wave's arrival)
// precedes.  A wave can thus run at most about three tiles ahead of the slowest wave of
// its workgroup (it needs tile k-3's prefix at iteration k-1), within the TILE_SLOTS
// slots.
template <int TB, int U, int GRP, int OW, int MINL>
__global__ __launch_bounds__(TB) __attribute__((amdgpu_waves_per_eu(4, 4))) void gh_tile_kernel(const TileParams p) {
  static_assert(4 * OW >= (128 + MINL - 1) / MINL, "OW words hold every codeword a segment can start");
  static_assert(U <= TILE_U, "shapes of at most TILE_U segments per lane");
  constexpr int NW = TB / 64;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint32_t stage_lds = p.lut_bytes;                                  // [2][NW] regions
  uint32_t* s_tot = (uint32_t*)(smem + p.lut_bytes + TILE_LAG * NW * p.stage_bytes);  // [SLOTS][NW] wave totals
  uint32_t* s_off = s_tot + TILE_SLOTS * NW;                                // [SLOTS][NW] wave offsets
  uint32_t* s_cnt = s_off + TILE_SLOTS * NW;                                // [SLOTS] arrivals
  unsigned long long* s_pfx = (unsigned long long*)(s_cnt + TILE_SLOTS);   // [SLOTS] prefixes (wave 0)
  uint32_t* s_ptile = (uint32_t*)(s_pfx + TILE_SLOTS);                      // [SLOTS] their tiles
  uint32_t* s_lead = s_ptile + TILE_SLOTS;                                  // [NW] (leader)
  uint32_t* s_ring = s_lead + NW;                                           // [SLOTS] (GH_TILE_DYN) tile of iteration k
  const uint32_t cnt_lds = (uint32_t)((uint8_t*)s_cnt - smem);
  const uint32_t ptile_lds = (uint32_t)((uint8_t*)s_ptile - smem);
  const uint32_t ring_lds = (uint32_t)((uint8_t*)s_ring - smem);

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
#if GH_TILE_STAMPS
  // per launch (ring of 1024 by epoch): shader-clock and 100 MHz times at the leader's start
  // and end, to read the clock the kernel ran at
  unsigned long long* const lring = p.tstamps + 3ull * p.ntiles + 64 + 4ull * (p.epoch & 1023u);
  if (blockIdx.x == 0 && tid == 0) {
    lring[0] = __builtin_amdgcn_s_memtime();
    lring[1] = __builtin_amdgcn_s_memrealtime();
  }
#endif
  // decoding workgroups: every block but 0 (the leader) and p.idle_block (if < grid)
  const uint32_t D = gridDim.x - 1 - (p.idle_block < gridDim.x ? 1u : 0u);
  if (blockIdx.x == 0) {
    if constexpr (GH_TILE_DYN) {
      if (tid == 0) p.tickets[2u * ((p.epoch + 1u) & 1u)] = 0u;  // the next launch's counter
      tile_frontier_leader<TB>(p, (uint32_t*)smem, tid, lane, wid);
    } else {
      tile_round_leader<TB>(p, D, s_lead, tid, lane, wid);
    }
#if GH_TILE_STAMPS
    if (tid == 0) {
      lring[2] = __builtin_amdgcn_s_memtime();
      lring[3] = __builtin_amdgcn_s_memrealtime();
    }
#endif
    return;
  }
  if (blockIdx.x == p.idle_block) return;  // the leader's CU partner (GH_TILE_IDLE): no decoding
#if GH_TILE_STAMPS
  // per workgroup: shader-clock and 100 MHz times at its start and end (its clock)
  unsigned long long* const wring = p.tstamps + 3ull * p.ntiles + 64 + 4ull * 1024 + 4ull * blockIdx.x;
  if (tid == 0) {
    wring[0] = __builtin_amdgcn_s_memtime();
    wring[1] = __builtin_amdgcn_s_memrealtime();
  }
#endif
  {  // LUT to LDS, replicated: dword i of LDS = entry i >> lgr (lane l reads copy l mod 2^lgr,
     // so up to 32 lanes of a ds_read_b32 hit distinct banks)
    const uint32_t nd = p.lut_bytes >> 2;
    uint32_t* sl = (uint32_t*)smem;
    for (uint32_t i = tid; i < nd; i += TB) sl[i] = p.lut[i >> p.lgr];
    if (tid < TILE_SLOTS) {
      s_cnt[tid] = 0;
      s_ptile[tid] = 0xFFFFFFFFu;
    }
    if (GH_TILE_DYN && tid <= TILE_TAHEAD) {  // iterations 0 .. TAHEAD: static tiles
      const uint32_t b0 = blockIdx.x - 1 - (blockIdx.x > p.idle_block ? 1u : 0u);
      const uint32_t tt = b0 + (uint32_t)tid * D;
      s_ring[tid] = tt < p.ntiles ? tt : 0xFFFFFFFFu;
    }
  }
  const uint32_t S = 30u - p.kbits - p.lgr;
  // (GH_TILE_ABLATE & 16, diagnostic: even LUT entries only, so a read's lanes never
  // collide in a bank; wrong output)
  const uint32_t amask = (((1u << p.kbits) - 1u) << (2u + p.lgr)) & ((GH_TILE_ABLATE & 16) ? ~(1u << (2u + p.lgr)) : ~0u);
  const uint32_t laneoff = ((uint32_t)lane & ((1u << p.lgr) - 1u)) << 2;
  check_lds_base(smem, p.status);

  const uint32_t G = D, b = blockIdx.x - 1 - (blockIdx.x > p.idle_block ? 1u : 0u);  // decoders, this one
  const uint32_t nseg = (uint32_t)p.nseg;                 // < 2^31 (checked by the host)
  constexpr uint32_t NONE = 0xFFFFFFFFu;
  __syncthreads();  // the LUT and the counters (the last barrier of a decoding workgroup)
  // (GH_TILE_DYN: the static bound below does not hold; every iteration then either
  // decodes a tile or drains a staged one, so 2 * ntiles iterations bound a sound run)
  const uint32_t last_tile_k = GH_TILE_DYN ? p.ntiles + 2u * TILE_SLOTS
                               : b < p.ntiles ? (p.ntiles - 1 - b) / G : NONE;
  uint32_t cur = b, nxt = b + G;
  // (GH_TILE_DYN) wave 0 lane 0 holds the ticket taken one iteration earlier; tickets
  // count tiles from (TAHEAD + 1) * D on
  const uint32_t dyn_base = (uint32_t)(TILE_TAHEAD + 1) * D;
  uint32_t tk = 0;
  bool tk_live = GH_TILE_DYN && dyn_base < p.ntiles;
  unsigned int* const tctr = GH_TILE_DYN ? p.tickets + 2u * (p.epoch & 1u) : nullptr;
  // the lane's segments in a tile: wave-contiguous, 64 per chain (chain u lane l: segment
  // 64u + l of the wave's 64U); lane-major (GH_TILE_LMAJ): lane l's U consecutive segments
  // Ul .. Ul + U - 1, so the staging stores of one instruction land ~U segments apart
  constexpr uint32_t CSTR = GH_TILE_LMAJ ? 1u : 64u;  // segment stride between chains
  const uint32_t lseg = (uint32_t)(wid * 64 * U) + (uint32_t)lane * (GH_TILE_LMAJ ? (uint32_t)U : 1u);
  constexpr int NSET = GH_TILE_PF2 ? 2 : 1;  // register sets of prefetched words
  static_assert(!(GH_TILE_PF2 && (GH_TILE_DYN || GH_TILE_HOLD)), "PF2: static schedule, no hold");
  uint4 wset[NSET][U];
  uint32_t w4set[NSET][U], gwset[NSET][U];
  auto load = [&](auto SS, uint32_t t) {
    constexpr int SI = decltype(SS)::value;
    uint4 (&w)[U] = wset[SI];
    uint32_t (&w4)[U] = w4set[SI];
    uint32_t (&gw)[U] = gwset[SI];
    const uint32_t seg0 = min(t, p.ntiles - 1) * (uint32_t)(U * TB) + lseg;
    if constexpr (GH_TILE_LMAJ) {
      // one lane's U consecutive segments: their 16 U bytes and the next segment's first
      // word (chain u's look-ahead word is chain u + 1's first word); past the shard end
      // the lane reads the zero padding (inactive)
      const uint32_t sb = min(seg0, nseg - 1);
#pragma unroll
      for (int u = 0; u < U; ++u) w[u] = *(const uint4*)(p.payload + 4ull * (sb + (uint32_t)u));
      w4[U - 1] = p.payload[4ull * (sb + (uint32_t)U)];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t sc = sb + (uint32_t)u;
        gw[u] = p.gaps[(p.gap_nib0 + (sc ? sc - 1u : 0u)) >> 3];
      }
    } else {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t sc = min(seg0 + (uint32_t)(64 * u), nseg - 1);
        w[u] = *(const uint4*)(p.payload + 4ull * sc);
        w4[u] = p.payload[4ull * sc + 4];
        gw[u] = p.gaps[(p.gap_nib0 + (sc ? sc - 1u : 0u)) >> 3];
      }
    }
  };
  // (GH_TILE_DYN) the ticket operation after every prefetch: wave 0 lane 0 takes the next
  // ticket (its tile posted one iteration later), every other wave, and wave 0 once the
  // tiles are out, issues a dropped store instead, so each wave has the same VMEM
  // operations after its loads on every path (a counted vmcnt that never waits for the
  // ticket, whose counter is contended: it is read a whole iteration later)
  const __amdgpu_buffer_rsrc_t rs_out = __builtin_amdgcn_make_buffer_rsrc(p.out, 0, 0x7FFFFFF0, 0x00020000);
  auto ticket_op = [&]() {
    if constexpr (GH_TILE_DYN) {
      if (wid == 0 && tk_live) {
        if (lane == 0) tk = atomicAdd(tctr, 1u);
      } else {
        __builtin_amdgcn_raw_buffer_store_b8((uint8_t)0, rs_out, (int)(OOB_OFF + 64u), 0, 2);
      }
    }
  };
  auto junk_stores = [&]() {  // as many stores after these loads as every iteration issues
     // after its prefetch (the copy-out's TILE_NS + 1, dropped here: out of range): the
     // loop's entry then matches its back edge, and the compiler waits for the loads with
     // a counted vmcnt
    const __amdgpu_buffer_rsrc_t rs = rs_out;
#pragma unroll
    for (int i = 0; i < TILE_NS; ++i)
      __builtin_amdgcn_raw_buffer_store_b128(tile_v4u{0, 0, 0, 0}, rs, (int)(OOB_OFF + 16u * (uint32_t)i), 0, 2);  // (distinct: not merged)
    __builtin_amdgcn_raw_buffer_store_b8((uint8_t)0, rs, (int)OOB_OFF, 0, 2);
  };
  load(std::integral_constant<int, 0>{}, cur);
  ticket_op();
  junk_stores();
  if constexpr (GH_TILE_PF2) {
    // (the iteration's two prefix loads, then the next tile's words: the back edge's order)
    (void)__hip_atomic_load(&p.prefix[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    (void)__hip_atomic_load(&p.prefix[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    load(std::integral_constant<int, NSET - 1>{}, nxt);
    junk_stores();
  }
  if (cur >= p.ntiles) cur = NONE;
  uint32_t th[TILE_LAG];          // this wave's pieces of iterations k-1 .. k-LAG (NONE: not staged)
#pragma unroll
  for (int i = 0; i < TILE_LAG; ++i) th[i] = NONE;
  // (GH_TILE_HOLD) the previous iteration's tile, held in registers until it is staged
  uint32_t owp[U][OW], cntp[U], bposp[U], wtp = 0, prevt = NONE;
  int gdp = 1;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    cntp[u] = 0;
    bposp[u] = 0;
#pragma unroll
    for (int k2 = 0; k2 < OW; ++k2) asm volatile("" : "=v"(owp[u][k2]));
  }
  uint32_t rank = 0;              // the wave's arrival rank at its last tile, in quarters
  const uint32_t region0 = stage_lds + (uint32_t)wid * p.stage_bytes;  // buffer 0; buffer 1 at + NW * stage_bytes
  const uint32_t piece_cap = p.stage_bytes - (uint32_t)(STAGE_PAD + 4 * OW + 4);
#if GH_TILE_STAMPS
  unsigned long long ts[9];
#endif
  auto body = [&](auto SS, uint32_t k) -> bool {
    constexpr int SI = decltype(SS)::value;  // the register set holding this tile's words
    uint4 (&w)[U] = wset[SI];
    uint32_t (&w4)[U] = w4set[SI];
    uint32_t (&gw)[U] = gwset[SI];
    TSTAMP(0);
    const bool have_cur = cur < p.ntiles;
    const uint32_t t2 = th[TILE_LAG - 1];  // the piece copied out this iteration (tile k - LAG)
    const bool have2 = t2 < p.ntiles;
    bool pending = have_cur || (GH_TILE_HOLD && prevt < p.ntiles);
#pragma unroll
    for (int i = 0; i < TILE_LAG; ++i) pending |= th[i] < p.ntiles;
    if (!pending) return false;
    if (last_tile_k != NONE && k > last_tile_k + TILE_LAG + 2) {  // cannot happen; never hang the GPU
      if (lane == 0) atomicOr(p.status, (unsigned)GH_ST_TIMEOUT);
      return false;
    }
    const uint32_t slot = k % TILE_SLOTS, slot2 = (k + TILE_SLOTS - TILE_LAG - GH_TILE_HOLD) % TILE_SLOTS;
    const uint32_t slotp = (k + TILE_SLOTS - 1) % TILE_SLOTS;  // (GH_TILE_HOLD) the held tile's
    const uint32_t buf = k % TILE_LAG;
    // issue priority by the wave's arrival rank at its last tile (0: first of the
    // workgroup's waves): the waves that arrive last gate the tile's aggregate, so they
    // issue first (the round-3/4 rule, priority 0 after a polled prefix, was slower)
    if (rank >= 3) __builtin_amdgcn_s_setprio(3);
    else if (rank == 2) __builtin_amdgcn_s_setprio(2);
    else if (rank == 1) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
    // prefix of tile k-LAG: loaded at the top and again mid-decode; the first that
    // shows it published is used (a load at the top alone often saw it a little before it
    // was published, and the re-poll then paid a full memory round trip)
    // (every lane loads the same word, one request; no branch around the load: the
    // compiler's wait counting over such a branch fell back to vmcnt(0), which then also
    // waited for the next tile's loads issued behind it)
    unsigned long long* const pf2 = &p.prefix[have2 ? t2 : 0u];
    unsigned long long gp0 = 0, gp = 0, gpl = 0;
    if (!(GH_TILE_ABLATE & 4)) gp0 = __hip_atomic_load(pf2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    auto mid = [&]() {
      if (!(GH_TILE_ABLATE & 4)) gp = __hip_atomic_load(pf2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    // ---- decode this tile (its words were loaded during the previous iteration) --------
    // Decoded unconditionally: in the last iterations (no tile) every chain is inactive
    // and the loop stops after one group (the loads were issued, clamped to the last
    // tile).  A branch around the decode made the compiler zero the output words before
    // it every iteration and wait vmcnt(0) after it.
    const uint32_t seg0 = cur * (uint32_t)(U * TB) + lseg;
    uint32_t ow[U][OW], cnt[U];
    int gdone;
    {
      int start[U];
      bool act[U];
      uint32_t e[U][5];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t seg = seg0 + (uint32_t)u * CSTR;
        act[u] = have_cur && seg < nseg;
        start[u] = seg == 0 ? (int)p.first_start : (int)gap_nib(gw[u], p.gap_nib0 + seg - 1u);
        make_ewin(w[u], (GH_TILE_LMAJ && u + 1 < U) ? w[u + 1 < U ? u + 1 : u].x : w4[u], start[u], S, e[u]);
      }
      TSTAMP(1);
      if (GH_TILE_ABLATE & 1) {  // diagnostic build: no decode, 16 bytes per segment (wrong output)
#pragma unroll
        for (int u = 0; u < U; ++u) {
          cnt[u] = act[u] ? 16u : 0u;
#pragma unroll
          for (int k2 = 0; k2 < OW; ++k2) ow[u][k2] = e[u][k2 % 5];
        }
        mid();
        gdone = (16 + GRP - 1) / GRP;
      } else {
        gdone = decode_tile_rolling<GRP, U, OW, MINL>(e, start, act, ow, cnt, amask, laneoff, mid);
      }
    }
    // The next tile's words, right after the decode (its windows are dead, so the
    // registers are free; issued during the decode they raised its register peak past
    // 128): they have the rest of the iteration (~6 K cycles) to arrive.  Issued after the
    // copy-out instead they had ~3 K cycles, and the next decode waited ~1.3 K cycles for
    // them.  They follow the prefix loads, whose waits therefore do not include them
    // (vmcnt is one in-order queue).
    if constexpr (GH_TILE_DYN) {
      // wave 0 posts the tile of iteration k + 1 + TAHEAD (the ticket it took last
      // iteration) and takes the next ticket; every wave reads the tile of iteration k + 1,
      // posted at least TAHEAD iterations ago by wave 0, which is never more than three
      // iterations behind another wave of its workgroup
      if (wid == 0) {
        uint32_t tpost = NONE;
        if (lane == 0 && tk_live) tpost = dyn_base + tk < p.ntiles ? dyn_base + tk : NONE;
        tpost = (uint32_t)__builtin_amdgcn_readfirstlane((int)tpost);
        tk_live = tk_live && tpost != NONE;
        if (lane == 0) lds_st_u32(ring_lds + 4u * ((k + 1u + TILE_TAHEAD) % TILE_SLOTS), tpost);
      }
      nxt = lds_ld_u32(ring_lds + 4u * ((k + 1u) % TILE_SLOTS));
      nxt = (uint32_t)__builtin_amdgcn_readfirstlane((int)nxt);
    }
    // (GH_TILE_LATEP) a third look at the prefix, after the decode and just BEFORE the
    // prefetch: vmcnt is one in-order queue, so a poll issued behind the prefetch cannot
    // be read before the prefetch has landed (~2-3 us under load); this one can
    if (GH_TILE_LATEP && !(GH_TILE_ABLATE & 4)) gpl = __hip_atomic_load(pf2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // (GH_TILE_PF2: the words of the tile after next, into this iteration's register set)
    load(SS, GH_TILE_PF2 ? nxt + G : nxt);
    ticket_op();
    TSTAMP(2);
    // ---- wave scans: the segments' offsets in the wave's piece, the piece's length -------
    uint32_t bpos[U], wave_tot = 0;
    if constexpr (GH_TILE_LMAJ) {  // lane l's segments are consecutive: one scan of their sum
      uint32_t sl = 0;
#pragma unroll
      for (int u = 0; u < U; ++u) sl += cnt[u];
      const uint32_t incl = wave_incl_scan(sl);
      uint32_t run = incl - sl;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        bpos[u] = run;
        run += cnt[u];
      }
      wave_tot = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    } else {
#pragma unroll
      for (int u = 0; u < U; ++u) bpos[u] = wave_incl_scan(cnt[u]);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t ct = (uint32_t)__builtin_amdgcn_readlane((int)bpos[u], 63);
        bpos[u] += wave_tot - cnt[u];
        wave_tot += ct;
      }
    }
    // ---- arrival at tile k: the last wave to arrive publishes its aggregate ------------
    uint32_t tile_total = 0;
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
        // every wave's total of this tile is in LDS (each wave stored it before its add)
        const uint32_t x = lane < NW ? s_tot[slot * NW + lane] : 0u;
        const uint32_t xi = wave_incl_scan(x);
        if (lane < NW) s_off[slot * NW + lane] = xi - x;
        tile_total = (uint32_t)__builtin_amdgcn_readlane((int)xi, NW - 1);
        if (lane == 0) {
          s_cnt[slot] = 0;
          // the offsets are in LDS before the aggregate leaves (a wave reads them once the
          // prefix this aggregate leads to has arrived)
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          __hip_atomic_store(&p.granules[cur], granule(p.epoch, 1, tile_total), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
#if GH_TILE_STAMPS
          p.tstamps[cur] = __builtin_amdgcn_s_memrealtime();  // tile cur's aggregate left
#endif
        }
      }
    }
    TSTAMP(3);
    // ---- the prefix of tile k-LAG -> this wave's piece's output offset -------------------
    unsigned long long goff = 0;
    uint32_t n2 = 0;
    if (have2 && (GH_TILE_ABLATE & 4)) {
      goff = ((unsigned long long)t2 * (U * TB * 16) + (uint32_t)wid * (U * 64 * 16)) % (p.out_cap - (U * TB * 32));
      n2 = s_tot[slot2 * NW + wid];
    } else if (have2) {
      // The wave's own early loads (top of the iteration, mid-decode) when they already
      // show the prefix; else the LDS post of the first wave of the workgroup that saw it,
      // or the wave's own poll, whichever comes first (the poll posts what it finds).
      unsigned long long g = rfl_u64(gp0);  // wave-uniform: each waits for its own load only
      bool polled = false, got = true;  // (polled: GH_TILE_STAMPS builds)
      (void)polled;
      if (!granule_ok(p, g, 2)) g = rfl_u64(gp);
      if (GH_TILE_LATEP && !granule_ok(p, g, 2)) g = rfl_u64(gpl);
      {
        if (!granule_ok(p, g, 2)) {
          polled = true;
          if (wid == 0 && lane == 0) atomicAdd(p.stats, 1ull);
          unsigned long long t0w = 0;
          // (two or three polls in flight measured slower: 0.440 vs 0.433 ms, round 5)
          unsigned long long pv = __hip_atomic_load(pf2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          for (uint32_t spins = 1;; ++spins) {
            bool found = false;
            if (lds_ld_u32(ptile_lds + 4u * slot2) == t2) {
              asm volatile("" ::: "memory");
              g = s_pfx[slot2];
              found = true;
            } else {
              g = rfl_u64(pv);
              if (granule_ok(p, g, 2)) {
                if (lane == 0) {  // post: the value, then its tile (LDS order)
                  s_pfx[slot2] = g;
                  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                  lds_st_u32(ptile_lds + 4u * slot2, t2);
                }
                found = true;
              } else if (GH_TILE_POLLDIV <= 1 || ((spins + (uint32_t)wid) % GH_TILE_POLLDIV) == 0u) {
                pv = __hip_atomic_load(pf2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              }
            }
            if (found) break;
            if ((spins & 63u) == 0u) {  // bounded like poll_granule: 4 s of the 100 MHz clock
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
          got = granule_ok(p, g, 2);  // false only after a timeout (then nothing is written)
        }
      }
      // the tile's offsets were in LDS before its aggregate left, and the aggregate before
      // its prefix: read them only now (no compiler hoisting above the check)
      asm volatile("" ::: "memory");
      goff = (g & GRAN_VMASK) + s_off[slot2 * NW + wid];
      if (GH_TILE_ABLATE & 32) goff &= ~15ull;  // (diagnostic: 16-byte aligned pieces, wrong output)
      n2 = s_tot[slot2 * NW + wid];
      if (wid == NW - 1 && t2 == p.ntiles - 1 && got && lane == 0) *p.total = goff + n2;
#if GH_TILE_STAMPS
      if (wid == 0 && lane == 0) p.tstamps[p.ntiles + t2] = __builtin_amdgcn_s_memrealtime() | ((unsigned long long)polled << 63);
#endif
      n2 = (!got || goff >= p.out_cap) ? 0u : (uint32_t)min<unsigned long long>(n2, p.out_cap - goff);
    }
    TSTAMP(4);
    // ---- copy this wave's piece of tile k-LAG out ----------------------------------------
    // Unconditional (nothing to copy: n2 = 0, every store dropped): the same store count
    // on every path lets the compiler wait for the prefetched loads with a counted vmcnt
    // at the top of the next iteration.
    if (!(GH_TILE_ABLATE & 8)) {
      tile_v4u cv[TILE_NS];
      uint32_t cb;
      copy_out_piece<TILE_NS, false>(p.out, region0 + buf * NW * p.stage_bytes, goff, n2, lane, cv, cb);
    }
    TSTAMP(5);
    // ---- stage this tile's piece (copied out LAG iterations later) ----------------------
    // a piece larger than the region (data whose shortest codewords cluster) waits for
    // the tile's prefix instead and stores its bytes straight from registers (it has
    // published its arrival, so the prefix cannot depend on it)
    // (GH_TILE_HOLD: the tile decoded last iteration, held in registers, is staged now and
    // this one is held in its place)
    const uint32_t st_t = GH_TILE_HOLD ? prevt : cur;
    const bool have_st = st_t < p.ntiles;
    const uint32_t st_tot = GH_TILE_HOLD ? wtp : wave_tot;
    const uint32_t st_slot = GH_TILE_HOLD ? slotp : slot;
    const bool staged = have_st && st_tot <= piece_cap;
    auto stage_or_store = [&](const uint32_t (&sow)[U][OW], const uint32_t (&scnt)[U], const uint32_t (&sbpos)[U],
                              int sgd) {
      if (have_st && !staged) {
        unsigned long long goffc = 0;
        bool got = true;
        if (lane == 0) {
          unsigned long long g = __hip_atomic_load(&p.prefix[st_t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (!granule_ok(p, g, 2)) g = poll_granule(p, &p.prefix[st_t], 2);
          got = granule_ok(p, g, 2);  // false only after a timeout (then nothing is written)
          asm volatile("" ::: "memory");
          goffc = (g & GRAN_VMASK) + s_off[st_slot * NW + wid];
          if (wid == NW - 1 && st_t == p.ntiles - 1 && got) *p.total = goffc + st_tot;
        }
        goffc = rfl_u64(goffc);
        if (__builtin_amdgcn_readfirstlane(got ? 1 : 0)) {
#pragma unroll
          for (int u = 0; u < U; ++u) store_direct(p.out, p.out_cap, goffc + sbpos[u], sow[u], scnt[u]);
        }
        // (rare path) drain its data-dependent loads and stores here, so that the
        // compiler's wait for the next tile's loads stays a counted vmcnt on the common path
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
      } else if (have_st && !(GH_TILE_ABLATE & 2)) {
        const uint32_t sbase = region0 + buf * NW * p.stage_bytes + STAGE_PAD;
        uint32_t o[U];
#pragma unroll
        for (int u = 0; u < U; ++u) o[u] = sbase + sbpos[u];
        // no segment of the wave holds more than GRP * gdone codewords: rounds above its
        // last dword are skipped
        stage_wave<U, OW>(sow, scnt, o, min(OW, (GRP * sgd + 3) >> 2));
      }
    };
    if constexpr (GH_TILE_HOLD) {
      stage_or_store(owp, cntp, bposp, gdp);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        cntp[u] = cnt[u];
        bposp[u] = bpos[u];
#pragma unroll
        for (int k2 = 0; k2 < OW; ++k2) owp[u][k2] = ow[u][k2];
      }
      wtp = wave_tot;
      gdp = gdone;
    } else {
      stage_or_store(ow, cnt, bpos, gdone);
    }
    TSTAMP(6);
#if GH_TILE_STAMPS
    TSTAMP(7);
    TSTAMP(8);
    if (lane == 0 && (wid == 0 || wid == NW / 2) && k < 128) {  // the first wave of each half
      uint4* st = p.stamps + (((unsigned long long)blockIdx.x * 2 + (wid ? 1 : 0)) * 128 + k) * 2;
      st[0] = make_uint4((uint32_t)(ts[1] - ts[0]), (uint32_t)(ts[2] - ts[1]), (uint32_t)(ts[3] - ts[2]),
                         (uint32_t)(ts[4] - ts[3]));
      st[1] = make_uint4((uint32_t)(ts[5] - ts[4]), (uint32_t)(ts[6] - ts[5]), (uint32_t)(ts[7] - ts[6]),
                         (uint32_t)(ts[8] - ts[7]));
    }
#endif
#pragma unroll
    for (int i = TILE_LAG - 1; i > 0; --i) th[i] = th[i - 1];
    th[0] = staged ? st_t : NONE;
    if constexpr (GH_TILE_HOLD) prevt = have_cur ? cur : NONE;
    cur = nxt < p.ntiles ? nxt : NONE;
    if constexpr (!GH_TILE_DYN) nxt += G;
    return true;
  };
  for (uint32_t k = 0;; k += NSET) {
    if (!body(std::integral_constant<int, 0>{}, k)) break;
    if constexpr (NSET == 2) {
      if (!body(std::integral_constant<int, NSET - 1>{}, k + 1)) break;
    }
  }
#if GH_TILE_STAMPS
  if (tid == 0) {
    wring[2] = __builtin_amdgcn_s_memtime();
    wring[3] = __builtin_amdgcn_s_memrealtime();
  }
#endif
}
