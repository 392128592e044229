// Tile kernel: the decode of grouped codes (complete, 4 <= len <= 12, e.g. BASELINE's
// r = 0.1 data), included by gh_decode.hip.  Reference counterpart: gpu_dec_l1_l2
// (decoder/src/decoder.cu:454-730) — its per-segment count (:529-569), decoupled
// look-back (:571-653) and second decode that writes the bytes (:655-728) — as ONE
// decode pass per segment in one persistent kernel.
//
// 512-thread workgroups, three segments per lane, a tile = 1536 consecutive segments.
// Workgroup 0 is the round leader; the D = grid - 1 others decode: workgroup b takes
// tiles b, b + D, b + 2D, ... (static round robin; grid <= 2048).  Iteration k of a
// decoding workgroup:
//
//   decode tile k into registers (one codeword per lookup, G codewords per window shift;
//     a codeword is kept iff it starts before the segment end: the reference's rule)
//     - mid-decode: load the global prefix of tile k-2
//   copy tile k-2 out of staging (its prefix has had an iteration to arrive), with a
//     fixed store count; the next tile's loads are issued just before
//   wave scans of the counts -> BARRIER -> publish tile k's aggregate
//   stage tile k (aligned dword stores, a second barrier, the 1-3 head bytes); a tile
//     larger than staging (20 bytes per segment) waits for its prefix and stores its
//     bytes straight from registers
//
// The leader takes the rounds (tiles rD .. rD + D - 1) in order: it waits for a round's
// aggregates, scans them and publishes every tile's global exclusive prefix.  The start
// of the next round stays in its registers, so the serial chain of round starts never
// crosses workgroups (rotating the leader role among the decoding workgroups made every
// round pay one cross-workgroup hand-off on that chain: 0.73 vs 0.70 ms on cfg4).  A
// decoupled look-back with 512 tiles in flight needed a window of ~512 granules per tile
// and mostly took its slow path.
//
// Issue priority: the second workgroup dispatched to a CU loses issue-arbitration ties to
// the first (age order), so one slot runs ~30 % slower and the other waits for its
// prefixes.  A wave whose last prefix had to be polled is ahead of the grid and drops to
// priority 0; one that found it published is behind and takes priority 2 (cfg4 0.70 ->
// 0.68 ms; alternating the two slots' priority by iteration gave 0.747 -> 0.729 ms).

// Build knobs (make variant VFLAGS=-D...; every alternative value is measured in
// DESIGN.md's tile-kernel section, the defaults are the fastest).
#ifndef GH_TILE_TB
#define GH_TILE_TB 512
#endif
constexpr int TILE_TB = GH_TILE_TB;  // threads per workgroup
#ifndef GH_TILE_U
#define GH_TILE_U 3
#endif
#ifndef GH_TILE_NOTAIL
#define GH_TILE_NOTAIL 0  // copy-out: NS = 4 fixed stores per thread, no loop for extra chunks
#endif
#if GH_TILE_NOTAIL
#undef GH_TILE_NS
#define GH_TILE_NS 4
#endif
#ifndef GH_TILE_NS
#define GH_TILE_NS 2
#endif
#ifndef GH_TILE_WPE
#define GH_TILE_WPE 4  // waves per SIMD the kernel is compiled for (2 workgroups per CU: 128 VGPRs)
#endif
constexpr int TILE_U = GH_TILE_U;    // segments per lane
constexpr int TILE_NS = GH_TILE_NS;  // 16-byte stores per thread per copy-out (the rest of a tile loops)
#ifndef GH_TILE_SCAPB
#define GH_TILE_SCAPB 20
#endif
constexpr int TILE_SCAP = GH_TILE_SCAPB;  // staging bytes per segment (larger tiles bypass staging)
#ifndef GH_TILE_MIDG
#define GH_TILE_MIDG 2
#endif
#ifndef GH_TILE_PHI
#define GH_TILE_PHI 2
#endif
#ifndef GH_TILE_ALTPRIO
#define GH_TILE_ALTPRIO 0
#endif
#ifndef GH_TILE_PLO
#define GH_TILE_PLO 0
#endif
#ifndef GH_POLL_SLEEP
#define GH_POLL_SLEEP 2
#endif
#ifndef GH_TILE_NOZERO
#define GH_TILE_NOZERO 1  // leave the decode's output words unzeroed (bytes past the count are never kept)
#endif
#ifndef GH_TILE_MERGEWAIT
#define GH_TILE_MERGEWAIT 1
#endif
#ifndef GH_TILE_EARLY
#define GH_TILE_EARLY 0  // issue the next tile's loads before the decode instead of before the copy-out
#endif
#ifndef GH_TILE_BATCH
#define GH_TILE_BATCH 0  // copy-out: the thread's LDS reads issued together behind one wait
#endif
#ifndef GH_TILE_WPRIO
#define GH_TILE_WPRIO 0  // waves 4-7 (the second wave on each SIMD) one issue priority level up
#endif
#ifndef GH_TILE_P1MIN
#define GH_TILE_P1MIN 0  // staging phase 1: the first dwords every kept segment fills, unmasked
#endif
#ifndef GH_TILE_IOVL
#define GH_TILE_IOVL 0  // copy-out parts between the decode groups of the next tile
#endif
#ifndef GH_TILE_IOB
#define GH_TILE_IOB 2   // (IOVL) the decode group after which the prefix is checked
#endif
#ifndef GH_TILE_STAMPS
#define GH_TILE_STAMPS 0  // diagnostic builds only: per-phase s_memtime deltas of waves 0 and 4
#endif
#if GH_TILE_STAMPS
#define TSTAMP(i) (ts[i] = __builtin_amdgcn_s_memtime())
#else
#define TSTAMP(i) ((void)0)
#endif
#ifndef GH_TILE_ABLATE
#define GH_TILE_ABLATE 0  // diagnostic builds only (make variant), bits: 1 no decode, 2 no staging
                          // stores, 4 no prefix wait (a fake offset), 8 no copy-out (wrong output)
#endif
#ifndef GH_TILE_LDSPTR
#define GH_TILE_LDSPTR 0  // LUT reads as plain LDS loads instead of inline ds_read + wait
#endif
#ifndef GH_TILE_ONEASM
#define GH_TILE_ONEASM 0  // the chains' borrow counts in one asm block per lookup step
#endif
#ifndef GH_TILE_TRIM
#define GH_TILE_TRIM 1  // stop shifting window words no kept codeword can still read
#endif
#ifndef GH_TILE_NT
#define GH_TILE_NT 2  // bits: 1 payload loads nontemporal, 2 copy-out 16-byte stores nontemporal (round 4: 2)
#endif
typedef unsigned int tile_v4u __attribute__((ext_vector_type(4)));
// 16-byte global store of the copy-out (GH_TILE_NT & 2: streaming, the output is not re-read)
__device__ __forceinline__ void tile_st16(uint4* d, const uint4& v) {
  if (GH_TILE_NT & 2) __builtin_nontemporal_store(tile_v4u{v.x, v.y, v.z, v.w}, (tile_v4u*)d);
  else *d = v;
}
__device__ __forceinline__ uint4 tile_ld16(const uint32_t* s) {
  if (GH_TILE_NT & 1) {
    const tile_v4u v = __builtin_nontemporal_load((const tile_v4u*)s);
    return make_uint4(v.x, v.y, v.z, v.w);
  }
  return *(const uint4*)s;
}
#ifndef GH_TILE_W4DPP
#define GH_TILE_W4DPP 0  // look-ahead dword from the next lane (DPP wave_shl:1); lane 63 and the
                         // shard's last segment from one wave-uniform load
#endif
constexpr int TILE_MIDG = GH_TILE_MIDG;  // decode group after which the mid-decode loads are issued
constexpr int STAGE_PAD = 16;      // staging byte STAGE_PAD + i = tile byte i
// Output words per segment: a segment holds at most ceil(128 / minlen) codewords (8
// words at minlen 4, 11 at minlen 3), kept in registers as OW words per chain.

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
  unsigned int stage_bytes;      // one staging buffer
  uint4* junk;                   // padding stores: 16 bytes per thread of the grid, (TILE_NS + 2) slots
  uint4* stamps;                 // GH_TILE_STAMPS builds: [grid][2 waves][128 iterations][2] phase deltas
  // fused count + write tile kernel (gh_ftile.hip): lut = count LUT (Kc = kbits, at LDS 0)
  const uint2* lutw;             // write LUT (2^kw u64 entries {symbols, b | n << 8})
  unsigned int kw, lutw_off, lutw_bytes;  // its width, LDS offset (a multiple of 8 << kw), bytes
  unsigned int stage_off;        // LDS offset of the staging
  unsigned int last_end;         // end bit of the stream's last segment when the shard holds it (else 0)
};

// LDS of the tile kernel: LUT, two staging buffers, wave sums, leader wave totals.
inline size_t tile_lds_bytes(size_t lut_bytes, size_t stage_bytes) {
  return lut_bytes + 2 * stage_bytes + 2 * (TILE_TB / 64) * 4 * TILE_U + 4 * (TILE_TB / 64) + 32;
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

// q[u] -= ent[u]; cnt[u] = pos1 where that borrows (the codeword that reaches the
// segment end), for the U chains in one asm block.
template <int U>
__device__ __forceinline__ void borrow_count(uint32_t (&q)[U], uint32_t (&cnt)[U], const uint32_t (&ent)[U],
                                             int pos1);
template <>
__device__ __forceinline__ void borrow_count<2>(uint32_t (&q)[2], uint32_t (&cnt)[2], const uint32_t (&ent)[2],
                                                int pos1) {
  asm("v_sub_co_u32 %0, vcc, %0, %4\n\tv_cndmask_b32_e64 %2, %2, %6, vcc\n\t"
      "v_sub_co_u32 %1, vcc, %1, %5\n\tv_cndmask_b32_e64 %3, %3, %6, vcc"
      : "+v"(q[0]), "+v"(q[1]), "+v"(cnt[0]), "+v"(cnt[1])
      : "v"(ent[0]), "v"(ent[1]), "i"(pos1) : "vcc");
}
template <>
__device__ __forceinline__ void borrow_count<3>(uint32_t (&q)[3], uint32_t (&cnt)[3], const uint32_t (&ent)[3],
                                                int pos1) {
  asm("v_sub_co_u32 %0, vcc, %0, %6\n\tv_cndmask_b32_e64 %3, %3, %9, vcc\n\t"
      "v_sub_co_u32 %1, vcc, %1, %7\n\tv_cndmask_b32_e64 %4, %4, %9, vcc\n\t"
      "v_sub_co_u32 %2, vcc, %2, %8\n\tv_cndmask_b32_e64 %5, %5, %9, vcc"
      : "+v"(q[0]), "+v"(q[1]), "+v"(q[2]), "+v"(cnt[0]), "+v"(cnt[1]), "+v"(cnt[2])
      : "v"(ent[0]), "v"(ent[1]), "v"(ent[2]), "i"(pos1) : "vcc");
}

// Decode of U segments per lane on e-windows, the U chains in lock-step (their LDS
// reads are independent, so their latencies overlap).  Each group decodes G codewords
// per chain from e0:e1 and then shifts the windows (G * maxlen <= 32, so the group's
// consumed bits fit Q's low byte).  Codeword j of a segment goes to byte j of ow (v_perm,
// static index); dead codewords go there too and are never staged.  `mid()` runs once,
// after group MIDG (or at the end if the loop stops earlier).
template <int G, int U, int OW, int MINL, class Hook, class Finish>
__device__ __forceinline__ void decode_tile_grouped(uint32_t (&e)[U][5], const int (&start)[U],
                                                    const bool (&act)[U], uint32_t (&ow)[U][OW],
                                                    uint32_t (&cnt)[U], uint32_t amask, uint32_t laneoff,
                                                    Hook&& hook, Finish&& finish) {
  constexpr int S = 4 * OW;
  constexpr int NG = (S + G - 1) / G;
  uint32_t q[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    q[u] = q_init(act[u], start[u]);
    cnt[u] = 0;
    // ow needs no zeroing: byte j is written by codeword j for every j < cnt, and the
    // bytes past cnt are never kept (staging phase 2 / the copy-out's length cover them);
    // an empty asm defines the registers without an instruction (24 v_mov per iteration)
#pragma unroll
    for (int k = 0; k < OW; ++k) {
      if (GH_TILE_NOZERO) asm volatile("" : "=v"(ow[u][k]));
      else ow[u][k] = 0;
    }
  }
  int gdone = NG;  // groups run (the loop stops once no chain is live)
#pragma unroll
  for (int gi = 0; gi < NG; ++gi) {
#pragma unroll
    for (int j = 0; j < G; ++j) {
      const int pos = gi * G + j;
      if (pos < S) {
        uint32_t ent[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const uint32_t x = j == 0 ? e[u][0] : __builtin_amdgcn_alignbit(e[u][0], e[u][1], q[u]);
          if (GH_TILE_LDSPTR)  // a plain LDS load: the compiler counts lgkmcnt itself
            ent[u] = *(const __attribute__((address_space(3))) uint32_t*)(
                (const __attribute__((address_space(3))) uint8_t*)0 + ((x & amask) | laneoff));
          else
            ent[u] = lds_u32_nowait((x & amask) | laneoff);
        }
        if (!GH_TILE_LDSPTR) lds_wait(ent);
        if (GH_TILE_ONEASM) {
          // the U borrow counts in one asm block: each inline asm boundary cost an s_nop
          borrow_count<U>(q, cnt, ent, pos + 1);
        } else {
#pragma unroll
          for (int u = 0; u < U; ++u)
            asm("v_sub_co_u32 %0, vcc, %0, %2\n\t"
                "v_cndmask_b32_e64 %1, %1, %3, vcc"
                : "+v"(q[u]), "+v"(cnt[u]) : "v"(ent[u]), "i"(pos + 1) : "vcc");
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
          ow[u][pos >> 2] = __builtin_amdgcn_perm(ent[u], ow[u][pos >> 2], perm_sel(pos & 3));
      }
    }
    uint32_t qmin = 0xFFFFFFFFu;
    // Window word k holds e-positions [C + 32k, +32) after this shift, C = the bits
    // consumed so far >= (gi + 1) * G * MINL (no codeword is shorter than MINL bits).
    // A kept codeword starts before segment bit 128, e-position 127 - start + S, and its
    // lookup reads K bits: nothing at e-position >= 157 - lgr - start is read for a kept
    // codeword, so a word lying wholly at or above 157 is no longer shifted (its stale
    // bits reach only such positions; dead codewords decode garbage, never counted).
    const int CMIN = (gi + 1) * G * MINL;  // a constant once the loop is unrolled
#pragma unroll
    for (int u = 0; u < U; ++u) {
      e[u][0] = __builtin_amdgcn_alignbit(e[u][0], e[u][1], q[u]);
      if (!GH_TILE_TRIM || CMIN + 32 < 157) e[u][1] = __builtin_amdgcn_alignbit(e[u][1], e[u][2], q[u]);
      if (!GH_TILE_TRIM || CMIN + 64 < 157) e[u][2] = __builtin_amdgcn_alignbit(e[u][2], e[u][3], q[u]);
      if (!GH_TILE_TRIM || CMIN + 96 < 157) e[u][3] = __builtin_amdgcn_alignbit(e[u][3], e[u][4], q[u]);
      if (!GH_TILE_TRIM || CMIN + 128 < 157) e[u][4] = __builtin_amdgcn_alignbit(e[u][4], 0u, q[u]);
      q[u] = (q[u] & 0xFFFFFF00u) | 32u;
      qmin = min(qmin, q[u]);
    }
    hook(gi);  // a constant in the unrolled loop
    if (gi + 1 < NG && !__any(qmin < Q_LIVE)) {
      gdone = gi + 1;
      break;
    }
  }
  finish(gdone);
}

__device__ __forceinline__ void lds_st32(uint32_t a, uint32_t v) {
  asm volatile("ds_write_b32 %0, %1" ::"v"(a), "v"(v) : "memory");
}

// Aligned staging of a segment's n bytes (ow, byte 0 first) at LDS byte address o.
// Phase 1 writes the aligned dwords holding the segment's bytes, except the first one
// when o is unaligned; its last dword carries whatever ow holds past byte n.  Phase 2,
// after a workgroup barrier, writes the segment's head bytes (the 1-3 bytes of that
// skipped first dword) exactly, over the previous segment's phase-1 tail.  Every dword
// store is aligned: unaligned ds_write_b32 measured about 3x the LDS time of aligned
// ones with per-lane offsets like these.  Returns the number of head bytes.
template <int OW, int MINW = 0>
__device__ __forceinline__ uint32_t stage_aligned_p1(const uint32_t (&ow)[OW], uint32_t n, uint32_t o) {
  const uint32_t ap = ((o - 1u) & 3u) + 1u;  // 1..4: bytes from the dword base to o
  const uint32_t base = o - ap;              // dword m at base + 4m holds segment bytes [4m - ap, +4)
  const uint32_t s = 4u - ap;                // alignbyte amount
  const uint32_t last = (n + ap - 1u) >> 2;  // last dword touched
#pragma unroll
  for (int m = 1; m <= OW; ++m) {
    const uint32_t hi = m < OW ? ow[m] : 0u;
    const uint32_t r = __builtin_amdgcn_alignbyte(hi, ow[m - 1], s);
    // dwords 1..MINW are touched by every segment of >= 4 * MINW codewords (the caller
    // guarantees it for every kept segment): stored without a per-lane test
    if (m <= MINW || (uint32_t)m <= last) lds_st32(base + 4u * m, r);
  }
  return min(4u - ap, n);  // (n >= 4 - ap for every grouped code; never write past n)
}
// Phase 2: the nb (1..3) head bytes h at o (o + (nb & 1) is even).
__device__ __forceinline__ void stage_head(uint32_t o, uint32_t h, uint32_t nb) {
  if (nb & 1u) asm volatile("ds_write_b8 %0, %1" ::"v"(o), "v"(h) : "memory");
  if (nb & 2u) asm volatile("ds_write_b16 %0, %1" ::"v"(o + (nb & 1u)), "v"(h >> (8u * (nb & 1u))) : "memory");
}

// Copy a tile staged at staging byte STAGE_PAD + i = tile byte i to out[goff, goff+n)
// (n already clamped at out_cap).  Output chunk c (16 bytes, aligned to the global
// address) is staging bytes [16c + s, +16), s = 16 - (goff & 15): one unaligned
// ds_read_b128 (gfx950 LDS runs in unaligned mode).  A fixed number of store
// instructions per thread: NS 16-byte stores (interior chunks; spare threads store the
// last interior chunk again, the same bytes, merged in L2) and one byte store (a byte of
// the two partial edge chunks, or the first edge byte again); the thread's junk slot
// only when there is nothing to duplicate.  gfx950 counts loads and stores in one
// in-order queue (vmcnt): with a fixed store count after the next tile's prefetch loads
// the compiler waits for those loads with vmcnt(NS + 1) instead of vmcnt(0), so a wave
// no longer waits for its previous copy-out's stores to be acknowledged.  Chunks beyond
// NS per thread (a tile larger than 16 * NS * TB bytes) loop.  stg: absolute LDS byte
// address of the staging buffer.
template <int TBK, int NS, bool TAIL>
__device__ __forceinline__ void copy_out_tile(uint8_t* out, uint32_t stg, unsigned long long goff, uint32_t n,
                                              int tid, uint4* junk) {
  const uint32_t lb = (uint32_t)(goff & 15);
  uint8_t* o = out + (goff - lb);          // 16-byte aligned
  const uint32_t src = stg + 16u - lb;     // staging address of output chunk 0
  const uint32_t cf = lb ? 1u : 0u;        // interior chunks [cf, ce)
  const uint32_t ce = n ? (lb + n) >> 4 : 0u;
  const bool have = ce > cf;
  if constexpr (TAIL && GH_TILE_BATCH) {
    // every read of this thread's chunks and edge byte issued, then one wait, then the
    // stores (one LDS round trip instead of one per chunk)
    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
    v4u v[NS];
    uint32_t cs[NS];
    v4u* d[NS];
#pragma unroll
    for (int i = 0; i < NS; ++i) {
      const uint32_t c = cf + (uint32_t)tid + (uint32_t)(TBK * i);
      const bool real = c < ce;
      cs[i] = real ? c : ce - 1u;
      asm volatile("ds_read_b128 %0, %1" : "=v"(v[i]) : "v"(src + 16u * ((real || have) ? cs[i] : cf)) : "memory");
      d[i] = (real || have) ? (v4u*)(o + 16ull * cs[i]) : (v4u*)junk;
    }
    const uint32_t nh = (lb && n) ? min(16u, lb + n) - lb : 0u;
    const uint32_t tl = (lb + n) & 15u;
    const uint32_t nt = (n && tl && (ce > 0 || !lb)) ? tl : 0u;
    const uint32_t t = (uint32_t)tid;
    const bool hb = nh + nt > 0;
    uint32_t k = nh ? lb : 16u * ce;
    bool real = false;
    if (t < nh) {
      k = lb + t;
      real = true;
    } else if (t < nh + nt) {
      k = 16u * ce + (t - nh);
      real = true;
    }
    uint32_t b;
    asm volatile("ds_read_u8 %0, %1" : "=v"(b) : "v"(src + ((real || hb) ? k : 0u)) : "memory");
    static_assert(NS == 2 || NS == 3, "batched copy-out: 2 or 3 chunks per thread");
    if constexpr (NS == 2) asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v[0]), "+v"(v[1]), "+v"(b)::"memory");
    else asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(b)::"memory");
#pragma unroll
    for (int i = 0; i < NS; ++i) *d[i] = v[i];
    *((real || hb) ? o + k : (uint8_t*)junk) = (uint8_t)b;
    for (uint32_t c = cf + (uint32_t)tid + (uint32_t)(TBK * NS); c < ce; c += TBK)
      *(uint4*)(o + 16ull * c) = lds_u128(src + 16u * c);
    return;
  }
  if (TAIL) {
#pragma unroll
    for (int i = 0; i < NS; ++i) {
      const uint32_t c = cf + (uint32_t)tid + (uint32_t)(TBK * i);
      const bool real = c < ce;
      const uint32_t cs = real ? c : ce - 1u;
      const uint4 v = lds_u128(src + 16u * ((real || have) ? cs : cf));
      tile_st16((real || have) ? (uint4*)(o + 16ull * cs) : junk, v);
    }
    for (uint32_t c = cf + (uint32_t)tid + (uint32_t)(TBK * NS); c < ce; c += TBK)
      tile_st16((uint4*)(o + 16ull * c), lds_u128(src + 16u * c));
  } else {
    // NS x TBK chunks cover every staged tile (the host sizes NS): no loop, so the
    // store count is fixed and the next iteration's wait for its prefetched loads
    // (issued before these stores) does not wait for these stores' acknowledgements.
    // A store past the tile rewrites the thread's first chunk (same bytes, its own
    // address: no two threads pad onto one line); no LDS read for it.
    const uint32_t c0 = cf + (uint32_t)tid;
    const bool real0 = c0 < ce;
    const uint32_t cs0 = real0 ? c0 : (have ? ce - 1u : cf);
    const uint4 v0 = lds_u128(src + 16u * cs0);
    uint4* const d0 = (real0 || have) ? (uint4*)(o + 16ull * cs0) : junk;
    tile_st16(d0, v0);
#pragma unroll
    for (int i = 1; i < NS; ++i) {
      const uint32_t c = c0 + (uint32_t)(TBK * i);
      uint4 v = v0;
      uint4* d = d0;
      if (c < ce) {
        v = lds_u128(src + 16u * c);
        d = (uint4*)(o + 16ull * c);
      }
      tile_st16(d, v);
    }
  }
  // edge bytes: the head chunk's [lb, min(16, lb + n)) when lb != 0, then the tail
  // chunk's [0, (lb + n) & 15) when it is another chunk; one byte per thread
  const uint32_t nh = (lb && n) ? min(16u, lb + n) - lb : 0u;
  const uint32_t tl = (lb + n) & 15u;
  const uint32_t nt = (n && tl && (ce > 0 || !lb)) ? tl : 0u;
  const uint32_t t = (uint32_t)tid;
  const bool hb = nh + nt > 0;
  uint32_t k = nh ? lb : 16u * ce;  // output byte offset from o (padding: the first edge byte)
  bool real = false;
  if (t < nh) {
    k = lb + t;
    real = true;
  } else if (t < nh + nt) {
    k = 16u * ce + (t - nh);
    real = true;
  }
  uint32_t b;
  asm volatile("ds_read_u8 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(b) : "v"(src + ((real || hb) ? k : 0u)) : "memory");
  *((real || hb) ? o + k : (uint8_t*)junk) = (uint8_t)b;
}

// The copy-out of copy_out_tile<TBK, NS, true> cut into parts (GH_TILE_IOVL): chunk i
// of every thread, then the edge byte, then the loop over chunks beyond NS per thread,
// so that the parts can run between the decode groups of the next tile.
template <int TBK, int NS>
struct CopyParts {
  uint8_t* o = nullptr;
  uint32_t src = 0, cf = 0, ce = 0, lb = 0, n = 0;
  bool have = false;
  __device__ __forceinline__ void init(uint8_t* out, uint32_t stg, unsigned long long goff, uint32_t n_) {
    n = n_;
    lb = (uint32_t)(goff & 15);
    o = out + (goff - lb);
    src = stg + 16u - lb;
    cf = lb ? 1u : 0u;
    ce = n ? (lb + n) >> 4 : 0u;
    have = ce > cf;
  }
  __device__ __forceinline__ void chunk(int i, int tid, uint4* junk) const {
    const uint32_t c = cf + (uint32_t)tid + (uint32_t)(TBK * i);
    const bool real = c < ce;
    const uint32_t cs = real ? c : ce - 1u;
    const uint4 v = lds_u128(src + 16u * ((real || have) ? cs : cf));
    *((real || have) ? (uint4*)(o + 16ull * cs) : junk) = v;
  }
  __device__ __forceinline__ void edge(int tid, uint4* junk) const {
    const uint32_t nh = (lb && n) ? min(16u, lb + n) - lb : 0u;
    const uint32_t tl = (lb + n) & 15u;
    const uint32_t nt = (n && tl && (ce > 0 || !lb)) ? tl : 0u;
    const uint32_t t = (uint32_t)tid;
    const bool hb = nh + nt > 0;
    uint32_t k = nh ? lb : 16u * ce;
    bool real = false;
    if (t < nh) {
      k = lb + t;
      real = true;
    } else if (t < nh + nt) {
      k = 16u * ce + (t - nh);
      real = true;
    }
    uint32_t b;
    asm volatile("ds_read_u8 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(b) : "v"(src + ((real || hb) ? k : 0u)) : "memory");
    *((real || hb) ? o + k : (uint8_t*)junk) = (uint8_t)b;
  }
  __device__ __forceinline__ void tail(int tid) const {
    for (uint32_t c = cf + (uint32_t)tid + (uint32_t)(TBK * NS); c < ce; c += TBK)
      *(uint4*)(o + 16ull * c) = lds_u128(src + 16u * c);
  }
};

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
    __builtin_amdgcn_s_sleep(GH_POLL_SLEEP);
  }
}

// The round leader (workgroup 0): for every round r of D = grid - 1 tiles, wait for the
// round's aggregates (thread t takes the A = ceil(D / TB) <= LEAD_A consecutive tiles
// t*A .. t*A + A - 1 of the round), scan them and publish each tile's global exclusive
// prefix; R, the start of the round, stays in a register.  (Spreading the rounds over the
// leader's waves, eight rounds' loads in flight, measured slower.)
constexpr int LEAD_A = 4;
template <int TB>
__device__ __forceinline__ void tile_round_leader(const TileParams& p, uint32_t* s_lead, int tid, int lane, int wid) {
  const uint32_t D = gridDim.x - 1;
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
    __syncthreads();
  }
}

// TB threads, U segments per lane, GRP codewords per window shift, OW output words per
// segment, codewords of at least MINL bits.  Compiled for at most 4 waves per SIMD (two
// workgroups per CU: 128 VGPRs).
template <int TB, int U, int GRP, int OW, int MINL>
__global__ __launch_bounds__(TB) __attribute__((amdgpu_waves_per_eu(GH_TILE_WPE, GH_TILE_WPE))) void gh_tile_kernel(const TileParams p) {
  static_assert(4 * OW >= (128 + MINL - 1) / MINL, "OW words hold every codeword a segment can start");
  static_assert(U * (TB / 64) <= 2 * TILE_U * (TB / 64), "wave sums fit tile_lds_bytes");
  constexpr int NWAVE_T = TB / 64;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint8_t* s_stage = smem + p.lut_bytes;                        // 2 buffers
  uint32_t* s_wsum = (uint32_t*)(s_stage + 2 * p.stage_bytes);  // [2][U][NWAVE_T]
  uint32_t* s_lead = s_wsum + 2 * U * NWAVE_T;                  // [NWAVE_T] (leader)

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  if (blockIdx.x == 0) {
    tile_round_leader<TB>(p, s_lead, tid, lane, wid);
    return;
  }
  {  // LUT to LDS, replicated: dword i of LDS = entry i >> lgr (lane l reads copy l mod 2^lgr,
     // so up to 32 lanes of a ds_read_b32 hit distinct banks)
    const uint32_t nd = p.lut_bytes >> 2;
    uint32_t* sl = (uint32_t*)smem;
    for (uint32_t i = tid; i < nd; i += TB) sl[i] = p.lut[i >> p.lgr];
  }
  const uint32_t S = 30u - p.kbits - p.lgr;
  const uint32_t amask = ((1u << p.kbits) - 1u) << (2u + p.lgr);
  const uint32_t laneoff = ((uint32_t)lane & ((1u << p.lgr) - 1u)) << 2;
  check_lds_base(smem, p.status);

  const uint32_t G = gridDim.x - 1, b = blockIdx.x - 1;  // decoding workgroups, this one
  const uint32_t nseg = (uint32_t)p.nseg;                 // < 2^31 (checked by the host)
  constexpr uint32_t NONE = 0xFFFFFFFFu;
  __syncthreads();
  const uint32_t last_tile_k = b < p.ntiles ? (p.ntiles - 1 - b) / G : NONE;
  uint32_t cur = b, nxt = b + G;
  uint4 w[U];
  uint32_t w4[U], gw[U];
  auto load = [&](uint32_t t) {
    const uint32_t seg0 = min(t, p.ntiles - 1) * (uint32_t)(U * TB) + (uint32_t)tid;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t sc = min(seg0 + (uint32_t)(u * TB), nseg - 1);
      w[u] = tile_ld16(p.payload + 4ull * sc);
      if (GH_TILE_W4DPP) {  // lane 63's look-ahead (every lane the same address)
        const uint32_t s63 = min(seg0 - (uint32_t)lane + 63u + (uint32_t)(u * TB), nseg - 1);
        w4[u] = p.payload[4ull * s63 + 4];
      } else {
        w4[u] = p.payload[4ull * sc + 4];
      }
      gw[u] = p.gaps[(p.gap_nib0 + (sc ? sc - 1u : 0u)) >> 3];
    }
  };
  load(cur);
  {  // as many stores after these loads as every iteration issues after its prefetch
     // (the copy-out's TILE_NS + 1): the loop's entry then matches its back edge, and
     // the compiler waits for the loads with a counted vmcnt instead of vmcnt(0)
    const unsigned long long slot = (unsigned long long)blockIdx.x * TB + tid, nslot = (unsigned long long)gridDim.x * TB;
#pragma unroll
    for (int i = 0; i <= TILE_NS; ++i) p.junk[slot + (unsigned long long)(i + 1) * nslot] = make_uint4(0, 0, 0, 0);
  }
  if (cur >= p.ntiles) cur = NONE;
  uint32_t t1 = NONE, t2 = NONE;  // tiles of iterations k-1, k-2
  uint32_t tot1 = 0, tot2 = 0;    // their totals
  uint32_t buf = 0;               // k & 1
  bool ahead = false;             // the last prefix had to be polled
  unsigned long long gpc = 0;     // (IOVL) prefix of the next iteration's tile k-2, loaded early
#if GH_TILE_STAMPS
  unsigned long long ts[9];
#endif
  for (uint32_t k = 0;; ++k) {
    TSTAMP(0);
    const bool have_cur = cur < p.ntiles;
    const bool have2 = t2 < p.ntiles;  // tile k-2 is copied out this iteration
    if (!have_cur && t1 >= p.ntiles && !have2) break;
    if (last_tile_k != NONE && k > last_tile_k + 4) {  // cannot happen; never hang the GPU
      if (tid == 0) atomicOr(p.status, (unsigned)GH_ST_TIMEOUT);
      break;
    }
    const uint32_t par = k & 1u;
    if (GH_TILE_ALTPRIO) {
      // the two workgroups of a CU (whichever they are: consecutive indices or 256
      // apart) take turns at the higher issue priority, so the younger one is not
      // always second (it otherwise ran ~5 % slower and the rounds waited for it)
      const uint32_t turn = (k + blockIdx.x + (blockIdx.x >> 8)) & 1u;
      if (turn) __builtin_amdgcn_s_setprio(2);
      else __builtin_amdgcn_s_setprio(1);
    } else if (GH_TILE_WPRIO && wid >= 4) {
      if (ahead) __builtin_amdgcn_s_setprio(GH_TILE_PLO + 1);
      else __builtin_amdgcn_s_setprio(GH_TILE_PHI + 1);
    } else {
      if (ahead) __builtin_amdgcn_s_setprio(GH_TILE_PLO);
      else __builtin_amdgcn_s_setprio(GH_TILE_PHI);
    }
    // prefix of tile k-2 (lane 0 of every wave): loaded mid-decode (a load issued at the
    // top often saw the value a little before it was published, and the re-poll then
    // paid a full memory round trip)
    unsigned long long gp = GH_TILE_IOVL ? gpc : 0ull;
    auto mid = [&]() {
      if (!GH_TILE_IOVL && have2 && lane == 0 && !(GH_TILE_ABLATE & 4))
        gp = __hip_atomic_load(&p.prefix[t2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    // ---- the prefix of tile k-2 -> its output offset (lane 0 of every wave) -----------
    unsigned long long goff = 0;
    uint32_t n2 = 0;
    auto prefix_check = [&]() {
      if (have2 && (GH_TILE_ABLATE & 4)) {
        goff = ((unsigned long long)t2 * (U * TB * 16)) % (p.out_cap - (U * TB * 32));
        n2 = tot2;
      } else if (have2) {
        bool polled = false, got = true;
        if (lane == 0) {
          polled = !granule_ok(p, gp, 2);
          if (polled) {
            if (wid == 0) atomicAdd(p.stats, 1ull);
            gp = poll_granule(p, &p.prefix[t2], 2);
            got = granule_ok(p, gp, 2);  // false only after a timeout (then nothing is written)
          }
          goff = gp & GRAN_VMASK;
          if (wid == 0 && t2 == p.ntiles - 1 && got) *p.total = goff + tot2;
        }
        goff = rfl_u64(goff);
        ahead = __builtin_amdgcn_readfirstlane(polled ? 1 : 0) != 0;
        got = __builtin_amdgcn_readfirstlane(got ? 1 : 0) != 0;
        n2 = (!got || goff >= p.out_cap) ? 0u : (uint32_t)min<unsigned long long>(tot2, p.out_cap - goff);
      }
    };
    // (IOVL) the copy-out of tile k-2 in parts after decode groups IOB .. IOB + NS
    CopyParts<TB, TILE_NS> co;
    uint4* const jk = p.junk + (unsigned long long)blockIdx.x * TB + tid;
    auto co_part = [&](int j) {
      if (j == 0) {
        prefix_check();
        co.init(p.out, p.lut_bytes + buf * p.stage_bytes, goff, n2);
      }
      if (j < TILE_NS) co.chunk(j, tid, jk);
      else co.edge(tid, jk);
    };
    auto hook = [&](int gi) {
      if (GH_TILE_IOVL) {
        if (gi >= GH_TILE_IOB && gi <= GH_TILE_IOB + TILE_NS) co_part(gi - GH_TILE_IOB);
      } else if (gi == TILE_MIDG) {
        mid();
      }
    };
    auto finish = [&](int gdone) {
      if (GH_TILE_IOVL) {
#pragma unroll
        for (int j = 0; j <= TILE_NS; ++j)
          if (gdone <= GH_TILE_IOB + j) co_part(j);
        co.tail(tid);
        // then the prefix of tile k-1 (the next iteration's copy-out; published about
        // an iteration ago) and the next tile's words, in that order: the copy-out's
        // stores are older than both, and the top of the next iteration waits only for
        // the loads (the stores, issued during the decode, have long completed)
        if (lane == 0 && t1 < p.ntiles && !(GH_TILE_ABLATE & 4))
          gpc = __hip_atomic_load(&p.prefix[t1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        load(nxt);
      } else if (gdone <= TILE_MIDG) {
        mid();
      }
    };
    // ---- decode this tile (its words were loaded during the previous iteration) --------
    const uint32_t seg0 = cur * (uint32_t)(U * TB) + (uint32_t)tid;
    uint32_t ow[U][OW], cnt[U];
    {
      int start[U];
      bool act[U];
      uint32_t e[U][5];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t seg = seg0 + (uint32_t)(u * TB);
        act[u] = have_cur && seg < nseg;
        start[u] = seg == 0 ? (int)p.first_start : (int)gap_nib(gw[u], p.gap_nib0 + seg - 1u);
        uint32_t la = w4[u];
        if (GH_TILE_W4DPP) {
          // segment seg + 1's first dword is the next lane's w.x (wave_shl:1; lane 63 keeps
          // the uniform load, and so does the shard's last segment, whose look-ahead is
          // the zero padding past it)
          const uint32_t nx = (uint32_t)__builtin_amdgcn_update_dpp((int)w4[u], (int)w[u].x, 0x130, 0xf, 0xf, false);
          la = (lane == 63 || seg + 1u >= nseg) ? w4[u] : nx;
        }
        make_ewin(w[u], la, start[u], S, e[u]);
      }
      TSTAMP(1);
      // GH_TILE_EARLY: the next tile's loads right here, into the registers the windows
      // were just built from, so they have the whole iteration to arrive (the prefix
      // load issued mid-decode then waits behind them in the in-order vmcnt queue)
      if (GH_TILE_EARLY) load(nxt);
      // Decoded unconditionally: in the last iterations (no tile) every chain is inactive
      // and the loop stops after one group (the loads were issued, clamped to the last
      // tile).  A branch around the decode made the compiler zero the 24 output words
      // before it every iteration, and merge at the scans a path on which the loads
      // were not yet waited for: a vmcnt(0) after every decode, which also waited there
      // for the mid-decode prefix load.  (GH_TILE_MERGEWAIT=0: the old branch.)
      if (GH_TILE_ABLATE & 1) {  // diagnostic build: no decode, 16 bytes per segment (wrong output)
#pragma unroll
        for (int u = 0; u < U; ++u) {
          cnt[u] = act[u] ? 16u : 0u;
#pragma unroll
          for (int k2 = 0; k2 < OW; ++k2) ow[u][k2] = e[u][k2 % 5];
        }
        finish(0);
      } else if (GH_TILE_MERGEWAIT || have_cur) {
        decode_tile_grouped<GRP, U, OW, MINL>(e, start, act, ow, cnt, amask, laneoff, hook, finish);
      } else {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          cnt[u] = 0;
#pragma unroll
          for (int k2 = 0; k2 < OW; ++k2) ow[u][k2] = 0;
        }
        finish(0);
      }
    }
    // wave scans of the counts, before the copy-out: placed after it, the compiler waited
    // for every outstanding load and store (vmcnt(0)) in the middle of the scans
    // (the U scans are independent: issued together, their DPP steps interleave without
    // the wait states one scan alone needs; then one exec-masked block for the stores)
    TSTAMP(2);
    uint32_t bpos[U], incl[U];
#pragma unroll
    for (int u = 0; u < U; ++u) incl[u] = wave_incl_scan(cnt[u]);
    if (lane == 63) {
#pragma unroll
      for (int u = 0; u < U; ++u) s_wsum[(par * U + u) * NWAVE_T + wid] = incl[u];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) bpos[u] = incl[u] - cnt[u];
    TSTAMP(3);
    // ---- copy tile k-2 out (its prefix was published about an iteration ago) ----------
    // (one call site of load(nxt), after the prefix check: with a call in each branch the
    // compiler hoisted the loads above the check, whose vmcnt(0) then waited for them)
    if (!GH_TILE_IOVL) prefix_check();
    TSTAMP(4);
    if (!GH_TILE_EARLY && !GH_TILE_IOVL) load(nxt);  // the next tile's words, issued before this copy-out's stores
    // Unconditional (no tile two iterations back: n2 = 0, every store goes to the thread's
    // junk slot): the same store count on every path lets the compiler wait for the
    // prefetched loads with a counted vmcnt at the top of the next iteration.
    if (!(GH_TILE_ABLATE & 8) && !GH_TILE_IOVL)
      copy_out_tile<TB, TILE_NS, !GH_TILE_NOTAIL>(p.out, p.lut_bytes + buf * p.stage_bytes, goff,
                                                   n2, tid,
                                                   p.junk + (unsigned long long)blockIdx.x * TB + tid);
    TSTAMP(5);
    __syncthreads();  // tile sums
    TSTAMP(6);
    // the U x NWAVE_T wave sums in chain-then-wave order, one per lane, scanned with DPP:
    // wave w's chain-u segments start at the exclusive prefix of entry u * NWAVE_T + w
    static_assert(U * NWAVE_T <= 64, "one wave sum per lane");
    const uint32_t xs = lane < U * NWAVE_T ? s_wsum[par * U * NWAVE_T + lane] : 0u;
    const uint32_t xi = wave_incl_scan(xs);
#pragma unroll
    for (int u = 0; u < U; ++u) bpos[u] += (uint32_t)__builtin_amdgcn_readlane((int)(xi - xs), u * NWAVE_T + wid);
    const uint32_t tile_total = (uint32_t)__builtin_amdgcn_readlane((int)xi, U * NWAVE_T - 1);
    if (tid == 0 && have_cur)
      __hip_atomic_store(&p.granules[cur], granule(p.epoch, 1, tile_total), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // staging holds a tile of up to stage_bytes - STAGE_PAD - 48 bytes (sized for the
    // typical tile, not the worst case: see tile_setup); a larger tile waits for its own
    // prefix here and stores its bytes straight from registers
    const bool staged = have_cur && tile_total + (uint32_t)(STAGE_PAD + 48) <= p.stage_bytes;
    if (have_cur && !staged) {
      unsigned long long goff = 0;
      bool got = true;
      if (lane == 0) {
        unsigned long long g = __hip_atomic_load(&p.prefix[cur], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (!granule_ok(p, g, 2)) g = poll_granule(p, &p.prefix[cur], 2);
        got = granule_ok(p, g, 2);  // false only after a timeout (then nothing is written)
        goff = g & GRAN_VMASK;
        if (wid == 0 && cur == p.ntiles - 1 && got) *p.total = goff + tile_total;
      }
      goff = rfl_u64(goff);
      if (__builtin_amdgcn_readfirstlane(got ? 1 : 0)) {
#pragma unroll
        for (int u = 0; u < U; ++u) store_direct(p.out, p.out_cap, goff + bpos[u], ow[u], cnt[u]);
      }
      // (rare path) drain its data-dependent loads and stores here, so that the
      // compiler's wait for the next tile's loads stays a counted vmcnt on the common path
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    } else if (have_cur) {
      // stage this tile into buffer k & 1 (copied out two iterations later) at its
      // absolute LDS address (the kernel's LDS starts at 0)
      const uint32_t sbase = p.lut_bytes + buf * p.stage_bytes + STAGE_PAD;
      uint32_t nb[U], hv[U], ha[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        nb[u] = 0;
        hv[u] = ow[u][0];
        ha[u] = sbase + bpos[u];
        // a kept segment spans >= 113 bits, so it holds >= ceil(113 / maxlen) codewords
        // (>= 12 when GRP >= 3, >= 10 otherwise; the stream's last segment may hold fewer,
        // and its extra dwords land in the staging margin behind the tile)
        constexpr int MINW = GH_TILE_P1MIN ? (GRP >= 3 ? 3 : 2) : 0;
        if (cnt[u] && !(GH_TILE_ABLATE & 2)) nb[u] = stage_aligned_p1<OW, MINW>(ow[u], cnt[u], ha[u]);
      }
      TSTAMP(7);
      __syncthreads();  // phase 1 done: every segment's tail dword is in place
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (nb[u]) stage_head(ha[u], hv[u], nb[u]);
    }
#if GH_TILE_STAMPS
    TSTAMP(8);
    if (!(have_cur && staged)) ts[7] = ts[8];
    if (lane == 0 && (wid & 3) == 0 && k < 128) {
      uint4* st = p.stamps + (((unsigned long long)blockIdx.x * 2 + (wid >> 2)) * 128 + k) * 2;
      st[0] = make_uint4((uint32_t)(ts[1] - ts[0]), (uint32_t)(ts[2] - ts[1]), (uint32_t)(ts[3] - ts[2]),
                         (uint32_t)(ts[4] - ts[3]));
      st[1] = make_uint4((uint32_t)(ts[5] - ts[4]), (uint32_t)(ts[6] - ts[5]), (uint32_t)(ts[7] - ts[6]),
                         (uint32_t)(ts[8] - ts[7]));
    }
#endif
    t2 = t1;
    tot2 = tot1;
    t1 = staged ? cur : NONE;
    tot1 = tile_total;
    buf ^= 1u;
    cur = nxt < p.ntiles ? nxt : NONE;
    nxt += G;
  }
}
