// gh_decode.hip — MI355X (gfx950) gap-array Huffman decoder: kernel + host context.
//
// Replaces the reference hot path gpu_dec_l1_l2 (Huffman_coding_Gap_arrays/decoder/
// src/decoder.cu:454-730) and its launcher decoder_l1_l2 (decoder.cu:732-815).
//
// Semantics kept from the reference:
//   * segment i (128 bits = 4 payload words) starts at bit 128*i + gap[i-1], the
//     gap being a 4-bit nibble, 8 per u32 (decoder.cu:501-507);
//   * a segment decodes every codeword that starts inside it (decoder.cu:529-569);
//   * outputs are concatenated in segment order via an exclusive scan of the
//     per-segment symbol counts with a decoupled look-back across tiles
//     (decoder.cu:571-653);
//   * the segment is decoded again to emit bytes (decoder.cu:655-728).
// Re-designed for CDNA4 rather than translated:
//   * 64-lane wavefront scans (ballot/shuffle), one 256-thread workgroup = one tile
//     of 256 segments, persistent grid with an atomic tile ticket;
//   * a multi-symbol lookup table (up to 4 symbols per lookup) staged in LDS, built
//     on the host from the (symbol,length) list for the real maximum length (the
//     reference's fixed 10-bit table is wrong when maxlen <= 10);
//     codes longer than the table width use a canonical limit search;
//   * the segment's 5 words live in an LDS slot and the 32-bit window at bit P is
//     one v_alignbit of two words — no 32-bit shift-by-32;
//   * look-back granules are {epoch, flag, value} in one 8-byte agent-scope atomic
//     (no per-call memset, no fences: the data is the flag);
//   * pass 2 writes the tile's bytes into an LDS staging buffer at their final
//     byte alignment; the tile is then stored with 16-byte global stores, the two
//     partial edge chunks with byte stores (no atomicOr on global memory), and
//     everything is clamped at the shard's output capacity (the reference wrote
//     past N, decoder.cu:672-728).
#include <hip/hip_runtime.h>

#include <map>
#include <mutex>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "gh_internal.hpp"

namespace gh {

constexpr int TB = 256;                  // workgroup size of the multi-symbol paths
constexpr int TB_G = 512;                // workgroup size of the grouped single-symbol path
constexpr int MAX_NWAVE = TB_G / 64;
constexpr int FB_WORDS = 3 * 17 + 64;    // limit16/base16/first + 256 symbol bytes
constexpr int FB_BYTES = ((4 * FB_WORDS) + 15) & ~15;
constexpr int MAX_SUPER = 8;             // sub-tiles per super-tile (template values 1,2,4,8)
constexpr int SCRATCH_BYTES = 4 * (MAX_SUPER * MAX_NWAVE + 8) + 16 * MAX_NWAVE + 16;
constexpr uint32_t EPOCH_MAX = (1u << 24) - 1;
constexpr uint32_t SPIN_LIMIT = 1u << 18;

struct DecodeParams {
  const uint32_t* payload;       // local segment j owns words [4j, 4j+4); +1 look-ahead, zero padded
  const uint32_t* gaps;          // gap words; nibble (gap_nib0 + j - 1) = start of local segment j>=1
  const uint4* lut;              // 2^K entries as {syms, meta} pairs (8 bytes)
  const uint32_t* fb;            // fallback tables
  uint8_t* out;                  // shard output
  unsigned long long* granules;  // one per super-tile
  unsigned int* ticket;
  unsigned int* status;
  unsigned long long* total;     // shard symbol total (written by the last super-tile)
  unsigned long long out_cap;
  unsigned long long nseg;
  unsigned int gap_nib0;
  unsigned int first_start;
  unsigned int nsuper;           // super-tiles of S*TB segments
  unsigned int kbits;
  unsigned int epoch;
  unsigned int lut_bytes;
  unsigned int stage_bytes;
  unsigned int fb_lo, fb_hi;     // fallback length range
  unsigned long long* stamps;    // diagnostic build only (GH_STAMPS): per-block phase cycles
  unsigned int ablate;           // diagnostic build only: 1 no resolve, 2 no copy-out, 4 no stage
  unsigned int sched;            // 0: tiles from the atomic ticket; 1: static round robin
  // split mode (count kernel -> scan kernel -> write kernel)
  uint8_t* seg_cnt;              // codewords kept per segment (<= 128)
  unsigned int* tile_cnt;        // codewords per tile
  unsigned long long* tile_off;  // (unused)
  unsigned long long* wg_tot;    // codewords per workgroup range (count kernel)
  unsigned int count_per;        // count workgroups per write workgroup
};
#ifdef GH_STAMPS
#define ABLATE(bit) (p.ablate & (bit))
#else
#define ABLATE(bit) 0
#endif

// Diagnostic phase stamps (compiled only with -DGH_STAMPS; never in the shipped
// library): lane 0 of wave 0 accumulates s_memtime deltas per phase.
#ifdef GH_STAMPS
#define GH_NSTAMP 10
#define STAMP_DECL unsigned long long st_acc[GH_NSTAMP] = {}; unsigned long long st_last = __builtin_amdgcn_s_memtime();
#define STAMP(i) do { if (tid == 0) { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); st_acc[i] += t_ - st_last; st_last = t_; } } while (0)
#define STAMP_FLUSH do { if (tid == 0 && p.stamps) { for (int i_ = 0; i_ < GH_NSTAMP; ++i_) p.stamps[blockIdx.x * 16 + i_] = st_acc[i_]; } } while (0)
#else
#define STAMP_DECL
#define STAMP(i) do {} while (0)
#define STAMP_FLUSH do {} while (0)
#endif

// ---- meta word of a LUT entry -------------------------------------------------
//  [4:0]   (32 - b) & 31: the v_alignbit amount that advances the window by b bits
//  [12:8]  b, bits consumed (0 for a fallback entry)
//  [18:16] n, symbols decoded (0 = codeword longer than K or invalid: fallback)
//  [23:20] e1, [27:24] e2, [31:28] e3: end of symbol k = start of symbol k+1
//          (15 when absent); used to drop symbols that start past the segment.
__device__ __forceinline__ uint32_t meta_n(uint32_t m) { return (m >> 16) & 7u; }
__device__ __forceinline__ uint32_t meta_b(uint32_t m) { return (m >> 8) & 31u; }
__host__ __device__ constexpr uint32_t make_meta(uint32_t n, uint32_t b, uint32_t e1,
                                                 uint32_t e2, uint32_t e3) {
  return ((32u - b) & 31u) | (b << 8) | (n << 16) | (e1 << 20) | (e2 << 24) | (e3 << 28);
}

// Canonical decode of a codeword longer than the LUT width (rare).  Returns
// (symbol << 8) | length; a pattern outside the code space sets GH_ST_BADCODE and
// yields the first symbol with the longest length (keeps the count bound).
__device__ __noinline__ uint32_t fallback_decode(const uint32_t* fb, uint32_t w16, uint32_t lo,
                                                 uint32_t hi, unsigned int* status) {
  const uint32_t* limit16 = fb;
  const uint32_t* base16 = fb + 17;
  const uint32_t* first = fb + 34;
  const uint8_t* syms = (const uint8_t*)(fb + 51);
  for (uint32_t l = lo; l <= hi; ++l) {
    if (w16 < limit16[l]) {
      const uint32_t idx = first[l] + ((w16 - base16[l]) >> (16 - l));
      return ((uint32_t)syms[idx & 255] << 8) | l;
    }
  }
  atomicOr(status, (unsigned)GH_ST_BADCODE);
  return ((uint32_t)syms[0] << 8) | hi;
}

template <class PRM>
__device__ __forceinline__ uint32_t fallback_meta(const uint32_t* fb, uint32_t t, const PRM& p,
                                                  uint32_t* syms) {
  const uint32_t r = fallback_decode(fb, t >> 16, p.fb_lo, p.fb_hi, p.status);
  *syms = r >> 8;
  return make_meta(1, r & 31u, 15, 15, 15);
}

// Symbols of the final lookup that start before the segment end (rem bits left).
__device__ __forceinline__ uint32_t kept_in_last(uint32_t meta, int rem) {
  const uint32_t r = (uint32_t)min(rem, 15);
  return 1u + (((meta >> 20) & 15u) < r) + (((meta >> 24) & 15u) < r) + ((meta >> 28) < r);
}

// The segment's bits live in a 160-bit funnel register d[0..4] (d[0] = the next
// 32 stream bits, MSB first).  Consuming b bits (1..16) is four v_alignbit with
// the LUT entry itself as the shift operand (alignbit reads its low 5 bits =
// 32-b) plus one shift: no shift-by-32 case and no LDS window.
// Starting at bit s <= 15 the register holds >= 145 valid bits, enough for the
// last codeword (ends by bit 143) and its lookahead.
struct Win {
  uint32_t d0, d1, d2, d3, d4;
};

__device__ __forceinline__ Win make_win(uint4 w, uint32_t w4, int s) {
  Win v;
  const uint32_t sh = (uint32_t)(32 - s);
  const bool z = (s == 0);
  v.d0 = z ? w.x : __builtin_amdgcn_alignbit(w.x, w.y, sh);
  v.d1 = z ? w.y : __builtin_amdgcn_alignbit(w.y, w.z, sh);
  v.d2 = z ? w.z : __builtin_amdgcn_alignbit(w.z, w.w, sh);
  v.d3 = z ? w.w : __builtin_amdgcn_alignbit(w.w, w4, sh);
  v.d4 = w4 << s;
  return v;
}

__device__ __forceinline__ void consume(Win& v, uint32_t meta) {
  v.d0 = __builtin_amdgcn_alignbit(v.d0, v.d1, meta);
  v.d1 = __builtin_amdgcn_alignbit(v.d1, v.d2, meta);
  v.d2 = __builtin_amdgcn_alignbit(v.d2, v.d3, meta);
  v.d3 = __builtin_amdgcn_alignbit(v.d3, v.d4, meta);
  v.d4 = v.d4 << meta_b(meta);
}

// Count pass over U segments per thread, walked in lock-step so the U LUT reads
// of an iteration are independent (ILP hides the LDS latency).  All U reads are
// issued before anything consumes them; the rare fallback is one branch for all
// chains so it does not split the read group.
template <bool FB, int U>
__device__ __forceinline__ void count_segments(Win (&v)[U], const int (&start)[U],
                                               const bool (&act)[U], uint32_t (&cnt)[U],
                                               const uint32_t* s_lut32, const uint32_t* fb,
                                               uint32_t kshift, const DecodeParams& p,
                                               uint32_t& bad) {
  int P[U], Plast[U];
  uint32_t mlast[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    P[u] = act[u] ? start[u] : 128;
    Plast[u] = P[u];
    mlast[u] = make_meta(1, 0, 15, 15, 15);
    cnt[u] = 0;
  }
  bool any;
  do {
    uint32_t meta[U];
#pragma unroll
    for (int u = 0; u < U; ++u) meta[u] = s_lut32[2 * (v[u].d0 >> kshift) + 1];
    if constexpr (FB) {
      bool need = false;
#pragma unroll
      for (int u = 0; u < U; ++u) need |= (meta_n(meta[u]) == 0) & (P[u] < 128);
      if (need) {
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (meta_n(meta[u]) == 0 && P[u] < 128) {
            uint32_t sy;
            meta[u] = fallback_meta(fb, v[u].d0, p, &sy);
          }
      }
    }
    any = false;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool live = P[u] < 128;
      if constexpr (!FB) bad |= (live && meta_n(meta[u]) == 0) ? 1u : 0u;
      cnt[u] += live ? meta_n(meta[u]) : 0u;
      Plast[u] = live ? P[u] : Plast[u];
      mlast[u] = live ? meta[u] : mlast[u];
      // an invalid pattern (no-fallback build) still advances so the loop ends
      P[u] += FB ? (int)meta_b(meta[u]) : max((int)meta_b(meta[u]), 1);
      consume(v[u], meta[u]);
      any |= P[u] < 128;
    }
  } while (any);
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (act[u]) cnt[u] -= meta_n(mlast[u]) - kept_in_last(mlast[u], 128 - Plast[u]);
}

// Emit pass: decode again and OR the bytes into the LDS staging buffer starting at
// byte bpos[u].  A word is flushed only once a later lookup of the same segment
// starts, so the final (possibly truncated) lookup's bytes are masked first.
// Book-keeping is predicated (v_cndmask), only the LDS OR is a branch.
template <bool FB, int U>
__device__ __forceinline__ void emit_segments(Win (&v)[U], const int (&start)[U],
                                              const bool (&act)[U], const uint32_t (&bpos)[U],
                                              const uint2* s_lut, const uint32_t* fb,
                                              uint32_t kshift, const DecodeParams& p,
                                              uint32_t* stg) {
  int P[U], Plast[U];
  uint32_t mlast[U], oidx[U], fill[U];
  unsigned long long acc[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    P[u] = act[u] ? start[u] : 128;
    Plast[u] = P[u];
    mlast[u] = make_meta(1, 0, 15, 15, 15);
    oidx[u] = bpos[u] >> 2;
    fill[u] = 8u * (bpos[u] & 3u);
    acc[u] = 0;
  }
  bool any;
  do {
    uint2 e[U];
#pragma unroll
    for (int u = 0; u < U; ++u) e[u] = s_lut[v[u].d0 >> kshift];
    if constexpr (FB) {
      bool need = false;
#pragma unroll
      for (int u = 0; u < U; ++u) need |= (meta_n(e[u].y) == 0) & (P[u] < 128);
      if (need) {
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (meta_n(e[u].y) == 0 && P[u] < 128) e[u].y = fallback_meta(fb, v[u].d0, p, &e[u].x);
      }
    }
    any = false;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool live = P[u] < 128;
      const uint32_t meta = e[u].y;
      // flush the word completed by earlier lookups (OR of 0 when none): no branch
      const bool flush = live && fill[u] >= 32;
      atomicOr(&stg[oidx[u]], flush ? (uint32_t)acc[u] : 0u);
      acc[u] = flush ? (acc[u] >> 32) : acc[u];
      fill[u] -= flush ? 32u : 0u;
      oidx[u] += flush ? 1u : 0u;
      acc[u] |= live ? ((unsigned long long)e[u].x << fill[u]) : 0ull;
      fill[u] += live ? 8u * meta_n(meta) : 0u;
      Plast[u] = live ? P[u] : Plast[u];
      mlast[u] = live ? meta : mlast[u];
      P[u] += FB ? (int)meta_b(meta) : max((int)meta_b(meta), 1);
      consume(v[u], meta);
      any |= P[u] < 128;
    }
  } while (any);
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if (!act[u]) continue;
    uint32_t f = fill[u] - 8u * (meta_n(mlast[u]) - kept_in_last(mlast[u], 128 - Plast[u]));
    const unsigned long long a = acc[u] & ((1ull << f) - 1ull);  // f < 64
    if (f > 0) atomicOr(&stg[oidx[u]], (uint32_t)a);
    if (f > 32) atomicOr(&stg[oidx[u] + 1], (uint32_t)(a >> 32));
  }
}

// Inclusive wave scan on the VALU with DPP: row_shr 1/2/4/8 scans each 16-lane row,
// row_bcast 15/31 carry the row totals forward (no LDS traffic, unlike
// ds_bpermute-based shuffles).
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, int /*lane*/) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, true);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, true);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, true);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);
  return v;
}

__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
  return v;
}

// Wave-uniform copy of a 64-bit value (lane 0's).  readfirstlane returns int: each half
// is taken as uint32_t before widening (an int low half with bit 31 set would
// sign-extend over the high half).
__device__ __forceinline__ unsigned long long rfl_u64(unsigned long long v) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
  return ((unsigned long long)hi << 32) | lo;
}

// Look-back granule: [37:0] value, [39:38] flag (1 aggregate, 2 inclusive prefix),
// [63:40] epoch of the launch that wrote it.
__device__ __forceinline__ unsigned long long granule(unsigned epoch, unsigned flag,
                                                      unsigned long long v) {
  return ((unsigned long long)epoch << 40) | ((unsigned long long)flag << 38) |
         (v & ((1ull << 38) - 1));
}

// Decoupled look-back, split so that publishing the aggregate (right after the
// count) and resolving the prefix (one tile later) are separate steps.  Resolve:
// one wave sums predecessors' aggregates back to the nearest inclusive prefix
// (256 granules per round: lane l reads distances l, l+64, l+128, l+192),
// publishes the inclusive prefix and returns the exclusive one.  Every predecessor
// publishes its aggregate right after counting, without waiting on anything, so
// the spin terminates (bounded anyway by SPIN_LIMIT).
__device__ __forceinline__ void publish_aggregate(const DecodeParams& p, uint32_t tile,
                                                  unsigned long long total) {
  __hip_atomic_store(&p.granules[tile], granule(p.epoch, tile == 0 ? 2 : 1, total),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Slow path of the look-back (one wave): rounds of 256 granules from `base` down,
// adding aggregates until an inclusive prefix; re-fetches while a predecessor
// has not published.  Returns the exclusive prefix of `tile` (does not publish).
template <class P>
__device__ unsigned long long resolve_slow(const P& p, long long base,
                                           unsigned long long excl, int lane) {
  constexpr unsigned long long VMASK = (1ull << 38) - 1;
  uint32_t spins = 0;
  for (;;) {
    unsigned long long g[4];
    uint32_t st[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const long long pi = base - lane - 64 * j;
      g[j] = 0;
      st[j] = 2;  // before the first tile: an inclusive 0
      if (pi >= 0)
        g[j] = __hip_atomic_load(&p.granules[pi], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (base - lane - 64 * j >= 0)
        st[j] = ((uint32_t)(g[j] >> 40) == p.epoch) ? (uint32_t)((g[j] >> 38) & 3u) : 0u;
    int fp = 256;  // nearest inclusive prefix: distance d = 64*j + lane
#pragma unroll
    for (int j = 3; j >= 0; --j) {
      const unsigned long long pm = __ballot(st[j] == 2);
      if (pm) fp = 64 * j + __builtin_ctzll(pm);
    }
    bool ok = true;
#pragma unroll
    for (int j = 0; j < 4; ++j) ok &= (64 * j + lane > fp) || (st[j] != 0);
    if (!__all(ok)) {
      if (++spins > SPIN_LIMIT) {
        if (lane == 0) atomicOr(p.status, (unsigned)GH_ST_TIMEOUT);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
      continue;
    }
    unsigned long long v = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (64 * j + lane <= fp && base - lane - 64 * j >= 0) v += g[j] & VMASK;
    excl += wave_sum_u64(v);
    if (fp < 256) break;
    base -= 256;
  }
  return excl;
}

// Fast path of the look-back, spread over the whole workgroup: wave w fetches the
// granules at distances [256w, 256w+256) before the tile (issued early, so the
// fabric round trip overlaps the staging), then summarises them: nearest
// inclusive prefix, whether everything up to it has published, and the sum.
struct LbSummary {
  unsigned long long sum;
  uint32_t fp;  // local distance of the nearest inclusive prefix (256: none)
  uint32_t ok;
};

__device__ __forceinline__ void lookback_issue(const DecodeParams& p, uint32_t tile, int wid,
                                               int lane, unsigned long long (&g)[4]) {
  // unconditional loads (clamped index): a skipped load would make the compiler
  // wait for every later load before the summary
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const long long pi = (long long)tile - 1 - 256 * wid - 64 * j - lane;
    g[j] = __hip_atomic_load(&p.granules[pi < 0 ? 0 : pi], __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
  }
}

__device__ __forceinline__ void lookback_summarise(const DecodeParams& p, uint32_t tile, int wid,
                                                   int lane, const unsigned long long (&g)[4],
                                                   LbSummary* out) {
  constexpr unsigned long long VMASK = (1ull << 38) - 1;
  const long long base = (long long)tile - 1 - 256 * wid;
  uint32_t st[4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
    st[j] = (base - 64 * j - lane < 0) ? 2u
            : ((uint32_t)(g[j] >> 40) == p.epoch) ? (uint32_t)((g[j] >> 38) & 3u) : 0u;
  int fp = 256;
#pragma unroll
  for (int j = 3; j >= 0; --j) {
    const unsigned long long pm = __ballot(st[j] == 2);
    if (pm) fp = 64 * j + __builtin_ctzll(pm);
  }
  bool ok = true;
  unsigned long long v = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int d = 64 * j + lane;
    ok &= (d > fp) || (st[j] != 0);
    if (d <= fp && base - d >= 0) v += g[j] & VMASK;
  }
  const bool all_ok = __all(ok);
  v = wave_sum_u64(v);
  if (lane == 0) *out = LbSummary{v, (uint32_t)fp, all_ok ? 1u : 0u};
}

// Load the U segments of a tile owned by this thread (16-byte loads, coalesced).
// The gap word is kept raw: extracting the nibble here would make the compiler
// wait for the loads right away; tile_starts() does it when the tile is decoded.
template <int U, int TBK>
__device__ __forceinline__ void load_tile(const DecodeParams& p, uint32_t tile, int tid,
                                          uint4 (&w)[U], uint32_t (&w4)[U], uint32_t (&gw)[U],
                                          bool (&act)[U]) {
  // Loads are unconditional (clamped to the last tile / segment): a load skipped
  // by a branch would make the compiler's wait counting fall back to vmcnt(0).
  const uint32_t t = min(tile, p.nsuper - 1);
  const unsigned long long seg0 = (unsigned long long)t * (U * TBK) + tid;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const unsigned long long seg = seg0 + (unsigned long long)u * TBK;
    act[u] = tile < p.nsuper && seg < p.nseg;
    const unsigned long long sc = min(seg, p.nseg - 1);
    w[u] = *(const uint4*)(p.payload + 4 * sc);
    w4[u] = p.payload[4 * sc + 4];
    gw[u] = p.gaps[((unsigned long long)p.gap_nib0 + (sc ? sc - 1 : 0)) >> 3];
  }
}

// Start bit of each segment of the tile (its gap nibble, or first_start for the
// shard's first segment).
template <int U, int TBK>
__device__ __forceinline__ void tile_starts(const DecodeParams& p, uint32_t tile, int tid,
                                            const uint32_t (&gw)[U], int (&start)[U]) {
  const unsigned long long seg0 = (unsigned long long)tile * (U * TBK) + tid;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const unsigned long long seg = seg0 + (unsigned long long)u * TBK;
    const uint32_t nib = (uint32_t)(p.gap_nib0 + seg - 1) & 7u;
    start[u] = seg == 0 ? (int)p.first_start : (int)((gw[u] >> (4 * nib)) & 15u);
  }
}

// ---------------------------------------------------------------------------
// Single-symbol path (codes with minlen >= 4, where multi-symbol lookups buy
// little, e.g. redundancy 0.1): ONE decode pass per segment.
//  * LUT entry (u32): [4:0] (32-b)&31, [12:8] b, [31:24] symbol; b = 0 marks a
//    codeword longer than K or an invalid pattern (fallback).
//  * The step loop is fully unrolled (at most 128/4 = 32 steps, checked for a
//    wave-wide exit every 4 steps), so step j's symbol goes to byte j of the
//    register out[j/4] with one v_perm: static indices, no LDS, no count pass,
//    and no truncation fixup (a lookup decodes exactly one codeword, which is
//    kept iff it starts before bit 128).
// ---------------------------------------------------------------------------
constexpr int OW = 8;  // output words per segment (32 symbols)

__device__ __forceinline__ uint32_t fallback_entry1(const uint32_t* fb, uint32_t t,
                                                    const DecodeParams& p) {
  const uint32_t r = fallback_decode(fb, t >> 16, p.fb_lo, p.fb_hi, p.status);
  const uint32_t b = r & 31u;
  return ((32u - b) & 31u) | (b << 8) | ((r >> 8) << 24);
}

// v_perm selector placing byte 3 of S0 (the symbol) at byte j, keeping S1's others.
__device__ __forceinline__ constexpr uint32_t perm_sel(int j) {
  return j == 0 ? 0x03020107u : j == 1 ? 0x03020700u : j == 2 ? 0x03070100u : 0x07020100u;
}

template <bool FB, int U>
__device__ __forceinline__ void decode1_segments(Win (&v)[U], const int (&start)[U],
                                                 const bool (&act)[U], uint32_t (&ow)[U][OW],
                                                 uint32_t (&cnt)[U], const uint32_t* s_lut32,
                                                 const uint32_t* fb, uint32_t kshift,
                                                 const DecodeParams& p, uint32_t& bad) {
  int P[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    P[u] = act[u] ? start[u] : 128;
    cnt[u] = 0;
#pragma unroll
    for (int k = 0; k < OW; ++k) ow[u][k] = 0;
  }
#pragma unroll
  for (int blk = 0; blk < OW; ++blk) {
    bool live_any = false;
#pragma unroll
    for (int u = 0; u < U; ++u) live_any |= P[u] < 128;
    if (!__any(live_any)) break;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      uint32_t e[U];
#pragma unroll
      for (int u = 0; u < U; ++u) e[u] = s_lut32[v[u].d0 >> kshift];
      if constexpr (FB) {
        bool need = false;
#pragma unroll
        for (int u = 0; u < U; ++u) need |= ((e[u] & 0x1F00u) == 0) & (P[u] < 128);
        if (need) {
#pragma unroll
          for (int u = 0; u < U; ++u)
            if ((e[u] & 0x1F00u) == 0 && P[u] < 128) e[u] = fallback_entry1(fb, v[u].d0, p);
        }
      } else {
        // an invalid pattern: flag it and step one bit so the walk still ends
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const bool inval = (e[u] & 0x1F00u) == 0;
          bad |= (inval && P[u] < 128) ? 1u : 0u;
          e[u] = inval ? (31u | (1u << 8)) : e[u];
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        ow[u][blk] = __builtin_amdgcn_perm(e[u], ow[u][blk], perm_sel(j));
        cnt[u] += (P[u] < 128) ? 1u : 0u;
        P[u] += (int)((e[u] >> 8) & 31u);
        v[u].d0 = __builtin_amdgcn_alignbit(v[u].d0, v[u].d1, e[u]);
        v[u].d1 = __builtin_amdgcn_alignbit(v[u].d1, v[u].d2, e[u]);
        v[u].d2 = __builtin_amdgcn_alignbit(v[u].d2, v[u].d3, e[u]);
        v[u].d3 = __builtin_amdgcn_alignbit(v[u].d3, v[u].d4, e[u]);
        v[u].d4 = __builtin_amdgcn_alignbit(v[u].d4, 0u, e[u]);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Grouped single-symbol path (complete codes, every codeword <= K bits, minlen
// >= 4 — e.g. redundancy 0.1).  Same static output positions as above, but the
// 160-bit window is shifted only once per group of G codewords (G*maxlen <= 31):
// inside a group the next codeword sits at bit p of d0:d1 and is extracted with
// one v_alignbit by q = 32 - p (q is decremented by the code length; the group's
// first lookup reads d0 directly, p = 0).  LUT entries are 8 bytes
// {len, sym << 24}, so q stays exact and doubles as the liveness test: a
// codeword is kept iff it starts before bit 128, i.e. q > T with T = F + 32 - L
// (F = bits flushed so far, L = 128 - start).  Dead lanes insert a zero byte, so
// the bytes past cnt are zero and staging needs no masks.  No invalid-pattern
// check: a complete prefix code decodes every bit pattern.
// ---------------------------------------------------------------------------
template <int U, int G>
__device__ __forceinline__ void decode1g(Win (&v)[U], const int (&start)[U], const bool (&act)[U],
                                         uint32_t (&ow)[U][OW], uint32_t (&cnt)[U],
                                         const uint8_t* s_lut8, uint32_t ksh8) {
  constexpr int S = 4 * OW;
  constexpr int NG = (S + G - 1) / G;
  uint32_t q[U];
  int T[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    q[u] = 32;
    T[u] = act[u] ? start[u] - 96 : 0x7FFFFFFF;  // 32 - L, L = 128 - start
    cnt[u] = 0;
#pragma unroll
    for (int k = 0; k < OW; ++k) ow[u][k] = 0;
  }
#pragma unroll
  for (int gi = 0; gi < NG; ++gi) {
#pragma unroll
    for (int j = 0; j < G; ++j) {
      const int pos = gi * G + j;
      if (pos < S) {
        uint2 e[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const uint32_t w = j == 0 ? v[u].d0 : __builtin_amdgcn_alignbit(v[u].d0, v[u].d1, q[u]);
          e[u] = *(const uint2*)(s_lut8 + ((w >> ksh8) & ~7u));
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const bool live = (int)q[u] > T[u];
          cnt[u] += live ? 1u : 0u;
          const uint32_t sb = live ? e[u].y : 0u;
          ow[u][pos >> 2] = __builtin_amdgcn_perm(sb, ow[u][pos >> 2], perm_sel(pos & 3));
          q[u] -= e[u].x;
        }
      }
    }
    // flush: shift the window left by p = 32 - q (1 <= p <= 31)
    bool more = false;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      v[u].d0 = __builtin_amdgcn_alignbit(v[u].d0, v[u].d1, q[u]);
      v[u].d1 = __builtin_amdgcn_alignbit(v[u].d1, v[u].d2, q[u]);
      v[u].d2 = __builtin_amdgcn_alignbit(v[u].d2, v[u].d3, q[u]);
      v[u].d3 = __builtin_amdgcn_alignbit(v[u].d3, v[u].d4, q[u]);
      v[u].d4 = __builtin_amdgcn_alignbit(v[u].d4, 0u, q[u]);
      T[u] += 32 - (int)q[u];
      q[u] = 32;
      more |= 32 > T[u];
    }
    if (gi + 1 < NG && !__any(more)) break;
  }
}

// Stage a segment's bytes whose tail (past n) is already zero: nine funnel-shifted
// words ORed at byte position pos.  For pos % 4 == 0 the funnel by 0 yields the
// previous word, so the words land one slot lower (slot -1 gets a harmless 0).
__device__ __forceinline__ void stage_bytes_z(uint32_t* stg, const uint32_t (&ow)[OW],
                                              uint32_t pos) {
  const uint32_t s8 = 8u * (pos & 3u);
  const uint32_t sh = (32u - s8) & 31u;
  uint32_t* base = stg + (pos >> 2) - (s8 == 0 ? 1 : 0);
  uint32_t prev = 0;
#pragma unroll
  for (int m = 0; m <= OW; ++m) {
    const uint32_t cur = m < OW ? ow[m] : 0u;
    atomicOr(base + m, __builtin_amdgcn_alignbit(cur, prev, sh));
    prev = cur;
  }
}

// OR a segment's n output bytes (held in registers) into the staging buffer at
// byte position pos.
__device__ __forceinline__ void stage_bytes(uint32_t* stg, const uint32_t (&ow)[OW], uint32_t n,
                                            uint32_t pos) {
  const uint32_t s8 = 8u * (pos & 3u);
  const uint32_t w0 = pos >> 2;
  uint32_t prev = 0;
#pragma unroll
  for (int m = 0; m <= OW; ++m) {
    uint32_t cur = 0;
    if (m < OW) {
      const int left = (int)n - 4 * m;
      const uint32_t mask = left >= 4 ? ~0u : left <= 0 ? 0u : ((1u << (8 * left)) - 1u);
      cur = ow[m] & mask;
    }
    const uint32_t x = s8 ? __builtin_amdgcn_alignbit(cur, prev, 32u - s8) : cur;
    if (4 * m < (int)((pos & 3u) + n)) atomicOr(&stg[w0 + m], x);
    prev = cur;
  }
}

// Copy a tile's staged bytes (tile-local offsets, after a 16-byte zero pad) to
// out[goff, goff+n), clamped at out_cap.  Each lane builds one 16-byte output
// chunk aligned to the global address from five aligned staging dwords and four
// v_alignbyte (the tile's global offset is only known after its look-back, so the
// staging cannot be pre-aligned); whole chunks go out as 16-byte stores, the two
// edge chunks byte by byte.
template <int TBK>
__device__ __forceinline__ void copy_out_shifted(const DecodeParams& p, const uint32_t* stg32,
                                                 unsigned long long goff, uint32_t n, int tid) {
  const uint32_t lb = (uint32_t)(goff & 15);
  const unsigned long long a0 = goff - lb;
  const unsigned long long end = min(goff + n, p.out_cap);
  const uint32_t nz = (lb + n + 15u) >> 4;
  for (uint32_t c = tid; c < nz; c += TBK) {
    const uint32_t sb = 16u * c + 16u - lb;  // staging byte of the chunk's first byte
    const uint32_t wi = sb >> 2, sh = sb & 3u;
    const uint32_t d0 = stg32[wi], d1 = stg32[wi + 1], d2 = stg32[wi + 2], d3 = stg32[wi + 3],
                   d4 = stg32[wi + 4];
    uint4 v;
    v.x = __builtin_amdgcn_alignbyte(d1, d0, sh);
    v.y = __builtin_amdgcn_alignbyte(d2, d1, sh);
    v.z = __builtin_amdgcn_alignbyte(d3, d2, sh);
    v.w = __builtin_amdgcn_alignbyte(d4, d3, sh);
    const unsigned long long gs = a0 + 16ull * c;
    if (gs >= goff && gs + 16 <= end) {
      *(uint4*)(p.out + gs) = v;
    } else {
      const uint8_t* b = (const uint8_t*)&v;
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const unsigned long long ga = gs + k;
        if (ga >= goff && ga < end) p.out[ga] = b[k];
      }
    }
  }
}

// The decode kernel.  One workgroup processes tiles of U*TB segments (thread t
// owns segments tile*U*TB + u*TB + t, so every 16-byte load is coalesced) drawn
// from an atomic ticket, software-pipelined across tiles:
//
//   iteration k:  decode/count tile k (its words were loaded during k-1)
//                 -> scan, publish tile k's aggregate, draw ticket k+1
//                 -> issue the loads of tile k+1
//                 -> resolve tile k-1's prefix (its predecessors have had a whole
//                    decode phase to publish), copy tile k-1 out
//                 -> stage tile k's bytes at tile-local offsets
//
// Staging is double-buffered; each buffer is zeroed behind the copy-out that
// drained it.  Three workgroup barriers per tile.
//   SINGLE = true : single-symbol LUT, one decode pass, bytes held in registers
//   SINGLE = false: multi-symbol LUT, count pass then emit pass.
template <bool SINGLE, bool FB, int U, int G, int TBK>
__global__ __launch_bounds__(TBK) void gh_decode_kernel(const DecodeParams p) {
  constexpr int NWAVE = TBK / 64;
  static_assert(G == 0 || (SINGLE && !FB), "grouped path: single-symbol, no fallback");
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint2* s_lut = (const uint2*)smem;
  const uint32_t* s_lut32 = (const uint32_t*)smem;
  uint32_t* s_fb = (uint32_t*)(smem + p.lut_bytes);
  uint8_t* s_stage0 = smem + p.lut_bytes + FB_BYTES;
  uint32_t* s_scr = (uint32_t*)(s_stage0 + 2 * p.stage_bytes);
  uint32_t* s_ticket = s_scr + MAX_SUPER * MAX_NWAVE;
  unsigned long long* s_goff = (unsigned long long*)(s_scr + MAX_SUPER * MAX_NWAVE + 2);
  LbSummary* s_lb = (LbSummary*)(s_goff + 1);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;

  {
    const uint4* g = p.lut;
    uint4* s = (uint4*)smem;
    for (uint32_t i = tid; i < p.lut_bytes / 16; i += TBK) s[i] = g[i];
    for (uint32_t i = tid; i < (uint32_t)FB_WORDS; i += TBK) s_fb[i] = p.fb[i];
    uint4* st = (uint4*)s_stage0;
    for (uint32_t i = tid; i < 2 * p.stage_bytes / 16; i += TBK) st[i] = make_uint4(0, 0, 0, 0);
  }
  // thread 0: ticket drawn for the iteration after next.  `pend` is only ever
  // written by the atomic (a plain write would have to wait for it); whether a
  // draw is outstanding is kept apart in `pend_ok`.
  uint32_t pend = 0;
  bool pend_ok = false;
  if (tid == 0 && p.sched) {
    // static round robin: workgroup b takes tiles b, b + grid, ...  (all
    // workgroups are co-resident, so the look-back still always progresses)
    *s_ticket = blockIdx.x;
    pend = blockIdx.x + gridDim.x;
  } else if (tid == 0) {
    const uint32_t t0 = atomicAdd(p.ticket, 1u);
    if (t0 == p.nsuper + gridDim.x - 1)
      __hip_atomic_store(p.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *s_ticket = t0;
    if (t0 < p.nsuper) {
      pend = atomicAdd(p.ticket, 1u);
      pend_ok = true;
    }
  }
  __syncthreads();

  const uint32_t kshift = 32u - p.kbits;
  STAMP_DECL

  uint32_t cur = *s_ticket;
  uint4 w[U];
  uint32_t w4[U];
  uint32_t gw[U];
  int start[U];
  bool act[U];
  load_tile<U, TBK>(p, cur, tid, w, w4, gw, act);
  uint32_t bad = 0;  // invalid bit pattern met (no-fallback build)
  bool have_prev = false;
  uint32_t prev = 0, prev_total = 0;
  uint32_t par = 0;                  // staging buffer of the current tile
  uint32_t used0 = 0, used1 = 0;     // bytes last staged into buffer 0 / 1

  for (uint32_t iter = 0;; ++iter) {
    STAMP(9);
    const bool have_cur = cur < p.nsuper;
    if (iter > p.nsuper + 1) {  // cannot happen; a guard so a logic error never hangs the GPU
      if (tid == 0) atomicOr(p.status, (unsigned)GH_ST_TIMEOUT);
      break;
    }
    if (!have_cur && !have_prev) break;
#ifdef GH_STAMPS
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): time spent waiting for tile loads/stores
    STAMP(7);
#endif

    // ---- decode / count tile k ----------------------------------------------------
    uint32_t cnt[U];
    uint32_t ow[SINGLE ? U : 1][SINGLE ? OW : 1];
    Win v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) cnt[u] = 0;
    if (have_cur) {
      tile_starts<U, TBK>(p, cur, tid, gw, start);
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = make_win(w[u], w4[u], start[u]);
      if (ABLATE(8)) {  // diagnostic: skip the decode, keep the output volume
#pragma unroll
        for (int u = 0; u < U; ++u) {
          cnt[u] = act[u] ? 16u : 0u;
          if constexpr (SINGLE) {
#pragma unroll
            for (int k = 0; k < OW; ++k) ow[u][k] = k < 4 ? v[u].d0 : 0u;
          }
        }
      } else if constexpr (G > 0) {
        decode1g<U, G>(v, start, act, ow, cnt, smem, kshift - 3u);
      } else if constexpr (SINGLE) {
        decode1_segments<FB, U>(v, start, act, ow, cnt, s_lut32, s_fb, kshift, p, bad);
      } else {
        count_segments<FB, U>(v, start, act, cnt, s_lut32, s_fb, kshift, p, bad);
      }
    }
    STAMP(0);
    uint32_t bpos[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t incl = wave_incl_scan(cnt[u], lane);
      if (lane == 63) s_scr[u * NWAVE + wid] = incl;
      bpos[u] = incl - cnt[u];
    }
    __syncthreads();  // B0: wave sums
    STAMP(1);
    uint32_t cur_total = 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t before = cur_total;
#pragma unroll
      for (int q = 0; q < NWAVE; ++q) {
        const uint32_t x = s_scr[u * NWAVE + q];
        bpos[u] += (q < wid) ? x : 0u;
        cur_total += x;
      }
      bpos[u] += before + 16u;  // 16-byte zero pad in front of the staged tile
    }
    if (tid == 0 && p.sched) {
      if (have_cur) publish_aggregate(p, cur, cur_total);
      *s_ticket = pend < p.nsuper ? pend : 0xFFFFFFFFu;
      pend += gridDim.x;
    } else if (tid == 0) {
      if (have_cur) publish_aggregate(p, cur, cur_total);
      // tickets are drawn one iteration ahead so the atomic's round trip is hidden;
      // the drawer of the last out-of-range ticket resets the counter for the next
      // launch (every workgroup draws exactly one out-of-range ticket)
      const uint32_t t = pend_ok ? pend : 0xFFFFFFFFu;
      if (t == p.nsuper + gridDim.x - 1)
        __hip_atomic_store(p.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *s_ticket = t;
      pend_ok = t < p.nsuper;
      if (pend_ok) pend = atomicAdd(p.ticket, 1u);
    }
    // clear this iteration's staging buffer (it held tile k-2, copied out at k-1)
    {
      uint4* st = (uint4*)(s_stage0 + par * p.stage_bytes);
      const uint32_t nclr = ((par ? used1 : used0) + 16u + 15u) >> 4;
      for (uint32_t i = tid; i < nclr; i += TBK) st[i] = make_uint4(0, 0, 0, 0);
    }
    __syncthreads();  // B1: ticket, cleared buffer
    STAMP(2);
    const uint32_t next = *s_ticket;
    // the words of tile k are still needed by the emit pass (two-pass path)
    // wave 0: issue the first look-back round of tile k-1 now; its fabric round
    // trip overlaps the staging of tile k below
    // look-back of tile k-1, first round issued by all four waves now: its fabric
    // round trip overlaps the staging of tile k
    const bool resolve = have_prev && !ABLATE(1);
    unsigned long long lbg[4];
    lookback_issue(p, prev, wid, lane, lbg);
    // then the next tile's loads (after the look-back loads, so waiting for the
    // look-back below does not wait for them)
    uint4 wn[U];
    uint32_t w4n[U];
    uint32_t gwn[U];
    bool actn[U];
    load_tile<U, TBK>(p, next, tid, wn, w4n, gwn, actn);
    __asm__ volatile("" ::: "memory");
    if (have_cur && !ABLATE(4)) {
      uint32_t* stg = (uint32_t*)(s_stage0 + par * p.stage_bytes);
      if constexpr (G > 0) {
#pragma unroll
        for (int u = 0; u < U; ++u) stage_bytes_z(stg, ow[u], bpos[u]);
      } else if constexpr (SINGLE) {
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (cnt[u]) stage_bytes(stg, ow[u], cnt[u], bpos[u]);
      } else {
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = make_win(w[u], w4[u], start[u]);
        emit_segments<FB, U>(v, start, act, bpos, s_lut, s_fb, kshift, p, stg);
      }
    }
    STAMP(6);
    if (resolve) lookback_summarise(p, prev, wid, lane, lbg, &s_lb[wid]);
    STAMP(3);
    __syncthreads();  // B2: tile k staged, look-back summaries of tile k-1
    STAMP(4);
    unsigned long long goff = 0;
    if (resolve) {
      // combine the four wave summaries (uniform across the workgroup)
      bool good = true, done = false;
#pragma unroll
      for (int q = 0; q < NWAVE; ++q) {
        const LbSummary sq = s_lb[q];
        if (!done && good) {
          good = sq.ok != 0;
          goff += sq.sum;
          done = good && sq.fp < 256;
        }
      }
      if (!done) {  // rare: predecessors not published yet, or prefix farther back
        if (wid == 0) {
          const unsigned long long ex = resolve_slow(p, (long long)prev - 1, 0ull, lane);
          if (lane == 0) *s_goff = ex;
        }
        __syncthreads();
        goff = *s_goff;
      }
      if (tid == 0) {
        __hip_atomic_store(&p.granules[prev], granule(p.epoch, 2, goff + prev_total),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (prev == p.nsuper - 1) *p.total = goff + prev_total;
      }
    } else if (have_prev && tid == 0 && prev == p.nsuper - 1) {
      *p.total = prev_total;  // ablation build only
    }
    if (have_prev && !ABLATE(2))
      copy_out_shifted<TBK>(p, (const uint32_t*)(s_stage0 + (par ^ 1u) * p.stage_bytes), goff,
                       prev_total, tid);
    STAMP(5);
    have_prev = have_cur;
    prev = cur;
    prev_total = cur_total;
    if (par) used1 = have_cur ? cur_total : 0u; else used0 = have_cur ? cur_total : 0u;
    par ^= 1u;
    cur = next;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      w[u] = wn[u];
      w4[u] = w4n[u];
      gw[u] = gwn[u];
      act[u] = actn[u];
    }
  }
  if (!FB && __any(bad != 0) && lane == 0) atomicOr(p.status, (unsigned)GH_ST_BADCODE);
  STAMP_FLUSH;
}

// ============================================================================
// Split mode: three kernels, no inter-workgroup waiting.
//   gh_count_kernel  decodes each tile's segments counting codewords (no output),
//                    writes the per-segment counts (1 byte each) and tile totals;
//   gh_scan_kernel   exclusive prefix of the tile totals (one workgroup);
//   gh_write_kernel  decodes each tile again, stages its bytes in LDS already at
//                    the output's 16-byte alignment (its offset is known), and
//                    copies them out with aligned 16-byte stores.
// The compressed tile is read twice (C extra bytes of traffic), in exchange the
// write kernel needs no look-back, no persistent loop and no funnel-shifted
// copy-out, and every workgroup is independent (occupancy hides latency).
// Reference counterpart: the fused count / scan / decode of gpu_dec_l1_l2
// (decoder.cu:529-728).
// ============================================================================
template <int TBK>
__device__ __forceinline__ void copy_lut_to_lds(const DecodeParams& p, uint8_t* smem, int tid) {
  const uint4* g = p.lut;
  uint4* s4 = (uint4*)smem;
  for (uint32_t i = tid; i < p.lut_bytes / 16; i += TBK) s4[i] = g[i];
  uint32_t* s_fb = (uint32_t*)(smem + p.lut_bytes);
  for (uint32_t i = tid; i < (uint32_t)FB_WORDS; i += TBK) s_fb[i] = p.fb[i];
}

template <bool SINGLE, bool FB, int U, int G, int TBK>
__device__ __forceinline__ void tile_decode(const DecodeParams& p, uint8_t* smem, Win (&v)[U],
                                            const int (&start)[U], const bool (&act)[U],
                                            uint32_t (&ow)[SINGLE ? U : 1][SINGLE ? OW : 1],
                                            uint32_t (&cnt)[U], uint32_t& bad) {
  const uint32_t kshift = 32u - p.kbits;
  const uint32_t* s_lut32 = (const uint32_t*)smem;
  const uint32_t* s_fb = (const uint32_t*)(smem + p.lut_bytes);
  if (ABLATE(8)) {  // diagnostic: no decode, plausible output volume
#pragma unroll
    for (int u = 0; u < U; ++u) {
      cnt[u] = act[u] ? 16u : 0u;
      if constexpr (SINGLE) {
#pragma unroll
        for (int k = 0; k < OW; ++k) ow[u][k] = k < 4 ? v[u].d0 : 0u;
      }
    }
    return;
  }
  if constexpr (G > 0) {
    decode1g<U, G>(v, start, act, ow, cnt, smem, kshift - 3u);
  } else if constexpr (SINGLE) {
    decode1_segments<FB, U>(v, start, act, ow, cnt, s_lut32, s_fb, kshift, p, bad);
  } else {
    count_segments<FB, U>(v, start, act, cnt, s_lut32, s_fb, kshift, p, bad);
  }
}

// Tiles [t0, t1) of workgroup b: contiguous ranges of (almost) equal length.
__device__ __forceinline__ void wg_range(uint32_t ntiles, uint32_t& t0, uint32_t& t1) {
  t0 = (uint32_t)(((unsigned long long)blockIdx.x * ntiles) / gridDim.x);
  t1 = (uint32_t)(((unsigned long long)(blockIdx.x + 1) * ntiles) / gridDim.x);
}

template <bool SINGLE, bool FB, int U, int G, int TBK>
__global__ __launch_bounds__(TBK) void gh_count_kernel(const DecodeParams p) {
  constexpr int NWAVE = TBK / 64;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  __shared__ uint32_t s_wsum[2][NWAVE];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  uint32_t t0, t1;
  wg_range(p.nsuper, t0, t1);
  uint4 w[U];
  uint32_t w4[U], gw[U];
  bool act[U];
  if (t0 < t1) load_tile<U, TBK>(p, t0, tid, w, w4, gw, act);
  copy_lut_to_lds<TBK>(p, smem, tid);
  __syncthreads();
  uint32_t bad = 0;
  unsigned long long wg_total = 0;
  uint32_t par = 0;
  for (uint32_t t = t0; t < t1; ++t, par ^= 1u) {
    int start[U];
    tile_starts<U, TBK>(p, t, tid, gw, start);
    Win v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = make_win(w[u], w4[u], start[u]);
    bool a[U];
#pragma unroll
    for (int u = 0; u < U; ++u) a[u] = act[u];
    if (t + 1 < t1) load_tile<U, TBK>(p, t + 1, tid, w, w4, gw, act);  // prefetch
    uint32_t cnt[U];
    uint32_t ow[SINGLE ? U : 1][SINGLE ? OW : 1];
    tile_decode<SINGLE, FB, U, G, TBK>(p, smem, v, start, a, ow, cnt, bad);
    const unsigned long long seg0 = (unsigned long long)t * (U * TBK) + tid;
    uint32_t sum = 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (a[u]) p.seg_cnt[seg0 + (unsigned long long)u * TBK] = (uint8_t)cnt[u];
      sum += a[u] ? cnt[u] : 0u;
    }
    sum = wave_incl_scan(sum, lane);
    if (lane == 63) s_wsum[par][wid] = sum;
    __syncthreads();
    if (tid == 0) {
      uint32_t tt = 0;
#pragma unroll
      for (int q = 0; q < NWAVE; ++q) tt += s_wsum[par][q];
      p.tile_cnt[t] = tt;
      wg_total += tt;
    }
  }
  if (tid == 0) p.wg_tot[blockIdx.x] = wg_total;
  if (!FB && __any(bad != 0) && lane == 0) atomicOr(p.status, (unsigned)GH_ST_BADCODE);
}

template <bool SINGLE, bool FB, int U, int G, int TBK>
__global__ __launch_bounds__(TBK) void gh_write_kernel(const DecodeParams p) {
  constexpr int NWAVE = TBK / 64;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  __shared__ uint32_t s_wsum[2][U * NWAVE];
  __shared__ unsigned long long s_base[NWAVE];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  uint8_t* s_stage = smem + p.lut_bytes + FB_BYTES;
  uint32_t t0, t1;
  wg_range(p.nsuper, t0, t1);
  uint4 w[U];
  uint32_t w4[U], gw[U], c8[U];
  bool act[U];
  auto load_counts = [&](uint32_t t) {
    const unsigned long long seg0 = (unsigned long long)t * (U * TBK) + tid;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const unsigned long long seg = min(seg0 + (unsigned long long)u * TBK, p.nseg - 1);
      c8[u] = p.seg_cnt[seg];
    }
  };
  if (t0 < t1) {
    load_tile<U, TBK>(p, t0, tid, w, w4, gw, act);
    load_counts(t0);
  }
  // output offset of this workgroup's range: the totals of the ranges before it
  {
    unsigned long long b = 0;
    const uint32_t nb = blockIdx.x * p.count_per;
    for (uint32_t i = tid; i < nb; i += TBK) b += p.wg_tot[i];
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) b += __shfl_xor(b, d, 64);
    if (lane == 0) s_base[wid] = b;
  }
  copy_lut_to_lds<TBK>(p, smem, tid);
  {
    uint4* st = (uint4*)s_stage;
    for (uint32_t i = tid; i < p.stage_bytes / 16; i += TBK) st[i] = make_uint4(0, 0, 0, 0);
  }
  __syncthreads();
  unsigned long long goff = 0;
#pragma unroll
  for (int q = 0; q < NWAVE; ++q) goff += s_base[q];
  uint32_t par = 0;
  uint32_t* stg = (uint32_t*)s_stage;
  const uint4* st4 = (const uint4*)s_stage;
  for (uint32_t t = t0; t < t1; ++t, par ^= 1u) {
    int start[U];
    tile_starts<U, TBK>(p, t, tid, gw, start);
    Win v[U];
    bool a[U];
    uint32_t cc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      v[u] = make_win(w[u], w4[u], start[u]);
      a[u] = act[u];
      cc[u] = a[u] ? c8[u] : 0u;
    }
    const uint32_t ttot = p.tile_cnt[t];
    if (t + 1 < t1) {  // prefetch the next tile
      load_tile<U, TBK>(p, t + 1, tid, w, w4, gw, act);
      load_counts(t + 1);
    }
    const uint32_t lb = (uint32_t)(goff & 15);
    uint32_t bpos[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t incl = wave_incl_scan(cc[u], lane);
      if (lane == 63) s_wsum[par][u * NWAVE + wid] = incl;
      bpos[u] = incl - cc[u];
    }
    __syncthreads();  // wave sums; the previous tile's copy-out and clear are done
    {
      uint32_t before = 0;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        uint32_t add = before;
#pragma unroll
        for (int q = 0; q < NWAVE; ++q) {
          const uint32_t x = s_wsum[par][u * NWAVE + q];
          add += (q < wid) ? x : 0u;
          before += x;
        }
        bpos[u] += add + 16u + lb;
      }
    }
    uint32_t bad = 0;
    if constexpr (SINGLE) {
      uint32_t cnt[U];
      uint32_t ow[U][OW];
      tile_decode<SINGLE, FB, U, G, TBK>(p, smem, v, start, a, ow, cnt, bad);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if constexpr (G > 0) {
          if (a[u]) stage_bytes_z(stg, ow[u], bpos[u]);
        } else {
          if (cnt[u]) stage_bytes(stg, ow[u], cnt[u], bpos[u]);
        }
      }
    } else {
      const uint2* s_lut = (const uint2*)smem;
      const uint32_t* s_fb = (const uint32_t*)(smem + p.lut_bytes);
      emit_segments<FB, U>(v, start, a, bpos, s_lut, s_fb, 32u - p.kbits, p, stg);
    }
    __syncthreads();  // tile staged
    // staging byte x <-> output byte a0 - 16 + x, a0 = goff - lb (16-byte aligned);
    // each thread clears the chunks it copied (the next tile stages after the
    // next barrier)
    const unsigned long long a0 = goff - lb;
    const unsigned long long end = min(goff + ttot, p.out_cap);
    const uint32_t nz = (16u + lb + ttot + 15u) >> 4;
    uint4* stw = (uint4*)s_stage;
    for (uint32_t c = tid; c < nz + 1; c += TBK) {
      const uint4 d = st4[c];
      stw[c] = make_uint4(0, 0, 0, 0);
      if (c == 0 || c >= nz) continue;
      const unsigned long long gs = a0 - 16 + 16ull * c;
      if (gs >= goff && gs + 16 <= end) {
        *(uint4*)(p.out + gs) = d;
      } else {
        const uint8_t* bb = (const uint8_t*)&d;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          const unsigned long long ga = gs + k;
          if (ga >= goff && ga < end) p.out[ga] = bb[k];
        }
      }
    }
    goff += ttot;
  }
  if (blockIdx.x == gridDim.x - 1 && tid == 0) *p.total = goff;
}

// ============================================================================
// Tile mode: ONE persistent kernel, 512-thread workgroups, one segment per lane,
// ONE workgroup barrier per tile.  Workgroup b takes tiles b, b + grid, ...
// (static round robin; grid <= 512 and every workgroup resident).  Iteration k:
//
//   issue: look-back loads for tile k-1 (512 granules, one per lane: tiles
//          k-1-1 .. k-1-512), then the loads of tile k+1
//   decode tile k (registers) -> wave scan -> summarise the look-back per wave
//   BARRIER
//   publish aggregate(k); combine the 8 look-back summaries -> prefix of tile k-1,
//   publish inclusive(k-1); copy tile k-1 out of staging buffer (k-1)&1;
//   stage tile k into buffer k&1 at tile-local offsets
//
// Why the look-back spans 512 tiles and is one tile late: a granule stored on one
// XCD becomes visible to another XCD's loads only after a fabric round trip, so a
// look-back issued right after the predecessor publishes nearly always misses
// (measured: 97% slow path).  One iteration later every predecessor of the round
// has published its aggregate, and tile k-1-512 is this workgroup's own tile of
// the previous round, whose inclusive prefix it published itself: the look-back
// completes in one round of loads whose latency hides under the decode.
//
// Staging needs no clearing: a segment's bytes go to LDS as byte/short writes for
// the partial head/tail dwords and dword writes in between, so no two lanes write
// the same byte.  Buffer k&1 is staged after barrier k and copied out after barrier
// k+1; its next staging is after barrier k+2.
//
// LUT: R = 2^lgr copies interleaved at dword granularity (entry i, copy c at
// dword i*R + c; lane l reads copy l mod R), so up to 32 lanes of a ds_read_b32
// group hit distinct banks.  The segment window is pre-shifted by
// S = 30 - K - lgr bits (the "e-window"): the lookup address of the codeword at
// window bit p is alignbit(e0, e1, 32 - p) & (mask << (2 + lgr)) | lane_offset,
// two VALU ops.  Reference counterpart: gpu_dec_l1_l2 (decoder.cu:454-730).
// ============================================================================
constexpr int STAGE_PAD = 16;  // staging byte STAGE_PAD + i = tile byte i
#ifndef GH_TILE_WPE
#define GH_TILE_WPE 4  // most waves per SIMD the tile kernel is compiled for (VGPR budget 512 / WPE)
#endif
#ifndef GH_TILE_FIXST
#define GH_TILE_FIXST 1        // grouped path: copy-out with a fixed store count per thread, prefetch before it
#endif
#ifndef GH_TILE_NS
#define GH_TILE_NS 2           // 16-byte stores per thread per copy-out (the rest of a large tile loops)
#endif
#ifndef GH_PREFETCH_LATE
#define GH_PREFETCH_LATE 1     // grouped path: issue the next tile's loads after the copy-out
#endif
#ifndef GH_TILE_LAG3
#define GH_TILE_LAG3 0         // grouped path: copy out at lag 3 (measured no faster than lag 2)
#endif
#ifndef GH_TILE_TOPCOPY
#define GH_TILE_TOPCOPY 0      // with LAG3: copy tile k-3 out at the top of iteration k, before the decode
#endif
#ifndef GH_TILE_PRIO
#define GH_TILE_PRIO 1         // alternate s_setprio between the two workgroup slots of a CU (cfg4 0.747 -> 0.729 ms)
#endif
#ifndef GH_LB_MIDG
#define GH_LB_MIDG 2           // decode group after which the round leader loads aggregates
#endif
// tile kernel paths
constexpr int TP_GROUPED = 0;  // single-symbol u32 LUT on e-windows, grouped window shifts
constexpr int TP_MULTI = 1;    // multi-symbol u64 LUT, count pass + emit pass
constexpr int TP_MULTI_FB = 2; // the same with the canonical fallback for codes longer than K

struct TileParams {
  const uint32_t* payload;       // local segment j owns words [4j, 4j+4); +1 look-ahead, zero padded
  const uint32_t* gaps;          // gap words; nibble (gap_nib0 + j - 1) = start of local segment j>=1
  const uint32_t* lut;           // grouped: 2^K u32 {len | sym << 24}; multi: 2^K u64 {syms, meta}
  const uint32_t* fb;            // multi FB: canonical fallback tables (FB_WORDS)
  uint8_t* out;
  unsigned long long* granules;  // one per tile: its symbol count (flag 1)
  unsigned long long* plocal;    // one per tile: exclusive prefix within its round (flag 2)
  unsigned long long* rprefix;   // one per round: its starting offset (flag 2); [0] unused
  unsigned int* status;
  unsigned long long* total;
  unsigned long long* stats;     // poll counters (diagnostics)
  unsigned long long out_cap;
  unsigned long long nseg;
  unsigned int gap_nib0, first_start, ntiles, kbits, lgr, epoch;
  unsigned int fb_lo, fb_hi;     // multi FB: fallback length range
  unsigned int lut_bytes;        // LUT bytes in LDS (grouped: replicated 4 << (K + lgr))
  unsigned int stage_bytes;      // one staging buffer
  unsigned long long* stamps;    // diagnostic build only (GH_STAMPS)
  unsigned int ablate;           // diagnostic build only: 2 no copy-out, 4 no staging, 8 no decode
  uint4* junk;                   // GH_TILE_FIXST: 16 bytes per thread of the grid for padding stores
};

// e-window of a segment starting at bit `start` (0..15): e-stream bit 0 is segment
// bit start - S (bits before the segment read as 0); requires 16 <= S <= 31.
__device__ __forceinline__ void make_ewin(uint4 w, uint32_t w4, int start, uint32_t S,
                                          uint32_t (&e)[5]) {
  const uint32_t r = S - (uint32_t)start;  // 1..31
  e[0] = __builtin_amdgcn_alignbit(0u, w.x, r);
  e[1] = __builtin_amdgcn_alignbit(w.x, w.y, r);
  e[2] = __builtin_amdgcn_alignbit(w.y, w.z, r);
  e[3] = __builtin_amdgcn_alignbit(w.z, w.w, r);
  e[4] = __builtin_amdgcn_alignbit(w.w, w4, r);
}

// LDS u32 read at an absolute LDS byte address, waited for at once (the lookups of a
// segment form one dependent chain).  Inline asm: the compiler would otherwise add
// the dynamic-LDS base (0 here: the tile kernel declares no static LDS, checked at
// kernel start) with one extra VALU op per lookup.
__device__ __forceinline__ uint32_t lds_u32(uint32_t byte_addr) {
  uint32_t v;
  asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(byte_addr) : "memory");
  return v;
}

// LDS u32 read without a wait, and a wait that ties the results (so the compiler
// cannot use them before it).  Used for the U independent lookups of a step.
__device__ __forceinline__ uint32_t lds_u32_nowait(uint32_t byte_addr) {
  uint32_t v;
  asm volatile("ds_read_b32 %0, %1" : "=v"(v) : "v"(byte_addr) : "memory");
  return v;
}
template <int U>
__device__ __forceinline__ void lds_wait_all(uint32_t (&v)[U]) {
  if constexpr (U == 1) {
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v[0]) :: "memory");
  } else if constexpr (U == 2) {
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v[0]), "+v"(v[1]) :: "memory");
  } else {
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]) :: "memory");
  }
}

// Grouped single-symbol decode of U segments per lane on e-windows, the U chains in
// lock-step (their LDS reads are independent, so their latencies overlap).  Each
// group decodes G codewords per chain from e0:e1 and then shifts the windows;
// codeword j of a chain is kept iff it starts before the segment end (q > T, see
// decode1g); dead codewords insert 0.  `mid()` is called once, after group MIDG
// (or at the end if the loop stops earlier): the tile kernel issues its look-back
// loads there, late enough for its predecessors to have published.
template <int G, int U, int MIDG, class Mid, bool EMIT = true>
__device__ __forceinline__ void decode_tile_grouped(uint32_t (&e)[U][5], const int (&start)[U],
                                                    const bool (&act)[U], uint32_t (&ow)[U][OW],
                                                    uint32_t (&cnt)[U], uint32_t amask,
                                                    uint32_t laneoff, Mid&& mid) {
  constexpr int S = 4 * OW;
  constexpr int NG = (S + G - 1) / G;
  uint32_t q[U];
  int T[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    q[u] = 32;
    T[u] = act[u] ? start[u] - 96 : 0x3FFFFFFF;  // inactive: never live, no overflow
    cnt[u] = 0;
#pragma unroll
    for (int k = 0; k < OW; ++k) ow[u][k] = 0;
  }
  bool mid_done = false;
  // q counts down from 32 by whole LUT entries {len | sym << 24}: its low 24 bits stay
  // exact, v_alignbit reads only the low 5, and the liveness test (q > T, the
  // codeword starts before the segment end) reads the low 16 sign-extended (SDWA).
  // Codewords past the end still go into ow: the staging never reads them.
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
          ent[u] = lds_u32_nowait((x & amask) | laneoff);
        }
        lds_wait_all(ent);
#pragma unroll
        for (int u = 0; u < U; ++u) {
          asm("v_cmp_gt_i32_sdwa vcc, sext(%1), %2 src0_sel:WORD_0 src1_sel:DWORD\n\t"
              "v_addc_co_u32 %0, vcc, 0, %0, vcc"
              : "+v"(cnt[u]) : "v"(q[u]), "v"(T[u]) : "vcc");
          if constexpr (EMIT) ow[u][pos >> 2] = __builtin_amdgcn_perm(ent[u], ow[u][pos >> 2], perm_sel(pos & 3));
          q[u] -= ent[u];
        }
      }
    }
    bool more = false;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      e[u][0] = __builtin_amdgcn_alignbit(e[u][0], e[u][1], q[u]);
      e[u][1] = __builtin_amdgcn_alignbit(e[u][1], e[u][2], q[u]);
      e[u][2] = __builtin_amdgcn_alignbit(e[u][2], e[u][3], q[u]);
      e[u][3] = __builtin_amdgcn_alignbit(e[u][3], e[u][4], q[u]);
      e[u][4] = __builtin_amdgcn_alignbit(e[u][4], 0u, q[u]);
      T[u] += 32 - (int)(int16_t)q[u];
      q[u] = 32;
      more |= 32 > T[u];
    }
    if (gi == MIDG) {
      mid();
      mid_done = true;
    }
    if (gi + 1 < NG && !__any(more)) break;
  }
  if (!mid_done) mid();
}

// LDS u64 read (multi-symbol LUT entry) at an absolute LDS byte address.
__device__ __forceinline__ uint2 lds_u64(uint32_t byte_addr) {
  uint2 v;
  asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(byte_addr) : "memory");
  return v;
}
// LDS stores at absolute byte addresses.  ds_write_b32 may be unaligned: gfx950
// LDS runs in unaligned mode and an unaligned dword store costs the same as an
// aligned one (scripts/ubench/lds_unaligned.hip).
__device__ __forceinline__ void lds_st32(uint32_t byte_addr, uint32_t v) {
  asm volatile("ds_write_b32 %0, %1" :: "v"(byte_addr), "v"(v) : "memory");
}
__device__ __forceinline__ void lds_st8(uint32_t byte_addr, uint32_t v) {
  asm volatile("ds_write_b8 %0, %1" :: "v"(byte_addr), "v"(v) : "memory");
}

// Per-lane select by a lane mask (mask bit set: a), opaque to the optimiser.
__device__ __forceinline__ uint32_t vsel(unsigned long long mask, uint32_t a, uint32_t b) {
  uint32_t r;
  asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(b), "v"(a), "s"(mask));
  return r;
}

// Stage a segment's n bytes (ow, byte 0 first) at absolute LDS byte address `pos`:
// the whole dwords as (mostly unaligned) dword stores, the last n & 3 bytes as byte
// stores, so no byte outside [pos, pos + n) is touched and segments need no
// coordination.
__device__ __forceinline__ void stage_unaligned(const uint32_t (&ow)[OW], uint32_t n, uint32_t pos) {
  const uint32_t nf = n >> 2;
#pragma unroll
  for (int m = 0; m < OW; ++m)
    if ((uint32_t)m < nf) lds_st32(pos + 4u * m, ow[m]);
  const uint32_t t = n & 3u;
  if (t) {
    // ow[nf], selected by a 3-level tree of opaque selects (a plain ?: tree is
    // turned back into an indexed load, which puts ow[] in scratch memory)
    const unsigned long long s1 = __ballot((nf & 1u) != 0), s2 = __ballot((nf & 2u) != 0),
                             s4 = __ballot((nf & 4u) != 0);
    const uint32_t a0 = vsel(s1, ow[1], ow[0]), a1 = vsel(s1, ow[3], ow[2]);
    const uint32_t a2 = vsel(s1, ow[5], ow[4]), a3 = vsel(s1, ow[7], ow[6]);
    const uint32_t b0 = vsel(s2, a1, a0), b1 = vsel(s2, a3, a2);
    const uint32_t x = vsel(s4, b1, b0);
    const uint32_t q = pos + 4u * nf;
    lds_st8(q, x);
    if (t > 1) lds_st8(q + 1, x >> 8);
    if (t > 2) lds_st8(q + 2, x >> 16);
  }
}

// Aligned staging of a segment's n bytes (ow, byte 0 first) at LDS byte address o.
// Phase 1 writes the aligned dwords holding the segment's bytes, except the first
// one when o is unaligned; its last dword carries whatever ow holds past byte n.
// Phase 2, after a workgroup barrier, writes the segment's head bytes (the 1-3 bytes
// of that skipped first dword) exactly, over the previous segment's phase-1 tail.
// Every dword store is aligned: unaligned ds_write_b32 measured about 3x the LDS
// time of aligned ones with per-lane offsets like these.
// Returns the number of head bytes (0 when o is aligned).
__device__ __forceinline__ uint32_t stage_aligned_p1(const uint32_t (&ow)[OW], uint32_t n, uint32_t o) {
  const uint32_t ap = ((o - 1u) & 3u) + 1u;  // 1..4: bytes from the dword base to o
  const uint32_t base = o - ap;              // dword m at base + 4m holds segment bytes [4m - ap, +4)
  const uint32_t s = 4u - ap;                // alignbyte amount
  const uint32_t last = (n + ap - 1u) >> 2;  // last dword touched (>= 2 for n >= 7)
#pragma unroll
  for (int m = 1; m <= OW; ++m) {
    const uint32_t hi = m < OW ? ow[m] : 0u;
    const uint32_t r = __builtin_amdgcn_alignbyte(hi, ow[m - 1], s);
    if ((uint32_t)m <= last) lds_st32(base + 4u * m, r);
  }
  return 4u - ap;
}
// Phase 2: the nb (1..3) head bytes h at o (o + (nb & 1) is even).
__device__ __forceinline__ void stage_head(uint32_t o, uint32_t h, uint32_t nb) {
  if (nb & 1u) asm volatile("ds_write_b8 %0, %1" :: "v"(o), "v"(h) : "memory");
  if (nb & 2u) asm volatile("ds_write_b16 %0, %1" :: "v"(o + (nb & 1u)), "v"(h >> (8u * (nb & 1u))) : "memory");
}

// ---- multi-symbol path ------------------------------------------------------------
// Count pass: codewords of the segment (window v at bit `start`) that start before
// bit 128, with the reference's segment rule (decoder.cu:529-569): the last lookup
// may hold codewords past the segment end; kept_in_last() drops them.
template <bool FB>
__device__ __forceinline__ uint32_t count_chain(Win v, int start, bool act, uint32_t kshift,
                                                const TileParams& p, const uint32_t* s_fb,
                                                uint32_t& bad) {
  int P = act ? start : 128, Plast = P;
  uint32_t mlast = make_meta(1, 0, 15, 15, 15), cnt = 0;
  do {
    uint32_t meta = lds_u32(((v.d0 >> kshift) << 3) + 4u);
    if constexpr (FB) {
      if (meta_n(meta) == 0 && P < 128) {
        uint32_t sy;
        meta = fallback_meta(s_fb, v.d0, p, &sy);
      }
    }
    const bool live = P < 128;
    if constexpr (!FB) bad |= (live && meta_n(meta) == 0) ? 1u : 0u;
    cnt += live ? meta_n(meta) : 0u;
    Plast = live ? P : Plast;
    mlast = live ? meta : mlast;
    P += FB ? (int)meta_b(meta) : max((int)meta_b(meta), 1);
    consume(v, meta);
  } while (__any(P < 128));
  if (act) cnt -= meta_n(mlast) - kept_in_last(mlast, 128 - Plast);
  return cnt;
}

// Emit pass: decode again and store the cnt bytes at absolute LDS byte address pos:
// a lookup's (up to 4) symbols go out as one unaligned dword while they fit below
// pos + cnt; the last < 4 bytes as byte stores.
template <bool FB>
__device__ __forceinline__ void emit_chain(Win v, int start, bool act, uint32_t cnt, uint32_t pos,
                                           uint32_t kshift, const TileParams& p,
                                           const uint32_t* s_fb) {
  int P = act ? start : 128;
  const uint32_t end = pos + cnt;
  uint32_t cur = pos;
  bool go = P < 128 && cur < end;
  while (__any(go)) {
    uint2 e = lds_u64((v.d0 >> kshift) << 3);
    if constexpr (FB) {
      if (meta_n(e.y) == 0 && go) e.y = fallback_meta(s_fb, v.d0, p, &e.x);
    }
    const uint32_t n = meta_n(e.y);
    if (go && cur + 4u <= end) {
      lds_st32(cur, e.x);
    } else if (go) {  // the last bytes
      const uint32_t t = min(end - cur, n);
      lds_st8(cur, e.x);
      if (t > 1) lds_st8(cur + 1, e.x >> 8);
      if (t > 2) lds_st8(cur + 2, e.x >> 16);
      if (t > 3) lds_st8(cur + 3, e.x >> 24);
    }
    cur += go ? n : 0u;
    P += FB ? (int)meta_b(e.y) : max((int)meta_b(e.y), 1);
    consume(v, e.y);
    go = go && P < 128 && cur < end;
  }
}

// Copy a tile staged at staging byte STAGE_PAD + i = tile byte i to out[goff, goff+n)
// (n already clamped at out_cap).  Output chunk c (16 bytes, aligned to the global
// address) is staging bytes [16c + s, 16c + s + 16), s = 16 - (goff & 15): one
// unaligned ds_read_b128 (gfx950 LDS runs in unaligned mode).  Interior chunks are
// one 16-byte store each; the (at most two) partial edge chunks are finished byte by
// byte by two lanes.  stg: absolute LDS byte address of the staging buffer.
__device__ __forceinline__ uint4 lds_u128(uint32_t byte_addr) {
  uint4 v;
  asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(byte_addr) : "memory");
  return v;
}
__device__ __forceinline__ void store_edge(uint8_t* oc, uint4 v, int k0, int k1) {
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const uint32_t wv = k < 4 ? v.x : k < 8 ? v.y : k < 12 ? v.z : v.w;
    if (k >= k0 && k < k1) oc[k] = (uint8_t)(wv >> (8 * (k & 3)));
  }
}
template <int TBK>
__device__ __forceinline__ void copy_out_tile(uint8_t* out, uint32_t stg, unsigned long long goff, uint32_t n,
                                              int tid, uint32_t abl = 0) {
  if (n == 0) return;
  const uint32_t lb = (uint32_t)(goff & 15);
  uint8_t* o = out + (goff - lb);          // 16-byte aligned
  const uint32_t src = stg + 16u - lb;     // staging address of output chunk 0
  const uint32_t cf = lb ? 1u : 0u;        // interior chunks [cf, ce)
  const uint32_t ce = (lb + n) >> 4;
  for (uint32_t c = cf + (uint32_t)tid; c < ce; c += TBK) {
    const uint4 v = (abl & 64) ? make_uint4(c, c + 1, c + 2, c + 3) : lds_u128(src + 16u * c);
    if (!(abl & 16) || v.x == 0x9E3779B9u) *(uint4*)(o + 16ull * c) = v;
  }
  const uint32_t tail = (lb + n) & 15u;
  if (tid == 0 && lb) {  // first chunk: tile bytes [0, 16 - lb), or all n if the tile ends in it
    store_edge(o, lds_u128(src), (int)lb, (int)min(16u, lb + n));
  } else if (tid == TBK - 1 && tail && (ce > 0 || !lb)) {  // last chunk ce: bytes [0, tail)
    store_edge(o + 16ull * ce, lds_u128(src + 16u * ce), 0, (int)tail);
  }
}

// The same copy with a fixed number of store instructions per thread: NS 16-byte
// stores (interior chunks; spare threads store the last interior chunk again, the
// same bytes) and one byte store (a byte of the two partial edge chunks, or the first
// edge byte again); the thread's junk slot only when there is nothing to duplicate.  On gfx950 loads and stores share one
// in-order counter (vmcnt); with a fixed store count after the next tile's prefetch
// loads, the compiler waits for those loads with vmcnt(NS + 1) instead of vmcnt(0),
// so a wave no longer waits for its previous copy-out's stores to be acknowledged.
// LOOP = false: the caller guarantees n + 32 <= 16 * NS * TBK (no chunk beyond the fixed
// stores), so the store count is the same on every call.
template <int TBK, int NS, bool LOOP = true>
__device__ __forceinline__ void copy_out_tile_fixed(uint8_t* out, uint32_t stg, unsigned long long goff, uint32_t n,
                                                    int tid, uint4* junk) {
  const uint32_t lb = (uint32_t)(goff & 15);
  uint8_t* o = out + (goff - lb);          // 16-byte aligned
  const uint32_t src = stg + 16u - lb;     // staging address of output chunk 0
  const uint32_t cf = lb ? 1u : 0u;        // interior chunks [cf, ce)
  const uint32_t ce = n ? (lb + n) >> 4 : 0u;
  const bool have = ce > cf;  // padding stores duplicate a real chunk / byte (merged in L2); junk when none
#pragma unroll
  for (int i = 0; i < NS; ++i) {
    const uint32_t c = cf + (uint32_t)tid + (uint32_t)(TBK * i);
    const bool real = c < ce;
    const uint32_t cs = real ? c : ce - 1u;  // padding: the last interior chunk again (same bytes)
    const uint4 v = lds_u128(src + 16u * ((real || have) ? cs : cf));
    *((real || have) ? (uint4*)(o + 16ull * cs) : junk) = v;
  }
  if constexpr (LOOP)
    for (uint32_t c = cf + (uint32_t)tid + (uint32_t)(TBK * NS); c < ce; c += TBK)
      *(uint4*)(o + 16ull * c) = lds_u128(src + 16u * c);
  // edge bytes: the head chunk's [lb, min(16, lb + n)) when lb != 0, then the tail
  // chunk's [0, (lb + n) & 15) when it is another chunk; one byte per thread
  const uint32_t nh = (lb && n) ? min(16u, lb + n) - lb : 0u;
  const uint32_t tl = (lb + n) & 15u;
  const uint32_t nt = (n && tl && (ce > 0 || !lb)) ? tl : 0u;
  const uint32_t t = (uint32_t)tid;
  const bool hb = nh + nt > 0;
  uint32_t k = nh ? lb : 16u * ce;         // output byte offset from o (padding: the first edge byte)
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

// ---- prefixes by round leaders ------------------------------------------------
// Tiles are processed in rounds: workgroup b takes tile rG + b in iteration r
// (static round robin over the G resident workgroups).  A tile publishes its
// symbol count (aggregate granule) right after its barrier.  Round r gets a leader,
// workgroup r mod G, which during iteration r+1 loads the round's G aggregates (one
// per lane, issued mid-decode: they were published a whole iteration earlier),
// scans them at its barrier and publishes each tile's within-round exclusive prefix
// (plocal) and the next round's starting offset R[r+1] = R[r] + round total.  The
// owner of a tile reads R[round] + plocal[tile] at the top of iteration r+2 and
// copies the tile out after its decode.  Every hand-off has about an iteration of
// slack, and the granule traffic is three 8-byte loads/stores per tile (decoupled
// look-back with 512 tiles in flight needs a window of ~512 granules per tile to
// keep up: measured as the slow path of most tiles at 64/256).
//
// Granules: {epoch:24, flag:2, value:38} in one 8-byte word (the data is the flag).
// Reference counterpart: the decoupled look-back of gpu_dec_l1_l2 (decoder.cu:601-653).
// LDS of the tile kernel: LUT, two staging buffers, wave sums, leader batch totals.
template <int TB, int U>
inline size_t tile_lds_bytes(size_t lut_bytes, size_t stage_bytes) {
  return lut_bytes + 2 * stage_bytes + 2 * (TB / 64) * 4 * U + 4 * (TB / 64) + 32;
}

// Poll a granule until it carries this launch's epoch with the wanted flag (bounded).
// Bounded by wall time, 4 s of the 100 MHz clock: a persistent grid that shares the GPU
// with another kernel (another stream or process) waits for its not-yet-resident
// workgroups until that kernel's workgroups retire — a delay, not a fault.  After a
// timeout every later poll returns at once (the decode then fails with GH_E_HIP).
// The clock and the status word are read only every 64th poll: a poll's load sits in
// the CU's memory queue behind its streaming traffic (microseconds), and the look-back
// chain pays every extra round trip.
__device__ __forceinline__ unsigned long long poll_granule(const TileParams& p,
                                                           unsigned long long* g, uint32_t flag) {
  unsigned long long t0 = 0;
  for (uint32_t spins = 1;; ++spins) {
    const unsigned long long v = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((uint32_t)(v >> 40) == p.epoch && (uint32_t)((v >> 38) & 3u) == flag) return v;
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

__device__ __forceinline__ bool granule_ok(const TileParams& p, unsigned long long v, uint32_t flag) {
  return (uint32_t)(v >> 40) == p.epoch && (uint32_t)((v >> 38) & 3u) == flag;
}

// TB threads, U segments per lane, PATH (TP_*), GRP codewords per window shift
// (grouped path).
template <int TB, int U, int PATH, int GRP>
__global__ __launch_bounds__(TB) __attribute__((amdgpu_waves_per_eu(4, GH_TILE_WPE)))
void gh_tile_kernel(const TileParams p) {
  constexpr int NWAVE_T = TB / 64;
  constexpr int LDR_NB = TB / 64;  // leader batches: one wave per 64 * LPL tiles of a round
  constexpr int LPL = TB >= 512 ? 1 : 1024 / TB;  // aggregates per leader lane (grid <= LPL * TB)
  constexpr bool MULTI = PATH != TP_GROUPED;
  constexpr bool FB = PATH == TP_MULTI_FB;
  static_assert(!MULTI || U == 1, "multi-symbol path: one segment per lane");
  constexpr unsigned long long VMASK = (1ull << 38) - 1;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint8_t* s_stage = smem + p.lut_bytes;                                   // 2 buffers
  uint32_t* s_wsum = (uint32_t*)(s_stage + 2 * p.stage_bytes);             // [2][U][NWAVE_T]
  uint32_t* s_lead = s_wsum + 2 * U * NWAVE_T;                             // [LDR_NB]
  uint32_t bad = 0;  // multi (no FB): an invalid bit pattern was met

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  uint32_t* s_fb = s_lead + LDR_NB;  // multi FB: fallback tables (FB_WORDS)
  {  // LUT to LDS (grouped: replicated, dword i of LDS = entry i >> lgr)
    const uint32_t nd = p.lut_bytes >> 2;
    uint32_t* sl = (uint32_t*)smem;
    if constexpr (MULTI) {
      for (uint32_t i = tid; i < nd; i += TB) sl[i] = p.lut[i];
      if constexpr (FB)
        for (uint32_t i = tid; i < (uint32_t)FB_WORDS; i += TB) s_fb[i] = p.fb[i];
    } else {
      for (uint32_t i = tid; i < nd; i += TB) sl[i] = p.lut[i >> p.lgr];
    }
  }
  const uint32_t kshift = 32u - p.kbits;
  const uint32_t S = 30u - p.kbits - p.lgr;
  const uint32_t amask = ((1u << p.kbits) - 1u) << (2u + p.lgr);
  const uint32_t laneoff = ((uint32_t)lane & ((1u << p.lgr) - 1u)) << 2;
  if (tid == 0 && (uint32_t)(size_t)(const __attribute__((address_space(3))) uint8_t*)smem != 0u)
    atomicOr(p.status, (unsigned)GH_ST_LAYOUT);
  __syncthreads();

  const uint32_t G = gridDim.x, b = blockIdx.x;  // grid size, workgroup
  const uint32_t nseg = (uint32_t)p.nseg;  // < 2^31 (checked by the host)
  constexpr uint32_t NONE = 0xFFFFFFFFu;
  // Static round robin: tile b + kG in iteration k.  (A dynamic ticket order can
  // deadlock here: a workgroup waiting for its tile's prefix may hold an undecoded
  // tile of the same round, whose leader then waits for it.)
  // The round led by this workgroup in iteration k is r = k - 1 when
  // r mod n_r == b (n_r = tiles in round r), so every round has a leader that
  // decoded one of its tiles.
  const uint32_t last_tile_k = b < p.ntiles ? (p.ntiles - 1 - b) / G : NONE;
  uint32_t cur = b, nxt = b + G;
  STAMP_DECL
  uint4 w[U];
  uint32_t w4[U], gw[U];
  auto load = [&](uint32_t t) {
    const uint32_t seg0 = min(t, p.ntiles - 1) * (uint32_t)(U * TB) + (uint32_t)tid;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t sc = min(seg0 + (uint32_t)(u * TB), nseg - 1);
      w[u] = *(const uint4*)(p.payload + 4ull * sc);
      w4[u] = p.payload[4ull * sc + 4];
      gw[u] = p.gaps[(p.gap_nib0 + (sc ? sc - 1u : 0u)) >> 3];
    }
  };
  load(cur);
  if (cur >= p.ntiles) cur = NONE;
  // Grouped path: a tile's bytes stay in registers for one iteration, are staged in
  // the next and copied out two iterations later (lag 3: two iterations of slack for
  // its prefix); multi path: staged at once (emit pass), copied out at lag 2.
  constexpr bool LAG3 = GH_TILE_LAG3 && !MULTI;
  constexpr bool TOP = LAG3 && GH_TILE_TOPCOPY;  // copy-out before the decode (prefix two iterations old)
  constexpr bool FIXST = GH_TILE_FIXST && !MULTI && !TOP;  // fixed-count copy-out, prefetch just before it
  uint32_t t1 = NONE, t2 = NONE, t3 = NONE;  // tiles of iterations k-1, k-2, k-3
  uint32_t tot1 = 0, tot2 = 0, tot3 = 0;     // their totals
  uint32_t buf = 0;               // k & 1
  uint32_t pow[LAG3 ? U : 1][LAG3 ? OW : 1], pcnt[U], pbpos[U];  // grouped: tile k-1, held
#pragma unroll
  for (int u = 0; u < U; ++u) pcnt[u] = 0;
  for (uint32_t k = 0;; ++k) {
    const bool have_cur = cur < p.ntiles;
    const uint32_t tx = LAG3 ? t3 : t2;  // the tile copied out this iteration
    const bool have2 = tx < p.ntiles;
    // the workgroup that decoded tile rG + (r mod n_r) leads round r (n_r tiles) one
    // iteration later: every round, the last partial one included, has a leader
    const uint32_t lr = t1 < p.ntiles ? t1 / G : NONE;
    const bool lead = lr != NONE && t1 % G == lr % min(G, p.ntiles - lr * G);
    if (!have_cur && t1 >= p.ntiles && t2 >= p.ntiles && !have2) break;
    if (last_tile_k != NONE && k > last_tile_k + 4) {  // cannot happen; never hang the GPU
      if (tid == 0) atomicOr(p.status, (unsigned)GH_ST_TIMEOUT);
      break;
    }
    const uint32_t par = k & 1u;
#if GH_TILE_PRIO
    // the second workgroup dispatched to a CU loses every issue-arbitration tie to the
    // first (age order): alternate the two slots' priority by iteration
    if (((k + (b >= (G >> 1) ? 1u : 0u)) & 1u) != 0u) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
#endif
    STAMP(9);
    // prefix of tile k-2: R[round] + plocal[tile], read by lane 0 of every wave
    // (loaded mid-decode: a load issued at the top often saw the value a little
    // before it was published, and the re-poll then paid a full memory round trip)
    unsigned long long gr = 0, gp = 0;
    unsigned long long rl = 0;  // leader: R[lr] (wave 0 lane 0)
    if (lead && tid == 0 && lr > 0)
      rl = __hip_atomic_load(&p.rprefix[lr], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // leader: the round's aggregates, LPL consecutive tiles per lane (issued mid-decode)
    const uint32_t lt = lr * G + (uint32_t)tid * LPL;  // first tile of this lane
    const uint32_t lend = min(p.ntiles, (lr + 1) * G);
    bool lvalid[LPL];
    unsigned long long la[LPL];
#pragma unroll
    for (int j = 0; j < LPL; ++j) {
      lvalid[j] = lead && lt + j < lend;
      la[j] = 0;
    }
    auto mid = [&]() {
      if (!TOP && have2 && lane == 0) {
        const uint32_t r2 = tx / G;
        gp = __hip_atomic_load(&p.plocal[tx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        gr = r2 == 0 ? 0ull
                     : __hip_atomic_load(&p.rprefix[r2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (lead)
#pragma unroll
        for (int j = 0; j < LPL; ++j)
          la[j] = __hip_atomic_load(&p.granules[lvalid[j] ? lt + j : 0], __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
    };
    auto copy_block = [&]() {
    // ---- copy tile k-2 out (its prefix was published about an iteration ago) -------
    if (have2) {
      unsigned long long goff = 0;
      if (ABLATE(32)) {  // diagnostic: no prefix wait (wrong offsets)
        goff = (unsigned long long)tx * 16000ull;
      } else if (lane == 0) {
        const uint32_t r2 = tx / G;
        if (!granule_ok(p, gp, 2)) {
          if (p.stats && wid == 0) atomicAdd(p.stats, 1ull);
          gp = poll_granule(p, &p.plocal[tx], 2);
        }
        if (r2 > 0 && !granule_ok(p, gr, 2)) {
          if (p.stats && wid == 0) atomicAdd(p.stats + 1, 1ull);
          gr = poll_granule(p, &p.rprefix[r2], 2);
        }
        goff = (gp & VMASK) + (r2 > 0 ? (gr & VMASK) : 0ull);
        if (wid == 0 && tx == p.ntiles - 1) *p.total = goff + (LAG3 ? tot3 : tot2);
      }
      goff = rfl_u64(goff);
      STAMP(6);
      const uint32_t n2 =
          goff >= p.out_cap ? 0u : (uint32_t)min<unsigned long long>(LAG3 ? tot3 : tot2, p.out_cap - goff);
      if constexpr (FIXST) {
        load(nxt);  // the next tile's words, issued before this copy-out's stores
        if (!ABLATE(2))
          copy_out_tile_fixed<TB, GH_TILE_NS>(p.out, p.lut_bytes + (LAG3 ? buf ^ 1u : buf) * p.stage_bytes, goff, n2,
                                              tid, p.junk + (unsigned long long)blockIdx.x * TB + tid);
      } else if (!ABLATE(2)) {
        copy_out_tile<TB>(p.out, p.lut_bytes + (LAG3 ? buf ^ 1u : buf) * p.stage_bytes, goff, n2, tid,
                          (uint32_t)ABLATE(0xFFFFFFFFu));
      }
    } else if constexpr (FIXST) {
      load(nxt);
    }
    };
    if constexpr (TOP) {
      if (have2 && lane == 0) {  // published two iterations ago: almost always there
        const uint32_t r2 = tx / G;
        gp = __hip_atomic_load(&p.plocal[tx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        gr = r2 == 0 ? 0ull : __hip_atomic_load(&p.rprefix[r2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      copy_block();
    }
    // ---- decode this tile (its words were loaded during the previous iteration) --
    const uint32_t seg0 = cur * (uint32_t)(U * TB) + (uint32_t)tid;
    uint32_t ow[MULTI ? 1 : U][MULTI ? 1 : OW], cnt[U];
    // multi: the segment's words and start, kept for the emit pass after the barrier
    uint4 mw[U];
    uint32_t mw4[U];
    int mstart[U];
    bool mact[U];
    if constexpr (MULTI) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t seg = seg0 + (uint32_t)(u * TB);
        mact[u] = have_cur && seg < nseg;
        const uint32_t nib = (p.gap_nib0 + seg - 1u) & 7u;
        mstart[u] = seg == 0 ? (int)p.first_start : (int)((gw[u] >> (4 * nib)) & 15u);
        mw[u] = w[u];
        mw4[u] = w4[u];
      }
      load(nxt);  // prefetch the next iteration's tile
#pragma unroll
      for (int u = 0; u < U; ++u)
        cnt[u] = (have_cur && !ABLATE(8))
                     ? count_chain<FB>(make_win(mw[u], mw4[u], mstart[u]), mstart[u], mact[u], kshift, p, s_fb, bad)
                     : (mact[u] ? 16u : 0u);
      mid();
    } else {
      int start[U];
      bool act[U];
      uint32_t e[U][5];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t seg = seg0 + (uint32_t)(u * TB);
        act[u] = have_cur && seg < nseg;
        const uint32_t nib = (p.gap_nib0 + seg - 1u) & 7u;
        start[u] = seg == 0 ? (int)p.first_start : (int)((gw[u] >> (4 * nib)) & 15u);
        make_ewin(w[u], w4[u], start[u], S, e[u]);
      }
      if constexpr (!FIXST && (TOP || !GH_PREFETCH_LATE)) load(nxt);  // prefetch the next iteration's tile
      if (have_cur && ABLATE(8)) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          cnt[u] = act[u] ? 16u : 0u;
#pragma unroll
          for (int k2 = 0; k2 < OW; ++k2) ow[u][k2] = k2 < 4 ? e[u][k2] : 0u;
        }
        mid();
      } else if (have_cur) {
        decode_tile_grouped<(GRP > 0 ? GRP : 2), U, GH_LB_MIDG>(e, start, act, ow, cnt, amask, laneoff, mid);
      } else {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          cnt[u] = 0;
#pragma unroll
          for (int k2 = 0; k2 < OW; ++k2) ow[u][k2] = 0;
        }
        mid();
      }
    }
    STAMP(0);
    if constexpr (!TOP) copy_block();
    STAMP(1);
    if constexpr (!MULTI && !TOP && !FIXST && GH_PREFETCH_LATE) load(nxt);  // prefetch the next tile after the copy-out's waits
    uint32_t bpos[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t incl = wave_incl_scan(cnt[u], lane);
      if (lane == 63) s_wsum[(par * U + u) * NWAVE_T + wid] = incl;
      bpos[u] = incl - cnt[u];
    }
    // leader: every aggregate of the round published?  (rarely not: poll)
    uint32_t lval[LPL], lsum = 0, lincl = 0;
    if (lead) {
      bool ready = true;
#pragma unroll
      for (int j = 0; j < LPL; ++j) ready &= !lvalid[j] || granule_ok(p, la[j], 1) || granule_ok(p, la[j], 2);
      if (!__all(ready)) {
        if (lane == 0 && p.stats) atomicAdd(p.stats + 2, 1ull);
#pragma unroll
        for (int j = 0; j < LPL; ++j)
          if (lvalid[j] && !(granule_ok(p, la[j], 1) || granule_ok(p, la[j], 2)))
            la[j] = poll_granule(p, &p.granules[lt + j], 1);
      }
#pragma unroll
      for (int j = 0; j < LPL; ++j) {
        lval[j] = lvalid[j] ? (uint32_t)(la[j] & VMASK) : 0u;  // a tile holds < 2^32 symbols
        lsum += lval[j];
      }
      lincl = wave_incl_scan(lsum, lane);
      if (lane == 63) s_lead[wid] = lincl;
    }
    STAMP(2);
    __syncthreads();  // the one barrier: tile sums, leader batch totals
    STAMP(3);
    uint32_t tile_total = 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      uint32_t add = tile_total;
#pragma unroll
      for (int q = 0; q < NWAVE_T; ++q) {
        const uint32_t x = s_wsum[(par * U + u) * NWAVE_T + q];
        add += (q < wid) ? x : 0u;
        tile_total += x;
      }
      bpos[u] += add;
    }
    tile_total = __builtin_amdgcn_readfirstlane(tile_total);
    if (tid == 0 && have_cur)
      __hip_atomic_store(&p.granules[cur], granule(p.epoch, 1, tile_total), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    if (lead) {  // publish the round's within-round prefixes and R[lr + 1]
      unsigned long long before = 0, total = 0;
#pragma unroll
      for (int q = 0; q < LDR_NB; ++q) {
        const uint32_t x = s_lead[q];
        before += (q < wid) ? x : 0u;
        total += x;
      }
      unsigned long long run = before + lincl - lsum;
#pragma unroll
      for (int j = 0; j < LPL; ++j) {
        if (lvalid[j])
          __hip_atomic_store(&p.plocal[lt + j], granule(p.epoch, 2, run), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
        run += lval[j];
      }
      if (tid == 0) {
        if (lr > 0 && !granule_ok(p, rl, 2)) {
          if (p.stats) atomicAdd(p.stats + 3, 1ull);
          rl = poll_granule(p, &p.rprefix[lr], 2);
        }
        const unsigned long long r0 = lr > 0 ? (rl & VMASK) : 0ull;
        __hip_atomic_store(&p.rprefix[lr + 1], granule(p.epoch, 2, r0 + total), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    STAMP(4);
    if ((LAG3 ? t1 < p.ntiles : have_cur) && !ABLATE(4)) {
      // absolute LDS address of the staging (the kernel's LDS starts at 0): this
      // tile's (multi), the tile of iteration k-1 (grouped)
      const uint32_t sbase = p.lut_bytes + (LAG3 ? buf ^ 1u : buf) * p.stage_bytes + STAGE_PAD;
      if constexpr (MULTI) {
#pragma unroll
        for (int u = 0; u < U; ++u)
          emit_chain<FB>(make_win(mw[u], mw4[u], mstart[u]), mstart[u], mact[u], cnt[u], sbase + bpos[u],
                         kshift, p, s_fb);
      } else {
        uint32_t nb[U], hv[U], ha[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          nb[u] = 0;
          if constexpr (LAG3) {
            hv[u] = pow[u][0];
            ha[u] = sbase + pbpos[u];
            if (pcnt[u]) nb[u] = stage_aligned_p1(pow[u], pcnt[u], ha[u]);
          } else {
            hv[u] = ow[u][0];
            ha[u] = sbase + bpos[u];
            if (cnt[u]) nb[u] = stage_aligned_p1(ow[u], cnt[u], ha[u]);
          }
        }
        __syncthreads();  // phase 1 done: every segment's tail dword is in place
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (nb[u]) stage_head(ha[u], hv[u], nb[u]);
      }
    }
    STAMP(5);
    if constexpr (LAG3) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        pcnt[u] = have_cur ? cnt[u] : 0u;
        pbpos[u] = bpos[u];
#pragma unroll
        for (int m = 0; m < OW; ++m) pow[u][m] = ow[MULTI ? 0 : u][MULTI ? 0 : m];
      }
    }
    t3 = t2;
    tot3 = tot2;
    t2 = t1;
    tot2 = tot1;
    t1 = have_cur ? cur : NONE;
    tot1 = tile_total;
    buf ^= 1u;
    cur = nxt < p.ntiles ? nxt : NONE;
    nxt += G;
  }
  if (!FB && MULTI && __any(bad != 0) && lane == 0) atomicOr(p.status, (unsigned)GH_ST_BADCODE);
  STAMP_FLUSH;
}

#include "gh_msplit.hip"
#include "gh_wsplit.hip"

// ============================================================================
// Host side
// ============================================================================
struct Tables {
  uint32_t K = 0;
  bool single = false;               // single-symbol single-pass path (u32 LUT)
  bool needs_fb = true;              // some codeword is longer than the LUT width K
  std::vector<uint2> lut;            // 2^K multi-symbol entries
  std::vector<uint32_t> lut1;        // 2^K single-symbol entries
  std::vector<uint2> lut2;           // 2^K grouped-path entries {len, sym << 24}
  int g = 0;                         // grouped single-symbol path: codewords per window shift
  uint32_t fb[FB_WORDS] = {};
  uint32_t fb_lo = 1, fb_hi = 1;
  uint32_t maxsyms_seg = 128;
};

static uint32_t lut_meta_for(const Canon& c, uint32_t idx, uint32_t K, uint32_t* syms) {
  const uint32_t bits = idx << (32 - K);
  uint32_t pos = 0, n = 0, s = 0;
  uint32_t ends[5] = {0, 15, 15, 15, 15};
  while (n < 4 && pos < K) {
    const uint32_t w16 = (bits << pos) >> 16;
    uint32_t fi = 0;
    const uint32_t l = canon_decode16(c, w16, &fi);
    if (l == 0 || pos + l > K) break;
    s |= (uint32_t)c.sym[fi] << (8 * n);
    ++n;
    pos += l;
    ends[n] = pos;
  }
  *syms = s;
  if (n == 0) return make_meta(0, 0, 15, 15, 15);
  return make_meta(n, pos, 1 < n ? ends[1] : 15u, 2 < n ? ends[2] : 15u, 3 < n ? ends[3] : 15u);
}

// Expected lookups per symbol for width K under the code's own model (P(code) =
// 2^-len); fallback lookups are weighted 3x.  Picks the cheapest K in [6,12],
// preferring smaller tables within 3%.
static uint32_t choose_k(const Canon& c) {
  double best = 1e30;
  uint32_t bestk = 12;
  double cost[13] = {};
  for (uint32_t K = 6; K <= 12; ++K) {
    double syms = 0, fbp = 0;
    for (uint32_t i = 0; i < (1u << K); ++i) {
      uint32_t s;
      const uint32_t m = lut_meta_for(c, i, K, &s);
      const uint32_t n = (m >> 16) & 7u;
      if (n == 0) {
        fbp += 1.0;
        syms += 1.0;
      } else {
        syms += n;
      }
    }
    syms /= (double)(1u << K);
    fbp /= (double)(1u << K);
    cost[K] = (1.0 + 2.0 * fbp) / syms;
    best = std::min(best, cost[K]);
  }
  for (uint32_t K = 6; K <= 12; ++K)
    if (cost[K] <= best * 1.03) {
      bestk = K;
      break;
    }
  return bestk;
}

// Expected symbols per lookup of the multi-symbol table at width K.
static double multi_gain(const Canon& c, uint32_t K) {
  double syms = 0;
  for (uint32_t i = 0; i < (1u << K); ++i) {
    uint32_t s;
    const uint32_t n = (lut_meta_for(c, i, K, &s) >> 16) & 7u;
    syms += n ? n : 1;
  }
  return syms / (double)(1u << K);
}

static int build_tables(const Canon& c, Tables& t, int force_k, int force_path) {
  if (c.nsyms == 0) return fail(GH_E_TABLE, "empty code");
  // Single-pass single-symbol path when every segment fits 32 symbols (minlen >= 4)
  // and 12-bit multi-symbol lookups would average < 1.5 symbols.
  t.single = (force_path == 1 || force_path == 3) ||
             (force_path != 2 && c.minlen >= 4 && multi_gain(c, 12) < 1.5);
  if (c.minlen < 4) t.single = false;
  if (t.single) {
    t.K = force_k > 0 ? (uint32_t)std::clamp(force_k, 1, 12) : std::min<uint32_t>(c.maxlen, 12);
    t.lut1.assign(1u << t.K, 0u);
    for (uint32_t i = 0; i < (1u << t.K); ++i) {
      uint32_t fi = 0;
      const uint32_t l = canon_decode16(c, (i << (32 - t.K)) >> 16, &fi);
      if (l == 0 || l > t.K) continue;  // fallback entry (b = 0)
      t.lut1[i] = ((32u - l) & 31u) | (l << 8) | ((uint32_t)c.sym[fi] << 24);
    }
    t.lut.clear();
    if (t.lut1.size() < 4) t.lut1.resize(4, 0u);  // LDS copy moves 16-byte chunks
    // grouped path: complete code (Kraft sum 1), all codewords within K bits
    uint64_t kraft = 0;
    for (uint32_t l = 1; l <= 16; ++l) kraft += (uint64_t)c.count[l] << (16 - l);
    t.g = 0;
    t.lut2.clear();
    if (force_path != 3 && kraft == 65536 && c.maxlen <= t.K && c.maxlen <= 15) {
      t.g = std::min<int>(4, 31 / (int)c.maxlen);
      t.lut2.assign(1u << t.K, make_uint2(0, 0));
      for (uint32_t i = 0; i < (1u << t.K); ++i) {
        uint32_t fi = 0;
        const uint32_t l = canon_decode16(c, (i << (32 - t.K)) >> 16, &fi);
        t.lut2[i] = make_uint2(l, (uint32_t)c.sym[fi] << 24);
      }
      if (t.lut2.size() < 2) t.lut2.resize(2, make_uint2(0, 0));
    }
  } else {
    t.g = 0;
    t.lut2.clear();
    t.K = force_k > 0 ? (uint32_t)std::clamp(force_k, 1, 12) : choose_k(c);
    t.lut.assign(1u << t.K, make_uint2(0, 0));
    for (uint32_t i = 0; i < (1u << t.K); ++i) {
      uint32_t s;
      const uint32_t m = lut_meta_for(c, i, t.K, &s);
      t.lut[i] = make_uint2(s, m);
    }
    if (t.lut.size() < 2) t.lut.resize(2, make_uint2(0, 0));
    t.lut1.clear();
  }
  // fallback: running limits so empty lengths never match
  uint32_t run = 0;
  for (uint32_t l = 1; l <= 16; ++l) {
    if (c.count[l]) run = c.limit16[l];
    t.fb[l] = run;             // limit16
    t.fb[17 + l] = c.base16[l];
    t.fb[34 + l] = c.first[l];
  }
  uint8_t* sy = (uint8_t*)(t.fb + 51);
  for (uint32_t i = 0; i < c.nsyms; ++i) sy[i] = c.sym[i];
  t.fb_lo = std::min<uint32_t>(t.K + 1, 16);
  t.fb_lo = std::max<uint32_t>(t.fb_lo, c.minlen);
  t.fb_hi = std::max<uint32_t>(c.maxlen, t.fb_lo);
  t.maxsyms_seg = (128 + c.minlen - 1) / c.minlen;
  t.needs_fb = c.maxlen > t.K;
  return GH_OK;
}

}  // namespace gh

using namespace gh;

#define GH_HIP(expr)                                                              \
  do {                                                                            \
    hipError_t e_ = (expr);                                                       \
    if (e_ != hipSuccess)                                                         \
      return fail(GH_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));   \
  } while (0)

static void** args_of(DecodeParams& p) {
  static thread_local void* a[1];
  a[0] = &p;
  return a;
}

template <bool SINGLE, bool FB>
static const void* kernel_for_u(int uv) {
  switch (uv) {
    case 4: return (const void*)gh_decode_kernel<SINGLE, FB, 4, 0, TB>;
    case 2: return (const void*)gh_decode_kernel<SINGLE, FB, 2, 0, TB>;
    default: return (const void*)gh_decode_kernel<SINGLE, FB, 1, 0, TB>;
  }
}

template <int G>
static const void* kernel_for_g(int uv) {
  return uv >= 2 ? (const void*)gh_decode_kernel<true, false, 2, G, TB_G>
                 : (const void*)gh_decode_kernel<true, false, 1, G, TB_G>;
}

// The no-fallback variants apply when every codeword fits the LUT width; the
// grouped variants (g > 0) when the code is also complete.
static const void* kernel_for(bool single, bool fb, int uv, int g = 0) {
  if (g > 0) return g >= 4 ? kernel_for_g<4>(uv) : g == 3 ? kernel_for_g<3>(uv) : kernel_for_g<2>(uv);
  if (single) return fb ? kernel_for_u<true, true>(uv) : kernel_for_u<true, false>(uv);
  return fb ? kernel_for_u<false, true>(uv) : kernel_for_u<false, false>(uv);
}

// Split-mode kernels: {count, write} for a path.  Workgroups of 256 threads.
constexpr int TB_S = 256;
struct SplitKernels {
  const void* count;
  const void* write;
};
template <bool SINGLE, bool FB, int U, int G>
static SplitKernels split_pair() {
  return {(const void*)gh_count_kernel<SINGLE, FB, U, G, TB_S>,
          (const void*)gh_write_kernel<SINGLE, FB, U, G, TB_S>};
}
static SplitKernels split_for(bool single, bool fb, int uv, int g) {
  if (g > 0)
    return g >= 4 ? split_pair<true, false, 2, 4>()
           : g == 3 ? split_pair<true, false, 2, 3>() : split_pair<true, false, 2, 2>();
  if (single) return fb ? split_pair<true, true, 2, 0>() : split_pair<true, false, 2, 0>();
  if (uv >= 2) return fb ? split_pair<false, true, 2, 0>() : split_pair<false, false, 2, 0>();
  return fb ? split_pair<false, true, 1, 0>() : split_pair<false, false, 1, 0>();
}

// Tile-mode kernel geometry: the grouped path runs 512-thread workgroups with two
// segments per lane; the multi-symbol paths 1024-thread workgroups with one (their
// staging is up to 64 bytes per segment).
#ifndef GH_TB_GRP
#define GH_TB_GRP 512  // grouped tile path workgroup size (256: 4 per CU, measured 1.5x slower: more stragglers per round)
#endif
#ifndef GH_U_GRP
#define GH_U_GRP 2  // grouped tile path: segments per lane
#endif
constexpr int TB_GRP = GH_TB_GRP, U_GRP = GH_U_GRP, TB_MUL = 1024, U_MUL = 1;
static const void* tile_kernel_for(int path, uint32_t g) {
  if (path == TP_MULTI) return (const void*)gh_tile_kernel<TB_MUL, U_MUL, TP_MULTI, 0>;
  if (path == TP_MULTI_FB) return (const void*)gh_tile_kernel<TB_MUL, U_MUL, TP_MULTI_FB, 0>;
  return g >= 4 ? (const void*)gh_tile_kernel<TB_GRP, U_GRP, TP_GROUPED, 4>
       : g == 3 ? (const void*)gh_tile_kernel<TB_GRP, U_GRP, TP_GROUPED, 3>
                : (const void*)gh_tile_kernel<TB_GRP, U_GRP, TP_GROUPED, 2>;
}

struct gh_ctx {
  int device = 0;
  bool tile = false;       // tile mode (gh_tile_kernel); else split or fused
  int tile_path = 0;       // tile mode: TP_*
  uint32_t tile_g = 0;     // tile mode: codewords per window shift (grouped path)
  uint32_t lgr = 0;        // tile mode: log2 of the LUT replication
  uint32_t* d_lut_t = nullptr;  // tile mode: compact u32 LUT
  bool split = true;       // split mode (count / scan / write) vs the fused persistent kernel
  bool ms = false;         // lean multi-symbol split kernels (gh_msplit.hip)
  bool ws = false;         // wave-independent split kernels (gh_wsplit.hip)
  uint32_t ws_nblocks = 0, ws_nranges = 0, ws_grid_c = 0;
  int ws_ns = 4;
  uint32_t ws_kc = 0;              // width of the wave-split count LUT
  bool ws_fb = false;              // wave split with the canonical fallback (long / incomplete codes)
  uint32_t* d_ws_lut_c = nullptr;  // its u32 entries {b | end mask << 16}
  uint4* d_ws_junk = nullptr;
  uint4* d_tile_junk = nullptr;  // tile mode: one 16-byte slot per thread of the grid
  unsigned long long* d_rng_tot = nullptr;
  unsigned long long* d_rng_off = nullptr;
  uint32_t ms_k = 0;       // their LUT width
  int ms_wu = 2;           // their write kernel's chains per thread
  uint32_t ms_last_end = 0;  // end bit of the stream's last segment when the shard holds it
  uint2* d_ms_lut_c = nullptr;  // count LUT {b, end mask}
  uint2* d_ms_lut_w = nullptr;  // write LUT {symbols, b | n << 8}
  uint32_t count_per = 1;  // split mode: count workgroups per write workgroup
  size_t lds_count = 0;    // split mode: dynamic LDS of the count / write kernels
  uint8_t* d_seg_cnt = nullptr;
  uint32_t* d_tile_cnt = nullptr;
  unsigned long long* d_tile_off = nullptr;
  unsigned long long* d_wg_tot = nullptr;
  int tb = TB;           // workgroup size of the loaded path
  size_t lut_bytes = 0;  // LDS bytes of the decode LUT of the loaded path
  hipStream_t stream = nullptr;
  hipEvent_t done = nullptr;  // recorded after every decode, on the stream it ran on
  bool done_rec = false;
  int num_cu = 0;
  bool loaded = false;
  Canon canon;
  Tables tables;
  uint64_t nseg = 0, seg_begin = 0, seg_end = 0, n_total = 0;
  uint32_t* d_payload = nullptr;
  uint32_t* d_gaps = nullptr;
  uint8_t* d_out = nullptr;
  uint64_t out_cap = 0;
  unsigned long long* d_gran = nullptr;
  unsigned int* d_misc = nullptr;  // [0] ticket, [1] status, [2..3] total
  uint2* d_lut = nullptr;
  uint32_t* d_fb = nullptr;
  unsigned long long* d_stamps = nullptr;  // GH_STAMPS builds only
  uint32_t epoch = 0;
  uint64_t gran_words = 0;  // u64 granules allocated at d_gran
  uint32_t ntiles = 0;   // super-tiles
  uint32_t super = 1;    // sub-tiles per super-tile (kernel template S)
  uint32_t grid = 0;
  uint32_t gap_nib0 = 0, first_start = 0;
  size_t lds = 0;
  uint32_t stage_bytes = 0;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> pending, pool;
  double acc_ms = 0;
  uint32_t nlaunch = 0;
};

static void free_shard(gh_ctx* c) {
  (void)hipSetDevice(c->device);
  (void)hipFree(c->d_payload);
  (void)hipFree(c->d_gaps);
  (void)hipFree(c->d_out);
  (void)hipFree(c->d_gran);
  (void)hipFree(c->d_lut);
  (void)hipFree(c->d_fb);
  (void)hipFree(c->d_stamps);
  (void)hipFree(c->d_seg_cnt);
  (void)hipFree(c->d_tile_cnt);
  (void)hipFree(c->d_tile_off);
  (void)hipFree(c->d_wg_tot);
  (void)hipFree(c->d_lut_t);
  (void)hipFree(c->d_ms_lut_c);
  (void)hipFree(c->d_ms_lut_w);
  (void)hipFree(c->d_rng_tot);
  (void)hipFree(c->d_rng_off);
  (void)hipFree(c->d_ws_junk);
  c->d_ws_junk = nullptr;
  (void)hipFree(c->d_ws_lut_c);
  c->d_ws_lut_c = nullptr;
  (void)hipFree(c->d_tile_junk);
  c->d_tile_junk = nullptr;
  c->d_rng_tot = nullptr;
  c->d_rng_off = nullptr;
  c->ws = false;
  c->d_ms_lut_c = nullptr;
  c->d_ms_lut_w = nullptr;
  c->ms = false;
  c->d_lut_t = nullptr;
  c->d_wg_tot = nullptr;
  c->d_seg_cnt = nullptr;
  c->d_tile_cnt = nullptr;
  c->d_tile_off = nullptr;
  c->d_stamps = nullptr;
  c->d_payload = nullptr;
  c->d_gaps = nullptr;
  c->d_out = nullptr;
  c->d_gran = nullptr;
  c->d_lut = nullptr;
  c->d_fb = nullptr;
  c->loaded = false;
}

struct MsKernels {
  const void* count;
  const void* write;
  int wu, tbw;  // write kernel: chains per thread, threads
};
template <int GL>
static MsKernels ms_pair(int wu) {
  if (wu == 1)
    return {(const void*)gh_ms_count_kernel<U_MS, TB_MS, GL>, (const void*)gh_ms_write_kernel<1, MS_TILE, GL>, 1,
            MS_TILE};
  return {(const void*)gh_ms_count_kernel<U_MS, TB_MS, GL>, (const void*)gh_ms_write_kernel<2, MS_TILE / 2, GL>, 2,
          MS_TILE / 2};
}
// Write-kernel chains per thread: one (512 threads) for LUTs of up to 10 bits, two
// otherwise (measured: cfg2, K=10, 120 vs 127 us; cfg3, K=11, 675 vs 655 us).
// GH_MS_WU=1|2 overrides.
static int ms_write_chains(uint32_t K) {
  if (const char* e = getenv("GH_MS_WU")) return atoi(e) == 1 ? 1 : 2;
  return K <= 10 ? 1 : 2;
}
static MsKernels ms_kernels(uint32_t K, int wu) {
  const int g = ms_group(K);
  return g >= 4 ? ms_pair<4>(wu) : g == 3 ? ms_pair<3>(wu) : ms_pair<2>(wu);
}

// Lean multi-symbol split kernels: LUTs, geometry, buffers (gh_msplit.hip).
// Entry i of the K-bit LUTs decodes, greedily, up to four codewords lying wholly in
// the K bits i: count LUT {b = their bits, end mask (bit e-1 per codeword end e)},
// write LUT {their symbols (byte k = k-th), b | n << 8}.  Requires a complete code
// with maxlen <= K, so every entry holds at least one codeword.
static int ms_build_luts(gh_ctx* c, uint32_t K, bool allow_fb = false) {
  const Canon& cn = c->canon;
  std::vector<uint2> lc(1u << K), lw(1u << K);
  for (uint32_t i = 0; i < (1u << K); ++i) {
    const uint32_t bits = i << (32 - K);
    uint32_t pos = 0, n = 0, syms = 0, mask = 0;
    while (n < 4 && pos < K) {
      uint32_t fi = 0;
      const uint32_t l = canon_decode16(cn, (bits << pos) >> 16, &fi);
      if (l == 0 || pos + l > K) break;
      syms |= (uint32_t)cn.sym[fi] << (8 * n);
      ++n;
      pos += l;
      mask |= 1u << (pos - 1);
    }
    if (n == 0 && !allow_fb) return fail(GH_E_TABLE, "msplit: LUT entry without a codeword");
    lc[i] = make_uint2(pos, mask);
    lw[i] = make_uint2(syms, pos | (n << 8));
  }
  const size_t lb = 8ull << K;  // >= 32 bytes: whole 16-byte chunks
  GH_HIP(hipMalloc(&c->d_ms_lut_c, lb));
  GH_HIP(hipMalloc(&c->d_ms_lut_w, lb));
  GH_HIP(hipMemcpy(c->d_ms_lut_c, lc.data(), lb, hipMemcpyHostToDevice));
  GH_HIP(hipMemcpy(c->d_ms_lut_w, lw.data(), lb, hipMemcpyHostToDevice));
  c->ms_k = K;
  c->lut_bytes = lb;
  return GH_OK;
}
// LUT width of the multi-symbol split kernels: GH_MS_K, default 10, at least maxlen.
static uint32_t ms_lut_bits(const Canon& cn) {
  const char* ek = getenv("GH_MS_K");
  return (uint32_t)std::clamp(ek ? atoi(ek) : 10, (int)std::min<uint32_t>(std::max<uint32_t>(cn.maxlen, 2), 12), 12);
}
static int ms_setup(gh_ctx* c) {
  const Canon& cn = c->canon;
  const uint32_t K = ms_lut_bits(cn);
  if (int rc = ms_build_luts(c, K)) return rc;
  const size_t lb = c->lut_bytes;
  c->tb = TB_MS;
  c->super = U_MS;
  c->ntiles = (uint32_t)ceil_div(c->nseg, (uint64_t)U_MS * TB_MS);
  // codewords per segment: wholly inside [start, E), E - start <= 143
  const uint32_t maxsyms = std::min<uint32_t>(143 / std::max<uint32_t>(cn.minlen, 1) + 1, 255);
  // Staging: the most workgroups per CU (8 .. 1) whose staging still holds one
  // chain's worst case (TB_MS segments x maxsyms); a tile that exceeds it is staged
  // one chain at a time (gh_ms_write_kernel).
  const MsKernels mk = ms_kernels(K, ms_write_chains(K));
  const int NW = mk.tbw / 64;
  const size_t misc = 4 * (mk.wu * NW + 2) + 8 * NW;
  const size_t chain_worst = (size_t)mk.tbw * maxsyms + 64 + 32;
  const size_t full_worst = (size_t)mk.wu * mk.tbw * maxsyms + 64 + 32;
  size_t stage = 0;
  for (int wg = 8; wg >= 1 && stage == 0; --wg) {
    const long avail = (long)(163840 / wg) - (long)lb - (long)misc;
    if (avail >= (long)chain_worst) stage = std::min<size_t>((size_t)avail & ~15ull, (full_worst + 15) & ~15ull);
  }
  if (stage == 0) return fail(GH_E_HIP, "msplit staging does not fit");
  if (const char* es = getenv("GH_MS_STAGE"))  // tests: force a small staging (per-chain tiles)
    stage = std::max<size_t>((size_t)atoll(es), (chain_worst + 15) & ~15ull) & ~15ull;
  c->stage_bytes = (uint32_t)stage;
  c->lds = lb + c->stage_bytes + misc;
  c->lds_count = std::max<size_t>(lb, 64);
  int pc_c = 0, pc_w = 0;
  c->ms_wu = mk.wu;
  GH_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&pc_c, mk.count, TB_MS, c->lds_count));
  GH_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&pc_w, mk.write, mk.tbw, c->lds));
  if (pc_c < 1 || pc_w < 1) return fail(GH_E_HIP, "msplit kernels do not fit on a CU");
  c->grid = (uint32_t)std::min<uint64_t>(c->ntiles, (uint64_t)pc_w * c->num_cu);
  // count ranges nest in write ranges (floor(b*n/grid) boundaries coincide for
  // grid_c = k*grid_w)
  const uint32_t kk = std::max(1, pc_c / pc_w);
  c->count_per = 1;
  for (uint32_t k2 = kk; k2 >= 1; --k2)
    if ((uint64_t)k2 * c->grid <= c->ntiles) { c->count_per = k2; break; }
  GH_HIP(hipMalloc(&c->d_seg_cnt, c->nseg + 16));
  GH_HIP(hipMalloc(&c->d_wg_tot, 8ull * c->grid * c->count_per + 16));
  c->ms = true;
  c->split = false;
  c->tile = false;
  return GH_OK;
}

// Wave-independent split kernels (gh_wsplit.hip): the msplit LUTs, a per-wave staging
// buffer, ranges of `bpr` blocks of 64 * WS_U segments handed out by tickets.
struct WsKernels {
  const void* count;
  const void* write;
};
template <int GL, bool FB = false>
static const void* ws_write_ns(int ns) {
  return ns <= 2 ? (const void*)gh_ws_write_kernel<WS_U, WS_TB, GL, 2, FB>
         : ns <= 3 ? (const void*)gh_ws_write_kernel<WS_U, WS_TB, GL, 3, FB>
         : ns <= 4 ? (const void*)gh_ws_write_kernel<WS_U, WS_TB, GL, 4, FB>
         : ns <= 6 ? (const void*)gh_ws_write_kernel<WS_U, WS_TB, GL, 6, FB>
                   : (const void*)gh_ws_write_kernel<WS_U, WS_TB, GL, 8, FB>;
}
// Count kernel by its LUT width Kc, write kernel by K and NS (store instructions per
// lane per piece: the typical piece's 16-byte chunks / 64).  fb: codes longer than the
// tables or incomplete codes (canonical fallback, two lookups per window shift).
static WsKernels ws_kernels(uint32_t Kc, uint32_t K, int ns, bool fb = false) {
  if (fb) return {(const void*)gh_ws_count_kernel<WS_UC, WS_TBC, 2, true>, ws_write_ns<2, true>(ns)};
  const int gc = ms_group(Kc), g = ms_group(K);
  const void* cnt = gc >= 4 ? (const void*)gh_ws_count_kernel<WS_UC, WS_TBC, 4>
                    : gc == 3 ? (const void*)gh_ws_count_kernel<WS_UC, WS_TBC, 3>
                              : (const void*)gh_ws_count_kernel<WS_UC, WS_TBC, 2>;
  const void* wr = g >= 4 ? ws_write_ns<4>(ns) : g == 3 ? ws_write_ns<3>(ns) : ws_write_ns<2>(ns);
  return {cnt, wr};
}

// Count LUT of width Kc (u32 entries b | end mask << 16, see gh_ws_count_kernel): every
// codeword wholly inside the Kc-bit window, greedily.  Returns the expected bits per
// lookup on random input bits (for a complete code each codeword then has probability
// 2^-len, about its frequency in the data it was built for).
static double ws_count_lut(const Canon& cn, uint32_t Kc, std::vector<uint32_t>* out) {
  double sum = 0;
  if (out) out->assign(1u << Kc, 0u);
  for (uint32_t i = 0; i < (1u << Kc); ++i) {
    const uint32_t bits = i << (32 - Kc);
    uint32_t pos = 0, mask = 0;
    while (pos < Kc) {
      uint32_t fi = 0;
      const uint32_t l = canon_decode16(cn, (bits << pos) >> 16, &fi);
      if (l == 0 || pos + l > Kc) break;
      pos += l;
      mask |= 1u << (pos - 1);
    }
    sum += pos;
    if (out) (*out)[i] = pos | (mask << 16);
  }
  return sum / (double)(1u << Kc);
}
// Kc in [max(maxlen, 2), 13] maximising bits per VALU op of a lookup group: GL lookups
// of ~7 ops each plus ~11 ops of window shift and mask upkeep per chain.  GH_WS_KC
// overrides (tests).
static uint32_t ws_count_bits(const Canon& cn) {
  const uint32_t lo = std::min<uint32_t>(std::max<uint32_t>(cn.maxlen, 2), 13);  // longer codes: fallback
  if (const char* e = getenv("GH_WS_KC")) return (uint32_t)std::clamp(atoi(e), (int)lo, 14);
  uint32_t best = lo;
  double best_eff = -1;
  for (uint32_t kc = lo; kc <= 13; ++kc) {  // 14 (64 KiB) measured no faster
    const int gl = ms_group(kc);
    const double eff = gl * ws_count_lut(cn, kc, nullptr) / (7.0 * gl + 11.0);
    if (eff > best_eff * 1.01) {  // prefer the smaller table unless clearly better
      best_eff = eff;
      best = kc;
    }
  }
  return best;
}
static int ws_ns_for(double avg_seg_bytes) {
  const double chunks = avg_seg_bytes * 64 * WS_U / 16.0 * 1.15 + 2;
  const int ns = (int)std::ceil(chunks / 64);
  return ns <= 2 ? 2 : ns <= 3 ? 3 : ns <= 4 ? 4 : ns <= 6 ? 6 : 8;
}
// Write-LUT width of the wave split: K in [max(maxlen, 10), 12] maximising the expected
// bits per lookup (entries hold up to four codewords, so a wider window helps only codes
// whose short codewords it can fit more of: r=0.5 codes 7.6 -> 10.4 bits at K 10 -> 12)
// times lookups per window shift over ~13 ops per lookup plus ~12 per shift; a wider
// table must win by 5 % (its LDS costs occupancy).  GH_MS_K overrides.
static uint32_t ws_write_bits(const Canon& cn) {
  if (getenv("GH_MS_K")) return ms_lut_bits(cn);
  const uint32_t lo = std::min<uint32_t>(std::max<uint32_t>(cn.maxlen, 10), 12);  // longer codes: fallback
  uint32_t best = lo;
  double best_eff = -1;
  for (uint32_t K = lo; K <= 12; ++K) {
    double sum = 0;
    for (uint32_t i = 0; i < (1u << K); ++i) {
      const uint32_t bits = i << (32 - K);
      uint32_t pos = 0, n = 0;
      while (n < 4 && pos < K) {
        uint32_t fi = 0;
        const uint32_t l = canon_decode16(cn, (bits << pos) >> 16, &fi);
        if (l == 0 || pos + l > K) break;
        pos += l;
        ++n;
      }
      sum += pos;
    }
    const int gl = ms_group(K);
    const double eff = gl * (sum / (double)(1u << K)) / (13.0 * gl + 12.0);
    if (best_eff < 0 || eff > best_eff * 1.05) {
      best_eff = eff;
      best = K;
    }
  }
  return best;
}

static int ws_setup(gh_ctx* c, double avg_seg_bytes) {
  const Canon& cn = c->canon;
  const uint32_t K = ws_write_bits(cn);
  // canonical fallback: codewords longer than a table, or patterns outside an incomplete
  // code (a LUT entry with no codeword)
  uint64_t kraft = 0;
  for (uint32_t l = 1; l <= 16; ++l) kraft += (uint64_t)cn.count[l] << (16 - l);
  const bool fb = kraft != 65536 || cn.maxlen > std::min<uint32_t>(K, ws_count_bits(cn));
  c->ws_fb = fb;
  if (int rc = ms_build_luts(c, K, fb)) return rc;
  const size_t lb = c->lut_bytes + (fb ? (size_t)FB_BYTES : 0);  // write kernel: LUT + fallback tables
  constexpr int NW = WS_TB / 64;
  {
    const uint32_t kc = ws_count_bits(cn);
    std::vector<uint32_t> lc;
    ws_count_lut(cn, kc, &lc);
    GH_HIP(hipMalloc(&c->d_ws_lut_c, 4ull << kc));
    GH_HIP(hipMemcpy(c->d_ws_lut_c, lc.data(), 4ull << kc, hipMemcpyHostToDevice));
    c->ws_kc = kc;
  }
  const uint32_t maxsyms = std::min<uint32_t>(143 / std::max<uint32_t>(cn.minlen, 1) + 1, 255);
  // per-wave staging: at least one chain's worst case (64 segments x maxsyms), and a
  // typical whole block (both chains) with room to spare when the LDS allows
  const size_t chain_worst = 64ull * maxsyms + 64;
  const size_t full_worst = 64ull * WS_U * maxsyms + 64;
  const size_t typical = (size_t)(1.3 * avg_seg_bytes * 64 * WS_U) + 64;
  const size_t want = std::max(chain_worst, std::min(full_worst, typical));
  size_t stage = 0;
  for (int wg = 8; wg >= 1 && stage == 0; --wg) {
    const long avail = ((long)(163840 / wg) - (long)lb) / NW;
    if (avail >= (long)want) stage = std::min<size_t>((size_t)avail, full_worst + 15) & ~15ull;
  }
  if (stage == 0) {
    const long avail = ((long)163840 - (long)lb) / NW;
    if (avail < (long)chain_worst) return fail(GH_E_HIP, "wsplit staging does not fit");
    stage = (size_t)avail & ~15ull;
  }
  if (const char* es = getenv("GH_MS_STAGE"))  // tests: force a small staging (per-chain blocks)
    stage = std::max<size_t>((size_t)atoll(es), (chain_worst + 15) & ~15ull) & ~15ull;
  c->stage_bytes = (uint32_t)stage;
  c->lds = lb + NW * stage;
  c->lds_count = std::max<size_t>(4ull << c->ws_kc, 64) + (fb ? FB_BYTES : 0);
  c->ws_ns = ws_ns_for(avg_seg_bytes);
  if (const char* en = getenv("GH_WS_NS")) c->ws_ns = std::clamp(atoi(en), 2, 8);
  const WsKernels k = ws_kernels(c->ws_kc, K, c->ws_ns, fb);
  int pc_c = 0, pc_w = 0;
  GH_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&pc_c, k.count, WS_TBC, c->lds_count));
  GH_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&pc_w, k.write, WS_TB, c->lds));
  if (pc_c < 1 || pc_w < 1) return fail(GH_E_HIP, "wsplit kernels do not fit on a CU");
  c->ws_nblocks = (uint32_t)ceil_div(c->nseg, (uint64_t)WS_SB);  // superblocks
  const uint64_t wg_blocks = ceil_div(c->ws_nblocks, (uint64_t)NW);  // workgroups that have a superblock
  c->grid = (uint32_t)std::min<uint64_t>((uint64_t)pc_w * c->num_cu, wg_blocks);
  c->ws_grid_c = (uint32_t)std::min<uint64_t>((uint64_t)pc_c * c->num_cu, ceil_div(c->ws_nblocks, (uint64_t)(WS_TBC / 64)));
  if (const char* eg = getenv("GH_WS_GRID")) {  // tests: few workgroups, many blocks per wave
    c->grid = (uint32_t)std::clamp<long>(atol(eg), 1, (long)c->grid);
    c->ws_grid_c = (uint32_t)std::clamp<long>(atol(eg), 1, (long)c->ws_grid_c);
  }
  c->ws_nranges = c->grid * (uint32_t)NW;  // one contiguous range per wave of the write grid
  c->ntiles = c->ws_nblocks;
  c->super = WS_U;
  c->tb = WS_TB;
  c->ms_wu = WS_U;
  GH_HIP(hipMalloc(&c->d_seg_cnt, c->nseg + 16));
  GH_HIP(hipMalloc(&c->d_ws_junk, 16ull * 64 * c->ws_nranges));
  GH_HIP(hipMalloc(&c->d_rng_tot, 8ull * c->ws_nranges + 16));
  GH_HIP(hipMalloc(&c->d_rng_off, 8ull * c->ws_nranges + 16));
  c->ws = true;
  c->ms = false;
  c->split = false;
  c->tile = false;
  return GH_OK;
}

// End bit of the stream's last segment (segment-relative) under the reference rule
// "codewords starting before bit 128" (decoder.cu:529-569), its zero padding
// decoded like the reference's: the end of the last codeword starting before 128.
static uint32_t last_segment_end(const Canon& cn, const uint32_t* w5, uint32_t start) {
  uint32_t pos = start;
  while (pos < 128) {
    const uint32_t wi = pos >> 5, sh = pos & 31;
    const uint32_t hi = w5[wi], lo = wi + 1 < 5 ? w5[wi + 1] : 0u;
    const uint32_t w32 = sh ? (hi << sh) | (lo >> (32 - sh)) : hi;
    uint32_t fi = 0;
    const uint32_t l = canon_decode16(cn, w32 >> 16, &fi);
    if (l == 0) break;
    pos += l;
  }
  return std::max<uint32_t>(pos, 128);
}

// Start bit of global segment i (i >= 1) from the host gap words.
static uint32_t seg_start_host(const gh_stream* s, uint64_t i) {
  const uint64_t nib = i - 1;
  uint32_t wv;
  std::memcpy(&wv, (const uint8_t*)s->gap_words + 4 * (nib >> 3), 4);
  return (wv >> (4 * (nib & 7))) & 15u;
}

extern "C" int gh_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

extern "C" int gh_ctx_create(int device, gh_ctx** out) {
  if (!out) return fail(GH_E_ARG, "null ctx pointer");
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0)
    return fail(GH_E_NODEV, "no HIP device visible (the decoder has no CPU fallback)");
  if (device < 0 || device >= n) return fail(GH_E_ARG, "device ordinal out of range");
  hipDeviceProp_t prop;
  GH_HIP(hipGetDeviceProperties(&prop, device));
  if (std::string(prop.gcnArchName).find("gfx950") == std::string::npos)
    return fail(GH_E_NODEV, std::string("device is ") + prop.gcnArchName + ", need gfx950");
  gh_ctx* c = new gh_ctx();
  c->device = device;
  c->num_cu = prop.multiProcessorCount;
  GH_HIP(hipSetDevice(device));
  GH_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
  GH_HIP(hipEventCreateWithFlags(&c->done, hipEventDisableTiming));
  GH_HIP(hipMalloc(&c->d_misc, 128));
  GH_HIP(hipMemset(c->d_misc, 0, 128));
  for (bool sg : {false, true})
    for (bool fbv : {false, true})
      for (int sv : {1, 2, 4})
        (void)hipFuncSetAttribute(kernel_for(sg, fbv, sv),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  for (int gv : {2, 3, 4})
    for (int sv : {1, 2})
      (void)hipFuncSetAttribute(kernel_for(true, false, sv, gv),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  for (int tp : {TP_GROUPED, TP_MULTI, TP_MULTI_FB})
    for (uint32_t gv : {2u, 3u, 4u})
      (void)hipFuncSetAttribute(tile_kernel_for(tp, gv), hipFuncAttributeMaxDynamicSharedMemorySize,
                                160 * 1024);
  for (int gv : {0, 2, 3, 4})
    for (bool sg : {false, true})
      for (bool fbv : {false, true})
        for (int sv : {1, 2}) {
          const SplitKernels k = split_for(sg, fbv, sv, gv);
          (void)hipFuncSetAttribute(k.count, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
          (void)hipFuncSetAttribute(k.write, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        }
  (void)hipGetLastError();
  *out = c;
  return GH_OK;
}

extern "C" int gh_ctx_device(gh_ctx* c, int* device) {
  if (!c || !device) return fail(GH_E_ARG, "null argument");
  *device = c->device;
  return GH_OK;
}

extern "C" int gh_ctx_destroy(gh_ctx* c) {
  if (!c) return GH_OK;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  free_shard(c);
  (void)hipFree(c->d_misc);
  for (auto& e : c->pending) {
    (void)hipEventDestroy(e.first);
    (void)hipEventDestroy(e.second);
  }
  for (auto& e : c->pool) {
    (void)hipEventDestroy(e.first);
    (void)hipEventDestroy(e.second);
  }
  if (c->done) (void)hipEventDestroy(c->done);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return GH_OK;
}

static int load_common(gh_ctx* c, const gh_stream* s, uint64_t b, uint64_t e, uint64_t out_cap) {
  if (!c || !s) return fail(GH_E_ARG, "null argument");
  if (b > e || e > s->g) return fail(GH_E_ARG, "shard range outside [0, G]");
  free_shard(c);
  int rc = build_canon(s->syms, s->nsyms, c->canon);
  if (rc) return rc;
  c->nseg = e - b;
  c->seg_begin = b;
  c->seg_end = e;
  c->n_total = s->n;
  if (c->nseg > 0) {
    const char* envk = getenv("GH_LUT_BITS");
    const char* envp = getenv("GH_PATH");
    rc = build_tables(c->canon, c->tables, envk ? atoi(envk) : 0, envp ? atoi(envp) : 0);
    if (rc) return rc;
    // tile mode runs the grouped single-symbol path or the multi-symbol paths
    const char* envm0 = getenv("GH_MODE");
    if (c->nseg < (1ull << 31) && envm0 && !strcmp(envm0, "tile") && c->tables.g == 0 &&
        c->tables.single) {
      rc = build_tables(c->canon, c->tables, envk ? atoi(envk) : 0, 2);
      if (rc) return rc;
    }
  }
  const uint64_t bound = c->nseg * (uint64_t)std::max<uint32_t>(c->tables.maxsyms_seg, 1);
  if (out_cap == 0) out_cap = std::min<uint64_t>(s->n, bound);
  c->out_cap = out_cap;
  GH_HIP(hipSetDevice(c->device));
  GH_HIP(hipMalloc(&c->d_out, std::max<uint64_t>(out_cap, 16) + 64));
  GH_HIP(hipMemset(c->d_misc, 0, 128));
  c->epoch = 0;
  c->ntiles = 0;
  c->grid = 0;
  if (c->nseg > 0) {
    const Tables& tb = c->tables;
    const size_t lut_bytes = tb.g > 0    ? tb.lut2.size() * sizeof(uint2)
                             : tb.single ? tb.lut1.size() * sizeof(uint32_t)
                                         : tb.lut.size() * sizeof(uint2);
    c->lut_bytes = lut_bytes;
    const void* lut_src = tb.g > 0    ? (const void*)tb.lut2.data()
                          : tb.single ? (const void*)tb.lut1.data()
                                      : (const void*)tb.lut.data();
    GH_HIP(hipMalloc(&c->d_lut, std::max<size_t>(lut_bytes, 16)));
    GH_HIP(hipMemset(c->d_lut, 0, std::max<size_t>(lut_bytes, 16)));
    GH_HIP(hipMemcpy(c->d_lut, lut_src, lut_bytes, hipMemcpyHostToDevice));
    GH_HIP(hipMalloc(&c->d_fb, sizeof(c->tables.fb)));
    GH_HIP(hipMemcpy(c->d_fb, c->tables.fb, sizeof(c->tables.fb), hipMemcpyHostToDevice));
    // Segments per thread (ILP): as many as keep the tile's staging <= 32 KiB.
    const char* envu = getenv("GH_U");
    int uv = envu ? atoi(envu) : 0;
    if (uv != 1 && uv != 2 && uv != 4) {
      const uint32_t per = TB * c->tables.maxsyms_seg;  // (multi-symbol paths)
      uv = c->tables.single ? 2 : (4 * per <= 16384) ? 4 : (2 * per <= 16384) ? 2 : 1;
    }
    if (c->tables.g > 0 && uv > 2) uv = 2;
    // Mode: the fused persistent kernel for the grouped single-symbol path, split
    // kernels (count / write) for the others (measured faster on MI355X for each);
    // GH_MODE=fused|split overrides.
    const char* envm = getenv("GH_MODE");
    // Mode: the tile kernel for the grouped single-symbol path (and for any path with
    // GH_MODE=tile); split kernels otherwise (measured faster for the multi-symbol
    // paths, whose tile staging allows one workgroup per CU).  GH_MODE=fused|split
    // override.
    c->tile = c->nseg < (1ull << 31) && (envm ? !strcmp(envm, "tile") : c->tables.g > 0);
    c->split = !c->tile && (envm ? !strcmp(envm, "split") : c->tables.g == 0);
    if (c->tile) {
      const bool grouped = c->tables.g > 0;
      c->tile_path = grouped ? TP_GROUPED : c->tables.needs_fb ? TP_MULTI_FB : TP_MULTI;
      const int TB = grouped ? TB_GRP : TB_MUL, U = grouped ? U_GRP : U_MUL;
      c->tb = TB;
      c->super = (uint32_t)U;
      c->ntiles = (uint32_t)ceil_div(c->nseg, (uint64_t)U * TB);
      c->stage_bytes =
          (uint32_t)((STAGE_PAD + (uint64_t)U * TB * c->tables.maxsyms_seg + 48 + 127) & ~127ull);
      auto lds_of = [&](size_t lut) {
        return grouped ? tile_lds_bytes<TB_GRP, U_GRP>(lut, c->stage_bytes)
                       : tile_lds_bytes<TB_MUL, U_MUL>(lut, c->stage_bytes) + FB_BYTES;
      };
      int per_cu = 0;
      if (grouped) {
        // compact LUT {len | sym << 24}, replicated 2^lgr times in LDS: the largest
        // replication that keeps the best occupancy
        const uint32_t K = c->tables.K;
        c->tile_g = std::min<uint32_t>(4, 32 / std::max<uint32_t>(c->canon.maxlen, 1));
        std::vector<uint32_t> lt(1u << K);
        for (uint32_t i = 0; i < (1u << K); ++i) lt[i] = c->tables.lut2[i].x | c->tables.lut2[i].y;
        GH_HIP(hipMalloc(&c->d_lut_t, 4ull << K));
        GH_HIP(hipMemcpy(c->d_lut_t, lt.data(), 4ull << K, hipMemcpyHostToDevice));
        const char* envr = getenv("GH_LGR");
        int lg = envr ? std::clamp(atoi(envr), 0, 14 - (int)K) : std::min(5, 14 - (int)K);
        int best = 0, best_lg = 0;
        for (int l2 = lg; l2 >= 0; --l2) {
          int pc = 0;
          GH_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&pc, tile_kernel_for(c->tile_path, c->tile_g),
                                                              TB, lds_of(4ull << (K + l2))));
          if (pc > best) { best = pc; best_lg = l2; }
          if (envr) break;
        }
        c->lgr = (uint32_t)best_lg;
        per_cu = best;
        c->lut_bytes = 4ull << (K + best_lg);
      } else {
        // multi-symbol u64 LUT {syms, meta}, one copy; a narrower table if the
        // staging leaves too little LDS (tried on a copy: the split kernels keep
        // the loaded tables if the tile kernel does not fit at all)
        Tables tt = c->tables;
        while (tt.K > 6 && lds_of(8ull << tt.K) > 160 * 1024) {
          rc = build_tables(c->canon, tt, (int)tt.K - 1, 2);
          if (rc) return rc;
        }
        const size_t lb = 8ull << tt.K;
        const int path = tt.needs_fb ? TP_MULTI_FB : TP_MULTI;
        GH_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, tile_kernel_for(path, 0), TB, lds_of(lb)));
        if (per_cu >= 1) {
          c->tables = tt;
          c->tile_path = path;
          GH_HIP(hipMalloc(&c->d_lut_t, lb));
          GH_HIP(hipMemcpy(c->d_lut_t, c->tables.lut.data(), lb, hipMemcpyHostToDevice));
          GH_HIP(hipMemcpy(c->d_fb, c->tables.fb, sizeof(c->tables.fb), hipMemcpyHostToDevice));
        }
        c->lgr = 0;
        c->lut_bytes = lb;
      }
      c->lds = lds_of(c->lut_bytes);
      if (per_cu >= 1) {
        // a round's aggregates are read by its leader, LPL per lane: grid <= LPL * TB
        const uint64_t gmax = (uint64_t)TB * (TB >= 512 ? 1 : 1024 / TB);
        if (const char* ep = getenv("GH_TILE_PERCU")) per_cu = std::clamp(atoi(ep), 1, per_cu);  // diagnostics
        c->grid = (uint32_t)std::min<uint64_t>({(uint64_t)c->ntiles, (uint64_t)per_cu * c->num_cu, gmax});
      } else {  // e.g. 1-2 bit codes: the staging does not fit; use the split kernels
        c->tile = false;
        (void)hipFree(c->d_lut_t);
        c->d_lut_t = nullptr;
        c->split = true;
      }
    }
    // Lean multi-symbol split kernels: multi-symbol codes that are complete and fit
    // 12 bits (GH_MODE=split / fused / tile keep the older kernels).
    {
      const bool eligible = c->nseg < (1ull << 31);  // any code: long and incomplete ones use the fallback
      const bool force_ms = envm && !strcmp(envm, "msplit"), force_ws = envm && !strcmp(envm, "wsplit");
      const bool want = envm ? (force_ms || force_ws) : c->tables.g == 0;
      if (eligible && want) {
        // default: the wave-independent kernels (measured faster than msplit on cfg2/3/5)
        rc = force_ms ? ms_setup(c) : ws_setup(c, s->g ? (double)s->n / (double)s->g : 16.0);
        if (rc) return rc;
      } else if (force_ms || force_ws) {
        c->split = true;  // not eligible: the older split kernels
      }
    }
    if (c->split && !c->ms && !c->ws) {
      // split mode: tiles of U*256 segments, U = 2 (single-symbol) or 1/2 (multi)
      if (c->tables.single || c->tables.g > 0) uv = 2;
      else if (!(envu && atoi(envu) == 2)) uv = (2u * TB_S * c->tables.maxsyms_seg <= 16384) ? 2 : 1;
      c->tb = TB_S;
      c->super = (uint32_t)uv;
      c->stage_bytes = (uint32_t)(((uint64_t)uv * TB_S * c->tables.maxsyms_seg + 112 + 15) & ~15ull);
      c->lds_count = lut_bytes + FB_BYTES;
      c->lds = lut_bytes + FB_BYTES + c->stage_bytes;
      c->ntiles = (uint32_t)ceil_div(c->nseg, (uint64_t)uv * TB_S);
      const SplitKernels k = split_for(c->tables.single, c->tables.needs_fb, uv, c->tables.g);
      int pc_c = 0, pc_w = 0;
      GH_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&pc_c, k.count, TB_S, c->lds_count));
      GH_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&pc_w, k.write, TB_S, c->lds));
      if (pc_c < 1 || pc_w < 1) return fail(GH_E_HIP, "split decode kernels do not fit on a CU");
      // both kernels walk the same contiguous tile ranges, one per workgroup
      // The count kernel may run more workgroups: its ranges nest k to a write range
      // (range boundaries floor(b*n/grid) coincide for grid_c = k*grid_w).
      const char* envg = getenv("GH_GRID_PER_CU");
      const int per_cu = envg ? std::max(1, atoi(envg)) : pc_w;
      c->grid = (uint32_t)std::min<uint64_t>(c->ntiles, (uint64_t)per_cu * c->num_cu);
      const uint32_t kk = std::max(1, pc_c / std::max(1, per_cu));
      c->count_per = 1;
      for (uint32_t k2 = kk; k2 >= 1; --k2)
        if ((uint64_t)k2 * c->grid <= c->ntiles) { c->count_per = k2; break; }
      GH_HIP(hipMalloc(&c->d_seg_cnt, c->nseg + 16));
      GH_HIP(hipMalloc(&c->d_tile_cnt, 4ull * c->ntiles + 16));
      GH_HIP(hipMalloc(&c->d_wg_tot, 8ull * c->grid * c->count_per + 16));
    }
    if (!c->tile && !c->ms && !c->ws) c->tb = c->split ? TB_S : c->tables.g > 0 ? TB_G : TB;
    for (; !c->split && !c->tile && !c->ms && !c->ws; uv >>= 1) {  // fall back to a narrower ILP width if the kernel does not fit
      c->super = (uint32_t)uv;
      c->stage_bytes = (uint32_t)(((uint64_t)uv * c->tb * c->tables.maxsyms_seg + 64 + 15) & ~15ull);
      c->lds = lut_bytes + FB_BYTES + 2 * c->stage_bytes + SCRATCH_BYTES;
      int per_cu = 0;
      GH_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(
          &per_cu, kernel_for(c->tables.single, c->tables.needs_fb, uv, c->tables.g), c->tb, c->lds));
      if (per_cu >= 1) {
        const uint64_t grid = (uint64_t)per_cu * c->num_cu;
        c->ntiles = (uint32_t)ceil_div(c->nseg, (uint64_t)uv * c->tb);
        c->grid = (uint32_t)std::min<uint64_t>(c->ntiles, grid);
        break;
      }
      if (uv == 1) break;
    }
    if (c->grid == 0) return fail(GH_E_HIP, "decode kernel does not fit on a CU");
    if (c->tile) GH_HIP(hipMalloc(&c->d_tile_junk, 16ull * c->grid * c->tb));
#ifdef GH_STAMPS
    GH_HIP(hipMalloc(&c->d_stamps, 16ull * 8 * c->grid));
    GH_HIP(hipMemset(c->d_stamps, 0, 16ull * 8 * c->grid));
#endif
  }
  // look-back granules; tile mode adds the within-round prefixes and the round offsets
  c->gran_words = std::max<uint64_t>(c->ntiles, 1);
  if (c->tile)
    c->gran_words = 2ull * c->ntiles + ceil_div(c->ntiles, std::max<uint32_t>(c->grid, 1)) + 2;
  GH_HIP(hipMalloc(&c->d_gran, 8ull * c->gran_words));
  GH_HIP(hipMemset(c->d_gran, 0, 8ull * c->gran_words));
  // start bit of local segment 0, and the gap nibble base for the rest
  c->first_start = 0;
  if (b > 0 && s->gap_words) {  // (gh_ctx_load_device reads it from device memory)
    const uint64_t nib = b - 1;
    uint32_t wv;
    std::memcpy(&wv, (const uint8_t*)s->gap_words + 4 * (nib >> 3), 4);
    c->first_start = (wv >> (4 * (nib & 7))) & 15u;
  }
  return GH_OK;
}

extern "C" int gh_ctx_load(gh_ctx* c, const gh_stream* s, uint64_t b, uint64_t e,
                           uint64_t out_cap) {
  int rc = load_common(c, s, b, e, out_cap);
  if (rc) return rc;
  if (c->nseg == 0) {
    c->loaded = true;
    return GH_OK;
  }
  // payload words [4b, 4e+1) (clipped at W) + zero padding
  const uint64_t w0 = 4 * b;
  const uint64_t want = 4 * c->nseg + 1;
  const uint64_t have = (w0 < s->w) ? std::min<uint64_t>(want, s->w - w0) : 0;
  const uint64_t alloc_words = 4 * c->nseg + 16;
  GH_HIP(hipMalloc(&c->d_payload, 4 * alloc_words));
  GH_HIP(hipMemset(c->d_payload, 0, 4 * alloc_words));
  if (have)
    GH_HIP(hipMemcpy(c->d_payload, (const uint8_t*)s->payload + 4 * w0, 4 * have,
                     hipMemcpyHostToDevice));
  // gap nibbles: starts of local segments 1..nseg-1 and ends of all: global [b-1, e)
  const uint64_t gw0 = b >> 3;
  const uint64_t gw1 = (e >= 1) ? ((e - 1) >> 3) + 1 : gw0 + 1;
  const uint64_t gwords = std::max<uint64_t>(gw1, gw0 + 1) - gw0;
  const uint64_t total_gw = ceil_div(s->g, GH_GAPS_PER_WORD);
  const uint64_t gcopy = (gw0 < total_gw) ? std::min<uint64_t>(gwords, total_gw - gw0) : 0;
  GH_HIP(hipMalloc(&c->d_gaps, 4 * (gwords + 4)));
  GH_HIP(hipMemset(c->d_gaps, 0, 4 * (gwords + 4)));
  if (gcopy)
    GH_HIP(hipMemcpy(c->d_gaps, (const uint8_t*)s->gap_words + 4 * gw0, 4 * gcopy,
                     hipMemcpyHostToDevice));
  c->gap_nib0 = (uint32_t)(b - 8 * gw0);
  c->ms_last_end = 0;
  if ((c->ms || c->ws) && e == s->g) {
    uint32_t w5[5] = {};
    for (uint64_t i = 0; i < 5; ++i)
      if (4 * (e - 1) + i < s->w) std::memcpy(&w5[i], (const uint8_t*)s->payload + 4 * (4 * (e - 1) + i), 4);
    c->ms_last_end = last_segment_end(c->canon, w5, c->nseg == 1 ? c->first_start : seg_start_host(s, e - 1));
  }
  c->loaded = true;
  return GH_OK;
}

extern "C" int gh_ctx_load_device(gh_ctx* c, const gh_stream* s, uint64_t b, uint64_t e,
                                  const uint32_t* d_payload, uint64_t d_words,
                                  const uint32_t* d_gap_words, uint64_t out_cap) {
  if (!d_payload || !d_gap_words) return fail(GH_E_ARG, "null device buffer");
  int rc = load_common(c, s, b, e, out_cap);
  if (rc) return rc;
  if (c->nseg == 0) {
    c->loaded = true;
    return GH_OK;
  }
  const uint64_t want = 4 * c->nseg + 1;
  const uint64_t have = std::min<uint64_t>(want, d_words);
  const uint64_t alloc_words = 4 * c->nseg + 16;
  GH_HIP(hipMalloc(&c->d_payload, 4 * alloc_words));
  GH_HIP(hipMemset(c->d_payload, 0, 4 * alloc_words));
  if (have)
    GH_HIP(hipMemcpy(c->d_payload, d_payload, 4 * have, hipMemcpyDeviceToDevice));
  const uint64_t gw0 = b >> 3;
  const uint64_t gw1 = (e >= 1) ? ((e - 1) >> 3) + 1 : gw0 + 1;
  const uint64_t gwords = std::max<uint64_t>(gw1, gw0 + 1) - gw0;
  const uint64_t total_gw = ceil_div(s->g, GH_GAPS_PER_WORD);
  const uint64_t gcopy = (gw0 < total_gw) ? std::min<uint64_t>(gwords, total_gw - gw0) : 0;
  GH_HIP(hipMalloc(&c->d_gaps, 4 * (gwords + 4)));
  GH_HIP(hipMemset(c->d_gaps, 0, 4 * (gwords + 4)));
  if (gcopy)
    GH_HIP(hipMemcpy(c->d_gaps, d_gap_words + gw0, 4 * gcopy, hipMemcpyDeviceToDevice));
  c->gap_nib0 = (uint32_t)(b - 8 * gw0);
  // first_start must come from device memory here
  c->first_start = 0;
  if (b > 0) {
    const uint64_t nib = b - 1;
    uint32_t wv = 0;
    GH_HIP(hipMemcpy(&wv, d_gap_words + (nib >> 3), 4, hipMemcpyDeviceToHost));
    c->first_start = (wv >> (4 * (nib & 7))) & 15u;
  }
  c->ms_last_end = 0;
  if ((c->ms || c->ws) && e == s->g) {
    uint32_t w5[5] = {};
    const uint64_t lw0 = 4 * (c->nseg - 1);  // local word of the last segment
    const uint64_t nw = std::min<uint64_t>(5, have > lw0 ? have - lw0 : 0);
    if (nw) GH_HIP(hipMemcpy(w5, c->d_payload + lw0, 4 * nw, hipMemcpyDeviceToHost));
    uint32_t st = c->first_start;
    if (c->nseg > 1) {
      const uint64_t nib = e - 2;
      uint32_t wv = 0;
      GH_HIP(hipMemcpy(&wv, d_gap_words + (nib >> 3), 4, hipMemcpyDeviceToHost));
      st = (wv >> (4 * (nib & 7))) & 15u;
    }
    c->ms_last_end = last_segment_end(c->canon, w5, st);
  }
  c->loaded = true;
  return GH_OK;
}

// Persistent kernels whose workgroups wait on each other (tile, fused) assume that the
// whole grid is resident.  Two of them running at once on one device (several shard
// contexts on one GPU, each on its own stream) can each hold half the CUs and wait
// forever for the rest (their bounded spins then report GH_ST_TIMEOUT).  So launches
// of such kernels on one device are chained: each waits for the previous one's
// completion event, whatever stream either was launched on.
struct DevChain {
  std::mutex mu;
  hipEvent_t last = nullptr;
  bool has = false;
};
static DevChain& dev_chain(int device) {
  static std::mutex mu;
  static std::map<int, DevChain*> m;
  std::lock_guard<std::mutex> g(mu);
  DevChain*& d = m[device];
  if (!d) d = new DevChain();  // one per device, for the life of the process
  return *d;
}

extern "C" int gh_ctx_decode(gh_ctx* c, void* hip_stream, int timed) {
  if (!c) return fail(GH_E_ARG, "null ctx");
  if (!c->loaded) return fail(GH_E_STATE, "gh_ctx_decode before gh_ctx_load");
  hipStream_t st = hip_stream ? (hipStream_t)hip_stream : c->stream;
  GH_HIP(hipSetDevice(c->device));
  if (c->nseg == 0) {
    GH_HIP(hipMemsetAsync(c->d_misc + 2, 0, 8, st));
    GH_HIP(hipEventRecord(c->done, st));
    c->done_rec = true;
    return GH_OK;
  }
  if (++c->epoch >= EPOCH_MAX) {  // granule epochs wrap: start clean
    GH_HIP(hipMemsetAsync(c->d_gran, 0, 8ull * c->gran_words, st));
    c->epoch = 1;
  }
  DecodeParams p{};
  p.payload = c->d_payload;
  p.gaps = c->d_gaps;
  p.lut = (const uint4*)c->d_lut;
  p.fb = c->d_fb;
  p.out = c->d_out;
  p.granules = c->d_gran;
  p.ticket = c->d_misc;
  p.status = c->d_misc + 1;
  p.total = (unsigned long long*)(c->d_misc + 2);
  p.out_cap = c->out_cap;
  p.nseg = c->nseg;
  p.gap_nib0 = c->gap_nib0;
  p.first_start = c->first_start;
  p.nsuper = c->ntiles;
  p.kbits = c->tables.K;
  p.epoch = c->epoch;
  p.lut_bytes = (uint32_t)c->lut_bytes;
  p.stage_bytes = c->stage_bytes;
  p.fb_lo = c->tables.fb_lo;
  p.fb_hi = c->tables.fb_hi;
  p.stamps = c->d_stamps;
  {
    const char* ab = getenv("GH_ABLATE");
    p.ablate = ab ? (unsigned)atoi(ab) : 0u;
    const char* sc = getenv("GH_SCHED");
    p.sched = (sc && !strcmp(sc, "dynamic")) ? 0u : 1u;
  }
  // Persistent kernels (tile, wave tile, fused) are chained per device: wait for the
  // previous one before the start event, so a decode's time excludes its queueing
  // behind other contexts' decodes.
  const bool chained = c->tile || (!c->ws && !c->ms && !c->split);
  DevChain& dc = dev_chain(c->device);
  std::unique_lock<std::mutex> chain_lock(dc.mu, std::defer_lock);
  if (chained) {
    chain_lock.lock();
    if (!dc.last) GH_HIP(hipEventCreateWithFlags(&dc.last, hipEventDisableTiming));
    if (dc.has) GH_HIP(hipStreamWaitEvent(st, dc.last, 0));
  }
  std::pair<hipEvent_t, hipEvent_t> ev{nullptr, nullptr};
  if (timed) {
    if (!c->pool.empty()) {
      ev = c->pool.back();
      c->pool.pop_back();
    } else {
      GH_HIP(hipEventCreate(&ev.first));
      GH_HIP(hipEventCreate(&ev.second));
    }
    GH_HIP(hipEventRecord(ev.first, st));
  }
  p.seg_cnt = c->d_seg_cnt;
  p.tile_cnt = c->d_tile_cnt;
  p.tile_off = c->d_tile_off;
  p.wg_tot = c->d_wg_tot;
  if (c->ws) {
    WsParams m{};
    m.payload = c->d_payload;
    m.gaps = c->d_gaps;
    m.seg_cnt = c->d_seg_cnt;
    m.rng_tot = c->d_rng_tot;
    m.rng_off = c->d_rng_off;
    m.out = c->d_out;
    m.junk = c->d_ws_junk;
    m.status = c->d_misc + 1;
    m.total = (unsigned long long*)(c->d_misc + 2);
    m.out_cap = c->out_cap;
    m.nseg = (uint32_t)c->nseg;
    m.nsb = c->ws_nblocks;
    m.nranges = c->ws_nranges;
    m.chk_pay = 4 * c->nseg + 16;
    m.chk_gap = c->nseg / 8 + 4;  // (at least; the allocation holds gwords + 4)
    m.chk_out = std::max<uint64_t>(c->out_cap, 16) + 64;
    m.gap_nib0 = c->gap_nib0;
    m.first_start = c->first_start;
    m.kbits = c->ms_k;
    m.lut_bytes = (uint32_t)c->lut_bytes;
    m.stage_bytes = c->stage_bytes;
    m.last_end = c->ms_last_end;
    m.fb = c->d_fb;
    m.fb_lo = std::max<uint32_t>(c->canon.minlen, 1);
    m.fb_hi = std::max<uint32_t>(c->canon.maxlen, m.fb_lo);
    static thread_local WsParams wc, ww;
    static thread_local void* ac[1];
    static thread_local void* aw[1];
    wc = m;
    wc.lut = (const uint2*)c->d_ws_lut_c;
    wc.kbits = c->ws_kc;
    wc.lut_bytes = (uint32_t)(4u << c->ws_kc);
    ww = m;
    ww.lut = c->d_ms_lut_w;
    ac[0] = &wc;
    aw[0] = &ww;
    const WsKernels wk = ws_kernels(c->ws_kc, c->ms_k, c->ws_ns, c->ws_fb);
    GH_HIP(hipLaunchKernel(wk.count, dim3(c->ws_grid_c), dim3(WS_TBC), ac, c->lds_count, st));
    GH_HIP(hipLaunchKernel((const void*)gh_ws_scan_kernel, dim3(1), dim3(WS_SCAN_TB), ac, 0, st));
    GH_HIP(hipLaunchKernel(wk.write, dim3(c->grid), dim3(WS_TB), aw, c->lds, st));
  } else if (c->ms) {
    MsParams m{};
    m.payload = c->d_payload;
    m.gaps = c->d_gaps;
    m.seg_cnt = c->d_seg_cnt;
    m.wg_tot = c->d_wg_tot;
    m.out = c->d_out;
    m.status = c->d_misc + 1;
    m.total = (unsigned long long*)(c->d_misc + 2);
    m.out_cap = c->out_cap;
    m.nseg = (uint32_t)c->nseg;
    m.ntiles = c->ntiles;
    m.gap_nib0 = c->gap_nib0;
    m.first_start = c->first_start;
    m.kbits = c->ms_k;
    m.lut_bytes = (uint32_t)c->lut_bytes;
    m.stage_bytes = c->stage_bytes;
    m.count_per = c->count_per;
    m.last_end = c->ms_last_end;
    m.ablate = p.ablate;
    static thread_local MsParams mc, mw;
    static thread_local void* ac[1];
    static thread_local void* aw[1];
    mc = m;
    mc.lut = c->d_ms_lut_c;
    mw = m;
    mw.lut = c->d_ms_lut_w;
    ac[0] = &mc;
    aw[0] = &mw;
    const MsKernels mk = ms_kernels(c->ms_k, c->ms_wu);
    GH_HIP(hipLaunchKernel(mk.count, dim3(c->grid * c->count_per), dim3(TB_MS), ac, c->lds_count, st));
    GH_HIP(hipLaunchKernel(mk.write, dim3(c->grid), dim3(mk.tbw), aw, c->lds, st));
  } else if (c->tile) {
    TileParams t{};
    t.payload = c->d_payload;
    t.gaps = c->d_gaps;
    t.lut = c->d_lut_t;
    t.fb = c->d_fb;
    t.fb_lo = c->tables.fb_lo;
    t.fb_hi = c->tables.fb_hi;
    t.out = c->d_out;
    t.granules = c->d_gran;
    t.plocal = c->d_gran + c->ntiles;
    t.rprefix = c->d_gran + 2ull * c->ntiles;
    t.status = c->d_misc + 1;
    t.total = (unsigned long long*)(c->d_misc + 2);
    t.stats = (unsigned long long*)(c->d_misc + 4);
    t.out_cap = c->out_cap;
    t.nseg = c->nseg;
    t.gap_nib0 = c->gap_nib0;
    t.first_start = c->first_start;
    t.ntiles = c->ntiles;
    t.kbits = c->tables.K;
    t.lgr = c->lgr;
    t.epoch = c->epoch;
    t.lut_bytes = (uint32_t)c->lut_bytes;
    t.stage_bytes = c->stage_bytes;
    t.stamps = c->d_stamps;
    t.ablate = p.ablate;
    t.junk = c->d_tile_junk;
    static thread_local void* ta[1];
    static thread_local TileParams tp;
    tp = t;
    ta[0] = &tp;
    GH_HIP(hipLaunchKernel(tile_kernel_for(c->tile_path, c->tile_g), dim3(c->grid), dim3(c->tb), ta, c->lds,
                           st));
    GH_HIP(hipEventRecord(dc.last, st));
    dc.has = true;
  } else if (c->split) {
    const SplitKernels k = split_for(c->tables.single, c->tables.needs_fb, (int)c->super,
                                     c->tables.g);
    p.count_per = c->count_per;
    GH_HIP(hipLaunchKernel(k.count, dim3(c->grid * c->count_per), dim3(TB_S), args_of(p),
                           c->lds_count, st));
    GH_HIP(hipLaunchKernel(k.write, dim3(c->grid), dim3(TB_S), args_of(p), c->lds, st));
  } else {
    GH_HIP(hipLaunchKernel(kernel_for(c->tables.single, c->tables.needs_fb, (int)c->super,
                                      c->tables.g),
                           dim3(c->grid), dim3(c->tb), args_of(p), c->lds, st));
    GH_HIP(hipEventRecord(dc.last, st));
    dc.has = true;
  }
  GH_HIP(hipGetLastError());
  if (timed) {
    GH_HIP(hipEventRecord(ev.second, st));
    c->pending.push_back(ev);
  }
  GH_HIP(hipEventRecord(c->done, st));
  c->done_rec = true;
  return GH_OK;
}

// Waits for the context's last decode, whatever stream it was launched on.
static int wait_decode(gh_ctx* c) {
  GH_HIP(hipStreamSynchronize(c->stream));
  if (c->done_rec) GH_HIP(hipEventSynchronize(c->done));
  return GH_OK;
}

extern "C" int gh_ctx_report(gh_ctx* c, void* hip_stream, gh_report* rep) {
  if (!c) return fail(GH_E_ARG, "null ctx");
  hipStream_t st = hip_stream ? (hipStream_t)hip_stream : c->stream;
  GH_HIP(hipSetDevice(c->device));
  GH_HIP(hipStreamSynchronize(st));
  if (int rc = wait_decode(c)) return rc;
  for (auto& e : c->pending) {
    float ms = 0;
    GH_HIP(hipEventElapsedTime(&ms, e.first, e.second));
    c->acc_ms += ms;
    c->nlaunch++;
    c->pool.push_back(e);
  }
  c->pending.clear();
  unsigned int misc[6] = {};
  GH_HIP(hipMemcpy(misc, c->d_misc, sizeof(misc), hipMemcpyDeviceToHost));
  if (rep) {
    std::memset(rep, 0, sizeof(*rep));
    uint64_t tot;
    std::memcpy(&tot, misc + 2, 8);
    rep->symbols = tot;
    rep->out_bytes = std::min<uint64_t>(tot, c->out_cap);
    rep->status = misc[1];
    rep->lut_bits = c->tables.K;
    rep->grid = c->grid;
    rep->tiles = c->ntiles;
    rep->mode = c->tile ? GH_MODE_TILE : (c->split || c->ms || c->ws) ? GH_MODE_SPLIT : GH_MODE_FUSED;
    std::memcpy(&rep->slow_lookbacks, misc + 4, 8);
    rep->path = c->ws ? GH_PATH_MULTI_WAVE : c->ms ? GH_PATH_MULTI_LEAN
                : c->tables.g > 0 ? GH_PATH_GROUPED : c->tables.single ? GH_PATH_SINGLE : GH_PATH_MULTI;
    if (c->ms || c->ws) rep->lut_bits = c->ms_k;
    rep->launches = c->nlaunch;
    rep->kernel_ms = c->nlaunch ? (float)(c->acc_ms / c->nlaunch) : 0.f;
  }
  return GH_OK;
}

extern "C" int gh_ctx_reset_timing(gh_ctx* c) {
  if (!c) return fail(GH_E_ARG, "null ctx");
  c->acc_ms = 0;
  c->nlaunch = 0;
  return GH_OK;
}

extern "C" int gh_ctx_download(gh_ctx* c, uint64_t off, uint8_t* dst, uint64_t nbytes) {
  if (!c || (nbytes && !dst)) return fail(GH_E_ARG, "null argument");
  if (off + nbytes > c->out_cap) return fail(GH_E_ARG, "download beyond the output capacity");
  if (!nbytes) return GH_OK;
  GH_HIP(hipSetDevice(c->device));
  if (int rc = wait_decode(c)) return rc;
  GH_HIP(hipMemcpy(dst, c->d_out + off, nbytes, hipMemcpyDeviceToHost));
  return GH_OK;
}

extern "C" int gh_ctx_output(gh_ctx* c, void** d_out, uint64_t* cap) {
  if (!c || !d_out) return fail(GH_E_ARG, "null argument");
  *d_out = c->d_out;
  if (cap) *cap = c->out_cap;
  return GH_OK;
}

extern "C" int gh_ctx_copy_output(gh_ctx* c, uint64_t off, void* dst, uint64_t nbytes,
                                  void* hip_stream) {
  if (!c || (nbytes && !dst)) return fail(GH_E_ARG, "null argument");
  if (off + nbytes > c->out_cap) return fail(GH_E_ARG, "copy beyond the output capacity");
  if (!nbytes) return GH_OK;
  hipStream_t st = hip_stream ? (hipStream_t)hip_stream : c->stream;
  GH_HIP(hipSetDevice(c->device));
  if (c->done_rec) GH_HIP(hipStreamWaitEvent(st, c->done, 0));  // after the last decode
  GH_HIP(hipMemcpyAsync(dst, c->d_out + off, nbytes, hipMemcpyDefault, st));
  return GH_OK;
}

extern "C" int gh_decode(const gh_stream* s, uint8_t* out, uint64_t out_len, const gh_opts* o,
                         gh_report* rep) {
  if (!s || (s->n && !out)) return fail(GH_E_ARG, "null argument");
  if (out_len < s->n) return fail(GH_E_SMALL, "output buffer smaller than N");
  int rc = gh_stream_validate(s);
  if (rc) return rc;
  const int ng = (o && o->ngpus > 1) ? o->ngpus : 1;
  const int reps = (o && o->reps > 1) ? o->reps : 1;
  std::vector<uint64_t> bounds(ng + 1);
  gh_plan_shards(s->g, (uint32_t)ng, bounds.data());
  std::vector<gh_ctx*> ctx(ng, nullptr);
  auto cleanup = [&]() {
    for (auto* c : ctx) gh_ctx_destroy(c);
  };
  for (int k = 0; k < ng; ++k) {
    const int dev = (o && o->devices) ? o->devices[k] : (ng > 1 ? k : 0);
    rc = gh_ctx_create(dev, &ctx[k]);
    if (!rc) rc = gh_ctx_load(ctx[k], s, bounds[k], bounds[k + 1], ng > 1 ? 0 : s->n);
    if (rc) {
      cleanup();
      return rc;
    }
  }
  for (int r = 0; r < reps; ++r)
    for (int k = 0; k < ng; ++k)
      if ((rc = gh_ctx_decode(ctx[k], nullptr, 1))) {
        cleanup();
        return rc;
      }
  std::vector<gh_report> reps_k(ng);
  uint64_t offset = 0;
  uint32_t status = 0;
  float worst_ms = 0;
  for (int k = 0; k < ng; ++k) {
    if ((rc = gh_ctx_report(ctx[k], nullptr, &reps_k[k]))) {
      cleanup();
      return rc;
    }
    status |= reps_k[k].status;
    worst_ms = std::max(worst_ms, reps_k[k].kernel_ms);
    const uint64_t want = (offset < s->n) ? std::min<uint64_t>(reps_k[k].symbols, s->n - offset) : 0;
    if (k + 1 < ng && reps_k[k].symbols > reps_k[k].out_bytes) {
      cleanup();
      return fail(GH_E_CORRUPT, "shard produced more symbols than its output capacity");
    }
    if (want && (rc = gh_ctx_download(ctx[k], 0, out + offset, want))) {
      cleanup();
      return rc;
    }
    offset += reps_k[k].symbols;
  }
  cleanup();
  if (rep) {
    *rep = reps_k[0];
    rep->symbols = offset;
    rep->out_bytes = std::min<uint64_t>(offset, s->n);
    rep->status = status;
    rep->kernel_ms = worst_ms;
  }
  if (status & GH_ST_TIMEOUT) return fail(GH_E_HIP, "look-back timed out");
  if (offset < s->n) return fail(GH_E_CORRUPT, "stream decoded to fewer than N symbols");
  if (status & GH_ST_BADCODE) return fail(GH_E_CORRUPT, "invalid code in stream");
  return GH_OK;
}

#ifdef GH_STAMPS
// Diagnostic build only: the tile kernel's look-back counters (cumulative).
extern "C" int gh_debug_stats(gh_ctx* c, unsigned long long* host) {
  if (!c || !host) return fail(GH_E_ARG, "null argument");
  GH_HIP(hipDeviceSynchronize());
  GH_HIP(hipMemcpy(host, c->d_misc + 4, 32, hipMemcpyDeviceToHost));
  return GH_OK;
}

// Diagnostic build only: per-block phase cycle totals of the last launch.
extern "C" int gh_debug_stamps(gh_ctx* c, unsigned long long* host, uint32_t max_blocks) {
  if (!c || !host || !c->d_stamps) return fail(GH_E_ARG, "no stamps");
  const uint32_t nb = std::min(max_blocks, c->grid);
  GH_HIP(hipDeviceSynchronize());
  GH_HIP(hipMemcpy(host, c->d_stamps, 16ull * 8 * nb, hipMemcpyDeviceToHost));
  return (int)nb;
}
#endif
