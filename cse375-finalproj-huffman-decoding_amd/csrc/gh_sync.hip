// gh_sync.hip — self-synchronising decode of gap-less Huffman streams (SURVEY.md
// §8(f) rank 3) for gfx950.
//
// Replaces CUHD's four-phase decoder (gpuhd/src/cuhd_gpu_decoder.cu:145-523,
// CUHDGPUDecoder::decode, decl gpuhd/include/cuhd_gpu_decoder.h:24-32).  CUHD has
// each thread decode fixed-size subsequences of a raw u32 stream
// (llhuffman_encoder.cc:200-238, MSB-first within each unit) from an arbitrary bit,
// and relies on Huffman codes resynchronising: phase 1/2 (:145-318) repeat the decode
// of later subsequences until a thread lands on the start its neighbour recorded, with
// a host loop over phase 2 (:439-475); phase 3 scans the symbol counts (:481-495);
// phase 4 decodes again and writes (:320-413).
//
// Here the raw stream is turned into the gap-array stream the hot path already
// decodes.  The "entry" of 128-bit segment j, the first codeword start at or after bit
// 128j, is exactly the gap nibble gap[j-1] of Huffman_coding_Gap_arrays
// (encoder.cu:307-312: end bit of the codeword crossing the boundary, minus the
// boundary; 0..15 since codes are at most 16 bits).  So synthesising the gap array
// on the device makes the raw stream decodable by the tuned count/write or tile
// kernels unchanged; the count pass, scan and write pass are the hot path's own.
//
//  gh_sync_kernel      lane L owns the SYNC_M consecutive segments [L*M, L*M + M): one
//                      continuous walk from the raw bit 128 (L*M - h) (h warm-up
//                      segments, possibly mid-codeword; bit 0 for lane 0), recording the
//                      entry at every boundary it passes inside its block as gap
//                      nibbles (two gap words per lane), and its own view of the entry
//                      at its block's first boundary L*M as check[L].  Codes
//                      resynchronise within a few codewords, so after h segments the
//                      walk is on the true path on ordinary data.  One walk per lane
//                      from start to end: no lock-step rounds, no lanes idling while
//                      neighbours' walks merge.
//  gh_sync_fix_kernel  verification: check[L] == entry of boundary L*M as lane L-1
//                      recorded it (its last nibble) for every L proves every nibble
//                      (induction: lane 0 starts at the true bit 0; if lane L-1's
//                      entries are true and lane L's walk stands on the same entry at
//                      L*M, its walk is the true one from there).  A mismatch is
//                      repaired by re-walking block L from the true entry until the
//                      new entry equals the stored one (the walks merged: the rest is
//                      true) or the block ends, then on into the next blocks while
//                      they disagree (the role of CUHD's phase 2).  The host repeats
//                      the pass until it finds no mismatch (CUHD's host loop,
//                      :439-475); each pass makes at least the lowest mismatching block
//                      true; on ordinary data the first pass finds none.
//
// One 14-bit LUT (32 KB) in LDS serves both walks: {step (the advance below, or the first
// length when no codeword fits), length of the first codeword (0 if > 14 bits), bits of
// the complete codewords that fit in the 14 bits (the advance)}.  Walks take the
// multi-codeword step except where a step could skip the start that has to be
// recorded; codes of 14-16 bits use the canonical thresholds.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "gh_internal.hpp"

namespace gh {
namespace {

#ifndef GH_SYNC_SK
#define GH_SYNC_SK 14  // (round 6, with the unclamped loads: cfg4 0.80 ms at 13, 0.70 at 14)
#endif
#ifndef GH_SYNC_TB
#define GH_SYNC_TB 256
#endif
constexpr int SK = GH_SYNC_SK;       // LUT prefix bits (round 2's kernel: 12: cfg4 2.28 ms, 13: 2.08, 14: 3.10 - occupancy)
constexpr int SYNC_TB = GH_SYNC_TB;  // threads per workgroup
#ifndef GH_SYNC_M
#define GH_SYNC_M 32  // (round 5: 32 with the code's own halo; 16 with 6 warm-up segments: cfg4 1.05 ms)
#endif
constexpr uint32_t SYNC_M = GH_SYNC_M;  // segments per lane (a multiple of 8: whole gap words)
static_assert(SYNC_M % 8 == 0, "a lane writes whole gap words");
#ifndef GH_SYNC_FAST
#define GH_SYNC_FAST 1  // walk kernel: unclamped 16-byte segment loads for waves inside the stream
#endif
#ifndef GH_SYNC_RING
#define GH_SYNC_RING 0  // walk kernel: prefetch ring of three register sets (loop unrolled by three)
#endif
#ifndef GH_SYNC_WPE
#define GH_SYNC_WPE 1  // walk kernel occupancy hint (waves per SIMD; 1: the compiler's choice)
#endif
#ifndef GH_SYNC_RUNR
#define GH_SYNC_RUNR 0  // in-wave repair: the block re-walk's segment loop unrolled (0: a loop)
#endif
// warm-up segments per lane: from the stream's resynchronisation distances (sync_halo_for;
// GH_SYNC_HALO overrides)

#define GH_HIPS(expr)                                                             \
  do {                                                                            \
    hipError_t e_ = (expr);                                                       \
    if (e_ != hipSuccess)                                                         \
      return fail(GH_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));   \
  } while (0)

struct SyncParams {
  const uint32_t* words;  // raw stream, 16-byte aligned
  uint64_t w;             // words
  uint64_t g;             // segments = ceil(w / 4)
  const uint16_t* lut;    // 1 << SK entries {step, first len << 5, multi-codeword advance << 10}
  uint32_t t13, t14, t15, t16;  // canonical left-aligned limits of lengths 13..16
  uint32_t* gaps;         // ceil(g / 8) gap words
  uint8_t* check;         // ceil(g / SYNC_M): lane L's entry at boundary L * SYNC_M
  unsigned int* counter;  // [0] fix-pass mismatches, [1] repairs reaching a wave's end, [2] in-wave mismatches
  uint32_t halo;          // warm-up segments per lane
};

__device__ __forceinline__ uint64_t ceil_div_d(uint64_t a, uint64_t b) { return (a + b - 1) / b; }

__device__ __forceinline__ uint32_t ld_word(const uint32_t* w, uint64_t nw, uint64_t i) {
  return i < nw ? w[i] : 0u;
}

// Length of a codeword longer than SK bits (or 1 for a pattern outside the code
// space, which only a walk that started mid-codeword meets).
__device__ __forceinline__ uint32_t long_len(uint32_t p16, const SyncParams& p) {
  return p16 < p.t13 ? 13u : p16 < p.t14 ? 14u : p16 < p.t15 ? 15u : p16 < p.t16 ? 16u : 1u;
}

// Walk the codeword starts inside one 32-bit word: `off` (0..31, or beyond when the
// previous word's last codeword reached into this one) is the next start relative to
// the top of `hi`; returns the first start at or after the next word, relative to it.
// BOUND: the returned start is recorded, so no multi-codeword step may pass it.
// LONG: the code has codewords longer than SK bits (else every LUT entry has a length:
// patterns outside the code space are stored as length 1, so no branch per step).
template <bool BOUND, bool LONG>
__device__ __forceinline__ uint32_t walk_word(uint32_t hi, uint32_t lo, uint32_t off,
                                              const uint16_t* lut, const SyncParams& p) {
  const uint64_t win = ((uint64_t)hi << 32) | lo;
  while (off < 32) {
    const uint32_t p16 = (uint32_t)((win << off) >> 48);
    const uint32_t e = lut[p16 >> (16 - SK)];
    if constexpr (!BOUND) {
      uint32_t st = e & 31u;  // precomputed: advance if any, else the first length
      if (LONG && st == 0) st = long_len(p16, p);
      off += st;
    } else {
      const uint32_t adv = e >> 10;
      uint32_t len = (e >> 5) & 31u;
      if (LONG && len == 0) len = long_len(p16, p);
      off += (adv != 0 && off + SK <= 32) ? adv : len;
    }
  }
  return off - 32;
}

__device__ __forceinline__ void stage_lut(uint16_t* lds, const uint16_t* g) {
  for (int i = threadIdx.x; i < (1 << SK) / 2; i += SYNC_TB)
    reinterpret_cast<uint32_t*>(lds)[i] = reinterpret_cast<const uint32_t*>(g)[i];
  __syncthreads();
}

// Walk segment j (words 4j..4j+4) from entry offset `off`; returns the entry offset at
// boundary 128(j+1).
// Words 4j..4j+4 of segment j (zero past the stream).
__device__ __forceinline__ void load_segment(uint64_t j, uint32_t (&w)[5], const SyncParams& p) {
  const uint64_t w0 = 4 * j;
  if (w0 + 5 <= p.w) {
    const uint4 x = *reinterpret_cast<const uint4*>(p.words + w0);
    w[0] = x.x; w[1] = x.y; w[2] = x.z; w[3] = x.w;
    w[4] = p.words[w0 + 4];
  } else {
#pragma unroll
    for (int i = 0; i < 5; ++i) w[i] = ld_word(p.words, p.w, w0 + i);
  }
}

// Walk a segment's words from entry offset `off`; returns the entry offset at the
// segment's end boundary.
template <bool LONG>
__device__ __forceinline__ uint32_t walk_words(const uint32_t (&w)[5], uint32_t off, const uint16_t* lut,
                                               const SyncParams& p) {
  off = walk_word<false, LONG>(w[0], w[1], off, lut, p);
  off = walk_word<false, LONG>(w[1], w[2], off, lut, p);
  off = walk_word<false, LONG>(w[2], w[3], off, lut, p);
  return walk_word<true, LONG>(w[3], w[4], off, lut, p);
}

// Walk segment j from entry offset `off`; returns the entry offset at boundary
// 128(j+1).
template <bool LONG>
__device__ __forceinline__ uint32_t walk_segment(uint64_t j, uint32_t off, const uint16_t* lut,
                                                 const SyncParams& p) {
  uint32_t w[5];
  load_segment(j, w, p);
  return walk_words<LONG>(w, off, lut, p);
}

// Words 4j..4j+4 of segment j, by value (kept in registers): seg_raw loads them with
// the index clamped into the stream (no branch: the compiler then keeps the prefetch
// in its own registers and waits for it only where it is used), seg_mask zeroes the
// words past the stream once they have arrived.
struct SegWords {
  uint32_t w0, w1, w2, w3, w4;
};
__device__ __forceinline__ SegWords seg_raw(uint64_t j, const SyncParams& p) {
  const uint64_t b = 4 * j, last = p.w - 1;  // (w >= 1 whenever a segment exists)
  return {p.words[min(b, last)], p.words[min(b + 1, last)], p.words[min(b + 2, last)],
          p.words[min(b + 3, last)], p.words[min(b + 4, last)]};
}
__device__ __forceinline__ SegWords seg_mask(const SegWords& r, uint64_t j, const SyncParams& p) {
  const uint64_t b = 4 * j;
  return {b < p.w ? r.w0 : 0u, b + 1 < p.w ? r.w1 : 0u, b + 2 < p.w ? r.w2 : 0u, b + 3 < p.w ? r.w3 : 0u,
          b + 4 < p.w ? r.w4 : 0u};
}

// One word of the wave's walks in step: q (< 32, else the lane is past this word) is
// the next codeword start relative to the top of hi; loops until every lane is past
// the word and returns q - 32, the start relative to the next word.  hi:lo is fixed
// for the word, so a step is a 64-bit shift, one LDS read and an add.  BOUND (the
// segment's last word): the start at or after the boundary is recorded, so no
// multi-codeword step may pass it.
template <bool BOUND, bool LONG>
__device__ __forceinline__ uint32_t walk_word_ls(uint32_t hi, uint32_t lo, uint32_t q, const uint16_t* lut,
                                                 const SyncParams& p) {
  const uint64_t win = ((uint64_t)hi << 32) | lo;
  while (__any(q < 32u)) {  // branch-free body: lanes past the word look up harmlessly
    const uint32_t p16 = (uint32_t)((win << (q & 31u)) >> 48);
    const uint32_t e = lut[p16 >> (16 - SK)];
    uint32_t st;
    if constexpr (!BOUND) {
      st = e & 31u;  // precomputed: the advance if any, else the first length
      if (LONG && st == 0) st = long_len(p16, p);
    } else {
      const uint32_t adv = e >> 10;
      uint32_t len = (e >> 5) & 31u;
      if (LONG && len == 0) len = long_len(p16, p);
      st = (adv != 0 && q + adv <= 32u) ? adv : len;
    }
    q += q < 32u ? st : 0u;
  }
  return q - 32u;
}

// The lanes of a wave walk their blocks in step: iteration i walks segment
// sb - h + i of every lane (a lane whose walk would start before segment 0 idles until
// it reaches segment 0, then starts at the true bit 0), so the next segments' loads are
// issued by the whole wave at once, two segments ahead, and waited for with a counted
// vmcnt.  (Lanes crossing boundaries at different steps, each loading its next
// segment then, made every step wait for the latest lane's loads: 1.7 ms on cfg4.)
template <bool LONG>
__global__ __launch_bounds__(SYNC_TB) __attribute__((amdgpu_waves_per_eu(GH_SYNC_WPE))) void gh_sync_kernel(SyncParams p) {
  __shared__ uint16_t lut[1 << SK];
  stage_lut(lut, p.lut);  // (the only barrier: waves past the stream may leave after it)
  const uint64_t L = (uint64_t)blockIdx.x * SYNC_TB + threadIdx.x;
  const uint64_t sb = L * SYNC_M;  // the lane's block [sb, se)
  if (__builtin_amdgcn_readfirstlane((uint32_t)(sb - (uint64_t)(threadIdx.x % 64) * SYNC_M >= p.g))) return;
  const uint64_t se = sb < p.g ? (sb + SYNC_M < p.g ? sb + SYNC_M : p.g) : sb;  // (empty past the stream)
  const int64_t s0 = (int64_t)sb - (int64_t)p.halo;  // segment of iteration 0
  auto seg_at = [&](int64_t s) { return (uint64_t)(s < 0 ? 0 : s); };
  uint32_t pos = 0;  // segment-relative bit of the next codeword start
  uint32_t g0 = 0, g1 = 0, g2 = 0, g3 = 0, chk = 0;
  const int nit = (int)p.halo + (int)SYNC_M;
  // iteration i: walk segment s = s0 + i (its words loaded two iterations earlier)
  auto body = [&](int i, const SegWords& raw) {
    const int64_t s = s0 + i;
    const SegWords w = seg_mask(raw, seg_at(s), p);
    const bool act = s >= 0 && s < (int64_t)se;
    // an idle lane walks nothing: q starts past every word (and stays there)
    uint32_t q = act ? pos : 512u;
    q = walk_word_ls<false, LONG>(w.w0, w.w1, q, lut, p);
    q = walk_word_ls<false, LONG>(w.w1, w.w2, q, lut, p);
    q = walk_word_ls<false, LONG>(w.w2, w.w3, q, lut, p);
    q = walk_word_ls<true, LONG>(w.w3, w.w4, q, lut, p);
    if (act) {  // boundary 128 (s + 1) passed: its entry
      uint32_t e = q;
      // no codeword crosses the end of the stream: the entry at 128g is 0, as the
      // encoder leaves the last gap (encoder.cu:414 memset, nothing crosses 128G)
      if ((uint64_t)s + 1 >= p.g) e = 0;
      if ((uint64_t)s >= sb) {
        const uint32_t k = (uint32_t)((uint64_t)s - sb);
        if (k < 8) g0 |= e << (4 * k);
        else if (k < 16) g1 |= e << (4 * (k - 8));
        else if (k < 24) g2 |= e << (4 * (k - 16));
        else g3 |= e << (4 * (k - 24));
      } else if ((uint64_t)s + 1 == sb) {
        chk = e;
      }
      pos = e;
    }
  };
  // Waves whose loads all lie inside the stream (all but the last few) take them as one
  // 16-byte load and one dword per segment from a per-lane pointer, with no clamps and
  // no masks (the general path: five clamped dword loads, masked on use).
  const int nitr = (nit + 2) / 3 * 3;
  const bool fast = GH_SYNC_FAST && __all(s0 >= 0 && (uint64_t)(s0 + nitr + 1) * 4 + 5 <= p.w);
  if (fast) {
    const uint32_t* lw = p.words + 4 * (uint64_t)(s0 < 0 ? 0 : s0);
    auto ld = [&](int i) {
      const uint4 x = *reinterpret_cast<const uint4*>(lw + 4 * i);
      return SegWords{x.x, x.y, x.z, x.w, lw[4 * i + 4]};
    };
    auto body_fast = [&](int i, const SegWords& w) {
      const int64_t s = s0 + i;
      const bool act = s < (int64_t)se;
      uint32_t q = act ? pos : 512u;
      q = walk_word_ls<false, LONG>(w.w0, w.w1, q, lut, p);
      q = walk_word_ls<false, LONG>(w.w1, w.w2, q, lut, p);
      q = walk_word_ls<false, LONG>(w.w2, w.w3, q, lut, p);
      q = walk_word_ls<true, LONG>(w.w3, w.w4, q, lut, p);
      if (act) {
        uint32_t e = q;
        if ((uint64_t)s + 1 >= p.g) e = 0;
        if ((uint64_t)s >= sb) {
          const uint32_t k = (uint32_t)((uint64_t)s - sb);  // (the same for every lane of the wave)
          if (k < 8) g0 |= e << (4 * k);
          else if (k < 16) g1 |= e << (4 * (k - 8));
          else if (k < 24) g2 |= e << (4 * (k - 16));
          else g3 |= e << (4 * (k - 24));
        } else if ((uint64_t)s + 1 == sb) {
          chk = e;
        }
        pos = e;
      }
    };
    SegWords X = ld(0), Y = ld(1), Z;
    for (int i = 0; i < nit; i += 3) {
      Z = ld(i + 2);
      body_fast(i, X);
      X = ld(i + 3);
      body_fast(i + 1, Y);
      Y = ld(i + 4);
      body_fast(i + 2, Z);
    }
  } else if (GH_SYNC_RING) {
    // three register sets in rotation, the loop unrolled by three: segment s + 2 is
    // loaded into the set that segment s - 1 used, and no set is copied, so a load is
    // waited for two iterations after it was issued (with the copies of a two-deep
    // prefetch, the compiler waited for it at the end of the iteration that issued it).
    // Iterations past nit walk nothing (idle lanes).
    SegWords X = seg_raw(seg_at(s0), p), Y = seg_raw(seg_at(s0 + 1), p), Z;
    for (int i = 0; i < nit; i += 3) {
      Z = seg_raw(seg_at(s0 + i + 2), p);
      body(i, X);
      X = seg_raw(seg_at(s0 + i + 3), p);
      body(i + 1, Y);
      Y = seg_raw(seg_at(s0 + i + 4), p);
      body(i + 2, Z);
    }
  } else {
    SegWords w = seg_raw(seg_at(s0), p), n1 = seg_raw(seg_at(s0 + 1), p);
    for (int i = 0; i < nit; ++i) {
      const SegWords n2 = seg_raw(seg_at(s0 + i + 2), p);  // two segments ahead
      body(i, w);
      w = n1;
      n1 = n2;
    }
  }
  // Verify and repair inside the wave: lane l's view of the entry at its block's start
  // (chk) against lane l-1's last nibble.  A mismatching block is re-walked from that
  // entry, in step with the wave's other mismatching blocks, until a recorded entry
  // equals the new one (the walks merged) or the block ends; rounds repeat while a
  // block's left neighbour changed.  Lane 0's block is verified by gh_sync_fix_kernel
  // against the previous wave's last block.
  auto nib_get = [&](int k) {
    const uint32_t gw_ = k < 8 ? g0 : k < 16 ? g1 : k < 24 ? g2 : g3;
    return (gw_ >> (4 * (k & 7))) & 15u;
  };
  auto nib_set = [&](int k, uint32_t v) {  // (by value: a reference select put g0..g3 in scratch)
    const uint32_t sh = 4u * (uint32_t)(k & 7), m = ~(15u << sh), x = v << sh;
    const int q = k >> 3;
    g0 = q == 0 ? (g0 & m) | x : g0;
    g1 = q == 1 ? (g1 & m) | x : g1;
    g2 = q == 2 ? (g2 & m) | x : g2;
    g3 = q == 3 ? (g3 & m) | x : g3;
  };
  const uint32_t lane = threadIdx.x % 64;
  for (int round = 0; round < 64; ++round) {
    const uint32_t left = (uint32_t)__shfl_up((int)nib_get(SYNC_M - 1), 1);
    const bool bad = lane > 0 && sb < p.g && chk != left;
    if (!__any(bad)) break;
    {  // (reported as mismatches) one atomic per wave: per lane, the same-address atomics
       // of a stream with many mismatching blocks serialised (cfg4 at halo 0: 18.8 ms)
      const unsigned long long bm = __ballot(bad);
      if (lane == 0) atomicAdd(p.counter + 2, (unsigned)__popcll(bm));
    }
    bool run = bad;
    uint32_t e = left;
#pragma unroll(GH_SYNC_RUNR ? GH_SYNC_M : 1)
    for (int k = 0; k < (int)SYNC_M; ++k) {
      if (!__any(run)) break;
      const uint64_t s = sb + (uint64_t)k;
      run = run && s < se;
      const SegWords ws = seg_mask(seg_raw(run ? s : 0, p), run ? s : 0, p);
      uint32_t q = run ? e : 512u;
      q = walk_word_ls<false, LONG>(ws.w0, ws.w1, q, lut, p);
      q = walk_word_ls<false, LONG>(ws.w1, ws.w2, q, lut, p);
      q = walk_word_ls<false, LONG>(ws.w2, ws.w3, q, lut, p);
      q = walk_word_ls<true, LONG>(ws.w3, ws.w4, q, lut, p);
      if (run) {
        const uint32_t e2 = s + 1 >= p.g ? 0u : q;
        if (nib_get(k) == e2) {
          run = false;  // merged: the rest of the block follows
        } else {
          nib_set(k, e2);
          e = e2;
        }
      }
    }
    if (bad) chk = left;
  }
  if (sb < p.g) {
    const uint64_t gw = sb / 8, ngw = ceil_div_d(p.g, 8);
    static_assert(SYNC_M == 16 || SYNC_M == 24 || SYNC_M == 32, "two to four gap words per lane");
    p.gaps[gw] = g0;
    if (gw + 1 < ngw) p.gaps[gw + 1] = g1;
    if (SYNC_M > 16 && gw + 2 < ngw) p.gaps[gw + 2] = g2;
    if (SYNC_M > 24 && gw + 3 < ngw) p.gaps[gw + 3] = g3;
    p.check[L] = (uint8_t)chk;
  }
}

__device__ __forceinline__ uint32_t nib_at(const uint32_t* gaps, uint64_t i) {
  return (__atomic_load_n(gaps + (i >> 3), __ATOMIC_RELAXED) >> (4 * (i & 7))) & 15u;
}

__device__ __forceinline__ void nib_store(uint32_t* gaps, uint64_t i, uint32_t v) {
  uint32_t* wp = gaps + (i >> 3);
  const uint32_t sh = 4 * (uint32_t)(i & 7);
  uint32_t old = __atomic_load_n(wp, __ATOMIC_RELAXED);
  for (;;) {
    const uint32_t nw = (old & ~(15u << sh)) | (v << sh);
    const uint32_t seen = atomicCAS(wp, old, nw);
    if (seen == old) break;
    old = seen;
  }
}

// Block L re-walked from the entry a at boundary sb = L * SYNC_M (lane L-1's): every
// entry that disagrees with the stored nibble is replaced, until a stored entry equals
// the new one (lane L's walk merged with this one there: the rest of the block follows)
// or the block ends; then check[L] := a.  Only lane L and this repair write block L's
// nibbles, so once a is true (block L-1 verified) the block is true, and a later change
// of a (block L-1 repaired after this) makes the next pass flag block L again.
template <bool LONG>
__device__ void repair_block(uint64_t L, uint32_t a, const uint16_t* lut, const SyncParams& p) {
  const uint64_t sb = L * SYNC_M, se = sb + SYNC_M < p.g ? sb + SYNC_M : p.g;
  uint32_t entry = a;
  for (uint64_t j = sb; j < se; ++j) {
    uint32_t e = walk_segment<LONG>(j, entry, lut, p);
    if (j + 1 >= p.g) e = 0;
    if (nib_at(p.gaps, j) == e) break;  // merged
    nib_store(p.gaps, j, e);
    entry = e;
  }
  p.check[L] = (uint8_t)a;
}

// The walk kernel verified every block against its left neighbour inside its wave; a
// thread here takes one wave's first block (its left neighbour is the previous wave's
// last) and, while a repaired block's successor no longer agrees, the wave's next
// blocks.  counter[0]: mismatching blocks; counter[1]: repairs that reached a wave's
// last block (whose successor, another wave's first block, must then be verified
// again: the host repeats the pass while it is non-zero).
template <bool LONG>
__global__ __launch_bounds__(SYNC_TB) void gh_sync_fix_kernel(SyncParams p) {
  __shared__ uint16_t lut[1 << SK];
  stage_lut(lut, p.lut);
  const uint64_t nb = ceil_div_d(p.g, SYNC_M), nwv = ceil_div_d(nb, 64);
  const uint64_t stride = (uint64_t)gridDim.x * SYNC_TB;
  uint32_t nrep = 0, nlast = 0;  // (summed per wave: one atomic each)
  for (uint64_t k = (uint64_t)blockIdx.x * SYNC_TB + threadIdx.x + 1; k < nwv; k += stride) {
    const uint64_t L1 = min(64 * k + 64, nb);
    for (uint64_t L = 64 * k; L < L1; ++L) {
      const uint32_t a = nib_at(p.gaps, L * SYNC_M - 1);  // block L-1's entry at boundary L * M
      if (p.check[L] == a) break;
      ++nrep;
      repair_block<LONG>(L, a, lut, p);
      if (L + 1 == L1) ++nlast;
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    nrep += (uint32_t)__shfl_xor((int)nrep, o);
    nlast += (uint32_t)__shfl_xor((int)nlast, o);
  }
  if (threadIdx.x % 64 == 0) {
    if (nrep) atomicAdd(p.counter, nrep);
    if (nlast) atomicAdd(p.counter + 1, nlast);
  }
}

// Host tables: LUT {first length, multi-codeword advance} over 12-bit prefixes and the
// left-aligned canonical limits T[l] = sum_{m <= l} count[m] << (16 - m).
struct SyncTables {
  std::vector<uint16_t> lut;
  uint32_t T[GH_MAX_CODE_LEN + 1] = {};
};

void build_sync_tables(const Canon& c, SyncTables& st) {
  uint32_t acc = 0;
  for (uint32_t l = 1; l <= GH_MAX_CODE_LEN; ++l) {
    acc += c.count[l] << (16 - l);
    st.T[l] = acc;
  }
  auto len_of = [&](uint32_t p16) -> uint32_t {
    for (uint32_t l = 1; l <= GH_MAX_CODE_LEN; ++l)
      if (p16 < st.T[l]) return l;
    return 0;  // outside the code space
  };
  st.lut.assign(1u << SK, 0);
  for (uint32_t v = 0; v < (1u << SK); ++v) {
    uint32_t s = 0, first = 0;
    while (s < (uint32_t)SK) {
      const uint32_t x = (v << s) & ((1u << SK) - 1);
      const uint32_t l = len_of(x << (16 - SK));
      if (l == 0 || l > SK - s) break;  // longer than the bits left (or invalid)
      if (s == 0) first = l;
      s += l;
    }
    // a prefix outside the code space (only met by walks that started mid-codeword)
    // steps one bit, like long_len's fallback
    if (first == 0 && (v << (16 - SK)) >= st.T[GH_MAX_CODE_LEN]) first = 1;
    // {step = advance, or the first length when no codeword fits (0: a long code),
    //  first length << 5, advance << 10}
    const uint32_t step = s ? s : first;
    st.lut[v] = (uint16_t)(step | (first << 5) | (s << 10));
  }
}

// Warm-up segments for a stream.  Walks from arbitrary bits resynchronise after a
// distance that depends on the code and the data (simulated on the oracle: r = 0.9
// codes 10 bits on average, r = 0.1 117, r = 0.5 326 with a p99 of 2390), and a block
// whose walk has not merged with the true path by its first boundary costs its whole
// wave a lock-step re-walk.  So the halo h minimises (M + h) + 64 * P(d > 128 h) * M / 2
// (the walk, plus the chance that one of a wave's 64 blocks is re-walked, about half a
// block), with P from the stream itself: its first words (a true codeword start at bit
// 0) decoded from the start, then walked from 4096 pseudo-random bit offsets with the
// kernels' rule (length 1 outside the code space) until a walk stands on a true start.
// A short stream (few waves per SIMD: one wave's repair rounds then extend the whole
// kernel) takes at least the p99.9 distance, rounded up to segments (cfg2: p99.9 ~4300
// bits; h = 32 0.144 ms, 35 0.154-0.156, 20 0.168, 43-48 0.169-0.178).  In [2, 48].  `sample`: the stream's first words (zero padded by 2).
uint32_t sync_halo_for(const SyncTables& st, const std::vector<uint32_t>& sample, uint64_t nbits, bool short_stream) {
  if (nbits < 4096) return 2;
  auto p16_at = [&](uint64_t pos) {
    const uint64_t w = ((uint64_t)sample[pos >> 5] << 32) | sample[(pos >> 5) + 1];
    return (uint32_t)((w << (pos & 31)) >> 48);
  };
  auto len_at = [&](uint64_t pos) {
    const uint32_t p16 = p16_at(pos);
    const uint32_t l = (st.lut[p16 >> (16 - SK)] >> 5) & 31u;
    if (l) return l;
    for (uint32_t m = SK + 1; m <= GH_MAX_CODE_LEN; ++m)
      if (p16 < st.T[m]) return m;
    return 1u;  // outside the code space
  };
  const uint64_t nb = nbits - 32;
  std::vector<uint8_t> start(nb + 1, 0);
  for (uint64_t pos = 0; pos < nb; pos += len_at(pos)) start[pos] = 1;
  uint64_t x = 0x9E3779B97F4A7C15ull;
  constexpr uint32_t NW = 4096, HMAX = 48;
  std::vector<uint32_t> over(HMAX + 2, 0);  // walks not merged after h segments
  std::vector<uint64_t> ds(NW);
  for (uint32_t k = 0; k < NW; ++k) {
    x ^= x << 13;
    x ^= x >> 7;
    x ^= x << 17;
    const uint64_t o = x % (nb / 2);
    uint64_t pos = o;
    while (pos < nb && !start[pos]) pos += len_at(pos);
    const uint64_t d = pos < nb ? pos - o : ~0ull;
    ds[k] = d;
    for (uint32_t h = 0; h <= HMAX; ++h)
      if (d > 128ull * h) ++over[h];
  }
  uint32_t best = 2;
  double best_c = 1e30;
  for (uint32_t h = 2; h <= HMAX; ++h) {
    const double c = (double)(SYNC_M + h) + 64.0 * ((double)over[h] / NW) * SYNC_M / 2;
    if (c < best_c) {
      best_c = c;
      best = h;
    }
  }
  if (short_stream) {
    std::sort(ds.begin(), ds.end());
    const uint64_t p999 = ds[NW - 1 - NW / 1000];  // ~0 when 5 or more walks never merged
    best = std::max<uint32_t>(best, p999 >= 128ull * HMAX ? HMAX : (uint32_t)((p999 + 127) / 128));
  }
  return best;
}

struct DevBuf {
  void* p = nullptr;
  ~DevBuf() { (void)hipFree(p); }
};

int grid_for(const void* k, uint64_t items) {
  int dev = 0, ncu = 0, per = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 1;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) ncu = 256;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k, SYNC_TB, 0) != hipSuccess || per < 1) per = 1;
  const uint64_t need = std::max<uint64_t>(1, ceil_div(items, SYNC_TB));
  return (int)std::min<uint64_t>(need, (uint64_t)ncu * per);
}

}  // namespace
}  // namespace gh

using namespace gh;

extern "C" int gh_sync_gaps(int device, const gh_sym* syms, uint32_t nsyms, const uint32_t* d_words,
                            uint64_t w, uint32_t* d_gap_words, void* hip_stream, gh_sync_report* rep) {
  if (rep) std::memset(rep, 0, sizeof(*rep));
  if (!syms || (w && (!d_words || !d_gap_words))) return fail(GH_E_ARG, "null argument");
  if (((uintptr_t)d_words & 15u) != 0) return fail(GH_E_ARG, "d_words must be 16-byte aligned");
  Canon canon;
  int rc = build_canon(syms, nsyms, canon);
  if (rc) return rc;
  if (nsyms == 0 && w) return fail(GH_E_TABLE, "empty code table for a non-empty stream");
  const uint64_t g = ceil_div(w, 4);
  if (rep) rep->g = g;
  if (g == 0) return GH_OK;
  GH_HIPS(hipSetDevice(device));
  hipStream_t st = (hipStream_t)hip_stream;
  SyncTables tabs;
  build_sync_tables(canon, tabs);
  DevBuf lut, check, counter;
  const uint64_t nblk = ceil_div(g, (uint64_t)SYNC_M);  // lanes of the walk kernel
  GH_HIPS(hipMalloc(&lut.p, 2u << SK));
  GH_HIPS(hipMalloc(&check.p, nblk + 16));
  GH_HIPS(hipMalloc(&counter.p, 16));
  GH_HIPS(hipMemcpyAsync(lut.p, tabs.lut.data(), 2u << SK, hipMemcpyHostToDevice, st));
  SyncParams p{};
  p.words = d_words;
  p.w = w;
  p.g = g;
  p.lut = (const uint16_t*)lut.p;
  p.t13 = tabs.T[13];
  p.t14 = tabs.T[14];
  p.t15 = tabs.T[15];
  p.t16 = tabs.T[16];
  p.gaps = d_gap_words;
  p.check = (uint8_t*)check.p;
  p.counter = (unsigned int*)counter.p;
  float host_ms = 0;
  {
    const char* eh = getenv("GH_SYNC_HALO");
    const auto h0 = std::chrono::steady_clock::now();
    if (eh) {
      p.halo = (uint32_t)std::clamp(atoi(eh), 0, 64);
    } else {  // from the stream's first words (at most 64 KiB; before the timed region)
      const uint64_t ns = std::min<uint64_t>(w, 16384);
      std::vector<uint32_t> sample(ns + 2, 0);
      GH_HIPS(hipMemcpyAsync(sample.data(), d_words, 4 * ns, hipMemcpyDeviceToHost, st));
      GH_HIPS(hipStreamSynchronize(st));
      int ncu = 256;
      if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) ncu = 256;
      const bool short_stream = ceil_div(nblk, (uint64_t)64) < 8ull * 4 * (uint64_t)ncu;  // < 8 waves per SIMD
      p.halo = sync_halo_for(tabs, sample, 32 * ns, short_stream);
      host_ms = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - h0).count();
    }
    if (getenv("GH_SYNC_VERBOSE")) fprintf(stderr, "gh_sync: %u segments per lane, halo %u\n", SYNC_M, p.halo);
  }
  hipEvent_t e0, e1;
  GH_HIPS(hipEventCreate(&e0));
  GH_HIPS(hipEventCreate(&e1));
  struct EvGuard {
    hipEvent_t a, b;
    ~EvGuard() { (void)hipEventDestroy(a); (void)hipEventDestroy(b); }
  } evg{e0, e1};
  const bool lng = canon.maxlen > (uint32_t)SK;
  const void* ks = lng ? (const void*)gh_sync_kernel<true> : (const void*)gh_sync_kernel<false>;
  const void* kf = lng ? (const void*)gh_sync_fix_kernel<true> : (const void*)gh_sync_fix_kernel<false>;
  const int gs = (int)ceil_div(nblk, (uint64_t)SYNC_TB);  // one lane per block (not persistent)
  const int gf = grid_for(kf, ceil_div(nblk, (uint64_t)64));  // one thread per wave of the walk
  void* kargs[] = {&p};
  GH_HIPS(hipMemsetAsync(counter.p, 0, 12, st));
  GH_HIPS(hipEventRecord(e0, st));
  GH_HIPS(hipLaunchKernel(ks, dim3(gs), dim3(SYNC_TB), kargs, 0, st));
  GH_HIPS(hipGetLastError());
  uint64_t mism = 0;
  uint32_t passes = 0;
  float ms = 0;
  for (;;) {
    GH_HIPS(hipLaunchKernel(kf, dim3(gf), dim3(SYNC_TB), kargs, 0, st));
    GH_HIPS(hipGetLastError());
    GH_HIPS(hipEventRecord(e1, st));
    unsigned int cnt[3] = {};
    GH_HIPS(hipMemcpyAsync(cnt, counter.p, 12, hipMemcpyDeviceToHost, st));
    GH_HIPS(hipStreamSynchronize(st));
    GH_HIPS(hipEventElapsedTime(&ms, e0, e1));
    ++passes;
    mism += cnt[0] + (passes == 1 ? cnt[2] : 0u);
    if (cnt[1] == 0) break;  // no repair reached a wave's last block: every block verified
    // each pass makes at least the lowest mismatching wave true, so one pass per wave
    // always suffices
    if (passes > nblk / 64 + 2) return fail(GH_E_CORRUPT, "self-synchronisation did not converge");
    GH_HIPS(hipMemsetAsync(counter.p, 0, 8, st));
  }
  if (rep) {
    rep->mismatches = mism;
    rep->passes = passes;
    rep->kernel_ms = ms;
    rep->host_ms = host_ms;
    rep->halo = p.halo;
  }
  return GH_OK;
}

extern "C" int gh_ctx_load_raw(gh_ctx* ctx, const gh_sym* syms, uint32_t nsyms, uint64_t n,
                               const uint32_t* words, uint64_t w, uint64_t out_cap,
                               gh_sync_report* rep) {
  if (!ctx || !syms || (w && !words)) return fail(GH_E_ARG, "null argument");
  int dev = 0;
  int rc = gh_ctx_device(ctx, &dev);
  if (rc) return rc;
  GH_HIPS(hipSetDevice(dev));
  const uint64_t g = ceil_div(w, 4);
  {  // N symbols of at least minlen bits each must fit the 32 w bits
    Canon cn;
    rc = build_canon(syms, nsyms, cn);
    if (rc) return rc;
    if (n && (cn.minlen == 0 || n > (32 * w) / cn.minlen))
      return fail(GH_E_FORMAT, "raw stream holds fewer bits than N symbols need");
  }
  DevBuf dw, dg;
  GH_HIPS(hipMalloc(&dw.p, 4 * (w + 16)));
  GH_HIPS(hipMemset(dw.p, 0, 4 * (w + 16)));
  if (w) GH_HIPS(hipMemcpy(dw.p, words, 4 * w, hipMemcpyHostToDevice));
  GH_HIPS(hipMalloc(&dg.p, 4 * (ceil_div(g, 8) + 4)));
  GH_HIPS(hipMemset(dg.p, 0, 4 * (ceil_div(g, 8) + 4)));
  rc = gh_sync_gaps(dev, syms, nsyms, (const uint32_t*)dw.p, w, (uint32_t*)dg.p, nullptr, rep);
  if (rc) return rc;
  gh_stream s{};
  s.syms = syms;
  s.nsyms = nsyms;
  s.version = 2;
  s.n = n;
  s.w = w;
  s.g = g;
  return gh_ctx_load_device(ctx, &s, 0, g, (const uint32_t*)dw.p, w, (const uint32_t*)dg.p, out_cap);
}

// Device-memory helpers for C/FFI callers that have no HIP binding of their own (e.g.
// ctypes): buffers for gh_sync_gaps / gh_ctx_load_device.
extern "C" int gh_dev_alloc(int device, uint64_t bytes, void** out) {
  if (!out) return fail(GH_E_ARG, "null argument");
  *out = nullptr;
  GH_HIPS(hipSetDevice(device));
  GH_HIPS(hipMalloc(out, std::max<uint64_t>(bytes, 1)));
  return GH_OK;
}

extern "C" int gh_dev_free(void* p) {
  GH_HIPS(hipFree(p));
  return GH_OK;
}

extern "C" int gh_dev_copy(void* dst, const void* src, uint64_t bytes) {
  if (bytes && (!dst || !src)) return fail(GH_E_ARG, "null argument");
  if (bytes) GH_HIPS(hipMemcpy(dst, src, bytes, hipMemcpyDefault));
  return GH_OK;
}
