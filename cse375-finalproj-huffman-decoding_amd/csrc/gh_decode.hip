// gh_decode.hip — MI355X (gfx950) gap-array Huffman decoder: the decode kernels and the
// host context behind the C ABI (include/gaphuff.h).
//
// Replaces the reference hot path gpu_dec_l1_l2 (Huffman_coding_Gap_arrays/decoder/
// src/decoder.cu:454-730) and its launcher decoder_l1_l2 (decoder.cu:732-815).
// Semantics kept from the reference:
//   * segment i (128 bits = 4 payload words) starts at bit 128*i + gap[i-1], the gap
//     being a 4-bit nibble, 8 per u32 (decoder.cu:501-507);
//   * a segment decodes every codeword that starts inside it (decoder.cu:529-569);
//   * outputs are concatenated in segment order by an exclusive scan of the
//     per-segment symbol counts (decoder.cu:571-653).
// Two decode structures, chosen per code on the host:
//   * gh_tile.hip — grouped codes (complete, 4 <= len <= 12, e.g. BASELINE r = 0.1): one
//     persistent kernel, one decode pass, round-leader prefixes;
//   * gh_wsplit.hip — every other code: count, scan and write kernels in which no wave
//     waits for another, four symbols per write lookup, a canonical fallback for
//     codewords longer than the tables and for incomplete codes.
// Every output write is clamped at the shard's output capacity (the reference wrote
// past N, decoder.cu:672-728).  Tables: gh_lut.hpp; device helpers: gh_device.hpp.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "gh_device.hpp"
#include "gh_internal.hpp"
#include "gh_lut.hpp"

namespace gh {

constexpr uint32_t EPOCH_MAX = (1u << 24) - 1;

#include "gh_tile.hip"
#include "gh_wsplit.hip"
#include "gh_mtile.hip"

}  // namespace gh

using namespace gh;

#define GH_HIP(expr)                                                              \
  do {                                                                            \
    hipError_t e_ = (expr);                                                       \
    if (e_ != hipSuccess)                                                         \
      return fail(GH_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));   \
  } while (0)

// Tile kernel shapes: codes of >= 4-bit codewords (at most 32 per segment) run three
// segments per lane with 8 output words each; codes with 3-bit codewords (at most 43
// per segment, e.g. BASELINE's r = 0.5 codes) two segments per lane with 11 words (the
// registers and the staging of a third segment would halve the workgroups per CU).
static uint32_t tile_u_for(uint32_t minlen) { return minlen >= 4 ? (uint32_t)TILE_U : (uint32_t)TILE_U3; }
#ifndef GH_TILE_OW7
#define GH_TILE_OW7 1  // codes of >= 5-bit codewords: 7 output words per segment (<= 26 codewords)
#endif
static const void* tile_kernel_for(uint32_t minlen, uint32_t g) {
  if (minlen >= 5 && GH_TILE_OW7)
    return g >= 4 ? (const void*)gh_tile_kernel<TILE_TB, TILE_U, 4, 7, 5>
         : g == 3 ? (const void*)gh_tile_kernel<TILE_TB, TILE_U, 3, 7, 5>
                  : (const void*)gh_tile_kernel<TILE_TB, TILE_U, 2, 7, 5>;
  if (minlen >= 4)
    return g >= 4 ? (const void*)gh_tile_kernel<TILE_TB, TILE_U, 4, 8, 4>
         : g == 3 ? (const void*)gh_tile_kernel<TILE_TB, TILE_U, 3, 8, 4>
                  : (const void*)gh_tile_kernel<TILE_TB, TILE_U, 2, 8, 4>;
  return g >= 4 ? (const void*)gh_tile_kernel<TILE_TB, TILE_U3, 4, 11, 3>
       : g == 3 ? (const void*)gh_tile_kernel<TILE_TB, TILE_U3, 3, 11, 3>
                : (const void*)gh_tile_kernel<TILE_TB, TILE_U3, 2, 11, 3>;
}

// Two-pass tile kernel by lookups per window shift and 16-byte stores per copy-out.
template <int GL, bool FB>
static const void* mtile_ns(int ns) {
  return ns <= 4 ? (const void*)gh_mtile_kernel<MT_TB, GL, 4, FB>
       : ns <= 6 ? (const void*)gh_mtile_kernel<MT_TB, GL, 6, FB>
       : ns <= 8 ? (const void*)gh_mtile_kernel<MT_TB, GL, 8, FB>
                 : (const void*)gh_mtile_kernel<MT_TB, GL, 5, FB, 2>;  // (10: two copy-out parts of 5 x 64 chunks)
}
// fb: codewords longer than the tables (K = 11..12, GL = 2) through the canonical fallback
static const void* mtile_kernel_for(int gl, int ns, bool fb = false) {
  if (fb) return mtile_ns<2, true>(ns);
  return gl >= 4 ? mtile_ns<4, false>(ns) : gl == 3 ? mtile_ns<3, false>(ns) : mtile_ns<2, false>(ns);
}

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
static WsKernels ws_kernels(uint32_t Kc, uint32_t K, int ns, bool fb) {
  if (fb) return {(const void*)gh_ws_count_kernel<WS_UC, WS_TBC, 2, true>, ws_write_ns<2, true>(ns)};
  const int gc = lookups_per_shift(Kc), g = lookups_per_shift(K);
  const void* cnt = gc >= 4 ? (const void*)gh_ws_count_kernel<WS_UC, WS_TBC, 4>
                    : gc == 3 ? (const void*)gh_ws_count_kernel<WS_UC, WS_TBC, 3>
                              : (const void*)gh_ws_count_kernel<WS_UC, WS_TBC, 2>;
  const void* wr = g >= 4 ? ws_write_ns<4>(ns) : g == 3 ? ws_write_ns<3>(ns) : ws_write_ns<2>(ns);
  return {cnt, wr};
}

struct gh_ctx {
  int device = 0;
  int num_cu = 0;
  hipStream_t stream = nullptr;
  hipEvent_t done = nullptr;  // recorded after every decode, on the stream it ran on
  bool done_rec = false;
  hipEvent_t done_ev = nullptr;    // marks the last decode: `done`, or the timed decode's end event
  bool loaded = false;
  Canon canon;
  // the loaded shard
  uint64_t nseg = 0, seg_begin = 0, seg_end = 0, n_total = 0;
  uint32_t gap_nib0 = 0, first_start = 0;
  uint32_t* d_payload = nullptr;
  uint32_t* d_gaps = nullptr;
  uint8_t* d_out = nullptr;
  uint64_t out_cap = 0;
  unsigned int* d_misc = nullptr;  // [1] status, [2..3] symbol total, [4..11] tile poll counters
  uint32_t grid = 0;               // workgroups of the tile kernel / the write kernel
  uint32_t ntiles = 0;             // tiles (tile kernel) / wave blocks (wave split)
  size_t lds = 0;                  // dynamic LDS of the tile / write kernel
  size_t lut_bytes = 0;            // LDS bytes of its LUT
  uint32_t stage_bytes = 0;        // one staging buffer (tile) / one wave's (write kernel)
  // tile kernel (grouped codes)
  bool tile = false;
  uint32_t tile_k = 0, tile_g = 0, lgr = 0;  // LUT width, codewords per window shift, log2 LUT copies
  uint32_t tile_minl = 4, tile_u = TILE_U;     // kernel shape (tile_kernel_for), segments per lane
  uint32_t idle_block = 0xFFFFFFFFu;           // GH_TILE_IDLE experiments: a block that exits at once
  bool mtile = false;              // the two-pass tile kernel (gh_mtile.hip; c->tile is set too)
  bool mt_fb = false;              // ... with the canonical fallback (codewords longer than its tables)
  uint32_t mt_kc = 0;              // its count table's width
  int mt_gl = 2, mt_ns = 4;        // its lookups per window shift, stores per copy-out
  uint32_t* d_lut_t = nullptr;
  uint4* d_stamps = nullptr;       // GH_TILE_STAMPS builds only
  unsigned long long* d_gran = nullptr;  // granules, within-round prefixes, round starts
  uint64_t gran_words = 0;
  uint32_t epoch = 0;
  // wave split (every other code)
  bool ws = false;
  bool ws_fb = false;              // with the canonical fallback
  uint32_t ws_k = 0, ws_kc = 0;    // write / count LUT widths
  uint32_t ws_lgc = 0;             // log2 count-LUT copies in LDS
  uint32_t ws_nblocks = 0, ws_nranges = 0, ws_grid_c = 0;
  int ws_ns = 4;
  size_t lds_count = 0;            // dynamic LDS of the count kernel
  uint32_t ws_last_end = 0;        // end bit of the stream's last segment when the shard holds it
  uint32_t* d_ws_lut_c = nullptr;  // count LUT {b | end mask << 16}
  uint64_t* d_ws_lut_w = nullptr;  // write LUT {symbols, b | n << 8}
  uint32_t* d_fb = nullptr;        // canonical fallback tables
  uint8_t* d_seg_cnt = nullptr;
  uint4* d_ws_junk = nullptr;
  unsigned long long* d_rng_tot = nullptr;
  unsigned long long* d_rng_off = nullptr;
  // timing
  std::vector<std::pair<hipEvent_t, hipEvent_t>> pending, pool;
  double acc_ms = 0;
  uint32_t nlaunch = 0;
};

static void free_shard(gh_ctx* c) {
  (void)hipSetDevice(c->device);
  for (void* p : {(void*)c->d_payload, (void*)c->d_gaps, (void*)c->d_out, (void*)c->d_gran, (void*)c->d_lut_t,
                  (void*)c->d_stamps, (void*)c->d_ws_lut_c, (void*)c->d_ws_lut_w, (void*)c->d_fb,
                  (void*)c->d_seg_cnt, (void*)c->d_ws_junk, (void*)c->d_rng_tot, (void*)c->d_rng_off})
    (void)hipFree(p);
  c->d_payload = nullptr;
  c->d_gaps = nullptr;
  c->d_out = nullptr;
  c->d_gran = nullptr;
  c->d_lut_t = nullptr;
  c->d_stamps = nullptr;
  c->d_ws_lut_c = nullptr;
  c->d_ws_lut_w = nullptr;
  c->d_fb = nullptr;
  c->d_seg_cnt = nullptr;
  c->d_ws_junk = nullptr;
  c->d_rng_tot = nullptr;
  c->d_rng_off = nullptr;
  c->tile = false;
  c->mtile = false;
  c->mt_fb = false;
  c->ws = false;
  c->loaded = false;
}

// ---- tile kernel setup -----------------------------------------------------------
// LUT width K (>= maxlen), replicated 2^lgr times in LDS: the largest replication that
// keeps the best occupancy.  Returns GH_OK with c->tile false when the kernel does not
// fit a CU (the wave split then takes the code).
static int tile_setup(gh_ctx* c, uint32_t K, double avg_seg_bytes) {
  const Canon& cn = c->canon;
  const uint32_t maxsyms = (128 + cn.minlen - 1) / cn.minlen;  // <= 43 (minlen >= 3)
  c->tile_k = K;
  c->tile_g = std::min<uint32_t>(4, 32 / cn.maxlen);
  c->tile_minl = cn.minlen >= 5 && GH_TILE_OW7 ? 5 : cn.minlen >= 4 ? 4 : 3;
  c->tile_u = tile_u_for(cn.minlen);
  c->ntiles = (uint32_t)ceil_div(c->nseg, (uint64_t)c->tile_u * TILE_TB);
  // Staging is sized for the typical piece, not the worst case (128 / minlen bytes per
  // segment): TILE_SCAP = 20 bytes per segment for grouped codes (r = 0.1: 16.5), the
  // stream's mean + 12 % for minlen-3 codes (r = 0.5: 21.5 -> 25), so that two
  // workgroups fit a CU.  A wave's piece is the sum of 128-192 segments, so it stays near
  // its mean; a larger one stores straight from registers (gh_tile_kernel).  The
  // copy-out's TILE_NS * 64 chunks cover a region.  GH_TILE_SCAP overrides (tests).
  double scapf = 1.12;
  if (const char* e = getenv("GH_TILE_SCAPF")) scapf = std::clamp(atof(e), 0.5, 4.0);
  uint64_t per_seg = std::min<uint64_t>(
      maxsyms, cn.minlen >= 4 ? (uint64_t)TILE_SCAP : (uint64_t)std::ceil(std::max(avg_seg_bytes, 1.0) * scapf + 1));
  if (const char* e = getenv("GH_TILE_SCAP")) per_seg = std::min<uint64_t>(maxsyms, (uint64_t)std::max(1, atoi(e)));
  const uint64_t margin = 4ull * (cn.minlen >= 4 ? 8 : 11) + 4;  // garbage past a piece's end (4 OW + 4, OW <= 8 / 11)
  const uint64_t seg_wave = 64ull * c->tile_u;
  per_seg = std::min<uint64_t>(per_seg, ((uint64_t)TILE_NS * 64 * 16 - 2 * STAGE_PAD - margin) / seg_wave);
  c->stage_bytes = (uint32_t)((STAGE_PAD + seg_wave * per_seg + margin + 15) & ~15ull);
  const std::vector<uint32_t> lt = grouped_lut(cn, K);
  const void* kern = tile_kernel_for(c->tile_minl, c->tile_g);
  const char* envr = getenv("GH_LGR");
  const int lg = envr ? std::clamp(atoi(envr), 0, 14 - (int)K) : std::min(5, 14 - (int)K);
  int best = 0, best_lg = 0;
  for (int l2 = lg; l2 >= 0; --l2) {
    int pc = 0;
    GH_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&pc, kern, TILE_TB, tile_lds_bytes(4ull << (K + l2), c->stage_bytes)));
    if (pc > best) {
      best = pc;
      best_lg = l2;
    }
    if (envr) break;
  }
  // The kernel is compiled for two workgroups per CU (4 waves per SIMD).  The occupancy
  // query can answer one more than the hardware admits at these SGPR counts (MI355X guide,
  // "Occupancy API one block/CU high"); a grid that is not resident at once never finishes
  // (its bounded polls then report GH_ST_TIMEOUT), so never plan more than two.
  best = std::min(best, 2);
  if (best < 1) return GH_OK;
  GH_HIP(hipMalloc(&c->d_lut_t, 4ull << K));
  GH_HIP(hipMemcpy(c->d_lut_t, lt.data(), 4ull << K, hipMemcpyHostToDevice));
  c->lgr = (uint32_t)best_lg;
  c->lut_bytes = 4ull << (K + best_lg);
  c->lds = tile_lds_bytes(c->lut_bytes, c->stage_bytes);
  // workgroup 0 leads the rounds (up to LEAD_A aggregates per thread: D = grid - 1 <=
  // LEAD_A * TILE_TB), the others decode; every workgroup must be resident at once
  // (the grid is sized from the occupancy; decodes on one device are chained, see DevChain)
  c->grid = (uint32_t)std::min<uint64_t>({(uint64_t)c->ntiles + 1, (uint64_t)best * c->num_cu, (uint64_t)LEAD_A * TILE_TB});
  c->idle_block = 0xFFFFFFFFu;
  if (const char* e = getenv("GH_TILE_IDLE"))  // experiment: block grid / 2 (the leader's CU partner) idles
    if (atoi(e) && c->grid == (uint32_t)best * c->num_cu && best == 2) {
      c->idle_block = c->grid / 2;
    }
  if (c->grid < 2) return GH_OK;  // (the wave split then takes the code)
  if (GH_TILE_STAMPS) {
    const size_t nb = 32ull * c->grid * 2 * 128 + 8ull * (3ull * c->ntiles + 64 + 4 * 1024 + 4ull * c->grid);
    GH_HIP(hipMalloc(&c->d_stamps, nb));
    GH_HIP(hipMemset(c->d_stamps, 0, nb));
  }
  c->tile = true;
  return GH_OK;
}

// ---- two-pass tile kernel setup (gh_mtile.hip) -------------------------------------
// Codes for it: complete, 1 <= len <= 16 (at most 128 codewords per segment), not taken
// by the single-pass tile kernel.  One LUT of width K (the wave split's write width; 11
// with a 1-bit codeword) with the codewords' start masks; one staging region per wave, sized for the stream's mean
// bytes per segment + 12 % and at least one chain's worst case (64 x 128 / minlen bytes: a larger
// piece is written and copied out chain by chain).  Returns GH_OK with c->tile false when
// it does not fit a CU.
static uint32_t ws_write_bits(const Canon& cn);
static int mtile_setup(gh_ctx* c, double avg_seg_bytes) {
  const Canon& cn = c->canon;
  // codes with a 1-bit codeword: segments of up to 128 codewords, a chain's worst case
  // 8 KB, so 11-bit tables (24 KB with the count table) leave 16 regions of 8.5 KB
  const bool one = cn.minlen == 1;
  const uint32_t K = one ? std::min<uint32_t>(ws_write_bits(cn), 11) : ws_write_bits(cn);
  // codewords longer than the tables (up to 16 bits) take the canonical fallback, with
  // two lookups per window shift (2 x 12 + 16 > 32 otherwise)
  const bool fb = K < cn.maxlen;
  // (and windows that reach a 16-bit codeword's last bit: K = 12, or 11 in the kernels
  // for codes with a 1-bit codeword, gh_mtile.hip)
  if (fb && (K != (one ? 11u : 12u) || cn.maxlen > 16)) return GH_OK;
  const uint32_t maxsyms = (128 + cn.minlen - 1) / cn.minlen;  // <= 128
  double scapf = 1.12;
  if (const char* e = getenv("GH_TILE_SCAPF")) scapf = std::clamp(atof(e), 0.5, 4.0);
  uint64_t per_seg = std::min<uint64_t>(maxsyms, (uint64_t)std::ceil(std::max(avg_seg_bytes, 1.0) * scapf + 1));
  if (const char* e = getenv("GH_TILE_SCAP")) per_seg = std::min<uint64_t>(maxsyms, (uint64_t)std::max(1, atoi(e)));
  // at most what the LDS (LUT + 16 regions + slots) and the copy-out's 8 x 64 chunks hold
  // count table width: wider than the write table's (more codewords per lookup) where
  // the LDS and a window shift allow it (GL lookups of Kc bits within 31 bits)
  uint32_t Kc = K;
  if (GH_MT_CLUT && !one) {
    const int gl = lookups_per_shift(K);
    Kc = std::min<uint32_t>(13, 31 / gl);
    if (const char* e = getenv("GH_MT_KC")) Kc = (uint32_t)std::clamp(atoi(e), (int)K, (int)std::min(14, 31 / gl));
    Kc = std::max(Kc, K);
  }
  // the count table's copies (log2; GH_MT_CLGR, default 0): Kc + copies <= 14 keeps the
  // count e-window's S >= 16
  uint32_t clgr = 0;
  if (const char* e = getenv("GH_MT_CLGR")) clgr = (uint32_t)std::clamp(atoi(e), 0, 3);
  if (!GH_MT_CLUT || one) clgr = 0;
  clgr = std::min<uint32_t>(clgr, Kc + clgr > 14 ? 14 - Kc : clgr);
  c->mt_kc = Kc;
  const uint64_t lut_b = (GH_MT_CLUT ? (8ull << K) + (4ull << (Kc + clgr)) : 8ull << K)  // write table (+ count table)
                         + (fb ? (uint64_t)FB_BYTES : 0);                         // (+ fallback tables)
  const uint64_t lds_free = 160ull * 1024 - lut_b - mtile_lds_bytes(0, 0);
  // (the copy-out: 8 x 64 chunks, or 2 x 5 x 64 for codes with a 1-bit codeword)
  const uint64_t region_max = std::min<uint64_t>(lds_free / (MT_TB / 64), (one ? 10 : 8) * 1024 + STAGE_PAD) & ~15ull;
  per_seg = std::min<uint64_t>(per_seg, (region_max - STAGE_PAD - 16) / (64ull * MT_U));
  {  // six copy-out stores per lane (the 8-store kernel spills at lag 3) when the mean + 5 % fits
    const uint64_t ps6 = (6144 - 16) / (64ull * MT_U);
    if (per_seg > ps6 && (double)ps6 >= std::max(avg_seg_bytes, 1.0) * 1.05 + 1) per_seg = ps6;
  }
  const uint64_t cap = std::max<uint64_t>(64ull * MT_U * per_seg, 64ull * maxsyms);  // piece bytes staged at once
  if (STAGE_PAD + cap + 16 > region_max) return GH_OK;
  c->mt_ns = cap + 16 <= 4096 ? 4 : cap + 16 <= 6144 ? 6 : cap + 16 <= 8192 ? 8 : 10;  // the copy-out's chunks cover a piece
  c->stage_bytes = (uint32_t)((STAGE_PAD + cap + 16 + 15) & ~15ull);  // + the write overrun
  c->mt_gl = lookups_per_shift(K);
  c->mt_fb = fb;
  const void* kern = mtile_kernel_for(c->mt_gl, c->mt_ns, fb);
  c->lut_bytes = lut_b;
  c->lds = mtile_lds_bytes(c->lut_bytes, c->stage_bytes);
  int pc = 0;
  GH_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&pc, kern, MT_TB, c->lds));
  pc = std::min(pc, 2);  // (as tile_setup: the occupancy query can answer one too many)
  if (pc < 1) return GH_OK;
  std::vector<uint64_t> lt = multi_lut(cn, K);
  if (GH_MT_CLUT) {  // the count table (u32 {b | start mask << 16}, every codeword of the window)
    std::vector<uint32_t> lc(1u << Kc);
    for (uint32_t i = 0; i < (1u << Kc); ++i) {
      uint32_t n = 0, m = 0;
      const uint32_t b = window_codewords(cn, i, Kc, 32, &n, nullptr, &m);
      lc[i] = b | ((n ? (1u | (m << 1)) & ((1u << b) - 1u) : 0u) << 16);
    }
    if (clgr) {  // replicated: dword i = entry i >> clgr
      std::vector<uint32_t> lr(1u << (Kc + clgr));
      for (uint32_t i = 0; i < lr.size(); ++i) lr[i] = lc[i >> clgr];
      lc.swap(lr);
    }
    std::vector<uint64_t> both(lut_b / 8);
    const uint64_t cb = 4ull << (Kc + clgr);
    const bool cfirst = cb > (8ull << K);  // the larger table first (gh_mtile.hip)
    std::memcpy((uint8_t*)both.data() + (cfirst ? 0 : 8ull << K), lc.data(), cb);
    std::memcpy((uint8_t*)both.data() + (cfirst ? cb : 0), lt.data(), 8ull << K);
    lt.swap(both);
  }
  if (fb) {  // the canonical tables after the LUTs (the kernel reads the last FB_BYTES)
    uint32_t fbt[FB_WORDS];
    fallback_tables(cn, fbt);
    const size_t at = lut_b - FB_BYTES;
    lt.resize(lut_b / 8, 0);
    std::memcpy((uint8_t*)lt.data() + at, fbt, sizeof(fbt));
  }
  GH_HIP(hipMalloc(&c->d_lut_t, lut_b));
  GH_HIP(hipMemcpy(c->d_lut_t, lt.data(), lut_b, hipMemcpyHostToDevice));
  c->tile_k = K;
  c->lgr = clgr;  // (the two-pass kernel: the count table's copies)
  c->tile_u = MT_U;
  c->ntiles = (uint32_t)ceil_div(c->nseg, (uint64_t)MT_U * MT_TB);
  c->grid = (uint32_t)std::min<uint64_t>({(uint64_t)c->ntiles + 1, (uint64_t)pc * c->num_cu, (uint64_t)LEAD_A * MT_TB});
  if (c->grid < 2) return GH_OK;
  c->idle_block = 0xFFFFFFFFu;
  c->mtile = true;
  c->tile = true;
  return GH_OK;
}

// ---- wave split setup ------------------------------------------------------------
// Count-LUT width Kc in [max(maxlen, 2), 13] maximising bits per VALU op of a lookup
// group: GL lookups of ~6 ops each plus ~8 ops of window shift and end upkeep per chain
// (r=0.9: Kc=13, 10.6 vs 8.5 bits per lookup at 11; r=0.5: Kc=12, 10.3 vs 7.1 at 9-10).
// Longer codes: the fallback.  GH_WS_KC overrides (tests).
static uint32_t ws_count_bits(const Canon& cn) {
  const uint32_t lo = std::min<uint32_t>(std::max<uint32_t>(cn.maxlen, 2), 13);
  if (const char* e = getenv("GH_WS_KC")) return (uint32_t)std::clamp(atoi(e), (int)lo, 14);
  uint32_t best = lo;
  double best_eff = -1;
  for (uint32_t kc = lo; kc <= 13; ++kc) {  // 14 (64 KiB) measured no faster
    const int gl = lookups_per_shift(kc);
    const double eff = gl * count_lut(cn, kc, nullptr) / (6.0 * gl + 8.0);
    if (eff > best_eff * 1.01) {  // prefer the smaller table unless clearly better
      best_eff = eff;
      best = kc;
    }
  }
  return best;
}
// Write-LUT width K in [max(maxlen, 10), 12] maximising the expected bits per lookup
// (entries hold up to four codewords, so a wider window helps only codes whose short
// codewords it can fit more of: r=0.5 codes 7.6 -> 10.4 bits at K 10 -> 12) times
// lookups per window shift over ~13 ops per lookup plus ~12 per shift; a wider table
// must win by 5 % (its LDS costs occupancy).  GH_WS_K overrides (tests).
static uint32_t ws_write_bits(const Canon& cn) {
  if (const char* ek = getenv("GH_WS_K"))  // (a width below maxlen takes the canonical fallback)
    return (uint32_t)std::clamp(atoi(ek), 2, 12);
  const uint32_t lo = std::min<uint32_t>(std::max<uint32_t>(cn.maxlen, 10), 12);
  uint32_t best = lo;
  double best_eff = -1;
  for (uint32_t K = lo; K <= 12; ++K) {
    double sum = 0;
    for (uint32_t i = 0; i < (1u << K); ++i) sum += window_codewords(cn, i, K, 4, nullptr, nullptr, nullptr);
    const int gl = lookups_per_shift(K);
    const double eff = gl * (sum / (double)(1u << K)) / (13.0 * gl + 12.0);
    if (best_eff < 0 || eff > best_eff * 1.05) {
      best_eff = eff;
      best = K;
    }
  }
  return best;
}
#ifndef GH_WS_CLUT_MAX
#define GH_WS_CLUT_MAX 0  // count-LUT bytes in LDS with its copies (0: one copy; round 5: copies at Kc 10-12
                          // measured no faster on cfg3 than one copy at Kc 13, gpurun_out/r05am)
#endif
constexpr uint64_t WS_CLUT_MAX = GH_WS_CLUT_MAX;
static int ws_ns_for(double avg_seg_bytes) {
  const double chunks = avg_seg_bytes * 64 * WS_U / 16.0 * 1.15 + 2;
  const int ns = (int)std::ceil(chunks / 64);
  return ns <= 2 ? 2 : ns <= 3 ? 3 : ns <= 4 ? 4 : ns <= 6 ? 6 : 8;
}

static int ws_setup(gh_ctx* c, double avg_seg_bytes) {
  const Canon& cn = c->canon;
  const uint32_t K = ws_write_bits(cn), kc = ws_count_bits(cn);
  // canonical fallback: codewords longer than a table, or patterns outside an incomplete
  // code (a LUT entry with no codeword)
  const bool fb = kraft16(cn) != 65536 || cn.maxlen > std::min(K, kc);
  c->ws_fb = fb;
  c->ws_k = K;
  c->ws_kc = kc;
  {
    const std::vector<uint64_t> lw = write_lut(cn, K);
    std::vector<uint32_t> lc;
    count_lut(cn, kc, &lc);
    GH_HIP(hipMalloc(&c->d_ws_lut_w, 8ull << K));
    GH_HIP(hipMemcpy(c->d_ws_lut_w, lw.data(), 8ull << K, hipMemcpyHostToDevice));
    GH_HIP(hipMalloc(&c->d_ws_lut_c, 4ull << kc));
    GH_HIP(hipMemcpy(c->d_ws_lut_c, lc.data(), 4ull << kc, hipMemcpyHostToDevice));
    uint32_t fbt[FB_WORDS];
    fallback_tables(cn, fbt);
    GH_HIP(hipMalloc(&c->d_fb, sizeof(fbt)));
    GH_HIP(hipMemcpy(c->d_fb, fbt, sizeof(fbt), hipMemcpyHostToDevice));
  }
  c->lut_bytes = 8ull << K;  // >= 32 bytes: whole 16-byte chunks
  const size_t lb = c->lut_bytes + (fb ? (size_t)FB_BYTES : 0);  // write kernel: LUT + fallback tables
  constexpr int NW = WS_TB / 64;
  // codewords per segment: wholly inside [start, E), E - start <= 143
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
    if (avail < (long)chain_worst) return fail(GH_E_HIP, "wave-split staging does not fit");
    stage = (size_t)avail & ~15ull;
  }
  if (const char* es = getenv("GH_WS_STAGE"))  // tests: force a small staging (per-chain blocks)
    stage = std::max<size_t>((size_t)atoll(es), (chain_worst + 15) & ~15ull) & ~15ull;
  c->stage_bytes = (uint32_t)stage;
  c->lds = lb + NW * stage;
  // count LUT copies (lane l reads copy l mod 2^lgc: fewer bank conflicts on the skewed
  // lookups), up to 32 KB in LDS; GH_WS_LGC overrides (tests, experiments)
  c->ws_lgc = 0;
  if (!fb) {
    uint32_t lgc = 0;
    while (lgc < 5 && (4ull << (kc + lgc + 1)) <= (uint64_t)WS_CLUT_MAX && 30u - kc - (lgc + 1) >= 16u) ++lgc;
    if (const char* e = getenv("GH_WS_LGC")) lgc = (uint32_t)std::clamp(atoi(e), 0, std::max(0, 14 - (int)kc));
    c->ws_lgc = lgc;
  }
  c->lds_count = std::max<size_t>(4ull << (kc + c->ws_lgc), 64) + (fb ? FB_BYTES : 0);
  c->ws_ns = ws_ns_for(avg_seg_bytes);
  if (const char* en = getenv("GH_WS_NS")) c->ws_ns = std::clamp(atoi(en), 2, 8);
  const WsKernels k = ws_kernels(kc, K, c->ws_ns, fb);
  int pc_c = 0, pc_w = 0;
  GH_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&pc_c, k.count, WS_TBC, c->lds_count));
  GH_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&pc_w, k.write, WS_TB, c->lds));
  if (pc_c < 1 || pc_w < 1) return fail(GH_E_HIP, "wave-split kernels do not fit on a CU");
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
  GH_HIP(hipMalloc(&c->d_seg_cnt, c->nseg + WS_CNT_PAD + 16));
  GH_HIP(hipMalloc(&c->d_ws_junk, 16ull * 64 * c->ws_nranges));
  GH_HIP(hipMalloc(&c->d_rng_tot, 8ull * c->ws_nranges + 16));
  GH_HIP(hipMalloc(&c->d_rng_off, 8ull * c->ws_nranges + 16));
  c->ws = true;
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
  for (uint32_t ml : {3u, 4u, 5u})
    for (uint32_t gv : {2u, 3u, 4u})
      (void)hipFuncSetAttribute(tile_kernel_for(ml, gv), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  for (int gl : {2, 3, 4})
    for (int ns : {4, 6, 8, 10})
      for (bool fb : {false, true})
        (void)hipFuncSetAttribute(mtile_kernel_for(gl, ns, fb), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  (void)hipGetLastError();
  *out = c;
  return GH_OK;
}

extern "C" int gh_ctx_device(gh_ctx* c, int* device) {
  if (!c || !device) return fail(GH_E_ARG, "null argument");
  *device = c->device;
  return GH_OK;
}

// The tile kernel's workgroups wait on each other (round prefixes): it assumes that the
// whole grid becomes resident.  Two of them running at once on one device (several shard
// contexts on one GPU, each on its own stream) can each hold half the CUs and wait
// forever for the rest (their bounded spins then report GH_ST_TIMEOUT).  So launches
// of such kernels on one device are chained: each waits for the previous one's
// completion event, whatever stream either was launched on.
struct DevChain {
  std::mutex mu;
  hipEvent_t last = nullptr;          // the last tile decode's done_ev (owned by `owner`)
  const gh_ctx* owner = nullptr;
  bool has = false;
  hipStream_t last_stream = nullptr;  // the stream the last tile kernel ran on
};
static DevChain& dev_chain(int device) {
  static std::mutex mu;
  static std::map<int, DevChain*> m;
  std::lock_guard<std::mutex> g(mu);
  DevChain*& d = m[device];
  if (!d) d = new DevChain();  // one per device, for the life of the process
  return *d;
}

extern "C" int gh_ctx_destroy(gh_ctx* c) {
  if (!c) return GH_OK;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->done_rec) (void)hipEventSynchronize(c->done_ev);
  {  // the device chain must not keep one of this context's events
    DevChain& dc = dev_chain(c->device);
    std::lock_guard<std::mutex> g(dc.mu);
    if (dc.owner == c) {
      dc.has = false;
      dc.owner = nullptr;
      dc.last = nullptr;
    }
  }
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
  if (e - b >= (1ull << 31))  // 32-bit segment indices in the kernels: 32 GiB of payload per shard
    return fail(GH_E_ARG, "shard of 2^31 or more segments: split the stream into more shards");
  free_shard(c);
  int rc = build_canon(s->syms, s->nsyms, c->canon);
  if (rc) return rc;
  const Canon& cn = c->canon;
  c->nseg = e - b;
  c->seg_begin = b;
  c->seg_end = e;
  c->n_total = s->n;
  if (c->nseg > 0 && cn.nsyms == 0) return fail(GH_E_TABLE, "empty code");
  const uint64_t per_seg = cn.minlen ? (128 + cn.minlen - 1) / cn.minlen : 128;  // codewords per segment, at most
  if (out_cap == 0) out_cap = std::min<uint64_t>(s->n, c->nseg * per_seg);
  c->out_cap = out_cap;
  GH_HIP(hipSetDevice(c->device));
  GH_HIP(hipMalloc(&c->d_out, std::max<uint64_t>(out_cap, 16) + 64));
  GH_HIP(hipMemset(c->d_misc, 0, 128));
  c->epoch = 0;
  c->ntiles = 0;
  c->grid = 0;
  if (c->nseg > 0) {
    // Structure: the tile kernel for grouped codes, the wave split for every other code.
    // GH_MODE=tile|wsplit forces one; GH_LUT_BITS sets the tile kernel's LUT width (a
    // width below maxlen leaves the code to the wave split).
    const char* envm = getenv("GH_MODE");
    const bool force_tile = envm && !strcmp(envm, "tile"), force_ws = envm && !strcmp(envm, "wsplit");
    const bool force_mt = envm && !strcmp(envm, "mtile");
    if (envm && *envm && !force_tile && !force_ws && !force_mt) return fail(GH_E_ARG, "GH_MODE: tile, mtile or wsplit");
    const char* envk = getenv("GH_LUT_BITS");
    const uint32_t K = envk ? (uint32_t)std::clamp(atoi(envk), 1, 12) : cn.maxlen;
    const bool grouped = (grouped_code(cn) || short_code(cn)) && K >= cn.maxlen;
    if (force_tile && !grouped)
      return fail(GH_E_ARG, "GH_MODE=tile: the code is not for the tile kernel (complete, 3..12 bits)");
    const double avg = s->g ? (double)s->n / (double)s->g : 16.0;
    if (grouped && !force_ws && !force_mt) {
      if ((rc = tile_setup(c, K, avg))) return rc;
      if (force_tile && !c->tile) return fail(GH_E_HIP, "GH_MODE=tile: the tile kernel does not fit a CU");
    }
    // the two-pass tile kernel: codes of 2..12-bit codewords the single-pass one does not
    // take (cfg3's r = 0.9 codes; GH_MTILE=0 leaves them to the wave split, GH_MODE=mtile
    // forces it)
    const bool multi = cn.maxlen <= 16 && kraft16(cn) == 65536;
    if (force_mt && !multi)
      return fail(GH_E_ARG, "GH_MODE=mtile: the code is not for the two-pass tile kernel (complete, 1..16 bits)");
    static const bool mt_on = [] {
      const char* e = getenv("GH_MTILE");
      return !(e && e[0] == '0');
    }();
    if (!c->tile && multi && (force_mt || (mt_on && !force_ws && !force_tile))) {
      if ((rc = mtile_setup(c, avg))) return rc;
      if (force_mt && !c->tile) return fail(GH_E_HIP, "GH_MODE=mtile: the two-pass tile kernel does not fit a CU");
    }
    if (!c->tile && (rc = ws_setup(c, avg))) return rc;
  }
  // tile kernel: per-tile aggregates and prefixes
  c->gran_words = c->tile ? 2ull * c->ntiles + 2 : 1;
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
  // zero only the padding past the copied words: the copies below may run on the
  // staging set's non-blocking stream, which is not ordered against this memset
  GH_HIP(hipMemset(c->d_payload + have, 0, 4 * (alloc_words - have)));
  if (have) {
    if (use_staged(4 * have)) {  // pinned double-buffered (concurrent across shards' threads)
      if (int rc2 = h2d_staged(c->device, (const uint8_t*)s->payload + 4 * w0, 4 * have, c->d_payload)) return rc2;
    } else {
      GH_HIP(hipMemcpy(c->d_payload, (const uint8_t*)s->payload + 4 * w0, 4 * have, hipMemcpyHostToDevice));
    }
  }
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
  c->ws_last_end = 0;
  if (c->ws && e == s->g) {
    uint32_t w5[5] = {};
    for (uint64_t i = 0; i < 5; ++i)
      if (4 * (e - 1) + i < s->w) std::memcpy(&w5[i], (const uint8_t*)s->payload + 4 * (4 * (e - 1) + i), 4);
    c->ws_last_end = last_segment_end(c->canon, w5, c->nseg == 1 ? c->first_start : seg_start_host(s, e - 1));
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
  GH_HIP(hipMemset(c->d_payload + have, 0, 4 * (alloc_words - have)));
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
  c->ws_last_end = 0;
  if (c->ws && e == s->g) {
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
    c->ws_last_end = last_segment_end(c->canon, w5, st);
  }
  c->loaded = true;
  return GH_OK;
}

extern "C" int gh_ctx_decode(gh_ctx* c, void* hip_stream, int timed) {
  if (!c) return fail(GH_E_ARG, "null ctx");
  if (!c->loaded) return fail(GH_E_STATE, "gh_ctx_decode before gh_ctx_load");
  hipStream_t st = hip_stream ? (hipStream_t)hip_stream : c->stream;
  GH_HIP(hipSetDevice(c->device));
  if (c->nseg == 0) {
    GH_HIP(hipMemsetAsync(c->d_misc + 2, 0, 8, st));
    GH_HIP(hipEventRecord(c->done, st));
    c->done_ev = c->done;
    c->done_rec = true;
    return GH_OK;
  }
  // Tile kernels are chained per device: wait for the previous one before the start
  // event, so a decode's time excludes its queueing behind other contexts' decodes.
  DevChain& dc = dev_chain(c->device);
  std::unique_lock<std::mutex> chain_lock(dc.mu, std::defer_lock);
  if (c->tile) {
    if (++c->epoch >= EPOCH_MAX) {  // granule epochs wrap: start clean
      GH_HIP(hipMemsetAsync(c->d_gran, 0, 8ull * c->gran_words, st));
      c->epoch = 1;
    }
    chain_lock.lock();
    // (the context's own stream, which the last tile decode of the device ran on for this
    // same context, is ordered behind it already: no wait packet.  A caller's stream is
    // never trusted that way: it may have been destroyed and its handle reused since.)
    const bool ordered = dc.owner == c && dc.last_stream == st && st == c->stream;
    if (dc.has && !ordered) GH_HIP(hipStreamWaitEvent(st, dc.last, 0));
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
    if (!c->tile) GH_HIP(hipEventRecord(ev.first, st));  // (tile: in the dispatch itself, below)
  }
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
    m.stage_bytes = c->stage_bytes;
    m.last_end = c->ws_last_end;
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
    wc.lgc = c->ws_lgc;
    ww = m;
    ww.lut = (const uint2*)c->d_ws_lut_w;
    ww.kbits = c->ws_k;
    ww.lut_bytes = (uint32_t)c->lut_bytes;
    ac[0] = &wc;
    aw[0] = &ww;
    const WsKernels wk = ws_kernels(c->ws_kc, c->ws_k, c->ws_ns, c->ws_fb);
    GH_HIP(hipLaunchKernel(wk.count, dim3(c->ws_grid_c), dim3(WS_TBC), ac, c->lds_count, st));
    GH_HIP(hipLaunchKernel((const void*)gh_ws_scan_kernel, dim3(1), dim3(WS_SCAN_TB), ac, 0, st));
    GH_HIP(hipLaunchKernel(wk.write, dim3(c->grid), dim3(WS_TB), aw, c->lds, st));
  } else {
    TileParams t{};
    t.payload = c->d_payload;
    t.gaps = c->d_gaps;
    t.lut = c->d_lut_t;
    t.out = c->d_out;
    t.granules = c->d_gran;
    t.prefix = c->d_gran + c->ntiles;
    t.status = c->d_misc + 1;
    t.total = (unsigned long long*)(c->d_misc + 2);
    t.stats = (unsigned long long*)(c->d_misc + 4);
    t.tickets = (unsigned int*)(c->d_gran + 2ull * c->ntiles);  // the two spare granule words
    t.out_cap = c->out_cap;
    t.nseg = c->nseg;
    t.gap_nib0 = c->gap_nib0;
    t.first_start = c->first_start;
    t.ntiles = c->ntiles;
    t.kbits = c->tile_k;
    t.lgr = c->lgr;
    t.epoch = c->epoch;
    t.lut_bytes = (uint32_t)c->lut_bytes;
    t.stage_bytes = c->stage_bytes;
    t.kbits_c = c->mt_kc;
    t.fb_hi = c->canon.maxlen;
    t.stamps = c->d_stamps;
    t.tstamps = c->d_stamps ? (unsigned long long*)((uint8_t*)c->d_stamps + 32ull * c->grid * 2 * 128) : nullptr;
    t.idle_block = c->idle_block;
    const void* kern = c->mtile ? mtile_kernel_for(c->mt_gl, c->mt_ns, c->mt_fb) : tile_kernel_for(c->tile_minl, c->tile_g);
    static thread_local void* ta[1];
    static thread_local TileParams tp;
    tp = t;
    ta[0] = &tp;
    // timed: the start and stop timestamps are taken by the dispatch packet itself
    // (hipExtLaunchKernel), not by marker packets around it, so back-to-back decodes
    // have no extra packets between them
    if (timed)
      GH_HIP(hipExtLaunchKernel(kern, dim3(c->grid), dim3(c->mtile ? MT_TB : TILE_TB), ta, c->lds, st, ev.first,
                                ev.second, 0));
    else
      GH_HIP(hipLaunchKernel(kern, dim3(c->grid), dim3(c->mtile ? MT_TB : TILE_TB), ta, c->lds, st));
  }
  GH_HIP(hipGetLastError());
  // one event after the kernel(s): the timed decode's end event, or `done` (each marker
  // between back-to-back decodes costs the GPU microseconds)
  if (timed) {
    if (!c->tile) GH_HIP(hipEventRecord(ev.second, st));
    c->pending.push_back(ev);
    c->done_ev = ev.second;
  } else {
    GH_HIP(hipEventRecord(c->done, st));
    c->done_ev = c->done;
  }
  c->done_rec = true;
  if (c->tile) {  // the device chain's last decode (chain_lock held)
    dc.last = c->done_ev;
    dc.owner = c;
    dc.has = true;
    dc.last_stream = st;
  }
  return GH_OK;
}

// Waits for the context's last decode, whatever stream it was launched on.
static int wait_decode(gh_ctx* c) {
  GH_HIP(hipStreamSynchronize(c->stream));
  if (c->done_rec) GH_HIP(hipEventSynchronize(c->done_ev));
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
  if (GH_TILE_STAMPS && c->d_stamps) {  // diagnostic builds: the last decode's phase deltas
    if (const char* f = getenv("GH_STAMPS_OUT")) {
      std::vector<uint8_t> h(32ull * c->grid * 2 * 128 + 8ull * (3ull * c->ntiles + 64 + 4 * 1024 + 4ull * c->grid));
      GH_HIP(hipMemcpy(h.data(), c->d_stamps, h.size(), hipMemcpyDeviceToHost));
      if (FILE* fp = fopen(f, "wb")) {
        fwrite(h.data(), 1, h.size(), fp);
        fclose(fp);
      }
    }
  }
  unsigned int misc[6] = {};
  GH_HIP(hipMemcpy(misc, c->d_misc, sizeof(misc), hipMemcpyDeviceToHost));
  if (rep) {
    std::memset(rep, 0, sizeof(*rep));
    uint64_t tot;
    std::memcpy(&tot, misc + 2, 8);
    rep->symbols = tot;
    rep->out_bytes = std::min<uint64_t>(tot, c->out_cap);
    rep->status = misc[1];
    rep->lut_bits = c->tile ? c->tile_k : c->ws_k;
    rep->grid = c->grid;
    rep->tiles = c->ntiles;
    rep->mode = c->mtile ? GH_MODE_MTILE : c->tile ? GH_MODE_TILE : GH_MODE_SPLIT;
    std::memcpy(&rep->slow_lookbacks, misc + 4, 8);
    rep->path = c->mtile ? GH_PATH_MULTI_TILE : c->tile ? GH_PATH_GROUPED : GH_PATH_MULTI_WAVE;
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
  if (use_staged(nbytes)) return d2h_staged(c->device, c->d_out + off, nbytes, dst);
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
  if (c->done_rec) GH_HIP(hipStreamWaitEvent(st, c->done_ev, 0));  // after the last decode
  GH_HIP(hipMemcpyAsync(dst, c->d_out + off, nbytes, hipMemcpyDefault, st));
  return GH_OK;
}

// Decode time of a set of shards: decodes on one device run in turn (DevChain), so a
// device's time is the sum of its shards' kernel times; devices run side by side.
static float shards_kernel_ms(const std::vector<gh_ctx*>& ctx, const std::vector<gh_report>& reps) {
  std::map<int, float> per_dev;
  for (size_t k = 0; k < ctx.size(); ++k) per_dev[ctx[k]->device] += reps[k].kernel_ms;
  float worst = 0;
  for (auto& d : per_dev) worst = std::max(worst, d.second);
  return worst;
}

// Runs f(k) for every shard k in its own host thread (one shard alone: inline);
// returns the first failure's code with its message moved to the calling thread.
template <class F>
static int for_each_shard(int n, F f) {
  if (n == 1) return f(0);
  std::vector<int> rc(n, GH_OK);
  std::vector<std::string> msg(n);
  std::vector<std::thread> th;
  for (int k = 0; k < n; ++k)
    th.emplace_back([&, k] {
      rc[k] = f(k);
      if (rc[k]) msg[k] = gh_last_error();
    });
  for (auto& t : th) t.join();
  for (int k = 0; k < n; ++k)
    if (rc[k]) {
      set_error(msg[k]);
      return rc[k];
    }
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
  // Phase 1, one host thread per shard: context, H2D of the shard's words (pinned,
  // double-buffered: the shards' PCIe transfers overlap across devices), the decodes
  // (chained per device), the report.  The reference loads, decodes and downloads one
  // device at a time (decoder.cu:759-801).
  std::vector<gh_report> reps_k(ng);
  rc = for_each_shard(ng, [&](int k) {
    const int dev = (o && o->devices) ? o->devices[k] : (ng > 1 ? k : 0);
    int r = gh_ctx_create(dev, &ctx[k]);
    if (!r) r = gh_ctx_load(ctx[k], s, bounds[k], bounds[k + 1], ng > 1 ? 0 : s->n);
    for (int i = 0; i < reps && !r; ++i) r = gh_ctx_decode(ctx[k], nullptr, 1);
    if (!r) r = gh_ctx_report(ctx[k], nullptr, &reps_k[k]);
    return r;
  });
  if (rc) {
    cleanup();
    return rc;
  }
  // output offsets: exclusive scan of the shards' symbol counts
  std::vector<uint64_t> offs(ng + 1, 0), want(ng, 0);
  uint32_t status = 0;
  for (int k = 0; k < ng; ++k) {
    status |= reps_k[k].status;
    if (k + 1 < ng && reps_k[k].symbols > reps_k[k].out_bytes) {
      cleanup();
      return fail(GH_E_CORRUPT, "shard produced more symbols than its output capacity");
    }
    want[k] = (offs[k] < s->n) ? std::min<uint64_t>(reps_k[k].symbols, s->n - offs[k]) : 0;
    offs[k + 1] = offs[k] + reps_k[k].symbols;
  }
  const uint64_t offset = offs[ng];
  // Phase 2, one host thread per shard: D2H into the caller's buffer at its offset.
  rc = for_each_shard(ng, [&](int k) { return want[k] ? gh_ctx_download(ctx[k], 0, out + offs[k], want[k]) : GH_OK; });
  const float dec_ms = shards_kernel_ms(ctx, reps_k);
  cleanup();
  if (rc) return rc;
  if (rep) {
    *rep = reps_k[0];
    rep->symbols = offset;
    rep->out_bytes = std::min<uint64_t>(offset, s->n);
    rep->status = status;
    rep->kernel_ms = dec_ms;
  }
  if (status & GH_ST_TIMEOUT) return fail(GH_E_HIP, "look-back timed out");
  if (offset < s->n) return fail(GH_E_CORRUPT, "stream decoded to fewer than N symbols");
  if (status & GH_ST_BADCODE) return fail(GH_E_CORRUPT, "invalid code in stream");
  return GH_OK;
}
