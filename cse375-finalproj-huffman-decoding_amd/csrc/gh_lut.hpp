// Decode tables built on the host from a stream's canonical code (gh_internal.hpp's
// Canon), shared by the two decode structures of gh_decode.hip.  The reference builds
// one fixed 10-bit single-symbol table (decoder/src/get_table.cpp:15-95) that is wrong
// for maxlen < 10; these tables are sized by the code itself.
//
//   tile kernel (grouped codes)  u32 {len | sym << 8 | len << 23}, one codeword per lookup;
//   wave split, count pass       u32 {b | end mask << 16}: every codeword wholly inside
//                                the Kc-bit window (bit e-1 of the mask per codeword
//                                end e, b = their bits);
//   wave split, write pass       u64 {up to four symbol bytes, b | n << 8};
//   canonical fallback           FB_WORDS u32: running limit16[1..16], base16[1..16],
//                                first[1..16], then the symbol bytes (file order) —
//                                for codewords longer than a table and for patterns
//                                outside an incomplete code.
// Not part of the C ABI.
#pragma once
#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <vector>

#include "gh_internal.hpp"

namespace gh {

constexpr int FB_WORDS = 3 * 17 + 64;  // limit16 / base16 / first (index 0..16) + 256 symbol bytes
constexpr int FB_BYTES = ((4 * FB_WORDS) + 15) & ~15;

// Kraft sum of the code on a 2^16 scale (65536: complete).
inline uint64_t kraft16(const Canon& c) {
  uint64_t k = 0;
  for (uint32_t l = 1; l <= 16; ++l) k += (uint64_t)c.count[l] << (16 - l);
  return k;
}

// Greedy decode of the K-bit window `idx` (MSB first): up to `cap` codewords lying
// wholly inside it.  Returns their bits b; n, the symbols (byte k = k-th, when cap <= 4)
// and the end mask (bit e-1 per codeword end e) go to the out-parameters.
inline uint32_t window_codewords(const Canon& c, uint32_t idx, uint32_t K, uint32_t cap, uint32_t* n,
                                 uint32_t* syms, uint32_t* mask) {
  const uint32_t bits = idx << (32 - K);
  uint32_t pos = 0, k = 0, s = 0, m = 0;
  while (k < cap && pos < K) {
    uint32_t fi = 0;
    const uint32_t l = canon_decode16(c, (bits << pos) >> 16, &fi);
    if (l == 0 || pos + l > K) break;
    if (k < 4) s |= (uint32_t)c.sym[fi] << (8 * k);
    ++k;
    pos += l;
    m |= 1u << (pos - 1);
  }
  if (n) *n = k;
  if (syms) *syms = s;
  if (mask) *mask = m;
  return pos;
}

// Expected symbols per lookup of a four-symbol table of width K on random input bits
// (a complete code's codeword of length l then has probability 2^-l); an entry with
// no codeword counts 1 (its fallback lookup).
inline double multi_gain(const Canon& c, uint32_t K) {
  double syms = 0;
  for (uint32_t i = 0; i < (1u << K); ++i) {
    uint32_t n = 0;
    window_codewords(c, i, K, 4, &n, nullptr, nullptr);
    syms += n ? n : 1;
  }
  return syms / (double)(1u << K);
}

// Codes for the tile kernel: complete, minlen >= 4 (a segment holds at most 32
// codewords, kept in registers), maxlen <= 12, and a multi-symbol lookup would
// average < 1.5 symbols (else the wave split's four-symbol lookups win).
inline bool grouped_code(const Canon& c) {
  return c.nsyms > 0 && c.minlen >= 4 && c.maxlen <= 12 && kraft16(c) == 65536 && multi_gain(c, 12) < 1.5;
}

// Codes for the tile kernel's minlen-3 shape: complete, shortest codeword 3 bits (at
// most 43 per segment), maxlen <= 12 (BASELINE's r = 0.5 codes: 3- and 8/9-bit).  One
// codeword per lookup in one payload read beats the wave split's two passes of
// four-symbol lookups there.  GH_TILE3=0 leaves them to the wave split.
inline bool short_code(const Canon& c) {
  static const bool off = [] {
    const char* e = getenv("GH_TILE3");
    return e && e[0] == '0';
  }();
  return !off && c.nsyms > 0 && c.minlen == 3 && c.maxlen <= 12 && kraft16(c) == 65536;
}

// Tile kernel LUT of width K >= maxlen: entry i = {len | sym << 8 | len << 23} of the
// codeword at the top of i (the layout of the tile kernel's decode state, gh_tile.hip).
inline std::vector<uint32_t> grouped_lut(const Canon& c, uint32_t K) {
  std::vector<uint32_t> t(std::max<uint32_t>(1u << K, 4), 0u);
  for (uint32_t i = 0; i < (1u << K); ++i) {
    uint32_t fi = 0;
    const uint32_t l = canon_decode16(c, (i << (32 - K)) >> 16, &fi);
    t[i] = l | ((uint32_t)c.sym[fi] << 8) | (l << 23);
  }
  return t;
}

// Wave-split write LUT: entry i = {symbols, b | n << 8}, up to four codewords (n = 0:
// the first codeword is longer than K or outside the code: the fallback decodes it).
inline std::vector<uint64_t> write_lut(const Canon& c, uint32_t K) {
  std::vector<uint64_t> t(1u << K);
  for (uint32_t i = 0; i < (1u << K); ++i) {
    uint32_t n = 0, s = 0;
    const uint32_t b = window_codewords(c, i, K, 4, &n, &s, nullptr);
    t[i] = (uint64_t)s | ((uint64_t)(b | (n << 8)) << 32);
  }
  return t;
}

// Two-pass tile kernel LUT (gh_mtile.hip): entry i = {symbols, b | n << 8 | startmask << 16},
// the write LUT's up to four codewords plus their starts (bit s: a codeword starts at
// window bit s; bit 0 whenever n > 0).
inline std::vector<uint64_t> multi_lut(const Canon& c, uint32_t K) {
  std::vector<uint64_t> t(1u << K);
  for (uint32_t i = 0; i < (1u << K); ++i) {
    uint32_t n = 0, s = 0, m = 0;
    const uint32_t b = window_codewords(c, i, K, 4, &n, &s, &m);
    const uint32_t starts = n ? (1u | (m << 1)) & ((1u << b) - 1u) : 0u;
    t[i] = (uint64_t)s | ((uint64_t)(b | (n << 8) | (starts << 16)) << 32);
  }
  return t;
}

// Wave-split count LUT: entry i = b | end mask << 16, every codeword of the window
// (Kc <= 14, so the mask fits 16 bits).  Returns the expected bits per lookup on random
// input bits (*out may be null: the estimate only).
inline double count_lut(const Canon& c, uint32_t Kc, std::vector<uint32_t>* out) {
  double sum = 0;
  if (out) out->assign(1u << Kc, 0u);
  for (uint32_t i = 0; i < (1u << Kc); ++i) {
    uint32_t m = 0;
    const uint32_t b = window_codewords(c, i, Kc, 32, nullptr, nullptr, &m);
    sum += b;
    if (out) (*out)[i] = b | (m << 16);
  }
  return sum / (double)(1u << Kc);
}

// Canonical fallback tables.  limit16 is carried forward over empty lengths, so a
// search from any length finds the codeword's own (or none: outside the code).
inline void fallback_tables(const Canon& c, uint32_t (&fb)[FB_WORDS]) {
  std::fill(fb, fb + FB_WORDS, 0u);
  uint32_t run = 0;
  for (uint32_t l = 1; l <= 16; ++l) {
    if (c.count[l]) run = c.limit16[l];
    fb[l] = run;
    fb[17 + l] = c.base16[l];
    fb[34 + l] = c.first[l];
  }
  uint8_t* sy = (uint8_t*)(fb + 51);
  for (uint32_t i = 0; i < c.nsyms; ++i) sy[i] = c.sym[i];
}

// Lookups per 32-bit window shift for a table of width K (GL * K <= 31 bits).
inline int lookups_per_shift(uint32_t K) { return K <= 7 ? 4 : K <= 10 ? 3 : 2; }

}  // namespace gh
