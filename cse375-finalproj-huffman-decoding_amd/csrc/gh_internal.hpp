// Internal helpers shared by the host library (gh_core.cpp) and the HIP decoder
// (gh_decode.hip).  Not part of the C ABI.
#pragma once
#include <cstdint>
#include <string>

#include "gaphuff.h"

namespace gh {

// Thread-local last-error message behind gh_last_error().
void set_error(const std::string& msg);
int fail(int code, const std::string& msg);

// Canonical code of a stream's (symbol,length) list in file order, restating the
// code assignment shared by the encoder (package_merge.cpp:168-181) and the
// decoder's table builder (get_table.cpp:70-83): code starts at 0 for the first
// (most frequent) entry and steps as code = (code+1) << (len[i+1]-len[i]).
struct Canon {
  uint32_t nsyms = 0;
  uint32_t minlen = 0, maxlen = 0;
  uint8_t sym[GH_MAX_SYMBOLS] = {};     // file order
  uint8_t len[GH_MAX_SYMBOLS] = {};
  uint32_t code[GH_MAX_SYMBOLS] = {};   // right-aligned code value
  // Per-length canonical ranges on a 16-bit left-aligned scale.
  uint32_t count[GH_MAX_CODE_LEN + 2] = {};
  uint32_t base16[GH_MAX_CODE_LEN + 2] = {};   // first code of length l << (16-l)
  uint32_t limit16[GH_MAX_CODE_LEN + 2] = {};  // base16[l] + count[l] << (16-l)
  uint32_t first[GH_MAX_CODE_LEN + 2] = {};    // file index of first length-l code
};

// Builds `c` from a stream's symbol list; returns GH_OK or GH_E_TABLE.
int build_canon(const gh_sym* syms, uint32_t nsyms, Canon& c);

// Decode one codeword from the top bits of `w16` (16 bits, left-aligned).
// Returns the length (1..16) and the file index, or 0 when the bits fall outside
// the code space.
inline uint32_t canon_decode16(const Canon& c, uint32_t w16, uint32_t* index) {
  for (uint32_t l = c.minlen; l <= c.maxlen; ++l) {
    if (c.count[l] == 0) continue;
    if (w16 < c.limit16[l]) {
      *index = c.first[l] + ((w16 - c.base16[l]) >> (16 - l));
      return l;
    }
  }
  return 0;
}

inline uint64_t ceil_div(uint64_t a, uint64_t b) { return (a + b - 1) / b; }

// Encoder plan from plan->n and plan->count[] (symbol order, package-merge lengths,
// canonical codes, sizes, header version); shared by the host and GPU encoders.
int plan_from_counts(gh_encode_plan* plan, int force_version);
// Writes the image header; returns its size.  out must hold file_bytes - payload.
size_t encode_header(const gh_encode_plan* plan, uint8_t* out);

// Host memory <-> device memory through the device's pinned staging buffers
// (gh_io.cpp): each 32 MiB chunk is copied to / from a pinned buffer by a few host
// threads while the DMA of the previous chunk runs (hipMemcpyAsync), so shards on
// different devices, loaded from different host threads, move concurrently.
int h2d_staged(int device, const void* src, uint64_t n, void* dst);
int d2h_staged(int device, const void* src, uint64_t n, void* dst);
// Large copies go through the staging unless GH_H2D=pageable (measurements).
bool use_staged(uint64_t n);

}  // namespace gh
