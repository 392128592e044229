// GPU encoder of the compressed.huff format: the reference's
// encoder.cu pipeline (histogram :118-140, cuencoder :142-355, cu_get_gaparray
// :358-379) re-designed for gfx950.  Byte-identical to the host encoder
// (gh_core.cpp gh_encode_write), which restates the reference's packing: codewords
// MSB-first inside u32 words; for every codeword crossing a 128-bit boundary, the
// nibble (end bit mod 16) at the index of the segment it starts in, 8 nibbles per
// u32, LSB-first.
//
// Kernels (input resident in HBM, 8 KiB chunks of 512 threads x 16 bytes; 4 KiB of 256
// until round 6: the write kernel's per-chunk work (two barriers, the last word's
// completion, edge gap words) is then spread over twice the bytes, cfg4 1.05 -> 0.93 ms):
//   gh_enc_hist_kernel   byte histogram; LDS counters replicated 32x (lane & 31), so
//                        one instruction's lanes collide at most 2-way even on the
//                        skewed r=0.9 data; 256 u64 atomics per workgroup.
//   (host)               package-merge + canonical codes (gh::plan_from_counts).
//   gh_enc_bits_kernel   code bits per chunk (u32).
//   gh_enc_scan_kernel   exclusive scan of the chunk bits in blocks of 8192 chunks,
//   gh_enc_blkscan_kernel  then of the block totals (u64).
//   gh_enc_write_kernel  one chunk per workgroup: block scan of the lanes' bits,
//                        codewords OR-ed
//                        into a zeroed LDS image of the chunk's words (positions in
//                        32 bits relative to the chunk's gap-word-aligned base),
//                        then written with coalesced stores.  No payload atomics: a
//                        chunk owns the words whose first bit it holds, and its last
//                        lane encodes the next chunk's first symbols (< 32 bits) to
//                        complete its last word.  Gap nibbles likewise in LDS; the two
//                        edge gap words of a chunk (shared with its neighbours) are
//                        atomicOr-ed into the zeroed gap array, the rest stored.
// Traffic: N (histogram, plan step) + 2N + C + gaps (encode) bytes.  A single pass
// with a decoupled look-back (one 4 KiB chunk per workgroup) measured 2.85 ms on
// cfg4, slower than these three kernels: its workgroups waited on their nearest
// predecessors' aggregates.
#include <hip/hip_runtime.h>

#include <cstring>
#include <vector>

#include "gaphuff.h"
#include "gh_internal.hpp"

namespace gh {

#ifndef GH_ENC_TB
#define GH_ENC_TB 512
#endif
constexpr int ETB = GH_ENC_TB;           // threads per workgroup
constexpr int EBPT = 16;                 // input bytes per thread
constexpr int ECHUNK = ETB * EBPT;       // input bytes per chunk
constexpr int EREP = 32;                 // histogram replicas
// LDS image of a chunk from its gap-word-aligned base: up to 1023 bits before it,
// 16 bits per byte, the last word's completion (< 32 + 16 bits).  These are the bounds;
// the write kernel's image is sized at launch for the code's longest codeword (dynamic
// LDS: 9-bit codes, cfg4, take 4.7 KB per 4 KiB instead of 8.3)
constexpr int EWORDS = (1024 + ECHUNK * GH_MAX_CODE_LEN + 64) / 32 + 2;
constexpr int EGAPW = (1024 + ECHUNK * GH_MAX_CODE_LEN) / 1024 + 2;

__device__ __forceinline__ uint32_t enc_byte(const uint4& v, int k) {
  const uint32_t w = k < 4 ? v.x : k < 8 ? v.y : k < 12 ? v.z : v.w;
  return (w >> (8 * (k & 3))) & 0xFFu;
}

// 16 input bytes of thread t of chunk c (bytes past n read as "absent": 0x100).
__device__ __forceinline__ void enc_load(const uint8_t* in, uint64_t n, uint64_t base, uint32_t (&b)[EBPT]) {
  if (base + EBPT <= n) {
    const uint4 v = *(const uint4*)(in + base);
#pragma unroll
    for (int k = 0; k < EBPT; ++k) b[k] = enc_byte(v, k);
  } else {
#pragma unroll
    for (int k = 0; k < EBPT; ++k) b[k] = base + k < n ? (uint32_t)in[base + k] : 0x100u;
  }
}

__global__ __launch_bounds__(ETB) void gh_enc_hist_kernel(const uint8_t* in, uint64_t n,
                                                          unsigned long long* count) {
  __shared__ uint32_t h[256 * EREP];
  const int tid = threadIdx.x;
  for (int i = tid; i < 256 * EREP; i += ETB) h[i] = 0;
  __syncthreads();
  const uint32_t rep = (uint32_t)tid & (EREP - 1);
  const uint64_t nchunks = (n + ECHUNK - 1) / ECHUNK;
  for (uint64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    uint32_t b[EBPT];
    enc_load(in, n, c * ECHUNK + (uint64_t)tid * EBPT, b);
#pragma unroll
    for (int k = 0; k < EBPT; ++k)
      if (b[k] < 256u) atomicAdd(&h[b[k] * EREP + rep], 1u);
  }
  __syncthreads();
  for (int v = tid; v < 256; v += ETB) {
    unsigned long long s = 0;
#pragma unroll
    for (int r = 0; r < EREP; ++r) s += h[v * EREP + ((r + v) & (EREP - 1))];
    if (s) atomicAdd(&count[v], s);
  }
}

// Inclusive wave scan on the VALU with DPP (row_shr 1/2/4/8 within 16-lane rows,
// row_bcast 15/31 across them): no LDS round trips, unlike ds_bpermute shuffles.
__device__ __forceinline__ uint32_t enc_wave_scan(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, true);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, true);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, true);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);
  return v;
}

// Workgroup exclusive scan of one u32 per thread; returns the exclusive prefix and
// sets total.  s_red: NWAVE u32 of LDS.
__device__ __forceinline__ uint32_t enc_block_scan(uint32_t x, uint32_t* s_red, uint32_t& total) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  uint32_t incl = x;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(incl, d, 64);
    if (lane >= d) incl += y;
  }
  if (lane == 63) s_red[wid] = incl;
  __syncthreads();
  uint32_t before = 0;
  total = 0;
#pragma unroll
  for (int q = 0; q < ETB / 64; ++q) {
    const uint32_t v = s_red[q];
    before += q < wid ? v : 0u;
    total += v;
  }
  return before + incl - x;
}

// Persistent: workgroup b takes chunk groups (b + EBQ*k*G + j*G, j < EBQ); the next
// group's bytes (EBQ 16-byte loads per thread: the bytes in flight per CU set this
// kernel's bandwidth) are loaded before the current group's reduction.  Loads are
// unconditional (chunk index clamped, input padded past n), bytes past n masked by index.
#ifndef GH_ENC_NT
#define GH_ENC_NT 3  // (round 4: 3) write kernel, bits: 1 input loads nontemporal, 2 payload word stores nontemporal; 4 bits-kernel loads nontemporal
#endif
#ifndef GH_ENC_OOB
#define GH_ENC_OOB 1  // write kernel: padding stores out of a buffer resource's range (dropped) instead of to a junk dword
#endif
#ifndef GH_ENC_UOR
#define GH_ENC_UOR 1  // write kernel: a quad's first two (1: three) image words ORed unconditionally
#endif
#ifndef GH_ENC_LSUM
#define GH_ENC_LSUM 1  // write kernel: lengths summed from the entries' low halves (no per-entry mask)
#endif
#ifndef GH_ENC_BQ
#define GH_ENC_BQ 2  // chunks in flight per thread (4 measured slower: 246 vs 229 us on cfg4)
#endif
#ifndef GH_ENC_BREP
#define GH_ENC_BREP 32  // code-length table copies in LDS (lane l reads copy l mod BREP: no bank conflicts at 32)
#endif
constexpr int EBQ = GH_ENC_BQ;
constexpr int EBREP = GH_ENC_BREP;
__global__ __launch_bounds__(ETB) void gh_enc_bits_kernel(const uint8_t* in, uint64_t n, uint32_t nchunks,
                                                          const uint32_t* lut, uint32_t* chunk_bits) {
  __shared__ uint32_t s_lenr[256 * EBREP];
  __shared__ uint32_t s_red[2][EBQ][ETB / 64];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  for (int i = tid; i < 256 * EBREP; i += ETB) s_lenr[i] = lut[i / EBREP] & 0xFFu;
  const uint32_t* s_len = s_lenr + (lane & (EBREP - 1));  // entry b of this lane's copy: s_len[b * EBREP]
  const uint32_t G = gridDim.x;
  auto ld = [&](uint32_t cc) {
    const uint8_t* src = in + (uint64_t)min(cc, nchunks - 1) * ECHUNK + (uint64_t)tid * EBPT;
    if (GH_ENC_NT & 4) {
      typedef unsigned int v4u __attribute__((ext_vector_type(4)));
      const v4u t = __builtin_nontemporal_load((const v4u*)src);
      return make_uint4(t.x, t.y, t.z, t.w);
    }
    return *(const uint4*)src;
  };
  auto chunk_bits_of = [&](const uint4& v, uint32_t cc) {
    const uint64_t ib = (uint64_t)cc * ECHUNK + (uint64_t)tid * EBPT;
    uint32_t bits = 0;
    if (ib + EBPT <= n) {
#pragma unroll
      for (int k = 0; k < EBPT; ++k) bits += s_len[enc_byte(v, k) * EBREP];
    } else {
      const uint32_t rem = ib < n ? (uint32_t)(n - ib) : 0u;
#pragma unroll
      for (int k = 0; k < EBPT; ++k) bits += (uint32_t)k < rem ? s_len[enc_byte(v, k) * EBREP] : 0u;
    }
    return bits;
  };
  uint32_t c = blockIdx.x;
  uint4 v[EBQ];
#pragma unroll
  for (int j = 0; j < EBQ; ++j) v[j] = ld(c + (uint32_t)j * G);
  __syncthreads();
  for (uint32_t it = 0; c < nchunks; c += EBQ * G, ++it) {
    uint32_t b[EBQ];
#pragma unroll
    for (int j = 0; j < EBQ; ++j) b[j] = chunk_bits_of(v[j], c + (uint32_t)j * G);
#pragma unroll
    for (int j = 0; j < EBQ; ++j) v[j] = ld(c + (uint32_t)(EBQ + j) * G);
#pragma unroll
    for (int j = 0; j < EBQ; ++j) {
      const uint32_t sc = enc_wave_scan(b[j]);  // lane 63: the wave total
      if (lane == 63) s_red[it & 1][j][wid] = sc;
    }
    __syncthreads();  // (double-buffered partial sums: one barrier per group)
    if (tid < EBQ) {
      uint32_t t = 0;
#pragma unroll
      for (int q = 0; q < ETB / 64; ++q) t += s_red[it & 1][tid][q];
      const uint32_t cc = c + (uint32_t)tid * G;
      if (cc < nchunks) chunk_bits[cc] = t;
    }
  }
}

// Chunk offsets in two levels.  gh_enc_scan_kernel: workgroup k scans chunks
// [8192k, 8192k + 8192) (8 consecutive per thread): local exclusive offsets and the
// block total.  gh_enc_blkscan_kernel (one workgroup): exclusive scan of the block
// totals.  The write kernel adds the two.
constexpr int SCAN_TB = 1024, SCAN_PT = 8, SCAN_BLK = SCAN_TB * SCAN_PT;
static_assert((unsigned long long)SCAN_BLK * ECHUNK * 16 < (1ull << 32), "scan block bits fit u32");
__global__ __launch_bounds__(SCAN_TB) void gh_enc_scan_kernel(const uint32_t* chunk_bits, uint32_t nchunks,
                                                              uint32_t* chunk_loc, unsigned long long* blk_tot) {
  __shared__ uint32_t s_w[SCAN_TB / 64];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const uint32_t i0 = blockIdx.x * (uint32_t)SCAN_BLK + (uint32_t)tid * SCAN_PT;
  uint32_t v[SCAN_PT], t = 0;
#pragma unroll
  for (int k = 0; k < SCAN_PT; ++k) v[k] = i0 + k < nchunks ? chunk_bits[i0 + k] : 0u;
#pragma unroll
  for (int k = 0; k < SCAN_PT; ++k) {
    const uint32_t x = v[k];
    v[k] = t;  // exclusive within the thread
    t += x;
  }
  uint32_t incl = t;  // a block holds < 2^32 bits (8192 chunks x 16 x ECHUNK, ECHUNK <= 16 KiB)
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(incl, d, 64);
    if (lane >= d) incl += y;
  }
  if (lane == 63) s_w[wid] = incl;
  __syncthreads();
  uint32_t before = 0, tot = 0;
#pragma unroll
  for (int q = 0; q < SCAN_TB / 64; ++q) {
    const uint32_t x = s_w[q];
    before += q < wid ? x : 0u;
    tot += x;
  }
  const uint32_t b0 = before + incl - t;
#pragma unroll
  for (int k = 0; k < SCAN_PT; ++k)
    if (i0 + k < nchunks) chunk_loc[i0 + k] = b0 + v[k];
  if (tid == 0) blk_tot[blockIdx.x] = tot;
}
__global__ __launch_bounds__(SCAN_TB) void gh_enc_blkscan_kernel(unsigned long long* blk, uint32_t nblk) {
  __shared__ unsigned long long s[SCAN_TB];
  const int tid = threadIdx.x;
  unsigned long long carry = 0;
  for (uint32_t base = 0; base < nblk; base += SCAN_TB) {
    const uint32_t i = base + (uint32_t)tid;
    const unsigned long long x = i < nblk ? blk[i] : 0ull;
    s[tid] = x;
    __syncthreads();
    for (int d = 1; d < SCAN_TB; d <<= 1) {
      const unsigned long long y = tid >= d ? s[tid - d] : 0ull;
      __syncthreads();
      s[tid] += y;
      __syncthreads();
    }
    if (i < nblk) blk[i] = carry + s[tid] - x;
    carry += s[SCAN_TB - 1];
    __syncthreads();
  }
}

struct EncParams {
  const uint8_t* in;
  const uint32_t* lut;                 // 256 x {code << 8 | len}
  const uint32_t* chunk_loc;           // bit offset of each chunk within its scan block
  const unsigned long long* blk_off;   // bit offset of each scan block
  uint32_t* words;                     // W payload words
  uint32_t* gaps;                      // GW gap words, zeroed
  uint32_t* junk;                      // one dword per thread of the grid (padding stores)
  uint64_t n;
  uint32_t nchunks;
  uint32_t ewords, egapw;  // LDS image words (payload, gaps): (1024 + ECHUNK x maxlen + 64) / 32 + 2, (1024 + ECHUNK x maxlen) / 1024 + 2
};

// Write-kernel LUT replicas (lane l reads copy l mod ELREP): 16 copies collide at most
// 2-way and leave room for 6 waves per SIMD; the long-code shapes (NSW >= 6: cfg4's
// r = 0.1 codes, ~8 bits per byte) take 32 (conflict-free, 3 workgroups per CU by LDS):
// cfg4 1.055 vs 1.096 ms, while cfg3 / cfg2 lose 6-11 % at 32 (round 4, gpurun_out/r04x).
#ifndef GH_ENC_LREP_LONG
#define GH_ENC_LREP_LONG 32
#endif
template <int NSW>
constexpr int enc_lrep() { return NSW * ETB * 4096 / ECHUNK >= 5 * 256 ? GH_ENC_LREP_LONG : 16; }  // (>= 0.3 words per input byte)
#ifndef GH_ENC_WPE
#define GH_ENC_WPE 4  // the write kernel's occupancy hint, waves per SIMD (6 and 8 spill)
#endif
// the write kernel's occupancy hint (its VGPR budget: 512 / waves per SIMD)
template <int NSW>
constexpr int enc_wpe() { return GH_ENC_WPE; }

// A thread's 16 codewords, combined in registers: LUT entries hold the code
// left-aligned, e = code << (32 - len) | len (len <= 16 sits in the low 5 bits, below
// the code), so a pair is one shift and one AND-OR (v_lshrrev reads only the low 5
// bits of the entry it shifts by), and two pairs make a left-aligned 64-bit quad.
// Each quad is ORed into the LDS image as up to three words.
__device__ __forceinline__ uint32_t enc_pair(uint32_t a, uint32_t c, uint32_t& len) {
  len = GH_ENC_LSUM ? (a + c) & 0xFFFFu : (a & 31u) + (c & 31u);
  return (a & 0xFFFF0000u) | ((c & 0xFFFF0000u) >> (a & 31u));
}

// Persistent: workgroup b encodes chunks b, b + G, ...  The next chunk's bytes and
// offset (and the 32 bytes after it, for its last word) are loaded while the current
// chunk is encoded; the LDS image is re-zeroed as it is written out.  NSW: payload
// store instructions per thread per chunk, a fixed count (padding stores go to the
// thread's junk dword; words past NSW * ETB loop), plus one gap-word store: loads and
// stores share one in-order counter (vmcnt), and with a fixed count of stores younger
// than the prefetch the next chunk waits for its loads with vmcnt(N) instead of also
// waiting for this chunk's stores.
template <int NSW>
__global__ __launch_bounds__(ETB) __attribute__((amdgpu_waves_per_eu(enc_wpe<NSW>()))) void gh_enc_write_kernel(
    const EncParams p) {
  constexpr int ELREP = enc_lrep<NSW>();
  __shared__ uint32_t s_lutr[257 * ELREP];  // left-aligned entries, replicated
  __shared__ uint32_t s_red[2][ETB / 64];
  extern __shared__ uint32_t s_dyn[];  // the image (p.ewords) and its gap words (p.egapw), sized for the code's longest codeword
  uint32_t* const s_w = s_dyn;
  uint32_t* const s_g = s_dyn + p.ewords;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  uint32_t c = blockIdx.x;
  const uint32_t G = gridDim.x;
  // chunk c's inputs: its 16 bytes per lane, its offset, and (last lane) the next 32 bytes
  uint4 v = make_uint4(0, 0, 0, 0);
  uint32_t xbyte = 0;
  unsigned long long offb = 0;  // chunk offset = block part + local part, added at use
  uint32_t offl = 0;            // (an add here would wait for the loads at once)
  // every load unconditional and in bounds (the input buffer is padded by ECHUNK + 64
  // bytes past n; bytes past n are masked by index), so no branch holds a load
  auto fetch = [&](uint32_t cc) {
    const uint64_t ib = (uint64_t)cc * ECHUNK + (uint64_t)tid * EBPT;
    if (GH_ENC_NT & 1) {
      typedef unsigned int v4u __attribute__((ext_vector_type(4)));
      const v4u t = __builtin_nontemporal_load((const v4u*)(p.in + ib));
      v = make_uint4(t.x, t.y, t.z, t.w);
    } else {
      v = *(const uint4*)(p.in + ib);
    }
    offb = p.blk_off[cc / SCAN_BLK];
    offl = p.chunk_loc[cc];
    xbyte = p.in[(uint64_t)(cc + 1) * ECHUNK + (uint64_t)(lane & 31)];  // the next chunk's byte lane & 31
  };
  if (c < p.nchunks) fetch(c);
  for (int i = tid; i < 257 * ELREP; i += ETB) {
    const uint32_t v = i / ELREP < 256 ? p.lut[i / ELREP] : 0u;
    const uint32_t l = v & 0xFFu;
    s_lutr[i] = l ? ((v >> 8) << (32u - l)) | l : 0u;
  }
  for (uint32_t i = tid; i < p.ewords + p.egapw; i += ETB) s_dyn[i] = 0;
  __syncthreads();
  for (uint32_t it = 0; c < p.nchunks; c += G, ++it) {
    // this chunk's bytes (absent past n: 0x100, length 0)
    const uint64_t ib = (uint64_t)c * ECHUNK + (uint64_t)tid * EBPT;
    uint32_t b[EBPT];
    if (ib + EBPT <= p.n) {  // (divergent only in the last chunk)
#pragma unroll
      for (int k = 0; k < EBPT; ++k) b[k] = enc_byte(v, k);
    } else {
      const uint32_t rem = ib < p.n ? (uint32_t)(p.n - ib) : 0u;
#pragma unroll
      for (int k = 0; k < EBPT; ++k) b[k] = (uint32_t)k < rem ? enc_byte(v, k) : 0x100u;
    }
    const uint32_t nx = xbyte;  // this iteration's copy (fetch() overwrites xbyte)
    const uint64_t xb = (uint64_t)(c + 1) * ECHUNK;
    const unsigned long long o0 = offb + offl;
    if (c + G < p.nchunks) fetch(c + G);  // prefetch
    uint32_t e[EBPT], bits = 0;
#pragma unroll
    for (int k = 0; k < EBPT; ++k) e[k] = s_lutr[b[k] * ELREP + (tid & (ELREP - 1))];
    if (GH_ENC_LSUM) {  // the entries' low 16 bits hold only their lengths: one sum, one mask
#pragma unroll
      for (int k = 0; k < EBPT; ++k) bits += e[k];
      bits &= 0xFFFFu;
    } else {
#pragma unroll
      for (int k = 0; k < EBPT; ++k) bits += e[k] & 31u;
    }
    // block scan (double-buffered wave sums: the barrier also orders the previous
    // iteration's write-out and re-zeroing before this iteration's OR-s)
    const uint32_t incl = enc_wave_scan(bits);
    if (lane == 63) s_red[it & 1][wid] = incl;
    __syncthreads();
    uint32_t before = 0, cbits = 0;
#pragma unroll
    for (int qq = 0; qq < ETB / 64; ++qq) {
      const uint32_t x = s_red[it & 1][qq];
      before += qq < wid ? x : 0u;
      cbits += x;
    }
    const uint32_t excl = before + incl - bits;
    // positions relative to B = the chunk's offset rounded down to a gap word (1024
    // bits): 128-bit boundaries, payload words and gap words keep their alignment
    const unsigned long long B = o0 & ~1023ull;
    const uint32_t qs = (uint32_t)(o0 - B);  // chunk start
    const uint32_t qend = qs + cbits;        // chunk end (the next chunk's first bit)
    const uint32_t q0 = qs + excl;           // this thread's first bit
    // pairs and quads (left-aligned), the quads ORed into the image
    uint32_t pl[EBPT / 2], pv[EBPT / 2];
#pragma unroll
    for (int j = 0; j < EBPT / 2; ++j) pv[j] = enc_pair(e[2 * j], e[2 * j + 1], pl[j]);
    uint32_t qa = q0, qe[EBPT / 4];
#pragma unroll
    for (int i = 0; i < EBPT / 4; ++i) {
      const uint32_t l0 = pl[2 * i], m = l0 + pl[2 * i + 1];
      const unsigned long long Q = ((unsigned long long)pv[2 * i] << 32) |
                                   ((unsigned long long)pv[2 * i + 1] << (32u - l0));
      const uint32_t hi = (uint32_t)(Q >> 32), lo = (uint32_t)Q, sft = qa & 31u;
      uint32_t* wp = &s_w[qa >> 5];
      if (GH_ENC_UOR) {  // ORing zero bits is harmless: no compares, no exec-mask changes
        atomicOr(wp, hi >> sft);
        atomicOr(wp + 1, __builtin_amdgcn_alignbit(hi, lo, sft));
        if (GH_ENC_UOR == 1 || sft + m > 64u) atomicOr(wp + 2, __builtin_amdgcn_alignbit(lo, 0u, sft));
      } else {
        if (m) atomicOr(wp, hi >> sft);
        if (sft + m > 32u) atomicOr(wp + 1, __builtin_amdgcn_alignbit(hi, lo, sft));
        if (sft + m > 64u) atomicOr(wp + 2, __builtin_amdgcn_alignbit(lo, 0u, sft));
      }
      qa += m;
      qe[i] = qa;
    }
    // gap nibbles: for each 128-bit boundary strictly inside [q0, qa), the codeword
    // holding bits bd-1 and bd (quad, then pair, then codeword by compare-selects)
    for (uint32_t bd = ((q0 >> 7) + 1u) << 7; bd < qa; bd += 128u) {
      const bool i0 = bd >= qe[0], i1 = bd >= qe[1], i2 = bd >= qe[2];
      const uint32_t qs4 = i2 ? qe[2] : i1 ? qe[1] : i0 ? qe[0] : q0;
      const uint32_t la = i2 ? pl[6] : i1 ? pl[4] : i0 ? pl[2] : pl[0];
      const uint32_t lb = i2 ? pl[7] : i1 ? pl[5] : i0 ? pl[3] : pl[1];
      const uint32_t ea = i2 ? e[12] : i1 ? e[8] : i0 ? e[4] : e[0];
      const uint32_t eb = i2 ? e[14] : i1 ? e[10] : i0 ? e[6] : e[2];
      const bool second = bd >= qs4 + la;  // in the quad's second pair
      const uint32_t ps = second ? qs4 + la : qs4;
      const uint32_t lp = second ? lb : la;
      const uint32_t l1 = (second ? eb : ea) & 31u;  // the pair's first codeword
      const bool c2 = bd >= ps + l1;
      const uint32_t cs = c2 ? ps + l1 : ps;        // codeword start
      const uint32_t ce = c2 ? ps + lp : ps + l1;   // codeword end
      const uint32_t gv = ce & 15u;
      if (cs < bd && gv && cs < qend) atomicOr(&s_g[cs >> 10], gv << (4 * ((cs >> 7) & 7u)));
    }
    if (wid == ETB / 64 - 1) {
      // complete the chunk's last word (bits [qend, wend)) with the next chunk's first
      // codewords, one per lane (lanes 0..31: bytes 0..31, codes >= 1 bit); their gap
      // nibbles belong to the next chunk
      const uint32_t wend = (qend + 31u) & ~31u;
      const uint32_t ex = (lane < 32 && xb + (uint32_t)lane < p.n) ? s_lutr[nx * ELREP + (tid & (ELREP - 1))] : 0u;
      const uint32_t lx = ex & 31u;
      const uint32_t st = qend + enc_wave_scan(lx) - lx;  // this codeword's first bit
      if (lx && st < wend) {
        const uint32_t cw = ex & 0xFFFF0000u, sh = st & 31u;  // left-aligned code
        atomicOr(&s_w[st >> 5], cw >> sh);
        if (sh + lx > 32u) atomicOr(&s_w[(st >> 5) + 1], cw << (32u - sh));
      }
    }
    __syncthreads();
    // payload words whose first bit lies in [o0, o0 + cbits): local [w0, w1); the
    // image is zeroed as it is read (up to the completion word)
    const uint32_t w0 = (qs + 31u) >> 5, w1 = (qend + 31u) >> 5;
    uint32_t* wout = p.words + (B >> 5);
    uint32_t* junk = p.junk + (size_t)blockIdx.x * ETB + tid;
    // (GH_ENC_OOB) buffer stores from the chunk's base (B is workgroup-uniform), the
    // padding ones out of range: dropped, no memory traffic
    const unsigned long long Bu = ((unsigned long long)(uint32_t)__builtin_amdgcn_readfirstlane((int)(B >> 32)) << 32) |
                                  (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)B);
    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(p.words + (Bu >> 5), 0, 0x7FFFFFF0, 0x00020000);
#pragma unroll
    for (int j = 0; j < NSW; ++j) {
      const uint32_t i = (uint32_t)tid + (uint32_t)(ETB * j);
      const uint32_t x = s_w[i < p.ewords ? i : 0u];
      if (i <= w1) s_w[i] = 0;
      if (GH_ENC_OOB) {
        const int off = (i >= w0 && i < w1) ? (int)(4u * i) : 0x7FFFFFF0;
        __builtin_amdgcn_raw_buffer_store_b32(x, rw, off, 0, (GH_ENC_NT & 2) ? 2 : 0);
      } else {
        uint32_t* d = (i >= w0 && i < w1) ? wout + i : junk;
        if (GH_ENC_NT & 2) __builtin_nontemporal_store(x, d);
        else *d = x;
      }
    }
    for (uint32_t i = tid + ETB * NSW; i <= w1; i += ETB) {
      const uint32_t x = s_w[i];
      s_w[i] = 0;
      if (i >= w0 && i < w1) wout[i] = x;
    }
    // gap words of this chunk's segments: local [0, g1]; the first and the last may
    // hold nibbles of the neighbouring chunks
    const uint32_t g1 = cbits ? (qend - 1u) >> 10 : 0u;
    uint32_t* gout = p.gaps + (B >> 10);
    static_assert(EGAPW <= ETB, "one gap word per thread");
    {
      const uint32_t i = (uint32_t)tid;
      const uint32_t x = s_g[i < p.egapw ? i : 0u];
      if (i <= g1) s_g[i] = 0;
      const bool in = cbits && i <= g1, edge = i == 0 || i == g1;
      if (GH_ENC_OOB) {  // interior: a plain store (always issued)
        const __amdgpu_buffer_rsrc_t rg = __builtin_amdgcn_make_buffer_rsrc(p.gaps + (Bu >> 10), 0, 0x7FFFFFF0, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b32(x, rg, (in && !edge) ? (int)(4u * i) : 0x7FFFFFF0, 0, 0);
      } else {
        *((in && !edge) ? gout + i : junk) = x;
      }
      if (in && edge && x) atomicOr(&gout[i], x);
    }
  }
}

}  // namespace gh

using namespace gh;

#define GH_EHIP(expr)                                                             \
  do {                                                                            \
    hipError_t e_ = (expr);                                                       \
    if (e_ != hipSuccess)                                                         \
      return fail(GH_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));   \
  } while (0)

struct gh_ectx {
  int device = 0;
  int num_cu = 0;
  hipStream_t stream = nullptr;
  uint8_t* d_in = nullptr;
  uint64_t n = 0, in_cap = 0;
  unsigned long long* d_count = nullptr;   // 256
  uint32_t* d_lut = nullptr;               // 256
  uint32_t* d_chunk_bits = nullptr;
  unsigned long long* d_chunk_off = nullptr;
  uint64_t chunk_cap = 0;
  uint32_t* d_words = nullptr;
  uint32_t* d_gaps = nullptr;
  uint32_t* d_junk = nullptr;              // write kernel padding stores: one dword per thread
  uint64_t junk_cap = 0;
  uint64_t words_cap = 0, gaps_cap = 0;
  gh_encode_plan plan{};
  bool planned = false, encoded = false;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
};

extern "C" int gh_ectx_create(int device, gh_ectx** out) {
  if (!out) return fail(GH_E_ARG, "null ctx pointer");
  *out = nullptr;
  int nd = 0;
  if (hipGetDeviceCount(&nd) != hipSuccess || nd == 0)
    return fail(GH_E_NODEV, "no HIP device visible (the GPU encoder has no CPU fallback)");
  if (device < 0 || device >= nd) return fail(GH_E_ARG, "device ordinal out of range");
  hipDeviceProp_t prop;
  GH_EHIP(hipGetDeviceProperties(&prop, device));
  if (std::string(prop.gcnArchName).find("gfx950") == std::string::npos)
    return fail(GH_E_NODEV, std::string("device is ") + prop.gcnArchName + ", need gfx950");
  GH_EHIP(hipSetDevice(device));
  gh_ectx* e = new gh_ectx();
  e->device = device;
  e->num_cu = prop.multiProcessorCount;
  GH_EHIP(hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking));
  GH_EHIP(hipMalloc(&e->d_count, 256 * 8));
  GH_EHIP(hipMalloc(&e->d_lut, 256 * 4));
  GH_EHIP(hipEventCreate(&e->ev0));
  GH_EHIP(hipEventCreate(&e->ev1));
  *out = e;
  return GH_OK;
}

extern "C" int gh_ectx_destroy(gh_ectx* e) {
  if (!e) return GH_OK;
  (void)hipSetDevice(e->device);
  if (e->stream) (void)hipStreamSynchronize(e->stream);
  for (void* p : {(void*)e->d_in, (void*)e->d_count, (void*)e->d_lut, (void*)e->d_chunk_bits,
                  (void*)e->d_chunk_off, (void*)e->d_words, (void*)e->d_gaps, (void*)e->d_junk})
    (void)hipFree(p);
  if (e->ev0) (void)hipEventDestroy(e->ev0);
  if (e->ev1) (void)hipEventDestroy(e->ev1);
  if (e->stream) (void)hipStreamDestroy(e->stream);
  delete e;
  return GH_OK;
}

extern "C" int gh_ectx_load(gh_ectx* e, const uint8_t* in, uint64_t n) {
  if (!e || (n && !in)) return fail(GH_E_ARG, "null argument");
  GH_EHIP(hipSetDevice(e->device));
  // padded: the write kernel's loads are unconditional (up to a chunk + 32 bytes past n)
  const uint64_t need = n + ECHUNK + 64;
  if (need > e->in_cap) {
    (void)hipFree(e->d_in);
    e->d_in = nullptr;
    e->in_cap = 0;
    GH_EHIP(hipMalloc(&e->d_in, need));
    e->in_cap = need;
  }
  if (n) GH_EHIP(hipMemcpyAsync(e->d_in, in, n, hipMemcpyHostToDevice, e->stream));
  GH_EHIP(hipStreamSynchronize(e->stream));
  e->n = n;
  e->planned = e->encoded = false;
  return GH_OK;
}

extern "C" int gh_ectx_plan(gh_ectx* e, int force_version, gh_encode_plan* plan) {
  if (!e) return fail(GH_E_ARG, "null ctx");
  GH_EHIP(hipSetDevice(e->device));
  GH_EHIP(hipMemsetAsync(e->d_count, 0, 256 * 8, e->stream));
  const uint64_t nchunks = ceil_div(e->n, ECHUNK);
  if (nchunks) {
    const uint32_t grid = (uint32_t)std::min<uint64_t>(nchunks, 4ull * e->num_cu);
    hipLaunchKernelGGL(gh_enc_hist_kernel, dim3(grid), dim3(ETB), 0, e->stream, e->d_in, e->n, e->d_count);
    GH_EHIP(hipGetLastError());
  }
  gh_encode_plan& pl = e->plan;
  std::memset(&pl, 0, sizeof(pl));
  pl.n = e->n;
  GH_EHIP(hipMemcpyAsync(pl.count, e->d_count, 256 * 8, hipMemcpyDeviceToHost, e->stream));
  GH_EHIP(hipStreamSynchronize(e->stream));
  const int rc = plan_from_counts(&pl, force_version);
  if (rc) return rc;
  e->planned = true;
  e->encoded = false;
  if (plan) *plan = pl;
  return GH_OK;
}

extern "C" int gh_ectx_encode(gh_ectx* e, float* kernel_ms) {
  if (!e) return fail(GH_E_ARG, "null ctx");
  if (!e->planned) return fail(GH_E_STATE, "gh_ectx_encode before gh_ectx_plan");
  GH_EHIP(hipSetDevice(e->device));
  const gh_encode_plan& pl = e->plan;
  for (int v = 0; v < 256; ++v)
    if (pl.len[v] > GH_MAX_CODE_LEN) return fail(GH_E_TABLE, "code longer than 16 bits");
  uint32_t lut[256];
  for (int v = 0; v < 256; ++v) lut[v] = (pl.code[v] << 8) | pl.len[v];
  const uint64_t nchunks = ceil_div(e->n, ECHUNK);
  const uint64_t GW = ceil_div(pl.g, GH_GAPS_PER_WORD);
  if (nchunks + 1 > e->chunk_cap) {
    (void)hipFree(e->d_chunk_bits);
    (void)hipFree(e->d_chunk_off);
    e->d_chunk_bits = nullptr;
    e->d_chunk_off = nullptr;
    e->chunk_cap = 0;
    GH_EHIP(hipMalloc(&e->d_chunk_bits, 4 * (nchunks + 1)));
    GH_EHIP(hipMalloc(&e->d_chunk_off, 4 * (nchunks + 1) + 8 * (nchunks / SCAN_BLK + 2) + 64));
    e->chunk_cap = nchunks + 1;
  }
  if (pl.w + 4 > e->words_cap) {
    (void)hipFree(e->d_words);
    e->d_words = nullptr;
    e->words_cap = 0;
    GH_EHIP(hipMalloc(&e->d_words, 4 * (pl.w + 4)));
    e->words_cap = pl.w + 4;
  }
  if (GW + 4 > e->gaps_cap) {
    (void)hipFree(e->d_gaps);
    e->d_gaps = nullptr;
    e->gaps_cap = 0;
    GH_EHIP(hipMalloc(&e->d_gaps, 4 * (GW + 4)));
    e->gaps_cap = GW + 4;
  }
  if (nchunks >= (1ull << 32)) return fail(GH_E_ARG, "input too large for the GPU encoder");
  GH_EHIP(hipMemcpyAsync(e->d_lut, lut, sizeof(lut), hipMemcpyHostToDevice, e->stream));
  GH_EHIP(hipEventRecord(e->ev0, e->stream));
  GH_EHIP(hipMemsetAsync(e->d_gaps, 0, 4 * (GW + 4), e->stream));
  if (nchunks) {
    // payload words per chunk ~ 4096 * W / n: NSW = store instructions per thread
    const double wpc = (double)ECHUNK * (double)pl.w / (double)std::max<uint64_t>(e->n, 1) + 2.0;
    const int need = (int)std::ceil(wpc * 1.05 / ETB);
    const void* wk = need <= 1   ? (const void*)gh_enc_write_kernel<1>
                     : need <= 2 ? (const void*)gh_enc_write_kernel<2>
                     : need <= 3 ? (const void*)gh_enc_write_kernel<3>
                     : need <= 4 ? (const void*)gh_enc_write_kernel<4>
                     : need <= 5 ? (const void*)gh_enc_write_kernel<5>
                     : need <= 6 ? (const void*)gh_enc_write_kernel<6>
                                 : (const void*)gh_enc_write_kernel<9>;
    // the LDS image holds a chunk at the code's longest codeword
    uint32_t maxlen = 1;
    for (int v = 0; v < 256; ++v) maxlen = std::max<uint32_t>(maxlen, pl.len[v]);
    const uint32_t ew = (1024u + ECHUNK * maxlen + 64u) / 32u + 2u, eg = (1024u + ECHUNK * maxlen) / 1024u + 2u;
    if (ew > (uint32_t)EWORDS || eg > (uint32_t)EGAPW) return fail(GH_E_TABLE, "code longer than 16 bits");
    const size_t dyn = 4ull * (ew + eg);
    int pb = 0, pw = 0;  // persistent grids: what is resident at once
    GH_EHIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&pb, (const void*)gh_enc_bits_kernel, ETB, 0));
    GH_EHIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&pw, wk, ETB, dyn));
    const uint32_t gb = (uint32_t)std::min<uint64_t>(nchunks, (uint64_t)std::max(pb, 1) * e->num_cu);
    hipLaunchKernelGGL(gh_enc_bits_kernel, dim3(gb), dim3(ETB), 0, e->stream, e->d_in, e->n, (uint32_t)nchunks,
                       e->d_lut, e->d_chunk_bits);
    const uint32_t nblk = (uint32_t)ceil_div(nchunks, SCAN_BLK);
    uint32_t* loc = (uint32_t*)e->d_chunk_off;
    unsigned long long* blk = e->d_chunk_off + (nchunks + 2) / 2 + 1;  // after the local offsets
    hipLaunchKernelGGL(gh_enc_scan_kernel, dim3(nblk), dim3(SCAN_TB), 0, e->stream, e->d_chunk_bits,
                       (uint32_t)nchunks, loc, blk);
    hipLaunchKernelGGL(gh_enc_blkscan_kernel, dim3(1), dim3(SCAN_TB), 0, e->stream, blk, nblk);
    const uint32_t gw = (uint32_t)std::min<uint64_t>(nchunks, (uint64_t)std::max(pw, 1) * e->num_cu);
    if ((uint64_t)gw * ETB > e->junk_cap) {
      (void)hipFree(e->d_junk);
      e->d_junk = nullptr;
      e->junk_cap = 0;
      GH_EHIP(hipMalloc(&e->d_junk, 4ull * gw * ETB));
      e->junk_cap = (uint64_t)gw * ETB;
    }
    EncParams p{e->d_in, e->d_lut, loc, blk, e->d_words, e->d_gaps, e->d_junk, e->n, (uint32_t)nchunks, ew, eg};
    void* args[] = {&p};
    GH_EHIP(hipLaunchKernel(wk, dim3(gw), dim3(ETB), args, dyn, e->stream));
    GH_EHIP(hipGetLastError());
  }
  GH_EHIP(hipEventRecord(e->ev1, e->stream));
  GH_EHIP(hipStreamSynchronize(e->stream));
  if (kernel_ms) GH_EHIP(hipEventElapsedTime(kernel_ms, e->ev0, e->ev1));
  e->encoded = true;
  return GH_OK;
}

extern "C" int gh_ectx_download(gh_ectx* e, void* out, uint64_t out_len) {
  if (!e || !out) return fail(GH_E_ARG, "null argument");
  if (!e->encoded) return fail(GH_E_STATE, "gh_ectx_download before gh_ectx_encode");
  const gh_encode_plan& pl = e->plan;
  if (out_len < pl.file_bytes) return fail(GH_E_SMALL, "output buffer too small");
  GH_EHIP(hipSetDevice(e->device));
  uint8_t* o = (uint8_t*)out;
  const size_t hdr = encode_header(&pl, o);
  const uint64_t GW = ceil_div(pl.g, GH_GAPS_PER_WORD);
  if (GW) GH_EHIP(hipMemcpyAsync(o + hdr, e->d_gaps, 4 * GW, hipMemcpyDeviceToHost, e->stream));
  if (pl.w) GH_EHIP(hipMemcpyAsync(o + hdr + 4 * GW, e->d_words, 4 * pl.w, hipMemcpyDeviceToHost, e->stream));
  GH_EHIP(hipStreamSynchronize(e->stream));
  return GH_OK;
}
