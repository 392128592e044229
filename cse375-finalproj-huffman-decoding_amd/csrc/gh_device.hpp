// Device helpers shared by the tile kernel (gh_tile.hip) and the wave split
// (gh_wsplit.hip): the segment window, gap nibbles, DPP wave scans, look-back granules
// and LDS accesses at absolute addresses.  Included by gh_decode.hip only.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "gh_lut.hpp"

namespace gh {

// A segment's bits in a 160-bit funnel register d0..d4 (d0 = the next 32 stream bits,
// MSB first).  Starting at bit s <= 15 it holds >= 145 valid bits: enough for the last
// codeword (a segment's codewords start before bit 128 and are at most 16 bits).  The
// window advances by whole 32-bit shifts of v_alignbit; there is no shift-by-32 case
// (the reference's `>> (32 - x)` with x = 0).
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

// The window pre-shifted right by S bits (the "e-window", 16 <= S <= 31, start <= 15):
// bits before the segment read as 0, and the K-bit index of the codeword at the window
// position sits at bits [31 - S - K + 1, 31 - S], so with S = 32 - K - log2(entry bytes)
// a lookup address is x & mask: one op fewer than (x >> sh) & mask.  It holds the
// segment's bits up to 160 - S past its start; a codeword that starts before bit 128 and
// is at most K bits long ends inside it.
__device__ __forceinline__ Win make_ewin(uint4 w, uint32_t w4, int start, uint32_t S) {
  const uint32_t r = S - (uint32_t)start;  // 1..31
  Win v;
  v.d0 = __builtin_amdgcn_alignbit(0u, w.x, r);
  v.d1 = __builtin_amdgcn_alignbit(w.x, w.y, r);
  v.d2 = __builtin_amdgcn_alignbit(w.y, w.z, r);
  v.d3 = __builtin_amdgcn_alignbit(w.z, w.w, r);
  v.d4 = __builtin_amdgcn_alignbit(w.w, w4, r);
  return v;
}

// Advance the window by 32 - (q & 31) bits (v_alignbit reads the low 5 bits of q).
__device__ __forceinline__ void win_shift(Win& v, uint32_t q) {
  v.d0 = __builtin_amdgcn_alignbit(v.d0, v.d1, q);
  v.d1 = __builtin_amdgcn_alignbit(v.d1, v.d2, q);
  v.d2 = __builtin_amdgcn_alignbit(v.d2, v.d3, q);
  v.d3 = __builtin_amdgcn_alignbit(v.d3, v.d4, q);
  v.d4 = __builtin_amdgcn_alignbit(v.d4, 0u, q);
}

// Gap nibble `nib` of a gap word (8 nibbles per word, low nibble first:
// decoder.cu:501-507).
__device__ __forceinline__ uint32_t gap_nib(uint32_t word, uint32_t nib) { return (word >> (4u * (nib & 7u))) & 15u; }

// Inclusive wave scan on the VALU with DPP: row_shr 1/2/4/8 scans each 16-lane row,
// row_bcast 15/31 carry the row totals forward (no LDS traffic, unlike
// ds_bpermute-based shuffles).
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
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

// Look-back granule: [37:0] value, [39:38] flag (1 aggregate, 2 prefix), [63:40] epoch
// of the launch that wrote it (the data is the flag: no memset between launches).
constexpr unsigned long long GRAN_VMASK = (1ull << 38) - 1;
__device__ __forceinline__ unsigned long long granule(unsigned epoch, unsigned flag, unsigned long long v) {
  return ((unsigned long long)epoch << 40) | ((unsigned long long)flag << 38) | (v & GRAN_VMASK);
}

// ---- LDS at absolute byte addresses ------------------------------------------------
// The decode kernels declare no static LDS, so the dynamic LDS starts at address 0
// (each kernel checks it and flags GH_ST_LAYOUT otherwise).  Inline ds_* instructions:
// a generic or volatile pointer would be compiled to flat accesses that wait for every
// outstanding global load and store of the wave (vmcnt(0)).
__device__ __forceinline__ uint32_t lds_u32_nowait(uint32_t a) {
  uint32_t v;
  asm volatile("ds_read_b32 %0, %1" : "=v"(v) : "v"(a) : "memory");
  return v;
}
__device__ __forceinline__ uint2 lds_u64_nowait(uint32_t a) {
  uint2 v;
  asm volatile("ds_read_b64 %0, %1" : "=v"(v) : "v"(a) : "memory");
  return v;
}
// One wait for the U (1-4) independent reads of a lookup step, tied to their results so the
// compiler cannot use them before it.
template <int U, class T>
__device__ __forceinline__ void lds_wait(T (&v)[U]) {
  static_assert(U >= 1 && U <= 4, "lds_wait: 1 to 4 reads");
  if constexpr (U == 1) {
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v[0])::"memory");
  } else if constexpr (U == 2) {
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v[0]), "+v"(v[1])::"memory");
  } else if constexpr (U == 3) {
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2])::"memory");
  } else {
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3])::"memory");
  }
}
__device__ __forceinline__ uint4 lds_u128(uint32_t a) {
  uint4 v;
  asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a) : "memory");
  return v;
}

// Flag GH_ST_LAYOUT when the dynamic LDS does not start at address 0.
__device__ __forceinline__ void check_lds_base(const uint8_t* smem, unsigned int* status) {
  if (threadIdx.x == 0 && (uint32_t)(size_t)(const __attribute__((address_space(3))) uint8_t*)smem != 0u)
    atomicOr(status, (unsigned)GH_ST_LAYOUT);
}

}  // namespace gh
