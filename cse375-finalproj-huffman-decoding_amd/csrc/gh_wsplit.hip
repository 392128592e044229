// Wave split: the decode of every code that is not grouped (gh_tile.hip), included by
// gh_decode.hip.  Reference counterpart: the count / scan / decode passes of
// gpu_dec_l1_l2 (decoder/src/decoder.cu:529-728), whose segment rule is kept: segment i
// decodes the codewords that start in [128i + gap[i-1], 128(i+1)).  Because gap[i] is the
// end bit (minus 128) of the codeword crossing the boundary, those are exactly the
// codewords lying wholly inside [start_i, E_i), E_i = 128 + gap[i] (segment-relative).
//
// Two decode passes as in the reference, but no workgroup barrier and no
// inter-workgroup wait inside either pass.  The unit of work is a wave block: U chains x
// 64 consecutive segments (lane l of chain u owns segment 64u + l of the block).  The
// blocks are cut into `nranges` contiguous ranges (range r = blocks [r*nb/R,
// (r+1)*nb/R)), one per wave of the write grid; a wave of the count grid takes ranges w,
// w + W, ...  (An atomic ticket per block measured ~0.4 ms per kernel on cfg2: one
// counter serves ~90 M tickets/s.  A scan over one total per block was latency-bound:
// 363 K totals on cfg5.)
//
//   gh_ws_count_kernel  counts the codewords of every segment (1 byte per segment)
//                       and each range's symbol total;
//   gh_ws_scan_kernel   one workgroup: exclusive scan of the range totals -> the
//                       output offset of every range, and the stream total (replaces
//                       the decoupled look-back, decoder.cu:571-653);
//   gh_ws_write_kernel  decodes each block again, ORs every lookup's four symbol bytes
//                       into the wave's own LDS staging at the scanned offset, and
//                       copies the block out with 16-byte stores aligned to the
//                       output address, re-zeroing the staging as it reads it.
//
// A wave never waits for another wave: it scans its block's counts with DPP, stages
// and copies out alone (LDS operations of one wave complete in order), and its stores
// drain while it decodes the next block.  The tables (gh_lut.hpp) hold up to four
// codewords per write lookup; codewords longer than a table and patterns outside an
// incomplete code go through the canonical fallback (template parameter FB).

#ifndef GH_WS_TB
#define GH_WS_TB 512
#endif
constexpr int WS_TB = GH_WS_TB;  // threads per workgroup of the write kernel
#ifndef GH_WS_TBC
#define GH_WS_TBC 256
#endif
constexpr int WS_TBC = GH_WS_TBC;  // threads per workgroup of the count kernel
constexpr int WS_U = 2;     // chains per lane of the write kernel (segments per lane per block)
#ifndef GH_WS_UC
#define GH_WS_UC 4
#endif
constexpr int WS_UC = GH_WS_UC;  // chains per lane of the count kernel
static_assert(GH_WS_UC <= 4, "seg_cnt padding (WS_CNT_PAD) covers a last block of at most 4 chains");
constexpr int WS_SB = 256;  // segments per superblock: ranges are cut at superblock edges
constexpr int WS_SCAN_TB = 1024;
#ifndef GH_WS_PRIO
#define GH_WS_PRIO 4  // rotate s_setprio over 4 workgroup slots by block (0: off); cfg3 0.579 -> 0.565 ms
#endif
// Workgroups dispatched later to a CU lose issue-arbitration ties to earlier ones (age
// order), so with static ranges the later slots finish last; rotating the priority by
// block gives every slot the lead in turn.  Slot = blockIdx / (grid / slots).
#if GH_WS_PRIO
#define WS_PRIO(blk, b, g)                                                            \
  do {                                                                                \
    const uint32_t slot_ = (b) / max(1u, (g) / (uint32_t)GH_WS_PRIO);                 \
    switch (((blk) + slot_) % (uint32_t)GH_WS_PRIO) {                                 \
      case 0: __builtin_amdgcn_s_setprio(0); break;                                   \
      case 1: __builtin_amdgcn_s_setprio(1); break;                                   \
      case 2: __builtin_amdgcn_s_setprio(2); break;                                   \
      default: __builtin_amdgcn_s_setprio(3); break;                                  \
    }                                                                                 \
  } while (0)
#else
#define WS_PRIO(blk, b, g) do {} while (0)
#endif

constexpr uint32_t WS_CNT_PAD = 64 * 4;  // seg_cnt entries past nseg (a last block of <= 4 chains)

struct WsParams {
  const uint32_t* payload;         // local segment j owns words [4j, 4j+4); +1 look-ahead, zero padded
  const uint32_t* gaps;            // nibble gap_nib0 + j - 1: start of segment j >= 1; gap_nib0 + j: its end
  const uint2* lut;                // count: u32 {b | end mask << 16}; write: u64 {symbols, b | n << 8}
  uint8_t* seg_cnt;                // codewords per segment
  unsigned long long* rng_tot;     // symbols per range
  unsigned long long* rng_off;     // output offset per range (scan kernel)
  uint8_t* out;
  uint4* junk;                     // write kernel: 64 16-byte slots per wave for padding stores
  unsigned int* status;
  unsigned long long* total;
  unsigned long long out_cap;
  uint32_t nseg, nsb, nranges, gap_nib0, first_start, kbits, lut_bytes, stage_bytes;
  uint32_t lgc;                    // count kernel: log2 of its LUT's copies in LDS (lane l reads copy l mod 2^lgc)
  uint32_t last_end;               // != 0: end of the stream's last segment (= local segment nseg-1)
  const uint32_t* fb;              // FB kernels: canonical tables (FB_WORDS: limit16, base16, first, symbols)
  uint32_t fb_lo, fb_hi;           // their length range (minlen, maxlen)
  unsigned long long chk_pay, chk_gap, chk_out;  // GH_WS_CHECK builds: allocation sizes (words, words, bytes)
};
#ifndef GH_WS_CHECK
#define GH_WS_CHECK 0  // diagnostic builds: bounds-check every global access, flag status bits instead
#endif
#if GH_WS_CHECK
#define WS_CK(cond, bit) (((cond)) ? true : (atomicOr(p.status, (unsigned)(bit)), false))
#else
#define WS_CK(cond, bit) true
#endif

#ifndef GH_WS_NT
#define GH_WS_NT 3  // (round 4: 3) bits: 1 payload loads nontemporal (both kernels), 2 write-kernel 16-byte stores nontemporal
#endif
typedef unsigned int ws_v4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void ws_st16(uint4* d, const uint4& v) {
  if (GH_WS_NT & 2) __builtin_nontemporal_store(ws_v4u{v.x, v.y, v.z, v.w}, (ws_v4u*)d);
  else *d = v;
}
__device__ __forceinline__ uint4 ws_ld16(const uint32_t* s) {
  if (GH_WS_NT & 1) {
    const ws_v4u v = __builtin_nontemporal_load((const ws_v4u*)s);
    return make_uint4(v.x, v.y, v.z, v.w);
  }
  return *(const uint4*)s;
}

// Blocks [b0, b1) of 64*U segments of range r (ranges are cut at superblock edges, so
// kernels with different U cover the same segments).
template <int U>
__device__ __forceinline__ void ws_range(const WsParams& p, uint32_t r, uint32_t& b0, uint32_t& b1) {
  constexpr uint32_t BPS = WS_SB / (64 * U);
  const uint32_t s0 = (uint32_t)((unsigned long long)r * p.nsb / p.nranges);
  const uint32_t s1 = (uint32_t)((unsigned long long)(r + 1) * p.nsb / p.nranges);
  const uint32_t nb = (p.nseg + 64 * U - 1) / (64 * U);
  b0 = min(s0 * BPS, nb);
  b1 = min(s1 * BPS, nb);
}

// Words and gap words of block `blk` for this lane (loads clamped, never skipped).
template <int U>
__device__ __forceinline__ void ws_load(const WsParams& p, uint32_t blk, int lane, uint4 (&w)[U],
                                        uint32_t (&w4)[U], uint32_t (&ga)[U], uint32_t (&gb)[U]) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint32_t seg = blk * (uint32_t)(64 * U) + (uint32_t)(64 * u + lane);
    const uint32_t sc = min(seg, p.nseg - 1);
    if (WS_CK(4ull * sc + 5 <= p.chk_pay || !GH_WS_CHECK, 0x100)) {
      w[u] = ws_ld16(p.payload + 4ull * sc);
      w4[u] = p.payload[4ull * sc + 4];
    }
    if (WS_CK(((p.gap_nib0 + sc) >> 3) < p.chk_gap || !GH_WS_CHECK, 0x200)) {
      ga[u] = p.gaps[(p.gap_nib0 + (sc ? sc - 1u : 0u)) >> 3];
      gb[u] = p.gaps[(p.gap_nib0 + sc) >> 3];
    }
  }
}

template <int TBK>
__device__ __forceinline__ void ws_lut_to_lds(const WsParams& p, uint8_t* smem, int tid) {
  const uint4* g = (const uint4*)p.lut;
  uint4* s4 = (uint4*)smem;
  for (uint32_t i = tid; i < p.lut_bytes / 16; i += TBK) s4[i] = g[i];
}

// Canonical decode of the codeword at the top of w16 (16 window bits) from the LDS
// tables (gh_core's Canon: limit16 / base16 / first / symbols): (symbol << 8) | length.
// Used where a LUT entry holds no codeword (the first one is longer than the table
// width, or the pattern is outside an incomplete code: then `bad`, and the longest
// length, which keeps the count and the write in step).
// allowed-ends mask for R bits left: bit e-1 set for ends e <= R; none once the segment
// is finished (R <= 0).  Without the fallback a lookup group ends its codewords at most
// GL * Kc <= 31 bits past its start, so R is clamped at 31 (v_med3 + v_bfm); with it
// (two lookups of up to 16 bits) ends reach bit 32: all ones for R >= 32.
template <bool FB>
__device__ __forceinline__ uint32_t ws_rmask(int R) {
  if constexpr (FB) {
    const uint32_t m = 0xFFFFFFFFu >> (32u - (uint32_t)min(max(R, 1), 32));
    return R > 0 ? m : 0u;
  } else {
    const uint32_t r = (uint32_t)min(max(R, 0), 31);
    return (1u << r) - 1u;
  }
}

__device__ __forceinline__ uint32_t ws_canon(const uint32_t* s_fb, uint32_t w16, uint32_t lo, uint32_t hi,
                                             uint32_t& bad) {
  const uint8_t* syms = (const uint8_t*)(s_fb + 51);
  for (uint32_t l = lo; l <= hi; ++l) {
    if (w16 < s_fb[l]) return ((uint32_t)syms[(s_fb[34 + l] + ((w16 - s_fb[17 + l]) >> (16 - l))) & 255u] << 8) | l;
  }
  bad = 1;
  return ((uint32_t)syms[0] << 8) | hi;
}
template <int TBK>
__device__ __forceinline__ void ws_fb_to_lds(const WsParams& p, uint32_t* s_fb, int tid) {
  for (uint32_t i = tid; i < (uint32_t)FB_WORDS; i += TBK) s_fb[i] = p.fb[i];
}

// The count kernel's LUT (its own width Kc <= 14, u32 entries, 4 << Kc bytes): entry
// = b | endmask << 16, b = bits of the complete codewords in the Kc-bit window (all
// of them, no cap), end-mask bit e-1 per codeword end e.  One lookup step:
//   cnt += popcount(endmask & rm)   (SDWA AND of the high half, v_bcnt)
//   rm >>= b                        (v_ashrrev reads only the low 5 bits of the entry)
//   q -= b                          (SDWA low half: q = -bits consumed in the group)
// FB: codes longer than Kc or incomplete codes; an entry with no codeword (b = 0) is
// replaced by the canonical codeword's {len, end mask 1 << (len-1)} (GL = 2 then: two
// lookups of up to 16 bits fit one 32-bit window shift).
template <int U, int TBK, int GL, bool FB = false>
__global__ __launch_bounds__(TBK) void gh_ws_count_kernel(const WsParams p) {
  static_assert(!FB || GL <= 2, "fallback lookups take up to 16 bits: two per window shift");
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  // index bits -> byte offset of a u32 entry of copy lane mod 2^lgc (the e-window's S
  // without FB; the FB kernels keep one copy)
  const uint32_t lgc = FB ? 0u : p.lgc;
  const uint32_t sh = 30u - p.kbits - lgc;
  const uint32_t amask = ((1u << p.kbits) - 1u) << (2u + lgc);
  const uint32_t laneoff = ((uint32_t)lane & ((1u << lgc) - 1u)) << 2;
  uint32_t* s_fb = (uint32_t*)(smem + (p.lut_bytes << lgc));
  uint32_t bad = 0;
  if (lgc) {  // dword i of LDS = entry i >> lgc
    uint32_t* sl = (uint32_t*)smem;
    const uint32_t* g = (const uint32_t*)p.lut;
    for (uint32_t i = tid; i < (p.lut_bytes / 4) << lgc; i += TBK) sl[i] = g[i >> lgc];
  } else {
    ws_lut_to_lds<TBK>(p, smem, tid);
  }
  if constexpr (FB) ws_fb_to_lds<TBK>(p, s_fb, tid);
  if (tid == 0 && (uint32_t)(size_t)(const __attribute__((address_space(3))) uint8_t*)smem != 0u)
    atomicOr(p.status, (unsigned)GH_ST_LAYOUT);
  __syncthreads();
  const uint32_t nw = gridDim.x * (uint32_t)(TBK / 64);
  uint4 w[U];
  uint32_t w4[U], ga[U], gb[U];
  for (uint32_t r = blockIdx.x * (uint32_t)(TBK / 64) + (uint32_t)(tid >> 6); r < p.nranges; r += nw) {
    uint32_t b0, b1;
    ws_range<U>(p, r, b0, b1);
    uint32_t tot = 0;
    if (b0 < b1) ws_load<U>(p, b0, lane, w, w4, ga, gb);
    for (uint32_t blk = b0; blk < b1; ++blk) {
      WS_PRIO(blk, blockIdx.x, gridDim.x);
      Win v[U];
      int R[U];
      uint32_t cnt[U];
      bool act[U];
  #pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t seg = blk * (uint32_t)(64 * U) + (uint32_t)(64 * u + lane);
        act[u] = seg < p.nseg;
        const int start = seg == 0 ? (int)p.first_start : (int)gap_nib(ga[u], p.gap_nib0 + seg - 1u);
        const int E = (p.last_end && seg == p.nseg - 1u) ? (int)p.last_end
                                                         : 128 + (int)gap_nib(gb[u], p.gap_nib0 + seg);
        v[u] = FB ? make_win(w[u], w4[u], start) : make_ewin(w[u], w4[u], start, sh);
        R[u] = act[u] ? E - start : 0;
        cnt[u] = 0;
      }
      ws_load<U>(p, min(blk + 1, b1 - 1), lane, w, w4, ga, gb);  // prefetch (always: fixed load count)
      for (int g = 0; g < 160; ++g) {
        uint32_t rm[U], q[U];
  #pragma unroll
        for (int u = 0; u < U; ++u) {
          rm[u] = ws_rmask<FB>(R[u]);
          q[u] = 0u;
        }
  #pragma unroll
        for (int j = 0; j < GL; ++j) {
          uint32_t e[U], xs[U];
  #pragma unroll
          for (int u = 0; u < U; ++u) {
            const uint32_t x = j == 0 ? v[u].d0 : __builtin_amdgcn_alignbit(v[u].d0, v[u].d1, q[u]);
            xs[u] = x;
            asm volatile("ds_read_b32 %0, %1" : "=v"(e[u]) : "v"(FB ? (x >> sh) & amask : (x & amask) | laneoff) : "memory");
          }
          lds_wait(e);
  #pragma unroll
          for (int u = 0; u < U; ++u) {
            if constexpr (FB) {
              if ((e[u] & 0xFFFFu) == 0u) {
                // only a lookup that starts before the segment end may flag the stream
                // (lanes past the shard end and finished segments decode stray bits)
                uint32_t b1 = 0;
                const uint32_t l = ws_canon(s_fb, xs[u] >> 16, p.fb_lo, p.fb_hi, b1) & 31u;
                bad |= ((int)(0u - q[u]) < R[u]) ? b1 : 0u;
                e[u] = l | ((1u << (l - 1u)) << 16);
              }
            }
            uint32_t m;
            asm("v_and_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD"
                : "=v"(m) : "v"(e[u]), "v"(rm[u]));
            cnt[u] = __builtin_popcount(m) + cnt[u];
            asm("v_ashrrev_i32 %0, %1, %0" : "+v"(rm[u]) : "v"(e[u]));
            asm("v_sub_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0"
                : "+v"(q[u]) : "v"(e[u]));
          }
        }
        bool more = false;
  #pragma unroll
        for (int u = 0; u < U; ++u) {
          win_shift(v[u], q[u]);  // q = -consumed (1..31 bits): v_alignbit reads q & 31 = 32 - consumed
          R[u] += (int)q[u];
          more |= R[u] > 0;
        }
        if (!__any(more)) break;
      }
      const unsigned long long seg0 = (unsigned long long)blk * (64 * U) + lane;
      // one store per chain, unconditional (segments past the shard's end land in the
      // allocation's padding): a fixed store count lets the compiler wait for the next
      // block's loads with vmcnt(U) instead of vmcnt(0) behind these stores
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (WS_CK(seg0 + 64ull * u < p.nseg + WS_CNT_PAD, 0x400)) p.seg_cnt[seg0 + 64ull * u] = (uint8_t)cnt[u];
        tot += act[u] ? cnt[u] : 0u;
      }
    }
    unsigned long long t64 = wave_sum_u64(tot);
    if (lane == 0 && WS_CK(r < p.nranges, 0x800)) p.rng_tot[r] = t64;
  }
  if (FB && __any(bad != 0) && lane == 0) atomicOr(p.status, (unsigned)GH_ST_BADCODE);
}

// Exclusive scan of the range totals (one workgroup), and the stream total.
__global__ __launch_bounds__(WS_SCAN_TB) void gh_ws_scan_kernel(const WsParams p) {
  __shared__ unsigned long long s_w[WS_SCAN_TB / 64];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const uint32_t per = (p.nranges + WS_SCAN_TB - 1) / WS_SCAN_TB;
  const uint32_t i0 = min((uint32_t)tid * per, p.nranges), i1 = min(i0 + per, p.nranges);
  unsigned long long s = 0;
  for (uint32_t i = i0; i < i1; ++i) s += p.rng_tot[i];
  unsigned long long incl = s;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const unsigned long long y = __shfl_up(incl, d, 64);
    if (lane >= d) incl += y;
  }
  if (lane == 63) s_w[wid] = incl;
  __syncthreads();
  unsigned long long base = 0, all = 0;
#pragma unroll
  for (int q = 0; q < WS_SCAN_TB / 64; ++q) {
    base += q < wid ? s_w[q] : 0ull;
    all += s_w[q];
  }
  unsigned long long run = base + incl - s;
  for (uint32_t i = i0; i < i1; ++i) {
    const unsigned long long t = p.rng_tot[i];
    p.rng_off[i] = run;
    run += t;
  }
  if (tid == 0) *p.total = all;
}

// ptr += byte 1 of meta (n, the lookup's symbols): one SDWA add.
__device__ __forceinline__ uint32_t add_n(uint32_t ptr, uint32_t meta) {
  uint32_t r;
  asm("v_add_u32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1"
      : "=v"(r) : "v"(ptr), "v"(meta));
  return r;
}

// OR the four bytes v at LDS byte address a (any alignment) into the two aligned
// dwords it spans: one 64-bit shift, two ds_or_b32, no branch (v = 0 is a no-op).
__device__ __forceinline__ void ws_lds_or4(uint32_t a, uint32_t v) {
  const unsigned long long d = (unsigned long long)v << ((a & 3u) << 3);
  asm volatile("ds_or_b32 %0, %1\n\tds_or_b32 %0, %2 offset:4" ::"v"(a & ~3u), "v"((uint32_t)d),
               "v"((uint32_t)(d >> 32))
               : "memory");
}

// Byte-exact store of staging chunk bytes [k0, k1) of one 16-byte chunk (lanes 0..15).
__device__ __forceinline__ void ws_store_bytes(uint8_t* dst, const uint4* chunk, uint32_t k0, uint32_t k1, int lane) {
  if (lane < 16 && (uint32_t)lane >= k0 && (uint32_t)lane < k1) {
    const uint8_t* b = (const uint8_t*)chunk;
    dst[lane] = b[lane];
  }
}

// NS: global store instructions per lane per staged piece (fixed, so the compiler can
// wait for the prefetched loads with vmcnt(NS + ...) instead of vmcnt(0): on gfx950
// loads and stores share one in-order counter, and a vmcnt(0) at the top of every block
// made each wave wait for its previous block's stores to be acknowledged).
// FB: an entry with no codeword (n = 0) is replaced by the canonical codeword's
// {symbol, len | 1 << 8} (tables after the staging; GL = 2 then).
template <int U, int TBK, int GL, int NS, bool FB = false>
__global__ __launch_bounds__(TBK) void gh_ws_write_kernel(const WsParams p) {
  static_assert(!FB || GL <= 2, "fallback lookups take up to 16 bits: two per window shift");
  constexpr int NWAVE = TBK / 64;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const uint32_t sh = 29u - p.kbits;  // index bits -> byte offset of a u64 entry (the e-window's S without FB)
  const uint32_t amask = ((1u << p.kbits) - 1u) << 3;
  uint32_t* s_fb = (uint32_t*)(smem + p.lut_bytes + (uint32_t)NWAVE * p.stage_bytes);
  uint32_t bad = 0;
  ws_lut_to_lds<TBK>(p, smem, tid);
  if constexpr (FB) ws_fb_to_lds<TBK>(p, s_fb, tid);
  for (uint32_t i = tid; i < (uint32_t)NWAVE * p.stage_bytes / 16; i += TBK)
    ((uint4*)(smem + p.lut_bytes))[i] = make_uint4(0, 0, 0, 0);
  if (tid == 0 && (uint32_t)(size_t)(const __attribute__((address_space(3))) uint8_t*)smem != 0u)
    atomicOr(p.status, (unsigned)GH_ST_LAYOUT);
  __syncthreads();
  const uint32_t stage0 = p.lut_bytes + (uint32_t)wid * p.stage_bytes;  // absolute LDS address
  uint4* st4 = (uint4*)(smem + stage0);
  uint4 w[U];
  uint32_t w4[U], ga[U], gb[U], c8[U];
  auto load_counts = [&](uint32_t blk) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t seg = blk * (uint32_t)(64 * U) + (uint32_t)(64 * u + lane);
      c8[u] = WS_CK(min(seg, p.nseg - 1) < p.nseg, 0x10000) ? p.seg_cnt[min(seg, p.nseg - 1)] : 0u;
    }
  };
  // one range per wave of this grid (nranges = waves of the grid)
  const uint32_t r = blockIdx.x * (uint32_t)NWAVE + (uint32_t)wid;
  uint32_t b0 = 0, b1 = 0;
  if (r < p.nranges) ws_range<U>(p, r, b0, b1);
  unsigned long long goff = 0;
  if (b0 < b1) {
    ws_load<U>(p, b0, lane, w, w4, ga, gb);
    load_counts(b0);
    const unsigned long long ro = WS_CK(r < p.nranges, 0x20000) ? p.rng_off[r] : 0ull;
    goff = rfl_u64(ro);
  }
  // Staging chunk 1 holds the output chunk containing goff.  Its bytes before goff
  // come from the previous piece of this range (carried), except at the range's start
  // where the first hs bytes belong to the previous range: that chunk is stored
  // byte-exact once, as is the range's last, partial chunk.
  uint32_t hs = (uint32_t)(goff & 15);
  const unsigned long long rs = goff;  // the range's first output byte
  uint4* junk = p.junk + ((unsigned long long)(blockIdx.x * (uint32_t)NWAVE + (uint32_t)wid) * 64u + lane);
  bool capped = false;  // the output ended at out_cap inside an earlier piece: nothing more to write
  for (uint32_t blk = b0; blk < b1 && !capped; ++blk) {
    WS_PRIO(blk, blockIdx.x, gridDim.x);
    {
      int start[U];
      uint32_t cc[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t seg = blk * (uint32_t)(64 * U) + (uint32_t)(64 * u + lane);
        start[u] = seg == 0 ? (int)p.first_start : (int)gap_nib(ga[u], p.gap_nib0 + seg - 1u);
        cc[u] = seg < p.nseg ? c8[u] : 0u;
      }
      uint4 wc[U];
      uint32_t w4c[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        wc[u] = w[u];
        w4c[u] = w4[u];
      }
      {  // prefetch the wave's next block (always issued: a fixed count of loads)
        const uint32_t nb = min(blk + 1, b1 - 1);
        ws_load<U>(p, nb, lane, w, w4, ga, gb);
        load_counts(nb);
      }
      // offsets inside the block: chain u's bytes follow chain u-1's
      uint32_t bpos[U], ctot[U], coff[U], btot = 0;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t incl = wave_incl_scan(cc[u]);
        bpos[u] = incl - cc[u];
        ctot[u] = __builtin_amdgcn_readlane(incl, 63);
        coff[u] = btot;
        btot += ctot[u];
      }
      // a block that does not fit the wave's staging is staged one chain at a time
      const uint32_t nh = btot + 64u <= p.stage_bytes ? 1u : (uint32_t)U;
      for (uint32_t h = 0; h < nh && !capped; ++h) {
        const uint32_t hbytes = nh == 1 ? btot : ctot[h];
        const uint32_t lb = (uint32_t)(goff & 15);
        // staging byte 16 + lb + i = byte i of this half: staging chunk c <-> output
        // bytes [goff - lb - 16 + 16c, +16), aligned 16-byte copies
        Win v[U];
        uint32_t ptr[U], end[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const bool on = nh == 1 || (uint32_t)u == h;
          v[u] = FB ? make_win(wc[u], w4c[u], start[u]) : make_ewin(wc[u], w4c[u], start[u], sh);
          // a chain not staged in this piece: an empty range inside the staging
          ptr[u] = on ? stage0 + 16u + lb + (nh == 1 ? coff[u] : 0u) + bpos[u] : stage0 + 4u * (uint32_t)lane;
          end[u] = on ? ptr[u] + cc[u] : ptr[u];
        }
        for (int g = 0; g < 160; ++g) {
          uint32_t q[U];
#pragma unroll
          for (int u = 0; u < U; ++u) q[u] = 32u;
#pragma unroll
          for (int j = 0; j < GL; ++j) {
            uint2 e[U];
            uint32_t xs[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
              const uint32_t x = j == 0 ? v[u].d0 : __builtin_amdgcn_alignbit(v[u].d0, v[u].d1, q[u]);
              xs[u] = x;
              e[u] = lds_u64_nowait(FB ? (x >> sh) & amask : x & amask);
            }
            lds_wait(e);
#pragma unroll
            for (int u = 0; u < U; ++u) {
              if constexpr (FB) {
                if ((e[u].y & 0x700u) == 0u) {  // n = 0
                  uint32_t b1 = 0;  // flags only a lookup whose symbol is written
                  const uint32_t r = ws_canon(s_fb, xs[u] >> 16, p.fb_lo, p.fb_hi, b1);
                  bad |= ptr[u] < end[u] ? b1 : 0u;
                  e[u] = make_uint2(r >> 8, (r & 31u) | (1u << 8));
                }
              }
              {  // branch-free: a lane past its end ORs zero at its end (inside the staging spill)
                const bool on = ptr[u] < end[u];
                ws_lds_or4(on ? ptr[u] : end[u], on ? e[u].x : 0u);
              }
              ptr[u] = add_n(ptr[u], e[u].y);
              q[u] -= e[u].y;
            }
          }
          bool more = false;
#pragma unroll
          for (int u = 0; u < U; ++u) {
            win_shift(v[u], q[u]);
            more |= ptr[u] < end[u];
          }
          if (!__any(more)) break;
        }
        // Copy out the complete chunks [c_lo, cend) of this piece: staging chunk c <->
        // output bytes [goff - lb - 16 + 16c, +16) (the OR-s above are complete: this
        // wave's LDS operations run in order).  Exactly NS store instructions per lane,
        // padded with duplicate stores; more chunks than 64 * NS (never with the host's
        // staging sizes) go through a loop of its own.
        const unsigned long long a0 = goff - lb;
        const uint32_t hb = goff + hbytes <= p.out_cap ? hbytes : (goff < p.out_cap ? (uint32_t)(p.out_cap - goff) : 0u);
        const uint32_t cend = ((lb + hb) >> 4) + 1u;  // chunks [1, cend) end inside the piece
        uint32_t c_lo = 1;
        if (hs != 0 && cend > 1u) {  // the range's first chunk is complete: its bytes [hs, 16)
          if (WS_CK(a0 + 16 <= p.chk_out || !GH_WS_CHECK, 0x1000))
            ws_store_bytes(p.out + a0, st4 + 1, hs, 16u, lane);
          c_lo = 2;
          hs = 0;
        }
        {
          // padding stores rewrite the piece's last complete chunk (same bytes: the
          // duplicate merges in L2 instead of costing an HBM write); the junk slot only
          // when the piece has no complete chunk
          const bool have = cend > c_lo;
          const uint32_t cdup = have ? cend - 1u : 0u;
#pragma unroll
          for (int i = 0; i < NS; ++i) {
            const uint32_t c = c_lo + (uint32_t)lane + 64u * (uint32_t)i;
            const bool real = c < cend;
            const uint32_t cs = real ? c : cdup;
            const uint4 d = st4[cs];
            uint4* dst = (real || have) ? (uint4*)(p.out + a0 - 16 + 16ull * cs) : junk;
            if (WS_CK(!real || a0 + 16ull * c <= p.chk_out || !GH_WS_CHECK, 0x2000)) ws_st16(dst, d);
          }
          for (uint32_t c = c_lo + (uint32_t)lane + 64u * NS; c < cend; c += 64u)
            if (WS_CK(a0 + 16ull * c <= p.chk_out || !GH_WS_CHECK, 0x4000))
              ws_st16((uint4*)(p.out + a0 - 16 + 16ull * c), st4[c]);
        }
        if (goff + hbytes >= p.out_cap) {
          // the output ends in this piece: its partial last chunk (staging chunk cend,
          // output bytes [out_cap & ~15, out_cap)) now, and no later piece writes
          const uint32_t te = (uint32_t)(p.out_cap & 15);
          if (te != 0 && p.out_cap > rs && WS_CK(p.out_cap <= p.chk_out || !GH_WS_CHECK, 0x8000))
            ws_store_bytes(p.out + (p.out_cap - te), st4 + cend, cend == 1 ? hs : 0u, te, lane);
          capped = true;
          break;
        }
        // carry the partial chunk cend to chunk 1 (the next piece's first output chunk;
        // bytes past the piece's end are that piece's first symbols, decoded here by the
        // last lookups, the same values it ORs in) and zero the rest, spill included
        const uint4 carry = st4[cend];
        const uint32_t nzero = cend + 2u;
        for (uint32_t c = lane; c < nzero; c += 64u) st4[c] = make_uint4(0, 0, 0, 0);
        if (lane == 0) st4[1] = carry;
        goff += hbytes;
      }
    }
  }
  // the range's last, partial chunk: its bytes [hs or 0, end & 15), end clamped at out_cap
  if (b0 < b1 && !capped) {
    const unsigned long long ge = min(goff, p.out_cap);
    const uint32_t te = (uint32_t)(ge & 15);
    if (te != 0 && ge > rs && WS_CK(ge <= p.chk_out || !GH_WS_CHECK, 0x8000))
      ws_store_bytes(p.out + (ge - te), st4 + 1, hs, te, lane);
  }
  if (FB && __any(bad != 0) && lane == 0) atomicOr(p.status, (unsigned)GH_ST_BADCODE);
}
