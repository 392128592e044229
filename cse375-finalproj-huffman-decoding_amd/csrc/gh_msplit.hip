// Multi-symbol split decode ("msplit"), included by gh_decode.hip.
//
// For complete codes whose codewords all fit the LUT width K (maxlen <= K <= 12):
// short-code streams (redundancy 0.5 / 0.9 in BASELINE.json) where one K-bit lookup
// yields up to four symbols.  Two kernels, no inter-workgroup waiting:
//
//   gh_ms_count_kernel  counts the codewords of every segment (1 byte each) and the
//                       symbol total of every workgroup's contiguous tile range;
//   gh_ms_write_kernel  offsets its range by the totals of the ranges before it,
//                       decodes each tile again, writes every lookup's symbols as one
//                       unaligned ds_write_b32 into LDS staging at the known segment
//                       offset, and copies the tile out with aligned 16-byte stores.
//
// Reference counterpart: the count / scan / decode passes of gpu_dec_l1_l2
// (decoder.cu:529-728), whose segment rule is kept: segment i decodes the codewords
// that start in [128i + gap[i-1], 128(i+1)).  Because gap[i] is the end bit (minus
// 128) of the codeword crossing the boundary, those are exactly the codewords lying
// wholly inside [start_i, E_i), E_i = 128 + gap[i] (segment-relative): the count
// pass counts codeword ENDS <= E_i, with no per-codeword "starts before 128" test.
//
// Per lookup the loops do: window (v_alignbit), address (v_lshrrev + v_and_or), one
// ds_read_b64, and
//   count: popcount(end mask & allowed-ends mask) accumulated with v_bcnt, the
//          allowed mask shifted by the consumed bits (v_ashrrev: its sign bit keeps
//          "all allowed" while more than 32 bits remain), q -= b;
//   write: ds_write_b32 of the four symbol bytes at ptr (lanes still inside their
//          segment), ptr += n (SDWA byte add), q -= meta (low 5 bits = b).
// The window is the 160-bit funnel Win; GL lookups share one 32-bit window before
// the funnel shifts (GL * K <= 31 bits).
//
// Staging writes are aligned ds_or_b32 pairs into a zeroed buffer (the lookup's
// four bytes shifted to the byte offset, low and high dword): unaligned
// ds_write_b32 measured about 3x the LDS time of aligned ones in this kernel.  OR
// needs no coordination between segments: a LUT entry's unused bytes are zero, and
// the symbols a segment's last lookup decodes past its end are the next segment's
// first symbols (the stream is contiguous and E is a codeword boundary), written
// with the same values at the same positions.  The copy-out zeroes what it read.

constexpr int TB_MS = 256;  // workgroup size of both kernels
constexpr int U_MS = 2;     // segments per thread (lock-step chains), count kernel
// write kernel: 1 or 2 chains per thread (512 or 256 threads), the same 512-segment
// tiles; the host picks per LUT width (ms_write_chains)
constexpr int MS_TILE = U_MS * TB_MS;
// lookups per funnel shift: G * K <= 31 (template parameter GL of the kernels)
inline int ms_group(uint32_t K) { return K <= 7 ? 4 : K <= 10 ? 3 : 2; }

struct MsParams {
  const uint32_t* payload;       // local segment j owns words [4j, 4j+4); +1 look-ahead, zero padded
  const uint32_t* gaps;          // nibble gap_nib0 + j - 1: start of segment j >= 1; gap_nib0 + j: its end
  const uint2* lut;              // count: {b, end mask}; write: {symbols, b | n << 8}; 2^K entries
  uint8_t* seg_cnt;              // codewords per segment
  unsigned long long* wg_tot;    // symbols per count-kernel workgroup range
  uint8_t* out;
  unsigned int* status;
  unsigned long long* total;
  unsigned long long out_cap;
  uint32_t nseg, ntiles, gap_nib0, first_start, kbits, lut_bytes, stage_bytes, count_per;
  uint32_t last_end;             // != 0: end of the stream's last segment (= local segment nseg-1)
  uint32_t ablate;               // diagnostics only (GH_ABLATE): 1 aligned writes, 2 no writes, 4 no copy-out, 8 no fix-up
};

// LDS reads/writes at absolute LDS byte addresses (these kernels declare no static
// LDS, so the dynamic LUT starts at address 0; checked at kernel start).
__device__ __forceinline__ uint2 ms_lds_u64(uint32_t a) {
  uint2 v;
  asm volatile("ds_read_b64 %0, %1" : "=v"(v) : "v"(a) : "memory");
  return v;
}
template <int U>
__device__ __forceinline__ void ms_wait(uint2 (&v)[U]) {
  static_assert(U == 1 || U == 2 || U == 4, "ms_wait: 1, 2 or 4 lookups");
  if constexpr (U == 1) {
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v[0]) :: "memory");
  } else if constexpr (U == 2) {
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v[0]), "+v"(v[1]) :: "memory");
  } else {
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]) :: "memory");
  }
}
// OR the four bytes v into LDS at byte address a (any alignment): two aligned
// ds_or_b32 (the high dword gets the bytes shifted out; zero when a is aligned).
__device__ __forceinline__ void ms_lds_or_bytes(uint32_t a, uint32_t v) {
  const uint32_t s = a << 3;                                   // low 5 bits: 8 * (a & 3)
  const uint32_t lo = v << (s & 31u);
  const uint32_t hi = __builtin_amdgcn_ubfe(v, (32u - s) & 31u, s & 31u);  // width 0 -> 0
  asm volatile("ds_or_b32 %0, %1" :: "v"(a & ~3u), "v"(lo) : "memory");
  if (hi) asm volatile("ds_or_b32 %0, %1 offset:4" :: "v"(a & ~3u), "v"(hi) : "memory");  // bytes crossed over
}
// ptr += byte 1 of meta (n), one SDWA add
__device__ __forceinline__ uint32_t ms_add_n(uint32_t ptr, uint32_t meta) {
  uint32_t r;
  asm("v_add_u32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1"
      : "=v"(r) : "v"(ptr), "v"(meta));
  return r;
}

__device__ __forceinline__ uint32_t ms_nib(uint32_t word, uint32_t nib) { return (word >> (4u * (nib & 7u))) & 15u; }

// Words and gap words of the tile's segments (loads clamped, never skipped).
template <int U, int TBK>
__device__ __forceinline__ void ms_load(const MsParams& p, uint32_t tile, int tid, uint4 (&w)[U],
                                        uint32_t (&w4)[U], uint32_t (&ga)[U], uint32_t (&gb)[U]) {
  const uint32_t t = min(tile, p.ntiles - 1);
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint32_t seg = t * (uint32_t)(U * TBK) + (uint32_t)(u * TBK + tid);
    const uint32_t sc = min(seg, p.nseg - 1);
    w[u] = *(const uint4*)(p.payload + 4ull * sc);
    w4[u] = p.payload[4ull * sc + 4];
    ga[u] = p.gaps[(p.gap_nib0 + (sc ? sc - 1u : 0u)) >> 3];
    gb[u] = p.gaps[(p.gap_nib0 + sc) >> 3];
  }
}

// LUT to LDS (16-byte chunks; lut_bytes is a multiple of 16).
template <int TBK>
__device__ __forceinline__ void ms_lut_to_lds(const MsParams& p, uint8_t* smem, int tid) {
  const uint4* g = (const uint4*)p.lut;
  uint4* s4 = (uint4*)smem;
  for (uint32_t i = tid; i < p.lut_bytes / 16; i += TBK) s4[i] = g[i];
}

__device__ __forceinline__ void ms_shift(Win& v, uint32_t q) {
  v.d0 = __builtin_amdgcn_alignbit(v.d0, v.d1, q);
  v.d1 = __builtin_amdgcn_alignbit(v.d1, v.d2, q);
  v.d2 = __builtin_amdgcn_alignbit(v.d2, v.d3, q);
  v.d3 = __builtin_amdgcn_alignbit(v.d3, v.d4, q);
  v.d4 = __builtin_amdgcn_alignbit(v.d4, 0u, q);
}

// allowed-ends mask for R bits left: bit e-1 set for ends e <= R (all ones if R >= 32).
// R is clamped to >= 1: a finished segment then allows an end at offset 1 only,
// which no codeword has (the path requires minlen >= 2).
__device__ __forceinline__ uint32_t ms_rmask(int R) {
  return 0xFFFFFFFFu >> (32u - (uint32_t)min(max(R, 1), 32));
}

template <int U, int TBK, int GL>
__global__ __launch_bounds__(TBK) void gh_ms_count_kernel(const MsParams p) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int tid = threadIdx.x;
  const uint32_t sh = 29u - p.kbits;                       // index bits -> byte offset of a u64 entry
  const uint32_t amask = ((1u << p.kbits) - 1u) << 3;
  uint32_t t0, t1;
  t0 = (uint32_t)(((unsigned long long)blockIdx.x * p.ntiles) / gridDim.x);
  t1 = (uint32_t)(((unsigned long long)(blockIdx.x + 1) * p.ntiles) / gridDim.x);
  uint4 w[U];
  uint32_t w4[U], ga[U], gb[U];
  if (t0 < t1) ms_load<U, TBK>(p, t0, tid, w, w4, ga, gb);
  ms_lut_to_lds<TBK>(p, smem, tid);
  if (tid == 0 && (uint32_t)(size_t)(const __attribute__((address_space(3))) uint8_t*)smem != 0u)
    atomicOr(p.status, (unsigned)GH_ST_LAYOUT);
  __syncthreads();
  unsigned long long wg_total = 0;  // summed by every thread, reduced at the end
  for (uint32_t t = t0; t < t1; ++t) {
    Win v[U];
    int R[U];
    uint32_t cnt[U];
    bool act[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t seg = t * (uint32_t)(U * TBK) + (uint32_t)(u * TBK + tid);
      act[u] = seg < p.nseg;
      const int start = seg == 0 ? (int)p.first_start : (int)ms_nib(ga[u], p.gap_nib0 + seg - 1u);
      // the stream's last segment: the codewords starting before bit 128 (its
      // zero padding decodes like the reference's), ending at last_end
      const int E = (p.last_end && seg == p.nseg - 1u) ? (int)p.last_end
                                                       : 128 + (int)ms_nib(gb[u], p.gap_nib0 + seg);
      v[u] = make_win(w[u], w4[u], start);
      R[u] = act[u] ? E - start : 0;
      cnt[u] = 0;
    }
    if (t + 1 < t1) ms_load<U, TBK>(p, t + 1, tid, w, w4, ga, gb);  // prefetch
    for (int g = 0; g < 160; ++g) {
      uint32_t rm[U], q[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        rm[u] = ms_rmask(R[u]);
        q[u] = 32u;
      }
#pragma unroll
      for (int j = 0; j < GL; ++j) {
        uint2 e[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const uint32_t x = j == 0 ? v[u].d0 : __builtin_amdgcn_alignbit(v[u].d0, v[u].d1, q[u]);
          e[u] = ms_lds_u64((x >> sh) & amask);
        }
        ms_wait(e);
#pragma unroll
        for (int u = 0; u < U; ++u) {
          cnt[u] = __builtin_popcount(e[u].y & rm[u]) + cnt[u];
          rm[u] = (uint32_t)((int)rm[u] >> e[u].x);
          q[u] -= e[u].x;
        }
      }
      bool more = false;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        ms_shift(v[u], q[u]);
        R[u] -= 32 - (int)q[u];
        more |= R[u] > 0;
      }
      if (!__any(more)) break;
    }
    const unsigned long long seg0 = (unsigned long long)t * (U * TBK) + tid;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (act[u]) p.seg_cnt[seg0 + (unsigned long long)u * TBK] = (uint8_t)cnt[u];
      wg_total += act[u] ? cnt[u] : 0u;
    }
  }
  // workgroup total: wave sums, then LDS (reuses the LUT area after a barrier)
  wg_total = wave_sum_u64(wg_total);
  __syncthreads();
  unsigned long long* s_red = (unsigned long long*)smem;
  if ((tid & 63) == 0) s_red[tid >> 6] = wg_total;
  __syncthreads();
  if (tid == 0) {
    unsigned long long s = 0;
    for (int q2 = 0; q2 < TBK / 64; ++q2) s += s_red[q2];
    p.wg_tot[blockIdx.x] = s;
  }
}

template <int U, int TBK, int GL>
__global__ __launch_bounds__(TBK) void gh_ms_write_kernel(const MsParams p) {
  constexpr int NWAVE = TBK / 64;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  uint8_t* s_stage = smem + p.lut_bytes;
  uint32_t* s_wsum = (uint32_t*)(s_stage + p.stage_bytes);          // [U][NWAVE]
  unsigned long long* s_base = (unsigned long long*)(s_wsum + U * NWAVE + 2);  // [NWAVE] (8-B aligned)
  const uint32_t sh = 29u - p.kbits;
  const uint32_t amask = ((1u << p.kbits) - 1u) << 3;
  uint32_t t0, t1;
  t0 = (uint32_t)(((unsigned long long)blockIdx.x * p.ntiles) / gridDim.x);
  t1 = (uint32_t)(((unsigned long long)(blockIdx.x + 1) * p.ntiles) / gridDim.x);
  uint4 w[U];
  uint32_t w4[U], ga[U], gb[U], c8[U];
  auto load_counts = [&](uint32_t t) {
    const uint32_t tt = min(t, p.ntiles - 1);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t seg = tt * (uint32_t)(U * TBK) + (uint32_t)(u * TBK + tid);
      c8[u] = p.seg_cnt[min(seg, p.nseg - 1)];
    }
  };
  if (t0 < t1) {
    ms_load<U, TBK>(p, t0, tid, w, w4, ga, gb);
    load_counts(t0);
  }
  {  // output offset of this range: the count totals of the ranges before it
    unsigned long long b = 0;
    const uint32_t nb = blockIdx.x * p.count_per;
    for (uint32_t i = tid; i < nb; i += TBK) b += p.wg_tot[i];
    b = wave_sum_u64(b);
    if (lane == 0) s_base[wid] = b;
  }
  ms_lut_to_lds<TBK>(p, smem, tid);
  for (uint32_t i = tid; i < p.stage_bytes / 16; i += TBK) ((uint4*)s_stage)[i] = make_uint4(0, 0, 0, 0);
  if (tid == 0 && (uint32_t)(size_t)(const __attribute__((address_space(3))) uint8_t*)smem != 0u)
    atomicOr(p.status, (unsigned)GH_ST_LAYOUT);
  __syncthreads();
  unsigned long long goff = 0;
#pragma unroll
  for (int q2 = 0; q2 < NWAVE; ++q2) goff += s_base[q2];
  const uint32_t stage0 = p.lut_bytes;  // absolute LDS address of the staging buffer
  for (uint32_t t = t0; t < t1; ++t) {
    int start[U];
    uint32_t cc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t seg = t * (uint32_t)(U * TBK) + (uint32_t)(u * TBK + tid);
      start[u] = seg == 0 ? (int)p.first_start : (int)ms_nib(ga[u], p.gap_nib0 + seg - 1u);
      cc[u] = seg < p.nseg ? c8[u] : 0u;
    }
    uint4 wc[U];
    uint32_t w4c[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      wc[u] = w[u];
      w4c[u] = w4[u];
    }
    if (t + 1 < t1) {  // prefetch the next tile
      ms_load<U, TBK>(p, t + 1, tid, w, w4, ga, gb);
      load_counts(t + 1);
    }
    // tile-local offsets: wave scans, then the wave totals through LDS
    uint32_t bpos[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t incl = wave_incl_scan(cc[u], lane);
      if (lane == 63) s_wsum[u * NWAVE + wid] = incl;
      bpos[u] = incl - cc[u];
    }
    __syncthreads();  // wave sums; the previous tile's copy-out is done
    uint32_t ttot = 0, ctot[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      uint32_t add = ttot;
      ctot[u] = 0;
#pragma unroll
      for (int q2 = 0; q2 < NWAVE; ++q2) {
        const uint32_t x = s_wsum[u * NWAVE + q2];
        add += (q2 < wid) ? x : 0u;
        ctot[u] += x;
      }
      ttot += ctot[u];
      bpos[u] += add;
    }
    // A tile whose bytes exceed the staging (rare: the staging is sized for typical
    // tiles so that four workgroups fit a CU) is staged one chain (TBK contiguous
    // segments) at a time.
    const uint32_t nh = ttot + 64u <= p.stage_bytes ? 1u : (uint32_t)U;
    uint32_t hoff = 0;  // tile bytes before this half
    for (uint32_t h = 0; h < nh; ++h) {
      const uint32_t hbytes = nh == 1 ? ttot : ctot[h];
      if (h > 0) __syncthreads();  // the previous half's copy-out is done
      const uint32_t lb = (uint32_t)(goff & 15);
      // staging byte 16 + lb + i = byte i of this half, so staging chunk c <-> output
      // bytes [goff - lb - 16 + 16c, +16): aligned 16-byte copies
      Win v[U];
      uint32_t ptr[U], end[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const bool on = nh == 1 || (uint32_t)u == h;
        v[u] = make_win(wc[u], w4c[u], start[u]);
        // a chain not staged in this half gets ptr == end == 0: it never writes, and
        // its ptr only grows (bpos - hoff would wrap below zero for chain 0 in half 1)
        ptr[u] = on ? stage0 + 16u + lb + bpos[u] - hoff : 0u;
        end[u] = on ? ptr[u] + cc[u] : 0u;
      }
      for (int g = 0; g < 160; ++g) {
        uint32_t q[U];
#pragma unroll
        for (int u = 0; u < U; ++u) q[u] = 32u;
#pragma unroll
        for (int j = 0; j < GL; ++j) {
          uint2 e[U];
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const uint32_t x = j == 0 ? v[u].d0 : __builtin_amdgcn_alignbit(v[u].d0, v[u].d1, q[u]);
            e[u] = ms_lds_u64((x >> sh) & amask);
          }
          ms_wait(e);
#pragma unroll
          for (int u = 0; u < U; ++u) {
            if (!(p.ablate & 2) && ptr[u] < end[u]) ms_lds_or_bytes(ptr[u], e[u].x);
            ptr[u] = ms_add_n(ptr[u], e[u].y);
            q[u] -= e[u].y;
          }
        }
        bool more = false;
#pragma unroll
        for (int u = 0; u < U; ++u) {
          ms_shift(v[u], q[u]);
          more |= ptr[u] < end[u];
        }
        if (!__any(more)) break;
      }
      __syncthreads();  // staged
      // copy out chunks [1, nz) (chunk 0 precedes the bytes), zero [0, nz + 1) (the
      // last segment may spill past the end); four chunks per thread in flight
      const unsigned long long a0 = goff - lb;
      const unsigned long long oend = min(goff + hbytes, p.out_cap);
      const uint32_t nz = (16u + lb + hbytes + 15u) >> 4;
      uint4* st4 = (uint4*)s_stage;
      for (uint32_t c0 = tid; c0 < nz + 1u; c0 += 4u * TBK) {
        uint4 d[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const uint32_t c = c0 + (uint32_t)i * TBK;
          d[i] = c < nz + 1u ? st4[c] : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const uint32_t c = c0 + (uint32_t)i * TBK;
          if (c < nz + 1u) st4[c] = make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const uint32_t c = c0 + (uint32_t)i * TBK;
          const unsigned long long gs = a0 - 16 + 16ull * c;
          if (c == 0 || c >= nz + 1u || gs >= oend || (p.ablate & 4)) continue;
          if (gs >= goff && gs + 16 <= oend) {
            *(uint4*)(p.out + gs) = d[i];
          } else {
            const uint32_t wv[4] = {d[i].x, d[i].y, d[i].z, d[i].w};
#pragma unroll
            for (int k = 0; k < 16; ++k) {
              const unsigned long long ga2 = gs + k;
              if (ga2 >= goff && ga2 < oend) p.out[ga2] = (uint8_t)(wv[k >> 2] >> (8 * (k & 3)));
            }
          }
        }
      }
      goff += hbytes;
      hoff += hbytes;
    }
  }
  if (blockIdx.x == gridDim.x - 1 && tid == 0) *p.total = goff;
}
