// Fused tile kernel: the count pass and the write pass of the wave split (gh_wsplit.hip)
// for codes the single-symbol tile kernel does not take (BASELINE's r = 0.9 codes: 2/3-
// and 10/11-bit codewords, ~41 per segment), in one persistent kernel that reads the
// payload ONCE.  Included by gh_decode.hip after gh_tile.hip and gh_wsplit.hip, whose
// round leader, windows, tables and LDS helpers it uses.
//
// Reference counterpart: gpu_dec_l1_l2 (decoder/src/decoder.cu:454-730): per segment a
// count of the codewords starting in it (:529-569), the scan of the counts (:571-653),
// and a second decode that writes the bytes (:655-728) -- in the reference the second
// decode re-reads the segment; here both passes decode the same words held in
// registers.
//
// 512-thread workgroups, U segments per lane (tile = U * 512 consecutive segments, chain
// u of wave w lane l = segment tile_base + 512u + 64w + l).  Workgroup 0 is the round
// leader of gh_tile.hip; the others take tiles b, b + D, ... (static round robin).
// Iteration of a decoding workgroup, tile t:
//   count pass: every chain counts its segment's codewords (end-mask LUT, wave split's
//     count kernel) -> wave scans -> BARRIER -> tile total published at once (the leader
//     resolves the tile's prefix while the write pass runs);
//   the next tile's words are loaded into a second register set;
//   write pass: the same words decoded again with the four-symbol LUT, every lookup's
//     symbol bytes ORed into the tile's staging at its scanned offset -> BARRIER;
//   copy-out: wait for the tile's prefix, copy the staging to the output with 16-byte
//     stores; every thread re-zeroes exactly the staging bytes it read (and thread 0 the
//     <= 3 bytes the last lookups ORed past the tile), so the next tile's ORs need no
//     further barrier.
// One staging buffer (the copy-out follows the write pass in the same iteration): a
// 1024-segment tile of r = 0.9 data is ~42 KB.  A tile larger than the staging waits
// for its own prefix and stores its bytes from the write pass directly (byte stores).

#ifndef GH_FT_U
#define GH_FT_U 2
#endif
constexpr int FT_U = GH_FT_U;    // segments per lane
constexpr int FT_TB = 512;
constexpr int FT_PAD = 16;       // staging byte FT_PAD + i = tile byte i

typedef unsigned int ft_v4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void lds_zero16(uint32_t a) {
  asm volatile("ds_write_b128 %0, %1" ::"v"(a), "v"(ft_v4u{0u, 0u, 0u, 0u}) : "memory");
}

// Copy-out of the fused kernel: like copy_out_tile, plus the zeroing of what was read.
template <int TBK, int NS>
__device__ __forceinline__ void ft_copy_out(uint8_t* out, uint32_t stg, unsigned long long goff, uint32_t n,
                                            uint32_t total, int tid, uint4* junk) {
  const uint32_t lb = (uint32_t)(goff & 15);
  uint8_t* o = out + (goff - lb);
  const uint32_t src = stg + (uint32_t)FT_PAD - lb;  // staging address of output chunk 0
  const uint32_t cf = lb ? 1u : 0u;
  const uint32_t ce = n ? (lb + n) >> 4 : 0u;
  const bool have = ce > cf;
  // A fixed NS stores per thread; a store past the tile rewrites the thread's own first
  // chunk from its register (another thread's chunk may already be re-zeroed in LDS).
  const uint32_t c0 = cf + (uint32_t)tid;
  const bool real0 = c0 < ce;
  const uint4 v0 = lds_u128(src + 16u * (real0 ? c0 : cf));
  uint4* const d0 = real0 ? (uint4*)(o + 16ull * c0) : junk;
  *d0 = v0;
  if (real0) lds_zero16(src + 16u * c0);
#pragma unroll
  for (int i = 1; i < NS; ++i) {
    const uint32_t c = c0 + (uint32_t)(TBK * i);
    uint4 v = v0;
    uint4* d = d0;
    if (c < ce) {
      v = lds_u128(src + 16u * c);
      d = (uint4*)(o + 16ull * c);
      lds_zero16(src + 16u * c);
    }
    *d = v;
  }
  (void)have;
  for (uint32_t c = cf + (uint32_t)tid + (uint32_t)(TBK * NS); c < ce; c += TBK) {
    *(uint4*)(o + 16ull * c) = lds_u128(src + 16u * c);
    lds_zero16(src + 16u * c);
  }
  // edge bytes (head chunk [lb, 16), tail chunk [0, (lb + n) & 15)): one byte per thread,
  // re-zeroed by its reader
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
  (void)hb;
  uint32_t b;
  asm volatile("ds_read_u8 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(b) : "v"(src + (real ? k : 0u)) : "memory");
  *(real ? o + k : (uint8_t*)junk) = (uint8_t)b;
  if (real) asm volatile("ds_write_b8 %0, %1" ::"v"(src + k), "v"(0u) : "memory");
  // the bytes the tile's last lookups ORed past its end (at most 3; a tile clamped at
  // out_cap: every byte past n) -- nobody reads them
  if (tid == 0) {
    for (uint32_t i = n; i < total + 4u; i += 4u)
      asm volatile("ds_write_b32 %0, %1" ::"v"(stg + (uint32_t)FT_PAD + i), "v"(0u) : "memory");
  }
}

template <int U, int GLC, int GLW, int NS>
__global__ __launch_bounds__(FT_TB) __attribute__((amdgpu_waves_per_eu(4, 4))) void gh_ftile_kernel(const TileParams p) {
  constexpr int TB = FT_TB, NWAVE_T = TB / 64;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint32_t* s_wsum = (uint32_t*)(smem + p.stage_off + p.stage_bytes);  // [U][NWAVE_T]
  uint32_t* s_lead = s_wsum + U * NWAVE_T;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  if (blockIdx.x == 0) {
    tile_round_leader<TB>(p, s_lead, tid, lane, wid);
    return;
  }
  {  // tables to LDS (count LUT at 0, write LUT at lutw_off), staging zeroed
    const uint4* gc = (const uint4*)p.lut;
    uint4* sc = (uint4*)smem;
    for (uint32_t i = tid; i < p.lut_bytes / 16; i += TB) sc[i] = gc[i];
    const uint4* gw = (const uint4*)p.lutw;
    uint4* sw = (uint4*)(smem + p.lutw_off);
    for (uint32_t i = tid; i < p.lutw_bytes / 16; i += TB) sw[i] = gw[i];
    uint4* st = (uint4*)(smem + p.stage_off);
    for (uint32_t i = tid; i < p.stage_bytes / 16; i += TB) st[i] = make_uint4(0, 0, 0, 0);
  }
  check_lds_base(smem, p.status);
  __syncthreads();
  const uint32_t shc = 30u - p.kbits, amc = ((1u << p.kbits) - 1u) << 2;         // count LUT (u32)
  const uint32_t shw = 29u - p.kw, amw = ((1u << p.kw) - 1u) << 3, wbase = p.lutw_off;  // write LUT (u64)
  const uint32_t G = gridDim.x - 1, b = blockIdx.x - 1;
  const uint32_t nseg = (uint32_t)p.nseg;
  constexpr uint32_t NONE = 0xFFFFFFFFu;
  const uint32_t last_tile_k = b < p.ntiles ? (p.ntiles - 1 - b) / G : NONE;
  uint32_t cur = b, nxt = b + G;
  uint4 w[U], wn[U];
  uint32_t w4[U], ga[U], gb[U], w4n[U], gan[U], gbn[U];
  auto load = [&](uint32_t t, uint4 (&x)[U], uint32_t (&x4)[U], uint32_t (&xa)[U], uint32_t (&xb)[U]) {
    const uint32_t seg0 = min(t, p.ntiles - 1) * (uint32_t)(U * TB) + (uint32_t)tid;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t sc = min(seg0 + (uint32_t)(u * TB), nseg - 1);
      x[u] = *(const uint4*)(p.payload + 4ull * sc);
      x4[u] = p.payload[4ull * sc + 4];
      xa[u] = p.gaps[(p.gap_nib0 + (sc ? sc - 1u : 0u)) >> 3];
      xb[u] = p.gaps[(p.gap_nib0 + sc) >> 3];
    }
  };
  uint4* const jk = p.junk + (unsigned long long)blockIdx.x * TB + tid;  // junk slot i: + i * grid * TB
  load(cur, w, w4, ga, gb);
#pragma unroll
  for (int i = 0; i <= NS; ++i)  // as after every later load (see below): NS + 1 stores
    jk[(uint32_t)i * (gridDim.x * (uint32_t)TB)] = make_uint4(0, 0, 0, 0);
  if (cur >= p.ntiles) cur = NONE;
  const uint32_t stg = p.stage_off;  // absolute LDS address of the staging (kernel LDS starts at 0)
  for (uint32_t k = 0;; ++k) {
    const bool have_cur = cur < p.ntiles;
    if (!have_cur) break;
    if (last_tile_k != NONE && k > last_tile_k + 2) {  // cannot happen; never hang the GPU
      if (tid == 0) atomicOr(p.status, (unsigned)GH_ST_TIMEOUT);
      break;
    }
    // ---- count pass ------------------------------------------------------------------
    const uint32_t seg0 = cur * (uint32_t)(U * TB) + (uint32_t)tid;
    int start[U], R[U];
    uint32_t cnt[U];
    bool act[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t seg = seg0 + (uint32_t)(u * TB);
      act[u] = seg < nseg;
      start[u] = seg == 0 ? (int)p.first_start : (int)gap_nib(ga[u], p.gap_nib0 + seg - 1u);
      const int E = (p.last_end && seg == nseg - 1u) ? (int)p.last_end : 128 + (int)gap_nib(gb[u], p.gap_nib0 + seg);
      R[u] = act[u] ? E - start[u] : 0;
      cnt[u] = 0;
    }
    {
      Win v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = make_ewin(w[u], w4[u], start[u], shc);
      int Rl[U];
#pragma unroll
      for (int u = 0; u < U; ++u) Rl[u] = R[u];
      for (int g = 0; g < 160; ++g) {
        uint32_t rm[U], q[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          rm[u] = ws_rmask<false>(Rl[u]);
          q[u] = 0u;
        }
#pragma unroll
        for (int j = 0; j < GLC; ++j) {
          uint32_t e[U];
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const uint32_t x = j == 0 ? v[u].d0 : __builtin_amdgcn_alignbit(v[u].d0, v[u].d1, q[u]);
            e[u] = lds_u32_nowait(x & amc);
          }
          lds_wait(e);
#pragma unroll
          for (int u = 0; u < U; ++u) {
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
          win_shift(v[u], q[u]);
          Rl[u] += (int)q[u];
          more |= Rl[u] > 0;
        }
        if (!__any(more)) break;
      }
    }
    // ---- scans, tile total, publish --------------------------------------------------
    uint32_t bpos[U], incl[U];
#pragma unroll
    for (int u = 0; u < U; ++u) incl[u] = wave_incl_scan(cnt[u]);
    if (lane == 63) {
#pragma unroll
      for (int u = 0; u < U; ++u) s_wsum[u * NWAVE_T + wid] = incl[u];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) bpos[u] = incl[u] - cnt[u];
    __syncthreads();  // tile sums; also every read of the previous tile's staging is done
    static_assert(U * NWAVE_T <= 64, "one wave sum per lane");
    const uint32_t xs = lane < U * NWAVE_T ? s_wsum[lane] : 0u;
    const uint32_t xi = wave_incl_scan(xs);
#pragma unroll
    for (int u = 0; u < U; ++u) bpos[u] += (uint32_t)__builtin_amdgcn_readlane((int)(xi - xs), u * NWAVE_T + wid);
    const uint32_t tile_total = (uint32_t)__builtin_amdgcn_readlane((int)xi, U * NWAVE_T - 1);
    if (tid == 0)
      __hip_atomic_store(&p.granules[cur], granule(p.epoch, 1, tile_total), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned long long goff = 0;
    bool got = true;
    auto prefix = [&]() {
      if (lane == 0) {
        unsigned long long g = __hip_atomic_load(&p.prefix[cur], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (!granule_ok(p, g, 2)) {
          if (wid == 0) atomicAdd(p.stats, 1ull);
          g = poll_granule(p, &p.prefix[cur], 2);
        }
        got = granule_ok(p, g, 2);  // false only after a timeout (then nothing is written)
        goff = g & GRAN_VMASK;
        if (wid == 0 && cur == p.ntiles - 1 && got) *p.total = goff + tile_total;
      }
      goff = rfl_u64(goff);
      got = __builtin_amdgcn_readfirstlane(got ? 1 : 0) != 0;
    };
    // ---- write pass --------------------------------------------------------------------
    // ST: ORed into the staging; else (a tile larger than the staging, rare) the lookups'
    // symbols stored straight to the output, clamped at out_cap.  Two copies of the loop,
    // so that the common one holds no global store.
    auto write_pass = [&](auto st_c) {
      constexpr bool ST = decltype(st_c)::value;
      Win v[U];
      uint32_t ptr[U], end[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        v[u] = make_ewin(w[u], w4[u], start[u], shw);
        ptr[u] = stg + (uint32_t)FT_PAD + bpos[u];
        end[u] = ptr[u] + cnt[u];
      }
      for (int g = 0; g < 160; ++g) {
        uint32_t q[U];
#pragma unroll
        for (int u = 0; u < U; ++u) q[u] = 32u;
#pragma unroll
        for (int j = 0; j < GLW; ++j) {
          uint2 e[U];
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const uint32_t x = j == 0 ? v[u].d0 : __builtin_amdgcn_alignbit(v[u].d0, v[u].d1, q[u]);
            e[u] = lds_u64_nowait((x & amw) | wbase);
          }
          lds_wait(e);
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const bool on = ptr[u] < end[u];
            if constexpr (ST) {
              ws_lds_or4(on ? ptr[u] : end[u], on ? e[u].x : 0u);
            } else if (on && got) {
              const unsigned long long o = goff + (ptr[u] - stg - (uint32_t)FT_PAD);
              const uint32_t nn = min((e[u].y >> 8) & 7u, end[u] - ptr[u]);
              for (uint32_t i = 0; i < nn; ++i)
                if (o + i < p.out_cap) p.out[o + i] = (uint8_t)(e[u].x >> (8 * i));
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
    };
    // Every path issues the next tile's loads followed by exactly NS + 1 stores per
    // thread (more only in the rare copy-out tail), so the compiler waits for those loads
    // at the next count pass with vmcnt(NS + 1), not behind the stores' completion.
    if (tile_total + (uint32_t)(FT_PAD + 64) <= p.stage_bytes) {
      load(nxt, wn, w4n, gan, gbn);  // the write pass and the copy-out to arrive
      write_pass(std::integral_constant<bool, true>{});
      __syncthreads();  // the staging holds the tile
      prefix();
      const uint32_t n = (!got || goff >= p.out_cap) ? 0u : (uint32_t)min<unsigned long long>(tile_total, p.out_cap - goff);
      ft_copy_out<TB, NS>(p.out, stg, goff, n, tile_total, tid, jk);
    } else {
      prefix();
      write_pass(std::integral_constant<bool, false>{});
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the data-dependent direct stores
      __syncthreads();                     // (the staging was not touched: it stays zero)
      load(nxt, wn, w4n, gan, gbn);
#pragma unroll
      for (int i = 0; i <= NS; ++i) jk[(uint32_t)i * (gridDim.x * (uint32_t)TB)] = make_uint4(0, 0, 0, 0);
    }
    // next tile
#pragma unroll
    for (int u = 0; u < U; ++u) {
      w[u] = wn[u];
      w4[u] = w4n[u];
      ga[u] = gan[u];
      gb[u] = gbn[u];
    }
    cur = nxt < p.ntiles ? nxt : NONE;
    nxt += G;
  }
}
