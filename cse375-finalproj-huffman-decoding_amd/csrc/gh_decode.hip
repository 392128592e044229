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

#include <algorithm>
#include <cmath>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "gh_internal.hpp"

namespace gh {

constexpr int TB = 256;                  // workgroup size = segments per tile
constexpr int NWAVE = TB / 64;
constexpr int SLOT_WORDS = 5;            // 4 segment words + 1 look-ahead word
constexpr int IN_BYTES = ((4 + 4 * SLOT_WORDS * TB) + 15) & ~15;
constexpr int FB_WORDS = 3 * 17 + 64;    // limit16/base16/first + 256 symbol bytes
constexpr int FB_BYTES = ((4 * FB_WORDS) + 15) & ~15;
constexpr int SCRATCH_BYTES = 64;
constexpr uint32_t EPOCH_MAX = (1u << 24) - 1;
constexpr uint32_t SPIN_LIMIT = 1u << 22;

struct DecodeParams {
  const uint32_t* payload;       // local segment j owns words [4j, 4j+4); +1 look-ahead, zero padded
  const uint32_t* gaps;          // gap words; nibble (gap_nib0 + j - 1) = start of local segment j>=1
  const uint4* lut;              // 2^K entries as {syms, meta} pairs (8 bytes)
  const uint32_t* fb;            // fallback tables
  uint8_t* out;                  // shard output
  unsigned long long* granules;  // one per tile
  unsigned int* ticket;
  unsigned int* status;
  unsigned long long* total;     // shard symbol total (written by the last tile)
  unsigned long long out_cap;
  unsigned long long nseg;
  unsigned int gap_nib0;
  unsigned int first_start;
  unsigned int ntiles;
  unsigned int kbits;
  unsigned int epoch;
  unsigned int lut_bytes;
  unsigned int stage_bytes;
  unsigned int fb_lo, fb_hi;     // fallback length range
};

// ---- meta word of a LUT entry -------------------------------------------------
//  [2:0] n symbols (0 = fallback), [7:3] bits consumed, [11:8] e1, [15:12] e2,
//  [19:16] e3: end of symbol k = start of symbol k+1 (15 when absent).
__device__ __forceinline__ uint32_t meta_n(uint32_t m) { return m & 7u; }
__device__ __forceinline__ uint32_t meta_b(uint32_t m) { return (m >> 3) & 31u; }

// 32 stream bits starting at segment-relative bit P (P in [0,128)); slot[-1] must
// be readable.  alignbit(a,b,s) = ({a,b} >> s)[31:0]; with q = (P-1)>>5 the shift
// (-P)&31 is in [0,31] for every P, so no shift-by-32 case exists.
__device__ __forceinline__ uint32_t window32(const uint32_t* slot, int P) {
  const int q = (P - 1) >> 5;
  const uint32_t a = slot[q];
  const uint32_t b = slot[q + 1];
  return __builtin_amdgcn_alignbit(a, b, (uint32_t)(-P));
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

__device__ __forceinline__ uint32_t fetch_meta(const uint2* lut, const uint32_t* fb, uint32_t t,
                                               uint32_t kshift, const DecodeParams& p,
                                               uint32_t* syms) {
  const uint2 e = lut[t >> kshift];
  uint32_t meta = e.y;
  *syms = e.x;
  if (meta_n(meta) == 0) {
    const uint32_t r = fallback_decode(fb, t >> 16, p.fb_lo, p.fb_hi, p.status);
    *syms = r >> 8;
    meta = 1u | ((r & 31u) << 3) | 0xFFF00u;
  }
  return meta;
}

// Symbols of the final lookup that start before the segment end (rem bits left).
__device__ __forceinline__ uint32_t kept_in_last(uint32_t meta, int rem) {
  const uint32_t r = (uint32_t)min(rem, 15);
  return 1u + (((meta >> 8) & 15u) < r) + (((meta >> 12) & 15u) < r) +
         (((meta >> 16) & 15u) < r);
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, int lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t t = __shfl_up(v, d, 64);
    if (lane >= d) v += t;
  }
  return v;
}

__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
  return v;
}

// Look-back granule: [37:0] value, [39:38] flag (1 aggregate, 2 inclusive prefix),
// [63:40] epoch of the launch that wrote it.
__device__ __forceinline__ unsigned long long granule(unsigned epoch, unsigned flag,
                                                      unsigned long long v) {
  return ((unsigned long long)epoch << 40) | ((unsigned long long)flag << 38) |
         (v & ((1ull << 38) - 1));
}

__global__ __launch_bounds__(TB) void gh_decode_kernel(const DecodeParams p) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint2* s_lut = (uint2*)smem;
  uint32_t* s_fb = (uint32_t*)(smem + p.lut_bytes);
  uint32_t* s_in = (uint32_t*)(smem + p.lut_bytes + FB_BYTES);
  uint8_t* s_stage = smem + p.lut_bytes + FB_BYTES + IN_BYTES;
  uint32_t* s_scr = (uint32_t*)(s_stage + p.stage_bytes);
  // scratch: [0..3] wave sums, [4] ticket, [6..7] tile offset (u64)

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;

  // Stage the decode tables in LDS once per persistent workgroup.
  {
    const uint4* g = p.lut;
    uint4* s = (uint4*)smem;
    for (uint32_t i = tid; i < p.lut_bytes / 16; i += TB) s[i] = g[i];
    for (uint32_t i = tid; i < (uint32_t)FB_WORDS; i += TB) s_fb[i] = p.fb[i];
    uint4* st = (uint4*)s_stage;
    for (uint32_t i = tid; i < p.stage_bytes / 16; i += TB) st[i] = make_uint4(0, 0, 0, 0);
    if (tid == 0) s_in[0] = 0;
  }

  const uint32_t kshift = 32u - p.kbits;
  uint32_t* slot = s_in + 1 + SLOT_WORDS * tid;

  for (;;) {
    if (tid == 0) s_scr[4] = atomicAdd(p.ticket, 1u);
    __syncthreads();
    const uint32_t tile = s_scr[4];
    if (tile >= p.ntiles) {
      if (tid == 0 && tile == p.ntiles + gridDim.x - 1)
        __hip_atomic_store(p.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      break;
    }
    const unsigned long long seg = (unsigned long long)tile * TB + tid;
    const bool active = seg < p.nseg;

    // ---- load the segment (16 B vector load, coalesced over the wave) ----------
    int start = 0;
    if (active) {
      const uint4 w = *(const uint4*)(p.payload + 4 * seg);
      const uint32_t w4 = p.payload[4 * seg + 4];
      slot[0] = w.x;
      slot[1] = w.y;
      slot[2] = w.z;
      slot[3] = w.w;
      slot[4] = w4;
      if (seg == 0) {
        start = (int)p.first_start;
      } else {
        const unsigned long long nib = (unsigned long long)p.gap_nib0 + seg - 1;
        start = (int)((p.gaps[nib >> 3] >> (4 * (nib & 7))) & 15u);
      }
    }

    // ---- pass 1: count codewords starting inside the segment ------------------
    uint32_t cnt = 0;
    if (active) {
      int P = start, Plast = start;
      uint32_t mlast = 0;
      do {
        uint32_t syms;
        const uint32_t meta = fetch_meta(s_lut, s_fb, window32(slot, P), kshift, p, &syms);
        cnt += meta_n(meta);
        Plast = P;
        mlast = meta;
        P += (int)meta_b(meta);
      } while (P < 128);
      cnt -= meta_n(mlast) - kept_in_last(mlast, 128 - Plast);
    }

    // ---- tile scan: wave scan + cross-wave combine ------------------------------
    const uint32_t incl = wave_incl_scan(cnt, lane);
    if (lane == 63) s_scr[wid] = incl;
    __syncthreads();
    uint32_t wpre = 0, tile_total = 0;
#pragma unroll
    for (int w = 0; w < NWAVE; ++w) {
      const uint32_t v = s_scr[w];
      wpre += (w < wid) ? v : 0u;
      tile_total += v;
    }
    const uint32_t excl_local = wpre + incl - cnt;

    // ---- decoupled look-back over preceding tiles (wave 0) ----------------------
    if (wid == 0) {
      unsigned long long excl_tile = 0;
      if (tile == 0) {
        if (lane == 0)
          __hip_atomic_store(&p.granules[0], granule(p.epoch, 2, tile_total), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
      } else {
        if (lane == 0)
          __hip_atomic_store(&p.granules[tile], granule(p.epoch, 1, tile_total), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
        long long base = (long long)tile - 1;
        uint32_t spins = 0;
        for (;;) {
          const long long pi = base - lane;
          unsigned long long g = 0;
          uint32_t st = 2;  // tiles before the first count as an inclusive 0
          if (pi >= 0) {
            g = __hip_atomic_load(&p.granules[pi], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            st = ((uint32_t)(g >> 40) == p.epoch) ? (uint32_t)((g >> 38) & 3u) : 0u;
          }
          const unsigned long long pm = __ballot(st == 2);
          const unsigned long long vm = __ballot(st != 0);
          const int fp = pm ? __builtin_ctzll(pm) : 64;
          const unsigned long long need = (fp >= 63) ? ~0ull : ((2ull << fp) - 1);
          if ((vm & need) != need) {
            if (++spins > SPIN_LIMIT) {
              if (lane == 0) atomicOr(p.status, (unsigned)GH_ST_TIMEOUT);
              break;
            }
            __builtin_amdgcn_s_sleep(1);
            continue;
          }
          const unsigned long long v =
              (lane <= fp && pi >= 0) ? (g & ((1ull << 38) - 1)) : 0ull;
          excl_tile += wave_sum_u64(v);
          if (fp < 64) break;
          base -= 64;
        }
        if (lane == 0)
          __hip_atomic_store(&p.granules[tile], granule(p.epoch, 2, excl_tile + tile_total),
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (lane == 0) {
        *(unsigned long long*)(s_scr + 6) = excl_tile;
        if (tile == p.ntiles - 1) *p.total = excl_tile + tile_total;
      }
    }
    __syncthreads();
    const unsigned long long goff = *(const unsigned long long*)(s_scr + 6);
    const uint32_t lbase = (uint32_t)(goff & 15);

    // ---- pass 2: decode again, pack bytes into the LDS staging buffer ----------
    if (active && cnt > 0) {
      uint32_t* stg = (uint32_t*)s_stage;
      const uint32_t bpos = lbase + excl_local;
      uint32_t oidx = bpos >> 2;
      uint32_t fill = 8u * (bpos & 3u);
      unsigned long long acc = 0;
      int P = start, Plast = start;
      uint32_t mlast = 0;
      do {
        uint32_t syms;
        const uint32_t meta = fetch_meta(s_lut, s_fb, window32(slot, P), kshift, p, &syms);
        if (fill >= 32) {  // flush a word completed by earlier (non-final) lookups
          atomicOr(&stg[oidx], (uint32_t)acc);
          acc >>= 32;
          fill -= 32;
          ++oidx;
        }
        acc |= (unsigned long long)syms << fill;
        fill += 8u * meta_n(meta);
        Plast = P;
        mlast = meta;
        P += (int)meta_b(meta);
      } while (P < 128);
      fill -= 8u * (meta_n(mlast) - kept_in_last(mlast, 128 - Plast));
      acc &= (1ull << fill) - 1ull;  // fill < 64
      if (fill > 0) atomicOr(&stg[oidx], (uint32_t)acc);
      if (fill > 32) atomicOr(&stg[oidx + 1], (uint32_t)(acc >> 32));
    }
    __syncthreads();

    // ---- copy-out: 16-byte chunks, partial edge chunks byte by byte -------------
    {
      const unsigned long long a0 = goff - lbase;
      const unsigned long long end = min(goff + tile_total, p.out_cap);
      const uint32_t nz = (lbase + tile_total + 15u) >> 4;
      uint4* st = (uint4*)s_stage;
      for (uint32_t c = tid; c < nz; c += TB) {
        const unsigned long long gs = a0 + 16ull * c;
        const uint4 v = st[c];
        st[c] = make_uint4(0, 0, 0, 0);
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
  }
}

// ============================================================================
// Host side
// ============================================================================
struct Tables {
  uint32_t K = 0;
  std::vector<uint2> lut;            // 2^K entries
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
  uint32_t meta = n | (pos << 3);
  for (uint32_t k = 1; k <= 3; ++k) meta |= ((k < n) ? ends[k] : 15u) << (4 + 4 * k);
  return meta;
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
      if ((m & 7) == 0) {
        fbp += 1.0;
        syms += 1.0;
      } else {
        syms += (m & 7);
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

static int build_tables(const Canon& c, Tables& t, int force_k) {
  if (c.nsyms == 0) return fail(GH_E_TABLE, "empty code");
  t.K = force_k > 0 ? (uint32_t)std::clamp(force_k, 1, 12) : choose_k(c);
  t.lut.assign(1u << t.K, make_uint2(0, 0));
  for (uint32_t i = 0; i < (1u << t.K); ++i) {
    uint32_t s;
    const uint32_t m = lut_meta_for(c, i, t.K, &s);
    t.lut[i] = make_uint2(s, m);
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

struct gh_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
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
  uint32_t epoch = 0;
  uint32_t ntiles = 0;
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
  c->d_payload = nullptr;
  c->d_gaps = nullptr;
  c->d_out = nullptr;
  c->d_gran = nullptr;
  c->d_lut = nullptr;
  c->d_fb = nullptr;
  c->loaded = false;
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
  GH_HIP(hipMalloc(&c->d_misc, 64));
  GH_HIP(hipMemset(c->d_misc, 0, 64));
  GH_HIP(hipFuncSetAttribute((const void*)gh_decode_kernel,
                             hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  *out = c;
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
  c->ntiles = (uint32_t)ceil_div(c->nseg, TB);
  if (c->nseg > 0) {
    const char* envk = getenv("GH_LUT_BITS");
    rc = build_tables(c->canon, c->tables, envk ? atoi(envk) : 0);
    if (rc) return rc;
  }
  const uint64_t bound = c->nseg * (uint64_t)std::max<uint32_t>(c->tables.maxsyms_seg, 1);
  if (out_cap == 0) out_cap = std::min<uint64_t>(s->n, bound);
  c->out_cap = out_cap;
  GH_HIP(hipSetDevice(c->device));
  GH_HIP(hipMalloc(&c->d_out, std::max<uint64_t>(out_cap, 16) + 64));
  GH_HIP(hipMalloc(&c->d_gran, 8ull * std::max<uint32_t>(c->ntiles, 1)));
  GH_HIP(hipMemset(c->d_gran, 0, 8ull * std::max<uint32_t>(c->ntiles, 1)));
  GH_HIP(hipMemset(c->d_misc, 0, 64));
  c->epoch = 0;
  if (c->nseg > 0) {
    const size_t lut_bytes = c->tables.lut.size() * sizeof(uint2);
    GH_HIP(hipMalloc(&c->d_lut, std::max<size_t>(lut_bytes, 16)));
    GH_HIP(hipMemcpy(c->d_lut, c->tables.lut.data(), lut_bytes, hipMemcpyHostToDevice));
    GH_HIP(hipMalloc(&c->d_fb, sizeof(c->tables.fb)));
    GH_HIP(hipMemcpy(c->d_fb, c->tables.fb, sizeof(c->tables.fb), hipMemcpyHostToDevice));
    c->stage_bytes = (uint32_t)(((uint64_t)TB * c->tables.maxsyms_seg + 32 + 15) & ~15ull);
    c->lds = lut_bytes + FB_BYTES + IN_BYTES + c->stage_bytes + SCRATCH_BYTES;
    int per_cu = 0;
    GH_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, gh_decode_kernel, TB, c->lds));
    if (per_cu < 1) return fail(GH_E_HIP, "decode kernel does not fit on a CU");
    c->grid = (uint32_t)std::min<uint64_t>(c->ntiles, (uint64_t)per_cu * c->num_cu);
  }
  // start bit of local segment 0, and the gap nibble base for the rest
  c->first_start = 0;
  if (b > 0) {
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
  // gap nibbles for local segments 1..nseg-1: global nibbles [b, e-1)
  const uint64_t gw0 = b >> 3;
  const uint64_t gw1 = (e >= 2) ? ((e - 2) >> 3) + 1 : gw0 + 1;
  const uint64_t gwords = std::max<uint64_t>(gw1, gw0 + 1) - gw0;
  const uint64_t total_gw = ceil_div(s->g, GH_GAPS_PER_WORD);
  const uint64_t gcopy = (gw0 < total_gw) ? std::min<uint64_t>(gwords, total_gw - gw0) : 0;
  GH_HIP(hipMalloc(&c->d_gaps, 4 * (gwords + 4)));
  GH_HIP(hipMemset(c->d_gaps, 0, 4 * (gwords + 4)));
  if (gcopy)
    GH_HIP(hipMemcpy(c->d_gaps, (const uint8_t*)s->gap_words + 4 * gw0, 4 * gcopy,
                     hipMemcpyHostToDevice));
  c->gap_nib0 = (uint32_t)(b - 8 * gw0);
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
  const uint64_t gw1 = (e >= 2) ? ((e - 2) >> 3) + 1 : gw0 + 1;
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
    return GH_OK;
  }
  if (++c->epoch >= EPOCH_MAX) {  // granule epochs wrap: start clean
    GH_HIP(hipMemsetAsync(c->d_gran, 0, 8ull * c->ntiles, st));
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
  p.ntiles = c->ntiles;
  p.kbits = c->tables.K;
  p.epoch = c->epoch;
  p.lut_bytes = (uint32_t)(c->tables.lut.size() * sizeof(uint2));
  p.stage_bytes = c->stage_bytes;
  p.fb_lo = c->tables.fb_lo;
  p.fb_hi = c->tables.fb_hi;
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
  hipLaunchKernelGGL(gh_decode_kernel, dim3(c->grid), dim3(TB), c->lds, st, p);
  GH_HIP(hipGetLastError());
  if (timed) {
    GH_HIP(hipEventRecord(ev.second, st));
    c->pending.push_back(ev);
  }
  return GH_OK;
}

extern "C" int gh_ctx_report(gh_ctx* c, void* hip_stream, gh_report* rep) {
  if (!c) return fail(GH_E_ARG, "null ctx");
  hipStream_t st = hip_stream ? (hipStream_t)hip_stream : c->stream;
  GH_HIP(hipSetDevice(c->device));
  GH_HIP(hipStreamSynchronize(st));
  for (auto& e : c->pending) {
    float ms = 0;
    GH_HIP(hipEventElapsedTime(&ms, e.first, e.second));
    c->acc_ms += ms;
    c->nlaunch++;
    c->pool.push_back(e);
  }
  c->pending.clear();
  unsigned int misc[4] = {};
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
  GH_HIP(hipStreamSynchronize(c->stream));
  GH_HIP(hipMemcpy(dst, c->d_out + off, nbytes, hipMemcpyDeviceToHost));
  return GH_OK;
}

extern "C" int gh_ctx_output(gh_ctx* c, void** d_out, uint64_t* cap) {
  if (!c || !d_out) return fail(GH_E_ARG, "null argument");
  *d_out = c->d_out;
  if (cap) *cap = c->out_cap;
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
