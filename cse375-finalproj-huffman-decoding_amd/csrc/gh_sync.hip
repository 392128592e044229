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
//  gh_sync_kernel      thread t starts decoding at the raw bit 128t (possibly
//                      mid-codeword); walks of neighbouring threads then advance in
//                      lock-step until they merge (below).  a_t = the entry offset
//                      at 128(t+1) (the candidate gap[t]); b_t = the entry offset at
//                      128(t+2) on the same walk.  Writes gap words and
//                      pairs[t] = a_t | b_t << 4.
//  gh_sync_fix_kernel  verification: b_t == a_{t+1} for every t proves every a_t
//                      (induction: thread 0 starts at the true bit 0; if a_t is on
//                      the true path then thread t's walk is true from there, so b_t
//                      is the true entry at 128(t+2), which a_{t+1} equals).  A
//                      mismatch is repaired by re-walking from b_t, following the
//                      chain while it disagrees with the stored entries (the role of
//                      CUHD's phase 2).  The host repeats the pass until it finds no
//                      mismatch (CUHD's host loop, :439-475); on ordinary data the
//                      first pass finds none.
//  gh_sync_pack_kernel after repairs: pairs -> gap words.
//
// One 13-bit LUT in LDS serves both walks: {step (the advance below, or the first
// length when no codeword fits), length of the first codeword (0 if > 13 bits), bits of
// the complete codewords that fit in the 13 bits (the advance)}.  Walks take the
// multi-codeword step except where a step could skip the start that has to be
// recorded; codes of 14-16 bits use the canonical thresholds.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "gh_internal.hpp"

namespace gh {
namespace {

constexpr int SK = 13;          // LUT prefix bits (12: cfg4 2.28 ms, 13: 2.08, 14: 3.10 - occupancy)
constexpr int SYNC_TB = 256;    // threads per workgroup
constexpr uint32_t SYNC_CHAIN = 256;  // segments one repair chain may walk per pass
constexpr int SYNC_HALO = 8;          // warm-up segments per wave (GH_SYNC_HALO overrides)

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
  uint32_t* pairs;        // g bytes {a | b << 4}, as words
  unsigned int* counter;  // mismatches found by a fix pass
  uint32_t halo;          // warm-up segments per wave (multiple of 8, < 64)
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

// Each wavefront owns `out` = 64 - halo consecutive output segments [wo, wo+out); its
// lanes walk segments [wo-halo, wo+out), so the first `halo` lanes are warm-up walks
// that overlap the previous wave's segments.  Lane i's walk starts at the raw bit 128t
// (t = wo-halo+i, possibly mid-codeword) and records its entry at boundary t+1.  Then,
// in lock-step rounds (CUHD phase 1's scheme, cuhd_gpu_decoder.cu:186-229, here per
// wavefront so no workgroup barrier is needed: a wave's LDS operations complete in
// issue order), every walk that has not merged goes one segment on and compares its
// entry with the record its right neighbour's walk left there: equal means the two
// walks coincide from here on, so it stops; otherwise it overwrites the record (the
// lower walk started earlier, so it is the one to keep).  Walks stop at boundary
// wo+out+1 (the last b the wave needs).  The halo makes the wave's first output entry
// come from a walk that started `halo` segments (128*halo bits) earlier, which on
// ordinary codes has long merged with the true path, so the verify pass rarely finds a
// seam to repair.
constexpr int SYNC_WAVE = 64;
template <bool LONG>
__global__ __launch_bounds__(SYNC_TB) void gh_sync_kernel(SyncParams p) {
  __shared__ uint16_t lut[1 << SK];
  __shared__ uint8_t rec_all[SYNC_TB / SYNC_WAVE][SYNC_WAVE + 4];
  stage_lut(lut, p.lut);
  const uint32_t lane = threadIdx.x % SYNC_WAVE;
  const uint32_t halo = p.halo, out = SYNC_WAVE - halo;
  volatile uint8_t* rec = rec_all[threadIdx.x / SYNC_WAVE];
  const uint64_t nwaves = ceil_div_d(p.g, out);
  const uint64_t wstride = (uint64_t)gridDim.x * (SYNC_TB / SYNC_WAVE);
  for (uint64_t wv = (uint64_t)blockIdx.x * (SYNC_TB / SYNC_WAVE) + threadIdx.x / SYNC_WAVE; wv < nwaves;
       wv += wstride) {
    const int64_t w0 = (int64_t)(wv * out) - (int64_t)halo;  // segment of lane 0
    const int64_t ts = w0 + (int64_t)lane;
    const uint64_t t = (uint64_t)ts;
    const uint64_t kcap = (uint64_t)(w0 + SYNC_WAVE);  // last segment walked: boundary w0+65
    bool active = ts >= 0 && t < p.g;
    uint32_t off = 0;
    uint64_t k = t + 1;  // boundary of the walk's current entry
    if (lane < 4) rec[SYNC_WAVE + lane] = 0xff;
    rec[lane] = 0xff;
    __builtin_amdgcn_wave_barrier();
    if (active) {
      off = walk_segment<LONG>(t, 0, lut, p);
      rec[lane] = (uint8_t)off;
    }
    __builtin_amdgcn_wave_barrier();
    while (__any(active)) {
      if (active) {
        if (k > kcap || k >= p.g) {
          active = false;
        } else {
          const uint32_t e = walk_segment<LONG>(k, off, lut, p);
          ++k;
          const uint32_t idx = (uint32_t)((int64_t)k - w0 - 1);
          if (rec[idx] == e) {
            active = false;
          } else {
            rec[idx] = (uint8_t)e;
            off = e;
          }
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
    const bool mine = lane >= halo && ts >= 0 && t < p.g;
    uint32_t a = 0, b = 0;
    if (mine) {
      a = rec[lane];
      b = rec[lane + 1];
      // no codeword crosses the end of the stream: the entry at 128g is 0, as the
      // encoder leaves the last gap (encoder.cu:414 memset, nothing crosses 128G)
      if (t + 1 >= p.g) a = 0;
      if (t + 2 >= p.g) b = 0;
    }
    // w0 is a multiple of 8, so lane groups of 8 (4) are gap (pair) words
    uint32_t v = a << (4 * (lane & 7));
    v |= __shfl_xor(v, 1);
    v |= __shfl_xor(v, 2);
    v |= __shfl_xor(v, 4);
    if ((lane & 7) == 0 && mine) p.gaps[t >> 3] = v;
    uint32_t q = (a | b << 4) << (8 * (lane & 3));
    q |= __shfl_xor(q, 1);
    q |= __shfl_xor(q, 2);
    if ((lane & 3) == 0 && mine) p.pairs[t >> 2] = q;
    __builtin_amdgcn_wave_barrier();  // rec is reused by the wave's next segments
  }
}

__device__ __forceinline__ uint32_t pair_at(const uint32_t* pairs, uint64_t i) {
  return (__atomic_load_n(pairs + (i >> 2), __ATOMIC_RELAXED) >> (8 * (i & 3))) & 0xffu;
}

__device__ __forceinline__ void pair_store(uint32_t* pairs, uint64_t i, uint32_t v) {
  uint32_t* wp = pairs + (i >> 2);
  const uint32_t sh = 8 * (uint32_t)(i & 3);
  uint32_t old = __atomic_load_n(wp, __ATOMIC_RELAXED);
  for (;;) {
    const uint32_t nw = (old & ~(0xffu << sh)) | (v << sh);
    const uint32_t seen = atomicCAS(wp, old, nw);
    if (seen == old) break;
    old = seen;
  }
}

// a_j := a (the entry at 128(j+1)); re-walk segment j+1 from it to get b_j, and keep
// going while the new entry disagrees with the stored one.  (a, b) of one segment are
// replaced together by one CAS, so a pass never sees a torn pair.
template <bool LONG>
__device__ void repair_chain(uint64_t j, uint32_t a, const uint16_t* lut, const SyncParams& p) {
  for (uint32_t s = 0; s < SYNC_CHAIN; ++s) {
    uint32_t b = walk_segment<LONG>(j + 1, a, lut, p);
    if (j + 2 >= p.g) b = 0;
    pair_store(p.pairs, j, a | b << 4);
    if (j + 2 >= p.g) break;
    if ((pair_at(p.pairs, j + 1) & 15u) == b) break;  // back on the stored path
    ++j;
    a = b;
  }
}

template <bool LONG>
__global__ __launch_bounds__(SYNC_TB) void gh_sync_fix_kernel(SyncParams p) {
  __shared__ uint16_t lut[1 << SK];
  stage_lut(lut, p.lut);
  if (p.g < 3) return;
  const uint64_t stride = (uint64_t)gridDim.x * SYNC_TB;
  for (uint64_t t = (uint64_t)blockIdx.x * SYNC_TB + threadIdx.x; t + 2 < p.g; t += stride) {
    const uint32_t pt = pair_at(p.pairs, t), pn = pair_at(p.pairs, t + 1);
    if ((pt >> 4) != (pn & 15u)) {
      atomicAdd(p.counter, 1u);
      repair_chain<LONG>(t + 1, pt >> 4, lut, p);
    }
  }
}

__global__ __launch_bounds__(SYNC_TB) void gh_sync_pack_kernel(SyncParams p) {
  const uint64_t nw = (p.g + 7) / 8;
  const uint64_t stride = (uint64_t)gridDim.x * SYNC_TB;
  for (uint64_t i = (uint64_t)blockIdx.x * SYNC_TB + threadIdx.x; i < nw; i += stride) {
    uint32_t v = 0;
#pragma unroll
    for (uint32_t k = 0; k < 8; ++k) {
      const uint64_t s = 8 * i + k;
      if (s + 1 < p.g) v |= (pair_at(p.pairs, s) & 15u) << (4 * k);
    }
    p.gaps[i] = v;
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
  DevBuf lut, pairs, counter;
  GH_HIPS(hipMalloc(&lut.p, 2u << SK));
  GH_HIPS(hipMalloc(&pairs.p, 4 * ceil_div(g, 4) + 16));
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
  p.pairs = (uint32_t*)pairs.p;
  p.counter = (unsigned int*)counter.p;
  {
    const char* eh = getenv("GH_SYNC_HALO");
    const int h = eh ? atoi(eh) : SYNC_HALO;
    p.halo = (uint32_t)std::clamp(h - h % 8, 0, 56);
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
  const int gs = grid_for(ks, ceil_div(g, SYNC_WAVE - p.halo) * SYNC_WAVE);
  const int gf = grid_for(kf, g);
  void* kargs[] = {&p};
  GH_HIPS(hipMemsetAsync(counter.p, 0, 4, st));
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
    unsigned int cnt = 0;
    GH_HIPS(hipMemcpyAsync(&cnt, counter.p, 4, hipMemcpyDeviceToHost, st));
    GH_HIPS(hipStreamSynchronize(st));
    GH_HIPS(hipEventElapsedTime(&ms, e0, e1));
    ++passes;
    if (cnt == 0) break;
    mism += cnt;
    // each pass makes at least one more boundary true (the first mismatch follows a
    // true entry), so g passes always suffice
    if (passes > g + 1) return fail(GH_E_CORRUPT, "self-synchronisation did not converge");
    GH_HIPS(hipMemsetAsync(counter.p, 0, 4, st));
  }
  if (mism) {
    hipLaunchKernelGGL(gh_sync_pack_kernel, dim3(grid_for((const void*)gh_sync_pack_kernel, ceil_div(g, 8))),
                       dim3(SYNC_TB), 0, st, p);
    GH_HIPS(hipGetLastError());
    GH_HIPS(hipStreamSynchronize(st));
  }
  if (rep) {
    rep->mismatches = mism;
    rep->passes = passes;
    rep->kernel_ms = ms;
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
