// Host side of the gap-array Huffman codec: compressed.huff v1/v2 format, the
// boundary package-merge code-length builder, canonical codes, the encoder that
// produces the decoder's input, and the seeded synthetic-input generator.
//
// Reference behaviour restated here (file:line relative to the reference repo):
//   format ......... encoder/src/huff.cpp:186-202 (writer), decoder/src/huff.cpp:36-100
//   histogram ...... encoder/src/encoder.cu:33-140, symbols.cpp:29-43
//   sort ........... encoder/src/huff.cpp:18-22,115 (qsort ascending by count; glibc's
//                    qsort is a stable merge sort for this size, so ties keep
//                    ascending symbol order)
//   code lengths ... encoder/src/package_merge.cpp:12-166 (boundary package-merge, L=16)
//   canonical codes  package_merge.cpp:168-181
//   bit packing .... encoder/src/encoder.cu:281-347 (MSB-first inside each u32)
//   gap array ...... encoder/src/encoder.cu:307-312,358-379
//   generator ...... generate.cpp:32-47
#include <algorithm>
#include <atomic>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "gh_internal.hpp"

namespace gh {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }
int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

int build_canon(const gh_sym* syms, uint32_t nsyms, Canon& c) {
  c = Canon();
  if (nsyms == 0) return GH_OK;
  if (nsyms > GH_MAX_SYMBOLS) return fail(GH_E_TABLE, "more than 256 symbols");
  bool seen[GH_MAX_SYMBOLS] = {};
  c.nsyms = nsyms;
  c.minlen = 99;
  uint32_t code = 0;
  for (uint32_t i = 0; i < nsyms; ++i) {
    const uint32_t l = syms[i].length;
    if (l < 1 || l > GH_MAX_CODE_LEN) return fail(GH_E_TABLE, "code length outside 1..16");
    if (seen[syms[i].symbol]) return fail(GH_E_TABLE, "duplicate symbol in header");
    seen[syms[i].symbol] = true;
    if (i > 0 && l < syms[i - 1].length)
      return fail(GH_E_TABLE, "lengths not non-decreasing (not canonical order)");
    if (i > 0) code = (code + 1) << (l - syms[i - 1].length);
    if (code >> l) return fail(GH_E_TABLE, "code space overflow (Kraft sum > 1)");
    c.sym[i] = syms[i].symbol;
    c.len[i] = (uint8_t)l;
    c.code[i] = code;
    c.minlen = std::min(c.minlen, l);
    c.maxlen = std::max(c.maxlen, l);
    if (c.count[l] == 0) {
      c.first[l] = i;
      c.base16[l] = code << (16 - l);
    }
    c.count[l]++;
  }
  for (uint32_t l = 1; l <= GH_MAX_CODE_LEN; ++l)
    if (c.count[l]) c.limit16[l] = c.base16[l] + (c.count[l] << (16 - l));
  return GH_OK;
}

static int n_threads(int t) {
  if (t > 0) return t;
  unsigned hc = std::thread::hardware_concurrency();
  if (hc == 0) hc = 1;
  return (int)std::min(hc, 32u);
}

template <class F>
static void parallel_for(int nt, F f) {
  if (nt <= 1) {
    f(0);
    return;
  }
  std::vector<std::thread> th;
  th.reserve(nt);
  for (int t = 0; t < nt; ++t) th.emplace_back(f, t);
  for (auto& x : th) x.join();
}

// ---------------------------------------------------------------------------
// Boundary package-merge (Katajainen/Moffat/Turpin) with lazily built lists,
// behaviour-identical to encoder/src/package_merge.cpp:12-166:
//  * 16 lists; every list starts with the package {c0+c1} holding 2 leaves;
//  * a list's next package takes two items, each the lower list's pending package
//    when no leaf is left or its weight <= the next leaf, else the next leaf;
//  * the top list selects 2n-2 items starting from the two smallest leaves;
//  * a symbol's length is the number of lists whose active leaves include it.
// ---------------------------------------------------------------------------
namespace {
struct PmNode {
  uint64_t weight;
  int leaves;      // leaves used by this list up to and including this package
  int chain_idx;   // package of the next lower list last consumed (-1: none)
};

struct Pm {
  const uint64_t* c;
  int n;
  std::vector<PmNode> list[GH_MAX_CODE_LEN];

  void extend(int l) {
    const PmNode tail = list[l].back();
    PmNode nx{0, tail.leaves, tail.chain_idx};
    if (l == 0) {
      nx.chain_idx = -1;
      for (int k = 0; k < 2; ++k)
        if (nx.leaves < n) nx.weight += c[nx.leaves++];
    } else {
      for (int k = 0; k < 2; ++k) {
        const int pend = (int)list[l - 1].size() - 1;
        const uint64_t pw = list[l - 1][pend].weight;
        if (nx.leaves >= n || pw <= c[nx.leaves]) {
          nx.weight += pw;
          nx.chain_idx = pend;
          extend(l - 1);
        } else {
          nx.weight += c[nx.leaves++];
        }
      }
    }
    list[l].push_back(nx);
  }
};
}  // namespace

}  // namespace gh

using namespace gh;

extern "C" int gh_package_merge(const uint64_t* sorted_counts, uint32_t nsyms,
                                uint8_t* lengths) {
  if (!lengths || (nsyms && !sorted_counts)) return fail(GH_E_ARG, "null argument");
  if (nsyms > GH_MAX_SYMBOLS) return fail(GH_E_ARG, "too many symbols");
  if (nsyms == 0) return GH_OK;
  if (nsyms == 1) {  // package_merge.cpp:159 gives the lone symbol length 1
    lengths[0] = 1;
    return GH_OK;
  }
  const int n = (int)nsyms;
  const int L = GH_MAX_CODE_LEN;
  Pm pm;
  pm.c = sorted_counts;
  pm.n = n;
  for (int l = 0; l < L; ++l) {
    pm.list[l].reserve(2 * n);
    pm.list[l].push_back(PmNode{sorted_counts[0] + sorted_counts[1], 2, -1});
  }
  int top_leaves = 2, head = -1;
  for (int i = 2; i < 2 * (n - 1); ++i) {
    const int pend = (int)pm.list[L - 2].size() - 1;
    if (top_leaves < n && pm.list[L - 2][pend].weight > sorted_counts[top_leaves]) {
      ++top_leaves;
    } else {
      head = pend;
      pm.extend(L - 2);
    }
  }
  std::vector<int> len(n, 0);
  for (int i = 0; i < top_leaves; ++i) len[i]++;
  for (int l = L - 2, idx = head; l >= 0 && idx >= 0; --l) {
    const PmNode& nd = pm.list[l][idx];
    for (int j = 0; j < nd.leaves && j < n; ++j) len[j]++;
    idx = nd.chain_idx;
  }
  for (int i = 0; i < n; ++i) {
    if (len[i] < 1 || len[i] > L) return fail(GH_E_TABLE, "package-merge produced bad length");
    lengths[i] = (uint8_t)len[i];
  }
  return GH_OK;
}

// ---------------------------------------------------------------------------
// Format
// ---------------------------------------------------------------------------
template <class T>
static T rd(const uint8_t* p) {
  T v;
  std::memcpy(&v, p, sizeof(T));
  return v;
}
template <class T>
static void wr(uint8_t* p, T v) {
  std::memcpy(p, &v, sizeof(T));
}

extern "C" int gh_stream_validate(const gh_stream* s) {
  if (!s) return fail(GH_E_ARG, "null stream");
  Canon c;
  int rc = build_canon(s->syms, s->nsyms, c);
  if (rc) return rc;
  if (s->n > 0 && s->nsyms == 0) return fail(GH_E_FORMAT, "N > 0 but no symbols");
  if (s->g == 0) {
    if (s->w != 0) return fail(GH_E_FORMAT, "G = 0 but W > 0");
  } else if (s->w > 4 * s->g || s->w + 3 < 4 * s->g) {
    return fail(GH_E_FORMAT, "W inconsistent with G (need 4G-3 <= W <= 4G)");
  }
  if (s->n > 0 && s->g == 0) return fail(GH_E_FORMAT, "N > 0 but G = 0");
  // every symbol takes >= minlen bits, so N * minlen <= 32 W
  if (s->nsyms && (unsigned __int128)s->n * c.minlen > (unsigned __int128)s->w * 32)
    return fail(GH_E_FORMAT, "N too large for the payload");
  return GH_OK;
}

extern "C" int gh_stream_parse(const void* file, size_t len, gh_stream* out) {
  if (!file || !out) return fail(GH_E_ARG, "null argument");
  const uint8_t* p = (const uint8_t*)file;
  gh_stream s{};
  size_t off = 0;
  if (len < 8) return fail(GH_E_FORMAT, "file shorter than the symbol-count field");
  uint64_t first = rd<uint64_t>(p);
  if (first == GH_V2_MAGIC) {
    s.version = 2;
    off = 8;
    if (len < 16) return fail(GH_E_FORMAT, "truncated v2 header");
    first = rd<uint64_t>(p + off);
  } else {
    s.version = 1;
  }
  off += 8;
  if (first > GH_MAX_SYMBOLS) return fail(GH_E_FORMAT, "symbol count > 256");
  s.nsyms = (uint32_t)first;
  if (len < off + 2 * s.nsyms) return fail(GH_E_FORMAT, "truncated symbol table");
  s.syms = (const gh_sym*)(p + off);
  off += 2 * s.nsyms;
  if (s.version == 1) {
    if (len < off + 12) return fail(GH_E_FORMAT, "truncated size fields");
    s.n = rd<uint32_t>(p + off);
    s.w = rd<uint32_t>(p + off + 4);
    s.g = rd<uint32_t>(p + off + 8);
    off += 12;
  } else {
    if (len < off + 24) return fail(GH_E_FORMAT, "truncated size fields");
    s.n = rd<uint64_t>(p + off);
    s.w = rd<uint64_t>(p + off + 8);
    s.g = rd<uint64_t>(p + off + 16);
    off += 24;
  }
  const uint64_t gw = ceil_div(s.g, GH_GAPS_PER_WORD);
  if (gw > (len - off) / 4 || s.w > (len - off) / 4 - gw)
    return fail(GH_E_FORMAT, "file shorter than gap array + payload");
  s.gap_words = (const uint32_t*)(p + off);
  off += 4 * gw;
  s.payload = (const uint32_t*)(p + off);
  int rc = gh_stream_validate(&s);
  if (rc) return rc;
  *out = s;
  return GH_OK;
}

// ---------------------------------------------------------------------------
// Encoder
// ---------------------------------------------------------------------------
extern "C" int gh_encode_plan_make(const uint8_t* in, uint64_t n, int threads,
                                   int force_version, gh_encode_plan* plan) {
  if (!plan || (n && !in)) return fail(GH_E_ARG, "null argument");
  std::memset(plan, 0, sizeof(*plan));
  plan->n = n;
  const int nt = (int)std::min<uint64_t>(n_threads(threads), std::max<uint64_t>(1, n >> 20));
  std::vector<uint64_t> hist((size_t)nt * 256, 0);
  parallel_for(nt, [&](int t) {
    const uint64_t a = n * t / nt, b = n * (t + 1) / nt;
    uint64_t* h = &hist[(size_t)t * 256];
    for (uint64_t i = a; i < b; ++i) h[in[i]]++;
  });
  for (int t = 0; t < nt; ++t)
    for (int v = 0; v < 256; ++v) plan->count[v] += hist[(size_t)t * 256 + v];
  return gh::plan_from_counts(plan, force_version);
}

// The plan from plan->n and plan->count[] (the host histogram above, or the GPU
// encoder's, gh_encode.hip).
int gh::plan_from_counts(gh_encode_plan* plan, int force_version) {
  // store_symbols (symbols.cpp:29-43): ascending symbol value, non-zero counts;
  // then a stable ascending sort by count (huff.cpp:115).
  uint32_t order[256];
  uint32_t ns = 0;
  for (uint32_t v = 0; v < 256; ++v)
    if (plan->count[v]) order[ns++] = v;
  std::stable_sort(order, order + ns,
                   [&](uint32_t a, uint32_t b) { return plan->count[a] < plan->count[b]; });
  uint64_t sc[256];
  uint8_t sl[256];
  for (uint32_t i = 0; i < ns; ++i) sc[i] = plan->count[order[i]];
  int rc = gh_package_merge(sc, ns, sl);
  if (rc) return rc;
  plan->nsyms = ns;
  // file order = most frequent first (huff.cpp:189-194)
  for (uint32_t i = 0; i < ns; ++i) {
    plan->syms[i].symbol = (uint8_t)order[ns - 1 - i];
    plan->syms[i].length = sl[ns - 1 - i];
  }
  Canon c;
  rc = build_canon(plan->syms, ns, c);
  if (rc) return rc;
  uint64_t bits = 0;
  for (uint32_t i = 0; i < ns; ++i) {
    plan->code[c.sym[i]] = c.code[i];
    plan->len[c.sym[i]] = c.len[i];
    bits += (uint64_t)c.len[i] * plan->count[c.sym[i]];
  }
  plan->bits = bits;
  plan->g = ceil_div(bits, GH_SEGMENT_BITS);
  plan->w = ceil_div(bits, 32);
  const uint64_t lim = 1ull << 31;
  plan->version = (plan->n >= lim || plan->w >= lim || plan->g >= lim) ? 2 : 1;
  if (force_version == 2) plan->version = 2;
  if (force_version == 1 && plan->version == 2)
    return fail(GH_E_ARG, "stream too large for the v1 (32-bit) header");
  const uint64_t hdr = (plan->version == 2 ? 16 : 8) + 2ull * ns + (plan->version == 2 ? 24 : 12);
  plan->file_bytes = hdr + 4 * ceil_div(plan->g, GH_GAPS_PER_WORD) + 4 * plan->w;
  return GH_OK;
}

// Header of the compressed image (encoder/src/huff.cpp:186-196; v2: 64-bit sizes
// behind a magic); returns its size in bytes.
size_t gh::encode_header(const gh_encode_plan* plan, uint8_t* out) {
  size_t off = 0;
  if (plan->version == 2) {
    wr<uint64_t>(out, GH_V2_MAGIC);
    off = 8;
  }
  wr<uint64_t>(out + off, plan->nsyms);
  off += 8;
  for (uint32_t i = 0; i < plan->nsyms; ++i) {
    out[off++] = plan->syms[i].symbol;
    out[off++] = plan->syms[i].length;
  }
  if (plan->version == 2) {
    wr<uint64_t>(out + off, plan->n);
    wr<uint64_t>(out + off + 8, plan->w);
    wr<uint64_t>(out + off + 16, plan->g);
    off += 24;
  } else {
    wr<uint32_t>(out + off, (uint32_t)plan->n);
    wr<uint32_t>(out + off + 4, (uint32_t)plan->w);
    wr<uint32_t>(out + off + 8, (uint32_t)plan->g);
    off += 12;
  }
  return off;
}

extern "C" int gh_encode_write(const uint8_t* in, const gh_encode_plan* plan, int threads,
                               void* out_v, uint64_t out_len) {
  if (!plan || !out_v || (plan->n && !in)) return fail(GH_E_ARG, "null argument");
  if (out_len < plan->file_bytes) return fail(GH_E_SMALL, "output buffer too small");
  uint8_t* out = (uint8_t*)out_v;
  const uint64_t n = plan->n, W = plan->w, G = plan->g;
  const uint64_t GW = ceil_div(G, GH_GAPS_PER_WORD);
  size_t off = gh::encode_header(plan, out);
  std::vector<uint32_t> gaps(GW + 1, 0), words(W + 1, 0);
  const int nt = (int)std::min<uint64_t>(n_threads(threads), std::max<uint64_t>(1, n >> 20));
  // per-thread bit totals -> exclusive bit offsets
  std::vector<uint64_t> tbits(nt + 1, 0);
  parallel_for(nt, [&](int t) {
    const uint64_t a = n * t / nt, b = n * (t + 1) / nt;
    uint64_t s = 0;
    for (uint64_t i = a; i < b; ++i) s += plan->len[in[i]];
    tbits[t + 1] = s;
  });
  for (int t = 0; t < nt; ++t) tbits[t + 1] += tbits[t];
  if (tbits[nt] != plan->bits) return fail(GH_E_ARG, "input does not match the plan");
  parallel_for(nt, [&](int t) {
    const uint64_t a = n * t / nt, b = n * (t + 1) / nt;
    uint64_t pos = tbits[t];
    uint64_t acc = 0;
    int nb = (int)(pos & 31);  // placeholder zero bits already in the first word
    uint64_t widx = pos >> 5;
    const uint64_t first_word = widx;
    auto emit = [&](uint32_t v) {
      if (widx == first_word) {
        __atomic_fetch_or(&words[widx], v, __ATOMIC_RELAXED);
      } else {
        words[widx] = v;
      }
      ++widx;
    };
    for (uint64_t i = a; i < b; ++i) {
      const uint8_t sym = in[i];
      const uint32_t l = plan->len[sym];
      const uint64_t end = pos + l;
      if ((end >> 7) != (pos >> 7)) {  // codeword crosses a 128-bit boundary
        const uint32_t gv = (uint32_t)(end & 15);
        const uint64_t j = pos >> 7;
        if (gv) __atomic_fetch_or(&gaps[j >> 3], gv << (4 * (j & 7)), __ATOMIC_RELAXED);
      }
      acc = (acc << l) | plan->code[sym];
      nb += (int)l;
      if (nb >= 32) {
        nb -= 32;
        emit((uint32_t)(acc >> nb));
        acc &= (nb ? ((1ull << nb) - 1) : 0ull);
      }
      pos = end;
    }
    if (nb > 0) {  // trailing partial word, shared with the next thread
      __atomic_fetch_or(&words[widx], (uint32_t)(acc << (32 - nb)), __ATOMIC_RELAXED);
    }
  });
  std::memcpy(out + off, gaps.data(), 4 * GW);
  off += 4 * GW;
  std::memcpy(out + off, words.data(), 4 * W);
  return GH_OK;
}

// ---------------------------------------------------------------------------
// Generator (generate.cpp:32-47 distribution, counter-based PRNG)
// ---------------------------------------------------------------------------
static inline uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

extern "C" int gh_generate(uint64_t seed, double redundancy, uint64_t offset, uint64_t n,
                           uint8_t* out, int threads) {
  if (n && !out) return fail(GH_E_ARG, "null output");
  if (!(redundancy >= 0.0)) redundancy = 0.0;  // also maps NaN to 0
  if (redundancy > 1.0) redundancy = 1.0;
  // P(u < r) with u = k * 2^-53: threshold on the 53-bit integer
  const uint64_t thr = (uint64_t)(redundancy * 9007199254740992.0);  // r * 2^53
  const uint64_t key = mix64(seed ^ 0x6A09E667F3BCC909ull);
  const int nt = (int)std::min<uint64_t>(n_threads(threads), std::max<uint64_t>(1, n >> 22));
  parallel_for(nt, [&](int t) {
    const uint64_t a = n * t / nt, b = n * (t + 1) / nt;
    for (uint64_t i = a; i < b; ++i) {
      const uint64_t z = mix64(key + (offset + i + 1) * 0x9E3779B97F4A7C15ull);
      const bool low = (z >> 11) < thr;
      out[i] = low ? (uint8_t)('A' + (z & 3)) : (uint8_t)(z & 0xFF);
    }
  });
  return GH_OK;
}

extern "C" int gh_plan_shards(uint64_t g, uint32_t nshards, uint64_t* bounds) {
  if (!bounds || nshards == 0) return fail(GH_E_ARG, "bad shard request");
  for (uint32_t k = 0; k <= nshards; ++k)
    bounds[k] = (uint64_t)((unsigned __int128)g * k / nshards);
  return GH_OK;
}

extern "C" const char* gh_version(void) { return "gaphuff-mi355x 0.1 (gfx950)"; }
extern "C" const char* gh_last_error(void) { return g_last_error.c_str(); }
