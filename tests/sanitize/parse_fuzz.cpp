// parse_fuzz — host-side parsers of untrusted files under AddressSanitizer + UBSan.
//
// Built by `make -C cse375-finalproj-huffman-decoding_amd asan` from this file plus the
// library's host sources (csrc/gh_core.cpp, csrc/gh_io.cpp) with
// -fsanitize=address,undefined; run by tests/test_sanitize.py (CPU, no GPU calls).
// Every mutated input lives in a heap block of exactly its length, so any read past
// it is reported.  Covers:
//   gh_stream_parse / gh_stream_validate   compressed.huff v1 and v2 headers, whole images
//                                          and the header-only view gh_ctx_load_file uses
//   gh_raw_parse                           raw-stream containers (bin/encoder --raw)
//   gh_package_merge, gh_plan_shards       random counts / sizes
// Usage: parse_fuzz [iterations] [seed]
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "gaphuff.h"

// gh_io.cpp's file entry points call into the device context (csrc/gh_decode.hip),
// which this host-only build does not link: stand-ins that fail like a box with no GPU.
extern "C" {
int gh_ctx_output(gh_ctx*, void**, uint64_t*) { return GH_E_NODEV; }
int gh_ctx_device(gh_ctx*, int*) { return GH_E_NODEV; }
int gh_ctx_report(gh_ctx*, void*, gh_report*) { return GH_E_NODEV; }
int gh_ctx_load_device(gh_ctx*, const gh_stream*, uint64_t, uint64_t, const uint32_t*, uint64_t,
                       const uint32_t*, uint64_t) {
  return GH_E_NODEV;
}
}

static uint64_t g_sink = 0;

static std::vector<uint8_t> make_image(uint64_t seed, double r, uint64_t n, int version) {
  std::vector<uint8_t> data(n);
  if (gh_generate(seed, r, 0, n, data.data(), 2)) std::abort();
  gh_encode_plan plan;
  if (gh_encode_plan_make(data.data(), n, 2, version, &plan)) std::abort();
  std::vector<uint8_t> img(plan.file_bytes);
  if (gh_encode_write(data.data(), &plan, 2, img.data(), img.size())) std::abort();
  return img;
}

static std::vector<uint8_t> make_raw(const std::vector<uint8_t>& img) {
  gh_stream s;
  if (gh_stream_parse(img.data(), img.size(), &s)) std::abort();
  std::vector<uint8_t> out;
  auto put64 = [&](uint64_t v) { for (int i = 0; i < 8; ++i) out.push_back((uint8_t)(v >> (8 * i))); };
  put64(GH_RAW_MAGIC);
  put64(s.nsyms);
  for (uint32_t i = 0; i < s.nsyms; ++i) {
    out.push_back(s.syms[i].symbol);
    out.push_back(s.syms[i].length);
  }
  put64(s.n);
  put64(s.w);
  const uint8_t* p = (const uint8_t*)s.payload;
  out.insert(out.end(), p, p + 4 * s.w);
  return out;
}

// Parse `buf` from an exact-size heap copy; on success touch every byte it points at.
static void check_stream(const std::vector<uint8_t>& buf, size_t claimed_len) {
  uint8_t* heap = (uint8_t*)std::malloc(buf.size() ? buf.size() : 1);
  if (!buf.empty()) std::memcpy(heap, buf.data(), buf.size());
  gh_stream s;
  if (gh_stream_parse(heap, claimed_len, &s) == GH_OK) {
    (void)gh_stream_validate(&s);
    for (uint32_t i = 0; i < s.nsyms; ++i) g_sink += s.syms[i].symbol + s.syms[i].length;
    if (claimed_len == buf.size()) {  // a whole image: gap words and payload are in it
      const uint8_t* gw = (const uint8_t*)s.gap_words;
      const uint8_t* pw = (const uint8_t*)s.payload;
      for (uint64_t i = 0; i < 4 * ((s.g + 7) / 8); ++i) g_sink += gw[i];
      for (uint64_t i = 0; i < 4 * s.w; ++i) g_sink += pw[i];
    }
  }
  std::free(heap);
}

static void check_raw(const std::vector<uint8_t>& buf) {
  uint8_t* heap = (uint8_t*)std::malloc(buf.size() ? buf.size() : 1);
  if (!buf.empty()) std::memcpy(heap, buf.data(), buf.size());
  gh_raw_stream r;
  if (gh_raw_parse(heap, buf.size(), &r) == GH_OK) {
    for (uint32_t i = 0; i < r.nsyms; ++i) g_sink += r.syms[i].length;
    const uint8_t* u = (const uint8_t*)r.units;
    for (uint64_t i = 0; i < 4 * r.w; ++i) g_sink += u[i];
  }
  std::free(heap);
}

static std::vector<uint8_t> mutate(const std::vector<uint8_t>& src, std::mt19937_64& rng) {
  std::vector<uint8_t> b = src;
  switch (rng() % 5) {
    case 0:  // truncate
      b.resize(rng() % (b.size() + 1));
      break;
    case 1:  // flip header bytes
      for (int k = 0, m = 1 + (int)(rng() % 6); k < m && !b.empty(); ++k)
        b[rng() % std::min<size_t>(b.size(), 600)] = (uint8_t)rng();
      break;
    case 2: {  // overwrite one header u32/u64 field with an extreme value
      static const uint64_t ext[] = {0, 1, 0x7fffffffull, 0x80000000ull, 0xffffffffull, 1ull << 40, ~0ull};
      if (b.size() >= 16) {
        const size_t o = rng() % std::min<size_t>(b.size() - 8, 600);
        const uint64_t v = ext[rng() % 7];
        std::memcpy(&b[o], &v, (rng() & 1) ? 8 : 4);
      }
      break;
    }
    case 3:  // extend with junk
      for (int k = 0, m = (int)(rng() % 64); k < m; ++k) b.push_back((uint8_t)rng());
      break;
    default:  // both
      b.resize(rng() % (b.size() + 1));
      if (!b.empty()) b[rng() % b.size()] ^= (uint8_t)(1u << (rng() % 8));
  }
  return b;
}

int main(int argc, char** argv) {
  const long iters = argc > 1 ? std::atol(argv[1]) : 20000;
  std::mt19937_64 rng(argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 375);
  std::vector<std::vector<uint8_t>> imgs = {
      make_image(1, 0.5, 20000, 0), make_image(2, 0.1, 3000, 2), make_image(3, 0.9, 1, 0),
      make_image(4, 0.999, 5000, 2), make_image(5, 0.0, 0, 0),
  };
  std::vector<std::vector<uint8_t>> raws;
  for (auto& im : imgs) raws.push_back(make_raw(im));
  for (auto& im : imgs) {
    check_stream(im, im.size());
    check_raw(raws.back());
  }
  for (long it = 0; it < iters; ++it) {
    const auto& base = imgs[rng() % imgs.size()];
    std::vector<uint8_t> b = mutate(base, rng);
    check_stream(b, b.size());
    // the header-only view of gh_ctx_load_file: a short buffer, the file's length
    std::vector<uint8_t> h(b.begin(), b.begin() + std::min<size_t>(b.size(), 8 + 8 + 2 * GH_MAX_SYMBOLS + 24));
    check_stream(h, b.size());
    check_raw(mutate(raws[rng() % raws.size()], rng));
    // package-merge on random histograms, shard plans on random sizes
    uint64_t cnt[GH_MAX_SYMBOLS];
    uint8_t len[GH_MAX_SYMBOLS];
    const uint32_t ns = (uint32_t)(rng() % (GH_MAX_SYMBOLS + 2));
    for (uint32_t i = 0; i < ns && i < GH_MAX_SYMBOLS; ++i) cnt[i] = (i ? cnt[i - 1] : 1) + (rng() % 1000);
    (void)gh_package_merge(cnt, ns, len);
    uint64_t bounds[33];
    (void)gh_plan_shards(rng() % (1ull << 40), (uint32_t)(rng() % 33), bounds);
  }
  std::printf("parse_fuzz: %ld iterations ok (sink %llu)\n", iters, (unsigned long long)(g_sink & 0xff));
  return 0;
}
