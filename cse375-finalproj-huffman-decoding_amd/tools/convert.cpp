// bin/convert — string-format <-> gap-array conversion.
//
//   bin/convert to-seq  <compressed.huff> <out.seq>
//   bin/convert to-gap  <in.seq> <compressed.huff>
//
// The "string format" is the one the reference's CPU baselines write and read:
// sequential.cpp:163-204 (writeHeader / readHeader) — [padding u8][N u16 big-endian]
// then N x {symbol u8, code length u8, the code as ASCII '0'/'1'}, followed by the
// bitstream packed MSB-first into bytes, `padding` zero bits at the end
// (sequential.cpp:37-51).  The same layout is used by parallel_cpu_decomp.cpp and
// parallel_cpu_prescan.cpp.
//
// to-seq writes the stream's canonical codes as the code strings and re-packs the
// payload words (MSB-first within u32) as bytes; the exact bit count comes from a walk
// over the N codewords.  to-gap takes any prefix code of lengths <= 16 (sequential.cpp
// builds a plain Huffman tree; its codes are not canonical): symbols are ordered by
// (length, code), each codeword is replaced by the canonical codeword of the same length
// (so every codeword keeps its bit position), and the gap nibbles are recorded as in
// encoder.cu:307-312.  Converting a canonical stream there and back is byte-identical.
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "gaphuff.h"

static int fail(const char* msg) {
  std::fprintf(stderr, "convert: %s\n", msg);
  return 1;
}

static bool read_all(const char* path, std::vector<uint8_t>& v) {
  FILE* f = std::fopen(path, "rb");
  if (!f) return false;
  std::fseek(f, 0, SEEK_END);
  const long n = std::ftell(f);
  std::fseek(f, 0, SEEK_SET);
  v.resize((size_t)std::max(n, 0L));
  const bool ok = n <= 0 || std::fread(v.data(), 1, (size_t)n, f) == (size_t)n;
  std::fclose(f);
  return ok;
}

static bool write_all(const char* path, const std::vector<uint8_t>& v) {
  FILE* f = std::fopen(path, "wb");
  if (!f) return false;
  const bool ok = v.empty() || std::fwrite(v.data(), 1, v.size(), f) == v.size();
  return std::fclose(f) == 0 && ok;
}

// 16-bit-prefix lookup of a prefix code: entry = index + 1 and length, 0 = no code.
struct Lut {
  std::vector<uint32_t> idx;
  std::vector<uint8_t> len;
  bool build(const std::vector<uint32_t>& code, const std::vector<uint8_t>& ln) {
    idx.assign(1u << 16, 0);
    len.assign(1u << 16, 0);
    for (size_t i = 0; i < code.size(); ++i) {
      const uint32_t l = ln[i];
      if (l < 1 || l > 16 || (code[i] >> l)) return false;
      const uint32_t lo = code[i] << (16 - l), hi = lo + (1u << (16 - l));
      for (uint32_t p = lo; p < hi; ++p) {
        if (len[p]) return false;  // not prefix-free
        idx[p] = (uint32_t)i + 1;
        len[p] = (uint8_t)l;
      }
    }
    return true;
  }
};

// MSB-first bit reader over bytes (16 bits peeked, zero beyond the end).
struct Bits {
  const uint8_t* p;
  uint64_t nbytes;
  uint32_t peek16(uint64_t pos) const {
    uint32_t v = 0;
    const uint64_t b = pos >> 3;
    for (int i = 0; i < 3; ++i) v = (v << 8) | (b + i < nbytes ? p[b + i] : 0u);
    return (v >> (8 - (pos & 7))) & 0xffffu;
  }
};

static int to_seq(const char* in, const char* out) {
  std::vector<uint8_t> file;
  if (!read_all(in, file)) return fail("cannot read input");
  gh_stream s;
  if (gh_stream_parse(file.data(), file.size(), &s)) return fail(gh_last_error());
  if (s.nsyms > 65535) return fail("too many symbols");
  std::vector<uint32_t> code(s.nsyms);
  std::vector<uint8_t> ln(s.nsyms);
  uint32_t c = 0;
  for (uint32_t i = 0; i < s.nsyms; ++i) {
    if (i) c = (c + 1) << (s.syms[i].length - s.syms[i - 1].length);
    code[i] = c;
    ln[i] = s.syms[i].length;
  }
  // payload words -> MSB-first bytes
  std::vector<uint8_t> bytes(4 * s.w);
  for (uint64_t i = 0; i < s.w; ++i) {
    uint32_t w;
    std::memcpy(&w, (const uint8_t*)s.payload + 4 * i, 4);
    bytes[4 * i] = (uint8_t)(w >> 24);
    bytes[4 * i + 1] = (uint8_t)(w >> 16);
    bytes[4 * i + 2] = (uint8_t)(w >> 8);
    bytes[4 * i + 3] = (uint8_t)w;
  }
  Lut lut;
  if (s.nsyms && !lut.build(code, ln)) return fail("invalid code table");
  Bits br{bytes.data(), bytes.size()};
  uint64_t pos = 0;
  for (uint64_t k = 0; k < s.n; ++k) {
    const uint32_t l = s.nsyms ? lut.len[br.peek16(pos)] : 0;
    if (!l) return fail("stream holds an invalid codeword");
    pos += l;
  }
  if (pos > 32 * s.w) return fail("stream shorter than N codewords");
  const uint64_t nb = (pos + 7) / 8;
  const int padding = (int)((8 - pos % 8) % 8);
  std::vector<uint8_t> o;
  o.push_back((uint8_t)padding);
  o.push_back((uint8_t)(s.nsyms >> 8));
  o.push_back((uint8_t)s.nsyms);
  for (uint32_t i = 0; i < s.nsyms; ++i) {
    o.push_back(s.syms[i].symbol);
    o.push_back(ln[i]);
    for (int b = ln[i] - 1; b >= 0; --b) o.push_back((code[i] >> b) & 1 ? '1' : '0');
  }
  o.insert(o.end(), bytes.begin(), bytes.begin() + nb);
  if (padding) o.back() &= (uint8_t)(0xff << padding);
  if (!write_all(out, o)) return fail("cannot write output");
  std::printf("to-seq: N=%llu bits=%llu symbols=%u padding=%d\n", (unsigned long long)s.n,
              (unsigned long long)pos, s.nsyms, padding);
  return 0;
}

static int to_gap(const char* in, const char* out) {
  std::vector<uint8_t> f;
  if (!read_all(in, f)) return fail("cannot read input");
  if (f.size() < 3) return fail("truncated string-format header");
  const int padding = f[0];
  const uint32_t ns = ((uint32_t)f[1] << 8) | f[2];
  if (padding > 7 || ns > 256) return fail("bad string-format header");
  size_t at = 3;
  struct E {
    uint8_t sym, len;
    uint32_t code;
  };
  std::vector<E> e;
  for (uint32_t i = 0; i < ns; ++i) {
    if (at + 2 > f.size()) return fail("truncated code table");
    E x{f[at], f[at + 1], 0};
    at += 2;
    if (x.len < 1 || x.len > GH_MAX_CODE_LEN)
      return fail("code length outside 1..16 (the gap-array format's limit)");
    if (at + x.len > f.size()) return fail("truncated code string");
    for (int b = 0; b < x.len; ++b) {
      const uint8_t ch = f[at + b];
      if (ch != '0' && ch != '1') return fail("code string is not binary");
      x.code = (x.code << 1) | (uint32_t)(ch == '1');
    }
    at += x.len;
    e.push_back(x);
  }
  // canonical order: by length, then code value (keeps a canonical input's order)
  std::sort(e.begin(), e.end(), [](const E& a, const E& b) {
    return a.len != b.len ? a.len < b.len : a.code < b.code;
  });
  std::vector<uint32_t> oc(ns), canon(ns);
  std::vector<uint8_t> ln(ns);
  uint32_t c = 0;
  for (uint32_t i = 0; i < ns; ++i) {
    if (i && e[i].sym == e[i - 1].sym) return fail("duplicate symbol");
    if (i) c = (c + 1) << (e[i].len - e[i - 1].len);
    if (c >> e[i].len) return fail("code table violates the Kraft inequality");
    canon[i] = c;
    oc[i] = e[i].code;
    ln[i] = e[i].len;
  }
  Lut lut;
  if (ns && !lut.build(oc, ln)) return fail("code table is not prefix-free");
  const uint64_t nbytes = f.size() - at;
  if (nbytes == 0 && padding) return fail("padding without payload");
  const uint64_t bits = 8 * nbytes - (uint64_t)padding;
  Bits br{f.data() + at, nbytes};
  const uint64_t w = (bits + 31) / 32, g = (bits + 127) / 128;
  std::vector<uint32_t> pay(w + 1, 0), gaps((g + 7) / 8 + 1, 0);
  uint64_t pos = 0, n = 0;
  while (pos < bits) {
    const uint32_t p = br.peek16(pos);
    const uint32_t l = ns ? lut.len[p] : 0;
    if (!l || pos + l > bits) return fail("bitstream holds an invalid or truncated codeword");
    const uint32_t cw = canon[lut.idx[p] - 1];
    // write l bits of cw at pos, MSB-first within u32 words
    const uint64_t wi = pos >> 5;
    const uint32_t o = (uint32_t)(pos & 31);
    const uint64_t v = (uint64_t)cw << (64 - l - o);
    pay[wi] |= (uint32_t)(v >> 32);
    if (o + l > 32) pay[wi + 1] |= (uint32_t)v;
    const uint64_t end = pos + l, seg = pos >> 7;
    if ((end - 1) >> 7 != seg && end > 128 * (seg + 1)) {
      const uint64_t gap = end - 128 * (seg + 1);  // encoder.cu:307-312
      gaps[seg >> 3] |= (uint32_t)gap << (4 * (seg & 7));
    }
    pos = end;
    ++n;
  }
  const bool v2 = n >= (1ull << 31) || w >= (1ull << 31) || g >= (1ull << 31);
  std::vector<uint8_t> o;
  auto put = [&](uint64_t x, int nb) {
    for (int i = 0; i < nb; ++i) o.push_back((uint8_t)(x >> (8 * i)));
  };
  if (v2) put(GH_V2_MAGIC, 8);
  put(ns, 8);
  for (uint32_t i = 0; i < ns; ++i) {
    o.push_back(e[i].sym);
    o.push_back(e[i].len);
  }
  const int fw = v2 ? 8 : 4;
  put(n, fw);
  put(w, fw);
  put(g, fw);
  const size_t h = o.size();
  o.resize(h + 4 * ((g + 7) / 8) + 4 * w);
  std::memcpy(o.data() + h, gaps.data(), 4 * ((g + 7) / 8));
  std::memcpy(o.data() + h + 4 * ((g + 7) / 8), pay.data(), 4 * w);
  gh_stream chk;
  if (gh_stream_parse(o.data(), o.size(), &chk)) return fail(gh_last_error());
  if (!write_all(out, o)) return fail("cannot write output");
  std::printf("to-gap: N=%llu bits=%llu W=%llu G=%llu symbols=%u v%d\n", (unsigned long long)n,
              (unsigned long long)bits, (unsigned long long)w, (unsigned long long)g, ns, v2 ? 2 : 1);
  return 0;
}

int main(int argc, char** argv) {
  if (argc != 4) {
    std::fprintf(stderr, "Usage: bin/convert to-seq <compressed.huff> <out.seq>\n"
                         "       bin/convert to-gap <in.seq> <compressed.huff>\n");
    return 2;
  }
  if (!std::strcmp(argv[1], "to-seq")) return to_seq(argv[2], argv[3]);
  if (!std::strcmp(argv[1], "to-gap")) return to_gap(argv[2], argv[3]);
  return fail("mode must be to-seq or to-gap");
}
