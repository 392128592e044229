// bin/generate <filesize> <redundancy> [--seed S] [--out FILE]
//
// Seeded counterpart of the reference generate.cpp:11-58 (same CLI, same default
// output name data.bin, same byte distribution: 'A'+U{0..3} with probability
// `redundancy`, else U{0..255}).  The reference seeds mt19937_64 from
// std::random_device (generate.cpp:32), so its files cannot be reproduced; this
// tool uses a counter-based PRNG keyed by --seed (default 375) instead.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "gaphuff.h"

int main(int argc, char** argv) {
  if (argc < 3) {
    std::fprintf(stderr,
                 "Usage: %s <filesize> <redundancy> [--seed S] [--out FILE]\n"
                 "  filesize   : number of bytes (e.g., 100000000 for 100MB)\n"
                 "  redundancy : 0.0 to 1.0\n",
                 argv[0]);
    return 1;
  }
  const unsigned long long n = std::strtoull(argv[1], nullptr, 10);
  const double r = std::strtod(argv[2], nullptr);
  unsigned long long seed = 375;
  std::string out = "data.bin";
  for (int i = 3; i < argc; ++i) {
    if (!std::strcmp(argv[i], "--seed") && i + 1 < argc) seed = std::strtoull(argv[++i], nullptr, 10);
    else if (!std::strcmp(argv[i], "--out") && i + 1 < argc) out = argv[++i];
    else {
      std::fprintf(stderr, "generate: unknown option %s\n", argv[i]);
      return 1;
    }
  }
  FILE* f = std::fopen(out.c_str(), "wb");
  if (!f) {
    std::fprintf(stderr, "Error: cannot open output file: %s\n", out.c_str());
    return 1;
  }
  const unsigned long long chunk = 1ull << 26;
  std::vector<uint8_t> buf((size_t)std::min(chunk, std::max(n, 1ull)));
  for (unsigned long long off = 0; off < n; off += chunk) {
    const unsigned long long m = std::min(chunk, n - off);
    gh_generate(seed, r, off, m, buf.data(), 0);
    if (std::fwrite(buf.data(), 1, (size_t)m, f) != (size_t)m) {
      std::fclose(f);
      std::fprintf(stderr, "Error writing to file: %s\n", out.c_str());
      return 1;
    }
  }
  std::fclose(f);
  std::printf("Generated %llu bytes in %s\n", n, out.c_str());
  return 0;
}
