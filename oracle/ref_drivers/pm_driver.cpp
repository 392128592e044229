// Driver (ours) around the REFERENCE code-length builder, compiled from the
// reference's own sources (encoder/src/package_merge.cpp, symbols.cpp) by
// oracle/Makefile.  Mirrors encoder/src/huff.cpp:114-116 + :189-194:
//   store_symbols -> qsort(ascending count) -> boundary_PM -> file order.
// Input: a binary file of 256 little-endian u32 counts (argv[1]).
// Output: one "symbol length" line per symbol, most frequent first.
#include <cstdio>
#include <cstdlib>
#include "constants.hpp"
#include "package_merge.hpp"
#include "symbols.hpp"

static int by_count(const void* p, const void* q) {  // huff.cpp:18-22 semantics
  const Symbol* a = (const Symbol*)p;
  const Symbol* b = (const Symbol*)q;
  return a->num - b->num;
}

int main(int argc, char** argv) {
  if (argc != 2) { std::fprintf(stderr, "usage: pm_driver counts.bin\n"); return 2; }
  FILE* f = std::fopen(argv[1], "rb");
  if (!f) return 2;
  unsigned int counts[MAX_CODE_NUM] = {};
  if (std::fread(counts, sizeof(unsigned int), MAX_CODE_NUM, f) != MAX_CODE_NUM) return 2;
  std::fclose(f);
  struct Symbol symbols[MAX_CODE_NUM] = {};
  struct Codetable table[MAX_CODE_NUM] = {};
  int n = store_symbols(counts, symbols);
  if (n < 2) { std::fprintf(stderr, "need >= 2 symbols\n"); return 3; }
  std::qsort(symbols, n, sizeof(struct Symbol), by_count);
  boundary_PM(symbols, n, table);
  for (int i = n - 1; i >= 0; i--) std::printf("%d %d\n", symbols[i].symbol, symbols[i].length);
  return 0;
}
