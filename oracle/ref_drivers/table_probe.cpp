// Driver (ours) around the REFERENCE decode-table builder (decoder/src/get_table.cpp,
// compiled from the reference's own sources by oracle/Makefile).  Mirrors
// decoder/src/huff.cpp:53-79: prefix_bit is fixed at FIXED_PREFIX_BIT (10).
// Input (argv[1]): text "symbol length" lines in file order.
// Output (stdout, binary): u32 l1, u32 l2, u32 ptr, u32 table_bytes, table bytes.
// Only streams whose longest code exceeds 10 bits are accepted: for shorter codes
// the reference fills a 10-bit level-1 table into a 2^maxlen buffer (heap
// overflow), which this probe refuses to execute.
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "constants.hpp"
#include "get_table.h"

int main(int argc, char** argv) {
  if (argc != 2) return 2;
  FILE* f = std::fopen(argv[1], "r");
  if (!f) return 2;
  std::vector<Symbol> syms;
  int s, l;
  while (std::fscanf(f, "%d %d", &s, &l) == 2) {
    Symbol x{};
    x.symbol = (unsigned char)s;
    x.length = (unsigned char)l;
    syms.push_back(x);
  }
  std::fclose(f);
  int n = (int)syms.size();
  if (n < 2 || syms[n - 1].length <= FIXED_PREFIX_BIT) { std::fprintf(stderr, "UNSUPPORTED\n"); return 3; }
  TableInfo info{};
  unsigned int bit = get_table_info(syms.data(), n, FIXED_PREFIX_BIT, info);
  if (bit != FIXED_PREFIX_BIT) { std::fprintf(stderr, "UNSUPPORTED\n"); return 3; }
  unsigned int bytes = sizeof(int) * info.ptrtable_size + MAX_CODE_NUM + info.l1table_size + info.l2table_size;
  std::vector<unsigned char> table(bytes + 64, 0);
  get_twolevel_table(table.data(), FIXED_PREFIX_BIT, syms.data(), n, info);
  unsigned int hdr[4] = {info.l1table_size, info.l2table_size, info.ptrtable_size, bytes};
  std::fwrite(hdr, sizeof(hdr), 1, stdout);
  std::fwrite(table.data(), 1, bytes, stdout);
  return 0;
}
