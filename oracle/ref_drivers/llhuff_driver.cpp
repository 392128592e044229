// Driver (ours) around the REFERENCE raw-stream encoder of the self-synchronising
// decoder, compiled from the reference's own sources
// (gpuhd/encoder/src/llhuffman_encoder.cc, gpuhd/src/cuhd_codetable.cc) by
// oracle/Makefile.  Mirrors gpuhd/src/demo.cc:100-116:
//   get_symbol_lengths -> get_encoder_table -> encode_memory(compressed_size units).
// Input: the data file (argv[1]).  Output (argv[2]): u32 nsyms, nsyms x {u8 symbol,
// u8 length} in the order get_encoder_table assigns canonical codes, u64 units,
// then the units (u32 LE).
#include <cstdint>
#include <cstdio>
#include <vector>

#include "llhuffman_encoder.h"

int main(int argc, char** argv) {
  if (argc != 3) { std::fprintf(stderr, "usage: llhuff_driver data out\n"); return 2; }
  FILE* f = std::fopen(argv[1], "rb");
  if (!f) return 2;
  std::vector<std::uint8_t> data;
  std::uint8_t buf[1 << 16];
  size_t k;
  while ((k = std::fread(buf, 1, sizeof(buf), f)) > 0) data.insert(data.end(), buf, buf + k);
  std::fclose(f);
  auto lengths = llhuff::LLHuffmanEncoder::get_symbol_lengths(data.data(), data.size());
  if (!lengths) { std::fprintf(stderr, "too many symbols\n"); return 3; }
  auto table = llhuff::LLHuffmanEncoder::get_encoder_table(lengths);
  std::vector<UNIT_TYPE> units(table->compressed_size + 1, 0);
  llhuff::LLHuffmanEncoder::encode_memory(units.data(), table->compressed_size, data.data(),
                                          data.size(), table);
  FILE* o = std::fopen(argv[2], "wb");
  if (!o) return 2;
  const std::uint32_t ns = (std::uint32_t)lengths->size();
  std::fwrite(&ns, 4, 1, o);
  for (auto& s : *lengths) {
    const std::uint8_t e[2] = {s.symbol, (std::uint8_t)s.length};
    std::fwrite(e, 1, 2, o);
  }
  const std::uint64_t nu = table->compressed_size;
  std::fwrite(&nu, 8, 1, o);
  std::fwrite(units.data(), sizeof(UNIT_TYPE), nu, o);
  std::fclose(o);
  return 0;
}
