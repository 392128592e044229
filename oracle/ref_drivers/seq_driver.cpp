// Driver (ours) around the REFERENCE string-format codec (sequential.cpp's
// HuffmanSequential::encode / decode, sequential.cpp:17-204), compiled from the
// reference's own source by oracle/Makefile (its main() is renamed out of the way).
//   seq_driver enc <data> <out.seq>      seq_driver dec <in.seq> <out.bin>
#define main reference_sequential_main
#include "sequential.cpp"
#undef main

#include <cstdio>
#include <cstring>

int main(int argc, char** argv) {
  if (argc != 4) { std::fprintf(stderr, "usage: seq_driver enc|dec in out\n"); return 2; }
  HuffmanSequential h;
  std::vector<uint8_t> in = read_file_to_vector(argv[2]);
  std::vector<uint8_t> out = !std::strcmp(argv[1], "enc") ? h.encode(in) : h.decode(in);
  FILE* f = std::fopen(argv[3], "wb");
  if (!f) return 2;
  if (!out.empty()) std::fwrite(out.data(), 1, out.size(), f);
  std::fclose(f);
  return 0;
}
