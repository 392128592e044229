// bin/encoder <input> <compressed.huff> [--threads T] [--v2]
//
// Drop-in for the reference encoder CLI (Huffman_coding_Gap_arrays/encoder/src/
// huff.cpp:30-220): same positional arguments, same output format (v1 header when
// the sizes fit the reference's 32-bit fields, the 64-bit v2 header otherwise), and
// the same stdout lines (:176-181).  Encoding runs on the host through the gaphuff C
// ABI (the GPU encoder is the next hot path).
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "gaphuff.h"

static double now_ms() {
  using namespace std::chrono;
  return duration<double, std::milli>(steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  if (argc < 3) {
    std::printf("Usage: bin/encoder input output\n");
    return 1;
  }
  int threads = 0, force = 0;
  for (int i = 3; i < argc; ++i) {
    if (!std::strcmp(argv[i], "--threads") && i + 1 < argc) threads = std::atoi(argv[++i]);
    else if (!std::strcmp(argv[i], "--v2")) force = 2;
    else {
      std::fprintf(stderr, "encoder: unknown option %s\n", argv[i]);
      return 2;
    }
  }
  FILE* f = std::fopen(argv[1], "rb");
  if (!f) {
    std::fprintf(stderr, "Could not open input file\n");
    return 1;
  }
  std::fseek(f, 0, SEEK_END);
  const long n = std::ftell(f);
  std::fseek(f, 0, SEEK_SET);
  std::vector<uint8_t> in((size_t)std::max(n, 0L));
  if (n > 0 && std::fread(in.data(), 1, (size_t)n, f) != (size_t)n) {
    std::fclose(f);
    std::fprintf(stderr, "File read error\n");
    return 1;
  }
  std::fclose(f);
  const double t0 = now_ms();
  gh_encode_plan* plan = new gh_encode_plan;
  int rc = gh_encode_plan_make(in.data(), in.size(), threads, force, plan);
  if (rc) {
    std::fprintf(stderr, "encoder: %s\n", gh_last_error());
    return 1;
  }
  std::vector<uint8_t> out(plan->file_bytes);
  const double t1 = now_ms();
  rc = gh_encode_write(in.data(), plan, threads, out.data(), out.size());
  if (rc) {
    std::fprintf(stderr, "encoder: %s\n", gh_last_error());
    return 1;
  }
  const double t2 = now_ms();
  FILE* o = std::fopen(argv[2], "wb");
  if (!o) {
    std::fprintf(stderr, "Could not open output file\n");
    return 1;
  }
  if (!out.empty() && std::fwrite(out.data(), 1, out.size(), o) != out.size()) {
    std::fclose(o);
    std::fprintf(stderr, "write error\n");
    return 1;
  }
  std::fclose(o);
  std::printf("Input file: %s\n", argv[1]);
  std::printf("Original size: %llu bytes\n", (unsigned long long)plan->n);
  std::printf("Compressed size: %llu bytes\n", (unsigned long long)(plan->w * 4));
  std::printf("Encode kernel time: %.3f ms\n", t2 - t1);
  std::printf("Total encode time: %.3f ms\n", t2 - t0);
  std::printf("Throughput: %.2f MB/s\n",
              (double)plan->n / (1024.0 * 1024.0) / std::max(1e-9, (t2 - t0) / 1000.0));
  delete plan;
  return 0;
}
