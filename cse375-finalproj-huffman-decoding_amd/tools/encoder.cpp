// bin/encoder <input> <compressed.huff> [--threads T] [--v2] [--gpu [DEVICE]] [--raw]
//
// Drop-in for the reference encoder CLI (Huffman_coding_Gap_arrays/encoder/src/
// huff.cpp:30-220): same positional arguments, same output format (v1 header when
// the sizes fit the reference's 32-bit fields, the 64-bit v2 header otherwise), and
// the same stdout lines (:176-181).  Encoding runs on the host through the gaphuff C
// ABI, or with --gpu on a gfx950 device (gh_ectx_*, byte-identical output; the
// reference's own encoder is a GPU one, encoder.cu:382-457).
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
  int threads = 0, force = 0, gpu = -1;
  bool raw = false;  // write the gap-less raw-stream container (GH_RAW_MAGIC) instead
  for (int i = 3; i < argc; ++i) {
    if (!std::strcmp(argv[i], "--threads") && i + 1 < argc) threads = std::atoi(argv[++i]);
    else if (!std::strcmp(argv[i], "--v2")) force = 2;
    else if (!std::strcmp(argv[i], "--raw")) raw = true;
    else if (!std::strcmp(argv[i], "--gpu")) gpu = (i + 1 < argc && argv[i + 1][0] != '-') ? std::atoi(argv[++i]) : 0;
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
  gh_encode_plan* plan = new gh_encode_plan;
  std::vector<uint8_t> out;
  double t0, t1, t2;
  int rc;
  if (gpu >= 0) {
    gh_ectx* e = nullptr;
    float ms = 0.f;
    rc = gh_ectx_create(gpu, &e);
    if (!rc) rc = gh_ectx_load(e, in.data(), in.size());
    t0 = now_ms();
    if (!rc) rc = gh_ectx_plan(e, force, plan);
    if (!rc) rc = gh_ectx_encode(e, &ms);
    t2 = now_ms();
    t1 = t2 - ms;  // "kernel time": the device encode's event time
    if (!rc) {
      out.resize(plan->file_bytes);
      rc = gh_ectx_download(e, out.data(), out.size());
    }
    if (rc) {
      std::fprintf(stderr, "encoder: %s\n", gh_last_error());
      return 1;
    }
    gh_ectx_destroy(e);
  } else {
    t0 = now_ms();
    rc = gh_encode_plan_make(in.data(), in.size(), threads, force, plan);
    if (rc) {
      std::fprintf(stderr, "encoder: %s\n", gh_last_error());
      return 1;
    }
    out.resize(plan->file_bytes);
    t1 = now_ms();
    rc = gh_encode_write(in.data(), plan, threads, out.data(), out.size());
    if (rc) {
      std::fprintf(stderr, "encoder: %s\n", gh_last_error());
      return 1;
    }
    t2 = now_ms();
  }
  if (raw) {  // same code and payload words, no gap array
    gh_stream st;
    if (gh_stream_parse(out.data(), out.size(), &st)) {
      std::fprintf(stderr, "encoder: %s\n", gh_last_error());
      return 1;
    }
    std::vector<uint8_t> r;
    auto put = [&](uint64_t x) {
      for (int i = 0; i < 8; ++i) r.push_back((uint8_t)(x >> (8 * i)));
    };
    put(GH_RAW_MAGIC);
    put(st.nsyms);
    for (uint32_t i = 0; i < st.nsyms; ++i) {
      r.push_back(st.syms[i].symbol);
      r.push_back(st.syms[i].length);
    }
    put(st.n);
    put(st.w);
    const uint8_t* pw = (const uint8_t*)st.payload;
    r.insert(r.end(), pw, pw + 4 * st.w);
    out.swap(r);
  }
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
