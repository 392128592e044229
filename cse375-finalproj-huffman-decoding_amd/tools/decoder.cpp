// bin/decoder <compressed.huff> <output> [--gpus N] [--reps R] [--json] [--verify FILE]
//
// Drop-in for the reference decoder CLI (Huffman_coding_Gap_arrays/decoder/src/
// huff.cpp:22-142, used as `./bin/decoder in out` by run_huffman.sh:38), decoding on
// MI355X through the gaphuff C ABI.  Differences from the reference, on purpose:
//   * the output goes to argv[2] (the reference always wrote "decodedfile", :32);
//   * malformed input exits non-zero with a message instead of decoding garbage;
//   * the decode kernel is timed per launch (hipEvents) instead of a wall-clock
//     span over 200 iterations + allocations (:106-129, decoder.cu:760).
// The reference's stdout lines are kept so existing log parsers keep working.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "gaphuff.h"

static double now_ms() {
  using namespace std::chrono;
  return duration<double, std::milli>(steady_clock::now().time_since_epoch()).count();
}

static int die(const char* what, int rc) {
  std::fprintf(stderr, "decoder: %s (code %d): %s\n", what, rc, gh_last_error());
  return 1;
}

int main(int argc, char** argv) {
  if (argc < 3) {
    std::fprintf(stderr,
                 "Usage: bin/decoder input output [--gpus N] [--reps R] [--json] [--verify FILE]\n");
    return 2;
  }
  int ngpus = 1, reps = 1;
  bool json = false;
  const char* verify = nullptr;
  for (int i = 3; i < argc; ++i) {
    if (!std::strcmp(argv[i], "--gpus") && i + 1 < argc) ngpus = std::atoi(argv[++i]);
    else if (!std::strcmp(argv[i], "--reps") && i + 1 < argc) reps = std::atoi(argv[++i]);
    else if (!std::strcmp(argv[i], "--json")) json = true;
    else if (!std::strcmp(argv[i], "--verify") && i + 1 < argc) verify = argv[++i];
    else {
      std::fprintf(stderr, "decoder: unknown option %s\n", argv[i]);
      return 2;
    }
  }
  if (ngpus < 1) ngpus = 1;
  if (reps < 1) reps = 1;

  FILE* f = std::fopen(argv[1], "rb");
  if (!f) {
    std::fprintf(stderr, "decoder: Could not open input file %s\n", argv[1]);
    return 1;
  }
  std::fseek(f, 0, SEEK_END);
  const long flen = std::ftell(f);
  std::fseek(f, 0, SEEK_SET);
  std::vector<uint8_t> file((size_t)std::max(flen, 0L));
  if (flen > 0 && std::fread(file.data(), 1, (size_t)flen, f) != (size_t)flen) {
    std::fclose(f);
    std::fprintf(stderr, "decoder: File read error\n");
    return 1;
  }
  std::fclose(f);

  gh_stream s;
  int rc = gh_stream_parse(file.data(), file.size(), &s);
  if (rc) return die("bad compressed stream", rc);

  std::printf("Input file: %s\n", argv[1]);
  std::printf("Original size: %llu bytes\n", (unsigned long long)s.n);
  std::printf("Compressed size: %llu bytes\n", (unsigned long long)s.w);  // reference prints W

  const int ndev = gh_device_count();
  if (ndev < 1) return die("no HIP device", GH_E_NODEV);
  if (ngpus > ndev) ngpus = ndev;

  std::vector<uint64_t> bounds(ngpus + 1);
  gh_plan_shards(s.g, (uint32_t)ngpus, bounds.data());
  std::vector<gh_ctx*> ctx(ngpus, nullptr);
  auto cleanup = [&]() {
    for (auto* c : ctx) gh_ctx_destroy(c);
  };
  const double t0 = now_ms();
  for (int k = 0; k < ngpus; ++k) {
    if ((rc = gh_ctx_create(k, &ctx[k]))) { cleanup(); return die("device init", rc); }
    if ((rc = gh_ctx_load(ctx[k], &s, bounds[k], bounds[k + 1], ngpus == 1 ? s.n : 0))) {
      cleanup();
      return die("upload", rc);
    }
  }
  const double t1 = now_ms();
  for (int r = 0; r < reps; ++r)
    for (int k = 0; k < ngpus; ++k)
      if ((rc = gh_ctx_decode(ctx[k], nullptr, 1))) { cleanup(); return die("decode", rc); }
  std::vector<gh_report> rep(ngpus);
  float dec_ms = 0;
  uint32_t status = 0;
  for (int k = 0; k < ngpus; ++k) {
    if ((rc = gh_ctx_report(ctx[k], nullptr, &rep[k]))) { cleanup(); return die("decode", rc); }
    dec_ms = std::max(dec_ms, rep[k].kernel_ms);
    status |= rep[k].status;
  }
  const double t2 = now_ms();
  std::vector<uint8_t> out((size_t)s.n + 16);
  uint64_t off = 0;
  for (int k = 0; k < ngpus; ++k) {
    const uint64_t want = off < s.n ? std::min<uint64_t>(rep[k].symbols, s.n - off) : 0;
    if (want && (rc = gh_ctx_download(ctx[k], 0, out.data() + off, want))) {
      cleanup();
      return die("download", rc);
    }
    off += rep[k].symbols;
  }
  const double t3 = now_ms();
  cleanup();
  if (status) {
    std::fprintf(stderr, "decoder: device reported status 0x%x (corrupted stream?)\n", status);
    return 1;
  }
  if (off < s.n) {
    std::fprintf(stderr, "decoder: stream decoded to %llu < N symbols\n", (unsigned long long)off);
    return 1;
  }
  std::printf("HtoD,%f, dec,%f, DtoH,%f,SEGMENTSIZE,%d,THREAD_NUM,%d,LOCAL_SEGMENT_NUM,%d\n",
              t1 - t0, dec_ms, t3 - t2, GH_SEGMENT_BITS, 256, 1);
  const double total_ms = (t1 - t0) + dec_ms + (t3 - t2);
  std::printf("Decode time: %.3f ms\n", total_ms);
  std::printf("Throughput: %.2f MB/s\n", (double)s.n / (1024.0 * 1024.0) / (total_ms / 1000.0));

  FILE* o = std::fopen(argv[2], "wb");
  if (!o) {
    std::fprintf(stderr, "decoder: Could not open output file %s\n", argv[2]);
    return 1;
  }
  if (s.n && std::fwrite(out.data(), 1, (size_t)s.n, o) != (size_t)s.n) {
    std::fclose(o);
    std::fprintf(stderr, "decoder: write error\n");
    return 1;
  }
  std::fclose(o);

  int ok = -1;
  if (verify) {
    FILE* v = std::fopen(verify, "rb");
    ok = 0;
    if (v) {
      std::vector<uint8_t> ref((size_t)s.n + 1);
      const size_t got = std::fread(ref.data(), 1, (size_t)s.n + 1, v);
      std::fclose(v);
      ok = (got == s.n && std::memcmp(ref.data(), out.data(), (size_t)s.n) == 0) ? 1 : 0;
    }
    std::printf("Verification: %s\n", ok ? "PASS" : "FAIL");
  }
  if (json) {
    const double kbytes = 4.0 * s.w + 4.0 * ((s.g + 7) / 8) + (double)s.n;
    std::printf(
        "{\"N\": %llu, \"W\": %llu, \"G\": %llu, \"gpus\": %d, \"reps\": %d, \"kernel_ms\": %.6f, "
        "\"h2d_ms\": %.3f, \"d2h_ms\": %.3f, \"decoded_GBps\": %.3f, \"alg_bytes\": %.0f, "
        "\"alg_GBps\": %.3f, \"lut_bits\": %u, \"bitexact\": %s}\n",
        (unsigned long long)s.n, (unsigned long long)s.w, (unsigned long long)s.g, ngpus, reps,
        dec_ms, t1 - t0, t3 - t2, dec_ms > 0 ? s.n / (dec_ms * 1e6) : 0.0, kbytes,
        dec_ms > 0 ? kbytes / (dec_ms * 1e6) : 0.0, rep[0].lut_bits,
        ok < 0 ? "null" : (ok ? "true" : "false"));
  }
  if (verify && !ok) return 3;
  return 0;
}
