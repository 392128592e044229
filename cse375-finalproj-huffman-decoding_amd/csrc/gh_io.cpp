// gh_io.cpp — streaming file I/O around a decode context.
//
// The reference reads the whole compressed.huff into pinned memory with fread, then
// copies it to the device with synchronous cudaMemcpy (decoder/src/huff.cpp:90-100,
// decoder.cu:759-768), and copies the whole output back before fwrite (huff.cpp:
// 121-140).  Here the file's gap words and the shard's payload words go through two
// pinned staging buffers: the read of chunk c+1 overlaps the H2D DMA of chunk c.  The
// output goes the other way: the D2H of chunk c+1 overlaps the pwrite of chunk c.
// Each shard (gh_ctx) reads only its own payload range, and writes its decoded bytes
// at its offset in the output file, so shards of one stream can load and store
// independently (one process or thread per GPU).
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <map>
#include <mutex>
#include <thread>
#include <cstring>
#include <string>
#include <vector>

#include "gh_internal.hpp"

namespace gh {
namespace {

constexpr size_t IO_CHUNK = 32ull << 20;  // bytes per staging buffer
constexpr size_t HDR_MAX = 8 + 8 + 2 * GH_MAX_SYMBOLS + 24;

#define GH_HIPI(expr)                                                             \
  do {                                                                            \
    hipError_t e_ = (expr);                                                       \
    if (e_ != hipSuccess)                                                         \
      return fail(GH_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));   \
  } while (0)

double now_ms() {
  using namespace std::chrono;
  return duration<double, std::milli>(steady_clock::now().time_since_epoch()).count();
}

struct Fd {
  int fd = -1;
  ~Fd() {
    if (fd >= 0) close(fd);
  }
};

// Two pinned buffers, a stream and one event per buffer, per device.  Pinning 64 MiB
// costs tens of milliseconds, so the buffers are kept for the life of the process and
// handed to one call at a time.
struct Staging {
  void* buf[2] = {nullptr, nullptr};
  hipEvent_t ev[2] = {nullptr, nullptr};
  hipStream_t st = nullptr;
  bool ready() const { return st && buf[0] && buf[1] && ev[0] && ev[1]; }
  // Frees whatever a failed init() left (a set is pooled only when ready()).
  void release() {
    for (int i = 0; i < 2; ++i) {
      if (ev[i]) (void)hipEventDestroy(ev[i]);
      if (buf[i]) (void)hipHostFree(buf[i]);
      ev[i] = nullptr;
      buf[i] = nullptr;
    }
    if (st) (void)hipStreamDestroy(st);
    st = nullptr;
  }
  int init() {
    if (ready()) return GH_OK;
    release();
    int rc = init_parts();
    if (rc) release();
    return rc;
  }
  int init_parts() {
    GH_HIPI(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    for (int i = 0; i < 2; ++i) {
      GH_HIPI(hipHostMalloc(&buf[i], IO_CHUNK, hipHostMallocDefault));
      GH_HIPI(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming));
    }
    return GH_OK;
  }
};

std::mutex g_pool_mu;
std::condition_variable g_pool_cv;
std::map<int, std::vector<Staging*>> g_pool;  // device -> idle staging sets (never freed)
std::map<int, int> g_live;                    // device -> sets checked out
// Sets per device in use at once: two double-buffered sets keep one device's PCIe link
// busy while a third call waits; more only cost pinning (~25 ms per 64 MiB set).
constexpr int SETS_PER_DEV = 2;

// Takes an idle staging set of the device (or makes one, up to SETS_PER_DEV per device;
// a further concurrent call on that device waits for one) for the duration of a call.
struct StagingLease {
  int dev;
  Staging* s = nullptr;
  bool counted = false;
  explicit StagingLease(int d) : dev(d) {}
  int acquire() {
    {
      std::unique_lock<std::mutex> g(g_pool_mu);
      g_pool_cv.wait(g, [&] { return g_live[dev] < SETS_PER_DEV; });
      ++g_live[dev];
      counted = true;
      auto& v = g_pool[dev];
      if (!v.empty()) {
        s = v.back();
        v.pop_back();
      }
    }
    if (!s) s = new Staging();
    return s->init();
  }
  ~StagingLease() {
    // an error return may leave copies of this call in flight: drain them before the
    // caller frees their buffers or the set goes back to the pool
    if (s && s->st) (void)hipStreamSynchronize(s->st);
    {
      std::lock_guard<std::mutex> g(g_pool_mu);
      if (counted) --g_live[dev];
      if (s) {
        auto& v = g_pool[dev];
        if (v.size() < (size_t)SETS_PER_DEV && s->ready()) {
          v.push_back(s);
          s = nullptr;
        }
      }
    }
    g_pool_cv.notify_all();
    if (s) {
      s->release();
      delete s;
    }
  }
};

bool read_full(int fd, void* dst, size_t n, uint64_t off) {
  uint8_t* p = (uint8_t*)dst;
  while (n) {
    const ssize_t r = pread(fd, p, n, (off_t)off);
    if (r <= 0) return false;
    p += r;
    n -= (size_t)r;
    off += (uint64_t)r;
  }
  return true;
}

bool write_full(int fd, const void* src, size_t n, uint64_t off) {
  const uint8_t* p = (const uint8_t*)src;
  while (n) {
    const ssize_t r = pwrite(fd, p, n, (off_t)off);
    if (r <= 0) return false;
    p += r;
    n -= (size_t)r;
    off += (uint64_t)r;
  }
  return true;
}

// A chunk's reads split over IO_THREADS threads (one page-cache copy stream per
// thread runs at a few GB/s).
constexpr int IO_THREADS = 4;
template <class F>
bool par_io(size_t n, F f) {
  if (n < (4u << 20)) return f(0, n);
  std::atomic<bool> ok{true};
  std::vector<std::thread> th;
  const size_t part = ((n + IO_THREADS - 1) / IO_THREADS + 4095) & ~size_t(4095);
  for (int i = 0; i < IO_THREADS; ++i) {
    const size_t a = std::min(n, i * part), b = std::min(n, a + part);
    if (a < b) th.emplace_back([&, a, b] { if (!f(a, b - a)) ok = false; });
  }
  for (auto& t : th) t.join();
  return ok;
}

// File bytes [off, off+n) -> device dst, double-buffered.
int stream_h2d(Staging& s, int fd, uint64_t off, uint64_t n, uint8_t* dst) {
  int b = 0;
  for (uint64_t done = 0; done < n; b ^= 1) {
    const size_t c = (size_t)std::min<uint64_t>(IO_CHUNK, n - done);
    GH_HIPI(hipEventSynchronize(s.ev[b]));  // the DMA that last used this buffer
    uint8_t* hb = (uint8_t*)s.buf[b];
    const uint64_t base = off + done;
    if (!par_io(c, [&](size_t a, size_t m) { return read_full(fd, hb + a, m, base + a); }))
      return fail(GH_E_FORMAT, "short read of the stream file");
    GH_HIPI(hipMemcpyAsync(dst + done, s.buf[b], c, hipMemcpyHostToDevice, s.st));
    GH_HIPI(hipEventRecord(s.ev[b], s.st));
    done += c;
  }
  GH_HIPI(hipStreamSynchronize(s.st));
  return GH_OK;
}

struct DevMem {
  void* p = nullptr;
  ~DevMem() { (void)hipFree(p); }
};

}  // namespace

bool use_staged(uint64_t n) {
  static const bool pageable = [] {
    const char* e = getenv("GH_H2D");
    return e && !strcmp(e, "pageable");
  }();
  return !pageable && n >= (8u << 20);
}

// Host bytes -> device, double-buffered: the host copy of chunk c+1 (split over
// IO_THREADS threads) overlaps the DMA of chunk c.
int h2d_staged(int device, const void* src, uint64_t n, void* dst) {
  GH_HIPI(hipSetDevice(device));
  StagingLease lease(device);
  int rc = lease.acquire();
  if (rc) return rc;
  Staging& s = *lease.s;
  int b = 0;
  for (uint64_t done = 0; done < n; b ^= 1) {
    const size_t c = (size_t)std::min<uint64_t>(IO_CHUNK, n - done);
    GH_HIPI(hipEventSynchronize(s.ev[b]));  // the DMA that last used this buffer
    uint8_t* hb = (uint8_t*)s.buf[b];
    const uint8_t* sp = (const uint8_t*)src + done;
    par_io(c, [&](size_t a, size_t m) { std::memcpy(hb + a, sp + a, m); return true; });
    GH_HIPI(hipMemcpyAsync((uint8_t*)dst + done, hb, c, hipMemcpyHostToDevice, s.st));
    GH_HIPI(hipEventRecord(s.ev[b], s.st));
    done += c;
  }
  GH_HIPI(hipStreamSynchronize(s.st));
  return GH_OK;
}

// Device bytes -> host: the DMA of chunk c+1 overlaps the host copy of chunk c.
int d2h_staged(int device, const void* src, uint64_t n, void* dst) {
  GH_HIPI(hipSetDevice(device));
  StagingLease lease(device);
  int rc = lease.acquire();
  if (rc) return rc;
  Staging& s = *lease.s;
  uint64_t pend_off = 0;
  size_t pend_n = 0;
  int pend_b = -1, b = 0;
  for (uint64_t done = 0;; b ^= 1) {
    const size_t c = (size_t)std::min<uint64_t>(IO_CHUNK, n - done);
    if (c) {
      GH_HIPI(hipMemcpyAsync(s.buf[b], (const uint8_t*)src + done, c, hipMemcpyDeviceToHost, s.st));
      GH_HIPI(hipEventRecord(s.ev[b], s.st));
    }
    if (pend_b >= 0) {
      GH_HIPI(hipEventSynchronize(s.ev[pend_b]));
      const uint8_t* hb = (const uint8_t*)s.buf[pend_b];
      uint8_t* dp = (uint8_t*)dst + pend_off;
      par_io(pend_n, [&](size_t a, size_t m) { std::memcpy(dp + a, hb + a, m); return true; });
    }
    if (!c) break;
    pend_b = b;
    pend_off = done;
    pend_n = c;
    done += c;
  }
  return GH_OK;
}

}  // namespace gh

using namespace gh;

extern "C" int gh_ctx_load_file(gh_ctx* ctx, const char* path, uint64_t seg_begin, uint64_t seg_end,
                                uint64_t out_cap, gh_file_info* info) {
  if (!ctx || !path) return fail(GH_E_ARG, "null argument");
  const double t0 = now_ms();
  Fd f;
  f.fd = open(path, O_RDONLY);
  if (f.fd < 0) return fail(GH_E_ARG, std::string("cannot open ") + path);
  struct stat stt;
  if (fstat(f.fd, &stt) != 0) return fail(GH_E_ARG, std::string("cannot stat ") + path);
  const uint64_t flen = (uint64_t)stt.st_size;
  uint8_t hdr[HDR_MAX + 8] = {};
  const size_t hn = (size_t)std::min<uint64_t>(flen, HDR_MAX);
  if (hn && !read_full(f.fd, hdr, hn, 0)) return fail(GH_E_FORMAT, "cannot read the header");
  // gh_stream_parse dereferences only the header; the file length bounds the rest
  gh_stream s;
  int rc = gh_stream_parse(hdr, (size_t)flen, &s);
  if (rc) return rc;
  if (seg_end == UINT64_MAX) seg_end = s.g;
  if (seg_begin > seg_end || seg_end > s.g) return fail(GH_E_ARG, "shard range outside [0, G]");
  const uint64_t gap_off = (uint64_t)((const uint8_t*)s.gap_words - hdr);
  const uint64_t gw = ceil_div(s.g, GH_GAPS_PER_WORD);
  const uint64_t pay_off = gap_off + 4 * gw;
  int dev = 0;
  if ((rc = gh_ctx_device(ctx, &dev))) return rc;
  GH_HIPI(hipSetDevice(dev));
  // the shard's payload words [4b, 4e+1) clipped at W, and the whole gap array
  const uint64_t w0 = std::min<uint64_t>(4 * seg_begin, s.w);
  const uint64_t w1 = std::min<uint64_t>(4 * seg_end + 1, s.w);
  DevMem dpay, dgap;
  GH_HIPI(hipMalloc(&dpay.p, 4 * (w1 - w0) + 64));
  GH_HIPI(hipMalloc(&dgap.p, 4 * gw + 64));
  StagingLease lease(dev);
  if ((rc = lease.acquire())) return rc;
  Staging& stg = *lease.s;
  const double t1 = now_ms();
  if ((rc = stream_h2d(stg, f.fd, gap_off, 4 * gw, (uint8_t*)dgap.p))) return rc;
  if ((rc = stream_h2d(stg, f.fd, pay_off + 4 * w0, 4 * (w1 - w0), (uint8_t*)dpay.p))) return rc;
  const double t2 = now_ms();
  // copy the (<= 256-entry) symbol list: s.syms points into hdr
  gh_sym syms[GH_MAX_SYMBOLS];
  std::memcpy(syms, s.syms, 2 * s.nsyms);
  gh_stream hs = s;
  hs.syms = syms;
  hs.gap_words = nullptr;
  hs.payload = nullptr;
  rc = gh_ctx_load_device(ctx, &hs, seg_begin, seg_end, (const uint32_t*)dpay.p, w1 - w0,
                          (const uint32_t*)dgap.p, out_cap);
  if (rc) return rc;
  if (info) {
    std::memset(info, 0, sizeof(*info));
    info->n = s.n;
    info->w = s.w;
    info->g = s.g;
    info->nsyms = s.nsyms;
    info->version = s.version;
    info->bytes_read = gap_off + 4 * gw + 4 * (w1 - w0);
    info->setup_ms = t1 - t0;
    info->transfer_ms = t2 - t1;
    info->total_ms = now_ms() - t0;
  }
  return GH_OK;
}

extern "C" int gh_ctx_save_file(gh_ctx* ctx, const char* path, uint64_t file_offset, uint64_t byte_offset,
                                uint64_t nbytes, int truncate, double* ms) {
  if (!ctx || !path) return fail(GH_E_ARG, "null argument");
  const double t0 = now_ms();
  void* dout = nullptr;
  uint64_t cap = 0;
  int rc = gh_ctx_output(ctx, &dout, &cap);
  if (rc) return rc;
  if (byte_offset > cap || nbytes > cap - byte_offset) return fail(GH_E_ARG, "save beyond the output capacity");
  int dev = 0;
  if ((rc = gh_ctx_device(ctx, &dev))) return rc;
  GH_HIPI(hipSetDevice(dev));
  Fd f;
  f.fd = open(path, O_WRONLY | O_CREAT | (truncate ? O_TRUNC : 0), 0644);
  if (f.fd < 0) return fail(GH_E_ARG, std::string("cannot open ") + path + " for writing");
  // the decode was enqueued on the context's stream: wait for it
  gh_report rep;
  if ((rc = gh_ctx_report(ctx, nullptr, &rep))) return rc;
  StagingLease lease(dev);
  if ((rc = lease.acquire())) return rc;
  Staging& stg = *lease.s;
  const uint8_t* src = (const uint8_t*)dout + byte_offset;
  // D2H of chunk c+1 overlaps the write of chunk c
  uint64_t pend_off = 0;
  size_t pend_n = 0;
  int pend_b = -1, b = 0;
  for (uint64_t done = 0;; b ^= 1) {
    const size_t c = (size_t)std::min<uint64_t>(IO_CHUNK, nbytes - done);
    if (c) {
      GH_HIPI(hipMemcpyAsync(stg.buf[b], src + done, c, hipMemcpyDeviceToHost, stg.st));
      GH_HIPI(hipEventRecord(stg.ev[b], stg.st));
    }
    if (pend_b >= 0) {
      GH_HIPI(hipEventSynchronize(stg.ev[pend_b]));
      const uint8_t* hb = (const uint8_t*)stg.buf[pend_b];
      const uint64_t base = file_offset + pend_off;
      const int fd = f.fd;
      // one writer: concurrent pwrites to one file serialise on its inode lock and
      // measured slower than a single stream of 32 MiB writes
      if (!write_full(fd, hb, pend_n, base))
        return fail(GH_E_ARG, std::string("write error on ") + path);
    }
    if (!c) break;
    pend_b = b;
    pend_off = done;
    pend_n = c;
    done += c;
  }
  if (ms) *ms = now_ms() - t0;
  return GH_OK;
}

extern "C" int gh_raw_parse(const void* file, size_t len, gh_raw_stream* out) {
  if (!file || !out) return fail(GH_E_ARG, "null argument");
  const uint8_t* p = (const uint8_t*)file;
  auto rd64 = [&](size_t o) {
    uint64_t v;
    std::memcpy(&v, p + o, 8);
    return v;
  };
  if (len < 16 || rd64(0) != GH_RAW_MAGIC) return fail(GH_E_FORMAT, "not a raw-stream container");
  const uint64_t ns = rd64(8);
  if (ns > GH_MAX_SYMBOLS) return fail(GH_E_FORMAT, "symbol count > 256");
  size_t off = 16 + 2 * ns;
  if (len < off + 16) return fail(GH_E_FORMAT, "truncated raw-stream header");
  gh_raw_stream r{};
  r.syms = (const gh_sym*)(p + 16);
  r.nsyms = (uint32_t)ns;
  r.n = rd64(off);
  r.w = rd64(off + 8);
  off += 16;
  if (r.w > (len - off) / 4) return fail(GH_E_FORMAT, "file shorter than its units");
  r.units = (const uint32_t*)(p + off);
  Canon c;
  int rc = build_canon(r.syms, r.nsyms, c);
  if (rc) return rc;
  // every symbol takes at least minlen bits: N symbols cannot fit fewer units
  if (r.n && (c.minlen == 0 || r.n > (32 * r.w) / c.minlen))
    return fail(GH_E_FORMAT, "raw stream holds fewer bits than N symbols need");
  *out = r;
  return GH_OK;
}
