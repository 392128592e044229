/*
 * gaphuff.h — C ABI of the MI355X-native gap-array Huffman codec.
 *
 * This is the drop-in boundary for the reference's decode path
 * (dek226/CSE375-FinalProj-Huffman-Decoding, Huffman_coding_Gap_arrays/):
 *
 *   reference                                   replaced by
 *   ------------------------------------------  --------------------------------------
 *   decoder/src/huff.cpp:36-100  (header+table   gh_stream_parse()  — parses v1/v2 files
 *        parse, fread of gap words + payload)
 *   decoder/src/get_table.cpp:3-139              built inside the library from the
 *        (get_table_info / get_twolevel_table)   (symbol,length) list (see gh_ctx_load)
 *   decoder/include/decoder.cuh:4-15             gh_decode()        — one-shot decode
 *        decoder_l1_l2(input, W, output, N, G,   gh_ctx_*()         — device-resident
 *        dectable, tablesize, prefix_bit, S,                          decode (bench/CLI)
 *        TableInfo)   [decoder.cu:732-815]
 *   decoder.cu:454-730 gpu_dec_l1_l2 kernel      HIP kernel gh_decode_kernel (gfx950)
 *   parallel_cpu_prescan.cpp:423-483             gh_decode() (count+scan on the GPU)
 *   gpuhd/src/cuhd_gpu_decoder.cu:16-523         (same kernel; self-sync format: next;
 *        and its gpuhd-gapArray / gpuhd-multigpu copies)
 *   encoder/src/huff.cpp:30-220 (+encoder.cu,    gh_encode_plan()/gh_encode_write()
 *        package_merge.cpp, symbols.cpp)          (host encoder of the same format)
 *   generate.cpp:11-58                           gh_generate()      — seeded generator
 *
 * Conventions: plain C types only; every entry point returns 0 (GH_OK) or a
 * negative GH_E_* code and never exits the process (the reference calls exit()
 * via CUERROR/fatal, decoder.cu:14-20, huff.cpp:11-14).  Buffers are owned by the
 * caller unless stated.  A gh_ctx is bound to one HIP device and must be used from
 * one host thread at a time.
 */
#ifndef GAPHUFF_H_
#define GAPHUFF_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GH_ABI_VERSION 1

/* ---- status codes ---------------------------------------------------------- */
#define GH_OK 0
#define GH_E_ARG -1       /* bad argument / NULL pointer / out-of-range shard      */
#define GH_E_FORMAT -2    /* malformed compressed.huff header or sizes             */
#define GH_E_TABLE -3     /* (symbol,length) list is not a valid canonical code     */
#define GH_E_HIP -4       /* HIP runtime error                                      */
#define GH_E_NODEV -5     /* no usable gfx950 device                                */
#define GH_E_NOMEM -6     /* host or device allocation failed                       */
#define GH_E_CORRUPT -7   /* stream decoded to fewer symbols than N, or bad code    */
#define GH_E_STATE -8     /* context used out of order                              */
#define GH_E_SMALL -9     /* caller buffer too small                                */

/* ---- constants of the on-disk format (reference constants.hpp) ------------- */
#define GH_SEGMENT_BITS 128   /* decoder/include/constants.hpp:9  SEGMENT_SIZE       */
#define GH_GAPS_PER_WORD 8    /* constants.hpp:22  GAP_FAC_NUM (4-bit gaps per u32)  */
#define GH_MAX_CODE_LEN 16    /* constants.hpp:5   MAX_CODEWORD_LENGTH               */
#define GH_MAX_SYMBOLS 256    /* constants.hpp:6   MAX_CODE_NUM                      */
/* v2 header magic ("GAPHUF2\0" little-endian); a v1 file starts with u64 S <= 256 */
#define GH_V2_MAGIC 0x0032465548504147ull

/* One header entry: reference struct Symbol{symbol,length} as written by
 * encoder/src/huff.cpp:189-194 (most frequent symbol first). */
typedef struct gh_sym {
  uint8_t symbol;
  uint8_t length;
} gh_sym;

/* A parsed compressed stream.  All pointers are views (no ownership). */
typedef struct gh_stream {
  const gh_sym* syms;         /* nsyms entries, file order                         */
  uint32_t nsyms;             /* S                                                 */
  uint32_t version;           /* 1 = reference v1 header, 2 = 64-bit v2 header     */
  uint64_t n;                 /* original bytes N (decoder/src/huff.cpp:83)        */
  uint64_t w;                 /* payload u32 words W (huff.cpp:85)                 */
  uint64_t g;                 /* 128-bit segments G (huff.cpp:87)                  */
  const uint32_t* gap_words;  /* ceil(G/8) words, 4-bit gaps LSB-first             */
  const uint32_t* payload;    /* W words, codewords MSB-first within each word     */
} gh_stream;

/* ---- format ----------------------------------------------------------------- */
/* Parse a whole compressed.huff image (v1 or v2).  The stream's pointers alias
 * `file`.  Validates sizes (W in [4G-3,4G], lengths 1..16, Kraft sum <= 1). */
int gh_stream_parse(const void* file, size_t file_len, gh_stream* out);
/* Validate a stream's code table (canonical order, lengths, distinct symbols). */
int gh_stream_validate(const gh_stream* s);

/* ---- encoder (host; reference encoder/src/huff.cpp:30-220) ------------------ */
typedef struct gh_encode_plan {
  uint64_t n;                       /* input bytes                                  */
  uint64_t bits;                    /* total code bits = sum len*count              */
  uint64_t w, g;                    /* payload words, segments                      */
  uint64_t file_bytes;              /* size of the compressed image                 */
  uint32_t nsyms;                   /* distinct symbols                             */
  uint32_t version;                 /* 1 or 2 (v2 when N, W or G >= 2^31)           */
  gh_sym syms[GH_MAX_SYMBOLS];      /* file order, most frequent first              */
  uint32_t code[GH_MAX_SYMBOLS];    /* canonical code per byte value                */
  uint8_t len[GH_MAX_SYMBOLS];      /* code length per byte value (0 = absent)      */
  uint64_t count[GH_MAX_SYMBOLS];   /* histogram                                    */
} gh_encode_plan;
/* Histogram + boundary package-merge (length limit 16) + canonical codes.
 * threads <= 0 selects all hardware threads.  force_version 0 = automatic. */
int gh_encode_plan_make(const uint8_t* in, uint64_t n, int threads, int force_version,
                        gh_encode_plan* plan);
/* Write the compressed image (plan->file_bytes bytes) into `out`. */
int gh_encode_write(const uint8_t* in, const gh_encode_plan* plan, int threads,
                    void* out, uint64_t out_len);
/* Code lengths only: boundary package-merge over `nsyms` counts sorted ascending
 * (stable), restating encoder/src/package_merge.cpp:107-166; lengths written in
 * the same (ascending-count) order. */
int gh_package_merge(const uint64_t* sorted_counts, uint32_t nsyms, uint8_t* lengths);

/* ---- synthetic input (reference generate.cpp:32-47, seeded) ----------------- */
/* Byte i: with probability `redundancy` 'A'+U{0..3}, else U{0..255}; counter-based
 * PRNG keyed by (seed, i) so any [offset, offset+n) slice is reproducible. */
int gh_generate(uint64_t seed, double redundancy, uint64_t offset, uint64_t n,
                uint8_t* out, int threads);

/* ---- GPU encoder ------------------------------------ */
/* Replaces the reference's GPU encoder: histogram (encoder/src/encoder.cu:118-140),
 * cuencoder (:142-355) and cu_get_gaparray (:358-379) behind encoder/src/huff.cpp:
 * 30-220.  The image is byte-identical to gh_encode_write's.  The code lengths are
 * built on the host (package-merge) from the GPU histogram.  An encoder context is
 * bound to one gfx950 device; no CPU fallback. */
typedef struct gh_ectx gh_ectx;
int gh_ectx_create(int device, gh_ectx** out);
int gh_ectx_destroy(gh_ectx* ctx);
/* Copy n input bytes to the device (kept resident across plan/encode calls). */
int gh_ectx_load(gh_ectx* ctx, const uint8_t* in, uint64_t n);
/* GPU histogram + host package-merge; fills *plan (may be NULL). */
int gh_ectx_plan(gh_ectx* ctx, int force_version, gh_encode_plan* plan);
/* Encode the loaded input on the device; kernel_ms (may be NULL): event time of the
 * encode kernels, input already resident. */
int gh_ectx_encode(gh_ectx* ctx, float* kernel_ms);
/* Header + gap words + payload words into out (plan->file_bytes bytes). */
int gh_ectx_download(gh_ectx* ctx, void* out, uint64_t out_len);

/* ---- GPU decoder -------------------------------------------------------------- */
typedef struct gh_ctx gh_ctx;

typedef struct gh_report {
  uint64_t symbols;        /* symbols decoded by the loaded shard (incl. padding)  */
  uint64_t out_bytes;      /* bytes written to the shard's device output           */
  uint32_t status;         /* device status bits (GH_ST_*)                          */
  uint32_t lut_bits;       /* K of the decode lookup table (write table: wave split) */
  uint32_t grid;           /* workgroups launched (write kernel in split mode)      */
  uint32_t tiles;          /* segment tiles in the shard                            */
  float kernel_ms;         /* average time of one decode (all its kernels), events  */
  uint32_t launches;       /* decodes averaged in kernel_ms                         */
  uint32_t mode;           /* GH_MODE_SPLIT, GH_MODE_TILE or GH_MODE_MTILE          */
  uint32_t path;           /* GH_PATH_*: table / decode-loop variant                */
  uint64_t slow_lookbacks; /* tile mode: prefix reads that had to poll              */
} gh_report;

#define GH_MODE_SPLIT 1u    /* wave split: count, scan and write kernels (gh_wsplit.hip) */
#define GH_MODE_TILE 2u     /* persistent tile kernel, round-leader prefixes (gh_tile.hip) */
#define GH_MODE_FUSED 3u    /* reserved: the fused count + write tile kernel (removed)    */
#define GH_MODE_MTILE 4u    /* two-pass tile kernel: count and write over register-resident
                               words, one payload read (gh_mtile.hip) */
#define GH_PATH_GROUPED 2u  /* one codeword per lookup, grouped window shifts (tile kernel) */
#define GH_PATH_MULTI_WAVE 4u /* up to four codewords per lookup, canonical fallback for
                                 longer or incomplete codes (wave split) */
#define GH_PATH_MULTI_TILE 8u /* up to four codewords per lookup, start masks (two-pass tile) */
/* (values 0, 1, 3 were retired structures; they are no longer reported) */

#define GH_ST_BADCODE 1u    /* a bit pattern outside the code space was met       */
#define GH_ST_TIMEOUT 2u    /* look-back spin gave up (never expected)            */
#define GH_ST_LAYOUT 4u     /* kernel LDS layout assumption violated (never expected) */

/* Create a context on HIP device `device` (ordinal among visible devices). */
int gh_ctx_create(int device, gh_ctx** out);
int gh_ctx_destroy(gh_ctx* ctx);
/* Build the decode tables from s->syms and upload segments [seg_begin, seg_end)
 * of the stream to the device (H2D, synchronous).  Allocates an output buffer of
 * out_cap bytes (0 = min(N, upper bound of the shard) rounded up). */
int gh_ctx_load(gh_ctx* ctx, const gh_stream* s, uint64_t seg_begin, uint64_t seg_end,
                uint64_t out_cap);
/* Same as gh_ctx_load but from device-resident words: `d_payload` must hold
 * words [4*seg_begin, 4*seg_end+1) (missing tail words read as zero) and
 * `d_gap_words` the whole gap array; both stay owned by the caller. */
int gh_ctx_load_device(gh_ctx* ctx, const gh_stream* s_header_only, uint64_t seg_begin,
                       uint64_t seg_end, const uint32_t* d_payload, uint64_t d_payload_words,
                       const uint32_t* d_gap_words, uint64_t out_cap);
/* Enqueue one decode of the loaded shard on `hip_stream` (NULL = the context's own
 * stream).  Asynchronous.  When `timed` != 0 the launch is bracketed by HIP events
 * whose average is reported by gh_ctx_report. */
int gh_ctx_decode(gh_ctx* ctx, void* hip_stream, int timed);
/* Wait for the context's work and fill `rep` (reads the device total + status). */
int gh_ctx_report(gh_ctx* ctx, void* hip_stream, gh_report* rep);
/* Copy the first `nbytes` bytes of the shard output to host memory. */
int gh_ctx_download(gh_ctx* ctx, uint64_t byte_offset, uint8_t* dst, uint64_t nbytes);
/* Device pointer of the shard output (for RCCL gathers / torch interop). */
int gh_ctx_output(gh_ctx* ctx, void** d_out, uint64_t* cap);
/* Asynchronously copy nbytes of the shard output (from byte_offset) to `dst`
 * (device or host memory) on `hip_stream` (NULL = the context's stream). */
int gh_ctx_copy_output(gh_ctx* ctx, uint64_t byte_offset, void* dst, uint64_t nbytes,
                       void* hip_stream);
/* Reset the accumulated kernel timing. */
int gh_ctx_reset_timing(gh_ctx* ctx);

/* HIP device ordinal the context is bound to. */
int gh_ctx_device(gh_ctx* ctx, int* device);

/* ---- streaming file I/O ------------------------------ */
/* Replaces the reference CLI's whole-file fread + synchronous copies
 * (decoder/src/huff.cpp:90-140, decoder.cu:759-768): the file's gap words and the
 * shard's payload words stream through two pinned buffers, the read of one chunk
 * overlapping the H2D of the previous one. */
typedef struct gh_file_info {
  uint64_t n, w, g;        /* stream sizes from the header                          */
  uint32_t nsyms, version;
  uint64_t bytes_read;     /* header + gap words + the shard's payload words        */
  double setup_ms;         /* open, header parse, allocations (wall)                */
  double transfer_ms;      /* overlapped file reads + H2D (wall)                    */
  double total_ms;         /* whole call (wall), including table build              */
} gh_file_info;
/* gh_ctx_load for segments [seg_begin, seg_end) of the compressed.huff at `path`
 * (seg_end = UINT64_MAX: to the end).  info may be NULL. */
int gh_ctx_load_file(gh_ctx* ctx, const char* path, uint64_t seg_begin, uint64_t seg_end,
                     uint64_t out_cap, gh_file_info* info);
/* Wait for the context's decode, then write output bytes [byte_offset,
 * byte_offset+nbytes) to `path` at file_offset (pwrite; the file is created, and
 * truncated first when `truncate`), the D2H of one chunk overlapping the write of the
 * previous one.  ms (may be NULL): wall time. */
int gh_ctx_save_file(gh_ctx* ctx, const char* path, uint64_t file_offset, uint64_t byte_offset,
                     uint64_t nbytes, int truncate, double* ms);

/* ---- self-synchronising decode of gap-less streams ---- */
/* Replaces CUHD's decoder for raw Huffman streams without a gap array
 * (gpuhd/src/cuhd_gpu_decoder.cu:145-523, CUHDGPUDecoder::decode declared at
 * gpuhd/include/cuhd_gpu_decoder.h:24-32; stream = u32 units, codewords MSB-first,
 * llhuffman_encoder.cc:200-238).  The GPU finds every 128-bit segment's first
 * codeword start by decoding from arbitrary bits and verifying that neighbouring
 * walks agree (repairing where they do not), which yields the gap array; the stream
 * is then decoded by the gap-array kernels.  Codes: the canonical (symbol,length)
 * list in file order (lengths 1..16, non-decreasing), as in gh_stream. */
typedef struct gh_sync_report {
  uint64_t g;           /* 128-bit segments = ceil(w / 4)                          */
  uint64_t mismatches;  /* segment boundaries the first walk got wrong (repaired)  */
  uint32_t passes;      /* verify/repair passes (1 when the first walk was right)  */
  float kernel_ms;      /* walk kernel to the last verify pass (HIP events; includes
                           the host turnaround between passes)                     */
  float host_ms;        /* the halo estimate before the walk (stream sample copied
                           back + host walks; 0 when GH_SYNC_HALO is set), wall time,
                           not inside kernel_ms: the whole call is host_ms + kernel_ms */
  uint32_t halo;        /* warm-up segments per lane the walk used                 */
} gh_sync_report;
/* Gap words (ceil(ceil(w/4)/8) u32, the gap-array file's layout) of the raw stream
 * d_words[0..w) (device memory, 16-byte aligned) into d_gap_words on `hip_stream`
 * (NULL = default stream) of `device`.  Synchronous (the verify loop reads a
 * counter back).  rep may be NULL. */
int gh_sync_gaps(int device, const gh_sym* syms, uint32_t nsyms, const uint32_t* d_words,
                 uint64_t w, uint32_t* d_gap_words, void* hip_stream, gh_sync_report* rep);
/* Raw-stream file container (this repo's; gpuhd keeps its streams in memory,
 * demo.cc:100-160): u64 GH_RAW_MAGIC ("GHRAW1\0\0"), u64 nsyms, nsyms x {u8 symbol,
 * u8 length} in code order, u64 N, u64 W, W x u32 units (codewords MSB-first). */
#define GH_RAW_MAGIC 0x0000315741524847ull
typedef struct gh_raw_stream {
  const gh_sym* syms;
  uint32_t nsyms;
  uint64_t n, w;
  const uint32_t* units;   /* view into the file image                             */
} gh_raw_stream;
int gh_raw_parse(const void* file, size_t file_len, gh_raw_stream* out);
/* gh_ctx_load for a raw stream held in host memory: uploads words[0..w), builds its
 * gap array with gh_sync_gaps and loads the whole stream (n output bytes) into ctx;
 * gh_ctx_decode / gh_ctx_report / gh_ctx_download then work as for a gap-array file. */
int gh_ctx_load_raw(gh_ctx* ctx, const gh_sym* syms, uint32_t nsyms, uint64_t n,
                    const uint32_t* words, uint64_t w, uint64_t out_cap, gh_sync_report* rep);

/* One-shot decode of a whole stream into host memory `out` (out_len >= N):
 * mirrors decoder_l1_l2 (decoder.cu:732-815) without its 200-iteration loop.
 * ngpus <= 0 or 1: device `devices ? devices[0] : 0`; ngpus > 1 shards the
 * segments evenly over `devices` (or 0..ngpus-1; a device may repeat), decodes each
 * shard on its own device, and places shard outputs at the scanned offsets.  Each
 * shard is loaded, decoded and downloaded from its own host thread through pinned
 * double-buffered copies, so the shards' PCIe transfers overlap across devices (the
 * reference's launcher runs one device after another, decoder.cu:759-801).
 * rep->kernel_ms: per device the SUM of its shards' average decode times (decodes on
 * one device run in turn), the maximum over devices. */
typedef struct gh_opts {
  int ngpus;
  const int* devices;
  int reps;          /* decode repetitions (timing); <= 1 means one             */
} gh_opts;
int gh_decode(const gh_stream* s, uint8_t* out, uint64_t out_len, const gh_opts* opts,
              gh_report* rep);

/* Evenly split G segments into `nshards` contiguous ranges: bounds[0..nshards]. */
int gh_plan_shards(uint64_t g, uint32_t nshards, uint64_t* bounds);

/* Device memory for FFI callers without a HIP binding (buffers for gh_sync_gaps /
 * gh_ctx_load_device).  gh_dev_copy: any direction (unified addressing). */
int gh_dev_alloc(int device, uint64_t bytes, void** out);
int gh_dev_free(void* p);
int gh_dev_copy(void* dst, const void* src, uint64_t bytes);

/* Diagnostic yardstick: one streaming copy of `bytes` (multiple of
 * 16, 16-byte aligned device buffers) on `hip_stream` (NULL = default stream) of the
 * current device, repeated `reps` times after one warm-up pass; *ms_avg = HIP-event
 * time per pass.  The decode's roofline is quoted as a fraction of this rate.  No
 * reference counterpart (the reference measures nothing on the device). */
int gh_bw_copy(void* dst, const void* src, uint64_t bytes, void* hip_stream, int reps, float* ms_avg);

/* Number of visible HIP devices (0 when none / no driver). */
int gh_device_count(void);
/* Library version string. */
const char* gh_version(void);
/* Last error message of the calling thread (empty when none). */
const char* gh_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* GAPHUFF_H_ */
