"""Python host mirror of the gaphuff C ABI (include/gaphuff.h) for tests and bench.

This is plumbing over ``lib/libgaphuff.so`` (ctypes, no torch types).  The product
path is the HIP kernel behind the C ABI; there is no CPU decode fallback here: if
the shared library or a gfx950 device is missing, the decode entry points raise.

Reference interfaces mirrored (paths relative to the reference repo):

* :func:`decoder_l1_l2` — ``void decoder_l1_l2(unsigned *input, int inputfilesize,
  unsigned *output, int outputfilesize, int gap_element_num, void *dectable, int
  tablesize, unsigned prefix_bit, unsigned symbol_count, TableInfo)``
  (Huffman_coding_Gap_arrays/decoder/include/decoder.cuh:4-15, decoder.cu:732-815):
  same argument meaning (``input`` = gap words followed by payload words,
  huff.cpp:90-100); the decode table is built inside the library from the
  (symbol, length) list instead of being passed pre-built (get_table.cpp:48-139),
  and errors raise :class:`GapHuffError` instead of ``exit()`` (decoder.cu:14-20).
* :func:`encode` — the encoder CLI pipeline (encoder/src/huff.cpp:30-220).
* :func:`generate` — generate.cpp:32-47 with an explicit seed.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GAPHUFF_LIB", os.path.join(_HERE, "lib", "libgaphuff.so"))

GH_OK = 0
GH_ERRORS = {
    -1: "GH_E_ARG", -2: "GH_E_FORMAT", -3: "GH_E_TABLE", -4: "GH_E_HIP", -5: "GH_E_NODEV",
    -6: "GH_E_NOMEM", -7: "GH_E_CORRUPT", -8: "GH_E_STATE", -9: "GH_E_SMALL",
}
GH_V2_MAGIC = 0x0032465548504147
GH_ST_BADCODE = 1
GH_ST_TIMEOUT = 2

# Every symbol include/gaphuff.h declares (checked by tests/test_abi.py).
EXPORTED = (
    "gh_stream_parse", "gh_stream_validate", "gh_encode_plan_make", "gh_encode_write",
    "gh_package_merge", "gh_generate", "gh_ctx_create", "gh_ctx_destroy", "gh_ctx_load",
    "gh_ctx_load_device", "gh_ctx_decode", "gh_ctx_report", "gh_ctx_download",
    "gh_ctx_output", "gh_ctx_copy_output", "gh_ctx_reset_timing", "gh_decode", "gh_plan_shards",
    "gh_device_count", "gh_version", "gh_last_error",
    "gh_ectx_create", "gh_ectx_destroy", "gh_ectx_load", "gh_ectx_plan", "gh_ectx_encode",
    "gh_ectx_download", "gh_ctx_device", "gh_sync_gaps", "gh_ctx_load_raw",
    "gh_ctx_load_file", "gh_ctx_save_file", "gh_dev_alloc", "gh_dev_free", "gh_dev_copy",
    "gh_raw_parse", "gh_bw_copy",
)


class GapHuffError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{GH_ERRORS.get(code, code)}: {msg}")
        self.code = code


class gh_sym(ctypes.Structure):
    _fields_ = [("symbol", ctypes.c_uint8), ("length", ctypes.c_uint8)]


class gh_stream(ctypes.Structure):
    _fields_ = [
        ("syms", ctypes.POINTER(gh_sym)), ("nsyms", ctypes.c_uint32), ("version", ctypes.c_uint32),
        ("n", ctypes.c_uint64), ("w", ctypes.c_uint64), ("g", ctypes.c_uint64),
        ("gap_words", ctypes.c_void_p), ("payload", ctypes.c_void_p),
    ]


class gh_encode_plan(ctypes.Structure):
    _fields_ = [
        ("n", ctypes.c_uint64), ("bits", ctypes.c_uint64), ("w", ctypes.c_uint64),
        ("g", ctypes.c_uint64), ("file_bytes", ctypes.c_uint64), ("nsyms", ctypes.c_uint32),
        ("version", ctypes.c_uint32), ("syms", gh_sym * 256), ("code", ctypes.c_uint32 * 256),
        ("len", ctypes.c_uint8 * 256), ("count", ctypes.c_uint64 * 256),
    ]


class gh_report(ctypes.Structure):
    _fields_ = [
        ("symbols", ctypes.c_uint64), ("out_bytes", ctypes.c_uint64), ("status", ctypes.c_uint32),
        ("lut_bits", ctypes.c_uint32), ("grid", ctypes.c_uint32), ("tiles", ctypes.c_uint32),
        ("kernel_ms", ctypes.c_float), ("launches", ctypes.c_uint32),
        ("mode", ctypes.c_uint32), ("path", ctypes.c_uint32),
        ("slow_lookbacks", ctypes.c_uint64),
    ]


class gh_file_info(ctypes.Structure):
    _fields_ = [("n", ctypes.c_uint64), ("w", ctypes.c_uint64), ("g", ctypes.c_uint64),
                ("nsyms", ctypes.c_uint32), ("version", ctypes.c_uint32), ("bytes_read", ctypes.c_uint64),
                ("setup_ms", ctypes.c_double), ("transfer_ms", ctypes.c_double), ("total_ms", ctypes.c_double)]


class gh_raw_stream(ctypes.Structure):
    _fields_ = [("syms", ctypes.POINTER(gh_sym)), ("nsyms", ctypes.c_uint32), ("n", ctypes.c_uint64),
                ("w", ctypes.c_uint64), ("units", ctypes.c_void_p)]


class gh_sync_report(ctypes.Structure):
    _fields_ = [("g", ctypes.c_uint64), ("mismatches", ctypes.c_uint64), ("passes", ctypes.c_uint32),
                ("kernel_ms", ctypes.c_float), ("host_ms", ctypes.c_float), ("halo", ctypes.c_uint32)]


MODE_NAMES = {1: "split", 2: "tile", 3: "fused", 4: "mtile"}
PATH_NAMES = {2: "grouped", 4: "multi_wave", 8: "multi_tile"}


class gh_opts(ctypes.Structure):
    _fields_ = [("ngpus", ctypes.c_int), ("devices", ctypes.POINTER(ctypes.c_int)),
                ("reps", ctypes.c_int)]


_lib: Optional[ctypes.CDLL] = None


def lib() -> ctypes.CDLL:
    """Load libgaphuff.so (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise GapHuffError(-5, f"{LIB_PATH} missing: run `make -C {_HERE}` (or build())")
        L = ctypes.CDLL(LIB_PATH)
        P, U8, U32, U64, I = ctypes.c_void_p, ctypes.c_uint8, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int
        sig = {
            "gh_stream_parse": ([P, ctypes.c_size_t, ctypes.POINTER(gh_stream)], I),
            "gh_stream_validate": ([ctypes.POINTER(gh_stream)], I),
            "gh_encode_plan_make": ([P, U64, I, I, ctypes.POINTER(gh_encode_plan)], I),
            "gh_encode_write": ([P, ctypes.POINTER(gh_encode_plan), I, P, U64], I),
            "gh_package_merge": ([P, U32, P], I),
            "gh_generate": ([U64, ctypes.c_double, U64, U64, P, I], I),
            "gh_ctx_create": ([I, ctypes.POINTER(P)], I),
            "gh_ctx_destroy": ([P], I),
            "gh_ctx_load": ([P, ctypes.POINTER(gh_stream), U64, U64, U64], I),
            "gh_ctx_load_device": ([P, ctypes.POINTER(gh_stream), U64, U64, P, U64, P, U64], I),
            "gh_ctx_decode": ([P, P, I], I),
            "gh_ctx_report": ([P, P, ctypes.POINTER(gh_report)], I),
            "gh_ctx_download": ([P, U64, P, U64], I),
            "gh_ctx_output": ([P, ctypes.POINTER(P), ctypes.POINTER(U64)], I),
            "gh_ctx_copy_output": ([P, U64, P, U64, P], I),
            "gh_ctx_reset_timing": ([P], I),
            "gh_decode": ([ctypes.POINTER(gh_stream), P, U64, ctypes.POINTER(gh_opts),
                           ctypes.POINTER(gh_report)], I),
            "gh_plan_shards": ([U64, U32, P], I),
            "gh_device_count": ([], I),
            "gh_ectx_create": ([I, ctypes.POINTER(P)], I),
            "gh_ectx_destroy": ([P], I),
            "gh_ectx_load": ([P, P, U64], I),
            "gh_ectx_plan": ([P, I, ctypes.POINTER(gh_encode_plan)], I),
            "gh_ectx_encode": ([P, ctypes.POINTER(ctypes.c_float)], I),
            "gh_ectx_download": ([P, P, U64], I),
            "gh_ctx_device": ([P, ctypes.POINTER(I)], I),
            "gh_sync_gaps": ([I, P, U32, P, U64, P, P, ctypes.POINTER(gh_sync_report)], I),
            "gh_ctx_load_raw": ([P, P, U32, U64, P, U64, U64, ctypes.POINTER(gh_sync_report)], I),
            "gh_ctx_load_file": ([P, ctypes.c_char_p, U64, U64, U64, ctypes.POINTER(gh_file_info)], I),
            "gh_ctx_save_file": ([P, ctypes.c_char_p, U64, U64, U64, I, ctypes.POINTER(ctypes.c_double)], I),
            "gh_raw_parse": ([P, ctypes.c_size_t, ctypes.POINTER(gh_raw_stream)], I),
            "gh_dev_alloc": ([I, U64, ctypes.POINTER(P)], I),
            "gh_dev_free": ([P], I),
            "gh_dev_copy": ([P, P, U64], I),
            "gh_bw_copy": ([P, P, U64, P, I, ctypes.POINTER(ctypes.c_float)], I),
            "gh_version": ([], ctypes.c_char_p),
            "gh_last_error": ([], ctypes.c_char_p),
        }
        for name, (args, res) in sig.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = res
        del U8
        _lib = L
    return _lib


def _check(rc: int) -> None:
    if rc != GH_OK:
        raise GapHuffError(rc, lib().gh_last_error().decode(errors="replace"))


def _u8(a) -> np.ndarray:
    if isinstance(a, (bytes, bytearray, memoryview)):
        return np.frombuffer(a, dtype=np.uint8)
    return np.ascontiguousarray(a, dtype=np.uint8)


def _ptr(a: np.ndarray) -> ctypes.c_void_p:
    return ctypes.c_void_p(a.ctypes.data)


# --------------------------------------------------------------------------- format
@dataclass
class Stream:
    """A parsed compressed.huff (keeps the file bytes alive)."""

    raw: np.ndarray
    c: gh_stream

    @property
    def n(self) -> int:
        return int(self.c.n)

    @property
    def w(self) -> int:
        return int(self.c.w)

    @property
    def g(self) -> int:
        return int(self.c.g)

    @property
    def version(self) -> int:
        return int(self.c.version)

    @property
    def symbols(self) -> list:
        return [(self.c.syms[i].symbol, self.c.syms[i].length) for i in range(self.c.nsyms)]


def parse(file_bytes) -> Stream:
    raw = _u8(file_bytes)
    s = gh_stream()
    _check(lib().gh_stream_parse(_ptr(raw), raw.size, ctypes.byref(s)))
    return Stream(raw, s)


# --------------------------------------------------------------------------- encoder
def encode_plan(data, threads: int = 0, force_version: int = 0) -> gh_encode_plan:
    d = _u8(data)
    plan = gh_encode_plan()
    _check(lib().gh_encode_plan_make(_ptr(d), d.size, threads, force_version, ctypes.byref(plan)))
    return plan


def encode(data, threads: int = 0, force_version: int = 0) -> np.ndarray:
    """Compress bytes into a compressed.huff image (np.uint8)."""
    d = _u8(data)
    plan = encode_plan(d, threads, force_version)
    out = np.empty(plan.file_bytes, dtype=np.uint8)
    _check(lib().gh_encode_write(_ptr(d), ctypes.byref(plan), threads, _ptr(out), out.size))
    return out


class Encoder:
    """One gh_ectx: the GPU encoder on one gfx950 device.

    Mirrors the reference encoder CLI's steps (encoder/src/huff.cpp:30-220): load the
    input, plan (histogram on the GPU, package-merge on the host), encode, download
    the compressed.huff image -- byte-identical to ``encode()``."""

    def __init__(self, device: int = 0):
        self._h = ctypes.c_void_p()
        _check(lib().gh_ectx_create(device, ctypes.byref(self._h)))
        self.plan: Optional[gh_encode_plan] = None

    def close(self) -> None:
        if self._h:
            lib().gh_ectx_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def load(self, data) -> None:
        d = _u8(data)
        _check(lib().gh_ectx_load(self._h, _ptr(d), d.size))

    def make_plan(self, force_version: int = 0) -> gh_encode_plan:
        p = gh_encode_plan()
        _check(lib().gh_ectx_plan(self._h, force_version, ctypes.byref(p)))
        self.plan = p
        return p

    def encode(self) -> float:
        """Encode on the device; returns the kernels' event time in ms."""
        ms = ctypes.c_float()
        _check(lib().gh_ectx_encode(self._h, ctypes.byref(ms)))
        return float(ms.value)

    def download(self) -> np.ndarray:
        if self.plan is None:
            raise GapHuffError(-8, "download before make_plan/encode")
        out = np.empty(self.plan.file_bytes, dtype=np.uint8)
        _check(lib().gh_ectx_download(self._h, _ptr(out), out.size))
        return out


def encode_gpu(data, device: int = 0, force_version: int = 0) -> np.ndarray:
    """Compress bytes on the GPU into a compressed.huff image (== ``encode(data)``)."""
    with Encoder(device) as e:
        e.load(data)
        e.make_plan(force_version)
        e.encode()
        return e.download()


def package_merge(sorted_counts: Sequence[int]) -> list:
    c = np.ascontiguousarray(sorted_counts, dtype=np.uint64)
    out = np.zeros(max(1, c.size), dtype=np.uint8)
    _check(lib().gh_package_merge(_ptr(c), c.size, _ptr(out)))
    return out[: c.size].tolist()


def generate(seed: int, redundancy: float, n: int, offset: int = 0, threads: int = 0) -> np.ndarray:
    out = np.empty(n, dtype=np.uint8)
    _check(lib().gh_generate(seed, float(redundancy), offset, n, _ptr(out), threads))
    return out


def plan_shards(g: int, nshards: int) -> list:
    b = np.zeros(nshards + 1, dtype=np.uint64)
    _check(lib().gh_plan_shards(g, nshards, _ptr(b)))
    return [int(x) for x in b]


def device_count() -> int:
    return int(lib().gh_device_count())


# --------------------------------------------------------------------------- decoder
class Decoder:
    """One gh_ctx: a shard of a stream resident on one GPU."""

    def __init__(self, device: int = 0):
        self._h = ctypes.c_void_p()
        _check(lib().gh_ctx_create(device, ctypes.byref(self._h)))
        self.device = device
        self._stream: Optional[Stream] = None

    def close(self) -> None:
        if self._h:
            lib().gh_ctx_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def load(self, stream: Stream, seg_begin: int = 0, seg_end: Optional[int] = None,
             out_cap: int = 0) -> None:
        seg_end = stream.g if seg_end is None else seg_end
        self._stream = stream
        _check(lib().gh_ctx_load(self._h, ctypes.byref(stream.c), seg_begin, seg_end, out_cap))

    def load_file(self, path: str, seg_begin: int = 0, seg_end: Optional[int] = None,
                  out_cap: int = 0) -> gh_file_info:
        """Stream segments [seg_begin, seg_end) of a compressed.huff file to the device
        (pinned double-buffered read -> H2D); returns the header sizes and timings."""
        info = gh_file_info()
        _check(lib().gh_ctx_load_file(self._h, os.fsencode(path), seg_begin,
                                      (1 << 64) - 1 if seg_end is None else seg_end, out_cap,
                                      ctypes.byref(info)))
        self._stream = None
        return info

    def save_file(self, path: str, nbytes: int, file_offset: int = 0, offset: int = 0,
                  truncate: bool = True) -> float:
        """Write decoded bytes [offset, offset+nbytes) to `path` at file_offset; wall ms."""
        ms = ctypes.c_double()
        _check(lib().gh_ctx_save_file(self._h, os.fsencode(path), file_offset, offset, nbytes,
                                      int(truncate), ctypes.byref(ms)))
        return ms.value

    def load_raw(self, symbols: Sequence[tuple], n: int, units, out_cap: int = 0) -> gh_sync_report:
        """Load a raw (gap-less) stream: u32 ``units``, canonical ``symbols`` list
        [(symbol, length)] in code order, ``n`` output bytes.  The gap array is
        built on the GPU (gh_sync_gaps); returns its report."""
        u = np.ascontiguousarray(units, dtype=np.uint32)
        sy = _syms(symbols)
        r = gh_sync_report()
        _check(lib().gh_ctx_load_raw(self._h, ctypes.byref(sy), len(symbols), n, _ptr(u), u.size, out_cap,
                                     ctypes.byref(r)))
        self._stream = None
        return r

    def decode(self, hip_stream: int = 0, timed: bool = True) -> None:
        _check(lib().gh_ctx_decode(self._h, ctypes.c_void_p(hip_stream or None), int(timed)))

    def report(self, hip_stream: int = 0) -> gh_report:
        r = gh_report()
        _check(lib().gh_ctx_report(self._h, ctypes.c_void_p(hip_stream or None), ctypes.byref(r)))
        return r

    def reset_timing(self) -> None:
        _check(lib().gh_ctx_reset_timing(self._h))

    def download(self, nbytes: int, offset: int = 0) -> np.ndarray:
        out = np.empty(nbytes, dtype=np.uint8)
        _check(lib().gh_ctx_download(self._h, offset, _ptr(out), nbytes))
        return out

    def copy_output(self, dst_ptr: int, nbytes: int, offset: int = 0, hip_stream: int = 0) -> None:
        """Async copy of shard output bytes to a device/host address (e.g. a torch tensor)."""
        _check(lib().gh_ctx_copy_output(self._h, offset, ctypes.c_void_p(dst_ptr), nbytes,
                                        ctypes.c_void_p(hip_stream or None)))

    def output(self):
        p = ctypes.c_void_p()
        cap = ctypes.c_uint64()
        _check(lib().gh_ctx_output(self._h, ctypes.byref(p), ctypes.byref(cap)))
        return int(p.value or 0), int(cap.value)


def decode(file_bytes, ngpus: int = 1, devices: Optional[Sequence[int]] = None,
           reps: int = 1) -> np.ndarray:
    """Decode a whole compressed.huff image on the GPU(s); returns the N bytes."""
    s = parse(file_bytes)
    out = np.empty(max(1, s.n), dtype=np.uint8)
    o = gh_opts()
    o.ngpus = ngpus
    o.reps = reps
    if devices is not None:
        arr = (ctypes.c_int * len(devices))(*devices)
        o.devices = ctypes.cast(arr, ctypes.POINTER(ctypes.c_int))
    r = gh_report()
    _check(lib().gh_decode(ctypes.byref(s.c), _ptr(out), out.size, ctypes.byref(o), ctypes.byref(r)))
    return out[: s.n]


def _syms(symbols: Sequence[tuple]):
    arr = (gh_sym * max(1, len(symbols)))()
    for i, (sy, ln) in enumerate(symbols):
        arr[i].symbol, arr[i].length = sy, ln
    return arr


class DeviceBuffer:
    """Device memory through the library's own HIP runtime (gh_dev_*)."""

    def __init__(self, nbytes: int, device: int = 0):
        self.ptr = ctypes.c_void_p()
        self.nbytes = nbytes
        _check(lib().gh_dev_alloc(device, nbytes, ctypes.byref(self.ptr)))

    @property
    def addr(self) -> int:
        return int(self.ptr.value or 0)

    def upload(self, a: np.ndarray) -> "DeviceBuffer":
        a = np.ascontiguousarray(a)
        assert a.nbytes <= self.nbytes
        _check(lib().gh_dev_copy(self.ptr, _ptr(a), a.nbytes))
        return self

    def download(self, a: np.ndarray) -> np.ndarray:
        assert a.flags.c_contiguous and a.nbytes <= self.nbytes
        _check(lib().gh_dev_copy(_ptr(a), self.ptr, a.nbytes))
        return a

    def close(self) -> None:
        if self.ptr:
            lib().gh_dev_free(self.ptr)
            self.ptr = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def sync_gaps(symbols: Sequence[tuple], d_words: int, w: int, d_gap_words: int, device: int = 0,
              hip_stream: int = 0) -> gh_sync_report:
    """Gap words of a device-resident raw stream (device addresses as ints, e.g. a
    torch tensor's data_ptr()); see gh_sync_gaps in include/gaphuff.h."""
    sy = _syms(symbols)
    r = gh_sync_report()
    _check(lib().gh_sync_gaps(device, ctypes.byref(sy), len(symbols), ctypes.c_void_p(d_words), w,
                              ctypes.c_void_p(d_gap_words), ctypes.c_void_p(hip_stream or None),
                              ctypes.byref(r)))
    return r


def bw_copy(dst_ptr: int, src_ptr: int, nbytes: int, hip_stream: int = 0, reps: int = 10) -> float:
    """Streaming-copy yardstick: ms per pass of a 16-B-lane copy of `nbytes` device
    bytes (gh_bw_copy, include/gaphuff.h)."""
    ms = ctypes.c_float()
    _check(lib().gh_bw_copy(ctypes.c_void_p(dst_ptr), ctypes.c_void_p(src_ptr), nbytes,
                            ctypes.c_void_p(hip_stream or None), reps, ctypes.byref(ms)))
    return float(ms.value)


def parse_raw(file_bytes):
    """Parse a raw-stream container (bin/encoder --raw): (symbols, n, units)."""
    raw = _u8(file_bytes)
    r = gh_raw_stream()
    _check(lib().gh_raw_parse(_ptr(raw), raw.size, ctypes.byref(r)))
    syms = [(r.syms[i].symbol, r.syms[i].length) for i in range(r.nsyms)]
    off = 16 + 2 * r.nsyms + 16
    units = raw[off: off + 4 * r.w].view(np.uint32).copy()
    return syms, int(r.n), units


def decode_raw(units, symbols: Sequence[tuple], n: int, device: int = 0) -> np.ndarray:
    """Self-synchronising decode of a raw stream: the role of CUHD's
    CUHDGPUDecoder::decode (gpuhd/include/cuhd_gpu_decoder.h:24-32) for u32 units
    packed MSB-first (llhuffman_encoder.cc:200-238).  Returns the n decoded bytes."""
    with Decoder(device) as d:
        d.load_raw(symbols, n, units)
        d.decode(timed=False)
        rep = d.report()
        if rep.status:
            raise GapHuffError(-7, f"device status {rep.status}")
        if rep.symbols < n:  # never hand back undecoded (uninitialised) output bytes
            raise GapHuffError(-7, f"raw stream decoded to {rep.symbols} of {n} symbols")
        return d.download(n) if n else np.zeros(0, dtype=np.uint8)


def decoder_l1_l2(input_words, inputfilesize: int, outputfilesize: int, gap_element_num: int,
                  symbols: Sequence[tuple], gpus: int = 1) -> np.ndarray:
    """Mirror of the reference launcher (decoder.cu:732-815).

    ``input_words``: u32 array holding ceil(G/8) gap words followed by W payload words
    (the reference's pinned ``input``, huff.cpp:90-100); ``inputfilesize`` = W,
    ``outputfilesize`` = N, ``gap_element_num`` = G, ``symbols`` = [(symbol, length)]
    in file order.  Returns the N decoded bytes.
    """
    words = np.ascontiguousarray(input_words, dtype=np.uint32)
    gw = (gap_element_num + 7) // 8
    if words.size < gw + inputfilesize:
        raise GapHuffError(-1, "input shorter than gap words + payload")
    hdr = np.zeros(8 + 2 * len(symbols) + 12, dtype=np.uint8)
    hdr[:8] = np.frombuffer(np.uint64(len(symbols)).tobytes(), dtype=np.uint8)
    for i, (sy, ln) in enumerate(symbols):
        hdr[8 + 2 * i] = sy
        hdr[9 + 2 * i] = ln
    o = 8 + 2 * len(symbols)
    hdr[o:o + 12] = np.frombuffer(np.array([outputfilesize, inputfilesize, gap_element_num],
                                           dtype=np.uint32).tobytes(), dtype=np.uint8)
    image = np.concatenate([hdr, words[: gw + inputfilesize].view(np.uint8)])
    return decode(image, ngpus=gpus)
