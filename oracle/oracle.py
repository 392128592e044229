"""CPU ORACLE (test infrastructure only).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module, and only as the checker.  It wraps:

* ``_build/liboracle.so`` — gh_oracle.c, a bit-serial C restatement of the
  reference encoder/decoder semantics (file:line citations in gh_oracle.c);
* ``_ref/*`` — the reference's own CPU programs/functions compiled from its
  sources by oracle/Makefile (sequential.cpp, parallel_cpu_decomp.cpp,
  parallel_cpu_prescan.cpp, boundary_PM via ref_drivers/pm_driver.cpp,
  get_twolevel_table via ref_drivers/table_probe.cpp).
"""
from __future__ import annotations

import ctypes
import os
import re
import shutil
import subprocess
import tempfile
import time
from typing import Optional

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "liboracle.so")
REF = os.path.join(HERE, "_ref")

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            raise RuntimeError(f"{LIB} missing: run `make -C {HERE} oracle`")
        L = ctypes.CDLL(LIB)
        P, U64, I = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int
        L.orc_package_merge.argtypes = [P, I, P]
        L.orc_package_merge.restype = I
        L.orc_plan_make.argtypes = [P, U64, I, P]
        L.orc_plan_make.restype = I
        L.orc_encode.argtypes = [P, P, P]
        L.orc_encode.restype = I
        L.orc_decode.argtypes = [P, U64, P, U64, ctypes.POINTER(U64)]
        L.orc_decode.restype = ctypes.c_int64
        L.orc_segment_count.argtypes = [P, U64, U64]
        L.orc_segment_count.restype = ctypes.c_int64
        L.orc_generate.argtypes = [U64, ctypes.c_double, U64, U64, P]
        L.orc_generate.restype = None
        _lib = L
    return _lib


class _Plan(ctypes.Structure):
    _fields_ = [
        ("n", ctypes.c_uint64), ("bits", ctypes.c_uint64), ("w", ctypes.c_uint64),
        ("g", ctypes.c_uint64), ("file_bytes", ctypes.c_uint64), ("nsyms", ctypes.c_int),
        ("version", ctypes.c_int), ("syms", ctypes.c_uint8 * 256), ("lens", ctypes.c_uint8 * 256),
        ("count", ctypes.c_uint64 * 256),
    ]


def _u8(a) -> np.ndarray:
    if isinstance(a, (bytes, bytearray, memoryview)):
        return np.frombuffer(a, dtype=np.uint8)
    return np.ascontiguousarray(a, dtype=np.uint8)


def _p(a: np.ndarray):
    return ctypes.c_void_p(a.ctypes.data)


def package_merge(sorted_counts) -> list:
    c = np.ascontiguousarray(sorted_counts, dtype=np.uint64)
    out = np.zeros(max(1, c.size), dtype=np.uint8)
    if lib().orc_package_merge(_p(c), c.size, _p(out)) != 0:
        raise RuntimeError("oracle package-merge failed")
    return out[: c.size].tolist()


def encode(data, force_v2: bool = False) -> np.ndarray:
    d = _u8(data)
    plan = _Plan()
    if lib().orc_plan_make(_p(d), d.size, int(force_v2), ctypes.byref(plan)) != 0:
        raise RuntimeError("oracle plan failed")
    out = np.zeros(plan.file_bytes, dtype=np.uint8)
    if lib().orc_encode(_p(d), ctypes.byref(plan), _p(out)) != 0:
        raise RuntimeError("oracle encode failed")
    return out


def symbols_of(data) -> list:
    """File-order (symbol, length) list the reference encoder would write."""
    d = _u8(data)
    plan = _Plan()
    if lib().orc_plan_make(_p(d), d.size, 0, ctypes.byref(plan)) != 0:
        raise RuntimeError("oracle plan failed")
    return [(plan.syms[i], plan.lens[i]) for i in range(plan.nsyms)]


def decode(file_bytes, out_cap: Optional[int] = None):
    """Returns (decoded bytes clamped at N, total symbols counted over all segments)."""
    f = _u8(file_bytes)
    cap = out_cap if out_cap is not None else max(1, f.size * 8)
    out = np.zeros(max(1, cap), dtype=np.uint8)
    total = ctypes.c_uint64()
    n = lib().orc_decode(_p(f), f.size, _p(out), out.size, ctypes.byref(total))
    if n < 0:
        raise RuntimeError("oracle decode failed (bad stream)")
    return out[:n].copy(), int(total.value)


def segment_count(file_bytes, i: int) -> int:
    f = _u8(file_bytes)
    r = lib().orc_segment_count(_p(f), f.size, i)
    if r < 0:
        raise RuntimeError("oracle segment_count failed")
    return int(r)


def generate(seed: int, redundancy: float, n: int, offset: int = 0) -> np.ndarray:
    out = np.empty(n, dtype=np.uint8)
    lib().orc_generate(seed, float(redundancy), offset, n, _p(out))
    return out


# ------------------------------------------------------------------ reference binaries
def ref_available(name: str) -> bool:
    return os.access(os.path.join(REF, name), os.X_OK)


def ref_package_merge(counts256) -> list:
    """Reference boundary_PM via _ref/pm_driver: file-order [(symbol, length)]."""
    c = np.ascontiguousarray(counts256, dtype="<u4")
    assert c.size == 256
    with tempfile.TemporaryDirectory() as td:
        fn = os.path.join(td, "c.bin")
        c.tofile(fn)
        out = subprocess.run([os.path.join(REF, "pm_driver"), fn], capture_output=True, text=True,
                             check=True).stdout
    return [tuple(int(x) for x in line.split()) for line in out.strip().splitlines()]


def ref_table_probe(symbols):
    """Reference get_twolevel_table via _ref/table_probe (maxlen > 10 only).

    Returns (l1_size, l2_size, ptr_size, table bytes) or None when unsupported."""
    with tempfile.TemporaryDirectory() as td:
        fn = os.path.join(td, "s.txt")
        with open(fn, "w") as f:
            for s, l in symbols:
                f.write(f"{s} {l}\n")
        r = subprocess.run([os.path.join(REF, "table_probe"), fn], capture_output=True)
    if r.returncode != 0:
        return None
    hdr = np.frombuffer(r.stdout[:16], dtype="<u4")
    return int(hdr[0]), int(hdr[1]), int(hdr[2]), np.frombuffer(r.stdout[16:16 + int(hdr[3])], dtype=np.uint8)


def ref_table_lookup(table_info, window: int, prefix_bit: int = 10):
    """Replay of the reference kernel lookup (decoder.cu:531-546) on a 32-bit window.

    Returns (symbol, length)."""
    l1, l2, ptr, tb = table_info
    ptr_table = tb[: 4 * ptr].view("<u4") if ptr else np.zeros(0, dtype="<u4")
    length_table = tb[4 * ptr: 4 * ptr + 256]
    l1_table = tb[4 * ptr + 256: 4 * ptr + 256 + l1]
    l2_table = tb[4 * ptr + 256 + l1: 4 * ptr + 256 + l1 + l2]
    prefix_mask = (~((0xFFFFFFFF) >> prefix_bit)) & 0xFFFFFFFF
    deccode = (window & prefix_mask) >> (32 - prefix_bit)
    if deccode < l1:
        sym = int(l1_table[deccode])
    else:
        t = int(ptr_table[deccode - l1])
        width = (t >> 16) & 0xFFFF
        idx = t & 0xFFFF
        l2_mask = ((~(0xFFFFFFFF >> width)) & 0xFFFFFFFF) >> prefix_bit
        l2_shift = 32 - prefix_bit - width
        sym = int(l2_table[idx + ((window & l2_mask) >> l2_shift)])
    return sym, int(length_table[sym])


_SEQ_RE = re.compile(r"Decompression time:\s+(\d+) mcs")
_PAR_RE = re.compile(r"Decompression time \(Parallel Decode\):\s+(\d+) us")
_VER_RE = re.compile(r"Verification:\s+(PASS|FAIL)")


def run_reference_cpu(name: str, data: np.ndarray, timeout: float = 600.0,
                      threads: Optional[int] = None) -> dict:
    """Run a reference CPU program (compiled from its own source) on `data`.

    sequential / parallel_cpu_prescan read data100_100.bin, parallel_decomp_cpu
    reads data.bin (sequential.cpp:240, parallel_cpu_prescan.cpp:596,
    parallel_cpu_decomp.cpp:655); each times decode() only and verifies.
    `threads` (prescan / decomp only) runs the reference's main() through our
    driver (_ref/prescan_driver, _ref/decomp_driver) with its hard-coded
    ``thread_count`` (parallel_cpu_prescan.cpp:25, parallel_cpu_decomp.cpp:24)
    set to that value; None runs the program as shipped.
    Returns {decode_us, verified, threads, wall_s}."""
    shipped = {"sequential": 1, "parallel_decomp_cpu": 1, "parallel_cpu_prescan": 16}
    drivers = {"parallel_decomp_cpu": "decomp_driver", "parallel_cpu_prescan": "prescan_driver"}
    exe_name, argv = name, []
    if threads is not None and name in drivers:
        exe_name, argv = drivers[name], [str(int(threads))]
    exe = os.path.join(REF, exe_name)
    if not os.access(exe, os.X_OK):
        raise FileNotFoundError(exe)
    infile = "data.bin" if name == "parallel_decomp_cpu" else "data100_100.bin"
    td = tempfile.mkdtemp(prefix="gh_ref_")
    try:
        _u8(data).tofile(os.path.join(td, infile))
        t0 = time.time()
        r = subprocess.run([exe, *argv], cwd=td, capture_output=True, text=True, timeout=timeout)
        wall = time.time() - t0
        m = (_SEQ_RE if name == "sequential" else _PAR_RE).search(r.stdout)
        v = _VER_RE.search(r.stdout)
        if not m:
            raise RuntimeError(f"{name} produced no timing: {r.stdout[-400:]} {r.stderr[-400:]}")
        return {"decode_us": int(m.group(1)), "verified": bool(v and v.group(1) == "PASS"),
                "threads": int(threads) if argv else shipped[name], "wall_s": wall}
    finally:
        shutil.rmtree(td, ignore_errors=True)


# ------------------------------------------------------- raw (gap-less) streams
# Restatement of the self-synchronising decoder's stream (gpuhd, SURVEY.md §8(f)
# rank 3): llhuffman_encoder.cc:173-198 (canonical codes in list order),
# :200-238 (codewords packed MSB-first into u32 units).  Test infrastructure only.
def canonical_codes(syms) -> list:
    """Codes of a (symbol, length) list in list order: llhuffman_encoder.cc:181-193,
    identical to package_merge.cpp:168-181 (code = (code+1) << (len' - len))."""
    codes, code = [], 0
    for i, (_, ln) in enumerate(syms):
        if i:
            code = (code + 1) << (ln - syms[i - 1][1])
        codes.append(code)
    return codes


def _code_arrays(data, syms):
    d = _u8(data)
    code = np.zeros(256, dtype=np.uint64)
    ln = np.zeros(256, dtype=np.uint64)
    for (s, l), c in zip(syms, canonical_codes(syms)):
        code[s], ln[s] = c, l
    if d.size and np.any(ln[d] == 0):
        raise ValueError("data holds a symbol outside the table")
    return d, code[d], ln[d]


def raw_encode(data, syms) -> np.ndarray:
    """u32 units of the raw stream (bit 0 = bit 31 of unit 0; the last unit
    zero-padded, where encode_memory's final unit is undefined, :228-232)."""
    d, c, l = _code_arrays(data, syms)
    bits = int(l.sum())
    w = (bits + 31) // 32
    out = np.zeros(w * 32 + 64, dtype=np.uint8)
    if d.size:
        ends = np.cumsum(l)
        starts = ends - l
        for k in range(16):  # bit k (from the MSB) of every codeword
            m = l > k
            pos = (starts[m] + k).astype(np.int64)
            out[pos] = ((c[m] >> (l[m] - 1 - k)) & 1).astype(np.uint8)
    return np.packbits(out[: w * 32]).view(">u4").astype(np.uint32)


def raw_gaps(data, syms) -> np.ndarray:
    """Gap words of the raw stream: entry of segment j+1 (first codeword start at
    or after 128(j+1), or the end of the last codeword when it crosses 128(j+1))
    minus 128(j+1) in nibble j, 8 per u32 LSB-first; the last nibble is 0
    (encoder.cu:307-312,358-379)."""
    d, _, l = _code_arrays(data, syms)
    bits = int(l.sum())
    g = ((bits + 31) // 32 + 3) // 4
    nib = np.zeros(8 * ((g + 7) // 8), dtype=np.uint32)
    if g > 1:
        # codeword starts plus the stream's end: a boundary crossed by the LAST codeword
        # gets that codeword's end, as encoder.cu:307-312 records every crossing codeword
        starts = np.append(np.cumsum(l) - l, bits)
        bnd = 128 * np.arange(1, g, dtype=np.uint64)
        idx = np.searchsorted(starts, bnd)
        entry = np.where(idx < starts.size, starts[np.minimum(idx, starts.size - 1)], bnd)
        nib[: g - 1] = (entry - bnd).astype(np.uint32)
    nib = nib.reshape(-1, 8) << (4 * np.arange(8, dtype=np.uint32))
    return np.bitwise_or.reduce(nib, axis=1).astype(np.uint32) if nib.size else np.zeros(0, np.uint32)


def raw_decode(units, syms, n: int) -> np.ndarray:
    """Bit-serial decode of n symbols (small cases only): the per-codeword table
    walk of cuhd_gpu_decoder.cu:86-118 run from bit 0."""
    by_code = {(l, c): s for (s, l), c in zip(syms, canonical_codes(syms))}
    bits = np.unpackbits(np.asarray(units, dtype=np.uint32).astype(">u4").view(np.uint8))
    out = np.zeros(n, dtype=np.uint8)
    pos = 0
    for i in range(n):
        c = 0
        for l in range(1, 17):
            c = (c << 1) | int(bits[pos + l - 1]) if pos + l - 1 < bits.size else c << 1
            if (l, c) in by_code:
                out[i] = by_code[(l, c)]
                pos += l
                break
        else:
            raise RuntimeError(f"invalid code at bit {pos}")
    return out


def ref_llhuff(data):
    """Reference raw-stream encoder (gpuhd/encoder, compiled into _ref/llhuff_driver):
    returns (syms in code order, units)."""
    exe = os.path.join(REF, "llhuff_driver")
    with tempfile.TemporaryDirectory() as td:
        fi, fo = os.path.join(td, "in.bin"), os.path.join(td, "out.llh")
        _u8(data).tofile(fi)
        subprocess.run([exe, fi, fo], check=True, capture_output=True)
        return read_llh(open(fo, "rb").read())


def read_llh(b: bytes):
    """Parse the llhuff_driver output: u32 nsyms, {u8 sym, u8 len}*, u64 units, units."""
    ns = int(np.frombuffer(b[:4], "<u4")[0])
    e = np.frombuffer(b[4 : 4 + 2 * ns], np.uint8).reshape(-1, 2)
    syms = [(int(s), int(l)) for s, l in e]
    o = 4 + 2 * ns
    nu = int(np.frombuffer(b[o : o + 8], "<u8")[0])
    units = np.frombuffer(b[o + 8 : o + 8 + 4 * nu], "<u4").astype(np.uint32)
    return syms, units
