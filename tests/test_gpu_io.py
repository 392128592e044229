"""Streaming file I/O: gh_ctx_load_file / gh_ctx_save_file and
the decoder CLI built on them.  Decoded files must equal the input bytes (the oracle
and the reference sequential.cpp pin the stream format, tests/test_oracle.py)."""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "bin")


def _write(tmp_path, gh, seed, r, n, name="c.huff"):
    d = gh.generate(seed, r, n)
    p = tmp_path / name
    gh.encode(d, threads=8).tofile(p)
    return d, str(p)


@pytest.mark.gpu
@pytest.mark.parametrize("r,n", [(0.5, 1), (0.5, 3_000_017), (0.1, 80_000_000)])
def test_gpu_load_save_file_roundtrip(gpu, tmp_path, r, n):
    """80 MB at r=0.1 streams in three 32 MiB chunks each way."""
    d, path = _write(tmp_path, gpu, 3, r, n)
    out = str(tmp_path / "out.bin")
    with gpu.Decoder(0) as dec:
        info = dec.load_file(path)
        assert info.n == n and info.bytes_read == os.path.getsize(path)
        dec.decode()
        assert dec.report().status == 0
        dec.save_file(out, n)
    assert np.array_equal(np.fromfile(out, dtype=np.uint8), d)


@pytest.mark.gpu
def test_gpu_load_file_shards(gpu, tmp_path):
    """Three shards, each loading only its payload range and writing at its offset."""
    d, path = _write(tmp_path, gpu, 4, 0.9, 5_000_000)
    out = str(tmp_path / "out.bin")
    g = gpu.parse(np.fromfile(path, dtype=np.uint8)).g
    b = gpu.plan_shards(g, 3)
    off = 0
    for k in range(3):
        with gpu.Decoder(0) as dec:
            info = dec.load_file(path, b[k], b[k + 1])
            dec.decode()
            sym = dec.report().symbols
            want = min(sym, d.size - off)
            dec.save_file(out, want, file_offset=off, truncate=(k == 0))
            off += sym
            assert info.bytes_read < os.path.getsize(path) or k == 2
    assert np.array_equal(np.fromfile(out, dtype=np.uint8), d)


@pytest.mark.gpu
def test_gpu_load_file_empty_and_truncated(gpu, tmp_path):
    d, path = _write(tmp_path, gpu, 5, 0.5, 0)
    with gpu.Decoder(0) as dec:
        info = dec.load_file(path)
        assert info.n == 0
        dec.decode()
        dec.save_file(str(tmp_path / "e.bin"), 0)
    assert os.path.getsize(tmp_path / "e.bin") == 0
    _, path = _write(tmp_path, gpu, 5, 0.5, 100_000, "t.huff")
    raw = open(path, "rb").read()
    open(path, "wb").write(raw[: len(raw) // 2])
    with gpu.Decoder(0) as dec:
        with pytest.raises(gpu.GapHuffError):
            dec.load_file(path)


@pytest.mark.gpu
@pytest.mark.parametrize("gpus,shards", [(1, 0), (2, 0), (1, 3), (1, 8)])
def test_gpu_cli_streaming_verify(gpu, tmp_path, gpus, shards):
    """bin/decoder on one or more devices (clamped to the visible ones) and with S
    shards on them (--shards: shard k on device k mod N), each shard streaming its
    payload range and writing at its offset of the output file."""
    if not os.access(os.path.join(BIN, "decoder"), os.X_OK):
        pytest.fail("bin/decoder not built")
    d, path = _write(tmp_path, gpu, 6, 0.1, 40_000_003)
    (tmp_path / "orig.bin").write_bytes(d.tobytes())
    out = str(tmp_path / "dec.bin")
    extra = ["--shards", str(shards)] if shards else []
    r = subprocess.run([os.path.join(BIN, "decoder"), path, out, "--gpus", str(gpus), *extra, "--verify",
                        str(tmp_path / "orig.bin")], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "Verification: PASS" in r.stdout
    assert np.array_equal(np.fromfile(out, dtype=np.uint8), d)


_CALLER_STREAM_SCRIPT = r"""
import sys, numpy as np, torch
torch.cuda.init()  # torch's HIP runtime first (as bench.py does), then the library's
sys.path.insert(0, sys.argv[1])
import gaphuff as gh
path, out, n = sys.argv[2], sys.argv[3], int(sys.argv[4])
d = np.fromfile(sys.argv[5], dtype=np.uint8)
s = torch.cuda.Stream()
with gh.Decoder(0) as dec:
    dec.load_file(path)
    for _ in range(3):
        dec.decode(s.cuda_stream, timed=True)
    dec.save_file(out, n)  # no caller sync before this
    assert np.array_equal(np.fromfile(out, dtype=np.uint8), d)
    dec.decode(s.cuda_stream, timed=True)
    assert np.array_equal(dec.download(n), d)
    dec.decode(s.cuda_stream, timed=True)
    t = torch.empty(n, dtype=torch.uint8, device="cuda")
    dec.copy_output(t.data_ptr(), n)  # context stream, ordered after the decode
    rep = dec.report()
    assert rep.status == 0 and rep.launches == 5, (rep.status, rep.launches)
    assert np.array_equal(t.cpu().numpy(), d)
print("caller-stream ok")
"""


@pytest.mark.gpu
def test_decode_on_caller_stream_then_save_and_download(gpu, tmp_path):
    """A decode launched on a caller's stream (as bench.py does with torch's stream) is
    waited for by save_file / download / copy_output on the context's own stream
    (gh_ctx completion event), with no synchronisation by the caller.  Runs in a child
    process that initialises torch before the library, as bench.py does."""
    import sys
    d, path = _write(tmp_path, gpu, 8, 0.1, 30_000_001)
    orig = tmp_path / "orig.bin"
    d.tofile(orig)
    r = subprocess.run([sys.executable, "-c", _CALLER_STREAM_SCRIPT, os.path.join(ROOT, "cse375-finalproj-huffman-decoding_amd"),
                        path, str(tmp_path / "o.bin"), str(d.size), str(orig)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "caller-stream ok" in r.stdout, r.stdout[-1000:] + r.stderr[-2000:]


@pytest.mark.gpu
def test_raw_stream_shorter_than_n_is_an_error(gpu):
    """decode_raw must not return undecoded bytes when the stream holds fewer than N
    symbols: the size check rejects it before any decode."""
    import oracle
    data = gpu.generate(9, 0.5, 10_000)
    syms = oracle.symbols_of(data)
    units = oracle.raw_encode(data, syms)
    with pytest.raises(gpu.GapHuffError):
        gpu.decode_raw(units, syms, 40_000)
    assert np.array_equal(gpu.decode_raw(units, syms, data.size), data)


def _load_shards(gpu, path, bounds, concurrent):
    """Loads every shard of `path` into its own context on device 0, one host thread per
    shard (ctypes releases the GIL) or one after another; returns (ms, contexts)."""
    import threading
    import time
    decs = [gpu.Decoder(0) for _ in range(len(bounds) - 1)]
    t0 = time.perf_counter()
    if concurrent:
        th = [threading.Thread(target=decs[k].load_file, args=(path, bounds[k], bounds[k + 1]))
              for k in range(len(decs))]
        for t in th:
            t.start()
        for t in th:
            t.join()
    else:
        for k, dec in enumerate(decs):
            dec.load_file(path, bounds[k], bounds[k + 1])
    return (time.perf_counter() - t0) * 1e3, decs


@pytest.mark.gpu
def test_gpu_eight_shards_one_device_concurrent(gpu, tmp_path):
    """Eight shards on ONE device through the multi-shard entry points, each shard in its
    own host thread with pinned double-buffered copies: gh_decode with devices [0] * 8
    and bin/decoder --gpus 1 --shards 8 are bit-exact, and loading the eight shards from
    eight threads is not slower than loading them one after another, within 20 % (their
    file reads, staging copies and DMA overlap; one device's copy engines and the shared
    staging lease bound the gain, so a strict win is not asserted)."""
    import json
    d, path = _write(tmp_path, gpu, 8, 0.1, 160_000_000)
    img = np.fromfile(path, dtype=np.uint8)
    assert np.array_equal(gpu.decode(img, ngpus=8, devices=[0] * 8), d)
    b = gpu.plan_shards(gpu.parse(img).g, 8)
    times = {True: [], False: []}
    for rnd in range(3):
        for conc in (True, False):
            ms, decs = _load_shards(gpu, path, b, conc)
            if rnd:  # round 0 pins the staging sets
                times[conc].append(ms)
            parts = []
            for dec in decs:
                dec.decode()
                parts.append(dec.download(int(dec.report().out_bytes)))
                dec.close()
            assert np.array_equal(np.concatenate(parts)[: d.size], d)
    con, ser = min(times[True]), min(times[False])
    print(f"eight shards: concurrent {con:.1f} ms, one after another {ser:.1f} ms")
    assert con < 1.2 * ser, (con, ser)
    (tmp_path / "orig.bin").write_bytes(d.tobytes())
    out = str(tmp_path / "dec.bin")
    r = subprocess.run([os.path.join(BIN, "decoder"), path, out, "--gpus", "1", "--shards", "8", "--json",
                        "--verify", str(tmp_path / "orig.bin")], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "Verification: PASS" in r.stdout
    j = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert j["bitexact"] is True
