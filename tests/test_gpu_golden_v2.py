"""GPU decode of the committed golden streams and of v2 (64-bit header) images.

* Golden: every ``tests/golden/*.huff`` (made by tests/golden/make_golden.py; layout of
  Huffman_coding_Gap_arrays/encoder/src/huff.cpp:186-202) goes through the HIP decoder
  three ways -- ``gh.decode`` (gh_decode), ``Decoder.load_file`` (gh_ctx_load_file) and
  ``bin/decoder`` -- and must equal the paired ``.bin`` input and the oracle's
  bit-serial decode.  ``geometric_long_codes`` carries 16-bit codes and every gap
  nibble value, so it runs the long-code kernels.
* v2: the reference header is 32-bit (``int original_size`` / ``compressed_size`` /
  ``gap_elements_num``, decoder/src/huff.cpp:80-88), so streams with N, W or G >= 2^31
  use this repo's v2 header.  A small forced-v2 image goes through the same three
  entry points; the slow tests build the cfg5 stream (8 * 10^9 bytes, r = 0.5, v2 by
  size) with the host encoder and decode it on device 0 as 8 shards and as one
  context, each shard checked against the generator's slice at its output offset.
"""
import glob
import json
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
BIN = os.path.join(ROOT, "bin")
CASES = sorted(os.path.splitext(os.path.basename(p))[0] for p in glob.glob(os.path.join(GOLDEN, "*.huff")))


def _three_ways(gpu, orc, img: np.ndarray, want: np.ndarray, tmp_path, name: str):
    ref, _ = orc.decode(img)
    assert np.array_equal(ref, want), "oracle disagrees with the fixture input"
    # gh_decode (one-shot, whole stream)
    out = gpu.decode(img)
    assert np.array_equal(out, want), f"{name}: gh_decode differs"
    # gh_ctx_load_file + download
    path = tmp_path / f"{name}.huff"
    img.tofile(path)
    with gpu.Decoder(0) as d:
        info = d.load_file(str(path))
        assert info.n == want.size
        d.decode()
        rep = d.report()
        assert rep.status == 0
        assert rep.symbols >= want.size
        got = d.download(want.size) if want.size else np.zeros(0, np.uint8)
    assert np.array_equal(got, want), f"{name}: load_file decode differs"
    # bin/decoder (file in, file out)
    if not os.access(os.path.join(BIN, "decoder"), os.X_OK):
        pytest.fail("bin/decoder not built")
    outp = tmp_path / f"{name}.out"
    r = subprocess.run([os.path.join(BIN, "decoder"), str(path), str(outp)], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    assert np.array_equal(np.fromfile(outp, dtype=np.uint8), want), f"{name}: bin/decoder differs"


@pytest.mark.parametrize("name", CASES)
def test_golden_streams_decode(gpu, orc, tmp_path, name):
    img = np.fromfile(os.path.join(GOLDEN, name + ".huff"), dtype=np.uint8)
    want = np.fromfile(os.path.join(GOLDEN, name + ".bin"), dtype=np.uint8)
    meta = json.load(open(os.path.join(GOLDEN, "golden.json"))).get(name)
    s = gpu.parse(img)
    if meta is not None:
        assert s.n == meta["n"] and s.g == meta["g"]
        assert [list(x) for x in s.symbols] == [list(x) for x in meta["symbols"]]
    if name == "geometric_long_codes":
        assert max(l for _, l in s.symbols) == 16
    _three_ways(gpu, orc, img, want, tmp_path, name)


def test_golden_cases_present():
    # the fixtures the decoder is pinned to (CPU-side check that the glob saw them)
    assert "geometric_long_codes" in CASES and len(CASES) >= 12


@pytest.mark.parametrize("r,n", [(0.5, 1), (0.1, 100_003), (0.9, 1_000_000), (0.999, 333_333)])
def test_v2_small_image(gpu, orc, tmp_path, r, n):
    data = gpu.generate(2024 + n, r, n)
    img = gpu.encode(data, force_version=2)
    s = gpu.parse(img)
    assert s.version == 2
    assert int.from_bytes(img[:8].tobytes(), "little") == gpu.GH_V2_MAGIC
    _three_ways(gpu, orc, img, data, tmp_path, f"v2_{r}_{n}")
    # same payload as the v1 image: only the header differs
    img1 = gpu.encode(data)
    s1 = gpu.parse(img1)
    assert s1.version == 1 and s1.w == s.w and s1.g == s.g
    assert np.array_equal(img1[img1.size - 4 * s1.w:], img[img.size - 4 * s.w:])


def _cfg5_image(gpu):
    n = 8 * 10**9
    img = gpu.encode(gpu.generate(375, 0.5, n, threads=16), threads=16)
    s = gpu.parse(img)
    assert s.version == 2 and s.n == n
    return img, s


@pytest.mark.slow
def test_cfg5_8GB_v2_eight_shards(gpu):
    """cfg5 (BASELINE.json configs[4]): 8 GB r=0.5, v2 header, decoded on device 0 as
    the 8 shards bench.py gives 8 GPUs; shard k's bytes == generate(offset = sum of
    the earlier shards' symbol counts)."""
    img, s = _cfg5_image(gpu)
    bounds = gpu.plan_shards(s.g, 8)
    off = 0
    for k in range(8):
        with gpu.Decoder(0) as d:
            d.load(s, bounds[k], bounds[k + 1])
            d.decode()
            rep = d.report()
            assert rep.status == 0
            cnt = min(int(rep.symbols), s.n - off)
            assert cnt > 0 and (k == 7 or int(rep.symbols) == int(rep.out_bytes))
            got = d.download(cnt)
        want = gpu.generate(375, 0.5, cnt, offset=off, threads=16)
        assert np.array_equal(got, want), f"shard {k} differs"
        off += cnt
    assert off == s.n


@pytest.mark.slow
def test_cfg5_8GB_v2_one_context(gpu):
    """The same 8 GB stream as ONE shard (371 M segments, 8 * 10^9 output bytes: output
    offsets past 2^32), checked slice by slice."""
    img, s = _cfg5_image(gpu)
    with gpu.Decoder(0) as d:
        d.load(s)
        d.decode()
        rep = d.report()
        assert rep.status == 0 and int(rep.out_bytes) == s.n
        step = 10**9
        for off in range(0, s.n, step):
            got = d.download(min(step, s.n - off), offset=off)
            want = gpu.generate(375, 0.5, got.size, offset=off, threads=16)
            assert np.array_equal(got, want), f"bytes [{off}, {off + got.size}) differ"
