"""Host library (product) vs the oracle: encoder bytes, package-merge, generator,
header validation, and the drop-in CLIs.  No GPU needed."""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "bin")


@pytest.mark.parametrize("r", [0.0, 0.1, 0.5, 0.9, 0.999, 1.0])
@pytest.mark.parametrize("n", [0, 1, 2, 7, 128, 129, 5000, 300_001])
def test_encoder_matches_oracle(gh, orc, r, n):
    d = gh.generate(31 + n, r, n)
    assert np.array_equal(d, orc.generate(31 + n, r, n))
    a = gh.encode(d)
    if n == 0:
        s = gh.parse(a)
        assert s.n == 0 and s.g == 0 and s.w == 0
        return
    b = orc.encode(d)
    assert np.array_equal(a, b)


def test_encoder_threads_invariant(gh):
    d = gh.generate(3, 0.5, 3_000_000)
    ref = gh.encode(d, threads=1)
    for t in (2, 3, 8):
        assert np.array_equal(gh.encode(d, threads=t), ref)


def test_v2_header(gh, orc):
    d = gh.generate(4, 0.9, 10_000)
    a = gh.encode(d, force_version=2)
    assert np.array_equal(a, orc.encode(d, force_v2=True))
    s = gh.parse(a)
    assert s.version == 2 and s.n == d.size
    out, _ = orc.decode(a)
    assert np.array_equal(out, d)


def test_package_merge_product_vs_oracle(gh, orc):
    rng = np.random.default_rng(2)
    for _ in range(300):
        ns = int(rng.integers(1, 257))
        c = np.sort((2.0 ** rng.uniform(0, 28, ns)).astype(np.uint64) + 1, kind="stable")
        assert gh.package_merge(c) == orc.package_merge(c)


def test_length_limit_16(gh):
    fib = [1, 1]
    while len(fib) < 40:
        fib.append(fib[-1] + fib[-2])
    lens = gh.package_merge(sorted(fib))
    assert max(lens) == 16 and sum(2.0 ** -l for l in lens) <= 1.0


def test_generator_distribution(gh):
    n = 2_000_000
    for r in (0.1, 0.5, 0.9):
        d = gh.generate(9, r, n)
        frac = np.isin(d, np.frombuffer(b"ABCD", dtype=np.uint8)).mean()
        assert abs(frac - (r + (1 - r) * 4 / 256)) < 0.003
        assert np.array_equal(gh.generate(9, r, 1000, offset=12345), d[12345:13345])


def _hdr(syms, n, w, g):
    b = np.uint64(len(syms)).tobytes() + bytes(x for s in syms for x in s)
    return b + np.array([n, w, g], dtype="<u4").tobytes()


def test_parse_rejects_malformed(gh):
    d = gh.generate(5, 0.5, 10_000)
    img = gh.encode(d).tobytes()
    gh.parse(img)
    bad = [
        img[:5],                                   # truncated S
        np.uint64(300).tobytes() + img[8:],       # S > 256
        img[:-4],                                 # truncated payload
        _hdr([(65, 0), (66, 1)], 1, 1, 1) + b"\0" * 8,     # zero length
        _hdr([(65, 1), (66, 1), (67, 1)], 1, 1, 1) + b"\0" * 8,  # Kraft > 1
        _hdr([(65, 2), (66, 1)], 1, 1, 1) + b"\0" * 8,     # not canonical order
        _hdr([(65, 1), (65, 1)], 1, 1, 1) + b"\0" * 8,     # duplicate symbol
        _hdr([(65, 1), (66, 1)], 10, 1, 3) + b"\0" * 8,    # W inconsistent with G
        _hdr([(65, 1), (66, 1)], 100, 1, 1) + b"\0" * 8,   # N too large for W
    ]
    for b in bad:
        with pytest.raises(gh.GapHuffError):
            gh.parse(b)


def test_shard_plan(gh):
    for g, k in [(0, 1), (10, 3), (1_000_003, 8), (5, 8)]:
        b = gh.plan_shards(g, k)
        assert b[0] == 0 and b[-1] == g and all(x <= y for x, y in zip(b, b[1:]))


@pytest.mark.skipif(not os.access(os.path.join(BIN, "encoder"), os.X_OK), reason="CLIs not built")
def test_cli_encoder_generate(tmp_path, gh, orc):
    subprocess.run([os.path.join(BIN, "generate"), "100000", "0.5", "--seed", "42",
                    "--out", str(tmp_path / "data.bin")], check=True, capture_output=True)
    d = np.fromfile(tmp_path / "data.bin", dtype=np.uint8)
    assert np.array_equal(d, gh.generate(42, 0.5, 100000))
    r = subprocess.run([os.path.join(BIN, "encoder"), str(tmp_path / "data.bin"),
                        str(tmp_path / "c.huff")], check=True, capture_output=True, text=True)
    assert "Original size: 100000 bytes" in r.stdout
    img = np.fromfile(tmp_path / "c.huff", dtype=np.uint8)
    assert np.array_equal(img, orc.encode(d))


@pytest.mark.skipif(not os.access(os.path.join(BIN, "decoder"), os.X_OK), reason="CLIs not built")
def test_cli_decoder_rejects_garbage(tmp_path):
    (tmp_path / "bad.huff").write_bytes(b"\x05\x00\x00")
    r = subprocess.run([os.path.join(BIN, "decoder"), str(tmp_path / "bad.huff"),
                        str(tmp_path / "out")], capture_output=True, text=True)
    assert r.returncode != 0
