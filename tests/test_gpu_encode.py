"""GPU encoder parity: the HIP encoder's compressed.huff
image, through the C ABI, byte-identical to the CPU oracle's restatement of the
reference encoder (encoder/src/huff.cpp:114-202, package_merge.cpp, encoder.cu:281-379)
and to the committed golden images; decoded back to the input by the GPU decoder."""
import glob
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _check(gh, orc, data, force_version=0):
    data = np.asarray(data, dtype=np.uint8)
    img = gh.encode_gpu(data, force_version=force_version)
    ref = orc.encode(data, force_v2=force_version == 2)
    assert img.size == ref.size
    if not np.array_equal(img, ref):
        bad = np.nonzero(img != ref)[0]
        raise AssertionError(f"{bad.size} differing bytes, first at {bad[0]} of {img.size}")
    return img


@pytest.mark.parametrize("r", [0.0, 0.1, 0.5, 0.9, 0.999, 1.0])
@pytest.mark.parametrize("n", [1, 2, 15, 16, 17, 1023, 1024, 1025, 2049, 4095, 4096, 4097, 65549, 1_000_003])
def test_generated_vs_oracle(gpu, orc, r, n):
    _check(gpu, orc, gpu.generate(2000 + n, r, n))


def test_golden_images(gpu):
    files = sorted(glob.glob(os.path.join(GOLDEN, "*.bin")))
    assert files
    for b in files:
        data = np.fromfile(b, dtype=np.uint8)
        want = np.fromfile(b[:-4] + ".huff", dtype=np.uint8)
        got = gpu.encode_gpu(data, force_version=2 if want[:8].tobytes() == b"GAPHUF2\0" else 0)
        assert np.array_equal(got, want), os.path.basename(b)


def test_single_and_two_symbols(gpu, orc):
    for n in (1, 5, 128, 129, 4096 * 3 + 1, 100_000):
        _check(gpu, orc, np.full(n, 65, dtype=np.uint8))
    rng = np.random.default_rng(5)
    for n in (10, 4097, 300_001):
        _check(gpu, orc, rng.integers(0, 2, n).astype(np.uint8) + 48)


def test_long_codes_and_all_gap_values(gpu, orc):
    # geometric frequencies: codes up to the 16-bit limit, gap nibbles 1..15
    rng = np.random.default_rng(11)
    data = np.minimum(rng.geometric(0.45, 2_000_000) - 1, 255).astype(np.uint8)
    img = _check(gpu, orc, data)
    s = gpu.parse(img)
    assert max(l for _, l in s.symbols) >= 14
    gaps = np.frombuffer(s.raw[s.raw.size - 4 * s.w - 4 * ((s.g + 7) // 8):][: 4 * ((s.g + 7) // 8)].tobytes(),
                         dtype=np.uint32)
    nib = {(int(w) >> (4 * k)) & 15 for w in gaps[:4096] for k in range(8)}
    assert len(nib) >= 12


@pytest.mark.parametrize("r", [0.1, 0.5])
@pytest.mark.parametrize("n", [8191, 8192, 8193, 16383, 16385, 24577])
def test_chunk_edges(gpu, orc, r, n):
    """Round 6: 8 KiB chunks of 512 threads: sizes around one, two and three chunks."""
    _check(gpu, orc, gpu.generate(3000 + n, r, n))


def test_chunks_of_longest_codewords(gpu, orc):
    """The write kernel's LDS image is sized at launch for the code's longest codeword: a
    run of 16 KiB of rare symbols (15-16-bit codewords) in a skewed stream fills two whole
    chunks' images close to that bound."""
    rng = np.random.default_rng(19)
    data = np.minimum(rng.geometric(0.5, 4_000_000) - 1, 40).astype(np.uint8)
    data[1_000_000:1_000_000 + 16384] = (np.arange(16384) % 200 + 50).astype(np.uint8)
    img = _check(gpu, orc, data)
    s = gpu.parse(img)
    assert max(l for _, l in s.symbols) >= 15


def test_v2_header(gpu, orc):
    _check(gpu, orc, gpu.generate(9, 0.5, 50_001), force_version=2)


def test_encoder_object_reuse_and_roundtrip(gpu):
    with gpu.Encoder(0) as e:
        for seed, r, n in ((1, 0.5, 3_000_001), (2, 0.9, 777), (3, 0.1, 2_000_000)):
            data = gpu.generate(seed, r, n)
            e.load(data)
            plan = e.make_plan()
            ms = e.encode()
            assert ms > 0.0
            img = e.download()
            assert img.size == plan.file_bytes
            assert np.array_equal(img, gpu.encode(data))
            assert np.array_equal(gpu.decode(img), data)


def test_large_roundtrip(gpu):
    data = gpu.generate(77, 0.5, 100_000_000)
    img = gpu.encode_gpu(data)
    assert np.array_equal(img, gpu.encode(data))


def test_cli_encoder_gpu(tmp_path, gpu, orc):
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    data = gpu.generate(4242, 0.9, 3_000_017)
    data.tofile(tmp_path / "in.bin")
    r = subprocess.run([os.path.join(root, "bin", "encoder"), str(tmp_path / "in.bin"), str(tmp_path / "c.huff"),
                        "--gpu", "0"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "Original size: 3000017 bytes" in r.stdout
    img = np.fromfile(tmp_path / "c.huff", dtype=np.uint8)
    assert np.array_equal(img, orc.encode(data))
    r = subprocess.run([os.path.join(root, "bin", "decoder"), str(tmp_path / "c.huff"), str(tmp_path / "out.bin")],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert np.array_equal(np.fromfile(tmp_path / "out.bin", dtype=np.uint8), data)


def test_empty_input(gpu, orc):
    img = gpu.encode_gpu(np.zeros(0, dtype=np.uint8))
    assert np.array_equal(img, gpu.encode(b""))
    assert gpu.decode(img).size == 0
