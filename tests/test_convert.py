"""String-format <-> gap-array conversion: bin/convert.

The string format is the reference CPU baselines' (sequential.cpp:163-204 header,
:37-51 MSB-first byte packing).  Pinned against the REFERENCE codec itself:
tests/golden/*.seq were written by sequential.cpp's encoder (made by
tests/golden/make_seq_golden.py through oracle/_ref/seq_driver), and when the
reference binaries are present the reference decoder reads our converted files."""
import hashlib
import json
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
CONVERT = os.path.join(ROOT, "bin", "convert")
SEQ = json.load(open(os.path.join(GOLD, "seq.json")))
HUFFS = sorted(f[:-5] for f in os.listdir(GOLD) if f.endswith(".huff"))

pytestmark = pytest.mark.skipif(not os.access(CONVERT, os.X_OK), reason="bin/convert not built")


def _run(*args):
    return subprocess.run([CONVERT, *map(str, args)], capture_output=True, text=True, timeout=60)


def _bin(name):
    return np.fromfile(os.path.join(GOLD, name + ".bin"), dtype=np.uint8)


@pytest.mark.parametrize("name", HUFFS)
def test_gap_seq_gap_roundtrip_identical(tmp_path, name):
    src = os.path.join(GOLD, name + ".huff")
    assert _run("to-seq", src, tmp_path / "a.seq").returncode == 0
    r = _run("to-gap", tmp_path / "a.seq", tmp_path / "b.huff")
    assert r.returncode == 0, r.stderr
    assert open(src, "rb").read() == open(tmp_path / "b.huff", "rb").read()


@pytest.mark.parametrize("name", HUFFS)
def test_reference_sequential_decodes_converted(orc, tmp_path, name):
    if not orc.ref_available("seq_driver"):
        pytest.skip("reference sequential.cpp not built (no /root/reference)")
    assert _run("to-seq", os.path.join(GOLD, name + ".huff"), tmp_path / "a.seq").returncode == 0
    subprocess.run([os.path.join(orc.REF, "seq_driver"), "dec", str(tmp_path / "a.seq"),
                    str(tmp_path / "out.bin")], check=True, timeout=60)
    assert np.array_equal(np.fromfile(tmp_path / "out.bin", dtype=np.uint8), _bin(name))


@pytest.mark.parametrize("name", sorted(SEQ))
def test_reference_seq_files_convert(orc, tmp_path, name):
    """Files the REFERENCE encoder wrote (plain Huffman tree, non-canonical codes):
    converted to gap arrays they decode (oracle) to the input; code lengths > 16
    (geometric input) are refused, the gap-array format's limit."""
    p = os.path.join(GOLD, name + ".seq")
    assert hashlib.sha256(open(p, "rb").read()).hexdigest() == SEQ[name]
    r = _run("to-gap", p, tmp_path / "c.huff")
    if name == "geometric_long_codes":
        assert r.returncode != 0 and "1..16" in r.stderr
        return
    assert r.returncode == 0, r.stderr
    out, _ = orc.decode(np.fromfile(tmp_path / "c.huff", dtype=np.uint8))
    assert np.array_equal(out, _bin(name))


def test_reference_encoder_live(orc, tmp_path):
    if not orc.ref_available("seq_driver"):
        pytest.skip("reference sequential.cpp not built (no /root/reference)")
    d = orc.generate(77, 0.7, 123457)
    d.tofile(tmp_path / "d.bin")
    subprocess.run([os.path.join(orc.REF, "seq_driver"), "enc", str(tmp_path / "d.bin"),
                    str(tmp_path / "d.seq")], check=True, timeout=60)
    assert _run("to-gap", tmp_path / "d.seq", tmp_path / "d.huff").returncode == 0
    out, _ = orc.decode(np.fromfile(tmp_path / "d.huff", dtype=np.uint8))
    assert np.array_equal(out, d)


@pytest.mark.parametrize("blob", [b"", b"\x09\x00\x01", b"\x00\x00\x02A\x01" + b"0" + b"B\x01" + b"0",
                                  b"\x00\x00\x01A\x02" + b"0x"])
def test_convert_rejects_bad_seq(tmp_path, blob):
    (tmp_path / "bad.seq").write_bytes(blob)
    assert _run("to-gap", tmp_path / "bad.seq", tmp_path / "o.huff").returncode != 0


@pytest.mark.gpu
def test_gpu_decodes_converted_reference_seq(gpu, tmp_path):
    name = "gen_r0.5_n20000"
    assert _run("to-gap", os.path.join(GOLD, name + ".seq"), tmp_path / "c.huff").returncode == 0
    assert np.array_equal(gpu.decode(np.fromfile(tmp_path / "c.huff", dtype=np.uint8)), _bin(name))
