"""Self-synchronising decode of gap-less (raw) streams — SURVEY.md §8(f) rank 3.

Reference: gpuhd's CUHD decoder (gpuhd/src/cuhd_gpu_decoder.cu:145-523) over raw u32
units from the LLHuff encoder (gpuhd/encoder/src/llhuffman_encoder.cc:200-238).
CPU tests pin the oracle's raw-stream restatement (oracle.raw_encode / raw_gaps /
raw_decode) against the REFERENCE encoder's own output (tests/golden/*.llh, made by
tests/golden/make_llhuff_golden.py from oracle/_ref/llhuff_driver) and against the
gap-array encoder.  GPU tests call the C ABI (gh_sync_gaps, gh_ctx_load_raw) and
compare bit-exactly with the oracle.
"""
import json
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
LLH = json.load(open(os.path.join(GOLD, "llhuff.json")))


def _llh(name):
    import oracle
    return oracle.read_llh(open(os.path.join(GOLD, name + ".llh"), "rb").read())


def _bin(name):
    return np.fromfile(os.path.join(GOLD, name + ".bin"), dtype=np.uint8)


# ------------------------------------------------------------------------- CPU
@pytest.mark.parametrize("name", sorted(LLH))
def test_llhuff_golden_units_reproduced(orc, name):
    """The oracle's packing == the reference encode_memory units (all but the last
    unit, which encode_memory leaves undefined when the data ends mid-unit)."""
    import hashlib
    b = open(os.path.join(GOLD, name + ".llh"), "rb").read()
    assert hashlib.sha256(b).hexdigest() == LLH[name]["sha256"]
    syms, units = _llh(name)
    data = _bin(name)
    mine = orc.raw_encode(data, syms)
    if len(syms) == 1:
        # reference defect: get_symbol_lengths leaves Symbol::count unset for a
        # one-symbol input (llhuffman_encoder.cc:39-47), so compressed_size is 0
        assert units.size == 0 and not mine.any()
        return
    assert mine.size == units.size == LLH[name]["units"]
    assert np.array_equal(mine[:-1], units[:-1])


@pytest.mark.parametrize("name", sorted(LLH))
def test_llhuff_golden_decodes(orc, name):
    syms, units = _llh(name)
    data = _bin(name)
    assert np.array_equal(orc.raw_decode(units, syms, data.size), data)


def test_llhuff_reference_live(orc):
    if not orc.ref_available("llhuff_driver"):
        pytest.skip("reference raw encoder not built (no /root/reference)")
    for seed, r in ((11, 0.3), (12, 0.95), (13, 0.05)):
        d = orc.generate(seed, r, 30011)
        syms, units = orc.ref_llhuff(d)
        assert max(l for _, l in syms) <= 11  # CUHD's MAX_CODEWORD_LENGTH
        assert np.array_equal(orc.raw_encode(d, syms)[:-1], units[:-1])


@pytest.mark.parametrize("r,n", [(0.5, 20000), (0.9, 20000), (0.1, 3000), (0.999, 50000), (0.5, 7),
                                 (0.5, 1)])
def test_raw_stream_is_gap_array_payload(orc, gh, r, n):
    """A gap-array file's payload is the raw stream of its code, and its gap words are
    the raw stream's segment entries (so the GPU's synthesised gaps have a fixed
    expected value)."""
    import ctypes
    d = orc.generate(1, r, n)
    s = gh.parse(orc.encode(d))
    nw = (s.g + 7) // 8
    gw = np.ctypeslib.as_array(ctypes.cast(s.c.gap_words, ctypes.POINTER(ctypes.c_uint32)), (max(nw, 1),))[:nw]
    pw = np.ctypeslib.as_array(ctypes.cast(s.c.payload, ctypes.POINTER(ctypes.c_uint32)), (max(s.w, 1),))[:s.w]
    assert np.array_equal(orc.raw_gaps(d, s.symbols), gw)
    assert np.array_equal(orc.raw_encode(d, s.symbols), pw)


@pytest.mark.parametrize("n", [200, 270, 290])
def test_raw_gaps_last_codeword_crossing(orc, gh, n):
    """r = 0.1, seed 11: at n = 270 the stream's last codeword crosses the boundary
    128 (g - 1) and ends 2 bits past it; the gap-array encoder records that end
    (encoder.cu:307-312), and so must the raw stream's gap words."""
    import ctypes
    d = orc.generate(11, 0.1, n)
    s = gh.parse(orc.encode(d))
    nw = (s.g + 7) // 8
    gw = np.ctypeslib.as_array(ctypes.cast(s.c.gap_words, ctypes.POINTER(ctypes.c_uint32)), (max(nw, 1),))[:nw]
    assert np.array_equal(orc.raw_gaps(d, s.symbols), gw)


def test_desync_table_oracle(orc):
    """The adversarial stream of the GPU repair test: a 1-bit code plus four 3-bit
    codes, data all '111' — a walk that starts off the 3-bit phase never resyncs."""
    syms = [(0, 1), (1, 3), (2, 3), (3, 3), (4, 3)]
    d = np.full(1000, 4, dtype=np.uint8)
    u = orc.raw_encode(d, syms)
    assert np.all(u[:-1] == 0xFFFFFFFF)
    assert np.array_equal(orc.raw_decode(u, syms, d.size), d)


def test_sync_abi_exports(gh):
    L = gh.lib()
    for name in ("gh_sync_gaps", "gh_ctx_load_raw", "gh_ctx_device"):
        assert hasattr(L, name)


# ------------------------------------------------------------------------- GPU
def _sync_on_gpu(gh, units, syms):
    w = int(units.size)
    g = (w + 3) // 4
    nw = (g + 7) // 8
    src = np.concatenate([units, np.zeros(4, np.uint32)]).astype(np.uint32)
    gaps = np.full(nw + 4, 0xFFFFFFFF, dtype=np.uint32)
    with gh.DeviceBuffer(src.nbytes) as dw, gh.DeviceBuffer(gaps.nbytes) as dg:
        dw.upload(src)
        dg.upload(gaps)
        rep = gh.sync_gaps(syms, dw.addr, w, dg.addr, device=0)
        dg.download(gaps)
    assert np.all(gaps[nw:] == 0xFFFFFFFF), "wrote past the gap words"
    return gaps[:nw], rep


@pytest.mark.gpu
@pytest.mark.parametrize("r,n", [(0.5, 1), (0.5, 7), (0.5, 20000), (0.9, 300007), (0.1, 300007),
                                 (0.999, 1 << 20), (0.0, 65536), (1.0, 4096)])
def test_gpu_sync_gaps_match_oracle(gpu, orc, r, n):
    d = orc.generate(7, r, n)
    syms = orc.symbols_of(d)
    units = orc.raw_encode(d, syms)
    gaps, rep = _sync_on_gpu(gpu, units, syms)
    assert rep.g == (units.size + 3) // 4
    assert np.array_equal(gaps, orc.raw_gaps(d, syms))


@pytest.mark.gpu
@pytest.mark.parametrize("n", [200, 270, 290, 16_720, 16_740, 16_760, 33_440, 33_460, 49_100])
def test_gpu_sync_block_and_wave_edges(gpu, orc, n):
    """r = 0.1 streams (~16 symbols per segment) whose segment counts fall around the
    walk kernel's block (16 segments per lane) and wave (1024 segments) edges: a last
    block shorter than 16 segments, exactly 16, 17 (g = 11, 16, 17, 1023, 1024, 1025,
    2048, 2049, 3008): a wave with one lane, the fix pass's wave starts."""
    d = orc.generate(11, 0.1, n)
    syms = orc.symbols_of(d)
    units = orc.raw_encode(d, syms)
    gaps, rep = _sync_on_gpu(gpu, units, syms)
    assert np.array_equal(gaps, orc.raw_gaps(d, syms))
    assert np.array_equal(gpu.decode_raw(units, syms, d.size), d)


@pytest.mark.gpu
def test_gpu_sync_long_codes(gpu, orc):
    """Codes longer than the 13-bit sync LUT (SK = 13, gh_sync.hip: the LONG kernels'
    canonical-threshold path), up to 16 bits, from the geometric fixture."""
    d = _bin("geometric_long_codes")
    syms = orc.symbols_of(d)
    assert max(l for _, l in syms) > SYNC_LUT_BITS
    units = orc.raw_encode(d, syms)
    gaps, _ = _sync_on_gpu(gpu, units, syms)
    assert np.array_equal(gaps, orc.raw_gaps(d, syms))
    assert np.array_equal(gpu.decode_raw(units, syms, d.size), d)


SYNC_LUT_BITS = 13  # SK in csrc/gh_sync.hip


@pytest.mark.gpu
@pytest.mark.parametrize("maxlen", [SYNC_LUT_BITS, SYNC_LUT_BITS + 1])
def test_gpu_sync_lut_boundary_codes(gpu, orc, maxlen):
    """Complete codes whose longest codeword is exactly SK bits (fits the LUT: plain
    kernel) and exactly SK + 1 bits (the LONG kernel): lengths 1, 2, ..., maxlen-1,
    maxlen, maxlen (Kraft sum 1), symbols drawn with probability 2^-length."""
    lens = list(range(1, maxlen)) + [maxlen, maxlen]
    syms = [(40 + i, l) for i, l in enumerate(lens)]
    p = np.array([2.0 ** -l for l in lens])
    rng = np.random.default_rng(maxlen)
    d = rng.choice(np.array([s for s, _ in syms], dtype=np.uint8), size=400_000, p=p / p.sum())
    assert max(l for _, l in syms) == maxlen
    units = orc.raw_encode(d, syms)
    gaps, _ = _sync_on_gpu(gpu, units, syms)
    assert np.array_equal(gaps, orc.raw_gaps(d, syms))
    assert np.array_equal(gpu.decode_raw(units, syms, d.size), d)


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(LLH))
def test_gpu_decode_reference_llhuff_streams(gpu, name):
    """Streams written by the REFERENCE raw encoder decode to the input."""
    syms, units = _llh(name)
    data = _bin(name)
    if units.size == 0:  # the reference's one-symbol defect: an empty, truncated stream
        with pytest.raises(gpu.GapHuffError):
            gpu.decode_raw(units, syms, data.size)
        return
    assert np.array_equal(gpu.decode_raw(units, syms, data.size), data)


@pytest.mark.gpu
@pytest.mark.parametrize("r", [0.1, 0.5, 0.9])
def test_gpu_decode_raw_roundtrip(gpu, orc, r):
    d = orc.generate(21, r, 3_000_017)
    syms = orc.symbols_of(d)
    units = orc.raw_encode(d, syms)
    with gpu.Decoder(0) as dec:
        rep = dec.load_raw(syms, d.size, units)
        dec.decode()
        out = dec.download(d.size)
        assert dec.report().status == 0
    assert rep.passes >= 1
    assert np.array_equal(out, d)


@pytest.mark.gpu
@pytest.mark.parametrize("n,stride", [(100_000, 0), (40_000, 997)])
def test_gpu_sync_repairs_desync(gpu, orc, n, stride, monkeypatch):
    """Adversarial code whose walks never resynchronise on their own: the in-wave
    verify and the fix pass must find the mismatches and the repairs must fix every
    boundary (a stream of one wave's blocks needs no second fix pass).  The halo is held
    at 6 segments (the stream-derived one would avoid the mismatches this test needs)."""
    monkeypatch.setenv("GH_SYNC_HALO", "6")
    syms = [(0, 1), (1, 3), (2, 3), (3, 3), (4, 3)]
    d = np.full(n, 4, dtype=np.uint8)
    if stride:
        d[::stride] = 0  # an occasional 1-bit codeword shifts the phase
    units = orc.raw_encode(d, syms)
    gaps, rep = _sync_on_gpu(gpu, units, syms)
    assert rep.mismatches > 0 and rep.passes >= 1
    assert np.array_equal(gaps, orc.raw_gaps(d, syms))
    assert np.array_equal(gpu.decode_raw(units, syms, d.size), d)
    monkeypatch.delenv("GH_SYNC_HALO")
    gaps, rep = _sync_on_gpu(gpu, units, syms)  # the stream-derived halo: exact gaps too
    assert np.array_equal(gaps, orc.raw_gaps(d, syms))


@pytest.mark.gpu
def test_gpu_sync_halo_follows_the_stream(gpu, orc, capfd, monkeypatch):
    """The warm-up halo is chosen per stream from its sampled resynchronisation distances
    (gh_sync.hip sync_halo_for): short for a fast-merging r = 0.9 code, long for r = 0.5
    (slow merging, and a short stream), and the gaps stay exact either way."""
    monkeypatch.setenv("GH_SYNC_VERBOSE", "1")
    halos = {}
    for r in (0.9, 0.5):
        d = gpu.generate(11, r, 2_000_000)
        s = gpu.parse(gpu.encode(d))
        import ctypes
        pw = np.ctypeslib.as_array(ctypes.cast(s.c.payload, ctypes.POINTER(ctypes.c_uint32)), (s.w,)).copy()
        capfd.readouterr()
        gaps, rep = _sync_on_gpu(gpu, pw, s.symbols)
        err = capfd.readouterr().err
        halos[r] = int(err.split("halo")[-1].split()[0])
        assert rep.halo == halos[r]  # the report carries the halo the walk used
        assert rep.host_ms > 0  # and the time of its estimate (not inside kernel_ms)
        gw = np.ctypeslib.as_array(ctypes.cast(s.c.gap_words, ctypes.POINTER(ctypes.c_uint32)), (gaps.size,))
        assert np.array_equal(gaps, gw)
    assert halos[0.9] <= 4 < 10 <= halos[0.5], halos


@pytest.mark.gpu
def test_gpu_sync_halo_saturates_when_walks_never_merge(gpu, orc, monkeypatch):
    """A code whose walks from a wrong offset never merge (every codeword 8 bits: 7 of 8
    sampled offsets stay out of phase for good) gives a p99.9 resync distance of 'never'.
    The short-stream halo then saturates at its maximum (48 segments) instead of wrapping
    to the minimum, and the verify passes still make every gap exact."""
    monkeypatch.delenv("GH_SYNC_HALO", raising=False)
    syms = [(i, 8) for i in range(256)]
    d = orc.generate(3, 0.5, 300_001)
    units = orc.raw_encode(d, syms)
    gaps, rep = _sync_on_gpu(gpu, units, syms)
    assert rep.halo == 48, rep.halo
    assert rep.host_ms > 0
    assert np.array_equal(gaps, orc.raw_gaps(d, syms))


@pytest.mark.gpu
@pytest.mark.parametrize("halo", ["0", "1"])
def test_gpu_sync_forced_small_halo_many_repairs(gpu, orc, halo, monkeypatch):
    """A 4 MB r = 0.5 stream (slow-merging code: walks from a wrong bit need ~330 bits on
    average, p99 ~2400) with the warm-up forced down to 0-1 segments: a large share of the
    blocks fail verification and are re-walked inside their waves (and across waves by the
    fix pass), and the gaps still equal the encoder's, the decode the input.  The time of
    this case at 10^8 B is recorded by scripts/bench_sync.py --halo (profiles/r06_sync.jsonl)."""
    monkeypatch.setenv("GH_SYNC_HALO", halo)
    import ctypes
    d = gpu.generate(23, 0.5, 4_000_000)
    s = gpu.parse(gpu.encode(d))
    pw = np.ctypeslib.as_array(ctypes.cast(s.c.payload, ctypes.POINTER(ctypes.c_uint32)), (s.w,)).copy()
    gaps, rep = _sync_on_gpu(gpu, pw, s.symbols)
    nblk = (s.g + 31) // 32
    assert rep.halo == int(halo)
    assert rep.mismatches > nblk // 20, (rep.mismatches, nblk)  # many repairs, not a few
    gw = np.ctypeslib.as_array(ctypes.cast(s.c.gap_words, ctypes.POINTER(ctypes.c_uint32)), (gaps.size,))
    assert np.array_equal(gaps, gw)
    assert np.array_equal(gpu.decode_raw(pw, s.symbols, d.size), d)


@pytest.mark.gpu
def test_gpu_decode_raw_empty(gpu):
    with gpu.Decoder(0) as dec:
        rep = dec.load_raw([(65, 1)], 0, np.zeros(0, np.uint32))
        assert rep.g == 0
    assert gpu.decode_raw(np.zeros(0, np.uint32), [(65, 1)], 0).size == 0


@pytest.mark.gpu
def test_gpu_decode_raw_large_property(gpu, orc):
    """64 MiB r=0.1 stream: decode == input (size-independent round trip)."""
    d = gpu.generate(5, 0.1, 1 << 26)
    s = gpu.parse(gpu.encode(d))
    import ctypes
    pw = np.ctypeslib.as_array(ctypes.cast(s.c.payload, ctypes.POINTER(ctypes.c_uint32)), (s.w,))
    assert np.array_equal(gpu.decode_raw(pw.copy(), s.symbols, d.size), d)


@pytest.mark.gpu
@pytest.mark.parametrize("halo", ["0", "8", "56"])
def test_gpu_sync_halo_variants(gpu, orc, halo, monkeypatch):
    """Warm-up segments per lane (GH_SYNC_HALO) change only how much the verify pass has to
    repair, never the gaps."""
    monkeypatch.setenv("GH_SYNC_HALO", halo)
    d = orc.generate(9, 0.5, 400_009)
    syms = orc.symbols_of(d)
    units = orc.raw_encode(d, syms)
    gaps, rep = _sync_on_gpu(gpu, units, syms)
    assert np.array_equal(gaps, orc.raw_gaps(d, syms))


def _random_code(rng, orc):
    """A random canonical (symbol, length) list: package-merge lengths of random counts,
    sometimes lengthened (incomplete code, Kraft < 1), lengths <= 16."""
    ns = int(rng.integers(2, 257))
    counts = np.sort(rng.geometric(rng.uniform(0.01, 0.5), ns).astype(np.uint64) *
                     rng.integers(1, 1000, ns).astype(np.uint64))
    lens = orc.package_merge(counts)  # ascending-count order
    lens = sorted(lens)
    if rng.random() < 0.5:  # make it incomplete
        for i in range(len(lens) - 1, max(-1, len(lens) - 4), -1):
            lens[i] = min(16, lens[i] + 1)
        lens = sorted(lens)
    syms = [int(x) for x in rng.permutation(256)[:ns]]
    return list(zip(syms, lens))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(12))
def test_gpu_sync_random_codes(gpu, orc, seed):
    """Random codes (complete and incomplete, up to 16-bit codewords) and data drawn
    with random skew: synthesised gaps equal the oracle's, the decode equals the data."""
    rng = np.random.default_rng(1000 + seed)
    syms = _random_code(rng, orc)
    p = rng.dirichlet(np.full(len(syms), rng.uniform(0.05, 2.0)))
    n = int(rng.integers(1, 200_000))
    d = np.array([s for s, _ in syms], dtype=np.uint8)[rng.choice(len(syms), n, p=p)]
    units = orc.raw_encode(d, syms)
    gaps, _ = _sync_on_gpu(gpu, units, syms)
    assert np.array_equal(gaps, orc.raw_gaps(d, syms))
    assert np.array_equal(gpu.decode_raw(units, syms, n), d)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [100_003, 8_191, 1_000_001])
def test_gpu_incomplete_code_large_unused_region(gpu, orc, n):
    """A code with a quarter of its code space unused ('11' of three 2-bit codewords):
    lanes past the shard end and segments past their end decode stray bits that hit
    the unused pattern; only lookups of kept codewords may flag the stream as corrupt
    (the wave split's canonical fallback).  nseg is not a multiple of a block."""
    syms = [(65, 2), (66, 2), (67, 2)]
    rng = np.random.default_rng(n)
    d = np.array([65, 66, 67], dtype=np.uint8)[rng.integers(0, 3, n)]
    units = orc.raw_encode(d, syms)
    assert (2 * n + 127) // 128 % 256 != 0
    assert np.array_equal(gpu.decode_raw(units, syms, n), d)


BIN = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bin")


@pytest.mark.skipif(not os.access(os.path.join(BIN, "encoder"), os.X_OK), reason="CLIs not built")
@pytest.mark.parametrize("r,n", [(0.5, 100_003), (0.9, 1), (0.5, 0)])
def test_cli_encoder_raw_container(orc, gh, tmp_path, r, n):
    """bin/encoder --raw: same code and payload as the gap-array file, no gaps."""
    import subprocess
    d = orc.generate(8, r, n)
    d.tofile(tmp_path / "d.bin")
    subprocess.run([os.path.join(BIN, "encoder"), str(tmp_path / "d.bin"), str(tmp_path / "d.raw"), "--raw"],
                   check=True, capture_output=True, timeout=60)
    syms, n2, units = gh.parse_raw(np.fromfile(tmp_path / "d.raw", dtype=np.uint8))
    assert n2 == n and syms == orc.symbols_of(d) if n else n2 == 0
    if n:
        assert np.array_equal(units, orc.raw_encode(d, syms))


def test_raw_parse_rejects_bad(gh):
    with pytest.raises(gh.GapHuffError):
        gh.parse_raw(b"GHRAW1\x00\x00" + b"\x00" * 4)
    with pytest.raises(gh.GapHuffError):
        gh.parse_raw(b"\x01" * 64)


@pytest.mark.gpu
def test_gpu_cli_decoder_raw_container(gpu, orc, tmp_path):
    import subprocess
    d = orc.generate(9, 0.5, 2_000_003)
    d.tofile(tmp_path / "d.bin")
    subprocess.run([os.path.join(BIN, "encoder"), str(tmp_path / "d.bin"), str(tmp_path / "d.raw"), "--raw"],
                   check=True, capture_output=True, timeout=60)
    r = subprocess.run([os.path.join(BIN, "decoder"), str(tmp_path / "d.raw"), str(tmp_path / "o.bin"),
                        "--verify", str(tmp_path / "d.bin")], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "Raw stream" in r.stdout and "Verification: PASS" in r.stdout


def test_raw_parse_fuzz(gh, orc):
    """Truncated / corrupted raw containers: an error or a valid parse, never a crash."""
    rng = np.random.default_rng(3)
    d = orc.generate(2, 0.5, 5000)
    syms = orc.symbols_of(d)
    units = orc.raw_encode(d, syms)
    hdr = np.concatenate([np.frombuffer(np.uint64(0x0000315741524847).tobytes(), np.uint8),
                          np.frombuffer(np.uint64(len(syms)).tobytes(), np.uint8),
                          np.array([x for e in syms for x in e], np.uint8),
                          np.frombuffer(np.array([d.size, units.size], np.uint64).tobytes(), np.uint8),
                          units.view(np.uint8)])
    s2, n2, u2 = gh.parse_raw(hdr)
    assert s2 == syms and n2 == d.size and np.array_equal(u2, units)
    for _ in range(300):
        b = hdr[: int(rng.integers(0, hdr.size + 1))].copy()
        for _ in range(int(rng.integers(0, 4))):
            if b.size:
                b[int(rng.integers(0, min(b.size, 600)))] = int(rng.integers(0, 256))
        try:
            gh.parse_raw(b)
        except gh.GapHuffError:
            pass


def test_sync_gaps_argument_checks(gh):
    """Checked before any device work (so they run without a GPU)."""
    with pytest.raises(gh.GapHuffError) as e:
        gh.sync_gaps([(65, 1), (66, 1)], 4, 8, 1 << 20)  # d_words not 16-byte aligned
    assert e.value.code == -1
    with pytest.raises(gh.GapHuffError) as e:
        gh.sync_gaps([(65, 2), (66, 1)], 1 << 20, 8, 1 << 20)  # lengths not canonical order
    assert e.value.code == -3
    with pytest.raises(gh.GapHuffError) as e:
        gh.sync_gaps([(65, 1), (66, 1), (67, 1)], 1 << 20, 8, 1 << 20)  # Kraft sum > 1
    assert e.value.code == -3
    assert gh.sync_gaps([(65, 1)], 1 << 20, 0, 1 << 20).g == 0  # empty stream: nothing to do
