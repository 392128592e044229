"""GPU parity tests: the HIP decoder (through the C ABI) against the CPU oracle and
the original input, bit-exact.  Reference semantics: Huffman_coding_Gap_arrays/
decoder/src/decoder.cu:454-730 (see oracle/gh_oracle.c for the restatement)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _roundtrip(gh, orc, data, **kw):
    img = gh.encode(data)
    out = gh.decode(img, **kw)
    ref, _ = orc.decode(img)
    assert ref.size == len(data) and np.array_equal(ref, np.asarray(data, dtype=np.uint8))
    assert out.size == len(data)
    if not np.array_equal(out, ref):
        bad = np.nonzero(out != ref)[0]
        raise AssertionError(f"{bad.size} mismatches, first at {bad[0]} of {out.size}")
    return img


@pytest.mark.parametrize("r", [0.0, 0.1, 0.5, 0.9, 0.999, 1.0])
@pytest.mark.parametrize("n", [1, 2, 7, 100, 4097, 65549, 1_000_003])
def test_generated_vs_oracle(gpu, orc, r, n):
    data = gpu.generate(1000 + n, r, n)
    _roundtrip(gpu, orc, data)


def test_single_symbol(gpu, orc):
    for n in (1, 5, 128, 129, 100_000):
        _roundtrip(gpu, orc, np.full(n, 65, dtype=np.uint8))


def test_two_symbols_one_bit_codes(gpu, orc):
    rng = np.random.default_rng(3)
    for n in (10, 1000, 300_001):
        data = rng.integers(0, 2, n).astype(np.uint8) + 48
        img = _roundtrip(gpu, orc, data)
        assert max(l for _, l in gpu.parse(img).symbols) == 1


def test_long_codes_up_to_16_bits(gpu, orc):
    # geometric counts force length-limited codes up to MAX_CODEWORD_LENGTH = 16
    counts = [max(1, int(2 ** (24 - 0.9 * i))) for i in range(40)]
    data = np.repeat(np.arange(40, dtype=np.uint8), counts)
    np.random.default_rng(5).shuffle(data)
    img = _roundtrip(gpu, orc, data)
    assert max(l for _, l in gpu.parse(img).symbols) == 16


def test_exact_segment_multiple(gpu, orc):
    # 256 equal counts -> all codes 8 bits; n = 16k -> bits is a multiple of 128
    data = np.tile(np.arange(256, dtype=np.uint8), 64)
    np.random.default_rng(9).shuffle(data)
    img = _roundtrip(gpu, orc, data)
    s = gpu.parse(img)
    assert s.w * 32 == s.g * 128


@pytest.mark.parametrize("k", [1, 6, 8, 10, 12])
def test_lut_widths(gpu, orc, k, monkeypatch):
    monkeypatch.setenv("GH_LUT_BITS", str(k))
    for r in (0.1, 0.9):
        _roundtrip(gpu, orc, gpu.generate(77, r, 200_000))


@pytest.mark.parametrize("nshards", [2, 3, 8])
def test_shards_on_one_device(gpu, orc, nshards):
    data = gpu.generate(11, 0.5, 2_000_000)
    _roundtrip(gpu, orc, data, ngpus=nshards, devices=[0] * nshards)


def test_shard_counts_match_oracle(gpu, orc):
    data = gpu.generate(12, 0.9, 300_000)
    img = gpu.encode(data)
    s = gpu.parse(img)
    bounds = gpu.plan_shards(s.g, 5)
    off = 0
    for k in range(5):
        with gpu.Decoder(0) as d:
            d.load(s, bounds[k], bounds[k + 1])
            d.decode()
            r = d.report()
            expect = sum(orc.segment_count(img, i) for i in range(bounds[k], bounds[k + 1]))
            assert r.symbols == expect
            keep = min(r.symbols, s.n - off)
            got = d.download(keep)
            assert np.array_equal(got, data[off:off + keep])
            off += r.symbols


def test_repeated_decodes_identical(gpu):
    data = gpu.generate(13, 0.5, 3_000_000)
    img = gpu.encode(data)
    s = gpu.parse(img)
    with gpu.Decoder(0) as d:
        d.load(s)
        for _ in range(5):
            d.decode()
        r = d.report()
        assert r.launches == 5 and r.status == 0 and r.symbols >= s.n
        assert np.array_equal(d.download(s.n), data)


def test_reference_launcher_mirror(gpu):
    data = gpu.generate(14, 0.9, 123_457)
    img = gpu.encode(data)
    s = gpu.parse(img)
    words = np.concatenate([np.frombuffer(s.raw[len(s.raw) - 4 * (s.w + (s.g + 7) // 8):].tobytes(),
                                          dtype=np.uint32)])
    out = gpu.decoder_l1_l2(words, s.w, s.n, s.g, s.symbols)
    assert np.array_equal(out, data)


@pytest.mark.parametrize("r", [0.9, 0.5, 0.1])
def test_corrupted_stream_terminates(gpu, r):
    """Flipped payload bytes (each structure: r = 0.9 wave split, r = 0.5 / 0.1 tile
    kernel shapes): an error or a bounded, wrong output, never a hang or a fault."""
    data = gpu.generate(15, r, 500_000)
    img = gpu.encode(data).copy()
    rng = np.random.default_rng(1)
    hdr = 8 + 2 * len(gpu.parse(img).symbols) + 12
    for pos in rng.integers(hdr, img.size, 200):
        img[pos] ^= 0xFF
    try:
        out = gpu.decode(img)  # either an error or a bounded, wrong output
        assert out.size == data.size
    except gpu.GapHuffError as e:
        assert e.code in (-7, -2)


def test_empty_stream(gpu):
    img = gpu.encode(b"")
    assert gpu.decode(img).size == 0


@pytest.mark.parametrize("cfg", [("cfg2", 10**8, 0.5)])
def test_config2_100MB_bitexact(gpu, cfg):
    _, n, r = cfg
    data = gpu.generate(375, r, n)
    img = gpu.encode(data)
    out = gpu.decode(img)
    assert np.array_equal(out, data)


@pytest.mark.slow
@pytest.mark.parametrize("cfg", [("cfg3", 10**9, 0.9), ("cfg4", 10**9, 0.1)])
def test_config_1GB_bitexact(gpu, cfg):
    # size-independent property at full size: decode(encode(x)) == x
    _, n, r = cfg
    data = gpu.generate(375, r, n)
    img = gpu.encode(data)
    out = gpu.decode(img)
    assert np.array_equal(out, data)


@pytest.mark.parametrize("mode", ["tile", "wsplit"])
def test_both_structures_on_grouped_codes(gpu, orc, mode, monkeypatch):
    """Grouped codes (complete, 4..12-bit codewords) decode to the same bytes through
    the tile kernel and through the wave split (GH_MODE), and so do codes the tile
    kernel does not take (codewords up to 16 bits: the wave split's canonical
    fallback)."""
    monkeypatch.setenv("GH_MODE", mode)
    cases = [gpu.generate(21, 0.1, 300_001), gpu.generate(22, 0.0, 77_777)]
    x = np.tile(np.arange(256, dtype=np.uint8), 300)
    np.random.default_rng(2).shuffle(x)
    cases.append(x)
    for d in cases:
        img = _roundtrip(gpu, orc, d)
        with gpu.Decoder(0) as dec:
            dec.load(gpu.parse(img))
            dec.decode()
            rep = dec.report()
        assert gpu.PATH_NAMES[rep.path] == ("grouped" if mode == "tile" else "multi_wave")
    if mode == "wsplit":
        counts = [max(1, int(2 ** (15 - 0.35 * i))) for i in range(40)]
        g = np.repeat(np.arange(40, dtype=np.uint8) + 60, counts)
        np.random.default_rng(4).shuffle(g)
        img = _roundtrip(gpu, orc, g)
        s = gpu.parse(img)
        assert max(l for _, l in s.symbols) > 12


def test_tile_mode_refuses_other_codes(gpu, monkeypatch):
    """GH_MODE=tile on a code the tile kernel does not take fails loudly at load."""
    monkeypatch.setenv("GH_MODE", "tile")
    s = gpu.parse(gpu.encode(gpu.generate(23, 0.9, 100_000)))
    with gpu.Decoder(0) as d:
        with pytest.raises(gpu.GapHuffError):
            d.load(s)


@pytest.mark.gpu
def test_bench_contract_small(gpu):
    """bench.py prints one JSON line with the contract keys (small size, no CPU leg)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--steps", "3", "--warmup", "1",
                        "--size", "3000000", "--cpu-sample", "0"], capture_output=True, text=True,
                       timeout=300, cwd=root)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1
    j = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config", "roofline"):
        assert k in j
    assert j["bitexact"] is True and j["value"] > 0
    assert 0 < j["roofline"]["frac"] < 1
    sub = j["sub"]  # configs[4]'s r=0.5 stream, timed in the same run
    assert sub["workload"] == "cfg5" and sub["redundancy"] == 0.5 and sub["bitexact"] is True
    assert sub["value"] > 0 and 0 < sub["roofline_frac"] < 1


@pytest.mark.gpu
def test_graft_smoke(gpu):
    import __graft_entry__
    __graft_entry__.smoke()


@pytest.mark.parametrize("k", ["", "8", "10", "11", "12"])
@pytest.mark.parametrize("stage", ["", "1"])
@pytest.mark.parametrize("grid", ["", "1", "3"])
def test_wave_split_widths_and_staging(gpu, orc, k, stage, grid, monkeypatch):
    """The wave split at every write-LUT width (GH_WS_K; below maxlen the canonical
    fallback takes the longer codewords), with the default staging and
    with the staging forced down to one chain's worst case, so that blocks are staged
    one chain at a time (GH_WS_STAGE), on the default grid and on grids of 1 and 3
    workgroups (GH_WS_GRID: each wave walks many blocks)."""
    monkeypatch.setenv("GH_MODE", "wsplit")
    if grid:
        monkeypatch.setenv("GH_WS_GRID", grid)
    if k:
        monkeypatch.setenv("GH_WS_K", k)
    if stage:
        monkeypatch.setenv("GH_WS_STAGE", stage)
    for seed, r, n in ((31, 0.9, 700_001), (32, 0.5, 400_003), (33, 0.999, 65_549), (34, 0.1, 9_999)):
        data = gpu.generate(seed, r, n)
        img = _roundtrip(gpu, orc, data)
        s = gpu.parse(img)
        with gpu.Decoder(0) as d:
            d.load(s)
            d.decode()
            rep = d.report()
        assert gpu.PATH_NAMES[rep.path] == "multi_wave"
        total = sum(orc.segment_count(img, i) for i in range(s.g)) if n < 100_000 else None
        if total is not None:
            assert rep.symbols == total


@pytest.mark.parametrize("r", [0.5, 0.1])
def test_shard_counts_both_structures(gpu, orc, r):
    """Shards through the default structure (r=0.5: wave split, r=0.1: tile kernel):
    per-shard symbol counts equal the reference segment rule's (decoder.cu:529-569),
    including the stream's last segment (its zero padding, last_segment_end)."""
    data = gpu.generate(35, r, 250_000)
    img = gpu.encode(data)
    s = gpu.parse(img)
    bounds = gpu.plan_shards(s.g, 4)
    off = 0
    for k in range(4):
        with gpu.Decoder(0) as d:
            d.load(s, bounds[k], bounds[k + 1])
            d.decode()
            r_ = d.report()
            expect = sum(orc.segment_count(img, i) for i in range(bounds[k], bounds[k + 1]))
            assert r_.symbols == expect and r_.status == 0
            keep = min(r_.symbols, s.n - off)
            assert np.array_equal(d.download(keep), data[off:off + keep])
            off += r_.symbols


@pytest.mark.parametrize("mode", ["tile"])
def test_grouped_split_and_tile(gpu, orc, mode, monkeypatch):
    """The grouped single-symbol codes (complete, minlen >= 4) through the tile kernel:
    bytes and symbol totals equal the oracle's (reference segment rule,
    decoder.cu:529-569)."""
    monkeypatch.setenv("GH_MODE", mode)
    for seed, n in ((41, 1_000_003), (42, 131_072), (43, 9_999)):
        data = gpu.generate(seed, 0.1, n)
        img = _roundtrip(gpu, orc, data)
        s = gpu.parse(img)
        with gpu.Decoder(0) as d:
            d.load(s)
            d.decode()
            rep = d.report()
        assert gpu.PATH_NAMES[rep.path] == "grouped" and rep.status == 0
        if n < 200_000:
            assert rep.symbols == sum(orc.segment_count(img, i) for i in range(s.g))


@pytest.mark.parametrize("grid", ["", "1", "7"])
def test_wave_split_repeated_and_default(gpu, orc, grid, monkeypatch):
    """The wave-independent split kernels (GH_MODE=wsplit): back-to-back decodes
    (timed and not) give identical bytes and totals, on the default grid and on
    small ones (GH_WS_GRID)."""
    monkeypatch.setenv("GH_MODE", "wsplit")
    if grid:
        monkeypatch.setenv("GH_WS_GRID", grid)
    for seed, r, n in ((51, 0.5, 3_000_001), (52, 0.9, 1_234_567)):
        data = gpu.generate(seed, r, n)
        s = gpu.parse(gpu.encode(data))
        with gpu.Decoder(0) as d:
            d.load(s)
            for i in range(4):
                d.decode(timed=bool(i & 1))
                rep = d.report()
                assert gpu.PATH_NAMES[rep.path] == "multi_wave" and rep.status == 0
                assert rep.symbols >= n
                assert np.array_equal(d.download(n), data)


@pytest.mark.parametrize("kc", ["2", "11", "12", "13", "14"])
def test_wave_split_count_lut_widths(gpu, orc, kc, monkeypatch):
    """The wave split's count LUT at every width it can take (GH_WS_KC, clamped up to
    maxlen): u32 entries b | end mask << 16 hold every complete codeword of the window,
    up to 7 on 2-bit codes at 14 bits.  Per-segment totals must equal the reference
    segment rule's (decoder.cu:529-569) and the bytes the oracle's decode."""
    monkeypatch.setenv("GH_MODE", "wsplit")
    monkeypatch.setenv("GH_WS_KC", kc)
    for seed, r, n in ((61, 0.9, 300_007), (62, 0.5, 200_003), (63, 0.99, 77_777), (64, 0.1, 50_001)):
        data = gpu.generate(seed, r, n)
        img = _roundtrip(gpu, orc, data)
        s = gpu.parse(img)
        with gpu.Decoder(0) as d:
            d.load(s)
            d.decode()
            rep = d.report()
        if max(l for _, l in s.symbols) <= 12:
            assert gpu.PATH_NAMES[rep.path] == "multi_wave"
        if n < 100_000:
            assert rep.symbols == sum(orc.segment_count(img, i) for i in range(s.g))


@pytest.mark.parametrize("mode,r,scap", [("wsplit", 0.5, None), ("wsplit", 0.9, None), ("tile", 0.1, None),
                                         ("tile", 0.1, "4"), ("tile", 0.5, None), ("tile", 0.5, "4")])
def test_output_capacity_below_total(gpu, mode, r, scap, monkeypatch):
    """An output capacity below the stream's total (gh_ctx_load out_cap) writes exactly
    the prefix that fits: caps inside the first chunk, mid-range, at a range edge and
    just below the end, on the default grid and (wave split) on 3 workgroups, whose
    long ranges are staged in many pieces (a piece that crosses the cap must not be
    followed by writes of later pieces).  scap: tile staging for 4 bytes per segment,
    so every tile takes the direct-store path."""
    monkeypatch.setenv("GH_MODE", mode)
    if scap:
        monkeypatch.setenv("GH_TILE_SCAP", scap)
    data = gpu.generate(81, r, 2_000_003)
    s = gpu.parse(gpu.encode(data))
    for grid in (("", "3") if mode == "wsplit" else ("",)):
        if grid:
            monkeypatch.setenv("GH_WS_GRID", grid)
        for cap in (1, 9, 16, 4099, 777_777, 1_999_990):
            with gpu.Decoder(0) as d:
                d.load(s, 0, s.g, out_cap=cap)
                d.decode()
                rep = d.report()
                assert rep.status == 0 and rep.out_bytes == cap
                got = d.download(cap)
                if not np.array_equal(got, data[:cap]):
                    bad = np.nonzero(got != data[:cap])[0]
                    raise AssertionError(f"{mode} grid={grid} cap={cap}: {bad.size} wrong bytes, first at {bad[0]}")


@pytest.mark.parametrize("r,scap", [(0.1, None), (0.1, "17"), (0.1, "4"), (0.5, None), (0.5, "22"), (0.5, "4")])
def test_tile_staging_overflow(gpu, orc, r, scap, monkeypatch):
    """The tile kernel's staging holds the typical tile, not the worst case 128 / minlen
    bytes per segment (20 bytes per segment for r = 0.1 codes, the mean + 12 % for the
    minlen-3 shape); a tile decoding to more bytes waits for its own prefix and stores
    straight from registers.  Data sorted by falling symbol frequency puts the shortest
    codewords first, so its first tiles overflow (25.6 symbols per segment on 5-bit
    codewords, 42.7 on 3-bit ones); smaller staging caps send about half / all of a
    random stream's tiles through the direct path."""
    monkeypatch.setenv("GH_MODE", "tile")
    if scap:
        monkeypatch.setenv("GH_TILE_SCAP", scap)
    d = gpu.generate(31, r, 3_000_001)
    vals, cnts = np.unique(d, return_counts=True)
    rank = np.zeros(256, np.int64)
    rank[vals[np.argsort(-cnts, kind="stable")]] = np.arange(vals.size)
    dense = d[np.argsort(rank[d], kind="stable")]
    for x in (dense, d):
        img = _roundtrip(gpu, orc, x)
        with gpu.Decoder(0) as dec:
            dec.load(gpu.parse(img))
            dec.decode()
            rep = dec.report()
        assert gpu.MODE_NAMES[rep.mode] == "tile" and rep.status == 0


@pytest.mark.parametrize("mode,r", [("tile", 0.1), ("tile", 0.5), ("wsplit", 0.5)])
def test_decode_beside_a_foreign_kernel(gpu, mode, r, monkeypatch):
    """A persistent decode grid sized to the whole GPU, launched while another stream's
    kernel (a 1 GiB streaming copy, 131 K workgroups, repeated) holds the CUs: its
    workgroups become resident only as the copy's retire, and the ones already running
    wait for them (a delay bounded by wall time, not a spin count).  The bytes must be
    exact and the status clean (reference: the atomic ticket of decoder.cu:494-499
    exists for the same reason)."""
    import threading

    import torch

    monkeypatch.setenv("GH_MODE", mode)
    data = gpu.generate(91, r, 100_000_007)
    s = gpu.parse(gpu.encode(data))
    src = torch.full((1 << 30,), 7, dtype=torch.uint8, device="cuda")
    dst = torch.empty_like(src)
    cs = torch.cuda.Stream()
    torch.cuda.synchronize()
    with gpu.Decoder(0) as d:
        d.load(s)
        err = []

        def copy():
            try:
                gpu.bw_copy(dst.data_ptr(), src.data_ptr(), src.numel(), cs.cuda_stream, reps=20)
            except Exception as e:  # reported below
                err.append(e)

        th = threading.Thread(target=copy)
        th.start()
        for _ in range(3):
            d.decode()
        rep = d.report()
        th.join()
        assert not err
        assert rep.status == 0
        assert np.array_equal(d.download(data.size), data)
    assert bool((dst[:4096] == 7).all())
