"""GPU parity tests of the two-pass tile kernel (gh_mtile.hip, GH_MODE=mtile): complete
codes of 1..16-bit codewords (those above the 11- or 12-bit tables through a canonical fallback; BASELINE's
r = 0.9 codes, and the r = 0.5 / 0.1 codes too when forced) decoded by one persistent kernel that reads the payload once: a count pass
and, one tile later, a write pass over the same register-resident words.  Bit-exact
against the CPU oracle and the original input (reference: decoder/src/decoder.cu:454-730,
restated in oracle/gh_oracle.c)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _check(gpu, orc, data, **kw):
    img = gpu.encode(data)
    out = gpu.decode(img, **kw)
    ref, _ = orc.decode(img)
    assert np.array_equal(ref, np.asarray(data, dtype=np.uint8))
    if not np.array_equal(out, ref):
        bad = np.nonzero(out != ref)[0]
        raise AssertionError(f"{bad.size} mismatches, first at {bad[0]} of {out.size}")
    return img


def _report(gpu, img):
    with gpu.Decoder(0) as d:
        d.load(gpu.parse(img))
        d.decode()
        return d.report()


@pytest.fixture
def mtile(monkeypatch):
    monkeypatch.setenv("GH_MODE", "mtile")


def _complete(syms):
    return sum(2.0 ** -l for _, l in syms) == 1.0


def _takes(syms):  # the kernel's codes: complete, codewords of 1..16 bits (longer than the tables: fallback)
    return _complete(syms) and max(l for _, l in syms) <= 16


@pytest.mark.parametrize("r", [0.1, 0.5, 0.9, 0.999])
@pytest.mark.parametrize("n", [1, 2, 7, 100, 4097, 65549, 1_000_003, 5_000_011])
def test_mtile_vs_oracle(gpu, orc, mtile, r, n):
    """Complete codes decode bit-exact; an incomplete one (e.g. the one-symbol code of a
    tiny input) or one with codewords longer than the tables is refused at load (the
    wave split's canonical fallback takes those)."""
    data = gpu.generate(2000 + n, r, n)
    img = gpu.encode(data)
    if not _takes(gpu.parse(img).symbols):
        with pytest.raises(gpu.GapHuffError):
            gpu.decode(img)
        return
    _check(gpu, orc, data)
    rep = _report(gpu, img)
    assert gpu.MODE_NAMES[rep.mode] == "mtile" and rep.status == 0


def test_mtile_small_codes(gpu, orc, mtile):
    # two-bit codes (four symbols: 64 codewords per segment), 8-bit codes, a
    # segment-multiple stream, one-bit codes (128 codewords per segment, the most) and a
    # code whose 1-bit codeword takes 97 % of the stream
    rng = np.random.default_rng(3)
    four = (rng.integers(0, 4, 300_001) + 48).astype(np.uint8)
    assert {l for _, l in gpu.parse(gpu.encode(four)).symbols} == {2}
    _check(gpu, orc, four)
    data = np.tile(np.arange(256, dtype=np.uint8), 64)
    rng.shuffle(data)
    _check(gpu, orc, data)
    for n in (3001, 1_000_003):
        two = (rng.integers(0, 2, n) + 48).astype(np.uint8)
        img = _check(gpu, orc, two)
        assert {l for _, l in gpu.parse(img).symbols} == {1}
        assert gpu.MODE_NAMES[_report(gpu, img).mode] == "mtile"
    skew = np.where(rng.random(2_000_003) < 0.97, 7, rng.integers(0, 256, 2_000_003)).astype(np.uint8)
    img = _check(gpu, orc, skew)
    assert min(l for _, l in gpu.parse(img).symbols) == 1


@pytest.mark.parametrize("q,n", [(0.7, 300_001), (0.7, 3_000_017), (0.75, 1_000_003), (0.5, 300_001),
                                 (0.5, 3_000_017), (0.6, 1_000_003)])
def test_mtile_long_codes_fallback(gpu, orc, monkeypatch, q, n):
    """Codes of 1..16-bit codewords (geometric byte distributions): the codewords longer
    than the tables (12 bits; 11 for codes with a 1-bit codeword) go through the canonical
    fallback inside the kernel; the launcher picks the two-pass kernel for them by default."""
    rng = np.random.default_rng(int(q * 100) + n)
    p = q ** np.arange(256, dtype=np.float64)
    p /= p.sum()
    data = rng.choice(256, size=n, p=p).astype(np.uint8)
    img = gpu.encode(data)
    lens = [l for _, l in gpu.parse(img).symbols]
    assert min(lens) == (1 if q <= 0.6 else 2) and max(lens) > 12
    _check(gpu, orc, data)
    rep = _report(gpu, img)
    assert gpu.MODE_NAMES[rep.mode] == "mtile" and rep.status == 0


@pytest.mark.parametrize("nsym,ratio,maxlen", [(40, 0.9, 16), (13, 1.0, 12), (12, 1.0, 11)])
def test_mtile_one_to_sixteen_bits(gpu, orc, mtile, nsym, ratio, maxlen):
    """Codes of 1..16-bit, 1..12-bit (one length past the 11-bit tables: the fallback)
    and 1..11-bit codewords, sorted runs: segments of 128 one-bit codewords first (their
    pieces go chain by chain), then long ones; and the same data shuffled."""
    counts = [max(1, int(2 ** (24 - ratio * i))) for i in range(nsym)]
    data = np.repeat(np.arange(nsym, dtype=np.uint8), counts)
    img = _check(gpu, orc, data)
    s = gpu.parse(img)
    assert min(l for _, l in s.symbols) == 1 and max(l for _, l in s.symbols) == maxlen
    _check(gpu, orc, np.random.default_rng(nsym).permutation(data))
    assert gpu.MODE_NAMES[_report(gpu, img).mode] == "mtile"


def test_mtile_refuses_incomplete_codes(gpu, mtile):
    """An incomplete code (a one-symbol input's) stays with the wave split: GH_MODE=mtile
    fails loudly at load."""
    s = gpu.parse(gpu.encode(np.full(1000, 5, np.uint8)))
    assert not _complete(s.symbols)
    with gpu.Decoder(0) as d:
        with pytest.raises(gpu.GapHuffError):
            d.load(s)


@pytest.mark.parametrize("r,scap", [(0.9, None), (0.9, "40"), (0.9, "4"), (0.5, None), (0.5, "4")])
def test_mtile_staging_overflow(gpu, orc, mtile, r, scap, monkeypatch):
    """A wave's staging region holds its mean piece + 12 % (and at least one chain's worst
    case); a larger piece is written and copied out chain by chain.  Data sorted by
    falling frequency puts the shortest codewords first (its first tiles overflow);
    smaller staging caps send about half / all of a random stream's pieces that way."""
    if scap:
        monkeypatch.setenv("GH_TILE_SCAP", scap)
    d = gpu.generate(31, r, 3_000_001)
    vals, cnts = np.unique(d, return_counts=True)
    rank = np.zeros(256, np.int64)
    rank[vals[np.argsort(-cnts, kind="stable")]] = np.arange(vals.size)
    dense = d[np.argsort(rank[d], kind="stable")]
    for x in (dense, d):
        img = _check(gpu, orc, x)
        rep = _report(gpu, img)
        assert gpu.MODE_NAMES[rep.mode] == "mtile" and rep.status == 0


def _geometric(q, n, seed):
    rng = np.random.default_rng(seed)
    p = q ** np.arange(256, dtype=np.float64)
    p /= p.sum()
    return rng.choice(256, size=n, p=p).astype(np.uint8)


@pytest.mark.parametrize("scap", [None, "66", "40", "4"])
def test_mtile_one_bit_staging(gpu, orc, mtile, scap, monkeypatch):
    """Codes with a 1-bit codeword (q = 0.5: 64 codewords per segment on average, 128 at
    most): 8.5 KB regions hold the mean piece of 8 KB, a chain's worst case (8 KB) is
    copied out in two parts; sorted data and smaller caps take the chain-by-chain path."""
    if scap:
        monkeypatch.setenv("GH_TILE_SCAP", scap)
    d = _geometric(0.5, 2_000_003, 41)
    dense = np.sort(d)  # symbol 0 (the 1-bit codeword) first
    for x in (dense, d):
        img = _check(gpu, orc, x)
        assert min(l for _, l in gpu.parse(img).symbols) == 1
        rep = _report(gpu, img)
        assert gpu.MODE_NAMES[rep.mode] == "mtile" and rep.status == 0


def test_mtile_one_bit_capacity_and_shards(gpu, orc, mtile):
    data = _geometric(0.5, 1_500_007, 43)
    s = gpu.parse(gpu.encode(data))
    for cap in (1, 15, 8193, 777_777, 1_500_000):
        with gpu.Decoder(0) as d:
            d.load(s, 0, s.g, out_cap=cap)
            d.decode()
            rep = d.report()
            assert rep.status == 0 and rep.out_bytes == cap
            assert np.array_equal(d.download(cap), data[:cap])
    _check(gpu, orc, data, ngpus=3, devices=[0] * 3)


@pytest.mark.parametrize("r,scap", [(0.9, None), (0.9, "4"), (0.5, None)])
def test_mtile_output_capacity_below_total(gpu, mtile, r, scap, monkeypatch):
    if scap:
        monkeypatch.setenv("GH_TILE_SCAP", scap)
    data = gpu.generate(81, r, 2_000_003)
    s = gpu.parse(gpu.encode(data))
    for cap in (1, 9, 16, 4099, 777_777, 1_999_990):
        with gpu.Decoder(0) as d:
            d.load(s, 0, s.g, out_cap=cap)
            d.decode()
            rep = d.report()
            assert rep.status == 0 and rep.out_bytes == cap
            got = d.download(cap)
            if not np.array_equal(got, data[:cap]):
                bad = np.nonzero(got != data[:cap])[0]
                raise AssertionError(f"cap={cap}: {bad.size} wrong bytes, first at {bad[0]}")


@pytest.mark.parametrize("nshards", [2, 3, 8])
def test_mtile_shards(gpu, orc, mtile, nshards):
    _check(gpu, orc, gpu.generate(11, 0.9, 2_000_000), ngpus=nshards, devices=[0] * nshards)


def test_mtile_shard_counts(gpu, orc, mtile):
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
            assert r.symbols == sum(orc.segment_count(img, i) for i in range(bounds[k], bounds[k + 1]))
            keep = min(r.symbols, s.n - off)
            assert np.array_equal(d.download(keep), data[off:off + keep])
            off += r.symbols


def test_mtile_repeated_decodes(gpu, mtile):
    data = gpu.generate(13, 0.9, 3_000_000)
    s = gpu.parse(gpu.encode(data))
    with gpu.Decoder(0) as d:
        d.load(s)
        for _ in range(5):
            d.decode()
        r = d.report()
        assert r.launches == 5 and r.status == 0 and r.symbols >= s.n
        assert np.array_equal(d.download(s.n), data)


def test_mtile_corrupted_stream_terminates(gpu, mtile):
    data = gpu.generate(15, 0.9, 500_000)
    img = gpu.encode(data).copy()
    rng = np.random.default_rng(1)
    hdr = 8 + 2 * len(gpu.parse(img).symbols) + 12
    for pos in rng.integers(hdr, img.size, 200):
        img[pos] ^= 0xFF
    try:
        out = gpu.decode(img)
        assert out.size == data.size
    except gpu.GapHuffError as e:
        assert e.code in (-7, -2)


@pytest.mark.parametrize("r", [0.9, 0.5])
def test_mtile_100MB(gpu, mtile, r):
    data = gpu.generate(375, r, 10**8)
    assert np.array_equal(gpu.decode(gpu.encode(data)), data)


def test_mtile_100MB_one_bit(gpu, mtile):
    data = _geometric(0.5, 10**8, 377)
    assert np.array_equal(gpu.decode(gpu.encode(data)), data)
