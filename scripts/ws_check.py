# Diagnostic: decode a stream as one context through a bounds-checked build of the wave
# split kernels (GAPHUFF_LIB=..._wscheck.so, GH_MODE=wsplit) and print the status bits.
import os, sys, numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "cse375-finalproj-huffman-decoding_amd"))
import gaphuff as gh
n = int(sys.argv[1]); r = float(sys.argv[2])
img = gh.encode(gh.generate(375, r, n, threads=16), threads=16)
s = gh.parse(img)
print("N", s.n, "G", s.g, "v", s.version, flush=True)
with gh.Decoder(0) as d:
    d.load(s)
    d.decode()
    rep = d.report()
    print("status 0x%x symbols %d out %d path %s grid %d" % (rep.status, rep.symbols, rep.out_bytes, gh.PATH_NAMES[rep.path], rep.grid), flush=True)
    ok = True
    for off in range(0, s.n, 10**9):
        got = d.download(min(10**9, s.n - off), offset=off)
        want = gh.generate(375, r, got.size, offset=off, threads=16)
        if not np.array_equal(got, want):
            bad = np.nonzero(got != want)[0]
            print("mismatch in slice", off, "first", off + bad[0], "count", bad.size, flush=True)
            ok = False
    print("bitexact", ok, flush=True)
