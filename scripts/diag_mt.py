# Diagnostic: two-pass kernel on geometric streams; status, mismatch count and position.
# Usage: python scripts/diag_mt.py Q N [ENV=VAL ...]
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "cse375-finalproj-huffman-decoding_amd"))
q, n = float(sys.argv[1]), int(sys.argv[2])
for kv in sys.argv[3:]:
    k, v = kv.split("=", 1)
    os.environ[k] = v
import numpy as np, gaphuff as gh
rng = np.random.default_rng(7)
p = q ** np.arange(256, dtype=np.float64)
p /= p.sum()
data = rng.choice(256, size=n, p=p).astype(np.uint8)
img = gh.encode(data, threads=16)
s = gh.parse(img)
for timed in (False, True, True):
    d = gh.Decoder(0); d.load(s)
    d.decode(timed=timed)
    rep = d.report()
    out = d.download(s.n)
    bad = np.nonzero(out != data)[0]
    print(f"q={q} n={n} {sys.argv[3:]} timed={timed} mode={gh.MODE_NAMES.get(rep.mode)} status={rep.status} "
          f"symbols={rep.symbols} bad={bad.size} first={bad[:4].tolist()} ms={rep.kernel_ms:.4f}", flush=True)
    if bad.size:
        i = bad[0]
        print("  got", out[i - 4:i + 12].tolist(), "\n  exp", data[i - 4:i + 12].tolist(), flush=True)
    d.close()
