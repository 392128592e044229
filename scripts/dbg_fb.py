# Diagnostic: wave split with the canonical fallback on minlen-1 / minlen-2 long codes:
# total symbols vs the oracle's segment rule, first wrong byte, per-segment count diffs.
import os, sys
here = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(here, "..", "cse375-finalproj-huffman-decoding_amd")); sys.path.insert(0, os.path.join(here, "..", "oracle"))
import numpy as np, gaphuff as gh, oracle
rng = np.random.default_rng(7)
for q in (0.5, 0.7):
    p = q ** np.arange(256, dtype=np.float64); p /= p.sum()
    data = rng.choice(256, size=30000, p=p).astype(np.uint8)
    img = gh.encode(data); s = gh.parse(img)
    lens = [l for _, l in s.symbols]
    counts = np.array([oracle.segment_count(img, i) for i in range(s.g)])
    for env in ("", "GH_WS_KC=16", "GH_WS_K=12"):
        for kv in env.split():
            k, v = kv.split("="); os.environ[k] = v
        with gh.Decoder(0) as d:
            d.load(s); d.decode(); rep = d.report()
            out = d.download(s.n)
        for kv in env.split():
            del os.environ[kv.split("=")[0]]
        bad = np.nonzero(out != data)[0]
        print(f"q={q} minlen={min(lens)} maxlen={max(lens)} env=[{env}] K={rep.lut_bits} symbols={rep.symbols} "
              f"oracle={counts.sum()} status={rep.status} wrong={bad.size} first={bad[0] if bad.size else -1}", flush=True)
        if bad.size:
            cum = np.concatenate([[0], np.cumsum(counts)])
            seg = int(np.searchsorted(cum, bad[0], side="right") - 1)
            print(f"   first wrong byte in segment {seg} (offset {cum[seg]}..{cum[seg+1]}), counts around: {counts[max(0,seg-2):seg+3]}")
            print(f"   got {out[bad[0]-4:bad[0]+8]} want {data[bad[0]-4:bad[0]+8]}")
