# Shader clock per launch over bursts (GH_TILE_STAMPS build: the leader workgroup stamps
# s_memtime and s_memrealtime at its start and end of every launch).  Bursts of 3, 20, 100
# and 400 decodes after idle; prints the launch time and clock by window.
# Usage: python scripts/clock_burst.py name:N:r [lib-suffix]
import os, sys, time, tempfile
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "cse375-finalproj-huffman-decoding_amd"))
suffix = sys.argv[2] if len(sys.argv) > 2 else "st"
os.environ["GAPHUFF_LIB"] = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                         "cse375-finalproj-huffman-decoding_amd", "lib", f"libgaphuff_{suffix}.so")
out = os.path.join(tempfile.gettempdir(), f"gh_clock_{os.getpid()}.bin")
os.environ["GH_STAMPS_OUT"] = out
import numpy as np, gaphuff as gh
name, n, r = sys.argv[1].split(":"); n = int(n); r = float(r)
data = gh.generate(375, r, n); img = gh.encode(data); s = gh.parse(img)
d = gh.Decoder(0); d.load(s)
for _ in range(3): d.decode(timed=False)
rep = d.report()
grid = rep.grid; ntiles = rep.tiles
for reps in (3, 20, 100, 400):
    time.sleep(0.5)
    for _ in range(reps): d.decode()
    d.report()  # dumps the stamps of the last decode, including the launch ring
    raw = np.fromfile(out, dtype=np.uint8)
    t = raw[32 * grid * 2 * 128:].view(np.uint64)
    ring = t[3 * ntiles + 64:3 * ntiles + 64 + 4 * 1024].reshape(1024, 4).astype(np.float64)
    ok = ring[:, 3] > ring[:, 1]
    # the last `reps` launches in epoch order: the ring is indexed by epoch & 1023
    order = np.argsort(ring[:, 1])
    sel = [i for i in order if ok[i]][-reps:]
    dur = (ring[sel, 3] - ring[sel, 1]) * 0.01  # us
    clk = (ring[sel, 2] - ring[sel, 0]) / (ring[sel, 3] - ring[sel, 1]) / 10.0  # GHz (memtime ticks / 10 ns)
    w = max(1, len(sel) // 8)
    print(f"burst {reps:4d}: leader span us " + " ".join(f"{dur[k:k + w].mean():.0f}" for k in range(0, len(sel), w)) +
          " | GHz " + " ".join(f"{clk[k:k + w].mean():.2f}" for k in range(0, len(sel), w)), flush=True)
os.unlink(out)
