# Shards on one device, loaded and saved from host threads (gh_ctx_load_file /
# gh_ctx_save_file, pinned double-buffered staging) versus one after another, and the
# one-shot gh_decode with 1 and 8 shards.  One JSON line per measurement.
# Usage: python scripts/bench_shards.py [--n 160000000,1000000000] [--shards 8]
import argparse, json, os, subprocess, sys, tempfile, threading, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "cse375-finalproj-huffman-decoding_amd"))
import numpy as np, gaphuff as gh

ap = argparse.ArgumentParser()
ap.add_argument("--n", default="160000000,1000000000")
ap.add_argument("--shards", type=int, default=8)
ap.add_argument("--dir", default=os.environ.get("TMPDIR", "/tmp"))
a = ap.parse_args()
root = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")


def loads(path, b, conc):
    decs = [gh.Decoder(0) for _ in range(len(b) - 1)]
    t0 = time.perf_counter()
    if conc:
        th = [threading.Thread(target=decs[k].load_file, args=(path, b[k], b[k + 1])) for k in range(len(decs))]
        [t.start() for t in th]
        [t.join() for t in th]
    else:
        for k, d in enumerate(decs):
            d.load_file(path, b[k], b[k + 1])
    ms = (time.perf_counter() - t0) * 1e3
    for d in decs:
        d.decode()
    offs = np.concatenate([[0], np.cumsum([int(d.report().out_bytes) for d in decs])])
    out = os.path.join(a.dir, "gh_shards.out")
    open(out, "wb").close()
    t0 = time.perf_counter()
    if conc:
        th = [threading.Thread(target=decs[k].save_file, args=(out, int(offs[k + 1] - offs[k]), int(offs[k]), 0, False))
              for k in range(len(decs))]
        [t.start() for t in th]
        [t.join() for t in th]
    else:
        for k, d in enumerate(decs):
            d.save_file(out, int(offs[k + 1] - offs[k]), int(offs[k]), 0, False)
    sms = (time.perf_counter() - t0) * 1e3
    for d in decs:
        d.close()
    return ms, sms, out


for n in [int(x) for x in a.n.split(",")]:
    data = gh.generate(375, 0.1, n)
    img = gh.encode(data)
    path = os.path.join(a.dir, "gh_shards.huff")
    img.tofile(path)
    g = gh.parse(img).g
    b = gh.plan_shards(g, a.shards)
    loads(path, b, True)  # pins the staging sets, warms the page cache
    for conc in (True, False, True, False):
        ms, sms, out = loads(path, b, conc)
        ok = bool(np.array_equal(np.fromfile(out, dtype=np.uint8)[:n], data))
        print(json.dumps({"what": "load_file/save_file x shards, device 0", "n": n, "compressed": int(img.size),
                          "shards": a.shards, "threads": conc, "load_ms": round(ms, 2), "save_ms": round(sms, 2),
                          "bitexact": ok}), flush=True)
    for ng in (1, a.shards):
        t0 = time.perf_counter()
        out = gh.decode(img, ngpus=ng, devices=[0] * ng)
        print(json.dumps({"what": "gh_decode (host in, host out)", "n": n, "shards": ng,
                          "wall_ms": round((time.perf_counter() - t0) * 1e3, 2),
                          "bitexact": bool(np.array_equal(out, data))}), flush=True)
    for sh in (1, a.shards):
        r = subprocess.run([os.path.join(root, "bin", "decoder"), path, os.path.join(a.dir, "gh_cli.out"), "--gpus", "1",
                            "--shards", str(sh), "--json"], capture_output=True, text=True, timeout=300)
        j = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]) if r.returncode == 0 else {}
        print(json.dumps({"what": "bin/decoder --gpus 1 (cold process)", "n": n, "shards": sh, "rc": r.returncode,
                          "load_ms": j.get("load_ms"), "save_ms": j.get("save_ms")}), flush=True)
    for f in (path, os.path.join(a.dir, "gh_shards.out"), os.path.join(a.dir, "gh_cli.out")):
        try:
            os.unlink(f)
        except OSError:
            pass
    del data, img
