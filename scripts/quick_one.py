import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'cse375-finalproj-huffman-decoding_amd'))
import numpy as np, gaphuff as gh
name, n, r = sys.argv[1].split(":"); n = int(n); r = float(r)
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
data = gh.generate(375, r, n); img = gh.encode(data); s = gh.parse(img)
d = gh.Decoder(0); d.load(s)
for _ in range(reps): d.decode()
rep = d.report()
print(name, "kernel_ms", rep.kernel_ms, "ok", np.array_equal(d.download(s.n), data), "alg_bytes", 4*s.w + 4*((s.g+7)//8) + s.n)
