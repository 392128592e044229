# Compare build variants of libgaphuff on the same inputs: for each workload, decode
# with each lib (own process, GAPHUFF_LIB) and print kernel time and bit-exactness.
# Usage: python scripts/cmp_libs.py "cfg4:1000000000:0.1,cfg3:1000000000:0.9" lib1 lib2 ...
# (a lib may carry environment settings: name@VAR=value@VAR2=value)
import os, subprocess, sys
here = os.path.dirname(os.path.abspath(__file__))
libdir = os.path.join(here, "..", "cse375-finalproj-huffman-decoding_amd", "lib")
for wl in sys.argv[1].split(","):
    for spec in sys.argv[2:]:
        name, *envs = spec.split("@")
        lib = os.path.join(libdir, f"libgaphuff{'' if name == 'base' else '_' + name}.so")
        env = dict(os.environ, GAPHUFF_LIB=lib, **dict(e.split("=", 1) for e in envs))
        try:
            r = subprocess.run([sys.executable, os.path.join(here, "quick_one.py"), wl, os.environ.get("CMP_REPS", "20")], env=env,
                           capture_output=True, text=True, timeout=90)
        except subprocess.TimeoutExpired:
            print(f"{spec:10s} TIMEOUT (90 s)", flush=True)
            break
        print(f"{spec:10s} {r.stdout.strip()} {r.stderr.strip()[-300:] if r.returncode else ''}", flush=True)
