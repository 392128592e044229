# Compare environment variants (decode-structure overrides) on the same inputs: each
# variant runs scripts/quick_one.py in its own process.
# Usage: python scripts/cmp_env.py "cfg3:1000000000:0.9,..." "" "GH_MODE=msplit" "GH_MODE=wsplit GH_WS_BPR=4"
import os, subprocess, sys
here = os.path.dirname(os.path.abspath(__file__))
for wl in sys.argv[1].split(","):
    for spec in sys.argv[2:] or [""]:
        env = dict(os.environ)
        for kv in spec.split():
            k, v = kv.split("=", 1)
            env[k] = v
        r = subprocess.run([sys.executable, os.path.join(here, "quick_one.py"), wl, "20"], env=env,
                           capture_output=True, text=True, timeout=300)
        print(f"[{spec or 'default':28s}] {r.stdout.strip()} {r.stderr.strip()[-400:] if r.returncode else ''}",
              flush=True)
