"""Generate string-format golden fixtures: for a few golden inputs, <name>.seq is the
output of the REFERENCE sequential.cpp encoder (HuffmanSequential::encode,
sequential.cpp:17-51), compiled from its own source with our driver
oracle/ref_drivers/seq_driver.cpp into oracle/_ref/seq_driver.  seq.json records
sha256s.  Data only; no reference source is kept."""
import hashlib
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402

CASES = ["gen_r0.5_n20000", "gen_r0.9_n20000", "gen_r0.1_n20000", "two_symbols", "geometric_long_codes"]


def main():
    exe = os.path.join(oracle.REF, "seq_driver")
    out = {}
    for name in CASES:
        p = os.path.join(HERE, name + ".seq")
        subprocess.run([exe, "enc", os.path.join(HERE, name + ".bin"), p], check=True)
        out[name] = hashlib.sha256(open(p, "rb").read()).hexdigest()
    with open(os.path.join(HERE, "seq.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
