"""Generate the raw-stream (self-synchronising decoder) golden fixtures.

Run in the build container, where oracle/Makefile has compiled the REFERENCE raw
encoder (gpuhd/encoder/src/llhuffman_encoder.cc + gpuhd/src/cuhd_codetable.cc) with
our driver oracle/ref_drivers/llhuff_driver.cpp into oracle/_ref/llhuff_driver.

For every input <name>.bin of golden.json it writes <name>.llh, the driver's output
(u32 nsyms, {u8 symbol, u8 length} in code order, u64 units, u32 units: the
reference's get_symbol_lengths / get_encoder_table / encode_memory, demo.cc:100-116),
and llhuff.json with sha256 of each .llh.  Data only; no reference source is kept.
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402


def main():
    meta = json.load(open(os.path.join(HERE, "golden.json")))
    out = {}
    for name in sorted(meta):
        data = np.fromfile(os.path.join(HERE, name + ".bin"), dtype=np.uint8)
        if data.size == 0:
            continue
        exe = os.path.join(oracle.REF, "llhuff_driver")
        path = os.path.join(HERE, name + ".llh")
        import subprocess
        subprocess.run([exe, os.path.join(HERE, name + ".bin"), path], check=True)
        b = open(path, "rb").read()
        syms, units = oracle.read_llh(b)
        out[name] = {"n": int(data.size), "units": int(units.size), "nsyms": len(syms),
                     "maxlen": max(l for _, l in syms), "sha256": hashlib.sha256(b).hexdigest()}
    with open(os.path.join(HERE, "llhuff.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
