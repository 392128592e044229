"""Generate the committed golden fixtures (run in the build container, where the
reference sources are present and compiled into oracle/_ref/ by oracle/Makefile).

For every case it writes, under tests/golden/:
  <name>.bin    input bytes (seeded product generator, or a crafted pattern)
  <name>.huff   compressed.huff produced by the CPU oracle (oracle/gh_oracle.c)
  golden.json   per case: N, W, G, sha256 of input and stream, the file-order
                (symbol, length) list produced by the REFERENCE boundary_PM
                (_ref/pm_driver: encoder/src/package_merge.cpp + symbols.cpp compiled
                from the reference's own sources), and the verdict of the REFERENCE
                sequential.cpp (_ref/sequential) on the same input.

Fixtures are data only (inputs and expected outputs); no reference source is kept.
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


def cases():
    out = []
    for r in (0.0, 0.1, 0.5, 0.9, 0.999, 1.0):
        out.append((f"gen_r{r}_n20000", oracle.generate(375, r, 20000)))
    out.append(("gen_r0.5_n7", oracle.generate(1, 0.5, 7)))
    out.append(("gen_r0.9_n1", oracle.generate(2, 0.9, 1)))
    out.append(("single_symbol", np.full(1000, 65, dtype=np.uint8)))
    out.append(("two_symbols", (np.random.default_rng(3).integers(0, 2, 5000) + 48).astype(np.uint8)))
    # 256 equal counts: 8-bit codes, bits a multiple of 128
    x = np.tile(np.arange(256, dtype=np.uint8), 16)
    np.random.default_rng(9).shuffle(x)
    out.append(("uniform256_exact_segments", x))
    # geometric counts: length-limited codes up to 16 bits, gap nibbles up to 15
    counts = [max(1, int(2 ** (17 - 0.9 * i))) for i in range(30)]
    g = np.repeat(np.arange(30, dtype=np.uint8), counts)
    np.random.default_rng(5).shuffle(g)
    out.append(("geometric_long_codes", g))
    return out


def main():
    meta = {}
    for name, data in cases():
        data = np.ascontiguousarray(data, dtype=np.uint8)
        img = oracle.encode(data)
        dec, _ = oracle.decode(img)
        assert np.array_equal(dec, data), name
        data.tofile(os.path.join(HERE, name + ".bin"))
        img.tofile(os.path.join(HERE, name + ".huff"))
        counts = np.bincount(data, minlength=256).astype(np.uint32)
        syms = oracle.symbols_of(data)
        ref_syms = oracle.ref_package_merge(counts) if (counts > 0).sum() >= 2 else None
        seq = oracle.run_reference_cpu("sequential", data) if data.size else None
        hdr = np.frombuffer(img[8 + 2 * len(syms):8 + 2 * len(syms) + 12].tobytes(), dtype="<u4")
        meta[name] = {
            "n": int(data.size), "w": int(hdr[1]), "g": int(hdr[2]),
            "sha256_input": hashlib.sha256(data.tobytes()).hexdigest(),
            "sha256_stream": hashlib.sha256(img.tobytes()).hexdigest(),
            "symbols_reference_boundary_pm": ref_syms,
            "symbols": [list(s) for s in syms],
            "reference_sequential_verified": None if seq is None else seq["verified"],
            "maxlen": max(l for _, l in syms),
        }
        print(name, meta[name]["n"], meta[name]["maxlen"], "ref PM match:",
              ref_syms is None or [tuple(s) for s in ref_syms] == [tuple(s) for s in syms])
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
