"""Generates the restatement-derived golden fixtures in tests/golden/.

The reference ships no golden vectors and its arithmetic libraries are not
available, so these fixtures come from the CPU oracle
(oracle/leoec_oracle.c) after it passed the KAT / cross-restatement pins of
tests/test_oracle.py.  They are a regression pin for both the oracle and the
GPU engine.  Data: numpy PCG64 with the listed seed.

    python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import oracle as O  # noqa: E402

CASES = [
    ("vandrs", 10, 4, 8, 4096 + 3), ("vandrs", 4, 2, 8, 65536), ("vandrs", 8, 3, 16, 10007),
    ("vandrs", 6, 3, 32, 12345), ("isars", 10, 4, 8, 20000), ("isars", 4, 2, 8, 1000),
    ("cauchyrs", 10, 4, 8, 30000), ("cauchyrs", 4, 2, 3, 777), ("cauchyrs", 6, 3, 4, 5000),
    ("liberation", 4, 2, 7, 9000), ("liberation", 10, 2, 11, 25000),
]


def main():
    index = []
    for cls, k, m, w, size in CASES:
        seed = 0x1E0E + size
        data = np.random.Generator(np.random.PCG64(seed)).integers(0, 256, size, dtype=np.uint8)
        blocks = O.encode(cls, k, m, w, data.tobytes())
        name = f"{cls}_{k}_{m}_{w}_{size}.npz"
        np.savez_compressed(os.path.join(HERE, name), data=data,
                            blocks=np.frombuffer(b"".join(blocks), dtype=np.uint8))
        index.append({"file": name, "class": cls, "k": k, "m": m, "w": w, "size": size,
                      "seed": seed, "block_size": len(blocks[0])})
    with open(os.path.join(HERE, "index.json"), "w") as fh:
        json.dump(index, fh, indent=1)


if __name__ == "__main__":
    main()
