#!/usr/bin/env python3
"""Synthetic Criteo-shaped libffm shard for input-path measurements:
`label\\tfield:feature:1 ...` lines, 39 fields, power-law feature ids.

    python tools/gen_libffm.py OUT_PREFIX ROWS [--seed S]   (writes OUT_PREFIX-00000)
"""
import argparse

import numpy as np


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prefix")
    ap.add_argument("rows", type=int)
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args()
    rng = np.random.default_rng(a.seed)
    fields = 39
    with open(a.prefix + "-00000", "w") as f:
        for r0 in range(0, a.rows, 10000):
            n = min(10000, a.rows - r0)
            ids = np.minimum(rng.zipf(1.2, size=(n, fields)), 10 ** 6)
            lab = (rng.random(n) < 0.25).astype(int)
            for i in range(n):
                f.write("%d\t%s\n" % (lab[i], " ".join(
                    "%d:%d:1" % (j, ids[i, j] * 64 + j) for j in range(fields))))


if __name__ == "__main__":
    main()
