#!/usr/bin/env python3
"""Per-kernel averages of rocprofv3 --pmc counters (counter_collection.csv).

    python tools/pmc_summary.py gpurun_out/pmc_x/ [...more dirs]
"""
from __future__ import annotations

import collections
import csv
import glob
import os
import sys


def main():
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in sys.argv[1:]:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                name = r["Kernel_Name"][:48]
                acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for name, ctrs in sorted(acc.items()):
        print(name)
        for c, v in sorted(ctrs.items()):
            print(f"    {c:28s} {sum(v) / len(v):16.1f}  (n={len(v)})")


if __name__ == "__main__":
    main()
