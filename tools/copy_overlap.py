#!/usr/bin/env python3
"""H2D copy / kernel overlap of a rocprofv3 run
(``rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d DIR``).

    python tools/copy_overlap.py DIR [--skip 0.4]

Prints, over the trace after --skip (fraction of the time span, warm-up):
host-to-device copy time and bytes (and the achieved link rate), kernel busy
time, and how much of the copy time ran while a kernel was executing -- the
evidence that the streamed input path (xflow_amd/data/upload.py BlockStream)
uploads block t+1 during step t instead of between steps.
"""
from __future__ import annotations

import argparse
import csv
import glob
import os


def _load(path, kind):
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            if kind == "copy":
                d = r.get("Direction", "")
                if "HOST_TO_DEVICE" not in d.upper() and "H2D" not in d.upper():
                    continue
                out.append((s, e, int(r.get("Bytes", 0) or 0)))
            else:
                out.append((s, e, 0))
    return sorted(out)


def _load_named(path):
    with open(path) as f:
        return sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), 0, r["Kernel_Name"])
                      for r in csv.DictReader(f))


def _union(iv):
    res = []
    for s, e, _ in iv:
        if res and s <= res[-1][1]:
            res[-1][1] = max(res[-1][1], e)
        else:
            res.append([s, e])
    return res


def _overlap(a, b):
    """Total length of the intersection of two sorted disjoint interval lists."""
    i = j = 0
    tot = 0
    while i < len(a) and j < len(b):
        lo, hi = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if hi > lo:
            tot += hi - lo
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--skip", type=float, default=0.4)
    a = ap.parse_args()
    kt = glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True)
    ct = glob.glob(os.path.join(a.dir, "**", "*memory_copy_trace.csv"), recursive=True)
    if not kt:
        raise SystemExit("need kernel_trace.csv under " + a.dir)
    ks = _load(kt[0], "kernel")
    if ct:
        cs = _load(ct[0], "copy")
    else:
        # HSA_ENABLE_SDMA=0: the copies run as blit kernels in the kernel trace
        blit = [x for x in _load_named(kt[0]) if "copyBuffer" in x[3]]
        ks = [(s, e, 0) for s, e, _, n in _load_named(kt[0]) if "copyBuffer" not in n]
        cs = [(s, e, 0) for s, e, _, _ in blit]
        print("(no memory-copy trace: copies taken from blit kernels, sizes unknown)")
    t0 = min(ks[0][0], cs[0][0]) if cs else ks[0][0]
    t1 = max(max(e for _, e, _ in ks), max((e for _, e, _ in cs), default=0))
    cut = t0 + a.skip * (t1 - t0)
    ks = [x for x in ks if x[0] >= cut]
    cs = [x for x in cs if x[0] >= cut]
    ku, cu = _union(ks), _union(cs)
    kbusy = sum(e - s for s, e in ku)
    cbusy = sum(e - s for s, e in cu)
    nbytes = sum(b for _, _, b in cs)
    ov = _overlap(ku, cu)
    span = (t1 - cut) / 1e6
    print(f"window {span:.2f} ms: kernels busy {kbusy / 1e6:.2f} ms, H2D copies {len(cs)} "
          f"({nbytes / 1e9:.2f} GB) busy {cbusy / 1e6:.2f} ms = {nbytes / max(cbusy, 1):.1f} GB/s "
          f"while copying")
    print(f"H2D time concurrent with kernels: {ov / 1e6:.2f} ms "
          f"({100.0 * ov / max(cbusy, 1):.1f}% of copy time, {100.0 * ov / max(kbusy, 1):.1f}% "
          f"of kernel time)")


if __name__ == "__main__":
    main()
