#!/usr/bin/env python3
"""Timeline summary of a rocprofv3 kernel trace: GPU busy vs idle time and the
idle gaps that follow each kernel (the host-side stalls between launches).

    python tools/trace_gaps.py gpurun_out/prof_x/run_kernel_trace.csv [--skip F]
    python tools/trace_gaps.py <trace> --marker k_synth --steps 18
    python tools/trace_gaps.py <trace rank 0> <trace rank 1> ...   (several
        processes sharing one GPU: the union of their kernels, i.e. whether
        the DEVICE idles; kernel names carry their rank)

--skip drops the first fraction of the trace (warmup, setup); --marker instead
cuts the trace at the dispatches of the step's first kernel and analyses the
last --steps complete steps (and prints the last one's timeline).
"""
from __future__ import annotations

import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace", nargs="+")
    ap.add_argument("--skip", type=float, default=0.3,
                    help="fraction of the trace (by time) to skip as warmup")
    ap.add_argument("--top", type=int, default=12)
    ap.add_argument("--marker", default="",
                    help="kernel that opens a step (e.g. k_synth): analyse the last --steps "
                         "complete steps only and print the last step's timeline")
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    rows = []
    for k, path in enumerate(a.trace):
        tag = f"[r{k}] " if len(a.trace) > 1 else ""
        with open(path) as f:
            for r in csv.DictReader(f):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                             tag + r["Kernel_Name"][:60]))
    rows.sort()
    if not rows:
        return
    if a.marker:
        starts = [i for i, r in enumerate(rows) if a.marker in r[2]]
        if len(starts) < 2:
            raise SystemExit(f"fewer than two '{a.marker}' dispatches")
        k = min(a.steps, len(starts) - 1)
        lo, hi = starts[-1 - k], starts[-1]
        print(f"{k} steps: {(rows[hi][0] - rows[lo][0]) / 1e3 / k:.1f} us/step (marker to marker)")
        print("-- last step timeline (start us, duration us)")
        for s, e, n in rows[starts[-2]:hi]:
            print(f"  {(s - rows[starts[-2]][0]) / 1e3:8.1f} {(e - s) / 1e3:7.1f}  {n}")
        rows = rows[lo:hi]
    else:
        t0, t1 = rows[0][0], max(r[1] for r in rows)
        cut = t0 + a.skip * (t1 - t0)
        rows = [r for r in rows if r[0] >= cut]
    busy = collections.Counter()
    gaps = collections.Counter()
    ngap = collections.Counter()
    end = rows[0][0]
    total_busy = 0
    for i, (s, e, n) in enumerate(rows):
        if i and s > end:
            gaps[rows[i - 1][2] + " -> " + n[:30]] += s - end
            ngap[rows[i - 1][2] + " -> " + n[:30]] += 1
        total_busy += max(0, e - max(s, end))
        busy[n] += e - s
        end = max(end, e)
    wall = end - rows[0][0]
    print(f"window {wall / 1e6:.3f} ms  busy {total_busy / 1e6:.3f} ms "
          f"({100.0 * total_busy / max(wall, 1):.1f}%)  idle {(wall - total_busy) / 1e6:.3f} ms")
    print("-- busy by kernel (us total)")
    for n, t in busy.most_common(a.top):
        print(f"  {t / 1e3:10.1f}  {n}")
    print("-- idle gaps after kernel (us total, count)")
    for n, t in gaps.most_common(a.top):
        print(f"  {t / 1e3:10.1f}  x{ngap[n]:<4d} {n}")


if __name__ == "__main__":
    main()
