#!/usr/bin/env python3
"""Per-rank device time of one emulated multi-GPU step (tools/w8_emulate.py)
from rocprofv3 output.

With a kernel-trace CSV (preferred) only the timed steps count: the window
starts at the owner pull of the first timed step (W pulls per step, after
`warmup` steps) and every dispatch in it is summed per kernel name, divided
by W x steps.  With a kernel-stats CSV every call counts (warm-up steps and
one-time setup fills included; table prefill/clear excluded), divided by the
pull's call count."""
from __future__ import annotations

import argparse
import collections
import csv

ONE_TIME = ("k_table_prefill", "k_table_clear")


def from_trace(path, world, warmup):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    pulls = [r for r in rows if "k_pull" in r["Kernel_Name"] and "values" not in r["Kernel_Name"]]
    if len(pulls) <= world * warmup:
        raise SystemExit("trace shorter than the warm-up")
    t0 = int(pulls[world * warmup]["Start_Timestamp"])
    steps = (len(pulls) - world * warmup) / world
    acc = collections.defaultdict(float)
    calls = collections.Counter()
    for r in rows:
        if int(r["Start_Timestamp"]) < t0:
            continue
        name = r["Kernel_Name"]
        acc[name] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0
        calls[name] += 1
    return {k: (v / (world * steps), calls[k]) for k, v in acc.items()}, steps


def from_stats(path, world):
    rows = list(csv.DictReader(open(path)))
    pull = [r for r in rows if "k_pull" in r["Name"]]
    steps = int(pull[0]["Calls"]) / world if pull else 1.0
    out = {}
    for r in rows:
        if any(t in r["Name"] for t in ONE_TIME):
            continue
        out[r["Name"]] = (float(r["TotalDurationNs"]) / 1000.0 / (world * steps), int(r["Calls"]))
    return out, steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv", help="rocprofv3 kernel_trace.csv (or kernel_stats.csv)")
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--top", type=int, default=16)
    a = ap.parse_args()
    head = open(a.csv).readline()
    if "Start_Timestamp" in head:
        per, steps = from_trace(a.csv, a.world, a.warmup)
        what = "timed steps"
    else:
        per, steps = from_stats(a.csv, a.world)
        what = "all calls"
    total = sum(v for v, _ in per.values())
    for name, (us, calls) in sorted(per.items(), key=lambda x: -x[1][0])[:a.top]:
        print(f"  {name[:64]:64s} calls={calls:6d} us/rank-step={us:8.1f}")
    print(f"  TOTAL device us per rank-step: {total:.1f}  ({what}, {steps:.0f} steps per rank)")


if __name__ == "__main__":
    main()
