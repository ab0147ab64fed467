#!/usr/bin/env python3
"""Time the device-side eval metrics (Engine.eval_metrics: stable radix sort
of pctr + exact rank-sum AUC + double logloss, csrc/hip/kernels_eval.hip) on a
synthetic N-row prediction set, against the host path it replaces (D2H copy +
the reference printer's sort, xflow_amd.metrics.reference_auc).

    python tools/eval_bench.py --rows 10000000 --reps 5
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from xflow_amd.config import EngineConfig, ModelConfig, OptimConfig  # noqa: E402
from xflow_amd.engine import Engine  # noqa: E402
from xflow_amd.metrics import reference_auc  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--host", action="store_true", help="also time the host reference path")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(7)
    n = args.rows
    # planted signal: labels drawn from the predictions
    p = torch.rand(n, device=dev, generator=g) * 0.98 + 0.01
    y = (torch.rand(n, device=dev, generator=g) < p).float()
    e = Engine(ModelConfig(), OptimConfig(), EngineConfig(table_log2_cap=8), device=dev)
    r = e.eval_metrics(p, y)  # warm (workspace allocation, code load)
    torch.cuda.synchronize()
    ts = []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        r = e.eval_metrics(p, y)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    out = {"rows": n, "device_ms_min": 1e3 * min(ts), "device_ms_median": 1e3 * sorted(ts)[len(ts) // 2],
           "auc": r["auc"], "ln_logloss": r["ln_logloss"], "line": r["line"]}
    if args.host:
        t0 = time.perf_counter()
        ph, yh = p.cpu().numpy(), y.cpu().numpy().astype(np.int32)
        ref = reference_auc(yh, ph)
        out["host_ms"] = 1e3 * (time.perf_counter() - t0)
        out["host_line"] = ref["line"]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
