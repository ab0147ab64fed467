#!/usr/bin/env python3
"""Real-data input path throughput: train LR-FTRL from an .xfb shard through
the Trainer (BlockStream upload, optional HBM-resident epochs) and print the
per-epoch samples/s.

    python scripts/xfb_bench.py --rows 4194304 --epochs 3 [--resident] [--csr-only]

The shard is synthetic (Criteo-shaped: 39 fields, power-law values, hashed
64-bit keys) and written once to --dir; everything after that is the
production path: mmap -> pinned staging -> H2D copy stream -> train step.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def make_shard(path: str, rows: int, fields: int, seed: int, hash_space: int = 0) -> None:
    from xflow_amd.data import binfmt

    rng = np.random.default_rng(seed)
    keys = np.empty(rows * fields, np.uint64)
    mult = np.uint64(0x9E3779B97F4A7C15)
    for f in range(fields):
        v = rng.zipf(1.1 + 0.02 * f, size=rows).astype(np.uint64)
        h = (v + np.uint64(f << 40)) * mult
        if hash_space:  # hashed into [0, hash_space): multiply-high of the 64-bit hash
            h = ((h >> np.uint64(32)) * np.uint64(hash_space)) >> np.uint64(32)
        keys[f::fields] = h
    labels = (rng.random(rows) < 0.25).astype(np.float32)
    fg = np.tile(np.arange(fields, dtype=np.int32), rows)
    binfmt.write(path, labels, np.arange(rows + 1, dtype=np.int64) * fields, keys, fg)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=4 << 20)
    ap.add_argument("--fields", type=int, default=39)
    ap.add_argument("--epochs", type=int, default=3)
    ap.add_argument("--block-rows", type=int, default=262144)
    ap.add_argument("--dir", default="/tmp/xfb_bench")
    ap.add_argument("--resident", action="store_true")
    ap.add_argument("--csr-only", action="store_true")
    ap.add_argument("--copy-threads", type=int, default=8)
    ap.add_argument("--cpu", action="store_true")
    ap.add_argument("--hash-space", type=int, default=0,
                    help="features hashed into [0, N) (Criteo-1TB: 1e9); N <= 2^32 makes the "
                         "shard compact (u32 keys, half the streamed bytes); 0 = 64-bit keys")
    ap.add_argument("--test-rows", type=int, default=65536,
                    help="rows of the test shard rank 0 predicts (pred file + AUC/logloss)")
    a = ap.parse_args()

    import torch

    from xflow_amd.config import EngineConfig, ModelConfig, TrainConfig
    from xflow_amd.trainer import Trainer

    os.makedirs(a.dir, exist_ok=True)
    tr = os.path.join(a.dir, "train-00000.xfb")
    te = os.path.join(a.dir, "test-00000.xfb")
    t0 = time.perf_counter()
    from xflow_amd.data import binfmt

    want_compact = 0 < a.hash_space <= (1 << 32)
    if (not os.path.exists(tr) or binfmt.Shard(tr).rows != a.rows
            or binfmt.Shard(tr).compact != want_compact):
        make_shard(tr, a.rows, a.fields, 1, a.hash_space)
    if (not os.path.exists(te) or binfmt.Shard(te).rows != a.test_rows
            or binfmt.Shard(te).compact != want_compact):
        make_shard(te, a.test_rows, a.fields, 2, a.hash_space)
    print(f"shard ready ({time.perf_counter() - t0:.1f}s, "
          f"{os.path.getsize(tr) / 1e9:.2f} GB)", flush=True)
    dev = torch.device("cpu" if a.cpu or not torch.cuda.is_available() else "cuda:0")
    mfile = os.path.join(a.dir, "metrics.jsonl")
    if os.path.exists(mfile):
        os.remove(mfile)
    cfg = TrainConfig(train_prefix=os.path.join(a.dir, "train"),
                      test_prefix=os.path.join(a.dir, "test"), epochs=a.epochs, threads=1,
                      pred_dir=a.dir, model=ModelConfig(kind="lr"),
                      engine=EngineConfig(table_log2_cap=27), block_rows=a.block_rows,
                      resident=a.resident, fixed_width=not a.csr_only,
                      copy_threads=a.copy_threads, metrics_file=mfile)
    t = Trainer(cfg, device=dev)
    t0 = time.perf_counter()
    t.train_epochs(cfg.epochs)
    t1 = time.perf_counter()
    res = t.predict(0)  # device AUC/logloss + pred_0_0.txt
    t2 = time.perf_counter()
    wall = t2 - t0
    eps = [json.loads(l) for l in open(mfile) if '"epoch"' in l]
    eps = [e for e in eps if e.get("event") == "epoch"]
    print(json.dumps({"path": "xfb", "device": str(dev), "rows": a.rows,
                      "compact_keys": binfmt.Shard(tr).compact,
                      "block_rows": a.block_rows, "resident": a.resident,
                      "fixed_width": not a.csr_only,
                      "samples_per_s_by_epoch": [round(e["samples_per_s"]) for e in eps],
                      "train_logloss": [round(e["train_logloss"], 5) for e in eps],
                      "train_s": round(t1 - t0, 2), "predict_rows": res["n"],
                      "predict_s": round(t2 - t1, 3), "test_auc": round(res["auc"], 5),
                      "wall_s_incl_eval": round(wall, 2),
                      # XFLOW_STREAM_TIMELINE=1: per epoch, H2D time and the part of it
                      # that ran while a step was executing (HIP events)
                      **({"timeline_by_epoch": [e["timeline"] for e in eps]}
                         if eps and "timeline" in eps[0] else {})}), flush=True)
    # release the engine (device memory, pinned buffers) before interpreter
    # teardown: under rocprofv3 a late hipFree from a module destructor crashed
    t.close()
    del t
    import gc

    gc.collect()
    if dev.type == "cuda":
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        if hasattr(torch._C, "_host_emptyCache"):
            torch._C._host_emptyCache()  # pinned staging blocks
    return 0


if __name__ == "__main__":
    sys.exit(main())
