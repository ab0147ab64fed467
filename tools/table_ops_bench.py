#!/usr/bin/env python3
"""Production-scale table operations on one device: how long the parameter
store's maintenance takes at the bench's occupancy.

    python tools/table_ops_bench.py [--log2-cap 31] [--keys 1000000000]

* prefill   --keys synthetic keys into 2^log2_cap slots (k_table_prefill)
* export    every (key, state) pair to host arrays (Engine.export_table: the
            checkpoint writer's source, csrc/engine/engine.cpp)
* save      the native shard file of a checkpoint (--save-dir; skipped when
            empty: a 1e9-key LR shard is 16 GB)
* grow      a 2x rehash of a table prefilled to --grow-load (k_table_rehash;
            the pause a run takes when the store outgrows its capacity,
            EngineConfig.table_grow), at 2^--grow-log2 slots

Prints one JSON line of seconds and rates.  The reference keeps its weights
in server RAM and never checkpoints or rehashes (ftrl.h:84,151).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from xflow_amd.config import EngineConfig, ModelConfig, OptimConfig  # noqa: E402
from xflow_amd.engine import Engine  # noqa: E402


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def main():
    ap = argparse.ArgumentParser(description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--log2-cap", type=int, default=31)
    ap.add_argument("--keys", type=int, default=1_000_000_000)
    ap.add_argument("--grow-log2", type=int, default=28)
    ap.add_argument("--grow-load", type=float, default=0.75)
    ap.add_argument("--save-dir", default="")
    a = ap.parse_args()
    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    if dev.type == "cpu":
        a.log2_cap, a.keys, a.grow_log2 = min(a.log2_cap, 20), min(a.keys, 400_000), 18
    out = {"tool": "table_ops_bench", "device": str(dev)}

    e = Engine(ModelConfig(kind="lr"), OptimConfig(),
               EngineConfig(table_log2_cap=a.log2_cap, max_rows=1024, max_nnz=1024 * 39,
                            table_grow=False), device=dev)
    t = time.perf_counter()
    e.prefill(a.keys)
    _sync(dev)
    out["prefill_s"] = time.perf_counter() - t
    out["keys"] = e.table_size()
    out["slots"] = 1 << a.log2_cap
    t = time.perf_counter()
    keys, words = e.export_table()
    out["export_s"] = time.perf_counter() - t
    nbytes = keys.nbytes + words.nbytes
    out["export_GB"] = nbytes / 1e9
    out["export_GBps"] = nbytes / 1e9 / max(out["export_s"], 1e-9)
    sample = keys[:: max(1, len(keys) // 4096)].copy()
    want = e.pull(sample)
    p = os.path.join(a.save_dir, "shard.xftb") if a.save_dir else ""
    if p:
        os.makedirs(a.save_dir, exist_ok=True)
        t = time.perf_counter()
        e.save(p)
        out["save_s"] = time.perf_counter() - t
        out["save_GB"] = os.path.getsize(p) / 1e9
    del e
    if dev.type == "cuda":
        torch.cuda.empty_cache()

    # import into a fresh table (the checkpoint loader's path), then the file
    f = Engine(ModelConfig(kind="lr"), OptimConfig(),
               EngineConfig(table_log2_cap=a.log2_cap, max_rows=1024, max_nnz=1024 * 39,
                            table_grow=False), device=dev)
    t = time.perf_counter()
    f.import_table(keys, words)
    _sync(dev)
    out["import_s"] = time.perf_counter() - t
    out["import_GBps"] = nbytes / 1e9 / max(out["import_s"], 1e-9)
    assert f.table_size() == out["keys"], (f.table_size(), out["keys"])
    assert (f.pull(sample) == want).all(), "imported table differs"
    del keys, words, f
    if p:
        g0 = Engine(ModelConfig(kind="lr"), OptimConfig(),
                    EngineConfig(table_log2_cap=a.log2_cap, max_rows=1024, max_nnz=1024 * 39,
                                 table_grow=False), device=dev)
        t = time.perf_counter()
        g0.load(p)
        _sync(dev)
        out["load_s"] = time.perf_counter() - t
        assert g0.table_size() == out["keys"]
        assert (g0.pull(sample) == want).all(), "loaded table differs"
        os.remove(p)
        del g0
    if dev.type == "cuda":
        torch.cuda.empty_cache()

    g = Engine(ModelConfig(kind="lr"), OptimConfig(),
               EngineConfig(table_log2_cap=a.grow_log2, max_rows=1024, max_nnz=1024 * 39,
                            max_log2_cap=a.grow_log2 + 1), device=dev)
    n = int(a.grow_load * (1 << a.grow_log2))
    g.prefill(n)
    _sync(dev)
    t = time.perf_counter()
    g.grow_table(a.grow_log2 + 1)
    _sync(dev)
    out["grow_s"] = time.perf_counter() - t
    out["grow_keys"] = g.table_size()
    out["grow_from_slots"] = 1 << a.grow_log2
    out["grow_Mkeys_per_s"] = g.table_size() / 1e6 / max(out["grow_s"], 1e-9)
    assert g.table_size() == n and g.table_capacity == 1 << (a.grow_log2 + 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
