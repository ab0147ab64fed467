#!/usr/bin/env python3
"""Production-scale table operations on one device: how long the parameter
store's maintenance takes at the bench's occupancy.

    python tools/table_ops_bench.py [--log2-cap 31] [--keys 1000000000]

* prefill   --keys synthetic keys into 2^log2_cap slots (k_table_prefill)
* export    every (key, state) pair to host arrays (Engine.export_table: the
            checkpoint writer's source, csrc/engine/engine.cpp)
* save      the native shard file of a checkpoint (--save-dir; skipped when
            empty: a 1e9-key LR shard is 16 GB)
* grow      every segment of a table prefilled to --grow-load split once
            (k_table_split_marks + k_table_split: the device work a run's
            growth adds, spread over the steps by EngineConfig.grow_start),
            at 2^--grow-log2 slots, for LR and FM-8 (--grow-kinds)

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
    ap.add_argument("--grow-kinds", default="lr,fm")
    ap.add_argument("--grow-only", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    if dev.type == "cpu":
        a.log2_cap, a.keys, a.grow_log2 = min(a.log2_cap, 20), min(a.keys, 400_000), 18
    out = {"tool": "table_ops_bench", "device": str(dev)}
    if not a.grow_only:
        ops(a, dev, out)
    for kind in a.grow_kinds.split(","):
        out[f"grow_{kind}"] = grow(a, dev, kind)
    print(json.dumps(out), flush=True)


def grow(a, dev, kind):
    """Split every segment of a 2^grow_log2-slot table at load grow_load once
    (explicit grow_table: a whole level at once; a run spreads these splits
    over its steps).  Device seconds, from synchronised wall clock."""
    g = Engine(ModelConfig(kind=kind, v_dim=8), OptimConfig(),
               EngineConfig(table_log2_cap=a.grow_log2, max_rows=1024, max_nnz=1024 * 39,
                            max_log2_cap=a.grow_log2 + 1, grow_start=0.79, grow_load=0.8),
               device=dev)
    n = int(a.grow_load * (1 << a.grow_log2))
    g.prefill(n)
    _sync(dev)
    assert g.table_growths == 0
    t = time.perf_counter()
    g.grow_table(a.grow_log2 + 1)
    _sync(dev)
    dt = time.perf_counter() - t
    r = {"slots_from": 1 << a.grow_log2, "slots_to": g.table_capacity, "keys": g.table_size(),
         "slot_bytes": g.state_words * 4 + 8, "segments_split": g.table_splits, "s": dt,
         "ms_per_1e8_keys": dt * 1e3 / max(g.table_size(), 1) * 1e8,
         "table_GB_to": g.table_capacity * (g.state_words * 4 + 8) / 1e9,
         "committed_GB": g.table_committed / 1e9}
    assert g.table_size() == n and g.table_capacity == 1 << (a.grow_log2 + 1)
    assert not g.overflowed()
    del g
    if dev.type == "cuda":
        torch.cuda.empty_cache()
    return r


def ops(a, dev, out):
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


if __name__ == "__main__":
    main()
