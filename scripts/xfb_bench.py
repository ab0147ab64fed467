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


def make_criteo_shard(path: str, rows: int, fields: int, seed: int, fmt: str,
                      block_rows: int) -> dict:
    """The bench's own synthetic Criteo-1TB-shaped rows (xflow_amd.data.synth:
    MLPerf cardinalities, 1e9 hashed features) written as an .xfb shard:
    fmt "v2" (compact u32 keys, CSR) or "packed" (version 3)."""
    import torch

    from xflow_amd.config import EngineConfig, ModelConfig, OptimConfig
    from xflow_amd.data import binfmt
    from xflow_amd.data.synth import SynthConfig, SyntheticCriteo
    from xflow_amd.engine import Engine

    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    chunk = 262144
    eng = Engine(ModelConfig(), OptimConfig(),
                 EngineConfig(table_log2_cap=10, max_rows=chunk, max_nnz=chunk * fields), device=dev)
    gen = SyntheticCriteo(eng, chunk, SynthConfig(seed=seed, n_fields=fields))
    keys = np.empty((rows, fields), np.uint64)
    labels = np.empty(rows, np.float32)
    for r0 in range(0, rows, chunk):
        n = min(chunk, rows - r0)
        gen.rows = n
        b = gen.next(out=SyntheticCriteo(eng, n, gen.cfg).alloc_batch())
        keys[r0:r0 + n] = b.keys.view(fields, n).t().cpu().numpy().view(np.uint64)
        labels[r0:r0 + n] = b.labels.cpu().numpy()
    if fmt == "packed":
        return binfmt.write_packed(path, labels, keys, block_rows=block_rows)
    binfmt.write(path, labels, np.arange(rows + 1, dtype=np.int64) * fields, keys.reshape(-1),
                 np.tile(np.arange(fields, dtype=np.int32), rows), compact="auto")
    return {"rows": rows, "F": fields, "bytes_per_row": (os.path.getsize(path) / rows)}


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
    ap.add_argument("--data", choices=["zipf", "criteo"], default="zipf",
                    help="criteo: the bench's synthetic Criteo-1TB shape (data/synth.py; MLPerf "
                         "cardinalities, 1e9 hashed features)")
    ap.add_argument("--format", choices=["v2", "packed"], default="v2",
                    help="--data criteo: the compact CSR shard (v2) or packed field-major "
                         "blocks with per-field dictionaries (v3)")
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

    info = {}
    if a.data == "criteo":
        tag = os.path.join(a.dir, "shard.json")
        want = {"rows": a.rows, "fields": a.fields, "format": a.format, "test_rows": a.test_rows,
                "block_rows": a.block_rows}
        if not os.path.exists(tag) or json.load(open(tag)) != want:
            info = make_criteo_shard(tr, a.rows, a.fields, 1234, a.format, a.block_rows)
            make_criteo_shard(te, a.test_rows, a.fields, 99, a.format, a.block_rows)
            json.dump(want, open(tag, "w"))
    else:
        want_compact = 0 < a.hash_space <= (1 << 32)
        if (not os.path.exists(tr) or binfmt.version_of(tr) == binfmt.VERSION_PACKED
                or binfmt.Shard(tr).rows != a.rows or binfmt.Shard(tr).compact != want_compact):
            make_shard(tr, a.rows, a.fields, 1, a.hash_space)
        if (not os.path.exists(te) or binfmt.version_of(te) == binfmt.VERSION_PACKED
                or binfmt.Shard(te).rows != a.test_rows or binfmt.Shard(te).compact != want_compact):
            make_shard(te, a.test_rows, a.fields, 2, a.hash_space)
    print(f"shard ready ({time.perf_counter() - t0:.1f}s, "
          f"{os.path.getsize(tr) / 1e9:.2f} GB, {os.path.getsize(tr) / a.rows:.1f} B/row) {info}",
          flush=True)
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
    ver = binfmt.version_of(tr)
    print(json.dumps({"path": "xfb", "device": str(dev), "rows": a.rows, "data": a.data,
                      "xfb_version": ver, "bytes_per_row": round(os.path.getsize(tr) / a.rows, 1),
                      "compact_keys": ver == binfmt.VERSION_PACKED or binfmt.Shard(tr).compact,
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
