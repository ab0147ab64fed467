#!/usr/bin/env python3
"""Emulated W-GPU node on one device: the per-rank cost of the multi-GPU
(sharded) LR/FM/MVM step at its real per-rank shape.

W engines ("virtual ranks") live on one GPU, each with its own table shard
(2^log2_cap slots, prefilled to --table-load like bench.py), its own
synthetic Criteo-shaped batch stream (262 144 rows x 39 fields per rank by
default) and its own host thread; the all-to-alls go through an in-process
device-copy bus (xflow_amd/parallel/loopback.py).  All ranks share one stream,
so their kernels execute one after another: under

    rocprofv3 --kernel-trace --stats -- python3 tools/w8_emulate.py

the kernel statistics divided by (W x steps) are the per-rank device time of
one step of the 8-GPU run -- the 8-range partitioned dedup,
k_partition_counts, the owner pull of all sources' keys, k_owner_group, the
multi-source apply -- everything but the xGMI transfer itself, which the
tool reports as bytes per link per step instead (the bus copies appear as
copy kernels in the trace).

Prints one JSON line: wall ms per emulated node step (all W ranks
serialised), the per-rank share, and the per-link a2a bytes.
Reference call sites replaced by this step: lr_worker.cc:170,175 (Pull/Push),
ftrl.h:54-80 (server apply).
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
from xflow_amd.data.synth import SynthConfig, SyntheticCriteo  # noqa: E402
from xflow_amd.engine import Engine  # noqa: E402
from xflow_amd.parallel.loopback import LoopbackBus, loopback_engine, run_ranks  # noqa: E402


def main():
    ap = argparse.ArgumentParser(description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rows", type=int, default=262144, help="rows per rank per step")
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", default="lr", choices=["lr", "fm", "mvm"])
    ap.add_argument("--v-dim", type=int, default=8)
    ap.add_argument("--log2-cap", type=int, default=28,
                    help="table slots per rank (2^31 / 8 on the real node)")
    ap.add_argument("--table-load", type=float, default=0.47)
    ap.add_argument("--features", type=int, default=1_000_000_000)
    ap.add_argument("--async", dest="async_p2p", action="store_true",
                    help="staleness-1 step (config 4)")
    ap.add_argument("--lambda1", type=float, default=5e-5)
    ap.add_argument("--out", default="", help="also write the JSON line here")
    a = ap.parse_args()

    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    W = a.world
    if dev.type == "cpu":
        a.rows = min(a.rows, 2048)
        a.log2_cap = min(a.log2_cap, 18)
    synth = SynthConfig(total_features=a.features, hash_space=a.features)
    engines, gens, bufs = [], [], []
    for r in range(W):
        e = Engine(ModelConfig(kind=a.model, v_dim=a.v_dim), OptimConfig(lambda1=a.lambda1),
                   EngineConfig(table_log2_cap=a.log2_cap, max_rows=a.rows,
                                max_nnz=a.rows * synth.fields), device=dev)
        n_pre = int(a.table_load * (1 << a.log2_cap))
        if n_pre:
            e.prefill(n_pre, seed=0x5eed + r)
        g = SyntheticCriteo(e, a.rows, synth, rank=r)
        engines.append(e)
        gens.append(g)
        bufs.append([g.alloc_batch(), g.alloc_batch()])
    bus = LoopbackBus(W)
    cls = None
    if a.async_p2p:
        from xflow_amd.parallel.async_p2p import AsyncShardedEngine

        cls = AsyncShardedEngine
    sh = [loopback_engine(bus, r, engines[r], **({"cls": cls} if cls else {})) for r in range(W)]
    marks = {}

    def rank_fn(r):
        s, g, b = sh[r], gens[r], bufs[r]
        g.next(out=b[0])
        cur = 0
        for it in range(a.warmup + a.steps):
            if it == a.warmup:
                bus.barrier.wait()
                if r == 0:
                    torch.cuda.synchronize() if dev.type == "cuda" else None
                    marks["links0"] = [row[:] for row in bus.link_bytes]
                    marks["t0"] = time.perf_counter()
                    marks["hw0"] = sum(x.host_waits for x in sh)
                bus.barrier.wait()
            i = cur
            s.train_step(b[i], prefetch=lambda: g.next(out=b[i ^ 1]), next_batch=b[i ^ 1])
            cur ^= 1
        if hasattr(s, "flush"):
            s.flush()

    run_ranks(bus, rank_fn)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    dt = time.perf_counter() - marks["t0"]
    ovf = any(e.overflowed() for e in engines)
    links = [[bus.link_bytes[s][d] - marks["links0"][s][d] for d in range(W)] for s in range(W)]
    off = [links[s][d] for s in range(W) for d in range(W) if s != d]
    st = [e.read_stats() for e in engines]
    rows = sum(x["rows"] for x in st)
    out = {
        "tool": "w8_emulate", "world": W, "model": a.model, "rows_per_rank": a.rows,
        "steps": a.steps, "warmup": a.warmup, "async": a.async_p2p,
        "table_slots_per_rank": 1 << a.log2_cap,
        "table_load": sum(e.table_size() for e in engines) / float(W << a.log2_cap),
        "ms_per_node_step_serialised": 1000.0 * dt / a.steps,
        "ms_per_rank_step": 1000.0 * dt / a.steps / W,
        "a2a_bytes_per_link_per_step_mean": sum(off) / len(off) / a.steps if off else 0,
        "a2a_bytes_per_link_per_step_max": max(off) / a.steps if off else 0,
        "a2a_bytes_per_rank_out_per_step": sum(off) / W / a.steps if off else 0,
        "host_waits": sum(x.host_waits for x in sh) - marks["hw0"],
        "train_logloss": sum(x["ln_loss"] for x in st) / max(rows, 1.0),
        "overflow": ovf,
        "device": str(dev),
    }
    line = json.dumps(out)
    print(line, flush=True)
    if a.out:
        with open(a.out, "w") as f:
            f.write(line + "\n")
    if ovf:
        raise SystemExit("w8_emulate: overflow flagged")


if __name__ == "__main__":
    main()
