#!/usr/bin/env python3
"""A parameter table past half of the device's memory keeps growing.

    python tools/table_grow_bench.py [--kind fm --v-dim 8] [--log2-cap 30]

The table starts at 2^--log2-cap slots and is filled with synthetic keys
(Engine.prefill, k_table_prefill) in chunks of --chunk keys; every chunk's
insert guard grows the table by segment splits (linear hashing,
csrc/engine/engine.cpp Engine::segments_for / split_to) once the fullest
segments pass grow_start.  Each split adds ONE segment of device memory,
mapped at the end of the table's reserved address range
(HipBackend::table_commit), and rewrites one segment -- so the table can grow
while it holds more than half of HBM, which a 2x rehash into a second table
(old + new resident at once) cannot.

Per chunk: keys, segments, table / committed GB, the device's used memory
fraction, and the chunk's synchronised wall time (splitting chunks vs plain
ones = the growth cost).  One JSON line per chunk, then a summary line.
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


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--kind", default="fm")
    ap.add_argument("--v-dim", type=int, default=8)
    ap.add_argument("--log2-cap", type=int, default=30)
    ap.add_argument("--max-log2-cap", type=int, default=31)
    ap.add_argument("--chunk", type=int, default=20_000_000)
    ap.add_argument("--fill", type=float, default=0.79,
                    help="stop at this load of 2^max-log2-cap slots")
    a = ap.parse_args()
    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    if dev.type == "cpu":
        a.log2_cap, a.max_log2_cap, a.chunk = 14, 16, 2000

    def mem():
        if dev.type != "cuda":
            return None, None
        fr, tot = torch.cuda.mem_get_info(dev)
        return (tot - fr) / tot, tot

    e = Engine(ModelConfig(kind=a.kind, v_dim=a.v_dim), OptimConfig(),
               EngineConfig(table_log2_cap=a.log2_cap, max_rows=1024, max_nnz=1024 * 39,
                            max_log2_cap=a.max_log2_cap), device=dev)
    slot_bytes = e.state_words * 4 + 8
    _, total = mem()
    start = {"kind": a.kind, "v_dim": a.v_dim, "slot_bytes": slot_bytes,
             "slots": e.table_capacity, "geometry": e.table_geometry,
             "table_GB": e.table_capacity * slot_bytes / 1e9,
             "device_GB": total / 1e9 if total else None}
    print(json.dumps({"start": start}), flush=True)
    # fill to just below the first split without timing every chunk
    first = int(0.59 * e.table_capacity)  # (grow_start 0.6)
    t = time.perf_counter()
    e.prefill(first, seed=1)
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    print(json.dumps({"prefill_keys": first, "s": time.perf_counter() - t,
                      "splits": e.table_splits}), flush=True)
    stop = int(a.fill * (1 << a.max_log2_cap))
    seed = 2
    rows = []
    while e.table_size() + a.chunk <= stop:
        seg0, spl0 = e.table_geometry["segments"], e.table_splits
        used0, _ = mem()
        t = time.perf_counter()
        e.prefill(a.chunk, seed=seed)
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        dt = time.perf_counter() - t
        seed += 1
        used1, _ = mem()
        g = e.table_geometry
        r = {"keys": e.table_size(), "segments": g["segments"], "level": g["level"],
             "split": g["split"], "new_splits": e.table_splits - spl0, "chunk_s": dt,
             "table_GB": e.table_capacity * slot_bytes / 1e9,
             "committed_GB": e.table_committed / 1e9,
             "device_used_before": used0, "device_used_after": used1,
             "load": e.table_size() / e.table_capacity}
        rows.append(r)
        print(json.dumps(r), flush=True)
        assert not e.overflowed()
        if g["segments"] == 1 << (a.max_log2_cap - g["seg_log2"]) and r["new_splits"] == 0 \
                and r["load"] > 0.75:
            break
    grew = [r for r in rows if r["new_splits"]]
    plain = [r for r in rows if not r["new_splits"]]
    big = [r for r in grew if r["device_used_before"] is not None and r["device_used_before"] >= 0.5]
    summ = {"splits": e.table_splits, "growths": e.table_growths,
            "final_slots": e.table_capacity, "final_table_GB": e.table_capacity * slot_bytes / 1e9,
            "grow_chunks": len(grew), "grow_chunks_at_or_above_half_hbm": len(big),
            "plain_chunk_s": (sum(r["chunk_s"] for r in plain) / len(plain)) if plain else None,
            "grow_chunk_s": (sum(r["chunk_s"] for r in grew) / len(grew)) if grew else None,
            "segments_per_grow_chunk": (sum(r["new_splits"] for r in grew) / len(grew)) if grew else None,
            "grow_seconds_host": e.grow_seconds,
            # device time of one segment split (splitting chunks minus plain ones)
            "ms_per_split": ((sum(r["chunk_s"] for r in grew)
                              - len(grew) * (sum(r["chunk_s"] for r in plain) / max(len(plain), 1)))
                             * 1e3 / max(sum(r["new_splits"] for r in grew), 1)) if grew else None,
            "segment_slots": 1 << e.table_geometry["seg_log2"],
            "max_device_used": max((r["device_used_after"] or 0) for r in rows) if rows else None}
    print(json.dumps({"summary": summ}), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
