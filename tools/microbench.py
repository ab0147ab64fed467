#!/usr/bin/env python3
"""Kernel-level micro benchmark on one GPU: times train_step and eval_step
(dedup + pull + forward) on the bench's synthetic batch, interleaved in one
process (run under rocprofv3 --kernel-trace --stats for per-kernel times)."""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from xflow_amd.config import EngineConfig, ModelConfig, OptimConfig  # noqa: E402
from xflow_amd.data.synth import SynthConfig, SyntheticCriteo  # noqa: E402
from xflow_amd.engine import Engine  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=262144)
ap.add_argument("--model", default="lr")
ap.add_argument("--v-dim", type=int, default=8)
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--log2-cap", type=int, default=28)
a = ap.parse_args()
dev = torch.device("cuda", 0)
cfg = SynthConfig()
eng = Engine(ModelConfig(kind=a.model, v_dim=a.v_dim), OptimConfig(),
             EngineConfig(table_log2_cap=a.log2_cap, max_rows=a.rows, max_nnz=a.rows * cfg.fields),
             device=dev)
gen = SyntheticCriteo(eng, a.rows, cfg)
b = gen.alloc_batch()
for _ in range(5):
    eng.train_step(gen.next(out=b))
pctr = torch.empty(a.rows, device=dev)
res = {}
for name in ("train", "eval"):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(a.iters):
        if name == "train":
            eng.train_step(b)
        else:
            eng.eval_step(b, pctr)
    torch.cuda.synchronize()
    res[name] = (time.perf_counter() - t) / a.iters * 1e3
print({k: f"{v:.3f} ms" for k, v in res.items()}, "n_unique", eng.n_unique())
