#!/usr/bin/env python3
"""A/B of the standard-math FM forward: VALU (k_fm<D,false,false>, one lane
per row) vs matrix cores (k_fm_fwd_mfma<D>, v_mfma_f32_16x16x4_f32) on the
bench shape (262144 rows x 39 fields, field-major synthetic Criteo batch).
Run under rocprofv3 --kernel-trace --stats for per-kernel times.

    python tools/fm_mfma_ab.py [--rows 262144] [--v-dim 8] [--iters 20]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from xflow_amd.config import EngineConfig, ModelConfig, OptimConfig  # noqa: E402
from xflow_amd.data.synth import SyntheticCriteo  # noqa: E402
from xflow_amd.engine import Engine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=262144)
    ap.add_argument("--v-dim", type=int, default=8)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    res = {}
    for mfma in (False, True):
        e = Engine(ModelConfig(kind="fm", v_dim=a.v_dim, fm_math="standard", fm_mfma=mfma),
                   OptimConfig(v_init_scale=0.1),
                   EngineConfig(table_log2_cap=26, max_rows=a.rows, max_nnz=a.rows * 39),
                   device=dev)
        gen = SyntheticCriteo(e, a.rows)
        b = gen.alloc_batch()
        for _ in range(2):
            gen.next(out=b)
            e.train_step(b)
        gen.next(out=b)
        pctr = e.eval_step(b)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            e.eval_step(b, pctr)
        torch.cuda.synchronize()
        res[mfma] = (time.perf_counter() - t0) / a.iters * 1e3
        print(f"{'mfma' if mfma else 'valu'}: eval step (dedup + pull + forward) "
              f"{res[mfma]:.3f} ms, mean pctr {float(pctr.mean()):.6f}", flush=True)


if __name__ == "__main__":
    main()
