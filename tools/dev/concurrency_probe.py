"""Do two latency-bound LR steps overlap?  Two independent engines (own tables,
own synthetic batches) issue their steps on two HIP streams; the aggregate
samples/s is compared with the same engines stepping one after the other on
one stream.  A probe for pipelining a step's dedup with the previous step's
apply (tools/dev, not part of the framework).

  python tools/dev/concurrency_probe.py [--steps 20] [--log2-cap 31]
"""
import argparse
import json
import math
import time

import torch

from xflow_amd.config import EngineConfig, ModelConfig, OptimConfig
from xflow_amd.data.synth import SynthConfig, SyntheticCriteo
from xflow_amd.engine import Engine


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--batch", type=int, default=262144)
    ap.add_argument("--log2-cap", type=int, default=31)
    ap.add_argument("--load", type=float, default=0.47)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    synth = SynthConfig(total_features=1_000_000_000, hash_space=1_000_000_000, seed=1234)
    engs, gens = [], []
    for r in range(2):
        e = Engine(ModelConfig(kind="lr"), OptimConfig(),
                   EngineConfig(table_log2_cap=a.log2_cap, max_rows=a.batch,
                                max_nnz=a.batch * synth.fields, monitor_lag=7), device=dev)
        e.prefill(int(a.load * 2 ** a.log2_cap), seed=0x5eed + r)
        engs.append(e)
        gens.append(SyntheticCriteo(e, a.batch, synth, rank=r))
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]

    def run(concurrent: bool, steps: int) -> float:
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(steps):
            for r in range(2):
                with torch.cuda.stream(streams[r] if concurrent else streams[0]):
                    engs[r].train_view(gens[r].next())
        torch.cuda.synchronize(dev)
        return time.perf_counter() - t0

    for conc in (False, True):
        run(conc, 5)  # warmup
    out = {}
    for rep in range(2):
        for conc in (False, True):
            dt = run(conc, a.steps)
            key = "concurrent" if conc else "serial"
            out.setdefault(key, []).append(round(2 * a.steps * a.batch / dt / 1e6, 1))
    print(json.dumps({"M_samples_per_s": out, "steps_per_engine": a.steps,
                      "log2_cap": a.log2_cap, "batch": a.batch}))


if __name__ == "__main__":
    main()
