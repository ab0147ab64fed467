"""The 8-rank sharded step at bench scale on one device (loopback transport,
xflow_amd/parallel/loopback.py): W = 8 virtual ranks x 32 768 rows x 39
Criteo-shaped fields x 5 pipelined steps (hot keys arrive at their owners from
every source), through the owner-partitioned 8-range dedup, the counts
exchange carried with the values, the owner pull of all sources' keys, the
owner grouping and the one-launch multi-source apply.

* bitwise reproducible run to run (fixed-point gradient sums, ordered
  per-source apply), and
* equal (rtol 1e-4) to ONE engine trained on the concatenated batches as 8
  ordered slices -- the lock-step serialisation of the reference's
  asynchronous workers (lr_worker.cc:170-175, ftrl.h:54-80).

A CPU variant at a reduced shape runs in the default suite."""
import numpy as np
import pytest
import torch

from xflow_amd.config import EngineConfig, ModelConfig, OptimConfig
from xflow_amd.data.synth import SynthConfig, SyntheticCriteo
from xflow_amd.engine import Batch, Engine
from xflow_amd.parallel.loopback import LoopbackBus, loopback_engine, run_ranks
from xflow_amd.testing.hashing import owner_of


def _mk(dev, kind, rows, log2_cap, slices=1):
    return Engine(ModelConfig(kind=kind, v_dim=4), OptimConfig(),
                  EngineConfig(table_log2_cap=log2_cap, max_rows=rows, max_nnz=rows * 39,
                               max_slices=slices), device=dev)


def _batches(W, rows, steps):
    """Per (rank, step) field-major synthetic batches (host tensors)."""
    gen_eng = Engine(ModelConfig(), OptimConfig(),
                     EngineConfig(table_log2_cap=10, max_rows=rows, max_nnz=rows * 39))
    cfg = SynthConfig(seed=4242)
    out = []
    for r in range(W):
        g = SyntheticCriteo(gen_eng, rows, cfg, rank=r)
        row = []
        for s in range(steps):
            b = g.alloc_batch()
            g.next(out=b)
            row.append(b)
        out.append(row)
    return out


def _to(dev, b):
    return Batch(keys=b.keys.to(dev), labels=b.labels.to(dev), nnz_per_row=b.nnz_per_row,
                 field_major=True)


def _run_w(dev, kind, data, rows, log2_cap):
    W, steps = len(data), len(data[0])
    engines = [_mk(dev, kind, rows, log2_cap) for _ in range(W)]
    bus = LoopbackBus(W)
    sh = [loopback_engine(bus, r, engines[r]) for r in range(W)]

    def fn(r):
        bs = [_to(dev, b) for b in data[r]]
        for s in range(steps):
            nxt = bs[s + 1] if s + 1 < steps else None
            assert sh[r].train_step(bs[s], S=1, next_batch=nxt)

    run_ranks(bus, fn)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    keys, vals = [], []
    for r, e in enumerate(engines):
        assert not e.overflowed()
        k, _ = e.export_table()
        assert (owner_of(k, W) == r).all()
        o = np.argsort(k)
        keys.append(k[o])
        vals.append(e.pull(k[o]))
    inline = [x.inline_prepares for x in sh]
    return np.concatenate(keys), np.concatenate(vals), inline


def _replay(dev, kind, data, rows, log2_cap):
    """One engine, each step = the W ranks' batches concatenated as W slices."""
    W, steps = len(data), len(data[0])
    ref = _mk(dev, kind, W * rows, log2_cap + 3, slices=W)
    for s in range(steps):
        keys = torch.cat([data[r][s].keys.view(39, rows) for r in range(W)], dim=1).reshape(-1)
        lab = torch.cat([data[r][s].labels for r in range(W)])
        ref.train_step(Batch(keys=keys.contiguous().to(dev), labels=lab.to(dev), nnz_per_row=39,
                             field_major=True, slice_rows=rows))
    return ref


def _check(dev, kind, W, rows, steps, log2_cap):
    data = _batches(W, rows, steps)
    k1, v1, inline = _run_w(dev, kind, data, rows, log2_cap)
    assert inline == [1] * W  # every later batch was prepared inside the previous step
    k2, v2, _ = _run_w(dev, kind, data, rows, log2_cap)
    np.testing.assert_array_equal(k1, k2)
    np.testing.assert_array_equal(v1.view(np.uint32), v2.view(np.uint32))  # bitwise
    ref = _replay(dev, kind, data, rows, log2_cap)
    assert ref.table_size() == len(k1) == len(np.unique(k1))
    np.testing.assert_allclose(v1, ref.pull(k1), rtol=1e-4, atol=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["lr", "fm"])
def test_w8_bench_scale_loopback_gpu(gpu_device, kind):
    _check(gpu_device, kind, W=8, rows=32768, steps=5, log2_cap=22)


def test_w4_loopback_cpu():
    _check(torch.device("cpu"), "lr", W=4, rows=512, steps=3, log2_cap=16)
