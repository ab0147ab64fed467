"""Bench-scale correctness gates on the GPU: the LR-FTRL bench shape (262144
rows x 39 fields, field-major synthetic Criteo batches, LDS pre-dedup chunks,
bucket reduction, pull-time (n, z) stash) over 22 steps including a device
side dedup-scratch rebuild is

* bitwise reproducible run to run (fixed-point gradient sums, see
  csrc/hip/hip_util.h fx_from), and
* equal to the native CPU backend within rtol 1e-4.

The reference keeps the same per-key sums (lr_worker.cc:100-119) in a
sequential float loop; the GPU sums exactly (integers) and rounds once."""
import numpy as np
import pytest
import torch

from xflow_amd.config import EngineConfig, ModelConfig, OptimConfig
from xflow_amd.data.synth import SynthConfig, SyntheticCriteo
from xflow_amd.engine import Batch, Engine

pytestmark = pytest.mark.gpu


def _train(kind, dev, rows, small, steps_small, steps, v_dim=8, gpu_batches=None, S=1):
    fm_math = "standard" if kind == "fm-std" else "reference"
    kind = "fm" if kind == "fm-std" else kind
    eng = Engine(ModelConfig(kind=kind, v_dim=v_dim, fm_math=fm_math), OptimConfig(),
                 EngineConfig(table_log2_cap=23, max_rows=rows, max_nnz=rows * 39, max_slices=S),
                 device=dev)
    caps = []
    # the CPU backend generates the (bit-identical) batches; the GPU trains on copies
    for i, r in enumerate([small] * steps_small + [rows] * (steps - steps_small)):
        b = gpu_batches[i]
        if dev.type == "cuda":
            b = Batch(keys=b.keys.to(dev), labels=b.labels.to(dev), nnz_per_row=b.nnz_per_row,
                      field_major=True, slice_rows=b.slice_rows)
        eng.train_step(b)
        caps.append(eng.scratch_capacity())
    assert not eng.overflowed()
    keys, _ = eng.export_table()
    keys = np.sort(keys)
    return keys, eng.pull(keys), caps, eng.read_stats()


def _batches(rows, small, steps_small, steps, S=1):
    gen_eng = Engine(ModelConfig(), OptimConfig(),
                     EngineConfig(table_log2_cap=10, max_rows=rows, max_nnz=rows * 39))
    out = []
    for i, r in enumerate([small] * steps_small + [rows] * (steps - steps_small)):
        g = SyntheticCriteo(gen_eng, r, SynthConfig(seed=11), slice_rows=r // S)
        g.step = i
        b = g.alloc_batch()
        g.next(out=b)
        out.append(b)
    return out


@pytest.mark.parametrize("kind,rows,small,steps_small,steps,S",
                         [("lr", 262144, 32768, 4, 22, 1), ("fm", 65536, 8192, 3, 8, 1),
                          ("lr", 262144, 32768, 3, 10, 8), ("fm", 65536, 8192, 2, 6, 4),
                          ("fm-std", 65536, 8192, 2, 6, 1), ("fm-std", 65536, 8192, 2, 6, 4)])
def test_bench_scale_deterministic_and_matches_cpu(gpu_device, kind, rows, small, steps_small,
                                                   steps, S):
    """S > 1: the reference's Hogwild slices (lr_worker.cc:190-199) at bench
    scale stay on the atomic-free fixed-point reduction.  fm-std: standard-math
    FM, per-component records through the same reduction (k_fm_std_red)."""
    batches = _batches(rows, small, steps_small, steps, S)
    k1, w1, caps1, st1 = _train(kind, gpu_device, rows, small, steps_small, steps,
                                gpu_batches=batches, S=S)
    k2, w2, caps2, _ = _train(kind, gpu_device, rows, small, steps_small, steps,
                              gpu_batches=batches, S=S)
    # the adaptive scratch grew on the device when the batches got larger
    assert caps1[steps_small] > caps1[0], caps1
    assert caps1 == caps2
    np.testing.assert_array_equal(k1, k2)
    np.testing.assert_array_equal(w1.view(np.uint32), w2.view(np.uint32))  # bitwise
    kc, wc, _, stc = _train(kind, torch.device("cpu"), rows, small, steps_small, steps,
                            gpu_batches=batches, S=S)
    np.testing.assert_array_equal(k1, kc)
    np.testing.assert_allclose(w1, wc, rtol=1e-4, atol=1e-6)
    assert st1["rows"] == stc["rows"]
    assert abs(st1["ln_loss"] - stc["ln_loss"]) <= 1e-5 * abs(stc["ln_loss"])


def _mvm_dup_train(dev, batches, S, optim):
    eng = Engine(ModelConfig(kind="mvm", v_dim=10), optim,
                 EngineConfig(table_log2_cap=20, max_rows=16384, max_nnz=16384 * 24, max_slices=S),
                 device=dev)
    for b in batches:
        if dev.type == "cuda":
            b = Batch(keys=b.keys.to(dev), labels=b.labels.to(dev), row_ptr=b.row_ptr.to(dev),
                      fgid=b.fgid.to(dev), slice_rows=b.slice_rows)
        eng.train_step(b)
    assert not eng.overflowed()
    keys, _ = eng.export_table()
    keys = np.sort(keys)
    return keys, eng.pull(keys), eng.native.step_plan(S)["grad"]


@pytest.mark.parametrize("S", [1, 64])
def test_mvm_repeated_fields_deterministic(gpu_device, S):
    """MVM rows with a repeated field (fields 16-17 hold 1-2 features, like
    the bundled data's multi-valued fields; mvm_worker.cc:137-170: the
    gradient divides by 1 + the FIELD sum) add their gradients in fixed point
    after the reduction (MvmDup): two GPU runs are bitwise equal, and equal
    the CPU backend within rounding -- on the unique-row layout (1 slice) and
    on CSR entries (64 slices)."""
    from helpers import random_csr, to_batch

    optim = OptimConfig(kind="sgd", sgd_v_init=0.9)  # (live products: gradients flow)
    batches = [to_batch(*random_csr(16384, 18, 400, seed=31 + i, variable=True), torch.device("cpu"),
                        slice_rows=16384 // S) for i in range(4)]
    assert (np.diff(batches[0].row_ptr.numpy()) > 18).any()  # rows with repeated fields
    k1, w1, grad = _mvm_dup_train(gpu_device, batches, S, optim)
    assert grad == ("unique_rows" if S == 1 else "csr"), grad
    k2, w2, _ = _mvm_dup_train(gpu_device, batches, S, optim)
    np.testing.assert_array_equal(k1, k2)
    np.testing.assert_array_equal(w1.view(np.uint32), w2.view(np.uint32))  # bitwise
    kc, wc, _ = _mvm_dup_train(torch.device("cpu"), batches, S, optim)
    np.testing.assert_array_equal(k1, kc)
    np.testing.assert_allclose(w1, wc, rtol=1e-4, atol=1e-6)
