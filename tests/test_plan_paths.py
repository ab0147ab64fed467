"""Every gradient layout the step planner (plan_step, csrc/engine/engine.cpp)
can pick, exercised end to end against the plain PyTorch fp32 reference
(xflow_amd/testing/torch_ref.py): each case first asserts which layout the
engine plans for it -- so a routing change shows up here, not as a silent
switch -- then trains 3 steps of random variable-width rows (repeated
fields included) and compares the weights.  The reference semantics are the
per-slice pushes of each slice's keys (lr_worker.cc:162-175,
fm_worker.cc:241-242, mvm_worker.cc:214-218)."""
import numpy as np
import pytest
import torch

from helpers import random_csr, to_batch
from xflow_amd.config import EngineConfig, ModelConfig, OptimConfig
from xflow_amd.engine import Engine
from xflow_amd.testing import torch_ref
from xflow_amd.testing.hashing import normal_init

# kind, fm_math, opt, slices, csr, sum_slices, v_scale -> the planned layout (GPU)
CASES = [
    ("lr", "reference", "ftrl", 1, True, False, 1e-2, "unique_lr"),
    ("lr", "reference", "ftrl", 8, True, False, 1e-2, "csr"),
    ("lr", "reference", "ftrl", 8, False, False, 1e-2, "unique_lr"),
    ("lr", "reference", "ftrl", 8, True, True, 1e-2, "slot_sums"),
    ("lr", "reference", "sgd", 1, True, False, 1e-2, "slot_rows"),
    ("fm", "reference", "ftrl", 1, True, False, 1e-2, "unique_fm_bc"),
    ("fm", "reference", "ftrl", 8, True, False, 1e-2, "csr"),
    ("fm", "reference", "ftrl", 40, False, False, 1e-2, "unique_fm_bc"),
    ("fm", "standard", "ftrl", 1, True, False, 1e-2, "unique_rows"),
    ("fm", "standard", "ftrl", 8, True, False, 1e-2, "csr"),
    ("fm", "standard", "sgd", 8, False, False, 1e-2, "unique_rows"),
    ("mvm", "reference", "ftrl", 1, True, False, 1.0, "unique_rows"),
    ("mvm", "reference", "sgd", 8, True, False, 1.0, "csr"),
    ("mvm", "reference", "ftrl", 8, False, False, 1.0, "slot_rows"),
]


def _run(device, kind, fm_math, opt, slices, csr, sum_slices, v_scale, rows_per_slice=4,
         steps=3, v_dim=4, fields=6):
    rows = slices * rows_per_slice
    m = ModelConfig(kind=kind, v_dim=v_dim, fm_math=fm_math)
    o = OptimConfig(kind=opt, v_init_scale=v_scale)
    eng = Engine(m, o, EngineConfig(table_log2_cap=14, max_rows=rows, max_nnz=rows * 16,
                                    max_slices=slices, sum_slices=sum_slices, csr=csr),
                 device=device)
    plan = eng.native.step_plan(slices)
    ref = torch_ref.RefTable(m.params_per_key, 0 if kind == "mvm" else 1, opt,
                             init_fn=lambda k, d: normal_init(k, d) * np.float32(v_scale))
    allk = []
    for step in range(steps):
        keys, rp, fg, lab = random_csr(rows, fields=fields, vocab=40, seed=900 + step)
        allk.append(keys)
        eng.train_step(to_batch(keys, rp, fg, lab, device, slice_rows=rows_per_slice))
        torch_ref.train_step(ref, kind, keys, lab, rp, rows_per_slice, fg, fm_math,
                             sum_slices=sum_slices)
    allk = np.unique(np.concatenate(allk))
    return plan, eng.pull(allk), ref.weights(allk, insert=False).numpy()


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=lambda c: "-".join(map(str, c)))
def test_planned_layout_matches_torch_reference_gpu(gpu_device, case):
    *args, grad = case
    plan, got, want = _run(gpu_device, *args)
    assert plan["grad"] == grad, plan
    assert np.abs(want).max() > 0
    np.testing.assert_allclose(got, want, rtol=1e-3, atol=1e-5)


def test_every_gpu_layout_is_covered():
    # the cases above reach every layout plan_step can return on the GPU
    assert {c[-1] for c in CASES} == {"csr", "unique_lr", "unique_fm_bc", "unique_rows",
                                      "slot_sums", "slot_rows"}


@pytest.mark.parametrize("case", CASES[:6], ids=lambda c: "-".join(map(str, c)))
def test_cpu_backend_same_weights_as_reference(case):
    # (the CPU backend plans slot rows for all of them; the same numerics)
    *args, _ = case
    plan, got, want = _run(torch.device("cpu"), *args)
    assert plan["grad"] == "slot_rows"
    np.testing.assert_allclose(got, want, rtol=1e-3, atol=1e-5)


@pytest.mark.gpu
def test_mvm_batches_alternating_repeated_fields_gpu(gpu_device):
    """One-slice MVM steps whose batches alternate between rows with a repeated
    field (their gradients reach the unique-order rows by atomics, and the step
    raises FwdArgs::red_dup) and none (the reduction then stores its rows
    without reading them): the same table as the CPU backend, whose MVM is
    checked against torch_ref above.  The flag words alternate per step, so
    the pattern dup, none, none, dup, dup, none covers a flag left over from
    either parity."""
    m = ModelConfig(kind="mvm", v_dim=4)
    o = OptimConfig(kind="sgd", sgd_v_init=0.9)
    engs = [Engine(m, o, EngineConfig(table_log2_cap=12, max_rows=256, max_nnz=256 * 16),
                   device=d) for d in (torch.device("cpu"), gpu_device)]
    assert engs[1].native.step_plan(1)["grad"] == "unique_rows"
    allk = []
    for step, variable in enumerate([True, False, False, True, True, False]):
        keys, rp, fg, lab = random_csr(200, fields=5, vocab=30, seed=70 + step, variable=variable)
        dups = sum(len(set(fg[rp[r]:rp[r + 1]])) < rp[r + 1] - rp[r] for r in range(200))
        assert (dups > 0) == variable
        allk.append(keys)
        for e in engs:
            e.train_step(to_batch(keys, rp, fg, lab, e.device))
    k = np.unique(np.concatenate(allk))
    cpu, gpu = engs[0].pull(k), engs[1].pull(k)
    assert np.abs(cpu).max() > 0
    np.testing.assert_allclose(gpu, cpu, rtol=2e-4, atol=1e-6)
