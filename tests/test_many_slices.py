"""Steps of more than 32 Hogwild slices (the reference's default slice count is
std::thread::hardware_concurrency(), lr_worker.h:40-41 / lr_worker.cc:190-199,
well above 32 on an MI355X host).  The engine runs such a step as groups of 32
slices over one dedup + pull (Engine::slice_groups); the result must equal an
S-slice step: every slice reads the same pulled weights and the pushes are
applied per key in global slice order -- checked against the plain PyTorch
fp32 reference (xflow_amd/testing/torch_ref.py), for every model family, on
the native CPU backend and the HIP backend, single-rank and sharded."""
import numpy as np
import pytest
import torch

from helpers import random_csr, to_batch
from xflow_amd.config import EngineConfig, ModelConfig, OptimConfig
from xflow_amd.engine import Engine
from xflow_amd.testing import torch_ref
from xflow_amd.testing.hashing import normal_init

CASES = [
    # kind, opt, fm_math, mvm_math, slices, v_scale, layout
    ("lr", "ftrl", "reference", "compat", 33, 1e-2, "csr"),
    ("lr", "ftrl", "reference", "compat", 64, 1e-2, "field"),
    ("lr", "sgd", "reference", "compat", 40, 1e-2, "csr"),
    ("fm", "ftrl", "reference", "compat", 33, 1e-2, "csr"),
    ("fm", "ftrl", "reference", "compat", 64, 1e-2, "field"),
    ("fm", "ftrl", "standard", "compat", 33, 1e-2, "csr"),
    ("fm", "ftrl", "standard", "compat", 64, 1e-2, "field"),
    ("mvm", "ftrl", "reference", "compat", 33, 1.0, "csr"),
    ("mvm", "ftrl", "reference", "fixed", 64, 1.0, "field"),
]


def run(device, kind, opt, fm_math, mvm_math, slices, v_scale, layout, rows_per_slice=3,
        steps=3, v_dim=4, fields=5):
    rows = slices * rows_per_slice
    m = ModelConfig(kind=kind, v_dim=v_dim, fm_math=fm_math, mvm_math=mvm_math)
    o = OptimConfig(kind=opt, v_init_scale=v_scale)
    eng = Engine(m, o, EngineConfig(table_log2_cap=14, max_rows=rows, max_nnz=rows * 16,
                                    max_slices=slices), device=device)
    ref = torch_ref.RefTable(m.params_per_key, 0 if kind == "mvm" else 1, opt,
                             init_fn=lambda k, d: normal_init(k, d) * np.float32(v_scale))
    allk = []
    for step in range(steps):
        keys, rp, fg, lab = random_csr(rows, fields=fields, vocab=40, seed=500 + step,
                                       variable=layout == "csr")
        allk.append(keys)
        b = to_batch(keys, rp, fg, lab, device, slice_rows=rows_per_slice)
        if layout != "csr":
            b.row_ptr, b.nnz_per_row = None, fields
            b = b.to_field_major()
        assert eng.slices_of(b) == slices
        eng.train_step(b)
        torch_ref.train_step(ref, kind, keys, lab, rp, rows_per_slice, fg, fm_math, mvm_math)
    allk = np.unique(np.concatenate(allk))
    return eng.pull(allk), ref.weights(allk, insert=False).numpy()


def test_slice_groups_layout():
    assert Engine.slice_groups(1) == [1]
    assert Engine.slice_groups(32) == [32]
    assert Engine.slice_groups(33) == [32, 2]   # a one-slice group runs masked, as two
    assert Engine.slice_groups(64) == [32, 32]
    assert Engine.slice_groups(256) == [32] * 8
    assert Engine.slice_groups(70) == [32, 32, 6]


@pytest.mark.parametrize("case", CASES, ids=lambda c: "-".join(map(str, c)))
def test_many_slices_match_torch_reference_cpu(case):
    got, want = run(torch.device("cpu"), *case)
    assert np.abs(want).max() > 0
    np.testing.assert_allclose(got, want, rtol=1e-3, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=lambda c: "-".join(map(str, c)))
def test_many_slices_match_torch_reference_gpu(gpu_device, case):
    got, want = run(gpu_device, *case)
    assert np.abs(want).max() > 0
    np.testing.assert_allclose(got, want, rtol=1e-3, atol=1e-5)


def test_sum_slices_rejects_slice_groups():
    eng = Engine(ModelConfig(kind="lr"), OptimConfig(),
                 EngineConfig(table_log2_cap=12, max_rows=128, max_nnz=1024, max_slices=64,
                              sum_slices=True), device=torch.device("cpu"))
    keys, rp, fg, lab = random_csr(128, fields=4, vocab=30, seed=1)
    with pytest.raises(Exception, match="sum_slices"):
        eng.train_step(to_batch(keys, rp, fg, lab, torch.device("cpu"), slice_rows=2))
