"""Many-slice steps at bench scale: 32 768 Criteo-shaped rows x 39 fields per
step, 64 and 256 Hogwild slices (the reference's default slice count is
hardware_concurrency, lr_worker.h:40-41; each slice pushes only its own keys,
lr_worker.cc:162-175).  The GPU runs every model on the CSR path
(Engine::train_step_csr: one reduction and one apply of the touched (key,
slice) pairs; full-row entries for standard FM and MVM); every model is
checked against the native CPU backend on the same (bit-identical) synthetic
batches -- the producers' narrow workgroups, widened buckets and multi-window
CSR buckets included."""
import numpy as np
import pytest
import torch

from xflow_amd.config import EngineConfig, ModelConfig, OptimConfig
from xflow_amd.data.synth import SynthConfig, SyntheticCriteo
from xflow_amd.engine import Engine

ROWS = 32768

CASES = [
    # kind, fm_math, v_dim, slices, v_init_scale
    ("lr", "reference", 4, 64, 1e-2),
    ("lr", "reference", 4, 256, 1e-2),
    ("fm", "reference", 8, 64, 1e-2),
    ("fm", "reference", 8, 256, 1e-2),
    ("fm", "standard", 8, 64, 1e-2),
    ("fm", "standard", 8, 256, 1e-2),
    ("mvm", "reference", 4, 64, 1.0),
    ("mvm", "reference", 4, 256, 1.0),
]


def _train(device, kind, fm_math, v_dim, slices, v_scale, steps=3, fields=39, csr=True):
    m = ModelConfig(kind=kind, v_dim=v_dim, fm_math=fm_math, mvm_math="fixed")
    eng = Engine(m, OptimConfig(kind="ftrl", v_init_scale=v_scale),
                 EngineConfig(table_log2_cap=22, max_rows=ROWS, max_nnz=ROWS * fields,
                              max_slices=slices, csr=csr), device=device)
    # (MVM: few fields keep the field products -- and the gradients -- live)
    cfg = SynthConfig(seed=11, n_fields=fields, total_features=10_000_000,
                      hash_space=10_000_000)
    gen = SyntheticCriteo(eng, ROWS, cfg, slice_rows=ROWS // slices)
    b = gen.alloc_batch()
    for _ in range(steps):
        gen.next(out=b)
        assert eng.slices_of(b) == slices
        eng.train_step(b)
    keys, _ = eng.export_table()
    keys = np.sort(keys)
    return eng, keys, eng.pull(keys), eng.read_stats()


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=lambda c: "-".join(map(str, c)))
def test_bench_scale_slices_gpu_equals_cpu(gpu_device, case):
    kind, fm_math, v_dim, slices, v_scale = case
    fields = 6 if kind == "mvm" else 39
    ge, gk, gw, gst = _train(gpu_device, kind, fm_math, v_dim, slices, v_scale, fields=fields)
    _, ck, cw, cst = _train(torch.device("cpu"), kind, fm_math, v_dim, slices, v_scale,
                            fields=fields)
    if kind == "lr" or (kind == "fm" and fm_math == "reference"):
        assert ge.csr_steps == 3, "expected the CSR path"
    np.testing.assert_array_equal(gk, ck)
    assert np.abs(cw).max() > 1e-3
    np.testing.assert_allclose(gw, cw, rtol=2e-4, atol=2e-6)
    np.testing.assert_allclose(gst["ln_loss"], cst["ln_loss"], rtol=1e-5)


@pytest.mark.gpu
def test_csr_step_deterministic(gpu_device):
    """Two identical runs of the CSR path give bit-identical tables (fixed-point
    sums; the entries' order is the dests' order, not the records')."""
    a = _train(gpu_device, "lr", "reference", 4, 256, 1e-2)
    b = _train(gpu_device, "lr", "reference", 4, 256, 1e-2)
    np.testing.assert_array_equal(a[1], b[1])
    np.testing.assert_array_equal(a[2], b[2])


@pytest.mark.gpu
@pytest.mark.parametrize("kind,fm_math,slices", [("lr", "reference", 64), ("lr", "reference", 256),
                                                 ("fm", "reference", 64), ("fm", "reference", 8)])
def test_csr_equals_slice_groups_bitwise(gpu_device, kind, fm_math, slices):
    """The CSR step and the slice-group step (EngineConfig.csr = False) push
    the same floats in the same order: bit-identical tables."""
    a = _train(gpu_device, kind, fm_math, 8, slices, 1e-2)
    b = _train(gpu_device, kind, fm_math, 8, slices, 1e-2, csr=False)
    assert a[0].csr_steps == 3 and b[0].csr_steps == 0
    np.testing.assert_array_equal(a[1], b[1])
    np.testing.assert_array_equal(a[2], b[2])


@pytest.mark.gpu
@pytest.mark.parametrize("kind,fm_math", [("lr", "reference"), ("fm", "reference"),
                                          ("fm", "standard"), ("mvm", "reference")])
def test_csr_steps_with_empty_and_tiny_batches(gpu_device, kind, fm_math):
    """A many-slice CSR step of 0 rows (a rank out of data), of fewer rows
    than slices (empty slices) and of one row per slice all run, leave the
    table consistent with the CPU backend and change nothing for 0 rows."""
    from helpers import random_csr, to_batch

    m = ModelConfig(kind=kind, v_dim=4, fm_math=fm_math)
    o = OptimConfig(kind="sgd", sgd_v_init=0.9) if kind == "mvm" else OptimConfig()
    engs = [Engine(m, o, EngineConfig(table_log2_cap=12, max_rows=256, max_nnz=256 * 16,
                                      max_slices=64), device=d)
            for d in (torch.device("cpu"), gpu_device)]
    assert engs[1].native.step_plan(64)["grad"] == "csr"
    allk = []
    for rows, rps, seed in [(128, 2, 1), (0, 2, 2), (64, 1, 3), (40, 2, 4)]:
        keys, rp, fg, lab = random_csr(rows, fields=5, vocab=30, seed=seed)
        allk.append(keys)
        for e in engs:
            b = to_batch(keys, rp, fg, lab, e.device, slice_rows=rps)
            e.train_step(b)
    k = np.unique(np.concatenate(allk))
    cpu, gpu = engs[0].pull(k), engs[1].pull(k)
    assert np.abs(cpu).max() > 0
    np.testing.assert_allclose(gpu, cpu, rtol=2e-4, atol=1e-6)
    assert engs[0].table_size() == engs[1].table_size()
