"""Engine (native C++ CPU backend and gfx950 HIP backend) vs the plain PyTorch
fp32 reference step (xflow_amd/testing/torch_ref.py), for every model family,
both optimizers, single- and multi-slice batches."""
import numpy as np
import pytest
import torch

from helpers import random_csr, to_batch
from xflow_amd.config import EngineConfig, ModelConfig, OptimConfig
from xflow_amd.engine import Engine
from xflow_amd.testing import torch_ref
from xflow_amd.testing.hashing import normal_init

CASES = [
    ("lr", "ftrl", "reference", "compat", 1),
    ("lr", "ftrl", "reference", "compat", 4),
    ("lr", "sgd", "reference", "compat", 1),
    ("fm", "ftrl", "reference", "compat", 1),
    ("fm", "ftrl", "standard", "compat", 3),
    ("fm", "sgd", "standard", "compat", 1),
    ("mvm", "ftrl", "reference", "compat", 1),
    ("mvm", "ftrl", "reference", "fixed", 2),
]


def _batch(layout, rows, step, fields=6):
    """CSR (variable rows) or fixed-width rows stored row-major / field-major."""
    fixed = layout != "csr"
    keys, rp, fg, lab = random_csr(rows, fields=fields, vocab=60, seed=100 + step,
                                   variable=not fixed)
    return keys, rp, fg, lab


def _run(device, kind, opt, fm_math, mvm_math, slices, steps=3, rows=96, v_dim=4,
         layout="csr", fields=6, v_scale=1e-2):
    m = ModelConfig(kind=kind, v_dim=v_dim, fm_math=fm_math, mvm_math=mvm_math)
    o = OptimConfig(kind=opt, v_init_scale=v_scale)
    eng = Engine(m, o, EngineConfig(table_log2_cap=14, max_rows=rows, max_nnz=rows * 16,
                                    max_slices=slices), device=device)
    P = m.params_per_key
    ref = torch_ref.RefTable(P, 0 if kind == "mvm" else 1, opt,
                             init_fn=lambda k, d: normal_init(k, d) * np.float32(v_scale))
    slice_rows = rows // slices
    for step in range(steps):
        keys, rp, fg, lab = _batch(layout, rows, step, fields)
        b = to_batch(keys, rp, fg, lab, device, slice_rows=slice_rows)
        if layout != "csr":
            b.row_ptr, b.nnz_per_row = None, fields
            if layout == "field":
                b = b.to_field_major()
        eng.train_step(b)
        torch_ref.train_step(ref, kind, keys, lab, rp, slice_rows, fg, fm_math, mvm_math)
    # all keys seen
    allk = np.unique(np.concatenate([_batch(layout, rows, s, fields)[0] for s in range(steps)]))
    got = eng.pull(allk)
    want = ref.weights(allk, insert=False).numpy()
    assert eng.table_size() == len(allk)
    return got, want, eng


@pytest.mark.parametrize("kind,opt,fm_math,mvm_math,slices", CASES)
def test_engine_matches_torch_reference_cpu(kind, opt, fm_math, mvm_math, slices):
    got, want, _ = _run(torch.device("cpu"), kind, opt, fm_math, mvm_math, slices)
    np.testing.assert_allclose(got, want, rtol=2e-4, atol=2e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("kind,opt,fm_math,mvm_math,slices", CASES)
def test_engine_matches_torch_reference_gpu(gpu_device, kind, opt, fm_math, mvm_math, slices):
    got, want, eng = _run(gpu_device, kind, opt, fm_math, mvm_math, slices)
    assert eng.is_gpu and eng.backend_name.startswith("hip:gfx950")
    np.testing.assert_allclose(got, want, rtol=2e-4, atol=2e-6)


LAYOUT_CASES = [
    ("lr", "ftrl", "reference", "compat", 1, "field"),
    ("lr", "ftrl", "reference", "compat", 4, "field"),
    ("lr", "sgd", "reference", "compat", 1, "fixed"),
    ("fm", "ftrl", "standard", "compat", 3, "field"),
    ("mvm", "ftrl", "reference", "fixed", 2, "field"),
]


@pytest.mark.parametrize("kind,opt,fm_math,mvm_math,slices,layout", LAYOUT_CASES)
def test_fixed_width_layouts_cpu(kind, opt, fm_math, mvm_math, slices, layout):
    got, want, _ = _run(torch.device("cpu"), kind, opt, fm_math, mvm_math, slices,
                        layout=layout)
    np.testing.assert_allclose(got, want, rtol=2e-4, atol=2e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("kind,opt,fm_math,mvm_math,slices,layout", LAYOUT_CASES)
def test_fixed_width_layouts_gpu(gpu_device, kind, opt, fm_math, mvm_math, slices, layout):
    got, want, _ = _run(gpu_device, kind, opt, fm_math, mvm_math, slices, layout=layout)
    np.testing.assert_allclose(got, want, rtol=2e-4, atol=2e-6)


# MVM with O(1) latent init and few fields: the field product stays far from
# zero, so the gradients are large enough to move the weights (with the default
# 1e-2 init, FTRL's L1 zeroes every touched v after its first update and the
# comparison above could not see a wrong MVM gradient).  Covers the GPU
# reduction path (dup-free rows: (dest, row) records; rows with a repeated
# field in the CSR layout: atomics).
MVM_LIVE = [("compat", 1, "csr"), ("fixed", 2, "csr"), ("compat", 1, "field"),
            ("fixed", 1, "fixed")]


def _mvm_live(device, mvm_math, slices, layout):
    got, want, _ = _run(device, "mvm", "ftrl", "reference", mvm_math, slices, layout=layout,
                        fields=4, v_scale=1.0)
    assert np.abs(want).max() > 1e-2  # the weights did move
    np.testing.assert_allclose(got, want, rtol=1e-3, atol=1e-5)


@pytest.mark.parametrize("mvm_math,slices,layout", MVM_LIVE)
def test_mvm_live_gradients_cpu(mvm_math, slices, layout):
    _mvm_live(torch.device("cpu"), mvm_math, slices, layout)


@pytest.mark.gpu
@pytest.mark.parametrize("mvm_math,slices,layout", MVM_LIVE)
def test_mvm_live_gradients_gpu(gpu_device, mvm_math, slices, layout):
    _mvm_live(gpu_device, mvm_math, slices, layout)


@pytest.mark.gpu
def test_gpu_matches_cpu_backend_eval(gpu_device):
    """Predictions of the HIP engine equal the CPU engine's after training."""
    outs = []
    for dev in (torch.device("cpu"), gpu_device):
        eng = Engine(ModelConfig(kind="fm", v_dim=8), OptimConfig(),
                     EngineConfig(table_log2_cap=14, max_rows=256, max_nnz=4096, max_slices=1),
                     device=dev)
        for s in range(4):
            k, rp, fg, lab = random_csr(256, 8, 200, seed=s)
            eng.train_step(to_batch(k, rp, fg, lab, dev))
        k, rp, fg, lab = random_csr(256, 8, 200, seed=99)
        outs.append(eng.eval_step(to_batch(k, rp, fg, lab, dev)).cpu().numpy())
    np.testing.assert_allclose(outs[0], outs[1], rtol=1e-4, atol=1e-6)


def test_slice_normalisation_f32_division_equals_reference_double():
    """The apply kernels normalise a float gradient sum by the slice's row count
    with an f32 division (kernels_table.hip norm_grad); the reference divides
    in double and rounds to float (lr_worker.cc:116-118).  Double rounding is
    innocuous for division when the wide format has >= 2p+2 bits, so both give
    the same float for rows < 2^24 -- checked here on random and edge values."""
    rng = np.random.default_rng(7)
    x = np.concatenate([
        rng.standard_normal(200_000).astype(np.float32) * np.float32(10.0) ** rng.integers(-30, 30, 200_000).astype(np.float32),
        np.array([0.0, -0.0, 1e-45, -1e-45, 1.17549435e-38, 3.4028235e38, -3.4028235e38], np.float32),
    ]).astype(np.float32)
    x = x[np.isfinite(x)]
    for n in [1, 2, 3, 7, 10, 25, 200, 4095, 32768, 262143, 262144, (1 << 24) - 1]:
        f32 = x / np.float32(n)
        f64 = (x.astype(np.float64) / np.float64(n)).astype(np.float32)
        assert np.array_equal(f32.view(np.uint32), f64.view(np.uint32)), n


# v_dim the device kernels are not compiled for runs padded to the next
# compiled width (ModelSpec::pad_dim): the padded dims must stay inert.  MVM
# with O(1) init and few fields so its products (and gradients) are live.
ODD_VDIM = [("fm", "reference", "compat", d, 1, "csr", 1e-2) for d in (3, 5, 9, 12)] + \
    [("fm", "standard", "compat", d, 3, "field", 1e-2) for d in (3, 9)] + \
    [("mvm", "reference", "fixed", d, 1, "field", 1.0) for d in (3, 5, 9, 12)]


def _odd(device, kind, fm_math, mvm_math, v_dim, slices, layout, v_scale):
    got, want, eng = _run(device, kind, "ftrl", fm_math, mvm_math, slices, v_dim=v_dim,
                          layout=layout, fields=4 if kind == "mvm" else 6, v_scale=v_scale)
    assert got.shape[1] == (1 + v_dim if kind == "fm" else v_dim)
    np.testing.assert_allclose(got, want, rtol=1e-3, atol=1e-5)
    return eng


@pytest.mark.parametrize("kind,fm_math,mvm_math,v_dim,slices,layout,v_scale", ODD_VDIM[:2])
def test_odd_v_dim_cpu(kind, fm_math, mvm_math, v_dim, slices, layout, v_scale):
    _odd(torch.device("cpu"), kind, fm_math, mvm_math, v_dim, slices, layout, v_scale)


@pytest.mark.gpu
@pytest.mark.parametrize("kind,fm_math,mvm_math,v_dim,slices,layout,v_scale", ODD_VDIM)
def test_odd_v_dim_gpu(gpu_device, kind, fm_math, mvm_math, v_dim, slices, layout, v_scale):
    """The GPU matches torch_ref for v_dim in {3, 5, 9, 12} (kernels at 4, 8,
    10, 16); the engine reports the padded kernel width in its row stride."""
    eng = _odd(gpu_device, kind, fm_math, mvm_math, v_dim, slices, layout, v_scale)
    p = (1 + v_dim) if kind == "fm" else v_dim
    assert eng.pstride >= p
