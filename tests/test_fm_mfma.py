"""Standard-math FM forward on the matrix cores (k_fm_fwd_mfma,
v_mfma_f32_16x16x4_f32) against the VALU forward and an fp32 torch reference
of the same op (xflow_amd/testing/torch_ref.forward, fm_math="standard")."""
import numpy as np
import pytest
import torch

from helpers import random_csr, to_batch
from xflow_amd.config import EngineConfig, ModelConfig, OptimConfig
from xflow_amd.engine import Engine
from xflow_amd.testing import torch_ref

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("v_dim,variable", [(8, False), (4, True), (8, True)])
def test_fm_mfma_forward_matches_valu_and_torch(gpu_device, v_dim, variable):
    rows = 1000  # not a multiple of 16: partial row tiles
    engines = [Engine(ModelConfig(kind="fm", v_dim=v_dim, fm_math="standard", fm_mfma=m),
                      OptimConfig(v_init_scale=0.5),
                      EngineConfig(table_log2_cap=16, max_rows=rows, max_nnz=rows * 24),
                      device=gpu_device) for m in (False, True)]
    for step in range(3):  # identical training (the training path is VALU in both)
        k, rp, fg, lab = random_csr(rows, 12, 400, seed=70 + step, variable=variable)
        for e in engines:
            e.train_step(to_batch(k, rp, fg, lab, gpu_device))
    k, rp, fg, lab = random_csr(rows, 12, 500, seed=99, variable=variable)
    b = to_batch(k, rp, fg, lab, gpu_device)
    p_valu, p_mfma = (e.eval_step(b).cpu() for e in engines)
    # fp32 torch reference of the same forward from the pulled weights
    uk, inv = np.unique(k, return_inverse=True)
    W = torch.from_numpy(engines[0].pull(uk))
    row_of = torch.from_numpy(np.repeat(np.arange(rows), np.diff(rp)))
    y, _ = torch_ref.forward("fm", W, torch.from_numpy(inv), row_of, rows, fm_math="standard")
    want = torch_ref.sigmoid_ref(y)
    assert float(p_valu.std()) > 1e-3  # the interaction is live
    torch.testing.assert_close(p_mfma, p_valu, rtol=2e-5, atol=2e-6)
    torch.testing.assert_close(p_mfma, want, rtol=1e-4, atol=1e-5)
    sv, sm = (e.read_stats(which=1) for e in engines)
    assert sv["rows"] == sm["rows"] == rows
