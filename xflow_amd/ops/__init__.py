"""Standalone ops of the engine's math, for users and tests.

* ``feature_hash``: the reference's feature key (std::hash<std::string>,
  load_data_from_disk.cc:154), native.
* ``owner_of``: the rank that owns a key in a W-way sharded table.
* ``sigmoid_ref``: the reference's clamped sigmoid (base.h:54-63), torch.
* ``ftrl_update`` / ``ftrl_weight``: vectorised FTRL-Proximal closed form
  (ftrl.h:58-74) on torch tensors -- the same recipe the table kernels run.
* ``unique_keys``: batch dedup on any device through the engine's scratch
  table (device kernels on GPU).
"""
from __future__ import annotations

import numpy as np
import torch

from xflow_amd import native
from xflow_amd.testing.hashing import owner_of  # noqa: F401
from xflow_amd.testing.torch_ref import sigmoid_ref  # noqa: F401


def feature_hash(text) -> int:
    b = text.encode() if isinstance(text, str) else bytes(text)
    return int(native.load().feature_hash(b))


def ftrl_weight(z: torch.Tensor, n: torch.Tensor, alpha=5e-2, beta=1.0, l1=5e-5, l2=10.0):
    tmpr = torch.where(z > 0, z - l1, torch.where(z < 0, z + l1, torch.zeros_like(z)))
    tmpl = -1.0 * ((beta + torch.sqrt(n)) / alpha + l2)
    return torch.where(z.abs() <= l1, torch.zeros_like(z), tmpr / tmpl)


def ftrl_update(n: torch.Tensor, z: torch.Tensor, g: torch.Tensor, alpha=5e-2, beta=1.0,
                l1=5e-5, l2=10.0):
    """One FTRL-Proximal push; returns (n', z', w')."""
    w = ftrl_weight(z, n, alpha, beta, l1, l2)
    nn = n + g * g
    z2 = z + (g - (torch.sqrt(nn) - torch.sqrt(n)) / alpha * w)
    return nn, z2, ftrl_weight(z2, nn, alpha, beta, l1, l2)


def unique_keys(keys: torch.Tensor) -> torch.Tensor:
    """Unique int64 keys (order unspecified) via the engine's dedup kernels."""
    from xflow_amd.config import EngineConfig, ModelConfig, OptimConfig
    from xflow_amd.engine import Batch, Engine

    n = keys.numel()
    eng = Engine(ModelConfig(), OptimConfig(),
                 EngineConfig(table_log2_cap=4, max_rows=max(n, 1), max_nnz=max(n, 1)),
                 device=keys.device)
    b = Batch(keys=keys.contiguous(), labels=torch.zeros(n, device=keys.device),
              nnz_per_row=1)
    counts = torch.zeros(1, dtype=torch.int64, device=keys.device)
    send = torch.empty(max(n, 1), dtype=torch.int64, device=keys.device)
    eng.w_prepare(b, 1, counts, send)
    return send[: int(counts.item())].clone()
