"""Common model wrapper: a ModelConfig + an Engine factory + scoring helpers."""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch

from xflow_amd.config import EngineConfig, ModelConfig, OptimConfig
from xflow_amd.engine import Batch, Engine


class SparseModel:
    kind = "lr"

    def __init__(self, v_dim: int = 10, optim: Optional[OptimConfig] = None, **model_kw):
        self.config = ModelConfig(kind=self.kind, v_dim=v_dim, **model_kw)
        self.optim = optim or OptimConfig()

    @property
    def params_per_key(self) -> int:
        return self.config.params_per_key

    def engine(self, device="cpu", **engine_kw) -> Engine:
        """A single-rank engine (HBM table + kernels) for this model."""
        return Engine(self.config, self.optim, EngineConfig(**engine_kw), device=device)

    def predict(self, engine: Engine, batch: Batch) -> torch.Tensor:
        return engine.eval_step(batch)

    def weights(self, engine: Engine, keys) -> np.ndarray:
        """Current pull values [len(keys), params_per_key] (no insertion)."""
        return engine.pull(np.asarray(keys, dtype=np.uint64))
