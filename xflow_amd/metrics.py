"""Metrics: the reference's AUC / logloss printer, device-side AUC for large
evaluations, and a JSON-lines metrics logger.

Reference printer (src/base/base.h:84-110): sort by pctr descending, rank-sum
AUC, "logloss" = signed mean log2-likelihood accumulated in float, printed as
``logloss: <x>\\tauc = <a>\\ttp = <T> fp = <F>`` (or ``tp_n = T`` when one class
is absent).  ``reference_auc`` runs the native C++ reproduction of it.
"""
from __future__ import annotations

import json
import os
import time
from typing import Optional

import numpy as np
import torch

from xflow_amd import native


def reference_auc(labels, pctr) -> dict:
    """Exact reference printer semantics (native, host)."""
    lab = np.ascontiguousarray(np.asarray(labels).astype(np.int32))
    p = np.ascontiguousarray(np.asarray(pctr, dtype=np.float32))
    return native.load().reference_auc(lab, p)


def device_auc(labels: torch.Tensor, pctr: torch.Tensor) -> dict:
    """AUC + ln-logloss on the device (torch sort / cumsum), any size.

    Ties are broken by the sort order, like the reference's unstable sort.
    """
    y = labels.float().flatten()
    p = pctr.float().flatten()
    n = y.numel()
    if n == 0:
        return {"auc": float("nan"), "ln_logloss": float("nan"), "n": 0}
    order = torch.argsort(p, descending=True)
    ys = y[order]
    tp = torch.cumsum(ys, 0)
    area = ((1.0 - ys) * tp).sum().double()
    npos = ys.sum().double()
    nneg = n - npos
    auc = (area / (npos * nneg)).item() if npos > 0 and nneg > 0 else float("nan")
    pc = p.clamp(1e-7, 1 - 1e-7).double()
    ll = -(y.double() * torch.log(pc) + (1 - y.double()) * torch.log1p(-pc)).mean().item()
    return {"auc": auc, "ln_logloss": ll, "n": int(n), "positives": int(npos.item())}


class MetricsLogger:
    """Append-only JSON-lines metrics (one object per record)."""

    def __init__(self, path: Optional[str], rank: int = 0):
        self.path = path if (path and rank == 0) else None
        self.t0 = time.time()
        if self.path:
            os.makedirs(os.path.dirname(os.path.abspath(self.path)), exist_ok=True)

    def log(self, **rec) -> None:
        if not self.path:
            return
        rec.setdefault("time", round(time.time() - self.t0, 6))
        with open(self.path, "a") as f:
            f.write(json.dumps(rec) + "\n")


class StepTimer:
    """Samples/s over a window of steps (device-synchronised on read)."""

    def __init__(self, device: torch.device):
        self.device = device
        self.reset()

    def reset(self) -> None:
        self.t = time.perf_counter()
        self.samples = 0
        self.steps = 0

    def add(self, samples: int) -> None:
        self.samples += samples
        self.steps += 1

    def rate(self) -> float:
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        dt = time.perf_counter() - self.t
        return self.samples / dt if dt > 0 else 0.0
