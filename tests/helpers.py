"""Shared test helpers: random CSR batches with power-law keys."""
from __future__ import annotations

import numpy as np
import torch

from xflow_amd.engine import Batch


def random_csr(rows: int, fields: int = 8, vocab: int = 500, seed: int = 0,
               variable: bool = True, multi_field_max: int = 2):
    """Rows of `fields` fields (field f may repeat up to multi_field_max times);
    returns numpy (keys u64, row_ptr i32, fgid i32, labels f32)."""
    rng = np.random.default_rng(seed)
    keys, fg, rp = [], [], [0]
    for _ in range(rows):
        for f in range(fields):
            reps = rng.integers(1, multi_field_max + 1) if (variable and f >= fields - 2) else 1
            if variable and rng.random() < 0.05:
                reps = 0
            for _ in range(reps):
                z = min(int(rng.zipf(1.3)), vocab)
                keys.append((f * 1_000_003 + z) * 0x9E3779B97F4A7C15 % (1 << 64))
                fg.append(f)
        rp.append(len(keys))
    labels = (rng.random(rows) < 0.3).astype(np.float32)
    return (np.array(keys, dtype=np.uint64), np.array(rp, dtype=np.int32),
            np.array(fg, dtype=np.int32), labels)


def to_batch(keys, row_ptr, fgid, labels, device, slice_rows=0, with_fgid=True) -> Batch:
    return Batch(keys=torch.from_numpy(keys.view(np.int64)).to(device),
                 labels=torch.from_numpy(labels).to(device),
                 row_ptr=torch.from_numpy(row_ptr).to(device),
                 fgid=torch.from_numpy(fgid).to(device) if with_fgid else None,
                 slice_rows=slice_rows)
