"""CSR step internals on a small batch: per-key entry counts vs the
(key, slice) pairs present (development probe)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from helpers import random_csr, to_batch  # noqa: E402
from xflow_amd.config import EngineConfig, ModelConfig, OptimConfig  # noqa: E402
from xflow_amd.engine import Engine  # noqa: E402

dev = torch.device("cuda", 0)
for S in [4, 32]:
    rows = 96
    eng = Engine(ModelConfig(kind="lr"), OptimConfig(),
                 EngineConfig(table_log2_cap=14, max_rows=rows, max_nnz=rows * 16, max_slices=S),
                 device=dev)
    keys, rp, fg, lab = random_csr(rows, fields=6, vocab=60, seed=100)
    eng.train_step(to_batch(keys, rp, fg, lab, dev, slice_rows=rows // S))
    off, cnt, words = eng._e.csr_debug()
    # expected pairs
    sr = rows // S
    pairs = {}
    for r in range(rows):
        for j in range(rp[r], rp[r + 1]):
            pairs.setdefault(int(keys[j]), set()).add(r // sr)
    nu = len(pairs)
    print(f"S={S} unique={len(off)} (expected {nu}) sum cnt={int(cnt.sum())} expected "
          f"{sum(len(v) for v in pairs.values())} entries={len(words)//2}")
    print(" cnt hist:", np.bincount(cnt)[:12], " expected:",
          np.bincount([len(v) for v in pairs.values()])[:12])
    print(" first keys off/cnt:", list(zip(off[:8].tolist(), cnt[:8].tolist())))
    ent = words.reshape(-1, 2)
    print(" first entries (slice, value):", [(int(a), float(np.frombuffer(np.uint32(b).tobytes(), np.float32)[0])) for a, b in ent[:12]])
