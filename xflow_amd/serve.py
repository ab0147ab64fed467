"""Inference from a trained model: ``Predictor`` (batch / online scoring from a
checkpoint) and a small HTTP service around it.

The reference only predicts inside its training job: rank 0 scores the test
file after the last epoch (lr_worker.cc:40-98, fm_worker.cc:40-122) and the
weights die with the servers (ftrl.h:84,151).  Here a checkpoint
(xflow_amd/checkpoint.py, any world size) is loaded into ONE engine -- its
HBM table holds every shard -- and rows are scored by the same forward
kernels the trainer's evaluation uses (keys looked up, never inserted; an
unseen key scores with the weight its pull would have: 0 for w, the lazy
N(0,1)*scale init for latent factors, ftrl.h:110-122).

    p = Predictor("ckpt/")                     # or a versioned root (LATEST)
    p.predict_libffm(open("test-00000", "rb").read())   -> np.float32 [rows]
    p.predict_csr(keys_u64, row_ptr)                      -> np.float32 [rows]

    python -m xflow_amd.serve --checkpoint ckpt/ --port 8080
        POST /predict {"libffm": "1 1:123:1 2:456:1\\n..."}
                   or {"keys": [[k, ...], ...]}  -> {"pctr": [...]}
        GET  /health

Rows are scored in batches of ``max_rows``; one engine serves requests one
at a time (a lock around the device work).
"""
from __future__ import annotations

import argparse
import glob
import math
import os
import threading
from typing import Optional, Sequence

import numpy as np
import torch

from xflow_amd import checkpoint
from xflow_amd import native as _native
from xflow_amd.config import EngineConfig, ModelConfig, OptimConfig
from xflow_amd.engine import Batch, Engine


def _resolve(path: str) -> str:
    """A checkpoint directory, or a versioned root whose LATEST names one."""
    if os.path.exists(os.path.join(path, "meta.json")):
        return path
    d = checkpoint.latest(path)
    if d is None:
        raise FileNotFoundError(f"{path}: no checkpoint (meta.json or LATEST)")
    return d


def _fields(cls, d: dict):
    names = {f.name for f in cls.__dataclass_fields__.values()}
    return cls(**{k: v for k, v in d.items() if k in names})


class Predictor:
    """Scores rows with a model loaded from a checkpoint (see module doc)."""

    def __init__(self, ckpt: str, device: Optional[torch.device] = None, max_rows: int = 65536,
                 max_nnz_per_row: int = 64):
        self.ckpt = _resolve(ckpt)
        meta = checkpoint.load_meta(self.ckpt)
        self.model = _fields(ModelConfig, meta["model"])
        self.optim = _fields(OptimConfig, meta["optim"])
        self.meta = meta
        # (key counts from the shard headers: nothing else is read twice)
        n_keys = sum(checkpoint.shard_keys(p) for p in glob.glob(
            os.path.join(self.ckpt, "shard-*-of-%05d.xftb" % int(meta["world"]))))
        # every shard's keys in one table at load <= 0.5 (no growth while serving)
        lg = max(16, int(math.ceil(math.log2(max(2 * n_keys, 1)))))
        if device is None:
            device = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
        self.device = device
        self.max_rows = int(max_rows)
        self.engine = Engine(self.model, self.optim,
                             EngineConfig(table_log2_cap=lg, max_rows=self.max_rows,
                                          max_nnz=self.max_rows * int(max_nnz_per_row),
                                          table_grow=False),
                             device=device)
        checkpoint.load(self.engine, self.ckpt, 0, 1)
        self.keys = self.engine.table_size()
        self._lock = threading.Lock()

    # ---------------------------------------------------------------- scoring
    def predict_csr(self, keys: np.ndarray, row_ptr: np.ndarray,
                    fgid: Optional[np.ndarray] = None) -> np.ndarray:
        """pctr of every row of a CSR batch (keys u64, row_ptr rows+1 offsets;
        fgid: the field ids MVM groups by -- required for an MVM model, whose
        field products would be wrong with every feature in one field)."""
        keys = np.ascontiguousarray(keys).view(np.uint64)
        row_ptr = np.asarray(row_ptr, dtype=np.int64)
        rows = len(row_ptr) - 1
        if rows < 0 or row_ptr[0] != 0 or row_ptr[-1] != len(keys):
            raise ValueError("row_ptr must hold rows+1 offsets from 0 to len(keys)")
        if fgid is None:
            if self.model.kind == "mvm":
                raise ValueError("an MVM model groups features by field: give the field ids "
                                 "(fgid / 'fields') with the keys")
            fgid = np.zeros(len(keys), np.int32)
        elif len(fgid) != len(keys):
            raise ValueError("fgid must hold one field id per key")
        out = np.empty(rows, np.float32)
        cap_nnz = self.engine.cfg.max_nnz
        r = 0
        with self._lock:
            while r < rows:
                r1 = min(rows, r + self.max_rows)
                while r1 > r + 1 and row_ptr[r1] - row_ptr[r] > cap_nnz:
                    r1 = r + (r1 - r) // 2
                k0, k1 = int(row_ptr[r]), int(row_ptr[r1])
                if k1 - k0 > cap_nnz:
                    raise ValueError(f"row {r} has more than {cap_nnz} features")
                dev = self.device
                b = Batch(keys=torch.from_numpy(keys[k0:k1].view(np.int64)).to(dev),
                          labels=torch.zeros(r1 - r, dtype=torch.float32, device=dev),
                          row_ptr=torch.from_numpy((row_ptr[r:r1 + 1] - k0).astype(np.int32)).to(dev),
                          fgid=torch.from_numpy(np.ascontiguousarray(fgid[k0:k1], np.int32)).to(dev),
                          slice_rows=r1 - r)
                out[r:r1] = self.engine.eval_step(b).cpu().numpy()
                r = r1
        return out

    def predict_libffm(self, text: bytes) -> np.ndarray:
        """pctr of every line of libffm text (``label fgid:fid:val ...``; the
        features hashed like the training reader, csrc/io/reader.cpp)."""
        if isinstance(text, str):
            text = text.encode()
        if text and not text.endswith(b"\n"):
            text += b"\n"
        blk = _native.load().parse_libffm(text)
        return self.predict_csr(np.asarray(blk["keys"]).view(np.uint64),
                                np.asarray(blk["row_ptr"], np.int64), np.asarray(blk["fgid"]))

    def predict_keys(self, rows: Sequence[Sequence[int]],
                     fields: Optional[Sequence[Sequence[int]]] = None) -> np.ndarray:
        """pctr of rows given as lists of (already hashed) u64 keys, with the
        keys' field ids (same shape; required for MVM)."""
        lens = np.array([len(r) for r in rows], np.int64)
        rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
        keys = (np.array([k for r in rows for k in r], dtype=np.uint64) if len(rp) > 1 and rp[-1]
                else np.zeros(0, np.uint64))
        fg = None
        if fields is not None:
            if [len(f) for f in fields] != lens.tolist():
                raise ValueError("'fields' must give one field id per key of every row")
            fg = np.array([g for f in fields for g in f], dtype=np.int32)
        return self.predict_csr(keys, rp, fg)


# -------------------------------------------------------------------- service
def make_app(pred: Predictor):
    """FastAPI app: POST /predict, GET /health."""
    from fastapi import FastAPI, HTTPException
    from pydantic import create_model

    # (built with explicit types: this module's postponed annotations would
    # leave FastAPI a string to resolve in a function scope)
    Req = create_model("PredictRequest", libffm=(Optional[str], None),
                       keys=(Optional[list[list[int]]], None),
                       fields=(Optional[list[list[int]]], None))

    app = FastAPI(title="xflow-amd predictor")

    @app.get("/health")
    def health():
        return {"status": "ok", "model": pred.model.kind, "keys": int(pred.keys),
                "device": str(pred.device), "checkpoint": pred.ckpt}

    def predict(req):
        if (req.libffm is None) == (req.keys is None):
            raise HTTPException(400, "give exactly one of 'libffm' or 'keys'")
        try:
            p = (pred.predict_libffm(req.libffm) if req.libffm is not None
                 else pred.predict_keys(req.keys, req.fields))
        except ValueError as e:
            raise HTTPException(400, str(e))
        return {"pctr": [float(x) for x in p]}

    predict.__annotations__ = {"req": Req}
    app.post("/predict")(predict)
    return app


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="python -m xflow_amd.serve", description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--checkpoint", required=True)
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=8080)
    ap.add_argument("--cpu", action="store_true")
    ap.add_argument("--max-rows", type=int, default=65536)
    a = ap.parse_args(argv)
    pred = Predictor(a.checkpoint, device=torch.device("cpu") if a.cpu else None,
                     max_rows=a.max_rows)
    import uvicorn

    uvicorn.run(make_app(pred), host=a.host, port=a.port, log_level="warning")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
