"""Logistic regression (reference: src/model/lr/lr_worker.{h,cc}).

p = sigmoid(sum_f w_f) with feature values ignored (x = 1, lr_worker.cc:128-138);
loss = p - y; per-key gradient = sum over the slice's occurrences of the loss,
divided by the slice's row count (lr_worker.cc:100-119).  Weights live in the
HBM table as FTRL (n, z) state (w recomputed by the closed form) or SGD w.
"""
from xflow_amd.models.base import SparseModel


class LR(SparseModel):
    kind = "lr"

    def __init__(self, **kw):
        kw.setdefault("v_dim", 1)
        super().__init__(**kw)
