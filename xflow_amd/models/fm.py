"""Factorization machine (reference: src/model/fm/fm_worker.{h,cc}).

Params per key: [w, v_0 .. v_{D-1}], D = v_dim (10 by default, fm_worker.h:92).

fm_math="reference" reproduces fm_worker.cc exactly: vs = sum_k sum_f v_fk
(one scalar over all k), y = sum_f w_f + vs^2 - sum_k sum_f v_fk^2, w gradient
accumulated once per k (x D), v gradient loss * (vs - v_fk).
fm_math="standard" is Rendle's FM: y = sum_f w_f + 1/2 sum_k [(sum_f v_fk)^2 -
sum_f v_fk^2], grad_v = loss * (sum_f' v_f'k - v_fk).
Latent params start at N(0,1) * 1e-2 (FTRL, ftrl.h:114-120) or 0.001 (SGD).
"""
from xflow_amd.models.base import SparseModel


class FM(SparseModel):
    kind = "fm"
