"""Multi-view machine (reference: src/model/mvm/mvm_worker.{h,cc}).

Params per key: [v_0 .. v_{D-1}].  Per latent dim k: S[k][g] = sum of v_fk
over the row's features in field g, M[k] = prod over fields of S[k][g],
y = sum_k M[k].  Gradient: loss * M[k] / (1 + S[k][g]) (0 when S == 0),
divided by slice rows (mvm_worker.cc:137-170).

mvm_math="compat" multiplies fields [0, max_fgid) like the reference (whose
per-row field vector is one short: the max field is written out of bounds
and never multiplied); "fixed" multiplies [0, max_fgid].
"""
from xflow_amd.models.base import SparseModel


class MVM(SparseModel):
    kind = "mvm"
