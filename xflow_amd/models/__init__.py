"""Model families of the reference (src/model/{lr,fm,mvm}) as configurations
of the native engine.

Each model is defined by its parameters per hashed key and its fused
forward/backward kernel (csrc/hip/kernels_model.hip, CPU twin in
csrc/cpu/cpu_backend.cpp):

========  ===================  =================================================
model     params per key       kernel / reference
========  ===================  =================================================
LR        [w]                  k_lr  -- lr_worker.cc:100-177
FM        [w, v_0..v_{D-1}]    k_fm  -- fm_worker.cc:126-245 (+ standard FM math)
MVM       [v_0..v_{D-1}]       k_mvm -- mvm_worker.cc:137-273
========  ===================  =================================================
"""
from xflow_amd.models.fm import FM  # noqa: F401
from xflow_amd.models.lr import LR  # noqa: F401
from xflow_amd.models.mvm import MVM  # noqa: F401

REGISTRY = {"lr": LR, "fm": FM, "mvm": MVM}


def get(name: str, **kw):
    return REGISTRY[name.lower()](**kw)
