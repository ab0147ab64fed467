"""Configuration dataclasses.  Defaults equal the reference's compile-time
constants:

=====================  ==========================  =====================================
knob                   default                     reference
=====================  ==========================  =====================================
FTRL alpha/beta/l1/l2  0.05 / 1.0 / 5e-5 / 10.0    src/optimizer/ftrl.h:17-20
latent dim             10                          fm_worker.h:92, mvm_worker.h:92
SGD lr                 0.001                       src/optimizer/sgd.h:16
SGD v init             0.001                       src/optimizer/sgd.h:69
FTRL v init            N(0,1) * 1e-2               src/optimizer/ftrl.h:117
train block            2 MB                        lr_worker.h:68
test block             4 MB (LR) / 2 MB (FM, MVM)  lr_worker.cc:80, fm_worker.cc:106
epochs                 60                          lr_worker.h:63
slices per block       hardware_concurrency        lr_worker.h:40
=====================  ==========================  =====================================
"""
from __future__ import annotations

import dataclasses
import os
from dataclasses import dataclass, field

MODEL_KINDS = {"lr": 0, "fm": 1, "mvm": 2}
MODEL_NAMES = {v: k for k, v in MODEL_KINDS.items()}
OPT_KINDS = {"ftrl": 0, "sgd": 1}
FM_MATH = {"reference": 0, "standard": 1}
MVM_MATH = {"compat": 0, "fixed": 1}


def model_kind(m) -> int:
    if isinstance(m, int):
        if m not in MODEL_NAMES:
            raise ValueError(f"model index must be 0 (LR), 1 (FM) or 2 (MVM), got {m}")
        return m
    m = str(m).lower()
    if m in ("0", "1", "2"):
        return int(m)
    if m not in MODEL_KINDS:
        raise ValueError(f"unknown model {m!r}; expected lr/fm/mvm")
    return MODEL_KINDS[m]


@dataclass
class ModelConfig:
    kind: str = "lr"             # lr | fm | mvm
    v_dim: int = 10
    fm_math: str = "reference"   # reference (fm_worker.cc math) | standard (Rendle FM)
    mvm_math: str = "compat"     # compat (fields [0,max)) | fixed (fields [0,max])
    # standard-math FM forward on the matrix cores (v_mfma_f32_16x16x4_f32,
    # GPU, v_dim <= 8); measured slower than the VALU form, see DESIGN.md 6
    fm_mfma: bool = False

    def native(self) -> dict:
        return {"kind": model_kind(self.kind), "v_dim": int(self.v_dim),
                "fm_math": FM_MATH[self.fm_math], "mvm_math": MVM_MATH[self.mvm_math],
                "fm_mfma": bool(self.fm_mfma)}

    @property
    def params_per_key(self) -> int:
        k = model_kind(self.kind)
        return 1 if k == 0 else (1 + self.v_dim if k == 1 else self.v_dim)


@dataclass
class OptimConfig:
    kind: str = "ftrl"           # ftrl | sgd
    alpha: float = 5e-2
    beta: float = 1.0
    lambda1: float = 5e-5
    lambda2: float = 10.0
    lr: float = 1e-3
    sgd_v_init: float = 1e-3
    v_init_scale: float = 1e-2
    seed: int = 0x5EED

    def native(self) -> dict:
        d = dataclasses.asdict(self)
        d["kind"] = OPT_KINDS[self.kind]
        return d


@dataclass
class EngineConfig:
    table_log2_cap: int = 22
    max_rows: int = 1 << 16
    max_nnz: int = 1 << 22
    max_slices: int = 1
    sum_slices: bool = False      # one push of Σ_s g_s instead of ordered per-slice pushes
    scratch_factor: float = 2.5
    # table capacity management (csrc/include/xflow/engine.h EngineConfig):
    # grow by segment splits (linear hashing) on a schedule that starts when
    # the fullest segments pass grow_start and keeps them <= grow_load, up to
    # 2^max_log2_cap slots (0: 2^31 or what free HBM allows); table_grow=False
    # keeps it fixed and an overflow raises within monitor_lag steps
    table_grow: bool = True
    grow_load: float = 0.8
    grow_start: float = 0.6
    max_log2_cap: int = 0
    monitor_lag: int = 2
    # owner apply of a multi-source sharded step on the GPU: 0 one launch per
    # source (default), 1 one grouped launch (csrc/include/xflow/engine.h)
    owner_group: int = 0
    # several slices on the GPU (LR-FTRL, reference FM): CSR gradients of the
    # touched (key, slice) pairs; False: slice groups of 32 (same pushes)
    csr: bool = True


@dataclass
class TrainConfig:
    train_prefix: str = ""
    test_prefix: str = ""
    epochs: int = 60
    threads: int = 0             # 0 => os.cpu_count() like hardware_concurrency
    train_block_bytes: int = 2 << 20
    block_rows: int = 0          # rows per block of binary (.xfb) shards; 0 => 65536
    fixed_width: bool = True     # blocks whose rows all hold F features train field-major
    resident: bool = False       # keep the first epoch's device batches in HBM for the rest
    copy_threads: int = 8        # host threads staging a block into pinned memory
    gpu_parse: bool = False      # libffm text shards tokenised on the GPU (data/textstream.py)
    test_block_bytes: int = 0    # 0 => 4 MB LR, 2 MB FM/MVM
    serial_slices: bool = False
    keep_remainder: bool = False
    mvm_predict_compat: bool = False
    init_push: bool = True
    pred_dir: str = "."
    write_pred: bool = True      # the reference's pred_<rank>_<block>.txt (lr_worker.cc:74-77)
    checkpoint_dir: str = ""
    save_every: int = 0          # versioned checkpoint every N epochs (checkpoint.publish)
    resume_dir: str = ""         # versioned checkpoint root: resume from LATEST, save there
    metrics_file: str = ""
    async_p2p: bool = False      # lock-step staleness-k steps, pushes riding the next exchange
    # the asynchronous parameter server (parallel/async_ps.py): per-rank server
    # threads, workers that never lock-step, no collective inside an epoch
    async_ps: bool = False
    staleness: int = 1           # async_ps: own pushes in flight; async_p2p: pushes missed
    model: ModelConfig = field(default_factory=ModelConfig)
    optim: OptimConfig = field(default_factory=OptimConfig)
    engine: EngineConfig = field(default_factory=EngineConfig)

    def resolved_threads(self) -> int:
        if self.threads > 0:
            return self.threads
        # hardware_concurrency (lr_worker.h:40-41); the native trainer's
        # XFLOW_HARDWARE_CONCURRENCY override applies here too
        hc = int(os.environ.get("XFLOW_HARDWARE_CONCURRENCY", "0") or 0)
        return hc if hc > 0 else (os.cpu_count() or 1)

    def resolved_test_block(self) -> int:
        if self.test_block_bytes > 0:
            return self.test_block_bytes
        return (4 << 20) if model_kind(self.model.kind) == 0 else (2 << 20)
