"""The single-rank step's layout decisions (Engine::train_step's gradient path)
as one pure function, plan_step(StepInputs, S): checked over the whole input
space on the CPU -- every combination picks exactly one gradient layout, the
flags agree with it, and the headline configurations land where DESIGN.md says.

Reference semantics being laid out: per-slice pushes of each slice's keys
(lr_worker.cc:162-175, fm_worker.cc:241-242, mvm_worker.cc:214-218).
"""
import itertools

import pytest
import torch

from xflow_amd import native
from xflow_amd.config import EngineConfig, ModelConfig, OptimConfig
from xflow_amd.engine import Engine

MODELS = {
    "lr": ModelConfig(kind="lr"),
    "fm_ref": ModelConfig(kind="fm", v_dim=8, fm_math="reference"),
    "fm_std": ModelConfig(kind="fm", v_dim=8, fm_math="standard"),
    "mvm": ModelConfig(kind="mvm", v_dim=10),
}
UNIQUE_FLAG = {"unique_lr": "lr16", "unique_fm_bc": "fmu", "unique_rows": "rowu", "slot_sums": "lr16s"}


def plan(model, opt="ftrl", S=1, **kw):
    d = {"model": MODELS[model].native(), "opt": OptimConfig(kind=opt).native()}
    d.update(kw)
    return native.load().plan_step(d, S)


def _cases():
    for model, opt, S, csr, sum_slices, gpu in itertools.product(
            MODELS, ("ftrl", "sgd"), (1, 2, 8, 32, 33, 64, 256, 1024), (True, False), (False, True),
            (True, False)):
        if sum_slices and S > 32:
            continue  # (rejected by train_step before planning)
        yield model, opt, S, csr, sum_slices, gpu


def test_every_input_picks_one_consistent_layout():
    n = 0
    for model, opt, S, csr, sum_slices, gpu in _cases():
        p = plan(model, opt, S, csr=csr, sum_slices=sum_slices, gpu=gpu)
        n += 1
        tag = (model, opt, S, csr, sum_slices, gpu, p)
        g = p["grad"]
        assert g in ("csr", "unique_lr", "unique_fm_bc", "unique_rows", "slot_sums", "slot_rows"), tag
        # the unique-order layouts are mutually exclusive and each matches its flag
        flags = [p[f] for f in ("lr16", "fmu", "rowu", "lr16s")]
        assert sum(flags) <= 1, tag
        for name, f in UNIQUE_FLAG.items():
            assert (g == name) == p[f], tag
        assert p["rowu"] == (p["mvmu"] or p["fsu"]), tag
        if g == "csr":
            assert S > 1 and csr and not sum_slices and gpu, tag
            assert S >= (8 if model in ("lr", "fm_std") else 4), tag  # (the A/B thresholds)
            assert (model == "lr" and opt == "ftrl") or model in ("fm_ref", "fm_std", "mvm"), tag
            assert p["csr_rows"] == (model in ("fm_std", "mvm")), tag
            assert (1 << p["csr_slog2"]) >= S > (1 << p["csr_slog2"]) // 2, tag
            continue
        assert p["csr_slog2"] == -1, tag
        # slice groups: ceil(S / 32) groups of 32 (masked per-slice paths)
        assert p["groups"] == (1 if S <= 32 else -(-S // 32)), tag
        assert p["Sf"] == (32 if p["groups"] > 1 else S), tag
        assert p["masks"] == (p["Sf"] > 1 and not sum_slices), tag
        assert not p["uq"] or p["Sf"] > 1, tag
        assert p["fm_keep_w"] == (model == "fm_ref" and gpu and p["groups"] > 1), tag
        if not gpu:  # the CPU backend: slot rows, nothing unique-order
            assert g == "slot_rows" and not p["upos"] and not p["grpst"], tag
    assert n == 384  # 4 models x 2 optimisers x 2 csr x 2 backends x (8 + 4) slice settings


@pytest.mark.parametrize("model,opt,S,kw,grad", [
    ("lr", "ftrl", 1, {}, "unique_lr"),                     # the headline step
    ("lr", "ftrl", 4, {}, "unique_lr"),                     # below CSR's slice threshold
    ("lr", "ftrl", 8, {}, "csr"),
    ("lr", "ftrl", 256, {}, "csr"),
    ("fm_ref", "ftrl", 2, {}, "unique_fm_bc"),
    ("fm_ref", "ftrl", 4, {}, "csr"),
    ("fm_std", "ftrl", 4, {}, "unique_rows"),
    ("mvm", "ftrl", 2, {}, "slot_rows"),
    ("mvm", "ftrl", 4, {}, "csr"),
    ("lr", "ftrl", 8, {"csr": False}, "unique_lr"),
    ("lr", "ftrl", 64, {"csr": False}, "unique_lr"),         # slice groups
    ("lr", "ftrl", 8, {"sum_slices": True}, "slot_sums"),
    ("lr", "sgd", 1, {}, "slot_rows"),
    ("fm_ref", "ftrl", 1, {}, "unique_fm_bc"),
    ("fm_ref", "ftrl", 8, {}, "csr"),
    ("fm_ref", "ftrl", 256, {}, "csr"),
    ("fm_ref", "ftrl", 64, {"csr": False}, "unique_fm_bc"),
    ("fm_ref", "sgd", 8, {}, "csr"),
    ("fm_std", "ftrl", 1, {}, "unique_rows"),
    ("fm_std", "ftrl", 64, {}, "csr"),                     # full-row entries
    ("fm_std", "sgd", 256, {}, "csr"),
    ("fm_std", "ftrl", 64, {"csr": False}, "unique_rows"),
    ("mvm", "ftrl", 1, {}, "unique_rows"),
    ("mvm", "ftrl", 8, {}, "csr"),
    ("mvm", "sgd", 256, {}, "csr"),
    ("mvm", "ftrl", 8, {"csr": False}, "slot_rows"),
    ("lr", "ftrl", 1, {"gpu": False}, "slot_rows"),
])
def test_pinned_layouts(model, opt, S, kw, grad):
    assert plan(model, opt, S, **kw)["grad"] == grad


def test_csr_falls_back_past_its_dest_bounds():
    # dests unique * 2^slog2 + slice: below 2^32 with max_nnz unique keys, and
    # one key's slices inside one reduction bucket (2^14 dests LR, 2^13 FM)
    assert plan("lr", "ftrl", 512)["grad"] == "csr"  # (max_nnz 2^22)
    assert plan("lr", "ftrl", 513)["grad"] == "unique_lr"
    assert plan("lr", "ftrl", 256, max_nnz=1e7)["grad"] == "csr"  # (a bench-sized step)
    assert plan("lr", "ftrl", 512, max_nnz=1e7)["grad"] == "unique_lr"
    small = {"max_nnz": float(1 << 16)}
    assert plan("lr", "ftrl", 1 << 14, **small)["grad"] == "csr"
    assert plan("lr", "ftrl", (1 << 14) + 1, **small)["grad"] == "unique_lr"
    assert plan("fm_ref", "ftrl", 1 << 13, **small)["grad"] == "csr"
    assert plan("fm_ref", "ftrl", (1 << 13) + 1, **small)["grad"] == "unique_fm_bc"
    # standard FM: 2^10 dests per key at most (the vector records' bucket)
    assert plan("fm_std", "ftrl", 1 << 10, **small)["grad"] == "csr"
    assert plan("fm_std", "ftrl", (1 << 10) + 1, **small)["grad"] == "unique_rows"
    # ... and the scatter-free producer form (<= 2048 workgroups of 512 rows)
    assert plan("fm_std", "ftrl", 8, max_rows=float(1 << 20))["grad"] == "csr"
    assert plan("fm_std", "ftrl", 8, max_rows=float((1 << 20) + 1))["grad"] == "unique_rows"


def test_engine_plan_matches_its_backend():
    e = Engine(ModelConfig(kind="lr"), OptimConfig(), EngineConfig(table_log2_cap=12, max_rows=64,
                                                                   max_nnz=1024, max_slices=8),
               device=torch.device("cpu"))
    for S in (1, 8):
        p = e.native.step_plan(S)
        assert p["grad"] == "slot_rows" and p["S"] == S
