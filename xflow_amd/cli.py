"""``xflow_lr``-compatible command line (multi-rank capable).

    python -m xflow_amd.cli <train_prefix> <test_prefix> <model 0|1|2> <epochs> [flags]

Positional arguments are the reference binary's (src/model/main.cc:15-48).
Process roles follow the reference launch scripts' DMLC_ROLE: scheduler and
server processes exit (the workers' GPUs hold the table shards); workers
train.  World size / rank come from torchrun env (RANK, WORLD_SIZE, ...) or
DMLC_NUM_WORKER / DMLC_WORKER_ID (scripts/local.sh sets both).
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

from xflow_amd.config import (EngineConfig, ModelConfig, OptimConfig, TrainConfig,
                              MODEL_NAMES, model_kind)


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog="xflow_lr", description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("train_prefix")
    ap.add_argument("test_prefix")
    ap.add_argument("model", help="0 = LR, 1 = FM, 2 = MVM (or lr/fm/mvm)")
    ap.add_argument("epochs", type=int)
    ap.add_argument("--threads", type=int, default=0,
                    help="slices per block (default: os.cpu_count(), like hardware_concurrency)")
    ap.add_argument("--serial-slices", action="store_true",
                    help="one step per slice instead of all slices in one step")
    ap.add_argument("--keep-remainder", action="store_true",
                    help="train rows %% threads too (the reference drops them)")
    ap.add_argument("--optimizer", choices=["ftrl", "sgd"], default="ftrl")
    ap.add_argument("--alpha", type=float, default=5e-2)
    ap.add_argument("--beta", type=float, default=1.0)
    ap.add_argument("--lambda1", type=float, default=5e-5)
    ap.add_argument("--lambda2", type=float, default=10.0)
    ap.add_argument("--lr", type=float, default=1e-3, help="SGD learning rate")
    ap.add_argument("--v-dim", type=int, default=10)
    ap.add_argument("--fm-math", choices=["reference", "standard"], default="reference")
    ap.add_argument("--mvm-math", choices=["compat", "fixed"], default="compat")
    ap.add_argument("--mvm-predict-compat", action="store_true")
    ap.add_argument("--sum-slices", action="store_true",
                    help="one FTRL push of the summed slice gradients per step")
    ap.add_argument("--no-init-push", action="store_true")
    ap.add_argument("--async", dest="async_ps", action="store_true",
                    help="multi-rank: the asynchronous parameter server (BASELINE config 4) -- a "
                         "server thread per rank, workers that never wait for each other")
    ap.add_argument("--async-lockstep", dest="async_p2p", action="store_true",
                    help="multi-rank: lock-step steps whose pushes ride in the next exchange")
    ap.add_argument("--staleness", type=int, default=1,
                    help="--async: own pushes in flight (0..7); --async-lockstep: pulls miss "
                         "the previous N steps' pushes (1..7)")
    ap.add_argument("--log2-cap", type=int, default=22,
                    help="initial table slots per rank = 2^N (the table grows)")
    ap.add_argument("--max-log2-cap", type=int, default=0,
                    help="growth limit 2^N slots per rank (0: 2^31, or what free HBM allows)")
    ap.add_argument("--no-table-grow", action="store_true",
                    help="fixed table capacity: an overflow raises within two steps")
    ap.add_argument("--train-block-bytes", type=int, default=2 << 20)
    ap.add_argument("--test-block-bytes", type=int, default=0)
    ap.add_argument("--gpu-parse", action="store_true",
                    help="tokenise libffm text on the GPU (raw blocks uploaded; keys, labels and "
                         "field ids bit-equal to the host parser)")
    ap.add_argument("--resident", action="store_true",
                    help="keep the training shard in HBM after the first epoch (no re-read)")
    ap.add_argument("--csr-only", action="store_true",
                    help="train fixed-width blocks through the CSR path as well")
    ap.add_argument("--block-rows", type=int, default=0,
                    help="rows per block when <prefix>-%%05d.xfb binary shards exist "
                         "(python -m xflow_amd.data.binfmt convert); default 65536")
    ap.add_argument("--cpu", action="store_true", help="use the native CPU backend")
    ap.add_argument("--pred-dir", default=".")
    ap.add_argument("--no-pred-file", action="store_true",
                    help="skip pred_<rank>_<block>.txt (AUC/logloss are computed on the device "
                         "either way; the file is the only reason predictions reach the host)")
    ap.add_argument("--fm-mfma", action="store_true",
                    help="standard-math FM forward on the matrix cores (v_dim <= 8; A/B option)")
    ap.add_argument("--save", default="", help="checkpoint directory to write after training")
    ap.add_argument("--load", default="", help="checkpoint directory to resume from")
    ap.add_argument("--resume", default="",
                    help="versioned checkpoint root: continue from its LATEST checkpoint if one "
                         "exists (epochs = total for the run) and write periodic saves there")
    ap.add_argument("--save-every", type=int, default=0,
                    help="versioned checkpoint every N epochs under --resume (or --save) root")
    ap.add_argument("--metrics", default="", help="JSON-lines metrics file (rank 0)")
    ap.add_argument("--trace-dir", default="", help="torch.profiler chrome trace directory")
    return ap


def config_from_args(a) -> TrainConfig:
    kind = MODEL_NAMES[model_kind(a.model)]
    return TrainConfig(
        train_prefix=a.train_prefix, test_prefix=a.test_prefix, epochs=a.epochs,
        threads=a.threads, train_block_bytes=a.train_block_bytes, block_rows=a.block_rows,
        resident=a.resident, fixed_width=not a.csr_only, gpu_parse=a.gpu_parse,
        test_block_bytes=a.test_block_bytes, serial_slices=a.serial_slices,
        keep_remainder=a.keep_remainder, mvm_predict_compat=a.mvm_predict_compat,
        init_push=not a.no_init_push, pred_dir=a.pred_dir, write_pred=not a.no_pred_file,
        checkpoint_dir=a.save,
        save_every=a.save_every, resume_dir=a.resume,
        metrics_file=a.metrics, async_p2p=a.async_p2p, async_ps=a.async_ps,
        staleness=a.staleness,
        model=ModelConfig(kind=kind, v_dim=a.v_dim, fm_math=a.fm_math, mvm_math=a.mvm_math,
                          fm_mfma=a.fm_mfma),
        optim=OptimConfig(kind=a.optimizer, alpha=a.alpha, beta=a.beta, lambda1=a.lambda1,
                          lambda2=a.lambda2, lr=a.lr),
        engine=EngineConfig(table_log2_cap=a.log2_cap, sum_slices=a.sum_slices,
                            max_log2_cap=a.max_log2_cap, table_grow=not a.no_table_grow))


def main(argv=None) -> int:
    from xflow_amd.parallel import dist as xdist

    if xdist.is_scheduler():
        return 0
    if xdist.is_server():
        print("init server success ", flush=True)
        return 0
    a = build_parser().parse_args(argv)
    cfg = config_from_args(a)
    print({0: "start LR ", 1: "start FM ", 2: "start MVM "}[model_kind(a.model)], flush=True)
    device = torch.device("cpu") if a.cpu else xdist.device_for_rank()
    from xflow_amd.trainer import Trainer
    from xflow_amd.utils.trace import torch_profile

    t = Trainer(cfg, device=device)
    try:
        if a.load:
            t.load(a.load)
        if a.resume:
            t.resume(a.resume)
        with torch_profile(a.trace_dir):
            t.train()
        if a.save:
            t.save(a.save)
    finally:
        t.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
