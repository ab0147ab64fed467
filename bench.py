#!/usr/bin/env python3
"""Headline benchmark: LR + FTRL-Proximal training throughput (samples/s,
whole node) and progressive train logloss on synthetic Criteo-1TB-shaped data
(39 fields, 1e9 hashed features), BASELINE.json config 2/3.

    python bench.py --gpus 1 --steps 20 --warmup 5
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N --steps K --warmup W

A step = one batch of --batch rows per GPU (weak scaling): generate the batch
on device, dedup its keys, pull weights (sharded table, sparse all-to-all over
RCCL when N > 1), fused forward/backward, push gradients, per-coordinate FTRL
update on the owners.  Nothing is skipped inside the timed region.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from xflow_amd.config import EngineConfig, ModelConfig, OptimConfig  # noqa: E402
from xflow_amd.data.synth import SynthConfig, SyntheticCriteo  # noqa: E402
from xflow_amd.engine import Engine  # noqa: E402

METRIC = "samples/sec (whole node) + logloss, LR-FTRL Criteo-1TB shape at 1/2/4/8 MI355X"


def parse():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawTextHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=262144, help="rows per GPU per step")
    ap.add_argument("--model", default="lr", choices=["lr", "fm", "mvm"])
    ap.add_argument("--v-dim", type=int, default=8)
    ap.add_argument("--fm-math", default="reference", choices=["reference", "standard"],
                    help="FM interaction: the reference's (fm_worker.cc:159-202) or Rendle's "
                         "standard 1/2 sum_k[(sum v)^2 - sum v^2] (BASELINE config 5)")
    ap.add_argument("--fm-mfma", action="store_true",
                    help="standard-math FM forward on the matrix cores (A/B option; measured "
                         "slower than the VALU form, docs/DESIGN.md section 6)")
    ap.add_argument("--slices", type=int, default=1,
                    help="Hogwild slices per step (lr_worker.cc:190-199): every slice reads the "
                         "same weights, gradients normalised per slice, pushes applied per key in "
                         "slice order")
    ap.add_argument("--optimizer", default="ftrl", choices=["ftrl", "sgd"])
    ap.add_argument("--log2-cap", type=int, default=0,
                    help="table slots per GPU = 2^N (default: 2^31 across the node)")
    ap.add_argument("--features", type=int, default=1_000_000_000)
    ap.add_argument("--table-load", type=float, default=-1.0,
                    help="before training (untimed), fill this fraction of every table shard's "
                         "slots with keys no batch touches -- the occupancy a long run reaches "
                         "(the reference store keeps every key ever pushed, ftrl.h:54-56,84).  "
                         "Default (-1): the whole --features model, i.e. features/N keys per "
                         "GPU (load 0.47 of 2^31/N slots for 1e9 features); 0 = empty table")
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--cpu", action="store_true", help="CPU backend (smoke only)")
    ap.add_argument("--sharded", action="store_true",
                    help="force the multi-rank (all-to-all) step even at 1 GPU (overhead probe)")
    ap.add_argument("--async", dest="async_ps", action="store_true",
                    help="config 4: the asynchronous parameter server (parallel/async_ps.py) -- "
                         "every rank a server thread + a worker that never lock-steps with the "
                         "others; keys, values and CSR gradient entries through HIP-IPC windows "
                         "in peer HBM, no collective inside training.  Each rank times its own "
                         "steps; value = total samples / the slowest rank's time")
    ap.add_argument("--async-lockstep", dest="async_p2p", action="store_true",
                    help="the lock-step staleness-k step (pushes over RCCL riding in the next "
                         "step's key exchange; every rank in every group call)")
    ap.add_argument("--staleness", type=int, default=1,
                    help="--async / --async-lockstep: staleness in steps")
    ap.add_argument("--pair-frac", type=float, default=1.0,
                    help="--async: inbox capacity per (source, owner) as a fraction of a step's "
                         "occurrences (1: any key skew fits)")
    ap.add_argument("--sgd-v-init", type=float, default=1e-3,
                    help="SGD latent init (sgd.h:69: the constant 0.001); MVM-SGD with 1.0 keeps "
                         "the field product live (FTRL's first push shrinks v by ~|g|)")
    ap.add_argument("--sgd-lr", type=float, default=1e-3,
                    help="SGD learning rate (sgd.h:16: 0.001).  The reference's gradient is a "
                         "mean over the slice's rows, so a 262 144-row slice moves a key by "
                         "~lr/262144 per occurrence: bench-shape MVM learns at a larger rate")
    ap.add_argument("--planted-bias", type=float, default=-1.2,
                    help="synthetic labels' planted logit bias (-1.2: a ~26 %% CTR).  The "
                         "reference MVM's output sigmoid(sum_k prod_f v_sum) cannot fall "
                         "below 0.5 once its field sums are positive, so MVM quality rows "
                         "also run on +1.2 (the same keys, a ~74 %% CTR)")
    ap.add_argument("--fields", type=int, default=39,
                    help="fields (= features) per row: 13 int + (F-13) categorical Criteo fields; "
                         "e.g. 18 like the bundled data (MVM's field product stays live)")
    ap.add_argument("--v-init-scale", type=float, default=1e-2,
                    help="latent init N(0,1)*scale (ftrl.h:114-120: 1e-2).  MVM on 39 fields "
                         "at 1e-2 has a field product that underflows to 0 (no gradient "
                         "traffic); 1.0 keeps it alive for measuring the backward")
    ap.add_argument("--lambda1", type=float, default=5e-5,
                    help="FTRL L1 (ftrl.h:19); config 4 reports the non-zero weight count")
    ap.add_argument("--clock-warmup-s", type=float, default=0.25,
                    help="GPU: before the --warmup steps, keep the GPU busy for this long with a "
                         "dense matmul that touches no engine state: a first process on an idle "
                         "GPU otherwise times its first steps at idle clocks (seen once in five "
                         "cold boxes: 315 vs 525 M samples/s).  Training warmup is exactly "
                         "--warmup steps, so logloss/table_keys do not depend on the box")
    ap.add_argument("--monitor-lag", type=int, default=7,
                    help="steps the host may run ahead of the table-capacity monitor "
                         "(EngineConfig.monitor_lag).  The host queues a step in ~40 us of "
                         "the device's ~470: 7 steps of run-ahead (~3 ms) absorb host "
                         "scheduling hiccups; 2, 7 and 32 measured the same throughput "
                         "(profiles/r3s3_monitor_lag.txt)")
    ap.add_argument("--csr", choices=["on", "off"], default="on",
                    help="several slices as CSR gradients (EngineConfig.csr); off: the slice-group "
                         "layouts (A/B)")
    ap.add_argument("--overlap", choices=["on", "off"], default="off",
                    help="generate batch t+1 on a side stream while step t runs (measured on "
                         "one MI355X: 2-4%% slower for the fused and the multi-rank step, the "
                         "generator competes with the step's kernels for CUs and LDS)")
    return ap.parse_args()


def _entropy(p: float) -> float:
    """ln-logloss of always predicting the base rate p."""
    if p <= 0.0 or p >= 1.0:
        return 0.0
    return -(p * math.log(p) + (1.0 - p) * math.log(1.0 - p))


def run_async(a, world, rank, device, use_gpu, shared_gpu, synth, log2_cap, nnz):
    """--async: BASELINE config 4 on the asynchronous parameter server.  Every
    rank warms up, meets the others at one barrier, then runs its --steps
    without any further meeting; its time ends when its own last pushes are
    applied.  A straggler (XFLOW_FAULT=slow_rank:<r>:<ms>) slows only itself:
    the per-rank rates in the JSON show it."""
    from xflow_amd.parallel.async_ps import AsyncParameterServer

    model = ModelConfig(kind=a.model, v_dim=a.v_dim, fm_math=a.fm_math, fm_mfma=a.fm_mfma)
    optim = OptimConfig(kind=a.optimizer, lambda1=a.lambda1, v_init_scale=a.v_init_scale,
                        sgd_v_init=a.sgd_v_init, lr=a.sgd_lr)
    cfg = EngineConfig(table_log2_cap=log2_cap, max_rows=a.batch, max_nnz=nnz,
                       max_slices=a.slices, monitor_lag=a.monitor_lag, csr=a.csr == "on")
    aps = AsyncParameterServer(model, optim, cfg, device, staleness=a.staleness,
                               slices=a.slices, pair_frac=a.pair_frac, start=False)
    if a.table_load < 0:
        n_prefill = a.features // world if use_gpu else 0
    else:
        n_prefill = int(a.table_load * 2 ** log2_cap)
    n_prefill = min(n_prefill, int(0.9 * 2 ** log2_cap))
    # (the server thread owns the table: prefill before it serves anything)
    if n_prefill > 0:
        aps.server.native.prefill(n_prefill, 0x5eed + rank)
        aps.server.synchronize()
    prefilled = aps.server.native.table_size()
    aps.start()
    gen = SyntheticCriteo(aps.worker, a.batch, synth, rank=rank, slice_rows=a.batch // a.slices)

    def sync():
        if use_gpu:
            torch.cuda.synchronize(device)

    for _ in range(a.warmup):
        aps.train_step(gen.next())
    sync()
    aps.native.finish()
    dist.barrier() if world > 1 else None
    aps.worker.read_stats(reset=True)
    p = aps.native
    s0 = (p.steps, p.bytes_moved, p.wait_slot_s, p.wait_pull_s, p.sync_s)
    p.max_staleness = 0
    p.max_lead = 0
    t0 = time.perf_counter()
    for _ in range(a.steps):
        aps.train_step(gen.next())
    aps.native.finish()  # this rank's last pushes applied: part of its timed work
    sync()
    elapsed = time.perf_counter() - t0
    st = aps.worker.read_stats(reset=True)
    mine = {"rank": rank, "elapsed_s": round(elapsed, 6),
            "steps_per_s": round(a.steps / elapsed, 3),
            "wait_slot_ms_per_step": round(1e3 * (p.wait_slot_s - s0[2]) / a.steps, 4),
            "wait_pull_ms_per_step": round(1e3 * (p.wait_pull_s - s0[3]) / a.steps, 4),
            "host_sync_ms_per_step": round(1e3 * (p.sync_s - s0[4]) / a.steps, 4),
            "bytes_moved_per_step": int((p.bytes_moved - s0[1]) // a.steps),
            "max_staleness": int(p.max_staleness), "max_lead": int(p.max_lead),
            "slow_ms": aps.slow_ms, "ln_loss": st["ln_loss"], "rows": st["rows"]}
    aps.close()  # barrier: every worker done; the server threads exit
    tbl = aps.server.native.table_size()
    nnzw = aps.server.nonzero_weights()
    ovf = float(aps.server.overflowed() or aps.worker.overflowed())
    mine.update(table_keys=int(tbl), nonzero=int(nnzw), ovf=ovf, prefilled=int(prefilled),
                served_pulls=int(p.served_pulls), applied_pushes=int(p.applied_pushes))
    if world > 1:
        allr = [None] * world
        dist.all_gather_object(allr, mine)
    else:
        allr = [mine]
    if any(r["ovf"] > 0 for r in allr):
        raise SystemExit("bench: a table or dedup-scratch overflow was flagged: the result is invalid")
    slowest = max(r["elapsed_s"] for r in allr)
    samples = a.batch * a.steps * world
    rows = sum(r["rows"] for r in allr)
    if rank == 0:
        out = {
            "metric": METRIC,
            "value": samples / slowest,
            "unit": "samples/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": 1000.0 * slowest / a.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic Criteo-1TB-shaped (%d fields, 1e9 hashed features, planted-logistic "
                    "labels); table prefilled (untimed) with %d keys no batch touches" % (
                        synth.fields, sum(r["prefilled"] for r in allr)),
            "config": {"model": f"{a.model.upper()}-{a.optimizer.upper()}",
                       "global_batch": a.batch * world, "seq_len": synth.fields,
                       "parallelism": f"dp{world}+table-shard{world}+async-ps(staleness={a.staleness})",
                       "rows_per_gpu": a.batch, "nnz_per_row": synth.fields, "slices": a.slices,
                       "grad_exchange": "csr" if aps.csr else "dense",
                       "hashed_features": a.features, "table_slots_per_gpu": 2 ** log2_cap,
                       "backend": aps.server.backend_name, "a2a_transport": aps.transport,
                       "lambda1": a.lambda1},
            **({"shared_gpu_rehearsal": True} if shared_gpu else {}),
            "logloss": sum(r["ln_loss"] for r in allr) / max(rows, 1.0),
            "table_keys": sum(r["table_keys"] for r in allr),
            "nonzero_weights": sum(r["nonzero"] for r in allr),
            "prefilled_keys": sum(r["prefilled"] for r in allr),
            "table_load": sum(r["table_keys"] for r in allr) / float(world * 2 ** log2_cap),
            # per-rank: each rank's own rate -- a straggler slows only itself
            "per_rank": [{k: r[k] for k in ("rank", "steps_per_s", "elapsed_s", "slow_ms",
                                            "max_staleness", "max_lead", "wait_slot_ms_per_step",
                                            "wait_pull_ms_per_step", "host_sync_ms_per_step",
                                            "bytes_moved_per_step")} for r in allr],
            "bytes_moved_per_step": int(sum(r["bytes_moved_per_step"] for r in allr) / world),
            "max_staleness": max(r["max_staleness"] for r in allr),
            "staleness_bound": a.staleness,
        }
        print(json.dumps(out), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        if world == 1 and a.gpus > 1:
            raise SystemExit("--gpus > 1 must be launched with torch.distributed.run")
    use_gpu = torch.cuda.is_available() and not a.cpu
    shared_gpu = False
    if use_gpu:
        from xflow_amd.parallel.dist import shared_gpu_setup

        # (XFLOW_SHARED_GPU=1: all ranks on this host's GPU 0 -- the
        # multi-process RCCL path rehearsed on a 1-GPU box, not a measurement)
        shared_gpu = world > 1 and shared_gpu_setup(rank)
        if shared_gpu:
            local = 0
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
    else:
        device = torch.device("cpu")
    if a.async_ps and world > 1:
        # the asynchronous parameter server needs no collective transport:
        # gloo carries only its start / end handshake
        dist.init_process_group("gloo", rank=rank, world_size=world)
    elif world > 1 or a.sharded or a.async_p2p:
        if world == 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29533")
        dist.init_process_group("nccl" if use_gpu else "gloo", rank=rank, world_size=world,
                                device_id=device if use_gpu else None)

    log2_cap = a.log2_cap or max(20, 31 - int(math.log2(world)))
    if not use_gpu:
        log2_cap = min(log2_cap, 24)
        a.batch = min(a.batch, 4096)
    synth = SynthConfig(total_features=a.features, hash_space=a.features, seed=a.seed,
                        n_fields=a.fields, planted_bias=a.planted_bias)
    nnz = a.batch * synth.fields
    if a.batch % a.slices:
        raise SystemExit("--batch must be a multiple of --slices")
    if a.async_ps:
        return run_async(a, world, rank, device, use_gpu, shared_gpu, synth, log2_cap, nnz)
    model = ModelConfig(kind=a.model, v_dim=a.v_dim, fm_math=a.fm_math, fm_mfma=a.fm_mfma)
    engine = Engine(model, OptimConfig(kind=a.optimizer, lambda1=a.lambda1,
                                       v_init_scale=a.v_init_scale, sgd_v_init=a.sgd_v_init,
                                       lr=a.sgd_lr),
                    EngineConfig(table_log2_cap=log2_cap, max_rows=a.batch, max_nnz=nnz,
                                 max_slices=a.slices, monitor_lag=a.monitor_lag,
                                 csr=a.csr == "on"),
                    device=device)
    if a.batch % a.slices:
        raise SystemExit("--batch must be a multiple of --slices")
    gen = SyntheticCriteo(engine, a.batch, synth, rank=rank, slice_rows=a.batch // a.slices)
    if a.table_load < 0:  # (the CPU smoke path runs on a small table: no default prefill)
        n_prefill = a.features // world if use_gpu else 0
    else:
        n_prefill = int(a.table_load * 2 ** log2_cap)
    n_prefill = min(n_prefill, int(0.9 * 2 ** log2_cap))
    if n_prefill > 0:
        engine.prefill(n_prefill, seed=0x5eed + rank)
    prefilled = engine.table_size()

    sharded = None
    if world > 1 or a.sharded or a.async_p2p:
        from xflow_amd.parallel.async_p2p import AsyncShardedEngine
        from xflow_amd.parallel.sparse_a2a import ShardedEngine

        sharded = (AsyncShardedEngine(engine, staleness=a.staleness) if a.async_p2p
                   else ShardedEngine(engine))
    overlap = a.overlap == "on"
    # XFLOW_FAULT=slow_rank:<r>:<ms>: rank r sleeps before every step (the
    # lock-step step then runs every rank at the straggler's pace; --async
    # applies the same knob inside the async parameter server)
    from xflow_amd.utils.faults import slow_ms_from_env

    slow_s = slow_ms_from_env(rank) / 1000.0
    if not overlap and sharded is not None:
        # double-buffered batches on the compute stream
        bufs = [gen.alloc_batch(), gen.alloc_batch()]
        gen.next(out=bufs[0])
        cur = [0]

        def step():
            # pipelined: batch t+1 is generated and prepared (dedup + counts
            # exchange) inside step t, so the host never waits on an in-flight
            # split-size copy (ShardedEngine.prepare)
            if slow_s:
                time.sleep(slow_s)
            i = cur[0]
            sharded.train_step(bufs[i], prefetch=lambda: gen.next(out=bufs[i ^ 1]),
                               next_batch=bufs[i ^ 1])
            cur[0] = i ^ 1
    elif not overlap:
        def step():
            engine.train_view(gen.next())
    else:
        # batch t+1 is generated on a side stream while step t runs
        # (xflow_amd.data.synth.DevicePipeline)
        pipe = gen.pipeline()
        run = sharded.train_step if sharded is not None else engine.train_step

        def step():
            run(pipe.next())
            pipe.done()

    def sync():
        if use_gpu:
            torch.cuda.synchronize(device)
        if world > 1:
            dist.barrier()

    if use_gpu and a.clock_warmup_s > 0:
        x = torch.randn(4096, 4096, device=device, dtype=torch.bfloat16)
        tw = time.perf_counter()
        while time.perf_counter() - tw < a.clock_warmup_s:
            for _ in range(8):
                x = torch.mm(x, x).clamp_(-1.0, 1.0)
            torch.cuda.synchronize(device)
        del x
    # MVM: the field products can vanish (FTRL's first push sets a latent from
    # (z, n), not from its init, and a product of ~fields small factors
    # underflows): the untimed warmup records each step's train logloss, so
    # the JSON says whether -- and after which step -- the model went dead
    warm_ll = []
    for _ in range(a.warmup):
        step()
        if a.model == "mvm":
            sync()
            stw = engine.read_stats(reset=True)
            warm_ll.append(stw["ln_loss"] / max(stw["rows"], 1.0))
    sync()
    engine.read_stats(reset=True)
    if sharded is not None:
        sharded.host_waits = 0
        sharded.mid_step_waits = 0
        sharded.host_wait_s = 0.0
        sharded.bytes_moved = 0
        sharded.csr_exchanges = 0
        sharded.csr_waits = 0
        sharded.csr_wait_s = 0.0
    mon0 = engine.monitor_wait_seconds
    sync()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    if hasattr(sharded, "flush"):
        sharded.flush()  # the last pushes are part of the timed work
    t_issue = time.perf_counter() - t0  # host time to queue the steps (bounded by monitor lag)
    # of which blocked: on the monitor's run-ahead bound (the device is
    # monitor_lag steps behind) and on split-size reads (multi-rank)
    t_blocked = engine.monitor_wait_seconds - mon0 + (
        sharded.host_wait_s + getattr(sharded, "csr_wait_s", 0.0) if sharded is not None else 0.0)
    comm = ({"bytes_moved_per_step": int(sharded.bytes_moved) // max(a.steps, 1),
             "csr_exchanges": int(getattr(sharded, "csr_exchanges", 0)),
             "csr_waits": int(getattr(sharded, "csr_waits", 0))} if sharded is not None else {})
    sync()
    elapsed = time.perf_counter() - t0
    st = engine.read_stats(reset=True)
    tbl = engine.table_size()
    # one more (untimed) step with the reduction's records counted: how much
    # gradient work a step of this model does (MVM: none for rows whose field
    # product vanished)
    records = -1
    if use_gpu:
        engine.count_records(True)
        step()
        sync()
        records = engine.take_records()
        engine.count_records(False)
        engine.read_stats(reset=True)
    nnzw = engine.nonzero_weights() if a.async_p2p else 0
    ovf = float(engine.overflowed())  # table probe wrap / dedup scratch overflow
    red = torch.tensor([elapsed, st["ln_loss"], st["rows"], float(tbl), float(nnzw), ovf,
                        float(prefilled), st["positives"]],
                       dtype=torch.float64, device=device)
    if world > 1:
        mx = red[:1].clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        dist.all_reduce(red, op=dist.ReduceOp.SUM)
        elapsed = float(mx.item())
    vals = red.tolist()
    # per-rank host time per step (issue net of blocked, and blocked)
    host_rank = [1000.0 * (t_issue - t_blocked) / a.steps, 1000.0 * t_blocked / a.steps,
                 int(getattr(sharded, "mid_step_waits", 0)), int(getattr(sharded, "host_waits", 0))]
    if world > 1:
        allh = [None] * world
        dist.all_gather_object(allh, host_rank)
    else:
        allh = [host_rank]
    ln_loss, rows, table_keys, nonzero = vals[1], vals[2], vals[3], vals[4]
    prefill_tot = vals[6]
    if vals[5] > 0:
        raise SystemExit("bench: a table or dedup-scratch overflow was flagged (keys would be "
                         "dropped or isolated): the result is invalid")
    samples = a.batch * a.steps * world
    if rank == 0:
        out = {
            "metric": METRIC,
            "value": samples / elapsed,
            "unit": "samples/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": 1000.0 * elapsed / a.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic Criteo-1TB-shaped (%d fields: %d log-binned int + %d categorical, "
                    "power-law values, 1e9 hashed features, planted-logistic labels); FTRL table "
                    "prefilled (untimed) with %d keys the batches never touch (a long run's "
                    "table occupancy), trained keys zero-init" % (
                        synth.fields, min(synth.fields, 13), max(0, synth.fields - 13),
                        int(prefill_tot)),
            "config": {"model": f"{a.model.upper()}-{a.optimizer.upper()}",
                       "global_batch": a.batch * world, "seq_len": synth.fields,
                       "parallelism": f"dp{world}+table-shard{world}",
                       "rows_per_gpu": a.batch, "nnz_per_row": synth.fields,
                       "slices": a.slices,
                       # the gradient layout the step planner picked (plan_step)
                       "grad_layout": engine.native.step_plan(a.slices)["grad"],
                       "hashed_features": a.features, "table_slots_per_gpu": 2 ** log2_cap,
                       "backend": engine.backend_name,
                       "a2a_transport": sharded.transport if sharded is not None else "none",
                       "input_overlap": overlap, "v_init_scale": a.v_init_scale,
                       "table_growths": engine.table_growths},
            **({"shared_gpu_rehearsal": True} if shared_gpu else {}),
            "logloss": ln_loss / max(rows, 1.0),
            # the constant predictor's logloss on the same labels (the base
            # rate's entropy): a model learns when logloss falls below it
            "constant_logloss": _entropy(vals[7] / max(rows, 1.0)),
            "table_keys": int(table_keys),
            "reduction_records_per_step": int(records),
            "table_load": table_keys / float(world * 2 ** log2_cap),
            "prefilled_keys": int(prefill_tot),
            "host_waits": int(sharded.host_waits) if sharded is not None else 0,
            # multi-rank: split-size reads of the next batch in the middle of a
            # step (for its early key exchange) that found the copy in flight
            "mid_step_waits": int(getattr(sharded, "mid_step_waits", 0)),
            # multi-rank: steps whose next batch's keys rode with the gradient
            # exchange (2 RCCL group calls per step instead of 3)
            "early_key_exchanges": int(getattr(sharded, "early_key_exchanges", 0)),
            # host time to issue a step, net of the time blocked (the device
            # being behind is not host cost), and the blocked time itself
            "host_issue_ms_per_step": 1000.0 * (t_issue - t_blocked) / a.steps,
            "host_blocked_ms_per_step": 1000.0 * t_blocked / a.steps,
            # every rank's [issue ms, blocked ms, mid-step waits, host waits]
            **({"host_per_rank": [[round(x, 4) if isinstance(x, float) else x for x in h]
                                  for h in allh]} if world > 1 else {}),
            "monitor_lag": a.monitor_lag,
            # multi-rank: bytes each rank sent + received per step (keys,
            # values, gradients; several slices: only the touched (key, slice)
            # entries), and the steps that ran on the CSR exchange
            **comm,
            "csr_steps": int(engine.csr_steps),
        }
        if a.model == "fm":
            out["config"]["v_dim"] = a.v_dim
            out["config"]["fm_math"] = a.fm_math
            # the path the interaction actually ran on (VALU per-row sums; the
            # MFMA form is an A/B option, slower on this sparse gather shape)
            out["config"]["fm_interaction"] = ("mfma" if a.fm_mfma and a.fm_math == "standard"
                                               else "valu")
        if a.model == "mvm":
            out["config"]["v_dim"] = a.v_dim
            # a live MVM: the field products did not all vanish (logloss != ln 2)
            out["mvm_live"] = abs(out["logloss"] - 0.6931471805599453) > 1e-4
            out["mvm_warmup_logloss"] = [round(x, 6) for x in warm_ll]
            dead = [i for i, x in enumerate(warm_ll) if abs(x - 0.6931471805599453) <= 1e-4]
            # first warmup step (0-based) whose rows all predicted exactly 0.5
            out["mvm_dead_from_step"] = dead[0] if dead else None
        if a.optimizer == "sgd":
            out["config"]["sgd_v_init"] = a.sgd_v_init
        if a.async_p2p:
            out["config"]["parallelism"] += "+async-p2p(staleness=%d)" % a.staleness
            out["config"]["lambda1"] = a.lambda1
            out["nonzero_weights"] = int(nonzero)
        print(json.dumps(out), flush=True)
    if sharded is not None and hasattr(sharded, "close"):
        sharded.close()
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
