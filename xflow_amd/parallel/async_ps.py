"""Asynchronous parameter server: BASELINE config 4 without lock-step.

The reference's workers never wait for each other.  Each Hogwild slice pulls
its keys, computes, pushes (``lr_worker.cc:145-177``), and every server
applies each push the moment it arrives, per coordinate
(``ftrl.h:54-80``).  M workers are started independently
(``scripts/local.sh:31-35``).  The lock-step ``ShardedEngine`` makes every rank
enter every all-to-all of every step, so one slow GPU stalls all of them.

This class runs the reference's process model on one node of MI355X GPUs,
without a single collective inside training:

* a **server thread** per process owns the rank's table shard (its own native
  Engine on its own HIP stream).  It serves pull requests and applies pushes
  of every source in arrival order (per source in step order), like a
  ps-lite ``KVServer`` request handle;
* the caller's thread is the **worker** (a second Engine: dedup, forward,
  backward).  Its keys go straight into the owners' inboxes in their HBM, the
  owners' pull kernels write the values straight into the worker's response
  slot, and its CSR (key, slice) gradient entries (several slices) or
  gradient rows go into the owners' inboxes;
* that memory is a per-rank window: fine-grained HBM exported by HIP IPC
  (xGMI peer writes) on GPUs, ``/dev/shm`` on the CPU backend.  Hand-over is
  by sequence words in a shared control segment
  (``csrc/comm/async_ps.cpp``).

Bounded staleness ``k``: a worker pulls for step t only once every owner has
applied its own pushes of steps <= t-k-1.  So at most k of its pushes are in
flight; ``k = 0`` is the reference's ``Push`` + ``Wait``.  Nothing ties a
fast worker to a slow one: the asynchronous data parallelism of the
reference.  The fault knob ``XFLOW_FAULT=slow_rank:<rank>:<ms>`` makes one
worker a straggler.

Every owner logs what its stream ran: (kind, source, step, count), kind 0 =
pull, 1 = push, 2 = eval pull.  ``replay_logs`` is the specification: it
re-executes the logs with plain engine phase calls in one process, and the
live tables equal the replay bit for bit (``tests/test_async_ps.py``).
"""
from __future__ import annotations

import dataclasses
import os
import uuid
from typing import Optional, Sequence

import numpy as np
import torch
import torch.distributed as dist

from xflow_amd import native
from xflow_amd.config import EngineConfig, ModelConfig, OptimConfig
from xflow_amd.engine import Batch, Engine
from xflow_amd.utils.faults import slow_ms_from_env

PULL, PUSH, EVAL = 0, 1, 2


def worker_config(cfg: EngineConfig) -> EngineConfig:
    """The worker engine's config: the same model / batch limits, a token
    table (the worker never owns keys)."""
    return dataclasses.replace(cfg, table_log2_cap=min(cfg.table_log2_cap, 16), table_grow=False)


class AsyncParameterServer:
    """One rank of the asynchronous parameter server (see the module doc).

        aps = AsyncParameterServer(model, optim, cfg, device, staleness=1, slices=S)
        gen = SyntheticCriteo(aps.worker, rows, ...)
        for _ in range(steps):
            aps.train_step(gen.next())
        aps.finish()          # own pushes applied; every rank's servers still serve
        ... rank 0 may aps.eval_step(batch) ...
        aps.close()           # barrier, then the server threads exit
    """

    def __init__(self, model: ModelConfig, optim: OptimConfig, cfg: EngineConfig,
                 device: str | torch.device = "cpu", staleness: int = 1, slices: int = 1,
                 group: Optional[dist.ProcessGroup] = None, pair_frac: float = 1.0,
                 timeout_s: Optional[float] = None, name: Optional[str] = None,
                 slow_ms: Optional[int] = None, start: bool = True):
        """start=False: call ``start()`` later (e.g. after preparing the
        server's table shard, which nothing may touch once it serves)."""
        self.group = group
        on = dist.is_initialized()
        self.world = dist.get_world_size(group) if on else 1
        self.rank = dist.get_rank(group) if on else 0
        self.device = torch.device(device)
        self.staleness = int(staleness)
        self.slices = int(slices)
        if cfg.max_slices < self.slices:
            cfg = dataclasses.replace(cfg, max_slices=self.slices)
        # the table shard: driven only by the server thread while it runs
        self.server = Engine(model, optim, cfg, self.device)
        self.worker = Engine(model, optim, worker_config(cfg), self.device)
        if name is None:
            name = "xflow_aps_%d_%s" % (os.getpid(), uuid.uuid4().hex[:8])
            if self.world > 1:
                box = [name]
                dist.broadcast_object_list(box, src=0, group=group)
                name = box[0]
        self.name = name
        if slow_ms is None:
            slow_ms = slow_ms_from_env(self.rank)
        self.slow_ms = int(slow_ms)
        timeout = float(timeout_s if timeout_s is not None
                        else os.environ.get("XFLOW_DIST_TIMEOUT", "600"))
        dev = self.device.index if self.device.type == "cuda" else -1
        if self.device.type == "cuda" and dev is None:
            dev = torch.cuda.current_device()
        self._ps = native.load().AsyncPS(self.worker.native, self.server.native, self.world,
                                         self.rank, self.staleness, self.slices, name,
                                         timeout_s=timeout, slow_ms=self.slow_ms,
                                         pair_frac=float(pair_frac), device=dev)
        self.closed = False
        self.started = False
        if start:
            self.start()

    def start(self) -> None:
        """Handshake (every rank maps every window), barrier, start the server
        thread.  Collective."""
        if self.started:
            return
        h = self._ps.handle()
        if self.world > 1:
            hs = [None] * self.world
            dist.all_gather_object(hs, h, group=self.group)
        else:
            hs = [h]
        self._ps.connect(hs)
        self._barrier()
        self._ps.start()
        self.started = True

    def _barrier(self) -> None:
        if self.world > 1:
            dist.barrier(group=self.group)

    @property
    def native(self):
        return self._ps

    @property
    def transport(self) -> str:
        """'ipc' (fine-grained HBM windows over HIP IPC), 'ipc-coarse', or 'shm'."""
        return self._ps.transport

    @property
    def csr(self) -> bool:
        """Gradients travel as CSR (key, slice) entries (else dense rows)."""
        return bool(self._ps.csr)

    def _view(self, batch):
        if isinstance(batch, Batch):
            batch.check(self.worker.device)
            return batch.view()
        return batch  # a native BatchView (engine-staged synthetic batch)

    def train_step(self, batch) -> bool:
        """One worker step; waits only for its own owners' responses and for
        its k-th previous pushes to be applied (never for another worker)."""
        self.worker._sync_stream()
        return bool(self._ps.train_step(self._view(batch)))

    def eval_step(self, batch, pctr: Optional[torch.Tensor] = None) -> Optional[torch.Tensor]:
        """Forward only over every owner's current weights (keys not inserted)."""
        rows = batch.rows if isinstance(batch, Batch) else int(batch.rows)
        if pctr is None:
            pctr = torch.empty(rows, dtype=torch.float32, device=self.device)
        self.worker._sync_stream()
        return pctr if self._ps.eval_step(self._view(batch), pctr.data_ptr()) else None

    def finish(self) -> None:
        """Wait until every push of this worker is applied (the owners keep
        serving until ``close``)."""
        self._ps.finish()

    def pause(self) -> None:
        """Every rank: finish, barrier, stop serving -- the server engine (the
        table shard) is then the caller's, e.g. for an epoch's statistics or a
        checkpoint.  ``resume`` serves again from where it stopped."""
        self._ps.finish()
        self._barrier()
        self._ps.stop()

    def resume(self) -> None:
        """Serve again after ``pause`` (the first call makes the handshake)."""
        if not self.started:
            self.start()
        else:
            self._ps.start()

    @property
    def serving(self) -> bool:
        return bool(self._ps.serving)

    def close(self) -> None:
        """Every rank: finish, barrier (no worker needs a server any more),
        stop the server thread."""
        if self.closed:
            return
        self._ps.finish()
        self._barrier()
        self._ps.stop()
        self.server._sync_stream()
        self.closed = True

    def log(self) -> np.ndarray:
        """This owner's operations in stream order: rows (kind, source, step, count)."""
        return np.asarray(self._ps.log(), dtype=np.int64).reshape(-1, 4)

    def stats(self) -> dict:
        p = self._ps
        return {"steps": int(p.steps), "evals": int(p.evals), "bytes_moved": int(p.bytes_moved),
                "max_staleness": int(p.max_staleness), "max_lead": int(p.max_lead),
                "wait_slot_s": float(p.wait_slot_s), "wait_pull_s": float(p.wait_pull_s),
                "sync_s": float(p.sync_s), "served_pulls": int(p.served_pulls),
                "applied_pushes": int(p.applied_pushes), "server_busy_s": float(p.server_busy_s),
                "transport": self.transport, "csr": self.csr, "staleness": self.staleness,
                "slow_ms": self.slow_ms}


def replay_logs(logs: Sequence[np.ndarray], batches: Sequence[Sequence[Batch]],
                workers: Sequence[Engine], servers: Sequence[Engine], staleness: int,
                slices: int) -> None:
    """The specification of the asynchronous server: re-execute every owner's
    log with plain engine phase calls in ONE process.

    logs[o]: owner o's (kind, source, step, count) rows; batches[s][t]: the
    batch worker s trained at step t; workers[s] / servers[o]: fresh engines
    (worker s's own, so its dedup history -- and send order -- is the live
    one).  Owners' operations run in their logged order; across owners any
    order that respects causality (a source's step-t gradients need every
    owner's step-t pull, its step t+1 keys need its step-t gradients) gives
    the same tables, since owners hold disjoint keys.  After the call
    ``servers[o]`` holds what the live owner o should hold."""
    W = len(servers)
    R = int(staleness) + 1
    S = int(slices)
    w0 = workers[0]
    vw, gw = w0.value_width, w0.grad_width
    csr = bool(w0.native.csr_exchange(S))
    masks = (not csr) and S > 1 and not w0.cfg.sum_slices
    fm_keep = w0.model.kind == "fm" and w0.model.fm_math == "reference"
    eb = int(w0.native.csr_entry_bytes)
    dev = w0.device
    for lg in logs:
        if len(lg) and (lg[:, 0] == EVAL).any():
            raise ValueError("replay_logs: training logs only (no eval pulls)")
    # per source: the prepared step, the step whose gradients exist, and per
    # step in flight its keys / pulled rows / gradients (kept until every
    # owner applied it: with k > 0 the source moves on before that)
    st = [dict(t=-1, ready=-1, steps={}) for _ in range(W)]

    def prepare(s: int, t: int) -> None:
        w = workers[s]
        b = batches[s][t]
        counts = torch.zeros(W, dtype=torch.int64, device=dev)
        send = torch.zeros(max(b.nnz, 1), dtype=torch.int64, device=dev)
        w.w_prepare(b, W, counts, send, wb=0, seq=-1)
        n = [max(0, int(c)) for c in counts.tolist()]
        off = np.concatenate([[0], np.cumsum(n)]).astype(np.int64)
        ns = int(off[-1])
        st[s]["t"] = t
        st[s]["steps"][t] = dict(
            counts=counts, n=n, off=off, ns=ns, batch=b, got=set(), applied=0,
            keys=[send[off[o]:off[o] + n[o]].clone() for o in range(W)],
            pulled=torch.zeros(max(ns, 1), vw, dtype=torch.float32, device=dev))

    def backward(s: int, t: int) -> None:
        x = st[s]["steps"][t]
        w = workers[s]
        b, ns, n, off = x["batch"], x["ns"], x["n"], x["off"]
        if csr:
            cnt = torch.zeros(max(ns, 1), dtype=torch.int32, device=dev)
            ent = torch.zeros(max(b.nnz, 1) * eb // 4 + 4, dtype=torch.int32, device=dev)
            tot = torch.zeros(W, dtype=torch.int64, device=dev)
            w.native.w_forward_backward_csr(b.view(), x["pulled"].data_ptr(), ns, S, 0,
                                            cnt.data_ptr(), ent.data_ptr(), x["counts"].data_ptr(),
                                            W, tot.data_ptr())
            w.w_finish()
            e = tot.tolist()
            eo = np.concatenate([[0], np.cumsum(e)]).astype(np.int64)
            entb = ent.view(torch.uint8)
            x["push"] = [(cnt[off[o]:off[o] + n[o]].clone(),
                          entb[eo[o] * eb:eo[o + 1] * eb].clone()) for o in range(W)]
        else:
            grads = torch.zeros(max(ns, 1), S * gw, dtype=torch.float32, device=dev)
            mk = torch.zeros(max(ns, 1), dtype=torch.int32, device=dev) if masks else None
            w.w_forward_backward(b, x["pulled"], ns, grads, mk, S, wb=0, group=0)
            w.w_finish()
            x["push"] = [(grads[off[o]:off[o] + n[o]].clone(),
                          mk[off[o]:off[o] + n[o]].clone() if masks else None) for o in range(W)]
        st[s]["ready"] = t

    ptr = [0] * W
    total = sum(len(lg) for lg in logs)
    done = 0
    while done < total:
        moved = False
        for o in range(W):
            while ptr[o] < len(logs[o]):
                kind, s, t, cnt = (int(v) for v in logs[o][ptr[o]])
                src = st[s]
                buf = s * R + t % R
                if kind == PULL:
                    if src["t"] != t:  # prepare step t once step t-1's gradients exist
                        if src["t"] != t - 1 or src["ready"] != t - 1:
                            break
                        prepare(s, t)
                    x = src["steps"][t]
                    n_o = x["n"][o]
                    if n_o != cnt:
                        raise AssertionError(f"replay: source {s} step {t} sends {n_o} keys to "
                                             f"owner {o}, the log says {cnt}")
                    out = x["pulled"][x["off"][o]:x["off"][o] + n_o] if n_o else x["pulled"]
                    servers[o].s_pull(x["keys"][o], n_o, out, insert=True, buf=buf,
                                      offsets=[0, n_o], keep_weights=fm_keep)
                    x["got"].add(o)
                    if len(x["got"]) == W:
                        backward(s, t)
                else:
                    if src["ready"] < t:
                        break
                    x = src["steps"][t]
                    g, m = x["push"][o]
                    n_o = x["n"][o]
                    if csr:
                        servers[o].native.s_apply_csr(x["keys"][o].data_ptr(), g.data_ptr(),
                                                      m.data_ptr(), [0, n_o], S, buf)
                    else:
                        servers[o].s_apply(x["keys"][o], g, m, [0, n_o], S, buf=buf)
                    servers[o].end_step()
                    x["applied"] += 1
                    if x["applied"] == W:
                        del src["steps"][t]
                ptr[o] += 1
                done += 1
                moved = True
        if not moved:
            raise AssertionError("replay: the logs are not causally consistent")
