"""Asynchronous (bounded-staleness) sharded training over RCCL point-to-point.

The reference's workers never wait for each other: a worker's Push is applied
by the server whenever it arrives, while other workers keep pulling
(lr_worker.cc:170-175 with ps-lite's asynchronous KVServer, ftrl.h:54-80).
BASELINE.json config 4 asks for that semantics emulated with RCCL
point-to-point.  This engine pipelines the sparse step with a staleness of k
steps (default 1):

    step t:  keys(t) + grads(t-k)      one group call of ncclSend/ncclRecv
             pull(t)                   [sees every push of steps <= t-k-1]
             values(t) + counts(t+1)   one group call
             owners apply(t-k)
             fwd/bwd(t) -> grads(t) wait k steps in their buffer
    end:     flush() exchanges and applies the pending pushes in order

so every pull reads weights that miss exactly the previous k steps' pushes --
the bounded-staleness form of the reference's asynchronous pushes -- while the
gradient transfer rides in a collective the step issues anyway (no extra
RCCL launch, no second communicator).  All of a rank's RCCL operations run on
ONE communicator in one stream order, identical on every rank, so the
kernels of different calls can never be scheduled in conflicting orders on
two GPUs (two communicators on two streams could deadlock).  ncclSend /
ncclRecv pairs are RCCL's point-to-point primitives; each group call posts one
pair per peer with that peer's slice.  On CPU (gloo) the same exchanges run
as torch.distributed all-to-alls in the same order.

Keys and pulled values still use the lock-step exchange (a pull is a
synchronous request/response in the reference too: KVWorker::Wait on Pull).
Ranks therefore still meet once per step: this bounds staleness, it does not
make a slow rank invisible to the others.
"""
from __future__ import annotations

from collections import deque
from typing import Optional

import torch
import torch.distributed as dist

from xflow_amd.engine import Batch, Engine
from xflow_amd.parallel.sparse_a2a import _native_counter, ShardedEngine, _Buf

_SRV_BUFS = 8  # server buffers of the native engine (Engine::kSrvBufs)


class AsyncShardedEngine(ShardedEngine):
    # (the native step -- csrc/comm/sharded_step.cpp train_step_async -- runs
    # the same staleness-k step when ShardedEngine selects it)
    p2p_ops = _native_counter("p2p_ops")  # gradient pushes exchanged (one per step)

    def __init__(self, engine: Engine, group: Optional[dist.ProcessGroup] = None,
                 staleness: int = 1, **kw):
        if not 1 <= int(staleness) <= _SRV_BUFS - 1:
            raise ValueError("staleness must be in [1, %d]" % (_SRV_BUFS - 1))
        self.staleness = int(staleness)  # (read by the native step's setup)
        super().__init__(engine, group, **kw)
        dev = engine.device
        nbuf = self.staleness + 1  # step t's buffers live until its apply at step t+k
        self._nbuf = nbuf
        self._rk = [_Buf(torch.int64, dev) for _ in range(nbuf)]
        # per step buffer: one gradient / mask buffer per slice group
        # (Engine.slice_groups: more than 32 slices run in groups of 32)
        self._gin = [[_Buf(torch.float32, dev)] for _ in range(nbuf)]
        self._gout = [[_Buf(torch.float32, dev)] for _ in range(nbuf)]
        self._min = [[_Buf(torch.int32, dev)] for _ in range(nbuf)]
        self._mout = [[_Buf(torch.int32, dev)] for _ in range(nbuf)]
        # compact-FM applies read the values their step's pull served
        self._vals_out = [_Buf(torch.float32, dev) for _ in range(nbuf)]
        self._step_no = 0
        self._pending: deque = deque()
        self.p2p_transport = self.transport

    # ---- pushes ---------------------------------------------------------------
    @staticmethod
    def _push_ops(p) -> list:
        """Exchange ops of a pending step's pushes: gradients (+ slice masks)
        to their owners, the reverse of the step's key exchange (one pair per
        slice group)."""
        ops = []
        for gin, gout, min_, mout, _ in p["groups"]:
            ops.append((gin, gout, p["recv_splits"], p["send_splits"]))
            if min_ is not None:
                ops.append((min_, mout, p["recv_splits"], p["send_splits"]))
        return ops

    def _apply(self, p) -> None:
        self._apply_groups(p["rk"], [(gin, min_, Sg) for gin, _, min_, _, Sg in p["groups"]],
                           p["offsets"], buf=p["buf"])

    def train_step(self, batch: Batch, S: Optional[int] = None, prefetch=None,
                   next_batch: Optional[Batch] = None) -> bool:
        if self._native is not None:
            return super().train_step(batch, S, prefetch, next_batch)
        e = self.engine
        S = int(S) if S else e.slices_of(batch)
        ps = e.value_width  # floats per pulled value row
        gw = e.grad_width
        ordered_masks = S > 1 and not e.cfg.sum_slices
        wb, send_splits, recv_splits, prefetch, any_data = self._take(batch, prefetch)
        if not any_data:
            self.empty_steps += 1
            return False
        buf = self._step_no % self._nbuf
        n_send, n_recv = self.last_send, self.last_recv
        alias = self._self_only()
        # this step's received keys stay alive until its pushes are applied
        rk = self._rk[buf].get(n_recv)
        ops = [(rk, self._send_keys[wb][:n_send], recv_splits, send_splits)]
        due = self._pending[0] if len(self._pending) == self.staleness else None
        if due is not None and not alias:
            ops += self._push_ops(due)  # step t-k's pushes ride with step t's keys
        self._a2a_ops(ops)
        if due is not None:
            self.p2p_ops += 1
        offsets = self._offsets(recv_splits)
        vals = self._vals_out[buf].get(n_recv * ps).view(n_recv, ps)
        # (applied after the next k pulls: keep the pulled weights)
        e.s_pull(rk, n_recv, vals, insert=True, buf=buf, offsets=offsets, keep_weights=True)
        if prefetch is not None:
            prefetch()
        pulled = vals if alias else self._pulled.get(n_send * ps).view(n_send, ps)
        ops = [] if alias else [(pulled, vals, send_splits, recv_splits)]
        if next_batch is not None:
            self.prepare(next_batch, exchange=False)
            cop = self._counts_op(self._prep[1])
            if cop is not None:
                ops.append(cop)
        self._a2a_ops(ops)
        if next_batch is not None and not alias:
            self._counts_sent(self._prep[1])
        # staleness k: step t-k's pushes land after this step's pull
        if due is not None:
            self._apply(self._pending.popleft())
        groups = e.slice_groups(S)
        for lst in (self._gin[buf], self._gout[buf], self._min[buf], self._mout[buf]):
            while len(lst) < len(groups):
                lst.append(_Buf(lst[0].dtype, lst[0].device))
        pend = []
        for k, Sg in enumerate(groups):
            W = Sg * gw
            om = ordered_masks and Sg > 1
            grads_out = self._gout[buf][k].get(n_send * W).view(n_send, W)
            masks_out = self._mout[buf][k].get(n_send) if om else None
            e.w_forward_backward(batch, pulled, n_send, grads_out, masks_out, S, wb=wb, group=k)
            if alias:  # world 1: the owner reads the pushes in place
                grads_in, masks_in = grads_out, masks_out
            else:
                grads_in = self._gin[buf][k].get(n_recv * W).view(n_recv, W)
                masks_in = self._min[buf][k].get(n_recv) if om else None
            pend.append((grads_in, grads_out, masks_in, masks_out, Sg))
        self._pending.append(dict(rk=rk, groups=pend, recv_splits=recv_splits,
                                  send_splits=send_splits, offsets=offsets, buf=buf))
        self._step_no += 1
        e.w_finish()
        self.bytes_moved += (n_send + n_recv) * (8 + 4 * ps + 4 * S * gw)
        return True

    def flush(self) -> None:
        """Exchange and apply every pending push in step order (call before
        evaluation/checkpoint; every rank must call it)."""
        if self._native is not None:
            self.engine._sync_stream()
            self._native.flush()
            return
        while self._pending:
            p = self._pending.popleft()
            if not self._self_only():
                self._a2a_ops(self._push_ops(p))
            self.p2p_ops += 1
            self._apply(p)

    def eval_step(self, batch: Batch, pctr: Optional[torch.Tensor] = None) -> Optional[torch.Tensor]:
        self.flush()
        return super().eval_step(batch, pctr)
