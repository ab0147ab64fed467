"""Asynchronous (bounded-staleness) sharded training over RCCL point-to-point.

The reference's workers never wait for each other: a worker's Push is applied
by the server whenever it arrives, while other workers keep pulling
(lr_worker.cc:170-175 with ps-lite's asynchronous KVServer).  BASELINE.json
config 4 asks for that semantics emulated with RCCL point-to-point.  This
engine pipelines the sparse step with a staleness of one step:

    step t:  dedup/bucket(t) -> keys a2a(t) -> pull(t)      [sees pushes <= t-2]
             wait P2P grads(t-1) -> owners apply(t-1)
             fwd/bwd(t) -> post grads(t) with batch_isend_irecv (RCCL P2P)
    end:     flush() applies the last pending pushes

so the gradient transfer of step t overlaps the next step's dedup, key
exchange and pull, and every pull reads weights that miss exactly the
previous step's pushes -- the bounded-staleness form of the reference's
asynchronous pushes.  On GPUs the pushes are grouped ncclSend/ncclRecv on a
second native RCCL communicator and stream (RcclComm::send_recv), so the
transfer really runs concurrently with the next step's work; on CPU (gloo)
they are torch.distributed batch_isend_irecv.  Keys and pulled values still use all-to-all (a pull is
a synchronous request/response in the reference too: KVWorker::Wait on Pull).
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist

from xflow_amd.engine import Batch, Engine
from xflow_amd.parallel.sparse_a2a import ShardedEngine, _Buf


class AsyncShardedEngine(ShardedEngine):
    def __init__(self, engine: Engine, group: Optional[dist.ProcessGroup] = None):
        super().__init__(engine, group)
        dev = engine.device
        # double buffers: step t's exchange must not overwrite step t-1's in flight
        self._rk = [_Buf(torch.int64, dev), _Buf(torch.int64, dev)]
        self._gin = [_Buf(torch.float32, dev), _Buf(torch.float32, dev)]
        self._gout = [_Buf(torch.float32, dev), _Buf(torch.float32, dev)]
        self._min = [_Buf(torch.int32, dev), _Buf(torch.int32, dev)]
        self._mout = [_Buf(torch.int32, dev), _Buf(torch.int32, dev)]
        self._parity = 0
        self._pending = None
        self.p2p_ops = 0
        # Native transport: the pushes travel over a second RCCL communicator
        # on their own stream, so step t's gradient transfer runs concurrently
        # with step t+1's key exchange and pull (one communicator's operations
        # execute in issue order on its stream; the two never wait on each
        # other, and every rank issues both in the same order).
        self._p2p_comm = None
        self._p2p_stream = None
        if self._comm is not None:
            self._p2p_comm = self._new_comm()
            if self._p2p_comm is not None:
                self._p2p_stream = torch.cuda.Stream(device=dev)
        self.p2p_transport = "rccl" if self._p2p_comm is not None else "torch"

    def _p2p(self, out: torch.Tensor, inp: torch.Tensor, out_splits, in_splits):
        """Post point-to-point sends of inp (split by in_splits) and receives
        into out (split by out_splits); returns what _wait_p2p waits for."""
        rb = self._row_bytes(inp)
        peers, sends, sbytes, recvs, rbytes = [], [], [], [], []
        ops = []
        so = ro = 0
        for peer in range(self.world):
            ns, nr = int(in_splits[peer]), int(out_splits[peer])
            if peer == self.rank:
                if ns:
                    out[ro:ro + nr].copy_(inp[so:so + ns])
            elif self._p2p_comm is not None:
                if ns or nr:
                    peers.append(peer)
                    sends.append(inp[so:].data_ptr())
                    sbytes.append(ns * rb)
                    recvs.append(out[ro:].data_ptr())
                    rbytes.append(nr * rb)
            else:
                if ns:
                    ops.append(dist.P2POp(dist.isend, inp[so:so + ns], peer, self.group))
                if nr:
                    ops.append(dist.P2POp(dist.irecv, out[ro:ro + nr], peer, self.group))
            so += ns
            ro += nr
        if self._p2p_comm is not None:
            if not peers:  # only the self part (copied on the compute stream)
                return []
            self.p2p_ops += sum(1 for b in sbytes if b) + sum(1 for b in rbytes if b)
            cur = torch.cuda.current_stream(self.engine.device)
            st = self._p2p_stream
            st.wait_stream(cur)  # the gradients are written on the compute stream
            for t in (inp, out):
                t.record_stream(st)
            self._p2p_comm.send_recv(peers, sends, sbytes, recvs, rbytes, st.cuda_stream)
            done = torch.cuda.Event()
            done.record(st)
            return [done]
        self.p2p_ops += len(ops)
        return dist.batch_isend_irecv(ops) if ops else []

    def _wait_p2p(self, reqs) -> None:
        for r in reqs:
            if isinstance(r, torch.cuda.Event):
                torch.cuda.current_stream(self.engine.device).wait_event(r)
            else:
                r.wait()

    def _apply_pending(self) -> None:
        if self._pending is None:
            return
        reqs, recv_keys, grads_in, masks_in, offsets, S, buf = self._pending
        self._wait_p2p(reqs)
        self.engine.s_apply(recv_keys, grads_in, masks_in, offsets, S, buf=buf)
        self._pending = None

    def train_step(self, batch: Batch, S: Optional[int] = None, prefetch=None,
                   next_batch: Optional[Batch] = None) -> None:
        e = self.engine
        S = int(S) if S else e.slices_of(batch)
        ps = e.value_width  # floats per pulled value row
        W = S * e.grad_width
        ordered_masks = S > 1 and not e.cfg.sum_slices
        buf = self._parity
        wb, send_splits, recv_splits, prefetch = self._take(batch, prefetch)
        n_send, n_recv = self.last_send, self.last_recv
        # this step's received keys stay alive until its pushes are applied
        rk = self._rk[buf].get(n_recv)
        self._a2a(rk, self._send_keys[wb][:n_send], recv_splits, send_splits)
        offsets = self._offsets(recv_splits)
        vals = self._vals_out[buf].get(n_recv * ps).view(n_recv, ps)
        # (applied after the next step's pull: keep the pulled weights)
        e.s_pull(rk, n_recv, vals, insert=True, buf=buf, offsets=offsets, keep_weights=True)
        if prefetch is not None:
            prefetch()
        pulled = self._pulled.get(n_send * ps).view(n_send, ps)
        ops = [(pulled, vals, send_splits, recv_splits)]
        if next_batch is not None:
            self.prepare(next_batch, exchange=False)
            cop = self._counts_op(self._prep[1])
            if cop is not None:
                ops.append(cop)
        self._a2a_ops(ops)
        if next_batch is not None and not self._self_only():
            self._counts_sent(self._prep[1])
        # staleness 1: the previous step's pushes land after this step's pull
        self._apply_pending()
        grads_out = self._gout[buf].get(n_send * W).view(n_send, W)
        masks_out = self._mout[buf].get(n_send) if ordered_masks else None
        e.w_forward_backward(batch, pulled, n_send, grads_out, masks_out, S, wb=wb)
        grads_in = self._gin[buf].get(n_recv * W).view(n_recv, W)
        reqs = self._p2p(grads_in, grads_out, recv_splits, send_splits)
        masks_in = None
        if ordered_masks:
            masks_in = self._min[buf].get(n_recv)
            reqs = list(reqs) + list(self._p2p(masks_in, masks_out, recv_splits, send_splits))
        self._pending = (reqs, rk, grads_in, masks_in, offsets, S, buf)
        self._parity ^= 1
        self.bytes_moved += (n_send + n_recv) * (8 + 4 * ps + 4 * W)

    def flush(self) -> None:
        """Apply the last in-flight pushes (call before evaluation/checkpoint)."""
        self._apply_pending()

    def eval_step(self, batch: Batch, pctr: Optional[torch.Tensor] = None) -> torch.Tensor:
        self.flush()
        return super().eval_step(batch, pctr)

    def close(self) -> None:
        if self._p2p_comm is not None:
            torch.cuda.synchronize(self.engine.device)
            self._p2p_comm = None
        super().close()
