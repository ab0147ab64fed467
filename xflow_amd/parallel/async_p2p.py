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
asynchronous pushes.  Keys and pulled values still use all-to-all (a pull is
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

    def _p2p(self, out: torch.Tensor, inp: torch.Tensor, out_splits, in_splits):
        """Post point-to-point sends of inp (split by in_splits) and receives
        into out (split by out_splits); returns the request handles."""
        ops = []
        so = ro = 0
        for peer in range(self.world):
            ns, nr = int(in_splits[peer]), int(out_splits[peer])
            if peer == self.rank:
                if ns:
                    out[ro:ro + nr].copy_(inp[so:so + ns])
            else:
                if ns:
                    ops.append(dist.P2POp(dist.isend, inp[so:so + ns], peer, self.group))
                if nr:
                    ops.append(dist.P2POp(dist.irecv, out[ro:ro + nr], peer, self.group))
            so += ns
            ro += nr
        self.p2p_ops += len(ops)
        return dist.batch_isend_irecv(ops) if ops else []

    def _apply_pending(self) -> None:
        if self._pending is None:
            return
        reqs, recv_keys, grads_in, masks_in, offsets, S, buf = self._pending
        for r in reqs:
            r.wait()
        self.engine.s_apply(recv_keys, grads_in, masks_in, offsets, S, buf=buf)
        self._pending = None

    def train_step(self, batch: Batch, S: Optional[int] = None, prefetch=None) -> None:
        e = self.engine
        S = int(S) if S else e.slices_of(batch)
        ps = e.pstride
        W = S * e.grad_width
        ordered_masks = S > 1 and not e.cfg.sum_slices
        buf = self._parity
        send_splits, recv_splits, recv_keys = self._exchange_keys(batch, prefetch)
        n_send, n_recv = self.last_send, self.last_recv
        # keep this step's received keys alive until its pushes are applied
        rk = self._rk[buf].get(n_recv)
        rk.copy_(recv_keys)
        pulled = self._pull(rk, send_splits, recv_splits, insert=True, buf=buf)
        # staleness 1: the previous step's pushes land after this step's pull
        self._apply_pending()
        grads_out = self._gout[buf].get(n_send * W).view(n_send, W)
        masks_out = self._mout[buf].get(n_send) if ordered_masks else None
        e.w_forward_backward(batch, pulled, n_send, grads_out, masks_out, S)
        grads_in = self._gin[buf].get(n_recv * W).view(n_recv, W)
        reqs = self._p2p(grads_in, grads_out, recv_splits, send_splits)
        masks_in = None
        if ordered_masks:
            masks_in = self._min[buf].get(n_recv)
            reqs = list(reqs) + list(self._p2p(masks_in, masks_out, recv_splits, send_splits))
        offsets = [0]
        for c in recv_splits:
            offsets.append(offsets[-1] + int(c))
        self._pending = (reqs, rk, grads_in, masks_in, offsets, S, buf)
        self._parity ^= 1
        self.bytes_moved += (n_send + n_recv) * (8 + 4 * ps + 4 * W)

    def flush(self) -> None:
        """Apply the last in-flight pushes (call before evaluation/checkpoint)."""
        self._apply_pending()

    def eval_step(self, batch: Batch, pctr: Optional[torch.Tensor] = None) -> torch.Tensor:
        self.flush()
        return super().eval_step(batch, pctr)
