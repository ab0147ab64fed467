"""Sharded sparse step: the ps-lite Pull/Push replacement over RCCL all-to-all.

Every rank is a worker (its own data shard) AND the server of a hash-owned
shard of the parameter table in its HBM (owner = fmix64(key) >> 32 mod world).
One training step, per rank (reference call sites: lr_worker.cc:170/175,
fm_worker.cc:228-242, the ps-lite DefaultSlicer, ftrl.h:38-152):

  1. w_prepare    dedup the batch's keys grouped by owner (owner-partitioned
                  scratch on the GPU, a bucket pass on the CPU backend)
  2. a2a counts   (int64 x world; -1 = "this source has no data this step",
                  so the loop ends when every source sent -1 -- no separate
                  per-step collective); the split sizes return through pinned
                  memory and are read when the batch's step starts -- with
                  next_batch, one step after they were produced (see prepare)
  3. a2a keys     -> each owner receives the keys it serves (steady state:
                  already received, in the previous step's gradient group
                  call -- two group calls per step, see early_keys)
  4. s_pull       owner probes/inserts its shard, evaluates pull values
  5. a2a values   -> back to the requesting workers (send order)
  6. w_forward_backward  fused fwd/bwd on the rank's rows, per-(key,slice)
                  gradient sums normalised by slice rows, in send order
  7. a2a grads    (+ slice masks when slices are applied in order)
  8. s_apply      owner applies every (source, slice) contribution of a key in
                  source order (deterministic, the analogue of ps-lite's
                  serialized handler) -- one launch per source (optionally one
                  grouped launch, EngineConfig.owner_group)

On GPUs the all-to-alls go through the native RCCL communicator on the
engine's stream (csrc/comm/rccl_comm.h; xGMI peer links between the node's
GPUs); otherwise through torch.distributed ("gloo" runs the same code on CPU
for tests).  Each all-to-all moves only the touched keys (8 B) and their P floats,
so a step's traffic is ~K*(8+8P) bytes per rank, spread over all 7 xGMI links
instead of a dense all-reduce of the table.

Consistency: steps are lock-step across ranks (every rank joins every
exchange; a rank without data passes an empty batch).  The reference's workers
are asynchronous; here all slices of all ranks in a step read the same table
state, and each owner applies the (source, slice) pushes one by one in source
order -- a deterministic serialisation of the reference's arrival-order pushes.
"""
from __future__ import annotations

import math
import os
import time
from typing import Callable, Optional

import torch
import torch.distributed as dist

from xflow_amd.engine import Batch, Engine


_COUNT_BITS = 40              # encode_count (csrc/include/xflow/backend.h)
_SEQ_MASK = (1 << 23) - 1


class _Buf:
    """Grow-only flat device buffer."""

    def __init__(self, dtype, device):
        self.dtype, self.device = dtype, device
        self.t = torch.empty(0, dtype=dtype, device=device)

    def get(self, n: int) -> torch.Tensor:
        if self.t.numel() < n:
            self.t = torch.empty(max(n, int(self.t.numel() * 1.25) + 1024), dtype=self.dtype,
                                 device=self.device)
        return self.t[:n]


def _native_counter(name: str):
    """A step counter kept by the native step when it runs (ShardedStep in
    csrc/comm/sharded_step.h), else on the Python object."""

    def fget(self):
        n = self.__dict__.get("_native")
        return getattr(n, name) if n is not None else self.__dict__.get("_c_" + name, 0)

    def fset(self, v):
        n = self.__dict__.get("_native")
        if n is not None:
            setattr(n, name, v)
        else:
            self.__dict__["_c_" + name] = v

    return property(fget, fset)


class ShardedEngine:
    """Runs Engine phases with sparse all-to-alls between them.

    Pipelined step: ``train_step(batch, next_batch=...)`` prepares the next
    batch (dedup + owner counts + counts exchange into the other worker buffer
    set, split sizes copied to pinned host memory) in the middle of the current
    step, before its forward/backward.  The host reads those split sizes only
    when it starts the next step, by which time the device copy finished long
    ago (it sits ahead of the current step's forward/backward, gradient
    exchange and apply in the queue): the host never waits on an in-flight
    exchange and stays about one step ahead of the device.  Without
    next_batch a step prepares its own batch first (one host wait per step).

    Native step: with the native RCCL communicator (or the world-1
    self-exchange) the whole step -- split decoding, op lists, group calls,
    applies -- runs in C++ (csrc/comm/sharded_step.cpp, one call per step;
    XFLOW_NATIVE_STEP=0 keeps it in Python; the staleness-k subclass too).  The methods below are the same
    step for the torch.distributed transport, and the specification the
    native one follows (tests/test_native_sharded.py)."""

    # steps the native implementation may run
    _native_ok = True
    host_waits = _native_counter("host_waits")
    mid_step_waits = _native_counter("mid_step_waits")
    host_wait_s = _native_counter("host_wait_s")
    early_key_exchanges = _native_counter("early_key_exchanges")
    inline_prepares = _native_counter("inline_prepares")
    empty_steps = _native_counter("empty_steps")
    bytes_moved = _native_counter("bytes_moved")
    drop_exchanges = _native_counter("drop_exchanges")
    last_send = _native_counter("last_send")
    last_recv = _native_counter("last_recv")
    # several slices as CSR entries (native GPU step): steps, and host waits
    # for the per-owner entry totals (the entries' all-to-all sizes)
    csr_exchanges = _native_counter("csr_exchanges")
    csr_waits = _native_counter("csr_waits")
    csr_wait_s = _native_counter("csr_wait_s")

    def __init__(self, engine: Engine, group: Optional[dist.ProcessGroup] = None,
                 world: Optional[int] = None, rank: Optional[int] = None,
                 transport: str = "auto", self_exchange: Optional[str] = None):
        """world/rank default to the process group's; passing them (with _a2a
        overridden) runs the step over another transport, e.g. in-process
        ranks in tests.  transport: see _init_transport.  self_exchange (world
        1 on a GPU): "alias" (default) reads the send buffers in place;
        "comm" sends every exchange through the transport anyway (RCCL
        ncclSend/ncclRecv to self) -- the multi-GPU code path on one GPU
        (XFLOW_SELF_EXCHANGE=comm)."""
        self.engine = engine
        self.self_exchange = self_exchange or os.environ.get("XFLOW_SELF_EXCHANGE", "alias")
        if self.self_exchange not in ("alias", "comm"):
            raise ValueError("self_exchange must be 'alias' or 'comm'")
        self.group = group
        custom = world is not None or rank is not None
        self.world = int(world) if world is not None else dist.get_world_size(group)
        self.rank = int(rank) if rank is not None else dist.get_rank(group)
        dev = engine.device
        W = self.world
        # per worker buffer set: send and receive counts side by side (one D2H
        # copy returns both), the owner-grouped send keys
        self._counts_both = [torch.zeros(2 * W, dtype=torch.int64, device=dev) for _ in range(2)]
        self._send_keys = [torch.empty(max(engine.cfg.max_nnz, 1), dtype=torch.int64, device=dev)
                           for _ in range(2)]
        # two receive-key buffers: the next batch's keys arrive (with this
        # step's gradients) while this step's apply still reads its own
        self._recv_keys = _Buf(torch.int64, dev)
        self._recv_keys_ahead = [_Buf(torch.int64, dev), _Buf(torch.int64, dev)]
        self._ahead = None         # the prepared batch whose keys already arrived
        self._ahead_no = 0
        self.early_key_exchanges = 0  # steps whose next keys rode with the gradients
        self.mid_step_waits = 0       # of those, split-size reads that waited
        self.host_wait_s = 0.0        # host seconds blocked on split-size reads (both kinds)
        # one per server buffer: compact-FM applies read the values served
        # by their step's pull (the async step applies after the next pull)
        self._vals_out = [_Buf(torch.float32, dev), _Buf(torch.float32, dev)]
        self._pulled = _Buf(torch.float32, dev)
        # one gradient / mask buffer pair per slice group of a step (more
        # than 32 Hogwild slices run as groups of 32: Engine.slice_groups)
        self._grads_out = [_Buf(torch.float32, dev)]
        self._grads_in = [_Buf(torch.float32, dev)]
        self._masks_out = [_Buf(torch.int32, dev)]
        self._masks_in = [_Buf(torch.int32, dev)]
        self.last_send = 0
        self.last_recv = 0
        self.bytes_moved = 0
        self.host_waits = 0        # split-size reads that found the copy still in flight
        self.inline_prepares = 0   # steps whose batch was not prepared ahead (epoch starts)
        self.drop_exchanges = 0    # fault injection (utils/faults.py drop_a2a): skip exchanges
        # the next batch's key exchange joins this step's gradient exchange
        # (XFLOW_EARLY_KEYS=0: its own exchange at the next step's start)
        self.early_keys = os.environ.get("XFLOW_EARLY_KEYS", "1") != "0"
        self.empty_steps = 0       # steps every rank passed without data (loop ends)
        self._counts_host = None
        self._counts_ready = None
        self._prep = None          # (batch, worker buffer set) prepared ahead
        self._seq = 0              # prepares so far (carried in the counts, world > 1)
        self._prep_seq = [0, 0]    # sequence number of each worker set's batch
        self._next_wb = 0
        self._comm = None
        self.__dict__["_native"] = None
        self.transport = "custom"
        if not custom:
            self._init_transport(transport)
            self._init_native()

    def _init_native(self) -> None:
        if not self._native_ok or os.environ.get("XFLOW_NATIVE_STEP", "1") == "0":
            return
        alias = self.world == 1 and self.self_exchange == "alias"
        if self._comm is None and not alias:
            return
        from xflow_amd import native

        # (world 1, aliased: no communicator -- the owner reads the send
        # buffers in place, as _self_only)
        self.__dict__["_native"] = native.load().ShardedStep(
            self.engine._e, None if alias else self._comm, self.world, self.rank, self.early_keys,
            int(getattr(self, "staleness", 0)))

    @property
    def native_step(self) -> bool:
        """True when train_step / eval_step run in C++ (ShardedStep)."""
        return self._native is not None

    # ---- transport ----------------------------------------------------------
    def _init_transport(self, transport: str) -> None:
        """"rccl": the native communicator (csrc/comm/rccl_comm.h) on the
        engine's stream; "torch": torch.distributed all_to_all_single on the
        process group's stream; "auto": rccl on a GPU unless XFLOW_A2A=torch.
        The native one is verified with a bounded self-test exchange on every
        rank and the job falls back to "torch" together if any rank fails."""
        self._comm = None
        if transport == "auto":
            transport = os.environ.get("XFLOW_A2A", "rccl" if self.engine.is_gpu else "torch")
        if transport == "torch" or not self.engine.is_gpu or self.group is not None:
            self.transport = "torch"
            return
        comm = self._new_comm()
        if comm is not None:
            self._comm = comm
            self.transport = "rccl"
        else:
            self.transport = "torch"

    def _new_comm(self):
        """A verified native RCCL communicator over the job's ranks, or None
        on every rank when any rank failed to create or self-test it."""
        from xflow_amd import native

        n = native.load()
        ok = 1
        comm = None
        try:
            obj = [n.RcclComm.unique_id() if self.rank == 0 else None]
            dist.broadcast_object_list(obj, src=0)
            comm = n.RcclComm(obj[0], self.world, self.rank, self.engine.device.index)
            ok = int(self._selftest(comm))
        except Exception as e:  # pragma: no cover - reported, then fall back
            print(f"[xflow] rank {self.rank}: native RCCL transport unavailable: {e}", flush=True)
            ok = 0
        flag = torch.tensor([ok], dtype=torch.int32, device=self.engine.device)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        if int(flag.item()) == 1:
            return comm
        if comm is not None:
            comm.abort()
        return None

    def _selftest(self, comm, timeout_s: float = 60.0) -> bool:
        W = self.world
        dev = self.engine.device
        send = torch.full((W,), self.rank, dtype=torch.int64, device=dev)
        recv = torch.full((W,), -1, dtype=torch.int64, device=dev)
        stream = torch.cuda.current_stream(dev)
        comm.alltoall(send.data_ptr(), recv.data_ptr(), 1, 8, stream.cuda_stream)
        ev = torch.cuda.Event()
        ev.record(stream)
        t0 = time.monotonic()
        while not ev.query():
            if time.monotonic() - t0 > timeout_s:
                return False
            time.sleep(0.001)
        return recv.cpu().tolist() == list(range(W))

    @staticmethod
    def _row_bytes(t: torch.Tensor) -> int:
        return math.prod(t.shape[1:]) * t.element_size()  # bytes per split unit

    def _a2a(self, out: torch.Tensor, inp: torch.Tensor, out_splits, in_splits) -> None:
        if self.drop_exchanges > 0:  # injected fault: this rank misses a collective
            self.drop_exchanges -= 1
            return
        if self._self_only():  # a self-exchange: one device copy
            if out.data_ptr() != inp.data_ptr():
                out.copy_(inp)
            return
        if self._comm is None:
            dist.all_to_all_single(out, inp, out_splits, in_splits, group=self.group)
            return
        stream = torch.cuda.current_stream(self.engine.device).cuda_stream
        if out_splits is None:
            self._comm.alltoall(inp.data_ptr(), out.data_ptr(), inp.shape[0] // self.world,
                                self._row_bytes(inp), stream)
        else:
            self._comm.alltoallv(inp.data_ptr(), [int(x) for x in in_splits], out.data_ptr(),
                                 [int(x) for x in out_splits], self._row_bytes(inp), stream)

    def _a2a_ops(self, ops) -> None:
        """Several all-to-alls, each (out, inp, out_splits, in_splits) with
        None splits meaning equal parts: ONE RCCL group call (one kernel)
        natively, one call each (in list order on every rank) otherwise."""
        if self._comm is None or len(ops) == 1 or self._self_only() or self.drop_exchanges:
            for out, inp, osp, isp in ops:
                self._a2a(out, inp, osp, isp)
            return
        W = self.world
        stream = torch.cuda.current_stream(self.engine.device).cuda_stream
        sc, rc = [], []
        for out, inp, osp, isp in ops:
            sc.append([inp.shape[0] // W] * W if isp is None else [int(x) for x in isp])
            rc.append([out.shape[0] // W] * W if osp is None else [int(x) for x in osp])
        self._comm.alltoallv_group([inp.data_ptr() for _, inp, _, _ in ops],
                                   [out.data_ptr() for out, _, _, _ in ops],
                                   [self._row_bytes(inp) for _, inp, _, _ in ops], sc, rc, stream)

    # ---- phases ---------------------------------------------------------------
    def prepare(self, batch: Batch, exchange: bool = True) -> None:
        """Dedup + owner grouping + counts exchange of ``batch`` into the next
        worker buffer set.  Collective: every rank prepares at the same point.
        exchange=False leaves the counts exchange to the caller, which joins it
        to another exchange's group call (_counts_op) and then calls
        _counts_sent."""
        e = self.engine
        W = self.world
        wb = self._next_wb
        self._next_wb ^= 1
        both = self._counts_both[wb]
        self._seq += 1  # (prepares are collective: every rank counts alike)
        e.w_prepare(batch, W, both[:W], self._send_keys[wb], wb, self._seq if W > 1 else -1)
        self._prep_seq[wb] = self._seq
        self._prep = (batch, wb)
        if self._self_only():  # receive counts = send counts (read from both[:W])
            self._counts_sent(wb)
        elif exchange:
            self._a2a(both[W:], both[:W], None, None)
            self._counts_sent(wb)

    def _counts_op(self, wb: int):
        """The counts exchange of buffer set wb, or None (world 1: none)."""
        if self._self_only():
            return None
        both = self._counts_both[wb]
        return (both[self.world:], both[:self.world], None, None)

    def _counts_sent(self, wb: int) -> None:
        both = self._counts_both[wb]
        if both.is_cuda:
            # the split sizes come back through pinned memory right behind the
            # counts exchange; read by the step that uses this batch
            if self._counts_host is None:
                self._counts_host = [torch.empty(2 * self.world, dtype=torch.int64,
                                                 pin_memory=True) for _ in range(2)]
                self._counts_ready = [torch.cuda.Event(), torch.cuda.Event()]
            self.engine.download_small(self._counts_host[wb], both)
            self._counts_ready[wb].record()

    def _take(self, batch: Batch, prefetch: Optional[Callable[[], None]] = None,
              mid_step: bool = False):
        """(worker buffer set, send splits, recv splits, prefetch, any data) of
        ``batch``, preparing it now unless it is the batch prepared ahead.
        A count of -1 marks a source without data (Engine.w_prepare on a
        batch of 0 rows); any data = some source (this rank included) has rows.
        mid_step: read for the early key exchange (a wait is expected there
        and counted in mid_step_waits)."""
        if self._prep is None or self._prep[0] is not batch:
            self.inline_prepares += 1
            self.prepare(batch)
            if prefetch is not None:  # device work to overlap the split-size round trip
                prefetch()
                prefetch = None
        _, wb = self._prep
        self._prep = None
        W = self.world
        both = self._counts_both[wb]
        if both.is_cuda:
            ev = self._counts_ready[wb]
            if not ev.query():
                if mid_step:
                    self.mid_step_waits += 1
                else:
                    self.host_waits += 1
                tw = time.perf_counter()
                ev.synchronize()
                self.host_wait_s += time.perf_counter() - tw
            both = self._counts_host[wb].tolist()
        else:
            both = both.tolist()
        send, recv = both[:W], (both[:W] if self._self_only() else both[W:])
        if W > 1:
            # (count + 1, sender's prepare number): a peer that skipped an
            # exchange shows up as a different number -- fail now, not later
            mask = (1 << _COUNT_BITS) - 1
            seqs = [int(c) >> _COUNT_BITS for c in recv]
            want = self._prep_seq[wb] & _SEQ_MASK
            if any(q != want for q in seqs):
                raise RuntimeError(f"rank {self.rank}: counts exchange out of step (expected "
                                   f"prepare {want}, peers sent {seqs}): a rank skipped or "
                                   f"repeated a collective")
            send = [(int(c) & mask) - 1 for c in send]
            recv = [(int(c) & mask) - 1 for c in recv]
        any_data = any(int(c) >= 0 for c in recv)
        send_splits = [max(int(c), 0) for c in send]
        recv_splits = [max(int(c), 0) for c in recv]
        self.last_send, self.last_recv = int(sum(send_splits)), int(sum(recv_splits))
        return wb, send_splits, recv_splits, prefetch, any_data

    def _exchange_keys(self, wb: int, send_splits, recv_splits) -> torch.Tensor:
        if self._self_only():  # world 1: the owner reads the send buffer in place
            return self._send_keys[wb][:self.last_send]
        recv_keys = self._recv_keys.get(self.last_recv)
        self._a2a(recv_keys, self._send_keys[wb][:self.last_send], recv_splits, send_splits)
        return recv_keys

    def _self_only(self) -> bool:
        """World 1 on a GPU: every exchange is a self-exchange, so the step
        aliases send and receive buffers instead of copying through RCCL
        (unless self_exchange == "comm")."""
        return self.world == 1 and self.engine.is_gpu and self.self_exchange == "alias"

    @staticmethod
    def _offsets(splits):
        offs = [0]
        for c in splits:
            offs.append(offs[-1] + int(c))
        return offs

    def train_step(self, batch: Batch, S: Optional[int] = None,
                   prefetch: Optional[Callable[[], None]] = None,
                   next_batch: Optional[Batch] = None) -> bool:
        """One lock-step training step.  S = slices per step, identical on every
        rank (defaults to this batch's slice count, fine when all ranks use the
        same batch shape).  ``prefetch``: device work producing the next batch
        (e.g. the synthetic generator), queued before ``next_batch`` is
        prepared.  Every rank must pass next_batch (or not) alike; a rank out
        of data passes an empty batch (0 rows).  Returns False, having done
        nothing, when no rank had data for ``batch`` -- every rank sees the
        same counts, so all of them stop at the same step."""
        e = self.engine
        S = int(S) if S else e.slices_of(batch)
        if self._native is not None:
            batch.check(e.device)
            if next_batch is not None:
                next_batch.check(e.device)
            e._sync_stream()
            # The native step tells batches apart by id(): the announced batch
            # stays referenced here until the step after it, so no other Batch
            # can take its id while its prepared dedup and keys are pending.
            self._native_announced = next_batch
            # (prefetch: called back once the pull is queued, as below)
            return bool(self._native.train_step(
                batch.view(), id(batch), S, next_batch.view() if next_batch is not None else None,
                id(next_batch) if next_batch is not None else 0, prefetch))
        ps = e.value_width  # floats per pulled value row
        ordered_masks = S > 1 and not e.cfg.sum_slices
        ahead = self._ahead
        self._ahead = None
        if ahead is not None and ahead["batch"] is batch:
            # prepared AND its keys received during the previous step
            wb, send_splits, recv_splits, any_data = (ahead["wb"], ahead["send"], ahead["recv"],
                                                      ahead["any"])
            self.last_send, self.last_recv = ahead["n_send"], ahead["n_recv"]
        else:
            # (a batch other than the announced next one: the keys exchanged
            # ahead are dropped -- every rank drops them at the same step, as a
            # prepared batch that is not trained next always was)
            wb, send_splits, recv_splits, prefetch, any_data = self._take(batch, prefetch)
        if not any_data:
            self.empty_steps += 1
            return False
        n_send, n_recv = self.last_send, self.last_recv
        # (keys received ahead belong to the announced batch only: another
        # batch re-exchanges its own)
        recv_keys = (ahead["keys"] if ahead is not None and ahead["batch"] is batch
                     else self._exchange_keys(wb, send_splits, recv_splits))
        offsets = self._offsets(recv_splits)
        vals = self._vals_out[0].get(n_recv * ps).view(n_recv, ps)
        # (slice groups apply after each other: compact FM rows then expand
        # with the kept pulled weights)
        e.s_pull(recv_keys, n_recv, vals, insert=True, buf=0, offsets=offsets,
                 keep_weights=len(e.slice_groups(S)) > 1)
        if prefetch is not None:
            prefetch()
        alias = self._self_only()
        pulled = vals if alias else self._pulled.get(n_send * ps).view(n_send, ps)
        ops = [] if alias else [(pulled, vals, send_splits, recv_splits)]
        if next_batch is not None:
            # the next batch's counts travel in the same group call as the values
            self.prepare(next_batch, exchange=False)
            cop = self._counts_op(self._prep[1])
            if cop is not None:
                ops.append(cop)
        self._a2a_ops(ops)
        if next_batch is not None and not self._self_only():
            self._counts_sent(self._prep[1])

        # one gradient exchange per step; a step of more than 32 slices sends
        # one (gradients, masks) pair per slice group in that exchange and
        # the owner applies the groups in order (every group's forward read
        # the same pulled rows: one S-slice step)
        gw = e.grad_width  # (B, C) per slice for reference-math FM on the GPU
        groups = e.slice_groups(S)
        for lst in (self._grads_out, self._grads_in, self._masks_out, self._masks_in):
            while len(lst) < len(groups):
                lst.append(_Buf(lst[0].dtype, lst[0].device))
        outs, ins, ops = [], [], []
        for k, Sg in enumerate(groups):
            W = Sg * gw
            om = ordered_masks and Sg > 1
            grads_out = self._grads_out[k].get(n_send * W).view(n_send, W)
            masks_out = self._masks_out[k].get(n_send) if om else None
            e.w_forward_backward(batch, pulled, n_send, grads_out, masks_out, S, wb=wb, group=k)
            outs.append((grads_out, masks_out))
            if alias:
                ins.append((grads_out, masks_out))
                continue
            grads_in = self._grads_in[k].get(n_recv * W).view(n_recv, W)
            masks_in = self._masks_in[k].get(n_recv) if om else None
            ins.append((grads_in, masks_in))
            ops.append((grads_in, grads_out, recv_splits, send_splits))
            if om:  # slice masks in the same group call
                ops.append((masks_in, masks_out, recv_splits, send_splits))
        if not alias:
            if next_batch is not None and self.early_keys:
                # the next batch's keys ride in this group call: its split sizes
                # came with the values exchange above, so the host reads them
                # now -- while the device still runs this step's forward/backward
                # -- and a steady-state step makes two exchanges, not three
                wb2, ss2, rs2, _, any2 = self._take(next_batch, mid_step=True)
                n2s, n2r = self.last_send, self.last_recv
                self._ahead_no ^= 1
                rk2 = self._recv_keys_ahead[self._ahead_no].get(n2r)
                ops.append((rk2, self._send_keys[wb2][:n2s], rs2, ss2))
                self._ahead = dict(batch=next_batch, wb=wb2, send=ss2, recv=rs2, any=any2,
                                   n_send=n2s, n_recv=n2r, keys=rk2)
                self.early_key_exchanges += 1
                self.last_send, self.last_recv = n_send, n_recv
            self._a2a_ops(ops)
        self._apply_groups(recv_keys, [(g, m, Sg) for (g, m), Sg in zip(ins, groups)], offsets)
        e.w_finish()
        self.bytes_moved += (n_send + n_recv) * (8 + 4 * ps + 4 * S * gw)
        return True

    def _apply_groups(self, recv_keys, groups, offsets, buf: int = 0) -> None:
        """Owner apply of one step's pushes: groups = [(grads, masks, slices)]
        per slice group.  One group: s_apply (sources in order).  Several: the
        pushes go in (source, slice) order -- source by source, each source's
        groups in order -- the order of one S-slice step."""
        e = self.engine
        if len(groups) == 1:
            g, m, Sg = groups[0]
            e.s_apply(recv_keys, g, m, offsets, Sg, buf=buf)
            return
        W = len(offsets) - 1
        for src in range(W):
            if offsets[src + 1] <= offsets[src]:
                continue
            # only this source's range is non-empty
            offs = [offsets[src]] * (src + 1) + [offsets[src + 1]] * (W - src)
            for g, m, Sg in groups:
                e.s_apply(recv_keys, g, m, offs, Sg, buf=buf)

    def eval_step(self, batch: Batch, pctr: Optional[torch.Tensor] = None) -> Optional[torch.Tensor]:
        """Forward-only sharded step (keys looked up, never inserted).  Every
        rank must call it (a rank without test data passes an empty batch);
        returns None on every rank when no rank had rows (the counts exchange
        says so: the evaluation loop's end, without another collective)."""
        e = self.engine
        if self._native is not None:
            batch.check(e.device)
            if pctr is None:
                pctr = torch.empty(batch.rows, dtype=torch.float32, device=e.device)
            e._sync_stream()
            ok = self._native.eval_step(batch.view(), pctr.data_ptr() if batch.rows else 0)
            return pctr if ok else None
        # (keys exchanged ahead for a training batch no step will take now:
        # every rank drops them at the same point)
        self._ahead = None
        wb, send_splits, recv_splits, _, any_data = self._take(batch)
        if not any_data:
            return None
        if pctr is None:
            pctr = torch.empty(batch.rows, dtype=torch.float32, device=e.device)
        recv_keys = self._exchange_keys(wb, send_splits, recv_splits)
        ps = e.value_width  # floats per pulled value row
        vals = self._vals_out[0].get(self.last_recv * ps).view(self.last_recv, ps)
        e.s_pull(recv_keys, self.last_recv, vals, insert=False, buf=0)
        pulled = self._pulled.get(self.last_send * ps).view(self.last_send, ps)
        self._a2a(pulled, vals, send_splits, recv_splits)
        e.w_forward(batch, pulled, self.last_send, pctr if batch.rows else None, wb=wb)
        return pctr

    def close(self) -> None:
        """Release the native step and communicator (before the process group
        goes)."""
        if self._native is not None or self._comm is not None:
            if self.engine.is_gpu:
                torch.cuda.synchronize(self.engine.device)
            self.__dict__["_native"] = None
            self._comm = None
