"""Host blocks -> device blocks: pinned staging ring, parallel host copy,
H2D on a copy stream, one block ahead of the step that consumes it.

The reference trains straight out of the parser's vectors on the CPU
(lr_worker.cc:179-205: load a block, then fan its slices out to the thread
pool), so it has no upload at all.  On MI355X the step of a 262144-row block
takes ~0.5 ms on the GPU while the block's keys alone are 80 MB, so the input
path is what bounds real-data training.  ``BlockStream`` keeps it off the
critical path:

* a background thread pulls the next host block (text parser or .xfb
  mapping) and copies its arrays into a free pinned slot, split over
  ``copy_threads`` threads (numpy releases the GIL for the copies);
* the consumer issues the slot's H2D copies on a dedicated HIP stream,
  makes the compute stream wait for them, and returns the slot to the free
  list behind an event -- the producer reuses it only after the DMA read it.

With ``nbuf`` slots, block t+1 is being copied on the host and block t is on
the DMA engine while step t-1 runs.
"""
from __future__ import annotations

import queue
import threading
import time
from concurrent.futures import ThreadPoolExecutor
from typing import Callable, Dict, Optional

import numpy as np
import torch

_DTYPES = {"keys": torch.int64, "labels": torch.float32, "row_ptr": torch.int32,
           "fgid": torch.int32, "packed": torch.uint8}
_CHUNK = 4 << 20  # bytes per host-copy task


def _np(a) -> np.ndarray:
    a = np.asarray(a)
    if a.dtype == np.uint64:
        return a.view(np.int64)
    return a.view(np.int32) if a.dtype == np.uint32 else a  # (compact .xfb keys)


class BlockStream:
    """Iterator of device blocks ({"keys", "labels", "row_ptr", ["fgid"]} as
    device tensors, plus "rows", "nnz", "nnz_per_row", "row_ptr_host") fed
    by ``source()`` returning host blocks (dicts of numpy arrays) or None."""

    def __init__(self, source: Callable[[], Optional[dict]], device: torch.device,
                 with_fgid: bool, nbuf: int = 3, copy_threads: int = 8, timeline=None):
        self.device = device
        self.timeline = timeline  # utils.trace.StreamTimeline: "h2d" intervals
        self.names = ["keys", "labels", "row_ptr"] + (["fgid"] if with_fgid else [])
        self.copy = torch.cuda.Stream(device)
        self.pool = ThreadPoolExecutor(max(1, copy_threads))
        self.pinned = [dict() for _ in range(nbuf)]
        self.free: "queue.Queue" = queue.Queue()
        for i in range(nbuf):
            self.free.put((i, None))
        self.ready: "queue.Queue" = queue.Queue()
        self.error: Optional[BaseException] = None
        self.stage_s = 0.0  # host time spent filling pinned slots (the timeline reports it)
        self.stop = False
        self.thread = threading.Thread(target=self._produce, args=(source,), daemon=True)
        self.thread.start()

    # ------------------------------------------------------------ producer
    def _buf(self, slot: int, name: str, n: int, dtype: torch.dtype) -> torch.Tensor:
        t = self.pinned[slot].get(name)
        if t is None or t.numel() < n or t.dtype != dtype:
            t = torch.empty(max(n, 1) + (max(n, 1) >> 3), dtype=dtype, pin_memory=True)
            self.pinned[slot][name] = t
        return t

    def _fill(self, dst: np.ndarray, src: np.ndarray) -> None:
        step = max(1, _CHUNK // max(src.itemsize, 1))
        if len(src) <= step:
            np.copyto(dst, src)
            return
        futs = [self.pool.submit(np.copyto, dst[i:i + step], src[i:i + step])
                for i in range(0, len(src), step)]
        for f in futs:
            f.result()

    def _produce(self, source) -> None:
        try:
            while not self.stop:
                blk = source()
                if blk is None:
                    break
                slot, ev = self.free.get()
                if ev is not None:
                    ev.synchronize()  # the previous H2D from this slot has read it
                meta = {}
                t0 = time.perf_counter()
                # a packed (v3 .xfb) block is one byte range: one copy, one H2D
                names = ["packed"] if "packed" in blk else self.names
                for name in names:
                    a = _np(blk[name])
                    # compact u32 keys travel as int32: half the H2D bytes, widened
                    # on the device (Batch.to_field_major / engine.widen_keys)
                    dt = torch.int32 if name == "keys" and a.dtype == np.int32 else _DTYPES[name]
                    buf = self._buf(slot, name, len(a), dt)
                    self._fill(buf.numpy()[:len(a)], a)
                    meta[name] = len(a)
                self.stage_s += time.perf_counter() - t0
                if "packed" in blk:
                    self.ready.put((slot, meta, None, blk["shard"].F,
                                    {"rows": blk["rows"], "shard": blk["shard"]}))
                    continue
                rp = _np(blk["row_ptr"])
                lens = np.diff(rp) if len(rp) > 1 else np.zeros(0, rp.dtype)
                F = int(lens[0]) if len(lens) and lens[0] > 0 and np.all(lens == lens[0]) else 0
                self.ready.put((slot, meta, np.array(rp, copy=True), F, None))
        except BaseException as e:  # surfaced by next()
            self.error = e
        self.ready.put(None)

    # ------------------------------------------------------------ consumer
    def next(self) -> Optional[dict]:
        item = self.ready.get()
        if item is None:
            if self.error is not None:
                raise self.error
            self.ready.put(None)  # stay exhausted
            return None
        slot, meta, rp_host, F, extra = item
        names = list(meta)
        compute = torch.cuda.current_stream(self.device)
        # No wait for the compute stream: block t+1's copies run while step t
        # computes.  The pinned slot is reused only after the event behind its
        # DMA, and the device tensors are allocated from the copy stream's
        # pool with record_stream(compute) -- the caching allocator hands a
        # block back only once the steps that read it have finished.
        out: Dict[str, object] = {}
        with torch.cuda.stream(self.copy):
            if self.timeline is not None:
                self.timeline.begin("h2d", self.copy)
            for name in names:
                out[name] = self.pinned[slot][name][:meta[name]].to(self.device, non_blocking=True)
            if self.timeline is not None:
                self.timeline.end("h2d", self.copy)
            ev = torch.cuda.Event()
            ev.record(self.copy)
        self.free.put((slot, ev))
        compute.wait_stream(self.copy)
        for name in names:
            out[name].record_stream(compute)
        if extra is not None:  # (packed: expanded by the trainer, Engine.unpack_packed)
            out.update(extra)
            out["nnz_per_row"] = F
            return out
        out["row_ptr_host"] = rp_host
        out["rows"] = len(rp_host) - 1
        out["nnz_per_row"] = F
        return out

    def close(self) -> None:
        self.stop = True
        while self.thread.is_alive():
            try:
                item = self.ready.get(timeout=0.05)
                if item is not None:
                    self.free.put((item[0], None))
            except queue.Empty:
                pass
        self.pool.shutdown(wait=True)
