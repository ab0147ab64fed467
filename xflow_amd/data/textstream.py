"""libffm text parsed on the GPU: raw blocks -> pinned ring -> H2D -> CSR.

The reference parses each 2 MB text block on its training threads
(/root/reference/src/io/load_data_from_disk.cc:103-210) and the native host
parser here (csrc/io/reader.cpp) reaches ~1.3 GB/s on 8 CPUs -- ~5 M Criteo
rows/s, two orders of magnitude below one MI355X step.  ``TextStream`` moves
the tokenising to the device:

* ``TextBlocks`` cuts the file into blocks with the reference's protocol
  (a buffer of ``block_bytes``: read up to block_bytes - 1 - carry bytes after
  the carried tail, cut after the last '\\n' when the buffer filled, carry the
  rest; BlockReader::fill_block) -- so blocks, and the rows the slicing rule
  drops from each, are the reference's -- reading straight into a pinned slot;
* a producer thread fills the slots (``readinto`` from the page cache is the
  only host copy), the consumer sends a slot's bytes on a copy stream and the
  compute stream parses them (Engine.parse_text: kernels_parse.hip) into
  device CSR arrays: keys = std::hash of the feature text, labels, field ids,
  row offsets -- bit-equal to reader.cpp (tests/test_gpu_parse.py).

A block the producer reads overlaps the previous block's upload and parse and
the steps that train on it.
"""
from __future__ import annotations

import os
import queue
import threading
import time
from typing import Optional

from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch


class TextBlocks:
    """Raw text blocks of a file with BlockReader::fill_block's protocol.  A
    block's fresh bytes are read with ``read_threads`` positional reads of
    contiguous pieces in parallel (the page-cache copy is the bound of a
    single reader: ~15 GB/s here)."""

    min_piece = 4 << 20  # bytes per parallel read at least

    def __init__(self, path: str, block_bytes: int, read_threads: int = 8):
        self.path = path
        self.block_bytes = max(2, int(block_bytes))
        self.fd = os.open(path, os.O_RDONLY)
        self.pos = 0
        self.carry = b""
        self.eof = False
        self.read_threads = max(1, int(read_threads))
        self.pool = (ThreadPoolExecutor(self.read_threads) if self.read_threads > 1 else None)

    def close(self) -> None:
        if self.pool is not None:
            self.pool.shutdown(wait=True)
        os.close(self.fd)

    def _pread(self, mv, off: int) -> int:
        got = 0
        while got < len(mv):
            k = os.preadv(self.fd, [mv[got:]], off + got)
            if k <= 0:
                break
            got += k
        return got

    def _read(self, mv) -> int:
        """Fill mv from the file position (parallel pieces); bytes read."""
        want = len(mv)
        piece = max(self.min_piece, -(-want // self.read_threads))
        if self.pool is None or want <= piece:
            got = self._pread(mv, self.pos)
        else:
            cuts = list(range(0, want, piece)) + [want]
            futs = [self.pool.submit(self._pread, mv[a:b], self.pos + a)
                    for a, b in zip(cuts[:-1], cuts[1:])]
            sizes = [f.result() for f in futs]
            got = 0
            for (a, b), k in zip(zip(cuts[:-1], cuts[1:]), sizes):
                got += k
                if k < b - a:  # end of file inside this piece
                    break
        self.pos += got
        if got < want:
            self.eof = True
        return got

    def read_into(self, buf: np.ndarray) -> int:
        """Next block into buf[:block_bytes] (uint8); returns its length (0: end)."""
        B = self.block_bytes
        c = len(self.carry)
        if c:
            buf[:c] = np.frombuffer(self.carry, dtype=np.uint8)
        top = c
        mv = memoryview(buf)
        if top < B - 1 and not self.eof:
            top += self._read(mv[top:B - 1])
        n = top
        self.carry = b""
        if top + 1 == B:  # buffer full: cut after the last newline
            m = top
            step = 1 << 16
            while m > 0:
                lo = max(0, m - step)
                k = bytes(mv[lo:m]).rfind(b"\n")
                if k >= 0:
                    m = lo + k + 1
                    break
                m = lo
            if m > 0:
                n = m
                self.carry = bytes(mv[m:top])
        return n


class TextStream:
    """Iterator of device blocks ({"keys", "labels", "row_ptr", "fgid"} device
    tensors + "rows", "nnz_per_row", "nnz_used") parsed on the GPU from the
    libffm file at ``path``.  ``row_mod``: the trainer's slice count (the
    used rows' occurrence count comes back with the parse)."""

    def __init__(self, engine, path: str, block_bytes: int, row_mod: int = 1, nbuf: int = 3,
                 timeline=None, read_threads: int = 8):
        self.engine = engine
        self.device = engine.device
        self.blocks = TextBlocks(path, block_bytes, read_threads)
        self.row_mod = max(1, int(row_mod))
        self.timeline = timeline
        cap = self.blocks.block_bytes + 64
        self.pinned = [torch.empty(cap, dtype=torch.uint8, pin_memory=self.device.type == "cuda")
                       for _ in range(nbuf)]
        self.copy = torch.cuda.Stream(self.device) if self.device.type == "cuda" else None
        self.free: "queue.Queue" = queue.Queue()
        for i in range(nbuf):
            self.free.put((i, None))
        self.ready: "queue.Queue" = queue.Queue()
        self.error: Optional[BaseException] = None
        self.stage_s = 0.0   # host seconds reading blocks into the pinned slots
        self.parse_s = 0.0   # host seconds waiting for parses (their counts)
        self.stop = False
        # (device output arrays: one set per block, _arrays; a line needs >= 2
        # bytes, a feature token >= 4 (" a:b"))
        self._texts = [None, None]  # device text buffers (block t parses while t+1 uploads)
        self._tb = 0
        self._pending = None        # an uploaded block not yet parsed
        self.thread = threading.Thread(target=self._produce, daemon=True)
        self.thread.start()

    def _produce(self) -> None:
        try:
            while not self.stop:
                slot, ev = self.free.get()
                if ev is not None:
                    ev.synchronize()  # the previous upload of this slot has read it
                t0 = time.perf_counter()
                n = self.blocks.read_into(self.pinned[slot].numpy())
                self.stage_s += time.perf_counter() - t0
                if n == 0:
                    self.free.put((slot, None))
                    break
                self.ready.put((slot, n))
        except BaseException as e:  # surfaced by next()
            self.error = e
        self.ready.put(None)

    def _arrays(self, n: int):
        """Fresh output arrays for one block.  Every block owns its arrays (the
        caching allocator on the compute stream recycles them once the block's
        tensors die, stream-ordered): a multi-rank step announces block t+1 --
        which parses right away -- before block t trains, and ``--resident``
        keeps the first epoch's blocks, so reused arrays would alias them."""
        rows = n // 2 + 2
        nnz = n // 4 + 2
        dev = self.device
        return {"keys": torch.empty(nnz, dtype=torch.int64, device=dev),
                "fgid": torch.empty(nnz, dtype=torch.int32, device=dev),
                "row_ptr": torch.empty(rows + 1, dtype=torch.int32, device=dev),
                "labels": torch.empty(rows, dtype=torch.float32, device=dev)}

    def next(self) -> Optional[dict]:
        while True:
            if self._pending is None:
                item = self.ready.get()
                if item is None:
                    if self.error is not None:
                        raise self.error
                    self.ready.put(None)
                    return None
                self._pending = self._upload(*item)
            cur, self._pending = self._pending, None
            if self.device.type == "cuda":
                # the next block's upload goes out now when it is read already:
                # its DMA then overlaps this block's parse and step
                try:
                    item = self.ready.get_nowait()
                except queue.Empty:
                    item = False
                if item is None:
                    self.ready.put(None)
                elif item is not False:
                    self._pending = self._upload(*item)
            blk = self._parse(*cur)
            if blk is not None:
                return blk
            # (a block of only malformed lines: the next one, as BlockReader)

    def _upload(self, slot: int, n: int):
        """H2D of a read slot into the next of two device text buffers (copy
        stream); the host synced on that buffer's previous parse already
        (parse_text waits for its counts)."""
        src = self.pinned[slot]
        if self.device.type != "cuda":
            return (src, n, None, slot)
        self._tb ^= 1
        buf = self._texts[self._tb]
        if buf is None or buf.numel() < n + 64:
            # (the parse kernels read aligned 16-byte chunks up to 32 bytes past the block)
            buf = torch.empty(self.blocks.block_bytes + 64, dtype=torch.uint8, device=self.device)
            self._texts[self._tb] = buf
        with torch.cuda.stream(self.copy):
            if self.timeline is not None:
                self.timeline.begin("h2d", self.copy)
            buf[:n].copy_(src[:n], non_blocking=True)
            if self.timeline is not None:
                self.timeline.end("h2d", self.copy)
            ev = torch.cuda.Event()
            ev.record(self.copy)
        self.free.put((slot, ev))
        return (buf, n, ev, slot)

    def _parse(self, text: torch.Tensor, n: int, ev, slot: int) -> Optional[dict]:
        e = self.engine
        if ev is not None:
            torch.cuda.current_stream(self.device).wait_event(ev)
        o = self._arrays(n)
        t0 = time.perf_counter()
        rows, nnz, lmin, lmax, nused = e.parse_text(text, n, o, self.row_mod)
        self.parse_s += time.perf_counter() - t0
        if ev is None:  # (CPU: parsed from the slot itself)
            self.free.put((slot, None))
        if rows == 0:
            return None
        return {"keys": o["keys"][:nnz], "labels": o["labels"][:rows],
                "row_ptr": o["row_ptr"][:rows + 1], "fgid": o["fgid"][:nnz], "rows": rows,
                "nnz_per_row": int(lmin) if lmin == lmax else 0, "nnz_used": int(nused)}

    def close(self) -> None:
        self.stop = True
        while self.thread.is_alive():
            try:
                item = self.ready.get(timeout=0.05)
                if item is not None:
                    self.free.put((item[0], None))
            except queue.Empty:
                pass
        self.blocks.close()


def parse_text_file(engine, path: str, block_bytes: int = 2 << 20):
    """Every block of a libffm file parsed on the engine's device, as host
    numpy CSR dicts (tests / tools)."""
    s = TextStream(engine, path, block_bytes)
    out = []
    try:
        while True:
            b = s.next()
            if b is None:
                break
            # (host copies of the block's device arrays)
            out.append({k: (v.cpu().numpy().copy() if isinstance(v, torch.Tensor) else v)
                        for k, v in b.items()})
    finally:
        s.close()
    return out


__all__ = ["TextBlocks", "TextStream", "parse_text_file"]
