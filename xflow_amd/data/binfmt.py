"""Binary CSR shards (.xfb): libffm text parsed once, then read at memory speed.

The reference re-parses its libffm text in every epoch
(LoadData::load_minibatch_hash_data_fread, src/io/load_data_from_disk.cc:
103-210); at ~2 M rows/s per core (csrc/io/reader.cpp, a few times that with
the parallel parse) that is two orders of magnitude slower than one MI355X
trains.  An .xfb shard holds exactly what the parser produces -- labels, row
offsets, hashed keys (std::hash of the feature text, the same keys as the text
path), field ids -- so an epoch maps the arrays instead of parsing them.

Layout (little endian):

    b"XFLOWCSR"                                   magic, 8 B
    u64 version (1; 2 = compact keys), rows, nnz,
        flags (bit 0: fgid present, bit 1: compact keys)
    f32 labels[rows]   (padded to 8 B)
    i64 row_ptr[rows + 1]
    u64 keys[nnz]      (compact: u32 keys[nnz], padded to 8 B)
    i32 fgid[nnz]      (flag bit 0)

Compact keys: when every key of a shard is below 2^32 (features hashed into
a space of at most 2^32, e.g. Criteo-1TB's 1e9), the writer stores them as
u32 (``compact="auto"``).  The streamed input path then moves half the key
bytes over the host link -- the bound of that path -- and the device widens
them to u64 inside its field-major transpose (csrc/hip/kernels_layout.hip).

    python -m xflow_amd.data.binfmt convert data/small_train-00000 /tmp/small_train-00000.xfb

The trainer reads ``<prefix>-%05d.xfb`` when it exists next to (or instead of)
the text shard, in blocks of ``--block-rows`` rows.
"""
from __future__ import annotations

import argparse
import os
import struct
import sys
import tempfile
from typing import Optional

import numpy as np

MAGIC = b"XFLOWCSR"
VERSION = 1
VERSION_COMPACT = 2
FLAG_FGID, FLAG_COMPACT = 1, 2
_HDR = struct.Struct("<8sQQQQ")


def _pad8(n: int) -> int:
    return (n + 7) & ~7


def _compact_ok(keys: np.ndarray, compact) -> bool:
    if compact == "auto":
        return len(keys) > 0 and int(keys.max()) < (1 << 32)
    return bool(compact)


def write(dst: str, labels: np.ndarray, row_ptr: np.ndarray, keys: np.ndarray,
          fgid: Optional[np.ndarray] = None, compact="auto") -> None:
    """Write one shard from whole arrays (row_ptr starts at 0, ends at nnz).
    compact: store u32 keys -- "auto" when every key is below 2^32."""
    labels = np.ascontiguousarray(labels, dtype=np.float32)
    row_ptr = np.ascontiguousarray(row_ptr, dtype=np.int64)
    keys = np.ascontiguousarray(keys).view(np.uint64)
    rows, nnz = len(labels), len(keys)
    if len(row_ptr) != rows + 1 or row_ptr[0] != 0 or row_ptr[-1] != nnz:
        raise ValueError("row_ptr must have rows+1 offsets from 0 to nnz")
    cmp = _compact_ok(keys, compact)
    if cmp and nnz and int(keys.max()) >= (1 << 32):
        raise ValueError("compact keys must be below 2^32")
    flags = (FLAG_FGID if fgid is not None else 0) | (FLAG_COMPACT if cmp else 0)
    with open(dst + ".tmp", "wb") as f:
        f.write(_HDR.pack(MAGIC, VERSION_COMPACT if cmp else VERSION, rows, nnz, flags))
        f.write(labels.tobytes())
        f.write(b"\0" * (_pad8(4 * rows) - 4 * rows))
        f.write(row_ptr.tobytes())
        if cmp:
            f.write(keys.astype(np.uint32).tobytes())
            f.write(b"\0" * (_pad8(4 * nnz) - 4 * nnz))
        else:
            f.write(keys.tobytes())
        if fgid is not None:
            f.write(np.ascontiguousarray(fgid, dtype=np.int32).tobytes())
    os.replace(dst + ".tmp", dst)


def convert(src: str, dst: str, block_bytes: int = 64 << 20, threads: int = 0,
            compact="auto") -> dict:
    """libffm text -> .xfb, streaming block by block through the native reader
    (parallel parse); arrays are staged in temporary files next to dst.
    compact="auto" stores u32 keys when every key is below 2^32."""
    from xflow_amd import native

    r = native.load().BlockReader(src, block_bytes)
    if threads > 0:
        r.parse_threads = threads
    d = os.path.dirname(os.path.abspath(dst)) or "."
    parts = {k: tempfile.TemporaryFile(dir=d) for k in ("labels", "row_ptr", "keys", "fgid")}
    rows = nnz = 0
    kmax = 0
    parts["row_ptr"].write(np.zeros(1, np.int64).tobytes())
    while True:
        b = r.next()
        if b is None:
            break
        parts["labels"].write(np.asarray(b["labels"], np.float32).tobytes())
        parts["row_ptr"].write((np.asarray(b["row_ptr"][1:], np.int64) + nnz).tobytes())
        k = np.asarray(b["keys"]).view(np.uint64)
        if len(k):
            kmax = max(kmax, int(k.max()))
        parts["keys"].write(k.tobytes())
        parts["fgid"].write(np.asarray(b["fgid"], np.int32).tobytes())
        rows += len(b["labels"])
        nnz += len(b["keys"])
    cmp = (nnz > 0 and kmax < (1 << 32)) if compact == "auto" else bool(compact)
    if cmp and kmax >= (1 << 32):
        raise ValueError("compact keys must be below 2^32")
    with open(dst + ".tmp", "wb") as f:
        f.write(_HDR.pack(MAGIC, VERSION_COMPACT if cmp else VERSION, rows, nnz,
                          FLAG_FGID | (FLAG_COMPACT if cmp else 0)))
        for k in ("labels", "row_ptr", "keys", "fgid"):
            fp = parts[k]
            fp.seek(0)
            while True:
                chunk = fp.read(64 << 20)
                if not chunk:
                    break
                if k == "keys" and cmp:
                    chunk = np.frombuffer(chunk, np.uint64).astype(np.uint32).tobytes()
                f.write(chunk)
            if k == "labels":
                f.write(b"\0" * (_pad8(4 * rows) - 4 * rows))
            if k == "keys" and cmp:
                f.write(b"\0" * (_pad8(4 * nnz) - 4 * nnz))
            fp.close()
    os.replace(dst + ".tmp", dst)
    return {"rows": rows, "nnz": nnz}


class Shard:
    """Memory-mapped .xfb shard (zero-copy numpy views)."""

    def __init__(self, path: str):
        with open(path, "rb") as f:
            magic, ver, rows, nnz, flags = _HDR.unpack(f.read(_HDR.size))
        if magic != MAGIC or ver not in (VERSION, VERSION_COMPACT):
            raise ValueError(f"{path}: not an xflow CSR shard")
        self.path, self.rows, self.nnz = path, rows, nnz
        self.compact = bool(flags & FLAG_COMPACT)
        off = _HDR.size
        self.labels = np.memmap(path, np.float32, "r", off, (rows,))
        off += _pad8(4 * rows)
        self.row_ptr = np.memmap(path, np.int64, "r", off, (rows + 1,))
        off += 8 * (rows + 1)
        kt = np.uint32 if self.compact else np.uint64  # (compact: u32, widened on use)
        self.keys = np.memmap(path, kt, "r", off, (nnz,)) if nnz else np.zeros(0, kt)
        off += _pad8(4 * nnz) if self.compact else 8 * nnz
        self.fgid = (np.memmap(path, np.int32, "r", off, (nnz,)) if (flags & FLAG_FGID) and nnz
                     else np.zeros(nnz, np.int32))


class ShardReader:
    """Blocks of ``block_rows`` rows of an .xfb shard, in the native readers'
    dict layout (row_ptr rebased to int32 per block; keys / fgid / labels are
    views of the mapping)."""

    def __init__(self, path: str, block_rows: int = 65536):
        if block_rows <= 0:
            raise ValueError("block_rows must be positive")
        self.shard = Shard(path)
        self.block_rows = int(block_rows)
        self.r = 0

    def next(self) -> Optional[dict]:
        s = self.shard
        if self.r >= s.rows:
            return None
        r0, r1 = self.r, min(self.r + self.block_rows, s.rows)
        self.r = r1
        k0, k1 = int(s.row_ptr[r0]), int(s.row_ptr[r1])
        return {"row_ptr": (np.asarray(s.row_ptr[r0:r1 + 1]) - k0).astype(np.int32),
                "keys": s.keys[k0:k1], "fgid": s.fgid[k0:k1], "labels": s.labels[r0:r1]}


def max_block(path: str, block_rows: int):
    """(rows, nnz) of the largest block of ``block_rows`` rows in a shard."""
    s = Shard(path)
    if s.rows == 0:
        return 0, 0
    starts = np.arange(0, s.rows, block_rows)
    ends = np.minimum(starts + block_rows, s.rows)
    rp = np.asarray(s.row_ptr)
    return int((ends - starts).max()), int((rp[ends] - rp[starts]).max())


def shard_file(path: str) -> Optional[str]:
    """The .xfb shard for a text shard path (or the path itself), if present."""
    if path.endswith(".xfb"):
        return path if os.path.exists(path) else None
    return path + ".xfb" if os.path.exists(path + ".xfb") else None


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="python -m xflow_amd.data.binfmt", description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    sub = ap.add_subparsers(dest="cmd", required=True)
    c = sub.add_parser("convert", help="libffm text shard -> .xfb")
    c.add_argument("src")
    c.add_argument("dst")
    c.add_argument("--block-bytes", type=int, default=64 << 20)
    c.add_argument("--threads", type=int, default=0)
    c.add_argument("--compact", choices=["auto", "on", "off"], default="auto",
                   help="u32 keys (all keys below 2^32): half the streamed H2D bytes")
    a = ap.parse_args(argv)
    info = convert(a.src, a.dst, a.block_bytes, a.threads,
                   {"auto": "auto", "on": True, "off": False}[a.compact])
    print(f"{a.dst}: {info['rows']} rows, {info['nnz']} features")
    return 0


if __name__ == "__main__":
    sys.exit(main())
