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

Packed field-major blocks (version 3, ``convert --packed`` / ``write_packed``;
fixed-width shards, every row F features, each column one field):

    b"XFLOWCSR", u64 version (3), rows, nnz, flags (bit 2: packed)
    u64 F, block_rows, nblocks
    F x {u32 width, u32 mode, u64 dict_size, u64 dict_off, i32 fgid, 4 pad}
    dictionaries (u64 keys, 16-B aligned), u64 block_off[nblocks + 1]
    blocks: u8 labels[rows_b], then per field a column of rows_b codes of
            `width` bytes (each part 16-B aligned)

A field with at most 65536 distinct keys is dictionary-coded (u8 codes up to
256 keys, u16 above); otherwise its keys are stored directly (u32 when below
2^32, else u64).  On Criteo-shaped data (13 binned integer fields, 26
categorical ones of which 18 have < 65536 values) a row is ~74 bytes against
168 for the compact v2 layout: the host link -- the streamed path's bound --
carries less than half, and the device expands a block into the engine's
field-major batch in one pass (Backend::unpack_block,
csrc/hip/kernels_layout.hip).

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
VERSION_PACKED = 3
FLAG_FGID, FLAG_COMPACT, FLAG_PACKED = 1, 2, 4
_HDR = struct.Struct("<8sQQQQ")
_PHDR = struct.Struct("<QQQ")          # F, block_rows, nblocks
_FDESC = struct.Struct("<IIQQi4x")     # width, mode (0 direct, 1 dictionary), dict size / offset, fgid
DICT_MAX = 65536


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


def _al16(n: int) -> int:
    return (n + 15) & ~15


def packed_columns(rows_b: int, widths) -> tuple:
    """(column byte offsets, block bytes) of a packed block of rows_b rows."""
    off = _al16(rows_b)  # u8 labels
    cols = []
    for w in widths:
        cols.append(off)
        off += _al16(rows_b * int(w))
    return cols, off


def write_packed(dst: str, labels: np.ndarray, keys: np.ndarray, fgid_cols=None,
                 block_rows: int = 262144) -> dict:
    """Write a version-3 packed shard from labels [rows] and row-major keys
    [rows][F] (u64); fgid_cols: the field id of each column (default 0..F-1).
    Returns {rows, F, widths, bytes_per_row}."""
    keys = np.ascontiguousarray(keys).view(np.uint64)
    if keys.ndim != 2:
        raise ValueError("write_packed: keys must be [rows][F]")
    rows, F = keys.shape
    if not 1 <= F <= 64:
        raise ValueError("write_packed: 1..64 fields")
    lab = (np.asarray(labels, dtype=np.float32).reshape(-1) != 0).astype(np.uint8)
    if len(lab) != rows:
        raise ValueError("write_packed: one label per row")
    fg = np.arange(F, dtype=np.int32) if fgid_cols is None else np.asarray(fgid_cols, np.int32)
    widths, modes, dicts, codes = [], [], [], []
    for f in range(F):
        col = keys[:, f]
        u = np.unique(col)
        if len(u) <= DICT_MAX:
            w = 1 if len(u) <= 256 else 2
            widths.append(w)
            modes.append(1)
            dicts.append(u)
            codes.append(np.searchsorted(u, col).astype(np.uint8 if w == 1 else np.uint16))
        else:
            big = len(u) and int(u[-1]) >= (1 << 32)
            widths.append(8 if big else 4)
            modes.append(0)
            dicts.append(None)
            codes.append(col if big else col.astype(np.uint32))
    block_rows = max(1, min(int(block_rows), max(rows, 1)))
    nblocks = (rows + block_rows - 1) // block_rows
    head = _HDR.size + _PHDR.size + F * _FDESC.size
    off = _al16(head)
    doffs = []
    for d in dicts:
        doffs.append(off if d is not None else 0)
        off += _al16(8 * len(d)) if d is not None else 0
    tab_off = off
    off = _al16(off + 8 * (nblocks + 1))
    boff = [off]
    for b in range(nblocks):
        rb = min(block_rows, rows - b * block_rows)
        off += packed_columns(rb, widths)[1]
        boff.append(off)
    with open(dst + ".tmp", "wb") as fp:
        fp.write(_HDR.pack(MAGIC, VERSION_PACKED, rows, rows * F, FLAG_PACKED | FLAG_FGID))
        fp.write(_PHDR.pack(F, block_rows, nblocks))
        for f in range(F):
            fp.write(_FDESC.pack(widths[f], modes[f], len(dicts[f]) if dicts[f] is not None else 0,
                                 doffs[f], int(fg[f])))
        fp.write(b"\0" * (_al16(head) - head))
        for d in dicts:
            if d is not None:
                fp.write(d.tobytes())
                fp.write(b"\0" * (_al16(8 * len(d)) - 8 * len(d)))
        assert fp.tell() == tab_off
        fp.write(np.asarray(boff, np.uint64).tobytes())
        fp.write(b"\0" * (boff[0] - tab_off - 8 * (nblocks + 1)))
        for b in range(nblocks):
            r0, r1 = b * block_rows, min((b + 1) * block_rows, rows)
            rb = r1 - r0
            fp.write(lab[r0:r1].tobytes())
            fp.write(b"\0" * (_al16(rb) - rb))
            for f in range(F):
                c = np.ascontiguousarray(codes[f][r0:r1])
                fp.write(c.tobytes())
                fp.write(b"\0" * (_al16(rb * widths[f]) - rb * widths[f]))
            assert fp.tell() == boff[b + 1]
    os.replace(dst + ".tmp", dst)
    return {"rows": rows, "F": F, "widths": widths,
            "bytes_per_row": (boff[-1] - boff[0]) / max(rows, 1)}


def convert_packed(src: str, dst: str, block_bytes: int = 64 << 20, threads: int = 0,
                   block_rows: int = 262144) -> dict:
    """libffm text (or a v1 / v2 .xfb) -> packed version 3.  Every row must
    hold the same number of features and each column one field id."""
    if src.endswith(".xfb") or version_of(src) in (VERSION, VERSION_COMPACT):
        sh = Shard(src)
        lens = np.diff(np.asarray(sh.row_ptr))
        labels, keys, fg = np.asarray(sh.labels), np.asarray(sh.keys), np.asarray(sh.fgid)
    else:
        from xflow_amd import native

        r = native.load().BlockReader(src, block_bytes)
        if threads > 0:
            r.parse_threads = threads
        parts = {"labels": [], "keys": [], "fgid": [], "lens": []}
        while True:
            b = r.next()
            if b is None:
                break
            parts["labels"].append(np.asarray(b["labels"], np.float32))
            parts["keys"].append(np.asarray(b["keys"]).view(np.uint64))
            parts["fgid"].append(np.asarray(b["fgid"], np.int32))
            parts["lens"].append(np.diff(np.asarray(b["row_ptr"])))
        labels = np.concatenate(parts["labels"]) if parts["labels"] else np.zeros(0, np.float32)
        keys = np.concatenate(parts["keys"]) if parts["keys"] else np.zeros(0, np.uint64)
        fg = np.concatenate(parts["fgid"]) if parts["fgid"] else np.zeros(0, np.int32)
        lens = np.concatenate(parts["lens"]) if parts["lens"] else np.zeros(0, np.int64)
    if len(lens) == 0 or not np.all(lens == lens[0]) or lens[0] <= 0:
        raise ValueError("convert --packed: every row must hold the same number of features")
    F = int(lens[0])
    fgm = fg.reshape(-1, F)
    if not np.all(fgm == fgm[0]):
        raise ValueError("convert --packed: each column must hold one field id")
    return write_packed(dst, labels, keys.astype(np.uint64).reshape(-1, F), fgm[0], block_rows)


class PackedShard:
    """Memory-mapped version-3 shard: per-field widths / dictionaries and the
    raw bytes of each block (zero-copy)."""

    def __init__(self, path: str):
        with open(path, "rb") as f:
            magic, ver, rows, nnz, flags = _HDR.unpack(f.read(_HDR.size))
            if magic != MAGIC or ver != VERSION_PACKED:
                raise ValueError(f"{path}: not a packed xflow shard")
            F, block_rows, nblocks = _PHDR.unpack(f.read(_PHDR.size))
            desc = [_FDESC.unpack(f.read(_FDESC.size)) for _ in range(F)]
        self.path, self.rows, self.nnz = path, rows, nnz
        self.F, self.block_rows, self.nblocks = int(F), int(block_rows), int(nblocks)
        self.widths = [int(d[0]) for d in desc]
        self.fgid_cols = [int(d[4]) for d in desc]
        self.mm = np.memmap(path, np.uint8, "r")
        self.dicts = [np.ndarray((int(d[2]),), np.uint64, self.mm, int(d[3])) if d[1] == 1 else None
                      for d in desc]
        head = _al16(_HDR.size + _PHDR.size + F * _FDESC.size)
        tab = head + sum(_al16(8 * len(x)) for x in self.dicts if x is not None)
        self.block_off = np.ndarray((self.nblocks + 1,), np.uint64, self.mm, tab)

    def device_dicts(self, device) -> list:
        """Per field: the device address of its dictionary (0: direct keys),
        uploaded once per device."""
        import torch

        key = str(device)
        cache = self.__dict__.setdefault("_dev", {})
        if key not in cache:
            tens = [torch.from_numpy(np.array(d).view(np.int64)).to(device) if d is not None else None
                    for d in self.dicts]
            cache[key] = (tens, [t.data_ptr() if t is not None else 0 for t in tens])
        return cache[key][1]

    def block_rows_of(self, b: int) -> int:
        return min(self.block_rows, self.rows - b * self.block_rows)

    def block(self, b: int) -> np.ndarray:
        o0, o1 = int(self.block_off[b]), int(self.block_off[b + 1])
        return self.mm[o0:o1]

    def columns(self, rows_b: int):
        return packed_columns(rows_b, self.widths)[0]


class PackedReader:
    """Blocks of a packed shard: {"packed": block bytes, "rows": rows, "shard": PackedShard}."""

    def __init__(self, path: str):
        self.shard = PackedShard(path)
        self.b = 0

    def next(self) -> Optional[dict]:
        s = self.shard
        if self.b >= s.nblocks:
            return None
        b = self.b
        self.b += 1
        return {"packed": s.block(b), "rows": s.block_rows_of(b), "shard": s}


def version_of(path: str) -> int:
    with open(path, "rb") as f:
        magic, ver = _HDR.unpack(f.read(_HDR.size))[:2]
    return int(ver) if magic == MAGIC else -1


def open_reader(path: str, block_rows: int = 65536):
    """The reader of an .xfb shard of any version (packed shards keep their
    own block size)."""
    return PackedReader(path) if version_of(path) == VERSION_PACKED else ShardReader(path, block_rows)


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
    if version_of(path) == VERSION_PACKED:
        p = PackedShard(path)
        return p.block_rows, p.block_rows * p.F
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
    c.add_argument("--packed", action="store_true",
                   help="version 3: packed field-major blocks (fixed-width rows; per-field "
                        "dictionaries of <= 65536 keys as u8 / u16 codes)")
    c.add_argument("--block-rows", type=int, default=262144, help="--packed: rows per block")
    a = ap.parse_args(argv)
    if a.packed:
        info = convert_packed(a.src, a.dst, a.block_bytes, a.threads, a.block_rows)
        print(f"{a.dst}: {info['rows']} rows x {info['F']} fields, {info['bytes_per_row']:.1f} "
              f"bytes per row, code widths {info['widths']}")
        return 0
    info = convert(a.src, a.dst, a.block_bytes, a.threads,
                   {"auto": "auto", "on": True, "off": False}[a.compact])
    print(f"{a.dst}: {info['rows']} rows, {info['nnz']} features")
    return 0


if __name__ == "__main__":
    sys.exit(main())
