"""Sharded checkpoint / resume of the HBM parameter table (an extension: the
reference keeps weights only in server RAM and loses them at exit,
src/optimizer/ftrl.h:84,151).

Layout of ``<dir>/``:
  meta.json                      model/optimizer config, world size, epoch, step
  shard-<rank>-of-<world>.xftb   native binary shard (csrc/engine/engine.cpp
                                 Engine::save): header + keys + state words

Resume is world-size agnostic: with the same world size each rank loads its
own shard; otherwise every rank scans all shards and imports exactly the keys
it owns under the new hash sharding (owner = fmix64(key) >> 32 mod world).

Periodic checkpoints (``--save-every``, the tracker's recovery) are versioned:
``<root>/epoch-NNNNNN/`` holds one complete checkpoint in the layout above and
``<root>/LATEST`` names the newest complete one.  LATEST is replaced
atomically by rank 0 only after every rank has written its shard, so a job
killed mid-save resumes from the previous version.
"""
from __future__ import annotations

import dataclasses
import glob
import json
import os
import shutil
import struct
import warnings
from typing import Callable, Optional

import numpy as np

from xflow_amd.testing.hashing import owner_of

MAGIC = b"XFLOWTB1"


def shard_name(rank: int, world: int) -> str:
    return f"shard-{rank:05d}-of-{world:05d}.xftb"


def shard_keys(path: str) -> int:
    """Number of keys in a native shard file, from its header only (48 bytes
    read, not the keys and state words)."""
    with open(path, "rb") as f:
        if f.read(8) != MAGIC:
            raise ValueError(f"{path}: not an xflow table shard")
        f.seek(32, os.SEEK_CUR)
        (n,) = struct.unpack("<Q", f.read(8))
    return int(n)


def read_shard(path: str):
    """(header ints, keys u64, words u32 [n, W]) of a native shard file."""
    with open(path, "rb") as f:
        magic = f.read(8)
        if magic != MAGIC:
            raise ValueError(f"{path}: not an xflow table shard")
        hdr = struct.unpack("<8i", f.read(32))
        (n,) = struct.unpack("<Q", f.read(8))
        keys = np.frombuffer(f.read(8 * n), dtype=np.uint64)
        W = hdr[6] - 2
        words = np.frombuffer(f.read(4 * n * W), dtype=np.uint32).reshape(n, W)
    return hdr, keys, words


def _fsync_file(path: str) -> None:
    fd = os.open(path, os.O_RDONLY)
    try:
        os.fsync(fd)
    finally:
        os.close(fd)


def _fsync_dir(path: str) -> None:
    try:
        _fsync_file(path)
    except OSError:  # pragma: no cover - directories cannot be opened on some filesystems
        pass


def _default_barrier() -> None:
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized():
        dist.barrier()


def save(engine, ckpt_dir: str, rank: int, world: int, meta: Optional[dict] = None,
         barrier: Optional[Callable[[], None]] = None) -> str:
    """Write this rank's shard (fsync'd), wait for every rank (``barrier``,
    default: the torch.distributed group when one is initialised), then rank 0
    writes meta.json -- so a valid meta.json only ever sits next to a complete
    set of shards of one save."""
    os.makedirs(ckpt_dir, exist_ok=True)
    path = os.path.join(ckpt_dir, shard_name(rank, world))
    tmp = path + ".tmp"
    engine.save(tmp)
    _fsync_file(tmp)
    os.replace(tmp, path)
    (barrier or _default_barrier)()
    if rank == 0:
        m = dict(meta or {})
        m.update(world=world, model=dataclasses.asdict(engine.model),
                 optim=dataclasses.asdict(engine.optim))
        mtmp = os.path.join(ckpt_dir, "meta.json.tmp")
        with open(mtmp, "w") as f:
            json.dump(m, f, indent=1)
            f.flush()
            os.fsync(f.fileno())
        os.replace(mtmp, os.path.join(ckpt_dir, "meta.json"))
        _fsync_dir(ckpt_dir)
    return path


# Fields that define what the table's state means: a resume must match them.
# Everything else (fm_mfma picks a kernel; lr/alpha/beta/lambda1/lambda2 are
# a schedule the user may change on resume) only warns.
_LAYOUT_FIELDS = {"model": ("kind", "v_dim", "fm_math", "mvm_math"),
                  "optim": ("kind", "v_init_scale", "sgd_v_init", "seed")}


def check_compatible(engine, meta: dict) -> None:
    """The checkpoint's layout-defining model/optimizer fields must equal the
    running ones; other differences (hyperparameters, kernel choices) are
    reported as warnings."""
    want = {"model": dataclasses.asdict(engine.model), "optim": dataclasses.asdict(engine.optim)}
    for k, cur in want.items():
        saved = meta.get(k)
        if saved is None:
            continue
        diff = {f: (saved.get(f), v) for f, v in cur.items() if f in saved and saved[f] != v}
        hard = {f: d for f, d in diff.items() if f in _LAYOUT_FIELDS[k]}
        if hard:
            raise ValueError(f"checkpoint {k} config differs from the running one: {hard}")
        if diff:
            warnings.warn(f"resuming with a changed {k} config (saved, now): {diff}")


def _check_header(engine, path: str, hdr) -> None:
    """Shard header (csrc/engine/engine.cpp Engine::save: version, kind, v_dim,
    P, p_w, opt, stride) against the engine's table layout."""
    if hdr[0] != 1:
        raise ValueError(f"{path}: unsupported shard version {hdr[0]}")
    lay = engine.layout
    got = {"kind": hdr[1], "P": hdr[3], "opt": hdr[5], "stride": hdr[6]}
    exp = {"kind": lay["kind"], "P": lay["P"], "opt": lay["opt"], "stride": lay["stride"]}
    if got != exp:
        raise ValueError(f"{path}: shard layout {got} does not match this engine {exp}")


def load_meta(ckpt_dir: str) -> dict:
    with open(os.path.join(ckpt_dir, "meta.json")) as f:
        return json.load(f)


def load(engine, ckpt_dir: str, rank: int, world: int) -> dict:
    meta = load_meta(ckpt_dir)
    check_compatible(engine, meta)
    saved_world = int(meta["world"])
    if saved_world == world:
        engine.load(os.path.join(ckpt_dir, shard_name(rank, world)))
        return meta
    shards = sorted(glob.glob(os.path.join(ckpt_dir, "shard-*-of-%05d.xftb" % saved_world)))
    if len(shards) != saved_world:
        raise FileNotFoundError(f"{ckpt_dir}: expected {saved_world} shards, found {len(shards)}")
    for p in shards:
        hdr, keys, words = read_shard(p)
        _check_header(engine, p, hdr)
        mine = owner_of(keys, world) == rank
        if mine.any():
            engine.import_table(keys[mine], words[mine].reshape(-1))
    return meta


LATEST = "LATEST"


def version_dir(root: str, epoch: int) -> str:
    return os.path.join(root, "epoch-%06d" % epoch)


def publish(root: str, epoch: int, keep: int = 2) -> None:
    """Rank 0, after every rank saved the epoch's shards: point LATEST at the
    version atomically and drop all but the newest ``keep`` versions."""
    tmp = os.path.join(root, LATEST + ".tmp")
    with open(tmp, "w") as f:
        f.write(os.path.basename(version_dir(root, epoch)) + "\n")
        f.flush()
        os.fsync(f.fileno())
    os.replace(tmp, os.path.join(root, LATEST))
    _fsync_dir(root)
    for d in sorted(glob.glob(os.path.join(root, "epoch-*")))[:-keep]:
        shutil.rmtree(d, ignore_errors=True)


def latest(root: str) -> Optional[str]:
    """Directory of the newest complete versioned checkpoint under root, or None."""
    p = os.path.join(root, LATEST)
    if not os.path.exists(p):
        return None
    with open(p) as f:
        d = os.path.join(root, f.read().strip())
    return d if os.path.exists(os.path.join(d, "meta.json")) else None
