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
from typing import Optional

import numpy as np

from xflow_amd.testing.hashing import owner_of

MAGIC = b"XFLOWTB1"


def shard_name(rank: int, world: int) -> str:
    return f"shard-{rank:05d}-of-{world:05d}.xftb"


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


def save(engine, ckpt_dir: str, rank: int, world: int, meta: Optional[dict] = None) -> str:
    os.makedirs(ckpt_dir, exist_ok=True)
    path = os.path.join(ckpt_dir, shard_name(rank, world))
    tmp = path + ".tmp"
    engine.save(tmp)
    os.replace(tmp, path)
    if rank == 0:
        m = dict(meta or {})
        m.update(world=world, model=dataclasses.asdict(engine.model),
                 optim=dataclasses.asdict(engine.optim))
        with open(os.path.join(ckpt_dir, "meta.json.tmp"), "w") as f:
            json.dump(m, f, indent=1)
        os.replace(os.path.join(ckpt_dir, "meta.json.tmp"), os.path.join(ckpt_dir, "meta.json"))
    return path


def load_meta(ckpt_dir: str) -> dict:
    with open(os.path.join(ckpt_dir, "meta.json")) as f:
        return json.load(f)


def load(engine, ckpt_dir: str, rank: int, world: int) -> dict:
    meta = load_meta(ckpt_dir)
    saved_world = int(meta["world"])
    if saved_world == world:
        engine.load(os.path.join(ckpt_dir, shard_name(rank, world)))
        return meta
    shards = sorted(glob.glob(os.path.join(ckpt_dir, "shard-*-of-%05d.xftb" % saved_world)))
    if len(shards) != saved_world:
        raise FileNotFoundError(f"{ckpt_dir}: expected {saved_world} shards, found {len(shards)}")
    for p in shards:
        _, keys, words = read_shard(p)
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
    os.replace(tmp, os.path.join(root, LATEST))
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
