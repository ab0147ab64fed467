"""Pure-Python/NumPy re-implementations of the native hashing recipes, used by
the test oracles so they do not depend on the code under test.

* ``std_hash``: libstdc++ ``std::hash<std::string>`` on 64-bit Linux =
  ``_Hash_bytes(ptr, len, seed=0xc70f6907)``, MurmurHash64A-style.  The
  reference keys every feature with it (src/io/io.h:53,
  load_data_from_disk.cc:154).
* ``fmix64`` / ``normal_init``: csrc/include/xflow/common.h.
"""
from __future__ import annotations

import numpy as np

M64 = (1 << 64) - 1


def _load_bytes(b: bytes, n: int) -> int:
    r = 0
    for i in range(n - 1, -1, -1):
        r = (r << 8) + b[i]
    return r


def std_hash(s: str | bytes, seed: int = 0xC70F6907) -> int:
    data = s.encode() if isinstance(s, str) else s
    mul = (0xC6A4A793 << 32) + 0x5BD1E995
    ln = len(data)
    h = (seed ^ (ln * mul)) & M64

    def shift_mix(v):
        return v ^ (v >> 47)

    nblk = ln & ~7
    for i in range(0, nblk, 8):
        d = int.from_bytes(data[i:i + 8], "little")
        d = (shift_mix((d * mul) & M64) * mul) & M64
        h ^= d
        h = (h * mul) & M64
    if ln & 7:
        d = _load_bytes(data[nblk:], ln & 7)
        h ^= d
        h = (h * mul) & M64
    h = (shift_mix(h) * mul) & M64
    h = shift_mix(h)
    return h


def fmix64_int(h: int) -> int:
    h &= M64
    h ^= h >> 33
    h = (h * 0xFF51AFD7ED558CCD) & M64
    h ^= h >> 33
    h = (h * 0xC4CEB9FE1A85EC53) & M64
    h ^= h >> 33
    return h


def fmix64(h: np.ndarray) -> np.ndarray:
    h = np.asarray(h, dtype=np.uint64).copy()
    with np.errstate(over="ignore"):
        h ^= h >> np.uint64(33)
        h *= np.uint64(0xFF51AFD7ED558CCD)
        h ^= h >> np.uint64(33)
        h *= np.uint64(0xC4CEB9FE1A85EC53)
        h ^= h >> np.uint64(33)
    return h


def owner_of(keys: np.ndarray, world: int) -> np.ndarray:
    if world <= 1:
        return np.zeros(len(keys), dtype=np.int64)
    return ((fmix64(keys) >> np.uint64(32)) % np.uint64(world)).astype(np.int64)


def normal_init(keys: np.ndarray, dim: int, seed: int = 0x5EED) -> np.ndarray:
    k = np.asarray(keys, dtype=np.uint64)
    with np.errstate(over="ignore"):
        s = np.uint64((seed * 0x9E3779B97F4A7C15) & M64)
        x = k ^ s ^ np.uint64((dim << 48) & M64) ^ np.uint64(0x243F6A8885A308D3)
        a = fmix64(x)
        b = fmix64(a ^ np.uint64(0x13198A2E03707344))
    u1 = ((a >> np.uint64(40)).astype(np.float32) + np.float32(1.0)) * np.float32(1.0 / 16777216.0)
    u2 = (b >> np.uint64(40)).astype(np.float32) * np.float32(1.0 / 16777216.0)
    r = np.sqrt(np.float32(-2.0) * np.log(u1))
    return (r * np.cos(np.float32(6.283185307179586) * u2)).astype(np.float32)
