"""Loader of the in-tree native extension (``_xflow_native``).

torch is imported first so that the HIP runtime torch ships with is the one
the extension binds to (both resolve ``libamdhip64.so.7`` by SONAME).  There
is no Python fallback for the compute path: if the extension is missing the
import fails loudly, and GPU engines additionally require the HIP backend.
"""
from __future__ import annotations

import importlib
import os

import torch  # noqa: F401  (must precede the extension: shared HIP runtime)

_mod = None


def load(build_if_missing: bool = True):
    global _mod
    if _mod is not None:
        return _mod
    try:
        _mod = importlib.import_module("xflow_amd._xflow_native")
    except ImportError:
        if not build_if_missing or os.environ.get("XFLOW_NO_AUTOBUILD"):
            raise
        from xflow_amd import _build

        _build.build()
        _mod = importlib.import_module("xflow_amd._xflow_native")
    return _mod


def hip_available() -> bool:
    return bool(load().hip_available())


def require_hip() -> None:
    """Raise unless the gfx950 HIP backend of the native core can run here."""
    if not torch.cuda.is_available():
        raise RuntimeError("xflow_amd: no ROCm GPU visible to torch")
    if not hip_available():
        raise RuntimeError("xflow_amd: native HIP backend found no device")


def module_path() -> str:
    return load().__file__
