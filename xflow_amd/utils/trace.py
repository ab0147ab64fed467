"""Tracing / profiling hooks.

* ``PhaseTimer``: per-phase wall time with HIP events (device) or perf_counter
  (CPU), enabled by XFLOW_TRACE=1; ``summary()`` gives mean ms per phase.
* ``roctx_range``: roctx push/pop markers (librocprofiler-sdk-roctx /
  libroctx64 via ctypes) so rocprofv3 --marker-trace timelines show the engine
  phases; a no-op when the library is absent.
* ``torch_profile``: context manager around torch.profiler writing a Chrome
  trace into a directory (the ``--trace-dir`` switch of the CLI).

The reference has no tracing at all; rocprofv3 kernel
traces + counters cover the device side (scripts/profile_bench.sh).
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import time
from collections import defaultdict
from typing import Optional

import torch

_roctx = None
_roctx_tried = False


def _load_roctx():
    global _roctx, _roctx_tried
    if _roctx_tried:
        return _roctx
    _roctx_tried = True
    for name in ("librocprofiler-sdk-roctx.so", "libroctx64.so"):
        try:
            lib = ctypes.CDLL(name)
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            _roctx = lib
            break
        except OSError:
            continue
    return _roctx


@contextlib.contextmanager
def roctx_range(name: str):
    lib = _load_roctx() if os.environ.get("XFLOW_ROCTX") else None
    if lib is not None:
        lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        if lib is not None:
            lib.roctxRangePop()


class PhaseTimer:
    def __init__(self, device: torch.device, enabled: bool = False):
        self.device = device
        self.enabled = enabled
        self.events = defaultdict(list)

    @contextlib.contextmanager
    def phase(self, name: str):
        if not self.enabled:
            yield
            return
        with roctx_range(name):
            if self.device.type == "cuda":
                s = torch.cuda.Event(enable_timing=True)
                e = torch.cuda.Event(enable_timing=True)
                s.record()
                yield
                e.record()
                self.events[name].append((s, e))
            else:
                t = time.perf_counter()
                yield
                self.events[name].append(time.perf_counter() - t)

    def summary(self) -> dict:
        out = {}
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        for k, v in self.events.items():
            if not v:
                continue
            if isinstance(v[0], tuple):
                ms = [s.elapsed_time(e) for s, e in v]
            else:
                ms = [x * 1e3 for x in v]
            out[k] = {"count": len(ms), "mean_ms": sum(ms) / len(ms)}
        return out


class StreamTimeline:
    """Device-side intervals of named activities on their own streams (HIP
    timing events), for overlap evidence without a profiler: e.g. the H2D
    copies of the streamed input path (copy stream) against the training
    steps (compute stream).  ``begin(kind, stream)`` / ``end(...)`` bracket
    one interval; ``overlap(a, b)`` = time of kind a that ran while some
    interval of kind b was running (intervals read back after a sync).
    Enabled by XFLOW_STREAM_TIMELINE=1 in the trainer."""

    def __init__(self, device: torch.device):
        self.device = device
        self.base = torch.cuda.Event(enable_timing=True)
        self.base.record(torch.cuda.current_stream(device))
        self.events = defaultdict(list)  # kind -> [(start, end)]
        self._open = {}

    def begin(self, kind: str, stream=None) -> None:
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(stream if stream is not None else torch.cuda.current_stream(self.device))
        self._open[kind] = ev

    def end(self, kind: str, stream=None) -> None:
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(stream if stream is not None else torch.cuda.current_stream(self.device))
        self.events[kind].append((self._open.pop(kind), ev))

    def intervals(self, kind: str):
        torch.cuda.synchronize(self.device)
        return sorted((self.base.elapsed_time(a), self.base.elapsed_time(b))
                      for a, b in self.events.get(kind, []))

    @staticmethod
    def _union(iv):
        out = []
        for a, b in iv:
            if out and a <= out[-1][1]:
                out[-1][1] = max(out[-1][1], b)
            else:
                out.append([a, b])
        return out

    def overlap(self, a: str, b: str) -> dict:
        ia, ub = self.intervals(a), self._union(self.intervals(b))
        tot = sum(y - x for x, y in ia)
        ov = 0.0
        for x, y in ia:
            for u, v in ub:
                ov += max(0.0, min(y, v) - max(x, u))
        return {f"{a}_ms": tot, f"{a}_during_{b}_ms": ov,
                f"{b}_busy_ms": sum(v - u for u, v in ub), f"{a}_n": len(ia)}


@contextlib.contextmanager
def torch_profile(trace_dir: Optional[str]):
    if not trace_dir:
        yield None
        return
    os.makedirs(trace_dir, exist_ok=True)
    acts = [torch.profiler.ProfilerActivity.CPU]
    if torch.cuda.is_available():
        acts.append(torch.profiler.ProfilerActivity.CUDA)
    with torch.profiler.profile(activities=acts) as prof:
        yield prof
    prof.export_chrome_trace(os.path.join(trace_dir, "trace_rank%s.json" %
                                          os.environ.get("RANK", "0")))
