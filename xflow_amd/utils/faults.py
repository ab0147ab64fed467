"""Failure detection and fault injection.

* ``Watchdog``: a daemon thread per rank.  The trainer calls ``beat()`` every
  step; if no beat arrives for ``timeout`` seconds the watchdog logs the stall
  with every thread's stack and (policy "abort") terminates the process with
  exit code 75, so a launcher sees a dead rank instead of a silent hang.  RCCL
  / gloo collectives additionally carry the process-group timeout
  (XFLOW_DIST_TIMEOUT) and async error handling (parallel/dist.py).
* Fault injection for tests, from the environment (never set in production):
    XFLOW_FAULT=kill:<rank>:<step>      rank exits abruptly before that step
    XFLOW_FAULT=hang:<rank>:<step>      rank stops making progress (sleeps)
    XFLOW_FAULT=slow_rank:<rank>:<ms>   rank sleeps <ms> before EVERY training step (a
                                        straggler: the asynchronous parameter server's
                                        other workers must keep their pace,
                                        parallel/async_ps.py; the lock-step step
                                        slows every rank to it)
    XFLOW_FAULT=drop_a2a:<rank>:<step>  rank skips one exchange of that step.  On
                                        the gloo / loopback transports its peers
                                        detect the out-of-step counts at the next
                                        exchange; on the native RCCL transport the
                                        skipped exchange is one send/recv inside a
                                        group call, so the peers block in that call
                                        and the fault surfaces only through the
                                        collective timeout / the watchdog
"""
from __future__ import annotations

import faulthandler
import os
import sys
import threading
import time
from typing import Optional


class Watchdog:
    def __init__(self, timeout: float, policy: str = "abort", name: str = "xflow"):
        self.timeout = float(timeout)
        self.policy = policy
        self.name = name
        self._last = time.monotonic()
        self._stop = threading.Event()
        self.fired = False
        self._th = threading.Thread(target=self._run, name=f"{name}-watchdog", daemon=True)

    def start(self) -> "Watchdog":
        self._th.start()
        return self

    def beat(self) -> None:
        self._last = time.monotonic()

    def stop(self) -> None:
        self._stop.set()

    def _run(self) -> None:
        while not self._stop.wait(min(1.0, self.timeout / 4)):
            if time.monotonic() - self._last > self.timeout:
                self.fired = True
                sys.stderr.write(f"[{self.name}] watchdog: no progress for {self.timeout:.0f}s\n")
                faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
                sys.stderr.flush()
                if self.policy == "abort":
                    os._exit(75)
                return


def watchdog_from_env(name: str = "xflow") -> Optional[Watchdog]:
    t = os.environ.get("XFLOW_WATCHDOG_SECS")
    return Watchdog(float(t), os.environ.get("XFLOW_WATCHDOG_POLICY", "abort"), name).start() \
        if t else None


class FaultInjector:
    def __init__(self, spec: Optional[str], rank: int):
        self.kind = None
        self.slow_ms = 0
        if spec:
            kind, r, step = spec.split(":")
            if int(r) == rank:
                self.kind, self.step = kind, int(step)
                if kind == "slow_rank":
                    self.slow_ms = int(step)

    def before_step(self, step: int) -> bool:
        """Returns False when this rank must skip an exchange of the step."""
        if self.kind == "slow_rank":
            time.sleep(self.slow_ms / 1000.0)
            return True
        if self.kind is None or step != self.step:
            return True
        if self.kind == "kill":
            sys.stderr.write(f"[fault] rank exits at step {step}\n")
            sys.stderr.flush()
            os._exit(17)
        if self.kind == "hang":
            time.sleep(3600)
        return self.kind != "drop_a2a"


def injector_from_env(rank: int) -> FaultInjector:
    return FaultInjector(os.environ.get("XFLOW_FAULT"), rank)


def slow_ms_from_env(rank: int) -> int:
    """XFLOW_FAULT=slow_rank:<rank>:<ms>: this rank's per-step sleep (0: none)."""
    return FaultInjector(os.environ.get("XFLOW_FAULT"), rank).slow_ms
