"""Job tracker: start the worker ranks, supervise them, and recover a failed
job from its last checkpoint.

Reference: the dmlc-core tracker vendored at scripts/tracker.py (not invoked
by the reference's own scripts).  RabitTracker hands out ranks over a socket
protocol and re-admits a restarted worker under its old rank (the ``recover``
command, tracker.py:62-67, 276-301); PSTracker starts the ps-lite scheduler
with DMLC_PS_ROOT_URI/PORT (tracker.py:317-359); submit() wires both to a
launcher (tracker.py:361-391) and the job end is logged with its wall time
(tracker.py:302-304).

Here rendezvous belongs to torch.distributed (one process per GPU, RCCL over
xGMI, MASTER_ADDR/PORT), so what is left for the tracker is supervision:

* launch ``-n`` ranks of ``python -m xflow_amd.cli <args>`` with torchrun-style
  env (RANK, LOCAL_RANK, WORLD_SIZE, MASTER_ADDR/PORT) and the reference's
  DMLC_* names, each rank in its own process group;
* fail fast: the first rank that exits non-zero (a crash, the per-rank
  watchdog's exit 75, a collective timeout) or an attempt that outlives
  ``--timeout`` stops every other rank -- survivors blocked in a collective
  would never finish alone;
* recover: a collective job cannot re-admit one rank into a live RCCL
  communicator, so the whole job is relaunched on a fresh rendezvous port with
  ``--resume <ckpt>``: every rank loads the newest complete per-epoch
  checkpoint (checkpoint.publish / latest) and trains the remaining epochs.
  A step is deterministic given the table state, so the recovered run ends
  with the same model as an uninterrupted one.  At most ``--max-restarts``.

    python -m xflow_amd.tracker -n 8 --max-restarts 3 --ckpt ckpt/ -- \\
        train/part test/part 0 20 --log2-cap 28
"""
from __future__ import annotations

import argparse
import os
import signal
import socket
import subprocess
import sys
import time
from typing import List, Optional

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def log(msg: str) -> None:
    sys.stderr.write(f"[tracker] {msg}\n")
    sys.stderr.flush()


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def rank_env(rank: int, world: int, port: int, attempt: int, keep_faults: bool) -> dict:
    env = dict(os.environ)
    env.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), DMLC_ROLE="worker",
               DMLC_NUM_WORKER=str(world), DMLC_NUM_SERVER="0", DMLC_WORKER_ID=str(rank),
               DMLC_PS_ROOT_URI="127.0.0.1", DMLC_PS_ROOT_PORT=str(port),
               XFLOW_RESTART_ATTEMPT=str(attempt),
               PYTHONPATH=ROOT + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else ""))
    if attempt > 0 and not keep_faults:
        env.pop("XFLOW_FAULT", None)  # injected faults fire in the first attempt only
    return env


class Job:
    """One attempt: ``world`` rank processes of the same command."""

    def __init__(self, cmd: List[str], world: int, attempt: int, keep_faults: bool = False):
        port = free_port()
        self.procs = [subprocess.Popen(cmd, env=rank_env(r, world, port, attempt, keep_faults),
                                       start_new_session=True) for r in range(world)]

    def stop(self, grace: float) -> None:
        """SIGTERM every live rank's process group, SIGKILL after ``grace``."""
        for sig in (signal.SIGTERM, signal.SIGKILL):
            for p in self.procs:
                if p.poll() is None:
                    try:
                        os.killpg(p.pid, sig)
                    except ProcessLookupError:
                        pass
            deadline = time.monotonic() + grace
            while time.monotonic() < deadline and any(p.poll() is None for p in self.procs):
                time.sleep(0.05)
        for p in self.procs:
            p.wait()

    def wait(self, timeout: Optional[float], grace: float, poll: float = 0.1) -> int:
        """0 when every rank exits 0; otherwise the first failing rank's exit
        code (128+signal for a signal, 124 for a timeout), after stopping the
        other ranks."""
        t0 = time.monotonic()
        while True:
            codes = [p.poll() for p in self.procs]
            bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
            if bad:
                r, c = bad[0]
                log(f"rank {r} exited with {c}; stopping the job")
                self.stop(grace)
                return c if c > 0 else 128 - c
            if all(c == 0 for c in codes):
                return 0
            if timeout and time.monotonic() - t0 > timeout:
                log(f"attempt exceeded {timeout:.0f}s; stopping the job")
                self.stop(grace)
                return 124
            time.sleep(poll)


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog="python -m xflow_amd.tracker", description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("-n", "--num-workers", type=int, required=True, help="ranks (one per GPU)")
    ap.add_argument("--max-restarts", type=int, default=0)
    ap.add_argument("--ckpt", default="",
                    help="versioned checkpoint root for per-epoch saves and recovery "
                         "(required with --max-restarts > 0)")
    ap.add_argument("--save-every", type=int, default=1, help="epochs between checkpoints")
    ap.add_argument("--timeout", type=float, default=0.0, help="seconds per attempt (0: none)")
    ap.add_argument("--grace", type=float, default=5.0,
                    help="seconds between SIGTERM and SIGKILL when stopping ranks")
    ap.add_argument("--keep-faults", action="store_true",
                    help="keep XFLOW_FAULT in restarted attempts (tests)")
    ap.add_argument("cli_args", nargs=argparse.REMAINDER,
                    help="-- then the xflow_lr arguments: train test model epochs [flags]")
    return ap


def main(argv=None) -> int:
    a = build_parser().parse_args(argv)
    args = a.cli_args[1:] if a.cli_args[:1] == ["--"] else a.cli_args
    if not args:
        build_parser().error("missing the xflow_lr arguments after --")
    if a.max_restarts > 0 and not a.ckpt:
        build_parser().error("--max-restarts needs --ckpt (recovery resumes from it)")
    cmd = [sys.executable, "-m", "xflow_amd.cli", *args]
    if a.ckpt:
        cmd += ["--resume", a.ckpt, "--save-every", str(a.save_every)]
    rc = 1
    for attempt in range(a.max_restarts + 1):
        t0 = time.monotonic()
        rc = Job(cmd, a.num_workers, attempt, a.keep_faults).wait(a.timeout or None, a.grace)
        log(f"attempt {attempt}: exit {rc}, {time.monotonic() - t0:.2f} secs between node start "
            f"and job finish")
        if rc == 0:
            return 0
        if attempt < a.max_restarts:
            log(f"recovering from {a.ckpt} (restart {attempt + 1} of {a.max_restarts})")
    return rc


if __name__ == "__main__":
    sys.exit(main())
