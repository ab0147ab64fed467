"""Failure detection and recovery: a dead, hung or
misbehaving rank makes the job fail fast (no silent hang), and training
resumes from a checkpoint with the same result as an uninterrupted run."""
import os
import subprocess
import sys
import time

import numpy as np
import pytest

from conftest import DATA, ROOT

TRAIN = os.path.join(DATA, "small_train")
TEST = os.path.join(DATA, "small_test")


def _launch(tmp_path, extra_env, epochs=4, workers=2, timeout=180):
    env = dict(os.environ, PYTHONPATH=ROOT, HIP_VISIBLE_DEVICES="", XFLOW_DIST_TIMEOUT="30",
               XFLOW_FLAGS="--threads 8 --cpu", **extra_env)
    t = time.time()
    r = subprocess.run(["bash", os.path.join(ROOT, "run_ps_local.sh"), "0", str(epochs),
                        str(workers)], cwd=tmp_path, env=env, capture_output=True, text=True,
                       timeout=timeout)
    return r, time.time() - t


@pytest.mark.parametrize("fault", ["kill:1:3", "drop_a2a:1:2"])
def test_faulty_rank_fails_the_job_fast(tmp_path, fault):
    r, dt = _launch(tmp_path, {"XFLOW_FAULT": fault})
    assert r.returncode != 0, r.stdout[-2000:]
    assert dt < 150


def test_hung_rank_is_killed_by_watchdog(tmp_path):
    r, dt = _launch(tmp_path, {"XFLOW_FAULT": "hang:1:2", "XFLOW_WATCHDOG_SECS": "8"})
    assert r.returncode != 0
    assert "watchdog: no progress" in r.stderr
    assert dt < 150


def test_healthy_run_with_watchdog_succeeds(tmp_path):
    r, _ = _launch(tmp_path, {"XFLOW_WATCHDOG_SECS": "60"}, epochs=2)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.count("train end......") == 2


def test_checkpoint_resume_equals_uninterrupted(tmp_path):
    env = dict(os.environ, PYTHONPATH=ROOT, HIP_VISIBLE_DEVICES="")
    base = [sys.executable, "-m", "xflow_amd.cli", TRAIN, TEST, "0"]
    flags = ["--threads", "8", "--cpu"]
    a = tmp_path / "straight"
    b = tmp_path / "resumed"
    a.mkdir()
    b.mkdir()
    subprocess.run(base + ["6"] + flags, cwd=a, env=env, check=True, capture_output=True)
    subprocess.run(base + ["4"] + flags + ["--save", str(b / "ck")], cwd=b, env=env, check=True,
                   capture_output=True)
    subprocess.run(base + ["2"] + flags + ["--load", str(b / "ck")], cwd=b, env=env, check=True,
                   capture_output=True)
    pa = np.loadtxt(a / "pred_0_0.txt")
    pb = np.loadtxt(b / "pred_0_0.txt")
    np.testing.assert_array_equal(pa, pb)


def _tracker(cwd, args, extra_env=None, timeout=300):
    env = dict(os.environ, PYTHONPATH=ROOT, HIP_VISIBLE_DEVICES="", XFLOW_DIST_TIMEOUT="30")
    env.update(extra_env or {})
    return subprocess.run([sys.executable, "-m", "xflow_amd.tracker", *args], cwd=cwd, env=env,
                          capture_output=True, text=True, timeout=timeout)


CLI_ARGS = [TRAIN, TEST, "0", "4", "--threads", "8", "--cpu"]


def test_tracker_recovers_killed_rank_from_checkpoint(tmp_path):
    """The tracker stops the job when a rank dies, relaunches it from the last
    per-epoch checkpoint, and the recovered run predicts exactly like an
    uninterrupted one (scripts/tracker.py 'recover' analogue)."""
    a, b = tmp_path / "straight", tmp_path / "recovered"
    a.mkdir()
    b.mkdir()
    r = _tracker(a, ["-n", "2", "--"] + CLI_ARGS)
    assert r.returncode == 0, r.stderr[-3000:]
    # one step per epoch on the bundled shards: rank 1 dies in the third epoch
    r = _tracker(b, ["-n", "2", "--max-restarts", "2", "--ckpt", str(b / "ck"), "--"] + CLI_ARGS,
                 {"XFLOW_FAULT": "kill:1:2"})
    assert r.returncode == 0, r.stderr[-3000:]
    assert "attempt 0: exit 17" in r.stderr and "attempt 1: exit 0" in r.stderr
    assert "resumed from" in r.stdout and "epoch-000002" in r.stdout
    np.testing.assert_array_equal(np.loadtxt(a / "pred_0_0.txt"), np.loadtxt(b / "pred_0_0.txt"))
    assert open(b / "ck" / "LATEST").read().strip() == "epoch-000004"


def test_tracker_gives_up_after_max_restarts(tmp_path):
    r = _tracker(tmp_path, ["-n", "2", "--max-restarts", "1", "--keep-faults",
                            "--ckpt", str(tmp_path / "ck"), "--"] + CLI_ARGS,
                 {"XFLOW_FAULT": "kill:1:0"})
    assert r.returncode == 17
    assert r.stderr.count("exit 17,") == 2


@pytest.mark.gpu
def test_tracker_recovery_equals_uninterrupted_on_gpu(tmp_path, gpu_device):
    """The same recovery on the HIP backend: the GPU gradient sums are
    fixed-point (order-independent), so a run restarted from its epoch-2
    checkpoint predicts bit-for-bit like the uninterrupted one."""
    args = [TRAIN, TEST, "0", "4", "--threads", "8"]
    env = {"HIP_VISIBLE_DEVICES": os.environ.get("HIP_VISIBLE_DEVICES", "0")}
    a, b = tmp_path / "straight", tmp_path / "recovered"
    a.mkdir()
    b.mkdir()
    r = _tracker(a, ["-n", "1", "--"] + args, env)
    assert r.returncode == 0, r.stderr[-3000:]
    r = _tracker(b, ["-n", "1", "--max-restarts", "2", "--ckpt", str(b / "ck"), "--"] + args,
                 dict(env, XFLOW_FAULT="kill:0:2"))
    assert r.returncode == 0, r.stderr[-3000:]
    assert "attempt 0: exit 17" in r.stderr and "attempt 1: exit 0" in r.stderr
    assert "resumed from" in r.stdout
    np.testing.assert_array_equal(np.loadtxt(a / "pred_0_0.txt"), np.loadtxt(b / "pred_0_0.txt"))
