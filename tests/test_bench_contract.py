"""bench.py driver contract, exercised on the CPU backend: one JSON line from
rank 0 with the whole-job aggregate, launched plain (N=1) and under
torch.distributed.run (N=2, gloo) exactly as the round driver launches the
multi-GPU scaling run (the N>1 path is the sharded table + sparse all-to-all
step of xflow_amd/parallel/sparse_a2a.py)."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
        "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"}


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(n, extra, cpu=True, env_extra=None):
    args = ["--gpus", str(n), "--steps", "2", "--warmup", "1"] + (["--cpu"] if cpu else []) + extra
    if n == 1:
        cmd = [sys.executable, os.path.join(ROOT, "bench.py")] + args
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
               f"--nproc-per-node={n}", "--master-addr", "127.0.0.1",
               "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py")] + args
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="2", **(env_extra or {}))
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT, env=env)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0 only
    return json.loads(lines[0])


@pytest.mark.parametrize("n,extra", [(1, []), (2, []), (2, ["--model", "fm", "--v-dim", "8"]),
                                     (2, ["--async"]), (2, ["--async-lockstep"]),
                                     (2, ["--slices", "4"])])
def test_bench_json_line(n, extra):
    d = _run(n, extra)
    assert KEYS <= set(d)
    assert d["n_gpus"] == n and d["steps"] == 2 and d["warmup"] == 1
    assert d["higher_is_better"] is True and d["scaling"] == "weak"
    cfg = d["config"]
    assert cfg["global_batch"] == cfg["rows_per_gpu"] * n
    assert cfg["parallelism"].startswith(f"dp{n}")
    # whole-job aggregate: samples over the slowest rank's time
    assert d["value"] == pytest.approx(cfg["global_batch"] * d["steps"] / (d["ms_per_step"] * d["steps"] / 1e3),
                                       rel=1e-6)
    assert 0.0 < d["logloss"] < 1.0 and d["table_keys"] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("extra", [[], ["--sharded"], ["--async"], ["--async-lockstep"], ["--slices", "8"],
                                   ["--model", "fm", "--v-dim", "8"], ["--model", "mvm", "--v-dim", "10"]])
def test_bench_json_line_on_gpu(gpu_device, extra):
    """The benchmark variants on the HIP backend (1 GPU, prefilled table):
    the contract line, no overflow (bench.py exits non-zero on one), and a
    table at the prefilled occupancy."""
    d = _run(1, extra + ["--clock-warmup-s", "0"], cpu=False)
    assert KEYS <= set(d)
    assert d["config"]["backend"].startswith("hip:gfx950")
    assert d["table_load"] > 0.4 and d["prefilled_keys"] > 0
    assert 0.0 < d["logloss"] < 1.0


@pytest.mark.gpu
@pytest.mark.parametrize("n,extra", [(2, []), (2, ["--async"]), (2, ["--async", "--slices", "64"]),
                                     (3, ["--model", "fm", "--v-dim", "8"])])
def test_bench_multirank_rccl_on_one_gpu(gpu_device, n, extra):
    """The driver's multi-GPU launch (torch.distributed.run, one process per
    rank, RCCL) with every rank on this box's GPU 0 (XFLOW_SHARED_GPU=1:
    RCCL's socket transport between the processes, parallel/dist.py): the
    contract line of the N-rank bench, the native RCCL transport, the
    steady-state two-exchange step (keys exchanged ahead), no overflow."""
    d = _run(n, extra + ["--batch", "16384", "--log2-cap", "24", "--clock-warmup-s", "0"],
             cpu=False, env_extra={"XFLOW_SHARED_GPU": "1"})
    assert KEYS <= set(d)
    assert d["n_gpus"] == n and d["shared_gpu_rehearsal"] is True
    assert d["config"]["a2a_transport"] == ("ipc" if "--async" in extra else "rccl")
    assert d["config"]["global_batch"] == 16384 * n
    if "--async" not in extra:
        assert d["early_key_exchanges"] >= d["steps"]
    else:  # one rate per rank, each its own
        assert len(d["per_rank"]) == n and d["max_staleness"] <= d["staleness_bound"]
    assert 0.0 < d["logloss"] < 1.0 and d["table_keys"] > 0
