"""Process/rank runtime: the ps-lite lifecycle API on torch.distributed.

Reference API (ps-lite, used at src/model/main.cc:22-47, lr_worker.cc:208):
``ps::Start() / ps::Finalize() / ps::IsServer() / ps::IsWorker() /
ps::MyRank()``.  Here every process is a worker that also serves one shard of
the table, so:

* ``start()``   = init the process group (RCCL over xGMI on GPUs, gloo on CPU)
                  from torchrun env (RANK, WORLD_SIZE, MASTER_ADDR/PORT) or the
                  reference's DMLC_* env (DMLC_NUM_WORKER -> world size,
                  DMLC_PS_ROOT_URI/PORT -> rendezvous, DMLC_WORKER_ID -> rank),
                  plus a global barrier like ps::Start;
* ``finalize()`` = barrier + teardown (ps::Finalize);
* ``is_worker()`` is true for every rank; ``is_server()`` reports whether the
  process was launched in the reference's server role (DMLC_ROLE=server): such
  processes have nothing to do (their job is done by the workers' HBM shards)
  and the CLI exits them immediately, as it does for the scheduler role.

Failure detection: every collective runs under the process-group timeout
(XFLOW_DIST_TIMEOUT seconds, default 600); RCCL async error handling is on,
so a dead peer raises on the survivors instead of hanging.
"""
from __future__ import annotations

import datetime
import os
from typing import Optional

import torch
import torch.distributed as dist

_started_here = False


def role() -> str:
    return os.environ.get("DMLC_ROLE", "worker").lower()


def is_scheduler() -> bool:
    return role() == "scheduler"


def is_server() -> bool:
    return role() == "server"


def is_worker() -> bool:
    return role() == "worker"


def _env_rank_world():
    if "WORLD_SIZE" in os.environ:
        return int(os.environ.get("RANK", "0")), int(os.environ["WORLD_SIZE"])
    if "DMLC_NUM_WORKER" in os.environ:
        return int(os.environ.get("DMLC_WORKER_ID", os.environ.get("RANK", "0"))), \
            int(os.environ["DMLC_NUM_WORKER"])
    return 0, 1


def shared_gpu_setup(rank: int) -> bool:
    """XFLOW_SHARED_GPU=1: several ranks of one job share a GPU (e.g. a 2- or
    4-rank run on a 1-GPU box, to exercise the multi-process RCCL path where
    no multi-GPU node is at hand).  RCCL refuses two ranks on one device of
    one host ("Duplicate GPU detected"), so each rank presents its own host id
    (NCCL_HOSTID) and RCCL connects the ranks through its socket transport on
    the loopback interface.  Correctness only: no xGMI, and the ranks share
    the GPU's CUs.  Must run before the first RCCL communicator is created.
    Returns whether the mode is on."""
    if os.environ.get("XFLOW_SHARED_GPU", "0") in ("", "0"):
        return False
    os.environ["NCCL_HOSTID"] = f"xflow-shared-gpu-rank{rank}"
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    os.environ.setdefault("NCCL_IB_DISABLE", "1")
    return True


def local_rank() -> int:
    return int(os.environ.get("LOCAL_RANK", os.environ.get("DMLC_WORKER_ID", "0")))


def device_for_rank(prefer_gpu: bool = True) -> torch.device:
    if prefer_gpu and torch.cuda.is_available():
        idx = local_rank() % torch.cuda.device_count()
        torch.cuda.set_device(idx)
        return torch.device("cuda", idx)
    return torch.device("cpu")


def start(device: Optional[torch.device] = None, backend: Optional[str] = None) -> int:
    """Initialise the rank runtime; returns the world size (1 => no group)."""
    global _started_here
    rank, world = _env_rank_world()
    if world <= 1 or dist.is_initialized():
        return dist.get_world_size() if dist.is_initialized() else 1
    if "MASTER_ADDR" not in os.environ:
        os.environ["MASTER_ADDR"] = os.environ.get("DMLC_PS_ROOT_URI", "127.0.0.1")
    if "MASTER_PORT" not in os.environ:
        os.environ["MASTER_PORT"] = os.environ.get("DMLC_PS_ROOT_PORT", "29500")
    if device is None:
        device = device_for_rank()
    if backend is None:
        backend = "nccl" if device.type == "cuda" else "gloo"
    timeout = datetime.timedelta(seconds=float(os.environ.get("XFLOW_DIST_TIMEOUT", "600")))
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    kw = dict(backend=backend, rank=rank, world_size=world, timeout=timeout)
    if backend == "nccl":
        shared_gpu_setup(rank)
        kw["device_id"] = device
    dist.init_process_group(**kw)
    _started_here = True
    barrier()
    return world


def finalize() -> None:
    global _started_here
    if dist.is_initialized():
        barrier()
        if _started_here:
            dist.destroy_process_group()
            _started_here = False


def barrier() -> None:
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.barrier()


def my_rank() -> int:
    return dist.get_rank() if dist.is_initialized() else _env_rank_world()[0]


def num_workers() -> int:
    return dist.get_world_size() if dist.is_initialized() else _env_rank_world()[1]


def all_any(flag: bool, device: torch.device) -> bool:
    """True if any rank passed True (lock-step loop control)."""
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return flag
    t = torch.tensor([1 if flag else 0], dtype=torch.int32, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return bool(t.item())


def all_sum(values, device: torch.device):
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return list(values)
    t = torch.tensor(list(values), dtype=torch.float64, device=device)
    dist.all_reduce(t)
    return t.tolist()
