"""Process-group bootstrap: one process per GPU, torch.distributed over RCCL (xGMI) or gloo.

Reference: train.py:24-35 (``init_process_group("nccl")`` unconditional, needs torchrun).
Here:
  * torchrun / torch.distributed.run env (RANK, LOCAL_RANK, WORLD_SIZE, MASTER_*) -> DDP run,
  * no env -> single process, no process group (plain ``python train.py`` works),
  * backend "nccl" is RCCL on ROCm; "gloo" for CPU runs and tests; "auto" picks by device.
RCCL-on-MI355X defaults are applied only when the user has not set them.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class DistInfo:
    ddp: bool
    rank: int
    local_rank: int
    world_size: int
    device: str
    backend: str

    @property
    def master(self) -> bool:
        return self.rank == 0


def rccl_env_defaults():
    """Set conservative RCCL knobs for a single 8x MI355X xGMI node (only if unset)."""
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # dmabuf IPC only on these hosts
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    os.environ.setdefault("NCCL_IB_DISABLE", "1")              # single node: xGMI only


def init_distributed(backend: str = "auto", device_type: str = "auto", timeout_s: int = 1800) -> DistInfo:
    ddp = int(os.environ.get("RANK", -1)) != -1
    want_cuda = torch.cuda.is_available() if device_type == "auto" else device_type == "cuda"
    if not ddp:
        dev = "cuda:0" if want_cuda else "cpu"
        if want_cuda:
            torch.cuda.set_device(0)
        return DistInfo(False, 0, 0, 1, dev, "none")
    rank = int(os.environ["RANK"])
    local_rank = int(os.environ.get("LOCAL_RANK", rank))
    world = int(os.environ["WORLD_SIZE"])
    if backend == "auto":
        backend = "nccl" if want_cuda else "gloo"
    if want_cuda:
        rccl_env_defaults()
        dev = f"cuda:{local_rank}"
        torch.cuda.set_device(dev)
    else:
        dev = "cpu"
    import datetime
    kw = {}
    if backend == "nccl" and want_cuda:
        kw["device_id"] = torch.device(dev)
    timeout = datetime.timedelta(seconds=timeout_s)
    if os.environ.get("TORCHELASTIC_USE_AGENT_STORE", "").lower() == "true":
        # under torchrun the agent hosts the rendezvous store and keeps it across worker restarts;
        # scope this attempt's keys so restarted workers never read the dead attempt's addresses
        attempt = os.environ.get("TORCHELASTIC_RESTART_COUNT", "0")
        base = dist.TCPStore(os.environ["MASTER_ADDR"], int(os.environ["MASTER_PORT"]), world, is_master=False,
                             timeout=timeout)
        store = dist.PrefixStore(f"mamba_amd/attempt{attempt}", base)
        dist.init_process_group(backend=backend, store=store, rank=rank, world_size=world, timeout=timeout, **kw)
    else:
        dist.init_process_group(backend=backend, timeout=timeout, **kw)
    return DistInfo(True, rank, local_rank, world, dev, backend)


def destroy():
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()


def all_reduce_avg(t: torch.Tensor) -> torch.Tensor:
    """AVG all-reduce (gloo has no native AVG on every version: SUM then divide)."""
    if not (dist.is_available() and dist.is_initialized()):
        return t
    if dist.get_backend() == "nccl":
        dist.all_reduce(t, op=dist.ReduceOp.AVG)
    else:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        t /= dist.get_world_size()
    return t


def all_reduce_max(t: torch.Tensor) -> torch.Tensor:
    if dist.is_available() and dist.is_initialized():
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t


def all_gather_object(obj):
    """List of every rank's ``obj`` (just ``[obj]`` without a process group)."""
    if not (dist.is_available() and dist.is_initialized()):
        return [obj]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, obj)
    return out


def barrier():
    if dist.is_available() and dist.is_initialized():
        if dist.get_backend() == "nccl" and torch.cuda.is_available():
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()
