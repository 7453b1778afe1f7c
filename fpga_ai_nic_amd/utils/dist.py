"""Process-group bootstrap: one process per GPU (torchrun env), RCCL on GPU, gloo on CPU.

Replaces the reference's MPI bootstrap (MPI_Init_thread / Comm_rank / Comm_size, sw/mlp_mpi_example_f32.cpp:195-300)
and the IKL ring wiring (sw/setup_route.sh): on a fully connected xGMI node no route setup is needed; ring
orders are computed by the planner.
"""
from __future__ import annotations

import contextlib
import datetime
import os
import sys

import torch
import torch.distributed as dist


def env_rank_world():
    return int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")), int(
        os.environ.get("LOCAL_RANK", "0"))


def init_distributed(backend: str | None = None, timeout_s: float = 600.0, force: bool = False):
    """Initialise torch.distributed from the torchrun environment (no-op for world 1 without env, unless
    ``force``: a 1-rank process group, used to exercise the multi-rank code path on one GPU).

    Returns (rank, world, local_rank, device)."""
    rank, world, local = env_rank_world()
    use_cuda = torch.cuda.is_available() and backend != "gloo"
    if use_cuda:
        torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
        device = torch.device("cuda", torch.cuda.current_device())
    else:
        device = torch.device("cpu")
    if (world > 1 or force) and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        # FAN_CTRL_BACKEND=gloo: control plane (bootstrap, broadcast, barrier) over gloo even on GPU — for
        # several ranks sharing one GPU with the P2P transport, where RCCL refuses duplicate devices
        be = backend or os.environ.get("FAN_CTRL_BACKEND") or ("nccl" if use_cuda else "gloo")
        local_world = int(os.environ.get("LOCAL_WORLD_SIZE", world))
        if be == "nccl" and local_world > max(1, torch.cuda.device_count()):
            # more ranks than GPUs on this node: ranks share a device, which RCCL refuses ("invalid usage");
            # the control plane goes over gloo (the P2P transport still moves the gradients between the ranks)
            print(f"[dist] {local_world} local ranks on {torch.cuda.device_count()} GPU(s): control plane over gloo",
                  file=sys.stderr, flush=True)
            be = "gloo"
        kw = dict(backend=be, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=timeout_s))
        if be == "nccl":
            kw["device_id"] = device
        with stdout_to_stderr():  # RCCL prints its version banner on stdout: keep stdout for the results
            dist.init_process_group(**kw)
    return rank, world, local, device


@contextlib.contextmanager
def stdout_to_stderr():
    """Route file descriptor 1 to 2 for the duration (native libraries that print banners on stdout, e.g. RCCL at
    communicator init), so a benchmark's stdout carries only its result lines."""
    sys.stdout.flush()
    saved = os.dup(1)
    try:
        os.dup2(2, 1)
        yield
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)


def barrier():
    if dist.is_initialized() and dist.get_world_size() > 1:
        if dist.get_backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def max_over_ranks(x: float) -> float:
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return x
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def backend() -> str | None:
    return dist.get_backend() if dist.is_initialized() else None


def all_gather_object(obj) -> list:
    """Every rank's ``obj`` in rank order (``[obj]`` without a multi-rank process group)."""
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return [obj]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, obj)
    return out


def cleanup():
    if dist.is_initialized():
        try:
            barrier()
        finally:
            dist.destroy_process_group()
