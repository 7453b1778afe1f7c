"""Probe: how long P2PComm's IPC handle exchange and import take with N ranks, per arena size, and whether a
small all-to-all then moves the right bytes. Run under torch.distributed.run (any backend for the control plane):

    FAN_P2P_DEBUG=1 python -m torch.distributed.run --nproc-per-node 4 --master-addr 127.0.0.1 \\
        tools/probes/p2p_connect_probe.py 16:2 128:2 128:4

Each argument is slot_MB:depth (arena = slot x world x depth). One JSON line per rank and config on stdout."""
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from fpga_ai_nic_amd import _ext  # noqa: E402


def main():
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    C = _ext.require()
    keep = []
    for spec in sys.argv[1:] or ["16:2"]:
        mb, depth = (int(v) for v in spec.split(":"))
        t0 = time.perf_counter()
        comm = C.P2PComm(rank, world, torch.cuda.current_device(), mb << 20, depth)
        t1 = time.perf_counter()
        blobs = [None] * world
        dist.all_gather_object(blobs, comm.handles())
        t2 = time.perf_counter()
        comm.connect(blobs)
        t3 = time.perf_counter()
        dist.barrier()
        n = 4096 * world
        send = torch.arange(n, dtype=torch.int32, device="cuda") + rank * n
        recv = torch.empty_like(send)
        comm.all_to_all(send, recv)
        torch.cuda.synchronize()
        blk = n // world
        ok = all(torch.equal(recv[s * blk:(s + 1) * blk].cpu(),
                             torch.arange(rank * blk, (rank + 1) * blk, dtype=torch.int32) + s * n)
                 for s in range(world))
        t4 = time.perf_counter()
        print(json.dumps({"rank": rank, "world": world, "slot_mb": mb, "depth": depth,
                          "arena_mb": mb * world * depth, "create_s": round(t1 - t0, 3),
                          "exchange_s": round(t2 - t1, 3), "connect_s": round(t3 - t2, 3),
                          "all_to_all_ok": ok, "all_to_all_s": round(t4 - t3, 3)}), flush=True)
        keep.append(comm)  # imports stay open until exit, as in a run that builds several arms
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
