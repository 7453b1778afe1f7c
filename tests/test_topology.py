"""Link-matrix discovery (fpga_ai_nic_amd/utils/topology.py) on the CPU: rocm-smi output parsing, the rank -> GPU
mapping by PCI bus id (rocm-smi numbers the node's GPUs, not the process's visible devices), and the multi-process
agreement — every rank plans its rings from rank 0's matrix even when its own tool calls answer differently (the
round-2 advice: a rank with a timed-out rocm-smi would otherwise plan different rings and post mismatched peers)."""
import os
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from fpga_ai_nic_amd.utils import topology as T

SHOWBUS = """
============================ ROCm System Management Interface ============================
=================================== PCI Bus ID ===================================
GPU[0]		: PCI Bus: 0000:05:00.0
GPU[1]		: PCI Bus: 0000:15:00.0
GPU[2]		: PCI Bus: 0000:65:00.0
GPU[3]		: PCI Bus: 0000:75:00.0
==================================================================================
"""


def test_parse_showbus_and_normalize():
    assert T.parse_showbus(SHOWBUS) == {0: "05:00", 1: "15:00", 2: "65:00", 3: "75:00"}
    assert T.normalize_bus_id("0000:8C:00.0") == "8c:00"
    assert T.normalize_bus_id("8c:00.0") == "8c:00"


def test_link_matrix_maps_ranks_by_bus_id():
    smi_bus = T.parse_showbus(SHOWBUS)
    # rocm-smi link types between node GPUs 0..3: 2 <-> 3 over PCIe, every other pair xGMI
    types = {(i, j): ("PCIE" if {i, j} == {2, 3} else "XGMI") for i in range(4) for j in range(4) if i != j}
    # ranks run on node GPUs 3, 2, 0 (e.g. HIP_VISIBLE_DEVICES=3,2,0): rank index != rocm-smi index
    links = T.link_matrix_for(["75:00", "65:00", "05:00"], types=types, smi_bus=smi_bus)
    assert links == [[0, 0, 1], [0, 0, 1], [1, 1, 0]]
    # two ranks on one GPU are linked; an unknown GPU falls back to the peer-access matrix
    links = T.link_matrix_for(["05:00", "05:00", "aa:00"], peer=[[1, 1, 0], [1, 1, 1], [0, 1, 1]], types=types,
                              smi_bus=smi_bus)
    assert links == [[0, 1, 0], [1, 0, 1], [0, 1, 0]]
    # no tool answer and no peer matrix: unknown (the planner then assumes a fully connected node)
    assert T.link_matrix_for(["05:00", "aa:00"], types=types, smi_bus=smi_bus) is None
    assert T.link_matrix_for([None, "05:00"], types=types, smi_bus=smi_bus) is None


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _agree_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        bus = ["05:00", "15:00", "65:00"]
        T.own_bus_id = lambda: bus[rank]  # this rank's GPU
        T.rocm_smi_bus_ids = lambda: T.parse_showbus(SHOWBUS)
        if rank == 0:
            T.rocm_smi_links = lambda: {(i, j): ("PCIE" if {i, j} == {0, 2} else "XGMI")
                                        for i in range(4) for j in range(4) if i != j}
        else:  # this rank's rocm-smi timed out: on its own it would report nothing usable
            T.rocm_smi_links = lambda: {}
        q.put((rank, T.agreed_link_matrix(world)))
    finally:
        dist.destroy_process_group()


@pytest.mark.slow
def test_agreed_link_matrix_is_rank0s():
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_agree_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    want = [[0, 1, 0], [1, 0, 1], [0, 1, 0]]  # node GPUs 0 and 2 (ranks 0 and 2) only over PCIe
    assert all(got[r] == want for r in range(world)), got
