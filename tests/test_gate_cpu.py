"""The all-reduce exactness gate (fpga_ai_nic_amd/parallel/gate.py) on CPU: virtual ranks of the Python engine over a
thread fabric. An honest engine passes bit for bit on every rank, for the mesh and the ring over several rings; an
engine whose message is corrupted in flight (fault injection) gives every rank the same wrong sum — the replicas
agree, the gate does not."""
import numpy as np
import pytest
import torch

from fpga_ai_nic_amd.parallel import gate
from fpga_ai_nic_amd.parallel.allreduce import CompressedAllReduce
from fpga_ai_nic_amd.parallel.transport import ThreadFabric


def _run_gate(world, algo, rings, fault=None, n=20000):
    fab = ThreadFabric(world)

    def body(t):
        eng = CompressedAllReduce(t, codec="bfp_rne", algo=algo, rings=rings, max_slice_elems=1024,
                                  device=torch.device("cpu"))
        if fault:
            from fpga_ai_nic_amd.utils.faults import FaultInjector

            eng.fault = FaultInjector(fault)
        return gate.allreduce_exactness(eng, n=n, timeout_s=60)

    return fab.run(body)


@pytest.mark.parametrize("world,algo,rings", [(2, "mesh", 1), (3, "mesh", 1), (3, "ring", 2), (4, "ring", 1)])
def test_gate_passes_an_exact_engine(world, algo, rings):
    for r in _run_gate(world, algo, rings):
        assert r["exact"] and r["checked"] and r["max_abs_diff"] == 0.0, r


def test_gate_rejects_a_corrupted_reduce():
    res = _run_gate(3, "mesh", 1, fault="mesh_pack:0:flip")
    # rank 0's first packed message was corrupted in flight: the owner of that shard reduces a wrong value, and the
    # all-gather hands the same wrong shard to every rank — their results agree with each other, not with the spec
    assert len(res) == 3 and not any(r["exact"] for r in res), res
    assert all(r["max_abs_diff"] > 0 for r in res)


def test_seeded_gradients_cover_many_exponents():
    g = gate.seeded_gradients(4096, 2, 1)
    assert len(g) == 2 and g[0].dtype == np.float32 and not np.array_equal(g[0], g[1])
    e = (g[0].view(np.uint32) >> 23) & 0xFF
    assert e.max() - e.min() > 16  # group scales span 2^-12 .. 2^3 on top of the normal spread
