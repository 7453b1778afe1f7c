"""Failure detection on CPU: the debug verify mode (per-message checksum + request
sequence number) catches injected corruption / dropped messages, and a missing peer ends in an error within
the fabric timeout instead of the reference's unbounded spin (sw/mlp_mpi_example_f32.cpp:163-168)."""
import numpy as np
import pytest
import torch

from fpga_ai_nic_amd.parallel.allreduce import ChecksumError, CompressedAllReduce
from fpga_ai_nic_amd.parallel.transport import ThreadFabric
from fpga_ai_nic_amd.utils.faults import FaultInjector


def _run(N, algo, verify, fault_rank=None, fault="", drop_round=None, n=3000, timeout=30):
    rng = np.random.default_rng(5)
    grads = [rng.standard_normal(n).astype(np.float32) for _ in range(N)]
    fabric = ThreadFabric(N, timeout_s=timeout)
    fabric.fault_drop_round = drop_round

    def fn(t):
        eng = CompressedAllReduce(t, codec="bfp_rne", algo=algo, max_slice_elems=512, device="cpu", verify=verify)
        if t.rank == fault_rank:
            eng.fault = FaultInjector(fault)
        L = eng.layout(n)
        g = torch.zeros(L.n_pad)
        g[:n] = torch.from_numpy(grads[t.rank])
        out = torch.zeros(L.n_pad)
        eng.allreduce(g, out, n_valid=n).synchronize()
        return out.numpy().copy()

    return fabric.run(fn)


def _root_causes(e):
    out = []
    while e is not None:
        out.append(e)
        e = e.__cause__
    return out


@pytest.mark.parametrize("algo", ["mesh", "ring"])
def test_verify_mode_is_transparent(algo):
    a = _run(3, algo, verify=False)
    b = _run(3, algo, verify=True)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)


@pytest.mark.parametrize("algo,site", [("mesh", "mesh_pack"), ("ring", "ring_send")])
def test_verify_catches_corruption(algo, site):
    with pytest.raises(RuntimeError) as ei:
        _run(3, algo, verify=True, fault_rank=1, fault=f"{site}:0:flip")
    assert any(isinstance(e, ChecksumError) for e in _root_causes(ei.value)), repr(ei.value)
    assert "corrupted" in str(ei.value.__cause__)


def test_corruption_undetected_without_verify_changes_result():
    clean = _run(3, "mesh", verify=False)
    bad = _run(3, "mesh", verify=False, fault_rank=1, fault="mesh_pack:0:flip")
    assert any(not np.array_equal(x, y) for x, y in zip(clean, bad))


def test_verify_catches_dropped_ring_message():
    with pytest.raises(RuntimeError) as ei:
        _run(3, "ring", verify=True, drop_round=1)
    assert any(isinstance(e, ChecksumError) for e in _root_causes(ei.value)), repr(ei.value)


def test_missing_peer_times_out():
    fabric = ThreadFabric(2, timeout_s=1.0)
    t0 = fabric.transport(0)
    eng = CompressedAllReduce(t0, codec="bfp_rne", device="cpu")
    L = eng.layout(1024)
    import threading

    with pytest.raises(threading.BrokenBarrierError):
        eng.allreduce(torch.ones(L.n_pad), torch.zeros(L.n_pad), n_valid=1024)  # rank 1 never shows up
