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


# ---------------------------------------------------------------------------------------------------------------
# The same checks on the production path: the C++ engine (csrc/comm/engine.cpp + verify.hip) with N virtual ranks
# on one GPU over the loopback communicator. Tags are computed and checked by GPU kernels; the host raises at
# synchronize().


def _run_native(N, algo, verify, fault_rank=None, fault="", lose_round=None, n=3000):
    import threading

    from fpga_ai_nic_amd import _ext
    from fpga_ai_nic_amd.parallel.native_engine import NativeAllReduce

    C = _ext.require()
    fabric = C.LoopbackFabric(N, 30.0)
    rng = np.random.default_rng(5)
    grads = [rng.standard_normal(n).astype(np.float32) for _ in range(N)]
    comms = [fabric.comm(r) for r in range(N)]
    if lose_round is not None:
        comms[1].lose_round(lose_round)
    engines = [NativeAllReduce(None, codec="bfp_rne", algo=algo, max_slice_elems=512, comm=comms[r], verify=verify,
                               fault=fault if r == fault_rank else "") for r in range(N)]
    out, errs = [None] * N, [None] * N

    def body(r):
        try:
            eng = engines[r]
            L = eng.layout(n)
            g = torch.zeros(L.n_pad, device="cuda")
            g[:n] = torch.from_numpy(grads[r]).cuda()
            o = torch.zeros(L.n_pad, device="cuda")
            torch.cuda.synchronize()
            eng.allreduce(g, o, n_valid=n).synchronize(30)
            out[r] = o.cpu().numpy()
        except Exception as e:  # noqa: BLE001
            errs[r] = e

    ts = [threading.Thread(target=body, args=(r,)) for r in range(N)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(90)
    assert not any(t.is_alive() for t in ts), "virtual rank hung"
    return out, errs, engines


@pytest.mark.gpu
@pytest.mark.parametrize("algo", ["mesh", "ring"])
def test_native_verify_mode_is_transparent(algo):
    a, ea, _ = _run_native(3, algo, verify=False)
    b, eb, engs = _run_native(3, algo, verify=True)
    assert not any(ea) and not any(eb), (ea, eb)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)
    assert engs[0].counters()["verified_rows"] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("algo,site", [("mesh", "mesh_pack"), ("mesh", "mesh_reduce"), ("ring", "ring_send")])
def test_native_verify_catches_corruption(algo, site):
    out, errs, _ = _run_native(3, algo, verify=True, fault_rank=1, fault=f"{site}:0:flip")
    caught = [e for e in errs if isinstance(e, ChecksumError)]
    assert caught, errs
    assert "corrupted" in str(caught[0])


@pytest.mark.gpu
def test_native_corruption_undetected_without_verify_changes_result():
    clean, e0, _ = _run_native(3, "mesh", verify=False)
    bad, e1, _ = _run_native(3, "mesh", verify=False, fault_rank=1, fault="mesh_pack:0:flip")
    assert not any(e0) and not any(e1)
    assert any(not np.array_equal(x, y) for x, y in zip(clean, bad))


@pytest.mark.gpu
def test_native_verify_catches_lost_ring_message():
    """Rank 1's second ring round is lost in flight (its receivers keep stale buffers): the stale tags carry the
    wrong request / checksum, so verify mode raises instead of silently training on stale data."""
    out, errs, _ = _run_native(3, "ring", verify=True, lose_round=1)
    assert any(isinstance(e, ChecksumError) for e in errs), errs


@pytest.mark.gpu
def test_native_missing_peer_times_out():
    from fpga_ai_nic_amd import _ext
    from fpga_ai_nic_amd.parallel.native_engine import NativeAllReduce

    C = _ext.require()
    fabric = C.LoopbackFabric(2, 1.0)
    eng = NativeAllReduce(None, codec="bfp_rne", comm=fabric.comm(0))
    L = eng.layout(1024)
    with pytest.raises(RuntimeError, match="timed out"):  # rank 1 never shows up
        eng.allreduce(torch.ones(L.n_pad, device="cuda"), torch.zeros(L.n_pad, device="cuda"), n_valid=1024)


@pytest.mark.gpu
@pytest.mark.parametrize("spec", ["mesh_pack:x:flip", "mesh_pack:0:boom", "ring_send:1:delay_ms=-1", "mesh_pack"])
def test_native_fault_spec_rejected_up_front(spec):
    """A malformed FAN_FAULT rule fails when the engine is configured (csrc/comm/fault_spec.cpp), not in the
    middle of a request; the grammar parser itself runs under ASan/UBSan in test_native_sanitizers.py."""
    from fpga_ai_nic_amd.parallel.native_engine import NativeAllReduce

    with pytest.raises(ValueError, match="FAN_FAULT"):
        NativeAllReduce(None, codec="bfp_rne", fault=spec)
