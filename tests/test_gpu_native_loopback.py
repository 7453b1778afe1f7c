"""The native C++ engine with N virtual ranks on one GPU (LoopbackFabric, one host thread per rank):
its multi-rank mesh / ring / multi-ring schedules bit-exact vs the spec simulators, replicas bit-identical,
and injected faults surface as errors instead of hangs."""
import threading

import numpy as np
import pytest
import torch

from fpga_ai_nic_amd import _ext
from fpga_ai_nic_amd.ops import bfp_oracle as O
from fpga_ai_nic_amd.parallel import sim
from fpga_ai_nic_amd.parallel.native_engine import NativeAllReduce

pytestmark = pytest.mark.gpu


def _threads(N, fn):
    out, errs = [None] * N, [None] * N

    def run(r):
        try:
            out[r] = fn(r)
        except Exception as e:  # noqa: BLE001
            errs[r] = e

    ts = [threading.Thread(target=run, args=(r,)) for r in range(N)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(120)
    assert not any(t.is_alive() for t in ts), "virtual rank thread hung"
    return out, errs


def _run(N, algo, rings, codec, n, max_slice=1024, lr=0.5, dtype=torch.float32, compat=False, epi_producer=False):
    C = _ext.require()
    fabric = C.LoopbackFabric(N, 60.0)
    rng = np.random.default_rng(N * 100 + rings)
    grads_np = [rng.standard_normal(n).astype(np.float32) * (1 + r) for r in range(N)]
    w0 = rng.standard_normal(n).astype(np.float32)
    engines = [NativeAllReduce(None, codec=codec, algo=algo, rings=rings, max_slice_elems=max_slice,
                               comm=fabric.comm(r), compat_owner_fp32=compat) for r in range(N)]
    for e in engines:
        e.epilogue_on_producer = epi_producer
        assert e.epilogue_on_producer == epi_producer
    L = engines[0].layout(n)

    def fn(r):
        eng = engines[r]
        g = torch.zeros(L.n_pad, device="cuda", dtype=dtype)
        g[:n] = torch.from_numpy(grads_np[r]).to(dtype)
        w = torch.zeros(L.n_pad, device="cuda")
        w[:n] = torch.from_numpy(w0)
        lp = torch.zeros(L.n_pad, device="cuda", dtype=torch.bfloat16)
        out = torch.zeros(L.n_pad, device="cuda")
        torch.cuda.synchronize()
        eng.allreduce(g, out, n_valid=n).synchronize(60)
        h = eng.allreduce_sgd(g, w, lp, n_valid=n, lr=lr, defer=True)
        h.commit_after_current()
        h.synchronize(60)
        torch.cuda.synchronize()
        return out.cpu().numpy(), w.cpu().numpy(), lp.cpu()

    res, errs = _threads(N, fn)
    for e in errs:
        if e is not None:
            raise e
    gin = [np.pad(g if dtype == torch.float32 else torch.from_numpy(g).to(dtype).float().numpy(),
                  (0, L.n_pad - n)) for g in grads_np]
    if algo == "mesh":
        exp = sim.mesh_allreduce(gin, L.shard, codec)
        per_rank = [exp] * N
    else:
        exp = sim.ring_allreduce(gin, engines[0].orders, L.slice_elems, L.blocks, codec)[0]
        per_rank = sim.ring_allreduce(gin, engines[0].orders, L.slice_elems, L.blocks, codec, owner_fp32=compat)
    for r in range(N):
        assert np.array_equal(res[r][0][:n], exp[:n]), f"rank {r}: reduced sum mismatch"
        ref_w, _ = O.sgd(w0, per_rank[r][:n], lr)
        ulp = np.abs(res[r][1][:n].view(np.int32).astype(np.int64) - ref_w.view(np.int32).astype(np.int64))
        assert ulp.max() <= 1, f"rank {r}: weights off by {ulp.max()} ulp"
        if not compat:
            assert np.array_equal(res[r][1], res[0][1]), "replicas must be bit-identical"
            assert torch.equal(res[r][2], res[0][2])
    return res, exp, L


@pytest.mark.parametrize("N", [2, 3, 4, 8])
@pytest.mark.parametrize("algo,rings", [("mesh", 1), ("ring", 1), ("ring", 7)])
def test_loopback_schedules_bitexact(N, algo, rings):
    _run(N, algo, rings, "bfp_rne", n=20000)


@pytest.mark.parametrize("algo,rings", [("mesh", 1), ("ring", 2)])
def test_loopback_epilogue_on_producer_stream(algo, rings):
    # the decode+SGD epilogue enqueued on the committing (compute) stream after the comm phase: same bits
    _run(4, algo, rings, "bfp_rne", n=20000, epi_producer=True)


@pytest.mark.parametrize("codec", ["bfp_trunc", "raw_f32", "raw_bf16"])
def test_loopback_codecs(codec):
    _run(4, "ring", 2, codec, n=5000)
    _run(4, "mesh", 1, codec, n=5000)


def test_loopback_bf16_grads():
    _run(3, "mesh", 1, "bfp_rne", n=4096, dtype=torch.bfloat16)
    _run(3, "ring", 2, "bfp_rne", n=4096, dtype=torch.bfloat16)


def test_loopback_compat_owner_fp32_quirk():
    # reference quirk: the owner of each slice updates from the un-quantised fp32 sum -> replicas differ
    res, exp, L = _run(3, "ring", 1, "bfp_trunc", n=6000, compat=True)
    assert any(not np.array_equal(res[r][1], res[0][1]) for r in range(1, 3)), "compat mode should diverge"


def test_loopback_fault_drop_raises_not_hangs():
    C = _ext.require()
    N = 3
    fabric = C.LoopbackFabric(N, 2.0)
    comms = [fabric.comm(r) for r in range(N)]
    comms[1].drop_after(0)
    engines = [NativeAllReduce(None, codec="bfp_rne", comm=comms[r]) for r in range(N)]
    n = 4096
    L = engines[0].layout(n)

    def fn(r):
        g = torch.ones(L.n_pad, device="cuda")
        w = torch.zeros(L.n_pad, device="cuda")
        torch.cuda.synchronize()
        engines[r].allreduce_sgd(g, w, n_valid=n, lr=0.1).synchronize(10)

    _, errs = _threads(N, fn)
    assert all(e is not None for e in errs)
    assert "fault injection" in str(errs[1])
    assert any("timed out" in str(e) or "aborted" in str(e) for e in (errs[0], errs[2]))


@pytest.mark.parametrize("N", [2, 3])
def test_chunked_mesh_bitexact_and_bounded(N):
    """Buckets above chunk_elems stream through the collectives chunk by chunk (two-stream block pipeline): every
    chunk is its own N-shard mesh all-reduce, so the result is bit-exact vs the spec simulator applied per chunk,
    for the immediate (per-chunk epilogue on the aux stream) and the deferred epilogue; the engine's scratch stays
    bounded by two chunks for immediate requests."""
    C = _ext.require()
    fabric = C.LoopbackFabric(N, 60.0)
    n, chunk = 50_000, 8_192
    rng = np.random.default_rng(N + 40)
    grads = [rng.standard_normal(n).astype(np.float32) * (1 + r) for r in range(N)]
    w0 = rng.standard_normal(n).astype(np.float32)
    engines = [NativeAllReduce(None, codec="bfp_rne", comm=fabric.comm(r), chunk_elems=chunk) for r in range(N)]
    L = engines[0].layout(n)
    assert L.chunks == -(-n // chunk) and L.n_pad == L.shard * N * L.chunks

    def fn(r):
        eng = engines[r]
        g = torch.zeros(L.n_pad, device="cuda")
        g[:n] = torch.from_numpy(grads[r]).cuda()
        out = torch.zeros(L.n_pad, device="cuda")
        w = torch.zeros(L.n_pad, device="cuda")
        w[:n] = torch.from_numpy(w0).cuda()
        w2 = w.clone()
        torch.cuda.synchronize()
        eng.allreduce(g, out, n_valid=n).synchronize(60)
        eng.allreduce_sgd(g, w, None, n_valid=n, lr=0.5).synchronize(60)  # immediate: per-chunk epilogues
        h = eng.allreduce_sgd(g, w2, None, n_valid=n, lr=0.5, defer=True)  # deferred: one epilogue at commit
        h.commit_after_current()
        h.synchronize(60)
        torch.cuda.synchronize()
        return out.cpu().numpy(), w.cpu().numpy(), w2.cpu().numpy()

    res, errs = _threads(N, fn)
    for e in errs:
        if e is not None:
            raise e
    cw = L.shard * N
    gin = [np.pad(x, (0, L.n_pad - n)) for x in grads]
    exp = np.concatenate([sim.mesh_allreduce([x[c * cw:(c + 1) * cw] for x in gin], L.shard, "bfp_rne")
                          for c in range(L.chunks)])
    ref_w, _ = O.sgd(w0, exp[:n], 0.5)
    for r in range(N):
        assert np.array_equal(res[r][0][:n], exp[:n]), f"rank {r}: chunked sum mismatch"
        for w in (res[r][1], res[r][2]):
            ulp = np.abs(w[:n].view(np.int32).astype(np.int64) - ref_w.view(np.int32).astype(np.int64))
            assert ulp.max() <= 1
        assert np.array_equal(res[r][1], res[0][1]) and np.array_equal(res[r][2], res[r][1])
