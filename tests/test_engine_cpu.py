"""Engine correctness on CPU: N virtual ranks (threads) running the real engine code with the oracle codec,
checked bit-exactly against the independent spec simulators (parallel/sim.py)."""
import numpy as np
import pytest
import torch

from fpga_ai_nic_amd.ops import bfp_oracle as O
from fpga_ai_nic_amd.parallel import sim
from fpga_ai_nic_amd.parallel.allreduce import CompressedAllReduce, ring_plan
from fpga_ai_nic_amd.parallel.transport import ThreadFabric


def run_engine(N, algo, rings, codec, n, max_slice=512, lr=0.5, compat=False, momentum=0.0):
    rng = np.random.default_rng(N * 10 + rings)
    grads = [rng.standard_normal(n).astype(np.float32) * (1 + r) for r in range(N)]
    w0 = rng.standard_normal(n).astype(np.float32)
    fabric = ThreadFabric(N, timeout_s=60)

    def fn(t):
        eng = CompressedAllReduce(t, codec=codec, algo=algo, rings=rings, max_slice_elems=max_slice,
                                  compat_owner_fp32=compat, device="cpu")
        L = eng.layout(n)
        g = torch.zeros(L.n_pad)
        g[:n] = torch.from_numpy(grads[t.rank])
        w = torch.zeros(L.n_pad)
        w[:n] = torch.from_numpy(w0)
        out = torch.zeros(L.n_pad)
        eng.allreduce(g, out, n_valid=n).synchronize()
        mom = torch.zeros(L.n_pad) if momentum else None
        eng.allreduce_sgd(g, w, None, mom, n_valid=n, lr=lr, momentum=momentum).synchronize()
        return out.numpy().copy(), w.numpy().copy(), L, eng.orders

    res = fabric.run(fn)
    return res, grads, w0


@pytest.mark.parametrize("N", [1, 2, 3, 4, 5, 8])
@pytest.mark.parametrize("algo,rings", [("mesh", 1), ("ring", 1), ("ring", 7)])
def test_engine_matches_spec(N, algo, rings):
    n = 3000
    res, grads, w0 = run_engine(N, algo, rings, "bfp_rne", n)
    L, orders = res[0][2], res[0][3]
    gin = [np.pad(g, (0, L.n_pad - n)) for g in grads]
    exp = sim.mesh_allreduce(gin, L.shard) if algo == "mesh" else \
        sim.ring_allreduce(gin, orders, L.slice_elems, L.blocks)[0]
    for r in range(N):
        assert np.array_equal(res[r][0][:n], exp[:n])
        assert np.array_equal(res[r][1], res[0][1])
    ref_w, _ = O.sgd(w0, exp[:n], 0.5)
    assert np.array_equal(res[0][1][:n], ref_w)
    assert np.all(res[0][1][n:] == 0), "padding untouched"


def test_multi_block_ring_and_trunc_codec():
    n = 10000  # several blocks with max_slice=512
    res, grads, _ = run_engine(3, "ring", 2, "bfp_trunc", n, max_slice=256)
    L, orders = res[0][2], res[0][3]
    assert L.blocks > 1
    gin = [np.pad(g, (0, L.n_pad - n)) for g in grads]
    exp = sim.ring_allreduce(gin, orders, L.slice_elems, L.blocks, "bfp_trunc")[0]
    assert np.array_equal(res[0][0][:n], exp[:n])


def test_ring_compat_owner_fp32_quirk():
    """Reference quirk (hw/all_reduce.sv:1174-1175): the owner updates from the un-quantised sum, so replicas
    diverge; the default (decoded everywhere) keeps them identical."""
    n = 2048
    res, grads, w0 = run_engine(3, "ring", 1, "bfp_rne", n, compat=True)
    L, orders = res[0][2], res[0][3]
    gin = [np.pad(g, (0, L.n_pad - n)) for g in grads]
    per_rank = sim.ring_allreduce(gin, orders, L.slice_elems, L.blocks, owner_fp32=True)
    for r in range(3):
        ref_w, _ = O.sgd(w0, per_rank[r][:n], 0.5)
        assert np.array_equal(res[r][1][:n], ref_w)
    assert not np.array_equal(res[0][1], res[1][1])


@pytest.mark.parametrize("codec", ["raw_f32", "raw_bf16"])
def test_raw_codecs(codec):
    n = 4000
    res, grads, _ = run_engine(4, "mesh", 1, codec, n)
    true = np.sum(grads, axis=0)
    tol = 1e-5 if codec == "raw_f32" else 0.1
    assert np.abs(res[0][0][:n] - true).max() < tol


def test_momentum_path():
    res, grads, w0 = run_engine(2, "mesh", 1, "bfp_rne", 1000, momentum=0.9)
    assert np.isfinite(res[0][1]).all()


def test_plan_every_slice_owned_once_and_all_received():
    for N in (1, 2, 3, 4, 6, 8):
        for blocks in (1, 3):
            owned, got = {}, [set() for _ in range(N)]
            for p in range(N):
                for row in ring_plan(N, p, blocks):
                    send_slice, src, recv_slice, recv_full, own = row
                    if own >= 0:
                        owned.setdefault(own, []).append(p)
                        got[p].add(own)
                    if recv_full:
                        got[p].add(recv_slice)
            assert sorted(owned) == list(range(N * blocks))
            assert all(len(v) == 1 for v in owned.values())
            assert all(g == set(range(N * blocks)) for g in got)


@pytest.mark.parametrize("N", [1, 2, 3])
@pytest.mark.parametrize("algo", ["mesh", "ring"])
def test_deferred_same_size_requests_keep_their_own_result(N, algo):
    """Two same-size requests issued with defer=True and committed only after both were issued (how the
    trainer commits at the end of backward): each epilogue must apply ITS OWN reduced gradient. A gathered
    wire buffer shared per bucket size let the second request's result overwrite the first's."""
    n = 2000
    rng = np.random.default_rng(7 + N)
    grads = [[rng.standard_normal(n).astype(np.float32) * (1 + r + 3 * b) for r in range(N)] for b in range(2)]
    w0 = rng.standard_normal(n).astype(np.float32)

    def fn(t):
        eng = CompressedAllReduce(t, codec="bfp_rne", algo=algo, device="cpu")
        L = eng.layout(n)
        outs = []
        for deferred in (True, False):
            ws, hs = [], []
            for b in range(2):
                g = torch.zeros(L.n_pad)
                g[:n] = torch.from_numpy(grads[b][t.rank])
                w = torch.zeros(L.n_pad)
                w[:n] = torch.from_numpy(w0)
                h = eng.allreduce_sgd(g, w, None, None, n_valid=n, lr=0.5, defer=deferred)
                if not deferred:
                    h.synchronize()
                ws.append(w)
                hs.append(h)
            for h in hs:
                h.commit()
                h.synchronize()
            outs.append([w.numpy().copy() for w in ws])
        return outs

    for deferred, immediate in fabric_run(N, fn):
        for a, b in zip(deferred, immediate):
            assert np.array_equal(a, b)
        assert not np.array_equal(deferred[0], deferred[1])


def fabric_run(N, fn):
    return ThreadFabric(N, timeout_s=60).run(fn)


@pytest.mark.parametrize("N", [1, 2])
@pytest.mark.parametrize("algo", ["mesh", "ring"])
def test_more_deferred_requests_than_slots(N, algo):
    """A 10-layer model (the reference run.sh workload) defers 10 same-size requests before committing: more
    than the 8 request slots. The 9th request reuses slot 0 — the engine must commit request 1 first (its
    per-slot scratch is about to be overwritten) so every request still applies ITS OWN reduced gradient."""
    n, R = 1000, 10
    rng = np.random.default_rng(11 + N)
    grads = [[rng.standard_normal(n).astype(np.float32) * (1 + r + b) for r in range(N)] for b in range(R)]
    w0 = rng.standard_normal(n).astype(np.float32)

    def fn(t):
        eng = CompressedAllReduce(t, codec="bfp_rne", algo=algo, device="cpu")
        L = eng.layout(n)
        outs = []
        for deferred in (True, False):
            ws, hs = [], []
            for b in range(R):
                g = torch.zeros(L.n_pad)
                g[:n] = torch.from_numpy(grads[b][t.rank])
                w = torch.zeros(L.n_pad)
                w[:n] = torch.from_numpy(w0)
                h = eng.allreduce_sgd(g, w, None, None, n_valid=n, lr=0.5, defer=deferred)
                if not deferred:
                    h.synchronize()
                ws.append(w)
                hs.append(h)
            for h in hs:
                h.commit()
                h.synchronize()
            outs.append([w.numpy().copy() for w in ws])
        return outs, eng.stats.get("forced_commits", 0)

    for (deferred, immediate), forced in fabric_run(N, fn):
        assert forced == R - 8
        for a, b in zip(deferred, immediate):
            assert np.array_equal(a, b)


def test_fused_update_only_on_the_single_rank_gpu_engine(monkeypatch):
    """The GEMM-fused update is a single-rank (inline engine), GPU, bf16, rne-codec schedule: the CPU / Python-engine
    trainer keeps the engine's decode + SGD pass (and FAN_FUSED_UPDATE=0 turns the fused path off everywhere)."""
    import torch

    from fpga_ai_nic_amd.models.mlp import MLP
    from fpga_ai_nic_amd.parallel.dp import DataParallelTrainer, make_engine
    from fpga_ai_nic_amd.parallel.transport import ThreadFabric

    eng = make_engine(ThreadFabric(1).transport(0), "bfp")
    m = MLP([32, 64, 16], dtype=torch.float32, device="cpu", pad_fn=lambda n: eng.layout(n).n_pad)
    tr = DataParallelTrainer(m, eng, lr=0.1)
    assert not tr.fused_update and not tr.prepack
    x = torch.randn(8, 32)
    y = torch.randint(0, 16, (8,), dtype=torch.int32)
    tr.step(x, y)
    tr.finish()
    assert tr.fused_updates == 0
    monkeypatch.setenv("FAN_FUSED_UPDATE", "0")
    assert not DataParallelTrainer(m, eng, lr=0.1).fused_update
