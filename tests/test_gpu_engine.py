"""The all-reduce engine on one GPU with N virtual ranks (threads): bit-exact vs the spec simulators."""
import numpy as np
import pytest
import torch

from fpga_ai_nic_amd.ops import bfp_oracle as O
from fpga_ai_nic_amd.parallel import sim
from fpga_ai_nic_amd.parallel.allreduce import CompressedAllReduce
from fpga_ai_nic_amd.parallel.transport import ThreadFabric

pytestmark = pytest.mark.gpu


def _run(N, algo, rings, codec, n, max_slice=1024, lr=0.5, dtype=torch.float32):
    rng = np.random.default_rng(N * 10 + rings)
    grads_np = [rng.standard_normal(n).astype(np.float32) * (1 + r) for r in range(N)]
    w0 = rng.standard_normal(n).astype(np.float32)
    fabric = ThreadFabric(N)

    def fn(t):
        eng = CompressedAllReduce(t, codec=codec, algo=algo, rings=rings, max_slice_elems=max_slice)
        L = eng.layout(n)
        g = torch.zeros(L.n_pad, device="cuda", dtype=dtype)
        g[:n] = torch.from_numpy(grads_np[t.rank]).to(dtype)
        w = torch.zeros(L.n_pad, device="cuda")
        w[:n] = torch.from_numpy(w0)
        lp = torch.zeros(L.n_pad, device="cuda", dtype=torch.bfloat16)
        out = torch.zeros(L.n_pad, device="cuda")
        eng.allreduce(g, out, n_valid=n).synchronize()
        eng.allreduce_sgd(g, w, lp, n_valid=n, lr=lr).synchronize()
        return out.cpu().numpy(), w.cpu().numpy(), L, eng.orders

    res = fabric.run(fn)
    L, orders = res[0][2], res[0][3]
    gin = [np.pad(g.astype(np.float32) if dtype == torch.float32 else
                  torch.from_numpy(g).to(dtype).float().numpy(), (0, L.n_pad - n)) for g in grads_np]
    if algo == "mesh":
        exp = sim.mesh_allreduce(gin, L.shard, codec)
    else:
        exp = sim.ring_allreduce(gin, orders, L.slice_elems, L.blocks, codec)[0]
    for r in range(N):
        assert np.array_equal(res[r][0][:n], exp[:n]), f"rank {r}: reduced gradient mismatch"
        assert np.array_equal(res[r][1], res[0][1]), "replicas must be bit-identical"
    ref_w, _ = O.sgd(w0, exp[:n], lr)
    ulp = np.abs(res[0][1][:n].view(np.int32).astype(np.int64) - ref_w.view(np.int32).astype(np.int64))
    assert ulp.max() <= 1
    return exp, grads_np


@pytest.mark.parametrize("N", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("algo,rings", [("mesh", 1), ("ring", 1), ("ring", 7)])
def test_engine_virtual_ranks_bitexact(N, algo, rings):
    _run(N, algo, rings, "bfp_rne", n=20000)


@pytest.mark.parametrize("codec", ["bfp_trunc", "raw_f32", "raw_bf16"])
def test_engine_codecs(codec):
    _run(4, "ring", 2, codec, n=5000)
    _run(4, "mesh", 1, codec, n=5000)


def test_engine_bf16_grads():
    _run(3, "mesh", 1, "bfp_rne", n=4096, dtype=torch.bfloat16)


def test_bfp_error_bound_vs_fp32():
    exp, grads = _run(8, "mesh", 1, "bfp_rne", n=1 << 16)
    true = np.sum(grads, axis=0)
    scale = np.abs(np.stack(grads)).max()
    # each contribution quantised once (+ the sum once): error <= (N+1) * 2^-7 * max|group| per element
    assert np.abs(exp[: true.size] - true).max() <= 9 * 2.0 ** -7 * scale * 2
