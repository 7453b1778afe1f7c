"""Multi-process data-parallel tests over torch.distributed gloo (CPU) — BASELINE config 1
("3-layer MLP f32 SGD, world_size=2 on CPU via gloo"). This is the same code path the GPU run takes with the
RCCL backend: TorchDistTransport -> engine -> trainer."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from fpga_ai_nic_amd.models.mlp import MLP
from fpga_ai_nic_amd.parallel import sim
from fpga_ai_nic_amd.parallel.allreduce import CompressedAllReduce
from fpga_ai_nic_amd.parallel.dp import DataParallelTrainer, make_engine
from fpga_ai_nic_amd.parallel.transport import TorchDistTransport

pytestmark = pytest.mark.slow


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)


def _engine_worker(rank, world, port, algo, rings, q):
    _init(rank, world, port)
    try:
        t = TorchDistTransport()
        n = 5000
        rng = np.random.default_rng(7)
        grads = [rng.standard_normal(n).astype(np.float32) for _ in range(world)]
        eng = CompressedAllReduce(t, codec="bfp_rne", algo=algo, rings=rings, max_slice_elems=512, device="cpu")
        L = eng.layout(n)
        g = torch.zeros(L.n_pad)
        g[:n] = torch.from_numpy(grads[rank])
        out = torch.zeros(L.n_pad)
        eng.allreduce(g, out, n_valid=n).synchronize()
        gin = [np.pad(x, (0, L.n_pad - n)) for x in grads]
        exp = sim.mesh_allreduce(gin, L.shard) if algo == "mesh" else \
            sim.ring_allreduce(gin, eng.orders, L.slice_elems, L.blocks)[0]
        q.put((rank, bool(np.array_equal(out.numpy()[:n], exp[:n]))))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,algo,rings", [(2, "mesh", 1), (3, "ring", 2), (4, "mesh", 1), (4, "ring", 2),
                                              (8, "ring", 7), (8, "mesh", 1)])
def test_engine_over_gloo(world, algo, rings):
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    pc = mp.start_processes(_engine_worker, args=(world, _free_port(), algo, rings, q), nprocs=world, join=False,
                            start_method="spawn")
    res = dict(q.get() for _ in range(world))
    while not pc.join():
        pass
    assert all(res.values()), res


def _mlp_worker(rank, world, port, kind, q):
    _init(rank, world, port)
    try:
        sizes = [64, 256, 256, 64]  # 3-layer MLP (BASELINE config 1), f32, SGD
        t = TorchDistTransport()
        eng = make_engine(t, kind)
        model = MLP(sizes, dtype=torch.float32, device="cpu", pad_fn=lambda n: eng.layout(n).n_pad, seed=3)
        for l in model.layers:
            t.broadcast_(l.master, 0)
        tr = DataParallelTrainer(model, eng, lr=0.1)
        g = torch.Generator().manual_seed(100)
        X = torch.rand(32, sizes[0], generator=g) * 2 - 1
        Y = torch.randint(0, sizes[-1], (32,), generator=g, dtype=torch.int32)
        mb = 32 // world
        x, y = X[rank * mb:(rank + 1) * mb], Y[rank * mb:(rank + 1) * mb]
        losses = []
        for _ in range(4):
            losses.append(float(tr.step(x, y).mean()))
        tr.finish()
        w = torch.cat([l.master for l in model.layers]).numpy()
        q.put((rank, w, losses))
    finally:
        dist.destroy_process_group()


def _single_process_reference(steps=4):
    sizes = [64, 256, 256, 64]
    model = MLP(sizes, dtype=torch.float32, device="cpu", seed=3)
    tr = DataParallelTrainer(model, None, lr=0.1)
    g = torch.Generator().manual_seed(100)
    X = torch.rand(32, sizes[0], generator=g) * 2 - 1
    Y = torch.randint(0, sizes[-1], (32,), generator=g, dtype=torch.int32)
    for _ in range(steps):
        tr.step(X, Y)
    return model


@pytest.mark.parametrize("kind", ["bfp", "raw", "rccl"])
def test_dp_mlp_gloo_world2(kind):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    pc = mp.start_processes(_mlp_worker, args=(world, _free_port(), kind, q), nprocs=world, join=False,
                            start_method="spawn")
    res = {r: (w, l) for r, w, l in (q.get() for _ in range(world))}
    while not pc.join():
        pass
    assert np.array_equal(res[0][0], res[1][0]), "replicas must stay bit-identical"
    ref = _single_process_reference()
    wref = torch.cat([torch.cat([l.w_master.reshape(-1), l.b_master]) for l in ref.layers]).numpy()
    sizes = [64, 256, 256, 64]

    _T = type("_T", (), {"rank": 0, "world": world, "name": "layout"})  # layout-only stand-in transport
    e = make_engine(_T(), kind)
    flat, off = [], 0
    for i in range(3):
        n = sizes[i] * sizes[i + 1] + sizes[i + 1]
        flat.append(res[0][0][off:off + n])
        off += e.layout(n).n_pad
    assert off == res[0][0].size
    w_dp = np.concatenate(flat)
    tol = 1e-5 if kind in ("raw", "rccl") else 2e-2
    assert np.abs(w_dp - wref).max() < tol, np.abs(w_dp - wref).max()
    assert res[0][1][-1] < res[0][1][0] + 1e-3
