"""Deferred bias-gradient reduces of the fused local update (GemmArgs::defer_colsum, ops/gemm.py flush_colsum).

A fused-update bwd-weight GEMM with an unsplit plan leaves its bias-gradient partials in a workspace of its own and
queues their ordered reduce (+ BFP round trip + SGD of the bias segment) on the stream; the next split-K wire reduce
of the stream runs the queue in its first blocks (splitk_reduce_wire4_kernel QCS), flush_colsum launches what is left
as one grouped launch. Same reduce, same order: bit-identical to the reduce launched right after its GEMM.
"""
import pytest
import torch

from fpga_ai_nic_amd.ops import gemm as G
from fpga_ai_nic_amd.ops import wire
from fpga_ai_nic_amd.parallel.transport import ThreadFabric

pytestmark = pytest.mark.gpu

RNE = wire.codec_id("bfp_rne")


def _layer(cin, cout, mb, seed):
    g = torch.Generator().manual_seed(seed)
    x = ((torch.rand(mb, cin, generator=g) * 2 - 1) * 0.5).to("cuda", torch.bfloat16)
    dz = ((torch.rand(mb, cout, generator=g) * 2 - 1) * 0.1).to("cuda", torch.bfloat16)
    n = cin * cout + cout
    n_pad = (n + 255) // 256 * 256
    master = ((torch.rand(n_pad, generator=g) * 2 - 1) * 0.05).cuda()
    return dict(x=x, dz=dz, n=n, n_pad=n_pad, cin=cin, cout=cout, master=master)


def _run(L, plan, defer, opt):
    """One fused-update bwd-weight GEMM of layer L; returns (master, lp, colsum) planes it updates."""
    master = L["master"].clone()
    lp = master.to(torch.bfloat16)
    grad = torch.zeros(L["n_pad"], device="cuda")
    buf = torch.zeros(wire.shard_bytes("bfp_rne", L["n_pad"]), dtype=torch.uint8, device="cuda")
    cin, cout, n = L["cin"], L["cout"], L["n"]
    G.gemm(L["x"], True, L["dz"], False, grad[: cin * cout].view(cin, cout), G.EPI_WIRE, colsum=grad[cin * cout:n],
           wire=(buf, L["n_pad"], -1, RNE), update=G.LocalUpdate(master, lp, **opt), defer_colsum=defer, **plan)
    return master, lp, grad


@pytest.mark.parametrize("tile", [(256, 256), (256, 128), (128, 128)])
def test_deferred_colsum_flush_bit_identical(tile):
    opt = dict(lr=0.05, weight_decay=1e-4)
    L = _layer(1024, 1024, 1024, 11)
    ref = _run(L, dict(split_k=1, tile=tile), False, opt)
    assert G.pending_colsum() == 0
    got = _run(L, dict(split_k=1, tile=tile), True, opt)
    assert G.pending_colsum() == 1, "the unsplit fused-update GEMM queues its bias-gradient reduce"
    assert G.flush_colsum() == 1
    assert G.pending_colsum() == 0
    torch.cuda.synchronize()
    for a, b in zip(ref, got):
        assert torch.equal(a, b)


def test_deferred_colsum_rides_on_split_reduce():
    """Two queued reduces (layers 2 and 1 of an MLP at MB 1792) run inside the next split-K fused update's reduce."""
    opt = dict(lr=0.02, momentum=0.0)
    La = _layer(1024, 1024, 1792, 21)
    Lb = _layer(512, 1024, 1792, 22)
    Ls = _layer(1024, 2048, 2048, 23)
    refs = [_run(La, dict(split_k=1, tile=(128, 128)), False, opt), _run(Lb, dict(split_k=1, tile=(256, 128)), False, opt),
            _run(Ls, dict(split_k=4, tile=(256, 256)), False, opt)]
    got_a = _run(La, dict(split_k=1, tile=(128, 128)), True, opt)
    got_b = _run(Lb, dict(split_k=1, tile=(256, 128)), True, opt)
    assert G.pending_colsum() == 2
    got_s = _run(Ls, dict(split_k=4, tile=(256, 256)), True, opt)  # split plan: nothing queued, the queue consumed
    assert G.pending_colsum() == 0
    assert G.flush_colsum() == 0
    torch.cuda.synchronize()
    for ref, got in zip(refs, (got_a, got_b, got_s)):
        for a, b in zip(ref, got):
            assert torch.equal(a, b)


@pytest.mark.parametrize("sizes,mb", [([1024, 4096, 4096, 1024], 1792), ([1024, 4096, 4096, 1024], 2048),
                                      ([512, 1024, 512, 256], 384)])
def test_trainer_deferred_colsum_bit_identical(sizes, mb):
    from fpga_ai_nic_amd.models.mlp import MLP
    from fpga_ai_nic_amd.parallel.dp import DataParallelTrainer, make_engine

    res = []
    for defer in (False, True):
        eng = make_engine(ThreadFabric(1).transport(0), "bfp", impl="native")
        m = MLP(sizes, dtype=torch.bfloat16, device="cuda", seed=3, bias=True,
                pad_fn=lambda n, e=eng: e.layout(n).n_pad)
        tr = DataParallelTrainer(m, eng, lr=0.02)
        assert tr.fused_update
        tr.defer_colsum = defer
        g = torch.Generator().manual_seed(5)
        x = (torch.rand(mb, sizes[0], generator=g) * 2 - 1).to("cuda", torch.bfloat16)
        y = torch.randint(0, sizes[-1], (mb,), generator=g, dtype=torch.int32).cuda()
        losses = [tr.step(x, y).float().mean().item() for _ in range(3)]
        assert G.pending_colsum() == 0, "every queued bias update lands within its step"
        tr.finish()
        res.append((losses, [(l.master.cpu(), l.lp.cpu(), l.gb.cpu()) for l in m.layers]))
    assert res[0][0] == res[1][0], "losses differ"
    for a, b in zip(res[0][1], res[1][1]):
        for u, v in zip(a, b):
            assert torch.equal(u, v)
