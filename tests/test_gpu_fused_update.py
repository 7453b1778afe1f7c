"""Fused local update: the single-rank step's decode + SGD pass folded into the bwd-weight GEMM's wire epilogue.

With one rank the compressed all-reduce is the identity, so the engine's epilogue applies SGD to exactly the BFP
round trip of the GEMM's dW. The fused epilogue (csrc/gemm/gemm_bf16_kernel.h WireOut::um) does the same round trip
in registers and updates master / lp / mom in place. These tests pin it BIT-EXACTLY to the unfused kernels:

* GEMM level: wire epilogue -> ``wire_sgd`` (the engine's epilogue kernel) vs the fused update, for every bwd-weight
  plan family (persistent 4-wave 256x256, 256x128, the 8-wave loop, split-K with the slab-reduce epilogue, the fused
  bias gradient both in-kernel and by the partial-slab reduce), with and without momentum / weight decay / nesterov;
* trainer level: ``DataParallelTrainer(fused_update=True)`` vs ``False`` on the world-1 native engine, several
  steps, bias / no bias, momentum + weight decay: identical losses and identical master, lp and momentum planes.
"""
import pytest
import torch

from fpga_ai_nic_amd.ops import gemm as G
from fpga_ai_nic_amd.ops import wire
from fpga_ai_nic_amd.parallel.transport import ThreadFabric

pytestmark = pytest.mark.gpu

RNE = wire.codec_id("bfp_rne")


def _planes(n_pad, seed, mom):
    g = torch.Generator().manual_seed(seed)
    master = ((torch.rand(n_pad, generator=g) * 2 - 1) * 0.05).cuda()
    lp = master.to(torch.bfloat16)
    m = ((torch.rand(n_pad, generator=g) * 2 - 1) * 0.01).cuda() if mom else None
    return master, lp, m


@pytest.mark.parametrize("plan", [dict(split_k=1, tile=(256, 256)), dict(split_k=1, tile=(256, 128)),
                                  dict(split_k=2, tile=(256, 256)), dict(split_k=4, tile=(256, 256)),
                                  dict(split_k=2, tile=(256, 128)), dict(split_k=1, tile=(128, 128))])
@pytest.mark.parametrize("bias", [True, False])
@pytest.mark.parametrize("opt", [dict(lr=0.05), dict(lr=0.02, weight_decay=1e-3, momentum=0.9),
                                 dict(lr=0.02, momentum=0.9, nesterov=True, grad_scale=0.5)])
def test_gemm_fused_update_matches_wire_sgd(plan, bias, opt):
    cin, cout, mb = 1024, 1024, 1024
    torch.manual_seed(cin + plan["split_k"])
    x = (torch.randn(mb, cin, device="cuda") * 0.5).to(torch.bfloat16)
    dz = (torch.randn(mb, cout, device="cuda") * 0.1).to(torch.bfloat16)
    n = cin * cout + cout
    n_pad = (n + 255) // 256 * 256
    mom = "momentum" in opt
    # reference: GEMM -> one-shard wire -> the engine's decode + SGD kernel
    grad = torch.zeros(n_pad, device="cuda")
    buf = torch.zeros(wire.shard_bytes("bfp_rne", n_pad), dtype=torch.uint8, device="cuda")
    G.gemm(x, True, dz, False, grad[: cin * cout].view(cin, cout), G.EPI_WIRE,
           colsum=grad[cin * cout:n] if bias else None, wire=(buf, n_pad, -1, RNE), **plan)
    m0, l0, mm0 = _planes(n_pad, 7, mom)
    m_ref, l_ref = m0.clone(), l0.clone()
    mm_ref = mm0.clone() if mom else None
    n_upd = n if bias else cin * cout
    wire.sgd(buf, n_pad, 1, m_ref, codec="bfp_rne", lp=l_ref, mom=mm_ref, n_valid=n_upd, **opt)
    # fused
    m_f, l_f = m0.clone(), l0.clone()
    mm_f = mm0.clone() if mom else None
    upd = G.LocalUpdate(m_f, l_f, mm_f, **opt)
    grad2 = torch.zeros(n_pad, device="cuda")
    buf2 = torch.zeros_like(buf)
    G.gemm(x, True, dz, False, grad2[: cin * cout].view(cin, cout), G.EPI_WIRE,
           colsum=grad2[cin * cout:n] if bias else None, wire=(buf2, n_pad, -1, RNE), update=upd, **plan)
    torch.cuda.synchronize()
    assert torch.equal(m_f, m_ref), f"master differs: {(m_f - m_ref).abs().max().item()}"
    assert torch.equal(l_f, l_ref), "bf16 copy differs"
    if mom:
        assert torch.equal(mm_f, mm_ref), "momentum differs"
    assert torch.all(buf2 == 0), "the fused update stores no wire"
    assert not torch.equal(m_f, m0), "weights not updated"


def test_gemm_fused_update_rejects_trunc_and_owner():
    x = torch.zeros(256, 256, device="cuda", dtype=torch.bfloat16)
    n = 256 * 256
    c = torch.zeros(256, 256, device="cuda")
    buf = torch.zeros(wire.shard_bytes("bfp_rne", n), dtype=torch.uint8, device="cuda")
    master = torch.zeros(n, device="cuda")
    with pytest.raises(RuntimeError, match="rne"):
        G.gemm(x, True, x, False, c, G.EPI_WIRE, wire=(buf, n, -1, wire.codec_id("bfp_trunc")),
               update=G.LocalUpdate(master, lr=0.1))
    with pytest.raises(RuntimeError, match="owner"):
        G.gemm(x, True, x, False, c, G.EPI_WIRE, wire=(buf, n, 0, RNE), update=G.LocalUpdate(master, lr=0.1))


@pytest.mark.parametrize("sizes,mb,bias,opt", [
    ([1024, 4096, 4096, 1024], 512, True, dict(lr=0.01)),
    ([512, 1024, 512, 256], 256, True, dict(lr=0.05, momentum=0.9, weight_decay=1e-4)),
    ([512, 1024, 512, 256], 384, False, dict(lr=0.05, momentum=0.9, nesterov=True)),
])
def test_trainer_fused_update_bit_identical(sizes, mb, bias, opt):
    from fpga_ai_nic_amd.models.mlp import MLP
    from fpga_ai_nic_amd.parallel.dp import DataParallelTrainer, make_engine

    res = []
    for fused in (False, True):
        eng = make_engine(ThreadFabric(1).transport(0), "bfp", impl="native")
        m = MLP(sizes, dtype=torch.bfloat16, device="cuda", seed=3, momentum="momentum" in opt, bias=bias,
                pad_fn=lambda n, e=eng: e.layout(n).n_pad)
        tr = DataParallelTrainer(m, eng, fused_update=fused, **opt)
        assert tr.fused_update == fused
        g = torch.Generator().manual_seed(5)
        x = (torch.rand(mb, sizes[0], generator=g) * 2 - 1).to("cuda", torch.bfloat16)
        y = torch.randint(0, sizes[-1], (mb,), generator=g, dtype=torch.int32).cuda()
        losses = [tr.step(x, y).float().mean().item() for _ in range(4)]
        tr.finish()
        assert tr.fused_updates == (4 * m.L if fused else 0)
        res.append((losses, [(l.master.cpu(), l.lp.cpu(), None if l.mom is None else l.mom.cpu()) for l in m.layers]))
    assert res[0][0] == res[1][0], "losses differ"
    for (a, b) in zip(res[0][1], res[1][1]):
        assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
        if a[2] is not None:
            assert torch.equal(a[2], b[2])
