"""Split-K classifier GEMM folded into the softmax-xent kernel (ops/gemm.py ``defer_reduce``, ops/nn.py
``softmax_xent_slabs``): the GEMM leaves its f32 slabs unreduced and the softmax sums them in split order plus the
bias — the GEMM's own reduce arithmetic — so logits, loss rows and dlogits are bit-identical to the two-launch path.
"""
import pytest
import torch

from fpga_ai_nic_amd.ops import gemm as G
from fpga_ai_nic_amd.ops import nn as NN
from fpga_ai_nic_amd.parallel.transport import ThreadFabric

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("M,K,C,split,tile", [(1792, 4096, 1024, 2, (128, 128)), (2048, 1024, 512, 4, (128, 128)),
                                              (512, 2048, 2048, 2, (256, 256))])
@pytest.mark.parametrize("out_bf16", [True, False])
def test_softmax_over_slabs_bit_identical(M, K, C, split, tile, out_bf16):
    g = torch.Generator().manual_seed(M + C)
    x = ((torch.rand(M, K, generator=g) * 2 - 1)).to("cuda", torch.bfloat16)
    w = ((torch.rand(K, C, generator=g) * 2 - 1) * 0.05).to("cuda", torch.bfloat16)
    b = ((torch.rand(C, generator=g) * 2 - 1) * 0.1).to("cuda", torch.bfloat16)
    y = torch.randint(0, C, (M,), generator=g, dtype=torch.int32).cuda()
    dt = torch.bfloat16 if out_bf16 else torch.float32
    # reference: the GEMM with its slab reduce, then the softmax over the logits
    lg_ref = torch.empty(M, C, device="cuda")
    G.gemm(x, False, w, False, lg_ref, G.EPI_BIAS, bias=b, split_k=split, tile=tile)
    dz_ref = torch.empty(M, C, device="cuda", dtype=dt)
    loss_ref = torch.empty(M, device="cuda")
    NN.softmax_xent(lg_ref, y, dz_ref, loss_ref, 1.0 / M)
    # folded
    slabs = {}
    lg = torch.full((M, C), float("nan"), device="cuda")
    G.gemm(x, False, w, False, lg, G.EPI_BIAS, bias=b, split_k=split, tile=tile, defer_reduce=slabs)
    assert slabs.get("sk") == split, "the split plan leaves its slabs"
    dz = torch.empty(M, C, device="cuda", dtype=dt)
    loss = torch.empty(M, device="cuda")
    NN.softmax_xent_slabs(slabs, b, lg, y, dz, loss, 1.0 / M)
    torch.cuda.synchronize()
    assert torch.equal(lg, lg_ref)
    assert torch.equal(loss, loss_ref)
    assert torch.equal(dz, dz_ref)


def test_unsplit_plan_writes_logits():
    x = torch.randn(512, 1024, device="cuda").to(torch.bfloat16)
    w = (torch.randn(1024, 1024, device="cuda") * 0.02).to(torch.bfloat16)
    b = torch.zeros(1024, device="cuda", dtype=torch.bfloat16)
    lg = torch.empty(512, 1024, device="cuda")
    slabs = {}
    G.gemm(x, False, w, False, lg, G.EPI_BIAS, bias=b, split_k=1, tile=(256, 256), defer_reduce=slabs)
    torch.cuda.synchronize()
    assert not slabs, "an unsplit plan writes C itself"
    assert torch.allclose(lg, x.float() @ w.float(), atol=0.05, rtol=0.02)


@pytest.mark.parametrize("mb", [1792, 2048])
def test_trainer_fold_logits_bit_identical(mb):
    from fpga_ai_nic_amd.models.mlp import MLP
    from fpga_ai_nic_amd.parallel.dp import DataParallelTrainer, make_engine

    sizes = [1024, 4096, 4096, 1024]
    res = []
    for fold in (False, True):
        eng = make_engine(ThreadFabric(1).transport(0), "bfp", impl="native")
        m = MLP(sizes, dtype=torch.bfloat16, device="cuda", seed=3, bias=True,
                pad_fn=lambda n, e=eng: e.layout(n).n_pad)
        tr = DataParallelTrainer(m, eng, lr=0.02)
        tr.fold_logits = fold
        g = torch.Generator().manual_seed(5)
        x = (torch.rand(mb, sizes[0], generator=g) * 2 - 1).to("cuda", torch.bfloat16)
        y = torch.randint(0, sizes[-1], (mb,), generator=g, dtype=torch.int32).cuda()
        losses = [tr.step(x, y).float().mean().item() for _ in range(4)]
        tr.finish()
        res.append((losses, m.logits.cpu(), [(l.master.cpu(), l.lp.cpu()) for l in m.layers]))
    assert res[0][0] == res[1][0], "losses differ"
    assert torch.equal(res[0][1], res[1][1]), "logits differ"
    for a, b in zip(res[0][2], res[1][2]):
        assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
