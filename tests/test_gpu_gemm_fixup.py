"""Split-K bwd-weight GEMMs with the wire epilogue: the tile's last workgroup reduces the f32 slabs inside the GEMM
(csrc/gemm/gemm_bf16_kernel.h split_fixup, an arrival counter per tile) instead of the separate slab-reduce kernel.
Both sum the slabs in split order, so every output must be the SAME BITS with the fixup on and off: the wire bytes,
the owner shard's f32 values, the fused bias gradient, the fused local update's master / bf16 / momentum planes —
over tile shapes, split counts, several tiles per persistent workgroup, repeated launches (the counters must be back
at zero after each), and a few flagship training steps."""
import pytest
import torch

from fpga_ai_nic_amd.ops import gemm as G
from fpga_ai_nic_amd.ops import wire

pytestmark = pytest.mark.gpu

RNE = wire.codec_id("bfp_rne")


@pytest.fixture
def C():
    from fpga_ai_nic_amd import _ext

    C = _ext.require()
    saved, persist = C.gemm_fixup(), C.gemm_persist()
    yield C
    C.gemm_set_fixup(saved)
    C.gemm_set_persist(persist)


def _wire_call(cin, cout, mb, sk, tile, codec, nsh, own, bias, seed, upd_opt=None):
    g = torch.Generator(device="cuda").manual_seed(seed)
    x = (torch.randn(mb, cin, device="cuda", generator=g) * 0.5).to(torch.bfloat16)
    dz = (torch.randn(mb, cout, device="cuda", generator=g) * 0.1).to(torch.bfloat16)
    n = cin * cout + (cout if bias else 0)
    shard = ((n + nsh - 1) // nsh + 255) // 256 * 256
    master = ((torch.rand(shard * nsh, device="cuda", generator=g) * 2 - 1) * 0.05)

    def run():
        grad = torch.full((shard * nsh,), 7.0, device="cuda")
        buf = torch.zeros(nsh * wire.shard_bytes(codec, shard), dtype=torch.uint8, device="cuda")
        out = {"grad": grad, "buf": buf}
        upd = None
        if upd_opt is not None:
            m = master.clone()
            lp = m.to(torch.bfloat16)
            mom = torch.zeros_like(m) if "momentum" in upd_opt else None
            upd = G.LocalUpdate(m, lp, mom, **upd_opt)
            out.update(master=m, lp=lp, mom=mom)
        G.gemm(x, True, dz, False, grad[: cin * cout].view(cin, cout), G.EPI_WIRE,
               colsum=grad[cin * cout:n] if bias else None, wire=(buf, shard, own, wire.codec_id(codec)),
               split_k=sk, tile=tile, update=upd)
        return out

    return run


def _same(a, b):
    for k in a:
        if a[k] is None:
            continue
        assert torch.equal(a[k], b[k]), f"{k} differs with the in-GEMM fixup"


@pytest.mark.parametrize("sk,tile", [(2, (256, 256)), (4, (256, 256)), (2, (256, 128)), (4, (256, 128)),
                                     (2, (128, 128)), (3, (256, 256))])
@pytest.mark.parametrize("bias", [True, False])
@pytest.mark.parametrize("codec", ["bfp_rne", "bfp_trunc"])
def test_fixup_wire_bit_identical(C, sk, tile, bias, codec):
    run = _wire_call(1024, 1024, 1536, sk, tile, codec, nsh=3, own=1, bias=bias, seed=sk * 7 + bias)
    C.gemm_set_fixup(0)
    ref = run()
    C.gemm_set_fixup(1)
    for _ in range(3):  # repeated launches: every tile counter is back at zero after each
        _same(ref, run())
    torch.cuda.synchronize()


@pytest.mark.parametrize("opt", [dict(lr=0.05), dict(lr=0.02, momentum=0.9, weight_decay=1e-3)])
@pytest.mark.parametrize("bias", [True, False])
def test_fixup_fused_update_bit_identical(C, opt, bias):
    """The flagship's 1024x4096 bwd-weight (K = 8192, 256x256 tiles split 4 ways) with the update fused."""
    run = _wire_call(1024, 4096, 8192, 4, (256, 256), "bfp_rne", nsh=1, own=-1, bias=bias, seed=11, upd_opt=opt)
    C.gemm_set_fixup(0)
    ref = run()
    C.gemm_set_fixup(1)
    _same(ref, run())


def test_fixup_several_tiles_per_workgroup(C):
    """Persistent workgroups that each take several (tile, split) items (grid capped at 8 workgroups)."""
    run = _wire_call(1024, 2048, 2048, 2, (256, 256), "bfp_rne", nsh=2, own=0, bias=False, seed=5)
    C.gemm_set_fixup(0)
    ref = run()
    C.gemm_set_fixup(1)
    C.gemm_set_persist(8)
    _same(ref, run())
    _same(ref, run())


def test_fixup_training_bit_identical(C):
    """The flagship step (update fused into the bwd-weight epilogue; its 1024-wide layers split 4 ways) trains to
    the same bits with the in-GEMM fixup and with the slab-reduce kernel."""
    from fpga_ai_nic_amd.models.mlp import MLP
    from fpga_ai_nic_amd.ops import gemm_tune
    from fpga_ai_nic_amd.parallel.dp import DataParallelTrainer, make_engine
    from fpga_ai_nic_amd.parallel.transport import ThreadFabric

    sizes = [1024, 4096, 4096, 1024]
    g = torch.Generator().manual_seed(3)
    x = (torch.rand(8192, sizes[0], generator=g) * 2 - 1).to("cuda", torch.bfloat16)
    y = torch.randint(0, sizes[-1], (8192,), generator=g, dtype=torch.int32).cuda()
    weights = []
    gemm_tune.reset(enabled=False)
    try:
        for fix in (0, 1):
            C.gemm_set_fixup(fix)
            eng = make_engine(ThreadFabric(1).transport(0), "bfp", rounding="rne", impl="native")
            m = MLP(sizes, dtype=torch.bfloat16, device="cuda", seed=9, pad_fn=lambda n: eng.layout(n).n_pad)
            tr = DataParallelTrainer(m, eng, lr=0.05)
            for _ in range(3):
                tr.step(x, y)
            tr.finish()
            torch.cuda.synchronize()
            weights.append([l.master.clone() for l in m.layers])
    finally:
        gemm_tune.reset()
    for a, b in zip(*weights):
        assert torch.equal(a, b)


@pytest.fixture
def R4():
    from fpga_ai_nic_amd import _ext

    C = _ext.require()
    saved, fix = C.gemm_reduce4(), C.gemm_fixup()
    C.gemm_set_fixup(0)
    yield C
    C.gemm_set_reduce4(saved)
    C.gemm_set_fixup(fix)


@pytest.mark.parametrize("sk,tile", [(2, (256, 256)), (4, (256, 256)), (3, (256, 256)), (4, (256, 128))])
@pytest.mark.parametrize("bias", [True, False])
@pytest.mark.parametrize("codec,own", [("bfp_rne", 1), ("bfp_trunc", 0), ("bfp_rne", -2)])
def test_reduce4_wire_bit_identical(R4, sk, tile, bias, codec, own):
    """The lane-contiguous split-K reduce (4 values per lane, the group exponent from quad shuffles;
    FAN_GEMM_REDUCE4 / gemm_set_reduce4) against the one-group-per-lane kernel: the same bits in every output
    (own -2: every shard's f32 copy)."""
    run = _wire_call(1024, 1024, 1536, sk, tile, codec, nsh=3, own=own, bias=bias, seed=sk * 5 + bias)
    R4.gemm_set_reduce4(0)
    ref = run()
    R4.gemm_set_reduce4(1)
    _same(ref, run())


@pytest.mark.parametrize("opt", [dict(lr=0.05), dict(lr=0.02, momentum=0.9, weight_decay=1e-3),
                                 dict(lr=0.02, momentum=0.9, nesterov=True)])
@pytest.mark.parametrize("bias", [True, False])
def test_reduce4_fused_update_bit_identical(R4, opt, bias):
    """The flagship's 1024x4096 bwd-weight with the update fused into the reduce."""
    run = _wire_call(1024, 4096, 8192, 4, (256, 256), "bfp_rne", nsh=1, own=-1, bias=bias, seed=13, upd_opt=opt)
    R4.gemm_set_reduce4(0)
    ref = run()
    R4.gemm_set_reduce4(1)
    _same(ref, run())
