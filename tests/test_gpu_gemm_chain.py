"""Layer-chain GEMM (csrc/gemm/gemm_chain.hip, ops/gemm.py linear_chain): the GEMMs of one MLP pass as ONE persistent
launch with row-panel hand-offs (ready counters, write-through producer stores, per-wave acquires). Same tiles and k
order as the per-GEMM launches, so every output must be the SAME BITS as the per-GEMM path:

* forward chains (bias + ReLU bf16 hidden stages, f32 logits or bf16 last stage) and backward-data chains (ReLU-mask
  bf16 stages) over several depths and batch sizes, including one row panel per workgroup group;
* repeated launches on one counter block (the last workgroup must leave it zeroed: a stale count would release a
  consumer early) and no spin gave up (the error word stays 0);
* the chain beside a bandwidth-heavy kernel on another stream (uneven load: some workgroups start late, the queue
  must not depend on co-residency) and with its outputs pre-poisoned;
* whole training steps of the flagship MLP with the chain on and off: bit-identical weights and losses.
"""
import pytest
import torch

from fpga_ai_nic_amd.ops import gemm as G

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _chain_on(monkeypatch):
    monkeypatch.setenv("FAN_GEMM_CHAIN", "1")


def _mlp_tensors(M, sizes, seed, logits_f32=True):
    g = torch.Generator(device="cuda").manual_seed(seed)
    x = (torch.randn(M, sizes[0], device="cuda", generator=g) * 0.5).to(torch.bfloat16)
    ws = [(torch.randn(a, b, device="cuda", generator=g) * a ** -0.5).to(torch.bfloat16)
          for a, b in zip(sizes[:-1], sizes[1:])]
    bs = [(torch.randn(b, device="cuda", generator=g) * 0.1).to(torch.bfloat16) for b in sizes[1:]]
    L = len(ws)
    outs = [torch.full((M, sizes[i + 1]), 3.0, device="cuda",
                       dtype=torch.float32 if (i == L - 1 and logits_f32) else torch.bfloat16) for i in range(L)]
    epis = [G.EPI_BIAS_RELU] * (L - 1) + [G.EPI_BIAS if logits_f32 else G.EPI_BIAS_RELU]
    return x, ws, bs, outs, epis


def _fwd_reference(x, ws, bs, outs, epis):
    a = x
    ref = []
    for w, b, o, e in zip(ws, bs, outs, epis):
        r = torch.empty_like(o)
        # the chain's tiles (256x256; f32 logits 256x128) without split-K: the planner / tuner may pick a split-K plan
        # for small grids, which sums in another order
        G.gemm(a, False, w, False, r, e, bias=b, tile=(256, 128) if o.dtype == torch.float32 else (256, 256),
               split_k=1)
        ref.append(r)
        a = r
    return ref


@pytest.mark.parametrize("M,sizes,logits_f32", [
    (8192, [1024, 4096, 4096, 1024], True),   # the flagship
    (2048, [1024, 2048, 1024, 512], True),    # one row panel per group
    (4096, [512, 1024, 1024, 1024, 256], True),
    (4096, [768, 1536, 2048], False),
])
def test_forward_chain_bit_identical(M, sizes, logits_f32):
    x, ws, bs, outs, epis = _mlp_tensors(M, sizes, M + len(sizes), logits_f32)
    ref = _fwd_reference(x, ws, bs, outs, epis)
    key = ("t_fwd", M, len(sizes))
    for rep in range(3):  # repeated launches on one counter block
        for o in outs:
            o.fill_(7.0)
        assert G.linear_chain(G.CHAIN_FWD, x, ws, outs, biases=bs, epis=epis, key=key)
        torch.cuda.synchronize()
        for i, (o, r) in enumerate(zip(outs, ref)):
            assert torch.equal(o, r), f"stage {i} differs (launch {rep})"
    assert G.chain_error(key) == 0


@pytest.mark.parametrize("M,sizes", [(8192, [1024, 4096, 4096, 1024]), (2048, [512, 1024, 1024, 768]),
                                     (4096, [256, 512, 1024, 2048, 512])])
def test_backward_data_chain_bit_identical(M, sizes):
    g = torch.Generator(device="cuda").manual_seed(M + 7)
    L = len(sizes) - 1
    ws = [(torch.randn(a, b, device="cuda", generator=g) * a ** -0.5).to(torch.bfloat16)
          for a, b in zip(sizes[:-1], sizes[1:])]
    acts = [torch.randn(M, sizes[i], device="cuda", generator=g).to(torch.bfloat16) for i in range(L)]
    dz_top = (torch.randn(M, sizes[-1], device="cuda", generator=g) * 0.1).to(torch.bfloat16)
    idx = list(range(L - 1, 0, -1))
    ref, a = [], dz_top
    for i in idx:
        r = torch.empty(M, sizes[i], device="cuda", dtype=torch.bfloat16)
        G.gemm(a, False, ws[i], True, r, G.EPI_RELU_MASK, aux=acts[i], tile=(256, 256), split_k=1)
        ref.append(r)
        a = r
    outs = [torch.empty(M, sizes[i], device="cuda", dtype=torch.bfloat16) for i in idx]
    key = ("t_bwd", M, L)
    for rep in range(3):
        for o in outs:
            o.fill_(-5.0)
        assert G.linear_chain(G.CHAIN_BWD_DATA, dz_top, [ws[i] for i in idx], outs, auxes=[acts[i] for i in idx],
                              key=key)
        torch.cuda.synchronize()
        for j, (o, r) in enumerate(zip(outs, ref)):
            assert torch.equal(o, r), f"stage {j} differs (launch {rep})"
    assert G.chain_error(key) == 0


def test_chain_beside_other_streams_work():
    """Uneven load: a bandwidth-heavy copy kernel and GEMMs on other streams hold some CUs when the chain starts, so
    its workgroups start at different times (and some late); results must still be the same bits, launch after
    launch."""
    M, sizes = 8192, [1024, 4096, 4096, 1024]
    x, ws, bs, outs, epis = _mlp_tensors(M, sizes, 11)
    ref = _fwd_reference(x, ws, bs, outs, epis)
    big = torch.empty(64 << 20, device="cuda")
    dst = torch.empty_like(big)
    a = torch.randn(4096, 4096, device="cuda").to(torch.bfloat16)
    c = torch.empty(4096, 4096, device="cuda", dtype=torch.bfloat16)
    side = [torch.cuda.Stream(), torch.cuda.Stream()]
    key = ("t_load", M)
    for rep in range(6):
        for o in outs:
            o.fill_(float("nan"))
        torch.cuda.synchronize()
        with torch.cuda.stream(side[0]):
            dst.copy_(big)
            dst.copy_(big)
        with torch.cuda.stream(side[1]):
            for _ in range(rep % 3 + 1):
                G.gemm(a, False, a, False, c, G.EPI_NONE)
        assert G.linear_chain(G.CHAIN_FWD, x, ws, outs, biases=bs, epis=epis, key=key)
        torch.cuda.synchronize()
        for i, (o, r) in enumerate(zip(outs, ref)):
            assert torch.equal(o, r), f"stage {i} differs under load (launch {rep})"
    assert G.chain_error(key) == 0


def test_chain_declines_unsupported_shapes():
    x, ws, bs, outs, epis = _mlp_tensors(1024, [512, 1024, 512], 3)  # 4 row panels: fewer than one per group
    assert not G.linear_chain(G.CHAIN_FWD, x, ws, outs, biases=bs, epis=epis, key="t_no")
    x, ws, bs, outs, epis = _mlp_tensors(2048, [256, 1024, 512], 3)  # K = 256: fewer than 6 K-tiles
    assert not G.linear_chain(G.CHAIN_FWD, x, ws, outs, biases=bs, epis=epis, key="t_no")


def test_training_steps_bit_identical_with_and_without_chain(monkeypatch):
    from fpga_ai_nic_amd.models.mlp import MLP
    from fpga_ai_nic_amd.parallel.dp import DataParallelTrainer, make_engine
    from fpga_ai_nic_amd.parallel.transport import ThreadFabric

    sizes = [1024, 4096, 4096, 1024]
    torch.manual_seed(5)
    xs = [torch.randn(8192, sizes[0], device="cuda").to(torch.bfloat16) for _ in range(3)]
    ys = [torch.randint(0, sizes[-1], (8192,), device="cuda", dtype=torch.int32) for _ in range(3)]
    out = {}
    for on in ("1", "0"):
        monkeypatch.setenv("FAN_GEMM_CHAIN", on)
        eng = make_engine(ThreadFabric(1).transport(0), "bfp", impl="native")
        model = MLP(sizes, dtype=torch.bfloat16, device="cuda", pad_fn=lambda n: eng.layout(n).n_pad)
        tr = DataParallelTrainer(model, eng, lr=0.05)
        losses = []
        for x, y in zip(xs, ys):
            losses.append(tr.step(x, y).clone())
        tr.finish()
        out[on] = ([l.master.clone() for l in model.layers], losses)
    for a, b in zip(out["1"][0], out["0"][0]):
        assert torch.equal(a, b)
    for a, b in zip(out["1"][1], out["0"][1]):
        assert torch.equal(a, b)
