"""GPU numerics of every hand-written HIP kernel against the NumPy oracle / a plain fp32 PyTorch reference."""
import numpy as np
import pytest
import torch

from fpga_ai_nic_amd.ops import bfp_oracle as O
from fpga_ai_nic_amd.ops import gemm as G
from fpga_ai_nic_amd.ops import nn as NN
from fpga_ai_nic_amd.ops import wire

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _special_vector(n, seed=0):
    rng = np.random.default_rng(seed)
    x = (rng.standard_normal(n) * np.exp2(rng.integers(-30, 30, n))).astype(np.float32)
    x[:16] = 0.0                                        # all-zero group
    x[16:32] = np.float32(1e-40)                        # denormals
    x[32:48] = rng.standard_normal(16).astype(np.float32)
    x[40] = np.float32(3e38)                            # huge max -> others flush
    x[48:64] = -np.float32(1.0)                         # -1 exact: trunc gives -128 edge
    x[64:80] = np.float32(2.0) ** -126
    x[80:96] = np.linspace(-1, 1, 16, dtype=np.float32) * 2.0 ** 100
    return x


@pytest.mark.parametrize("codec", ["bfp_trunc", "bfp_rne", "raw_f32", "raw_bf16"])
@pytest.mark.parametrize("in_dtype", [torch.float32, torch.bfloat16])
def test_pack_unpack_bitexact(C, codec, in_dtype):
    n_s, shards = 4096, 3
    x = _special_vector(n_s * shards)
    xt = torch.from_numpy(x).to(in_dtype)
    xin = xt.float().numpy()  # what the kernel sees (bf16-rounded when bf16)
    sb = O.shard_bytes(codec, n_s)
    out = torch.zeros(sb * shards, dtype=torch.uint8, device=DEV)
    wire.pack(xt.to(DEV), out, n_s, codec)
    ref = O.pack(xin, n_s, codec)
    assert np.array_equal(out.cpu().numpy(), ref), f"pack mismatch for {codec}"
    for od in (torch.float32, torch.bfloat16):
        dec = torch.empty(n_s * shards, dtype=od, device=DEV)
        wire.unpack(out, dec, n_s, codec)
        r = O.unpack(ref, n_s * shards, n_s, codec)
        if od == torch.bfloat16:
            r = O.bf16_bits_to_f32(O.f32_to_bf16_bits(r))
        got = dec.float().cpu().numpy()
        assert np.array_equal(got.view(np.uint32), r.view(np.uint32)) or np.array_equal(
            np.nan_to_num(got), np.nan_to_num(r)), f"unpack mismatch {codec} {od}"


def test_pack_random_large(C):
    n_s = 1 << 20
    x = torch.randn(n_s * 2, device=DEV) * 1e-3
    out = torch.empty(O.shard_bytes("bfp_rne", n_s) * 2, dtype=torch.uint8, device=DEV)
    wire.pack(x, out, n_s, "bfp_rne")
    assert np.array_equal(out.cpu().numpy(), O.pack(x.cpu().numpy(), n_s, "bfp_rne"))


@pytest.mark.parametrize("codec", ["bfp_trunc", "bfp_rne", "raw_f32", "raw_bf16"])
@pytest.mark.parametrize("local_dtype", [torch.float32, torch.bfloat16])
def test_reduce_bitexact(C, codec, local_dtype):
    n_s, N, me = 2048, 5, 2
    rng = np.random.default_rng(1)
    parts = [rng.standard_normal(n_s).astype(np.float32) * (r + 1) for r in range(N)]
    slots = np.concatenate([O.pack(p, n_s, codec) for p in parts])
    local = torch.from_numpy(parts[me]).to(local_dtype)
    sb = O.shard_bytes(codec, n_s)
    ow = torch.zeros(sb, dtype=torch.uint8, device=DEV)
    of = torch.zeros(n_s, dtype=torch.float32, device=DEV)
    wire.reduce(torch.from_numpy(slots).to(DEV), N, me, local.to(DEV), ow, of, n_s, codec)
    acc = O.reduce_slots([slots[r * sb:(r + 1) * sb] for r in range(N)], local.float().numpy(), me, codec, n_s)
    assert np.array_equal(of.cpu().numpy(), acc)
    assert np.array_equal(ow.cpu().numpy(), O.pack(acc, n_s, codec))


@pytest.mark.parametrize("codec", ["bfp_trunc", "bfp_rne", "raw_f32"])
@pytest.mark.parametrize("momentum", [0.0, 0.9])
def test_sgd_epilogue(C, codec, momentum):
    n_s, N = 1024, 4
    n_valid = n_s * N - 77
    rng = np.random.default_rng(2)
    g = rng.standard_normal(n_s * N).astype(np.float32)
    w = rng.standard_normal(n_s * N).astype(np.float32)
    m = rng.standard_normal(n_s * N).astype(np.float32) if momentum else None
    buf = O.pack(g, n_s, codec)
    wt = torch.from_numpy(w.copy()).to(DEV)
    lp = torch.zeros(n_s * N, dtype=torch.bfloat16, device=DEV)
    mt = torch.from_numpy(m.copy()).to(DEV) if momentum else None
    wire.sgd(torch.from_numpy(buf).to(DEV), n_s, N, wt, codec=codec, lp=lp, mom=mt, lr=0.1, grad_scale=0.25,
             weight_decay=1e-4, momentum=momentum, n_valid=n_valid, skip_shard=1, skip_period=N)
    gd = O.unpack(buf, n_s * N, n_s, codec)
    ref_w = w.copy()
    for s in range(N):
        if s == 1:
            continue
        lo, hi = s * n_s, min((s + 1) * n_s, n_valid)
        nw, _ = O.sgd(w[lo:hi], gd[lo:hi], 0.1, 0.25, 1e-4, momentum, None if m is None else m[lo:hi])
        ref_w[lo:hi] = nw
    got = wt.cpu().numpy()
    # fma emulated in float64 (double rounding is possible but vanishingly rare): allow 1 ulp
    ulp = np.abs(got.view(np.int32).astype(np.int64) - ref_w.view(np.int32).astype(np.int64))
    assert ulp.max() <= 1
    assert np.array_equal(got[n_valid:], w[n_valid:]), "padding must not be touched"
    assert np.array_equal(got[n_s:2 * n_s], w[n_s:2 * n_s]), "skipped shard must not be touched"
    assert torch.equal(lp[:n_s].float().cpu(), wt[:n_s].to(torch.bfloat16).float().cpu())


def _ref_mm(a, b):
    return a.double() @ b.double()


def _elem_bound(a, b):
    """Per-element error bound of an f32-accumulated product of (already rounded) operands: 2e-5 * sum_k |a b|
    (covers f32 summation with a wide margin at these K; a misplaced product breaks it by orders of magnitude)."""
    return 2e-5 * (a.double().abs() @ b.double().abs()) + 1e-6


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("M,N,K", [(256, 384, 512), (2048, 1024, 4096), (512, 4096, 1024)])
def test_gemm_layouts_vs_fp32(C, dt, M, N, K):
    torch.manual_seed(0)
    A = torch.randn(M, K, device=DEV).to(dt)
    Bkn = torch.randn(K, N, device=DEV).to(dt)
    ref = _ref_mm(A.float(), Bkn.float())
    bound = _elem_bound(A.float(), Bkn.float())
    for a_t in (False, True):
        for b_t in (False, True):
            Ain = A.t().contiguous() if a_t else A
            Bin = Bkn.t().contiguous() if b_t else Bkn
            Cout = torch.empty(M, N, device=DEV, dtype=torch.float32)
            G.gemm(Ain, a_t, Bin, b_t, Cout, split_k=1)
            err = (Cout.double() - ref).abs()
            assert bool((err <= bound).all()), f"layout a_t={a_t} b_t={b_t}: max err {err.max().item()}"


def test_gemm_asymmetric_identity(C):
    # A = I with an asymmetric B catches C-write transposes (guide: "always A=I-check with asymmetric B")
    n = 256
    A = torch.eye(n, device=DEV).to(torch.bfloat16)
    B = (torch.arange(n * n, device=DEV).float().view(n, n) % 97).to(torch.bfloat16)
    Cout = torch.empty(n, n, device=DEV)
    G.gemm(A, False, B, False, Cout)
    assert torch.equal(Cout, B.float())


def test_gemm_epilogues_and_splitk(C):
    torch.manual_seed(1)
    M, N, K = 512, 256, 2048
    X = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    W = (torch.randn(K, N, device=DEV) / K ** 0.5).to(torch.bfloat16)
    b = torch.randn(N, device=DEV).to(torch.bfloat16)
    ref = (X.float() @ W.float() + b.float())
    for sk in (1, 2, 4):
        Y = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        G.gemm(X, False, W, False, Y, G.EPI_BIAS_RELU, bias=b, split_k=sk)
        assert (Y.float() - torch.relu(ref)).abs().max().item() < 5e-2
    # ReLU-mask epilogue (bwd-data) with bf16 aux
    dZ = torch.randn(M, N, device=DEV).to(torch.bfloat16)
    act = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    dX = torch.empty(M, K, device=DEV, dtype=torch.bfloat16)
    G.linear_bwd_data(dZ, W, dX, relu_input=act)
    r = (dZ.float() @ W.float().t()) * (act.float() > 0)
    assert (dX.float() - r).abs().max().item() < 5e-2
    # accumulate into f32
    dW = torch.ones(K, N, device=DEV)
    G.linear_bwd_weight(act, dZ, dW, accumulate=True)
    r = act.float().t() @ dZ.float() + 1.0
    assert (dW - r).abs().max().item() < 2e-1


@pytest.mark.parametrize("in_dt,out_dt", [(torch.float32, torch.bfloat16), (torch.float32, torch.float32),
                                          (torch.bfloat16, torch.bfloat16)])
@pytest.mark.parametrize("Cc", [1024, 8, 1544, 2048, 4096])
def test_softmax_xent(C, in_dt, out_dt, Cc):
    """Register-resident rows (C <= 2048, C % 8 == 0; partial last chunk at 1544) and the streaming kernel."""
    torch.manual_seed(2)
    M = 300
    x = (torch.randn(M, Cc, device=DEV) * 3).to(in_dt)
    y = torch.randint(0, Cc, (M,), device=DEV, dtype=torch.int32)
    d = torch.empty(M, Cc, device=DEV, dtype=out_dt)
    loss = torch.empty(M, device=DEV)
    NN.softmax_xent(x, y, d, loss, 0.5)
    xf = x.float()
    ref_loss = torch.nn.functional.cross_entropy(xf, y.long(), reduction="none")
    assert (loss - ref_loss).abs().max().item() < 1e-3
    p = torch.softmax(xf, 1)
    p[torch.arange(M), y.long()] -= 1
    assert (d.float() - p * 0.5).abs().max().item() < 1e-2


def test_col_sum(C):
    torch.manual_seed(3)
    x = torch.randn(1000, 640, device=DEV).to(torch.bfloat16)
    out = torch.zeros(640, device=DEV)
    NN.col_sum(x, out, 2.0)
    assert (out - x.float().sum(0) * 2).abs().max().item() < 1e-2


@pytest.mark.parametrize("M,N,K,sk,tile", [(1024, 4096, 2048, None, None), (4096, 1024, 2048, None, None),
                                            (4096, 4096, 2048, None, None), (512, 384, 256, None, None),
                                            (1024, 4096, 8192, None, None), (1024, 1024, 2048, 4, (256, 256)),
                                            (512, 768, 1024, 2, None)])
def test_gemm_fused_bias_grad(C, M, N, K, sk, tile):
    """bwd-weight GEMM with the bias gradient (column sums of dZ) fused: both outputs vs fp32 references.
    With split-K (auto at 1024x4096, K 8192; forced otherwise) the per-split partial column sums are reduced
    after the slabs."""
    torch.manual_seed(5)
    X = torch.randn(K, M, device=DEV).to(torch.bfloat16)   # activations [batch][in]
    dZ = torch.randn(K, N, device=DEV).to(torch.bfloat16)  # upstream grad [batch][out]
    dW = torch.empty(M, N, device=DEV)
    db = torch.full((N,), float("nan"), device=DEV)
    G.gemm(X, True, dZ, False, dW, G.EPI_NONE, colsum=db, split_k=sk, tile=tile)
    assert (dW - X.float().t() @ dZ.float()).abs().max().item() < 0.25
    assert (db - dZ.float().sum(0)).abs().max().item() < 1e-2 * K ** 0.5


@pytest.fixture(params=[0, 2, 3, 5], ids=["oneloop", "pipelined", "pipelined4", "pipelined8"])
def main_loop(request, C):
    """Every 256x256 main loop: one-role, software-pipelined by layout, 4-wave and 8-wave (gemm_set_main_loop)."""
    Cx = G._ext.require()
    mode0 = Cx.gemm_main_loop()
    Cx.gemm_set_main_loop(request.param)
    yield request.param
    Cx.gemm_set_main_loop(mode0)


@pytest.mark.parametrize("K", [64, 128, 192, 1024, 4096])
def test_gemm_256_tile_all_layouts_and_k(C, main_loop, K):
    """The 256x256 main loops (forced tile) on all four operand layouts, K-tile counts 1, 2, 3 and
    long loops, with and without split-K: vs an fp64 reference."""
    torch.manual_seed(K)
    M, N = 512, 768
    A = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    Bkn = torch.randn(K, N, device=DEV).to(torch.bfloat16)
    ref = _ref_mm(A.float(), Bkn.float())
    bound = _elem_bound(A.float(), Bkn.float())
    for a_t in (False, True):
        for b_t in (False, True):
            Ain = A.t().contiguous() if a_t else A
            Bin = Bkn.t().contiguous() if b_t else Bkn
            for sk in (1, 2) if K % 128 == 0 else (1,):
                Cout = torch.full((M, N), float("nan"), device=DEV)
                G.gemm(Ain, a_t, Bin, b_t, Cout, split_k=sk, tile=(256, 256))
                err = (Cout.double() - ref).abs()
                assert bool((err <= bound).all()), f"a_t={a_t} b_t={b_t} split_k={sk}: max err {err.max().item()}"


@pytest.mark.parametrize("K", [64, 192, 2048])
def test_gemm_256x128_tile_all_layouts(C, main_loop, K):
    """256x128 tiles (the 4-wave pipelined loop with 128x64 per wave under the default selection) on all four
    operand layouts, with and without split-K and the fused bias gradient: vs an fp64 reference."""
    torch.manual_seed(K + 1)
    M, N = 512, 384
    A = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    Bkn = torch.randn(K, N, device=DEV).to(torch.bfloat16)
    ref = _ref_mm(A.float(), Bkn.float())
    bound = _elem_bound(A.float(), Bkn.float())
    for a_t in (False, True):
        for b_t in (False, True):
            Ain = A.t().contiguous() if a_t else A
            Bin = Bkn.t().contiguous() if b_t else Bkn
            for sk in (1, 3) if K % 192 == 0 else (1,):
                Cout = torch.full((M, N), float("nan"), device=DEV)
                cs = torch.full((N,), float("nan"), device=DEV) if (a_t and not b_t) else None
                G.gemm(Ain, a_t, Bin, b_t, Cout, split_k=sk, tile=(256, 128), colsum=cs)
                err = (Cout.double() - ref).abs()
                assert bool((err <= bound).all()), f"a_t={a_t} b_t={b_t} split_k={sk}: max err {err.max().item()}"
                if cs is not None:  # column sums of B over K (the bias gradient of the bwd-weight layout)
                    assert (cs.double() - Bkn.double().sum(0)).abs().max().item() < 1e-3 * K ** 0.5


def test_gemm_256_tile_epilogues(C, main_loop):
    torch.manual_seed(9)
    M, N, K = 512, 512, 768
    X = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    W = (torch.randn(K, N, device=DEV) / K ** 0.5).to(torch.bfloat16)
    b = torch.randn(N, device=DEV).to(torch.bfloat16)
    Y = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    G.gemm(X, False, W, False, Y, G.EPI_BIAS_RELU, bias=b, split_k=1, tile=(256, 256))
    assert (Y.float() - torch.relu(X.float() @ W.float() + b.float())).abs().max().item() < 5e-2
    dZ = torch.randn(M, N, device=DEV).to(torch.bfloat16)
    act = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    dX = torch.empty(M, K, device=DEV, dtype=torch.bfloat16)
    G.gemm(dZ, False, W, True, dX, G.EPI_RELU_MASK, aux=act, split_k=1, tile=(256, 256))
    assert (dX.float() - (dZ.float() @ W.float().t()) * (act.float() > 0)).abs().max().item() < 5e-2
    dW = torch.empty(K, N, device=DEV)
    db = torch.zeros(N, device=DEV)
    G.gemm(act, True, dZ, False, dW, G.EPI_NONE, split_k=1, tile=(256, 256), colsum=db)
    assert (dW - act.float().t() @ dZ.float()).abs().max().item() < 0.25
    assert (db - dZ.float().sum(0)).abs().max().item() < 1e-2 * M ** 0.5


@pytest.fixture
def persist_cap(C):
    cap0 = C.gemm_persist()
    yield C
    C.gemm_set_persist(cap0)


@pytest.mark.parametrize("tile", [(256, 256), (256, 128)])
@pytest.mark.parametrize("cap", [3, 8])
def test_gemm_persistent_grid_bit_identical(persist_cap, tile, cap):
    """The 4-wave pipelined kernel loops over tiles when its grid is capped below the tile count: every layout /
    epilogue / split-K result is bit-identical to one workgroup per tile (grid caps 3 and 8, 16-32 tiles)."""
    C = persist_cap
    mode0 = C.gemm_main_loop()
    C.gemm_set_main_loop(3)  # 4-wave pipelined loop for the 256x256 tiles
    try:
        torch.manual_seed(11)
        M, N, K = 1024, 1024, 512
        bf = torch.bfloat16
        for a_t in (False, True):
            for b_t in (False, True):
                A = (torch.randn(K, M, device=DEV) if a_t else torch.randn(M, K, device=DEV)).to(bf)
                B = (torch.randn(N, K, device=DEV) if b_t else torch.randn(K, N, device=DEV)).to(bf)
                bias = torch.randn(N, device=DEV).to(bf)
                act = torch.randn(M, N, device=DEV).to(bf)
                cases = [(G.EPI_BIAS_RELU, bf, dict(bias=bias)), (G.EPI_RELU_MASK, bf, dict(aux=act)),
                         (G.EPI_NONE, torch.float32, dict()), (G.EPI_NONE, torch.float32, dict(split_k=2))]
                for epi, odt, kw in cases:
                    kw = dict(kw)
                    sk = kw.pop("split_k", 1)
                    outs = []
                    for c in (0, cap):
                        C.gemm_set_persist(c)
                        out = torch.full((M, N), 7.0, device=DEV, dtype=odt)
                        G.gemm(A, a_t, B, b_t, out, epi, split_k=sk, tile=tile, **kw)
                        torch.cuda.synchronize()
                        outs.append(out)
                    assert torch.equal(outs[0], outs[1]), f"a_t={a_t} b_t={b_t} epi={epi} sk={sk}: persistent differs"
                    ref = (A.double().t() if a_t else A.double()) @ (B.double().t() if b_t else B.double())
                    if epi == G.EPI_BIAS_RELU:
                        ref = torch.relu(ref + bias.double())
                    if epi == G.EPI_RELU_MASK:
                        ref = ref * (act.double() > 0)
                    assert (outs[1].double() - ref).abs().max().item() < 0.02 * (1 + ref.abs().max().item())
    finally:
        C.gemm_set_main_loop(mode0)


@pytest.mark.parametrize("M,N,K", [(1792, 512, 1024), (672, 384, 2048), (224, 128, 64)])
def test_gemm_224x128_tile(C, M, N, K):
    """224x128 tiles (M % 224 == 0: the reference's per-rank batch 1792 = 8 x 224 rows fills 256 CUs on 4096-wide
    outputs; 672 = 5376 / 8 ranks), K-contiguous A on both B layouts, with and without split-K, bias / ReLU /
    ReLU-mask epilogues, persistent grids capped below the tile count: vs an fp64 reference."""
    torch.manual_seed(M + K)
    A = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    Bkn = torch.randn(K, N, device=DEV).to(torch.bfloat16)
    ref = _ref_mm(A.float(), Bkn.float())
    bound = _elem_bound(A.float(), Bkn.float())
    assert tuple(C.gemm_plan(M, N, K, 1, 224, 128, 0))[:3] == (224, 128, 1)
    assert C.gemm_plan(M, N, K, 1, 224, 256, 0)[0] == 0  # 224 rows pair with 128 columns only
    cap0 = C.gemm_persist()
    try:
        for b_t in (False, True):
            Bin = Bkn.t().contiguous() if b_t else Bkn
            for sk in (1, 2) if K % 128 == 0 else (1,):
                for cap in (cap0, 3):
                    C.gemm_set_persist(cap)
                    Cout = torch.full((M, N), float("nan"), device=DEV)
                    G.gemm(A, False, Bin, b_t, Cout, split_k=sk, tile=(224, 128))
                    err = (Cout.double() - ref).abs()
                    assert bool((err <= bound).all()), f"b_t={b_t} split_k={sk} cap={cap}: max err {err.max().item()}"
    finally:
        C.gemm_set_persist(cap0)
    bias = torch.randn(N, device=DEV).to(torch.bfloat16)
    Y = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    G.gemm(A, False, Bkn, False, Y, G.EPI_BIAS_RELU, bias=bias, split_k=1, tile=(224, 128))
    want = torch.relu(ref + bias.double())
    assert (Y.double() - want).abs().max().item() <= (bound.max().item() + 1e-2 * want.abs().max().item())
    act = torch.randn(M, N, device=DEV).to(torch.bfloat16)
    Bnk = Bkn.t().contiguous()
    dX = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    G.gemm(A, False, Bnk, True, dX, G.EPI_RELU_MASK, aux=act, split_k=1, tile=(224, 128))
    want = ref * (act.double() > 0)
    assert (dX.double() - want).abs().max().item() <= (bound.max().item() + 1e-2 * want.abs().max().item())
    with pytest.raises(Exception):  # an MN-contiguous A has no 224-row image
        G.gemm(A.t().contiguous(), True, Bkn, False, torch.empty(M, N, device=DEV), split_k=1, tile=(224, 128))
