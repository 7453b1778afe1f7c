"""Gradient encode fused into the bwd-weight GEMM (kEpiWire) and the engine's prepacked-input path.

* the GEMM's wire output is byte-identical to packing the same GEMM's f32 output (oracle pack), for several
  shard splits and both BFP codecs; the owner shard is also written in f32;
* pack_range (bias + padding tail) matches the oracle;
* the engine with prepacked input gives the same weights as without (world 1 inline, forced 1-rank RCCL, and
  N = 3 virtual ranks on the C++ loopback fabric);
* the MLP trainer with the fused path matches the unfused trainer bit-exactly.
"""
import threading

import numpy as np
import pytest
import torch

from fpga_ai_nic_amd import _ext
from fpga_ai_nic_amd.ops import bfp_oracle as O
from fpga_ai_nic_amd.ops import gemm as G
from fpga_ai_nic_amd.ops import wire
from fpga_ai_nic_amd.parallel.native_engine import NativeAllReduce
from fpga_ai_nic_amd.parallel.transport import ThreadFabric

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("codec", ["bfp_rne", "bfp_trunc"])
@pytest.mark.parametrize("cin,cout,mb,nsh", [(1024, 4096, 512, 1), (4096, 1024, 256, 3), (512, 768, 384, 8),
                                              (256, 256, 128, 2), (1000, 2048, 672, 3), (2048, 1008, 200, 2)])
def test_gemm_wire_epilogue_matches_pack(codec, cin, cout, mb, nsh):
    torch.manual_seed(cin + nsh)
    x = (torch.randn(mb, cin, device="cuda") * 0.5).to(torch.bfloat16)
    dz = (torch.randn(mb, cout, device="cuda") * 0.1).to(torch.bfloat16)
    n = cin * cout + cout
    shard = (n + nsh - 1) // nsh
    shard = (shard + 255) // 256 * 256
    own = nsh // 2
    ref = torch.empty(cin, cout, device="cuda")
    G.gemm(x, True, dz, False, ref, G.EPI_NONE, split_k=1)
    gw = torch.full((shard * nsh,), 7.0, device="cuda")
    buf = torch.zeros(nsh * wire.shard_bytes(codec, shard), dtype=torch.uint8, device="cuda")
    cid = wire.codec_id(codec)
    G.linear_bwd_weight(x, dz, gw[: cin * cout].view(cin, cout), wire=(buf, shard, own, cid))
    torch.cuda.synchronize()
    flat = np.zeros(shard * nsh, np.float32)
    flat[: cin * cout] = ref.cpu().numpy().reshape(-1)
    exp = O.pack(flat, shard, codec)
    got = buf.cpu().numpy()
    sb = wire.shard_bytes(codec, shard)
    # compare only the bytes that cover W (the bias / padding tail is the engine's pack_range job)
    for s in range(nsh):
        lo, hi = s * shard, min((s + 1) * shard, cin * cout)
        if hi <= lo:
            continue
        m_lo, m_hi = s * sb, s * sb + (hi - lo)
        assert np.array_equal(got[m_lo:m_hi], exp[m_lo:m_hi]), f"shard {s}: mantissas differ"
        e_lo = s * sb + shard
        assert np.array_equal(got[e_lo:e_lo + (hi - lo) // 16], exp[e_lo:e_lo + (hi - lo) // 16]), "exponents"
    # owner shard in f32, the rest untouched
    gw_h = gw.cpu()
    lo, hi = own * shard, min((own + 1) * shard, cin * cout)
    assert torch.equal(gw_h[lo:hi], ref.cpu().reshape(-1)[lo:hi])
    others = torch.ones(cin * cout, dtype=torch.bool)
    others[lo:hi] = False
    assert torch.all(gw_h[: cin * cout][others] == 7.0)


@pytest.mark.parametrize("codec", ["bfp_rne", "bfp_trunc"])
def test_pack_range_matches_oracle(C, codec):
    shard, nsh = 1024, 3
    x = torch.randn(shard * nsh, device="cuda")
    buf = torch.zeros(nsh * wire.shard_bytes(codec, shard), dtype=torch.uint8, device="cuda")
    begin, end = 1600, shard * nsh  # mid-shard start, covers the tail of shard 1 and all of shard 2
    C.wire_pack_range(x, buf, shard, begin, end, wire.codec_id(codec))
    exp = O.pack(x.cpu().numpy(), shard, codec)
    got = buf.cpu().numpy()
    sb = wire.shard_bytes(codec, shard)
    assert np.array_equal(got[sb + (begin - shard):sb + shard], exp[sb + (begin - shard):sb + shard])
    assert np.array_equal(got[2 * sb:], exp[2 * sb:])
    assert np.all(got[:sb] == 0)  # untouched shard 0


class _Store(dict):
    def set(self, k, v):
        self[k] = v

    def get(self, k):
        return self[k]


_NT = {}


def _native_transport():  # one 1-rank RCCL communicator for the module
    from fpga_ai_nic_amd.parallel.transport import NativeTransport

    if "t" not in _NT:
        _NT["t"] = NativeTransport(rank=0, world=1, device=0, store=_Store(), force_collectives=True)
    return _NT["t"]


def _engine_case(N, prepack, force=False, n=20000, codec="bfp_rne", algo="mesh", rings=1):
    C = _ext.require()
    rng = np.random.default_rng(3)
    grads = [rng.standard_normal(n).astype(np.float32) for _ in range(N)]
    w0 = rng.standard_normal(n).astype(np.float32)
    kw = dict(codec=codec, algo=algo, rings=rings, max_slice_elems=2048)
    if N > 1:
        fabric = C.LoopbackFabric(N, 60.0)
        engines = [NativeAllReduce(None, comm=fabric.comm(r), **kw) for r in range(N)]
    else:
        if force:
            engines = [NativeAllReduce(_native_transport(), force_comm=True, **kw)]
        else:
            engines = [NativeAllReduce(ThreadFabric(1).transport(0), **kw)]
    L = engines[0].layout(n)
    w_elems = (n // 2) // 16 * 16  # pretend the producer encoded the first half

    def fn(r):
        eng = engines[r]
        g = torch.zeros(L.n_pad, device="cuda")
        g[:n] = torch.from_numpy(grads[r])
        w = torch.zeros(L.n_pad, device="cuda")
        w[:n] = torch.from_numpy(w0)
        kw = {}
        if prepack:
            buf, shard, own, cid = eng.prepack_target(g, n)[:4]
            full = torch.zeros(L.n_pad, device="cuda")
            full[:n] = g[:n]
            _ext.require().wire_pack_range(full, buf, shard, 0, w_elems, cid)  # the "producer"
            if own == -2:  # ring: every local slice is read in f32 too (each hop adds the local contribution)
                pass
            elif own >= 0:  # the owner shard must be in f32 in grad (already true here); poison the rest
                keep = g[own * shard:(own + 1) * shard].clone()
                g[:w_elems] = float("nan")
                g[own * shard:(own + 1) * shard] = keep
            else:
                g[:w_elems] = float("nan")  # nothing but the wire may be read
            kw["prepacked"] = (buf, w_elems)
        torch.cuda.synchronize()
        h = eng.allreduce_sgd(g, w, n_valid=n, lr=0.5, defer=True, **kw)
        h.commit_after_current()
        h.synchronize(60)
        torch.cuda.synchronize()
        return w.cpu()

    if N == 1:
        return [fn(0)]
    out, errs = [None] * N, [None] * N

    def run(r):
        try:
            out[r] = fn(r)
        except Exception as e:  # noqa: BLE001
            errs[r] = e

    ts = [threading.Thread(target=run, args=(r,)) for r in range(N)]
    [t.start() for t in ts]
    [t.join(120) for t in ts]
    for e in errs:
        if e is not None:
            raise e
    return out


@pytest.mark.parametrize("N,force", [(1, False), (1, True), (3, False), (8, False)])
@pytest.mark.parametrize("codec", ["bfp_rne", "bfp_trunc"])
def test_engine_prepacked_equals_unpacked(N, force, codec):
    a = _engine_case(N, False, force, codec=codec)
    b = _engine_case(N, True, force, codec=codec)
    for x, y in zip(a, b):
        assert torch.equal(x, y)


@pytest.mark.parametrize("N,force,rings", [(1, True, 1), (3, False, 1), (3, False, 2), (8, False, 1), (8, False, 7)])
def test_ring_prepacked_equals_unpacked(N, force, rings):
    """The ring takes GEMM-encoded input too: each SEND_LOCAL hop sends the producer's encoding of the slice
    instead of re-encoding it; the sums (and the trained weights) are bit-identical."""
    a = _engine_case(N, False, force, algo="ring", rings=rings)
    b = _engine_case(N, True, force, algo="ring", rings=rings)
    for x, y in zip(a, b):
        assert torch.equal(x, y)


def test_trainer_fused_encode_matches_unfused():
    from fpga_ai_nic_amd.models.mlp import MLP
    from fpga_ai_nic_amd.parallel.dp import DataParallelTrainer, make_engine

    res = []
    for prepack in (False, True):
        eng = make_engine(ThreadFabric(1).transport(0), "bfp", impl="native")
        m = MLP([512, 1024, 512, 256], dtype=torch.bfloat16, device="cuda", seed=4, momentum=True,
                pad_fn=lambda n, e=eng: e.layout(n).n_pad)
        tr = DataParallelTrainer(m, eng, lr=0.05, momentum=0.9, prepack=prepack)
        assert tr.prepack == prepack
        g = torch.Generator().manual_seed(1)
        x = (torch.rand(256, 512, generator=g) * 2 - 1).to("cuda", torch.bfloat16)
        y = torch.randint(0, 256, (256,), generator=g, dtype=torch.int32).cuda()
        losses = [tr.step(x, y).float().mean().item() for _ in range(4)]
        tr.finish()
        res.append((losses, [l.master.cpu() for l in m.layers]))
    assert res[0][0] == res[1][0]
    assert all(torch.equal(a, b) for a, b in zip(res[0][1], res[1][1]))


@pytest.mark.parametrize("codec", ["bfp_rne", "bfp_trunc"])
@pytest.mark.parametrize("nsh", [1, 3])
def test_gemm_wire_epilogue_encodes_fused_bias(codec, nsh):
    cin, cout, mb = 1024, 1024, 256
    torch.manual_seed(nsh)
    x = (torch.randn(mb, cin, device="cuda") * 0.5).to(torch.bfloat16)
    dz = (torch.randn(mb, cout, device="cuda") * 0.1).to(torch.bfloat16)
    n = cin * cout + cout
    shard = ((n + nsh - 1) // nsh + 255) // 256 * 256
    grad = torch.zeros(shard * nsh, device="cuda")
    buf = torch.zeros(nsh * wire.shard_bytes(codec, shard), dtype=torch.uint8, device="cuda")
    G.linear_bwd_weight(x, dz, grad[: cin * cout].view(cin, cout), bias_grad=grad[cin * cout:n],
                        wire=(buf, shard, nsh - 1, wire.codec_id(codec)))
    torch.cuda.synchronize()
    flat = np.zeros(shard * nsh, np.float32)
    ref = torch.empty(cin, cout, device="cuda")
    G.gemm(x, True, dz, False, ref, G.EPI_NONE, split_k=1)
    flat[: cin * cout] = ref.cpu().numpy().reshape(-1)
    flat[cin * cout:n] = grad[cin * cout:n].cpu().numpy()  # the fused column sums (f32, always written)
    exp = O.pack(flat, shard, codec)
    got = buf.cpu().numpy()
    sb = wire.shard_bytes(codec, shard)
    for s in range(nsh):
        lo, hi = s * shard, min((s + 1) * shard, n)
        if hi <= lo:
            continue
        assert np.array_equal(got[s * sb:s * sb + hi - lo], exp[s * sb:s * sb + hi - lo]), f"shard {s} mantissas"
        e0 = s * sb + shard
        assert np.array_equal(got[e0:e0 + (hi - lo) // 16], exp[e0:e0 + (hi - lo) // 16]), f"shard {s} exponents"


@pytest.mark.parametrize("codec", ["bfp_rne", "bfp_trunc"])
@pytest.mark.parametrize("sk,tile", [(2, None), (4, (256, 256)), (2, (256, 256)), (1, (256, 256)), (1, (256, 128)),
                                     (2, (256, 128))])
def test_gemm_wire_epilogue_splitk(codec, sk, tile):
    """Split-K bwd-weight with the wire epilogue: the slab reduce encodes W and the fused bias gradient. Byte-
    identical to packing the same split GEMM's f32 output (slabs summed in the same order)."""
    cin, cout, mb, nsh = 1024, 1024, 1024, 3
    torch.manual_seed(sk)
    x = (torch.randn(mb, cin, device="cuda") * 0.5).to(torch.bfloat16)
    dz = (torch.randn(mb, cout, device="cuda") * 0.1).to(torch.bfloat16)
    n = cin * cout + cout
    shard = ((n + nsh - 1) // nsh + 255) // 256 * 256
    own = 1
    grad = torch.full((shard * nsh,), 7.0, device="cuda")
    buf = torch.zeros(nsh * wire.shard_bytes(codec, shard), dtype=torch.uint8, device="cuda")
    G.gemm(x, True, dz, False, grad[: cin * cout].view(cin, cout), G.EPI_WIRE, colsum=grad[cin * cout:n],
           wire=(buf, shard, own, wire.codec_id(codec)), split_k=sk, tile=tile)
    ref = torch.empty(cin, cout, device="cuda")
    G.gemm(x, True, dz, False, ref, G.EPI_NONE, split_k=sk, tile=tile)
    torch.cuda.synchronize()
    db = grad[cin * cout:n].cpu()
    assert (db - dz.float().sum(0).cpu()).abs().max().item() < 1e-2 * mb ** 0.5
    flat = np.zeros(shard * nsh, np.float32)
    flat[: cin * cout] = ref.cpu().numpy().reshape(-1)
    flat[cin * cout:n] = db.numpy()
    exp = O.pack(flat, shard, codec)
    got = buf.cpu().numpy()
    sb = wire.shard_bytes(codec, shard)
    for s in range(nsh):
        lo, hi = s * shard, min((s + 1) * shard, n)
        assert np.array_equal(got[s * sb:s * sb + hi - lo], exp[s * sb:s * sb + hi - lo]), f"shard {s} mantissas"
        e0 = s * sb + shard
        assert np.array_equal(got[e0:e0 + (hi - lo) // 16], exp[e0:e0 + (hi - lo) // 16]), f"shard {s} exponents"
    gw = grad.cpu()
    lo, hi = own * shard, min((own + 1) * shard, cin * cout)
    assert torch.equal(gw[lo:hi], ref.cpu().reshape(-1)[lo:hi]), "owner shard f32"
    assert torch.all(gw[: lo] == 7.0) and torch.all(gw[hi: cin * cout] == 7.0), "non-owner shards untouched"
