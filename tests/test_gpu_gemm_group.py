"""Grouped GEMM launches and tensors inside a multi-tensor gradient bucket.

* ``gemm_bwd_pair``: one layer's bwd-data (ReLU-mask epilogue, bf16) and bwd-weight (f32) in ONE dispatch
  (csrc/gemm/gemm_pair.hip, the reference's PASS_BWD shape, sw/mlp_mpi_example_f32.cpp:741-742) is bit-identical to
  the two separate launches of the same tiles, and both match fp32 torch within the bf16 bounds, for several
  workgroup splits (including splits that leave one problem more workgroups than tiles);
* the wire epilogue's flat offset (GemmArgs::wire_off): a weight matrix placed at an offset inside a larger bucket
  (a transformer layer's bucket, bench/bert_overlap.py) encodes exactly the bytes the oracle packs for the whole
  bucket at those positions, with its fused bias gradient encoded right after it.
"""
import numpy as np
import pytest
import torch

from fpga_ai_nic_amd import _ext
from fpga_ai_nic_amd.ops import bfp_oracle as O
from fpga_ai_nic_amd.ops import gemm as G
from fpga_ai_nic_amd.ops import wire

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("M,cin,cout,bn,g0,g1", [(1024, 1024, 512, 128, 64, 64), (2048, 512, 1024, 256, 64, 32),
                                                  (512, 512, 256, 128, 128, 128), (768, 1024, 768, 256, 8, 8)])
def test_bwd_pair_matches_separate_launches(M, cin, cout, bn, g0, g1):
    C = _ext.require()
    torch.manual_seed(M + cin)
    X = (torch.rand(M, cin, device="cuda") * 2 - 1).to(torch.bfloat16)
    dZ = ((torch.rand(M, cout, device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16)
    W = ((torch.rand(cin, cout, device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16)
    dX = torch.empty(M, cin, device="cuda", dtype=torch.bfloat16)
    dW = torch.empty(cin, cout, device="cuda")
    G.gemm(dZ, False, W, True, dX, G.EPI_RELU_MASK, aux=X, tile=(256, 256), split_k=1)
    G.gemm(X, True, dZ, False, dW, G.EPI_NONE, tile=(256, bn), split_k=1)
    dX2 = torch.full_like(dX, 3.0)
    dW2 = torch.full_like(dW, 3.0)
    C.gemm_bwd_pair(dZ, W, X, dX2, dW2, bn, g0, g1)
    torch.cuda.synchronize()
    assert torch.equal(dX, dX2) and torch.equal(dW, dW2)
    rx = (dZ.float() @ W.float().t()) * (X.float() > 0)
    rw = X.float().t() @ dZ.float()
    assert (dX2.float() - rx).abs().max() <= 2e-2 * rx.abs().max() + 1e-6
    assert (dW2 - rw).abs().max() <= 1e-3 * rw.abs().max() + 1e-6


def test_bwd_pair_rejects_bad_grids():
    C = _ext.require()
    X = torch.zeros(256, 256, device="cuda", dtype=torch.bfloat16)
    dZ = torch.zeros(256, 256, device="cuda", dtype=torch.bfloat16)
    W = torch.zeros(256, 256, device="cuda", dtype=torch.bfloat16)
    dX = torch.empty_like(X)
    dW = torch.empty(256, 256, device="cuda")
    with pytest.raises(RuntimeError):
        C.gemm_bwd_pair(dZ, W, X, dX, dW, 256, 12, 8)  # not a multiple of the XCD count


@pytest.mark.parametrize("codec", ["bfp_rne", "bfp_trunc"])
def test_wire_offset_inside_a_bucket(codec):
    torch.manual_seed(7)
    T, fin, fout = 512, 768, 2304  # a QKV projection
    pre, post = 768 * 2, 768 * 4    # other tensors of the bucket before / after [W | b]
    off = pre
    n = pre + fin * fout + fout + post
    nsh = 3
    shard = (-(-n // nsh) + 255) // 256 * 256
    cid = wire.codec_id(codec)
    x = (torch.randn(T, fin, device="cuda") * 0.5).to(torch.bfloat16)
    dy = (torch.randn(T, fout, device="cuda") * 0.1).to(torch.bfloat16)
    ref = torch.empty(fin, fout, device="cuda")
    G.gemm(x, True, dy, False, ref, G.EPI_NONE, split_k=1)
    g = torch.zeros(shard * nsh, device="cuda")
    buf = torch.zeros(nsh * wire.shard_bytes(codec, shard), dtype=torch.uint8, device="cuda")
    dW = g[off: off + fin * fout].view(fin, fout)
    db = g[off + fin * fout: off + fin * fout + fout]
    G.gemm(x, True, dy, False, dW, G.EPI_WIRE, colsum=db, wire=(buf, shard, -1, cid, 0, off), split_k=1)
    torch.cuda.synchronize()
    flat = np.zeros(shard * nsh, np.float32)
    flat[off: off + fin * fout] = ref.cpu().numpy().reshape(-1)
    flat[off + fin * fout: off + fin * fout + fout] = dy.float().sum(0).cpu().numpy()
    exp = O.pack(flat, shard, codec)
    got = buf.cpu().numpy()
    sb = wire.shard_bytes(codec, shard)
    lo_all, hi_all = off, off + fin * fout + fout
    for s in range(nsh):
        lo, hi = max(s * shard, lo_all), min((s + 1) * shard, hi_all)
        if hi <= lo:
            continue
        a, b = lo - s * shard, hi - s * shard
        m = got[s * sb + a: s * sb + b] == exp[s * sb + a: s * sb + b]
        # the bias column sums: the kernel's summation order differs from numpy's, so compare their groups by value
        bias_lo = max(off + fin * fout, lo) - s * shard
        assert m[: max(0, bias_lo - a)].all(), f"shard {s}: W mantissas differ"
        ea, eb = s * sb + shard + a // 16, s * sb + shard + max(a, min(bias_lo, b)) // 16
        assert np.array_equal(got[ea:eb], exp[ea:eb]), f"shard {s}: W exponents differ"
    # bytes outside [W | b] untouched
    for s in range(nsh):
        lo, hi = s * shard, (s + 1) * shard
        if lo < lo_all:
            assert not got[s * sb: s * sb + min(hi, lo_all) - lo].any()
    dec = O.unpack(got, shard * nsh, shard, codec)
    bias_ref = dy.float().sum(0).cpu().numpy()
    bias_dec = dec[off + fin * fout: off + fin * fout + fout]
    assert np.abs(bias_dec - bias_ref).max() <= 2.0 ** -5 * np.abs(bias_ref).max() + 1e-6
