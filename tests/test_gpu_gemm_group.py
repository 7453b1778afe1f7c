"""Grouped GEMM launches and tensors inside a multi-tensor gradient bucket.

* ``gemm_wgrad_group``: up to 8 bwd-weight GEMMs in ONE dispatch (csrc/gemm/gemm_group.hip) against fp32 torch, and
  its wire epilogue against the oracle's encode of its own f32 result;
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


def _wgrad_problems(shapes, T, seed):
    torch.manual_seed(seed)
    out = []
    for fin, fout in shapes:
        X = (torch.rand(T, fin, device="cuda") * 2 - 1).to(torch.bfloat16)
        dY = ((torch.rand(T, fout, device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16)
        out.append((X, dY))
    return out


@pytest.mark.parametrize("shapes,T", [([(768, 2304), (768, 768), (768, 3072), (3072, 768)], 1024),
                                      ([(256, 128)], 512), ([(512, 384), (256, 256), (1024, 128)], 2048)])
def test_wgrad_group_matches_fp32(shapes, T):
    """The grouped bwd-weight launch (a transformer layer's projections in one dispatch): every dW and its fused
    bias gradient against fp32 torch."""
    probs = _wgrad_problems(shapes, T, T + len(shapes))
    assert G.wgrad_group_supported(probs)
    outs = [(torch.full((x.shape[1], y.shape[1]), 7.0, device="cuda"), torch.full((y.shape[1],), 7.0, device="cuda"))
            for x, y in probs]
    G.gemm_wgrad_group([(x, y, c, b) for (x, y), (c, b) in zip(probs, outs)])
    torch.cuda.synchronize()
    for (x, y), (c, b) in zip(probs, outs):
        rw = x.float().t() @ y.float()
        rb = y.float().sum(0)
        assert (c - rw).abs().max() <= 1e-3 * rw.abs().max() + 1e-6
        assert (b - rb).abs().max() <= 1e-4 * rb.abs().max() + 1e-6


@pytest.mark.parametrize("codec", ["bfp_rne", "bfp_trunc"])
def test_wgrad_group_wire_encodes_its_f32_result(codec):
    """With the wire epilogue each problem's dW (and bias gradient, right after it) is encoded into ONE bucket at its
    flat offset, bit-exactly what the oracle packs from the same group's f32 result; bytes of the bucket outside
    the problems stay untouched."""
    T = 1024
    shapes = [(768, 2304), (768, 768), (768, 3072), (3072, 768)]
    probs = _wgrad_problems(shapes, T, 11)
    offs, o = [], 512  # a leading tensor of 512 elements, then [W_i | b_i] back to back
    for fin, fout in shapes:
        offs.append(o)
        o += fin * fout + fout
    n = o + 256  # a trailing tensor
    nsh = 3
    shard = (-(-n // nsh) + 255) // 256 * 256
    cid = wire.codec_id(codec)
    g = torch.zeros(shard * nsh, device="cuda")
    ref = [(torch.empty(fin, fout, device="cuda"), torch.empty(fout, device="cuda")) for fin, fout in shapes]
    G.gemm_wgrad_group([(x, y, c, b) for (x, y), (c, b) in zip(probs, ref)])
    buf = torch.zeros(nsh * wire.shard_bytes(codec, shard), dtype=torch.uint8, device="cuda")
    pr = []
    for (x, y), off, (fin, fout) in zip(probs, offs, shapes):
        pr.append((x, y, g[off: off + fin * fout].view(fin, fout), g[off + fin * fout: off + fin * fout + fout], off))
    G.gemm_wgrad_group(pr, wire=(buf, shard, -1, cid, 0))
    torch.cuda.synchronize()
    flat = np.zeros(shard * nsh, np.float32)
    for (c, b), off in zip(ref, offs):
        flat[off: off + c.numel()] = c.cpu().numpy().reshape(-1)
        flat[off + c.numel(): off + c.numel() + b.numel()] = b.cpu().numpy()
    exp = O.pack(flat, shard, codec)
    # outside the problems the buffer keeps its zeros (the oracle's truncating codec packs a zero group with non-zero
    # mantissa bytes: the reference's q = -128 quirk)
    sb = wire.shard_bytes(codec, shard)
    inside = np.zeros(shard * nsh, bool)
    for (fin, fout), off in zip(shapes, offs):
        inside[off: off + fin * fout + fout] = True
    for s_ in range(nsh):
        seg = inside[s_ * shard:(s_ + 1) * shard]
        exp[s_ * sb: s_ * sb + shard][~seg] = 0
        exp[s_ * sb + shard: (s_ + 1) * sb][~seg.reshape(-1, 16).any(1)] = 0
    got = buf.cpu().numpy()
    if not np.array_equal(got, exp):
        sb = wire.shard_bytes(codec, shard)
        bad = np.nonzero(got != exp)[0]
        where = []
        for i in bad[:4].tolist() + bad[-2:].tolist():
            s_, r = divmod(i, sb)
            f = s_ * shard + (r if r < shard else (r - shard) * 16)
            where.append((i, "mant" if r < shard else "exp", f, [k for k, off in enumerate(offs) if off <= f]))
        raise AssertionError(f"{bad.size} wire bytes differ: (byte, plane, flat, problems at or before) {where}")
