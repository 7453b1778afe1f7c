"""Wire-format ops of the all-reduce engine: pack / unpack / reduce / fused SGD epilogue.

GPU tensors run the hand-written CDNA4 kernels of ``csrc/bfp/bfp_kernels.hip`` (a missing extension is
a hard error on GPU). CPU tensors run the bit-exact NumPy oracle (``bfp_oracle``) so that the gloo
multi-process tests exercise exactly the same numerics as the GPU path.
"""
from __future__ import annotations

import numpy as np
import torch

from .. import _ext
from . import bfp_oracle as O

CODEC_IDS = O.CODECS


def codec_id(codec) -> int:
    return O.codec_id(codec)


def is_raw(codec) -> bool:
    return codec_id(codec) in (2, 3)


def shard_bytes(codec, n_s: int) -> int:
    return O.shard_bytes(codec, n_s)


def _np_f32(t: torch.Tensor) -> np.ndarray:
    return t.detach().to(torch.float32).contiguous().view(-1).numpy()


def _np_u8(t: torch.Tensor) -> np.ndarray:
    return t.detach().contiguous().view(torch.uint8).view(-1).numpy()


def as_bytes(t: torch.Tensor) -> torch.Tensor:
    """uint8 view of a contiguous tensor (zero copy)."""
    return t.contiguous().view(torch.uint8).view(-1)


def pack(x: torch.Tensor, out: torch.Tensor, shard_elems: int, codec) -> torch.Tensor:
    """Encode dense x (f32/bf16, numel % shard_elems == 0) into ``out`` (uint8)."""
    c = codec_id(codec)
    if x.is_cuda:
        _ext.require().wire_pack(x, out, int(shard_elems), c)
        return out
    buf = O.pack(_np_f32(x), shard_elems, c)
    out.view(-1)[: buf.size].copy_(torch.from_numpy(buf))
    return out


def unpack(packed: torch.Tensor, out: torch.Tensor, shard_elems: int, codec) -> torch.Tensor:
    c = codec_id(codec)
    if out.is_cuda:
        _ext.require().wire_unpack(packed, out, int(shard_elems), c)
        return out
    v = O.unpack(_np_u8(packed), out.numel(), shard_elems, c)
    out.view(-1).copy_(torch.from_numpy(v).to(out.dtype))
    return out


def reduce(slots: torch.Tensor, n_slots: int, self_pos: int, local: torch.Tensor | None,
           out_wire: torch.Tensor | None, out_f32: torch.Tensor | None, shard_elems: int, codec):
    """Sum ``n_slots`` wire shards stored back to back in ``slots`` (slot ``self_pos`` replaced by the
    dense ``local`` operand when given) and write the result as wire (``out_wire``) and/or f32."""
    c = codec_id(codec)
    if slots.is_cuda:
        _ext.require().wire_reduce(slots, int(n_slots), int(self_pos), local, out_wire, out_f32,
                                   int(shard_elems), c)
        return
    sb = O.shard_bytes(c, shard_elems)
    raw = _np_u8(slots)
    slot_list = [raw[r * sb:(r + 1) * sb] for r in range(n_slots)]
    acc = O.reduce_slots(slot_list, None if local is None else _np_f32(local), self_pos, c, shard_elems)
    if out_f32 is not None:
        out_f32.view(-1)[:shard_elems].copy_(torch.from_numpy(acc))
    if out_wire is not None:
        buf = O.pack(acc, shard_elems, c)
        as_bytes(out_wire)[: buf.size].copy_(torch.from_numpy(buf))


def sgd(wire: torch.Tensor, shard_elems: int, n_shards: int, master: torch.Tensor, *, codec,
        lp: torch.Tensor | None = None, mom: torch.Tensor | None = None, lr: float, grad_scale: float = 1.0,
        weight_decay: float = 0.0, momentum: float = 0.0, nesterov: bool = False, n_valid: int | None = None,
        skip_shard: int = -1, skip_period: int = 0):
    """Fused decode + SGD in place: master -= lr * (scale * g [+ wd * w], momentum); lp = bf16(master)."""
    c = codec_id(codec)
    n_valid = master.numel() if n_valid is None else int(n_valid)
    if master.is_cuda:
        _ext.require().wire_sgd(wire, int(shard_elems), int(n_shards), int(skip_shard), int(skip_period), master,
                                lp, mom, float(lr), float(grad_scale), float(weight_decay), float(momentum),
                                bool(nesterov), n_valid, c)
        return
    n = shard_elems * n_shards
    g = O.unpack(_np_u8(wire), n, shard_elems, c)
    w = master.view(-1).numpy()
    m = mom.view(-1).numpy() if mom is not None else None
    period = skip_period if skip_period >= 1 else (1 << 30)
    for s in range(n_shards):
        if skip_shard >= 0 and s % period == skip_shard:
            continue
        lo, hi = s * shard_elems, min((s + 1) * shard_elems, n_valid)
        if hi <= lo:
            continue
        nw, nm = O.sgd(w[lo:hi], g[lo:hi], lr, grad_scale, weight_decay, momentum,
                       None if m is None else m[lo:hi], nesterov)
        w[lo:hi] = nw
        if m is not None and nm is not None:
            m[lo:hi] = nm
    if lp is not None:
        lp.view(-1)[:n_valid].copy_(master.view(-1)[:n_valid].to(lp.dtype))
