"""Bit-exact NumPy oracles for the BFP wire format (the ground truth every kernel is tested against).

Two numerics are modelled:

* ``trunc`` — the reference NIC, bit for bit (NX_MODE=0, MANT_SIZE=8, group 16):
  encode = hw/bf16_to_bfp_core.sv:97-126 + hw/bfp_adapter.sv:145-154 (shared exponent = max biased exponent,
  hidden bit forced to 1 even for zeros/denormals, right shift with shifts >= 32 clearing
  (hw/barrel_shifter.sv:44-51), 25-bit two's complement, keep bits [24:17] => floor);
  decode = hw/bfp_to_bf16_core.sv:55-117 (magnitude |q|<<16 with |-128| = 128, exponent field
  E + 1 - lzc24 wrapping mod 256, mantissa bit 0 forced to 0; so q = 0 decodes to 2^(E-150)).
* ``rne`` — this framework's default: q = clamp(rint(x * 2^(133-E)), -127, 127), decode q * 2^(E-133)
  (exact zero, symmetric range, half the error bound of truncation). E = 255 (Inf/NaN in the group)
  decodes to NaN so corrupted gradients fail loudly.

Packed layout of a shard of n_s elements (n_s % 256 == 0): ``[int8 mant[n_s]][uint8 exp[n_s/16]]``;
multi-shard buffers are shards back to back.
"""
from __future__ import annotations

import numpy as np

GROUP = 16
CODECS = {"bfp_trunc": 0, "bfp_rne": 1, "raw_f32": 2, "raw_bf16": 3}
CODEC_NAMES = {v: k for k, v in CODECS.items()}


def codec_id(codec) -> int:
    if isinstance(codec, str):
        return CODECS[codec]
    return int(codec)


def shard_bytes(codec, n_s: int) -> int:
    c = codec_id(codec)
    if c in (0, 1):
        return n_s + n_s // 16
    return n_s * (4 if c == 2 else 2)


# --------------------------------------------------------------------------- bf16 helpers
def f32_to_bf16_bits(x: np.ndarray) -> np.ndarray:
    """RNE fp32 -> bf16 (NaN preserving), returned as uint16."""
    u = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32).astype(np.uint64)
    nan = np.isnan(np.ascontiguousarray(x, dtype=np.float32))
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    r = np.where(nan, ((u >> 16) | 0x40).astype(np.uint16), r)
    return r.astype(np.uint16)


def bf16_bits_to_f32(b: np.ndarray) -> np.ndarray:
    return (np.asarray(b, dtype=np.uint16).astype(np.uint32) << 16).view(np.float32)


# --------------------------------------------------------------------------- group primitives
def _shared_exp(bits: np.ndarray) -> np.ndarray:
    """bits: uint32 [G, 16] -> E uint32 [G, 1] (max biased exponent of the group)."""
    return (((bits & 0x7FFFFFFF).max(axis=1, keepdims=True)) >> 23).astype(np.uint32)


def encode_groups(x: np.ndarray, rounding: str = "rne"):
    """x: float32 [..] (size % 16 == 0) -> (q int8 [n], E uint8 [n/16])."""
    x = np.ascontiguousarray(x, dtype=np.float32).reshape(-1, GROUP)
    bits = x.view(np.uint32)
    E = _shared_exp(bits)
    if rounding == "trunc":
        e = (bits >> 23) & 0xFF
        m = ((bits & 0x7FFFFF) | 0x800000).astype(np.int64)
        d = (E - e).astype(np.int64)  # 0..255 (E >= e)
        a = np.where(d >= 32, 0, m >> np.minimum(d, 31))
        t = np.where((bits >> 31) == 1, -a, a)
        q = (t >> 17).astype(np.int8)
    elif rounding == "rne":
        with np.errstate(over="ignore", invalid="ignore"):
            s = np.ldexp(x, (133 - E.astype(np.int32)))
            s = np.rint(s)
            s = np.clip(np.nan_to_num(s, nan=-127.0, posinf=127.0, neginf=-127.0), -127, 127)
        q = s.astype(np.int8)
    else:
        raise ValueError(rounding)
    return q.reshape(-1), E.reshape(-1).astype(np.uint8)


def decode_groups(q: np.ndarray, E: np.ndarray, rounding: str = "rne") -> np.ndarray:
    q = np.asarray(q, dtype=np.int8).reshape(-1, GROUP).astype(np.int32)
    Eu = np.asarray(E, dtype=np.uint8).reshape(-1, 1).astype(np.uint32)
    if rounding == "trunc":
        sign = (q < 0).astype(np.uint32)
        M = (np.abs(q).astype(np.uint32)) << 16  # |-128| = 128 -> 2^23
        # 24-bit leading-zero count (24 for 0)
        zc = np.where(M == 0, 24, 23 - np.floor(np.log2(np.maximum(M, 1))).astype(np.int64)).astype(np.uint32)
        ex = (Eu + 1 - zc) & 0xFF
        frac = (M << zc) & 0x7FFFFE
        bits = (sign << 31) | (ex << 23) | frac
        return bits.astype(np.uint32).view(np.float32).reshape(-1)
    if rounding == "rne":
        v = np.ldexp(q.astype(np.float32), (Eu.astype(np.int32) - 133)).astype(np.float32)
        v = np.where(Eu == 255, np.float32(np.nan), v)
        return v.reshape(-1).astype(np.float32)
    raise ValueError(rounding)


def _rounding_of(codec) -> str:
    c = codec_id(codec)
    return "trunc" if c == 0 else "rne"


# --------------------------------------------------------------------------- packed buffers
def pack(x: np.ndarray, shard_elems: int, codec="bfp_rne") -> np.ndarray:
    """Dense f32 (or bf16 given as float32 values) -> packed uint8 buffer (per-shard layout)."""
    c = codec_id(codec)
    x = np.ascontiguousarray(x, dtype=np.float32).reshape(-1)
    assert x.size % shard_elems == 0 and shard_elems % 256 == 0
    if c == 2:
        return x.view(np.uint8).copy()
    if c == 3:
        return f32_to_bf16_bits(x).view(np.uint8).copy()
    out = []
    for s in range(x.size // shard_elems):
        q, E = encode_groups(x[s * shard_elems:(s + 1) * shard_elems], _rounding_of(c))
        out.append(q.view(np.uint8))
        out.append(E)
    return np.concatenate(out)


def unpack(buf: np.ndarray, n: int, shard_elems: int, codec="bfp_rne") -> np.ndarray:
    c = codec_id(codec)
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    if c == 2:
        return buf[: 4 * n].view(np.float32).copy()
    if c == 3:
        return bf16_bits_to_f32(buf[: 2 * n].view(np.uint16))
    sb = shard_bytes(c, shard_elems)
    out = []
    for s in range(n // shard_elems):
        sh = buf[s * sb:(s + 1) * sb]
        out.append(decode_groups(sh[:shard_elems].view(np.int8), sh[shard_elems:], _rounding_of(c)))
    return np.concatenate(out) if out else np.zeros(0, np.float32)


def quantize(x: np.ndarray, codec="bfp_rne") -> np.ndarray:
    """decode(encode(x)) for a dense vector (size % 16 == 0)."""
    c = codec_id(codec)
    x = np.ascontiguousarray(x, dtype=np.float32).reshape(-1)
    if c == 2:
        return x.copy()
    if c == 3:
        return bf16_bits_to_f32(f32_to_bf16_bits(x))
    q, E = encode_groups(x, _rounding_of(c))
    return decode_groups(q, E, _rounding_of(c))


def reduce_slots(slots, local=None, self_pos: int = -1, codec="bfp_rne", shard_elems: int | None = None):
    """Sum decoded slots (packed single-shard buffers) in slot order, with the dense ``local`` operand
    standing in for slot ``self_pos``. Returns the float32 sum (the caller re-encodes)."""
    c = codec_id(codec)
    n = shard_elems
    acc = np.zeros(n, np.float32)
    nslots = len(slots)
    for r in range(nslots):
        if local is not None and r == self_pos:
            v = np.asarray(local, np.float32).reshape(-1)[:n]
        else:
            v = unpack(slots[r], n, n, c)
        acc = (acc + v).astype(np.float32)
    return acc


def sgd(w: np.ndarray, g: np.ndarray, lr: float, grad_scale: float = 1.0, weight_decay: float = 0.0,
        momentum: float = 0.0, mom: np.ndarray | None = None, nesterov: bool = False):
    """fp32 SGD with the kernel's operation order (fma emulated in float64, then rounded)."""
    w = np.asarray(w, np.float32)
    g = (np.asarray(g, np.float32) * np.float32(grad_scale)).astype(np.float32)
    if weight_decay:
        g = (np.float64(np.float32(weight_decay)) * w.astype(np.float64) + g).astype(np.float32)
    new_mom = None
    if momentum:
        m = (np.float64(np.float32(momentum)) * mom.astype(np.float64) + g).astype(np.float32)
        new_mom = m
        g = (np.float64(np.float32(momentum)) * m.astype(np.float64) + g).astype(np.float32) if nesterov else m
    w = (np.float64(-np.float32(lr)) * g.astype(np.float64) + w.astype(np.float64)).astype(np.float32)
    return w, new_mom
