"""Spec-level simulators of the all-reduce algorithms (pure NumPy, independent of the planner/engine).

They compute, from the algorithm definitions alone, the exact decoded result every rank must end up with —
the role the reference's 3-NIC RTL testbench golden model played (readme.pdf p.3-5 §3.2-3.3), but
tolerance-free: with the bit-exact codec oracle the engine must match these results bit for bit.

* ring  (SURVEY.md Appendix B): the chain for slice j of a block starts at ring position j (SEND_LOCAL) and
  moves to position j-1, j-2, ... each hop computing enc(dec(partial) + local); the position j+1 (= j-N+1)
  finishes the sum and owns slice j; the encoded full slice is then forwarded unchanged.
* mesh: owner s of shard s sums slot r = dec(enc(g_r[s])) for r != s and its own un-quantised g_s[s]
  (in rank order), re-encodes, and everyone decodes the gathered result.
"""
from __future__ import annotations

import numpy as np

from ..ops import bfp_oracle as O


def _enc_dec(x, codec):
    return O.quantize(x, codec)


def mesh_allreduce(grads: list[np.ndarray], shard: int, codec="bfp_rne") -> np.ndarray:
    N = len(grads)
    n_pad = shard * N
    out = np.zeros(n_pad, np.float32)
    for s in range(N):
        acc = np.zeros(shard, np.float32)
        for r in range(N):
            v = grads[r][s * shard:(s + 1) * shard].astype(np.float32)
            if r != s:
                v = _enc_dec(v, codec)
            acc = (acc + v).astype(np.float32)
        out[s * shard:(s + 1) * shard] = _enc_dec(acc, codec)
    return out


def ring_allreduce(grads: list[np.ndarray], orders: list[list[int]], slice_elems: int, blocks: int,
                   codec="bfp_rne", owner_fp32: bool = False) -> list[np.ndarray]:
    """Returns per-rank decoded results (identical unless owner_fp32 reproduces the reference quirk)."""
    N = len(grads)
    S = slice_elems
    part = blocks * N * S
    outs = [np.zeros(part * len(orders), np.float32) for _ in range(N)]
    for i, order in enumerate(orders):
        off = i * part
        for b in range(blocks):
            for j in range(N):
                lo = off + (b * N + j) * S
                chain = [order[(j - k) % N] for k in range(N)]  # ring positions j, j-1, ..., j-N+1
                val = _enc_dec(grads[chain[0]][lo:lo + S], codec)
                full_f32 = grads[chain[0]][lo:lo + S].astype(np.float32)
                for k in range(1, N):
                    s = (np.zeros(S, np.float32) + val).astype(np.float32)
                    s = (s + grads[chain[k]][lo:lo + S].astype(np.float32)).astype(np.float32)
                    full_f32 = s
                    val = _enc_dec(s, codec)
                owner = chain[-1]
                for r in range(N):
                    outs[r][lo:lo + S] = full_f32 if (owner_fp32 and r == owner and N > 1) else val
    return outs
