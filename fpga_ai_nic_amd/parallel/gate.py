"""Exactness gate for a multi-rank all-reduce: one request through the engine's production path, checked bit for bit
against the spec simulators on every rank.

Replica identity after a run cannot catch a wrong-but-consistent reduce (a stale read of a peer's slot by the owner of
a shard corrupts that shard for everyone alike). So before a benchmark trusts an engine, every rank regenerates the
seeded gradients of ALL ranks, runs one request of its own gradient through the engine exactly as training does
(BFP-encoded by the "producer" into the engine's wire layout when the engine takes prepacked input, the direct P2P
rounds when the communicator is the P2P transport), and compares the decoded sum with the NumPy simulator of the
engine's algorithm (:mod:`.sim`, over the bit-exact codec oracle :mod:`..ops.bfp_oracle`). The reference has no such
check at all: its RTL testbench prints FAILED for every compressed run (readme.pdf p.5), and the host never checks
the NIC's result (sw/mlp_mpi_example_f32.cpp:818-826 is disabled).
"""
from __future__ import annotations

import numpy as np
import torch

from . import sim


def seeded_gradients(n: int, world: int, seed: int) -> list[np.ndarray]:
    """Rank r's gradient: normal values with a per-16-group scale of 2^[-12, 4) (every group a different shared
    exponent, some groups 2^16 apart) — regenerable by every rank."""
    out = []
    for r in range(world):
        rng = np.random.default_rng(seed + 7919 * r)
        g = rng.standard_normal(n).astype(np.float32)
        scale = np.exp2(rng.integers(-12, 4, size=(n + 15) // 16)).astype(np.float32)
        out.append((g * np.repeat(scale, 16)[:n]).astype(np.float32))
    return out


def reference_sum(engine, grads: list[np.ndarray], n: int, rank: int) -> np.ndarray | None:
    """What rank ``rank`` must decode for this engine's layout and algorithm (None: no bit-exact spec, e.g. RCCL's
    own summation order)."""
    algo = getattr(engine, "algo", "mesh")
    codec = getattr(engine, "codec", "bfp_rne")
    L = engine.layout(n)
    gin = [np.pad(g, (0, L.n_pad - n)) for g in grads]
    if algo == "mesh":
        N = len(grads)
        chunks = max(1, int(getattr(L, "chunks", 1) or 1))
        span = N * L.shard
        out = np.zeros(L.n_pad, np.float32)
        for c in range(chunks):
            sl = slice(c * span, (c + 1) * span)
            out[sl] = sim.mesh_allreduce([x[sl] for x in gin], L.shard, codec)
        return out
    if algo == "ring":
        return sim.ring_allreduce(gin, [list(o) for o in engine.orders], L.slice_elems, L.blocks, codec)[rank]
    return None


def allreduce_exactness(engine, *, n: int = 1 << 20, seed: int = 20260417, prepacked: bool = True,
                        timeout_s: float = 120.0) -> dict:
    """Run the gate on this rank (collective over the default group when it is initialised). Returns
    ``{"exact": bool (all ranks), "checked": bool, "n", "prepacked", "mismatch_ranks", "max_abs_diff"}``."""
    from ..utils import dist as D

    world = engine.world
    rank = getattr(engine, "rank", 0)
    dev = getattr(engine, "device", torch.device("cuda" if torch.cuda.is_available() else "cpu"))
    grads = seeded_gradients(n, world, seed)
    L = engine.layout(n)
    g = torch.zeros(L.n_pad, dtype=torch.float32, device=dev)
    g[:n] = torch.from_numpy(grads[rank]).to(dev)
    out = torch.zeros(L.n_pad, dtype=torch.float32, device=dev)
    kw = {}
    used_pre = False
    if prepacked and getattr(engine, "prepack", False) and g.is_cuda:
        tgt = engine.prepack_target(g, n)
        if tgt is not None:  # the producer's role (the bwd-weight GEMM's wire epilogue): encode [0, n) itself
            from .. import _ext

            buf, shard, _, cid = tgt[:4]
            _ext.require().wire_pack_range(g, buf, shard, 0, n, cid)
            kw["prepacked"] = (buf, L.n_pad)
            used_pre = True
    err = None
    try:
        engine.allreduce(g, out, n_valid=n, **kw).synchronize(timeout_s)
        if g.is_cuda:
            torch.cuda.synchronize(dev)
    except Exception as e:  # noqa: BLE001 - agreed below: a rank whose request failed must not leave its peers
        err = f"rank {rank}: {e}"  # at a different collective (one rank's abort can let another's request finish)
    err = next((x for x in D.all_gather_object(err) if x), None)
    if err:
        raise RuntimeError(f"exactness gate request failed: {err}"[:600])
    got = out[:n].cpu().numpy()
    ref = reference_sum(engine, grads, n, rank)
    mine = {"checked": ref is not None, "exact": True, "max_abs_diff": 0.0}
    if ref is not None:
        ref = ref[:n]
        same = np.array_equal(got.view(np.uint32), ref.view(np.uint32))
        mine["exact"] = bool(same)
        if not same:
            with np.errstate(invalid="ignore"):
                mine["max_abs_diff"] = float(np.nanmax(np.abs(got.astype(np.float64) - ref.astype(np.float64))))
    every = D.all_gather_object(mine)
    return {
        "exact": all(e["exact"] for e in every),
        "checked": all(e["checked"] for e in every),
        "n": n,
        "prepacked": used_pre,
        "mismatch_ranks": [r for r, e in enumerate(every) if not e["exact"]],
        "max_abs_diff": max(e["max_abs_diff"] for e in every),
    }


def allreduce_exactness_layouts(engine, sizes, **kw) -> dict:
    """:func:`allreduce_exactness` once per distinct bucket size of the trained model (each layer's ``n``): the
    production layouts themselves — at this world's arena slot the engine chunks a bucket differently, and a ring
    splits it into more blocks — not just one 1 Mi-element request. Same keys as the single gate (``n`` is the list
    of sizes checked) plus ``layouts``: one entry per size."""
    res = []
    for n in sorted({int(x) for x in sizes}):
        g = allreduce_exactness(engine, n=n, **kw)
        L = engine.layout(n)
        res.append({"n": n, "exact": g["exact"], "max_abs_diff": g["max_abs_diff"], "prepacked": g["prepacked"],
                    "n_pad": int(L.n_pad), "shard": int(getattr(L, "shard", 0) or 0),
                    "chunks": int(getattr(L, "chunks", 1) or 1), "blocks": int(getattr(L, "blocks", 0) or 0),
                    "mismatch_ranks": g["mismatch_ranks"]})
    return {
        "exact": all(r["exact"] for r in res),
        "checked": True,
        "n": [r["n"] for r in res],
        "prepacked": all(r["prepacked"] for r in res),
        "mismatch_ranks": sorted({q for r in res for q in r["mismatch_ranks"]}),
        "max_abs_diff": max((r["max_abs_diff"] for r in res), default=0.0),
        "layouts": res,
    }


def update_exactness(engine, *, n: int = 1 << 18, seed: int = 20261018, lr: float = 0.05, momentum: float = 0.9,
                     timeout_s: float = 120.0) -> dict:
    """The weight-update half of a request, checked bit for bit: every rank starts from the same seeded master /
    momentum planes, runs ONE all-reduce + SGD request of its seeded gradient through the engine's production
    ``allreduce_sgd`` (the sharded-update schedule when the engine runs it: owner reduce + SGD, bf16 weight
    all-gather), then compares its bf16 weights and — gathered from their owners when sharded — its master and
    momentum with the oracle: the simulator's decoded sum through fp32 SGD (:func:`..ops.bfp_oracle.sgd`, the
    kernel's operation order). Collective. ``{"exact", "checked", "n", "sharded", "mismatch_ranks"}``."""
    from ..ops import bfp_oracle as O
    from ..utils import dist as D

    world = engine.world
    rank = getattr(engine, "rank", 0)
    dev = getattr(engine, "device", torch.device("cuda" if torch.cuda.is_available() else "cpu"))
    grads = seeded_gradients(n, world, seed)
    rng = np.random.default_rng(seed + 1)
    w0 = rng.standard_normal(n).astype(np.float32)
    m0 = (rng.standard_normal(n) * 0.01).astype(np.float32)
    L = engine.layout(n)
    g = torch.zeros(L.n_pad, dtype=torch.float32, device=dev)
    g[:n] = torch.from_numpy(grads[rank]).to(dev)
    w = torch.zeros(L.n_pad, dtype=torch.float32, device=dev)
    w[:n] = torch.from_numpy(w0).to(dev)
    mom = torch.zeros(L.n_pad, dtype=torch.float32, device=dev)
    mom[:n] = torch.from_numpy(m0).to(dev)
    lp = torch.zeros(L.n_pad, dtype=torch.bfloat16, device=dev)
    err = None
    try:
        engine.allreduce_sgd(g, w, lp, mom, n_valid=n, lr=lr, grad_scale=1.0 / world, momentum=momentum
                             ).synchronize(timeout_s)
        if g.is_cuda:
            torch.cuda.synchronize(dev)
    except Exception as e:  # noqa: BLE001
        err = f"rank {rank}: {e}"
    err = next((x for x in D.all_gather_object(err) if x), None)
    if err:
        raise RuntimeError(f"update gate request failed: {err}"[:600])
    sharded = bool(getattr(engine, "shard_update", False))
    if sharded:
        engine.gather_owned(w, n)
        engine.gather_owned(mom, n)
    ref = reference_sum(engine, grads, n, rank)
    mine = {"checked": ref is not None, "exact": True}
    if ref is not None:
        w_ref, m_ref = O.sgd(w0, ref[:n], lr, grad_scale=1.0 / world, momentum=momentum, mom=m0)
        lp_ref = O.f32_to_bf16_bits(w_ref)
        got_lp = lp[:n].view(torch.int16).cpu().numpy().view(np.uint16)
        mine["exact"] = bool(np.array_equal(w[:n].cpu().numpy().view(np.uint32), w_ref.view(np.uint32))
                             and np.array_equal(mom[:n].cpu().numpy().view(np.uint32), m_ref.view(np.uint32))
                             and np.array_equal(got_lp, lp_ref.astype(np.uint16)))
    every = D.all_gather_object(mine)
    return {"exact": all(e["exact"] for e in every), "checked": all(e["checked"] for e in every), "n": n,
            "sharded": sharded, "mismatch_ranks": [r for r, e in enumerate(every) if not e["exact"]]}
