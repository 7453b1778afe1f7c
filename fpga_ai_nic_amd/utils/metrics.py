"""Metrics and the reference-compatible report.

Keeps the reference's stdout lines (sw/mlp_mpi_example_f32.cpp:353-377, 800-814) — the setup banner,
``GFLOP``, ``fp time``, ``GFLOPS``, the machine-readable ``PERFDUMP,BP,...`` CSV line and the three
DETAILED_PROFILE lines — and adds samples/s, all-reduce algo-BW / bus-BW and a JSONL sink.
"""
from __future__ import annotations

import json
import os
import time

from .. import __version__


def mlp_gflop(sizes, global_mb: int, kind: str = "A") -> float:
    """The reference formulas. 'A' (sw:794-798): 6*MB*C_i*C_{i+1} for layers >= 1, 4*MB*C0*C1 for layer 0;
    'F' (sw:574-577): 2*MB*C_i*C_{i+1}; 'B' (sw:654-658): 4*MB*C_i*C_{i+1} for layers >= 1, 2*MB*C0*C1."""
    hi, lo = {"A": (6.0, 4.0), "F": (2.0, 2.0), "B": (4.0, 2.0)}[kind]
    g = 0.0
    L = len(sizes) - 1
    for i in range(L - 1, 0, -1):
        g += hi * global_mb * sizes[i] * sizes[i + 1] / 1e9
    g += lo * global_mb * sizes[0] * sizes[1] / 1e9
    return g


def setup_banner(sizes, global_mb: int, iters: int, threads: int, bytes_per_el: int = 4,
                 show_threads: bool = True) -> str:
    """The reference's "Setting Up (Common)" block (sw:353-377). As there, the thread count is printed only
    when ``CHECK`` is 0 (``show_threads``)."""
    L = len(sizes) - 1
    lines = ["##########################################", "#          Setting Up (Common)           #",
             "##########################################", f"PARAMS: N:{global_mb}", f"PARAMS: Layers: {L}",
             f"PARAMS: ITERS:{iters}  Threads:{threads}" if show_threads else f"PARAMS: ITERS:{iters}"]
    mib = 1024.0 * 1024.0
    act = fil = 0.0
    for i in range(L):
        if i == 0:
            a = global_mb * sizes[i] * bytes_per_el / mib
            act += a
            lines.append(f"SIZE Activations  {i} ({global_mb}x{sizes[i]}): {a:10.2f} MiB")
        a = global_mb * sizes[i + 1] * bytes_per_el / mib
        f = sizes[i] * sizes[i + 1] * bytes_per_el / mib
        act += a
        fil += f
        lines.append(f"SIZE Filter       {i} ({sizes[i]}x{sizes[i + 1]}): {f:10.2f} MiB")
        lines.append(f"SIZE Activations  {i + 1} ({global_mb}x{sizes[i + 1]}): {a:10.2f} MiB")
    a = global_mb * sizes[-1] * bytes_per_el / mib
    act += a
    lines.append(f"SIZE Activations softmax ({global_mb}x{sizes[-1]}): {a:10.2f} MiB")
    lines += ["", f"TOTAL SIZE Activations:    {act:10.2f} MiB", f"TOTAL SIZE Filter:         {fil:10.2f} MiB",
              f"TOTAL SIZE delActivations: {act:10.2f} MiB", f"TOTAL SIZE delFilter:      {fil:10.2f} MiB",
              f"TOTAL SIZE MLP:            {2 * fil + 2 * act:10.2f} MiB"]
    return "\n".join(lines)


def result_report(sizes, global_mb: int, mb_local: int, iters: int, total_s: float, threads: int,
                  times: dict | None = None, kind: str = "A") -> str:
    gflop = mlp_gflop(sizes, global_mb, kind)
    t = total_s / max(iters, 1)
    gflops = gflop / t if t > 0 else 0.0
    L = len(sizes) - 1
    lines = [f"GFLOP  = {gflop:.5g}", f"fp time = {t:.5g}", f"GFLOPS  = {gflops:.5g}",
             f"PERFDUMP,{'FP' if kind == 'F' else 'BP'},fan-" + __version__ + f",{threads},{mb_local}," + "".join(f"{c}," for c in sizes[:L])
             + f"{t:f},{gflops:f}",
             f"SAMPLES/S = {global_mb / t if t > 0 else 0.0:.5g}"]
    if times and times.get("steps"):
        n = times["steps"]
        tot = times["fwd"] + times["loss"] + times["bwd"]
        lines.append(f"FC time compute/loss = {tot / n:.5g}")
        lines.append(f"Bwdupd compute FIRST time overlaped = {times['bwd_first'] / n:.5g}")
        lines.append(f"Bwdupd compute time overlaped = {(times['bwd'] - times['bwd_first']) / n:.5g}")
    return "\n".join(lines)


def matdiff(ref, tst) -> dict:
    """Norms of a test matrix against a reference (the libxsmm_matdiff report the reference links, sw:818-826):
    l1/l2/linf of the difference, their values relative to the reference, and the two L1 norms."""
    import numpy as np

    r = np.asarray(ref, dtype=np.float64).reshape(-1)
    t = np.asarray(tst, dtype=np.float64).reshape(-1)
    d = t - r
    l1_ref, l1_tst = float(np.abs(r).sum()), float(np.abs(t).sum())
    l2_abs, linf_abs = float(np.sqrt((d * d).sum())), float(np.abs(d).max()) if d.size else 0.0
    nr2 = float(np.sqrt((r * r).sum()))
    return {"l1_ref": l1_ref, "l1_tst": l1_tst, "l1_abs": float(np.abs(d).sum()),
            "l2_abs": l2_abs, "l2_rel": l2_abs / nr2 if nr2 else 0.0,
            "linf_abs": linf_abs, "linf_rel": linf_abs / float(np.abs(r).max()) if r.size and np.abs(r).max() else 0.0}


def allreduce_bw(logical_bytes: float, seconds: float, world: int):
    """(algo-BW, bus-BW) in GB/s: bus = algo * 2(N-1)/N (nccl-tests convention)."""
    if seconds <= 0:
        return 0.0, 0.0
    algo = logical_bytes / seconds / 1e9
    bus = algo * (2.0 * (world - 1) / world if world > 1 else 0.0)
    return algo, bus


class JsonlSink:
    def __init__(self, path: str | None):
        self.path = path
        if path:
            os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)

    def write(self, **rec):
        if not self.path:
            return
        rec.setdefault("ts", time.time())
        with open(self.path, "a") as f:
            f.write(json.dumps(rec) + "\n")
