#!/usr/bin/env python3
"""Compute/communication overlap from a rocprofv3 kernel trace (``--kernel-trace`` CSV).

Kernels are split by HIP stream (``Stream_Id``): the stream that runs the MFMA GEMMs is "compute", every
other stream that runs all-reduce work (RCCL collectives, BFP reduce / SGD kernels) is "comm". Reports, over
the steady-state window (after the first ``--skip`` fraction of the trace):

* comm busy time, and the part of it that ran while a compute kernel was running (overlapped);
* compute busy time and the whole window, so exposed-comm = comm busy - overlapped;
* the exposed stretches themselves (comm running while no compute kernel runs): their count, the longest, and the
  median — at world > 1 the per-step communication tail after the last backward GEMM is one such stretch per step.

Usage: python tools/overlap_report.py gpurun_out/prof_x/run_kernel_trace.csv [--skip 0.3] [--json out.json]
"""
from __future__ import annotations

import argparse
import csv
import json


def _union(iv):
    iv = sorted(iv)
    out = []
    for s, e in iv:
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def _length(iv):
    return sum(e - s for s, e in iv)


def _intersect(a, b):
    i = j = 0
    out = 0
    while i < len(a) and j < len(b):
        s, e = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if s < e:
            out += e - s
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return out


def _subtract(a, b):
    """Intervals of a not covered by b (both sorted, disjoint)."""
    out = []
    j = 0
    for s, e in a:
        cur = s
        while j < len(b) and b[j][1] <= cur:
            j += 1
        k = j
        while k < len(b) and b[k][0] < e:
            if b[k][0] > cur:
                out.append((cur, b[k][0]))
            cur = max(cur, b[k][1])
            k += 1
        if cur < e:
            out.append((cur, e))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--skip", type=float, default=0.3, help="fraction of the trace to skip (warmup)")
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"], r["Kernel_Name"]) for r in rows]
    t0, t1 = min(k[0] for k in ks), max(k[1] for k in ks)
    cut = t0 + (t1 - t0) * a.skip
    ks = [k for k in ks if k[0] >= cut]
    gemm_streams = {k[2] for k in ks if "gemm" in k[3]}
    compute = _union([(s, e) for s, e, st, _ in ks if st in gemm_streams])
    comm = _union([(s, e) for s, e, st, _ in ks if st not in gemm_streams])
    comm_names = sorted({n.split("(")[0][-60:] for _, _, st, n in ks if st not in gemm_streams})
    win = max(k[1] for k in ks) - min(k[0] for k in ks)
    ov = _intersect(compute, comm)
    exposed = sorted((e - s for s, e in _subtract(comm, compute) if e - s > 1000), reverse=True)  # > 1 us
    rep = {
        "window_us": win / 1e3,
        "compute_busy_us": _length(compute) / 1e3,
        "comm_busy_us": _length(comm) / 1e3,
        "comm_overlapped_us": ov / 1e3,
        "comm_exposed_us": (_length(comm) - ov) / 1e3,
        "overlap_fraction_of_comm": (ov / _length(comm)) if comm else 0.0,
        "exposed_stretches_over_1us": len(exposed),
        "exposed_stretch_max_us": exposed[0] / 1e3 if exposed else 0.0,
        "exposed_stretch_median_us": exposed[len(exposed) // 2] / 1e3 if exposed else 0.0,
        "compute_streams": sorted(gemm_streams),
        "comm_kernels": comm_names[:20],
    }
    print(json.dumps(rep, indent=1))
    if a.json:
        json.dump(rep, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
