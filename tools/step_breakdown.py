"""Per-dispatch-shape breakdown of a rocprofv3 kernel trace: which kernel, at which grid, costs what per step.

``rocprofv3 --stats`` folds every shape of one kernel template into one row; this groups the dispatches of
``*_kernel_trace.csv`` by (kernel template with its arguments, grid, workgroup, LDS) — so the fwd / bwd-data /
bwd-weight GEMMs of each layer, which share a template, show up as separate rows — and reports count, mean and
µs per step (total over the trace / --steps). Rows are per position in the step (the trace's period).

    python tools/step_breakdown.py gpurun_out/x/prof/run_kernel_trace.csv --steps 28 [--top 30] [--csv out.csv]
"""
from __future__ import annotations

import argparse
import csv
import re
import sys
from collections import OrderedDict


def short_name(n: str) -> str:
    n = n.strip().replace("(anonymous namespace)::", "")
    n = re.sub(r"\(.*\)$", "", n)  # drop the parameter list
    n = n.replace("void ", "").replace("fan::gemm_detail::", "").replace("fan::", "")
    n = n.replace("unsigned short", "bf16").replace("at::native::", "")
    return n[:110]


def _steady_window(keys, steps, max_p=400):
    """(P, start) of the LAST window of steps*P dispatches that repeats with period P, for the smallest such P
    (kernels per training step): the timed steps, wherever warmup / plan-tuning launches before them and the
    run's own bookkeeping after them sit in the trace. (0, 0) if none."""
    n = len(keys)
    for p in range(1, min(max_p, n // max(steps, 2)) + 1):
        need = (steps - 1) * p  # consecutive positions i with keys[i] == keys[i + p]
        run = 0
        for i in range(n - p - 1, -1, -1):  # scan from the end: the last such window
            run = run + 1 if keys[i] == keys[i + p] else 0
            if run >= need and need > 0:
                return p, i
    return 0, 0


def breakdown(path: str, steps: int):
    """Rows per (position in the step, kernel, grid): the last ``steps`` periods of the trace (the timed steps,
    when the trace ends with them); without a detectable period, all dispatches grouped by (kernel, grid)."""
    disp = []
    with open(path) as f:
        for r in csv.DictReader(f):
            key = (short_name(r["Kernel_Name"]), int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"])),
                   int(r["Workgroup_Size_X"]), int(r.get("LDS_Block_Size", 0) or 0))
            disp.append((int(r["Start_Timestamp"]), key, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
    disp.sort()
    keys = [k for _, k, _ in disp]
    P, lo = _steady_window(keys, steps)
    rows = OrderedDict()
    if P:
        disp = disp[lo:lo + P * steps]
    for i, (_, key, d) in enumerate(disp):
        k = ((i % P) if P else -1,) + key
        e = rows.setdefault(k, [0, 0.0, 1e30, 0.0])
        e[0] += 1
        e[1] += d
        e[2] = min(e[2], d)
        e[3] = max(e[3], d)
    out = []
    for (pos, name, wgs, wg, lds), (n, tot, mn, mx) in rows.items():
        out.append({"pos": pos, "kernel": name, "workgroups": wgs, "wg_size": wg, "lds": lds, "calls": n,
                    "mean_us": tot / n, "min_us": mn, "max_us": mx, "us_per_step": tot / max(1, steps)})
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, required=True, help="training steps the trace covers (divides totals)")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--csv", default=None)
    ap.add_argument("--by-cost", action="store_true", help="sort by us/step instead of step order")
    a = ap.parse_args(argv)
    rows = breakdown(a.trace, a.steps)
    if not a.by_cost:
        rows.sort(key=lambda r: r["pos"])
    else:
        rows.sort(key=lambda r: -r["us_per_step"])
    total = sum(r["us_per_step"] for r in rows)
    print(f"{'pos':>4} {'us/step':>9} {'mean':>8} {'min':>8} {'calls':>6} {'WGs':>6}  kernel   (total {total:.1f} us/step)")
    for r in rows[: a.top]:
        print(f"{r['pos']:4d} {r['us_per_step']:9.1f} {r['mean_us']:8.1f} {r['min_us']:8.1f} {r['calls']:6d} "
              f"{r['workgroups']:6d}  {r['kernel']}")
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
            w.writeheader()
            w.writerows(rows)
    return 0


if __name__ == "__main__":
    sys.exit(main())
