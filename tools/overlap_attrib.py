#!/usr/bin/env python3
"""Where a comm/compute overlap loses its time: per-kernel attribution from three rocprofv3 kernel traces of the same
workload run as compute only, comm only and both (bench/bert_overlap.py --only compute|comm|overlap).

Each trace is cut into rounds at host gaps (idle > --gap-ms: the bench's host-side bookkeeping between rounds) and
only the LAST round is used (warmup, plan tuning and buffer setup come before it). Kernels seen in the compute-only
round are "compute", the others "comm". Reported: each round's length, busy time (union of all kernels) and idle time
(the GPU running nothing: launch gaps, waits); per kernel the mean duration alone vs in the overlapped round; for the
comm kernels of the overlapped round the share of their time during which a compute kernel ran (hidden) and how many
started right at the end of a compute kernel (they could not get CUs while it ran: a persistent GEMM holds them all).

    python tools/overlap_attrib.py compute.csv comm.csv overlap.csv [--gap-ms 5]
"""
from __future__ import annotations

import argparse
import bisect
import csv
import re
import statistics
from collections import defaultdict


def short(n: str) -> str:
    n = re.sub(r"\(.*\)$", "", n.strip().replace("(anonymous namespace)::", "").replace("void ", ""))
    n = n.replace("fan::gemm_detail::", "").replace("fan::", "")
    m = re.match(r"([A-Za-z0-9_]+)", n)
    return m.group(1) if m else n[:40]


def union(iv):
    out = []
    for s, e in sorted(iv):
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def covered(s, e, iv):
    tot = 0
    for a, b in iv:
        if b <= s:
            continue
        if a >= e:
            break
        tot += min(b, e) - max(a, s)
    return tot


def last_round(path, gap_ns):
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]))
                  for r in csv.DictReader(open(path)))
    iv = union([[s, e] for s, e, _ in rows])
    start = iv[0][0]
    for i in range(1, len(iv)):
        if iv[i][0] - iv[i - 1][1] > gap_ns:
            start = iv[i][0]
    return [r for r in rows if r[0] >= start]


def stats(rows):
    iv = union([[s, e] for s, e, _ in rows])
    win = rows[-1][1] - rows[0][0] if rows else 0
    busy = sum(e - s for s, e in iv)
    return win, busy


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("compute")
    ap.add_argument("comm")
    ap.add_argument("overlap")
    ap.add_argument("--gap-ms", type=float, default=5.0)
    a = ap.parse_args()
    g = a.gap_ms * 1e6
    R = {k: last_round(p, g) for k, p in (("compute", a.compute), ("comm", a.comm), ("overlap", a.overlap))}
    fam_compute = {n for _, _, n in R["compute"]}
    print("round          length_us  busy_us  idle_us  kernels")
    for k, rows in R.items():
        win, busy = stats(rows)
        print(f"{k:12s} {win / 1e3:10.1f} {busy / 1e3:8.1f} {(win - busy) / 1e3:8.1f} {len(rows):8d}")
    dur = {k: defaultdict(list) for k in R}
    for k, rows in R.items():
        for s, e, n in rows:
            dur[k][n].append((e - s) / 1e3)
    ov = R["overlap"]
    comp_iv = union([[s, e] for s, e, n in ov if n in fam_compute])
    comp_ends = sorted(e for s, e, n in ov if n in fam_compute)
    hidden = defaultdict(lambda: [0, 0])
    at_end = defaultdict(lambda: [0, 0])
    for s, e, n in ov:
        if n in fam_compute:
            continue
        hidden[n][0] += covered(s, e, comp_iv)
        hidden[n][1] += e - s
        i = bisect.bisect_right(comp_ends, s) - 1
        at_end[n][1] += 1
        if i >= 0 and 0 <= s - comp_ends[i] <= 3000:
            at_end[n][0] += 1
    print()
    print(f"{'kernel':34s} {'role':7s} {'alone us':>9s} {'overlap us':>10s} {'x':>5s} {'hidden %':>8s} {'at GEMM end':>11s} "
          f"{'n':>4s}")
    for n in sorted(dur["overlap"], key=lambda n: -sum(dur["overlap"][n])):
        role = "compute" if n in fam_compute else "comm"
        alone = dur[role].get(n, [])
        ma = statistics.mean(alone) if alone else float("nan")
        mo = statistics.mean(dur["overlap"][n])
        h = hidden.get(n)
        hp = f"{100 * h[0] / h[1]:8.1f}" if h and h[1] else f"{'-':>8s}"
        ae = f"{at_end[n][0]}/{at_end[n][1]}" if n in at_end else "-"
        print(f"{n[:34]:34s} {role:7s} {ma:9.1f} {mo:10.1f} {mo / ma if alone else float('nan'):5.2f} {hp} {ae:>11s} "
              f"{len(dur['overlap'][n]):4d}")
    tc = sum(v[1] for v in hidden.values())
    th = sum(v[0] for v in hidden.values())
    print(f"\ncomm kernel time in the overlapped round {tc / 1e3:.1f} us, {100 * th / max(1, tc):.1f} % of it beside a "
          f"compute kernel")


if __name__ == "__main__":
    main()
