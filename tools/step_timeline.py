"""One training step of a rocprofv3 kernel trace as a timeline: every dispatch between two consecutive occurrences of
a marker kernel (default: the softmax-xent kernel, once per step), with its start offset from the marker, its
duration, the HIP stream it ran on and its name — so the compute stream's GEMM chain and the comm stream's requests
can be read side by side, and the critical path after the last backward GEMM measured.

    python tools/step_timeline.py prof/run_kernel_trace.csv|prof/run_results.db [--marker softmax_xent] [--step -2]

``--step`` picks which step (Python index over the marker occurrences; -2 = the last complete one).
``--tail-after PATTERN`` also reports the post-backward critical path: from the end of the last dispatch matching
PATTERN on the marker's stream before the next step's first forward GEMM, to the start of that forward GEMM.
"""
from __future__ import annotations

import argparse
import csv
import re


def short(n: str) -> str:
    n = n.strip().replace("(anonymous namespace)::", "")
    n = re.sub(r"\(.*\)$", "", n).replace("void ", "").replace("fan::gemm_detail::", "").replace("fan::", "")
    return n.replace("unsigned short", "bf16")[:100]


def load(path):
    rows = []
    if path.endswith(".db"):  # rocprofv3's default (rocpd sqlite) output: the `kernels` view
        import sqlite3

        con = sqlite3.connect(path)
        for name, t0, t1, sid, gx in con.execute("select name, start, end, stream_id, grid_x from kernels"):
            rows.append({"name": short(name), "t0": int(t0), "t1": int(t1), "stream": str(sid), "grid": gx})
        rows.sort(key=lambda x: x["t0"])
        return rows
    with open(path) as f:
        for r in csv.DictReader(f):
            if r.get("Kind", "KERNEL_DISPATCH") != "KERNEL_DISPATCH":
                continue
            rows.append({"name": short(r["Kernel_Name"]), "t0": int(r["Start_Timestamp"]), "t1": int(r["End_Timestamp"]),
                         "stream": r.get("Stream_Id", r.get("Queue_Id", "?")), "grid": r.get("Grid_Size_X", "")})
    rows.sort(key=lambda x: x["t0"])
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--marker", default="softmax_xent")
    ap.add_argument("--step", type=int, default=-2)
    ap.add_argument("--tail-after", default="gemm_pl4_kernel<false, false")
    a = ap.parse_args()
    rows = load(a.csv)
    marks = [i for i, r in enumerate(rows) if a.marker in r["name"]]
    if len(marks) < 3:
        raise SystemExit(f"fewer than 3 '{a.marker}' dispatches in the trace")
    k = a.step if a.step >= 0 else len(marks) - 1 + a.step
    i0, i1 = marks[k], marks[k + 1]
    base = rows[i0]["t0"]
    mstream = rows[i0]["stream"]
    print(f"# step {k}: {i1 - i0} dispatches between marker {i0} and {i1}; step period "
          f"{(rows[i1]['t0'] - base) / 1e3:.1f} us; offsets from the marker's start, us; s = HIP stream id")
    print(f"{'start':>9} {'dur':>8} {'s':>3}  kernel")
    for r in rows[i0:i1]:
        print(f"{(r['t0'] - base) / 1e3:9.1f} {(r['t1'] - r['t0']) / 1e3:8.1f} {r['stream']:>3}  {r['name']}")
    # post-backward critical path: last matching dispatch (the last bwd-weight GEMM) on the marker stream -> next
    # forward GEMM (the first gemm after it on that stream whose name is not a bwd-weight one)
    seg = rows[i0:i1 + 1]
    last = max((j for j, r in enumerate(seg) if a.tail_after in r["name"] and r["stream"] == mstream), default=None)
    if last is not None:
        nxt = next((j for j in range(last + 1, len(seg)) if seg[j]["name"].startswith("gemm")
                    and seg[j]["stream"] == mstream and a.tail_after not in seg[j]["name"]), None)
        if nxt is None:  # the next step's forward: search past the segment
            after = rows[i1 + 1:]
            nf = next((r for r in after if r["name"].startswith("gemm") and r["stream"] == mstream), None)
        else:
            nf = seg[nxt]
        if nf is not None:
            gap = (nf["t0"] - seg[last]["t1"]) / 1e3
            print(f"# post-backward critical path: end of the last '{a.tail_after}' dispatch -> next forward GEMM: "
                  f"{gap:.1f} us")


if __name__ == "__main__":
    main()
