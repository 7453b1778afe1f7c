"""Probe: per-hop timing of the direct P2P ring (and the direct mesh) with N virtual ranks on ONE GPU.

N ranks in one process, each with its own P2PComm arena + flag block wired with ``P2PComm.connect_local`` (no IPC),
one host thread and one stream per rank (run with GPU_MAX_HW_QUEUES=32 so no rank's stream shares a hardware queue
with another's flag wait). Every rank all-reduces a SIZE-MB f32 gradient ITERS times with request tracing on; the
engine's per-round ring trace (credit wait / hop kernels / upstream-ready wait, csrc/comm/engine.cpp hop_mark) and
its phase split are printed per (algo, rings) as one JSON line (rank 0's view; ranks share one GPU, so the times are
those of N ranks time-sharing it, not of an xGMI ring).

    GPU_MAX_HW_QUEUES=32 python tools/probes/ring_hops_local.py --world 8 --size-mb 64
"""
import argparse
import json
import os
import sys
import threading
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from fpga_ai_nic_amd import _ext  # noqa: E402
from fpga_ai_nic_amd.parallel.native_engine import NativeAllReduce  # noqa: E402


def run(world, algo, rings, sub, n, iters, max_slice, prepacked):
    C = _ext.require()
    comms = [C.P2PComm(r, world, 0, 64 << 20, max(2, sub + 1)) for r in range(world)]
    C.P2PComm.connect_local(comms)
    engines = [NativeAllReduce(None, codec="bfp_rne", algo=algo, rings=rings, max_slice_elems=max_slice,
                               comm=comms[r], ring_sub=sub) for r in range(world)]
    out, errs = [None] * world, [None] * world
    bar = threading.Barrier(world)

    def body(r):
        try:
            torch.cuda.set_device(0)
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                eng = engines[r]
                L = eng.layout(n)
                g = torch.randn(L.n_pad, device="cuda") * 1e-3
                res = torch.zeros(L.n_pad, device="cuda")
                kw = {}
                if prepacked:
                    tgt = eng.prepack_target(g, n)
                    if tgt is not None:
                        C.wire_pack_range(g, tgt[0], tgt[1], 0, n, tgt[3])
                        kw["prepacked"] = (tgt[0], L.n_pad)
                eng.allreduce(g, res, n_valid=n, **kw).synchronize(120)  # warm (scratch, arena parities)
                s.synchronize()
                bar.wait()
                eng.trace(True)
                t0 = time.perf_counter()
                hs = [eng.allreduce(g, res, n_valid=n, **kw) for _ in range(iters)]
                for h in hs:
                    h.synchronize(120)
                s.synchronize()
                wall = time.perf_counter() - t0
                tr = eng.trace_summary()
                eng.trace(False)
                out[r] = (wall, tr, len(eng.orders), L.slice_elems, L.blocks)
        except Exception as e:  # noqa: BLE001
            errs[r] = repr(e)
            bar.abort()

    ts = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(300)
    if any(t.is_alive() for t in ts):
        raise RuntimeError("virtual rank hung")
    if any(errs):
        raise RuntimeError(str(errs))
    wall = max(o[0] for o in out)
    tr = out[0][1]
    rec = {"probe": "ring_hops_local", "world": world, "algo": algo, "rings": out[0][2], "sub": sub,
           "size_MB_f32": n * 4 / 2**20,
           "input": "prepacked" if prepacked else "f32", "iters": iters, "us_per_request": round(wall / iters * 1e6, 1),
           "comm_us_per_request": round(tr["comm_ms"] * 1e3 / max(1, tr["requests"]), 1)}
    if tr.get("hop_rounds"):
        k = tr["hop_rounds"]
        rec.update({"slice_elems": out[0][3], "blocks": out[0][4], "rounds_per_request": k // max(1, tr["requests"]),
                    "hop_credit_us": round(tr["hop_credit_ms"] * 1e3 / k, 2),
                    "hop_kernel_us": round(tr["hop_kernel_ms"] * 1e3 / k, 2),
                    "hop_ready_us": round(tr["hop_ready_ms"] * 1e3 / k, 2),
                    "hop_max_us": round(tr["hop_max_ms"] * 1e3, 2)})
    else:
        rec["phase_us"] = {p: round(tr[p] * 1e3 / max(1, tr["requests"]), 1)
                           for p in ("pack_ms", "exchange_ms", "reduce_ms", "gather_ms", "epilogue_ms")}
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--size-mb", type=float, default=64)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--max-slice", type=int, default=1 << 22)
    ap.add_argument("--arms", default="ring:1,ring:7,ring:7:3,mesh:1", help="algo:rings[:sub-slices per hop]")
    ap.add_argument("--prepacked", action="store_true")
    a = ap.parse_args()
    n = int(a.size_mb * (1 << 20)) // 4 // 16 * 16
    for arm in a.arms.split(","):
        f = arm.split(":")
        algo, rings, sub = f[0], int(f[1]), int(f[2]) if len(f) > 2 else 1
        print(json.dumps(run(a.world, algo, rings, sub, n, a.iters, a.max_slice, a.prepacked)), flush=True)


if __name__ == "__main__":
    main()
