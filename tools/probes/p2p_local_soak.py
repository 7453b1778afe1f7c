"""Soak of the direct P2P schedules with N virtual ranks in one process (P2PComm.connect_local on one GPU), verify
mode on: R requests per schedule through the production path (prepacked input, direct rounds), every result
compared bit for bit with the spec simulator. Usage: p2p_local_soak.py [world] [requests]. One JSON line per
schedule: requests, verified messages, mismatching requests."""
import json
import os
import sys
import threading

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from fpga_ai_nic_amd import _ext  # noqa: E402
from fpga_ai_nic_amd.parallel import sim  # noqa: E402
from fpga_ai_nic_amd.parallel.native_engine import NativeAllReduce  # noqa: E402


def soak(world, algo, rings, sub, requests, m=200000):
    C = _ext.require()
    comms = [C.P2PComm(r, world, 0, 8 << 20, 4) for r in range(world)]
    C.P2PComm.connect_local(comms)
    engines = [NativeAllReduce(None, codec="bfp_rne", algo=algo, rings=rings, max_slice_elems=1 << 14, comm=comms[r],
                               verify=True, ring_sub=sub) for r in range(world)]
    L = engines[0].layout(m)
    bad = [0] * world
    errs = [None] * world
    ref_cache = {}

    def ref_for(it, grads):
        if it not in ref_cache:
            gin = [np.pad(x, (0, L.n_pad - m)) for x in grads]
            ref_cache[it] = (sim.mesh_allreduce(gin, L.shard) if algo == "mesh" else
                             sim.ring_allreduce(gin, engines[0].orders, L.slice_elems, L.blocks)[0])[:m]
        return ref_cache[it]

    barrier = threading.Barrier(world)

    def run(r):
        try:
            torch.cuda.set_device(0)
            s = torch.cuda.Stream()
            eng = engines[r]
            with torch.cuda.stream(s):
                for it in range(requests):
                    rng = np.random.default_rng(1000 + it)
                    grads = [(rng.standard_normal(m) * 2.0 ** rng.integers(-8, 4)).astype(np.float32)
                             for _ in range(world)]
                    g = torch.zeros(L.n_pad, device="cuda")
                    g[:m] = torch.from_numpy(grads[r]).cuda()
                    buf, shard, own, cid = eng.prepack_target(g, m)[:4]
                    C.wire_pack_range(g, buf, shard, 0, m // 16 * 16, cid)
                    out = torch.zeros(L.n_pad, device="cuda")
                    eng.allreduce(g, out, n_valid=m, prepacked=(buf, m // 16 * 16)).synchronize(60)
                    s.synchronize()
                    if it % 10 == 0 or it == requests - 1:  # the simulator is the slow part: every 10th request
                        barrier.wait()
                        if r == 0:
                            ref_for(it, grads)
                        barrier.wait()
                        if not np.array_equal(out.cpu().numpy()[:m], ref_cache[it]):
                            bad[r] += 1
        except Exception as e:  # noqa: BLE001
            errs[r] = repr(e)[:300]
            barrier.abort()

    ts = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(600)
    hung = any(t.is_alive() for t in ts)
    cn = [e.counters() for e in engines] if not hung else []
    return {"world": world, "algo": algo, "rings": len(engines[0].orders) if algo == "ring" else 1, "ring_sub": sub,
            "requests": requests, "checked_requests": len(ref_cache), "mismatching_rank_requests": sum(bad),
            "verified_messages": sum(c["verified_rows"] for c in cn), "direct_rounds": sum(c["direct_rounds"] for c in cn),
            "errors": [e for e in errs if e], "hung": hung}


def main():
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    requests = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    for algo, rings, sub in (("mesh", 1, 1), ("ring", world - 1, 1), ("ring", world - 1, 3)):
        print(json.dumps(soak(world, algo, rings, sub, requests)), flush=True)


if __name__ == "__main__":
    main()
