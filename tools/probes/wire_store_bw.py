"""Wide wire stores into the P2P receive arena: ``wire_pack_to`` (the direct transport's producer kernel, storing
each encoded shard into an uncached receive-arena slot, as it does into a peer's arena over xGMI) against
``wire_pack`` into ordinary device memory, same shards, same codec, interleaved rounds in one process.

Since round 3 every wire shard leaves a lane as 16-B vector stores: 16 mantissa bytes per lane and the exponents
of 16 lanes as one 16-B store (bfp_format.h WireLane16); before, each exponent byte was its own store. The
verdict's criterion: pack_to into the uncached arena >= 90 % of pack into HBM.

    python tools/probes/wire_store_bw.py [--elems 33554432] [--shards 8]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from fpga_ai_nic_amd import _ext  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--elems", type=int, default=32 << 20)
    ap.add_argument("--shards", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=7)
    a = ap.parse_args()
    C = _ext.require()
    torch.cuda.set_device(0)
    n_s = a.elems // a.shards // 256 * 256
    codec = 1  # bfp_rne
    sb = C.wire_shard_bytes(codec, n_s)
    x = (torch.randn(n_s * a.shards, device="cuda") * 3).to(torch.bfloat16)
    out = torch.empty(sb * a.shards, dtype=torch.uint8, device="cuda")
    comm = C.P2PComm(0, a.shards, 0, sb)  # world = shards: one arena slot pair per "peer"
    arena = comm.arena_view()
    dsts = [arena[q * 2 * ((sb + 255) // 256 * 256):][:sb] for q in range(a.shards)]
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]

    def t(fn, it=20):
        fn()
        ev[0].record()
        for _ in range(it):
            fn()
        ev[1].record()
        ev[1].synchronize()
        return ev[0].elapsed_time(ev[1]) / it * 1e3

    pack = lambda: C.wire_pack(x, out, n_s, codec)  # noqa: E731
    pack_to = lambda: C.wire_pack_to(x, dsts, n_s, codec)  # noqa: E731
    flat = arena[: sb * a.shards]
    wire_src = torch.randint(0, 255, (sb * a.shards,), dtype=torch.uint8, device="cuda")
    copy_in = lambda: flat.copy_(wire_src)  # noqa: E731  (torch copy kernel into the arena: store-path reference)
    modes = {"thread": 2, "block": 1, "none": 0}
    m0 = C.p2p_release_mode()
    tp, tc, tt = [], [], {k: [] for k in modes}
    for _ in range(a.rounds):
        tp.append(t(pack))
        tc.append(t(copy_in))
        for k, m in modes.items():
            C.set_p2p_release_mode(m)
            tt[k].append(t(pack_to))
    C.set_p2p_release_mode(m0)
    pack_to()
    torch.cuda.synchronize()
    same = all(torch.equal(out[q * sb:(q + 1) * sb], dsts[q]) for q in range(a.shards))
    byt = x.numel() * 2 + sb * a.shards  # bf16 read + wire written
    mp = statistics.median(tp)
    rec = {"probe": "wire_store_bw", "arena_memory": comm.arena_memory, "shard_elems": n_s, "shards": a.shards,
           "wire_bytes": sb * a.shards, "pack_hbm_us": round(mp, 2), "pack_hbm_GBps": round(byt / mp / 1e3, 1),
           "torch_copy_into_arena_us": round(statistics.median(tc), 2), "default_release": m0,
           "bit_identical": same}
    for k in modes:
        mt = statistics.median(tt[k])
        rec[f"pack_to_arena_{k}_us"] = round(mt, 2)
        rec[f"arena_vs_hbm_{k}"] = round(mp / mt, 3)
    # grid cap of the peer-storing kernels (one release per workgroup), default release form
    g0 = C.p2p_grid_cap()
    tg = {g: [] for g in (256, 512, 1024, 2048)}
    for _ in range(a.rounds):
        for g in tg:
            C.set_p2p_grid_cap(g)
            tg[g].append(t(pack_to))
    C.set_p2p_grid_cap(g0)
    rec["default_grid_cap"] = g0
    rec["pack_to_arena_block_us_by_grid_cap"] = {g: round(statistics.median(v), 2) for g, v in tg.items()}
    rec["arena_vs_hbm_by_grid_cap"] = {g: round(mp / statistics.median(v), 3) for g, v in tg.items()}
    print(json.dumps(rec), flush=True)
    return 0 if same else 1


if __name__ == "__main__":
    sys.exit(main())
