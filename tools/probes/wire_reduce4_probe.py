"""Probe: the lane-contiguous BFP reduce kernels (4 values per lane, FAN_WIRE_REDUCE4 / C.set_wire_reduce4) against
the one-group-per-lane form, in isolation: C.wire_reduce of 2 and 7 wire slots + a dense f32 local operand into a
re-encoded wire shard (the ring / owner reduce shape) at a 16.8 M-element shard, interleaved, median us; outputs
compared bit for bit. Prints one JSON line per slot count."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from fpga_ai_nic_amd import _ext  # noqa: E402
from fpga_ai_nic_amd.ops import wire  # noqa: E402


def t_us(fn, iters=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    C = _ext.require()
    codec = wire.codec_id("bfp_rne")
    n = 16781312
    sb = wire.shard_bytes("bfp_rne", n)
    g = torch.Generator(device="cuda").manual_seed(0)
    for n_slots in (2, 8):
        slots = torch.empty(n_slots * sb, dtype=torch.uint8, device="cuda")
        for r in range(n_slots):  # valid encodings in every slot
            x = torch.randn(n, device="cuda", generator=g)
            C.wire_reduce(x.view(torch.uint8)[:0].new_zeros(sb), 1, 0, x, slots[r * sb:(r + 1) * sb], None, n, codec)
        local = torch.randn(n, device="cuda", generator=g)
        outs = {e: torch.zeros(sb, dtype=torch.uint8, device="cuda") for e in (0, 1)}
        tm = {0: [], 1: []}
        for _ in range(7):
            for e in (0, 1):
                C.set_wire_reduce4(e)
                tm[e].append(t_us(lambda: C.wire_reduce(slots, n_slots, 0, local, outs[e], None, n, codec)))
        C.set_wire_reduce4(1)
        same = bool(torch.equal(outs[0], outs[1]))
        gb = ((n_slots - 1) * sb + n * 4 + sb) / 1e9
        print(json.dumps({"n_slots": n_slots, "elems": n, "group_per_lane_us": round(statistics.median(tm[0]), 2),
                          "lane4_us": round(statistics.median(tm[1]), 2), "bit_identical": same,
                          "lane4_TBps": round(gb / statistics.median(tm[1]) * 1e6 / 1e3, 2)}), flush=True)


if __name__ == "__main__":
    main()
