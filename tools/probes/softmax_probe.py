"""Probe: the fused softmax + cross-entropy kernel at the flagship's logits (8192 x 1024 f32 -> bf16 dlogits) and at
the reference batch (1792 rows), us per call (median of 5 x 50 launches)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from fpga_ai_nic_amd.ops import nn as NN  # noqa: E402


def main():
    out = {}
    for M in (8192, 1792):
        C = 1024
        x = torch.randn(M, C, device="cuda") * 3
        y = torch.randint(0, C, (M,), device="cuda", dtype=torch.int32)
        d = torch.empty(M, C, device="cuda", dtype=torch.bfloat16)
        loss = torch.empty(M, device="cuda")
        ts = []
        for _ in range(5):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            NN.softmax_xent(x, y, d, loss, 1.0 / M)
            s.record()
            for _ in range(50):
                NN.softmax_xent(x, y, d, loss, 1.0 / M)
            e.record()
            torch.cuda.synchronize()
            ts.append(s.elapsed_time(e) / 50 * 1e3)
        out[f"M{M}"] = round(sorted(ts)[2], 2)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
