"""GEMM time with a few CUs held by concurrent kernels (the comm stream's collectives at world > 1), one-tile-per-
workgroup launch vs persistent work-queue launch (gemm_set_persist). Hog = N single-wave spin kernels on
high-priority side streams, launched right before each GEMM: each makes its CU unable to host a GEMM workgroup
while it runs. Arms are interleaved per repetition; medians of per-call event timings."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from fpga_ai_nic_amd.ops import gemm as G  # noqa: E402

torch.manual_seed(0)
dev = "cuda"
Cx = G._ext.require()
shapes = {"fwd0": (8192, 4096, 1024, False, False), "bwdd2": (8192, 4096, 1024, False, True),
          "bwdd1": (8192, 4096, 4096, False, True), "fwd1": (8192, 4096, 4096, False, False),
          "sq8k": (8192, 8192, 8192, False, True)}
hogs = [torch.cuda.Stream(priority=-1) for _ in range(32)]
CYC = int(os.environ.get("HOG_CYCLES", "100000"))


def one(fn, nhog):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for i in range(nhog):
        with torch.cuda.stream(hogs[i]):
            torch.cuda._sleep(CYC)
    s.record()
    fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3


for name, (M, N, K, a_t, b_t) in shapes.items():
    A = (torch.rand(K, M, device=dev) * 2 - 1).bfloat16() if a_t else (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
    B = (torch.rand(N, K, device=dev) * 2 - 1).bfloat16() if b_t else (torch.rand(K, N, device=dev) * 2 - 1).bfloat16()
    C = torch.empty(M, N, device=dev)
    fn = lambda: G.gemm(A, a_t, B, b_t, C)  # noqa: E731
    for p in (False, True):
        Cx.gemm_set_persist(p)
        for _ in range(5):
            fn()
    torch.cuda.synchronize()
    t = {}
    for _ in range(15):
        for p in (False, True):
            Cx.gemm_set_persist(p)
            for nhog in (0, 16):
                t.setdefault(f"{'persist' if p else 'grid'}_hog{nhog}", []).append(one(fn, nhog))
    Cx.gemm_set_persist(False)
    print(name, json.dumps({k: round(statistics.median(v), 1) for k, v in t.items()}), flush=True)
