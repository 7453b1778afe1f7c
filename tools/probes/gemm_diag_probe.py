"""Probe: main-loop variants of a diagnostic build against the production build, one process each. With
FAN_DIAG_SO=<path to a _C.so built with FAN_EXTRA_CFLAGS=-D...> the probe loads that library as the extension
(e.g. -DFAN_GEMM_NODMA: the persistent 4-wave loop without its in-loop operand DMA; outputs are wrong, only the
time matters) and times the flagship's big GEMM shapes at their production plans. Prints one JSON line."""
import importlib.util
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
so = os.environ.get("FAN_DIAG_SO")
if so:  # the diagnostic library under the extension's module name, before anything imports the real one
    spec = importlib.util.spec_from_file_location("fpga_ai_nic_amd._C", so)
    mod = importlib.util.module_from_spec(spec)
    sys.modules["fpga_ai_nic_amd._C"] = mod
    spec.loader.exec_module(mod)
from fpga_ai_nic_amd.ops import gemm as G  # noqa: E402


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
    torch.manual_seed(0)
    out = {"build": os.path.basename(so) if so else "production"}
    M, N = 8192, 4096
    for K in (1024, 4096):
        A = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        B = (torch.rand(K, N, device="cuda") * 2 - 1).to(torch.bfloat16)
        Bt = B.t().contiguous()
        bias = (torch.rand(N, device="cuda") - 0.5).to(torch.bfloat16)
        Cb = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        Cf = torch.empty(M, N, device="cuda", dtype=torch.float32)
        for tag, fn in (("nn_bias_relu", lambda: G.gemm(A, False, B, False, Cb, G.EPI_BIAS_RELU, bias=bias)),
                        ("nt_f32", lambda: G.gemm(A, False, Bt, True, Cf, G.EPI_NONE)),
                        ("nn_f32", lambda: G.gemm(A, False, B, False, Cf, G.EPI_NONE))):
            out[f"{tag}_K{K}"] = round(statistics.median(t_us(fn) for _ in range(5)), 2)
    X = (torch.rand(8192, 4096, device="cuda") * 2 - 1).to(torch.bfloat16)
    dZ = (torch.rand(8192, 4096, device="cuda") * 2 - 1).to(torch.bfloat16)
    Cw = torch.empty(4096, 4096, device="cuda", dtype=torch.float32)
    out["tn_f32_4096x4096x8192"] = round(statistics.median(
        t_us(lambda: G.gemm(X, True, dZ, False, Cw, G.EPI_NONE)) for _ in range(5)), 2)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
