"""What the fused epilogues cost on the MLP's bwd-data / forward GEMMs at MB 8192: the same GEMM timed with a bf16
output and no epilogue, with the ReLU-mask epilogue (reads the bf16 activation), and with bias+ReLU. (A packed 1-bit mask variant, written
by the forward and read by bwd-data, measured slower: profiles/r2_epi_cost_bits_probe.jsonl.) One process, arms interleaved per round, median of rounds."""
from __future__ import annotations

import json
import statistics
import sys

import torch

sys.path.insert(0, ".")
from fpga_ai_nic_amd.ops import gemm as G  # noqa: E402


def t(fn, iters=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000 / iters


def main():
    mb = 8192
    dev = "cuda"
    bf = torch.bfloat16
    shapes = [("bwdd1", mb, 4096, 4096, True), ("bwdd2", mb, 4096, 1024, True), ("fwd1", mb, 4096, 4096, False)]
    for name, M, N, K, b_t in shapes:
        A = (torch.rand(M, K, device=dev) * 2 - 1).to(bf)
        B = ((torch.rand(N, K, device=dev) if b_t else torch.rand(K, N, device=dev)) * 2 - 1).to(bf)
        C = torch.empty(M, N, device=dev, dtype=bf)
        aux = (torch.rand(M, N, device=dev) - 0.5).to(bf)
        bias = (torch.rand(N, device=dev) - 0.5).to(bf)
        arms = {"none_bf16": lambda: G.gemm(A, False, B, b_t, C, G.EPI_NONE),
                "relu_mask": lambda: G.gemm(A, False, B, b_t, C, G.EPI_RELU_MASK, aux=aux),
                "bias_relu": lambda: G.gemm(A, False, B, b_t, C, G.EPI_BIAS_RELU, bias=bias)}
        res = {k: [] for k in arms}
        for _ in range(7):
            for k, fn in arms.items():
                res[k].append(t(fn))
        print(json.dumps({"shape": name, "M": M, "N": N, "K": K,
                          **{k: round(statistics.median(v), 2) for k, v in res.items()}}), flush=True)


if __name__ == "__main__":
    main()
