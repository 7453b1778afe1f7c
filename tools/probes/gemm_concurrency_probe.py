"""Probe: do two independent backward GEMMs sharing the chip (each on half the CUs, desynchronised epilogues) beat
the two run back to back on the whole chip? The layer pairs of the flagship backward at MB 8192:
  layer 2: bwd-data 8192x4096x1024 (ReLU mask) + bwd-weight 4096x1024x8192 (f32)
  layer 1: bwd-data 8192x4096x4096 (ReLU mask) + bwd-weight 4096x4096x8192 (f32)
Arms (interleaved, median of 5 x 20 launches): sequential default plans; both on two streams with the persistent
grid capped at 128 workgroups each; plus each GEMM alone at 128 workgroups and at its best standalone plans."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from fpga_ai_nic_amd import _ext  # noqa: E402
from fpga_ai_nic_amd.ops import gemm as G  # noqa: E402


def t_us(fn, iters=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    C = _ext.require()
    M = 8192
    torch.manual_seed(0)
    dev = "cuda"
    s1 = torch.cuda.Stream()
    s2 = torch.cuda.Stream()
    main_s = torch.cuda.current_stream()
    out = []
    for name, cin, cout in (("layer2", 4096, 1024), ("layer1", 4096, 4096), ("layer0", 1024, 4096)):
        X = (torch.rand(M, cin, device=dev) * 2 - 1).to(torch.bfloat16)      # act[i] (ReLU input of bwd-data)
        dZ = ((torch.rand(M, cout, device=dev) * 2 - 1) * 0.01).to(torch.bfloat16)
        W = ((torch.rand(cin, cout, device=dev) * 2 - 1) * 0.02).to(torch.bfloat16)
        dX = torch.empty(M, cin, device=dev, dtype=torch.bfloat16)
        dW = torch.empty(cin, cout, device=dev, dtype=torch.float32)
        ws = torch.empty(8 * cin * cout + (1 << 20), device=dev, dtype=torch.float32)

        def bd(tile=None, sk=None):
            G.gemm(dZ, False, W, True, dX, G.EPI_RELU_MASK, aux=X, tile=tile, split_k=sk)

        def bw(tile=None, sk=None):
            G.gemm(X, True, dZ, False, dW, G.EPI_NONE, tile=tile, split_k=sk)

        def seq():
            bd()
            bw()

        def conc(bw_tile, bw_sk, cap_bd=128, cap_bw=128):
            def f():
                s1.wait_stream(main_s)
                s2.wait_stream(main_s)
                with torch.cuda.stream(s1):
                    C.gemm_set_persist(cap_bd)
                    bd()
                with torch.cuda.stream(s2):
                    C.gemm_set_persist(cap_bw)
                    bw(bw_tile, bw_sk)
                C.gemm_set_persist(256)
                main_s.wait_stream(s1)
                main_s.wait_stream(s2)
            return f

        def capped(fn, cap):
            def f():
                C.gemm_set_persist(cap)
                fn()
                C.gemm_set_persist(256)
            return f

        arms = {
            "bd_default": lambda: bd(),
            "bw_default": lambda: bw(),
            "seq_default": seq,
            "bd_cap128": capped(lambda: bd(), 128),
            "bw_256x128_sk1": lambda: bw((256, 128), 1),
            "bw_128x128_sk1": lambda: bw((128, 128), 1),
            "bw_256x256_sk2": lambda: bw((256, 256), 2),
            "conc_bw256x128": conc((256, 128), 1),
            "conc_bw256x256sk2": conc((256, 256), 2),
            "conc_bw128x128_cap": conc((128, 128), 1),
        }
        if name == "layer0":  # no bwd-data for the first layer: only the bwd-weight plans
            arms = {k: v for k, v in arms.items() if k.startswith("bw_")}
        tm = {k: [] for k in arms}
        for _ in range(5):
            for k, fn in arms.items():
                try:
                    tm[k].append(t_us(fn))
                except Exception as e:  # noqa: BLE001
                    tm[k].append(float("nan"))
                    print(json.dumps({"layer": name, "arm": k, "error": str(e)[:200]}), flush=True)
        rec = {"layer": name, "cin": cin, "cout": cout, "M": M,
               **{k: round(statistics.median(v), 2) for k, v in tm.items()},
               "plan_bd": C.gemm_plan(M, cin, cout, 0), "plan_bw": C.gemm_plan(cin, cout, M, 0)}
        print(json.dumps(rec), flush=True)
        out.append(rec)
    path = os.environ.get("PROBE_OUT")
    if path:
        with open(path, "w") as f:
            for r in out:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
