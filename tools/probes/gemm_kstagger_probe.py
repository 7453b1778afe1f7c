"""Probe: K-start stagger of the 4-wave 256x256 loops (gemm_set_kstagger / FAN_GEMM_KSTAGGER, kstagger_of in
csrc/gemm/gemm_bf16_kernel.h) against the unstaggered loop, at the flagship's GEMM shapes and layouts:
  fwd   8192x4096xK   A K-contiguous, B N-contiguous, bias+ReLU bf16
  bwdd  8192x4096xK   A, B K-contiguous (NT), ReLU-mask bf16
  bwdw  4096x4096x8192 A, B MN-contiguous, f32
K = 4096 and 1024. Codes: step | starts << 8 | selector << 16 (selector 0 row panel, 1 column panel, 2 both).
Interleaved, median of 5 x 20 launches, us; static plans (FAN_GEMM_TUNE=0 is set here)."""
import json
import os
import sys

os.environ.setdefault("FAN_GEMM_TUNE", "0")
import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from fpga_ai_nic_amd import _ext  # noqa: E402
from fpga_ai_nic_amd.ops import gemm as G  # noqa: E402

CODES = {"off": 0, "r4s2": 0x0402, "r8s1": 0x0801, "r8s4": 0x0804, "rc8s1": 0x20801, "rc8s4": 0x20804,
         "c8s2": 0x10802, "rc16s1": 0x21001}


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
    torch.manual_seed(0)
    M, N = 8192, 4096
    codes = CODES
    if os.environ.get("KSTG_CODES"):
        codes = {k: CODES[k] for k in os.environ["KSTG_CODES"].split(",")}
    out = []
    for K in (4096, 1024):
        X = ((torch.rand(M, K, device="cuda") * 2 - 1)).to(torch.bfloat16)
        W = ((torch.rand(K, N, device="cuda") * 2 - 1) * 0.02).to(torch.bfloat16)
        b = torch.zeros(N, device="cuda", dtype=torch.bfloat16)
        Y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        # bwd-data dX[M,N] = dZ[M,K] . Wb[N,K]^T masked by act[M,N] (the layer's W [cin][cout] given as [N][K])
        dZk = ((torch.rand(M, K, device="cuda") * 2 - 1) * 0.01).to(torch.bfloat16)
        Wb = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.02).to(torch.bfloat16)
        act = (torch.rand(M, N, device="cuda") - 0.5).to(torch.bfloat16)
        dX = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        shapes = {
            "fwd": lambda: G.gemm(X, False, W, False, Y, G.EPI_BIAS_RELU, bias=b),
            "bwdd": lambda: G.gemm(dZk, False, Wb, True, dX, G.EPI_RELU_MASK, aux=act),
        }
        if K == 4096:  # bwd-weight dW[4096,4096] = Xt[8192,4096]^T . dZ[8192,4096]
            dZ = ((torch.rand(M, N, device="cuda") * 2 - 1) * 0.01).to(torch.bfloat16)
            dW = torch.empty(K, N, device="cuda", dtype=torch.float32)
            Xt = ((torch.rand(M, K, device="cuda") * 2 - 1)).to(torch.bfloat16)
            shapes["bwdw"] = lambda: G.gemm(Xt, True, dZ, False, dW, G.EPI_NONE)
        res = {f"{s}_{c}": [] for s in shapes for c in codes}
        ref = {}
        for rnd in range(5):
            for s, fn in shapes.items():
                for c, code in codes.items():
                    C.gemm_set_kstagger(code)
                    res[f"{s}_{c}"].append(t_us(fn))
                    if rnd == 0:  # numerics: staggered results stay within rounding of the unstaggered ones
                        o = {"fwd": Y, "bwdd": dX}.get(s)
                        if s == "bwdw":
                            o = dW
                        v = o.float().clone()
                        if c == "off":
                            ref[s] = v
                        else:
                            d = (v - ref[s]).abs().max().item()
                            sc = ref[s].abs().max().item()
                            if d > 0.02 * sc:
                                print(json.dumps({"K": K, "shape": s, "code": c, "MISMATCH": d, "scale": sc}),
                                      flush=True)
        C.gemm_set_kstagger(0)
        rec = {"M": M, "N": N, "K": K, **{k: round(sorted(v)[2], 2) for k, v in res.items()}}
        print(json.dumps(rec), flush=True)
        out.append(rec)
    path = os.environ.get("PROBE_OUT")
    if path:
        with open(path, "w") as f:
            for r in out:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
