"""Where a K-tile of the pipelined GEMM loop spends its cycles: s_memtime stamps (diagnostic build with
FAN_EXTRA_CFLAGS=-DFAN_GEMM_STAMPS, see gemm_bf16_kernel.h). Per wave and K-tile: k-step-0 block issue (32 MFMAs +
reads), the vmcnt/lgkmcnt wait, the barrier, k-step-1 block issue (32 MFMAs + reads + DMA). Median / p90 over the
first 8 workgroups, all waves, K-tiles 1..nk-2."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from fpga_ai_nic_amd.ops import gemm as G  # noqa: E402

Cx = G._ext.require()
WG, W, KT, P = 8, 8, 64, 5  # waves: up to 8 (the 4-wave kernel fills 4)
buf = torch.zeros(WG * W * KT * P, dtype=torch.int64, device="cuda")
shapes = {"fwd1": (8192, 4096, 4096, False, False), "bwdd1": (8192, 4096, 4096, False, True),
          "bwdw1": (4096, 4096, 8192, True, False),
          # bf16 outputs: the flagship's persistent loop with overlapped tile transitions (pl4_run OVL)
          "fwd1_bf16": (8192, 4096, 4096, False, False, torch.bfloat16),
          "bwdd1_bf16": (8192, 4096, 4096, False, True, torch.bfloat16)}
for name, (M, N, K, a_t, b_t, *dt) in shapes.items():
    A = (torch.rand(K, M, device="cuda") * 2 - 1).bfloat16() if a_t else (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
    B = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16() if b_t else (torch.rand(K, N, device="cuda") * 2 - 1).bfloat16()
    C = torch.empty(M, N, device="cuda", dtype=dt[0] if dt else torch.float32)
    for _ in range(5):
        G.gemm(A, a_t, B, b_t, C)
    buf.zero_()
    Cx.gemm_set_stamp_buffer(buf)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    G.gemm(A, a_t, B, b_t, C)
    e.record()
    torch.cuda.synchronize()
    Cx.gemm_set_stamp_buffer(None)
    t = buf.view(WG, W, KT, P).cpu().numpy().astype(np.int64)
    t = t[:, [w for w in range(W) if t[:, w].any()]]  # the waves the kernel has (4 or 8)
    nk = min(KT, K // 64)
    r = slice(1, nk - 2)
    r2 = slice(2, nk - 1)
    seg = {"ks0_block": t[:, :, r, 1] - t[:, :, r, 0], "wait": t[:, :, r, 2] - t[:, :, r, 1],
           "barrier": t[:, :, r, 3] - t[:, :, r, 2], "ks1_block": t[:, :, r, 4] - t[:, :, r, 3],
           "to_next_top": t[:, :, r2, 0] - t[:, :, r, 4]}
    tot = t[:, :, r2, 0] - t[:, :, r, 0]
    out = {k: {"median": int(np.median(v)), "p90": int(np.percentile(v, 90))} for k, v in seg.items()}
    out["ktile_total"] = {"median": int(np.median(tot)), "p90": int(np.percentile(tot, 90))}
    out["mfma_cycles_per_simd_ktile"] = 2 * 64 * 16
    print(name, f"{s.elapsed_time(e) * 1e3:.1f}us", json.dumps(out), flush=True)
