"""Where a K-tile of the one-role GEMM loop spends its cycles: s_memtime stamps (diagnostic build with
FAN_EXTRA_CFLAGS=-DFAN_GEMM_STAMPS). Per wave and K-tile: vmcnt wait, barrier, DMA issue, fragment-read issue,
then the MFMA section up to the next loop top. Median / p90 over the first 8 workgroups, all waves, K-tiles 1..62."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from fpga_ai_nic_amd.ops import gemm as G  # noqa: E402

Cx = G._ext.require()
WG, W, KT, P = 8, 8, 64, 5
buf = torch.zeros(WG * W * KT * P, dtype=torch.int64, device="cuda")
shapes = {"fwd1": (8192, 4096, 4096, False, False), "bwdd1": (8192, 4096, 4096, False, True),
          "bwdw1": (4096, 4096, 8192, True, False)}
for name, (M, N, K, a_t, b_t) in shapes.items():
    A = (torch.rand(K, M, device="cuda") * 2 - 1).bfloat16() if a_t else (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
    B = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16() if b_t else (torch.rand(K, N, device="cuda") * 2 - 1).bfloat16()
    C = torch.empty(M, N, device="cuda")
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
    nk = min(KT, K // 64)
    seg = {"vmcnt": t[:, :, 1:nk - 1, 1] - t[:, :, 1:nk - 1, 0], "barrier": t[:, :, 1:nk - 1, 2] - t[:, :, 1:nk - 1, 1],
           "dma_issue": t[:, :, 1:nk - 1, 3] - t[:, :, 1:nk - 1, 2], "read_issue": t[:, :, 1:nk - 1, 4] - t[:, :, 1:nk - 1, 3],
           "mfma_to_next_top": t[:, :, 2:nk, 0] - t[:, :, 1:nk - 1, 4]}
    tot = t[:, :, 2:nk, 0] - t[:, :, 1:nk - 1, 0]
    out = {k: {"median": int(np.median(v)), "p90": int(np.percentile(v, 90))} for k, v in seg.items()}
    out["ktile_total"] = {"median": int(np.median(tot)), "p90": int(np.percentile(tot, 90))}
    out["mfma_cycles_per_wave_ktile"] = 64 * 16 * (2 if True else 1) // 2
    print(name, f"{s.elapsed_time(e) * 1e3:.1f}us", json.dumps(out), flush=True)
