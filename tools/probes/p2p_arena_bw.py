"""Arena memory type A/B for the direct P2P transport: streaming write / read bandwidth of this rank's receive arena
(the memory peers store into over xGMI and the consuming kernels read), per FAN_P2P_MEM=uncached|fine|coarse,
against ordinary device memory. One process, no flags."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from fpga_ai_nic_amd import _ext  # noqa: E402

C = _ext.require()
torch.cuda.set_device(0)
nbytes = 64 << 20
c = C.P2PComm(0, 1, 0, nbytes // 2)
arena = c.arena_view()[:nbytes]
src = torch.randint(0, 255, (nbytes,), dtype=torch.uint8, device="cuda")
dst = torch.empty_like(src)


def bw(fn, n=10):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return nbytes / ((time.perf_counter() - t0) / n) / 1e9


w = bw(lambda: arena.copy_(src))
r = bw(lambda: dst.copy_(arena))
base = bw(lambda: dst.copy_(src))
print(f"arena={c.arena_memory}: write {w:.0f} GB/s, read {r:.0f} GB/s (device->device copy {base:.0f} GB/s), "
      f"correct={bool(torch.equal(dst, src))}", flush=True)
