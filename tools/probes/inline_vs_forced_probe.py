"""Forced 1-rank multi-rank path vs the inline world-1 engine on the flagship MLP: which layers / elements differ
after each of 3 steps, per minibatch (bit-identical training is the contract)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from fpga_ai_nic_amd.models.mlp import MLP  # noqa: E402
from fpga_ai_nic_amd.parallel.dp import DataParallelTrainer, make_engine  # noqa: E402
from fpga_ai_nic_amd.parallel.native_engine import NativeAllReduce  # noqa: E402
from fpga_ai_nic_amd.parallel.transport import NativeTransport, ThreadFabric  # noqa: E402


class _Store(dict):
    def set(self, k, v): self[k] = v
    def get(self, k): return self[k]


T = NativeTransport(rank=0, world=1, device=0, store=_Store(), force_collectives=True)


def train(forced, mb, steps, chunk=0, sync_each=True, on_producer=True):
    eng = NativeAllReduce(T, codec="bfp_rne", force_comm=True, chunk_elems=chunk) if forced else \
        make_engine(ThreadFabric(1).transport(0), "bfp", impl="native")
    if forced:
        eng.epilogue_on_producer = on_producer
    sizes = (1024, 4096, 4096, 1024)
    m = MLP(list(sizes), dtype=torch.bfloat16, device="cuda", seed=3, pad_fn=lambda n, e=eng: e.layout(n).n_pad)
    tr = DataParallelTrainer(m, eng, lr=0.05)
    g = torch.Generator().manual_seed(0)
    x = (torch.rand(mb, sizes[0], generator=g) * 2 - 1).to("cuda", torch.bfloat16)
    y = torch.randint(0, sizes[-1], (mb,), generator=g, dtype=torch.int32).cuda()
    out = []
    for _ in range(steps):
        tr.step(x, y)
        if sync_each:
            tr.finish()
            out.append([l.master[: l.n].cpu().clone() for l in m.layers])
    tr.finish()
    if not sync_each:
        out.append([l.master[: l.n].cpu().clone() for l in m.layers])
    return out


SYNC = os.environ.get("PROBE_SYNC", "1") == "1"
for mb in (512, 2048):
    for chunk in (0, 1 << 20):
      for onp in (True, False):
       for rep in range(2):
        a = train(False, mb, 3, sync_each=SYNC)
        b = train(True, mb, 3, chunk, sync_each=SYNC, on_producer=onp)
        print(f"mb={mb} chunk={chunk} on_producer={onp} rep={rep} sync_each={SYNC}", flush=True)
        for s in range(len(a)):
            for i, (x, y) in enumerate(zip(a[s], b[s])):
                d = (x != y).nonzero().flatten()
                if len(d):
                    print(f"  step {s} layer {i}: {len(d)} differ, first {d[:6].tolist()} max|diff| "
                          f"{(x - y).abs().max().item():.3g}", flush=True)
