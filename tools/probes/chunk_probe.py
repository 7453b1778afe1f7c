"""Diagnose chunked-mesh training differences: forced 1-rank RCCL path, chunked vs unchunked, with and without the
GEMM-fused encode (prepack); reports which layers / elements differ after each step."""
import sys, os
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from fpga_ai_nic_amd.models.mlp import MLP
from fpga_ai_nic_amd.parallel.dp import DataParallelTrainer
from fpga_ai_nic_amd.parallel.native_engine import NativeAllReduce
from fpga_ai_nic_amd.parallel.transport import NativeTransport


class _Store(dict):
    def set(self, k, v): self[k] = v
    def get(self, k): return self[k]


T = NativeTransport(rank=0, world=1, device=0, store=_Store(), force_collectives=True)


def train(chunk, prepack, on_producer, steps, sync_each=True):
    eng = NativeAllReduce(T, codec="bfp_rne", force_comm=True, chunk_elems=chunk)
    eng.epilogue_on_producer = on_producer
    sizes = (1024, 4096, 4096, 1024)
    m = MLP(list(sizes), dtype=torch.bfloat16, device="cuda", seed=3, pad_fn=lambda n, e=eng: e.layout(n).n_pad)
    tr = DataParallelTrainer(m, eng, lr=0.05, prepack=prepack)
    g = torch.Generator().manual_seed(0)
    x = (torch.rand(512, sizes[0], generator=g) * 2 - 1).to("cuda", torch.bfloat16)
    y = torch.randint(0, sizes[-1], (512,), generator=g, dtype=torch.int32).cuda()
    out = []
    for _ in range(steps):
        tr.step(x, y)
        if sync_each:
            tr.finish()
            out.append([l.master[: l.n].cpu().clone() for l in m.layers])
    tr.finish()
    if not sync_each:
        out.append([l.master[: l.n].cpu().clone() for l in m.layers])
    return out, [eng.layout(l.n) for l in m.layers]


for prepack in (False, True):
    for onp in (True, False):
        a, la = train(0, prepack, onp, 3, sync_each=False)
        b, lb = train(1 << 20, prepack, onp, 3, sync_each=False)
        print(f"prepack={prepack} on_producer={onp} chunks={[L.chunks for L in lb]}", flush=True)
        for s in range(len(a)):
            for i, (x, y) in enumerate(zip(a[s], b[s])):
                d = (x != y).nonzero().flatten()
                if len(d):
                    print(f"  step {s} layer {i}: {len(d)} differ, first at {d[:5].tolist()} shard={lb[i].shard}", flush=True)
        print("  done", flush=True)
