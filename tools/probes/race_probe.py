"""Locate the comm-stream-epilogue discrepancy: one training step per arm, per-layer diff of the updated master
weights vs the inline engine (count, max |diff|, first differing flat indices)."""
import sys

import torch

sys.path.insert(0, ".")
from fpga_ai_nic_amd.models.mlp import MLP  # noqa: E402
from fpga_ai_nic_amd.parallel.dp import DataParallelTrainer, make_engine  # noqa: E402
from fpga_ai_nic_amd.parallel.native_engine import NativeAllReduce  # noqa: E402
from fpga_ai_nic_amd.parallel.transport import NativeTransport, ThreadFabric  # noqa: E402


class _Store(dict):
    def set(self, k, v):
        self[k] = v

    def get(self, k):
        return self[k]


T = NativeTransport(rank=0, world=1, device=0, store=_Store(), force_collectives=True)
sizes, mb = [1024, 4096, 4096, 1024], 2048
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 1


def run(arm, sync_each=False):
    serialize = arm.endswith("_serial")
    arm = arm.replace("_serial", "")
    if arm == "inline":
        eng = make_engine(ThreadFabric(1).transport(0), "bfp", impl="native")
    else:
        eng = NativeAllReduce(T, codec="bfp_rne", force_comm=True)
        eng.epilogue_on_producer = arm == "producer"
    m = MLP(sizes, dtype=torch.bfloat16, device="cuda", seed=3, pad_fn=lambda n, e=eng: e.layout(n).n_pad)
    tr = DataParallelTrainer(m, eng, lr=0.05, prepack=arm != "comm_noprepack")
    if serialize:  # drain both streams before every backward GEMM: no comm/compute concurrency
        bw, bd = m.backward_weight, m.backward_data

        def bw_s(*a, **k):
            torch.cuda.synchronize()
            return bw(*a, **k)

        def bd_s(*a, **k):
            torch.cuda.synchronize()
            i = a[0]
            l = m.layers[i]
            SNAP.setdefault(arm, []).append((i, l.lp.float().cpu().clone(), l.master.cpu().clone(),
                                              m.dz[i + 1].float().cpu().clone()))
            return bd(*a, **k)
        m.backward_weight, m.backward_data = bw_s, bd_s
    g = torch.Generator().manual_seed(0)
    x = (torch.rand(mb, sizes[0], generator=g) * 2 - 1).to("cuda", torch.bfloat16)
    y = torch.randint(0, sizes[-1], (mb,), generator=g, dtype=torch.int32).cuda()
    for _ in range(steps):
        tr.step(x, y)
        if sync_each:
            tr.finish()
    tr.finish()
    torch.cuda.synchronize()
    return [l.master.cpu() for l in m.layers] + [d.float().cpu() for d in m.dz[1:]], [l.n for l in m.layers] + [0] * 3


SNAP = {}
ref, ns = run("inline")
for arm in (sys.argv[2].split(",") if len(sys.argv) > 2 else ("producer_serial", "comm_serial")):
    w, _ = run(arm)
    for i, (a, b) in enumerate(zip(w, ref)):
        d = (a - b).abs()
        nz = torch.nonzero(d).flatten()
        print(f"{arm:14s} {'master' if i < 3 else 'dz'} {i % 3 + (i >= 3)} n={ns[i]} n_pad={a.numel()} differing={nz.numel()} max={d.max().item():.3e} "
              f"first={nz[:6].tolist()} last={nz[-3:].tolist()}", flush=True)

for (i, lp_a, ms_a, dz_a), (j, lp_b, ms_b, dz_b) in zip(SNAP.get("producer", []), SNAP.get("comm", [])):
    print(f"before bwd-data of layer {i}: lp differs at {int((lp_a != lp_b).sum())}, master at "
          f"{int((ms_a != ms_b).sum())}, input dz at {int((dz_a != dz_b).sum())}", flush=True)
