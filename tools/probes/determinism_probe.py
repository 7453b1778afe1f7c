"""Run-to-run determinism of the trainer over the engine paths (same seeds, fresh engine + model per run):
prints per-run losses and whether weights are bit-identical to the first run of the same arm."""
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


def run(arm, sizes, mb):
    if arm == "inline":
        eng = make_engine(ThreadFabric(1).transport(0), "bfp", impl="native")
    else:
        eng = NativeAllReduce(T, codec="bfp_rne", force_comm=True)
        eng.epilogue_on_producer = arm == "producer"
    m = MLP(sizes, dtype=torch.bfloat16, device="cuda", seed=3, pad_fn=lambda n, e=eng: e.layout(n).n_pad)
    tr = DataParallelTrainer(m, eng, lr=0.05)
    g = torch.Generator().manual_seed(0)
    x = (torch.rand(mb, sizes[0], generator=g) * 2 - 1).to("cuda", torch.bfloat16)
    y = torch.randint(0, sizes[-1], (mb,), generator=g, dtype=torch.int32).cuda()
    losses = [tr.step(x, y).float().mean().item() for _ in range(4)]
    tr.finish()
    torch.cuda.synchronize()
    return losses, [l.master.cpu() for l in m.layers]


for sizes, mb in (([256, 512, 256, 128], 256), ([1024, 4096, 4096, 1024], 2048)):
    first = {}
    for rep in range(3):
        for arm in ("inline", "comm", "producer"):
            losses, w = run(arm, sizes, mb)
            ref = first.setdefault(arm, (losses, w))
            same = all(torch.equal(a, b) for a, b in zip(w, ref[1]))
            xarm = first.get("inline")
            same_inline = xarm is not None and all(torch.equal(a, b) for a, b in zip(w, xarm[1]))
            print(f"{sizes} rep {rep} {arm:8s} losses {[f'{v:.9f}' for v in losses]} same_as_rep0 {same} "
                  f"same_as_inline {same_inline}", flush=True)
