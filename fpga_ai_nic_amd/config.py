"""Typed run configuration (replaces the reference's positional CLI + compile-time constants).

Reference knobs and where they went:
  iters / MB / fuse_type / type / bn bk bc / C1..CN  -> positional CLI, kept (sw/mlp_mpi_example_f32.cpp:270-320)
  NUM_NODES=3 (sw:38)                               -> world size from the launcher (any N >= 1)
  `BFP_EN (hw/all_reduce.sv:13)                     -> compress = bfp | raw | rccl | local
  NUM_FP=16, MANT_SIZE=8 (hw/bfp_adapter.sv:34-36)   -> fixed wire format; rounding = rne | trunc (bit-exact ref)
  BUF_SIZE=512 CL slice (hw/all_reduce.sv:102)      -> slice_elems (ring)
  lr 0.1 hard-coded (hw/weight_update.sv:444)        -> lr, momentum, weight_decay
  loss_weight 0.1 (sw:250)                           -> loss_scale
"""
from __future__ import annotations

import argparse
import dataclasses
from dataclasses import dataclass, field


@dataclass
class TrainConfig:
    iters: int = 10
    global_mb: int = 32
    fuse_type: int = 0
    type: str = "A"
    bn: int = 64
    bk: int = 64
    bc: int = 64
    sizes: list = field(default_factory=lambda: [1024, 4096, 4096, 1024])
    dtype: str = "bf16"            # bf16 | f32
    compress: str = "bfp"          # bfp | raw | raw_bf16 | rccl | local
    rounding: str = "rne"          # rne | trunc
    algo: str = "mesh"             # mesh | ring
    rings: int = 1
    slice_elems: int = 1 << 22
    transport: str = "torch"       # torch | native | p2p
    engine: str = "native"         # native (C++ engine, GPU) | python; CPU runs always use python
    compat_owner_fp32: bool = False
    lr: float = 0.1
    momentum: float = 0.0
    weight_decay: float = 0.0
    loss_scale: float = 1.0
    warmup: int = 2
    seed: int = 1
    profile: bool = False
    checkpoint: str = ""
    resume: str = ""
    metrics_jsonl: str = ""
    timeout_s: float = 600.0
    device: str = "auto"           # auto | cpu | cuda

    def to_dict(self):
        return dataclasses.asdict(self)


def add_named_flags(ap: argparse.ArgumentParser):
    d = TrainConfig()
    ap.add_argument("--dtype", default=d.dtype, choices=["bf16", "f32"])
    ap.add_argument("--compress", default=d.compress, choices=["bfp", "raw", "raw_bf16", "rccl", "local"])
    ap.add_argument("--rounding", default=d.rounding, choices=["rne", "trunc"])
    ap.add_argument("--algo", default=d.algo, choices=["mesh", "ring"])
    ap.add_argument("--rings", type=int, default=d.rings)
    ap.add_argument("--slice-elems", type=int, default=d.slice_elems)
    ap.add_argument("--transport", default=d.transport, choices=["torch", "native", "p2p"])
    ap.add_argument("--engine", default=d.engine, choices=["python", "native"],
                    help="request path: Python-issued engine (any transport) or the C++ engine (GPU)")
    ap.add_argument("--compat-owner-fp32", action="store_true")
    ap.add_argument("--lr", type=float, default=d.lr)
    ap.add_argument("--momentum", type=float, default=d.momentum)
    ap.add_argument("--weight-decay", type=float, default=d.weight_decay)
    ap.add_argument("--loss-scale", type=float, default=d.loss_scale)
    ap.add_argument("--warmup", type=int, default=d.warmup)
    ap.add_argument("--seed", type=int, default=d.seed)
    ap.add_argument("--profile", action="store_true")
    ap.add_argument("--checkpoint", default="")
    ap.add_argument("--resume", default="")
    ap.add_argument("--metrics-jsonl", default="")
    ap.add_argument("--timeout-s", type=float, default=d.timeout_s)
    ap.add_argument("--device", default=d.device, choices=["auto", "cpu", "cuda"])
    return ap


def config_from_args(a, positional_sizes=None) -> TrainConfig:
    c = TrainConfig()
    for f in dataclasses.fields(TrainConfig):
        key = f.name
        if hasattr(a, key):
            setattr(c, key, getattr(a, key))
    if positional_sizes:
        c.sizes = list(positional_sizes)
    return c
