"""``mlp_mpi`` — the reference's training benchmark entry point, MI355X-native.

Positional signature kept from sw/mlp_mpi_example_f32.cpp:270-320::

    python -m fpga_ai_nic_amd.cli.mlp_mpi iters MB fuse_type type bn bk bc C1 C2 ... CN [--named flags]

``MB`` is the GLOBAL minibatch, split across ranks (sw:301). Launch one process per GPU, e.g.::

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m fpga_ai_nic_amd.cli.mlp_mpi \
        20 5376 0 A 32 32 32 2048 2048 2048 2048 2048 2048 2048 2048 2048 2048 2048 --dtype f32

(the reference run.sh workload: 10 FC layers of 2048, global MB 5376). ``type``: 'A' FWD+BWD+UPD (the
reference's live path), 'F' forward only, 'B' backward+all-reduce/UPD only (the reference's commented-out
modes, sw:543-680, with their GFLOP formulas and PERFDUMP,FP / PERFDUMP,BP lines). ``fuse_type`` selects the
layer epilogue fused into the GEMMs exactly as the reference maps it (sw:479-489): 0 none, 1 bias,
2 ReLU (with mask), 3 bias+ReLU, 4/5 fall back to none. ``--model-fuse hidden`` instead applies bias+ReLU to
the hidden layers only (the bench.py model).
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import torch

from ..config import add_named_flags, config_from_args
from ..models.mlp import MLP
from ..parallel.dp import DataParallelTrainer, make_engine
from ..parallel.transport import NativeTransport, P2PTransport, TorchDistTransport
from ..utils import checkpoint, dist as D, metrics


def build_parser():
    ap = argparse.ArgumentParser(prog="mlp_mpi", description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("iters", type=int, nargs="?", default=10)
    ap.add_argument("MB", type=int, nargs="?", default=32)
    ap.add_argument("fuse_type", type=int, nargs="?", default=0)
    ap.add_argument("type", nargs="?", default="A")
    ap.add_argument("bn", type=int, nargs="?", default=64)
    ap.add_argument("bk", type=int, nargs="?", default=64)
    ap.add_argument("bc", type=int, nargs="?", default=64)
    ap.add_argument("C", type=int, nargs="*")
    ap.add_argument("--dump-norms", action="store_true",
                    help="after training print the L1 norm of every layer's weight gradient (the reference's "
                         "disabled libxsmm_matdiff block, sw:818-826)")
    ap.add_argument("--verify-fwd", action="store_true",
                    help="check one forward of the trained model against an fp32 PyTorch reference (matdiff)")
    ap.add_argument("--model-fuse", default="ref", choices=["ref", "hidden"],
                    help="ref: fuse_type semantics on every layer; hidden: bias+ReLU on hidden layers only")
    return add_named_flags(ap)


def make_data(mb_local: int, c_in: int, n_classes: int, rank: int, seed: int, device, dtype):
    g = torch.Generator().manual_seed(seed * 1000003 + rank)
    x = (torch.rand(mb_local, c_in, generator=g) * 2 - 1).to(device=device, dtype=dtype)
    y = torch.randint(0, n_classes, (mb_local,), generator=g, dtype=torch.int32).to(device)
    return x, y


def run(argv=None, out=sys.stdout):
    a = build_parser().parse_args(argv)
    if a.type not in ("A", "F", "B"):
        raise SystemExit("type needs to be 'A' (ALL), 'F' (FWD) or 'B' (BWD)")
    if a.fuse_type not in (0, 1, 2, 3, 4, 5):
        raise SystemExit("fuse_type needs to be 0..5")
    sizes = a.C if a.C else [1024, 4096, 4096, 1024]
    if len(sizes) < 2:
        raise SystemExit("need at least two feature sizes C1 C2")
    cfg = config_from_args(a, sizes)
    cfg.iters, cfg.global_mb = a.iters, a.MB

    backend = "gloo" if cfg.device == "cpu" else None
    rank, world, local, device = D.init_distributed(backend, cfg.timeout_s)
    if cfg.device == "cpu":
        device = torch.device("cpu")
    if cfg.global_mb % world:
        raise SystemExit(f"global MB {cfg.global_mb} not divisible by world size {world}")
    mb = cfg.global_mb // world
    dtype = torch.bfloat16 if cfg.dtype == "bf16" else torch.float32

    transport = None
    if world > 1 or cfg.compress not in ("local",):
        if world > 1:
            if cfg.transport == "p2p" and device.type == "cuda":
                transport = P2PTransport()
            else:
                transport = NativeTransport() if cfg.transport == "native" else TorchDistTransport()
        else:
            from ..parallel.transport import ThreadFabric

            transport = ThreadFabric(1).transport(0)
    kind = cfg.compress if transport is not None else "local"
    impl = cfg.engine if device.type == "cuda" else "python"
    engine = make_engine(transport, kind, rounding=cfg.rounding, algo=cfg.algo, rings=cfg.rings,
                         max_slice_elems=cfg.slice_elems, compat_owner_fp32=cfg.compat_owner_fp32,
                         timeout_s=cfg.timeout_s, impl=impl,
                         comm=transport.comm if isinstance(transport, P2PTransport) and impl == "native" else None)
    pad_fn = (lambda n: engine.layout(n).n_pad) if engine is not None else None
    if a.model_fuse == "hidden":
        bias, relu = True, "hidden"
    else:  # reference fuse_type mapping (sw:479-489)
        bias, relu = {1: (True, "none"), 2: (False, "all"), 3: (True, "all")}.get(a.fuse_type, (False, "none"))
    model = MLP(sizes, dtype=dtype, device=device, pad_fn=pad_fn, seed=cfg.seed, momentum=cfg.momentum > 0,
                bias=bias, relu=relu)
    if world > 1:  # reference C3/C4: broadcast weights + bias from rank 0
        for l in model.layers:
            transport.broadcast_(l.master, 0)
        model.sync_lp()
    start_iter = 0
    if cfg.resume:
        start_iter = int(checkpoint.load(cfg.resume, model).get("iteration", 0))
    trainer = DataParallelTrainer(model, engine, lr=cfg.lr, weight_decay=cfg.weight_decay, momentum=cfg.momentum,
                                  loss_scale=cfg.loss_scale, profile=cfg.profile)
    x, y = make_data(mb, sizes[0], sizes[-1], rank, cfg.seed, device, dtype)
    threads = int(os.environ.get("OMP_NUM_THREADS", "1"))
    check = abs(float(os.environ.get("CHECK", "1") or 1))  # reference: env CHECK (sw:227-228)
    if rank == 0:
        print(" ".join(str(v) for v in (argv if argv is not None else sys.argv[1:])), file=out)
        print(metrics.setup_banner(sizes, cfg.global_mb, cfg.iters, threads, 2 if dtype == torch.bfloat16 else 4,
                                   show_threads=check == 0), file=out)
    def one_iter():
        if a.type == "A":
            trainer.step(x, y)
        elif a.type == "F":  # forward + loss forward (the fused softmax-xent kernel also emits dlogits)
            trainer.forward_pass(x)
            model.loss_backward(y, grad_scale=cfg.loss_scale / mb)
        else:  # 'B': loss bwd + backward + all-reduce/UPD on the activations of one forward
            trainer.backward_pass(y)

    if a.type == "B":
        trainer.forward_pass(x)
    for _ in range(cfg.warmup):
        one_iter()
    trainer.finish()
    trainer.times = {k: 0 if k == "steps" else 0.0 for k in trainer.times}
    D.barrier()
    t0 = time.perf_counter()
    for _ in range(cfg.iters):
        one_iter()
    loss_rows = model.loss_rows
    trainer.finish()
    D.barrier()
    total = D.max_over_ranks(time.perf_counter() - t0)
    loss = float(loss_rows.float().mean().item())
    if rank == 0:
        print(metrics.result_report(sizes, cfg.global_mb, mb, cfg.iters, total, threads,
                                    trainer.times if cfg.profile else None, kind=a.type), file=out)
        print(f"LOSS = {loss:.6g}", file=out)
        if engine is not None:
            print(f"ALLREDUCE: algo={engine.algo} codec={engine.codec} rings={engine.rings} "
                  f"wire_bytes/step={engine.stats['wire_bytes'] / max(1, engine.stats['requests']) * model.L:.4g}",
                  file=out)
            if cfg.profile and hasattr(engine, "counters"):
                # the NIC's host-stall register (get_host_stall_cycles, sw/mlp_mpi_example_f32.cpp:108-112)
                c = engine.counters()
                print(f"ALLREDUCE host wait = {c['host_wait_s'] / max(1, cfg.iters):.6g} s/iter "
                      f"({c['host_waits']} blocking waits, {c['requests']} requests)", file=out)
    if a.dump_norms and rank == world - 1:  # the reference prints from the last rank
        for i, l in enumerate(model.layers):
            print(f"L1 of layer's {i} dweights after training : {float(l.gw.double().abs().sum()):.25g}", file=out)
    if a.verify_fwd and rank == 0:
        xs = x[: min(64, x.shape[0])]
        got = model.forward(xs).float().cpu()
        h = xs.float()
        for i, l in enumerate(model.layers):
            h = h @ l.w.float() + (l.b.float() if model.bias else 0)
            if model._relu_at(i):
                h = torch.relu(h)
        nd = metrics.matdiff(h.cpu().numpy(), got.numpy())
        print("VERIFY fwd vs fp32 reference: " + " ".join(f"{k}={v:.6g}" for k, v in nd.items()), file=out)
    sink = metrics.JsonlSink(cfg.metrics_jsonl if rank == 0 else None)
    sink.write(kind="mlp_mpi", sizes=sizes, global_mb=cfg.global_mb, world=world, iters=cfg.iters,
               s_per_iter=total / max(cfg.iters, 1), samples_per_s=cfg.global_mb * cfg.iters / total, loss=loss,
               config=cfg.to_dict())
    if cfg.checkpoint:
        # a sharded-update engine leaves each rank's master / momentum current only on the shards it owns: gather them
        # first (collective, every rank; a no-op for the other engines)
        trainer.gather_state()
    if cfg.checkpoint and rank == 0:
        checkpoint.save(cfg.checkpoint, model, iteration=start_iter + cfg.warmup + cfg.iters, dtype=cfg.dtype,
                        meta={"bn": a.bn, "bk": a.bk, "bc": a.bc, "world": world})
    D.cleanup()
    return {"loss": loss, "s_per_iter": total / max(cfg.iters, 1), "model": model}


def main():
    run()


if __name__ == "__main__":
    main()
