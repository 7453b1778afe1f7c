"""Sharded weight update (engine ``shard_update``, ZeRO-1 style): the owner of each mesh shard fuses its reduce with
the codec round trip + SGD of that shard, and the ranks all-gather the updated bf16 weights instead of the reduced
gradient (csrc/comm/engine.cpp run_mesh / run_mesh_direct, bfp_kernels.hip wire_reduce_sgd_kernel).

It must train bit-identically to the unsharded schedule (the reference applies the NIC's SGD to the reduced stream
every node receives, hw/weight_update.sv:433-452): per rank, the weights it writes (``lp``) equal the unsharded
engine's bf16 weights, and its master / momentum planes, once gathered from their owners (``gather_owned``), equal the
unsharded engine's — for N virtual ranks on one GPU over the direct P2P transport (N = 2, 3, 8; f32 and prepacked
input; momentum; a bucket whose valid length ends inside a shard) and over the copying loopback fabric, and for the
1-rank forced multi-rank path. Each P2P case runs in a child process with one hardware queue per stream (see
test_gpu_p2p_local.py)."""
import json
import os
import subprocess
import sys
import threading

import numpy as np
import pytest
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fpga_ai_nic_amd import _ext  # noqa: E402
from fpga_ai_nic_amd.parallel.native_engine import NativeAllReduce  # noqa: E402

pytestmark = pytest.mark.gpu


def _case(world, fabric, n=50000 - 48, momentum=0.9, steps=2):
    C = _ext.require()
    rng = np.random.default_rng(7 + world)
    w0 = rng.standard_normal(n).astype(np.float32)
    grads = [[(rng.standard_normal(n) * (1 + r)).astype(np.float32) for r in range(world)] for _ in range(steps)]

    def comms():
        if fabric == "p2p":
            cs = [C.P2PComm(r, world, 0, 2 << 20, 2) for r in range(world)]
            C.P2PComm.connect_local(cs)
            return cs
        f = C.LoopbackFabric(world, 60.0)
        return [f.comm(r) for r in range(world)]

    arms = {}
    for shard in (False, True):
        cs = comms()
        arms[shard] = ([NativeAllReduce(None, codec="bfp_rne", algo="mesh", comm=cs[r], shard_update=shard)
                        for r in range(world)], cs)
    assert all(e.shard_update for e in arms[True][0]) and not any(e.shard_update for e in arms[False][0])
    res = {False: [None] * world, True: [None] * world}
    errs = []

    def run(r):
        try:
            torch.cuda.set_device(0)
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                for shard in (False, True):
                    eng = arms[shard][0][r]
                    L = eng.layout(n)
                    w = torch.zeros(L.n_pad, device="cuda")
                    w[:n] = torch.from_numpy(w0).cuda()
                    lp = w.to(torch.bfloat16)
                    mom = torch.zeros(L.n_pad, device="cuda")
                    for k in range(steps):
                        g = torch.zeros(L.n_pad, device="cuda")
                        g[:n] = torch.from_numpy(grads[k][r]).cuda()
                        kw = {}
                        tgt = eng.prepack_target(g, n) if k == 1 else None
                        if tgt is not None:  # the producer's encoding as the input (second step)
                            C.wire_pack_range(g, tgt[0], tgt[1], 0, n // 16 * 16, tgt[3])
                            kw["prepacked"] = (tgt[0], n // 16 * 16)
                        out = torch.zeros_like(lp) if shard else lp  # the sharded request writes the NEXT buffer
                        h = eng.allreduce_sgd(g, w, out, mom, n_valid=n, lr=0.05, grad_scale=1.0 / world,
                                              momentum=momentum, weight_decay=1e-3, defer=True, **kw)
                        h.commit_after_current()
                        h.synchronize(60)
                        lp = out
                    s.synchronize()
                    eng.gather_owned(w, n)
                    eng.gather_owned(mom, n)
                    res[shard][r] = (w.cpu().numpy(), lp.float().cpu().numpy(), mom.cpu().numpy(),
                                     eng.counters()["sharded_updates"])
        except Exception as e:  # noqa: BLE001
            errs.append(f"rank {r}: {e!r}")

    ts = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(120)
    why = list(errs)
    if any(t.is_alive() for t in ts):
        why.append("virtual rank thread hung")
    if not why:
        for r in range(world):
            wa, la, ma, _ = res[False][r]
            wb, lb, mb, cnt = res[True][r]
            if cnt != steps:
                why.append(f"rank {r}: {cnt} sharded updates, expected {steps}")
            for name, a, b in (("master", wa, wb), ("weights", la, lb), ("momentum", ma, mb)):
                if not np.array_equal(a.view(np.uint32), b.view(np.uint32)):
                    why.append(f"rank {r}: {name} differ from the unsharded schedule")
            if not np.array_equal(res[True][0][1], lb):
                why.append(f"rank {r}: weights differ from rank 0's")
    return {"ok": not why, "why": why}


def _child(world, fabric, **extra_env):
    env = dict(os.environ, GPU_MAX_HW_QUEUES="32", **extra_env)
    try:
        r = subprocess.run([sys.executable, os.path.abspath(__file__), str(world), fabric], env=env,
                           capture_output=True, text=True, timeout=150)
    except subprocess.TimeoutExpired as e:
        pytest.fail(f"world {world} {fabric}: child timed out\n{(e.stderr or '')[-3000:]}")
    recs = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert r.returncode == 0 and len(recs) == 1, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    assert recs[0]["ok"], recs[0]["why"]


@pytest.mark.parametrize("world,fabric", [(2, "p2p"), (3, "p2p"), (8, "p2p"), (3, "loopback")])
def test_shard_update_bit_identical_to_unsharded(world, fabric):
    _child(world, fabric)


def test_shard_update_group_per_lane_reduce():
    """The owner reduce + SGD kernel in its one-group-per-lane form (FAN_WIRE_REDUCE4=0; the default runs 4 values
    per lane): the same bits as the unsharded schedule too."""
    _child(3, "p2p", FAN_WIRE_REDUCE4="0")


def test_shard_update_forced_one_rank_matches_inline():
    """World 1 through the multi-rank path (1-rank RCCL group): the sharded request's weights equal the inline
    engine's fused decode + SGD, and it needs no deferred epilogue."""
    from fpga_ai_nic_amd.parallel.transport import NativeTransport
    from fpga_ai_nic_amd.utils import dist as D

    if not torch.distributed.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(29500 + os.getpid() % 1000))
        D.init_distributed(force=True)
    n = 1 << 18
    rng = np.random.default_rng(3)
    g = torch.from_numpy(rng.standard_normal(n).astype(np.float32)).cuda()
    w0 = torch.from_numpy(rng.standard_normal(n).astype(np.float32)).cuda()
    ref = NativeAllReduce(None, codec="bfp_rne")  # inline world 1
    sh = NativeAllReduce(NativeTransport(force_collectives=True), codec="bfp_rne", force_comm=True, shard_update=True)
    assert sh.shard_update and ref.inline
    out = {}
    for name, eng in (("ref", ref), ("shard", sh)):
        L = eng.layout(n)
        gg = torch.zeros(L.n_pad, device="cuda")
        gg[:n] = g
        w = torch.zeros(L.n_pad, device="cuda")
        w[:n] = w0
        lp = torch.zeros(L.n_pad, device="cuda", dtype=torch.bfloat16)
        eng.allreduce_sgd(gg, w, lp, n_valid=n, lr=0.1).synchronize(60)
        torch.cuda.synchronize()
        out[name] = (w[:n].clone(), lp[:n].clone())
    assert torch.equal(out["ref"][0], out["shard"][0]) and torch.equal(out["ref"][1], out["shard"][1])
    assert sh.counters()["sharded_updates"] == 1


if __name__ == "__main__":
    print(json.dumps(_case(int(sys.argv[1]), sys.argv[2])), flush=True)
