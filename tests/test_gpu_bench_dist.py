"""The multi-GPU bench path rehearsed on ONE MI355X: ``bench.py --gpus 2`` starts its two ranks itself (a
torch.distributed.run child), the ranks share the GPU, the gradient plane is the direct P2P transport (HIP-IPC
receive arenas + stream-ordered flags: the same protocol that runs over xGMI between GPUs) and the control plane is
gloo (RCCL refuses two ranks on one device). Everything the round-end 8-GPU run reports must already be present and
self-consistent here: exactly one JSON line, a measured all-reduce (extra.allreduce, from the traced pass), the
communicator's own rank count, direct P2P rounds, and bit-identical replicas after the run (extra.dist)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(tmp_path, *extra, timeout=420):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--transport", "p2p", "--steps", "3",
           "--warmup", "1", "--mb-per-gpu", "512", "--ref-mb", "256", "--timeout", "150", *extra]
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env.update(FAN_CTRL_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=timeout)
    recs = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    return r, recs


def test_bench_two_ranks_p2p_one_gpu(tmp_path):
    r, recs = _bench(tmp_path)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert len(recs) == 1, r.stdout
    rec = recs[0]
    assert rec["n_gpus"] == 2 and rec["config"]["parallelism"] == "dp2" and rec["config"]["transport"] == "p2p"
    ex = rec["extra"]
    ar = ex["allreduce"]
    assert ar is not None and ar["requests"] > 0 and ar["wire_bw_GBps"] > 0 and ar["allreduce_algo_bw_GBps"] > 0
    d = ex["dist"]
    assert d["replicas_identical"] is True, d
    assert d["engine_comm"] == "p2p" and d["comm_ranks"] == [2, 2], d
    assert d["torch_backend"] == "gloo" and d["world"] == 2
    assert len(d["bus_ids"]) == 2 and d["bus_ids"][0] == d["bus_ids"][1]  # both ranks on the one GPU
    assert ex["engine_counters"]["direct_rounds"] > 0
    assert ex["mb256"]["samples_per_s"] > 0


def test_bench_watchdog_fires_on_a_hung_peer(tmp_path):
    """A rank that never takes part in the exchange (FAN_BENCH_STALL_RANK: rank 1 sleeps before its first step)
    leaves rank 0's comm stream parked on a P2P flag: the watchdog must end the run non-zero within its budget and
    print the engine's debug_status (slots, comm rank count, flag words) instead of hanging."""
    cmd_env = dict(FAN_BENCH_STALL_RANK="1", FAN_BENCH_STALL_S="600")
    os.environ.update(cmd_env)
    try:
        r, recs = _bench(tmp_path, "--timeout", "20", timeout=300)
    finally:
        for k in cmd_env:
            os.environ.pop(k, None)
    assert r.returncode != 0 and not recs
    assert "exceeded 20 s" in r.stderr and "debug_status" in r.stderr, r.stderr[-4000:]
    assert '"comm_kind": "p2p"' in r.stderr, r.stderr[-4000:]
