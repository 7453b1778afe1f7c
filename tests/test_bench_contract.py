"""bench.py driver contract, rehearsed on CPU: the same script the round-end scaling run launches under
torch.distributed.run (one rank per GPU over RCCL) runs here with gloo ranks, and rank 0 alone prints ONE JSON
line whose fields match the contract (whole-job value, weak scaling, dp<N>, steps / warmup echoed)."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.slow


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _json_lines(out):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


@pytest.mark.parametrize("world", [1, 2, 3, 4])  # 3: the reference's world size (sw/run.sh: mpirun -n 3)
def test_bench_json_contract(world, tmp_path):
    args = [os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--steps", "2", "--warmup", "1",
            "--mb-per-gpu", "16"]
    if world > 1:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port())] + args
    else:
        cmd = [sys.executable] + args
    env = dict(os.environ, OMP_NUM_THREADS="2", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    r = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    recs = _json_lines(r.stdout)
    assert len(recs) == 1, r.stdout  # rank 0 only, one line
    rec = recs[0]
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in rec, k
    assert rec["n_gpus"] == world and rec["steps"] == 2 and rec["warmup"] == 1
    assert rec["scaling"] == "weak" and rec["higher_is_better"] is True and rec["dtype"] == "bf16"
    cfg = rec["config"]
    assert cfg["model"] == "mlp-1024-4096-4096-1024" and cfg["parallelism"] == f"dp{world}"
    assert cfg["global_batch"] == 16 * world
    # value is the whole-job aggregate: global batch x steps / (max-over-ranks) elapsed time
    assert rec["value"] == pytest.approx(cfg["global_batch"] / (rec["ms_per_step"] / 1e3), rel=1e-2)
    assert rec["extra"]["final_loss"] > 0
    ex = rec["extra"]
    if world > 1:
        # the self-selection machinery the driver's multi-GPU run relies on, rehearsed over gloo ranks: one A/B arm
        # (the Python engine on CPU), chosen, gate-checked bit-exact on every rank; every extra recorded
        ab = ex["schedule_ab"]
        assert len(ab) == 1 and ab[0].get("chosen") and ab[0]["exact"] is True, ab
        g = ex["dist"]["allreduce_gate"]
        assert g["exact"] and g["checked"] and g["max_abs_diff"] == 0.0, g
        assert ex["dist"]["replicas_identical"] is True
        assert ex["uncompressed"]["torch_f32"]["ms_per_step"] > 0 and ex["uncompressed"]["speedup_vs_best_uncompressed"]
        assert ex["config4"] == {"skipped": "CPU run"} and ex["config5"] == {"skipped": "CPU run"}
        assert cfg["schedule"] == ab[0]["arm"]


def test_bench_self_launches_ranks(tmp_path):
    """``python bench.py --gpus 2`` with no torch.distributed environment starts its 2 ranks itself (a
    torch.distributed.run child; the parent never touches the GPU) and still prints exactly one JSON line."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--mb-per-gpu", "16", "--ref-mb", "8"]
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env.update(OMP_NUM_THREADS="2", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    r = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    recs = _json_lines(r.stdout)
    assert len(recs) == 1, r.stdout
    rec = recs[0]
    assert rec["n_gpus"] == 2 and rec["config"]["parallelism"] == "dp2" and rec["config"]["global_batch"] == 32
    ref = rec["extra"]["mb8"]
    assert ref["global_batch"] == 16 and ref["samples_per_s"] > 0
    assert "effective_allreduce_algo_bw_GBps" not in rec["extra"]


def test_bench_watchdog_ends_a_hung_run(tmp_path):
    """A rank that stops taking part (test hook FAN_BENCH_STALL_RANK) leaves its peer blocked in a collective:
    the per-phase watchdog ends the whole job non-zero within its budget and reports which phase hung."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--mb-per-gpu", "16", "--ref-mb", "0", "--timeout", "15"]
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env.update(OMP_NUM_THREADS="2", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", FAN_BENCH_STALL_RANK="1",
               FAN_BENCH_STALL_S="600")
    r = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode != 0 and not _json_lines(r.stdout)
    assert "phase 'warmup timed mb=16' exceeded 15 s" in r.stderr, r.stderr[-3000:]


def test_bench_prints_the_headline_when_an_extra_hangs(tmp_path):
    """Rank 1 stops inside an extra (test hook FAN_BENCH_STALL_EXTRA): rank 0 waits in that extra's next collective
    until its watchdog fires — which prints the record of the headline measured before (one JSON line, the phase it
    was aborted in) before ending the run, instead of losing the measurement."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--mb-per-gpu", "16", "--ref-mb", "0", "--timeout", "20"]
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env.update(OMP_NUM_THREADS="2", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="",
               FAN_BENCH_STALL_EXTRA="uncompressed:1")
    r = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0, r.stderr[-3000:]
    recs = _json_lines(r.stdout)
    assert len(recs) == 1, (r.stdout, r.stderr[-3000:])
    rec = recs[0]
    assert rec["extra"]["aborted_in"] == "extra uncompressed" and rec["value"] > 0 and rec["n_gpus"] == 2
    assert "config4" in rec["extra"] and rec["extra"]["dist"] is None


def test_uncompressed_speedup_guard():
    """extra.uncompressed.speedup_vs_best_uncompressed is withheld when it would not measure the codec: ranks
    time-sharing one GPU, or an uncompressed arm dominated by its own P2P flag-wait stalls."""
    import bench

    arms = {"p2p_raw_f32_mesh": {"ms_per_step": 4.0, "p2p_stall_ms_per_step": 0.5}, "rccl_f32": {"skipped": "x"}}
    sp, note = bench._uncompressed_speedup(arms, 2.0, ["a", "b", "c"])
    assert sp == 2.0 and "fastest" in note
    sp, note = bench._uncompressed_speedup(arms, 2.0, ["a", "a", "a"])
    assert sp is None and "share a GPU" in note
    arms["p2p_raw_f32_mesh"]["p2p_stall_ms_per_step"] = 3.0
    sp, note = bench._uncompressed_speedup(arms, 2.0, ["a", "b"])
    assert sp is None and "stall" in note
    assert bench._uncompressed_speedup({"rccl_f32": {"skipped": "x"}}, 2.0, [None])[0] is None


def test_colocated_ranks_cap_hw_queues(monkeypatch):
    """Ranks sharing a GPU get GPU_MAX_HW_QUEUES=2 from the self-launcher (queue oversubscription across processes
    time-slices their flag hand-offs); one GPU per rank, a smaller setting or FAN_KEEP_HW_QUEUES=1 is left alone."""
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench

    monkeypatch.setattr(bench, "_device_count", lambda: 1)
    assert bench.colocated_hw_queues(3, {}) == "2"
    assert bench.colocated_hw_queues(3, {"GPU_MAX_HW_QUEUES": "4"}) == "2"  # the boxes export HIP's default
    assert bench.colocated_hw_queues(3, {"GPU_MAX_HW_QUEUES": "1"}) is None  # a smaller setting is kept
    assert bench.colocated_hw_queues(3, {"FAN_KEEP_HW_QUEUES": "1"}) is None
    assert bench.colocated_hw_queues(1, {}) is None
    monkeypatch.setattr(bench, "_device_count", lambda: 8)
    assert bench.colocated_hw_queues(8, {}) is None and bench.colocated_hw_queues(16, {}) == "2"
    monkeypatch.setattr(bench, "_device_count", lambda: 0)  # CPU: nothing to cap
    assert bench.colocated_hw_queues(2, {}) is None
