"""The multi-GPU bench path rehearsed on ONE MI355X: ``bench.py --gpus 2`` starts its two ranks itself (a
torch.distributed.run child), the ranks share the GPU, the gradient plane is the direct P2P transport (HIP-IPC
receive arenas + stream-ordered flags: the same protocol that runs over xGMI between GPUs) and the control plane is
gloo (RCCL refuses two ranks on one device). Everything the round-end 8-GPU run reports must already be present and
self-consistent here: exactly one JSON line, a measured all-reduce (extra.allreduce, from the traced pass), the
communicator's own rank count, direct P2P rounds, and bit-identical replicas after the run (extra.dist) — and the
self-selection the driver's multi-GPU run relies on: the schedule A/B in warmup (every arm timed or excluded with
its error: RCCL refuses two ranks on one device, so only the P2P arms run here), the bit-exact all-reduce gate of
the chosen arm, and the config-4 / uncompressed / config-5 extras, all within the run's budget. A peer slot
corrupted after its ready flag makes every arm fail the gate and the run exit non-zero."""
import json
import os
import subprocess
import sys
import time

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
    ab = ex["schedule_ab"]
    timed = [x for x in ab if "ms_per_step" in x]
    assert len(timed) >= 3 and sum(bool(x.get("chosen")) for x in ab) == 1, ab
    assert all(x["exact"] for x in timed), ab
    assert any(x["arm"].startswith("rccl") and "error" in x for x in ab), ab  # excluded, not fatal
    assert d["allreduce_exact"] is True and d["allreduce_gate"]["prepacked"] is True, d
    c4 = ex["config4"]
    assert c4["bfp_mesh_p2p"]["algo_bw_GBps"] > 0 and c4["bfp_ring_p2p"]["algo_bw_GBps"] > 0, c4
    assert c4["raw_f32_mesh_p2p"]["algo_bw_GBps"] > 0 and "skipped" in c4["rccl_f32"], c4
    un = ex["uncompressed"]
    assert un["p2p_raw_f32_mesh"]["ms_per_step"] > 0, un
    # both ranks on one GPU: the speedup would time the shared GPU, not the codec -> withheld, with the reason
    assert un["speedup_vs_best_uncompressed"] is None and "share a GPU" in un["speedup_note"], un
    c5 = ex["config5"]  # BERT-base backward + per-layer all-reduce over the headline's transport
    assert c5["t_compute_ms"] > 0 and c5["t_comm_ms"] > 0 and c5["t_overlap_ms"] > 0 and c5["transport"] == "p2p", c5
    assert ex["extras_s"] < 240 and ex["run_s"] < 400, (ex["extras_s"], ex["run_s"])


@pytest.mark.parametrize("flags,queues", [("cp", "1"), ("kernel", "1"), ("kernel", "4")])
def test_bench_two_ranks_hw_queues_and_kernel_flags(tmp_path, flags, queues):
    """Each rank with ONE hardware queue (GPU_MAX_HW_QUEUES=1: every stream of the process, compute and comm, in one
    in-order queue, so a flag wait parks the rank's GEMMs behind it) and the flag writes / waits either as command-
    processor packets or as kernels (--p2p-flags kernel): the fixed-schedule step must neither deadlock nor lose
    exactness -- the gate passes, the replicas stay bit-identical, no kernel-flag wait reaches its bound. (A peer's
    ready write is queued before that rank's own waits in every round -- p2p_round_flags -- so one queue per rank
    cannot close a cycle.)"""
    saved = {k: os.environ.get(k) for k in ("GPU_MAX_HW_QUEUES", "FAN_KEEP_HW_QUEUES")}
    os.environ.update(GPU_MAX_HW_QUEUES=queues, FAN_KEEP_HW_QUEUES="1")  # exactly this many (no co-location cap)
    try:
        r, recs = _bench(tmp_path, "--schedule", "fixed", "--p2p-flags", flags, "--extra-budget", "0", timeout=300)
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    assert r.returncode == 0 and len(recs) == 1, (r.stdout[-2000:], r.stderr[-4000:])
    ex = recs[0]["extra"]
    d = ex["dist"]
    assert d["replicas_identical"] is True and d["allreduce_exact"] is True, d
    assert ex["engine_counters"]["direct_rounds"] > 0
    assert recs[0]["config"].get("p2p_flags", "cp") == flags, recs[0]["config"]
    if flags == "kernel":
        assert ex["p2p_stats"]["kernel_flag_error"] == 0, ex["p2p_stats"]


def test_bench_gate_rejects_a_corrupted_peer_slot(tmp_path):
    """Every engine flips a byte of the first message it receives, after that message's ready flag was raised
    (fault site p2p_recv): the owner reduces a wrong shard and every rank decodes the same wrong sum (the replicas
    would still agree). The exactness gate catches it on every P2P arm, which is excluded and listed in
    extra.gates_failed; the record comes from the last-resort arm (or, without one, the bench exits non-zero)."""
    os.environ["FAN_FAULT"] = "p2p_recv:0:flip"
    try:
        r, recs = _bench(tmp_path, "--extra-budget", "0", timeout=300)
    finally:
        os.environ.pop("FAN_FAULT", None)
    assert "exactness gate failed" in r.stderr, r.stderr[-4000:]
    assert r.returncode != 124
    if recs:  # the record of the last-resort arm, with every P2P arm listed as failing its gate
        assert r.returncode == 0 and recs[0]["config"]["schedule"] == "torch_mesh_python", recs
        failed = {g["arm"] for g in recs[0]["extra"]["gates_failed"]}
        assert {a["arm"] for a in recs[0]["extra"]["schedule_ab"] if a["arm"].startswith("p2p")} <= failed, failed
    else:
        assert r.returncode != 0


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


def test_bench_survives_a_hung_transport(tmp_path):
    """Every engine's first direct P2P round is never announced (FAN_FAULT p2p_publish:0:drop: the ready flags are
    not written, what a dead link looks like to the peers). The first P2P arm's exactness gate then times out at
    --arm-timeout on both ranks, the engine aborts the transport (poisoned flags release the parked streams), the
    ranks agree to drop P2P and exclude its remaining arms — a hung link costs its arms, not the whole record. Here
    RCCL refuses two ranks on one GPU, so what is left is the last-resort arm (_ends_on_the_fallback_arm); the
    watchdog never fires."""
    os.environ["FAN_FAULT"] = "p2p_publish:0:drop"
    t0 = time.monotonic()
    try:
        r, recs = _bench(tmp_path, "--extra-budget", "0", "--arm-timeout", "15", timeout=300)
    finally:
        os.environ.pop("FAN_FAULT", None)
    took = time.monotonic() - t0
    assert "transport p2p aborted and excluded after arm p2p_mesh_persistent" in r.stderr, r.stderr[-4000:]
    assert "exceeded" not in r.stderr, r.stderr[-4000:]  # the watchdog never fired
    assert "P2P transport unavailable: aborted after arm p2p_mesh_persistent" in r.stderr, r.stderr[-4000:]
    _ends_on_the_fallback_arm(r, recs)
    assert took < 240, took


def _ends_on_the_fallback_arm(r, recs):
    """With the P2P transport gone and RCCL refused (two ranks on one GPU), the run either completes on the last
    resort arm (the Python engine over the control plane's collectives: one gate-checked JSON line) or, where that
    backend cannot run the step on GPU tensors, ends non-zero — never by the watchdog."""
    assert r.returncode != 124, r.stderr[-3000:]
    if r.returncode == 0:
        assert len(recs) == 1 and recs[0]["config"]["schedule"] == "torch_mesh_python", recs
        assert recs[0]["extra"]["dist"]["allreduce_gate"]["exact"] is True
        assert all("ms_per_step" not in a for a in recs[0]["extra"]["schedule_ab"] if a["arm"].startswith("p2p"))
    else:
        assert not recs, r.stdout[-2000:]


def test_bench_survives_a_stuck_p2p_connect(tmp_path):
    """The P2P bootstrap's IPC imports are bounded (FAN_P2P_CONNECT_TIMEOUT; a 2 GiB arena's import once never
    returned): with a zero bound every rank reports the connect as stuck, all ranks drop the P2P transport together
    and its arms are excluded with that error instead of the run hanging in connect()."""
    os.environ["FAN_P2P_CONNECT_TIMEOUT"] = "0"
    try:
        r, recs = _bench(tmp_path, "--extra-budget", "0", timeout=300)
    finally:
        os.environ.pop("FAN_P2P_CONNECT_TIMEOUT", None)
    assert "did not return within 0 s" in r.stderr, r.stderr[-4000:]
    _ends_on_the_fallback_arm(r, recs)
