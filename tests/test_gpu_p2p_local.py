"""Direct P2P schedules at world 3, 4 and 8 on ONE GPU: N virtual ranks in one process, each with its own P2PComm
(receive arena + flag block) wired to the others with ``P2PComm.connect_local`` (no IPC), one host thread and one
stream per rank. The two-process test (test_gpu_p2p.py) covers the IPC bootstrap at world 2, where a ring has one
neighbour each way; here the direct ring runs over several arc-disjoint rings at once (every rank a different
downstream peer per ring, hw/all_reduce.sv's single ring generalised: sw/setup_route.sh), and the direct mesh over
N - 1 peers. Each schedule is bit-exact against the spec simulator, from f32 and from producer-encoded (prepacked)
input, and counts its direct rounds — also in verify mode (every message tagged in its slot's trailer where it landed
and checked on arrival: ``verified_rows`` > 0) and with the pure copies on the copy engines (FAN_P2P_COPY=sdma). A
fault rule that corrupts a received slot AFTER its ready flag was raised (``p2p_recv``) must be caught by verify mode
with the site and row of that message.

The ranks' flag waits are command-processor waits (hipStreamWaitValue64): a stream parked on a peer's flag blocks the
hardware queue it runs on. HIP multiplexes a process's streams onto GPU_MAX_HW_QUEUES queues (4 by default), so N
ranks' 2N+ streams in ONE process can park one rank behind another's wait (a deadlock a one-process-per-GPU job
cannot have). Each case therefore runs in a child process with one hardware queue per stream (GPU_MAX_HW_QUEUES=32,
the pool's limit) under its own time limit."""
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
from fpga_ai_nic_amd.parallel import sim  # noqa: E402
from fpga_ai_nic_amd.parallel.native_engine import NativeAllReduce  # noqa: E402

pytestmark = pytest.mark.gpu


def _run(world, algo, rings, m=40000, max_slice=2048, mode="plain"):
    C = _ext.require()
    stream = mode.startswith("stream")
    comms = [C.P2PComm(r, world, 0, 2 << 20, 4 if stream else 2) for r in range(world)]
    C.P2PComm.connect_local(comms)
    if mode == "sdma":
        for c in comms:
            c.sdma = True
    if mode.startswith("kflag"):  # flag writes / waits as kernels instead of command-processor packets
        for c in comms:
            c.kernel_flags = True
    rng = np.random.default_rng(100 + world)
    grads = [rng.standard_normal(m).astype(np.float32) for _ in range(world)]
    res, errs = [None] * world, [None] * world
    verify = mode in ("verify", "fault", "stream_verify", "block_verify", "kflag_verify")
    fault = "p2p_recv:0:flip" if mode == "fault" else None
    engines = [NativeAllReduce(None, codec="bfp_rne", algo=algo, rings=rings, max_slice_elems=max_slice,
                               comm=comms[r], verify=verify, fault=fault, ring_sub=3 if stream else 1)
               for r in range(world)]
    if stream:
        assert all(e.ring_sub == 3 for e in engines) and engines[0].layout(m).sub == 3

    def run(r):
        try:
            torch.cuda.set_device(0)
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                eng = engines[r]
                L = eng.layout(m)
                g = torch.zeros(L.n_pad, device="cuda")
                g[:m] = torch.from_numpy(grads[r]).cuda()
                out = torch.zeros(L.n_pad, device="cuda")
                eng.allreduce(g, out, n_valid=m).synchronize(60)
                tgt = eng.prepack_target(g, m)
                out_p = None
                if tgt is not None:  # the producer's encoding as the input
                    buf, shard, own, cid = tgt[:4]
                    C.wire_pack_range(g, buf, shard, 0, m // 16 * 16, cid)
                    out_p = torch.zeros(L.n_pad, device="cuda")
                    eng.allreduce(g, out_p, n_valid=m, prepacked=(buf, m // 16 * 16)).synchronize(60)
                s.synchronize()
                cn = eng.counters()
                res[r] = (out.cpu().numpy(), None if out_p is None else out_p.cpu().numpy(), L,
                          cn["direct_rounds"], [list(o) for o in eng.orders], cn["verified_rows"],
                          comms[r].kernel_flag_error())
        except Exception as e:  # noqa: BLE001
            errs[r] = e

    ts = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(180)
    assert not any(t.is_alive() for t in ts), "virtual rank thread hung"
    if mode == "fault":
        return errs, None, None
    assert not any(errs), errs
    L = res[0][2]
    gin = [np.pad(x, (0, L.n_pad - m)) for x in grads]
    if algo == "mesh":
        ref = sim.mesh_allreduce(gin, L.shard)
    else:
        ref = sim.ring_allreduce(gin, res[0][4], L.slice_elems, L.blocks)[0]
    return res, ref, L


def _check(world, algo, rings, mode="plain"):
    res, ref, L = _run(world, algo, rings, mode=mode)
    m = 40000
    if mode == "fault":  # every rank corrupted the first message it received, after that message's ready flag
        site, row = ("mesh direct send", 1) if algo == "mesh" else ("ring direct hop", 0)
        why = []
        for r, e in enumerate(res):
            want_row = (1 if r == 0 else 0) if algo == "mesh" else row
            if e is None or "corrupted" not in str(e) or f"{site} row {want_row} " not in str(e):
                why.append(f"rank {r}: expected a '{site} row {want_row}' corruption, got {e!r}")
        return {"ok": not why, "why": why, "rings": 0}
    out = {"ok": True, "why": [], "rings": len(res[0][4]), "release_mode": _ext.require().p2p_release_mode()}
    for r in range(world):
        o, o_p, _, direct, orders, verified, kerr = res[r]
        if kerr:
            out["why"].append(f"rank {r}: a kernel-flag wait gave up")
        if mode in ("verify", "stream_verify", "block_verify", "kflag_verify") and verified <= 0:
            out["why"].append(f"rank {r}: verify mode checked no message")
        if not np.array_equal(o[:m], ref[:m]):
            out["why"].append(f"rank {r}: {algo} x{rings} differs from the simulator")
        if o_p is not None and not np.array_equal(o_p, o):
            out["why"].append(f"rank {r}: prepacked input differs")
        if direct <= 0:
            out["why"].append(f"rank {r}: the direct path did not run")
        if orders != res[0][4]:
            out["why"].append(f"rank {r}: ring orders differ")
    out["ok"] = not out["why"]
    return out


def _child(world, algo, rings, mode):
    env = dict(os.environ, GPU_MAX_HW_QUEUES="32")
    if mode.startswith(("block", "thread")):  # the in-kernel release forms (cross-device peers default to "block")
        env["FAN_P2P_RELEASE"] = mode.split("_")[0]
    try:
        r = subprocess.run([sys.executable, os.path.abspath(__file__), str(world), algo, str(rings), mode], env=env,
                           capture_output=True, text=True, timeout=150)
    except subprocess.TimeoutExpired as e:
        pytest.fail(f"world {world} {algo}: child timed out\n{(e.stderr or '')[-3000:]}")
    recs = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert r.returncode == 0 and len(recs) == 1, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    rec = recs[0]
    assert rec["ok"], rec["why"]
    return rec


@pytest.mark.parametrize("world,algo,rings", [(3, "ring", 2), (4, "ring", 3), (8, "ring", 7), (3, "mesh", 1),
                                              (8, "mesh", 1)])
def test_direct_p2p_schedules_bit_exact(world, algo, rings):
    rec = _child(world, algo, rings, "plain")
    if algo == "ring":
        assert rec["rings"] >= min(rings, 2)  # several arc-disjoint rings at once (N = 4 has 2, not 3)


@pytest.mark.parametrize("world,algo,rings", [(4, "ring", 3), (4, "mesh", 1)])
@pytest.mark.parametrize("mode", ["verify", "sdma"])
def test_direct_p2p_verify_and_sdma_bit_exact(world, algo, rings, mode):
    """verify mode runs the direct paths (no copying fallback) and checks every message; the copy-engine path moves
    the same bytes."""
    _child(world, algo, rings, mode)


@pytest.mark.parametrize("world,rings,mode", [(3, 2, "stream"), (8, 7, "stream"), (4, 3, "stream_verify")])
def test_direct_ring_streamed_hops_bit_exact(world, rings, mode):
    """Each hop's message in 3 sub-slices with a ready flag each (4-slot arenas): the sums, summation order and
    results are the lock-step ring's, bit for bit, from f32 and from prepacked input (sub-shard wire layout)."""
    _child(world, "ring", rings, mode)


@pytest.mark.parametrize("world,algo,rings", [(4, "ring", 3), (4, "mesh", 1)])
@pytest.mark.parametrize("mode", ["block", "thread", "block_verify"])
def test_direct_p2p_in_kernel_release_bit_exact(world, algo, rings, mode):
    """The in-kernel release forms of the peer-storing kernels (p2p_release: "block" = per-workgroup drain + one
    system-scope release, the mode a process with peers on OTHER GPUs runs unless FAN_P2P_RELEASE says otherwise;
    "thread" = a system fence per wave): same sums, bit for bit, also with verify mode checking every message."""
    rec = _child(world, algo, rings, mode)
    assert rec["release_mode"] == (1 if mode.startswith("block") else 2), rec


@pytest.mark.parametrize("world,algo,rings", [(3, "mesh", 1), (4, "ring", 3), (8, "mesh", 1)])
@pytest.mark.parametrize("mode", ["kflag", "kflag_verify"])
def test_direct_p2p_kernel_flags_bit_exact(world, algo, rings, mode):
    """Kernel flags (P2PComm.kernel_flags): each round's flag writes are one kernel's system-scope release stores and
    its waits one kernel's bounded spin + acquire -- the CP-independent path, same flag words (p2p_round_flags),
    same sums bit for bit, no wait reaching its bound."""
    _child(world, algo, rings, mode)


@pytest.mark.parametrize("algo,rings", [("mesh", 1), ("ring", 2)])
def test_direct_p2p_verify_catches_a_slot_corrupted_after_its_flag(algo, rings):
    _child(3, algo, rings, "fault")


if __name__ == "__main__":
    mode = sys.argv[4] if len(sys.argv) > 4 else "plain"
    print(json.dumps(_check(int(sys.argv[1]), sys.argv[2], int(sys.argv[3]), mode)), flush=True)
