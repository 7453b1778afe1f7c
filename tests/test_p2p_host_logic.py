"""Host-side logic of the direct P2P transport (csrc/comm/p2p_comm.cpp), no GPU needed.

* When a round records the system-scope release event before its flag writes: always in release mode 3 (cp); in
  the in-kernel modes (1 block, 2 thread, 0 none) only when bytes of the round were moved outside a peer-storing
  kernel (copy engines / hipMemcpyAsync fallback) — those bytes were released by no kernel, and a cross-device peer
  could otherwise read the flag before them (the reference's done flag is written after the data,
  hw/all_reduce.sv:1368-1375).
* The copy-engine path issues one command per contiguous run of segments, not one per segment.
"""
import pytest

from fpga_ai_nic_amd import _ext

C = _ext.load()
pytestmark = pytest.mark.skipif(C is None, reason="native extension not built")


@pytest.mark.parametrize("mode", [0, 1, 2, 3])
@pytest.mark.parametrize("copy_engine_bytes", [False, True])
def test_release_event_decision(mode, copy_engine_bytes):
    assert C.p2p_release_event_needed(mode, copy_engine_bytes) == (mode == 3 or copy_engine_bytes)


def test_coalesce_contiguous_runs():
    # three segments continuing each other in source and destination -> one run; a gap in either breaks the run
    segs = [(0x1000, 0x9000, 256), (0x1100, 0x9100, 256), (0x1200, 0x9200, 512),
            (0x2000, 0x9400, 256),   # source jumps
            (0x2100, 0xA000, 256),   # destination jumps
            (0x2200, 0xA100, 0),     # empty: dropped
            (0x2200, 0xA100, 64)]
    assert C.p2p_coalesce_copies(segs) == [(0x1000, 0x9000, 1024), (0x2000, 0x9400, 256), (0x2100, 0xA000, 320)]


def test_coalesce_keeps_order_and_bytes():
    segs = [(0x10000 * (i % 3), 0x80000 + 0x100 * i, 0x100) for i in range(12)]
    runs = C.p2p_coalesce_copies(segs)
    assert sum(r[2] for r in runs) == sum(s[2] for s in segs)
    assert [r[1] for r in runs] == sorted(r[1] for r in runs)


# ---------------------------------------------------------------------------------------------------------------------
# The flag protocol itself: C.p2p_round_flags is the one function P2PComm's rounds (begin/publish/wait/release and
# sendrecv) take their flag words from, in both the command-processor arm and the kernel-flag arm (the flag kernels
# only change WHO spins, not which words). Simulated here over N ranks under random interleavings with a host model of
# the flag words and of the arena slots: every receiver reads the message of its round, no sender overwrites a slot its
# receiver has not drained (the credit words), and no schedule deadlocks.

def _simulate(world, depth, rounds, pattern, seed, drop_credits=False):
    import random

    rng = random.Random(seed)
    flags = [[0] * (2 * world) for _ in range(world)]      # words 0..world-1 ready-from-q, world+p ack-from-p
    slots = {}                                              # (dst, src, parity) -> (seq, consumed)
    progs = []
    for r in range(world):
        ops = []
        last = [[0] * world for _ in range(depth)]
        for k in range(1, rounds + 1):
            to, frm = pattern(r, world, k)
            par = k % depth
            plan = C.p2p_round_flags(r, world, k, to, frm, last[par])
            ops += [("wait", w) for w in ([] if drop_credits else plan["credit_waits"])]
            ops += [("put", (p, r, par, k)) for p in to]
            ops += [("write", w) for w in plan["ready_writes"]]
            for p in to:
                last[par][p] = k
            ops += [("wait", w) for w in plan["ready_waits"]]
            ops += [("get", (r, q, par, k)) for q in frm]
            ops += [("write", w) for w in plan["ack_writes"]]
        progs.append(ops)
    pc = [0] * world
    hazards = []
    while any(pc[r] < len(progs[r]) for r in range(world)):
        ready = []
        for r in range(world):
            if pc[r] >= len(progs[r]):
                continue
            kind, arg = progs[r][pc[r]]
            if kind == "wait":
                peer, word, val = arg
                assert peer == r, "a rank only ever waits on its own flag words"
                if flags[r][word] < val:
                    continue
            ready.append(r)
        if not ready:
            return "deadlock", hazards
        r = rng.choice(ready)
        kind, arg = progs[r][pc[r]]
        pc[r] += 1
        if kind == "write":
            peer, word, val = arg
            flags[peer][word] = max(flags[peer][word], val)
        elif kind == "put":
            dst, src, par, k = arg
            prev = slots.get((dst, src, par))
            if prev is not None and not prev[1]:
                hazards.append(("overwrite", dst, src, par, prev[0], k))
            slots[(dst, src, par)] = (k, False)
        elif kind == "get":
            dst, src, par, k = arg
            got = slots.get((dst, src, par))
            if got is None or got[0] != k:
                hazards.append(("stale", dst, src, par, got, k))
            else:
                slots[(dst, src, par)] = (k, True)
    return "done", hazards


def _mesh(r, world, k):
    o = [p for p in range(world) if p != r]
    return o, o


def _ring(r, world, k):
    return [(r + 1) % world], [(r - 1) % world]


def _sparse(r, world, k):
    # round k: rank r sends to r+s and receives from r-s, s cycling over 1..world-1 (the shifted all-to-all schedule)
    s = 1 + k % (world - 1)
    return [(r + s) % world], [(r - s) % world]


def test_round_flag_words():
    plan = C.p2p_round_flags(1, 4, 9, [2, 3], [0], [0, 0, 5, 0])
    assert plan["credit_waits"] == [(1, 4 + 2, 5)]          # only the peer whose slot held a message (seq 5)
    assert plan["ready_writes"] == [(2, 1, 9), (3, 1, 9)]   # "ready from 1" in each destination's words
    assert plan["ready_waits"] == [(1, 0, 9)]
    assert plan["ack_writes"] == [(0, 4 + 1, 9)]            # "ack from 1" in the source's words


@pytest.mark.parametrize("world", [2, 3, 5, 8])
@pytest.mark.parametrize("depth", [1, 2, 3])
@pytest.mark.parametrize("pattern", [_mesh, _ring, _sparse])
def test_round_protocol_no_hazard_no_deadlock(world, depth, pattern):
    for seed in range(6):
        state, hazards = _simulate(world, depth, 12, pattern, seed)
        assert state == "done" and not hazards, (seed, hazards[:3])


def test_round_protocol_needs_its_credits():
    # without the credit waits a fast sender laps a slow receiver: the simulator must see that (else it proves nothing)
    seen = any(_simulate(3, 1, 10, _mesh, seed, drop_credits=True)[1] for seed in range(40))
    assert seen
