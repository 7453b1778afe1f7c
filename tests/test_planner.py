"""Native ring planner: geometry, schedule shape, multi-ring decomposition (runs on CPU)."""
import itertools

import pytest

from fpga_ai_nic_amd import _ext
from fpga_ai_nic_amd.parallel import allreduce as A


def test_rounds_per_block():
    for N in (2, 3, 4, 8):
        plan = A.ring_plan(N, 0, 2)
        assert len(plan) == 2 * (2 * N - 2)
        kinds = [r[1] for r in plan[: 2 * N - 2]]
        assert kinds == [0] + [1] * (N - 1) + [2] * (N - 2)  # SEND_LOCAL, REDUCE.., REDUCE_OUTPUT, FORWARD..


def test_reference_slice_order_and_ownership():
    # node n reads slices n, n+1, ... (hw/all_reduce.sv:361) and owns slice n-1 (hw/all_reduce.sv:1230)
    N = 5
    for p in range(N):
        plan = A.ring_plan(N, p, 1)
        reduce_order = [r[0] for r in plan[:N]]
        assert reduce_order == [(p + k) % N for k in range(N - 1)] + [(p - 1) % N]
        owned = [r[4] for r in plan if r[4] >= 0]
        assert owned == [(p - 1) % N]
        # all-gather output order n-1, n, n+1, ..., n-2
        outs = owned + [r[2] for r in plan if r[3] == 1]
        assert outs == [(p - 1 + k) % N for k in range(N)]


def test_neighbour_consistency():
    """What position p sends in row j is exactly what its downstream p-1 receives in row j."""
    for N in (2, 3, 4, 7):
        plans = [A.ring_plan(N, p, 2) for p in range(N)]
        for p in range(N):
            down = (p - 1) % N
            for a, b in zip(plans[p], plans[down]):
                assert a[0] == b[2]  # slice id
                assert (a[1] in (1, 2) and a[4] >= 0) or a[1] == 0 or b[3] == 0 or a[1] == 2


@pytest.mark.skipif(not _ext.available(), reason="native extension not built")
def test_native_matches_python_fallback():
    for N, p, b in itertools.product((1, 2, 3, 5, 8), range(3), (1, 2)):
        if p >= N:
            continue
        assert A.ring_plan(N, p, b) == A._py_ring_plan(N, p, b)


@pytest.mark.skipif(not _ext.available(), reason="native extension not built")
@pytest.mark.parametrize("N,expect", [(2, 1), (3, 2), (4, 2), (5, 4), (6, 4), (7, 6), (8, 7)])
def test_ring_orders_arc_disjoint_hamiltonian(N, expect):
    orders = A.ring_orders(N, N - 1)
    assert len(orders) == expect
    arcs = set()
    for o in orders:
        assert sorted(o) == list(range(N))
        for i in range(N):
            arc = (o[i], o[i - 1])  # position i sends to position i-1
            if N > 2:
                assert arc not in arcs
            arcs.add(arc)
    assert orders[0] == list(range(N))  # ring 0 = reference ring n -> n-1


def test_geometry():
    n, sl, blocks, n_pad = A.ring_geometry(1000, 3, 256)
    assert sl % 256 == 0 and n_pad == blocks * 3 * sl and n_pad >= 1000
    n, sl, blocks, n_pad = A.ring_geometry(25_000_000, 8, 1 << 22)
    assert blocks == 1 and n_pad - 25_000_000 < 8 * 256


def test_gemm_plans_for_workload_shapes():
    """bf16 GEMM tile / split-K plans (host code, CPU): the MLP flagship shapes at minibatch 8192 and the measured
    table for the BERT-base backward shapes (profiles/r1_gemm_bert_sweep.jsonl)."""
    if not _ext.available():
        pytest.skip("native extension not built")
    C = _ext.require()
    expect = {
        (8192, 4096, 4096): (256, 256, 1),   # fwd1 / bwd-data 1: 512 tiles
        (8192, 1024, 4096): (256, 128, 1),   # fwd2: 256 tiles (4-wave pipelined loop)
        (4096, 4096, 8192): (256, 256, 1),   # bwd-weight 1
        (4096, 1024, 8192): (256, 256, 4),   # bwd-weight 2: 64 tiles x split 4
        (1024, 4096, 8192): (256, 256, 4),   # bwd-weight 0
        (4096, 3072, 768): (256, 256, 1),    # BERT ffn_out dgrad (table)
        (3072, 768, 4096): (256, 256, 4),    # BERT ffn_out wgrad (table)
        (768, 768, 4096): (128, 128, 4),     # BERT attn_out wgrad (table)
        (768, 2304, 4096): (128, 256, 4),    # BERT qkv wgrad (table)
    }
    for (M, N, K), (bm, bn, sk) in expect.items():
        p = C.gemm_plan(M, N, K)
        assert (p[0], p[1], p[2]) == (bm, bn, sk), f"{M}x{N}x{K}: {p}"
        # re-planning with the resolved tile and split is the identity (what ops/gemm.py launches)
        assert tuple(C.gemm_plan(M, N, K, p[2], p[0], p[1])[:3]) == (bm, bn, sk)
    assert C.gemm_plan(100, 128, 64)[0] == 0  # unsupported: M % 128


def test_gemm_plan_env_override():
    """FAN_GEMM_PLAN overrides the planned tile / split for listed shapes (in-step A/B without a rebuild);
    a malformed value raises instead of being ignored. Runs in a subprocess (the env is read once)."""
    import os
    import subprocess
    import sys

    if not _ext.available():
        pytest.skip("native extension not built")
    code = ("import fpga_ai_nic_amd._ext as E; C = E.require(); "
            "print(C.gemm_plan(8192, 4096, 1024)[:3], C.gemm_plan(1024, 4096, 8192)[:3], "
            "C.gemm_plan(8192, 4096, 4096)[:3])")
    env = dict(os.environ, FAN_GEMM_PLAN="8192x4096x1024=128,256,1;1024x4096x8192=256,256,2")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.split("\n")[-2] == "(128, 256, 1) (256, 256, 2) (256, 256, 1)"
    env["FAN_GEMM_PLAN"] = "8192x4096x1024=96,256,1"
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "FAN_GEMM_PLAN" in r.stderr


def _check_rings(orders, N, links=None):
    arcs = set()
    for o in orders:
        assert sorted(o) == list(range(N))
        for p in range(N):
            src, dst = o[p], o[(p - 1) % N]  # position p sends to p-1
            assert (src, dst) not in arcs, "rings must be arc-disjoint"
            arcs.add((src, dst))
            if links is not None:
                assert links[src][dst], f"ring uses the missing link {src}->{dst}"


def test_ring_orders_follow_the_link_matrix():
    """Topology-aware rings (the reference wires its ring from the physical links, sw/setup_route.sh:12-40): a
    ring-wired node (each GPU linked to its two neighbours) gets exactly the physical ring; a full node with one
    GPU pair unlinked still gets arc-disjoint rings that avoid that pair; no Hamiltonian cycle -> identity."""
    N = 8
    ring_links = [[int(b in ((a + 1) % N, (a - 1) % N)) for b in range(N)] for a in range(N)]
    orders = A.ring_orders(N, 7, ring_links)
    assert len(orders) == 2  # the physical ring, one per direction
    _check_rings(orders, N, ring_links)
    holes = [[int(a != b and {a, b} != {0, 1}) for b in range(N)] for a in range(N)]
    orders = A.ring_orders(N, 7, holes)
    assert len(orders) >= 5
    _check_rings(orders, N, holes)
    two_islands = [[int(a != b and a // 4 == b // 4) for b in range(N)] for a in range(N)]
    assert A.ring_orders(N, 7, two_islands) == [list(range(N))]
    full = [[int(a != b) for b in range(N)] for a in range(N)]
    assert A.ring_orders(N, 7, full) == A.ring_orders(N, 7)
