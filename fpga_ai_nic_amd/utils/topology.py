"""Topology discovery and ring construction (replaces the reference's IKL route setup).

Reference: ``ikl_setup()`` shells out ``iko areset/reset`` and ``setup_route.sh N`` which wires a unidirectional
Ethernet ring f{i} p0 -> f{i+1} p1 for N in 3..6 only (sw/mlp_mpi_example_f32.cpp:50-63, sw/setup_route.sh:12-40).

MI355X: an 8-GPU node is fully connected by xGMI (7 links per GPU), so no routing step exists. What matters is
(1) which peers are reachable over xGMI (P2P access, link type/weight), and (2) how to spread ring traffic over
all 7 links: ``ring_orders`` decomposes the complete digraph into arc-disjoint directed Hamiltonian cycles
(7 for 8 GPUs), one per link. ``python -m fpga_ai_nic_amd.utils.topology`` prints the report.
"""
from __future__ import annotations

import json
import re
import shutil
import subprocess

import torch


def device_info():
    out = []
    if not torch.cuda.is_available():
        return out
    for i in range(torch.cuda.device_count()):
        p = torch.cuda.get_device_properties(i)
        out.append({"index": i, "name": p.name, "gcn_arch": getattr(p, "gcnArchName", ""),
                    "cus": p.multi_processor_count, "hbm_GB": round(p.total_memory / 1e9, 1)})
    return out


def peer_matrix():
    n = torch.cuda.device_count() if torch.cuda.is_available() else 0
    return [[(i == j) or bool(torch.cuda.can_device_access_peer(i, j)) for j in range(n)] for i in range(n)]


def rocm_smi_links():
    """Parse ``rocm-smi --showtopotype`` (link type per GPU pair) when available; {} otherwise."""
    exe = shutil.which("rocm-smi")
    if not exe:
        return {}
    try:
        txt = subprocess.run([exe, "--showtopotype"], capture_output=True, text=True, timeout=20).stdout
    except Exception:  # pragma: no cover - tool missing / restricted
        return {}
    links = {}
    rows = [l for l in txt.splitlines() if re.match(r"^GPU\d+", l.strip())]
    for r in rows:
        parts = r.split()
        i = int(parts[0][3:])
        for j, t in enumerate(parts[1:]):
            links[(i, j)] = t
    return links


def link_matrix(world: int):
    """Direct-link matrix of the first ``world`` GPUs (rank r = device r, one process per GPU on one node):
    links[a][b] = 1 when a reaches b over xGMI — rocm-smi's link type when it reports one (XGMI), else HIP peer
    access. None when the devices are not all visible (the planner then assumes a fully connected node)."""
    if not torch.cuda.is_available() or torch.cuda.device_count() < world:
        return None
    peer = peer_matrix()
    types = rocm_smi_links()
    out = [[0] * world for _ in range(world)]
    for a in range(world):
        for b in range(world):
            if a == b:
                continue
            t = types.get((a, b))
            out[a][b] = int(t.upper() == "XGMI") if t else int(peer[a][b])
    return out


def ring_orders(world: int, max_rings: int | None = None, links=None):
    from ..parallel.allreduce import ring_orders as _ro

    return _ro(world, world - 1 if max_rings is None else max_rings, links)


def report(world: int | None = None) -> dict:
    devs = device_info()
    n = world or max(1, len(devs))
    rings = ring_orders(n, links=link_matrix(n))
    return {"devices": devs, "peer_access": peer_matrix(), "links": {f"{k[0]}-{k[1]}": v for k, v in
                                                                     rocm_smi_links().items()},
            "world": n, "rings": rings,
            "note": f"{len(rings)} arc-disjoint directed Hamiltonian ring(s) over {n} GPUs"}


if __name__ == "__main__":
    import sys

    w = int(sys.argv[1]) if len(sys.argv) > 1 else None
    print(json.dumps(report(w), indent=1))
