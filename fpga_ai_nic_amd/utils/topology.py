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


def rocm_smi_bus_ids():
    """rocm-smi GPU index -> PCI bus id (``rocm-smi --showbus``), {} when unavailable. rocm-smi numbers the GPUs
    of the whole node and ignores HIP_VISIBLE_DEVICES, so its indices are matched to HIP devices by bus id."""
    exe = shutil.which("rocm-smi")
    if not exe:
        return {}
    try:
        txt = subprocess.run([exe, "--showbus"], capture_output=True, text=True, timeout=20).stdout
    except Exception:  # pragma: no cover - tool missing / restricted
        return {}
    return parse_showbus(txt)


def parse_showbus(txt: str) -> dict:
    out = {}
    for l in txt.splitlines():
        m = re.match(r"^\s*GPU\[(\d+)\]\s*:\s*PCI Bus:\s*([0-9A-Fa-f:.]+)", l)
        if m:
            out[int(m.group(1))] = normalize_bus_id(m.group(2))
    return out


def normalize_bus_id(b: str) -> str:
    """'0000:05:00.0' / '05:00.0' -> '05:00' (domain and function dropped: one GPU per bus on a node)."""
    parts = b.strip().lower().split(":")
    if len(parts) >= 3:
        parts = parts[-2:]
    return f"{int(parts[0], 16):02x}:{int(parts[1].split('.')[0], 16):02x}"


def device_bus_id(index: int) -> str | None:
    """PCI bus id of HIP device ``index`` (as the current process numbers it), normalised."""
    if not torch.cuda.is_available():
        return None
    p = torch.cuda.get_device_properties(index)
    try:
        return f"{int(p.pci_bus_id):02x}:{int(p.pci_device_id):02x}"
    except (AttributeError, TypeError, ValueError):  # pragma: no cover - older torch
        return None


def own_bus_id() -> str | None:
    """PCI bus id of this process's current HIP device (None without a GPU)."""
    return device_bus_id(torch.cuda.current_device()) if torch.cuda.is_available() else None


def link_matrix_for(bus_ids, peer=None, types=None, smi_bus=None):
    """Direct-link matrix between the GPUs of the ranks (rank r runs on the GPU with PCI bus id ``bus_ids[r]``):
    links[a][b] = 1 when a reaches b over xGMI — rocm-smi's link type when it reports one for that pair (XGMI),
    else ``peer[a][b]`` (HIP peer access between the ranks' devices) when given. None when the ranks' GPUs cannot
    be identified (the planner then assumes a fully connected node). Ranks that share a GPU are linked."""
    world = len(bus_ids)
    if world == 0 or any(b is None for b in bus_ids):
        return None
    types = rocm_smi_links() if types is None else types
    smi_bus = rocm_smi_bus_ids() if smi_bus is None else smi_bus
    smi_of = {b: i for i, b in smi_bus.items()}
    out = [[0] * world for _ in range(world)]
    for a in range(world):
        for b in range(world):
            if a == b:
                continue
            if bus_ids[a] == bus_ids[b]:
                out[a][b] = 1
                continue
            ia, ib = smi_of.get(bus_ids[a]), smi_of.get(bus_ids[b])
            t = types.get((ia, ib)) if ia is not None and ib is not None else None
            if t:
                out[a][b] = int(t.upper() == "XGMI")
            elif peer is not None:
                out[a][b] = int(bool(peer[a][b]))
            else:
                return None
    return out


def link_matrix(world: int, devices=None):
    """Direct-link matrix of the GPUs of ``world`` ranks of ONE process view: rank r runs on HIP device
    ``devices[r]`` (default r). None when those devices are not all visible. For a multi-process job use
    :func:`agreed_link_matrix`, which makes every rank use rank 0's answer."""
    devices = list(range(world)) if devices is None else list(devices)
    if not torch.cuda.is_available() or max(devices) >= torch.cuda.device_count():
        return None
    pm = peer_matrix()
    peer = [[pm[devices[a]][devices[b]] for b in range(world)] for a in range(world)]
    return link_matrix_for([device_bus_id(d) for d in devices], peer=peer)


_AGREED: dict = {}


def agreed_link_matrix(world: int):
    """The link matrix every rank of the default process group uses: each rank reports the PCI bus id of its own
    device; rank 0 derives the matrix (rocm-smi link types of those GPUs, else peer access from its view) and
    broadcasts it, so all ranks plan the SAME rings even if their local tool calls would disagree (a timed-out
    or restricted rocm-smi on one rank would otherwise give that rank different rings and mismatched peers).
    Ranks that span several hosts get None (bus ids are only unique within a host)."""
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized() and dist.get_world_size() == world):
        return link_matrix(world)
    key = (world, id(dist.distributed_c10d._get_default_group()))
    if key in _AGREED:  # one rocm-smi query + agreement per process group (every ring engine asks)
        return _AGREED[key]
    import socket

    ident = [None] * world
    dist.all_gather_object(ident, (socket.gethostname(), own_bus_id()))
    bus = [b for _, b in ident]
    obj = [None]
    if len({h for h, _ in ident}) > 1:
        # ranks on several hosts: PCI bus ids repeat across hosts and rank 0's rocm-smi describes only its own node,
        # so no link matrix is derived (the planner assumes a fully connected world)
        obj = [{"links": None, "bus_ids": bus}]
    elif dist.get_rank() == 0:
        peer = None
        if torch.cuda.is_available():  # peer access from rank 0's view, for the devices it can see
            local = {device_bus_id(i): i for i in range(torch.cuda.device_count())}
            if all(b in local for b in bus):
                pm = peer_matrix()
                peer = [[pm[local[a]][local[b]] for b in bus] for a in bus]
        obj = [{"links": link_matrix_for(bus, peer=peer), "bus_ids": bus}]
    dist.broadcast_object_list(obj, src=0)
    _AGREED[key] = obj[0]["links"]
    return obj[0]["links"]


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
