"""Test-only fault injection for the communication engine.

The reference has no failure handling at all (its ``wait()`` spins forever, sw/mlp_mpi_example_f32.cpp:163-168;
``kill_syn_e0`` is unused, hw/all_reduce.sv:83). This hook lets tests exercise the timeout / checksum paths.

Configure with ``FAN_FAULT="<site>:<call-index>:<kind>"`` (comma separated list), e.g.
``ring_send:3:flip`` (xor the first byte of the 4th ring message), ``mesh_pack:0:nan`` (plant an Inf exponent
in the packed gradient), ``ring_send:0:delay_ms=200``. The native engine also knows ``p2p_publish:<k>:drop``: the
k-th direct P2P round's ready flags are never written (a lost message: the peers' waits never complete), which the
bench uses to show that a hung transport is aborted and excluded instead of ending the run.
"""
from __future__ import annotations

import os
import time

import torch


class FaultInjector:
    def __init__(self, spec: str = ""):
        self.rules = []
        for item in filter(None, (s.strip() for s in spec.split(","))):
            site, idx, kind = item.split(":", 2)
            self.rules.append((site, int(idx), kind))
        self.counts: dict[str, int] = {}

    @classmethod
    def from_env(cls) -> "FaultInjector":
        return cls(os.environ.get("FAN_FAULT", ""))

    @property
    def active(self) -> bool:
        return bool(self.rules)

    def maybe_corrupt(self, site: str, buf: torch.Tensor) -> None:
        if not self.rules:
            return
        k = self.counts.get(site, 0)
        self.counts[site] = k + 1
        for s, idx, kind in self.rules:
            if s != site or idx != k:
                continue
            b = buf.view(torch.uint8).view(-1)
            if kind == "flip":
                b[:1].bitwise_xor_(0xFF)
            elif kind == "nan":
                b[-1:].fill_(0xFF)  # an exponent byte of 255 => group decodes to NaN (rne codec)
            elif kind.startswith("delay_ms="):
                if b.is_cuda:
                    torch.cuda.current_stream().synchronize()
                time.sleep(float(kind.split("=", 1)[1]) / 1000.0)
            else:
                raise ValueError(f"unknown fault kind {kind!r}")
