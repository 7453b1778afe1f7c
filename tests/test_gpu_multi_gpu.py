"""Distributed GPU checks over real RCCL on every GPU of the box: the engine's mesh / ring /
multi-ring schedules (Python and C++ engines, both BFP codecs) bit-exact vs the spec simulators, fused SGD within
1 ulp of the oracle, replicas bit-identical, the uncompressed f32 ring equal to RCCL's all-reduce, and the
data-parallel trainer (bwd-weight GEMM encoding straight into the wire) keeping replicas identical.

Runs ``tools/dist_probe.py`` under torch.distributed.run with one rank per GPU (up to 8); skipped on a box with
fewer than 2 GPUs (RCCL refuses two ranks on one device; the single-GPU multi-rank paths are covered by
test_gpu_p2p.py and test_gpu_native_loopback.py)."""
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("transport", ["torch", "native", "p2p"])
def test_rccl_probe_all_gpus(transport):
    n = torch.cuda.device_count()
    if n < 2:
        pytest.skip("needs >= 2 GPUs (one rank per GPU)")
    world = min(n, 8)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "tools", "dist_probe.py"),
           "--transport", transport]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "FAIL" not in r.stdout, out[-4000:]
    assert r.stdout.count("PASS") >= world * 5, out[-4000:]
