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
