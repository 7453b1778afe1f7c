"""Row-panel layout planning (NativeAllReduce.panel_plan) on CPU: every chunk is whole 16-B-aligned rows of dW
whose element count is world shards of a 256-multiple, the last chunk holds the remaining rows (>= 8) + the bias,
and the padding stays small."""
import pytest

from fpga_ai_nic_amd.parallel.native_engine import NativeAllReduce


class _FakeC:
    def layout(self, n, shard, chunks):
        assert shard % 256 == 0 and shard * chunks >= 0
        return {}


def _eng(world, **kw):
    e = NativeAllReduce.__new__(NativeAllReduce)
    e.algo, e.prepack, e.inline, e.codec, e.world, e.C = "mesh", True, False, "bfp_rne", world, _FakeC()
    for k, v in kw.items():
        setattr(e, k, v)
    return e


@pytest.mark.parametrize("world", [1, 2, 4, 8, 16])
@pytest.mark.parametrize("cin,cout,panels", [(1024, 4096, 4), (256, 512, 4), (4096, 1024, 3), (1000, 1024, 4),
                                             (2048, 2048, 8)])
def test_panel_plan_invariants(world, cin, cout, panels):
    pp = _eng(world).panel_plan(cin, cout, panels)
    assert pp is not None
    R, C, S = pp["rows"], pp["chunks"], pp["shard"]
    assert R % 8 == 0 and S % 256 == 0 and R * cout == world * S
    assert C >= 2 and (C - 1) * R < cin and cin - (C - 1) * R >= 8  # last panel: real rows
    assert cin * cout + cout <= pp["n_pad"] == C * world * S
    assert pp["n_pad"] - (cin * cout + cout) <= R * cout  # at most one panel of padding


def test_panel_plan_refuses_unsupported_engines():
    assert _eng(8, algo="ring").panel_plan(1024, 4096, 4) is None
    assert _eng(8, inline=True).panel_plan(1024, 4096, 4) is None
    assert _eng(8, codec="raw_f32").panel_plan(1024, 4096, 4) is None
    assert _eng(8).panel_plan(1024, 4096, 1) is None
    assert _eng(8).panel_plan(1024, 4100, 4) is None  # widths must be whole BFP groups
