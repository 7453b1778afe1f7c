"""Properties of the bit-exact BFP oracle (reference numerics + the framework's RNE variant)."""
import numpy as np
import pytest

from fpga_ai_nic_amd.ops import bfp_oracle as O


def _E(x):
    return (np.abs(x.reshape(-1, 16)).view(np.uint32).max(axis=1) >> 23).astype(np.int64)


def test_known_values_trunc():
    ones = np.ones(16, np.float32)
    q, E = O.encode_groups(ones, "trunc")
    assert E[0] == 127 and np.all(q == 64)
    assert np.array_equal(O.decode_groups(q, E, "trunc"), ones)
    q, E = O.encode_groups(-ones, "trunc")
    assert np.all(q == -64)
    assert np.array_equal(O.decode_groups(q, E, "trunc"), -ones)


def test_zero_group_and_q0_quirk_trunc():
    z = np.zeros(16, np.float32)
    q, E = O.encode_groups(z, "trunc")
    # hidden bit forced: zeros encode as q=64 with E=0, and decode back to +0.0 (exponent field 0)
    assert E[0] == 0 and np.all(q == 64)
    assert np.all(O.decode_groups(q, E, "trunc") == 0)
    x = np.zeros(16, np.float32)
    x[0] = 1.0
    x[1] = 2.0 ** -10
    q, E = O.encode_groups(x, "trunc")
    assert q[1] == 0
    # the reference decodes q=0 as 2^(E-150), not 0 (hw/bfp_to_bf16_core.sv normalise path)
    assert O.decode_groups(q, E, "trunc")[1] == np.float32(2.0 ** (127 - 150))


def test_minus_128_decodes_to_magnitude_128():
    q = np.full(16, -128, np.int8)
    E = np.array([127], np.uint8)
    v = O.decode_groups(q, E, "trunc")
    assert np.all(v == -2.0)  # 128 * 2^(127-133)


@pytest.mark.parametrize("rounding", ["trunc", "rne"])
def test_error_bound(rounding):
    rng = np.random.default_rng(0)
    x = (rng.standard_normal(16 * 4096) * np.exp2(rng.integers(-20, 20, 16 * 4096))).astype(np.float32)
    q, E = O.encode_groups(x, rounding)
    d = O.decode_groups(q, E, rounding)
    step = np.exp2(_E(x) - 133.0).repeat(16)
    err = np.abs(d.astype(np.float64) - x)
    bound = step * (1.0 + 2.0 ** -10) if rounding == "trunc" else step * 1.0
    assert np.all(err <= bound)
    if rounding == "rne":
        # away from the clamp, RNE halves the bound
        ok = np.abs(x) < 127 * step
        assert np.all(err[ok] <= 0.5 * step[ok] * (1 + 1e-6))


def test_trunc_is_floor_biased():
    rng = np.random.default_rng(1)
    x = rng.standard_normal(16 * 2048).astype(np.float32)
    d = O.quantize(x, "bfp_trunc")
    nz = O.encode_groups(x, "trunc")[0] != 0
    assert np.all(d[nz] <= x[nz])
    assert (d - x).mean() < 0
    r = O.quantize(x, "bfp_rne")
    assert abs((r - x).mean()) < abs((d - x).mean()) / 5


def test_idempotent_rne():
    """Re-encoding a decoded group reproduces it (RNE): re-encoding all-gather hops would add no error."""
    rng = np.random.default_rng(2)
    x = (rng.standard_normal(16 * 1024) * 1e3).astype(np.float32)
    once = O.quantize(x, "bfp_rne")
    assert np.array_equal(O.quantize(once, "bfp_rne"), once)


def test_trunc_idempotent_except_minus_128():
    """Reference numerics: idempotent unless a group holds q = -128, whose decoded magnitude 2^(E-126) raises the
    shared exponent on re-encode. The engine therefore forwards encoded all-gather bytes untouched."""
    rng = np.random.default_rng(2)
    x = (rng.standard_normal(16 * 1024) * 1e3).astype(np.float32)
    q, _ = O.encode_groups(x, "trunc")
    has_m128 = (q.reshape(-1, 16) == -128).any(axis=1).repeat(16)
    once = O.quantize(x, "bfp_trunc")
    twice = O.quantize(once, "bfp_trunc")
    assert np.array_equal(twice[~has_m128], once[~has_m128])
    assert has_m128.any() and not np.array_equal(twice[has_m128], once[has_m128])


def test_nan_inf_policy_rne():
    x = np.ones(32, np.float32)
    x[3] = np.inf
    x[20] = np.nan
    d = O.quantize(x, "bfp_rne")
    assert np.all(np.isnan(d))  # whole groups poisoned: corrupted gradients fail loudly


def test_denormals_rne():
    x = (np.arange(16, dtype=np.float32) + 1) * np.float32(1e-41)
    d = O.quantize(x, "bfp_rne")
    assert np.abs(d - x).max() <= 2.0 ** -133 * 0.5 + 1e-45


def test_layout_and_ratio():
    n_s = 512
    x = np.random.default_rng(3).standard_normal(n_s * 3).astype(np.float32)
    buf = O.pack(x, n_s, "bfp_rne")
    assert buf.size == 3 * (n_s + n_s // 16)
    assert 4 * x.size / buf.size == pytest.approx(64 / 17)  # 3.76x vs fp32 (reference: 64 flits -> 17)
    assert np.array_equal(O.unpack(buf, x.size, n_s, "bfp_rne"), O.quantize(x, "bfp_rne"))
    # shard s mantissas start at s * 17 n_s / 16, exponents right after its mantissas
    q, E = O.encode_groups(x[n_s:2 * n_s], "rne")
    sb = n_s + n_s // 16
    assert np.array_equal(buf[sb:sb + n_s].view(np.int8), q)
    assert np.array_equal(buf[sb + n_s:2 * sb], E)


def test_bf16_helpers_roundtrip():
    x = np.array([1.0, -2.5, 3.14159, 1e-30, 65504.0], np.float32)
    b = O.f32_to_bf16_bits(x)
    y = O.bf16_bits_to_f32(b)
    assert np.allclose(x, y, rtol=2 ** -8)
