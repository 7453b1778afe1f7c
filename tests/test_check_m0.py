"""tools/check_m0.py: the build-time check that no kernel running the LDS-DMA inline asm (which writes M0 and leaves
it) also holds a compiler value in M0 (hipcc does not honour an "m0" clobber)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import check_m0  # noqa: E402

OK = """
0000000000001000 <k_ok>:
\ts_mov_b32 m0, s12
\ts_nop 0
\tglobal_load_lds_dwordx4 v2, s[4:5]
\ts_add_u32 m0, s13, 0x400
\ts_nop 0
\tglobal_load_lds_dwordx4 v3, s[4:5]
\tv_mfma_f32_16x16x32_bf16 a[0:3], v[4:7], v[8:11], a[0:3]
0000000000002000 <k_other>:
\ts_mov_b32 m0, -1
\tds_write_b32 v1, v2
"""

BAD = """
0000000000001000 <k_bad>:
\ts_mov_b32 m0, s12
\ts_nop 0
\tglobal_load_lds_dwordx4 v2, s[4:5]
\tv_readlane_b32 s3, v1, m0
"""


def test_lds_dma_only_kernels_pass():
    # a kernel without the LDS-DMA pattern may use M0 freely
    assert check_m0.check_text(OK) == []


def test_foreign_m0_access_is_reported():
    bad = check_m0.check_text(BAD)
    assert len(bad) == 1 and "v_readlane_b32" in bad[0]


def test_gpr_index_mode_is_reported_anywhere():
    assert check_m0.check_text("0000 <k>:\n\ts_set_gpr_idx_on s2, gpr_idx(SRC0)\n")
