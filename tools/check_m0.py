"""Build-time check of the LDS-DMA statements' M0 contract (csrc/gemm/glds.h, gemm_bf16_kernel.h glds16_s/_si).

Those inline-asm statements write M0 and leave it written: hipcc reserves M0 and does not honour an "m0" clobber
(it only warns that a reserved register "may not be preserved"), so correctness rests on the compiler never keeping
its own value live in M0 across them in any kernel that also runs them. This script disassembles every gfx950
code object of the build (build/obj/*.o: .hip_fatbin -> clang-offload-bundler -> llvm-objdump) and, per kernel
symbol that contains the LDS-DMA pattern (``s_mov_b32 m0`` / ``s_add_u32 m0`` followed by
``global_load_lds_dwordx4``), fails on any OTHER instruction that reads or writes M0 (GPR-index mode, s_movrel,
v_readlane/v_writelane with an M0 lane select, s_sendmsg, ds_gws, an M0 spill or reload ...).

Usage: python tools/check_m0.py [build/obj]   (exit 1 and a listing on a violation)
"""
from __future__ import annotations

import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
OURS = re.compile(r"^\s*(s_mov_b32|s_add_u32)\s+m0,")
M0 = re.compile(r"\bm0\b")
FORBIDDEN = re.compile(r"\b(s_movrel\w*|s_set_gpr_idx\w*)\b")


def disasm(obj: str, tmp: str) -> str | None:
    fat = os.path.join(tmp, "x.fatbin")
    co = os.path.join(tmp, "x.co")
    for f in (fat, co):
        if os.path.exists(f):
            os.remove(f)
    r = subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", obj, os.path.join(tmp, "junk.o")],
                       capture_output=True)
    if r.returncode != 0 or not os.path.exists(fat):
        return None  # host-only object
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                    f"--targets={TARGET}", f"--output={co}"], check=True, capture_output=True)
    return subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co], check=True,
                          capture_output=True, text=True).stdout


def check_text(text: str) -> list[str]:
    """Violations in one disassembly: per function, foreign M0 accesses where the LDS-DMA pattern is present."""
    bad = []
    funcs: dict[str, list[str]] = {}
    cur = None
    for line in text.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            cur = m.group(1)
            funcs[cur] = []
            continue
        if cur is not None and line.strip():
            funcs[cur].append(line.split("//")[0].rstrip())
    for name, ins in funcs.items():
        has_glds = any("global_load_lds" in x for x in ins)
        for i, x in enumerate(ins):
            if FORBIDDEN.search(x):
                bad.append(f"{name}: {x.strip()}")
                continue
            if not has_glds or not M0.search(x):
                continue
            if "global_load_lds" in x:
                continue
            if OURS.match(x) and any("global_load_lds" in y for y in ins[i + 1:i + 3]):
                continue
            bad.append(f"{name}: {x.strip()}")
    return bad


def main(argv: list[str]) -> int:
    objdir = argv[1] if len(argv) > 1 else os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                        "build", "obj")
    bad, n = [], 0
    with tempfile.TemporaryDirectory() as tmp:
        for fn in sorted(os.listdir(objdir)):
            if not fn.endswith(".o"):
                continue
            text = disasm(os.path.join(objdir, fn), tmp)
            if text is None:
                continue
            n += 1
            bad += [f"{fn}: {b}" for b in check_text(text)]
    if bad:
        print(f"[check_m0] {len(bad)} foreign M0 / GPR-index accesses in LDS-DMA kernels:")
        for b in bad[:50]:
            print("  " + b)
        return 1
    print(f"[check_m0] ok: {n} gfx950 code objects, no foreign M0 access beside the LDS-DMA statements")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
