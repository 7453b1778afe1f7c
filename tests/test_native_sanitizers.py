"""Host C++ under AddressSanitizer + UndefinedBehaviorSanitizer.

GPU ASan / XNACK builds are not available on the MI355X pool, so the sanitizers cover the host-side native
code: the ring planner (csrc/comm/planner.cpp: every ring position simulated, link-matrix-restricted rings), the
FAN_FAULT grammar parser (csrc/comm/fault_spec.cpp: valid and malformed specs, every prefix of a long one) and the
engine's request-slot state machine (csrc/comm/slot_table.h, the host logic of engine.cpp's submit / commit /
wait / query: driven against a simulated device with random stream interleavings in every engine mode, > 8
deferred requests, superseded handles, the null-stream producer and 32-bit sequence wrap-around) are compiled with
-fsanitize=address,undefined together with self-tests, and must run clean.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
@pytest.mark.parametrize("selftest, unit", [("planner_selftest", "planner"), ("fault_spec_selftest", "fault_spec"),
                                            ("slot_table_selftest", None)])
def test_host_cpp_asan_ubsan(tmp_path, selftest, unit):
    exe = tmp_path / selftest
    units = [os.path.join(ROOT, "csrc", "comm", f"{unit}.cpp")] if unit else []  # slot_table.h is header-only
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=all", "-I", os.path.join(ROOT, "csrc"),
           os.path.join(ROOT, "tests", "native", f"{selftest}.cpp")] + units + ["-o", str(exe)]
    subprocess.run(cmd, check=True, capture_output=True, timeout=300)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:verify_asan_link_order=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip().endswith("OK")
    assert "runtime error" not in r.stderr
