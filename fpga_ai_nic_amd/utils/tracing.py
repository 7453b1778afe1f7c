"""Tracing: roctx ranges (visible in rocprofv3 --marker-trace / sys-trace timelines) + host timers.

Reference: DETAILED_PROFILE per-phase accumulators (sw/mlp_mpi_example_f32.cpp:32-33, 238-267, 702-814) and the
NIC's cycle counters (hw/all_reduce.sv:892-1085). Enable ranges with ``FAN_ROCTX=1``.
"""
from __future__ import annotations

import contextlib
import ctypes
import os

_lib = None
_enabled = os.environ.get("FAN_ROCTX", "0") == "1"


def _roctx():
    global _lib, _enabled
    if _lib is None and _enabled:
        for name in ("librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so", "libroctx64.so.4", "libroctx64.so"):
            try:
                _lib = ctypes.CDLL(name)
                _lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                break
            except OSError:
                continue
        if _lib is None:
            _enabled = False
    return _lib


def enable(flag: bool = True):
    global _enabled
    _enabled = flag


@contextlib.contextmanager
def range(name: str):  # noqa: A001 - mirrors roctx naming
    lib = _roctx() if _enabled else None
    if lib is not None:
        lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        if lib is not None:
            lib.roctxRangePop()


def mark(name: str):
    lib = _roctx() if _enabled else None
    if lib is not None:
        lib.roctxMarkA(name.encode())
