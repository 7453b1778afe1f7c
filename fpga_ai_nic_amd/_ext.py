"""Loader for the in-tree native extension ``fpga_ai_nic_amd/_C.so``.

The extension holds every hand-written CDNA4 kernel (BFP codec, fused reduce / SGD epilogues,
MFMA GEMMs, softmax-xent), the native ring planner and the native RCCL communicator.

Policy: on a machine with a GPU, a missing or stale extension is a hard error (``require()``) —
GPU code paths never fall back silently to PyTorch. CPU code paths (gloo tests, the bit-exact
oracles) do not need it, but the planner is still used from it when importable.
"""
from __future__ import annotations

import importlib
import os
import threading

_lock = threading.Lock()
_mod = None
_err: Exception | None = None

_SO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_C.so")


def load():
    """Import the extension if present; returns the module or None (never raises)."""
    global _mod, _err
    if _mod is not None:
        return _mod
    with _lock:
        if _mod is not None:
            return _mod
        try:
            import torch  # noqa: F401  (torch must be loaded first: shared HIP runtime / RCCL)

            _mod = importlib.import_module("fpga_ai_nic_amd._C")
        except Exception as e:  # pragma: no cover - exercised when the build is missing
            _err = e
            _mod = None
    return _mod


def available() -> bool:
    return load() is not None


def require():
    """Return the extension or raise a loud error explaining how to build it."""
    m = load()
    if m is None:
        raise RuntimeError(
            "fpga_ai_nic_amd native extension (_C.so) is not built or failed to load "
            f"({_err!r}). Build it with: python tools/build_ext.py"
        )
    return m


def so_path() -> str:
    return _SO
