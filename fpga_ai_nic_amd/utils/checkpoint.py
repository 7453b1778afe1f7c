"""Checkpoint / resume in the reference-compatible weight layout.

The reference never writes weights to disk; its in-memory layout is one contiguous row-major
``C[i] x C[i+1]`` fp32 buffer per layer (sw/mlp_mpi_example_f32.cpp:396-401) plus a ``C[i+1]`` bias. This module
defines the on-disk format as exactly that:

* ``<path>.safetensors`` — tensors ``fc{i}.weight`` [C_i, C_{i+1}] and ``fc{i}.bias`` [C_{i+1}] in f32 (or bf16),
  optional ``fc{i}.momentum`` (flat, f32);
* ``<path>.json`` — index: layer shapes / dtypes / byte offsets into a plain concatenated ``.bin`` image, the
  libxsmm blocking ``bn/bk/bc`` as metadata, iteration counter, world size and engine settings.
* ``<path>.bin`` — the raw concatenation (weight_0, bias_0, weight_1, ...) so a C/C++ consumer (e.g. the
  reference's ``fil_libxsmm[i]`` arrays) can ``fread`` each layer directly.

Only rank 0 writes; loading uses safetensors (no pickle).
"""
from __future__ import annotations

import json
import os

import numpy as np
import torch
from safetensors.torch import load_file, save_file


def save(path: str, model, *, iteration: int = 0, dtype: str = "f32", meta: dict | None = None):
    tdt = torch.float32 if dtype == "f32" else torch.bfloat16
    tensors, index, off = {}, [], 0
    blobs = []
    for i, l in enumerate(model.layers):
        w = l.w_master.detach().to("cpu", tdt).contiguous()
        b = l.b_master.detach().to("cpu", tdt).contiguous()
        tensors[f"fc{i}.weight"] = w
        tensors[f"fc{i}.bias"] = b
        if l.mom is not None:
            tensors[f"fc{i}.momentum"] = l.mom[: l.n].detach().to("cpu").contiguous()
        for name, t in ((f"fc{i}.weight", w), (f"fc{i}.bias", b)):
            raw = t.view(torch.uint8).numpy().tobytes() if tdt == torch.bfloat16 else t.numpy().tobytes()
            index.append({"name": name, "shape": list(t.shape), "dtype": dtype, "offset": off, "nbytes": len(raw)})
            blobs.append(raw)
            off += len(raw)
    os.makedirs(os.path.dirname(os.path.abspath(path)) or ".", exist_ok=True)
    save_file(tensors, path + ".safetensors")
    with open(path + ".bin", "wb") as f:
        for raw in blobs:
            f.write(raw)
    info = {"format": "fpga_ai_nic_amd/mlp-v1", "sizes": model.sizes, "iteration": iteration, "dtype": dtype,
            "layout": "row-major C[i] x C[i+1] (reference fil_libxsmm order)", "tensors": index}
    info.update(meta or {})
    with open(path + ".json", "w") as f:
        json.dump(info, f, indent=1)
    return path


def load(path: str, model) -> dict:
    with open(path + ".json") as f:
        info = json.load(f)
    if list(info["sizes"]) != list(model.sizes):
        raise ValueError(f"checkpoint sizes {info['sizes']} != model sizes {model.sizes}")
    sd = load_file(path + ".safetensors")
    for i, l in enumerate(model.layers):
        l.w_master.copy_(sd[f"fc{i}.weight"].to(l.master.device, torch.float32))
        l.b_master.copy_(sd[f"fc{i}.bias"].to(l.master.device, torch.float32))
        if l.mom is not None and f"fc{i}.momentum" in sd:
            l.mom[: l.n].copy_(sd[f"fc{i}.momentum"].to(l.mom.device))
    model.sync_lp()
    return info


def read_raw_layer(path: str, name: str) -> np.ndarray:
    """Read one layer from the plain ``.bin`` image via the JSON index (what a C++ consumer does)."""
    with open(path + ".json") as f:
        info = json.load(f)
    ent = next(t for t in info["tensors"] if t["name"] == name)
    with open(path + ".bin", "rb") as f:
        f.seek(ent["offset"])
        raw = f.read(ent["nbytes"])
    if ent["dtype"] == "f32":
        return np.frombuffer(raw, dtype=np.float32).reshape(ent["shape"])
    u = np.frombuffer(raw, dtype=np.uint16).astype(np.uint32) << 16
    return u.view(np.float32).reshape(ent["shape"])
