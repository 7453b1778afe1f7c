"""In-tree builder for the native extension ``fpga_ai_nic_amd/_C.so``.

Drives ``hipcc --offload-arch=gfx950`` directly (no cpp_extension hipify pass):
every ``.hip``/``.cpp`` under ``csrc/`` is compiled to an object in ``build/``
and linked against the torch / HIP / RCCL libraries that ``torch`` itself ships
(same SONAMEs, so the process holds exactly one HIP runtime and one RCCL).

Usage::

    python tools/build_ext.py            # incremental build
    python tools/build_ext.py --clean    # full rebuild
    python tools/build_ext.py -j 8 -v
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
BUILD = os.path.join(ROOT, "build", "obj")
OUT = os.path.join(ROOT, "fpga_ai_nic_amd", "_C.so")
ARCH = os.environ.get("FAN_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _torch_dirs():
    import torch  # noqa: WPS433  (build-time only)

    tdir = os.path.dirname(torch.__file__)
    inc = [os.path.join(tdir, "include"), os.path.join(tdir, "include", "torch", "csrc", "api", "include")]
    return tdir, inc, os.path.join(tdir, "lib"), int(torch._C._GLIBCXX_USE_CXX11_ABI)


def sources():
    out = []
    for dp, _, fns in os.walk(CSRC):
        for fn in sorted(fns):
            if fn.endswith((".hip", ".cpp")):
                out.append(os.path.join(dp, fn))
    return sorted(out)


def headers_digest():
    h = hashlib.sha1()
    for dp, _, fns in os.walk(CSRC):
        for fn in sorted(fns):
            if fn.endswith((".h", ".hpp", ".cuh", ".inc")):
                p = os.path.join(dp, fn)
                with open(p, "rb") as f:
                    h.update(p.encode())
                    h.update(f.read())
    return h.hexdigest()


def compile_flags(tinc, abi):
    py_inc = sysconfig.get_paths()["include"]
    fl = [
        "-std=c++17", "-O3", "-fPIC", f"--offload-arch={ARCH}",
        "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
        "-DTORCH_EXTENSION_NAME=_C", "-DTORCH_API_INCLUDE_EXTENSION_H",
        "-Wno-unused-result", "-Wno-deprecated-declarations",
        "-munsafe-fp-atomics",
        f"-I{CSRC}", f"-I{py_inc}", "-I/opt/rocm/include",
    ]
    fl += [f"-I{d}" for d in tinc]
    fl += os.environ.get("FAN_EXTRA_CFLAGS", "").split()  # e.g. -DFAN_GEMM_4WAVE (experimental kernel variants)
    return fl


def _obj_for(src):
    rel = os.path.relpath(src, CSRC).replace(os.sep, "__")
    return os.path.join(BUILD, rel + ".o")


def build(jobs: int = 8, verbose: bool = False, clean: bool = False) -> str:
    tdir, tinc, tlib, abi = _torch_dirs()
    if clean and os.path.isdir(BUILD):
        shutil.rmtree(BUILD)
    os.makedirs(BUILD, exist_ok=True)
    flags = compile_flags(tinc, abi)
    hdig = headers_digest()
    stamp_path = os.path.join(BUILD, "flags.stamp")
    stamp = hashlib.sha1((" ".join(flags) + hdig).encode()).hexdigest()
    old = open(stamp_path).read() if os.path.exists(stamp_path) else ""
    force = old != stamp

    srcs = sources()
    todo = []
    for s in srcs:
        o = _obj_for(s)
        if force or not os.path.exists(o) or os.path.getmtime(o) < os.path.getmtime(s):
            todo.append((s, o))

    def _cc(item):
        s, o = item
        cmd = [HIPCC] + flags + ["-c", s, "-o", o]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"compile failed: {s}\n{r.stdout}\n{r.stderr}")
        if r.stderr.strip() and verbose:
            print(r.stderr, file=sys.stderr)
        return s

    if todo:
        with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
            for s in ex.map(_cc, todo):
                print(f"[build_ext] compiled {os.path.relpath(s, ROOT)}", flush=True)
    objs = [_obj_for(s) for s in srcs]
    need_link = bool(todo) or not os.path.exists(OUT) or any(
        os.path.getmtime(o) > os.path.getmtime(OUT) for o in objs)
    if need_link:
        tmp = OUT + ".tmp"
        cmd = [HIPCC, "-shared", f"--offload-arch={ARCH}", "-o", tmp] + objs + [
            f"-L{tlib}", f"-Wl,-rpath,{tlib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu",
            "-ltorch_hip", "-ltorch_python", "-lamdhip64", "-lrccl",
        ]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, OUT)
        print(f"[build_ext] linked {os.path.relpath(OUT, ROOT)}", flush=True)
        # the LDS-DMA statements leave M0 written (hipcc ignores an "m0" clobber): no kernel that runs them may hold a
        # compiler value in M0 (tools/check_m0.py)
        if os.path.exists(f"{os.path.dirname(HIPCC)}/../lib/llvm/bin/clang-offload-bundler"):
            sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
            import check_m0  # noqa: WPS433

            if check_m0.main(["check_m0", BUILD]) != 0:
                os.remove(OUT)
                raise RuntimeError("M0 contract violated by a compiled kernel (tools/check_m0.py)")
    with open(stamp_path, "w") as f:
        f.write(stamp)
    return OUT


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", "--jobs", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--clean", action="store_true")
    a = ap.parse_args()
    build(a.jobs, a.verbose, a.clean)


if __name__ == "__main__":
    main()
