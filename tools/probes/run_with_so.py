"""Run a script with another build of the extension: ``python tools/probes/run_with_so.py <_C.so> <script> [args]``
loads that library under the module name fpga_ai_nic_amd._C first (A/B of two builds on one box, e.g. bench.py
with a diagnostic or previous build), then runs the script as __main__. World-1 runs only (no self-launch)."""
import importlib.util
import os
import runpy
import sys

so, script = sys.argv[1], sys.argv[2]
sys.argv = [script] + sys.argv[3:]
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402,F401  (first, as fpga_ai_nic_amd/_ext.py does: the extension must bind torch's HIP runtime)

spec = importlib.util.spec_from_file_location("fpga_ai_nic_amd._C", so)
mod = importlib.util.module_from_spec(spec)
sys.modules["fpga_ai_nic_amd._C"] = mod
spec.loader.exec_module(mod)
runpy.run_path(script, run_name="__main__")
