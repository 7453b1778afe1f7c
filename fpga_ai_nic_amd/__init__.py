"""fpga_ai_nic_amd — an MI355X-native compressed-all-reduce data-parallel training engine.

Capabilities of libxsmm/fpga_ai_nic (an FPGA "AI smart NIC" that BFP-compresses the gradient
all-reduce and applies SGD on the NIC), re-designed for AMD Instinct MI355X (gfx950):

* ``ops``       hand-written CDNA4 HIP kernels: BFP wire codec, fused reduce / SGD epilogues,
                MFMA GEMMs with fused epilogues, softmax-xent, bias-grad reductions;
* ``parallel``  transports (RCCL over xGMI via torch.distributed or a native RCCL comm; gloo; virtual
                ranks), the compressed all-reduce engine (mesh + ring/multi-ring), the DP trainer;
* ``models``    the MLP family of the reference (+ BERT-base gradient-shape buckets for comm benches);
* ``utils``     config, metrics/report, tracing, checkpoints, fault injection, topology;
* ``cli``       the ``mlp_mpi`` entry point with the reference's positional signature.
"""
__version__ = "0.1.0"

import torch  # noqa: F401  (before any import of _C.so: a C++ exception raised by _C with torch's Python module
#                            not yet initialised corrupted the heap at interpreter exit)

from . import _ext  # noqa: F401
