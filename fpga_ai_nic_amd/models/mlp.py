"""N-layer fully connected MLP + softmax cross-entropy (the reference's only model family).

Reference: sw/mlp_mpi_example_f32.cpp — layers C[0] -> C[1] -> ... -> C[L] with ReLU (fuse_type), a softmax
layer over C[L+1] = C[L] classes (sw:322, 525-531), libxsmm fc fwd/bwd (sw:498-510).

MI355X-first memory layout: every layer owns ONE flat, padded parameter bucket
``[W (C_i x C_{i+1}, row-major) | b (C_{i+1}) | pad]`` in HBM, in three dtype planes:
``master`` (fp32, optimizer state of record), ``lp`` (bf16 compute copy, bf16 models only) and ``grad`` (fp32).
The bucket is exactly the unit the all-reduce engine moves, so gradients are produced by the bwd-weight
GEMM directly into the wire-ready buffer and the fused SGD epilogue writes the weights in place —
no gather/scatter copies, no separate optimizer pass.
"""
from __future__ import annotations


import math
from dataclasses import dataclass

import torch

from ..ops import gemm as G
from ..ops import nn as NN


@dataclass
class LayerBucket:
    cin: int
    cout: int
    n: int            # valid elements (W + b)
    n_pad: int
    master: torch.Tensor
    grad: torch.Tensor
    lp: torch.Tensor | None
    mom: torch.Tensor | None

    @property
    def w_master(self):
        return self.master[: self.cin * self.cout].view(self.cin, self.cout)

    @property
    def b_master(self):
        return self.master[self.cin * self.cout: self.n]

    @property
    def w(self):  # compute weights
        src = self.lp if self.lp is not None else self.master
        return src[: self.cin * self.cout].view(self.cin, self.cout)

    @property
    def b(self):
        src = self.lp if self.lp is not None else self.master
        return src[self.cin * self.cout: self.n]

    @property
    def gw(self):
        return self.grad[: self.cin * self.cout].view(self.cin, self.cout)

    @property
    def gb(self):
        return self.grad[self.cin * self.cout: self.n]


class MLP:
    """Manual-backprop MLP whose hot ops are the framework's HIP kernels (on GPU)."""

    def __init__(self, sizes, *, dtype=torch.bfloat16, device="cpu", pad_fn=None, seed: int = 1,
                 momentum: bool = False, init_scale: float | None = None, bias: bool = True,
                 relu: str = "hidden"):
        """``bias`` / ``relu`` select the layer epilogue. ``relu``: 'hidden' (every layer but the classifier,
        the default model), 'all' or 'none'. The reference's fuse_type (sw:479-489) maps to
        0 -> (bias=False, relu='none'), 1 -> (True, 'none'), 2 -> (False, 'all'), 3 -> (True, 'all')."""
        if len(sizes) < 2:
            raise ValueError("need at least one layer")
        if relu not in ("hidden", "all", "none"):
            raise ValueError(f"relu must be hidden|all|none, got {relu!r}")
        self.bias, self.relu = bias, relu
        self.sizes = list(sizes)
        self.L = len(sizes) - 1
        self.dtype = dtype
        self.device = torch.device(device)
        pad_fn = pad_fn or (lambda n: (n + 255) // 256 * 256)
        gen = torch.Generator().manual_seed(seed)
        self.layers: list[LayerBucket] = []
        for i in range(self.L):
            cin, cout = sizes[i], sizes[i + 1]
            n = cin * cout + cout
            n_pad = pad_fn(n)
            master = torch.zeros(n_pad, dtype=torch.float32)
            bound = init_scale if init_scale is not None else 1.0 / math.sqrt(cin)
            master[: cin * cout] = (torch.rand(cin * cout, generator=gen) * 2 - 1) * bound
            b0 = (torch.rand(cout, generator=gen) * 2 - 1) * bound
            master[cin * cout: n] = b0 if bias else 0.0  # without bias the segment stays 0 (zero gradient)
            master = master.to(self.device)
            lp = master.to(torch.bfloat16) if dtype == torch.bfloat16 else None
            grad = torch.zeros(n_pad, dtype=torch.float32, device=self.device)
            mom = torch.zeros(n_pad, dtype=torch.float32, device=self.device) if momentum else None
            self.layers.append(LayerBucket(cin, cout, n, n_pad, master, grad, lp, mom))
        self._act_mb = None
        self._zero_b: dict[int, torch.Tensor] = {}

    def _relu_at(self, i: int) -> bool:
        return self.relu == "all" or (self.relu == "hidden" and i + 1 < self.L)

    def _bias_of(self, l: LayerBucket):
        if self.bias:
            return l.b
        z = self._zero_b.get(l.cout)
        if z is None:
            z = self._zero_b[l.cout] = torch.zeros(l.cout, dtype=l.b.dtype, device=self.device)
        return z

    # ------------------------------------------------------------------ parameters
    def num_params(self) -> int:
        return sum(l.n for l in self.layers)

    def flops_per_sample(self) -> int:
        """fwd + bwd-data + bwd-weight FLOPs (2 per MAC), excluding layer 0's unneeded bwd-data
        (the reference's GFLOP formula, sw:794-798)."""
        f = 0
        for i, l in enumerate(self.layers):
            f += (6 if i > 0 else 4) * l.cin * l.cout
        return f

    def sync_lp(self):
        for l in self.layers:
            if l.lp is not None:
                l.lp.copy_(l.master.to(torch.bfloat16))

    def state_dict(self):
        out = {}
        for i, l in enumerate(self.layers):
            out[f"fc{i}.weight"] = l.w_master.detach().clone()
            out[f"fc{i}.bias"] = l.b_master.detach().clone()
        return out

    def load_state_dict(self, sd):
        for i, l in enumerate(self.layers):
            l.w_master.copy_(sd[f"fc{i}.weight"].to(l.master.dtype))
            l.b_master.copy_(sd[f"fc{i}.bias"].to(l.master.dtype))
        self.sync_lp()

    def repad(self, i: int, n_pad: int):
        """Grow layer i's bucket planes to ``n_pad`` elements (values kept, new tail zero): an engine layout that pads
        a bucket further than the model's default."""
        l = self.layers[i]
        if n_pad <= l.n_pad:
            return

        def grow(t):
            if t is None:
                return None
            u = torch.zeros(n_pad, dtype=t.dtype, device=t.device)
            u[: l.n_pad] = t
            return u

        l.master, l.grad, l.lp, l.mom = grow(l.master), grow(l.grad), grow(l.lp), grow(l.mom)
        l.n_pad = n_pad

    # ------------------------------------------------------------------ activations
    def alloc_activations(self, mb: int):
        if self._act_mb == mb:
            return
        adt = self.dtype
        dev = self.device
        self.act = [torch.empty(mb, c, dtype=adt, device=dev) for c in self.sizes[:-1]]
        self.logits = torch.empty(mb, self.sizes[-1], dtype=torch.float32, device=dev)
        self.dz = [None] + [torch.empty(mb, c, dtype=adt, device=dev) for c in self.sizes[1:]]
        self.loss_rows = torch.empty(mb, dtype=torch.float32, device=dev)
        self._act_mb = mb

    # ------------------------------------------------------------------ compute
    def forward_layer(self, i: int, fold_logits: bool = False):
        """Layer i's forward GEMM. ``fold_logits`` (training, last layer): a split-K classifier GEMM leaves its slabs
        for :meth:`loss_backward`'s softmax to fold (one launch less; the logits are written there)."""
        l = self.layers[i]
        out = self.act[i + 1] if i + 1 < self.L else self.logits
        self._slabs = None
        if fold_logits and i + 1 == self.L and out.is_cuda and self.dtype == torch.bfloat16 and not self._relu_at(i):
            self._slabs = {}
        G.linear_fwd(self.act[i], l.w, self._bias_of(l), out, relu=self._relu_at(i), defer_reduce=self._slabs)

    def forward_chain(self) -> bool:
        """Every layer's forward GEMM as ONE layer-chain launch (GPU bf16; ops/gemm.py linear_chain); False when the
        chain does not take this model / batch (the caller then runs forward_layer per layer)."""
        if not (self.device.type == "cuda" and self.dtype == torch.bfloat16 and self.L >= 2):
            return False
        outs = [self.act[i + 1] for i in range(self.L - 1)] + [self.logits]
        epis = [G.EPI_BIAS_RELU if self._relu_at(i) else G.EPI_BIAS for i in range(self.L)]
        return G.linear_chain(G.CHAIN_FWD, self.act[0], [l.w for l in self.layers], outs,
                              biases=[self._bias_of(l) for l in self.layers], epis=epis, key=("fwd", id(self)))

    def backward_data_chain(self) -> bool:
        """The bwd-data GEMMs of layers L-1 .. 1 as ONE layer-chain launch (each masked by its input's ReLU); False
        when the chain does not take them (the caller then runs backward_data per layer)."""
        if not (self.device.type == "cuda" and self.dtype == torch.bfloat16 and self.L >= 3):
            return False
        if not all(self._relu_at(i - 1) for i in range(1, self.L)):
            return False
        idx = list(range(self.L - 1, 0, -1))
        return G.linear_chain(G.CHAIN_BWD_DATA, self.dz[self.L], [self.layers[i].w for i in idx],
                              [self.dz[i] for i in idx], auxes=[self.act[i] for i in idx], key=("bwd", id(self)))

    def loss_backward(self, labels, grad_scale: float):
        slabs, self._slabs = getattr(self, "_slabs", None), None
        if slabs:  # the classifier GEMM's split-K slabs, folded here (forward_layer fold_logits)
            NN.softmax_xent_slabs(slabs, self._bias_of(self.layers[-1]), self.logits, labels, self.dz[self.L],
                                  self.loss_rows, grad_scale)
        else:
            NN.softmax_xent(self.logits, labels, self.dz[self.L], self.loss_rows, grad_scale)
        if self._relu_at(self.L - 1):  # ReLU on the classifier output (reference fuse_type 2/3)
            self.dz[self.L].mul_(self.logits > 0)

    def backward_weight(self, i: int, wire=None, update=None, defer_colsum=False):
        """dW (+ db) of layer i into the gradient bucket. ``wire`` (GPU bf16 only): the all-reduce engine's
        prepack target — dW is BFP-encoded straight into the wire shards by the GEMM epilogue. ``update`` (with
        ``wire``, single-rank engine): a :class:`~fpga_ai_nic_amd.ops.gemm.LocalUpdate` — the epilogue applies the
        decoded gradient to this layer's weights in place instead of storing the wire (the layer's bwd-data GEMM,
        which reads the weights, must already be enqueued). ``defer_colsum`` (with ``update``): the bias part may be
        queued on the stream (ops/gemm.py :func:`~fpga_ai_nic_amd.ops.gemm.flush_colsum` completes it)."""
        l = self.layers[i]
        if wire is not None:
            G.linear_bwd_weight(self.act[i], self.dz[i + 1], l.gw, bias_grad=l.gb if self.bias else None, wire=wire,
                                update=update, defer_colsum=defer_colsum)
        elif not self.bias:
            G.linear_bwd_weight(self.act[i], self.dz[i + 1], l.gw)
        elif l.gw.is_cuda and self.dtype == torch.bfloat16:  # bias gradient fused into the bwd-weight GEMM
            G.linear_bwd_weight(self.act[i], self.dz[i + 1], l.gw, bias_grad=l.gb)
        else:
            G.linear_bwd_weight(self.act[i], self.dz[i + 1], l.gw)
            NN.col_sum(self.dz[i + 1], l.gb)

    def backward_data(self, i: int):
        if i == 0:
            return
        l = self.layers[i]
        G.linear_bwd_data(self.dz[i + 1], l.w, self.dz[i], relu_input=self.act[i] if self._relu_at(i - 1) else None)

    def forward(self, x):
        """Inference forward (returns f32 logits)."""
        self.alloc_activations(x.shape[0])
        self.act[0].copy_(x)
        for i in range(self.L):
            self.forward_layer(i)
        return self.logits
