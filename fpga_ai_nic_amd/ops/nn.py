"""Loss and reduction kernels (csrc/nn/nn_kernels.hip) with CPU reference fallbacks."""
from __future__ import annotations

import torch

from .. import _ext

_ws: dict = {}


def softmax_xent(logits: torch.Tensor, labels: torch.Tensor, dlogits: torch.Tensor, loss_rows: torch.Tensor,
                 grad_scale: float):
    """Fused softmax + cross-entropy: writes per-row loss and dlogits = (softmax - onehot) * grad_scale."""
    if logits.is_cuda:
        _ext.require().softmax_xent(logits, labels, dlogits, loss_rows, float(grad_scale))
        return
    x = logits.float()
    lse = torch.logsumexp(x, dim=1)
    loss_rows.copy_(lse - x.gather(1, labels.long().view(-1, 1)).view(-1))
    p = torch.softmax(x, dim=1)
    p[torch.arange(x.shape[0]), labels.long()] -= 1.0
    dlogits.copy_((p * grad_scale).to(dlogits.dtype))


def softmax_xent_slabs(slabs: dict, bias: torch.Tensor, logits: torch.Tensor, labels: torch.Tensor,
                       dlogits: torch.Tensor, loss_rows: torch.Tensor, grad_scale: float):
    """:func:`softmax_xent` over the classifier GEMM's unreduced split-K slabs (``slabs`` from ``ops.gemm.gemm``'s
    ``defer_reduce``): logits = the slabs' sum in split order + bias, as the GEMM's own reduce computes them (also
    written to ``logits``), then the fused softmax + cross-entropy — one launch instead of two."""
    _ext.require().softmax_xent_slabs(slabs["ws"], int(slabs["sk"]), bias, logits, labels, dlogits, loss_rows,
                                      float(grad_scale))


def col_sum(x: torch.Tensor, out: torch.Tensor, scale: float = 1.0, accumulate: bool = False):
    """out[n] (+)= scale * sum_m x[m][n] (bias gradient)."""
    if x.is_cuda:
        C = _ext.require()
        M, N = x.shape
        need = C.col_sum_workspace_floats(M, N)
        key = (x.device, torch.cuda.current_stream(x.device).cuda_stream)  # per stream: concurrent callers
        ws = _ws.get(key)
        if ws is None or ws.numel() < need:
            ws = torch.empty(max(need, 1 << 16), dtype=torch.float32, device=x.device)
            _ws[key] = ws
        C.col_sum(x, out, float(scale), bool(accumulate), ws)
        return out
    s = x.float().sum(0) * scale
    if accumulate:
        s = s + out.float()
    out.copy_(s.to(out.dtype))
    return out
