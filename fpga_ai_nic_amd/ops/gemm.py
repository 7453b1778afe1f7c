"""Fully-connected layer GEMMs on the hand-written MFMA kernels (csrc/gemm/).

Weight layout is the reference's checkpoint layout: ``W[in][out]`` row-major (C[i] x C[i+1],
sw/mlp_mpi_example_f32.cpp:396-401). The three products of a layer map onto the kernel's operand
layouts without any transpose pass:

* forward      Y[M,N]  = X[M,K] · W[K,N] (+bias, ReLU)           A K-contig, B MN-contig
* bwd-data     dX[M,K] = dZ[M,N] · W[K,N]ᵀ  (⊙ ReLU mask of X)    A K-contig, B K-contig
* bwd-weight   dW[K,N] = X[M,K]ᵀ · dZ[M,N]                        A MN-contig, B MN-contig

GPU tensors always run the MFMA kernels (unsupported shapes raise); CPU tensors (the gloo / CPU test
path only) use torch reference math in fp32.
"""
from __future__ import annotations

import torch

from .. import _ext

EPI_NONE, EPI_BIAS, EPI_BIAS_RELU, EPI_RELU_MASK, EPI_WIRE = 0, 1, 2, 3, 4

_ws: dict = {}


def _workspace(device, numel):
    """Split-K slab / bias-partial workspace, one per (device, stream): GEMMs issued on different streams (virtual
    ranks on one GPU, side streams) may run at the same time and must not share slabs."""
    key = (device, torch.cuda.current_stream(device).cuda_stream if device.type == "cuda" else 0)
    t = _ws.get(key)
    if t is None or t.numel() < numel:
        t = torch.empty(max(numel, 1 << 20), dtype=torch.float32, device=device)
        _ws[key] = t
    return t


def _bf16_ws_floats(M: int, N: int, sk: int, bm: int, colsum) -> int:
    """f32 workspace of a bf16 GEMM plan: split-K slabs, then bias-gradient partials (split_k per tile row)."""
    return (sk * M * N if sk > 1 else 0) + (sk * (-(-M // bm)) * N if colsum is not None else 0)


def choose_split_k(M: int, N: int, K: int, target_wg: int = 256) -> int:
    """Split K so small output grids still fill the 256 CUs (ordered, deterministic slab reduce)."""
    tiles = (M // 128) * (N // 128)
    if tiles == 0:
        return 1
    best = 1
    for s in (2, 3, 4, 6, 8):
        if tiles * best >= target_wg:
            break
        if K % (64 * s) == 0 and K // s >= 256:
            best = s
    return best


def gemm(A, a_t: bool, B, b_t: bool, C, epilogue: int = EPI_NONE, bias=None, aux=None, accumulate=False,
         split_k: int | None = None, tile: tuple | None = None, colsum=None, wire=None, update=None,
         defer_colsum: bool = False, defer_reduce: dict | None = None):
    """C = op(A)·op(B) with a fused epilogue. a_t: A given as [K][M]; b_t: B given as [N][K].
    ``tile=(BM, BN)`` / ``split_k`` override the kernel planner (bf16 only).
    ``colsum`` (f32 [N]): also write sum_k B(k, n) — the fused bias gradient of bwd-weight (bf16, B [K][N]).
    ``wire=(buf_u8, shard_elems, own_shard, codec_id[, period[, off]])``: BFP-encode the f32 result straight into
    all-reduce wire shards (flat index off + m*ldc + n: ``off`` places a tensor inside a larger bucket; shard
    ``own_shard`` — with ``period``, every shard s with s % period == own_shard — is also written to C) — bf16
    bwd-weight only.
    ``update`` (with ``wire``, single-rank engine): a :class:`LocalUpdate` — the encoded groups are not stored but
    decoded in registers and applied by SGD to the bucket planes in place (the fused local update, see
    csrc/gemm/gemm_bf16_kernel.h WireOut::um).
    ``defer_colsum`` (with ``update`` and ``colsum``): the bias-gradient reduce of an unsplit plan is queued on the
    stream instead of launched — the next split-K wire reduce of the stream runs it in its first blocks, and
    :func:`flush_colsum` launches what is left in one grouped launch (the partials get a workspace of their own);
    ``colsum`` and the bias update are only complete after that.
    ``defer_reduce`` (a dict; f32 ``EPI_BIAS`` output, bf16 operands): when the plan splits K, the slab reduce is not
    launched and C is NOT written — the dict receives ``ws`` (the slabs, [sk][M][N] f32) and ``sk`` for a consumer
    that folds them (:func:`fpga_ai_nic_amd.ops.nn.softmax_xent_slabs`); it stays empty when C was written."""
    if wire is not None:
        if not C.is_cuda or A.dtype != torch.bfloat16 or not a_t or b_t:
            raise ValueError("wire epilogue: bf16 GPU bwd-weight layout only")
        _bf16(_ext.require(), A, a_t, B, b_t, C, EPI_WIRE, None, None, False, split_k, tile, colsum, wire, update,
              defer_colsum=defer_colsum)
        return C
    if update is not None:
        raise ValueError("update needs the wire epilogue")
    if C.is_cuda:
        Cx = _ext.require()
        if colsum is not None and (A.dtype != torch.bfloat16 or b_t):
            from . import nn as _nn

            gemm(A, a_t, B, b_t, C, epilogue, bias, aux, accumulate, split_k, tile)
            _nn.col_sum(B.t() if b_t else B, colsum)
            return C
        if A.dtype == torch.bfloat16:
            if C.dtype == torch.bfloat16 and not _aligned16(C, bias, aux if epilogue == EPI_RELU_MASK else None):
                # the bf16 epilogue stores 16 B per lane: stage misaligned operands through aligned copies
                Ct = torch.empty(C.shape, dtype=C.dtype, device=C.device)
                if accumulate:
                    Ct.copy_(C)
                _bf16(Cx, A, a_t, B, b_t, Ct, epilogue, None if bias is None else bias.clone(),
                      aux if aux is None or epilogue != EPI_RELU_MASK else aux.contiguous().clone(), accumulate,
                      split_k, tile, colsum, None)
                C.copy_(Ct)
                return C
            _bf16(Cx, A, a_t, B, b_t, C, epilogue, bias, aux, accumulate, split_k, tile, colsum, None,
                  defer_reduce=defer_reduce)
            return C
        M = A.shape[1] if a_t else A.shape[0]
        K = A.shape[0] if a_t else A.shape[1]
        N = B.shape[0] if b_t else B.shape[1]
        ws = None
        tbm, tbn, tw = (tuple(tile) + (0,))[:3] if tile is not None else (0, 0, 0)
        sk = Cx.gemm_f32_split(M, N, K, 0 if split_k is None else int(split_k))
        if sk > 1:
            ws = _workspace(C.device, sk * M * N)
        Cx.gemm(A, a_t, B, b_t, C, epilogue, bias, aux, accumulate, sk, ws, tbm, tbn, colsum, tw)
        return C
    # CPU reference path
    a = (A.t() if a_t else A).float()
    b = (B.t() if b_t else B).float()
    r = a @ b
    if epilogue in (EPI_BIAS, EPI_BIAS_RELU):
        r = r + bias.float()
    if epilogue == EPI_BIAS_RELU:
        r = torch.relu(r)
    if epilogue == EPI_RELU_MASK:
        r = r * (aux.float() > 0)
    if accumulate:
        r = r + C.float()
    C.copy_(r.to(C.dtype))
    if colsum is not None:
        colsum.copy_(b.sum(0).to(colsum.dtype))
    return C


def wgrad_group_supported(problems) -> bool:
    """Shapes the grouped bwd-weight launch takes: X [K][M], dY [K][N] bf16 with M % 256, N % 128, K % 64 == 0,
    at most 8 problems (see :func:`gemm_wgrad_group`)."""
    if not 1 <= len(problems) <= 8:
        return False
    for p in problems:
        X, dY = p[0], p[1]
        K, M, N = X.shape[0], X.shape[1], dY.shape[1]
        if M % 256 or N % 128 or K % 64 or dY.shape[0] != K or X.dtype != torch.bfloat16 or not X.is_cuda:
            return False
    return True


def gemm_wgrad_group(problems, wire=None):
    """Up to 8 bwd-weight GEMMs in ONE dispatch: for each ``(X, dY, C, colsum[, off])`` C = X^T . dY (f32, or with
    ``wire=(buf, shard, own, codec[, period])`` BFP-encoded into the bucket's wire buffer at flat offset ``off``,
    the bias segment right after C) and colsum = the column sums of dY (the fused bias gradient). 256x128 tiles, one
    per workgroup, no split-K: a transformer layer's projections (each too small to fill the CUs alone) fill them
    together (csrc/gemm/gemm_group.hip launch_gemm_wgrad_group)."""
    Cx = _ext.require()
    Xs = [p[0] for p in problems]
    dYs = [p[1] for p in problems]
    Cs = [p[2] for p in problems]
    css = [p[3] for p in problems]
    offs = [int(p[4]) if len(p) > 4 else 0 for p in problems]
    ws = _workspace(Cs[0].device, Cx.gemm_wgrad_group_ws([(x.shape[1], y.shape[1]) for x, y in zip(Xs, dYs)]))
    if wire is None:
        Cx.gemm_wgrad_group(Xs, dYs, Cs, css, offs, ws)
    else:
        buf, shard, own, codec = wire[:4]
        period = wire[4] if len(wire) > 4 else 0
        Cx.gemm_wgrad_group(Xs, dYs, Cs, css, offs, ws, buf, int(shard), int(own), int(codec), int(period))


def _aligned16(C, bias, aux) -> bool:
    """A bf16 output's epilogue stores (and the bias / activation loads beside them) are 16 B per lane."""
    ok = C.data_ptr() % 16 == 0 and C.stride(0) % 8 == 0
    if bias is not None:
        ok = ok and bias.data_ptr() % 16 == 0
    if aux is not None:
        ok = ok and aux.data_ptr() % 16 == 0 and aux.stride(0) % 8 == 0
    return ok


def _shares_storage(C, *ts) -> bool:
    c = C.untyped_storage().data_ptr()
    return any(t is not None and t.untyped_storage().data_ptr() == c for t in ts)


class LocalUpdate:
    """SGD target of the fused local update: the bucket planes (flat, padded) and the hyper-parameters, the same
    operation as the engine's decode + SGD epilogue (csrc/bfp/bfp_kernels.hip wire_sgd_kernel)."""

    __slots__ = ("master", "lp", "mom", "lr", "grad_scale", "weight_decay", "momentum", "nesterov")

    def __init__(self, master, lp=None, mom=None, *, lr, grad_scale=1.0, weight_decay=0.0, momentum=0.0,
                 nesterov=False):
        self.master, self.lp, self.mom = master, lp, mom
        self.lr, self.grad_scale, self.weight_decay = float(lr), float(grad_scale), float(weight_decay)
        self.momentum, self.nesterov = float(momentum), bool(nesterov)

    def kwargs(self):
        return dict(upd_master=self.master, upd_lp=self.lp, upd_mom=self.mom, upd_lr=self.lr,
                    upd_grad_scale=self.grad_scale, upd_weight_decay=self.weight_decay, upd_momentum=self.momentum,
                    upd_nesterov=self.nesterov)


_defer_ws: dict = {}


def _colsum_ws(Cx, device, colsum, numel):
    """Workspace of a deferred bias-gradient reduce (one per stream and colsum tensor): its partials must outlive
    the later GEMMs of the stream until the queued reduce runs."""
    key = (device, torch.cuda.current_stream(device).cuda_stream, colsum.data_ptr())
    t = _defer_ws.get(key)
    if t is None or t.numel() < numel:
        if t is not None:
            Cx.gemm_flush_colsum()  # a queued reduce may still read the buffer being replaced
        t = torch.empty(numel, dtype=torch.float32, device=device)
        _defer_ws[key] = t
    return t


def _slab_ws(device, numel):
    """Workspace of a GEMM whose split-K slabs a later kernel folds (defer_reduce): one per stream, not shared with
    the GEMMs that run before that consumer."""
    key = ("slabs", device, torch.cuda.current_stream(device).cuda_stream)
    t = _defer_ws.get(key)
    if t is None or t.numel() < numel:
        t = torch.empty(numel, dtype=torch.float32, device=device)
        _defer_ws[key] = t
    return t


def flush_colsum() -> int:
    """Launch the bias-gradient reduces queued on the current stream by ``defer_colsum`` GEMMs (one grouped launch
    per 8); returns how many ran."""
    if not torch.cuda.is_available():
        return 0
    return int(_ext.require().gemm_flush_colsum())


def pending_colsum() -> int:
    return int(_ext.require().gemm_pending_colsum()) if torch.cuda.is_available() else 0


def _bf16(Cx, A, a_t, B, b_t, C, epilogue, bias, aux, accumulate, split_k, tile, colsum, wire, update=None,
          defer_colsum=False, defer_reduce=None):
    """bf16 MFMA GEMM launch with its plan: explicit (tile / split_k given), tuned on the device on a shape's first
    call (ops/gemm_tune.py), or the static planner's. With a fused ``update`` the tuner's trial launches store the
    wire instead (an update is not re-runnable); the chosen plan then runs once more with the update."""
    M = A.shape[1] if a_t else A.shape[0]
    K = A.shape[0] if a_t else A.shape[1]
    N = B.shape[0] if b_t else B.shape[1]
    tbm, tbn, tw = (tuple(tile) + (0,))[:3] if tile is not None else (0, 0, 0)
    sk0 = 0 if split_k is None else int(split_k)
    static = Cx.gemm_plan(M, N, K, sk0, tbm, tbn, tw)
    if static[0] == 0:
        raise ValueError(f"gemm: unsupported bf16 shape M={M} N={N} K={K} split_k={split_k} tile={tile}")
    if wire is not None:
        buf, shard, own, codec = wire[:4]
        period = int(wire[4]) if len(wire) > 4 else 0
        woff = int(wire[5]) if len(wire) > 5 else 0

    def run(plan, waves=0, upd=None, final=False):
        bm, bn, sk = plan  # launch exactly this tile (re-planning with an explicit split_k differs)
        need = _bf16_ws_floats(M, N, sk, bm, colsum)
        defer = bool(defer_colsum and upd is not None and colsum is not None and sk == 1)
        # (not in the tuner's trial launches: their timing must include the reduce)
        dred = bool(final and defer_reduce is not None and sk > 1 and epilogue == EPI_BIAS and colsum is None
                    and C.dtype == torch.float32 and not accumulate)
        if dred:
            ws = _slab_ws(C.device, need)
        else:
            ws = (_colsum_ws(Cx, C.device, colsum, need) if defer else _workspace(C.device, need)) if need else None
        if wire is not None:
            Cx.gemm(A, a_t, B, b_t, C, EPI_WIRE, None, None, False, sk, ws, bm, bn, colsum, waves, buf, int(shard),
                    int(own), int(codec), period, woff, **(upd.kwargs() if upd is not None else {}),
                    defer_colsum=defer)
        else:
            Cx.gemm(A, a_t, B, b_t, C, epilogue, bias, aux, accumulate, sk, ws, bm, bn, colsum, waves,
                    defer_reduce=dred)
            if dred:
                defer_reduce.update(ws=ws, sk=sk)

    from . import gemm_tune

    T = gemm_tune.tuner()
    if (tile is not None or split_k is not None or not T.enabled or accumulate
            or _shares_storage(C, A, B, aux, bias)):
        run(tuple(static[:3]), tw, update, final=True)
        return
    # a fused-update call shares the key of the wire call (the tuner's trial launches store the wire either way): the
    # fused and the unfused schedule of one shape then run the SAME plan, so their dW rounding — and the weights they
    # train — stay bit-identical (a split-K or tile change alters the summation order)
    k = T.key(M, N, K, a_t, b_t, epilogue, colsum is not None, 0 if wire is None else 1, C.device)
    plan = T.lookup(k)
    if torch.cuda.is_current_stream_capturing():
        # a HIP-graph capture records the plan this shape was tuned to in the eager steps before it (no trial
        # launches while capturing); an untuned shape takes the static plan
        run(plan if plan is not None else tuple(static[:3]), 0, update, final=True)
        return
    if plan is None and not T.worth_tuning(M, N, static, C.device):
        plan = T.keep_static(k, static)
    if plan is None:
        plan = T.tune(k, static, T.candidates(Cx, M, N, K, a_kcontig=not a_t, colsum=colsum is not None), run)
        if update is not None:
            run(plan, 0, update)
    else:
        run(plan, 0, update, final=True)


# ---------------------------------------------------------------------------------------------------------------
# Layer chain: the GEMMs of one MLP pass as ONE persistent launch (csrc/gemm/gemm_chain.hip): layer s + 1's tiles of a
# 256-row panel start as soon as layer s has stored that panel, so the per-launch fill / drain is paid once per pass
# (the reference runs its whole FWD / BWD loop in one OpenMP region, sw/mlp_mpi_example_f32.cpp:690-788). Same tiles,
# same k order as the per-GEMM launches: bit-identical outputs. FAN_GEMM_CHAIN=1 enables it.
CHAIN_FWD, CHAIN_BWD_DATA = 0, 1
_chain_ctr: dict = {}


def chain_enabled() -> bool:
    import os

    return os.environ.get("FAN_GEMM_CHAIN", "0") == "1"


def _chain_counters(key, device, n: int, M: int):
    """The chain's counter block for one call site (key) and stream: zeroed once, left zeroed by every launch."""
    Cx = _ext.require()
    words = int(Cx.gemm_chain_words(n, M))
    sk = (key, device, torch.cuda.current_stream(device).cuda_stream)
    t = _chain_ctr.get(sk)
    if t is None or t.numel() < words:
        if torch.cuda.is_current_stream_capturing():
            return None
        t = torch.zeros(words, dtype=torch.int32, device=device)
        _chain_ctr[sk] = t
    return t


def chain_error(key=None) -> int:
    """Error word of the chain counter blocks (0: none; else 1 + the ready-counter word a spin gave up on). Host sync."""
    worst = 0
    for (k, _, _), t in _chain_ctr.items():
        if key is None or k == key:
            worst = max(worst, int(t[9 * 16].item()))
    return worst


def linear_chain(kind: int, a0, ws, outs, biases=None, auxes=None, epis=None, key="chain", dry_run=False) -> bool:
    """Run the layers' GEMMs as one chain launch; False (nothing launched) when the chain does not take them.
    kind CHAIN_FWD: a0 = X, ws[i] = W_i [K][N], outs[i] = layer outputs (bf16, the last may be f32 logits), biases,
    epis[i] = EPI_BIAS_RELU / EPI_BIAS. kind CHAIN_BWD_DATA: a0 = dZ, ws[i] = W [N][K] used transposed, outs[i] = dX
    (bf16), auxes[i] = the activations whose ReLU mask applies (EPI_RELU_MASK)."""
    if not (chain_enabled() and a0.is_cuda and a0.dtype == torch.bfloat16 and 1 <= len(ws) <= 8):
        return False
    n = len(ws)
    biases = list(biases) if biases is not None else [None] * n
    auxes = list(auxes) if auxes is not None else [None] * n
    epis = list(epis) if epis is not None else [EPI_RELU_MASK if kind == CHAIN_BWD_DATA else EPI_BIAS_RELU] * n
    ctr = _chain_counters(key, a0.device, n, a0.shape[0])
    if ctr is None:
        return False
    return bool(_ext.require().gemm_chain(kind, a0, list(ws), list(outs), biases, auxes, [int(e) for e in epis], ctr,
                                          dry_run))


def linear_fwd(x, w, b, out, relu: bool, defer_reduce: dict | None = None):
    """Y = X · W + b (ReLU); ``defer_reduce`` (no ReLU): see :func:`gemm`."""
    return gemm(x, False, w, False, out, EPI_BIAS_RELU if relu else EPI_BIAS, bias=b,
                defer_reduce=None if relu else defer_reduce)


def linear_bwd_data(dz, w, out, relu_input=None):
    """dX = dZ · Wᵀ, optionally masked by (relu_input > 0) (ReLU backward fused)."""
    if relu_input is not None:
        return gemm(dz, False, w, True, out, EPI_RELU_MASK, aux=relu_input)
    return gemm(dz, False, w, True, out, EPI_NONE)


def linear_bwd_weight(x, dz, out, accumulate=False, bias_grad=None, wire=None, update=None, defer_colsum=False):
    """dW = Xᵀ · dZ (f32 out); with ``bias_grad`` also db = colsum(dZ), fused into the same kernel; with
    ``wire`` dW is written BFP-encoded into the all-reduce wire buffer instead (see :func:`gemm`); with ``update``
    (single-rank engine) the encoded dW updates the weights in place instead (``defer_colsum``: the bias part
    queued, see :func:`gemm`)."""
    if wire is not None:
        return gemm(x, True, dz, False, out, EPI_WIRE, colsum=bias_grad, wire=wire, update=update,
                    defer_colsum=defer_colsum)
    return gemm(x, True, dz, False, out, EPI_NONE, accumulate=accumulate, colsum=bias_grad)
