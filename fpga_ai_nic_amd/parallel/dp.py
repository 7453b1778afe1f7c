"""Data-parallel trainer: per-layer gradient all-reduce overlapped with backward on a side HIP stream.

Reference schedule (sw/mlp_mpi_example_f32.cpp:701-787): forward all layers; softmax fwd/bwd; for layer
i = L-1..0: backward, then issue the NIC all-reduce(+SGD) of layer i asynchronously while layer i-1's
backward runs. MI355X mapping:

* main stream: fwd GEMMs (bias+ReLU fused), softmax-xent, bwd-weight GEMM of layer i, then bwd-data GEMM;
* comm stream (high priority): as soon as dW_i is written, the engine packs + exchanges layer i's bucket
  (overlapping the bwd-data GEMM of layer i and the whole backward of layers < i);
* the fused SGD epilogue of layer i waits (GPU-side event) for the bwd-data GEMM that still reads W_i;
* the NEXT step's forward of layer i waits (GPU-side event) for that epilogue — the host never blocks.
"""
from __future__ import annotations

import os
import time

import torch

from ..models.mlp import MLP
from ..ops import gemm as G
from ..ops import wire
from ..utils import tracing
from .allreduce import CompressedAllReduce, Handle, _round_up
from .transport import Transport


class RcclAllReduce(CompressedAllReduce):
    """Uncompressed baseline: transport all-reduce (RCCL ring/tree) + a separate SGD kernel
    (BASELINE config 2; the reference's commented MPI_Iallreduce path, sw:615-647)."""

    def __init__(self, transport: Transport, **kw):
        kw.pop("codec", None)
        kw.pop("algo", None)
        super().__init__(transport, codec="raw_f32", algo="mesh", **kw)
        self.algo = "rccl"

    def layout(self, n):
        from .allreduce import BucketLayout

        n_pad = _round_up(max(n, 1), 256 * self.world)
        return BucketLayout(n=n, n_pad=n_pad, algo="rccl", world=self.world, shard=n_pad)

    def wire_bytes(self, L):
        N = self.world
        return 0 if N == 1 else int(2 * (N - 1) / N * L.n_pad * 4)

    def _run(self, L, grad, finish, owner_fp32, allow_compat=True):
        g = grad.view(-1)[: L.n_pad]
        self.transport.all_reduce_(g)
        return [lambda: finish(wire.as_bytes(g), L.n_pad, 1, 0, L.n_pad)]


def make_engine(transport: Transport | None, kind: str = "bfp", *, rounding: str = "rne", algo: str = "mesh",
                rings: int = 1, max_slice_elems: int = 1 << 22, compat_owner_fp32: bool = False,
                timeout_s: float = 600.0, force_comm: bool = False, impl: str = "python", comm=None,
                side_stream: bool = False, ring_sub: int = 0, shard_update: bool | None = None):
    """kind: 'bfp' (compressed engine), 'raw' (engine, uncompressed fp32 wire), 'rccl' (baseline),
    'local' (no communication: world 1). impl: 'python' (request path issued from Python over any
    transport) or 'native' (C++ engine over its own RCCL communicator, or over ``comm``, e.g. the direct P2P
    communicator of :func:`~fpga_ai_nic_amd.parallel.transport.make_p2p_comm`; GPU only)."""
    if kind == "local" or transport is None:
        return None
    if kind == "rccl":
        return RcclAllReduce(transport, timeout_s=timeout_s, force_comm=force_comm)
    codec = {"bfp": f"bfp_{rounding}", "raw": "raw_f32", "raw_bf16": "raw_bf16"}[kind]
    if impl == "native":
        from .native_engine import NativeAllReduce

        return NativeAllReduce(transport, codec=codec, algo=algo, rings=rings, max_slice_elems=max_slice_elems,
                               compat_owner_fp32=compat_owner_fp32, timeout_s=timeout_s, force_comm=force_comm,
                               comm=comm, side_stream=side_stream, ring_sub=ring_sub, shard_update=shard_update)
    return CompressedAllReduce(transport, codec=codec, algo=algo, rings=rings, max_slice_elems=max_slice_elems,
                               compat_owner_fp32=compat_owner_fp32, timeout_s=timeout_s, force_comm=force_comm)


class DataParallelTrainer:
    def __init__(self, model: MLP, engine: CompressedAllReduce | None, *, lr: float = 0.1,
                 weight_decay: float = 0.0, momentum: float = 0.0, nesterov: bool = False,
                 loss_scale: float = 1.0, average: bool = True, profile: bool = False, prepack: bool = True,
                 commit_at_end: bool | None = None, fused_update: bool | None = None,
                 gemm_inflight: str | None = None):
        """``fused_update`` (default env FAN_FUSED_UPDATE, else on): with a single-rank engine (world 1, requests
        inline: the all-reduce of one rank is the identity) and the GEMM-encoded wire, the bwd-weight GEMM's epilogue
        takes each encoded gradient group through its BFP round trip in registers and applies the SGD update to the
        layer's weights in place — the engine's decode + SGD pass over the whole bucket (master read + write, bf16
        copy write, wire read) disappears into the GEMM. Same operations in the same order: bit-identical weights
        to the unfused schedule. The layer's bwd-data GEMM (which reads the weights) is issued first.

        ``gemm_inflight`` (default env FAN_GEMM_INFLIGHT, else 'persistent'): the GEMM form while a request of this
        step is in flight on the side stream (multi-rank engines only). 'persistent': one 4-wave workgroup per CU
        looping over tiles — it holds every CU until it ends, so the comm stream's kernels start only at GEMM
        boundaries; 'grid': one workgroup per tile from the first submit to the end of backward, so comm kernels
        start at tile boundaries (the forced 1-rank path's comm phase took half the device time that way,
        profiles/r3_persist_vs_tile_grid_forced.txt). bench.py picks between them by timing both at world > 1."""
        self.m = model
        self.engine = engine
        self.world = engine.world if engine is not None else 1
        self.lr, self.wd, self.momentum, self.nesterov = lr, weight_decay, momentum, nesterov
        self.loss_scale = loss_scale
        # gradients are of the LOCAL mean loss; the all-reduce sums over ranks -> average with 1/N
        self.grad_scale = (1.0 / self.world) if average else 1.0
        self.pending: list[Handle | None] = [None] * model.L
        self.last_handle: Handle | None = None
        self.cuda = model.device.type == "cuda"
        self.profile = profile
        self.times = {"fwd": 0.0, "loss": 0.0, "bwd": 0.0, "bwd_first": 0.0, "steps": 0}
        self.step_count = 0
        # fuse the BFP encode into the bwd-weight GEMM when the engine accepts prepacked wire input
        # commit every request's epilogue after the whole backward is enqueued (required when the engine runs
        # epilogues on the compute stream: a per-layer commit would stall it on that layer's communication)
        self.commit_at_end = (bool(getattr(engine, "epilogue_on_producer", False)) if commit_at_end is None
                              else commit_at_end)
        self.prepack = (prepack and engine is not None and getattr(engine, "prepack", False) and self.cuda
                        and model.dtype == torch.bfloat16)
        fu = os.environ.get("FAN_FUSED_UPDATE", "1") != "0" if fused_update is None else bool(fused_update)
        self.fused_update = (fu and self.prepack and bool(getattr(engine, "inline", False))
                             and getattr(engine, "codec", "") == "bfp_rne")
        self.fused_updates = 0
        # fused update: the layers' bias-gradient reduces of unsplit bwd-weight plans are queued and run by the next
        # split-K wire reduce of the backward, or all in one grouped launch after it (FAN_DEFER_COLSUM=0: one launch
        # each, right after its GEMM; bit-identical either way)
        self.defer_colsum = os.environ.get("FAN_DEFER_COLSUM", "1") != "0"
        # a split-K classifier GEMM leaves its slabs to the softmax-xent kernel, which folds them (FAN_FOLD_LOGITS=0:
        # the GEMM's own slab reduce launch; bit-identical either way)
        self.fold_logits = os.environ.get("FAN_FOLD_LOGITS", "1") != "0"
        # layer-chain launches (ops/gemm.py linear_chain, FAN_GEMM_CHAIN): the forward at every world size; the
        # bwd-data chain only with the fused world-1 update — with a multi-rank engine each layer's all-reduce is
        # issued right after its own bwd-weight GEMM and overlaps that layer's bwd-data GEMM, which a chain of the
        # bwd-data GEMMs would postpone
        self.chain_fwd = G.chain_enabled()
        self.chain_bwd = G.chain_enabled()
        gi = os.environ.get("FAN_GEMM_INFLIGHT", "persistent") if gemm_inflight is None else gemm_inflight
        if gi not in ("persistent", "grid"):
            raise ValueError(f"gemm_inflight must be persistent|grid, got {gi!r}")
        self.gemm_inflight = gi if (self.cuda and engine is not None and not getattr(engine, "inline", True)) \
            else "persistent"
        self._persist_saved = None
        # sharded-update engine (bf16 model): each request writes the layer's NEXT weight buffer (lp_next), which no
        # GEMM of this step reads, so it needs no ordering after the layer's bwd-data GEMM; the buffers swap once the
        # step's backward is enqueued (the next forward waits for its layer's request, _wait_layer)
        self.shard = bool(getattr(engine, "shard_update", False)) and self.cuda and model.dtype == torch.bfloat16
        self.lp_next = [l.lp.clone() if self.shard else None for l in model.layers]
        # multi-rank native engine: layer 0's request (the backward's last) on the compute stream itself
        # (FAN_LAST_ON_PRODUCER=0: on the comm stream like the others)
        self.last_on_producer = (self.cuda and engine is not None and not getattr(engine, "inline", True)
                                 and hasattr(engine, "C") and os.environ.get("FAN_LAST_ON_PRODUCER", "1") != "0")

    def _sgd_local(self, l):
        wire.sgd(wire.as_bytes(l.grad), l.n_pad, 1, l.master, codec="raw_f32", lp=l.lp, mom=l.mom, lr=self.lr,
                 grad_scale=self.grad_scale, weight_decay=self.wd, momentum=self.momentum, nesterov=self.nesterov,
                 n_valid=l.n)

    def step(self, x: torch.Tensor, labels: torch.Tensor):
        """One training iteration (reference type 'A': FWD + loss + BWD + all-reduce/UPD)."""
        self.forward_pass(x)
        self.backward_pass(labels)
        self.times["steps"] += 1
        self.step_count += 1
        return self.m.loss_rows

    def forward_pass(self, x: torch.Tensor):
        """Forward of every layer (reference type 'F' times this plus the loss forward)."""
        m = self.m
        m.alloc_activations(x.shape[0])
        m.act[0] = x
        t0 = time.perf_counter()
        with tracing.range("fwd"):
            # the whole forward as one layer-chain launch when it takes the model (every layer's update must have
            # landed first: layer 0's, the last request of the backward, is the one it waits on in practice)
            if self.cuda and self.chain_fwd:
                for i in range(m.L):
                    self._wait_layer(i)
                chained = m.forward_chain()
            else:
                chained = False
            if not chained:
                for i in range(m.L):
                    self._wait_layer(i)  # layer i's weights updated (reference: per-layer wait, sw:757-787)
                    m.forward_layer(i, fold_logits=self.fold_logits and self.cuda)
            self.last_handle = None
        if self.profile:
            self._sync()
            self.times["fwd"] += time.perf_counter() - t0

    def _wait_layer(self, i: int):
        """Layer i's weights must be updated before its forward reads them: a GPU-side wait on layer i's
        request(s) only (free when its epilogue already runs on this stream), so layer i's forward starts as soon
        as ITS update lands rather than after the whole step's (reference: the host waits per layer request,
        sw/mlp_mpi_example_f32.cpp:757-787)."""
        h = self.pending[i]
        if h is None:
            return
        for x in (h if isinstance(h, list) else [h]):
            if self.cuda:
                x.wait()
            else:
                x.synchronize()
        self.pending[i] = None

    def _wait_updates(self):
        """Every outstanding update has landed (GPU-side order on the current stream; host waits on CPU)."""
        for i in range(self.m.L):
            self._wait_layer(i)
        self.last_handle = None

    def backward_pass(self, labels: torch.Tensor):
        """Loss fwd+bwd, then per layer L-1..0: dW -> async all-reduce+SGD -> dX (reference type 'B')."""
        m = self.m
        prof = self.profile
        self._wait_updates()  # no-op after forward_pass; needed when backward passes run back to back
        t0 = time.perf_counter()
        with tracing.range("loss"):
            m.loss_backward(labels, grad_scale=self.loss_scale / m.act[0].shape[0])
        if prof:
            self._sync()
            t1 = time.perf_counter()
            self.times["loss"] += t1 - t0
            t0 = t1
        # world 1 with the fused update on every layer: the bwd-data GEMMs of layers L-1 .. 1 as one layer-chain
        # launch first (each layer's weights are read there before its bwd-weight GEMM updates them in place)
        tgts = [(self.engine.prepack_target(l.grad, l.n, None if m.bias else l.cin * l.cout)
                 if self.prepack and l.cout % 16 == 0 else None) for l in m.layers]
        chained = (self.fused_update and self.chain_bwd and all(t is not None for t in tgts)
                   and m.backward_data_chain())
        try:
            for i in reversed(range(m.L)):
                l = m.layers[i]
                with tracing.range(f"bwd{i}"):
                    # the bwd-weight GEMM encodes dW (and the fused bias gradient) straight into the wire buffer;
                    # the zero tail (padding, or the bias segment of a bias-free model) is encoded once
                    # (the wire epilogue encodes whole 16-column groups: output widths that are multiples of 16)
                    tgt = tgts[i]
                    if tgt is not None and self.fused_update:
                        # single-rank engine: bwd-data first (it reads W_i), then dW's BFP round trip + SGD in the
                        # bwd-weight epilogue
                        if not chained:
                            m.backward_data(i)
                        upd = G.LocalUpdate(l.master, l.lp, l.mom, lr=self.lr, grad_scale=self.grad_scale,
                                            weight_decay=self.wd, momentum=self.momentum, nesterov=self.nesterov)
                        # (the bwd-weight GEMMs of layers >= 1 on a second stream, beside the next GEMM, measured 1.5-2 %
                        # slower: profiles/r3_fused_update_ab.txt)
                        m.backward_weight(i, wire=tgt, update=upd, defer_colsum=self.defer_colsum)
                        self.fused_updates += 1
                    else:
                        m.backward_weight(i, wire=tgt)
                        h = None
                        if self.engine is not None:
                            kw = {"prepacked": (tgt[0], l.n_pad)} if tgt is not None else {}
                            lp_out = self.lp_next[i] if self.shard else l.lp
                            if i == 0 and self.last_on_producer:
                                # the backward's last request: nothing left to overlap it with, so it runs on this
                                # stream (no hand-off to the comm stream and back before the next forward)
                                kw["on_producer"] = True
                            h = self.engine.allreduce_sgd(l.grad, l.master, lp_out, l.mom, n_valid=l.n, lr=self.lr,
                                                          grad_scale=self.grad_scale, weight_decay=self.wd,
                                                          momentum=self.momentum, nesterov=self.nesterov, defer=True,
                                                          name=f"fc{i}", **kw)
                            self._gemm_grid(True)
                        m.backward_data(i)
                        if h is not None:
                            self.pending[i] = h if self.commit_at_end else h.commit_after_current()
                            self.last_handle = self.pending[i]
                        else:
                            self._sgd_local(l)
                if prof and i == m.L - 1:
                    self._sync()
                    t1 = time.perf_counter()
                    self.times["bwd_first"] += t1 - t0
                    self.times["bwd"] += t1 - t0
                    t0 = t1
        finally:
            # the bias updates still queued (every layer's lands before the next forward; after an exception too, so
            # no queued reduce is left for an unrelated later GEMM of the stream to run)
            if self.fused_updates and self.defer_colsum and self.cuda:
                G.flush_colsum()
            # the grid GEMM form must not outlive this backward (an exception in between would leave every later
            # GEMM of the process on one workgroup per tile while records report the persistent form)
            self._gemm_grid(False)
        if self.shard:  # this step's requests write lp_next: it holds the weights the next forward uses
            for i, l in enumerate(m.layers):
                l.lp, self.lp_next[i] = self.lp_next[i], l.lp
        if self.commit_at_end:  # issue order L-1..0: the epilogues run in the order their all-reduces finish
            for i in reversed(range(m.L)):
                h = self.pending[i]
                for x in (h if isinstance(h, list) else [] if h is None else [h]):
                    x.commit_after_current()
        if prof:
            self._sync()
            self.times["bwd"] += time.perf_counter() - t0

    def _gemm_grid(self, on: bool):
        """gemm_inflight='grid': GEMMs enqueued while a request is in flight run one workgroup per tile."""
        if self.gemm_inflight != "grid":
            return
        from .. import _ext

        C = _ext.require()
        if on and self._persist_saved is None:
            self._persist_saved = C.gemm_persist()
            C.gemm_set_persist(0)
        elif not on and self._persist_saved is not None:
            C.gemm_set_persist(self._persist_saved)
            self._persist_saved = None

    def _sync(self):
        if self.cuda:
            torch.cuda.synchronize()

    def finish_async(self):
        """GPU-side: order the current stream after every outstanding update (no host wait; usable while
        capturing a HIP graph)."""
        self._wait_updates()

    def gather_state(self):
        """Sharded-update engine: collect every layer's owner-sharded master (and momentum) onto every rank, so the
        planes are whole again (checkpoint, replica check). Collective; a no-op for other engines."""
        if not self.shard:
            return
        self.finish()
        for l in self.m.layers:
            self.engine.gather_owned(l.master, l.n)
            if l.mom is not None:
                self.engine.gather_owned(l.mom, l.n)

    def finish(self, timeout: float | None = None):
        """Wait (host) for every outstanding all-reduce/update."""
        self._gemm_grid(False)
        for i, h in enumerate(self.pending):
            if h is not None:
                for x in (h if isinstance(h, list) else [h]):
                    x.synchronize(timeout)
                self.pending[i] = None
        self.last_handle = None
        self._sync()
