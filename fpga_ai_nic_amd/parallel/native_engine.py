"""Python face of the native C++ all-reduce engine (csrc/comm/engine.{h,cpp}).

Same request API as :class:`~fpga_ai_nic_amd.parallel.allreduce.CompressedAllReduce` (``layout``,
``allreduce_sgd(defer=...)`` -> handle with ``commit_after_current / wait / synchronize / done /
latency_ms``), but every request is issued by C++: slot bookkeeping, cross-stream events, the mesh / ring
schedule over the engine's own RCCL communicator and the fused decode+SGD epilogue launch — no Python per
kernel or per ring round. This is the counterpart of the reference's C++ host driver
(sw/mlp_mpi_example_f32.cpp:65-180: all_reduce_setup / all_reduce / wait / get_all_reduce_latency):

* completion: 8 request slots; the GPU writes the request's sequence number into host-mapped memory
  (``hipStreamWriteValue32``) the way the NIC DMA-writes ``done_buf[done_id]`` (hw/all_reduce.sv:1368-1375);
  ``synchronize`` polls it with a bounded timeout instead of the reference's unbounded spin (sw:163-168);
* world 1 (no forced collectives): requests run inline on the caller's stream.

GPU only (the engine launches HIP kernels); CPU paths use the Python engine.
"""
from __future__ import annotations

import os
import time

import torch

from .. import _ext
from ..ops import wire
from .allreduce import NUM_SLOTS, BucketLayout, ChecksumError, CommTimeoutError
from .transport import NativeTransport, Transport

_ALGOS = {"mesh": 0, "ring": 1}


class NativeHandle:
    def __init__(self, engine: "NativeAllReduce", slot: int, seq: int, name: str, pending: bool):
        self.engine = engine
        self.slot = slot
        self.seq = seq
        self.name = name
        self.t_issue = time.time()
        self._pending = pending

    def _superseded(self) -> bool:
        return self.engine.C.slot_seq(self.slot) != self.seq

    @property
    def pending(self) -> bool:
        """Epilogue not yet enqueued (a request whose slot was reused was committed by the engine then)."""
        if self._pending and self._superseded():
            self._pending = False
        return self._pending

    def commit(self, update_after=None):
        """Enqueue the deferred epilogue; with ``update_after`` (any truthy value, e.g. an event recorded on
        the current stream) it is ordered after everything enqueued so far on the current stream."""
        if self.pending:
            self.engine.C.commit(self.slot, update_after is not None, self.seq)
            self._pending = False
        return self

    def commit_after_current(self):
        if self.pending:
            self.engine.C.commit(self.slot, True, self.seq)
            self._pending = False
        return self

    def done(self) -> bool:
        if self.pending:
            return False
        return bool(self.engine.C.query(self.slot, self.seq))

    def wait(self, stream=None):
        self.commit_after_current()
        if stream is None:
            self.engine.C.wait_stream(self.slot, self.seq)
        else:
            with torch.cuda.stream(stream):
                self.engine.C.wait_stream(self.slot, self.seq)

    def synchronize(self, timeout: float | None = None):
        self.commit_after_current()
        if self.done():
            try:
                self.engine.C.check_verify()
            except RuntimeError as e:
                raise ChecksumError(f"all-reduce '{self.name}': {e}") from e
            return
        try:
            self.engine.C.synchronize(self.slot, -1.0 if timeout is None else float(timeout), self.seq)
        except RuntimeError as e:
            if "verify:" in str(e):
                raise ChecksumError(f"all-reduce '{self.name}': {e}") from e
            raise CommTimeoutError(f"all-reduce '{self.name}': {e}") from e

    def latency_ms(self) -> float | None:
        if self._pending or self._superseded():
            return None
        v = self.engine.C.latency_ms(self.slot)
        return None if v < 0 else v


class NativeAllReduce:
    """Compressed all-reduce + fused SGD driven entirely from C++."""

    def __init__(self, transport: Transport | None, *, codec: str = "bfp_rne", algo: str = "mesh", rings: int = 1,
                 max_slice_elems: int = 1 << 22, device=None, compat_owner_fp32: bool = False,
                 timeout_s: float = 600.0, stream_priority: int = -1, force_comm: bool = False, comm=None,
                 side_stream: bool = False, verify: bool | None = None, fault: str | None = None,
                 chunk_elems: int = 0, links="auto", ring_sub: int = 0, shard_update: bool | None = None):
        """``comm``: an explicit ``_C.Comm`` (e.g. ``_C.LoopbackFabric(N).comm(r)`` for virtual ranks on one
        GPU); otherwise the engine's own RCCL communicator is created from ``transport``. ``side_stream``
        (world 1): run requests on the engine's comm stream instead of inline (overlap measurements).
        ``verify`` (default: env FAN_VERIFY): debug mode — every message carries a GPU-computed checksum + the
        request sequence number, checked on arrival (csrc/comm/verify.h); ``fault``: test-only fault injection
        rules (FAN_FAULT grammar, default from the environment). ``chunk_elems`` (mesh, multi-rank): buckets above it
        stream through the collectives in chunks — all-to-all / owner reduce / all-gather / epilogue pipelined over
        two streams with scratch bounded by two chunks (0: env FAN_CHUNK_ELEMS, default 64 Mi elements).
        ``links`` (ring): direct-link matrix the rings must follow (``"auto"``: this node's xGMI links from
        :func:`~fpga_ai_nic_amd.utils.topology.link_matrix`; None: fully connected). ``ring_sub`` (direct-P2P ring):
        each hop's message streams in this many sub-slices with a ready flag each, so the downstream rank starts on
        sub-slice s while this one still encodes the rest (0: env FAN_RING_SUB, default 1 = lock-step hops; capped at
        the P2P arena depth - 1). ``shard_update`` (mesh, multi-rank; default env FAN_SHARD_UPDATE): the owner of each
        shard fuses its reduce with the SGD of that shard and the ranks all-gather the updated bf16 weights (ZeRO-1
        style: master / momentum current on the owner only, :meth:`gather_owned` collects them); update requests of
        bf16 buckets write the ``lp`` they are given (the trainer's next weight buffer) and need no deferred
        epilogue."""
        if algo not in _ALGOS:
            raise ValueError(f"unknown algo {algo!r}")
        C = _ext.require()
        self.transport = transport
        self.rank = transport.rank if transport is not None else 0
        self.world = transport.world if transport is not None else 1
        if comm is not None:
            self.rank, self.world = comm.rank, comm.world
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        if self.device.type != "cuda":
            raise RuntimeError("the native engine runs on GPU only")
        if comm is None and (self.world > 1 or force_comm):
            if not isinstance(transport, NativeTransport):
                transport = NativeTransport(self.rank, self.world, self.device.index, force_collectives=force_comm)
                self.transport = transport
            comm = transport.comm
        self.codec, self.codec_id, self.algo = codec, wire.codec_id(codec), algo
        self.timeout_s = timeout_s
        if isinstance(links, str):
            links = None
            if algo == "ring" and self.world > 1 and not isinstance(comm, C.LoopbackComm):
                from ..utils import topology

                links = topology.agreed_link_matrix(self.world)  # rank 0 decides, every rank plans the same rings
        self.links = links
        if os.environ.get("FAN_COMM_PRIORITY"):  # comm / aux stream priority override (-1 high, 0 normal)
            stream_priority = int(os.environ["FAN_COMM_PRIORITY"])
        self.C = C.AllReduceEngine(comm, self.rank, self.world, self.codec_id, _ALGOS[algo], rings, max_slice_elems,
                                   compat_owner_fp32, timeout_s, stream_priority, force_comm or side_stream,
                                   self.device.index, -1 if verify is None else int(bool(verify)), int(chunk_elems),
                                   links, int(ring_sub), -1 if shard_update is None else int(bool(shard_update)))
        self.ring_sub = int(self.C.ring_sub)
        self.shard_update = bool(self.C.shard_update)
        if fault is not None:
            self.C.set_fault(fault)
        self.verify = bool(self.C.verify)
        self.orders = [list(o) for o in self.C.orders]
        self.rings = len(self.orders)
        self.inline = bool(self.C.inline)
        self.cuda = True
        # producers (the bwd-weight GEMM) may write BFP wire shards directly: see prepack_target()
        self.prepack = self.C.prepack_shape(1 << 20)[0] > 0
        self._prepack_bufs: dict = {}
        self._timing = False
        self.stats = {"requests": 0, "wire_bytes": 0, "logical_bytes": 0}
        # Side-stream engines run their decode+SGD epilogues on the committing (compute) stream by default
        # (1.22 vs 1.25 ms/step on the forced 1-rank RCCL path, profiles/r1_null_stream_commit_fix.txt);
        # FAN_EPI=comm runs them on the comm stream, committed per layer. Both train bit-identically to the
        # inline engine since commit() stopped reading torch's default stream (handle 0) as "no producer".
        self.epilogue_on_producer = os.environ.get("FAN_EPI", "producer") != "comm"

    def gather_owned(self, plane: torch.Tensor, n: int):
        """Sharded-update engines: all-gather an owner-sharded f32 bucket plane (a layer's master or momentum) in
        place, so every rank holds the whole plane (checkpoints, replica checks). Collective; no-op otherwise."""
        if self.shard_update:
            self.C.gather_owned(plane.view(-1), int(n))

    @property
    def timing(self):
        return self._timing

    @timing.setter
    def timing(self, on):
        self._timing = bool(on)
        self.C.set_timing(self._timing)

    @property
    def epilogue_on_producer(self) -> bool:
        """Side-stream engine: each request's decode+SGD epilogue runs on the stream that commits it (after the
        request's communication phase) rather than on the comm stream, so it never shares CUs with the
        producer's GEMMs. Callers then commit once the producer's overlapped work is enqueued (the trainer
        commits all of a step's requests after the last backward GEMM)."""
        return bool(self.C.epilogue_on_producer)

    @epilogue_on_producer.setter
    def epilogue_on_producer(self, on):
        self.C.epilogue_on_producer = bool(on) and not self.inline

    @property
    def stream(self):
        return torch.cuda.ExternalStream(self.C.stream, device=self.device)

    def layout(self, n: int, shard: int = 0, chunks: int = 0) -> BucketLayout:
        """Bucket layout; ``shard`` / ``chunks`` > 0: an explicit chunked mesh layout."""
        d = self.C.layout(int(n), int(shard), int(chunks))
        return BucketLayout(n=d["n"], n_pad=d["n_pad"], algo=self.algo, world=self.world, shard=d["shard"],
                            slice_elems=d["slice"], blocks=d["blocks"], rings=d["rings"], part=d["part"],
                            chunks=d["chunks"], sub=d["sub"])

    def wire_bytes(self, L: BucketLayout) -> int:
        return int(self.C.wire_bytes(L.n))

    def prepack_target(self, grad: torch.Tensor, n: int, static_from: int | None = None, layout=None):
        """Wire target for a producer that encodes the gradient itself (GEMM ``kEpiWire`` epilogue):
        ``(wire_u8, shard_elems, own_shard, codec_id, period)`` — one persistent buffer per gradient bucket — or None
        when this configuration (ring / raw codec) cannot take prepacked input.

        ``static_from``: flat elements [static_from, padded end) are always zero (padding, or a bias segment
        the model does not have); they are encoded once here, so the producer's encoding plus this tail is
        the whole bucket (pass ``prepacked=(buf, layout(n).n_pad)``)."""
        shard, shards, own = self.C.prepack_shape(int(n))
        if shard == 0 or n % 16:
            return None
        if layout is not None:  # explicit chunked layout: shard x world x chunks
            shard, shards = int(layout[0]), int(layout[1]) * self.world
        need = shards * wire.shard_bytes(self.codec_id, shard)
        static_from = n if static_from is None else int(static_from)
        key = (grad.data_ptr(), static_from, shard, shards)
        buf = self._prepack_bufs.get(key)
        if buf is None or buf.numel() < need:
            buf = torch.empty(need, dtype=torch.uint8, device=self.device)
            total = shard * shards
            if static_from < total:
                _ext.require().wire_pack_range(torch.zeros(total, device=self.device), buf, shard, static_from,
                                               total, self.codec_id)
            self._prepack_bufs[key] = buf
        return buf, shard, own, self.codec_id, self.world  # owner shard period: one owner shard per chunk

    def allreduce_sgd(self, grad: torch.Tensor, master: torch.Tensor, lp: torch.Tensor | None = None,
                      mom: torch.Tensor | None = None, *, n_valid: int | None = None, lr: float,
                      grad_scale: float = 1.0, weight_decay: float = 0.0, momentum: float = 0.0,
                      nesterov: bool = False, update_after=None, defer: bool = False,
                      name: str = "bucket", prepacked=None, layout=None, on_producer: bool = False) -> NativeHandle:
        """``prepacked=(wire_u8, elems)``: flat elements [0, elems) were already encoded into ``wire_u8``
        (from :meth:`prepack_target`); the engine encodes the rest and skips its pack pass. ``layout=(shard,
        chunks)``: an explicit chunked mesh layout (shard elements x world x chunks). ``on_producer``: run the request on the
        current (producer) stream instead of the engine's comm stream — the last request of a backward, which has
        nothing left to overlap with (saves two cross-stream hand-offs on the critical path)."""
        n_valid = int(n_valid if n_valid is not None else master.numel())
        pre, pre_n = (None, 0) if prepacked is None else prepacked
        ls, lc = (0, 0) if layout is None else (int(layout[0]), int(layout[1]))
        # an immediate request (no ordering after the producer's later work) is committed by the engine itself, so
        # a chunked bucket runs its per-chunk epilogues inside the pipeline (bounded scratch)
        eng_defer = defer or update_after is not None
        slot = self.C.submit(grad.view(-1), master.view(-1), None if lp is None else lp.view(-1),
                             None if mom is None else mom.view(-1), n_valid, lr, grad_scale, weight_decay, momentum,
                             nesterov, eng_defer, True, None, pre, int(pre_n), ls, lc, bool(on_producer))
        h = NativeHandle(self, slot, self.C.slot_seq(slot), name, pending=eng_defer)
        self._account(n_valid)
        return h if defer else h.commit(update_after)

    def allreduce(self, grad: torch.Tensor, out: torch.Tensor, *, n_valid: int | None = None,
                  name: str = "bucket", prepacked=None) -> NativeHandle:
        """Sum-only all-reduce: decoded f32 result written to ``out`` (padded length)."""
        n_valid = int(n_valid if n_valid is not None else grad.numel())
        if out.dtype != torch.float32:
            raise TypeError("native allreduce writes f32 sums")
        pre, pre_n = (None, 0) if prepacked is None else prepacked
        slot = self.C.submit(grad.view(-1), out.view(-1), None, None, n_valid, 0.0, 1.0, 0.0, 0.0, False, False,
                             False, out.view(-1), pre, int(pre_n))
        self._account(n_valid)
        return NativeHandle(self, slot, self.C.slot_seq(slot), name, pending=False)

    def _account(self, n):
        self.stats["requests"] += 1
        self.stats["wire_bytes"] += self.C.wire_bytes(n)
        self.stats["logical_bytes"] += n * 4

    def diagnostics(self, h: NativeHandle) -> str:
        return self.C.diagnostics(h.slot)

    def debug_status(self) -> dict:
        """Snapshot of the engine (the NIC's debug_status register, hw/all_reduce.sv:1415-1421): configuration,
        every request slot, per-peer bytes, communicator error and, on the P2P transport, its flag words and
        device stall counters."""
        import json

        return json.loads(self.C.debug_status())

    def counters(self) -> dict:
        """Engine perf counters (reference: the NIC's lpbk_latency / stall_host registers read by
        get_all_reduce_latency / get_host_stall_cycles, sw/mlp_mpi_example_f32.cpp:100-112): requests, logical and
        wire bytes, host time blocked in synchronize(), summed device time of timed requests."""
        return dict(self.C.counters())

    def reset_counters(self):
        self.C.reset_counters()

    def trace(self, on: bool = True, capacity: int = 1024):
        """Start (reset) or stop device-side request tracing: GPU timestamps at every phase boundary of each
        request (pack / all-to-all / reduce / all-gather / epilogue), see :meth:`trace_summary`."""
        self.C.set_tracing(bool(on), int(capacity))

    def trace_summary(self) -> dict:
        """Per-phase device time (ms) summed over the requests traced since :meth:`trace` — the NIC's per-state
        cycle counters (hw/all_reduce.sv:892-1085) — plus ``comm_ms`` (request start to end of the all-gather)
        and the traced requests' logical / wire bytes. Waits for the traced requests."""
        return dict(self.C.trace_summary())


__all__ = ["NativeAllReduce", "NativeHandle", "NUM_SLOTS"]
