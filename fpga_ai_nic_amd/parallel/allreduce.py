"""Compressed all-reduce engine with the SGD weight update fused into the all-gather epilogue.

This is the MI355X-native replacement for the reference NIC (hw/all_reduce.sv + hw/weight_update.sv +
hw/bfp_adapter.sv) and its host driver (sw/mlp_mpi_example_f32.cpp:65-180):

* request API ``allreduce_sgd(grad, weights, ...) -> Handle`` mirrors ``all_reduce(buf, weight_out, flags,
  done, count)`` + ``wait(done)`` (sw:114-180); completion slots round-robin 0..7 like the NIC's 3-bit
  ``done_id`` (hw/all_reduce.sv:1228, 1373). ``Handle.synchronize(timeout)`` replaces the reference's
  unbounded busy-spin (sw:163-168) with a bounded wait + diagnostics.
* weights live in HBM next to the gradients; the epilogue decodes the reduced gradient and applies
  ``w = fma(-lr, g, w)`` (hw/weight_update.sv:442-451) in place — with lr / grad scaling / momentum /
  weight decay as runtime parameters instead of the hard-coded 0.1.
* every rank applies the update to the SAME decoded values (owner included), so replicas stay
  bit-identical (the reference's owner used the un-quantised sum: SURVEY.md §2.6 quirk; available as
  ``compat_owner_fp32=True`` on the ring algorithm).

Algorithms
----------
``mesh`` (default on xGMI): pack -> all-to-all -> owner sums its shard (local contribution un-quantised)
-> re-encode -> all-gather -> fused decode+SGD. On a fully connected 8-GPU xGMI node every link carries
traffic at once, and every contribution is quantised once (instead of N-1 re-quantisations in a ring).

``ring``: the reference schedule (SEND_LOCAL, REDUCE x(N-2), REDUCE_OUTPUT, FORWARD_OUTPUT x(N-2)),
planned natively (``_C.ring_plan``), generalised to any N >= 1 and to R arc-disjoint directed rings
(``_C.ring_orders``: 7 rings on 8 GPUs so each of the 7 xGMI links of a GPU carries one ring). Each hop is
one fused HIP kernel (decode recv + add local + re-encode); all-gather hops forward the encoded bytes
untouched (re-encoding a decoded group is idempotent).
"""
from __future__ import annotations

import math
import os
import time
from dataclasses import dataclass, field

import torch

from .. import _ext
from ..ops import wire
from ..utils import faults
from .transport import Transport

NUM_SLOTS = 8  # reference: 3-bit done_id


class CommTimeoutError(RuntimeError):
    pass


class ChecksumError(RuntimeError):
    """A message failed verification (debug ``verify`` mode): corrupted payload or out-of-order request."""


def _checksum(rows: torch.Tensor) -> torch.Tensor:
    """Per-row Fletcher-style checksum of byte rows [k, nbytes] (nbytes % 4 == 0) -> int64 [k, 2]."""
    w = rows.contiguous().view(torch.int32).to(torch.int64)
    idx = torch.arange(1, w.shape[1] + 1, device=w.device, dtype=torch.int64)
    return torch.stack([w.sum(1), (w * idx).sum(1)], 1)


def _cdiv(a, b):
    return (a + b - 1) // b


def _round_up(a, b):
    return _cdiv(a, b) * b


# ------------------------------------------------------------------------------------------ planning
def ring_geometry(n: int, world: int, max_slice_elems: int):
    C = _ext.load()
    if C is not None:
        return tuple(C.ring_geometry(int(n), int(world), int(max_slice_elems)))
    ms = max(256, max_slice_elems // 256 * 256)
    nn = max(n, 1)
    blocks = _cdiv(nn, world * ms)
    sl = _round_up(_cdiv(nn, world * blocks), 256)
    return (n, sl, blocks, blocks * world * sl)


def ring_plan(world: int, position: int, blocks: int):
    """List of [send_slice, send_src, recv_slice, recv_full, owned] rows (see csrc/comm/planner.h)."""
    C = _ext.load()
    if C is not None:
        return [list(r) for r in C.ring_plan(int(world), int(position), int(blocks))]
    return _py_ring_plan(world, position, blocks)


def _py_ring_plan(N, p, blocks):  # identical to csrc/comm/planner.cpp (used only without the extension)
    out = []
    for b in range(blocks):
        base = b * N
        if N == 1:
            out.append([base, 0, -1, 0, base])
            continue
        out.append([base + p % N, 0, base + (p + 1) % N, 0, -1])
        for k in range(1, N - 1):
            out.append([base + (p + k) % N, 1, base + (p + k + 1) % N, 0, -1])
        out.append([base + (p - 1) % N, 1, base + p % N, 1, base + (p - 1) % N])
        for i in range(1, N - 1):
            out.append([base + (p + i - 1) % N, 2, base + (p + i) % N, 1, -1])
    return out


def ring_orders(world: int, max_rings: int, links=None):
    """Arc-disjoint directed Hamiltonian rings (native planner); ``links[a][b]`` truthy: rank a has a direct link
    to rank b (None: fully connected)."""
    C = _ext.load()
    if C is not None:
        lk = None if links is None else [[int(bool(x)) for x in row] for row in links]
        return [list(o) for o in C.ring_orders(int(world), int(max_rings), lk)]
    return [list(range(world))]


@dataclass
class BucketLayout:
    n: int
    n_pad: int
    algo: str
    world: int
    shard: int = 0          # mesh: shard elements
    slice_elems: int = 0    # ring: slice elements
    blocks: int = 0         # ring: blocks per ring part
    rings: int = 1
    part: int = 0           # ring: padded elements per ring part
    chunks: int = 1         # mesh (C++ engine): chunks of `world` shards streamed through the collectives
    sub: int = 1            # ring (C++ engine, direct P2P): sub-slices per hop message (streamed hops)

    @property
    def key(self):
        return (self.n_pad, self.algo, self.world, self.shard, self.slice_elems, self.blocks, self.rings)


class Handle:
    """Async completion of one all-reduce request (reference: a done slot, sw:157-180)."""

    def __init__(self, engine, slot: int, event, name: str, pending=None):
        self.engine = engine
        self.slot = slot
        self.event = event
        self.name = name
        self.t_issue = time.time()
        self._pending = pending  # deferred epilogue thunks (see CompressedAllReduce.allreduce_sgd(defer=True))

    def commit(self, update_after=None):
        """Enqueue the deferred weight-update epilogue, after ``update_after`` (an event on the producer
        stream marking the last read of the old weights, e.g. the bwd-data GEMM)."""
        if self._pending is None:
            return self
        thunks, self._pending = self._pending, None
        self.event = self.engine._run_thunks(thunks, update_after)
        return self

    def commit_after_current(self):
        """commit() ordered after everything enqueued so far on the current stream."""
        ev = None
        if self._pending is not None and self.engine.cuda and not self.engine.inline:
            ev = self.engine._event()
            ev.record()
        return self.commit(update_after=ev)

    def done(self) -> bool:
        if self._pending is not None:
            return False
        return self.event is None or self.event.query()

    def latency_ms(self) -> float | None:
        """Device-side latency of the request (start of its comm phase -> end of the epilogue); requires
        ``engine.timing = True`` (the reference's get_all_reduce_latency(), sw/mlp_mpi_example_f32.cpp:100-106)."""
        t = getattr(self, "_timing", None)
        if t is None or self._pending is not None:
            return None
        t[1].synchronize()
        return t[0].elapsed_time(t[1])

    def wait(self, stream=None):
        """GPU-side wait: make ``stream`` (default: current) wait for completion; host does not block."""
        self.commit()
        if self.event is not None:
            (stream or torch.cuda.current_stream()).wait_event(self.event)

    def synchronize(self, timeout: float | None = None):
        """Host wait with a bounded timeout and diagnostics (never spins forever)."""
        self.commit()
        if self.event is None:
            return
        timeout = self.engine.timeout_s if timeout is None else timeout
        t0 = time.time()
        sleep = 1e-5
        while not self.event.query():
            err = self.engine.transport.async_error()
            if err:
                raise CommTimeoutError(f"all-reduce '{self.name}' (slot {self.slot}) failed: {err}")
            if time.time() - t0 > timeout:
                diag = self.engine.diagnostics(self)
                self.engine.transport.abort()
                raise CommTimeoutError(f"all-reduce '{self.name}' timed out after {timeout:.1f}s: {diag}")
            time.sleep(sleep)
            sleep = min(sleep * 2, 1e-3)


@dataclass
class _Scratch:
    tensors: dict = field(default_factory=dict)


class CompressedAllReduce:
    """Compressed (or raw) all-reduce + fused SGD over a :class:`Transport`."""

    def __init__(self, transport: Transport, *, codec: str = "bfp_rne", algo: str = "mesh", rings: int = 1,
                 max_slice_elems: int = 1 << 22, device=None, compat_owner_fp32: bool = False,
                 timeout_s: float = 600.0, stream=None, stream_priority: int = -1, force_comm: bool = False,
                 verify: bool | None = None):
        if algo not in ("mesh", "ring"):
            raise ValueError(f"unknown algo {algo!r}")
        self.transport = transport
        self.rank, self.world = transport.rank, transport.world
        self.codec = codec
        self.codec_id = wire.codec_id(codec)
        self.algo = algo
        self.max_slice_elems = max_slice_elems
        self.compat_owner_fp32 = compat_owner_fp32
        self.timeout_s = timeout_s
        self.device = torch.device(device) if device is not None else (
            torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu"))
        self.cuda = self.device.type == "cuda"
        self.orders = ring_orders(self.world, rings) if algo == "ring" else [list(range(self.world))]
        self.rings = len(self.orders)
        # world 1: nothing to overlap -> run inline on the caller's stream (no side stream, no event packets).
        # force_comm keeps the multi-rank code path (side stream, collectives) even at world 1.
        self.force_comm = force_comm
        self.inline = self.world == 1 and not force_comm
        if self.cuda and not self.inline:
            self.stream = stream or torch.cuda.Stream(device=self.device, priority=stream_priority)
        else:
            self.stream = None
        self._events: list = []
        self.timing = False  # per-request device timestamps (Handle.latency_ms)
        self._scratch: dict = {}
        self._cur_slot = 0
        self._slot = 0
        self._slot_owner: list = [None] * NUM_SLOTS  # last request issued on each slot
        self.fault = faults.FaultInjector.from_env()
        self.stats = {"requests": 0, "wire_bytes": 0, "logical_bytes": 0}
        # debug mode: every message travels with a checksum + the request sequence number,
        # verified on arrival (host-synchronous: for bisecting corruption / desync, not for speed)
        self.verify = bool(int(os.environ.get("FAN_VERIFY", "0"))) if verify is None else verify

    # -------------------------------------------------------------------------------- layout
    def layout(self, n: int) -> BucketLayout:
        N = self.world
        if self.algo == "mesh":
            shard = _round_up(max(_cdiv(n, N), 1), 256)
            return BucketLayout(n=n, n_pad=shard * N, algo="mesh", world=N, shard=shard)
        R = self.rings
        chunk = _cdiv(max(n, 1), R)
        _, sl, blocks, part = ring_geometry(chunk, N, self.max_slice_elems)
        return BucketLayout(n=n, n_pad=part * R, algo="ring", world=N, slice_elems=sl, blocks=blocks, rings=R,
                            part=part)

    def wire_bytes(self, L: BucketLayout) -> int:
        """Bytes this rank sends for one request (for bus-bandwidth accounting)."""
        N = self.world
        if N == 1:
            return 0
        if L.algo == "mesh":
            return 2 * (N - 1) * wire.shard_bytes(self.codec_id, L.shard)
        return L.rings * L.blocks * 2 * (N - 1) * wire.shard_bytes(self.codec_id, L.slice_elems)

    def _buf(self, L: BucketLayout, name: str, nbytes: int, dtype=torch.uint8, per_slot: bool = False):
        """Persistent scratch per bucket layout. ``per_slot``: a buffer a deferred epilogue reads — one per
        request slot, so a later same-size request cannot overwrite it before this request commits."""
        key = (L.key, name, self._cur_slot) if per_slot else (L.key, name)
        t = self._scratch.get(key)
        if t is None:
            t = torch.zeros(nbytes // torch.empty(0, dtype=dtype).element_size(), dtype=dtype, device=self.device)
            self._scratch[key] = t
        return t

    # -------------------------------------------------------------------------------- requests
    def allreduce_sgd(self, grad: torch.Tensor, master: torch.Tensor, lp: torch.Tensor | None = None,
                      mom: torch.Tensor | None = None, *, n_valid: int | None = None, lr: float,
                      grad_scale: float = 1.0, weight_decay: float = 0.0, momentum: float = 0.0,
                      nesterov: bool = False, update_after=None, defer: bool = False,
                      name: str = "bucket") -> Handle:
        """All-reduce ``grad`` (flat, padded to ``layout(n).n_pad``) and apply SGD to ``master`` (+bf16 ``lp``)."""
        n_valid = int(n_valid if n_valid is not None else master.numel())
        L = self.layout(n_valid)
        self._check(grad, L)
        sgd_kw = dict(lr=lr, grad_scale=grad_scale, weight_decay=weight_decay, momentum=momentum, nesterov=nesterov)

        def finish(G, shard, n_shards, off, length, skip=(-1, 0)):
            nv = max(0, min(n_valid - off, length))
            if nv == 0:
                return
            wire.sgd(G, shard, n_shards, master.view(-1)[off:off + length], codec=self.codec_id,
                     lp=None if lp is None else lp.view(-1)[off:off + length],
                     mom=None if mom is None else mom.view(-1)[off:off + length], n_valid=nv,
                     skip_shard=skip[0], skip_period=skip[1], **sgd_kw)

        def owner_fp32(buf, off, length):  # compat: owner applies SGD from the un-quantised fp32 sum
            nv = max(0, min(n_valid - off, length))
            if nv:
                wire.sgd(buf, length, 1, master.view(-1)[off:off + length], codec="raw_f32",
                         lp=None if lp is None else lp.view(-1)[off:off + length],
                         mom=None if mom is None else mom.view(-1)[off:off + length], n_valid=nv, **sgd_kw)

        return self._launch(lambda: self._run(L, grad, finish, owner_fp32), name, L, defer, update_after)

    def allreduce(self, grad: torch.Tensor, out: torch.Tensor, *, n_valid: int | None = None,
                  name: str = "bucket") -> Handle:
        """Sum-only all-reduce: decoded result written to ``out`` (f32 or bf16, same padded length)."""
        n_valid = int(n_valid if n_valid is not None else grad.numel())
        L = self.layout(n_valid)
        self._check(grad, L)

        def finish(G, shard, n_shards, off, length, skip=(-1, 0)):
            wire.unpack(G, out.view(-1)[off:off + length], shard, self.codec_id)

        def owner_fp32(buf, off, length):
            pass

        return self._launch(lambda: self._run(L, grad, finish, owner_fp32, allow_compat=False), name, L, False,
                            None)

    def _check(self, grad, L):
        if grad.numel() < L.n_pad:
            raise ValueError(f"gradient buffer has {grad.numel()} elements; layout needs {L.n_pad} (use "
                             f"engine.layout(n).n_pad to size flat buffers)")
        if grad.dtype not in (torch.float32, torch.bfloat16):
            raise TypeError("gradients must be f32 or bf16")

    def _launch(self, comm_fn, name, L, defer=False, update_after=None) -> Handle:
        slot = self._slot
        self._slot = (slot + 1) % NUM_SLOTS
        prev = self._slot_owner[slot]
        if prev is not None and prev._pending is not None:
            # more than NUM_SLOTS requests deferred: the slot's previous request must commit before its per-slot
            # scratch is reused (ordered after everything enqueued so far on the producer stream)
            prev.commit_after_current()
            self.stats["forced_commits"] = self.stats.get("forced_commits", 0) + 1
        self._cur_slot = slot  # per-slot scratch of the request comm_fn builds
        self.stats["requests"] += 1
        self.stats["wire_bytes"] += self.wire_bytes(L)
        self.stats["logical_bytes"] += L.n * 4
        if not self.cuda or self.inline:
            thunks = comm_fn()
            h = Handle(self, slot, None, name, pending=thunks)
            self._slot_owner[slot] = h
            return h if defer else h.commit()
        ready = self._event()
        ready.record(torch.cuda.current_stream(self.device))
        t_start = None
        with torch.cuda.stream(self.stream):
            self.stream.wait_event(ready)
            if self.timing:
                t_start = torch.cuda.Event(enable_timing=True)
                t_start.record(self.stream)
            thunks = comm_fn()
        if t_start is not None:
            t_end = torch.cuda.Event(enable_timing=True)
            thunks = list(thunks) + [lambda: t_end.record(self.stream)]
        h = Handle(self, slot, None, name, pending=thunks)
        self._slot_owner[slot] = h
        if t_start is not None:
            h._timing = (t_start, t_end)
        return h if defer else h.commit(update_after)

    def _event(self):
        """Events are recycled round-robin (a pool deeper than the requests in flight)."""
        if len(self._events) < 4 * NUM_SLOTS:
            e = torch.cuda.Event()
            self._events.append(e)
            return e
        e = self._events.pop(0)
        self._events.append(e)
        return e

    def _run_thunks(self, thunks, update_after=None):
        if not self.cuda or self.inline:
            for t in thunks:
                t()
            return None
        with torch.cuda.stream(self.stream):
            if update_after is not None:
                self.stream.wait_event(update_after)
            for t in thunks:
                t()
            done = self._event()
            done.record(self.stream)
        return done

    def _tag(self, rows: torch.Tensor) -> torch.Tensor:
        """[k, 3] int64: checksum of each byte row + the request sequence number."""
        seq = torch.full((rows.shape[0], 1), self.stats["requests"], dtype=torch.int64, device=rows.device)
        return torch.cat([_checksum(rows), seq], 1)

    def _verify_rows(self, rows, tags, peers, what):
        got = _checksum(rows).cpu()
        tags = tags.cpu()
        for i, peer in enumerate(peers):
            if int(tags[i, 2]) != self.stats["requests"]:
                raise ChecksumError(f"rank {self.rank}: {what}: message from peer {peer} belongs to request "
                                    f"#{int(tags[i, 2])}, expected #{self.stats['requests']} (out of order)")
            if not torch.equal(got[i], tags[i, :2]):
                raise ChecksumError(f"rank {self.rank}: {what}: message from peer {peer} is corrupted "
                                    f"(checksum {got[i].tolist()} != {tags[i, :2].tolist()}, request "
                                    f"#{self.stats['requests']})")

    def diagnostics(self, h: Handle) -> str:
        return (f"rank={self.rank} world={self.world} algo={self.algo} codec={self.codec} rings={self.rings} "
                f"slot={h.slot} elapsed={time.time() - h.t_issue:.1f}s transport={self.transport.name} "
                f"async_error={self.transport.async_error()!r}")

    # -------------------------------------------------------------------------------- execution
    def _run(self, L, grad, finish, owner_fp32, allow_compat=True):
        """Issue the communication phase; returns the epilogue thunks (run now or at commit)."""
        if L.algo == "mesh":
            return self._mesh(L, grad, finish)
        return self._ring(L, grad, finish, owner_fp32, allow_compat)

    def _mesh(self, L, grad, finish):
        N, r, s, c = self.world, self.rank, L.shard, self.codec_id
        sb = wire.shard_bytes(c, s)
        g = grad.view(-1)[: L.n_pad]
        S = self._buf(L, "mesh_S", sb, per_slot=N == 1 and not self.force_comm)
        if N == 1 and not self.force_comm:
            wire.reduce(S, 1, 0, g[:s], S, None, s, c)
            return [lambda: finish(S, s, 1, 0, s)]
        if c == 2 and g.dtype == torch.float32:
            P = wire.as_bytes(g)
        elif c == 3 and g.dtype == torch.bfloat16:
            P = wire.as_bytes(g)
        else:
            P = self._buf(L, "mesh_P", sb * N)
            wire.pack(g, P, s, c)
        cs = self._tag(P.view(N, sb)) if self.verify else None
        self.fault.maybe_corrupt("mesh_pack", P)
        R = self._buf(L, "mesh_R", sb * N)
        self.transport.all_to_all(P, R)
        if cs is not None:
            cs_r = torch.empty_like(cs)
            self.transport.all_to_all(cs, cs_r)
            self._verify_rows(R.view(N, sb), cs_r, list(range(N)), "mesh all_to_all")
        wire.reduce(R, N, r, g[r * s:(r + 1) * s], S, None, s, c)
        G = self._buf(L, "mesh_G", sb * N, per_slot=True)
        self.transport.all_gather(S, G)
        if self.verify:
            cs_g = torch.empty(N, 3, dtype=torch.int64, device=G.device)
            self.transport.all_gather(self._tag(S.view(1, sb)), cs_g)
            self._verify_rows(G.view(N, sb), cs_g, list(range(N)), "mesh all_gather")
        return [lambda: finish(G, s, N, 0, L.n_pad)]

    def _ring(self, L, grad, finish, owner_fp32, allow_compat):
        N, c = self.world, self.codec_id
        S = L.slice_elems
        sb = wire.shard_bytes(c, S)
        nsl = L.blocks * N
        g = grad.view(-1)
        compat = allow_compat and self.compat_owner_fp32 and N > 1
        rings = []
        for i, order in enumerate(self.orders):
            pos = order.index(self.rank)
            rings.append(dict(
                off=i * L.part,
                down=order[(pos - 1) % N], up=order[(pos + 1) % N], pos=pos,
                plan=ring_plan(N, pos, L.blocks),
                G=self._buf(L, f"ring_G{i}", sb * nsl, per_slot=True),
                send=self._buf(L, f"ring_send{i}", sb),
                recv=[self._buf(L, f"ring_recv{i}_0", sb), self._buf(L, f"ring_recv{i}_1", sb)],
                last_partial=None,
                fp32=self._buf(L, f"ring_fp32_{i}", 4 * S * L.blocks, torch.float32, per_slot=True) if compat else None,
            ))
        nrows = len(rings[0]["plan"])
        # group rows into communication rounds: a SEND_LOCAL row joins the previous round (OUTPUT_SEND overlap)
        rounds, cur = [], []
        for j in range(nrows):
            if cur and not (rings[0]["plan"][j][1] == 0 and j > 0):
                rounds.append(cur)
                cur = []
            cur.append(j)
        if cur:
            rounds.append(cur)

        def local(ring, x):
            o = ring["off"] + x * S
            return g[o:o + S]

        checks = []
        for ri, rnd in enumerate(rounds):
            sends, recvs = [], []
            for j in rnd:
                for ring in rings:
                    send_slice, src, recv_slice, recv_full, owned = ring["plan"][j]
                    Gs = lambda x, ring=ring: ring["G"][x * sb:(x + 1) * sb]  # noqa: E731
                    out = None
                    if src == 0:  # SEND_LOCAL
                        out = Gs(send_slice) if owned >= 0 else ring["send"]
                        wire.pack(local(ring, send_slice), out, S, c)
                    elif src == 1:  # REDUCE / REDUCE_OUTPUT
                        out = Gs(send_slice) if owned >= 0 else ring["send"]
                        f32 = None
                        if compat and owned >= 0:
                            blk = owned // N
                            f32 = ring["fp32"][blk * S:(blk + 1) * S]
                        wire.reduce(ring["last_partial"], 2, 1, local(ring, send_slice), out, f32, S, c)
                    elif src == 2:  # FORWARD (already-encoded full slice)
                        out = Gs(send_slice)
                    if out is not None and N > 1:
                        cs = self._tag(out.view(1, sb)) if self.verify else None
                        self.fault.maybe_corrupt("ring_send", out)
                        sends.append((out, ring["down"]))
                        if cs is not None:
                            sends.append((cs, ring["down"]))
                    if recv_slice >= 0:
                        if recv_full:
                            tgt = Gs(recv_slice)
                        else:
                            tgt = ring["recv"][j % 2]
                            ring["last_partial"] = tgt
                        recvs.append((tgt, ring["up"]))
                        if self.verify:
                            cs_r = torch.empty(1, 3, dtype=torch.int64, device=tgt.device)
                            recvs.append((cs_r, ring["up"]))
                            checks.append((tgt, cs_r, ring["up"], f"ring round {ri} slice {recv_slice}"))
            if N > 1:
                self.transport.sendrecv(sends, recvs)
                for tgt, cs_r, peer, what in checks:
                    self._verify_rows(tgt.view(1, sb), cs_r, [peer], what)
                checks.clear()
        thunks = []
        for i, ring in enumerate(rings):
            off = ring["off"]
            if compat:
                own = (ring["pos"] - 1) % N
                thunks.append(lambda ring=ring, off=off, own=own: finish(ring["G"], S, nsl, off, L.part,
                                                                        skip=(own, N)))
                for b in range(L.blocks):
                    x = b * N + own
                    thunks.append(lambda ring=ring, b=b, x=x, off=off: owner_fp32(
                        ring["fp32"][b * S:(b + 1) * S], off + x * S, S))
            else:
                thunks.append(lambda ring=ring, off=off: finish(ring["G"], S, nsl, off, L.part))
        return thunks


def uncompressed_allreduce_sgd(transport: Transport, grad, master, lp=None, mom=None, *, n_valid=None, lr,
                               grad_scale=1.0, weight_decay=0.0, momentum=0.0, nesterov=False):
    """Baseline: RCCL all-reduce (sum) of the raw gradients + a separate SGD kernel (BASELINE config 2;
    the reference's commented MPI_Iallreduce + libxsmm opt path, sw:615-647)."""
    transport.all_reduce_(grad)
    n_valid = master.numel() if n_valid is None else n_valid
    n = _round_up(n_valid, 256)
    codec = "raw_f32" if grad.dtype == torch.float32 else "raw_bf16"
    wire.sgd(wire.as_bytes(grad.view(-1)[:n]) if grad.numel() >= n else wire.as_bytes(grad), n, 1,
             master.view(-1), codec=codec, lp=None if lp is None else lp.view(-1),
             mom=None if mom is None else mom.view(-1), lr=lr, grad_scale=grad_scale, weight_decay=weight_decay,
             momentum=momentum, nesterov=nesterov, n_valid=n_valid)
