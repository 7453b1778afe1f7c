"""On-device plan tuning for the MFMA GEMMs (the hipBLASLt-heuristics / MIOpen-find role, for our own kernels).

The planner's static rule ("the largest tile that still gives one workgroup per CU, split K when the grid is
under half the CUs", csrc/gemm/gemm_bf16_plan.hip) was measured on the flagship's MB-8192 shapes. At the
reference's own per-rank batch (1792 rows, sw/run.sh:16) every grid is between 0.4 and 1.75 waves of the 256 CUs,
and there the rule is wrong by up to 1.5x: 1792x4096x4096 runs 256x256 tiles split 4 ways in 80 µs where 256x128
tiles without a split take 55-59 µs (profiles/r3_gemm_sweep_mb1792.jsonl). Rather than another hand-fitted rule,
the first call of every (shape, layout, epilogue) times the candidate plans on the device, in place, on the call's
own operands, and keeps the fastest:

* only shapes whose static plan leaves the last wave of workgroups part-empty are tuned (whole-wave plans were
  chosen by in-step A/B and are kept);
* candidates: BM x BN in {256, 128}^2 (plus 224x128 for a K-contiguous A: 1792 = 8 x 224 rows) x split-K in
  {1, 2, 3, 4, 6, 8}, those the planner accepts for the shape, with at most 4 waves of workgroups and at least 256
  K-elements per split;
* two interleaved rounds of 3 timed launches each (hip events), a candidate's score is its best round median;
  the static plan keeps the shape unless a candidate beats it by more than ``margin`` (5 %);
* the winner runs last, so the caller's outputs are the winner's (every candidate computes the same product, and
  every epilogue is re-runnable: no accumulate, colsum / wire written not added — accumulating calls, calls whose
  output aliases an input, and calls during HIP-graph capture are never tuned);
* decisions persist in ``FAN_GEMM_TUNE_FILE`` (JSON) when set; ``FAN_GEMM_TUNE=0`` turns tuning off (static plans:
  bit-reproducible runs).

Different ranks may pick different plans for their (different) data: that changes only the rounding of each
rank's own gradient contribution, never the replicas' agreement (every rank applies the same all-reduced update).
"""
from __future__ import annotations

import json
import os
import threading

import torch

TILES = ((256, 256), (256, 128), (128, 256), (128, 128))
# 224x128: 1792 rows (the reference's per-rank batch) in 8 row tiles -> one workgroup per CU on 4096-wide outputs;
# K-contiguous A only (the planner refuses it otherwise), no fused bias gradient
TILES_KA = ((224, 128),)
SPLITS = (1, 2, 3, 4, 6, 8)


class GemmTuner:
    def __init__(self, margin: float = 0.05, reps: int = 3, rounds: int = 2):
        self.enabled = os.environ.get("FAN_GEMM_TUNE", "1") != "0"
        self.path = os.environ.get("FAN_GEMM_TUNE_FILE") or None
        self.margin, self.reps, self.rounds = margin, reps, rounds
        self.plans: dict[str, tuple[int, int, int]] = {}
        self.log: list[dict] = []
        self._lock = threading.Lock()
        if self.path and os.path.exists(self.path):
            try:
                with open(self.path) as f:
                    self.plans = {k: tuple(v) for k, v in json.load(f).items()}
            except (OSError, ValueError):
                self.plans = {}

    @staticmethod
    def key(M, N, K, a_t, b_t, epilogue, colsum, wire, dev) -> str:
        name = torch.cuda.get_device_properties(dev).gcnArchName.split(":")[0] if torch.cuda.is_available() else ""
        return f"{name}|{M}x{N}x{K}|{int(a_t)}{int(b_t)}|e{epilogue}|c{int(colsum)}|w{int(wire)}"

    def candidates(self, Cx, M, N, K, a_kcontig=False, colsum=False):
        out, seen = [], set()
        for bm, bn in TILES + (TILES_KA if a_kcontig and not colsum else ()):
            for sk in SPLITS:
                if sk > 1 and K // sk < 256:
                    continue
                p = tuple(Cx.gemm_plan(M, N, K, sk, bm, bn, 0))
                if p[0] == 0 or (p[0], p[1], p[2]) != (bm, bn, sk):
                    continue
                wgs = -(-M // bm) * -(-N // bn) * sk
                if wgs > 1024 or p[:3] in seen:
                    continue
                seen.add(p[:3])
                out.append(p[:3])
        return out

    def lookup(self, k):
        return self.plans.get(k)

    @staticmethod
    def worth_tuning(M, N, static, dev) -> bool:
        """Only grids that leave part of the last wave of workgroups idle: the static plans of whole-wave grids were
        chosen by in-step A/B (round 2) and a micro-benchmark in place, with cache-warm operands, can misrank them
        (a profiled run once swapped the MB-8192 forward's 256x256 tiles for 256x128: 76 vs 64.5 us in the step)."""
        cus = torch.cuda.get_device_properties(dev).multi_processor_count if torch.cuda.is_available() else 256
        wgs = -(-M // static[0]) * -(-N // static[1]) * static[2]
        return wgs % cus != 0

    def keep_static(self, k, static):
        with self._lock:
            self.plans[k] = tuple(static[:3])
        return tuple(static[:3])

    def tune(self, k, static_plan, cands, run):
        """run(plan) launches the GEMM with that (bm, bn, sk) plan on the current stream. Returns the winner (which
        has run last)."""
        static_plan = tuple(static_plan[:3])
        if static_plan not in cands:
            cands = [static_plan] + cands
        s = torch.cuda.current_stream()
        times = {c: [] for c in cands}
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        for c in cands:  # first touch: code objects, workspace
            run(c)
        for _ in range(self.rounds):
            for c in cands:
                ev[0].record(s)
                for _ in range(self.reps):
                    run(c)
                ev[1].record(s)
                ev[1].synchronize()
                times[c].append(ev[0].elapsed_time(ev[1]) * 1e3 / self.reps)
        score = {c: min(v) for c, v in times.items()}
        best = min(score, key=score.get)
        if score[best] > score[static_plan] * (1.0 - self.margin):
            best = static_plan
        run(best)
        with self._lock:
            self.plans[k] = best
            self.log.append({"key": k, "static": list(static_plan), "static_us": round(score[static_plan], 2),
                             "chosen": list(best), "chosen_us": round(score[best], 2)})
            if self.path:
                try:
                    tmp = self.path + ".tmp"
                    with open(tmp, "w") as f:
                        json.dump({kk: list(v) for kk, v in self.plans.items()}, f, indent=0)
                    os.replace(tmp, self.path)
                except OSError:
                    pass
        return best


_tuner: GemmTuner | None = None


def tuner() -> GemmTuner:
    global _tuner
    if _tuner is None:
        _tuner = GemmTuner()
    return _tuner


def reset(enabled: bool | None = None):
    """Forget every decision (tests / A/B); optionally force tuning on or off."""
    global _tuner
    _tuner = GemmTuner()
    if enabled is not None:
        _tuner.enabled = bool(enabled)
    return _tuner
