#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter_collection CSVs per kernel (mean over dispatches).

Usage: python tools/pmc_summary.py gpurun_out/pmc1/p_counter_collection.csv [more.csv ...] [--filter gemm]
Derived: effective clock (GRBM_GUI_ACTIVE / 8 XCDs / kernel time; reads high below ~0.3 ms), MFMA busy share,
L2 hit rate, FETCH/WRITE bandwidth (GB/s over the dispatch; counters from separate passes are averaged per kernel).

MFMA utilisation without the saturating SQ_VALU_MFMA_BUSY_CYCLES (it wraps at 2^28 on a 200 µs GEMM summed over
1024 SIMDs): SQ_INSTS_MFMA (MFMA instructions issued, summed over SEs) x 16 cycles per v_mfma_f32_16x16x32_bf16 on
one SIMD / (kernel cycles x 1024 SIMDs), kernel cycles = GRBM_GUI_ACTIVE / 8; achieved TFLOP/s from
SQ_INSTS_VALU_MFMA_MOPS_BF16 x 512 / kernel time, and its share of the 2.5 PF dense bf16 peak. ``--table`` prints one
line per kernel shape instead (sorted by total time).
"""
import argparse
import collections
import csv
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv", nargs="+")
    ap.add_argument("--filter", default="")
    ap.add_argument("--table", action="store_true", help="one line per kernel shape: MFMA utilisation table")
    ap.add_argument("--mfma-cycles", type=float, default=16.0, help="SIMD cycles per MFMA instruction (16x16x32 bf16)")
    a = ap.parse_args()
    agg = collections.OrderedDict()
    for f in a.csv:
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if a.filter and a.filter not in name:
                continue
            key = (name[:110], r["Grid_Size"])
            d = agg.setdefault(key, {"_n": collections.Counter(), "_dur": []})
            c = r["Counter_Name"]
            d.setdefault(c, collections.defaultdict(float))
            d[c][(f, r["Dispatch_Id"])] += float(r["Counter_Value"])  # per pass: dispatch ids restart
            d["_meta"] = (r["VGPR_Count"], r["Accum_VGPR_Count"], r["SGPR_Count"], r["LDS_Block_Size"])
            d.setdefault("_t", {})[(f, r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    if a.table:
        # per dispatch, then grouped by (kernel, grid, MFMA FLOPs): a persistent GEMM launches the same grid for every
        # shape, so the FLOP count (SQ_INSTS_VALU_MFMA_MOPS_BF16 x 512) is what tells its shapes apart
        per = collections.defaultdict(dict)
        for f in a.csv:
            for r in csv.DictReader(open(f)):
                if a.filter and a.filter not in r["Kernel_Name"]:
                    continue
                k = (f, r["Dispatch_Id"])
                d = per[k]
                d["name"], d["grid"] = r["Kernel_Name"], r["Grid_Size"]
                d["t"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
                d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        groups = collections.defaultdict(list)
        for d in per.values():
            fl = d.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0.0) * 512
            groups[(d["name"], d["grid"], float(f"{fl:.3g}"))].append(d)
        rows = []
        for (name, grid, fl), ds in groups.items():
            t_ns = statistics.mean(d["t"] for d in ds)
            cyc = statistics.mean(d.get("GRBM_GUI_ACTIVE", 0.0) for d in ds) / 8
            mf = statistics.mean(d.get("SQ_INSTS_MFMA", 0.0) for d in ds)
            busy = mf * a.mfma_cycles / (cyc * 1024) if cyc and mf else None
            rows.append((t_ns * len(ds), name, grid, len(ds), t_ns, cyc / t_ns if cyc else None, busy,
                         fl / t_ns / 1e3 if fl else None, fl))
        rows.sort(key=lambda r: -r[0])
        print(f"{'kernel':58s} {'GFLOP':>7s} {'n':>4s} {'us':>8s} {'GHz':>5s} {'mfma_busy%':>10s} {'TFLOP/s':>8s} "
              f"{'%2.5PF':>7s}")
        for tot, name, grid, n, t_ns, ghz, busy, tf, fl in rows:
            print(f"{name[:58]:58s} {fl / 1e9:7.1f} {n:4d} {t_ns / 1e3:8.1f} {ghz or 0:5.2f} "
                  f"{(busy or 0) * 100:10.1f} {tf or 0:8.1f} {(tf or 0) / 25:7.1f}")
        return
    for (name, grid), d in agg.items():
        m = {c: sum(v.values()) / len(v) for c, v in d.items() if not c.startswith("_")}
        t_ns = sum(d["_t"].values()) / len(d["_t"])
        print(f"{name}  grid={grid} vgpr/agpr/sgpr/lds={d['_meta']}  t={t_ns/1e3:.1f}us")
        for c, v in sorted(m.items()):
            print(f"    {c:28s} {v:16.0f}")
        if "GRBM_GUI_ACTIVE" in m:
            print(f"    eff_clock_GHz               {m['GRBM_GUI_ACTIVE'] / 8 / t_ns:16.3f}")
        if "SQ_WAVE_CYCLES" in m and "SQ_VALU_MFMA_BUSY_CYCLES" in m and "SQ_BUSY_CYCLES" in m:
            print(f"    mfma_busy/(busy*4simd*?)    {m['SQ_VALU_MFMA_BUSY_CYCLES'] / max(1, m['SQ_BUSY_CYCLES']):16.3f}")
        if "SQ_WAVE_CYCLES" in m:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                if c in m:
                    print(f"    {c+'/WAVE':28s} {m[c] / m['SQ_WAVE_CYCLES']:16.3f}")
        if "TCC_HIT_sum" in m and "TCC_MISS_sum" in m:
            print(f"    L2_hit                      {m['TCC_HIT_sum'] / max(1, m['TCC_HIT_sum'] + m['TCC_MISS_sum']):16.3f}")
        for c in ("FETCH_SIZE", "WRITE_SIZE"):  # KiB per dispatch -> GB/s over the dispatch
            if c in m:
                print(f"    {c + '_GBps':28s} {m[c] * 1024 / t_ns:16.1f}")


if __name__ == "__main__":
    main()
