"""Summarize a rocprofv3 run made by tools/scripts/profile.sh: per-kernel average duration and
per-dispatch PMC counters. Writes <dir>/summary.txt (human) and <dir>/summary.json (read by bench.py
for roofline.traffic). FETCH_SIZE/WRITE_SIZE are KB per dispatch as rocprofv3 reports them; the
MI355X guide's gfx950 correction (FETCH_SIZE x 2 for wide coalesced streams) is applied in
`hbm_bytes_est`; for the search kernel's 12-B-per-lane random row loads the same factor was calibrated on known
bytes (tools/scripts/chase_calib.py: 2.000-2.001, profiles/r06/fetch_calib_chase_rows.txt)."""
import collections
import csv
import glob
import json
import os
import sys

d = sys.argv[1]
out, js = [], {"kernels": {}}
stats = os.path.join(d, "trace", "run_kernel_stats.csv")
if os.path.exists(stats):
    out.append("## kernel stats (rocprofv3 --kernel-trace --stats)")
    for r in csv.DictReader(open(stats)):
        out.append(f"{r['Name'][:90]:90s} calls={r['Calls']:>3s} avg_ms={float(r['AverageNs'])/1e6:9.3f} pct={float(r['Percentage']):6.2f}")
        js["kernels"].setdefault(r["Name"], {})["avg_ms"] = float(r["AverageNs"]) / 1e6
        js["kernels"][r["Name"]]["calls"] = int(r["Calls"])
trace = os.path.join(d, "trace", "run_kernel_trace.csv")
if os.path.exists(trace):
    # the first dispatch of each kernel is bench.py's warm-up (cold caches, first-touch bitmaps):
    # the steady-state average over the rest is what bench.py's timed region compares with
    durs = collections.defaultdict(list)
    for r in csv.DictReader(open(trace)):
        durs[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    out.append("## steady-state dispatch durations (first dispatch = warm-up, excluded)")
    for k, v in durs.items():
        if len(v) > 1 and k in js["kernels"]:
            js["kernels"][k]["avg_ms_steady"] = sum(v[1:]) / len(v[1:])
            out.append(f"{k[:90]:90s} n={len(v) - 1:>3d} avg_ms={sum(v[1:]) / len(v[1:]):9.3f} "
                       f"all=[{', '.join(f'{x:.3f}' for x in v)}]")
out.append("## PMC (per dispatch averages)")
for f in sorted(glob.glob(os.path.join(d, "*", "run_counter_collection.csv"))):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "fillBuffer" in k:
            continue
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    for k, v in agg.items():
        n = len(disp[k])
        out.append(f"{k[:70]:70s} " + " ".join(f"{c}={x / n:.4g}" for c, x in sorted(v.items())))
        js["kernels"].setdefault(k, {}).update({c: x / n for c, x in v.items()})
for k, v in js["kernels"].items():
    if "FETCH_SIZE" in v and "WRITE_SIZE" in v:
        v["hbm_bytes_est"] = (2.0 * v["FETCH_SIZE"] + v["WRITE_SIZE"]) * 1024.0
    if "SQ_INSTS_VALU" in v and "avg_ms" in v:
        # VALU issue share: each wave64 VALU op occupies its SIMD for 4 cycles (1024 SIMDs, 2.4 GHz)
        v["valu_issue_frac"] = v["SQ_INSTS_VALU"] * 4.0 / (1024 * 2.4e9 * v["avg_ms"] * 1e-3)
print("\n".join(out))
json.dump(js, open(os.path.join(d, "summary.json"), "w"), indent=1)
