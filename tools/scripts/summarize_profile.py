"""Summarize a rocprofv3 run made by tools/scripts/profile.sh: per-kernel average duration and
per-dispatch PMC counters (FETCH_SIZE corrected x2 on gfx950 for wide streams, see MI355X guide)."""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
out = []
stats = os.path.join(d, "trace", "run_kernel_stats.csv")
if os.path.exists(stats):
    out.append("## kernel stats (rocprofv3 --kernel-trace --stats)")
    for r in csv.DictReader(open(stats)):
        out.append(f"{r['Name'][:90]:90s} calls={r['Calls']:>3s} avg_ms={float(r['AverageNs'])/1e6:9.3f} pct={float(r['Percentage']):6.2f}")
out.append("## PMC (per dispatch averages)")
for f in sorted(glob.glob(os.path.join(d, "pmc*", "run_counter_collection.csv"))):
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
print("\n".join(out))
