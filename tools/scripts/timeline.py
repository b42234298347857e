"""Prints the GPU timeline of a rocprofv3 kernel + memory-copy trace (csv) from the fifth-last search kernel
on: start/end/duration in ms, kind, name, stream. Usage: python tools/scripts/timeline.py DIR [PREFIX]"""
import csv
import os
import sys

d = sys.argv[1]
pre = sys.argv[2] if len(sys.argv) > 2 else "pipe"
ev = []
for k in csv.DictReader(open(os.path.join(d, f"{pre}_kernel_trace.csv"))):
    ev.append((int(k["Start_Timestamp"]), int(k["End_Timestamp"]), "K", k["Kernel_Name"][:48], k["Stream_Id"]))
for m in csv.DictReader(open(os.path.join(d, f"{pre}_memory_copy_trace.csv"))):
    ev.append((int(m["Start_Timestamp"]), int(m["End_Timestamp"]), "C", m["Direction"][12:], m["Stream_Id"]))
ev.sort()
starts = [e[0] for e in ev if "hnsw" in e[3]]
t0 = starts[-min(len(starts), int(os.environ.get("NSEARCH", "4")))]
first = [e for e in ev if e[0] >= t0 - 2_000_000]
for e in first:
    print(f"{(e[0] - t0) / 1e6:8.3f} {(e[1] - t0) / 1e6:8.3f} {(e[1] - e[0]) / 1e6:7.3f} {e[2]} s{e[4]} {e[3]}")
print(f"span {(max(e[1] for e in first) - min(e[0] for e in first)) / 1e6:.3f} ms")
