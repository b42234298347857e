"""Per-basic-block instruction mix of one kernel in a hipcc -S listing (diagnostic).
Usage: python tools/scripts/isa_blocks.py file.s KERNEL_SYMBOL_SUBSTRING [first_block last_block]"""
import re
import sys

path, kname = sys.argv[1], sys.argv[2]
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and kname in l.split(":")[0] and ":" in l)
end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
blocks, cur = [], None
for l in lines[start:end + 1]:
    m = re.match(r"^(\.LBB\d+_\d+|; %bb\.\d+):?\s*(;.*)?$", l)
    if m:
        cur = {"name": m.group(1), "note": (m.group(2) or "").strip("; "), "v": 0, "s": 0, "ds": 0, "mem": 0, "br": 0}
        blocks.append(cur)
        continue
    if cur is None or not l.startswith("\t"):
        continue
    op = l.strip().split()[0] if l.strip() else ""
    if op.startswith("s_cbranch") or op == "s_branch":
        cur["br"] += 1
    elif op.startswith("v_"):
        cur["v"] += 1
    elif op.startswith("s_"):
        cur["s"] += 1
    elif op.startswith("ds_"):
        cur["ds"] += 1
    elif op.startswith(("global_", "buffer_", "flat_")):
        cur["mem"] += 1
lo = sys.argv[3] if len(sys.argv) > 3 else None
hi = sys.argv[4] if len(sys.argv) > 4 else None
on = lo is None
for b in blocks:
    if b["name"] == lo:
        on = True
    if on:
        print(f"{b['name']:14s} v={b['v']:3d} s={b['s']:3d} ds={b['ds']:2d} mem={b['mem']:2d} br={b['br']} {b['note'][:60]}")
    if b["name"] == hi:
        break
