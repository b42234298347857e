"""FETCH_SIZE calibration for the search's row-load shape.

`run` (under rocprofv3 --pmc FETCH_SIZE): drm_device_chase_rows with 1, 2 and 3 lines of each 384-B row, 5,120 waves
x HOPS dependent rows over 16 GB (each call: one fill_random_kernel, one 50-hop warm-up chase, one timed chase).
The bytes are known: waves x hops x lines x 128 B per chase dispatch (12 B per lane on 10 / 21 / 32 lanes: every line
the wave touches is whole).
`parse DIR`: reads DIR/run_counter_collection.csv and prints, per chase dispatch, FETCH_SIZE (KB as reported),
the known bytes and their ratio -- the factor bench.py applies to the search kernel's FETCH_SIZE."""
import csv
import ctypes as C
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

WAVES, HOPS, FOOT = 5120, 2000, 16 << 30
LINES = (1, 2, 3)


def run():
    from deepreadmapper_amd._native import check, lib
    for lines in LINES:
        ns = C.c_double(0.0)
        check(lib().drm_device_chase_rows(0, FOOT, WAVES, HOPS, lines, C.byref(ns)))
        print(f"lines {lines}: {ns.value:.0f} ns per row", flush=True)


def parse(d):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    per = {}
    for r in csv.DictReader(open(f)):
        if "chase_rows_kernel" not in r["Kernel_Name"] or r["Counter_Name"] != "FETCH_SIZE":
            continue
        per[int(r["Dispatch_Id"])] = per.get(int(r["Dispatch_Id"]), 0.0) + float(r["Counter_Value"])
    ids = sorted(per)
    if len(ids) != 2 * len(LINES):
        raise SystemExit(f"expected {2 * len(LINES)} chase dispatches, found {len(ids)}")
    out = []
    for i, lines in enumerate(LINES):
        for j, hops in enumerate((50, HOPS)):
            kb = per[ids[2 * i + j]]
            known = WAVES * hops * lines * 128
            out.append({"lines": lines, "hops": hops, "fetch_size_kb": kb, "known_bytes": known,
                        "factor": known / (kb * 1024.0)})
    for o in out:
        print(f"lines {o['lines']} hops {o['hops']:5d}: FETCH_SIZE {o['fetch_size_kb'] * 1024 / 1e9:8.3f} GB "
              f"known {o['known_bytes'] / 1e9:8.3f} GB factor {o['factor']:.3f}")
    timed = [o for o in out if o["hops"] == HOPS]
    json.dump({"dispatches": out, "factor_by_lines": {str(o["lines"]): o["factor"] for o in timed},
               "shape": f"{WAVES} waves x {HOPS} dependent rows, 12 B per lane, 384-B row stride, 16 GB random table"},
              open(os.path.join(d, "calib.json"), "w"), indent=1)


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    else:
        parse(sys.argv[2])
