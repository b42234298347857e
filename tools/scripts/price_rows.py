"""Prices a level-0 row load gated on the row's valid link count:
  1. drm_device_chase_rows: the search's dependent row load with 1, 2 or 3 of the 384-B row's 128-B lines loaded,
     at the search's resident wave count (CUs x 20) and at one wave per CU, over a 16 GB table;
  2. the valid-link histogram of the C5 GPU-built graph's level-0 rows (faiss layout: the links first, -1 after),
     read from the bench's IHNp file by memory map (the bench cache is built here if absent).
The hop-weighted form (lines per expanded row) comes from the stamped kernel: tools/scripts/stamps.py c5gru.
Run on the GPU box: python tools/scripts/price_rows.py [--no-hist]."""
import argparse
import ctypes as C
import os
import struct
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from deepreadmapper_amd._native import check, lib  # noqa: E402


def chase(lines, waves, footprint=16 << 30, hops=2000):
    ns = C.c_double(0.0)
    check(lib().drm_device_chase_rows(0, int(footprint), int(waves), int(hops), int(lines), C.byref(ns)))
    return ns.value


def level0_counts(path):
    """Valid links per level-0 row (index of the first -1, else the row length) of an IHNp file, by memory map
    (layout: csrc/faiss_io.cpp; vec = u64 count + data)."""
    with open(path, "rb") as f:
        def one(fmt):
            return struct.unpack("<" + fmt, f.read(struct.calcsize(fmt)))[0]

        def skip_vec(itemsize):
            n = one("Q")
            pos = f.tell()
            f.seek(pos + n * itemsize)
            return n, pos
        assert f.read(4) == b"IHNp"
        one("i"), one("q"), one("q"), one("q"), one("B")
        if one("i") > 1:
            one("f")
        skip_vec(8)                                  # assign_probas
        ncum = one("Q")
        cum = np.frombuffer(f.read(4 * ncum), dtype="<i4")
        skip_vec(4)                                  # levels
        noff, off_pos = skip_vec(8)                  # offsets
        nnb, nb_pos = skip_vec(4)                    # neighbors
    offsets = np.memmap(path, dtype="<u8", mode="r", offset=off_pos, shape=(noff,))
    nbrs = np.memmap(path, dtype="<i4", mode="r", offset=nb_pos, shape=(nnb,))
    deg0 = int(cum[1] - cum[0])
    ntotal = noff - 1
    counts = np.empty(ntotal, dtype=np.int32)
    step = 1 << 21
    for s in range(0, ntotal, step):
        e = min(ntotal, s + step)
        o = np.asarray(offsets[s:e]).astype(np.int64)
        rows = nbrs[o[:, None] + np.arange(deg0)[None, :]]
        neg = rows < 0
        counts[s:e] = np.where(neg.any(axis=1), neg.argmax(axis=1), deg0)
    return counts, deg0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--no-hist", action="store_true")
    a = ap.parse_args()
    import bench
    from deepreadmapper_amd.device import device_props
    ncu = device_props(0)["cu_count"]
    for waves in (ncu * 20, ncu):
        row = []
        for lines in (1, 2, 3):
            ns = chase(lines, waves)
            row.append(ns)
        print(f"chase 16 GB, {waves} waves: ns per dependent row load with 1 / 2 / 3 lines: "
              f"{row[0]:.0f} / {row[1]:.0f} / {row[2]:.0f}  (random lines/s at 5120 waves: "
              f"{' / '.join(f'{waves * l / (r * 1e-9) / 1e9:.1f}G' for l, r in zip((1, 2, 3), row))})", flush=True)
    if a.no_hist:
        return
    args = argparse.Namespace(cache="/tmp/drm_bench_cache", queries=1_250_000, embed="gru")
    wl = bench.prepare_c5(args, bench.Dist(), 0)
    counts, deg0 = level0_counts(wl["index_path"])
    h = np.bincount(counts, minlength=deg0 + 1)
    n = counts.size
    l1, l2 = int((counts <= 10).sum()), int(((counts > 10) & (counts <= 21)).sum())
    l3 = n - l1 - l2
    print(f"C5 level-0 rows: {n}, deg0 {deg0}, mean valid links {counts.mean():.2f}; rows spanning 1 / 2 / 3 lines: "
          f"{l1 / n * 100:.1f} / {l2 / n * 100:.1f} / {l3 / n * 100:.1f} %, {(l1 + 2 * l2 + 3 * l3) / n:.3f} lines per row")
    print("histogram (valid links: rows): " + ", ".join(f"{i}: {int(c)}" for i, c in enumerate(h) if c))


if __name__ == "__main__":
    main()
