"""Locality of the visited-bitmap test at C5: for a sample of level-0 rows of the bench's index, how many
distinct bitmap lines (64 B = 512 node bits) and words the row's links touch, under the index's own ids and
under candidate relabelings (a random one as the no-locality baseline, lexicographic order of the PQ codes).
One visited test of the search touches one word per link, so the distinct-line count is the number of memory
requests a hop's test sends. Reads the IHNp file through numpy memmaps (header walk of the faiss layout,
csrc/faiss_io.cpp)."""
import argparse
import struct
import sys
import time

import numpy as np

sys.path.insert(0, ".")
import bench  # noqa: E402


def ihnp_arrays(path):
    """offsets, neighbors, cum, codes (memmaps) of a faiss IHNp + IxPq file."""
    f = open(path, "rb")

    def one(fmt):
        n = struct.calcsize(fmt)
        return struct.unpack("<" + fmt, f.read(n))[0]

    def vec(dtype):
        n = one("Q")
        off = f.tell()
        f.seek(n * np.dtype(dtype).itemsize, 1)
        return np.memmap(path, dtype=dtype, mode="r", offset=off, shape=(n,)) if n else np.zeros(0, dtype)

    def header():
        one("i"), one("q"), one("q"), one("q"), one("B")
        if one("i") > 1:
            one("f")

    assert f.read(4) == b"IHNp"
    header()
    vec("<f8")
    cum = np.array(vec("<i4"))
    vec("<i4")
    offsets = vec("<u8")
    neighbors = vec("<i4")
    one("i"), one("i"), one("i"), one("i"), one("i")
    assert f.read(4) == b"IxPq"
    header()
    one("Q"), one("Q"), one("Q")
    vec("<f4")
    codes = vec("<u1")
    return offsets, neighbors, cum, codes


def lines_per_row(rows, lab, shift):
    x = np.where(rows >= 0, lab[np.maximum(rows, 0)] >> shift, -1).astype(np.int64)
    x.sort(axis=1)
    distinct = (np.diff(x, axis=1) != 0) & (x[:, 1:] >= 0)
    return (distinct.sum(axis=1) + (x[:, 0] >= 0)).mean()


ap = argparse.ArgumentParser()
ap.add_argument("--sample", type=int, default=1_000_000)
a = ap.parse_args()
wl = bench.prepare_c5(argparse.Namespace(cache="/tmp/drm_bench_cache", queries=1000, embed="gru"), bench.Dist(), 0)
t0 = time.time()
offsets, neighbors, cum, codes = ihnp_arrays(wl["index_path"])
n = len(offsets) - 1
deg0 = int(cum[1] - cum[0])
rng = np.random.default_rng(0)
nodes = np.sort(rng.choice(n, size=a.sample, replace=False))
rows = np.stack([np.asarray(neighbors[offsets[nodes] + j]) for j in range(deg0)], axis=1)
valid = (rows >= 0).sum(axis=1).mean()
d = np.abs(rows.astype(np.int64) - nodes[:, None])[rows >= 0]
print(f"C5 index: {n} nodes, deg0 {deg0}, {valid:.2f} valid links per row (sample {a.sample}, read in {time.time() - t0:.1f}s)")
print(f"|link - node|: median {np.median(d):.0f}, < 64: {(d < 64).mean():.3f}, < 512: {(d < 512).mean():.3f}, "
      f"< 4096: {(d < 4096).mean():.3f}")
labs = {"index ids": np.arange(n, dtype=np.int64), "random relabel": rng.permutation(n).astype(np.int64)}
t0 = time.time()
cm = np.asarray(codes).reshape(n, -1)
order = np.lexsort(tuple(cm[:, m] for m in reversed(range(cm.shape[1]))))
lab = np.empty(n, dtype=np.int64)
lab[order] = np.arange(n)
labs["PQ-code lexicographic"] = lab
print(f"(lexsort of the codes {time.time() - t0:.1f}s)")
for name, lab in labs.items():
    print(f"{name:>24}: bitmap lines (64 B) per row {lines_per_row(rows, lab, 9):.2f}, "
          f"128-B lines {lines_per_row(rows, lab, 10):.2f}, words {lines_per_row(rows, lab, 5):.2f}", flush=True)
