"""Tiny IHNp graphs for the hand-derived traversal fixtures (tests/golden/hnsw_tie_cases.json) and for random
tie-heavy graphs -- TEST INFRASTRUCTURE ONLY. Writes the faiss on-disk layout (impl/index_write.cpp, fourcc
"IHNp" + storage "IxPq") with its own struct packing, independent of the library's writer.

PQ of every graph: d = 128, M = 8, nbits = 8; sub-quantizer m's centroid c is (c, 0, ..., 0). With the zero
query, a node with code (v, 0, ..., 0) is at ADC distance v^2 exactly (small integers, exact in fp32), so equal
distances are designed, not hoped for."""
import json
import os
import struct

import numpy as np

from conftest import GOLDEN

D, M_PQ, NBITS, DSUB, KSUB = 128, 8, 8, 16, 256
M_HNSW = 2
CUM = [0, 2 * M_HNSW] + [2 * M_HNSW + M_HNSW * l for l in range(1, 8)]  # level 0: 2M links, upper: M each


def centroids():
    c = np.zeros((M_PQ, KSUB, DSUB), dtype=np.float32)
    c[:, :, 0] = np.arange(KSUB, dtype=np.float32)[None, :]
    return c


def codes_for(dist):
    """Node codes (v, 0, ..., 0) with v^2 = dist."""
    v = np.rint(np.sqrt(np.asarray(dist, dtype=np.float64))).astype(np.int64)
    assert (v * v == np.asarray(dist)).all() and (v < KSUB).all(), "distances must be squares of codes < 256"
    codes = np.zeros((len(dist), M_PQ), dtype=np.uint8)
    codes[:, 0] = v
    return codes


def write_ihnp(path, rows, codes, entry_point, max_level, ef_search=16):
    """rows[i] = list of per-level link lists (level 0 first, 2*M_HNSW then M_HNSW slots, -1 padded)."""
    n = len(rows)
    levels = [len(r) for r in rows]
    offsets = [0]
    nbrs = []
    for r in rows:
        for l, lst in enumerate(r):
            width = CUM[l + 1] - CUM[l]
            assert len(lst) == width, (l, lst)
            nbrs.extend(int(v) for v in lst)
        offsets.append(len(nbrs))
    out = bytearray()

    def vec(fmt, vals):
        vals = list(vals)
        out.extend(struct.pack("<Q", len(vals)))
        out.extend(struct.pack("<%d%s" % (len(vals), fmt), *vals))

    def header():
        out.extend(struct.pack("<iqqqBi", D, n, 1 << 20, 1 << 20, 1, 1))

    out.extend(b"IHNp")
    header()
    vec("d", [0.5 ** (l + 1) for l in range(max(levels))])         # assign_probas (unused by search)
    vec("i", CUM[:max(levels) + 1])                                 # cum_nneighbor_per_level
    vec("i", levels)
    vec("Q", offsets)
    vec("i", nbrs)
    out.extend(struct.pack("<iiiii", entry_point, max_level, 40, ef_search, 1))
    out.extend(b"IxPq")
    header()
    out.extend(struct.pack("<QQQ", D, M_PQ, NBITS))
    vec("f", centroids().ravel().tolist())
    vec("B", np.asarray(codes, dtype=np.uint8).ravel().tolist())
    out.extend(struct.pack("<iBi", 0, 0, 0))
    with open(path, "wb") as f:
        f.write(bytes(out))
    return path


def load_cases():
    return json.load(open(os.path.join(GOLDEN, "hnsw_tie_cases.json")))["cases"]


def write_case(case, directory):
    n = len(case["dist"])
    rows = [case["rows"][str(i)] for i in range(n)]
    path = os.path.join(directory, case["name"] + ".index")
    write_ihnp(path, rows, codes_for(case["dist"]), case["entry_point"], case["max_level"])
    return path


def random_tie_graph(rng, n, n_levels_max=3, n_values=4, hole_p=0.2):
    """A random graph over n nodes whose distances take only `n_values` distinct values (ties everywhere),
    duplicate links and holes included. Returns (rows, codes, entry_point, max_level)."""
    vals = rng.choice(np.arange(1, 16), size=n_values, replace=False)
    codes = np.zeros((n, M_PQ), dtype=np.uint8)
    codes[:, 0] = rng.choice(vals, size=n)
    codes[:, 1] = rng.integers(0, 2, size=n)  # a second sub-quantizer adds 0 or 1: still few distinct sums
    levels = np.ones(n, dtype=np.int64)
    for l in range(1, n_levels_max):
        levels[rng.random(n) < 0.3 ** l] += 1
    max_level = int(levels.max()) - 1
    entry = int(rng.choice(np.flatnonzero(levels == levels.max())))
    rows = []
    for i in range(n):
        r = []
        for l in range(levels[i]):
            width = CUM[l + 1] - CUM[l]
            pool = np.flatnonzero(levels > l)
            pool = pool[pool != i]
            k = int(rng.integers(0, width + 1)) if len(pool) else 0
            lst = [int(v) for v in rng.choice(pool, size=k)] if k else []  # with replacement: duplicates
            if lst and rng.random() < hole_p:
                lst = lst[:int(rng.integers(0, len(lst)))]
            r.append(lst + [-1] * (width - len(lst)))
        rows.append(r)
    return rows, codes, entry, max_level
