"""Host models of the lean search kernel (tools/emu/): its wave-parallel MinimaxHeap with node ids
(Heap::replace128 / push_fill, pop_min's slot marking, Heap::holds) against a literal faiss MinimaxHeap under
random pushes and pops with many equal distances, and its level-0 loop -- the heap as the visited set, the log of
tied evictions, the result set from the heap plus that log -- over the committed C1 fixture, which must give the
committed rows with no node pushed twice and the log within its capacity. CPU only: each lane of the wave is a loop index."""
import ctypes as C
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import GOLDEN, ROOT

EMU = os.path.join(ROOT, "tools", "emu")


def _build(tmp, src, shared):
    out = os.path.join(tmp, os.path.basename(src).replace(".cpp", ".so" if shared else ""))
    cmd = ["g++", "-O2", "-std=c++17", os.path.join(EMU, src), "-o", out] + (["-shared", "-fPIC"] if shared else [])
    subprocess.run(cmd, check=True)
    return out


def test_heap_model_vs_literal_faiss_heap(tmp_path):
    exe = _build(str(tmp_path), "heap_emu.cpp", False)
    r = subprocess.run([exe, "120"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and r.stdout.startswith("ok:"), r.stdout + r.stderr


def test_kernel_model_c1_fixture(tmp_path):
    sys.path.insert(0, os.path.dirname(__file__))
    import faiss_literal as FL
    from oracle import faiss_file, oracle as O
    lib = C.CDLL(_build(str(tmp_path), "kernel_emu.cpp", True))
    path = os.path.join(GOLDEN, "c1_hnswpq.index")
    fx = faiss_file.read(path)
    q = np.load(os.path.join(GOLDEN, "c1_queries.npy"))
    exp = np.load(os.path.join(GOLDEN, "c1_expected_k128_ef128.npz"))
    ix = FL.LiteralIndex(fx)
    n, deg0 = fx.ntotal, ix.cum[1]
    nbr0 = np.ascontiguousarray(np.stack([fx.neighbors[ix.offsets[i]:ix.offsets[i] + deg0] for i in range(n)]),
                                dtype=np.int32)
    codes = np.ascontiguousarray(fx.codes, dtype=np.uint8)
    vp = C.c_void_p
    for r in range(len(q)):
        lut = np.ascontiguousarray(O.pq_distance_table(fx, q[r:r + 1])[0], dtype=np.float32)
        lut_l = FL.distance_table(ix, q[r])
        st = {"ndis": 0, "nhops": 0}
        nearest, dn = ix.entry_point, FL.distance_to_code(ix, lut_l, ix.entry_point)
        for level in range(ix.max_level, 0, -1):
            nearest, dn = FL.greedy_update_nearest(ix, lut_l, level, nearest, dn, st)
        ids, keys, stats = np.empty(128, np.int32), np.empty(128, np.uint32), np.zeros(4, np.int32)
        rc = lib.emu_search_one(nbr0.ctypes.data_as(vp), codes.ctypes.data_as(vp), C.c_int64(n), C.c_int(deg0),
                                lut.ctypes.data_as(vp), C.c_int32(nearest), C.c_float(dn), ids.ctypes.data_as(vp),
                                keys.ctypes.data_as(vp), stats.ctypes.data_as(vp))
        assert rc == 0, r
        assert ids.astype(np.int64).tolist() == exp["I"][r].tolist(), r
        assert stats[2] == 0 and stats[3] == 0, (r, stats.tolist())  # no node pushed twice, log within capacity
