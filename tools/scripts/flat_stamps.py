"""Diagnostic: section time shares of the fp32 search kernel (DRM_SEARCH_STAMPS=1), C3-flat workload.
Run on the GPU box after `bench.py --index flat` built the cache."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from deepreadmapper_amd import synth  # noqa: E402
from deepreadmapper_amd.device import DeviceBuffer, synchronize  # noqa: E402
from deepreadmapper_amd.flat import HnswFlatIndex  # noqa: E402
from deepreadmapper_amd._native import lib, check  # noqa: E402

w = synth.Workload("c3", 500_149, 100_000, seed=42, read_seed=7).generate("/tmp/drm_bench_cache")
ix = HnswFlatIndex("/tmp/drm_bench_cache/c3_flat_M64_efc128.hnsw")
Q = 100_000
dq = DeviceBuffer.from_host(w.q_emb[:Q])
dD, dL = DeviceBuffer((Q, 128), np.float32), DeviceBuffer((Q, 128), np.uint64)
nd, nh = DeviceBuffer(Q, np.int32), DeviceBuffer(Q, np.int32)
ix.search_device(dq, Q, 128, 128, dD, dL, nd, nh)
synchronize()
out = np.zeros(8, dtype=np.uint64)
L = lib()
L.drm_debug_flat_stamps.argtypes = [C.c_void_p, C.c_void_p]
check(L.drm_debug_flat_stamps(ix.handle, out.ctypes.data))
names = ["setup+upper levels", "candidate_set pop", "row+visited", "distances", "heap pushes/pops (lane 0)",
         "result order+reset", "-", "-"]
tot = float(out.sum())
for n, v in zip(names, out):
    print(f"{n:28s} {v / tot * 100:6.2f} %")
