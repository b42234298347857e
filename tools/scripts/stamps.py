"""Diagnostic: section time shares of the HNSW-PQ search kernel (stamped build, DRM_SEARCH_STAMPS=1).
Run on the GPU box after the bench cache exists: DRM_SEARCH_STAMPS=1 python tools/scripts/stamps.py
(DRM_SEARCH_FAST=0 stamps the general exact kernel instead of the lean one)."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from deepreadmapper_amd import synth  # noqa: E402
from deepreadmapper_amd.device import DeviceBuffer, synchronize  # noqa: E402
from deepreadmapper_amd.search import HnswPqIndex  # noqa: E402
from deepreadmapper_amd._native import lib, check  # noqa: E402

if len(sys.argv) > 1 and sys.argv[1] in ("c5", "c5gru"):  # the bench's C5 workload (built here if absent)
    import argparse
    import bench
    args = argparse.Namespace(cache="/tmp/drm_bench_cache", queries=1_250_000,
                              embed="gru" if sys.argv[1] == "c5gru" else "kmer3")
    wl = bench.prepare_c5(args, bench.Dist(), 0)
    q_emb, index_path = wl["q_emb"], wl["index_path"]
else:
    w = synth.Workload("c3", 500_149, 100_000, seed=42, read_seed=7).generate("/tmp/drm_bench_cache")
    q_emb, index_path = w.q_emb, w.index_path
ix = HnswPqIndex(index_path)
Q = len(q_emb)
dq = DeviceBuffer.from_host(q_emb[:Q])
dD, dI = DeviceBuffer((Q, 128), np.float32), DeviceBuffer((Q, 128), np.int64)
ix.search_device(dq, Q, 128, 128, dD, dI)
synchronize()
out = np.zeros(16, dtype=np.uint64)
L = lib()
L.drm_debug_search_stamps.argtypes = [C.c_void_p, C.c_void_p]
check(L.drm_debug_search_stamps(ix.handle, out.ctypes.data))
if os.environ.get("DRM_SEARCH_FAST", "1") != "0":
    names = ["lut", "greedy_upper", "pop_min+count_below", "distances+prediction+row prefetch", "-",
             "push loop (heap-id tests, pushes, log)", "output", "queue/top", "-", "-", "row wait (hop start)", "-"]
else:
    names = ["lut", "greedy_upper", "pop_min+count_below", "row+visited(+spec codes)", "distances+prefetch",
             "push loop: fetch/reject/overhead", "output+clear", "queue/top", "push loop: add_result",
             "push loop: evict (heap_pop)", "push loop: heap_push", "-"]
if os.environ.get("DRM_SEARCH_FAST", "1") != "0":
    print(f"row prediction hits {int(out[8])} of {int(out[9])} hops ({out[8] / max(out[9], 1) * 100:.1f} %)")
    if out[11]:
        print(f"full-heap replace pushes {int(out[11])} ({out[11] / max(out[9], 1):.2f} per hop)")
    if out[4]:
        print(f"links tested against the heap's ids {int(out[4])} ({out[4] / max(out[9], 1):.2f} per hop)")
    if out[12] + out[13] + out[14]:
        nl = out[12] + out[13] + out[14]
        print(f"level-0 hops whose row's valid links span 1 / 2 / 3 lines: {int(out[12])} / {int(out[13])} / "
              f"{int(out[14])} ({out[12] / nl * 100:.1f} / {out[13] / nl * 100:.1f} / {out[14] / nl * 100:.1f} %), "
              f"{(out[12] + 2 * out[13] + 3 * out[14]) / nl:.3f} lines per hop")
    out[4] = out[8] = out[9] = out[11] = out[12] = out[13] = out[14] = 0  # counts; out[10] is the hop-start row wait
out = out[:12]
tot = float(out.sum())
for n, v in zip(names, out):
    print(f"{n:32s} {v / tot * 100:6.2f} %")
