"""Experiment: overlap search(batch i+1) with SW rerank(batch i) on two streams (C3 workload).
Usage (GPU box): DRM_SEARCH_WAVES_PER_CU=8 python tools/scripts/overlap_probe.py"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from deepreadmapper_amd import synth  # noqa: E402
from deepreadmapper_amd.device import DeviceBuffer, Event, Stream, synchronize  # noqa: E402
from deepreadmapper_amd.search import HnswPqIndex  # noqa: E402
from deepreadmapper_amd.rerank import WindowTable  # noqa: E402
from deepreadmapper_amd._native import check, lib  # noqa: E402

Q, K, B = 100_000, 128, int(os.environ.get("BATCHES", "6"))
w = synth.Workload("c3", 500_149, Q, seed=42, read_seed=7).generate("/tmp/drm_bench_cache")
ix = HnswPqIndex(w.index_path)
table = WindowTable(w.refs)
d_x = DeviceBuffer.from_host(w.q_emb[:Q])
d_q = DeviceBuffer.from_host(np.ascontiguousarray(w.queries[:Q]))
d_ql = DeviceBuffer.from_host(np.full(Q, w.queries.shape[1], dtype=np.int32))
bufs = [dict(D=DeviceBuffer((Q, K), np.float32), I=DeviceBuffer((Q, K), np.int64),
             sc=DeviceBuffer((Q, K), np.int32), id=DeviceBuffer((Q, K), np.uint64), st=DeviceBuffer(Q, np.int32))
        for _ in range(2)]
sA, sB = Stream(), Stream()


def search(b, s):
    ix.search_device(d_x, Q, K, 128, b["D"], b["I"], None, None, s)


def sw(b, s):
    check(lib().drm_post_process_sw_static_device(table.handle, b["I"].ptr, Q, K, d_q.ptr, d_ql.ptr,
                                                  w.queries.shape[1], 1, K, K, b["sc"].ptr, b["id"].ptr,
                                                  b["st"].ptr, s.handle))


def run(overlap):
    synchronize()
    t0 = time.perf_counter()
    done = [Event(), Event()]
    searched = [Event(), Event()]
    for i in range(B):
        b = bufs[i % 2]
        if overlap:
            if i >= 2:
                sA.wait(done[i % 2])  # buffer reuse
            search(b, sA)
            searched[i % 2].record(sA)
            sB.wait(searched[i % 2])
            sw(b, sB)
            done[i % 2].record(sB)
        else:
            search(b, sA)
            sw(b, sA)
    synchronize()
    return (time.perf_counter() - t0) / B * 1e3


run(False)
for _ in range(2):
    print(f"sequential {run(False):.2f} ms/batch   overlapped {run(True):.2f} ms/batch", flush=True)
