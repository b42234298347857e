"""Diagnostic: does running the SW rerank of chunk c (stream B) beside the search of chunk c+1
(stream A) beat the sequential step? C3-flat workload (bench.py's default), run on the GPU box after
bench.py built the cache. Prints ms per 100k-read step for sequential and C-chunk pipelines."""
import ctypes as C
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from deepreadmapper_amd import synth  # noqa: E402
from deepreadmapper_amd.device import DeviceBuffer, Event, Stream, synchronize  # noqa: E402
from deepreadmapper_amd.flat import HnswFlatIndex  # noqa: E402
from deepreadmapper_amd.rerank import WindowTable  # noqa: E402
from deepreadmapper_amd._native import lib, check  # noqa: E402

Q, K, EF = 100_000, 128, 128
w = synth.Workload("c3", 500_149, Q, seed=42, read_seed=7).generate("/tmp/drm_bench_cache")
ix = HnswFlatIndex("/tmp/drm_bench_cache/c3_flat_M64_efc128.hnsw")
table = WindowTable(w.refs, 0)
queries = np.ascontiguousarray(w.queries[:Q])
QL = queries.shape[1]
d_x = DeviceBuffer.from_host(w.q_emb[:Q])
d_q = DeviceBuffer.from_host(queries)
d_ql = DeviceBuffer.from_host(np.full(Q, QL, dtype=np.int32))
d_D, d_L = DeviceBuffer((Q, K), np.float32), DeviceBuffer((Q, K), np.uint64)
d_nd, d_nh = DeviceBuffer(Q, np.int32), DeviceBuffer(Q, np.int32)
d_sc, d_id, d_st = DeviceBuffer((Q, K), np.int32), DeviceBuffer((Q, K), np.uint64), DeviceBuffer(Q, np.int32)
sa, sb = Stream(), Stream()
L = lib()


def search(lo, n, s):
    check(L.drm_flat_search_device(ix.handle, d_x.ptr + lo * 128 * 4, n, K, EF, d_D.ptr + lo * K * 4,
                                   d_L.ptr + lo * K * 8, d_nd.ptr + lo * 4, d_nh.ptr + lo * 4, None, s.handle))


def rerank(lo, n, s):
    check(L.drm_post_process_sw_static_device(table.handle, d_L.ptr + lo * K * 8, n, K, d_q.ptr + lo * QL,
                                              d_ql.ptr + lo * 4, QL, 1, K, K, d_sc.ptr + lo * K * 4,
                                              d_id.ptr + lo * K * 8, d_st.ptr + lo * 4, s.handle))


def step(chunks):
    if chunks == 0:
        search(0, Q, sa)
        rerank(0, Q, sa)
        return
    n = Q // chunks
    for c in range(chunks):
        search(c * n, n, sa)
        e = Event()
        e.record(sa)
        sb.wait(e)
        rerank(c * n, n, sb)
    e = Event()
    e.record(sb)
    sa.wait(e)


ref = None
for chunks in [0, 2, 4, 5, 8, 0]:
    step(chunks)
    synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        step(chunks)
    synchronize()
    ms = (time.perf_counter() - t0) / 5 * 1e3
    ids = d_id.download()
    if ref is None:
        ref = ids
    print(f"chunks={chunks} ms/step={ms:.3f} same_ids={np.array_equal(ids, ref)} "
          f"waves_per_cu={os.environ.get('DRM_SEARCH_WAVES_PER_CU', 'default')}", flush=True)
