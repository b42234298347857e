"""Search / SW rerank overlap at C5 (1.25M reads, inputs resident): one stream (search all, then SW all)
vs P batches with the search of batch b+1 running beside the SW of batch b on a second stream."""
import argparse
import sys

import numpy as np

sys.path.insert(0, ".")
import bench  # noqa: E402
from deepreadmapper_amd import HnswPqIndex, WindowTable  # noqa: E402
from deepreadmapper_amd._native import check, lib  # noqa: E402
from deepreadmapper_amd.device import DeviceBuffer, Event, Stream  # noqa: E402

args = argparse.Namespace(cache="/tmp/drm_bench_cache", queries=1_250_000)
D = bench.Dist()
wl = bench.prepare_c5(args, D, 0)
Q, K = wl["Q"], 128
ix = HnswPqIndex(wl["index_path"], 0)
table = WindowTable(wl["refs"], 0)
q = wl["queries"]
d_x, d_q = DeviceBuffer.from_host(wl["q_emb"]), DeviceBuffer.from_host(q)
d_ql = DeviceBuffer.from_host(np.full(Q, q.shape[1], dtype=np.int32))
d_D, d_I = DeviceBuffer((Q, K), np.float32), DeviceBuffer((Q, K), np.int64)
d_sc, d_id, d_st = DeviceBuffer((Q, K), np.int32), DeviceBuffer((Q, K), np.uint64), DeviceBuffer(Q, np.int32)
s0, s1 = Stream(), Stream()
L = lib()


def search(lo, hi, st):
    check(L.drm_search_device_ex(ix.handle, d_x.ptr + lo * 512, hi - lo, K, 128, d_D.ptr + lo * K * 4,
                                 d_I.ptr + lo * K * 8, None, None, None, st.handle))


def sw(lo, hi, st):
    check(L.drm_post_process_sw_static_device(table.handle, d_I.ptr + lo * K * 8, hi - lo, K, d_q.ptr + lo * q.shape[1],
                                              d_ql.ptr + lo * 4, q.shape[1], 1, K, K, d_sc.ptr + lo * K * 4,
                                              d_id.ptr + lo * K * 8, d_st.ptr + lo * 4, st.handle))


def run(P):
    b = [Q * i // P for i in range(P + 1)]
    ev = [Event() for _ in range(P)]
    t0, t1 = Event(), Event()
    t0.record(s0)
    s1.wait(t0)
    for i in range(P):
        search(b[i], b[i + 1], s0)
        ev[i].record(s0)
        s1.wait(ev[i])
        sw(b[i], b[i + 1], s1)
    t1.record(s1)
    s1.synchronize()
    return t0.elapsed_ms(t1)


ref = None
for P in (1, 2, 4, 8, 1, 3, 6):
    run(P)
    ms = min(run(P) for _ in range(2))
    ids = d_id.download()
    same = ref is None or np.array_equal(ids, ref)
    ref = ids if ref is None else ref
    print(f"P={P}: {ms:.1f} ms  {Q / ms * 1e3 / 1e6:.3f} M reads/s  identical={same}", flush=True)
