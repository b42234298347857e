"""Co-resident search + SW rerank at C5 (1.25M reads, inputs resident in HBM).

Measures, on one GPU:
  * the search alone at 20 / 12 / 11 resident waves per CU, the SW rerank alone uncapped and capped at
    4 waves per CU (one per SIMD);
  * the lockstep pipeline over P chunks: phase p runs search(p) (capped grid) beside SW(p-1) (capped grid)
    on two streams, phase 0 the first search alone (full grid), phase P the last SW alone (full grid);
and checks that every schedule's SW ids / scores equal the sequential run's.
"""
import argparse
import sys
import time

import numpy as np

sys.path.insert(0, ".")
import bench  # noqa: E402
from deepreadmapper_amd import HnswPqIndex, WindowTable  # noqa: E402
from deepreadmapper_amd._native import check, lib  # noqa: E402
from deepreadmapper_amd.device import DeviceBuffer, Event, Stream  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--queries", type=int, default=1_250_000)
ap.add_argument("--embed", default="gru")
ap.add_argument("--chunks", default="4,6,8")
ap.add_argument("--search-waves", default="12,11")
ap.add_argument("--sw-waves", default="4")
ap.add_argument("--lockstep", action="store_true", help="also time the script-level lockstep schedule")
a = ap.parse_args()
args = argparse.Namespace(cache="/tmp/drm_bench_cache", queries=a.queries, embed=a.embed)
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


d_nd0, d_nh0 = DeviceBuffer(Q, np.int32), DeviceBuffer(Q, np.int32)


def search(lo, hi, st, waves):
    # ndis / nhops buffers given: without them drm_search_device_ex allocates a temporary and synchronises
    check(L.drm_index_set_search_waves(ix.handle, waves))
    check(L.drm_search_device_ex(ix.handle, d_x.ptr + lo * 512, hi - lo, K, 128, d_D.ptr + lo * K * 4,
                                 d_I.ptr + lo * K * 8, d_nd0.ptr + lo * 4, d_nh0.ptr + lo * 4, None, st.handle))


def sw(lo, hi, st, waves):
    check(L.drm_refs_set_sw_waves(table.handle, waves))
    check(L.drm_post_process_sw_static_device(table.handle, d_I.ptr + lo * K * 8, hi - lo, K, d_q.ptr + lo * q.shape[1],
                                              d_ql.ptr + lo * 4, q.shape[1], 1, K, K, d_sc.ptr + lo * K * 4,
                                              d_id.ptr + lo * K * 8, d_st.ptr + lo * 4, st.handle))


def timed(fn, reps=2):
    fn()
    s0.synchronize()
    s1.synchronize()
    best = 1e30
    for _ in range(reps):
        t0, t1 = Event(), Event()
        t0.record(s0)
        s1.wait(t0)
        fn()
        e = Event()
        e.record(s1)
        s0.wait(e)
        t1.record(s0)
        s0.synchronize()
        best = min(best, t0.elapsed_ms(t1))
    return best


def seq():
    search(0, Q, s0, 20)
    e = Event()
    e.record(s0)
    s1.wait(e)
    sw(0, Q, s1, 0)


def lockstep(P, ws, wsw):
    b = [Q * i // P for i in range(P + 1)]
    prev_s1 = None
    for p in range(P + 1):
        # phase p: search(p) on s0 beside SW(p-1) on s1; both start together
        e0 = Event()
        e0.record(s0)
        s1.wait(e0)
        if prev_s1 is not None:
            s0.wait(prev_s1)
        alone_search = p == 0
        alone_sw = p == P
        if p < P:
            search(b[p], b[p + 1], s0, 20 if alone_search else ws)
        if p > 0:
            # SW(p-1) needs search(p-1): it ran in the previous phase, which s1 waited for above
            sw(b[p - 1], b[p], s1, 0 if alone_sw else wsw)
        prev_s1 = Event()
        prev_s1.record(s1)
    s0.wait(prev_s1)


print(f"[co] C5 Q={Q}", flush=True)
for w in (20,) + tuple(int(x) for x in a.search_waves.split(",")):
    ms = timed(lambda: search(0, Q, s0, w))
    print(f"search alone, {w} waves/CU: {ms:.1f} ms", flush=True)
for w in (0,) + tuple(int(x) for x in a.sw_waves.split(",")):
    ms = timed(lambda: sw(0, Q, s0, w))
    print(f"SW alone, cap {w} waves/CU: {ms:.1f} ms", flush=True)
ms = timed(seq)
ref_id, ref_sc = d_id.download(), d_sc.download()
print(f"sequential (search 20 + SW uncapped): {ms:.1f} ms  {Q / ms * 1e3 / 1e6:.3f} M reads/s", flush=True)
# independent pair: the search of all reads on s0 beside the SW of all reads (the previous run's neighbours) on s1
for ws in (int(x) for x in a.search_waves.split(",")):
    for wsw in (int(x) for x in a.sw_waves.split(",")):
        def pair():
            search(0, Q, s0, ws)
            sw(0, Q, s1, wsw)
        ms = timed(pair)
        print(f"independent pair: search {ws} waves/CU on s0 beside SW {wsw} waves/CU on s1: {ms:.1f} ms", flush=True)
for P in (int(x) for x in a.chunks.split(",")) if a.lockstep else ():
    for ws in (int(x) for x in a.search_waves.split(",")):
        for wsw in (int(x) for x in a.sw_waves.split(",")):
            d_id.zero()
            ms = timed(lambda: lockstep(P, ws, wsw))
            same = np.array_equal(d_id.download(), ref_id) and np.array_equal(d_sc.download(), ref_sc)
            print(f"lockstep P={P} search {ws} + SW {wsw} waves/CU: {ms:.1f} ms  {Q / ms * 1e3 / 1e6:.3f} M reads/s"
                  f"  identical={same}", flush=True)
check(L.drm_index_set_search_waves(ix.handle, 0))
check(L.drm_refs_set_sw_waves(table.handle, 0))

# the library's own co-scheduled entry point (drm_search_rerank_device)
import os  # noqa: E402
from deepreadmapper_amd.executor import search_rerank_device  # noqa: E402
d_nd, d_nh, d_nu = DeviceBuffer(Q, np.int32), DeviceBuffer(Q, np.int32), DeviceBuffer(Q, np.int32)
for P in (int(x) for x in a.chunks.split(",")):
    for ws in (int(x) for x in a.search_waves.split(",")):
        os.environ.update(DRM_CO_BATCHES=str(P), DRM_CO_SEARCH_WAVES=str(ws), DRM_CO_SW_WAVES=a.sw_waves.split(",")[-1])
        d_id.zero()
        best = None
        for _ in range(3):
            st = search_rerank_device(ix, table, d_x, Q, d_q, d_ql, q.shape[1], d_D, d_I, d_sc, d_id, d_st, k=K,
                                      ef=128, d_ndis=d_nd, d_nhops=d_nh, d_nhops_upper=d_nu, stream=s0, stats=True)
            best = st if best is None or st.kernel_ms < best.kernel_ms else best
        same = np.array_equal(d_id.download(), ref_id) and np.array_equal(d_sc.download(), ref_sc)
        print(f"drm_search_rerank_device P={P} search {ws}: span {best.kernel_ms:.1f} ms "
              f"({Q / best.kernel_ms * 1e3 / 1e6:.3f} M reads/s), search launches {best.search_ms:.1f}, SW launches "
              f"{best.sw_ms:.1f}, first search {best.first_search_ms:.1f}, last SW {best.last_sw_ms:.1f}  "
              f"identical={same}", flush=True)
