"""Spatial partition of the C5 step: the search on one set of CUs beside the SW rerank on the complementary set.

The search is a latency-bound pointer chase whose throughput grows sub-linearly with the waves in flight (20 / 12 / 8
waves per CU: 157 / 220 / 273 ms, profiles/r03/coresident_probe_v4_prefetch.txt), while the SW rerank is VALU-bound
and needs two waves per SIMD. If the search's limit is a chip-wide resource, it loses little on a subset of the CUs at
full occupancy, and the SW rerank of the previous batch can run on the rest. This probe measures, on one GPU:
  * the search alone on CU-masked streams covering a fraction f of the CUs (mask bits 0 .. f*CUs; the driver deals
    a stream's mask bits across the XCDs), and the SW rerank alone on the complement;
  * the concurrent pair (search of all reads on mask A beside the SW of all reads on mask B), and checks that the
    pair's outputs equal the sequential run's.
"""
import argparse
import ctypes as C
import sys

import numpy as np

sys.path.insert(0, ".")
import bench  # noqa: E402
from deepreadmapper_amd import HnswPqIndex, WindowTable  # noqa: E402
from deepreadmapper_amd._native import check, lib  # noqa: E402
from deepreadmapper_amd.device import DeviceBuffer, Event, Stream  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--queries", type=int, default=1_250_000)
ap.add_argument("--embed", default="gru")
ap.add_argument("--fracs", default="0.5,0.375,0.3125,0.25")
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
d_I2 = DeviceBuffer((Q, K), np.int64)
d_sc, d_id, d_st = DeviceBuffer((Q, K), np.int32), DeviceBuffer((Q, K), np.uint64), DeviceBuffer(Q, np.int32)
d_nd, d_nh = DeviceBuffer(Q, np.int32), DeviceBuffer(Q, np.int32)
L = lib()
hip = C.CDLL("libamdhip64.so")
ncu = C.c_int(0)
hip.hipDeviceGetAttribute(C.byref(ncu), 63, 0)  # hipDeviceAttributeMultiprocessorCount (ROCm 7 enum)
ncu = ncu.value
print(f"[cumask] C5 Q={Q}, {ncu} CUs", flush=True)


def masked_stream(bits):
    words = (ncu + 31) // 32
    m = (C.c_uint32 * words)()
    for b in bits:
        m[b // 32] |= 1 << (b % 32)
    s = C.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(C.byref(s), C.c_uint32(words), m)
    if rc != 0:
        raise RuntimeError(f"hipExtStreamCreateWithCUMask: {rc}")
    st = Stream.__new__(Stream)
    st.handle = s.value
    return st


def search(st, dI):
    check(L.drm_search_device_ex(ix.handle, d_x.ptr, Q, K, 128, d_D.ptr, dI.ptr, d_nd.ptr, d_nh.ptr, None, st.handle))


def sw(st, dI):
    check(L.drm_post_process_sw_static_device(table.handle, dI.ptr, Q, K, d_q.ptr, d_ql.ptr, q.shape[1], 1, K, K,
                                              d_sc.ptr, d_id.ptr, d_st.ptr, st.handle))


def timed(streams, fn, reps=2):
    fn()
    for s in streams:
        s.synchronize()
    best = 1e30
    for _ in range(reps):
        t0 = Event()
        t0.record(streams[0])
        for s in streams[1:]:
            s.wait(t0)
        fn()
        for s in streams[1:]:
            e = Event()
            e.record(s)
            streams[0].wait(e)
        t1 = Event()
        t1.record(streams[0])
        streams[0].synchronize()
        best = min(best, t0.elapsed_ms(t1))
    return best


full = masked_stream(range(ncu))
ms_s = timed([full], lambda: search(full, d_I))
ms_w = timed([full], lambda: sw(full, d_I))
ref_I, ref_id, ref_sc = d_I.download(), d_id.download(), d_sc.download()
print(f"full chip: search {ms_s:.1f} ms, SW {ms_w:.1f} ms, sequential {ms_s + ms_w:.1f} ms "
      f"({Q / (ms_s + ms_w) * 1e3 / 1e6:.3f} M reads/s)", flush=True)
d_I2.upload(ref_I)  # the pair's SW reranks the previous batch's neighbours (here: the same reads')
for f in (float(x) for x in a.fracs.split(",")):
    n = int(round(f * ncu))
    sa, sb = masked_stream(range(n)), masked_stream(range(n, ncu))
    t_s = timed([sa], lambda: search(sa, d_I))
    t_w = timed([sb], lambda: sw(sb, d_I2))
    same_s = np.array_equal(d_I.download(), ref_I)

    def pair():
        search(sa, d_I)
        sw(sb, d_I2)

    t_p = timed([sa, sb], pair)
    same = same_s and np.array_equal(d_I.download(), ref_I) and np.array_equal(d_id.download(), ref_id) and \
        np.array_equal(d_sc.download(), ref_sc)
    print(f"search on {n} CUs: {t_s:.1f} ms ({ms_s / t_s * ncu / n:.2f}x per-CU rate); SW on {ncu - n} CUs: {t_w:.1f} ms; "
          f"pair {t_p:.1f} ms ({Q / t_p * 1e3 / 1e6:.3f} M reads/s)  identical={same}", flush=True)

import os  # noqa: E402
os._exit(0)  # skip interpreter teardown of the CU-masked streams (the first run hung there after its last line)
