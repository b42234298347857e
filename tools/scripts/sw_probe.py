"""SW rerank throughput probe for the 64- and 152-column builds of sw_score_f16_kernel: random 150 bp windows,
random candidate ids, Q reads of 62 / 150 bases (tagged to 64 / 152 bytes). Prints ms and G cell-updates/s per
configuration; DRM_LIB selects the library (tools/scripts/ab_sw.sh). (Until round 4 it also capped the grid's
waves per CU, drm_refs_set_sw_waves, for the occupancy measurements of DESIGN.md sec. 4.4.)"""
import argparse
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from deepreadmapper_amd import WindowTable, synth  # noqa: E402
from deepreadmapper_amd._native import check, lib  # noqa: E402
from deepreadmapper_amd.device import DeviceBuffer, Event, Stream  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--queries", type=int, default=200_000)
ap.add_argument("--windows", type=int, default=1_000_000)
ap.add_argument("--band", type=int, default=0, help="opt-in banded DP half-width (drm_refs_set_sw_band), 0 = full")
a = ap.parse_args()
K = 128
g = synth.genome(a.windows // 2 + 149, seed=3)
refs = synth.windows_lookup(g, 150, 1)
table = WindowTable(refs)
table.sw_band = a.band
rng = np.random.default_rng(1)
I = rng.integers(0, len(refs), size=(a.queries, K)).astype(np.int64)
d_I = DeviceBuffer.from_host(I)
st = Stream()
for rl in (62, 150):
    reads, _, _ = synth.simulate_reads(g, a.queries, read_len=rl, seed=5)
    q = synth.tag(reads)
    d_q = DeviceBuffer.from_host(q)
    d_ql = DeviceBuffer.from_host(np.full(a.queries, q.shape[1], dtype=np.int32))
    d_sc, d_id, d_st = (DeviceBuffer((a.queries, K), np.int32), DeviceBuffer((a.queries, K), np.uint64),
                        DeviceBuffer(a.queries, np.int32))
    cells = float(a.queries) * K * 150 * q.shape[1]

    def run():
        check(lib().drm_post_process_sw_static_device(table.handle, d_I.ptr, a.queries, K, d_q.ptr, d_ql.ptr,
                                                      q.shape[1], 1, K, K, d_sc.ptr, d_id.ptr, d_st.ptr, st.handle))
    run()
    st.synchronize()
    ts = []
    for _ in range(3):
        e0, e1 = Event(), Event()
        e0.record(st)
        run()
        e1.record(st)
        st.synchronize()
        ts.append(e0.elapsed_ms(e1))
    ms = min(ts)
    print(f"band {a.band} query {q.shape[1]} B: {ms:.2f} ms, {cells / ms / 1e6:.1f} G cells/s (full-DP cells)",
          flush=True)
