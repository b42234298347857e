"""C5 search alone (the bench's workload, built here if absent): HIP-event time of full-batch searches at
EF = K (default 128), plus mean ndis / nhops and a checksum of the ids. Knobs come from the environment
(e.g. DRM_SEARCH_INLINE=0/1), so alternate invocations A/B kernel variants on one box."""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, ".")
import bench  # noqa: E402
from deepreadmapper_amd import HnswPqIndex  # noqa: E402
from deepreadmapper_amd.device import DeviceBuffer, Event, Stream  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--k", type=int, default=128)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--embed", default="gru")
a = ap.parse_args()
wl = bench.prepare_c5(argparse.Namespace(cache="/tmp/drm_bench_cache", queries=1_250_000, embed=a.embed), bench.Dist(), 0)
Q, K = wl["Q"], a.k
ix = HnswPqIndex(wl["index_path"], 0)
d_x = DeviceBuffer.from_host(wl["q_emb"])
d_D, d_I = DeviceBuffer((Q, K), np.float32), DeviceBuffer((Q, K), np.int64)
nd, nh = DeviceBuffer(Q, np.int32), DeviceBuffer(Q, np.int32)
st = Stream()
ix.search_device(d_x, Q, K, 128, d_D, d_I, nd, nh, st)
st.synchronize()
ts = []
for _ in range(a.reps):
    e0, e1 = Event(), Event()
    e0.record(st)
    ix.search_device(d_x, Q, K, 128, d_D, d_I, nd, nh, st)
    e1.record(st)
    st.synchronize()
    ts.append(e0.elapsed_ms(e1))
I = d_I.download()
print(f"search K={K} inline={os.environ.get('DRM_SEARCH_INLINE', '1')}: {min(ts):.2f} ms (all {[round(t, 2) for t in ts]}), "
      f"ndis {nd.download().mean():.1f}, nhops {nh.download().mean():.1f}, ids checksum {int(I.sum() % 1000003)}", flush=True)
