"""GPU microbench of the L2 rerank (drm_post_process_l2_static_device) at C5's per-GPU shape: 1.25M reads x
K = 128 candidates over a window-embedding table (random windows, embedded by the GRU model on the GPU),
labels drawn at random. Prints one JSON line; run under rocprofv3 --kernel-trace --stats for the split."""
import json
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from deepreadmapper_amd._native import check, lib  # noqa: E402
from deepreadmapper_amd.device import DeviceBuffer, Event, Stream  # noqa: E402
from deepreadmapper_amd.encoder import Encoder  # noqa: E402
from deepreadmapper_amd.rerank import WindowTable, embed_windows  # noqa: E402

n_ref = int(sys.argv[1]) if len(sys.argv) > 1 else 8_000_000
Q, K = int(sys.argv[2]) if len(sys.argv) > 2 else 1_250_000, 128
rng = np.random.default_rng(1)
win = np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, size=(n_ref, 150), dtype=np.uint8)]
t = WindowTable(win)
del win
enc = Encoder()
t0 = time.time()
embed_windows(t, enc)
embed_s = time.time() - t0
nb = rng.integers(0, n_ref, size=(Q, K), dtype=np.int64)
qe = rng.standard_normal((Q, 128), dtype=np.float32) * 0.1
d_nb, d_qe = DeviceBuffer.from_host(nb), DeviceBuffer.from_host(qe)
d_d, d_i, d_s = DeviceBuffer((Q, K), np.float32), DeviceBuffer((Q, K), np.uint64), DeviceBuffer(Q, np.int32)
st = Stream()


def run():
    check(lib().drm_post_process_l2_static_device(t.handle, d_nb.ptr, Q, K, d_qe.ptr, 128, 1, K, d_d.ptr, d_i.ptr,
                                                  d_s.ptr, st.handle))


run()
st.synchronize()
ts = []
for _ in range(5):
    a, b = Event(), Event()
    a.record(st)
    run()
    b.record(st)
    st.synchronize()
    ts.append(a.elapsed_ms(b))
assert (d_s.download() == K).all()
ms = float(np.mean(ts))
algo = float(Q) * K * (4 * 128 + 8) + Q * 4 * 128 + Q * K * 12  # fused path (K <= 128): no workspace
print(json.dumps({"n_ref": n_ref, "Q": Q, "K": K, "ms": round(ms, 3), "all_ms": [round(x, 3) for x in ts],
                  "embed_s": round(embed_s, 2), "GBps": round(algo / ms / 1e6, 1),
                  "frac": round(algo / ms / 1e6 / 8000, 4)}), flush=True)
