"""Time the GRU read encoder (drm_vectorize_device) on N synthetic 150 bp tagged reads resident in HBM."""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from deepreadmapper_amd import Encoder, synth  # noqa: E402
from deepreadmapper_amd.device import DeviceBuffer, Event, Stream  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_250_000
g = synth.genome(2_000_149, seed=1)
reads, _, _ = synth.simulate_reads(g, n, seed=3)
q = synth.tag(reads)
e = Encoder()
d_s, d_l = DeviceBuffer.from_host(q), DeviceBuffer.from_host(np.full(n, q.shape[1], dtype=np.int32))
d_o = DeviceBuffer((n, 128), np.float32)
st = Stream()
e.vectorize_device(d_s, d_l, n, q.shape[1], d_o, st)
st.synchronize()
ts = []
for _ in range(3):
    a, b = Event(), Event()
    a.record(st)
    e.vectorize_device(d_s, d_l, n, q.shape[1], d_o, st)
    b.record(st)
    st.synchronize()
    ts.append(a.elapsed_ms(b))
ms = min(ts)
flop = n * 2 * 123 * 2 * 64 * 3 * ((64 + 128) + (256 + 128))  # MFMA flops incl. the hi/lo split
print(f"n={n} encoder {ms:.2f} ms  {n / ms * 1e3 / 1e6:.2f} M reads/s  MFMA {flop / ms / 1e9:.1f} TFLOP/s "
      f"(f16 dense peak 2500)  times {['%.2f' % t for t in ts]}")
o = d_o.download()
print("finite", np.isfinite(o).all(), "max|v|", float(np.abs(o).max()))
