import ctypes as C, sys
sys.path.insert(0, ".")
from deepreadmapper_amd._native import lib
for gb in (0.25, 1, 4, 16, 32):
    for waves in (256, 5120):
        ns = C.c_double(0)
        rc = lib().drm_device_chase_latency(0, int(gb * (1 << 30)), waves, 2000, C.byref(ns))
        print(f"footprint {gb:6.2f} GB, {waves:5d} waves: {ns.value:7.0f} ns per dependent 384-B row load (rc {rc})", flush=True)
