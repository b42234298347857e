"""Which of the round-5 suspects makes a device checksum return a stale sum.

The first form of drm_device_checksum (drm_debug_checksum_pool: hipMallocAsync + hipMemsetAsync + per-wave atomics +
an async copy into pageable host memory, on the caller's stream) against the suspects the review named:
  cross   the caller's writes on another stream, no event: a delayed writer (drm_debug_delayed_fill, 100 ms) on
          stream A, the checksum on stream B; then the same with an event recorded on A and waited for on B;
  pool    pool reuse across streams after hipFreeAsync: 200 checksums alternating between two streams, with
          unrelated hipMallocAsync / hipFreeAsync churn on the other stream between them, each of a buffer written on
          the checksum's own stream just before;
  h2d     pageable H2D copies (hipMemcpy from numpy) immediately followed by a checksum on a non-blocking stream.
Each line: scenario, form (pool = the first form, current = drm_device_checksum), checks, stale sums. Run on the
GPU box: python tools/scripts/checksum_hazard.py [--quick]."""
import argparse
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from deepreadmapper_amd._native import check, lib  # noqa: E402
from deepreadmapper_amd.device import DeviceBuffer, Event, Stream, host_checksum, synchronize  # noqa: E402

NB = 16 << 20


def fill_sum(v, cache={}):
    if v not in cache:
        cache[v] = host_checksum(np.full(NB, v, dtype=np.uint8))
    return cache[v]


def bind():
    L = lib()
    L.drm_debug_checksum_pool.argtypes = [C.c_void_p, C.c_int64, C.POINTER(C.c_uint64), C.c_void_p]
    L.drm_debug_delayed_fill.argtypes = [C.c_void_p, C.c_int64, C.c_int32, C.c_int64, C.c_void_p]
    L.drm_debug_malloc_async.argtypes = [C.POINTER(C.c_void_p), C.c_size_t, C.c_void_p]
    L.drm_debug_free_async.argtypes = [C.c_void_p, C.c_void_p]
    return L


def csum(L, form, ptr, s):
    out = C.c_uint64(0)
    f = L.drm_debug_checksum_pool if form == "pool" else L.drm_device_checksum
    check(f(C.c_void_p(ptr), C.c_int64(NB), C.byref(out), C.c_void_p(s.handle if s is not None else None)))
    return int(out.value)


def cross(L, form, buf, event):
    a, b = Stream(), Stream()
    check(L.drm_debug_delayed_fill(C.c_void_p(buf.ptr), NB, 0, 0, None))
    synchronize()
    check(L.drm_debug_delayed_fill(C.c_void_p(buf.ptr), NB, 0x5A, 100_000, C.c_void_p(a.handle)))
    if event:
        e = Event()
        e.record(a)
        b.wait(e)
    got = csum(L, form, buf.ptr, b)
    synchronize()
    return got == fill_sum(0x5A), got == fill_sum(0)


def pool(L, form, buf, n):
    sa, sb = Stream(), Stream()
    stale = 0
    churn = []
    for i in range(n):
        s, o = (sa, sb) if i % 2 == 0 else (sb, sa)
        v = (i * 37 + 11) & 0xFF
        check(L.drm_debug_delayed_fill(C.c_void_p(buf.ptr), NB, v, 0, C.c_void_p(s.handle)))
        # unrelated stream-ordered allocations on the other stream (sizes spread over the pool's bins)
        p = C.c_void_p()
        check(L.drm_debug_malloc_async(C.byref(p), C.c_size_t(4096 << (i % 12)), C.c_void_p(o.handle)))
        churn.append((p, o))
        if len(churn) > 4:
            q, so = churn.pop(0)
            check(L.drm_debug_free_async(q, C.c_void_p(so.handle)))
        stale += csum(L, form, buf.ptr, s) != fill_sum(v)
    for q, so in churn:
        check(L.drm_debug_free_async(q, C.c_void_p(so.handle)))
    synchronize()
    return stale


def h2d(L, form, buf, n):
    s = Stream()
    stale = 0
    for i in range(n):
        v = (i * 53 + 7) & 0xFF
        host = np.full(NB, v, dtype=np.uint8)
        check(lib().drm_memcpy_h2d(C.c_void_p(buf.ptr), host.ctypes.data_as(C.c_void_p), C.c_size_t(NB)))
        stale += csum(L, form, buf.ptr, s) != fill_sum(v)
    return stale


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    n = 20 if ap.parse_args().quick else 200
    L = bind()
    buf = DeviceBuffer(NB, np.uint8)
    for form in ("pool", "current"):
        for event in (False, True):
            new, old = cross(L, form, buf, event)
            print(f"cross form={form:7s} event={int(event)}: {'correct' if new else ('STALE (the old contents)' if old else 'WRONG')}",
                  flush=True)
    for form in ("pool", "current"):
        print(f"pool  form={form:7s}: {n} checks, {pool(L, form, buf, n)} stale", flush=True)
        print(f"h2d   form={form:7s}: {n // 4} checks, {h2d(L, form, buf, n // 4)} stale", flush=True)


if __name__ == "__main__":
    main()
