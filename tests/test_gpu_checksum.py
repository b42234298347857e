"""The device checksum that guards the replica broadcast and the N > 1 result gather (drm_device_checksum, DESIGN.md
sec. 5): its round-5 stale sums, reproduced and fixed.

The hazard: a checksum enqueued on one stream reads the buffer while writes the caller issued on another stream, with
no event between them, are still in flight -- it returns the sum of the old contents. A writer kernel that holds its
stream for 50 ms before filling the buffer (drm_debug_delayed_fill) makes that deterministic. The round-5 first form
(drm_debug_checksum_pool: stream-ordered pool, memset, atomics, async copy into pageable memory) returns the stale sum
without an event and the right one with it; drm_device_checksum now waits for all of the process's device work before
it reads, and returns the right sum either way -- also right after a pageable hipMemcpy H2D, whose DMA the first form
could still see landing (profiles/r06/checksum_hazard.txt: 7 stale sums in 50). The other two suspects of the review
(pool reuse across streams after hipFreeAsync, the pageable async D2H) are exercised with ordered writes: no stale
sum."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

NB = 4 << 20


@pytest.fixture(scope="module")
def env():
    from deepreadmapper_amd._native import lib
    from deepreadmapper_amd.device import DeviceBuffer, host_checksum
    L = lib()
    L.drm_debug_checksum_pool.argtypes = [C.c_void_p, C.c_int64, C.POINTER(C.c_uint64), C.c_void_p]
    L.drm_debug_delayed_fill.argtypes = [C.c_void_p, C.c_int64, C.c_int32, C.c_int64, C.c_void_p]
    L.drm_debug_malloc_async.argtypes = [C.POINTER(C.c_void_p), C.c_size_t, C.c_void_p]
    L.drm_debug_free_async.argtypes = [C.c_void_p, C.c_void_p]
    sums = {v: host_checksum(np.full(NB, v, dtype=np.uint8)) for v in (0x00, 0x5A, 0xC3)}
    return L, DeviceBuffer(NB, np.uint8), sums


def _sum(L, form, buf, stream):
    from deepreadmapper_amd._native import check
    out = C.c_uint64(0)
    f = L.drm_debug_checksum_pool if form == "pool" else L.drm_device_checksum
    check(f(C.c_void_p(buf.ptr), C.c_int64(NB), C.byref(out), C.c_void_p(stream.handle)))
    return int(out.value)


def _delayed(L, buf, value, delay_us, stream):
    from deepreadmapper_amd._native import check
    check(L.drm_debug_delayed_fill(C.c_void_p(buf.ptr), NB, value, delay_us,
                                   C.c_void_p(stream.handle if stream is not None else None)))


def _cross(env, form, event, value):
    from deepreadmapper_amd.device import Event, Stream, synchronize
    L, buf, sums = env
    _delayed(L, buf, 0, 0, None)
    synchronize()
    a, b = Stream(), Stream()
    _delayed(L, buf, value, 50_000, a)  # stream a: 50 ms, then the new contents
    if event:
        e = Event()
        e.record(a)
        b.wait(e)
    got = _sum(L, form, buf, b)
    synchronize()
    return got


def test_first_form_reads_stale_without_event(env):
    """The round-5 first form on stream b, the writer on stream a, no event: the sum of the OLD contents."""
    _, _, sums = env
    assert _cross(env, "pool", False, 0x5A) == sums[0x00]
    assert _cross(env, "pool", True, 0x5A) == sums[0x5A]


def test_device_checksum_orders_after_other_streams(env):
    """drm_device_checksum returns the new contents' sum with or without the caller's event."""
    _, _, sums = env
    assert _cross(env, "current", False, 0xC3) == sums[0xC3]
    assert _cross(env, "current", True, 0x5A) == sums[0x5A]


def test_pool_reuse_and_pageable_copy_with_ordered_writes(env):
    """The first form with the writes ordered on its own stream, 40 times, alternating two streams with unrelated
    hipMallocAsync / hipFreeAsync on the other one between them (pool reuse across streams), each result through the
    async copy into pageable memory: every sum is right."""
    from deepreadmapper_amd._native import check
    from deepreadmapper_amd.device import Stream, host_checksum, synchronize
    L, buf, _ = env
    sa, sb = Stream(), Stream()
    cache, churn, bad = {}, [], 0
    for i in range(40):
        s, o = (sa, sb) if i % 2 == 0 else (sb, sa)
        v = (i * 37 + 11) & 0xFF
        _delayed(L, buf, v, 0, s)
        p = C.c_void_p()
        check(L.drm_debug_malloc_async(C.byref(p), C.c_size_t(4096 << (i % 12)), C.c_void_p(o.handle)))
        churn.append((p, o))
        if len(churn) > 4:
            q, so = churn.pop(0)
            check(L.drm_debug_free_async(q, C.c_void_p(so.handle)))
        if v not in cache:
            cache[v] = host_checksum(np.full(NB, v, dtype=np.uint8))
        bad += _sum(L, "pool", buf, s) != cache[v]
    for q, so in churn:
        check(L.drm_debug_free_async(q, C.c_void_p(so.handle)))
    synchronize()
    assert bad == 0


def test_pageable_h2d_then_checksum_on_a_nonblocking_stream(env):
    """A pageable hipMemcpy H2D (the legacy null stream) followed at once by drm_device_checksum on a non-blocking
    stream: the sum is the copied contents' every time (the first form returned 7 stale sums in 50 on the box,
    profiles/r06/checksum_hazard.txt: the DMA can still be landing when hipMemcpy returns)."""
    from deepreadmapper_amd._native import check, lib
    from deepreadmapper_amd.device import Stream, host_checksum
    L, buf, sums = env
    s = Stream()
    bad = 0
    for i in range(20):
        v = (0x00, 0x5A, 0xC3)[i % 3]
        host = np.full(NB, v, dtype=np.uint8)
        check(lib().drm_memcpy_h2d(C.c_void_p(buf.ptr), host.ctypes.data_as(C.c_void_p), C.c_size_t(NB)))
        bad += _sum(L, "current", buf, s) != sums[v]
    assert bad == 0
