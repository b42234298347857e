"""Device memory / stream / event plumbing over the C ABI (no torch on the product path)."""
import ctypes as C

import numpy as np

from ._native import check, lib, ptr


def device_count():
    n = C.c_int(0)
    check(lib().drm_device_count(C.byref(n)))
    return n.value


def set_device(dev):
    check(lib().drm_set_device(int(dev)))


def synchronize():
    check(lib().drm_device_sync())


class DeviceBuffer:
    """A hipMalloc'd buffer with a numpy dtype/shape attached."""

    def __init__(self, shape, dtype):
        self.shape = tuple(int(s) for s in (shape if isinstance(shape, (tuple, list)) else (shape,)))
        self.dtype = np.dtype(dtype)
        self.nbytes = int(np.prod(self.shape, dtype=np.int64)) * self.dtype.itemsize
        p = C.c_void_p()
        check(lib().drm_malloc(C.byref(p), max(self.nbytes, 1)))
        self.ptr = p.value

    @classmethod
    def from_host(cls, a):
        a = np.ascontiguousarray(a)
        b = cls(a.shape, a.dtype)
        b.upload(a)
        return b

    def upload(self, a):
        a = np.ascontiguousarray(a, dtype=self.dtype)
        assert a.nbytes == self.nbytes, (a.nbytes, self.nbytes)
        if self.nbytes:
            check(lib().drm_memcpy_h2d(self.ptr, ptr(a), self.nbytes))

    def download(self):
        out = np.empty(self.shape, dtype=self.dtype)
        if self.nbytes:
            check(lib().drm_memcpy_d2h(ptr(out), self.ptr, self.nbytes))
        return out

    def zero(self):
        check(lib().drm_memset(self.ptr, 0, max(self.nbytes, 1)))

    def free(self):
        if self.ptr:
            check(lib().drm_free(self.ptr))
            self.ptr = None

    def __del__(self):
        try:
            if getattr(self, "ptr", None):
                lib().drm_free(self.ptr)
        except Exception:
            pass


class Stream:
    def __init__(self):
        p = C.c_void_p()
        check(lib().drm_stream_create(C.byref(p)))
        self.handle = p.value

    def wait(self, event):
        """Work enqueued on this stream after the call waits for `event`."""
        check(lib().drm_stream_wait_event(self.handle, event.handle))

    def synchronize(self):
        check(lib().drm_stream_sync(self.handle))

    def __del__(self):
        try:
            if self.handle:
                lib().drm_stream_destroy(self.handle)
        except Exception:
            pass


class Event:
    def __init__(self):
        p = C.c_void_p()
        check(lib().drm_event_create(C.byref(p)))
        self.handle = p.value

    def record(self, stream=None):
        check(lib().drm_event_record(self.handle, stream.handle if stream is not None else None))

    def elapsed_ms(self, end):
        ms = C.c_float(0)
        check(lib().drm_event_elapsed_ms(self.handle, end.handle, C.byref(ms)))
        return ms.value

    def __del__(self):
        try:
            if self.handle:
                lib().drm_event_destroy(self.handle)
        except Exception:
            pass
