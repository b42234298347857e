"""Device memory / stream / event plumbing over the C ABI (no torch on the product path)."""
import ctypes as C

import numpy as np

from ._native import check, lib, ptr


def device_count():
    n = C.c_int(0)
    check(lib().drm_device_count(C.byref(n)))
    return n.value


class DeviceProps(C.Structure):
    _fields_ = [("cu_count", C.c_int32), ("clock_khz", C.c_int32), ("total_mem", C.c_int64), ("lds_per_cu", C.c_int32),
                ("arch", C.c_char * 64)]


def device_props(dev=0):
    """drm_device_get_props: CU count, peak engine clock (kHz), HBM bytes, LDS per CU, arch, read at run time."""
    p = DeviceProps()
    check(lib().drm_device_get_props(int(dev), C.byref(p)))
    return {"cu_count": p.cu_count, "clock_hz": p.clock_khz * 1e3, "total_mem": p.total_mem,
            "lds_per_cu": p.lds_per_cu, "arch": p.arch.decode()}


def set_device(dev):
    check(lib().drm_set_device(int(dev)))


def synchronize():
    check(lib().drm_device_sync())


_GOLD = np.uint64(0x9E3779B97F4A7C15)


def host_checksum(a):
    """The host form of drm_device_checksum over the bytes of array a: sum mod 2^64 over its 8-byte little-endian
    words w_i (the last zero-padded) of splitmix64(w_i + i * 0x9E3779B97F4A7C15)."""
    b = np.ascontiguousarray(a).reshape(-1).view(np.uint8)
    pad = (-len(b)) % 8
    if pad:
        b = np.concatenate([b, np.zeros(pad, np.uint8)])
    w = b.view("<u8")
    with np.errstate(over="ignore"):
        z = w + np.arange(len(w), dtype=np.uint64) * _GOLD
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
        return int(z.sum(dtype=np.uint64))


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

    def checksum(self, row_lo=0, row_hi=None, stream=None):
        """drm_device_checksum of rows [row_lo, row_hi) (first axis); equals host_checksum of the same rows."""
        row = self.nbytes // self.shape[0] if self.shape and self.shape[0] else 0
        row_hi = self.shape[0] if row_hi is None else row_hi
        out = C.c_uint64(0)
        check(lib().drm_device_checksum(C.c_void_p(self.ptr + row_lo * row), C.c_int64((row_hi - row_lo) * row),
                                        C.byref(out), stream.handle if stream is not None else None))
        return int(out.value)

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
