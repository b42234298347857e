"""HNSW-PQ search: the drop-in for `faiss_search` (includes/hnswpq/search.hpp:18-21,
src/hnswpq/search.cpp:6-56) and for the faiss::IndexHNSWPQ handle `pipeline` loads
(src/main.cpp:236-237)."""
import ctypes as C

import numpy as np

from ._native import IndexInfo, SearchStats, check, lib, ptr

EF_DEFAULT = 128  # Config::Search::EF (includes/utils/config.hpp:47)
K_DEFAULT = 128   # Config::Search::K  (includes/utils/config.hpp:48)
K_CLUSTERS_DEFAULT = 5  # Config::Search::K_CLUSTERS (:49)


class HnswPqIndex:
    """Device-resident faiss IndexHNSWPQ, loaded from the faiss on-disk file."""

    def __init__(self, path, device=0):
        h = C.c_void_p()
        check(lib().drm_index_load(str(path).encode(), int(device), C.byref(h)))
        self._adopt(h.value, device)

    def _adopt(self, handle, device):
        self._h = handle
        self.device = int(device)
        info = IndexInfo()
        check(lib().drm_index_get_info(self._h, C.byref(info)))
        self.info = info
        self.d = info.d
        self.ntotal = info.ntotal

    @classmethod
    def broadcast(cls, comm, index=None, root=0, copy=False):
        """drm_index_broadcast: collective over `comm` (executor.Comm). The root passes its loaded index and gets it
        back (or, with copy=True, a separate replica received through the same path); every other rank passes None
        and gets a new replica on the communicator's device, received over RCCL instead of parsed from the file."""
        h = C.c_void_p()
        want = comm.rank != root or copy
        check(lib().drm_index_broadcast(comm.handle, index.handle if index is not None else None, int(root),
                                        C.byref(h) if want else None))
        if not want:
            return index
        obj = cls.__new__(cls)
        obj._adopt(h.value, comm.device)
        return obj

    def clone(self, device=None):
        """drm_index_clone: a replica on `device` (default: this index's device), copied device to device."""
        device = self.device if device is None else int(device)
        h = C.c_void_p()
        check(lib().drm_index_clone(self.handle, device, C.byref(h)))
        obj = type(self).__new__(type(self))
        obj._adopt(h.value, device)
        return obj

    @property
    def handle(self):
        if not self._h:
            raise RuntimeError("index was freed")
        return self._h

    def search(self, x, k, ef=EF_DEFAULT):
        """faiss `index->hnsw.efSearch = ef; index->search(n, x, k, D, I)`. Returns D, I, stats."""
        x = np.ascontiguousarray(x, dtype=np.float32)
        if x.ndim != 2:
            raise ValueError("queries must be [n, d]")
        n, d = x.shape
        D = np.empty((n, k), dtype=np.float32)
        I = np.empty((n, k), dtype=np.int64)
        st = SearchStats()
        check(lib().drm_search(self.handle, ptr(x), n, d, int(k), int(ef), ptr(D), ptr(I), C.byref(st)))
        return D, I, st

    def search_device(self, d_x, n, k, ef, d_D, d_I, d_ndis=None, d_nhops=None, stream=None, d_nhops_upper=None):
        """Search on device buffers (DeviceBuffer), enqueued on `stream`."""
        check(lib().drm_search_device_ex(self.handle, d_x.ptr, int(n), int(k), int(ef), d_D.ptr, d_I.ptr,
                                         d_ndis.ptr if d_ndis is not None else None,
                                         d_nhops.ptr if d_nhops is not None else None,
                                         d_nhops_upper.ptr if d_nhops_upper is not None else None,
                                         stream.handle if stream is not None else None))

    def set_exact_stats(self, on=True):
        """ndis as faiss counts it (links never visited before), from a visited bitmap kept for the count; off
        (the default) the lean kernel reports the distances it computed. Results do not depend on it."""
        check(lib().drm_index_set_exact_stats(self.handle, 1 if on else 0))

    def search_errors(self):
        """drm_index_search_errors: queries past the hop bound / waves past the item bound since the last check
        (syncs, resets the count); drm_search itself fails with DRM_ERR_INTERNAL when it is non-zero."""
        import ctypes as C
        c = C.c_int64(0)
        check(lib().drm_index_search_errors(self.handle, C.byref(c)))
        return int(c.value)

    def free(self):
        if self._h:
            check(lib().drm_index_free(self._h))
            self._h = None

    def __del__(self):
        try:
            if getattr(self, "_h", None):
                lib().drm_index_free(self._h)
        except Exception:
            pass


def read_index(path, device=0):
    """faiss::read_index + dynamic_cast<IndexHNSWPQ*> (src/main.cpp:236-237)."""
    return HnswPqIndex(path, device)


def faiss_search(index, query_data, k=K_DEFAULT, ef=EF_DEFAULT):
    """Same contract as the reference's faiss_search: returns (neighbor ids, distances), each a list
    of n lists of k. Raises RuntimeError("Query data is empty") on empty input (search.cpp:16-19)."""
    if query_data is None or len(query_data) == 0:
        raise RuntimeError("Query data is empty")
    x = np.asarray(query_data, dtype=np.float32)
    D, I, _ = index.search(x, k, ef)
    return [list(map(int, r)) for r in I], [list(map(float, r)) for r in D]
