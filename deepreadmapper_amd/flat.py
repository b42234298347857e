"""fp32-L2 HNSW search on hnswlib index files: the drop-in for the reference's hnswlib backend --
`new hnswlib::HierarchicalNSW<float>(&space, index_file)` (src/hnswlib_dir/test_search.cpp:33) and
`search(index, query_data, k, ef)` (src/hnswlib_dir/search.cpp:7-52, includes/hnswlib_dir/search.hpp)."""
import ctypes as C

import numpy as np

from ._native import FlatIndexInfo, SearchStats, check, lib, ptr

EF_DEFAULT = 128  # Config::Search::EF (includes/utils/config.hpp:46)
K_DEFAULT = 128   # Config::Search::K  (includes/utils/config.hpp:47)


class HnswFlatIndex:
    """Device-resident hnswlib HierarchicalNSW<float> (vectors, level-0 rows, upper links, labels)."""

    def __init__(self, path, device=0):
        h = C.c_void_p()
        check(lib().drm_flat_index_load(str(path).encode(), int(device), C.byref(h)))
        self._h = h.value
        self.device = int(device)
        info = FlatIndexInfo()
        check(lib().drm_flat_index_get_info(self._h, C.byref(info)))
        self.info = info
        self.d = info.d
        self.ntotal = info.ntotal

    @property
    def handle(self):
        if not self._h:
            raise RuntimeError("index was freed")
        return self._h

    def search(self, x, k, ef=EF_DEFAULT):
        """setEf(ef) + searchKnnCloserFirst(q, k) per row of x. Returns D [n,k] f32 (squared L2,
        ascending), labels [n,k] u64 (padding 2^64-1), stats."""
        x = np.ascontiguousarray(x, dtype=np.float32)
        if x.ndim != 2:
            raise ValueError("queries must be [n, d]")
        n, d = x.shape
        D = np.empty((n, k), dtype=np.float32)
        L = np.empty((n, k), dtype=np.uint64)
        st = SearchStats()
        check(lib().drm_flat_search(self.handle, ptr(x), n, d, int(k), int(ef), ptr(D), ptr(L), C.byref(st)))
        return D, L, st

    def search_device(self, d_x, n, k, ef, d_D, d_L, d_ndis, d_nhops, stream=None, d_nhops_upper=None):
        """Search on device buffers (DeviceBuffer), enqueued on `stream`."""
        check(lib().drm_flat_search_device(self.handle, d_x.ptr, int(n), int(k), int(ef), d_D.ptr, d_L.ptr,
                                           d_ndis.ptr, d_nhops.ptr,
                                           d_nhops_upper.ptr if d_nhops_upper is not None else None,
                                           stream.handle if stream is not None else None))

    def overflows(self):
        c = C.c_int64(0)
        check(lib().drm_flat_search_overflows(self.handle, C.byref(c)))
        return int(c.value)

    def search_errors(self):
        """drm_flat_search_errors: queries past the hop bound / waves past the item bound (syncs, resets)."""
        c = C.c_int64(0)
        check(lib().drm_flat_search_errors(self.handle, C.byref(c)))
        return int(c.value)

    def free(self):
        if self._h:
            check(lib().drm_flat_index_free(self._h))
            self._h = None

    def __del__(self):
        try:
            if getattr(self, "_h", None):
                lib().drm_flat_index_free(self._h)
        except Exception:
            pass


def load_flat_index(path, device=0):
    """new hnswlib::HierarchicalNSW<float>(&space, index_file) (src/hnswlib_dir/test_search.cpp:33)."""
    return HnswFlatIndex(path, device)


def search(index, query_data, k=K_DEFAULT, ef=EF_DEFAULT):
    """Same contract as the reference's hnswlib search(): (labels, distances), each a list of n lists,
    closest first. Raises RuntimeError("Query data is empty") on empty input (search.cpp:20-23)."""
    if query_data is None or len(query_data) == 0:
        raise RuntimeError("Query data is empty")
    D, L, _ = index.search(np.asarray(query_data, dtype=np.float32), k, ef)
    labels, dists = [], []
    for i in range(D.shape[0]):
        m = L[i] != np.uint64(2 ** 64 - 1)
        labels.append(L[i][m].tolist())
        dists.append(D[i][m].tolist())
    return labels, dists
