"""Batch executor (csrc/exec.cpp): the fused search -> SW rerank pass of the reference's batch driver
(faiss_search then post_process_sw_static, src/main.cpp:278, :333-341), its multi-GPU fan-out
(replicated index, contiguous query shards) and the RCCL gather of device-resident
result rows across the ranks of a one-process-per-GPU job."""
import ctypes as C

import numpy as np

from ._native import IndexInfo, PipelineStats, SearchStats, check, lib, ptr


def _outputs(n, k_clusters, k, rerank):
    out = {"D": np.empty((n, k_clusters), dtype=np.float32), "I": np.empty((n, k_clusters), dtype=np.int64)}
    if rerank:
        out.update(sw_scores=np.empty((n, k), dtype=np.int32), sw_ids=np.empty((n, k), dtype=np.uint64),
                   status=np.empty(n, dtype=np.int32))
    return out


def _query_args(x, queries):
    x = np.ascontiguousarray(x, dtype=np.float32)
    if x.ndim != 2:
        raise ValueError("embeddings must be [n, d]")
    if queries is None:
        return x, None, None, 0
    if isinstance(queries, tuple):  # (qbuf [n, q_stride] u8, q_len [n] i32), e.g. rerank.pack_queries
        qbuf, ql = queries
    else:
        qbuf = np.ascontiguousarray(queries, dtype=np.uint8)
        ql = np.full(len(qbuf), qbuf.shape[1], dtype=np.int32)
    qbuf, ql = np.ascontiguousarray(qbuf, dtype=np.uint8), np.ascontiguousarray(ql, dtype=np.int32)
    if len(qbuf) != len(x) or len(ql) != len(x):
        raise ValueError("one query sequence per embedding")
    return x, qbuf, ql, qbuf.shape[1]


class _Pinned:
    def __init__(self, nbytes):
        p = C.c_void_p()
        check(lib().drm_host_alloc(C.byref(p), max(int(nbytes), 1)))
        self.ptr = p.value

    def __del__(self):
        try:
            lib().drm_host_free(self.ptr)
        except Exception:  # noqa: BLE001
            pass


def pinned_empty(shape, dtype):
    """A numpy array in pinned host memory (drm_host_alloc): the executor's copies to and from it are
    DMA transfers that overlap the kernels. The array keeps its allocation alive."""
    dtype = np.dtype(dtype)
    n = int(np.prod(shape, dtype=np.int64))
    buf = _Pinned(n * dtype.itemsize)
    raw = (C.c_uint8 * max(n * dtype.itemsize, 1)).from_address(buf.ptr)
    a = np.frombuffer(raw, dtype=np.uint8, count=n * dtype.itemsize).view(dtype).reshape(shape)
    _KEEP.append(buf)  # pinned buffers live as long as the process (the bench's few large arrays)
    return a


_KEEP = []


def prepare(index, n, d, k_clusters, k=0, q_stride=0):
    """drm_search_rerank_prepare: streams and device buffers for a batch of n queries, ahead of the call."""
    check(lib().drm_search_rerank_prepare(index.handle, int(n), int(d), int(k_clusters), int(k), int(q_stride)))


def search_rerank(index, table, x, queries=None, k=128, ef=128, k_clusters=None, stride=1, out=None):
    """drm_search_rerank: search (k_clusters results) then, when `table` (WindowTable) and `queries`
    are given, the SW rerank to k. Returns a dict of D, I (+ sw_scores, sw_ids, status) and stats."""
    kc = k if k_clusters is None else k_clusters
    x, qbuf, ql, qs = _query_args(x, queries)
    rr = table is not None and qbuf is not None
    o = out if out is not None else _outputs(len(x), kc, k, rr)
    st = SearchStats()
    check(lib().drm_search_rerank(index.handle, table.handle if rr else None, ptr(x), len(x), x.shape[1], int(kc),
                                  int(ef), ptr(qbuf) if rr else None, ptr(ql) if rr else None, qs, int(stride),
                                  int(k), ptr(o["D"]), ptr(o["I"]), ptr(o.get("sw_scores")), ptr(o.get("sw_ids")),
                                  ptr(o.get("status")), C.byref(st)))
    o["stats"] = st
    return o


def search_rerank_device(index, table, d_x, n, d_queries, d_q_len, q_stride, d_D, d_I, d_sw_scores, d_sw_ids,
                         d_status, k=128, ef=128, k_clusters=None, stride=1, d_ndis=None, d_nhops=None,
                         d_nhops_upper=None, stream=None, stats=False):
    """drm_search_rerank_device: search, then SW rerank, on DeviceBuffers (the caller's stream). stats=True
    synchronises and returns the PipelineStats."""
    kc = k if k_clusters is None else k_clusters
    st = PipelineStats() if stats else None
    p = lambda b: b.ptr if b is not None else None  # noqa: E731
    check(lib().drm_search_rerank_device(index.handle, table.handle, d_x.ptr, int(n), int(kc), int(ef), d_queries.ptr,
                                         d_q_len.ptr, int(q_stride), int(stride), int(k), d_D.ptr, d_I.ptr, p(d_ndis),
                                         p(d_nhops), p(d_nhops_upper), d_sw_scores.ptr, d_sw_ids.ptr, d_status.ptr,
                                         stream.handle if stream is not None else None,
                                         C.byref(st) if st is not None else None))
    return st


class MultiIndex:
    """drm_multi: one IndexHNSWPQ replica (+ window table) per entry of `devices` (repeats allowed)."""

    def __init__(self, path, devices, windows=None, genome=None, ref_len=150):
        devs = np.ascontiguousarray(devices, dtype=np.int32)
        h = C.c_void_p()
        if genome is not None:  # dynamic lookup (use_dynamic)
            g = np.frombuffer(genome, dtype=np.uint8) if isinstance(genome, (bytes, bytearray)) else \
                np.ascontiguousarray(genome, dtype=np.uint8)
            check(lib().drm_multi_create_genome(str(path).encode(), ptr(devs), len(devs), ptr(g), g.size, int(ref_len),
                                                C.byref(h)))
        elif windows is not None:
            w = np.ascontiguousarray(windows, dtype=np.uint8)
            check(lib().drm_multi_create(str(path).encode(), ptr(devs), len(devs), ptr(w), w.shape[0], w.shape[1],
                                         w.shape[1], C.byref(h)))
        else:
            check(lib().drm_multi_create(str(path).encode(), ptr(devs), len(devs), None, 0, 0, 0, C.byref(h)))
        self._h = h.value
        self.devices = list(devs)
        self.has_refs = windows is not None or genome is not None
        info = IndexInfo()
        check(lib().drm_multi_get_index_info(self._h, C.byref(info)))
        self.info = info

    def search_rerank(self, x, queries=None, k=128, ef=128, k_clusters=None, stride=1):
        kc = k if k_clusters is None else k_clusters
        x, qbuf, ql, qs = _query_args(x, queries)
        rr = self.has_refs and qbuf is not None
        o = _outputs(len(x), kc, k, rr)
        st = SearchStats()
        check(lib().drm_multi_search_rerank(self._h, ptr(x), len(x), x.shape[1], int(kc), int(ef),
                                            ptr(qbuf) if rr else None, ptr(ql) if rr else None, qs, int(stride),
                                            int(k), ptr(o["D"]), ptr(o["I"]), ptr(o.get("sw_scores")),
                                            ptr(o.get("sw_ids")), ptr(o.get("status")), C.byref(st)))
        o["stats"] = st
        return o

    def free(self):
        if self._h:
            check(lib().drm_multi_free(self._h))
            self._h = None

    def __del__(self):
        try:
            self.free()
        except Exception:  # noqa: BLE001 -- interpreter shutdown
            pass


class Comm:
    """drm_comm: RCCL communicator of a one-process-per-GPU job. Rank 0 makes the id (unique_id()); the
    job hands it to every rank out of band (bench.py: torch.distributed gloo broadcast)."""

    ID_BYTES = 128

    @staticmethod
    def unique_id():
        buf = (C.c_uint8 * Comm.ID_BYTES)()
        check(lib().drm_comm_unique_id(buf))
        return bytes(buf)

    def __init__(self, uid, nranks, rank, device):
        if len(uid) != Comm.ID_BYTES:
            raise ValueError("RCCL unique id must be 128 bytes")
        buf = (C.c_uint8 * Comm.ID_BYTES).from_buffer_copy(uid)
        h = C.c_void_p()
        check(lib().drm_comm_init(buf, int(nranks), int(rank), int(device), C.byref(h)))
        self._h = h.value
        self.nranks, self.rank, self.device = int(nranks), int(rank), int(device)

    @property
    def handle(self):
        if not self._h:
            raise RuntimeError("communicator was freed")
        return self._h

    def gather_rows(self, d_send, n_total, row_bytes, d_recv=None, root=0, stream=None):
        """Rows [r*n/G, (r+1)*n/G) of every rank's d_send (DeviceBuffer) land in the root's d_recv."""
        check(lib().drm_comm_gather_rows(self._h, d_send.ptr, int(n_total), int(row_bytes),
                                         d_recv.ptr if d_recv is not None else None, int(root),
                                         stream.handle if stream is not None else None))

    def free(self):
        if self._h:
            check(lib().drm_comm_free(self._h))
            self._h = None

    def __del__(self):
        try:
            self.free()
        except Exception:  # noqa: BLE001
            pass
