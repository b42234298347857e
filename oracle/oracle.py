"""ctypes bindings for the TEST-ONLY oracle libraries (oracle/liboracle.so, libstl_sort.so,
_ref/libdrm_ref.so). See oracle/drm_oracle.h for what each function restates."""
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_lib = None
_stl = None
_ref = None
_hl = None


def _p(a, t):
    return a.ctypes.data_as(C.POINTER(t))


def lib():
    global _lib
    if _lib is None:
        _lib = C.CDLL(os.path.join(_HERE, "liboracle.so"))
        _lib.oracle_calc_sw_score.restype = C.c_int
        _lib.oracle_calc_sw_score.argtypes = [C.c_char_p, C.c_int64, C.c_char_p, C.c_int64]
        _lib.oracle_partial_sort_desc.restype = None
        _lib.oracle_post_process_sw_static.restype = C.c_int64
        _lib.oracle_post_process_sw_dynamic.restype = C.c_int64
        _lib.oracle_calc_sw_score_banded.restype = C.c_int
        _lib.oracle_calc_sw_score_banded.argtypes = [C.c_char_p, C.c_int64, C.c_char_p, C.c_int64, C.c_int64]
        _lib.oracle_post_process_sw_static_banded.restype = C.c_int64
        _lib.oracle_post_process_sw_dynamic_banded.restype = C.c_int64
        _lib.oracle_hnswpq_search.restype = C.c_int
        _lib.oracle_pq_distance_table.restype = None
        _lib.oracle_calc_l2_dist.restype = C.c_float
        _lib.oracle_calc_l2_dist.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_int]
        _lib.oracle_partial_sort_asc_f32.restype = None
        _lib.oracle_post_process_l2_static.restype = C.c_int64
        _lib.oracle_post_process_l2_dynamic.restype = C.c_int64
    return _lib


def stl():
    global _stl
    if _stl is None:
        _stl = C.CDLL(os.path.join(_HERE, "libstl_sort.so"))
        _stl.stl_partial_sort_desc.restype = None
        _stl.stl_partial_sort_asc_f32.restype = None
    return _stl


def ref_available():
    return os.path.exists(os.path.join(_HERE, "_ref", "libdrm_ref.so"))


def ref():
    global _ref
    if _ref is None:
        _ref = C.CDLL(os.path.join(_HERE, "_ref", "libdrm_ref.so"))
        _ref.ref_calc_sw_score.restype = C.c_int
        _ref.ref_calc_sw_score.argtypes = [C.c_char_p, C.c_int64, C.c_char_p, C.c_int64]
        if hasattr(_ref, "ref_calc_l2_dist"):
            _ref.ref_calc_l2_dist.restype = C.c_float
            _ref.ref_calc_l2_dist.argtypes = [C.c_void_p, C.c_void_p, C.c_int64]
    return _ref


def calc_sw_score(a: bytes, b: bytes) -> int:
    return lib().oracle_calc_sw_score(a, len(a), b, len(b))


def calc_sw_score_banded(a: bytes, b: bytes, band: int) -> int:
    """Banded SW (opt-in, non-parity; drm_oracle.c oracle_calc_sw_score_banded): cells |i - j| <= band."""
    return lib().oracle_calc_sw_score_banded(a, len(a), b, len(b), band)


def ref_calc_sw_score(a: bytes, b: bytes) -> int:
    return ref().ref_calc_sw_score(a, len(a), b, len(b))


def partial_sort_desc(scores, k):
    scores = np.ascontiguousarray(scores, dtype=np.int32)
    idx = np.arange(len(scores), dtype=np.int64)
    lib().oracle_partial_sort_desc(_p(idx, C.c_int64), C.c_int64(len(scores)), C.c_int64(k), _p(scores, C.c_int32))
    return idx[:k]


def stl_partial_sort_desc(scores, k):
    scores = np.ascontiguousarray(scores, dtype=np.int32)
    idx = np.zeros(len(scores), dtype=np.int64)
    stl().stl_partial_sort_desc(_p(idx, C.c_int64), C.c_int64(len(scores)), C.c_int64(k), _p(scores, C.c_int32))
    return idx[:k]


def post_process_sw_static(neighbors, refs, ref_len, queries, q_len, stride, k, k_clusters, nthreads=0, band=0):
    """neighbors [nq, kk] int64; refs [n_ref, ref_stride] uint8; queries [nq, q_stride] uint8.
    band > 0: the banded SW score (opt-in, non-parity) instead of calc_sw_score."""
    neighbors = np.ascontiguousarray(neighbors, dtype=np.int64)
    refs = np.ascontiguousarray(refs, dtype=np.uint8)
    queries = np.ascontiguousarray(queries, dtype=np.uint8)
    q_len = np.ascontiguousarray(q_len, dtype=np.int32)
    nq, kk = neighbors.shape
    scores = np.zeros((nq, k), dtype=np.int32)
    ids = np.zeros((nq, k), dtype=np.uint64)
    counts = np.zeros(nq, dtype=np.int32)
    rc = lib().oracle_post_process_sw_static_banded(
        _p(neighbors, C.c_int64), C.c_int64(nq), C.c_int64(kk),
        _p(refs, C.c_uint8), C.c_int64(refs.shape[0]), C.c_int64(ref_len), C.c_int64(refs.shape[1]),
        _p(queries, C.c_uint8), _p(q_len, C.c_int32), C.c_int64(queries.shape[1]),
        C.c_int64(stride), C.c_int64(k), C.c_int64(k_clusters), C.c_int64(band), C.c_int(nthreads),
        _p(scores, C.c_int32), _p(ids, C.c_uint64), _p(counts, C.c_int32))
    return int(rc), scores, ids, counts


def post_process_sw_dynamic(neighbors, genome, ref_len, queries, q_len, stride, k, k_clusters, nthreads=0, band=0):
    """post_process_sw_dynamic: neighbors [nq, kk] int64; genome uint8 (extract_FASTA_sequence);
    queries [nq, q_stride] uint8."""
    neighbors = np.ascontiguousarray(neighbors, dtype=np.int64)
    genome = np.ascontiguousarray(genome, dtype=np.uint8)
    queries = np.ascontiguousarray(queries, dtype=np.uint8)
    q_len = np.ascontiguousarray(q_len, dtype=np.int32)
    nq, kk = neighbors.shape
    scores = np.zeros((nq, k), dtype=np.int32)
    ids = np.zeros((nq, k), dtype=np.uint64)
    counts = np.zeros(nq, dtype=np.int32)
    rc = lib().oracle_post_process_sw_dynamic_banded(
        _p(neighbors, C.c_int64), C.c_int64(nq), C.c_int64(kk), _p(genome, C.c_uint8), C.c_int64(genome.size),
        C.c_int64(ref_len), _p(queries, C.c_uint8), _p(q_len, C.c_int32), C.c_int64(queries.shape[1]),
        C.c_int64(stride), C.c_int64(k), C.c_int64(k_clusters), C.c_int64(band), C.c_int(nthreads),
        _p(scores, C.c_int32), _p(ids, C.c_uint64), _p(counts, C.c_int32))
    return int(rc), scores, ids, counts


class OracleIndex(C.Structure):
    _fields_ = [("d", C.c_int32), ("ntotal", C.c_int64), ("pq_M", C.c_int32), ("pq_nbits", C.c_int32),
                ("dsub", C.c_int32), ("ksub", C.c_int32), ("code_size", C.c_int32),
                ("centroids", C.c_void_p), ("codes", C.c_void_p), ("levels", C.c_void_p),
                ("offsets", C.c_void_p), ("neighbors", C.c_void_p), ("cum_nneighbor_per_level", C.c_void_p),
                ("n_cum", C.c_int32), ("entry_point", C.c_int32), ("max_level", C.c_int32)]


def make_index(fx):
    """fx: oracle.faiss_file.HnswPqFile. Keeps numpy arrays alive on the returned struct."""
    s = OracleIndex()
    keep = {
        "centroids": np.ascontiguousarray(fx.centroids, dtype=np.float32),
        "codes": np.ascontiguousarray(fx.codes, dtype=np.uint8),
        "levels": np.ascontiguousarray(fx.levels, dtype=np.int32),
        "offsets": np.ascontiguousarray(fx.offsets, dtype=np.uint64),
        "neighbors": np.ascontiguousarray(fx.neighbors, dtype=np.int32),
        "cum": np.ascontiguousarray(fx.cum_nneighbor_per_level, dtype=np.int32),
    }
    s.d = fx.d
    s.ntotal = fx.ntotal
    s.pq_M = fx.pq_M
    s.pq_nbits = fx.pq_nbits
    s.dsub = fx.d // fx.pq_M
    s.ksub = 1 << fx.pq_nbits
    s.code_size = (fx.pq_M * fx.pq_nbits + 7) // 8
    s.centroids = keep["centroids"].ctypes.data
    s.codes = keep["codes"].ctypes.data
    s.levels = keep["levels"].ctypes.data
    s.offsets = keep["offsets"].ctypes.data
    s.neighbors = keep["neighbors"].ctypes.data
    s.cum_nneighbor_per_level = keep["cum"].ctypes.data
    s.n_cum = len(keep["cum"])
    s.entry_point = fx.entry_point
    s.max_level = fx.max_level
    s._keep = keep
    return s


def hnswpq_search(fx_or_struct, x, k, ef, nthreads=0):
    s = fx_or_struct if isinstance(fx_or_struct, OracleIndex) else make_index(fx_or_struct)
    x = np.ascontiguousarray(x, dtype=np.float32)
    n = x.shape[0]
    D = np.empty((n, k), dtype=np.float32)
    I = np.empty((n, k), dtype=np.int64)
    ndis = np.empty(n, dtype=np.int32)
    nhops = np.empty(n, dtype=np.int32)
    rc = lib().oracle_hnswpq_search(C.byref(s), _p(x, C.c_float), C.c_int64(n), C.c_int(k), C.c_int(ef),
                                    _p(D, C.c_float), _p(I, C.c_int64), _p(ndis, C.c_int32), _p(nhops, C.c_int32),
                                    C.c_int(nthreads))
    if rc != 0:
        raise RuntimeError("oracle_hnswpq_search failed")
    return D, I, ndis, nhops


def pq_distance_table(fx_or_struct, x):
    s = fx_or_struct if isinstance(fx_or_struct, OracleIndex) else make_index(fx_or_struct)
    x = np.ascontiguousarray(x, dtype=np.float32)
    lut = np.empty(s.pq_M * s.ksub, dtype=np.float32)
    lib().oracle_pq_distance_table(C.byref(s), _p(x, C.c_float), _p(lut, C.c_float))
    return lut.reshape(s.pq_M, s.ksub)


def set_lut_order(order):
    """faiss LUT sum order variant of the oracle (drm_oracle.c oracle_set_lut_order); 0 = default."""
    lib().oracle_set_lut_order(C.c_int(int(order)))


def set_l2_order(order):
    """hnswlib L2 kernel variant of the oracle (hnswlib_oracle.cpp oracle_set_l2_order); 0 = default."""
    hnswlib_lib().oracle_set_l2_order(C.c_int(int(order)))


def hnswlib_lib():
    global _hl
    if _hl is None:
        _hl = C.CDLL(os.path.join(_HERE, "libhnswlib_oracle.so"))
        _hl.oracle_hnswlib_search.restype = C.c_int
        _hl.oracle_l2_avx.restype = C.c_float
        _hl.oracle_l2_avx.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
    return _hl


def l2_avx(x, y):
    x = np.ascontiguousarray(x, dtype=np.float32)
    y = np.ascontiguousarray(y, dtype=np.float32)
    return float(hnswlib_lib().oracle_l2_avx(x.ctypes.data, y.ctypes.data, int(x.size)))


def hnswlib_search(fx, q, k, ef, nthreads=0):
    """hnswlib searchKnnCloserFirst per query (src/hnswlib_dir/search.cpp:7-52) on a parsed index
    (oracle/hnswlib_file.read). Returns (D [n,k] f32, I [n,k] i64 labels, ndis, nhops)."""
    q = np.ascontiguousarray(q, dtype=np.float32)
    n = q.shape[0]
    D = np.empty((n, k), dtype=np.float32)
    I = np.empty((n, k), dtype=np.int64)
    nd = np.empty(n, dtype=np.int32)
    nh = np.empty(n, dtype=np.int32)
    vp = C.c_void_p
    rc = hnswlib_lib().oracle_hnswlib_search(
        C.c_int(fx["d"]), C.c_int64(fx["n"]), C.c_int(fx["maxM0"]), C.c_int(fx["maxM"]), C.c_int(fx["maxlevel"]),
        C.c_uint32(fx["ep"]), vp(fx["vec"].ctypes.data), vp(fx["l0"].ctypes.data), vp(fx["up_off"].ctypes.data),
        vp(fx["up"].ctypes.data), vp(fx["labels"].ctypes.data), vp(q.ctypes.data), C.c_int64(n), C.c_int(k),
        C.c_int(ef), vp(D.ctypes.data), vp(I.ctypes.data), vp(nd.ctypes.data), vp(nh.ctypes.data),
        C.c_int(nthreads))
    assert rc == 0
    return D, I, nd, nh


# ------------------------------------------------------------------ L2 rerank (post_process_l2_static)
def calc_l2_dist(cand, query, mode=2):
    """calc_l2_dist (src/utils/metrics.cpp:48-61) restated (drm_oracle.c): mode 2 = the reference's g++
    -O3 -march=native schedule (vector body: rounded squares added in order; scalar tail fused), 0 = no
    fusion (identical to 2 when d % 4 == 0, e.g. the model's d = 128), 1 = every element fused."""
    a = np.ascontiguousarray(cand, dtype=np.float32)
    b = np.ascontiguousarray(query, dtype=np.float32)
    return float(lib().oracle_calc_l2_dist(a.ctypes.data, b.ctypes.data, len(a), int(mode)))


def ref_calc_l2_dist(cand, query):
    """The reference's own calc_l2_dist (oracle/_ref, built with -mavx2 -mfma)."""
    a = np.ascontiguousarray(cand, dtype=np.float32)
    b = np.ascontiguousarray(query, dtype=np.float32)
    return float(ref().ref_calc_l2_dist(a.ctypes.data, b.ctypes.data, len(a)))


def partial_sort_asc_f32(dists, k):
    dists = np.ascontiguousarray(dists, dtype=np.float32)
    idx = np.arange(len(dists), dtype=np.int64)
    lib().oracle_partial_sort_asc_f32(_p(idx, C.c_int64), C.c_int64(len(dists)), C.c_int64(k), _p(dists, C.c_float))
    return idx[:k]


def stl_partial_sort_asc_f32(dists, k):
    dists = np.ascontiguousarray(dists, dtype=np.float32)
    idx = np.zeros(len(dists), dtype=np.int64)
    stl().stl_partial_sort_asc_f32(_p(idx, C.c_int64), C.c_int64(len(dists)), C.c_int64(k), _p(dists, C.c_float))
    return idx[:k]


def post_process_l2_static(emb, neighbors, query_emb, stride, k_clusters, mode=2):
    """post_process_l2_static -> batch_reranker(k = k_clusters) over window embeddings emb [n_ref, d].
    Returns (rc, dists [nq, k_clusters], ids [nq, k_clusters] u64, status [nq]); rc as the C oracle."""
    emb = np.ascontiguousarray(emb, dtype=np.float32)
    nb = np.ascontiguousarray(neighbors, dtype=np.int64)
    qe = np.ascontiguousarray(query_emb, dtype=np.float32)
    nq, kk = nb.shape
    dists = np.zeros((nq, k_clusters), dtype=np.float32)
    ids = np.zeros((nq, k_clusters), dtype=np.uint64)
    status = np.zeros(nq, dtype=np.int32)
    rc = lib().oracle_post_process_l2_static(
        _p(emb, C.c_float), C.c_int64(emb.shape[0]), C.c_int64(emb.shape[1]), _p(nb, C.c_int64), C.c_int64(nq),
        C.c_int64(kk), _p(qe, C.c_float), C.c_int64(stride), C.c_int64(k_clusters), C.c_int(int(mode)),
        _p(dists, C.c_float), _p(ids, C.c_uint64), _p(status, C.c_int32))
    return int(rc), dists, ids, status


def post_process_l2_dynamic(emb, neighbors, query_emb, stride, k, k_clusters, mode=2):
    """post_process_l2_dynamic(_streaming)'s stride > 1 rerank over the dynamic-lookup window embeddings
    emb [glen, d] (row w = window w). Returns (rc, dists [nq, k], ids [nq, k] u64, status [nq])."""
    emb = np.ascontiguousarray(emb, dtype=np.float32)
    nb = np.ascontiguousarray(neighbors, dtype=np.int64)
    qe = np.ascontiguousarray(query_emb, dtype=np.float32)
    nq, kk = nb.shape
    dists = np.zeros((nq, k), dtype=np.float32)
    ids = np.zeros((nq, k), dtype=np.uint64)
    status = np.zeros(nq, dtype=np.int32)
    rc = lib().oracle_post_process_l2_dynamic(
        _p(emb, C.c_float), C.c_int64(emb.shape[0]), C.c_int64(emb.shape[1]), _p(nb, C.c_int64), C.c_int64(nq),
        C.c_int64(kk), _p(qe, C.c_float), C.c_int64(stride), C.c_int64(k), C.c_int64(k_clusters),
        C.c_int(int(mode)), _p(dists, C.c_float), _p(ids, C.c_uint64), _p(status, C.c_int32))
    return int(rc), dists, ids, status
