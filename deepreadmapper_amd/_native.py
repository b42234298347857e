"""ctypes binding of libdrm_hip.so (include/drm_hip.h).

The library is built in-tree (`make` / `__graft_entry__.build()`). Importing this module without it
raises ImportError: there is no CPU fallback on the product path.
"""
import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# DRM_LIB selects another in-tree build of the same ABI (A/B timing of kernel variants)
LIB_PATH = os.environ.get("DRM_LIB") or os.path.join(_HERE, "libdrm_hip.so")

DRM_OK = 0
DRM_ERR_ARG = -1
DRM_ERR_IO = -2
DRM_ERR_FORMAT = -3
DRM_ERR_HIP = -4
DRM_ERR_CANDS = -5
DRM_ERR_K = -6
DRM_ERR_UNSUPPORTED = -7
DRM_ERR_INTERNAL = -8

# Every symbol include/drm_hip.h declares (checked by tests/test_capi_exports.py).
EXPORTS = [
    "drm_last_error", "drm_version", "drm_device_count", "drm_set_device", "drm_device_sync", "drm_malloc",
    "drm_free", "drm_memset", "drm_device_checksum", "drm_device_get_props", "drm_memcpy_h2d", "drm_memcpy_d2h", "drm_stream_create", "drm_stream_destroy",
    "drm_stream_sync", "drm_event_create", "drm_event_destroy", "drm_event_record", "drm_stream_wait_event", "drm_event_elapsed_ms",
    "drm_index_load", "drm_index_free", "drm_index_get_info", "drm_search", "drm_search_device",
    "drm_search_device_ex", "drm_index_search_errors", "drm_sw_scores",
    "drm_refs_create", "drm_refs_free", "drm_post_process_sw_static", "drm_post_process_sw_static_device",
    "drm_build_hnswpq", "drm_build_hnsw_flat", "drm_embed_kmer3", "drm_build_hnswpq_device",
    "drm_embed_kmer3_device",
    "drm_flat_index_load", "drm_flat_index_free", "drm_flat_index_get_info", "drm_flat_search",
    "drm_flat_search_device", "drm_flat_search_overflows", "drm_flat_search_errors",
    "drm_refs_get_info", "drm_host_alloc", "drm_host_free", "drm_search_rerank", "drm_multi_create",
    "drm_multi_free", "drm_multi_get_index_info", "drm_multi_search_rerank", "drm_comm_unique_id", "drm_comm_init",
    "drm_comm_free", "drm_comm_gather_rows", "drm_refs_create_genome", "drm_refs_is_genome",
    "drm_refs_set_sw_band", "drm_refs_get_sw_band",
    "drm_extract_fasta_sequence", "drm_post_process_sw_dynamic", "drm_post_process_sw_dynamic_device",
    "drm_multi_create_genome", "drm_search_rerank_prepare",
    "drm_encoder_load", "drm_encoder_export", "drm_encoder_free", "drm_encoder_get_info", "drm_tokenize",
    "drm_vectorize", "drm_vectorize_device", "drm_encoder_flags",
    "drm_refs_embed", "drm_refs_embeddings", "drm_post_process_l2_static", "drm_post_process_l2_static_device",
    "drm_post_process_l2_dynamic", "drm_post_process_l2_dynamic_device",
    "drm_index_set_search_waves", "drm_search_rerank_device",
    "drm_index_set_exact_stats", "drm_index_broadcast", "drm_index_clone", "drm_device_chase_latency", "drm_device_chase_rows",
]


class DrmError(RuntimeError):
    """Raised for a non-zero return code; `.code` is the DRM_ERR_* value."""

    def __init__(self, code, msg):
        super().__init__(msg)
        self.code = code


class IndexInfo(C.Structure):
    _fields_ = [("d", C.c_int32), ("ntotal", C.c_int64), ("pq_M", C.c_int32), ("pq_nbits", C.c_int32),
                ("M_hnsw", C.c_int32), ("max_level", C.c_int32), ("entry_point", C.c_int32),
                ("efConstruction", C.c_int32), ("efSearch", C.c_int32), ("metric_type", C.c_int32),
                ("device_bytes", C.c_int64), ("device", C.c_int32)]


class FlatIndexInfo(C.Structure):
    _fields_ = [("d", C.c_int32), ("ntotal", C.c_int64), ("M", C.c_int32), ("maxM0", C.c_int32),
                ("maxM", C.c_int32), ("max_level", C.c_int32), ("entry_point", C.c_uint32),
                ("efConstruction", C.c_int32), ("device_bytes", C.c_int64)]


class EncoderInfo(C.Structure):
    _fields_ = [("hidden", C.c_int32), ("emb_dim", C.c_int32), ("max_len", C.c_int32), ("out_dim", C.c_int32),
                ("n_token_rows", C.c_int32), ("device", C.c_int32), ("h0", C.c_float), ("device_bytes", C.c_int64)]


class PipelineStats(C.Structure):
    _fields_ = [("nq", C.c_int64), ("n_batches", C.c_int32), ("kernel_ms", C.c_double), ("search_ms", C.c_double),
                ("sw_ms", C.c_double), ("first_search_ms", C.c_double), ("last_sw_ms", C.c_double)]


class SearchStats(C.Structure):
    _fields_ = [("nq", C.c_int64), ("ndis", C.c_int64), ("nhops", C.c_int64), ("kernel_ms", C.c_double)]


_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: build it with `make` (or __graft_entry__.build()); "
                          "deepreadmapper_amd has no CPU fallback")
    L = C.CDLL(LIB_PATH)
    vp, i32, i64, sz = C.c_void_p, C.c_int32, C.c_int64, C.c_size_t
    sigs = {
        "drm_last_error": (C.c_char_p, []),
        "drm_version": (C.c_int, []),
        "drm_device_count": (C.c_int, [C.POINTER(C.c_int)]),
        "drm_set_device": (C.c_int, [C.c_int]),
        "drm_device_sync": (C.c_int, []),
        "drm_malloc": (C.c_int, [C.POINTER(vp), sz]),
        "drm_free": (C.c_int, [vp]),
        "drm_memset": (C.c_int, [vp, C.c_int, sz]),
        "drm_device_checksum": (C.c_int, [vp, C.c_int64, C.POINTER(C.c_uint64), vp]),
        "drm_device_get_props": (C.c_int, [C.c_int, vp]),
        "drm_memcpy_h2d": (C.c_int, [vp, vp, sz]),
        "drm_memcpy_d2h": (C.c_int, [vp, vp, sz]),
        "drm_stream_create": (C.c_int, [C.POINTER(vp)]),
        "drm_stream_destroy": (C.c_int, [vp]),
        "drm_stream_sync": (C.c_int, [vp]),
        "drm_event_create": (C.c_int, [C.POINTER(vp)]),
        "drm_event_destroy": (C.c_int, [vp]),
        "drm_event_record": (C.c_int, [vp, vp]),
        "drm_stream_wait_event": (C.c_int, [vp, vp]),
        "drm_event_elapsed_ms": (C.c_int, [vp, vp, C.POINTER(C.c_float)]),
        "drm_index_load": (C.c_int, [C.c_char_p, C.c_int, C.POINTER(vp)]),
        "drm_index_free": (C.c_int, [vp]),
        "drm_index_get_info": (C.c_int, [vp, C.POINTER(IndexInfo)]),
        "drm_index_set_search_waves": (C.c_int, [vp, i32]),
        "drm_index_set_exact_stats": (C.c_int, [vp, i32]),
        "drm_search_rerank_device": (C.c_int, [vp, vp, vp, i64, i32, i32, vp, vp, i32, i64, i32, vp, vp, vp, vp, vp,
                                               vp, vp, vp, vp, C.POINTER(PipelineStats)]),
        "drm_search": (C.c_int, [vp, vp, i64, i32, i32, i32, vp, vp, C.POINTER(SearchStats)]),
        "drm_search_device": (C.c_int, [vp, vp, i64, i32, i32, vp, vp, vp, vp, vp]),
        "drm_search_device_ex": (C.c_int, [vp, vp, i64, i32, i32, vp, vp, vp, vp, vp, vp]),
        "drm_index_search_errors": (C.c_int, [vp, C.POINTER(i64)]),
        "drm_sw_scores": (C.c_int, [vp, vp, vp, vp, vp, vp, i64, vp]),
        "drm_refs_create": (C.c_int, [vp, i64, i32, i64, C.c_int, C.POINTER(vp)]),
        "drm_refs_free": (C.c_int, [vp]),
        "drm_post_process_sw_static": (C.c_int, [vp, vp, i64, i32, vp, vp, i32, i64, i32, i32, vp, vp, vp,
                                                 C.POINTER(i64)]),
        "drm_post_process_sw_static_device": (C.c_int, [vp, vp, i64, i32, vp, vp, i32, i64, i32, i32, vp, vp, vp,
                                                        vp]),
        "drm_build_hnswpq": (C.c_int, [vp, i64, i32, i32, i32, i32, i32, C.c_double, i32, C.c_uint64,
                                       C.c_char_p]),
        "drm_flat_index_load": (C.c_int, [C.c_char_p, C.c_int, C.POINTER(vp)]),
        "drm_flat_index_free": (C.c_int, [vp]),
        "drm_flat_index_get_info": (C.c_int, [vp, C.POINTER(FlatIndexInfo)]),
        "drm_flat_search": (C.c_int, [vp, vp, i64, i32, i32, i32, vp, vp, C.POINTER(SearchStats)]),
        "drm_flat_search_device": (C.c_int, [vp, vp, i64, i32, i32, vp, vp, vp, vp, vp, vp]),
        "drm_flat_search_overflows": (C.c_int, [vp, C.POINTER(i64)]),
        "drm_flat_search_errors": (C.c_int, [vp, C.POINTER(i64)]),
        "drm_build_hnsw_flat": (C.c_int, [vp, i64, i32, i32, i32, i32, C.c_uint64, C.c_char_p]),
        "drm_embed_kmer3": (C.c_int, [vp, vp, vp, i64, i32, C.c_uint64, vp]),
        "drm_build_hnswpq_device": (C.c_int, [vp, i64, i32, i32, i32, i32, i32, C.c_double, C.c_uint64, C.c_int,
                                              C.c_char_p]),
        "drm_embed_kmer3_device": (C.c_int, [vp, i64, i32, i64, i32, C.c_uint64, vp, vp]),
        "drm_refs_get_info": (C.c_int, [vp, C.POINTER(i64), C.POINTER(i32), C.POINTER(C.c_int)]),
        "drm_host_alloc": (C.c_int, [C.POINTER(vp), sz]),
        "drm_host_free": (C.c_int, [vp]),
        "drm_search_rerank": (C.c_int, [vp, vp, vp, i64, i32, i32, i32, vp, vp, i32, i64, i32, vp, vp, vp, vp, vp,
                                        C.POINTER(SearchStats)]),
        "drm_multi_create": (C.c_int, [C.c_char_p, vp, C.c_int, vp, i64, i32, i64, C.POINTER(vp)]),
        "drm_multi_free": (C.c_int, [vp]),
        "drm_multi_get_index_info": (C.c_int, [vp, C.POINTER(IndexInfo)]),
        "drm_multi_search_rerank": (C.c_int, [vp, vp, i64, i32, i32, i32, vp, vp, i32, i64, i32, vp, vp, vp, vp,
                                              vp, C.POINTER(SearchStats)]),
        "drm_comm_unique_id": (C.c_int, [vp]),
        "drm_comm_init": (C.c_int, [vp, C.c_int, C.c_int, C.c_int, C.POINTER(vp)]),
        "drm_comm_free": (C.c_int, [vp]),
        "drm_comm_gather_rows": (C.c_int, [vp, vp, i64, i64, vp, C.c_int, vp]),
        "drm_index_broadcast": (C.c_int, [vp, vp, C.c_int, C.POINTER(vp)]),
        "drm_index_clone": (C.c_int, [vp, C.c_int, C.POINTER(vp)]),
        "drm_device_chase_latency": (C.c_int, [C.c_int, i64, C.c_int32, C.c_int32, C.POINTER(C.c_double)]),
        "drm_device_chase_rows": (C.c_int, [C.c_int, i64, C.c_int32, C.c_int32, C.c_int32, C.POINTER(C.c_double)]),
        "drm_refs_create_genome": (C.c_int, [vp, i64, i32, C.c_int, C.POINTER(vp)]),
        "drm_refs_is_genome": (C.c_int, [vp, C.POINTER(C.c_int)]),
        "drm_refs_set_sw_band": (C.c_int, [vp, i32]),
        "drm_refs_get_sw_band": (C.c_int, [vp, C.POINTER(i32)]),
        "drm_multi_create_genome": (C.c_int, [C.c_char_p, vp, C.c_int, vp, i64, i32, C.POINTER(vp)]),
        "drm_search_rerank_prepare": (C.c_int, [vp, i64, i32, i32, i32, i32]),
        "drm_extract_fasta_sequence": (C.c_int, [C.c_char_p, vp, C.POINTER(i64)]),
        "drm_post_process_sw_dynamic": (C.c_int, [vp, vp, i64, i32, vp, vp, i32, i64, i32, i32, vp, vp, vp,
                                                  C.POINTER(i64)]),
        "drm_post_process_sw_dynamic_device": (C.c_int, [vp, vp, i64, i32, vp, vp, i32, i64, i32, i32, vp, vp, vp,
                                                         vp]),
        "drm_encoder_load": (C.c_int, [C.c_char_p, C.c_int, C.POINTER(vp)]),
        "drm_encoder_export": (C.c_int, [C.c_char_p, C.c_char_p]),
        "drm_encoder_free": (C.c_int, [vp]),
        "drm_encoder_get_info": (C.c_int, [vp, C.POINTER(EncoderInfo)]),
        "drm_tokenize": (C.c_int, [vp, vp, vp, i64, i64, vp]),
        "drm_vectorize": (C.c_int, [vp, vp, vp, i64, i64, vp, C.POINTER(i64)]),
        "drm_vectorize_device": (C.c_int, [vp, vp, vp, i64, i64, vp, vp]),
        "drm_encoder_flags": (C.c_int, [vp, C.POINTER(i64), C.POINTER(i64)]),
        "drm_refs_embed": (C.c_int, [vp, vp, vp]),
        "drm_refs_embeddings": (C.c_int, [vp, C.POINTER(vp), C.POINTER(i32)]),
        "drm_post_process_l2_static": (C.c_int, [vp, vp, i64, i32, vp, i32, i64, i32, vp, vp, vp, C.POINTER(i64)]),
        "drm_post_process_l2_static_device": (C.c_int, [vp, vp, i64, i32, vp, i32, i64, i32, vp, vp, vp, vp]),
        "drm_post_process_l2_dynamic": (C.c_int, [vp, vp, i64, i32, vp, i32, i64, i32, i32, vp, vp, vp,
                                                  C.POINTER(i64)]),
        "drm_post_process_l2_dynamic_device": (C.c_int, [vp, vp, i64, i32, vp, i32, i64, i32, i32, vp, vp, vp, vp]),
    }
    for name, (res, args) in sigs.items():
        f = getattr(L, name, None)
        if f is None:
            if os.environ.get("DRM_LIB"):  # an A/B build of an older ABI: bind what it has
                continue
            raise ImportError(f"{LIB_PATH} does not export {name}")
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def check(rc):
    if rc != DRM_OK:
        msg = lib().drm_last_error()
        raise DrmError(rc, msg.decode() if msg else f"error {rc}")
    return rc


def ptr(a):
    """Host pointer of a C-contiguous numpy array (None -> NULL)."""
    if a is None:
        return None
    if not a.flags["C_CONTIGUOUS"]:
        raise ValueError("array must be C-contiguous")
    return a.ctypes.data
