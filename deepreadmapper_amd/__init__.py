"""deepreadmapper_amd -- MI355X-native drop-in for DeepReadMapper's query hot path:
HNSW-PQ candidate search (faiss_search), fp32-L2 HNSW search on hnswlib indexes (search), and the
Smith-Waterman rerank (post_process_sw_static), implemented as HIP kernels for gfx950 behind the C
ABI in include/drm_hip.h."""
from ._native import DrmError, lib  # noqa: F401  (ImportError if libdrm_hip.so is missing)
from .search import HnswPqIndex, faiss_search, read_index  # noqa: F401
from .flat import HnswFlatIndex, load_flat_index  # noqa: F401  (fp32-L2 hnswlib backend)
from .rerank import (WindowTable, calc_sw_score, calc_sw_scores, post_process_sw_static,  # noqa: F401
                     rerank_arrays, sw_reranker, GenomeTable, extract_fasta_sequence, post_process_sw_dynamic,
                     rerank_dynamic_arrays, embed_windows, l2_rerank_arrays, post_process_l2_static,
                     l2_rerank_dynamic_arrays, post_process_l2_dynamic)

__version__ = "0.1.0"
from .executor import Comm, MultiIndex, search_rerank  # noqa: F401  (batch executor, multi-GPU, RCCL gather)
from .encoder import Encoder, Preprocessor, Vectorizer, export_encoder  # noqa: F401  (GRU read encoder)
