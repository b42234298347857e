"""Diagnostic: wall time of consecutive drm_search_rerank calls at C3 in one process (first call pays
lazy code-object loading and buffer setup), next to the device span the executor reports."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from deepreadmapper_amd import synth, read_index, WindowTable  # noqa: E402
from deepreadmapper_amd.executor import search_rerank  # noqa: E402

w = synth.Workload("c3", 500_149, 100_000, seed=42, read_seed=7).generate("/tmp/drm_bench_cache")
t0 = time.time()
ix, table = read_index(w.index_path), WindowTable(w.refs)
print(f"load {time.time() - t0:.3f}s", flush=True)
for rep in range(4):
    t0 = time.perf_counter()
    o = search_rerank(ix, table, w.q_emb, w.queries, k=128, ef=128)
    print(f"call {rep}: wall {(time.perf_counter() - t0) * 1e3:.1f} ms, device {o['stats'].kernel_ms:.1f} ms", flush=True)
