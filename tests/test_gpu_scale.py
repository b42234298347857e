"""GPU parity at the BASELINE.json configurations, not just the fixtures:

* C3 -- synthetic 1M x 150 bp dense windows, 100k reads: the live-path IndexHNSWPQ (M_hnsw 16,
  EFC 200, PQ 8x8) and the hnswlib fp32 index (M 64, EFC 128), both built here on the box.
* C4 -- BASELINE configs[3] at its configured size: a seeded 20,000,299 bp genome, stride-4 sparse
  IndexHNSWPQ of 10,000,000 windows (PQ 8x8, M_hnsw 16, EFC 200) built on the GPU (builder_gpu.hip,
  seconds), 1,000,000 reads, K = 128 and the reference's sparse default k_clusters = K = 5
  (src/main.cpp:56-63,278), and the sparse SW rerank (post_process_sw_static at stride 4).

On each: the HIP search + SW rerank on a fixed query sample equal the oracle bit for bit (ids,
0-ulp distances, ndis / nhops, SW scores and their partial_sort order), and every query of the
full batch passes the size-independent checks (ascending rows, status == K, sample rows identical
inside the full batch, per-query ndis / nhops equal to the oracle's on the sample).
Reference call sites: src/main.cpp:278 (faiss_search), src/hnswpq/search.cpp:13,39-40,
src/utils/post_processor.cpp:454-549 (post_process_sw_static)."""
import os

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

CACHE = os.environ.get("DRM_TEST_CACHE", "/tmp/drm_test_cache")
NSAMPLE = 2000


def _threads():
    return max(1, min(16, len(os.sched_getaffinity(0))))


@pytest.fixture(scope="module")
def c3():
    from deepreadmapper_amd import synth
    from oracle import faiss_file
    w = synth.Workload("c3", 500_149, 100_000, seed=42, read_seed=7).generate(CACHE, nthreads=_threads())
    return {"w": w, "fx": faiss_file.read(w.index_path)}


@pytest.fixture(scope="module")
def c4():
    from deepreadmapper_amd import synth
    from oracle import faiss_file
    w = synth.Workload("c4", 20_000_299, 1_000_000, stride=4, seed=43, read_seed=8).generate(
        CACHE, need_refs=False, gpu_build=True)
    fx = faiss_file.read(w.index_path)
    assert fx.ntotal == 2 * ((20_000_299 - 150) // 4 + 1)  # 10,000,076 fwd/RC windows at stride 4
    return {"w": w, "fx": fx}


def _sample(n):
    return np.linspace(0, n - 1, NSAMPLE).astype(np.int64)


def _search_full(index_path, q, k, ef):
    """All queries through the device entry point (one launch), with per-query ndis / nhops."""
    from deepreadmapper_amd import read_index
    from deepreadmapper_amd.device import DeviceBuffer, synchronize
    n = len(q)
    ix = read_index(index_path)
    dq = DeviceBuffer.from_host(np.ascontiguousarray(q))
    dD, dI = DeviceBuffer((n, k), np.float32), DeviceBuffer((n, k), np.int64)
    nd, nh = DeviceBuffer(n, np.int32), DeviceBuffer(n, np.int32)
    ix.search_device(dq, n, k, ef, dD, dI, nd, nh)
    synchronize()
    out = dD.download(), dI.download(), nd.download(), nh.download()
    ix.free()
    return out


def _check_search(index_path, fx, q, k, ef, ntotal):
    D, I, nd, nh = _search_full(index_path, q, k, ef)
    # size-independent properties on every query
    assert np.all(np.diff(D, axis=1) >= 0), "rows must be ascending"
    assert (I[:, 0] >= 0).all() and (I < ntotal).all()
    assert np.all(nd > 0) and np.all(nh > 0)
    # bit-exact on the sample
    s = _sample(len(q))
    Do, Io, ndo, nho = O.hnswpq_search(fx, q[s], k, ef, nthreads=_threads())
    assert np.array_equal(I[s], Io)
    assert np.array_equal(D[s].view(np.uint32), Do.view(np.uint32))  # 0 ulp
    assert np.array_equal(nh[s], nho)
    # the same queries searched alone give the same rows as inside the full batch, and with exact statistics
    # the same rows plus faiss's ndis
    from deepreadmapper_amd import read_index
    ix = read_index(index_path)
    D2, I2, _ = ix.search(q[s[:256]], k, ef)
    ix.set_exact_stats(True)
    D3, I3, st3 = ix.search(q[s[:256]], k, ef)
    ix.free()
    assert np.array_equal(I2, I[s[:256]]) and np.array_equal(D2.view(np.uint32), D[s[:256]].view(np.uint32))
    assert np.array_equal(I3, I2) and np.array_equal(D3.view(np.uint32), D2.view(np.uint32))
    assert st3.ndis == int(ndo[:256].sum()) and st3.nhops == int(nho[:256].sum())
    return D, I


def _check_rerank(refs, I, queries, stride, k, kc):
    from deepreadmapper_amd import WindowTable, rerank_arrays
    s = _sample(len(I))
    table = WindowTable(refs)
    ql = np.full(len(I), queries.shape[1], dtype=np.int32)
    sc, ids, cnt = rerank_arrays(table, I, (queries, ql), stride, k, kc)
    assert (cnt == k).all()
    assert np.all(np.diff(sc, axis=1) <= 0), "SW scores must be descending"
    rc, sc_o, id_o, cnt_o = O.post_process_sw_static(I[s], refs, refs.shape[1], queries[s], ql[s], stride, k, kc,
                                                     nthreads=_threads())
    assert rc == 0 and np.array_equal(cnt_o, cnt[s])
    assert np.array_equal(sc[s], sc_o) and np.array_equal(ids[s], id_o)
    table.free()


def test_c3_pq_search_and_rerank_k128(c3):
    w = c3["w"]
    D, I = _check_search(w.index_path, c3["fx"], w.q_emb, 128, 128, len(w.refs))
    _check_rerank(w.refs, I, w.queries, 1, 128, 128)


def test_c3_pq_search_exact_kernel(c3, monkeypatch):
    """The general exact kernel (DRM_SEARCH_FAST=0) on the same C3 sample."""
    monkeypatch.setenv("DRM_SEARCH_FAST", "0")
    w = c3["w"]
    q = w.q_emb[_sample(len(w.q_emb))]
    _check_search(w.index_path, c3["fx"], q, 128, 128, len(w.refs))


def test_c3_flat_search_sample(c3):
    """The hnswlib fp32 index at the reference's defaults (M 64, EFC 128) over the C3 windows."""
    from deepreadmapper_amd import synth, HnswFlatIndex
    from oracle import hnswlib_file
    w = c3["w"]
    path = os.path.join(CACHE, "c3_flat_M64_efc128.hnsw")
    if not os.path.exists(path):
        synth.build_flat_index(synth.embed(synth.tag(w.refs)), path + ".tmp", M=64, efc=128, nthreads=_threads())
        os.replace(path + ".tmp", path)
    fx = hnswlib_file.read(path)
    s = _sample(len(w.q_emb))
    ix = HnswFlatIndex(path)
    D, L, st = ix.search(w.q_emb[s], 128, 128)
    assert ix.overflows() == 0
    ix.free()
    Do, Io, nd, nh = O.hnswlib_search(fx, w.q_emb[s], 128, 128, nthreads=_threads())
    assert np.array_equal(L.astype(np.int64), Io)
    assert np.array_equal(D.view(np.uint32), Do.view(np.uint32))
    assert st.ndis == int(nd.sum()) and st.nhops == int(nh.sum())


@pytest.mark.parametrize("k", [128, 5])
def test_c4_sparse_pq_search(c4, k):
    """All 1M C4 queries through the device search (property checks), a 2,000-query sample bit-exact
    against the oracle (ids, 0-ulp distances, ndis, nhops); src/hnswpq/index.cpp:215,270 (stride 4),
    src/main.cpp:278 (search k = k_clusters)."""
    w = c4["w"]
    _check_search(w.index_path, c4["fx"], w.q_emb, k, 128, c4["fx"].ntotal)


def test_c4_sparse_rerank(c4):
    """post_process_sw_static on the stride-4 10M-window index over the stride-1 window table of the same
    genome (src/utils/post_processor.cpp:238-335): the reference's sparse defaults (k_clusters = 5, K = 5)
    and K = 128 over k_clusters = 20 (K <= k_clusters * 2 * stride, post_processor.cpp:486-489, and 20 ids
    expand to up to 140 >= K windows, reranker.cpp:26-29), 20,000 reads, a 2,000-read sample against the
    oracle."""
    from deepreadmapper_amd import synth
    w = c4["w"]
    refs = synth.windows_lookup(w.genome, 150, 1)
    assert len(refs) == 2 * (20_000_299 - 149)
    for k, kc in ((5, 5), (128, 20)):
        _, I, _, _ = _search_full(w.index_path, w.q_emb[:20_000], kc, 128)
        _check_rerank(refs, I, w.queries[:20_000], 4, k, kc)


def test_c3_device_pipeline(c3):
    """drm_search_rerank_device (the search, then the SW rerank, on device buffers) gives byte-identical outputs to
    drm_search_device + drm_post_process_sw_static_device over the whole C3 batch (100k reads)."""
    from deepreadmapper_amd import read_index, WindowTable
    from deepreadmapper_amd.device import DeviceBuffer, synchronize
    from deepreadmapper_amd.executor import search_rerank_device
    from deepreadmapper_amd._native import check, lib
    w = c3["w"]
    K = 128
    Q = len(w.q_emb)
    ix = read_index(w.index_path)
    table = WindowTable(w.refs)
    q = w.queries
    d_x, d_q = DeviceBuffer.from_host(w.q_emb), DeviceBuffer.from_host(q)
    d_ql = DeviceBuffer.from_host(np.full(Q, q.shape[1], dtype=np.int32))
    outs = []
    for co in (False, True):
        b = {"D": DeviceBuffer((Q, K), np.float32), "I": DeviceBuffer((Q, K), np.int64),
             "nd": DeviceBuffer(Q, np.int32), "nh": DeviceBuffer(Q, np.int32), "nu": DeviceBuffer(Q, np.int32),
             "sc": DeviceBuffer((Q, K), np.int32), "id": DeviceBuffer((Q, K), np.uint64), "st": DeviceBuffer(Q, np.int32)}
        if co:
            st = search_rerank_device(ix, table, d_x, Q, d_q, d_ql, q.shape[1], b["D"], b["I"], b["sc"], b["id"],
                                      b["st"], k=K, ef=128, d_ndis=b["nd"], d_nhops=b["nh"], d_nhops_upper=b["nu"],
                                      stats=True)
            assert st.n_batches == 1 and st.kernel_ms > 0 and st.search_ms > 0 and st.sw_ms > 0
        else:
            ix.search_device(d_x, Q, K, 128, b["D"], b["I"], b["nd"], b["nh"], d_nhops_upper=b["nu"])
            check(lib().drm_post_process_sw_static_device(table.handle, b["I"].ptr, Q, K, d_q.ptr, d_ql.ptr, q.shape[1],
                                                          1, K, K, b["sc"].ptr, b["id"].ptr, b["st"].ptr, None))
        synchronize()
        outs.append({k: v.download() for k, v in b.items()})
    for key in outs[0]:
        assert np.array_equal(outs[0][key].view(np.uint8), outs[1][key].view(np.uint8)), key
    assert (outs[1]["st"] == K).all()
    table.free()
    ix.free()
