"""C5 at full size (BASELINE configs[4]): 50,000,000 stride-1 windows of a seeded
25,000,149 bp genome, embedded by the GRU model and indexed on the GPU (the bench's default workload).
A 512-read sample is checked bit-exactly against the oracle at this scale -- search ids, 0-ulp
distances, ndis, nhops, SW scores and ids -- and the whole sample passes the size-independent checks
(rows ascending, status == K). About two minutes on one MI355X, most of it building the workload."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

C5_GENOME = 25_000_149
SAMPLE = 512


@pytest.fixture(scope="module")
def c5(tmp_path_factory):
    from deepreadmapper_amd import synth
    d = tmp_path_factory.mktemp("c5")
    g = synth.genome(C5_GENOME, seed=44)
    refs = synth.windows_lookup(g, 150, 1)
    assert refs.shape == (50_000_000, 150)
    path = str(d / "c5_gru.index")
    synth.build_index_gpu_from_rows(refs, path, embed="gru")
    reads, truth = synth.simulate_reads_range(g, 0, SAMPLE, seed=9)
    q = synth.tag(reads)
    return {"refs": refs, "index": path, "q": q, "x": synth.embed_gru(q), "truth": truth}


def test_c5_search_and_rerank_vs_oracle(c5):
    from deepreadmapper_amd import read_index, WindowTable, rerank_arrays
    from oracle import faiss_file, oracle as O
    K = EF = 128
    ix = read_index(c5["index"])
    ix.set_exact_stats(True)  # ndis as faiss counts it (the full-slice test runs the default mode)
    D, I, st = ix.search(c5["x"], K, EF)
    fx = faiss_file.read(c5["index"])
    Do, Io, nd, nh = O.hnswpq_search(fx, c5["x"], K, EF)
    del fx
    assert np.array_equal(I, Io)
    assert np.array_equal(D.view(np.uint32), Do.view(np.uint32))
    assert st.ndis == int(nd.sum()) and st.nhops == int(nh.sum())
    assert (np.diff(D, axis=1) >= 0).all()
    table = WindowTable(c5["refs"])
    q = c5["q"]
    ql = np.full(len(q), q.shape[1], dtype=np.int32)
    sc, ids, cnt = rerank_arrays(table, I, (q, ql), 1, K, K)
    rc, sco, ido, cnto = O.post_process_sw_static(I, c5["refs"], 150, q, ql, 1, K, K)
    assert rc == 0 and (cnt == K).all()
    assert np.array_equal(sc, sco) and np.array_equal(ids, ido)
    # the GRU embeddings put most reads on their source window
    assert float(np.mean(ids[:, 0].astype(np.int64) == c5["truth"])) > 0.6
    table.free()
    ix.free()


def test_c5_l2_rerank_vs_oracle(c5):
    """post_process_l2_static at full size: the 50M-window GRU embedding table built on the device, the sample's
    search neighbours reranked by L2 and compared bit-exactly with the oracle on the gathered table rows."""
    import ctypes as C
    from deepreadmapper_amd import read_index, WindowTable, Encoder
    from deepreadmapper_amd._native import lib
    from deepreadmapper_amd.rerank import embed_windows, l2_rerank_arrays, window_embeddings_ptr
    from oracle import oracle as O
    K = EF = 128
    ix = read_index(c5["index"])
    _, I, _ = ix.search(c5["x"], K, EF)
    ix.free()
    table = WindowTable(c5["refs"])
    enc = Encoder()
    embed_windows(table, enc)
    enc.free()
    d, ids, cnt = l2_rerank_arrays(table, I, c5["x"], 1, K)
    # gather the candidates' rows from the device table, relabel the neighbours compactly for the oracle
    p, dim = window_embeddings_ptr(table)
    uniq, inv = np.unique(I, return_inverse=True)
    rows = np.empty((len(uniq), dim), np.float32)
    for r, w in enumerate(uniq):
        assert lib().drm_memcpy_d2h(rows[r].ctypes.data_as(C.c_void_p), C.c_void_p(p + int(w) * dim * 4), dim * 4) == 0
    rc, wd, wi, st = O.post_process_l2_static(rows, inv.reshape(I.shape).astype(np.int64), c5["x"], 1, K)
    assert rc == 0 and (cnt == K).all()
    assert np.array_equal(d.view(np.uint32), wd.view(np.uint32))
    assert np.array_equal(ids, uniq[wi.astype(np.int64)].astype(np.uint64))
    table.free()


def test_c5_full_slice_properties(c5):
    """The bench's whole per-GPU slice (1,250,000 reads of the same seeded stream, GRU-embedded): device
    search + device SW rerank at EF = K = 128 over every read, with the size-independent checks on every
    row -- ascending search rows, labels inside the table, ndis / nhops > 0, status == K, SW scores
    descending and within [0, 150], each row's SW ids a permutation of its search ids (dense, all 128 ids
    valid: find_sequences keeps them all, post_processor.cpp:215-236) -- and the first 512 rows equal to
    the oracle-checked sample above (reads [0, 512) of the stream); and a strided sample across the whole slice (every
    977th read) equal to the oracle bit for bit."""
    from deepreadmapper_amd import read_index, synth, WindowTable
    from deepreadmapper_amd.device import DeviceBuffer, synchronize
    from deepreadmapper_amd._native import check, lib
    K = EF = 128
    Q = 1_250_000
    g = synth.genome(C5_GENOME, seed=44)
    reads, truth = synth.simulate_reads_range(g, 0, Q, seed=9)
    q = synth.tag(reads)
    x = synth.embed_gru(q)
    assert np.array_equal(x[:SAMPLE], c5["x"])
    ix = read_index(c5["index"])
    table = WindowTable(c5["refs"])
    d_x, d_q = DeviceBuffer.from_host(x), DeviceBuffer.from_host(q)
    d_ql = DeviceBuffer.from_host(np.full(Q, q.shape[1], dtype=np.int32))
    d_D, d_I = DeviceBuffer((Q, K), np.float32), DeviceBuffer((Q, K), np.int64)
    nd, nh = DeviceBuffer(Q, np.int32), DeviceBuffer(Q, np.int32)
    d_sc, d_id, d_st = DeviceBuffer((Q, K), np.int32), DeviceBuffer((Q, K), np.uint64), DeviceBuffer(Q, np.int32)
    ix.search_device(d_x, Q, K, EF, d_D, d_I, nd, nh)
    check(lib().drm_post_process_sw_static_device(table.handle, d_I.ptr, Q, K, d_q.ptr, d_ql.ptr, q.shape[1], 1, K, K,
                                                  d_sc.ptr, d_id.ptr, d_st.ptr, None))
    synchronize()
    D, I = d_D.download(), d_I.download()
    assert (np.diff(D, axis=1) >= 0).all()
    assert (I >= 0).all() and (I < len(c5["refs"])).all()
    assert (nd.download() > 0).all() and (nh.download() > 0).all()
    st, sc, ids = d_st.download(), d_sc.download(), d_id.download()
    assert (st == K).all()
    assert (np.diff(sc, axis=1) <= 0).all() and (sc >= 0).all() and (sc <= 150).all()
    assert np.array_equal(np.sort(ids.astype(np.int64), axis=1), np.sort(I, axis=1))
    D0, I0, _ = ix.search(c5["x"], K, EF)
    assert np.array_equal(I[:SAMPLE], I0) and np.array_equal(D[:SAMPLE].view(np.uint32), D0.view(np.uint32))
    assert float(np.mean(ids[:, 0].astype(np.int64) == truth)) > 0.6
    # a strided sample across the whole slice (every 977th read, 1,280 reads) against the oracle, bit for bit: the
    # device rows of the full launch -- search ids, 0-ulp distances, nhops -- and the SW rerank's scores and ids
    from oracle import faiss_file, oracle as O
    idx = np.arange(0, Q, 977)
    fx = faiss_file.read(c5["index"])
    Do, Io, ndo, nho = O.hnswpq_search(fx, np.ascontiguousarray(x[idx]), K, EF)
    del fx
    assert np.array_equal(I[idx], Io) and np.array_equal(D[idx].view(np.uint32), Do.view(np.uint32))
    assert np.array_equal(nh.download()[idx], nho)
    qs = np.ascontiguousarray(q[idx])
    rc, sco, ido, cnto = O.post_process_sw_static(np.ascontiguousarray(I[idx]), c5["refs"], 150, qs,
                                                  np.full(len(idx), q.shape[1], dtype=np.int32), 1, K, K)
    assert rc == 0 and np.array_equal(sc[idx], sco) and np.array_equal(ids[idx], ido)
    table.free()
    ix.free()
