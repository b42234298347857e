"""Batch executor and multi-GPU fan-out (csrc/exec.cpp; SURVEY.md sec. 8b drm_search_rerank, sec. 8e):

* drm_search_rerank (batched, three streams, ping-pong device buffers) equals drm_search followed by
  drm_post_process_sw_static bit for bit, for one batch and for many uneven batches;
* drm_multi_search_rerank over G replicas (the file parsed once, the others drm_index_clone copies) -- here
  G "logical devices" that all map to device 0 of the one-GPU box -- writes outputs byte-identical to the
  one-device run (contiguous shards, no exchange);
* the RCCL gather (drm_comm_gather_rows) of a one-rank job returns the rank's rows;
* bin/pipeline with DRM_DEVICES=0,0,0 writes the same .npy files as with one device.
Reference call sites: src/main.cpp:278 (faiss_search), :333-341 (post_process_sw_static), the OpenMP
over queries of src/utils/post_processor.cpp:491."""
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def _separate(index_path, w, k, ef):
    from deepreadmapper_amd import read_index, WindowTable, rerank_arrays
    ix = read_index(index_path)
    D, I, st = ix.search(w.q_emb, k, ef)
    ix.free()
    table = WindowTable(w.refs)
    ql = np.full(len(I), w.queries.shape[1], dtype=np.int32)
    sc, ids, cnt = rerank_arrays(table, I, (w.queries, ql), 1, k, k)
    table.free()
    return D, I, sc, ids, cnt, st


@pytest.mark.parametrize("batch", [None, "333"])
def test_search_rerank_fused_equals_separate(syn20k, monkeypatch, batch):
    from deepreadmapper_amd import read_index, WindowTable
    from deepreadmapper_amd.executor import search_rerank
    if batch:
        monkeypatch.setenv("DRM_BATCH", batch)  # 2000 queries -> 7 batches, the last one short
    w = syn20k["w"]
    D, I, sc, ids, cnt, st = _separate(w.index_path, w, 128, 128)
    ix, table = read_index(w.index_path), WindowTable(w.refs)
    o = search_rerank(ix, table, w.q_emb, w.queries, k=128, ef=128)
    assert np.array_equal(o["I"], I) and np.array_equal(o["D"].view(np.uint32), D.view(np.uint32))
    assert np.array_equal(o["sw_scores"], sc) and np.array_equal(o["sw_ids"], ids)
    assert (o["status"] == 128).all() and (cnt == 128).all()
    assert o["stats"].ndis == st.ndis and o["stats"].nhops == st.nhops and o["stats"].nq == len(w.q_emb)
    # search only (no window table)
    o2 = search_rerank(ix, None, w.q_emb, None, k=64, ef=128)
    D2, I2, _ = ix.search(w.q_emb, 64, 128)
    assert np.array_equal(o2["I"], I2) and "sw_scores" not in o2
    ix.free()
    table.free()


def test_search_rerank_ramped_batches(syn20k):
    """The default batch plan at scale (no DRM_BATCH): 140,000 queries make four or more batches, so the executor
    runs a quarter-size first and last batch around equal middle ones, each search after the previous rerank
    (DESIGN.md sec. 5); the outputs equal the separate whole-array search and rerank bit for bit."""
    from deepreadmapper_amd import read_index, WindowTable, rerank_arrays
    from deepreadmapper_amd.executor import search_rerank
    w = syn20k["w"]
    reps = 70
    x, qb = np.tile(w.q_emb, (reps, 1)), np.tile(w.queries, (reps, 1))
    ix, table = read_index(w.index_path), WindowTable(w.refs)
    D, I, st = ix.search(x, 128, 128)
    sc, ids, cnt = rerank_arrays(table, I, (qb, np.full(len(I), qb.shape[1], dtype=np.int32)), 1, 128, 128)
    o = search_rerank(ix, table, x, qb, k=128, ef=128)
    assert np.array_equal(o["I"], I) and np.array_equal(o["D"].view(np.uint32), D.view(np.uint32))
    assert np.array_equal(o["sw_scores"], sc) and np.array_equal(o["sw_ids"], ids)
    assert (o["status"] == 128).all() and o["stats"].nq == len(x) and o["stats"].nhops == st.nhops
    ix.free()
    table.free()


def test_search_rerank_errors(syn20k):
    from deepreadmapper_amd import read_index, WindowTable
    from deepreadmapper_amd.executor import search_rerank
    from deepreadmapper_amd._native import DrmError, DRM_ERR_K
    w = syn20k["w"]
    ix, table = read_index(w.index_path), WindowTable(w.refs)
    with pytest.raises(DrmError) as e:  # k > k_clusters * 2 * stride (post_processor.cpp:486-489)
        search_rerank(ix, table, w.q_emb[:10], w.queries[:10], k=128, ef=128, k_clusters=50)
    assert e.value.code == DRM_ERR_K
    with pytest.raises(DrmError, match="Query data is empty"):
        search_rerank(ix, table, w.q_emb[:0], w.queries[:0], k=16, ef=16)
    ix.free()
    table.free()


@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0]])
def test_multi_logical_devices_byte_identical(syn20k, devices, monkeypatch):
    from deepreadmapper_amd import read_index, WindowTable
    from deepreadmapper_amd.executor import MultiIndex, search_rerank
    monkeypatch.setenv("DRM_BATCH", "500")
    w = syn20k["w"]
    ix, table = read_index(w.index_path), WindowTable(w.refs)
    n = 1999  # shards of unequal size
    one = search_rerank(ix, table, w.q_emb[:n], w.queries[:n], k=128, ef=128)
    ix.free()
    table.free()
    m = MultiIndex(w.index_path, devices, w.refs)
    assert m.info.ntotal == syn20k["fx"].ntotal
    many = m.search_rerank(w.q_emb[:n], w.queries[:n], k=128, ef=128)
    m.free()
    for key in ("I", "sw_scores", "sw_ids", "status"):
        assert np.array_equal(many[key], one[key]), key
    assert np.array_equal(many["D"].view(np.uint32), one["D"].view(np.uint32))
    assert many["stats"].ndis == one["stats"].ndis and many["stats"].nq == n


def test_rccl_gather_one_rank():
    from deepreadmapper_amd.device import DeviceBuffer, synchronize
    from deepreadmapper_amd.executor import Comm
    c = Comm(Comm.unique_id(), 1, 0, 0)
    rows = np.arange(1000 * 24, dtype=np.uint8).reshape(1000, 24)
    src, dst = DeviceBuffer.from_host(rows), DeviceBuffer((1000, 24), np.uint8)
    c.gather_rows(src, 1000, 24, dst, root=0)
    synchronize()
    assert np.array_equal(dst.download(), rows)
    c.free()


def test_index_broadcast_one_rank_copy(syn20k):
    """drm_index_broadcast's receive side on a one-rank job (copy=True: the root receives a separate replica through
    the header, agreement, grouped ncclBroadcast and checksum steps): the replica searches bit-identically to the
    loaded index (ids, 0-ulp distances, ndis, nhops) and reports the same header."""
    from deepreadmapper_amd import read_index
    from deepreadmapper_amd.executor import Comm
    from deepreadmapper_amd.search import HnswPqIndex
    w = syn20k["w"]
    c = Comm(Comm.unique_id(), 1, 0, 0)
    ix = read_index(w.index_path)
    same = HnswPqIndex.broadcast(c, ix, root=0)  # the root's own index is the replica
    assert same is ix
    rep = HnswPqIndex.broadcast(c, ix, root=0, copy=True)
    assert rep.handle != ix.handle
    for f in ("d", "ntotal", "pq_M", "pq_nbits", "M_hnsw", "max_level", "entry_point", "efConstruction", "efSearch",
              "metric_type", "device_bytes"):
        assert getattr(rep.info, f) == getattr(ix.info, f), f
    q = w.q_emb[:1000]
    D0, I0, s0 = ix.search(q, 128, 128)
    ix.free()  # the replica owns its buffers
    D1, I1, s1 = rep.search(q, 128, 128)
    assert np.array_equal(I0, I1) and np.array_equal(D0.view(np.uint32), D1.view(np.uint32))
    assert (s0.ndis, s0.nhops) == (s1.ndis, s1.nhops)
    rep.free()
    c.free()


def test_index_clone_searches_identically(syn20k):
    """drm_index_clone (what drm_multi_create uses for every device after the first): the clone searches
    bit-identically and survives the source being freed."""
    from deepreadmapper_amd import read_index
    w = syn20k["w"]
    ix = read_index(w.index_path)
    cl = ix.clone()
    assert cl.handle != ix.handle and cl.info.device_bytes == ix.info.device_bytes
    q = w.q_emb[:1000]
    D0, I0, s0 = ix.search(q, 64, 128)
    ix.free()
    D1, I1, s1 = cl.search(q, 64, 128)
    assert np.array_equal(I0, I1) and np.array_equal(D0.view(np.uint32), D1.view(np.uint32))
    assert (s0.ndis, s0.nhops) == (s1.ndis, s1.nhops)
    cl.free()


def test_index_broadcast_argument_errors(syn20k):
    from deepreadmapper_amd._native import DrmError, DRM_ERR_ARG
    from deepreadmapper_amd.executor import Comm
    from deepreadmapper_amd.search import HnswPqIndex
    c = Comm(Comm.unique_id(), 1, 0, 0)
    with pytest.raises(DrmError) as e:  # the root without an index: refused on every rank before any transfer
        HnswPqIndex.broadcast(c, None, root=0, copy=True)
    assert e.value.code == DRM_ERR_ARG
    with pytest.raises(DrmError) as e:
        HnswPqIndex.broadcast(c, None, root=1)
    assert e.value.code == DRM_ERR_ARG
    c.free()


def test_pipeline_cli_multi_devices(tmp_path):
    fna = os.path.join(GOLDEN, "ecoli_150.fna")
    fq = os.path.join(GOLDEN, "test_data.fastq")
    env = dict(os.environ, DRM_BUILD_THREADS="1")
    r = subprocess.run([os.path.join(ROOT, "bin", "hnswpq_index"), fna, "c1", "150"], cwd=tmp_path, env=env,
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    outs = {}
    for name, devs in (("one", None), ("three", "0,0,0")):
        e = dict(os.environ, DRM_BATCH="64")
        if devs:
            e["DRM_DEVICES"] = devs
        r = subprocess.run([os.path.join(ROOT, "bin", "pipeline"), "c1", fq, fna, "128", "128", "5", name],
                           cwd=tmp_path, env=e, capture_output=True, text=True)
        assert r.returncode == 0, r.stdout + r.stderr
        outs[name] = {f: open(tmp_path / name / f, "rb").read() for f in
                      ("indices.npy", "distances.npy", "sw_scores.npy", "sw_ids.npy")}
    assert "3 device(s)" in r.stdout
    assert outs["one"] == outs["three"]


def test_device_chase_latency_probe():
    """drm_device_chase_latency (bench.py's live dependent-load latency): a plausible per-hop time on a small table,
    and its argument checks."""
    import ctypes as C
    from deepreadmapper_amd._native import DRM_ERR_ARG, lib
    ns = C.c_double(0.0)
    assert lib().drm_device_chase_latency(0, 256 << 20, 256, 200, C.byref(ns)) == 0
    assert 100.0 < ns.value < 20000.0, ns.value
    assert lib().drm_device_chase_latency(0, 100, 256, 200, C.byref(ns)) == DRM_ERR_ARG
    assert lib().drm_device_chase_latency(0, 256 << 20, 0, 200, C.byref(ns)) == DRM_ERR_ARG
