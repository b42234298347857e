"""L2 rerank on the GPU (post_process_l2_static -> batch_reranker -> calc_l2_dist, the reference's live
post-processing, src/main.cpp:330) against the oracle (oracle/drm_oracle.c, pinned to the reference's own
calc_l2_dist build and to libstdc++'s std::partial_sort in tests/test_l2_oracle.py).

Bars:
* window embedding table (drm_refs_embed): bit-identical to drm_vectorize of the same windows;
* distances and ids: bit-exact against the oracle on the same embedding table, ties included (duplicate
  labels give exactly equal distances, so the partial_sort tie order is exercised: those queries go to the
  heap replay, the others through the sorted fast path), for k_clusters == kk and < kk, 1 to 800
  candidates per query, dense and sparse (stride > 1: the reference's global expansion stream);
* errors: a label outside the table -> "Invalid mapping index" (DRM_ERR_ARG), kk*stride < k_clusters ->
  DRM_ERR_CANDS;
* the dynamic form (post_process_l2_dynamic, stride > 1) on a genome handle: window table rows equal to
  drm_vectorize of find_sequence's windows (reverse complement for odd ids), reranks bit-exact against the
  oracle's restatement of its stream and boundaries, and its errors."""
import ctypes as C

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def enc():
    from deepreadmapper_amd import Encoder
    e = Encoder()
    yield e
    e.free()


@pytest.fixture(scope="module")
def table(enc):
    from deepreadmapper_amd.rerank import WindowTable, embed_windows
    rng = np.random.default_rng(11)
    win = np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, size=(3000, 150))]
    win[5] = win[6]  # two equal windows: equal embeddings
    t = WindowTable(win)
    embed_windows(t, enc)
    yield t, win
    t.free()


def _download_table(t):
    from deepreadmapper_amd._native import lib
    from deepreadmapper_amd.rerank import window_embeddings_ptr
    p, d = window_embeddings_ptr(t)
    assert p and d == 128
    out = np.empty((t.n_ref, d), dtype=np.float32)
    assert lib().drm_memcpy_d2h(out.ctypes.data_as(C.c_void_p), C.c_void_p(p), out.nbytes) == 0
    return out


def test_embedding_table_equals_vectorize(enc, table):
    t, win = table
    emb = _download_table(t)
    sample = np.r_[0:64, 1000:1064, t.n_ref - 64:t.n_ref]
    want = enc.vectorize([bytes(win[i]) for i in sample])
    assert np.array_equal(emb[sample], want)
    assert np.array_equal(emb[5], emb[6])


@pytest.mark.parametrize("nq,kk,kc,seed", [(400, 128, 128, 1), (300, 128, 50, 2), (64, 40, 1, 3), (1, 1, 1, 4)])
def test_l2_static_dense_bitexact(enc, table, nq, kk, kc, seed):
    from deepreadmapper_amd.rerank import l2_rerank_arrays
    t, win = table
    emb = _download_table(t)
    rng = np.random.default_rng(seed)
    nb = rng.integers(0, t.n_ref, size=(nq, kk)).astype(np.int64)
    nb[:, -1] = nb[:, 0]  # duplicate label per query: an exact tie
    if kk > 3:
        nb[0, 1], nb[0, 2] = 5, 6  # equal windows: an exact tie between different ids
    qe = enc.vectorize([bytes(win[i][::-1]) for i in rng.integers(0, t.n_ref, size=nq)])
    d, ids, counts = l2_rerank_arrays(t, nb, qe, 1, kc)
    rc, wd, wi, st = O.post_process_l2_static(emb, nb, qe, 1, kc)
    assert rc == 0 and (counts == kc).all()
    assert np.array_equal(d.view(np.uint32), wd.view(np.uint32))
    assert np.array_equal(ids, wi)
    assert (np.diff(d, axis=1) >= 0).all()


@pytest.mark.parametrize("stride,kk,kc", [(3, 8, 8), (4, 16, 30), (2, 32, 64), (4, 64, 200), (8, 100, 128)])
def test_l2_static_sparse_stream_bitexact(enc, table, stride, kk, kc):
    from deepreadmapper_amd.rerank import l2_rerank_arrays
    t, win = table
    emb = _download_table(t)
    rng = np.random.default_rng(stride * 7 + kk)
    nq = 120
    nb = rng.integers(0, t.n_ref // stride, size=(nq, kk)).astype(np.int64)
    qe = enc.vectorize([bytes(win[i]) for i in rng.integers(0, t.n_ref, size=nq)])
    d, ids, counts = l2_rerank_arrays(t, nb, qe, stride, kc)
    rc, wd, wi, st = O.post_process_l2_static(emb, nb, qe, stride, kc)
    assert rc == 0 and (counts == kc).all()
    assert np.array_equal(d.view(np.uint32), wd.view(np.uint32))
    assert np.array_equal(ids, wi)


@pytest.mark.parametrize("kc", [128, 37, 1])
def test_l2_static_tie_heavy(enc, table, kc):
    """Labels drawn from 6 windows (two of them equal): every query is full of exact distance ties, so the
    rows come from the libstdc++ heap replay; a few queries without ties take the sorted fast path."""
    from deepreadmapper_amd.rerank import l2_rerank_arrays
    t, win = table
    emb = _download_table(t)
    rng = np.random.default_rng(kc)
    nq = 200
    nb = rng.choice(np.array([5, 6, 7, 8, 9, 10]), size=(nq, 128)).astype(np.int64)
    nb[:20] = rng.integers(0, t.n_ref, size=(20, 128))  # mostly tie-free
    qe = enc.vectorize([bytes(win[i]) for i in rng.integers(0, t.n_ref, size=nq)])
    d, ids, counts = l2_rerank_arrays(t, nb, qe, 1, kc)
    rc, wd, wi, st = O.post_process_l2_static(emb, nb, qe, 1, kc)
    assert rc == 0 and (counts == kc).all()
    assert np.array_equal(d.view(np.uint32), wd.view(np.uint32))
    assert np.array_equal(ids, wi)


def test_l2_static_errors(enc, table):
    from deepreadmapper_amd._native import DRM_ERR_ARG, DRM_ERR_CANDS, DrmError
    from deepreadmapper_amd.rerank import l2_rerank_arrays
    t, _ = table
    qe = np.zeros((2, 128), np.float32)
    nb = np.array([[1, 2, 3], [4, -1, 5]], np.int64)
    with pytest.raises(DrmError) as e:
        l2_rerank_arrays(t, nb, qe, 1, 3)
    assert e.value.code == DRM_ERR_ARG and "Invalid mapping index" in str(e.value)
    with pytest.raises(DrmError) as e:
        l2_rerank_arrays(t, nb[:1], qe[:1], 1, 4)
    assert e.value.code == DRM_ERR_CANDS
    with pytest.raises(DrmError):
        l2_rerank_arrays(t, nb[:1], np.zeros((1, 64), np.float32), 1, 3)  # width mismatch


def test_post_process_l2_static_reference_shape(enc, table):
    """The reference-shaped entry: flattened (final_seqs, final_dists, final_ids), k_clusters per query."""
    from deepreadmapper_amd import post_process_l2_static
    t, win = table
    refs = [bytes(w) for w in win[:500]]
    rng = np.random.default_rng(9)
    nb = rng.integers(0, 500, size=(10, 16)).astype(np.int64)
    qe = enc.vectorize([refs[i] for i in nb[:, 0]])
    seqs, dists, ids = post_process_l2_static(nb, None, refs, None, 150, 1, 5, qe, enc, 16)
    assert len(seqs) == len(dists) == len(ids) == 160
    assert all(seqs[i] == refs[ids[i]] for i in range(160))
    assert dists[0] == 0.0 and ids[0] == nb[0, 0]  # the query is window nb[0,0] itself


@pytest.fixture(scope="module")
def genome_table(enc):
    from deepreadmapper_amd.rerank import GenomeTable, embed_windows
    rng = np.random.default_rng(21)
    g = bytes(np.frombuffer(b"ACGTN", dtype=np.uint8)[rng.choice(5, size=6000, p=[.24, .24, .24, .24, .04])])
    t = GenomeTable(g, 150)
    embed_windows(t, enc)
    yield t, g
    t.free()


def _window(g, w, L=150):
    """find_sequence (src/utils/post_processor.cpp:47-64): window w of the dynamic lookup"""
    comp = {ord("A"): "T", ord("T"): "A", ord("C"): "G", ord("G"): "C", ord("N"): "N"}
    pos = w // 2
    s = g[pos:pos + L]
    return "".join(comp[c] for c in s[::-1]).encode() if w % 2 else s


def test_genome_embedding_table(enc, genome_table):
    t, g = genome_table
    emb = _genome_emb(t, len(g))
    sample = [0, 1, 2, 3, 101, 2999, 3000, len(g) - 1]
    want = enc.vectorize([_window(g, w) for w in sample])
    assert np.array_equal(emb[sample], want)


def _genome_emb(t, n):
    from deepreadmapper_amd._native import lib
    from deepreadmapper_amd.rerank import window_embeddings_ptr
    p, d = window_embeddings_ptr(t)
    emb = np.empty((n, d), dtype=np.float32)
    assert lib().drm_memcpy_d2h(emb.ctypes.data_as(C.c_void_p), C.c_void_p(p), emb.nbytes) == 0
    return emb


@pytest.mark.parametrize("stride,kk,k,kc", [(2, 16, 5, 16), (3, 32, 40, 20), (4, 8, 8, 8)])
def test_l2_dynamic_sparse_bitexact(enc, genome_table, stride, kk, k, kc):
    """Interior labels (no clipping): each query reranks its own first min(k_clusters, kk) labels' windows."""
    from deepreadmapper_amd.rerank import l2_rerank_dynamic_arrays
    t, g = genome_table
    emb = _genome_emb(t, len(g))
    rng = np.random.default_rng(stride * 13 + kk)
    nq = 80
    nb = rng.integers(1, (len(g) - stride) // stride, size=(nq, kk)).astype(np.int64)
    qe = enc.vectorize([_window(g, int(w)) for w in rng.integers(0, len(g), size=nq)])
    dd, ids, counts = l2_rerank_dynamic_arrays(t, nb, qe, stride, k, kc)
    rc, wd, wi, st = O.post_process_l2_dynamic(emb, nb, qe, stride, k, kc)
    assert rc == 0 and (counts == k).all()
    assert np.array_equal(dd.view(np.uint32), wd.view(np.uint32))
    assert np.array_equal(ids, wi)


def test_l2_dynamic_sparse_clipped_stream(enc, genome_table):
    """Labels at the genome's ends clip their expansion: the reference's boundaries then straddle queries, and
    the tail queries run past the stream (status -4). Device form, compared query by query."""
    from deepreadmapper_amd._native import check, lib
    from deepreadmapper_amd.device import DeviceBuffer, Stream
    t, g = genome_table
    emb = _genome_emb(t, len(g))
    rng = np.random.default_rng(77)
    nq, kk, stride, k, kc = 40, 12, 3, 10, 12
    nb = rng.integers(1, (len(g) - stride) // stride, size=(nq, kk)).astype(np.int64)
    nb[0, 0], nb[3, 5], nb[7, 2] = 0, len(g) // stride + 5, (len(g) - 1) // stride  # clipped / dropped labels
    qe = enc.vectorize([_window(g, int(w)) for w in rng.integers(0, len(g), size=nq)])
    d_nb, d_qe = DeviceBuffer.from_host(nb), DeviceBuffer.from_host(qe)
    d_d, d_i, d_s = DeviceBuffer((nq, k), np.float32), DeviceBuffer((nq, k), np.uint64), DeviceBuffer(nq, np.int32)
    st = Stream()
    check(lib().drm_post_process_l2_dynamic_device(t.handle, d_nb.ptr, nq, kk, d_qe.ptr, 128, stride, k, kc,
                                                   d_d.ptr, d_i.ptr, d_s.ptr, st.handle))
    st.synchronize()
    rc, wd, wi, ws = O.post_process_l2_dynamic(emb, nb, qe, stride, k, kc)
    status = d_s.download()
    assert rc < 0 and np.array_equal(status, ws) and (ws == -4).any() and (ws == k).sum() > nq // 2
    ok = ws == k
    assert np.array_equal(d_d.download()[ok].view(np.uint32), wd[ok].view(np.uint32))
    assert np.array_equal(d_i.download()[ok], wi[ok])


def test_l2_dynamic_errors(enc, genome_table):
    from deepreadmapper_amd._native import DRM_ERR_ARG, DRM_ERR_K, DrmError
    from deepreadmapper_amd.rerank import l2_rerank_dynamic_arrays
    t, g = genome_table
    qe = np.zeros((1, 128), np.float32)
    nb = np.zeros((1, 4), np.int64)
    with pytest.raises(DrmError) as e:
        l2_rerank_dynamic_arrays(t, nb, qe, 1, 2, 4)  # stride 1: a pass-through of the search
    assert e.value.code == DRM_ERR_ARG
    with pytest.raises(DrmError) as e:
        l2_rerank_dynamic_arrays(t, nb, qe, 2, 17, 4)  # k > k_clusters * 2 * stride
    assert e.value.code == DRM_ERR_K
    nb = np.full((2, 4), len(g), np.int64)  # every label past the genome: an empty stream
    with pytest.raises(DrmError) as e:
        l2_rerank_dynamic_arrays(t, nb, np.zeros((2, 128), np.float32), 2, 4, 4)
    assert e.value.code == DRM_ERR_ARG and "Invalid mapping index" in str(e.value)


def test_pipeline_cli_dynamic_sparse_sam(tmp_path):
    """bin/pipeline use_dynamic=1 use_streaming=1 on a stride-2 index with the GRU model.
    Default: the reference's observable output, a header-only SAM -- its sparse-branch write_sam_streaming
    call (src/utils/post_processor.cpp:1004-1005) leaves batch_query_count at its default 0
    (includes/utils/utils.hpp:99), so no row is written. DRM_SAM_L2_ROWS=1: the L2 rerank's rows. Sparse labels
    run to ~2 * genome length / stride while the expansion keeps only label * stride < genome length, so the
    stream is shorter than the reference's query boundaries and the tail queries' ranges run past it (the
    reference reads out of bounds there): those queries are written without rows, the run still succeeds."""
    import os
    import subprocess
    from deepreadmapper_amd.encoder import DEFAULT_MODEL
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    fna = os.path.join(root, "tests", "golden", "ecoli_150.fna")
    fq = os.path.join(root, "tests", "golden", "test_data.fastq")
    env = dict(os.environ, DRM_BUILD_THREADS="1", DRM_ENCODER=DEFAULT_MODEL)
    r = subprocess.run([os.path.join(root, "bin", "hnswpq_index"), fna, "s2", "150", "2"], cwd=tmp_path, env=env,
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    # ef 128, k 10, k_clusters 64 (src/main.cpp:54-62): 64 labels x 3 windows of boundary per query
    argv = [os.path.join(root, "bin", "pipeline"), "s2", fq, fna, "128", "10", "64", "out", "1", "1"]
    r = subprocess.run(argv, cwd=tmp_path, env=env, capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    sam = open(tmp_path / "out" / "results.sam").read()
    assert sam == "@HD\tVN:1.0\tSO:unsorted\n@SQ\tSN:ref\tLN:150\n"
    r = subprocess.run(argv, cwd=tmp_path, env=dict(env, DRM_SAM_L2_ROWS="1"), capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "clipped expansion stream" in r.stdout
    lines = open(tmp_path / "out" / "results.sam").read().splitlines()
    rows = [l.split("\t") for l in lines[2:]]
    assert lines[:2] == ["@HD\tVN:1.0\tSO:unsorted", "@SQ\tSN:ref\tLN:150"] and len(rows) > 0
    per_q = {}
    for f in rows:
        per_q[f[0]] = per_q.get(f[0], 0) + 1
        assert f[2] == "ref" and f[4] == "60" and f[5] == "150M" and 1 <= int(f[3]) <= 1000
    assert all(c == 10 for c in per_q.values()) and len(per_q) < 150


def test_post_process_l2_dynamic_reference_shape(enc, genome_table):
    """The reference-shaped dynamic entry: stride 1 passes the first min(k, kk) search neighbours through with
    their search distances; stride 2 returns the L2 rerank's k rows per query with their windows."""
    from deepreadmapper_amd import post_process_l2_dynamic
    t, g = genome_table
    rng = np.random.default_rng(5)
    nb = rng.integers(1, (len(g) - 2) // 2, size=(6, 10)).astype(np.int64)
    dist = rng.random((6, 10)).astype(np.float32)
    qe = enc.vectorize([_window(g, int(w)) for w in nb[:, 0]])
    seqs, dd, ids = post_process_l2_dynamic(nb, dist, g, None, 150, 1, 4, qe, enc, 10)
    assert ids == [int(x) for x in nb[:, :4].reshape(-1)] and dd == [float(x) for x in dist[:, :4].reshape(-1)]
    assert seqs[0] == _window(g, int(nb[0, 0]))
    seqs, dd, ids = post_process_l2_dynamic(nb, dist, t, None, 150, 2, 7, qe, enc, 10)
    assert len(ids) == 42 and all(s is None for s in seqs)
    assert all(dd[i] <= dd[i + 1] for q in range(6) for i in range(q * 7, q * 7 + 6))
