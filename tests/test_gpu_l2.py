"""L2 rerank on the GPU (post_process_l2_static -> batch_reranker -> calc_l2_dist, the reference's live
post-processing, src/main.cpp:330) against the oracle (oracle/drm_oracle.c, pinned to the reference's own
calc_l2_dist build and to libstdc++'s std::partial_sort in tests/test_l2_oracle.py).

Bars:
* window embedding table (drm_refs_embed): bit-identical to drm_vectorize of the same windows;
* distances and ids: bit-exact against the oracle on the same embedding table, ties included (duplicate
  labels give exactly equal distances, so the partial_sort tie order is exercised), for k_clusters == kk
  and < kk, dense and sparse (stride > 1: the reference's global expansion stream);
* errors: a label outside the table -> "Invalid mapping index" (DRM_ERR_ARG), kk*stride < k_clusters ->
  DRM_ERR_CANDS."""
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


@pytest.mark.parametrize("stride,kk,kc", [(3, 8, 8), (4, 16, 30), (2, 32, 64)])
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
