"""GPU parity of the fp32-L2 hnswlib kernel (hnsw_flat_search.hip) against the oracle restatement
(oracle/hnswlib_oracle.cpp, libstdc++'s own priority_queue): labels, fp32 distances (0 ulp, same op
order) and ndis/nhops bit-exact, including an index full of exact distance ties (the launch is the exact heap
replay; the opt-in tie-free sorted-array pass was removed in round 5)."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _both(index_path, fx, q, k, ef):
    from deepreadmapper_amd import HnswFlatIndex
    ix = HnswFlatIndex(index_path)
    D, L, st = ix.search(q, k, ef)
    Do, Io, nd, nh = O.hnswlib_search(fx, q, k, ef)
    pad = Io < 0
    assert np.array_equal(L.astype(np.int64)[~pad], Io[~pad]) and (L[pad] == np.uint64(2 ** 64 - 1)).all()
    assert np.array_equal(D.view(np.uint32), Do.view(np.uint32))  # 0 ulp
    assert st.ndis == int(nd.sum()) and st.nhops == int(nh.sum())
    assert ix.search_errors() == 0
    ix.free()
    return D, L


@pytest.mark.parametrize("k,ef", [(128, 128), (10, 64), (1, 1), (200, 100), (32, 400)])
def test_flat_c1_bitexact(c1_flat, k, ef):
    _both(c1_flat["index"], c1_flat["fx"], c1_flat["q"], k, ef)


def test_flat_syn20k_bitexact(syn_flat):
    _both(syn_flat["index"], syn_flat["fx"], syn_flat["q"], 128, 128)


def test_flat_ties_bitexact(rep_flat):
    """identical vectors (repeated genome segments): equal distances everywhere, so the heap layouts
    of top_candidates and candidate_set decide the traversal and the k cut"""
    _both(rep_flat["index"], rep_flat["fx"], rep_flat["q"], 64, 128)
    _both(rep_flat["index"], rep_flat["fx"], rep_flat["x"][::7], 16, 40)


def test_flat_exhaustive_and_random(syn_flat):
    rng = np.random.default_rng(4)
    q = rng.standard_normal((40, 128)).astype(np.float32)
    _both(syn_flat["index"], syn_flat["fx"], q, 50, 96)
    _both(syn_flat["index"], syn_flat["fx"], syn_flat["q"][:20], 30, 25000)  # ef > ntotal


def test_flat_search_api(c1_flat):
    from deepreadmapper_amd import load_flat_index
    from deepreadmapper_amd.flat import search
    ix = load_flat_index(c1_flat["index"])
    labels, dists = search(ix, c1_flat["q"][:3].tolist(), 7, 32)
    assert len(labels) == 3 and all(len(r) == 7 for r in labels) and len(dists[0]) == 7
    assert all(dists[0][i] <= dists[0][i + 1] for i in range(6))
    with pytest.raises(RuntimeError, match="Query data is empty"):
        search(ix, [], 7, 32)
    assert ix.overflows() == 0


def test_flat_large_batch(c1_flat, rep_flat):
    """A batch larger than the resident wave slots (1200 queries: slots are re-used across queries, so
    the visited bitmaps must be cleared exactly) against the oracle, at several (k, ef)."""
    q = np.concatenate([c1_flat["q"]] * 8)
    for k, ef in [(128, 128), (10, 64), (200, 100)]:
        _both(c1_flat["index"], c1_flat["fx"], q, k, ef)
    qr = np.concatenate([rep_flat["q"]] * (1024 // len(rep_flat["q"]) + 1))
    _both(rep_flat["index"], rep_flat["fx"], qr, 64, 128)
