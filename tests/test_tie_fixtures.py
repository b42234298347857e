"""Search parity beyond "HIP == restatement" (SURVEY.md sec. 8c(ii)): hand-derived traversal fixtures on tiny
tie-heavy graphs (tests/golden/hnsw_tie_cases.json), checked against a literal restatement of upstream faiss
(tests/faiss_literal.py, statement by statement, no code shared with oracle/drm_oracle.c) and against the C
oracle; random tie-heavy graphs then compare the two restatements with each other. The GPU kernels meet the
same fixtures in tests/test_gpu_parity.py::test_search_tie_fixtures."""
import numpy as np
import pytest

import faiss_literal as FL
import tie_graphs as TG
from oracle import faiss_file, oracle as O


@pytest.mark.parametrize("case", TG.load_cases(), ids=lambda c: c["name"])
def test_literal_restatement_reproduces_hand_trace(case, tmp_path):
    path = TG.write_case(case, str(tmp_path))
    fx = faiss_file.read(path)
    q = np.zeros((1, TG.D), dtype=np.float32)
    Dl, Il, ndl, nhl = FL.search(fx, q, case["k"], case["ef"])
    e = case["expected"]
    assert Il[0].tolist() == e["I"] and Dl[0].tolist() == e["D"]
    assert int(ndl[0]) == e["ndis"] and int(nhl[0]) == e["nhops"]


@pytest.mark.parametrize("case", TG.load_cases(), ids=lambda c: c["name"])
def test_c_oracle_reproduces_hand_trace(case, tmp_path):
    path = TG.write_case(case, str(tmp_path))
    fx = faiss_file.read(path)
    q = np.zeros((1, TG.D), dtype=np.float32)
    Do, Io, nd, nh = O.hnswpq_search(fx, q, case["k"], case["ef"])
    e = case["expected"]
    assert Io[0].tolist() == e["I"] and Do[0].tolist() == e["D"]
    assert int(nd[0]) == e["ndis"] and int(nh[0]) == e["nhops"]


def test_random_tie_graphs_literal_vs_oracle(tmp_path):
    """60 random graphs of 6-40 nodes with 4 distinct code values (ties everywhere), duplicate links, holes and
    up to 3 levels, searched from several queries (the zero query plus random ones) at several (k, ef):
    the literal restatement and the C oracle agree on ids, distances (0 ulp), ndis and nhops."""
    rng = np.random.default_rng(2024)
    checked = 0
    for g in range(60):
        n = int(rng.integers(6, 41))
        rows, codes, entry, max_level = TG.random_tie_graph(rng, n)
        path = TG.write_ihnp(str(tmp_path / f"g{g}.index"), rows, codes, entry, max_level)
        fx = faiss_file.read(path)
        q = np.zeros((3, TG.D), dtype=np.float32)
        q[1, 0] = float(rng.integers(1, 12))
        q[2] = rng.standard_normal(TG.D).astype(np.float32)
        for k, ef in ((1, 1), (2, 3), (3, 3), (4, 2), (5, 8), (8, 8)):
            Dl, Il, ndl, nhl = FL.search(fx, q, k, ef)
            Do, Io, ndo, nho = O.hnswpq_search(fx, q, k, ef)
            assert np.array_equal(Il, Io), (g, k, ef)
            assert np.array_equal(Dl.view(np.uint32), Do.view(np.uint32)), (g, k, ef)
            assert np.array_equal(ndl, ndo) and np.array_equal(nhl, nho), (g, k, ef)
            checked += 1
    assert checked == 360


def test_committed_c1_index_fixture(tmp_path):
    """tests/golden/c1_hnswpq.index (the C1 IHNp file committed for a faiss-equipped cross-check,
    tests/golden/make_c1_index.py): a fresh single-threaded build is byte-identical, the committed queries are the
    C1 reads' embeddings, and the committed expected rows are the oracle's (both restatements agree on them)."""
    import os
    import sys
    from conftest import GOLDEN
    sys.path.insert(0, GOLDEN)
    import make_c1_index
    fresh = str(tmp_path / "c1.index")
    q = make_c1_index.build(fresh)
    committed = os.path.join(GOLDEN, "c1_hnswpq.index")
    assert open(fresh, "rb").read() == open(committed, "rb").read()
    assert np.array_equal(np.load(os.path.join(GOLDEN, "c1_queries.npy")), q.astype(np.float32))
    exp = np.load(os.path.join(GOLDEN, "c1_expected_k128_ef128.npz"))
    fx = faiss_file.read(committed)
    Do, Io, _, _ = O.hnswpq_search(fx, q, 128, 128)
    assert np.array_equal(Io, exp["I"]) and np.array_equal(Do.view(np.uint32), exp["D"].view(np.uint32))
    Dl, Il, _, _ = FL.search(fx, q[:6], 128, 128)  # the literal restatement on a few reads (it is slow)
    assert np.array_equal(Il, exp["I"][:6]) and np.array_equal(Dl.view(np.uint32), exp["D"][:6].view(np.uint32))
