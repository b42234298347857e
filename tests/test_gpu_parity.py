"""GPU parity tests: the HIP path (through the C ABI) vs the oracle restatement and the golden
vectors. Integer work (SW scores, top-k ids, ndis/nhops) must be bit-exact; fp32 distances are
bit-exact too because kernel and oracle use the same op order (tolerance: 0 ulp)."""
import json
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, ROOT, read_fastq_tagged
from oracle import oracle as O

pytestmark = pytest.mark.gpu


# ------------------------------------------------------------------------------------------ SW
def test_sw_kat_gpu():
    from deepreadmapper_amd import calc_sw_scores
    kat = json.load(open(os.path.join(GOLDEN, "sw_kat.json")))
    quer = [l.strip() for l in open(os.path.join(GOLDEN, "test_data_quer.txt")).read().splitlines() if l.strip()]
    got = calc_sw_scores([quer[i] for i, _ in kat["harness_pairs"]], [quer[j] for _, j in kat["harness_pairs"]])
    assert got.tolist() == kat["harness_scores"]
    for group in ("edge_cases", "random_pairs"):
        pairs = kat[group]
        got = calc_sw_scores([a for a, _, _ in pairs], [b for _, b, _ in pairs])
        assert got.tolist() == [s for _, _, s in pairs], group


def _c1_refs():
    return np.frombuffer(b"".join(l.strip() for l in open(os.path.join(GOLDEN, "test_data_ref.txt"), "rb")
                                  if l.strip()), dtype=np.uint8).reshape(1702, 150)


def test_sw_c1_matrix_through_rerank_kernel():
    """Every read of test_data.fastq against every window, through the rerank kernel (k = all
    candidates), equals the reference-built matrix in the libstdc++ partial_sort order."""
    from deepreadmapper_amd import WindowTable, rerank_arrays
    mat = np.load(os.path.join(GOLDEN, "sw_c1_matrix.npy")).astype(np.int32)
    reads = read_fastq_tagged(os.path.join(GOLDEN, "test_data.fastq"))
    table = WindowTable(_c1_refs())
    for lo, hi in ((0, 1000), (1000, 1702)):
        nb = np.tile(np.arange(lo, hi, dtype=np.int64), (len(reads), 1))
        sc, ids, cnt = rerank_arrays(table, nb, reads, 1, hi - lo, hi - lo)
        assert (cnt == hi - lo).all()
        for i in range(len(reads)):
            order = O.stl_partial_sort_desc(mat[i, lo:hi], hi - lo)
            assert ids[i].astype(np.int64).tolist() == (order + lo).tolist()
            assert sc[i].tolist() == mat[i, lo:hi][order].tolist()


def _rerank_both(refs, nb, reads, stride, k, kc):
    from deepreadmapper_amd import WindowTable, rerank_arrays
    from deepreadmapper_amd.rerank import pack_queries
    qbuf, ql = pack_queries(reads)
    rc, sc_o, id_o, cnt_o = O.post_process_sw_static(nb, refs, refs.shape[1], qbuf, ql, stride, k, kc)
    assert rc == 0
    sc, ids, cnt = rerank_arrays(WindowTable(refs), nb, (qbuf, ql), stride, k, kc)
    assert np.array_equal(cnt, cnt_o)
    for i in range(len(nb)):
        n = cnt[i]
        assert np.array_equal(sc[i, :n], sc_o[i, :n]) and np.array_equal(ids[i, :n], id_o[i, :n]), i


def test_rerank_dense_vs_oracle(c1):
    D, I, _, _ = O.hnswpq_search(c1["fx"], c1["q"], 128, 128)
    _rerank_both(c1["refs"], I, c1["reads"], 1, 128, 128)
    _rerank_both(c1["refs"], I, c1["reads"], 1, 10, 40)  # k < k_clusters


def test_rerank_many_distinct_bytes(c1):
    """Queries over a 40-letter alphabet (more than 15 distinct bytes) take the bit-profile kernel,
    short/ragged DNA queries the fp16 class-profile kernel; both must equal the oracle, in one batch."""
    rng = np.random.default_rng(21)
    refs = rng.integers(33, 73, size=(300, 150)).astype(np.uint8)
    refs[::3] = c1["refs"][:100]  # some DNA windows too
    reads = []
    for i in range(80):
        if i % 2:
            reads.append(bytes(rng.integers(33, 73, size=int(rng.integers(1, 153))).astype(np.uint8)))
        else:
            r = c1["reads"][i]
            reads.append(r[: int(rng.integers(1, len(r) + 1))])
    nb = rng.integers(0, 300, size=(80, 24)).astype(np.int64)
    _rerank_both(refs, nb, reads, 1, 24, 24)
    _rerank_both(refs, nb, reads, 1, 5, 20)


def test_rerank_nonacgt_query_ends(c1):
    """The fp16/int class-profile kernel drops leading and trailing non-ACGT query bytes (the "<" ">" tags) from
    its DP: reads with such ends of every shape -- tags, runs of N, a read of tags only, 150 / 151 / 152 DNA bytes
    (more than 150 columns go to the bit-profile kernel) -- against windows with N runs and with "<" / ">" bytes
    (which must flag the query, since they match its tags) equal the oracle."""
    rng = np.random.default_rng(33)
    refs = c1["refs"][:240].copy()
    refs[10:20, 40:45] = ord("N")
    refs[30, 0] = ord("<")
    refs[31, 149] = ord(">")
    refs[32, 70] = ord(">")
    dna = lambda n: bytes(rng.choice(np.frombuffer(b"ACGT", np.uint8), size=n).astype(np.uint8))
    reads = []
    for i in range(96):
        body = c1["reads"][i % len(c1["reads"])][1:-1] if i % 3 else dna(int(rng.integers(1, 151)))
        pre = [b"<", b"", b"N", b"NN<", b"<N", b"X<"][i % 6]
        post = [b">", b"", b"N", b">>", b"N>", b">X"][(i // 6) % 6]
        reads.append(pre + body[: 150 - len(pre) - len(post) + 2] + post if len(pre + body + post) > 152 else
                     pre + body + post)
    reads += [b"<>", b"<NN>", b"N", dna(150), dna(151), dna(152), b"<" + dna(150), dna(150) + b">", b"<" + dna(150) + b">"]
    assert max(map(len, reads)) <= 152
    n = len(reads)
    nb = rng.integers(0, len(refs), size=(n, 24)).astype(np.int64)
    nb[:, 0] = 30 + np.arange(n) % 3  # the windows with tag bytes in every list
    _rerank_both(refs, nb, reads, 1, 24, 24)


@pytest.mark.parametrize("stride", [2, 3, 4])
def test_rerank_sparse_vs_oracle(c1, stride):
    rng = np.random.default_rng(stride)
    nb = rng.integers(-1, 1702 // stride + 40, size=(60, 8)).astype(np.int64)
    _rerank_both(c1["refs"], nb, c1["reads"][:60], stride, 5, 5)


def test_rerank_errors(c1):
    from deepreadmapper_amd import WindowTable, rerank_arrays, DrmError, post_process_sw_static
    from deepreadmapper_amd._native import DRM_ERR_CANDS, DRM_ERR_K
    t = WindowTable(c1["refs"])
    nb = np.arange(8, dtype=np.int64)[None]
    with pytest.raises(DrmError) as e:
        rerank_arrays(t, nb, c1["reads"][:1], 1, 17, 8)
    assert e.value.code == DRM_ERR_K
    nb2 = np.array([[0, 1, -1, 5, 99999]], dtype=np.int64)
    with pytest.raises(DrmError) as e:
        rerank_arrays(t, nb2, c1["reads"][:1], 1, 4, 5)
    assert e.value.code == DRM_ERR_CANDS and "Not enough candidates (3 < 4)" in str(e.value)
    sc, ids, cnt = rerank_arrays(t, np.full((2, 5), -1, np.int64), c1["reads"][:2], 1, 4, 5)
    assert cnt.tolist() == [0, 0]
    with pytest.raises(RuntimeError, match="Not enough candidates"):
        post_process_sw_static(nb2, None, list(map(bytes, c1["refs"])), c1["reads"][:1], 150, 1, 4, 5)


def test_sw_reranker_api():
    from deepreadmapper_amd import sw_reranker
    cands = ["ACGTACGTAA", "TTTT", "ACGTACGTAC", "ACG", "ACGTACGTAC"]
    seqs, scores, ids = sw_reranker(cands, [10, 11, 12, 13, 14], "<ACGTACGTAC>", 3)
    exp_scores = [O.calc_sw_score(c.encode(), b"<ACGTACGTAC>") for c in cands]
    order = O.stl_partial_sort_desc(np.array(exp_scores, np.int32), 3).tolist()
    assert ids == [[10, 11, 12, 13, 14][i] for i in order] and scores == [exp_scores[i] for i in order]
    with pytest.raises(RuntimeError, match="Not enough candidates"):
        sw_reranker(cands, [1, 2, 3, 4, 5], "ACGT", 6)


# ------------------------------------------------------------------------------------------ search
def _search_both(index_path, fx, q, k, ef):
    """The default search (ids, 0-ulp distances, nhops) and the exact-statistics search (the same, plus faiss's
    ndis) against the oracle."""
    from deepreadmapper_amd import read_index
    ix = read_index(index_path)
    D, I, st = ix.search(q, k, ef)
    Do, Io, nd, nh = O.hnswpq_search(fx, q, k, ef)
    assert np.array_equal(I, Io)
    assert np.array_equal(D.view(np.uint32), Do.view(np.uint32))  # 0-ulp fp32
    assert st.nhops == int(nh.sum())
    ix.set_exact_stats(True)
    D2, I2, st2 = ix.search(q, k, ef)
    assert np.array_equal(I2, Io) and np.array_equal(D2.view(np.uint32), Do.view(np.uint32))
    assert st2.ndis == int(nd.sum()) and st2.nhops == int(nh.sum())
    ix.free()
    return D, I


@pytest.mark.parametrize("k,ef", [(128, 128), (5, 128), (10, 16), (1, 1), (200, 64), (64, 300)])
def test_search_c1_bitexact(c1, k, ef):
    _search_both(c1["index"], c1["fx"], c1["q"], k, ef)


def test_search_c1_random_and_exhaustive(c1):
    rng = np.random.default_rng(9)
    q = rng.standard_normal((64, 128)).astype(np.float32)
    _search_both(c1["index"], c1["fx"], q, 32, 96)
    _search_both(c1["index"], c1["fx"], c1["q"][:40], 50, 2048)  # ef >= ntotal


def test_search_syn20k_bitexact(syn20k):
    w = syn20k["w"]
    _search_both(syn20k["index"], syn20k["fx"], w.q_emb, 128, 128)


def test_search_heap_visited_repeated_launches(syn20k):
    """The lean kernel keeps no visited table (its heap is the visited set): nothing carries over between queries
    or launches. A small grid (1 wave per CU, ~80 queries per slot), repeated launches on one handle, K = 128 / K = 5
    interleaved and the exact-statistics mode switched on and off between them all give the oracle's results."""
    from deepreadmapper_amd import read_index
    from deepreadmapper_amd._native import check, lib
    w, fx = syn20k["w"], syn20k["fx"]
    q = w.q_emb
    ix = read_index(syn20k["index"])
    check(lib().drm_index_set_search_waves(ix.handle, 1))
    Do, Io, nd, nh = O.hnswpq_search(fx, q, 128, 128)
    D5o, I5o, nd5, nh5 = O.hnswpq_search(fx, q, 5, 128)
    for stats in (False, True, False):
        ix.set_exact_stats(stats)
        for _ in range(2):
            D, I, st = ix.search(q, 128, 128)
            bad = np.flatnonzero((I != Io).any(axis=1))
            assert bad.size == 0, f"stats={stats}: {bad.size} rows differ, first {bad[:8]}"
            assert np.array_equal(D.view(np.uint32), Do.view(np.uint32))
            assert st.nhops == int(nh.sum()) and (not stats or st.ndis == int(nd.sum()))
            D5, I5, st5 = ix.search(q, 5, 128)
            assert np.array_equal(I5, I5o) and np.array_equal(D5.view(np.uint32), D5o.view(np.uint32))
            assert st5.nhops == int(nh5.sum()) and (not stats or st5.ndis == int(nd5.sum()))
    check(lib().drm_index_set_search_waves(ix.handle, 0))
    D, I, st = ix.search(q, 128, 128)
    assert np.array_equal(I, Io) and st.nhops == int(nh.sum())
    ix.free()


@pytest.mark.parametrize("fast", ["1", "0"])
def test_search_tie_fixtures(tmp_path, fast, monkeypatch):
    """The hand-derived traversal fixtures (tests/golden/hnsw_tie_cases.json: pop_min among equal minima, the
    v >= dis[0] rejection at equality, result insertion order among equal distances, a duplicate link, upper-level
    ties) through the lean kernel (default and exact statistics) and the general kernel (DRM_SEARCH_FAST=0); then 40
    random tie-heavy graphs against the C oracle."""
    import tie_graphs as TG
    from deepreadmapper_amd import read_index
    from oracle import faiss_file
    monkeypatch.setenv("DRM_SEARCH_FAST", fast)
    q = np.zeros((1, TG.D), dtype=np.float32)
    for case in TG.load_cases():
        ix = read_index(TG.write_case(case, str(tmp_path)))
        e = case["expected"]
        for stats in (False, True):
            ix.set_exact_stats(stats)
            D, I, st = ix.search(q, case["k"], case["ef"])
            assert I[0].tolist() == e["I"] and D[0].tolist() == e["D"], (case["name"], stats)
            assert st.nhops == e["nhops"], case["name"]
            if stats or fast == "0":
                assert st.ndis == e["ndis"], case["name"]
        ix.free()
    rng = np.random.default_rng(77)
    for g in range(40):
        rows, codes, entry, max_level = TG.random_tie_graph(rng, int(rng.integers(6, 41)))
        path = TG.write_ihnp(str(tmp_path / f"r{g}.index"), rows, codes, entry, max_level)
        fx = faiss_file.read(path)
        qq = np.zeros((3, TG.D), dtype=np.float32)
        qq[1, 0] = float(rng.integers(1, 12))
        qq[2] = rng.standard_normal(TG.D).astype(np.float32)
        ix = read_index(path)
        ix.set_exact_stats(True)
        for k, ef in ((1, 1), (2, 3), (3, 3), (4, 2), (5, 8), (8, 8)):
            D, I, st = ix.search(qq, k, ef)
            Do, Io, nd, nh = O.hnswpq_search(fx, qq, k, ef)
            assert np.array_equal(I, Io) and np.array_equal(D.view(np.uint32), Do.view(np.uint32)), (g, k, ef)
            assert st.ndis == int(nd.sum()) and st.nhops == int(nh.sum()), (g, k, ef)
        ix.free()


def test_search_committed_c1_fixture():
    """The committed C1 IHNp file and queries (tests/golden/make_c1_index.py) give the committed expected rows."""
    from deepreadmapper_amd import read_index
    exp = np.load(os.path.join(GOLDEN, "c1_expected_k128_ef128.npz"))
    ix = read_index(os.path.join(GOLDEN, "c1_hnswpq.index"))
    D, I, st = ix.search(np.load(os.path.join(GOLDEN, "c1_queries.npy")), 128, 128)
    ix.free()
    assert np.array_equal(I, exp["I"]) and np.array_equal(D.view(np.uint32), exp["D"].view(np.uint32))


@pytest.mark.parametrize("k,ef", [(128, 128), (16, 64), (100, 128)])
def test_search_ties_exact_kernel(repeats, k, ef, monkeypatch):
    """Repeated genome segments give identical PQ codes: the general exact kernel (DRM_SEARCH_FAST=0) replays
    faiss's heap layout through the ties and equals the oracle."""
    monkeypatch.setenv("DRM_SEARCH_FAST", "0")
    _search_both(repeats["index"], repeats["fx"], repeats["q"], k, ef)


@pytest.mark.parametrize("fast", ["1", "0"])
@pytest.mark.parametrize("k,ef", [(128, 128), (64, 64), (5, 128), (16, 100), (100, 100), (32, 32)])
def test_search_lean_and_exact_kernels_ties(repeats, k, ef, fast, monkeypatch):
    """The lean kernel (hnsw_pq_fast.hip: packed-u64 pair heap, logged result set at k == ef,
    register result set at k <= 64) and the general exact kernel (DRM_SEARCH_FAST=0) on the
    tie-heavy index: both bit-identical to the oracle."""
    monkeypatch.setenv("DRM_SEARCH_FAST", fast)
    _search_both(repeats["index"], repeats["fx"], repeats["q"], k, ef)


def test_search_lean_kernel_log_compaction(syn20k, repeats, monkeypatch):
    """The smallest log capacity (ef + max(ef, 64)) forces the in-place compaction of the log of tied
    evictions on the tie-heavy index (and before the heap's entries join it at the end): still bit-identical."""
    monkeypatch.setenv("DRM_SEARCH_LOG_CAP", "1")  # clamped to ef + max(ef, 64)
    w = syn20k["w"]
    _search_both(syn20k["index"], syn20k["fx"], w.q_emb[:600], 128, 128)
    _search_both(repeats["index"], repeats["fx"], repeats["q"], 96, 96)


def test_search_syn20k_exact_kernel(syn20k, monkeypatch):
    monkeypatch.setenv("DRM_SEARCH_FAST", "0")
    w = syn20k["w"]
    _search_both(syn20k["index"], syn20k["fx"], w.q_emb, 128, 128)


@pytest.mark.parametrize("kernel", ["lean", "exact", "lds", "flat"])
def test_search_bounds_fail_loudly(syn20k, c1_flat, kernel, monkeypatch):
    """Every search kernel family bounds its loops: lowered through the load-time knobs, a
    query past the level-0 hop bound (DRM_SEARCH_HOP_BOUND) and a persistent wave past its work-item bound
    (DRM_WAVE_ITEM_BOUND) end with DRM_ERR_INTERNAL from the search instead of looping; the default bounds (ntotal
    hops, n items) never trigger."""
    from deepreadmapper_amd import HnswFlatIndex, read_index
    from deepreadmapper_amd._native import DrmError
    monkeypatch.setenv("DRM_SEARCH_FAST", "0" if kernel == "exact" else "1")
    monkeypatch.setenv("DRM_SEARCH_LDS_KERNEL", "1" if kernel == "lds" else "0")
    if kernel == "flat":
        path, q = c1_flat["index"], c1_flat["q"]
        load = lambda: HnswFlatIndex(path)  # noqa: E731
    else:
        path, q = syn20k["index"], syn20k["w"].q_emb
        load = lambda: read_index(path)  # noqa: E731
    q = np.ascontiguousarray(np.resize(q, (12_000, q.shape[1])))  # more queries than resident waves
    ix = load()
    ix.search(q, 32, 64)  # the natural bounds: no error
    ix.free()
    for knob, val in (("DRM_SEARCH_HOP_BOUND", "2"), ("DRM_WAVE_ITEM_BOUND", "1")):
        monkeypatch.setenv(knob, val)
        ix = load()
        with pytest.raises(DrmError) as e:
            ix.search(q, 32, 64)
        assert e.value.code == -8, str(e.value)  # DRM_ERR_INTERNAL
        assert ix.search_errors() == 0  # reported once, then reset
        ix.free()
        monkeypatch.delenv(knob)


def test_search_device_stats(syn20k):
    from deepreadmapper_amd import read_index
    from deepreadmapper_amd.device import DeviceBuffer, synchronize
    w = syn20k["w"]
    q = w.q_emb[:500]
    ix = read_index(syn20k["index"])
    ix.set_exact_stats(True)  # ndis as faiss counts it (the default mode reports the distances computed)
    dq = DeviceBuffer.from_host(q)
    dD, dI = DeviceBuffer((500, 128), np.float32), DeviceBuffer((500, 128), np.int64)
    nd, nh = DeviceBuffer(500, np.int32), DeviceBuffer(500, np.int32)
    ix.search_device(dq, 500, 128, 128, dD, dI, nd, nh)
    synchronize()
    Do, Io, ndo, nho = O.hnswpq_search(syn20k["fx"], q, 128, 128)
    assert np.array_equal(dI.download(), Io) and np.array_equal(nd.download(), ndo)
    assert np.array_equal(nh.download(), nho)


def test_faiss_search_api(c1):
    from deepreadmapper_amd import faiss_search, read_index
    ix = read_index(c1["index"])
    ids, dists = faiss_search(ix, c1["q"][:3].tolist(), 7, 32)
    assert len(ids) == 3 and all(len(r) == 7 for r in ids) and len(dists[0]) == 7
    with pytest.raises(RuntimeError, match="Query data is empty"):
        faiss_search(ix, [], 7, 32)


# ------------------------------------------------------------------------------------------ CLI
def test_pipeline_cli_c1(tmp_path, c1):
    """bin/hnswpq_index + bin/pipeline on the C1 fixture: indices/distances.npy equal the oracle's
    faiss search, sw_scores/sw_ids equal the oracle's post_process_sw_static."""
    fna = os.path.join(GOLDEN, "ecoli_150.fna")
    fq = os.path.join(GOLDEN, "test_data.fastq")
    env = dict(os.environ, DRM_BUILD_THREADS="1")
    r = subprocess.run([os.path.join(ROOT, "bin", "hnswpq_index"), fna, "c1", "150"], cwd=tmp_path, env=env,
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([os.path.join(ROOT, "bin", "pipeline"), "c1", fq, fna, "128", "128", "5", "out"],
                       cwd=tmp_path, capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    I = np.load(tmp_path / "out" / "indices.npy")
    D = np.load(tmp_path / "out" / "distances.npy")
    assert I.dtype == np.dtype("<u8") and D.dtype == np.dtype("<f4") and I.shape == (150, 128)
    hdr = open(tmp_path / "out" / "indices.npy", "rb").read(128)
    assert hdr.startswith(b"\x93NUMPY\x01\x00") and b"{'descr': '<u8', 'fortran_order': False, 'shape': (150, 128), }" in hdr
    from oracle import faiss_file
    from deepreadmapper_amd import synth
    fx = faiss_file.read(str(tmp_path / "c1" / "c1.index"))
    q = synth.embed(c1["reads"])
    Do, Io, _, _ = O.hnswpq_search(fx, q, 128, 128)
    assert np.array_equal(I.astype(np.int64), Io) and np.array_equal(D, Do)
    from deepreadmapper_amd.rerank import pack_queries
    qbuf, ql = pack_queries(c1["reads"])
    rc, sc_o, id_o, cnt_o = O.post_process_sw_static(Io, c1["refs"], 150, qbuf, ql, 1, 128, 128)
    assert np.array_equal(np.load(tmp_path / "out" / "sw_scores.npy"), sc_o)
    assert np.array_equal(np.load(tmp_path / "out" / "sw_ids.npy"), id_o)
    # the opt-in banded SW through the CLI (DRM_SW_BAND, not parity with the reference): the banded oracle's rows
    r = subprocess.run([os.path.join(ROOT, "bin", "pipeline"), "c1", fq, fna, "128", "128", "5", "out16"],
                       cwd=tmp_path, env=dict(os.environ, DRM_SW_BAND="16"), capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    rc, sc_b, id_b, _ = O.post_process_sw_static(Io, c1["refs"], 150, qbuf, ql, 1, 128, 128, band=16)
    assert np.array_equal(np.load(tmp_path / "out16" / "sw_scores.npy"), sc_b)
    assert np.array_equal(np.load(tmp_path / "out16" / "sw_ids.npy"), id_b)
    assert not np.array_equal(sc_b, sc_o)  # the band is in effect
    r = subprocess.run([os.path.join(ROOT, "bin", "pipeline"), "nope", fq, fna], cwd=tmp_path,
                       capture_output=True, text=True)
    assert r.returncode == 1 and r.stderr.startswith("Error: Config file does not exist")
