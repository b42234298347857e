"""L2 rerank oracle (post_process_l2_static -> batch_reranker -> calc_l2_dist, the reference's live
post-processing at src/main.cpp:330), CPU only.

Pins:
* calc_l2_dist: the oracle's restatement of the reference's g++ -O3 -march=native schedule (vector body
  of rounded squares added in order, fused scalar tail) equals the reference's own metrics.cpp compiled
  with -mavx2 -mfma (oracle/_ref) bit for bit for every d; at d % 4 == 0 (the model's 128) that is the
  unfused order the GPU kernel uses; an all-fused chain differs in the last bits only;
* the ascending std::partial_sort replay equals the host libstdc++'s std::partial_sort on tie-heavy inputs;
* the candidate-list semantics, against a pure-Python walk of the reference's data flow (all labels
  flattened, find_sequences' expansion stream, query boundaries of kk*stride per query)."""
import numpy as np
import pytest

from oracle import oracle as O


def test_l2_dist_matches_reference_build():
    if not O.ref_available() or not hasattr(O.ref(), "ref_calc_l2_dist"):
        pytest.skip("oracle/_ref not built (reference sources absent)")
    rng = np.random.default_rng(5)
    diffs = 0
    for t in range(400):
        d = 128 if t % 4 else int(rng.integers(1, 300))
        a = rng.standard_normal(d).astype(np.float32)
        b = (a + rng.standard_normal(d).astype(np.float32) * 0.1).astype(np.float32)
        r = O.ref_calc_l2_dist(a, b)
        assert O.calc_l2_dist(a, b, mode=2) == r
        if d % 4 == 0:
            assert O.calc_l2_dist(a, b, mode=0) == r
        fused = O.calc_l2_dist(a, b, mode=1)
        diffs += fused != r
        assert abs(fused - r) <= 1e-6 * max(r, 1e-30)
    assert diffs > 0  # fused and unfused orders are distinguishable, so the pin above is not vacuous


@pytest.mark.parametrize("n,k", [(1, 1), (7, 3), (128, 128), (128, 50), (300, 128), (1000, 1)])
def test_partial_sort_asc_matches_libstdcxx(n, k):
    rng = np.random.default_rng(n * 31 + k)
    for trial in range(5):
        vals = rng.integers(0, 6 if trial % 2 else 1000, size=n).astype(np.float32) * 0.25
        assert list(O.partial_sort_asc_f32(vals, k)) == list(O.stl_partial_sort_asc_f32(vals, k))


def _py_reference(emb, nb, qe, stride, k_clusters):
    """The reference's post_process_l2_static data flow, step by step (post_processor.cpp:1023-1162)."""
    n_ref = emb.shape[0]
    flat = [int(x) & (2**64 - 1) for x in nb.reshape(-1)]
    if stride == 1:
        valid = [(i, x) for i, x in enumerate(flat) if x < n_ref]
        results = [x for _, x in valid]
        mapping = [i for i, _ in valid]
        dense_ids = results
    else:
        order, seen, mapping = [], {}, []
        for x in flat:
            act = (x * stride) & (2**64 - 1)
            if act >= n_ref:
                continue
            for pos in range(act - stride + 1 if act >= stride - 1 else 0, min(act + stride, n_ref)):
                if pos not in seen:
                    seen[pos] = len(order)
                    order.append(pos)
                mapping.append(seen[pos])
        results = dense_ids = order
    if any(m >= len(results) for m in mapping):
        return "invalid"
    per = nb.shape[1] * (stride if stride > 1 else 1)
    out = []
    for q in range(nb.shape[0]):
        lo, hi = q * per, (q + 1) * per
        if hi > len(mapping):
            return "invalid"
        if per < k_clusters:
            return "short"
        cand = [dense_ids[mapping[i]] for i in range(lo, hi)]
        d = np.array([O.calc_l2_dist(emb[c], qe[q]) for c in cand], dtype=np.float32)
        idx = O.stl_partial_sort_asc_f32(d, k_clusters)
        out.append(([float(d[i]) for i in idx], [cand[i] for i in idx]))
    return out


@pytest.mark.parametrize("stride,kk,kc", [(1, 16, 16), (1, 16, 5), (3, 8, 8), (4, 6, 20)])
def test_oracle_l2_static_semantics(stride, kk, kc):
    rng = np.random.default_rng(stride * 100 + kk)
    n_ref, d, nq = 200, 16, 12
    emb = rng.integers(-3, 4, size=(n_ref, d)).astype(np.float32)  # small integers: many exact ties
    qe = rng.integers(-3, 4, size=(nq, d)).astype(np.float32)
    hi = n_ref if stride == 1 else n_ref // stride + 2  # sparse labels near the end get clipped / dropped
    nb = rng.integers(0, hi, size=(nq, kk)).astype(np.int64)
    nb[0, 0] = nb[0, 1]  # duplicate label -> exact tie
    rc, dists, ids, status = O.post_process_l2_static(emb, nb, qe, stride, kc)
    want = _py_reference(emb, nb, qe, stride, kc)
    if want == "invalid":
        assert rc < 0 and (status == -4).any()
        return
    assert rc == 0 and (status == kc).all()
    for q, (wd, wi) in enumerate(want):
        assert list(dists[q]) == wd
        assert [int(x) for x in ids[q]] == wi


def test_oracle_l2_static_errors():
    emb = np.zeros((10, 8), np.float32)
    qe = np.zeros((2, 8), np.float32)
    nb = np.array([[1, 2, 3], [4, -1, 5]], np.int64)
    rc, _, _, status = O.post_process_l2_static(emb, nb, qe, 1, 3)
    assert rc == -2 and list(status) == [3, -4]  # label -1 is size_t max: the reference throws / over-reads
    rc, _, _, status = O.post_process_l2_static(emb, nb[:1], qe[:1], 1, 4)
    assert rc == -(1 + 1 + 0) and list(status) == [-1]  # 3 candidates < k_clusters = 4
