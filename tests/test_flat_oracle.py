"""CPU tests of the fp32-L2 (hnswlib) path: the oracle restatement (oracle/hnswlib_oracle.cpp),
hnswlib's 8-accumulator L2 order, the hnswlib file written by our builder, and exhaustive search
against brute force. Parity of hnswlib itself is unpinned (the submodule is absent
and unpinned); these tests pin the restatement's own invariants."""
import numpy as np

from oracle import oracle as O


def _l2_avx_numpy(x, y):
    acc = [np.float32(0)] * 8
    for j in range(0, x.size, 8):
        for i in range(8):
            t = np.float32(x[j + i] - y[j + i])
            acc[i] = np.float32(acc[i] + np.float32(t * t))
    r = acc[0]
    for i in range(1, 8):
        r = np.float32(r + acc[i])
    return r


def test_l2_order_matches_float32_emulation():
    rng = np.random.default_rng(3)
    for _ in range(50):
        x = rng.standard_normal(128).astype(np.float32)
        y = rng.standard_normal(128).astype(np.float32)
        assert np.float32(O.l2_avx(x, y)).view(np.uint32) == _l2_avx_numpy(x, y).view(np.uint32)


def test_hnswlib_file_structure(c1_flat):
    fx = c1_flat["fx"]
    assert fx["d"] == 128 and fx["n"] == c1_flat["x"].shape[0]
    assert fx["maxM0"] == 128 and fx["maxM"] == 64 and fx["M"] == 64
    assert np.array_equal(fx["vec"], c1_flat["x"])
    assert np.array_equal(fx["labels"], np.arange(fx["n"], dtype=np.uint64))
    cnt = fx["l0"][:, 0] & 0xFFFF
    assert (cnt <= 128).all() and (cnt > 0).all()
    assert fx["levels"][fx["ep"]] == fx["maxlevel"]


def _reachable(fx):
    n, cnt = fx["n"], fx["l0"][:, 0] & 0xFFFF
    seen = np.zeros(n, bool)
    stack = [fx["ep"]]
    seen[fx["ep"]] = True
    while stack:
        v = stack.pop()
        for u in fx["l0"][v, 1:1 + cnt[v]]:
            if not seen[u]:
                seen[u] = True
                stack.append(u)
    return seen


def test_exhaustive_search_equals_brute_force(syn_flat):
    """ef >= ntotal: while top_candidates is not full every discovered node is in it, so the stop
    rule never fires and the search visits the whole level-0 component of the entry point (pruning
    can strand a few nodes, as in hnswlib). The result is the exact top-k by (distance, label) over
    that component under the restated L2."""
    fx = syn_flat["fx"]
    n = fx["n"]
    reach = np.flatnonzero(_reachable(fx))
    q = syn_flat["q"][:6]
    D, I, nd, nh = O.hnswlib_search(fx, q, 20, n + 10)
    for i in range(len(q)):
        d = np.array([O.l2_avx(q[i], fx["vec"][j]) for j in reach], dtype=np.float32)
        order = reach[np.lexsort((reach, d))[:20]]
        dd = np.array([O.l2_avx(q[i], fx["vec"][j]) for j in range(n)], dtype=np.float32)
        # distances are exact; labels are exact below the cutoff distance, and at the cutoff (a tie
        # trimmed by top_candidates.pop(), i.e. by heap layout) they come from the tied group
        assert np.array_equal(D[i].view(np.uint32), dd[order].view(np.uint32))
        cut = D[i][-1]
        below = D[i] < cut
        assert I[i][below].tolist() == order[dd[order] < cut].tolist()
        tied = set(reach[d == cut].tolist())
        assert set(I[i][~below].tolist()) <= tied
