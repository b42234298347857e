"""A second, literal restatement of faiss's HNSW-PQ search -- TEST INFRASTRUCTURE ONLY.

faiss is absent here (conda `faiss-cpu`, version unpinned, environment.yml:13); the
reference's call sites are src/main.cpp:236-237,278 and src/hnswpq/search.cpp:13,39-40. oracle/drm_oracle.c
restates the same algorithm in C for speed, with its own data layout. This module follows the upstream code
statement by statement -- arrays, 1-based heap indexing, the same loop order -- so that it can be read side by
side with faiss and checked against hand-derived traces (tests/golden/hnsw_tie_cases.json) without sharing any
code with the C oracle or the HIP kernels. It is slow (pure Python); use it on tiny graphs only.

Upstream faiss >= 1.8 functions restated:
  faiss/utils/Heap.h          heap_pop, heap_push, heap_replace_top, heap_reorder (CMax<float, int>: cmp2)
  faiss/impl/HNSW.cpp         MinimaxHeap::push / pop_min / count_below, greedy_update_nearest,
                              search_from_candidates, HNSW::search (bounded queue branch)
  faiss/impl/ResultHandler.h  HeapBlockResultHandler::SingleResultHandler (begin, add_result, end)
  faiss/IndexPQ.cpp,          PQDistanceComputer (compute_distance_table, distance_to_code: a sequential
  faiss/impl/ProductQuantizer.cpp   fp32 sum over the sub-quantizers starting from 0)
"""
import numpy as np

F32 = np.float32
INF = F32(np.inf)


def cmp2_max(a1, b1, a2, b2):
    """CMax<float, int>::cmp2(a1, b1, a2, b2): (a1 > b1) || (a1 == b1 && a2 > b2)."""
    return (a1 > b1) or (a1 == b1 and a2 > b2)


def heap_pop(k, val, ids):
    """faiss heap_pop<CMax>(k, bh_val, bh_ids) on 0-based lists (written 1-based as upstream)."""
    bv = [None] + val  # bh_val--
    bi = [None] + ids
    v, idv = bv[k], bi[k]
    i = 1
    while True:
        i1 = i << 1
        i2 = i1 + 1
        if i1 > k:
            break
        if i2 == k + 1 or cmp2_max(bv[i1], bv[i2], bi[i1], bi[i2]):
            if cmp2_max(v, bv[i1], idv, bi[i1]):
                break
            bv[i], bi[i] = bv[i1], bi[i1]
            i = i1
        else:
            if cmp2_max(v, bv[i2], idv, bi[i2]):
                break
            bv[i], bi[i] = bv[i2], bi[i2]
            i = i2
    bv[i], bi[i] = bv[k], bi[k]
    val[:] = bv[1:]
    ids[:] = bi[1:]


def heap_push(k, val, ids, v, idv):
    """faiss heap_push<CMax>(k, bh_val, bh_ids, val, id): the new element enters at 1-based k and sifts up."""
    bv = [None] + val
    bi = [None] + ids
    i = k
    while i > 1:
        f = i >> 1
        if not cmp2_max(v, bv[f], idv, bi[f]):
            break
        bv[i], bi[i] = bv[f], bi[f]
        i = f
    bv[i], bi[i] = v, idv
    val[:] = bv[1:]
    ids[:] = bi[1:]


def heap_replace_top(k, val, ids, v, idv):
    """faiss heap_replace_top<CMax>: the root replaced by (v, idv), sifted down."""
    bv = [None] + val
    bi = [None] + ids
    i = 1
    while True:
        i1 = i << 1
        i2 = i1 + 1
        if i1 > k:
            break
        if i2 == k + 1 or cmp2_max(bv[i1], bv[i2], bi[i1], bi[i2]):
            if cmp2_max(v, bv[i1], idv, bi[i1]):
                break
            bv[i], bi[i] = bv[i1], bi[i1]
            i = i1
        else:
            if cmp2_max(v, bv[i2], idv, bi[i2]):
                break
            bv[i], bi[i] = bv[i2], bi[i2]
            i = i2
    bv[i], bi[i] = v, idv
    val[:] = bv[1:]
    ids[:] = bi[1:]


def heap_reorder(k, val, ids):
    """faiss heap_reorder<CMax>: ascending (distance, id), invalid (-1) entries dropped then padded."""
    ii = 0
    for i in range(k):
        v, idv = val[0], ids[0]
        sub_v, sub_i = val[:k - i], ids[:k - i]
        heap_pop(k - i, sub_v, sub_i)
        val[:k - i], ids[:k - i] = sub_v, sub_i
        val[k - ii - 1], ids[k - ii - 1] = v, idv
        if idv != -1:
            ii += 1
    nel = ii
    val[:ii] = val[k - ii:k]
    ids[:ii] = ids[k - ii:k]
    for j in range(ii, k):
        val[j], ids[j] = INF, -1
    return nel


class MinimaxHeap:
    """faiss HNSW::MinimaxHeap (n slots, k used, nvalid not popped)."""

    def __init__(self, n):
        self.n, self.k, self.nvalid = n, 0, 0
        self.ids = [0] * n
        self.dis = [F32(0)] * n

    def push(self, i, v):
        if self.k == self.n:
            if v >= self.dis[0]:
                return
            if self.ids[0] != -1:
                self.nvalid -= 1
            d, ix = self.dis[:self.k], self.ids[:self.k]
            heap_pop(self.k, d, ix)
            self.dis[:self.k], self.ids[:self.k] = d, ix
            self.k -= 1
        self.k += 1
        d, ix = self.dis[:self.k], self.ids[:self.k]
        heap_push(self.k, d, ix, v, i)
        self.dis[:self.k], self.ids[:self.k] = d, ix
        self.nvalid += 1

    def size(self):
        return self.nvalid

    def pop_min(self):
        """The smallest valid slot; among equal minima the highest index (the scan runs downwards and only a
        strictly smaller value replaces the current one). Returns (id, d) or (-1, None)."""
        i = self.k - 1
        while i >= 0:
            if self.ids[i] != -1:
                break
            i -= 1
        if i == -1:
            return -1, None
        imin, vmin = i, self.dis[i]
        i -= 1
        while i >= 0:
            if self.ids[i] != -1 and self.dis[i] < vmin:
                vmin, imin = self.dis[i], i
            i -= 1
        ret = self.ids[imin]
        self.ids[imin] = -1
        self.nvalid -= 1
        return ret, vmin

    def count_below(self, thresh):
        return sum(1 for i in range(self.k) if self.dis[i] < thresh)


class ResultHeap:
    """HeapBlockResultHandler::SingleResultHandler for one query (k results, CMax)."""

    def __init__(self, k):
        self.k = k
        self.dis = [INF] * k  # heap_heapify: all (+inf, -1)
        self.ids = [-1] * k
        self.threshold = self.dis[0]

    def add_result(self, d, i):
        if self.threshold > d:  # C::cmp(threshold, dis)
            heap_replace_top(self.k, self.dis, self.ids, d, i)
            self.threshold = self.dis[0]
            return True
        return False

    def end(self):
        heap_reorder(self.k, self.dis, self.ids)
        return list(self.dis), list(self.ids)


class LiteralIndex:
    """The arrays of an IHNp file as faiss holds them (HNSW offsets / neighbors / levels, PQ codes)."""

    def __init__(self, fx):
        self.ntotal = int(fx.ntotal)
        self.d = int(fx.d)
        self.M = int(fx.pq_M)
        self.ksub = 1 << int(fx.pq_nbits)
        assert int(fx.pq_nbits) == 8, "the literal restatement reads 8-bit codes"
        self.dsub = self.d // self.M
        self.cum = [int(c) for c in fx.cum_nneighbor_per_level]
        self.offsets = [int(o) for o in fx.offsets]
        self.neighbors = [int(v) for v in fx.neighbors]
        self.levels = [int(v) for v in fx.levels]
        self.entry_point = int(fx.entry_point)
        self.max_level = int(fx.max_level)
        self.codes = np.asarray(fx.codes, dtype=np.uint8).reshape(self.ntotal, self.M)
        self.centroids = np.asarray(fx.centroids, dtype=F32).reshape(self.M, self.ksub, self.dsub)

    def neighbor_range(self, no, level):
        o = self.offsets[no]
        return o + self.cum[level], o + self.cum[level + 1]


def distance_table(ix, x):
    """compute_distance_table: LUT[m][c] = sum_t (x[m*dsub + t] - C[m][c][t])^2, sequential fp32, no FMA."""
    lut = np.zeros((ix.M, ix.ksub), dtype=F32)
    for m in range(ix.M):
        xs = np.asarray(x[m * ix.dsub:(m + 1) * ix.dsub], dtype=F32)
        acc = np.zeros(ix.ksub, dtype=F32)
        for t in range(ix.dsub):
            diff = (xs[t] - ix.centroids[m, :, t]).astype(F32)
            acc = (acc + (diff * diff).astype(F32)).astype(F32)
        lut[m] = acc
    return lut


def distance_to_code(ix, lut, node):
    r = F32(0)
    for m in range(ix.M):
        r = F32(r + lut[m, ix.codes[node, m]])
    return r


def greedy_update_nearest(ix, lut, level, nearest, d_nearest, stats):
    while True:
        prev = nearest
        begin, end = ix.neighbor_range(nearest, level)
        ndis = 0
        for j in range(begin, end):  # the 4-wide batching gives the same distances in the same order
            v = ix.neighbors[j]
            if v < 0:
                break
            dis = distance_to_code(ix, lut, v)
            ndis += 1
            if dis < d_nearest:
                nearest, d_nearest = v, dis
        stats["ndis"] += ndis
        stats["nhops"] += 1
        if nearest == prev:
            return nearest, d_nearest


def search_from_candidates(ix, lut, res, candidates, visited, stats, ef_search, level=0):
    threshold = res.threshold
    for i in range(candidates.size()):
        v1, d = candidates.ids[i], candidates.dis[i]
        if d < threshold:
            if res.add_result(d, v1):
                threshold = res.threshold
        visited.add(v1)
    nstep = ndis = 0
    while candidates.size() > 0:
        v0, d0 = candidates.pop_min()
        if candidates.count_below(d0) >= ef_search:  # do_dis_check (check_relative_distance = true)
            break
        begin, end = ix.neighbor_range(v0, level)
        jmax = begin
        for j in range(begin, end):
            if ix.neighbors[j] < 0:
                break
            jmax += 1
        threshold = res.threshold
        fresh = []
        for j in range(begin, jmax):  # vt.get then vt.set for the whole row, then the distances in row order
            v1 = ix.neighbors[j]
            if v1 not in visited:
                fresh.append(v1)
            visited.add(v1)
        for v1 in fresh:
            dis = distance_to_code(ix, lut, v1)
            if dis < threshold:
                if res.add_result(dis, v1):
                    threshold = res.threshold
            candidates.push(v1, dis)
        ndis += len(fresh)
        nstep += 1
    stats["ndis"] += ndis
    stats["nhops"] += nstep


def search_one(ix, x, k, ef_search):
    """IndexHNSW::search for one query: HNSW::search (bounded queue) + HeapBlockResultHandler.
    Returns (D[k], I[k], ndis, nhops)."""
    res = ResultHeap(k)
    stats = {"ndis": 0, "nhops": 0}
    if ix.entry_point == -1:
        d, i = res.end()
        return d, i, 0, 0
    lut = distance_table(ix, x)
    nearest = ix.entry_point
    d_nearest = distance_to_code(ix, lut, nearest)
    for level in range(ix.max_level, 0, -1):
        nearest, d_nearest = greedy_update_nearest(ix, lut, level, nearest, d_nearest, stats)
    ef = max(ef_search, k)
    candidates = MinimaxHeap(ef)
    candidates.push(nearest, d_nearest)
    search_from_candidates(ix, lut, res, candidates, set(), stats, ef_search)
    d, i = res.end()
    return d, i, stats["ndis"], stats["nhops"]


def search(fx, q, k, ef_search):
    ix = LiteralIndex(fx)
    n = len(q)
    D = np.empty((n, k), dtype=F32)
    I = np.empty((n, k), dtype=np.int64)
    nd = np.empty(n, dtype=np.int64)
    nh = np.empty(n, dtype=np.int64)
    for r in range(n):
        d, i, nd[r], nh[r] = search_one(ix, q[r], k, ef_search)
        D[r], I[r] = d, i
    return D, I, nd, nh
