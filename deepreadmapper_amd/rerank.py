"""Smith-Waterman rerank: drop-ins for calc_sw_score (src/utils/metrics.cpp:10-45), sw_reranker
(src/utils/reranker.cpp:3-51) and post_process_sw_static (src/utils/post_processor.cpp:454-549).
All scoring runs in the HIP kernels of libdrm_hip.so."""
import ctypes as C

import numpy as np

from ._native import DrmError, DRM_ERR_CANDS, check, lib, ptr


def _as_bytes(s):
    return s.encode() if isinstance(s, str) else bytes(s)


def calc_sw_scores(seqs1, seqs2):
    """Batched calc_sw_score(seqs1[p], seqs2[p])."""
    a = [_as_bytes(s) for s in seqs1]
    b = [_as_bytes(s) for s in seqs2]
    if len(a) != len(b):
        raise ValueError("length mismatch")
    n = len(a)
    if n == 0:
        return np.zeros(0, dtype=np.int32)
    buf1 = np.frombuffer(b"".join(a) or b"\0", dtype=np.uint8).copy()
    buf2 = np.frombuffer(b"".join(b) or b"\0", dtype=np.uint8).copy()
    l1 = np.array([len(s) for s in a], dtype=np.int32)
    l2 = np.array([len(s) for s in b], dtype=np.int32)
    o1 = np.concatenate([[0], np.cumsum(l1[:-1], dtype=np.int64)]).astype(np.int64)
    o2 = np.concatenate([[0], np.cumsum(l2[:-1], dtype=np.int64)]).astype(np.int64)
    out = np.empty(n, dtype=np.int32)
    check(lib().drm_sw_scores(ptr(buf1), ptr(o1), ptr(l1), ptr(buf2), ptr(o2), ptr(l2), n, ptr(out)))
    return out


def calc_sw_score(seq1, seq2):
    return int(calc_sw_scores([seq1], [seq2])[0])


class _SwBand:
    """The opt-in banded SW of a window / genome handle (drm_refs_set_sw_band): 0 = the reference's full DP
    (default, bit-exact); 8, 16 or 32 = only the cells |i - j| <= band (non-parity, see include/drm_hip.h)."""

    @property
    def sw_band(self):
        b = C.c_int32(0)
        check(lib().drm_refs_get_sw_band(self._h, C.byref(b)))
        return b.value

    @sw_band.setter
    def sw_band(self, band):
        check(lib().drm_refs_set_sw_band(self._h, int(band)))


class WindowTable(_SwBand):
    """Device-resident `ref_seqs` (static lookup table of equal-length windows)."""

    def __init__(self, windows, device=0):
        if isinstance(windows, np.ndarray):
            arr = np.ascontiguousarray(windows, dtype=np.uint8)
        else:
            ws = [_as_bytes(w) for w in windows]
            L = len(ws[0]) if ws else 0
            if any(len(w) != L for w in ws):
                raise ValueError("static window table needs equal-length windows")
            arr = np.frombuffer(b"".join(ws), dtype=np.uint8).reshape(len(ws), L) if ws else np.zeros((0, 0), np.uint8)
        self.n_ref, self.ref_len = arr.shape
        h = C.c_void_p()
        check(lib().drm_refs_create(ptr(arr) if arr.size else None, self.n_ref, self.ref_len, self.ref_len,
                                    int(device), C.byref(h)))
        self._h = h.value

    @property
    def handle(self):
        return self._h

    def free(self):
        if self._h:
            check(lib().drm_refs_free(self._h))
            self._h = None

    def __del__(self):
        try:
            if getattr(self, "_h", None):
                lib().drm_refs_free(self._h)
        except Exception:
            pass


class GenomeTable(_SwBand):
    """Device-resident genome string for the dynamic lookup (use_dynamic): window id w is
    genome[w // 2 : w // 2 + ref_len], reverse-complemented when w is odd (find_sequence,
    src/utils/post_processor.cpp:47-64)."""

    def __init__(self, genome, ref_len, device=0):
        g = np.frombuffer(genome, dtype=np.uint8) if isinstance(genome, (bytes, bytearray)) else \
            np.ascontiguousarray(genome, dtype=np.uint8)
        self.glen, self.ref_len = int(g.size), int(ref_len)
        h = C.c_void_p()
        check(lib().drm_refs_create_genome(ptr(g) if g.size else None, g.size, int(ref_len), int(device), C.byref(h)))
        self._h = h.value

    @property
    def handle(self):
        return self._h

    def free(self):
        if self._h:
            check(lib().drm_refs_free(self._h))
            self._h = None

    def __del__(self):
        try:
            if getattr(self, "_h", None):
                self.free()
        except Exception:
            pass


def extract_fasta_sequence(path):
    """extract_FASTA_sequence (src/utils/parse_inputs.cpp:174-220) -> bytes."""
    n = C.c_int64(0)
    check(lib().drm_extract_fasta_sequence(str(path).encode(), None, C.byref(n)))
    out = np.empty(max(n.value, 1), dtype=np.uint8)
    n2 = C.c_int64(n.value)
    check(lib().drm_extract_fasta_sequence(str(path).encode(), ptr(out), C.byref(n2)))
    return bytes(out[:n.value])


def rerank_dynamic_arrays(genome_table, neighbors, query_seqs, stride, k, k_clusters):
    """Array form of post_process_sw_dynamic on a GenomeTable: (scores, ids, counts) like rerank_arrays."""
    nb = np.ascontiguousarray(neighbors, dtype=np.int64)
    nq, kk = nb.shape
    qbuf, qlen = query_seqs if isinstance(query_seqs, tuple) else pack_queries(query_seqs)
    scores = np.empty((nq, k), dtype=np.int32)
    ids = np.empty((nq, k), dtype=np.uint64)
    counts = np.empty(nq, dtype=np.int32)
    bad = C.c_int64(-1)
    check(lib().drm_post_process_sw_dynamic(genome_table.handle, ptr(nb), nq, kk, ptr(qbuf), ptr(qlen), qbuf.shape[1],
                                            int(stride), int(k), int(k_clusters), ptr(scores), ptr(ids), ptr(counts),
                                            C.byref(bad)))
    return scores, ids, counts


def post_process_sw_dynamic(neighbors, distances, ref_genome, query_seqs, ref_len, stride, k, k_clusters):
    """post_process_sw_dynamic (src/utils/post_processor.cpp:357-452): flattened (final_seqs,
    final_scores, final_ids); ref_genome is the genome string (bytes / str) or a GenomeTable."""
    g = ref_genome.encode() if isinstance(ref_genome, str) else ref_genome
    table = g if isinstance(g, GenomeTable) else GenomeTable(g, ref_len)
    nb = np.asarray([list(r) for r in neighbors], dtype=np.int64) if not isinstance(neighbors, np.ndarray) else neighbors
    try:
        scores, ids, counts = rerank_dynamic_arrays(table, nb, query_seqs, stride, k, k_clusters)
    except DrmError as e:
        raise RuntimeError(str(e)) from e
    seqs, sc, fid = [], [], []
    for i in range(len(counts)):
        for j in range(int(counts[i])):
            wid = int(ids[i, j])
            sc.append(int(scores[i, j]))
            fid.append(wid)
            if not isinstance(g, GenomeTable):
                pos = wid // 2
                w = g[pos:pos + ref_len] if pos + ref_len <= len(g) else b""
                if wid % 2 == 1 and w:
                    w = bytes(_COMP_TABLE[np.frombuffer(w, dtype=np.uint8)[::-1]])
                seqs.append(bytes(w))
    return seqs, sc, fid


_COMP_TABLE = np.zeros(256, dtype=np.uint8)
for _a, _b in zip(b"ATCGN", b"TAGCN"):
    _COMP_TABLE[_a] = _b


def pack_queries(query_seqs):
    qs = [_as_bytes(q) for q in query_seqs]
    stride = max([len(q) for q in qs] + [1])
    buf = np.zeros((len(qs), stride), dtype=np.uint8)
    for i, q in enumerate(qs):
        buf[i, :len(q)] = np.frombuffer(q, dtype=np.uint8)
    return buf, np.array([len(q) for q in qs], dtype=np.int32)


def rerank_arrays(table, neighbors, query_seqs, stride, k, k_clusters):
    """Array form of post_process_sw_static: returns (scores [nq,k] i32, ids [nq,k] u64, counts [nq])."""
    nb = np.ascontiguousarray(neighbors, dtype=np.int64)
    nq, kk = nb.shape
    qbuf, qlen = query_seqs if isinstance(query_seqs, tuple) else pack_queries(query_seqs)
    scores = np.empty((nq, k), dtype=np.int32)
    ids = np.empty((nq, k), dtype=np.uint64)
    counts = np.empty(nq, dtype=np.int32)
    bad = C.c_int64(-1)
    rc = lib().drm_post_process_sw_static(table.handle, ptr(nb), nq, kk, ptr(qbuf), ptr(qlen), qbuf.shape[1],
                                          int(stride), int(k), int(k_clusters), ptr(scores), ptr(ids), ptr(counts),
                                          C.byref(bad))
    check(rc)
    return scores, ids, counts


def post_process_sw_static(neighbors, distances, ref_seqs, query_seqs, ref_len, stride, k, k_clusters):
    """Reference-shaped result: flattened (final_seqs, final_scores, final_ids) over all queries
    (post_processor.cpp:533-548). Raises RuntimeError like the reference on k / candidate errors."""
    table = ref_seqs if isinstance(ref_seqs, WindowTable) else WindowTable(ref_seqs)
    nb = np.asarray([list(r) for r in neighbors], dtype=np.int64) if not isinstance(neighbors, np.ndarray) else neighbors
    try:
        scores, ids, counts = rerank_arrays(table, nb, query_seqs, stride, k, k_clusters)
    except DrmError as e:
        raise RuntimeError(str(e)) from e
    seqs, sc, fid = [], [], []
    for i in range(len(counts)):
        for j in range(int(counts[i])):
            wid = int(ids[i, j])
            sc.append(int(scores[i, j]))
            fid.append(wid)
            if not isinstance(ref_seqs, WindowTable):
                seqs.append(ref_seqs[wid])
    return seqs, sc, fid


def sw_reranker(cand_seqs, cand_ids, query_seq, k):
    """sw_reranker(cand_seqs, cand_ids, query_seq, k) -> (top_seqs, top_scores, top_ids)."""
    n = len(cand_seqs)
    if n == 0 or k == 0:
        return [], [], []
    scores = calc_sw_scores(cand_seqs, [query_seq] * n)
    if n < k:
        raise RuntimeError(f"Not enough candidates ({n} < {k})")
    order = partial_sort_order(scores, k)
    return [cand_seqs[i] for i in order], [int(scores[i]) for i in order], [cand_ids[i] for i in order]


def partial_sort_order(scores, k):
    """std::partial_sort order of reranker.cpp:38-40 computed on the device: the rerank kernel sorts
    candidate windows of a one-query table whose scores are the given ones."""
    scores = np.asarray(scores, dtype=np.int32)
    n = len(scores)
    # A window table whose window c scores exactly scores[c] against a query of 'A'*m:
    # window c = 'A'*scores[c] + 'C'*(L - scores[c]) with L = max score (calc_sw_score = run of A's).
    L = max(int(scores.max()) if n else 0, 1)
    if scores.min(initial=0) < 0:
        raise ValueError("scores must be >= 0")
    win = np.full((n, L), ord("C"), dtype=np.uint8)
    for c, s in enumerate(scores):
        win[c, :s] = ord("A")
    table = WindowTable(win)
    q = b"A" * L
    nb = np.arange(n, dtype=np.int64)[None, :]
    _, ids, _ = rerank_arrays(table, nb, [q], 1, k, n)
    table.free()
    return [int(i) for i in ids[0]]


# ------------------------------------------------------------------------------------------- L2 rerank
def embed_windows(table, encoder, stream=None):
    """Fill the table's device embedding of every window with the read encoder (drm_refs_embed): the rows the
    reference's post_process_l2_static re-embeds per run (src/utils/post_processor.cpp:1075-1080)."""
    check(lib().drm_refs_embed(table.handle, encoder.handle, stream.handle if stream is not None else None))


def window_embeddings_ptr(table):
    """(device pointer, width) of the table's window embeddings (0, 0 before embed_windows)."""
    p, d = C.c_void_p(), C.c_int32(0)
    check(lib().drm_refs_embeddings(table.handle, C.byref(p), C.byref(d)))
    return p.value or 0, d.value


def l2_rerank_arrays(table, neighbors, query_embeddings, stride, k_clusters):
    """Array form of post_process_l2_static on an embedded WindowTable: (dists [nq,k_clusters] f32,
    ids [nq,k_clusters] u64, counts [nq])."""
    nb = np.ascontiguousarray(neighbors, dtype=np.int64)
    nq, kk = nb.shape
    qe = np.ascontiguousarray(query_embeddings, dtype=np.float32)
    if qe.shape[0] != nq:
        raise ValueError("one query embedding per neighbor row")
    dists = np.empty((nq, k_clusters), dtype=np.float32)
    ids = np.empty((nq, k_clusters), dtype=np.uint64)
    counts = np.empty(nq, dtype=np.int32)
    bad = C.c_int64(-1)
    check(lib().drm_post_process_l2_static(table.handle, ptr(nb), nq, kk, ptr(qe), qe.shape[1], int(stride),
                                           int(k_clusters), ptr(dists), ptr(ids), ptr(counts), C.byref(bad)))
    return dists, ids, counts


def post_process_l2_static(neighbors, distances, ref_seqs, query_seqs, ref_len, stride, k, query_embeddings,
                           vectorizer, k_clusters):
    """post_process_l2_static (src/utils/post_processor.cpp:1023-1162), the reference's live rerank
    (src/main.cpp:330): flattened (final_seqs, final_dists, final_ids), k_clusters rows per query
    (batch_reranker is called with k = k_clusters; `k` and `query_seqs` are unused there too). ref_seqs is a
    WindowTable or a list of windows; vectorizer an Encoder (embeds the table once on the device)."""
    table = ref_seqs if isinstance(ref_seqs, WindowTable) else WindowTable(ref_seqs)
    if window_embeddings_ptr(table)[0] == 0:
        embed_windows(table, getattr(vectorizer, "encoder", vectorizer))
    nb = np.asarray([list(r) for r in neighbors], dtype=np.int64) if not isinstance(neighbors, np.ndarray) else neighbors
    try:
        dists, ids, counts = l2_rerank_arrays(table, nb, query_embeddings, stride, k_clusters)
    except DrmError as e:
        raise RuntimeError(str(e)) from e
    seqs, dd, fid = [], [], []
    for i in range(len(counts)):
        for j in range(int(counts[i])):
            wid = int(ids[i, j])
            dd.append(float(dists[i, j]))
            fid.append(wid)
            if not isinstance(ref_seqs, WindowTable):
                seqs.append(ref_seqs[wid])
    return seqs, dd, fid


def l2_rerank_dynamic_arrays(genome_table, neighbors, query_embeddings, stride, k, k_clusters):
    """post_process_l2_dynamic's rerank (stride > 1) on an embedded GenomeTable: (dists [nq,k] f32,
    ids [nq,k] u64, counts [nq])."""
    nb = np.ascontiguousarray(neighbors, dtype=np.int64)
    nq, kk = nb.shape
    qe = np.ascontiguousarray(query_embeddings, dtype=np.float32)
    if qe.shape[0] != nq:
        raise ValueError("one query embedding per neighbor row")
    dists = np.empty((nq, k), dtype=np.float32)
    ids = np.empty((nq, k), dtype=np.uint64)
    counts = np.empty(nq, dtype=np.int32)
    bad = C.c_int64(-1)
    check(lib().drm_post_process_l2_dynamic(genome_table.handle, ptr(nb), nq, kk, ptr(qe), qe.shape[1], int(stride),
                                            int(k), int(k_clusters), ptr(dists), ptr(ids), ptr(counts), C.byref(bad)))
    return dists, ids, counts


def post_process_l2_dynamic(neighbors, distances, ref_genome, query_seqs, ref_len, stride, k, query_embeddings,
                            vectorizer, k_clusters):
    """post_process_l2_dynamic (src/utils/post_processor.cpp:553-750): flattened (final_seqs, final_dists,
    final_ids). At stride 1 the reference reranks nothing: each query's first min(k, kk) search neighbours with
    their search distances (:633-660). At stride > 1 the L2 rerank of l2_rerank_dynamic_arrays, k rows per query.
    ref_genome is the genome string (bytes / str) or a GenomeTable; vectorizer an Encoder or Vectorizer."""
    g = ref_genome.encode() if isinstance(ref_genome, str) else ref_genome
    table = g if isinstance(g, GenomeTable) else GenomeTable(g, ref_len)
    nb = np.asarray([list(r) for r in neighbors], dtype=np.int64) if not isinstance(neighbors, np.ndarray) else neighbors

    def window(wid):
        if isinstance(g, GenomeTable):
            return None
        pos = wid // 2
        w = g[pos:pos + ref_len] if pos + ref_len <= len(g) else b""
        if wid % 2 == 1 and w:
            w = bytes(_COMP_TABLE[np.frombuffer(w, dtype=np.uint8)[::-1]])
        return bytes(w)

    seqs, dd, fid = [], [], []
    if stride == 1:
        for i in range(nb.shape[0]):
            for j in range(min(k, nb.shape[1])):
                wid = int(nb[i, j]) & (2**64 - 1)
                fid.append(wid)
                dd.append(float(distances[i][j]))
                seqs.append(window(wid))
        return seqs, dd, fid
    if window_embeddings_ptr(table)[0] == 0:
        embed_windows(table, getattr(vectorizer, "encoder", vectorizer))
    try:
        dists, ids, counts = l2_rerank_dynamic_arrays(table, nb, query_embeddings, stride, k, k_clusters)
    except DrmError as e:
        raise RuntimeError(str(e)) from e
    for i in range(len(counts)):
        for j in range(int(counts[i])):
            wid = int(ids[i, j])
            dd.append(float(dists[i, j]))
            fid.append(wid)
            seqs.append(window(wid))
    return seqs, dd, fid
