"""The opt-in banded Smith-Waterman rerank (drm_refs_set_sw_band; an extension -- the reference scores the full DP
and leaves banding as a TODO, includes/utils/reranker.hpp:12). It is not parity with the reference: its oracle is
oracle_calc_sw_score_banded (the recurrence of metrics.cpp:30-41 on the cells |i - j| <= band, 0 outside), and the
kernel must equal it bit for bit -- scores, the libstdc++ partial_sort order and the counts -- on the static table
(dense and sparse), the genome lookup, ragged and empty queries, N bytes, and candidates shifted off the diagonal
by more and less than the band. Band 0 is the reference's full DP again."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

BANDS = [8, 16, 32]


@pytest.fixture(scope="module")
def band_case():
    """A random 4,000-base genome (a few N runs), its forward windows, and 64 tagged 150 bp reads cut from it with
    substitutions and small indels; read r's candidates are the windows at its origin shifted by -45 .. +45 (step 3)
    plus random windows."""
    rng = np.random.default_rng(17)
    g = rng.choice(np.frombuffer(b"ACGT", np.uint8), size=4000).astype(np.uint8)
    g[500:520] = ord("N")
    g[2500:2503] = ord("N")
    nwin = len(g) - 150 + 1
    refs = np.stack([g[p:p + 150] for p in range(nwin)])
    reads, origin = [], []
    for r in range(64):
        p = int(rng.integers(60, nwin - 60))
        s = bytearray(g[p:p + 170].tobytes())
        for _ in range(int(rng.integers(0, 6))):  # substitutions
            s[int(rng.integers(0, 150))] = int(rng.choice(np.frombuffer(b"ACGT", np.uint8)))
        if r % 3 == 0:  # a deletion
            i = int(rng.integers(20, 130))
            del s[i:i + int(rng.integers(1, 5))]
        if r % 3 == 1:  # an insertion
            i = int(rng.integers(20, 130))
            s[i:i] = bytes(rng.choice(np.frombuffer(b"ACGT", np.uint8), size=int(rng.integers(1, 5))))
        body = bytes(s[:150])
        if r % 8 == 5:
            body = body[:40] + b"NNNN" + body[44:]
        reads.append(b"<" + body + b">")
        origin.append(p)
    shifts = np.arange(-45, 46, 3)
    nb = np.empty((64, 64), dtype=np.int64)
    for r, p in enumerate(origin):
        nb[r, :len(shifts)] = np.clip(p + shifts, 0, nwin - 1)
        nb[r, len(shifts):] = rng.integers(0, nwin, size=64 - len(shifts))
    return {"g": g, "refs": refs, "reads": reads, "nb": nb, "nwin": nwin}


def _static(refs, nb, reads, stride, k, kc, band):
    from deepreadmapper_amd import WindowTable, rerank_arrays
    from deepreadmapper_amd.rerank import pack_queries
    qbuf, ql = pack_queries(reads)
    rc, sco, ido, cnto = O.post_process_sw_static(nb, refs, refs.shape[1], qbuf, ql, stride, k, kc, band=band)
    assert rc == 0
    t = WindowTable(refs)
    t.sw_band = band
    assert t.sw_band == band
    sc, ids, cnt = rerank_arrays(t, nb, (qbuf, ql), stride, k, kc)
    t.free()
    assert np.array_equal(cnt, cnto)
    for i in range(len(nb)):
        n = cnt[i]
        assert np.array_equal(sc[i, :n], sco[i, :n]) and np.array_equal(ids[i, :n], ido[i, :n]), (band, i)
    return sc, ids


@pytest.mark.parametrize("band", BANDS)
def test_band_static_dense_vs_oracle(band_case, band):
    c = band_case
    _static(c["refs"], c["nb"], c["reads"], 1, 64, 64, band)
    _static(c["refs"], c["nb"], c["reads"], 1, 10, 40, band)  # k < k_clusters


def test_band_changes_scores_and_band0_is_full(band_case):
    """Band 8 scores the -45 shift's window below the full DP (its alignment lies outside the band), and a handle
    set back to band 0 runs the reference's full DP (the oracle's calc_sw_score)."""
    c = band_case
    lo = [O.calc_sw_score_banded(bytes(c["refs"][c["nb"][r, 0]]), c["reads"][r], 8) for r in range(8)]
    hi = [O.calc_sw_score(bytes(c["refs"][c["nb"][r, 0]]), c["reads"][r]) for r in range(8)]
    assert all(a <= b for a, b in zip(lo, hi)) and any(a < b for a, b in zip(lo, hi))
    _static(c["refs"], c["nb"], c["reads"], 1, 64, 64, 0)


@pytest.mark.parametrize("stride", [2, 4])
def test_band_static_sparse_vs_oracle(band_case, stride):
    c = band_case
    rng = np.random.default_rng(stride)
    nb = rng.integers(-1, c["nwin"] // stride + 10, size=(64, 8)).astype(np.int64)
    _static(c["refs"], nb, c["reads"], stride, 5, 5, 16)


def test_band_ragged_queries(band_case):
    """Queries of 0 .. 256 bytes (all of the band's edge cases: shorter than the band, rows past qlen + W, the
    256-byte limit), windows of 150."""
    c = band_case
    rng = np.random.default_rng(5)
    lens = [0, 1, 2, 7, 8, 9, 16, 17, 31, 33, 64, 100, 149, 150, 151, 152, 180, 200, 255, 256]
    reads = []
    for n in lens:
        base = c["reads"][n % 64] * 2
        reads.append(base[:n])
    nb = rng.integers(0, c["nwin"], size=(len(reads), 24)).astype(np.int64)
    for band in BANDS:
        _static(c["refs"], nb, reads, 1, 24, 24, band)


def test_band_limits_fail_loudly(band_case):
    """Past the banded kernel's limits (a query longer than 256 bytes, a query with 8 distinct byte values) the
    rerank fails with DRM_ERR_UNSUPPORTED; a band other than 0 / 8 / 16 / 32 is DRM_ERR_ARG."""
    from deepreadmapper_amd import WindowTable, rerank_arrays, DrmError
    from deepreadmapper_amd._native import DRM_ERR_ARG, DRM_ERR_UNSUPPORTED
    c = band_case
    t = WindowTable(c["refs"])
    with pytest.raises(DrmError) as e:
        t.sw_band = 12
    assert e.value.code == DRM_ERR_ARG and t.sw_band == 0
    t.sw_band = 16
    nb = c["nb"][:2, :8]
    with pytest.raises(DrmError) as e:
        rerank_arrays(t, nb, [c["reads"][0], c["reads"][1] * 2], 1, 8, 8)  # 304 bytes
    assert e.value.code == DRM_ERR_UNSUPPORTED
    with pytest.raises(DrmError) as e:
        rerank_arrays(t, nb, [c["reads"][0], b"ACGTN<>X" * 10], 1, 8, 8)  # 8 distinct bytes
    assert e.value.code == DRM_ERR_UNSUPPORTED
    sc, _, _ = rerank_arrays(t, nb, [c["reads"][0], b"ACGTN<>" * 10], 1, 8, 8)  # 7: supported
    t.free()


@pytest.mark.parametrize("band", BANDS)
def test_band_dynamic_vs_oracle(band_case, band):
    """The genome lookup (window w = genome[w/2 ..], reverse-complemented for odd w; ids past the genome end are
    empty windows) with the band."""
    from deepreadmapper_amd import GenomeTable, rerank_dynamic_arrays
    from deepreadmapper_amd.rerank import pack_queries
    c = band_case
    g = c["g"]
    nwin2 = 2 * c["nwin"]
    rng = np.random.default_rng(band)
    nb = np.concatenate([2 * c["nb"][:, :32], rng.integers(0, nwin2, size=(64, 32))], axis=1).astype(np.int64)
    nb[::5, 3] = -1
    nb[::7, 4] = nwin2 + 9
    qbuf, ql = pack_queries(c["reads"])
    rc, sco, ido, cnto = O.post_process_sw_dynamic(nb, g, 150, qbuf, ql, 1, 64, 64, band=band)
    assert rc == 0
    t = GenomeTable(g, 150)
    t.sw_band = band
    sc, ids, cnt = rerank_dynamic_arrays(t, nb, (qbuf, ql), 1, 64, 64)
    t.free()
    assert np.array_equal(cnt, cnto) and np.array_equal(sc, sco) and np.array_equal(ids, ido)
