"""Dynamic genome lookup + SAM output on the GPU (use_dynamic / use_streaming):
* drm_post_process_sw_dynamic (windows cut from the device-resident genome, reverse-complemented for odd
  ids) equals the oracle's post_process_sw_dynamic bit for bit -- dense with -1 / past-the-end ids, and
  sparse strides 2-4 whose expansion is checked against the genome length (post_processor.cpp:72-201);
* genome bytes N (and query N) go through the exact bit-profile re-score;
* the batch executor with a genome handle equals the direct call;
* bin/pipeline with use_dynamic=1 writes the same .npy files as the static lookup, and with
  use_streaming=1 writes results.sam exactly as write_sam_streaming formats it (src/utils/utils.cpp:409-503)
  for the rows post_process_l2_dynamic_streaming streams at stride 1 (the first k search neighbours)
  and no .npy files (src/main.cpp:371, :409-412)."""
import os
import subprocess

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")


@pytest.fixture(scope="module")
def genome_case():
    from deepreadmapper_amd import synth, extract_fasta_sequence
    g = np.frombuffer(extract_fasta_sequence(os.path.join(GOLDEN, "ecoli_150.fna")), dtype=np.uint8).copy()
    reads, _, _ = synth.simulate_reads(g, 96, seed=21)
    q = synth.tag(reads)
    return {"g": g, "q": q, "ql": np.full(len(q), q.shape[1], dtype=np.int32), "nwin": 2 * (len(g) - 149)}


def _both(table, g, nb, q, ql, stride, k, kc):
    from deepreadmapper_amd import rerank_dynamic_arrays
    from deepreadmapper_amd._native import DrmError, DRM_ERR_CANDS
    rc, sco, ido, cnto = O.post_process_sw_dynamic(nb, g, 150, q, ql, stride, k, kc)
    if rc < 0:  # some query has 0 < candidates < k: sw_reranker throws (reranker.cpp:26-29), so does the GPU
        with pytest.raises(DrmError) as e:
            rerank_dynamic_arrays(table, nb, (q, ql), stride, k, kc)
        assert e.value.code == DRM_ERR_CANDS
        return None, None
    sc, ids, cnt = rerank_dynamic_arrays(table, nb, (q, ql), stride, k, kc)
    assert np.array_equal(cnt, cnto) and np.array_equal(sc, sco) and np.array_equal(ids, ido)
    return sc, ids


def test_dynamic_dense_vs_oracle(genome_case):
    from deepreadmapper_amd import GenomeTable
    c = genome_case
    rng = np.random.default_rng(7)
    nb = rng.integers(0, c["nwin"], size=(len(c["q"]), 160)).astype(np.int64)
    nb[::3, 5] = -1                      # faiss padding: kept, empty window, id 2^64-1
    nb[::4, 9] = c["nwin"] + 17          # past the genome end: kept, empty window
    nb[::5, 11] = c["nwin"] - 1          # the last reverse-complement window
    t = GenomeTable(c["g"], 150)
    _both(t, c["g"], nb, c["q"], c["ql"], 1, 128, 160)
    sc, ids = _both(t, c["g"], nb, c["q"], c["ql"], 1, 160, 160)  # k = all: the empty windows are kept, score 0
    assert (ids == np.uint64(2 ** 64 - 1)).any() and (sc[ids == np.uint64(2 ** 64 - 1)] == 0).all()
    _both(t, c["g"], nb, c["q"], c["ql"], 1, 5, 5)
    t.free()


@pytest.mark.parametrize("stride", [2, 3, 4])
def test_dynamic_sparse_vs_oracle(genome_case, stride):
    from deepreadmapper_amd import GenomeTable
    c = genome_case
    rng = np.random.default_rng(stride)
    nb = rng.integers(0, len(c["g"]) // stride + 3, size=(len(c["q"]), 20)).astype(np.int64)
    nb[::7, 0] = -1
    t = GenomeTable(c["g"], 150)
    _both(t, c["g"], nb, c["q"], c["ql"], stride, 5, 5)
    _both(t, c["g"], nb, c["q"], c["ql"], stride, 32, 20)
    _both(t, c["g"], nb, c["q"], c["ql"], stride, 64, 20)  # stride 2: 20 x 3 < 64 -> the reference's error
    t.free()


def test_dynamic_n_bytes_exact(genome_case):
    """Genome N against query N scores +1 (raw byte equality, metrics.cpp:18-20): the fp16 kernel
    flags such queries and the bit-profile kernel re-scores them exactly."""
    from deepreadmapper_amd import GenomeTable
    c = genome_case
    g = c["g"].copy()
    g[100:130] = ord("N")
    q = c["q"].copy()
    q[::2, 20:40] = ord("N")
    rng = np.random.default_rng(11)
    nb = rng.integers(0, c["nwin"], size=(len(q), 128)).astype(np.int64)
    nb[:, 0] = 2 * 90  # a window through the N run, forward
    nb[:, 1] = 2 * 95 + 1  # and reverse-complemented (N stays N)
    t = GenomeTable(g, 150)
    _both(t, g, nb, q, c["ql"], 1, 128, 128)
    t.free()


def test_executor_with_genome_handle(syn20k):
    from deepreadmapper_amd import read_index, GenomeTable, rerank_dynamic_arrays
    from deepreadmapper_amd.executor import search_rerank, MultiIndex
    w = syn20k["w"]
    ix, t = read_index(w.index_path), GenomeTable(w.genome, 150)
    o = search_rerank(ix, t, w.q_emb, w.queries, k=128, ef=128)
    sc, ids, cnt = rerank_dynamic_arrays(t, o["I"], w.queries, 1, 128, 128)
    assert np.array_equal(o["sw_scores"], sc) and np.array_equal(o["sw_ids"], ids) and (o["status"] == cnt).all()
    m = MultiIndex(w.index_path, [0, 0], genome=w.genome, ref_len=150)
    o2 = m.search_rerank(w.q_emb, w.queries, k=128, ef=128)
    m.free()
    assert np.array_equal(o2["sw_ids"], o["sw_ids"]) and np.array_equal(o2["I"], o["I"])
    ix.free()
    t.free()


def _sam_ref(read_ids, reads, ids, counts):
    """write_sam_streaming's lines (src/utils/utils.cpp:468-500)."""
    out = ["@HD\tVN:1.0\tSO:unsorted", "@SQ\tSN:ref\tLN:150"]
    for i, (qid, r) in enumerate(zip(read_ids, reads)):
        clean = r[1:-1] if len(r) > 2 else r
        for j in range(int(counts[i])):
            sid = int(ids[i, j])
            flag = (0 if j == 0 else 256) | (16 if sid % 2 == 1 else 0)
            out.append(f"{qid}\t{flag}\tref\t{sid // 2 + 1}\t60\t{len(clean)}M\t*\t0\t0\t{clean.decode()}\t*")
    return "\n".join(out) + "\n"


def test_pipeline_cli_dynamic_and_sam_streaming(tmp_path):
    fna = os.path.join(GOLDEN, "ecoli_150.fna")
    fq = os.path.join(GOLDEN, "test_data.fastq")
    env = dict(os.environ, DRM_BUILD_THREADS="1")
    r = subprocess.run([os.path.join(ROOT, "bin", "hnswpq_index"), fna, "c1", "150"], cwd=tmp_path, env=env,
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    pipe = os.path.join(ROOT, "bin", "pipeline")
    base = [pipe, "c1", fq, fna, "128", "128", "5"]
    for name, extra in (("static", ["0", "0"]), ("dyn", ["1", "0"]), ("stream", ["1", "1"])):
        e = dict(os.environ, DRM_SAM_BLOCK="40")  # several SAM blocks for 150 reads
        r = subprocess.run(base + [name] + extra, cwd=tmp_path, env=e, capture_output=True, text=True)
        assert r.returncode == 0, r.stdout + r.stderr
    files = ("indices.npy", "distances.npy", "sw_scores.npy", "sw_ids.npy")
    for f in files:
        assert open(tmp_path / "static" / f, "rb").read() == open(tmp_path / "dyn" / f, "rb").read(), f
    assert not any(os.path.exists(tmp_path / "stream" / f) for f in files)
    sam = open(tmp_path / "stream" / "results.sam").read()
    lines = open(fq, "rb").read().split(b"\n")
    recs = [(lines[i], lines[i + 1]) for i in range(0, len(lines) - 1, 4) if lines[i].startswith(b"@")]
    qids = [h[1:].split(b" ")[0].split(b"\t")[0].split(b"/")[0].decode() for h, _ in recs]
    reads = [b"<" + s + b">" for _, s in recs]
    # post_process_l2_dynamic_streaming at stride 1 (src/utils/post_processor.cpp:833-878): the first
    # min(k, k_clusters) search neighbours in search order (k = 128 and k_clusters = k at stride 1,
    # src/main.cpp:54-62), i.e. the static run's indices.npy (save_results keeps k columns at stride 1)
    ids = np.load(tmp_path / "static" / "indices.npy")
    assert ids.shape == (len(reads), 128)
    assert sam == _sam_ref(qids, reads, ids, np.full(len(reads), 128))
