"""Read encoder on the GPU against the oracle (oracle/gru_oracle.py,
float64 on the same f16 weights; parity unpinned against OpenVINO, see that header).

Bars:
* tokens (drm_tokenize): bit-exact with the oracle's restatement of Preprocessor::preprocess, incl.
  the tag quirk, truncation at 123, ragged lengths 2..200, mixed case, N (out-of-table -> -1);
* embeddings (drm_vectorize): max |gpu - oracle| <= ENC_ATOL. The recurrence runs in f32 with the state
  entering the f16 MFMA as hi + lo terms (~2^-22 relative), so the f32-level error of 123 x 2 layers
  of gate math is what remains;
* bit-identical results for a read wherever it sits in the batch, for the device entry point, and for
  any number of tiles per launch (chunking)."""
import os

import numpy as np
import pytest

from oracle import gru_oracle as G

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
ENC_ATOL = 2e-5


@pytest.fixture(scope="module")
def enc():
    from deepreadmapper_amd import Encoder
    e = Encoder()
    yield e
    e.free()


@pytest.fixture(scope="module")
def weights():
    from deepreadmapper_amd.encoder import DEFAULT_MODEL
    return G.load_drmenc(DEFAULT_MODEL)


@pytest.fixture(scope="module")
def c1_seqs():
    from conftest import read_fastq_tagged
    reads = read_fastq_tagged(os.path.join(GOLDEN, "test_data.fastq"))
    refs = [b"<" + l + b">" for l in open(os.path.join(GOLDEN, "test_data_ref.txt"), "rb").read().split(b"\n") if l]
    return reads + refs[:400]


def _ragged(n, seed):
    rng = np.random.default_rng(seed)
    alpha = np.frombuffer(b"ACGTacgtN<>", dtype=np.uint8)
    p = np.array([.22, .22, .22, .22, .02, .02, .02, .02, .02, .01, .01])
    out = []
    for i in range(n):
        L = int(rng.integers(2, 201))
        s = alpha[rng.choice(len(alpha), size=L, p=p / p.sum())].tobytes()
        out.append(b"<" + s + b">" if i % 3 == 0 else s)
    return out


def test_tokenize_matches_preprocess(enc, c1_seqs):
    seqs = c1_seqs[:60] + _ragged(500, 1) + [b"AC", b"ACG", b"<" + b"A" * 121 + b">", b"<" + b"C" * 122, b"G" * 124]
    got = enc.tokenize(seqs)
    assert np.array_equal(got, G.model_input(seqs))
    assert (got == -1).any()   # N-containing 3-mers hit the reference's undefined read


def test_vectorize_c1_vs_oracle(enc, weights, c1_seqs):
    got = enc.vectorize(c1_seqs)
    ref = G.vectorize(weights, c1_seqs)
    err = np.abs(got.astype(np.float64) - ref)
    print(f"C1 max abs err {err.max():.3g}, mean {err.mean():.3g}")
    assert err.max() <= ENC_ATOL


def test_vectorize_ragged_vs_oracle(enc, weights):
    seqs = _ragged(1027, 2)                     # 33 tiles, the last one partial
    got, und = enc.vectorize(seqs, return_undefined=True)
    ref = G.vectorize(weights, seqs)
    err = np.abs(got.astype(np.float64) - ref)
    print(f"ragged max abs err {err.max():.3g}")
    assert err.max() <= ENC_ATOL
    assert und == int((G.model_input(seqs) == -1).sum())


def test_position_and_chunking_invariance(enc, c1_seqs):
    from deepreadmapper_amd import Encoder
    seqs = (c1_seqs * 4)[:1500]
    a = enc.vectorize(seqs)
    perm = np.random.default_rng(3).permutation(len(seqs))
    b = enc.vectorize([seqs[i] for i in perm])
    assert np.array_equal(a[perm], b)
    os.environ["DRM_ENC_TILES"] = "3"          # 3 tiles per launch: 16 launches instead of 1
    try:
        e3 = Encoder()
        assert np.array_equal(e3.vectorize(seqs), a)
        e3.free()
    finally:
        del os.environ["DRM_ENC_TILES"]


def test_vectorize_device_entry(enc, c1_seqs):
    from deepreadmapper_amd.device import DeviceBuffer, Stream
    from deepreadmapper_amd.rerank import pack_queries
    buf, lens = pack_queries(c1_seqs)
    d_s, d_l = DeviceBuffer.from_host(buf), DeviceBuffer.from_host(lens)
    d_o = DeviceBuffer((len(lens), 128), np.float32)
    st = Stream()
    enc.vectorize_device(d_s, d_l, len(lens), buf.shape[1], d_o, st)
    st.synchronize()
    assert np.array_equal(d_o.download(), enc.vectorize(c1_seqs))
    assert enc.flags() == (0, 0)


def test_errors(enc):
    from deepreadmapper_amd._native import DrmError, DRM_ERR_ARG, DRM_ERR_IO
    from deepreadmapper_amd import Encoder
    with pytest.raises(DrmError) as e:
        enc.vectorize([b"ACGT", b"A"])          # the reference reads past a 1-byte sequence
    assert e.value.code == DRM_ERR_ARG
    with pytest.raises(DrmError) as e:
        Encoder("/nonexistent/model.xml")
    assert e.value.code == DRM_ERR_IO
    assert enc.vectorize([]).shape == (0, 128)


def test_gpu_embeddings_map_reads_to_source_windows(enc):
    """End to end on C1: GRU embeddings of reads and windows, nearest window = best SW window for
    >= 90 % of the reads that come from the genome (the oracle's own rate, test_encoder_cpu.py)."""
    from conftest import read_fastq_tagged
    reads = read_fastq_tagged(os.path.join(GOLDEN, "test_data.fastq"))
    refs = [b"<" + l + b">" for l in open(os.path.join(GOLDEN, "test_data_ref.txt"), "rb").read().split(b"\n") if l]
    M = np.load(os.path.join(GOLDEN, "sw_c1_matrix.npy"))
    eq, er = enc.vectorize(reads), enc.vectorize(refs)
    nn = ((eq[:, None, :].astype(np.float64) - er[None, :, :]) ** 2).sum(-1).argmin(1)
    mapped = M.max(1) >= 100
    assert (M[np.arange(len(reads)), nn] == M.max(1))[mapped].mean() >= 0.9


def test_cli_with_gru_encoder(tmp_path, enc):
    """bin/hnswpq_index + bin/pipeline with DRM_ENCODER: windows and reads embedded by the GRU on the GPU
    (the reference's index.cpp:279-280 and main.cpp:249-268 path). The index's vectors decode to the
    encoder's window embeddings (PQ codes equal the oracle's encoding of them), and the pipeline's
    indices/distances equal the oracle's faiss search over those encoder embeddings of the reads."""
    import subprocess
    from deepreadmapper_amd.encoder import DEFAULT_MODEL
    from conftest import read_fastq_tagged
    from oracle import faiss_file, oracle as O
    fna = os.path.join(GOLDEN, "ecoli_150.fna")
    fq = os.path.join(GOLDEN, "test_data.fastq")
    env = dict(os.environ, DRM_BUILD_THREADS="1", DRM_ENCODER=DEFAULT_MODEL)
    r = subprocess.run([os.path.join(ROOT, "bin", "hnswpq_index"), fna, "g1", "150"], cwd=tmp_path, env=env,
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "embedded by the GRU model" in r.stdout
    r = subprocess.run([os.path.join(ROOT, "bin", "pipeline"), "g1", fq, fna, "128", "128", "5", "out"],
                       cwd=tmp_path, env=env, capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "Inference (GRU model" in r.stdout
    reads = read_fastq_tagged(fq)
    q = enc.vectorize(reads)
    fx = faiss_file.read(str(tmp_path / "g1" / "g1.index"))
    Do, Io, _, _ = O.hnswpq_search(fx, q, 128, 128)
    I = np.load(tmp_path / "out" / "indices.npy")
    D = np.load(tmp_path / "out" / "distances.npy")
    assert np.array_equal(I.astype(np.int64), Io) and np.array_equal(D, Do)
    # reads land on their source windows through the whole GRU -> PQ -> HNSW -> SW path
    M = np.load(os.path.join(GOLDEN, "sw_c1_matrix.npy"))
    ids = np.load(tmp_path / "out" / "sw_ids.npy").astype(np.int64)
    mapped = M.max(1) >= 100
    assert (M[np.arange(len(reads)), ids[:, 0]] == M.max(1))[mapped].mean() >= 0.9
