import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")


def read_fastq_tagged(path):
    """format_fastq semantics (src/utils/parse_inputs.cpp:843-950) for the fixture."""
    lines = open(path, "rb").read().split(b"\n")
    return [b"<" + lines[i + 1] + b">" for i in range(0, len(lines) - 1, 4) if lines[i].startswith(b"@")]


@pytest.fixture(scope="session")
def c1(tmp_path_factory):
    """BASELINE config C1: tests/ecoli_150.fna (1702 windows) + tests/test_data.fastq (150 reads),
    stand-in embeddings, IndexHNSWPQ(M_pq=8, nbits=8, M_hnsw=16, EFC=200) built single-threaded."""
    from deepreadmapper_amd import synth
    from oracle import faiss_file
    d = tmp_path_factory.mktemp("c1")
    fna = open(os.path.join(GOLDEN, "ecoli_150.fna"), "rb").read().split(b"\n")
    g = np.frombuffer(b"".join(l.strip() for l in fna[1:]).upper(), dtype=np.uint8)
    refs = synth.windows_lookup(g, 150, 1)
    x = synth.embed(synth.tag(refs))
    path = str(d / "c1.index")
    synth.build_index(x, path, nthreads=1)
    reads = read_fastq_tagged(os.path.join(GOLDEN, "test_data.fastq"))
    return {"index": path, "fx": faiss_file.read(path), "refs": refs, "x": x, "reads": reads,
            "q": synth.embed(reads), "dir": str(d)}


@pytest.fixture(scope="session")
def syn20k(tmp_path_factory):
    """A 20k-window synthetic dense index (genome 10,149 bp) + 2,000 simulated reads."""
    from deepreadmapper_amd import synth
    from oracle import faiss_file
    d = tmp_path_factory.mktemp("syn")
    w = synth.Workload("syn20k", 10_149, 2000, seed=5, read_seed=11).generate(str(d), nthreads=4)
    return {"index": w.index_path, "fx": faiss_file.read(w.index_path), "w": w}


@pytest.fixture(scope="session")
def repeats(tmp_path_factory):
    """Tie-heavy index: a genome built from a 600 bp unit repeated 6 times inside random flanks, so
    many windows (and their PQ codes) are identical and equal distances are everywhere. Exercises
    the exact fallback of the sorted-array search kernel."""
    from deepreadmapper_amd import synth
    from oracle import faiss_file
    d = tmp_path_factory.mktemp("rep")
    unit = synth.genome(600, seed=3)
    g = np.concatenate([synth.genome(900, seed=4)] + [unit] * 6 + [synth.genome(900, seed=5)])
    refs = synth.windows_lookup(g, 150, 1)
    x = synth.embed(synth.tag(refs))
    path = str(d / "rep.index")
    synth.build_index(x, path, nthreads=1)
    reads, _, _ = synth.simulate_reads(g, 300, seed=13)
    q = np.concatenate([synth.embed(synth.tag(reads)), x[::29]])  # plus exact window embeddings
    return {"index": path, "fx": faiss_file.read(path), "x": x, "q": np.ascontiguousarray(q)}


def _flat(tmp_path_factory, name, x, M, efc=128):
    from deepreadmapper_amd import synth
    from oracle import hnswlib_file
    d = tmp_path_factory.mktemp(name)
    path = str(d / f"{name}.hnsw")
    synth.build_flat_index(x, path, M=M, efc=efc, nthreads=4)
    return path, hnswlib_file.read(path)


@pytest.fixture(scope="session")
def c1_flat(tmp_path_factory, c1):
    """C1 windows in an hnswlib fp32 index at the reference's defaults (M = 64, EFC = 128)."""
    path, fx = _flat(tmp_path_factory, "c1flat", c1["x"], 64)
    return {"index": path, "fx": fx, "q": c1["q"], "x": c1["x"]}


@pytest.fixture(scope="session")
def syn_flat(tmp_path_factory, syn20k):
    """The 20k-window synthetic set in an hnswlib fp32 index (M = 16: deeper graph, more hops)."""
    from oracle import hnswlib_file  # noqa: F401
    w = syn20k["w"]
    from deepreadmapper_amd import synth
    x = synth.embed(synth.tag(synth.windows_lookup(w.genome, 150, 1)))
    path, fx = _flat(tmp_path_factory, "synflat", x, 16, efc=64)
    return {"index": path, "fx": fx, "q": w.q_emb, "x": x}


@pytest.fixture(scope="session")
def rep_flat(tmp_path_factory, repeats):
    """Tie-heavy fp32 index: repeated genome segments give identical vectors, i.e. equal distances."""
    path, fx = _flat(tmp_path_factory, "repflat", repeats["x"], 32)
    return {"index": path, "fx": fx, "q": repeats["q"], "x": repeats["x"]}
