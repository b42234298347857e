"""Writes the committed C1 IHNp fixture, so that a faiss-equipped host can cross-check the search later
(faiss is absent here: SURVEY.md sec. 8c; the reference's call site is src/main.cpp:236-237,278):

  c1_hnswpq.index   faiss IndexHNSWPQ (M_pq=8, nbits=8, M_hnsw=16, EFC=200) over the 1702 C1 windows
                    (tests/ecoli_150.fna, stride 1, fwd/RC interleaved: format_fasta, parse_inputs.cpp:223-369),
                    embedded with the deterministic 3-mer stand-in; built single-threaded by the host builder
                    (drm_build_hnswpq, the hnswpq_index back end), so a rebuild is byte-identical
  c1_queries.npy    [150 x 128] f32: the stand-in embeddings of tests/test_data.fastq's reads, tagged "<read>"
  c1_expected_k128_ef128.npz  I [150 x 128] int64, D [150 x 128] f32 of the oracle restatement
                    (faiss_search(index, queries, 128, 128)), the values a faiss build should reproduce

Cross-check on a faiss host:  index = faiss.read_index("c1_hnswpq.index"); index.hnsw.efSearch = 128;
D, I = index.search(np.load("c1_queries.npy"), 128)  -> compare with the npz (ties: see DESIGN.md sec. 2).
Run from the repo root after `make`: python tests/golden/make_c1_index.py"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))


def build(path):
    from deepreadmapper_amd import synth
    from conftest import read_fastq_tagged
    fna = open(os.path.join(HERE, "ecoli_150.fna"), "rb").read().split(b"\n")
    g = np.frombuffer(b"".join(l.strip() for l in fna[1:]).upper(), dtype=np.uint8)
    x = synth.embed(synth.tag(synth.windows_lookup(g, 150, 1)))
    synth.build_index(x, path, nthreads=1)
    return synth.embed(read_fastq_tagged(os.path.join(HERE, "test_data.fastq")))


def main():
    from oracle import faiss_file, oracle as O
    path = os.path.join(HERE, "c1_hnswpq.index")
    q = build(path)
    np.save(os.path.join(HERE, "c1_queries.npy"), q.astype(np.float32))
    D, I, _, _ = O.hnswpq_search(faiss_file.read(path), q, 128, 128)
    np.savez(os.path.join(HERE, "c1_expected_k128_ef128.npz"), I=I, D=D)
    print("C1 index fixture written")


if __name__ == "__main__":
    main()
