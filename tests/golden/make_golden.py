"""Regenerates the committed golden vectors from the reference's own code, built here.

  sw_kat.json          calc_sw_score (reference src/utils/metrics.cpp, compiled in place by
                       oracle/Makefile -> oracle/_ref/libdrm_ref.so): the reference harness pairing
                       of src/test_sw_score.cpp:45-51 (100 consecutive pairs of test_data_quer.txt),
                       edge cases, and seeded random ragged pairs.
  sw_c1_matrix.npy     int16 [150 reads x 1702 windows]: calc_sw_score(window, "<"+read+">") for the
                       C1 fixture (test_data.fastq x test_data_ref.txt), the post_process_sw_static call.
  partial_sort.json    libstdc++ std::partial_sort orders for the reranker's comparator
                       (src/utils/reranker.cpp:38-40), from oracle/libstl_sort.so.
Run from the repo root after `make -C oracle`: python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import oracle as O  # noqa: E402


def main():
    if not O.ref_available():
        sys.exit("oracle/_ref/libdrm_ref.so missing (needs /root/reference): run make -C oracle")
    quer = [l.strip().encode() for l in open(os.path.join(HERE, "test_data_quer.txt"), "rb").read().decode().splitlines() if l.strip()]
    kat = {"harness_pairs": [[i, i + 1] for i in range(100)],
           "harness_scores": [O.ref_calc_sw_score(quer[i], quer[i + 1]) for i in range(100)]}
    edges = [("", "ACGT"), ("ACGT", ""), ("", ""), ("NNNN", "NNNN"), ("acgt", "ACGT"), ("ACGTTACGT", "ACGTACGT"),
             ("ACGTAACGT", "ACGTCACGT"), ("A", "A"), ("A", "C"), ("<ACGT>", "<ACGT>"), ("ACGT", "<ACGT>"),
             (quer[0].decode(), quer[0].decode()), (quer[0].decode(), "<" + quer[0].decode() + ">"),
             ("G" * 150, "C" * 150), ("AT" * 75, "TA" * 76)]
    kat["edge_cases"] = [[a, b, O.ref_calc_sw_score(a.encode(), b.encode())] for a, b in edges]
    rng = np.random.default_rng(2024)
    rnd = []
    for _ in range(300):
        l1, l2 = int(rng.integers(0, 200)), int(rng.integers(0, 250))
        alpha = b"ACGTN<>a"[: int(rng.integers(2, 9))]
        a = bytes(rng.choice(list(alpha), size=l1).astype(np.uint8)) if l1 else b""
        b = bytes(rng.choice(list(alpha), size=l2).astype(np.uint8)) if l2 else b""
        rnd.append([a.decode(), b.decode(), O.ref_calc_sw_score(a, b)])
    kat["random_pairs"] = rnd
    with open(os.path.join(HERE, "sw_kat.json"), "w") as f:
        json.dump(kat, f)

    ref = [l.strip() for l in open(os.path.join(HERE, "test_data_ref.txt"), "rb") if l.strip()]
    fq = open(os.path.join(HERE, "test_data.fastq"), "rb").read().split(b"\n")
    reads = [b"<" + fq[i + 1] + b">" for i in range(0, len(fq) - 1, 4) if fq[i].startswith(b"@")]
    mat = np.array([[O.ref_calc_sw_score(w, r) for w in ref] for r in reads], dtype=np.int16)
    np.save(os.path.join(HERE, "sw_c1_matrix.npy"), mat)

    cases = []
    for t in range(200):
        n = int(rng.integers(1, 400))
        k = int(rng.integers(1, n + 1)) if t % 3 else n
        s = rng.integers(0, int(rng.integers(1, 40)), size=n).astype(np.int32)
        cases.append({"scores": s.tolist(), "k": k, "order": O.stl_partial_sort_desc(s, k).tolist()})
    with open(os.path.join(HERE, "partial_sort.json"), "w") as f:
        json.dump(cases, f)
    print("golden vectors written")


if __name__ == "__main__":
    main()
