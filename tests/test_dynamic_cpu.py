"""Dynamic genome lookup (use_dynamic), CPU side:
* drm_extract_fasta_sequence == extract_FASTA_sequence (src/utils/parse_inputs.cpp:174-220): first line
  skipped, whitespace dropped, upper-cased, only A/C/G/T/N kept (later header lines included);
* the oracle's post_process_sw_dynamic equals post_process_sw_static when every window id is inside the
  genome (both cut the same fwd / RC windows), and follows the dynamic rules where they differ."""
import os

import numpy as np

from oracle import oracle as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def extract_ref(data: bytes) -> bytes:
    p = data.find(b"\n")
    p = len(data) if p < 0 else p + 1
    out = bytearray()
    for c in data[p:]:
        if chr(c).isspace():
            continue
        u = chr(c).upper()
        if u in "ACGTN":
            out += u.encode()
    return bytes(out)


def test_extract_fasta_sequence(tmp_path):
    from deepreadmapper_amd import extract_fasta_sequence
    fna = os.path.join(GOLDEN, "ecoli_150.fna")
    assert extract_fasta_sequence(fna) == extract_ref(open(fna, "rb").read())
    odd = b">first header acgt\nacgtNNxx\r\n  ggTT\n>chrA second\nTTAA\n\nn\n"
    (tmp_path / "odd.fa").write_bytes(odd)
    g = extract_fasta_sequence(str(tmp_path / "odd.fa"))
    assert g == extract_ref(odd) == b"ACGTNNGGTTCACNTTAAN"  # ">chrA second" contributes C A C N
    (tmp_path / "hdr.fa").write_bytes(b">only a header")
    assert extract_fasta_sequence(str(tmp_path / "hdr.fa")) == b""


def test_oracle_dynamic_equals_static_inside_genome():
    from deepreadmapper_amd import synth, extract_fasta_sequence
    g = np.frombuffer(extract_fasta_sequence(os.path.join(GOLDEN, "ecoli_150.fna")), dtype=np.uint8)
    refs = synth.windows_lookup(g, 150, 1)
    rng = np.random.default_rng(3)
    reads, _, _ = synth.simulate_reads(g, 40, seed=4)
    q = synth.tag(reads)
    ql = np.full(len(q), q.shape[1], dtype=np.int32)
    nb = rng.integers(0, len(refs), size=(40, 64)).astype(np.int64)
    rs, ss, is_, cs = O.post_process_sw_static(nb, refs, 150, q, ql, 1, 32, 64)
    rd, sd, id_, cd = O.post_process_sw_dynamic(nb, g, 150, q, ql, 1, 32, 64)
    assert rs == rd == 0 and np.array_equal(ss, sd) and np.array_equal(is_, id_) and np.array_equal(cs, cd)
    # where they differ: -1 and past-the-end ids stay candidates (score 0, id kept) in the dynamic lookup
    nb2 = nb.copy()
    nb2[:, 0] = -1
    nb2[:, 1] = len(refs) + 5
    rd, sd, id_, cd = O.post_process_sw_dynamic(nb2, g, 150, q, ql, 1, 64, 64)
    assert rd == 0 and (cd == 64).all()
    for i in range(len(q)):
        row = dict(zip(id_[i].tolist(), sd[i].tolist()))
        assert row[2 ** 64 - 1] == 0 and row[len(refs) + 5] == 0
    rs, _, _, cs = O.post_process_sw_static(nb2, refs, 150, q, ql, 1, 64, 64)
    assert rs < 0  # static drops both ids: 62 < 64 candidates (reranker.cpp:26-29)
