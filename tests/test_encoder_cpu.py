"""Read encoder, CPU side: the oracle's restatement of the reference's
tokenizer and GRU model, pinned where the reference offers anything to pin against, and the product's
IR reader / .drmenc exporter (host-only C-ABI calls, no GPU).

Pins (skipped where /root/reference is absent, i.e. on the GPU box):
* the tokenizer table against models/tok2index.txt (the reference's vocabulary file);
* the IR's W/R/B layout (z, r, h gates; B = [Wb_z + Rb_z, Wb_r + Rb_r, Wb_h, Rb_h]) against the ONNX
  export shipped beside it, read by a minimal protobuf walk (no onnx/OpenVINO here);
* the shipped deepreadmapper_amd/models/*.drmenc against the oracle's own IR walk and against a fresh
  drm_encoder_export of the IR, byte for byte.
The model's output itself is parity unpinned (OpenVINO absent, no reference embeddings ship); as a
semantic check the oracle's embeddings must put C1 reads next to their best-scoring windows."""
import os

import numpy as np
import pytest

from oracle import gru_oracle as G

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_MODELS = "/root/reference/models"
IR = os.path.join(REF_MODELS, "finetuned_sgn33-new-a-Apr6.xml")
SHIPPED = os.path.join(ROOT, "deepreadmapper_amd", "models", "finetuned_sgn33-new-a-Apr6.drmenc")
need_ref = pytest.mark.skipif(not os.path.exists(IR), reason="reference models/ not present (GPU box)")


@need_ref
def test_tok2index_matches_reference_vocabulary():
    pairs = dict(l.split(":") for l in open(os.path.join(REF_MODELS, "tok2index.txt")).read().split())
    assert len(pairs) == 96
    for tok, idx in pairs.items():
        assert G._IDX[G.hash_token(*tok.encode())] == int(idx), tok


def test_preprocess_quirks():
    # tagged read: token 0 = hash('<', '<', 'a') = 28 -> "ta>" (7618); token 1 = "<ac"; 3-mers "acg",
    # "cgt", "gta"; "ta>" from the tag; last = ('a', '>', '>') -> 16 + 0 + char2Val('>') = 23
    t = G.preprocess(b"<ACGTA>")
    assert list(t) == [7618, 7543, G._IDX[38], G._IDX[59], G._IDX[76], G._IDX[28], G._IDX[23]]
    assert len(G.preprocess(b"<" + b"A" * 150 + b">")) == 123          # truncated to MAX_LEN
    assert G.preprocess(b"AC")[-1] == G._IDX[16 + 1]                   # "ac>" (seq end inside the window)
    assert len(G.preprocess(b"AC")) == 2
    assert (G.preprocess(b"<NNNNA>") == -1).any()                      # hash > 95: the reference's UB read
    assert list(G.preprocess(b"acgt")) == list(G.preprocess(b"ACGT"))  # tolower
    with pytest.raises(ValueError):
        G.preprocess(b"A")
    m = G.model_input([b"<ACG>", b"<" + b"T" * 130 + b">"])
    assert m.shape == (2, 123) and (m[0, 5:] == 0).all() and (m[1] != 0).all()


@need_ref
def test_ir_layout_matches_onnx_export():
    w = G.load_ir(IR)
    grus = G.load_onnx_gru(os.path.join(REF_MODELS, "finetuned_sgn33-new-a-Apr6.onnx"))
    H = G.HIDDEN
    assert len(grus) == 2
    for li, g in enumerate(grus):
        assert g["attrs"]["direction"] == b"bidirectional" or g["attrs"]["direction"] == "bidirectional"
        assert g["attrs"]["linear_before_reset"] == 1 and g["attrs"]["hidden_size"] == H
        assert np.array_equal(g["W"].astype(np.float16).astype(np.float64), w[f"W{li + 1}"])
        assert np.array_equal(g["R"].astype(np.float16).astype(np.float64), w[f"R{li + 1}"])
        Wb, Rb = g["B"][:, :3 * H].astype(np.float32), g["B"][:, 3 * H:].astype(np.float32)
        fused = np.concatenate([Wb[:, :H] + Rb[:, :H], Wb[:, H:2 * H] + Rb[:, H:2 * H], Wb[:, 2 * H:], Rb[:, 2 * H:]],
                               axis=1)
        assert np.array_equal(fused.astype(np.float16).astype(np.float64), w[f"B{li + 1}"])
    assert w["h0"] == 0.0


@need_ref
def test_shipped_drmenc_equals_ir(tmp_path):
    from deepreadmapper_amd import export_encoder
    a, b = G.load_ir(IR), G.load_drmenc(SHIPPED)
    for k in ("W1", "R1", "B1", "W2", "R2", "B2"):
        assert np.array_equal(a[k], b[k]), k
    assert b["vocab_rows"][0] == 0 and np.array_equal(b["vocab_rows"][1:], G._IDX)
    assert np.array_equal(b["emb_rows"], a["emb"][b["vocab_rows"]]) and b["h0"] == a["h0"]
    out = tmp_path / "m.drmenc"
    export_encoder(IR, out)
    assert open(out, "rb").read() == open(SHIPPED, "rb").read()
    export_encoder(SHIPPED, tmp_path / "again.drmenc")                 # .drmenc round trip
    assert open(tmp_path / "again.drmenc", "rb").read() == open(SHIPPED, "rb").read()


def test_export_rejects_bad_inputs(tmp_path):
    from deepreadmapper_amd import export_encoder
    from deepreadmapper_amd._native import DrmError, DRM_ERR_IO, DRM_ERR_FORMAT
    with pytest.raises(DrmError) as e:
        export_encoder(tmp_path / "missing.xml", tmp_path / "o.drmenc")
    assert e.value.code == DRM_ERR_IO
    bad = tmp_path / "bad.drmenc"
    bad.write_bytes(b"not an encoder file at all, just bytes" * 4)
    with pytest.raises(DrmError) as e:
        export_encoder(bad, tmp_path / "o.drmenc")
    assert e.value.code == DRM_ERR_FORMAT
    trunc = tmp_path / "trunc.drmenc"
    trunc.write_bytes(open(SHIPPED, "rb").read()[:5000])
    with pytest.raises(DrmError) as e:
        export_encoder(trunc, tmp_path / "o.drmenc")
    assert e.value.code == DRM_ERR_FORMAT


def test_oracle_embeddings_find_source_windows():
    """The decoded model is the trained one: on C1 the nearest window by embedding is the best
    Smith-Waterman window for most reads that come from the genome (best SW >= 100)."""
    from conftest import GOLDEN, read_fastq_tagged
    w = G.load_drmenc(SHIPPED)
    reads = read_fastq_tagged(os.path.join(GOLDEN, "test_data.fastq"))
    refs = [l for l in open(os.path.join(GOLDEN, "test_data_ref.txt"), "rb").read().split(b"\n") if l]
    M = np.load(os.path.join(GOLDEN, "sw_c1_matrix.npy"))
    eq, er = G.vectorize(w, reads), G.vectorize(w, [b"<" + r + b">" for r in refs])
    assert np.abs(eq).max() < 1.0 and np.isfinite(eq).all()
    nn = ((eq[:, None, :] - er[None, :, :]) ** 2).sum(-1).argmin(1)
    mapped = M.max(1) >= 100
    hit = M[np.arange(len(reads)), nn] == M.max(1)
    assert mapped.sum() > 100 and hit[mapped].mean() >= 0.9
