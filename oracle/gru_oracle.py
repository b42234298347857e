"""TEST INFRASTRUCTURE ONLY -- CPU restatement of the reference's read encoder (the checker for the
HIP encoder in deepreadmapper_amd/csrc/encoder_gru.hip; never imported by the product).

Reference path: Vectorizer::vectorize (src/inference/vectorize.cpp:34-141)
  -> Preprocessor::preprocess (src/inference/preprocess.cpp:20-42, hashToken/char2Val
     includes/inference/preprocess.hpp:10-49, _Tok2Index src/utils/tok2index.cpp:3-99)
  -> zero padding to MAX_LEN = 123 positions, [max_len][batch] int64 input
     (vectorize.cpp:345-365, includes/utils/config.hpp:20-22)
  -> FastModel (OpenVINO, src/inference/fast_model.cpp:34-68) running the IR
     models/finetuned_sgn33-new-a-Apr6.xml: Gather(emb [7638, 64] f16->f32) -> GRUSequence
     (bidirectional, hidden 64, linear_before_reset, sigmoid/tanh, h0 = 0) -> GRUSequence (input 128)
     -> concat(final forward h, final backward h) of the second layer = 128-d embedding.
     The graph's TopK / Gather / ScatterElements over the all-equal sequence lengths is a batch
     permutation and its inverse (no effect); every position of the 123 runs (lengths = max_len).

PARITY UNPINNED: OpenVINO is absent here (and no embedding the reference produced ships with it),
so this is a restatement of the IR's published semantics (OpenVINO GRUCell/GRUSequence-5: gate order
z, r, h; B = [Wb_z + Rb_z, Wb_r + Rb_r, Wb_h, Rb_h] under linear_before_reset). The layout reading is
cross-checked against the ONNX export that ships beside the IR (tests/test_encoder_cpu.py). Math is
float64 on the f16-exact weights; the GPU is held to an absolute tolerance (written in the tests).

Tokenizer quirks kept exactly: the first token is hashToken('<', seq[0], seq[1]) with seq[0] the tag
'<' itself (char2Val('<') = 7); a hash > 95 indexes past the 96-entry table in the reference
(undefined behaviour) -- returned here as -1 and mapped to the padding row by the GPU.
"""
import os
import struct
import xml.etree.ElementTree as ET

import numpy as np

MAX_LEN = 123   # Config::Inference::MAX_LEN (includes/utils/config.hpp:21)
HIDDEN = 64
OUT_DIM = 128   # Config::Inference::MODEL_OUT_SIZE

_CV = {ord("a"): 0, ord("c"): 1, ord("g"): 2, ord("t"): 3}


def char2val(c):
    """preprocess.hpp:10-25 (c already lower-cased)."""
    return _CV.get(c, 7)


def hash_token(t0, t1, t2):
    """preprocess.hpp:32-49."""
    if t0 == ord("<"):
        return (char2val(t1) << 2) + char2val(t2)
    if t2 == ord(">"):
        return 16 + (char2val(t0) << 2) + char2val(t1)
    return 32 + (char2val(t0) << 4) + (char2val(t1) << 2) + char2val(t2)


def tok2index():
    """indices_ of Preprocessor (preprocess.cpp:5-18): _Tok2Index (tok2index.cpp:3-99) ordered by hash.
    The vocabulary ids follow the tokenizer's sorted vocabulary: "<xy" -> 7542 + 4x + y, and for the
    pair xy the block 7558 + 5(4x + y) holds "xy>" then "xya".."xyt"."""
    idx = np.zeros(96, dtype=np.int64)
    for x in range(4):
        for y in range(4):
            idx[(x << 2) + y] = 7542 + 4 * x + y
            base = 7558 + 5 * (4 * x + y)
            idx[16 + (x << 2) + y] = base
            for z in range(4):
                idx[32 + (x << 4) + (y << 2) + z] = base + 1 + z
    return idx


_IDX = tok2index()


def _lower(c):
    return c + 32 if 65 <= c <= 90 else c


def preprocess(seq, max_len=MAX_LEN):
    """Preprocessor::preprocess (preprocess.cpp:20-42): token ids of one sequence (bytes), length
    min(max_len, len(seq)); -1 where the reference indexes past its table (hash > 95)."""
    s = bytes(seq)
    if len(s) < 2:
        raise ValueError("sequence shorter than 2 bytes (the reference reads past it)")
    n = min(max_len, len(s))
    lo = [_lower(c) for c in s]
    hashes = [0] * n
    hashes[0] = hash_token(ord("<"), lo[0], lo[1])
    i = 0
    while i < n - 2:
        hashes[i + 1] = hash_token(lo[i], lo[i + 1], lo[i + 2])
        i += 1
    hashes[n - 1] = hash_token(lo[i], lo[i + 1], lo[i + 2] if i + 2 < len(s) else ord(">"))
    return np.array([_IDX[h] if h < 96 else -1 for h in hashes], dtype=np.int64)


def model_input(seqs, max_len=MAX_LEN):
    """[n][max_len] token ids, zero-padded (Vectorizer::prepareBatch, vectorize.cpp:345-365)."""
    out = np.zeros((len(seqs), max_len), dtype=np.int64)
    for r, s in enumerate(seqs):
        t = preprocess(s, max_len)
        out[r, :len(t)] = t
    return out


# ------------------------------------------------------------------------------------- weights
def load_ir(xml_path, bin_path=None):
    """Weights of the IR by following the graph (independent of the product's C++ reader):
    GRUSequence ports 3/4/5 <- Convert <- Const (f16), the embedding Gather's port 0, h0's scalar."""
    bin_path = bin_path or os.path.splitext(xml_path)[0] + ".bin"
    blob = open(bin_path, "rb").read()
    root = ET.parse(xml_path).getroot()
    layers = {l.get("id"): l for l in root.iter("layer")}
    into = {}
    for e in root.iter("edge"):
        into[(e.get("to-layer"), e.get("to-port"))] = e.get("from-layer")

    def const(lid):
        l = layers[lid]
        if l.get("type") == "Convert":
            l = layers[into[(lid, "0")]]
        assert l.get("type") == "Const", l.get("name")
        d = l.find("data")
        dt = {"f16": "<f2", "f32": "<f4", "i64": "<i8"}[d.get("element_type")]
        shape = tuple(int(x) for x in d.get("shape").split(",") if x.strip())
        off, size = int(d.get("offset")), int(d.get("size"))
        a = np.frombuffer(blob[off:off + size], dtype=dt)
        return a.reshape(shape) if shape else a.reshape(())

    grus = sorted((l for l in root.iter("layer") if l.get("type") == "GRUSequence"), key=lambda l: int(l.get("id")))
    assert len(grus) == 2
    w = {}
    for li, g in enumerate(grus):
        d = g.find("data")
        assert d.get("direction") == "bidirectional" and d.get("linear_before_reset") == "true"
        assert int(d.get("hidden_size")) == HIDDEN and d.get("activations").replace(" ", "") == "sigmoid,tanh"
        gid = g.get("id")
        w[f"W{li + 1}"] = const(into[(gid, "3")]).astype(np.float64)
        w[f"R{li + 1}"] = const(into[(gid, "4")]).astype(np.float64)
        w[f"B{li + 1}"] = const(into[(gid, "5")]).astype(np.float64)
    emb_gather = [l for l in root.iter("layer") if l.get("type") == "Gather"
                  and layers[into[(l.get("id"), "1")]].get("type") == "Parameter"]
    assert len(emb_gather) == 1
    w["emb"] = const(into[(emb_gather[0].get("id"), "0")]).astype(np.float64)
    # initial state: GRU port 1 <- Transpose <- StridedSlice <- Gather <- Broadcast(ConstantOfShape) <- scalar
    h0 = []
    for g in grus:
        lid = into[(g.get("id"), "1")]
        while layers[lid].get("type") != "Broadcast":
            lid = into[(lid, "0")]
        h0.append(float(const(into[(lid, "0")])))
    assert h0[0] == h0[1]
    w["h0"] = h0[0]
    return w


def load_drmenc(path):
    """The product's compact weight file (drm_encoder_export, csrc/encoder.cpp)."""
    b = open(path, "rb").read()
    magic, ver, hid, edim, mlen, nrows, nl, _ = struct.unpack_from("<8s7I", b, 0)
    assert magic == b"DRMENC1\0" and ver == 1 and nl == 2
    o = 36
    vocab = np.frombuffer(b, dtype="<u2", count=nrows, offset=o).astype(np.int64)
    o += 2 * nrows
    o = (o + 15) // 16 * 16
    h0 = struct.unpack_from("<f", b, o)[0]
    o += 16
    rows = np.frombuffer(b, dtype="<f2", count=nrows * edim, offset=o).reshape(nrows, edim)
    o += 2 * nrows * edim
    w = {"vocab_rows": vocab, "emb_rows": rows.astype(np.float64), "h0": h0}
    ins = [edim, 2 * hid]
    for li in range(2):
        for name, shape in (("W", (2, 3 * hid, ins[li])), ("R", (2, 3 * hid, hid)), ("B", (2, 4 * hid))):
            cnt = int(np.prod(shape))
            w[f"{name}{li + 1}"] = np.frombuffer(b, dtype="<f2", count=cnt, offset=o).reshape(shape).astype(np.float64)
            o += 2 * cnt
    assert o == len(b)
    return w


def emb_table(w):
    """vocab id -> embedding row, from either source (compact files carry only the reachable rows)."""
    if "emb" in w:
        return lambda ids: w["emb"][ids]
    pos = {int(v): i for i, v in enumerate(w["vocab_rows"])}
    return lambda ids: w["emb_rows"][np.vectorize(pos.__getitem__)(ids)]


# ------------------------------------------------------------------------------------- model
def _sig(x):
    return 1.0 / (1.0 + np.exp(-x))


def gru_direction(X, W, R, B, reverse, h0=0.0):
    """One direction of an OpenVINO GRUSequence with linear_before_reset (GRUCell-3 formulas):
    z = f(x Wz' + h Rz' + bz), r = f(x Wr' + h Rr' + br), n = g(x Wh' + Wbh + r * (h Rh' + Rbh)),
    h = (1 - z) * n + z * h. X [n, L, in]; returns Y [n, L, 64] and the final h [n, 64]."""
    n, L, _ = X.shape
    H = HIDDEN
    h = np.full((n, H), h0, dtype=np.float64)
    Y = np.empty((n, L, H), dtype=np.float64)
    GX = X @ W.T  # [n, L, 3H]
    for s in range(L):
        t = L - 1 - s if reverse else s
        gx = GX[:, t]
        gh = h @ R.T
        z = _sig(gx[:, :H] + gh[:, :H] + B[:H])
        r = _sig(gx[:, H:2 * H] + gh[:, H:2 * H] + B[H:2 * H])
        nn = np.tanh(gx[:, 2 * H:] + B[2 * H:3 * H] + r * (gh[:, 2 * H:] + B[3 * H:]))
        h = (1.0 - z) * nn + z * h
        Y[:, t] = h
    return Y, h


def encode_tokens(w, tokens):
    """tokens [n, L] vocab ids (-1 -> the padding row, as the GPU does) -> embeddings [n, 128] f64."""
    tok = np.where(tokens < 0, 0, tokens)
    X = emb_table(w)(tok)
    h0 = w.get("h0", 0.0)
    yf, _ = gru_direction(X, w["W1"][0], w["R1"][0], w["B1"][0], False, h0)
    yb, _ = gru_direction(X, w["W1"][1], w["R1"][1], w["B1"][1], True, h0)
    Y1 = np.concatenate([yf, yb], axis=2)
    _, hf = gru_direction(Y1, w["W2"][0], w["R2"][0], w["B2"][0], False, h0)
    _, hb = gru_direction(Y1, w["W2"][1], w["R2"][1], w["B2"][1], True, h0)
    return np.concatenate([hf, hb], axis=1)


def vectorize(w, seqs, max_len=MAX_LEN, batch=4096):
    """Vectorizer::vectorize: list of byte strings -> [n, 128] (float64)."""
    out = np.empty((len(seqs), OUT_DIM), dtype=np.float64)
    for b in range(0, len(seqs), batch):
        out[b:b + batch] = encode_tokens(w, model_input(seqs[b:b + batch], max_len))
    return out


# ------------------------------------------------------------------------------------- ONNX
def _varint(b, o):
    v = s = 0
    while True:
        c = b[o]
        o += 1
        v |= (c & 0x7F) << s
        s += 7
        if c < 0x80:
            return v, o


def _fields(b):
    o, out = 0, []
    while o < len(b):
        key, o = _varint(b, o)
        f, wt = key >> 3, key & 7
        if wt == 0:
            v, o = _varint(b, o)
        elif wt == 1:
            v, o = b[o:o + 8], o + 8
        elif wt == 5:
            v, o = b[o:o + 4], o + 4
        elif wt == 2:
            ln, o = _varint(b, o)
            v, o = b[o:o + ln], o + ln
        else:
            raise ValueError("unsupported wire type")
        out.append((f, wt, v))
    return out


def load_onnx_gru(path):
    """Minimal protobuf walk of the ONNX export (ModelProto.graph = 7; GraphProto node = 1,
    initializer = 5; NodeProto input = 1, op_type = 4, attribute = 5; TensorProto dims = 1,
    data_type = 2, name = 8, raw_data = 9): the two GRU nodes' attributes and W/R/B initializers."""
    data = open(path, "rb").read()
    graph = [v for f, _, v in _fields(data) if f == 7][0]
    inits, nodes = {}, []
    for f, _, v in _fields(graph):
        if f == 5:
            dims, dt, name, raw, fl = [], None, None, None, []
            for g, wt, x in _fields(v):
                if g == 1:
                    dims.append(x)
                elif g == 2:
                    dt = x
                elif g == 8:
                    name = x.decode()
                elif g == 9:
                    raw = x
                elif g == 4 and wt == 2:
                    fl = np.frombuffer(x, dtype="<f4")
            if dt == 1:
                a = np.frombuffer(raw, dtype="<f4") if raw is not None else np.asarray(fl, dtype=np.float32)
                inits[name] = a.reshape(dims)
        elif f == 1:
            ins, op, attrs = [], None, {}
            for g, _, x in _fields(v):
                if g == 1:
                    ins.append(x.decode())
                elif g == 4:
                    op = x.decode()
                elif g == 5:
                    an, av = None, None
                    for h, wt, y in _fields(x):
                        if h == 1:
                            an = y.decode()
                        elif h == 3:
                            av = y
                        elif h == 4:
                            av = y.decode()
                    attrs[an] = av
            nodes.append((op, ins, attrs))
    grus = [(ins, attrs) for op, ins, attrs in nodes if op == "GRU"]
    return [{"W": inits.get(i[1]), "R": inits.get(i[2]), "B": inits.get(i[3]) if len(i) > 3 else None,
             "attrs": a} for i, a in grus]
