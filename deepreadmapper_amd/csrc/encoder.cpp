// deepreadmapper_amd/csrc/encoder.cpp -- host side of the read encoder.
//
// Reads the reference's OpenVINO IR (models/finetuned_sgn33-new-a-Apr6.xml + .bin, loaded by
// FastModel, src/inference/fast_model.cpp:3-29) by following its graph, or this library's compact
// .drmenc file (the same f16 tensors, only the 97 embedding rows the tokenizer can reach).
// Graph contract (checked, anything else is DRM_ERR_UNSUPPORTED):
//   Parameter [max_len, batch] i64 -> Gather(emb [V, 64] f16) -> GRUSequence(bidirectional, hidden 64,
//   linear_before_reset, sigmoid/tanh, clip 0; W/R/B f16 Consts through Convert) -> GRUSequence
//   (input 128) -> final hidden states; h0 = a scalar Const broadcast (ConstantOfShape).
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <map>
#include <sstream>

#include "drm_internal.h"

namespace drm {

namespace {

using Attrs = std::map<std::string, std::string>;

// attributes of the tag starting at s[pos] ('<'), up to its '>'
Attrs parse_tag(const std::string &s, size_t pos, size_t *end) {
    Attrs a;
    size_t e = s.find('>', pos);
    if (e == std::string::npos) throw Error(DRM_ERR_FORMAT, "IR: unterminated tag");
    size_t i = s.find_first_of(" \t\r\n", pos);
    while (i < e) {
        while (i < e && isspace((unsigned char)s[i])) ++i;
        size_t eq = s.find('=', i);
        if (eq == std::string::npos || eq > e) break;
        std::string key = s.substr(i, eq - i);
        size_t q0 = s.find('"', eq), q1 = q0 == std::string::npos ? q0 : s.find('"', q0 + 1);
        if (q1 == std::string::npos || q1 > e) throw Error(DRM_ERR_FORMAT, "IR: bad attribute " + key);
        a[key] = s.substr(q0 + 1, q1 - q0 - 1);
        i = q1 + 1;
    }
    if (end) *end = e;
    return a;
}

struct IrLayer {
    Attrs attr, data;
};

std::vector<int64_t> parse_shape(const std::string &s) {
    std::vector<int64_t> v;
    std::stringstream ss(s);
    std::string tok;
    while (std::getline(ss, tok, ','))
        if (tok.find_first_not_of(" ") != std::string::npos) v.push_back(std::stoll(tok));
    return v;
}

std::string read_all(const std::string &path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw Error(DRM_ERR_IO, "cannot open " + path);
    std::ostringstream ss;
    ss << f.rdbuf();
    return ss.str();
}

float f16_bits_to_f32(uint16_t b) {
    const uint32_t sign = uint32_t(b >> 15) << 31, ex = (b >> 10) & 31, man = b & 1023;
    uint32_t u;
    if (ex == 31) u = sign | 0x7f800000u | (man << 13);
    else if (ex) u = sign | ((ex + 112) << 23) | (man << 13);
    else if (!man) u = sign;
    else { // subnormal: man * 2^-24
        float f = float(man) * 5.9604644775390625e-8f;
        memcpy(&u, &f, 4);
        u |= sign;
    }
    float f;
    memcpy(&f, &u, 4);
    return f;
}

struct Ir {
    std::map<std::string, IrLayer> layers;
    std::map<std::pair<std::string, std::string>, std::string> into; // (to-layer, to-port) -> from-layer
    std::string blob;

    const IrLayer &layer(const std::string &id) const {
        auto it = layers.find(id);
        if (it == layers.end()) throw Error(DRM_ERR_FORMAT, "IR: missing layer " + id);
        return it->second;
    }
    std::string src(const std::string &id, const char *port) const {
        auto it = into.find({id, port});
        if (it == into.end()) throw Error(DRM_ERR_FORMAT, "IR: layer " + id + " port " + port + " unconnected");
        return it->second;
    }
    // f16 Const (directly or through a Convert): shape + raw bits
    std::vector<uint16_t> const_f16(const std::string &id0, std::vector<int64_t> *shape) const {
        std::string id = id0;
        if (layer(id).attr.at("type") == "Convert") id = src(id, "0");
        const IrLayer &c = layer(id);
        if (c.attr.at("type") != "Const") throw Error(DRM_ERR_UNSUPPORTED, "IR: expected a Const at layer " + id);
        if (c.data.at("element_type") != "f16")
            throw Error(DRM_ERR_UNSUPPORTED, "IR: weights must be f16-compressed (layer " + c.attr.at("name") + ")");
        *shape = parse_shape(c.data.at("shape"));
        int64_t off = std::stoll(c.data.at("offset")), size = std::stoll(c.data.at("size"));
        int64_t cnt = 1;
        for (int64_t d : *shape) cnt *= d;
        if (size != 2 * cnt || off < 0 || off + size > (int64_t)blob.size())
            throw Error(DRM_ERR_FORMAT, "IR: Const " + c.attr.at("name") + " outside the .bin");
        std::vector<uint16_t> v(cnt);
        memcpy(v.data(), blob.data() + off, size);
        return v;
    }
};

Ir parse_ir(const std::string &xml_path) {
    Ir ir;
    std::string s = read_all(xml_path);
    std::string bin = xml_path.substr(0, xml_path.size() - 4) + ".bin";
    ir.blob = read_all(bin);
    size_t pos = 0;
    while ((pos = s.find("<layer ", pos)) != std::string::npos) {
        size_t e;
        IrLayer L;
        L.attr = parse_tag(s, pos, &e);
        size_t close = s.find("</layer>", e);
        size_t self_close = s[e - 1] == '/' ? e : std::string::npos;
        size_t stop = self_close != std::string::npos ? e : close;
        size_t d = s.find("<data", e);
        if (d != std::string::npos && d < stop) L.data = parse_tag(s, d, nullptr);
        if (!L.attr.count("id") || !L.attr.count("type")) throw Error(DRM_ERR_FORMAT, "IR: layer without id/type");
        ir.layers[L.attr["id"]] = L;
        pos = e;
    }
    pos = 0;
    while ((pos = s.find("<edge ", pos)) != std::string::npos) {
        size_t e;
        Attrs a = parse_tag(s, pos, &e);
        ir.into[{a.at("to-layer"), a.at("to-port")}] = a.at("from-layer");
        pos = e;
    }
    if (ir.layers.empty()) throw Error(DRM_ERR_FORMAT, "IR: no layers in " + xml_path);
    return ir;
}

void expect_shape(const std::vector<int64_t> &got, std::initializer_list<int64_t> want, const char *what) {
    if (!std::equal(got.begin(), got.end(), want.begin(), want.end()))
        throw Error(DRM_ERR_UNSUPPORTED, std::string("IR: unexpected shape of ") + what);
}

EncoderHost from_ir(const std::string &xml_path) {
    Ir ir = parse_ir(xml_path);
    std::vector<std::string> grus;
    for (auto &kv : ir.layers)
        if (kv.second.attr.at("type") == "GRUSequence") grus.push_back(kv.first);
    std::sort(grus.begin(), grus.end(), [](const std::string &a, const std::string &b) { return std::stoi(a) < std::stoi(b); });
    if (grus.size() != 2) throw Error(DRM_ERR_UNSUPPORTED, "IR: expected two GRUSequence layers");
    EncoderHost e;
    for (int l = 0; l < 2; ++l) {
        const Attrs &d = ir.layer(grus[l]).data;
        std::string act = d.count("activations") ? d.at("activations") : "";
        act.erase(std::remove(act.begin(), act.end(), ' '), act.end());
        if (d.at("direction") != "bidirectional" || d.at("linear_before_reset") != "true" ||
            std::stoi(d.at("hidden_size")) != e.hidden || act != "sigmoid,tanh" ||
            (d.count("clip") && std::stof(d.at("clip")) != 0.f))
            throw Error(DRM_ERR_UNSUPPORTED, "IR: GRUSequence attributes differ from the supported model");
        std::vector<int64_t> sw, sr, sb;
        e.W[l] = ir.const_f16(ir.src(grus[l], "3"), &sw);
        e.R[l] = ir.const_f16(ir.src(grus[l], "4"), &sr);
        e.B[l] = ir.const_f16(ir.src(grus[l], "5"), &sb);
        expect_shape(sw, {2, 3 * e.hidden, e.in_dim(l)}, "GRU W");
        expect_shape(sr, {2, 3 * e.hidden, e.hidden}, "GRU R");
        expect_shape(sb, {2, 4 * e.hidden}, "GRU B");
        // h0: port 1 <- Transpose <- StridedSlice <- Gather <- Broadcast(scalar)
        std::string id = ir.src(grus[l], "1");
        for (int hop = 0; ir.layer(id).attr.at("type") != "Broadcast"; ++hop) {
            if (hop > 8) throw Error(DRM_ERR_UNSUPPORTED, "IR: initial state is not a broadcast constant");
            id = ir.src(id, "0");
        }
        std::vector<int64_t> s0;
        auto h0 = ir.const_f16(ir.src(id, "0"), &s0);
        if (!s0.empty() || h0.size() != 1) throw Error(DRM_ERR_UNSUPPORTED, "IR: initial state is not a scalar");
        float v = f16_bits_to_f32(h0[0]);
        if (l == 1 && v != e.h0) throw Error(DRM_ERR_UNSUPPORTED, "IR: layers have different initial states");
        e.h0 = v;
    }
    std::string emb_id;
    for (auto &kv : ir.layers)
        if (kv.second.attr.at("type") == "Gather" && ir.into.count({kv.first, "1"}) &&
            ir.layer(ir.src(kv.first, "1")).attr.at("type") == "Parameter")
            emb_id = ir.src(kv.first, "0");
    if (emb_id.empty()) throw Error(DRM_ERR_UNSUPPORTED, "IR: no embedding Gather on the input");
    std::vector<int64_t> se;
    std::vector<uint16_t> emb = ir.const_f16(emb_id, &se);
    if (se.size() != 2 || se[1] != e.emb_dim) throw Error(DRM_ERR_UNSUPPORTED, "IR: embedding table is not [V, 64]");
    const int64_t V = se[0];
    std::vector<uint16_t> vocab = token_vocab_rows();
    e.vocab_rows = vocab;
    e.emb_rows.resize(vocab.size() * e.emb_dim);
    for (size_t r = 0; r < vocab.size(); ++r) {
        if (vocab[r] >= V) throw Error(DRM_ERR_UNSUPPORTED, "IR: embedding table smaller than the vocabulary");
        memcpy(&e.emb_rows[r * e.emb_dim], &emb[(size_t)vocab[r] * e.emb_dim], 2 * e.emb_dim);
    }
    return e;
}

constexpr char kMagic[8] = {'D', 'R', 'M', 'E', 'N', 'C', '1', '\0'};

EncoderHost from_drmenc(const std::string &path) {
    std::string b = read_all(path);
    if (b.size() < 36 || memcmp(b.data(), kMagic, 8) != 0) throw Error(DRM_ERR_FORMAT, path + " is not a .drmenc file");
    uint32_t h[7];
    memcpy(h, b.data() + 8, sizeof h);
    EncoderHost e;
    if (h[0] != 1 || (int)h[1] != e.hidden || (int)h[2] != e.emb_dim || (int)h[3] != e.max_len || h[5] != 2)
        throw Error(DRM_ERR_UNSUPPORTED, path + ": unsupported encoder shape");
    const size_t nrows = h[4];
    size_t o = 36;
    auto take = [&](void *dst, size_t n) {
        if (o + n > b.size()) throw Error(DRM_ERR_FORMAT, path + " is truncated");
        memcpy(dst, b.data() + o, n);
        o += n;
    };
    e.vocab_rows.resize(nrows);
    take(e.vocab_rows.data(), 2 * nrows);
    o = (o + 15) / 16 * 16;
    float h0[4];
    take(h0, 16);
    e.h0 = h0[0];
    e.emb_rows.resize(nrows * e.emb_dim);
    take(e.emb_rows.data(), 2 * e.emb_rows.size());
    for (int l = 0; l < 2; ++l) {
        e.W[l].resize(2 * 3 * e.hidden * e.in_dim(l));
        e.R[l].resize(2 * 3 * e.hidden * e.hidden);
        e.B[l].resize(2 * 4 * e.hidden);
        take(e.W[l].data(), 2 * e.W[l].size());
        take(e.R[l].data(), 2 * e.R[l].size());
        take(e.B[l].data(), 2 * e.B[l].size());
    }
    if (o != b.size()) throw Error(DRM_ERR_FORMAT, path + " has trailing bytes");
    if (e.vocab_rows != token_vocab_rows()) throw Error(DRM_ERR_UNSUPPORTED, path + ": token table differs");
    return e;
}

bool ends_with(const std::string &s, const char *suf) {
    size_t n = strlen(suf);
    return s.size() >= n && s.compare(s.size() - n, n, suf) == 0;
}

} // namespace

std::vector<uint16_t> token_vocab_rows() {
    // row 0: vocabulary id 0 (the padding of Vectorizer::prepareBatch, vectorize.cpp:351);
    // row 1 + h: indices_[h] of Preprocessor (preprocess.cpp:5-18 over _Tok2Index, tok2index.cpp:3-99):
    // "<xy" = 7542 + 4x + y; for the pair xy the block 7558 + 5(4x + y) holds "xy>", then "xya".."xyt".
    std::vector<uint16_t> v(1 + kTokenHashes, 0);
    for (int x = 0; x < 4; ++x)
        for (int y = 0; y < 4; ++y) {
            v[1 + (x << 2) + y] = uint16_t(7542 + 4 * x + y);
            const int base = 7558 + 5 * (4 * x + y);
            v[1 + 16 + (x << 2) + y] = uint16_t(base);
            for (int z = 0; z < 4; ++z) v[1 + 32 + (x << 4) + (y << 2) + z] = uint16_t(base + 1 + z);
        }
    return v;
}

std::string encoder_model_path() {
    if (const char *e = std::getenv("DRM_ENCODER")) {
        std::string v(e);
        return v == "kmer3" ? std::string() : v;
    }
    const char *ref_model = "models/finetuned_sgn33-new-a-Apr6.xml";
    std::ifstream f(ref_model);
    return f ? std::string(ref_model) : std::string();
}

void vectorize_host(const std::string &model, int device, const std::vector<std::string> &seqs, float *out) {
    drm_encoder *enc = nullptr;
    auto chk = [](int rc) {
        if (rc != DRM_OK) throw Error(rc, drm_last_error());
    };
    chk(drm_encoder_load(model.c_str(), device, &enc));
    try {
        size_t stride = 2;
        for (auto &q : seqs) stride = std::max(stride, q.size());
        std::vector<uint8_t> buf(seqs.size() * stride, 0);
        std::vector<int32_t> lens(seqs.size());
        for (size_t i = 0; i < seqs.size(); ++i) {
            memcpy(&buf[i * stride], seqs[i].data(), seqs[i].size());
            lens[i] = (int32_t)seqs[i].size();
        }
        int64_t undef = 0;
        chk(drm_vectorize(enc, buf.data(), lens.data(), (int64_t)seqs.size(), (int64_t)stride, out, &undef));
        if (undef)
            std::cerr << "[INFERENCE] warning: " << undef
                      << " tokens hash past the 96-entry token table (undefined in the reference; encoded as padding)"
                      << std::endl;
    } catch (...) {
        drm_encoder_free(enc);
        throw;
    }
    chk(drm_encoder_free(enc));
}

EncoderHost read_encoder(const std::string &path) {
    if (ends_with(path, ".xml")) return from_ir(path);
    return from_drmenc(path);
}

void write_encoder(const EncoderHost &e, const std::string &path) {
    std::ofstream f(path, std::ios::binary);
    if (!f) throw Error(DRM_ERR_IO, "cannot write " + path);
    uint32_t h[7] = {1, uint32_t(e.hidden), uint32_t(e.emb_dim), uint32_t(e.max_len), uint32_t(e.vocab_rows.size()), 2, 0};
    std::string out(kMagic, 8);
    out.append((const char *)h, sizeof h);
    out.append((const char *)e.vocab_rows.data(), 2 * e.vocab_rows.size());
    out.resize((out.size() + 15) / 16 * 16, '\0');
    float h0[4] = {e.h0, 0.f, 0.f, 0.f};
    out.append((const char *)h0, sizeof h0);
    out.append((const char *)e.emb_rows.data(), 2 * e.emb_rows.size());
    for (int l = 0; l < 2; ++l) {
        out.append((const char *)e.W[l].data(), 2 * e.W[l].size());
        out.append((const char *)e.R[l].data(), 2 * e.R[l].size());
        out.append((const char *)e.B[l].data(), 2 * e.B[l].size());
    }
    f.write(out.data(), out.size());
    if (!f) throw Error(DRM_ERR_IO, "short write to " + path);
}

} // namespace drm
