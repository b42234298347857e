// deepreadmapper_amd/csrc/formats.cpp -- host-side formats of the reference path.
//   config.txt   save_config / load_config      src/utils/utils.cpp:505-597
//   .npy         cnpy::npy_save / npy_load       src/utils/utils.cpp:284-285, src/main.cpp:109
//   FASTA        format_fasta (+ reverse_complement) src/utils/parse_inputs.cpp:43-53, :223-369
//   FASTQ        format_fastq                    src/utils/parse_inputs.cpp:843-950
//   .txt         read_txt_mmap                   src/utils/utils.cpp:94-186
#include <array>
#include <cctype>
#include <cstdio>
#include <cstring>
#include <filesystem>
#include <fstream>
#include <sstream>

#include "drm_internal.h"

namespace drm {

// ------------------------------------------------------------------------------ config.txt
void save_config(const std::unordered_map<std::string, ConfigValue> &config, const std::string &folder,
                 const std::string &file)
{
    std::filesystem::create_directories(folder);
    std::string path = folder + "/" + file;
    std::ofstream out(path);
    if (!out)
        throw Error(DRM_ERR_IO, "Could not create config file: " + file);
    // unordered_map iteration order, exactly as utils.cpp:517-533 emits it
    for (const auto &kv : config) {
        out << kv.first << ": ";
        if (std::holds_alternative<size_t>(kv.second))
            out << std::get<size_t>(kv.second);
        else if (std::holds_alternative<float>(kv.second))
            out << std::get<float>(kv.second);
        else
            out << std::get<std::string>(kv.second);
        out << "\n";
    }
}

std::unordered_map<std::string, ConfigValue> load_config(const std::string &path)
{
    std::ifstream in(path);
    if (!in)
        throw Error(DRM_ERR_IO, "Could not open config file: " + path);
    std::unordered_map<std::string, ConfigValue> config;
    std::string line;
    while (std::getline(in, line)) {
        size_t delim = line.find(':');
        if (delim == std::string::npos)
            continue;
        std::string key = line.substr(0, delim);
        std::string val = line.substr(delim + 1);
        key.erase(0, key.find_first_not_of(" \t"));
        key.erase(key.find_last_not_of(" \t") + 1);
        val.erase(0, val.find_first_not_of(" \t"));
        val.erase(val.find_last_not_of(" \t") + 1);
        // size_t, then float, else string (utils.cpp:565-592)
        try {
            size_t idx;
            size_t v = std::stoull(val, &idx);
            if (idx == val.size()) {
                config[key] = v;
                continue;
            }
        } catch (...) {
        }
        try {
            size_t idx;
            float v = std::stof(val, &idx);
            if (idx == val.size()) {
                config[key] = v;
                continue;
            }
        } catch (...) {
        }
        config[key] = val;
    }
    return config;
}

// ------------------------------------------------------------------------------ npy (cnpy layout)
void npy_save(const std::string &path, const void *data, const std::vector<size_t> &shape, char kind, int itemsize)
{
    std::string dict = "{'descr': '<";
    dict += kind;
    dict += std::to_string(itemsize);
    dict += "', 'fortran_order': False, 'shape': (";
    dict += std::to_string(shape.empty() ? 0 : shape[0]);
    for (size_t i = 1; i < shape.size(); i++) {
        dict += ", ";
        dict += std::to_string(shape[i]);
    }
    if (shape.size() == 1)
        dict += ",";
    dict += "), }";
    int remainder = 16 - (10 + (int)dict.size()) % 16; // cnpy pads even when already aligned
    dict.append((size_t)remainder, ' ');
    dict.back() = '\n';
    std::string header;
    header += (char)0x93;
    header += "NUMPY";
    header += (char)0x01;
    header += (char)0x00;
    uint16_t hl = (uint16_t)dict.size();
    header.append((const char *)&hl, 2);
    header += dict;
    size_t nel = 1;
    for (size_t s : shape)
        nel *= s;
    std::FILE *f = std::fopen(path.c_str(), "wb");
    if (!f)
        throw Error(DRM_ERR_IO, "Could not create file: " + path);
    std::fwrite(header.data(), 1, header.size(), f);
    if (nel)
        std::fwrite(data, (size_t)itemsize, nel, f);
    std::fclose(f);
}

NpyArray npy_load(const std::string &path)
{
    std::string s = read_whole_file(path);
    if (s.size() < 10 || (unsigned char)s[0] != 0x93 || s.compare(1, 5, "NUMPY") != 0)
        throw Error(DRM_ERR_FORMAT, "not a .npy file: " + path);
    int major = (unsigned char)s[6];
    size_t hl, off;
    if (major == 1) {
        hl = (unsigned char)s[8] | ((unsigned char)s[9] << 8);
        off = 10;
    } else {
        if (s.size() < 12)
            throw Error(DRM_ERR_FORMAT, "truncated .npy: " + path);
        hl = (unsigned char)s[8] | ((unsigned char)s[9] << 8) | ((unsigned char)s[10] << 16) |
             ((size_t)(unsigned char)s[11] << 24);
        off = 12;
    }
    if (off + hl > s.size())
        throw Error(DRM_ERR_FORMAT, "truncated .npy header: " + path);
    std::string h = s.substr(off, hl);
    NpyArray a;
    size_t p = h.find("'descr'");
    size_t q1 = h.find('\'', h.find(':', p) + 1);
    size_t q2 = h.find('\'', q1 + 1);
    std::string descr = h.substr(q1 + 1, q2 - q1 - 1);
    if (descr.size() < 3 || (descr[0] != '<' && descr[0] != '|'))
        throw Error(DRM_ERR_FORMAT, "unsupported npy descr " + descr);
    a.kind = descr[1];
    a.itemsize = std::stoi(descr.substr(2));
    a.fortran = h.find("'fortran_order': True") != std::string::npos;
    size_t sp = h.find('(', h.find("'shape'"));
    size_t se = h.find(')', sp);
    std::string shp = h.substr(sp + 1, se - sp - 1);
    std::stringstream ss(shp);
    std::string tok;
    while (std::getline(ss, tok, ',')) {
        tok.erase(0, tok.find_first_not_of(" "));
        tok.erase(tok.find_last_not_of(" ") + 1);
        if (!tok.empty())
            a.shape.push_back(std::stoull(tok));
    }
    size_t nel = 1;
    for (size_t d : a.shape)
        nel *= d;
    size_t need = nel * (size_t)a.itemsize;
    if (off + hl + need > s.size())
        throw Error(DRM_ERR_FORMAT, "truncated .npy data: " + path);
    a.bytes.assign(s.begin() + off + hl, s.begin() + off + hl + need);
    return a;
}

// ------------------------------------------------------------------------------ sequences
static const std::array<char, 128> &comp_table()
{
    static const std::array<char, 128> t = [] {
        std::array<char, 128> x{};
        x['A'] = 'T';
        x['T'] = 'A';
        x['C'] = 'G';
        x['G'] = 'C';
        x['N'] = 'N';
        return x;
    }();
    return t;
}

std::string reverse_complement(const std::string &seq)
{
    const auto &t = comp_table();
    std::string rc;
    rc.reserve(seq.size());
    for (auto it = seq.rbegin(); it != seq.rend(); ++it) {
        unsigned char c = (unsigned char)*it;
        rc.push_back(c < 128 ? t[c] : '\0');
    }
    return rc;
}

std::vector<std::string> format_fasta(const std::string &data, size_t ref_len, size_t stride, bool lookup_mode)
{
    // Step 1 (:233-272): contigs = ACGTN letters (upper-cased) after each '>' header line
    std::vector<std::string> contigs;
    std::string cur;
    bool in_seq = false;
    size_t i = 0, n = data.size();
    while (i < n) {
        if (data[i] == '>') {
            if (!cur.empty()) {
                contigs.push_back(std::move(cur));
                cur.clear();
            }
            while (i < n && data[i] != '\n')
                i++;
            if (i < n)
                i++;
            in_seq = true;
            continue;
        }
        if (in_seq) {
            char c = data[i];
            if (!std::isspace((unsigned char)c)) {
                c = (char)std::toupper((unsigned char)c);
                if (c == 'A' || c == 'T' || c == 'C' || c == 'G' || c == 'N')
                    cur.push_back(c);
            }
        }
        i++;
    }
    if (!cur.empty())
        contigs.push_back(std::move(cur));
    // Step 4 (:325-362): per contig, window i at i*stride, forward then reverse complement
    std::vector<std::string> out;
    for (const auto &seq : contigs) {
        if (seq.size() < ref_len)
            continue;
        size_t nw = (seq.size() - ref_len) / stride + 1;
        for (size_t w = 0; w < nw; ++w) {
            std::string win = seq.substr(w * stride, ref_len);
            std::string rev = reverse_complement(win);
            if (!lookup_mode) {
                out.push_back("<" + win + ">");
                out.push_back("<" + rev + ">");
            } else {
                out.push_back(win);
                out.push_back(rev);
            }
        }
    }
    return out;
}

void format_fastq(const std::string &data, std::vector<std::string> &seqs, std::vector<std::string> &ids)
{
    const char *cur = data.data();
    const char *end = cur + data.size();
    int line = 0;
    while (cur < end) {
        const char *ls = cur;
        while (cur < end && *cur != '\n')
            cur++;
        if (line % 4 == 0) {
            const char *hs = ls;
            if (hs < cur && *hs == '@')
                hs++;
            const char *ie = hs;
            while (ie < cur && *ie != ' ' && *ie != '\t' && *ie != '/')
                ie++;
            ids.emplace_back(hs, ie - hs);
        } else if (line % 4 == 1) {
            std::string s;
            s.reserve((size_t)(cur - ls) + 2);
            s += '<';
            s.append(ls, cur - ls);
            s += '>';
            seqs.push_back(std::move(s));
        }
        if (cur < end)
            cur++;
        line++;
    }
}

void read_file(const std::string &path, std::vector<std::string> &seqs, std::vector<std::string> &ids,
               size_t ref_len, size_t stride, bool lookup_mode)
{
    std::string ext = std::filesystem::path(path).extension().string();
    if (ext != ".fna" && ext != ".fasta" && ext != ".fa" && ext != ".fastq" && ext != ".fq" && ext != ".txt")
        throw Error(DRM_ERR_ARG, "Unsupported file format: " + ext + ". Only .fna/.fastq/.txt are supported.");
    std::string data = read_whole_file(path);
    seqs.clear();
    ids.clear();
    if (ext == ".fna" || ext == ".fasta" || ext == ".fa") {
        seqs = format_fasta(data, ref_len, stride, lookup_mode);
        return;
    }
    if (ext == ".fastq" || ext == ".fq") {
        format_fastq(data, seqs, ids);
        return;
    }
    // read_txt_mmap (utils.cpp:140-165): non-empty lines, split on '\n' / '\r'
    const char *c = data.data(), *e = c + data.size();
    while (c < e) {
        const char *ls = c;
        while (c < e && *c != '\n' && *c != '\r')
            c++;
        if (c > ls)
            seqs.emplace_back(ls, c - ls);
        while (c < e && (*c == '\n' || *c == '\r'))
            c++;
    }
}

} // namespace drm

// ----------------------------------------------------------------------- extract_FASTA_sequence
std::string drm::extract_fasta_sequence(const std::string &path)
{
    const std::string data = read_whole_file(path);
    size_t p = data.find('\n');
    p = p == std::string::npos ? data.size() : p + 1; // skip the first (header) line
    std::string g;
    g.reserve(data.size() - p);
    for (; p < data.size(); ++p) {
        const unsigned char c = (unsigned char)data[p];
        if (std::isspace(c))
            continue;
        const char u = (char)std::toupper(c);
        if (u == 'A' || u == 'T' || u == 'C' || u == 'G' || u == 'N')
            g.push_back(u);
    }
    return g;
}

// ----------------------------------------------------------------------- SAM (write_sam)
void drm::write_sam_block(const std::string &path, bool header, const std::string &ref_name, size_t ref_len,
                          const std::vector<std::string> &query_seqs, const std::vector<std::string> &query_ids,
                          size_t q0, size_t nq, const uint64_t *ids, const int32_t *counts, size_t k)
{
    std::ofstream out(path, header ? std::ios::out : std::ios::app);
    if (!out.is_open())
        throw Error(DRM_ERR_IO, "Failed to open SAM file: " + path);
    if (header) {
        out << "@HD\tVN:1.0\tSO:unsorted\n";
        out << "@SQ\tSN:" << ref_name << "\tLN:" << ref_len << "\n";
    }
    std::string buf;
    for (size_t i = 0; i < nq; ++i) {
        const size_t g = q0 + i;
        std::string clean = query_seqs[g]; // PREFIX "<" / POSTFIX ">" stripped (parse_inputs.hpp:10-11)
        if (clean.size() > 2)
            clean = clean.substr(1, clean.size() - 2);
        const std::string qname = (g < query_ids.size() && !query_ids[g].empty()) ? query_ids[g]
                                                                                  : "S1/" + std::to_string(g + 1) + "/0";
        const std::string cigar = std::to_string(clean.size()) + "M";
        for (int j = 0; j < counts[i] && (size_t)j < k; ++j) {
            const uint64_t sid = ids[i * k + (size_t)j];
            int flag = j == 0 ? 0 : 256; // primary / secondary
            if (sid % 2 == 1)
                flag |= 16; // reverse complement
            buf += qname;
            buf += '\t';
            buf += std::to_string(flag);
            buf += '\t';
            buf += ref_name;
            buf += '\t';
            buf += std::to_string(sid / 2 + 1); // 1-based position
            buf += "\t60\t";
            buf += cigar;
            buf += "\t*\t0\t0\t";
            buf += clean;
            buf += "\t*\n";
        }
        if (buf.size() > (1u << 22)) {
            out << buf;
            buf.clear();
        }
    }
    out << buf;
}

extern "C" int drm_extract_fasta_sequence(const char *path, uint8_t *out, int64_t *len)
{
    try {
        if (!path || !len)
            throw drm::Error(DRM_ERR_ARG, "null argument");
        const std::string g = drm::extract_fasta_sequence(path);
        if (out)
            std::memcpy(out, g.data(), std::min<size_t>(g.size(), (size_t)std::max<int64_t>(*len, 0)));
        *len = (int64_t)g.size();
        return DRM_OK;
    } catch (const drm::Error &e) {
        drm::set_last_error(e.what());
        return e.code;
    } catch (const std::exception &e) {
        drm::set_last_error(e.what());
        return DRM_ERR_IO;
    }
}
