// deepreadmapper_amd/csrc/faiss_io.cpp
//
// Reader/writer for the on-disk index the reference produces and consumes:
//   written by faiss::write_index(&index, index_file)   (src/hnswpq/index.cpp:188)
//   read by    faiss::read_index(index_file) + cast      (src/main.cpp:236-237)
// Layout [faiss impl/index_write.cpp / index_read.cpp, restated], little-endian:
//   u32 "IHNp" | header | HNSW | storage: u32 "IxPq" | header | PQ | vec<u8> codes | i32 search_type
//   | u8 encode_signs | i32 polysemous_ht
//   header = i32 d, i64 ntotal, i64 dummy (1<<20), i64 dummy, u8 is_trained, i32 metric_type,
//            [f32 metric_arg if metric_type > 1]
//   HNSW   = vec<f64> assign_probas, vec<i32> cum_nneighbor_per_level, vec<i32> levels,
//            vec<u64> offsets, vec<i32> neighbors, i32 entry_point, i32 max_level,
//            i32 efConstruction, i32 efSearch, i32 upper_beam
//   PQ     = u64 d, u64 M, u64 nbits, vec<f32> centroids
//   vec<T> = u64 count + count * sizeof(T) bytes
// The faiss version the reference links is unpinned (environment.yml:13), so the loader validates
// every size relation and refuses anything else with a precise message.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <memory>

#include "drm_internal.h"

namespace drm {

static uint32_t fourcc(const char *s)
{
    const unsigned char *x = (const unsigned char *)s;
    return x[0] | x[1] << 8 | x[2] << 16 | x[3] << 24;
}

static std::string fourcc_str(uint32_t h)
{
    char s[5] = {char(h & 0xff), char((h >> 8) & 0xff), char((h >> 16) & 0xff), char((h >> 24) & 0xff), 0};
    for (int i = 0; i < 4; ++i)
        if (s[i] < 32 || s[i] > 126)
            s[i] = '?';
    return s;
}

namespace {
struct Reader {
    std::string path;
    std::vector<uint8_t> buf;
    size_t pos = 0;

    void need(size_t n, const char *what)
    {
        if (pos + n > buf.size() || pos + n < pos)
            throw Error(DRM_ERR_FORMAT, "truncated index file " + path + " while reading " + what + " at byte " +
                                            std::to_string(pos));
    }
    template <class T> T read1(const char *what)
    {
        need(sizeof(T), what);
        T v;
        std::memcpy(&v, buf.data() + pos, sizeof(T));
        pos += sizeof(T);
        return v;
    }
    template <class T> void readvec(std::vector<T> &v, const char *what)
    {
        uint64_t n = read1<uint64_t>(what);
        if (n > (uint64_t(1) << 40) / sizeof(T))
            throw Error(DRM_ERR_FORMAT, std::string("implausible vector size for ") + what + " in " + path);
        need(n * sizeof(T), what);
        v.resize(n);
        if (n)
            std::memcpy(v.data(), buf.data() + pos, n * sizeof(T));
        pos += n * sizeof(T);
    }
    IndexHeader header()
    {
        IndexHeader h;
        h.d = read1<int32_t>("d");
        h.ntotal = read1<int64_t>("ntotal");
        (void)read1<int64_t>("dummy");
        (void)read1<int64_t>("dummy");
        h.is_trained = read1<uint8_t>("is_trained");
        h.metric_type = read1<int32_t>("metric_type");
        if (h.metric_type > 1)
            h.metric_arg = read1<float>("metric_arg");
        return h;
    }
};

struct Writer {
    std::vector<uint8_t> buf;
    template <class T> void write1(const T &v)
    {
        const uint8_t *p = (const uint8_t *)&v;
        buf.insert(buf.end(), p, p + sizeof(T));
    }
    template <class T> void writevec(const std::vector<T> &v)
    {
        write1<uint64_t>(v.size());
        const uint8_t *p = (const uint8_t *)v.data();
        buf.insert(buf.end(), p, p + v.size() * sizeof(T));
    }
    void header(const IndexHeader &h)
    {
        write1<int32_t>(h.d);
        write1<int64_t>(h.ntotal);
        int64_t dummy = 1 << 20;
        write1<int64_t>(dummy);
        write1<int64_t>(dummy);
        write1<uint8_t>(h.is_trained);
        write1<int32_t>(h.metric_type);
        if (h.metric_type > 1)
            write1<float>(h.metric_arg);
    }
};
} // namespace

std::string read_whole_file(const std::string &path)
{
    std::ifstream f(path, std::ios::binary);
    if (!f)
        throw Error(DRM_ERR_IO, "Could not open file: " + path);
    f.seekg(0, std::ios::end);
    std::streamoff n = f.tellg();
    f.seekg(0, std::ios::beg);
    std::string s((size_t)n, '\0');
    if (n > 0)
        f.read(&s[0], n);
    return s;
}

void hnsw_default_probas(int M, std::vector<double> &probas, std::vector<int32_t> &cum)
{
    // HNSW::set_default_probas(M, 1.0 / log(M)) [faiss impl/HNSW.cpp]
    double levelMult = 1.0 / std::log((double)M);
    probas.clear();
    cum.clear();
    int nn = 0;
    cum.push_back(0);
    for (int level = 0;; level++) {
        double proba = std::exp(-level / levelMult) * (1 - std::exp(-1 / levelMult));
        if (proba < 1e-9)
            break;
        probas.push_back(proba);
        nn += level == 0 ? M * 2 : M;
        cum.push_back(nn);
    }
}

void validate_hnswpq(const HnswPqHost &ix)
{
    auto bad = [](const std::string &m) { throw Error(DRM_ERR_FORMAT, "invalid IndexHNSWPQ: " + m); };
    const int64_t n = ix.hdr.ntotal;
    if (ix.hdr.d <= 0)
        bad("d <= 0");
    if (ix.hdr.metric_type != 1)
        bad("metric_type " + std::to_string(ix.hdr.metric_type) + " (only METRIC_L2 = 1 is supported)");
    if (ix.storage_hdr.d != ix.hdr.d || ix.storage_hdr.ntotal != n)
        bad("storage header (d, ntotal) differs from the HNSW header");
    if ((int64_t)ix.levels.size() != n)
        bad("levels.size() = " + std::to_string(ix.levels.size()) + " != ntotal = " + std::to_string(n));
    if ((int64_t)ix.offsets.size() != n + 1)
        bad("offsets.size() != ntotal + 1");
    if (ix.offsets.empty() || ix.offsets[0] != 0 || ix.offsets.back() != ix.neighbors.size())
        bad("offsets.back() != neighbors.size()");
    if (ix.cum_nneighbor_per_level.size() < 2 || ix.cum_nneighbor_per_level[0] != 0)
        bad("cum_nneighbor_per_level malformed");
    for (size_t i = 1; i < ix.cum_nneighbor_per_level.size(); ++i)
        if (ix.cum_nneighbor_per_level[i] < ix.cum_nneighbor_per_level[i - 1])
            bad("cum_nneighbor_per_level not monotone");
    const int nlev = (int)ix.cum_nneighbor_per_level.size() - 1;
    for (int64_t i = 0; i < n; ++i) {
        int l = ix.levels[i];
        if (l < 1 || l > nlev)
            bad("node " + std::to_string(i) + " has levels = " + std::to_string(l));
        if (ix.offsets[i + 1] - ix.offsets[i] != (uint64_t)ix.cum_nneighbor_per_level[l])
            bad("offsets of node " + std::to_string(i) + " disagree with its level");
    }
    for (int32_t v : ix.neighbors)
        if (v < -1 || v >= n)
            bad("neighbor id " + std::to_string(v) + " out of range");
    // a level-l link must point at a node that exists on level l: the search reads the target's
    // level-l list, which is only laid out for nodes with levels[target] > l
    for (int64_t i = 0; i < n; ++i)
        for (int l = 1; l < ix.levels[i]; ++l)
            for (int32_t j = ix.cum_nneighbor_per_level[l]; j < ix.cum_nneighbor_per_level[l + 1]; ++j) {
                const int32_t v = ix.neighbors[ix.offsets[i] + (uint64_t)j];
                if (v >= 0 && ix.levels[v] <= l)
                    bad("node " + std::to_string(i) + " links to node " + std::to_string(v) + " on level " +
                        std::to_string(l) + ", which that node does not reach");
            }
    if (n > 0) {
        if (ix.entry_point < 0 || ix.entry_point >= n)
            bad("entry_point out of range");
        if (ix.max_level < 0 || ix.max_level + 1 > nlev || ix.levels[ix.entry_point] != ix.max_level + 1)
            bad("max_level / entry_point level mismatch");
    } else if (ix.entry_point != -1) {
        bad("empty index with an entry point");
    }
    if (ix.upper_beam != 1)
        bad("upper_beam = " + std::to_string(ix.upper_beam) + " (faiss default 1 expected)");
    if (ix.pq_d != (uint64_t)ix.hdr.d || ix.pq_M == 0 || ix.pq_d % ix.pq_M != 0)
        bad("PQ d / M inconsistent");
    if (ix.pq_nbits < 1 || ix.pq_nbits > 16)
        bad("PQ nbits = " + std::to_string(ix.pq_nbits));
    if (ix.centroids.size() != ix.pq_d * (size_t(1) << ix.pq_nbits))
        bad("centroids.size() != d * 2^nbits");
    if (ix.codes.size() != (size_t)n * (size_t)ix.code_size())
        bad("codes.size() != ntotal * code_size");
}

HnswPqHost read_hnswpq(const std::string &path)
{
    Reader r;
    r.path = path;
    {
        std::string s = read_whole_file(path);
        r.buf.assign(s.begin(), s.end());
    }
    HnswPqHost ix;
    uint32_t h = r.read1<uint32_t>("fourcc");
    if (h != fourcc("IHNp"))
        throw Error(DRM_ERR_FORMAT, "index file " + path + " has fourcc '" + fourcc_str(h) +
                                        "', expected 'IHNp' (faiss::IndexHNSWPQ); dynamic_cast<IndexHNSWPQ*> would fail");
    ix.hdr = r.header();
    r.readvec(ix.assign_probas, "assign_probas");
    r.readvec(ix.cum_nneighbor_per_level, "cum_nneighbor_per_level");
    r.readvec(ix.levels, "levels");
    r.readvec(ix.offsets, "offsets");
    r.readvec(ix.neighbors, "neighbors");
    ix.entry_point = r.read1<int32_t>("entry_point");
    ix.max_level = r.read1<int32_t>("max_level");
    ix.efConstruction = r.read1<int32_t>("efConstruction");
    ix.efSearch = r.read1<int32_t>("efSearch");
    ix.upper_beam = r.read1<int32_t>("upper_beam");
    uint32_t hs = r.read1<uint32_t>("storage fourcc");
    if (hs != fourcc("IxPq"))
        throw Error(DRM_ERR_FORMAT, "IHNp storage has fourcc '" + fourcc_str(hs) + "', expected 'IxPq' (IndexPQ)");
    ix.storage_hdr = r.header();
    ix.pq_d = r.read1<uint64_t>("pq.d");
    ix.pq_M = r.read1<uint64_t>("pq.M");
    ix.pq_nbits = r.read1<uint64_t>("pq.nbits");
    r.readvec(ix.centroids, "pq.centroids");
    r.readvec(ix.codes, "codes");
    ix.search_type = r.read1<int32_t>("search_type");
    ix.encode_signs = r.read1<uint8_t>("encode_signs");
    ix.polysemous_ht = r.read1<int32_t>("polysemous_ht");
    if (r.pos != r.buf.size())
        throw Error(DRM_ERR_FORMAT, "index file " + path + " has " + std::to_string(r.buf.size() - r.pos) +
                                        " trailing bytes after the IndexPQ storage");
    validate_hnswpq(ix);
    return ix;
}

void write_hnswpq(const HnswPqHost &ix, const std::string &path)
{
    validate_hnswpq(ix);
    Writer w;
    w.write1<uint32_t>(fourcc("IHNp"));
    w.header(ix.hdr);
    w.writevec(ix.assign_probas);
    w.writevec(ix.cum_nneighbor_per_level);
    w.writevec(ix.levels);
    w.writevec(ix.offsets);
    w.writevec(ix.neighbors);
    w.write1<int32_t>(ix.entry_point);
    w.write1<int32_t>(ix.max_level);
    w.write1<int32_t>(ix.efConstruction);
    w.write1<int32_t>(ix.efSearch);
    w.write1<int32_t>(ix.upper_beam);
    w.write1<uint32_t>(fourcc("IxPq"));
    w.header(ix.storage_hdr);
    w.write1<uint64_t>(ix.pq_d);
    w.write1<uint64_t>(ix.pq_M);
    w.write1<uint64_t>(ix.pq_nbits);
    w.writevec(ix.centroids);
    w.writevec(ix.codes);
    w.write1<int32_t>(ix.search_type);
    w.write1<uint8_t>(ix.encode_signs);
    w.write1<int32_t>(ix.polysemous_ht);
    std::FILE *f = std::fopen(path.c_str(), "wb");
    if (!f)
        throw Error(DRM_ERR_IO, "Could not create index file: " + path);
    size_t nw = std::fwrite(w.buf.data(), 1, w.buf.size(), f);
    std::fclose(f);
    if (nw != w.buf.size())
        throw Error(DRM_ERR_IO, "short write to " + path);
}

} // namespace drm
