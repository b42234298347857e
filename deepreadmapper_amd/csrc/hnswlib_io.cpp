// deepreadmapper_amd/csrc/hnswlib_io.cpp
//
// Reader/writer for hnswlib's index file (the reference's fp32-L2 backend):
//   written by HierarchicalNSW<float>::saveIndex(index_file)      (src/hnswlib_dir/index.cpp:47)
//   read by    new HierarchicalNSW<float>(&space, index_file)      (src/hnswlib_dir/test_search.cpp:33)
// Layout [upstream hnswlib saveIndex/loadIndex, restated], little-endian:
//   size_t offsetLevel0 (0), max_elements, cur_element_count, size_data_per_element, label_offset,
//   offsetData; int maxlevel; u32 enterpoint_node; size_t maxM, maxM0, M; double mult;
//   size_t ef_construction;
//   cur_element_count level-0 records, each size_data_per_element bytes:
//     u32 linklist header (count in the low 16 bits, delete mark in byte 2) | maxM0 u32 links
//     | d f32 (the vector) | u64 label
//   then per element: u32 byte size of its upper-level blocks (level * (4 + 4*maxM), 0 if level 0)
//   and the blocks, each u32 header + maxM u32 links, block l-1 holding level l.
// hnswlib's commit is unpinned (an absent submodule, .gitmodules:1-3), so the loader checks every
// size relation and rejects deleted elements, which the search path does not support.
#include <cstring>
#include <fstream>

#include "drm_internal.h"

namespace drm {

namespace {
struct Buf {
    std::string path;
    std::vector<uint8_t> b;
    size_t pos = 0;
    template <class T> T get(const char *what)
    {
        if (pos + sizeof(T) > b.size())
            throw Error(DRM_ERR_FORMAT, "truncated hnswlib index " + path + " while reading " + what);
        T v;
        std::memcpy(&v, b.data() + pos, sizeof(T));
        pos += sizeof(T);
        return v;
    }
};
} // namespace

HnswFlatHost read_hnswlib(const std::string &path)
{
    Buf r;
    r.path = path;
    {
        std::ifstream f(path, std::ios::binary);
        if (!f)
            throw Error(DRM_ERR_IO, "cannot open index file " + path);
        f.seekg(0, std::ios::end);
        r.b.resize((size_t)f.tellg());
        f.seekg(0);
        f.read((char *)r.b.data(), (std::streamsize)r.b.size());
    }
    HnswFlatHost ix;
    const uint64_t off_l0 = r.get<uint64_t>("offsetLevel0");
    ix.max_elements = r.get<uint64_t>("max_elements");
    const uint64_t n = r.get<uint64_t>("cur_element_count");
    const uint64_t sz_el = r.get<uint64_t>("size_data_per_element");
    const uint64_t label_off = r.get<uint64_t>("label_offset");
    const uint64_t off_data = r.get<uint64_t>("offsetData");
    ix.maxlevel = r.get<int32_t>("maxlevel");
    ix.ep = r.get<uint32_t>("enterpoint_node");
    ix.maxM = r.get<uint64_t>("maxM");
    ix.maxM0 = r.get<uint64_t>("maxM0");
    ix.M = r.get<uint64_t>("M");
    ix.mult = r.get<double>("mult");
    ix.efc = r.get<uint64_t>("ef_construction");
    auto bad = [&](const std::string &m) { return Error(DRM_ERR_FORMAT, "hnswlib index " + path + ": " + m); };
    if (off_l0 != 0)
        throw bad("offsetLevel0 != 0");
    if (ix.maxM0 == 0 || ix.maxM0 > 65535 || ix.maxM == 0 || ix.maxM > 65535)
        throw bad("implausible maxM/maxM0");
    if (off_data != 4 * (1 + ix.maxM0))
        throw bad("offsetData != 4 * (1 + maxM0)");
    if (label_off <= off_data || (label_off - off_data) % 4 != 0)
        throw bad("bad label_offset");
    if (sz_el != label_off + 8)
        throw bad("size_data_per_element != label_offset + 8");
    if (n > ix.max_elements)
        throw bad("cur_element_count > max_elements");
    ix.d = (int32_t)((label_off - off_data) / 4);
    ix.n = (int64_t)n;
    if (n > 0 && (ix.ep >= n || ix.maxlevel < 0))
        throw bad("entry point out of range");
    if (r.pos + n * sz_el > r.b.size())
        throw bad("truncated level-0 data");
    ix.vec.resize(n * (size_t)ix.d);
    ix.l0.resize(n * (1 + ix.maxM0));
    ix.labels.resize(n);
    for (uint64_t i = 0; i < n; ++i) {
        const uint8_t *rec = r.b.data() + r.pos + i * sz_el;
        std::memcpy(&ix.l0[i * (1 + ix.maxM0)], rec, off_data);
        std::memcpy(&ix.vec[i * ix.d], rec + off_data, 4 * (size_t)ix.d);
        std::memcpy(&ix.labels[i], rec + label_off, 8);
        const uint32_t hdr = ix.l0[i * (1 + ix.maxM0)];
        if ((hdr >> 16) & 0x1u)
            throw bad("deleted elements are not supported (element " + std::to_string(i) + ")");
        if ((hdr & 0xFFFFu) > ix.maxM0)
            throw bad("level-0 link count > maxM0 at element " + std::to_string(i));
    }
    r.pos += n * sz_el;
    const uint64_t blk = 1 + ix.maxM;
    ix.levels.assign(n, 0);
    ix.up_off.assign(n, -1);
    for (uint64_t i = 0; i < n; ++i) {
        const uint32_t size = r.get<uint32_t>("linkListSize");
        if (size == 0)
            continue;
        if (size % (4 * blk) != 0)
            throw bad("upper link list size not a multiple of the block size at element " + std::to_string(i));
        if (r.pos + size > r.b.size())
            throw bad("truncated upper links");
        ix.levels[i] = (int32_t)(size / (4 * blk));
        if (ix.levels[i] > ix.maxlevel)
            throw bad("element level > maxlevel");
        ix.up_off[i] = (int64_t)ix.up.size();
        const size_t w = size / 4;
        ix.up.resize(ix.up.size() + w);
        std::memcpy(&ix.up[ix.up.size() - w], r.b.data() + r.pos, size);
        r.pos += size;
    }
    if (r.pos != r.b.size())
        throw bad("trailing bytes");
    // link targets in range
    for (uint64_t i = 0; i < n; ++i) {
        const uint32_t *row = &ix.l0[i * (1 + ix.maxM0)];
        for (uint32_t j = 0; j < (row[0] & 0xFFFFu); ++j)
            if (row[1 + j] >= n)
                throw bad("level-0 link out of range at element " + std::to_string(i));
    }
    // block l-1 of node i lists its level-l links; every target must itself reach level l (the
    // search reads the target's level-l block, which only exists for levels[target] >= l)
    for (uint64_t i = 0; i < n; ++i)
        for (int32_t l = 1; l <= ix.levels[i]; ++l) {
            const size_t b = (size_t)ix.up_off[i] + (size_t)(l - 1) * blk;
            if ((ix.up[b] & 0xFFFFu) > ix.maxM)
                throw bad("upper link count > maxM");
            for (uint32_t j = 0; j < (ix.up[b] & 0xFFFFu); ++j) {
                const uint32_t v = ix.up[b + 1 + j];
                if (v >= n)
                    throw bad("upper link out of range");
                if (ix.levels[v] < l)
                    throw bad("element " + std::to_string(i) + " links to element " + std::to_string(v) +
                              " on level " + std::to_string(l) + ", which that element does not reach");
            }
        }
    if (n > 0 && ix.levels[ix.ep] != ix.maxlevel)
        throw bad("entry point is not on the top level");
    return ix;
}

void write_hnswlib(const HnswFlatHost &ix, const std::string &path)
{
    std::ofstream f(path, std::ios::binary);
    if (!f)
        throw Error(DRM_ERR_IO, "cannot write index file " + path);
    auto put = [&](const auto &v) { f.write((const char *)&v, sizeof(v)); };
    const uint64_t off_data = 4 * (1 + ix.maxM0);
    const uint64_t label_off = off_data + 4 * (uint64_t)ix.d;
    const uint64_t sz_el = label_off + 8;
    put((uint64_t)0);
    put((uint64_t)ix.max_elements);
    put((uint64_t)ix.n);
    put(sz_el);
    put(label_off);
    put(off_data);
    put((int32_t)ix.maxlevel);
    put((uint32_t)ix.ep);
    put((uint64_t)ix.maxM);
    put((uint64_t)ix.maxM0);
    put((uint64_t)ix.M);
    put((double)ix.mult);
    put((uint64_t)ix.efc);
    std::vector<uint8_t> rec(sz_el);
    for (int64_t i = 0; i < ix.n; ++i) {
        std::memcpy(rec.data(), &ix.l0[(size_t)i * (1 + ix.maxM0)], off_data);
        std::memcpy(rec.data() + off_data, &ix.vec[(size_t)i * ix.d], 4 * (size_t)ix.d);
        std::memcpy(rec.data() + label_off, &ix.labels[i], 8);
        f.write((const char *)rec.data(), (std::streamsize)sz_el);
    }
    const uint64_t blk = 1 + ix.maxM;
    for (int64_t i = 0; i < ix.n; ++i) {
        const uint32_t size = (uint32_t)(ix.levels[i] * blk * 4);
        put(size);
        if (size)
            f.write((const char *)&ix.up[(size_t)ix.up_off[i]], size);
    }
    if (!f)
        throw Error(DRM_ERR_IO, "write failed: " + path);
}

} // namespace drm
