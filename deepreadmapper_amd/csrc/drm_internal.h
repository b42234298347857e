// deepreadmapper_amd/csrc/drm_internal.h -- private C++ API shared by the library and the CLIs.
#pragma once
#include <cstdint>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <variant>
#include <vector>

#include "drm_hip.h"

namespace drm {

struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};

void set_last_error(const std::string &msg);

// RCCL helpers over a drm_comm (exec.cpp), for collectives the C ABI builds on (drm_index_broadcast, capi.cpp):
// a grouped ncclBroadcast of byte ranges from `root` (send is read on the root only; recv may equal send there),
// synchronised on `stream`; and an agreement step (min over ranks of `ok`) that every rank reaches before a
// collective that a failed rank would not enter
struct BcastItem {
    const void *send;
    void *recv;
    size_t bytes;
};
int comm_rank(const drm_comm *c);
int comm_nranks(const drm_comm *c);
int comm_device(const drm_comm *c);
void comm_broadcast(drm_comm *c, const BcastItem *items, int n, int root, void *stream); // throws Error
int comm_all_ok(drm_comm *c, bool ok, void *stream);                                   // throws Error

// ---------------------------------------------------------------------------------------------
// Host image of a faiss IndexHNSWPQ: exactly the fields faiss::write_index / read_index touch
// for fourcc "IHNp" + storage "IxPq" [faiss impl/index_write.cpp, impl/index_read.cpp].
// ---------------------------------------------------------------------------------------------
struct IndexHeader {
    int32_t d = 0;
    int64_t ntotal = 0;
    uint8_t is_trained = 1;
    int32_t metric_type = 1; // METRIC_L2
    float metric_arg = 0.f;
};

struct HnswPqHost {
    IndexHeader hdr;
    // faiss::HNSW
    std::vector<double> assign_probas;
    std::vector<int32_t> cum_nneighbor_per_level;
    std::vector<int32_t> levels;   // level + 1 per node
    std::vector<uint64_t> offsets; // ntotal + 1
    std::vector<int32_t> neighbors;
    int32_t entry_point = -1;
    int32_t max_level = -1;
    int32_t efConstruction = 40;
    int32_t efSearch = 16;
    int32_t upper_beam = 1;
    // storage: faiss::IndexPQ
    IndexHeader storage_hdr;
    uint64_t pq_d = 0, pq_M = 0, pq_nbits = 0;
    std::vector<float> centroids; // [M][ksub][dsub]
    std::vector<uint8_t> codes;   // [ntotal][code_size]
    int32_t search_type = 0;
    uint8_t encode_signs = 0;
    int32_t polysemous_ht = 0;

    int dsub() const { return pq_M ? int(pq_d / pq_M) : 0; }
    int ksub() const { return 1 << int(pq_nbits); }
    int code_size() const { return int((pq_M * pq_nbits + 7) / 8); }
    int deg0() const { return cum_nneighbor_per_level.size() > 1 ? cum_nneighbor_per_level[1] - cum_nneighbor_per_level[0] : 0; }
    int nb_at(int level) const { return cum_nneighbor_per_level[level + 1] - cum_nneighbor_per_level[level]; }
};

HnswPqHost read_hnswpq(const std::string &path);                 // throws Error
void write_hnswpq(const HnswPqHost &ix, const std::string &path); // throws Error
void validate_hnswpq(const HnswPqHost &ix);                      // throws Error(DRM_ERR_FORMAT)

// ---------------------------------------------------------------------------------------------
// Host image of an hnswlib HierarchicalNSW<float> file (saveIndex/loadIndex, hnswlib_io.cpp):
// the reference's fp32-L2 backend (src/hnswlib_dir/*).
// ---------------------------------------------------------------------------------------------
struct HnswFlatHost {
    int32_t d = 0;
    int64_t n = 0;
    uint64_t max_elements = 0, maxM = 0, maxM0 = 0, M = 0, efc = 0;
    int32_t maxlevel = -1;
    uint32_t ep = 0;
    double mult = 0.0;
    std::vector<float> vec;       // [n][d]
    std::vector<uint32_t> l0;     // [n][1 + maxM0]: header (count in low 16 bits), links
    std::vector<uint64_t> labels; // [n]
    std::vector<int32_t> levels;  // [n]
    std::vector<int64_t> up_off;  // [n]: first word of the node's upper blocks in `up`, -1 if none
    std::vector<uint32_t> up;     // blocks of (1 + maxM) words, block l-1 = level l
};
HnswFlatHost read_hnswlib(const std::string &path);                  // throws Error
void write_hnswlib(const HnswFlatHost &ix, const std::string &path); // throws Error
void build_hnsw_flat(const float *x, int64_t n, int d, int M, int efc, int nthreads, uint64_t seed,
                     const std::string &path);

// faiss HNSW::set_default_probas(M, 1/log(M)) [faiss impl/HNSW.cpp]
void hnsw_default_probas(int M, std::vector<double> &probas, std::vector<int32_t> &cum);

// ---------------------------------------------------------------------------------------------
// Formats (src/utils/utils.cpp, src/utils/parse_inputs.cpp)
// ---------------------------------------------------------------------------------------------
using ConfigValue = std::variant<size_t, float, std::string>; // includes/utils/utils.hpp:102

void save_config(const std::unordered_map<std::string, ConfigValue> &config, const std::string &folder,
                 const std::string &file = "config.txt");
std::unordered_map<std::string, ConfigValue> load_config(const std::string &path);

// cnpy-compatible npy v1.0 writer/reader (descr '<u8', '<f4', '<i4', ...)
void npy_save(const std::string &path, const void *data, const std::vector<size_t> &shape, char kind, int itemsize);
struct NpyArray {
    std::vector<size_t> shape;
    char kind = 'f';
    int itemsize = 4;
    bool fortran = false;
    std::vector<uint8_t> bytes;
};
NpyArray npy_load(const std::string &path);

std::string reverse_complement(const std::string &seq);
// format_fasta (parse_inputs.cpp:223-369): fwd/RC interleaved windows; lookup_mode=false adds "<" ">".
std::vector<std::string> format_fasta(const std::string &data, size_t ref_len, size_t stride, bool lookup_mode);
// format_fastq (parse_inputs.cpp:843-950): "<"+seq+">" and ids up to ' ', '\t', '/'.
void format_fastq(const std::string &data, std::vector<std::string> &seqs, std::vector<std::string> &ids);
// read_file (utils.cpp:188-215) dispatch on extension; .txt = one sequence per non-empty line.
void read_file(const std::string &path, std::vector<std::string> &seqs, std::vector<std::string> &ids,
               size_t ref_len = 150, size_t stride = 1, bool lookup_mode = false);
std::string read_whole_file(const std::string &path);
// extract_FASTA_sequence (parse_inputs.cpp:174-220): skip the first line, keep the upper-cased
// A/C/G/T/N letters of everything after it (later header lines included), drop the rest.
std::string extract_fasta_sequence(const std::string &path);
// write_sam / write_sam_streaming (utils.cpp:336-503) for one block of queries: the SAM lines of
// queries [q0, q0 + nq) whose ids[i][0 .. counts[i]) are dense window ids (ids[i] at ids + i * k).
// `header` writes @HD / @SQ first (SN ref_name, LN ref_len: the reference's quirk) and truncates.
void write_sam_block(const std::string &path, bool header, const std::string &ref_name, size_t ref_len,
                     const std::vector<std::string> &query_seqs, const std::vector<std::string> &query_ids,
                     size_t q0, size_t nq, const uint64_t *ids, const int32_t *counts, size_t k);

void build_hnswpq(const float *x, int64_t n, int d, int M_pq, int nbits, int M_hnsw, int efc, double sample_rate,
                  int nthreads, uint64_t seed, const std::string &path);
// Shared by the CPU builder (builder.cpp) and the GPU builder (builder_gpu.hip):
// create_training_set's evenly spaced rows (src/hnswpq/index.cpp:57-84), subsampled to 256 * ksub;
std::vector<size_t> pq_training_rows(int64_t n, double sample_rate, int ksub, uint64_t seed);
// k-means (25 iterations) per sub-quantizer on rows [n_fit][d] -> centroids [M][2^nbits][d / M];
void pq_train_subspaces(const float *rows, size_t n_fit, int d, int M, int nbits, uint64_t seed, int nthreads,
                        float *centroids);
// HNSW::set_default_probas + random_level for n nodes: fills assign_probas, cum_nneighbor_per_level,
// levels (level + 1) and offsets of ix; returns the top level.
int hnsw_assign_levels(HnswPqHost &ix, int64_t n, int M_hnsw, uint64_t seed);
// GPU construction (builder_gpu.hip) from device-resident vectors d_x [n][d]: same file layout and
// levels as build_hnswpq, PQ trained on the host, codes and graph built on `device`.
void build_hnswpq_gpu(const float *d_x, int64_t n, int d, int M_pq, int nbits, int M_hnsw, int efc,
                      double sample_rate, uint64_t seed, int device, const std::string &path);
void embed_kmer3(const uint8_t *seqs, const int64_t *off, const int32_t *len, int64_t n, int dim, uint64_t seed,
                 float *out);
// the [64 x dim] N(0,1) projection of the stand-in embedder (splitmix64(seed) + Box-Muller)
std::vector<double> kmer3_matrix(int dim, uint64_t seed);
constexpr uint64_t kEmbedSeed = 42; // seed of the stand-in embedder used by the CLIs

// ---------------------------------------------------------------------------------------------
// Read encoder (encoder.cpp): the reference's OpenVINO GRU model (models/finetuned_sgn33-new-a-Apr6.xml,
// src/inference/fast_model.cpp), f16 tensors as the IR stores them.
// ---------------------------------------------------------------------------------------------
constexpr int kTokenHashes = 96; // hashToken range backed by _Tok2Index (includes/inference/preprocess.hpp:32-49)

struct EncoderHost {
    int32_t hidden = 64, emb_dim = 64, max_len = 123; // config.hpp:21 (MAX_LEN), the IR's GRU/embedding sizes
    float h0 = 0.f;
    std::vector<uint16_t> vocab_rows; // [1 + 96] vocabulary id of each embedding row (token_vocab_rows)
    std::vector<uint16_t> emb_rows;   // [rows][emb_dim] f16 bits
    std::vector<uint16_t> W[2], R[2], B[2]; // f16 bits: W [2][3H][in], R [2][3H][H], B [2][4H] (zrh)
    int in_dim(int layer) const { return layer == 0 ? emb_dim : 2 * hidden; }
};
std::vector<uint16_t> token_vocab_rows();
EncoderHost read_encoder(const std::string &path); // .xml (IR + sibling .bin) or .drmenc; throws Error
// Model the CLIs embed sequences with: DRM_ENCODER=<.xml|.drmenc> ("kmer3" or empty: the 3-mer stand-in),
// else the reference's Config::Inference::MODEL_PATH relative to the working directory when it exists
// (includes/utils/config.hpp:18), else "" (stand-in).
std::string encoder_model_path();
// Vectorizer::vectorize on `device` for host sequences: out [n][128]
void vectorize_host(const std::string &model, int device, const std::vector<std::string> &seqs, float *out);
void write_encoder(const EncoderHost &e, const std::string &path);

} // namespace drm
