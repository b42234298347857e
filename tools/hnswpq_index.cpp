// tools/hnswpq_index.cpp -- drop-in for the reference `hnswpq_index` executable
// (src/hnswpq/index.cpp:195-316). Same argv contract (:197-206):
//   hnswpq_index <ref_seq.fna|.txt|.npy> <index_prefix> <ref_len> [stride M_pq nbits M_hnsw EFC]
// Writes <index_prefix>/config.txt (keys of :289-302, save_config) and
// <index_prefix>/<index_prefix>.index (:212) in faiss IndexHNSWPQ format.
// Sequence inputs are read as tagged windows (read_file(ref, ref_len, stride), :270) and embedded
// by the GRU model on the GPU (DRM_ENCODER, or the reference's models/ path in the working directory,
// :279-280) or else the deterministic 3-mer stand-in.
// The graph (build_faiss_index, :86-193) is built on the GPU (drm_build_hnswpq_device, builder_gpu.hip:
// 50M windows in about half a minute) when a GPU is present and the shape is the one it supports (d = 128,
// M_pq = 8, nbits = 8, M_hnsw <= 32), else by the host builder (drm_build_hnswpq, OpenMP like the
// reference's omp_set_num_threads(128) at :116). Extra knobs via env: DRM_BUILD_DEVICE (auto | gpu | cpu),
// DRM_BUILD_THREADS (host builder threads, default: all cores), DRM_BUILD_SEED (default 0), DRM_DEVICE
// (the GPU for the encoder and the builder).
#include <cstdlib>
#include <cstring>
#include <filesystem>
#include <iostream>

#include "drm_hip.h"
#include "drm_internal.h"

int main(int argc, char *argv[])
{
    if (argc < 4 || argc > 9) {
        std::cerr << "Usage: " << argv[0] << " <ref_seq.txt> <index_prefix> <ref_len> [stride] [M_pq] [nbits] [M_hnsw] [EFC]"
                  << std::endl;
        std::cerr << "  stride: step size for sliding window (default: 1)" << std::endl;
        std::cerr << "  M_pq: number of PQ subquantizers (default: 8)" << std::endl;
        std::cerr << "  nbits: bits per subquantizer (default: 8)" << std::endl;
        std::cerr << "  M_hnsw: HNSW connectivity (default: 16)" << std::endl;
        std::cerr << "  EFC: efConstruction parameter (default: 200)" << std::endl;
        return 1;
    }
    try {
        const std::string ref_file = argv[1];
        const std::string prefix = argv[2];
        const std::string index_file = prefix + "/" + prefix + ".index";
        const size_t ref_len = std::stoul(argv[3]);
        const size_t stride = argc >= 5 ? std::stoul(argv[4]) : 1;
        const int M_pq = argc >= 6 ? std::stoi(argv[5]) : 8;
        const int nbits = argc >= 7 ? std::stoi(argv[6]) : 8;
        const int M_hnsw = argc >= 8 ? std::stoi(argv[7]) : 16;
        const int EFC = argc >= 9 ? std::stoi(argv[8]) : 200;
        const int threads = std::getenv("DRM_BUILD_THREADS") ? std::atoi(std::getenv("DRM_BUILD_THREADS")) : 0;
        const uint64_t seed = std::getenv("DRM_BUILD_SEED") ? std::strtoull(std::getenv("DRM_BUILD_SEED"), 0, 10) : 0;

        std::vector<float> emb;
        size_t n = 0, dim = 128;
        if (std::filesystem::path(ref_file).extension() == ".npy") {
            drm::NpyArray a = drm::npy_load(ref_file);
            if (a.shape.size() != 2) {
                std::cerr << "Error: Expected 2D array in .npy file" << std::endl;
                return 1;
            }
            if (a.kind != 'f' || a.itemsize != 4)
                throw drm::Error(DRM_ERR_FORMAT, "embeddings .npy must be float32 ('<f4')");
            n = a.shape[0];
            dim = a.shape[1];
            emb.resize(n * dim);
            std::memcpy(emb.data(), a.bytes.data(), emb.size() * sizeof(float));
        } else {
            std::vector<std::string> seqs, ids;
            drm::read_file(ref_file, seqs, ids, ref_len, stride, false);
            if (seqs.empty()) {
                std::cerr << "No sequences found in file: " << ref_file << std::endl;
                return 1;
            }
            n = seqs.size();
            emb.resize(n * dim);
            const std::string model = drm::encoder_model_path();
            if (!model.empty()) { // Vectorizer on the GPU (index.cpp:279-280)
                const int device = std::getenv("DRM_DEVICE") ? std::atoi(std::getenv("DRM_DEVICE")) : 0;
                drm::vectorize_host(model, device, seqs, emb.data());
                std::cout << "[BUILD INDEX] " << n << " windows embedded by the GRU model " << model << std::endl;
            } else {
                std::string all;
                std::vector<int64_t> off(n);
                std::vector<int32_t> len(n);
                for (size_t i = 0; i < n; ++i) {
                    off[i] = (int64_t)all.size();
                    len[i] = (int32_t)seqs[i].size();
                    all += seqs[i];
                }
                drm::embed_kmer3((const uint8_t *)all.data(), off.data(), len.data(), (int64_t)n, (int)dim,
                                 drm::kEmbedSeed, emb.data());
            }
        }
        std::cout << "[BUILD INDEX] " << n << " vectors of dimension " << dim << std::endl;
        std::unordered_map<std::string, drm::ConfigValue> config = {
            {"index_type", std::string("HNSWPQ")},
            {"stride", stride},
            {"ref_len", ref_len},
            {"n_vects", n},
            {"dim", dim},
            {"M_hnsw", (size_t)M_hnsw},
            {"EFC", (size_t)EFC},
            {"M_pq", (size_t)M_pq},
            {"nbits", (size_t)nbits},
            {"index_file", index_file},
        };
        drm::save_config(config, prefix);
        std::filesystem::create_directories(prefix);
        const std::string mode = std::getenv("DRM_BUILD_DEVICE") ? std::getenv("DRM_BUILD_DEVICE") : "auto";
        if (mode != "auto" && mode != "gpu" && mode != "cpu")
            throw drm::Error(DRM_ERR_ARG, "DRM_BUILD_DEVICE must be auto, gpu or cpu");
        int ndev = 0;
        if (mode != "cpu" && drm_device_count(&ndev) != DRM_OK)
            ndev = 0;
        const bool gpu_shape = dim == 128 && M_pq == 8 && nbits == 8 && M_hnsw >= 2 && M_hnsw <= 32;
        if (mode == "gpu" && (ndev < 1 || !gpu_shape))
            throw drm::Error(DRM_ERR_UNSUPPORTED, ndev < 1 ? "DRM_BUILD_DEVICE=gpu but no GPU is visible"
                                                           : "the GPU builder supports d = 128, M_pq = 8, nbits = 8, "
                                                             "M_hnsw <= 32");
        if (mode != "cpu" && ndev >= 1 && gpu_shape) {
            const int device = std::getenv("DRM_DEVICE") ? std::atoi(std::getenv("DRM_DEVICE")) : 0;
            void *d_x = nullptr;
            auto chk = [](int rc) {
                if (rc != DRM_OK)
                    throw drm::Error(rc, drm_last_error());
            };
            chk(drm_set_device(device));
            chk(drm_malloc(&d_x, sizeof(float) * n * dim));
            int rc = drm_memcpy_h2d(d_x, emb.data(), sizeof(float) * n * dim);
            if (rc == DRM_OK)
                rc = drm_build_hnswpq_device(static_cast<const float *>(d_x), (int64_t)n, (int32_t)dim, M_pq, nbits,
                                             M_hnsw, EFC, 0.5, seed, device, index_file.c_str());
            const std::string err = rc == DRM_OK ? "" : drm_last_error();
            drm_free(d_x);
            if (rc != DRM_OK)
                throw drm::Error(rc, err);
            std::cout << "[BUILD INDEX] graph built on GPU " << device << std::endl;
        } else {
            drm::build_hnswpq(emb.data(), (int64_t)n, (int)dim, M_pq, nbits, M_hnsw, EFC, 0.5, threads, seed,
                              index_file);
        }
        std::cout << "[BUILD INDEX] IndexHNSWPQ written to " << index_file << std::endl;
    } catch (const std::exception &e) {
        std::cerr << "Error: " << e.what() << std::endl;
        return 1;
    }
    return 0;
}
