// tools/pipeline.cpp -- MI355X drop-in for the reference `pipeline` executable (src/main.cpp).
//
// Same argv contract (src/main.cpp:12-22):
//   pipeline <index_prefix> <query_seqs.fastq|.fq|.txt|.npy> <ref_seqs.fasta> [EF] [K] [K_clusters]
//            [output_dir] [use_dynamic] [use_streaming]
// Same files: <prefix>/<basename(prefix)>.index + <prefix>/config.txt in (:34-47), and
// <output_dir>/indices.npy (<u8) + distances.npy (<f4) out (:371-384), written from the raw
// HNSW results exactly like save_results. The north-star tail (SW rerank, the commented-out
// post_process_sw_static call at :333-341) runs on the GPU when query sequences are available and
// adds sw_scores.npy (<i4) and sw_ids.npy (<u8) [n, k] (rows of a query with no candidate: -1 / 2^64-1).
// use_dynamic cuts the candidate windows from the genome string on the device (post_process_sw_dynamic
// instead of the static window table); use_streaming writes <output_dir>/results.sam block by block
// (write_sam_streaming) and, like the reference, skips the .npy outputs -- the reference streams only in
// its dynamic branch, so static + streaming writes no result file there either.
// Sequence inputs are embedded by the reference's GRU model on the GPU (drm_vectorize) when
// DRM_ENCODER names it (.xml IR or .drmenc) or when the reference's models/ path exists in the working
// directory (Config::Inference::MODEL_PATH); otherwise by the deterministic 3-mer stand-in. The rerank is
// the north star's SW rerank (the reference's main runs an L2 rerank with the model at this point,
// src/main.cpp:312-331).
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <filesystem>
#include <iostream>
#include <numeric>
#include <thread>

#include "drm_hip.h"
#include "drm_internal.h"

using clk = std::chrono::high_resolution_clock;
static long ms_since(clk::time_point t0)
{
    return (long)std::chrono::duration_cast<std::chrono::milliseconds>(clk::now() - t0).count();
}

static void check(int rc)
{
    if (rc != DRM_OK)
        throw drm::Error(rc, drm_last_error());
}

// pinned host buffer (drm_host_alloc): the executor's copies become DMA transfers beside the kernels
template <class T> struct Pinned {
    T *p = nullptr;
    explicit Pinned(size_t n)
    {
        void *v = nullptr;
        check(drm_host_alloc(&v, sizeof(T) * std::max<size_t>(n, 1)));
        p = static_cast<T *>(v);
    }
    ~Pinned() { drm_host_free(p); }
    Pinned(const Pinned &) = delete;
    Pinned &operator=(const Pinned &) = delete;
};

int main(int argc, char *argv[])
{
    if (argc < 4 || argc > 10) {
        std::cerr << "Usage: " << argv[0]
                  << " <index_prefix> <query_seqs.fastq> <ref_seqs.fasta> [EF] [K] [K_clusters] [output_dir] "
                     "[use_dynamic] [use_streaming]"
                  << std::endl;
        std::cerr << "  - query input: Can be FASTQ/FASTA/TXT file or pre-computed embeddings in .npy format" << std::endl;
        std::cerr << "  - EF: Optional HNSW search parameter (default: 128)" << std::endl;
        std::cerr << "  - K: Optional number of nearest neighbors to return (default: 128)" << std::endl;
        std::cerr << "  - output_dir: Optional output directory (default: current directory)" << std::endl;
        return 1;
    }
    try {
        auto master = clk::now();
        std::cout << "=== DeepReadMapper MI355X Pipeline ===" << std::endl << std::endl;
        const std::string prefix = argv[1];
        const std::string base = std::filesystem::path(prefix).filename().string();
        const std::string index_file = prefix + "/" + base + ".index";
        const std::string config_file = prefix + "/config.txt";
        if (!std::filesystem::exists(config_file))
            throw drm::Error(DRM_ERR_IO, "Config file does not exist: " + config_file);
        auto config = drm::load_config(config_file);
        if (!config.count("ref_len") || !std::holds_alternative<size_t>(config["ref_len"]) || !config.count("stride") ||
            !std::holds_alternative<size_t>(config["stride"]))
            throw drm::Error(DRM_ERR_FORMAT, "config.txt lacks integer ref_len / stride");
        const size_t ref_len = std::get<size_t>(config["ref_len"]);
        const size_t stride = std::get<size_t>(config["stride"]);
        const std::string query_file = argv[2], ref_file = argv[3];
        const int ef = argc >= 5 ? std::stoi(argv[4]) : 128;
        const int k = argc >= 6 ? std::stoi(argv[5]) : 128;
        int k_clusters = 5;
        if (stride == 1)
            k_clusters = k;
        else if (argc >= 7)
            k_clusters = std::stoi(argv[6]);
        const std::string out_dir = argc >= 8 ? argv[7] : ".";
        const bool use_dynamic = argc >= 9 && std::stoi(argv[8]) != 0;
        const bool use_streaming = argc >= 10 && std::stoi(argv[9]) != 0;
        const std::string sam_file = out_dir + "/results.sam"; // src/main.cpp:67
        // devices: DRM_DEVICES=0,1,... fans the batch out over several GPUs (contiguous query shards,
        // replicated index); DRM_DEVICE=i picks one (default 0)
        std::vector<int> devices;
        if (const char *dl = std::getenv("DRM_DEVICES")) {
            std::string sdl(dl);
            for (size_t p = 0; p < sdl.size();) {
                size_t q = sdl.find(',', p);
                if (q == std::string::npos)
                    q = sdl.size();
                if (q > p)
                    devices.push_back(std::stoi(sdl.substr(p, q - p)));
                p = q + 1;
            }
        }
        if (devices.empty())
            devices.push_back(std::getenv("DRM_DEVICE") ? std::atoi(std::getenv("DRM_DEVICE")) : 0);
        const int device = devices[0];

        // ---- data loading
        std::vector<float> emb;
        size_t nq = 0, dim = 0;
        std::vector<std::string> qseqs, qids;
        const bool is_npy = std::filesystem::path(query_file).extension() == ".npy";
        auto t0 = clk::now();
        if (is_npy) {
            drm::NpyArray a = drm::npy_load(query_file);
            if (a.shape.size() != 2)
                throw drm::Error(DRM_ERR_FORMAT, "Error: Expected 2D array in .npy file");
            if (a.kind != 'f' || a.itemsize != 4)
                throw drm::Error(DRM_ERR_FORMAT, "embeddings .npy must be float32 ('<f4')");
            nq = a.shape[0];
            dim = a.shape[1];
            emb.resize(nq * dim);
            std::memcpy(emb.data(), a.bytes.data(), emb.size() * sizeof(float));
            std::cout << "[MAIN] Loaded " << nq << " embeddings of dimension " << dim << std::endl;
        } else {
            drm::read_file(query_file, qseqs, qids);
            if (qseqs.empty()) {
                std::cerr << "No query_sequences found in input file!" << std::endl;
                return 1;
            }
            nq = qseqs.size();
        }
        // ---- reference: the static window table (read_file(ref, ref_len, 1, lookup)), or with use_dynamic the
        //      genome string (extract_FASTA_sequence), windows cut on the device (src/main.cpp:182-192)
        const bool dyn = use_dynamic && !is_npy;
        std::vector<std::string> refs;
        std::string genome;
        if (dyn) {
            std::cout << "[MAIN] Using DYNAMIC fetching for reference sequences" << std::endl;
            genome = drm::extract_fasta_sequence(ref_file);
            std::cout << "[MAIN] Loaded a " << genome.size() << " bp genome from " << ref_file << std::endl;
        } else if (!is_npy) {
            std::cout << "[MAIN] Using STATIC fetching for reference sequences" << std::endl;
            std::vector<std::string> dummy;
            drm::read_file(ref_file, refs, dummy, ref_len, 1, true);
            std::cout << "[MAIN] Loaded " << refs.size() << " reference sequences from " << ref_file << std::endl;
            // the device window table is fixed-width: a .txt / .fastq reference whose lines are not
            // all ref_len bytes would be over-read or silently truncated (the reference scores the
            // whole string), so it is refused before anything touches the GPU
            for (size_t r = 0; r < refs.size(); ++r)
                if (refs[r].size() != ref_len)
                    throw drm::Error(DRM_ERR_FORMAT, "reference sequence " + std::to_string(r) + " has " +
                                                         std::to_string(refs[r].size()) +
                                                         " bytes; the window table needs ref_len = " +
                                                         std::to_string(ref_len) + " for every window");
        }
        std::cout << "[MAIN] Total Data loading time: " << ms_since(t0) << " ms" << std::endl << std::endl;

        // ---- window table (static ref_seqs) as one fixed-width block
        std::string table;
        if (!is_npy && !dyn) {
            table.assign(refs.size() * ref_len, '\0');
            for (size_t r = 0; r < refs.size(); ++r)
                std::memcpy(&table[r * ref_len], refs[r].data(), ref_len);
        }

        // ---- index (one replica per device)
        t0 = clk::now();
        if (!std::filesystem::exists(index_file))
            throw drm::Error(DRM_ERR_IO, "Index file does not exist: " + index_file);
        drm_index *index = nullptr;
        drm_refs *rt = nullptr;
        drm_multi *multi = nullptr;
        drm_index_info info;
        if (devices.size() == 1) {
            check(drm_index_load(index_file.c_str(), device, &index));
            check(drm_index_get_info(index, &info));
            if (dyn)
                check(drm_refs_create_genome((const uint8_t *)genome.data(), (int64_t)genome.size(), (int32_t)ref_len,
                                             device, &rt));
            else if (!is_npy)
                check(drm_refs_create((const uint8_t *)table.data(), (int64_t)refs.size(), (int32_t)ref_len,
                                      (int64_t)ref_len, device, &rt));
        } else {
            if (dyn)
                check(drm_multi_create_genome(index_file.c_str(), devices.data(), (int)devices.size(),
                                              (const uint8_t *)genome.data(), (int64_t)genome.size(), (int32_t)ref_len,
                                              &multi));
            else
                check(drm_multi_create(index_file.c_str(), devices.data(), (int)devices.size(),
                                       is_npy ? nullptr : (const uint8_t *)table.data(), (int64_t)refs.size(),
                                       (int32_t)ref_len, (int64_t)ref_len, &multi));
            check(drm_multi_get_index_info(multi, &info));
        }
        if (index) { // the executor's streams and buffers for this batch, outside the search timing
            size_t qs_max = 0;
            for (auto &q : qseqs)
                qs_max = std::max(qs_max, q.size());
            check(drm_search_rerank_prepare(index, (int64_t)nq, (int32_t)(is_npy ? dim : info.d), k_clusters, k,
                                            is_npy ? 0 : (int32_t)qs_max));
        }
        std::cout << "[MAIN] Index loaded time: " << ms_since(t0) << " ms (" << info.ntotal << " vectors, "
                  << info.device_bytes / (1 << 20) << " MiB on each of " << devices.size() << " device(s))"
                  << std::endl;

        // ---- embedding (Vectorizer::vectorize, src/main.cpp:249-268), into pinned host memory: the GRU model
        //      on the GPU (DRM_ENCODER or the reference's models/ path), else the deterministic 3-mer stand-in
        if (!is_npy)
            dim = (size_t)info.d;
        Pinned<float> x(nq * dim);
        if (!is_npy) {
            t0 = clk::now();
            const std::string model = drm::encoder_model_path();
            if (!model.empty()) {
                if (dim != 128)
                    throw drm::Error(DRM_ERR_ARG, "the GRU model emits 128-d embeddings; the index has d = " +
                                                      std::to_string(dim));
                drm::vectorize_host(model, device, qseqs, x.p);
                std::cout << "[MAIN] Inference (GRU model " << model << ", GPU) time: " << ms_since(t0) << " ms"
                          << std::endl;
            } else {
                std::string all;
                std::vector<int64_t> off(nq);
                std::vector<int32_t> len(nq);
                for (size_t i = 0; i < nq; ++i) {
                    off[i] = (int64_t)all.size();
                    len[i] = (int32_t)qseqs[i].size();
                    all += qseqs[i];
                }
                check(drm_embed_kmer3((const uint8_t *)all.data(), off.data(), len.data(), (int64_t)nq, (int32_t)dim,
                                      drm::kEmbedSeed, x.p));
                std::cout << "[MAIN] Inference (3-mer stand-in) time: " << ms_since(t0) << " ms" << std::endl;
            }
        } else {
            std::memcpy(x.p, emb.data(), sizeof(float) * nq * dim);
        }

        // ---- HNSW search (faiss_search(alg_hnsw, embeddings, k_clusters, ef), src/main.cpp:278) streamed into
        //      the SW rerank (post_process_sw_static, :333-341) batch by batch
        size_t qs = 0;
        for (auto &q : qseqs)
            qs = std::max(qs, q.size());
        Pinned<uint8_t> qbuf(nq * std::max<size_t>(qs, 1));
        Pinned<int32_t> ql(nq), status(nq);
        for (size_t i = 0; i < nq && !is_npy; ++i) {
            std::memset(qbuf.p + i * qs, 0, qs);
            std::memcpy(qbuf.p + i * qs, qseqs[i].data(), qseqs[i].size());
            ql.p[i] = (int32_t)qseqs[i].size();
        }
        Pinned<float> D(nq * (size_t)k_clusters);
        Pinned<int64_t> I(nq * (size_t)k_clusters);
        Pinned<int32_t> sw_scores(is_npy ? 0 : nq * (size_t)k);
        Pinned<uint64_t> sw_ids(is_npy ? 0 : nq * (size_t)k);
        t0 = clk::now();
        drm_search_stats st{};
        // The reference streams its SAM from post_process_l2_dynamic_streaming (src/main.cpp:316-319). With a
        // dense index (stride 1) that function skips every reranker and writes the first min(k, k_clusters)
        // search neighbours of each query in search order (src/utils/post_processor.cpp:833-878), so the SAM
        // here comes straight from the search and no rerank runs. A sparse index reranks the expanded windows of
        // the whole run by L2 (:884-1010): drm_post_process_l2_dynamic over every query after the search, on a
        // window-embedding table of the genome built by the GRU model. Without the model (3-mer stand-in) or
        // across several devices, those SAM rows come from the SW rerank instead.
        //
        // What the reference's sparse branch writes is only the SAM header: its write_sam_streaming call there
        // (post_processor.cpp:1004-1005) leaves out batch_query_count, which defaults to 0
        // (includes/utils/utils.hpp:99), so the row loop (utils.cpp:452) never runs. That header-only file is
        // the default here too (no rerank is computed for it). DRM_SAM_L2_ROWS=1 opts into the rows the
        // reranker meant to write: the L2 rows of every query, and none for a query whose
        // candidate range runs past the clipped expansion stream (the reference reads out of bounds there).
        const bool stream_sam = use_streaming && dyn;
        const bool sam_from_search = stream_sam && stride == 1;
        const bool l2_rows = std::getenv("DRM_SAM_L2_ROWS") && std::atoi(std::getenv("DRM_SAM_L2_ROWS")) != 0;
        const bool sam_header_only = stream_sam && stride > 1 && !l2_rows;
        const bool sam_l2 = stream_sam && stride > 1 && l2_rows && rt && !is_npy && !drm::encoder_model_path().empty();
        if (stream_sam && (size_t)k > (size_t)k_clusters * 2 * stride) // post_processor.cpp:769-772
            throw drm::Error(DRM_ERR_K, "Final k too large. Ensure k < k_clusters * 2 * stride to have enough candidates.");
        if (stream_sam && stride > 1 && l2_rows && !sam_l2)
            std::cout << "[MAIN] stride > 1 without the GRU model on one device: SAM rows from the SW rerank (the "
                         "reference reranks them by L2 here)"
                      << std::endl;
        // one pass over queries [lo, lo + m) into the output arrays at row lo
        auto run = [&](size_t lo, size_t m, drm_search_stats *sp) {
            const bool search_only = sam_from_search || sam_l2 || sam_header_only;
            const uint8_t *qb = (is_npy || search_only) ? nullptr : qbuf.p + lo * qs;
            if (multi)
                return drm_multi_search_rerank(multi, x.p + lo * dim, (int64_t)m, (int32_t)dim, k_clusters, ef, qb,
                                               ql.p + lo, (int32_t)qs, (int64_t)stride, k, D.p + lo * k_clusters,
                                               I.p + lo * k_clusters, sw_scores.p + lo * k, sw_ids.p + lo * k,
                                               status.p + lo, sp);
            return drm_search_rerank(index, search_only ? nullptr : rt, x.p + lo * dim, (int64_t)m,
                                     (int32_t)dim,
                                     k_clusters, ef, qb, ql.p + lo,
                                     (int32_t)qs, (int64_t)stride, k, D.p + lo * k_clusters, I.p + lo * k_clusters,
                                     sw_scores.p + lo * k, sw_ids.p + lo * k, status.p + lo, sp);
        };
        int rc = DRM_OK;
        if (sam_header_only) {
            std::cout << "[MAIN] Using STREAMING output to SAM file: " << sam_file << std::endl;
            std::filesystem::create_directories(out_dir);
            rc = run(0, nq, &st); // faiss_search of the whole run (src/main.cpp:278)
            if (rc == DRM_OK)
                drm::write_sam_block(sam_file, true, "ref", ref_len, qseqs, qids, 0, 0, nullptr, nullptr, (size_t)k);
        } else if (sam_l2) {
            std::cout << "[MAIN] Using STREAMING output to SAM file: " << sam_file << std::endl;
            std::filesystem::create_directories(out_dir);
            rc = run(0, nq, &st);
            if (rc == DRM_OK) {
                const auto tl = clk::now();
                drm_encoder *enc = nullptr;
                check(drm_encoder_load(drm::encoder_model_path().c_str(), device, &enc));
                const int erc = drm_refs_embed(rt, enc, nullptr);
                drm_encoder_free(enc);
                check(erc);
                std::vector<float> l2d(nq * (size_t)k);
                std::vector<uint64_t> l2i(nq * (size_t)k);
                std::vector<int32_t> cnt(nq);
                int64_t bad = -1;
                const int lrc = drm_post_process_l2_dynamic(rt, I.p, (int64_t)nq, k_clusters, x.p, (int32_t)dim,
                                                            (int64_t)stride, k, k_clusters, l2d.data(), l2i.data(),
                                                            cnt.data(), &bad);
                // a candidate range past the clipped stream (status -4): that query keeps no row, the others are
                // written (every output was downloaded before the error was raised)
                if (lrc == DRM_ERR_ARG && bad >= 0) {
                    size_t clipped = 0;
                    for (size_t i = 0; i < nq; ++i)
                        clipped += cnt[i] == 0;
                    std::cout << "[MAIN] " << clipped << " queries (first " << bad
                              << ") rerank past the clipped expansion stream: written without rows" << std::endl;
                } else {
                    check(lrc);
                }
                std::cout << "[MAIN] L2 rerank (dynamic, stride " << stride << ") time: " << ms_since(tl) << " ms"
                          << std::endl;
                size_t block = 1u << 20;
                if (const char *e = std::getenv("DRM_SAM_BLOCK"))
                    block = std::max<size_t>(1, std::strtoull(e, nullptr, 10));
                for (size_t lo = 0; lo < nq; lo += block) // write_sam_streaming per reranked batch (:1004-1006)
                    drm::write_sam_block(sam_file, lo == 0, "ref", ref_len, qseqs, qids, lo, std::min(block, nq - lo),
                                         l2i.data() + lo * k, cnt.data() + lo, (size_t)k);
            }
        } else if (stream_sam) {
            // post_process_*_dynamic_streaming + write_sam_streaming (src/main.cpp:316-319,
            // src/utils/utils.cpp:409-503): the SAM lines of each block are written by a host thread while the
            // GPU works on the next block (blocks of DRM_SAM_BLOCK queries; the file does not depend on it)
            std::cout << "[MAIN] Using STREAMING output to SAM file: " << sam_file << std::endl;
            std::filesystem::create_directories(out_dir);
            size_t block = 1u << 20;
            if (const char *e = std::getenv("DRM_SAM_BLOCK"))
                block = std::max<size_t>(1, std::strtoull(e, nullptr, 10));
            std::thread writer;
            std::string werr;
            for (size_t lo = 0; lo < nq && rc == DRM_OK; lo += block) {
                const size_t m = std::min(block, nq - lo);
                drm_search_stats bs{};
                rc = run(lo, m, &bs);
                st.nq += bs.nq;
                st.ndis += bs.ndis;
                st.nhops += bs.nhops;
                st.kernel_ms += bs.kernel_ms;
                if (writer.joinable())
                    writer.join();
                if (rc == DRM_OK && werr.empty())
                    writer = std::thread([&, lo, m] {
                        try {
                            std::vector<int32_t> cnt(m);
                            if (sam_from_search) {
                                std::fill(cnt.begin(), cnt.end(), std::min(k, k_clusters));
                                drm::write_sam_block(sam_file, lo == 0, "ref", ref_len, qseqs, qids, lo, m,
                                                     reinterpret_cast<const uint64_t *>(I.p) + lo * k_clusters,
                                                     cnt.data(), (size_t)k_clusters);
                                return;
                            }
                            for (size_t i = 0; i < m; ++i)
                                cnt[i] = std::max(status.p[lo + i], 0);
                            drm::write_sam_block(sam_file, lo == 0, "ref", ref_len, qseqs, qids, lo, m,
                                                 sw_ids.p + lo * k, cnt.data(), (size_t)k);
                        } catch (const std::exception &e) {
                            werr = e.what();
                        }
                    });
            }
            if (writer.joinable())
                writer.join();
            if (rc == DRM_OK && !werr.empty())
                throw drm::Error(DRM_ERR_IO, werr);
        } else {
            rc = run(0, nq, &st);
        }
        const std::string err = rc == DRM_OK ? "" : drm_last_error();
        const long search_ms = ms_since(t0);
        if (rt)
            drm_refs_free(rt);
        if (index)
            drm_index_free(index);
        if (multi)
            drm_multi_free(multi);
        if (rc != DRM_OK)
            throw drm::Error(rc, err);
        std::cout << "[MAIN] Search" << (is_npy ? "" : " + SW rerank") << " time: " << search_ms << " ms (device "
                  << st.kernel_ms << " ms, ndis " << st.ndis << ", nhops " << st.nhops << ", " << devices.size()
                  << " device(s))" << std::endl;
        if (!is_npy) // rows of a query with no candidate at all (reranker.cpp:10-11) stay -1 / 2^64-1
            for (size_t i = 0; i < nq; ++i)
                for (int j = std::max(status.p[i], 0); j < k; ++j) {
                    sw_scores.p[i * (size_t)k + (size_t)j] = -1;
                    sw_ids.p[i * (size_t)k + (size_t)j] = ~0ull;
                }

        // ---- outputs (save_results, src/utils/utils.cpp:264-334); skipped with use_streaming (src/main.cpp:371, :409-412)
        if (use_streaming) {
            std::cout << "[MAIN] Skip normal output saving since streaming output is used." << std::endl;
            std::cout << "[MAIN] Total pipeline time: " << ms_since(master) << " ms" << std::endl;
            std::cout << "=== Pipeline Completed Successfully! ===" << std::endl;
            return 0;
        }
        t0 = clk::now();
        std::filesystem::create_directories(out_dir);
        const size_t kout = stride == 1 ? (size_t)k : (size_t)k_clusters;
        std::vector<uint64_t> idx(nq * kout);
        std::vector<float> dis(nq * kout);
        for (size_t i = 0; i < nq; ++i)
            for (size_t j = 0; j < kout; ++j) {
                idx[i * kout + j] = (uint64_t)I.p[i * k_clusters + j];
                dis[i * kout + j] = D.p[i * k_clusters + j];
            }
        drm::npy_save(out_dir + "/indices.npy", idx.data(), {nq, kout}, 'u', 8);
        drm::npy_save(out_dir + "/distances.npy", dis.data(), {nq, kout}, 'f', 4);
        if (!is_npy) {
            drm::npy_save(out_dir + "/sw_scores.npy", sw_scores.p, {nq, (size_t)k}, 'i', 4);
            drm::npy_save(out_dir + "/sw_ids.npy", sw_ids.p, {nq, (size_t)k}, 'u', 8);
        }
        std::cout << "[MAIN] Output saving time: " << ms_since(t0) << " ms" << std::endl;
        std::cout << "[MAIN] Total pipeline time: " << ms_since(master) << " ms" << std::endl;
        std::cout << "=== Pipeline Completed Successfully! ===" << std::endl;
    } catch (const std::exception &e) {
        std::cerr << "Error: " << e.what() << std::endl;
        return 1;
    }
    return 0;
}
