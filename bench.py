#!/usr/bin/env python3
"""bench.py -- mapped reads/s of the MI355X hot path (HNSW search + SW rerank, EF=128, K=128).

Contract (driver): `python bench.py --gpus N --steps K --warmup W`; N>1 is launched by
torch.distributed.run, one rank per GPU. One step = one pass of the hot path over this rank's batch
of synthetic 150 bp reads, inputs already resident in HBM: the HNSW search kernel followed by the SW
rerank kernel (post_process_sw_static(..., k=K, k_clusters=K), src/main.cpp:340). Rank 0 prints ONE
JSON line.

Workload (`--workload`, default c5): BASELINE.json configs[4], the configuration the 1/2/4/8-GPU metric is
quoted on, per GPU: a seeded 25,000,149 bp genome -> 50,000,000 stride-1 fwd/RC 150 bp windows, a GPU-built
faiss IndexHNSWPQ (M_pq=8 nbits=8 M_hnsw=16 EFC=200; faiss is absent), 1.25M reads per GPU (weak scaling:
rank r searches its own contiguous shard of one seeded read stream), windows and reads embedded by the
reference's GRU model on the GPU (`--embed kmer3`: the 3-mer stand-in). c3: 1M windows, 100k reads; c4: the
10M-window stride-4 index, search only at K = 128 and 5.

Search (`--index`): pq (default), faiss_search(index, emb, k_clusters=K, ef=EF) (src/main.cpp:278), the live
pipeline's index; flat (C3 only): hnswlib fp32-L2 searchKnn (src/hnswlib_dir/search.cpp:7-52), M=64, EFC=128.
The timed region excludes inference and file I/O, as the reference's "Search time" window does
(src/main.cpp:272-285); the encoder, the L2 rerank and the PCIe-inclusive host path are reported beside it.
`--sw-band W` adds the opt-in banded SW rerank (not parity with the reference) on the same search rows as
`sw_band_opt_in`; the headline is always the full DP.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# dependent-load latency of the search's pointer chase, measured by tools/microbench/memlat.hip on an MI355X box
# (profiles/r03/box_diag_A.txt): the fallback when the live probe (dep_load_latency) cannot run
DEP_LOAD_LATENCY_S = 1.08e-6
SEARCH_LUT_BYTES = 8 * 256 * 4  # the lean search kernel's LDS per resident query (PQ 8 x 8 LUT)
SEARCH_KERNEL = "hnsw_pq_fast_kernel<true, false, true, false>"  # what C3/C4/C5 (ef = k = efSearch = 128, PQ8x8, inline rows) launch (hnsw_pq_fast.hip)
FLAT_KERNEL = "hnsw_flat_search_kernel<16, 0, false, 0>"  # --index flat: what C3 (d = 128, ef = 128) launches
SW_KERNEL = "sw_score_f16_kernel<150>"  # 150 DP columns: a tagged 150 bp read without its "<" / ">" ends
SW_VALU_PER_CELL_PAIR = 1053 / 300  # static ISA count of sw_score_f16_kernel<150>'s two-row block: 1053 VALU per 2 x 150 cell pairs
# its mix (integer cells, DRM_SW_INT): 751 packed 16-bit (v_pk_maximum3_f16, v_pk_sub_u16) at 4 cycles per wave64
# instruction per SIMD and 302 32-bit (v_add_u32, ...) at 2 (profiles/r02/valu_rate_probe.txt): average issue cycles
SW_ISSUE_CYC_PER_VALU = (751 * 4.0 + 302 * 2.0) / 1053
# what that exact mix (per cell pair: v_add_u32, v_pk_maximum3_f16, v_pk_sub_u16 clamp, half a v_pk_maximum3_f16),
# free of memory and dependency stalls, issues at on one MI355X: cycles per cell pair per SIMD at the nominal clock,
# at the kernel's 2 waves per SIMD and at 8 (tools/microbench/valu_rate.hip, profiles/r04/valu_rate_mix.txt)
SW_MIX_CYC_PER_PAIR = {2: 4.31 * 3.5, 8: 3.98 * 3.5}


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def committed_pmc(kernel_substr, workload):
    """Per-dispatch PMC summary of `kernel_substr` on `workload` from the newest committed profile
    (profiles/rNN/summary_<workload>.json, written by tools/scripts/profile.sh + summarize_profile.py)."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", f"summary_{workload}.json")), reverse=True):
        try:
            ks = json.load(open(path))["kernels"]
        except (OSError, ValueError, KeyError):
            continue
        for name, v in ks.items():
            if kernel_substr in name:
                return os.path.relpath(path, ROOT), v
    return None, None


VALU_CYC = 2.4  # cycles per wave64 32-bit VALU instruction per SIMD at >= 4 waves (profiles/r02/valu_rate_probe.txt)


def issue_ceiling(pmc, hops, ms, ncu, clock_hz):
    """Issue-bound ceiling of the search kernel from its committed PMC counters: wave-instructions per
    hop, and the launch time the VALU stream alone (4 SIMDs per CU at VALU_CYC cycles per instruction) and
    the scalar stream alone (one scalar unit per CU, one instruction per cycle) would take; CU count and clock are
    the device's (drm_device_get_props)."""
    if not pmc or "SQ_INSTS_VALU" not in pmc or hops <= 0:
        return None
    v, sc, lds = pmc["SQ_INSTS_VALU"], pmc.get("SQ_INSTS_SALU", 0.0), pmc.get("SQ_INSTS_LDS", 0.0)
    valu_ms = v * VALU_CYC / (4 * ncu * clock_hz) * 1e3
    salu_ms = sc / (ncu * clock_hz) * 1e3
    return {"valu_per_hop": round(v / hops, 1), "salu_per_hop": round(sc / hops, 1), "lds_per_hop": round(lds / hops, 1),
            "valu_bound_ms": round(valu_ms, 2), "salu_bound_ms": round(salu_ms, 2),
            "frac_of_issue_ceiling": round(max(valu_ms, salu_ms) / ms, 3),
            "note": "PMC from the committed profile of this workload; hops = this run's measured nhops"}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# The contract is ONE JSON line on stdout. Native libraries (gloo, RCCL) print banners to fd 1, so
# fd 1 is pointed at stderr for the whole run and the result goes to a saved copy of the original.
_RESULT_OUT = None


def emit(obj):
    out = _RESULT_OUT or sys.stdout
    out.write(json.dumps(obj) + "\n")
    out.flush()


def _claim_stdout():
    global _RESULT_OUT
    sys.stdout.flush()
    _RESULT_OUT = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)


class Dist:
    """Control plane for N>1 ranks (barrier, max, sum) over torch.distributed gloo; the data path
    has no collective (queries are independent, the index is replicated per GPU)."""

    def __init__(self):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", str(self.rank)))
        self.dist = None
        self.comm = None  # RCCL communicator (drm_comm) for the end-of-run result gather
        if self.world > 1:
            import torch.distributed as dist  # imported before libdrm_hip.so is loaded
            dist.init_process_group("gloo")
            self.dist = dist

    def barrier(self):
        if self.dist:
            self.dist.barrier()

    def allreduce(self, v, op):
        if not self.dist:
            return v
        import torch
        t = torch.tensor([float(v)], dtype=torch.float64)
        self.dist.all_reduce(t, op=getattr(self.dist.ReduceOp, op))
        return float(t.item())

    def close(self):
        if self.comm is not None:
            self.comm.free()
        if self.dist:
            self.dist.destroy_process_group()


def ref_sw_rerank(refs, I, queries, threads):
    """The SW half of the CPU baseline on the reference's own scorer: oracle/_ref/libdrm_ref.so (the reference's
    src/utils/metrics.cpp compiled where it lies, oracle/Makefile) scores every candidate with calc_sw_score and orders
    them as sw_reranker does (std::partial_sort by score, descending), OpenMP over queries. Returns the sorted scores
    [n, kk], or None when the library is absent (a box without it)."""
    import ctypes as C
    from oracle import oracle as O
    if not O.ref_available():
        return None
    lib = O.ref()
    f = lib.ref_sw_rerank_rows
    f.restype = C.c_int
    f.argtypes = [C.c_void_p, C.c_int64, C.c_int64, C.c_int64, C.c_void_p, C.c_int64, C.c_int64, C.c_void_p, C.c_int64,
                  C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
    n, kk = I.shape
    refs_c = refs if isinstance(refs, np.memmap) else np.ascontiguousarray(refs)
    I64, qb = np.ascontiguousarray(I, dtype=np.int64), np.ascontiguousarray(queries)
    ql = np.full(n, queries.shape[1], dtype=np.int32)
    sc, order = np.empty((n, kk), np.int32), np.empty((n, kk), np.int32)
    f(refs_c.ctypes.data, refs.shape[0], refs.shape[1], refs.shape[1], I64.ctypes.data, n, kk, qb.ctypes.data,
      queries.shape[1], ql.ctypes.data, sc.ctypes.data, order.ctypes.data, threads)
    return sc


def cpu_baseline(refs, index_path, queries, q_emb, k, ef, budget_s, log_fn, flat=False):
    """CPU baseline on a bounded sample of this workload, OpenMP over queries on the process's cores: the search is
    the oracle's restatement of faiss / hnswlib (neither library exists here), the SW rerank the reference's own
    calc_sw_score (oracle/_ref, ref_sw_rerank) when that library is present, else the oracle's restatement. Both SW
    forms are checked against each other on the sample's first 64 reads."""
    from oracle import faiss_file, hnswlib_file, oracle as O
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    threads = max(1, min(threads, len(os.sched_getaffinity(0))))
    if flat:
        fx = hnswlib_file.read(index_path)
    else:
        s = O.make_index(faiss_file.read(index_path))
    use_ref = O.ref_available()

    def run(n):
        q = q_emb[:n]
        t0 = time.perf_counter()
        if flat:
            D, I, nd, nh = O.hnswlib_search(fx, q, k, ef, nthreads=threads)
        else:
            D, I, nd, nh = O.hnswpq_search(s, q, k, ef, nthreads=threads)
        t1 = time.perf_counter()
        qbuf, ql = queries[:n], np.full(n, queries.shape[1], dtype=np.int32)
        if use_ref:
            sc = ref_sw_rerank(refs, I, qbuf, threads)
        else:
            rc, sc, ids, cnt = O.post_process_sw_static(I, refs, refs.shape[1], qbuf, ql, 1, k, k, nthreads=threads)
        t2 = time.perf_counter()
        return t1 - t0, t2 - t1, I, sc

    ts, tw, I, sc = run(min(256, len(q_emb)))
    sw_check = None
    if use_ref:  # the reference's scorer against the oracle's restatement on the same rows
        m = min(64, len(I))
        _, sc_o, _, _ = O.post_process_sw_static(I[:m], refs, refs.shape[1], queries[:m],
                                                 np.full(m, queries.shape[1], dtype=np.int32), 1, k, k,
                                                 nthreads=threads)
        sw_check = bool(np.array_equal(np.asarray(sc_o)[:, :k], sc[:m, :k]))
    per_q = (ts + tw) / min(256, len(q_emb))
    n = int(max(256, min(len(q_emb), budget_s / max(per_q, 1e-6))))
    ts, tw, _, _ = run(n)
    sw_src = ("the reference's own calc_sw_score + sw_reranker ordering (oracle/_ref: src/utils/metrics.cpp compiled "
              "here)" if use_ref else "the oracle's restatement")
    log_fn(f"[cpu] {n} queries x {threads} threads: search (oracle) {ts:.2f}s, SW ({'reference' if use_ref else 'oracle'})"
           f" {tw:.2f}s")
    return {"value": n / (ts + tw), "unit": "reads/s", "cores": threads, "kind": "port",
            "sw_kind": "reference" if use_ref else "port", "sw_matches_oracle": sw_check,
            "node_cpus": os.cpu_count(),
            "sample": f"first {n} of this rank's reads, OpenMP {threads} threads -- the process's CPU lease -- of the "
                      f"node's {os.cpu_count()} logical CPUs, {cpu_model()}: search = oracle/ C restatement of faiss "
                      f"(faiss absent) {n / ts:.1f} reads/s; SW rerank = {sw_src} {n / tw:.1f} reads/s"}


def prepare_c3(args, D, dev):
    """C3 (BASELINE.json configs[2]): a seeded 500,149 bp genome, stride-1 window
    table of 1,000,000 fwd/RC windows, IndexHNSWPQ built by the host builder, 100k reads per GPU."""
    from deepreadmapper_amd import synth
    from deepreadmapper_amd.shard import shard_range
    N, Q = D.world, args.queries or 100_000
    w = synth.Workload("c3", 500_149, N * Q, seed=42, read_seed=7)
    # rank 0 builds the shared index file; the others wait, then every rank loads its own replica
    if D.rank == 0:
        t0 = time.time()
        w.generate(args.cache, nthreads=args.build_threads, log=log)
        log(f"[bench] workload ready in {time.time() - t0:.1f}s: {len(w.refs)} windows, index {w.index_path}")
    D.barrier()
    if D.rank != 0:
        w.generate(args.cache)
    lo, hi = shard_range(N * Q, D.rank, N)  # contiguous query shard of this rank
    return {"Q": Q, "refs": w.refs, "index_path": w.index_path, "q_emb": np.ascontiguousarray(w.q_emb[lo:hi]),
            "queries": np.ascontiguousarray(w.queries[lo:hi]), "truth": w.truth[lo:hi],
            "desc": "C3: synthetic 1M x 150 bp dense IndexHNSWPQ (M_pq=8 nbits=8 M_hnsw=16 EFC=200), search + SW "
                    "rerank, EF=128 K=128"}


C5_GENOME = 25_000_149  # 2 * (L - 149) = 50,000,000 stride-1 windows


def prepare_c5(args, D, dev):
    """C5 per-GPU slice (BASELINE.json configs[4], the configuration the 1/2/4/8-GPU
    metric is quoted on): a seeded 25,000,149 bp genome, stride-1 window table of 50,000,000 fwd/RC
    150 bp windows, an IndexHNSWPQ (M_pq 8, nbits 8, M_hnsw 16, EFC 200) over them built on the GPU
    (builder_gpu.hip) and replicated on every GPU, and 1.25M reads per GPU (weak scaling: rank r takes
    reads [r*Q, (r+1)*Q) of one seeded read stream, so the 8-GPU job searches 10M reads). Rank 0
    writes the window table and the index once; every rank memory-maps the table and loads the file."""
    from deepreadmapper_amd import synth
    N, Q = D.world, args.queries or 1_250_000
    os.makedirs(args.cache, exist_ok=True)
    g = synth.genome(C5_GENOME, seed=44)
    n_ref = 2 * (C5_GENOME - 149)
    refs_path = os.path.join(args.cache, "c5_refs_150.u8")
    index_path = os.path.join(args.cache, "c5_M16_efc200_s1_gpu" + ("_gru" if args.embed == "gru" else "") + ".index")
    if D.rank == 0:
        t0 = time.time()
        if not os.path.exists(refs_path):
            synth.windows_lookup(g, 150, 1).tofile(refs_path + ".tmp")
            os.replace(refs_path + ".tmp", refs_path)
            log(f"[bench] C5 window table ({n_ref} windows) written in {time.time() - t0:.1f}s")
        if not os.path.exists(index_path):
            rows = np.memmap(refs_path, dtype=np.uint8, mode="r", shape=(n_ref, 150))
            synth.build_index_gpu_from_rows(rows, index_path + ".tmp", device=dev, log=log, embed=args.embed)
            os.replace(index_path + ".tmp", index_path)
            del rows
        log(f"[bench] C5 workload ready in {time.time() - t0:.1f}s")
    D.barrier()
    refs = np.memmap(refs_path, dtype=np.uint8, mode="r", shape=(n_ref, 150))
    t0 = time.time()
    reads, truth = synth.simulate_reads_range(g, D.rank * Q, (D.rank + 1) * Q, seed=9)
    queries = synth.tag(reads)
    q_emb = synth.embed_gru(queries, dev) if args.embed == "gru" else synth.embed(queries)
    log(f"[bench] {Q} reads simulated + embedded ({args.embed}) in {time.time() - t0:.1f}s")
    return {"Q": Q, "refs": refs, "index_path": index_path, "q_emb": q_emb, "queries": queries, "truth": truth,
            "desc": f"C5 per-GPU slice: synthetic 50M x 150 bp dense IndexHNSWPQ (M_pq=8 nbits=8 M_hnsw=16 EFC=200, "
                    f"GPU-built over {EMBED_DESC[args.embed]} window embeddings), replicated per GPU, {Q} reads per "
                    f"GPU, search + SW rerank, EF=128 K=128"}


EMBED_DESC = {"kmer3": "3-mer stand-in", "gru": "GRU-model (the reference's OpenVINO IR, on the GPU)"}
ENC_PEAK_TFLOPS = 2500.0  # MI355X dense f16 MFMA (MI355X_MICROARCH.md matrix-core table)


def encoder_timing(d_q, Q, q_stride, dev, reps=3):
    """The GRU read encoder (drm_vectorize_device, encoder_gru.hip) on this rank's tagged reads resident
    in HBM: HIP-event time of one launch sequence, reads/s, and MFMA rate against the f16 dense peak.
    MFMA work per read (the hi/lo split counted): 2 dirs x 123 steps x 3 gates x 64 units x 2 flop x
    (K1 = 64 h_hi + 64 h_lo + 64 x) + (K2 = 128 h + 256 x)."""
    from deepreadmapper_amd.encoder import Encoder
    from deepreadmapper_amd.device import DeviceBuffer, Event, Stream
    enc = Encoder(device=dev)
    d_l = DeviceBuffer.from_host(np.full(Q, q_stride, dtype=np.int32))
    d_o = DeviceBuffer((Q, 128), np.float32)
    st = Stream()
    enc.vectorize_device(d_q, d_l, Q, q_stride, d_o, st)
    st.synchronize()
    ts = []
    for _ in range(reps):
        a, b = Event(), Event()
        a.record(st)
        enc.vectorize_device(d_q, d_l, Q, q_stride, d_o, st)
        b.record(st)
        st.synchronize()
        ts.append(a.elapsed_ms(b))
    ms = float(np.mean(ts))
    flop_read = 2 * 123 * 3 * 64 * 2 * ((64 + 64 + 64) + (128 + 256))  # issued: the f32 state as hi + lo f16 terms
    useful_read = 2 * 123 * 3 * 64 * 2 * ((64 + 64) + (64 + 128))      # the model's own products (h and x once)
    tflops = Q * flop_read / (ms * 1e-3) / 1e12
    und, short = enc.flags()
    enc.free()
    return {"kernel": "gru_encode_kernel", "ms": round(ms, 3), "reads_per_s": round(Q / (ms * 1e-3), 1),
            "roofline": {"bound": "mfma", "achieved": round(tflops, 1), "peak": ENC_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": round(tflops / ENC_PEAK_TFLOPS, 4), "counts": "issued MFMA flops (hi/lo split of the f32 state)",
                         "useful_frac": round(tflops * useful_read / flop_read / ENC_PEAK_TFLOPS, 4)},
            "flop_per_read": flop_read, "undefined_tokens": und + short,
            "note": "Vectorizer::vectorize on the GPU; not inside `value` (the north star's path starts at embeddings)"}


def l2_timing(table, d_I, d_x, d_q, q_stride, gru_queries, Q, K, truth, dev, reps=3):
    """The reference's live post-processing, post_process_l2_static (src/main.cpp:330), on this step's
    neighbours: drm_refs_embed builds the window-embedding table once (GRU, on the GPU), then
    drm_post_process_l2_static_device (l2_rerank.hip) is timed with HIP events. Algorithmic bytes per launch:
    Q*K*(4*128 embedding row + 8 label) + Q*4*128 query + Q*K*(4 + 8) top-k rows (K <= 128 runs the fused
    distance + sort kernel, which keeps the candidates on chip). Not inside `value` (the metric's rerank is the
    SW one)."""
    from deepreadmapper_amd.encoder import Encoder
    from deepreadmapper_amd.device import DeviceBuffer, Event, Stream
    from deepreadmapper_amd.rerank import embed_windows
    from deepreadmapper_amd._native import check, lib
    enc = Encoder(device=dev)
    st = Stream()
    t0 = time.time()
    embed_windows(table, enc, st)
    table_s = time.time() - t0
    if not gru_queries:  # the table is the GRU's, so the query side must be too (the search ran on the stand-in)
        d_l = DeviceBuffer.from_host(np.full(Q, q_stride, dtype=np.int32))
        d_x = DeviceBuffer((Q, 128), np.float32)
        enc.vectorize_device(d_q, d_l, Q, q_stride, d_x, st)
        st.synchronize()
    enc.free()
    d_d, d_i, d_s = DeviceBuffer((Q, K), np.float32), DeviceBuffer((Q, K), np.uint64), DeviceBuffer(Q, np.int32)

    def run():
        check(lib().drm_post_process_l2_static_device(table.handle, d_I.ptr, Q, K, d_x.ptr, 128, 1, K, d_d.ptr,
                                                      d_i.ptr, d_s.ptr, st.handle))
    run()
    st.synchronize()
    ts = []
    for _ in range(reps):
        a, b = Event(), Event()
        a.record(st)
        run()
        b.record(st)
        st.synchronize()
        ts.append(a.elapsed_ms(b))
    ms = float(np.mean(ts))
    status = d_s.download()
    if not (status == K).all():
        raise SystemExit(f"L2 rerank status != K for {(status != K).sum()} queries")
    ids = d_i.download()
    algo = float(Q) * K * (4 * 128 + 8) + Q * 4 * 128 + Q * K * 12 + (Q * K * 12 * 2 if K > 128 else 0)
    gbs = algo / (ms * 1e-3) / 1e9
    # HBM bytes per dispatch from the committed PMC of tools/scripts/l2_bench.py (same Q and K, random labels)
    prof_path, pmc = committed_pmc("l2_fused_kernel" if K <= 128 else "l2_dist_staged_kernel", "l2_c5shape")
    traffic = float(pmc["hbm_bytes_est"]) if pmc and "hbm_bytes_est" in pmc and (Q, K) == (1_250_000, 128) else None
    return {"kernel": "l2_fused_kernel (+ l2_topk_kernel for ties)" if K <= 128 else "l2_dist_staged_kernel + l2_sort_kernel", "ms": round(ms, 3), "reads_per_s": round(Q / (ms * 1e-3), 1),
            "roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(gbs / HBM_PEAK_GBS, 4), "bytes_per_launch": algo, "traffic": traffic,
                         "traffic_source": (f"{prof_path}: (2*FETCH_SIZE + WRITE_SIZE) per dispatch of "
                                            "tools/scripts/l2_bench.py (1.25M reads x 128 random labels)")
                         if traffic is not None else None},
            "window_table_embed_s": round(table_s, 2),
            "truth_top1": round(float(np.mean(ids[:, 0].astype(np.int64) == truth)), 4),
            "note": "post_process_l2_static on this step's neighbours (the reference's live rerank, whose outputs "
                    "its main does not save); not inside `value`"}


def host_path(ix, table, q_emb, queries, K, EF, flat):
    """The drop-in boundary's own rate (not `value`): drm_search_rerank from pinned host buffers to pinned
    host outputs -- PCIe transfers in, kernels, PCIe transfers out, batches overlapped (exec.cpp) --
    timed once after one warm call, on this rank's reads."""
    if flat:
        return None
    from deepreadmapper_amd.executor import pinned_empty, prepare, search_rerank
    n = len(q_emb)
    x = pinned_empty(q_emb.shape, np.float32)
    x[...] = q_emb
    qb = pinned_empty(queries.shape, np.uint8)
    qb[...] = queries
    ql = pinned_empty((n,), np.int32)
    ql[...] = queries.shape[1]
    out = {"D": pinned_empty((n, K), np.float32), "I": pinned_empty((n, K), np.int64),
           "sw_scores": pinned_empty((n, K), np.int32), "sw_ids": pinned_empty((n, K), np.uint64),
           "status": pinned_empty((n,), np.int32)}
    bytes_io = x.nbytes + qb.nbytes + ql.nbytes + sum(v.nbytes for v in out.values())
    prepare(ix, n, q_emb.shape[1], K, K, queries.shape[1])
    search_rerank(ix, table, x, (qb, ql), k=K, ef=EF, out=out)
    t0 = time.perf_counter()
    o = search_rerank(ix, table, x, (qb, ql), k=K, ef=EF, out=out)
    ms = (time.perf_counter() - t0) * 1e3
    return {"value": round(n / (ms * 1e-3), 1), "unit": "reads/s", "ms": round(ms, 2),
            "device_span_ms": round(o["stats"].kernel_ms, 2), "pcie_bytes": int(bytes_io),
            "status_ok": bool((o["status"] == K).all()),
            "note": "drm_search_rerank, pinned host in/out, one rank, PCIe-inclusive (not the metric)"}


def dep_load_latency(dev, waves, footprint=16 << 30, hops=2000):
    """The search's dependent row load on this box, measured now (drm_device_chase_latency: `waves` waves -- the
    search's resident count -- each walking 384-B rows of a 16 GB random table, one row behind the other), in seconds,
    with its source. Falls back to the round-3 box measurement (DEP_LOAD_LATENCY_S) if the probe fails."""
    import ctypes as C
    from deepreadmapper_amd._native import lib
    ns = C.c_double(0.0)
    rc = lib().drm_device_chase_latency(int(dev), int(footprint), int(waves), int(hops), C.byref(ns))
    if rc != 0 or not ns.value > 0:
        return DEP_LOAD_LATENCY_S, "profiles/r03/box_diag_A.txt (the live probe failed)"
    return ns.value * 1e-9, (f"measured in this run: drm_device_chase_latency, {waves} waves x {hops} dependent "
                             f"384-B row loads over {footprint >> 30} GB")


def comm_unique_id(D):
    """Rank 0's RCCL unique id, broadcast over the gloo control plane (None if it failed, or if rank 0's
    communicator exists already). Collective, whatever state a rank is in: every rank calls it at the same point."""
    from deepreadmapper_amd.executor import Comm
    obj = [None]
    if D.rank == 0 and D.comm is None:
        try:
            obj = [Comm.unique_id()]
        except Exception as e:  # noqa: BLE001
            log(f"[bench] rank 0: RCCL unique id failed: {e}")
    D.dist.broadcast_object_list(obj, src=0)
    return obj[0]


def ensure_comm(D, dev, uid):
    """The job's RCCL communicator (drm_comm), created once from comm_unique_id's id."""
    if D.comm is None:
        from deepreadmapper_amd.executor import Comm
        if uid is None:
            raise RuntimeError("no RCCL unique id from rank 0")
        D.comm = Comm(uid, D.world, D.rank, dev)
    return D.comm


def load_index(args, D, path, dev):
    """The C5/C3 index replica of this rank. N > 1 with one GPU per rank (args.index_bcast, the default): rank 0
    parses the IHNp file and drm_index_broadcast replicates it over RCCL, each receiver
    checking the root's buffer checksums; otherwise, or if the broadcast failed on any rank (the ranks agree on that
    over gloo), every rank loads the file itself. Returns (index, {how the replica was made})."""
    from deepreadmapper_amd.device import device_count
    from deepreadmapper_amd.search import HnswPqIndex
    t0 = time.time()
    if D.world == 1 or not args.index_bcast or D.world > device_count():
        why = "one rank" if D.world == 1 else ("--no-index-bcast" if not args.index_bcast else
                                                 "ranks share a device (RCCL needs one GPU per rank)")
        ix = HnswPqIndex(path, dev)
        return ix, {"mode": "file per rank", "why": why, "s": round(time.time() - t0, 2)}
    uid = comm_unique_id(D)
    ix, err = None, None
    try:
        comm = ensure_comm(D, dev, uid)
        root_ix = HnswPqIndex(path, dev) if D.rank == 0 else None
        t_load = time.time() - t0
        t1 = time.time()
        ix = HnswPqIndex.broadcast(comm, root_ix, root=0)
        t_bcast = time.time() - t1
    except Exception as e:  # noqa: BLE001 -- every rank then falls back together
        err = f"{type(e).__name__}: {e}"
        log(f"[bench] rank {D.rank}: index broadcast failed: {err}")
    if D.allreduce(1.0 if err else 0.0, "SUM") > 0:
        if ix is not None:
            ix.free()
        ix = HnswPqIndex(path, dev)
        return ix, {"mode": "file per rank", "why": "broadcast failed", "error": err, "s": round(time.time() - t0, 2)}
    return ix, {"mode": "rccl broadcast (drm_index_broadcast)", "root_load_s": round(t_load, 2),
                "broadcast_s": round(t_bcast, 2), "device_bytes": int(ix.info.device_bytes)}


def gather_results(D, dev, n_total, bufs):
    """End-of-run exchange: every rank's device-resident result rows are gathered to
    rank 0 over RCCL by the library's own C++ path (drm_comm_gather_rows: grouped ncclSend/ncclRecv over
    xGMI), after the timed region. Verification (shard_checksums): every rank checksums its own rows on the device
    (drm_device_checksum, position-dependent), rank 0 checksums each rank's row range of the gathered buffers on the
    device, and the sums are compared over the gloo control plane -- every rank's shard is checked and nothing is
    copied to the host. An exception is returned as {"error": ...}: gather_verdict turns it into a failed job."""
    if D.world == 1:
        return None
    from deepreadmapper_amd.device import device_count
    ndev = device_count()
    if D.world > ndev:  # RCCL needs one GPU per rank (drm_comm_init: DRM_ERR_UNSUPPORTED)
        return {"skipped": f"{D.world} ranks share {ndev} device(s): the RCCL gather needs one GPU per rank"}
    # the unique-id broadcast and the checksum exchange are collectives on the gloo control plane: every rank reaches
    # them whatever happened to its own gather (an error is carried in the exchange), so a failing rank cannot leave
    # the others waiting in a collective it never enters
    from deepreadmapper_amd.device import DeviceBuffer, synchronize
    uid = comm_unique_id(D)
    out, full, local = {}, {}, None
    try:
        ensure_comm(D, dev, uid)
        synchronize()
        t0 = time.perf_counter()
        nbytes = 0
        for name, b in bufs:
            row = b.nbytes // b.shape[0]
            recv = DeviceBuffer((n_total,) + tuple(b.shape[1:]), b.dtype) if D.rank == 0 else None
            D.comm.gather_rows(b, n_total, row, recv, root=0)
            full[name] = recv
            nbytes += b.nbytes
        synchronize()
        ms = (time.perf_counter() - t0) * 1e3
        out = {"backend": "RCCL (drm_comm_gather_rows, C++)", "ms": round(ms, 3), "bytes_per_rank": int(nbytes)}
        local = {name: b.checksum() for name, b in bufs}
    except Exception as e:  # noqa: BLE001 -- reported in the JSON line
        out = {"error": f"{type(e).__name__}: {e}"}
        local = None
    ok0 = "error" not in out
    match = shard_checksums(D, n_total, local, (lambda lo, hi: {k: v.checksum(lo, hi) for k, v in full.items()})
                            if ok0 else (lambda lo, hi: None))
    if D.rank == 0 and ok0:
        out["shards_match"] = match
        out["rows"] = int(n_total)
    return out


def shard_checksums(D, n_total, local_sums, slice_sums):
    """Every rank's checksums of its own result rows (local_sums: {buffer: sum}) against rank 0's checksums of that
    rank's row range [lo_r, hi_r) of the gathered buffers (slice_sums(lo, hi) -> {buffer: sum}), exchanged over the
    gloo control plane. Returns rank 0's list of per-rank matches (None on the other ranks)."""
    from deepreadmapper_amd.shard import shard_range
    sums = [None] * D.world
    D.dist.all_gather_object(sums, local_sums)
    if D.rank != 0:
        return None
    # a rank whose gather failed sends None: its shard does not match
    return [sums[r] is not None and slice_sums(*shard_range(n_total, r, D.world)) == sums[r] for r in range(D.world)]


def gather_verdict(D, gather):
    """N > 1: did the end-of-run RCCL gather work on every rank? True / False, or None when there is nothing to
    check (one rank, or ranks sharing a device, where RCCL cannot run). Every rank reaches the same answer (sums
    over ranks of failure and skip flags on the gloo control plane), so a broken gather fails the whole job: the
    JSON line carries `gather_ok` and the bench exits non-zero."""
    if D.world == 1:
        return None
    skipped = gather is not None and "skipped" in gather
    bad = not skipped and (gather is None or "error" in gather or
                           (D.rank == 0 and not all(gather.get("shards_match") or [False])))
    n_bad = D.allreduce(1.0 if bad else 0.0, "SUM")
    n_skip = D.allreduce(1.0 if skipped else 0.0, "SUM")
    if n_bad > 0:
        return False
    return None if n_skip > 0 else True


def run_c4(args, D):
    """C4: genome ~20 Mbp, stride-4 sparse index of 10M windows, 1M queries per
    GPU, HNSW + PQ-ADC only, at K=128 (headline) and k=5 (K_CLUSTERS, the reference's sparse default).
    The index (80 MB codes + 1.28 GB level-0 rows) is far larger than the 256 MB Infinity Cache."""
    from deepreadmapper_amd import synth
    from deepreadmapper_amd.device import DeviceBuffer, Event, Stream, device_count, set_device, synchronize
    from deepreadmapper_amd.shard import shard_range
    from deepreadmapper_amd.search import HnswPqIndex

    ndev = device_count()
    set_device(D.local_rank % max(ndev, 1))
    N = D.world
    Q = args.queries or 1_000_000
    w = synth.Workload("c4", 20_000_299, N * Q, stride=4, seed=43, read_seed=8)
    if D.rank == 0:
        t0 = time.time()
        w.generate(args.cache, nthreads=args.build_threads, log=log, need_refs=False, gpu_build=True,
                   device=D.local_rank % max(ndev, 1))
        log(f"[bench] C4 workload ready in {time.time() - t0:.1f}s: index {w.index_path}")
    D.barrier()
    if D.rank != 0:
        w.generate(args.cache, need_refs=False, gpu_build=True)
    lo, hi = shard_range(N * Q, D.rank, N)
    q_emb = np.ascontiguousarray(w.q_emb[lo:hi])
    ix = HnswPqIndex(w.index_path, D.local_rank % max(ndev, 1))
    info = ix.info
    d_x = DeviceBuffer.from_host(q_emb)
    stream = Stream()
    runs = {}
    for K in (args.k, 5):
        d_D, d_I = DeviceBuffer((Q, K), np.float32), DeviceBuffer((Q, K), np.int64)
        d_nd, d_nh, d_nu = DeviceBuffer(Q, np.int32), DeviceBuffer(Q, np.int32), DeviceBuffer(Q, np.int32)
        for _ in range(args.warmup):
            ix.search_device(d_x, Q, K, args.ef, d_D, d_I, d_nd, d_nh, stream, d_nhops_upper=d_nu)
        stream.synchronize()
        ev = [(Event(), Event()) for _ in range(args.steps)]
        D.barrier()
        synchronize()
        t0 = time.perf_counter()
        for e in ev:
            e[0].record(stream)
            ix.search_device(d_x, Q, K, args.ef, d_D, d_I, d_nd, d_nh, stream, d_nhops_upper=d_nu)
            e[1].record(stream)
        stream.synchronize()
        synchronize()
        el = D.allreduce(time.perf_counter() - t0, "MAX")
        ms = float(np.mean([e[0].elapsed_ms(e[1]) for e in ev]))
        # faiss's ndis for the algorithmic bytes: one untimed exact-statistics search (see main())
        ix.set_exact_stats(True)
        ix.search_device(d_x, Q, K, args.ef, d_D, d_I, d_nd, d_nh, stream, d_nhops_upper=d_nu)
        stream.synchronize()
        ix.set_exact_stats(False)
        ndis, nhops, nup = d_nd.download().astype(np.int64), d_nh.download().astype(np.int64), d_nu.download()
        code = (info.pq_M * info.pq_nbits + 7) // 8
        bytes_q = 4 * info.d + (nhops - nup) * 2 * info.M_hnsw * 4 + nup * info.M_hnsw * 4 + ndis * code + K * 12
        bl = float(bytes_q.sum() + info.pq_M * (1 << info.pq_nbits) * (info.d // info.pq_M) * 4)
        runs[K] = {"value": N * Q * args.steps / el, "ms": ms, "ndis": float(ndis.mean()), "nhops": float(nhops.mean()),
                   "achieved": bl / (ms * 1e-3) / 1e9}
    cpu = None
    if D.rank == 0 and N == 1 and not args.no_cpu:
        from oracle import faiss_file, oracle as O
        threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
        threads = max(1, min(threads, len(os.sched_getaffinity(0))))
        s_ix = O.make_index(faiss_file.read(w.index_path))
        n = 2000
        t0 = time.perf_counter()
        O.hnswpq_search(s_ix, q_emb[:n], args.k, args.ef, nthreads=threads)
        dt = time.perf_counter() - t0
        n = int(max(n, min(len(q_emb), args.cpu_budget / max(dt / n, 1e-9))))
        t0 = time.perf_counter()
        O.hnswpq_search(s_ix, q_emb[:n], args.k, args.ef, nthreads=threads)
        dt = time.perf_counter() - t0
        cpu = {"value": n / dt, "unit": "reads/s", "cores": threads, "kind": "port",
               "sample": f"first {n} C4 queries, oracle search only (OpenMP {threads} threads on {cpu_model()})"}
    if D.rank == 0:
        r = runs[args.k]
        emit({
            "metric": f"searched reads/sec (HNSW-PQ only), EF={args.ef} K={args.k}",
            "value": round(r["value"], 1), "unit": "reads/s", "n_gpus": N, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(r["ms"], 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "fp32 (PQ-ADC distances)",
            "data": f"synthetic (seeded genome/reads, {EMBED_DESC[args.embed]} embeddings; no network)",
            "config": {"workload": "C4: synthetic 20 Mbp genome, stride-4 sparse IndexHNSWPQ of "
                                   f"{info.ntotal} windows (M_pq=8 nbits=8 M_hnsw=16 EFC=200, GPU-built), search only",
                       "n_refs": int(info.ntotal), "queries_per_gpu": Q, "ef": args.ef, "k": args.k,
                       "parallelism": f"dp{N} (query shards, index replicated per GPU)"},
            "roofline": {"bound": "hbm", "kernel": SEARCH_KERNEL, "achieved": round(r["achieved"], 2),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(r["achieved"] / HBM_PEAK_GBS, 5),
                         "traffic": None, "avg_launch_ms": round(r["ms"], 4)},
            "cpu_baseline": cpu,
            "k5": {"value": round(runs[5]["value"], 1), "ms": round(runs[5]["ms"], 3),
                   "achieved_gbs": round(runs[5]["achieved"], 2)},
            "breakdown": {"ndis_mean": round(r["ndis"], 1), "nhops_mean": round(r["nhops"], 1)},
        })
    D.close()


def sw_band_timing(table, d_I, d_q, d_ql, qstride, Q, K, band, search_ms, sw_ms, ids_full, sc_full, truth, stream):
    """The opt-in banded SW rerank (an extension; the reference scores the full DP) on the timed step's search rows:
    its time, the step it would make, and how far its results move from the full DP's (NOT the headline)."""
    from deepreadmapper_amd.device import DeviceBuffer, Event
    from deepreadmapper_amd._native import check, lib
    d_sc, d_id, d_st = DeviceBuffer((Q, K), np.int32), DeviceBuffer((Q, K), np.uint64), DeviceBuffer(Q, np.int32)

    def run():
        check(lib().drm_post_process_sw_static_device(table.handle, d_I.ptr, Q, K, d_q.ptr, d_ql.ptr, qstride, 1, K, K,
                                                      d_sc.ptr, d_id.ptr, d_st.ptr, stream.handle))
    table.sw_band = band
    try:
        run()
        ts = []
        for _ in range(3):
            e0, e1 = Event(), Event()
            e0.record(stream)
            run()
            e1.record(stream)
            stream.synchronize()
            ts.append(e0.elapsed_ms(e1))
    finally:
        table.sw_band = 0
    ms = float(np.mean(ts))
    ids, sc = d_id.download(), d_sc.download()
    return {"band": band, "note": "opt-in banded DP (cells |i - j| <= band), not parity with the reference; the "
                                  "headline above is the full DP",
            "sw_rerank_ms": round(ms, 3), "full_dp_sw_rerank_ms": round(sw_ms, 3),
            "step_ms": round(search_ms + ms, 3), "reads_per_s_device": round(Q / ((search_ms + ms) * 1e-3), 1),
            "top1_id_equal_full": round(float(np.mean(ids[:, 0] == ids_full[:, 0])), 4),
            "topk_scores_equal_full": round(float(np.mean(sc == sc_full)), 4),
            "truth_top1": round(float(np.mean(ids[:, 0].astype(np.int64) == truth)), 4)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--queries", type=int, default=0, help="reads per GPU (weak scaling); 0 = the workload's own")
    ap.add_argument("--ef", type=int, default=128)
    ap.add_argument("--k", type=int, default=128)
    ap.add_argument("--cache", default=os.environ.get("DRM_BENCH_CACHE", "/tmp/drm_bench_cache"))
    ap.add_argument("--cpu-budget", type=float, default=12.0, help="seconds of oracle CPU work")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-host-path", action="store_true", help="skip the pinned-host drm_search_rerank timing")
    ap.add_argument("--no-encoder", action="store_true", help="skip the GRU read-encoder timing")
    ap.add_argument("--no-l2", action="store_true", help="skip the L2 rerank (post_process_l2_static) timing (always "
                                                         "skipped at N > 1)")
    ap.add_argument("--embed", choices=["kmer3", "gru"], default=None,
                    help="embeddings of windows and reads: gru (default for c5: the reference's GRU model, run on the "
                         "GPU by drm_vectorize) or kmer3 (the deterministic 3-mer stand-in; default for c3/c4)")
    ap.add_argument("--build-threads", type=int, default=0)
    ap.add_argument("--index", choices=["pq", "flat"], default="pq",
                    help="pq (default): faiss IndexHNSWPQ, the live pipeline's index (src/main.cpp:236-237); flat: "
                         "hnswlib fp32-L2 index (M=64, EFC=128, the reference's hnswlib defaults) over the C3 windows")
    ap.add_argument("--index-bcast", action=argparse.BooleanOptionalAction, default=True,
                    help="N > 1 (one GPU per rank): rank 0 loads the index file and drm_index_broadcast replicates it "
                         "over RCCL (default); --no-index-bcast: every rank parses the file itself")
    ap.add_argument("--sw-band", type=int, default=0, choices=[0, 8, 16, 32],
                    help="also time the opt-in banded SW rerank (drm_refs_set_sw_band, NOT parity with the reference) on "
                         "the same search rows, reported beside the headline as `sw_band_opt_in`; 0 = skip")
    ap.add_argument("--workload", choices=["c3", "c4", "c5"], default="c5",
                    help="c5 (default): the metric's configuration (50M windows, 1.25M reads per GPU), search + SW "
                         "rerank; c3: 1M windows, 100k reads per GPU, search + SW rerank; c4: search only on a 10M-vector "
                         "sparse (stride 4) index, SURVEY.md sec. 8d")
    args = ap.parse_args()
    _claim_stdout()

    D = Dist()
    if args.embed is None:
        args.embed = "gru" if args.workload == "c5" else "kmer3"
    if args.embed == "gru" and (args.workload != "c5" or args.index != "pq"):
        raise SystemExit("--embed gru builds the C5 PQ index only")
    if args.workload == "c4":
        return run_c4(args, D)
    from deepreadmapper_amd import synth
    from deepreadmapper_amd.device import DeviceBuffer, Event, Stream, device_count, device_props, set_device, synchronize
    from deepreadmapper_amd.shard import shard_range
    from deepreadmapper_amd.search import HnswPqIndex
    from deepreadmapper_amd.rerank import WindowTable
    from deepreadmapper_amd._native import check, lib

    ndev = device_count()
    dev = D.local_rank % max(ndev, 1)  # one rank per GPU; ranks share GPUs only on smaller boxes
    set_device(dev)
    N, K, EF = D.world, args.k, args.ef
    flat = args.index == "flat"
    if args.workload == "c5":
        if flat:
            raise SystemExit("--index flat is a C3 variant")
        wl = prepare_c5(args, D, dev)
    else:
        wl = prepare_c3(args, D, dev)
    Q = wl["Q"]
    q_emb, queries, truth, refs = wl["q_emb"], wl["queries"], wl["truth"], wl["refs"]

    if flat:
        from deepreadmapper_amd.flat import HnswFlatIndex
        fpath = os.path.join(args.cache, "c3_flat_M64_efc128.hnsw")
        if D.rank == 0 and not os.path.exists(fpath):
            t0 = time.time()
            synth.build_flat_index(synth.embed(synth.tag(refs)), fpath + ".tmp", M=64, efc=128,
                                   nthreads=args.build_threads)
            os.replace(fpath + ".tmp", fpath)
            log(f"[bench] hnswlib fp32 index built in {time.time() - t0:.1f}s")
        D.barrier()
        ix = HnswFlatIndex(fpath, dev)
        replication = {"mode": "file per rank", "why": "hnswlib index"}
        d_L = DeviceBuffer((Q, K), np.uint64)
    else:
        t0 = time.time()
        ix, replication = load_index(args, D, wl["index_path"], dev)
        log(f"[bench] index replica ready in {time.time() - t0:.1f}s: {replication}")
    t0 = time.time()
    table = WindowTable(refs, dev)
    log(f"[bench] window table ({len(refs)} x {refs.shape[1]} B) uploaded in {time.time() - t0:.1f}s")
    d_x = DeviceBuffer.from_host(q_emb)
    d_q = DeviceBuffer.from_host(queries)
    d_ql = DeviceBuffer.from_host(np.full(Q, queries.shape[1], dtype=np.int32))
    d_D = DeviceBuffer((Q, K), np.float32)
    d_I = DeviceBuffer((Q, K), np.int64)
    d_nd, d_nh, d_nu = DeviceBuffer(Q, np.int32), DeviceBuffer(Q, np.int32), DeviceBuffer(Q, np.int32)
    d_sc, d_id, d_st = DeviceBuffer((Q, K), np.int32), DeviceBuffer((Q, K), np.uint64), DeviceBuffer(Q, np.int32)
    stream = Stream()
    def step(ev=None):
        if ev:
            ev[0].record(stream)
        if flat:
            ix.search_device(d_x, Q, K, EF, d_D, d_L, d_nd, d_nh, stream, d_nhops_upper=d_nu)
        else:
            ix.search_device(d_x, Q, K, EF, d_D, d_I, d_nd, d_nh, stream, d_nhops_upper=d_nu)
        if ev:
            ev[1].record(stream)
        check(lib().drm_post_process_sw_static_device(table.handle, (d_L if flat else d_I).ptr, Q, K, d_q.ptr,
                                                      d_ql.ptr,
                                                      queries.shape[1], 1, K, K, d_sc.ptr, d_id.ptr, d_st.ptr,
                                                      stream.handle))
        if ev:
            ev[2].record(stream)

    for _ in range(args.warmup):
        step()
    stream.synchronize()
    events = [[Event(), Event(), Event()] for _ in range(args.steps)]
    D.barrier()
    synchronize()
    t0 = time.perf_counter()
    for s in range(args.steps):
        step(events[s])
    stream.synchronize()
    synchronize()
    elapsed = time.perf_counter() - t0
    D.barrier()
    elapsed_max = D.allreduce(elapsed, "MAX")
    search_ms = float(np.mean([e[0].elapsed_ms(e[1]) for e in events]))
    sw_ms = float(np.mean([e[1].elapsed_ms(e[2]) for e in events]))
    span_ms = search_ms + sw_ms
    if os.environ.get("DRM_BENCH_VERBOSE"):
        print("per-step search ms", [round(e[0].elapsed_ms(e[1]), 2) for e in events],
              "sw ms", [round(e[1].elapsed_ms(e[2]), 2) for e in events], file=sys.stderr, flush=True)

    # correctness / quality of this rank's last step
    if flat and ix.overflows():
        raise SystemExit(f"{ix.overflows()} queries outgrew the GPU candidate heap")
    n_err = ix.search_errors()  # queries past the hop bound / waves past the item bound
    if n_err:
        raise SystemExit(f"{n_err} search errors (hop / work-item bounds): search state broken")
    st = d_st.download()
    if not (st == K).all():
        raise SystemExit(f"rerank status != K for {(st != K).sum()} queries")
    ndis, nhops, nup = d_nd.download().astype(np.int64), d_nh.download().astype(np.int64), d_nu.download()
    if (nhops < 0).any():
        raise SystemExit(f"{int((nhops < 0).sum())} queries ended on the search's hop bound")
    ndis_computed = ndis
    if not flat:
        # faiss's ndis (the links each hop finds not yet visited: SURVEY.md sec. 8d's algorithmic bytes) from one
        # untimed exact-statistics search of the same reads (a visited bitmap kept beside the search only for the
        # count); the lean kernel's own ndis counts every distance it computed. Its rows must equal the timed run's.
        I_timed = d_I.download()
        ix.set_exact_stats(True)
        ix.search_device(d_x, Q, K, EF, d_D, d_I, d_nd, d_nh, stream, d_nhops_upper=d_nu)
        stream.synchronize()
        ix.set_exact_stats(False)
        if not np.array_equal(d_I.download(), I_timed):
            raise SystemExit("the exact-statistics search returned different rows")
        ndis = d_nd.download().astype(np.int64)
        del I_timed
    ids = d_id.download()
    top1 = float(np.mean(ids[:, 0].astype(np.int64) == truth))
    intop = float(np.mean((ids.astype(np.int64) == truth[:, None]).any(axis=1)))

    # algorithmic bytes of the search kernel, per launch:
    #   512 (query) + 2*M*4 per level-0 hop + M*4 per upper hop + ndis*code_size + K*12 (ids+dists)
    info = ix.info
    l0 = nhops - nup
    if flat:
        # fp32: a level-0 row is maxM0 links + count, an upper row maxM + count, a distance a 4d-byte vector
        bytes_q = 4 * info.d + l0 * (info.maxM0 + 1) * 4 + nup * (info.maxM + 1) * 4 + ndis * 4 * info.d + K * 12
        bytes_launch = float(bytes_q.sum())
    else:
        deg0 = 2 * info.M_hnsw
        code = (info.pq_M * info.pq_nbits + 7) // 8
        bytes_q = 4 * info.d + l0 * deg0 * 4 + nup * info.M_hnsw * 4 + ndis * code + K * 12
        codebook = info.pq_M * (1 << info.pq_nbits) * (info.d // info.pq_M) * 4
        bytes_launch = float(bytes_q.sum() + codebook)
    achieved = bytes_launch / (search_ms * 1e-3) / 1e9
    # the device, read at run time: the issue ceilings below use its CU count and peak engine clock
    props = device_props(dev)
    ncu, clock_hz = props["cu_count"], props["clock_hz"]
    # latency floor of the pointer chase: every hop (upper or level 0) waits for one dependent row load, and a CU
    # holds lds_per_cu / LUT queries in flight (20 at 160 KB / 8 KB), so no schedule of this design finishes sooner
    # than hops / (CUs x queries per CU) x the dependent-load latency
    q_per_cu = max(1, props["lds_per_cu"] // SEARCH_LUT_BYTES) if not flat else None
    dep_lat_s, dep_lat_src = (dep_load_latency(dev, ncu * q_per_cu) if not flat else (None, None))
    lat_floor_ms = (float(nhops.sum()) / (ncu * q_per_cu) * dep_lat_s * 1e3) if not flat else None
    cells = float(Q) * K * refs.shape[1] * queries.shape[1]
    search_kernel = FLAT_KERNEL if flat else SEARCH_KERNEL
    pkey = args.workload + ("_flat" if flat else "") + ("_gru" if args.embed == "gru" else "")
    prof_path, pmc = committed_pmc(search_kernel, pkey)
    traffic = None
    if pmc and "hbm_bytes_est" in pmc:
        traffic = float(pmc["hbm_bytes_est"])
    sw_prof_path, sw_pmc = committed_pmc(SW_KERNEL, pkey)
    sw_gcups = cells / (sw_ms * 1e-3) / 1e9
    # SW roofline = the hardware's VALU issue rate: 4 SIMDs per CU, each issuing one wave64 VALU instruction per 4
    # cycles (packed 16-bit) or per 2 cycles (32-bit). Instructions per launch: the committed PMC count of this
    # workload's SW kernel when there is one (SQ_INSTS_VALU per dispatch), else the static DP count (one wave
    # instruction advances 64 lanes x 2 candidates by one cell; 3.51 per cell pair); issue cycles = instructions x
    # the DP block's average cycles per instruction (SW_ISSUE_CYC_PER_VALU)
    sw_peak_cyc = ncu * 4 * clock_hz
    # the DP's own cells: the tags of the 152-byte queries are not DP columns (sw_rerank.hip)
    dp_cells = float(Q) * K * refs.shape[1] * max(queries.shape[1] - 2, 1)
    sw_instr_static = dp_cells / 128.0 * SW_VALU_PER_CELL_PAIR
    sw_instr, sw_instr_src = sw_instr_static, "static ISA count of the DP block"
    if sw_pmc and "SQ_INSTS_VALU" in sw_pmc and (Q, K) == (1_250_000, 128):
        sw_instr, sw_instr_src = float(sw_pmc["SQ_INSTS_VALU"]), f"{sw_prof_path}: SQ_INSTS_VALU per dispatch"
    sw_achieved_cyc = sw_instr * SW_ISSUE_CYC_PER_VALU / (sw_ms * 1e-3)
    # the whole rerank's time (scoring, top-k, flagged re-scores) per DP cell pair per SIMD, against the mix floor
    sw_cyc_pair = (sw_ms * 1e-3) * clock_hz * ncu * 4 / (dp_cells / 2.0 / 64.0)

    host = None if args.no_host_path else host_path(ix, table, q_emb, queries, K, EF, flat)
    enc = None if args.no_encoder else encoder_timing(d_q, Q, queries.shape[1], dev)
    # the L2 rerank is outside the metric's path: its window-embedding table (25.6 GB, ~3 s
    # per rank at C5) stays off the multi-GPU scaling runs
    l2 = None if (args.no_l2 or flat or N > 1) else l2_timing(table, d_I, d_x, d_q, queries.shape[1],
                                                               args.embed == "gru", Q, K, truth, dev)
    if l2 is None and N > 1 and not (args.no_l2 or flat):
        l2 = {"skipped": "N > 1: the L2 rerank leg (not part of the metric) runs at N = 1 only"}

    band = sw_band_timing(table, d_I, d_q, d_ql, queries.shape[1], Q, K, args.sw_band, search_ms, sw_ms, ids,
                          d_sc.download(), truth, stream) if (args.sw_band and not flat) else None

    total_reads = float(N * Q * args.steps)
    value = total_reads / elapsed_max
    gather = gather_results(D, dev, N * Q, [("sw_ids", d_id), ("sw_scores", d_sc), ("search_ids", d_L if flat else d_I),
                                           ("search_dists", d_D)])
    gather_ok = gather_verdict(D, gather)
    result = None
    if D.rank == 0:
        cpu = None
        if N == 1 and not args.no_cpu:
            cpu = cpu_baseline(refs, fpath if flat else wl["index_path"], queries, q_emb, K, EF, args.cpu_budget, log,
                               flat=flat)
        workload = wl["desc"] if not flat else (
                    "C3-flat: the same 1M windows in an hnswlib fp32-L2 index (M=64, EFC=128), hnswlib searchKnn + "
                    "SW rerank, EF=128 K=128")
        result = {
            "metric": "mapped reads/sec, 150 bp queries, EF=128 K=128",
            "value": round(value, 1), "unit": "reads/s", "n_gpus": N, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed_max / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None,
            "dtype": ("fp32 (L2 distances)" if flat else "fp32 (PQ-ADC distances)") + (
                " + int32 (SW DP, bit-profile u16 kernel)" if os.environ.get("DRM_SW_BITPROFILE") == "1" else
                " + u16 integer SW DP (two cells per register)"),
            "data": f"synthetic (seeded genome/reads, {EMBED_DESC[args.embed]} embeddings; no network)",
            "config": {"workload": workload, "n_refs": int(len(refs)), "queries_per_gpu": Q, "ef": EF, "k": K,
                       "parallelism": f"dp{N} (query shards, index replicated per GPU)"},
            "roofline": {"bound": "hbm", "kernel": search_kernel, "achieved": round(achieved, 2),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                         "traffic": traffic, "bytes_per_launch": bytes_launch, "avg_launch_ms": round(search_ms, 4),
                         "latency_floor_ms": round(lat_floor_ms, 2) if lat_floor_ms else None,
                         "frac_of_latency_floor": round(lat_floor_ms / search_ms, 3) if lat_floor_ms else None,
                         "hbm_frac_at_latency_floor": round(bytes_launch / (lat_floor_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
                         if lat_floor_ms else None,
                         "latency_floor_note": (f"{float(nhops.sum()):.4g} hops / ({ncu} CUs x {q_per_cu} queries in "
                                                f"flight per CU, the LDS limit at {SEARCH_LUT_BYTES} B of LUT each) x "
                                                f"{dep_lat_s * 1e6:.3f} us dependent-load latency ({dep_lat_src}): the "
                                                "pointer chase's floor; frac is read against it") if lat_floor_ms else None,
                         "dep_load_latency_us": round(dep_lat_s * 1e6, 4) if dep_lat_s else None,
                         "device": {"cu_count": ncu, "clock_hz": clock_hz, "arch": props["arch"]},
                         "traffic_source": (f"{prof_path}: (2*FETCH_SIZE + WRITE_SIZE) per dispatch; the x2 read "
                                            "factor calibrated on this access shape (chase_rows_kernel: 12 B per lane, "
                                            "384-B rows at random, known bytes: FETCH_SIZE x 2.000-2.001 at 1, 2 and 3 "
                                            "lines per row, profiles/r06/fetch_calib_chase_rows.txt)")
                         if traffic is not None else None,
                         "valu_issue_frac_pmc": round(pmc["valu_issue_frac"], 3)
                         if pmc and "valu_issue_frac" in pmc else None,
                         "issue": issue_ceiling(pmc, float(nhops.sum()), search_ms, ncu, clock_hz)},
            "sw_roofline": {"bound": "valu", "kernel": SW_KERNEL, "achieved": round(sw_achieved_cyc / 1e9, 2),
                            "peak": round(sw_peak_cyc / 1e9, 2), "unit": "G SIMD VALU-issue cycles/s",
                            "frac": round(sw_achieved_cyc / sw_peak_cyc, 4), "instr_per_launch": sw_instr,
                            "instr_source": sw_instr_src, "gcups": round(sw_gcups, 1),
                            "valu_per_cell_pair": round(SW_VALU_PER_CELL_PAIR, 3),
                            "issue_cycles_per_cell_pair": round(SW_VALU_PER_CELL_PAIR * SW_ISSUE_CYC_PER_VALU, 2),
                            "note": "frac = VALU issue cycles used (packed 16-bit 4, 32-bit 2 cycles per wave64 "
                                    "instruction) / the SIMDs' capacity (4 x the device's CUs x its peak clock); the DP's op count per "
                                    "cell pair is reported separately",
                            "mix_floor": {"rerank_cycles_per_cell_pair": round(sw_cyc_pair, 2),
                                          "floor_cycles_per_cell_pair_2_waves": round(SW_MIX_CYC_PER_PAIR[2], 2),
                                          "floor_cycles_per_cell_pair_8_waves": round(SW_MIX_CYC_PER_PAIR[8], 2),
                                          "frac_2_waves": round(SW_MIX_CYC_PER_PAIR[2] / sw_cyc_pair, 4),
                                          "frac_8_waves": round(SW_MIX_CYC_PER_PAIR[8] / sw_cyc_pair, 4),
                                          "source": "profiles/r04/valu_rate_mix.txt (the DP's instruction mix alone, "
                                                    "all operands in registers; the kernel holds 2 waves per SIMD)"}},
            "cpu_baseline": cpu,
            "index_replication": replication,
            "gather": gather,
            "gather_ok": gather_ok,
            "host_path": host,
            "encoder": dict(enc, with_search_rerank_reads_per_s=round(Q / ((elapsed_max / args.steps) + enc["ms"] * 1e-3), 1))
            if enc else None,
            "l2_rerank": l2,
            "sw_band_opt_in": band,
            "breakdown": {"schedule": "sequential: search, then SW rerank, each with the whole chip",
                          "device_span_ms": round(span_ms, 3),
                          "search_ms": round(search_ms, 3), "sw_rerank_ms": round(sw_ms, 3),
                          "sw_gcups": round(cells / (sw_ms * 1e-3) / 1e9, 1),
                          "ndis_mean": round(float(ndis.mean()), 1), "nhops_mean": round(float(nhops.mean()), 1),
                          "distances_computed_mean": round(float(ndis_computed.mean()), 1),
                          "bytes_per_query": round(float(bytes_q.mean()), 1),
                          "truth_top1": round(top1, 4), "truth_in_topk": round(intop, 4)},
        }
        emit(result)
    D.close()
    if gather_ok is False:
        raise SystemExit(f"rank {D.rank}: the RCCL result gather failed on some rank ({gather})")


if __name__ == "__main__":
    main()
