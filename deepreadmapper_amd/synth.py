"""Synthetic workloads of BASELINE.json: seeded genome, fwd/RC window table,
simulated 150 bp reads with DWGSIM-style names, stand-in embeddings. No network, no datasets:
everything is generated here, deterministically from the seed."""
import ctypes as C
import os

import numpy as np

from ._native import check, lib, ptr

ACGT = np.frombuffer(b"ACGT", dtype=np.uint8)
_COMP = np.zeros(256, dtype=np.uint8)
for a, b in zip(b"ACGTN", b"TGCAN"):
    _COMP[a] = b
EMBED_SEED = 42  # drm::kEmbedSeed: the CLIs embed with this seed


def genome(length, seed=42):
    rng = np.random.default_rng(seed)
    return ACGT[rng.integers(0, 4, size=length)]


def revcomp(seq):
    """reverse_complement (src/utils/parse_inputs.cpp:43-53) on uint8 arrays (ACGTN)."""
    return _COMP[np.asarray(seq, dtype=np.uint8)[::-1]]


def windows_lookup(g, ref_len=150, stride=1):
    """format_fasta(lookup_mode=True) for one contig: row 2i = g[i*stride : +ref_len], row 2i+1 = its RC."""
    g = np.asarray(g, dtype=np.uint8)
    L = len(g)
    if L < ref_len:
        return np.zeros((0, ref_len), dtype=np.uint8)
    nw = (L - ref_len) // stride + 1
    fwd = np.lib.stride_tricks.sliding_window_view(g, ref_len)[::stride][:nw]
    rcg = _COMP[g[::-1]]
    rcw = np.lib.stride_tricks.sliding_window_view(rcg, ref_len)
    starts = np.arange(nw) * stride
    rev = rcw[L - ref_len - starts]
    out = np.empty((2 * nw, ref_len), dtype=np.uint8)
    out[0::2] = fwd
    out[1::2] = rev
    return out


def simulate_reads(g, n, read_len=150, sub_rate=0.01, seed=7):
    """Reads drawn uniformly from both strands with `sub_rate` substitutions. Returns
    (reads [n, read_len] uint8, names, truth window ids) -- truth id = 2*pos + strand, i.e. the
    dense id of the window the read came from."""
    rng = np.random.default_rng(seed)
    g = np.asarray(g, dtype=np.uint8)
    pos = rng.integers(0, len(g) - read_len + 1, size=n)
    strand = rng.integers(0, 2, size=n)
    idx = pos[:, None] + np.arange(read_len)[None, :]
    reads = g[idx]
    rc = strand == 1
    reads[rc] = _COMP[reads[rc][:, ::-1]]
    subs = rng.random((n, read_len)) < sub_rate
    shift = rng.integers(1, 4, size=(n, read_len))
    code = np.searchsorted(ACGT, reads)
    code = np.where(subs, (code + shift) % 4, code)
    reads = ACGT[code]
    names = [f"_{p + 1}_{1 - s}_{s}_0_0_0_{int(subs[i].sum())}:0:0_0:0:0_{i:x}" for i, (p, s) in
             enumerate(zip(pos.tolist(), strand.tolist()))]
    return reads, names, (2 * pos + strand).astype(np.int64)


READ_BLOCK = 1 << 16


def simulate_reads_range(g, lo, hi, read_len=150, sub_rate=0.01, seed=7, block=READ_BLOCK):
    """Reads [lo, hi) of an unbounded seeded read stream, generated in fixed blocks of `block` reads
    (block b from default_rng([seed, b])), so any shard of a C5-sized batch (10M reads) is produced
    without materialising the others: rank r of N gets the same reads whatever N is. Same model as
    simulate_reads (uniform position and strand, `sub_rate` substitutions); names are omitted."""
    g = np.asarray(g, dtype=np.uint8)
    n = max(0, hi - lo)
    reads = np.empty((n, read_len), dtype=np.uint8)
    truth = np.empty(n, dtype=np.int64)
    L = len(g)
    for b in range(lo // block, (hi + block - 1) // block if n else lo // block):
        rng = np.random.default_rng([seed, b])
        pos = rng.integers(0, L - read_len + 1, size=block)
        strand = rng.integers(0, 2, size=block)
        subs = rng.random((block, read_len)) < sub_rate
        shift = rng.integers(1, 4, size=(block, read_len), dtype=np.uint8)
        s0, s1 = max(lo, b * block), min(hi, (b + 1) * block)   # the part of block b inside [lo, hi)
        j = slice(s0 - b * block, s1 - b * block)
        p, st, sb, sh = pos[j], strand[j], subs[j], shift[j]
        r = np.lib.stride_tricks.sliding_window_view(g, read_len)[p]
        rc = st == 1
        r[rc] = _COMP[r[rc][:, ::-1]]
        code = _CODE[r]
        code = np.where(sb, (code + sh) % 4, code)
        reads[s0 - lo:s1 - lo] = ACGT[code]
        truth[s0 - lo:s1 - lo] = 2 * p + st
    return reads, truth


_CODE = np.zeros(256, dtype=np.uint8)
for _i, _c in enumerate(b"ACGT"):
    _CODE[_c] = _i


def tag(reads):
    """format_fastq's "<" + seq + ">" (src/utils/parse_inputs.cpp:905-912) on a [n, L] uint8 array."""
    n, L = reads.shape
    out = np.empty((n, L + 2), dtype=np.uint8)
    out[:, 0] = ord("<")
    out[:, 1:-1] = reads
    out[:, -1] = ord(">")
    return out


def embed(seqs, dim=128, seed=EMBED_SEED):
    """drm_embed_kmer3 on a [n, L] uint8 array (or a list of byte strings)."""
    if isinstance(seqs, np.ndarray):
        arr = np.ascontiguousarray(seqs, dtype=np.uint8)
        n, L = arr.shape
        lens = np.full(n, L, dtype=np.int32)
        offs = np.arange(n, dtype=np.int64) * L
        flat = arr.reshape(-1)
    else:
        bs = [s.encode() if isinstance(s, str) else bytes(s) for s in seqs]
        n = len(bs)
        lens = np.array([len(s) for s in bs], dtype=np.int32)
        offs = np.concatenate([[0], np.cumsum(lens[:-1], dtype=np.int64)]).astype(np.int64) if n else np.zeros(0, np.int64)
        flat = np.frombuffer(b"".join(bs) or b"\0", dtype=np.uint8)
    out = np.empty((n, dim), dtype=np.float32)
    if n:
        check(lib().drm_embed_kmer3(ptr(flat), ptr(offs), ptr(lens), n, dim, C.c_uint64(seed), ptr(out)))
    return out


def build_index(x, path, M_pq=8, nbits=8, M_hnsw=16, efc=200, sample_rate=0.5, nthreads=0, seed=0):
    """hnswpq_index back end (build_faiss_index, src/hnswpq/index.cpp:86-193) -> faiss IHNp file."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    check(lib().drm_build_hnswpq(ptr(x), x.shape[0], x.shape[1], M_pq, nbits, M_hnsw, efc, sample_rate, nthreads,
                                 C.c_uint64(seed), str(path).encode()))


def build_index_gpu_from_rows(rows, path, M_pq=8, nbits=8, M_hnsw=16, efc=200, sample_rate=0.5, seed=0, device=0,
                              log=None, embed="kmer3"):
    """GPU build (drm_build_hnswpq_device) over embeddings of fixed-length rows (e.g. the window table),
    computed on the device and never leaving it: embed="kmer3" the stand-in (drm_embed_kmer3_device),
    embed="gru" the reference's GRU model (drm_vectorize_device) on the tagged rows '<' + row + '>', as
    hnswpq_index embeds its windows (src/hnswpq/index.cpp:270-280)."""
    from .device import DeviceBuffer, set_device, synchronize
    import time
    rows = np.asarray(rows)
    n, L = rows.shape
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    set_device(device)
    t0 = time.time()
    d_x = DeviceBuffer((n, 128), np.float32)
    if embed == "gru":
        from .encoder import Encoder
        enc = Encoder(device=device)
        chunk = 1 << 21
        tagged = np.empty((min(chunk, n), L + 2), dtype=np.uint8)
        tagged[:, 0], tagged[:, -1] = ord("<"), ord(">")
        d_t = DeviceBuffer(tagged.shape, np.uint8)
        d_l = DeviceBuffer.from_host(np.full(len(tagged), L + 2, dtype=np.int32))
        for lo in range(0, n, chunk):
            m = min(chunk, n - lo)
            tagged[:m, 1:-1] = rows[lo:lo + m]
            check(lib().drm_memcpy_h2d(d_t.ptr, ptr(tagged), m * (L + 2)))  # ordered after the last launch
            check(lib().drm_vectorize_device(enc.handle, d_t.ptr, d_l.ptr, m, L + 2, d_x.ptr + lo * 512, None))
        synchronize()
        d_t.free()
        enc.free()
    else:
        d_rows = DeviceBuffer.from_host(np.ascontiguousarray(rows, dtype=np.uint8))
        check(lib().drm_embed_kmer3_device(d_rows.ptr, n, L, L, 128, C.c_uint64(EMBED_SEED), d_x.ptr, None))
        d_rows.free()
    if log:
        log(f"[synth] embedded {n} rows ({embed}) on the GPU in {time.time() - t0:.1f}s")
    check(lib().drm_build_hnswpq_device(d_x.ptr, n, 128, M_pq, nbits, M_hnsw, efc, sample_rate, C.c_uint64(seed),
                                        device, str(path).encode()))
    synchronize()
    d_x.free()
    if log:
        log(f"[synth] GPU-built IndexHNSWPQ over {n} vectors in {time.time() - t0:.1f}s")


def embed_gru(tagged, device=0):
    """GRU embeddings [n, 128] f32 of tagged sequences (rows of a [n, L] u8 array) on the GPU."""
    from .encoder import Encoder
    enc = Encoder(device=device)
    t = np.ascontiguousarray(tagged, dtype=np.uint8)
    out = enc.vectorize((t, np.full(len(t), t.shape[1], dtype=np.int32)))
    enc.free()
    return out


def build_flat_index(x, path, M=64, efc=128, nthreads=0, seed=0):
    """hnswlib build_index back end (src/hnswlib_dir/index.cpp:3-49) -> hnswlib file (fp32 L2)."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    check(lib().drm_build_hnsw_flat(ptr(x), x.shape[0], x.shape[1], M, efc, nthreads, C.c_uint64(seed),
                                    str(path).encode()))


def write_fasta(path, g, header="> Synthetic genome", width=80):
    g = bytes(np.asarray(g, dtype=np.uint8))
    with open(path, "wb") as f:
        f.write(header.encode() + b"\n")
        for i in range(0, len(g), width):
            f.write(g[i:i + width] + b"\n")


def write_fastq(path, reads, names):
    with open(path, "wb") as f:
        for r, nm in zip(reads, names):
            s = bytes(r)
            f.write(b"@" + nm.encode() + b"/1\n" + s + b"\n+\n" + b"I" * len(s) + b"\n")


class Workload:
    """One BASELINE config: genome, window table, reads, embeddings, index file."""

    def __init__(self, name, genome_len, n_queries, ref_len=150, stride=1, seed=42, read_seed=7, sub_rate=0.01):
        self.name, self.genome_len, self.n_queries = name, genome_len, n_queries
        self.ref_len, self.stride, self.seed, self.read_seed, self.sub_rate = ref_len, stride, seed, read_seed, sub_rate

    def generate(self, workdir, efc=200, M_hnsw=16, M_pq=8, nbits=8, nthreads=0, build_seed=0, log=None,
                 need_refs=True, gpu_build=False, device=0):
        """need_refs=False skips the stride-1 window table (search-only workloads such as C4).
        gpu_build=True embeds the windows and builds the index on the GPU (builder_gpu.hip); the file
        name carries a _gpu suffix so host- and GPU-built indexes never mix."""
        os.makedirs(workdir, exist_ok=True)
        self.genome = genome(self.genome_len, self.seed)
        # static ref_seqs: stride 1 always
        self.refs = windows_lookup(self.genome, self.ref_len, 1) if need_refs else None
        self.reads, self.names, self.truth = simulate_reads(self.genome, self.n_queries, self.ref_len,
                                                            self.sub_rate, self.read_seed)
        self.queries = tag(self.reads)
        self.q_emb = embed(self.queries)
        suffix = "_gpu" if gpu_build else ""
        self.index_path = os.path.join(workdir, f"{self.name}_M{M_hnsw}_efc{efc}_s{self.stride}{suffix}.index")
        if not os.path.exists(self.index_path) and gpu_build:
            base = windows_lookup(self.genome, self.ref_len, self.stride) if (self.refs is None or self.stride != 1) \
                else self.refs
            tmp = self.index_path + ".tmp"
            build_index_gpu_from_rows(base, tmp, M_pq, nbits, M_hnsw, efc, 0.5, build_seed, device, log)
            os.replace(tmp, self.index_path)
        if not os.path.exists(self.index_path):
            base = windows_lookup(self.genome, self.ref_len, self.stride)
            if log:
                log(f"[synth] embedding {len(base)} windows")
            x = embed(tag(base))
            if log:
                log(f"[synth] building IndexHNSWPQ over {len(x)} vectors (efC={efc}, M={M_hnsw})")
            tmp = self.index_path + ".tmp"
            build_index(x, tmp, M_pq, nbits, M_hnsw, efc, 0.5, nthreads, build_seed)
            os.replace(tmp, self.index_path)
        return self


def c1_fixture_paths():
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    g = os.path.join(here, "tests", "golden")
    return {"fna": os.path.join(g, "ecoli_150.fna"), "fastq": os.path.join(g, "test_data.fastq"),
            "ref_txt": os.path.join(g, "test_data_ref.txt"), "quer_txt": os.path.join(g, "test_data_quer.txt")}
