"""Independent (numpy) reader of the faiss IndexHNSWPQ file -- TEST INFRASTRUCTURE ONLY.

Restates faiss impl/index_read.cpp for fourcc "IHNp" + storage "IxPq" (layout in
deepreadmapper_amd/csrc/faiss_io.cpp). Used to feed the oracle the same index the HIP path
loads, and to cross-check the C++ reader/writer."""
import struct

import numpy as np


class HnswPqFile:
    pass


class _R:
    def __init__(self, b):
        self.b, self.p = b, 0

    def take(self, n):
        if self.p + n > len(self.b):
            raise ValueError("truncated faiss index")
        v = self.b[self.p:self.p + n]
        self.p += n
        return v

    def one(self, fmt):
        n = struct.calcsize(fmt)
        return struct.unpack("<" + fmt, self.take(n))[0]

    def vec(self, dtype):
        n = self.one("Q")
        dt = np.dtype(dtype)
        return np.frombuffer(self.take(n * dt.itemsize), dtype=dt).copy()

    def header(self):
        h = {"d": self.one("i"), "ntotal": self.one("q")}
        self.one("q")
        self.one("q")
        h["is_trained"] = self.one("B")
        h["metric_type"] = self.one("i")
        if h["metric_type"] > 1:
            h["metric_arg"] = self.one("f")
        return h


def read(path):
    with open(path, "rb") as f:
        r = _R(f.read())
    fx = HnswPqFile()
    if r.take(4) != b"IHNp":
        raise ValueError("not an IndexHNSWPQ (fourcc IHNp) file")
    h = r.header()
    fx.d, fx.ntotal, fx.metric_type = h["d"], h["ntotal"], h["metric_type"]
    fx.assign_probas = r.vec("<f8")
    fx.cum_nneighbor_per_level = r.vec("<i4")
    fx.levels = r.vec("<i4")
    fx.offsets = r.vec("<u8")
    fx.neighbors = r.vec("<i4")
    fx.entry_point = r.one("i")
    fx.max_level = r.one("i")
    fx.efConstruction = r.one("i")
    fx.efSearch = r.one("i")
    fx.upper_beam = r.one("i")
    if r.take(4) != b"IxPq":
        raise ValueError("storage is not IndexPQ (IxPq)")
    r.header()
    fx.pq_d = r.one("Q")
    fx.pq_M = r.one("Q")
    fx.pq_nbits = r.one("Q")
    fx.centroids = r.vec("<f4")
    fx.codes = r.vec("<u1")
    fx.search_type = r.one("i")
    fx.encode_signs = r.one("B")
    fx.polysemous_ht = r.one("i")
    if r.p != len(r.b):
        raise ValueError("trailing bytes")
    return fx
