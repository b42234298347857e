"""TEST INFRASTRUCTURE ONLY: numpy reader of hnswlib's saveIndex file format (upstream hnswlib
HierarchicalNSW::saveIndex/loadIndex, unvendored in the reference -- its call sites are
src/hnswlib_dir/index.cpp:47 (saveIndex) and src/hnswlib_dir/test_search.cpp:33 (load)).

Layout (little-endian): size_t offsetLevel0, max_elements, cur_element_count, size_data_per_element,
label_offset, offsetData; int maxlevel; uint32 enterpoint_node; size_t maxM, maxM0, M; double mult;
size_t ef_construction; then cur_element_count level-0 records of size_data_per_element bytes
[u32 count (low 16 bits) + maxM0 u32 links | d f32 | u64 label]; then per element a u32 byte size
of its upper-level blocks followed by those blocks, each [u32 count + maxM u32 links]."""
import numpy as np


def read(path):
    raw = np.fromfile(path, dtype=np.uint8)
    pos = 0

    def take(fmt, count=1):
        nonlocal pos
        dt = np.dtype(fmt)
        v = raw[pos:pos + dt.itemsize * count].view(dt)
        pos += dt.itemsize * count
        return v if count > 1 else v[0]

    off_l0, max_el, n, sz_el, label_off, off_data = (int(take("<u8")) for _ in range(6))
    maxlevel = int(take("<i4"))
    ep = int(take("<u4"))
    maxM, maxM0, M = (int(take("<u8")) for _ in range(3))
    mult = float(take("<f8"))
    efc = int(take("<u8"))
    d = (label_off - off_data) // 4
    assert off_l0 == 0 and off_data == 4 * (1 + maxM0) and sz_el == label_off + 8, "unexpected hnswlib layout"
    rec = raw[pos:pos + n * sz_el].reshape(n, sz_el)
    pos += n * sz_el
    l0 = np.ascontiguousarray(rec[:, :off_data]).view("<u4").reshape(n, 1 + maxM0)
    vec = np.ascontiguousarray(rec[:, off_data:label_off]).view("<f4").reshape(n, d)
    labels = np.ascontiguousarray(rec[:, label_off:label_off + 8]).view("<u8").reshape(n)
    blk = 1 + maxM
    up_off = np.full(n, -1, dtype=np.int64)
    levels = np.zeros(n, dtype=np.int32)
    chunks, total = [], 0
    for i in range(n):
        size = int(raw[pos:pos + 4].view("<u4")[0])
        pos += 4
        if size:
            words = raw[pos:pos + size].view("<u4")
            pos += size
            up_off[i] = total
            levels[i] = size // (4 * blk)
            chunks.append(words)
            total += words.size
    up = np.concatenate(chunks) if chunks else np.zeros(1, dtype=np.uint32)
    assert pos == raw.size, "trailing bytes in hnswlib file"
    return {"d": d, "n": n, "maxM0": maxM0, "maxM": maxM, "M": M, "maxlevel": maxlevel, "ep": ep,
            "mult": mult, "efc": efc, "vec": vec, "l0": np.ascontiguousarray(l0), "labels": labels,
            "up_off": up_off, "up": np.ascontiguousarray(up, dtype=np.uint32), "levels": levels,
            "max_elements": max_el}
