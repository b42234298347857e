"""CPU tests of the boundary: the C-ABI library loads and exports every symbol include/drm_hip.h
declares; host-only entry points (index build, embedder, argument validation) work without a GPU."""
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import ROOT


def _declared():
    src = open(os.path.join(ROOT, "include", "drm_hip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(drm_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    from deepreadmapper_amd import _native
    lib = _native.lib()
    declared = _declared()
    assert len(declared) >= 25
    for name in declared:
        assert hasattr(lib, name), name
    assert sorted(_native.EXPORTS) == declared


def test_nm_exports_are_plain_c():
    out = subprocess.run(["nm", "-D", "--defined-only", os.path.join(ROOT, "deepreadmapper_amd", "libdrm_hip.so")],
                         capture_output=True, text=True, check=True).stdout
    syms = {l.split()[-1] for l in out.splitlines() if l.strip()}
    for name in _declared():
        assert name in syms, name  # unmangled extern "C"


def test_embedder_deterministic_and_normalised():
    from deepreadmapper_amd import synth
    a = synth.embed([b"<ACGTACGTAC>", b"NNNN", b"ACGTTGCA"])
    b = synth.embed([b"ACGTACGTAC", b"NNNN", b"ACGTTGCA"])
    assert np.array_equal(a, b)  # tags are not ACGT 3-mers
    assert abs(np.linalg.norm(a[0]) - 1) < 1e-5 and not a[1].any()


def test_build_and_reader_roundtrip(tmp_path):
    from deepreadmapper_amd import synth
    from oracle import faiss_file
    rng = np.random.default_rng(1)
    x = rng.standard_normal((600, 32)).astype(np.float32)
    p1, p2 = str(tmp_path / "a.index"), str(tmp_path / "b.index")
    synth.build_index(x, p1, M_pq=4, nbits=8, M_hnsw=8, efc=40, nthreads=1, seed=3)
    synth.build_index(x, p2, M_pq=4, nbits=8, M_hnsw=8, efc=40, nthreads=1, seed=3)
    assert open(p1, "rb").read() == open(p2, "rb").read()  # single-threaded build is deterministic
    fx = faiss_file.read(p1)
    assert fx.d == 32 and fx.ntotal == 600 and fx.pq_M == 4 and fx.pq_nbits == 8
    assert len(fx.offsets) == 601 and fx.offsets[-1] == len(fx.neighbors)
    assert fx.cum_nneighbor_per_level[1] == 16 and fx.codes.size == 600 * 4
    assert fx.levels[fx.entry_point] == fx.max_level + 1
    assert ((fx.neighbors >= -1) & (fx.neighbors < 600)).all()


def test_build_rejects_bad_args(tmp_path):
    from deepreadmapper_amd import synth, DrmError
    with pytest.raises(DrmError):
        synth.build_index(np.zeros((10, 30), np.float32), str(tmp_path / "x.index"), M_pq=8)


def test_index_load_rejects_non_hnswpq(tmp_path):
    from deepreadmapper_amd import read_index, DrmError
    from deepreadmapper_amd._native import DRM_ERR_FORMAT, DRM_ERR_IO
    bad = tmp_path / "bad.index"
    bad.write_bytes(b"IHNf" + b"\0" * 64)
    with pytest.raises(DrmError) as e:
        read_index(str(bad))
    assert e.value.code == DRM_ERR_FORMAT and "IHNf" in str(e.value)
    with pytest.raises(DrmError) as e:
        read_index(str(tmp_path / "missing.index"))
    assert e.value.code == DRM_ERR_IO


def test_index_load_rejects_truncated(tmp_path, c1):
    from deepreadmapper_amd import read_index, DrmError
    from deepreadmapper_amd._native import DRM_ERR_FORMAT
    data = open(c1["index"], "rb").read()
    t = tmp_path / "trunc.index"
    t.write_bytes(data[: len(data) // 2])
    with pytest.raises(DrmError) as e:
        read_index(str(t))
    assert e.value.code == DRM_ERR_FORMAT and "truncated" in str(e.value)


def test_hnswpq_index_cli(tmp_path):
    """bin/hnswpq_index mirrors src/hnswpq/index.cpp:195-316: config.txt keys + prefix/prefix.index."""
    exe = os.path.join(ROOT, "bin", "hnswpq_index")
    fna = os.path.join(ROOT, "tests", "golden", "ecoli_150.fna")
    env = dict(os.environ, DRM_BUILD_THREADS="1")
    r = subprocess.run([exe, fna, "c1idx", "150"], cwd=tmp_path, capture_output=True, text=True, env=env)
    assert r.returncode == 0, r.stderr
    cfg = dict(l.split(": ", 1) for l in (tmp_path / "c1idx" / "config.txt").read_text().splitlines())
    assert cfg == {"index_type": "HNSWPQ", "stride": "1", "ref_len": "150", "n_vects": "1702", "dim": "128",
                   "M_hnsw": "16", "EFC": "200", "M_pq": "8", "nbits": "8", "index_file": "c1idx/c1idx.index"}
    from oracle import faiss_file
    fx = faiss_file.read(str(tmp_path / "c1idx" / "c1idx.index"))
    assert fx.ntotal == 1702
    r = subprocess.run([exe, fna], capture_output=True, text=True)
    assert r.returncode == 1 and "Usage" in r.stderr


def test_index_load_rejects_upper_link_to_lower_node(tmp_path, c1):
    """A level-l link must target a node that reaches level l (faiss IHNp): the kernel would read
    the target's level-l list, which does not exist. Rejected as DRM_ERR_FORMAT before any GPU use."""
    from deepreadmapper_amd import read_index, DrmError
    from deepreadmapper_amd._native import DRM_ERR_FORMAT
    fx = c1["fx"]
    lv, cum, offs = fx.levels, fx.cum_nneighbor_per_level, fx.offsets
    pos = 4 + 33 + (8 + 8 * len(fx.assign_probas)) + (8 + 4 * len(cum)) + (8 + 4 * len(lv)) + (8 + 8 * len(offs)) + 8
    src = int(np.flatnonzero(lv >= 2)[0])
    low = int(np.flatnonzero(lv == 1)[0])
    slot = int(offs[src]) + int(cum[1])  # first level-1 link of src
    data = bytearray(open(c1["index"], "rb").read())
    data[pos + 4 * slot: pos + 4 * slot + 4] = np.int32(low).tobytes()
    bad = tmp_path / "uplink.index"
    bad.write_bytes(bytes(data))
    with pytest.raises(DrmError) as e:
        read_index(str(bad))
    assert e.value.code == DRM_ERR_FORMAT and "does not reach" in str(e.value)


def test_flat_index_load_rejects_upper_link_to_lower_node(tmp_path):
    """Same check on the hnswlib reader (an upper link to a level-0 element)."""
    from deepreadmapper_amd import synth, DrmError
    from deepreadmapper_amd.flat import HnswFlatIndex
    from deepreadmapper_amd._native import DRM_ERR_FORMAT
    from oracle import hnswlib_file
    rng = np.random.default_rng(0)
    x = rng.standard_normal((3000, 16)).astype(np.float32)
    path = str(tmp_path / "f.hnsw")
    synth.build_flat_index(x, path, M=8, efc=32, nthreads=1)
    fx = hnswlib_file.read(path)
    n, maxM0, maxM, d = fx["n"], fx["maxM0"], fx["maxM"], fx["d"]
    sz_el = 4 * (1 + maxM0) + 4 * d + 8
    pos = 96 + n * sz_el
    low = int(np.flatnonzero(fx["levels"] == 0)[0])
    data = bytearray(open(path, "rb").read())
    for i in range(n):
        size = int(np.frombuffer(data[pos:pos + 4], np.uint32)[0])
        pos += 4
        if size and int(np.frombuffer(data[pos:pos + 4], np.uint32)[0]) & 0xFFFF:
            data[pos + 4:pos + 8] = np.uint32(low).tobytes()  # first level-1 link
            break
        pos += size
    bad = tmp_path / "bad.hnsw"
    bad.write_bytes(bytes(data))
    with pytest.raises(DrmError) as e:
        HnswFlatIndex(str(bad))
    assert e.value.code == DRM_ERR_FORMAT and "does not reach" in str(e.value)


def test_pipeline_rejects_ragged_reference(tmp_path):
    """a .txt reference with a line shorter than ref_len is refused with a format
    error before the GPU is touched (the fixed-width window table would over-read it)."""
    exe = os.path.join(ROOT, "bin", "pipeline")
    prefix = tmp_path / "idx"
    prefix.mkdir()
    (prefix / "config.txt").write_text("ref_len: 150\nstride: 1\n")
    (prefix / "idx.index").write_bytes(b"")
    ref = tmp_path / "ref.txt"
    ref.write_text("A" * 150 + "\n" + "C" * 149 + "\n")
    q = tmp_path / "q.txt"
    q.write_text("A" * 150 + "\n")
    r = subprocess.run([exe, str(prefix), str(q), str(ref)], capture_output=True, text=True)
    assert r.returncode == 1 and "reference sequence 1 has 149 bytes" in r.stderr
