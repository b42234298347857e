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
