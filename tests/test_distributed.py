"""CPU tests of the N>1 path: gloo, world_size 2. Each rank searches + reranks its contiguous query
shard with the oracle (same code path structure as bench/pipeline), results are gathered to rank 0
and must be byte-identical to the single-process run."""
import os
import socket

import numpy as np
import pytest

from conftest import ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, index_path, q, refs, reads, out_path):
    import sys
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    from deepreadmapper_amd.shard import gather_rows, shard_range
    from deepreadmapper_amd.rerank import pack_queries
    from oracle import faiss_file, oracle as O
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = shard_range(len(q), rank, world)
    fx = faiss_file.read(index_path)
    D, I, nd, nh = O.hnswpq_search(fx, q[lo:hi], 32, 64, nthreads=1)
    qbuf, ql = pack_queries(reads[lo:hi])
    rc, sc, ids, cnt = O.post_process_sw_static(I, refs, 150, qbuf, ql, 1, 32, 32, nthreads=1)
    assert rc == 0
    gI = gather_rows(I, len(q), rank, world, dist)
    gD = gather_rows(D, len(q), rank, world, dist)
    gS = gather_rows(sc, len(q), rank, world, dist)
    if rank == 0:
        np.savez(out_path, I=gI, D=gD, S=gS)
    dist.barrier()
    dist.destroy_process_group()


def test_shard_ranges_cover_exactly():
    from deepreadmapper_amd.shard import shard_range
    for n in (0, 1, 7, 150, 100_003):
        for w in (1, 2, 3, 8):
            rs = [shard_range(n, r, w) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(w - 1))


def test_two_rank_gather_equals_single_process(c1, tmp_path):
    import torch.multiprocessing as mp
    from deepreadmapper_amd.rerank import pack_queries
    from oracle import oracle as O
    q, reads = c1["q"], c1["reads"]
    out = str(tmp_path / "g.npz")
    mp.spawn(_worker, args=(2, _free_port(), c1["index"], q, c1["refs"], reads, out), nprocs=2, join=True)
    g = np.load(out)
    D, I, _, _ = O.hnswpq_search(c1["fx"], q, 32, 64, nthreads=1)
    qbuf, ql = pack_queries(reads)
    rc, sc, ids, cnt = O.post_process_sw_static(I, c1["refs"], 150, qbuf, ql, 1, 32, 32, nthreads=1)
    assert np.array_equal(g["I"], I) and np.array_equal(g["D"].view(np.uint32), D.view(np.uint32))
    assert np.array_equal(g["S"], sc)


def _verdict_worker(rank, world, port, mode, out_path):
    """One rank of a gloo job calling bench.gather_verdict with a gather result forced per `mode`."""
    import json
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    import bench
    D = bench.Dist()
    good = {"backend": "RCCL", "ms": 1.0, "rows": 10}
    if rank == 0:
        good["shards_match"] = [True, mode != "mismatch"]
    gather = {"error": "RuntimeError: forced"} if (mode == "error" and rank == 1) else (
        {"skipped": "2 ranks share 1 device(s)"} if mode == "skipped" else good)
    v = bench.gather_verdict(D, gather)
    with open(f"{out_path}.{rank}", "w") as f:
        json.dump(v, f)
    D.close()


@pytest.mark.parametrize("mode,expect", [("ok", True), ("error", False), ("mismatch", False), ("skipped", None)])
def test_bench_gather_verdict_two_ranks(tmp_path, mode, expect):
    """bench.py at N > 1: a gather error on any rank (here rank 1 only) or a shard mismatch fails the job on
    every rank (gather_ok false, non-zero exit); a gather skipped because ranks share a device is not checked."""
    import json
    import torch.multiprocessing as mp
    out = str(tmp_path / "v")
    mp.spawn(_verdict_worker, args=(2, _free_port(), mode, out), nprocs=2, join=True)
    for r in range(2):
        assert json.load(open(f"{out}.{r}")) == expect


def _checksum_worker(rank, world, port, shift, out_path):
    """One rank of a gloo job: its result rows (seeded, distinct per rank) are 'gathered' to rank 0 with rank 1's
    rows placed `shift` rows off their range, then verified as bench.py does (bench.shard_checksums on every rank's
    own checksum against rank 0's checksum of that rank's range of the gathered rows, then bench.gather_verdict)."""
    import json
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    import bench
    from deepreadmapper_amd.device import host_checksum
    from deepreadmapper_amd.shard import shard_range
    D = bench.Dist()
    n_total = 1001
    lo, hi = shard_range(n_total, rank, world)
    rows = {"sw_ids": np.random.default_rng(rank).integers(0, 1 << 40, (hi - lo, 16)).astype(np.uint64),
            "sw_scores": np.random.default_rng(10 + rank).integers(0, 150, (hi - lo, 16)).astype(np.int32)}
    parts = [None] * world
    D.dist.all_gather_object(parts, rows)  # stands in for the RCCL gather: rank 0 assembles the rows
    full = None
    if rank == 0:
        full = {k: np.zeros((n_total, 16), v.dtype) for k, v in rows.items()}
        for r in range(world):
            rl, rh = shard_range(n_total, r, world)
            d0 = rl + (shift if r == 1 else 0)  # where rank r's rows land
            j0, j1 = max(d0, 0), min(d0 + rh - rl, n_total)
            for k in full:
                full[k][j0:j1] = parts[r][k][j0 - d0:j1 - d0]
    local = {k: host_checksum(v) for k, v in rows.items()}
    match = bench.shard_checksums(D, n_total, local, lambda a, b: {k: host_checksum(v[a:b]) for k, v in full.items()})
    gather = {"backend": "gloo stand-in", "rows": n_total}
    if rank == 0:
        gather["shards_match"] = match
    v = bench.gather_verdict(D, gather)
    with open(f"{out_path}.{rank}", "w") as f:
        json.dump({"ok": v, "match": match}, f)
    D.close()


@pytest.mark.parametrize("shift,expect", [(0, True), (1, False), (-1, False)])
def test_bench_gather_checksums_every_rank(tmp_path, shift, expect):
    """bench.py's gather check covers every rank's rows: rank 1's rows one row off their range (a wrong offset in
    the gather) make gather_ok false on every rank, with rank 0's match list naming rank 1."""
    import json
    import torch.multiprocessing as mp
    out = str(tmp_path / "c")
    mp.spawn(_checksum_worker, args=(2, _free_port(), shift, out), nprocs=2, join=True)
    for r in range(2):
        got = json.load(open(f"{out}.{r}"))
        assert got["ok"] == expect
    assert json.load(open(f"{out}.0"))["match"][1] == expect  # (shift -1 also overwrites rank 0's last row)


@pytest.mark.parametrize("shift,expect", [(0, True), (1, False)])
def test_bench_gather_checksums_four_ranks(tmp_path, shift, expect):
    """The same check at world size 4 (uneven shards of 1,001 rows: 250 / 250 / 250 / 251): every rank's slice of the
    gathered rows is checked, and a one-row offset of rank 1's rows fails the job on every rank."""
    import json
    import torch.multiprocessing as mp
    out = str(tmp_path / "c4")
    mp.spawn(_checksum_worker, args=(4, _free_port(), shift, out), nprocs=4, join=True)
    for r in range(4):
        assert json.load(open(f"{out}.{r}"))["ok"] == expect
    match = json.load(open(f"{out}.0"))["match"]
    assert len(match) == 4 and match[1] == expect and match[3] is True


def _replica_worker(rank, world, port, mode, out_path):
    """One rank of a gloo job running bench.load_index with the GPU pieces stood in: two devices, a communicator
    that only records itself, an index class whose file load and RCCL broadcast are tagged (the broadcast fails on
    rank 1 when mode == "fail")."""
    import json
    import sys
    import types
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    import bench
    import deepreadmapper_amd.device as dev_mod
    import deepreadmapper_amd.executor as ex_mod
    import deepreadmapper_amd.search as se_mod
    dev_mod.device_count = lambda: 2
    events = []

    class FakeComm:
        @staticmethod
        def unique_id():
            return b"u" * 128

        def __init__(self, uid, nranks, rank_, device):
            assert uid == b"u" * 128 and nranks == world and rank_ == rank
            self.rank, self.device = rank_, device

        def free(self):
            pass

    class FakeIndex:
        def __init__(self, path, device, how="file"):
            self.how, self.info = how, types.SimpleNamespace(device_bytes=123)
            events.append(how)

        @classmethod
        def broadcast(cls, comm, index, root=0, copy=False):
            assert (index is not None) == (comm.rank == root)
            if mode == "fail" and comm.rank == 1:
                raise RuntimeError("forced")
            return index if comm.rank == root else cls(None, comm.device, how="bcast")

        def free(self):
            events.append("free")

    ex_mod.Comm, se_mod.HnswPqIndex = FakeComm, FakeIndex
    D = bench.Dist()
    args = types.SimpleNamespace(index_bcast=mode != "off")
    ix, info = bench.load_index(args, D, "x.index", rank)
    with open(f"{out_path}.{rank}", "w") as f:
        json.dump({"mode": info["mode"], "why": info.get("why"), "how": ix.how, "events": events}, f)
    D.close()


@pytest.mark.parametrize("mode", ["ok", "fail", "off"])
def test_bench_index_replication_two_ranks(tmp_path, mode):
    """bench.py at N > 1: rank 0 loads the index file and the others receive it by drm_index_broadcast; a broadcast
    failing on any rank (here rank 1 only) sends every rank back to loading the file itself, and the JSON line says
    so; --no-index-bcast loads the file on every rank."""
    import json
    import torch.multiprocessing as mp
    out = str(tmp_path / "r")
    mp.spawn(_replica_worker, args=(2, _free_port(), mode, out), nprocs=2, join=True)
    got = [json.load(open(f"{out}.{r}")) for r in range(2)]
    if mode == "ok":
        assert [g["mode"] for g in got] == ["rccl broadcast (drm_index_broadcast)"] * 2
        assert got[0]["events"] == ["file"] and got[1]["events"] == ["bcast"]
        assert got[0]["how"] == "file" and got[1]["how"] == "bcast"
    else:
        assert all(g["mode"] == "file per rank" and g["how"] == "file" for g in got)
        assert got[0]["why"] == ("broadcast failed" if mode == "fail" else "--no-index-bcast")
        if mode == "fail":  # rank 0 dropped its loaded replica and loaded again with everyone
            assert got[0]["events"] == ["file", "free", "file"] and got[1]["events"] == ["file"]


def test_host_checksum_properties():
    """drm_device_checksum's host form: position-dependent (swapped words, a shifted row, a changed byte in the
    zero-padded tail all change it), and the empty buffer sums to 0."""
    from deepreadmapper_amd.device import host_checksum
    a = np.random.default_rng(3).integers(0, 1 << 62, 1000).astype(np.int64)
    b = a.copy()
    b[[10, 11]] = b[[11, 10]]
    assert host_checksum(a) != host_checksum(b)
    assert host_checksum(a[1:]) != host_checksum(a[:-1])
    t = np.arange(13, dtype=np.uint8)
    t2 = t.copy()
    t2[12] ^= 1
    assert host_checksum(t) != host_checksum(t2)
    assert host_checksum(np.zeros(0, np.uint8)) == 0
