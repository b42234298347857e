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
        good["rank0_shard_matches"] = mode != "mismatch"
    gather = {"error": "RuntimeError: forced"} if (mode == "error" and rank == 1) else (
        {"skipped": "2 ranks share 1 device(s)"} if mode == "skipped" else good)
    v = bench.gather_verdict(D, gather)
    with open(f"{out_path}.{rank}", "w") as f:
        json.dump(v, f)
    D.close()


@pytest.mark.parametrize("mode,expect", [("ok", True), ("error", False), ("mismatch", False), ("skipped", None)])
def test_bench_gather_verdict_two_ranks(tmp_path, mode, expect):
    """bench.py at N > 1: a gather error on any rank (here rank 1 only) or a rank-0 shard mismatch fails the job on
    every rank (gather_ok false, non-zero exit); a gather skipped because ranks share a device is not checked."""
    import json
    import torch.multiprocessing as mp
    out = str(tmp_path / "v")
    mp.spawn(_verdict_worker, args=(2, _free_port(), mode, out), nprocs=2, join=True)
    for r in range(2):
        assert json.load(open(f"{out}.{r}")) == expect
