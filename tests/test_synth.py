"""Synthetic workload generators: the blockwise read stream used for C5 shards."""
import numpy as np

from deepreadmapper_amd import synth


def test_read_stream_shards_are_independent_of_the_split():
    g = synth.genome(40_000, seed=3)
    whole, t_whole = synth.simulate_reads_range(g, 0, 5000, seed=9, block=1024)
    parts = [synth.simulate_reads_range(g, lo, hi, seed=9, block=1024) for lo, hi in
             ((0, 1), (1, 1023), (1023, 1025), (1025, 4096), (4096, 5000))]
    assert np.array_equal(np.concatenate([p[0] for p in parts]), whole)
    assert np.array_equal(np.concatenate([p[1] for p in parts]), t_whole)
    r, t = synth.simulate_reads_range(g, 7, 7, seed=9)
    assert r.shape == (0, 150) and t.shape == (0,)


def test_read_stream_truth_and_substitution_rate():
    g = synth.genome(40_000, seed=3)
    reads, truth = synth.simulate_reads_range(g, 0, 3000, seed=9, block=1024)
    refs = synth.windows_lookup(g, 150, 1)
    assert set(np.unique(reads).tolist()) <= set(b"ACGT")
    mism = (refs[truth] != reads).mean()
    assert 0.005 < mism < 0.015  # 1 % substitutions against the source window (fwd or RC)
