"""The counter-based synthetic generator: the
library's host side (lengths, tables) against the numpy restatement in
synth.py — no GPU needed.  The device fill is checked in
tests/test_gpu_synth.py."""
import numpy as np


def test_tables_match_synth_py(sw):
    L, lut = sw.capi.synth_tables()
    assert np.array_equal(lut, sw.synth._lut())
    assert L.min() >= 5 and L.max() <= 35213
    assert 250 <= np.median(L) <= 330 and 320 <= L.mean() <= 400  # median 290, mean ~360
    assert np.all(np.diff(L) >= 0)  # quantiles


def test_lengths_match_restatement(sw):
    L, _ = sw.capi.synth_tables()
    for seed, base in [(1782, 0), (1782, 6_250_000), (7, 123)]:
        lib = sw.capi.synth_lengths(seed, base, 5000)
        cpu = sw.synth.counter_lengths(seed, np.arange(base, base + 5000), L)
        assert np.array_equal(lib, cpu)


def test_hash_known_values(sw):
    # splitmix64 with state 0 returns mix(0x9E3779B97F4A7C15) first: the
    # algorithm's published first output
    assert int(sw.synth._mix(np.uint64(0x9E3779B97F4A7C15))) == 0xE220A8397B1DCDAF
    assert int(sw.synth._mix(np.uint64(0))) == 0
