"""The seen-set spill's cold-run search on the host (kc_cold_find_selftest:
the same run_find every GPU lookup of a spilled fingerprint runs, compiled
for the host): found iff present, through whole runs and staging windows,
for run sizes around the directory's bucket and line boundaries.  The GPU
tests (test_gpu_seenspill.py) cover the kernels around it."""
import pytest

from kubecheck import load


@pytest.mark.parametrize("n", [1, 7, 8, 9, 31, 32, 33, 100, 1000, 4096, 100_003, 1 << 20])
def test_cold_run_search(n):
    for seed in (1, 2, 3):
        assert load().kc_cold_find_selftest(n, seed) == 0
