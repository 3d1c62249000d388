"""bench.py's host-side pieces that need no GPU: the all-cores CPU
baseline's thread choice (cgroup quota, not the oversubscribed affinity set)
and its sweep record."""
import numpy as np

import bench


def test_cpu_thread_counts_follow_the_quota(monkeypatch):
    monkeypatch.setattr(bench, "affinity_cpus", lambda: 256)
    monkeypatch.setattr(bench, "cpu_quota", lambda: 16.0)
    assert bench.cpu_thread_counts() == [16, 32, 256]
    monkeypatch.setattr(bench, "cpu_quota", lambda: None)
    monkeypatch.setenv("OMP_NUM_THREADS", "16")
    assert bench.cpu_thread_counts() == [16, 32, 256]
    monkeypatch.delenv("OMP_NUM_THREADS")
    assert bench.cpu_thread_counts() == [256]
    assert bench.cpu_thread_counts(explicit=7) == [7]
    monkeypatch.setattr(bench, "affinity_cpus", lambda: 8)
    monkeypatch.setattr(bench, "cpu_quota", lambda: 2.5)
    assert bench.cpu_thread_counts() == [2, 4, 8]


def test_cpu_baseline_parallel_reports_the_sweep(lib_built):
    rng = np.random.default_rng(0)
    lengths = np.array([5_000, 3_000, 7_000], np.int64)
    tid = np.repeat(np.arange(3, dtype=np.int32), 400)
    pos = np.concatenate([np.sort(rng.integers(0, L - 100, 400)) for L in lengths]).astype(np.int32)
    span = np.full(len(tid), 100, np.int32)
    r = bench.cpu_baseline_parallel(lengths, tid, pos, span, [1, 2], min_s=0.01)
    assert [x["threads"] for x in r["sweep"]] == [1, 2]
    assert r["cores"] in (1, 2) and r["value"] == max(x["value"] for x in r["sweep"])
    assert "cpu_quota" in r and r["unit"] == "aligned bases/s"
