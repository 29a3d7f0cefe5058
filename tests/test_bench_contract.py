"""CPU tests of bench.py's contract pieces that need no GPU: the algorithmic
bytes per expansion, the CPU-baseline leg's schema and its
exact-score gate, and the workload table against the golden fixtures."""
import os
import subprocess
import sys

import pytest

from conftest import ROOT, golden

sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_bytes_per_expansion_matches_survey():
    # 321 / 720 / 1551 / 14764 B for N = 3, 4, 5, 8
    assert [bench.bytes_per_expansion(n) for n in (3, 4, 5, 8)] == [321, 720, 1551, 14764]


def test_workloads_point_at_fixtures(kat):
    for name, (fasta, cfg, known) in bench.WORKLOADS.items():
        assert os.path.exists(golden(fasta)), fasta
        assert cfg
        if name in kat["inputs"]:
            assert kat["inputs"][name]["score"] == known


def test_cpu_baseline_schema():
    line = bench.cpu_baseline(golden("test2.fasta"), 0.2, 45037)
    assert line["unit"] == "nodes/s" and line["kind"] == "port" and line["value"] > 0
    assert line["score"] == 45037 and line["cores"] >= 1
    runs = line["runs"]
    assert "t1" in runs and len(runs) == 2
    assert runs["t1"]["cores"] == 1
    # the baseline is the leg that reaches the optimum sooner, not the one with more nodes/s
    assert line["wall_to_optimal_s"] == min(r["wall_to_optimal_s"] for r in runs.values())
    assert line["chosen_by"] == "wall_to_optimal_s"


def test_sharded_shift_choice():
    assert bench.sharded_shift(5, 1) == 12 and bench.sharded_shift(8, 1) == 12
    assert bench.sharded_shift(4, 8) == 18 and bench.sharded_shift(5, 2) == 18 and bench.sharded_shift(8, 8) == 12


def test_cpu_baseline_rejects_a_wrong_score():
    with pytest.raises(RuntimeError):
        bench.cpu_baseline(golden("test2.fasta"), 0.05, 45036)


def test_bench_help_runs_without_gpu():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--help"], capture_output=True, text=True,
                       timeout=60)
    assert r.returncode == 0 and "--workload" in r.stdout
