"""The non-myopic BO loop (mrbo/bayesopt.py): CSV formats of utils.jl:155-172
on the CPU, and a small end-to-end experiment on the GPU.  Parity of BO trajectories with the
reference is unpinned (its rollout solver is undefined and Julia is absent); the GPU test checks
the loop's invariants instead."""
import csv
import os

import numpy as np
import pytest


def test_csv_layout(tmp_path):
    from mrbo.bayesopt import create_csv, write_to_csv
    fn = str(tmp_path / "rollout_1_ei_gaps")
    create_csv(fn, 4)
    write_to_csv(fn, [0.0, 0.25, 0.5, 1.0])
    write_to_csv(fn, np.array([0.1, np.nan, 2.0, -3.5]))
    rows = list(csv.reader(open(fn + ".csv")))
    assert rows[0] == ["trial", "1", "2", "3", "4"]
    assert rows[1] == ["-1.0"] * 5                    # DataFrame(-ones(1, budget+1))
    assert rows[2] == ["0.0", "0.25", "0.5", "1.0"]   # appended rows carry the budget values only
    assert rows[3] == ["0.1", "NaN", "2.0", "-3.5"]


def test_metadata_and_cli(tmp_path):
    from mrbo.bayesopt import parse, write_metadata
    write_metadata(str(tmp_path), 15, 60, 16)
    assert open(tmp_path / "metadata.txt").read() == "Budget: 15\nNumber of Trials: 60\nNumber of Starts: 16\n"
    a = parse(["--output-dir", str(tmp_path), "--function-name", "gramacylee"])
    assert (a.budget, a.trials, a.starts, a.horizon, a.mc_samples, a.batch_size, a.sgd_iterations, a.seed) == \
        (15, 60, 16, 0, 200, 8, 50, 1906)


@pytest.mark.gpu
@pytest.mark.parametrize("horizon,optimize", [(0, False), (1, True)])
def test_bayesopt_end_to_end(gpu, tmp_path, horizon, optimize):
    from mrbo import bayesopt
    res = bayesopt.run("gramacylee", str(tmp_path), budget=3, trials=2, starts=8, horizon=horizon, mc_samples=16,
                       batch_size=4, sgd_iterations=5, optimize=optimize, log=lambda *a: None)
    d = tmp_path / "gramacylee"
    for acq in [f"rollout_{horizon}_ei", f"rollout_{horizon}_poi", f"rollout_{horizon}_lcb"]:
        for metric in bayesopt.METRICS:
            rows = list(csv.reader(open(d / f"{acq}_{metric}.csv")))
            assert len(rows) == 2 + 2 and all(len(r) == 3 for r in rows[2:])
        for trial in range(2):
            r = res[(acq, trial)]
            assert r["y"].size == 5 + 3
            lo, hi = 0.5, 2.5
            assert (r["X"] >= lo).all() and (r["X"] <= hi).all()
            assert np.all(np.diff(r["minimum_observations"]) <= 0)          # running minimum
            assert np.all(r["gaps"] <= 1.0 + 1e-12) and np.all(r["gaps"] >= 0.0)
            assert np.all(r["simple_regret"] >= 0.0)
    assert os.path.exists(d / "metadata.txt")
