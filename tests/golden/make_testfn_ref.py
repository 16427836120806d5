#!/usr/bin/env python3
"""Extract (x, f(x)) pairs the reference itself evaluated into tests/golden/testfn_ref.json.

Data only: the archived non-myopic experiments recorded every observation of every trial
(`<acq>_observations.csv` under experiments/archived/…/nonmyopic_bayesopt/<fn>/: per trial, d rows
of coordinates then one row of objective values, each row led by the trial id; an all −1.0
placeholder row after the header).  Those y = testfn.f(x) values were computed by the reference's
testfns.jl, so they pin the build's test functions (mrbo/testfns.py) -- the objectives that
generate the synthetic base data of every BASELINE configuration (Gramacy–Lee C1, Branin C2,
Hartmann-6 C3/C4, Ackley-8 C5) -- and the BO comparison's functions.

For each function: up to PAIRS distinct pairs, taken evenly over the file's trials and steps.
Also writes tests/golden/bo_ref_observations.json: for the archived rollout runs the BO comparison
uses, the first trials' objective values in observation order beside their recorded gap rows.
Run here, where /root/reference exists; the JSON travels with the repo.
usage: python tests/golden/make_testfn_ref.py [--reference /root/reference]
"""
import argparse
import csv
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
SHORT = "experiments/archived/nonmyopic-shortrun-gaps-and-time/nonmyopic_bayesopt"
DIMS = "experiments/archived/dimensions-timing/nonmyopic_bayesopt"
PAIRS = 48

# fixture key -> (relative observation file, input dimension); keys are mrbo.bayesopt.TESTFNS names
# except ackley8d / ackley16d (TestAckley(8), TestAckley(16))
SOURCES = {fn: (f"{SHORT}/{fn}/rollout_h0_observations.csv", d) for fn, d in [
    ("gramacylee", 1), ("braninhoo", 2), ("hartmann6d", 6), ("rosenbrock", 2), ("ackley1d", 1), ("ackley2d", 2),
    ("ackley3d", 3), ("ackley4d", 4), ("rastrigin4d", 4), ("hartmann3d", 3), ("sixhump", 2), ("goldsteinprice", 2)]}
SOURCES["ackley8d"] = (f"{DIMS}/ackley8d/rollout_h0_observations.csv", 8)
SOURCES["ackley16d"] = (f"{DIMS}/ackley16d/rollout_h0_observations.csv", 16)


def read_pairs(path, d):
    rows = [r for r in csv.reader(open(path))][1:]
    rows = [[float(v) for v in r] for r in rows]
    rows = [r for r in rows if not all(v == -1.0 for v in r)]
    pairs = []
    for t in range(0, len(rows) - d, d + 1):
        block = rows[t:t + d + 1]
        xs = [r[1:] for r in block[:d]]
        ys = block[d][1:]
        for j, y in enumerate(ys):
            pairs.append(([x[j] for x in xs], y))
    return pairs


ROLLOUT_FNS = ["braninhoo", "gramacylee", "ackley1d", "ackley2d", "ackley3d", "ackley4d", "rosenbrock", "hartmann3d",
               "sixhump", "goldsteinprice"]
OBS_TRIALS = 10


def read_rows(path):
    rows = [[float(v) for v in r] for r in list(csv.reader(open(path)))[1:]]
    return [r for r in rows if not all(v == -1.0 for v in r)]


def bo_observations(ref, fn, h, d):
    """The first OBS_TRIALS trials of an archived rollout run: the objective values in observation
    order (the initial point, then the 20 BO steps) and the trial's recorded gap row (labels 0..20)."""
    obs = read_rows(os.path.join(ref, f"{SHORT}/{fn}/rollout_h{h}_observations.csv"))
    gaps = read_rows(os.path.join(ref, f"{SHORT}/{fn}/rollout_h{h}_gaps.csv"))
    out = []
    for t in range(OBS_TRIALS):
        y = obs[t * (d + 1) + d]
        g = gaps[t]
        assert y[0] == g[0]                    # rows led by the same trial id (failed trials are absent)
        out.append({"trial": int(y[0]), "y": y[1:], "gaps": g[1:]})
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    a = ap.parse_args()
    out = {}
    for key, (rel, d) in SOURCES.items():
        allp = read_pairs(os.path.join(a.reference, rel), d)
        seen, keep = set(), []
        stride = max(1, len(allp) // PAIRS)
        for x, y in allp[::stride]:
            k = tuple(x)
            if k in seen:
                continue
            seen.add(k)
            keep.append({"x": x, "y": y})
            if len(keep) == PAIRS:
                break
        out[key] = {"source": rel, "d": d, "pairs_in_file": len(allp), "pairs": keep}
    path = os.path.join(HERE, "testfn_ref.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=0)
    print(path, {k: len(v["pairs"]) for k, v in out.items()})
    # the archived runs' observation values beside their recorded gaps (utils.jl `gap`)
    bo = {f"rollout_h{h}_{fn}": {"source": f"{SHORT}/{fn}/rollout_h{h}_{{observations,gaps}}.csv",
                                 "trials": bo_observations(a.reference, fn, h, SOURCES[fn][1])}
          for fn in ROLLOUT_FNS for h in (0, 1)}
    path = os.path.join(HERE, "bo_ref_observations.json")
    with open(path, "w") as f:
        json.dump(bo, f, indent=0)
    print(path, len(bo))


if __name__ == "__main__":
    main()
