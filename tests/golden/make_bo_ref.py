#!/usr/bin/env python3
"""Extract the reference's recorded BO gap curves into tests/golden/bo_ref_gaps.json.

Data only: the per-trial `gaps` rows the reference's experiment drivers wrote (create_csv /
write_to_csv, utils.jl:155-172; gap = (initial_best − observed_best)/(initial_best − f*), utils.jl
`gap`), for the cases tools/bo_compare.py runs against the MI355X BO loop (mrbo/bayesopt.py):

  myopic_<fn>_<rule> experiments/myopic/<fn>/<rule>_gaps.csv (myopic_bayesopt.jl: EI / POI / LCB
                     multistart solve, 64 starts, 5 initial points, budget 100 -- steps 1..30
                     kept --, 60 trials, optimize!)
  rollout_h<h>_<fn>  experiments/archived/nonmyopic-shortrun-gaps-and-time/nonmyopic_bayesopt/
                     <fn>/rollout_h<h>_gaps.csv (an earlier nonmyopic_bayesopt.jl: rollout
                     acquisition, 8 starts, batch 8, 100 MC samples, 50 SGD iterations, budget 20,
                     60 trials, optimize!; header columns 0..20)

Each case keeps the header (the budget labels) and the trial rows (the −1.0 placeholder row of
create_csv dropped), and the same of the matching `times` file (seconds per acquisition solve).  Run here, where /root/reference exists; the JSON travels with the repo.
usage: python tests/golden/make_bo_ref.py [--reference /root/reference]
"""
import argparse
import csv
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))

ARCHIVE = "experiments/archived/nonmyopic-shortrun-gaps-and-time/nonmyopic_bayesopt"
MYOPIC_FNS = ["braninhoo", "hartmann6d", "ackley5d", "goldsteinprice", "sixhump", "griewank3d", "levy10d"]
ROLLOUT_FNS = ["braninhoo", "gramacylee", "ackley1d", "ackley2d", "ackley3d", "ackley4d", "rosenbrock", "hartmann3d",
               "sixhump", "goldsteinprice"]
CASES = {f"myopic_{fn}_{rule}": f"experiments/myopic/{fn}/{rule}_gaps.csv"
         for fn in MYOPIC_FNS for rule in ("ei", "poi", "lcb")}
CASES.update({f"rollout_h{h}_{fn}": f"{ARCHIVE}/{fn}/rollout_h{h}_gaps.csv" for fn in ROLLOUT_FNS for h in (0, 1)})
MYOPIC_LABELS = 30   # the myopic files run to budget 100; the comparison uses steps 1..30


def read_gaps(path):
    rows = list(csv.reader(open(path)))
    header = rows[0][1:]
    trials = []
    for r in rows[1:]:
        v = [float(x) for x in r]
        if all(x == -1.0 for x in v):          # create_csv's placeholder row
            continue
        # rows of the current write_to_csv carry the budget values only; the archived ones a
        # leading trial id, and their times rows the whole preallocated container (zeros after)
        trials.append(v[1:1 + len(header)] if len(v) > len(header) else v)
    return header, trials


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    a = ap.parse_args()
    out = {}
    for key, rel in CASES.items():
        header, trials = read_gaps(os.path.join(a.reference, rel))
        trel = rel.replace("_gaps.csv", "_times.csv")
        theader, times = read_gaps(os.path.join(a.reference, trel))
        if key.startswith("myopic"):   # keep the compared steps only (the fixture travels with the repo)
            header, trials = header[:MYOPIC_LABELS], [r[:MYOPIC_LABELS] for r in trials]
            theader, times = theader[:MYOPIC_LABELS], [r[:MYOPIC_LABELS] for r in times]
        out[key] = {"source": rel, "budget_labels": header, "gaps": trials, "times_source": trel,
                    "times_labels": theader, "times": times}
    with open(os.path.join(HERE, "bo_ref_gaps.json"), "w") as f:
        json.dump(out, f, separators=(",", ":"))
    for k, v in out.items():
        print(k, len(v["gaps"]), "trials x", len(v["budget_labels"]))


if __name__ == "__main__":
    main()
