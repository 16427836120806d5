#!/usr/bin/env python3
"""Statistical comparison of the MI355X BO loop (mrbo/bayesopt.py) with the reference's recorded
BO runs (parity of BO trajectories is unpinned -- Julia's RNG, Optim.jl and the
reference's undefined rollout solver cannot be reproduced -- so the evidence is distributional).

For every case of tests/golden/bo_ref_gaps.json (extracted by tests/golden/make_bo_ref.py from
the reference's experiment CSVs) this runs the loop on the GPU with the reference's recorded
settings and compares the per-trial `gaps` (utils.jl `gap`, recorded before conditioning, as
nonmyopic_bayesopt.jl:273-281) at the compared budget labels: means with standard errors, the
two-sided Mann–Whitney U and Kolmogorov–Smirnov p-values, and the seconds per acquisition solve
beside the reference's recorded ones (earlier code versions on unstated hardware).

  myopic_<fn>_ei     vs. the myopic loop (bayesopt.run_myopic): multistart_base_solve! of the
                     analytic EI from generate_initial_guesses(64) on the base surrogate, the
                     reference's solver shape (experiments/myopic_bayesopt.jl:224-233) with the
                     build's projected Newton in place of IPNewton
  rollout_h<h>_<fn>  vs. the rollout acquisition at horizon h, the archived run's settings
                     (1 initial point, 8 starts, batch 8, 100 MC samples, 50 SGD iterations)

usage: python tools/bo_compare.py [--trials 20] [--cases a,b] [--out gpurun_out/bo_compare.jsonl]
One JSON line per case (stdout and --out); progress on stderr.
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "rollout-bayesian-optimization_amd"), ROOT]

FIXTURE = os.path.join(ROOT, "tests", "golden", "bo_ref_gaps.json")

# per case: our run() settings and the budget labels compared (the reference's column labels)
MYOPIC_FNS = ["braninhoo", "hartmann6d", "ackley5d", "goldsteinprice", "sixhump", "griewank3d", "levy10d"]
ROLLOUT_FNS = ["braninhoo", "gramacylee", "ackley1d", "ackley2d", "ackley3d", "ackley4d", "rosenbrock", "hartmann3d",
               "sixhump", "goldsteinprice"]
# myopic: the reference ran budget 100 with one surrogate of capacity 100 reused over the trials
# (myopic_bayesopt.jl:205-217); each trial starts from the lengthscale the previous trial's 100th
# optimize! left, so the loop runs the same 100 steps (run_budget) and compares the first 30 labels
SETTINGS = {f"myopic_{fn}_{rule}": dict(fn=fn, rule=rule, horizon=0, budget=30, run_budget=100, capacity=100, initial=5,
                                        starts=64, batch=0, labels=["10", "20", "30"])
            for fn in MYOPIC_FNS for rule in ("ei", "poi", "lcb")}
SETTINGS.update({f"rollout_h{h}_{fn}": dict(fn=fn, rule="ei", horizon=h, budget=20, initial=1, starts=8, batch=8,
                                            labels=["5", "10", "20"])
                 for fn in ROLLOUT_FNS for h in (0, 1)})
# The cases with a MEASURED deficit against the reference's recorded runs, each
# with what is known of its cause.  The GPU test (tests/test_bayesopt.py) asserts every other case.
EXCEPTIONS = {
    "myopic_sixhump_poi": "UNEXPLAINED: ours closes less (-0.08 at 30, 3 of 4 seeds); not the faces (3 % of "
                          "observations, solve margins leave it), not repeats (no-repeat pick leaves it); what "
                          "remains is which interior KKT point of POI the solver returns or the MLE lengthscale "
                          "path -- IPNewton / Optim.jl, absent here (profiles/r05/bo_myopic/)",
    "myopic_sixhump_lcb": "borderline: one-sided p = 0.04 at 60 trials, no two-sided difference "
                          "(profiles/r04/bo_compare_myopic_all_reuse_60trials_r4e.jsonl); same solver question as POI",
    "myopic_hartmann6d_poi": "the faces: projected Newton stops on a face where IPNewton's barrier keeps its iterate "
                             "inside; the deficit shrinks with the solve margin (-0.091 -> -0.085 -> -0.034 at "
                             "margins 0, 0.01, 0.05; profiles/r05/bo_myopic/)",
    "rollout_h0_rosenbrock": "EI underflow regime: |fmini - mu| >> sigma on the whole batch of Rosenbrock's "
                             "10^2-10^3 scale, EI = 0 and zero gradients; 90 % of trials repeat a point "
                             "(DESIGN.md §10; profiles/r03/bo_trace/)",
}
# the cases the GPU test asserts: every recorded case without a measured deficit
ASSERTED = [k for k in SETTINGS if k not in EXCEPTIONS]


def load_reference(path=FIXTURE):
    with open(path) as f:
        return json.load(f)


def our_gap_columns(res, true_minimum, budget):
    """Per-trial gaps at labels 0..budget: label k = after k BO observations, i.e. run()'s
    gaps[k] (recorded before conditioning at step k+1) for k < budget, and the gap of the final
    minimum observation for k = budget.  Returns (trials, budget+1)."""
    rows = []
    for r in res:
        g = list(r["gaps"])
        ib = r["initial_best"]
        g.append((ib - r["minimum_observations"][-1]) / (ib - true_minimum))
        rows.append(g)
    return np.array(rows)


def ref_column(case, label):
    """Reference gaps at a budget label, with the label convention of its file: the myopic files
    label budget steps 1..B (gap before conditioning at step b = after b-1 observations); the
    archived rollout files label 0..B (after k observations)."""
    labels = case["budget_labels"]
    return np.array([row[labels.index(label)] for row in case["gaps"]])


def our_column(gcols, label, myopic):
    k = int(label) - 1 if myopic else int(label)
    return gcols[:, k]


def compare(a, b):
    """ours (a) vs reference (b): means, standard errors, the difference of means with its Welch 95 %
    confidence interval, Mann–Whitney U and KS p-values.  A large p-value means no significant
    difference was DETECTED at these sample sizes -- not equivalence; the interval says how large a
    difference the data still allow."""
    from scipy.stats import ks_2samp, mannwhitneyu, t as student_t
    a, b = np.asarray(a, float), np.asarray(b, float)
    se = lambda x: float(x.std(ddof=1) / np.sqrt(x.size)) if x.size > 1 else float("nan")
    out = {"ours_mean": float(a.mean()), "ours_se": se(a), "ref_mean": float(b.mean()), "ref_se": se(b),
           "n_ours": int(a.size), "n_ref": int(b.size)}
    va, vb = a.var(ddof=1) / a.size, b.var(ddof=1) / b.size
    diff, sd = float(a.mean() - b.mean()), float(np.sqrt(va + vb))
    dof = (va + vb) ** 2 / (va ** 2 / (a.size - 1) + vb ** 2 / (b.size - 1)) if va + vb > 0 else 1.0
    half = float(student_t.ppf(0.975, dof) * sd)
    out["diff_mean"], out["diff_ci95"] = diff, [diff - half, diff + half]
    out["mannwhitney_p"] = float(mannwhitneyu(a, b, alternative="two-sided").pvalue)
    # one-sided: evidence that ours is stochastically SMALLER (gaps: worse) than the reference's
    out["mannwhitney_p_worse"] = float(mannwhitneyu(a, b, alternative="less").pvalue)
    out["ks_p"] = float(ks_2samp(a, b).pvalue)
    return out


def detected(cmp, alpha=0.05):
    """Two-sided verdict beside the one-sided assertion: 'none' when the two-sided Mann–Whitney test
    finds no difference at level alpha, else which side closes more of the gap."""
    if not cmp["mannwhitney_p"] < alpha:
        return "none"
    return "ours closes more" if cmp["diff_mean"] > 0 else "ours closes less"


def trajectory_diagnostics(Xs, lbs, ubs, initial):
    """Shape of the BO observation sequences (same statistics as for the reference's archived
    observation CSVs in DESIGN.md §10): the fraction of BO observations with a coordinate on the box
    boundary, the fraction of trials whose first BO step is on it, and the fraction of trials that
    observed one point twice (a wasted evaluation)."""
    lb, ub = np.asarray(lbs, float)[:, None], np.asarray(ubs, float)[:, None]
    atb, first, rep = [], [], []
    for X in Xs:
        x = np.asarray(X, float)[:, initial:]
        b = (np.isclose(x, lb, atol=1e-6) | np.isclose(x, ub, atol=1e-6)).any(0)
        atb.append(b.mean())
        first.append(bool(b[0]))
        dd = np.linalg.norm(x[:, :, None] - x[:, None, :], axis=0)
        np.fill_diagonal(dd, 1.0)
        rep.append(bool((dd < 1e-6).any()))
    return {"obs_at_boundary": float(np.mean(atb)), "first_step_at_boundary": float(np.mean(first)),
            "trials_with_repeats": float(np.mean(rep))}


def run_case(key, case, trials, seed, log, solver="sga", eta=0.01, q3=True, incumbent=True, reuse=None,
             run_budget=None, solve_margin=0.0, no_repeat=False):
    """One comparison case.  run_budget (myopic cases) overrides the steps each trial runs (default
    the reference's 100, whose last optimize! sets the next trial's starting lengthscale).
    reuse=None takes the surrogate semantics of the driver that produced the case's records: the
    myopic records come from experiments/myopic_bayesopt.jl, which reuses ONE surrogate over the
    trials (:205-217, the lengthscale carries over); the archived rollout records come from the
    earlier driver experiments/adaptive_bayesopt.jl, which fits a fresh surrogate per trial
    (`sur = fit_surrogate(ψ, Xinit, yinit)`, :498, ψ defined once at :407)."""
    if reuse is None:
        reuse = key.startswith("myopic")
    from mrbo import bayesopt
    s = SETTINGS[key]
    testfn = bayesopt.TESTFNS[s["fn"]]()
    true_minimum = float(testfn.f(np.asarray(testfn.xopt[0], dtype=np.float64)))
    myopic = key.startswith("myopic")
    with tempfile.TemporaryDirectory() as tmp:
        t0 = time.perf_counter()
        lg = lambda *m: log(f"[{key}] " + " ".join(map(str, m)))
        if myopic:
            rb = (run_budget or s["run_budget"]) if reuse else s["budget"]
            res = bayesopt.run_myopic(s["fn"], tmp, budget=rb, trials=trials, starts=s["starts"], seed=seed,
                                      rules=(s["rule"],), initial_observations=s["initial"], log=lg,
                                      reuse_surrogate=reuse, capacity=s["capacity"] if reuse else None,
                                      solve_margin=solve_margin, no_repeat=no_repeat)
        else:
            res = bayesopt.run(s["fn"], tmp, budget=s["budget"], trials=trials, starts=s["starts"], horizon=s["horizon"],
                               mc_samples=100, batch_size=s["batch"], sgd_iterations=50, optimize=True, seed=seed,
                               rules=("ei",), initial_observations=s["initial"], solver=solver, eta=eta,
                               fmini_over_capacity=q3, incumbent=incumbent, reuse_surrogate=reuse, log=lg)
        wall = time.perf_counter() - t0
    trials_res = []
    for t in range(trials):
        r = res[(s["rule"], t) if myopic else (f"rollout_{s['horizon']}_ei", t)]
        y = r["y"]
        r = dict(r, initial_best=float(np.min(y[:s["initial"]])))
        trials_res.append(r)
    gcols = our_gap_columns(trials_res, true_minimum, len(trials_res[0]["gaps"]))
    lbs, ubs = testfn.get_bounds()
    diag = trajectory_diagnostics([r["X"] for r in trials_res], lbs, ubs, s["initial"])
    if myopic:   # repeated observations per trial within the compared budget
        nb = int(s["labels"][-1])
        diag["repeats_per_trial_in_budget"] = float(np.mean([np.sum(r["repeats"][:nb]) for r in trials_res]))
    per_label = {lab: compare(our_column(gcols, lab, myopic), ref_column(case, lab)) for lab in s["labels"]}
    our_times = np.concatenate([r["times"] for r in trials_res])
    ref_times = np.array(case["times"], float)[:, :s["budget"]].ravel()
    ref_times = ref_times[ref_times >= 0]
    return {"case": key, "reference": case["source"], "settings": dict(s, trials=trials, mc_samples=100,
                                                                        sgd_iterations=50, optimize=True, solver=solver,
                                                                        eta=eta, seed=seed, q3_fmini_over_capacity=q3,
                                                                        incumbent_restart=incumbent,
                                                                        reuse_surrogate=reuse,
                                                                        solve_margin=solve_margin,
                                                                        no_repeat=no_repeat),
            "gaps": per_label, "difference_detected": {lab: detected(v) for lab, v in per_label.items()},
            "ours_lengthscale": {"start_median": float(np.median([r["ell_start"] for r in trials_res])),
                                 "end_median": float(np.median([r["ell_end"] for r in trials_res])),
                                 "start_first_trials": [r["ell_start"] for r in trials_res[:5]]},
            "ours_trajectory_diagnostics": diag, "ours_mean_curve": gcols.mean(axis=0).tolist(),
            "seconds_per_solve": {"ours_median": float(np.median(our_times)), "ref_median": float(np.median(ref_times)),
                                  "ref_note": "reference times from earlier code versions on unstated hardware"},
            "wall_s": wall}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=20)
    ap.add_argument("--seed", type=int, default=1906)
    ap.add_argument("--cases", default=",".join(SETTINGS), help="comma list, or 'asserted'")
    ap.add_argument("--out", default="")
    ap.add_argument("--solver", default="sga", choices=["sga", "adam"],
                    help="outer solver of the build-defined rollout acquisition (mrbo/bayesopt.py)")
    ap.add_argument("--eta", type=float, default=0.0, help="step (default 0.01 for sga -- StandardSGA's default, optimizers.jl:9 -- and 0.02 box widths "
                         "for adam)")
    ap.add_argument("--no-q3", action="store_true",
                    help="diagnostic: fmini over the observed points instead of the zero-padded buffer (Q3 off)")
    ap.add_argument("--reuse", choices=("auto", "yes", "no"), default="auto",
                    help="surrogate reuse over trials: auto = the recording driver's semantics (myopic: reused, "
                         "myopic_bayesopt.jl:205-217; archived rollout runs: fresh per trial, "
                         "adaptive_bayesopt.jl:498); yes / no force it (diagnostics)")
    ap.add_argument("--no-incumbent", action="store_true",
                    help="diagnostic: the round-2 solver (no incumbent restart, no no-repeat pick)")
    ap.add_argument("--solve-margin", type=float, default=0.0,
                    help="diagnostic (myopic cases): solve the acquisition on the box shrunk by this fraction of "
                         "its width per side -- a proxy for IPNewton's interior iterates")
    ap.add_argument("--no-repeat", action="store_true",
                    help="diagnostic (myopic cases): take the best start whose minimiser is not an observed point")
    a = ap.parse_args()
    ref = load_reference()
    log = lambda m: print(m, file=sys.stderr, flush=True)
    for key in (ASSERTED if a.cases == "asserted" else a.cases.split(",")):
        eta = a.eta or (0.01 if a.solver == "sga" else 0.02)
        row = run_case(key, ref[key], a.trials, a.seed, log, solver=a.solver, eta=eta, q3=not a.no_q3, incumbent=not a.no_incumbent,
                       reuse={"auto": None, "yes": True, "no": False}[a.reuse], solve_margin=a.solve_margin, no_repeat=a.no_repeat)
        line = json.dumps(row)
        print(line, flush=True)
        if a.out:
            with open(a.out, "a") as f:
                f.write(line + "\n")
        g = row["gaps"][SETTINGS[key]["labels"][-1]]
        log(f"{key} [{a.solver}{'' if not a.no_q3 else ', Q3 off'}{'' if not a.no_incumbent else ', no incumbent'}"
            f"{'' if not a.solve_margin else f', margin {a.solve_margin:g}'}{', no repeat' if a.no_repeat else ''}]: final gap ours {g['ours_mean']:.3f}±{g['ours_se']:.3f} ref {g['ref_mean']:.3f}±{g['ref_se']:.3f} "
            f"diff {g['diff_mean']:+.3f} [{g['diff_ci95'][0]:+.3f}, {g['diff_ci95'][1]:+.3f}] "
            f"MW p={g['mannwhitney_p']:.3f} ({row['difference_detected'][SETTINGS[key]['labels'][-1]]}); s/solve ours {row['seconds_per_solve']['ours_median']:.3f} "
            f"ref {row['seconds_per_solve']['ref_median']:.2f}; diag {row['ours_trajectory_diagnostics']}")


if __name__ == "__main__":
    main()
