#!/usr/bin/env python3
"""Trace one trial of the rollout BO loop (mrbo/bayesopt.py): per budget step the restarts'
final ETO means, how far each restart moved, the chosen xnext and its distance to the observed
points.  Diagnostic for DESIGN.md §10 (the loop's observation sequences vs. the reference's
archived ones).

usage: python tools/bo_trace.py rosenbrock [--horizon 0] [--budget 20] [--trial 0] [--no-incumbent]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "rollout-bayesian-optimization_amd"), ROOT]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fn")
    ap.add_argument("--horizon", type=int, default=0)
    ap.add_argument("--budget", type=int, default=20)
    ap.add_argument("--trial", type=int, default=0)
    ap.add_argument("--initial", type=int, default=1)
    ap.add_argument("--solver", default="sga")
    ap.add_argument("--eta", type=float, default=0.01)
    ap.add_argument("--seed", type=int, default=1906)
    ap.add_argument("--no-incumbent", action="store_true")
    ap.add_argument("--no-q3", action="store_true", help="fmini over the observed points (Q3 off)")
    a = ap.parse_args()
    from mrbo import bayesopt
    from mrbo.decision_rules import EI
    from mrbo.kernels import Matern52
    from mrbo.mle import optimize as mle_optimize
    from mrbo.surrogates import Surrogate
    np.set_printoptions(precision=4, linewidth=160)
    tf = bayesopt.TESTFNS[a.fn]()
    lbs, ubs = tf.get_bounds()
    rng = np.random.default_rng(a.seed)
    samples = [lbs[:, None] + (ubs - lbs)[:, None] * rng.random((tf.dim, a.initial)) for _ in range(a.trial + 1)]
    X0 = samples[a.trial]
    sur = Surrogate(Matern52(), X0, tf(X0), capacity=a.budget + a.initial, decision_rule=EI(), σn2=1e-6)
    sur.fmini_over_capacity = not a.no_q3
    print("initial", X0.ravel(), tf(X0))
    for b in range(a.budget):
        tr = []
        Xa = sur.get_active_covariates().copy()
        xn, _ = bayesopt.rollout_solve(sur, lbs, ubs, a.horizon, 100, 8, 8, 50, 0.0, eta=a.eta, solver=a.solver,
                                       incumbent=not a.no_incumbent, trace=tr)
        t = tr[0]
        dmin = float(np.min(np.linalg.norm(Xa - xn[:, None], axis=0)))
        print(f"step {b:2d} pick {t['pick']} x {xn} f {tf.f(xn):.4g} dist-to-observed {dmin:.2e} "
              f"kernel {sur.get_kernel()}")
        print("   ETO at finals", t["means"])
        print("   moved        ", np.linalg.norm(t["x"] - t["batch"], axis=0))
        sur.condition(xn, float(tf.f(xn)))
        mle_optimize(sur, bayesopt.KERNEL_LBS, bayesopt.KERNEL_UBS)


if __name__ == "__main__":
    main()
