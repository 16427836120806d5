"""Non-myopic Bayesian-optimisation loop on the rollout acquisition.

Mirrors experiments/nonmyopic_bayesopt.jl -- its CLI, its experiment layout and its CSV outputs
(create_csv / write_to_csv, utils.jl:155-172) -- with the acquisition step routed through the
rollout path as the survey prescribes: the reference's main loop calls the myopic
multistart_base_solve! (:245-253) and its adaptive driver names a rollout_solver that is
defined nowhere (experiments/adaptive_bayesopt.jl:490), so the solver here is build-defined:

  batch = generate_batch(batch_size)             utils.jl:97-106 (Sobol + two near-bound points)
          + one restart next to the incumbent     (build-defined, rollout_solve)
  x_r  ← stochastic_solve from every batch point  utils.jl:235-265 (StandardSGA, eswavs stop),
         all restarts in one rollout launch per SGA iteration (stochastic_solve_batch)
  xnext = the restart with the largest final ETO mean, clamped to the box, that is not an
          already observed point

Per budget step the metrics are recorded as in the reference (:268-289): time of the solve,
gap and simple regret of the observations BEFORE conditioning on xnext, then condition!,
optionally optimize! (lengthscale MLE on the device, bounds [0.1, 5]), then the minimum
observation.  `allocations` is the reference's @timed byte count; the build records the
device workspace is preallocated and writes 0.

Parity with the reference's BO trajectories is unpinned: Julia's MersenneTwister initial
designs, Optim.jl's inner solves and the undefined rollout solver cannot be reproduced.
"""
import argparse
import os
import time

import numpy as np

from . import testfns as T
from .decision_rules import EI, LCB, POI
from .kernels import Matern52
from .optimizers import Adam, StandardSGA
from .rollout import simulate_trajectory_mc_batch
from .surrogates import FantasySurrogate, Surrogate
from .trajectory import Trajectory, TrajectoryParameters
from .utils import ExperimentSetup, gap, generate_batch, simple_regret, stochastic_solve_batch

INITIAL_OBSERVATIONS = 5            # nonmyopic_bayesopt.jl:131
METRICS = ["times", "gaps", "allocations", "simple_regret", "minimum_observations"]   # :191
KERNEL_LBS, KERNEL_UBS = [0.1], [5.0]   # :230

TESTFNS = {
    "gramacylee": T.TestGramacyLee,
    "braninhoo": T.TestBraninHoo,
    "hartmann6d": T.TestHartmann6D,
    "rosenbrock": T.TestRosenbrock,
    **{f"ackley{d}d": (lambda d=d: T.TestAckley(d)) for d in (1, 2, 3, 4, 5, 8)},
    **{f"rastrigin{d}d": (lambda d=d: T.TestRastrigin(d)) for d in (1, 4)},
    "hartmann3d": T.TestHartmann3D,
    "sixhump": T.TestSixHump,
    "goldsteinprice": T.TestGoldsteinPrice,
    "griewank3d": lambda: T.TestGriewank(3),
    "levy10d": lambda: T.TestLevy(10),
}


# ---- CSV outputs (utils.jl:155-172) --------------------------------------------------------
def _fmt(v):
    v = float(v)
    return repr(v) if np.isfinite(v) else ("NaN" if np.isnan(v) else ("Inf" if v > 0 else "-Inf"))


def create_csv(filename, budget):
    """create_csv: header [trial; 1..budget] and one placeholder row of −1.0."""
    with open(filename + ".csv", "w") as f:
        f.write(",".join(["trial"] + [str(b) for b in range(1, budget + 1)]) + "\n")
        f.write(",".join(["-1.0"] * (budget + 1)) + "\n")


def write_to_csv(filename, data):
    """write_to_csv: append `data` as one row (CSV.write(Tables.table(data'), append=true) writes
    the budget values only, without a trial column)."""
    with open(filename + ".csv", "a") as f:
        f.write(",".join(_fmt(v) for v in np.asarray(data, dtype=np.float64).ravel()) + "\n")


def write_metadata(directory, budget, trials, starts):
    """write_metadata_to_file (:102-118)."""
    with open(os.path.join(directory, "metadata.txt"), "w") as f:
        f.write(f"Budget: {budget}\nNumber of Trials: {trials}\nNumber of Starts: {starts}\n")


# ---- one acquisition solve -------------------------------------------------------------------
class BoxAdam:
    """Adam (optimizers.jl:25-74) on the box-normalised coordinates u = (x − lb)/(ub − lb), projected
    onto the box after every step: a step of ≈ η box widths per coordinate whatever the scale of
    the objective (StandardSGA's fixed η either stalls or throws restarts out of the box when the
    acquisition's gradient is large, e.g. Branin's).  Build-defined: the reference's rollout solver
    is undefined (experiments/adaptive_bayesopt.jl:490)."""

    def __init__(self, lbs, ubs, η=0.02):
        self.lbs, self.ubs = np.asarray(lbs, float), np.asarray(ubs, float)
        self.w = self.ubs - self.lbs
        self.adam = Adam(η=η)

    def update(self, x, grad_f):
        u = (x - self.lbs) / self.w
        self.adam.update(u, np.asarray(grad_f, float) * self.w)
        x[:] = np.clip(self.lbs + self.w * u, self.lbs, self.ubs)
        return x


INCUMBENT_NUDGE = 1e-2     # box widths: the incumbent restart starts this far off the observed point


def incumbent_start(sur, lbs, ubs):
    """The incumbent restart: the best observed point moved INCUMBENT_NUDGE box widths towards the
    box centre in every coordinate (at an observed point σ and its gradient vanish, so a restart
    placed exactly there cannot move)."""
    X, y = sur.get_active_covariates(), sur.get_active_observations()
    xb = np.asarray(X[:, int(np.argmin(y))], float)
    w = ubs - lbs
    step = np.where(xb <= 0.5 * (lbs + ubs), 1.0, -1.0) * INCUMBENT_NUDGE * w
    return np.clip(xb + step, lbs, ubs)


def rollout_solve(sur, lbs, ubs, horizon, mc_samples, batch_size, starts, sgd_iterations, theta, eta=0.01,
                  device=0, solver="sga", incumbent=True, trace=None):
    """xnext from the rollout acquisition: restarts from a Sobol batch (StandardSGA with step `eta`,
    or BoxAdam with `eta` box widths per step), best final ETO mean.

    incumbent=True adds one restart next to the best observed point (incumbent_start) and never
    returns an already observed point while another restart ends elsewhere.  Both are the build's
    answer to an acquisition that underflows to exactly 0 on the whole Sobol batch -- an objective
    of large scale under the reference's unit-variance, zero-mean surrogate (Rosenbrock,
    Goldstein–Price): every batch restart then has a zero gradient, the argmax ties at the first
    restart and the loop re-observes it for the rest of the budget.
    `trace`, a list, receives one dict per call (batch, final points, final ETO means, pick)."""
    lbs, ubs = np.asarray(lbs, float), np.asarray(ubs, float)
    batch = generate_batch(batch_size, lbs, ubs)
    if incumbent:
        batch = np.hstack([batch, incumbent_start(sur, lbs, ubs)[:, None]])
    tp = TrajectoryParameters(start=batch[:, 0], hypers=[theta], horizon=horizon, mc_iterations=mc_samples,
                              use_low_discrepancy_sequence=True, spatial_lowerbounds=lbs, spatial_upperbounds=ubs)
    es = ExperimentSetup(tp, number_of_starts=starts)
    traj = Trajectory(sur, FantasySurrogate(sur, horizon), start=batch[:, 0], hypers=[theta], horizon=horizon)
    opts = [StandardSGA(η=eta) if solver == "sga" else BoxAdam(lbs, ubs, η=eta) for _ in range(batch.shape[1])]
    x, _ = stochastic_solve_batch(opts, sur, tp, es, batch, T=traj, iterations=sgd_iterations, device=device)
    x = np.clip(x, lbs[:, None], ubs[:, None])
    etos = simulate_trajectory_mc_batch(traj, tp, x, es.get_starts(), with_gradient=False, device=device).etos(
        with_gradient=False)
    means = np.array([e.mean() for e in etos])
    means = np.where(np.isfinite(means), means, -np.inf)
    rank = means.copy()
    if incumbent:
        Xa = sur.get_active_covariates()
        w = ubs - lbs
        d = np.abs((x[:, :, None] - Xa[:, None, :]) / w[:, None, None]).max(axis=0).min(axis=1)
        rank = np.where(d > 1e-9, rank, -np.inf) if (d > 1e-9).any() else rank
    k = int(np.argmax(rank))
    if trace is not None:
        trace.append(dict(batch=batch, x=x.copy(), means=means, pick=k))
    return x[:, k].copy(), float(means[k])


# ---- the experiment loop (nonmyopic_bayesopt.jl:120-300) -------------------------------------
def run(function_name, output_dir, budget=15, trials=60, starts=16, horizon=0, mc_samples=200, batch_size=8,
        sgd_iterations=50, optimize=False, seed=1906, device=0, log=print, rules=("ei", "poi", "lcb"), eta=0.01,
        initial_observations=INITIAL_OBSERVATIONS, solver="sga", fmini_over_capacity=True, incumbent=True,
        reuse_surrogate=True):
    """The experiment loop; `rules` selects a subset of the reference's three acquisitions (all by
    default, as nonmyopic_bayesopt.jl), `eta` the StandardSGA step of the build-defined solver
    (default 0.01, StandardSGA's own default, optimizers.jl:9),
    `initial_observations` the initial design size (5 in the current script, :131), `solver` "sga"
    (StandardSGA, η = eta) or "adam" (BoxAdam, eta box widths per step); fmini_over_capacity=False
    turns the reference's Q3 off (fmini over the observed points, not the zero-padded buffer),
    incumbent=False drops rollout_solve's incumbent restart and no-repeat pick (the round-2 solver).
    reuse_surrogate=True (the reference, :233-235): one surrogate of capacity budget + initial for
    every rule and trial, reset! per trial -- the kernel carries over between trials, and fmini over
    the capacity buffer (Q3) sees the stale observations of the previous trial past the initial
    design; False: a fresh surrogate per trial (the round-3 loop)."""
    testfn = TESTFNS[function_name]()
    lbs, ubs = testfn.get_bounds()
    directory = os.path.join(output_dir, function_name)
    os.makedirs(directory, exist_ok=True)
    table = {"ei": (EI(), 0.0), "poi": (POI(), 0.0), "lcb": (LCB(), 2.0)}
    acquisitions = [f"rollout_{horizon}_{r}" for r in rules]
    dr_hypers = [table[r][1] for r in rules]
    rules = [table[r][0] for r in rules]
    for metric in METRICS:
        for acq in acquisitions:
            create_csv(os.path.join(directory, f"{acq}_{metric}"), budget)
    write_metadata(directory, budget, trials, starts)
    rng = np.random.default_rng(seed)
    initial_samples = [lbs[:, None] + (ubs - lbs)[:, None] * rng.random((testfn.dim, initial_observations))
                       for _ in range(trials)]
    true_minimum = float(testfn.f(np.asarray(testfn.xopt[0], dtype=np.float64)))
    results = {}
    sur = None
    if reuse_surrogate:    # :233 "Preallocate entire surrogate object and reuse"
        sur = Surrogate(Matern52(), np.zeros((testfn.dim, 1)), np.zeros(1), capacity=budget + initial_observations,
                        σn2=1e-6)
    for acq, rule, theta in zip(acquisitions, rules, dr_hypers):
        if reuse_surrogate:
            sur.set_decision_rule(rule)                                   # :241
        log(f"Conducting experiments with acquisition = {acq}")
        for trial in range(trials):
            Xinit = initial_samples[trial]
            yinit = testfn(Xinit)
            if reuse_surrogate:
                sur.reset(Xinit, yinit)                                   # :253
            else:
                sur = Surrogate(Matern52(), Xinit, yinit, capacity=budget + initial_observations, decision_rule=rule,
                                σn2=1e-6)
            sur.fmini_over_capacity = fmini_over_capacity
            ell_start = float(sur.ψ.lengthscale)
            initial_best = float(np.min(yinit))
            times, gaps, allocs, regrets, minobs = (np.zeros(budget) for _ in range(5))
            repeats = np.zeros(budget, dtype=bool)
            for b in range(budget):
                t0 = time.perf_counter()
                xnext, _ = rollout_solve(sur, lbs, ubs, horizon, mc_samples, batch_size, starts, sgd_iterations,
                                         theta, eta=eta, device=device, solver=solver, incumbent=incumbent)
                times[b] = time.perf_counter() - t0
                observed_best = float(np.min(sur.get_active_observations()))
                regrets[b] = simple_regret(true_minimum, observed_best)
                gaps[b] = gap(initial_best, observed_best, true_minimum)
                sur.condition(xnext, float(testfn.f(xnext)))
                if optimize:
                    from .mle import optimize as mle_optimize
                    mle_optimize(sur, KERNEL_LBS, KERNEL_UBS)
                minobs[b] = float(np.min(sur.get_active_observations()))
            log(f"{acq} trial {trial + 1}/{trials}: gap {gaps[-1]:.4f}, {times.sum():.2f} s of solves")
            for metric, data in zip(METRICS, (times, gaps, allocs, regrets, minobs)):
                write_to_csv(os.path.join(directory, f"{acq}_{metric}"), data)
            results[(acq, trial)] = dict(times=times, gaps=gaps, simple_regret=regrets, minimum_observations=minobs,
                                         X=sur.get_active_covariates().copy(), y=sur.get_active_observations().copy(),
                                         ell_start=ell_start, ell_end=float(sur.ψ.lengthscale), repeats=repeats)
    return results


# ---- the myopic experiment loop (experiments/myopic_bayesopt.jl:93-270) -----------------------
MYOPIC_RULES = {"ei": (EI, 0.0), "poi": (POI, 0.0), "lcb": (LCB, 2.0)}   # :151-153 (random: no solve)


def run_myopic(function_name, output_dir, budget=100, trials=60, starts=64, seed=1906, device=0, log=print,
               rules=("ei", "poi", "lcb"), optimize=True, initial_observations=INITIAL_OBSERVATIONS,
               reuse_surrogate=True, capacity=None, solve_margin=0.0, no_repeat=False):
    """myopic_bayesopt.jl's loop: per budget step xnext = multistart_base_solve!(sur, …; guesses =
    generate_initial_guesses(starts, lbs, ubs), θfixed) -- the deterministic multistart local solve of
    the analytic acquisition on the base surrogate (:224-233), here mrbo_base_solve on the device --
    then the metrics before conditioning (:234-245), condition!, optimize! (lengthscale MLE, bounds
    [0.1, 5], :248-249) and the minimum observation.  CSVs `<acq>_<metric>.csv` as the reference.

    reuse_surrogate=True (the reference): ONE surrogate, built once with capacity = budget (:205),
    serves every rule (set_decision_rule!, :208) and every trial (reset!(sur, Xinit, yinit), :217).
    reset! keeps the kernel, so each trial starts from the lengthscale the previous trial's last
    optimize! left (only the very first trial starts at Matern52()'s ℓ = 1), and past `capacity`
    observations condition! conditions a discarded resized copy (Surrogate.condition).  False: a
    fresh surrogate with ℓ = 1 and capacity budget + initial per trial (the round-3 loop).

    solve_margin (diagnostic, build-defined; 0 = the reference's box): the acquisition is solved on
    the box shrunk by solve_margin·(ub − lb) per side -- a proxy for IPNewton's interior iterates
    (rbf_optim.jl:24-30: a log barrier keeps them off the faces), used to test whether the
    projected Newton's stops on the faces explain a difference.
    no_repeat (diagnostic, build-defined; False = the reference's findmin): the best start whose
    minimiser is not an observed point (within 1e-6 of a box width) is taken, to test whether
    re-observing a point explains a difference; every trial records its repeated observations."""
    from .rbf_optim import base_solve_batch, findmin_candidates, multistart_base_solve
    from .utils import generate_initial_guesses
    testfn = TESTFNS[function_name]()
    lbs, ubs = testfn.get_bounds()
    directory = os.path.join(output_dir, "myopic", function_name)
    os.makedirs(directory, exist_ok=True)
    for metric in METRICS:
        for acq in rules:
            create_csv(os.path.join(directory, f"{acq}_{metric}"), budget)
    write_metadata(directory, budget, trials, starts)
    guesses = generate_initial_guesses(starts, lbs, ubs)                     # :186
    rng = np.random.default_rng(seed)
    initial_samples = [lbs[:, None] + (ubs - lbs)[:, None] * rng.random((testfn.dim, initial_observations))
                       for _ in range(trials)]                              # :187
    true_minimum = float(testfn.f(np.asarray(testfn.xopt[0], dtype=np.float64)))
    results = {}
    sur = None
    if reuse_surrogate:    # :205 "Preallocate entire surrogate object and reuse"
        # capacity = BUDGET as the reference; it must hold the initial design (a reset! past
        # capacity is a BoundsError in Julia), so a budget below it gets the design's size
        sur = Surrogate(Matern52(), np.zeros((testfn.dim, 1)), np.zeros(1),
                        capacity=capacity or max(budget, initial_observations), σn2=1e-6)
    for acq in rules:
        make_rule, theta = MYOPIC_RULES[acq]
        if reuse_surrogate:
            sur.set_decision_rule(make_rule())                            # :208
        log(f"Conducting experiments with acquisition = {acq}")
        for trial in range(trials):
            Xinit = initial_samples[trial]
            yinit = testfn(Xinit)
            if reuse_surrogate:
                sur.reset(Xinit, yinit)                                   # :217
            else:
                sur = Surrogate(Matern52(), Xinit, yinit, capacity=capacity or budget + initial_observations,
                                decision_rule=make_rule(), σn2=1e-6)
            ell_start = float(sur.ψ.lengthscale)
            initial_best = float(np.min(yinit))
            times, gaps, allocs, regrets, minobs = (np.zeros(budget) for _ in range(5))
            repeats = np.zeros(budget, dtype=bool)
            xnext = np.zeros(testfn.dim)
            for b in range(budget):
                t0 = time.perf_counter()
                w = (ubs - lbs) * solve_margin
                if no_repeat:
                    xs_, fs_, _ = base_solve_batch(sur, lbs + w, ubs - w, guesses, [theta], device=device)
                    Xo = sur.X[:, :sur.observed]
                    tol = 1e-6 * (ubs - lbs)[:, None]
                    fresh = [i for i in range(xs_.shape[1])
                             if not (np.abs(Xo - xs_[:, i:i + 1]) <= tol).all(axis=0).any()]
                    pick = findmin_candidates(xs_[:, fresh], fs_[fresh]) if fresh else None
                    xnext[:] = xs_[:, fresh[pick]] if fresh else xs_[:, findmin_candidates(xs_, fs_)]
                elif solve_margin > 0.0:
                    multistart_base_solve(sur, xnext, lbs + w, ubs - w, guesses, [theta], device=device)
                else:
                    multistart_base_solve(sur, xnext, lbs, ubs, guesses, [theta], device=device)
                times[b] = time.perf_counter() - t0
                Xo = sur.X[:, :sur.observed]
                repeats[b] = bool((np.abs(Xo - xnext[:, None]) <= 1e-6 * (ubs - lbs)[:, None]).all(axis=0).any())
                observed_best = float(np.min(sur.get_active_observations()))
                regrets[b] = simple_regret(true_minimum, observed_best)
                gaps[b] = gap(initial_best, observed_best, true_minimum)
                sur.condition(xnext, float(testfn.f(xnext)))
                if optimize:
                    from .mle import optimize as mle_optimize
                    mle_optimize(sur, KERNEL_LBS, KERNEL_UBS)
                minobs[b] = float(np.min(sur.get_active_observations()))
            log(f"myopic {acq} trial {trial + 1}/{trials}: gap {gaps[-1]:.4f}, {times.sum():.2f} s of solves")
            for metric, data in zip(METRICS, (times, gaps, allocs, regrets, minobs)):
                write_to_csv(os.path.join(directory, f"{acq}_{metric}"), data)
            results[(acq, trial)] = dict(times=times, gaps=gaps, simple_regret=regrets, minimum_observations=minobs,
                                         X=sur.get_active_covariates().copy(), y=sur.get_active_observations().copy(),
                                         ell_start=ell_start, ell_end=float(sur.ψ.lengthscale), repeats=repeats)
    return results


def parse(argv=None):
    """parse_command_line (nonmyopic_bayesopt.jl:4-75)."""
    ap = argparse.ArgumentParser("Non-myopic Bayesian optimisation on the MI355X rollout acquisition")
    ap.add_argument("--seed", type=int, default=1906)
    ap.add_argument("--optimize", action="store_true", help="optimize the surrogate's lengthscale (MLE)")
    ap.add_argument("--starts", type=int, default=16)
    ap.add_argument("--trials", type=int, default=60)
    ap.add_argument("--budget", type=int, default=15)
    ap.add_argument("--output-dir", required=True)
    ap.add_argument("--mc-samples", type=int, default=200)
    ap.add_argument("--horizon", type=int, default=0)
    ap.add_argument("--batch-size", type=int, default=8)
    ap.add_argument("--function-name", required=True, choices=sorted(TESTFNS))
    ap.add_argument("--sgd-iterations", type=int, default=50)
    return ap.parse_args(argv)


def main(argv=None):
    a = parse(argv)
    run(a.function_name, a.output_dir, budget=a.budget, trials=a.trials, starts=a.starts, horizon=a.horizon,
        mc_samples=a.mc_samples, batch_size=a.batch_size, sgd_iterations=a.sgd_iterations, optimize=a.optimize,
        seed=a.seed)


if __name__ == "__main__":
    main()
