"""The BASELINE.json configurations as synthetic problems (SURVEY.md §8d "Synthetic inputs").

Kernel Matern52(ℓ=1), σn2 = 1e-6 (nonmyopic_bayesopt.jl:228), EI with θ = [0].  Base X is a
Kronecker low-discrepancy design (low_discrepancy.jl:7-28) scaled to the test-function box,
y = f(X); restarts x0 continue the same Kronecker sequence; the rnstream is Sobol →
Box–Muller(log10); inner starts are 16 Sobol points + 2 near-bound points (utils.jl:145-153).
"""
from dataclasses import dataclass

import numpy as np

from . import testfns
from .decision_rules import EI
from .kernels import Matern52
from .surrogates import FantasySurrogate, Surrogate
from .trajectory import Trajectory, TrajectoryParameters
from .utils import ExperimentSetup, kronecker_quasirand


@dataclass
class Config:
    name: str
    testfn: str
    d: int
    h: int
    M: int
    R: int
    N: int
    gpus: int
    note: str = ""


CONFIGS = {
    "C1": Config("C1", "gramacylee", 1, 1, 32, 4, 8, 1, "1D GramacyLee, h=1, 32 MC x 4 restarts, n=8"),
    "C2": Config("C2", "braninhoo", 2, 2, 256, 16, 32, 1, "2D Branin, h=2, 256 MC x 16 restarts, n=32"),
    "C3": Config("C3", "hartmann6d", 6, 3, 1024, 64, 64, 1, "6D Hartmann, h=3, 1024 MC x 64 restarts, n=64 (headline)"),
    "C4": Config("C4", "hartmann6d", 6, 4, 8192, 256, 128, 8, "6D Hartmann, h=4, 8192 MC x 256 restarts, n=128"),
    # BASELINE names "8D Ackley + NonUniformCost": NonUniformCost (cost_functions.jl:5-20) is
    # referenced by no decision rule, surrogate or trajectory (SURVEY.md §0 finding 5); the build
    # defines the cost-weighted inner-solve rule α/c(x) (include/mrbo.h mrbo_cost_t, parity
    # unpinned) and C5 runs it with Problem(cost=True) / bench.py --cost
    "C5": Config("C5", "ackley", 8, 5, 16384, 512, 256, 8, "8D Ackley, h=5, 16384 MC x 512 restarts, n=256"),
}

# C5's NonUniformCost: c(x) = 1 + Σ_a u_a², u = (x − lb)/(ub − lb) -- a bowl from 1 at the lower
# corner to 1 + d at the upper one (build-defined)
C5_COST = ("quadratic", 1.0, 1.0)


def make_testfn(name, d):
    return {"gramacylee": testfns.TestGramacyLee, "braninhoo": testfns.TestBraninHoo,
            "hartmann6d": testfns.TestHartmann6D}.get(name, lambda: testfns.TestAckley(d))()


class Problem:
    def __init__(self, cfg, M=None, R=None, capacity=None, nstarts=16, cost=False):
        self.cfg = cfg
        self.cost = (C5_COST[0], C5_COST[1], np.full(cfg.d, C5_COST[2])) if cost else None
        tf = make_testfn(cfg.testfn, cfg.d)
        lbs, ubs = tf.get_bounds()
        self.lbs, self.ubs = lbs, ubs
        w = (ubs - lbs)[:, None]
        X = lbs[:, None] + w * kronecker_quasirand(cfg.d, cfg.N)
        y = tf(X)
        self.surrogate = Surrogate(Matern52(), X, y, capacity=capacity or cfg.N, decision_rule=EI(), σn2=1e-6)
        self.M = M or cfg.M
        self.R = R or cfg.R
        self.x0s = lbs[:, None] + w * kronecker_quasirand(cfg.d, self.R, cfg.N)
        self.tp = TrajectoryParameters(start=self.x0s[:, 0], hypers=[0.0], horizon=cfg.h, mc_iterations=self.M,
                                       use_low_discrepancy_sequence=True, spatial_lowerbounds=lbs,
                                       spatial_upperbounds=ubs)
        self.es = ExperimentSetup(tp=self.tp, number_of_starts=nstarts)
        self.fs = FantasySurrogate(self.surrogate, cfg.h)
        self.T = Trajectory(self.surrogate, self.fs, start=self.x0s[:, 0], hypers=[0.0], horizon=cfg.h)


    def cost_model(self):
        """(kind, c0, w) of the NonUniformCost weighting, or None"""
        return self.cost

    def plan_opts(self):
        """RolloutPlan options of this problem beyond the defaults (the cost model)"""
        if self.cost is None:
            return {}
        kind, c0, w = self.cost
        return dict(cost=kind, cost_c0=float(c0), cost_w=tuple(float(v) for v in w))


def problem(name, **kw):
    return Problem(CONFIGS[name], **kw)
