"""Trajectory, TrajectoryParameters, ExpectedTrajectoryOutput -- mirror of trajectory.jl."""
import numpy as np

from .engine import rnstream as _rnstream


class Trajectory:
    """trajectory.jl:17-37"""

    def __init__(self, base_surrogate, fantasy_surrogate, start, hypers, horizon):
        self.s = base_surrogate
        self.fs = fantasy_surrogate
        self.x0 = np.array(start, dtype=np.float64).ravel()
        self.θ = np.array(hypers, dtype=np.float64).ravel()
        self.horizon = int(horizon)
        self.observable = None

    def set_start(self, x0):
        """set_start! trajectory.jl:26"""
        self.x0[:] = x0

    def get_starting_point(self):
        return self.x0

    def get_hyperparameters(self):
        return self.θ

    def get_horizon(self):
        return self.horizon

    def get_base_surrogate(self):
        return self.s

    def get_fantasy_surrogate(self):
        return self.fs


def gen_low_discrepancy_sequence(samples, dim, horizon):
    """utils.jl:65-74: M×(d+1)×H Sobol → Box–Muller(log10) stream (Q1, Q2)."""
    return _rnstream(samples, dim, horizon)


class TrajectoryParameters:
    """trajectory.jl:43-94"""

    def __init__(self, start, hypers, horizon, mc_iterations, use_low_discrepancy_sequence, spatial_lowerbounds,
                 spatial_upperbounds, rnstream=None, rng=None):
        x0 = np.array(start, dtype=np.float64).ravel()
        lbs = np.array(spatial_lowerbounds, dtype=np.float64).ravel()
        ubs = np.array(spatial_upperbounds, dtype=np.float64).ravel()
        assert lbs.size == x0.size and ubs.size == x0.size, \
            "Lower and upper bounds must be the same length as the initial point"
        d = x0.size
        if rnstream is None:
            if use_low_discrepancy_sequence:
                rnstream = gen_low_discrepancy_sequence(mc_iterations, d, horizon + 1)
            else:
                rng = rng or np.random.default_rng()
                rnstream = np.asfortranarray(rng.standard_normal((mc_iterations, d + 1, horizon + 1)))
        rnstream = np.asarray(rnstream, dtype=np.float64)
        assert rnstream.shape[1] == d + 1 and rnstream.shape[2] <= horizon + 1, \
            "Random number stream must have d + 1 rows and h + 1 columns for each sample"
        assert rnstream.shape[0] == mc_iterations, "Random number stream must have mc_iters samples"
        self.x0 = x0
        self.horizon = int(horizon)
        self.mc_iters = int(mc_iterations)
        self.rnstream_sequence = rnstream
        self.spatial_lbs = lbs
        self.spatial_ubs = ubs
        self.θ = np.array(hypers, dtype=np.float64).ravel()

    def get_spatial_bounds(self):
        return self.spatial_lbs, self.spatial_ubs

    def get_starting_point(self):
        return self.x0.copy()

    def set_starting_point(self, x):
        self.x0[:] = x

    def get_hyperparameters(self):
        return self.θ.copy()

    def get_samples_rnstream(self, sample_index):
        return self.rnstream_sequence[sample_index]

    def each_trajectory(self, start=0):
        return range(start, self.mc_iters)


class ExpectedTrajectoryOutput:
    """trajectory.jl:112-134"""

    def __init__(self, μxθ, σ_μxθ, grad_μx=None, σ_grad_μx=None, grad_μθ=None, σ_grad_μθ=None):
        self.μxθ = μxθ
        self.σ_μxθ = σ_μxθ
        self.grad_μx = grad_μx
        self.σ_grad_μx = σ_grad_μx
        self.grad_μθ = grad_μθ
        self.σ_grad_μθ = σ_grad_μθ

    def mean(self):
        return self.μxθ

    def std(self):
        return self.σ_μxθ

    def gradient(self, wrt_hypers=False):
        return self.grad_μθ if wrt_hypers else self.grad_μx

    def std_gradient(self, wrt_hypers=False):
        return self.σ_grad_μθ if wrt_hypers else self.σ_grad_μx

    @classmethod
    def from_row(cls, row, d, with_gradient=True):
        row = np.asarray(row, dtype=np.float64)
        if not with_gradient:
            return cls(float(row[0]), float(row[1]))
        return cls(float(row[0]), float(row[1]), row[2:2 + d].copy(), row[2 + d:2 + 2 * d].copy(),
                   row[2 + 2 * d:3 + 2 * d].copy(), row[3 + 2 * d:4 + 2 * d].copy())

    def __repr__(self):
        return f"ExpectedTrajectoryOutput(μxθ={self.μxθ}, σ_μxθ={self.σ_μxθ}, grad_μx={self.grad_μx})"
