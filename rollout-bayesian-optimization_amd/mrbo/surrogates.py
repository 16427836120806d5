"""Surrogate / FantasySurrogate -- host mirror of radial_basis_surrogates.jl.

The base ``Surrogate`` keeps the reference's preallocated, zero-padded buffers
(radial_basis_surrogates.jl:77-118) because ``fmini`` for the rollout is the minimum over the
whole capacity buffer (Q3).  Between-BO-step maintenance (condition!, reset!, set_kernel!) is
host bookkeeping; evaluation on the rollout path goes to libmrbo.so.
"""
import numpy as np

from .decision_rules import EI
from .kernels import eval_KXX, eval_KxX

DEFAULT_CAPACITY = 100          # constants.jl:13
GROUND_TRUTH_OBSERVATIONS = -1  # constants.jl:7


class Surrogate:
    """radial_basis_surrogates.jl:30-41, constructor :77-118."""

    def __init__(self, ψ, X, y, capacity=DEFAULT_CAPACITY, decision_rule=None, σn2=1e-6):
        X = np.asarray(X, dtype=np.float64)
        y = np.asarray(y, dtype=np.float64).ravel()
        assert y.size <= capacity, "Capacity must be >= number of observations."
        d, N = X.shape
        self.ψ = ψ
        self.σn2 = float(σn2)
        self.g = decision_rule if decision_rule is not None else EI()
        self.capacity = int(capacity)
        self.X = np.zeros((d, capacity))
        self.K = np.zeros((capacity, capacity))
        self.L = np.zeros((capacity, capacity))
        self.y = np.zeros(capacity)
        self.c = np.zeros(capacity)
        self.observed = 0
        self.version = 0
        self._fit(X, y)

    def _fit(self, X, y):
        d, N = X.shape
        self.X[:, :N] = X
        self.K[:N, :N] = eval_KXX(self.ψ, X, σn2=self.σn2)
        self.L[:N, :N] = np.linalg.cholesky(self.K[:N, :N])
        self.c[:N] = np.linalg.solve(self.L[:N, :N].T, np.linalg.solve(self.L[:N, :N], y))
        self.y[:N] = y
        self.observed = N
        self.version += 1

    # accessors (radial_basis_surrogates.jl:17-57)
    def get_observed(self):
        return self.observed

    def get_capacity(self):
        return self.capacity

    def get_active_covariates(self):
        return self.X[:, : self.observed]

    def get_active_cholesky(self):
        return self.L[: self.observed, : self.observed]

    def get_active_observations(self):
        return self.y[: self.observed]

    def get_active_coefficients(self):
        return self.c[: self.observed]

    def get_kernel(self):
        return self.ψ

    def get_decision_rule(self):
        return self.g

    def set_decision_rule(self, g):
        self.g = g

    # Q3 as the reference has it; False (build option, not the reference) takes the minimum over
    # the observed points only -- a diagnostic of the quirk's effect on positive objectives
    fmini_over_capacity = True

    def fmini(self):
        """minimum(get_observations(base)) over the zero-padded capacity buffer (rollout.jl:109, Q3)."""
        if not self.fmini_over_capacity:
            return float(np.min(self.y[:self.observed]))
        return float(np.min(self.y))

    def reset(self, X, y):
        """reset!(s, X, y) :147-164: refit on (X, y) with s's CURRENT kernel (a lengthscale set by
        an earlier optimize! carries over) and leave the buffers past N as they are (y[N+1:cap]
        keeps earlier observations, which fmini over the capacity buffer, Q3, then sees)."""
        self._fit(np.asarray(X, dtype=np.float64), np.asarray(y, dtype=np.float64).ravel())

    def set_kernel(self, kernel):
        """set_kernel!(s, kernel) :123-135"""
        self.ψ = kernel
        self._fit(self.get_active_covariates().copy(), self.get_active_observations().copy())

    def resize(self):
        """resize(s) :137-145: a NEW surrogate of twice the capacity refit on the whole buffers
        (get_covariates / get_observations, all `capacity` columns), with s's kernel and rule."""
        return Surrogate(self.ψ, self.X.copy(), self.y.copy(), capacity=2 * self.capacity, decision_rule=self.g,
                         σn2=self.σn2)

    def condition(self, xnew, ynew):
        """condition!(s, x, y) :214-222 (rank-1 Cholesky append, full coefficient re-solve).
        Returns the conditioned surrogate, like the reference.  On a full surrogate the reference
        rebinds its LOCAL `s = resize(s)` (:215) and conditions that new object: the caller's
        surrogate is left unchanged and the observation reaches only the returned copy (the loops
        of experiments/*_bayesopt.jl ignore the return value, so past capacity they stop learning).
        This mirror does the same."""
        if self.observed == self.capacity:
            return self.resize().condition(xnew, ynew)
        n = self.observed
        x = np.asarray(xnew, dtype=np.float64).ravel()
        self.X[:, n] = x
        self.y[n] = float(ynew)
        self.observed = n + 1
        kx = eval_KxX(self.ψ, x, self.X[:, :n])
        self.K[n, n] = self.ψ(0.0) + self.σn2
        self.K[n, :n] = kx
        self.K[:n, n] = kx
        L21 = np.linalg.solve(self.L[:n, :n], kx) if n > 0 else np.zeros(0)
        S = self.K[n, n] - L21 @ L21
        if not S > 0:
            raise np.linalg.LinAlgError("PosDefException (radial_basis_surrogates.jl:196)")
        self.L[n, :n] = L21
        self.L[n, n] = np.sqrt(S)
        Ln = self.L[: n + 1, : n + 1]
        self.c[: n + 1] = np.linalg.solve(Ln.T, np.linalg.solve(Ln, self.y[: n + 1]))
        self.version += 1
        return self

    def __call__(self, x, θ):
        """eval(s, x, θ) :224-310 -> SurrogateEval (computed on the GPU)."""
        from .rollout import evaluate_base
        return evaluate_base(self, np.asarray(x, dtype=np.float64).reshape(-1, 1), θ)[0]


class FantasySurrogate:
    """radial_basis_surrogates.jl:320-381.  The per-trajectory fantasy state (rank-1 appended
    rows, coefficient history) lives on the device, one copy per wavefront, and is reset for
    every trajectory (reset! :476-480); this host object only ties a base surrogate to h."""

    def __init__(self, s, horizon):
        self.s = s
        self.h = int(horizon)
        self.g = s.g
        self.observed = s.observed
        self.fantasies_observed = 0

    def get_known_observations(self):
        return self.observed

    def get_decision_rule(self):
        return self.g

    def set_decision_rule(self, g):
        self.g = g

    def update(self, s):
        """update!(fs, s) :453-473 -- re-point at the (conditioned) base surrogate."""
        self.s = s
        self.observed = s.observed
        self.fantasies_observed = 0

    def reset(self):
        self.fantasies_observed = 0


def get_observations(s):
    return s.y


def get_covariates(s):
    return s.X


def get_kernel(s):
    return s.ψ
