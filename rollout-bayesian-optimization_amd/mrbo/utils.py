"""Outer stochastic-gradient ascent and helpers -- mirror of utils.jl / low_discrepancy.jl."""
import numpy as np

from .engine import initial_guesses as _initial_guesses
from .trajectory import gen_low_discrepancy_sequence  # noqa: F401  (re-export, utils.jl:65-74)


def kronecker_quasirand(d, N, start=0):
    """low_discrepancy.jl:7-28"""
    ϕ = 1.0 + 1.0 / d
    for _ in range(10):
        g = ϕ ** (d + 1) - ϕ - 1
        dg = (d + 1) * ϕ ** d - 1
        ϕ -= g / dg
    αs = np.array([np.mod(1.0 / ϕ ** j, 1.0) for j in range(1, d + 1)])
    Z = np.zeros((d, N))
    for j in range(1, N + 1):
        Z[:, j - 1] = np.mod(0.5 + (start + j) * αs, 1.0)
    return Z


def generate_initial_guesses(N, lbs, ubs):
    """utils.jl:145-153: N Sobol points in [lbs, ubs] plus lbs+1e-6 and ubs-1e-6."""
    return _initial_guesses(N, lbs, ubs)


def generate_batch(N, lbs, ubs, ϵinterior=1e-2):
    """utils.jl:97-106"""
    B = _initial_guesses(N, lbs, ubs)
    B[:, N] = np.asarray(lbs, dtype=np.float64) + ϵinterior
    B[:, N + 1] = np.asarray(ubs, dtype=np.float64) - ϵinterior
    return B


def generate_indices(num_nodes, max_depth):
    """utils.jl:217-221: every node-index vector of length max_depth, in Julia's
    `collect(product(fill(1:n, depth)...))` order (first position fastest); 0-based."""
    import itertools
    return [tuple(reversed(p)) for p in itertools.product(range(num_nodes), repeat=max_depth)]


def gauss_hermite(n):
    """Physicists' Gauss–Hermite rule: ∫ e^{−t²} f(t) dt ≈ Σ w_i f(t_i) (the √2 / √π scalings of
    GaussHermiteObservable, observables.jl:58-72, assume this rule)."""
    return np.polynomial.hermite.hermgauss(n)


class GaussHermiteObservable:
    """observables.jl:32-81 — host-side description of the sampler; the device kernel computes the
    observations (y = μ + √2σt, ∇y = ∇μ + √2∇σt) and weighted resolutions."""

    def __init__(self, nodes, weights, max_invocations):
        self.nodes = np.array(nodes, dtype=np.float64)
        self.weights = np.array(weights, dtype=np.float64)
        self.trajectory_length = int(max_invocations)

    def set_nodes(self, nodes):
        self.nodes[:] = nodes

    def set_weights(self, weights):
        self.weights[:] = weights


def early_stopping_without_a_validation_set(grad_f, var_grad_f, sample_size):
    """utils.jl:114-123 (Mahsereci et al.); NaN ratios keep iterating, as in Julia."""
    grad_f = np.asarray(grad_f, dtype=np.float64)
    with np.errstate(divide="ignore", invalid="ignore"):
        ratio = np.sum((grad_f ** 2) / np.asarray(var_grad_f, dtype=np.float64))
    return bool((1.0 - (sample_size / grad_f.size) * ratio) > 0.0)


eswavs = early_stopping_without_a_validation_set


def sga_step_batch(x0, active, grad, std_grad, sample_size, eta, lbs=None, ubs=None, clip=False):
    """One outer step of R restarts at once (columns of x0, d×R), in place: eswavs per restart
    (utils.jl:114-123) retires the restarts it stops, then StandardSGA.update! (optimizers.jl:16-22)
    x += η·∇ for the rest -- per column exactly the arithmetic of eswavs and StandardSGA (NaN ratios
    keep iterating), without a Python loop over restarts.  The reference does not clip x to the
    box; clip=True (build-defined, off by default) projects onto [lbs, ubs] after the step."""
    d = x0.shape[0]
    with np.errstate(divide="ignore", invalid="ignore"):
        ratio = np.sum(grad ** 2 / std_grad ** 2, axis=0)
    active &= ~((1.0 - (sample_size / d) * ratio) > 0.0)
    if active.any():
        x0[:, active] = x0[:, active] + eta * grad[:, active]
        if clip:
            x0[:, active] = np.clip(x0[:, active], np.asarray(lbs)[:, None], np.asarray(ubs)[:, None])
    return x0, active


def adam_step_batch(x0, active, m, v, t, grad, std_grad, sample_size, eta=0.001, beta1=0.9, beta2=0.999, eps=1e-8):
    """sga_step_batch with Adam update! (optimizers.jl:49-74) in place of StandardSGA, in place on
    x0, m, v (d×R) and active: t is the update count of the active restarts (1 on the first
    update; a stopped restart never updates again, so they share it).  Per column exactly the
    arithmetic of mrbo.optimizers.Adam.update."""
    d = x0.shape[0]
    with np.errstate(divide="ignore", invalid="ignore"):
        ratio = np.sum(grad ** 2 / std_grad ** 2, axis=0)
    active &= ~((1.0 - (sample_size / d) * ratio) > 0.0)
    if active.any():
        g = grad[:, active]
        m[:, active] = beta1 * m[:, active] + (1 - beta1) * g
        v[:, active] = beta2 * v[:, active] + (1 - beta2) * g ** 2
        m_hat = m[:, active] / (1 - beta1 ** t)
        v_hat = v[:, active] / (1 - beta2 ** t)
        x0[:, active] = x0[:, active] + eta * m_hat / (np.sqrt(v_hat) + eps)
    return x0, active


class ExperimentSetup:
    """utils.jl:174-208"""

    def __init__(self, tp, number_of_starts):
        lbs, ubs = tp.get_spatial_bounds()
        self.tp = tp
        self.inner_solve_xstarts = generate_initial_guesses(number_of_starts, lbs, ubs)
        self.resolutions = np.zeros(tp.mc_iters)
        self.spatial_gradients_container = np.zeros((tp.x0.size, tp.mc_iters))
        self.hyperparameter_gradients_container = np.zeros((tp.θ.size, tp.mc_iters))

    def get_container(self, symbol):
        return {"f": self.resolutions, "grad_f": self.spatial_gradients_container,
                "grad_hypers": self.hyperparameter_gradients_container}[symbol]

    def get_starts(self):
        return self.inner_solve_xstarts


def gap(initial_best, observed_best, actual_best):
    """utils.jl:126-128"""
    return (initial_best - observed_best) / (initial_best - actual_best)


def simple_regret(actual_minimum, observation):
    """utils.jl:143"""
    return observation - actual_minimum


def stochastic_solve(optimizer, surrogate, tp, es, start, T=None, iterations=50, device=0, **opts):
    """utils.jl:235-265 for one start (the intended callee simulate_trajectory_mc)."""
    x, _ = stochastic_solve_batch([optimizer], surrogate, tp, es, np.asarray(start, dtype=np.float64).reshape(-1, 1),
                                  T=T, iterations=iterations, device=device, **opts)
    return x[:, 0]


def stochastic_solve_batch(optimizers, surrogate, tp, es, starts, T=None, iterations=50, device=0, **opts):
    """R restarts of the outer ascent at once: one batched rollout launch per SGA iteration;
    each restart keeps its own optimizer state and eswavs stop flag."""
    from .rollout import simulate_trajectory_mc_batch
    from .surrogates import FantasySurrogate
    from .trajectory import Trajectory
    x = np.array(starts, dtype=np.float64)
    d, R = x.shape
    if T is None:
        T = Trajectory(surrogate, FantasySurrogate(surrogate, tp.horizon), start=x[:, 0], hypers=tp.θ,
                       horizon=tp.horizon)
    active = np.ones(R, dtype=bool)
    history = []
    for _ in range(iterations):
        if not active.any():
            break
        br = simulate_trajectory_mc_batch(T, tp, x, es.get_starts(), device=device, **opts)
        etos = br.etos()
        history.append(etos)
        for r in range(R):
            if not active[r]:
                continue
            e = etos[r]
            if eswavs(e.gradient(), e.std_gradient() ** 2, tp.mc_iters):
                active[r] = False
                continue
            optimizers[r].update(x[:, r], e.gradient())
    return x, history
