"""simulate_trajectory_mc -- mirror of rollout.jl:279-340, running on libmrbo.so.

``simulate_trajectory_mc(T, tp; inner_solve_xstarts, resolutions, spatial_gradients_container,
hyperparameter_gradients_container)`` keeps the reference signature (one start point, M
samples, caller-owned containers overwritten in place, ExpectedTrajectoryOutput returned).
``simulate_trajectory_mc_batch`` is the MI355X-shaped entry: R restarts × M samples in one
launch, outputs left on the device.
"""
import numpy as np

from . import _lib
from .engine import RolloutPlan, from_device, to_device
from .trajectory import ExpectedTrajectoryOutput

_PLANS = {}


def _plan_for(s, h, M, R, nstarts, lbs, ubs, theta, device, opts):
    g = s.get_decision_rule()
    opts = dict(opts)
    opts.setdefault("rule", g.rule_id)       # the surrogate's base decision rule (Q12: T.θ)
    opts.setdefault("sigma_tol", g.σtol)
    key = (id(s), s.version, h, M, R, nstarts, tuple(np.asarray(lbs).ravel()), tuple(np.asarray(ubs).ravel()),
           float(theta), device, tuple(sorted(opts.items())))
    p = _PLANS.get(key)
    if p is None:
        n = s.observed
        p = RolloutPlan(s.X[:, :n], s.L[:n, :n], s.c[:n], s.y[:n], s.ψ.kind, s.ψ.lengthscale, s.σn2, s.fmini(),
                        h, M, R, nstarts, lbs, ubs, theta, device=device, period=s.ψ.period, **opts)
        if len(_PLANS) > 16:
            _PLANS.clear()
        _PLANS[key] = p
    return p


def raise_on_status(status):
    st = np.asarray(status)
    bad = st[st != 0]
    if bad.size:
        bits = int(np.bitwise_or.reduce(bad))
        msgs = [m for b, m in _lib.STATUS_BITS.items() if bits & b]
        raise FloatingPointError(f"{bad.size} trajectories failed: " + "; ".join(msgs))


class BatchResult:
    """Device-resident outputs of one batched launch (flat, column-major)."""

    def __init__(self, plan, out, eto):
        self.plan = plan
        self.out = out
        self.eto_dev = eto

    def numpy(self):
        p = self.plan
        d, M, R, h = p.d, p.M, p.R, p.h
        o = self.out
        res = dict(values=from_device(o["values"], (M, R)), status=from_device(o["status"], (M, R)))
        if "grad_x" in o:
            res["grad_x"] = from_device(o["grad_x"], (d, M, R))
            res["grad_theta"] = from_device(o["grad_theta"], (1, M, R))
        if "policy_x" in o:
            res["policy_x"] = from_device(o["policy_x"], (d, h + 1, M, R))
        if "obs" in o:
            res["obs"] = from_device(o["obs"], (h + 1, M, R))
        if "evals" in o:
            res["evals"] = from_device(o["evals"], (_lib.NCOUNTERS, M, R))
        if self.eto_dev is not None:
            res["eto"] = from_device(self.eto_dev, (2 + 2 * d + 2, R))
        return res

    def etos(self, with_gradient=True):
        e = from_device(self.eto_dev, (2 + 2 * self.plan.d + 2, self.plan.R))
        return [ExpectedTrajectoryOutput.from_row(e[:, r], self.plan.d, with_gradient) for r in range(self.plan.R)]


def simulate_trajectory_mc_batch(T, tp, x0s, inner_solve_xstarts, with_gradient=True, dual_y_dx=None, replay_x=None,
                                 want_policy=False, want_obs=False, device=0, rnstream=None, **opts):
    """R restarts (columns of x0s) × tp.mc_iters samples in one kernel launch."""
    import torch
    x0s = np.asarray(x0s, dtype=np.float64)
    if x0s.ndim == 1:
        x0s = x0s.reshape(-1, 1)
    d, R = x0s.shape
    lbs, ubs = tp.get_spatial_bounds()
    rn = tp.rnstream_sequence if rnstream is None else rnstream
    M = rn.shape[0]
    plan = _plan_for(T.s, tp.horizon, M, R, inner_solve_xstarts.shape[1], lbs, ubs, T.θ[0], device, opts)
    dev = f"cuda:{device}"
    dx0 = to_device(x0s, dev)
    drn = rn if isinstance(rn, torch.Tensor) else to_device(rn, dev)
    dxs = to_device(inner_solve_xstarts, dev)
    ddy = None if dual_y_dx is None else to_device(dual_y_dx, dev)
    drp = None if replay_x is None else to_device(replay_x, dev)
    out = plan.alloc_outputs(with_gradient=with_gradient, want_policy=want_policy, want_obs=want_obs)
    plan.simulate(dx0, drn, dxs, out, dual_y_dx=ddy, replay_x=drp)
    eto = plan.eto(out)
    return BatchResult(plan, out, eto)


def simulate_trajectory_mc(T, tp, inner_solve_xstarts, resolutions, spatial_gradients_container=None,
                           hyperparameter_gradients_container=None, device=0, **opts):
    """rollout.jl:279-340 (the reference signature; one start point tp.x0)."""
    T.set_start(tp.get_starting_point())  # set_start!(T, get_starting_point(tp)) :287  (T.θ kept, Q12)
    with_gradient = spatial_gradients_container is not None and hyperparameter_gradients_container is not None
    br = simulate_trajectory_mc_batch(T, tp, T.x0.reshape(-1, 1), np.asarray(inner_solve_xstarts),
                                      with_gradient=with_gradient, device=device, **opts)
    res = br.numpy()
    raise_on_status(res["status"])
    resolutions[:] = res["values"][:, 0]
    if with_gradient:
        spatial_gradients_container[:, :] = res["grad_x"][:, :, 0]
        hyperparameter_gradients_container[:, :] = res["grad_theta"][:, :, 0]
    return ExpectedTrajectoryOutput.from_row(res["eto"][:, 0], T.x0.size, with_gradient)


def ghq_node_arrays(nodes, weights, indices):
    """nodes[indices[m]], weights[indices[m]] as M×depth column-major arrays (the sampler state
    set_nodes!/set_weights! receives per sample, rollout.jl:431-432)."""
    idx = np.asarray([np.asarray(ix, dtype=np.int64) for ix in indices])
    nodes = np.asarray(nodes, dtype=np.float64)
    weights = np.asarray(weights, dtype=np.float64)
    return np.asfortranarray(nodes[idx]), np.asfortranarray(weights[idx])


def simulate_trajectory_ghq_batch(T, tp, x0s, inner_solve_xstarts, nodes, weights, indices, with_gradient=True,
                                  dual_y_dx=None, replay_x=None, want_policy=False, want_obs=False, device=0, **opts):
    """Gauss–Hermite estimator for R restarts (columns of x0s) × len(indices) node vectors."""
    x0s = np.asarray(x0s, dtype=np.float64)
    if x0s.ndim == 1:
        x0s = x0s.reshape(-1, 1)
    d, R = x0s.shape
    tn, tw = ghq_node_arrays(nodes, weights, indices)
    M, depth = tn.shape
    if depth != tp.horizon + 1:   # GaussHermiteObservable max_invocations (observables.jl:59 assertion)
        raise ValueError(f"node vectors of depth {depth}; the rollout observes horizon+1 = {tp.horizon + 1} times")
    lbs, ubs = tp.get_spatial_bounds()
    plan = _plan_for(T.s, tp.horizon, M, R, inner_solve_xstarts.shape[1], lbs, ubs, T.θ[0], device, opts)
    dev = f"cuda:{device}"
    out = plan.alloc_outputs(with_gradient=with_gradient, want_policy=want_policy, want_obs=want_obs)
    plan.simulate_ghq(to_device(x0s, dev), to_device(tn, dev), to_device(tw, dev), to_device(inner_solve_xstarts, dev),
                      out, dual_y_dx=None if dual_y_dx is None else to_device(dual_y_dx, dev),
                      replay_x=None if replay_x is None else to_device(replay_x, dev))
    return BatchResult(plan, out, plan.eto(out))


def simulate_trajectory_ghq(T, tp, inner_solve_xstarts, resolutions, nodes, weights, indices,
                            spatial_gradients_container=None, hyperparameter_gradients_container=None, device=0,
                            **opts):
    """rollout.jl:409-467 (the reference signature): ETO of the Gauss–Hermite resolutions, mean and
    n−1 std exactly as the Monte-Carlo version (:452-466)."""
    T.set_start(tp.get_starting_point())
    with_gradient = spatial_gradients_container is not None and hyperparameter_gradients_container is not None
    br = simulate_trajectory_ghq_batch(T, tp, T.x0.reshape(-1, 1), np.asarray(inner_solve_xstarts), nodes, weights,
                                       indices, with_gradient=with_gradient, device=device, **opts)
    res = br.numpy()
    raise_on_status(res["status"])
    resolutions[:] = res["values"][:, 0]
    if with_gradient:
        spatial_gradients_container[:, :] = res["grad_x"][:, :, 0]
        hyperparameter_gradients_container[:, :] = res["grad_theta"][:, :, 0]
    return ExpectedTrajectoryOutput.from_row(res["eto"][:, 0], T.x0.size, with_gradient)


class SurrogateEval:
    """The lazily-forced quantities of eval(s, x, θ) (radial_basis_surrogates.jl:224-310)."""

    def __init__(self, col, d):
        self.μ = float(col[0])
        self.σ = float(col[1])
        self.αxθ = float(col[2])
        self.grad_μ = col[3:3 + d].copy()
        self.grad_σ = col[3 + d:3 + 2 * d].copy()
        self.grad_αx = col[3 + 2 * d:3 + 3 * d].copy()
        self.Hαx = col[3 + 3 * d:3 + 3 * d + d * d].reshape((d, d), order="F").copy()
        self.d2α_dxdθ = col[3 + 3 * d + d * d:3 + 4 * d + d * d].copy()


def evaluate_base(s, xs, θ, device=0):
    xs = np.asarray(xs, dtype=np.float64)
    d = xs.shape[0]
    lb = np.zeros(d)
    plan = _plan_for(s, 0, 1, 1, 1, lb, lb + 1.0, float(np.asarray(θ).ravel()[0]), device, {})
    out = plan.eval_base(xs)
    return [SurrogateEval(out[:, j], d) for j in range(out.shape[1])]
