"""Python mirror of the Julia drop-in's call sequence (julia/MRBO.jl).

julia is absent from this image, so MRBO.jl cannot execute here.  This module makes the same
C-ABI calls in the same order with the same arguments, so that the GPU tests and tools/shim_rate.py
measure and check what the Julia shim does:
  * plans come from a bounded cache keyed by the surrogate's identity and state, the trajectory
    parameters, θ, the start count, M, R and the device (MRBO.jl mrbo_cached_plan); eviction and
    release_plans() destroy them deterministically (mrbo_plan_destroy);
  * simulate_trajectory_mc: ONE x0 (R = 1), host arrays passed with MRBO_FLAG_HOST_POINTERS, the
    status check, then the ExpectedTrajectoryOutput reductions on the host (MRBO.jl mrbo_eto, the
    reference's rollout.jl:328-339);
  * simulate_trajectory_mc_batch: the batched method, the columns of X0 in one launch;
  * stochastic_solve: utils.jl:235-265 (50 iterations, eswavs, StandardSGA update!) driving the
    R = 1 method, i.e. the reference's own outer loop on the drop-in;
  * stochastic_solve_batch: MRBO.jl's device-resident method of that loop -- the whole ascent of
    a restart batch in ONE mrbo_stochastic_solve call on one cached plan.
There is no CPU path: every call goes through libmrbo.so on the GPU.
"""
import ctypes
import hashlib

import numpy as np

from . import _lib
from .engine import RolloutPlan
from .trajectory import ExpectedTrajectoryOutput

PLAN_CACHE_MAX = 8
_PLAN_CACHE = {}
stats = dict(plans_created=0, launches=0)


def release_plans():
    """mrbo_release_plans!(): destroy every cached plan now."""
    for p in _PLAN_CACHE.values():
        p.close()
    _PLAN_CACHE.clear()


def _digest(a):
    """hash(x) of MRBO.jl's key: the bytes of the array's active part."""
    return hashlib.blake2b(np.ascontiguousarray(a, dtype=np.float64).tobytes(), digest_size=16).hexdigest()


def _key(s, tp, theta, nstarts, device, M, R):
    """mrbo_plan_key (MRBO.jl): the surrogate's identity AND the hashes of its active covariates,
    observations and Cholesky factor and of every observation (fmini, Q3), so that a surrogate
    freed and replaced by another at the same id() -- CPython reuses ids -- never meets a stale plan."""
    lbs, ubs = tp.get_spatial_bounds()
    n = s.observed
    return (id(s), s.version, n, _digest(s.X[:, :n]), _digest(s.y[:n]), _digest(s.L[:n, :n]), _digest(s.y),
            float(s.σn2), tp.horizon, tuple(np.asarray(lbs).ravel()), tuple(np.asarray(ubs).ravel()),
            float(theta), int(nstarts), int(M), int(R), int(device), s.get_decision_rule().rule_id,
            float(s.ψ.lengthscale), float(s.ψ.period))


def cached_plan(s, tp, theta, nstarts, device=0, M=None, R=1):
    """mrbo_cached_plan (MRBO.jl): the plan for this surrogate state and parameter set, built once."""
    M = tp.mc_iters if M is None else M
    key = _key(s, tp, theta, nstarts, device, M, R)
    p = _PLAN_CACHE.get(key)
    if p is not None:
        return p
    if len(_PLAN_CACHE) >= PLAN_CACHE_MAX:
        release_plans()
    n = s.observed
    lbs, ubs = tp.get_spatial_bounds()
    g = s.get_decision_rule()
    # MRBO.jl's MrboPlan: max_iters 50, max_ls 20, x/f tol 1e-3, g_tol 1e-8, htol 1e-4, σtol 1e-8, seed 1906
    p = RolloutPlan(s.X[:, :n], s.L[:n, :n], s.c[:n], s.y[:n], s.ψ.kind, s.ψ.lengthscale, s.σn2, s.fmini(),
                    tp.horizon, M, R, nstarts, lbs, ubs, theta, device=device, period=s.ψ.period,
                    rule=g.rule_id, max_iters=50, max_ls=20, x_tol=1e-3, f_tol=1e-3, g_tol=1e-8, htol=1e-4,
                    sigma_tol=1e-8, seed=1906)
    stats["plans_created"] += 1
    _PLAN_CACHE[key] = p
    return p


def _eto(resolutions, gx, gt):
    """MRBO.jl mrbo_eto = rollout.jl:328-339: mean and n−1 std over the samples."""
    mu = float(np.mean(resolutions))
    sd = float(np.std(resolutions, ddof=1))
    if gx is None:
        return ExpectedTrajectoryOutput(mu, sd)
    gm = gx.mean(axis=1)
    gs = gx.std(axis=1, ddof=1)
    tm = gt.mean(axis=1)
    ts = gt.std(axis=1, ddof=1)
    return ExpectedTrajectoryOutput(mu, sd, gm, gs, tm, ts)


def _launch(plan, x0, rn, xs, vals, gx, gt, status):
    pv = lambda a: None if a is None else ctypes.c_void_p(a.ctypes.data)
    flags = _lib.MRBO_FLAG_HOST_POINTERS | (0 if gx is not None else _lib.MRBO_FLAG_NO_GRADIENT)
    _lib.check(plan.lib.mrbo_simulate_mc(plan.handle, pv(x0), pv(rn), pv(xs), None, None, pv(vals), pv(gx), pv(gt),
                                         pv(status), None, None, None, flags, None))
    stats["launches"] += 1


def _raise(status):
    bad = np.asarray(status) != 0
    if bad.any():
        raise RuntimeError(f"rollout failed on {int(bad.sum())} trajectories "
                           f"(status bits {int(np.bitwise_or.reduce(np.asarray(status)[bad]))})")


def simulate_trajectory_mc(T, tp, inner_solve_xstarts, resolutions, spatial_gradients_container=None,
                           hyperparameter_gradients_container=None, device=0):
    """MRBO.jl simulate_trajectory_mc(T, tp, ::MrboBackend; …): one x0, host pointers, cached plan."""
    T.set_start(tp.get_starting_point())
    xs = np.asfortranarray(inner_solve_xstarts, dtype=np.float64)
    plan = cached_plan(T.s, tp, T.θ[0], xs.shape[1], device=device)
    with_grad = spatial_gradients_container is not None and hyperparameter_gradients_container is not None
    x0 = np.array(T.x0, dtype=np.float64)
    rn = np.asfortranarray(tp.rnstream_sequence, dtype=np.float64)
    status = np.zeros(tp.mc_iters, dtype=np.int32)
    vals = np.zeros(tp.mc_iters)
    gx = np.zeros((x0.size, tp.mc_iters), order="F") if with_grad else None
    gt = np.zeros((1, tp.mc_iters), order="F") if with_grad else None
    _launch(plan, x0, rn, xs, vals, gx, gt, status)
    _raise(status)
    resolutions[:] = vals
    if with_grad:
        spatial_gradients_container[:, :] = gx
        hyperparameter_gradients_container[:, :] = gt
    return _eto(vals, gx, gt)


def simulate_trajectory_mc_batch(T, tp, X0, inner_solve_xstarts, with_gradient=True, device=0):
    """MRBO.jl batched method: the columns of X0 in one launch.  Returns (list of ETOs, values M×R,
    grad_x d×M×R or None, grad_theta 1×M×R or None)."""
    X0 = np.asfortranarray(X0, dtype=np.float64)
    d, R = X0.shape
    M = tp.mc_iters
    xs = np.asfortranarray(inner_solve_xstarts, dtype=np.float64)
    plan = cached_plan(T.s, tp, T.θ[0], xs.shape[1], device=device, R=R)
    rn = np.asfortranarray(tp.rnstream_sequence, dtype=np.float64)
    vals = np.zeros((M, R), order="F")
    status = np.zeros((M, R), dtype=np.int32, order="F")
    gx = np.zeros((d, M, R), order="F") if with_gradient else None
    gt = np.zeros((1, M, R), order="F") if with_gradient else None
    _launch(plan, X0, rn, xs, vals, gx, gt, status)
    _raise(status)
    # per restart exactly the R = 1 method's reductions (_eto), so that the two call sequences agree
    # bit for bit (numpy's axis reductions may sum in another order)
    etos = [_eto(vals[:, r], None if gx is None else gx[:, :, r], None if gt is None else gt[:, :, r])
            for r in range(R)]
    return etos, vals, gx, gt


def eswavs(grad, var_grad, sample_size):
    """utils.jl:114-123 early stopping without a validation set."""
    d = grad.size
    with np.errstate(divide="ignore", invalid="ignore"):
        ratio = np.sum(grad ** 2 / var_grad)
    return bool((1.0 - (sample_size / d) * ratio) > 0.0)


def stochastic_solve(T, tp, xstarts, start, eta=0.01, iterations=50, device=0, trace=None):
    """utils.jl:235-265 on the drop-in: up to 50 R = 1 calls of simulate_trajectory_mc at the moving
    x0, eswavs stop, StandardSGA update! x += η∇ (optimizers.jl:16-22).  trace (a list) receives
    every call's per-trajectory (values, grad_x) for bitwise comparisons."""
    x = np.array(start, dtype=np.float64)
    d, M = x.size, tp.mc_iters
    res = np.zeros(M)
    gx = np.zeros((d, M), order="F")
    gt = np.zeros((1, M), order="F")
    for _ in range(iterations):
        tp.set_starting_point(x.copy())
        eto = simulate_trajectory_mc(T, tp, xstarts, res, gx, gt, device=device)
        if trace is not None:
            trace.append((res.copy(), gx.copy()))
        if eswavs(eto.gradient(), eto.std_gradient() ** 2, M):
            break
        x = x + eta * eto.gradient()
    return x


def stochastic_solve_batch(T, tp, xstarts, starts, optimizer="sga", eta=None, iterations=50, device=0):
    """MRBO.jl stochastic_solve(backend::MrboBackend; optimizer, surrogate, tp, es, starts): the
    reference's outer loop (utils.jl:235-265) for every column of `starts` (d×R, e.g. the
    generate_batch points) in ONE C-ABI call -- up to `iterations` × (launch, ETO, eswavs +
    update!) on the device on one cached plan, host arrays staged once.  Returns (X d×R: every
    restart's get_starting_point(tpc), eto R×W: its final ETO rows (mrbo_eto_reduce's layout),
    active R: 1 where eswavs never stopped it, result: [iterations launched, iteration after which
    no restart was active, status bits])."""
    X = np.array(starts, dtype=np.float64, order="F")
    d, R = X.shape
    xs = np.asfortranarray(xstarts, dtype=np.float64)
    plan = cached_plan(T.s, tp, T.θ[0], xs.shape[1], device=device, R=R)
    rn = np.asfortranarray(tp.rnstream_sequence, dtype=np.float64)
    W = 2 + 2 * d + 2
    eto = np.zeros((R, W))
    active = np.zeros(R, dtype=np.int32)
    opt = _lib.MRBO_OPT_SGA if optimizer == "sga" else _lib.MRBO_OPT_ADAM
    eta = (0.01 if opt == _lib.MRBO_OPT_SGA else 0.001) if eta is None else eta
    o = _lib.SolveOpts(opt, int(iterations), float(eta), 0.9, 0.999, 1e-8, 0.0)
    res = (ctypes.c_int32 * 3)()
    pv = lambda a: ctypes.c_void_p(a.ctypes.data)
    _lib.check(plan.lib.mrbo_stochastic_solve(plan.handle, pv(X), pv(rn), pv(xs), None, ctypes.byref(o), pv(eto),
                                              pv(active), res, _lib.MRBO_FLAG_HOST_POINTERS, None))
    stats["launches"] += int(res[0])
    if res[2]:
        raise RuntimeError(f"rollout failed during the ascent (status bits {int(res[2])})")
    return X, eto, active, [int(v) for v in res]
