"""base_solve / multistart_base_solve! on the base surrogate -- mirror of rbf_optim.jl:35-135.

The myopic experiments (experiments/myopic_bayesopt.jl:224-248) choose xnext with
``multistart_base_solve!(sur, xnext; spatial_lbs, spatial_ubs, guesses, θfixed)``: a local solve of
−α from every column of ``guesses`` (generate_initial_guesses(64, …): 66 starts), NaN minimisers
dropped, ``findmin`` over the minima.  Here every start is one wavefront of ``mrbo_base_solve``
(the rollout kernel's inner solve on surface −1, the build's projected Newton of DESIGN.md §3 in
place of Optim.jl's IPNewton, which is absent and unpinned); the findmin runs on the host.
"""
import ctypes

import numpy as np

from . import _lib
from .engine import _torch, from_device, to_device
from .rollout import _plan_for


def base_solve_batch(surrogate, spatial_lbs, spatial_ubs, guesses, θfixed, device=0, **opts):
    """base_solve(s; xstart, θfixed) (rbf_optim.jl:35-66) from every column of `guesses` (d×n), all
    starts in one launch.  Returns (minimizers d×n, minima n, work counters NCOUNTERS×n); raises
    like the reference on a negative posterior variance (DomainError, radial_basis_surrogates.jl:528)."""
    torch = _torch()
    guesses = np.asarray(guesses, dtype=np.float64)
    if guesses.ndim == 1:
        guesses = guesses.reshape(-1, 1)
    d, n = guesses.shape
    theta = float(np.asarray(θfixed, dtype=np.float64).ravel()[0])
    plan = _plan_for(surrogate, 0, 1, 1, 1, spatial_lbs, spatial_ubs, theta, device, opts)
    dev = f"cuda:{device}"
    dxs = to_device(guesses, dev)
    xmin = torch.empty(d * n, dtype=torch.float64, device=dev)
    fmin = torch.empty(n, dtype=torch.float64, device=dev)
    status = torch.empty(n, dtype=torch.int32, device=dev)
    evals = torch.empty(_lib.NCOUNTERS * n, dtype=torch.int64, device=dev)
    st = torch.cuda.current_stream(device)
    p = lambda t: ctypes.c_void_p(t.data_ptr())
    _lib.check(plan.lib.mrbo_base_solve(plan.handle, n, p(dxs), p(xmin), p(fmin), p(status), p(evals), 0,
                                        ctypes.c_void_p(st.cuda_stream)))
    torch.cuda.synchronize(device)
    stv = from_device(status, (n,))
    if np.any(stv != 0):
        from .rollout import raise_on_status
        raise_on_status(stv)
    return from_device(xmin, (d, n)), from_device(fmin, (n,)), from_device(evals, (_lib.NCOUNTERS, n))


def findmin_candidates(xs, fs):
    """multistart_base_solve!'s selection (rbf_optim.jl:129-131): drop candidates whose minimiser has a
    NaN, then findmin over the minima (a NaN minimum sorts first, else the first minimum wins).
    Returns the index of the chosen start; raises ArgumentError's analogue on an empty list."""
    keep = [i for i in range(xs.shape[1]) if not np.any(np.isnan(xs[:, i]))]
    if not keep:
        raise ValueError("findmin over an empty candidate list (rbf_optim.jl:130)")
    best = keep[0]
    for i in keep[1:]:
        fi, fb = fs[i], fs[best]
        if np.isnan(fb):
            break
        if np.isnan(fi) or fi < fb:
            best = i
    return best


def multistart_base_solve(surrogate, xfinal, spatial_lbs, spatial_ubs, guesses, θfixed, device=0, **opts):
    """multistart_base_solve!(s::Surrogate, xfinal; spatial_lbs, spatial_ubs, guesses, θfixed)
    (rbf_optim.jl:103-135): xfinal is overwritten with the best local minimiser of −α; returns None
    as the reference does.  The Random rule draws uniformly in the box (:110-113)."""
    if surrogate.get_decision_rule().name == "Random":
        lb, ub = np.asarray(spatial_lbs, float), np.asarray(spatial_ubs, float)
        xfinal[:] = lb + (ub - lb) * np.random.random(lb.size)
        return None
    xs, fs, _ = base_solve_batch(surrogate, spatial_lbs, spatial_ubs, guesses, θfixed, device=device, **opts)
    xfinal[:] = xs[:, findmin_candidates(xs, fs)]
    return None
