"""Between-step surrogate maintenance: marginal likelihood and its maximisation.

Mirrors radial_basis_surrogates.jl:
  log_likelihood(s)       :770-776
  ∇log_likelihood(s)      :787-799 (δlog_likelihood :778-785, eval_Dθ_KXX radial_basis_functions.jl:264-284)
  optimize!(s; lowerbounds, upperbounds, optim_options=Optim.Options(iterations=30))  :805-829
The likelihood and its lengthscale derivative are evaluated on the GPU (mrbo_gp_fit: one
workgroup per candidate lengthscale, refit K → L → c on device).  The outer minimiser of
−log_likelihood is build-defined: the reference's Fminbox(LBFGS()) lives in Optim.jl, absent
and unpinned here, so `optimize` runs a deterministic projected L-BFGS with a batched
backtracking line search (all trial step lengths evaluated in one launch); both reach the
box-constrained stationary point of the same objective from the same start.
"""
import ctypes

import numpy as np

from . import _lib

# the trial step lengths of one line search, evaluated together
_STEPS = 0.5 ** np.arange(12)


def _nt(s):
    """Hyperparameters of the kernel: (ℓ), or (ℓ, p) for Periodic (radial_basis_functions.jl:98-103)."""
    return len(s.ψ.θ)


def gp_fit_batch(s, thetas, want_fit=False):
    """Refit the base GP of `s` at each hyperparameter vector on the device (mrbo_gp_fit_theta).

    `thetas` is (P,) -- lengthscales -- or (P, nt) with nt = len(s.ψ.θ).  Returns dict(ll, grad
    (P, nt), dll (= grad[:, 0]), status[, L (N×N×P), c (N×P)]); status 1 = PosDefException."""
    L = _lib.load()
    th = np.asarray(thetas, dtype=np.float64)
    th = np.ascontiguousarray(th.reshape(th.shape[0], -1) if th.ndim > 1 else th.reshape(-1, 1))
    P, nt = th.shape
    n = s.observed
    X = np.asfortranarray(s.X[:, :n])
    y = np.ascontiguousarray(s.y[:n])
    dp = ctypes.POINTER(ctypes.c_double)
    sd = _lib.SurrogateDesc(X.shape[0], n, int(s.ψ.kind), float(s.ψ.lengthscale), float(s.σn2), float(s.fmini()),
                            X.ctypes.data_as(dp), None, n, None, y.ctypes.data_as(dp), float(s.ψ.period))
    ll, grad = np.zeros(P), np.zeros((P, nt))
    st = np.zeros(P, dtype=np.int32)
    Lo = np.zeros((n, n, P), order="F") if want_fit else None
    co = np.zeros((n, P), order="F") if want_fit else None
    vp = lambda a: ctypes.c_void_p(a.ctypes.data) if a is not None else None
    _lib.check(L.mrbo_gp_fit_theta(ctypes.byref(sd), P, nt, vp(th), vp(ll), vp(grad), vp(st), vp(Lo), vp(co),
                                   _lib.MRBO_FLAG_HOST_POINTERS, None))
    out = dict(ll=ll, grad=grad, dll=grad[:, 0].copy(), status=st)
    if want_fit:
        out["L"], out["c"] = Lo, co
    return out


def log_likelihood(s):
    """log_likelihood(s) at the surrogate's current hyperparameters (radial_basis_surrogates.jl:770-776)."""
    r = gp_fit_batch(s, s.ψ.θ[None, :])
    if r["status"][0]:
        raise np.linalg.LinAlgError("PosDefException (cholesky of K)")
    return float(r["ll"][0])


def grad_log_likelihood(s):
    """∇log_likelihood(s) (radial_basis_surrogates.jl:787-799): ∂/∂θ_t for every kernel hyperparameter."""
    r = gp_fit_batch(s, s.ψ.θ[None, :])
    if r["status"][0]:
        raise np.linalg.LinAlgError("PosDefException (cholesky of K)")
    return r["grad"][0].copy()


def projected_lbfgs(fg_batch, x0, lower, upper, iterations=30, g_tol=1e-8, m=10, c1=1e-4):
    """Minimise f over the box [lower, upper] from x0.

    fg_batch(X) takes a (P, n) array of points and returns (f (P,), g (P, n)); a point where f
    cannot be evaluated returns f = NaN.  Each iteration: L-BFGS direction on the free
    variables (bounds active with an outward gradient are fixed), then the first step length
    of 1, 1/2, ..., 1/2048 along the projected path meeting the Armijo condition -- all
    lengths evaluated in one batch.  Returns (x, f, g, iterations)."""
    lo, hi = np.asarray(lower, float), np.asarray(upper, float)
    x = np.clip(np.asarray(x0, float), lo, hi)
    f, g = fg_batch(x[None])
    f, g = float(f[0]), g[0]
    S, Y = [], []
    it = 0
    for it in range(1, iterations + 1):
        free = ~(((x <= lo) & (g > 0)) | ((x >= hi) & (g < 0)))
        if not free.any() or np.max(np.abs(g[free])) <= g_tol:
            it -= 1
            break
        # two-loop recursion on the free variables
        q = np.where(free, g, 0.0)
        al = []
        for s_, y_ in reversed(list(zip(S, Y))):
            a = (s_ @ q) / (y_ @ s_)
            al.append(a)
            q = q - a * y_
        if S:
            q = q * ((S[-1] @ Y[-1]) / (Y[-1] @ Y[-1]))
        else:
            q = q / max(np.max(np.abs(q)), 1.0)     # first step: at most unit length
        for (s_, y_), a in zip(zip(S, Y), reversed(al)):
            b = (y_ @ q) / (y_ @ s_)
            q = q + (a - b) * s_
        p = -np.where(free, q, 0.0)
        if g @ p >= 0:                                # not a descent direction: steepest descent
            p = -np.where(free, g, 0.0)
        trial = np.clip(x[None] + _STEPS[:, None] * p[None], lo, hi)
        ft, gt = fg_batch(trial)
        ok = np.isfinite(ft) & (ft <= f + c1 * ((trial - x[None]) @ g))
        if not ok.any():
            break
        k = int(np.argmax(ok))
        xn, fn, gn = trial[k], float(ft[k]), gt[k]
        sk, yk = xn - x, gn - g
        if sk @ yk > 1e-12 * max(np.linalg.norm(sk) * np.linalg.norm(yk), 1e-300):
            S.append(sk)
            Y.append(yk)
            if len(S) > m:
                S.pop(0)
                Y.pop(0)
        moved = np.max(np.abs(sk))
        x, f, g = xn, fn, gn
        if moved == 0.0:
            break
    return x, f, g, it


def optimize(s, lowerbounds, upperbounds, iterations=30):
    """optimize!(s; lowerbounds, upperbounds) (radial_basis_surrogates.jl:805-829): maximise the
    log likelihood over the kernel hyperparameters (ℓ; Periodic ℓ and p) within the box, then
    set_kernel! at the optimum."""
    def fg(T):
        r = gp_fit_batch(s, T)
        f = np.where(r["status"] == 0, -r["ll"], np.nan)
        return f, -r["grad"]

    θ, f, g, it = projected_lbfgs(fg, s.ψ.θ.copy(), lowerbounds, upperbounds, iterations)
    from .kernels import set_hyperparameters
    s.set_kernel(set_hyperparameters(s.ψ, θ))
    return dict(theta=θ, neg_log_likelihood=f, gradient=g, iterations=it)
