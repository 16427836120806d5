"""Between-step surrogate maintenance: log_likelihood, ∇log_likelihood and
optimize! (radial_basis_surrogates.jl:770-829).

CPU: the oracle's restatement against an independent NumPy/SciPy one and central finite
differences (the reference's FD methodology, runtests.jl:11-20), and the host minimiser driven
by the oracle.  GPU (marked): mrbo_gp_fit against the oracle, and optimize! on the device
against the same minimiser driven by the oracle.  Parity of the optimum with Optim.jl's
Fminbox(LBFGS()) is unpinned (Optim.jl absent); both target the same box-constrained
stationary point, which the tests check through its KKT conditions.
"""
import numpy as np
import pytest
from scipy.linalg import cho_factor, cho_solve

KERNELS = ["matern52", "matern32", "matern12", "se"]


def _psi(kernel, ell, rho):
    if kernel == "matern52":
        s = np.sqrt(5.0) / ell * rho
        return (1 + s + s * s / 3) * np.exp(-s)
    if kernel == "matern32":
        s = np.sqrt(3.0) / ell * rho
        return (1 + s) * np.exp(-s)
    if kernel == "matern12":
        return np.exp(-rho / ell)
    return np.exp(-rho * rho / (2 * ell * ell))


def _numpy_ll(X, y, kernel, ell, sn2, h=1e-5):
    """Independent restatement: K via SciPy's Cholesky; dll via the trace formula with δK from a
    central difference of ψ in ℓ."""
    rho = np.sqrt(((X[:, :, None] - X[:, None, :]) ** 2).sum(0))
    K = _psi(kernel, ell, rho) + sn2 * np.eye(len(y))
    cf = cho_factor(K, lower=True)
    c = cho_solve(cf, y)
    ll = -y @ c / 2 - np.log(np.diag(cf[0])).sum() - len(y) * np.log(2 * np.pi) / 2
    dK = (_psi(kernel, ell + h, rho) - _psi(kernel, ell - h, rho)) / (2 * h)
    np.fill_diagonal(dK, 0.0)
    dll = (c @ dK @ c - np.trace(cho_solve(cf, dK))) / 2
    return ll, dll


def _ll_tol(ll, L, c):
    """Tolerance of log_likelihood between two backward-stable factorisations: rel 1e-10, or
    where K is ill-conditioned the first-order perturbation of yᵀK⁻¹y/2 under a backward error
    ‖δK‖ = u·‖K‖₂ in each of them: u·‖K‖₂·‖c‖² (cᵀδK c, both sides).  At κ₂(K) ≈ 1e8 this is what
    separates them: against an extended-precision evaluation the oracle's own ll is off by up
    to 1.3e-10 relative there (test_oracle_loglik_vs_extended_precision)."""
    u = 2.0 ** -53
    return max(1e-10 * abs(ll), 1e-9, u * np.linalg.norm(L, 2) ** 2 * float(c @ c))


def _ll_extended(X, y, ell, sn2):
    """Matern52 log_likelihood in numpy long double (x87 extended: 64-bit significand), with the
    unblocked Cholesky and substitutions: the reference value the fp64 evaluations are held to."""
    ld = np.longdouble
    X, y = X.astype(ld), y.astype(ld)
    rho = np.sqrt(((X[:, :, None] - X[:, None, :]) ** 2).sum(0))
    sc = np.sqrt(ld(5)) / ld(ell) * rho
    A = (1 + sc + sc * sc / 3) * np.exp(-sc) + ld(sn2) * np.eye(len(y), dtype=ld)
    n = len(y)
    L = np.zeros_like(A)
    for j in range(n):
        L[j, j] = np.sqrt(A[j, j])
        L[j + 1:, j] = A[j + 1:, j] / L[j, j]
        A[j + 1:, j + 1:] -= np.outer(L[j + 1:, j], L[j + 1:, j])
    z = np.zeros(n, dtype=ld)
    for i in range(n):
        z[i] = (y[i] - L[i, :i] @ z[:i]) / L[i, i]
    c = np.zeros(n, dtype=ld)
    for i in reversed(range(n)):
        c[i] = (z[i] - L[i + 1:, i] @ c[i + 1:]) / L[i, i]
    return float(-y @ c / 2 - np.log(np.diag(L)).sum() - n * np.log(2 * np.pi) / 2)


def test_oracle_loglik_vs_extended_precision(oracle):
    """The oracle's log_likelihood against a long-double evaluation of the same formula
    (radial_basis_surrogates.jl:770-776) from well- to ill-conditioned K (κ₂ 3e3 .. 1.3e8): within
    the first-order bound _ll_tol uses for the GPU comparison."""
    X, y = _data(4, 128, seed=4)
    for ell in np.array([0.2, 0.5, 1.0, 2.0, 4.0]) * 2.0:
        ll, dll, L, c = oracle.log_likelihood(X, y, "matern52", ell, 1e-6, want_fit=True)
        ref = _ll_extended(X, y, ell, 1e-6)
        u = 2.0 ** -53
        assert abs(ll - ref) <= max(1e-12 * abs(ref), u * np.linalg.norm(L, 2) ** 2 * float(c @ c) / 2), (ell, ll, ref)


def _data(d, N, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.random((d, N))
    y = np.sin(3 * X.sum(0)) + 0.1 * rng.standard_normal(N)
    return X, y


# SE's K is numerically singular on 30 points in [0,1]³ beyond ℓ ≈ 1: keep its cases conditioned
@pytest.mark.parametrize("kernel,ell", [(k, e) for k in KERNELS[:3] for e in (0.3, 1.0, 2.5)] +
                         [("se", 0.1), ("se", 0.3), ("se", 0.6)])
def test_oracle_loglik_vs_numpy_and_fd(oracle, kernel, ell):
    X, y = _data(3, 30)
    ll, dll = oracle.log_likelihood(X, y, kernel, ell, 1e-6)
    ll_np, dll_np = _numpy_ll(X, y, kernel, ell, 1e-6)
    assert ll == pytest.approx(ll_np, rel=1e-9)
    assert dll == pytest.approx(dll_np, rel=1e-6, abs=1e-6)
    h = 1e-6 * ell
    fd = (oracle.log_likelihood(X, y, kernel, ell + h, 1e-6)[0] - oracle.log_likelihood(X, y, kernel, ell - h, 1e-6)[0]) / (2 * h)
    assert dll == pytest.approx(fd, rel=1e-6, abs=1e-6)


def test_oracle_loglik_posdef_failure(oracle):
    X, y = _data(2, 10)
    # σn2 = −1 zeroes the diagonal (ψ(0) = 1): the first pivot is 0 → PosDefException.  (A
    # duplicated point with σn2 = 0 leaves a pivot of ±rounding, passing or failing by order.)
    ll, dll = oracle.log_likelihood(X, y, "se", 0.5, -1.0)
    assert np.isnan(ll) and np.isnan(dll)


def _oracle_fg(oracle, X, y, kernel, sn2):
    def fg(T):
        r = [oracle.log_likelihood(X, y, kernel, float(t), sn2) for t in T[:, 0]]
        return np.array([-a for a, _ in r]), np.array([[-b] for _, b in r])
    return fg


def _assert_kkt(theta, g, lo, hi, tol):
    if theta <= lo:
        assert g >= -tol
    elif theta >= hi:
        assert g <= tol
    else:
        assert abs(g) <= tol


@pytest.mark.parametrize("kernel", KERNELS)
def test_projected_lbfgs_reaches_box_stationary_point(oracle, kernel):
    """optimize!'s objective −log_likelihood over ℓ ∈ [0.1, 5] (experiments/nonmyopic_bayesopt.jl:230)."""
    from mrbo.mle import projected_lbfgs
    X, y = _data(2, 25, seed=3)
    fg = _oracle_fg(oracle, X, y, kernel, 1e-6)
    θ, f, g, it = projected_lbfgs(fg, np.array([1.0]), [0.1], [5.0], iterations=60)
    _assert_kkt(θ[0], g[0], 0.1, 5.0, 1e-5 * max(1.0, abs(f)))
    # no better point on a dense grid around the optimum's basin
    grid = np.linspace(max(0.1, θ[0] * 0.8), min(5.0, θ[0] * 1.2), 41)
    fgrid, _ = fg(grid[:, None])
    assert f <= np.nanmin(fgrid) + 1e-9 * abs(f)


def test_projected_lbfgs_respects_bounds(oracle):
    from mrbo.mle import projected_lbfgs
    X, y = _data(2, 25, seed=3)
    fg = _oracle_fg(oracle, X, y, "matern52", 1e-6)
    θ, f, g, it = projected_lbfgs(fg, np.array([0.5]), [0.1], [0.2], iterations=30)
    assert 0.1 <= θ[0] <= 0.2
    _assert_kkt(θ[0], g[0], 0.1, 0.2, 1e-6 * max(1.0, abs(f)))


# ---------------------------------------------------------------------------------- GPU
def _surrogate(X, y, kernel, ell, sn2=1e-6):
    from mrbo import kernels
    from mrbo.surrogates import Surrogate
    k = {"matern52": kernels.Matern52, "matern32": kernels.Matern32, "matern12": kernels.Matern12,
         "se": kernels.SquaredExponential}[kernel]([ell])
    return Surrogate(k, X, y, capacity=len(y), σn2=sn2)


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("d,N", [(1, 8), (3, 20), (6, 64), (6, 80), (6, 100), (4, 128), (12, 96), (5, 150), (8, 256),
                                 (6, 300), (3, 384), (8, 512), (16, 200)])
def test_gp_fit_vs_oracle(gpu, oracle, kernel, d, N):
    from mrbo.mle import gp_fit_batch
    X, y = _data(d, N, seed=d)
    ells = np.array([0.2, 0.5, 1.0, 2.0, 4.0]) * np.sqrt(d) * (0.15 if kernel == "se" else 1.0)
    s = _surrogate(X, y, kernel, 1.0)
    r = gp_fit_batch(s, ells, want_fit=True)
    rr = gp_fit_batch(s, ells)   # no factor outputs: N ≤ 32 the tile kernel, ≤ 64 the register kernel, ≤ 80 the LDS kernel
    for p, ell in enumerate(ells):
        ll, dll, L, c = oracle.log_likelihood(X, y, kernel, ell, 1e-6, want_fit=True)
        if np.isnan(ll):
            assert r["status"][p] == 1 and rr["status"][p] == 1
            continue
        assert r["status"][p] == 0 and rr["status"][p] == 0
        tol = _ll_tol(ll, L, c)
        for q in (r, rr):
            assert abs(q["ll"][p] - ll) <= tol, (q["ll"][p], ll, tol)
            assert q["dll"][p] == pytest.approx(dll, rel=1e-8, abs=1e-8 * (1 + abs(ll)))
        # the factor's forward error: first-order perturbation theory bounds it by ≈ √κ₂(K)·u
        # relative to ‖L‖ for two backward-stable factorizations that round differently (the
        # blocked, tile-ordered one of N > 128 against the oracle's column order)
        kap = np.linalg.cond(L @ L.T)
        atol = max(1e-12, 10.0 * np.sqrt(kap) * 2.0 ** -53) * np.abs(L).max()
        np.testing.assert_allclose(r["L"][:, :, p], L, rtol=1e-10, atol=atol)
        np.testing.assert_allclose(r["c"][:, p], c, rtol=1e-8, atol=1e-8 * np.abs(c).max())


@pytest.mark.gpu
def test_gp_fit_wide_inputs_and_lds_limit(gpu, oracle):
    """d > 16 runs the tile kernel, whose LDS holds X (d·⌈N/32⌉·32 doubles): d = 24 at N = 100 fits
    and matches the oracle; d = 40 at N = 512 needs more than the CU's 160 KB, and the call fails
    with MRBO_ERR_UNSUPPORTED before any launch instead of a HIP launch error."""
    from mrbo import _lib
    from mrbo.mle import gp_fit_batch
    X, y = _data(24, 100, seed=5)
    s = _surrogate(X, y, "matern52", 1.0)
    ells = np.array([2.0, 5.0])
    r = gp_fit_batch(s, ells)
    for p, ell in enumerate(ells):
        ll, dll = oracle.log_likelihood(X, y, "matern52", ell, 1e-6)
        assert r["status"][p] == 0
        assert r["ll"][p] == pytest.approx(ll, rel=1e-10, abs=1e-9)
        assert r["dll"][p] == pytest.approx(dll, rel=1e-8, abs=1e-8 * (1 + abs(ll)))
    X, y = _data(40, 512, seed=6)
    s = _surrogate(X, y, "matern52", 5.0)
    with pytest.raises(_lib.MrboError, match="LDS"):
        gp_fit_batch(s, [5.0])


@pytest.mark.gpu
def test_gp_fit_posdef_failure(gpu):
    from mrbo.mle import gp_fit_batch
    X, y = _data(2, 10)
    s = _surrogate(X, y, "se", 0.5)
    s.σn2 = -1.0                   # zero diagonal: first pivot 0 (see the oracle test above)
    r = gp_fit_batch(s, [0.5, 1.0])
    assert (r["status"] == 1).all() and np.isnan(r["ll"]).all()


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", KERNELS)
def test_optimize_on_device_vs_oracle_driven(gpu, oracle, kernel):
    """optimize!(s; lowerbounds=[0.1], upperbounds=[5.]) on the device: same minimiser as the
    oracle-driven run (same iterates up to rounding), a KKT point, and the surrogate refit."""
    from mrbo.mle import log_likelihood, optimize, projected_lbfgs
    X, y = _data(2, 25, seed=3)
    s = _surrogate(X, y, kernel, 1.0)
    res = optimize(s, [0.1], [5.0], iterations=30)
    θo, fo, go, _ = projected_lbfgs(_oracle_fg(oracle, X, y, kernel, 1e-6), np.array([1.0]), [0.1], [5.0], 30)
    assert res["theta"][0] == pytest.approx(θo[0], rel=1e-7)
    assert s.ψ.lengthscale == pytest.approx(θo[0], rel=1e-7)
    assert log_likelihood(s) == pytest.approx(-fo, rel=1e-10)
    _assert_kkt(res["theta"][0], res["gradient"][0], 0.1, 5.0, 1e-5 * max(1.0, abs(fo)))


# ---------------------------------------------------------------------------------- Periodic
# θ = (ℓ, p) (radial_basis_functions.jl:98-103); ∇log_likelihood over both (r_b_s.jl:787-799).
# The kernel of a Euclidean distance is positive definite in one dimension: 1-D data.
def _per_data(N, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.random((1, N)) * 3.0
    return X, np.sin(3 * X[0]) + 0.1 * rng.standard_normal(N)


def _numpy_ll_per(X, y, th, sn2):
    rho = np.abs(X[0][:, None] - X[0][None, :])
    K = np.exp(-2 * np.sin(np.pi * rho / th[1]) ** 2 / th[0] ** 2) + sn2 * np.eye(len(y))
    cf = cho_factor(K, lower=True)
    c = cho_solve(cf, y)
    return -y @ c / 2 - np.log(np.diag(cf[0])).sum() - len(y) * np.log(2 * np.pi) / 2


@pytest.mark.parametrize("th", [(0.7, 1.3), (1.5, 0.8), (2.0, 2.5)])
def test_oracle_periodic_grad_vs_fd(oracle, th):
    X, y = _per_data(20)
    sn2 = 1e-3
    ll, g = oracle.log_likelihood_theta(X, y, "periodic", th, sn2)
    assert ll == pytest.approx(_numpy_ll_per(X, y, th, sn2), rel=1e-9)
    for t in range(2):
        h = 1e-6 * th[t]
        e = np.eye(2)[t] * h
        fd = (_numpy_ll_per(X, y, np.add(th, e), sn2) - _numpy_ll_per(X, y, np.subtract(th, e), sn2)) / (2 * h)
        assert g[t] == pytest.approx(fd, rel=1e-5, abs=1e-5 * (1 + abs(ll)))
    # one-element θ keeps the period: ∂/∂ℓ only, equal to the first component
    ll1, g1 = oracle.log_likelihood_theta(X, y, "periodic", th[:1], sn2, period=th[1])
    assert ll1 == ll and g1[0] == g[0]


def _per_surrogate(X, y, th, sn2):
    from mrbo import kernels
    from mrbo.surrogates import Surrogate
    return Surrogate(kernels.Periodic(list(th)), X, y, capacity=X.shape[1], σn2=sn2)


@pytest.mark.gpu
@pytest.mark.parametrize("N", [16, 64, 100, 300])
def test_gp_fit_periodic_vs_oracle(gpu, oracle, N):
    from mrbo.mle import gp_fit_batch
    X, y = _per_data(N, seed=N)
    sn2 = 1e-3
    th = np.array([[0.7, 1.3], [1.5, 0.8], [2.0, 2.5], [0.5, 1.9]])
    s = _per_surrogate(X, y, th[0], sn2)
    for want_fit in (False, True):
        r = gp_fit_batch(s, th, want_fit=want_fit)
        for p in range(len(th)):
            ll, g = oracle.log_likelihood_theta(X, y, "periodic", th[p], sn2)
            assert r["status"][p] == 0
            assert r["ll"][p] == pytest.approx(ll, rel=1e-10, abs=1e-9)
            np.testing.assert_allclose(r["grad"][p], g, rtol=1e-8, atol=1e-8 * (1 + abs(ll)))
    # one hyperparameter: ∂/∂ℓ at the surrogate's period
    r1 = gp_fit_batch(s, th[:, 0])
    for p in range(len(th)):
        ll, g = oracle.log_likelihood_theta(X, y, "periodic", th[p, :1], sn2, period=th[0, 1])
        assert r1["ll"][p] == pytest.approx(ll, rel=1e-10, abs=1e-9)
        assert r1["dll"][p] == pytest.approx(g[0], rel=1e-8, abs=1e-8 * (1 + abs(ll)))


@pytest.mark.gpu
def test_optimize_periodic_on_device_vs_oracle_driven(gpu, oracle):
    """optimize! over (ℓ, p) for the Periodic kernel: the device run and the oracle-driven run of
    the same minimiser reach the same KKT point."""
    from mrbo.mle import optimize, projected_lbfgs
    rng = np.random.default_rng(7)   # period-1.2 data: the likelihood has a clear optimum in p
    X = rng.random((1, 30)) * 3.0
    y = np.sin(2 * np.pi * X[0] / 1.2) + 0.1 * rng.standard_normal(30)
    sn2 = 1e-2
    s = _per_surrogate(X, y, (1.0, 1.5), sn2)
    lo, hi = [0.2, 0.5], [3.0, 3.0]
    res = optimize(s, lo, hi, iterations=30)

    def fg(T):
        f, g = np.zeros(len(T)), np.zeros_like(T)
        for i, t in enumerate(T):
            ll, gr = oracle.log_likelihood_theta(X, y, "periodic", t, sn2)
            f[i], g[i] = -ll, -gr
        return f, g

    θo, fo, go, _ = projected_lbfgs(fg, np.array([1.0, 1.5]), lo, hi, 30)
    np.testing.assert_allclose(res["theta"], θo, rtol=1e-6)
    np.testing.assert_allclose(s.ψ.θ, θo, rtol=1e-6)
    assert abs(res["theta"][1] - 1.2) < 0.05      # the data's period
    for t in range(2):
        _assert_kkt(res["theta"][t], res["gradient"][t], lo[t], hi[t], 1e-4 * max(1.0, abs(fo)))
