#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ from an independent NumPy restatement.

The Julia reference cannot run here (no julia binary) and ships no golden
vectors, so these fixtures come from a second, independent restatement of the reference
algorithm written directly from the Julia sources -- dense algebra with LAPACK solves,
nothing shared with oracle/rbo_oracle.c or the HIP kernels:

  rnstream      utils.jl:4-74 (scipy's unscrambled Sobol = Joe-Kuo table, Box–Muller log10,
                column-major reshape)
  inner starts  utils.jl:145-153
  eval_base     radial_basis_surrogates.jl:224-310 + decision_rules.jl:84-99 (partials in
                closed form)
  replay        rollout.jl:39-277 with the policy points INJECTED (the inner solve uses
                Optim.IPNewton, which is unavailable; every other quantity of the forward
                rollout and the adjoint gradient is restated here, quirks Q1-Q16 included)

Run: python tests/golden/make_golden.py   (writes golden_*.npz next to this file)
"""
import os

import numpy as np
from scipy.linalg import cho_factor, cho_solve, solve_triangular
from scipy.special import erfc
from scipy.stats import qmc

HERE = os.path.dirname(os.path.abspath(__file__))
SQ5 = np.sqrt(5.0)


# ---------------- kernels (radial_basis_functions.jl:60-68, 127-159) ----------------------
def psi(r, ell=1.0):
    s = SQ5 / ell * r
    return (1 + s * (1 + s / 3.0)) * np.exp(-s)


def dpsi(r, ell=1.0):
    c = SQ5 / ell
    s = c * r
    return -c * (s / 3.0) * (1 + s) * np.exp(-s)


def d2psi(r, ell=1.0):
    c = SQ5 / ell
    s = c * r
    return c * c * (s * s - s - 1) * np.exp(-s) / 3.0


def grad_k(r):
    rho = np.linalg.norm(r)
    return np.zeros_like(r) if rho == 0 else dpsi(rho) * r / rho


def hess_k(r):
    p = np.linalg.norm(r)
    d = r.size
    if p > 0:
        u = r / p
        Dpr = dpsi(p) / p
        return (d2psi(p) - Dpr) * np.outer(u, u) + Dpr * np.eye(d)
    return d2psi(0.0) * np.eye(d)


# ---------------- EI and partials (decision_rules.jl:84-99) -------------------------------
def ei_all(mu, sig, theta, fmin, tol=1e-8):
    keys = ("g", "gmu", "gsig", "gth", "gmumu", "gsigsig", "gthth", "gmuth", "gsigth")
    if sig < tol:
        return {k: 0.0 for k in keys}
    imp = fmin - mu - theta
    z = imp / sig
    Phi = erfc(-z / np.sqrt(2)) / 2
    phi = np.exp(-z * z / 2) / np.sqrt(2 * np.pi)
    return dict(g=imp * Phi + sig * phi, gmu=-Phi, gsig=phi, gth=-Phi, gmumu=phi / sig,
                gsigsig=z * z * phi / sig, gthth=phi / sig, gmuth=phi / sig, gsigth=z * phi / sig)


# ---------------- fantasy surrogate (radial_basis_surrogates.jl:320-611) -----------------
class Fantasy:
    def __init__(self, X, y, L, c, sn2=1e-6):
        self.X = [X[:, j].copy() for j in range(X.shape[1])]
        self.y = list(y)
        self.L = L.copy()
        self.cs = [c.copy()]
        self.N = X.shape[1]
        self.sn2 = sn2

    def condition(self, x, yv):
        Xa = np.array(self.X).T
        kvec = psi(np.linalg.norm(Xa - x[:, None], axis=0))
        L21 = solve_triangular(self.L, kvec, lower=True)
        S = psi(0.0) + self.sn2 - L21 @ L21
        assert S > 0, "PosDefException"
        n = self.L.shape[0]
        Ln = np.zeros((n + 1, n + 1))
        Ln[:n, :n] = self.L
        Ln[n, :n] = L21
        Ln[n, n] = np.sqrt(S)
        self.L = Ln
        self.X.append(x.copy())
        self.y.append(yv)
        self.cs.append(solve_triangular(Ln.T, solve_triangular(Ln, np.array(self.y), lower=True), lower=False))

    def eval(self, x, theta, fi):
        n = self.N + fi + 1
        X = np.array(self.X[:n]).T
        L = self.L[:n, :n]
        c = self.cs[fi + 1]
        y = np.array(self.y[:n])
        d = x.size
        R = x[:, None] - X
        kx = psi(np.linalg.norm(R, axis=0))
        gkx = np.array([grad_k(R[:, j]) for j in range(n)]).T  # d×n
        Kinv = lambda B: solve_triangular(L.T, solve_triangular(L, B, lower=True), lower=False)
        sx = dict(x=x.copy(), n=n, kx=kx, gkx=gkx, c=c, fmin=y.min())
        sx["mu"] = kx @ c
        sx["gmu"] = gkx @ c
        sx["Hmu"] = sum(c[j] * hess_k(R[:, j]) for j in range(n))
        sx["w"] = Kinv(kx)
        sx["Dw"] = Kinv(gkx.T)
        var = psi(0.0) - kx @ sx["w"]
        sx["sigma"] = np.sqrt(var)
        sx["gsig"] = -(gkx @ sx["w"]) / sx["sigma"]
        Hs = -np.outer(sx["gsig"], sx["gsig"]) - gkx @ sx["Dw"]
        Hs -= sum(sx["w"][j] * hess_k(R[:, j]) for j in range(n))
        sx["Hsig"] = Hs / sx["sigma"]
        e = ei_all(sx["mu"], sx["sigma"], theta, sx["fmin"])
        sx["e"] = e
        sx["alpha"] = e["g"]
        sx["galpha"] = e["gmu"] * sx["gmu"] + e["gsig"] * sx["gsig"]
        sx["Halpha"] = (e["gmumu"] * np.outer(sx["gmu"], sx["gmu"]) + e["gmu"] * sx["Hmu"]
                        + e["gsigsig"] * np.outer(sx["gsig"], sx["gsig"]) + e["gsig"] * sx["Hsig"])  # Q11
        sx["mixed"] = sx["gmu"] * e["gmuth"] + sx["gsig"] * e["gsigth"]
        kxX = np.vstack([kx[None, :], gkx])
        Dk0 = np.diag([psi(0.0)] + [-d2psi(0.0)] * d)
        Sig = Dk0 - kxX @ Kinv(kxX.T)
        sx["Sig"] = np.triu(Sig) + np.triu(Sig, 1).T  # Symmetric(σx) reads the upper triangle
        return sx

    def draw(self, x, theta, fi, z):
        sx = self.eval(x, theta, fi)
        Ls = np.linalg.cholesky(sx["Sig"])
        out = np.concatenate([[sx["mu"]], sx["gmu"]]) + Ls @ z
        return out[0], out[1:]

    def perturb(self, sx, S, q, delta, data):
        """Spatial/DataPerturbationSurrogate (r_b_s.jl:652-757) with dense δK (:210-262)."""
        n = self.N + S + 1
        X = np.array(self.X[:n]).T
        L = self.L[:n, :n]
        c = self.cs[S + 1]
        d = X.shape[0]
        dX = np.zeros((d, n))
        dX[:, self.N + q] = delta
        dK = np.zeros((n, n))
        for j in range(n):
            for i in range(j + 1, n):
                v = grad_k(X[:, i] - X[:, j]) @ (dX[:, i] - dX[:, j])
                dK[i, j] = dK[j, i] = v
        Kinv = lambda B: solve_triangular(L.T, solve_triangular(L, B, lower=True), lower=False)
        dc = -Kinv(dK @ c)
        x = sx["x"]
        dkx = np.array([grad_k(x - X[:, j]) @ (-dX[:, j]) for j in range(n)])
        dgkx = np.array([hess_k(x - X[:, j]) @ (-dX[:, j]) for j in range(n)]).T
        dmu = dkx @ c + sx["kx"] @ dc
        dgmu = dgkx @ c + sx["gkx"] @ dc
        w = sx["w"]
        dsig = (-2 * dkx @ w + w @ (dK @ w)) / (2 * sx["sigma"])
        gw = sx["Dw"].T
        dgsig = (gw @ (dK @ w) - dgkx @ w - gw @ dkx - dsig * sx["gsig"]) / sx["sigma"]
        de = ei_all(dmu, dsig, 0.0 if "theta" not in sx else sx["theta"], sx["fmin"])
        e = sx["e"]
        if data:
            return e["gmu"] * dgmu + de["gmu"] * sx["gmu"] + de["gsig"] * sx["gsig"]
        return e["gmu"] * dgmu + e["gsig"] * dgsig + de["gmu"] * sx["gmu"] + de["gsig"] * sx["gsig"]


def trajectory_replay(X, y, L, c, fmini, x0, z, policy, dual_dx, theta=0.0, htol=1e-4):
    """rollout! + resolve + gradient(T) for one trajectory with injected policy points."""
    fs = Fantasy(X, y, L, c)
    h = policy.shape[1]
    d = x0.size
    obs, grads = [], []
    for k in range(h + 1):
        xk = x0 if k == 0 else policy[:, k - 1]
        yv, gy = fs.draw(xk, theta, k - 1, z[:, k])
        obs.append(yv)
        grads.append(gy)
        fs.condition(xk, yv)
    obs = np.array(obs)
    t = int(np.argmin(obs))
    fb = obs[t]
    value = max(fmini - fb, 0.0)
    if fmini <= fb:
        return value, np.zeros(d), 0.0, obs
    if t == 0:
        return value, -grads[0], 0.0, obs
    rec = [fs.eval(fs.X[fs.N + i], theta, i - 1) for i in range(t + 1)]
    xb = [None] + [np.zeros(d) for _ in range(t)]
    yb = np.zeros(t + 1)
    yb[t] = 1.0
    for j in range(t, 0, -1):
        H = rec[j]["Halpha"]
        if np.linalg.det(H) < htol:
            xd = np.zeros(d)
        else:
            xd = -grads[j - 1] * yb[j]
            for i in range(j + 1, t + 1):
                dri = np.column_stack([fs.perturb(rec[i], i - 1, j, np.eye(d)[:, k], False) for k in range(d)])
                xd = xd - dri.T @ xb[i]
            xd = np.linalg.solve(H.T, xd)
        xb[j] = xd
        dx = dual_dx[:, j - 1]
        yb[j - 1] = sum(fs.perturb(rec[i], i - 1, j - 1, dx, True) @ xb[i] for i in range(j, t + 1))
    gx = rec[0]["gmu"] * yb[0]
    gth = 0.0
    for j in range(1, t + 1):
        g = np.column_stack([fs.perturb(rec[j], j - 1, 0, np.eye(d)[:, k], False) for k in range(d)])
        gx = gx + g.T @ xb[j]
        gth += rec[j]["mixed"] @ xb[j]
    return value, -gx, -gth, obs


# ---------------- rnstream / starts (utils.jl) ---------------------------------------------
def rnstream(M, d, H):
    off = 1 if (d + 1) % 2 == 1 else 0
    Dp = d + 1 + off
    S = qmc.Sobol(Dp, scramble=False).random(M * H + 1)[1:].T  # Sobol.jl skips the zero point
    N = np.zeros_like(S)
    for i in range(Dp):
        if i % 2 == 0:
            N[i] = np.sqrt(-2 * np.log10(S[i])) * np.cos(2 * np.pi * S[i + 1])
        else:
            N[i] = np.sqrt(-2 * np.log10(S[i - 1])) * np.sin(2 * np.pi * S[i])
    return N.reshape((M, Dp, H), order="F")[:, :d + 1, :]


def initial_guesses(n, lbs, ubs):
    P = qmc.Sobol(lbs.size, scramble=False).random(n + 1)[1:].T
    G = lbs[:, None] + (ubs - lbs)[:, None] * P
    return np.column_stack([G, lbs + 1e-6, ubs - 1e-6])


def kronecker(d, N, start=0):
    phi = 1.0 + 1.0 / d
    for _ in range(10):
        phi -= (phi ** (d + 1) - phi - 1) / ((d + 1) * phi ** d - 1)
    a = np.array([np.mod(1.0 / phi ** j, 1.0) for j in range(1, d + 1)])
    return np.array([np.mod(0.5 + (start + j) * a, 1.0) for j in range(1, N + 1)]).T


def hartmann6(x):
    al = np.array([1.0, 1.2, 3.0, 3.2])
    A = np.array([[10, 3, 17, 3.5, 1.7, 8], [0.05, 10, 17, 0.1, 8, 14], [3, 3.5, 1.7, 10, 17, 8],
                  [17, 8, 0.05, 10, 0.1, 14]])
    P = 1e-4 * np.array([[1312, 1696, 5569, 124, 8283, 5886], [2329, 4135, 8307, 3736, 1004, 9991],
                         [2348, 1451, 3522, 2883, 3047, 6650], [4047, 8828, 8732, 5743, 1091, 381]])
    return -np.sum(al * np.exp(-np.sum(A * (x - P) ** 2, axis=1)))


FUNCS = {
    "gramacylee": (lambda x: np.sin(10 * np.pi * x[0]) / (2 * x[0]) + (x[0] - 1.0) ** 4, [0.5], [2.5]),
    "braninhoo": (lambda x: (x[1] - 5.1 / (4 * np.pi ** 2) * x[0] ** 2 + 5 / np.pi * x[0] - 6) ** 2
                  + 10 * (1 - 1 / (8 * np.pi)) * np.cos(x[0]) + 10, [-5.0, 0.0], [10.0, 15.0]),
    "hartmann6d": (hartmann6, [0.0] * 6, [1.0] * 6),
}


def make_case(name, fn, N, h, M, R, capacity=None, seed=7, near_best=False):
    f, lbs, ubs = FUNCS[fn]
    lbs, ubs = np.array(lbs), np.array(ubs)
    d = lbs.size
    w = (ubs - lbs)[:, None]
    X = lbs[:, None] + w * kronecker(d, N)
    y = np.array([f(X[:, j]) for j in range(N)])
    K = psi(np.linalg.norm(X[:, :, None] - X[:, None, :], axis=0))
    np.fill_diagonal(K, psi(0.0))
    K += 1e-6 * np.eye(N)
    L = np.linalg.cholesky(K)
    c = cho_solve(cho_factor(K, lower=True), y)
    cap = capacity or N
    fmini = min(y.min(), 0.0) if cap > N else y.min()  # Q3: zero padding enters the minimum
    x0s = lbs[:, None] + w * kronecker(d, R, N)
    rn = rnstream(M, d, h + 1)
    rng = np.random.default_rng(seed)
    policy = lbs[:, None, None, None] + w[:, :, None, None] * rng.uniform(0.05, 0.95, size=(d, h, M, R))
    if near_best:  # keep the trajectory in the low region so improvements (and adjoints) are non-trivial
        xb = X[:, np.argmin(y)]
        policy = np.clip(xb[:, None, None, None] + 0.08 * w[:, :, None, None] * rng.standard_normal((d, h, M, R)),
                         lbs[:, None, None, None], ubs[:, None, None, None])
        x0s = np.clip(xb[:, None] + 0.08 * w * rng.standard_normal((d, R)), lbs[:, None], ubs[:, None])
    dual = rng.uniform(size=(d, h, M, R))
    values = np.zeros((M, R))
    gx = np.zeros((d, M, R))
    gth = np.zeros((1, M, R))
    obs = np.zeros((h + 1, M, R))
    for r in range(R):
        for m in range(M):
            v, g, gt, o = trajectory_replay(X, y, L, c, fmini, x0s[:, r], rn[m], policy[:, :, m, r], dual[:, :, m, r])
            values[m, r], gx[:, m, r], gth[0, m, r], obs[:, m, r] = v, g, gt, o
    # base-surrogate primitives at Sobol points
    pts = lbs[:, None] + w * qmc.Sobol(d, scramble=False).random(9)[1:].T
    fs = Fantasy(X, y, L, c)
    prim = []
    for j in range(pts.shape[1]):
        sx = fs.eval(pts[:, j], 0.0, -1)
        prim.append(np.concatenate([[sx["mu"], sx["sigma"], sx["alpha"]], sx["gmu"], sx["gsig"], sx["galpha"],
                                    sx["Halpha"].ravel(order="F"), sx["mixed"]]))
    np.savez(os.path.join(HERE, f"golden_{name}.npz"), X=X, y=y, L=L, c=c, fmini=fmini, lbs=lbs, ubs=ubs,
             x0s=x0s, rnstream=rn, replay_x=policy, dual_y_dx=dual, values=values, grad_x=gx, grad_theta=gth,
             obs=obs, h=h, pts=pts, prim=np.array(prim).T, xstarts=initial_guesses(16, lbs, ubs))
    print(name, "values", values.ravel()[:4], "grad", gx.reshape(d, -1)[:, :2].ravel())


if __name__ == "__main__":
    make_case("c1", "gramacylee", N=8, h=1, M=8, R=2)
    make_case("c2", "braninhoo", N=12, h=2, M=6, R=2)
    make_case("c2cap", "braninhoo", N=12, h=2, M=4, R=2, capacity=20)
    make_case("c3", "hartmann6d", N=16, h=3, M=6, R=2, near_best=True)
    make_case("c2near", "braninhoo", N=12, h=3, M=6, R=2, near_best=True)
