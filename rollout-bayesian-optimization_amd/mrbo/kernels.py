"""Stationary radial kernels -- host mirror of radial_basis_functions.jl.

Only the host-side bookkeeping lives here (building K, L, c for a base ``Surrogate``, which
the reference does once per BO step, radial_basis_surrogates.jl:77-118).  Every evaluation
on the rollout path runs in libmrbo.so; the kernel id selects the same closed forms there.
"""
import numpy as np

MATERN52, MATERN32, MATERN12, SE, PERIODIC = 0, 1, 2, 3, 4


class RadialBasisFunction:
    """radial_basis_functions.jl:7-14: ψ(ρ; θ) with its ρ-derivatives (closed forms of the
    ForwardDiff derivatives taken in compute_derivatives, :41-46)."""

    def __init__(self, name, kind, theta):
        self.name = name
        self.kind = kind
        self.θ = np.array(theta, dtype=np.float64)

    @property
    def lengthscale(self):
        return float(self.θ[0])

    @property
    def period(self):
        """θ[2] of the Periodic kernel (1.0 for the one-parameter kernels)."""
        return float(self.θ[1]) if self.kind == PERIODIC else 1.0

    def _per(self):
        # Periodic: A = 2π/(pℓ²), B = 2π/p; ψ = exp(−2 sin²(πρ/p)/ℓ²), ψ' = −ψ A sin(Bρ),
        # ψ'' = ψ (A² sin²(Bρ) − A B cos(Bρ))
        l, p = self.θ
        return 2 * np.pi / (p * l * l), 2 * np.pi / p

    def _c(self):
        l = self.lengthscale
        return {MATERN52: np.sqrt(5.0) / l, MATERN32: np.sqrt(3.0) / l, MATERN12: 1.0 / l, SE: 1.0 / (l * l),
                PERIODIC: 1.0 / (l * l)}[self.kind]

    def __call__(self, rho):
        rho = np.asarray(rho, dtype=np.float64)
        c = self._c()
        if self.kind == PERIODIC:
            return np.exp(-2 * np.sin(np.pi * rho / self.θ[1]) ** 2 * c)
        if self.kind == MATERN52:
            s = c * rho
            return (1 + s * (1 + s / 3.0)) * np.exp(-s)
        if self.kind == MATERN32:
            s = c * rho
            return (1 + s) * np.exp(-s)
        if self.kind == MATERN12:
            return np.exp(-c * rho)
        return np.exp(-0.5 * rho * rho * c)

    def derivative(self, rho):
        rho = np.asarray(rho, dtype=np.float64)
        c = self._c()
        if self.kind == PERIODIC:
            A, B = self._per()
            return -self(rho) * A * np.sin(B * rho)
        if self.kind == MATERN52:
            s = c * rho
            return -c * (s / 3.0) * (1 + s) * np.exp(-s)
        if self.kind == MATERN32:
            s = c * rho
            return -c * s * np.exp(-s)
        if self.kind == MATERN12:
            return -c * np.exp(-c * rho)
        return -(rho * c) * np.exp(-0.5 * rho * rho * c)

    def second_derivative(self, rho):
        rho = np.asarray(rho, dtype=np.float64)
        c = self._c()
        if self.kind == PERIODIC:
            A, B = self._per()
            return self(rho) * (A * A * np.sin(B * rho) ** 2 - A * B * np.cos(B * rho))
        if self.kind == MATERN52:
            s = c * rho
            return c * c * (s * s - s - 1) * np.exp(-s) / 3.0
        if self.kind == MATERN32:
            s = c * rho
            return c * c * (s - 1) * np.exp(-s)
        if self.kind == MATERN12:
            return c * c * np.exp(-c * rho)
        return (rho * rho * c * c - c) * np.exp(-0.5 * rho * rho * c)

    def __repr__(self):
        return f"RadialBasisFunction{{{self.name}, θ={self.θ.tolist()}}}"


def Matern52(θ=(1.0,)):
    return RadialBasisFunction("Matern52", MATERN52, θ)


def Matern32(θ=(1.0,)):
    return RadialBasisFunction("Matern32", MATERN32, θ)


def Matern12(θ=(1.0,)):
    return RadialBasisFunction("Matern12", MATERN12, θ)


def SquaredExponential(θ=(1.0,)):
    return RadialBasisFunction("SquaredExponential", SE, θ)


def Periodic(θ=(1.0, 1.0)):
    """radial_basis_functions.jl:98-103: θ = [ℓ, p]."""
    return RadialBasisFunction("Periodic", PERIODIC, θ)


def get_hyperparameters(k):
    return k.θ


def set_hyperparameters(k, θ):
    k.θ[:] = θ
    return k


def eval_KXX(rbf, X, σn2=1e-6):
    """radial_basis_functions.jl:161-178 (host; once per base fit)."""
    X = np.asarray(X, dtype=np.float64)
    diff = X[:, :, None] - X[:, None, :]
    K = rbf(np.sqrt((diff * diff).sum(axis=0)))
    np.fill_diagonal(K, rbf(0.0))
    return K + σn2 * np.eye(X.shape[1])


def eval_KxX(rbf, x, X):
    """radial_basis_functions.jl:180-191 (host)."""
    r = np.asarray(x, dtype=np.float64)[:, None] - np.asarray(X, dtype=np.float64)
    return rbf(np.sqrt((r * r).sum(axis=0)))
