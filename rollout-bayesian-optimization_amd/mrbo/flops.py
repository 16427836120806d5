"""Algorithmic FLOP model of the rollout kernel.

Counts the useful fp64 arithmetic of the formulation the kernel executes (explicit inverse
factor L⁻¹ = [[L0⁻¹, 0], [E, Dinv]], lanes over data rows), per operation, at N base rows,
nf fantasy rows and dimension d.  A transcendental (exp, sqrt, erfc) counts as one flop, an
FMA as two.  Excluded: masked-lane waste (upper-triangle lanes of the triangular products)
and wave-redundant lane-uniform bookkeeping -- those are overheads, not algorithmic work.
The per-trajectory counts of each operation come from the kernel's own counters
(mrbo_simulate_mc `evals`: full / value-only / rich evaluations, adjoint pairs).
"""


def _rows(n, d):  # kernel row + gradient: r, ρ², sqrt, exp, ψ, ψ', ∇k
    return n * (5 * d + 12)


def f_value(N, nf, d):
    return N * (N + 1) + N * (3 * d + 10) + nf * (3 * d + 10) + 2 * N * (2 + nf) + 2 * nf * (nf + 1) + 40


def _forward_all(N, nf, d):
    D1 = d + 1
    return (_rows(N + nf, d) + D1 * N * (N + 1)          # L0⁻¹ · [kx, ∇kx]
            + N * D1 * (D1 + 1) + 2 * d * N              # Gram products, ∇μ partials
            + 2 * D1 * nf * N + D1 * nf * (nf + 1)       # fantasy rows E·B, Dinv·Bf
            + D1 * (D1 + 1) * nf                         # fantasy Gram update
            + N * (N + 1) + 2 * nf * N + nf * (nf + 1))  # backward w = L⁻ᵀ v


def f_draw(N, nf, d):
    D1 = d + 1
    return _forward_all(N, nf, d) + D1 ** 3 // 3 + 2 * D1 * D1 + 4 * N + 60   # + Σ chol, draw, condition!


def f_full(N, nf, d):
    nh = d * (d + 1) // 2
    return (_forward_all(N, nf, d) + 60
            + N * (3 * nh + 6 * d + 20)                  # Σ_j coef_j Hk_j per data row
            + nh * (12 + nf * (5 * d + 20))              # Hα assembly incl. fantasy rows
            + d ** 3 // 3 + 4 * d * d)                   # Newton step (Cholesky + solves)


def f_rich(N, nf, d):
    return f_full(N, nf, d) + d * N * (N + 1) + 2 * d * nf * N + 2 * d * nf * (nf + 1)  # + P = L⁻ᵀ V


def f_pair(N, nf, d):
    return N * (5 * d + 12 + 2 * (d * d + 2 * d)) + nf * (5 * d + 12 + 2 * (d * d + 2 * d)) + (d + 1) * (6 * d * d + 40 * d)


def trajectory_flops(counts, N, d, h):
    """counts: (full, value, rich, pairs) of one trajectory (or sums over many, with the draw
    term multiplied by the number of trajectories via `ntraj`)."""
    full, value, rich, pairs = counts[:4]
    nf_solve = (1 + h) / 2.0  # solves run on surfaces with 1..h fantasy rows
    f = (full * f_full(N, nf_solve, d) + value * f_value(N, nf_solve, d) + rich * f_rich(N, nf_solve, d)
         + pairs * f_pair(N, nf_solve, d))
    return f


def launch_flops(evals, N, d, h):
    """evals: (4, M, R) counters of one launch → total algorithmic flops of the launch."""
    import numpy as np
    e = np.asarray(evals, dtype=np.float64).reshape(4, -1)
    ntraj = e.shape[1]
    draws = sum(f_draw(N, k, d) for k in range(h + 1))
    return float(trajectory_flops(e.sum(axis=1), N, d, h) + ntraj * draws)
