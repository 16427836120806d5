"""Algorithmic FLOP model of the rollout kernel.

Counts the useful fp64 arithmetic of the formulation the kernel executes (explicit inverse
factor L⁻¹ = [[L0⁻¹, 0], [E, Dinv]], lanes over data rows), per operation, at N base rows,
nf fantasy rows and dimension d.  A transcendental (exp, sqrt, erfc) counts as one flop, an
FMA as two.  Excluded: masked-lane waste (upper-triangle lanes of the triangular products)
and wave-redundant lane-uniform bookkeeping -- those are overheads, not algorithmic work.
The per-trajectory counts of each operation come from the kernel's own counters
(mrbo_simulate_mc `evals`: gradient / value-only evaluations, Hessian completions, adjoint rich
evaluations, adjoint pairs).
"""


def _rows(n, d):  # kernel row + gradient: r, ρ², sqrt, exp, ψ, ψ', ∇k
    return n * (5 * d + 12)


def f_value(N, nf, d):
    return N * (N + 1) + N * (3 * d + 10) + nf * (3 * d + 10) + 2 * N * (2 + nf) + 2 * nf * (nf + 1) + 40


def _front(N, nf, d):
    """Kernel rows, forward product, Gram, μ/∇μ, fantasy rows (every mode but value)."""
    D1 = d + 1
    return (_rows(N + nf, d) + D1 * N * (N + 1)          # L0⁻¹ · [kx, ∇kx]
            + N * D1 * (D1 + 1) + 2 * d * N              # Gram products, ∇μ partials
            + 2 * D1 * nf * N + D1 * nf * (nf + 1)       # fantasy rows E·B, Dinv·Bf
            + D1 * (D1 + 1) * nf)                        # fantasy Gram update


def _backward(N, nf):
    return N * (N + 1) + 2 * nf * N + nf * (nf + 1)      # w = L⁻ᵀ v (base + fantasy rows)


def f_grad(N, nf, d):
    """Gradient completion of a value-only evaluation (GRADC): rows again, columns 1..d."""
    return _front(N, nf, d) - N * (N + 1) + 20           # column 0 of L0⁻¹ B comes from the value pass


def f_hess(N, nf, d):
    """Deferred completion of a gradient evaluation: backward product, Hα, Newton step."""
    nh = d * (d + 1) // 2
    return (_backward(N, nf)
            + N * (3 * nh + 6 * d + 20)                  # Σ_j coef_j Hk_j per data row
            + nh * (12 + nf * (5 * d + 20))              # Hα assembly incl. fantasy rows
            + d ** 3 // 3 + 4 * d * d)                   # Newton step (Cholesky + solves)


def f_draw(N, nf, d):
    D1 = d + 1
    return _front(N, nf, d) + 60 + _backward(N, nf) + D1 ** 3 // 3 + 2 * D1 * D1 + 4 * N   # + chol, draw, condition!


def f_full(N, nf, d):
    return _front(N, nf, d) + 60 + f_hess(N, nf, d)


def f_rich(N, nf, d):
    return f_full(N, nf, d) + d * N * (N + 1) + 2 * d * nf * N + 2 * d * nf * (nf + 1)  # + P = L⁻ᵀ V


def f_pair(N, nf, d):
    return N * (5 * d + 12 + 2 * (d * d + 2 * d)) + nf * (5 * d + 12 + 2 * (d * d + 2 * d)) + (d + 1) * (6 * d * d + 40 * d)


def f_batch_start(N, nf, d):
    """One start point of the batched start-value pass (batch_start_values): the base part of μ
    and of the fantasy rows from the launch's kernel-row table (c·kxb, E_r·kxb over N rows), the
    fantasy radial functions, Dinv·pf, σ² from the tabled |L0⁻¹kx|², EI and the certificate."""
    return 2 * N * (1 + nf) + nf * (3 * d + 10) + nf * (nf + 1) + 4 * nf + 40


def f_start_table(N, d):
    """Launch constants of one start point (stage_start_tables / start_tables_kernel): base kernel
    rows and gradients, Y = L0⁻¹[kx, ∇kx], the base Gram YᵀY."""
    D1 = d + 1
    return _rows(N, d) + D1 * N * (N + 1) + N * D1 * (D1 + 1)


NCOUNTERS = 5   # mrbo_simulate_mc evals: grad, value, hess, rich, pairs


def trajectory_flops(counts, N, d, h):
    """counts: (gradient completions, value evals, Hessian completions, rich evals, adjoint
    pairs) of one trajectory (or sums over many)."""
    grad, value, hess, rich, pairs = counts[:NCOUNTERS]
    nf_solve = (1 + h) / 2.0  # solves run on surfaces with 1..h fantasy rows
    return (grad * f_grad(N, nf_solve, d) + value * f_value(N, nf_solve, d) + hess * f_hess(N, nf_solve, d)
            + rich * f_rich(N, nf_solve, d) + pairs * f_pair(N, nf_solve, d))


def launch_flops(evals, N, d, h, info=None, nstarts=0):
    """evals: (NCOUNTERS, M, R) counters of one launch → total algorithmic flops of the launch.

    info: RolloutPlan.info() of the launch.  With batched start values the counters still count
    every start point as a value evaluation (as the oracle does); those h·nstarts evaluations per
    trajectory are charged at the batched pass's cost instead, plus the start tables (staged once
    per workgroup for the square layout, once per launch for the packed ones)."""
    import numpy as np
    e = np.asarray(evals, dtype=np.float64).reshape(NCOUNTERS, -1)
    ntraj = e.shape[1]
    draws = sum(f_draw(N, k, d) for k in range(h + 1))
    tot = e.sum(axis=1)
    extra = 0.0
    if info is not None and info.get("batch") and nstarts:
        nb = min(float(h * nstarts * ntraj), float(tot[1]))   # batched start values of the launch
        tot[1] -= nb
        nf_solve = (1 + h) / 2.0
        tables = info["blocks"] if info.get("rpl", 1) == 1 else 1
        extra = nb * f_batch_start(N, nf_solve, d) + tables * nstarts * f_start_table(N, d)
    return float(trajectory_flops(tot, N, d, h) + ntraj * draws + extra)
