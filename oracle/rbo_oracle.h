/*
 * rbo_oracle.h -- CPU restatement of the Rollout-Bayesian-Optimization hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity checker for the MI355X
 * product (libmrbo.so).  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.  The product never links or calls it.
 *
 * It restates, in plain C and in the reference's own (column-major, Julia) layout:
 *   rollout.jl:39-340            rollout!, resolve, gradient (adjoint), simulate_trajectory_mc
 *   radial_basis_surrogates.jl   Surrogate/FantasySurrogate eval, condition!, gp_draw,
 *                                log_likelihood / ∇log_likelihood (:770-799),
 *                                Spatial/DataPerturbationSurrogate (dense δK, as written)
 *   radial_basis_functions.jl    Matern52/32/12, SquaredExponential, Periodic and their ρ-derivatives
 *   decision_rules.jl:84-127     EI, POI, LCB and their partials (closed forms of the ForwardDiff partials)
 *   observables.jl:83-124        StochasticObservable (gp_draw with gradient)
 *   utils.jl:4-74,145-153        Sobol uniforms, Box–Muller(log10), rnstream reshape, inner starts
 *   low_discrepancy.jl:7-28      kronecker_quasirand
 * The inner policy solve (rbf_optim.jl:1-101, Optim.jl IPNewton -- absent, unpinned) is
 * replaced by the build's deterministic projected Newton spec; the GPU
 * implements the same spec.
 *
 * Parity status: UNPINNED against the Julia reference (julia is not installed, the
 * reference ships no golden vectors).  Cross-checked against an independent NumPy
 * restatement (tests/golden), scipy's Sobol, closed forms and the reference's own
 * finite-difference methodology (runtests.jl:11-157).
 */
#ifndef RBO_ORACLE_H
#define RBO_ORACLE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

enum { RBO_K_MATERN52 = 0, RBO_K_MATERN32 = 1, RBO_K_MATERN12 = 2, RBO_K_SE = 3, RBO_K_PERIODIC = 4 };

/* per-trajectory status bits (reference: Julia exceptions, see SURVEY.md §8b "Errors") */
enum {
  RBO_ST_OK = 0,
  RBO_ST_SIGMA_NEG = 1,      /* DomainError: sqrt of negative posterior variance (r_b_s.jl:528) */
  RBO_ST_DRAW_NOT_PD = 2,    /* PosDefException in gp_draw covariance (r_b_s.jl:537)          */
  RBO_ST_COND_NOT_PD = 4,    /* PosDefException in update_cholesky! (r_b_s.jl:412)            */
  RBO_ST_ALL_NAN = 8,        /* findmin on empty candidate list (rbf_optim.jl:96-97)          */
  RBO_ST_SINGULAR = 16       /* singular Hessian in solve_dual_x (rollout.jl:188)             */
};

typedef struct {
  int32_t d, N;            /* dimension, base observations                       */
  int32_t kernel;          /* RBO_K_*                                            */
  double ell;              /* kernel lengthscale θ[1]                            */
  double sigma_n2;         /* σn2                                                */
  double fmini;            /* minimum(s.y) over the capacity buffer (Q3)         */
  const double* X;         /* d×N column-major                                   */
  const double* L;         /* N×N lower Cholesky of K, column-major, ld = N      */
  const double* c;         /* N, L'\(L\y)                                        */
  const double* y;         /* N                                                  */
  double period;           /* Periodic kernel θ[2] (radial_basis_functions.jl:98-103) */
} rbo_surrogate;

typedef struct {
  int32_t h, M, R, nstarts;
  double theta;            /* decision-rule hyperparameter T.θ[1] (EI ξ)         */
  const double* lbs;       /* d */
  const double* ubs;       /* d */
  int32_t max_iters, max_ls;
  double x_tol, f_tol, g_tol;
  double htol;             /* det threshold in solve_dual_x (rollout.jl:156)     */
  double sigma_tol;        /* EI σtol (decision_rules.jl:84)                     */
  uint64_t seed;           /* counter-based δx for solve_dual_y when dual_y_dx==NULL */
  int32_t sample_offset;   /* global index of the first sample (sharded runs), 0      */
  int32_t samples_total;   /* global samples per restart (informational; the δx RNG is */
                           /* keyed by the global sample index sample_offset + m)      */
  int32_t with_gradient;
  int32_t nthreads;        /* OpenMP threads for the (restart, sample) loop      */
  int32_t rule;            /* RBO_RULE_* base decision rule of the trajectory    */
  int32_t cost;            /* RBO_COST_*: NonUniformCost weighting of the inner-solve rule */
  double cost_c0;          /* cost family parameters (see RBO_COST_*)            */
  const double* cost_w;    /* d weights, or NULL when cost == RBO_COST_NONE      */
  double* kappa;           /* diagnostic output M×R, or NULL: per trajectory the largest of
                              cond₁(H_j) = ‖H_j‖₁‖H_j⁻¹‖₁ over the adjoint solves H_j'\x̄ and
                              ‖Dk(0)‖₁‖σx⁻¹‖₁ over the draws (the cancellation condition of the
                              draw covariance σx = Dk(0) − G); the parity tests scale the
                              gradient tolerance by it                                        */
  double* vbound;          /* diagnostic output M×R, or NULL: per trajectory a first-order bound on
                              the absolute rounding difference of its value between two fp64
                              implementations of the path (the parity tests' T2/T3 value bound):
                              2·max_k δy_k with, per observation y_k = μ_k + σ_k·z_k,
                                δy_k = n·u·κ_L·(Σ_j|kx_j c_j| + |z_k|·(ψ(0) + Σ_j|kx_j w_j|)/(2σ_k))
                                       + Σ_{i<k} |w_k[N+i]|·δy_i,
                              n = N + h, u = 2⁻⁵³, κ_L = ‖L0‖₁‖L0⁻¹‖₁ of the base factor, w = K⁻¹kx:
                              the rounding of μ's and σ²'s n-term sums amplified by the base
                              factor's conditioning (an explicit L0⁻¹ or substitution), σ² → σ
                              by 1/(2σ), and the earlier fantasy observations' errors through
                              ∂μ_k/∂y_i = w_k[N+i] (the conditions that feed resolve, rollout.jl:108-111);
                              Gauss–Hermite: × the largest weight/√π                          */
  double* ylip;            /* diagnostic output M×R, or NULL: max_k ‖∂y_k/∂x_k‖₁ = ‖∇μ + z_k∇σ‖₁ at the
                              trajectory's observations (first-order effect of a policy point's
                              own rounding difference on the value, T3)                       */
} rbo_params;

/* NonUniformCost (cost_functions.jl:5-20) as closed-form families.  The reference's cost is an
 * arbitrary closure that no rule, surrogate or trajectory references (SURVEY.md §0 finding 5);
 * the build defines the cost-weighted acquisition α(x)/c(x) of the inner policy solve with it
 * (parity unpinned).  u_a = (x_a − lb_a)/(ub_a − lb_a):
 *   QUADRATIC  c(x) = c0 + Σ_a w_a u_a²        LOGLINEAR  c(x) = c0 · exp(Σ_a w_a u_a)      */
enum { RBO_COST_NONE = 0, RBO_COST_QUADRATIC = 1, RBO_COST_LOGLINEAR = 2 };

/* base decision rules (decision_rules.jl:84-127) */
enum { RBO_RULE_EI = 0, RBO_RULE_POI = 1, RBO_RULE_LCB = 2 };

/* utils.jl:4-13: D×samples Sobol uniforms (zero point skipped), column-major. */
int rbo_gen_uniform(int32_t samples, int32_t dim, double* out);
/* utils.jl:65-74: M×(d+1)×H rnstream, Julia column-major layout. */
int rbo_gen_low_discrepancy_sequence(int32_t M, int32_t d, int32_t H, double* out);
/* utils.jl:145-153: d×(n+2) inner starts. */
int rbo_generate_initial_guesses(int32_t n, int32_t d, const double* lbs, const double* ubs, double* out);
/* low_discrepancy.jl:7-28 */
int rbo_kronecker_quasirand(int32_t d, int32_t N, int32_t start, double* out);
/* counter-based uniform used for solve_dual_y's δx when the caller supplies none */
double rbo_dual_uniform(uint64_t seed, int64_t traj, int32_t j, int32_t k);

/* Evaluate the base surrogate (fantasy_index = -1) at P points: per point writes
 * out[0]=μ, [1]=σ, [2]=α, [3..3+d)=∇μ, [3+d..3+2d)=∇σ, [3+2d..3+3d)=∇α,
 * [3+3d..3+3d+d²)=Hα (col-major), then d2α/dxdθ (d).  stride = 3+4d+d². */
int rbo_eval_base(const rbo_surrogate* s, int32_t rule, double theta, double sigma_tol, int32_t P,
                  const double* xs, double* out);
/* The same with the rule, θ, σtol and the NonUniformCost model of p (the cost-weighted α/c(x),
 * ∇, H and ∂∇/∂θ; p->lbs / p->ubs define u).                                              */
int rbo_eval_base_p(const rbo_surrogate* s, const rbo_params* p, int32_t P, const double* xs, double* out);

/* base_solve(s::Surrogate; xstart) (rbf_optim.jl:35-66) from each column of xstarts (d×n) on the
 * base surrogate with p's rule, θ, box and solver options: xmin d×n, fmin n (minima of −α),
 * status n, evals 3×n [gradient, value, Hessian] (optional).  The findmin of
 * multistart_base_solve!(s, …) (:103-135) is the caller's. */
int rbo_base_solve(const rbo_surrogate* s, const rbo_params* p, int32_t n, const double* xstarts, double* xmin,
                   double* fmin, int32_t* status, int64_t* evals);

/* simulate_trajectory_mc (rollout.jl:279-340) for R restarts x0s (d×R).
 * Outputs (caller-allocated, Julia layout):
 *   values   M×R, grad_x d×M×R, grad_theta 1×M×R, status M×R,
 *   policy_x d×(h+1)×M×R (optional), obs (h+1)×M×R (optional).
 * dual_y_dx: optional d×h×M×R uniforms (δx of solve_dual_y call j at column j-1).
 * replay_x:  optional d×h×M×R policy points injected instead of the inner solve.
 * eto: optional R×(2+2d+2) rows [μ, σ, ∇μx(d), σ∇x(d), ∇μθ, σ∇θ].
 * evals: optional 3×M×R inner-solve work per trajectory [gradient evals, value-only evals,
 *        Hessians] of the lazy Newton iteration (rbo_oracle.c newton_solve). */
int rbo_simulate_mc(const rbo_surrogate* s, const rbo_params* p, const double* x0s,
                    const double* rnstream, const double* xstarts,
                    const double* dual_y_dx, const double* replay_x,
                    double* values, double* grad_x, double* grad_theta, int32_t* status,
                    double* policy_x, double* obs, double* eto, int64_t* evals);

/* simulate_trajectory_ghq (rollout.jl:409-467): the Gauss–Hermite estimator.  Sample m uses the
 * node vector nodes[m, 0..h] and weights[m, 0..h] (M×(h+1), column-major), i.e. the caller's
 * nodes[indices[m]] / weights[indices[m]] (generate_indices, utils.jl:217-221); observations
 * y = μ + √2σ t (GaussHermiteObservable, observables.jl:32-81, 157); values weighted by
 * weights[best]/√π.  Other arguments and outputs as rbo_simulate_mc. */
int rbo_simulate_ghq(const rbo_surrogate* s, const rbo_params* p, const double* x0s, const double* nodes,
                     const double* weights, const double* xstarts, const double* dual_y_dx, const double* replay_x,
                     double* values, double* grad_x, double* grad_theta, int32_t* status, double* policy_x,
                     double* obs, double* eto, int64_t* evals);

/* Base-GP refit at lengthscale ell (Surrogate ctor, radial_basis_surrogates.jl:77-118) and its
 * log_likelihood (:770-776) and ∂/∂ℓ (∇log_likelihood :787-799 via δlog_likelihood :778-785).
 * Returns 1 (ll = dll = NaN) on PosDefException.  L_out (N×N, lower) and c_out optional. */
/* ∇log_likelihood over θ = (ℓ) or, for Periodic, (ℓ, p) (nt = 2; nt = 1 keeps `period`):
 * grad[t] = (cᵀδK_t c − tr(L'\(L\δK_t)))/2.  Returns 0, 1 (PosDefException), −1 (bad nt). */
int rbo_log_likelihood_theta(int32_t d, int32_t N, int32_t kernel, int32_t nt, const double* theta, double period,
                             double sigma_n2, const double* X, const double* y, double* ll, double* grad,
                             double* L_out, double* c_out);
int rbo_log_likelihood(int32_t d, int32_t N, int32_t kernel, double ell, double sigma_n2, const double* X,
                       const double* y, double* ll, double* dll, double* L_out, double* c_out);

/* Test functions (testfns.jl) used to make base data y. id: 0 GramacyLee, 1 BraninHoo,
 * 2 Hartmann6D, 3 Ackley(d), 4 Rosenbrock, 5 Rastrigin(d). */
double rbo_testfn(int32_t id, int32_t d, const double* x);

#ifdef __cplusplus
}
#endif
#endif
