/*
 * mrbo.h -- C ABI of the MI355X rollout-acquisition evaluator (libmrbo.so).
 *
 * Drop-in boundary for the reference's Monte-Carlo rollout path.  The reference is pure
 * Julia and has no FFI; each entry point below replaces one Julia function (file:line in
 * /root/reference) and is what a `ccall` shim binds (INTEGRATION.md shows the shim):
 *
 *   mrbo_simulate_mc       simulate_trajectory_mc(T, tp; inner_solve_xstarts, resolutions,
 *                          spatial_gradients_container, hyperparameter_gradients_container)
 *                          rollout.jl:279-340 -- batched over R restarts (the x0 batch of the
 *                          outer ascent, utils.jl:97-106 / stochastic_solve utils.jl:235-265)
 *   mrbo_eto_reduce        the mean / std(n-1) tail of simulate_trajectory_mc, rollout.jl:328-339
 *   mrbo_stochastic_solve  stochastic_solve utils.jl:235-265 (eswavs + StandardSGA / Adam update!)
 *                          over a restart batch, the whole ascent in one call
 *   mrbo_eval_base         eval(s::Surrogate, x, θ) radial_basis_surrogates.jl:224-310 (μ, σ, ∇, Hα)
 *   mrbo_rnstream          gen_low_discrepancy_sequence utils.jl:65-74 (Sobol→Box–Muller(log10))
 *   mrbo_initial_guesses   generate_initial_guesses utils.jl:145-153
 *   mrbo_gp_fit            Surrogate(ψ, X, y) radial_basis_surrogates.jl:77-118 and its
 *                          log_likelihood / ∇log_likelihood (:770-799) for a batch of
 *                          lengthscales -- the evaluations behind optimize! (:805-829)
 *
 * Conventions
 *   - Plain pointers and sizes; matrices are column-major with the reference's (Julia) shapes.
 *   - Arrays passed to mrbo_simulate_mc / mrbo_eto_reduce / mrbo_eval_base are DEVICE pointers
 *     (hipMalloc'd or from a framework allocator) unless MRBO_FLAG_HOST_POINTERS is set, in
 *     which case the library stages them through device memory (PCIe-inclusive).
 *   - The plan owns the device copy of the base surrogate and all workspace; a call never
 *     allocates (graph-capturable) and is re-entrant per (plan, stream) pair.
 *   - Return value: 0 on success, negative mrbo_err_t on argument/launch errors (message via
 *     mrbo_last_error()).  Per-trajectory numerical failures -- the reference's Julia
 *     exceptions -- are reported in status[] (MRBO_ST_*), never as a return code.
 */
#ifndef MRBO_H
#define MRBO_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

#define MRBO_ABI_VERSION 2

typedef enum {
  MRBO_OK = 0,
  MRBO_ERR_ARG = -1,      /* invalid argument (dimension, size, null pointer)            */
  MRBO_ERR_UNSUPPORTED = -2, /* shape outside the compiled kernels: d > 16, N > 512,
                                d > 8 with N > 128, h > 5 (gp_fit: N > 512) */
  MRBO_ERR_HIP = -3,      /* HIP runtime error                                          */
  MRBO_ERR_NOMEM = -4
} mrbo_err_t;

typedef enum {
  MRBO_KERNEL_MATERN52 = 0, /* radial_basis_functions.jl:60-68  */
  MRBO_KERNEL_MATERN32 = 1, /* :70-78 */
  MRBO_KERNEL_MATERN12 = 2, /* :80-88 */
  MRBO_KERNEL_SE = 3,       /* :90-96 */
  MRBO_KERNEL_PERIODIC = 4  /* :98-103  exp(−2 sin²(πρ/p)/ℓ²), p = mrbo_surrogate_t.period */
} mrbo_kernel_t;

typedef enum {
  MRBO_RULE_EI = 0,   /* decision_rules.jl:84-99   expected improvement                 */
  MRBO_RULE_POI = 1,  /* decision_rules.jl:101-115 probability of improvement           */
  MRBO_RULE_LCB = 2   /* decision_rules.jl:117-127 θσ − μ (negated lower confidence bound) */
} mrbo_rule_t;

/* NonUniformCost (cost_functions.jl:5-20: NonUniformCost(f) with ∇f, Hf) as closed-form families.
 * The reference's cost is an arbitrary closure referenced by no rule, surrogate or trajectory;
 * the build defines the cost-weighted acquisition f(x) = α(x)/c(x) of the inner policy solve
 * (α, ∇f, Hf, ∂∇f/∂θ and the adjoint perturbations all weighted; parity unpinned, the oracle
 * implements the same definition).  u_a = (x_a − lb_a)/(ub_a − lb_a) over the plan's box:
 *   MRBO_COST_QUADRATIC  c(x) = c0 + Σ_a w_a u_a²        MRBO_COST_LOGLINEAR  c(x) = c0·exp(Σ_a w_a u_a)
 * mrbo_plan_create refuses (MRBO_ERR_ARG) any model that is not positive on the box: c0 ≤ 0 or
 * non-finite, a non-finite weight, a negative QUADRATIC weight, or ub ≤ lb in some dimension. */
typedef enum { MRBO_COST_NONE = 0, MRBO_COST_QUADRATIC = 1, MRBO_COST_LOGLINEAR = 2 } mrbo_cost_t;

/* per-trajectory status bits: the reference's exceptions (SURVEY.md §8b "Errors") */
enum {
  MRBO_ST_OK = 0,
  MRBO_ST_SIGMA_NEG = 1,   /* DomainError sqrt(negative variance)   r_b_s.jl:528 */
  MRBO_ST_DRAW_NOT_PD = 2, /* PosDefException, gp_draw covariance    r_b_s.jl:537 */
  MRBO_ST_COND_NOT_PD = 4, /* PosDefException, update_cholesky!      r_b_s.jl:412 */
  MRBO_ST_ALL_NAN = 8,     /* findmin on an empty candidate list     rbf_optim.jl:96 */
  MRBO_ST_SINGULAR = 16    /* singular Hessian in solve_dual_x       rollout.jl:188 */
};

enum {
  MRBO_FLAG_HOST_POINTERS = 1, /* arrays are host memory; stage through the device  */
  MRBO_FLAG_NO_GRADIENT = 2    /* skip gradient(T): containers == nothing branch    */
};

/* Base GP surrogate (Surrogate struct, radial_basis_surrogates.jl:30-41), HOST memory. */
typedef struct {
  int32_t d;            /* input dimension                                        */
  int32_t N;            /* observed points (get_observed)                         */
  int32_t kernel;       /* mrbo_kernel_t                                          */
  double lengthscale;   /* ψ.θ[1]                                                 */
  double sigma_n2;      /* σn2                                                    */
  double fmini;         /* minimum(s.y) over the whole capacity buffer (Q3)       */
  const double* X;      /* d×N, column-major, leading dim d                       */
  const double* L;      /* N×N lower Cholesky factor of K, column-major, ld = ldL */
  int32_t ldL;
  const double* c;      /* N coefficients L'\(L\y)                                */
  const double* y;      /* N observations                                        */
  double period;        /* ψ.θ[2] of the Periodic kernel (unused otherwise)      */
} mrbo_surrogate_t;

/* TrajectoryParameters (trajectory.jl:43-94) + inner-solve options (rbf_optim.jl:24-30). */
typedef struct {
  int32_t h;            /* horizon (≤ 5)                                         */
  int32_t M;            /* MC samples per restart (tp.mc_iters)                  */
  int32_t R;            /* restarts (x0 batch)                                   */
  int32_t nstarts;      /* inner starts = columns of inner_solve_xstarts         */
  int32_t rule;         /* mrbo_rule_t                                           */
  double theta;         /* T.θ[1]: decision-rule hyperparameter (Q12: T.θ, not tp.θ) */
  const double* lbs;    /* d, HOST */
  const double* ubs;    /* d, HOST */
  int32_t max_iters;    /* inner Newton iterations per start      */
  int32_t max_ls;       /* backtracking steps                                    */
  double x_tol;         /* Optim x_tol (rbf_optim.jl:27) = 1e-3                  */
  double f_tol;         /* Optim f_tol = 1e-3                                    */
  double g_tol;         /* Optim default g_tol = 1e-8                            */
  double htol;          /* solve_dual_x det threshold (rollout.jl:156) = 1e-4    */
  double sigma_tol;     /* EI / POI σtol (decision_rules.jl:84, :102) = 1e-8     */
  uint64_t seed;        /* δx for solve_dual_y (rollout.jl:133) when dual_y_dx == NULL */
  int32_t sample_offset;/* global index of this plan's first MC sample (multi-GPU shard), 0 */
  int32_t samples_total;/* DEPRECATED, ignored (kept for the struct layout).  The δx counter */
                        /* RNG is keyed by the global sample index sample_offset + m alone */
                        /* (round 5), so all R restarts of a launch share the δx of sample */
                        /* m, and restart r equals an R = 1 launch at its x0.  The         */
                        /* reference draws a fresh rand(dim) per solve_dual_y call         */
                        /* (rollout.jl:133): restarts are NOT decorrelated. */
  int32_t cost;         /* mrbo_cost_t: NonUniformCost weighting of the inner-solve rule      */
  double cost_c0;       /* cost family parameter c0                                          */
  const double* cost_w; /* d weights, HOST (NULL with MRBO_COST_NONE)                        */
} mrbo_params_t;

typedef struct mrbo_plan mrbo_plan_t;

const char* mrbo_version(void);
const char* mrbo_last_error(void);
int mrbo_device_count(void);

/* Build the device state for (surrogate, params): copies X, L⁻¹ (packed), c; sizes the
 * persistent-wave grid and workspace.  `device` is a HIP ordinal.                         */
int mrbo_plan_create(const mrbo_surrogate_t* s, const mrbo_params_t* p, int32_t device, mrbo_plan_t** out);
int mrbo_plan_destroy(mrbo_plan_t* plan);

/* simulate_trajectory_mc for the R×M trajectories of the plan.
 *   x0s        d×R          start of each restart (tp.x0 / set_start!, rollout.jl:287)
 *   rnstream   M×(d+1)×(h+1) tp.rnstream_sequence (trajectory.jl:52-68), shared by restarts
 *   xstarts    d×nstarts    inner_solve_xstarts
 *   dual_y_dx  d×h×M×R or NULL: δx of solve_dual_y call j (column j-1); NULL → counter RNG(seed)
 *   replay_x   d×h×M×R or NULL: inject policy points x_1..x_h instead of the inner solve
 *   values     M×R          resolutions
 *   grad_x     d×M×R        spatial_gradients_container          (may be NULL with NO_GRADIENT)
 *   grad_theta 1×M×R        hyperparameter_gradients_container   (may be NULL with NO_GRADIENT)
 *   status     M×R          MRBO_ST_* bits
 *   policy_x   d×(h+1)×M×R or NULL: x_0..x_h of every trajectory (fs.X[:, N+1:N+h+1])
 *   obs        (h+1)×M×R or NULL:   sampled observations y_0..y_h
 *   evals      MRBO_NCOUNTERS×M×R or NULL: per trajectory [gradient evals, value-only evals,
 *              Hessian completions, adjoint rich evals, adjoint perturbation pairs] -- the work
 *              counters of the FLOP roofline model (inner-solve counts are identical to the
 *              oracle's: same lazy Newton iteration)
 * Launches on `stream` (hipStream_t, may be NULL) and returns without synchronising.       */
int mrbo_simulate_mc(mrbo_plan_t* plan, const double* x0s, const double* rnstream, const double* xstarts,
                     const double* dual_y_dx, const double* replay_x, double* values, double* grad_x,
                     double* grad_theta, int32_t* status, double* policy_x, double* obs, int64_t* evals,
                     uint32_t flags, void* stream);

#define MRBO_NCOUNTERS 5

/* simulate_trajectory_ghq(T, tp; inner_solve_xstarts, resolutions, nodes, weights, indices, …)
 * rollout.jl:409-467 — the Gauss–Hermite estimator.  Sample m (of M = length(indices)) uses the
 * node vector nodes[m, 0..h] = nodes[indices[m]] and weights[m, 0..h] = weights[indices[m]]
 * (M×(h+1), column-major; generate_indices utils.jl:217-221 builds the tensor product): step k
 * observes y = μ + √2·σ·t_k with recorded gradient weights[k]·(∇μ + √2·∇σ·t_k)
 * (GaussHermiteObservable observables.jl:32-81, get_gradient :157) and the resolution is
 * weights[best]·max(fmini − y_best, 0)/√π.  All other arguments and outputs as mrbo_simulate_mc
 * (the plan's M is the number of node vectors).                                              */
int mrbo_simulate_ghq(mrbo_plan_t* plan, const double* x0s, const double* nodes, const double* weights,
                      const double* xstarts, const double* dual_y_dx, const double* replay_x, double* values,
                      double* grad_x, double* grad_theta, int32_t* status, double* policy_x, double* obs,
                      int64_t* evals, uint32_t flags, void* stream);

/* ExpectedTrajectoryOutput per restart: eto R×W (row-major per restart, W = 2+2d+2):
 * [μxθ, σ_μxθ, ∇μx(d), σ_∇μx(d), ∇μθ, σ_∇μθ]; std uses n-1 (Q14).                     */
int mrbo_eto_reduce(mrbo_plan_t* plan, const double* values, const double* grad_x, const double* grad_theta,
                    double* eto, uint32_t flags, void* stream);

/* One step of the outer stochastic gradient ascent for the plan's R restarts, on the device
 * (stochastic_solve utils.jl:235-265): for every restart r with active[r] ≠ 0, eswavs
 * (utils.jl:114-123) on the ETO row r of eto (mrbo_eto_reduce's layout) with sample_size = the
 * global MC samples -- 1 − (sample_size/d)·Σ_a ∇μx_a²/σ_∇μx_a² > 0 sets active[r] = 0 -- else
 * StandardSGA update! (optimizers.jl:16-22) x0s[:, r] += η·∇μx.  Device pointers only (eto R×W,
 * x0s d×R, active R int32); asynchronous on `stream`, so consecutive launches of the ascent need
 * no host round trip.                                                                           */
int mrbo_sga_step(mrbo_plan_t* plan, const double* eto, double* x0s, int32_t* active, double sample_size, double eta,
                  uint32_t flags, void* stream);

/* The same step with Adam update! (optimizers.jl:49-74) in place of StandardSGA: m, v (device,
 * d×R, zero before the first update) are the restarts' moment estimates, t ≥ 1 the update count
 * of the active restarts (a restart that eswavs stops never updates again, so the active ones
 * share it); x0s[:, r] += η·m̂/(√v̂ + ε) with m̂ = m/(1 − β1^t), v̂ = v/(1 − β2^t).  The reference's
 * defaults: η = 0.001, β1 = 0.9, β2 = 0.999, ε = 1e-8 (optimizers.jl:35-40).                 */
int mrbo_adam_step(mrbo_plan_t* plan, const double* eto, double* x0s, int32_t* active, double* m, double* v, int32_t t,
                   double sample_size, double eta, double beta1, double beta2, double eps, uint32_t flags,
                   void* stream);

/* The reference's outer loop in ONE call: stochastic_solve(; optimizer, surrogate, tp, es, start)
 * (utils.jl:235-265) for the plan's R restarts at once -- the columns of x0s, e.g. the
 * generate_batch points (utils.jl:97-106) -- on the plan's surrogate, TrajectoryParameters and
 * inner starts.  Each iteration is [mrbo_simulate_mc at the current x0s, mrbo_eto_reduce,
 * mrbo_sga_step (StandardSGA update!, optimizers.jl:16-22) or mrbo_adam_step (Adam update!,
 * optimizers.jl:49-74)], at most opts->iterations (the reference: 50) times.  A restart stops
 * for good when its eswavs test (utils.jl:114-123) fires, as the reference's `break`; the call
 * returns once no restart is active (read back a few iterations behind the launches: the
 * iterations queued after the last stop find x0 unchanged and reproduce the same outputs) or the
 * budget is spent.  No host round trip per iteration, one plan, no plan rebuild.
 *   x0s      d×R in: the starts, out: get_starting_point(tpc) of every restart
 *   rnstream, xstarts, dual_y_dx   as mrbo_simulate_mc (dual_y_dx may be NULL)
 *   eto      R×W or NULL: the ETO rows (mrbo_eto_reduce's layout) of the last launch -- for a
 *            stopped restart, those at its final point
 *   active   R or NULL: 1 where eswavs never stopped the restart within the budget
 *   result   int32[3]: iterations launched, the iteration after which no restart was active (or
 *            the iterations launched), the OR of every launch's trajectory status bits (non-zero:
 *            the reference would have thrown -- the Julia method throws)
 * Arrays are device pointers unless MRBO_FLAG_HOST_POINTERS (then staged once for the whole
 * ascent); synchronises `stream` before returning.                                            */
typedef enum { MRBO_OPT_SGA = 0, MRBO_OPT_ADAM = 1 } mrbo_optimizer_t;
typedef struct {
  int32_t optimizer;    /* mrbo_optimizer_t                                                  */
  int32_t iterations;   /* ≥ 1; the reference's loop: 50                                      */
  double eta;           /* StandardSGA η (default 0.01) / Adam η (default 0.001)              */
  double beta1;         /* Adam β1 (0.9); ignored by StandardSGA                              */
  double beta2;         /* Adam β2 (0.999)                                                    */
  double eps;           /* Adam ε (1e-8)                                                      */
  double sample_size;   /* eswavs sample size: global MC samples per restart (0 → the plan's M) */
} mrbo_solve_opts_t;
int mrbo_stochastic_solve(mrbo_plan_t* plan, double* x0s, const double* rnstream, const double* xstarts,
                          const double* dual_y_dx, const mrbo_solve_opts_t* opts, double* eto, int32_t* active,
                          int32_t* result, uint32_t flags, void* stream);

/* Shard moments for the multi-GPU exchange: moments R×(2+2d+2) = [Σα, M2α, Σ∇x(d), M2∇x(d), Σ∇θ, M2∇θ]
 * over the first M_local samples of each restart (the outputs keep the plan's M as the restart
 * stride; 1 ≤ M_local ≤ M), M2 = Σ(x − x̄_local)² by two passes.  Ranks all-gather
 * (n, Σ, M2) and merge them with Chan's formula (mrbo/parallel.py merge_moments), which gives the
 * two-pass mean / std(n-1) of rollout.jl:328-339 without one-pass cancellation.            */
int mrbo_partial_moments(mrbo_plan_t* plan, const double* values, const double* grad_x, const double* grad_theta,
                         int32_t M_local, double* moments, uint32_t flags, void* stream);

/* The exchange's merge on the device (no host round trip per SGA step): moments = the nshards
 * ranks' mrbo_partial_moments blocks concatenated in rank order (nshards × R×W, what one
 * all-gather of the flat blocks produces), counts = their sample counts (HOST int64[nshards],
 * the shard sizes every rank knows; 1 ≤ nshards ≤ 64, a zero-count shard is skipped).  Chan's
 * pairwise merge left to right, then the ETO rows (mrbo_eto_reduce's layout, std n−1, Q14) into
 * eto (device, R×W) -- the same operations in the same order as mrbo/parallel.py merge_moments +
 * eto_from_moments.  Device pointers only; asynchronous on `stream`.                       */
int mrbo_merge_moments(mrbo_plan_t* plan, int32_t nshards, const double* moments, const int64_t* counts, double* eto,
                       uint32_t flags, void* stream);

/* eval(s, x, θ) of the base surrogate at P points xs (d×P); out stride 3+4d+d²:
 * [μ, σ, α, ∇μ(d), ∇σ(d), ∇α(d), Hα(d×d col-major), d2α/dxdθ(d)].                       */
int mrbo_eval_base(mrbo_plan_t* plan, int32_t P, const double* xs, double* out, uint32_t flags, void* stream);

/* base_solve(s::Surrogate; spatial_lbs, spatial_ubs, xstart, θfixed) rbf_optim.jl:35-66 for each
 * of n starts (columns of xstarts, d×n; any n ≥ 1) on the plan's BASE surrogate, with the plan's
 * rule, θ, box and solver options (the build's projected Newton, DESIGN.md §3, as the rollout's
 * inner solve): xmin d×n = the minimizers, fmin n = the minima of −α, status n (MRBO_ST_* bits
 * except ALL_NAN), evals MRBO_NCOUNTERS×n or NULL.  One wavefront per start.  The caller takes
 * multistart_base_solve!'s findmin over the candidates (rbf_optim.jl:103-135: drop minimizers
 * with a NaN, a NaN minimum wins, else the first minimum) -- mrbo/rbf_optim.py does.  Arrays are
 * device pointers unless MRBO_FLAG_HOST_POINTERS; launches on `stream` without synchronising. */
int mrbo_base_solve(mrbo_plan_t* plan, int32_t n, const double* xstarts, double* xmin, double* fmin, int32_t* status,
                    int64_t* evals, uint32_t flags, void* stream);

/* Base-GP fit at P hyperparameter vectors θ_p = thetas[p·nt .. p·nt+nt−1] (kernel, σn2, X d×N,
 * y N from s; s->L, s->c unused) -- the evaluations behind optimize!'s fg! (r_b_s.jl:810-814):
 * K = Ψ(‖Xi−Xj‖; θ_p)+σn2·I, L = chol(K), c = L'\(L\y), and
 *   ll[p]         = log_likelihood  (r_b_s.jl:770-776) = −yᵀc/2 − Σ log L_ii − N·log(2π)/2
 *   grad[p·nt+t]  = ∇log_likelihood (r_b_s.jl:787-799) = (cᵀ δK_t c − tr(L'\(L\δK_t)))/2,
 *                   δK_t = eval_Dθ_KXX(ψ, X, e_t) (radial_basis_functions.jl:264-284)
 * θ = (ℓ) for Matérn-5/2, -3/2, -1/2 and SE (nt = 1); Periodic (radial_basis_functions.jl:98-103)
 * takes θ = (ℓ, p) (nt = 2) or (ℓ) with p = s->period (nt = 1: ∂/∂ℓ only).
 * status[p] = 0, or 1 when cholesky throws PosDefException (ll, grad = NaN).  L_out (N×N×P,
 * lower, zeros above) and c_out (N×P) are optional (NULL).  thetas / ll / grad / status / L_out
 * / c_out are device pointers unless MRBO_FLAG_HOST_POINTERS; N ≤ 512 (every N the rollout
 * accepts).  Kernel by size: N ≤ 32 (and any N > 80) runs the 32 × 32-tile kernel on the fp64
 * matrix cores with ((2 + nt)·T(T+1)/2 + T)·1024·P doubles of workspace, T = ⌈N/32⌉, from the
 * per-device pool; 32 < N ≤ 64 with d ≤ 16 and without L_out / c_out runs the register kernel
 * (one candidate per workgroup, no workspace); otherwise 32 < N ≤ 80 with d ≤ 16 runs the LDS
 * kernel (the candidate in LDS, no workspace); d > 16 runs the tile kernel.  A configuration whose LDS (dynamic + the kernel's static arrays) exceeds
 * the device limit fails with MRBO_ERR_UNSUPPORTED.  Synchronises the stream before returning. */
int mrbo_gp_fit_theta(const mrbo_surrogate_t* s, int32_t P, int32_t nt, const double* thetas, double* ll,
                      double* grad, int32_t* status, double* L_out, double* c_out, uint32_t flags, void* stream);
/* mrbo_gp_fit_theta with nt = 1: ells[p] = ℓ_p, dll[p] = ∂ll/∂ℓ (Periodic: p = s->period). */
int mrbo_gp_fit(const mrbo_surrogate_t* s, int32_t P, const double* ells, double* ll, double* dll, int32_t* status,
                double* L_out, double* c_out, uint32_t flags, void* stream);

/* Host helpers (HOST memory). */
int mrbo_rnstream(int32_t M, int32_t d, int32_t H, double* out);                 /* M×(d+1)×H */
int mrbo_initial_guesses(int32_t n, int32_t d, const double* lbs, const double* ubs, double* out); /* d×(n+2) */
double mrbo_dual_uniform(uint64_t seed, int64_t traj, int32_t j, int32_t k);

/* Timing of the last mrbo_simulate_mc / _ghq rollout kernel on its stream (HIP events around the
 * kernel launch alone), milliseconds; -1 before the first launch.  Waits for that launch.      */
double mrbo_last_kernel_ms(mrbo_plan_t* plan);

/* The same for the plan's last min(n, launches, 64) launches, oldest first, into ms[]; returns the
 * number written (≥ 0) or a negative mrbo_err_t.  Waits for those launches.                    */
int mrbo_kernel_times(mrbo_plan_t* plan, int32_t n, double* ms);

/* Kernel time of the last mrbo_gp_fit launch (HIP events around it), milliseconds; -1 before
 * the first call.  Process-wide (the last call on any stream). */
double mrbo_last_gp_fit_ms(void);

/* Launch geometry of a plan (no reference counterpart; measurement and FLOP accounting):
 * info[0..6] = rows per lane (1/2/4), workgroups, waves per workgroup, batched start values
 * (0/1), compile-time specialised kernel (0 generic, 1 Matérn-5/2 + EI, 2 its half-wave form: N ≤ 32, d ≤ 4, h ≤ 3, 3 Matérn-5/2 + EI + quadratic cost), LDS bytes per workgroup,
 * fantasy capacity of the kernel unit (4: the FMAX = 4 units of h ≤ 3, d ≤ 8; else 6).  Writes min(n, 7). */
int mrbo_plan_info(const mrbo_plan_t* plan, int32_t* info, int32_t n);

/* Work order of the plan's later mrbo_simulate_mc / mrbo_simulate_ghq launches (no reference
 * counterpart; scheduling only, results do not depend on it): `order` is a DEVICE array of n =
 * M×R int32 trajectory indices (m + M·r), a permutation, handed to the persistent waves in that
 * order -- e.g. longest first by the previous launch's work counters, which shortens the launch's
 * tail.  Caller-owned; it must stay valid while launches use it.  NULL restores the identity.
 * n != M×R: MRBO_ERR_ARG.  An entry outside [0, M×R) runs the trajectory of its own queue index
 * (no write outside the outputs); tests/test_gpu_schedule.py holds every output bit-identical
 * under permuted, out-of-range and longest-first orders.  The library does not check that the
 * order is a permutation: with a duplicated index (or a mix of out-of-range entries and valid
 * ones that name the same trajectory) one trajectory runs on two waves at once and another never
 * runs -- its outputs are left undefined.  The Python mirror (RolloutPlan.set_order) checks. */
int mrbo_plan_set_order(mrbo_plan_t* plan, const int32_t* order, int64_t n);

/* The same, with the order computed on the device by the library (no reference counterpart;
 * scheduling only): `evals` is a DEVICE array of M×R×5 work counters as a previous
 * mrbo_simulate_mc on this plan wrote them.  The rollout kernel's waves drain one queue per XCD
 * over a contiguous eighth of the queue positions, chunk x = [x·T/8, (x+1)·T/8), before the
 * others; the order keeps every trajectory in its own chunk and puts each chunk's trajectories
 * longest first by their weighted work (grad 2.5, value 1, Hessian 3, adjoint rich evaluation 5,
 * adjoint pair 3, in value-evaluation units; one stable descending radix sort, ties in index
 * order), so the launch no longer ends on its longest trajectories and each XCD still writes one
 * contiguous range of output rows.  The plan owns the order (grown on demand, freed with the
 * plan); the plan's later launches use it until mrbo_plan_set_order replaces it (NULL:
 * identity).  Stream-ordered: no host round trip.  `order_out` (DEVICE, M×R int32, or NULL)
 * receives a copy of the order.  mrbo_stochastic_solve does this after its first launch when the
 * caller has set no order.  M×R ≥ 2^31: MRBO_ERR_ARG.                                          */
int mrbo_plan_order_longest_first(mrbo_plan_t* plan, const int64_t* evals, int32_t* order_out, void* stream);

#ifdef __cplusplus
}
#endif
#endif
