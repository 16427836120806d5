/*
 * rbo_oracle.c -- CPU restatement of the Rollout-Bayesian-Optimization hot path.
 *
 * TEST INFRASTRUCTURE (parity checker + cpu_baseline port).  See rbo_oracle.h for the
 * rules; every function cites the reference file:line it restates.  Layout is Julia's:
 * column-major matrices, 0-based indices here where Julia is 1-based.
 *
 * Parity: UNPINNED against Julia (no julia binary, no golden vectors in the reference).
 */
#include "rbo_oracle.h"
#include "sobol_table_oracle.h"

#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define JL_PI 3.141592653589793           /* Julia π as Float64                       */
#define INVSQRT2 0.7071067811865476        /* StatsFuns.invsqrt2                       */
#define SQRT2 1.4142135623730951
#define SQRTPI 1.7724538509055159
#define INVSQRT2PI 0.3989422804014327      /* StatsFuns.invsqrt2π                      */

/* ------------------------------------------------------------------------------------
 * Sobol (Sobol.jl SobolSeq / next!, Joe-Kuo directions, Gray-code order, zero skipped)
 * ---------------------------------------------------------------------------------- */
typedef struct {
  int dim;
  uint32_t v[RBO_ORACLE_SOBOL_TABLE_MAXDIM][32];
  uint32_t x[RBO_ORACLE_SOBOL_TABLE_MAXDIM];
  uint64_t n;
} sobol_t;

static int sobol_init(sobol_t* s, int dim) {
  if (dim < 1 || dim > RBO_ORACLE_SOBOL_TABLE_MAXDIM) return -1;
  s->dim = dim;
  s->n = 0;
  for (int j = 0; j < dim; ++j) {
    s->x[j] = 0;
    const int deg = rbo_oracle_sobol_table[j].s;
    const int a = rbo_oracle_sobol_table[j].a;
    uint32_t m[33];
    if (deg == 0) {
      for (int k = 1; k <= 32; ++k) m[k] = 1;
    } else {
      for (int k = 1; k <= deg; ++k) m[k] = rbo_oracle_sobol_table[j].m[k - 1];
      for (int k = deg + 1; k <= 32; ++k) {
        uint32_t mk = m[k - deg] ^ (m[k - deg] << deg);
        for (int l = 1; l <= deg - 1; ++l) {
          if ((a >> (deg - 1 - l)) & 1) mk ^= m[k - l] << l;
        }
        m[k] = mk;
      }
    }
    for (int k = 1; k <= 32; ++k) s->v[j][k - 1] = m[k] << (32 - k);
  }
  return 0;
}

/* next point, u in [0,1) -- point index n = 1, 2, ... (the zero point is skipped) */
static void sobol_next(sobol_t* s, double* u) {
  uint64_t n = s->n;
  int c = 0;
  while ((n >> c) & 1ULL) ++c; /* lowest zero bit of n == ctz(n+1) */
  for (int j = 0; j < s->dim; ++j) {
    s->x[j] ^= s->v[j][c];
    u[j] = (double)s->x[j] / 4294967296.0;
  }
  s->n = n + 1;
}

int rbo_gen_uniform(int32_t samples, int32_t dim, double* out) {
  sobol_t s;
  if (sobol_init(&s, dim)) return -1;
  for (int32_t j = 0; j < samples; ++j) sobol_next(&s, out + (int64_t)j * dim);
  return 0;
}

/* utils.jl:23-43 (log10 quirk Q1) + utils.jl:65-74 reshape (Q2) */
int rbo_gen_low_discrepancy_sequence(int32_t M, int32_t d, int32_t H, double* out) {
  const int offset = ((d + 1) % 2 == 1) ? 1 : 0;
  const int Dp = d + 1 + offset;
  const int64_t cols = (int64_t)M * H;
  double* S = (double*)malloc(sizeof(double) * Dp * cols);
  double* Nm = (double*)malloc(sizeof(double) * Dp * cols);
  if (!S || !Nm) { free(S); free(Nm); return -2; }
  if (rbo_gen_uniform((int32_t)cols, Dp, S)) { free(S); free(Nm); return -1; }
  for (int64_t j = 0; j < cols; ++j) {
    const double* x = S + j * Dp;
    double* y = Nm + j * Dp;
    for (int i = 0; i < Dp; ++i) { /* 1-based i odd <=> 0-based i even */
      if (i % 2 == 0) y[i] = sqrt(-2.0 * log10(x[i])) * cos(2.0 * JL_PI * x[i + 1]);
      else y[i] = sqrt(-2.0 * log10(x[i - 1])) * sin(2.0 * JL_PI * x[i]);
    }
  }
  /* reshape(N, M, Dp, H) then drop the padded component */
  for (int t = 0; t < H; ++t)
    for (int k = 0; k < d + 1; ++k)
      for (int m = 0; m < M; ++m) {
        const int64_t l = (int64_t)m + (int64_t)M * k + (int64_t)M * Dp * t;
        out[(int64_t)m + (int64_t)M * k + (int64_t)M * (d + 1) * t] = Nm[l];
      }
  free(S);
  free(Nm);
  return 0;
}

/* utils.jl:145-153 */
int rbo_generate_initial_guesses(int32_t n, int32_t d, const double* lbs, const double* ubs, double* out) {
  sobol_t s;
  double u[RBO_ORACLE_SOBOL_TABLE_MAXDIM];
  if (sobol_init(&s, d)) return -1;
  for (int32_t j = 0; j < n; ++j) {
    sobol_next(&s, u);
    for (int i = 0; i < d; ++i) out[(int64_t)j * d + i] = lbs[i] + (ubs[i] - lbs[i]) * u[i];
  }
  for (int i = 0; i < d; ++i) out[(int64_t)n * d + i] = lbs[i] + 1e-6;
  for (int i = 0; i < d; ++i) out[(int64_t)(n + 1) * d + i] = ubs[i] - 1e-6;
  return 0;
}

/* low_discrepancy.jl:7-28 */
int rbo_kronecker_quasirand(int32_t d, int32_t N, int32_t start, double* out) {
  double phi = 1.0 + 1.0 / d;
  for (int k = 0; k < 10; ++k) {
    double g = pow(phi, d + 1) - phi - 1.0;
    double dg = (d + 1) * pow(phi, d) - 1.0;
    phi -= g / dg;
  }
  for (int j = 0; j < N; ++j)
    for (int i = 0; i < d; ++i) {
      double alpha = fmod(1.0 / pow(phi, i + 1), 1.0);
      out[(int64_t)j * d + i] = fmod(0.5 + (double)(start + j + 1) * alpha, 1.0);
    }
  return 0;
}

/* splitmix64 finaliser; counter-based uniform in [0,1) shared bit-for-bit with the GPU */
static uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}
double rbo_dual_uniform(uint64_t seed, int64_t traj, int32_t j, int32_t k) {
  uint64_t key = splitmix64(seed ^ 0x5851F42D4C957F2DULL);
  key = splitmix64(key ^ (uint64_t)traj);
  key = splitmix64(key ^ ((uint64_t)(uint32_t)j << 32 | (uint32_t)k));
  return (double)(key >> 11) * (1.0 / 9007199254740992.0);
}

/* ------------------------------------------------------------------------------------
 * testfns.jl (only used to make base observations y)
 * ---------------------------------------------------------------------------------- */
double rbo_testfn(int32_t id, int32_t d, const double* x) {
  switch (id) {
    case 0: /* TestGramacyLee testfns.jl:227-235 */
      return sin(10 * JL_PI * x[0]) / (2 * x[0]) + pow(x[0] - 1.0, 4);
    case 1: { /* TestBraninHoo testfns.jl:136-152 */
      const double a = 1, b = 5.1 / (4 * JL_PI * JL_PI), c = 5 / JL_PI, r = 6, s = 10, t = 1 / (8 * JL_PI);
      const double u = x[1] - b * x[0] * x[0] + c * x[0] - r;
      return a * u * u + s * (1 - t) * cos(x[0]) + s;
    }
    case 2: { /* TestHartmann6D testfns.jl:532-565 */
      static const double al[4] = {1.0, 1.2, 3.0, 3.2};
      static const double A[4][6] = {{10, 3, 17, 3.5, 1.7, 8}, {0.05, 10, 17, 0.1, 8, 14},
                                     {3, 3.5, 1.7, 10, 17, 8}, {17, 8, 0.05, 10, 0.1, 14}};
      static const double P[4][6] = {{1312, 1696, 5569, 124, 8283, 5886}, {2329, 4135, 8307, 3736, 1004, 9991},
                                      {2348, 1451, 3522, 2883, 3047, 6650}, {4047, 8828, 8732, 5743, 1091, 381}};
      double f = 0.0;
      for (int i = 0; i < 4; ++i) {
        double tt = 0.0;
        for (int j = 0; j < 6; ++j) {
          const double pij = 1e-4 * P[i][j];
          tt += A[i][j] * (x[j] - pij) * (x[j] - pij);
        }
        f += al[i] * exp(-tt);
      }
      return -f;
    }
    case 3: { /* TestAckley testfns.jl:173-199 */
      const double a = 20.0, b = 0.2, c = 2 * JL_PI;
      double nx = 0, cx = 0;
      for (int i = 0; i < d; ++i) { nx += x[i] * x[i]; cx += cos(c * x[i]); }
      nx = sqrt(nx);
      return -a * exp(-b / sqrt((double)d) * nx) - exp(cx / d) + a + exp(1.0);
    }
    case 4: /* TestRosenbrock */
      return (1 - x[0]) * (1 - x[0]) + 100 * (x[1] - x[0] * x[0]) * (x[1] - x[0] * x[0]);
    case 5: { /* TestRastrigin */
      double f = 10.0 * d;
      for (int i = 0; i < d; ++i) f += x[i] * x[i] - 10 * cos(2 * JL_PI * x[i]);
      return f;
    }
  }
  return NAN;
}

/* ------------------------------------------------------------------------------------
 * Kernels: radial_basis_functions.jl:60-103 (ψ) and the ρ-derivatives that
 * compute_derivatives (:41-46) takes by ForwardDiff -- restated in closed form.
 * ---------------------------------------------------------------------------------- */
typedef struct { int kind; double ell, per; } kern_t;

/* Periodic (:98-103): ψ = exp(−2 sin²(πρ/p)/ℓ²).  With A = 2π/(pℓ²), B = 2π/p, t = Bρ:
 * ψ' = −ψ A sin t,  ψ'' = ψ (A² sin²t − A B cos t). */
#define PER_A(k) (2 * JL_PI / ((k)->per * (k)->ell * (k)->ell))
#define PER_B(k) (2 * JL_PI / (k)->per)

static double k_psi(const kern_t* k, double rho) {
  switch (k->kind) {
    case RBO_K_MATERN52: { const double c = sqrt(5.0) / k->ell, s = c * rho; return (1 + s * (1 + s / 3.0)) * exp(-s); }
    case RBO_K_MATERN32: { const double c = sqrt(3.0) / k->ell, s = c * rho; return (1 + s) * exp(-s); }
    case RBO_K_MATERN12: { const double s = rho / k->ell; return exp(-s); }
    case RBO_K_PERIODIC: { const double sn = sin(JL_PI * rho / k->per); return exp(-2 * sn * sn / (k->ell * k->ell)); }
    default: return exp(-rho * rho / (2 * k->ell * k->ell));
  }
}
static double k_dpsi(const kern_t* k, double rho) {
  switch (k->kind) {
    case RBO_K_MATERN52: { const double c = sqrt(5.0) / k->ell, s = c * rho; return -c * (s / 3.0) * (1 + s) * exp(-s); }
    case RBO_K_MATERN32: { const double c = sqrt(3.0) / k->ell, s = c * rho; return -c * s * exp(-s); }
    case RBO_K_MATERN12: { const double c = 1.0 / k->ell; return -c * exp(-c * rho); }
    case RBO_K_PERIODIC: return -k_psi(k, rho) * PER_A(k) * sin(PER_B(k) * rho);
    default: { const double l2 = k->ell * k->ell; return -(rho / l2) * exp(-rho * rho / (2 * l2)); }
  }
}
static double k_d2psi(const kern_t* k, double rho) {
  switch (k->kind) {
    case RBO_K_MATERN52: { const double c = sqrt(5.0) / k->ell, s = c * rho; return c * c * (s * s - s - 1) * exp(-s) / 3.0; }
    case RBO_K_MATERN32: { const double c = sqrt(3.0) / k->ell, s = c * rho; return c * c * (s - 1) * exp(-s); }
    case RBO_K_MATERN12: { const double c = 1.0 / k->ell; return c * c * exp(-c * rho); }
    case RBO_K_PERIODIC: {
      const double A = PER_A(k), B = PER_B(k), t = B * rho, st = sin(t);
      return k_psi(k, rho) * (A * A * st * st - A * B * cos(t));
    }
    default: { const double l2 = k->ell * k->ell; return (rho * rho / (l2 * l2) - 1.0 / l2) * exp(-rho * rho / (2 * l2)); }
  }
}

static double vnorm(const double* r, int d) { /* LinearAlgebra.generic_norm2 (unscaled branch) */
  double s = 0;
  for (int i = 0; i < d; ++i) s += r[i] * r[i];
  return sqrt(s);
}

/* eval_∇k radial_basis_functions.jl:127-134 */
static void eval_grad_k(const kern_t* k, const double* r, int d, double* out) {
  const double rho = vnorm(r, d);
  if (rho == 0) { for (int i = 0; i < d; ++i) out[i] = 0; return; }
  const double dp = k_dpsi(k, rho);
  for (int i = 0; i < d; ++i) out[i] = dp * (r[i] / rho);
}
/* eval_Hk radial_basis_functions.jl:141-150, H col-major d×d */
static void eval_Hk(const kern_t* k, const double* r, int d, double* H) {
  const double p = vnorm(r, d);
  if (p > 0) {
    const double Dpr = k_dpsi(k, p) / p, D2 = k_d2psi(k, p);
    for (int b = 0; b < d; ++b)
      for (int a = 0; a < d; ++a)
        H[a + d * b] = (D2 - Dpr) * (r[a] / p) * (r[b] / p) + (a == b ? Dpr : 0.0);
  } else {
    const double D2 = k_d2psi(k, 0.0);
    for (int b = 0; b < d; ++b)
      for (int a = 0; a < d; ++a) H[a + d * b] = (a == b) ? D2 : 0.0;
  }
}

/* ------------------------------------------------------------------------------------
 * EI (decision_rules.jl:84-99) and the partials DecisionRule takes by ForwardDiff
 * (:23-34) -- closed forms; all zero when σ < σtol (the branch returns a constant).
 * ---------------------------------------------------------------------------------- */
typedef struct { double g, gmu, gsig, gth, gmumu, gsigsig, gthth, gmuth, gsigth; } ei_t;

static double normcdf(double z) { return erfc(-z * INVSQRT2) / 2; }
static double normpdf(double z) { return exp(-(z * z) / 2) * INVSQRT2PI; }

/* POI (decision_rules.jl:101-115): g = Φ(z), zero for σ < σtol; closed-form partials with
 * z_μ = z_θ = −1/σ, z_σ = −z/σ, φ' = −zφ.  LCB (:117-127): g = θσ − μ (no σtol branch). */
static ei_t rule_partials(int rule, double mu, double sig, double theta, double fmin, double sigma_tol) {
  ei_t e;
  memset(&e, 0, sizeof e);
  if (rule == RBO_RULE_LCB) {
    e.g = theta * sig - mu;
    e.gmu = -1.0;
    e.gsig = theta;
    e.gth = sig;
    e.gsigth = 1.0;
    return e;
  }
  if (sig < sigma_tol) return e;
  if (rule == RBO_RULE_POI) {
    const double z = (fmin - mu - theta) / sig;
    const double Phi = normcdf(z), phi = normpdf(z), s2 = sig * sig;
    e.g = Phi;
    e.gmu = -phi / sig;
    e.gsig = -z * phi / sig;
    e.gth = -phi / sig;
    e.gmumu = -z * phi / s2;
    e.gsigsig = z * phi * (2.0 - z * z) / s2;
    e.gthth = -z * phi / s2;
    e.gmuth = -z * phi / s2;
    e.gsigth = phi * (1.0 - z * z) / s2;
    return e;
  }
  const double imp = fmin - mu - theta;
  const double z = imp / sig;
  const double Phi = normcdf(z), phi = normpdf(z);
  e.g = imp * Phi + sig * phi;
  e.gmu = -Phi;
  e.gsig = phi;
  e.gth = -Phi;
  e.gmumu = phi / sig;
  e.gsigsig = z * z * phi / sig;
  e.gthth = phi / sig;
  e.gmuth = phi / sig;
  e.gsigth = z * phi / sig;
  return e;
}

/* ------------------------------------------------------------------------------------
 * Triangular solves: the reference solves with SubArray views of LowerTriangular,
 * which LinearAlgebra routes to plain substitution (Q16).  L col-major, ld.
 * ---------------------------------------------------------------------------------- */
static void lsolve(const double* L, int ld, int n, const double* b, double* x) { /* L\b */
  for (int j = 0; j < n; ++j) {
    double s = b[j];
    for (int i = 0; i < j; ++i) s -= L[j + (int64_t)ld * i] * x[i];
    x[j] = s / L[j + (int64_t)ld * j];
  }
}
static void ltsolve(const double* L, int ld, int n, const double* b, double* x) { /* L'\b */
  for (int j = n - 1; j >= 0; --j) {
    double s = b[j];
    for (int i = j + 1; i < n; ++i) s -= L[i + (int64_t)ld * j] * x[i];
    x[j] = s / L[j + (int64_t)ld * j];
  }
}
static void kinv(const double* L, int ld, int n, const double* b, double* x, double* tmp) { /* L'\(L\b) */
  lsolve(L, ld, n, b, tmp);
  ltsolve(L, ld, n, tmp, x);
}

/* small dense Cholesky (LAPACK potrf semantics: fails on a non-positive pivot) */
static int chol_small(const double* A, int n, double* Lo) {
  memset(Lo, 0, sizeof(double) * n * n);
  for (int j = 0; j < n; ++j) {
    double s = A[j + n * j];
    for (int k = 0; k < j; ++k) s -= Lo[j + n * k] * Lo[j + n * k];
    if (!(s > 0)) return -1;
    const double ljj = sqrt(s);
    Lo[j + n * j] = ljj;
    for (int i = j + 1; i < n; ++i) {
      double t = A[i + n * j];
      for (int k = 0; k < j; ++k) t -= Lo[i + n * k] * Lo[j + n * k];
      Lo[i + n * j] = t / ljj;
    }
  }
  return 0;
}

/* LU with partial pivoting (Julia det / \ on a Matrix).  A overwritten. */
static int lu_small(double* A, int n, int* piv) {
  int info = 0;
  for (int k = 0; k < n; ++k) {
    int p = k;
    double mx = fabs(A[k + n * k]);
    for (int i = k + 1; i < n; ++i)
      if (fabs(A[i + n * k]) > mx) { mx = fabs(A[i + n * k]); p = i; }
    piv[k] = p;
    if (p != k)
      for (int j = 0; j < n; ++j) { double t = A[k + n * j]; A[k + n * j] = A[p + n * j]; A[p + n * j] = t; }
    if (A[k + n * k] == 0.0) { info = k + 1; continue; }
    for (int i = k + 1; i < n; ++i) A[i + n * k] /= A[k + n * k];
    for (int j = k + 1; j < n; ++j)
      for (int i = k + 1; i < n; ++i) A[i + n * j] -= A[i + n * k] * A[k + n * j];
  }
  return info;
}
static double lu_det(const double* LU, const int* piv, int n) {
  double dt = 1.0;
  for (int k = 0; k < n; ++k) { dt *= LU[k + n * k]; if (piv[k] != k) dt = -dt; }
  return dt;
}
static void lu_solve(const double* LU, const int* piv, int n, double* b) {
  for (int k = 0; k < n; ++k) if (piv[k] != k) { double t = b[k]; b[k] = b[piv[k]]; b[piv[k]] = t; }
  for (int i = 0; i < n; ++i) { double s = b[i]; for (int k = 0; k < i; ++k) s -= LU[i + n * k] * b[k]; b[i] = s; }
  for (int i = n - 1; i >= 0; --i) { double s = b[i]; for (int k = i + 1; k < n; ++k) s -= LU[i + n * k] * b[k]; b[i] = s / LU[i + n * i]; }
}
/* cond₁(A) = ‖A‖₁‖A⁻¹‖₁ from A (n×n) and its LU factors, by n unit solves (diagnostic only:
 * the parity tests scale the adjoint-gradient tolerance by it) */
static double cond1(const double* A, const double* LU, const int* piv, int n) {
  double na = 0, ni = 0, e[16];
  for (int j = 0; j < n; ++j) {
    double s = 0;
    for (int i = 0; i < n; ++i) s += fabs(A[i + n * j]);
    na = fmax(na, s);
    for (int i = 0; i < n; ++i) e[i] = (i == j) ? 1.0 : 0.0;
    lu_solve(LU, piv, n, e);
    s = 0;
    for (int i = 0; i < n; ++i) s += fabs(e[i]);
    ni = fmax(ni, s);
  }
  return na * ni;
}

/* ------------------------------------------------------------------------------------
 * FantasySurrogate (radial_basis_surrogates.jl:320-481)
 * ---------------------------------------------------------------------------------- */
typedef struct {
  int d, N, h, cap;
  kern_t k;
  double sn2;
  double* X;   /* d × cap          */
  double* L;   /* cap × cap, ld cap */
  double* y;   /* cap              */
  double* cs;  /* (h+2) × cap : cs[s+1] = coefficient vector of fantasy_index s */
  int nfant;   /* fantasies_observed */
  int rule;    /* RBO_RULE_*: the trajectory's base decision rule */
  int cost;    /* RBO_COST_*: cost weighting of the rule (inner solve), see cost_eval */
  double c0, cw[16], clb[16], cub[16];
} fsur_t;

static int fsur_alloc(fsur_t* fs, const rbo_surrogate* s, int h, int rule, const rbo_params* p) {
  fs->d = s->d; fs->N = s->N; fs->h = h; fs->cap = s->N + h + 1; fs->rule = rule;
  fs->cost = (p && p->cost_w) ? p->cost : RBO_COST_NONE;
  if (fs->cost) {
    fs->c0 = p->cost_c0;
    for (int a = 0; a < s->d; ++a) { fs->cw[a] = p->cost_w[a]; fs->clb[a] = p->lbs[a]; fs->cub[a] = p->ubs[a]; }
  }
  fs->k.kind = s->kernel; fs->k.ell = s->ell; fs->k.per = s->period; fs->sn2 = s->sigma_n2;
  fs->X = (double*)calloc((size_t)fs->d * fs->cap, sizeof(double));
  fs->L = (double*)calloc((size_t)fs->cap * fs->cap, sizeof(double));
  fs->y = (double*)calloc((size_t)fs->cap, sizeof(double));
  fs->cs = (double*)calloc((size_t)(h + 2) * fs->cap, sizeof(double));
  if (!fs->X || !fs->L || !fs->y || !fs->cs) return -1;
  memcpy(fs->X, s->X, sizeof(double) * s->d * s->N);
  for (int j = 0; j < s->N; ++j)
    for (int i = j; i < s->N; ++i) fs->L[i + (int64_t)fs->cap * j] = s->L[i + (int64_t)s->N * j];
  memcpy(fs->y, s->y, sizeof(double) * s->N);
  memcpy(fs->cs, s->c, sizeof(double) * s->N); /* cs = [c[1:N]]  (:373) */
  fs->nfant = 0;
  return 0;
}
static void fsur_free(fsur_t* fs) { free(fs->X); free(fs->L); free(fs->y); free(fs->cs); }
static void fsur_reset(fsur_t* fs) { fs->nfant = 0; } /* reset! :476-480 */

/* condition!(fs, x, y) :431-441 = insert! + increment! + update_covariance! +
 * update_cholesky! + update_coefficients! (full re-solve, Q13) */
static int fsur_condition(fsur_t* fs, const double* x, double yv, double* tmp) {
  const int d = fs->d, cap = fs->cap;
  const int idx = fs->N + fs->nfant; /* insert index (0-based) */
  memcpy(fs->X + (int64_t)d * idx, x, sizeof(double) * d);
  fs->y[idx] = yv;
  fs->nfant += 1;
  const int n = idx + 1;
  double* B = tmp;          /* K[n, 1:n-1] */
  double* L21 = tmp + cap;  /* B / L'       */
  double r[64];
  for (int j = 0; j < n - 1; ++j) {
    for (int a = 0; a < d; ++a) r[a] = x[a] - fs->X[(int64_t)d * j + a];
    B[j] = k_psi(&fs->k, vnorm(r, d));
  }
  const double C = k_psi(&fs->k, 0.0) + fs->sn2;
  lsolve(fs->L, cap, n - 1, B, L21);
  double ss = 0;
  for (int j = 0; j < n - 1; ++j) ss += L21[j] * L21[j];
  const double S = C - ss;
  for (int j = 0; j < n - 1; ++j) fs->L[(n - 1) + (int64_t)cap * j] = L21[j];
  if (!(S > 0)) { fs->L[(n - 1) + (int64_t)cap * (n - 1)] = NAN; return RBO_ST_COND_NOT_PD; }
  fs->L[(n - 1) + (int64_t)cap * (n - 1)] = sqrt(S);
  kinv(fs->L, cap, n, fs->y, fs->cs + (int64_t)fs->nfant * cap, tmp + 2 * cap);
  return 0;
}

/* Lazy posterior quantities of eval(fs, x, θ; fantasy_index) :482-581. */
typedef struct {
  int n, d, fi;
  double x[16];
  double mu, sigma, fmin, alpha;
  double gmu[16], gsig[16], galpha[16], mixed[16];
  double Halpha[256];
  double alpha_raw, cost, gcost[16], gcmax; /* NonUniformCost: rule value g, c(x), ∇c(x), max|∇c| */
  ei_t e;
  double *kx, *gkx, *w, *Dw; /* n, d×n, n, n×d  (scratch owned by caller) */
  int status;
} sx_t;

typedef struct {
  double *kx, *gkx, *w, *Dw, *tmp, *tmp2, *tmp3;
} scratch_t;

static void scratch_alloc(scratch_t* sc, int cap, int d) {
  sc->kx = (double*)malloc(sizeof(double) * cap);
  sc->gkx = (double*)malloc(sizeof(double) * cap * d);
  sc->w = (double*)malloc(sizeof(double) * cap);
  sc->Dw = (double*)malloc(sizeof(double) * cap * d);
  sc->tmp = (double*)malloc(sizeof(double) * cap * (d + 4) * 2);
  sc->tmp2 = (double*)malloc(sizeof(double) * cap * cap);
  sc->tmp3 = (double*)malloc(sizeof(double) * cap * (d + 4));
}
static void scratch_free(scratch_t* sc) {
  free(sc->kx); free(sc->gkx); free(sc->w); free(sc->Dw); free(sc->tmp); free(sc->tmp2); free(sc->tmp3);
}

/* NonUniformCost families (rbo_oracle.h RBO_COST_*): c(x), ∇c(x) and Hc = diag(hd) + β v vᵀ. */
static void cost_eval(const fsur_t* fs, const double* x, double* c, double* gc, double* hd, double* beta, double* v) {
  const int d = fs->d;
  if (fs->cost == RBO_COST_QUADRATIC) {
    double s = fs->c0;
    for (int a = 0; a < d; ++a) {
      const double del = fs->cub[a] - fs->clb[a], u = (x[a] - fs->clb[a]) / del;
      s += fs->cw[a] * u * u;
      gc[a] = 2.0 * fs->cw[a] * u / del;
      hd[a] = 2.0 * fs->cw[a] / (del * del);
      v[a] = 0.0;
    }
    *c = s;
    *beta = 0.0;
  } else {
    double t = 0;
    for (int a = 0; a < d; ++a) t += fs->cw[a] * (x[a] - fs->clb[a]) / (fs->cub[a] - fs->clb[a]);
    const double cv = fs->c0 * exp(t);
    for (int a = 0; a < d; ++a) {
      v[a] = fs->cw[a] / (fs->cub[a] - fs->clb[a]);
      gc[a] = cv * v[a];
      hd[a] = 0.0;
    }
    *c = cv;
    *beta = cv;
  }
}

/* value_only: α only (the line-search path); full: gradient, Hessian, mixed partials.
 * With a cost model the acquisition is f = α/c (cost-weighted rule, build-defined):
 *   ∇f = ∇α/c − α∇c/c²,  Hf = (Hα − ∇f∇cᵀ − ∇c∇fᵀ)/c − (α/c²)Hc,  ∂∇f/∂θ = ∂∇α/∂θ/c − g_θ∇c/c². */
static void fsur_eval(const fsur_t* fs, const double* x, double theta, double sigma_tol, int fi,
                      int value_only, sx_t* sx, scratch_t* sc) {
  const int d = fs->d, cap = fs->cap, n = fs->N + fi + 1;
  const double* X = fs->X;
  const double* L = fs->L;
  const double* c = fs->cs + (int64_t)(fi + 1) * cap;
  sx->n = n; sx->d = d; sx->fi = fi; sx->status = 0;
  memcpy(sx->x, x, sizeof(double) * d);
  sx->kx = sc->kx; sx->gkx = sc->gkx; sx->w = sc->w; sx->Dw = sc->Dw;
  double r[16];
  /* sx.kx, sx.∇kx (eval_KxX :180-191, eval_∇KxX :193-208) */
  for (int j = 0; j < n; ++j) {
    for (int a = 0; a < d; ++a) r[a] = x[a] - X[(int64_t)d * j + a];
    const double rho = vnorm(r, d);
    sc->kx[j] = k_psi(&fs->k, rho);
    if (!value_only) {
      if (rho > 0) { const double dp = k_dpsi(&fs->k, rho); for (int a = 0; a < d; ++a) sc->gkx[a + d * j] = dp * r[a] / rho; }
      else for (int a = 0; a < d; ++a) sc->gkx[a + d * j] = 0.0;
    }
  }
  double mu = 0;
  for (int j = 0; j < n; ++j) mu += sc->kx[j] * c[j];
  sx->mu = mu;
  kinv(L, cap, n, sc->kx, sc->w, sc->tmp); /* sx.w */
  double kw = 0;
  for (int j = 0; j < n; ++j) kw += sc->kx[j] * sc->w[j];
  const double var = k_psi(&fs->k, 0.0) - kw;
  if (var < 0) sx->status |= RBO_ST_SIGMA_NEG;
  sx->sigma = sqrt(var);
  double fmin = fs->y[0];
  for (int j = 1; j < n; ++j) if (fs->y[j] < fmin) fmin = fs->y[j];
  sx->fmin = fmin;
  sx->e = rule_partials(fs->rule, sx->mu, sx->sigma, theta, fmin, sigma_tol);
  sx->alpha = sx->e.g;
  sx->alpha_raw = sx->e.g;
  sx->cost = 1.0;
  sx->gcmax = 0.0;
  double chd[16], cbeta = 0.0, cv[16];
  if (fs->cost) {
    cost_eval(fs, x, &sx->cost, sx->gcost, chd, &cbeta, cv);
    for (int a = 0; a < d; ++a) sx->gcmax = fmax(sx->gcmax, fabs(sx->gcost[a]));
    sx->alpha = sx->e.g / sx->cost;
  }
  if (value_only) return;
  /* ∇μ, Dw, ∇σ */
  for (int a = 0; a < d; ++a) {
    double s = 0;
    for (int j = 0; j < n; ++j) s += sc->gkx[a + d * j] * c[j];
    sx->gmu[a] = s;
  }
  for (int a = 0; a < d; ++a) {
    for (int j = 0; j < n; ++j) sc->tmp3[j] = sc->gkx[a + d * j];
    kinv(L, cap, n, sc->tmp3, sc->Dw + (int64_t)a * n, sc->tmp);
  }
  for (int a = 0; a < d; ++a) {
    double s = 0;
    for (int j = 0; j < n; ++j) s += sc->gkx[a + d * j] * sc->w[j];
    sx->gsig[a] = -s / sx->sigma;
  }
  /* Hμ, Hσ (:516-523, :540-548) */
  double Hmu[256], Hsig[256], Hk[256];
  memset(Hmu, 0, sizeof(double) * d * d);
  memset(Hsig, 0, sizeof(double) * d * d);
  for (int j = 0; j < n; ++j) {
    for (int a = 0; a < d; ++a) r[a] = x[a] - X[(int64_t)d * j + a];
    eval_Hk(&fs->k, r, d, Hk);
    for (int q = 0; q < d * d; ++q) { Hmu[q] += c[j] * Hk[q]; Hsig[q] -= sc->w[j] * Hk[q]; }
  }
  for (int b = 0; b < d; ++b)
    for (int a = 0; a < d; ++a) {
      double gDw = 0; /* (∇kx * Dw)[a,b] */
      for (int j = 0; j < n; ++j) gDw += sc->gkx[a + d * j] * sc->Dw[j + (int64_t)n * b];
      Hsig[a + d * b] = (-sx->gsig[a] * sx->gsig[b] - gDw + Hsig[a + d * b]) / sx->sigma;
    }
  const ei_t* e = &sx->e;
  for (int a = 0; a < d; ++a) {
    sx->galpha[a] = e->gmu * sx->gmu[a] + e->gsig * sx->gsig[a];
    sx->mixed[a] = sx->gmu[a] * e->gmuth + sx->gsig[a] * e->gsigth; /* d2α_dxdθ :575-577 */
  }
  /* Hαx :568 (no μσ cross term, Q11) */
  for (int b = 0; b < d; ++b)
    for (int a = 0; a < d; ++a)
      sx->Halpha[a + d * b] = e->gmumu * sx->gmu[a] * sx->gmu[b] + e->gmu * Hmu[a + d * b] +
                              e->gsigsig * sx->gsig[a] * sx->gsig[b] + e->gsig * Hsig[a + d * b];
  if (fs->cost) {
    const double c = sx->cost, ac2 = sx->alpha_raw / (c * c);
    for (int a = 0; a < d; ++a) {
      sx->galpha[a] = sx->galpha[a] / c - ac2 * sx->gcost[a];
      sx->mixed[a] = sx->mixed[a] / c - e->gth * sx->gcost[a] / (c * c);
    }
    for (int b = 0; b < d; ++b)
      for (int a = 0; a < d; ++a) {
        const double hc = ((a == b) ? chd[a] : 0.0) + cbeta * cv[a] * cv[b];
        sx->Halpha[a + d * b] =
            (sx->Halpha[a + d * b] - sx->galpha[a] * sx->gcost[b] - sx->gcost[a] * sx->galpha[b]) / c - ac2 * hc;
      }
  }
}

/* gp_draw(fs, x, θ; stdnormal, with_gradient=true, fantasy_index) :588-611; sx.dσ :530-539 */
/* kappa (diagnostic, may be NULL): raised to ‖Dk(0)‖₁‖σx⁻¹‖₁, the cancellation condition of the
 * draw covariance σx = Dk(0) − G (its rounding error is relative to Dk(0), not to σx) */
static int fsur_draw(const fsur_t* fs, const double* x, double theta, double sigma_tol, int fi, const double* z,
                     double* y_out, double* grad_out, sx_t* sx, scratch_t* sc, double* kappa) {
  const int d = fs->d, cap = fs->cap, n = fs->N + fi + 1, D1 = d + 1;
  fsur_eval(fs, x, theta, sigma_tol, fi, 0, sx, sc);
  /* kxX = [kx'; ∇kx]  ((d+1)×n);  σx = Dk(0) - kxX*(L'\(L\kxX')) */
  double Sig[289], Ls[289];
  double* Z = sc->tmp2; /* n × (d+1) */
  for (int col = 0; col < D1; ++col) {
    for (int j = 0; j < n; ++j) sc->tmp3[j] = (col == 0) ? sc->kx[j] : sc->gkx[(col - 1) + d * j];
    kinv(fs->L, cap, n, sc->tmp3, Z + (int64_t)n * col, sc->tmp);
  }
  const double psi0 = k_psi(&fs->k, 0.0), d2psi0 = k_d2psi(&fs->k, 0.0);
  for (int b = 0; b < D1; ++b)
    for (int a = 0; a < D1; ++a) {
      double s = 0;
      for (int j = 0; j < n; ++j) {
        const double ka = (a == 0) ? sc->kx[j] : sc->gkx[(a - 1) + d * j];
        s += ka * Z[j + (int64_t)n * b];
      }
      const double kxx = (a == b) ? (a == 0 ? psi0 : -d2psi0) : 0.0; /* eval_Dk(0) */
      Sig[a + D1 * b] = kxx - s;
    }
  /* Symmetric(σx) reads the upper triangle */
  for (int b = 0; b < D1; ++b) for (int a = b + 1; a < D1; ++a) Sig[a + D1 * b] = Sig[b + D1 * a];
  if (chol_small(Sig, D1, Ls)) return RBO_ST_DRAW_NOT_PD;
  if (kappa) {
    double ni = 0, e[17];
    for (int j = 0; j < D1; ++j) {   /* column j of σx⁻¹ = Ls'\(Ls\e_j) */
      for (int i = 0; i < D1; ++i) e[i] = (i == j) ? 1.0 : 0.0;
      for (int i = 0; i < D1; ++i) { double t = e[i]; for (int k = 0; k < i; ++k) t -= Ls[i + D1 * k] * e[k]; e[i] = t / Ls[i + D1 * i]; }
      for (int i = D1 - 1; i >= 0; --i) { double t = e[i]; for (int k = i + 1; k < D1; ++k) t -= Ls[k + D1 * i] * e[k]; e[i] = t / Ls[i + D1 * i]; }
      double sc1 = 0;
      for (int i = 0; i < D1; ++i) sc1 += fabs(e[i]);
      ni = fmax(ni, sc1);
    }
    *kappa = fmax(*kappa, fmax(fabs(psi0), fabs(d2psi0)) * ni);
  }
  double dmu[17];
  dmu[0] = sx->mu;
  for (int a = 0; a < d; ++a) dmu[a + 1] = sx->gmu[a];
  for (int a = 0; a < D1; ++a) {
    double s = 0;
    for (int k = 0; k <= a; ++k) s += Ls[a + D1 * k] * z[k];
    dmu[a] += s;
  }
  *y_out = dmu[0];
  for (int a = 0; a < d; ++a) grad_out[a] = dmu[a + 1];
  return sx->status;
}

/* ------------------------------------------------------------------------------------
 * Inner policy solve.  Reference: multistart_base_solve!(fs, …) rbf_optim.jl:68-101 with
 * Optim IPNewton per start (:1-33), x_tol = f_tol = 1e-3.  IPNewton is absent here; the
 * build defines the deterministic projected Newton of DESIGN.md §4 (same on the GPU).
 * ---------------------------------------------------------------------------------- */
/* n_grad / n_value / n_hess: evaluations the lazy iteration needs (below) -- the same counts
 * the GPU kernel reports, so tests can assert identical Newton work. */
typedef struct {
  const fsur_t* fs;
  const rbo_params* p;
  int fi;
  scratch_t* sc;
  int64_t n_grad, n_value, n_hess;
  int st;
  double cabs; /* Σ|c| of the surface (grad_certified) */
} solve_ctx;

/* max_ρ |ψ'(ρ)| (+1%) and √(ψ(0)·(−ψ''(0))) (+1%; -1 when ψ''(0) > 0, Matérn-1/2) -- the
 * constants of the gradient certificate, in closed form. */
static void k_gcert(const kern_t* k, double* gmu, double* gsig) {
  const double d2 = k_d2psi(k, 0.0);
  switch (k->kind) {
    case RBO_K_MATERN52: {
      const double c = sqrt(5.0) / k->ell, s = 0.5 * (1.0 + sqrt(5.0));
      *gmu = 1.01 * c * (s / 3.0) * (1.0 + s) * exp(-s);
      break;
    }
    case RBO_K_MATERN32: *gmu = 1.01 * (sqrt(3.0) / k->ell) * exp(-1.0); break;
    case RBO_K_MATERN12: *gmu = 1.01 / k->ell; break;
    case RBO_K_PERIODIC: *gmu = 1.01 * PER_A(k); break;   /* |ψ'| = ψ A |sin t| ≤ A */
    default: *gmu = 1.01 * (1.0 / k->ell) * exp(-0.5); break;
  }
  *gsig = (d2 < 0) ? 1.01 * sqrt(k_psi(k, 0.0) * -d2) : -1.0;
}

/* Gradient certificate from a value-only evaluation: ‖∇α‖∞ ≤ g_tol guaranteed:
 * |∂μ| ≤ Σ|c| max|ψ'|, |∂σ| ≤ √(ψ(0)(−ψ''(0)))/σ, factor 4 for rounding; gμ = gσ = 0 makes
 * ∇α zero or NaN, which stops the iteration as well.  When that cheap bound fails, the tight
 * one at the point itself: |∂_a μ| ≤ Σ_j |c_j| |ψ'(ρ_j)| over the surface's data rows, and
 * |∂_a σ| = |∂_a kxᵀK⁻¹kx|/σ ≤ √(−ψ''(0)) √(kxᵀK⁻¹kx)/σ with kxᵀK⁻¹kx = ψ(0) − σ². */
/* With a cost model, f = α/c: |∂_a f| ≤ B/c + |α|·max|∇c|/c² for any bound B on |∂_a α|, and
 * gμ = gσ = 0 certifies only where α = 0 as well (POI can sit at Φ = 1 with ∇f = −∇c/c²). */
static int grad_certified(const solve_ctx* cx, const sx_t* sx, const double* x) {
  const double gm = sx->e.gmu, gs = sx->e.gsig;
  const int cost = cx->fs->cost;
  if (gm == 0.0 && gs == 0.0 && (!cost || sx->alpha_raw == 0.0)) return 1;
  const double isc = cost ? 1.0 / sx->cost : 1.0;
  const double add = cost ? fabs(sx->alpha_raw) * sx->gcmax / (sx->cost * sx->cost) : 0.0;
  double cmu, csig;
  k_gcert(&cx->fs->k, &cmu, &csig);
  if (!(csig > 0.0)) return 0;
  const double bound = fabs(gm) * cmu * cx->cabs + fabs(gs) * csig / sx->sigma;
  if (bound * isc + add <= 0.25 * cx->p->g_tol) return 1;
  const fsur_t* fs = cx->fs;
  const int d = fs->d, n = fs->N + cx->fi + 1;
  const double* c = fs->cs + (int64_t)(cx->fi + 1) * fs->cap;
  double bmu = 0, r[16];
  for (int j = 0; j < n; ++j) {
    for (int a = 0; a < d; ++a) r[a] = x[a] - fs->X[(int64_t)d * j + a];
    bmu += fabs(c[j]) * fabs(k_dpsi(&fs->k, vnorm(r, d)));
  }
  const double psi0 = k_psi(&fs->k, 0.0), d2 = k_d2psi(&fs->k, 0.0);
  const double q = fmax(psi0 - sx->sigma * sx->sigma, 0.0);
  const double tight = fabs(gm) * bmu + fabs(gs) * 1.01 * sqrt(-d2) * sqrt(q) / sx->sigma;
  return tight * isc + add <= 0.25 * cx->p->g_tol;
}

static double clampd(double v, double lo, double hi) { return v < lo ? lo : (v > hi ? hi : v); }

/* Projected Newton with projected-Armijo backtracking.  Evaluation is lazy:
 * every point gets a value-only evaluation; the gradient only where the certificate cannot
 * rule out a step, the Hessian only where a step is taken.  fsur_eval in full mode yields
 * ∇α and Hα together (the counters record what the iteration needs: n_grad, n_hess).
 * Values are identical in either mode, so the iterates do not depend on the laziness. */
static void newton_solve(solve_ctx* cx, const double* xs, double* xout, double* fout) {
  const fsur_t* fs = cx->fs;
  const rbo_params* p = cx->p;
  const int d = fs->d;
  double x[16] = {0}, g[16], H[256], xt[16], pdir[16], Hs[256], Lc[256];
  sx_t sx;
  int free_[16];
  for (int a = 0; a < d; ++a) x[a] = clampd(xs[a], p->lbs[a], p->ubs[a]);
  fsur_eval(fs, x, p->theta, p->sigma_tol, cx->fi, 1, &sx, cx->sc);
  cx->n_value++;
  cx->st |= sx.status;
  double f = -sx.alpha;
  double box = 0;
  for (int a = 0; a < d; ++a) box = fmax(box, p->ubs[a] - p->lbs[a]);
  int it = 0;
  for (;;) {
    /* decision point at x; sx holds its value-only evaluation */
    if (it >= p->max_iters) break;
    if (isnan(f)) break;
    if (grad_certified(cx, &sx, x)) break;
    fsur_eval(fs, x, p->theta, p->sigma_tol, cx->fi, 0, &sx, cx->sc);
    cx->n_grad++;
    for (int a = 0; a < d; ++a) g[a] = -sx.galpha[a];
    for (int q = 0; q < d * d; ++q) H[q] = -sx.Halpha[q];
    double pg = 0;
    for (int a = 0; a < d; ++a) {
      const int act = (x[a] <= p->lbs[a] && g[a] > 0) || (x[a] >= p->ubs[a] && g[a] < 0);
      free_[a] = !act;
      if (!act) pg = fmax(pg, fabs(g[a]));
    }
    if (!(pg > p->g_tol)) break;
    cx->n_hess++;
    /* reduced Hessian on the free set */
    int idx[16], m = 0;
    for (int a = 0; a < d; ++a) if (free_[a]) idx[m++] = a;
    for (int jb = 0; jb < m; ++jb)
      for (int ia = 0; ia < m; ++ia) Hs[ia + m * jb] = H[idx[ia] + d * idx[jb]];
    int ok = (chol_small(Hs, m, Lc) == 0);
    if (!ok) {
      double tau = 0, hmax = 0;
      for (int ia = 0; ia < m; ++ia) {
        double off = 0;
        for (int jb = 0; jb < m; ++jb) if (jb != ia) off += fabs(Hs[ia + m * jb]);
        tau = fmax(tau, off - Hs[ia + m * ia]);
        hmax = fmax(hmax, fabs(Hs[ia + m * ia]));
      }
      tau += 1e-8 * (1.0 + hmax);
      for (int ia = 0; ia < m; ++ia) Hs[ia + m * ia] += tau;
      ok = (chol_small(Hs, m, Lc) == 0);
    }
    for (int a = 0; a < d; ++a) pdir[a] = 0;
    if (ok) {
      double rhs[16], t1[16], t2[16];
      for (int ia = 0; ia < m; ++ia) rhs[ia] = g[idx[ia]];
      lsolve(Lc, m, m, rhs, t1);
      ltsolve(Lc, m, m, t1, t2);
      for (int ia = 0; ia < m; ++ia) pdir[idx[ia]] = -t2[ia];
    } else {
      for (int ia = 0; ia < m; ++ia) pdir[idx[ia]] = -g[idx[ia]];
    }
    double pn = 0;
    for (int a = 0; a < d; ++a) pn = fmax(pn, fabs(pdir[a]));
    if (pn > box) for (int a = 0; a < d; ++a) pdir[a] *= box / pn;
    /* projected backtracking Armijo line search, value-only trials */
    double t = 1.0, ft = NAN;
    int accepted = 0;
    for (int ls = 0; ls < p->max_ls; ++ls) {
      double dec = 0;
      for (int a = 0; a < d; ++a) {
        xt[a] = clampd(x[a] + t * pdir[a], p->lbs[a], p->ubs[a]);
        dec += g[a] * (xt[a] - x[a]);
      }
      fsur_eval(fs, xt, p->theta, p->sigma_tol, cx->fi, 1, &sx, cx->sc);
      cx->n_value++;
      cx->st |= sx.status;
      ft = -sx.alpha;
      if (!isnan(ft) && ft <= f + 1e-4 * dec) { accepted = 1; break; }
      t *= 0.5;
    }
    if (!accepted) break;
    double dx = 0;
    for (int a = 0; a < d; ++a) dx = fmax(dx, fabs(xt[a] - x[a]));
    const double df = fabs(ft - f);
    for (int a = 0; a < d; ++a) x[a] = xt[a];
    f = ft;
    ++it;
    if (dx <= p->x_tol || df <= p->f_tol * fabs(f)) break;
  }
  for (int a = 0; a < d; ++a) xout[a] = x[a];
  *fout = f;
}

static int multistart(solve_ctx* cx, const double* xstarts, double* xfinal) {
  { /* Σ|c| of the solve surface (base + fantasy coefficients) for the gradient certificate */
    const fsur_t* fs = cx->fs;
    const double* c = fs->cs + (int64_t)(cx->fi + 1) * fs->cap;
    double s = 0;
    for (int j = 0; j < fs->N + cx->fi + 1; ++j) s += fabs(c[j]);
    cx->cabs = s;
  }
  const int d = cx->fs->d;
  int best = -1, best_nan = -1;
  double bestf = INFINITY, xc[16], fc, xb[16];
  for (int i = 0; i < cx->p->nstarts; ++i) {
    newton_solve(cx, xstarts + (int64_t)d * i, xc, &fc);
    int xnan = 0;
    for (int a = 0; a < d; ++a) xnan |= isnan(xc[a]);
    if (xnan) continue; /* filter(!any(isnan.(minimizer))) :96 */
    if (isnan(fc)) { if (best_nan < 0) { best_nan = i; memcpy(xb, xc, sizeof(double) * d); } continue; }
    if (best_nan < 0 && (best < 0 || fc < bestf)) { best = i; bestf = fc; memcpy(xb, xc, sizeof(double) * d); }
  }
  if (cx->st) return cx->st;
  if (best < 0 && best_nan < 0) return RBO_ST_ALL_NAN;
  memcpy(xfinal, xb, sizeof(double) * d); /* findmin: NaN sorts first, first minimum wins */
  return 0;
}

/* ------------------------------------------------------------------------------------
 * Perturbation surrogates :633-764 (dense δK exactly as written).
 * δ∇α of the gradient of the acquisition at sx when data point `sample_index` of the
 * fantasised trajectory moves by δ.  data=1: DataPerturbationSurrogate (no g_σ·δ∇σ).
 * ---------------------------------------------------------------------------------- */
static void perturb_grad(const fsur_t* fs, const sx_t* sx, int S, int q, const double* dlt, int data,
                         double theta, double sigma_tol, scratch_t* sc, double* out) {
  const int d = fs->d, cap = fs->cap, n = fs->N + S + 1, col = fs->N + q;
  const double* X = fs->X;
  const double* c = fs->cs + (int64_t)(S + 1) * cap;
  double* dK = sc->tmp2;               /* n×n */
  double* dKc = sc->tmp3;              /* n   */
  double* dc = sc->tmp3 + cap;         /* n   */
  double* dKw = sc->tmp3 + 2 * cap;    /* n   */
  double* tmp = sc->tmp;
  double r[16], gk[16], Hk[256];
  /* eval_δKXX :210-228 with δX zero except column `col` */
  for (int j = 0; j < n; ++j) {
    dK[j + (int64_t)n * j] = 0;
    for (int i = j + 1; i < n; ++i) {
      for (int a = 0; a < d; ++a) r[a] = X[(int64_t)d * i + a] - X[(int64_t)d * j + a];
      eval_grad_k(&fs->k, r, d, gk);
      double s = 0;
      for (int a = 0; a < d; ++a) {
        const double dxi = (i == col) ? dlt[a] : 0.0, dxj = (j == col) ? dlt[a] : 0.0;
        s += gk[a] * (dxi - dxj);
      }
      dK[i + (int64_t)n * j] = s;
      dK[j + (int64_t)n * i] = s;
    }
  }
  for (int i = 0; i < n; ++i) {
    double s = 0, sw = 0;
    for (int j = 0; j < n; ++j) { s += dK[i + (int64_t)n * j] * c[j]; sw += dK[i + (int64_t)n * j] * sx->w[j]; }
    dKc[i] = s;
    dKw[i] = sw;
  }
  kinv(fs->L, cap, n, dKc, dc, tmp);
  for (int i = 0; i < n; ++i) dc[i] = -dc[i];
  /* δkx :230-245, δ∇kx :247-262 (only column `col` of δX is non-zero) */
  double dkx_col, dgkx_col[16];
  for (int a = 0; a < d; ++a) r[a] = sx->x[a] - X[(int64_t)d * col + a];
  eval_grad_k(&fs->k, r, d, gk);
  dkx_col = 0;
  for (int a = 0; a < d; ++a) dkx_col += gk[a] * (-dlt[a]);
  eval_Hk(&fs->k, r, d, Hk);
  for (int a = 0; a < d; ++a) {
    double s = 0;
    for (int b = 0; b < d; ++b) s += Hk[a + d * b] * (-dlt[b]);
    dgkx_col[a] = s;
  }
  /* δμ, δ∇μ, δσ, δ∇σ (:680-684) */
  double dmu = dkx_col * c[col];
  for (int j = 0; j < n; ++j) dmu += sx->kx[j] * dc[j];
  double dgmu[16];
  for (int a = 0; a < d; ++a) {
    double s = dgkx_col[a] * c[col];
    for (int j = 0; j < n; ++j) s += sx->gkx[a + d * j] * dc[j];
    dgmu[a] = s;
  }
  double wdKw = 0;
  for (int j = 0; j < n; ++j) wdKw += sx->w[j] * dKw[j];
  const double dsig = (-2 * dkx_col * sx->w[col] + wdKw) / (2 * sx->sigma);
  double dgsig[16];
  for (int a = 0; a < d; ++a) {
    double t1 = 0; /* (∇w * (δK*w))[a],  ∇w = Dw' */
    for (int j = 0; j < n; ++j) t1 += sx->Dw[j + (int64_t)n * a] * dKw[j];
    const double t2 = dgkx_col[a] * sx->w[col];            /* δ∇kx * w  */
    const double t3 = sx->Dw[col + (int64_t)n * a] * dkx_col; /* ∇w * δkx  */
    dgsig[a] = (t1 - t2 - t3 - dsig * sx->gsig[a]) / sx->sigma;
  }
  /* δsx.dg_dμ / dg_dσ: first partials evaluated at (δμ, δσ)  (Q7, Q8) */
  const ei_t de = rule_partials(fs->rule, dmu, dsig, theta, sx->fmin, sigma_tol);
  for (int a = 0; a < d; ++a) {
    if (data)
      out[a] = sx->e.gmu * dgmu[a] + de.gmu * sx->gmu[a] + de.gsig * sx->gsig[a];
    else
      out[a] = sx->e.gmu * dgmu[a] + sx->e.gsig * dgsig[a] + de.gmu * sx->gmu[a] + de.gsig * sx->gsig[a];
  }
  if (fs->cost) {   /* δ∇(α/c) = δ∇α/c − δα ∇c/c², δα = gμ δμ + gσ δσ (first order; build-defined) */
    const double c = sx->cost, da = sx->e.gmu * dmu + sx->e.gsig * dsig;
    for (int a = 0; a < d; ++a) out[a] = out[a] / c - da * sx->gcost[a] / (c * c);
  }
}

/* ------------------------------------------------------------------------------------
 * One trajectory: rollout! (rollout.jl:39-74), resolve (:108-111), gradient (:233-277)
 * ---------------------------------------------------------------------------------- */
typedef struct {
  const rbo_surrogate* s;
  const rbo_params* p;
  const double* rnstream;
  const double* xstarts;
  const double* dual_y_dx;
  const double* replay_x;
  const double* ghq_nodes; /* M×(h+1) Gauss–Hermite nodes per sample, or NULL (Monte Carlo) */
  const double* ghq_w;     /* M×(h+1) their weights                                        */
} traj_in;

static int run_trajectory(const traj_in* in, int r, int m, const double* x0, fsur_t* fs, scratch_t* sc,
                          double* value, double* gx, double* gth, double* pol, double* obs_out, int64_t* evals,
                          double* kappa, double* vbound, double* ylip, double kappa_L) {
  const rbo_params* p = in->p;
  const int d = fs->d, h = p->h, M = p->M, D1 = d + 1;
  double obs[64] = {0}, grads[64 * 16], z[17], xnext[16], dy[64] = {0};
  double wmax = 0.0;
  const double nu = (double)(fs->N + h) * 0x1p-53;
  if (ylip) *ylip = 0.0;
  sx_t sx;
  int st = 0;
  fsur_reset(fs);
  solve_ctx cx = {fs, p, -1, sc, 0, 0, 0, 0, 0.0};
  /* StochasticObservable (observables.jl:106-121): step k uses rns[m, :, k+1], fantasy_index k-1 */
  for (int k = 0; k <= h; ++k) {
    const double* xk;
    if (k == 0) {
      xk = x0;
    } else {
      if (in->replay_x) {
        const double* rx = in->replay_x + (int64_t)d * ((k - 1) + (int64_t)h * (m + (int64_t)M * r));
        memcpy(xnext, rx, sizeof(double) * d);
      } else {
        cx.fi = k - 1;
        st |= multistart(&cx, in->xstarts, xnext);
        if (st) break;
      }
      xk = xnext;
    }
    if (pol) memcpy(pol + (int64_t)d * (k + (int64_t)(h + 1) * (m + (int64_t)M * r)), xk, sizeof(double) * d);
    if (in->ghq_w) {
      /* GaussHermiteObservable (observables.jl:58-66): y = μ + √2 σ t_k, ∇y = ∇μ + √2 ∇σ t_k on
       * fantasy_index k-1; the recorded gradient is get_gradient's weights[k]·∇y (the later
       * override at observables.jl:157 is the one Julia dispatches to). */
      const double tk = in->ghq_nodes[(int64_t)m + (int64_t)M * k], wk = in->ghq_w[(int64_t)m + (int64_t)M * k];
      fsur_eval(fs, xk, p->theta, p->sigma_tol, k - 1, 0, &sx, sc);
      st |= sx.status;
      obs[k] = sx.mu + SQRT2 * sx.sigma * tk;
      for (int a = 0; a < d; ++a) grads[a + d * k] = wk * (sx.gmu[a] + SQRT2 * sx.gsig[a] * tk);
      z[0] = SQRT2 * tk;
      wmax = fmax(wmax, wk);
    } else {
      for (int a = 0; a < D1; ++a) z[a] = in->rnstream[(int64_t)m + (int64_t)M * a + (int64_t)M * D1 * k];
      st |= fsur_draw(fs, xk, p->theta, p->sigma_tol, k - 1, z, &obs[k], grads + d * k, &sx, sc, kappa);
    }
    if (st) break;
    if (vbound || ylip) {   /* the value bound's terms (rbo_params.vbound / ylip) */
      const int n = fs->N + k;
      const double* cv = fs->cs + (int64_t)k * fs->cap;
      double smu = 0.0, skw = 0.0, yl = 0.0;
      for (int j = 0; j < n; ++j) { smu += fabs(sc->kx[j] * cv[j]); skw += fabs(sc->kx[j] * sc->w[j]); }
      dy[k] = nu * kappa_L * (smu + fabs(z[0]) * (k_psi(&fs->k, 0.0) + skw) / (2.0 * sx.sigma));
      for (int i = 0; i < k; ++i) dy[k] += fabs(sc->w[fs->N + i]) * dy[i];
      if (ylip) {
        for (int a = 0; a < d; ++a) yl += fabs(sx.gmu[a] + z[0] * sx.gsig[a]);
        *ylip = fmax(*ylip, yl);
      }
    }
    st |= fsur_condition(fs, xk, obs[k], sc->tmp);
    if (st) break;
  }
  evals[0] = cx.n_grad;
  evals[1] = cx.n_value;
  evals[2] = cx.n_hess;
  if (obs_out) for (int k = 0; k <= h; ++k) obs_out[k] = st ? NAN : obs[k];
  if (st) {
    *value = NAN;
    for (int a = 0; a < d; ++a) gx[a] = NAN;
    *gth = NAN;
    if (vbound) *vbound = NAN;
    return st;
  }
  if (vbound) {
    double mx = 0.0;
    for (int k = 0; k <= h; ++k) mx = fmax(mx, dy[k]);
    *vbound = 2.0 * mx * (in->ghq_w ? wmax / SQRTPI : 1.0);
  }
  /* resolve (observables.jl:12-14) with fmini over the capacity buffer (Q3) */
  double bo = obs[0];
  int t = 0;
  for (int k = 1; k <= h; ++k) if (obs[k] < bo) { bo = obs[k]; t = k; }
  *value = fmax(in->s->fmini - bo, 0.0);
  /* resolve(gho; fmini) observables.jl:66-72: weight of the best step, / √π */
  if (in->ghq_w) *value *= in->ghq_w[(int64_t)m + (int64_t)M * t] / SQRTPI;
  for (int a = 0; a < d; ++a) gx[a] = 0;
  *gth = 0;
  if (!p->with_gradient) return 0;
  if (in->s->fmini <= bo) return 0;                 /* Case #1 */
  if (t == 0) {                                     /* Case #2 (Q10) */
    for (int a = 0; a < d; ++a) gx[a] = -grads[a];
    return 0;
  }
  /* Case #3: recover_policy_solve (:114-124) evaluations, cached (deterministic) */
  sx_t* rec = (sx_t*)malloc(sizeof(sx_t) * (t + 1));
  double** rec_w = (double**)malloc(sizeof(double*) * (t + 1));
  double** rec_Dw = (double**)malloc(sizeof(double*) * (t + 1));
  double** rec_kx = (double**)malloc(sizeof(double*) * (t + 1));
  double** rec_gkx = (double**)malloc(sizeof(double*) * (t + 1));
  for (int i = 0; i <= t; ++i) {
    fsur_eval(fs, fs->X + (int64_t)d * (fs->N + i), p->theta, p->sigma_tol, i - 1, 0, &rec[i], sc);
    const int n = rec[i].n;
    rec_w[i] = (double*)malloc(sizeof(double) * n);
    rec_kx[i] = (double*)malloc(sizeof(double) * n);
    rec_Dw[i] = (double*)malloc(sizeof(double) * n * d);
    rec_gkx[i] = (double*)malloc(sizeof(double) * n * d);
    memcpy(rec_w[i], sc->w, sizeof(double) * n);
    memcpy(rec_kx[i], sc->kx, sizeof(double) * n);
    memcpy(rec_Dw[i], sc->Dw, sizeof(double) * n * d);
    memcpy(rec_gkx[i], sc->gkx, sizeof(double) * n * d);
    rec[i].w = rec_w[i]; rec[i].kx = rec_kx[i]; rec[i].Dw = rec_Dw[i]; rec[i].gkx = rec_gkx[i];
  }
  double xbars[16][16], ybars[17];
  memset(xbars, 0, sizeof xbars);
  for (int i = 0; i <= t; ++i) ybars[i] = 0;
  ybars[t] = 1.0;
  double e_k[16], col[16], dri[256], LU[256];
  int piv[16];
  for (int j = t; j >= 1; --j) {
    /* solve_dual_x (:150-191), solve_index = j */
    {
      const sx_t* sxj = &rec[j];
      memcpy(LU, sxj->Halpha, sizeof(double) * d * d);
      const int sing = lu_small(LU, d, piv);
      const double det = sing ? 0.0 : lu_det(LU, piv, d);
      double xd[16];
      if (det < p->htol) {
        for (int a = 0; a < d; ++a) xd[a] = 0; /* Q4 */
      } else {
        for (int a = 0; a < d; ++a) xd[a] = -grads[a + d * (j - 1)] * ybars[j]; /* Q5 */
        for (int i = j + 1; i <= t; ++i) {
          for (int k = 0; k < d; ++k) {
            for (int a = 0; a < d; ++a) e_k[a] = (a == k) ? 1.0 : 0.0;
            perturb_grad(fs, &rec[i], i - 1, j, e_k, 0, p->theta, p->sigma_tol, sc, col);
            for (int a = 0; a < d; ++a) dri[a + d * k] = col[a];
          }
          for (int k = 0; k < d; ++k) { /* x_dual -= dri_dxj' * xbars[i] */
            double s = 0;
            for (int a = 0; a < d; ++a) s += dri[a + d * k] * xbars[i][a];
            xd[k] -= s;
          }
        }
        /* hessian(sx)' \ x_dual (Hα is symmetric; transpose kept for fidelity) */
        double HT[256];
        for (int b = 0; b < d; ++b) for (int a = 0; a < d; ++a) HT[a + d * b] = sxj->Halpha[b + d * a];
        if (lu_small(HT, d, piv)) { st |= RBO_ST_SINGULAR; }
        else {
          lu_solve(HT, piv, d, xd);
          if (kappa) {
            double A[256];
            for (int b = 0; b < d; ++b) for (int a = 0; a < d; ++a) A[a + d * b] = sxj->Halpha[b + d * a];
            *kappa = fmax(*kappa, cond1(A, HT, piv, d));
          }
        }
      }
      for (int a = 0; a < d; ++a) xbars[j][a] = xd[a];
    }
    /* solve_dual_y (:126-148), solve_index = j-1; δx = rand(dim) (Q6) */
    {
      double dx[16];
      for (int k = 0; k < d; ++k)
        dx[k] = in->dual_y_dx ? in->dual_y_dx[(int64_t)k + (int64_t)d * ((j - 1) + (int64_t)h * (m + (int64_t)M * r))]
                              : rbo_dual_uniform(p->seed, (int64_t)(p->sample_offset + m), j, k);
      double yd = 0;
      for (int i = j; i <= t; ++i) {
        perturb_grad(fs, &rec[i], i - 1, j - 1, dx, 1, p->theta, p->sigma_tol, sc, col);
        double s = 0;
        for (int a = 0; a < d; ++a) s += col[a] * xbars[i][a];
        yd += s;
      }
      ybars[j - 1] = yd;
    }
  }
  /* gather_g (:193-218), gather_q (:220-231) */
  double grad_x[16], grad_t = 0;
  for (int a = 0; a < d; ++a) grad_x[a] = rec[0].gmu[a] * ybars[0];
  for (int j = 1; j <= t; ++j) {
    for (int k = 0; k < d; ++k) {
      for (int a = 0; a < d; ++a) e_k[a] = (a == k) ? 1.0 : 0.0;
      perturb_grad(fs, &rec[j], j - 1, 0, e_k, 0, p->theta, p->sigma_tol, sc, col);
      for (int a = 0; a < d; ++a) dri[a + d * k] = col[a];
    }
    for (int k = 0; k < d; ++k) {
      double s = 0;
      for (int a = 0; a < d; ++a) s += dri[a + d * k] * xbars[j][a];
      grad_x[k] += s;
    }
    double s = 0;
    for (int a = 0; a < d; ++a) s += rec[j].mixed[a] * xbars[j][a];
    grad_t += s;
  }
  for (int a = 0; a < d; ++a) gx[a] = -grad_x[a];
  *gth = -grad_t;
  for (int i = 0; i <= t; ++i) { free(rec_w[i]); free(rec_kx[i]); free(rec_Dw[i]); free(rec_gkx[i]); }
  free(rec); free(rec_w); free(rec_Dw); free(rec_kx); free(rec_gkx);
  if (st) { *value = NAN; for (int a = 0; a < d; ++a) gx[a] = NAN; *gth = NAN; }
  return st;
}

static int simulate_impl(const rbo_surrogate* s, const rbo_params* p, const double* x0s, const double* rnstream,
                         const double* ghq_nodes, const double* ghq_w, const double* xstarts, const double* dual_y_dx,
                         const double* replay_x, double* values, double* grad_x, double* grad_theta, int32_t* status,
                         double* policy_x, double* obs, double* eto, int64_t* evals) {
  if (!s || !p || s->d < 1 || s->d > 16 || p->h < 0 || p->h > 60 || p->M < 1 || p->R < 1) return -1;
  const int d = s->d, M = p->M, R = p->R, h = p->h;
  const int64_t T = (int64_t)M * R;
  traj_in in = {s, p, rnstream, xstarts, dual_y_dx, replay_x, ghq_nodes, ghq_w};
  /* κ_L = ‖L0‖₁‖L0⁻¹‖₁ of the base factor, for the value bound (rbo_params.vbound) */
  double kappa_L = 1.0;
  if (p->vbound) {
    const int N = s->N;
    double* Li = (double*)calloc((size_t)N * N, sizeof(double));
    double nL = 0.0, nLi = 0.0;
    for (int j = 0; j < N; ++j) {   /* column j of L0⁻¹ by forward substitution */
      Li[j + (int64_t)N * j] = 1.0 / s->L[j + (int64_t)N * j];
      for (int i = j + 1; i < N; ++i) {
        double t = 0.0;
        for (int q = j; q < i; ++q) t -= s->L[i + (int64_t)N * q] * Li[q + (int64_t)N * j];
        Li[i + (int64_t)N * j] = t / s->L[i + (int64_t)N * i];
      }
    }
    for (int j = 0; j < N; ++j) {
      double a = 0.0, b = 0.0;
      for (int i = j; i < N; ++i) { a += fabs(s->L[i + (int64_t)N * j]); b += fabs(Li[i + (int64_t)N * j]); }
      nL = fmax(nL, a);
      nLi = fmax(nLi, b);
    }
    kappa_L = nL * nLi;
    free(Li);
  }
#ifdef _OPENMP
  if (p->nthreads > 0) omp_set_num_threads(p->nthreads);
#endif
#pragma omp parallel
  {
    fsur_t fs;
    scratch_t sc;
    fsur_alloc(&fs, s, h, p->rule, p);
    scratch_alloc(&sc, fs.cap, d);
#pragma omp for schedule(dynamic, 1)
    for (int64_t tr = 0; tr < T; ++tr) {
      const int r = (int)(tr / M), m = (int)(tr % M);
      int64_t ev[3] = {0, 0, 0};
      double* kap = p->kappa ? p->kappa + tr : NULL;
      if (kap) *kap = 1.0;
      const int st = run_trajectory(&in, r, m, x0s + (int64_t)d * r, &fs, &sc, values + tr, grad_x + (int64_t)d * tr,
                                    grad_theta + tr, policy_x, obs ? obs + (int64_t)(h + 1) * tr : NULL, ev, kap,
                                    p->vbound ? p->vbound + tr : NULL, p->ylip ? p->ylip + tr : NULL, kappa_L);
      status[tr] = st;
      if (evals) for (int k = 0; k < 3; ++k) evals[3 * tr + k] = ev[k];
    }
    scratch_free(&sc);
    fsur_free(&fs);
  }
  if (eto) {
    /* mean / std(corrected) per restart (rollout.jl:328-339) */
    const int W = 2 + 2 * d + 2;
    for (int r = 0; r < R; ++r) {
      double* e = eto + (int64_t)W * r;
      const double* v = values + (int64_t)M * r;
      double mu = 0;
      for (int m = 0; m < M; ++m) mu += v[m];
      mu /= M;
      double ss = 0;
      for (int m = 0; m < M; ++m) ss += (v[m] - mu) * (v[m] - mu);
      e[0] = mu;
      e[1] = sqrt(ss / (M - 1));
      for (int a = 0; a < d; ++a) {
        double gm = 0, gs = 0;
        for (int m = 0; m < M; ++m) gm += grad_x[(int64_t)a + (int64_t)d * (m + (int64_t)M * r)];
        gm /= M;
        for (int m = 0; m < M; ++m) {
          const double dv = grad_x[(int64_t)a + (int64_t)d * (m + (int64_t)M * r)] - gm;
          gs += dv * dv;
        }
        e[2 + a] = gm;
        e[2 + d + a] = sqrt(gs / (M - 1));
      }
      double tm = 0, ts = 0;
      for (int m = 0; m < M; ++m) tm += grad_theta[m + (int64_t)M * r];
      tm /= M;
      for (int m = 0; m < M; ++m) ts += (grad_theta[m + (int64_t)M * r] - tm) * (grad_theta[m + (int64_t)M * r] - tm);
      e[2 + 2 * d] = tm;
      e[3 + 2 * d] = sqrt(ts / (M - 1));
    }
  }
  return 0;
}

/* base-surrogate evaluation for primitive parity (a6/a7/a8 at fantasy_index = -1) */
int rbo_simulate_mc(const rbo_surrogate* s, const rbo_params* p, const double* x0s, const double* rnstream,
                    const double* xstarts, const double* dual_y_dx, const double* replay_x, double* values,
                    double* grad_x, double* grad_theta, int32_t* status, double* policy_x, double* obs,
                    double* eto, int64_t* evals) {
  if (!rnstream) return -1;
  return simulate_impl(s, p, x0s, rnstream, NULL, NULL, xstarts, dual_y_dx, replay_x, values, grad_x, grad_theta,
                       status, policy_x, obs, eto, evals);
}

int rbo_simulate_ghq(const rbo_surrogate* s, const rbo_params* p, const double* x0s, const double* nodes,
                     const double* weights, const double* xstarts, const double* dual_y_dx, const double* replay_x,
                     double* values, double* grad_x, double* grad_theta, int32_t* status, double* policy_x,
                     double* obs, double* eto, int64_t* evals) {
  if (!nodes || !weights) return -1;
  return simulate_impl(s, p, x0s, NULL, nodes, weights, xstarts, dual_y_dx, replay_x, values, grad_x, grad_theta,
                       status, policy_x, obs, eto, evals);
}

/* ------------------------------------------------------------------------------------
 * Base-GP fit and marginal likelihood (between-step surrogate maintenance)
 *   Surrogate ctor           radial_basis_surrogates.jl:77-118 (K, L = cholesky(K), c = L'\(L\y))
 *   log_likelihood           :770-776   −y'c/2 − Σ log diag(L) − n log(2π)/2
 *   δlog_likelihood          :778-785   (c'δK c − tr(L'\(L\δK)))/2
 *   ∇log_likelihood          :787-799   δθ = e_t for every hyperparameter (ℓ; Periodic ℓ, p)
 *   eval_Dθ_KXX              radial_basis_functions.jl:264-284 (δK_jj = ∇θψ(0)'δθ = 0)
 * ∇θ_ψ (ForwardDiff there, :43) in closed form.
 * ---------------------------------------------------------------------------------- */
static double k_dpsi_dell(const kern_t* k, double rho) {
  switch (k->kind) {
    case RBO_K_MATERN52: { const double s = sqrt(5.0) / k->ell * rho; return (s * s / 3.0) * (1 + s) * exp(-s) / k->ell; }
    case RBO_K_MATERN32: { const double s = sqrt(3.0) / k->ell * rho; return s * s * exp(-s) / k->ell; }
    case RBO_K_MATERN12: { const double s = rho / k->ell; return s * exp(-s) / k->ell; }
    case RBO_K_PERIODIC: {   /* ∂/∂ℓ exp(−2 sin²(πρ/p)/ℓ²) = ψ · 4 sin²(πρ/p)/ℓ³ */
      const double sn = sin(JL_PI * rho / k->per);
      return k_psi(k, rho) * 4 * sn * sn / (k->ell * k->ell * k->ell);
    }
    default: { const double t = rho * rho / (k->ell * k->ell); return exp(-t / 2) * t / k->ell; }
  }
}
/* Periodic: ∂/∂p exp(−2 sin²(πρ/p)/ℓ²) = ψ · (4 sin(u) cos(u)/ℓ²) · πρ/p², u = πρ/p */
static double k_dpsi_dper(const kern_t* k, double rho) {
  const double u = JL_PI * rho / k->per;
  return k_psi(k, rho) * 4 * sin(u) * cos(u) / (k->ell * k->ell) * (JL_PI * rho / (k->per * k->per));
}

int rbo_log_likelihood_theta(int32_t d, int32_t N, int32_t kernel, int32_t nt, const double* theta, double period,
                             double sigma_n2, const double* X, const double* y, double* ll, double* grad,
                             double* L_out, double* c_out) {
  if (nt < 1 || nt > (kernel == RBO_K_PERIODIC ? 2 : 1)) return -1;
  const kern_t k = {kernel, theta[0], (kernel == RBO_K_PERIODIC) ? (nt == 2 ? theta[1] : period) : 1.0};
  const int64_t NN = (int64_t)N * N;
  double* K = (double*)calloc((size_t)NN, sizeof(double));
  double* dK = (double*)calloc((size_t)NN, sizeof(double));
  double* L = (double*)malloc(sizeof(double) * NN);
  double* c = (double*)malloc(sizeof(double) * N);
  double* col = (double*)malloc(sizeof(double) * N);
  double* tmp = (double*)malloc(sizeof(double) * N);
  double r[64];
  for (int j = 0; j < N; ++j)
    for (int i = 0; i < N; ++i) {
      for (int a = 0; a < d; ++a) r[a] = X[a + (int64_t)d * i] - X[a + (int64_t)d * j];
      const double rho = vnorm(r, d);
      K[i + (int64_t)N * j] = (i == j) ? k_psi(&k, 0.0) + sigma_n2 : k_psi(&k, rho);
    }
  int rc = chol_small(K, N, L);
  if (rc == 0) {
    kinv(L, N, N, y, c, tmp);
    double yc = 0, ld = 0;
    for (int i = 0; i < N; ++i) { yc += y[i] * c[i]; ld += log(L[i + (int64_t)N * i]); }
    *ll = -yc / 2 - ld - N * log(2 * JL_PI) / 2;
    /* ∇log_likelihood (:787-799): δlog_likelihood (:778-785) at δθ = e_t, δK = eval_Dθ_KXX */
    for (int t = 0; t < nt; ++t) {
      for (int j = 0; j < N; ++j)
        for (int i = 0; i < N; ++i) {
          for (int a = 0; a < d; ++a) r[a] = X[a + (int64_t)d * i] - X[a + (int64_t)d * j];
          const double rho = vnorm(r, d);
          dK[i + (int64_t)N * j] = (i == j) ? 0.0 : (t == 0 ? k_dpsi_dell(&k, rho) : k_dpsi_dper(&k, rho));
        }
      double cgc = 0, tr = 0;
      for (int j = 0; j < N; ++j) {
        double sj = 0;
        for (int i = 0; i < N; ++i) sj += dK[i + (int64_t)N * j] * c[i];
        cgc += c[j] * sj;
        kinv(L, N, N, dK + (int64_t)N * j, col, tmp);   /* column j of L'\(L\δK) */
        tr += col[j];
      }
      grad[t] = (cgc - tr) / 2;
    }
    if (L_out) memcpy(L_out, L, sizeof(double) * NN);
    if (c_out) memcpy(c_out, c, sizeof(double) * N);
  } else {
    *ll = NAN;
    for (int t = 0; t < nt; ++t) grad[t] = NAN;
  }
  free(K); free(dK); free(L); free(c); free(col); free(tmp);
  return rc == 0 ? 0 : 1;
}

/* one lengthscale (Periodic: ∂/∂ℓ at period 1 is not ∇log_likelihood -- use the θ form) */
int rbo_log_likelihood(int32_t d, int32_t N, int32_t kernel, double ell, double sigma_n2, const double* X,
                       const double* y, double* ll, double* dll, double* L_out, double* c_out) {
  if (kernel == RBO_K_PERIODIC) return -1;
  return rbo_log_likelihood_theta(d, N, kernel, 1, &ell, 1.0, sigma_n2, X, y, ll, dll, L_out, c_out);
}

static int eval_base_impl(const rbo_surrogate* s, int32_t rule, double theta, double sigma_tol, int32_t P,
                          const double* xs, double* out, const rbo_params* cost_p) {
  fsur_t fs;
  scratch_t sc;
  if (rule < 0 || rule > RBO_RULE_LCB) return -1;
  if (fsur_alloc(&fs, s, 0, rule, cost_p)) return -2;
  scratch_alloc(&sc, fs.cap, s->d);
  const int d = s->d, stride = 3 + 4 * d + d * d;
  sx_t sx;
  for (int i = 0; i < P; ++i) {
    fsur_eval(&fs, xs + (int64_t)d * i, theta, sigma_tol, -1, 0, &sx, &sc);
    double* o = out + (int64_t)stride * i;
    o[0] = sx.mu; o[1] = sx.sigma; o[2] = sx.alpha;
    for (int a = 0; a < d; ++a) { o[3 + a] = sx.gmu[a]; o[3 + d + a] = sx.gsig[a]; o[3 + 2 * d + a] = sx.galpha[a]; }
    for (int q = 0; q < d * d; ++q) o[3 + 3 * d + q] = sx.Halpha[q];
    for (int a = 0; a < d; ++a) o[3 + 3 * d + d * d + a] = sx.mixed[a];
  }
  scratch_free(&sc);
  fsur_free(&fs);
  return 0;
}

/* base_solve(s::Surrogate; xstart) rbf_optim.jl:35-66 for every column of xstarts (d×n) on the
 * base surrogate (fantasy index -1): the build's projected Newton (newton_solve) with p's rule,
 * θ, box and options; the caller's findmin over the candidates is multistart_base_solve!(s, …)
 * (:103-135).  evals: optional 3×n [gradient, value, Hessian] counts. */
int rbo_base_solve(const rbo_surrogate* s, const rbo_params* p, int32_t n, const double* xstarts, double* xmin,
                   double* fmin, int32_t* status, int64_t* evals) {
  fsur_t fs;
  scratch_t sc;
  if (!s || !p || n < 1 || p->rule < 0 || p->rule > RBO_RULE_LCB) return -1;
  if (fsur_alloc(&fs, s, 0, p->rule, p)) return -2;
  scratch_alloc(&sc, fs.cap, s->d);
  const int d = s->d;
  double cabs = 0;
  for (int j = 0; j < s->N; ++j) cabs += fabs(fs.cs[j]);
  for (int i = 0; i < n; ++i) {
    solve_ctx cx;
    memset(&cx, 0, sizeof cx);
    cx.fs = &fs;
    cx.p = p;
    cx.fi = -1;
    cx.sc = &sc;
    cx.cabs = cabs;
    newton_solve(&cx, xstarts + (int64_t)d * i, xmin + (int64_t)d * i, fmin + i);
    status[i] = cx.st;
    if (evals) {
      evals[3 * (int64_t)i + 0] = cx.n_grad;
      evals[3 * (int64_t)i + 1] = cx.n_value;
      evals[3 * (int64_t)i + 2] = cx.n_hess;
    }
  }
  scratch_free(&sc);
  fsur_free(&fs);
  return 0;
}

int rbo_eval_base(const rbo_surrogate* s, int32_t rule, double theta, double sigma_tol, int32_t P, const double* xs,
                  double* out) {
  return eval_base_impl(s, rule, theta, sigma_tol, P, xs, out, NULL);
}

int rbo_eval_base_p(const rbo_surrogate* s, const rbo_params* p, int32_t P, const double* xs, double* out) {
  if (!p) return -1;
  return eval_base_impl(s, p->rule, p->theta, p->sigma_tol, P, xs, out, p);
}
