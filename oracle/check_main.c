/*
 * check_main.c -- sanitizer driver for the CPU oracle (TEST INFRASTRUCTURE, SURVEY.md §5:
 * "ASan/UBSan on the CPU restatement").  `make -C oracle check` builds rbo_oracle.c with
 * -fsanitize=address,undefined and runs every entry point on small synthetic problems:
 * rnstream / starts / Kronecker, base evaluation, full rollouts with the inner Newton solve and
 * the adjoint (MC and Gauss–Hermite), replayed rollouts, h = 0, the log likelihood, and the
 * NonUniformCost variant.  Any invalid access, leak or UB aborts with a report; exit 0 means clean.
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "rbo_oracle.h"

static int fails = 0;
#define CHECK(cond, ...)                         \
  do {                                           \
    if (!(cond)) {                               \
      fprintf(stderr, "check failed: " __VA_ARGS__); \
      fputc('\n', stderr);                       \
      ++fails;                                   \
    }                                            \
  } while (0)

/* K = Matérn-5/2(ρ/ℓ) + σn2 I, L = chol(K), c = K⁻¹y (plain, independent of the oracle) */
static void fit(int d, int N, double ell, const double* X, const double* y, double* L, double* c) {
  double* K = calloc((size_t)N * N, sizeof(double));
  for (int j = 0; j < N; ++j)
    for (int i = 0; i < N; ++i) {
      double r2 = 0;
      for (int a = 0; a < d; ++a) { const double t = X[a + d * i] - X[a + d * j]; r2 += t * t; }
      const double s = sqrt(5.0) * sqrt(r2) / ell;
      K[i + N * j] = (1 + s + s * s / 3) * exp(-s) + (i == j ? 1e-6 : 0.0);
    }
  memset(L, 0, sizeof(double) * N * N);
  for (int j = 0; j < N; ++j) {
    double s = K[j + N * j];
    for (int k = 0; k < j; ++k) s -= L[j + N * k] * L[j + N * k];
    L[j + N * j] = sqrt(s);
    for (int i = j + 1; i < N; ++i) {
      double t = K[i + N * j];
      for (int k = 0; k < j; ++k) t -= L[i + N * k] * L[j + N * k];
      L[i + N * j] = t / L[j + N * j];
    }
  }
  double* t = malloc(sizeof(double) * N);
  for (int i = 0; i < N; ++i) {
    double s = y[i];
    for (int k = 0; k < i; ++k) s -= L[i + N * k] * t[k];
    t[i] = s / L[i + N * i];
  }
  for (int i = N - 1; i >= 0; --i) {
    double s = t[i];
    for (int k = i + 1; k < N; ++k) s -= L[k + N * i] * c[k];
    c[i] = s / L[i + N * i];
  }
  free(t);
  free(K);
}

static void run_case(int testfn, int d, int N, int h, int M, int R, double lo, double hi, double ell, int cost) {
  const int ns = 16, S = ns + 2, D1 = d + 1;
  double* X = malloc(sizeof(double) * d * N);
  double* y = malloc(sizeof(double) * N);
  double* L = malloc(sizeof(double) * N * N);
  double* c = malloc(sizeof(double) * N);
  double lbs[16], ubs[16], w[16];
  for (int a = 0; a < d; ++a) { lbs[a] = lo; ubs[a] = hi; w[a] = 0.5 + 0.25 * a; }
  rbo_kronecker_quasirand(d, N, 0, X);
  for (int i = 0; i < d * N; ++i) X[i] = lo + (hi - lo) * X[i];
  for (int i = 0; i < N; ++i) y[i] = rbo_testfn(testfn, d, X + d * i);
  fit(d, N, ell, X, y, L, c);
  double fmini = y[0];
  for (int i = 1; i < N; ++i) fmini = fmin(fmini, y[i]);
  rbo_surrogate s = {d, N, RBO_K_MATERN52, ell, 1e-6, fmini, X, L, c, y, 1.0};
  double* x0s = malloc(sizeof(double) * d * R);
  rbo_kronecker_quasirand(d, R, N, x0s);
  for (int i = 0; i < d * R; ++i) x0s[i] = lo + (hi - lo) * x0s[i];
  double* rn = malloc(sizeof(double) * M * D1 * (h + 1));
  CHECK(rbo_gen_low_discrepancy_sequence(M, d, h + 1, rn) == 0, "rnstream d=%d", d);
  double* xs = malloc(sizeof(double) * d * S);
  CHECK(rbo_generate_initial_guesses(ns, d, lbs, ubs, xs) == 0, "starts d=%d", d);
  const int64_t T = (int64_t)M * R;
  const int W = 2 + 2 * d + 2;
  double* values = malloc(sizeof(double) * T);
  double* gx = malloc(sizeof(double) * d * T);
  double* gt = malloc(sizeof(double) * T);
  int32_t* st = malloc(sizeof(int32_t) * T);
  double* pol = malloc(sizeof(double) * d * (h + 1) * T);
  double* obs = malloc(sizeof(double) * (h + 1) * T);
  double* eto = malloc(sizeof(double) * W * R);
  int64_t* ev = malloc(sizeof(int64_t) * 3 * T);
  rbo_params p = {h, M, R, S, 0.0, lbs, ubs, 50, 20, 1e-3, 1e-3, 1e-8, 1e-4, 1e-8, 1906, 0, 0, 1, 1, RBO_RULE_EI,
                  cost, 1.0, w};
  double* kap = malloc(sizeof(double) * T);
  double* vb = malloc(sizeof(double) * T);
  double* yl = malloc(sizeof(double) * T);
  p.kappa = kap;
  p.vbound = vb;
  p.ylip = yl;
  CHECK(rbo_simulate_mc(&s, &p, x0s, rn, xs, NULL, NULL, values, gx, gt, st, pol, obs, eto, ev) == 0, "mc d=%d", d);
  p.kappa = NULL;
  p.vbound = NULL;
  p.ylip = NULL;
  int ok = 0;
  for (int64_t t = 0; t < T; ++t)
    ok += (st[t] == 0) && isfinite(values[t]) && kap[t] >= 1.0 && vb[t] > 0.0 && isfinite(vb[t]) && yl[t] >= 0.0;
  CHECK(ok == T, "mc d=%d: %d of %lld trajectories ok", d, ok, (long long)T);
  free(kap);
  free(vb);
  free(yl);
  /* replay the policy points just found: same values */
  if (h > 0) {
    double* rp = malloc(sizeof(double) * d * h * T);
    for (int64_t t = 0; t < T; ++t)
      for (int k = 1; k <= h; ++k) memcpy(rp + d * ((k - 1) + h * t), pol + d * (k + (h + 1) * t), sizeof(double) * d);
    double* v2 = malloc(sizeof(double) * T);
    CHECK(rbo_simulate_mc(&s, &p, x0s, rn, xs, NULL, rp, v2, gx, gt, st, NULL, obs, eto, ev) == 0, "replay d=%d", d);
    for (int64_t t = 0; t < T; ++t) CHECK(v2[t] == values[t], "replay value d=%d t=%lld", d, (long long)t);
    free(rp);
    free(v2);
  }
  /* Gauss–Hermite estimator with 3 nodes per step */
  {
    const double tn[3] = {-1.2247448713915890, 0.0, 1.2247448713915890};
    const double tw[3] = {0.29540897515091934, 1.1816359006036772, 0.29540897515091934};
    int Mg = 1;
    for (int k = 0; k <= h; ++k) Mg *= 3;
    if (Mg > M) Mg = M;
    double* nodes = malloc(sizeof(double) * Mg * (h + 1));
    double* wts = malloc(sizeof(double) * Mg * (h + 1));
    for (int m = 0; m < Mg; ++m) {
      int q = m;
      for (int k = 0; k <= h; ++k) { nodes[m + Mg * k] = tn[q % 3]; wts[m + Mg * k] = tw[q % 3]; q /= 3; }
    }
    rbo_params pg = p;
    pg.M = Mg;
    CHECK(rbo_simulate_ghq(&s, &pg, x0s, nodes, wts, xs, NULL, NULL, values, gx, gt, st, pol, obs, eto, ev) == 0,
          "ghq d=%d", d);
    free(nodes);
    free(wts);
  }
  /* base evaluation and the likelihood */
  {
    const int stride = 3 + 4 * d + d * d;
    double* out = malloc(sizeof(double) * stride * S);
    CHECK(rbo_eval_base(&s, RBO_RULE_EI, 0.0, 1e-8, S, xs, out) == 0, "eval_base d=%d", d);
    free(out);
    double ll, dll;
    double* Lo = malloc(sizeof(double) * N * N);
    double* co = malloc(sizeof(double) * N);
    CHECK(rbo_log_likelihood(d, N, RBO_K_MATERN52, ell, 1e-6, X, y, &ll, &dll, Lo, co) == 0 && isfinite(ll),
          "log_likelihood d=%d", d);
    free(Lo);
    free(co);
  }
  free(X); free(y); free(L); free(c); free(x0s); free(rn); free(xs);
  free(values); free(gx); free(gt); free(st); free(pol); free(obs); free(eto); free(ev);
}

int main(void) {
  /* testfn ids: 0 GramacyLee, 1 BraninHoo, 2 Hartmann6D, 3 Ackley */
  run_case(0, 1, 8, 1, 16, 2, 0.5, 2.5, 1.0, 0);
  run_case(1, 2, 24, 2, 8, 2, 0.0, 15.0, 1.0, 0);
  run_case(2, 6, 24, 3, 4, 2, 0.0, 1.0, 0.5, 0);
  run_case(3, 8, 40, 2, 2, 1, -32.768, 32.768, 20.0, 1);
  run_case(2, 6, 16, 0, 4, 1, 0.0, 1.0, 1.0, 2);
  if (fails) {
    fprintf(stderr, "%d oracle checks failed\n", fails);
    return 1;
  }
  printf("oracle sanitizer check: clean\n");
  return 0;
}
