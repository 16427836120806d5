// mrbo_device.h -- device-side building blocks of the MI355X rollout evaluator.
//
// Execution model: one 64-lane wavefront owns one trajectory at a time
// (persistent waves pull (restart, sample) pairs from a device work queue).  Lane i owns GP
// data row i of the base surrogate (RPL rows per lane when N > 64).  The base inverse
// Cholesky factor L0⁻¹ is staged once per workgroup in LDS (packed, column-major, padded so
// that both the row- and the column-walk of the triangular products are bank-conflict
// free); the ≤ h+1 fantasy rows of the trajectory live in a per-wave global slot (L1/L2
// resident) and in per-wave LDS.  Quantities that are uniform across the wave (μ, σ, the
// Gram matrix, the acquisition Hessian, the Newton state) are produced by wave reductions
// and then finished by *distributed* lane-uniform math: lane l owns entry l of the small
// matrix in LDS, so no lane replays the whole O(d²)–O(d³) bookkeeping.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mrbo {

constexpr int FMAX = 6;    // fantasy points per trajectory = h+1  (h ≤ 5)
constexpr int WAVE = 64;

// evaluation modes (wave-uniform)
enum { EV_VALUE = 0, EV_DRAW = 1, EV_FULL = 2, EV_RICH = 3 };

struct KParams {
  int d, N, Npad, h, M, R, nstarts;
  int kernel;
  double ell, cK, psi0, d2psi0, sn2;
  double fmin_base, fmini, theta;
  int max_iters, max_ls;
  double x_tol, f_tol, g_tol, htol, sigma_tol;
  unsigned long long seed;
  int sample_offset, samples_total;
  int with_gradient;
  const double* X0;     // [d][NR]   lane-major base covariates
  const double* c0;     // [NR]      base coefficients
  const double* Linv;   // packed L0⁻¹ (see linv_index)
  const double* lbs;    // d
  const double* ubs;    // d
  const double* x0s;    // d×R
  const double* rn;     // M×(d+1)×(h+1)
  const double* xstarts;// d×nstarts
  const double* dual_y; // d×h×M×R or null
  const double* replay; // d×h×M×R or null
  double* values;
  double* grad_x;
  double* grad_theta;
  int* status;
  double* policy;
  double* obs;
  long long* evals;
  double* work;         // per wave-slot global scratch
  long long work_stride;
  int* queue;           // work-queue head (zeroed before every launch)
  long long T;          // trajectories (or points for eval_base)
  const double* pts;    // eval_base: d×P
  double* pts_out;      // eval_base output
};

// ---- packed L0⁻¹ layout: column j holds rows j..Npad-1 contiguously ----------------------
__host__ __device__ __forceinline__ long long linv_colstart(int j, int Npad) {
  return (long long)j * Npad - (long long)j * (j - 1) / 2;
}
__host__ __device__ __forceinline__ long long linv_size(int Npad) { return (long long)Npad * (Npad + 1) / 2; }

// ---- wave-scope synchronisation for LDS hand-offs between lanes of ONE wave ------------
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ double shfl_xor_d(double v, int m) { return __shfl_xor(v, m, WAVE); }

// Transpose-reduce K per-lane values across the 64 lanes: after log2(K) butterfly steps
// each lane holds one partial, then plain xor steps finish; one lane per group writes
// red[idx].  Cost ≈ K+log2(64/K) shuffles instead of 6K.  Deterministic order.
template <int K>
__device__ __forceinline__ void wave_reduce(double (&v)[K], double* red, int lane) {
  constexpr int S = (K == 1) ? 0 : (K == 2) ? 1 : (K == 4) ? 2 : (K == 8) ? 3 : (K == 16) ? 4 : 5;
  static_assert((1 << S) == K, "K must be a power of two <= 32");
  int idx = 0;
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const int m = 32 >> s;
    constexpr int dummy = 0;
    (void)dummy;
    const int half = K >> (s + 1);
    const bool up = (lane & m) != 0;
#pragma unroll
    for (int q = 0; q < (K >> (s + 1)); ++q) {
      const double send = up ? v[q] : v[q + half];
      const double keep = up ? v[q + half] : v[q];
      v[q] = keep + shfl_xor_d(send, m);
    }
    idx += up ? half : 0;
  }
#pragma unroll
  for (int m = (32 >> S); m >= 1; m >>= 1) v[0] += shfl_xor_d(v[0], m);
  if ((lane & ((64 >> S) - 1)) == 0) red[idx] = v[0];
}

// ---- transcendentals behind leaf calls ---------------------------------------------------
// The fp64 exp/erfc expansions carry tens of 64-bit polynomial constants; inlined into the
// Newton/horizon loops, LICM hoists their materialisation out of the loops and the kernel
// spills them.  As leaf calls the constants stay local to the callee.
#ifdef MRBO_INLINE_TRANSCENDENTALS
__device__ __forceinline__ double xexp(double x) { return exp(x); }
__device__ __forceinline__ double xerfc(double x) { return erfc(x); }
#else
__device__ __attribute__((noinline)) double xexp(double x) { return exp(x); }
__device__ __attribute__((noinline)) double xerfc(double x) { return erfc(x); }
#endif

// ---- radial kernels (radial_basis_functions.jl:60-96; derivatives in closed form) -------
struct Radial {
  int kind;
  double cK;   // √5/ℓ, √3/ℓ, 1/ℓ  (Matérn) ; 1/ℓ² (SE)
};

__device__ __forceinline__ void rad_psi(const Radial& k, double rho, double& psi, double& dpsi) {
  if (k.kind == 0) {
    const double s = k.cK * rho, e = xexp(-s);
    psi = (1.0 + s * (1.0 + s / 3.0)) * e;
    dpsi = -k.cK * (s / 3.0) * (1.0 + s) * e;
  } else if (k.kind == 1) {
    const double s = k.cK * rho, e = xexp(-s);
    psi = (1.0 + s) * e;
    dpsi = -k.cK * s * e;
  } else if (k.kind == 2) {
    const double e = xexp(-k.cK * rho);
    psi = e;
    dpsi = -k.cK * e;
  } else {
    const double e = xexp(-0.5 * rho * rho * k.cK);
    psi = e;
    dpsi = -(rho * k.cK) * e;
  }
}
__device__ __forceinline__ void rad_psi12(const Radial& k, double rho, double& dpsi, double& d2psi) {
  if (k.kind == 0) {
    const double s = k.cK * rho, e = xexp(-s);
    dpsi = -k.cK * (s / 3.0) * (1.0 + s) * e;
    d2psi = k.cK * k.cK * (s * s - s - 1.0) * e / 3.0;
  } else if (k.kind == 1) {
    const double s = k.cK * rho, e = xexp(-s);
    dpsi = -k.cK * s * e;
    d2psi = k.cK * k.cK * (s - 1.0) * e;
  } else if (k.kind == 2) {
    const double e = xexp(-k.cK * rho);
    dpsi = -k.cK * e;
    d2psi = k.cK * k.cK * e;
  } else {
    const double e = xexp(-0.5 * rho * rho * k.cK);
    dpsi = -(rho * k.cK) * e;
    d2psi = (rho * rho * k.cK * k.cK - k.cK) * e;
  }
}

// EI and its partials (decision_rules.jl:84-99); zero when σ < σtol.
struct EIp {
  double g, gmu, gsig, gmumu, gsigsig, gmuth, gsigth;
};
__device__ __forceinline__ EIp ei_partials(double mu, double sig, double theta, double fmin, double sigma_tol) {
  EIp e;
  if (!(sig >= sigma_tol) && !(sig != sig)) {  // σ < σtol (NaN falls through, as in Julia)
    e.g = e.gmu = e.gsig = e.gmumu = e.gsigsig = e.gmuth = e.gsigth = 0.0;
    return e;
  }
  const double imp = fmin - mu - theta;
  const double z = imp / sig;
  const double Phi = xerfc(-z * 0.7071067811865476) / 2.0;
  const double phi = xexp(-(z * z) / 2.0) * 0.3989422804014327;
  e.g = imp * Phi + sig * phi;
  e.gmu = -Phi;
  e.gsig = phi;
  e.gmumu = phi / sig;
  e.gsigsig = z * z * phi / sig;
  e.gmuth = phi / sig;
  e.gsigth = z * phi / sig;
  return e;
}
// first partials only, at (μ', σ') -- the perturbation "second-order" coefficients (Q7, Q8)
__device__ __forceinline__ void ei_first(double mu, double sig, double theta, double fmin, double sigma_tol,
                                         double& gmu, double& gsig) {
  if (!(sig >= sigma_tol) && !(sig != sig)) { gmu = 0.0; gsig = 0.0; return; }
  const double z = (fmin - mu - theta) / sig;
  gmu = -(xerfc(-z * 0.7071067811865476) / 2.0);
  gsig = xexp(-(z * z) / 2.0) * 0.3989422804014327;
}

// counter-based uniform (bit-identical to the host / oracle version)
__host__ __device__ __forceinline__ unsigned long long splitmix64(unsigned long long z) {
  z += 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}
__host__ __device__ __forceinline__ double dual_uniform(unsigned long long seed, long long traj, int j, int k) {
  unsigned long long key = splitmix64(seed ^ 0x5851F42D4C957F2DULL);
  key = splitmix64(key ^ (unsigned long long)traj);
  key = splitmix64(key ^ (((unsigned long long)(unsigned)j << 32) | (unsigned)k));
  return (double)(key >> 11) * (1.0 / 9007199254740992.0);
}

__device__ __forceinline__ double clampd(double v, double lo, double hi) { return v < lo ? lo : (v > hi ? hi : v); }

}  // namespace mrbo
