// mrbo_gpfit.hip -- base-GP fit and its marginal likelihood for a batch of lengthscales.
//
// Restates, one workgroup per candidate lengthscale ℓ_p:
//   Surrogate(ψ, X, y)       radial_basis_surrogates.jl:77-118   K = Ψ(‖Xi−Xj‖) + σn2·I, L = chol(K),
//                                                               c = L'\(L\y)
//   log_likelihood(s)        radial_basis_surrogates.jl:770-776  −yᵀc/2 − Σ log L_ii − n·log(2π)/2
//   δlog_likelihood(s, δθ)   radial_basis_surrogates.jl:778-785  (cᵀ δK c − tr(L'\(L\δK)))/2,
//   eval_Dθ_KXX              radial_basis_functions.jl:264-284   δK_ij = ∂ψ/∂ℓ(‖Xi−Xj‖), δK_jj = ∂ψ/∂ℓ(0) = 0
// which optimize! (radial_basis_surrogates.jl:805-829) evaluates once per L-BFGS iterate.
//
// N ≤ 64 (gpfit_wave_kernel): ONE WAVE per candidate, lanes = rows (columns in the inverse), the
// factor and L⁻¹ in the wave's LDS (leading dimension 65: row and column walks conflict free),
// no workgroup barriers.  tr(K⁻¹δK) = Σ_ab (L⁻ᵀL⁻¹)_ab δK_ab from V = L⁻¹ (N³/6) and the lower
// triangle of VᵀV (N³/6); δK lives in the unused upper triangle of the factor.
// N > 64 (gpfit_kernel): one workgroup per candidate; N³/3 (Cholesky) + N³/2 (Z = L⁻¹δK) + N³/6
// (L⁻¹) FMAs on a global workspace (3·N² doubles per candidate, L2-resident at N ≤ 256).
// Column-parallel steps map one thread to one column; the right-looking Cholesky updates the
// trailing triangle with all 256 threads between block barriers.
#include <hip/hip_runtime.h>

#include "mrbo_dispatch.h"

namespace mrbo {

// ψ(ρ) and ∂ψ/∂ℓ(ρ) for the radial kernels (radial_basis_functions.jl:60-96; ∇θ_ψ by
// ForwardDiff there, closed forms here)
__device__ __forceinline__ void psi_dell(int kind, double ell, double rho, double& psi, double& dpsi) {
  if (kind == 3) {  // SE: exp(−ρ²/(2ℓ²))
    const double t = rho * rho / (ell * ell);
    psi = exp(-0.5 * t);
    dpsi = psi * t / ell;
    return;
  }
  const double c = (kind == 0) ? sqrt(5.0) / ell : (kind == 1) ? sqrt(3.0) / ell : 1.0 / ell;
  const double s = c * rho, e = exp(-s);
  if (kind == 0) {          // (1+s+s²/3)e⁻ˢ ; ∂/∂ℓ = (s²/3)(1+s)e⁻ˢ/ℓ
    psi = (1.0 + s * (1.0 + s / 3.0)) * e;
    dpsi = (s * s / 3.0) * (1.0 + s) * e / ell;
  } else if (kind == 1) {   // (1+s)e⁻ˢ ; ∂/∂ℓ = s²e⁻ˢ/ℓ
    psi = (1.0 + s) * e;
    dpsi = s * s * e / ell;
  } else {                  // e⁻ˢ ; ∂/∂ℓ = s e⁻ˢ/ℓ
    psi = e;
    dpsi = s * e / ell;
  }
}

constexpr int GPFIT_THREADS = 256;

__device__ __forceinline__ double block_sum(double v, double* sh) {
  const int t = threadIdx.x;
  sh[t] = v;
  __syncthreads();
  for (int s = GPFIT_THREADS / 2; s > 0; s >>= 1) {
    if (t < s) sh[t] += sh[t + s];
    __syncthreads();
  }
  const double r = sh[0];
  __syncthreads();
  return r;
}

// one workgroup per candidate p; work = 3·N² doubles per candidate: A (K → L, column-major),
// G (δK, then L⁻¹δK row-major) and V (L⁻¹, row-major), leading dimension N
__global__ void __launch_bounds__(GPFIT_THREADS) gpfit_kernel(GpFitParams q) {
  __shared__ double sh[GPFIT_THREADS];
  __shared__ double cv[256];
  __shared__ int fail;
  const int N = q.N, d = q.d, t = threadIdx.x, p = blockIdx.x;
  const double ell = q.ells[p];
  double* A = q.work + (size_t)3 * N * N * p;
  double* G = A + (size_t)N * N;
  double* V = G + (size_t)N * N;
  if (t == 0) fail = 0;
  // K and δK (eval_KXX :161-178 with ψ(0) on the diagonal; eval_Dθ_KXX :264-284)
  for (int idx = t; idx < N * N; idx += GPFIT_THREADS) {
    const int i = idx % N, j = idx / N;
    double r2 = 0.0;
    for (int a = 0; a < d; ++a) {
      const double r = q.X[a + d * i] - q.X[a + d * j];
      r2 += r * r;
    }
    double psi, dpsi;
    psi_dell(q.kernel, ell, (i == j) ? 0.0 : sqrt(r2), psi, dpsi);
    A[idx] = (i == j) ? psi + q.sn2 : psi;
    G[idx] = (i == j) ? 0.0 : dpsi;
  }
  __syncthreads();
  // right-looking Cholesky, lower triangle of A in place (PosDefException → status 1)
  for (int k = 0; k < N; ++k) {
    const double piv = A[k + N * k];
    if (!(piv > 0.0)) {
      if (t == 0) fail = 1;
      break;
    }
    const double lkk = sqrt(piv);
    __syncthreads();   // every thread has read the pivot before it is overwritten
    for (int i = k + t; i < N; i += GPFIT_THREADS) A[i + N * k] = (i == k) ? lkk : A[i + N * k] / lkk;
    __syncthreads();
    const int m = N - k - 1;
    for (int idx = t; idx < m * m; idx += GPFIT_THREADS) {
      const int i = k + 1 + idx % m, j = k + 1 + idx / m;
      if (j <= i) A[i + N * j] -= A[i + N * k] * A[j + N * k];
    }
    __syncthreads();
  }
  __syncthreads();
  if (fail) {
    if (t == 0) { q.ll[p] = NAN; q.dll[p] = NAN; q.status[p] = 1; }
    return;
  }
  // c = L'\(L\y): column-oriented substitutions, c in LDS
  for (int i = t; i < N; i += GPFIT_THREADS) cv[i] = q.y[i];
  __syncthreads();
  for (int k = 0; k < N; ++k) {
    const double ck = cv[k] / A[k + N * k];
    __syncthreads();
    if (t == 0) cv[k] = ck;
    for (int i = k + 1 + t; i < N; i += GPFIT_THREADS) cv[i] -= A[i + N * k] * ck;
    __syncthreads();
  }
  for (int k = N - 1; k >= 0; --k) {
    const double ck = cv[k] / A[k + N * k];
    __syncthreads();
    if (t == 0) cv[k] = ck;
    for (int i = t; i < k; i += GPFIT_THREADS) cv[i] -= A[k + N * i] * ck;
    __syncthreads();
  }
  // log_likelihood (:770-776) and cᵀδKc (thread j: c_j Σ_i δK_ij c_i)
  double yc = 0.0, ld = 0.0, cgc = 0.0;
  for (int j = t; j < N; j += GPFIT_THREADS) {
    yc += q.y[j] * cv[j];
    ld += log(A[j + N * j]);
    double s = 0.0;
    for (int i = 0; i < N; ++i) s += G[(size_t)N * i + j] * cv[i];   // δK symmetric: coalesced in j
    cgc += cv[j] * s;
  }
  yc = block_sum(yc, sh);
  ld = block_sum(ld, sh);
  cgc = block_sum(cgc, sh);
  // tr(L'\(L\δK)) = tr(L⁻ᵀL⁻¹δK) = Σ_ij (L⁻¹δK)_ij (L⁻¹)_ij: thread j forward-substitutes
  // column j of δK (in place → Z) and of the identity (→ V), rows ascending.  Z and V are kept
  // row-major (entry (i, j) at i·N + j) so that the threads' loads are coalesced; δK is
  // symmetric, so G read row-major is δK itself.  L[i][k] is a wave-uniform broadcast.
  double tr = 0.0;
  for (int j = t; j < N; j += GPFIT_THREADS) {
    for (int i = 0; i < N; ++i) {
      double z = G[(size_t)N * i + j], v = (i == j) ? 1.0 : 0.0;
      for (int k = 0; k < i; ++k) {
        const double lik = A[i + N * k];
        z -= lik * G[(size_t)N * k + j];
        v -= lik * V[(size_t)N * k + j];
      }
      const double li = A[i + N * i];
      z /= li;
      v /= li;
      G[(size_t)N * i + j] = z;
      V[(size_t)N * i + j] = v;
      tr += z * v;
    }
  }
  tr = block_sum(tr, sh);
  if (t == 0) {
    q.ll[p] = -0.5 * yc - ld - 0.5 * N * log(2.0 * 3.141592653589793);
    q.dll[p] = 0.5 * (cgc - tr);
    q.status[p] = 0;
  }
  // optional fit outputs: L (lower, zeros above) and c of each candidate
  if (q.L_out) {
    double* Lo = q.L_out + (size_t)N * N * p;
    for (int idx = t; idx < N * N; idx += GPFIT_THREADS) {
      const int i = idx % N, j = idx / N;
      Lo[idx] = (i >= j) ? A[idx] : 0.0;
    }
  }
  if (q.c_out)
    for (int i = t; i < N; i += GPFIT_THREADS) q.c_out[(size_t)N * p + i] = cv[i];
}

// ---- N ≤ 64: one wave per candidate ---------------------------------------------------
#ifndef MRBO_GW_WAVES
#define MRBO_GW_WAVES 1   // A/B at P = 256, N = 64: 1 wave per group 0.287 ms, 2 waves 0.292 ms
#endif
constexpr int GW_N = 64, GW_LD = GW_N + 1, GW_WAVES = MRBO_GW_WAVES;   // waves (candidates) per workgroup
constexpr int GW_WAVE_DOUBLES = 2 * GW_N * GW_LD + GW_N;   // A, V, c

__device__ __forceinline__ double gw_sum(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__global__ void __launch_bounds__(64 * GW_WAVES) gpfit_wave_kernel(GpFitParams q, int P) {
  extern __shared__ __attribute__((aligned(16))) double gsm[];
  const int w = threadIdx.x / 64, lane = threadIdx.x & 63;
  const int p = blockIdx.x * GW_WAVES + w;
  if (p >= P) return;   // whole waves: no barrier follows
  double* A = gsm + (size_t)w * GW_WAVE_DOUBLES;   // L lower (row-major i·LD + j), δK strict upper (j·LD + i)
  double* V = A + GW_N * GW_LD;                    // L⁻¹ lower, zeros above
  double* cs = V + GW_N * GW_LD;
  const int N = q.N, d = q.d, i = lane;
  const bool act = i < N;
  const double ell = q.ells[p];
#ifdef MRBO_GPFIT_STAMPS
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
#define WSTAMP(id) do { const unsigned long long t1 = __builtin_amdgcn_s_memtime(); \
    if (p == 0 && lane == 0) printf("gw %d %d\n", id, (int)(t1 - t0)); t0 = t1; } while (0)
#else
#define WSTAMP(id) ((void)0)
#endif
  // K (eval_KXX :161-178, ψ(0) + σn2 on the diagonal) and δK (eval_Dθ_KXX :264-284)
  double xi[8];
#pragma unroll
  for (int a = 0; a < 8; ++a) xi[a] = (a < d && act) ? q.X[a + d * i] : 0.0;
  for (int j = 0; j < N; ++j) {
    double r2 = 0.0;
#pragma unroll
    for (int a = 0; a < 8; ++a)
      if (a < d) { const double r = xi[a] - q.X[a + d * j]; r2 += r * r; }
    double psi, dpsi;
    psi_dell(q.kernel, ell, (i == j) ? 0.0 : sqrt(r2), psi, dpsi);
    if (act && j <= i) A[i * GW_LD + j] = (i == j) ? psi + q.sn2 : psi;
    if (act && j < i) A[j * GW_LD + i] = dpsi;
    V[j * GW_LD + i] = 0.0;
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  WSTAMP(0);
  // right-looking Cholesky in place (lane i owns row i); PosDefException → status 1
  bool fail = false;
  for (int k = 0; k < N; ++k) {
    const double piv = A[k * GW_LD + k];
    if (!(piv > 0.0)) { fail = true; break; }
    const double lkk = sqrt(piv);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    if (act && i == k) A[k * GW_LD + k] = lkk;
    if (act && i > k) A[i * GW_LD + k] /= lkk;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    const double lik = (act && i > k) ? A[i * GW_LD + k] : 0.0;
#pragma unroll 8
    for (int j = k + 1; j < N; ++j) {
      const double ljk = A[j * GW_LD + k];
      if (act && j <= i) A[i * GW_LD + j] -= lik * ljk;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  }
  if (fail) {
    if (lane == 0) { q.ll[p] = NAN; q.dll[p] = NAN; q.status[p] = 1; }
    return;
  }
  // c = L'\(L\y)
  WSTAMP(1);
  double c = act ? q.y[i] : 0.0;
  for (int k = 0; k < N; ++k) {
    const double ck = __shfl(c, k, 64) / A[k * GW_LD + k];
    if (i == k) c = ck;
    else if (act && i > k) c -= A[i * GW_LD + k] * ck;
  }
  for (int k = N - 1; k >= 0; --k) {
    const double ck = __shfl(c, k, 64) / A[k * GW_LD + k];
    if (i == k) c = ck;
    else if (i < k) c -= A[k * GW_LD + i] * ck;
  }
  cs[lane] = act ? c : 0.0;
  // log_likelihood (:770-776)
  const double yc = gw_sum(act ? q.y[i] * c : 0.0);
  const double ld = gw_sum(act ? log(A[i * GW_LD + i]) : 0.0);
  WSTAMP(2);
  // V = L⁻¹, lane j = column j, rows ascending (same order as a forward substitution of e_j)
  for (int r = 0; r < N; ++r) {
    double acc = (r == i) ? 1.0 : 0.0;
#pragma unroll 8
    for (int m = 0; m < r; ++m) acc -= A[r * GW_LD + m] * V[m * GW_LD + i];
    if (r >= i) V[r * GW_LD + i] = acc / A[r * GW_LD + r];
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  WSTAMP(3);
  // K⁻¹_ab = Σ_{m ≥ a} V_ma V_mb (lane a, b < a); tr(K⁻¹δK) and cᵀδKc over a > b (δK_aa = 0)
  double tr = 0.0, cgc = 0.0;
  for (int b = 0; b < N; ++b) {
    double kab = 0.0;
#pragma unroll 8
    for (int m = b; m < N; ++m) kab += V[m * GW_LD + i] * V[m * GW_LD + b];
    if (act && b < i) {
      const double dk = A[b * GW_LD + i];
      tr += kab * dk;
      cgc += c * cs[b] * dk;
    }
  }
  WSTAMP(4);
  tr = 2.0 * gw_sum(tr);
  cgc = 2.0 * gw_sum(cgc);
  if (lane == 0) {
    q.ll[p] = -0.5 * yc - ld - 0.5 * N * log(2.0 * 3.141592653589793);
    q.dll[p] = 0.5 * (cgc - tr);
    q.status[p] = 0;
  }
  if (q.L_out) {
    double* Lo = q.L_out + (size_t)N * N * p;
    for (int j = 0; j < N; ++j)
      if (act) Lo[i + (size_t)N * j] = (i >= j) ? A[i * GW_LD + j] : 0.0;
  }
  if (q.c_out && act) q.c_out[(size_t)N * p + i] = c;
}

void launch_gpfit(int P, hipStream_t st, const GpFitParams& q) {
  if (gpfit_in_lds(q.N, q.d)) {
    hipLaunchKernelGGL(gpfit_wave_kernel, dim3((P + GW_WAVES - 1) / GW_WAVES), dim3(64 * GW_WAVES),
                       sizeof(double) * GW_WAVES * GW_WAVE_DOUBLES, st, q, P);
    return;
  }
  hipLaunchKernelGGL(gpfit_kernel, dim3(P), dim3(GPFIT_THREADS), 0, st, q);
}

}  // namespace mrbo
