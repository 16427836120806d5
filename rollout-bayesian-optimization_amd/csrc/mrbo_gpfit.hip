// mrbo_gpfit.hip -- base-GP fit and its marginal likelihood for a batch of hyperparameters.
//
// Restates, one candidate θ_p per wave / workgroup:
//   Surrogate(ψ, X, y)       radial_basis_surrogates.jl:77-118   K = Ψ(‖Xi−Xj‖) + σn2·I, L = chol(K),
//                                                               c = L'\(L\y)
//   log_likelihood(s)        radial_basis_surrogates.jl:770-776  −yᵀc/2 − Σ log L_ii − n·log(2π)/2
//   δlog_likelihood(s, δθ)   radial_basis_surrogates.jl:778-785  (cᵀ δK c − tr(L'\(L\δK)))/2,
//   ∇log_likelihood(s)       radial_basis_surrogates.jl:787-799  δθ = e_t for every hyperparameter t
//   eval_Dθ_KXX              radial_basis_functions.jl:264-284   δK_ij = ∂ψ/∂θ_t(‖Xi−Xj‖), δK_jj = 0
// which optimize! (radial_basis_surrogates.jl:805-829) evaluates once per L-BFGS iterate.
// θ = (ℓ) for the Matérn / SE kernels, (ℓ, p) for Periodic (radial_basis_functions.jl:98-103).
//
// N ≤ 32: gpfit_tile_kernel (below) on its single 32 × 32 tile -- the register factor, inverse
// and substitutions of the diagonal step without a panel (a quarter of the 64-row kernel's work).
// 32 < N ≤ 64, no factor output (gpfit_reg_kernel): one workgroup per candidate whose four waves
// evaluate K and δK (one per SIMD); then ONE WAVE, lane i owning row i of K in REGISTERS.  The right-looking Cholesky broadcasts column k with DPP row_newbcast fused into
// v_fmac_f64 (the column's 16-row blocks replicated by permlane swaps, gpfit_asm.h), so the
// N³/6 trailing updates run at the FMA rate with no LDS round trip; c by substitution with
// readlane broadcasts; V = L⁻¹ by columns (lane j = column j) and K⁻¹ = VᵀV with the same DPP
// broadcasts; tr(K⁻¹δK) and cᵀδKc from K⁻¹.  K and δK are evaluated once per pair j ≤ i.  The
// reference's operations (chol, then triangular solves); summation orders differ (tolerance).
// 64 < N ≤ MRBO_GPFIT_LDS_MAX (80), or 32 < N ≤ 64 with L / c requested: gpfit_lds_kernel (below;
// everything in LDS; it holds candidates up to N = 128, but the tile kernel is faster above 80).
// 80 < N ≤ 512: gpfit_tile_kernel (below): one workgroup per candidate, the blocked algorithm on
// 32 × 32 tiles in a global workspace with the tile products on the fp64 matrix cores.
#include <hip/hip_runtime.h>

#include <type_traits>
#include <utility>

#include "mrbo_dispatch.h"
#include "gpfit_asm.h"

namespace mrbo {

// ψ(ρ) and ∂ψ/∂θ_t(ρ) for the radial kernels (radial_basis_functions.jl:60-103; ∇θ_ψ by
// ForwardDiff there, closed forms here).  dps[0] = ∂/∂ℓ; Periodic also dps[1] = ∂/∂p.
// Divisions by the candidate's constants are multiplications by reciprocals formed once per
// candidate (1/ℓ, 1/3, 1/p: loop invariants the compiler hoists out of the pair loops): an IEEE
// f64 division is a ten-instruction dependent chain, three per entry in the Matérn 5/2 case.
template <int KIND>
__device__ __forceinline__ void psi_dtheta_k(double ell, double per, double rho, double& psi, double (&dps)[2]) {
  constexpr double third = 1.0 / 3.0;
  const double il = 1.0 / ell;
  dps[1] = 0.0;
  if constexpr (KIND == 4) {  // Periodic: exp(−2 sin²(πρ/p)/ℓ²)
    const double ip = 1.0 / per;
    const double u = 3.141592653589793 * rho * ip, su = sin(u), il2 = il * il;
    psi = exp(-2.0 * su * su * il2);
    dps[0] = psi * 4.0 * su * su * il2 * il;                                    // ∂/∂ℓ
    dps[1] = psi * 2.0 * u * il2 * sin(2.0 * u) * ip;                           // ∂/∂p = ψ·2πρ sin(2u)/(ℓ²p²)
  } else if constexpr (KIND == 3) {  // SE: exp(−ρ²/(2ℓ²))
    const double t = rho * rho * (il * il);
    psi = exp(-0.5 * t);
    dps[0] = psi * t * il;
  } else {
    const double c = (KIND == 0) ? sqrt(5.0) * il : (KIND == 1) ? sqrt(3.0) * il : il;
    const double s = c * rho, e = exp(-s);
    if constexpr (KIND == 0) {          // (1+s+s²/3)e⁻ˢ ; ∂/∂ℓ = (s²/3)(1+s)e⁻ˢ/ℓ
      psi = (1.0 + s * (1.0 + s * third)) * e;
      dps[0] = (s * s * third) * (1.0 + s) * e * il;
    } else if constexpr (KIND == 1) {   // (1+s)e⁻ˢ ; ∂/∂ℓ = s²e⁻ˢ/ℓ
      psi = (1.0 + s) * e;
      dps[0] = s * s * e * il;
    } else {                            // e⁻ˢ ; ∂/∂ℓ = s e⁻ˢ/ℓ
      psi = e;
      dps[0] = s * e * il;
    }
  }
}
__device__ __forceinline__ void psi_dtheta(int kind, double ell, double per, double rho, double& psi,
                                           double (&dps)[2]) {
  switch (kind) {
    case 0: psi_dtheta_k<0>(ell, per, rho, psi, dps); break;
    case 1: psi_dtheta_k<1>(ell, per, rho, psi, dps); break;
    case 2: psi_dtheta_k<2>(ell, per, rho, psi, dps); break;
    case 3: psi_dtheta_k<3>(ell, per, rho, psi, dps); break;
    default: psi_dtheta_k<4>(ell, per, rho, psi, dps); break;
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

// candidate p's hyperparameters: θ_p = thetas[p·nt .. p·nt + nt − 1] = (ℓ[, p]); with nt = 1 the
// Periodic kernel keeps the surrogate's period
__device__ __forceinline__ void cand_theta(const GpFitParams& q, int p, double& ell, double& per) {
  ell = q.thetas[(size_t)p * q.nt];
  per = (q.nt > 1) ? q.thetas[(size_t)p * q.nt + 1] : q.period;
}

// ---- N ≤ 64: one wave per candidate, K rows in registers --------------------------------
constexpr int GR_LD = 65;   // LDS leading dimension (odd: row and column walks conflict free)

__device__ __forceinline__ double gr_sum(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ void gr_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// Ordering of one wave's own LDS accesses: the LDS executes a wave's operations in issue order, so
// a store followed by a load of the same address needs no wait -- only the compiler must not move
// accesses across this point (no instruction is emitted)
__device__ __forceinline__ void lds_order() {
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

// a[j/16][j%16] += L[j][k]·m for j = k+1..63: the column (lane j holds L[j][k]) broadcast block by
// block (replicated by permlane swaps, DPP row_newbcast inside the fused FMAs, gpfit_asm.h)
template <int K>
__device__ __forceinline__ void gr_rank1(double (&a)[4][16], double col, double m) {
  constexpr int J0 = K + 1, B0 = J0 / 16, N0 = J0 % 16;
  if constexpr (J0 < 64) {
    double b0, b2, b1, b3;
    if constexpr (B0 <= 2) row_blocks<0>(col, b0, b2);
    if constexpr (B0 <= 3) row_blocks<1>(col, b1, b3);
    if constexpr (B0 == 0) RankAsm<N0>::run(a[0], b0, m);
    if constexpr (B0 <= 1) RankAsm<(B0 == 1) ? N0 : 0>::run(a[1], b1, m);
    if constexpr (B0 <= 2) RankAsm<(B0 == 2) ? N0 : 0>::run(a[2], b2, m);
    RankAsm<(B0 == 3) ? N0 : 0>::run(a[3], b3, m);
  }
}

// Steps k ≥ N run too (straight-line code the scheduler can overlap across steps): the padding
// rows are identity rows, so their pivots are 1 and their columns zero -- no change to rows < N.
// Look-ahead: lane K+1 forms the next pivot a[K+1][K+1] − L[K+1][K]² itself (the same fused
// multiply-add the broadcast update applies to that entry), so step K+1's pivot chain (readlane,
// rsq, Newton steps) does not wait for step K's trailing update.
template <int K>
__device__ __forceinline__ bool gr_chol_step(double (&a)[4][16], double& dg, double& piv, int lane) {
  double& akk = a[K / 16][K % 16];
  const bool ok = piv > 0.0;   // PosDefException; NaNs propagate harmlessly until the end
  double lkk, ilkk;
  sqrt_rsqrt(piv, lkk, ilkk);   // √piv and 1/√piv: no IEEE sqrt + division in the step's chain
  const double col = (lane > K) ? akk * ilkk : akk;
  akk = (lane == K) ? lkk : col;
  dg = (lane == K) ? lkk : dg;
  if constexpr (K + 1 < 64) piv = readlane_d(fma(col, -col, a[(K + 1) / 16][(K + 1) % 16]), K + 1);
  gr_rank1<K>(a, col, (lane > K) ? -col : 0.0);
  return ok;
}

template <int... K>
__device__ __forceinline__ bool gr_chol(double (&a)[4][16], double& dg, int lane, std::integer_sequence<int, K...>) {
  bool ok = true;
  double piv = readlane_d(a[0][0], 0);
  ((ok = gr_chol_step<K>(a, dg, piv, lane) && ok), ...);
  return ok;
}

// The same register Cholesky for one 32 × 32 diagonal tile of gpfit_tile_kernel: lane i holds row
// i & 31 in a[2][16] (lanes 32-63 duplicate lanes 0-31: they consume broadcasts, produce none),
// the pivot column broadcast by DPP inside the fused FMAs, the next pivot formed ahead by its own
// lane.  Every operation is the one the LDS-broadcast formulation applied (a_ij + l_jc·(−l_ic) by
// one fused multiply-add), so the factor is bit-identical to it.  rl = 1/L_ii of this lane's row.
template <int K>
__device__ __forceinline__ void tt_rank1(double (&a)[2][16], double col, double m) {
  constexpr int J0 = K + 1, B0 = J0 / 16, N0 = J0 % 16;
  if constexpr (J0 < 32) {
    double b0, b2, b1, b3;
    if constexpr (B0 == 0) {
      row_blocks<0>(col, b0, b2);
      RankAsm<N0>::run(a[0], b0, m);
    }
    row_blocks<1>(col, b1, b3);
    RankAsm<(B0 == 1) ? N0 : 0>::run(a[1], b1, m);
  }
}
template <int K>
__device__ __forceinline__ bool tt_chol_step(double (&a)[2][16], double& rl, double& piv, int i) {
  double& akk = a[K / 16][K % 16];
  const bool ok = piv > 0.0;   // PosDefException; NaNs propagate harmlessly until the end
  double lkk, ilkk;
  sqrt_rsqrt(piv, lkk, ilkk);
  const double col = (i > K) ? akk * ilkk : akk;
  akk = (i == K) ? lkk : col;
  rl = (i == K) ? ilkk : rl;
  if constexpr (K + 1 < 32) piv = readlane_d(fma(col, -col, a[(K + 1) / 16][(K + 1) % 16]), K + 1);
  tt_rank1<K>(a, col, (i > K) ? -col : 0.0);
  return ok;
}
// Forward substitution in a factored diagonal tile, rows in registers (lane i: a = row i of L_kk,
// rl = 1/L_ii): the solved entry z_M broadcast by readlane, eliminated from the rows below.
template <int M>
__device__ __forceinline__ void tt_fwd_step(double& r, const double (&a)[2][16], double rl, int i) {
  const double zm = readlane_d(r, M) * readlane_d(rl, M);
  r = (i == M) ? zm : ((i > M) ? fma(-a[M / 16][M % 16], zm, r) : r);
}
template <int... M>
__device__ __forceinline__ void tt_fwd(double& r, const double (&a)[2][16], double rl, int i,
                                       std::integer_sequence<int, M...>) {
  (tt_fwd_step<M>(r, a, rl, i), ...);
}
template <int... K>
__device__ __forceinline__ bool tt_chol(double (&a)[2][16], double& rl, int i, std::integer_sequence<int, K...>) {
  bool ok = true;
  double piv = readlane_d(a[0][0], 0);
  ((ok = tt_chol_step<K>(a, rl, piv, i) && ok), ...);
  return ok;
}

// c = L'\(L\y), column-oriented substitutions with ck broadcast by readlane: forward step K uses
// this lane's L[i][K] (register), backward step K its L[K][i] (LDS, row K of L)
template <int K>
__device__ __forceinline__ void gr_fwd(double& c, const double (&a)[4][16], double rdg, int lane, int N) {
  const double ck = readlane_d(c, K) * readlane_d(rdg, K);
  c = (lane == K) ? ck : ((lane > K) ? c - a[K / 16][K % 16] * ck : c);
}
template <int K>
__device__ __forceinline__ void gr_bwd(double& c, const double* LV, double rdg, int lane, int N) {
  const double ck = readlane_d(c, K) * readlane_d(rdg, K);
  const double lki = LV[K * GR_LD + lane];
  c = (lane == K) ? ck : ((lane < K) ? c - lki * ck : c);
}
template <int... K>
__device__ __forceinline__ void gr_solve(double& c, const double (&a)[4][16], const double* LV, double rdg, int lane,
                                         int N, std::integer_sequence<int, K...>) {
  (gr_fwd<K>(c, a, rdg, lane, N), ...);
  (gr_bwd<63 - K>(c, LV, rdg, lane, N), ...);
}

// row R of V = L⁻¹ by columns (lane j = column j): v[R] = (δ_Rj − Σ_{m<R} L[R][m] v[m]) / L[R][R].
// lr = L[R][lane] (row R of L, read by lanes) is replicated block by block; lane j's sum over m
// broadcasts L[R][m] from lane m (DPP row_newbcast in the fused FMAs, two chains).
template <int R>
__device__ __forceinline__ void gr_inv_row(double (&v)[64], const double* LV, double rdg, int lane, int N) {
  const double lr = LV[R * GR_LD + lane];
  double acc0 = (lane == R) ? 1.0 : 0.0, acc1 = 0.0;
  constexpr int NB = (R + 15) / 16;   // blocks of m < R
  if constexpr (NB > 0) {
    double b0, b1, b2, b3;
    row_blocks<0>(lr, b0, b2);
    if constexpr (NB > 1) row_blocks<1>(lr, b1, b3);
    double t0 = 0.0, t1 = 0.0;   // −Σ: accumulate the products, subtract once per row
    DotAsm<(R < 16 ? R : 16)>::run(t0, t1, b0, &v[0]);
    if constexpr (NB > 1) DotAsm<(R - 16 < 16 ? R - 16 : 16)>::run(t0, t1, b1, &v[16]);
    if constexpr (NB > 2) DotAsm<(R - 32 < 16 ? R - 32 : 16)>::run(t0, t1, b2, &v[32]);
    if constexpr (NB > 3) DotAsm<R - 48>::run(t0, t1, b3, &v[48]);
    acc0 -= t0 + t1;
  }
  v[R] = (acc0 + acc1) * readlane_d(rdg, R);
}
template <int... R>
__device__ __forceinline__ void gr_inv(double (&v)[64], const double* LV, double rdg, int lane, int N,
                                       std::integer_sequence<int, R...>) {
  (gr_inv_row<R>(v, LV, rdg, lane, N), ...);
}

// K⁻¹ = VᵀV by columns: lane i accumulates K⁻¹[i][b] = Σ_m V[m][i]·V[m][b] for the 16 columns b of
// block P + 2·HI, broadcasting lane b's V[m][b] (its v[m]) with DPP (RankAsm)
template <int P, int HI, int... M>
__device__ __forceinline__ void gr_kinv_block(const double (&v)[64], double (&kb)[16], std::integer_sequence<int, M...>) {
  auto step = [&](double vm) {
    double r0, r2;
    row_blocks<P>(vm, r0, r2);
    RankAsm<0>::run(kb, HI ? r2 : r0, vm);
  };
  (step(v[M]), ...);
}

// -DMRBO_GPFIT_STAMPS: cycles per phase of candidate 0 (one printf at the end): X staging, K rows,
// Cholesky, c, L⁻¹, K⁻¹·δK traces
#ifdef MRBO_GPFIT_STAMPS
#define GR_STAMP(id) do { gr_ts[id] = __builtin_amdgcn_s_memtime(); } while (0)
#else
#define GR_STAMP(id) ((void)0)
#endif

// GR_WAVES waves per candidate: all of them evaluate the K / δK pairs (one per SIMD), then wave 0
// alone runs the register phases (no workgroup barrier after the pairs)
constexpr int GR_WAVES = 4;

template <int NT>
__global__ void __launch_bounds__(64 * GR_WAVES) gpfit_reg_kernel(GpFitParams q, int P) {
  extern __shared__ __attribute__((aligned(16))) double gsm[];
  const int p = blockIdx.x, lane = threadIdx.x & 63, tid = threadIdx.x;
  if (p >= P) return;   // whole workgroups
#ifdef MRBO_GPFIT_STAMPS
  unsigned long long gr_ts[6], gr_t0 = __builtin_amdgcn_s_memtime();
#endif
  double* LV = gsm;                     // K, then L, row-major (i·LD + j)
  double* DK = LV + 64 * GR_LD;         // δK_t (symmetric) at t·64·LD + i·LD + j
  double* cs = DK + NT * 64 * GR_LD;    // c
  double* XS = cs + 64;                 // X[u][j] at u·64 + j (u < d)
  double* VS = XS + 16 * 64;            // V = L⁻¹, row-major (m·LD + j)
  const int N = q.N, d = q.d;
  const bool act = lane < N;
  double ell, per;
  cand_theta(q, p, ell, per);
  if (tid < 64)
    for (int u = 0; u < d; ++u) XS[u * 64 + lane] = act ? q.X[u + d * lane] : 0.0;
  __syncthreads();
  GR_STAMP(0);
  // K (eval_KXX :161-178, ψ(0) + σn2 on the diagonal; padding = identity) and δK_t (eval_Dθ_KXX
  // :264-284) over the 2080 pairs j ≤ i of the lower triangle, lanes over pairs, both halves written
  // (two pairs per thread and pass as independent chains: one wave per SIMD, nothing else hides
  // the LDS and transcendental latencies)
  constexpr int NPAIR = 64 * 65 / 2;
  // (the kernel kind dispatched once around the pass: the two chains interleave)
  auto kpairs = [&](auto kind_c) {
  constexpr int KIND = decltype(kind_c)::value;
  for (int q0 = 0; q0 < NPAIR; q0 += 2 * 64 * GR_WAVES) {
    int ii[2], jj[2];
    double r2[2] = {0.0, 0.0};
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int qq = min(q0 + 64 * GR_WAVES * e + tid, NPAIR - 1);
      int i = (int)((sqrt(8.0 * qq + 1.0) - 1.0) * 0.5);
      i += ((i + 1) * (i + 2) / 2 <= qq) ? 1 : 0;   // exact row of the triangle index
      i -= (i * (i + 1) / 2 > qq) ? 1 : 0;
      ii[e] = i;
      jj[e] = qq - i * (i + 1) / 2;
    }
#pragma unroll
    for (int u = 0; u < 16; ++u)
      if (u < d) {
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const double r = XS[u * 64 + ii[e]] - XS[u * 64 + jj[e]];
          r2[e] = fma(r, r, r2[e]);
        }
      }
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int i = ii[e], j = jj[e];
      double psi, dps[2];
      psi_dtheta_k<KIND>(ell, per, (i == j) ? 0.0 : sqrt(r2[e]), psi, dps);
      if (q0 + 64 * GR_WAVES * e + tid < NPAIR) {
        const bool v = i < N;   // j ≤ i
        const double kij = v ? ((i == j) ? psi + q.sn2 : psi) : ((i == j) ? 1.0 : 0.0);
        LV[i * GR_LD + j] = kij;
        LV[j * GR_LD + i] = kij;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const double dk = (v && i != j) ? dps[t] : 0.0;
          DK[t * 64 * GR_LD + i * GR_LD + j] = dk;
          DK[t * 64 * GR_LD + j * GR_LD + i] = dk;
        }
      }
    }
  }
  };
  switch (q.kernel) {
    case 0: kpairs(std::integral_constant<int, 0>{}); break;
    case 1: kpairs(std::integral_constant<int, 1>{}); break;
    case 2: kpairs(std::integral_constant<int, 2>{}); break;
    case 3: kpairs(std::integral_constant<int, 3>{}); break;
    default: kpairs(std::integral_constant<int, 4>{}); break;
  }
  __syncthreads();
  GR_STAMP(1);
  // wave 0: the Cholesky in registers; then wave 0 solves for c while wave 1 forms V = L⁻¹
  __shared__ double part[GR_WAVES][2 * NT + 2];   // per-wave partial sums; [0][2NT..] = yc, log det
  __shared__ int failed;
  const int w = tid >> 6;
  double a[4][16];
  double dg = 1.0;
  if (w == 0) {
#pragma unroll
    for (int j = 0; j < 64; ++j) a[j / 16][j % 16] = LV[lane * GR_LD + j];
    // right-looking Cholesky in registers (PosDefException → status 1); dg = L_ii of this row
    const bool chol_ok = gr_chol(a, dg, lane, std::make_integer_sequence<int, 64>{});
    GR_STAMP(2);
    gr_sync();
#pragma unroll
    for (int j = 0; j < 64; ++j) LV[lane * GR_LD + j] = a[j / 16][j % 16];
    const double ld = gr_sum(act ? log(dg) : 0.0);
    if (lane == 0) {
      failed = !chol_ok;
      part[0][2 * NT + 1] = ld;
    }
  }
  __syncthreads();
  if (w == 0) {
    // c = L'\(L\y), column-oriented substitutions (ck broadcast by readlane)
    const double rdg = 1.0 / dg;
    double c = act ? q.y[lane] : 0.0;
    gr_solve(c, a, LV, rdg, lane, N, std::make_integer_sequence<int, 64>{});
    GR_STAMP(3);
    cs[lane] = c;
    const double yc = gr_sum(act ? q.y[lane] * c : 0.0);
    if (lane == 0) part[0][2 * NT] = yc;
  } else if (w == 1) {
    // V = L⁻¹ by columns (lane j = column j), rows ascending (rows ≥ N: identity, no effect on
    // rows < N); 1/L_jj from the stored factor (the same division wave 0 makes)
    const double rdg = 1.0 / LV[lane * GR_LD + lane];
    double v[64];
#pragma unroll
    for (int r = 0; r < 64; ++r) v[r] = 0.0;
    gr_inv(v, LV, rdg, lane, N, std::make_integer_sequence<int, 64>{});
#pragma unroll
    for (int m = 0; m < 64; ++m) VS[m * GR_LD + lane] = v[m];   // V row-major for every wave
  }
  __syncthreads();
  GR_STAMP(4);
  if (failed) {
    if (tid == 0) {
      q.ll[p] = NAN;
      for (int t = 0; t < NT; ++t) q.grad[(size_t)p * NT + t] = NAN;
      q.status[p] = 1;
    }
    return;
  }
  // tr(K⁻¹δK_t) = Σ_ib K⁻¹_ib δK_t[i][b] and cᵀδK_t c = Σ_ib c_i δK_t[i][b] c_b (full sums; δK_ii = 0).
  // Wave w: K⁻¹ columns b of block w (K⁻¹ = VᵀV by DPP broadcasts of V[m][b]), lane i = row.
  double v[64];
#pragma unroll
  for (int m = 0; m < 64; ++m) v[m] = VS[m * GR_LD + lane];
  const double c = cs[lane];
  double kb[16];
#pragma unroll
  for (int n = 0; n < 16; ++n) kb[n] = 0.0;
  if (w == 0) gr_kinv_block<0, 0>(v, kb, std::make_integer_sequence<int, 64>{});
  else if (w == 1) gr_kinv_block<1, 0>(v, kb, std::make_integer_sequence<int, 64>{});
  else if (w == 2) gr_kinv_block<0, 1>(v, kb, std::make_integer_sequence<int, 64>{});
  else gr_kinv_block<1, 1>(v, kb, std::make_integer_sequence<int, 64>{});
  double tr[NT], cgc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) tr[t] = cgc[t] = 0.0;
#pragma unroll
  for (int n = 0; n < 16; ++n) {
    const int b = 16 * w + n;
    const double cb = cs[b];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const double dk = DK[t * 64 * GR_LD + b * GR_LD + lane];
      tr[t] = fma(kb[n], dk, tr[t]);
      cgc[t] = fma(c * cb, dk, cgc[t]);
    }
  }
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const double trs = gr_sum(act ? tr[t] : 0.0), cgs = gr_sum(act ? cgc[t] : 0.0);
    if (lane == 0) {
      part[w][t] = trs;
      part[w][NT + t] = cgs;
    }
  }
  GR_STAMP(5);
  __syncthreads();
  if (tid == 0) {
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const double trs = (part[0][t] + part[1][t]) + (part[2][t] + part[3][t]);
      const double cgs = (part[0][NT + t] + part[1][NT + t]) + (part[2][NT + t] + part[3][NT + t]);
      q.grad[(size_t)p * NT + t] = 0.5 * (cgs - trs);
    }
    q.ll[p] = -0.5 * part[0][2 * NT] - part[0][2 * NT + 1] - 0.5 * N * log(2.0 * 3.141592653589793);
    q.status[p] = 0;
  }
#ifdef MRBO_GPFIT_STAMPS
  if (p == 0 && tid == 0)
    printf("gpfit_reg cycles: X %llu  K rows %llu  chol %llu  c %llu  inv beyond c %llu  traces %llu\n", gr_ts[0] - gr_t0,
           gr_ts[1] - gr_ts[0], gr_ts[2] - gr_ts[1], gr_ts[3] - gr_ts[2], gr_ts[4] - gr_ts[3], gr_ts[5] - gr_ts[4]);
#endif
}

// ---- 64 < N ≤ 128 (dispatched up to 80): one workgroup per candidate, factor and inverse in LDS
// S (128 × 129 doubles, column-major r + LD·c, odd LD: row and column walks conflict free) holds
// K → L in its lower triangle and V = L⁻¹ transposed in its strict upper triangle (V[i][j], i > j,
// at j + LD·i); L's diagonal in ld_, V's (1/L_ii) in dv.  Four waves:
//   K pairs (all) → right-looking Cholesky, thread (row i, parity) updating S[i][j] for j ≡ parity
//   (one barrier per column, no global workspace) → V = L⁻¹ by columns (waves 0-1, lane = column)
//   beside c = L'\(L\y) by column-
//   oriented substitutions (wave 2, two rows per lane, readlane broadcasts) → tr(K⁻¹δK_t) and
//   cᵀδK_t c over the pairs j < i with K⁻¹_ij = Σ_{m ≥ i} V_mi V_mj (δK_ii = 0), δK on the fly.
// N³/3 + N³/6 + N³/6 FMAs instead of the workspace kernel's N³/3 + N³/2·nt + N³/6.
constexpr int GL_N = 128, GL_LD = 129, GL_THREADS = 256;

template <int NT>
__global__ void __launch_bounds__(GL_THREADS) gpfit_lds_kernel(GpFitParams q, int P) {
  extern __shared__ __attribute__((aligned(16))) double gsm[];
  double* S = gsm;                      // GL_N × GL_LD
  double* XS = S + GL_N * GL_LD;        // X[u][i] at u·GL_N + i (u < d ≤ 16)
  double* ld_ = XS + 16 * GL_N;         // L_ii
  double* dv = ld_ + GL_N;              // 1/L_ii
  double* cv = dv + GL_N;               // y, then c
  __shared__ double part[GL_THREADS / 64][2 * NT + 2];
  __shared__ int fail;
  const int p = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (p >= P) return;   // whole workgroups
#ifdef MRBO_GPFIT_STAMPS
  unsigned long long gl_ts[6], gl_t0 = __builtin_amdgcn_s_memtime();
#define GL_STAMP(k) gl_ts[k] = __builtin_amdgcn_s_memtime()
#else
#define GL_STAMP(k) ((void)0)
#endif
  const int N = q.N, d = q.d;
  double ell, per;
  cand_theta(q, p, ell, per);
  if (tid == 0) fail = 0;
  for (int idx = tid; idx < d * N; idx += GL_THREADS) {
    const int u = idx % d, i = idx / d;
    XS[u * GL_N + i] = q.X[idx];
  }
  for (int i = tid; i < N; i += GL_THREADS) cv[i] = q.y[i];
  __syncthreads();
  // K (eval_KXX :161-178, ψ(0) + σn2 on the diagonal) over the pairs j ≤ i, lower triangle
  const int npair = N * (N + 1) / 2;
  for (int qq = tid; qq < npair; qq += GL_THREADS) {
    int i = (int)((sqrt(8.0 * qq + 1.0) - 1.0) * 0.5);
    i += ((i + 1) * (i + 2) / 2 <= qq) ? 1 : 0;   // exact row of the triangle index
    i -= (i * (i + 1) / 2 > qq) ? 1 : 0;
    const int j = qq - i * (i + 1) / 2;
    double r2 = 0.0;
    for (int u = 0; u < d; ++u) { const double r = XS[u * GL_N + i] - XS[u * GL_N + j]; r2 = fma(r, r, r2); }
    double psi, dps[2];
    psi_dtheta(q.kernel, ell, per, (i == j) ? 0.0 : sqrt(r2), psi, dps);
    S[i + GL_LD * j] = (i == j) ? psi + q.sn2 : psi;
  }
  __syncthreads();
  GL_STAMP(0);
  // right-looking Cholesky (PosDefException → status 1), ONE barrier per column: column k is final
  // (unscaled) when step k starts, every thread scales the entries it reads by 1/L_kk itself, and
  // thread (row i, parity 0) writes its scaled L_ik one step later, when no thread reads column k
  // any more.  The pivot entry keeps K's value; L_kk goes to ld_.  Thread (row i, parity) updates
  // S[i][j] for j ≡ parity, in batches of 8 whose 16 loads issue before the FMAs and stores.
  {
    const int i = tid & (GL_N - 1), par = tid >> 7;
    double lprev = 0.0;
    for (int k = 0; k < N; ++k) {
      const double piv = S[k + GL_LD * k];
      if (!(piv > 0.0)) {   // every thread reads the same pivot: a uniform exit
        if (tid == 0) fail = 1;
        break;
      }
      double lkk, rl;
      sqrt_rsqrt(piv, lkk, rl);
      if (tid == 0) { ld_[k] = lkk; dv[k] = rl; }
      if (k > 0 && par == 0 && i > k - 1 && i < N) S[i + GL_LD * (k - 1)] = lprev;   // scaled L_i,k-1
      if (i > k && i < N) {
        const double lik = S[i + GL_LD * k] * rl;
        lprev = lik;
        for (int jb = k + 1 + par; jb <= i; jb += 16) {
          double lv[8], av[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const int j = min(jb + 2 * u, i);
            lv[u] = S[j + GL_LD * k];
            av[u] = S[i + GL_LD * j];
          }
#pragma unroll
          for (int u = 0; u < 8; ++u) av[u] = fma(-lik, lv[u] * rl, av[u]);
#pragma unroll
          for (int u = 0; u < 8; ++u)
            if (jb + 2 * u <= i) S[i + GL_LD * (jb + 2 * u)] = av[u];
        }
      }
      __syncthreads();
    }
  }
  __syncthreads();
  GL_STAMP(1);
  if (fail) {
    if (tid == 0) {
      q.ll[p] = NAN;
      for (int t = 0; t < NT; ++t) q.grad[(size_t)p * NT + t] = NAN;
      q.status[p] = 1;
    }
    return;
  }
  if (w < 2) {
    // V = L⁻¹, column j = tid: V_jj = 1/L_jj, V_ij = −(Σ_{k=j}^{i−1} L_ik V_kj)/L_ii, rows ascending.
    // Lane j runs its own k range j..i−1 (no masks: L_ik is read at per-lane addresses), in
    // batches of 8 whose 16 loads issue before the FMAs; k = j contributes L_ij/L_jj.
    const int j = tid;
    const double djj = dv[j];
    for (int i = 64 * w + 1; i < N; ++i) {
      if (i <= j) continue;
      double sc[4] = {S[i + GL_LD * j] * djj, 0.0, 0.0, 0.0};
      int k = j + 1;
      for (; k + 8 <= i; k += 8) {
        double lv[8], vv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          lv[u] = S[i + GL_LD * (k + u)];
          vv[u] = S[j + GL_LD * (k + u)];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) sc[u & 3] = fma(lv[u], vv[u], sc[u & 3]);
      }
      for (; k < i; ++k) sc[0] = fma(S[i + GL_LD * k], S[j + GL_LD * k], sc[0]);
      if (j < N) S[j + GL_LD * i] = -((sc[0] + sc[1]) + (sc[2] + sc[3])) * dv[i];
    }
    GL_STAMP(2);
  } else if (w == 2) {
    // c = L'\(L\y): column-oriented substitutions, rows lane and lane + 64 in registers, the
    // solved entry broadcast by readlane
    double r[2];
    r[0] = (lane < N) ? cv[lane] : 0.0;
    r[1] = (lane + 64 < N) ? cv[lane + 64] : 0.0;
    for (int k = 0; k < N; ++k) {
      const double zk = readlane_d(r[k >> 6], k & 63) * dv[k];
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const int i = lane + 64 * s2;
        if (i == k) r[s2] = zk;
        else if (i > k && i < N) r[s2] = fma(-S[i + GL_LD * k], zk, r[s2]);
      }
    }
    for (int k = N - 1; k >= 0; --k) {
      const double ck = readlane_d(r[k >> 6], k & 63) * dv[k];
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const int i = lane + 64 * s2;
        if (i == k) r[s2] = ck;
        else if (i < k) r[s2] = fma(-S[k + GL_LD * i], ck, r[s2]);
      }
    }
    double yc = 0.0, lg = 0.0;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const int i = lane + 64 * s2;
      if (i < N) {
        yc = fma(q.y[i], r[s2], yc);
        lg += log(ld_[i]);
      }
    }
    if (lane < N) cv[lane] = r[0];
    if (lane + 64 < N) cv[lane + 64] = r[1];
    yc = gr_sum(yc);
    lg = gr_sum(lg);
    if (lane == 0) { part[0][2 * NT] = yc; part[0][2 * NT + 1] = lg; }
    GL_STAMP(3);
  }
  __syncthreads();
  GL_STAMP(4);
  // traces over the pairs j < i: wave w takes rows i ≡ w (mod 4), lanes over j in chunks of 64
  double tr[NT], cgc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) tr[t] = cgc[t] = 0.0;
  for (int i = 1 + w; i < N; i += GL_THREADS / 64) {
    const double ci = cv[i];
    for (int jb = 0; jb < i; jb += 64) {
      const int j = jb + lane;
      if (j >= i) break;
      // K⁻¹_ij = V_ii V_ij + Σ_{m > i} V_mi V_mj
      double kc[4] = {dv[i] * S[j + GL_LD * i], 0.0, 0.0, 0.0};
      for (int mb = i + 1; mb < N; mb += 8) {
        double av[8], bv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int m = min(mb + u, N - 1);
          double x = S[i + GL_LD * m];
          bv[u] = S[j + GL_LD * m];
          asm volatile("" : "+v"(x), "+v"(bv[u]));
          av[u] = (mb + u < N) ? x : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) kc[u & 3] = fma(av[u], bv[u], kc[u & 3]);
      }
      const double kij = (kc[0] + kc[1]) + (kc[2] + kc[3]);
      double r2 = 0.0;
      for (int u = 0; u < d; ++u) { const double r = XS[u * GL_N + i] - XS[u * GL_N + j]; r2 = fma(r, r, r2); }
      double psi, dps[2];
      psi_dtheta(q.kernel, ell, per, sqrt(r2), psi, dps);
      const double cc = ci * cv[j];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        tr[t] = fma(kij, dps[t], tr[t]);
        cgc[t] = fma(cc, dps[t], cgc[t]);
      }
    }
  }
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const double trs = gr_sum(tr[t]), cgs = gr_sum(cgc[t]);
    if (lane == 0) { part[w][t] = trs; part[w][NT + t] = cgs; }
  }
  __syncthreads();
  if (tid == 0) {
#pragma unroll
    for (int t = 0; t < NT; ++t) {   // both triangles: 2·Σ_{j<i}
      const double trs = (part[0][t] + part[1][t]) + (part[2][t] + part[3][t]);
      const double cgs = (part[0][NT + t] + part[1][NT + t]) + (part[2][NT + t] + part[3][NT + t]);
      q.grad[(size_t)p * NT + t] = cgs - trs;
    }
    q.ll[p] = -0.5 * part[0][2 * NT] - part[0][2 * NT + 1] - 0.5 * N * log(2.0 * 3.141592653589793);
    q.status[p] = 0;
  }
  GL_STAMP(5);
#ifdef MRBO_GPFIT_STAMPS
  if (p == 0 && (tid == 0 || tid == 128))
    printf("gpfit_lds cycles (thread %d): K %llu  chol %llu  V %llu  c %llu  wait %llu  traces %llu\n", tid,
           gl_ts[0] - gl_t0, gl_ts[1] - gl_ts[0], gl_ts[2] - gl_ts[1], gl_ts[3] - gl_ts[1], gl_ts[4] - gl_ts[1],
           gl_ts[5] - gl_ts[4]);
#endif
#undef GL_STAMP
  if (q.L_out) {
    double* Lo = q.L_out + (size_t)N * N * p;
    for (int idx = tid; idx < N * N; idx += GL_THREADS) {
      const int i = idx % N, j = idx / N;
      Lo[idx] = (i > j) ? S[i + GL_LD * j] : ((i == j) ? ld_[i] : 0.0);
    }
  }
  if (q.c_out)
    for (int i = tid; i < N; i += GL_THREADS) q.c_out[(size_t)N * p + i] = cv[i];
}

// ---- 128 < N ≤ 512: blocked on 32 × 32 tiles, the products on the fp64 matrix cores ----------
// One workgroup (four waves) per candidate.  Global workspace per candidate (tile_work_doubles):
// the lower tiles of K → L (column-major), of V = L⁻¹ (row-major) and the diagonal-tile inverses
// W_k = L_kk⁻¹ (column-major), then the lower tiles of δK_t = ∂K/∂θ_t (the K pass evaluates ψ and
// ∂ψ/∂θ together; the traces read them back instead of evaluating the radial function again);
// T = ⌈N/32⌉, rows and columns past N are identity rows of K (their L, V and K⁻¹ rows are identity
// rows too, and they take no part in the sums).
//   Cholesky, right-looking by tile columns k: wave 0 factors A_kk and inverts L_kk in LDS; the
//   panel L_Ik = A_Ik·L_kk⁻ᵀ by substitution (one row per lane); the trailing updates
//   A_IJ −= L_Ik·L_Jkᵀ are 32³ products spread over the four waves, each 32 v_mfma_f64_16x16x4
//   (tile_xyt: C += X·Yᵀ with X and Y read as column-major tiles -- both fragment loads coalesced).
//   V = L⁻¹ by tile rows I: V_IJ = −W_I·Σ_{J≤M<I} L_IM V_MJ.  V is stored row-major, i.e. as the
//   column-major Vᵀ the later products read.
//   c = L'\(L\y) by blocked substitution, and K⁻¹_IJ = Σ_{M≥I} V_MIᵀ V_MJ for I ≥ J, whose tile the
//   wave holds in registers while it adds K⁻¹_ij·δK_t,ij and c_i c_j·δK_t,ij over the strictly
//   lower entries (δK stored by the K pass; δK_ii = 0), as the LDS kernel above does.
// ≈ N³/2 multiply-adds (N³/6 each for L, V and K⁻¹), all but the diagonal tiles' on the MFMA pipe.
constexpr int TT = 32, TT_THREADS = 256, TT_LD = 33;
typedef double f64x4 __attribute__((ext_vector_type(4)));

// c[bi][bj][j] holds tile entry (16·bi + (lane >> 4) + 4·j, 16·bj + (lane & 15)) (the f64 MFMA's
// accumulator map)
__device__ __forceinline__ void tile_zero(f64x4 (&c)[2][2]) {
#pragma unroll
  for (int bi = 0; bi < 2; ++bi)
#pragma unroll
    for (int bj = 0; bj < 2; ++bj) c[bi][bj] = f64x4{0.0, 0.0, 0.0, 0.0};
}
template <bool ROWMAJOR>
__device__ __forceinline__ void tile_load(f64x4 (&c)[2][2], const double* t, int lane) {
#pragma unroll
  for (int bi = 0; bi < 2; ++bi)
#pragma unroll
    for (int bj = 0; bj < 2; ++bj)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = 16 * bi + (lane >> 4) + 4 * j, col = 16 * bj + (lane & 15);
        c[bi][bj][j] = ROWMAJOR ? t[row * TT + col] : t[col * TT + row];
      }
}
template <bool ROWMAJOR>
__device__ __forceinline__ void tile_store(const f64x4 (&c)[2][2], double* t, int lane) {
#pragma unroll
  for (int bi = 0; bi < 2; ++bi)
#pragma unroll
    for (int bj = 0; bj < 2; ++bj)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = 16 * bi + (lane >> 4) + 4 * j, col = 16 * bj + (lane & 15);
        if (ROWMAJOR) t[row * TT + col] = c[bi][bj][j];
        else t[col * TT + row] = c[bi][bj][j];
      }
}
// c += ±X·Yᵀ, X and Y 32 × 32 column-major (X's A-fragment: X[r][k] at k·32 + r; Yᵀ's
// B-fragment: Y[n][k] at k·32 + n -- sixteen consecutive doubles per lane group)
template <bool NEG>
__device__ __forceinline__ void tile_xyt(f64x4 (&c)[2][2], const double* X, const double* Y, int lane) {
  const int r = lane & 15, kk = lane >> 4;
#pragma unroll
  for (int k0 = 0; k0 < TT; k0 += 4) {
    double a0 = X[(k0 + kk) * TT + r], a1 = X[(k0 + kk) * TT + 16 + r];
    const double b0 = Y[(k0 + kk) * TT + r], b1 = Y[(k0 + kk) * TT + 16 + r];
    if (NEG) {
      a0 = -a0;
      a1 = -a1;
    }
    c[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, c[0][0], 0, 0, 0);
    c[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, c[0][1], 0, 0, 0);
    c[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, c[1][0], 0, 0, 0);
    c[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, c[1][1], 0, 0, 0);
  }
}
__device__ __forceinline__ size_t tile_at(int I, int J) { return (size_t)(I * (I + 1) / 2 + J) * (TT * TT); }
// The operands of one tile_xyt in registers (the A- and B-fragments of its eight k-steps), so
// that a loop over tiles can load tile n + 1's operands while tile n's products run
struct TileFrag {
  double a[TT / 4][2], b[TT / 4][2];
};
__device__ __forceinline__ void frag_load(TileFrag& f, const double* X, const double* Y, int lane) {
  const int r = lane & 15, kk = lane >> 4;
#pragma unroll
  for (int s = 0; s < TT / 4; ++s) {
    f.a[s][0] = X[(4 * s + kk) * TT + r];
    f.a[s][1] = X[(4 * s + kk) * TT + 16 + r];
    f.b[s][0] = Y[(4 * s + kk) * TT + r];
    f.b[s][1] = Y[(4 * s + kk) * TT + 16 + r];
  }
}
// c −= X·Yᵀ from the fragments (tile_xyt<true>'s products, in its order)
__device__ __forceinline__ void frag_sub(f64x4 (&c)[2][2], const TileFrag& f) {
#pragma unroll
  for (int s = 0; s < TT / 4; ++s) {
    const double a0 = -f.a[s][0], a1 = -f.a[s][1];
    c[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, f.b[s][0], c[0][0], 0, 0, 0);
    c[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, f.b[s][1], c[0][1], 0, 0, 0);
    c[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, f.b[s][0], c[1][0], 0, 0, 0);
    c[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, f.b[s][1], c[1][1], 0, 0, 0);
  }
}

// lower-triangle index q = I(I+1)/2 + J → (I, J)
__device__ __forceinline__ void tile_ij(int q, int& I, int& J) {
  I = (int)((sqrt(8.0 * q + 1.0) - 1.0) * 0.5);
  I += ((I + 1) * (I + 2) / 2 <= q) ? 1 : 0;
  I -= (I * (I + 1) / 2 > q) ? 1 : 0;
  J = q - I * (I + 1) / 2;
}

// Triangular substitution step of the tile kernel with the L row broadcast by DPP (the
// gpfit_reg_kernel idiom): v[R] = (init − Σ_{m<R} L[R][m]·v[m]) · rdR, where lane m holds
// lr = L[R][m] (read from the column-major diagonal tile) and v is this lane's vector in
// registers -- W_k by columns (lane j: v = column j of L_kk⁻¹, init = δ_Rj) and the panel by rows
// (lane r: v = row r of L_Ik, init = A_Ik[r][R]).  Two FMA chains per step, no LDS access inside
// the sums; lanes 32-63 receive the same broadcasts as lanes 0-31.
template <int R>
__device__ __forceinline__ void tt_subst_step(double (&v)[TT], double init, double lr, double rdR) {
  double t0 = 0.0, t1 = 0.0;
  if constexpr (R > 0) {
    double b0, b2;
    row_blocks<0>(lr, b0, b2);
    DotAsm<(R < 16 ? R : 16)>::run(t0, t1, b0, &v[0]);
    if constexpr (R > 16) {
      double b1, b3;
      row_blocks<1>(lr, b1, b3);
      DotAsm<R - 16>::run(t0, t1, b1, &v[16]);
    }
  }
  v[R] = (init - (t0 + t1)) * rdR;
}
template <int... R>
__device__ __forceinline__ void tt_inverse(double (&v)[TT], const double* Dk, const double* rd, int i,
                                           std::integer_sequence<int, R...>) {
  ((tt_subst_step<R>(v, (i == R) ? 1.0 : 0.0, Dk[i * TT_LD + R], rd[R])), ...);
}
template <int... R>
__device__ __forceinline__ void tt_panel(double (&v)[TT], const double* Dk, const double* rd, int i,
                                         std::integer_sequence<int, R...>) {
  ((tt_subst_step<R>(v, v[R], Dk[i * TT_LD + R], rd[R])), ...);
}

// -DMRBO_GPFIT_STAMPS: cycles per phase of candidate 0 (thread 0, after each workgroup barrier):
// K, then per tile column the diagonal factor + inverse, the panel, the trailing update (summed
// over k), V by tile rows, c, K⁻¹ + traces
#ifdef MRBO_GPFIT_STAMPS
#define TT_STAMP(k)                                                   \
  do {                                                                \
    const unsigned long long now_ = __builtin_amdgcn_s_memtime();     \
    tt_acc[k] += now_ - tt_last;                                      \
    tt_last = now_;                                                   \
  } while (0)
#else
#define TT_STAMP(k) ((void)0)
#endif

template <int NT>
__global__ void __launch_bounds__(TT_THREADS) gpfit_tile_kernel(GpFitParams q, int P) {
  extern __shared__ __attribute__((aligned(16))) double tsm[];
  const int p = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (p >= P) return;   // whole workgroups
#ifdef MRBO_GPFIT_STAMPS
  unsigned long long tt_acc[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, tt_last = __builtin_amdgcn_s_memtime();
#endif
  const int N = q.N, d = q.d, T = (N + TT - 1) / TT, NP = T * TT;
  double* XS = tsm;                      // X[u][i] at u·NP + i, zero-padded
  double* Dk = XS + (size_t)d * NP;      // diagonal tile A_kk → L_kk, 32 × 33 column-major
  double* Wk = Dk + TT * TT_LD;          // W_k = L_kk⁻¹, 32 × 33 column-major
  double* rd = Wk + TT * TT_LD;          // 1/L_ii of the tile
  double* Sw = rd + TT;                  // per-wave 32 × 32 scratch (row-major S)
  double* yv = Sw + 4 * TT * TT;         // y, then c
  double* uv = yv + NP;                  // z = L⁻¹y
  double* rdall = uv + NP;               // 1/L_ii of every row (the substitutions multiply)
  __shared__ double part[TT_THREADS / 64][2 * NT + 2];
  __shared__ int fail;
  double ell, per;
  cand_theta(q, p, ell, per);
  const size_t ntile = (size_t)T * (T + 1) / 2;
  double* Lt = q.work + (size_t)p * ((2 + NT) * ntile + T) * (TT * TT);
  double* Vt = Lt + ntile * (TT * TT);
  double* Wt = Vt + ntile * (TT * TT);
  double* Dt = Wt + (size_t)T * (TT * TT);   // δK_t = ∂K/∂θ_t in the tile layout of Lt, kept for the traces
  if (tid == 0) fail = 0;
  for (int idx = tid; idx < d * NP; idx += TT_THREADS) {
    const int u = idx / NP, i = idx % NP;
    XS[idx] = (i < N) ? q.X[u + (size_t)d * i] : 0.0;
  }
  for (int i = tid; i < NP; i += TT_THREADS) yv[i] = (i < N) ? q.y[i] : 0.0;
  __syncthreads();
  // K (eval_KXX :161-178, ψ(0) + σn2 on the diagonal), every entry of the lower tiles
  // (tile by tile: the tile's (I, J) once per tile instead of a square root per entry; the
  // diagonal tiles' strict upper triangles are never read -- the factor, the copy-out and the
  // traces take the lower part -- so they are zero-filled without a radial evaluation)
  // Each thread takes TT²/TT_THREADS = 4 entries of a tile -- one row gi, columns gj + 8m --
  // as four independent chains (one wave per SIMD: the chains' interleaving is the latency
  // hiding), with the row's coordinates loaded once per dimension.
  static_assert(TT * TT == 4 * TT_THREADS, "K pass: four entries per thread and tile");
  // (the kernel kind is dispatched once around the pass, and every entry is evaluated without a
  // branch -- padding and upper entries on a dummy radius, selected away -- so that the four
  // chains really interleave instead of running as four exec-masked regions)
  auto kpass = [&](auto kind_c) {
    constexpr int KIND = decltype(kind_c)::value;
    for (int qt = 0; qt < (int)ntile; ++qt) {
      int I, J;
      tile_ij(qt, I, J);
      const int gi = TT * I + (tid & 31), gj0 = TT * J + (tid >> 5);
      double r2[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll 3
      for (int u = 0; u < d; ++u) {
        const double* xu = XS + (size_t)u * NP;
        const double xi = xu[gi];
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const double r = xi - xu[gj0 + 8 * m];
          r2[m] = fma(r, r, r2[m]);
        }
      }
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const int gj = gj0 + 8 * m;
        const size_t e = (size_t)qt * (TT * TT) + tid + TT_THREADS * m;
        const bool ok = gi < N && gj < N && gj <= gi;
        double psi, dps[2];
        psi_dtheta_k<KIND>(ell, per, (gi == gj || !ok) ? 0.0 : sqrt(r2[m]), psi, dps);
        Lt[e] = ok ? ((gi == gj) ? psi + q.sn2 : psi) : ((gi == gj) ? 1.0 : 0.0);
#pragma unroll
        for (int t = 0; t < NT; ++t)   // the same bits the traces used to recompute
          Dt[(size_t)t * ntile * (TT * TT) + e] = ok ? dps[t] : 0.0;
      }
    }
  };
  switch (q.kernel) {
    case 0: kpass(std::integral_constant<int, 0>{}); break;
    case 1: kpass(std::integral_constant<int, 1>{}); break;
    case 2: kpass(std::integral_constant<int, 2>{}); break;
    case 3: kpass(std::integral_constant<int, 3>{}); break;
    default: kpass(std::integral_constant<int, 4>{}); break;
  }
  __syncthreads();
  TT_STAMP(1);
  double lgl = 0.0;   // Σ log L_ii: lane i < 32 of wave 0 sums row i of every diagonal tile
  for (int k = 0; k < T; ++k) {
    if (w == 0) {
      // A_kk → L_kk (PosDefException → status 1) and the forward substitution's z_k
      const int i = lane & 31, h = lane >> 5;
      const double* A = Lt + tile_at(k, k);
      // A_kk → L_kk with the rows in registers (tt_chol: lane i holds row i, the pivot column
      // broadcast by DPP inside the fused FMAs, no LDS round trip per column).  The round-4
      // formulations before it -- each column of L through one LDS broadcast, or every l_jc by
      // readlane into scalar FMA operands -- ran 71 k and 186 k cycles per tile at N = 128.
      double a[2][16];
#pragma unroll
      for (int j = 0; j < TT; ++j) a[j / 16][j % 16] = A[j * TT + i];
      double rl = 0.0;
      const bool bad = !tt_chol(a, rl, i, std::make_integer_sequence<int, TT>{});
      if (!bad && h == 0) {
#pragma unroll
        for (int j = 0; j < TT; ++j) Dk[j * TT_LD + i] = a[j / 16][j % 16];
        rd[i] = rl;
        rdall[TT * k + i] = rl;
      }
      if (!bad) {
        // the forward half of c = L'\(L\y), fused into the factorisation: z_k = L_kk⁻¹ r_k, where
        // r_k = y_k − Σ_{J<k} L_kJ z_J was accumulated by the panels of the earlier tile columns
        double r = yv[TT * k + i];
        tt_fwd(r, a, rl, i, std::make_integer_sequence<int, TT>{});
        if (lane < TT) uv[TT * k + i] = r;
      }
      gr_sync();
      TT_STAMP(8);
      if (bad) {
        if (lane == 0) fail = 1;
      } else {
        if (lane < TT && TT * k + lane < N) lgl += log(Dk[lane * TT_LD + lane]);
        if (T - k - 1 > 6) {
          // more panel tiles than waves 1-3 take in one round: W_k here, serially (below, it
          // would delay wave 0's own panel tiles), copied out by the whole workgroup
          double wc[TT];
          tt_inverse(wc, Dk, rd, i, std::make_integer_sequence<int, TT>{});
          if (lane < TT) {
#pragma unroll
            for (int r = 0; r < TT; ++r) Wk[lane * TT_LD + r] = wc[r];
          }
          gr_sync();
        }
        TT_STAMP(9);
      }
    }
    __syncthreads();
    TT_STAMP(2);
    if (fail) break;
    {
      // L_kk to the workspace by the whole workgroup, beside the panel (Dk stays in LDS until the
      // next diagonal step; the readers come after later barriers), coalesced
      double* Lkk = Lt + tile_at(k, k);
      double* Vkk = Vt + tile_at(k, k);
      double* Wkk = Wt + (size_t)k * (TT * TT);
      const bool w_done = T - k - 1 > 6;
      for (int e = tid; e < TT * TT; e += TT_THREADS) {
        const int r = e & 31, cc = e >> 5;                 // column-major (r, cc)
        Lkk[e] = (r >= cc) ? Dk[cc * TT_LD + r] : 0.0;
        if (w_done) {
          Wkk[e] = Wk[cc * TT_LD + r];
          Vkk[e] = Wk[r * TT_LD + cc];                     // row-major: V_kk = W_k
        }
      }
    }
    TT_STAMP(10);
    // panel: L_Ik = A_Ik·L_kk⁻ᵀ by forward substitution, one row per lane, the row in registers:
    // L_Ik[r][c] = (A_Ik[r][c] − Σ_{m<c} L_Ik[r][m]·L_kk[c][m]) / L_kk[c][c], the factor's own
    // recurrence (a product with the explicit inverse W_k is ≈ κ(L_kk) less accurate), row c of
    // L_kk broadcast by DPP.  Meanwhile wave 0 forms W_k = L_kk⁻¹ (needed only by the V pass):
    // the panel tiles go to the half-waves of waves 1-3 first (slots 0-5 of every round of 8),
    // wave 0's two halves take slots 6 and 7.
    {
      const int i = lane & 31, h = lane >> 5, npanel = T - k - 1;
      auto form_w = [&]() {
        // W column j = lane & 31: W_ij = (δ_ij − Σ_{m<i} L_im W_mj)/L_ii, the column in registers
        // (W_mj = 0 for m < j comes out of the same recursion), row i of L broadcast by DPP
        double wc[TT];
        tt_inverse(wc, Dk, rd, i, std::make_integer_sequence<int, TT>{});
        if (lane < TT) {
#pragma unroll
          for (int r = 0; r < TT; ++r) Wk[lane * TT_LD + r] = wc[r];
        }
        gr_sync();
        double* Vkk = Vt + tile_at(k, k);
        double* Wkk = Wt + (size_t)k * (TT * TT);
        for (int e = lane; e < TT * TT; e += 64) {
          const int r = e & 31, cc = e >> 5;
          Wkk[e] = Wk[cc * TT_LD + r];                     // column-major
          Vkk[e] = Wk[r * TT_LD + cc];                     // row-major: V_kk = W_k
        }
      };
      // with at most six panel tiles wave 0 has none and W_k runs entirely beside the panel
      // (with more, the diagonal step formed it)
      if (w == 0 && npanel <= 6) form_w();
      const int slot0 = (w == 0) ? 6 : 2 * (w - 1), slot = slot0 + h;
      for (int t0 = 0; t0 + slot0 < npanel; t0 += 8) {     // wave-uniform: some half has a tile
        const int t = t0 + slot;
        const bool has = t < npanel;
        const int I = k + 1 + (has ? t : 0);
        double* A = Lt + tile_at(I, k);
        double lrow[TT];
#pragma unroll
        for (int c = 0; c < TT; ++c) lrow[c] = has ? A[c * TT + i] : 0.0;
        tt_panel(lrow, Dk, rd, i, std::make_integer_sequence<int, TT>{});
        // r_I −= L_Ik z_k (the forward substitution's update of the rows below; z_k by DPP)
        double t0s = 0.0, t1s = 0.0, b0, b1, b2, b3;
        const double zl = uv[TT * k + i];
        row_blocks<0>(zl, b0, b2);
        DotAsm<16>::run(t0s, t1s, b0, &lrow[0]);
        row_blocks<1>(zl, b1, b3);
        DotAsm<16>::run(t0s, t1s, b1, &lrow[16]);
        if (has) {
#pragma unroll
          for (int c = 0; c < TT; ++c) A[c * TT + i] = lrow[c];
          yv[TT * I + i] -= t0s + t1s;
        }
      }
    }
    __syncthreads();
    TT_STAMP(3);
    // trailing update A_IJ −= L_Ik·L_Jkᵀ, k < J ≤ I
    // (software-pipelined: a wave loads its next pair's C tile and operands before the current
    // pair's products, so one global round trip per pair overlaps the matrix-core work)
    const int m = T - k - 1, npair = m * (m + 1) / 2;
    if (w < npair) {
      int I, J;
      tile_ij(w, I, J);
      I += k + 1;
      J += k + 1;
      f64x4 c[2][2];
      TileFrag f;
      tile_load<false>(c, Lt + tile_at(I, J), lane);
      frag_load(f, Lt + tile_at(I, k), Lt + tile_at(J, k), lane);
      for (int pi = w; pi < npair; pi += 4) {
        const bool more = pi + 4 < npair;
        int In = I, Jn = J;
        f64x4 cn[2][2];
        TileFrag fn;
        if (more) {
          tile_ij(pi + 4, In, Jn);
          In += k + 1;
          Jn += k + 1;
          tile_load<false>(cn, Lt + tile_at(In, Jn), lane);
          frag_load(fn, Lt + tile_at(In, k), Lt + tile_at(Jn, k), lane);
        }
        frag_sub(c, f);
        tile_store<false>(c, Lt + tile_at(I, J), lane);
        if (more) {
#pragma unroll
          for (int bi = 0; bi < 2; ++bi)
#pragma unroll
            for (int bj = 0; bj < 2; ++bj) c[bi][bj] = cn[bi][bj];
          f = fn;
          I = In;
          J = Jn;
        }
      }
    }
    __syncthreads();
    TT_STAMP(4);
  }
  if (fail) {
    if (tid == 0) {
      q.ll[p] = NAN;
      for (int t = 0; t < NT; ++t) q.grad[(size_t)p * NT + t] = NAN;
      q.status[p] = 1;
    }
    return;
  }
  if (w == 0) {
    const double lg = gr_sum(lgl);
    if (lane == 0) part[0][2 * NT + 1] = lg;   // wave 0's sum
  }
  // V = L⁻¹ below the diagonal tiles, by tile rows
  for (int I = 1; I < T; ++I) {
    for (int J = w; J < I; J += 4) {
      f64x4 c[2][2];
      tile_zero(c);
      for (int M = J; M < I; ++M) tile_xyt<false>(c, Lt + tile_at(I, M), Vt + tile_at(M, J), lane);   // L_IM·V_MJ
      double* S = Sw + w * (TT * TT);
      tile_store<true>(c, S, lane);
      gr_sync();
      tile_zero(c);
      tile_xyt<true>(c, Wt + (size_t)I * (TT * TT), S, lane);   // −W_I·S
      tile_store<true>(c, Vt + tile_at(I, J), lane);
      gr_sync();
    }
    __syncthreads();
    TT_STAMP(5);
  }
  // c = L'\(L\y) by blocked substitution (wave 0; lane i < 32 = row i of the current tile):
  // forward z_I = L_II⁻¹(y_I − Σ_{J<I} L_IJ z_J) (done during the factorisation), backward
  // c_I = L_II⁻ᵀ(z_I − Σ_{J>I} L_JIᵀ c_J);
  // inside a tile the column-oriented substitution with the solved entry broadcast by readlane.
  // yᵀc as the reference's log_likelihood forms it.
  if (w == 0) {
    const int i = lane & 31;
    double yc = 0.0;
    // (z = L⁻¹y is in uv: the factorisation's diagonal steps and panels formed it; the
    // backward tiles' loads are software-pipelined: tile J + 1's loads are in flight during tile
    // J's products, which run as four partial sums)
    for (int I = T - 1; I >= 0; --I) {
      double r = uv[TT * I + i];
      double lm[TT], lj[TT];
      const double* LD_ = Lt + tile_at(I, I);
#pragma unroll
      for (int m = 0; m < TT; ++m) lm[m] = LD_[i * TT + m];
      if (I + 1 < T) {
#pragma unroll
        for (int j = 0; j < TT; ++j) lj[j] = Lt[tile_at(I + 1, I) + i * TT + j];
      }
      double r4[4] = {0.0, 0.0, 0.0, 0.0};
      for (int J = I + 1; J < T; ++J) {
        double cur[TT];
#pragma unroll
        for (int j = 0; j < TT; ++j) cur[j] = lj[j];
        if (J + 1 < T) {
#pragma unroll
          for (int j = 0; j < TT; ++j) lj[j] = Lt[tile_at(J + 1, I) + i * TT + j];
        }
#pragma unroll
        for (int j = 0; j < TT; ++j) r4[j & 3] = fma(-cur[j], yv[TT * J + j], r4[j & 3]);
      }
      r += (r4[0] + r4[1]) + (r4[2] + r4[3]);
#pragma unroll
      for (int m = TT - 1; m >= 0; --m) {
        const double cm = readlane_d(r, m) * rdall[TT * I + m];
        if (i == m) r = cm;
        else if (i < m) r = fma(-lm[m], cm, r);
      }
      gr_sync();
      if (lane < TT) {
        if (TT * I + i < N) yc = fma(q.y[TT * I + i], r, yc);
        yv[TT * I + i] = r;   // c (y_I is no longer needed: rows > I are done)
      }
      gr_sync();
    }
    yc = gr_sum(yc);
    if (lane == 0) part[0][2 * NT] = yc;
  }
  __syncthreads();
  TT_STAMP(6);
  // K⁻¹ tiles and the traces over the strictly lower entries
  double tr[NT], cgc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) tr[t] = cgc[t] = 0.0;
  for (int pi = w; pi < (int)ntile; pi += 4) {
    int I, J;
    tile_ij(pi, I, J);
    // this lane's δK_t entries of the tile (from the K pass) and c_i·c_j, loaded before the
    // products so that their latency hides behind the MFMA chain
    double dk[NT][16], cc[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int bi = e >> 3, bj = (e >> 2) & 1, j = e & 3;
      const int li = 16 * bi + (lane >> 4) + 4 * j, lj = 16 * bj + (lane & 15);
      cc[e] = yv[TT * I + li] * yv[TT * J + lj];
#pragma unroll
      for (int t = 0; t < NT; ++t) dk[t][e] = Dt[(size_t)t * ntile * (TT * TT) + tile_at(I, J) + lj * TT + li];
    }
    f64x4 c[2][2];
    tile_zero(c);
    for (int M = I; M < T; ++M) tile_xyt<false>(c, Vt + tile_at(M, I), Vt + tile_at(M, J), lane);   // V_MIᵀ·V_MJ
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int bi = e >> 3, bj = (e >> 2) & 1, j = e & 3;
      const int li = 16 * bi + (lane >> 4) + 4 * j, lj = 16 * bj + (lane & 15);
      const int gi = TT * I + li, gj = TT * J + lj;
      if (gi > gj && gi < N) {
        const double kij = c[bi][bj][j];
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          tr[t] = fma(kij, dk[t][e], tr[t]);
          cgc[t] = fma(cc[e], dk[t][e], cgc[t]);
        }
      }
    }
  }
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const double trs = gr_sum(tr[t]), cgs = gr_sum(cgc[t]);
    if (lane == 0) { part[w][t] = trs; part[w][NT + t] = cgs; }
  }
  __syncthreads();
  TT_STAMP(7);
  if (tid == 0) {
#pragma unroll
    for (int t = 0; t < NT; ++t) {   // both triangles: 2·Σ_{j<i}, halved by δlog_likelihood's 1/2
      const double trs = (part[0][t] + part[1][t]) + (part[2][t] + part[3][t]);
      const double cgs = (part[0][NT + t] + part[1][NT + t]) + (part[2][NT + t] + part[3][NT + t]);
      q.grad[(size_t)p * NT + t] = cgs - trs;
    }
    q.ll[p] = -0.5 * part[0][2 * NT] - part[0][2 * NT + 1] - 0.5 * N * log(2.0 * 3.141592653589793);
    q.status[p] = 0;
  }
#ifdef MRBO_GPFIT_STAMPS
  if (p == 0 && tid == 0)
    printf("gpfit_tile N=%d cycles: K %llu  diag %llu (factor %llu, W %llu, copy %llu, wait %llu)  panel %llu  trailing %llu  "
           "V %llu  c %llu  traces %llu\n", N, tt_acc[1], tt_acc[2] + tt_acc[8] + tt_acc[9] + tt_acc[10], tt_acc[8],
           tt_acc[9], tt_acc[10], tt_acc[2], tt_acc[3], tt_acc[4], tt_acc[5], tt_acc[6], tt_acc[7]);
#endif
  if (q.L_out) {
    double* Lo = q.L_out + (size_t)N * N * p;
    for (size_t idx = tid; idx < (size_t)N * N; idx += TT_THREADS) {
      const int i = (int)(idx % N), j = (int)(idx / N);
      Lo[idx] = (i >= j) ? Lt[tile_at(i / TT, j / TT) + (j % TT) * TT + i % TT] : 0.0;
    }
  }
  if (q.c_out)
    for (int i = tid; i < N; i += TT_THREADS) q.c_out[(size_t)N * p + i] = yv[i];
}

size_t gpfit_tile_lds(int d, int N) {
  const int NP = ((N + TT - 1) / TT) * TT;
  return sizeof(double) * ((size_t)d * NP + 2 * TT * TT_LD + TT + 4 * TT * TT + 3 * (size_t)NP);
}

size_t gpfit_tile_work_doubles(int N, int nt) {
  const size_t T = (N + TT - 1) / TT, ntile = T * (T + 1) / 2;
  return ((2 + (size_t)nt) * ntile + T) * TT * TT;
}

size_t gpfit_lds_bytes() { return sizeof(double) * ((size_t)GL_N * GL_LD + 16 * GL_N + 3 * GL_N); }

size_t gpfit_reg_lds(int nt) { return sizeof(double) * ((size_t)(2 + nt) * 64 * GR_LD + 64 + 16 * 64); }

// dynamic LDS of the launch plus the selected kernel's static __shared__ arrays (part[][], the
// failure flags), so that mrbo_gp_fit_theta's limit check sees what the launch will request
size_t gpfit_launch_lds(const GpFitParams& q) {
  size_t dyn;
  const void* fn;
  if (gpfit_in_regs(q)) {
    dyn = gpfit_reg_lds(q.nt);
    fn = q.nt == 2 ? (const void*)gpfit_reg_kernel<2> : (const void*)gpfit_reg_kernel<1>;
  } else if (gpfit_in_lds(q)) {
    dyn = gpfit_lds_bytes();
    fn = q.nt == 2 ? (const void*)gpfit_lds_kernel<2> : (const void*)gpfit_lds_kernel<1>;
  } else {
    dyn = gpfit_tile_lds(q.d, q.N);
    fn = q.nt == 2 ? (const void*)gpfit_tile_kernel<2> : (const void*)gpfit_tile_kernel<1>;
  }
  hipFuncAttributes fa{};
  if (hipFuncGetAttributes(&fa, fn) == hipSuccess) dyn += fa.sharedSizeBytes;
  else dyn += 4096;   // attributes unavailable: keep a margin for the static arrays
  return dyn;
}

void launch_gpfit(int P, hipStream_t st, const GpFitParams& q) {
  if (gpfit_in_regs(q)) {
    if (q.nt == 2)
      hipLaunchKernelGGL(gpfit_reg_kernel<2>, dim3(P), dim3(64 * GR_WAVES), gpfit_reg_lds(2), st, q, P);
    else
      hipLaunchKernelGGL(gpfit_reg_kernel<1>, dim3(P), dim3(64 * GR_WAVES), gpfit_reg_lds(1), st, q, P);
    return;
  }
  if (gpfit_in_lds(q)) {
    if (q.nt == 2)
      hipLaunchKernelGGL(gpfit_lds_kernel<2>, dim3(P), dim3(GL_THREADS), gpfit_lds_bytes(), st, q, P);
    else
      hipLaunchKernelGGL(gpfit_lds_kernel<1>, dim3(P), dim3(GL_THREADS), gpfit_lds_bytes(), st, q, P);
    return;
  }
  if (q.nt == 2)
    hipLaunchKernelGGL(gpfit_tile_kernel<2>, dim3(P), dim3(TT_THREADS), gpfit_tile_lds(q.d, q.N), st, q, P);
  else
    hipLaunchKernelGGL(gpfit_tile_kernel<1>, dim3(P), dim3(TT_THREADS), gpfit_tile_lds(q.d, q.N), st, q, P);
}

}  // namespace mrbo
