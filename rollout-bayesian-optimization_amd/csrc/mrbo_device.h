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

#define MRBO_QUEUE_INTS (8 * 16)   // eight work-queue heads, one 64-B line each

namespace mrbo {

// work counters per trajectory (for the algorithmic-FLOP roofline):
// evals[NCOUNT·t + k], k = gradient evals, value evals, Hessians, adjoint rich evals, pairs
constexpr int NCOUNT = 5;
constexpr int NSTAMP = 22;        // MRBO_STAMPS regions (names in mrbo_api.hip)
constexpr int STAMP_RETRY = 22;   // slot counting Gershgorin retries
constexpr int NSTAMP_SLOTS = 24;  // accumulator slots per wave (U_STAMP) and in kp.stamps
#ifndef MRBO_FMAX
#define MRBO_FMAX 6
#endif
constexpr int FMAX = MRBO_FMAX;   // fantasy points per trajectory = h+1  (h ≤ 5)
constexpr int WAVE = 64;
constexpr int MAXD = 16;   // widest input dimension of a cost model (mrbo_plan_create check)
enum { COST_NONE = 0, COST_QUADRATIC = 1, COST_LOGLINEAR = 2 };   // mrbo_cost_t

// N ≤ 256 (L0⁻¹ from L2, four rows per lane): blocks (1,0), (2,0), (2,1) of the block triangle
// (packed indices 1, 3, 4) are also staged in workgroup LDS, in the LD = 65 layout of the N ≤ 128
// kernel; their products read LDS instead of L2 (device and host agree through gl_lds_slot).
// MRBO_GL_LDS_BLOCKS=0: every block from L2.  The chained / streamed A/B variants read L2 only.
#ifndef MRBO_GL_LDS_BLOCKS
#define MRBO_GL_LDS_BLOCKS 3
#endif
#if defined(MRBO_GL_CHAIN) || defined(MRBO_K1_STREAM)
constexpr int GL_LDS_BLOCKS = 0;
#else
constexpr int GL_LDS_BLOCKS = MRBO_GL_LDS_BLOCKS;
#endif
static_assert(GL_LDS_BLOCKS >= 0 && GL_LDS_BLOCKS <= 3, "LDS-resident L2-layout blocks: 0..3");
#ifdef MRBO_GL_LDS_DIAG
// A/B: the diagonal blocks (0,0), (1,1), (2,2) instead, walked by the folded LDS products
constexpr int GL_LDS_B0 = 0, GL_LDS_B1 = 2, GL_LDS_B2 = 5;
constexpr bool GL_LDS_FOLD = true;
#else
constexpr int GL_LDS_B0 = 1, GL_LDS_B1 = 3, GL_LDS_B2 = 4;
constexpr bool GL_LDS_FOLD = false;
#endif
__host__ __device__ constexpr int gl_lds_slot(int b) {
  return (b == GL_LDS_B0 && GL_LDS_BLOCKS > 0) ? 0 : (b == GL_LDS_B1 && GL_LDS_BLOCKS > 1) ? 1
       : (b == GL_LDS_B2 && GL_LDS_BLOCKS > 2) ? 2 : -1;
}

// evaluation modes (wave-uniform).  The front part (kernel rows, forward product, Gram, μ, σ,
// EI and its gradient) runs in every mode but BACK; the back part (backward product w, and
// the Hessian for FULL / RICH / BACK) resumes from state the front part left in LDS.
//   VALUE  α only                      GRAD  α, ∇α (Hessian deferrable: BACK may follow)
//   DRAW   GRAD + w (condition!)       FULL  GRAD + w + Hα
//   RICH   FULL + P = L⁻ᵀV (adjoint)   BACK  w + Hα at the point of the preceding GRAD(C)
//   GRADC  completes a VALUE evaluation to GRAD (gradient columns only; same results)
//   GSTART GRAD at an inner-solve start point: the base forward product and base Gram come
//          from the launch's start tables (stage_start_tables), only surface terms are computed
enum { EV_VALUE = 0, EV_GRAD = 1, EV_DRAW = 2, EV_FULL = 3, EV_RICH = 4, EV_BACK = 5, EV_GRADC = 6, EV_GSTART = 7 };

struct KParams {
  int d, N, Npad, h, M, R, nstarts;
  int kernel;
  int rule;             // mrbo_rule_t: EI, POI, LCB
  double ell, cK, cP, psi0, d2psi0, sn2;   // cP: Periodic 2π/p
  double fmin_base, fmini, theta;
  // gradient certificate (newton_grad_certified): max_ρ |ψ'(ρ)| and √(ψ(0)·(−ψ''(0))), the
  // latter ≤ 0 when the derivative process has no finite variance (Matérn-1/2: disabled)
  double gcert_mu, gcert_sig;
  double gcert_d2;      // tight certificate: 1.01·√(−ψ''(0)) (used when gcert_sig > 0)
  int max_iters, max_ls;
  double x_tol, f_tol, g_tol, htol, sigma_tol;
  unsigned long long seed;
  int sample_offset, samples_total;
  int with_gradient;
  int xs_lds;           // xstarts staged in LDS after L0⁻¹ (rollout launches)
  int batch;            // batched start-point values (needs xs_lds, RPL = 1, nstarts ≤ 64)
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
  double* ytab;         // kp.batch, square layout: per-workgroup slices [blockIdx][nstarts][NR] of Y0(x_start)
  double* kxb_g;        // kp.batch, packed layouts (N > 64): global start tables [nstarts][NR] and
  double* gtab_g;       //   [nstarts][NG] written by start_tables_kernel before the rollout launch
  const double* ghq_nodes;  // Gauss–Hermite estimator: M×(h+1) nodes and weights per sample (else null)
  const double* ghq_w;
  int* queue;           // work-queue heads, one per XCD at queue[16·x] (zeroed before every launch)
  const int* order;     // optional: queue position -> trajectory (mrbo_plan_set_order), else identity
  const int* skip_active;  // mrbo_stochastic_solve: a restart r with skip_active[r] == 0 has stopped
                           // (eswavs); its trajectories are not re-run (x0 unchanged: the outputs
                           // the previous launch left are the ones they would reproduce).  Else null
  long long T;          // trajectories (or points for eval_base)
  const double* pts;    // eval_base: d×P
  double* pts_out;      // eval_base output
  unsigned long long* stamps;  // MRBO_STAMPS builds: per-region cycle totals (else null)
  // NonUniformCost weighting of the inner-solve rule (mrbo_cost_t; 0 = none): f = α/c(x) with
  // u_a = (x_a − lb_a)/del_a, QUADRATIC c = c0 + Σ w_a u_a², LOGLINEAR c = c0·exp(Σ w_a u_a)
  // (a pointer, not arrays: array members would put the kernel's copy of KParams in scratch)
  int cost;
  double cost_c0;
  const double* cost_tab;   // device [lb (d), del = ub − lb (d), w (d)]
  // mrbo_base_solve: item k of the launch = base_solve(s::Surrogate; xstart = column k of
  // xstarts) on the base surrogate (rbf_optim.jl:35-66); minimizer -> policy (d×T), minimum ->
  // values (T), no trajectory
  int base_solve;
};


// ---- packed L0⁻¹ layout: column j holds rows j..Npad-1 contiguously ----------------------
__host__ __device__ __forceinline__ constexpr long long linv_colstart(int j, int Npad) {
  return (long long)j * Npad - (long long)j * (j - 1) / 2;
}
__host__ __device__ __forceinline__ constexpr long long linv_size(int Npad) { return (long long)Npad * (Npad + 1) / 2; }

// ---- wave-scope synchronisation for LDS hand-offs between lanes of ONE wave ------------
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---- 64-bit cross-lane exchange ----------------------------------------------------------
__device__ __forceinline__ void dsplit(double v, int& lo, int& hi) {
  const long long b = __builtin_bit_cast(long long, v);
  lo = (int)b;
  hi = (int)(b >> 32);
}
__device__ __forceinline__ double djoin(int lo, int hi) {
  return __builtin_bit_cast(double, (long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}

// A fresh register pair holding v's bits: ONE v_mov_b64.  v_permlane16/32_swap overwrite both of
// their operands, so a swap of a double with itself needs two copies of it while it stays live; the
// compiler made them per dword (two v_mov_b32 per operand, four per double).  TAG makes the two
// copies distinct asm statements, so that they are not merged into one.  MRBO_NO_DCOPY: the
// compiler's copies (A/B).
template <int TAG>
__device__ __forceinline__ double dcopy(double v) {
  double r;
  if constexpr (TAG == 0) asm("v_mov_b64 %0, %1" : "=v"(r) : "v"(v));
  else asm("v_mov_b64 %0, %1 ; copy %2" : "=v"(r) : "v"(v), "i"(TAG));
  return r;
}

// v_permlane16_swap (M = 16) / v_permlane32_swap (M = 32) of a double with itself, per dword:
// first = [r0 r0 r2 r2] / [lo lo], second = [r1 r1 r3 r3] / [hi hi] (16-lane rows / 32-lane
// halves).  KEEP: v stays live after the swap (two copies); else v itself is one operand.
// COPY = false: the compiler's own copies (the L2-fed and GP-fit kernels at 512 registers, where
// the explicit copies' fixed live ranges cost spills: C5 + cost scratch 352 → 896 B per lane).
template <int M, bool KEEP, bool COPY = true>
__device__ __forceinline__ void self_swap(double v, double& first, double& second) {
#ifdef MRBO_NO_DCOPY
  const double c0 = v, c1 = v;
#else
  const double c0 = (KEEP && COPY) ? dcopy<0>(v) : v;
  const double c1 = COPY ? dcopy<1>(v) : v;
#endif
  int al, ah, bl, bh;
  dsplit(c0, al, ah);
  dsplit(c1, bl, bh);
  if constexpr (M == 16) {
    const auto l = __builtin_amdgcn_permlane16_swap(al, bl, false, false);
    const auto h = __builtin_amdgcn_permlane16_swap(ah, bh, false, false);
    first = djoin(l[0], h[0]);
    second = djoin(l[1], h[1]);
  } else {
    static_assert(M == 32, "self_swap: M is 16 or 32");
    const auto l = __builtin_amdgcn_permlane32_swap(al, bl, false, false);
    const auto h = __builtin_amdgcn_permlane32_swap(ah, bh, false, false);
    first = djoin(l[0], h[0]);
    second = djoin(l[1], h[1]);
  }
}

// M = 32 / 16: lanes with bit M clear get a(l) + a(l^M), lanes with it set get b(l^M) + b(l).
// gfx950's v_permlane32_swap / v_permlane16_swap exchange exactly these cross halves of the
// register pair in place: two swaps per double and one add -- no select, no LDS round trip.
// A zero padding operand (a reduction slot past the values' count, known at compile time after
// unrolling) is made by one v_mov_b64 instead of the compiler's two v_mov_b32: the swap overwrites
// it, so it cannot stay an inline constant.
__device__ __forceinline__ double swap_operand(double v) {
#ifndef MRBO_NO_DCOPY
  if (__builtin_constant_p(v) && v == 0.0) {
    double z;
    asm("v_mov_b64 %0, 0" : "=v"(z));
    return z;
  }
#endif
  return v;
}

template <int M>
__device__ __forceinline__ double swap_fold(double a, double b) {
  int alo, ahi, blo, bhi;
  dsplit(swap_operand(a), alo, ahi);
  dsplit(swap_operand(b), blo, bhi);
  if constexpr (M == 32) {
    const auto lo = __builtin_amdgcn_permlane32_swap(alo, blo, false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap(ahi, bhi, false, false);
    return djoin(lo[0], hi[0]) + djoin(lo[1], hi[1]);
  } else {
    static_assert(M == 16, "swap_fold: M is 32 or 16");
    const auto lo = __builtin_amdgcn_permlane16_swap(alo, blo, false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap(ahi, bhi, false, false);
    return djoin(lo[0], hi[0]) + djoin(lo[1], hi[1]);
  }
}

// Register broadcast (rollout products, GP-fit Cholesky): blocks p and p+2 of v (lane j holds
// row j), each replicated into all four 16-lane rows, so that DPP row_newbcast:n then reads
// row 16b + n in every lane.
template <int P, bool COPY = false>
__device__ __forceinline__ void row_blocks(double v, double& blk_p, double& blk_p2) {
  double a0, a1;
  self_swap<16, true, COPY>(v, a0, a1);                  // [r0 r0 r2 r2], [r1 r1 r3 r3]
  self_swap<32, false, COPY>(P ? a1 : a0, blk_p, blk_p2); // [rP ×4], [rP+2 ×4]
}

// All four blocks at once: one v_permlane16_swap and two v_permlane32_swap per dword (blocks 0, 2
// from the first pl16 half, 1, 3 from the second) instead of a pl16 + pl32 pair per block pair.
template <bool COPY = false>
__device__ __forceinline__ void row_blocks4(double v, double& b0, double& b1, double& b2, double& b3) {
  double a0, a1;
  self_swap<16, true, COPY>(v, a0, a1);    // [r0 r0 r2 r2], [r1 r1 r3 r3]
  self_swap<32, false, COPY>(a0, b0, b2);  // [r0 ×4], [r2 ×4]
  self_swap<32, false, COPY>(a1, b1, b3);  // [r1 ×4], [r3 ×4]
}

// The three broadcast operands of a folded product (bcast_fold_fwd / _bwd) in 3 swaps and 2 copies
// per dword, instead of all four blocks (row_blocks4: 3 swaps, 3 copies) plus a per-row select of
// the folded pass's operand (2 v_cndmask per double).  With a0 = [r0 r0 r2 r2], a1 = [r1 r1 r3 r3]
// from the first swap, v_permlane32_swap(a1, a0) gives X = [r1 r1 r0 r0] and Y = [r3 r3 r2 r2]:
//   forward:  Y is the folded operand (row 1: block 3, rows 2, 3: block 2, row 0 idle) and the
//             self-swap of X gives blocks 1 and 0;
//   backward: X is the folded operand (rows 0, 1: block 1, row 2: block 0, row 3 idle) and the
//             self-swap of Y gives blocks 3 and 2.
__device__ __forceinline__ void fold_blocks(double v, bool fwd, double& p0, double& p1, double& m) {
  double a0, a1;
  self_swap<16, true>(v, a0, a1);   // [r0 r0 r2 r2], [r1 r1 r3 r3]
  int a0l, a0h, a1l, a1h;
  dsplit(a0, a0l, a0h);
  dsplit(a1, a1l, a1h);
  const auto xl = __builtin_amdgcn_permlane32_swap(a1l, a0l, false, false);   // X, Y (low dwords)
  const auto xh = __builtin_amdgcn_permlane32_swap(a1h, a0h, false, false);
  const int sl = fwd ? xl[0] : xl[1], sh = fwd ? xh[0] : xh[1];   // the pair to self-swap
  const auto cl = __builtin_amdgcn_permlane32_swap(sl, sl, false, false);
  const auto ch = __builtin_amdgcn_permlane32_swap(sh, sh, false, false);
  p0 = djoin(cl[1], ch[1]);   // forward: block 0; backward: block 2
  p1 = djoin(cl[0], ch[0]);   // forward: block 1; backward: block 3
  m = fwd ? djoin(xl[1], xh[1]) : djoin(xl[0], xh[0]);
}

// The value of lane (l & 31) + 32·H in every lane l: one v_permlane32_swap per dword of the
// register with itself leaves the lower half's values in both halves of the first result and the
// upper half's in both halves of the second (H a compile-time constant after unrolling).
__device__ __forceinline__ double half_value(double v, int H) {
  double lo, hi;
  self_swap<32, true>(v, lo, hi);
  return H ? hi : lo;
}

// M = 8, 4, 2, 1: v from a partner lane that differs in bit M and agrees on all higher bits
// (DPP row_mirror, row_half_mirror, quad_perm xor2 / xor1 -- one VALU move per dword).
template <int M>
__device__ __forceinline__ double dpp_partner(double v) {
  constexpr int ctrl = (M == 8) ? 0x140 : (M == 4) ? 0x141 : (M == 2) ? 0x4E : 0xB1;
  static_assert(M == 8 || M == 4 || M == 2 || M == 1, "dpp_partner: M in {8,4,2,1}");
  int lo, hi;
  dsplit(v, lo, hi);
  // every lane has an in-row source for these controls: mov_dpp needs no 'old' operand (an
  // update_dpp with old = 0 materialised two zero moves per double)
  lo = __builtin_amdgcn_mov_dpp(lo, ctrl, 0xF, 0xF, true);
  hi = __builtin_amdgcn_mov_dpp(hi, ctrl, 0xF, 0xF, true);
  return djoin(lo, hi);
}

// One transpose step: H pairs (v[q], v[q+H]) become H partial sums over twice as many lanes;
// lanes with bit M set continue with the upper half of the values.
template <int M, int H>
__device__ __forceinline__ void fold_step(double* v, int lane, int& idx) {
  const bool up = (lane & M) != 0;
#pragma unroll
  for (int q = 0; q < H; ++q) {
    if constexpr (M >= 16) {
      v[q] = swap_fold<M>(v[q], v[q + H]);
    } else {
      const double send = up ? v[q] : v[q + H];
      const double keep = up ? v[q + H] : v[q];
      v[q] = keep + dpp_partner<M>(send);
    }
  }
  idx += up ? H : 0;
}
template <int M>
__device__ __forceinline__ double fold_all(double v) {
  if constexpr (M >= 16) {
    double a, b;   // a(l) + a(l^M) in every lane: the self-swap's two halves summed
    self_swap<M, false>(v, a, b);
    return a + b;
  } else {
    return v + dpp_partner<M>(v);
  }
}

// Transpose-reduce K per-lane values across the 64 lanes: log2(K) transpose steps (pairs
// across lane bits 5, 4, …) leave one partial per lane, then plain all-reduce steps finish;
// one lane per group writes red[idx].  Cost ≈ K + log2(64/K) exchanges instead of 6K.
// The pairing and summation order are fixed: the result is deterministic.
template <int K>
__device__ __forceinline__ void wave_reduce(double (&v)[K], double* red, int lane) {
  constexpr int S = (K == 1) ? 0 : (K == 2) ? 1 : (K == 4) ? 2 : (K == 8) ? 3 : (K == 16) ? 4 : 5;
  static_assert((1 << S) == K, "K must be a power of two <= 32");
  int idx = 0;
  if constexpr (S >= 1) fold_step<32, K / 2>(v, lane, idx);
  if constexpr (S >= 2) fold_step<16, K / 4>(v, lane, idx);
  if constexpr (S >= 3) fold_step<8, K / 8>(v, lane, idx);
  if constexpr (S >= 4) fold_step<4, K / 16>(v, lane, idx);
  if constexpr (S >= 5) fold_step<2, K / 32>(v, lane, idx);
  if constexpr (S < 1) v[0] = fold_all<32>(v[0]);
  if constexpr (S < 2) v[0] = fold_all<16>(v[0]);
  if constexpr (S < 3) v[0] = fold_all<8>(v[0]);
  if constexpr (S < 4) v[0] = fold_all<4>(v[0]);
  if constexpr (S < 5) v[0] = fold_all<2>(v[0]);
  v[0] = fold_all<1>(v[0]);
#ifndef MRBO_REDUCE_LEADER_STORE
  // every lane of a group holds the same bits and the same idx: an unconditional store keeps the
  // reductions of one phase in one scheduling region (no exec-mask branch between them; C3 −0.3 %)
  red[idx] = v[0];
#else
  if ((lane & ((64 >> S) - 1)) == 0) red[idx] = v[0];
#endif
}

// wave_reduce within each 32-lane half of the wave (half-wave mode: two trajectories per wave, one
// per half): the same transpose steps from lane bit 4 down, no v_permlane32_swap; each half stores
// its own K sums through its own red pointer.  K ≤ 16.
template <int K>
__device__ __forceinline__ void half_reduce(double (&v)[K], double* red, int lane) {
  constexpr int S = (K == 1) ? 0 : (K == 2) ? 1 : (K == 4) ? 2 : (K == 8) ? 3 : 4;
  static_assert((1 << S) == K && K <= 16, "half_reduce: K a power of two <= 16");
  int idx = 0;
  if constexpr (S >= 1) fold_step<16, K / 2>(v, lane, idx);
  if constexpr (S >= 2) fold_step<8, K / 4>(v, lane, idx);
  if constexpr (S >= 3) fold_step<4, K / 8>(v, lane, idx);
  if constexpr (S >= 4) fold_step<2, K / 16>(v, lane, idx);
  if constexpr (S < 1) v[0] = fold_all<16>(v[0]);
  if constexpr (S < 2) v[0] = fold_all<8>(v[0]);
  if constexpr (S < 3) v[0] = fold_all<4>(v[0]);
  if constexpr (S < 4) v[0] = fold_all<2>(v[0]);
  v[0] = fold_all<1>(v[0]);
  red[idx] = v[0];
}

// min over the first LANES lanes' values (LANES = 64, or 32 within each half-wave) in every lane, by
// the butterfly of wave_allreduce1: permlane self-swaps across lane bits 5 / 4, DPP moves below
// (no ds_bpermute and no per-lane shuffle address).  min is exact, so every lane holds the same bits.
template <int LANES>
__device__ __forceinline__ double lanes_min(double v) {
  double a, b;
  if constexpr (LANES == 64) {
    self_swap<32, false>(v, a, b);
    v = fmin(a, b);
  }
  self_swap<16, false>(v, a, b);
  v = fmin(a, b);
  v = fmin(v, dpp_partner<8>(v));
  v = fmin(v, dpp_partner<4>(v));
  v = fmin(v, dpp_partner<2>(v));
  return fmin(v, dpp_partner<1>(v));
}

// Sum over the 64 lanes in EVERY lane, no LDS round trip: the butterfly of wave_reduce<1>
// (each step adds the partner's value; a + b == b + a, so all lanes hold the same bits, those
// wave_reduce<1> stores for lane 0).
__device__ __forceinline__ double wave_allreduce1(double v) {
  v = fold_all<32>(v);
  v = fold_all<16>(v);
  v = fold_all<8>(v);
  v = fold_all<4>(v);
  v = fold_all<2>(v);
  return fold_all<1>(v);
}

// ---- transcendentals behind leaf calls ---------------------------------------------------
// The fp64 exp/erfc expansions carry tens of 64-bit polynomial constants; inlined into the
// Newton/horizon loops, LICM hoists their materialisation out of the loops and the kernel
// spills them.  As leaf calls the constants stay local to the callee.
// 64-bit constant materialised in an SGPR pair at its point of use: the volatile moves cannot be
// hoisted out of loops, so polynomial coefficients never occupy registers across the Newton /
// horizon loops (two SALU moves per use, issued beside the VALU stream)
template <unsigned LO, unsigned HI>
__device__ __forceinline__ double sconst() {
  int lo, hi;
  asm volatile("s_mov_b32 %0, %1" : "=s"(lo) : "i"(LO));
  asm volatile("s_mov_b32 %0, %1" : "=s"(hi) : "i"(HI));
  return djoin(lo, hi);
}

// A quiet NaN materialised at its use (two SALU moves): the compiler hoisted the NAN literal of the
// failure outputs into a VGPR pair held across the persistent loop, and spilled it.
__device__ __forceinline__ double qnan() { return sconst<0u, 0x7ff80000u>(); }

// a·b + C with C = the compile-time double of bits (HI, LO), materialised in an SGPR pair (sconst):
// one VOP3 v_fma_f64 with the SGPR operand.  A plain fma() with an SGPR addend is shrunk by the
// compiler to v_fmac_f64, whose addend is also its destination, so every Horner step copied its
// coefficient into a VGPR pair first (two v_mov_b32 per step, three VALU instructions per
// polynomial term).  The addend is a template constant, so only a lane-uniform value can reach the
// "s" operand (a per-lane value there would be silently read from lane 0).  Not volatile: the
// scheduler moves it like any arithmetic.  MRBO_NO_FMA_SC: plain fma (A/B).
template <unsigned LO, unsigned HI>
__device__ __forceinline__ double fma_sc(double a, double b) {
#ifdef MRBO_NO_FMA_SC
  return fma(a, b, sconst<LO, HI>());
#else
  double d;
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "s"(sconst<LO, HI>()));
  return d;
#endif
}

// exp(x), inlined: the device library's algorithm and coefficients in the same operation order
// (Cody–Waite reduction by ln2, degree-11 polynomial, 2^k by v_ldexp_f64, overflow / underflow
// selects), so results are bit-identical to exp() -- without a call's prologue (scratch save of
// a VGPR and a full s_waitcnt on entry) or VALU moves for the coefficients.
__device__ __forceinline__ double fexp(double x) {
  const double k = __builtin_rint(x * sconst<0x652b82feu, 0x3ff71547u>());            // x·log2(e)
  double r = fma(sconst<0xfefa39efu, 0xbfe62e42u>(), k, x);                          // − k·ln2_hi
  r = fma(sconst<0x3b39803fu, 0xbc7abc9eu>(), k, r);                                 // − k·ln2_lo
#ifdef MRBO_EXP_ESTRIN
  // the same degree-11 polynomial P(r) = Σ c_k r^k (c0 = c1 = 1) in Estrin form: pairs
  // b_j = c_{2j} + c_{2j+1} r, then q = b + r²·b', then P = q0 + r⁴(q1 + r⁴ q2) -- dependent
  // depth 5 instead of 11, three more multiplies; not bit-identical to the device library's exp
  const double r2 = r * r, r4 = r2 * r2;
  double c10e = sconst<0xfca7ab0cu, 0x3e928af3u>();
  asm volatile("" : "+v"(c10e));
  const double b5 = fma(sconst<0x6a5dcb37u, 0x3e5ade15u>(), r, c10e);                 // c10 + c11 r
  const double b4 = fma_sc<0x7c89e6b0u, 0x3efa0199u>(r, sconst<0x623fde64u, 0x3ec71deeu>());   // c8 + c9 r
  const double b3 = fma_sc<0x1852b7b0u, 0x3f56c16cu>(r, sconst<0x14761f6eu, 0x3f2a01a0u>());
  const double b2 = fma_sc<0x555502a1u, 0x3fa55555u>(r, sconst<0x11122322u, 0x3f811111u>());
  const double b1 = fma_sc<0x0000000bu, 0x3fe00000u>(r, sconst<0x55555511u, 0x3fc55555u>());
  const double b0 = r + 1.0;
  const double q2 = fma(b5, r2, b4), q1 = fma(b3, r2, b2), q0 = fma(b1, r2, b0);
  const double p = fma(fma(q2, r4, q1), r4, q0);
  double e = __builtin_ldexp(p, (int)k);
#else
  double c10 = sconst<0xfca7ab0cu, 0x3e928af3u>();
  asm volatile("" : "+v"(c10));   // one of the first step's two constants must live in VGPRs
  double p = fma(sconst<0x6a5dcb37u, 0x3e5ade15u>(), r, c10);
  p = fma_sc<0x623fde64u, 0x3ec71deeu>(r, p);
  p = fma_sc<0x7c89e6b0u, 0x3efa0199u>(r, p);
  p = fma_sc<0x14761f6eu, 0x3f2a01a0u>(r, p);
  p = fma_sc<0x1852b7b0u, 0x3f56c16cu>(r, p);
  p = fma_sc<0x11122322u, 0x3f811111u>(r, p);
  p = fma_sc<0x555502a1u, 0x3fa55555u>(r, p);
  p = fma_sc<0x55555511u, 0x3fc55555u>(r, p);
  p = fma_sc<0x0000000bu, 0x3fe00000u>(r, p);
  p = fma(r, p, 1.0);
  p = fma(r, p, 1.0);
  double e = __builtin_ldexp(p, (int)k);
#endif
  e = (x > sconst<0u, 0x40900000u>()) ? __builtin_inf() : e;   // x > 1024
  e = (x < sconst<0u, 0xc090cc00u>()) ? 0.0 : e;               // x < −1075
  return e;
}

// Default (round 5): fexp inlined at every use, the paired xexp2 too.  Round 1 measured no gain from
// inlining (the calls' latency hidden by the second wave, VGPR spills 66 → 93); on the round-5
// kernel a leaf call costs ≈ 15 v_readlane reloads of spilled SGPRs before every s_swappc, and
// inlining runs C3 1.2 % faster with the spill count unchanged (6 VGPRs).  MRBO_LEAF_EXP: the
// round-4 leaf calls (A/B).
#ifdef MRBO_INLINE_TRANSCENDENTALS
__device__ __forceinline__ double xexp(double x) { return exp(x); }
__device__ __forceinline__ double xerfc(double x) { return erfc(x); }
#elif !defined(MRBO_LEAF_EXP)
__device__ __forceinline__ double xexp(double x) { return fexp(x); }
__device__ __attribute__((noinline)) double xerfc(double x) { return erfc(x); }
#else
__device__ __attribute__((noinline)) double xexp(double x) { return exp(x); }
__device__ __attribute__((noinline)) double xerfc(double x) { return erfc(x); }
#endif

// √s and 1/√s (s > 0) from one hardware reciprocal square root and two Newton–Raphson steps
// y ← y(1.5 − ½s·y²): ~1 ulp, and a much shorter dependent chain than a correctly rounded
// sqrt followed by an IEEE division (Cholesky pivots of the Newton step and of gp_draw).
__device__ __forceinline__ void sqrt_rsqrt(double s, double& r, double& ir) {
  const double h = 0.5 * s;
  double y = __builtin_amdgcn_rsq(s);
  y = fma(y, fma(-h * y, y, 0.5), y);
  y = fma(y, fma(-h * y, y, 0.5), y);
  ir = y;
  r = s * y;
}

// √s for s ≥ 0 (sums of squares) from sqrt_rsqrt: ~8 dependent operations instead of the IEEE
// expansion's ~14, within 2 ulp.  s ≤ 1e-290 (zero, subnormal) gives 0 and NaN stays NaN; the
// Matérn-5/2 forms and the certificates absorb a subnormal's root exactly (1 + 1e-145 = 1).
__device__ __forceinline__ double fast_sqrt0(double s) {
  double r, ir;
  sqrt_rsqrt(s, r, ir);
  return s > 1e-290 ? r : s * 0.0;
}

// σ = √var and 1/σ of a posterior variance: sqrt_rsqrt where var is a normal positive number,
// the IEEE root and division otherwise (σ = 0 → 1/σ = inf, var < 0 or NaN → NaN, as Julia)
__device__ __forceinline__ void sig_isig(double var, double& sig, double& isig) {
  if (var > 1e-290 && var < 1e290) {
    sqrt_rsqrt(var, sig, isig);
  } else {
    sig = sqrt(var);
    isig = 1.0 / sig;
  }
}

// ---- radial kernels (radial_basis_functions.jl:60-96; derivatives in closed form) -------
// kind ids = mrbo_kernel_t (include/mrbo.h)
enum { KERNEL_MATERN52 = 0, KERNEL_MATERN32 = 1, KERNEL_MATERN12 = 2, KERNEL_SE = 3, KERNEL_PERIODIC = 4 };
struct Radial {
  int kind;
  double cK;   // √5/ℓ, √3/ℓ, 1/ℓ  (Matérn) ; 1/ℓ² (SE, Periodic)
  double cP;   // Periodic: 2π/p
};

// ψ(ρ), g1 = ψ'(ρ)/ρ and g2 = (ψ''(ρ) − ψ'(ρ)/ρ)/ρ² from ρ², so that
//   k(r) = ψ,   ∇k(r) = g1·r,   ∇²k(r) = g2·r rᵀ + g1·I.
// The closed forms cancel the 1/ρ factors for Matérn-5/2 and SE (no division, no ρ = 0
// branch); Matérn-3/2 and -1/2 keep one reciprocal.  At ρ = 0, g1 = ψ''(0) and g2 = 0 — the
// reference's ρ = 0 branches (∇k = 0, ∇²k = ψ''(0)·I).
__device__ __forceinline__ void rad_eval(const Radial& k, double rho2, double& psi, double& g1, double& g2) {
  const double c = k.cK;
  if (k.kind == 4) {
    // Periodic (:98-103) ψ = exp(−2 sin²(πρ/p)/ℓ²).  With B = 2π/p, A = B/ℓ², t = Bρ:
    //   g1 = ψ'/ρ = −ψ A B sinc t,   g2 = ψ B² (A² sinc²t + A B (sinc t − cos t)/t²)
    // (sinc t − cos t)/t² = (sin t − t cos t)/t³ by its series below t = 0.1 (cancellation)
    const double B = k.cP, A = B * c;
    const double rho = sqrt(rho2), t = B * rho;
    double su, cu;
    sincos(0.5 * t, &su, &cu);
    psi = xexp(-2.0 * su * su * c);
    const double st = 2.0 * su * cu, ct = fma(-2.0 * su, su, 1.0);
    const double t2 = t * t;
    const bool small = t < 0.1;
    const double sinc = small ? fma(t2, fma(t2, 1.0 / 120.0, -1.0 / 6.0), 1.0) : st / t;
    const double f = small ? fma(t2, fma(t2, fma(t2, -1.0 / 45360.0, 1.0 / 840.0), -1.0 / 30.0), 1.0 / 3.0)
                           : (st - t * ct) / (t2 * t);
    g1 = -psi * A * B * sinc;
    g2 = psi * B * B * A * fma(A, sinc * sinc, B * f);
    return;
  }
  if (k.kind == 3) {
    const double e = xexp(-0.5 * c * rho2);
    psi = e;
    g1 = -c * e;
    g2 = c * c * e;
    return;
  }
  const double rho = (k.kind == 0) ? fast_sqrt0(rho2) : sqrt(rho2);
  const double s = c * rho, e = xexp(-s);
  if (k.kind == 0) {
    const double c23 = c * c * (1.0 / 3.0);
    psi = fma(s, fma(s, 1.0 / 3.0, 1.0), 1.0) * e;
    g1 = -c23 * (1.0 + s) * e;
    g2 = c23 * (c * c) * e;
  } else if (k.kind == 1) {
    psi = (1.0 + s) * e;
    g1 = -(c * c) * e;
    g2 = (rho > 0.0) ? (c * c * c) * e / rho : 0.0;
  } else {
    psi = e;
    if (rho > 0.0) {
      const double ir = 1.0 / rho;
      g1 = -c * e * ir;
      g2 = ((c * c) * e - g1) * (ir * ir);
    } else {
      g1 = c * c;
      g2 = 0.0;
    }
  }
}

// Two radial evaluations at once (a base row and a fantasy row of the same lane): for Matérn-5/2
// both exponentials come from one leaf call whose two inlined fexp chains interleave, instead of
// two calls in sequence.  Same closed forms as rad_eval; other kernels take two rad_eval calls.
struct Exp2 {
  double a, b;
};
#ifndef MRBO_LEAF_EXP
__device__ __forceinline__ Exp2 xexp2(double a, double b) {
#else
__device__ __attribute__((noinline)) Exp2 xexp2(double a, double b) {
#endif
  Exp2 r;
  r.a = fexp(a);
  r.b = fexp(b);
  return r;
}
__device__ __forceinline__ void rad_eval2(const Radial& k, double rho2a, double rho2b, double& psia, double& g1a,
                                          double& g2a, double& psib, double& g1b, double& g2b) {
  if (k.kind != 0) {
    rad_eval(k, rho2a, psia, g1a, g2a);
    rad_eval(k, rho2b, psib, g1b, g2b);
    return;
  }
  const double c = k.cK, c23 = c * c * (1.0 / 3.0);
  const double sa = c * fast_sqrt0(rho2a), sb = c * fast_sqrt0(rho2b);
  const Exp2 e = xexp2(-sa, -sb);
  psia = fma(sa, fma(sa, 1.0 / 3.0, 1.0), 1.0) * e.a;
  g1a = -c23 * (1.0 + sa) * e.a;
  g2a = c23 * (c * c) * e.a;
  psib = fma(sb, fma(sb, 1.0 / 3.0, 1.0), 1.0) * e.b;
  g1b = -c23 * (1.0 + sb) * e.b;
  g2b = c23 * (c * c) * e.b;
}

// φ(z) and Φ(z) of the EI / POI rules from ONE exponential.  With u = |z|/√2 and
// E = exp(−z²/2) = exp(−u²):  φ = E/√(2π),  the tail Q = P(Z > |z|) = ½·E·erfcx(u), and
// Φ = Q (z ≤ 0) or 1 − Q (z > 0).  erfcx(u) = P(t)/(1 + 2u) with t = (u − K)/(u + K), K = 3.5,
// P a degree-23 polynomial from the Chebyshev series of (1 + 2u)·erfcx(u) on u ∈ [0, ∞)
// (tools/fit_erfcx.py, mpmath at 60 digits): max relative error 4.2e-16 over [0, 27] in fp64.
// Replaces two leaf calls (exp, erfc -- the latter with exponentials of its own) evaluated in
// sequence by two independent inline chains (the exponential and the polynomial).  Sharing E
// also makes φ + zΦ (the EI tail, where both nearly cancel) carry E's rounding as one factor.
// Not bit-identical to libm erfc; GPU-vs-oracle parity is a tolerance.
struct PhiPair {
  double phi, Phi;
};
__device__ __forceinline__ PhiPair ei_phi_Phi(double z) {
  const double u = fmin(fabs(z) * 0.7071067811865476, 40.0);   // E = 0 beyond; keeps t finite
  const double E = fexp(-0.5 * (z * z));
  // one reciprocal for both quotients: r = 1/((u + K)(1 + 2u)), t = (u − K)(1 + 2u)·r
  const double a = u + 3.5, b = fma(2.0, u, 1.0), ab = a * b;
  double r = __builtin_amdgcn_rcp(ab);
  r = fma(r, fma(-ab, r, 1.0), r);
  r = fma(r, fma(-ab, r, 1.0), r);
  const double t = (u - 3.5) * b * r, t2 = t * t;
  // even / odd halves of P(t) = Pe(t²) + t·Po(t²), each split once more (Estrin):
  // Pe = Pe_lo(t²) + t¹²·Pe_hi(t²), six-term Horner chains that run side by side (dependent depth
  // 6 instead of 11; MRBO_NO_ESTRIN: the two plain Horner chains)
#ifndef MRBO_NO_ESTRIN
  const double u2 = t2 * t2, u3 = u2 * t2, u6 = u3 * u3;   // u = t²: u⁶ = t¹²
  double pe, po;
  {
    double pe_h = sconst<0xf1ab7ccbu, 0x3dd09a8bu>();
    asm volatile("" : "+v"(pe_h));
    pe_h = fma_sc<0x73fda30du, 0x3e06db11u>(t2, pe_h);
    pe_h = fma_sc<0xf4266242u, 0xbe427e42u>(t2, pe_h);
    pe_h = fma_sc<0x1ed381c5u, 0xbe672292u>(t2, pe_h);
    pe_h = fma_sc<0xb901a919u, 0x3ec385e7u>(t2, pe_h);
    pe_h = fma_sc<0x645605dcu, 0xbf066e11u>(t2, pe_h);
    double pe_l = sconst<0xfbfa9e67u, 0x3f427e65u>();
    asm volatile("" : "+v"(pe_l));
    pe_l = fma_sc<0xc891e642u, 0xbf7143c4u>(t2, pe_l);
    pe_l = fma_sc<0xf77381b3u, 0xbfa8ff5eu>(t2, pe_l);
    pe_l = fma_sc<0x0c35056au, 0xbfbd7683u>(t2, pe_l);
    pe_l = fma_sc<0x284b1971u, 0xbf859e2cu>(t2, pe_l);
    pe_l = fma_sc<0x9a0ee914u, 0x3ff3e0a9u>(t2, pe_l);
    const double pe_ = fma(u6, pe_h, pe_l);
    pe = pe_;
    double po_h = sconst<0x617fb329u, 0xbe1406aau>();
    asm volatile("" : "+v"(po_h));
    po_h = fma_sc<0xdb5ecc9au, 0x3e4d421du>(t2, po_h);
    po_h = fma_sc<0x3786431fu, 0xbe79e096u>(t2, po_h);
    po_h = fma_sc<0xc09ddffau, 0x3ea42eb1u>(t2, po_h);
    po_h = fma_sc<0x97b263b0u, 0xbecffe87u>(t2, po_h);
    po_h = fma_sc<0x306b92a0u, 0x3ef97053u>(t2, po_h);
    double po_l = sconst<0x5777da87u, 0xbf1fda8au>();
    asm volatile("" : "+v"(po_l));
    po_l = fma_sc<0xf98105c2u, 0xbf33cf36u>(t2, po_l);
    po_l = fma_sc<0x67477473u, 0x3f938ec6u>(t2, po_l);
    po_l = fma_sc<0x6045eed1u, 0x3fb68610u>(t2, po_l);
    po_l = fma_sc<0xec6b3bb9u, 0x3fb8f702u>(t2, po_l);
    po_l = fma_sc<0x20ea5946u, 0xbfc1ebd2u>(t2, po_l);
    const double po_ = fma(u6, po_h, po_l);
    po = po_;
  }
#else
  double pe, po;
  {
    double pe_ = sconst<0xf1ab7ccbu, 0x3dd09a8bu>();
    asm volatile("" : "+v"(pe_));
    pe_ = fma_sc<0x73fda30du, 0x3e06db11u>(t2, pe_);
    pe_ = fma_sc<0xf4266242u, 0xbe427e42u>(t2, pe_);
    pe_ = fma_sc<0x1ed381c5u, 0xbe672292u>(t2, pe_);
    pe_ = fma_sc<0xb901a919u, 0x3ec385e7u>(t2, pe_);
    pe_ = fma_sc<0x645605dcu, 0xbf066e11u>(t2, pe_);
    pe_ = fma_sc<0xfbfa9e67u, 0x3f427e65u>(t2, pe_);
    pe_ = fma_sc<0xc891e642u, 0xbf7143c4u>(t2, pe_);
    pe_ = fma_sc<0xf77381b3u, 0xbfa8ff5eu>(t2, pe_);
    pe_ = fma_sc<0x0c35056au, 0xbfbd7683u>(t2, pe_);
    pe_ = fma_sc<0x284b1971u, 0xbf859e2cu>(t2, pe_);
    pe_ = fma_sc<0x9a0ee914u, 0x3ff3e0a9u>(t2, pe_);
    pe = pe_;
    double po_ = sconst<0x617fb329u, 0xbe1406aau>();
    asm volatile("" : "+v"(po_));
    po_ = fma_sc<0xdb5ecc9au, 0x3e4d421du>(t2, po_);
    po_ = fma_sc<0x3786431fu, 0xbe79e096u>(t2, po_);
    po_ = fma_sc<0xc09ddffau, 0x3ea42eb1u>(t2, po_);
    po_ = fma_sc<0x97b263b0u, 0xbecffe87u>(t2, po_);
    po_ = fma_sc<0x306b92a0u, 0x3ef97053u>(t2, po_);
    po_ = fma_sc<0x5777da87u, 0xbf1fda8au>(t2, po_);
    po_ = fma_sc<0xf98105c2u, 0xbf33cf36u>(t2, po_);
    po_ = fma_sc<0x67477473u, 0x3f938ec6u>(t2, po_);
    po_ = fma_sc<0x6045eed1u, 0x3fb68610u>(t2, po_);
    po_ = fma_sc<0xec6b3bb9u, 0x3fb8f702u>(t2, po_);
    po_ = fma_sc<0x20ea5946u, 0xbfc1ebd2u>(t2, po_);
    po = po_;
  }
#endif

  const double P = fma(t, po, pe);
  const double q = 0.5 * E * (P * (a * r));   // ½·E·erfcx(u)
  PhiPair o;
  o.phi = E * 0.3989422804014327;
  o.Phi = (z > 0.0) ? 1.0 - q : q;
  return o;
}
#ifdef MRBO_LIBM_EI   // A/B: the libm pair (two leaf calls)
__device__ __forceinline__ PhiPair ei_pp(double z) {
  PhiPair o;
  o.phi = xexp(-0.5 * (z * z)) * 0.3989422804014327;
  o.Phi = 0.5 * xerfc(-z * 0.7071067811865476);
  return o;
}
#else
__device__ __forceinline__ PhiPair ei_pp(double z) { return ei_phi_Phi(z); }
#endif

// The base decision rule g(μ, σ, θ) and the partials DecisionRule takes by ForwardDiff
// (decision_rules.jl:23-34), in closed form.
//   EI  (:84-99)   g = IΦ(z) + σφ(z), I = fmin − μ − θ, z = I/σ; zero when σ < σtol
//   POI (:101-115) g = Φ(z); zero when σ < σtol
//   LCB (:117-127) g = θσ − μ (no σtol branch)
struct EIp {
  double g, gmu, gsig, gmumu, gsigsig, gmuth, gsigth;
};
// ∂g/∂θ: −Φ (EI) and −φ/σ (POI) equal ∂g/∂μ; σ for LCB
__device__ __forceinline__ double rule_gth(int rule, double gmu, double sig) { return rule == 2 ? sig : gmu; }
enum { RULE_EI = 0, RULE_POI = 1, RULE_LCB = 2 };
__device__ __forceinline__ EIp rule_partials(int rule, double mu, double sig, double theta, double fmin,
                                             double sigma_tol, double isig) {
  EIp e;
  if (rule == RULE_LCB) {
    e.g = theta * sig - mu;
    e.gmu = -1.0;
    e.gsig = theta;
    e.gmumu = e.gsigsig = e.gmuth = 0.0;
    e.gsigth = 1.0;
    return e;
  }
  if (!(sig >= sigma_tol) && !(sig != sig)) {  // σ < σtol (NaN falls through, as in Julia)
    e.g = e.gmu = e.gsig = e.gmumu = e.gsigsig = e.gmuth = e.gsigth = 0.0;
    return e;
  }
  const double imp = fmin - mu - theta;
  const double z = imp * isig;
  const PhiPair pp = ei_pp(z);
  const double phi = pp.phi, Phi = pp.Phi;
  const double pis = phi * isig;
  if (rule == RULE_POI) {
    const double pis2 = pis * isig;
    e.g = Phi;
    e.gmu = -pis;
    e.gsig = -z * pis;
    e.gmumu = -z * pis2;
    e.gsigsig = z * (2.0 - z * z) * pis2;
    e.gmuth = -z * pis2;
    e.gsigth = (1.0 - z * z) * pis2;
    return e;
  }
  e.g = imp * Phi + sig * phi;
  e.gmu = -Phi;
  e.gsig = phi;
  e.gmumu = pis;
  e.gsigsig = z * z * pis;
  e.gmuth = pis;
  e.gsigth = z * pis;
  return e;
}
__device__ __forceinline__ EIp rule_partials(int rule, double mu, double sig, double theta, double fmin,
                                             double sigma_tol) {
  return rule_partials(rule, mu, sig, theta, fmin, sigma_tol, 1.0 / sig);
}
// first partials only, at (μ', σ') -- the perturbation "second-order" coefficients (Q7, Q8)
__device__ __forceinline__ void rule_first(int rule, double mu, double sig, double theta, double fmin, double sigma_tol,
                                           double& gmu, double& gsig) {
  const EIp e = rule_partials(rule, mu, sig, theta, fmin, sigma_tol);
  gmu = e.gmu;
  gsig = e.gsig;
}

// c(x) and ∇c(x) of the cost model (lane-uniform; D compile-time).  Hc = diag(hd) + β v vᵀ:
// QUADRATIC hd_a = 2w_a/del_a², β = 0; LOGLINEAR hd = 0, β = c, v_a = w_a/del_a.
template <int D>
__device__ __forceinline__ double cost_eval(const KParams& kp, const double (&x)[D], double (&gc)[D]) {
  const double* lb = kp.cost_tab;
  const double* del = kp.cost_tab + D;
  const double* w = kp.cost_tab + 2 * D;
  if (kp.cost == COST_QUADRATIC) {
    double c = kp.cost_c0;
#pragma unroll
    for (int a = 0; a < D; ++a) {
      const double u = (x[a] - lb[a]) / del[a];
      c = fma(w[a] * u, u, c);
      gc[a] = 2.0 * w[a] * u / del[a];
    }
    return c;
  }
  double t = 0.0;
#pragma unroll
  for (int a = 0; a < D; ++a) t = fma(w[a], (x[a] - lb[a]) / del[a], t);
  const double c = kp.cost_c0 * xexp(t);
#pragma unroll
  for (int a = 0; a < D; ++a) gc[a] = c * (w[a] / del[a]);
  return c;
}
// entry (a, b) of Hc at cost c (d = D)
template <int D>
__device__ __forceinline__ double cost_hess(const KParams& kp, double c, int a, int b) {
  const double* del = kp.cost_tab + D;
  const double* w = kp.cost_tab + 2 * D;
  if (kp.cost == COST_QUADRATIC) return (a == b) ? 2.0 * w[a] / (del[a] * del[a]) : 0.0;
  return c * (w[a] / del[a]) * (w[b] / del[b]);
}

// counter-based uniform (bit-identical to the host / oracle version)
__host__ __device__ __forceinline__ unsigned long long splitmix64(unsigned long long z) {
  z += 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}
__host__ __device__ __forceinline__ unsigned long long dual_key0(unsigned long long seed) {
  return splitmix64(seed ^ 0x5851F42D4C957F2DULL);
}
// the same from the seed's first key (dual_key0), which the kernel keeps in LDS
__host__ __device__ __forceinline__ double dual_uniform_k(unsigned long long key0, long long traj, int j, int k) {
  unsigned long long key = splitmix64(key0 ^ (unsigned long long)traj);
  key = splitmix64(key ^ (((unsigned long long)(unsigned)j << 32) | (unsigned)k));
  return (double)(key >> 11) * (1.0 / 9007199254740992.0);
}
__host__ __device__ __forceinline__ double dual_uniform(unsigned long long seed, long long traj, int j, int k) {
  return dual_uniform_k(dual_key0(seed), traj, j, k);
}

// value of a double in lane k (wave-uniform k)
__device__ __forceinline__ double readlane_d(double v, int k) {
  int lo, hi;
  dsplit(v, lo, hi);
  return djoin(__builtin_amdgcn_readlane(lo, k), __builtin_amdgcn_readlane(hi, k));
}

__device__ __forceinline__ double clampd(double v, double lo, double hi) { return v < lo ? lo : (v > hi ? hi : v); }

}  // namespace mrbo
