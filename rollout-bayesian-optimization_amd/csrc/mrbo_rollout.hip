// mrbo_rollout.hip -- the MI355X rollout-trajectory kernel (forward rollout + adjoint).
//
// Restates, for one wavefront per trajectory:
//   rollout!              rollout.jl:39-74        (draw at x0, h × [inner solve, draw, condition!])
//   gp_draw / observable  radial_basis_surrogates.jl:588-611, observables.jl:106-121
//   condition!            radial_basis_surrogates.jl:431-441 (rank-1 append; inverse-factor row)
//   eval(fs, x, θ)        radial_basis_surrogates.jl:482-581 (μ, σ, ∇, H of EI; no μσ term, Q11)
//   multistart solve      rbf_optim.jl:1-101 (deterministic projected Newton)
//   resolve               rollout.jl:108-111 (fmini over the capacity buffer, Q3)
//   gradient(T)           rollout.jl:126-277 (adjoint back-substitution, sparse δK)
// Numerics follow the reference formulas; the triangular solves use the explicit inverse
// factor L⁻¹ = [[L0⁻¹,0],[E,Dinv]] instead of substitution (same maths, fp64).
#include <utility>

#include "mrbo_device.h"
#ifdef MRBO_BCAST_HEADER   // A/B: an alternative generated header (tools/gen_bcast_asm.py BCAST_OUT=…)
#include MRBO_BCAST_HEADER
#else
#include "bcast_asm.h"
#endif

#ifndef MRBO_WAVES_PER_SIMD
#define MRBO_WAVES_PER_SIMD 2
#endif
#ifndef MRBO_HESS16   // 1: the Hessian reduction's tail chunk as a 16-value reduction (A/B)
#define MRBO_HESS16 0
#endif
// Everything below is compiled per fantasy capacity FMAX (-DMRBO_FMAX, default 6 = h ≤ 5; the
// kernel units are also built with FMAX = 4 for h ≤ 3): an inline namespace per FMAX keeps the
// two builds' kernels and helpers distinct symbols in one library.
#define MRBO_FNS_CAT_(a, b) a##b
#define MRBO_FNS_CAT(a, b) MRBO_FNS_CAT_(a, b)
#define MRBO_FNS MRBO_FNS_CAT(fmax, MRBO_FMAX)
#ifndef MRBO_WAVES_PER_SIMD_GL   // N ≤ 256 (L2-fed layout): 512 registers per wave at 1
#define MRBO_WAVES_PER_SIMD_GL 1
#endif

namespace mrbo {
inline namespace MRBO_FNS {

constexpr double PAD_FAR = 1e100;   // coordinate of padded data rows (WaveCtx::rowv)

// MRBO_SQ_EAGER (A/B, not the default): the eager all-column value pass of the square layout
// (Lay::SQ_EAGER).  Measured neutral (C3 −0.3 %, C3-MLE +0.2 %, within the spread) while it issues
// 4 % more VALU per wave: about half of C3's non-batched value passes are NOT followed by a GRADC
// pass (the iteration converges on x_tol / f_tol after an accepted trial), and their extra columns
// are wasted work.
#ifdef MRBO_SQ_EAGER
constexpr bool SQ_EAGER_ON = true;
#else
constexpr bool SQ_EAGER_ON = false;
#endif

template <int D, int RPL, int HW = 1>
struct Lay {
  static constexpr int D1 = D + 1;
  static constexpr int BS = (D1 + 1) & ~1;         // B row stride in doubles (16-B aligned rows)
  static constexpr int NR = RPL * WAVE;            // base-row capacity (global arrays: X0, c0, tables)
  // half-wave mode (HW = 2, N ≤ 32, RPL = 1): two trajectories per wave, lanes 32h..32h+31 own
  // trajectory h; LANES lanes per trajectory, NRL rows of per-trajectory LDS state (E, C, G12)
  static constexpr int LANES = WAVE / HW;
  static constexpr int NRL = RPL * LANES;
  // L0⁻¹ layout (see LINV_DOUBLES below).  BC: register-broadcast triangular products over
  // square 64×64 blocks of L0⁻¹ in LDS (RPL = 1: one block; RPL = 2: the three blocks of the
  // lower block triangle), which also moves the base kernel rows out of LDS.  SQ (RPL = 1)
  // additionally keeps the per-wave E / C rows and the start tables in LDS.
  static constexpr bool SQ = (RPL == 1);
  static constexpr bool BC = (RPL <= 2);
  static constexpr int FR0 = 0;                    // first fantasy row in B (base rows stay in registers)
  static constexpr int BROWS = FR0 + FMAX;         // [base rows +] fantasy rows
  static constexpr int NG = D1 * (D1 + 1) / 2;     // Gram entries (a ≤ b)
  static constexpr int NH = D * (D + 1) / 2;       // Hessian entries (a ≤ b)
  // reduction-total layout
  static constexpr int R_VAL = 0;                  // [vv, μ0, E_r·B0 (r<FMAX)]  (8)
  static constexpr int R_G = 8;                    // Gram entries 1..NG-1
  static constexpr int NGC = (NG - 1 + 15) / 16;   // G chunks
  static constexpr int R_MF = R_G + 16 * NGC;      // [c·∇k (D), E_r·∇k (D each)]
  static constexpr int NMF = D * (1 + FMAX);
  static constexpr int NMFC = (NMF + 15) / 16;
  static constexpr int NPAIR = D * D + 2 * D;      // adjoint pair products
  static constexpr int NPC = (NPAIR + 15) / 16;
  static constexpr int NHC = (NH + 1 + 15) / 16;
  static constexpr int REDN_A = R_MF + 16 * NMFC;
  static constexpr int REDN_B = 16 * (NPC > NHC ? NPC : NHC);
  static constexpr int REDN = ((REDN_A > REDN_B ? REDN_A : REDN_B) + 1) & ~1;
  // lane-uniform LDS area (doubles)
  static constexpr int U_X = 0;                          // eval point            D
  static constexpr int DE = (D + 1) & ~1;               // D rounded up to an even count
  static constexpr int U_XB = U_X + (DE > 8 ? DE : 8);   // best multistart point D
  static constexpr int U_XF = U_XB + (DE > 8 ? DE : 8);  // fantasy points        FMAX*D
  static constexpr int U_YF = U_XF + FMAX * D;           // fantasy observations  FMAX
  static constexpr int U_GF = U_YF + FMAX;               // sampled gradients     FMAX*D
  static constexpr int U_DINV = U_GF + FMAX * D;         // Dinv row-major        FMAX*FMAX
  static constexpr int U_CF = U_DINV + FMAX * FMAX;      // fantasy coeffs/surf.  (FMAX+1)*FMAX
  static constexpr int U_FMIN = U_CF + (FMAX + 1) * FMAX;// fmin per surface      FMAX+1
  static constexpr int U_SC = U_FMIN + FMAX + 1;         // scalars: μ,σ,α,G00,σ²,... 20
  static constexpr int U_GMU = U_SC + 20;                // ∇μ   D
  static constexpr int U_GSIG = U_GMU + D;               // ∇σ   D
  static constexpr int U_GAL = U_GSIG + D;               // ∇α   D
  static constexpr int U_MIX = U_GAL + D;                // d2α/dxdθ D
  static constexpr int U_G = U_MIX + D;                  // Gram D1×D1
  static constexpr int U_H = U_G + D1 * D1;              // Hα   D×D
  static constexpr int U_YFV = U_H + D * D;              // Yf   FMAX×D1
  static constexpr int U_WF = U_YFV + FMAX * D1;         // w_f  FMAX
  static constexpr int U_PF = U_WF + FMAX;               // P_f  FMAX×D
  static constexpr int U_GMU0 = U_PF + FMAX * D;         // ∇μ(x0) on the base surface  D
  static constexpr int U_XBAR = U_GMU0 + D;              // x̄_j  FMAX×D
  static constexpr int U_ACC = U_XBAR + FMAX * D;        // Σ dri' x̄  FMAX×D
  static constexpr int U_YBAR = U_ACC + FMAX * D;        // ȳ_j  FMAX+1
  static constexpr int U_DX = U_YBAR + FMAX + 1;         // δx    D
  static constexpr int U_NX = U_DX + D;                  // Newton iterate x      D
  static constexpr int U_NG = U_NX + D;                  // Newton gradient -∇α   D
  static constexpr int U_NP = U_NG + D;                  // Newton direction p    D
  static constexpr int U_LB = U_NP + D;                  // box lower bounds      D
  static constexpr int U_UB = U_LB + D;                  // box upper bounds      D
  static constexpr int U_HF = U_UB + D;                  // fantasy rows: [x - X_r (D), g1, g2]  FMAX×(D+2)
  static constexpr int U_STAMP = U_HF + FMAX * (D + 2);   // cycle accumulators (MRBO_STAMPS)
  static constexpr int U_KC = U_STAMP + NSTAMP_SLOTS;             // launch constants (KC_*), see wave_setup
  static constexpr int U_SIZE = ((U_KC + 15) + 1) & ~1;
  static constexpr int G12 = 3 * NRL;                    // per-lane [g1, g2, Y0] of the base rows
  static constexpr int EC = SQ ? (2 * FMAX + 1) * NRL : 0;  // E (FMAX×NRL) + C ((FMAX+1)×NRL) in LDS
  // SQ_EAGER (the square layout of the FMAX = 4 units, full-wave): the value pass runs all D1
  // columns of the forward product and stashes columns 1..d here for the GRADC pass that follows
  static constexpr bool SQ_EAGER = SQ_EAGER_ON && SQ && HW == 1 && FMAX <= 4;
  static constexpr int STASH = SQ_EAGER ? D * NRL : 0;
  static constexpr int WAVE_LDS = BROWS * BS + REDN + U_SIZE + G12 + EC + STASH;
  // L0⁻¹ in LDS, shared by the waves of a workgroup.  BC: dense zero-padded 64×64 blocks,
  // column-major with odd leading dimension LD = 65, so the column walk (forward product,
  // lane i reads [i][j]) and the row walk (backward product, lane i reads [k][i]) are both
  // bank-conflict free and neither needs a triangle mask.  RPL = 2 stores the blocks (0,0),
  // (1,0), (1,1) of the block triangle (block (s,t) holds rows 64s.., columns 64t..; the
  // all-zero block (0,1) is skipped), 99.8 KB.
  static constexpr int LD = WAVE + 1;
  static constexpr int NBLK = RPL * (RPL + 1) / 2;
  static constexpr int BLK = WAVE * LD;            // doubles per block
  __host__ __device__ static constexpr int blk(int s, int t) { return s * (s + 1) / 2 + t; }   // t ≤ s
  // RPL > 2 (N ≤ 256): L0⁻¹ does not fit in LDS next to the wave areas (263 KB packed); it stays
  // in global memory (L2-resident, shared by every wave of the XCD) as two packed copies --
  // by columns for the forward product, by rows for the backward one -- so that both row walks
  // are coalesced 512-byte loads
  static constexpr bool GL = (RPL > 2);
  // GL with RPL = 4: NLB of the ten blocks (gl_lds_slot, mrbo_device.h) also live in workgroup LDS
  // in the BC layout, shared by the workgroup's waves and read by the LDS register broadcast
  // instead of from L2 (both directions, as the BC layout); the others stay L2-fed
  static constexpr int NLB = (GL && RPL == 4) ? GL_LDS_BLOCKS : 0;
  static constexpr long long LINV_DOUBLES = GL ? (long long)NLB * BLK : (((BC ? (long long)NBLK * BLK : linv_size(NR)) + 1) & ~1LL);
  // device image; GL: the NBLK blocks twice, 64×64 each with the lane index fastest -- forward
  // copy (i, j) at j·64 + i, backward copy (k, i) at k·64 + i -- zero-padded
  static constexpr long long LINV_GLOBAL = GL ? 2LL * NBLK * WAVE * WAVE + (long long)NLB * BLK : LINV_DOUBLES;
  // where the LDS staging copy starts in the device image (GL: after the two global copies)
  static constexpr long long LINV_LDS_SRC = GL ? 2LL * NBLK * WAVE * WAVE : 0;
};
// scalar slots in U_SC
enum { SC_MU = 0, SC_SIG = 1, SC_ALPHA = 2, SC_G00 = 3, SC_VAR = 4, SC_GMU = 5, SC_GSIG = 6, SC_GMUMU = 7,
       SC_GSIGSIG = 8, SC_GMUTH = 9, SC_GSIGTH = 10, SC_FMIN = 11, SC_ST = 12, SC_CABS = 13,
       // NonUniformCost (kp.cost): the rule value g before weighting, c(x), max_a |∂_a c(x)|
       SC_ARAW = 14, SC_COSTC = 15, SC_GCMAX = 16,
       SC_ISIG = 17,     // 1/σ
       SC_FREE = 18 };   // free set of the last projected-gradient test (bit a: coordinate a free)

// Launch constants the trajectory code reads in its loops, copied into each wave's lane-uniform
// LDS at wave_setup: read back with ds_read at the point of use instead of being held in SGPRs
// for the whole kernel, where they overflowed the 102-SGPR budget and were spilled to VGPR lanes
// (a v_readlane per reload, on the VALU).  Branch conditions keep the kernel-argument copy.
enum { KC_PSI0 = 0, KC_D2PSI0 = 1, KC_THETA = 2, KC_SIGTOL = 3, KC_GTOL = 4, KC_GCMU = 5, KC_GCSIG = 6,
       KC_GCD2 = 7, KC_XTOL = 8, KC_FTOL = 9, KC_HTOL = 10, KC_SN2 = 11,
       KC_BOX = 12,     // max_a (ub_a − lb_a): the Newton step's length cap
       KC_FMINB = 13,   // fmin of the base surrogate (each trajectory's surface −1)
       KC_DXKEY = 14 }; // splitmix64(seed ^ C): the δx counter RNG's first key (bits of a double)
#define KCV(F) (W.U[Lay<D, RPL, HW>::U_KC + KC_##F])

// ∂_lane c(x) by unrolled select (lane < D; a runtime index would put gc in scratch)
template <int D>
__device__ __forceinline__ double lane_pick(const double (&v)[D], int lane) {
  double r = 0.0;
#pragma unroll
  for (int a = 0; a < D; ++a) r = (a == lane) ? v[a] : r;
  return r;
}

// Per-workgroup LDS after L0⁻¹: [xstarts (d×nstarts)] [kxb (NR×nstarts)] [gtab (nstarts×NG)],
// each rounded to an even number of doubles; then the per-wave areas.  gtab[k] is the base
// Gram of start k, (L0⁻¹B)ᵀ(L0⁻¹B) with B = [kx, ∇kx](x_k), upper triangle row-major; its
// entry 0 is |L0⁻¹kx(x_k)|².
template <int D, int RPL, int HW = 1>
struct WgTables {
  long long xs, kxb, gtab, end;   // offsets in doubles from smem
  __device__ __forceinline__ WgTables(const KParams& kp) {
    using Ly = Lay<D, RPL, HW>;
    xs = Ly::LINV_DOUBLES;
    const long long nxs = kp.xs_lds ? (((long long)kp.nstarts * D + 1) & ~1LL) : 0;
    kxb = xs + nxs;
    const bool lt = Ly::SQ && kp.batch;   // packed layouts keep the start tables in global memory
    const long long nk = lt ? (((long long)Ly::NR * kp.nstarts + 1) & ~1LL) : 0;
    gtab = kxb + nk;
    end = gtab + (lt ? (((long long)kp.nstarts * Ly::NG + 1) & ~1LL) : 0);
  }
};

template <int D, int RPL, int HW = 1>
struct WaveCtx {
  using Ly = Lay<D, RPL, HW>;
  int lane;             // lane within the trajectory's lanes (0..LANES-1)
  int half;             // HW = 2: which half of the wave (its trajectory); 0 otherwise
  double* B;            // LDS: BROWS × BS
  double* red;          // LDS: REDN
  double* U;            // LDS: U_SIZE
  const double* Linv;   // L0⁻¹: LDS blocks (BC) or the forward copy of the global blocks (GL)
  const double* LinvT;  // GL: the backward copy of the global L0⁻¹ blocks
  const double* LinvL;  // GL: the LDS-resident blocks (Lay::NLB of them, BC layout), or null
  const double* XS;     // inner-solve start points: LDS copy (kp.xs_lds) or kp.xstarts
  const double* KXB;    // ψ(|clamp(x_k) − X_i|) (kp.batch): LDS [NR][nstarts]; packed layouts: global [nstarts][NR]
  const double* GTAB;   // [nstarts][NG]: base Gram of the start points (kp.batch; LDS, global for packed)
  const double* YTAB;   // global [nstarts][NR]: this workgroup's Y0(x_k) = L0⁻¹kx(x_k) (kp.batch)
  double* G12;          // LDS: per-lane [g1, g2, Y0] of the base rows (GRAD / FULL / RICH)
  double* E;            // LDS (SQ) or global: FMAX × NR  inverse-factor fantasy rows (base columns)
  double* C;            // LDS (SQ) or global: (FMAX+1) × NR  base part of c for surfaces -1..h
  double* SUMS;         // packed layouts: global [64][8] per-start sums of the batched start pass
  double* STASH;        // L2-fed layouts (GL): global [RPL][D][64] gradient columns of the last value pass
  double X0[RPL][D];    // own base rows
  bool valid[RPL];
  int N, Npad;
  Radial rad;
  unsigned long long tlast;
  // Does row slot s hold a data point?  Padded rows (i ≥ N) sit at X0 = PAD_FAR (wave_setup), where
  // every non-periodic radial function and both derivative factors are exactly 0 (exp underflows),
  // and their c, w, E, P entries are 0 as well -- so for those kernels no select is needed: true at
  // compile time in the Matérn-5/2 specialisation.  The Periodic kernel keeps the per-row mask.
  // base covariate a of row slot s.  MRBO_X0_GLOBAL (A/B, N ≤ 256 layout): read from the L2-resident
  // device copy at each use instead of holding 4·d registers per lane across the trajectory
  __device__ __forceinline__ double x0(const KParams& kp, int s, int a) const {
#ifdef MRBO_X0_GLOBAL
    if constexpr (Ly::GL) {
      const double v = kp.X0[(long long)a * Ly::NR + lane + WAVE * s];
#ifndef MRBO_NO_PAD_FAR
      return (valid[s] || kp.kernel == KERNEL_PERIODIC) ? v : PAD_FAR;
#else
      return v;
#endif
    }
#endif
    return X0[s][a];
  }
  __device__ __forceinline__ bool rowv(const KParams& kp, int s) const {
#ifdef MRBO_NO_PAD_FAR
    return valid[s];
#else
    return kp.kernel != KERNEL_PERIODIC ? true : valid[s];
#endif
  }
  // opaque lane index (see evaluate): per-lane addresses are rematerialised where used
  __device__ __forceinline__ int ln() const {
    int l = lane;
    asm volatile("" : "+v"(l));
    return l;
  }
};

// ---- cross-lane primitives of one trajectory's lanes ----------------------------------------
// HW = 1: the whole wave.  HW = 2 (half-wave mode): the 32-lane half holding the trajectory -- its
// reductions stop at lane bit 4, its ballots are its 32 bits, lane k of a half is lane k + 32·half
template <int HW, int K>
__device__ __forceinline__ void hw_reduce(double (&v)[K], double* red, int lane) {
  if constexpr (HW == 1) wave_reduce<K>(v, red, lane);
  else half_reduce<K>(v, red, lane);
}
template <int HW>
__device__ __forceinline__ double hw_allreduce1(double v) {
  if constexpr (HW == 1) {
    return wave_allreduce1(v);
  } else {
    v = fold_all<16>(v);
    v = fold_all<8>(v);
    v = fold_all<4>(v);
    v = fold_all<2>(v);
    return fold_all<1>(v);
  }
}
template <int HW>
__device__ __forceinline__ unsigned long long hw_ballot(bool c, int half) {
  const unsigned long long m = __ballot(c);
  if constexpr (HW == 1) return m;
  else return half ? (m >> 32) : (m & 0xffffffffull);
}
// value of lane k (k a compile-time or wave-uniform index) of this trajectory's lanes
template <int HW>
__device__ __forceinline__ double hw_readlane_d(double v, int k, int half) {
  if constexpr (HW == 1) {
    return readlane_d(v, k);
  } else {
    const double a = readlane_d(v, k), b = readlane_d(v, k + 32);
    return half ? b : a;
  }
}
template <int HW>
__device__ __forceinline__ int hw_readlane_i(int v, int k, int half) {
  if constexpr (HW == 1) {
    return __builtin_amdgcn_readlane(v, k);
  } else {
    const int a = __builtin_amdgcn_readlane(v, k), b = __builtin_amdgcn_readlane(v, k + 32);
    return half ? b : a;
  }
}
// value of lane k of this trajectory's lanes for a per-trajectory (HW = 2: per-half, divergent) k
template <int HW>
__device__ __forceinline__ double hw_lane_d(double v, int k, int half) {
  if constexpr (HW == 1) return readlane_d(v, k);
  else return __shfl(v, k + 32 * half, WAVE);
}

// work counters per trajectory (NCOUNT, mrbo_device.h)
struct Counters {
  int grad = 0, value = 0, hess = 0, rich = 0, pairs = 0;
};

// Optional per-phase cycle accounting (build with -DMRBO_STAMPS): STAMP(W, k) charges the
// s_memtime ticks since the previous stamp to region k (accumulated by lane 0 in LDS, summed
// into kp.stamps at kernel exit).  Regions: see mrbo_api.hip stamp_names.
#ifdef MRBO_STAMPS
#define STAMP(W, k) stamp_region(W, k)
#else
#define STAMP(W, k) ((void)0)
#endif

// Per-lane results of an evaluation that later phases (conditioning, adjoint) need.
template <int D, int RPL, int HW = 1>
struct LaneRes {
  double w[RPL];
  double P[RPL][D];
  double cb[RPL];
};

#ifdef MRBO_STAMPS
template <int D, int RPL, int HW>
__device__ __forceinline__ void stamp_count(WaveCtx<D, RPL, HW>& W, int k, unsigned long long v) {
  if (W.lane == 0) reinterpret_cast<unsigned long long*>(W.U + Lay<D, RPL, HW>::U_STAMP)[k] += v;
}
template <int D, int RPL, int HW>
__device__ __forceinline__ void stamp_region(WaveCtx<D, RPL, HW>& W, int k) {
  const unsigned long long now = __builtin_amdgcn_s_memtime();
  if (W.lane == 0) reinterpret_cast<unsigned long long*>(W.U + Lay<D, RPL, HW>::U_STAMP)[k] += now - W.tlast;
  W.tlast = now;
}
#endif

// ---- register-broadcast triangular products (RPL == 1) -----------------------------------
// acc[c] += Σ_j L(j) · V[j][c], where row j of V lives in lane j's registers (the kernel rows
// B for the forward product, Y for the backward one) and L(j) is this lane's L0⁻¹ entry.
// Two permlane swaps replicate 16-row block b of V into every 16-lane row (lane t holds row
// 16b + t); v_fmac_f64 with DPP row_newbcast:n then broadcasts row 16b + n inside each row,
// fused into the FMA (bcast_asm.h: one software-pipelined asm statement per block).  V never goes through LDS: the only LDS traffic is one ds_read_b64 of
// L0⁻¹ per step (the row broadcast through LDS cost 8× that and bounded the whole loop).

// LDS byte address of a pointer into the dynamic shared array
__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

// acc[c] += Σ_{j < nrows} L(j) v[c](j) with L(j) = lbase[j · JSTRIDE] (zero-padded past N).
// Blocks run in the order 0, 2, 1, 3 (two swaps yield blocks p and p+2 together).
// Column chunks of at most 8 (the generated asm statements cover K ≤ 9; d > 8 runs 2-3 chunks,
// each re-reading this lane's L0⁻¹ entries)
template <int K>
__device__ __forceinline__ double (&head8(double (&a)[K]))[8] { return *reinterpret_cast<double(*)[8]>(&a[0]); }
template <int K>
__device__ __forceinline__ double (&tail8(double (&a)[K]))[K - 8] { return *reinterpret_cast<double(*)[K - 8]>(&a[8]); }
template <int K>
__device__ __forceinline__ const double (&head8(const double (&a)[K]))[8] {
  return *reinterpret_cast<const double(*)[8]>(&a[0]);
}
template <int K>
__device__ __forceinline__ const double (&tail8(const double (&a)[K]))[K - 8] {
  return *reinterpret_cast<const double(*)[K - 8]>(&a[8]);
}

// One 16-step block of a register-broadcast product.  MRBO_K1_SPLIT: K = 1 (the value product
// L0⁻¹kx and the backward w = L0⁻ᵀY0) with two accumulators over the even and odd steps -- measured
// 0.6 % SLOWER on C3 (round 5: the chain is not what the product waits on), so off by default.
template <int K, int STRIDE>
__device__ __forceinline__ void bcast_run(double (&acc)[K], const double (&bq)[K], unsigned addr) {
#ifdef MRBO_K1_SPLIT
  if constexpr (K == 1) {
    BcastAsmSplit<STRIDE>::run(acc, bq, addr);
    return;
  }
#endif
  BcastAsm<K, STRIDE>::run(acc, bq, addr);
}

// COPY: the row replication's operand copies as v_mov_b64 (self_swap); false for the 512-register
// L2-fed kernels' LDS-resident blocks (gl_block), where they cost spills
template <int K, int JSTRIDE, int HW = 1, bool COPY = true>
__device__ __forceinline__ void bcast_product_k(double (&acc)[K], const double (&v)[K], const double* lbase, int nrows) {
  const unsigned a0 = lds_addr(lbase);
  if constexpr (HW == 2) {
    // half-wave mode (N ≤ 32): each half holds its trajectory's rows 0..31 in DPP rows 2h, 2h+1,
    // so ONE v_permlane16_swap per dword yields block 0 of both halves ([r0 r0 r2 r2]) and block 1
    // ([r1 r1 r3 r3]); no swap crosses the halves
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      if (16 * p >= nrows) break;
      double bp[K];
#pragma unroll
      for (int c = 0; c < K; ++c) {
        double b0, b1;
        self_swap<16, true>(v[c], b0, b1);
        bp[c] = p == 0 ? b0 : b1;
      }
      bcast_run<K, 8 * JSTRIDE>(acc, bp, a0 + 8u * 16u * p * JSTRIDE);
    }
    return;
  }
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    if (16 * p >= nrows) break;
    double bp[K], bp2[K];
#pragma unroll
    for (int c = 0; c < K; ++c) {
      if (p == 0) row_blocks<0, COPY>(v[c], bp[c], bp2[c]);
      else row_blocks<1, COPY>(v[c], bp[c], bp2[c]);
    }
    bcast_run<K, 8 * JSTRIDE>(acc, bp, a0 + 8u * 16u * p * JSTRIDE);
    if (16 * (p + 2) < nrows) bcast_run<K, 8 * JSTRIDE>(acc, bp2, a0 + 8u * 16u * (p + 2) * JSTRIDE);
  }
}

template <int K, int JSTRIDE, int HW = 1, bool COPY = true>
__device__ __forceinline__ void bcast_product(double (&acc)[K], const double (&v)[K], const double* lbase, int nrows) {
  if constexpr (K > 9) {
    bcast_product<8, JSTRIDE, HW, COPY>(head8(acc), head8(v), lbase, nrows);
    bcast_product<K - 8, JSTRIDE, HW, COPY>(tail8(acc), tail8(v), lbase, nrows);
  } else {
    bcast_product_k<K, JSTRIDE, HW, COPY>(acc, v, lbase, nrows);
  }
}

// ---- folded triangular products (RPL = 1, N > 48) ------------------------------------------
// L0⁻¹ is lower triangular, so DPP row q (lanes 16q..16q+15, output rows 16q..16q+15) needs only
// the row blocks b ≤ q of the forward product and b ≥ q of the backward one: 10 of the 16
// (row, block) pairs the four unfolded 16-step passes issue.  Three passes cover them: two plain
// passes (forward blocks 0, 1; backward blocks 3, 2), then one pass in which a row that is already
// finished works for another -- forward: row 1 takes block 3 of output rows 48.. (row 3's last
// block), rows 2, 3 their block 2; backward: row 2 takes block 0 of output rows 0.. (row 0's last
// block), rows 0, 1 their block 1 -- into a second accumulator f.  v_permlane32_swap then moves
// the helper's partial sums by 32 lanes (row 1 ↔ row 3, row 2 ↔ row 0) beside the rows' own, and
// two adds finish: 48 steps instead of 64.  The lanes of the idle row read one zero of the upper
// triangle (a broadcast address on the bank half the helper row does not use), so their f is 0
// and every read of the third pass is conflict-free.  The caller passes the LD = 65 square block.
template <int K>
__device__ __forceinline__ void fold_finish(double (&acc)[K], const double (&f)[K], bool fwd) {
#pragma unroll
  for (int c = 0; c < K; ++c) {
    int lo, hi;
    dsplit(f[c], lo, hi);
    // forward: swap(vdst = 0, f) -> [0 0 f0 f1] and [0 0 f2 f3] (f0 = 0);
    // backward: swap(vdst = f, 0) -> [f0 f1 0 0] and [f2 f3 0 0] (f3 = 0)
    const auto l = fwd ? __builtin_amdgcn_permlane32_swap(0, lo, false, false)
                       : __builtin_amdgcn_permlane32_swap(lo, 0, false, false);
    const auto h = fwd ? __builtin_amdgcn_permlane32_swap(0, hi, false, false)
                       : __builtin_amdgcn_permlane32_swap(hi, 0, false, false);
    acc[c] += djoin(l[0], h[0]);
    acc[c] += djoin(l[1], h[1]);
  }
}

// forward: acc[c] += Σ_{j ≤ i} L(i, j) v[c](j), L(i, j) at Lsq[j·65 + i]
template <int K>
__device__ __forceinline__ void bcast_fold_fwd_k(double (&acc)[K], const double (&v)[K], const double* Lsq, int lane) {
  constexpr unsigned LD = WAVE + 1;
  const unsigned a0 = lds_addr(Lsq + lane);
  const int q = lane >> 4;
  double b0[K], b1[K], m[K], f[K];
#pragma unroll
  for (int c = 0; c < K; ++c) {
#ifdef MRBO_FOLD_SELECT   // round-5 first form: all four blocks, then a per-row select
    double b2, b3;
    row_blocks4<true>(v[c], b0[c], b1[c], b2, b3);
    m[c] = (q == 1) ? b3 : b2;
#else
    fold_blocks(v[c], true, b0[c], b1[c], m[c]);
#endif
    f[c] = 0.0;
  }
  // row 1: (48 + t, 48 + n) = own address + 32 + 16·LD; row 0: the zeros (15, 33 + n); rows 2, 3: block 2
  const unsigned a3 = (q == 1) ? a0 + 8u * (48u * LD + 32u) : (q == 0) ? lds_addr(Lsq + 33 * LD + 15) : a0 + 8u * 32u * LD;
#ifdef MRBO_FOLD3_MERGED   // A/B: +1.2 % on C3 (round 5), so off
  if constexpr (K == 1) {   // the three passes in one software-pipelined statement
    BcastAsm3<8 * LD>::run(acc, f, b0, b1, m, a0, a3);
  } else
#endif
  {
    bcast_run<K, 8 * LD>(acc, b0, a0);
    bcast_run<K, 8 * LD>(acc, b1, a0 + 8u * 16u * LD);
    bcast_run<K, 8 * LD>(f, m, a3);
  }
  fold_finish<K>(acc, f, true);
}

// backward: acc[c] += Σ_{k ≥ i} L(k, i) v[c](k), L(k, i) at Lsq[i·65 + k]
template <int K>
__device__ __forceinline__ void bcast_fold_bwd_k(double (&acc)[K], const double (&v)[K], const double* Lsq, int lane) {
  constexpr unsigned LD = WAVE + 1;
  const unsigned a0 = lds_addr(Lsq + lane * LD);
  const int q = lane >> 4;
  double b2[K], b3[K], m[K], f[K];
#pragma unroll
  for (int c = 0; c < K; ++c) {
#ifdef MRBO_FOLD_SELECT
    double b0, b1;
    row_blocks4<true>(v[c], b0, b1, b2[c], b3[c]);
    m[c] = (q == 2) ? b0 : b1;
#else
    fold_blocks(v[c], false, b2[c], b3[c], m[c]);
#endif
    f[c] = 0.0;
  }
  // row 2: (n, t) of output row t = lane − 32; row 3: the zeros (17 + n, 63); rows 0, 1: block 1
  const unsigned a3 = (q == 2) ? lds_addr(Lsq + (lane - 32) * LD) : (q == 3) ? lds_addr(Lsq + 63 * LD + 17) : a0 + 8u * 16u;
#ifdef MRBO_FOLD3_MERGED
  if constexpr (K == 1) {   // blocks 2 then 3 (at +16 steps), then the folded pass, in one statement
    BcastAsm3<8>::run(acc, f, b2, b3, m, a0 + 8u * 32u, a3);
  } else
#endif
  {
    bcast_run<K, 8>(acc, b3, a0 + 8u * 48u);
    bcast_run<K, 8>(acc, b2, a0 + 8u * 32u);
    bcast_run<K, 8>(f, m, a3);
  }
  fold_finish<K>(acc, f, false);
}

// column chunks of at most 8 beyond K = 9 (the generated asm statements), as bcast_product
template <int K>
__device__ __forceinline__ void bcast_fold_fwd(double (&acc)[K], const double (&v)[K], const double* Lsq, int lane) {
  if constexpr (K > 9) {
    bcast_fold_fwd<8>(head8(acc), head8(v), Lsq, lane);
    bcast_fold_fwd<K - 8>(tail8(acc), tail8(v), Lsq, lane);
  } else {
    bcast_fold_fwd_k<K>(acc, v, Lsq, lane);
  }
}
template <int K>
__device__ __forceinline__ void bcast_fold_bwd(double (&acc)[K], const double (&v)[K], const double* Lsq, int lane) {
  if constexpr (K > 9) {
    bcast_fold_bwd<8>(head8(acc), head8(v), Lsq, lane);
    bcast_fold_bwd<K - 8>(tail8(acc), tail8(v), Lsq, lane);
  } else {
    bcast_fold_bwd_k<K>(acc, v, Lsq, lane);
  }
}

// Sum n per-lane values fill(t), t < n (n runtime, wave-uniform), over the 64 lanes into red[t]:
// chunks of 16, the last one in the smallest power of two that holds it -- a wave_reduce<K> costs
// ≈ K + log2(64/K) exchanges, so a chunk of 6 values in wave_reduce<8> saves ≈ 30 VALU against
// wave_reduce<16> (the Hessian's tail chunk: C3 −1 %).  Slots t ≥ n of a chunk hold junk.  t is a
// compile-time constant in every call of fill.  MRBO_REDUCE16: every chunk of 16 (A/B).
template <int HW, int CH, class F>
__device__ __forceinline__ void wave_reduce_n(F&& fill, int n, double* red, int lane) {
#pragma unroll
  for (int ch = 0; ch < CH; ++ch) {
    const int rem = n - 16 * ch;
    if (rem <= 0) break;
#ifndef MRBO_REDUCE16
    if (rem <= 2) {
      double v[2];
#pragma unroll
      for (int q = 0; q < 2; ++q) v[q] = fill(16 * ch + q);
      hw_reduce<HW, 2>(v, red + 16 * ch, lane);
    } else if (rem <= 4) {
      double v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = fill(16 * ch + q);
      hw_reduce<HW, 4>(v, red + 16 * ch, lane);
    } else if (rem <= 8) {
      double v[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = fill(16 * ch + q);
      hw_reduce<HW, 8>(v, red + 16 * ch, lane);
    } else
#endif
    {
      double v[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) v[q] = fill(16 * ch + q);
      hw_reduce<HW, 16>(v, red + 16 * ch, lane);
    }
  }
}

#ifdef MRBO_NO_FOLD
constexpr bool FOLD = false;
#else
constexpr bool FOLD = true;
#endif

// The same product with this lane's L entries from global memory (L2-resident image):
// step n of the block at lb[n·64].  All 64 steps of both row blocks of a pass are loaded into
// registers before their FMAs (the image is zero-padded, so the loads need no bounds).
template <int K>
__device__ __forceinline__ void gl_bcast_product_k(double (&acc)[K], const double (&v)[K], const double* lb, int nrows) {
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    if (16 * p >= nrows) break;
    double l[4][8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      l[0][u] = lb[(16 * p + u) * WAVE];
      l[1][u] = lb[(16 * p + 8 + u) * WAVE];
      l[2][u] = lb[(16 * (p + 2) + u) * WAVE];
      l[3][u] = lb[(16 * (p + 2) + 8 + u) * WAVE];
    }
    double bp[K], bp2[K];
#pragma unroll
    for (int c = 0; c < K; ++c) {
      if (p == 0) row_blocks<0>(v[c], bp[c], bp2[c]);
      else row_blocks<1>(v[c], bp[c], bp2[c]);
    }
    BcastRegAsm<K, 0>::run(acc, bp, l[0]);
    BcastRegAsm<K, 8>::run(acc, bp, l[1]);
    if (16 * (p + 2) < nrows) {
      BcastRegAsm<K, 0>::run(acc, bp2, l[2]);
      BcastRegAsm<K, 8>::run(acc, bp2, l[3]);
    }
  }
}

// Rows 16q..16q+15 of the 64×64 L2 block at lb (lane offset applied): 16 loads into l.
__device__ __forceinline__ void gl_load_q(double (&l)[16], const double* lb, int q) {
#pragma unroll
  for (int u = 0; u < 16; ++u) l[u] = lb[(16 * q + u) * WAVE];
}

template <int K>
__device__ __forceinline__ void gl_quarter(double (&acc)[K], const double (&b)[K], const double (&l)[16]) {
  if constexpr (K > 9) {
    gl_quarter<8>(head8(acc), head8(b), l);
    gl_quarter<K - 8>(tail8(acc), tail8(b), l);
  } else {
    BcastRegAsm<K, 0>::run(acc, b, head8(l));
    BcastRegAsm<K, 8>::run(acc, b, tail8(l));
  }
}

// The blocks t = t0..t1 of one row slot as ONE software-pipelined chain (MRBO_GL_CHAIN): the same
// quarters in the same order as gl_bcast_product (rows 0-15, 32-47, 16-31, 48-63 of each block,
// blocks in t order: bit-identical sums), with two 16-row buffers -- each quarter's loads are
// issued one quarter ahead, the next block's first two quarters during this block's last two.
// gl_bcast_product waits for all 32 rows of a half-block before its first FMA, and the inline
// FMA blocks are scheduling barriers, so at one wave per SIMD that L2 round trip was exposed
// twice per block.  lb[t]: block base (lane offset applied), nr[t] = min(64, N − 64t).
template <int K, int NT>
__device__ __forceinline__ void gl_chain(double (&acc)[K], const double (&v)[NT][K], const double* const (&lb)[NT],
                                         const int (&nr)[NT], int t0, int t1) {
  double la[16], lc[16];
  gl_load_q(la, lb[t0], 0);
  if (nr[t0] > 32) gl_load_q(lc, lb[t0], 2);
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    if (t < t0 || t > t1 || nr[t] <= 0) continue;
    double b0[K], b2[K];
#pragma unroll
    for (int c = 0; c < K; ++c) row_blocks<0>(v[t][c], b0[c], b2[c]);
    gl_quarter<K>(acc, b0, la);                              // rows 0-15
    if (nr[t] > 16) gl_load_q(la, lb[t], 1);
    if (nr[t] > 32) gl_quarter<K>(acc, b2, lc);             // rows 32-47
    if (nr[t] > 48) gl_load_q(lc, lb[t], 3);
    double b1[K], b3[K];
#pragma unroll
    for (int c = 0; c < K; ++c) row_blocks<1>(v[t][c], b1[c], b3[c]);
    if (nr[t] > 16) gl_quarter<K>(acc, b1, la);             // rows 16-31
    const bool more = t + 1 <= t1 && t + 1 < NT && nr[t + 1 < NT ? t + 1 : t] > 0;
    if (more) gl_load_q(la, lb[t + 1 < NT ? t + 1 : t], 0);
    if (nr[t] > 48) gl_quarter<K>(acc, b3, lc);             // rows 48-63
    if (more && nr[t + 1 < NT ? t + 1 : t] > 32) gl_load_q(lc, lb[t + 1 < NT ? t + 1 : t], 2);
  }
}

// The single-column (K = 1) products over the L2 blocks -- the value pass's forward product and
// the backward w = L0⁻ᵀY0 -- as ONE stream of 16-row quarters with MRBO_K1_NB − 1 quarters of
// loads in flight (MRBO_K1_STREAM).  A K = 1 quarter is 16 dependent FMAs, far shorter than an L2
// round trip at one wave per SIMD, so gl_bcast_product<1> waited on every half-block's loads.
// Same quarters, same order, same single accumulation chain per row slot: bit-identical sums.
// FWD: out[s] = Σ_{t ≤ s} L0⁻¹(s,t) v[t] from the forward copy; else out[s] = Σ_{t ≥ s} of the
// backward copy's block (t,s) times v[t].  base: the copy's first block, lane offset applied.
#ifndef MRBO_K1_NB
#define MRBO_K1_NB 4
#endif
template <int RPL, bool FWD>
struct K1Seq {
  static constexpr int NP = RPL * (RPL + 1) / 2, NQ = 4 * NP;
  // pair p → (s, t): FWD s-major with t = 0..s; backward s-major with t = s..RPL-1
  static constexpr int ps(int p) {
    int s = 0;
    for (;;) {
      const int n = FWD ? s + 1 : RPL - s;
      if (p < n) return s;
      p -= n;
      ++s;
    }
  }
  static constexpr int pt(int p) {
    int s = 0;
    for (;;) {
      const int n = FWD ? s + 1 : RPL - s;
      if (p < n) return FWD ? p : s + p;
      p -= n;
      ++s;
    }
  }
  static constexpr int blk(int p) {   // block index of pair p in the packed block triangle
    const int s = ps(p), t = pt(p);
    return FWD ? s * (s + 1) / 2 + t : t * (t + 1) / 2 + s;
  }
  static constexpr int qrow(int i) { return (i & 1) * 2 + ((i >> 1) & 1); }   // quarters 0, 2, 1, 3
  static constexpr bool last_of_s(int p) { return p + 1 == NP || ps(p + 1) != ps(p); }
};

template <int RPL, bool FWD>
__device__ __forceinline__ void gl_k1_stream(double (&out)[RPL], const double (&v)[RPL], const double* base, int N) {
  using S = K1Seq<RPL, FWD>;
  constexpr int NB = MRBO_K1_NB;
  double rb[RPL][4];   // row blocks 0..3 of v[t], broadcast to every 16-lane row
#pragma unroll
  for (int t = 0; t < RPL; ++t) row_blocks4(v[t], rb[t][0], rb[t][1], rb[t][2], rb[t][3]);
  double buf[NB][16];
  auto load = [&](double (&l)[16], int i) {
    const double* lb = base + (long long)S::blk(i >> 2) * WAVE * WAVE + 16 * S::qrow(i & 3) * WAVE;
#pragma unroll
    for (int u = 0; u < 16; ++u) l[u] = lb[u * WAVE];
  };
#pragma unroll
  for (int j = 0; j < NB - 1; ++j)
    if (j < S::NQ) load(buf[j], j);
  double acc[1] = {0.0};
#pragma unroll
  for (int i = 0; i < S::NQ; ++i) {
    if (i + NB - 1 < S::NQ) load(buf[(i + NB - 1) % NB], i + NB - 1);
    const int p = i >> 2, q = S::qrow(i & 3), t = S::pt(p);
    const int nr = N - WAVE * t;
    if (16 * q < nr) {
      const double b[1] = {rb[t][q]};
      BcastRegAsm<1, 0>::run(acc, b, head8(buf[i % NB]));
      BcastRegAsm<1, 8>::run(acc, b, tail8(buf[i % NB]));
    }
    if ((i & 3) == 3 && S::last_of_s(p)) {
      out[S::ps(p)] = acc[0];
      acc[0] = 0.0;
    }
  }
}

template <int K>
__device__ __forceinline__ void gl_bcast_product(double (&acc)[K], const double (&v)[K], const double* lb, int nrows) {
  if constexpr (K > 9) {
    gl_bcast_product<8>(head8(acc), head8(v), lb, nrows);
    gl_bcast_product<K - 8>(tail8(acc), tail8(v), lb, nrows);
  } else {
    gl_bcast_product_k<K>(acc, v, lb, nrows);
  }
}

// One block of an L2-fed (GL) product, from LDS where the block is LDS-resident (gl_lds_slot) and
// from L2 otherwise.  Both walks sum rows 0-15, 32-47, 16-31, 48-63 in order: bit-identical.
// Forward: block (s, t), lane i reads (i, j); backward: block (t, s) of the backward copy, lane i
// reads (k, i) -- in LDS the same BC block walked with stride 1 from lane·LD.
template <int K, int LD, int NLB>
__device__ __forceinline__ void gl_block(double (&acc)[K], const double (&v)[K], const double* Lg, const double* LinvL,
                                         int b, bool fwd, int lane, int nrows) {
  const int li = NLB > 0 ? gl_lds_slot(b) : -1;
  if (li >= 0) {
    const double* sq = LinvL + (long long)li * WAVE * LD;
    if (GL_LDS_FOLD) {   // a diagonal block: the folded three-pass products of the N ≤ 64 kernel
      if (fwd) bcast_fold_fwd<K>(acc, v, sq, lane);
      else bcast_fold_bwd<K>(acc, v, sq, lane);
    } else if (fwd) {
      bcast_product<K, LD, 1, false>(acc, v, sq + lane, nrows);
    } else {
      bcast_product<K, 1, 1, false>(acc, v, sq + lane * LD, nrows);
    }
  } else {
    gl_bcast_product<K>(acc, v, Lg + (long long)b * WAVE * WAVE + lane, nrows);
  }
}

template <int D, int RPL, int HW>
__device__ __forceinline__ bool newton_pg_ok(WaveCtx<D, RPL, HW>& W, const KParams& kp);

// ================================================================================
// eval(fs, x, θ; fantasy_index = S)  -- radial_basis_surrogates.jl:482-581
//   x is read from U[U_X].  Results land in U (lane-uniform) and `lr` (per lane).
// ================================================================================
// back_after (GRAD / GRADC / GSTART of the Newton iteration): the projected-gradient test runs
// here and, when the step continues, the BACK part (backward product, Hα) follows in the same
// call with the forward state still in registers.  Returns 1 when that BACK part ran.
template <int D, int RPL, int HW>
__device__ __forceinline__ int evaluate(WaveCtx<D, RPL, HW>& W, const KParams& kp, int S, int mode, LaneRes<D, RPL, HW>& lr,
                                        int kst = 0, bool back_after = false) {
  using Ly = Lay<D, RPL, HW>;
  constexpr int D1 = Ly::D1, BS = Ly::BS, NR = Ly::NR;
  // Opaque copy of the lane index: keeps the per-lane LDS/global addresses derived from it
  // inside this evaluation instead of being hoisted (and held live in VGPRs) across the
  // caller's Newton / horizon loops -- the difference between 1 and 3-4 waves per SIMD.
  int lane = W.lane;
  asm volatile("" : "+v"(lane));
  const int nf = S + 1;
  double* U = W.U;
  double* B = W.B;
  double* red = W.red;
  const bool all_cols = (mode != EV_VALUE);   // gradient columns
  const bool do_val = (mode != EV_GRADC);     // value part: column 0, μ, σ, EI (GRADC keeps the
                                              // preceding VALUE evaluation's, bit-identical)
  STAMP(W, 8);

  double x[D];
#pragma unroll
  for (int a = 0; a < D; ++a) x[a] = U[Ly::U_X + a];

  // base coefficients of surface S and this lane's entries of the fantasy inverse-factor rows
  double Ev[RPL][FMAX];
#pragma unroll
  for (int s = 0; s < RPL; ++s) {
    lr.cb[s] = W.C[(long long)(S + 1) * Ly::NRL + lane + WAVE * s];
#pragma unroll
    for (int r = 0; r < FMAX; ++r) Ev[s][r] = W.E[(long long)r * Ly::NRL + lane + WAVE * s];   // unconditional
#pragma unroll
    for (int r = 0; r < FMAX; ++r) Ev[s][r] = (r < nf) ? Ev[s][r] : 0.0;
  }

  const int N = W.N;
  double acc[RPL][D1];   // Y = L0⁻¹ [kx, ∇kx] rows owned by this lane
  if (mode != EV_BACK) {
  // ---- 1. kernel rows B[i] = [k(x,X_i), ∇k(x - X_i)]  (eval_KxX :180-191, eval_∇KxX :193-208)
  double Bown[RPL][D1];
  double rf[D], psif = 0.0, g1f = 0.0, g2f = 0.0;   // fantasy row of this lane (paired radial evaluation)
  // GRADC follows the VALUE evaluation at the same x: its g1 (G12), fantasy rows (B) and
  // fantasy Hessian terms (U_HF) are still in LDS, so no radial function is re-evaluated
  const bool rows_kept = (mode == EV_GRADC);
#pragma unroll
  for (int s = 0; s < RPL; ++s) {
    double r[D], rho2 = 0.0;
#pragma unroll
    for (int a = 0; a < D; ++a) { r[a] = x[a] - W.x0(kp, s, a); rho2 = fma(r[a], r[a], rho2); }
    if (rows_kept) {
      const double g1 = W.G12[3 * (lane + WAVE * s)];
      const bool v = W.rowv(kp, s);
      Bown[s][0] = 0.0;   // column 0 comes from the VALUE pass
#pragma unroll
      for (int a = 0; a < D; ++a) Bown[s][1 + a] = v ? g1 * r[a] : 0.0;
      continue;
    }
    double psi, g1, g2;
#ifndef MRBO_NO_PAIRED_RAD
    if constexpr (RPL == 1) {
      // this lane's fantasy row (lanes < nf) shares the radial evaluation of its base row
      const int fl = lane < nf ? lane : 0;
      double rho2f = 0.0;
#pragma unroll
      for (int a = 0; a < D; ++a) { rf[a] = x[a] - U[Ly::U_XF + fl * D + a]; rho2f = fma(rf[a], rf[a], rho2f); }
      rad_eval2(W.rad, rho2, rho2f, psi, g1, g2, psif, g1f, g2f);
    } else
#endif
    rad_eval(W.rad, rho2, psi, g1, g2);
    const bool v = W.rowv(kp, s);
    Bown[s][0] = v ? psi : 0.0;
#pragma unroll
    for (int a = 0; a < D; ++a) Bown[s][1 + a] = v ? g1 * r[a] : 0.0;
    W.G12[3 * (lane + WAVE * s)] = g1;       // kept for a Hessian (phase 6, maybe deferred)
    W.G12[3 * (lane + WAVE * s) + 1] = g2;
  }
  if (lane < nf && !rows_kept) {  // fantasy rows B[N + r]; [x − X_r, g1, g2] kept for the Hessian
    double r[D], psi, g1, g2;
#ifndef MRBO_NO_PAIRED_RAD
    if constexpr (RPL == 1) {
#pragma unroll
      for (int a = 0; a < D; ++a) r[a] = rf[a];
      psi = psif;
      g1 = g1f;
      g2 = g2f;
    } else
#endif
    {
      double rho2 = 0.0;
#pragma unroll
      for (int a = 0; a < D; ++a) { r[a] = x[a] - U[Ly::U_XF + lane * D + a]; rho2 = fma(r[a], r[a], rho2); }
      rad_eval(W.rad, rho2, psi, g1, g2);
    }
    double* row = B + (Ly::FR0 + lane) * BS;
    row[0] = psi;
#pragma unroll
    for (int a = 0; a < D; ++a) row[1 + a] = g1 * r[a];
    {
      double* hf = U + Ly::U_HF + lane * (D + 2);
#pragma unroll
      for (int a = 0; a < D; ++a) hf[a] = r[a];
      hf[D] = g1;
      hf[D + 1] = g2;
    }
  }
  wave_sync();
  STAMP(W, 0);

  // ---- 2. forward product  Y[i] = Σ_{j ≤ i} L0⁻¹[i,j] B[j]   (L\kxX' , r_b_s.jl:525-526)
#pragma unroll
  for (int s = 0; s < RPL; ++s)
#pragma unroll
    for (int c = 0; c < D1; ++c) acc[s][c] = 0.0;
  if constexpr (Ly::BC) {
    // lane i reads L0⁻¹[64s+i][64t+j] at blk(s,t)·BLK + j·LD + i; rows j of block column t are
    // broadcast from register slot t.  Row slot s sums block columns t = 0..s in order.
    auto nrows = [&](int t) { const int n = N - WAVE * t; return n < WAVE ? n : WAVE; };
    // RPL = 1 with N > 48: the folded three-pass products (bcast_fold_fwd / _bwd)
    const bool fold = FOLD && Ly::SQ && HW == 1 && N > 48;
    // N ≤ 128 (two rows per lane): the diagonal blocks (s, s) by the same folded products
    // (MRBO_BC_DIAG_FOLD, A/B)
#ifdef MRBO_BC_DIAG_FOLD
    constexpr bool DFOLD = !Ly::SQ && HW == 1;
#else
    constexpr bool DFOLD = false;
#endif
    if (Ly::SQ_EAGER && mode == EV_VALUE) {
      // The K = 1 value product is bound by LDS reads (one ds_read_b64 per FMA, eight waves on
      // one LDS); ≈ 95 % of C3's non-batched value passes are followed by a GRADC pass at the same
      // x.  So the value pass runs all D1 columns (seven FMAs per read) and stashes columns 1..d
      // in the wave's LDS, where the GRADC pass reads them instead of its K = d product.  Same
      // fold, same steps per column: bit-identical sums.  Off by default (SQ_EAGER_ON above).
      if (fold) bcast_fold_fwd<D1>(acc[0], Bown[0], W.Linv, lane);
      else bcast_product<D1, Ly::LD, HW>(acc[0], Bown[0], W.Linv + lane, nrows(0));
#pragma unroll
      for (int a = 0; a < D; ++a) W.STASH[a * WAVE + lane] = acc[0][1 + a];
    } else if (Ly::SQ_EAGER && mode == EV_GRADC) {
#pragma unroll
      for (int a = 0; a < D; ++a) acc[0][1 + a] = W.STASH[a * WAVE + lane];
      acc[0][0] = W.G12[3 * lane + 2];
    } else if (mode == EV_VALUE) {
#pragma unroll
      for (int s = 0; s < RPL; ++s) {
        double a1[1] = {0.0};
#pragma unroll
        for (int t = 0; t <= s; ++t) {
          const double v1[1] = {Bown[t][0]};
          if (fold) bcast_fold_fwd<1>(a1, v1, W.Linv, lane);
          else if (DFOLD && s == t && nrows(t) > 48) bcast_fold_fwd<1>(a1, v1, W.Linv + Ly::blk(s, t) * Ly::BLK, lane);
          else bcast_product<1, Ly::LD, HW>(a1, v1, W.Linv + Ly::blk(s, t) * Ly::BLK + lane, nrows(t));
        }
        acc[s][0] = a1[0];
      }
    } else if (mode == EV_GSTART) {  // base forward product of start kst from the launch tables
      if constexpr (Ly::SQ) acc[0][0] = W.YTAB[(long long)kst * NR + lane];
    } else if (mode == EV_GRADC) {   // columns 1..d; column 0 from the VALUE pass
#pragma unroll
      for (int s = 0; s < RPL; ++s) {
        double ag[D];
#pragma unroll
        for (int a = 0; a < D; ++a) ag[a] = 0.0;
#pragma unroll
        for (int t = 0; t <= s; ++t) {
          double vg[D];
#pragma unroll
          for (int a = 0; a < D; ++a) vg[a] = Bown[t][1 + a];
          if (fold) bcast_fold_fwd<D>(ag, vg, W.Linv, lane);
          else if (DFOLD && s == t && nrows(t) > 48) bcast_fold_fwd<D>(ag, vg, W.Linv + Ly::blk(s, t) * Ly::BLK, lane);
          else bcast_product<D, Ly::LD, HW>(ag, vg, W.Linv + Ly::blk(s, t) * Ly::BLK + lane, nrows(t));
        }
#pragma unroll
        for (int a = 0; a < D; ++a) acc[s][1 + a] = ag[a];
        acc[s][0] = W.G12[3 * (lane + WAVE * s) + 2];
      }
    } else {
#pragma unroll
      for (int s = 0; s < RPL; ++s)
#pragma unroll
        for (int t = 0; t <= s; ++t) {
          if (fold) bcast_fold_fwd<D1>(acc[s], Bown[t], W.Linv, lane);
          else if (DFOLD && s == t && nrows(t) > 48) bcast_fold_fwd<D1>(acc[s], Bown[t], W.Linv + Ly::blk(s, t) * Ly::BLK, lane);
          else bcast_product<D1, Ly::LD, HW>(acc[s], Bown[t], W.Linv + Ly::blk(s, t) * Ly::BLK + lane, nrows(t));
        }
    }
  } else {
    // GL (N ≤ 256): the same register broadcast with L0⁻¹ from L2: lane i reads (i, j) of block
    // (s,t) at blk(s,t)·4096 + j·64 + i, 16 steps' entries loaded ahead into registers
    auto nrows = [&](int t) { const int n = N - WAVE * t; return n < WAVE ? n : WAVE; };
    const double* L0 = W.Linv + lane;
#ifdef MRBO_GL_CHAIN
    int nr[RPL];
#pragma unroll
    for (int t = 0; t < RPL; ++t) nr[t] = nrows(t);
    if (mode == EV_VALUE) {
      double v1[RPL][1];
#pragma unroll
      for (int t = 0; t < RPL; ++t) v1[t][0] = Bown[t][0];
#pragma unroll
      for (int s = 0; s < RPL; ++s) {
        const double* lb[RPL];
#pragma unroll
        for (int t = 0; t < RPL; ++t) lb[t] = L0 + Ly::blk(s, t <= s ? t : s) * WAVE * WAVE;
        double a1[1] = {0.0};
        gl_chain<1, RPL>(a1, v1, lb, nr, 0, s);
        acc[s][0] = a1[0];
      }
    } else if (mode == EV_GRADC) {
      double vg[RPL][D];
#pragma unroll
      for (int t = 0; t < RPL; ++t)
#pragma unroll
        for (int a = 0; a < D; ++a) vg[t][a] = Bown[t][1 + a];
#pragma unroll
      for (int s = 0; s < RPL; ++s) {
        const double* lb[RPL];
#pragma unroll
        for (int t = 0; t < RPL; ++t) lb[t] = L0 + Ly::blk(s, t <= s ? t : s) * WAVE * WAVE;
        double ag[D];
#pragma unroll
        for (int a = 0; a < D; ++a) ag[a] = 0.0;
        gl_chain<D, RPL>(ag, vg, lb, nr, 0, s);
#pragma unroll
        for (int a = 0; a < D; ++a) acc[s][1 + a] = ag[a];
        acc[s][0] = W.G12[3 * (lane + WAVE * s) + 2];
      }
    } else {
#pragma unroll
      for (int s = 0; s < RPL; ++s) {
        const double* lb[RPL];
#pragma unroll
        for (int t = 0; t < RPL; ++t) lb[t] = L0 + Ly::blk(s, t <= s ? t : s) * WAVE * WAVE;
        gl_chain<D1, RPL>(acc[s], Bown, lb, nr, 0, s);
      }
    }
#else
    // MRBO_GL_EAGER (A/B, not the default): with NonUniformCost ≈ 54 % of C5 + cost's value
    // passes are followed by a gradient pass at the same x, so the value pass could run all D1
    // columns and stash columns 1..d in the wave's global slot for that GRADC pass (same blocks,
    // same rows in the same order per column: bit-identical sums).  Measured (round 6, C5 + cost
    // 256 × 128, same box): 1 278 → 1 386 ms, +8.5 % -- at one wave per SIMD the nine-column
    // walk costs far more than the L0⁻¹ stream it saves.
#ifdef MRBO_GL_EAGER
    const bool eager = kp.cost != COST_NONE;
#else
    const bool eager = false;
#endif
    if (mode == EV_VALUE && eager) {
#pragma unroll
      for (int s = 0; s < RPL; ++s)
#pragma unroll
        for (int t = 0; t <= s; ++t)
          gl_block<D1, Ly::LD, Ly::NLB>(acc[s], Bown[t], W.Linv, W.LinvL, Ly::blk(s, t), true, lane, nrows(t));
#pragma unroll
      for (int s = 0; s < RPL; ++s)
#pragma unroll
        for (int a = 0; a < D; ++a) W.STASH[(long long)(s * D + a) * WAVE + lane] = acc[s][1 + a];
    } else if (mode == EV_GRADC && eager) {
#pragma unroll
      for (int s = 0; s < RPL; ++s) {
#pragma unroll
        for (int a = 0; a < D; ++a) acc[s][1 + a] = W.STASH[(long long)(s * D + a) * WAVE + lane];
        acc[s][0] = W.G12[3 * (lane + WAVE * s) + 2];
      }
    } else if (mode == EV_VALUE) {
#ifdef MRBO_K1_STREAM
      double v1[RPL], o1[RPL];
#pragma unroll
      for (int t = 0; t < RPL; ++t) v1[t] = Bown[t][0];
      gl_k1_stream<RPL, true>(o1, v1, L0, N);
#pragma unroll
      for (int s = 0; s < RPL; ++s) acc[s][0] = o1[s];
#else
#pragma unroll
      for (int s = 0; s < RPL; ++s) {
        double a1[1] = {0.0};
#pragma unroll
        for (int t = 0; t <= s; ++t) {
          const double v1[1] = {Bown[t][0]};
          gl_block<1, Ly::LD, Ly::NLB>(a1, v1, W.Linv, W.LinvL, Ly::blk(s, t), true, lane, nrows(t));
        }
        acc[s][0] = a1[0];
      }
#endif
    } else if (mode == EV_GRADC) {
#pragma unroll
      for (int s = 0; s < RPL; ++s) {
        double ag[D];
#pragma unroll
        for (int a = 0; a < D; ++a) ag[a] = 0.0;
#pragma unroll
        for (int t = 0; t <= s; ++t) {
          double vg[D];
#pragma unroll
          for (int a = 0; a < D; ++a) vg[a] = Bown[t][1 + a];
          gl_block<D, Ly::LD, Ly::NLB>(ag, vg, W.Linv, W.LinvL, Ly::blk(s, t), true, lane, nrows(t));
        }
#pragma unroll
        for (int a = 0; a < D; ++a) acc[s][1 + a] = ag[a];
        acc[s][0] = W.G12[3 * (lane + WAVE * s) + 2];
      }
    } else {
#pragma unroll
      for (int s = 0; s < RPL; ++s)
#pragma unroll
        for (int t = 0; t <= s; ++t)
          gl_block<D1, Ly::LD, Ly::NLB>(acc[s], Bown[t], W.Linv, W.LinvL, Ly::blk(s, t), true, lane, nrows(t));
    }
#endif
  }

  if (do_val) {   // Y0 kept for a deferred GRADC / BACK evaluation
#pragma unroll
    for (int s = 0; s < RPL; ++s) W.G12[3 * (lane + WAVE * s) + 2] = acc[s][0];
  }
  STAMP(W, 1);
  // ---- 3. per-lane products and wave reductions
  if (do_val) {   // [|v|² = kx'K⁻¹kx, μ = kx·c (base parts), E_r·kx (r < nf)]: 2 + nf values
    static_assert(2 + FMAX <= 8, "value reduction: one chunk");
    wave_reduce_n<HW, 1>([&](int t) {
      double s_ = 0.0;
#pragma unroll
      for (int s = 0; s < RPL; ++s) {
        if (t == 0) s_ = fma(acc[s][0], acc[s][0], s_);
        else if (t == 1) s_ = fma(lr.cb[s], Bown[s][0], s_);
        else if (t - 2 < FMAX) s_ = fma(Ev[s][t - 2], Bown[s][0], s_);
      }
      return s_;
    }, 2 + nf, red + Ly::R_VAL, lane);
  }
  if (all_cols) {
    // Gram entries (a ≤ b) except (0,0); GSTART takes them from the start tables
#pragma unroll
    for (int ch = 0; ch < Ly::NGC; ++ch) {
      if (mode == EV_GSTART) break;
      double v[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int t = 1 + 16 * ch + q;  // linear pair index
        double s_ = 0.0;
        if (t < Ly::NG) {
          // unrank t -> (a, b), a ≤ b, row-major upper triangle
          int a = 0, rem = t;
#pragma unroll
          for (int aa = 0; aa < D1; ++aa) if (a == aa && rem >= D1 - aa) { rem -= D1 - aa; a = aa + 1; }
          const int b = a + rem;
#pragma unroll
          for (int s = 0; s < RPL; ++s) s_ = fma(acc[s][a], acc[s][b], s_);
        }
        v[q] = s_;
      }
      hw_reduce<HW, 16>(v, red + Ly::R_G + 16 * ch, lane);
    }
    // ∇μ and fantasy cross products for the gradient columns
    // (fantasy rows ≥ nf carry nothing: D·(1 + nf) values)
    wave_reduce_n<HW, Ly::NMFC>([&](int t) {
      double s_ = 0.0;
      if (t < Ly::NMF) {
        const int grp = t / D, a = t % D;  // grp 0: c ; grp r+1: E_r
        if (grp == 0) {
#pragma unroll
          for (int s = 0; s < RPL; ++s) s_ = fma(lr.cb[s], Bown[s][1 + a], s_);
        } else {
#pragma unroll
          for (int s = 0; s < RPL; ++s) s_ = fma(Ev[s][grp - 1], Bown[s][1 + a], s_);
        }
      }
      return s_;
    }, D * (1 + nf), red + Ly::R_MF, lane);
  }
  wave_sync();
  STAMP(W, 2);

  // ---- 4a. column 0 in every lane: fantasy rows Yf[r][0] = E_r·B0 + Σ_q Dinv[r][q] Bf[q][0],
  // G00 = |Y0|² + Σ_r Yf[r][0]², μ = c·kx + Σ_r c_r Bf[r][0].  One batch of unconditional LDS
  // reads instead of three dependent lane-distributed phases (same FMA order).
  double mu_v = 0.0, g00_v = 0.0;
  if (do_val) {
    double bf[FMAX], yf[FMAX];
#pragma unroll
    for (int r = 0; r < FMAX; ++r) bf[r] = B[(Ly::FR0 + r) * BS];
    g00_v = red[Ly::R_VAL];
    mu_v = red[Ly::R_VAL + 1];
#pragma unroll
    for (int r = 0; r < FMAX; ++r) {
      double y = red[Ly::R_VAL + 2 + r];
#pragma unroll
      for (int q = 0; q <= r; ++q) y = fma(U[Ly::U_DINV + r * FMAX + q], bf[q], y);
      yf[r] = y;
    }
#pragma unroll
    for (int r = 0; r < FMAX; ++r) {
      if (r < nf) {
        g00_v = fma(yf[r], yf[r], g00_v);
        mu_v = fma(U[Ly::U_CF + (S + 1) * FMAX + r], bf[r], mu_v);
      }
    }
    if (lane < FMAX) {
      double mine = 0.0;
#pragma unroll
      for (int r = 0; r < FMAX; ++r) mine = (lane == r) ? yf[r] : mine;
      if (lane < nf) U[Ly::U_YFV + lane * D1] = mine;
    }
    if (lane == 0) {
      U[Ly::U_G] = g00_v;
      U[Ly::U_SC + SC_MU] = mu_v;
    }
  }
  // ---- 4b. gradient columns of the fantasy rows: Yf = Fpart + Dinv · Bf   (lane = (r, c), c ≥ 1)
  if (all_cols) {
  {
    const int ncol = D;
    // entry t = (r, c) per lane; d > 10 has more entries than lanes: lane, lane + 64, …
    for (int t = lane; t < (FMAX * D <= Ly::LANES ? Ly::LANES : FMAX * D); t += Ly::LANES) {
      if (t >= nf * ncol) break;
      const int r = t / ncol, c = 1 + t % ncol;
      double y = red[Ly::R_MF + D + r * D + (c - 1)];
      for (int q = 0; q <= r; ++q) y = fma(U[Ly::U_DINV + r * FMAX + q], B[(Ly::FR0 + q) * BS + c], y);
      U[Ly::U_YFV + r * D1 + c] = y;
      if constexpr (FMAX * D <= Ly::LANES) break;
    }
  }
  wave_sync();
  // ---- Gram (incl. fantasy rows) and ∇μ  (lanes own entries; G00 and μ above)
  {
    auto gram_entry = [&](int t) {
      int a = 0, rem = t;
#pragma unroll
      for (int aa = 0; aa < D1; ++aa) if (a == aa && rem >= D1 - aa) { rem -= D1 - aa; a = aa + 1; }
      const int b = a + rem;
      double g = (mode == EV_GSTART) ? W.GTAB[kst * Ly::NG + t] : red[Ly::R_G + t - 1];
      for (int r = 0; r < nf; ++r) g = fma(U[Ly::U_YFV + r * D1 + a], U[Ly::U_YFV + r * D1 + b], g);
      U[Ly::U_G + a * D1 + b] = g;
      U[Ly::U_G + b * D1 + a] = g;
    };
    auto gmu_entry = [&](int c) {   // c = 1..D
      double mu = red[Ly::R_MF + c - 1];
      for (int r = 0; r < nf; ++r) mu = fma(U[Ly::U_CF + (S + 1) * FMAX + r], B[(Ly::FR0 + r) * BS + c], mu);
      U[Ly::U_GMU + c - 1] = mu;
    };
    if constexpr (HW == 2) {        // half-wave (d ≤ 4): Gram on lanes 1..NG-1, ∇μ on lanes 16..15+d
      static_assert(Ly::NG <= 16 && 16 + D <= 32, "half-wave Gram placement");
      if (lane > 0 && lane < Ly::NG) gram_entry(lane);
      if (lane >= 16 && lane < 16 + D) gmu_entry(lane - 15);
    } else if constexpr (Ly::NG <= 49) {   // d ≤ 8: Gram entries on lanes 1..NG-1, ∇μ on lanes 49..48+d
      if (lane > 0 && lane < Ly::NG) gram_entry(lane);
      if (lane >= 49 && lane < 48 + D1) gmu_entry(lane - 48);
    } else {                        // wider: both as lane-strided loops
      for (int t = lane; t < Ly::NG; t += WAVE)
        if (t > 0) gram_entry(t);
      if (lane >= 1 && lane <= D) gmu_entry(lane);
    }
  }
  wave_sync();
  }
  STAMP(W, 3);

  // ---- σ, EI partials (all lanes, wave-uniform values)
  double isig_f;
  EIp e_f;
  if (do_val) {
  const double mu = mu_v;
  const double var = KCV(PSI0) - g00_v;
  double sig, isig;
  sig_isig(var, sig, isig);
  const double fmin = U[Ly::U_FMIN + S + 1];
  const EIp e = rule_partials(kp.rule, mu, sig, KCV(THETA), fmin, KCV(SIGTOL), isig);
  double alpha = e.g;
  if (kp.cost) {   // cost-weighted rule f = α/c(x) (NonUniformCost, cost_functions.jl:5-20)
    double gc[D];
    const double c = cost_eval<D>(kp, x, gc);
    double gmax = 0.0;
#pragma unroll
    for (int a = 0; a < D; ++a) gmax = fmax(gmax, fabs(gc[a]));
    alpha = e.g / c;
    if (lane == 0) {
      U[Ly::U_SC + SC_ARAW] = e.g;
      U[Ly::U_SC + SC_COSTC] = c;
      U[Ly::U_SC + SC_GCMAX] = gmax;
    }
  }
  if (lane == 0) {
    U[Ly::U_SC + SC_SIG] = sig;
    U[Ly::U_SC + SC_ISIG] = isig;
    U[Ly::U_SC + SC_VAR] = var;
    U[Ly::U_SC + SC_ALPHA] = alpha;
    U[Ly::U_SC + SC_GMU] = e.gmu;
    U[Ly::U_SC + SC_GSIG] = e.gsig;
    U[Ly::U_SC + SC_GMUMU] = e.gmumu;
    U[Ly::U_SC + SC_GSIGSIG] = e.gsigsig;
    U[Ly::U_SC + SC_GMUTH] = e.gmuth;
    U[Ly::U_SC + SC_GSIGTH] = e.gsigth;
    U[Ly::U_SC + SC_FMIN] = fmin;
  }
  if (mode == EV_VALUE) { wave_sync(); STAMP(W, 4); return 0; }
  isig_f = isig;
  e_f = e;
  } else {   // GRADC: σ and the EI partials of the VALUE pass at this point
    isig_f = U[Ly::U_SC + SC_ISIG];
    e_f.gmu = U[Ly::U_SC + SC_GMU];
    e_f.gsig = U[Ly::U_SC + SC_GSIG];
    e_f.gmuth = U[Ly::U_SC + SC_GMUTH];
    e_f.gsigth = U[Ly::U_SC + SC_GSIGTH];
  }
  if (lane < D) {
    const double gs = -U[Ly::U_G + (1 + lane) * D1] * isig_f;  // ∇σ = -(∇kx·w)/σ
    const double gm = U[Ly::U_GMU + lane];
    U[Ly::U_GSIG + lane] = gs;
    double gal = e_f.gmu * gm + e_f.gsig * gs;                         // ∇αx :567
    double mix = gm * e_f.gmuth + gs * e_f.gsigth;                     // d2α_dxdθ :575-577
    if (kp.cost) {   // ∇(α/c) = ∇α/c − α∇c/c²,  ∂∇(α/c)/∂θ = ∂∇α/∂θ/c − g_θ∇c/c²
      double gc[D];
      (void)cost_eval<D>(kp, x, gc);
      const double gca = lane_pick<D>(gc, lane);
      const double c = U[Ly::U_SC + SC_COSTC], araw = U[Ly::U_SC + SC_ARAW];
      gal = gal / c - (araw / (c * c)) * gca;
      mix = mix / c - rule_gth(kp.rule, e_f.gmu, U[Ly::U_SC + SC_SIG]) * gca / (c * c);
    }
    U[Ly::U_GAL + lane] = gal;
    U[Ly::U_MIX + lane] = mix;
  }
  if (mode == EV_GRAD || mode == EV_GRADC || mode == EV_GSTART) {   // a BACK evaluation may follow
    wave_sync();
    STAMP(W, 4);
    if (!back_after) return 0;
    // the Newton iteration's P_GRAD decision (newton below): g = −∇α, stop when stationary
    if (lane < D) U[Ly::U_NG + lane] = -U[Ly::U_GAL + lane];
    wave_sync();
    if (!newton_pg_ok<D, RPL, HW>(W, kp)) return 0;
    STAMP(W, 12);
  }
  } else {   // EV_BACK: resume at the point of the preceding GRAD evaluation
#pragma unroll
    for (int s = 0; s < RPL; ++s) acc[s][0] = W.G12[3 * (lane + WAVE * s) + 2];
  }
  wave_sync();   // U_SC / gradients of the front part visible to all lanes
  EIp e;
  e.gmu = U[Ly::U_SC + SC_GMU];
  e.gsig = U[Ly::U_SC + SC_GSIG];
  e.gmumu = U[Ly::U_SC + SC_GMUMU];
  e.gsigsig = U[Ly::U_SC + SC_GSIGSIG];

  STAMP(W, 4);
  // ---- 5. backward product w = L⁻ᵀ v (and P = L⁻ᵀ V for the adjoint)
  const bool rich = (mode == EV_RICH);
  {
    double wv[RPL], pv[RPL][D];
#pragma unroll
    for (int s = 0; s < RPL; ++s) {
      wv[s] = 0.0;
#pragma unroll
      for (int a = 0; a < D; ++a) pv[s][a] = 0.0;
    }
    if constexpr (Ly::BC) {
      // lane i (row slot s) reads L0⁻¹[64t+k][64s+i] at blk(t,s)·BLK + i·LD + k for block rows
      // t = s..RPL-1; rows k of Y are broadcast from register slot t
      auto nrows = [&](int t) { const int n = N - WAVE * t; return n < WAVE ? n : WAVE; };
      const bool fold = FOLD && Ly::SQ && HW == 1 && N > 48;
#ifdef MRBO_BC_DIAG_FOLD
      constexpr bool DFOLD = !Ly::SQ && HW == 1;
#else
      constexpr bool DFOLD = false;
#endif
#pragma unroll
      for (int s = 0; s < RPL; ++s) {
        if (rich) {
          double a7[D1];
#pragma unroll
          for (int c = 0; c < D1; ++c) a7[c] = 0.0;
#pragma unroll
          for (int t = s; t < RPL; ++t) {
            if (fold) bcast_fold_bwd<D1>(a7, acc[t], W.Linv, lane);
            else if (DFOLD && s == t && nrows(t) > 48) bcast_fold_bwd<D1>(a7, acc[t], W.Linv + Ly::blk(t, s) * Ly::BLK, lane);
            else bcast_product<D1, 1, HW>(a7, acc[t], W.Linv + Ly::blk(t, s) * Ly::BLK + lane * Ly::LD, nrows(t));
          }
          wv[s] = a7[0];
#pragma unroll
          for (int a = 0; a < D; ++a) pv[s][a] = a7[1 + a];
        } else {
          double a1[1] = {0.0};
#pragma unroll
          for (int t = s; t < RPL; ++t) {
            const double v1[1] = {acc[t][0]};
            if (fold) bcast_fold_bwd<1>(a1, v1, W.Linv, lane);
            else if (DFOLD && s == t && nrows(t) > 48) bcast_fold_bwd<1>(a1, v1, W.Linv + Ly::blk(t, s) * Ly::BLK, lane);
            else bcast_product<1, 1, HW>(a1, v1, W.Linv + Ly::blk(t, s) * Ly::BLK + lane * Ly::LD, nrows(t));
          }
          wv[s] = a1[0];
        }
      }
    } else {
      // GL: lane i (row slot s) reads (k, i) of block (t,s) from the backward copy at
      // blk(t,s)·4096 + k·64 + i; rows k of Y from register slot t
      auto nrows = [&](int t) { const int n = N - WAVE * t; return n < WAVE ? n : WAVE; };
      const double* LT = W.LinvT + lane;
#ifdef MRBO_GL_CHAIN
      int nr[RPL];
#pragma unroll
      for (int t = 0; t < RPL; ++t) nr[t] = nrows(t);
      double y1[RPL][1];
#pragma unroll
      for (int t = 0; t < RPL; ++t) y1[t][0] = acc[t][0];
#pragma unroll
      for (int s = 0; s < RPL; ++s) {
        const double* lb[RPL];
#pragma unroll
        for (int t = 0; t < RPL; ++t) lb[t] = LT + Ly::blk(t >= s ? t : s, s) * WAVE * WAVE;
        if (rich) {
          double a7[D1];
#pragma unroll
          for (int c = 0; c < D1; ++c) a7[c] = 0.0;
          gl_chain<D1, RPL>(a7, acc, lb, nr, s, RPL - 1);
          wv[s] = a7[0];
#pragma unroll
          for (int a = 0; a < D; ++a) pv[s][a] = a7[1 + a];
        } else {
          double a1[1] = {0.0};
          gl_chain<1, RPL>(a1, y1, lb, nr, s, RPL - 1);
          wv[s] = a1[0];
        }
      }
#else
#ifdef MRBO_K1_STREAM
      if (!rich) {
        double y1[RPL];
#pragma unroll
        for (int t = 0; t < RPL; ++t) y1[t] = acc[t][0];
        gl_k1_stream<RPL, false>(wv, y1, LT, N);
      } else
#endif
#pragma unroll
      for (int s = 0; s < RPL; ++s) {
        if (rich) {
          double a7[D1];
#pragma unroll
          for (int c = 0; c < D1; ++c) a7[c] = 0.0;
#pragma unroll
          for (int t = s; t < RPL; ++t)
            gl_block<D1, Ly::LD, Ly::NLB>(a7, acc[t], W.LinvT, W.LinvL, Ly::blk(t, s), false, lane, nrows(t));
          wv[s] = a7[0];
#pragma unroll
          for (int a = 0; a < D; ++a) pv[s][a] = a7[1 + a];
        } else {
          double a1[1] = {0.0};
#pragma unroll
          for (int t = s; t < RPL; ++t) {
            const double v1[1] = {acc[t][0]};
            gl_block<1, Ly::LD, Ly::NLB>(a1, v1, W.LinvT, W.LinvL, Ly::blk(t, s), false, lane, nrows(t));
          }
          wv[s] = a1[0];
        }
      }
#endif
    }
    // fantasy part: + Σ_r E[r][i] Yf[r]
#pragma unroll
    for (int s = 0; s < RPL; ++s) {
#pragma unroll
      for (int r = 0; r < FMAX; ++r) {
        if (r >= nf) break;
        const double er = Ev[s][r];
        wv[s] = fma(er, U[Ly::U_YFV + r * D1], wv[s]);
        if (rich) {
#pragma unroll
          for (int a = 0; a < D; ++a) pv[s][a] = fma(er, U[Ly::U_YFV + r * D1 + 1 + a], pv[s][a]);
        }
      }
    }
#pragma unroll
    for (int s = 0; s < RPL; ++s) {
      lr.w[s] = wv[s];
#pragma unroll
      for (int a = 0; a < D; ++a) lr.P[s][a] = pv[s][a];
    }
  }
  // w_f[q] = Σ_{r ≥ q} Dinv[r][q] Yf[r][0]  (and P_f)
  {
    const int ncol = rich ? D1 : 1;
    for (int e = lane; e < (FMAX * D1 <= Ly::LANES ? Ly::LANES : FMAX * D1); e += Ly::LANES) {   // d > 9: lane-strided
      if (e >= nf * ncol) break;
      const int q = e / ncol, c = e % ncol;
      double t = 0.0;
      for (int r = q; r < nf; ++r) t = fma(U[Ly::U_DINV + r * FMAX + q], U[Ly::U_YFV + r * D1 + c], t);
      if (c == 0) U[Ly::U_WF + q] = t; else U[Ly::U_PF + q * D + c - 1] = t;
      if constexpr (FMAX * D1 <= Ly::LANES) break;
    }
  }
  if (mode == EV_DRAW) { wave_sync(); STAMP(W, 5); return 0; }
  STAMP(W, 5);

  // ---- 6. Hessian  Hα = gμμ∇μ∇μ' + gσσ∇σ∇σ' − (gσ/σ)(∇σ∇σ' + ∇kx·Dw) + Σ_j coef_j Hk_j
  // Σ_i coef_i ∇²k(x − X_i) with ∇²k = g2·r rᵀ + g1·I (g1, g2 kept from phase 1)
  const double gsig_over = (e.gsig == 0.0) ? 0.0 : e.gsig * U[Ly::U_SC + SC_ISIG];
  {
    double nv[RPL][D], ca[RPL], tb[RPL];
#pragma unroll
    for (int s = 0; s < RPL; ++s) {
#pragma unroll
      for (int a = 0; a < D; ++a) nv[s][a] = x[a] - W.x0(kp, s, a);
      const double coef = W.rowv(kp, s) ? (e.gmu * lr.cb[s] - gsig_over * lr.w[s]) : 0.0;
      ca[s] = coef * W.G12[3 * (lane + WAVE * s) + 1];
      tb[s] = coef * W.G12[3 * (lane + WAVE * s)];
    }
    wave_sync();  // previous users of red are done (all lanes passed phase 4)
    // NH + 1 values: full chunks of 16, then the tail in a chunk of 8 when it fits (d = 6: 16 + 6)
    auto hval = [&](int t) {
      double s_ = 0.0;
      if (t < Ly::NH) {
        int a = 0, rem = t;
#pragma unroll
        for (int aa = 0; aa < D; ++aa) if (a == aa && rem >= D - aa) { rem -= D - aa; a = aa + 1; }
        const int b = a + rem;
#pragma unroll
        for (int s = 0; s < RPL; ++s) s_ = fma(ca[s], nv[s][a] * nv[s][b], s_);
      } else if (t == Ly::NH) {
#pragma unroll
        for (int s = 0; s < RPL; ++s) s_ += tb[s];
      }
      return s_;
    };
    constexpr int HTAIL = (Ly::NH + 1) % 16;
    constexpr int HFULL = (HTAIL > 0 && HTAIL <= 8 && !MRBO_HESS16) ? (Ly::NH + 1) / 16 : Ly::NHC;
#pragma unroll
    for (int ch = 0; ch < HFULL; ++ch) {
      double vv[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) vv[q] = hval(16 * ch + q);
      hw_reduce<HW, 16>(vv, red + 16 * ch, lane);
    }
    if constexpr (HFULL < Ly::NHC) {
      double vv[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) vv[q] = hval(16 * HFULL + q);
      hw_reduce<HW, 8>(vv, red + 16 * HFULL, lane);
    }
  }
  wave_sync();
  STAMP(W, 6);
  for (int he = lane; he < (Ly::NH <= Ly::LANES ? Ly::LANES : Ly::NH); he += Ly::LANES) {   // d > 10: lane-strided
    if (he >= Ly::NH) break;
    int a = 0, rem = he;
#pragma unroll
    for (int aa = 0; aa < D; ++aa) if (a == aa && rem >= D - aa) { rem -= D - aa; a = aa + 1; }
    const int b = a + rem;
    const double gma = U[Ly::U_GMU + a], gmb = U[Ly::U_GMU + b];
    const double gsa = U[Ly::U_GSIG + a], gsb = U[Ly::U_GSIG + b];
    const double rdiag = red[Ly::NH];
    double hv = red[he] + ((a == b) ? rdiag : 0.0);
    // fantasy data points ([x − X_r, g1, g2] from phase 1)
    for (int r = 0; r < nf; ++r) {
      const double* hf = U + Ly::U_HF + r * (D + 2);
      const double coef = e.gmu * U[Ly::U_CF + (S + 1) * FMAX + r] - gsig_over * U[Ly::U_WF + r];
      hv = fma(coef * hf[D + 1], hf[a] * hf[b], hv);
      if (a == b) hv = fma(coef, hf[D], hv);
    }
    hv += e.gmumu * gma * gmb + e.gsigsig * gsa * gsb - gsig_over * (gsa * gsb + U[Ly::U_G + (1 + a) * D1 + 1 + b]);
    if (kp.cost) {   // H(α/c) = (Hα − ∇f∇cᵀ − ∇c∇fᵀ)/c − (α/c²)Hc, ∇f = U_GAL (weighted)
      double gc[D];
      (void)cost_eval<D>(kp, x, gc);
      const double gca = lane_pick<D>(gc, a), gcb = lane_pick<D>(gc, b);
      const double c = U[Ly::U_SC + SC_COSTC], araw = U[Ly::U_SC + SC_ARAW];
      hv = (hv - U[Ly::U_GAL + a] * gcb - gca * U[Ly::U_GAL + b]) / c - (araw / (c * c)) * cost_hess<D>(kp, c, a, b);
    }
    U[Ly::U_H + a * D + b] = hv;
    U[Ly::U_H + b * D + a] = hv;
    if constexpr (Ly::NH <= Ly::LANES) break;
  }
  wave_sync();
  STAMP(W, 7);
  return 1;
}

// ================================================================================
// condition!(fs, x, y) -- radial_basis_surrogates.jl:431-441, after an EV_DRAW eval at x
// on surface S = nf-1.  Appends the inverse-factor row and the new coefficient vector.
// ================================================================================
template <int D, int RPL, int HW>
__device__ __forceinline__ int condition(WaveCtx<D, RPL, HW>& W, const KParams& kp, int S, double yv, const double* gy,
                         const LaneRes<D, RPL, HW>& lr) {
  using Ly = Lay<D, RPL, HW>;
  constexpr int NR = Ly::NR;
  double* U = W.U;
  const int lane = W.ln();
  const int nf = S + 1;   // index of the new fantasy row
  const double g00 = U[Ly::U_G];
  const double mu = U[Ly::U_SC + SC_MU];
  const double l22sq = KCV(PSI0) + KCV(SN2) - g00;   // C - L21·L21 (update_cholesky! :405-418)
  if (!(l22sq > 0.0)) return 4;                  // PosDefException
  const double inv = 1.0 / sqrt(l22sq);
  const double gam = (yv - mu) / l22sq;          // c_new = [c - γ w; γ]
#pragma unroll
  for (int s = 0; s < RPL; ++s) {
    const int i = lane + WAVE * s;
    W.E[(long long)nf * Ly::NRL + i] = W.rowv(kp, s) ? -lr.w[s] * inv : 0.0;
    W.C[(long long)(S + 2) * Ly::NRL + i] = W.rowv(kp, s) ? (lr.cb[s] - gam * lr.w[s]) : 0.0;
  }
  wave_sync();
  if (lane < nf) {
    const double wq = U[Ly::U_WF + lane];
    U[Ly::U_DINV + nf * FMAX + lane] = -wq * inv;
    U[Ly::U_CF + (S + 2) * FMAX + lane] = U[Ly::U_CF + (S + 1) * FMAX + lane] - gam * wq;
  }
  if (lane == nf) {
    U[Ly::U_DINV + nf * FMAX + nf] = inv;
    U[Ly::U_CF + (S + 2) * FMAX + nf] = gam;
    U[Ly::U_YF + nf] = yv;
    const double fm = U[Ly::U_FMIN + S + 1];
    U[Ly::U_FMIN + S + 2] = (yv < fm) ? yv : fm;
  }
  double gmine = 0.0;   // gy[lane] by unrolled select: a runtime index would put gy in scratch
#pragma unroll
  for (int a = 0; a < D; ++a) gmine = (a == lane) ? gy[a] : gmine;
  if (lane < D) {
    U[Ly::U_XF + nf * D + lane] = U[Ly::U_X + lane];
    U[Ly::U_GF + nf * D + lane] = gmine;
  }
  wave_sync();
  return 0;
}

// gp_draw with gradient (r_b_s.jl:588-611): [y;∇y] = [μ;∇μ] + chol(Dk(0) − G)·z.
// Every lane computes the (d+1)² Cholesky redundantly (wave-uniform registers).
template <int D, int RPL, int HW>
__device__ __forceinline__ int draw(WaveCtx<D, RPL, HW>& W, const KParams& kp, const double* z, double& yv, double* gy) {
  using Ly = Lay<D, RPL, HW>;
  constexpr int D1 = Ly::D1;
  const double* U = W.U;
  double Lc[D1 * (D1 + 1) / 2];
#define TRI(i, j) ((i) * ((i) + 1) / 2 + (j))
#pragma unroll
  for (int j = 0; j < D1; ++j) {
    // Symmetric(σx) uses the upper triangle: σx[j][i] for i ≥ j
    const double kjj = (j == 0) ? KCV(PSI0) : -KCV(D2PSI0);
    double sdiag = kjj - U[Ly::U_G + j * D1 + j];
#pragma unroll
    for (int k = 0; k < j; ++k) sdiag -= Lc[TRI(j, k)] * Lc[TRI(j, k)];
    if (!(sdiag > 0.0)) return 2;
    double ljj, ij;
    sqrt_rsqrt(sdiag, ljj, ij);
    Lc[TRI(j, j)] = ljj;
#pragma unroll
    for (int i = j + 1; i < D1; ++i) {
      double t = -U[Ly::U_G + j * D1 + i];
#pragma unroll
      for (int k = 0; k < j; ++k) t -= Lc[TRI(i, k)] * Lc[TRI(j, k)];
      Lc[TRI(i, j)] = t * ij;
    }
  }
  double out[D1];
  out[0] = U[Ly::U_SC + SC_MU];
#pragma unroll
  for (int a = 0; a < D; ++a) out[1 + a] = U[Ly::U_GMU + a];
#pragma unroll
  for (int a = 0; a < D1; ++a) {
    double s = 0.0;
#pragma unroll
    for (int k = 0; k <= a; ++k) s += Lc[TRI(a, k)] * z[k];
    out[a] += s;
  }
#undef TRI
  yv = out[0];
#pragma unroll
  for (int a = 0; a < D; ++a) gy[a] = out[1 + a];
  return 0;
}

// ================================================================================
// Inner solve: deterministic projected Newton on f = -α, surface S.
// ================================================================================
// packed lower Cholesky in place; idg receives the reciprocals of the diagonal
// The first non-positive pivot ends the factorization (wave-uniform branch): the caller discards
// A then -- the Gershgorin retry refills it -- so the remaining columns would be wasted issue.
template <int D>
__device__ __forceinline__ bool chol_packed(double (&A)[D * (D + 1) / 2], double (&idg)[D]) {
#define TRI(i, j) ((i) * ((i) + 1) / 2 + (j))
  bool ok = true;
#pragma unroll
  for (int j = 0; j < D; ++j) {
    double s = A[TRI(j, j)];
#pragma unroll
    for (int k = 0; k < j; ++k) s -= A[TRI(j, k)] * A[TRI(j, k)];
    ok = ok && (s > 0.0);
#ifndef MRBO_NO_CHOL_EXIT
    if (!ok) return false;
#endif
    double ljj;
    sqrt_rsqrt(s, ljj, idg[j]);
    A[TRI(j, j)] = ljj;
#pragma unroll
    for (int i = j + 1; i < D; ++i) {
      double t = A[TRI(i, j)];
#pragma unroll
      for (int k = 0; k < j; ++k) t -= A[TRI(i, k)] * A[TRI(j, k)];
      A[TRI(i, j)] = t * idg[j];
    }
  }
#undef TRI
  return ok;
}

// Projected-gradient test of the Newton iteration: max |g_a| over the free coordinates > g_tol,
// i.e. some free coordinate's |g_a| exceeds g_tol (NaN components count in neither form).  Lane
// a < D tests coordinate a; the free set (bit a: coordinate a free, i.e. not at a bound with the
// gradient pushing out of the box) is kept in U_SC + SC_FREE for the direction that follows.
template <int D, int RPL, int HW>
__device__ __forceinline__ bool newton_pg_ok(WaveCtx<D, RPL, HW>& W, const KParams& kp) {
  using Ly = Lay<D, RPL, HW>;
  const double* U = W.U;
  const int lane = W.ln();
  const int a = lane < D ? lane : 0;
  const double xs = U[Ly::U_NX + a], gs = U[Ly::U_NG + a], lb = U[Ly::U_LB + a], ub = U[Ly::U_UB + a];
  const bool act = ((xs <= lb) & (gs > 0.0)) | ((xs >= ub) & (gs < 0.0));
  const bool fr = (lane < D) & !act;
  const unsigned long long fm = hw_ballot<HW>(fr, W.half);
  const unsigned long long big = hw_ballot<HW>(fr & (fabs(gs) > KCV(GTOL)), W.half);
  if (lane == 0) W.U[Ly::U_SC + SC_FREE] = (double)(unsigned)fm;
  return big != 0ull;
}

// One projected-Newton direction from the state in U (g = U_NG, H = U_H, the free set of the
// projected-gradient test that just passed in U_SC + SC_FREE).  Writes p to U_NP.
// The reduced Hessian A0 (identity on the active set) is formed once; the Gershgorin shift's row
// sums run over it directly (its masked entries are exact zeros, so the sums are those over the
// free columns).  The two factorisations of the sequential rule -- A0, and on failure A0 + τ on
// the free diagonal -- run at once in the two half-waves (lanes 0-31 factor A0, lanes 32-63 the
// shifted matrix; the shift is formed by every lane from A0 alone), and p comes from lane 0 when
// A0 factored, else from lane 32: the same values as the sequential retry, in the time of one
// factorisation (the retry is taken at ~80-90 % of C3's directions).
// ALL_FREE: every coordinate is free (the common interior case; a wave-uniform branch in
// newton_direction): the masks below are compile-time true and their selects fold away -- the
// same values as the masked form, whose selects then pick the unmasked operand.
template <int D, int RPL, int HW, bool ALL_FREE>
__device__ __forceinline__ bool newton_direction_fm(WaveCtx<D, RPL, HW>& W, const KParams& kp, int fm) {
  using Ly = Lay<D, RPL, HW>;
  constexpr int NH = D * (D + 1) / 2;
  double* U = W.U;
  const int lane = W.ln();
  bool fr[D];
  double gs[D];
#pragma unroll
  for (int a = 0; a < D; ++a) {
    fr[a] = ALL_FREE || ((fm >> a) & 1);
    gs[a] = U[Ly::U_NG + a];
  }
  // masked reduced Hessian of f = -α, packed lower; H read unconditionally (a load under a
  // select becomes a branch with a full LDS round trip per element)
  double A0[NH];
#pragma unroll
  for (int i = 0; i < D; ++i)
#pragma unroll
    for (int j = 0; j <= i; ++j) {
      const double h = U[Ly::U_H + i * D + j];
      A0[i * (i + 1) / 2 + j] = (fr[i] && fr[j]) ? -h : ((i == j) ? 1.0 : 0.0);
    }
  // Gershgorin shift over the free block
  double tau = 0.0, hmax = 0.0;
#pragma unroll
  for (int i = 0; i < D; ++i) {
    double off = 0.0;
#pragma unroll
    for (int j = 0; j < D; ++j)
      if (j != i) off += fabs((j < i) ? A0[i * (i + 1) / 2 + j] : A0[j * (j + 1) / 2 + i]);
    const double hii = A0[i * (i + 1) / 2 + i];
    tau = fr[i] ? fmax(tau, off - hii) : tau;
    hmax = fr[i] ? fmax(hmax, fabs(hii)) : hmax;
  }
  tau += 1e-8 * (1.0 + hmax);
  constexpr int SPLIT = Lay<D, RPL, HW>::LANES / 2;   // the lanes that factor the shifted matrix
  const bool shifted = lane >= SPLIT;
  double A[NH], idg[D];
#pragma unroll
  for (int t = 0; t < NH; ++t) A[t] = A0[t];
#pragma unroll
  for (int i = 0; i < D; ++i) {
    const int ii = i * (i + 1) / 2 + i;
    A[ii] = shifted ? (fr[i] ? A0[ii] + tau : 1.0) : A0[ii];
    idg[i] = 0.0;
  }
  const bool okl = chol_packed<D>(A, idg);
  const bool ok0 = hw_readlane_i<HW>((int)okl, 0, W.half) != 0;
  const bool ok1 = hw_readlane_i<HW>((int)okl, SPLIT, W.half) != 0;
  STAMP(W, 13);
#ifdef MRBO_STAMPS
  if (!ok0) stamp_count(W, STAMP_RETRY, 1);   // Gershgorin retries (taken at ~80 % of C3's Newton directions)
#endif
  STAMP(W, 17);
  const bool ok = ok0 || ok1;
  double p[D];
  if (ok) {
    double t1[D];
#pragma unroll
    for (int i = 0; i < D; ++i) {
      double s = fr[i] ? gs[i] : 0.0;
#pragma unroll
      for (int k = 0; k < i; ++k) s -= A[i * (i + 1) / 2 + k] * t1[k];
      t1[i] = s * idg[i];
    }
#pragma unroll
    for (int i = D - 1; i >= 0; --i) {
      double s = t1[i];
#pragma unroll
      for (int k = i + 1; k < D; ++k) s -= A[k * (k + 1) / 2 + i] * p[k];
      p[i] = s * idg[i];
    }
#pragma unroll
    for (int i = 0; i < D; ++i) p[i] = fr[i] ? -p[i] : 0.0;
  } else {
#pragma unroll
    for (int i = 0; i < D; ++i) p[i] = fr[i] ? -gs[i] : 0.0;
  }
  double pn = 0.0;
#pragma unroll
  for (int i = 0; i < D; ++i) pn = fmax(pn, fabs(p[i]));
  const double box = KCV(BOX);
  const double sc = (pn > box) ? box / pn : 1.0;
  wave_sync();
  if (lane == (ok0 ? 0 : SPLIT)) {
#pragma unroll
    for (int a = 0; a < D; ++a) U[Ly::U_NP + a] = (pn > box) ? p[a] * sc : p[a];
  }
  wave_sync();
  STAMP(W, 18);
  return true;
}

template <int D, int RPL, int HW>
__device__ __forceinline__ bool newton_direction(WaveCtx<D, RPL, HW>& W, const KParams& kp) {
  using Ly = Lay<D, RPL, HW>;
  // the free set of this lane's trajectory (U is per trajectory: in half-wave mode the two halves
  // hold different sets, so the mask stays per lane there); written by the trajectory's lane 0
  int fm = (int)W.U[Ly::U_SC + SC_FREE];
  if constexpr (HW == 1) fm = __builtin_amdgcn_readfirstlane(fm);
#ifndef MRBO_NO_ALLFREE
  if (__builtin_amdgcn_ballot_w64(fm != (1 << D) - 1) == 0ull) return newton_direction_fm<D, RPL, HW, true>(W, kp, fm);
#endif
  return newton_direction_fm<D, RPL, HW, false>(W, kp, fm);
}

// x_t = clamp(x + t p) -> U_X ; returns gᵀ(x_t - x).  Lane a < D computes coordinate a (its own
// LDS loads and clamp, one store); the inner product is then summed in coordinate order from the
// lanes' terms by readlane -- the same fused multiply-adds in the same order as a lane-uniform loop.
template <int D, int RPL, int HW>
__device__ __forceinline__ double newton_trial_point(WaveCtx<D, RPL, HW>& W, double t) {
  using Ly = Lay<D, RPL, HW>;
  double* U = W.U;
  const int lane = W.ln();
  const int a = lane < D ? lane : 0;
  const double xa = U[Ly::U_NX + a];
  const double xt = clampd(xa + t * U[Ly::U_NP + a], U[Ly::U_LB + a], U[Ly::U_UB + a]);
  const double ga = U[Ly::U_NG + a], da = xt - xa;
  wave_sync();
  if (lane < D) U[Ly::U_X + lane] = xt;
  double dec = 0.0;
#pragma unroll
  for (int b = 0; b < D; ++b) dec = fma(hw_readlane_d<HW>(ga, b, W.half), hw_readlane_d<HW>(da, b, W.half), dec);
  wave_sync();
  return dec;
}

// Gradient certificate at a point whose VALUE evaluation is in U: true when ‖∇α‖∞ ≤ g_tol is
// guaranteed, so the Newton iteration stops there whatever the gradient columns hold.
//   ∇α = gμ ∇μ + gσ ∇σ,  |∂_a μ| ≤ Σ|c| max|ψ'|,
//   |∂_a σ| = |kxᵀK⁻¹∂_a kx| / σ ≤ √(kxᵀK⁻¹kx · ∂_a kxᵀK⁻¹∂_a kx) / σ ≤ √(ψ(0)(−ψ''(0))) / σ
// (posterior variances of f and ∂_a f are ≥ 0).  A factor 4 covers rounding.  gμ = gσ = 0
// (σ < σtol, or Φ and φ underflowed) makes ∇α zero or NaN, which also stops the iteration.
template <int D, int RPL, int HW>
__device__ __forceinline__ bool grad_certified(const WaveCtx<D, RPL, HW>& W, const KParams& kp) {
  using Ly = Lay<D, RPL, HW>;
  const double* U = W.U;
  const double gm = U[Ly::U_SC + SC_GMU], gs = U[Ly::U_SC + SC_GSIG];
  const double cabs = U[Ly::U_SC + SC_CABS], isig = U[Ly::U_SC + SC_ISIG];   // unconditional loads
  double bound = fabs(gm) * KCV(GCMU) * cabs + fabs(gs) * KCV(GCSIG) * isig;
  bool zero = (gm == 0.0) & (gs == 0.0);
  if (kp.cost) {   // f = α/c: |∂f| ≤ B/c + |α| max|∇c|/c²; gμ = gσ = 0 certifies only where α = 0
    const double araw = U[Ly::U_SC + SC_ARAW], c = U[Ly::U_SC + SC_COSTC];
    bound = bound * (1.0 / c) + fabs(araw) * U[Ly::U_SC + SC_GCMAX] / (c * c);
    zero = zero & (araw == 0.0);
  }
  return zero | ((kp.gcert_sig > 0.0) & (bound <= 0.25 * KCV(GTOL)));
}

// Tight certificate at x = U[U_X] on surface S, where grad_certified's cheap bound failed
// (gμ, gσ, σ of the value evaluation at x).  At the point itself:
//   |∂_a μ| = |Σ_j c_j g1_j (x − X_j)_a| ≤ Σ_j |c_j| |ψ'(ρ_j)|  over base and fantasy rows,
//   |∂_a σ| ≤ √(−ψ''(0)) √(kxᵀK⁻¹kx) / σ  with kxᵀK⁻¹kx = ψ(0) − σ²,
// i.e. the cheap bound with max|ψ'| replaced by the actual |ψ'(ρ_j)| and ψ(0) by the explained
// variance; far from the data both vanish.  One radial evaluation per row and one reduction --
// instead of the gradient columns (O(N²d)).  Factor 4 for rounding, as above; the oracle
// (rbo_oracle.c grad_certified) applies the same test.
// ROWS_KEPT: the VALUE evaluation at x just ran on surface S, so g1 = ψ'(ρ)/ρ of every base
// row (G12) and fantasy row (U_HF) is still in LDS -- the same bits a new radial evaluation
// would give; only ρ is recomputed.
// With a cost model (f = α/c, araw = α at x) every bound B on |∂α| becomes B/c + |α| max|∇c|/c².
template <int D, int RPL, int HW, bool ROWS_KEPT = false>
__device__ __forceinline__ bool tight_certified(WaveCtx<D, RPL, HW>& W, const KParams& kp, int S, double gm, double gs,
                                                double sig, double isig, double araw = 0.0) {
  using Ly = Lay<D, RPL, HW>;
  constexpr int NR = Ly::NR;
  const double* U = W.U;
  const int lane = W.ln();
  const int nf = S + 1;
  double isc = 1.0, add = 0.0;
  if (kp.cost) {
    double xc[D], gc[D];
#pragma unroll
    for (int a = 0; a < D; ++a) xc[a] = U[Ly::U_X + a];
    const double c = cost_eval<D>(kp, xc, gc);
    double gmax = 0.0;
#pragma unroll
    for (int a = 0; a < D; ++a) gmax = fmax(gmax, fabs(gc[a]));
    isc = 1.0 / c;
    add = fabs(araw) * gmax / (c * c);
  }
  // the σ part needs no rows: if it alone exceeds the threshold the test fails, and with the
  // cheap μ part (Σ|c|·max|ψ'| ≥ the row sum) it may already pass -- same decisions as the
  // full test, without the row pass
  const double q = fmax(KCV(PSI0) - sig * sig, 0.0);
  const double bsig = fabs(gs) * KCV(GCD2) * fast_sqrt0(q) * isig, thr = 0.25 * KCV(GTOL);
  if (!(bsig * isc + add <= thr)) return false;
  if ((fabs(gm) * KCV(GCMU) * U[Ly::U_SC + SC_CABS] + bsig) * isc + add <= thr) return true;
  double x[D];
#pragma unroll
  for (int a = 0; a < D; ++a) x[a] = U[Ly::U_X + a];
  double v[1] = {0.0};
#pragma unroll
  for (int s = 0; s < RPL; ++s) {
    double rho2 = 0.0;
#pragma unroll
    for (int a = 0; a < D; ++a) { const double r = x[a] - W.x0(kp, s, a); rho2 = fma(r, r, rho2); }
    double psi, g1, g2;
    if constexpr (ROWS_KEPT) g1 = W.G12[3 * (lane + WAVE * s)];
    else rad_eval(W.rad, rho2, psi, g1, g2);
    const double cb = W.C[(long long)(S + 1) * Ly::NRL + lane + WAVE * s];
    v[0] += W.rowv(kp, s) ? fabs(cb) * fabs(g1) * fast_sqrt0(rho2) : 0.0;
  }
  if (lane < nf) {
    double rho2 = 0.0;
#pragma unroll
    for (int a = 0; a < D; ++a) { const double r = x[a] - U[Ly::U_XF + lane * D + a]; rho2 = fma(r, r, rho2); }
    double psi, g1, g2;
    if constexpr (ROWS_KEPT) g1 = U[Ly::U_HF + lane * (D + 2) + D];
    else rad_eval(W.rad, rho2, psi, g1, g2);
    v[0] += fabs(U[Ly::U_CF + (S + 1) * FMAX + lane]) * fabs(g1) * fast_sqrt0(rho2);
  }
  const double bmu = hw_allreduce1<HW>(v[0]);
  return (fabs(gm) * bmu + bsig) * isc + add <= thr;
}

// Deterministic projected Newton on f = -α over the box, from start k.
// A state machine around ONE evaluate() call site.  Work is lazy, decisions are not: every
// point gets a value-only evaluation; the gradient columns are completed (GRADC) only where
// the certificate cannot rule out a step, the backward product and Hα (BACK) only where a
// step is taken.  Values and gradients are bit-identical to a FULL evaluation at the same
// point (same code path), so the iterates are those of the eager iteration, and the work
// counts equal the oracle's (rbo_oracle.c newton_solve).  Result: x in U_NX, f returned.
template <int D, int RPL, int HW>
__device__ __forceinline__ double newton(WaveCtx<D, RPL, HW>& W, const KParams& kp, int S, int k, Counters& nevals,
                                         int& st, LaneRes<D, RPL, HW>& lr, double f0, bool have_f0, double gm0 = 0.0,
                                         double gs0 = 0.0, double sig0 = 0.0, double a0 = 0.0) {
  using Ly = Lay<D, RPL, HW>;
  double* U = W.U;
  const int lane = W.ln();
  enum { P_VAL = 0, P_TRIAL = 1, P_GRAD = 2, P_HESS = 3 };
#ifdef MRBO_NO_FUSE_BACK
  constexpr bool FUSE_BACK = false;
#else
  constexpr bool FUSE_BACK = true;   // GRAD + BACK in one evaluation call (evaluate back_after)
#endif
  if (lane < D) {
    const double xa = clampd(W.XS[(long long)k * D + lane], U[Ly::U_LB + lane], U[Ly::U_UB + lane]);
    U[Ly::U_NX + lane] = xa;
    U[Ly::U_X + lane] = xa;
  }
  wave_sync();
  // a batched start whose cheap certificate failed: the tight one at x_start (gμ, gσ, σ of the
  // batched value) before any gradient work
  if (have_f0 && kp.gcert_sig > 0.0 && tight_certified<D, RPL, HW>(W, kp, S, gm0, gs0, sig0, 1.0 / sig0, a0)) {
    wave_sync();
    return f0;
  }
  // have_f0: the start's value (and certificate) came from batch_start_values and did not
  // stop the iteration, so it begins with the gradient at x_start
  // (GSTART takes the base forward product from the square layout's per-workgroup tables; the
  // packed layouts evaluate the gradient at the start point in full)
  int phase = have_f0 ? P_GRAD : P_VAL, mode = have_f0 ? (Ly::SQ ? EV_GSTART : EV_GRAD) : EV_VALUE, it = 0, ls = 0;
  double f = have_f0 ? f0 : 0.0, ft = 0.0, t = 1.0, dec = 0.0;
  for (;;) {
    const int back = evaluate<D, RPL, HW>(W, kp, S, mode, lr, k, FUSE_BACK && phase == P_GRAD);
    if (mode == EV_VALUE) ++nevals.value;
    else if (mode == EV_GRADC || mode == EV_GRAD || mode == EV_GSTART) ++nevals.grad;
    else ++nevals.hess;
    if (FUSE_BACK && phase == P_GRAD) {   // the projected-gradient test ran inside the evaluation
      if (!back) break;                   // stationary
      ++nevals.hess;                      // the BACK part (Hα) ran in the same call
      phase = P_HESS;
    }
    if (phase == P_HESS) {                 // Hα at x ready: step
      STAMP(W, 12);
      const bool go = newton_direction<D, RPL, HW>(W, kp);
      STAMP(W, 13);
      if (!go) break;
      t = 1.0;
      ls = 0;
      dec = newton_trial_point<D, RPL, HW>(W, t);
      STAMP(W, 14);
      phase = P_TRIAL;
      mode = EV_VALUE;
      continue;
    }
    if (phase == P_GRAD) {                 // ∇α at x ready
      if (lane < D) U[Ly::U_NG + lane] = -U[Ly::U_GAL + lane];
      wave_sync();
      if (!newton_pg_ok<D, RPL, HW>(W, kp)) break;     // stationary
      STAMP(W, 21);
      phase = P_HESS;
      mode = EV_BACK;
      continue;
    }
    // a VALUE evaluation: the start point (P_VAL) or a line-search trial (P_TRIAL)
    if (U[Ly::U_SC + SC_VAR] < 0.0) st |= 1;
    const double fe = -U[Ly::U_SC + SC_ALPHA];
    if (phase == P_TRIAL) {
      ft = fe;
      if (!(ft == ft && ft <= f + 1e-4 * dec)) {   // projected Armijo, backtrack
        ++ls;
        if (ls >= kp.max_ls) break;                // no acceptable step
        t *= 0.5;
        dec = newton_trial_point<D, RPL, HW>(W, t);
        continue;
      }
      // accept x_t: lane a < D moves its coordinate; ‖Δx‖∞ from the lanes' |Δx_a| (max: order-free)
      const int ca = lane < D ? lane : 0;
      const double xt = U[Ly::U_X + ca];
      const double dxa = fabs(xt - U[Ly::U_NX + ca]);
      double dx = 0.0;
#pragma unroll
      for (int a = 0; a < D; ++a) dx = fmax(dx, hw_readlane_d<HW>(dxa, a, W.half));
      const double df = fabs(ft - f);
      wave_sync();
      if (lane < D) U[Ly::U_NX + lane] = xt;
      wave_sync();
      f = ft;
      ++it;
      if (dx <= KCV(XTOL) || df <= KCV(FTOL) * fabs(f)) break;
    } else {
      f = fe;
    }
    STAMP(W, 19);
    // decision point at x = U_NX (= U_X), whose VALUE evaluation is in U
    if (it >= kp.max_iters) break;
    if (f != f) break;
    if (grad_certified<D, RPL, HW>(W, kp)) break;     // ‖∇α‖ ≤ g_tol guaranteed: stationary
    if (kp.gcert_sig > 0.0 &&
        tight_certified<D, RPL, HW, true>(W, kp, S, U[Ly::U_SC + SC_GMU], U[Ly::U_SC + SC_GSIG], U[Ly::U_SC + SC_SIG],
                                      U[Ly::U_SC + SC_ISIG], kp.cost ? U[Ly::U_SC + SC_ARAW] : 0.0))
      break;
    STAMP(W, 20);
    phase = P_GRAD;
    mode = EV_GRADC;
  }
  wave_sync();
  return f;
}

// Workgroup prologue (kp.batch): base kernel rows of the clamped start points and the squared
// norms of their forward products -- constants of the launch shared by every multistart.
//   kxb[i][k] = ψ(|x_k − X_i|) (0 on padded rows);  per start, Y = L0⁻¹[kx, ∇kx](x_k):
//   base Gram YᵀY → gtab (LDS); with store_y (ytab_kernel only) Y0 → the launch's table kp.ytab
// The per-wave areas (not yet initialised) serve as scratch for the squares.
template <int D, int RPL, int HW>
__device__ __forceinline__ void stage_start_tables(const KParams& kp, double* smem, bool store_y) {
  using Ly = Lay<D, RPL, HW>;
  constexpr int NR = Ly::NR;
  const WgTables<D, RPL, HW> tb(kp);
  const int ns = kp.nstarts;
  const double* xs = smem + tb.xs;
  double* kxb = smem + tb.kxb;
  Radial rad;
  rad.kind = kp.kernel;
  rad.cK = kp.cK;
  rad.cP = kp.cP;
  for (int q = threadIdx.x; q < NR * ns; q += blockDim.x) {
    const int i = q / ns, k = q - (q / ns) * ns;
    double v = 0.0;
    if (i < kp.N) {
      double rho2 = 0.0;
#pragma unroll
      for (int a = 0; a < D; ++a) {
        const double r = clampd(xs[k * D + a], kp.lbs[a], kp.ubs[a]) - kp.X0[(long long)a * NR + i];
        rho2 = fma(r, r, rho2);
      }
      double g1, g2;
      rad_eval(rad, rho2, v, g1, g2);
    }
    kxb[q] = v;
  }
  __syncthreads();
  // per start (waves in turn): Y = L0⁻¹[kx, ∇kx](x_k) by the register-broadcast product, the base
  // Gram YᵀY (upper triangle) to gtab, and (store_y) Y0 to the launch's table
  const int lane = threadIdx.x & (WAVE - 1), wv = threadIdx.x / WAVE, nw = blockDim.x / WAVE;
  double* red = smem + tb.end + (long long)wv * Ly::WAVE_LDS;   // wave-area scratch
  // One Y0 table for the launch, written once by ytab_kernel (one workgroup, launched before the
  // rollout kernel on the same stream, running this same code) and only read by the rollout
  // workgroups.  Round 5 had every rollout workgroup write the same bits to the shared slice (a
  // benign but formal race); per-workgroup slices had cost 2.4 MB of HBM writes per C3 launch.
  double* ytab = kp.ytab;
  for (int k = wv; k < ns; k += nw) {
    double bv[Ly::D1], acc[Ly::D1];
    double rho2 = 0.0, r[D];
#pragma unroll
    for (int a = 0; a < D; ++a) {
      r[a] = clampd(xs[k * D + a], kp.lbs[a], kp.ubs[a]) - kp.X0[(long long)a * NR + lane];
      rho2 = fma(r[a], r[a], rho2);
    }
    double psi, g1, g2;
    rad_eval(rad, rho2, psi, g1, g2);
    const bool v = lane < kp.N;
    bv[0] = v ? psi : 0.0;
#pragma unroll
    for (int a = 0; a < D; ++a) bv[1 + a] = v ? g1 * r[a] : 0.0;
#pragma unroll
    for (int c = 0; c < Ly::D1; ++c) acc[c] = 0.0;
    bcast_product<Ly::D1, Ly::LD>(acc, bv, smem + lane, kp.N);
    if (store_y) ytab[(long long)k * NR + lane] = acc[0];
#pragma unroll
    for (int ch = 0; ch < (Ly::NG + 15) / 16; ++ch) {
      double gv[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int t = 16 * ch + q;
        double s_ = 0.0;
        if (t < Ly::NG) {
          int a = 0, rem = t;
#pragma unroll
          for (int aa = 0; aa < Ly::D1; ++aa) if (a == aa && rem >= Ly::D1 - aa) { rem -= Ly::D1 - aa; a = aa + 1; }
          s_ = acc[a] * acc[a + rem];
        }
        gv[q] = s_;
      }
      wave_reduce<16>(gv, red + 16 * ch, lane);
    }
    wave_sync();
    for (int t = lane; t < Ly::NG; t += WAVE) smem[tb.gtab + (long long)k * Ly::NG + t] = red[t];
    wave_sync();
  }
  __syncthreads();
}

// Values of ALL start points of a multistart on surface S at once (kp.batch): lane k takes start
// k.  With the launch constants kxb, gtab only the surface-dependent parts remain:
//   μ_k = c_S·kxb[:,k] + Σ_r c_r ψ(x_k, X_r),  Yf_r = E_r·kxb[:,k] + Σ_{q≤r} Dinv[r][q] ψ(x_k, X_q),
//   σ_k² = ψ(0) − gtab[k][0] − Σ_r Yf_r²,  then α and the gradient certificate per lane.
// Replaces nstarts value evaluations (and their wave-redundant EI) by one pass.
template <int D, int RPL, int HW>
__device__ __forceinline__ void batch_start_values(WaveCtx<D, RPL, HW>& W, const KParams& kp, int S, double& f_lane,
                                                   double& gm_lane, double& gs_lane, double& sig_lane,
                                                   double& a_lane, unsigned long long& stopmask,
                                                   unsigned long long& xnanmask, bool& varneg) {
  using Ly = Lay<D, RPL, HW>;
  constexpr int NR = Ly::NR;
  const double* U = W.U;
  const int lane = W.ln();
  const int ns = kp.nstarts, nf = S + 1;
#ifndef MRBO_NO_BATCH_SPLIT
  // ns ≤ 32: both half-waves take every start (lane k and k + 32); the lower half sums the
  // even data rows, the upper half the odd ones, one permlane32 swap per value adds the halves,
  // and each half evaluates every other fantasy radial function.  Both halves then hold the
  // same per-start values; the ballots below read the lower half.
  const bool split = HW == 1 && ns <= 32;   // half-wave mode: each half takes every start itself
#else
  const bool split = false;
#endif
  const int kl = split ? (lane & 31) : lane;
  const int hf = split ? (lane >> 5) : 0;
  const bool act = lane < ns;
  const int k = kl < ns ? kl : 0;
  double x[D];
#pragma unroll
  for (int a = 0; a < D; ++a) x[a] = clampd(W.XS[k * D + a], U[Ly::U_LB + a], U[Ly::U_UB + a]);
  double amu = 0.0, ae[FMAX];
#pragma unroll
  for (int r = 0; r < FMAX; ++r) ae[r] = 0.0;
  const double* cS = W.C + (long long)(S + 1) * Ly::NRL;
  // all FMAX rows unconditionally (rows ≥ nf hold finite stale values, masked below): a load
  // under a condition would become a branch with a full LDS round trip per row.  Rows N..NR-1
  // of the tables are zero.
  if constexpr (!Ly::SQ) {
    // packed layouts (E, c and the kernel-row table in global memory): lanes own data rows and
    // the starts run in a loop, so every load is a coalesced row walk (a lane-per-start loop over
    // rows would chain NR dependent global round trips).  Per start the 1 + FMAX base products
    // [c_S·kxb_k, E_r·kxb_k] are transpose-reduced (two starts per 16-value reduction) into the
    // wave's global scratch (after E / C in its work slot), then lane k reads its start's sums.
    double cv[RPL], ev[RPL][FMAX];
#pragma unroll
    for (int s2 = 0; s2 < RPL; ++s2) {
      const int i = lane + WAVE * s2;
      cv[s2] = cS[i];
#pragma unroll
      for (int r = 0; r < FMAX; ++r) ev[s2][r] = W.E[(long long)r * Ly::NRL + i];
    }
    double* sums = W.SUMS;   // [ns][8]
    // the kernel-row table entries of the next pair of starts are loaded while this pair is
    // reduced (one L2 round trip in flight behind the reduction instead of one per pair)
    auto load_pair = [&](int kc, double (&kxp)[2][RPL]) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int kq = (kc + kk < ns) ? kc + kk : (kc < ns ? kc : 0);
#pragma unroll
        for (int s2 = 0; s2 < RPL; ++s2) kxp[kk][s2] = W.KXB[(long long)kq * NR + lane + WAVE * s2];
      }
    };
    double kxn[2][RPL];
    load_pair(0, kxn);
    for (int kc = 0; kc < ns; kc += 2) {
      double kxc[2][RPL];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int s2 = 0; s2 < RPL; ++s2) kxc[kk][s2] = kxn[kk][s2];
      load_pair(kc + 2, kxn);
      double v[16];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const double* kx = kxc[kk];
        double a0 = 0.0;
#pragma unroll
        for (int s2 = 0; s2 < RPL; ++s2) a0 = fma(cv[s2], kx[s2], a0);
        v[8 * kk] = a0;
#pragma unroll
        for (int r = 0; r < FMAX; ++r) {
          double a = 0.0;
#pragma unroll
          for (int s2 = 0; s2 < RPL; ++s2) a = fma(ev[s2][r], kx[s2], a);
          v[8 * kk + 1 + r] = a;
        }
        v[8 * kk + 7] = 0.0;
      }
      wave_reduce<16>(v, sums + 8 * kc, lane);
    }
    wave_sync();
    amu = sums[8 * k];
#pragma unroll
    for (int r = 0; r < FMAX; ++r) ae[r] = sums[8 * k + 1 + r];
    wave_sync();   // sums read before the scratch is reused
  } else if (split) {
#pragma unroll 8
    for (int j = 0; j < NR / 2; ++j) {
      const int i = 2 * j + hf;
      const double kv = W.KXB[i * ns + k];
      amu = fma(cS[i], kv, amu);
#pragma unroll
      for (int r = 0; r < FMAX; ++r) ae[r] = fma(W.E[(long long)r * Ly::NRL + i], kv, ae[r]);
    }
    amu = swap_fold<32>(amu, amu);
#pragma unroll
    for (int r = 0; r < FMAX; ++r) ae[r] = swap_fold<32>(ae[r], ae[r]);
  } else {
#pragma unroll 8
    for (int i = 0; i < W.N; ++i) {
      const double kv = W.KXB[i * ns + k];
      amu = fma(cS[i], kv, amu);
#pragma unroll
      for (int r = 0; r < FMAX; ++r) ae[r] = fma(W.E[(long long)r * Ly::NRL + i], kv, ae[r]);
    }
  }
  double pf[FMAX];
  if (split) {
    // half h evaluates fantasy points q = 2e + h; one swap hands each half the other's values
#pragma unroll
    for (int e = 0; e < FMAX / 2; ++e) {
      const int q = 2 * e + hf;
      double v = 0.0;
      if (2 * e < nf) {
        double rho2 = 0.0;
#pragma unroll
        for (int a = 0; a < D; ++a) { const double r = x[a] - U[Ly::U_XF + q * D + a]; rho2 = fma(r, r, rho2); }
        double g1, g2;
        rad_eval(W.rad, rho2, v, g1, g2);
      }
      self_swap<32, false>(v, pf[2 * e], pf[2 * e + 1]);   // lower half's value (q = 2e), upper half's (2e + 1)
    }
#pragma unroll
    for (int q = 0; q < FMAX; ++q) pf[q] = (q < nf) ? pf[q] : 0.0;
  } else {
#pragma unroll
    for (int q = 0; q < FMAX; ++q) {
      pf[q] = 0.0;
      if (q < nf) {
        double rho2 = 0.0;
#pragma unroll
        for (int a = 0; a < D; ++a) { const double r = x[a] - U[Ly::U_XF + q * D + a]; rho2 = fma(r, r, rho2); }
        double g1, g2;
        rad_eval(W.rad, rho2, pf[q], g1, g2);
      }
    }
  }
  double g00 = W.GTAB[k * Ly::NG], mu = amu;
#pragma unroll
  for (int r = 0; r < FMAX; ++r) {
    if (r < nf) {
      double y = ae[r];
#pragma unroll
      for (int q = 0; q <= r; ++q) y = fma(U[Ly::U_DINV + r * FMAX + q], pf[q], y);
      g00 = fma(y, y, g00);
      mu = fma(U[Ly::U_CF + (S + 1) * FMAX + r], pf[r], mu);
    }
  }
  const double var = KCV(PSI0) - g00;
  double sig, isig;
  sig_isig(var, sig, isig);
  const EIp e = rule_partials(kp.rule, mu, sig, KCV(THETA), U[Ly::U_FMIN + S + 1], KCV(SIGTOL), isig);
  double fval = e.g, cval = 1.0, gcm = 0.0;
  if (kp.cost) {   // cost-weighted rule at the start point (see grad_certified)
    double gc[D];
    cval = cost_eval<D>(kp, x, gc);
#pragma unroll
    for (int a = 0; a < D; ++a) gcm = fmax(gcm, fabs(gc[a]));
    fval = e.g / cval;
  }
  bool cert = (e.gmu == 0.0 && e.gsig == 0.0) && (!kp.cost || e.g == 0.0);
  if (!cert && kp.gcert_sig > 0.0) {
    double b = fabs(e.gmu) * KCV(GCMU) * U[Ly::U_SC + SC_CABS] + fabs(e.gsig) * KCV(GCSIG) * isig;
    if (kp.cost) b = b * (1.0 / cval) + fabs(e.g) * gcm / (cval * cval);
    cert = b <= 0.25 * KCV(GTOL);
  }
  f_lane = -fval;
  a_lane = e.g;
  gm_lane = e.gmu;
  gs_lane = e.gsig;
  sig_lane = sig;
  // the iteration stops at the start point: certified, f NaN, or no iterations allowed
  const bool stop = cert || (f_lane != f_lane) || kp.max_iters <= 0;
  bool xn = false;
#pragma unroll
  for (int a = 0; a < D; ++a) xn = xn || (x[a] != x[a]);
  stopmask = hw_ballot<HW>(act && stop, W.half);
  xnanmask = hw_ballot<HW>(act && xn, W.half);
  varneg = hw_ballot<HW>(act && var < 0.0, W.half) != 0;
}

// multistart_base_solve!(fs, …) rbf_optim.jl:68-101 -> U[U_XB], over the starts k0 ≤ k < k1.
// kp.base_solve: one start per launch item, whose (minimizer, minimum) is the output -- the
// candidate list multistart_base_solve!(s::Surrogate, …) (:103-135) takes its findmin over.
template <int D, int RPL, int HW>
__device__ __forceinline__ int multistart(WaveCtx<D, RPL, HW>& W, const KParams& kp, int S, Counters& nevals,
                                          LaneRes<D, RPL, HW>& lr, int k0, int k1) {
  using Ly = Lay<D, RPL, HW>;
  double* U = W.U;
  const int lane = W.ln();
  int st = 0;
  int best = -1;
  bool best_nan = false;
  double bestf = 0.0;
  {   // Σ|c| of surface S (base + fantasy coefficients) for the gradient certificate
    double v[1] = {0.0};
#pragma unroll
    for (int s = 0; s < RPL; ++s) v[0] += fabs(W.C[(long long)(S + 1) * Ly::NRL + lane + WAVE * s]);
    double cabs = hw_allreduce1<HW>(v[0]);
    for (int r = 0; r <= S; ++r) cabs += fabs(U[Ly::U_CF + (S + 1) * FMAX + r]);
    if (lane == 0) U[Ly::U_SC + SC_CABS] = cabs;
    wave_sync();
  }
  double f_lane = 0.0, gm_lane = 0.0, gs_lane = 0.0, sig_lane = 0.0, a_lane = 0.0;
  unsigned long long stopmask = 0, xnanmask = 0;
  if (kp.batch) {
    bool varneg = false;
    STAMP(W, 16);
    batch_start_values<D, RPL, HW>(W, kp, S, f_lane, gm_lane, gs_lane, sig_lane, a_lane, stopmask, xnanmask, varneg);
    STAMP(W, 15);
    nevals.value += kp.nstarts;
    if (varneg) st |= 1;
    wave_sync();
  }
  // starts that need a Newton iteration, in index order (all of them without kp.batch)
  for (int k = k0; k < k1; ++k) {
    if ((stopmask >> k) & 1ull) continue;
    const double fo = kp.batch ? newton<D, RPL, HW>(W, kp, S, k, nevals, st, lr, hw_lane_d<HW>(f_lane, k, W.half), true,
                                                hw_lane_d<HW>(gm_lane, k, W.half), hw_lane_d<HW>(gs_lane, k, W.half),
                                                hw_lane_d<HW>(sig_lane, k, W.half),
                                                kp.cost ? hw_lane_d<HW>(a_lane, k, W.half) : 0.0)
                               : newton<D, RPL, HW>(W, kp, S, k, nevals, st, lr, 0.0, false);
    if (kp.base_solve) {   // (Optim.minimizer(res), minimum(res)) of base_solve, rbf_optim.jl:127-128
      if (lane < D) kp.policy[(long long)k * D + lane] = U[Ly::U_NX + lane];
      if (lane == 0) kp.values[k] = fo;
    }
    bool xnan = false;
#pragma unroll
    for (int a = 0; a < D; ++a) xnan = xnan || (U[Ly::U_NX + a] != U[Ly::U_NX + a]);
    if (xnan) continue;
    bool take = false;
    if (fo != fo) {
      if (!best_nan) { best_nan = true; best = k; take = true; }
    } else if (!best_nan && (best < 0 || fo < bestf)) {
      best = k;
      bestf = fo;
      take = true;
    }
    if (take) {
      if (lane < D) U[Ly::U_XB + lane] = U[Ly::U_NX + lane];
      wave_sync();
    }
  }
  if (stopmask) {
    // starts that stopped at x = clamp(x_start) with f = f_lane, merged under findmin's order
    // semantics (rbf_optim.jl:96-98): the first NaN f wins, else the first minimum; NaN x dropped
    const int ns = kp.nstarts;
    const bool mine = lane < ns && ((stopmask >> lane) & 1ull) && !((xnanmask >> lane) & 1ull);
    const unsigned long long nanm = hw_ballot<HW>(mine && f_lane != f_lane, W.half);
    int win = -1;
    bool win_nan = false;
    if (nanm) {
      const int kn = __builtin_ctzll(nanm);
      if (!best_nan || kn < best) { win = kn; win_nan = true; }
    } else if (!best_nan) {
      const double m = lanes_min<Lay<D, RPL, HW>::LANES>(mine ? f_lane : INFINITY);
      const unsigned long long eq = hw_ballot<HW>(mine && f_lane == m, W.half);
      if (eq) {
        const int km = __builtin_ctzll(eq);
        if (best < 0 || m < bestf || (m == bestf && km < best)) win = km;
      }
    }
    if (win >= 0) {
      if (lane < D) U[Ly::U_XB + lane] = clampd(W.XS[win * D + lane], U[Ly::U_LB + lane], U[Ly::U_UB + lane]);
      wave_sync();
      best = win;
      best_nan = best_nan || win_nan;
    }
    STAMP(W, 16);
  }
  if (st) return st;
  if (best < 0 && !best_nan) return 8;
  wave_sync();
  return 0;
}

// ================================================================================
// Adjoint pair (i, q): perturb fantasy point q (data index N+q) in the surface S=i-1
// seen from x_i (RICH eval in U/lr).  Lane k < D handles spatial direction e_k and adds
// dri[:,k]'·x̄_i to ACC[q][k]; lane D handles the data direction δx and adds to ȳ_q.
// Reference: SpatialPerturbationSurrogate r_b_s.jl:652-694, DataPerturbation :711-757,
// solve_dual_x rollout.jl:173-186, solve_dual_y :135-145, gather_g :199-215.
// ================================================================================
template <int D, int RPL, int HW>
__device__ __forceinline__ void adjoint_pair(WaveCtx<D, RPL, HW>& W, const KParams& kp, int S, int q, int i_pol,
                             const LaneRes<D, RPL, HW>& lr) {
  using Ly = Lay<D, RPL, HW>;
  constexpr int NR = Ly::NR;
  double* U = W.U;
  double* red = W.red;
  const int lane = W.ln();
  const int nf = S + 1;
  STAMP(W, 8);
  double Xq[D];
#pragma unroll
  for (int a = 0; a < D; ++a) Xq[a] = U[Ly::U_XF + q * D + a];
  // per-lane U_a = ∇k(X_q - X_a) and products  [Uᵀc (D), Uᵀw (D), PᵀU (D×D, m-major)]
  double u[RPL][D];
#pragma unroll
  for (int s = 0; s < RPL; ++s) {
    double r[D], rho2 = 0.0;
#pragma unroll
    for (int a = 0; a < D; ++a) { r[a] = Xq[a] - W.x0(kp, s, a); rho2 = fma(r[a], r[a], rho2); }
    double psi, g1, g2;
    rad_eval(W.rad, rho2, psi, g1, g2);
#pragma unroll
    for (int a = 0; a < D; ++a) u[s][a] = W.rowv(kp, s) ? g1 * r[a] : 0.0;
  }
  wave_sync();
#pragma unroll
  for (int ch = 0; ch < Ly::NPC; ++ch) {
    double v[16];
#pragma unroll
    for (int qq = 0; qq < 16; ++qq) {
      const int t = 16 * ch + qq;
      double s_ = 0.0;
      if (t < D) {
#pragma unroll
        for (int s = 0; s < RPL; ++s) s_ = fma(lr.cb[s], u[s][t], s_);
      } else if (t < 2 * D) {
#pragma unroll
        for (int s = 0; s < RPL; ++s) s_ = fma(lr.w[s], u[s][t - D], s_);
      } else if (t < Ly::NPAIR) {
        const int m = (t - 2 * D) / D, k = (t - 2 * D) % D;
#pragma unroll
        for (int s = 0; s < RPL; ++s) s_ = fma(lr.P[s][m], u[s][k], s_);
      }
      v[qq] = s_;
    }
    hw_reduce<HW, 16>(v, red + 16 * ch, lane);
  }
  wave_sync();
  if (lane > D) { STAMP(W, 9); return; }
  // direction δ: e_lane (spatial) or δx (data, lane D).  Needed: u·c, u·w and Pᵀu for
  // u_a = ∇k(X_q − X_a)·δ over the surface's data; base rows come from the reduction, the
  // fantasy rows r ≤ S are added here (∇k(X_q − X_q) = 0 drops r = q).
  double dl[D];
#pragma unroll
  for (int a = 0; a < D; ++a) {
    const double dxa = U[Ly::U_DX + a];
    dl[a] = (lane == D) ? dxa : ((a == lane) ? 1.0 : 0.0);
  }
  double udc = 0.0, udw = 0.0, Pu[D];
#pragma unroll
  for (int k = 0; k < D; ++k) { udc = fma(red[k], dl[k], udc); udw = fma(red[D + k], dl[k], udw); }
#pragma unroll
  for (int mm = 0; mm < D; ++mm) {
    double s_ = 0.0;
#pragma unroll
    for (int k = 0; k < D; ++k) s_ = fma(red[2 * D + mm * D + k], dl[k], s_);
    Pu[mm] = s_;
  }
  for (int rr_ = 0; rr_ < nf; ++rr_) {
    double rr[D], rho2 = 0.0;
#pragma unroll
    for (int a = 0; a < D; ++a) { rr[a] = Xq[a] - U[Ly::U_XF + rr_ * D + a]; rho2 = fma(rr[a], rr[a], rho2); }
    if (!(rho2 > 0.0)) continue;   // ∇k(0) = 0 (r = q)
    double psi, g1, g2;
    rad_eval(W.rad, rho2, psi, g1, g2);
    double ud = 0.0;
#pragma unroll
    for (int k = 0; k < D; ++k) ud = fma(rr[k], dl[k], ud);
    ud *= g1;
    udc = fma(U[Ly::U_CF + (S + 1) * FMAX + rr_], ud, udc);
    udw = fma(U[Ly::U_WF + rr_], ud, udw);
#pragma unroll
    for (int mm = 0; mm < D; ++mm) Pu[mm] = fma(U[Ly::U_PF + rr_ * D + mm], ud, Pu[mm]);
  }
  // δkx_q, δ∇kx_q at x = x_i
  double rq[D], rho2 = 0.0;
#pragma unroll
  for (int a = 0; a < D; ++a) { rq[a] = U[Ly::U_X + a] - Xq[a]; rho2 = fma(rq[a], rq[a], rho2); }
  double dkx, dgkx[D];
  {
    double psi, g1, g2;
    rad_eval(W.rad, rho2, psi, g1, g2);   // ρ = 0: g1 = ψ''(0), g2 = 0
    double dot = 0.0;
#pragma unroll
    for (int a = 0; a < D; ++a) dot = fma(rq[a], dl[a], dot);
    dkx = -g1 * dot;
#pragma unroll
    for (int a = 0; a < D; ++a) dgkx[a] = -fma(g2 * rq[a], dot, g1 * dl[a]);
  }
  const double cq = U[Ly::U_CF + (S + 1) * FMAX + q];
  const double wq = U[Ly::U_WF + q];
  const double gmu = U[Ly::U_SC + SC_GMU], gsig = U[Ly::U_SC + SC_GSIG];
  const double kxdc = -(wq * udc + udw * cq);
  const double dmu = dkx * cq + kxdc;
  const double isig = U[Ly::U_SC + SC_ISIG];
  const double dsig = wq * (udw - dkx) * isig;
  double dgm, dgs;
  rule_first(kp.rule, dmu, dsig, KCV(THETA), U[Ly::U_SC + SC_FMIN], KCV(SIGTOL), dgm, dgs);
  // cost-weighted rule: δ∇(α/c) = δ∇α/c − δα ∇c/c², δα = gμ δμ + gσ δσ (build-defined)
  double gcx[D], cc = 1.0, dal = 0.0;
  if (kp.cost) {
    double xi[D];
#pragma unroll
    for (int a = 0; a < D; ++a) xi[a] = U[Ly::U_X + a];
    (void)cost_eval<D>(kp, xi, gcx);
    cc = U[Ly::U_SC + SC_COSTC];
    dal = gmu * dmu + gsig * dsig;
  }
  double contrib = 0.0;
#pragma unroll
  for (int a = 0; a < D; ++a) {
    const double Pqa = U[Ly::U_PF + q * D + a];
    const double gkdc = -(Pqa * udc + Pu[a] * cq);
    const double dgmu = dgkx[a] * cq + gkdc;
    const double gsa = U[Ly::U_GSIG + a];
    double da = gmu * dgmu + dgm * U[Ly::U_GMU + a] + dgs * gsa;
    if (lane < D) {
      const double dgsig = (Pqa * udw + Pu[a] * wq - dgkx[a] * wq - Pqa * dkx - dsig * gsa) * isig;
      da += gsig * dgsig;
    }
    if (kp.cost) da = da / cc - dal * gcx[a] / (cc * cc);
    contrib = fma(da, U[Ly::U_XBAR + (i_pol - 1) * D + a], contrib);
  }
  if (lane < D) U[Ly::U_ACC + q * D + lane] += contrib;
  else U[Ly::U_YBAR + q] += contrib;
  STAMP(W, 9);
}

// small LU with partial pivoting (Julia det / \ on a Matrix), all lanes redundantly.
template <int D>
__device__ __forceinline__ bool lu_det_solve(double (&A)[D][D], double* b, double& det, bool do_solve) {
  int piv[D];
  bool sing = false;
  // the right-hand side is permuted beside A's rows, step by step (the same swaps, in the same
  // order, as applying the pivots after the factorisation): applied afterwards from piv[], the
  // select chains were turned into an indexed load of a scratch copy of b
  double bw[D];
#pragma unroll
  for (int i = 0; i < D; ++i) bw[i] = b[i];
#pragma unroll
  for (int k = 0; k < D; ++k) {
    int p = k;
    double mx = fabs(A[k][k]);
#pragma unroll
    for (int i = k + 1; i < D; ++i) if (fabs(A[i][k]) > mx) { mx = fabs(A[i][k]); p = i; }
    piv[k] = p;
    // row swap k <-> p as selects (a conditional swap becomes a dynamically indexed scratch array)
#pragma unroll
    for (int j = 0; j < D; ++j) {
      double rowp = A[k][j];
#pragma unroll
      for (int i = k + 1; i < D; ++i) rowp = (i == p) ? A[i][j] : rowp;
#pragma unroll
      for (int i = k + 1; i < D; ++i) A[i][j] = (i == p) ? A[k][j] : A[i][j];
      A[k][j] = rowp;
    }
    if (do_solve) {
      double bp = bw[k];
#pragma unroll
      for (int i = k + 1; i < D; ++i) bp = (i == p) ? bw[i] : bp;
#pragma unroll
      for (int i = k + 1; i < D; ++i) bw[i] = (i == p) ? bw[k] : bw[i];
      bw[k] = bp;
    }
    if (A[k][k] == 0.0) { sing = true; continue; }
#pragma unroll
    for (int i = k + 1; i < D; ++i) A[i][k] /= A[k][k];
#pragma unroll
    for (int j = k + 1; j < D; ++j)
#pragma unroll
      for (int i = k + 1; i < D; ++i) A[i][j] -= A[i][k] * A[k][j];
  }
  det = 1.0;
#pragma unroll
  for (int k = 0; k < D; ++k) { det *= A[k][k]; if (piv[k] != k) det = -det; }
  if (sing) det = 0.0;
  if (!do_solve || sing) return !sing;
#pragma unroll
  for (int i = 0; i < D; ++i) b[i] = bw[i];
#pragma unroll
  for (int i = 0; i < D; ++i) {
    double s = b[i];
#pragma unroll
    for (int k = 0; k < i; ++k) s -= A[i][k] * b[k];
    b[i] = s;
  }
#pragma unroll
  for (int i = D - 1; i >= 0; --i) {
    double s = b[i];
#pragma unroll
    for (int k = i + 1; k < D; ++k) s -= A[i][k] * b[k];
    b[i] = s / A[i][i];
  }
  return true;
}

// set U_X to fantasy point j and run a RICH eval on surface j-1
template <int D, int RPL, int HW>
__device__ __forceinline__ void rich_eval_at(WaveCtx<D, RPL, HW>& W, const KParams& kp, int j, LaneRes<D, RPL, HW>& lr) {
  using Ly = Lay<D, RPL, HW>;
  wave_sync();
  const int lane = W.ln();
  if (lane < D) W.U[Ly::U_X + lane] = W.U[Ly::U_XF + j * D + lane];
  wave_sync();
  evaluate<D, RPL, HW>(W, kp, j - 1, EV_RICH, lr);
}

// ================================================================================
// One trajectory.
// ================================================================================
template <int D, int RPL, int HW>
__device__ __forceinline__ void trajectory(WaveCtx<D, RPL, HW>& W, const KParams& kp, long long tr) {
  using Ly = Lay<D, RPL, HW>;
  constexpr int D1 = Ly::D1, NR = Ly::NR;
  double* U = W.U;
  const int lane = W.ln();
  const int M = kp.M, h = kp.h;
  const int r = (int)(tr / M), m = (int)(tr % M);
  Counters nevals;
  int st = 0;
  LaneRes<D, RPL, HW> lr;

  // surface -1 = the base surrogate; C[0] = c0
#pragma unroll
  for (int s = 0; s < RPL; ++s) W.C[lane + WAVE * s] = kp.c0[lane + WAVE * s];
  if (lane == 0) U[Ly::U_FMIN] = U[Ly::U_KC + KC_FMINB];
  // kp.base_solve: this item is start tr of a base_solve launch (one multistart call site: the
  // loop below runs its solve step once, on surface -1, for start tr alone)
  const bool bsolve = kp.base_solve != 0;
  if (lane < D) {
    if (!bsolve) U[Ly::U_X + lane] = kp.x0s[(long long)r * D + lane];
    U[Ly::U_LB + lane] = kp.lbs[lane];
    U[Ly::U_UB + lane] = kp.ubs[lane];
  }
  wave_sync();

  const int kend = bsolve ? 1 : h;
  for (int k = bsolve ? 1 : 0; k <= kend; ++k) {
    const int S = bsolve ? -1 : k - 1;
    if (k > 0) {
      if (kp.replay && !bsolve) {
        if (lane < D) U[Ly::U_X + lane] = kp.replay[(long long)lane + D * ((k - 1) + (long long)h * (m + (long long)M * r))];
        wave_sync();
      } else {
#ifndef MRBO_EXP_NO_NEWTON
        st |= multistart<D, RPL, HW>(W, kp, S, nevals, lr, bsolve ? (int)tr : 0, bsolve ? (int)tr + 1 : kp.nstarts);
#endif
        if (bsolve) {   // the start's minimizer and minimum were written by multistart
          if (lane == 0) kp.status[tr] = st & ~8;   // a NaN minimizer is the host's filter, not an error
          if (kp.evals && lane == 0) {
            kp.evals[NCOUNT * tr + 0] = nevals.grad;
            kp.evals[NCOUNT * tr + 1] = nevals.value;
            kp.evals[NCOUNT * tr + 2] = nevals.hess;
            kp.evals[NCOUNT * tr + 3] = 0;
            kp.evals[NCOUNT * tr + 4] = 0;
          }
          wave_sync();
          return;
        }
        if (st) break;
        if (lane < D) U[Ly::U_X + lane] = U[Ly::U_XB + lane];
        wave_sync();
      }
    }
    if (kp.policy && lane < D) kp.policy[(long long)lane + D * (k + (long long)(h + 1) * (m + (long long)M * r))] = U[Ly::U_X + lane];
    evaluate<D, RPL, HW>(W, kp, S, EV_DRAW, lr);
    if (U[Ly::U_SC + SC_VAR] < 0.0) { st |= 1; break; }
    if (k == 0 && lane < D) U[Ly::U_GMU0 + lane] = U[Ly::U_GMU + lane];
    double yv, gy[D];
    if (kp.ghq_w) {
      // GaussHermiteObservable (observables.jl:58-66): y = μ + √2σ t_k, ∇y = ∇μ + √2∇σ t_k; the
      // gradient recorded for the adjoint is get_gradient's weights[k]·∇y (observables.jl:157)
      const long long ik = (long long)m + (long long)M * k;
      const double tk = kp.ghq_nodes[ik], wk = kp.ghq_w[ik];
      yv = U[Ly::U_SC + SC_MU] + 1.4142135623730951 * U[Ly::U_SC + SC_SIG] * tk;
#pragma unroll
      for (int a = 0; a < D; ++a) gy[a] = wk * (U[Ly::U_GMU + a] + 1.4142135623730951 * U[Ly::U_GSIG + a] * tk);
    } else {
      double z[D1];
#pragma unroll
      for (int a = 0; a < D1; ++a) z[a] = kp.rn[(long long)m + (long long)M * a + (long long)M * D1 * k];
      st |= draw<D, RPL, HW>(W, kp, z, yv, gy);
      if (st) break;
    }
    wave_sync();
    st |= condition<D, RPL, HW>(W, kp, S, yv, gy, lr);
    STAMP(W, 10);
    if (st) break;
  }
  wave_sync();
  const long long oidx = (long long)m + (long long)M * r;
  if (kp.obs && lane <= h) kp.obs[oidx * (h + 1) + lane] = st ? qnan() : U[Ly::U_YF + lane];
  if (kp.evals && lane == 0) {
    kp.evals[NCOUNT * oidx + 0] = nevals.grad;
    kp.evals[NCOUNT * oidx + 1] = nevals.value;
    kp.evals[NCOUNT * oidx + 2] = nevals.hess;
    kp.evals[NCOUNT * oidx + 3] = 0;   // adjoint counters: overwritten below unless the trajectory failed
    kp.evals[NCOUNT * oidx + 4] = 0;
  }
  if (st) {
    if (lane == 0) { kp.values[oidx] = qnan(); kp.status[oidx] = st; if (kp.grad_theta) kp.grad_theta[oidx] = qnan(); }
    if (kp.grad_x && lane < D) kp.grad_x[oidx * D + lane] = qnan();
    return;
  }
  STAMP(W, 11);
  // resolve (observables.jl:12-14, Q3)
  double bo = U[Ly::U_YF];
  int t = 0;
  for (int k = 1; k <= h; ++k) { const double yk = U[Ly::U_YF + k]; if (yk < bo) { bo = yk; t = k; } }
  double value = fmax(kp.fmini - bo, 0.0);
  // resolve(gho; fmini) observables.jl:66-72: the best step's weight / √π
  if (kp.ghq_w) value *= kp.ghq_w[(long long)m + (long long)M * t] * 0.5641895835477563;
  double gth = 0.0;
  bool grad_zero = true;
#ifndef MRBO_EXP_NO_ADJOINT
  if (kp.with_gradient && kp.fmini > bo) {
    if (t == 0) {
      grad_zero = false;  // ∇x = -∇y₀ (Q10)
      if (lane < D) U[Ly::U_ACC + lane] = U[Ly::U_GF + lane];  // reuse ACC[0] as output staging
      if (lane == 0) U[Ly::U_YBAR] = 0.0;
      if (lane < D) U[Ly::U_GMU0 + lane] = 0.0;
      wave_sync();
    } else {
      grad_zero = false;
      // zero adjoint state
      for (int q = lane; q < FMAX * D; q += Ly::LANES) { U[Ly::U_ACC + q] = 0.0; U[Ly::U_XBAR + q] = 0.0; }
      if (lane <= FMAX) U[Ly::U_YBAR + lane] = 0.0;
      wave_sync();
      if (lane == 0) U[Ly::U_YBAR + t] = 1.0;
      wave_sync();
      for (int j = t; j >= 1; --j) {
        // δx of solve_dual_y call j (rollout.jl:133)
        wave_sync();
        if (lane < D) {
          U[Ly::U_DX + lane] = kp.dual_y
              ? kp.dual_y[(long long)lane + D * ((j - 1) + (long long)h * (m + (long long)M * r))]
              : dual_uniform_k(__builtin_bit_cast(unsigned long long, U[Ly::U_KC + KC_DXKEY]),
                               (long long)(kp.sample_offset + m), j, lane);   // keyed by the global sample alone
        }
        wave_sync();
        // i == j: solve_dual_x(j) (rollout.jl:150-191) then pair (j, j-1);
        // i > j : pairs (i, q = j-1) -- data part → ȳ_{j-1}, spatial part → ACC[j-1]
        for (int i = j; i <= t; ++i) {
          if (i > j) {
            bool xz = true;
#pragma unroll
            for (int a = 0; a < D; ++a) xz = xz && (U[Ly::U_XBAR + (i - 1) * D + a] == 0.0);
            if (xz) continue;   // zero dual: contributes exactly nothing
          }
          rich_eval_at<D, RPL, HW>(W, kp, i, lr);   // recover_policy_solve(T, i) :114-124
          ++nevals.rich;
          if (i == j) {
            double Hm[D][D], xd[D], det;
#pragma unroll
            for (int a = 0; a < D; ++a)
#pragma unroll
              for (int b = 0; b < D; ++b) Hm[a][b] = U[Ly::U_H + b * D + a];  // hessian(sx)'
            const double ybj = U[Ly::U_YBAR + j];
#pragma unroll
            for (int a = 0; a < D; ++a) xd[a] = -U[Ly::U_GF + (j - 1) * D + a] * ybj - U[Ly::U_ACC + j * D + a];
            // det(Hα) == det(Hα'): one LU serves the det test (Q4) and the solve
            const bool nonsing = lu_det_solve<D>(Hm, xd, det, true);
            bool zero = !(det >= KCV(HTOL));  // det(H) < htol → zeros; a NaN det keeps going (Julia)
            if (det != det) zero = false;
            if (zero) {
#pragma unroll
              for (int a = 0; a < D; ++a) xd[a] = 0.0;
            } else if (!nonsing) {
              st |= 16;
            }
            double gq = 0.0;   // gather_q: ∇θ += mixed_jᵀ x̄_j
            double mine = 0.0;
#pragma unroll
            for (int a = 0; a < D; ++a) { gq = fma(U[Ly::U_MIX + a], xd[a], gq); if (a == lane) mine = xd[a]; }
            gth += gq;
            wave_sync();
            if (lane < D) U[Ly::U_XBAR + (j - 1) * D + lane] = mine;
            wave_sync();
            if (zero) continue;
          }
          adjoint_pair<D, RPL, HW>(W, kp, i - 1, j - 1, i, lr);
          ++nevals.pairs;
          wave_sync();
        }
      }
    }
  }
#endif
  // outputs: ∇x = -(∇μ(x0)·ȳ0 + ACC[0]),  ∇θ = -Σ mixed·x̄
  wave_sync();
  const long long base = oidx;
  if (lane == 0) {
    kp.values[base] = value;
    kp.status[base] = st;
    if (kp.grad_theta) kp.grad_theta[base] = (grad_zero || st) ? (st ? qnan() : 0.0) : -gth;
  }
  if (kp.grad_x && lane < D) {
    double gx = 0.0;
    if (!grad_zero) gx = -(U[Ly::U_GMU0 + lane] * U[Ly::U_YBAR] + U[Ly::U_ACC + lane]);
    if (st) gx = qnan();
    kp.grad_x[base * D + lane] = gx;
  }
  if (st && lane == 0) kp.values[base] = qnan();
  if (kp.evals && lane == 0) {
    kp.evals[NCOUNT * base + 3] = nevals.rich;
    kp.evals[NCOUNT * base + 4] = nevals.pairs;
  }
  wave_sync();
  STAMP(W, 11);
}

// ================================================================================
// Kernels
// ================================================================================
// launch bounds: 2 waves per SIMD (256 VGPRs each) up to N = 128 at d ≤ 8; the N > 128 layouts
// and d > 8 run one wave per SIMD, whose 512-entry register file (256 VGPRs + 256 AGPRs) holds the
// multi-row / wide state (N ≤ 512 and d ≤ 16 compile, with scratch spills: coverage, not speed)
template <int D, int RPL, int HW = 1>
struct KBounds {
  static constexpr bool WIDE = (RPL > 2) || (D > 8);
  static constexpr int threads = WIDE ? 256 : 512;
  static constexpr int waves_per_simd = WIDE ? MRBO_WAVES_PER_SIMD_GL : MRBO_WAVES_PER_SIMD;
};

template <int D, int RPL, int HW>
__device__ __forceinline__ void wave_setup(WaveCtx<D, RPL, HW>& W, const KParams& kp, double* smem, int wave_in_block) {
  using Ly = Lay<D, RPL, HW>;
  W.lane = threadIdx.x & (Ly::LANES - 1);
  W.half = HW == 2 ? (int)((threadIdx.x >> 5) & 1) : 0;
  const WgTables<D, RPL, HW> tb(kp);
  // one per-trajectory area per half in half-wave mode
  double* wbase = smem + tb.end + ((long long)wave_in_block * HW + W.half) * Ly::WAVE_LDS;
  W.XS = kp.xs_lds ? smem + tb.xs : kp.xstarts;
  W.KXB = Ly::SQ ? smem + tb.kxb : kp.kxb_g;
  W.GTAB = Ly::SQ ? smem + tb.gtab : kp.gtab_g;
  W.YTAB = kp.ytab;   // the launch's table (ytab_kernel)
  W.B = wbase;
  W.red = wbase + Ly::BROWS * Ly::BS;
  W.U = W.red + Ly::REDN;
  W.G12 = W.U + Ly::U_SIZE;
  W.Linv = Ly::GL ? kp.Linv : smem;
  W.LinvT = kp.Linv + (long long)Ly::NBLK * WAVE * WAVE;   // GL: backward copy
  W.LinvL = smem;                                            // GL: LDS-resident blocks
  const long long slot = (long long)blockIdx.x * (blockDim.x / WAVE) + wave_in_block;
  if constexpr (Ly::SQ) W.E = W.G12 + Ly::G12;
  else W.E = kp.work + slot * kp.work_stride;
  W.C = W.E + (long long)FMAX * Ly::NRL;
  W.SUMS = W.E + (long long)(2 * FMAX + 1) * Ly::NR;   // packed layouts only (work_stride covers it)
  if constexpr (Ly::SQ) W.STASH = W.G12 + Ly::G12 + Ly::EC;   // SQ_EAGER: wave LDS
  else W.STASH = W.SUMS + 64 * 8;                              // GL layouts (work_stride covers it)
  W.N = kp.N;
  W.Npad = kp.Npad;
  W.rad.kind = kp.kernel;
  W.rad.cK = kp.cK;
  W.rad.cP = kp.cP;
#pragma unroll
  for (int s = 0; s < RPL; ++s) {
    const int i = W.lane + WAVE * s;
    W.valid[s] = i < kp.N;
#pragma unroll
    for (int a = 0; a < D; ++a) W.X0[s][a] = kp.X0[(long long)a * Ly::NR + i];
#ifndef MRBO_NO_PAD_FAR
    // padded rows far from every point (see WaveCtx::rowv): |x − X_i|² ≈ d·1e200 stays finite, and
    // ψ, g1 = ψ'/ρ, g2 underflow to exactly 0 for the Matérn and SE kernels
    if (!W.valid[s] && kp.kernel != KERNEL_PERIODIC)
#pragma unroll
      for (int a = 0; a < D; ++a) W.X0[s][a] = PAD_FAR;
#endif
  }
  // zero this wave's LDS so that padded rows read as zeros
  for (int q = W.lane; q < Ly::WAVE_LDS; q += Ly::LANES) wbase[q] = 0.0;
  wave_sync();
  if (W.lane == 0) {
    double* kc = W.U + Ly::U_KC;
    kc[KC_PSI0] = kp.psi0;
    kc[KC_D2PSI0] = kp.d2psi0;
    kc[KC_THETA] = kp.theta;
    kc[KC_SIGTOL] = kp.sigma_tol;
    kc[KC_GTOL] = kp.g_tol;
    kc[KC_GCMU] = kp.gcert_mu;
    kc[KC_GCSIG] = kp.gcert_sig;
    kc[KC_GCD2] = kp.gcert_d2;
    kc[KC_XTOL] = kp.x_tol;
    kc[KC_FTOL] = kp.f_tol;
    kc[KC_HTOL] = kp.htol;
    kc[KC_SN2] = kp.sn2;
    double box = 0.0;
    for (int a = 0; a < D; ++a) box = fmax(box, kp.ubs[a] - kp.lbs[a]);
    kc[KC_BOX] = box;
    // read back per trajectory from LDS: held in registers across the persistent loop, these two
    // 64-bit values were VGPR spills (8 B of scratch per lane each)
    kc[KC_FMINB] = kp.fmin_base;
    kc[KC_DXKEY] = __builtin_bit_cast(double, dual_key0(kp.seed));
  }
}

// SPEC = 1: the kernel function and decision rule fixed at compile time to Matérn-5/2 and EI
// (every configuration of BASELINE.json).  The other kernels' and rules' code paths fold away,
// which frees registers in the whole trajectory (VGPR spills 94 -> 33 at d = 6).  SPEC = 0
// reads both from the launch parameters.
template <int SPEC>
__device__ __forceinline__ void spec_params(KParams& kp) {
  if constexpr (SPEC == 1) {
    kp.kernel = KERNEL_MATERN52;
    kp.rule = RULE_EI;
    kp.cost = COST_NONE;
  } else if constexpr (SPEC == 2) {   // the same with the quadratic NonUniformCost weighting (C5 --cost)
    kp.kernel = KERNEL_MATERN52;
    kp.rule = RULE_EI;
    kp.cost = COST_QUADRATIC;
  }
}

// stage L0⁻¹ (and the inner-solve start points) once per workgroup (the only block barrier)
template <int D, int RPL, int HW>
__device__ __forceinline__ void stage_linv(const KParams& kp, double* smem) {
  using Ly = Lay<D, RPL, HW>;
  for (int q = threadIdx.x; q < (int)Ly::LINV_DOUBLES; q += blockDim.x) smem[q] = kp.Linv[Ly::LINV_LDS_SRC + q];
  if (kp.xs_lds)
    for (int q = threadIdx.x; q < kp.nstarts * D; q += blockDim.x) smem[Ly::LINV_DOUBLES + q] = kp.xstarts[q];
  __syncthreads();
}

// The Y0(x_start) table of the square layouts (kp.batch), written ONCE per launch: one workgroup of
// the rollout launch's shape and LDS size, launched just before rollout_kernel on the same stream,
// runs the rollout prologue's own code with store_y (so its rows are the bits the rollout
// workgroups' own Gram tables come from).
template <int D, int RPL, int SPEC, int HW = 1>
__global__ void __launch_bounds__((KBounds<D, RPL, HW>::threads), (KBounds<D, RPL, HW>::waves_per_simd)) ytab_kernel(KParams kp_in) {
  KParams kp = kp_in;
  spec_params<SPEC>(kp);
  extern __shared__ __attribute__((aligned(16))) double smem[];
  using Ly = Lay<D, RPL, HW>;
  if constexpr (Ly::SQ) {
    stage_linv<D, RPL, HW>(kp, smem);
    stage_start_tables<D, RPL, HW>(kp, smem, true);
  }
}

template <int D, int RPL, int SPEC, int HW = 1>
__global__ void __launch_bounds__((KBounds<D, RPL, HW>::threads), (KBounds<D, RPL, HW>::waves_per_simd)) rollout_kernel(KParams kp_in) {
  KParams kp = kp_in;   // a local copy: the fixed fields below propagate as constants
  spec_params<SPEC>(kp);
  extern __shared__ __attribute__((aligned(16))) double smem[];
  using Ly = Lay<D, RPL, HW>;
  stage_linv<D, RPL, HW>(kp, smem);
  if constexpr (Ly::SQ) {
    if (kp.batch) stage_start_tables<D, RPL, HW>(kp, smem, false);   // Y0 itself: ytab_kernel
  }
  WaveCtx<D, RPL, HW> W;
  wave_setup<D, RPL, HW>(W, kp, smem, threadIdx.x / WAVE);
  wave_sync();
#ifdef MRBO_STAMPS
  W.tlast = __builtin_amdgcn_s_memtime();
#endif
#ifdef MRBO_TAIL   // per-wave start / end (100 MHz REFCLK, one clock for all XCDs) and trajectory count
  const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
  int n_taken = 0;
#endif
#ifndef MRBO_QUEUE_SINGLE
  // One queue per XCD over a contiguous eighth of the trajectories (chunk x = [x·T/8, (x+1)·T/8),
  // its head at kp.queue[16·x], one 64-B line each): the waves of an XCD first drain the chunk of
  // their own XCD (HW_REG_XCC_ID), then the others in turn.  Consecutive trajectories then finish
  // on one XCD, so the 8-byte output rows (values, ∇θ, status, counters) fill whole cache lines
  // in one L2: with one queue for the chip, neighbouring rows came from all 8 L2s and each wrote
  // back its own partial line (C3: 17.6 MB written per launch for 7.1 MB of outputs).  Placement
  // is used for speed only: any wave may take any chunk, every trajectory is taken exactly once.
  int xcc = 0, visited = 0;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  int chunk = xcc & 7;
#endif
  for (;;) {
    long long tr = 0;
#ifdef MRBO_QUEUE_SINGLE
    if (W.lane == 0) tr = atomicAdd(kp.queue, 1);
#else
    if (W.lane == 0) {
      for (;;) {
        const long long lo = (long long)chunk * kp.T / 8, hi = (long long)(chunk + 1) * kp.T / 8;
        const long long idx = lo + atomicAdd(kp.queue + 16 * chunk, 1);
        if (idx < hi) { tr = idx; break; }
        if (++visited == 8) { tr = kp.T; break; }
        chunk = (chunk + 1) & 7;
      }
    }
#endif
    tr = __shfl(tr, 32 * W.half, WAVE);   // HW = 2: each half took its own trajectory
    if (tr >= kp.T) break;
    if (kp.order) {   // caller's schedule (a permutation; an out-of-range entry falls back to tr)
      const long long id = kp.order[tr];
      tr = (id >= 0 && id < kp.T) ? id : tr;
    }
    if (kp.skip_active && kp.skip_active[tr / kp.M] == 0) continue;   // a stopped restart (outer ascent)
#ifdef MRBO_TAIL
    const unsigned long long t_tr = __builtin_amdgcn_s_memrealtime();
#endif
    trajectory<D, RPL, HW>(W, kp, tr);
#ifdef MRBO_TAIL
    ++n_taken;
    // per-trajectory wall time after the per-wave records (3 per wave of the grid)
    if (kp.stamps && (W.lane & 31) == 0)
      kp.stamps[3ll * gridDim.x * (blockDim.x / WAVE) + tr] = __builtin_amdgcn_s_memrealtime() - t_tr;
#endif
  }
#ifdef MRBO_TAIL
  if (kp.stamps && W.lane == 0 && W.half == 0) {
    const unsigned long long t_end = __builtin_amdgcn_s_memrealtime();
    const long long g = (long long)blockIdx.x * (blockDim.x / WAVE) + threadIdx.x / WAVE;
    kp.stamps[3 * g] = t_start;
    kp.stamps[3 * g + 1] = t_end;
    kp.stamps[3 * g + 2] = (unsigned long long)n_taken;
  }
#endif
#ifdef MRBO_STAMPS
  if (kp.stamps && W.lane == 0)
    for (int k = 0; k < NSTAMP_SLOTS; ++k)
      atomicAdd(kp.stamps + k, reinterpret_cast<unsigned long long*>(W.U + Lay<D, RPL, HW>::U_STAMP)[k]);
#endif
}

// Start tables of the packed layouts (N > 64, kp.batch), one wave per start point k, written to
// global memory before the rollout launch (every workgroup reads the same copy through L2):
//   kxb_g[k][i] = ψ(|clamp(x_k) − X_i|) (0 on padded rows; start-major, unlike the LDS table),
//   gtab_g[k]   = base Gram YᵀY of Y = L0⁻¹[kx, ∇kx](x_k), upper triangle row-major (entry 0 is
//                 |L0⁻¹kx|², the only entry batch_start_values reads).
// The forward product walks the packed-by-columns image of L0⁻¹ (column j: rows j..Npad-1).
template <int D, int RPL, int HW = 1>
__global__ void __launch_bounds__(WAVE) start_tables_kernel(KParams kp) {
  using Ly = Lay<D, RPL, HW>;
  constexpr int NR = Ly::NR, D1 = Ly::D1;
  __shared__ double Bs[NR * D1];
  __shared__ double red[16 * ((Ly::NG + 15) / 16)];
  const int lane = threadIdx.x, k = blockIdx.x, ns = kp.nstarts;
  Radial rad;
  rad.kind = kp.kernel;
  rad.cK = kp.cK;
  rad.cP = kp.cP;
  double xk[D];
#pragma unroll
  for (int a = 0; a < D; ++a) xk[a] = clampd(kp.xstarts[(long long)k * D + a], kp.lbs[a], kp.ubs[a]);
#pragma unroll
  for (int s = 0; s < RPL; ++s) {
    const int i = lane + WAVE * s;
    double r[D], rho2 = 0.0;
#pragma unroll
    for (int a = 0; a < D; ++a) { r[a] = xk[a] - kp.X0[(long long)a * NR + i]; rho2 = fma(r[a], r[a], rho2); }
    double psi, g1, g2;
    rad_eval(rad, rho2, psi, g1, g2);
    const bool v = i < kp.N;
    Bs[i * D1] = v ? psi : 0.0;
#pragma unroll
    for (int a = 0; a < D; ++a) Bs[i * D1 + 1 + a] = v ? g1 * r[a] : 0.0;
    kp.kxb_g[(long long)k * NR + i] = v ? psi : 0.0;
  }
  __syncthreads();
  double acc[RPL][D1];
#pragma unroll
  for (int s = 0; s < RPL; ++s)
#pragma unroll
    for (int c = 0; c < D1; ++c) acc[s][c] = 0.0;
  for (int j = 0; j < kp.N; ++j) {
    double bj[D1];
#pragma unroll
    for (int c = 0; c < D1; ++c) bj[c] = Bs[j * D1 + c];
#pragma unroll
    for (int s = 0; s < RPL; ++s) {
      const int i = lane + WAVE * s;
      long long li;
      if constexpr (Ly::BC) li = (long long)Ly::blk(s, j / WAVE) * Ly::BLK + (j % WAVE) * Ly::LD + lane;
      else li = (long long)Ly::blk(s, j / WAVE) * WAVE * WAVE + (j % WAVE) * WAVE + lane;
      const double l = (i >= j && i < kp.N) ? kp.Linv[li] : 0.0;
#pragma unroll
      for (int c = 0; c < D1; ++c) acc[s][c] = fma(l, bj[c], acc[s][c]);
    }
  }
#pragma unroll
  for (int ch = 0; ch < (Ly::NG + 15) / 16; ++ch) {
    double gv[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int t = 16 * ch + q;
      double s_ = 0.0;
      if (t < Ly::NG) {
        int a = 0, rem = t;
#pragma unroll
        for (int aa = 0; aa < D1; ++aa) if (a == aa && rem >= D1 - aa) { rem -= D1 - aa; a = aa + 1; }
#pragma unroll
        for (int s = 0; s < RPL; ++s) s_ = fma(acc[s][a], acc[s][a + rem], s_);
      }
      gv[q] = s_;
    }
    wave_reduce<16>(gv, red + 16 * ch, lane);
  }
  __syncthreads();
  for (int t = lane; t < Ly::NG; t += WAVE) kp.gtab_g[(long long)k * Ly::NG + t] = red[t];
}

// eval(s, x, θ) on the base surrogate for P points (fixture / primitive parity path)
template <int D, int RPL, int HW = 1>
__global__ void __launch_bounds__((KBounds<D, RPL, HW>::threads), (KBounds<D, RPL, HW>::waves_per_simd)) eval_base_kernel(KParams kp) {
  using Ly = Lay<D, RPL, HW>;
  extern __shared__ __attribute__((aligned(16))) double smem[];
  for (int q = threadIdx.x; q < (int)Ly::LINV_DOUBLES; q += blockDim.x) smem[q] = kp.Linv[Ly::LINV_LDS_SRC + q];
  __syncthreads();
  WaveCtx<D, RPL, HW> W;
  wave_setup<D, RPL, HW>(W, kp, smem, threadIdx.x / WAVE);
  const int lane = W.ln();
#pragma unroll
  for (int s = 0; s < RPL; ++s) W.C[lane + WAVE * s] = kp.c0[lane + WAVE * s];
  if (lane == 0) W.U[Ly::U_FMIN] = kp.fmin_base;
  wave_sync();
  LaneRes<D, RPL, HW> lr;
  const int stride = 3 + 4 * D + D * D;
  for (;;) {
    long long p = 0;
    if (lane == 0) p = atomicAdd(kp.queue, 1);
    p = __shfl(p, 0, WAVE);
    if (p >= kp.T) break;
    if (lane < D) W.U[Ly::U_X + lane] = kp.pts[p * D + lane];
    wave_sync();
    evaluate<D, RPL, HW>(W, kp, -1, EV_FULL, lr);
    double* o = kp.pts_out + p * stride;
    const double* U = W.U;
    if (lane == 0) { o[0] = U[Ly::U_SC + SC_MU]; o[1] = U[Ly::U_SC + SC_SIG]; o[2] = U[Ly::U_SC + SC_ALPHA]; }
    if (lane < D) {
      o[3 + lane] = U[Ly::U_GMU + lane];
      o[3 + D + lane] = U[Ly::U_GSIG + lane];
      o[3 + 2 * D + lane] = U[Ly::U_GAL + lane];
      o[3 + 3 * D + D * D + lane] = U[Ly::U_MIX + lane];
    }
    for (int q = lane; q < D * D; q += WAVE) o[3 + 3 * D + q] = U[Ly::U_H + (q % D) * D + q / D];
    wave_sync();
  }
}

}  // namespace MRBO_FNS
}  // namespace mrbo
