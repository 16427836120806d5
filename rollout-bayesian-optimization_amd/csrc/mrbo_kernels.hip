// mrbo_kernels.hip -- the rollout / eval_base kernels for ONE input dimension d = MRBO_D and one
// fantasy capacity FMAX = MRBO_FMAX (compiled once per d with FMAX = 6, and for d ≤ 8 again
// with FMAX = 4 for horizons h ≤ 3; mrbo_api.hip dispatches through mrbo_dispatch.h).
// Rows per lane (RPL) compiled: d ≤ 8: 1, 2, 4, 8 (N ≤ 64, 128, 256, 512); d = 9..16: 1, 2
// (N ≤ 128).  The compile-time Matérn-5/2 + EI specialisation (SPEC = 1) exists for d ≤ 8 and
// RPL ≤ 4 -- the configurations of BASELINE.json; everything else runs the generic kernel.
#include "mrbo_dispatch.h"
#include "mrbo_rollout.hip"

#ifndef MRBO_D
#error "compile with -DMRBO_D=<1..16>"
#endif

#define MRBO_CAT_(a, b) a##b
#define MRBO_CAT(a, b) MRBO_CAT_(a, b)
// entry points of this unit: <name><d> for FMAX = 6, <name><d>_f<FMAX> otherwise (mrbo_dispatch.h)
#if MRBO_FMAX == 6
#define MRBO_SFX(name) MRBO_CAT(name, MRBO_D)
#else
#define MRBO_SFX(name) MRBO_CAT(MRBO_CAT(MRBO_CAT(name, MRBO_D), _f), MRBO_FMAX)
#endif

namespace mrbo {

// MRBO_AB_MIN (A/B variant builds of one configuration only, tools/ab_variant.py): the unit holds
// RPL = MRBO_AB_RPL (default 1) and the specialised kernel alone (it also stands in for the generic one), so a variant of
// the N ≤ 64 kernel compiles in seconds instead of minutes; plans of other shapes fail to create.
#ifdef MRBO_AB_MIN
#ifndef MRBO_AB_RPL
#define MRBO_AB_RPL 1
#endif
constexpr bool has_rpl(int d, int rpl) { return rpl == MRBO_AB_RPL; }
#else
constexpr bool has_rpl(int d, int rpl) { return rpl == 1 || rpl == 2 || (d <= 8 && (rpl == 4 || rpl == 8)); }
#endif
constexpr bool has_spec(int d, int rpl) { return d <= 8 && rpl <= 4; }
// half-wave kernel rollout_kernel<D, 1, 1, 2> (two trajectories per wave, N ≤ 32): the FMAX = 4
// units of d ≤ 4, Matérn-5/2 + EI (C1, C2)
// Matérn-5/2 + EI + the quadratic NonUniformCost fixed at compile time, rollout_kernel<D, RPL, 2>:
// the FMAX = 6 units of d ≤ 8 at N = 65..256 (C5 --cost); other cost plans run the generic kernel
#if MRBO_FMAX == 6 && MRBO_D <= 8 && !defined(MRBO_AB_MIN) && !defined(MRBO_NO_COST_SPEC)
#define MRBO_HAS_COST 1
#else
#define MRBO_HAS_COST 0
#endif
constexpr bool has_cost(int d, int rpl) { return MRBO_HAS_COST && d <= 8 && (rpl == 2 || rpl == 4); }
#if MRBO_FMAX == 4 && MRBO_D <= 4 && !(defined(MRBO_AB_MIN) && (defined(MRBO_AB_GENERIC) || defined(MRBO_AB_COST))) && !defined(MRBO_STAMPS)
#define MRBO_HAS_HALF 1
#else
#define MRBO_HAS_HALF 0
#endif

template <int D, int RPL>
static KernelSet kset() {
  using Ly = Lay<D, RPL>;
  const void* spec = nullptr;
#if defined(MRBO_AB_MIN) && defined(MRBO_AB_COST)      // Matérn-5/2 + EI + quadratic cost alone
  spec = (const void*)&rollout_kernel<D, RPL, 2>;
#elif defined(MRBO_AB_MIN) && defined(MRBO_AB_GENERIC)   // the generic kernel alone (cost, other rules)
  spec = (const void*)&rollout_kernel<D, RPL, 0>;
#else
  if constexpr (has_spec(D, RPL)) spec = (const void*)&rollout_kernel<D, RPL, 1>;
#endif
#ifdef MRBO_AB_MIN
  KernelSet ks{spec, spec, (const void*)&eval_base_kernel<D, RPL>,
#else
  KernelSet ks{(const void*)&rollout_kernel<D, RPL, 0>, spec, (const void*)&eval_base_kernel<D, RPL>,
#endif
               sizeof(double) * Ly::WAVE_LDS, Ly::SQ, Ly::BC && !Ly::SQ, Ly::LD, Ly::LINV_DOUBLES, Ly::GL,
               Ly::LINV_GLOBAL, KBounds<D, RPL>::threads};
#if MRBO_HAS_HALF
  if constexpr (RPL == 1) {
    ks.rollout_half = (const void*)&rollout_kernel<D, 1, 1, 2>;
    ks.wave_bytes_half = 2 * sizeof(double) * Lay<D, 1, 2>::WAVE_LDS;
  }
#endif
#if MRBO_HAS_COST
  if constexpr (has_cost(D, RPL)) ks.rollout_cost = (const void*)&rollout_kernel<D, RPL, 2>;
#endif
  ks.kparams_bytes = sizeof(KParams);
  return ks;
}

bool MRBO_SFX(kset_d)(int rpl, KernelSet& ks) {
#ifdef MRBO_AB_MIN
  if (rpl != MRBO_AB_RPL) return false;
  ks = kset<MRBO_D, MRBO_AB_RPL>();
  return true;
#else
  if (rpl == 1) ks = kset<MRBO_D, 1>();
  else if (rpl == 2) ks = kset<MRBO_D, 2>();
#if MRBO_D <= 8
  else if (rpl == 4) ks = kset<MRBO_D, 4>();
  else if (rpl == 8) ks = kset<MRBO_D, 8>();
#endif
  else return false;
  return true;
#endif
}

template <int RPL, int SPEC>
static void launch_one(dim3 g, dim3 b, size_t sm, hipStream_t st, const KParams& kp) {
#if defined(MRBO_AB_MIN) && defined(MRBO_AB_COST)
  if constexpr (has_rpl(MRBO_D, RPL))
    hipLaunchKernelGGL((rollout_kernel<MRBO_D, RPL, 2>), g, b, sm, st, kp);
#elif defined(MRBO_AB_MIN) && defined(MRBO_AB_GENERIC)
  if constexpr (has_rpl(MRBO_D, RPL))
    hipLaunchKernelGGL((rollout_kernel<MRBO_D, RPL, 0>), g, b, sm, st, kp);
#elif defined(MRBO_AB_MIN)
  if constexpr (has_rpl(MRBO_D, RPL) && has_spec(MRBO_D, RPL))
    hipLaunchKernelGGL((rollout_kernel<MRBO_D, RPL, 1>), g, b, sm, st, kp);
#else
  if constexpr (has_rpl(MRBO_D, RPL) && (SPEC == 0 || has_spec(MRBO_D, RPL)))
    hipLaunchKernelGGL((rollout_kernel<MRBO_D, RPL, SPEC>), g, b, sm, st, kp);
#endif
}

template <int SPEC>
static void launch_rollout_spec(int rpl, dim3 g, dim3 b, size_t sm, hipStream_t st, const KParams& kp) {
  if (rpl == 1) launch_one<1, SPEC>(g, b, sm, st, kp);
  else if (rpl == 2) launch_one<2, SPEC>(g, b, sm, st, kp);
  else if (rpl == 4) launch_one<4, SPEC>(g, b, sm, st, kp);
  else launch_one<8, SPEC>(g, b, sm, st, kp);
}

// spec: 0 generic, 1 Matérn-5/2 + EI, 2 the half-wave kernel (rows per lane 1), 3 Matérn-5/2 + EI +
// quadratic cost (rollout_kernel<D, RPL, 2>)
void MRBO_SFX(launch_rollout_d)(int rpl, int spec, dim3 g, dim3 b, size_t sm, hipStream_t st,
                                       const KParams& kp) {
#if MRBO_HAS_HALF
  if (spec == 2) {
    if (rpl == 1) hipLaunchKernelGGL((rollout_kernel<MRBO_D, 1, 1, 2>), g, b, sm, st, kp);
    return;
  }
#endif
#if MRBO_HAS_COST
  if (spec == 3) {
    if (rpl == 2) hipLaunchKernelGGL((rollout_kernel<MRBO_D, 2, 2>), g, b, sm, st, kp);
    else if (rpl == 4) hipLaunchKernelGGL((rollout_kernel<MRBO_D, 4, 2>), g, b, sm, st, kp);
    return;
  }
#endif
  if (spec) launch_rollout_spec<1>(rpl, g, b, sm, st, kp);
  else launch_rollout_spec<0>(rpl, g, b, sm, st, kp);
}

// The Y0 table of a square-layout launch (rows per lane 1) with batched starts: ONE workgroup of
// the rollout launch's shape (b, sm) and kernel variant (spec as launch_rollout_d) writes it just
// before the rollout kernel, on the same stream
void MRBO_SFX(launch_ytab_d)(int spec, dim3 b, size_t sm, hipStream_t st, const KParams& kp) {
#if MRBO_HAS_HALF
  if (spec == 2) {
    hipLaunchKernelGGL((ytab_kernel<MRBO_D, 1, 1, 2>), dim3(1), b, sm, st, kp);
    return;
  }
#endif
#if defined(MRBO_AB_MIN) && (defined(MRBO_AB_COST) || MRBO_AB_RPL != 1)
  (void)spec; (void)b; (void)sm; (void)st; (void)kp;
#elif defined(MRBO_AB_MIN) && defined(MRBO_AB_GENERIC)
  hipLaunchKernelGGL((ytab_kernel<MRBO_D, 1, 0>), dim3(1), b, sm, st, kp);
#elif defined(MRBO_AB_MIN)
  if constexpr (has_spec(MRBO_D, 1)) hipLaunchKernelGGL((ytab_kernel<MRBO_D, 1, 1>), dim3(1), b, sm, st, kp);
#else
  if constexpr (has_spec(MRBO_D, 1))
    if (spec == 1) {
      hipLaunchKernelGGL((ytab_kernel<MRBO_D, 1, 1>), dim3(1), b, sm, st, kp);
      return;
    }
  hipLaunchKernelGGL((ytab_kernel<MRBO_D, 1, 0>), dim3(1), b, sm, st, kp);
#endif
}

template <int RPL>
static void launch_tables_one(int nstarts, hipStream_t st, const KParams& kp) {
  if constexpr (has_rpl(MRBO_D, RPL))
    hipLaunchKernelGGL((start_tables_kernel<MRBO_D, RPL>), dim3(nstarts), dim3(WAVE), 0, st, kp);
}

void MRBO_SFX(launch_tables_d)(int rpl, int nstarts, hipStream_t st, const KParams& kp) {
  if (rpl == 2) launch_tables_one<2>(nstarts, st, kp);
  else if (rpl == 4) launch_tables_one<4>(nstarts, st, kp);
  else if (rpl == 8) launch_tables_one<8>(nstarts, st, kp);
}

template <int RPL>
static void launch_evalb_one(dim3 g, dim3 b, size_t sm, hipStream_t st, const KParams& kp) {
  if constexpr (has_rpl(MRBO_D, RPL)) hipLaunchKernelGGL((eval_base_kernel<MRBO_D, RPL>), g, b, sm, st, kp);
}

void MRBO_SFX(launch_evalb_d)(int rpl, dim3 g, dim3 b, size_t sm, hipStream_t st, const KParams& kp) {
  if (rpl == 1) launch_evalb_one<1>(g, b, sm, st, kp);
  else if (rpl == 2) launch_evalb_one<2>(g, b, sm, st, kp);
  else if (rpl == 4) launch_evalb_one<4>(g, b, sm, st, kp);
  else launch_evalb_one<8>(g, b, sm, st, kp);
}

}  // namespace mrbo
