// mrbo_kernels.hip -- the rollout / eval_base kernels for ONE input dimension d = MRBO_D
// (compiled once per d, in parallel; mrbo_api.hip dispatches through mrbo_dispatch.h).
#include "mrbo_dispatch.h"
#include "mrbo_rollout.hip"

#ifndef MRBO_D
#error "compile with -DMRBO_D=<1..8>"
#endif

#define MRBO_CAT_(a, b) a##b
#define MRBO_CAT(a, b) MRBO_CAT_(a, b)

namespace mrbo {

template <int D, int RPL>
static KernelSet kset() {
  using Ly = Lay<D, RPL>;
  return KernelSet{(const void*)&rollout_kernel<D, RPL, 0>, (const void*)&rollout_kernel<D, RPL, 1>,
                   (const void*)&eval_base_kernel<D, RPL>,
                   sizeof(double) * Ly::WAVE_LDS, Ly::SQ, Ly::BC && !Ly::SQ, Ly::LD, Ly::LINV_DOUBLES, Ly::GL, Ly::LINV_GLOBAL,
                   KBounds<RPL>::threads};
}

bool MRBO_CAT(kset_d, MRBO_D)(int rpl, KernelSet& ks) {
  if (rpl == 1) ks = kset<MRBO_D, 1>();
  else if (rpl == 2) ks = kset<MRBO_D, 2>();
  else if (rpl == 4) ks = kset<MRBO_D, 4>();
  else return false;
  return true;
}

template <int SPEC>
static void launch_rollout_spec(int rpl, dim3 g, dim3 b, size_t sm, hipStream_t st, const KParams& kp) {
  if (rpl == 1) hipLaunchKernelGGL((rollout_kernel<MRBO_D, 1, SPEC>), g, b, sm, st, kp);
  else if (rpl == 2) hipLaunchKernelGGL((rollout_kernel<MRBO_D, 2, SPEC>), g, b, sm, st, kp);
  else hipLaunchKernelGGL((rollout_kernel<MRBO_D, 4, SPEC>), g, b, sm, st, kp);
}

void MRBO_CAT(launch_rollout_d, MRBO_D)(int rpl, int spec, dim3 g, dim3 b, size_t sm, hipStream_t st,
                                       const KParams& kp) {
  if (spec) launch_rollout_spec<1>(rpl, g, b, sm, st, kp);
  else launch_rollout_spec<0>(rpl, g, b, sm, st, kp);
}

void MRBO_CAT(launch_tables_d, MRBO_D)(int rpl, int nstarts, hipStream_t st, const KParams& kp) {
  if (rpl == 2) hipLaunchKernelGGL((start_tables_kernel<MRBO_D, 2>), dim3(nstarts), dim3(WAVE), 0, st, kp);
  else if (rpl == 4) hipLaunchKernelGGL((start_tables_kernel<MRBO_D, 4>), dim3(nstarts), dim3(WAVE), 0, st, kp);
}

void MRBO_CAT(launch_evalb_d, MRBO_D)(int rpl, dim3 g, dim3 b, size_t sm, hipStream_t st, const KParams& kp) {
  if (rpl == 1) hipLaunchKernelGGL((eval_base_kernel<MRBO_D, 1>), g, b, sm, st, kp);
  else if (rpl == 2) hipLaunchKernelGGL((eval_base_kernel<MRBO_D, 2>), g, b, sm, st, kp);
  else hipLaunchKernelGGL((eval_base_kernel<MRBO_D, 4>), g, b, sm, st, kp);
}

}  // namespace mrbo
