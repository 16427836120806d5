// mrbo_dispatch.h -- interface between the host API (mrbo_api.hip) and the per-dimension
// kernel translation units (mrbo_kernels.hip compiled once per d = 1..16 with -DMRBO_D=d).
#pragma once
#include <hip/hip_runtime.h>

#include "mrbo_device.h"

namespace mrbo {

// launch geometry and L0⁻¹ image of one rollout_kernel<D, RPL> / eval_base_kernel<D, RPL> pair
struct KernelSet {
  const void* rollout;      // generic: kernel function and decision rule from KParams
  const void* rollout_spec; // Matérn-5/2 + EI fixed at compile time (rollout_kernel SPEC = 1), or null
  const void* evalb;
  size_t wave_bytes;        // per-wave LDS
  bool square;              // L0⁻¹ layout: dense square (ld) or packed triangle
  bool blocks;              // L0⁻¹ layout: the three 64×64 blocks (0,0), (1,0), (1,1), each ld-square
  int ld;
  long long linv_doubles;   // LDS-resident L0⁻¹ (0 when it stays in global memory)
  bool gl;                  // L0⁻¹ in global memory: packed by columns, then packed by rows
  long long linv_dev;       // doubles of the device image
  int max_threads;          // launch bound (threads per workgroup)
  // half-wave mode (N ≤ 32, d ≤ 4, h ≤ 3): rollout_kernel<D, 1, 1, 2>, two trajectories per wave
  // (Matérn-5/2 + EI), with its per-wave LDS (two trajectory areas); null where not compiled
  const void* rollout_half = nullptr;
  size_t wave_bytes_half = 0;
  // Matérn-5/2 + EI + quadratic NonUniformCost at compile time (rollout_kernel<D, RPL, 2>), or null
  const void* rollout_cost = nullptr;
  // sizeof(KParams) in the unit that filled this set: the host API refuses a unit compiled against
  // another KParams layout (a stale object would read every launch parameter at a shifted offset)
  size_t kparams_bytes = 0;
};

// The host API sees every unit's entry points as weak references (MRBO_API_TU): a library
// linked from a subset of the units (__graft_entry__.compile_lib: the default build carries the
// dimensions the configurations and tests use) resolves the missing ones to null, and
// mrbo_plan_create reports those dimensions as not compiled instead of failing to link.
#ifdef MRBO_API_TU
#define MRBO_UNIT __attribute__((weak))
#else
#define MRBO_UNIT
#endif
#define MRBO_DECLARE_D(DD)                                                                      \
  MRBO_UNIT bool kset_d##DD(int rpl, KernelSet& ks);                                            \
  MRBO_UNIT void launch_rollout_d##DD(int rpl, int spec, dim3 g, dim3 b, size_t sm, hipStream_t st, const KParams& kp); \
  MRBO_UNIT void launch_evalb_d##DD(int rpl, dim3 g, dim3 b, size_t sm, hipStream_t st, const KParams& kp); \
  MRBO_UNIT void launch_tables_d##DD(int rpl, int nstarts, hipStream_t st, const KParams& kp); \
  MRBO_UNIT void launch_ytab_d##DD(int spec, dim3 b, size_t sm, hipStream_t st, const KParams& kp);
MRBO_DECLARE_D(1) MRBO_DECLARE_D(2) MRBO_DECLARE_D(3) MRBO_DECLARE_D(4)
MRBO_DECLARE_D(5) MRBO_DECLARE_D(6) MRBO_DECLARE_D(7) MRBO_DECLARE_D(8)
MRBO_DECLARE_D(9) MRBO_DECLARE_D(10) MRBO_DECLARE_D(11) MRBO_DECLARE_D(12)
MRBO_DECLARE_D(13) MRBO_DECLARE_D(14) MRBO_DECLARE_D(15) MRBO_DECLARE_D(16)
#undef MRBO_DECLARE_D
// the same entry points of the FMAX = 4 units (h ≤ 3, d ≤ 8): fewer fantasy rows per wave in
// LDS and registers
#define MRBO_DECLARE_DF4(DD)                                                                    \
  MRBO_UNIT bool kset_d##DD##_f4(int rpl, KernelSet& ks);                                       \
  MRBO_UNIT void launch_rollout_d##DD##_f4(int rpl, int spec, dim3 g, dim3 b, size_t sm, hipStream_t st, const KParams& kp); \
  MRBO_UNIT void launch_evalb_d##DD##_f4(int rpl, dim3 g, dim3 b, size_t sm, hipStream_t st, const KParams& kp); \
  MRBO_UNIT void launch_tables_d##DD##_f4(int rpl, int nstarts, hipStream_t st, const KParams& kp); \
  MRBO_UNIT void launch_ytab_d##DD##_f4(int spec, dim3 b, size_t sm, hipStream_t st, const KParams& kp);
MRBO_DECLARE_DF4(1) MRBO_DECLARE_DF4(2) MRBO_DECLARE_DF4(3) MRBO_DECLARE_DF4(4)
MRBO_DECLARE_DF4(5) MRBO_DECLARE_DF4(6) MRBO_DECLARE_DF4(7) MRBO_DECLARE_DF4(8)
#undef MRBO_DECLARE_DF4
#undef MRBO_UNIT
constexpr int F4_HMAX = 3;   // horizons served by the FMAX = 4 units
constexpr int F4_DMAX = 8;

// base-GP fit + marginal likelihood for P lengthscales (mrbo_gpfit.hip)
struct GpFitParams {
  int d, N, kernel;
  double sn2;
  const double* X;       // d×N
  const double* y;       // N
  int nt;                // hyperparameters per candidate: 1 (ℓ) or 2 (ℓ, p: Periodic)
  const double* thetas;  // nt×P
  double period;         // Periodic with nt = 1: the surrogate's period
  double* ll;            // P
  double* grad;          // nt×P: ∂ll/∂θ_t
  int* status;           // P: 0, or 1 = PosDefException
  double* L_out;         // optional N×N×P
  double* c_out;         // optional N×P
  double* work;          // gpfit_tile_work_doubles(N, nt)·P (the tile kernel only)
};
// MRBO_GPFIT_LDS_MAX < N ≤ 512: gpfit_tile_kernel's workspace per candidate
size_t gpfit_tile_work_doubles(int N, int nt);
// LDS bytes per workgroup of the kernel launch_gpfit selects for q (the tile kernel stages X:
// d·⌈N/32⌉·32 doubles, so large d can exceed the CU's 160 KB)
size_t gpfit_launch_lds(const GpFitParams& q);
void launch_gpfit(int P, hipStream_t st, const GpFitParams& q);
// 32 < N ≤ 64, d ≤ 16 and no factor / coefficient outputs: the one-wave-per-candidate register
// kernel (no workspace).  N ≤ 32 is one tile of the tile kernel: its register factor and inverse
// of a 32 × 32 tile do a quarter of the 64-row kernel's work (N = 32: 0.045 ms per 256 candidates
// in the register kernel)
inline bool gpfit_in_regs(const GpFitParams& q) {
  return q.N > 32 && q.N <= 64 && q.d <= 16 && !q.L_out && !q.c_out;
}
// 64 < N ≤ 80 (and N ≤ 64 with factor outputs): gpfit_lds_kernel, no global workspace.  The
// ceiling is measured: the tile kernel pads N to a multiple of 32 and overtakes
// the LDS kernel above N ≈ 80 (N = 96: 0.28 vs 0.36 ms, N = 128: 0.40 vs 0.60 ms per 256
// candidates; N = 72: 0.27 vs 0.22 ms)
#ifndef MRBO_GPFIT_LDS_MAX
#define MRBO_GPFIT_LDS_MAX 80
#endif
inline bool gpfit_in_lds(const GpFitParams& q) {
  return q.N > 32 && q.N <= MRBO_GPFIT_LDS_MAX && q.d <= 16 && !gpfit_in_regs(q);
}

}  // namespace mrbo
