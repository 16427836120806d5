// mrbo_api.hip -- C ABI (include/mrbo.h) of the MI355X rollout evaluator: plans, launches,
// ETO reductions and host helpers.  Single translation unit with the device code.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

#include "../../include/mrbo.h"
#define MRBO_API_TU
#include "mrbo_dispatch.h"
#include "sobol_table.h"

namespace mrbo {   // mrbo_order.hip
size_t order_buffer_bytes(int T);
hipError_t order_longest_first(const long long* evals, int T, void* buf, size_t bytes, int** order, hipStream_t st);
}

using namespace mrbo;

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIP_TRY(expr)                                                                  \
  do {                                                                                 \
    hipError_t e_ = (expr);                                                            \
    if (e_ != hipSuccess) return fail(MRBO_ERR_HIP, "%s: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

}  // namespace

struct mrbo_plan {
  int device = 0;
  int d = 0, N = 0, RPL = 1, NR = 64, Npad = 64;
  mrbo_params_t p{};
  std::vector<double> lbs, ubs, cost_w;
  int kernel = 0;
  double ell = 1, cK = 1, cP = 0, psi0 = 1, d2psi0 = -1, sn2 = 1e-6;
  double gcert_mu = 0, gcert_sig = -1;
  double fmin_base = 0, fmini = 0;
  // device state
  double* dX0 = nullptr;    // [d][NR]
  double* dc0 = nullptr;    // [NR]
  double* dLinv = nullptr;  // L0⁻¹ in the kernel's LDS layout (Lay::SQ)
  double* dlbs = nullptr;
  double* dubs = nullptr;
  double* dcost = nullptr;  // NonUniformCost table [lb (d), ub − lb (d), w (d)] (cost models only)
  double* dwork = nullptr;
  double* dytab = nullptr;  // batched starts: the launch's Y0(x_start) table (square layout, ytab_kernel)
  double* dkxb = nullptr;   // batched starts, packed layouts: global start tables (start_tables_kernel)
  double* dgtab = nullptr;
  long long work_stride = 0;
  int* dqueue = nullptr;    // work-queue heads: one per XCD, 64 B apart (rollout_kernel)
  const int32_t* order = nullptr;   // mrbo_plan_set_order: caller-owned device permutation of M×R
                                    // (or the plan's own, mrbo_plan_order_longest_first)
  void* oorder = nullptr;           // mrbo_plan_order_longest_first: keys, ranking, sort scratch, order
  size_t oorder_bytes = 0;
  const int32_t* skip_active = nullptr;   // set by mrbo_stochastic_solve for its launches only
  int wpg = 4, blocks = 0;
  size_t smem = 0;
  int spec = 0;             // 1: rollout_kernel<D, RPL, 1> (Matérn-5/2 + EI fixed); 2: its half-wave form <D, 1, 1, 2>;
                            // 3: <D, RPL, 2> (Matérn-5/2 + EI + quadratic cost)
  int fx = 0;               // 1: the FMAX = 4 kernel units (h ≤ 3, d ≤ 8)
  int xs_lds = 0;           // rollout launches stage xstarts in LDS (≤ 8 KB)
  int batch = 0;            // batched start-point values (start tables in LDS)
  int ewpg = 4, eblocks = 0;
  size_t esmem = 0;
  // HIP events around every rollout kernel launch (the kernel alone: after the queue memset and
  // the packed layouts' start-table kernel), a ring of the last NEV launches (mrbo_kernel_times)
  static constexpr int NEV = 64;
  hipEvent_t ev[2 * NEV] = {};
  long long nlaunch = 0;
  // MRBO_FLAG_HOST_POINTERS staging: device buffers kept across calls, one slot per staged
  // argument in call order, grown on demand and freed with the plan
  std::vector<std::pair<void*, size_t>> stage;
  // mrbo_stochastic_solve: the outer ascent's device state (one slot per buffer, grown on demand),
  // a pinned ring of per-iteration checks read back behind the launches, and its events
  std::vector<std::pair<void*, size_t>> solve;
  static constexpr int NCHK = 8;
  int32_t* hchk = nullptr;   // pinned, 2 × NCHK: [status bits of the iteration, restarts still active]
  hipEvent_t chk_ev[NCHK] = {};
};

namespace {

double g_gpfit_ms = -1.0;   // kernel time of the last mrbo_gp_fit (HIP events around the launch)

// ---- kernel dispatch: one translation unit per input dimension (mrbo_kernels.hip) -------
// fx = 1 selects the FMAX = 4 units (horizon ≤ 3, d ≤ 8), fx = 0 the FMAX = 6 ones.  The units'
// entry points are weak references here (mrbo_dispatch.h): null when the unit is not linked in.
#define MRBO_FOR_D(X) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15) X(16)
#define MRBO_FOR_DF4(X) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8)

// is the unit (d, fx) linked into this library?
bool unit_present(int d, int fx) {
#define K6(DD) case DD: return kset_d##DD != nullptr;
#define K4(DD) case DD: return kset_d##DD##_f4 != nullptr;
  if (fx) { switch (d) { MRBO_FOR_DF4(K4) default: return false; } }
  switch (d) { MRBO_FOR_D(K6) default: return false; }
#undef K6
#undef K4
}

bool get_kset(int d, int rpl, int fx, KernelSet& ks) {
  if (!unit_present(d, fx)) return false;
#define K6(DD) case DD: return kset_d##DD(rpl, ks);
#define K4(DD) case DD: return kset_d##DD##_f4(rpl, ks);
  if (fx) { switch (d) { MRBO_FOR_DF4(K4) default: return false; } }
  switch (d) { MRBO_FOR_D(K6) default: return false; }
#undef K6
#undef K4
}

// the launchers below are reached only through a plan whose unit get_kset found
// start tables of the packed layouts (rpl 2 / 4), before a rollout launch with kp.batch
void launch_tables(int d, int rpl, int fx, int nstarts, hipStream_t st, const KParams& kp) {
#define K6(DD) case DD: launch_tables_d##DD(rpl, nstarts, st, kp); return;
#define K4(DD) case DD: launch_tables_d##DD##_f4(rpl, nstarts, st, kp); return;
  if (fx) { switch (d) { MRBO_FOR_DF4(K4) default: return; } }
  switch (d) { MRBO_FOR_D(K6) default: return; }
#undef K6
#undef K4
}

// the Y0 table of the square layouts (rpl 1) with batched starts, before a rollout launch
void launch_ytab(int d, int fx, int spec, dim3 b, size_t sm, hipStream_t st, const KParams& kp) {
#define K6(DD) case DD: launch_ytab_d##DD(spec, b, sm, st, kp); return;
#define K4(DD) case DD: launch_ytab_d##DD##_f4(spec, b, sm, st, kp); return;
  if (fx) { switch (d) { MRBO_FOR_DF4(K4) default: return; } }
  switch (d) { MRBO_FOR_D(K6) default: return; }
#undef K6
#undef K4
}

void launch_rollout(int d, int rpl, int fx, int spec, dim3 g, dim3 b, size_t sm, hipStream_t st, const KParams& kp) {
#define K6(DD) case DD: launch_rollout_d##DD(rpl, spec, g, b, sm, st, kp); return;
#define K4(DD) case DD: launch_rollout_d##DD##_f4(rpl, spec, g, b, sm, st, kp); return;
  if (fx) { switch (d) { MRBO_FOR_DF4(K4) default: return; } }
  switch (d) { MRBO_FOR_D(K6) default: return; }
#undef K6
#undef K4
}

void launch_evalb(int d, int rpl, int fx, dim3 g, dim3 b, size_t sm, hipStream_t st, const KParams& kp) {
#define K6(DD) case DD: launch_evalb_d##DD(rpl, g, b, sm, st, kp); return;
#define K4(DD) case DD: launch_evalb_d##DD##_f4(rpl, g, b, sm, st, kp); return;
  if (fx) { switch (d) { MRBO_FOR_DF4(K4) default: return; } }
  switch (d) { MRBO_FOR_D(K6) default: return; }
#undef K6
#undef K4
}

// choose waves per workgroup maximising resident waves per CU (LDS + register limits)
// fixed_bytes: per-workgroup tables; the wave areas double as prologue scratch of scratch_bytes
int pick_grid(const void* fn, size_t fixed_bytes, size_t wave_bytes, int ncu, int& wpg, int& blocks, size_t& smem,
              size_t scratch_bytes = 0, int maxw = 8) {
  int best_w = 0;
  for (int w = 1; w <= maxw; ++w) {
    const size_t sm = fixed_bytes + std::max(w * wave_bytes, scratch_bytes);
    if (sm > 160 * 1024) break;
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, w * WAVE, sm) != hipSuccess) continue;
    const int waves = nb * w;
    if (waves > best_w) { best_w = waves; wpg = w; blocks = nb * ncu; smem = sm; }
  }
  return best_w;
}

// ---- reductions: per (restart, component) block, deterministic tree order --------------
// comp 0: values, 1..d: grad_x[a], d+1: grad_theta.  Two passes (mean, then centred squares)
// in both modes.  mode 0: ETO (mean, std n-1) -> eto; mode 1: shard moments (Σx, M2 = Σ(x − x̄)²)
// -> moments, merged across ranks by Chan's formula (mrbo/parallel.py).
// M samples of each restart are reduced; Ms is the restart stride of the outputs (the plan's M)
__global__ void __launch_bounds__(256) reduce_kernel(const double* values, const double* grad_x,
                                                     const double* grad_theta, int M, int Ms, int d, int mode,
                                                     double* out) {
  __shared__ double sh[256];
  const int r = blockIdx.x, comp = blockIdx.y, tid = threadIdx.x;
  const int W = 2 + 2 * d + 2;
  auto elem = [&](int m) -> double {
    const long long idx = (long long)m + (long long)Ms * r;
    if (comp == 0) return values[idx];
    if (comp <= d) return grad_x ? grad_x[idx * d + (comp - 1)] : 0.0;
    return grad_theta ? grad_theta[idx] : 0.0;
  };
  auto block_sum = [&](double v) -> double {
    sh[tid] = v;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
      if (tid < s) sh[tid] += sh[tid + s];
      __syncthreads();
    }
    const double t = sh[0];
    __syncthreads();
    return t;
  };
  double s = 0.0;
  for (int m = tid; m < M; m += 256) s += elem(m);
  const double tot = block_sum(s);
  double s2 = 0.0;
  const double mu = tot / M;
  for (int m = tid; m < M; m += 256) { const double dv = elem(m) - mu; s2 += dv * dv; }
  const double tot2 = block_sum(s2);
  if (tid == 0) {
    int c0, c1;
    if (comp == 0) { c0 = 0; c1 = 1; }
    else if (comp <= d) { c0 = 2 + (comp - 1); c1 = 2 + d + (comp - 1); }
    else { c0 = 2 + 2 * d; c1 = 3 + 2 * d; }
    if (mode == 0) {
      out[(long long)W * r + c0] = tot / M;
      out[(long long)W * r + c1] = sqrt(tot2 / (M - 1));
    } else {
      out[(long long)W * r + c0] = tot;
      out[(long long)W * r + c1] = tot2;
    }
  }
}

// ---- outer ascent step on the device (stochastic_solve utils.jl:235-265): per active restart r,
// eswavs (utils.jl:114-123) on the ETO's ∇μx and σ_∇μx -- stop when 1 − (M/d)·Σ_a ∇_a²/σ_a² > 0 (a
// NaN ratio keeps iterating, as in Julia) -- else the optimizer's update! of x (StandardSGA
// optimizers.jl:16-22 or Adam :49-74).  One thread per restart; the x0 batch and the Adam moments
// never leave the device between launches.
__device__ __forceinline__ bool eswavs_stops(const double* e, int d, double sample_size) {
#pragma clang fp contract(off)   // the host mirror's (numpy) roundings: no fused multiply-adds
  double ratio = 0.0;
  for (int a = 0; a < d; ++a) {
    const double g = e[2 + a], s = e[2 + d + a];
    ratio += (g * g) / (s * s);
  }
  return 1.0 - (sample_size / d) * ratio > 0.0;
}

__global__ void __launch_bounds__(64) sga_kernel(const double* eto, double* x0s, int* active, int R, int d,
                                                 double sample_size, double eta) {
#pragma clang fp contract(off)
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R || !active[r]) return;
  const double* e = eto + (size_t)(2 + 2 * d + 2) * r;
  if (eswavs_stops(e, d, sample_size)) {
    active[r] = 0;
    return;
  }
  for (int a = 0; a < d; ++a) x0s[(size_t)d * r + a] = x0s[(size_t)d * r + a] + eta * e[2 + a];
}

// Adam update! (optimizers.jl:49-74) with its moments m, v (d×R) kept on the device: m ← β1·m +
// (1−β1)·∇, v ← β2·v + (1−β2)·∇², x += η·(m/c1) / (√(v/c2) + ε), c1 = 1 − β1^t and c2 = 1 − β2^t
// formed on the host (the same pow as the host mirror's).  sqrt and division are IEEE-rounded.
__global__ void __launch_bounds__(64) adam_kernel(const double* eto, double* x0s, int* active, double* m, double* v,
                                                  int R, int d, double sample_size, double eta, double b1, double b2,
                                                  double eps, double c1, double c2) {
#pragma clang fp contract(off)
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R || !active[r]) return;
  const double* e = eto + (size_t)(2 + 2 * d + 2) * r;
  if (eswavs_stops(e, d, sample_size)) {
    active[r] = 0;
    return;
  }
  for (int a = 0; a < d; ++a) {
    const size_t k = (size_t)d * r + a;
    const double g = e[2 + a];
    const double mk = b1 * m[k] + (1.0 - b1) * g;
    const double vk = b2 * v[k] + (1.0 - b2) * (g * g);
    m[k] = mk;
    v[k] = vk;
    x0s[k] = x0s[k] + (eta * (mk / c1)) / (__builtin_sqrt(vk / c2) + eps);
  }
}

// ---- multi-GPU exchange on the device: Chan merge of the all-gathered shard moments ---------
// One thread per (restart r, component c of [α, ∇x (d), ∇θ]): the shards' (Σ, M2) are merged
// left to right in rank order with Chan et al.'s pairwise formula and turned into the ETO row
// (mean, std(n−1), rollout.jl:328-339) -- the same operations, in the same order and without
// contraction, as mrbo/parallel.py merge_moments + eto_from_moments.
constexpr int MERGE_MAX_SHARDS = 64;
struct MergeCounts { long long n[MERGE_MAX_SHARDS]; };

__global__ void __launch_bounds__(64) merge_kernel(const double* moments, int nshards, MergeCounts cnt, int R, int d,
                                                   double* eto) {
#pragma clang fp contract(off)
  const int W = 2 + 2 * d + 2;
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= R * (d + 2)) return;
  const int r = idx / (d + 2), comp = idx % (d + 2);
  int c0, c1;
  if (comp == 0) { c0 = 0; c1 = 1; }
  else if (comp <= d) { c0 = 2 + (comp - 1); c1 = 2 + d + (comp - 1); }
  else { c0 = 2 + 2 * d; c1 = 3 + 2 * d; }
  double n = 0.0, sm = 0.0, q = 0.0;
  bool any = false;
  for (int k = 0; k < nshards; ++k) {
    const double nk = (double)cnt.n[k];
    if (cnt.n[k] == 0) continue;
    const double* blk = moments + (size_t)k * W * R + (size_t)W * r;
    const double sk = blk[c0], qk = blk[c1];
    if (!any) { n = nk; sm = sk; q = qk; any = true; continue; }
    const double delta = sk / nk - sm / n;
    q = q + qk + delta * delta * (n * nk / (n + nk));
    sm = sm + sk;
    n = n + nk;
  }
  double* e = eto + (size_t)W * r;
  e[c0] = sm / n;
  e[c1] = n > 1.0 ? sqrt(q / (n - 1.0)) : __builtin_nan("");
}

// mrbo_stochastic_solve's per-iteration check: the OR of the launch's trajectory status bits and
// the count of restarts still active after the step, into chk[0..1] (one workgroup)
__global__ void __launch_bounds__(256) solve_check_kernel(const int* status, long long T, const int* active, int R,
                                                         int* chk) {
  __shared__ int sb[256], sa[256];
  int b = 0, a = 0;
  for (long long t = threadIdx.x; t < T; t += blockDim.x) b |= status[t];
  for (int r = threadIdx.x; r < R; r += blockDim.x) a += active[r] != 0;
  sb[threadIdx.x] = b;
  sa[threadIdx.x] = a;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) {
      sb[threadIdx.x] |= sb[threadIdx.x + w];
      sa[threadIdx.x] += sa[threadIdx.x + w];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    chk[0] = sb[0];
    chk[1] = sa[0];
  }
}

__global__ void __launch_bounds__(64) fill_int_kernel(int* a, int n, int v) {
  const int i = blockIdx.x * 64 + threadIdx.x;
  if (i < n) a[i] = v;
}

// ---- host Sobol (Joe-Kuo directions, Gray code, zero point skipped) ---------------------
struct Sobol {
  int dim;
  std::vector<uint32_t> v;  // dim × 32
  std::vector<uint32_t> x;
  uint64_t n = 0;
  explicit Sobol(int dim_) : dim(dim_), v((size_t)dim_ * 32), x(dim_, 0u) {
    for (int j = 0; j < dim; ++j) {
      const int s = mrbo_sobol_table[j].s, a = mrbo_sobol_table[j].a;
      uint32_t m[33];
      for (int k = 1; k <= 32; ++k) {
        if (s == 0) m[k] = 1;
        else if (k <= s) m[k] = mrbo_sobol_table[j].m[k - 1];
        else {
          uint32_t mk = m[k - s] ^ (m[k - s] << s);
          for (int l = 1; l < s; ++l)
            if ((a >> (s - 1 - l)) & 1) mk ^= m[k - l] << l;
          m[k] = mk;
        }
      }
      for (int k = 1; k <= 32; ++k) v[(size_t)j * 32 + k - 1] = m[k] << (32 - k);
    }
  }
  void next(double* u) {
    int c = 0;
    while ((n >> c) & 1ULL) ++c;
    for (int j = 0; j < dim; ++j) {
      x[j] ^= v[(size_t)j * 32 + c];
      u[j] = (double)x[j] * (1.0 / 4294967296.0);
    }
    ++n;
  }
};

}  // namespace

static void fill_common(const mrbo_plan_t* P, KParams& kp) {
  memset(&kp, 0, sizeof kp);
  kp.d = P->d; kp.N = P->N; kp.Npad = P->Npad; kp.h = P->p.h; kp.M = P->p.M; kp.R = P->p.R;
  kp.nstarts = P->p.nstarts;
  kp.kernel = P->kernel; kp.rule = P->p.rule; kp.ell = P->ell; kp.cK = P->cK; kp.cP = P->cP; kp.psi0 = P->psi0; kp.d2psi0 = P->d2psi0; kp.sn2 = P->sn2;
  kp.gcert_mu = P->gcert_mu; kp.gcert_sig = P->gcert_sig;
  kp.gcert_d2 = (P->d2psi0 < 0.0) ? 1.01 * std::sqrt(-P->d2psi0) : -1.0;
  kp.fmin_base = P->fmin_base; kp.fmini = P->fmini; kp.theta = P->p.theta;
  kp.max_iters = P->p.max_iters; kp.max_ls = P->p.max_ls;
  kp.x_tol = P->p.x_tol; kp.f_tol = P->p.f_tol; kp.g_tol = P->p.g_tol; kp.htol = P->p.htol;
  kp.sigma_tol = P->p.sigma_tol; kp.seed = P->p.seed;
  kp.sample_offset = P->p.sample_offset;
  kp.samples_total = P->p.samples_total > 0 ? P->p.samples_total : P->p.M;
  kp.X0 = P->dX0; kp.c0 = P->dc0; kp.Linv = P->dLinv; kp.lbs = P->dlbs; kp.ubs = P->dubs;
  kp.work = P->dwork; kp.work_stride = P->work_stride; kp.queue = P->dqueue; kp.ytab = P->dytab;
  kp.cost = P->p.cost;
  kp.cost_c0 = P->p.cost_c0;
  kp.cost_tab = P->dcost;
}

// Device buffers of plan-less calls (mrbo_gp_fit: staging and the tile kernel's workspace) are
// pooled per device across calls -- a hipMalloc + hipFree pair costs ≈ 0.1 ms, the whole N = 128
// fit 0.4 ms.  A call takes the smallest free buffer that fits (or allocates one) and gives it back
// when it returns, after its stream has synchronised; concurrent calls never share a buffer.
struct DevPool {
  std::mutex m;
  std::vector<std::tuple<int, void*, size_t>> free;   // (device, pointer, bytes)
};
static DevPool g_pool;

static std::pair<void*, size_t> pool_take(size_t bytes) {
  int dev = 0;
  (void)hipGetDevice(&dev);
  {
    std::lock_guard<std::mutex> lk(g_pool.m);
    size_t best = g_pool.free.size();
    for (size_t i = 0; i < g_pool.free.size(); ++i) {
      const auto& [d, p, n] = g_pool.free[i];
      if (d == dev && n >= bytes && (best == g_pool.free.size() || n < std::get<2>(g_pool.free[best]))) best = i;
    }
    if (best < g_pool.free.size()) {
      auto r = std::make_pair(std::get<1>(g_pool.free[best]), std::get<2>(g_pool.free[best]));
      g_pool.free.erase(g_pool.free.begin() + best);
      return r;
    }
    // nothing fits: the free buffers of this device are smaller than what calls now ask for (a
    // BO loop's N grows by one per step), so release them instead of letting the pool grow
    for (size_t i = g_pool.free.size(); i-- > 0;)
      if (std::get<0>(g_pool.free[i]) == dev) {
        (void)hipFree(std::get<1>(g_pool.free[i]));
        g_pool.free.erase(g_pool.free.begin() + i);
      }
  }
  void* p = nullptr;
  if (hipMalloc(&p, bytes) != hipSuccess) return {nullptr, 0};
  return {p, bytes};
}

static void pool_give(void* p, size_t bytes) {
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> lk(g_pool.m);
  g_pool.free.emplace_back(dev, p, bytes);
}

// staging helper for MRBO_FLAG_HOST_POINTERS: the plan's persistent device buffers (slot k =
// the k-th staged argument of the call), so a host-pointer call allocates nothing once warm;
// without a plan (mrbo_gp_fit) the buffers come from the device pool and return to it
// Pinned host bounce buffers for the plan-less calls' packed transfers (mrbo_gp_fit: its inputs
// go to the device in one copy and its small outputs come back in one): pooled like DevPool, a
// hipHostMalloc costs far more than the copies it serves.
struct HostPool {
  std::mutex m;
  std::vector<std::pair<void*, size_t>> free;
};
static HostPool g_hpool;

struct Pinned {
  void* p = nullptr;
  size_t n = 0;
  explicit Pinned(size_t bytes) {
    if (!bytes) return;
    {
      std::lock_guard<std::mutex> lk(g_hpool.m);
      size_t best = g_hpool.free.size();
      for (size_t i = 0; i < g_hpool.free.size(); ++i)
        if (g_hpool.free[i].second >= bytes &&
            (best == g_hpool.free.size() || g_hpool.free[i].second < g_hpool.free[best].second))
          best = i;
      if (best < g_hpool.free.size()) {
        p = g_hpool.free[best].first;
        n = g_hpool.free[best].second;
        g_hpool.free.erase(g_hpool.free.begin() + best);
        return;
      }
      for (size_t i = g_hpool.free.size(); i-- > 0;) {   // too small for what calls now ask for
        (void)hipHostFree(g_hpool.free[i].first);
        g_hpool.free.erase(g_hpool.free.begin() + i);
      }
    }
    if (hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) p = nullptr;
    else n = bytes;
  }
  ~Pinned() {
    if (!p) return;
    std::lock_guard<std::mutex> lk(g_hpool.m);
    g_hpool.free.push_back({p, n});
  }
  void abandon() { p = nullptr; }   // a copy may still read it: keep it out of the pool
};

struct Stage {
  mrbo_plan_t* P;
  std::vector<std::pair<void*, size_t>> own;
  size_t k = 0;
  explicit Stage(mrbo_plan_t* plan = nullptr) : P(plan) {}
  ~Stage() { for (auto& b : own) if (b.first) pool_give(b.first, b.second); }
  // a launch that may still be running after an error: keep its buffers out of the pool (leaked)
  void abandon() { own.clear(); }
  void* slot(size_t bytes) {
    if (!P) {
      own.push_back(pool_take(bytes));
      return own.back().first;
    }
    auto& pool = P->stage;
    if (pool.size() <= k) pool.resize(k + 1, {nullptr, 0});
    auto& b = pool[k++];
    if (b.second < bytes) {
      if (b.first) (void)hipFree(b.first);
      b = {nullptr, 0};
      if (hipMalloc(&b.first, bytes) != hipSuccess) { b.first = nullptr; return nullptr; }
      b.second = bytes;
    }
    return b.first;
  }
  template <class T>
  int in(const T* h, size_t n, const T** dptr) {
    if (!h) { *dptr = nullptr; return 0; }
    void* d = slot(sizeof(T) * n);
    if (!d || hipMemcpy(d, h, sizeof(T) * n, hipMemcpyHostToDevice) != hipSuccess) return -1;
    *dptr = (const T*)d;
    return 0;
  }
  template <class T>
  int out(size_t n, T* h, T** dptr) {
    if (!h) { *dptr = nullptr; return 0; }
    void* d = slot(sizeof(T) * n);
    if (!d) return -1;
    *dptr = (T*)d;
    return 0;
  }
};

static int reduce_common(mrbo_plan_t* P, const double* values, const double* grad_x, const double* grad_theta,
                         int M, double* out, int mode, uint32_t flags, void* stream) {
  if (!P || !values || !out) return fail(MRBO_ERR_ARG, "null argument");
  hipStream_t st = (hipStream_t)stream;
  const int d = P->d, R = P->p.R, Ms = P->p.M;
  const size_t T = (size_t)Ms * R, W = 2 + 2 * d + 2;
  Stage sg(P);
  const double *dv = values, *dg = grad_x, *dt = grad_theta;
  double* dout = out;
  if (flags & MRBO_FLAG_HOST_POINTERS) {
    if (sg.in(values, T, &dv) || sg.in(grad_x, (size_t)d * T, &dg) || sg.in(grad_theta, T, &dt) ||
        sg.out(W * R, out, &dout))
      return fail(MRBO_ERR_NOMEM, "staging allocation failed");
  }
  hipLaunchKernelGGL(reduce_kernel, dim3(R, d + 2), dim3(256), 0, st, dv, dg, dt, M, Ms, d, mode, dout);
  HIP_TRY(hipGetLastError());
  if (flags & MRBO_FLAG_HOST_POINTERS) {
    HIP_TRY(hipStreamSynchronize(st));
    HIP_TRY(hipMemcpy(out, dout, sizeof(double) * W * R, hipMemcpyDeviceToHost));
  }
  return MRBO_OK;
}

// =========================================================================================
extern "C" {

const char* mrbo_version(void) { return "mrbo 0.2.0 (gfx950, fp64, ABI 2)"; }
const char* mrbo_last_error(void) { return g_err.c_str(); }

int mrbo_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int mrbo_plan_create(const mrbo_surrogate_t* s, const mrbo_params_t* p, int32_t device, mrbo_plan_t** out) {
  if (!s || !p || !out) return fail(MRBO_ERR_ARG, "null argument");
  *out = nullptr;
  const int d = s->d, N = s->N;
  if (d < 1 || N < 1 || !s->X || !s->L || !s->c || !s->y) return fail(MRBO_ERR_ARG, "bad surrogate (d=%d N=%d)", d, N);
  if (d > 16) return fail(MRBO_ERR_UNSUPPORTED, "d=%d > 16 not compiled", d);
  if (N > 512) return fail(MRBO_ERR_UNSUPPORTED, "N=%d > 512 not compiled", N);
  if (d > 8 && N > 128) return fail(MRBO_ERR_UNSUPPORTED, "d=%d > 8 with N=%d > 128 not compiled", d, N);
  if (p->h < 0 || p->h > FMAX - 1) return fail(MRBO_ERR_UNSUPPORTED, "h=%d outside [0,%d]", p->h, FMAX - 1);
  if (p->M < 1 || p->R < 1 || p->nstarts < 1 || !p->lbs || !p->ubs) return fail(MRBO_ERR_ARG, "bad params");
  if (p->rule != MRBO_RULE_EI && p->rule != MRBO_RULE_POI && p->rule != MRBO_RULE_LCB)
    return fail(MRBO_ERR_ARG, "unknown decision rule %d", (int)p->rule);
  if (s->kernel < 0 || s->kernel > 4) return fail(MRBO_ERR_ARG, "kernel id %d", s->kernel);
  if (p->cost < MRBO_COST_NONE || p->cost > MRBO_COST_LOGLINEAR) return fail(MRBO_ERR_ARG, "cost model %d", p->cost);
  if (p->cost != MRBO_COST_NONE && !p->cost_w) return fail(MRBO_ERR_ARG, "cost model without weights");
  if (p->cost != MRBO_COST_NONE && d > MAXD) return fail(MRBO_ERR_UNSUPPORTED, "cost model at d=%d > %d", d, MAXD);
  if (p->cost != MRBO_COST_NONE) {
    // c(x) must stay positive and finite on the box: α/c and the certificates' bound·(1/c) flip
    // sign otherwise (a negative bound would falsely certify a stationary point)
    if (!(p->cost_c0 > 0.0) || !std::isfinite(p->cost_c0)) return fail(MRBO_ERR_ARG, "cost_c0=%g must be > 0", p->cost_c0);
    for (int a = 0; a < d; ++a) {
      if (!std::isfinite(p->cost_w[a])) return fail(MRBO_ERR_ARG, "cost weight %d is not finite", a);
      if (p->cost == MRBO_COST_QUADRATIC && p->cost_w[a] < 0.0)
        return fail(MRBO_ERR_ARG, "quadratic cost weight %d = %g < 0", a, p->cost_w[a]);
      if (!(p->ubs[a] > p->lbs[a])) return fail(MRBO_ERR_ARG, "cost model needs ub > lb (dimension %d)", a);
    }
  }
  if (s->kernel == MRBO_KERNEL_PERIODIC && !(s->period > 0.0)) return fail(MRBO_ERR_ARG, "period %g", s->period);
  const int ldL = s->ldL > 0 ? s->ldL : N;

  mrbo_plan* P = new mrbo_plan();
  P->device = device;
  P->d = d;
  P->N = N;
  P->RPL = (N <= 64) ? 1 : (N <= 128) ? 2 : (N <= 256) ? 4 : 8;
  P->NR = 64 * P->RPL;
  P->Npad = P->NR;
  P->p = *p;
  P->lbs.assign(p->lbs, p->lbs + d);
  P->ubs.assign(p->ubs, p->ubs + d);
  P->p.lbs = nullptr;
  P->p.ubs = nullptr;
  if (p->cost != MRBO_COST_NONE) P->cost_w.assign(p->cost_w, p->cost_w + d);
  P->p.cost_w = nullptr;
  P->kernel = s->kernel;
  P->ell = s->lengthscale;
  P->sn2 = s->sigma_n2;
  P->fmini = s->fmini;
  P->fmin_base = s->y[0];
  for (int i = 1; i < N; ++i) P->fmin_base = std::min(P->fmin_base, s->y[i]);
  const double ell = s->lengthscale;
  switch (s->kernel) {
    case 0: P->cK = std::sqrt(5.0) / ell; P->d2psi0 = -P->cK * P->cK / 3.0; break;
    case 1: P->cK = std::sqrt(3.0) / ell; P->d2psi0 = -P->cK * P->cK; break;
    case 2: P->cK = 1.0 / ell; P->d2psi0 = P->cK * P->cK; break;
    case 4: P->cK = 1.0 / (ell * ell); P->cP = 2.0 * M_PI / s->period; P->d2psi0 = -P->cK * P->cP * P->cP; break;
    default: P->cK = 1.0 / (ell * ell); P->d2psi0 = -P->cK; break;
  }
  P->psi0 = 1.0;
  // max_ρ |ψ'(ρ)| in closed form (+1% margin) and √(ψ(0)·(−ψ''(0))) for the gradient certificate
  switch (P->kernel) {
    case 0: { const double s = 0.5 * (1.0 + std::sqrt(5.0));
              P->gcert_mu = 1.01 * P->cK * (s / 3.0) * (1.0 + s) * std::exp(-s); break; }
    case 1: P->gcert_mu = 1.01 * P->cK * std::exp(-1.0); break;
    case 2: P->gcert_mu = 1.01 * P->cK; break;
    case 4: P->gcert_mu = 1.01 * P->cK * P->cP; break;   // |ψ'| = ψ (2π/(pℓ²)) |sin t| ≤ 2π/(pℓ²)
    default: P->gcert_mu = 1.01 * std::sqrt(P->cK) * std::exp(-0.5); break;
  }
  P->gcert_sig = (P->d2psi0 < 0.0) ? 1.01 * std::sqrt(P->psi0 * -P->d2psi0) : -1.0;

  // L0^-1 by forward substitution on the unit columns, packed column-major (Npad rows)
  const int Npad = P->Npad;
  std::vector<double> Li((size_t)N * N, 0.0);  // col-major N×N
  for (int j = 0; j < N; ++j) {
    double* col = &Li[(size_t)j * N];
    for (int i = j; i < N; ++i) {
      double sacc = (i == j) ? 1.0 : 0.0;
      for (int k = j; k < i; ++k) sacc -= s->L[i + (size_t)ldL * k] * col[k];
      col[i] = sacc / s->L[i + (size_t)ldL * i];
    }
  }
  std::vector<double> X0((size_t)d * P->NR, 0.0), c0(P->NR, 0.0);
  for (int i = 0; i < N; ++i) {
    for (int a = 0; a < d; ++a) X0[(size_t)a * P->NR + i] = s->X[a + (size_t)d * i];
    c0[i] = s->c[i];
  }

  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) { delete P; return fail(MRBO_ERR_HIP, "hipSetDevice(%d): %s", device, hipGetErrorString(e)); }
  KernelSet ks;
  // the FMAX = 4 unit when the horizon allows it and the library carries it
  P->fx = (p->h <= F4_HMAX && d <= F4_DMAX && unit_present(d, 1)) ? 1 : 0;
  if (!get_kset(d, P->RPL, P->fx, ks)) {
    delete P;
    return fail(MRBO_ERR_UNSUPPORTED, "d=%d (rows per lane %d) not compiled into this library", d, P->RPL);
  }
  if (ks.kparams_bytes != sizeof(KParams)) {
    delete P;
    return fail(MRBO_ERR_UNSUPPORTED, "kernel unit d=%d (FMAX %d) was compiled against another KParams layout "
                "(%zu vs %zu bytes): rebuild the library", d, P->fx ? 4 : 6, ks.kparams_bytes, sizeof(KParams));
  }
  // the kernel's image of L0⁻¹ (zero above the diagonal and on padded rows); the global
  // variant appends a row-packed copy (row k: columns 0..k) for the backward product
  std::vector<double> packed((size_t)ks.linv_dev, 0.0);
  for (int j = 0; j < N; ++j)
    for (int i = j; i < N; ++i) {
      const size_t blk = (size_t)(i / 64) * (i / 64 + 1) / 2 + j / 64;   // block (i/64, j/64), j/64 ≤ i/64
      size_t at;
      if (ks.blocks)   // LDS blocks, column-major inside with leading dimension ld
        at = blk * 64 * ks.ld + (size_t)(j % 64) * ks.ld + i % 64;
      else if (ks.gl)  // L2 blocks, forward copy: (i, j) at j·64 + i
        at = blk * 64 * 64 + (size_t)(j % 64) * 64 + i % 64;
      else
        at = (size_t)j * ks.ld + i;
      packed[at] = Li[i + (size_t)N * j];
      if (ks.gl) {     // backward copy (after all forward blocks): (i, j) at i·64 + j
        const size_t nblk = (size_t)P->RPL * (P->RPL + 1) / 2;
        packed[(nblk + blk) * 64 * 64 + (size_t)(i % 64) * 64 + j % 64] = Li[i + (size_t)N * j];
        // the LDS-resident blocks (gl_lds_slot) once more, after both copies, in the LD = 65
        // layout of the LDS kernels ((i, j) at j·65 + i), staged into LDS by every workgroup
        const int nlb = (int)(ks.linv_doubles / (64 * 65));
        const int slot = gl_lds_slot((int)blk);
        if (slot >= 0 && slot < nlb)
          packed[2 * nblk * 64 * 64 + (size_t)slot * 64 * 65 + (size_t)(j % 64) * 65 + i % 64] = Li[i + (size_t)N * j];
      }
    }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) { delete P; return fail(MRBO_ERR_HIP, "device props"); }
  const size_t linv_bytes = sizeof(double) * (size_t)ks.linv_doubles;
  const int ns = P->p.nstarts;
  const size_t xs_bytes = sizeof(double) * (size_t)(((size_t)ns * d + 1) & ~(size_t)1);
  P->xs_lds = xs_bytes <= 8192 ? 1 : 0;
  // batched start values: start tables kxb (NR × ns) and y0sq (ns), square L0⁻¹ only; kept only
  // if they cost no resident waves
  const size_t ng = (size_t)(d + 1) * (d + 2) / 2;
  const size_t kxb_bytes = sizeof(double) * ((((size_t)P->NR * ns + 1) & ~(size_t)1) + (((size_t)ns * ng + 1) & ~(size_t)1));
  const size_t fixed = linv_bytes + (P->xs_lds ? xs_bytes : 0);
  int wpg0 = 0, blocks0 = 0;
  size_t smem0 = 0;
  int maxw = ks.max_threads / WAVE;
  // MRBO_MAX_WPG (A/B runs only): at most this many waves per rollout workgroup -- fewer resident
  // waves per XCD, a smaller L2 footprint of their work slots and scratch
  if (const char* mw = getenv("MRBO_MAX_WPG")) maxw = std::max(1, std::min(maxw, atoi(mw)));
  // Matérn-5/2 + EI: the compile-time specialised rollout kernel
  // (MRBO_GENERIC_KERNEL=1 forces the generic instantiation, for A/B runs and tests)
  const char* gen = getenv("MRBO_GENERIC_KERNEL");
  P->spec = (P->kernel == MRBO_KERNEL_MATERN52 && P->p.rule == MRBO_RULE_EI && P->p.cost == MRBO_COST_NONE &&
             ks.rollout_spec && !(gen && gen[0] == '1')) ? 1 : 0;
  // N ≤ 32 with at most 32 inner-solve starts: the half-wave kernel, two trajectories per wave
  // (MRBO_HALF=0 keeps the full-wave one, for A/B runs and tests)
  const char* half = getenv("MRBO_HALF");
  if (P->spec == 1 && ks.rollout_half && N <= 32 && ns <= 32 && !(half && half[0] == '0')) P->spec = 2;
  // Matérn-5/2 + EI + the quadratic cost (C5 --cost): its own specialisation where compiled
  if (P->kernel == MRBO_KERNEL_MATERN52 && P->p.rule == MRBO_RULE_EI && P->p.cost == MRBO_COST_QUADRATIC &&
      ks.rollout_cost && !(gen && gen[0] == '1'))
    P->spec = 3;
  const void* rk = P->spec == 3 ? ks.rollout_cost : P->spec == 2 ? ks.rollout_half : P->spec ? ks.rollout_spec
                                                                                              : ks.rollout;
  const size_t wave_bytes = P->spec == 2 ? ks.wave_bytes_half : ks.wave_bytes;
  const int waves0 =
      pick_grid(rk, fixed, wave_bytes, prop.multiProcessorCount, wpg0, blocks0, smem0, 0, maxw);
  P->batch = 0;
  if (ks.square && P->xs_lds && ns <= 64) {
    int wpg1 = 0, blocks1 = 0;
    size_t smem1 = 0;
    const int waves1 = pick_grid(rk, fixed + kxb_bytes, wave_bytes, prop.multiProcessorCount, wpg1, blocks1,
                                 smem1);
    if (waves1 >= waves0 && waves1 > 0) { P->batch = 1; P->wpg = wpg1; P->blocks = blocks1; P->smem = smem1; }
  }
  if (!P->batch) { P->wpg = wpg0; P->blocks = blocks0; P->smem = smem0; }
  // packed layouts: the start tables live in global memory (no LDS, no occupancy cost)
  if (!ks.square && P->xs_lds && ns <= 64) P->batch = 1;
  if (!waves0 ||
      !pick_grid(ks.evalb, linv_bytes, ks.wave_bytes, prop.multiProcessorCount, P->ewpg, P->eblocks, P->esmem, 0,
                 maxw)) {
    delete P;
    return fail(MRBO_ERR_UNSUPPORTED, "no feasible launch configuration");
  }
  const int slots = std::max(P->blocks * P->wpg, P->eblocks * P->ewpg);
  // per wave slot: E (FMAX × NR) and C ((FMAX+1) × NR), then the batched start pass's per-start
  // sums (64 × 8) for the packed layouts
  // and, for the L2-fed layouts, room for the value pass's stashed gradient columns (RPL × d × 64,
  // MRBO_GL_EAGER builds)
  P->work_stride = (long long)(2 * FMAX + 1) * P->NR + 64 * 8 + (ks.gl ? (long long)P->NR * d : 0);
  bool ok = hipMalloc(&P->dX0, sizeof(double) * X0.size()) == hipSuccess &&
            hipMalloc(&P->dc0, sizeof(double) * c0.size()) == hipSuccess &&
            hipMalloc(&P->dLinv, sizeof(double) * packed.size()) == hipSuccess &&
            hipMalloc(&P->dlbs, sizeof(double) * d) == hipSuccess &&
            hipMalloc(&P->dubs, sizeof(double) * d) == hipSuccess &&
            hipMalloc(&P->dwork, sizeof(double) * (size_t)slots * P->work_stride) == hipSuccess &&
            (!P->batch || !ks.square ||
             hipMalloc(&P->dytab, sizeof(double) * (size_t)ns * P->NR) == hipSuccess) &&
            (!P->batch || ks.square ||
             (hipMalloc(&P->dkxb, sizeof(double) * (size_t)P->NR * ns) == hipSuccess &&
              hipMalloc(&P->dgtab, sizeof(double) * (size_t)ns * ng) == hipSuccess)) &&
            hipMalloc(&P->dqueue, sizeof(int) * MRBO_QUEUE_INTS) == hipSuccess &&
            (P->p.cost == MRBO_COST_NONE || hipMalloc(&P->dcost, sizeof(double) * 3 * d) == hipSuccess);
  if (ok && P->p.cost != MRBO_COST_NONE) {
    std::vector<double> tab(3 * (size_t)d);
    for (int a = 0; a < d; ++a) {
      tab[a] = P->lbs[a];
      tab[d + a] = P->ubs[a] - P->lbs[a];
      tab[2 * d + a] = P->cost_w[a];
    }
    ok = hipMemcpy(P->dcost, tab.data(), sizeof(double) * 3 * d, hipMemcpyHostToDevice) == hipSuccess;
  }
  ok = ok && hipMemcpy(P->dX0, X0.data(), sizeof(double) * X0.size(), hipMemcpyHostToDevice) == hipSuccess &&
       hipMemcpy(P->dc0, c0.data(), sizeof(double) * c0.size(), hipMemcpyHostToDevice) == hipSuccess &&
       hipMemcpy(P->dLinv, packed.data(), sizeof(double) * packed.size(), hipMemcpyHostToDevice) == hipSuccess &&
       hipMemcpy(P->dlbs, P->lbs.data(), sizeof(double) * d, hipMemcpyHostToDevice) == hipSuccess &&
       hipMemcpy(P->dubs, P->ubs.data(), sizeof(double) * d, hipMemcpyHostToDevice) == hipSuccess &&
       hipMemset(P->dwork, 0, sizeof(double) * (size_t)slots * P->work_stride) == hipSuccess;
  // the timing ring's events are created on first use by a launch (launch_events), not here: a plan
  // used for a few launches (the Julia drop-in's R = 1 calls) creates only what it records
  if (!ok) {
    mrbo_plan_destroy(P);
    return fail(MRBO_ERR_NOMEM, "device allocation failed");
  }
  *out = P;
  return MRBO_OK;
}

int mrbo_plan_destroy(mrbo_plan_t* P) {
  if (!P) return MRBO_OK;
  for (void* b : {(void*)P->dX0, (void*)P->dc0, (void*)P->dLinv, (void*)P->dlbs, (void*)P->dubs, (void*)P->dwork, (void*)P->dytab,
                  (void*)P->dkxb, (void*)P->dgtab, (void*)P->dqueue, (void*)P->dcost, P->oorder})
    if (b) (void)hipFree(b);
  for (auto& b : P->stage)
    if (b.first) (void)hipFree(b.first);
  for (auto& b : P->solve)
    if (b.first) (void)hipFree(b.first);
  if (P->hchk) (void)hipHostFree(P->hchk);
  for (hipEvent_t e : P->ev)
    if (e) (void)hipEventDestroy(e);
  for (hipEvent_t e : P->chk_ev)
    if (e) (void)hipEventDestroy(e);
  delete P;
  return MRBO_OK;
}

// one launch of the rollout kernel: Monte-Carlo draws from rnstream, or the Gauss–Hermite
// observable from (ghq_nodes, ghq_w) when those are given
static int simulate_common(mrbo_plan_t* P, const double* x0s, const double* rnstream, const double* ghq_nodes,
                           const double* ghq_w, const double* xstarts, const double* dual_y_dx,
                           const double* replay_x, double* values, double* grad_x, double* grad_theta,
                           int32_t* status, double* policy_x, double* obs, int64_t* evals, uint32_t flags,
                           void* stream) {
  if (!P || !x0s || !(rnstream || (ghq_nodes && ghq_w)) || !xstarts || !values || !status)
    return fail(MRBO_ERR_ARG, "null argument");
  const bool with_grad = !(flags & MRBO_FLAG_NO_GRADIENT);
  if (with_grad && (!grad_x || !grad_theta)) return fail(MRBO_ERR_ARG, "gradient containers required");
  hipStream_t st = (hipStream_t)stream;
  if (hipSetDevice(P->device) != hipSuccess) return fail(MRBO_ERR_HIP, "hipSetDevice");
  const int d = P->d, h = P->p.h, M = P->p.M, R = P->p.R;
  const size_t T = (size_t)M * R;
  KParams kp;
  fill_common(P, kp);
  kp.with_gradient = with_grad ? 1 : 0;
  kp.T = (long long)T;
  Stage sg(P);
  const bool host = flags & MRBO_FLAG_HOST_POINTERS;
  double *dvalues = values, *dgx = grad_x, *dgt = grad_theta, *dpol = policy_x, *dobs = obs;
  int32_t* dstatus = status;
  int64_t* devals = evals;
  if (host) {
    if (sg.in(x0s, (size_t)d * R, &kp.x0s) || sg.in(rnstream, (size_t)M * (d + 1) * (h + 1), &kp.rn) ||
        sg.in(ghq_nodes, (size_t)M * (h + 1), &kp.ghq_nodes) || sg.in(ghq_w, (size_t)M * (h + 1), &kp.ghq_w) ||
        sg.in(xstarts, (size_t)d * P->p.nstarts, &kp.xstarts) ||
        sg.in(dual_y_dx, (size_t)d * std::max(h, 1) * T, &kp.dual_y) ||
        sg.in(replay_x, (size_t)d * std::max(h, 1) * T, &kp.replay) || sg.out(T, values, &dvalues) ||
        sg.out((size_t)d * T, with_grad ? grad_x : nullptr, &dgx) || sg.out(T, with_grad ? grad_theta : nullptr, &dgt) ||
        sg.out(T, status, &dstatus) || sg.out((size_t)d * (h + 1) * T, policy_x, &dpol) ||
        sg.out((size_t)(h + 1) * T, obs, &dobs) || sg.out((size_t)NCOUNT * T, evals, &devals))
      return fail(MRBO_ERR_NOMEM, "staging allocation failed");
  } else {
    kp.x0s = x0s; kp.rn = rnstream; kp.xstarts = xstarts; kp.dual_y = dual_y_dx; kp.replay = replay_x;
    kp.ghq_nodes = ghq_nodes; kp.ghq_w = ghq_w;
  }
  kp.values = dvalues; kp.grad_x = with_grad ? dgx : nullptr; kp.grad_theta = with_grad ? dgt : nullptr;
  kp.status = (int*)dstatus; kp.policy = dpol; kp.obs = dobs; kp.evals = (long long*)devals;
  kp.order = P->order;
  kp.skip_active = P->skip_active;
  HIP_TRY(hipMemsetAsync(P->dqueue, 0, sizeof(int) * MRBO_QUEUE_INTS, st));
#ifdef MRBO_STAMPS
  static unsigned long long* dstamps = nullptr;
  if (!dstamps) HIP_TRY(hipMalloc(&dstamps, sizeof(unsigned long long) * NSTAMP_SLOTS));
  HIP_TRY(hipMemsetAsync(dstamps, 0, sizeof(unsigned long long) * NSTAMP_SLOTS, st));
  kp.stamps = dstamps;
#endif
#ifdef MRBO_TAIL   // per-wave (start, end, trajectories) of the rollout launch: the tail of the persistent grid
  static unsigned long long* dtail = nullptr;
  static int ntail = 0;
  const int nwaves = P->blocks * P->wpg;
  const size_t ntailw = 3 * (size_t)nwaves + (size_t)T;   // + one wall time per trajectory
  if ((long long)ntailw > ntail) {
    if (dtail) HIP_TRY(hipFree(dtail));
    HIP_TRY(hipMalloc(&dtail, sizeof(unsigned long long) * ntailw));
    ntail = (int)ntailw;
  }
  HIP_TRY(hipMemsetAsync(dtail, 0, sizeof(unsigned long long) * ntailw, st));
  kp.stamps = dtail;
#endif
  kp.xs_lds = P->xs_lds;
  kp.batch = P->batch;
  if (P->batch && P->RPL > 1) {   // packed layouts: global start tables for this launch's xstarts
    kp.kxb_g = P->dkxb;
    kp.gtab_g = P->dgtab;
    launch_tables(d, P->RPL, P->fx, P->p.nstarts, st, kp);
    HIP_TRY(hipGetLastError());
  }
  if (P->batch && P->RPL == 1) {   // square layout: the launch's Y0(x_start) table, written once
    launch_ytab(d, P->fx, P->spec, dim3(P->wpg * WAVE), P->smem, st, kp);
    HIP_TRY(hipGetLastError());
  }
  const int slot = (int)(P->nlaunch % mrbo_plan::NEV);
  if (!P->ev[2 * slot]) {   // lazily created ring slot (destroyed with the plan)
    HIP_TRY(hipEventCreate(&P->ev[2 * slot]));
    HIP_TRY(hipEventCreate(&P->ev[2 * slot + 1]));
  }
  HIP_TRY(hipEventRecord(P->ev[2 * slot], st));
  launch_rollout(d, P->RPL, P->fx, P->spec, dim3(P->blocks), dim3(P->wpg * WAVE), P->smem, st, kp);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipEventRecord(P->ev[2 * slot + 1], st));
  ++P->nlaunch;
#ifdef MRBO_TAIL
  {
    std::vector<unsigned long long> h(3 * (size_t)nwaves + (size_t)T);
    HIP_TRY(hipStreamSynchronize(st));
    HIP_TRY(hipMemcpy(h.data(), dtail, sizeof(unsigned long long) * h.size(), hipMemcpyDeviceToHost));
    unsigned long long t0 = ~0ull, t1 = 0;
    long long ntr = 0;
    int nmin = 1 << 30, nmax = 0, nw = 0;
    for (int w = 0; w < nwaves; ++w) {
      if (!h[3 * w + 1]) continue;
      ++nw;
      t0 = std::min(t0, h[3 * w]);
      t1 = std::max(t1, h[3 * w + 1]);
      ntr += (long long)h[3 * w + 2];
      nmin = std::min(nmin, (int)h[3 * w + 2]);
      nmax = std::max(nmax, (int)h[3 * w + 2]);
    }
    std::vector<double> ends;
    double busy = 0, headv = 0;
    for (int w = 0; w < nwaves; ++w) {
      if (!h[3 * w + 1]) continue;
      ends.push_back((double)(h[3 * w + 1] - t0));
      busy += (double)(h[3 * w + 1] - h[3 * w]);
      headv += (double)(h[3 * w] - t0);
    }
    std::sort(ends.begin(), ends.end());
    const double span = (double)(t1 - t0);
    auto pct = [&](double q) { return ends[std::min(ends.size() - 1, (size_t)(q * ends.size()))] / span; };
    fprintf(stderr, "[mrbo tail] waves %d span %.1f us  busy %.4f  start skew %.4f  idle tail %.4f  "
            "ends p0 %.4f p10 %.4f p50 %.4f p90 %.4f  traj/wave %d..%d  us/traj/wave %.2f\n",
            nw, span / 100.0, busy / (nw * span), headv / (nw * span), 1.0 - (busy + headv) / (nw * span),
            pct(0.0), pct(0.1), pct(0.5), pct(0.9), nmin, nmax, busy / 100.0 / (double)std::max(ntr, 1ll));
    // MRBO_TAIL_DUMP=path: append this launch's per-trajectory wall times (int64 REFCLK ticks, T)
    // and, when the caller asked for them, its work counters (int64, NCOUNT·T) -- calibration data
    // for the schedule's work weights
    if (const char* path = getenv("MRBO_TAIL_DUMP")) {
      if (FILE* f = fopen(path, "ab")) {
        const long long hdr[2] = {(long long)T, evals ? (long long)NCOUNT : 0ll};
        fwrite(hdr, sizeof(hdr), 1, f);
        fwrite(h.data() + 3 * (size_t)nwaves, sizeof(unsigned long long), (size_t)T, f);
        if (evals) {
          std::vector<long long> ev((size_t)NCOUNT * T);
          HIP_TRY(hipMemcpy(ev.data(), devals, sizeof(long long) * ev.size(), hipMemcpyDeviceToHost));
          fwrite(ev.data(), sizeof(long long), ev.size(), f);
        }
        fclose(f);
      }
    }
  }
#endif
#ifdef MRBO_STAMPS
  {
    // region names follow the STAMP(W, k) sites in mrbo_rollout.hip
    static const char* stamp_names[NSTAMP] = {"kernel rows", "forward L0^-1 B", "wave reductions", "fantasy rows+Gram+mu",
                                              "sigma+EI partials", "backward w/P", "Hessian reductions",
                                              "Hessian assembly", "Newton/draw bookkeeping (outside eval)",
                                              "adjoint pair", "draw+condition", "resolve+adjoint setup",
                                              "Newton accept/convergence", "Newton direction", "Newton trial point",
                                              "batched start values", "multistart loop (certified starts)",
                                              "Newton Gershgorin retry", "Newton substitutions",
                                              "Newton Armijo/accept", "Newton certificates", "Newton projected-gradient test"};
    unsigned long long hs[NSTAMP_SLOTS];
    HIP_TRY(hipStreamSynchronize(st));
    HIP_TRY(hipMemcpy(hs, dstamps, sizeof(hs), hipMemcpyDeviceToHost));
    double tot = 0;
    for (int k = 0; k < NSTAMP; ++k) tot += (double)hs[k];
    for (int k = 0; k < NSTAMP; ++k)
      fprintf(stderr, "[mrbo stamps] %-40s %6.2f%%  %.3e ticks/traj\n", stamp_names[k], 100.0 * hs[k] / tot,
              (double)hs[k] / (double)T);
    fprintf(stderr, "[mrbo stamps] Gershgorin retries per trajectory: %.3f\n", (double)hs[STAMP_RETRY] / (double)T);
  }
#endif
  if (host) {
    HIP_TRY(hipStreamSynchronize(st));
    HIP_TRY(hipMemcpy(values, dvalues, sizeof(double) * T, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(status, dstatus, sizeof(int32_t) * T, hipMemcpyDeviceToHost));
    if (with_grad) {
      HIP_TRY(hipMemcpy(grad_x, dgx, sizeof(double) * d * T, hipMemcpyDeviceToHost));
      HIP_TRY(hipMemcpy(grad_theta, dgt, sizeof(double) * T, hipMemcpyDeviceToHost));
    }
    if (policy_x) HIP_TRY(hipMemcpy(policy_x, dpol, sizeof(double) * d * (h + 1) * T, hipMemcpyDeviceToHost));
    if (obs) HIP_TRY(hipMemcpy(obs, dobs, sizeof(double) * (h + 1) * T, hipMemcpyDeviceToHost));
    if (evals) HIP_TRY(hipMemcpy(evals, devals, sizeof(int64_t) * NCOUNT * T, hipMemcpyDeviceToHost));
  }
  return MRBO_OK;
}

int mrbo_simulate_mc(mrbo_plan_t* P, const double* x0s, const double* rnstream, const double* xstarts,
                     const double* dual_y_dx, const double* replay_x, double* values, double* grad_x,
                     double* grad_theta, int32_t* status, double* policy_x, double* obs, int64_t* evals,
                     uint32_t flags, void* stream) {
  if (!rnstream) return fail(MRBO_ERR_ARG, "null rnstream");
  return simulate_common(P, x0s, rnstream, nullptr, nullptr, xstarts, dual_y_dx, replay_x, values, grad_x,
                         grad_theta, status, policy_x, obs, evals, flags, stream);
}

int mrbo_simulate_ghq(mrbo_plan_t* P, const double* x0s, const double* nodes, const double* weights,
                      const double* xstarts, const double* dual_y_dx, const double* replay_x, double* values,
                      double* grad_x, double* grad_theta, int32_t* status, double* policy_x, double* obs,
                      int64_t* evals, uint32_t flags, void* stream) {
  if (!nodes || !weights) return fail(MRBO_ERR_ARG, "null nodes / weights");
  return simulate_common(P, x0s, nullptr, nodes, weights, xstarts, dual_y_dx, replay_x, values, grad_x, grad_theta,
                         status, policy_x, obs, evals, flags, stream);
}

int mrbo_eto_reduce(mrbo_plan_t* P, const double* values, const double* grad_x, const double* grad_theta,
                    double* eto, uint32_t flags, void* stream) {
  return reduce_common(P, values, grad_x, grad_theta, P ? P->p.M : 0, eto, 0, flags, stream);
}

int mrbo_partial_moments(mrbo_plan_t* P, const double* values, const double* grad_x, const double* grad_theta,
                         int32_t M_local, double* moments, uint32_t flags, void* stream) {
  // the launch's outputs are laid out with the plan's M as the restart stride: M_local < M
  // reduces the first M_local samples of every restart
  if (P && (M_local < 1 || M_local > P->p.M)) return fail(MRBO_ERR_ARG, "M_local=%d outside [1, %d]", M_local, P->p.M);
  return reduce_common(P, values, grad_x, grad_theta, M_local, moments, 1, flags, stream);
}

int mrbo_sga_step(mrbo_plan_t* P, const double* eto, double* x0s, int32_t* active, double sample_size, double eta,
                  uint32_t flags, void* stream) {
  if (!P || !eto || !x0s || !active) return fail(MRBO_ERR_ARG, "null argument");
  if (flags & MRBO_FLAG_HOST_POINTERS) return fail(MRBO_ERR_ARG, "mrbo_sga_step takes device pointers");
  if (hipSetDevice(P->device) != hipSuccess) return fail(MRBO_ERR_HIP, "hipSetDevice");
  const int R = P->p.R;
  hipLaunchKernelGGL(sga_kernel, dim3((R + 63) / 64), dim3(64), 0, (hipStream_t)stream, eto, x0s, (int*)active, R, P->d,
                     sample_size, eta);
  HIP_TRY(hipGetLastError());
  return MRBO_OK;
}

int mrbo_adam_step(mrbo_plan_t* P, const double* eto, double* x0s, int32_t* active, double* m, double* v, int32_t t,
                   double sample_size, double eta, double beta1, double beta2, double eps, uint32_t flags,
                   void* stream) {
  if (!P || !eto || !x0s || !active || !m || !v) return fail(MRBO_ERR_ARG, "null argument");
  if (flags & MRBO_FLAG_HOST_POINTERS) return fail(MRBO_ERR_ARG, "mrbo_adam_step takes device pointers");
  if (t < 1) return fail(MRBO_ERR_ARG, "t=%d: the update count starts at 1", t);
  if (hipSetDevice(P->device) != hipSuccess) return fail(MRBO_ERR_HIP, "hipSetDevice");
  const int R = P->p.R;
  const double c1 = 1.0 - std::pow(beta1, (double)t), c2 = 1.0 - std::pow(beta2, (double)t);
  hipLaunchKernelGGL(adam_kernel, dim3((R + 63) / 64), dim3(64), 0, (hipStream_t)stream, eto, x0s, (int*)active, m, v,
                     R, P->d, sample_size, eta, beta1, beta2, eps, c1, c2);
  HIP_TRY(hipGetLastError());
  return MRBO_OK;
}

int mrbo_merge_moments(mrbo_plan_t* P, int32_t nshards, const double* moments, const int64_t* counts, double* eto,
                       uint32_t flags, void* stream) {
  if (!P || !moments || !counts || !eto) return fail(MRBO_ERR_ARG, "null argument");
  if (flags & MRBO_FLAG_HOST_POINTERS) return fail(MRBO_ERR_ARG, "mrbo_merge_moments takes device moments / eto");
  if (nshards < 1 || nshards > MERGE_MAX_SHARDS)
    return fail(MRBO_ERR_ARG, "nshards=%d outside [1, %d]", nshards, MERGE_MAX_SHARDS);
  MergeCounts cnt{};
  long long tot = 0;
  for (int k = 0; k < nshards; ++k) {
    if (counts[k] < 0) return fail(MRBO_ERR_ARG, "negative shard count %lld", (long long)counts[k]);
    cnt.n[k] = counts[k];
    tot += counts[k];
  }
  if (tot < 1) return fail(MRBO_ERR_ARG, "no samples in any shard");
  if (hipSetDevice(P->device) != hipSuccess) return fail(MRBO_ERR_HIP, "hipSetDevice");
  const int R = P->p.R, d = P->d, nthr = R * (d + 2);
  hipLaunchKernelGGL(merge_kernel, dim3((nthr + 63) / 64), dim3(64), 0, (hipStream_t)stream, moments, (int)nshards, cnt,
                     R, d, eto);
  HIP_TRY(hipGetLastError());
  return MRBO_OK;
}

// slot k of the plan's outer-ascent buffers, at least `bytes` (contents kept only while large enough)
static void* solve_slot(mrbo_plan_t* P, size_t k, size_t bytes) {
  auto& pool = P->solve;
  if (pool.size() <= k) pool.resize(k + 1, {nullptr, 0});
  auto& b = pool[k];
  if (b.second < bytes) {
    if (b.first) (void)hipFree(b.first);
    b = {nullptr, 0};
    if (hipMalloc(&b.first, bytes) != hipSuccess) return nullptr;
    b.second = bytes;
  }
  return b.first;
}

int mrbo_stochastic_solve(mrbo_plan_t* P, double* x0s, const double* rnstream, const double* xstarts,
                          const double* dual_y_dx, const mrbo_solve_opts_t* o, double* eto, int32_t* active,
                          int32_t* result, uint32_t flags, void* stream) {
  if (!P || !x0s || !rnstream || !xstarts || !o || !result) return fail(MRBO_ERR_ARG, "null argument");
  if (o->iterations < 1) return fail(MRBO_ERR_ARG, "iterations=%d: at least one", o->iterations);
  if (o->optimizer != MRBO_OPT_SGA && o->optimizer != MRBO_OPT_ADAM)
    return fail(MRBO_ERR_ARG, "optimizer=%d unknown", o->optimizer);
  if (flags & ~(uint32_t)MRBO_FLAG_HOST_POINTERS) return fail(MRBO_ERR_ARG, "flags: only MRBO_FLAG_HOST_POINTERS");
  if (hipSetDevice(P->device) != hipSuccess) return fail(MRBO_ERR_HIP, "hipSetDevice");
  hipStream_t st = (hipStream_t)stream;
  const bool host = flags & MRBO_FLAG_HOST_POINTERS;
  const int d = P->d, M = P->p.M, R = P->p.R, h = P->p.h, W = 2 + 2 * d + 2;
  const size_t T = (size_t)M * R;
  const size_t nx = (size_t)d * R, nrn = (size_t)M * (d + 1) * (h + 1), nxs = (size_t)d * P->p.nstarts;
  const size_t ndual = (size_t)d * std::max(h, 1) * T;
  const double sample_size = o->sample_size > 0 ? o->sample_size : (double)M;
  // device state: x0 (d×R), the launch outputs, the ETO rows, the stop flags, Adam's moments, the checks
  double* dx0 = host ? (double*)solve_slot(P, 0, sizeof(double) * nx) : x0s;
  const double* drn = host ? (const double*)solve_slot(P, 1, sizeof(double) * nrn) : rnstream;
  const double* dxs = host ? (const double*)solve_slot(P, 2, sizeof(double) * nxs) : xstarts;
  const double* ddual = (host && dual_y_dx) ? (const double*)solve_slot(P, 3, sizeof(double) * ndual) : dual_y_dx;
  double* deto = (host || !eto) ? (double*)solve_slot(P, 4, sizeof(double) * R * W) : eto;
  int32_t* dact = (host || !active) ? (int32_t*)solve_slot(P, 5, sizeof(int32_t) * R) : active;
  double* dvals = (double*)solve_slot(P, 6, sizeof(double) * T);
  double* dgx = (double*)solve_slot(P, 7, sizeof(double) * d * T);
  double* dgt = (double*)solve_slot(P, 8, sizeof(double) * T);
  int32_t* dst = (int32_t*)solve_slot(P, 9, sizeof(int32_t) * T);
  double* dm = o->optimizer == MRBO_OPT_ADAM ? (double*)solve_slot(P, 10, sizeof(double) * nx) : nullptr;
  double* dv = o->optimizer == MRBO_OPT_ADAM ? (double*)solve_slot(P, 11, sizeof(double) * nx) : nullptr;
  int32_t* dchk = (int32_t*)solve_slot(P, 12, sizeof(int32_t) * 2 * mrbo_plan::NCHK);
  if (!dx0 || !drn || !dxs || (dual_y_dx && !ddual) || !deto || !dact || !dvals || !dgx || !dgt || !dst || !dchk ||
      (o->optimizer == MRBO_OPT_ADAM && (!dm || !dv)))
    return fail(MRBO_ERR_NOMEM, "outer-ascent buffers");
  if (!P->hchk && hipHostMalloc(&P->hchk, sizeof(int32_t) * 2 * mrbo_plan::NCHK) != hipSuccess) {
    P->hchk = nullptr;
    return fail(MRBO_ERR_NOMEM, "pinned check ring");
  }
  for (auto& e : P->chk_ev)
    if (!e) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  if (host) {
    HIP_TRY(hipMemcpyAsync(dx0, x0s, sizeof(double) * nx, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync((void*)drn, rnstream, sizeof(double) * nrn, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync((void*)dxs, xstarts, sizeof(double) * nxs, hipMemcpyHostToDevice, st));
    if (dual_y_dx) HIP_TRY(hipMemcpyAsync((void*)ddual, dual_y_dx, sizeof(double) * ndual, hipMemcpyHostToDevice, st));
  }
  // every restart starts active (stochastic_solve's loop runs until its eswavs break); Adam's
  // moment estimates start at zero
  hipLaunchKernelGGL(fill_int_kernel, dim3((R + 63) / 64), dim3(64), 0, st, (int*)dact, R, 1);
  if (dm) {
    HIP_TRY(hipMemsetAsync(dm, 0, sizeof(double) * nx, st));
    HIP_TRY(hipMemsetAsync(dv, 0, sizeof(double) * nx, st));
  }
  // The iterations follow each other on the stream without a host round trip.  Behind them the
  // host reads iteration j's check (status bits, restarts still active) LAG iterations later: once
  // every restart has stopped, the launches already queued find x0 unchanged and reproduce the
  // same trajectories and ETO rows bit for bit, so stopping a few iterations late changes no output.
  constexpr int LAG = 2;
  int it = 0, stopped_at = 0, bits = 0;
  auto read_check = [&](int j) -> int {   // iteration j ≥ 1 (its slot not yet reused)
    const int k = (j - 1) % mrbo_plan::NCHK;
    if (hipEventSynchronize(P->chk_ev[k]) != hipSuccess) return -1;
    bits |= P->hchk[2 * k];
    if (P->hchk[2 * k + 1] == 0 && !stopped_at) stopped_at = j;
    return 0;
  };
  // A restart that eswavs has stopped keeps its x0, so its trajectories would reproduce the
  // outputs of its last launch bit for bit: the later launches skip them (kp.skip_active)
  struct SkipGuard {
    mrbo_plan_t* P;
    ~SkipGuard() { P->skip_active = nullptr; }
  } guard{P};
  P->skip_active = dact;
  // Without a caller's schedule (mrbo_plan_set_order), the launches after the first take their
  // trajectories longest first by the first launch's work counters (mrbo_plan_order_longest_first:
  // the launch's idle tail, C3 7.0 → 1.2 %); the plan's order is restored on return
  struct OrderGuard {
    mrbo_plan_t* P;
    const int32_t* saved;
    ~OrderGuard() { P->order = saved; }
  } oguard{P, P->order};
  const bool auto_order = P->order == nullptr && o->iterations > 1;
  int64_t* devals = auto_order ? (int64_t*)solve_slot(P, 13, sizeof(int64_t) * NCOUNT * T) : nullptr;
  if (auto_order && !devals) return fail(MRBO_ERR_NOMEM, "outer-ascent work counters");
  int rc = MRBO_OK;
  while (it < o->iterations && !stopped_at && !bits) {
    ++it;
    rc = mrbo_simulate_mc(P, dx0, drn, dxs, ddual, nullptr, dvals, dgx, dgt, dst, nullptr, nullptr,
                          (auto_order && it == 1) ? devals : nullptr, 0, st);
    if (rc != MRBO_OK) return rc;
    if (auto_order && it == 1) {
      rc = mrbo_plan_order_longest_first(P, devals, nullptr, st);
      if (rc != MRBO_OK) return rc;
    }
    rc = mrbo_eto_reduce(P, dvals, dgx, dgt, deto, 0, st);
    if (rc != MRBO_OK) return rc;
    if (o->optimizer == MRBO_OPT_SGA)
      rc = mrbo_sga_step(P, deto, dx0, dact, sample_size, o->eta, 0, st);
    else
      rc = mrbo_adam_step(P, deto, dx0, dact, dm, dv, it, sample_size, o->eta, o->beta1, o->beta2, o->eps, 0, st);
    if (rc != MRBO_OK) return rc;
    const int k = (it - 1) % mrbo_plan::NCHK;
    hipLaunchKernelGGL(solve_check_kernel, dim3(1), dim3(256), 0, st, (const int*)dst, (long long)T, (const int*)dact, R,
                       (int*)dchk + 2 * k);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(P->hchk + 2 * k, dchk + 2 * k, sizeof(int32_t) * 2, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipEventRecord(P->chk_ev[k], st));
    if (it > LAG && read_check(it - LAG)) return fail(MRBO_ERR_HIP, "hipEventSynchronize");
  }
  for (int j = std::max(1, it - LAG + 1); j <= it; ++j)   // the checks still in flight
    if (read_check(j)) return fail(MRBO_ERR_HIP, "hipEventSynchronize");
  if (host) {
    HIP_TRY(hipMemcpyAsync(x0s, dx0, sizeof(double) * nx, hipMemcpyDeviceToHost, st));
    if (eto) HIP_TRY(hipMemcpyAsync(eto, deto, sizeof(double) * R * W, hipMemcpyDeviceToHost, st));
    if (active) HIP_TRY(hipMemcpyAsync(active, dact, sizeof(int32_t) * R, hipMemcpyDeviceToHost, st));
  }
  HIP_TRY(hipStreamSynchronize(st));
  result[0] = it;                              // iterations launched
  result[1] = stopped_at ? stopped_at : it;    // the iteration after which no restart was active
  result[2] = bits;                            // OR of every launch's trajectory status bits
  return MRBO_OK;
}

int mrbo_eval_base(mrbo_plan_t* P, int32_t npts, const double* xs, double* out, uint32_t flags, void* stream) {
  if (!P || !xs || !out || npts < 1) return fail(MRBO_ERR_ARG, "bad arguments");
  hipStream_t st = (hipStream_t)stream;
  if (hipSetDevice(P->device) != hipSuccess) return fail(MRBO_ERR_HIP, "hipSetDevice");
  const int d = P->d;
  const size_t stride = 3 + 4 * d + d * d;
  KParams kp;
  fill_common(P, kp);
  kp.T = npts;
  Stage sg(P);
  const double* dxs = xs;
  double* dout = out;
  if (flags & MRBO_FLAG_HOST_POINTERS) {
    if (sg.in(xs, (size_t)d * npts, &dxs) || sg.out(stride * npts, out, &dout))
      return fail(MRBO_ERR_NOMEM, "staging allocation failed");
  }
  kp.pts = dxs;
  kp.pts_out = dout;
  HIP_TRY(hipMemsetAsync(P->dqueue, 0, sizeof(int) * MRBO_QUEUE_INTS, st));
  launch_evalb(d, P->RPL, P->fx, dim3(P->eblocks), dim3(P->ewpg * WAVE), P->esmem, st, kp);
  HIP_TRY(hipGetLastError());
  if (flags & MRBO_FLAG_HOST_POINTERS) {
    HIP_TRY(hipStreamSynchronize(st));
    HIP_TRY(hipMemcpy(out, dout, sizeof(double) * stride * npts, hipMemcpyDeviceToHost));
  }
  return MRBO_OK;
}

int mrbo_base_solve(mrbo_plan_t* P, int32_t n, const double* xstarts, double* xmin, double* fmin, int32_t* status,
                    int64_t* evals, uint32_t flags, void* stream) {
  if (!P || !xstarts || !xmin || !fmin || !status || n < 1) return fail(MRBO_ERR_ARG, "bad arguments");
  hipStream_t st = (hipStream_t)stream;
  if (hipSetDevice(P->device) != hipSuccess) return fail(MRBO_ERR_HIP, "hipSetDevice");
  const int d = P->d;
  KParams kp;
  fill_common(P, kp);
  // one launch item per start, on the base surrogate; no trajectory, no start tables (the
  // per-workgroup LDS layout shrinks to L0⁻¹ + the wave areas, within the plan's smem)
  kp.base_solve = 1;
  kp.nstarts = n;
  kp.M = n;
  kp.R = 1;
  kp.T = n;
  kp.with_gradient = 0;
  kp.xs_lds = 0;
  kp.batch = 0;
  Stage sg(P);
  const double* dxs = xstarts;
  double *dx = xmin, *df = fmin;
  int32_t* dst = status;
  int64_t* dev = evals;
  const bool host = flags & MRBO_FLAG_HOST_POINTERS;
  if (host) {
    if (sg.in(xstarts, (size_t)d * n, &dxs) || sg.out((size_t)d * n, xmin, &dx) || sg.out((size_t)n, fmin, &df) ||
        sg.out((size_t)n, status, &dst) || sg.out((size_t)NCOUNT * n, evals, &dev))
      return fail(MRBO_ERR_NOMEM, "staging allocation failed");
  }
  kp.xstarts = dxs;
  kp.policy = dx;
  kp.values = df;
  kp.status = (int*)dst;
  kp.evals = (long long*)dev;
  HIP_TRY(hipMemsetAsync(P->dqueue, 0, sizeof(int) * MRBO_QUEUE_INTS, st));
  const int blocks = std::min(P->blocks, (n + P->wpg - 1) / P->wpg);
  launch_rollout(d, P->RPL, P->fx, P->spec, dim3(blocks), dim3(P->wpg * WAVE), P->smem, st, kp);
  HIP_TRY(hipGetLastError());
  if (host) {
    HIP_TRY(hipStreamSynchronize(st));
    HIP_TRY(hipMemcpy(xmin, dx, sizeof(double) * d * n, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(fmin, df, sizeof(double) * n, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(status, dst, sizeof(int32_t) * n, hipMemcpyDeviceToHost));
    if (evals) HIP_TRY(hipMemcpy(evals, dev, sizeof(int64_t) * NCOUNT * n, hipMemcpyDeviceToHost));
  }
  return MRBO_OK;
}

int mrbo_gp_fit_theta(const mrbo_surrogate_t* s, int32_t np, int32_t nt, const double* thetas, double* ll,
                      double* grad, int32_t* status, double* L_out, double* c_out, uint32_t flags, void* stream) {
  if (!s || !thetas || !ll || !grad || !status || np < 1) return fail(MRBO_ERR_ARG, "null argument");
  const int d = s->d, N = s->N;
  if (d < 1 || N < 1 || !s->X || !s->y) return fail(MRBO_ERR_ARG, "bad surrogate (d=%d N=%d)", d, N);
  if (N > 512) return fail(MRBO_ERR_UNSUPPORTED, "N=%d > 512", N);
  if (s->kernel < 0 || s->kernel > 4) return fail(MRBO_ERR_UNSUPPORTED, "gp_fit: kernel id %d", s->kernel);
  // θ = (ℓ) for the one-parameter kernels; Periodic takes (ℓ) (period fixed at s->period) or (ℓ, p)
  if (nt < 1 || nt > (s->kernel == 4 ? 2 : 1)) return fail(MRBO_ERR_ARG, "gp_fit: nt=%d for kernel %d", nt, s->kernel);
  if (s->kernel == 4 && nt == 1 && !(s->period > 0.0)) return fail(MRBO_ERR_ARG, "gp_fit: period %g", s->period);
  hipStream_t st = (hipStream_t)stream;
  const size_t P = (size_t)np, NN = (size_t)N * N, NTP = (size_t)nt * P;
  const bool host = flags & MRBO_FLAG_HOST_POINTERS;
  Stage sg;
  // inputs [θ (host calls) | X | y] packed into one pinned buffer and one host→device copy; the
  // small outputs of host calls [ll | grad | status] in one device block and one copy back
  const size_t n_th = host ? NTP : 0, n_in = n_th + (size_t)d * N + N;
  const size_t out_bytes = sizeof(double) * (P + NTP) + sizeof(int32_t) * P;
  double* din = (double*)sg.slot(sizeof(double) * n_in);
  if (!din) return fail(MRBO_ERR_NOMEM, "staging the inputs");
  const double* dth = host ? din : thetas;
  const double* dX = din + n_th;
  const double* dy = dX + (size_t)d * N;
  double *dll_ = ll, *dgr = grad, *dL = L_out, *dc = c_out;
  int32_t* dst = status;
  if (host) {
    char* dout = (char*)sg.slot(out_bytes);
    if (!dout || sg.out(NN * P, L_out, &dL) || sg.out((size_t)N * P, c_out, &dc))
      return fail(MRBO_ERR_NOMEM, "staging allocation failed");
    dll_ = (double*)dout;
    dgr = dll_ + P;
    dst = (int32_t*)(dgr + NTP);
  }
  GpFitParams q{d, N, s->kernel, s->sigma_n2, dX, dy, nt, dth, s->period, dll_, dgr, (int*)dst, dL, dc, nullptr};
  {
    int dev = 0, lds_max = 0;
    HIP_TRY(hipGetDevice(&dev));
    HIP_TRY(hipDeviceGetAttribute(&lds_max, hipDeviceAttributeMaxSharedMemoryPerBlock, dev));
    const size_t need = gpfit_launch_lds(q);
    if (need > (size_t)lds_max)
      return fail(MRBO_ERR_UNSUPPORTED, "gp_fit: d=%d N=%d needs %zu B of LDS per workgroup, the device has %d", d, N,
                  need, lds_max);
  }
  if (!gpfit_in_regs(q) && !gpfit_in_lds(q)) {   // the register (N ≤ 64) and LDS (N ≤ 80) kernels need none
    q.work = (double*)sg.slot(sizeof(double) * gpfit_tile_work_doubles(N, nt) * P);
    if (!q.work) return fail(MRBO_ERR_NOMEM, "gp_fit workspace");
  }
  Pinned pin_in(sizeof(double) * n_in), pin_out(host ? out_bytes : 0);
  if (!pin_in.p || (host && !pin_out.p)) return fail(MRBO_ERR_NOMEM, "pinned staging");
  {
    double* h = (double*)pin_in.p;
    if (host) std::memcpy(h, thetas, sizeof(double) * NTP);
    std::memcpy(h + n_th, s->X, sizeof(double) * d * N);
    std::memcpy(h + n_th + (size_t)d * N, s->y, sizeof(double) * N);
  }
  // timing events per device (an event records only on streams of the device it was created on)
  static std::mutex gev_m;
  static std::vector<std::pair<hipEvent_t, hipEvent_t>> gevs;
  hipEvent_t gev[2];
  {
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lk(gev_m);
    if ((int)gevs.size() <= dev) gevs.resize(dev + 1, {nullptr, nullptr});
    if (!gevs[dev].first) {
      hipEvent_t a = nullptr, b = nullptr;
      if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) {
        if (a) (void)hipEventDestroy(a);
        return fail(MRBO_ERR_HIP, "gp_fit: hipEventCreate");
      }
      gevs[dev] = {a, b};
    }
    gev[0] = gevs[dev].first;
    gev[1] = gevs[dev].second;
  }
  // from here on every return path synchronises the stream first (the copy reads pin_in)
  {
    const hipError_t e = hipMemcpyAsync(din, pin_in.p, sizeof(double) * n_in, hipMemcpyHostToDevice, st);
    if (e != hipSuccess) {
      if (hipStreamSynchronize(st) != hipSuccess) { sg.abandon(); pin_in.abandon(); }
      return fail(MRBO_ERR_HIP, "gp_fit: staging copy: %s", hipGetErrorString(e));
    }
  }
  if (const hipError_t e = hipEventRecord(gev[0], st); e != hipSuccess) {
    if (hipStreamSynchronize(st) != hipSuccess) { sg.abandon(); pin_in.abandon(); }
    return fail(MRBO_ERR_HIP, "gp_fit: hipEventRecord: %s", hipGetErrorString(e));
  }
  launch_gpfit(np, st, q);
  // the staging buffers and the workspace go back to the pool on return: once the launch is
  // issued, every path synchronises the stream first (an error after the launch must not hand
  // memory a running kernel still uses to another call), and keeps them out of the pool when
  // even that fails
  {
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipEventRecord(gev[1], st);
    // the small outputs of a host call come back on the same stream (into pinned memory), so
    // one synchronisation covers the kernel and the copy
    if (e == hipSuccess && host) e = hipMemcpyAsync(pin_out.p, dll_, out_bytes, hipMemcpyDeviceToHost, st);
    const hipError_t es = hipStreamSynchronize(st);
    if (es != hipSuccess) {
      sg.abandon();
      pin_in.abandon();
      pin_out.abandon();
      return fail(MRBO_ERR_HIP, "gp_fit: hipStreamSynchronize: %s", hipGetErrorString(es));
    }
    if (e != hipSuccess) return fail(MRBO_ERR_HIP, "gp_fit launch: %s", hipGetErrorString(e));
  }
  {
    float ms = -1.f;
    if (hipEventElapsedTime(&ms, gev[0], gev[1]) == hipSuccess) g_gpfit_ms = ms;
  }
  if (host) {
    const double* h = (const double*)pin_out.p;
    std::memcpy(ll, h, sizeof(double) * P);
    std::memcpy(grad, h + P, sizeof(double) * NTP);
    std::memcpy(status, h + P + NTP, sizeof(int32_t) * P);
    if (L_out) HIP_TRY(hipMemcpy(L_out, dL, sizeof(double) * NN * P, hipMemcpyDeviceToHost));
    if (c_out) HIP_TRY(hipMemcpy(c_out, dc, sizeof(double) * N * P, hipMemcpyDeviceToHost));
  }
  return MRBO_OK;
}

int mrbo_gp_fit(const mrbo_surrogate_t* s, int32_t np, const double* ells, double* ll, double* dll, int32_t* status,
                double* L_out, double* c_out, uint32_t flags, void* stream) {
  return mrbo_gp_fit_theta(s, np, 1, ells, ll, dll, status, L_out, c_out, flags, stream);
}

double mrbo_last_gp_fit_ms(void) { return g_gpfit_ms; }

int mrbo_plan_set_order(mrbo_plan_t* P, const int32_t* order, int64_t n) {
  if (!P) return fail(MRBO_ERR_ARG, "null plan");
  if (order && n != (int64_t)P->p.M * P->p.R) return fail(MRBO_ERR_ARG, "order length != M*R");
  P->order = order;
  return MRBO_OK;
}

int mrbo_plan_order_longest_first(mrbo_plan_t* P, const int64_t* evals, int32_t* order_out, void* stream) {
  if (!P || !evals) return fail(MRBO_ERR_ARG, "null argument");
  if (hipSetDevice(P->device) != hipSuccess) return fail(MRBO_ERR_HIP, "hipSetDevice");
  const long long T = (long long)P->p.M * P->p.R;
  if (T > 0x7FFFFFFFll) return fail(MRBO_ERR_ARG, "M*R = %lld: more than 2^31 - 1 trajectories", T);
  const size_t need = mrbo::order_buffer_bytes((int)T);
  if (P->oorder_bytes < need) {
    if (P->oorder) HIP_TRY(hipFree(P->oorder));
    P->oorder = nullptr;
    P->oorder_bytes = 0;
    HIP_TRY(hipMalloc(&P->oorder, need));
    P->oorder_bytes = need;
  }
  int* order = nullptr;
  HIP_TRY(mrbo::order_longest_first((const long long*)evals, (int)T, P->oorder, P->oorder_bytes, &order,
                                    (hipStream_t)stream));
  P->order = order;
  if (order_out)
    HIP_TRY(hipMemcpyAsync(order_out, order, sizeof(int32_t) * T, hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return MRBO_OK;
}

int mrbo_plan_info(const mrbo_plan_t* P, int32_t* info, int32_t n) {
  if (!P || !info || n < 0) return fail(MRBO_ERR_ARG, "bad arguments");
  const int32_t v[7] = {P->RPL, P->blocks, P->wpg, P->batch, P->spec, (int32_t)P->smem, P->fx ? 4 : 6};
  for (int i = 0; i < n && i < 7; ++i) info[i] = v[i];
  return MRBO_OK;
}

static double launch_ms(mrbo_plan_t* P, long long launch) {
  const int slot = (int)(launch % mrbo_plan::NEV);
  float ms = -1.f;
  if (!P->ev[2 * slot] || !P->ev[2 * slot + 1]) return -1.0;
  if (hipEventSynchronize(P->ev[2 * slot + 1]) != hipSuccess) return -1.0;
  if (hipEventElapsedTime(&ms, P->ev[2 * slot], P->ev[2 * slot + 1]) != hipSuccess) return -1.0;
  return ms;
}

double mrbo_last_kernel_ms(mrbo_plan_t* P) {
  if (!P || P->nlaunch == 0) return -1.0;
  return launch_ms(P, P->nlaunch - 1);
}

int mrbo_kernel_times(mrbo_plan_t* P, int32_t n, double* ms) {
  if (!P || !ms || n < 0) return fail(MRBO_ERR_ARG, "bad arguments");
  const long long k = std::min<long long>({(long long)n, P->nlaunch, (long long)mrbo_plan::NEV});
  for (long long i = 0; i < k; ++i) {
    ms[i] = launch_ms(P, P->nlaunch - k + i);
    if (ms[i] < 0) return fail(MRBO_ERR_HIP, "hipEventElapsedTime");
  }
  return (int)k;
}

// utils.jl:4-74 -- Sobol uniforms → Box–Muller with log10 (Q1) → column-major reshape (Q2)
int mrbo_rnstream(int32_t M, int32_t d, int32_t H, double* out) {
  if (M < 1 || d < 1 || H < 1 || !out) return fail(MRBO_ERR_ARG, "bad arguments");
  const int off = ((d + 1) % 2 == 1) ? 1 : 0, Dp = d + 1 + off;
  if (Dp > MRBO_SOBOL_TABLE_MAXDIM) return fail(MRBO_ERR_UNSUPPORTED, "dimension");
  Sobol sob(Dp);
  const long long cols = (long long)M * H;
  std::vector<double> u(Dp), y(Dp);
  const double twopi = 2.0 * 3.141592653589793;
  for (long long j = 0; j < cols; ++j) {
    sob.next(u.data());
    for (int i = 0; i < Dp; ++i)
      y[i] = (i % 2 == 0) ? std::sqrt(-2.0 * std::log10(u[i])) * std::cos(twopi * u[i + 1])
                          : std::sqrt(-2.0 * std::log10(u[i - 1])) * std::sin(twopi * u[i]);
    for (int i = 0; i < Dp; ++i) {
      const long long l = j * Dp + i;             // linear index in the Dp × (M·H) matrix
      const long long m = l % M, rest = l / M;    // reshape to M × Dp × H
      const long long k = rest % Dp, t = rest / Dp;
      if (k < d + 1) out[m + (long long)M * k + (long long)M * (d + 1) * t] = y[i];
    }
  }
  return MRBO_OK;
}

int mrbo_initial_guesses(int32_t n, int32_t d, const double* lbs, const double* ubs, double* out) {
  if (n < 0 || d < 1 || d > MRBO_SOBOL_TABLE_MAXDIM || !lbs || !ubs || !out) return fail(MRBO_ERR_ARG, "bad arguments");
  Sobol sob(d);
  std::vector<double> u(d);
  for (int j = 0; j < n; ++j) {
    sob.next(u.data());
    for (int a = 0; a < d; ++a) out[(size_t)j * d + a] = lbs[a] + (ubs[a] - lbs[a]) * u[a];
  }
  for (int a = 0; a < d; ++a) out[(size_t)n * d + a] = lbs[a] + 1e-6;
  for (int a = 0; a < d; ++a) out[(size_t)(n + 1) * d + a] = ubs[a] - 1e-6;
  return MRBO_OK;
}

double mrbo_dual_uniform(uint64_t seed, int64_t traj, int32_t j, int32_t k) { return dual_uniform(seed, traj, j, k); }

}  // extern "C"
