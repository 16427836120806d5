// mrbo_order.hip -- the longest-first trajectory schedule on the device
// (mrbo_plan_order_longest_first, mrbo_stochastic_solve).
//
// The rollout kernel's persistent waves drain one work queue per XCD over a contiguous eighth of
// the queue positions, then the other chunks in turn (mrbo_rollout.hip rollout_kernel).  In index
// order the launch ends with whatever trajectories happen to sit last in each chunk; C3's heavy-tailed
// Newton work (a few trajectories run ~3× the mean) then leaves 7 % of the grid idle at the end.
// Consecutive SGA steps move x0 a little and reuse the MC streams, so a trajectory's work repeats
// closely: each chunk's OWN trajectories (index range [x·T/8, (x+1)·T/8)) are re-ordered longest
// first by the previous launch's work counters.  A chunk keeps its index range, so each XCD still
// writes the output rows of one contiguous range (whole cache lines in one L2); an XCD that drains
// its chunk early takes the short ends of the others.  Scheduling only: every output is
// bit-identical under any order (tests/test_gpu_schedule.py).  The Python mirror is
// RolloutPlan.longest_first_order.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "mrbo_device.h"

namespace mrbo {

namespace {

// 2 × the work counters weighted in value-evaluation units (grad 2.5, value 1, Hessian 3, adjoint
// rich evaluation 5, adjoint pair 3: RolloutPlan.ORDER_WEIGHTS) -- integers, so the key is exact
constexpr unsigned KW[NCOUNT] = {5u, 2u, 6u, 10u, 6u};

constexpr int Q = MRBO_QUEUE_INTS / 16;   // queue heads: one per XCD
constexpr unsigned WBITS = 29;             // work key bits below the 3 chunk bits

__global__ void order_keys_kernel(const long long* __restrict__ evals, int T, unsigned* __restrict__ key,
                                  int* __restrict__ idx) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= T) return;
  unsigned long long k = 0;
#pragma unroll
  for (int c = 0; c < NCOUNT; ++c) {
    const long long e = evals[(long long)NCOUNT * t + c];
    k += (unsigned long long)(e > 0 ? e : 0) * KW[c];
  }
  int x = 0;   // the per-XCD queue chunk that holds t in index order: x·T/8 ≤ t < (x+1)·T/8
  while (x + 1 < Q && (long long)(x + 1) * T / Q <= t) ++x;
  const unsigned long long wmax = (1ull << WBITS) - 1;
  // descending order of (Q − 1 − x, work): chunk 0 first, each chunk longest first
  key[t] = ((unsigned)(Q - 1 - x) << WBITS) | (unsigned)(k > wmax ? wmax : k);
  idx[t] = t;
}

size_t sort_tmp_bytes(int T) {
  size_t b = 0;
  (void)hipcub::DeviceRadixSort::SortPairsDescending(nullptr, b, (const unsigned*)nullptr, (unsigned*)nullptr,
                                                     (const int*)nullptr, (int*)nullptr, T, 0, 32);
  return b;
}

size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }

}  // namespace

// device bytes order_longest_first needs for T trajectories (the order itself included)
size_t order_buffer_bytes(int T) {
  return 4 * align256(sizeof(int) * (size_t)T) + align256(sort_tmp_bytes(T));
}

// the schedule from one launch's work counters (evals[NCOUNT·t + k], mrbo_simulate_mc's layout)
// into buf (order_buffer_bytes(T)); *order points into buf.  Stream-ordered, no host round trip.
hipError_t order_longest_first(const long long* evals, int T, void* buf, size_t bytes, int** order, hipStream_t st) {
  if (T <= 0 || bytes < order_buffer_bytes(T)) return hipErrorInvalidValue;
  char* p = (char*)buf;
  const size_t a = align256(sizeof(int) * (size_t)T);
  unsigned* key = (unsigned*)p;
  unsigned* key_sorted = (unsigned*)(p + a);
  int* idx = (int*)(p + 2 * a);
  int* out = (int*)(p + 3 * a);
  void* tmp = p + 4 * a;
  size_t tb = sort_tmp_bytes(T);
  const int tpb = 256, nb = (T + tpb - 1) / tpb;
  hipLaunchKernelGGL(order_keys_kernel, dim3(nb), dim3(tpb), 0, st, evals, T, key, idx);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  // stable: equal keys keep index order; position r of the result is queue position r, and the
  // chunk-major key keeps every trajectory inside its own chunk's positions
  e = hipcub::DeviceRadixSort::SortPairsDescending(tmp, tb, key, key_sorted, idx, out, T, 0, 32, st);
  if (e != hipSuccess) return e;
  *order = out;
  return hipSuccess;
}

}  // namespace mrbo
