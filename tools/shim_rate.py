#!/usr/bin/env python3
"""Rate of the Julia drop-in's call sequences at a BASELINE configuration (default C3), through
mrbo.shim (the Python mirror of julia/MRBO.jl's C-ABI calls, host pointers):
  per_call_plan  R = 1, a new plan per call and destroyed after it (the round-4 shim)
  cached_r1      R = 1 on the cached plan (MRBO.jl simulate_trajectory_mc(T, tp, ::MrboBackend))
  batched        the R restarts of the config in ONE launch (MRBO.jl's batched method)
  stochastic_solve_r1_loop / _device   the reference's outer loop over the R restarts: through the
                 R = 1 method, and as ONE mrbo_stochastic_solve call (MRBO.jl's device-resident method)
Each row: trajectories per second over whole calls (host staging, launch, copies back, host
ETO), and the per-call time.  Not the bench metric (bench.py's value is the device-resident rate).

usage: python tools/shim_rate.py [--config C3] [--calls 8]
One JSON line on stdout.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "rollout-bayesian-optimization_amd"), ROOT]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--calls", type=int, default=8)
    a = ap.parse_args()
    import torch
    from mrbo import configs, shim
    cfg = configs.CONFIGS[a.config]
    pb = configs.problem(a.config)
    M, R, d = cfg.M, cfg.R, cfg.d
    T, tp, xs = pb.T, pb.tp, pb.es.get_starts()
    res, g, t = np.zeros(M), np.zeros((d, M), order="F"), np.zeros((1, M), order="F")

    def r1_call(k):
        tp.set_starting_point(pb.x0s[:, k % R].copy())
        shim.simulate_trajectory_mc(T, tp, xs, res, g, t)

    def fresh_call(k):
        r1_call(k)
        shim.release_plans()

    def batch_call(k):
        shim.simulate_trajectory_mc_batch(T, tp, pb.x0s, xs)

    def timed(fn, n):
        fn(0)                       # warm-up (and the cached plan)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(n):
            fn(k + 1)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n

    # the C-ABI call alone (host pointers, staging included, no host reductions), batched shape
    import ctypes
    from mrbo import _lib
    plan_b = shim.cached_plan(T.s, tp, T.θ[0], xs.shape[1], R=R)
    X0 = np.asfortranarray(pb.x0s, dtype=np.float64)
    rn = np.asfortranarray(tp.rnstream_sequence, dtype=np.float64)
    vals, st = np.zeros((M, R), order="F"), np.zeros((M, R), dtype=np.int32, order="F")
    gxb, gtb = np.zeros((d, M, R), order="F"), np.zeros((1, M, R), order="F")

    def c_call(k):
        shim._launch(plan_b, X0, rn, np.asfortranarray(xs), vals, gxb, gtb, st)

    rows = {"batched_c_call_only": None}
    s_c = timed(c_call, max(2, a.calls // 4))
    rows["batched_c_call_only"] = {"trajectories_per_call": M * R, "ms_per_call": s_c * 1e3,
                                   "trajectories_per_s": M * R / s_c}
    shim.release_plans()
    for name, fn, per in (("per_call_plan", fresh_call, M), ("cached_r1", r1_call, M), ("batched", batch_call, M * R)):
        n = a.calls if name != "batched" else max(2, a.calls // 4)
        s = timed(fn, n)
        rows[name] = {"trajectories_per_call": per, "ms_per_call": s * 1e3, "trajectories_per_s": per / s}
        shim.release_plans()
    # the reference's outer loop (stochastic_solve, utils.jl:235-265) over the R restarts: through the
    # R = 1 method (MRBO.jl simulate_trajectory_mc, one call per restart and iteration), and as ONE
    # mrbo_stochastic_solve call (MRBO.jl's device-resident method).  Both do the same rollout work:
    # the R = 1 loop's calls are the useful trajectories, the rate of either row counts those alone.
    steps = []
    t0 = time.perf_counter()
    for r in range(R):
        trace = []
        shim.stochastic_solve(T, tp, xs, pb.x0s[:, r], eta=0.01, trace=trace)
        steps.append(len(trace))
    s_loop = time.perf_counter() - t0
    useful = int(sum(steps)) * M
    rows["stochastic_solve_r1_loop"] = {"calls": int(sum(steps)), "s_per_ascent": s_loop,
                                        "trajectories": useful, "trajectories_per_s": useful / s_loop}
    shim.release_plans()
    shim.stochastic_solve_batch(T, tp, xs, pb.x0s, eta=0.01)          # warm-up (the cached plan)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    X, _, _, res = shim.stochastic_solve_batch(T, tp, xs, pb.x0s, eta=0.01)
    s_dev = time.perf_counter() - t0
    rows["stochastic_solve_device"] = {"iterations_launched": res[0], "all_stopped_after": res[1],
                                       "trajectories_launched": res[0] * M * R, "s_per_ascent": s_dev,
                                       "useful_trajectories": useful, "trajectories_per_s": useful / s_dev,
                                       "launched_trajectories_per_s": res[0] * M * R / s_dev,
                                       "steps_per_restart": steps}
    shim.release_plans()
    print(json.dumps({"config": a.config, "M": M, "R": R, "rows": rows,
                      "note": "whole calls through the C ABI with host pointers (mrbo.shim = MRBO.jl's sequence)"}),
          flush=True)


if __name__ == "__main__":
    main()
