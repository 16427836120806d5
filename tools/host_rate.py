#!/usr/bin/env python3
"""PCIe-inclusive rate of the C-ABI boundary: mrbo_simulate_mc with MRBO_FLAG_HOST_POINTERS (the
Julia shim's path: host arrays in, host arrays out, staged through device memory by the library)
beside the device-pointer launch on the same plan.  Not the bench metric (bench.py's value has
the inputs resident in HBM); DESIGN.md §8 quotes both.

usage: python tools/host_rate.py [--config C3] [--steps 5] [--warmup 2]
One JSON line on stdout.
"""
import argparse
import ctypes
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
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    a = ap.parse_args()
    import torch
    from mrbo import _lib, configs
    from mrbo.engine import to_device
    from mrbo.rollout import _plan_for
    cfg = configs.CONFIGS[a.config]
    pb = configs.problem(a.config)
    M, R, d = cfg.M, cfg.R, cfg.d
    T = pb.T
    plan = _plan_for(T.s, cfg.h, M, R, pb.es.get_starts().shape[1], pb.lbs, pb.ubs, T.θ[0], 0,
                     dict(sample_offset=0, samples_total=M, **pb.plan_opts()))
    # host arrays (column-major, as the Julia caller holds them)
    x0 = np.asfortranarray(pb.x0s, dtype=np.float64)
    rn = np.asfortranarray(pb.tp.rnstream_sequence[:M], dtype=np.float64)
    xs = np.asfortranarray(pb.es.get_starts(), dtype=np.float64)
    vals = np.zeros((M, R), order="F")
    gx = np.zeros((d, M, R), order="F")
    gt = np.zeros((1, M, R), order="F")
    st = np.zeros((M, R), dtype=np.int32, order="F")
    pv = lambda arr: ctypes.c_void_p(arr.ctypes.data)

    def host_call():
        _lib.check(plan.lib.mrbo_simulate_mc(plan.handle, pv(x0), pv(rn), pv(xs), None, None, pv(vals), pv(gx),
                                             pv(gt), pv(st), None, None, None, _lib.MRBO_FLAG_HOST_POINTERS, None))

    # device-pointer launch on the same plan (inputs resident in HBM)
    dev = "cuda:0"
    dx0, drn, dxs = to_device(x0, dev), to_device(rn, dev), to_device(xs, dev)
    out = plan.alloc_outputs(with_gradient=True)

    def dev_call():
        plan.simulate(dx0, drn, dxs, out)

    def timed(fn):
        for _ in range(a.warmup):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / a.steps

    t_dev = timed(dev_call)
    t_host = timed(host_call)
    np.testing.assert_array_equal(vals, out["values"].cpu().numpy().reshape((M, R), order="F"))
    in_b = x0.nbytes + rn.nbytes + xs.nbytes
    out_b = vals.nbytes + gx.nbytes + gt.nbytes + st.nbytes
    print(json.dumps({"config": a.config, "trajectories_per_launch": M * R,
                      "device_pointers": {"ms_per_launch": t_dev * 1e3, "trajectories_per_s": M * R / t_dev},
                      "host_pointers": {"ms_per_launch": t_host * 1e3, "trajectories_per_s": M * R / t_host},
                      "staged_bytes": {"host_to_device": in_b, "device_to_host": out_b},
                      "pcie_overhead": t_host / t_dev - 1.0, "values_equal": True}), flush=True)


if __name__ == "__main__":
    main()
