#!/usr/bin/env python3
"""Trajectory schedule A/B on one plan (mrbo_plan_set_order): the C3 launch with the trajectories
handed to the persistent waves in index order (m + M·r, MC sample fastest), interleaved by restart
(r fastest), longest first by the previous launch's work counters, and in a random order.
Kernel time per launch by HIP events, several rounds alternating the orders.

usage: python tools/order_ab.py [--config C3] [--launches 5] [--rounds 2]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "rollout-bayesian-optimization_amd"), ROOT]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--launches", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=2)
    a = ap.parse_args()
    import torch
    from mrbo import configs
    from mrbo.engine import to_device
    from mrbo.rollout import _plan_for
    cfg = configs.CONFIGS[a.config]
    pb = configs.problem(a.config)
    M, R = cfg.M, cfg.R
    plan = _plan_for(pb.T.s, cfg.h, M, R, pb.es.get_starts().shape[1], pb.lbs, pb.ubs, pb.T.θ[0], 0,
                     dict(sample_offset=0, samples_total=M, **pb.plan_opts()))
    dev = "cuda:0"
    dx0 = to_device(np.asfortranarray(pb.x0s), dev)
    drn = to_device(np.asfortranarray(pb.tp.rnstream_sequence[:M]), dev)
    dxs = to_device(pb.es.get_starts(), dev)
    out = plan.alloc_outputs(with_gradient=True)
    plan.simulate(dx0, drn, dxs, out)
    torch.cuda.synchronize()
    ref_vals = out["values"].clone()
    idx = torch.arange(M * R, dtype=torch.int64, device=dev)
    orders = {
        "index": None,
        "interleave": ((idx % R) * M + idx // R).to(torch.int32),
        "random": torch.randperm(M * R, device=dev).to(torch.int32),
    }
    ev = out["evals"].view(-1, 5).to(torch.float64)
    w = torch.tensor(plan.ORDER_WEIGHTS, dtype=torch.float64, device=dev)
    orders["longest_first"] = torch.argsort(ev @ w, descending=True).to(torch.int32)
    times = {k: [] for k in orders}
    for _ in range(a.rounds):
        for name, order in orders.items():
            plan.set_order(order)
            for _ in range(a.launches):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                plan.simulate(dx0, drn, dxs, out)
                e1.record()
                torch.cuda.synchronize()
                times[name].append(e0.elapsed_time(e1))
            assert torch.equal(out["values"], ref_vals), name     # same results in any order
    plan.set_order(None)
    res = {k: {"median_ms": float(np.median(v)), "min_ms": float(np.min(v)), "n": len(v)} for k, v in times.items()}
    print(json.dumps({"config": a.config, "trajectories": M * R, "orders": res}), flush=True)


if __name__ == "__main__":
    main()
