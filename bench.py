#!/usr/bin/env python3
"""bench.py -- rollout trajectories/s on BASELINE.json's headline configuration.

One *step* = one outer stochastic-gradient-ascent iteration of the rollout acquisition
(utils.jl:235-265): simulate_trajectory_mc for R restarts × M MC samples (forward rollout +
adjoint gradient, rollout.jl:279-340) on the device, per-restart partial sums, one all-reduce
across ranks, ETO + eswavs + SGA update of the R start points.

Workload C3 (headline): Hartmann6 d=6, horizon h=3, N=64 base observations, M=1024 MC
samples × R=64 restarts per GPU, 18 inner starts, fp64.  With --gpus N the per-GPU work is
fixed (weak scaling): rank k runs samples [kM, (k+1)M) of one N·M-sample rnstream.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
       (N>1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...)
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "rollout-bayesian-optimization_amd"), ROOT]

import numpy as np  # noqa: E402

FP64_PEAK_TFLOPS = 78.6  # MI355X dense fp64 (vector = matrix), spec
METRIC = "rollout trajectories/sec (MC samples × restarts) at horizon h=3, n=64 GP"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="C3")
    ap.add_argument("--mc-per-gpu", type=int, default=0,
                    help="MC samples per GPU (default: the config's M; the metric config is C3 at M=1024)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--longest-first", action="store_true",
                    help="hand trajectories to the waves longest first by the previous step's work "
                         "counters (default: index order; measured 1 %% slower at C3, DESIGN.md §9)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--eta", type=float, default=0.5, help="StandardSGA step (optimizers.jl:6-23)")
    return ap.parse_args()


def cpu_baseline(pb, M_full, R_full, budget_s):
    """The oracle (C restatement, 'port') on the same workload, bounded sample, host cores."""
    from oracle import oracle as O
    nthreads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    s = pb.surrogate
    n = s.observed
    osur = O.OracleSurrogate(s.X[:, :n], s.L[:n, :n], s.c[:n], s.y[:n], fmini=s.fmini())
    rn = pb.tp.rnstream_sequence[:M_full]
    xs = pb.es.get_starts()

    def run(Ms, Rs):
        t = time.perf_counter()
        O.simulate_mc(osur, pb.x0s[:, :Rs], np.asfortranarray(rn[:Ms]), xs, pb.lbs, pb.ubs, pb.cfg.h,
                      nthreads=nthreads, want_policy=False)
        return time.perf_counter() - t

    def run1(Ms):   # the reference itself is single-process, single-thread
        t = time.perf_counter()
        O.simulate_mc(osur, pb.x0s[:, :1], np.asfortranarray(rn[:Ms]), xs, pb.lbs, pb.ubs, pb.cfg.h,
                      nthreads=1, want_policy=False)
        return time.perf_counter() - t

    Ms, Rs = min(M_full, max(nthreads * 4, 32)), 1
    dt = run(Ms, Rs)
    rate = Ms * Rs / dt
    # scale the sample to ~budget_s seconds of CPU work (never beyond the full workload)
    target = int(rate * budget_s)
    Rs = max(1, min(R_full, target // M_full)) if target >= M_full else 1
    Ms = M_full if target >= M_full else max(Ms, min(M_full, target))
    dt = run(Ms, Rs)
    M1 = min(M_full, 64)
    dt1 = run1(M1)
    M1 = min(M_full, max(M1, int(M1 / dt1 * budget_s * 0.3)))
    dt1 = run1(M1)
    return dict(value=Ms * Rs / dt, unit="trajectories/s", cores=nthreads, kind="port",
                sample=f"{pb.cfg.name} workload, first {Rs} restart(s) x {Ms} MC samples "
                       f"({Ms * Rs} trajectories, {dt:.1f} s), oracle/rbo_oracle.c OpenMP x{nthreads}",
                single_thread={"value": M1 / dt1, "cores": 1,
                               "sample": f"first restart x {M1} MC samples ({dt1:.1f} s), 1 thread"})


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    from mrbo import configs, flops, parallel
    from mrbo.engine import to_device
    from mrbo.rollout import _plan_for
    from mrbo.utils import sga_step_batch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one process per GPU; MRBO_DIST_BACKEND=gloo + device wrap-around only for rehearsing the
    # multi-rank path on a box with fewer GPUs than ranks
    ndev = torch.cuda.device_count()
    local = local % max(ndev, 1)
    torch.cuda.set_device(local)
    backend = os.environ.get("MRBO_DIST_BACKEND", "nccl")
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        else:
            dist.init_process_group(backend)
    cfg = configs.CONFIGS[args.config]
    M_local, R, d, h = (args.mc_per_gpu or cfg.M), cfg.R, cfg.d, cfg.h
    M_total = M_local * world
    lo, hi = parallel.shard(M_total, world, rank)
    pb = configs.problem(args.config, M=M_total)
    T = pb.T
    plan = _plan_for(T.s, h, hi - lo, R, pb.es.get_starts().shape[1], pb.lbs, pb.ubs, T.θ[0], local,
                     dict(sample_offset=lo, samples_total=M_total))
    dev = f"cuda:{local}"
    drn = to_device(np.asfortranarray(pb.tp.rnstream_sequence[lo:hi]), dev)   # resident in HBM
    dxs = to_device(pb.es.get_starts(), dev)
    x0 = np.array(pb.x0s, dtype=np.float64)
    dx0 = to_device(x0, dev)
    out = plan.alloc_outputs(with_gradient=True)
    evals_acc = torch.zeros_like(out["evals"])
    active = np.ones(R, dtype=bool)
    W = 2 + 2 * d + 2
    kernel_ms = []

    def step(timed):
        dx0.copy_(torch.from_numpy(x0.ravel(order="F")), non_blocking=False)
        plan.simulate(dx0, drn, dxs, out)
        sums = plan.partial_sums(out, hi - lo)
        evals_acc.add_(out["evals"])        # also in warmup: no first-use op inside the timed region
        if args.longest_first:
            plan.order_longest_first(out)   # the next step's schedule (same work)
        parallel.allreduce_sums(sums)
        s = sums.cpu().numpy().reshape((W, R), order="F")
        eto = parallel.eto_from_sums(s, M_total, d)
        # eswavs + StandardSGA of every active restart at once (utils.jl:114-123, optimizers.jl:6-23)
        sga_step_batch(x0, active, eto[2:2 + d], eto[2 + d:2 + 2 * d], M_total, args.eta, pb.lbs, pb.ubs)
        if timed:
            kernel_ms.append(plan.last_kernel_ms())

    for _ in range(args.warmup):
        step(False)
    evals_acc.zero_()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    el = torch.tensor([elapsed], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())

    st = out["status"].cpu().numpy()
    ev = evals_acc.cpu().numpy().reshape((flops.NCOUNTERS, hi - lo, R), order="F") / max(args.steps, 1)
    info = plan.info()
    fl = flops.launch_flops(ev, cfg.N, d, h, info=info, nstarts=pb.es.get_starts().shape[1])
    kms = float(np.mean(kernel_ms)) if kernel_ms else float("nan")
    achieved = fl / (kms * 1e-3) / 1e12
    traffic = None
    tpath = os.path.join(ROOT, "profiles", f"traffic_{cfg.name}.json")
    if os.path.exists(tpath):
        with open(tpath) as f:
            traffic = json.load(f).get("bytes_per_launch")
    total = world * (hi - lo) * R * args.steps
    res = {
        "metric": METRIC,
        "value": total / elapsed,
        "unit": "trajectories/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (Kronecker base design on the test function, Sobol/Box-Muller(log10) rnstream)",
        "config": {"workload": f"{cfg.name}: {cfg.testfn} d={d} h={h} N={cfg.N} M={M_local}/GPU x R={R} restarts, "
                               f"18 inner starts, forward rollout + adjoint gradient per trajectory",
                   "trajectories_per_step": world * (hi - lo) * R, "M_per_gpu": hi - lo, "R": R, "h": h,
                   "N": cfg.N, "d": d, "parallelism": f"mc-shard x{world}",
                   "schedule": "longest first (previous step's work counters)" if args.longest_first else "index order"},
        "roofline": {"bound": "mfma", "achieved": achieved, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": achieved / FP64_PEAK_TFLOPS, "traffic": traffic,
                     "kernel": f"rollout_kernel<{d},{info['rpl']},{info['spec']}>", "kernel_ms": kms, "flops_per_launch": fl,
                     "launch": info,
                     "note": "compute-bound fp64: peak = the dense fp64 matrix peak, equal to the fp64 vector "
                             "peak on MI355X; the kernel issues VALU v_fma_f64 (matrix-vector work, not "
                             "GEMM-shaped); algorithmic FLOP model in DESIGN.md §5; HBM algorithmic "
                             "bytes/traj ~0.3 KB so an HBM roofline does not bind; traffic = PMC bytes per "
                             "launch from profiles/traffic_<config>.json"},
        "status_errors": int((st != 0).sum()),
        "work_per_traj": {"grad_evals": float(ev[0].mean()), "value_evals": float(ev[1].mean()),
                          "hessians": float(ev[2].mean()), "rich_evals": float(ev[3].mean()),
                          "pairs": float(ev[4].mean())},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline(pb, M_local, R, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(res))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
