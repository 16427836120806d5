#!/usr/bin/env python3
"""bench.py -- rollout trajectories/s on BASELINE.json's headline configuration.

One *step* = one outer stochastic-gradient-ascent iteration of the rollout acquisition
(utils.jl:235-265): simulate_trajectory_mc for R restarts × M MC samples (forward rollout +
adjoint gradient, rollout.jl:279-340) on the device, the per-restart ETO (mean / std n−1,
rollout.jl:328-339), eswavs and StandardSGA.update! of the R start points (utils.jl:114-123,
optimizers.jl:16-22; η = 0.01, the reference default, no box clip).

Workload C3 (headline): Hartmann6 d=6, horizon h=3, N=64 base observations, M=1024 MC
samples × R=64 restarts per GPU, 18 inner starts, fp64.  With --gpus N the per-GPU work is
fixed (weak scaling): rank k runs samples [kM, (k+1)M) of one N·M-sample rnstream and the
ranks exchange their per-restart moments once per step (one all-gather, Chan merge,
mrbo/parallel.py).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config C3] [--ell L | --mle]
  N > 1 without WORLD_SIZE in the environment: this process starts N ranks itself
  (python -m torch.distributed.run --nproc-per-node N ...) before touching the GPU, and exits
  with their status; under torchrun (WORLD_SIZE set) each rank runs one GPU.
"""
import argparse
import json
import os
import shutil
import socket
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "rollout-bayesian-optimization_amd"), ROOT]

import numpy as np  # noqa: E402

FP64_PEAK_TFLOPS = 78.6  # MI355X dense fp64 (vector = matrix), spec
METRIC = "rollout trajectories/sec (MC samples × restarts) at horizon h=3, n=64 GP"
KERNEL_BOUNDS = ([0.1], [5.0])   # optimize!(sur, lowerbounds=kernel_lbs, ...) nonmyopic_bayesopt.jl:230,285



def kernel_label(d, info):
    """The rollout kernel's name as rocprofv3 prints it: plan info spec 0 = generic <D, RPL, 0>,
    1 = Matérn-5/2 + EI <D, RPL, 1>, 2 = the half-wave kernel <D, 1, 1, 2>, 3 = Matérn-5/2 + EI +
    quadratic cost <D, RPL, 2>; the unit's fantasy capacity names the namespace (fmax4 / fmax6)."""
    rpl, spec = info["rpl"], info["spec"]
    targs = {0: f"{d}, {rpl}, 0, 1", 1: f"{d}, {rpl}, 1, 1", 2: f"{d}, 1, 1, 2", 3: f"{d}, {rpl}, 2, 1"}[spec]
    return f"mrbo::fmax{info['fmax']}::rollout_kernel<{targs}>"

def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="C3")
    ap.add_argument("--mc-per-gpu", type=int, default=0,
                    help="MC samples per GPU (default: the config's M; the metric config is C3 at M=1024)")
    ap.add_argument("--restarts", type=int, default=0, help="restarts R (default: the config's)")
    ap.add_argument("--ell", type=float, default=0.0, help="Matérn-5/2 lengthscale (default 1.0, SURVEY §8d)")
    ap.add_argument("--mle", action="store_true",
                    help="fit the lengthscale first by optimize! (radial_basis_surrogates.jl:805-829) on the "
                         "config's base data within [0.1, 5] (nonmyopic_bayesopt.jl:230)")
    ap.add_argument("--cost", action="store_true",
                    help="cost-weighted EI with NonUniformCost (cost_functions.jl:5-20; build-defined, "
                         "parity unpinned)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--schedule", choices=("auto", "index", "longest-first"), default="auto",
                    help="order in which the persistent waves take the trajectories: index order, or "
                         "longest first by the first step's work counters within each of the kernel's "
                         "eight per-XCD queue chunks (mrbo_plan_order_longest_first); auto (default) = "
                         "longest first (C3: idle tail of the persistent grid 6.6 -> 1.1 %%, kernel "
                         "9.21 -> 8.66 ms; C3-MLE 46.1 -> 45.0 ms; DESIGN.md §2)")
    ap.add_argument("--longest-first", action="store_true", help="same as --schedule longest-first")
    ap.add_argument("--resort", type=int, default=0,
                    help="longest-first schedule: re-rank from every K-th step's work counters "
                         "(0, default: from the first step's only)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--solver", choices=("sga", "adam"), default="sga",
                    help="outer update!: StandardSGA (default) or Adam (optimizers.jl:25-74), both on the device")
    ap.add_argument("--eta", type=float, default=0.0,
                    help="step: default 0.01 for StandardSGA, 0.001 for Adam (the reference's defaults, "
                         "optimizers.jl:10, 35)")
    ap.add_argument("--dump", default="", help="write the final ETO and x0 (npz) here (rank 0)")
    ap.add_argument("--sharded", action="store_true",
                    help="take the multi-rank path (process group, per-step all-gather of the shard moments, "
                         "MAX all-reduce of the clock) even at one rank: exercises the RCCL exchange on a "
                         "one-GPU box")
    return ap.parse_args()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(args):
    """--gpus N > 1 outside torchrun: start the N ranks (one process per GPU) and return their exit
    status.  Runs before anything initialises the GPU in this process (device_count() does not)."""
    import torch
    ndev = torch.cuda.device_count()
    rehearse = os.environ.get("MRBO_DIST_BACKEND", "nccl") == "gloo"
    if args.gpus > ndev and not rehearse:
        print(f"bench.py: --gpus {args.gpus} but only {ndev} GPU(s) visible", file=sys.stderr)
        return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def julia_probe():
    """BASELINE.md CPU-baseline step 1: is the Julia reference runnable on this host?"""
    j = shutil.which("julia")
    return f"julia at {j} (reference not timed: Optim/Sobol/ForwardDiff are unpinned)" if j else \
        "unavailable (no julia on this host): the baseline is the C restatement of the same path"


def oracle_timing_lib():
    """The oracle built for timing: -O3 -march=native on THIS host when gcc is present (compiled
    into a temp dir, a few seconds; the checker build stays -O2 -ffp-contract=off), else the
    shipped -O3 -march=x86-64-v3 build.  Returns (path, flags)."""
    src = os.path.join(ROOT, "oracle", "rbo_oracle.c")
    gcc = shutil.which("gcc")
    if gcc:
        out = os.path.join(tempfile.mkdtemp(prefix="rbo_native_"), "librbo_oracle_native.so")
        flags = ["-O3", "-march=native", "-fPIC", "-fopenmp", "-shared"]
        r = subprocess.run([gcc] + flags + ["-o", out, src, "-lm"], capture_output=True)
        if r.returncode == 0:
            return out, " ".join(flags)
    fast = os.path.join(ROOT, "oracle", "build", "librbo_oracle_fast.so")
    return fast, "-O3 -march=x86-64-v3 -fopenmp (prebuilt)"


def cpu_baseline(pb, M_full, R_full, budget_s, cost=None):
    """The oracle (C restatement, 'port') on the same workload, bounded sample, host cores."""
    from oracle import oracle as O
    path, flags = oracle_timing_lib()
    O.use_library(path)
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    nthreads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or aff
    s = pb.surrogate
    n = s.observed
    osur = O.OracleSurrogate(s.X[:, :n], s.L[:n, :n], s.c[:n], s.y[:n], ell=s.ψ.lengthscale, fmini=s.fmini())
    rn = pb.tp.rnstream_sequence[:M_full]
    xs = pb.es.get_starts()

    def run(Ms, Rs, nt):
        t = time.perf_counter()
        O.simulate_mc(osur, pb.x0s[:, :Rs], np.asfortranarray(rn[:Ms]), xs, pb.lbs, pb.ubs, pb.cfg.h,
                      nthreads=nt, want_policy=False, cost=cost)
        return time.perf_counter() - t

    def bounded(nt, seconds):
        """trajectories/s of nt threads over a sample of about `seconds` of this leg's work"""
        m = min(M_full, max(nt * 4, 32))
        t = run(m, 1, nt)
        m = min(M_full, max(m, int(m / t * seconds)))
        return m, run(m, 1, nt)

    Ms = min(M_full, max(nthreads * 4, 32))
    dt = run(Ms, 1, nthreads)
    rate = Ms / dt
    # scale the sample to ~budget_s seconds of CPU work (never beyond the full workload)
    target = int(rate * budget_s)
    Rs = max(1, min(R_full, target // M_full)) if target >= M_full else 1
    Ms = M_full if target >= M_full else max(Ms, min(M_full, target))
    dt = run(Ms, Rs, nthreads)
    M1 = min(M_full, 64)
    dt1 = run(M1, 1, 1)
    M1 = min(M_full, max(M1, int(M1 / dt1 * budget_s * 0.3)))
    dt1 = run(M1, 1, 1)
    # every CPU of this process's affinity set, whatever OMP_NUM_THREADS says
    # (it only sets the default; nthreads is passed to omp_set_num_threads for this leg alone)
    Ma, dta = bounded(aff, 3.0)
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()
            quota = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    O.use_library(None)
    return dict(value=Ms * Rs / dt, unit="trajectories/s", cores=nthreads, kind="port",
                sample=f"{pb.cfg.name} workload, first {Rs} restart(s) x {Ms} MC samples "
                       f"({Ms * Rs} trajectories, {dt:.1f} s), oracle/rbo_oracle.c OpenMP x{nthreads}",
                build=flags, host_cpus=os.cpu_count(), affinity_cpus=aff, reference=julia_probe(),
                single_thread={"value": M1 / dt1, "cores": 1,
                               "sample": f"first restart x {M1} MC samples ({dt1:.1f} s), 1 thread"},
                all_cores={"value": Ma / dta, "cores": aff,
                           "sample": f"first restart x {Ma} MC samples ({dta:.1f} s), {aff} threads = the "
                                     f"process's whole affinity set",
                           "cgroup_cpu_quota": quota})


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "0") or 0)
    if world == 0:
        if args.gpus > 1:
            return launch_ranks(args)
        world = 1
    elif world != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}", file=sys.stderr)
        return 2
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist
    from mrbo import configs, flops, parallel
    from mrbo.engine import from_device, to_device
    from mrbo.rollout import _plan_for

    # one process per GPU; MRBO_DIST_BACKEND=gloo + device wrap-around only for rehearsing the
    # multi-rank path on a box with fewer GPUs than ranks
    ndev = torch.cuda.device_count()
    local = local % max(ndev, 1)
    torch.cuda.set_device(local)
    backend = os.environ.get("MRBO_DIST_BACKEND", "nccl")
    sharded = world > 1 or args.sharded
    if sharded:
        # a one-rank --sharded run outside torch.distributed.run has no rendezvous in the env
        init = {} if "MASTER_ADDR" in os.environ else dict(init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0,
                                                           world_size=1)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"), **init)
        else:
            dist.init_process_group(backend, **init)
    cfg = configs.CONFIGS[args.config]
    M_local, R, d, h = (args.mc_per_gpu or cfg.M), (args.restarts or cfg.R), cfg.d, cfg.h
    M_total = M_local * world
    shards = [parallel.shard(M_total, world, k) for k in range(world)]
    lo, hi = shards[rank]
    pb = configs.problem(args.config, M=M_total, R=R, cost=args.cost)
    mle = None
    if args.mle:
        from mrbo import mle as mle_mod
        mle = mle_mod.optimize(pb.surrogate, *KERNEL_BOUNDS)
    elif args.ell > 0:
        from mrbo.kernels import Matern52
        pb.surrogate.set_kernel(Matern52([args.ell]))
    ell = pb.surrogate.ψ.lengthscale
    T = pb.T
    plan = _plan_for(T.s, h, hi - lo, R, pb.es.get_starts().shape[1], pb.lbs, pb.ubs, T.θ[0], local,
                     dict(sample_offset=lo, samples_total=M_total, **pb.plan_opts()))
    longest_first = args.longest_first or args.schedule in ("auto", "longest-first")
    dev = f"cuda:{local}"
    drn = to_device(np.asfortranarray(pb.tp.rnstream_sequence[lo:hi]), dev)   # resident in HBM
    dxs = to_device(pb.es.get_starts(), dev)
    dx0 = to_device(np.array(pb.x0s, dtype=np.float64), dev)
    out = plan.alloc_outputs(with_gradient=True)
    evals_acc = torch.zeros_like(out["evals"])
    dactive = torch.ones(R, dtype=torch.int32, device=dev)
    W = parallel.width(d)
    last = {}
    eta = args.eta or (0.01 if args.solver == "sga" else 0.001)
    if args.solver == "adam":   # Adam's moment estimates, resident beside x0 (m = v = 0 before update 1)
        dm, dv = torch.zeros_like(dx0), torch.zeros_like(dx0)

    shard_sizes = [b - a for a, b in shards]

    def step():
        plan.simulate(dx0, drn, dxs, out)   # the library records HIP events around the rollout kernel
        if not sharded:
            e = plan.eto(out)                           # two-pass mean / std(n-1) on the device
        else:
            # this shard's (Σ, M2) rows, ONE all-gather of the device tensors, Chan merge + ETO on
            # the device (mrbo_merge_moments): the same host profile as the one-GPU step
            e = parallel.sharded_eto_device(plan, plan.partial_moments(out, hi - lo), shard_sizes)
        evals_acc.add_(out["evals"])        # also in warmup: no first-use op inside the timed region
        last["n"] = last.get("n", 0) + 1
        if longest_first and ("ordered" not in last or (args.resort and last["n"] % args.resort == 0)):
            # the schedule of every later step, from this (first) step's work counters: an SGA step
            # moves x0 a little and the MC streams repeat, so a trajectory's work repeats closely
            # (--resort K: again from every K-th step's counters).  On the device, no host sync
            # (mrbo_plan_order_longest_first)
            plan.order_longest_first(out)
            last["ordered"] = True
        # eswavs + update! of every active restart on the device (mrbo_sga_step / mrbo_adam_step):
        # x0, the stop flags and Adam's moments stay in HBM, so the next launch follows without a
        # host round trip
        if args.solver == "sga":
            plan.sga_step(e, dx0, dactive, M_total, eta)
        else:
            last["t"] = last.get("t", 0) + 1
            plan.adam_step(e, dx0, dactive, dm, dv, last["t"], M_total, eta)
        last["eto_dev"] = e

    for _ in range(args.warmup):
        step()
    evals_acc.zero_()
    torch.cuda.synchronize()
    if sharded:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if sharded:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    el = torch.tensor([elapsed], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
    if sharded:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())
    # HIP events around each timed step's rollout kernel alone, on its launch stream (mrbo_kernel_times)
    kernel_ms = plan.kernel_times(args.steps) if args.steps > 0 else []
    if args.steps > len(kernel_ms):
        print(f"bench: kernel_ms averages the last {len(kernel_ms)} of {args.steps} timed launches (event ring)",
              file=sys.stderr)
    last["eto"] = last["eto_dev"].cpu().numpy().reshape((W, R), order="F")
    x0 = from_device(dx0, (d, R))
    active = dactive.cpu().numpy().astype(bool)

    st = out["status"].cpu().numpy()
    ev = evals_acc.cpu().numpy().reshape((flops.NCOUNTERS, hi - lo, R), order="F") / max(args.steps, 1)
    info = plan.info()
    fl = flops.launch_flops(ev, cfg.N, d, h, info=info, nstarts=pb.es.get_starts().shape[1])
    kms = float(np.mean(kernel_ms)) if kernel_ms else float("nan")
    achieved = fl / (kms * 1e-3) / 1e12
    traffic = None
    tag = cfg.name + ("" if ell == 1.0 and not args.cost else f"_ell{ell:.4g}" + ("_cost" if args.cost else ""))
    tpath = os.path.join(ROOT, "profiles", f"traffic_{tag}.json")
    if os.path.exists(tpath):
        with open(tpath) as f:
            traffic = json.load(f).get("bytes_per_launch")
    total = world * (hi - lo) * R * args.steps if world == 1 else sum(b - a for a, b in shards) * R * args.steps
    rule = "cost-weighted EI (NonUniformCost)" if args.cost else "EI"
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
                   "trajectories_per_step": sum(b - a for a, b in shards) * R, "M_per_gpu": hi - lo, "R": R,
                   "h": h, "N": cfg.N, "d": d, "kernel": f"Matern52(ℓ={ell:.6g})",
                   "lengthscale_source": "optimize! MLE in [0.1, 5]" if mle else ("--ell" if args.ell > 0 else
                                                                                 "ℓ = 1 (SURVEY §8d)"),
                   "rule": rule, "parallelism": f"mc-shard x{world}",
                   "exchange": "none" if not sharded else f"all-gather of (Σ, M2) moments, {W * R * 8} B/rank/step",
                   "outer_step": (f"eswavs + StandardSGA η={eta:g}, no clip (utils.jl:114-123, optimizers.jl:16-22)"
                                  if args.solver == "sga" else
                                  f"eswavs + Adam η={eta:g} β=(0.9, 0.999) ε=1e-8 (utils.jl:114-123, "
                                  f"optimizers.jl:49-74)"),
                   "schedule": "longest first within the per-XCD queue chunks (first step's work counters)" if longest_first else "index order"},
        "roofline": {"bound": "mfma", "achieved": achieved, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": achieved / FP64_PEAK_TFLOPS, "traffic": traffic,
                     "kernel": kernel_label(d, info), "kernel_ms": kms, "flops_per_launch": fl,
                     "kernel_ms_launches": len(kernel_ms),   # the plan keeps the last 64 launches' events
                     "launch": info,
                     "note": "compute-bound fp64: peak = the dense fp64 matrix peak, equal to the fp64 vector "
                             "peak on MI355X; the kernel issues VALU v_fma_f64 (matrix-vector work, not "
                             "GEMM-shaped); algorithmic FLOP model in DESIGN.md §5; HBM algorithmic "
                             "bytes/traj ~0.3 KB so an HBM roofline does not bind; traffic = PMC bytes per "
                             f"launch from profiles/traffic_{tag}.json"},
        "status_errors": int((st != 0).sum()),
        "work_per_traj": {"grad_evals": float(ev[0].mean()), "value_evals": float(ev[1].mean()),
                          "hessians": float(ev[2].mean()), "rich_evals": float(ev[3].mean()),
                          "pairs": float(ev[4].mean())},
    }
    if mle:
        res["config"]["mle"] = {"theta": float(mle["theta"][0]), "neg_log_likelihood": float(mle["neg_log_likelihood"]),
                                "iterations": int(mle["iterations"])}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline(pb, M_local, R, args.cpu_seconds, cost=pb.cost_model())
    if rank == 0:
        print(json.dumps(res), flush=True)
        if args.dump:
            np.savez(args.dump, eto=last["eto"], x0=x0, active=active)
    if sharded:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
