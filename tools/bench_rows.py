#!/usr/bin/env python3
"""Measurements of the SURVEY §8(f) rows beside the headline bench (one JSON line per row).

  ghq     simulate_trajectory_ghq (rollout.jl:409-467) at the C3 shape: 5 Gauss–Hermite nodes,
          depth h+1 = 4 → 625 node vectors × 64 restarts per launch; trajectories/s, with the
          oracle on the host cores beside it (bounded sample).
  gp_fit  the base-GP refit + log-likelihood + ∂/∂ℓ behind optimize! (radial_basis_surrogates.jl:
          770-829) for P = 256 candidate lengthscales at N = 64 / 128 / 256 (d = 6); fits/s and
          the kernel's algorithmic fp64 rate (N³/3 + N³/2 + N³/6 FMAs per fit), with the oracle
          (one fit per call, threads over candidates) beside it.

Kernel times come from HIP events on the launch stream; run under rocprofv3 --kernel-trace
--stats for the per-kernel averages (profiles/).
usage: python tools/bench_rows.py [--rows ghq,gp_fit] [--cpu-seconds 5]
"""
import argparse
import ctypes
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "rollout-bayesian-optimization_amd"), ROOT]

FP64_PEAK_TFLOPS = 78.6


def cpu_threads():
    return int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)


def row_ghq(args):
    import torch
    from mrbo import configs
    from mrbo.engine import to_device
    from mrbo.rollout import _plan_for, ghq_node_arrays
    from mrbo.utils import gauss_hermite, generate_indices
    from oracle import oracle as O
    pb = configs.problem("C3")
    h, R = pb.cfg.h, pb.cfg.R
    t, w = gauss_hermite(5)
    nodes, weights = ghq_node_arrays(t, w, generate_indices(5, h + 1))
    M = nodes.shape[0]
    xs = pb.es.get_starts()
    plan = _plan_for(pb.T.s, h, M, R, xs.shape[1], pb.lbs, pb.ubs, 0.0, 0, {})
    dev = "cuda:0"
    dx0, dn, dw, dxs = (to_device(a, dev) for a in (pb.x0s, nodes, weights, xs))
    out = plan.alloc_outputs(with_gradient=True)
    st = torch.cuda.current_stream()
    for _ in range(2):
        plan.simulate_ghq(dx0, dn, dw, dxs, out)
    torch.cuda.synchronize()
    steps = 5
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(st)
    for _ in range(steps):
        plan.simulate_ghq(dx0, dn, dw, dxs, out)
    e1.record(st)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / steps
    kms = e0.elapsed_time(e1) / steps
    assert (out["status"].cpu().numpy() == 0).all()
    # oracle beside it: first restarts × all node vectors, threads over (restart, node vector)
    s = pb.surrogate
    n = s.observed
    osur = O.OracleSurrogate(s.X[:, :n], s.L[:n, :n], s.c[:n], s.y[:n], fmini=s.fmini())
    nt = cpu_threads()
    Rs = 1
    t0 = time.perf_counter()
    O.simulate_mc(osur, pb.x0s[:, :Rs], None, xs, pb.lbs, pb.ubs, h, ghq=(nodes, weights), nthreads=nt,
                  want_policy=False)
    dt = time.perf_counter() - t0
    Rs = int(max(1, min(R, args.cpu_seconds / dt)))
    if Rs > 1:
        t0 = time.perf_counter()
        O.simulate_mc(osur, pb.x0s[:, :Rs], None, xs, pb.lbs, pb.ubs, h, ghq=(nodes, weights), nthreads=nt,
                      want_policy=False)
        dt = time.perf_counter() - t0
    return {"row": "ghq", "metric": "Gauss-Hermite rollout trajectories/sec", "value": M * R / wall,
            "unit": "trajectories/s", "kernel_ms": kms, "config": {"workload": "C3 shape, 5 nodes, depth 4",
                                                                   "node_vectors": M, "R": R, "h": h},
            "cpu_baseline": {"value": M * Rs / dt, "unit": "trajectories/s", "cores": nt, "kind": "port",
                             "sample": f"{Rs} restart(s) x {M} node vectors ({dt:.1f} s)"}}


def row_gp_fit(args, N, P=256, d=6):
    import torch
    from mrbo import _lib
    from oracle import oracle as O
    L = _lib.load()
    rng = np.random.default_rng(N)
    X = np.asfortranarray(rng.random((d, N)))
    y = np.sin(3 * X.sum(0))
    ells = np.linspace(0.3, 3.0, P)
    dp = ctypes.POINTER(ctypes.c_double)
    sd = _lib.SurrogateDesc(d, N, 0, 1.0, 1e-6, float(y.min()), X.ctypes.data_as(dp), None, N, None,
                            y.ctypes.data_as(dp))
    dev = "cuda:0"
    de = torch.from_numpy(ells).to(dev)
    ll = torch.empty(P, dtype=torch.float64, device=dev)
    dll = torch.empty_like(ll)
    stt = torch.empty(P, dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream()
    vp = lambda t: ctypes.c_void_p(t.data_ptr())

    def call():
        _lib.check(L.mrbo_gp_fit(ctypes.byref(sd), P, vp(de), vp(ll), vp(dll), vp(stt), None, None, 0,
                                 ctypes.c_void_p(st.cuda_stream)))

    call()
    torch.cuda.synchronize()
    steps = 5
    kms, calls, t0 = [], [], time.perf_counter()
    for _ in range(steps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        call()
        e1.record(st)
        torch.cuda.synchronize()
        kms.append(L.mrbo_last_gp_fit_ms())        # the kernel alone (events inside the call)
        calls.append(e0.elapsed_time(e1))           # the whole call: X/y staging, launch, sync
    wall = (time.perf_counter() - t0) / steps
    assert (stt.cpu().numpy() == 0).all()
    kms, call_ms = float(np.median(kms)), float(np.median(calls))
    # algorithmic FMAs per fit: Cholesky N³/6, L⁻¹ N³/6, lower(VᵀV) N³/6 (register / LDS kernels
    # and the tile kernel alike); 2 flops per FMA
    flops = 2.0 * (N ** 3 / 2) * P
    # oracle: one fit per call, threads over candidates
    nt = cpu_threads()
    nP = min(P, 16)
    t0 = time.perf_counter()
    with ThreadPoolExecutor(nt) as ex:
        list(ex.map(lambda e: O.log_likelihood(X, y, "matern52", e, 1e-6), ells[:nP]))
    dt = time.perf_counter() - t0
    if dt < args.cpu_seconds / 4 and nP < P:
        nP = int(min(P, nP * args.cpu_seconds / 4 / max(dt, 1e-3)))
        t0 = time.perf_counter()
        with ThreadPoolExecutor(nt) as ex:
            list(ex.map(lambda e: O.log_likelihood(X, y, "matern52", e, 1e-6), ells[:nP]))
        dt = time.perf_counter() - t0
    return {"row": "gp_fit", "metric": "GP refits (K, chol, c, log-likelihood, d/dl)/sec",
            "value": P / (call_ms * 1e-3), "unit": "fits/s", "kernel_ms": kms, "call_ms": call_ms,
            "kernel_fits_per_s": P / (kms * 1e-3), "wall_ms_per_call": wall * 1e3,
            "roofline": {"bound": "mfma", "achieved": flops / (kms * 1e-3) / 1e12, "peak": FP64_PEAK_TFLOPS,
                         "unit": "TFLOP/s", "frac": flops / (kms * 1e-3) / 1e12 / FP64_PEAK_TFLOPS, "traffic": None},
            "config": {"workload": f"N={N} d={d} Matern52, {P} lengthscales per launch"},
            "cpu_baseline": {"value": nP / dt, "unit": "fits/s", "cores": nt, "kind": "port",
                             "sample": f"{nP} fits ({dt:.2f} s), oracle rbo_log_likelihood, {nt} threads"}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", default="ghq,gp_fit")
    ap.add_argument("--cpu-seconds", type=float, default=5.0)
    ap.add_argument("--gpfit-n", default="64,128,256,384,512", help="gp_fit rows: comma list of N")
    args = ap.parse_args()
    rows = args.rows.split(",")
    if "ghq" in rows:
        print(json.dumps(row_ghq(args)), flush=True)
    if "gp_fit" in rows:
        for N in (int(n) for n in args.gpfit_n.split(",")):
            print(json.dumps(row_gp_fit(args, N)), flush=True)


if __name__ == "__main__":
    main()
