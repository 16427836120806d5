"""World-size-2 gloo test of the multi-GPU path's reduction (no GPU): each rank rolls out its
contiguous MC shard (the CPU oracle stands in for the device here -- test infrastructure),
reduces per-restart partial sums, one all_reduce, and every rank derives the same ETO as a
single-process run over all samples."""
import os
import socket

import numpy as np
import torch.multiprocessing as mp

from conftest import ROOT, load_golden


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_q):
    import sys
    sys.path[:0] = [os.path.join(ROOT, "rollout-bayesian-optimization_amd"), ROOT]
    import torch
    import torch.distributed as dist
    from mrbo.parallel import allreduce_sums, eto_from_sums, shard
    from oracle import oracle as O
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = load_golden("c2near")
    h, M = int(g["h"]), g["rnstream"].shape[0]
    d, R = g["x0s"].shape
    lo, hi = shard(M, world, rank)
    s = O.OracleSurrogate(g["X"], g["L"], g["c"], g["y"], fmini=float(g["fmini"]))
    o = O.simulate_mc(s, g["x0s"], np.asfortranarray(g["rnstream"][lo:hi]), g["xstarts"], g["lbs"], g["ubs"], h,
                      sample_offset=lo, samples_total=M, nthreads=1)
    W = 2 + 2 * d + 2
    sums = np.zeros((W, R))
    v, gx, gt = o["values"], o["grad_x"], o["grad_theta"][0]
    sums[0], sums[1] = v.sum(0), (v ** 2).sum(0)
    sums[2:2 + d], sums[2 + d:2 + 2 * d] = gx.sum(1), (gx ** 2).sum(1)
    sums[2 + 2 * d], sums[3 + 2 * d] = gt.sum(0), (gt ** 2).sum(0)
    t = torch.from_numpy(sums.ravel(order="F").copy())
    allreduce_sums(t)
    eto = eto_from_sums(t.numpy().reshape((W, R), order="F"), M, d)
    out_q.put((rank, eto))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_eto_matches_single_process(oracle):
    g = load_golden("c2near")
    h = int(g["h"])
    s = oracle.OracleSurrogate(g["X"], g["L"], g["c"], g["y"], fmini=float(g["fmini"]))
    full = oracle.simulate_mc(s, g["x0s"], g["rnstream"], g["xstarts"], g["lbs"], g["ubs"], h, nthreads=1)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    np.testing.assert_allclose(res[0], res[1], rtol=0, atol=0)
    np.testing.assert_allclose(res[0], full["eto"], rtol=1e-9, atol=1e-15)
