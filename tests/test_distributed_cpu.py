"""World-size-2/3/8 gloo tests of the multi-GPU path's exchange (no GPU): each rank rolls out its
contiguous MC shard (the CPU oracle stands in for the device here -- test infrastructure),
reduces its per-restart moments (Σ, M2), one all_gather, Chan merge, and every rank derives the
same ETO as a single-process run over all samples."""
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


def _case(world):
    """golden c2near (6 MC × 2 restarts) for 2 and 3 ranks; 8 ranks -- the 8-GPU node's world --
    on C2's base data at 24 MC × 2 restarts (3 samples per rank)"""
    if world <= 3:
        return load_golden("c2near")
    import sys
    sys.path[:0] = [os.path.join(ROOT, "rollout-bayesian-optimization_amd"), os.path.join(ROOT, "tests")]
    from parity import _problem_arrays
    return _problem_arrays("C2", 24, 2)


def _worker(rank, world, port, out_q):
    import sys
    sys.path[:0] = [os.path.join(ROOT, "rollout-bayesian-optimization_amd"), ROOT]
    import torch
    import torch.distributed as dist
    from mrbo.parallel import local_moments, sharded_eto, shard
    from oracle import oracle as O
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = _case(world)
    h, M = int(g["h"]), g["rnstream"].shape[0]
    d, R = g["x0s"].shape
    lo, hi = shard(M, world, rank)
    s = O.OracleSurrogate(g["X"], g["L"], g["c"], g["y"], fmini=float(g["fmini"]))
    o = O.simulate_mc(s, g["x0s"], np.asfortranarray(g["rnstream"][lo:hi]), g["xstarts"], g["lbs"], g["ubs"], h,
                      sample_offset=lo, samples_total=M, nthreads=1)
    mom = local_moments(o["values"], o["grad_x"], o["grad_theta"][0])
    t = torch.from_numpy(mom.ravel(order="F").copy())
    sizes = [b - a for a, b in (shard(M, world, k) for k in range(world))]
    eto = sharded_eto(t, sizes, d)
    out_q.put((rank, eto))
    dist.barrier()
    dist.destroy_process_group()


import pytest


@pytest.mark.parametrize("world", [2, 3, 8])
def test_gloo_eto_matches_single_process(oracle, world):
    g = _case(world)
    h = int(g["h"])
    s = oracle.OracleSurrogate(g["X"], g["L"], g["c"], g["y"], fmini=float(g["fmini"]))
    full = oracle.simulate_mc(s, g["x0s"], g["rnstream"], g["xstarts"], g["lbs"], g["ubs"], h, nthreads=1)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(1, world):
        np.testing.assert_array_equal(res[0], res[r])      # every rank takes the same step
    np.testing.assert_allclose(res[0], full["eto"], rtol=1e-12, atol=1e-15)
