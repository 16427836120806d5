"""The trajectory schedule (mrbo_plan_set_order, include/mrbo.h) changes only WHICH wave runs a
trajectory and when, never a result: every output of a launch -- values, gradients, status, policy
points, observations and work counters -- is bit-identical under any permutation of the M×R
trajectory indices.  Each trajectory is one wave's sequential program over its own MC stream
(rollout.jl:279-340 runs the samples independently), so this is what the reference's independent
sample loop guarantees too.  An out-of-range entry of the order falls back to the queue index
(mrbo_rollout.hip rollout_kernel), so a malformed schedule cannot write outside the outputs.
"""
import ctypes

import numpy as np
import pytest

import conftest  # noqa: F401  (sys.path)

pytestmark = pytest.mark.gpu


def _setup(name, M, R):
    import torch
    from mrbo import configs
    from mrbo.engine import to_device
    from mrbo.rollout import _plan_for
    cfg = configs.CONFIGS[name]
    pb = configs.problem(name, M=M, R=R)
    plan = _plan_for(pb.T.s, cfg.h, M, R, pb.es.get_starts().shape[1], pb.lbs, pb.ubs, pb.T.θ[0], 0,
                     dict(sample_offset=0, samples_total=M, **pb.plan_opts()))
    dev = "cuda:0"
    args = (to_device(np.asfortranarray(pb.x0s), dev), to_device(np.asfortranarray(pb.tp.rnstream_sequence[:M]), dev),
            to_device(pb.es.get_starts(), dev))
    return torch, plan, args


def _launch(torch, plan, args):
    out = plan.alloc_outputs(with_gradient=True, want_policy=True, want_obs=True)
    plan.simulate(*args, out)
    torch.cuda.synchronize()
    return out


@pytest.mark.parametrize("name,M,R", [("C2", 256, 16), ("C3", 128, 8)])
def test_results_independent_of_schedule(gpu, name, M, R):
    torch, plan, args = _setup(name, M, R)
    ref = _launch(torch, plan, args)
    assert (ref["status"] == 0).all()
    assert (ref["values"] != 0).any() and (ref["grad_x"] != 0).any()   # not a vacuous comparison
    T = M * R
    idx = torch.arange(T, dtype=torch.int64, device="cuda:0")
    g = torch.Generator(device="cuda:0").manual_seed(7)
    ev = ref["evals"].view(T, -1).to(torch.float64)
    w = torch.tensor(plan.ORDER_WEIGHTS, dtype=torch.float64, device="cuda:0")
    orders = {
        "reversed": (T - 1 - idx).to(torch.int32),
        "interleave": ((idx % R) * M + idx // R).to(torch.int32),
        "random": torch.randperm(T, device="cuda:0", generator=g).to(torch.int32),
        "longest_first": torch.argsort(ev @ w, descending=True).to(torch.int32),
        # every entry out of range: each queue index runs its own trajectory (the guard)
        "out_of_range": torch.full((T,), -1, dtype=torch.int32, device="cuda:0"),
    }
    try:
        for oname, order in orders.items():
            plan.set_order(order, check=oname != "out_of_range")
            out = _launch(torch, plan, args)
            for k, v in ref.items():
                assert torch.equal(out[k], v), f"{name} order {oname}: output {k} differs"
    finally:
        plan.set_order(None)
    assert all(torch.equal(_launch(torch, plan, args)[k], v) for k, v in ref.items())


def test_set_order_rejects_wrong_length(gpu):
    """The C ABI refuses an order whose length is not M×R (MRBO_ERR_ARG); the Python mirror refuses
    it before the call."""
    torch, plan, _ = _setup("C2", 32, 2)
    bad = torch.arange(63, dtype=torch.int32, device="cuda:0")
    with pytest.raises(ValueError):
        plan.set_order(bad)
    dup = torch.zeros(64, dtype=torch.int32, device="cuda:0")     # right length, not a permutation
    with pytest.raises(ValueError, match="permutation"):
        plan.set_order(dup)
    rc = plan.lib.mrbo_plan_set_order(plan.handle, ctypes.c_void_p(bad.data_ptr()), bad.numel())
    assert rc == -1   # MRBO_ERR_ARG


@pytest.mark.parametrize("name,M,R", [("C2", 256, 16), ("C3", 128, 8), ("C3", 100, 3)])
def test_library_longest_first_order(gpu, name, M, R):
    """mrbo_plan_order_longest_first: the device-computed order is a permutation, equals the torch
    mirror (each per-XCD queue chunk's own trajectories, longest first by the weighted counters, ties
    in index order: RolloutPlan.longest_first_order), is what the plan's next launches use, and
    leaves every output bit-identical.  M·R = 300 checks the ragged chunk sizes."""
    torch, plan, args = _setup(name, M, R)
    ref = _launch(torch, plan, args)
    T = M * R
    got = torch.full((T,), -7, dtype=torch.int32, device="cuda:0")
    try:
        plan.order_longest_first(ref, order_out=got)
        torch.cuda.synchronize()
        assert torch.equal(torch.sort(got.to(torch.int64)).values, torch.arange(T, device="cuda:0"))
        assert torch.equal(got, plan.longest_first_order(ref["evals"]))
        # the first position of every chunk holds that chunk's longest trajectory
        ev = ref["evals"].view(T, -1).to(torch.float64) @ torch.tensor(plan.ORDER_WEIGHTS, dtype=torch.float64,
                                                                       device="cuda:0")
        for x in range(8):
            lo, hi = x * T // 8, (x + 1) * T // 8
            if hi > lo:
                assert ev[got[lo].long()] == ev[lo:hi].max()
        out = _launch(torch, plan, args)     # runs in the library's order
        for k, v in ref.items():
            assert torch.equal(out[k], v), f"{name}: output {k} differs under the library's order"
    finally:
        plan.set_order(None)


def test_library_longest_first_order_rejects_null_counters(gpu):
    """mrbo_plan_order_longest_first refuses a null work-counter array (MRBO_ERR_ARG) and leaves the
    plan's schedule as it was: the next launch's outputs equal an index-order launch's."""
    torch, plan, args = _setup("C2", 32, 2)
    ref = _launch(torch, plan, args)
    assert plan.lib.mrbo_plan_order_longest_first(plan.handle, None, None, None) == -1   # MRBO_ERR_ARG
    out = _launch(torch, plan, args)
    for k, v in ref.items():
        assert torch.equal(out[k], v)
