"""GPU parity tests: libmrbo.so (HIP, gfx950) against the CPU oracle and the golden fixtures.

Tolerances (fp64 throughout):
  primitives (μ, σ, ∇, Hα at base points)            rtol 1e-9
  replay against the NumPy goldens                     obs rtol 1e-9, values 1e-8, gradients 1e-6
                                                       (the goldens' own LAPACK-vs-substitution
                                                       agreement, tests/golden/make_golden.py)
  end-to-end against the oracle                        the T2 / T3 bounds and the non-vacuity
                                                       guard of tests/parity.py
The GPU computes triangular solves through the explicit inverse factor and sums in a
different order than the oracle's substitution, hence tolerances rather than bit equality.
"""
import ctypes

import numpy as np
import pytest

from conftest import GOLDEN_CASES, load_golden
from parity import _assert_grads_close, _end_to_end, _osur, _plan, _problem_arrays, _replay_t2, _run

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("case", GOLDEN_CASES)
def test_eval_base_vs_golden(gpu, case):
    g = load_golden(case)
    p = _plan(g)
    np.testing.assert_allclose(p.eval_base(g["pts"]), g["prim"], rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize("case", GOLDEN_CASES)
def test_replay_vs_golden(gpu, case):
    g = load_golden(case)
    r = _run(_plan(g), g, dual=g["dual_y_dx"], replay=g["replay_x"])
    assert (r["status"] == 0).all()
    np.testing.assert_allclose(r["obs"], g["obs"], rtol=1e-9, atol=1e-11)
    np.testing.assert_allclose(r["values"], g["values"], rtol=1e-8, atol=1e-11)
    _assert_grads_close(r["grad_x"], g["grad_x"])
    _assert_grads_close(r["grad_theta"], g["grad_theta"])


# (config, M, R, ℓ, kind): d = 1 (C1) always meets Q4 (det(H) < 1e-4 at a strict maximum of odd
# dimension, rollout.jl:159-161), so its adjoint does no back-substitution; C5 at ℓ = 1 likewise at
# d = 8.  C4 runs at ℓ = 0.5 (at ℓ = 1 no C4 trajectory improves on fmini).
SMALL_CASES = [("C1", 32, 4, None, "forward"), ("C2", 32, 4, None, "full"), ("C3", 32, 4, None, "full"),
               ("C4", 8, 2, 0.5, "full"), ("C5", 4, 2, None, "forward"), ("C5", 4, 2, 20.0, "full")]


@pytest.mark.parametrize("name,M,R,ell,kind", SMALL_CASES)
def test_end_to_end_vs_oracle(gpu, oracle, name, M, R, ell, kind):
    """Both sides run the full rollout including the inner Newton solves, then the oracle replays
    the GPU's policy points: the T2 / T3 bounds of tests/parity.py at small M × R.  C5 also runs
    with a lengthscale at the design spacing (dense K; at ℓ = 1 its K is nearly the identity)."""
    g = _problem_arrays(name, M, R, ell=ell)
    _end_to_end(oracle, f"{name} small ({M} x {R}, l={ell or 1.0:.4g}, {kind})", g, M, kind=kind,
                work_exact="steps" if name == "C4" else True, envelope=name == "C4")


@pytest.mark.parametrize("rule,rid,theta", [("POI", 1, 0.0), ("POI", 1, 0.05), ("LCB", 2, 2.0)])
def test_other_rules_vs_oracle(gpu, oracle, rule, rid, theta):
    """POI / LCB base rules (decision_rules.jl:101-127): primitives, then full rollouts with the
    inner Newton solves on both sides and the oracle's replay of the GPU's policy points, under the
    same T2 / T3 bounds and non-vacuity guard as EI (tests/parity.py)."""
    g = _problem_arrays("C2", 64, 4)
    p = _plan(g, theta=theta, rule=rid)
    osur = _osur(oracle, g)
    pts = np.asfortranarray(g["xstarts"][:, :8] * 0.9 + 0.05)
    np.testing.assert_allclose(p.eval_base(pts), oracle.eval_base(osur, pts, theta=theta, rule=rule),
                               rtol=1e-9, atol=1e-12)
    _end_to_end(oracle, f"C2 {rule} theta={theta} (64 x 4)", g, 64, rule=rule, theta=theta)


def test_ghq_vs_oracle(gpu, oracle):
    """Gauss–Hermite estimator (rollout.jl:409-467): h = 2, 5 nodes → 125 node vectors × 4 restarts,
    full rollouts with inner solves on both sides and the oracle's replay of the GPU's policy
    points, under the T2 / T3 bounds and non-vacuity guard of tests/parity.py."""
    from mrbo.rollout import ghq_node_arrays
    from mrbo.utils import gauss_hermite, generate_indices
    g = _problem_arrays("C2", 8, 4)
    t, w = gauss_hermite(5)
    nodes, weights = ghq_node_arrays(t, w, generate_indices(5, int(g["h"]) + 1))
    _end_to_end(oracle, f"C2 Gauss-Hermite ({nodes.shape[0]} node vectors x 4)", g, nodes.shape[0],
                ghq=(np.asfortranarray(nodes), np.asfortranarray(weights)))


@pytest.mark.parametrize("kernel,kid", [("matern32", 1), ("matern12", 2), ("se", 3), ("periodic", 4)])
def test_other_kernels_replay_vs_oracle(gpu, oracle, kernel, kid):
    g = _problem_arrays("C2", 16, 2, kernel=kernel)
    p = _plan(g, kernel=kid)
    pts = np.asfortranarray(g["xstarts"][:, :8] * 0.9 + 0.05 * g["x0s"][:, :1])
    np.testing.assert_allclose(p.eval_base(pts), oracle.eval_base(_osur(oracle, g, kernel), pts), rtol=1e-9,
                               atol=1e-12)
    r = _run(p, g)
    rp = np.asfortranarray(r["policy_x"][:, 1:])
    o = oracle.simulate_mc(_osur(oracle, g, kernel), g["x0s"], g["rnstream"], g["xstarts"], g["lbs"], g["ubs"],
                           int(g["h"]), replay_x=rp, nthreads=8, want_kappa=True)
    assert (r["status"] == o["status"]).all()
    if kernel == "matern12":  # ψ''(0) > 0: Dk(0) is indefinite, gp_draw's cholesky fails (PosDefException)
        assert (r["status"] & 2).all()
    _replay_t2(g, r, o, r["status"] == 0)


@pytest.mark.parametrize("d,N,h", [(1, 12, 2), (3, 24, 2), (4, 40, 3), (5, 30, 2), (7, 48, 2), (8, 64, 3), (3, 96, 2),
                                   (6, 128, 4), (3, 150, 2), (5, 200, 5), (8, 256, 3),
                                   (9, 20, 2), (10, 24, 3), (12, 60, 2), (16, 24, 2), (16, 100, 2),
                                   (4, 300, 2), (6, 384, 2), (8, 512, 2)])
def test_dimensions_and_sizes_replay_vs_oracle(gpu, oracle, d, N, h):
    """d = 1..16 and N up to 512 on Ackley(d): one data row per lane (N ≤ 64, L0⁻¹ square in
    LDS), two (N ≤ 128, three square 64×64 blocks in LDS), four or eight (N ≤ 256 / 512, L0⁻¹ in
    global memory); d > 8 up to N = 128 (the reference's 10-D / 16-D experiments run budgets of
    15, experiments/archived/dimensions-timing/nonmyopic_bayesopt/metadata.txt); ragged N.  The
    lengthscale tracks the design spacing (0.6 · width · N^(-1/d)) so that K is dense: with ℓ = 1
    on Ackley's 65-wide box K ≈ I and the triangular products would multiply zeros."""
    ell = 0.6 * 65.536 * N ** (-1.0 / d)
    g = _problem_arrays(None, 8, 2, testfn="ackley", d=d, N=N, h=h, ell=ell)
    p = _plan(g)
    pts = np.asfortranarray(g["xstarts"][:, :6] * 0.9 + 0.05 * g["x0s"][:, :1])
    np.testing.assert_allclose(p.eval_base(pts), oracle.eval_base(_osur(oracle, g), pts), rtol=1e-9, atol=1e-12)
    r = _run(p, g)
    assert (r["status"] == 0).all()
    rp = np.asfortranarray(r["policy_x"][:, 1:])
    o = oracle.simulate_mc(_osur(oracle, g), g["x0s"], g["rnstream"], g["xstarts"], g["lbs"], g["ubs"], h,
                           replay_x=rp, nthreads=8, want_kappa=True)
    _replay_t2(g, r, o)


def test_full_size_c3_properties(gpu):
    """Headline size (65 536 trajectories): size-independent properties."""
    g = _problem_arrays("C3", 1024, 64)
    p = _plan(g)
    a = _run(p, g, want_policy=False)
    b = _run(p, g, want_policy=False)
    assert (a["status"] == 0).all()
    np.testing.assert_array_equal(a["values"], b["values"])          # deterministic
    np.testing.assert_array_equal(a["grad_x"], b["grad_x"])
    assert (a["values"] >= 0).all()
    z = a["values"] == 0                                               # case 1: no improvement -> ∇ = 0
    assert (a["grad_x"][:, z] == 0).all() and (a["grad_theta"][:, z] == 0).all()
    # obs consistency: value = max(fmini - min(obs), 0)
    np.testing.assert_allclose(a["values"], np.maximum(g["fmini"] - a["obs"].min(axis=0), 0.0), rtol=0, atol=0)
    # ETO kernel == two-pass mean / std(n-1) (rollout.jl:328-339)
    np.testing.assert_allclose(a["eto"][0], a["values"].mean(0), rtol=1e-12)
    np.testing.assert_allclose(a["eto"][1], a["values"].std(0, ddof=1), rtol=1e-10)
    np.testing.assert_allclose(a["eto"][2:8], a["grad_x"].mean(1), rtol=1e-10, atol=1e-18)


def test_sharded_plans_equal_single_plan(gpu):
    """Two MC shards (multi-GPU decomposition) reproduce the single launch bit for bit."""
    g = _problem_arrays("C2", 64, 4)
    full = _run(_plan(g), g)
    parts = []
    for lo, hi in [(0, 24), (24, 64)]:
        gg = dict(g)
        gg["rnstream"] = np.asfortranarray(g["rnstream"][lo:hi])
        parts.append(_run(_plan(gg, M=hi - lo, sample_offset=lo, samples_total=64), gg))
    np.testing.assert_array_equal(np.concatenate([q["values"] for q in parts], 0), full["values"])
    np.testing.assert_array_equal(np.concatenate([q["grad_x"] for q in parts], 1), full["grad_x"])


def test_horizon_zero_and_single_sample(gpu, oracle):
    g = _problem_arrays("C2", 8, 2)
    g["rnstream"] = np.asfortranarray(g["rnstream"][:, :, :1])
    r = _run(_plan(g, h=0), g)
    o = oracle.simulate_mc(_osur(oracle, g), g["x0s"], g["rnstream"], g["xstarts"], g["lbs"], g["ubs"], 0)
    np.testing.assert_allclose(r["values"], o["values"], rtol=1e-9, atol=1e-12)
    _assert_grads_close(r["grad_x"], o["grad_x"])
    # M = 1: std with n-1 is NaN (Q14)
    g1 = dict(g)
    g1["rnstream"] = np.asfortranarray(g["rnstream"][:1])
    r1 = _run(_plan(g1, M=1, h=0), g1)
    assert np.isnan(r1["eto"][1]).all()


def test_explicit_dual_draws_and_no_gradient(gpu):
    g = load_golden("c2near")
    p = _plan(g)
    a = _run(p, g, dual=g["dual_y_dx"], replay=g["replay_x"])
    b = _run(p, g, dual=g["dual_y_dx"], replay=g["replay_x"], with_gradient=False)
    np.testing.assert_array_equal(a["values"], b["values"])
    assert "grad_x" not in b


def test_host_pointer_flag_matches_device_path(gpu):
    """MRBO_FLAG_HOST_POINTERS: the Julia-shim path with host arrays (PCIe staging)."""
    from mrbo import _lib
    g = load_golden("c2")
    p = _plan(g)
    dev = _run(p, g, dual=g["dual_y_dx"], replay=g["replay_x"], want_policy=False)
    d, M, R = p.d, p.M, p.R
    vals = np.zeros((M, R), order="F")
    gx = np.zeros((d, M, R), order="F")
    gt = np.zeros((1, M, R), order="F")
    st = np.zeros((M, R), dtype=np.int32, order="F")
    keep = [np.asfortranarray(g[k], dtype=np.float64) for k in ("x0s", "rnstream", "xstarts", "dual_y_dx", "replay_x")]
    ptr = [ctypes.c_void_p(a.ctypes.data) for a in keep]
    outp = [ctypes.c_void_p(a.ctypes.data) for a in (vals, gx, gt, st)]
    _lib.check(p.lib.mrbo_simulate_mc(p.handle, *ptr, *outp, None, None, None, _lib.MRBO_FLAG_HOST_POINTERS, None))
    np.testing.assert_array_equal(vals, dev["values"])
    np.testing.assert_array_equal(gx, dev["grad_x"])


def test_reference_signature_and_outer_ascent(gpu):
    """simulate_trajectory_mc(T, tp; …) fills the caller's containers (rollout.jl:318-322) and
    stochastic_solve runs the outer SGA (utils.jl:235-265)."""
    from mrbo import StandardSGA, configs, simulate_trajectory_mc, stochastic_solve
    pb = configs.problem("C2", M=64, R=1)
    es = pb.es
    eto = simulate_trajectory_mc(pb.T, pb.tp, es.get_starts(), es.get_container("f"),
                                 es.get_container("grad_f"), es.get_container("grad_hypers"))
    assert eto.mean() == pytest.approx(es.resolutions.mean(), rel=1e-12)
    np.testing.assert_allclose(eto.gradient(), es.spatial_gradients_container.mean(axis=1), rtol=1e-10)
    x = stochastic_solve(StandardSGA(η=0.5), pb.surrogate, pb.tp, es, pb.x0s[:, 0], T=pb.T, iterations=3)
    assert x.shape == (2,) and np.all(np.isfinite(x))


@pytest.mark.parametrize("name,M,R", [("C2", 32, 4), ("C3", 32, 4), ("C4", 8, 2)])
def test_specialised_kernel_equals_generic(gpu, monkeypatch, name, M, R):
    """Matérn-5/2 + EI runs rollout_kernel<D, RPL, 1> (kernel and rule fixed at compile time);
    MRBO_GENERIC_KERNEL=1 forces the generic instantiation.  Same source and operation order; the
    compiler schedules the two differently (measured: a few results differ by 1 ulp), so the
    comparison is to rtol 1e-12, with identical policy paths and identical Newton work."""
    g = _problem_arrays(name, M, R)
    r_spec = _run(_plan(g), g)
    monkeypatch.setenv("MRBO_GENERIC_KERNEL", "1")
    r_gen = _run(_plan(g), g)
    assert (r_spec["status"] == 0).all() and (r_gen["status"] == 0).all()
    np.testing.assert_array_equal(r_spec["evals"], r_gen["evals"])
    for k in ("values", "obs", "policy_x"):
        np.testing.assert_allclose(r_spec[k], r_gen[k], rtol=1e-12, atol=1e-15, err_msg=k)
    for k in ("grad_x", "grad_theta"):
        _assert_grads_close(r_spec[k], r_gen[k], rtol=1e-10)


@pytest.mark.gpu
@pytest.mark.parametrize("name,M,R,ell", [("C4", 16, 2, 0.5), ("C5", 16, 2, 20.0)])
def test_cost_kernel_equals_generic(gpu, monkeypatch, name, M, R, ell):
    """Matérn-5/2 + EI + the quadratic NonUniformCost at N = 65..256 run rollout_kernel<D, RPL, 2>
    (plan info spec = 3, the rule, kernel and cost fixed at compile time); MRBO_GENERIC_KERNEL=1
    runs the generic kernel.  Same bars as the Matérn-5/2 + EI specialisation, except policy points
    to 1e-10: C4 at ℓ = 0.5 takes ≈ 500 Newton steps per trajectory under α/c, and a Newton endpoint
    carries the few-ulp differences of the two schedules amplified by the step (measured 2.3e-12)."""
    g = _problem_arrays(name, M, R, ell=ell)
    w = tuple(np.linspace(0.5, 1.5, g["X"].shape[0]))
    opts = dict(cost="quadratic", cost_c0=1.0, cost_w=w)
    p_spec = _plan(g, **opts)
    assert p_spec.info()["spec"] == 3
    r_spec = _run(p_spec, g)
    monkeypatch.setenv("MRBO_GENERIC_KERNEL", "1")
    p_gen = _plan(g, **opts)
    assert p_gen.info()["spec"] == 0
    r_gen = _run(p_gen, g)
    assert (r_spec["status"] == 0).all() and (r_gen["status"] == 0).all()
    np.testing.assert_array_equal(r_spec["evals"], r_gen["evals"])
    for k, rtol in (("values", 1e-12), ("obs", 1e-12), ("policy_x", 1e-10)):
        np.testing.assert_allclose(r_spec[k], r_gen[k], rtol=rtol, atol=1e-15, err_msg=k)
    for k in ("grad_x", "grad_theta"):
        _assert_grads_close(r_spec[k], r_gen[k], rtol=1e-10)


@pytest.mark.gpu
@pytest.mark.parametrize("name,M,R", [("C1", 32, 4), ("C2", 64, 4)])
def test_half_wave_kernel_equals_full_wave(gpu, monkeypatch, name, M, R):
    """N ≤ 32, d ≤ 4, h ≤ 3 (C1, C2) run the half-wave kernel rollout_kernel<D, 1, 1, 2> (two
    trajectories per wave, plan info spec = 2); MRBO_HALF=0 keeps the full-wave kernel.  The
    32-lane reductions sum the same terms in another order, so: identical Newton work and
    policy path, values to rtol 1e-12, gradients to 1e-10 (as spec vs generic)."""
    g = _problem_arrays(name, M, R)
    p_half = _plan(g)
    assert p_half.info()["spec"] == 2
    r_half = _run(p_half, g)
    monkeypatch.setenv("MRBO_HALF", "0")
    p_full = _plan(g)
    assert p_full.info()["spec"] == 1
    r_full = _run(p_full, g)
    assert (r_half["status"] == 0).all() and (r_full["status"] == 0).all()
    np.testing.assert_array_equal(r_half["evals"], r_full["evals"])
    for k in ("values", "obs", "policy_x"):
        np.testing.assert_allclose(r_half[k], r_full[k], rtol=1e-12, atol=1e-15, err_msg=k)
    for k in ("grad_x", "grad_theta"):
        _assert_grads_close(r_half[k], r_full[k], rtol=1e-10)


@pytest.mark.gpu
@pytest.mark.parametrize("d,N,h", [(1, 7, 1), (2, 20, 2), (3, 24, 2), (4, 32, 3)])
def test_half_wave_kernel_ragged_sizes(gpu, monkeypatch, d, N, h):
    """The half-wave kernel at ragged N (rows N..31 of each half padded), h = 1..3 on Ackley(d) at
    the design-spacing lengthscale: the same bars as the full-wave comparison (the default library
    carries the FMAX = 4 units, which hold the half-wave kernel, for d = 1..4: __graft_entry__.F4_DIMS).
    A plan with more than 32 inner starts keeps the full-wave kernel (one lane per start in a half)."""
    ell = 0.6 * 65.536 * N ** (-1.0 / d)
    g = _problem_arrays(None, 32, 2, testfn="ackley", d=d, N=N, h=h, ell=ell)
    p_half = _plan(g)
    assert p_half.info()["spec"] == 2
    r_half = _run(p_half, g)
    monkeypatch.setenv("MRBO_HALF", "0")
    r_full = _run(_plan(g), g)
    assert (r_half["status"] == 0).all() and (r_full["status"] == 0).all()
    np.testing.assert_array_equal(r_half["evals"], r_full["evals"])
    for k in ("values", "obs", "policy_x"):
        np.testing.assert_allclose(r_half[k], r_full[k], rtol=1e-12, atol=1e-15, err_msg=k)
    for k in ("grad_x", "grad_theta"):
        _assert_grads_close(r_half[k], r_full[k], rtol=1e-10)
    monkeypatch.delenv("MRBO_HALF")
    xs = np.asfortranarray(np.tile(g["xstarts"], (1, 3))[:, :33])
    assert _plan(dict(g, xstarts=xs)).info()["spec"] == 1


@pytest.mark.gpu
@pytest.mark.parametrize("name,M,R", [("C3", 32, 4), ("C4", 8, 2)])
def test_work_order_changes_nothing_but_the_schedule(gpu, name, M, R):
    """mrbo_plan_set_order only reorders the work queue: a reversed permutation and the
    longest-first schedule of a previous launch give bit-identical results and work counters;
    a wrong-length order is rejected, None restores the identity."""
    import torch
    g = _problem_arrays(name, M, R)
    plan = _plan(g)
    r_id = _run(plan, g)
    plan.set_order(torch.arange(M * R - 1, -1, -1, dtype=torch.int32, device="cuda:0"))
    r_rev = _run(plan, g)
    out = plan.alloc_outputs(with_gradient=True)
    from mrbo.engine import to_device
    plan.simulate(to_device(g["x0s"], "cuda:0"), to_device(g["rnstream"], "cuda:0"), to_device(g["xstarts"], "cuda:0"), out)
    plan.order_longest_first(out)
    r_lpt = _run(plan, g)
    for r in (r_rev, r_lpt):
        for k in r_id:
            np.testing.assert_array_equal(r_id[k], r[k], err_msg=k)
    with pytest.raises(Exception):
        plan.set_order(torch.zeros(M * R + 1, dtype=torch.int32, device="cuda:0"))
    plan.set_order(None)
    r_none = _run(plan, g)
    np.testing.assert_array_equal(r_id["values"], r_none["values"])


def test_device_sga_step_matches_host(gpu):
    """mrbo_sga_step (eswavs utils.jl:114-123 + StandardSGA optimizers.jl:16-22 on the device, as
    bench.py's outer step) against the host mirror sga_step_batch, bit for bit: both branches of
    the stop rule, an already-stopped restart untouched."""
    import torch
    from mrbo.engine import from_device, to_device
    from mrbo.utils import sga_step_batch
    g = _problem_arrays("C3", 32, 8)
    p = _plan(g)
    r = _run(p, g, want_policy=False)
    d, R = p.d, p.R
    eto = np.asfortranarray(r["eto"])
    for sample_size in (32.0, 1e-3, 1e6):     # iterate / stop everything / mixed
        x0 = np.array(g["x0s"], dtype=np.float64, order="F")
        active = np.ones(R, dtype=bool)
        active[3] = False
        dx, da = to_device(x0, "cuda:0"), torch.tensor(active.astype(np.int32), device="cuda:0")
        p.sga_step(to_device(eto, "cuda:0"), dx, da, sample_size, 0.01)
        torch.cuda.synchronize()
        sga_step_batch(x0, active, eto[2:2 + d], eto[2 + d:2 + 2 * d], sample_size, 0.01)
        np.testing.assert_array_equal(from_device(dx, (d, R)), x0)
        np.testing.assert_array_equal(da.cpu().numpy().astype(bool), active)


def test_device_adam_step_matches_host(gpu):
    """mrbo_adam_step (eswavs + Adam update!, optimizers.jl:49-74, moments kept on the device)
    against the host mirror adam_step_batch over consecutive updates, bit for bit: x, m, v and the
    active flags after every step, including steps where the stop rule retires restarts."""
    import torch
    from mrbo.engine import from_device, to_device
    from mrbo.utils import adam_step_batch
    g = _problem_arrays("C3", 32, 8)
    p = _plan(g)
    r = _run(p, g, want_policy=False)
    d, R = p.d, p.R
    eto0 = np.asfortranarray(r["eto"])
    x0 = np.array(g["x0s"], dtype=np.float64, order="F")
    m, v = np.zeros((d, R), order="F"), np.zeros((d, R), order="F")
    active = np.ones(R, dtype=bool)
    active[3] = False
    dx, dm, dv = (to_device(a, "cuda:0") for a in (x0, m, v))
    da = torch.tensor(active.astype(np.int32), device="cuda:0")
    for t, sample_size in enumerate((32.0, 1e6, 32.0, 1e-3, 32.0), start=1):
        eto = eto0.copy(order="F")
        eto[2:2 + d] *= (1.0 + 0.25 * t) * (-1.0) ** t
        p.adam_step(to_device(eto, "cuda:0"), dx, da, dm, dv, t, sample_size, eta=0.02)
        torch.cuda.synchronize()
        adam_step_batch(x0, active, m, v, t, eto[2:2 + d], eto[2 + d:2 + 2 * d], sample_size, eta=0.02)
        np.testing.assert_array_equal(da.cpu().numpy().astype(bool), active)
        np.testing.assert_array_equal(from_device(dm, (d, R)), m)
        np.testing.assert_array_equal(from_device(dv, (d, R)), v)
        np.testing.assert_array_equal(from_device(dx, (d, R)), x0)


def test_shim_call_sequence_matches_batched_launch(gpu):
    """The Julia drop-in's call sequence (mrbo.shim, the Python mirror of julia/MRBO.jl: R = 1,
    host pointers, plans from the bounded cache) against its batched method, bit for bit: every
    restart's R = 1 launch equals that restart's column of one batched launch (values, ∇x, ∇θ and
    the ETO), and the reference's outer loop (stochastic_solve, utils.jl:235-265: 50 iterations,
    eswavs, StandardSGA) driven through the R = 1 method reaches the same x0 as the batched loop,
    with every call's per-trajectory outputs equal -- on ONE plan reused for all of its calls."""
    from mrbo import configs, shim
    M, R = 256, 8
    pb = configs.problem("C3", M=M, R=R)
    T, tp, xs = pb.T, pb.tp, pb.es.get_starts()
    d = pb.x0s.shape[0]
    shim.release_plans()
    etos, vals, gx, gt = shim.simulate_trajectory_mc_batch(T, tp, pb.x0s, xs)
    assert (vals > 0).mean() > 0.25 and (np.abs(gx).max(axis=0) > 0).mean() > 0.1   # not vacuous
    n0 = shim.stats["plans_created"]
    for r in range(R):
        tp.set_starting_point(pb.x0s[:, r].copy())
        res, g, t = np.zeros(M), np.zeros((d, M), order="F"), np.zeros((1, M), order="F")
        e = shim.simulate_trajectory_mc(T, tp, xs, res, g, t)
        np.testing.assert_array_equal(res, vals[:, r])
        np.testing.assert_array_equal(g, gx[:, :, r])
        np.testing.assert_array_equal(t, gt[:, :, r])
        assert e.μxθ == etos[r].μxθ and e.σ_μxθ == etos[r].σ_μxθ
        np.testing.assert_array_equal(e.gradient(), etos[r].gradient())
    assert shim.stats["plans_created"] == n0 + 1          # one R = 1 plan served every restart
    # the outer loop: batched (all restarts per launch) vs the R = 1 sequence per restart
    x = np.array(pb.x0s, dtype=np.float64, order="F")
    active = np.ones(R, dtype=bool)
    steps = np.zeros(R, dtype=int)
    hist = []
    for _ in range(50):
        if not active.any():
            break
        es_, v_, g_, _ = shim.simulate_trajectory_mc_batch(T, tp, x, xs)
        hist.append((v_, g_))
        for r in np.flatnonzero(active):
            steps[r] += 1
            if shim.eswavs(es_[r].gradient(), es_[r].std_gradient() ** 2, M):
                active[r] = False
            else:
                x[:, r] = x[:, r] + 0.01 * es_[r].gradient()
    n1 = shim.stats["plans_created"]
    for r in range(R):
        trace = []
        xr = shim.stochastic_solve(T, tp, xs, pb.x0s[:, r], eta=0.01, trace=trace)
        np.testing.assert_array_equal(xr, x[:, r])
        assert len(trace) == steps[r]
        for k, (rv, rg) in enumerate(trace):
            np.testing.assert_array_equal(rv, hist[k][0][:, r])
            np.testing.assert_array_equal(rg, hist[k][1][:, :, r])
    assert shim.stats["plans_created"] == n1               # the cached R = 1 plan, reused
    assert steps.max() > 1                                  # the loop moved x0
    shim.release_plans()


@pytest.mark.parametrize("opt,eta", [("sga", 0.01), ("adam", 0.001)])
def test_device_stochastic_solve_equals_stepwise_device_loop(gpu, opt, eta):
    """mrbo_stochastic_solve -- MRBO.jl's device-resident stochastic_solve (utils.jl:235-265) over a
    restart batch in ONE C-ABI call -- against the stepwise device loop bench.py times
    (mrbo_simulate_mc, mrbo_eto_reduce, mrbo_sga_step / mrbo_adam_step per iteration, driven from
    Python) over the reference's full budget of 50 iterations: the final x0, the ETO rows and the
    stop flags are identical bit for bit; the host-pointer call of the Julia method (mrbo.shim)
    equals the device-pointer one on the same cached plan; and the call returns within two
    iterations of the one after which eswavs had stopped every restart."""
    import torch
    from mrbo import configs, shim
    from mrbo.engine import from_device, to_device
    M, R, budget = 256, 8, 50
    pb = configs.problem("C3", M=M, R=R)
    T, tp, xs = pb.T, pb.tp, pb.es.get_starts()
    d = pb.x0s.shape[0]
    W = 2 + 2 * d + 2
    shim.release_plans()
    plan = shim.cached_plan(T.s, tp, T.θ[0], xs.shape[1], R=R)
    dev = "cuda:0"
    drn = to_device(np.asfortranarray(tp.rnstream_sequence), dev)
    dxs = to_device(xs, dev)
    # the stepwise loop
    dx = to_device(pb.x0s, dev)
    act = torch.ones(R, dtype=torch.int32, device=dev)
    out = plan.alloc_outputs(with_gradient=True, want_evals=False)
    dm, dv = torch.zeros_like(dx), torch.zeros_like(dx)
    all_stopped = None
    for it in range(1, budget + 1):
        plan.simulate(dx, drn, dxs, out)
        e = plan.eto(out)
        if opt == "sga":
            plan.sga_step(e, dx, act, M, eta)
        else:
            plan.adam_step(e, dx, act, dm, dv, it, M, eta)
        if all_stopped is None and int(act.sum()) == 0:
            all_stopped = it
        assert int((out["status"] != 0).sum()) == 0
    x_ref, e_ref, a_ref = from_device(dx, (d, R)), e.cpu().numpy().reshape(R, W), act.cpu().numpy()
    # one call, device pointers
    dx2 = to_device(pb.x0s, dev)
    e2 = torch.full((W * R,), np.nan, dtype=torch.float64, device=dev)
    a2 = torch.full((R,), 7, dtype=torch.int32, device=dev)
    n_launch, n_stop, bits = plan.stochastic_solve(dx2, drn, dxs, optimizer=opt, iterations=budget, eta=eta,
                                                   eto=e2, active=a2)
    assert bits == 0
    np.testing.assert_array_equal(from_device(dx2, (d, R)), x_ref)
    np.testing.assert_array_equal(e2.cpu().numpy().reshape(R, W), e_ref)
    np.testing.assert_array_equal(a2.cpu().numpy(), a_ref)
    if all_stopped is None:
        assert n_launch == budget and n_stop == budget
    else:
        assert n_stop == all_stopped and n_launch <= min(budget, all_stopped + 2)
    assert not np.array_equal(x_ref, pb.x0s)                # the ascent moved x0
    # the Julia method's host-pointer call on the same cached plan
    n0 = shim.stats["plans_created"]
    X, eto_h, act_h, res = shim.stochastic_solve_batch(T, tp, xs, pb.x0s, optimizer=opt, eta=eta, iterations=budget)
    assert shim.stats["plans_created"] == n0
    np.testing.assert_array_equal(X, x_ref)
    np.testing.assert_array_equal(eto_h, e_ref)
    np.testing.assert_array_equal(act_h, a_ref)
    assert res == [n_launch, n_stop, 0]
    shim.release_plans()
