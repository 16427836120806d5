"""CPU tests of the host side: the reference-API mirror (mrbo package), the C-ABI library's
exports and host helpers, and the multi-GPU reduction logic (no GPU compute here)."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import GOLDEN_CASES, ROOT, load_golden


def test_library_exports_every_header_symbol():
    """libmrbo.so loads without a GPU and exports every entry point include/mrbo.h declares."""
    from mrbo import _lib
    hdr = open(os.path.join(ROOT, "include", "mrbo.h")).read()
    declared = sorted(set(re.findall(r"\b(mrbo_[a-z_]+)\s*\(", hdr)))
    assert set(declared) == set(_lib.EXPORTS), (declared, _lib.EXPORTS)
    L = _lib.load()
    for sym in declared:
        assert hasattr(L, sym), sym
    assert b"gfx950" in L.mrbo_version()


@pytest.mark.parametrize("case", GOLDEN_CASES)
def test_library_rnstream_matches_golden_and_oracle(oracle, case):
    from mrbo.engine import initial_guesses, rnstream
    g = load_golden(case)
    M, D1, H = g["rnstream"].shape
    rn = rnstream(M, D1 - 1, H)
    np.testing.assert_allclose(rn, g["rnstream"], rtol=1e-15, atol=1e-15)
    np.testing.assert_array_equal(rn, oracle.gen_low_discrepancy_sequence(M, D1 - 1, H))
    np.testing.assert_array_equal(initial_guesses(16, g["lbs"], g["ubs"]),
                                  oracle.generate_initial_guesses(16, g["lbs"], g["ubs"]))


def test_library_dual_uniform_bit_identical_to_oracle(oracle):
    from mrbo.engine import dual_uniform
    for t, j, k in [(0, 1, 0), (12345, 3, 5), (2 ** 31 + 7, 5, 7)]:
        assert dual_uniform(1906, t, j, k) == oracle.dual_uniform(1906, t, j, k)


@pytest.mark.parametrize("d,N,msg", [(17, 4, b"d=17"), (9, 129, b"N=129"), (4, 513, b"N=513")])
def test_plan_create_rejects_unsupported_shapes(d, N, msg):
    """Argument errors come back as negative codes with a message (no exception inside C), before
    any device call: d ≤ 16, N ≤ 512, and N ≤ 128 when d > 8 are compiled."""
    from mrbo import _lib
    L = _lib.load()
    dp = ctypes.POINTER(ctypes.c_double)
    X = np.zeros((d, N), order="F")
    Lm = np.eye(N, order="F")
    c = np.zeros(N)
    sd = _lib.SurrogateDesc(d, N, 0, 1.0, 1e-6, 0.0, X.ctypes.data_as(dp), Lm.ctypes.data_as(dp), N,
                            c.ctypes.data_as(dp), c.ctypes.data_as(dp))
    lb = np.zeros(d)
    pd = _lib.ParamsDesc(3, 8, 2, 18, 0, 0.0, lb.ctypes.data_as(dp), lb.ctypes.data_as(dp), 50, 20, 1e-3, 1e-3,
                         1e-8, 1e-4, 1e-8, 1906, 0, 0)
    h = ctypes.c_void_p()
    rc = L.mrbo_plan_create(ctypes.byref(sd), ctypes.byref(pd), 0, ctypes.byref(h))
    assert rc == -2 and msg in L.mrbo_last_error()


@pytest.mark.parametrize("kind,c0,w,ub,msg", [
    (1, 0.0, 1.0, 1.0, b"cost_c0"), (2, -1.0, 1.0, 1.0, b"cost_c0"), (1, float("nan"), 1.0, 1.0, b"cost_c0"),
    (1, 1.0, -0.5, 1.0, b"quadratic cost weight"), (2, 1.0, float("inf"), 1.0, b"not finite"),
    (1, 1.0, 1.0, 0.0, b"ub > lb")])
def test_plan_create_rejects_non_positive_cost_models(kind, c0, w, ub, msg):
    """NonUniformCost models that are not positive on the box (c0 ≤ 0, negative quadratic weights,
    non-finite parameters, ub ≤ lb) are refused with MRBO_ERR_ARG before any device call: α/c and
    the gradient certificates' bound·(1/c) would flip sign and could certify a non-stationary point."""
    from mrbo import _lib
    L = _lib.load()
    dp = ctypes.POINTER(ctypes.c_double)
    d, N = 2, 4
    X = np.zeros((d, N), order="F")
    Lm = np.eye(N, order="F")
    c = np.zeros(N)
    sd = _lib.SurrogateDesc(d, N, 0, 1.0, 1e-6, 0.0, X.ctypes.data_as(dp), Lm.ctypes.data_as(dp), N,
                            c.ctypes.data_as(dp), c.ctypes.data_as(dp))
    lb, ubs, cw = np.zeros(d), np.full(d, ub), np.full(d, w)
    pd = _lib.ParamsDesc(2, 8, 2, 18, 0, 0.0, lb.ctypes.data_as(dp), ubs.ctypes.data_as(dp), 50, 20, 1e-3, 1e-3,
                         1e-8, 1e-4, 1e-8, 1906, 0, 0, kind, c0, cw.ctypes.data_as(dp))
    h = ctypes.c_void_p()
    rc = L.mrbo_plan_create(ctypes.byref(sd), ctypes.byref(pd), 0, ctypes.byref(h))
    assert rc == -1 and msg in L.mrbo_last_error(), (rc, L.mrbo_last_error())


def test_kronecker_matches_oracle(oracle):
    from mrbo.utils import kronecker_quasirand
    for d, N, s in [(1, 8, 0), (2, 32, 0), (6, 64, 64), (8, 16, 3)]:
        np.testing.assert_allclose(kronecker_quasirand(d, N, s), oracle.kronecker_quasirand(d, N, s), rtol=0,
                                   atol=1e-15)


def test_surrogate_fit_and_condition_match_dense_refit():
    """Surrogate ctor (r_b_s.jl:77-118) and condition! (:214-222) vs a dense re-fit."""
    from mrbo import EI, Matern52, Surrogate
    from mrbo.kernels import eval_KXX
    rng = np.random.default_rng(0)
    X = rng.uniform(size=(3, 10))
    y = rng.normal(size=10)
    s = Surrogate(Matern52(), X, y, capacity=16, decision_rule=EI(), σn2=1e-6)
    x, yn = rng.uniform(size=3), 0.3
    s.condition(x, yn)
    X2, y2 = np.column_stack([X, x]), np.append(y, yn)
    K = eval_KXX(Matern52(), X2, σn2=1e-6)
    np.testing.assert_allclose(s.get_active_cholesky() @ s.get_active_cholesky().T, K, atol=1e-12)
    np.testing.assert_allclose(s.get_active_coefficients(), np.linalg.solve(K, y2), rtol=1e-8, atol=1e-10)
    assert s.fmini() == min(0.0, y2.min())  # Q3: zero padding of the capacity buffer


def test_surrogate_reuse_semantics_of_the_experiment_loops():
    """What experiments/*_bayesopt.jl rely on when they reuse one surrogate: reset!(s, X, y)
    (r_b_s.jl:147-164) refits with the CURRENT kernel and keeps the buffers past N; condition! on a
    full surrogate (:214-222) rebinds a local `s = resize(s)` (:137-145), so the caller's surrogate
    is unchanged and only the returned copy holds the new point."""
    from mrbo import EI, Matern52, Surrogate
    from mrbo.kernels import set_hyperparameters
    rng = np.random.default_rng(1)
    s = Surrogate(Matern52(), np.zeros((2, 1)), np.zeros(1), capacity=6, decision_rule=EI(), σn2=1e-6)
    X, y = rng.uniform(size=(2, 4)), rng.normal(size=4) + 5.0
    s.reset(X, y)
    s.condition(rng.uniform(size=2), -3.0)
    s.set_kernel(set_hyperparameters(s.ψ, np.array([0.4])))           # what optimize! leaves
    X2, y2 = rng.uniform(size=(2, 3)), rng.normal(size=3) + 5.0
    s.reset(X2, y2)
    assert s.ψ.lengthscale == 0.4 and s.observed == 3
    assert s.y[4] == -3.0 and s.fmini() == -3.0                         # stale tail seen by Q3
    s.condition(rng.uniform(size=2), 1.0)
    s.condition(rng.uniform(size=2), 2.0)
    s.condition(rng.uniform(size=2), 3.0)
    assert s.observed == 6 == s.capacity
    before = (s.X.copy(), s.y.copy(), s.L.copy(), s.c.copy())
    r = s.condition(rng.uniform(size=2), 4.0)
    assert r is not s and r.capacity == 12 and r.observed == 7 and r.y[6] == 4.0
    for a, b in zip(before, (s.X, s.y, s.L, s.c)):
        np.testing.assert_array_equal(a, b)


def test_reference_myopic_runs_show_the_carried_lengthscale():
    """The evidence behind the myopic loop's reuse_surrogate default: in the
    reference's recorded Ackley-5 runs (tests/golden/bo_ref_gaps.json, from
    experiments/myopic/ackley5d/*_gaps.csv) the first trial -- the only one that starts from
    Matern52()'s ℓ = 1 -- observes the box centre (Ackley's minimiser, the first Sobol start) at
    once, as the round-3 loop did in every trial, while the later trials, which start from the
    previous trial's optimised lengthscale, mostly do not."""
    import json
    ref = json.load(open(os.path.join(ROOT, "tests", "golden", "bo_ref_gaps.json")))
    g = np.array(ref["myopic_ackley5d_ei"]["gaps"])
    assert ref["myopic_ackley5d_ei"]["budget_labels"][1] == "2"
    assert g[0, 1] == 1.0 and g[0, 29] == 1.0
    assert g[1:, 29].mean() < 0.2 and (g[1:, 1] == 1.0).mean() < 0.1


def test_trajectory_parameters_contract():
    from mrbo import TrajectoryParameters
    tp = TrajectoryParameters(start=[0.1, 0.2], hypers=[0.0], horizon=2, mc_iterations=8,
                              use_low_discrepancy_sequence=True, spatial_lowerbounds=[0, 0], spatial_upperbounds=[1, 1])
    assert tp.rnstream_sequence.shape == (8, 3, 3)
    with pytest.raises(AssertionError):
        TrajectoryParameters(start=[0.1], hypers=[0.0], horizon=2, mc_iterations=8, use_low_discrepancy_sequence=True,
                             spatial_lowerbounds=[0, 0], spatial_upperbounds=[1, 1])


def _moments_data(rng, M, R, d, mean, spread):
    v = rng.normal(mean, spread, size=(M, R))
    gx = mean * 1e-3 + rng.normal(size=(d, M, R)) * spread * 1e-3
    gt = mean + rng.normal(size=(M, R)) * spread
    return v, gx, gt


@pytest.mark.parametrize("mean,spread", [(0.2, 0.1), (1e6, 1.0), (1e8, 1e-3)])
def test_moments_merge_equals_two_pass(mean, spread):
    """Chan merge of per-shard (Σ, M2) == the two-pass mean / std(n-1) of rollout.jl:328-337, also
    where a one-pass Σx² − (Σx)²/n cancels catastrophically (mean/std ≈ 1e6 … 1e11)."""
    from mrbo.parallel import eto_from_moments, local_moments, merge_moments, shard
    rng = np.random.default_rng(3)
    M, R, d = 1000, 3, 2
    v, gx, gt = _moments_data(rng, M, R, d, mean, spread)
    want_mu, want_sd = v.mean(0), v.std(0, ddof=1)
    # both sides round x − x̄ at ~eps·|x|: agreement to ~eps·mean/spread is the two-pass bound
    tol = max(1e-10, 100 * np.finfo(float).eps * mean / spread)
    if mean / spread >= 1e9:   # the one-pass form this replaced loses all digits here
        s1, s2 = v.sum(0), (v ** 2).sum(0)
        one_pass = np.sqrt(np.maximum((s2 - s1 * (s1 / M)) / (M - 1), 0.0))
        assert np.max(np.abs(one_pass / want_sd - 1)) > 1e-3
    for world in (1, 2, 3, 8):
        parts = []
        for k in range(world):
            lo, hi = shard(M, world, k)
            parts.append((hi - lo, local_moments(v[lo:hi], gx[:, lo:hi], gt[lo:hi])))
        n, merged = merge_moments(parts, d)
        assert n == M
        e = eto_from_moments(merged, M, d)
        np.testing.assert_allclose(e[0], want_mu, rtol=1e-14)
        np.testing.assert_allclose(e[1], want_sd, rtol=tol)
        np.testing.assert_allclose(e[2:2 + d], gx.mean(1), rtol=1e-12)
        np.testing.assert_allclose(e[2 + d:2 + 2 * d], gx.std(1, ddof=1), rtol=tol)
        np.testing.assert_allclose(e[2 + 2 * d], gt.mean(0), rtol=1e-14)
        np.testing.assert_allclose(e[3 + 2 * d], gt.std(0, ddof=1), rtol=tol)
        assert (e[1] > 0).all()


def test_moments_single_sample_and_empty_shard():
    """M = 1: std(n-1) is NaN (Q14); a rank with no samples contributes nothing."""
    from mrbo.parallel import eto_from_moments, local_moments, merge_moments
    v, gx, gt = np.array([[2.0]]), np.ones((2, 1, 1)), np.array([[3.0]])
    n, m = merge_moments([(1, local_moments(v, gx, gt)), (0, np.zeros((8, 1)))], 2)
    e = eto_from_moments(m, n, 2)
    assert n == 1 and e[0, 0] == 2.0 and np.isnan(e[1, 0])


def test_shard_partition():
    from mrbo.parallel import shard
    for M, W in [(1024, 1), (1024, 8), (1000, 3), (5, 8)]:
        parts = [shard(M, W, r) for r in range(W)]
        assert parts[0][0] == 0 and parts[-1][1] == M
        assert all(parts[i][1] == parts[i + 1][0] for i in range(W - 1))


def test_eswavs_and_optimizers():
    from mrbo import Adam, StandardSGA, eswavs
    assert eswavs(np.array([1e-6, 1e-6]), np.array([1.0, 1.0]), 16)        # noise dominates: stop
    assert not eswavs(np.array([1.0, 1.0]), np.array([1e-3, 1e-3]), 16)    # clear signal: keep going
    assert not eswavs(np.zeros(2), np.zeros(2), 16)                         # 0/0 -> NaN -> continue
    x = np.zeros(2)
    StandardSGA(η=0.5).update(x, np.array([1.0, -2.0]))
    np.testing.assert_allclose(x, [0.5, -1.0])
    a, x = Adam(η=0.1), np.zeros(2)
    a.update(x, np.array([1.0, -1.0]))
    np.testing.assert_allclose(x, [0.1, -0.1], rtol=1e-6)


def test_flop_model_batched_starts():
    """flops.launch_flops: the h·nstarts batched start values per trajectory are charged at the
    batched pass's cost plus the start tables (once per workgroup for the square layout, once per
    launch for the packed ones), not as full value evaluations."""
    from mrbo import flops
    N, d, h, ns, M = 64, 6, 3, 18, 10
    ev = np.zeros((flops.NCOUNTERS, M))
    ev[1] = h * ns + 5          # 54 batched + 5 line-search values per trajectory
    ev[0], ev[2] = 4, 4
    plain = flops.launch_flops(ev, N, d, h)
    nf = (1 + h) / 2.0
    sq = dict(rpl=1, blocks=256, batch=1)
    got = flops.launch_flops(ev, N, d, h, info=sq, nstarts=ns)
    nb = h * ns * M
    want = plain - nb * flops.f_value(N, nf, d) + nb * flops.f_batch_start(N, nf, d) + 256 * ns * flops.f_start_table(N, d)
    assert got == pytest.approx(want, rel=1e-12)
    packed = flops.launch_flops(ev, N, d, h, info=dict(rpl=2, blocks=256, batch=1), nstarts=ns)
    assert packed == pytest.approx(want - 255 * ns * flops.f_start_table(N, d), rel=1e-12)
    assert flops.launch_flops(ev, N, d, h, info=dict(rpl=1, blocks=256, batch=0), nstarts=ns) == plain
    assert flops.f_batch_start(N, nf, d) < flops.f_value(N, nf, d) / 5


def test_sga_step_batch_equals_per_restart_rules():
    """bench.py's vectorised outer step == eswavs + StandardSGA.update! per restart (no clip: the
    reference's update! has none, optimizers.jl:16-22); clip=True adds the build-defined box clip."""
    from mrbo.optimizers import StandardSGA
    from mrbo.utils import eswavs, sga_step_batch
    rng = np.random.default_rng(0)
    d, R, M = 6, 64, 1024
    lbs, ubs = np.zeros(d), np.ones(d)
    for trial in range(30):
        clip = trial % 2 == 1
        g = rng.standard_normal((d, R)) * rng.choice([1e-3, 1.0, 1e3])
        sd = np.abs(rng.standard_normal((d, R))) * rng.choice([1e-3, 1.0, 1e3])
        sd[:, rng.integers(0, R, 3)] = 0.0
        g[0, rng.integers(0, R, 2)] = np.nan
        x = rng.random((d, R))
        act = rng.random(R) > 0.2
        x1, a1 = x.copy(), act.copy()
        for r in range(R):
            if not a1[r]:
                continue
            if eswavs(g[:, r], sd[:, r] ** 2, M):
                a1[r] = False
                continue
            StandardSGA(0.01).update(x1[:, r], g[:, r])
            if clip:
                np.clip(x1[:, r], lbs, ubs, out=x1[:, r])
        x2, a2 = sga_step_batch(x.copy(), act.copy(), g, sd, M, 0.01, lbs, ubs, clip=clip)
        assert (a1 == a2).all()
        np.testing.assert_array_equal(x1, x2)


def test_adam_step_batch_equals_per_restart_rules():
    """The vectorised Adam outer step == eswavs + Adam.update! per restart (optimizers.jl:49-74)
    over consecutive steps: one optimizer per restart, a stopped restart never updates again."""
    from mrbo.optimizers import Adam
    from mrbo.utils import adam_step_batch, eswavs
    rng = np.random.default_rng(1)
    d, R, M = 5, 48, 1024
    x = rng.random((d, R))
    act = rng.random(R) > 0.1
    x1, a1, opts = x.copy(), act.copy(), [Adam(η=0.05) for _ in range(R)]
    x2, a2, m, v = x.copy(), act.copy(), np.zeros((d, R)), np.zeros((d, R))
    for t in range(1, 8):
        g = rng.standard_normal((d, R)) * rng.choice([1e-3, 1.0, 1e3])
        sd = np.abs(rng.standard_normal((d, R))) * rng.choice([1e-2, 1.0, 30.0])
        g[0, rng.integers(0, R, 1)] = np.nan
        for r in range(R):
            if not a1[r]:
                continue
            if eswavs(g[:, r], sd[:, r] ** 2, M):
                a1[r] = False
                continue
            opts[r].update(x1[:, r], g[:, r])
        adam_step_batch(x2, a2, m, v, t, g, sd, M, eta=0.05)
        assert (a1 == a2).all()
        np.testing.assert_array_equal(x1, x2)
        for r in np.flatnonzero(a1):
            assert opts[r].t == t
            np.testing.assert_array_equal(opts[r].m[-1], m[:, r])
            np.testing.assert_array_equal(opts[r].v[-1], v[:, r])


def test_tight_value_check_has_teeth():
    """tests/parity.py's tight value check (rel 1e-9, absolute floor 1e-12·max|v|)
    flags a per-trajectory error 1000× the measured C3 one, which the first-order bound vb alone
    (~1e5× above the measured errors) would let through."""
    import numpy as np
    from parity import tight_value_stats, value_bound_stats
    rng = np.random.default_rng(0)
    v = rng.uniform(1e-4, 1.0, 4096)
    err = 5e-14 * np.ones_like(v)                  # the C3 launch's largest replay error (abs)
    vb = 3e-9 * np.ones_like(v)                    # the order of the C3 bounds
    assert tight_value_stats(err, v, v.max())["over_tight"] == 0
    worse = 1000 * err
    assert value_bound_stats(worse, vb)["over_bound"] == 0      # the bound alone misses it
    assert tight_value_stats(worse, v, v.max())["over_tight"] > 0


def test_shim_plan_key_tracks_the_surrogate_data():
    """mrbo.shim's plan cache key mirrors MRBO.jl's mrbo_plan_key: besides the surrogate's identity
    it hashes the active covariates, observations and Cholesky factor (CPython reuses id() once a
    surrogate is freed, so identity + version alone could hand a new surrogate a stale plan)."""
    from mrbo import configs, shim
    pb = configs.problem("C2", M=8, R=2)
    s, tp = pb.surrogate, pb.tp
    k0 = shim._key(s, tp, 0.0, 18, 0, 8, 2)
    assert shim._key(s, tp, 0.0, 18, 0, 8, 2) == k0
    n = s.observed
    for arr, idx in ((s.X, (0, n - 1)), (s.y, (n - 1,)), (s.L, (n - 1, n - 1))):
        old = arr[idx]
        arr[idx] = old + 1e-3        # same id, version and observation count: other data
        assert shim._key(s, tp, 0.0, 18, 0, 8, 2) != k0
        arr[idx] = old
    assert shim._key(s, tp, 0.0, 18, 0, 8, 2) == k0


def test_bench_kernel_label_names_the_profiled_kernel():
    """bench.py's roofline.kernel is the rollout kernel's name as rocprofv3 prints it, per plan spec
    (0 generic, 1 Matérn-5/2 + EI, 2 the half-wave kernel, 3 the cost kernel) and kernel unit."""
    import bench
    assert bench.kernel_label(6, dict(rpl=1, spec=1, fmax=4)) == "mrbo::fmax4::rollout_kernel<6, 1, 1, 1>"
    assert bench.kernel_label(2, dict(rpl=1, spec=2, fmax=4)) == "mrbo::fmax4::rollout_kernel<2, 1, 1, 2>"
    assert bench.kernel_label(8, dict(rpl=4, spec=3, fmax=6)) == "mrbo::fmax6::rollout_kernel<8, 4, 2, 1>"
    assert bench.kernel_label(6, dict(rpl=2, spec=0, fmax=6)) == "mrbo::fmax6::rollout_kernel<6, 2, 0, 1>"
    # the committed rocprof summary of the headline names that kernel
    import csv
    rows = list(csv.DictReader(open(os.path.join(ROOT, "profiles", "r05", "kernel_stats_c3_r5l.csv"))))
    assert any(bench.kernel_label(6, dict(rpl=1, spec=1, fmax=4)) in r["Name"] for r in rows)


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="hipcc needed")
def test_every_kernel_unit_matches_the_kparams_layout(tmp_path):
    """Each kernel unit's KernelSet carries sizeof(KParams) from its own compile; mrbo_plan_create
    refuses a mismatch at run time (a unit left stale by an edit during a long build once read every
    launch parameter at a shifted offset).  This checks every unit of the built library on the CPU."""
    import subprocess
    src = os.path.join(ROOT, "tests", "kparams_layout_check.cpp")
    csrc = os.path.join(ROOT, "rollout-bayesian-optimization_amd", "csrc")
    libdir = os.path.join(ROOT, "rollout-bayesian-optimization_amd", "mrbo")
    obj, exe = str(tmp_path / "k.o"), str(tmp_path / "k")
    hipcc = "/opt/rocm/bin/hipcc"
    subprocess.check_call([hipcc, "--offload-arch=gfx950", "-std=c++17", f"-I{csrc}", "-c", src, "-o", obj])
    subprocess.check_call([hipcc, "--offload-arch=gfx950", obj, "-o", exe, f"-L{libdir}", "-l:libmrbo.so",
                           f"-Wl,-rpath,{libdir}"])
    out = subprocess.run([exe], capture_output=True, text=True)
    assert out.returncode == 0 and " 0 mismatched" in out.stdout, out.stdout + out.stderr


@pytest.mark.parametrize("T", [1, 7, 8, 19, 4096, 65536 + 5])
def test_longest_first_stays_within_the_xcd_chunks(T):
    """The longest-first order (mrbo_plan_order_longest_first's mirror) re-orders each per-XCD queue
    chunk [x·T/8, (x+1)·T/8) over its OWN trajectories: a permutation, every chunk's positions hold
    exactly the trajectories of its index range (so each XCD writes one contiguous range of output
    rows), longest first, ties in index order."""
    import torch
    from mrbo.engine import XCD_QUEUES, longest_first_within_chunks
    g = torch.Generator().manual_seed(T)
    work = torch.randint(0, 50, (T,), generator=g)
    order = longest_first_within_chunks(work).to(torch.int64)
    assert torch.equal(torch.sort(order).values, torch.arange(T))
    lo = [x * T // XCD_QUEUES for x in range(XCD_QUEUES + 1)]
    for x in range(XCD_QUEUES):
        seg = order[lo[x]:lo[x + 1]]
        assert torch.equal(torch.sort(seg).values, torch.arange(lo[x], lo[x + 1]))
        w = work[seg]
        assert (w[:-1] >= w[1:]).all()
        ties = (w[:-1] == w[1:])
        assert (seg[:-1][ties] < seg[1:][ties]).all()
