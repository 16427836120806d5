"""mrbo_base_solve -- base_solve / multistart_base_solve! on the base surrogate (rbf_optim.jl:35-135),
the acquisition step of the reference's myopic experiments (experiments/myopic_bayesopt.jl:224-233),
against the oracle's rbo_base_solve (the same projected Newton).

Per start (66 = generate_initial_guesses(64, …), the myopic driver's default): the minimiser within
1e-9·(1 + |x|) and the minimum within 1e-9 relative for every start whose two solves follow the
same path; a start may end on x_tol one rounding-level step apart (drift, bounded by x_tol) on at
most 5 % of the starts; work per counter in total within 1 % (tests/parity.py T3).  The chosen
candidate (findmin after the NaN filter) is the same start on both sides.
"""
import numpy as np
import pytest

from parity import _osur, _plan, _problem_arrays

pytestmark = pytest.mark.gpu

CASES = [("C2", None, "EI", 0.0), ("C3", None, "EI", 0.0), ("C3", 0.5, "EI", 0.0), ("C4", 0.5, "EI", 0.0),
         ("C3", None, "POI", 0.0), ("C2", None, "LCB", 2.0), ("C5", 20.0, "EI", 0.0)]


@pytest.mark.parametrize("name,ell,rule,theta", CASES)
def test_base_solve_vs_oracle(gpu, oracle, name, ell, rule, theta):
    import torch
    from mrbo import _lib
    from mrbo.engine import from_device, to_device
    from mrbo.rbf_optim import findmin_candidates
    from mrbo.utils import generate_initial_guesses
    g = _problem_arrays(name, 4, 1, ell=ell)
    d = g["X"].shape[0]
    xs = generate_initial_guesses(64, g["lbs"], g["ubs"])
    n = xs.shape[1]
    assert n == 66
    rid = {"EI": 0, "POI": 1, "LCB": 2}[rule]
    p = _plan(g, h=0, M=1, R=1, nstarts=1, rule=rid, theta=theta)
    dev = "cuda:0"
    xmin = torch.empty(d * n, dtype=torch.float64, device=dev)
    fmin = torch.empty(n, dtype=torch.float64, device=dev)
    st = torch.empty(n, dtype=torch.int32, device=dev)
    ev = torch.empty(_lib.NCOUNTERS * n, dtype=torch.int64, device=dev)
    dxs = to_device(xs, dev)
    import ctypes
    pp = lambda t: ctypes.c_void_p(t.data_ptr())
    _lib.check(p.lib.mrbo_base_solve(p.handle, n, pp(dxs), pp(xmin), pp(fmin), pp(st), pp(ev), 0,
                                     ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)))
    torch.cuda.synchronize()
    xg, fg = from_device(xmin, (d, n)), from_device(fmin, (n,))
    sg, eg = from_device(st, (n,)), from_device(ev, (_lib.NCOUNTERS, n))[:3]
    xo, fo, so, eo = oracle.base_solve(_osur(oracle, g), xs, g["lbs"], g["ubs"], theta=theta, rule=rule)
    assert (sg == 0).all() and (so == 0).all()
    dx = (np.abs(xg - xo) / (1 + np.abs(xo))).max(axis=0)
    same = dx <= 1e-9
    assert (dx[~same] <= 2e-3).all(), dx          # drift ends within x_tol of each other
    assert same.mean() >= 0.95, dx
    np.testing.assert_allclose(fg[same], fo[same], rtol=1e-9, atol=1e-300)
    assert eg[0].sum() > 0 and eg[2].sum() > 0   # the Newton solve did gradient and Hessian work
    np.testing.assert_allclose(eg[:, same].sum(1), eo[:, same].sum(1), rtol=0.01)
    assert findmin_candidates(xg, fg) == findmin_candidates(xo, fo)
    # the host mirror: multistart_base_solve! picks that candidate
    kg = findmin_candidates(xg, fg)
    assert np.isfinite(fg[kg]) and fg[kg] <= np.nanmin(fo) + 1e-9 * abs(np.nanmin(fo)) + 1e-300


def test_multistart_base_solve_mirror(gpu):
    """multistart_base_solve!(s, xfinal; …) through the host mirror on a Surrogate: xfinal is the best
    start's minimiser, inside the box, and no worse than every start point's own −α."""
    from mrbo import testfns
    from mrbo.decision_rules import EI
    from mrbo.kernels import Matern52
    from mrbo.rbf_optim import base_solve_batch, multistart_base_solve
    from mrbo.rollout import evaluate_base
    from mrbo.surrogates import Surrogate
    from mrbo.utils import generate_initial_guesses
    tf = testfns.TestBraninHoo()
    lbs, ubs = tf.get_bounds()
    rng = np.random.default_rng(7)
    X = lbs[:, None] + (ubs - lbs)[:, None] * rng.random((2, 6))
    s = Surrogate(Matern52(), X, tf(X), capacity=20, decision_rule=EI())
    guesses = generate_initial_guesses(64, lbs, ubs)
    x = np.zeros(2)
    assert multistart_base_solve(s, x, lbs, ubs, guesses, [0.0]) is None
    assert np.all(x >= lbs) and np.all(x <= ubs)
    xs, fs, ev = base_solve_batch(s, lbs, ubs, guesses, [0.0])
    a_best = evaluate_base(s, x.reshape(-1, 1), [0.0])[0].αxθ
    a_starts = np.array([e.αxθ for e in evaluate_base(s, np.clip(guesses, lbs[:, None], ubs[:, None]), [0.0])])
    assert a_best >= a_starts.max() - 1e-12
    assert np.isclose(-a_best, np.nanmin(fs), rtol=1e-12, atol=1e-300)
