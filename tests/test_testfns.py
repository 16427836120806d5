"""The build's test functions (mrbo/testfns.py, testfns.jl) against values the reference itself
computed: tests/golden/testfn_ref.json holds (x, y) pairs from the reference's archived
experiment observation files (tests/golden/make_testfn_ref.py), y = testfn.f(x) evaluated by
testfns.jl.  These objectives generate the synthetic base data of every BASELINE configuration
(Gramacy–Lee C1, Branin C2, Hartmann-6 C3/C4, Ackley-8 C5), so the pin covers the path's inputs.
Every recorded x lies in the build's box; f(x) agrees to 1e-13 relative (Julia and NumPy round
the same expressions differently at ~1e-15; Rosenbrock's cancellations reach 1.1e-14)."""
import json
import os

import numpy as np
import pytest

from conftest import ROOT

REF = os.path.join(ROOT, "tests", "golden", "testfn_ref.json")


def _fn(key):
    from mrbo import bayesopt, testfns
    if key in ("ackley8d", "ackley16d"):
        return testfns.TestAckley(int(key[6:-1]))
    return bayesopt.TESTFNS[key]()


def _cases():
    with open(REF) as f:
        return json.load(f)


@pytest.mark.parametrize("key", sorted(_cases()))
def test_testfn_matches_reference_evaluations(key):
    case = _cases()[key]
    tf = _fn(key)
    X = np.array([p["x"] for p in case["pairs"]], dtype=np.float64).T
    y = np.array([p["y"] for p in case["pairs"]], dtype=np.float64)
    assert X.shape == (case["d"], len(y)) and tf.dim == case["d"] and len(y) >= 40
    lbs, ubs = tf.get_bounds()
    assert np.all((X >= lbs[:, None]) & (X <= ubs[:, None]))
    f = np.array([tf.f(X[:, j]) for j in range(X.shape[1])])
    np.testing.assert_allclose(f, y, rtol=1e-13, atol=1e-13)
    np.testing.assert_allclose(tf(X), y, rtol=1e-13, atol=1e-13)   # the batched call (columns)
