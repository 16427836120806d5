"""Synthetic objectives (testfns.jl) used to make base observations for the configs."""
import numpy as np


class TestFunction:
    """testfns.jl:5-11"""

    def __init__(self, dim, bounds, xopt, f, grad=None, name=""):
        self.dim = dim
        self.bounds = np.asarray(bounds, dtype=np.float64)
        self.xopt = xopt
        self.f = f
        self.grad = grad
        self.name = name

    def __call__(self, X):
        X = np.asarray(X, dtype=np.float64)
        if X.ndim == 1:
            return self.f(X)
        return np.array([self.f(X[:, j]) for j in range(X.shape[1])])

    def get_bounds(self):
        return self.bounds[:, 0].copy(), self.bounds[:, 1].copy()


def TestGramacyLee():
    """testfns.jl:227-235"""
    f = lambda x: np.sin(10 * np.pi * x[0]) / (2 * x[0]) + (x[0] - 1.0) ** 4
    return TestFunction(1, [[0.5, 2.5]], ([0.548563],), f, name="gramacylee")


def TestBraninHoo(a=1, b=5.1 / (4 * np.pi ** 2), c=5 / np.pi, r=6, s=10, t=1 / (8 * np.pi)):
    """testfns.jl:136-152"""
    f = lambda xy: a * (xy[1] - b * xy[0] ** 2 + c * xy[0] - r) ** 2 + s * (1 - t) * np.cos(xy[0]) + s
    return TestFunction(2, [[-5.0, 10.0], [0.0, 15.0]], ([-np.pi, 12.275], [np.pi, 2.275], [9.42478, 2.475]), f,
                        name="braninhoo")


_H6_ALPHA = np.array([1.0, 1.2, 3.0, 3.2])
_H6_A = np.array([[10, 3, 17, 3.5, 1.7, 8], [0.05, 10, 17, 0.1, 8, 14], [3, 3.5, 1.7, 10, 17, 8],
                  [17, 8, 0.05, 10, 0.1, 14]])
_H6_P = 1e-4 * np.array([[1312, 1696, 5569, 124, 8283, 5886], [2329, 4135, 8307, 3736, 1004, 9991],
                         [2348, 1451, 3522, 2883, 3047, 6650], [4047, 8828, 8732, 5743, 1091, 381]])


def TestHartmann6D():
    """testfns.jl:532-565"""
    def f(x):
        x = np.asarray(x)
        return -float(np.sum(_H6_ALPHA * np.exp(-np.sum(_H6_A * (x - _H6_P) ** 2, axis=1))))
    return TestFunction(6, [[0.0, 1.0]] * 6, ([0.20169, 0.150011, 0.476874, 0.275332, 0.311652, 0.6573],), f,
                        name="hartmann6d")


def TestAckley(d, a=20.0, b=0.2, c=2 * np.pi):
    """testfns.jl:173-199"""
    def f(x):
        x = np.asarray(x)
        return -a * np.exp(-b / np.sqrt(d) * np.linalg.norm(x)) - np.exp(np.sum(np.cos(c * x)) / d) + a + np.exp(1)
    return TestFunction(d, [[-32.768, 32.768]] * d, (np.zeros(d),), f, name=f"ackley{d}d")


def TestRosenbrock():
    f = lambda xy: (1 - xy[0]) ** 2 + 100 * (xy[1] - xy[0] ** 2) ** 2
    return TestFunction(2, [[-2.0, 2.0], [-1.0, 3.0]], (np.ones(2),), f, name="rosenbrock")


def TestRastrigin(n):
    f = lambda x: 10 * n + float(np.sum(np.asarray(x) ** 2 - 10 * np.cos(2 * np.pi * np.asarray(x))))
    return TestFunction(n, [[-5.12, 5.12]] * n, (np.zeros(n),), f, name=f"rastrigin{n}d")
