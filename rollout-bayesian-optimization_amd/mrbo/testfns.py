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


def TestHartmann3D():
    """testfns.jl:460-494"""
    alpha = np.array([1.0, 1.2, 3.0, 3.2])
    A = np.array([[3.0, 10, 30], [0.1, 10, 35], [3.0, 10, 30], [0.1, 10, 35]])
    P = 1e-4 * np.array([[3689, 1170, 2673], [4699, 4387, 7470], [1091, 8732, 5547], [381, 5743, 8828]])

    def f(x):
        x = np.asarray(x)
        return -float(np.sum(alpha * np.exp(-np.sum(A * (x - P) ** 2, axis=1))))
    return TestFunction(3, [[0.0, 1.0]] * 3, ([0.114614, 0.555649, 0.852547],), f, name="hartmann3d")


def TestSixHump():
    """testfns.jl:202-225 (six-hump camel)"""
    def f(xy):
        x, y = xy[0], xy[1]
        return (4.0 - 2.1 * x ** 2 + x ** 4 / 3) * x ** 2 + x * y + (-4.0 + 4.0 * y ** 2) * y ** 2
    return TestFunction(2, [[-3.0, 3.0], [-2.0, 2.0]], ([0.089842, -0.712656], [-0.089842, 0.712656]), f,
                        name="sixhump")


def TestGoldsteinPrice():
    """testfns.jl:238-278"""
    def f(xy):
        x1, x2 = xy[0], xy[1]
        t1, t2 = x1 + x2 + 1, 2 * x1 - 3 * x2
        term1 = 1 + t1 ** 2 * (19 - 14 * x1 + 3 * x1 ** 2 - 14 * x2 + 6 * x1 * x2 + 3 * x2 ** 2)
        term2 = 30 + t2 ** 2 * (18 - 32 * x1 + 12 * x1 ** 2 + 48 * x2 - 36 * x1 * x2 + 27 * x2 ** 2)
        return term1 * term2
    return TestFunction(2, [[-2.0, 2.0]] * 2, ([0.0, -1.0],), f, name="goldsteinprice")


def TestGriewank(d):
    """testfns.jl:695-720 (the later definition, which Julia keeps)"""
    def f(x):
        x = np.asarray(x, dtype=np.float64)
        s, prod = 0.0, 1.0
        for i in range(x.size):
            s += x[i] ** 2
            prod *= np.cos(x[i] / np.sqrt(i + 1))
        return 1 + s / 4000 - prod
    return TestFunction(d, [[-600.0, 600.0]] * d, (np.zeros(d),), f, name=f"griewank{d}d")


def TestLevy(d):
    """testfns.jl:116-134 (as written: sin(π w_i + 1) in the middle sum)"""
    def f(x):
        w = 1 + (np.asarray(x, dtype=np.float64) - 1) / 4
        term1 = np.sin(np.pi * w[0]) ** 2
        sum_terms = np.sum((w[:-1] - 1) ** 2 * (1 + 10 * np.sin(np.pi * w[:-1] + 1) ** 2))
        term3 = (w[-1] - 1) ** 2 * (1 + np.sin(2 * np.pi * w[-1]) ** 2)
        return float(term1 + sum_terms + term3)
    return TestFunction(d, [[-10.0, 10.0]] * d, (np.ones(d),), f, name=f"levy{d}d")
