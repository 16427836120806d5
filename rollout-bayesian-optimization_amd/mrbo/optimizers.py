"""Stochastic gradient ascent rules -- mirror of optimizers.jl (host, one update per SGA step)."""
import numpy as np


class StandardSGA:
    """optimizers.jl:6-23"""

    def __init__(self, η=0.01):
        self.η = η

    def update(self, x, grad_f):
        x += self.η * np.asarray(grad_f)
        return x


class Adam:
    """optimizers.jl:25-74"""

    def __init__(self, η=0.001, β1=0.9, β2=0.999, ε=1e-8, t=0):
        self.η, self.β1, self.β2, self.ε, self.t = η, β1, β2, ε, t
        self.m = []
        self.v = []

    def update(self, x, grad_f):
        grad_f = np.asarray(grad_f, dtype=np.float64)
        if len(self.m) == 0 and len(self.v) == 0:
            self.m.append(np.zeros(grad_f.size))
            self.v.append(np.zeros(grad_f.size))
        self.t += 1
        self.m.append(self.β1 * self.m[-1] + (1 - self.β1) * grad_f)
        self.v.append(self.β2 * self.v[-1] + (1 - self.β2) * grad_f ** 2)
        m̂ = self.m[-1] / (1 - self.β1 ** self.t)
        v̂ = self.v[-1] / (1 - self.β2 ** self.t)
        x += self.η * m̂ / (np.sqrt(v̂) + self.ε)
        return x


def update(optimizer, x, grad_f):
    return optimizer.update(x, grad_f)
