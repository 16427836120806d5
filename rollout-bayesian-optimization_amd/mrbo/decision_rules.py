"""Decision rules -- host mirror of decision_rules.jl.

A DecisionRule names the base acquisition g(μ, σ, θ, sx) whose value, gradient and Hessian
the device kernel evaluates in closed form (the reference takes the 8 partials by
ForwardDiff, decision_rules.jl:23-34).  EI is the rule compiled into libmrbo.so; POI, LCB
and Random are declared for API parity and rejected by the rollout plan.
"""
import numpy as np
from scipy.special import erfc

RULES = {"EI": 0}


class DecisionRule:
    def __init__(self, name, sigma_tol=1e-8):
        self.name = name
        self.σtol = sigma_tol

    def __repr__(self):
        return f"DecisionRule{{{self.name}}}"

    # Host-side closed-form value (for tests and docs; the rollout path never calls this).
    def __call__(self, μ, σ, θ, fmini):
        if self.name != "EI":
            raise NotImplementedError(self.name)
        if σ < self.σtol:
            return 0.0
        imp = fmini - μ - θ[0]
        z = imp / σ
        return imp * (erfc(-z / np.sqrt(2.0)) / 2.0) + σ * np.exp(-(z * z) / 2.0) / np.sqrt(2.0 * np.pi)


def get_name(dr):
    return dr.name


def EI(σtol=1e-8):
    """decision_rules.jl:84-99"""
    return DecisionRule("EI", σtol)


def POI(σtol=1e-8):
    """decision_rules.jl:101-115 (declared; not compiled into the rollout kernel)"""
    return DecisionRule("POI", σtol)


def LCB():
    """decision_rules.jl:117-127 (declared; not compiled into the rollout kernel)"""
    return DecisionRule("LCB")


def RandomAcquisition():
    """decision_rules.jl:129-135 (declared; not compiled into the rollout kernel)"""
    return DecisionRule("Random")
