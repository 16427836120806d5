"""Decision rules -- host mirror of decision_rules.jl.

A DecisionRule names the base acquisition g(μ, σ, θ, sx) whose value, gradient and Hessian
the device kernel evaluates in closed form (the reference takes the 8 partials by
ForwardDiff, decision_rules.jl:23-34).  EI, POI and LCB are compiled into libmrbo.so
(mrbo_rule_t); Random (g ≡ 0) is declared for API parity and rejected by the rollout plan.
"""
import numpy as np
from scipy.special import erfc

RULES = {"EI": 0, "POI": 1, "LCB": 2}   # mrbo_rule_t (include/mrbo.h)


class DecisionRule:
    def __init__(self, name, sigma_tol=1e-8):
        self.name = name
        self.σtol = sigma_tol

    def __repr__(self):
        return f"DecisionRule{{{self.name}}}"

    @property
    def rule_id(self):
        """mrbo_rule_t of this rule (KeyError for rules the kernel does not compile)."""
        return RULES[self.name]

    # Host-side closed-form value (for tests and docs; the rollout path never calls this).
    def __call__(self, μ, σ, θ, fmini):
        if self.name == "LCB":
            return θ[0] * σ - μ
        if self.name == "Random":
            return 0.0
        if σ < self.σtol:
            return 0.0
        imp = fmini - μ - θ[0]
        z = imp / σ
        Φ = erfc(-z / np.sqrt(2.0)) / 2.0
        if self.name == "POI":
            return Φ
        return imp * Φ + σ * np.exp(-(z * z) / 2.0) / np.sqrt(2.0 * np.pi)


def get_name(dr):
    return dr.name


def EI(σtol=1e-8):
    """decision_rules.jl:84-99"""
    return DecisionRule("EI", σtol)


def POI(σtol=1e-8):
    """decision_rules.jl:101-115"""
    return DecisionRule("POI", σtol)


def LCB():
    """decision_rules.jl:117-127"""
    return DecisionRule("LCB")


def RandomAcquisition():
    """decision_rules.jl:129-135 (declared; not compiled into the rollout kernel)"""
    return DecisionRule("Random")
