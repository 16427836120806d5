"""mrbo -- MI355X-native rollout-acquisition evaluator (host mirror of the reference API).

Reference API surface kept (DarianNwankwo/Rollout-Bayesian-Optimization):
  kernels            Matern52/32/12, SquaredExponential, Periodic  radial_basis_functions.jl
  decision rules     EI, POI, LCB (compiled), Random (declared)  decision_rules.jl
  surrogates         Surrogate, FantasySurrogate               radial_basis_surrogates.jl
  trajectories       Trajectory, TrajectoryParameters, ExpectedTrajectoryOutput  trajectory.jl
  rollout            simulate_trajectory_mc                    rollout.jl:279-340
  outer ascent       StandardSGA, Adam, eswavs, stochastic_solve  optimizers.jl, utils.jl
  surrogate upkeep   log_likelihood, ∇log_likelihood, optimize!  radial_basis_surrogates.jl:770-829
Compute runs in libmrbo.so (hand-written HIP for gfx950); see include/mrbo.h.
"""
from .decision_rules import EI, LCB, POI, DecisionRule, RandomAcquisition, get_name
from .kernels import Matern12, Matern32, Matern52, Periodic, SquaredExponential, eval_KxX, eval_KXX
from .mle import grad_log_likelihood, gp_fit_batch, log_likelihood, optimize
from .optimizers import Adam, StandardSGA, update
from .rollout import (simulate_trajectory_ghq, simulate_trajectory_ghq_batch, simulate_trajectory_mc,
                      simulate_trajectory_mc_batch)
from .surrogates import DEFAULT_CAPACITY, GROUND_TRUTH_OBSERVATIONS, FantasySurrogate, Surrogate
from .trajectory import ExpectedTrajectoryOutput, Trajectory, TrajectoryParameters, gen_low_discrepancy_sequence
from .utils import (ExperimentSetup, GaussHermiteObservable, eswavs, gauss_hermite, generate_batch,
                    generate_indices, generate_initial_guesses, kronecker_quasirand, stochastic_solve,
                    stochastic_solve_batch)

__version__ = "0.1.0"
