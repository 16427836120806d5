"""ctypes binding of libmrbo.so (include/mrbo.h) -- the product's only compute path.

The library is built in-tree by ``__graft_entry__.build()`` (hipcc --offload-arch=gfx950).
There is no CPU fallback: importing a compute entry point without the library, or calling
one without a GPU, raises.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MRBO_LIB") or os.path.join(_HERE, "libmrbo.so")  # MRBO_LIB: A/B variant builds

_dp = ctypes.POINTER(ctypes.c_double)
_vp = ctypes.c_void_p

# NonUniformCost families (mrbo_cost_t)
COSTS = {"none": 0, "quadratic": 1, "loglinear": 2}
MRBO_FLAG_HOST_POINTERS = 1
MRBO_FLAG_NO_GRADIENT = 2
# per-trajectory work counters of mrbo_simulate_mc `evals` (MRBO_NCOUNTERS in include/mrbo.h)
NCOUNTERS = 5
COUNTER_NAMES = ("grad_evals", "value_evals", "hessians", "rich_evals", "pairs")

STATUS_BITS = {
    1: "DomainError: sqrt of a negative posterior variance (radial_basis_surrogates.jl:528)",
    2: "PosDefException: gp_draw covariance (radial_basis_surrogates.jl:537)",
    4: "PosDefException: update_cholesky! (radial_basis_surrogates.jl:412)",
    8: "ArgumentError: findmin over an empty candidate list (rbf_optim.jl:96-97)",
    16: "SingularException: solve_dual_x Hessian (rollout.jl:188)",
}

# exported symbols of include/mrbo.h (the library must export all of them)
EXPORTS = [
    "mrbo_version", "mrbo_last_error", "mrbo_device_count", "mrbo_plan_create", "mrbo_plan_destroy",
    "mrbo_simulate_mc", "mrbo_simulate_ghq", "mrbo_eto_reduce", "mrbo_partial_moments", "mrbo_eval_base", "mrbo_rnstream",
    "mrbo_initial_guesses", "mrbo_dual_uniform", "mrbo_last_kernel_ms", "mrbo_gp_fit", "mrbo_gp_fit_theta",
    "mrbo_plan_info", "mrbo_last_gp_fit_ms", "mrbo_plan_set_order", "mrbo_base_solve", "mrbo_sga_step",
    "mrbo_kernel_times", "mrbo_merge_moments", "mrbo_adam_step", "mrbo_stochastic_solve",
    "mrbo_plan_order_longest_first",
]

MRBO_OPT_SGA, MRBO_OPT_ADAM = 0, 1


class SurrogateDesc(ctypes.Structure):
    _fields_ = [("d", ctypes.c_int32), ("N", ctypes.c_int32), ("kernel", ctypes.c_int32),
                ("lengthscale", ctypes.c_double), ("sigma_n2", ctypes.c_double), ("fmini", ctypes.c_double),
                ("X", _dp), ("L", _dp), ("ldL", ctypes.c_int32), ("c", _dp), ("y", _dp), ("period", ctypes.c_double)]


class ParamsDesc(ctypes.Structure):
    _fields_ = [("h", ctypes.c_int32), ("M", ctypes.c_int32), ("R", ctypes.c_int32), ("nstarts", ctypes.c_int32),
                ("rule", ctypes.c_int32), ("theta", ctypes.c_double), ("lbs", _dp), ("ubs", _dp),
                ("max_iters", ctypes.c_int32), ("max_ls", ctypes.c_int32), ("x_tol", ctypes.c_double),
                ("f_tol", ctypes.c_double), ("g_tol", ctypes.c_double), ("htol", ctypes.c_double),
                ("sigma_tol", ctypes.c_double), ("seed", ctypes.c_uint64),
                ("sample_offset", ctypes.c_int32), ("samples_total", ctypes.c_int32),
                ("cost", ctypes.c_int32), ("cost_c0", ctypes.c_double), ("cost_w", _dp)]


class SolveOpts(ctypes.Structure):
    """mrbo_solve_opts_t (include/mrbo.h)."""
    _fields_ = [("optimizer", ctypes.c_int32), ("iterations", ctypes.c_int32), ("eta", ctypes.c_double),
                ("beta1", ctypes.c_double), ("beta2", ctypes.c_double), ("eps", ctypes.c_double),
                ("sample_size", ctypes.c_double)]


_lib = None


class MrboError(RuntimeError):
    pass


def load():
    """Load libmrbo.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise MrboError(f"libmrbo.so not built at {LIB_PATH}: run __graft_entry__.build()")
    # torch ships its own libamdhip64.so.7 (same SONAME as /opt/rocm's): whichever loads first
    # serves the whole process, and torch cannot initialise on the other one.  Load torch's
    # first so that the process has one HIP runtime shared by torch and libmrbo.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(LIB_PATH)
    L.mrbo_version.restype = ctypes.c_char_p
    L.mrbo_last_error.restype = ctypes.c_char_p
    L.mrbo_device_count.restype = ctypes.c_int
    L.mrbo_plan_create.argtypes = [ctypes.POINTER(SurrogateDesc), ctypes.POINTER(ParamsDesc), ctypes.c_int32,
                                   ctypes.POINTER(_vp)]
    L.mrbo_plan_destroy.argtypes = [_vp]
    L.mrbo_simulate_mc.argtypes = [_vp] + [_vp] * 12 + [ctypes.c_uint32, _vp]
    L.mrbo_simulate_ghq.argtypes = [_vp] + [_vp] * 13 + [ctypes.c_uint32, _vp]
    L.mrbo_eto_reduce.argtypes = [_vp, _vp, _vp, _vp, _vp, ctypes.c_uint32, _vp]
    L.mrbo_partial_moments.argtypes = [_vp, _vp, _vp, _vp, ctypes.c_int32, _vp, ctypes.c_uint32, _vp]
    L.mrbo_eval_base.argtypes = [_vp, ctypes.c_int32, _vp, _vp, ctypes.c_uint32, _vp]
    L.mrbo_sga_step.argtypes = [_vp, _vp, _vp, _vp, ctypes.c_double, ctypes.c_double, ctypes.c_uint32, _vp]
    L.mrbo_adam_step.argtypes = [_vp, _vp, _vp, _vp, _vp, _vp, ctypes.c_int32] + [ctypes.c_double] * 5 + [
        ctypes.c_uint32, _vp]
    L.mrbo_stochastic_solve.argtypes = [_vp, _vp, _vp, _vp, _vp, ctypes.POINTER(SolveOpts), _vp, _vp,
                                        ctypes.POINTER(ctypes.c_int32), ctypes.c_uint32, _vp]
    L.mrbo_base_solve.argtypes = [_vp, ctypes.c_int32, _vp, _vp, _vp, _vp, _vp, ctypes.c_uint32, _vp]
    L.mrbo_rnstream.argtypes = [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, _dp]
    L.mrbo_initial_guesses.argtypes = [ctypes.c_int32, ctypes.c_int32, _dp, _dp, _dp]
    L.mrbo_dual_uniform.argtypes = [ctypes.c_uint64, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32]
    L.mrbo_dual_uniform.restype = ctypes.c_double
    L.mrbo_gp_fit.argtypes = [ctypes.POINTER(SurrogateDesc), ctypes.c_int32, _vp, _vp, _vp, _vp, _vp, _vp,
                              ctypes.c_uint32, _vp]
    L.mrbo_gp_fit_theta.argtypes = [ctypes.POINTER(SurrogateDesc), ctypes.c_int32, ctypes.c_int32, _vp, _vp, _vp,
                                    _vp, _vp, _vp, ctypes.c_uint32, _vp]
    L.mrbo_last_kernel_ms.argtypes = [_vp]
    L.mrbo_last_kernel_ms.restype = ctypes.c_double
    L.mrbo_plan_info.argtypes = [_vp, ctypes.POINTER(ctypes.c_int32), ctypes.c_int32]
    L.mrbo_kernel_times.argtypes = [_vp, ctypes.c_int32, ctypes.POINTER(ctypes.c_double)]
    L.mrbo_merge_moments.argtypes = [_vp, ctypes.c_int32, _vp, ctypes.POINTER(ctypes.c_int64), _vp, ctypes.c_uint32,
                                     _vp]
    L.mrbo_plan_set_order.argtypes = [_vp, _vp, ctypes.c_int64]
    L.mrbo_plan_order_longest_first.argtypes = [_vp, _vp, _vp, _vp]
    L.mrbo_last_gp_fit_ms.restype = ctypes.c_double
    _lib = L
    return L


def check(rc):
    if rc != 0:
        raise MrboError(f"mrbo error {rc}: {load().mrbo_last_error().decode()}")
    return rc
