"""RolloutPlan -- owns one libmrbo plan (device copy of the base surrogate + workspace) and
launches the rollout kernel on device-resident torch tensors.

torch is plumbing here (device memory, streams, torch.distributed); every arithmetic step of
the rollout path runs in libmrbo.so.
"""
import ctypes

import numpy as np

from . import _lib

DEFAULTS = dict(max_iters=50, max_ls=20, x_tol=1e-3, f_tol=1e-3, g_tol=1e-8, htol=1e-4, sigma_tol=1e-8, seed=1906,
                sample_offset=0, samples_total=0, cost="none", cost_c0=1.0, cost_w=())


def _torch():
    import torch
    if not torch.cuda.is_available():
        raise _lib.MrboError("libmrbo requires a ROCm GPU (torch.cuda.is_available() is False); there is no CPU path")
    return torch


def _f64(a):
    return np.asfortranarray(np.asarray(a, dtype=np.float64))


def to_device(a, device):
    """numpy (any order) -> flat column-major float64 device tensor"""
    torch = _torch()
    flat = np.asarray(a, dtype=np.float64).ravel(order="F").copy()
    return torch.from_numpy(flat).to(device)


def from_device(t, shape):
    return t.detach().cpu().numpy().reshape(shape, order="F")


class RolloutPlan:
    """Device state for (surrogate, trajectory parameters)."""

    def __init__(self, X, L, c, y, kernel, lengthscale, sigma_n2, fmini, h, M, R, nstarts, lbs, ubs, theta,
                 device=0, period=1.0, **opts):
        self.lib = _lib.load()
        o = dict(DEFAULTS)
        o.update(opts)
        self.opts = o
        self._X, self._L, self._c, self._y = _f64(X), _f64(L), _f64(c), _f64(y)
        self.d, self.N = self._X.shape
        self.h, self.M, self.R, self.nstarts = int(h), int(M), int(R), int(nstarts)
        self._lbs, self._ubs = _f64(lbs).ravel(), _f64(ubs).ravel()
        self.theta = float(theta)
        self.device = device
        dp = ctypes.POINTER(ctypes.c_double)
        sd = _lib.SurrogateDesc(self.d, self.N, int(kernel), float(lengthscale), float(sigma_n2), float(fmini),
                                self._X.ctypes.data_as(dp), self._L.ctypes.data_as(dp), self.N,
                                self._c.ctypes.data_as(dp), self._y.ctypes.data_as(dp), float(period))
        ck = _lib.COSTS[o["cost"]] if isinstance(o["cost"], str) else int(o["cost"])
        self._cost_w = _f64(o["cost_w"]).ravel() if ck else None
        if ck and self._cost_w.size != self.d:
            raise ValueError(f"cost_w has {self._cost_w.size} weights for d = {self.d}")
        pd = _lib.ParamsDesc(self.h, self.M, self.R, self.nstarts, int(o.get("rule", 0)), self.theta,
                             self._lbs.ctypes.data_as(dp),
                             self._ubs.ctypes.data_as(dp), int(o["max_iters"]), int(o["max_ls"]), float(o["x_tol"]),
                             float(o["f_tol"]), float(o["g_tol"]), float(o["htol"]), float(o["sigma_tol"]),
                             int(o["seed"]), int(o.get("sample_offset", 0)), int(o.get("samples_total", 0)),
                             ck, float(o["cost_c0"]), self._cost_w.ctypes.data_as(dp) if ck else None)
        h_ = ctypes.c_void_p()
        _lib.check(self.lib.mrbo_plan_create(ctypes.byref(sd), ctypes.byref(pd), int(device), ctypes.byref(h_)))
        self.handle = h_

    def close(self):
        if getattr(self, "handle", None):
            self.lib.mrbo_plan_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---------------------------------------------------------------------------------
    def alloc_outputs(self, with_gradient=True, want_policy=False, want_obs=False, want_evals=True):
        torch = _torch()
        dev = f"cuda:{self.device}"
        T = self.M * self.R
        out = dict(values=torch.empty(T, dtype=torch.float64, device=dev),
                   status=torch.empty(T, dtype=torch.int32, device=dev))
        if with_gradient:
            out["grad_x"] = torch.empty(self.d * T, dtype=torch.float64, device=dev)
            out["grad_theta"] = torch.empty(T, dtype=torch.float64, device=dev)
        if want_policy:
            out["policy_x"] = torch.empty(self.d * (self.h + 1) * T, dtype=torch.float64, device=dev)
        if want_obs:
            out["obs"] = torch.empty((self.h + 1) * T, dtype=torch.float64, device=dev)
        if want_evals:
            out["evals"] = torch.empty(_lib.NCOUNTERS * T, dtype=torch.int64, device=dev)
        return out

    def simulate(self, x0s, rnstream, xstarts, out, dual_y_dx=None, replay_x=None, stream=None):
        """Launch mrbo_simulate_mc on device tensors (flat, column-major)."""
        torch = _torch()
        st = stream if stream is not None else torch.cuda.current_stream(self.device)
        p = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None
        flags = 0 if "grad_x" in out else _lib.MRBO_FLAG_NO_GRADIENT
        _lib.check(self.lib.mrbo_simulate_mc(
            self.handle, p(x0s), p(rnstream), p(xstarts), p(dual_y_dx), p(replay_x), p(out["values"]),
            p(out.get("grad_x")), p(out.get("grad_theta")), p(out["status"]), p(out.get("policy_x")),
            p(out.get("obs")), p(out.get("evals")), flags, ctypes.c_void_p(st.cuda_stream)))
        return out

    def simulate_ghq(self, x0s, nodes, weights, xstarts, out, dual_y_dx=None, replay_x=None, stream=None):
        """Launch mrbo_simulate_ghq: nodes / weights are M×(h+1) device tensors (flat, column-major)."""
        torch = _torch()
        st = stream if stream is not None else torch.cuda.current_stream(self.device)
        p = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None
        flags = 0 if "grad_x" in out else _lib.MRBO_FLAG_NO_GRADIENT
        _lib.check(self.lib.mrbo_simulate_ghq(
            self.handle, p(x0s), p(nodes), p(weights), p(xstarts), p(dual_y_dx), p(replay_x), p(out["values"]),
            p(out.get("grad_x")), p(out.get("grad_theta")), p(out["status"]), p(out.get("policy_x")),
            p(out.get("obs")), p(out.get("evals")), flags, ctypes.c_void_p(st.cuda_stream)))
        return out

    def eto(self, out, stream=None):
        torch = _torch()
        st = stream if stream is not None else torch.cuda.current_stream(self.device)
        W = 2 + 2 * self.d + 2
        e = torch.empty(W * self.R, dtype=torch.float64, device=f"cuda:{self.device}")
        p = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None
        _lib.check(self.lib.mrbo_eto_reduce(self.handle, p(out["values"]), p(out.get("grad_x")),
                                            p(out.get("grad_theta")), p(e), 0, ctypes.c_void_p(st.cuda_stream)))
        return e

    def partial_moments(self, out, M_local, stream=None):
        """mrbo_partial_moments: this shard's (W·R) [Σ, M2] rows, device tensor (parallel.py)."""
        torch = _torch()
        st = stream if stream is not None else torch.cuda.current_stream(self.device)
        W = 2 + 2 * self.d + 2
        e = torch.empty(W * self.R, dtype=torch.float64, device=f"cuda:{self.device}")
        p = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None
        _lib.check(self.lib.mrbo_partial_moments(self.handle, p(out["values"]), p(out.get("grad_x")),
                                              p(out.get("grad_theta")), int(M_local), p(e), 0,
                                              ctypes.c_void_p(st.cuda_stream)))
        return e

    def merge_moments(self, gathered, counts, stream=None):
        """mrbo_merge_moments: gathered = the ranks' partial_moments blocks concatenated in rank
        order (one flat device tensor of len(counts)·W·R), counts = their sample counts; returns
        the merged ETO rows (device tensor, eto()'s layout)."""
        torch = _torch()
        st = stream if stream is not None else torch.cuda.current_stream(self.device)
        W = 2 + 2 * self.d + 2
        n = len(counts)
        if gathered.numel() != n * W * self.R or not gathered.is_cuda:
            raise ValueError(f"gathered must be a device tensor of {n}·{W}·{self.R} moments")
        e = torch.empty(W * self.R, dtype=torch.float64, device=f"cuda:{self.device}")
        c = (ctypes.c_int64 * n)(*[int(k) for k in counts])
        _lib.check(self.lib.mrbo_merge_moments(self.handle, n, ctypes.c_void_p(gathered.data_ptr()), c,
                                               ctypes.c_void_p(e.data_ptr()), 0, ctypes.c_void_p(st.cuda_stream)))
        return e

    def sga_step(self, eto, x0s, active, sample_size, eta, stream=None):
        """mrbo_sga_step: eswavs + StandardSGA for every active restart, in place on the device
        tensors x0s (d·R, column-major) and active (R, int32); eto from `eto()`."""
        torch = _torch()
        st = stream if stream is not None else torch.cuda.current_stream(self.device)
        p = lambda t: ctypes.c_void_p(t.data_ptr())
        _lib.check(self.lib.mrbo_sga_step(self.handle, p(eto), p(x0s), p(active), float(sample_size), float(eta), 0,
                                          ctypes.c_void_p(st.cuda_stream)))

    def adam_step(self, eto, x0s, active, m, v, t, sample_size, eta=0.001, beta1=0.9, beta2=0.999, eps=1e-8,
                  stream=None):
        """mrbo_adam_step: eswavs + Adam update! (optimizers.jl:49-74) for every active restart, in
        place on the device tensors x0s, m, v (d·R, column-major, m = v = 0 before update 1) and
        active (R, int32); t is this update's count (1, 2, ...)."""
        torch = _torch()
        st = stream if stream is not None else torch.cuda.current_stream(self.device)
        p = lambda t_: ctypes.c_void_p(t_.data_ptr())
        _lib.check(self.lib.mrbo_adam_step(self.handle, p(eto), p(x0s), p(active), p(m), p(v), int(t),
                                           float(sample_size), float(eta), float(beta1), float(beta2), float(eps), 0,
                                           ctypes.c_void_p(st.cuda_stream)))

    def stochastic_solve(self, x0s, rnstream, xstarts, optimizer="sga", iterations=50, eta=None, beta1=0.9,
                         beta2=0.999, eps=1e-8, sample_size=0, eto=None, active=None, dual_y_dx=None, stream=None):
        """mrbo_stochastic_solve on device tensors: the whole outer ascent (utils.jl:235-265) for the
        plan's R restarts in one call; x0s (d·R, column-major) is updated in place, eto (W·R) and
        active (R, int32) receive the final rows and stop flags when given.  Returns (iterations
        launched, iteration after which no restart was active, OR of the status bits)."""
        torch = _torch()
        st = stream if stream is not None else torch.cuda.current_stream(self.device)
        p = lambda t_: None if t_ is None else ctypes.c_void_p(t_.data_ptr())
        opt = _lib.MRBO_OPT_SGA if optimizer == "sga" else _lib.MRBO_OPT_ADAM
        eta = (0.01 if opt == _lib.MRBO_OPT_SGA else 0.001) if eta is None else eta
        o = _lib.SolveOpts(opt, int(iterations), float(eta), float(beta1), float(beta2), float(eps), float(sample_size))
        res = (ctypes.c_int32 * 3)()
        _lib.check(self.lib.mrbo_stochastic_solve(self.handle, p(x0s), p(rnstream), p(xstarts), p(dual_y_dx),
                                                  ctypes.byref(o), p(eto), p(active), res, 0,
                                                  ctypes.c_void_p(st.cuda_stream)))
        return int(res[0]), int(res[1]), int(res[2])

    def eval_base(self, xs):
        """eval(s, x, θ) at the columns of xs (d×P); returns (3+4d+d²)×P numpy."""
        torch = _torch()
        xs = _f64(xs)
        d, P = xs.shape
        stride = 3 + 4 * d + d * d
        dx = to_device(xs, f"cuda:{self.device}")
        do = torch.empty(stride * P, dtype=torch.float64, device=f"cuda:{self.device}")
        st = torch.cuda.current_stream(self.device)
        _lib.check(self.lib.mrbo_eval_base(self.handle, P, ctypes.c_void_p(dx.data_ptr()),
                                           ctypes.c_void_p(do.data_ptr()), 0, ctypes.c_void_p(st.cuda_stream)))
        torch.cuda.synchronize(self.device)
        return from_device(do, (stride, P))

    def last_kernel_ms(self):
        return self.lib.mrbo_last_kernel_ms(self.handle)

    def kernel_times(self, n):
        """mrbo_kernel_times: HIP-event durations (ms) of the rollout kernel alone in the plan's
        last min(n, launches, 64) mrbo_simulate_mc / _ghq launches, oldest first (waits for them)."""
        buf = (ctypes.c_double * max(int(n), 1))()
        k = self.lib.mrbo_kernel_times(self.handle, int(n), buf)
        _lib.check(min(k, 0))
        return [buf[i] for i in range(k)]

    # relative cost of one unit of each work counter (grad, value, hess, rich, pairs), in value
    # evaluations -- only the ORDER of the work depends on these, never a result
    ORDER_WEIGHTS = (2.5, 1.0, 3.0, 5.0, 3.0)

    def set_order(self, order, check=True):
        """mrbo_plan_set_order: an int32 device tensor holding a permutation of the M×R trajectory
        indices (m + M·r), or None for the identity.  The plan keeps a reference.  check=True
        refuses anything but a permutation (a duplicated index would run one trajectory on two waves
        at once and leave another unrun, its outputs undefined); check=False passes any order of the
        right length to the library (tests: the all-out-of-range guard)."""
        if order is None:
            _lib.check(self.lib.mrbo_plan_set_order(self.handle, None, 0))
            self._order = None
            return
        torch = _torch()
        if order.dtype != torch.int32 or not order.is_cuda or order.numel() != self.M * self.R:
            raise ValueError("order must be an int32 device tensor of M*R trajectory indices")
        if check and not torch.equal(torch.sort(order.to(torch.int64)).values,
                                     torch.arange(order.numel(), dtype=torch.int64, device=order.device)):
            raise ValueError("order is not a permutation of 0..M*R-1")
        self._order = order.contiguous()
        _lib.check(self.lib.mrbo_plan_set_order(self.handle, ctypes.c_void_p(self._order.data_ptr()),
                                                self._order.numel()))

    def order_longest_first(self, out, stream=None, order_out=None):
        """Schedule the next launches longest-first by the per-trajectory work counters of the
        launch that filled `out`: mrbo_plan_order_longest_first, on the device (no host round trip).
        Consecutive SGA steps move x0 a little and reuse the MC streams, so a trajectory's work
        repeats closely and the longest ones no longer start last (the launch's tail).

        The kernel's waves drain one queue per XCD over a contiguous eighth of the queue positions
        first (mrbo_rollout.hip rollout_kernel); the library re-orders each chunk's own trajectories
        longest first, so every XCD still writes the output rows of one contiguous index range
        (whole cache lines in one L2), and an XCD that drains its chunk early takes the short ends
        of the others.  The plan owns the order; order_out (int32 device tensor of M·R) receives a
        copy.  longest_first_order() is the torch mirror."""
        torch = _torch()
        st = stream if stream is not None else torch.cuda.current_stream(self.device)
        p = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None
        _lib.check(self.lib.mrbo_plan_order_longest_first(self.handle, p(out["evals"]), p(order_out),
                                                          ctypes.c_void_p(st.cuda_stream)))
        self._order = None

    @classmethod
    def longest_first_order(cls, evals):
        """Torch mirror of mrbo_plan_order_longest_first (longest_first_within_chunks of the
        integer work keys 2 × Σ ORDER_WEIGHTS · counters)."""
        import torch
        ev = evals.view(-1, _lib.NCOUNTERS).clamp(min=0)
        w2 = torch.tensor([int(round(2 * w)) for w in cls.ORDER_WEIGHTS], dtype=torch.int64, device=ev.device)
        return longest_first_within_chunks((ev.to(torch.int64) * w2).sum(1))

    def info(self):
        """Launch geometry: rows per lane, workgroups, waves per workgroup, batched start values,
        specialised kernel, LDS bytes per workgroup, fantasy capacity of the kernel unit (FMAX)."""
        v = (ctypes.c_int32 * 7)()
        _lib.check(self.lib.mrbo_plan_info(self.handle, v, 7))
        keys = ("rpl", "blocks", "waves_per_group", "batch", "spec", "lds_bytes", "fmax")
        return dict(zip(keys, (int(x) for x in v)))


XCD_QUEUES = 8   # work-queue heads of the rollout kernel (MRBO_QUEUE_INTS / 16)
ORDER_WBITS = 29  # work-key bits of mrbo_plan_order_longest_first (csrc/mrbo_order.hip) below the chunk


def xcd_chunks(T, device=None):
    """Per-XCD queue chunk of every queue position 0..T-1: chunk x = [x·T/8, (x+1)·T/8) (integer
    division, as rollout_kernel computes them).  Pure index arithmetic (CPU-testable)."""
    import torch
    p = torch.arange(T, dtype=torch.int64, device=device)
    lo = torch.tensor([x * T // XCD_QUEUES for x in range(1, XCD_QUEUES)], dtype=torch.int64, device=device)
    return torch.bucketize(p, lo, right=True)


def longest_first_within_chunks(work, device=None):
    """The order of mrbo_plan_order_longest_first from integer work keys (2 × the weighted counters):
    every chunk's own trajectories, longest first, stable in index order on ties -- queue position r
    takes trajectory order[r] and stays in the chunk it had in index order."""
    import torch
    work = torch.as_tensor(work, dtype=torch.int64, device=device).clamp(0, (1 << ORDER_WBITS) - 1)
    chunk = xcd_chunks(work.numel(), work.device)
    key = ((XCD_QUEUES - 1 - chunk) << ORDER_WBITS) | work
    return torch.sort(key, descending=True, stable=True).indices.to(torch.int32)


def rnstream(M, d, H):
    """gen_low_discrepancy_sequence (utils.jl:65-74) via the library's host Sobol."""
    lib = _lib.load()
    out = np.zeros((M, d + 1, H), order="F")
    _lib.check(lib.mrbo_rnstream(int(M), int(d), int(H), out.ctypes.data_as(ctypes.POINTER(ctypes.c_double))))
    return out


def initial_guesses(n, lbs, ubs):
    lib = _lib.load()
    lbs, ubs = _f64(lbs).ravel(), _f64(ubs).ravel()
    d = lbs.size
    out = np.zeros((d, n + 2), order="F")
    dp = ctypes.POINTER(ctypes.c_double)
    _lib.check(lib.mrbo_initial_guesses(int(n), d, lbs.ctypes.data_as(dp), ubs.ctypes.data_as(dp),
                                        out.ctypes.data_as(dp)))
    return out


def dual_uniform(seed, traj, j, k):
    return _lib.load().mrbo_dual_uniform(int(seed), int(traj), int(j), int(k))
