"""Multi-GPU sharding of the rollout: one process per GPU.

The M Monte-Carlo samples of every restart are split into contiguous blocks of the shared
rnstream; each rank runs its block for all R restarts (no data-path communication), reduces
its per-restart partial sums [Σα, Σα², Σ∇x, Σ∇x², Σ∇θ, Σ∇θ²] on the device, and ONE
all-reduce (RCCL over xGMI on the GPU box, gloo on CPU tests) per outer SGA step combines
them.  Every rank then derives the same ETO and takes the same ascent step.
"""
import numpy as np


def shard(M, world, rank):
    """contiguous MC block [lo, hi) of rank (first M % world ranks get one extra sample)"""
    base, extra = divmod(M, world)
    lo = rank * base + min(rank, extra)
    hi = lo + base + (1 if rank < extra else 0)
    return lo, hi


def eto_from_sums(sums, M, d):
    """sums: (W, R) of [Σα, Σα², Σ∇x(d), Σ∇x²(d), Σ∇θ, Σ∇θ²] over all M samples → ETO rows
    [μ, σ(n-1), grad_μx, σ∇x, grad_μθ, σ∇θ] (rollout.jl:328-339)."""
    sums = np.asarray(sums, dtype=np.float64)
    W, R = sums.shape
    out = np.zeros_like(sums)

    def ms(s1, s2):
        mu = s1 / M
        var = (s2 - s1 * mu) / (M - 1) if M > 1 else np.full_like(s1, np.nan)
        return mu, np.sqrt(np.maximum(var, 0.0))

    out[0], out[1] = ms(sums[0], sums[1])
    mu, sd = ms(sums[2:2 + d], sums[2 + d:2 + 2 * d])
    out[2:2 + d], out[2 + d:2 + 2 * d] = mu, sd
    out[2 + 2 * d], out[3 + 2 * d] = ms(sums[2 + 2 * d], sums[3 + 2 * d])
    return out


def allreduce_sums(sums_tensor, group=None):
    """one sum all-reduce of the (W·R) partial sums (fp64)."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        if sums_tensor.is_cuda and dist.get_backend(group) == "gloo":
            host = sums_tensor.cpu()
            dist.all_reduce(host, op=dist.ReduceOp.SUM, group=group)
            sums_tensor.copy_(host)
        else:
            dist.all_reduce(sums_tensor, op=dist.ReduceOp.SUM, group=group)
    return sums_tensor
