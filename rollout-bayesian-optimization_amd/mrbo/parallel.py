"""Multi-GPU sharding of the rollout: one process per GPU.

The M Monte-Carlo samples of every restart are split into contiguous blocks of the shared
rnstream; each rank runs its block for all R restarts (no data-path communication) and reduces
its per-restart moments on the device -- the local sum Σx and the local centred second moment
M2 = Σ(x − x̄_local)² of [α, ∇x (d), ∇θ] (two passes over its samples, mrbo_partial_moments).
ONE all-gather (RCCL over xGMI on the GPU box, gloo on CPU tests) per outer SGA step hands every
rank the world's (n_k, Σ_k, M2_k); each rank merges them with Chan's parallel formula in rank
order, so all ranks derive the same ETO -- the two-pass mean and n−1 std of rollout.jl:328-337,
without the cancellation of a one-pass Σx² − (Σx)²/n -- and take the same ascent step.
"""
import numpy as np


def shard(M, world, rank):
    """contiguous MC block [lo, hi) of rank (first M % world ranks get one extra sample)"""
    base, extra = divmod(M, world)
    lo = rank * base + min(rank, extra)
    hi = lo + base + (1 if rank < extra else 0)
    return lo, hi


def width(d):
    """rows per restart of an ETO / moments block: [α, σα, ∇x (d), σ∇x (d), ∇θ, σ∇θ]"""
    return 2 + 2 * d + 2


def _split(a, d):
    """(first moments, second moments) rows of a (W, R) block, component order [α, ∇x (d), ∇θ]"""
    s = np.concatenate([a[0:1], a[2:2 + d], a[2 + 2 * d:3 + 2 * d]])
    q = np.concatenate([a[1:2], a[2 + d:2 + 2 * d], a[3 + 2 * d:4 + 2 * d]])
    return s, q


def _join(s, q, d):
    out = np.empty((width(d), s.shape[1]))
    out[0], out[1] = s[0], q[0]
    out[2:2 + d], out[2 + d:2 + 2 * d] = s[1:1 + d], q[1:1 + d]
    out[2 + 2 * d], out[3 + 2 * d] = s[1 + d], q[1 + d]
    return out


def local_moments(values, grad_x, grad_theta):
    """Host restatement of mrbo_partial_moments for one shard: values (M, R), grad_x (d, M, R),
    grad_theta (M, R) -> (W, R) rows [Σα, M2α, Σ∇x, M2∇x, Σ∇θ, M2∇θ] (two-pass M2)."""
    v = np.asarray(values, dtype=np.float64)
    gx = np.asarray(grad_x, dtype=np.float64)
    gt = np.asarray(grad_theta, dtype=np.float64).reshape(v.shape)
    d = gx.shape[0]
    comps = np.concatenate([v[None], gx, gt[None]])          # (d+2, M, R)
    n = comps.shape[1]
    s = comps.sum(axis=1)
    q = ((comps - (s / n)[:, None, :]) ** 2).sum(axis=1)
    return _join(s, q, d)


def merge_moments(parts, d):
    """Chan et al.'s pairwise merge of per-shard moments, left to right (rank order).
    parts: sequence of (n_k, (W, R) moments block).  Returns (n, merged block)."""
    n, acc = None, None
    for nk, blk in parts:
        sk, qk = _split(np.asarray(blk, dtype=np.float64), d)
        if nk == 0:
            continue
        if acc is None:
            n, s, q = nk, sk.copy(), qk.copy()
            acc = True
            continue
        delta = sk / nk - s / n
        q = q + qk + delta * delta * (n * nk / (n + nk))
        s = s + sk
        n = n + nk
    if acc is None:
        raise ValueError("no samples in any shard")
    return n, _join(s, q, d)


def eto_from_moments(moments, M, d):
    """(W, R) merged [Σ, M2] rows over all M samples -> ETO rows [μ, σ(n-1), ∇μx, σ∇x, ∇μθ, σ∇θ]
    (rollout.jl:328-339; M = 1 gives NaN std, Q14)."""
    s, q = _split(np.asarray(moments, dtype=np.float64), d)
    mu = s / M
    with np.errstate(invalid="ignore", divide="ignore"):
        sd = np.sqrt(q / (M - 1)) if M > 1 else np.full_like(q, np.nan)
    return _join(mu, sd, d)


def allgather_moments(moments_tensor, group=None):
    """ONE all-gather of every rank's flat (W·R) moments tensor; returns a list, rank order.
    gloo cannot gather device tensors: they travel through host memory on that backend.  Without a
    process group the tensor is returned as is; with one the collective runs at any world size
    (bench.py --sharded exercises RCCL at one rank)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return [moments_tensor]
    src = moments_tensor
    if src.is_cuda and dist.get_backend(group) == "gloo":
        src = src.cpu()
    outs = [torch.empty_like(src) for _ in range(dist.get_world_size(group))]
    dist.all_gather(outs, src, group=group)
    return outs


def allgather_moments_device(moments_tensor, group=None):
    """ONE all-gather of every rank's flat (W·R) device moments into one flat device tensor, rank
    order (RCCL gathers device tensors in place; gloo, the CPU rehearsal backend, goes through host
    memory and the result is copied back to the device)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return moments_tensor
    world = dist.get_world_size(group)
    if dist.get_backend(group) == "gloo":
        outs = [torch.empty_like(moments_tensor, device="cpu") for _ in range(world)]
        dist.all_gather(outs, moments_tensor.cpu(), group=group)
        return torch.cat(outs).to(moments_tensor.device)
    out = torch.empty(world * moments_tensor.numel(), dtype=moments_tensor.dtype, device=moments_tensor.device)
    dist.all_gather_into_tensor(out, moments_tensor, group=group)
    return out


def sharded_eto_device(plan, moments_tensor, shard_sizes, group=None):
    """The per-SGA-step exchange kept on the device: all-gather (device tensors) + Chan merge and
    ETO in mrbo_merge_moments.  Returns the ETO rows as a device tensor (plan.eto()'s layout), for
    plan.sga_step -- the same host profile as the one-GPU step (no .cpu() per step)."""
    gathered = allgather_moments_device(moments_tensor, group)
    return plan.merge_moments(gathered, shard_sizes)


def sharded_eto(moments_tensor, shard_sizes, d, group=None):
    """all-gather + Chan merge + ETO: the per-SGA-step exchange of the sharded rollout."""
    gathered = allgather_moments(moments_tensor, group)
    R = moments_tensor.numel() // width(d)
    parts = [(n, g.cpu().numpy().reshape((width(d), R), order="F")) for n, g in zip(shard_sizes, gathered)]
    n, merged = merge_moments(parts, d)
    return eto_from_moments(merged, n, d)
