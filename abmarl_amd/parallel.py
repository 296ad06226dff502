"""Multi-GPU: independent env shards, one process per GPU.

Envs never interact, so a step has no exchange: the global env range
[0, E) is split contiguously over ranks, every env is seeded from its global
id (results are bit-identical for any world size), and the only collective
is an all-gather of per-env episode statistics at report time (RCCL over
xGMI with backend 'nccl', gloo on CPU).
"""
import torch


def shard_envs(total_envs, rank, world):
    """Contiguous shard (first_env, n_envs) of rank in [0, world)."""
    assert 0 <= rank < world and total_envs >= world
    base, rem = divmod(total_envs, world)
    first = rank * base + min(rank, rem)
    return first, base + (1 if rank < rem else 0)


def gather_episode_stats(acting, steps, dist=None):
    """All-gather per-env counters (acting agent-steps, steps into the current
    episode) from every rank and summarise them on every rank."""
    local = torch.stack([acting.to(torch.float64), steps.to(torch.float64)], dim=1)
    if dist is not None and dist.is_initialized() and dist.get_world_size() > 1:
        n = torch.tensor([local.shape[0]], device=local.device)
        sizes = [torch.zeros_like(n) for _ in range(dist.get_world_size())]
        dist.all_gather(sizes, n)
        mx = int(max(s.item() for s in sizes))
        pad = torch.zeros((mx, 2), dtype=local.dtype, device=local.device)
        pad[:local.shape[0]] = local
        parts = [torch.zeros_like(pad) for _ in sizes]
        dist.all_gather(parts, pad)
        allv = torch.cat([p[:int(s.item())] for p, s in zip(parts, sizes)])
    else:
        allv = local
    return {'envs': int(allv.shape[0]),
            'acting_agent_steps_total': float(allv[:, 0].sum().item()),
            'acting_per_env_min': float(allv[:, 0].min().item()),
            'acting_per_env_max': float(allv[:, 0].max().item()),
            'mean_episode_step': float(allv[:, 1].mean().item())}
