"""Multi-GPU plumbing for bench.py: one process per GPU, no data-path
collective.

The hot path shards by sequence (each rank owns an independent synthetic
camera sequence / set of BA problems), so the only
collective is the end-of-run gather of per-rank stats: elapsed time is the
max over ranks, work is the sum.  torch.distributed is plumbing here
(backend "nccl" = RCCL on GPUs, "gloo" in the CPU tests).
"""
import os

import numpy as np


def env():
    """(world, rank, local_rank) from the torchrun environment."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def visible_gpus():
    """GPUs this process can see (torch.cuda.device_count() does not
    initialise the GPU on this image); 0 without torch or GPU."""
    try:
        import torch
        return torch.cuda.device_count()
    except Exception:   # noqa: BLE001
        return 0


def shard_seed(base, rank):
    """Seed of the sequence a rank owns (weak scaling: fixed work per rank)."""
    return base + rank


def gather_stats(stats, dist=None, device="cpu"):
    """All-gather a float64 vector of per-rank stats; returns a
    (world, len(stats)) array on every rank (a (1, n) array without dist)."""
    stats = np.asarray(stats, np.float64)
    if dist is None:
        return stats[None, :].copy()
    import torch
    t = torch.tensor(stats, dtype=torch.float64, device=device)
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return torch.stack(out).cpu().numpy()


def job_rate(all_stats, time_col=0, work_col=1):
    """Whole-job throughput: total work over the slowest rank's time."""
    elapsed = float(all_stats[:, time_col].max())
    work = float(all_stats[:, work_col].sum())
    return work / elapsed if elapsed > 0 else 0.0, elapsed, work
