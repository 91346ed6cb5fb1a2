"""Multi-GPU plumbing of the batched boundary-OCP path: one process per GPU (torch.distributed,
backend "nccl" = RCCL on ROCm; "gloo" in the CPU tests).

The reference fans problems out with `Pool(30).map(data_generation, range(P))`
(VBOC/triplependulum_vboc.py:399-405): problems are independent, so the batch shards with no
data-path collective.  Problem ids are a global counter and the initial conditions are a pure
function of the id (Philox, vboc_amd/ics.py), so any GPU count produces the same problems.  The one
real exchange is the all-gather of the boundary states that feed the NN fit
(VBOC/triplependulum_vboc.py:409-423 consumes the concatenated samples).
"""
import numpy as np


def shard_ids(step, world, rank, per_rank):
    """Problem ids solved by `rank` in batch `step`: a contiguous block of `per_rank` ids.
    Per-rank work is fixed as `world` grows (weak scaling)."""
    base = (step * world + rank) * per_rank
    return np.arange(base, base + per_rank, dtype=np.int64)


def gather_boundary_states(x0, group=None):
    """All-gather the per-rank boundary states x0 [B, nx] (equal B on every rank) into
    [world * B, nx] ordered by rank, i.e. by problem id for `shard_ids` blocks.  On GPU this is one
    RCCL all-gather over xGMI."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    x0 = x0.contiguous()
    out = torch.empty((world * x0.shape[0],) + tuple(x0.shape[1:]), dtype=x0.dtype, device=x0.device)
    dist.all_gather_into_tensor(out, x0, group=group)   # concatenated along dim 0 (RCCL and gloo)
    return out


def gather_samples(rows, group=None):
    """All-gather variable-length per-rank sample blocks rows [n_r, d] (float64) into
    [sum n_r, d] ordered by rank: one all-gather of the counts, then one all-gather of
    the blocks padded to max n_r (an all-gatherv emulation; RCCL over xGMI on GPU, gloo on CPU)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rows = rows.contiguous()
    n = torch.tensor([rows.shape[0]], dtype=torch.int64, device=rows.device)
    counts = torch.empty(world, dtype=torch.int64, device=rows.device)
    dist.all_gather_into_tensor(counts, n, group=group)
    counts = counts.tolist()
    cap = max(counts)
    d = rows.shape[1]
    pad = torch.zeros((cap, d), dtype=rows.dtype, device=rows.device)
    pad[:rows.shape[0]] = rows
    out = torch.empty((world * cap, d), dtype=rows.dtype, device=rows.device)
    if cap:
        dist.all_gather_into_tensor(out, pad, group=group)
    return torch.cat([out[r * cap: r * cap + c] for r, c in enumerate(counts)])
