"""Spectral (g-point) sharding of a correlated-k band over ranks.

pyharp sums the per-g fluxes of a band with the ck weights after the solve
(examples/amars_lw.cpp:84-88: ``bflx = (flux * weights.view({-1,1,1,1})).sum(0)``;
legacy accumulation src/rtsolver/rt_solver_disort.cpp_:268-271).  With the
g-points of a band spread over ranks, each rank solves its own g-points and the
band flux is completed by ONE all-reduce (sum) of the weighted partial band
flux (ncol, nlyr+1, 2) -- the only exchange step of the path (RCCL over xGMI
with the "nccl" backend; gloo on CPU in the tests).
"""

from __future__ import annotations

from typing import List

import torch


def shard_gpoints(ngpoint: int, world: int, rank: int) -> List[int]:
    """g-points owned by `rank`: {g : g mod world == rank} (round-robin)."""
    if not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world {world}")
    return [g for g in range(ngpoint) if g % world == rank]


def band_flux(flux: torch.Tensor, weights: torch.Tensor) -> torch.Tensor:
    """sum_g w_g F_g for flux (G, ncol, nlyr+1, 2) and weights (G,)."""
    return torch.einsum("g,gcld->cld", weights.to(flux.dtype), flux)


def allreduce_band_flux(partial: torch.Tensor, group=None) -> torch.Tensor:
    """Complete the band sum across ranks (in place; returns the tensor)."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(partial, op=dist.ReduceOp.SUM, group=group)
    return partial
