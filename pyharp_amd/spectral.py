"""Spectral (g-point) sharding of a correlated-k band over ranks, and the band
epilogue after the solve (band flux, heating rate, spherical correction).

pyharp sums the per-g fluxes of a band with the ck weights after the solve
(examples/amars_lw.cpp:84-88: ``bflx = (flux * weights.view({-1,1,1,1})).sum(0)``;
legacy accumulation src/rtsolver/rt_solver_disort.cpp_:268-271).  With the
g-points of a band spread over ranks, each rank solves its own g-points and the
band flux is completed by ONE all-reduce (sum) of the weighted partial band
flux (ncol, nlyr+1, 2) -- the only exchange step of the path (RCCL over xGMI
with the "nccl" backend; gloo on CPU in the tests).
"""

from __future__ import annotations

import ctypes
from typing import List, Optional

import torch

from . import _lib


def shard_gpoints(ngpoint: int, world: int, rank: int) -> List[int]:
    """g-points owned by `rank`: {g : g mod world == rank} (round-robin)."""
    if not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world {world}")
    return [g for g in range(ngpoint) if g % world == rank]


def _stream(dev):
    return torch.cuda.current_stream(dev).cuda_stream


def _dev_f64(t: torch.Tensor, what: str) -> torch.Tensor:
    if not isinstance(t, torch.Tensor) or t.device.type != "cuda":
        raise RuntimeError(f"{what}: expects a device (HIP) tensor -- pyharp_amd has no CPU path")
    return t.to(torch.float64).contiguous()


def band_flux(flux: torch.Tensor, weights: torch.Tensor,
              out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """sum_g w_g F_g for flux (G, ncol, nlev, 2) and weights (G,), in g order
    (hd_band_flux; examples/amars_lw.cpp:84-88, amars_sw.cpp:169-196 with
    w = d(wavenumber))."""
    f = _dev_f64(flux, "band_flux")
    G, ncol, nlev, two = f.shape
    if two != 2:
        raise RuntimeError("band_flux: flux must be (G, ncol, nlev, 2)")
    w = torch.as_tensor(weights, dtype=torch.float64).to(f.device).contiguous()
    if w.numel() != G:
        raise RuntimeError(f"band_flux: {w.numel()} weights for {G} g-points")
    if out is None:
        out = torch.empty((ncol, nlev, 2), dtype=torch.float64, device=f.device)
    with torch.cuda.device(f.device):
        _lib.check(_lib.load().hd_band_flux(f.data_ptr(), w.data_ptr(), G, ncol, nlev,
                                            out.data_ptr(), _stream(f.device)))
    return out


def heating_rate(bflux: torch.Tensor, dz: torch.Tensor, rho: torch.Tensor,
                 cp: float) -> torch.Tensor:
    """dT/dt (ncol, nlyr) [K/s] = -(1/(rho c_p)) d(F_up - F_dn)/dz from the band
    flux (ncol, nlyr+1, 2), level 0 = bottom (examples/amars_sw.cpp:291-302)."""
    f = _dev_f64(bflux, "heating_rate")
    ncol, nlev, _ = f.shape
    nlyr = nlev - 1
    d = torch.as_tensor(dz, dtype=torch.float64).to(f.device)
    r = torch.as_tensor(rho, dtype=torch.float64).to(f.device)
    d = d.reshape(-1)[:nlyr].expand(ncol, nlyr).contiguous() if d.numel() == nlyr else \
        d.reshape(ncol, nlyr).contiguous()
    r = r.reshape(-1).expand(ncol, nlyr).contiguous() if r.numel() == nlyr else \
        r.reshape(ncol, nlyr).contiguous()
    out = torch.empty((ncol, nlyr), dtype=torch.float64, device=f.device)
    with torch.cuda.device(f.device):
        _lib.check(_lib.load().hd_heating_rate(f.data_ptr(), d.data_ptr(), r.data_ptr(),
                                               float(cp), ncol, nlyr, out.data_ptr(),
                                               _stream(f.device)))
    return out


def spherical_flux_correction(bflux: torch.Tensor, x1f: torch.Tensor, area: torch.Tensor,
                              vol: torch.Tensor) -> torch.Tensor:
    """In place on the band flux (ncol, nlev, 2) along the level axis
    (src/utils/spherical_flux_correction.cpp:3-17; legacy
    rt_solver_disort.cpp_:186-207): top-level fluxes stay, lower levels are
    rescaled so the flux divergence per volume matches the plane-parallel one."""
    f = _dev_f64(bflux, "spherical_flux_correction")
    if f.data_ptr() != bflux.data_ptr():
        raise RuntimeError("spherical_flux_correction: bflux must be a contiguous f64 tensor")
    ncol, nlev, _ = f.shape
    dev = f.device
    x = torch.as_tensor(x1f, dtype=torch.float64).to(dev).contiguous()
    a = torch.as_tensor(area, dtype=torch.float64).to(dev).contiguous()
    v = torch.as_tensor(vol, dtype=torch.float64).to(dev).contiguous()
    if x.numel() != nlev or a.numel() != nlev or v.numel() < nlev - 1:
        raise RuntimeError("spherical_flux_correction: x1f/area need nlev entries, vol nlev-1")
    with torch.cuda.device(dev):
        _lib.check(_lib.load().hd_spherical_flux_correction(f.data_ptr(), x.data_ptr(),
                                                            a.data_ptr(), v.data_ptr(), ncol,
                                                            nlev, _stream(dev)))
    return bflux


def allreduce_band_flux(partial: torch.Tensor, group=None) -> torch.Tensor:
    """Complete the band sum across ranks (in place; returns the tensor)."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(partial, op=dist.ReduceOp.SUM, group=group)
    return partial
