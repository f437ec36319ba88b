"""The N>1 path with real device solves: 2 ranks on this box's GPU(s).

Each rank solves its spectral shard with the HIP kernels, forms its partial
band flux with hd_band_flux and completes it with allreduce_band_flux.  The
pool's test box has one GPU, so both ranks share cuda:0 and the collective is
gloo over device tensors (RCCL refuses two ranks on one device); bench.py's
RCCL path differs only in the backend string.  The result must equal the
single-process solve + band sum.
"""

import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _problem():
    rng = np.random.default_rng(31)
    G, C, L, nstr = 12, 40, 30, 16
    prop = np.zeros((G, C, L, 2 + nstr))
    prop[..., 0] = 10 ** rng.uniform(-4, 0.7, (G, C, L))
    prop[..., 1] = rng.uniform(0, 0.99, (G, C, L))
    g = rng.uniform(0, 0.85, (G, C, L))
    for l in range(nstr):
        prop[..., 2 + l] = g ** (l + 1)
    bc = {"fbeam": np.ones((G, C)), "umu0": rng.uniform(0.1, 1, (G, C)),
          "albedo": rng.uniform(0, 1, (G, C))}
    w = rng.uniform(0.1, 1.0, G)
    return prop, bc, w / w.sum(), nstr


def _solve(prop, bc, nstr, dev):
    from pyharp_amd import Disort, DisortOptions
    G, C, L, _ = prop.shape
    op = DisortOptions().flags("lamber,quiet,onlyfl").nwave(G).ncol(C)
    op.ds().nlyr, op.ds().nstr, op.ds().nmom = L, nstr, nstr
    return Disort(op).forward(torch.as_tensor(prop, device=dev),
                              {k: torch.as_tensor(v, device=dev) for k, v in bc.items()})


def _worker(rank, world, port, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dev = torch.device("cuda", rank % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from pyharp_amd.spectral import allreduce_band_flux, band_flux, shard_gpoints
    prop, bc, w, nstr = _problem()
    mine = shard_gpoints(prop.shape[0], world, rank)
    flux = _solve(prop[mine], {k: v[mine] for k, v in bc.items()}, nstr, dev)
    part = band_flux(flux, torch.as_tensor(w[mine], device=dev))
    allreduce_band_flux(part)
    if rank == 0:
        np.save(out_path, part.cpu().numpy())
    dist.destroy_process_group()


def test_two_ranks_band_flux_matches_single_process(tmp_path):
    out = str(tmp_path / "band.npy")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    prop, bc, w, nstr = _problem()
    from pyharp_amd.spectral import band_flux
    dev = torch.device("cuda", 0)
    ref = band_flux(_solve(prop, bc, nstr, dev), torch.as_tensor(w, device=dev)).cpu().numpy()
    got = np.load(out)
    np.testing.assert_allclose(got, ref, rtol=1e-13, atol=1e-15)
