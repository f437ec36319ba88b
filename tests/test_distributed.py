"""The N>1 path on CPU: spectral sharding + one all-reduce of the band flux.

2, 4 and 8 gloo ranks each solve their own g-points (with the CPU oracle standing in
for the device solve and the device band sum -- test infrastructure only) and
complete the band flux with pyharp_amd.spectral.allreduce_band_flux; the
result must equal the single-process band sum.
"""

import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _problem(G=6):
    rng = np.random.default_rng(3)
    C, L, nstr = 3, 5, 4
    prop = np.zeros((G, C, L, 2 + nstr))
    prop[..., 0] = 10 ** rng.uniform(-2, 0.5, (G, C, L))
    prop[..., 1] = rng.uniform(0, 0.9, (G, C, L))
    bc = {"fbeam": np.ones((G, C)), "umu0": rng.uniform(0.2, 1, (G, C)),
          "albedo": rng.uniform(0, 1, (G, C))}
    w = rng.uniform(0.1, 1.0, G)
    return prop, bc, w / w.sum(), nstr


def _worker(rank, world, port, out_path, G=6):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle_c
    from pyharp_amd.spectral import allreduce_band_flux, shard_gpoints
    prop, bc, w, nstr = _problem(G)
    mine = shard_gpoints(prop.shape[0], world, rank)
    if mine:
        flux = oracle_c.forward(prop[mine], {k: v[mine] for k, v in bc.items()}, nstr=nstr)
        # the rank's partial band sum (on the GPU: hd_band_flux; here the test's own)
        part = torch.as_tensor(np.einsum("g,gcld->cld", w[mine], flux))
    else:  # more ranks than g-points: this rank adds zeros
        part = torch.zeros((prop.shape[1], prop.shape[2] + 1, 2), dtype=torch.float64)
    allreduce_band_flux(part)
    np.save(out_path + f".rank{rank}.npy", part.numpy())
    dist.destroy_process_group()


def test_shard_gpoints_partition():
    from pyharp_amd.spectral import shard_gpoints
    for world in (1, 2, 3, 8):
        allg = sorted(g for r in range(world) for g in shard_gpoints(64, world, r))
        assert allg == list(range(64))
    with pytest.raises(ValueError):
        shard_gpoints(8, 2, 2)


@pytest.mark.parametrize("world,G", [(2, 6), (4, 16), (8, 16), (8, 6)])
def test_multi_rank_band_flux(tmp_path, oracle_c, world, G):
    """N = 2, 4, 8 ranks (the driver's scaling legs; (8, 6): two ranks own no
    g-point) complete the same band flux as one process, and every rank holds the
    identical all-reduced tensor (so any rank may write it)."""
    out = str(tmp_path / "band")
    mp.spawn(_worker, args=(world, _free_port(), out, G), nprocs=world, join=True)
    prop, bc, w, nstr = _problem(G)
    ref = np.einsum("g,gcld->cld", w, oracle_c.forward(prop, bc, nstr=nstr))
    got = [np.load(out + f".rank{r}.npy") for r in range(world)]
    np.testing.assert_allclose(got[0], ref, rtol=1e-13, atol=1e-16)
    for r in range(1, world):
        assert np.array_equal(got[r], got[0]), r
