"""Jacobi sweeps needed per layer on the GPU, with and without the warm start.

    HD_JACOBI_WARM=0|1 python scripts/micro/sweep_count.py NSTR [NCOL]

One-layer solves (so a solve's HD_STATUS_EIGEN bit is one layer kernel item's)
with C4's distributions (omega in [0, 0.99], HG g in [0, 0.85]; nstr 32: the
band-loop aerosol mix of two HG, omega in [0.8, 1)); for each sweep cap k the
layers still rotating at k are flagged, so the wave maximum (64 items per wave
on the register path, 4 on the team path) is the first k with no flag in it.
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "tests"))
from pyharp_amd import _lib  # noqa: E402
from pyharp_amd.disort import _context  # noqa: E402
from test_gpu_parity import _disort, _run  # noqa: E402

nstr = int(sys.argv[1])
ncol = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
rng = np.random.default_rng(5)
prop = np.zeros((1, ncol, 1, 2 + nstr))
prop[..., 0] = 10.0 ** rng.uniform(-5, 0.7, (1, ncol, 1))
if nstr <= 16:
    prop[..., 1] = rng.uniform(0, 0.99, (1, ncol, 1))
    g = rng.uniform(0, 0.85, (1, ncol, 1))
    for l in range(nstr):
        prop[..., 2 + l] = g ** (l + 1)
else:
    prop[..., 1] = rng.uniform(0.8, 0.9999, (1, ncol, 1))
    w = rng.uniform(0, 1, (1, ncol, 1))
    gb = rng.uniform(0.6, 0.85, (1, ncol, 1))
    for l in range(nstr):
        prop[..., 2 + l] = w * 0.75 ** (l + 1) + (1 - w) * gb ** (l + 1)
bc = {"albedo": rng.uniform(0, 1, (1, ncol)), "fbeam": np.ones((1, ncol)),
      "umu0": rng.uniform(0.05, 1.0, (1, ncol))}
d = _disort(nstr, 1, 1, ncol)
dev = torch.device("cuda", 0)
ctx = _context(0)
per_wave = 64 if nstr <= 16 else 4
need = np.zeros(ncol, dtype=int)
for k in range(1, 9):
    st = torch.zeros(ncol, dtype=torch.int32, device=dev)
    ctx.set_max_sweeps(k)
    _run(d, prop, bc, status=st)
    torch.cuda.synchronize()
    flag = ((st & _lib.HD_STATUS_EIGEN) != 0).cpu().numpy()
    need[(need == 0) & ~flag] = k
ctx.set_max_sweeps(0)
wmax = need[: ncol // per_wave * per_wave].reshape(-1, per_wave).max(1)
print(f"nstr {nstr} warm {os.environ.get('HD_JACOBI_WARM', '1')}: per layer mean {need.mean():.3f} "
      f"hist {np.bincount(need).tolist()}; wave max mean {wmax.mean():.3f} hist {np.bincount(wmax).tolist()}")
