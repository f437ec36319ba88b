"""Probe one solve (from find_worst's dump): GPU vs the C restatement for the solve as
dumped and with one input perturbed at a time (a layer's ssa, or umu0), to locate the
layer / input behind a large deviation.

    python scripts/micro/probe_solve.py WORST.npz
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from helpers import rel_err  # noqa: E402
from oracle import oracle_c  # noqa: E402
from pyharp_amd import Disort, DisortOptions  # noqa: E402

z = np.load(sys.argv[1])
dev = torch.device("cuda", 0)
L, nstr = z["prop"].shape[0], z["prop"].shape[1] - 2
oracle_c.build()
op = DisortOptions().flags("lamber,quiet,onlyfl").nwave(1).ncol(1)
op.ds().nlyr, op.ds().nstr, op.ds().nmom = L, nstr, nstr
d = Disort(op)


def run(prop, umu0):
    bc = {"fbeam": np.array([[float(z["fbeam"])]]), "umu0": np.array([[umu0]]),
          "albedo": np.array([[float(z["albedo"])]])}
    p = prop[None, None]
    f = d.forward(torch.as_tensor(p, device=dev), {k: torch.as_tensor(v, device=dev)
                                                   for k, v in bc.items()}).cpu().numpy()
    ref = oracle_c.forward(p, bc, None, nstr=nstr)
    return rel_err(f, ref).max()


prop0 = z["prop"].copy()
mu0 = float(z["umu0"])
e0 = run(prop0, mu0)
print(f"as dumped: {e0:.3e}")
for eps in (1e-6, 1e-4):
    print(f"umu0 * (1 + {eps}): {run(prop0, mu0 * (1 + eps)):.3e}")
for l in range(L):
    p = prop0.copy()
    p[l, 1] *= 1 - 1e-3
    e = run(p, mu0)
    if e < 0.1 * e0:
        print(f"layer {l} ssa * (1 - 1e-3): {e:.3e}")
