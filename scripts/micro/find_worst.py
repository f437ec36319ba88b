"""Every solve of a bench workload (C4 by default, or a g-point range of it): the GPU
path against the C restatement, per (g-point, column), in slabs of 8 g-points.  Prints
the worst solves and the error histogram; dumps the worst solve's inputs and both flux
profiles.

    python scripts/micro/find_worst.py OUT.npz [G0 G1] [NCOL] [CONFIG]
"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import bench  # noqa: E402
from helpers import rel_err  # noqa: E402
from oracle import oracle_c  # noqa: E402
from pyharp_amd import Disort, DisortOptions  # noqa: E402

out_path = sys.argv[1]
g0 = int(sys.argv[2]) if len(sys.argv) > 2 else 0
g1 = int(sys.argv[3]) if len(sys.argv) > 3 else 64
config = sys.argv[5] if len(sys.argv) > 5 else "c4"
cfg = bench.CONFIGS[config]
ncol = int(sys.argv[4]) if len(sys.argv) > 4 and int(sys.argv[4]) > 0 else cfg["ncol"]
G = cfg["ngpoint"]
dev = torch.device("cuda", 0)
L, nstr = cfg["nlyr"], cfg["nstr"]
oracle_c.build()
errs, worst = [], (-1.0, None)
t0 = time.time()
for a in range(g0, g1, 8):
    gp = list(range(a, min(a + 8, g1)))
    W = len(gp)
    if cfg.get("aerosol"):
        prop, bc, _ = bench.make_aerosol_inputs(gp, G, ncol, L, nstr, dev, umu0=cfg["umu0"])
    else:
        prop, bc, _ = bench.make_inputs(gp, ncol, L, nstr, False, dev, ssa=cfg["ssa"],
                                        gasym=cfg["g"], umu0=cfg["umu0"])
    op = DisortOptions().flags("lamber,quiet,onlyfl").nwave(W).ncol(ncol)
    op.ds().nlyr, op.ds().nstr, op.ds().nmom = L, nstr, nstr
    f = Disort(op).forward(prop, bc).cpu().numpy()
    p = prop.cpu().numpy()
    b = {k: v.cpu().numpy() for k, v in bc.items()}
    ref = oracle_c.forward(p, b, None, nstr=nstr, nmom=p.shape[-1] - 2, nthreads=16)
    e = rel_err(f, ref).max(axis=(-2, -1))  # (W, ncol)
    errs.append(e.ravel())
    k = int(np.argmax(e))
    w, c = divmod(k, ncol)
    if e[w, c] > worst[0]:
        worst = (float(e[w, c]), dict(g=gp[w], col=c, prop=p[w, c], fbeam=b["fbeam"][w, c],
                                      umu0=b["umu0"][w, c], albedo=b["albedo"][w, c],
                                      gpu=f[w, c], ref=ref[w, c]))
    print(f"g {gp[0]}..{gp[-1]}: max {e.max():.3e} (g {gp[w]} col {c}), {time.time() - t0:.0f} s",
          flush=True)
e = np.concatenate(errs)
print(f"{e.size} solves: max {e.max():.3e} at g {worst[1]['g']} col {worst[1]['col']}; "
      f"> 1e-8: {int((e > 1e-8).sum())}, > 1e-9: {int((e > 1e-9).sum())}, "
      f"> 1e-10: {int((e > 1e-10).sum())}; median {np.median(e):.2e}")
np.savez(out_path, err=e, **{k: v for k, v in worst[1].items()})
