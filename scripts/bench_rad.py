"""Throughput of the intensity path (hd_solve_radiance), not the driver's metric.

    python scripts/bench_rad.py [--ncol 1000] [--ngpoint 16] [--nstr 16] [--nlyr 80]
                                [--numu 8] [--nphi 4] [--ntau 1] [--steps 5]

Workload: the C4 column statistics with a beam, radiances at
numu user cosines x nphi azimuths at ntau user depths (ntau = 1: TOA, the legacy
driver's case, src/rtsolver/rt_solver_disort.cpp_:218-221).  Prints one JSON
line: solves/s (every azimuthal mode of every (g-point, column)), ms/step,
and a subsample check against the radiance oracle.
"""

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ncol", type=int, default=1000)
    ap.add_argument("--ngpoint", type=int, default=16)
    ap.add_argument("--nstr", type=int, default=16)
    ap.add_argument("--nlyr", type=int, default=80)
    ap.add_argument("--numu", type=int, default=8)
    ap.add_argument("--nphi", type=int, default=4)
    ap.add_argument("--ntau", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--chunk", type=int, default=0, help="solves per chunk (0: by scratch budget)")
    a = ap.parse_args()
    from pyharp_amd import Disort, DisortOptions
    dev = torch.device("cuda", 0)
    G, C, L, n = a.ngpoint, a.ncol, a.nlyr, a.nstr
    rng = np.random.default_rng(20250217)
    prop = np.zeros((G, C, L, 2 + n))
    prop[..., 0] = 10.0 ** rng.uniform(-5, np.log10(5.0), (G, C, L))
    prop[..., 1] = rng.uniform(0.0, 0.99, (G, C, L))
    g = rng.uniform(0.0, 0.85, (G, C, L))
    for l in range(n):
        prop[..., 2 + l] = g ** (l + 1)
    bc = {"fbeam": np.ones((G, C)), "umu0": rng.uniform(0.05, 1.0, (G, C)),
          "phi0": rng.uniform(0, 360, (G, C)), "albedo": rng.uniform(0, 1, (G, C))}
    umu = list(np.linspace(-1, 1, a.numu + 2)[1:-1]) if a.numu % 2 else \
        list(np.concatenate([-np.linspace(1, 0.1, a.numu // 2), np.linspace(0.1, 1, a.numu // 2)]))
    phi = list(np.linspace(0, 180, a.nphi))
    utau = list(np.linspace(0.0, 1e-5 * L, a.ntau)) if a.ntau > 1 else [0.0]
    op = DisortOptions().flags("usrtau,usrang,lamber,quiet").nwave(G).ncol(C)
    op.user_mu(umu).user_phi(phi).user_tau(utau)
    op.ds().nlyr, op.ds().nstr, op.ds().nmom = L, n, n
    d = Disort(op)
    if a.chunk:
        from pyharp_amd.disort import _context
        _context(0).set_chunk(a.chunk)
    p = torch.as_tensor(prop, device=dev)
    b = {k: torch.as_tensor(v, device=dev) for k, v in bc.items()}
    for _ in range(a.warmup):
        d.forward(p, b)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        flux = d.forward(p, b)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.steps
    uu = d.get_rad().cpu().numpy()
    # subsample check (oracle: test infrastructure, used here as the checker only)
    from oracle.disort_rad_np import disort_rad_forward
    idx = rng.choice(G * C, 4, replace=False)
    err = 0.0
    for s in idx:
        w, c = divmod(int(s), C)
        sub = {k: v[w:w + 1, c:c + 1] for k, v in bc.items()}
        _, ur = disort_rad_forward(prop[w:w + 1, c:c + 1], sub, nstr=n, umu=umu, phi=phi,
                                   utau=utau)
        err = max(err, np.abs(uu[w, c] - ur[0, 0]).max() / np.abs(ur).max())
    print(json.dumps({"metric": "radiance solves/s (all azimuthal modes)",
                      "value": G * C / dt, "unit": "solves/s", "ms_per_step": dt * 1e3,
                      "chunk": a.chunk or "auto", "config": {"ncol": C, "ngpoint": G, "nstr": n, "nlyr": L, "numu": a.numu,
                                 "nphi": a.nphi, "ntau": len(utau)},
                      "max_rel_err_subsample": err}))


if __name__ == "__main__":
    main()
