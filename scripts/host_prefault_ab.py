"""A/B of the host-array path's output allocation (Disort.forward on CPU tensors):
torch.empty (the D2H copies fault the fresh pages in) against torch.zeros (pages
faulted in by torch's parallel fill before the call).  C4 shape.

    python scripts/host_prefault_ab.py [--reps 3]
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from pyharp_amd import Disort, DisortOptions, _lib  # noqa: E402
from pyharp_amd.disort import _context  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    W, C, L, n = 64, 10000, 80, 16
    dev = torch.device("cuda", 0)
    prop_d, bc_d, _ = bench.make_inputs(list(range(W)), C, L, n, False, dev)
    hp = prop_d.cpu()
    hb = {k: v.cpu() for k, v in bc_d.items()}
    del prop_d, bc_d
    op = DisortOptions().flags("lamber,quiet,onlyfl").nwave(W).ncol(C)
    op.ds().nlyr, op.ds().nstr, op.ds().nmom = L, n, n
    d = Disort(op)
    ctx = _context(0)
    cfg = _lib.HdConfig(nstr=n, nmom=n, nlyr=L, nprop=2 + n,
                        flags=_lib.HD_FLAG_LAMBER | _lib.HD_FLAG_ONLYFL)
    inp = _lib.HdInputs(nwave=W, ncol=C, prop=hp.data_ptr(), fbeam=hb["fbeam"].data_ptr(),
                        umu0=hb["umu0"].data_ptr(), albedo=hb["albedo"].data_ptr())
    out = {}
    for name, alloc in (("empty", torch.empty), ("zeros", torch.zeros),
                        ("empty", torch.empty), ("zeros", torch.zeros)):
        ts = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            f = alloc((W, C, L + 1, 2), dtype=torch.float64)
            t1 = time.perf_counter()
            ctx.solve_host(cfg, inp, f.data_ptr())
            t2 = time.perf_counter()
            ts.append((t2 - t0, t1 - t0))
            del f
        ts.sort()
        out.setdefault(name, []).append({"ms_total": round(ts[len(ts) // 2][0] * 1e3, 2),
                                         "ms_alloc": round(ts[len(ts) // 2][1] * 1e3, 2)})
    ref = d.forward(hp, hb)  # the module's own path, for the record
    print(json.dumps({"host_prefault_ab": out, "torch_threads": torch.get_num_threads(),
                      "flux_sum": float(ref.sum())}))


if __name__ == "__main__":
    main()
