"""PCIe-inclusive throughput of the C4 step when the caller hands over HOST arrays
(pydisort's CPU-tensor contract): hd_solve_band_host (include/hdisort.h) copies
prop and the boundary arrays to the device, solves and sums the band there, and
copies the band flux back.  The headline `value` of bench.py is the device-resident
rate; this is the number DESIGN.md quotes beside it.

    python scripts/bench_host.py [--steps K] [--pinned]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from pyharp_amd import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--pinned", action="store_true", help="page-locked host arrays")
    a = ap.parse_args()
    W, C, L, nstr = 64, 10000, 80, 16
    dev = torch.device("cuda", 0)
    prop_d, bc_d, _ = bench.make_inputs(list(range(W)), C, L, nstr, False, dev)

    def host(t):
        h = torch.empty(t.shape, dtype=t.dtype, pin_memory=a.pinned)
        h.copy_(t)
        return h.numpy()

    prop = host(prop_d)
    bc = {k: host(v) for k, v in bc_d.items()}
    del prop_d, bc_d
    torch.cuda.empty_cache()
    lib = _lib.load()
    ctx = ctypes.c_void_p()
    assert lib.hd_context_create(ctypes.byref(ctx), 0) == 0
    p = lambda x: x.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    cfg = _lib.HdConfig(nstr, nstr, L, 2 + nstr, _lib.HD_FLAG_LAMBER | _lib.HD_FLAG_ONLYFL)
    inp = _lib.HdInputs(W, C, p(prop), p(bc["fbeam"]), p(bc["umu0"]), p(bc["albedo"]),
                        None, None, None, None, None, None, None)
    w = np.full(W, 1.0 / W)
    bflux = np.zeros((C, L + 1, 2))
    run = lambda: lib.hd_solve_band_host(ctx, ctypes.byref(cfg), ctypes.byref(inp), p(w),  # noqa: E731
                                         p(bflux), None, None)
    assert run() == 0, lib.hd_last_error(ctx)
    t = []
    for _ in range(a.steps):
        t0 = time.perf_counter()
        rc = run()
        t.append(time.perf_counter() - t0)
        assert rc == 0
    ms = 1e3 * min(t)
    lib.hd_context_destroy(ctx)
    print(json.dumps({"metric": "DISORT column-solves/sec, host arrays in and out (PCIe-inclusive)",
                      "value": round(W * C / (ms / 1e3), 1), "unit": "column-solves/s",
                      "ms_per_call": round(ms, 2), "host_bytes_in": int(prop.nbytes + 3 * W * C * 8),
                      "pinned": a.pinned, "entry": "hd_solve_band_host",
                      "config": {"workload": "C4: 10000 columns x 64 g-points, nstr=16, nlyr=80"}}))


if __name__ == "__main__":
    main()
