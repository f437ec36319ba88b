"""Layer kernel alone: one 32 768-solve chunk of the C4 distributions (the chunk's
layer kernel runs with nothing beside it), hd_context timing over 5 calls.

    [HD_LIB_PATH=mb/NAME/libhdisort.so] python scripts/micro/layer_alone.py [TAG]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import bench  # noqa: E402
from pyharp_amd import Disort, DisortOptions  # noqa: E402
from pyharp_amd.disort import _context  # noqa: E402

dev = torch.device("cuda", 0)
nstr = int(os.environ.get("LAYER_NSTR", "16"))
if nstr > 16:  # C5-like team-path chunk (16 384 solves)
    W, C, L = 4, 4096, 80
    prop, bc, _ = bench.make_inputs(list(range(W)), C, L, nstr, False, dev, ssa=(0.9, 0.9999),
                                    gasym=(0.6, 0.9), umu0=(0.1, 1.0))
else:
    W, C, L = 4, 8192, 80
    prop, bc, _ = bench.make_inputs(list(range(W)), C, L, nstr, False, dev)
op = DisortOptions().flags("lamber,quiet,onlyfl").nwave(W).ncol(C)
op.ds().nlyr, op.ds().nstr, op.ds().nmom = L, nstr, nstr
d = Disort(op)
ctx = _context(0)
ctx.set_chunk(W * C)
out = d.forward(prop, bc)
torch.cuda.synchronize()
sweeps = int(os.environ.get("HD_MAX_SWEEPS", "0"))
if sweeps:  # debug cap on the Jacobi sweeps (the results are then not converged)
    ctx.set_max_sweeps(sweeps)
lay, swp = [], []
for _ in range(5):
    ctx.set_timing(True)
    try:
        out = d.forward(prop, bc)
    except RuntimeError:  # capped sweeps flag HD_STATUS_EIGEN
        pass
    torch.cuda.synchronize()
    tm = ctx.timing()
    lay.append(tm.layer_ms)
    swp.append(tm.sweep_ms)
lay.sort()
swp.sort()
print(f"{sys.argv[1] if len(sys.argv) > 1 else 'cur'} (max sweeps {sweeps or 'default'}): layer alone {lay[2]:.3f} ms (min {lay[0]:.3f}), "
      f"sweep+backsub {swp[2]:.3f} ms, checksum {float(out.sum()):.12e}")
