"""Per-phase wave cycles of the nstr-16 layer kernel (debug variant built from an
instrumented copy of hd_kernels.hip: HD_TICK(k) adds the s_memtime delta of phase k,
lane 0 of each wave, into d_phase[k]; read by hd_debug_phase).  One 32 768-solve chunk
(C4 distributions) run alone.

    HD_LIB_PATH=mb/inst/libhdisort.so python scripts/micro/phase_time.py
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import bench  # noqa: E402
from pyharp_amd import Disort, DisortOptions, _lib  # noqa: E402
from pyharp_amd.disort import _context  # noqa: E402

NAMES = ["", "assembly (loads, Legendre)", "chol L + beam vectors", "Planck vectors",
         "chol C + X = L^T C", "park L in LDS", "Jacobi + polish", "k, 1/k",
         "beam part 1 + L reload", "beam part 2", "Delta^1/2 (expm1)", "Psi^T -> LDS",
         "Omega = L B K^-1 D^1/2", "A- (Gram, chol, inverse)", "A+ (LDS, Gram, chol, inverse)",
         "stores R~ T~ S~", "  first loads (tau, ssa, f)", "  umu0, fbeam", "  Legendre loop"]
TEAM = ["", "assembly (loads, Legendre)", "chol S- (L)", "beam vectors", "Planck, L^-T",
        "chol S+ (C), B0", "warm start (MFMA), C^-T", "Jacobi", "k, Delta, Gamma",
        "MFMA W, U, U^T", "beam", "Psi, Omega, Grams (MFMA)", "A- (chol, inverse, MFMA)",
        "A+ (chol, inverse, MFMA)", "", "stores R~ T~ S~", "", "", ""]
dev = torch.device("cuda", 0)
nstr = int(os.environ.get("PHASE_NSTR", "16"))
if nstr > 16:  # C5-like: one 16 384-solve chunk of the team path
    NAMES = TEAM
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
lib = _lib.load()
buf = (ctypes.c_ulonglong * 32)()
d.forward(prop, bc)
torch.cuda.synchronize()
lib.hd_debug_phase(buf, 1)
d.forward(prop, bc)
torch.cuda.synchronize()
lib.hd_debug_phase(buf, 1)
waves = W * C * L // (64 if nstr <= 16 else 4)
tot = sum(buf[k] for k in range(1, 19))
print(f"{waves} waves; cycles per wave by phase (s_memtime):")
for k in [k for k in list(range(1, 16)) + [16, 17, 18] if k < len(NAMES) and NAMES[k]]:
    print(f"  {k:2d} {NAMES[k]:32s} {buf[k] / waves:9.0f}  {100.0 * buf[k] / tot:5.1f} %")
print(f"  total {tot / waves:.0f}")
