# small fixed workload for counter collection: one chunk of the C4 shape
# (65 536 solves, nstr=16) or, with PMC_NSTR=32, a 16 384-solve chunk of C5.
import os, sys, torch
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/scripts')
import bench
dev = torch.device('cuda', 0)
from pyharp_amd import Disort, DisortOptions
nstr = int(os.environ.get("PMC_NSTR", "16"))
W, C, L = (8, int(os.environ.get("PMC_C", "8192")), 80) if nstr <= 16 else (4, 4096, 80)
kw = {} if nstr <= 16 else dict(ssa=(0.9, 0.9999), gasym=(0.6, 0.9), umu0=(0.1, 1.0))
prop, bc, _ = bench.make_inputs(list(range(W)), C, L, nstr, False, dev, **kw)
op = DisortOptions().flags('lamber,quiet,onlyfl').nwave(W).ncol(C)
op.ds().nlyr, op.ds().nstr, op.ds().nmom = L, nstr, nstr
d = Disort(op)
# the bench's path: the band sum fused into the solve (PMC_UNFUSED=1: hd_solve)
wts = torch.full((W,), 1.0 / W, dtype=torch.float64, device=dev)
for _ in range(2):
    if os.environ.get("PMC_UNFUSED") == "1":
        out = d.forward(prop, bc)
    else:
        out = d.forward_band(prop, bc, weights=wts)
torch.cuda.synchronize()
print('done', float(out.flatten()[-1]))
