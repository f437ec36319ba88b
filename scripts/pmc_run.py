# small fixed workload for counter collection: one 65536-solve chunk of C4 shape
import sys, torch
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/scripts')
import bench
dev = torch.device('cuda', 0)
from pyharp_amd import Disort, DisortOptions
W, C, L, nstr = 8, 8192, 80, 16
prop, bc, _ = bench.make_inputs(list(range(W)), C, L, nstr, False, dev)
op = DisortOptions().flags('lamber,quiet,onlyfl').nwave(W).ncol(C)
op.ds().nlyr, op.ds().nstr, op.ds().nmom = L, nstr, nstr
d = Disort(op)
for _ in range(2):
    out = d.forward(prop, bc)
torch.cuda.synchronize()
print('done', float(out[0, 0, -1, 0]))
