import time, numpy as np, torch, sys
sys.path.insert(0, '/root/repo')
from pyharp_amd import Disort, DisortOptions
from pyharp_amd.disort import _context
C, W, L, nstr = int(sys.argv[1]) if len(sys.argv)>1 else 10000, 64, 80, 16
dev = torch.device('cuda',0)
g = torch.Generator(device=dev); g.manual_seed(1)
prop = torch.zeros((W,C,L,2+nstr), dtype=torch.float64, device=dev)
prop[...,0] = 10**(torch.rand((W,C,L),generator=g,device=dev,dtype=torch.float64)*5.7-5)
prop[...,1] = torch.rand((W,C,L),generator=g,device=dev,dtype=torch.float64)*0.99
gg = torch.rand((W,C,L),generator=g,device=dev,dtype=torch.float64)*0.85
for l in range(nstr): prop[...,2+l] = gg**(l+1)
bc = {'fbeam': torch.ones((W,C),dtype=torch.float64,device=dev), 'umu0': 0.05+0.95*torch.rand((W,C),generator=g,device=dev,dtype=torch.float64), 'albedo': torch.rand((W,C),generator=g,device=dev,dtype=torch.float64)}
op = DisortOptions().flags('lamber,quiet,onlyfl').nwave(W).ncol(C)
op.ds().nlyr, op.ds().nstr, op.ds().nmom = L, nstr, nstr
d = Disort(op)
out = d.forward(prop, bc); torch.cuda.synchronize()
ctx = _context(0)
for it in range(3):
    ctx.set_timing(True); t=time.time(); out = d.forward(prop, bc); torch.cuda.synchronize(); dt=time.time()-t
    tm = ctx.timing()
    print(f"solves {W*C} time {dt*1e3:.1f} ms  -> {W*C/dt:.3e} solves/s ; layer {tm.layer_ms:.1f} ms sweep {tm.sweep_ms:.1f} ms ({tm.layer_launches} chunks)")
print('finite', bool(torch.isfinite(out).all()))
