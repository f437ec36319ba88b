import sys, numpy as np, torch, traceback
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/tests')
from helpers import rel_err
from test_gpu_parity import _disort, _run, _random_batch
from oracle import oracle_c as oc
nstr = int(sys.argv[1]); planck = sys.argv[2] == '1'
rng = np.random.default_rng(1000 + nstr + 100 * planck)
nwave, ncol, nlyr = 4, 8, 40
prop, bc, kw = _random_batch(rng, nwave, ncol, nlyr, nstr, planck)
ref = oc.forward(prop, bc, kw.get('temf'), nstr=nstr, planck=planck, wave_lower=kw.get('wave_lower'), wave_upper=kw.get('wave_upper'))
d = _disort(nstr, nlyr, nwave, ncol, planck=planck, wl=kw.get('wave_lower'), wu=kw.get('wave_upper'))
st = torch.zeros(nwave*ncol, dtype=torch.int32, device='cuda')
dev = torch.device('cuda', 0)
try:
    p = torch.as_tensor(prop, device=dev)
    b = {k: torch.as_tensor(v, device=dev) for k, v in bc.items()}
    t = None if kw.get('temf') is None else torch.as_tensor(kw['temf'], device=dev)
    f = d.forward(p, b, t, status=st)
    torch.cuda.synchronize()
    print('status', st.cpu().numpy())
    f = f.cpu().numpy()
    e = rel_err(f, ref)
    print('err', e.max(), 'nan', np.isnan(f).sum())
except Exception as ex:
    traceback.print_exc()
