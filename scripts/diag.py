import sys, numpy as np, torch
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/tests')
from helpers import load_cases, case_bc, rel_err
from test_gpu_parity import _disort, _run
from oracle import oracle_c as oc
d = load_cases()['mix_n16_l10']
prop = d['prop']; nwave, ncol, nlyr, _ = prop.shape
bc = case_bc(d)
for nstr in (16, 8, 4):
  for beam in (True, False):
    for planck in (True, False):
      b = dict(bc)
      if not beam: b.pop('fbeam'); b.pop('umu0')
      ref = oc.forward(prop, b, d['temf'], nstr=nstr, nmom=16, planck=planck, wave_lower=d['wave_lower'], wave_upper=d['wave_upper'])
      dis = _disort(nstr, nlyr, nwave, ncol, nmom=16, planck=planck, wl=d['wave_lower'], wu=d['wave_upper'])
      f = _run(dis, prop, b, d['temf'])
      e = rel_err(f, ref)
      print(nstr, 'beam', beam, 'planck', planck, 'err %.3e' % e.max(), 'argmax', np.unravel_index(e.argmax(), e.shape))
