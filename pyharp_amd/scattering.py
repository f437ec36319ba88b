"""Phase-function moments for ``prop[..., IPM:]`` (pydisort's
``disort::scattering_moments(nmom, PhaseMomentOptions().type(...))``, used at
``tests/test_disort.cpp:44-47``): chi_1..chi_nmom of the phase functions whose
Legendre moments are closed-form.  Host-side setup; no solver arithmetic.
"""

from __future__ import annotations

import torch

kIsotropic = "isotropic"
kRayleigh = "rayleigh"
kHenyeyGreenstein = "henyey_greenstein"


class PhaseMomentOptions:
    def __init__(self):
        self._type = kIsotropic
        self._gg = 0.0

    def type(self, *v):
        if v:
            if v[0] not in (kIsotropic, kRayleigh, kHenyeyGreenstein):
                raise RuntimeError(f"scattering_moments: unknown phase function {v[0]!r}")
            self._type = v[0]
            return self
        return self._type

    def gg(self, *v):
        if v:
            self._gg = float(v[0])
            return self
        return self._gg


def scattering_moments(nmom: int, op: PhaseMomentOptions | None = None) -> torch.Tensor:
    """(nmom,) float64: isotropic 0, Rayleigh chi_2 = 0.1, Henyey-Greenstein g^l."""
    op = op or PhaseMomentOptions()
    m = torch.zeros(nmom, dtype=torch.float64)
    if op.type() == kRayleigh and nmom >= 2:
        m[1] = 0.1
    elif op.type() == kHenyeyGreenstein:
        m[:] = op.gg() ** torch.arange(1, nmom + 1, dtype=torch.float64)
    return m
