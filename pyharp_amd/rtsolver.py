"""RT-solver plugin surface (mirror of src/rtsolver/rtsolver.hpp:21-32).

``RTSolver.forward(prop, bc, temf=None)`` is the contract pyharp's radiation
band loop calls (src/radiation/radiation_band.cpp:123-128).  The base class
raises, exactly like ``RTSolverImpl::forward``.
"""

from __future__ import annotations


class RTSolver:
    """Common base class for all RT solvers."""

    def forward(self, prop, bc, temf=None):
        raise RuntimeError("RTSolverImpl::forward: not implemented")

    def __call__(self, prop, bc, temf=None):
        return self.forward(prop, bc, temf)
