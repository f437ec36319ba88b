"""pyharp_amd -- MI355X-native drop-in for pyharp's DISORT flux path.

Hot path: pyharp's RT-solver plugin (src/rtsolver/rtsolver.hpp:21-32) calling
pydisort's DisortImpl::forward (examples/amars_sw.cpp:280, amars_lw.cpp:80,
src/radiation/radiation_band.cpp:124-127).  Here the solve runs in
hand-written HIP kernels for gfx950 (libhdisort.so, C-ABI include/hdisort.h).
"""

from .index import IDN, IEX, IPM, ISS, IUP  # noqa: F401
from .rtsolver import RTSolver  # noqa: F401
from .disort import Disort, DisortOptions, night_side_beam  # noqa: F401
from .layer2level import Layer2LevelOptions, layer2level  # noqa: F401
from .scattering import PhaseMomentOptions, scattering_moments  # noqa: F401

__all__ = ["Disort", "DisortOptions", "RTSolver", "layer2level", "Layer2LevelOptions",
           "IEX", "ISS", "IPM", "IUP", "IDN", "PhaseMomentOptions",
           "scattering_moments", "night_side_beam"]
