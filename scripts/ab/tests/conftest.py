"""GPU tests of the kernel variants that were measured and not kept (DESIGN.md
section 9).  They are compiled only into the A/B build of the library:

    bash scripts/ab/build_variant.sh ab          # -> ab_libs/libhdisort_ab.so
    python -m pytest scripts/ab/tests -m gpu      # (scripts/gpu.sh step abtests)

Each test runs the product's default kernel in this process (the in-tree library)
and the variant in a child process on the A/B library (HD_LIB_PATH).  Not part of
`pytest tests/`: the product library carries none of these kernels."""
import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(HERE)))
for p in (ROOT, os.path.join(ROOT, "tests"), HERE):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); runs the HIP path")


@pytest.fixture(scope="session")
def ab_lib():
    path = os.environ.get("HD_AB_LIB", os.path.join(ROOT, "ab_libs", "libhdisort_ab.so"))
    if not os.path.exists(path):
        pytest.skip(f"A/B library {path} not built (bash scripts/ab/build_variant.sh ab)")
    return path
