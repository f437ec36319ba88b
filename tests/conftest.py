import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); runs the HIP path")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def oracle_c():
    from oracle import oracle_c as oc
    oc.build()
    return oc


def pytest_sessionfinish(session, exitstatus):
    """With HD_MARGINS_OUT set (scripts/gpu.sh does), write every recorded parity
    margin (tests/helpers.py margin()): per test the largest error and its tolerance
    ratio, sorted worst first."""
    out = os.environ.get("HD_MARGINS_OUT")
    if not out:
        return
    import json
    import helpers
    worst = {}
    for node, err in helpers.MARGINS:
        worst[node] = max(err, worst.get(node, 0.0))
    rows = sorted(({"test": k, "max_rel_err": v, "tol": helpers.TOL, "frac_of_tol": v / helpers.TOL}
                   for k, v in worst.items()), key=lambda r: -r["max_rel_err"])
    os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
    with open(out, "w") as f:
        json.dump({"n_tests": len(rows), "n_checks": len(helpers.MARGINS), "worst": rows[:1],
                   "tests": rows}, f, indent=1)
