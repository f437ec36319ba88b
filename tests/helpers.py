"""Shared test helpers: golden fixtures and the flux error metric."""

import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

# Error metric: per column, |F - F_ref| / max(|F_ref|, FLOOR * scale)
# with scale = max |F_ref| over that column's levels and both directions.  Fluxes
# below FLOOR*scale are therefore compared absolutely at FLOOR*scale*tol.
FLOOR = 1.0e-6
TOL = 1.0e-6  # north-star bound: max |dF|/F < 1e-6


# Parity margins (tests/conftest.py writes them to $HD_MARGINS_OUT at the end of the
# session): every GPU-vs-oracle assertion `assert margin(err) < TOL` records its error
# under the running test's node id, so a speed change that eats tolerance shows up
# as a number, not only as a pass/fail.
MARGINS = []


def margin(err):
    err = float(np.max(err))
    node = os.environ.get("PYTEST_CURRENT_TEST", "?").rsplit(" (", 1)[0]
    MARGINS.append((node, err))
    return err


def rel_err(f, ref, floor=FLOOR):
    f = np.asarray(f, np.float64)
    ref = np.asarray(ref, np.float64)
    scale = np.abs(ref).max(axis=(-2, -1), keepdims=True)
    denom = np.maximum(np.abs(ref), floor * np.maximum(scale, 1e-300))
    return np.abs(f - ref) / denom


def load_cases():
    z = np.load(os.path.join(GOLDEN, "cases.npz"))
    cases = {}
    for key in z.files:
        name, field = key.split("/", 1)
        cases.setdefault(name, {})[field] = z[key]
    return cases


def case_bc(d):
    return {k[3:]: v for k, v in d.items() if k.startswith("bc_")}


def disotest():
    with open(os.path.join(GOLDEN, "disotest1.json")) as f:
        return json.load(f)
