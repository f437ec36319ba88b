"""SURVEY 8(b) "Threading": modules on several streams and host threads.

pyharp builds one solver module per band (src/radiation/radiation_band.cpp:57-69)
and may drive bands from several streams or threads.  libhdisort keeps one
hd_context per (device, host thread); the modules of a thread share it, and
hd_solve orders each solve behind the context's previous one whatever stream it
ran on, so scratch, status and error flags are never used twice at once.  These
tests enqueue solves asynchronously on two streams (no synchronisation between
them) and from two host threads, and compare every result with the oracle.
"""

import os
import subprocess
import threading

import numpy as np
import pytest
import torch

from helpers import TOL, rel_err, margin

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _batch(seed, nwave, ncol, nlyr, nstr, planck=False):
    rng = np.random.default_rng(seed)
    prop = np.zeros((nwave, ncol, nlyr, 2 + nstr))
    prop[..., 0] = 10.0 ** rng.uniform(-4, 0.7, (nwave, ncol, nlyr))
    prop[..., 1] = rng.uniform(0, 0.99, (nwave, ncol, nlyr))
    g = rng.uniform(0, 0.85, (nwave, ncol, nlyr))
    for l in range(nstr):
        prop[..., 2 + l] = g ** (l + 1)
    bc = {"albedo": rng.uniform(0, 1, (nwave, ncol)), "fbeam": np.ones((nwave, ncol)),
          "umu0": rng.uniform(0.05, 1.0, (nwave, ncol))}
    kw = {}
    if planck:
        from oracle.disort_np import layer2level
        kw["temf"] = layer2level(np.linspace(300, 150, nlyr)[None, :]
                                 + rng.uniform(-5, 5, (ncol, nlyr)))
        bc["btemp"] = np.full((nwave, ncol), 295.0)
        kw["wave_lower"] = np.sort(rng.uniform(10, 2500, nwave))
        kw["wave_upper"] = kw["wave_lower"] + rng.uniform(1, 300, nwave)
    return prop, bc, kw


def _module(nstr, nlyr, nwave, ncol, planck=False, kw=None):
    from pyharp_amd import Disort, DisortOptions
    op = DisortOptions().flags("lamber,quiet,onlyfl" + (",planck" if planck else ""))
    op.nwave(nwave).ncol(ncol)
    if planck:
        op.wave_lower(list(map(float, kw["wave_lower"])))
        op.wave_upper(list(map(float, kw["wave_upper"])))
    op.ds().nlyr, op.ds().nstr, op.ds().nmom = nlyr, nstr, nstr
    return Disort(op)


def _dev(prop, bc, kw):
    dev = torch.device("cuda", 0)
    p = torch.as_tensor(prop, device=dev)
    b = {k: torch.as_tensor(v, device=dev) for k, v in bc.items()}
    t = torch.as_tensor(kw["temf"], device=dev) if "temf" in kw else None
    return p, b, t


def _oracle(oracle_c, prop, bc, kw, nstr, planck=False):
    return oracle_c.forward(prop, bc, kw.get("temf"), nstr=nstr, planck=planck,
                            wave_lower=kw.get("wave_lower"), wave_upper=kw.get("wave_upper"))


@pytest.mark.parametrize("shapes", [((8, 16), 300), ((16, 24), 700)])
def test_two_modules_two_streams(oracle_c, shapes):
    """Two modules (different nstr, multi-chunk sizes) solve asynchronously on two
    torch streams with no synchronisation between the streams; both match the
    oracle.  Without the context's ordering the second call's kernels would
    rewrite the shared scratch while the first call's are still reading it."""
    (na, nb), chunk = shapes
    nlyr = 24
    pa, ba, ka = _batch(11, 4, 300, nlyr, na, planck=True)
    pb, bb, kb = _batch(12, 5, 260, nlyr, nb)
    A = _module(na, nlyr, 4, 300, planck=True, kw=ka)
    B = _module(nb, nlyr, 5, 260)
    dev = torch.device("cuda", 0)
    from pyharp_amd.disort import _context
    ctx = _context(0)
    ctx.set_chunk(chunk)  # every call runs several chunks (three-stream pipeline)
    try:
        ta, tb = _dev(pa, ba, ka), _dev(pb, bb, kb)
        s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
        s1.wait_stream(torch.cuda.current_stream(dev))
        s2.wait_stream(torch.cuda.current_stream(dev))
        sta = torch.empty(4 * 300, dtype=torch.int32, device=dev)
        stb = torch.empty(5 * 260, dtype=torch.int32, device=dev)
        outs = []
        for it in range(3):
            with torch.cuda.stream(s1):
                fa = A.forward(ta[0], ta[1], ta[2], status=sta)
            with torch.cuda.stream(s2):
                fb = B.forward(tb[0], tb[1], status=stb)
            outs.append((fa, fb))
        torch.cuda.synchronize(dev)
    finally:
        ctx.set_chunk(0)
    assert int(sta.max()) & 0x0F == 0 and int(stb.max()) & 0x0F == 0
    ref_a = _oracle(oracle_c, pa, ba, ka, na, planck=True)
    ref_b = _oracle(oracle_c, pb, bb, kb, nb)
    for fa, fb in outs:
        ea = rel_err(fa.cpu().numpy(), ref_a).max()
        eb = rel_err(fb.cpu().numpy(), ref_b).max()
        assert margin(ea) < TOL and margin(eb) < TOL, f"stream A {ea:.3e}, stream B {eb:.3e}"


def test_two_host_threads(oracle_c):
    """Two host threads, each with its own module and (per-thread) context, solve
    concurrently three times each; both match the oracle."""
    nlyr = 30
    cases = [(8, _batch(21, 6, 200, nlyr, 8)), (16, _batch(22, 3, 150, nlyr, 16))]
    results, errors = {}, []

    def work(i):
        try:
            nstr, (prop, bc, kw) = cases[i]
            torch.cuda.set_device(0)
            m = _module(nstr, nlyr, prop.shape[0], prop.shape[1])
            p, b, _ = _dev(prop, bc, kw)
            for _ in range(3):
                results.setdefault(i, []).append(m.forward(p, b).cpu().numpy())
        except Exception as e:  # surfaced in the main thread
            errors.append(repr(e))

    th = [threading.Thread(target=work, args=(i,)) for i in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not errors, errors
    for i, (nstr, (prop, bc, kw)) in enumerate(cases):
        ref = _oracle(oracle_c, prop, bc, kw, nstr)
        for f in results[i]:
            assert margin(rel_err(f, ref).max()) < TOL


def _swap_inputs(band, nwave, ncol, nlyr, nstr):
    """tests/cpp/radiation_band_swap.cpp's inputs()."""
    prop = np.zeros((nwave, ncol, nlyr, 2 + nstr))
    bc, temf = {}, None
    for w in range(nwave):
        for c in range(ncol):
            for l in range(nlyr):
                prop[w, c, l, 0] = 0.02 * (1 + w) * (1 + (l * 7 + c) % 5)
                if band == 0:
                    prop[w, c, l, 1] = 0.5 + 0.04 * ((w + 2 * l + c) % 12)
                    g = 0.1 + 0.05 * ((l + w) % 10)
                    for m in range(1, nstr + 1):
                        prop[w, c, l, 1 + m] = g ** m
    ones = np.ones((nwave, ncol))
    if band == 0:
        bc["fbeam"] = ones
        bc["umu0"] = 0.3 + 0.1 * (np.arange(nwave * ncol) % 7).reshape(nwave, ncol)
        bc["albedo"] = 0.2 * ones
    else:
        temf = np.array([[260.0 - 100.0 * l / nlyr + 5.0 * c for l in range(nlyr + 1)]
                         for c in range(ncol)])
        bc["albedo"] = 0.1 * ones
        bc["btemp"] = 265.0 * ones
    return prop, bc, temf


def test_cpp_radiation_band_swap(oracle_c):
    """The INTEGRATION.md swap (radiation_band.cpp:57-69 with to_harp_amd) compiled
    in tests/cpp/radiation_band_swap.cpp: two bands through torch::nn::AnyModule
    on two host threads, forward(prop, &bc) and forward(prop, &bc, temf)."""
    exe = os.path.join(ROOT, "tests", "cpp", "radiation_band_swap")
    if not os.path.exists(exe):
        subprocess.run([os.path.join(ROOT, "tests", "cpp", "build.sh")], check=True)
    out = subprocess.run([exe], check=True, capture_output=True, text=True,
                         timeout=120).stdout
    nwave, ncol, nlyr, nstr = (7, 6), (3, 2), (12, 9), (8, 4)
    got = [np.full((nwave[b], ncol[b], nlyr[b] + 1, 2), np.nan) for b in range(2)]
    for line in out.strip().splitlines():
        b, w, c, l, up, dn = line.split()
        got[int(b)][int(w), int(c), int(l)] = (float(up), float(dn))
    for b in range(2):
        prop, bc, temf = _swap_inputs(b, nwave[b], ncol[b], nlyr[b], nstr[b])
        wl = 100.0 + 50.0 * np.arange(nwave[b])
        ref = oracle_c.forward(prop, bc, temf, nstr=nstr[b], planck=b == 1,
                               wave_lower=wl, wave_upper=wl + 50.0)
        err = rel_err(got[b], ref).max()
        assert margin(err) < TOL, f"band {b}: max rel err {err:.3e}"
