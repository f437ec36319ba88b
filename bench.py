"""Benchmark of the DISORT flux hot path on MI355X (driver contract).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c4|c5|c1|c3|c3l] [--planck]
                    [--ncol C] [--ngpoint G]

Default workload (BASELINE.json configs[3], SURVEY.md 8(d) "C4 GCM", the
configuration the metric is quoted on): 1e4 synthetic columns x 64 g-points,
nstr=16, nmom=16 (Henyey-Greenstein chi_l = g^l), nlyr=80, tau log-uniform
[1e-5, 5], omega in [0, 0.99], g in [0, 0.85], umu0 in [0.05, 1], albedo in
[0, 1], fbeam = 1 (``--planck`` adds thermal emission, T 150-300 K).
``--config c5`` is SURVEY 8(d) "C5 aerosol" (BASELINE.json configs[4], "h2so4 +
s8_k_fuller phase moments"): 1e3 columns x 64 spectral points, nstr=32, nmom=32,
nlyr=80, umu0 in [0.1, 1]; prop is assembled on the device (untimed) by the
band loop's mixing (hd_band_loop_optics, radiation_band.cpp:86-116) from the
reference's s8_k_fuller.txt and h2so4.txt tables with Henyey-Greenstein
asymmetry tables (g 0.6-0.85 for S8, 0.75 for H2SO4: the tables carry none),
the amars_sw aerosol profile regridded to 80 layers and scaled per column.
``--config c5s`` is the round-1/2 synthetic C5 (omega in [0.9, 0.9999], g in
[0.6, 0.9]).
One step = one flux solve of every (g-point, column) pair of the rank's shard
+ the g-weighted band flux (C, L+1, 2) -- fused into the solve
(hd_solve_band: the per-g fluxes are never stored; ``--no-fuse`` = hd_solve
writing them + hd_band_flux) -- all-reduced over ranks.  Inputs are generated on the device before the timed
region (seeded per g-point, so the global problem does not depend on N).
Spectral sharding: rank r owns g-points {g : g mod N == r} (fixed global
problem -> "scaling": "strong").

Printed (rank 0): one JSON line with the contract fields plus
  roofline      dominant kernel (the layer-setup kernel), algorithmic FLOP per
                launch / average launch time from HIP events on the solve stream
  cpu_baseline  oracle/ C restatement (a port of the DISORT algorithm, not
                cdisort, which is absent) timed on the host cores, N=1 only
  max_rel_err   GPU vs that CPU restatement on a subsample of the workload
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "DISORT column-solves/sec (nstr=16, nlyr=80); max |dF|/F vs cdisort"
FP64_PEAK_TFLOPS = 78.6  # MI355X: 256 CU x 2.4 GHz x 128 FP64 FLOP/clk (vector = matrix)
HBM_PEAK_GBS = 8000.0


def algorithmic_flop(nstr: int, nlyr: int, planck: bool):
    """SURVEY.md 8(d) convention: per solve L*(10.5 n^3 + 12 n^2) (+ L*(2/3 n^3 + 4 n^2) planck).

    Split per kernel: per-layer setup (assembly 1.5n^3 + eigen 3.625n^3 + beam
    LU 2/3 n^3, + Planck LU) -> hd_layer_kernel; boundary sweep (14/3 n^3 +
    12 n^2) -> hd_sweep_kernel.
    """
    n = float(nstr)
    k1 = nlyr * (1.5 + 3.625 + 2.0 / 3.0) * n ** 3
    k2 = nlyr * (14.0 / 3.0 * n ** 3 + 12.0 * n ** 2)
    total = nlyr * (10.5 * n ** 3 + 12.0 * n ** 2)
    if planck:
        k1 += nlyr * (2.0 / 3.0 * n ** 3 + 4.0 * n ** 2)
        total += nlyr * (2.0 / 3.0 * n ** 3 + 4.0 * n ** 2)
    return total, k1, k2


CONFIGS = {
    # name: ncol, ngpoint, nstr, nlyr, (ssa lo, hi), (g lo, hi), (umu0 lo, hi), label
    "c4": dict(ncol=10000, ngpoint=64, nstr=16, nlyr=80, ssa=(0.0, 0.99), g=(0.0, 0.85),
               umu0=(0.05, 1.0), label="C4 GCM batch"),
    "c5": dict(ncol=1000, ngpoint=64, nstr=32, nlyr=80, aerosol=True, umu0=(0.1, 1.0),
               label="C5 high-scatter aerosol (s8 + h2so4 band-loop optics, HG moments)"),
    "c5s": dict(ncol=1000, ngpoint=64, nstr=32, nlyr=80, ssa=(0.9, 0.9999), g=(0.6, 0.9),
                umu0=(0.1, 1.0), label="C5 high-scatter aerosol (synthetic omega, HG g)"),
    # thermal, non-scattering (SURVEY 8(d) C1 amars_lw ck and C3 line-by-line)
    "c1": dict(ncol=1, ngpoint=16, nstr=8, nlyr=40, lw=True, tau=(1e-4, 20.0), band=(1.0, 150.0),
               label="C1 amars_lw ck (synthetic k)"),
    "c3": dict(ncol=1, ngpoint=19990, nstr=8, nlyr=40, lw=True, tau=(1e-5, 5.0),
               band=(1.0, 2000.0), label="C3 line-by-line (synthetic k)"),
    # BASELINE.json configs[2] "~1e5 spectral points": 0.1 cm^-1 bins tiling [1, 10001]
    "c3l": dict(ncol=1, ngpoint=100000, nstr=8, nlyr=40, lw=True, tau=(1e-5, 5.0),
                band=(1.0, 10001.0), label="C3 line-by-line 1e5 bins (synthetic k)"),
}


def make_lw_inputs(gpoints, ngpoint, ncol, nlyr, nstr, band, tau, dev, seed=20250217):
    """Thermal, omega = 0: tau log-uniform, T linear 250 -> 150 K
    bottom -> top, temf = layer2level (4th order), albedo 0 (even g) / 1 (odd g),
    btemp = T_surface, spectral bins tiling `band` (ck: every g spans the band)."""
    f64 = torch.float64
    W = len(gpoints)
    prop = torch.zeros((W, ncol, nlyr, 2 + nstr), dtype=f64, device=dev)
    for i, g in enumerate(gpoints):
        gen = torch.Generator(device=dev)
        gen.manual_seed(seed * 1000 + int(g))
        u = torch.rand((ncol, nlyr), generator=gen, dtype=f64, device=dev)
        prop[i, ..., 0] = 10.0 ** (np.log10(tau[0]) + u * np.log10(tau[1] / tau[0]))
    tl = torch.linspace(250.0, 150.0, nlyr, dtype=f64, device=dev)[None, :].expand(ncol, nlyr)
    from pyharp_amd import layer2level
    temf = layer2level(tl.contiguous())
    alb = torch.tensor([float(g % 2) for g in gpoints], dtype=f64, device=dev)
    bc = {"albedo": alb[:, None].expand(W, ncol).contiguous(),
          "btemp": temf[:, 0][None, :].expand(W, ncol).contiguous()}
    return prop, bc, temf


def make_inputs(gpoints, ncol, nlyr, nstr, planck, dev, seed=20250217, ssa=(0.0, 0.99),
                gasym=(0.0, 0.85), umu0=(0.05, 1.0)):
    """Synthetic inputs (SURVEY 8(d) distributions) for the given g-points, on `dev`."""
    nmom = nstr
    W = len(gpoints)
    f64 = torch.float64
    prop = torch.empty((W, ncol, nlyr, 2 + nmom), dtype=f64, device=dev)
    bc = {k: torch.empty((W, ncol), dtype=f64, device=dev) for k in ("fbeam", "umu0", "albedo")}
    if planck:
        bc["btemp"] = torch.empty((W, ncol), dtype=f64, device=dev)
    for i, g in enumerate(gpoints):
        gen = torch.Generator(device=dev)
        gen.manual_seed(seed * 1000 + int(g))
        r = lambda *shape: torch.rand(shape, generator=gen, dtype=f64, device=dev)  # noqa: E731
        prop[i, ..., 0] = 10.0 ** (r(ncol, nlyr) * np.log10(5.0 / 1e-5) - 5.0)
        prop[i, ..., 1] = ssa[0] + (ssa[1] - ssa[0]) * r(ncol, nlyr)
        gg = gasym[0] + (gasym[1] - gasym[0]) * r(ncol, nlyr)
        for l in range(nmom):
            prop[i, ..., 2 + l] = gg ** (l + 1)
        bc["fbeam"][i] = 1.0
        bc["umu0"][i] = umu0[0] + (umu0[1] - umu0[0]) * r(ncol)
        bc["albedo"][i] = r(ncol)
        if planck:
            bc["btemp"][i] = 300.0
    temf = None
    if planck:
        gen = torch.Generator(device=dev)
        gen.manual_seed(seed)
        tl = torch.linspace(300.0, 150.0, nlyr, dtype=f64, device=dev)[None, :] + \
            5.0 * (torch.rand((ncol, nlyr), generator=gen, dtype=f64, device=dev) - 0.5)
        from pyharp_amd import layer2level
        temf = layer2level(tl)
    return prop, bc, temf


def make_aerosol_inputs(gpoints, ngpoint, ncol, nlyr, nstr, dev, seed=20250217,
                        umu0=(0.1, 1.0)):
    """C5 through the band loop (hd_band_loop_optics, radiation_band.cpp:86-116): S8 and
    H2SO4 from the reference's tables (tests/golden/data, the reference's data/), HG
    asymmetry tables, the amars_sw aerosol profile on nlyr layers with a per-column
    concentration scale log-uniform in [0.3, 30]; spectral point g = wavenumber
    linspace(2000, 50000, ngpoint)[g] (the amars_sw band)."""
    from examples.amars_sw import atmosphere
    from pyharp_amd.opacity import (AttenuatorOptions, H2SO4Simple, S8Fuller,
                                    add_resource_directory, band_loop_optics)
    add_resource_directory(os.path.join(ROOT, "tests", "golden", "data"))
    op = AttenuatorOptions().species_names(["S8", "H2SO4"]).species_weights([256.e-3, 98.e-3])
    s8 = S8Fuller(op.copy().species_ids([0]).opacity_files(["s8_k_fuller.txt"]))
    h2 = H2SO4Simple(op.copy().species_ids([1]).opacity_files(["h2so4.txt"]))
    s8.set_asymmetry(np.linspace(0.6, 0.85, s8.kwave.numel()))
    h2.set_asymmetry(0.75)
    conc0, _, dz, _ = atmosphere(nlyr)
    rng = np.random.default_rng(seed)
    scale = 10.0 ** rng.uniform(np.log10(0.3), np.log10(30.0), (ncol, 1, 1))
    conc = torch.as_tensor(conc0 * scale, device=dev)
    wave = np.linspace(2000.0, 50000.0, ngpoint)[list(gpoints)]
    prop = band_loop_optics([s8, h2], conc, torch.as_tensor(dz, device=dev),
                            {"wavenumber": torch.as_tensor(wave, device=dev)}, nstr)
    W = len(gpoints)
    f64 = torch.float64
    bc = {k: torch.empty((W, ncol), dtype=f64, device=dev) for k in ("fbeam", "umu0", "albedo")}
    for i, g in enumerate(gpoints):
        gen = torch.Generator(device=dev)
        gen.manual_seed(seed * 1000 + int(g))
        r = torch.rand((2, ncol), generator=gen, dtype=f64, device=dev)
        bc["fbeam"][i] = 1.0
        bc["umu0"][i] = umu0[0] + (umu0[1] - umu0[0]) * r[0]
        bc["albedo"][i] = r[1]
    return prop, bc, None


def gpoint_weights(ngpoint):
    # fixed synthetic correlated-k weights (sum to 1)
    x = np.arange(ngpoint, dtype=np.float64)
    w = 1.0 + 0.5 * np.cos(x)
    return w / w.sum()


def wave_bounds(ngpoint, band=None, ck=False):
    if band is None:
        lo = 10.0 + 30.0 * np.arange(ngpoint, dtype=np.float64)
        return lo, lo + 30.0
    if ck:  # correlated-k: every g-point spans the whole band (amars_lw.cpp:23-31)
        return np.full(ngpoint, band[0]), np.full(ngpoint, band[1])
    edges = np.linspace(band[0], band[1], ngpoint + 1)
    return edges[:-1].copy(), edges[1:].copy()


def load_pmc(nstr: int, nlyr: int, planck: bool):
    """Measured HBM bytes per solve per kernel for this shape: the profiles/pmc_*.json
    (scripts/pmc_summarize.py) whose (nstr, nlyr, planck) match."""
    import glob
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_*.json"))):
        try:
            with open(p) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        if (d.get("nstr"), d.get("nlyr"), bool(d.get("planck"))) == (nstr, nlyr, bool(planck)):
            return d
    return None


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(prop, bc, temf, nstr, planck, wl, wu, target_s=10.0, target_1core_s=3.0):
    """Time the C restatement (oracle/) on a bounded sample of the same workload.

    The sample is the workload's first solves, (g-point, column) order, grown until it
    takes ~target_s; a workload smaller than that (C1: 16 solves) is solved repeatedly.
    Threads: OMP_NUM_THREADS (the GPU box exports its per-GPU CPU share, 16) else every
    core in this process's affinity set; nproc, the affinity set and the CPU model are
    reported, and the same sample is timed again on one core."""
    from oracle import oracle_c
    oracle_c.build()
    affinity = len(os.sched_getaffinity(0))
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or affinity
    W, ncol, nlyr = prop.shape[0], prop.shape[1], prop.shape[2]
    S = W * ncol
    host = {}

    def slabs(m):
        if host.get("m", 0) < m:
            host["m"] = m
            host["p"] = prop[:m].cpu().numpy()
            host["b"] = {k: v[:m].cpu().numpy() for k, v in bc.items()}
        return host["p"][:m], {k: v[:m] for k, v in host["b"].items()}

    tf = None if temf is None else temf.cpu().numpy()

    def run(n, nthreads):
        m = min(W, -(-n // ncol))
        p, b = slabs(m)
        count = min(n, m * ncol)
        reps = -(-n // count)
        out = np.zeros((m, ncol, nlyr + 1, 2))
        kw = dict(nstr=nstr, planck=planck, wave_lower=wl[:m], wave_upper=wu[:m],
                  nthreads=nthreads)
        t0 = time.perf_counter()
        for _ in range(reps):
            oracle_c.forward(p, b, tf, first=0, count=count, out=out, **kw)
        return time.perf_counter() - t0, reps * count, count, out

    def timed(nthreads, target):
        n = max(4 * nthreads, 1)
        while True:
            dt, done, count, out = run(n, nthreads)
            if dt >= 0.5 or n >= 64 * S + 1000000:
                break
            n *= 4
        n = int(max(1, done * target / max(dt, 1e-9)))
        return run(n, nthreads)

    dt, done, count, out = timed(threads, target_s)
    dt1, done1, _, _ = timed(1, target_1core_s)
    reps = done // max(count, 1)
    sample = (f"{done} solves: the first {count} (g-point, column) solves of the same "
              f"workload (nstr={nstr}, nlyr={nlyr})" + (f" x {reps} passes" if reps > 1 else "")
              + f", {threads} OpenMP threads, {dt:.1f} s; 1 core: {done1} solves in "
              f"{dt1:.1f} s; oracle/disort_oracle.c = C restatement of the DISORT algorithm "
              "(cdisort itself is absent from the reference)")
    return {"value": round(done / dt, 1), "unit": "column-solves/s", "cores": threads,
            "kind": "port", "value_1core": round(done1 / dt1, 1), "nproc": os.cpu_count(),
            "affinity_cores": affinity, "cpu_model": _cpu_model(),
            "threads_note": "threads = OMP_NUM_THREADS when set (the GPU box sets its per-GPU "
                            "CPU share, 16, and asks that pools stay within it), else the "
                            "affinity set",
            "sample_seconds": round(dt, 2), "sample": sample}, out, count


def extra_legs(disort, prop, bc, temf, wts, steps, dev):
    """SURVEY 8(d)'s companions of the headline (untimed by the driver, rank 0, N = 1):
      unfused     -- Disort.forward on device tensors (hd_solve: the per-g fluxes stored,
                     as every reference call site receives them) + hd_band_flux
      end_to_end  -- Disort.forward on CPU tensors, CPU flux back: pydisort's contract as
                     the reference calls it (examples/amars_sw.cpp:280, amars_lw.cpp:80,
                     radiation_band.cpp:124-127) -> hd_solve_host, H2D/D2H included
      end_to_end_band -- Disort.forward_band on CPU tensors (hd_solve_band_host: only the
                     band flux comes back)
    Host arrays are ordinary (pageable) CPU tensors, as the reference's are."""
    from pyharp_amd.spectral import band_flux
    W, ncol, nlyr = prop.shape[0], prop.shape[1], prop.shape[2]
    nsolve = W * ncol
    out = {}
    flux = torch.empty((W, ncol, nlyr + 1, 2), dtype=torch.float64, device=dev)
    band = torch.empty((ncol, nlyr + 1, 2), dtype=torch.float64, device=dev)

    def unfused():
        disort.forward(prop, bc, temf, out=flux)
        band_flux(flux, wts, out=band)

    unfused()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        unfused()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    out["unfused"] = {"value": round(nsolve / dt, 1), "unit": "column-solves/s",
                      "ms_per_step": round(dt * 1e3, 3), "steps": steps,
                      "entry": "Disort.forward on device tensors (hd_solve, per-g fluxes "
                               "stored) + hd_band_flux"}
    del flux
    hp = prop.cpu()
    hb = {k: v.cpu() for k, v in bc.items()}
    ht = None if temf is None else temf.cpu()
    hw = wts.cpu()
    host_bytes = int(hp.numel() * 8 + sum(v.numel() * 8 for v in hb.values()) +
                     (0 if ht is None else ht.numel() * 8))
    reps = 3
    for name, call, back in (
            ("end_to_end", lambda: disort.forward(hp, hb, ht), nsolve * (nlyr + 1) * 16),
            ("end_to_end_band", lambda: disort.forward_band(hp, hb, ht, weights=hw),
             ncol * (nlyr + 1) * 16)):
        r = call()
        assert r.device.type == "cpu"
        del r
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            r = call()
            ts.append(time.perf_counter() - t0)
            del r
        dt = sorted(ts)[len(ts) // 2]
        out[name] = {"value": round(nsolve / dt, 1), "unit": "column-solves/s",
                     "ms_per_step": round(dt * 1e3, 3), "reps": reps, "timing": "median wall",
                     "host_bytes_in": host_bytes, "host_bytes_out": int(back),
                     "entry": ("Disort.forward on CPU tensors -> hd_solve_host (per-g fluxes "
                               "back to the host)" if name == "end_to_end" else
                               "Disort.forward_band on CPU tensors -> hd_solve_band_host")}
    return out


def launch_mode(gpus: int, env) -> str:
    """How this invocation runs (the driver's contract: ``bench.py --gpus N`` alone,
    or under ``torch.distributed.run`` with N ranks):
      "single" -- one process, N = 1, no launcher;
      "rank"   -- one rank of an N-rank job started by a launcher (WORLD_SIZE set);
      "spawn"  -- --gpus N > 1 without a launcher: this process starts the N ranks.
    A launcher's WORLD_SIZE that disagrees with --gpus is an error (the line's
    n_gpus must be the number of ranks that ran)."""
    if gpus < 1:
        raise SystemExit(f"bench.py: --gpus {gpus} must be >= 1")
    if "WORLD_SIZE" in env:
        world = int(env["WORLD_SIZE"])
        if world != gpus:
            raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {gpus}: run "
                             "--gpus N under a launcher with N ranks, or --gpus N alone")
        return "rank"
    return "spawn" if gpus > 1 else "single"


def spawn_ranks(n: int, argv, env=None, program=None) -> int:
    """Start n fresh rank processes of ``program`` (default: this script with argv) with
    torch.distributed.run's environment (RANK, LOCAL_RANK, WORLD_SIZE, MASTER_ADDR
    127.0.0.1, a free MASTER_PORT) and wait for all of them.  This parent never touches
    the GPU (it only starts children; no exec from a GPU process).  Returns 0 if every
    rank exited 0, else the first nonzero exit code (a rank killed by a signal counts
    as 128 + signal); the other ranks are terminated once one has failed."""
    import signal
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    base = dict(os.environ if env is None else env)
    base.update(WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1",
                MASTER_PORT=str(port))
    cmd = program if program is not None else [sys.executable, os.path.abspath(__file__)] + \
        list(argv)
    procs = []
    pending = []

    def _on_term(signum, frame):  # a SIGTERM to this parent unwinds through finally
        raise SystemExit(128 + signum)

    old_term = signal.signal(signal.SIGTERM, _on_term)
    rc = 0
    try:
        for r in range(n):
            e = dict(base, RANK=str(r), LOCAL_RANK=str(r))
            procs.append(subprocess.Popen(cmd, env=e))
            pending.append(procs[-1])
        while pending:
            for p in list(pending):
                code = p.poll()
                if code is None:
                    continue
                pending.remove(p)
                code = 128 - code if code < 0 else code
                if code and not rc:
                    rc = code
                    for q in pending:  # a failed rank would leave the others in a collective
                        q.send_signal(signal.SIGTERM)
            if pending:
                time.sleep(0.05)
    finally:
        # interrupted or terminated: no rank outlives this parent (they hold GPUs and
        # would block the next run in a collective) -- SIGTERM, then SIGKILL after 10 s.
        # A second SIGTERM during this cleanup only records itself: raising again here
        # would skip the SIGKILL escalation and leave ranks behind.
        signal.signal(signal.SIGTERM, lambda signum, frame: None)
        for q in pending:
            if q.poll() is None:
                q.send_signal(signal.SIGTERM)
        deadline = time.time() + 10.0
        for q in pending:
            try:
                q.wait(timeout=max(0.0, deadline - time.time()))
            except subprocess.TimeoutExpired:
                q.kill()
                q.wait()
        # None: the previous handler was not installed from Python -- leave ours
        if old_term is not None:
            signal.signal(signal.SIGTERM, old_term)
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", choices=sorted(CONFIGS), default="c4")
    ap.add_argument("--ncol", type=int, default=None)
    ap.add_argument("--ngpoint", type=int, default=None)
    ap.add_argument("--nlyr", type=int, default=None)
    ap.add_argument("--nstr", type=int, default=None)
    ap.add_argument("--planck", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--chunk", type=int, default=0,
                    help="max solves per internal chunk (hd_context_set_chunk; 0 = auto)")
    ap.add_argument("--no-fuse", action="store_true",
                    help="unfused epilogue: per-g fluxes stored by hd_solve, then hd_band_flux")
    ap.add_argument("--no-extra", action="store_true",
                    help="skip the unfused and host-array (end-to-end) legs")
    ap.add_argument("--graph", action="store_true",
                    help="replay the solve + band sum as one captured HIP graph per step")
    args = ap.parse_args()
    mode = launch_mode(args.gpus, os.environ)
    if mode == "spawn":
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    cfgd = CONFIGS[args.config]
    for k in ("ncol", "ngpoint", "nlyr", "nstr"):
        if getattr(args, k) is None:
            setattr(args, k, cfgd[k])

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # HD_BENCH_REHEARSE=1: rehearse the N>1 path on a box with fewer GPUs than
    # ranks (ranks share devices, gloo instead of RCCL); never set by the driver
    rehearse = os.environ.get("HD_BENCH_REHEARSE") == "1"
    dev_index = local_rank % torch.cuda.device_count() if rehearse else local_rank
    # under torch.distributed.run the process group is set up even at one rank, so
    # the RCCL initialisation and the band all-reduce run at every N
    dist_on = world > 1 or "LOCAL_RANK" in os.environ
    # RCCL prints a version banner on stdout when a communicator is created: send
    # fd 1 to stderr until the warm-up's all-reduce is done, so stdout carries
    # only the JSON line
    saved_stdout = None
    if dist_on:
        sys.stdout.flush()
        saved_stdout = os.dup(1)
        os.dup2(2, 1)
    if dist_on:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(dev_index)
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_index))
    dev = torch.device("cuda", dev_index)
    torch.cuda.set_device(dev)

    from pyharp_amd import Disort, DisortOptions
    from pyharp_amd.disort import _context

    ncol, nlyr, nstr, G = args.ncol, args.nlyr, args.nstr, args.ngpoint
    from pyharp_amd.spectral import band_flux, shard_gpoints
    gpoints = shard_gpoints(G, world, rank)
    W = len(gpoints)
    lw = cfgd.get("lw", False)
    if lw:
        args.planck = True
    wl_all, wu_all = wave_bounds(G, cfgd.get("band"), ck=args.config == "c1")
    wl, wu = wl_all[gpoints], wu_all[gpoints]
    if lw:
        prop, bc, temf = make_lw_inputs(gpoints, G, ncol, nlyr, nstr, cfgd["band"], cfgd["tau"],
                                        dev)
    elif cfgd.get("aerosol"):
        prop, bc, temf = make_aerosol_inputs(gpoints, G, ncol, nlyr, nstr, dev,
                                             umu0=cfgd["umu0"])
    else:
        prop, bc, temf = make_inputs(gpoints, ncol, nlyr, nstr, args.planck, dev,
                                     ssa=cfgd["ssa"], gasym=cfgd["g"], umu0=cfgd["umu0"])
    wts = torch.tensor(gpoint_weights(G)[gpoints], dtype=torch.float64, device=dev)

    op = DisortOptions().flags("lamber,quiet,onlyfl" + (",planck" if args.planck else ""))
    op.nwave(W).ncol(ncol).device(dev_index)
    if args.planck:
        op.wave_lower(list(wl)).wave_upper(list(wu))
    op.ds().nlyr, op.ds().nstr, op.ds().nmom = nlyr, nstr, nstr
    disort = Disort(op)
    fuse = not args.no_fuse
    flux = None if fuse else torch.empty((W, ncol, nlyr + 1, 2), dtype=torch.float64, device=dev)
    status = torch.zeros(W * ncol, dtype=torch.int32, device=dev)

    band = torch.empty((ncol, nlyr + 1, 2), dtype=torch.float64, device=dev)

    def solve():
        if fuse:
            disort.forward_band(prop, bc, temf, weights=wts, out=band, status=status)
        else:
            disort.forward(prop, bc, temf, status=status, out=flux)
            band_flux(flux, wts, out=band)

    if args.chunk:
        _context(dev_index).set_chunk(args.chunk)
    graph = None
    if args.graph:
        solve()  # sizes the context's scratch and tables before capture
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        cs = torch.cuda.Stream(device=dev)
        cs.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(cs):
            with torch.cuda.graph(graph, stream=cs):
                solve()
        torch.cuda.synchronize()

    def step():
        if graph is not None:
            graph.replay()
        else:
            solve()
        if dist_on:
            import torch.distributed as dist
            dist.all_reduce(band, op=dist.ReduceOp.SUM)
        return band

    for _ in range(max(args.warmup, 1 if dist_on else 0)):
        step()
    torch.cuda.synchronize()
    if saved_stdout is not None:
        sys.stdout.flush()
        os.dup2(saved_stdout, 1)
        os.close(saved_stdout)
    if int((status & 0xF).any()):
        raise RuntimeError("bench: solver reported errors in the warm-up")
    ctx = _context(dev_index)
    if dist_on:
        import torch.distributed as dist
        dist.barrier()
    torch.cuda.synchronize()
    ctx.set_timing(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        band = step()
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    tm = ctx.timing()
    ctx.set_timing(False)
    timing_note = "HIP events on the solve stream over the timed steps"
    if graph is not None:  # replays carry no timing events: one eager step for the kernels
        torch.cuda.synchronize()
        ctx.set_timing(True)
        solve()
        torch.cuda.synchronize()
        tm = ctx.timing()
        ctx.set_timing(False)
        steps_timed = 1
        timing_note = "HIP events on one eager step after the graph-replayed timed steps"
    else:
        steps_timed = args.steps
    if dist_on:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    band_sum = float(band.sum().item())
    nsolve_total = G * ncol
    value = nsolve_total * args.steps / elapsed
    total_flop, k1_flop, k2_flop = algorithmic_flop(nstr, nlyr, args.planck)
    workload = (f"{cfgd['label']}: {ncol} columns x {G} g-points, nstr={nstr}, nmom={nstr}, "
                f"nlyr={nlyr}, " + ("thermal (planck), omega=0" if lw else
                                    f"beam{' + planck' if args.planck else ''}"))

    team_valu = os.environ.get("HD_AB") == "1" and os.environ.get("HD_TEAM_LAYER") == "valu"  # A/B switch of the team path
    layer_kernel = ("hd_layer_kernel" if nstr <= 16 else
                    "hd_team_layer_kernel" if team_valu else "hd_team_mfma_layer_kernel")
    mfma = nstr > 16 and not team_valu
    if rank == 0:
        # dominant kernel roofline (the layer-setup kernel), per launch
        k1_avg_ms = tm.layer_ms / max(tm.layer_launches, 1)
        solves_per_launch = W * ncol * steps_timed / max(tm.layer_launches, 1)
        ach = k1_flop * solves_per_launch / (k1_avg_ms * 1e-3) / 1e12
        pmc = load_pmc(nstr, nlyr, args.planck)
        traffic = None
        path_bytes = None
        if pmc:
            k1 = pmc["kernels"].get(f"{layer_kernel}<{nstr // 2}>")
            if k1:
                traffic = round(k1["bytes_per_solve"] * solves_per_launch)
            # HBM bytes per solve of every kernel of the path (one chunk's launches)
            path_bytes = round(sum(k["bytes_per_solve"] for k in pmc["kernels"].values()))
        roofline = {"bound": "fp64-mfma+valu" if mfma else "fp64-valu", "kernel": f"{layer_kernel}<{nstr // 2}>", "achieved": round(ach, 3),
                    "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                    "frac": round(ach / FP64_PEAK_TFLOPS, 4),
                    "traffic": traffic,
                    "traffic_note": None if pmc is None else
                    f"HBM bytes per launch from rocprofv3 PMC run {pmc['source']} "
                    "(2 x FETCH_SIZE + WRITE_SIZE, scaled to this launch's solves); "
                    "algorithmic bytes per solve are much smaller: the layer records "
                    f"({nstr // 2 * (nstr // 2 + 1) + nstr + 1 if nstr <= 16 else nstr * nstr // 2 + nstr + 2}"
                    " doubles per layer) are written to HBM scratch for the sweep",
                    "path_bytes_per_solve": path_bytes,
                    "algorithmic_bytes_per_solve": int(nlyr * (2 + nstr) * 8 + 48 + (nlyr + 1) * 16
                                                       + (nlyr + 1) * 8 * int(bool(args.planck))),
                    "avg_launch_ms": round(k1_avg_ms, 3),
                    "flop_per_solve": k1_flop,
                    "note": ("FP64 compute bound: dense 16x16 products on FP64 MFMA, the "
                             "Cholesky/Jacobi/triangular algebra on the VALU (gfx950's FP64 "
                             "vector and MFMA peaks are both 78.6 TF/s)" if mfma else
                             "FP64 compute bound, VALU (no MFMA in this kernel; gfx950's FP64 "
                             "vector and MFMA peaks are both 78.6 TF/s)") + "; achieved uses the SURVEY 8(d) algorithmic FLOP convention"
                            + ("; nstr<=16: each launch runs on its own stream beside the "
                               "previous chunk's sweep, so its duration includes that "
                               "co-running (path_roofline is what the throughput follows)"
                               if nstr <= 16 else "")}
        whole = {"achieved_tflops": round(total_flop * value / 1e12, 3),
                 "frac": round(total_flop * value / 1e12 / FP64_PEAK_TFLOPS / world, 4),
                 "layer_ms_per_step": round(tm.layer_ms / steps_timed, 3),
                 "sweep_ms_per_step": round(tm.sweep_ms / steps_timed, 3),
                 "timing": timing_note}
        cpu = None
        max_err = None
        fused_vs_unfused = None
        if fuse and world == 1:
            # per-g fluxes (untimed) for the parity checks, from the timed step's own
            # kernel schedule (hd_solve_band with the per-point fluxes kept: bitwise
            # hd_solve's, tests/test_gpu_band.py), so that a rocprofv3 trace of this
            # command averages launches of one kind; the fused band against
            # hd_band_flux over them (only the summation order differs)
            band_fused = band.clone()
            flux = torch.empty((W, ncol, nlyr + 1, 2), dtype=torch.float64, device=dev)
            disort.forward_band(prop, bc, temf, weights=wts, flux=flux, status=status)
            bunf = band_flux(flux, wts)
            fused_vs_unfused = float(((band_fused - bunf).abs().max() /
                                      bunf.abs().max()).item())
        extra = None
        if world == 1 and not args.no_extra:
            extra = extra_legs(disort, prop, bc, temf, wts, args.steps, dev)
        if world == 1 and not args.no_cpu_baseline:
            cpu, ref, n = cpu_baseline(prop, bc, temf, nstr, args.planck, wl, wu)
            m = ref.shape[0]
            got = flux[:m].cpu().numpy().reshape(-1, nlyr + 1, 2)[:n]
            r = ref.reshape(-1, nlyr + 1, 2)[:n]
            scale = np.abs(r).max(axis=(1, 2), keepdims=True)
            max_err = float((np.abs(got - r) / np.maximum(np.abs(r), 1e-6 * scale)).max())
        line = {
            "metric": METRIC if (nstr, nlyr) == (16, 80) else
            METRIC.replace("nstr=16, nlyr=80", f"nstr={nstr}, nlyr={nlyr}"), "value": round(value, 1), "unit": "column-solves/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
            "config": {"workload": workload, "ncol": ncol, "ngpoint": G, "nstr": nstr,
                       "nmom": nstr, "nlyr": nlyr, "planck": bool(args.planck),
                       "parallelism": f"spectral g mod {world}",
                       "hip_graph": bool(args.graph), "chunk": args.chunk or "auto",
                       "epilogue": ("band sum fused into the solve (hd_solve_band; per-g "
                                    "fluxes not stored)" if fuse else
                                    "per-g fluxes stored (hd_solve) + hd_band_flux"),
                       "collective": ("all_reduce of the g-weighted band flux (" +
                                      ("gloo, rehearsal" if rehearse else "RCCL") + ")") if dist_on
                       else "none"},
            "roofline": roofline, "path_roofline": whole, "cpu_baseline": cpu,
            "unfused": None if extra is None else extra["unfused"],
            "end_to_end": None if extra is None else extra["end_to_end"],
            "end_to_end_band": None if extra is None else extra["end_to_end_band"],
            "max_rel_err_vs_cpu_restatement": max_err,
            "band_fused_vs_unfused_max_rel": fused_vs_unfused,
            # sum of the (all-reduced) band flux of the last step: equal at every N for a
            # given workload (tests/test_bench_launch.py, the rehearsal in DESIGN.md 7)
            "band_flux_sum": band_sum,
        }
        print(json.dumps(line), flush=True)
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
