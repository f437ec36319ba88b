"""Build libhdisort.so (HIP, gfx950) in-tree with hipcc.

The shared library lands next to this file (pyharp_amd/libhdisort.so) so the
gpurun snapshot carries it to the GPU box; no JIT cache is involved.
"""

from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libhdisort.so")
SOURCES = ["hd_kernels.hip", "hd_team.hip", "hd_team_mfma.hip", "hd_rad.hip", "hd_harp.hip",
           "hd_api.cpp", "hd_ncread.cpp", "hd_rad_wide.hip"]
HEADERS = ["hd_device.hpp", "hd_kernels.hpp", "hd_rad.hpp", "hd_team_prims.hpp", os.path.join("..", "..", "include", "hdisort.h"),
           os.path.join("..", "..", "include", "hdharp.h"),
           os.path.join("..", "..", "include", "hdnc.h"),
           os.path.join("..", "..", "include", "harp_amd", "ncread.hpp"),
           os.path.join("..", "..", "include", "harp_amd", "nc4read.hpp")]
ARCH = os.environ.get("HD_OFFLOAD_ARCH", "gfx950")
# per-source extra flags.  hd_team_mfma.hip: without MachineLICM the loop-invariant
# constants of the lean team sweep (hd_team_mfma_sweep_lean_kernel) are formed where
# they are used instead of being hoisted out of its layer loop -- 254 VGPRs and 20 B
# of scratch at nstr 32 instead of 156 B of spills at the two-waves-per-SIMD cap;
# the team layer kernel is unchanged (239)
EXTRA = {"hd_team_mfma.hip": ["-mllvm", "-disable-machine-licm"]}


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if cand and (os.path.sep not in cand or os.path.exists(cand)):
            return cand
    return "hipcc"


def _stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    for f in SOURCES + HEADERS:
        if os.path.getmtime(os.path.join(CSRC, f)) > t:
            return True
    return False


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not _stale():
        return LIB
    objs, procs = [], []
    for src in SOURCES:  # one hipcc per source, in parallel (the team TU dominates)
        obj = os.path.join(CSRC, src + ".o")
        cmd = [_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
               "-x", "hip", "-c", os.path.join(CSRC, src), "-o", obj] + EXTRA.get(src, [])
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        procs.append((cmd, subprocess.Popen(cmd)))
        objs.append(obj)
    for cmd, p in procs:
        if p.wait() != 0:
            raise subprocess.CalledProcessError(p.returncode, cmd)
    tmp = LIB + ".tmp"
    cmd = [_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs + ["-lz"]
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB)
    for o in objs:
        os.remove(o)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
