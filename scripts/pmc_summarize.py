"""Fold rocprofv3 FETCH_SIZE / WRITE_SIZE passes into profiles/pmc_<shape>.json (read by bench.py).

    python scripts/pmc_summarize.py FETCH_DIR WRITE_DIR [--solves 65536] [--nstr 16] [--nlyr 80]
                                    [--out profiles/pmc_c4.json]

Inputs are the two separate `--pmc` passes (scripts/gpu.sh step pmc=NAME:NSTR) over
scripts/pmc_run.py (one chunk of the C4 or C5 shape per launch).  Units:
rocprofv3 reports both counters in KiB.  gfx950 correction
(MI355X_MICROARCH.md, HBM section): FETCH_SIZE counts half the bytes of a wide
coalesced streaming read, so fetch is doubled; WRITE_SIZE is exact.  Our
kernels' loads are 64 consecutive doubles per wave instruction; the doubling is
confirmed on this access pattern by hd_sweep_kernel, whose algorithmic read
bytes (layer records + back-substitution records) match 2 x FETCH_SIZE to 2 %.
"""

import argparse
import csv
import glob
import json
import os
import re


def per_kernel(run_dir, counter):
    acc = {}
    path = sorted(glob.glob(os.path.join(run_dir, "**", "*counter_collection.csv"),
                            recursive=True))[0]
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] != counter:
                continue
            name = r["Kernel_Name"]
            if not name.startswith(("void hd::", "hd::")):
                continue
            key = name.split("(")[0].replace("void ", "").replace("hd::", "")
            # the record-access variant (NT template argument) is one kernel here
            key = re.sub(r",\s*(true|false)>", ">", key)
            acc.setdefault(key, []).append(float(r["Counter_Value"]) * 1024.0)
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--solves", type=int, default=65536)
    ap.add_argument("--nstr", type=int, default=16)
    ap.add_argument("--nlyr", type=int, default=80)
    ap.add_argument("--planck", action="store_true")
    ap.add_argument("--out", default=os.path.join(os.path.dirname(__file__), "..", "profiles",
                                                   "pmc_c4.json"))
    a = ap.parse_args()
    fetch = per_kernel(a.fetch_dir, "FETCH_SIZE")
    write = per_kernel(a.write_dir, "WRITE_SIZE")
    kernels = {}
    for k in sorted(set(fetch) | set(write)):
        rd = 2.0 * fetch.get(k, 0.0)
        wr = write.get(k, 0.0)
        kernels[k] = {"fetch_bytes_raw": fetch.get(k), "read_bytes": rd, "write_bytes": wr,
                      "bytes_per_launch": rd + wr, "bytes_per_solve": (rd + wr) / a.solves}
    out = {"nstr": a.nstr, "nlyr": a.nlyr, "planck": bool(a.planck),
           "solves_per_launch": a.solves, "source": os.path.normpath(a.fetch_dir).replace("_fetch", ""),
           "correction": "read = 2 x FETCH_SIZE (gfx950 half-count), write = WRITE_SIZE; KiB -> B",
           "kernels": kernels}
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
