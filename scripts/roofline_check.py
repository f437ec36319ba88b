"""Recompute a bench line's roofline.frac from a rocprofv3 --kernel-trace --stats summary.

    python scripts/roofline_check.py BENCH_LINE.json KERNEL_STATS.csv [KERNEL_TRACE.csv]

frac = flop_per_solve x solves per launch / (trace average duration x 78.6 TF/s), the
SURVEY 8(d) convention bench.py uses with its HIP-event average.  With the kernel
trace, the average over the launches of the timed steps alone is printed too (the
stats file averages every launch of the process: warm-up, timed, parity solve).
"""

import csv
import json
import sys

PEAK = 78.6e12


def main():
    line = json.load(open(sys.argv[1]))
    rf = line["roofline"]
    kern = rf["kernel"].split("<")[0]
    cfg = line["config"]
    solves = cfg["ncol"] * cfg["ngpoint"] // line["n_gpus"]
    rows = [r for r in csv.DictReader(open(sys.argv[2])) if f"hd::{kern}<" in r["Name"]]
    if not rows:
        raise SystemExit(f"{kern} not in {sys.argv[2]}")
    r = rows[0]
    calls, avg = int(r["Calls"]), float(r["AverageNs"]) * 1e-9
    # solves per launch from the line itself (achieved x its average launch / FLOP per
    # solve): the stats file also holds the launches of the line's extra legs
    # (unfused, end-to-end), so calls / steps does not give it
    per_launch = round(rf["achieved"] * 1e12 * rf["avg_launch_ms"] * 1e-3 / rf["flop_per_solve"])
    launches_per_step = round(solves / per_launch)
    frac = rf["flop_per_solve"] * per_launch / avg / PEAK
    print(f"{r['Name']}: {calls} launches, trace average {avg * 1e3:.3f} ms "
          f"({launches_per_step} per step, {per_launch:.0f} solves each)")
    print(f"  frac from the trace   = {frac:.4f}")
    print(f"  frac in the bench line = {rf['frac']:.4f} (HIP events, avg {rf['avg_launch_ms']} ms)")
    if len(sys.argv) > 3:
        tr = [t for t in csv.DictReader(open(sys.argv[3])) if f"hd::{kern}<" in t["Kernel_Name"]]
        tr.sort(key=lambda t: int(t["Start_Timestamp"]))
        n = line["steps"] * launches_per_step
        first = line["warmup"] * launches_per_step
        timed = tr[first:first + n]
        d = sum(int(t["End_Timestamp"]) - int(t["Start_Timestamp"]) for t in timed) / len(timed)
        print(f"  timed steps only ({len(timed)} launches): average {d * 1e-6:.3f} ms, "
              f"frac {rf['flop_per_solve'] * per_launch / (d * 1e-9) / PEAK:.4f}")


if __name__ == "__main__":
    main()
