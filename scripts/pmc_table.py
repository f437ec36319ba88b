"""Per-kernel averages of every counter in a pmc run directory (one or more passes).

    python scripts/pmc_table.py DIR [DIR ...] [--json out.json]   (every *counter_collection.csv below)
"""
import argparse
import csv
import glob
import json
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("run_dirs", nargs="+")
    ap.add_argument("--json")
    a = ap.parse_args()
    acc = {}
    paths = [p for d in a.run_dirs
             for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)]
    for path in sorted(paths):
        with open(path) as f:
            for r in csv.DictReader(f):
                name = r["Kernel_Name"]
                if "hd::" not in name:
                    continue
                key = name.split("(")[0].replace("void ", "").replace("hd::", "")
                d = acc.setdefault(key, {})
                d.setdefault(r["Counter_Name"], {}).setdefault(r["Dispatch_Id"], 0.0)
                d[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    out = {}
    for k, d in acc.items():
        out[k] = {c: sum(v.values()) / len(v) for c, v in sorted(d.items())}
    for k, d in out.items():
        print(k)
        for c, v in d.items():
            print(f"   {c:28s} {v:16.1f}")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
