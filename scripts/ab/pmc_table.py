"""Per-kernel mean of every counter in rocprofv3 --pmc runs: python pmc_table.py DIR..."""
import csv
import glob
import os
import sys

acc = {}
for d in sys.argv[1:]:
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                name = r["Kernel_Name"]
                if not name.startswith(("void hd::", "hd::")):
                    continue
                key = name.split("(")[0].replace("void ", "").replace("hd::", "")
                acc.setdefault(key, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
for k, cs in sorted(acc.items()):
    print(k)
    for c, v in sorted(cs.items()):
        print(f"    {c:28s} {sum(v) / len(v):.4g}")
