"""Print the hd:: kernel timeline of the last solve in a rocprofv3 kernel trace
(kernel_trace.csv): name, queue, start/end relative to the last step's first
layer kernel [ms], duration."""
import csv
import re
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "hd::" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
nlay = int(sys.argv[2]) if len(sys.argv) > 2 else 10
lay = [i for i, r in enumerate(rows) if "layer_kernel" in r["Kernel_Name"]]
first = lay[-nlay]
t0 = int(rows[first]["Start_Timestamp"])
for r in rows[max(0, first - 3):]:
    name = re.search(r"hd::(?:\(anonymous namespace\)::)?(\w+)", r["Kernel_Name"]).group(1)
    s = (int(r["Start_Timestamp"]) - t0) / 1e6
    e = (int(r["End_Timestamp"]) - t0) / 1e6
    print(f"{name:26s} q{r['Queue_Id']:>2} {s:8.3f} {e:8.3f} {e - s:7.3f}")
