"""Highest VGPR / AGPR index referenced in each sched_barrier-delimited region of a
kernel in a hipcc --save-temps gfx950 assembly file (where the register peak sits).

    python scripts/isa_regions.py FILE.s KERNEL_SUBSTRING
"""
import re
import sys


def main():
    s = open(sys.argv[1]).read()
    pat = sys.argv[2]
    m = next(m for m in re.finditer(r"^(\S+):\s*; @", s, re.M) if pat in m.group(1))
    i = m.start()
    body = s[i:s.index(".Lfunc_end", i)].split("\n")
    reg = re.compile(r"\b([va])\[?(\d+)(?::(\d+))?\]?")
    seg, start = {"v": -1, "a": -1, "n": 0}, 0
    for k, line in enumerate(body + ["; sched_barrier"]):
        if "sched_barrier" in line:
            print(f"lines {start:5d}-{k:5d}: {seg['n']:5d} instr, max v{seg['v']}, max a{seg['a']}")
            seg, start = {"v": -1, "a": -1, "n": 0}, k
            continue
        t = line.strip()
        if not t or t.startswith((";", ".", "s_")):
            continue
        seg["n"] += 1
        for kind, lo, hi in reg.findall(t.split(";")[0]):
            seg[kind] = max(seg[kind], int(hi or lo))


if __name__ == "__main__":
    main()
