"""Per-kernel register, LDS and spill figures and memory-instruction counts of a
hipcc --save-temps gfx950 assembly file.

    python scripts/isa_stats.py FILE.s [SUBSTRING ...]
"""
import re
import sys


def main():
    s = open(sys.argv[1]).read()
    pats = sys.argv[2:]
    for m in re.finditer(r"\.amdhsa_kernel (\S+)\n(.*?)\.end_amdhsa_kernel", s, re.S):
        name, blk = m.group(1), m.group(2)
        if pats and not any(p in name for p in pats):
            continue
        d = dict(re.findall(r"\.amdhsa_(\w+) (\S+)", blk))
        i = s.index(name + ":")
        body = s[i:s.index(".Lfunc_end", i)]
        cnt = {}
        for line in body.split("\n"):
            t = line.strip().split(" ")[0]
            if t.startswith(("global_", "buffer_", "scratch_", "flat_", "ds_", "v_mfma")):
                cnt[t] = cnt.get(t, 0) + 1
        print(f"{name}: vgpr {d.get('next_free_vgpr')} accum_offset {d.get('accum_offset')} "
              f"sgpr {d.get('next_free_sgpr')} lds {d.get('group_segment_fixed_size')} "
              f"scratch {d.get('private_segment_fixed_size')}")
        print("   ", dict(sorted(cnt.items())))


if __name__ == "__main__":
    main()
