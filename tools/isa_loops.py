"""Static instruction counts per loop of one kernel in a hipcc -S listing (gfx950).

    hipcc ... --cuda-device-only -S -o k.s  &&  python tools/isa_loops.py k.s [kernel-substring] [min-VALU]

For every loop, counts the instructions of the blocks whose innermost loop it is (child loops,
e.g. the ring-space waits, excluded; rarely taken blocks included): VALU, SGPR reloads from VGPR
lanes (v_readlane), fp64 ops, LDS and global memory instructions.  The loop nest comes from the
compiler's block comments ("in Loop: Header=BB.. Depth=d", "This Loop Header").
"""
import re
import sys
from collections import Counter, defaultdict


def main():
    text = open(sys.argv[1]).read().split("\n")
    key = sys.argv[2] if len(sys.argv) > 2 else "lm2_kernel"
    vmin = int(sys.argv[3]) if len(sys.argv) > 3 else 100
    start = next(i for i, l in enumerate(text) if re.match(r"^_Z\w*" + key + r"\w*:", l))
    end = next(i for i in range(start, len(text)) if text[i].startswith(".Lfunc_end"))
    lines = text[start:end]
    counts = defaultdict(Counter)
    first = {}
    cur = None
    for i, l in enumerate(lines):
        if l.startswith(".LBB") or l.startswith("; %bb."):
            label = l.split(":")[0].strip().lstrip(".").replace("; %bb.", "BB?")
            notes = " ".join([l] + [m for m in lines[i + 1:i + 3] if m.strip().startswith(";")])
            if "This Loop Header" in notes or "This Inner Loop Header" in notes:
                cur = label.lstrip("L") if label.startswith("LBB") else label
            else:
                m = re.search(r"in Loop: Header=(BB\w+)", notes)
                cur = m.group(1) if m else None
            if cur is not None:
                first.setdefault(cur, i)
            continue
        s = l.strip()
        if cur is None or not s or s.startswith((".", ";")):
            continue
        counts[cur][s.split()[0]] += 1
    for h in sorted(counts, key=lambda h: first[h]):
        c = counts[h]
        v = sum(n for k, n in c.items() if k.startswith("v_"))
        if v < vmin:
            continue
        print(f"{h:10s} line {first[h] + start:6d} VALU {v:4d} readlane {c['v_readlane_b32']:3d} "
              f"f64 {sum(n for k, n in c.items() if k.startswith('v_') and 'f64' in k):4d} "
              f"ds {sum(n for k, n in c.items() if k.startswith('ds_')):3d} "
              f"glob {sum(n for k, n in c.items() if k.startswith('global_')):3d} "
              f"SALU {sum(n for k, n in c.items() if k.startswith('s_')):4d} "
              f"scratch {sum(n for k, n in c.items() if k.startswith('scratch_')):3d}")


if __name__ == "__main__":
    main()
