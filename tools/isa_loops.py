"""Static instruction counts per loop of one kernel in a hipcc -S listing (gfx950).

    hipcc ... --cuda-device-only -S -o k.s  &&  python tools/isa_loops.py k.s <kernel-symbol-substring>

Prints, for every loop with more than 100 VALU instructions, its VALU count, SGPR
reloads from VGPR lanes (v_readlane), fp64 multiplies, scratch accesses and scalar loads.
"""
import re
import sys
from collections import Counter


def main():
    text = open(sys.argv[1]).read().split("\n")
    key = sys.argv[2] if len(sys.argv) > 2 else "lm2_kernel"
    start = next(i for i, l in enumerate(text) if re.match(r"^_Z\w*" + key + r"\w*:", l))
    end = next(i for i in range(start, len(text)) if text[i].startswith(".Lfunc_end"))
    lines = text[start:end]
    # the "Loop Header" note is on the label's line, or on the next one for nested loops
    heads = [(i, l.split(":")[0]) for i, l in enumerate(lines) if l.startswith(".LBB") and
             ("Loop Header" in l or (i + 1 < len(lines) and "Loop Header" in lines[i + 1] and
                                     not lines[i + 1].startswith(".LBB")))]
    for i, h in heads:
        ends = [j for j, l in enumerate(lines) if re.search(r"s_c?branch\w* " + re.escape(h) + r"$", l)]
        if not ends:
            continue
        body = lines[i:max(ends) + 1]
        c = Counter(l.strip().split()[0] for l in body if l.strip() and not l.strip().startswith((".", ";")))
        v = sum(n for k, n in c.items() if k.startswith("v_"))
        if v > 100:
            print(h, i, "VALU", v, "readlane", c["v_readlane_b32"], "f64mul", c["v_mul_f64"],
                  "scratch", sum(n for k, n in c.items() if k.startswith("scratch")),
                  "s_load", sum(n for k, n in c.items() if k.startswith("s_load")))


if __name__ == "__main__":
    main()
