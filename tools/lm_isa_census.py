"""Static ISA census of the LM kernel's residual (EVAL) and Jacobian (JAC) chunks.

    python tools/lm_isa_census.py [--asm /tmp/lm2g.s] [--out profiles/r06_lm_isa_census.json]

Compiles csrc/fm3d_lm2.hip for gfx950 exactly as the Makefile does, plus -gline-tables-only (the
.loc line table; the instruction stream differs from the production build by a handful of moves,
waits and spill slots, listed in the output), then, in lm2_kernel<false, false> (one pose, pixel-order
sums: the default launch), takes the software-pipelined chunk loops of the FAST evaluation passes:

  * EVAL -- one residual evaluation per entry (NEV = 1, `front` / `back` lambdas): an iteration
    handles 4 chunks of 64 entries, 4 x 64 pixel evaluations;
  * JAC  -- both forward-difference columns per entry (NEV = 2, `front2` / `back2`): an iteration
    handles 2 chunks, 2 x 2 x 64 pixel evaluations.

Every instruction of the loop's own blocks (child loops -- the ring-space waits -- excluded) is
attributed to the source construct its line belongs to (geometry2's ray-plane, bounding box,
projection, gather-address lines; the division sequences; bilinear_f; enorm_term2; the ring
writes; the slab loads / stores; lane masks ...) and to an opcode class.  Blocks that only the rare
paths reach (a failing pixel's plane_code, the enorm slow branch, the ring counter re-read) are
"cold": they are reported apart and left out of the per-pixel-evaluation figures.  VALU counts are
wave instructions; per pixel evaluation they are lane instructions (x 64 / 64 entries).
"""
from __future__ import annotations

import argparse
import json
import os
import re
import subprocess
import sys
from collections import Counter, defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "3dfeaturematcher_amd", "csrc")
KERNEL = "_ZN4fm3d10lm2_kernelILb0ELb0EEEvNS_8LMParamsE"


def compile_asm(path, debug):
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off", "-fno-fast-math",
           "-fhip-fp32-correctly-rounded-divide-sqrt", "-I.", "-I../../include", "-x", "hip", "--cuda-device-only",
           "-S", "fm3d_lm2.hip", "-o", path] + (["-gline-tables-only"] if debug else [])
    subprocess.run(cmd, cwd=CSRC, check=True, capture_output=True)


def func_lines(text, name):
    s = next(i for i, l in enumerate(text) if l.startswith(name + ":"))
    e = next(i for i in range(s, len(text)) if text[i].startswith(".Lfunc_end"))
    return text[s:e]


def opcodes(lines):
    out = []
    for l in lines:
        x = l.strip()
        if not x or x.startswith((".", ";")) or x.endswith(":"):
            continue
        out.append(x.split()[0])
    return out


# source constructs: (file, first line, last line) -> tag, found by pattern in the sources so the
# tool follows edits
def source_map():
    def span(path, start_pat, end_pat=None, n=None):
        lines = open(path).read().split("\n")
        s = next(i for i, l in enumerate(lines) if re.search(start_pat, l)) + 1
        if n is not None:
            return s, s + n - 1
        e = next(i for i in range(s, len(lines)) if re.search(end_pat, lines[i])) + 1
        return s, e

    lm = os.path.join(CSRC, "fm3d_lm2.hip")
    fd = os.path.join(CSRC, "fm3d_fastdiv.h")
    m = []
    g0, g1 = span(lm, r"Geo2 geometry2\(", r"^}")
    src = open(lm).read().split("\n")

    def gline(pat):
        return next(i for i in range(g0 - 1, g1) if re.search(pat, src[i])) + 1

    l_nn = gline(r"const double nn = n0")
    l_kk = gline(r"const double kk =")
    l_P = gline(r"const double P0 = kk")
    l_box = gline(r"r.inbox = __ballot")
    l_x = gline(r"double x = pc->R\[0\]")
    l_v = gline(r"const double v = yd")
    l_good = gline(r"r.good = r.inbox")
    l_fx = gline(r"r.fx = \(float\)")
    l_off = gline(r"r.off = sel_mask_u32")
    m += [("fm3d_lm2.hip", g0, l_nn - 1, "geometry: setup"),
          ("fm3d_lm2.hip", l_nn, l_nn, "ray-plane: n.v (IEEE f64)"),
          ("fm3d_lm2.hip", l_kk, l_kk, "ray-plane: k = mm / nn (division)"),
          ("fm3d_lm2.hip", l_P, l_P, "ray-plane: P = k v (IEEE f64)"),
          ("fm3d_lm2.hip", l_box, l_box, "isInBoundingBox: compares + ballots (lane masks)"),
          ("fm3d_lm2.hip", l_x, l_v, "projectPoints: rotation, distortion, intrinsics (IEEE f64; 1/z division)"),
          ("fm3d_lm2.hip", l_good, l_good + 1, "isPixelGood: compares + ballots (lane masks)"),
          ("fm3d_lm2.hip", l_fx, l_fx + 1, "sample coordinates: (float)(scale u) (conversion)"),
          ("fm3d_lm2.hip", l_fx + 2, l_off, "gather address: floor, int, offset, mask (addressing)"),
          ("fm3d_lm2.hip", *span(lm, r"float bilinear_f\(", r"^}"), "getBilinearInterpPix32f (IEEE f32; u8 -> f32)"),
          ("fm3d_lm2.hip", *span(lm, r"float bilinear_w\(", r"^}"), "getBilinearInterpPix32f (IEEE f32; u8 -> f32)"),
          ("fm3d_lm2.hip", *span(lm, r"double enorm_term2\(", r"^}"), "enorm: x*x term + slow-path ballots"),
          ("fm3d_lm2.hip", *span(lm, r"double sel_mask\(", r"^}"), "lane masks: sel_mask"),
          ("fm3d_lm2.hip", *span(lm, r"unsigned sel_mask_u32\(", r"^}"), "lane masks: sel_mask"),
          ("fm3d_lm2.hip", *span(lm, r"LaneMask in_mask\(", r"^}"), "lane masks: in_mask"),
          ("fm3d_lm2.hip", *span(lm, r"void reserve\(int c\)", r"^    }"), "ring: reserve (space check)"),
          ("fm3d_lm2.hip", *span(lm, r"void write_terms\(", r"^    }"), "ring: term rows + tag (LDS)"),
          ("fm3d_lm2.hip", *span(lm, r"int plane_code\(", r"^}"), "rare: plane_code"),
          ("fm3d_lm2.hip", *span(lm, r"auto load = \[&\]", r"^                        };"), "slab loads (global)"),
          ("fm3d_lm2.hip", *span(lm, r"auto gather = \[&\]", r"^                        };"), "image-2 gathers (global)"),
          ("fm3d_fastdiv.h", *span(fd, r"double mdiv_fast\(", r"^}"), "division: Jacobian (r - F) / h (mdiv_fast)"),
          ("fm3d_fastdiv.h", *span(fd, r"double mdiv\(", r"^}"), "division: Jacobian (r - F) / h (mdiv)"),
          ("fm3d_fastdiv.h", *span(fd, r"double recip_z_lo\(", r"^}"), "division: 1 / z (recip_z_lo)"),
          ("fm3d_fastdiv.h", *span(fd, r"double div_nn\(", r"^}"), "ray-plane: k = mm / nn (division)")]
    return m


# which categories restate the reference's IEEE arithmetic (the 91 algorithmic flops and the casts
# the reference performs), which are the kernel's own machinery
ALGORITHMIC = ("ray-plane", "projectPoints", "getBilinearInterpPix32f", "enorm: x*x", "division",
               "sample coordinates", "residual", "tests as ballots", "floorf")


def opclass(op):
    if op.startswith(("global_", "buffer_", "scratch_")):
        return "global memory"
    if op.startswith("ds_"):
        return "LDS"
    if op.startswith("s_"):
        return "scalar"
    if not op.startswith("v_"):
        return "other"
    if op.startswith(("v_div_", "v_rcp_", "v_rsq_", "v_frexp", "v_ldexp", "v_trig", "v_sqrt")):
        return "VALU div/rcp/scale"
    if op.startswith("v_cvt") or op.startswith("v_cvt_"):
        return "VALU conversion"
    if op.startswith(("v_cmp", "v_cmpx")):
        return "VALU compare"
    if op.startswith("v_cndmask"):
        return "VALU select"
    if op.startswith(("v_mov", "v_readfirstlane", "v_readlane", "v_writelane", "v_accvgpr")):
        return "VALU move"
    if "_f64" in op:
        return "VALU f64"
    if "_f32" in op or "_f16" in op:
        return "VALU f32"
    return "VALU integer/bit"


def parse(text):
    """blocks of the kernel: label, loop header, instructions with (file, line)"""
    lines = func_lines(text, KERNEL)
    files = {}
    for l in text:
        mm = re.match(r"\s*\.file\s+(\d+)\s+\"([^\"]*)\"\s+\"([^\"]*)\"", l)
        if mm:
            files[int(mm.group(1))] = os.path.basename(mm.group(3))
    blocks, cur, loc = [], None, ("?", 0)
    for i, l in enumerate(lines):
        if l.startswith(".LBB") or l.startswith("; %bb."):
            label = l.split(":")[0].strip().lstrip(".").replace("; %bb.", "BB?")
            notes = " ".join([l] + [x for x in lines[i + 1:i + 3] if x.strip().startswith(";")])
            header = None
            if "This Loop Header" in notes or "This Inner Loop Header" in notes:
                header = label.lstrip("L")
            else:
                mm = re.search(r"in Loop: Header=(BB\w+)", notes)
                header = mm.group(1) if mm else None
            depth = re.search(r"Depth=(\d+)", notes)
            cur = {"label": label.lstrip("L"), "loop": header, "depth": int(depth.group(1)) if depth else 0,
                   "ins": [], "succ": []}
            blocks.append(cur)
            continue
        s = l.strip()
        mm = re.match(r"\.loc\s+(\d+)\s+(\d+)", s)
        if mm:
            loc = (files.get(int(mm.group(1)), "?"), int(mm.group(2)))
            continue
        if cur is None or not s or s.startswith((".", ";")):
            continue
        op = s.split()[0]
        cur["ins"].append((op, loc, s))
        if op.startswith("s_cbranch") or op == "s_branch":
            cur["succ"].append(s.split()[1].lstrip(".").lstrip("L"))
    return blocks


def tag_of(loc, smap, lm_ranges):
    f, ln = loc
    for (sf, a, b, tag) in smap:
        if f == sf and a <= ln <= b:
            return tag
    if f == "amd_warp_functions.h":
        return "tests as ballots: bounding box, isPixelGood, enorm's classes (v_cmp -> SGPR mask)"
    if f == "fm3d_fastdiv.h":
        return "division: helper sequences (rcp + Newton + Markstein)"
    if f == "__clang_hip_math.h":
        return "floorf (bilinear window, gather address)"
    if f == "fm3d_lm2.hip":
        for (a, b, tag) in lm_ranges:
            if a <= ln <= b:
                return tag
        return "pass loop glue (fm3d_lm2.hip)"
    return f"other ({f})"


def census(blocks, header, smap, lm_ranges, evals_per_iter):
    mine = [b for b in blocks if b["loop"] == header]
    # cold blocks: those that hold a rare construct (failure code, enorm slow rows, ring counter
    # re-read) -- their instructions run only when a pixel fails, a chunk has raw values, or the
    # ring space seen last is used up
    def cold(b):
        tags = {tag_of(loc, smap, lm_ranges) for (_, loc, _) in b["ins"]}
        txt = " ".join(x for (_, _, x) in b["ins"])
        return ("rare: plane_code" in tags or "s_swappc" in txt or "v_ffbl" in txt
                or any(t == "ring: reserve (space check)" for t in tags) and "ds_read" in txt
                or "slow rows" in tags
                # the division operator (v_div_scale / v_div_fmas / v_div_fixup): only the guarded
                # fallbacks of mdiv / recip_z_lo / div_nn use it, on lanes outside their ranges
                or "v_div_scale" in txt or "v_div_fixup" in txt)
    hot = [b for b in mine if not cold(b)]
    colds = [b for b in mine if cold(b)]
    by_tag = defaultdict(Counter)
    by_class = Counter()
    for b in hot:
        for (op, loc, _) in b["ins"]:
            t = tag_of(loc, smap, lm_ranges)
            c = opclass(op)
            by_tag[t][c] += 1
            by_class[c] += 1
    valu = sum(n for c, n in by_class.items() if c.startswith("VALU"))
    per = lambda n: round(n * 64 / evals_per_iter, 2)  # lane instructions per pixel evaluation
    tags = {}
    for t, cc in sorted(by_tag.items(), key=lambda kv: -sum(n for c, n in kv[1].items() if c.startswith("VALU"))):
        v = sum(n for c, n in cc.items() if c.startswith("VALU"))
        tags[t] = {"valu_wave_instructions": v, "valu_lane_per_pixel_eval": per(v),
                   "algorithmic": any(t.startswith(a) or a in t for a in ALGORITHMIC),
                   "by_class": dict(cc)}
    alg = sum(d["valu_wave_instructions"] for t, d in tags.items() if d["algorithmic"])
    return {
        "loop_header": header,
        "blocks_hot": len(hot), "blocks_cold": len(colds),
        "pixel_evaluations_per_iteration": evals_per_iter,
        "valu_wave_instructions_per_iteration": valu,
        "valu_lane_instructions_per_pixel_eval": per(valu),
        "of_which_algorithmic_per_pixel_eval": per(alg),
        "of_which_overhead_per_pixel_eval": per(valu - alg),
        "by_class_per_pixel_eval": {c: per(n) for c, n in sorted(by_class.items(), key=lambda kv: -kv[1])},
        "by_construct": tags,
        "cold_blocks_valu": sum(sum(1 for (op, _, _) in b["ins"] if op.startswith("v_")) for b in colds),
    }


def find_loop(blocks, text_src, lines):
    """the loop whose own blocks carry the most lines of the given source line range"""
    score = Counter()
    for b in blocks:
        if not b["loop"]:
            continue
        for (op, loc, _) in b["ins"]:
            if loc[0] == "fm3d_lm2.hip" and lines[0] <= loc[1] <= lines[1]:
                score[b["loop"]] += 1
    return score


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--asm", default="/tmp/lm2g.s")
    ap.add_argument("--plain-asm", default="/tmp/lm2.s")
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r06_lm_isa_census.json"))
    ap.add_argument("--rebuild", action="store_true")
    args = ap.parse_args()
    if args.rebuild or not os.path.exists(args.asm):
        compile_asm(args.asm, True)
    if args.rebuild or not os.path.exists(args.plain_asm):
        compile_asm(args.plain_asm, False)
    text = open(args.asm).read().split("\n")
    plain = open(args.plain_asm).read().split("\n")
    d_ops = Counter(opcodes(func_lines(text, KERNEL))) - Counter(opcodes(func_lines(plain, KERNEL)))
    d_ops2 = Counter(opcodes(func_lines(plain, KERNEL))) - Counter(opcodes(func_lines(text, KERNEL)))
    blocks = parse(text)
    smap = source_map()
    src = open(os.path.join(CSRC, "fm3d_lm2.hip")).read().split("\n")

    def rng(start_pat, end_pat):
        s = next(i for i, l in enumerate(src) if re.search(start_pat, l)) + 1
        e = next(i for i in range(s, len(src)) if re.search(end_pat, src[i])) + 1
        return s, e

    # the lambdas of the two pipelined loops (their own lines: glue, residual, stores)
    eval_front = rng(r"auto front = \[&\]\(const Ld& A, const Ld& B, int k\)", r"^                            };")
    eval_back = rng(r"auto value = \[&\]\(float xf", r"^                            };")
    eval_pub = rng(r"auto publish = \[&\]", r"^                            };")
    eval_b2 = rng(r"auto back = \[&\]\(const St& S", r"^                            };")
    jac_front = rng(r"auto front2 = \[&\]", r"^                            };")
    jac_back = rng(r"auto back2 = \[&\]", r"^                            };")
    lm_ranges = [(eval_back[0], eval_back[1], "residual: w (I1 - I2), float -> double (IEEE)"),
                 (jac_back[0], jac_back[1], "residual + Jacobian glue (back2)"),
                 (eval_pub[0], eval_pub[1], "slab store dI + enorm term (publish)"),
                 (eval_front[0], eval_front[1], "stage glue (front)"), (jac_front[0], jac_front[1], "stage glue (front2)"),
                 (eval_b2[0], eval_b2[1], "stage glue (back)")]
    s_eval = find_loop(blocks, src, eval_back)
    s_jac = find_loop(blocks, src, jac_back)
    # the FAST variants: of the loops carrying these lambdas, the one with fewer VALU per block set
    def pick(score):
        cands = [h for h, _ in score.most_common(4)]
        def valu(h):
            return sum(1 for b in blocks if b["loop"] == h for (op, _, _) in b["ins"] if op.startswith("v_"))
        return min(cands, key=valu), {h: valu(h) for h in cands}
    h_eval, c_eval = pick(s_eval)
    h_jac, c_jac = pick(s_jac)
    out = {
        "kernel": KERNEL + " (lm2_kernel<false, false>: one pose, pixel-order sums -- the default launch)",
        "build": "csrc/Makefile flags + -gline-tables-only (for the .loc table) + --cuda-device-only -S",
        "build_difference_vs_production": {"more_in_census_build": dict(d_ops), "more_in_production": dict(d_ops2)},
        "candidates_valu": {"eval": c_eval, "jac": c_jac},
        "EVAL": census(blocks, h_eval, smap, lm_ranges, 4 * 64),
        "JAC": census(blocks, h_jac, smap, lm_ranges, 2 * 2 * 64),
    }
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)
    for k in ("EVAL", "JAC"):
        c = out[k]
        print(f"{k}: loop {c['loop_header']} {c['valu_lane_instructions_per_pixel_eval']} VALU lane-instr / pixel eval "
              f"(algorithmic {c['of_which_algorithmic_per_pixel_eval']}, overhead {c['of_which_overhead_per_pixel_eval']}); "
              f"cold blocks {c['blocks_cold']}")
        for t, d in c["by_construct"].items():
            print(f"   {d['valu_lane_per_pixel_eval']:7.2f}  {'A' if d['algorithmic'] else ' '}  {t}  {d['by_class']}")
    print("->", args.out)


if __name__ == "__main__":
    main()
