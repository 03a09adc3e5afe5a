"""Summarise a tools/prof_lm.sh run (rocprofv3 kernel trace + separate --pmc passes) for
one kernel: HBM bytes per launch (FETCH_SIZE doubled per MI355X_MICROARCH.md, + WRITE_SIZE),
L2 hit rate, VALU activity and wave wait fractions.

    python tools/pmc_summary.py gpurun_out/prof_<tag> [kernel-substring] [--out profiles/x.json]
"""
import csv
import glob
import json
import os
import sys


def main():
    d = sys.argv[1]
    kname = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else "lm2_kernel"
    out = sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else None
    agg, n = {}, {}
    for f in sorted(glob.glob(os.path.join(d, "pmc*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            if kname in r["Kernel_Name"]:
                c = r["Counter_Name"]
                agg[c] = agg.get(c, 0.0) + float(r["Counter_Value"])
                n.setdefault(c, set()).add(r["Dispatch_Id"])
    agg = {c: v / len(n[c]) for c, v in agg.items()}  # per launch
    dur = None
    for r in csv.DictReader(open(os.path.join(d, "trace", "run_kernel_stats.csv"))):
        if kname in r["Name"]:
            dur = float(r["AverageNs"])
    res = {"kernel": kname, "trace_avg_ns": dur, "counters_per_launch": agg,
           "launches": max((len(v) for v in n.values()), default=0)}
    if "FETCH_SIZE" in agg and "WRITE_SIZE" in agg:
        rd, wr = 2 * agg["FETCH_SIZE"] * 1024, agg["WRITE_SIZE"] * 1024
        res.update(hbm_read_bytes=rd, hbm_write_bytes=wr, hbm_bytes_per_launch=rd + wr,
                   hbm_GBps=(rd + wr) / dur if dur else None)
    if "TCC_HIT_sum" in agg:
        res["l2_hit"] = agg["TCC_HIT_sum"] / max(agg["TCC_HIT_sum"] + agg["TCC_MISS_sum"], 1)
    if "SQ_WAVE_CYCLES" in agg:
        wc = agg["SQ_WAVE_CYCLES"]
        res["wait_any_frac"] = agg["SQ_WAIT_ANY"] / wc
        res["wait_inst_frac"] = agg["SQ_WAIT_INST_ANY"] / wc
        res["active_frac"] = agg["SQ_ACTIVE_INST_ANY"] / wc
        if dur:
            # SQ_ACTIVE_INST_VALU counts quad-cycles per wave; 1024 SIMDs at the busy clock
            simd_cycles = 1024 * dur * 1e-9 * (agg["SQ_BUSY_CYCLES"] / 32 / (dur * 1e-9))
            res["valu_busy_per_simd"] = 4 * agg["SQ_ACTIVE_INST_VALU"] / simd_cycles
            res["busy_clock_ghz"] = agg["SQ_BUSY_CYCLES"] / 32 / dur
    if "SQ_LDS_IDX_ACTIVE" in agg:
        # LDS: extra cycles from bank conflicts per LDS-array cycle; instructions per wave-cycle
        res["lds_bank_conflict_frac"] = agg.get("SQ_LDS_BANK_CONFLICT", 0.) / max(agg["SQ_LDS_IDX_ACTIVE"], 1)
        res["lds_addr_conflict_frac"] = agg.get("SQ_LDS_ADDR_CONFLICT", 0.) / max(agg["SQ_LDS_IDX_ACTIVE"], 1)
        res["lds_unaligned_stall_frac"] = agg.get("SQ_LDS_UNALIGNED_STALL", 0.) / max(agg["SQ_LDS_IDX_ACTIVE"], 1)
    if "--workload" in sys.argv:  # keypoints,ray,levels of the bench command profiled
        k, r, l = (int(x) for x in sys.argv[sys.argv.index("--workload") + 1].split(","))
        res["workload"] = {"keypoints": k, "ray": r, "levels": l}
    if "--command" in sys.argv:
        res["command"] = sys.argv[sys.argv.index("--command") + 1]
    calib = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles", "r02_fetch_calibration.json")
    if os.path.exists(calib):
        res["calibration"] = os.path.relpath(os.path.abspath(calib), os.path.join(os.path.dirname(calib), ".."))
    res["note"] = ("FETCH_SIZE/WRITE_SIZE in KiB; gfx950 FETCH_SIZE reads half the bytes of wide streaming loads "
                   "(doubled here); each counter group measured in its own rocprofv3 --pmc pass")
    print(json.dumps(res, indent=1))
    if out:
        with open(out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
