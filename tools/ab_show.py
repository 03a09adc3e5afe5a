"""Summarises tools/ab.sh results: python tools/ab_show.py [glob]"""
import glob
import json
import sys

for f in sorted(glob.glob(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ab_*.json")):
    d = json.load(open(f))
    l = d["lm_profile"]
    print(f"{f:40s} lm {d['stages_ms']['lm_ms']:7.1f} ms kept {d['counts']['kept']} "
          f"kc/pass {l['kcycles_per_pass_by_class']} life {l['group_life_mean_over_max']:.3f} "
          f"chain c/round {l.get('chain_cycles_per_round', 0):.0f}")
