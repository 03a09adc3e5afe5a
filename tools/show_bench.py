"""Print the headline numbers of a bench JSON line (gpurun_out/bench_<tag>.json)."""
import json
import sys

for path in sys.argv[1:]:
    d = json.load(open(path))
    lp = d.get("lm_profile", {})
    print(path, f"value {d['value']:.0f} kp/s  lm {d['stages_ms']['lm_ms']:.1f} ms  kept {d['counts']['kept']}",
          "kcyc/pass", lp.get("kcycles_per_pass_by_class"), "wait", round(lp.get("wait_over_terms", 0), 3),
          "life", round(lp.get("group_life_mean_over_max", 0), 3), "chain", round(lp.get("chain_busy") or 0, 3))
