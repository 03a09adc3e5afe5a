"""Analyse an FM3D_LM_TRACE dump: per-point fetch/finish ticks (100 MHz wall clock),
passes and workgroup.  python tools/lm_trace.py trace.bin [nfev.npy]"""
import sys

import numpy as np

t = np.fromfile(sys.argv[1], dtype=np.int64).reshape(-1, 4)
t0 = t[t[:, 0] > 0, 0].min()
start = (t[:, 0] - t0) / 1e5  # ms
end = (t[:, 1] - t0) / 1e5
passes = t[:, 2]
dur = end - start
T = end.max()
print(f"points {len(t)}  span {T:.1f} ms")
for q in (50, 90, 99, 100):
    print(f"  passes p{q}: {np.percentile(passes, q):.0f}   duration p{q}: {np.percentile(dur, q):.1f} ms")
late = np.argsort(-end)[:10]
print("last finishers (start ms, end ms, passes, us/pass, group):")
for i in late:
    print(f"  {start[i]:8.1f} {end[i]:8.1f} {passes[i]:6d} {1e3 * dur[i] / max(passes[i], 1):8.1f} {t[i, 3]}")
hist = np.histogram(end, bins=20, range=(0, T))[0]
print("finish-time histogram (20 bins):", hist.tolist())
grp = t[:, 3]
gend = np.zeros(grp.max() + 1)
np.maximum.at(gend, grp, end)
print(f"group end: mean {gend.mean():.1f} ms, max {gend.max():.1f}, p10 {np.percentile(gend, 10):.1f}")
busy = passes > 50
print(f"us/pass for points with > 50 passes: median {np.median(1e3 * dur[busy] / passes[busy]):.1f}")
