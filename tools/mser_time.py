import importlib, os, time, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
fm3d = importlib.import_module("3dfeaturematcher_amd")
S = importlib.import_module("3dfeaturematcher_amd.synth")
img = S.make_frame_pair(2000, seed=71).img1
ctx = fm3d.Context(fm3d.Settings.default())
F = fm3d.Features(ctx)
for i in range(4):
    t = time.perf_counter(); k = F.mser(img); print("mser", len(k), 1e3 * (time.perf_counter() - t), "ms", flush=True)
imgs = [S.make_frame_pair(2000, seed=71 + i).img1 for i in range(16)]
for i in range(3):
    t = time.perf_counter(); ks = F.mser_batch(imgs); dt = time.perf_counter() - t
    print("mser batch", len(imgs), "images", sum(len(k) for k in ks), "keypoints", 1e3 * dt, "ms",
          len(imgs) / dt, "images/s", flush=True)
ctx.close()
