"""List-scheduling model of the LM launch's point order: per-point cost = measured
evaluations x m_dat + a fixed overhead, 3,840 slots.  Compares index order, the true longest-first
order and a dynamic image-cell order (pilot points per cell, then the cell with the highest mean
measured cost).  Input: gpurun_out/lm_cost.npz written by tools/lm_cost_features.py on the GPU box.
"""
import sys, importlib, heapq, numpy as np
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
syn = importlib.import_module('3dfeaturematcher_amd.synth')
d = np.load(__import__('os').path.join(__import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))),'gpurun_out','lm_cost.npz'))
pts, nfev = d['pts'], d['nfev']
pair = syn.make_frame_pair(100000, 640, 480, seed=7)
uv = syn.project(pair.cam, pts)
ev = nfev[:, :4].sum(1).astype(float)
R=64; u,v=uv[:,0],uv[:,1]
mdat = ((np.minimum(u + R, 639) - np.maximum(u - R, 0) + 1).clip(0) * (np.minimum(v + R, 479) - np.maximum(v - R, 0) + 1).clip(0) * np.pi / 4)
cost = ev * mdat + 2000.0   # + fixed per-point overhead
S = 3840
def makespan_static(order):
    h = [0.0]*S
    for i in order:
        t = heapq.heappop(h); heapq.heappush(h, t + cost[i])
    return max(h)
def makespan_dynamic(cell_px, pilot_per_cell=1, est='mean'):
    cx = np.clip((u // cell_px).astype(int), 0, 10**6); cy = np.clip((v // cell_px).astype(int), 0, 10**6)
    ncx = cx.max()+1; cell = cy*ncx + cx
    nc = cell.max()+1
    lists = [list(np.where(cell==c)[0]) for c in range(nc)]
    nxt = [0]*nc; csum = np.zeros(nc); ccnt = np.zeros(nc)
    gmean = [cost.mean()]
    # pilot: round-robin over cells, pilot_per_cell points each
    pilot = []
    for k in range(pilot_per_cell):
        for c in range(nc):
            if nxt[c] < len(lists[c]): pilot.append(lists[c][nxt[c]]); nxt[c]+=1
    events = []  # (finish_time, slot, point)
    t_slots = [(0.0, s) for s in range(S)]
    heapq.heapify(t_slots)
    pi = 0; done_cost = []
    pending = []  # completions not yet "known" (known when their finish time <= current time)
    total = 0
    while True:
        t, s = heapq.heappop(t_slots)
        # reveal completions finished before t
        while pending and pending[0][0] <= t:
            ft, i = heapq.heappop(pending); c = cell[i]; csum[c] += cost[i]; ccnt[c] += 1
        if pi < len(pilot):
            i = pilot[pi]; pi += 1
        else:
            best, bc = -1, -1
            m = csum.sum()/max(ccnt.sum(),1)
            for c in range(nc):
                if nxt[c] < len(lists[c]):
                    e = csum[c]/ccnt[c] if ccnt[c] > 0 else m
                    if e > best: best, bc = e, c
            if bc < 0:
                heapq.heappush(t_slots, (t, s)); break
            i = lists[bc][nxt[bc]]; nxt[bc] += 1
        heapq.heappush(pending, (t + cost[i], i))
        heapq.heappush(t_slots, (t + cost[i], s))
    return max(ft for ft, _ in pending) if pending else max(tt for tt,_ in t_slots)
base = makespan_static(np.arange(len(pts)))
orac = makespan_static(np.argsort(-cost))
ideal = cost.sum()/S
print("index", base/ideal, "oracle", orac/ideal)
for cp in ():
    for pp in (1, 2):
        m = makespan_dynamic(cp, pp)
        print("cell", cp, "pilot", pp, m/ideal, "gain vs index", 1 - m/base)
for cp in (14, 10):
    m = makespan_dynamic(cp, 1)
    print("cell", cp, "pilot 1", m/ideal, "gain vs index", 1 - m/base)
