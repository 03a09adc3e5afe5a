"""Independent pure-Python statement of OpenCV 2.4.9's grey-image MSER flood (features2d/src/mser.cpp:
preprocessMSER_8UC1, extractMSER_8UC1_Pass, MSERMergeComp, MSERNewHistory, MSERVariationCalc,
MSERStableCheck) and of cvFitEllipse2 (imgproc/src/shapedescr.cpp) with cv::solve(DECOMP_SVD)
(core/src/lapack.cpp: JacobiSVDImpl_, SVBkSbImpl_) -- test infrastructure that pins oracle/orc_mser.c.

Written index-based over flat Python lists (no pointers, no padded image), so it shares no code or
layout with the C oracle: pixel p = y * w + x, neighbours in OpenCV's direction order (right, down,
left, up), one LIFO list per grey level, components as dicts.  Small images only (pure Python).
"""
import math

import numpy as np

_EPS = 2.220446049250313e-16
_DBL_MIN = 2.2250738585072014e-308


def _f32(v):
    return float(np.float32(v))


def mser_regions(img, delta=5, min_area=60, max_area=14400, max_variation=0.25, min_diversity=0.2):
    """[(colour, [(x, y), ...])] in emission order, points in region-list order"""
    img = np.asarray(img, dtype=np.uint8)
    h, w = img.shape
    out = []
    for color, vals in ((-1, 255 - img.astype(np.int32)), (1, img.astype(np.int32))):
        out += _pass(vals.ravel().tolist(), w, h, color, delta, min_area, max_area, max_variation, min_diversity)
    return out


def _pass(v, w, h, color, delta, min_area, max_area, max_var, min_div):
    n = w * h
    visited = [False] * n
    dirn = [0] * n
    buckets = [[] for _ in range(256)]
    nxt = [-1] * n  # point list links (by pixel index)
    hist = []  # [shortcut, child, stable, val, size]
    regions = []

    def new_comp(level):
        return {"level": level, "size": 0, "var": 0.0, "dvar": 1, "hist": -1, "head": -1, "tail": -1}

    def stable_check(c):
        hi = c["hist"]
        if hi < 0 or hist[hi][4] <= min_area or hist[hi][4] >= max_area:
            return False
        H = hist[hi]
        div = _f32(_f32(H[4] - H[2]) / _f32(H[4]))
        # MSERVariationCalc
        sc = H[0]
        while sc != hist[sc][0] and hist[sc][3] + delta > c["level"]:
            sc = hist[sc][0]
        ch = hist[sc][1]
        while ch != hist[ch][1] and hist[ch][3] + delta <= c["level"]:
            sc = ch
            ch = hist[ch][1]
        H[0] = sc
        var = _f32(_f32(c["size"] - hist[sc][4]) / _f32(hist[sc][4]))
        dvar = c["var"] < var or H[3] + 1 < c["level"]
        stable = dvar and not c["dvar"] and c["var"] < max_var and div > min_div
        c["var"] = var
        c["dvar"] = 1 if dvar else 0
        if stable:
            H[2] = H[4]
        return stable

    def new_history(c):
        hi = len(hist)
        if c["hist"] < 0:
            hist.append([hi, hi, 0, c["level"], c["size"]])
        else:
            P = hist[c["hist"]]
            P[1] = hi
            hist.append([P[0], hi, P[2], c["level"], c["size"]])
        c["hist"] = hi

    def emit(c):
        pts, p = [], c["head"]
        for _ in range(hist[c["hist"]][4]):
            pts.append((p % w, p // w))
            p = nxt[p]
        regions.append((color, pts))

    def merge(top, below):
        """MSERMergeComp(top, below, below, history): returns the merged component"""
        win, lose = (top, below) if top["size"] >= below["size"] else (below, top)
        hi = len(hist)
        if win["hist"] < 0:
            rec = [hi, hi, 0, win["level"], win["size"]]
        else:
            P = hist[win["hist"]]
            P[1] = hi
            rec = [P[0], hi, P[2], win["level"], win["size"]]
        if lose["hist"] >= 0 and hist[lose["hist"]][2] > rec[2]:
            rec[2] = hist[lose["hist"]][2]
        hist.append(rec)
        if top["size"] > 0 and below["size"] > 0:
            nxt[win["tail"]] = lose["head"]
        m = {"level": below["level"], "var": win["var"], "dvar": win["dvar"], "hist": hi,
             "head": win["head"] if win["size"] > 0 else lose["head"],
             "tail": lose["tail"] if lose["size"] > 0 else win["tail"],
             "size": top["size"] + below["size"]}
        return m

    stack = [{"level": 256}]
    cur = 0
    visited[cur] = True
    stack.append(new_comp(v[cur]))
    level = v[cur]
    while True:
        descended = False
        while dirn[cur] < 4:
            x, y = cur % w, cur // w
            d = dirn[cur]
            nx, ny = x + (1, 0, -1, 0)[d], y + (0, 1, 0, -1)[d]
            if 0 <= nx < w and 0 <= ny < h:
                nb = ny * w + nx
                if not visited[nb]:
                    visited[nb] = True
                    if v[nb] < v[cur]:
                        buckets[level].append(cur)
                        dirn[cur] += 1
                        level = v[nb]
                        cur = nb
                        stack.append(new_comp(level))
                        descended = True
                        break
                    buckets[v[nb]].append(nb)
            dirn[cur] += 1
        if descended:
            continue
        c = stack[-1]
        if c["size"] > 0:
            nxt[c["tail"]] = cur
        else:
            c["head"] = cur
        nxt[cur] = -1
        c["tail"] = cur
        c["size"] += 1
        if buckets[level]:
            cur = buckets[level].pop()
            continue
        nl = next((g for g in range(v[cur] + 1, 256) if buckets[g]), None)
        if nl is None:
            break
        level = nl
        cur = buckets[level].pop()
        if nl < stack[-2]["level"]:
            if stable_check(stack[-1]):
                emit(stack[-1])
            new_history(stack[-1])
            stack[-1]["level"] = nl
        else:
            while True:
                top = stack.pop()
                stack[-1] = merge(top, stack[-1])
                if nl <= stack[-1]["level"]:
                    break
                if nl < stack[-2]["level"]:
                    if stable_check(stack[-1]):
                        emit(stack[-1])
                    new_history(stack[-1])
                    stack[-1]["level"] = nl
                    break
    return regions


def _svd_solve(At, b):
    """cv::solve(A, b, DECOMP_SVD) with At = A^T as a list of rows (destroyed)"""
    n, m = len(At), len(At[0])
    W = [sum_sq(r) for r in At]
    Vt = [[1.0 if i == k else 0.0 for k in range(n)] for i in range(n)]
    eps = _EPS * 10
    for _ in range(max(m, 30)):
        changed = False
        for i in range(n - 1):
            for j in range(i + 1, n):
                Ai, Aj = At[i], At[j]
                a, bb = W[i], W[j]
                p = 0.0
                for k in range(m):
                    p += Ai[k] * Aj[k]
                if abs(p) <= eps * math.sqrt(a * bb):
                    continue
                p *= 2
                beta = a - bb
                gamma = math.sqrt(p * p + beta * beta)
                if beta < 0:
                    dl = (gamma - beta) * 0.5
                    s = math.sqrt(dl / gamma)
                    c = p / (gamma * s * 2)
                else:
                    c = math.sqrt((gamma + beta) / (gamma * 2))
                    s = p / (gamma * c * 2)
                a = bb = 0.0
                for k in range(m):
                    t0 = c * Ai[k] + s * Aj[k]
                    t1 = -s * Ai[k] + c * Aj[k]
                    Ai[k] = t0
                    Aj[k] = t1
                    a += t0 * t0
                    bb += t1 * t1
                W[i], W[j] = a, bb
                changed = True
                Vi, Vj = Vt[i], Vt[j]
                for k in range(n):
                    t0 = c * Vi[k] + s * Vj[k]
                    t1 = -s * Vi[k] + c * Vj[k]
                    Vi[k], Vj[k] = t0, t1
        if not changed:
            break
    W = [math.sqrt(sum_sq(r)) for r in At]
    for i in range(n - 1):
        j = i
        for k in range(i + 1, n):
            if W[j] < W[k]:
                j = k
        if i != j:
            W[i], W[j] = W[j], W[i]
            At[i], At[j] = At[j], At[i]
            Vt[i], Vt[j] = Vt[j], Vt[i]
    for i in range(n):
        if W[i] > _DBL_MIN:
            t = 1.0 / W[i]
            At[i] = [u * t for u in At[i]]
    x = [0.0] * n
    thr = 0.0
    for wi in W:
        thr += wi
    thr *= _EPS * 2
    for i in range(n):
        if abs(W[i]) <= thr:
            continue
        wi = 1 / W[i]
        s = 0.0
        for k in range(m):
            s += At[i][k] * b[k]
        s *= wi
        for k in range(n):
            x[k] = x[k] + s * Vt[i][k]
    return x


def sum_sq(r):
    s = 0.0
    for t in r:
        s += t * t
    return s


def fit_ellipse(points):
    """cvFitEllipse2 on integer points (list of (x, y)): (cx, cy, width, height, angle) as Python floats
    holding float32 values; atan2 / sin are passed in by the caller's module (numpy's differ from the
    oracle's deterministic ones in the last bit), so this returns the three solves too."""
    n = len(points)
    cx = cy = np.float32(0)
    for x, y in points:
        cx = np.float32(cx + np.float32(x))
        cy = np.float32(cy + np.float32(y))
    cx = np.float32(cx / np.float32(n))
    cy = np.float32(cy / np.float32(n))
    P = [(float(np.float32(np.float32(x) - cx)), float(np.float32(np.float32(y) - cy))) for x, y in points]
    At = [[-px * px for px, py in P], [-py * py for px, py in P], [-px * py for px, py in P],
          [px for px, py in P], [py for px, py in P]]
    g = _svd_solve(At, [10000.0] * n)
    rp = _svd_solve([[2 * g[0], g[2]], [g[2], 2 * g[1]]], [g[3], g[4]])
    At = [[(px - rp[0]) * (px - rp[0]) for px, py in P], [(py - rp[1]) * (py - rp[1]) for px, py in P],
          [(px - rp[0]) * (py - rp[1]) for px, py in P]]
    g2 = _svd_solve(At, [1.0] * n)
    return float(cx), float(cy), g, rp, g2
