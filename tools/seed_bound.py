"""How tight a per-query kNN seed bound from Morton-ordered candidate windows is (CPU, numpy):
the K-th smallest distance of a window of Morton neighbours around the query's cell, or the largest
of per-group minima, against the query's true K-th distance, and how many candidates fall inside it
(the candidates a seeded scan would still insert).  DESIGN.md section 3, "kNN"."""
import numpy as np
rng = np.random.default_rng(0)
def morton(c):
    code = np.zeros(len(c), dtype=np.int64)
    for bit in range(4):
        for a in range(3):
            code |= ((c[:, a] >> bit) & 1) << (3 * bit + a)
    return code
def analyse(p, K=16, W=16, win_mult=1):
    N = len(p)
    lo, hi = p.min(0), p.max(0)
    sc = 16.0 / (hi - lo)
    cell = np.clip(((p - lo) * sc).astype(int), 0, 15)
    code = morton(cell)
    order = np.argsort(code, kind='stable')
    sorted_codes = code[order]
    d2 = ((p[:, None, :] - p[None, :, :]) ** 2).sum(-1)
    true_k = np.sort(d2, axis=1)[:, K - 1]
    res_T, counts = [], []
    for q in range(N):
        c = code[q]
        lo_i = np.searchsorted(sorted_codes, c, 'left'); hi_i = np.searchsorted(sorted_codes, c, 'right')
        Wt = W * win_mult
        w0 = min(max(lo_i + (hi_i - lo_i) // 2 - Wt // 2, 0), N - Wt)
        win = order[w0:w0 + Wt]
        dw = np.sort(d2[q, win])
        T = dw[K - 1]   # K-th smallest of the window (= max when Wt == K)
        res_T.append(T / true_k[q]); counts.append((d2[q] <= T).sum())
    return np.median(res_T), np.mean(counts), np.percentile(counts, 90)
g = rng.standard_normal((2048, 3))
v = rng.standard_normal((2048, 3)); s = v / np.linalg.norm(v, axis=1, keepdims=True) * np.array([1, 0.6, 0.3])
for name, p in [("gauss", g), ("ellipsoid surface", s)]:
    for wm in (1, 2, 4):
        r = analyse(p, win_mult=wm)
        print(f"{name:18s} window {16*wm:3d}: T/d16 median {r[0]:.2f}, candidates within T mean {r[1]:.1f} (p90 {r[2]:.0f})")

def analyse2(p, K=16, Wt=64, G=16):
    N = len(p)
    lo, hi = p.min(0), p.max(0)
    sc = 16.0 / (hi - lo)
    cell = np.clip(((p - lo) * sc).astype(int), 0, 15)
    code = morton(cell)
    order = np.argsort(code, kind='stable')
    sorted_codes = code[order]
    d2 = ((p[:, None, :] - p[None, :, :]) ** 2).sum(-1)
    true_k = np.sort(d2, axis=1)[:, K - 1]
    rs, cs = [], []
    for q in range(N):
        c = code[q]
        lo_i = np.searchsorted(sorted_codes, c, 'left'); hi_i = np.searchsorted(sorted_codes, c, 'right')
        w0 = min(max(lo_i + (hi_i - lo_i) // 2 - Wt // 2, 0), N - Wt)
        dw = d2[q, order[w0:w0 + Wt]].reshape(G, Wt // G)
        T = dw.min(1).max()
        rs.append(T / true_k[q]); cs.append((d2[q] <= T).sum())
    return np.median(rs), np.mean(cs), np.percentile(cs, 90)
for name, p in [("gauss", g), ("ellipsoid surface", s)]:
    for Wt in (32, 64, 96, 128):
        r = analyse2(p, Wt=Wt)
        print(f"{name:18s} group-min bound, window {Wt:3d} (16 groups of {Wt//16}): T/d16 {r[0]:.2f}, within T {r[1]:.1f} (p90 {r[2]:.0f})")
