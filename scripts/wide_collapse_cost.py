import sys, time, numpy as np
sys.path.insert(0, '/root/repo/pathtracer-cpp_amd')
from ptamd import scenes
import ptamd
sc = scenes.sphere_in_cornell(223, (64, 64))
b = ptamd.BVH.from_scene(sc); b.build()
N = b.nodes
print(N.dtype, len(N))
left = N['left'].astype(np.int64); right = N['right'].astype(np.int64)
lb = np.stack([N['lb'][:, i] for i in range(3)], 1).astype(np.float64) if N['lb'].ndim == 2 else None
rt = np.stack([N['rt'][:, i] for i in range(3)], 1).astype(np.float64)
ext = rt - lb
SA = 2 * (ext[:, 0] * ext[:, 1] + ext[:, 1] * ext[:, 2] + ext[:, 2] * ext[:, 0])
SA /= SA[0]
isleaf = (left == -1) & (right == -1)
nn = len(N)
W = 8
# greedy (build_wide)
area = ext[:, 0] * ext[:, 1] + ext[:, 1] * ext[:, 2] + ext[:, 2] * ext[:, 0]
queue = [0]; greedy = 0.0; nw = 0; kids_tot = 0
w = 0
while w < len(queue):
    n = queue[w]; w += 1
    nw += 1; greedy += SA[n]
    kids = [left[n], right[n]]
    while len(kids) < W:
        best = -1; ba = -1
        for i, k in enumerate(kids):
            if not isleaf[k] and area[k] > ba: ba = area[k]; best = i
        if best < 0: break
        k = kids[best]; kids[best] = left[k]; kids.append(right[k])
    kids_tot += len(kids)
    for k in kids:
        if not isleaf[k]: queue.append(k)
print('greedy: wide nodes', nw, 'avg kids %.2f' % (kids_tot / nw), 'sum SA (node visits per line) %.3f' % greedy)
# DP
t0 = time.time()
INF = float('inf')
# post-order
order = []
st = [0]
while st:
    n = st.pop(); order.append(n)
    if not isleaf[n]: st.append(left[n]); st.append(right[n])
order.reverse()
Cin = np.zeros(nn); D = np.full((nn, W + 1), INF)
Cnode = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
for n in order:
    if isleaf[n]:
        D[n, 1:] = 0.0
        continue
    l, r = left[n], right[n]
    Dl, Dr = D[l], D[r]
    # open n into <= 8 slots
    best8 = min(Dl[k] + Dr[W - k] for k in range(1, W))
    Cin[n] = Cnode * SA[n] + best8
    D[n, 1] = Cin[n]
    for i in range(2, W + 1):
        v = min(Dl[k] + Dr[i - k] for k in range(1, i))
        D[n, i] = min(Cin[n], v)
print('dp: sum SA %.3f (%.1f s)' % (Cin[0], time.time() - t0))
