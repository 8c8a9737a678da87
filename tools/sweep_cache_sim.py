"""Plaintext simulation of the c2sweep candidate trajectory (CPU only).

Replays bench.py --config c2sweep's synthetic reports (same generators and
seeds as tools/sweep_probe.py), runs the threshold sweep on plaintext weights
and, for every level, finds the deepest tree level that is identical in some
earlier call's tree: the level a sweep could resume from if the frontier cache
kept snapshots of every earlier call.  Prints the per-level trees' node counts.
    python3 tools/sweep_cache_sim.py [n_reports]
"""
import sys, numpy as np
import os
sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__)))]
from bench import _attrs
n_rep = int(sys.argv[1]) if len(sys.argv) > 1 else 1000000
bits, mx = 32, 255
seed = 0x4D41 + 2
pool = _attrs(np.random.default_rng(seed), bits, 10000)
rrng = np.random.default_rng(seed * 1000003)
ranks = rrng.zipf(1.1, size=n_rep)
while (ranks > len(pool)).any():
    bad = ranks > len(pool); ranks[bad] = rrng.zipf(1.1, size=int(bad.sum()))
alpha = pool[ranks - 1].view(">u4").reshape(-1).astype(np.uint64)
w = rrng.integers(0, mx + 1, size=n_rep)
thr = max(1, int(np.ceil(0.0005 * n_rep * mx / 2)))
def nodes(cands, L):
    # tree levels 0..L for candidate prefixes (ints of L+1 bits): per level the node set
    lv = []
    for k in range(L + 1):
        path_par = set(int(c) >> (L - k + 1) for c in cands) if k > 0 else {0}
        lv.append(frozenset((p << 1) | b for p in path_par for b in (0, 1)))
    return lv
prev = []  # trees of earlier calls
cands = [0, 1]
for L in range(bits):
    t = nodes(cands, L)
    # deepest k such that some earlier call's tree (level m >= k) has identical levels 0..k
    best = -1; age = None
    for j, (m, tm) in enumerate(reversed(prev)):
        k = 0
        while k <= min(m, L) and tm[k] == t[k]: k += 1
        k -= 1
        if k > best: best, age = k, j + 1
    nn = sum(len(x) for x in t)
    print("L=%2d cands=%4d nodes_lastlevel=%4d resume_from=%2d (snapshot age %s) levels_to_eval=%d" % (
        L, len(cands), len(t[L]), best + 1, age, L - best))
    prev.append((L, t))
    pref = alpha >> (bits - 1 - L)
    cnt = np.bincount(np.searchsorted(np.array(sorted(cands), dtype=np.uint64), pref), minlength=len(cands) + 1)
    sc = sorted(cands); srt = np.array(sc, dtype=np.uint64)
    idx = np.searchsorted(srt, pref); ok = (idx < len(sc)); ok[ok] &= srt[idx[ok]] == pref[ok]
    sums = np.bincount(idx[ok], weights=w[ok], minlength=len(sc))
    surv = [c for c, s in zip(sc, sums) if s >= thr]
    cands = [(c << 1) | b for c in surv for b in (0, 1)]
print("node counts per level of each call's tree:")
for (m, tm) in prev:
    print("%2d" % m, [len(x) for x in tm])
