"""Probe (GPU box, under rocprofv3 --kernel-trace): one cache-off prep_init of
the north_star sweep's level-L miss (its plaintext candidate list) over a
chunk-sized batch, to time the top tree levels' launches (1-2 parents per
report) by themselves.  Knobs via the experiment build (bench.py --lib style):
  python3 tools/tiny_level_probe.py <lib.so or ''> <L> <reports>
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "draft-mouris-cfrg-mastic_amd"))
import torch  # noqa: E402,F401  (one HIP runtime, see tests/conftest.py)
import bench  # noqa: E402

lib, L, n = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
if lib:
    from mastic_amd import _lib
    _lib.load(lib)
from mastic_amd import Mastic  # noqa: E402

cfg = bench.CONFIGS["c2sweep"]
kw = dict(cfg["kw"])
bits = kw.pop("bits")
seed = 0x4D41 + 2
N = 1000000
alphas, w, betas, nonces, rrng = bench.sweep_population(cfg, bits, kw, seed, N, seed * 1000003)
thr = bench.sweep_threshold(cfg, kw, N)
vals = np.zeros(N, dtype=np.uint64)
for j in range(4):
    vals = (vals << np.uint64(8)) | alphas[:, j].astype(np.uint64)
cands = [0, 1]
for lev in range(L):
    pre = vals >> np.uint64(31 - lev)
    cs = np.array(sorted(cands), dtype=np.uint64)
    idx = np.minimum(np.searchsorted(cs, pre), len(cs) - 1)
    hit = cs[idx] == pre
    ws = np.bincount(idx[hit], weights=w[hit], minlength=len(cs))
    cands = [(int(c) << 1) | b for (c, x) in zip(cs, ws) if x >= thr for b in (0, 1)]
prefixes = tuple(tuple(bool((c >> (L - i)) & 1) for i in range(L + 1)) for c in sorted(cands))
m = Mastic(bits, "Sum", **kw)
rands = rrng.integers(0, 256, size=m.RAND_SIZE * n, dtype=np.uint8).tobytes()
ctx = b"mastic-mi355x-bench"
reps = m.reports_shard(ctx, alphas[:n].tobytes(), betas[:n].tobytes(), nonces[:16 * n].tobytes(), rands)
vk = bytes(16)
ap = m.encode_agg_param((L, prefixes, L == 0))
for i in range(3):
    m.prep_init_device(reps, vk, ctx, 0, ap)
    m.synchronize()
    print("rep %d" % i, m.last_timing3(), flush=True)
