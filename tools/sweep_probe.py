"""Host-side timing of one c2sweep (bench.py --config c2sweep) level by level.

Wraps the Mastic calls the sweep driver makes (prep_init_device x2,
decide_results, aggregate_device x2) with wall-clock timers and prints, per
level: candidates, whether the frontier cache hit, the host time spent inside
each call, the GPU time of each prep_init (HIP events) and the level's wall
time.  GPU box only:  python3 tools/sweep_probe.py [n_reports]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "draft-mouris-cfrg-mastic_amd")]

from bench import _attrs  # noqa: E402
from mastic_amd import Mastic  # noqa: E402
from mastic_amd.heavy_hitters import compute_heavy_hitters  # noqa: E402


def main():
    n_rep = int(sys.argv[1]) if len(sys.argv) > 1 else 1000000
    if os.environ.get("PROBE_TORCH") == "1":  # the bench's process state: torch's HIP context first
        import torch
        torch.cuda.synchronize()
    bits, mx = 32, 255
    m = Mastic(bits, "Sum", device=0, max_measurement=mx)
    ctx = b"mastic-mi355x-bench"
    seed = 0x4D41 + 2
    pool = _attrs(np.random.default_rng(seed), bits, 10000)
    rrng = np.random.default_rng(seed * 1000003)
    ranks = rrng.zipf(1.1, size=n_rep)
    while (ranks > len(pool)).any():
        bad = ranks > len(pool)
        ranks[bad] = rrng.zipf(1.1, size=int(bad.sum()))
    alpha_b = pool[ranks - 1].tobytes()
    w = rrng.integers(0, mx + 1, size=n_rep)
    nb = mx.bit_length()
    off = 2 ** nb - 1 - mx
    betas = np.concatenate([(w[:, None] >> np.arange(nb)) & 1, ((w + off)[:, None] >> np.arange(nb)) & 1],
                           axis=1).astype("<u8").tobytes()
    threshold = max(1, int(np.ceil(0.0005 * n_rep * mx / 2)))
    nonces = rrng.integers(0, 256, size=16 * n_rep, dtype=np.uint8).tobytes()
    rands = rrng.integers(0, 256, size=m.RAND_SIZE * n_rep, dtype=np.uint8).tobytes()
    reps = m.reports_shard(ctx, alpha_b, betas, nonces, rands)
    vk = np.random.default_rng(0x4D41).integers(0, 256, size=16, dtype=np.uint8).tobytes()
    m.synchronize()

    rows = []
    cur = {}

    def wrap(name):
        f = getattr(m, name)

        def g(*a, **k):
            t = time.perf_counter()
            r = f(*a, **k)
            cur[name] = cur.get(name, 0.0) + time.perf_counter() - t
            if name == "prep_init_device":
                cur["cached"] = cur.get("cached", 0) + int(m.last_prep_was_cached())
            return r
        setattr(m, name, g)

    for nm in ("prep_init_device", "decide_results", "aggregate_device", "last_timing3", "select_timing"):
        wrap(nm)
    timing = []
    t_prev = [time.perf_counter()]

    class Trace(list):
        def append(self, lv):
            now = time.perf_counter()
            cur["wall"] = now - t_prev[0]
            t_prev[0] = now
            cur["level"] = lv.level
            cur["cands"] = len(lv.prefixes)
            sys.stderr.write("[probe] level %d done\n" % lv.level)
            rows.append(dict(cur))
            cur.clear()
            super().append(lv)

    tr = Trace()
    t0 = time.perf_counter()
    hh = compute_heavy_hitters(m, ctx, {"default": threshold}, reps, verify_key=vk, trace=tr, timing=timing,
                               frontier_cache=True)
    m.synchronize()
    total = time.perf_counter() - t0
    print("level cands cached  prep0+1_host  decide  agg   gpu_prep_ms(a0,a1)  wall_ms")
    for i, r in enumerate(rows):
        g = timing[2 * i:2 * i + 2]
        gp = [x[6] for x in g]  # total ms of each aggregator's prep_init (HIP events)
        print("%5d %5d %6d %12.1f %7.1f %5.1f   %8.1f %8.1f %9.1f" % (
            r["level"], r["cands"], r.get("cached", 0), 1e3 * r.get("prep_init_device", 0),
            1e3 * r.get("decide_results", 0), 1e3 * r.get("aggregate_device", 0),
            gp[0] if gp else 0, gp[1] if len(gp) > 1 else 0, 1e3 * r["wall"]))
    print("total %.2f s, %d heavy hitters, timing tuple example %s" % (total, len(hh), timing[:1]))


if __name__ == "__main__":
    main()
