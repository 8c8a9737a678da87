"""Strong-scaling split of the north_star job (bench.py --split, the
north_star leg of the default bench) on CPU: the job's reports are divided
over the ranks, every rank sees the same job-wide per-level aggregates (merged
over gloo here, RCCL + GPU fold on the box), and all ranks return the heavy
hitters of the whole job, equal to the single-rank sweep and to the plaintext.
The aggregator is a numpy stand-in returning plaintext per-candidate sums
(bench.prefix_sums); the GPU run of the same driver is test_gpu_sweep.py."""
import os
import socket

import numpy as np
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG_ROOT, ROOT  # noqa: F401

N_JOB = 20000


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _job():
    import sys
    sys.path.insert(0, ROOT)
    import bench
    cfg = bench.CONFIGS["c2sweep"]
    kw = dict(cfg["kw"])
    bits = kw.pop("bits")
    seed = 0x4D41 + 2
    (alphas, w, _betas, _nonces, _rrng) = bench.sweep_population(cfg, bits, kw, seed, N_JOB, seed * 1000003)
    return bench, cfg, kw, bits, alphas, w


class _Reports:
    def __init__(self, alphas, w):
        self.alphas, self.w, self.n = alphas, w, len(w)


class _NumpyStub:
    """Stands in for mastic_amd.Mastic on CPU: aggregator 0's 'share' is the
    plaintext weight sum per candidate, aggregator 1's is zero."""
    VERIFY_KEY_SIZE = 32
    OUTPUT_LEN = 0
    JOINT_RAND_LEN = 0

    def __init__(self, bits, prefix_sums):
        class V:
            BITS = bits
        self.vidpf = V()
        self.prefix_sums = prefix_sums

    def is_valid(self, agg_param, prev):
        return True

    def encode_agg_param(self, agg_param):
        return agg_param

    def prep_init_device(self, dev, vk, ctx, agg_id, agg_param):
        self._dev = dev

    def prep_result(self, dev, agg_id, agg_param):
        return (agg_id, None, None, np.zeros(dev.n, np.int32))

    def decide_batch(self, ctx, agg_param, ps0, ps1):
        return (b"", np.ones(self._dev.n, np.uint8))

    def aggregate_device(self, agg_id, agg_param, mask):
        if agg_id == 1 or not agg_param[1]:
            return [0] * len(agg_param[1])
        (_cnt, ws) = self.prefix_sums(self._dev.alphas, self._dev.w, agg_param[0], agg_param[1])
        return ws.tolist()

    def agg_init(self, agg_param):
        return [0] * len(agg_param[1])

    def unshard(self, agg_param, agg_shares, n):
        return [a + b for (a, b) in zip(*agg_shares)]


def _worker(rank, world, port, out_q):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, PKG_ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mastic_amd.heavy_hitters import compute_heavy_hitters
    (bench, cfg, kw, bits, alphas, w) = _job()
    (lo, hi) = bench.split_bounds(N_JOB, world)[rank]

    def merge(agg_share):  # plaintext ints: all-gather + sum (the GPU path: RCCL + GF(p) fold)
        parts = [None] * world
        dist.all_gather_object(parts, list(agg_share))
        return [sum(col) for col in zip(*parts)] if agg_share else agg_share

    hh = compute_heavy_hitters(_NumpyStub(bits, bench.prefix_sums), b"ctx",
                               {"default": bench.sweep_threshold(cfg, kw, N_JOB)},
                               _Reports(alphas[lo:hi], w[lo:hi]), bytes(32), merge=merge)
    out_q.put((rank, hi - lo, hh))
    dist.destroy_process_group()


def test_split_bounds_cover_the_job():
    import sys
    sys.path.insert(0, ROOT)
    import bench
    for (n, k) in [(1000000, 1), (1000000, 2), (1000000, 8), (1000001, 8), (7, 3)]:
        b = bench.split_bounds(n, k)
        assert b[0][0] == 0 and b[-1][1] == n
        assert all(b[i][1] == b[i + 1][0] for i in range(k - 1))
        sizes = [hi - lo for (lo, hi) in b]
        assert max(sizes) - min(sizes) <= 1
    assert bench.split_bounds(1000000, 8)[0] == (0, 125000)


def test_prefix_sums_match_plaintext():
    (bench, _cfg, _kw, _bits, alphas, w) = _job()
    a, ww = alphas[:3000], w[:3000]
    for level in (0, 5, 17, 31):
        pfx = sorted(set(tuple(bool((int.from_bytes(bytes(r), "big") >> (31 - i)) & 1) for i in range(level + 1))
                         for r in a[:40]))
        (cnt, ws) = bench.prefix_sums(a, ww, level, pfx)
        ints = [int.from_bytes(bytes(r), "big") >> (31 - level) for r in a]
        for (j, p) in enumerate(pfx):
            v = int("".join("1" if b else "0" for b in p), 2)
            assert cnt[j] == sum(1 for x in ints if x == v)
            assert ws[j] == sum(int(x2) for (x, x2) in zip(ints, ww) if x == v)


def test_split_over_two_ranks_same_heavy_hitters():
    """--gpus 2 --split: each rank sweeps half of the job's reports, the
    thresholds come from the job total, and both ranks return the heavy
    hitters of the whole job (equal to one rank sweeping all of it, and to the
    plaintext rule: every attribute whose total weight reaches the threshold)."""
    from mastic_amd.heavy_hitters import compute_heavy_hitters
    (bench, cfg, kw, bits, alphas, w) = _job()
    th = bench.sweep_threshold(cfg, kw, N_JOB)
    whole = compute_heavy_hitters(_NumpyStub(bits, bench.prefix_sums), b"ctx", {"default": th},
                                  _Reports(alphas, w), bytes(32))
    keys, inv = np.unique(alphas, axis=0, return_inverse=True)
    tot = np.bincount(inv.ravel(), weights=w)
    want = sorted(bytes(k) for (k, t) in zip(keys, tot) if t >= th)
    assert sorted(np.packbits(np.array(p, dtype=bool)).tobytes() for p in whole) == want and len(want) > 20
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(2):
        (rank, n, hh) = q.get(timeout=300)
        got[rank] = (n, hh)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got[0][0] == got[1][0] == N_JOB // 2
    assert got[0][1] == got[1][1] == whole
