"""World-size-2 gloo rehearsal of the multi-GPU exchange (CPU only): reports
are split across ranks, each rank produces its aggregate share, the shares are
all-gathered in rank order (mastic_amd.merge.gather_shares) and their GF(p)
sum equals the aggregate of the whole report set.  The field sum here is the
oracle's (the GPU fold kernel itself is covered by tests/test_gpu_merge.py)."""
import os
import random
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG_ROOT, ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, shares, out_q):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, PKG_ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mastic_amd.merge import gather_shares
    local = torch.frombuffer(bytearray(shares[rank]), dtype=torch.uint8)
    g = gather_shares(local, dist)
    out_q.put((rank, bytes(g.numpy().tobytes())))
    dist.destroy_process_group()


def test_gather_and_fold_two_ranks():
    from oracle.field import Field64
    rng = random.Random(5)
    n_elems = 37
    # report out shares split over 2 ranks; each rank's agg share = sum of its reports
    reports = [[Field64(rng.getrandbits(64)) for _ in range(n_elems)] for _ in range(6)]
    per_rank = [reports[:4], reports[4:]]
    shares = []
    for rk in per_rank:
        acc = [Field64(0)] * n_elems
        for o in rk:
            acc = [a + b for (a, b) in zip(acc, o)]
        shares.append(Field64.encode_vec(acc))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, shares, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got[0] == got[1] == shares[0] + shares[1]
    # GF(p) merge of the gathered buffer == aggregate over all reports
    g = got[0]
    k = n_elems * 8
    merged = [a + b for (a, b) in zip(Field64.decode_vec(g[:k]), Field64.decode_vec(g[k:]))]
    want = [Field64(0)] * n_elems
    for o in reports:
        want = [a + b for (a, b) in zip(want, o)]
    assert merged == want


def _sweep_worker(rank, world, port, meas, thresholds, bits, out_q):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, PKG_ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mastic_amd.heavy_hitters import compute_heavy_hitters
    from test_sweep import _StubMastic, _StubReports

    def merge(agg_share):  # the stub's shares are plaintext ints: all-gather + sum
        parts = [None] * world
        dist.all_gather_object(parts, list(agg_share))
        return [sum(col) for col in zip(*parts)] if agg_share else agg_share

    mine = meas[rank::world]
    hh = compute_heavy_hitters(_StubMastic(bits), b"ctx", thresholds, _StubReports(mine), bytes(32), merge=merge)
    out_q.put((rank, hh))
    dist.destroy_process_group()


def test_sweep_over_two_ranks_matches_whole_batch():
    """C3 shape: reports sharded over 2 ranks, each level's
    agg shares merged across ranks before pruning, so both ranks walk the
    same frontier and return the heavy hitters of the whole report set."""
    from test_sweep import index, plain_heavy_hitters
    rng = random.Random(11)
    bits = 10
    pool = [index(rng.getrandbits(bits), bits) for _ in range(12)]
    meas = [(pool[min(int(rng.paretovariate(1.1)) - 1, len(pool) - 1)], 1) for _ in range(300)]
    thresholds = {"default": 15}
    want = plain_heavy_hitters(meas, thresholds, bits)
    assert want  # the workload has heavy hitters
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sweep_worker, args=(r, 2, port, meas, thresholds, bits, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got[0] == got[1] == want
