"""N ranks on one GPU (gloo process group, each rank its own Mastic context
on cuda:0 with its own HBM budget): the multi-rank sweep (SweepMerge: both
aggregators' agg shares folded in HBM, all-gathered, merged mod p on the GPU)
and the C2 bench step's merge (merge_agg_shares) over a report set split N
ways give exactly the single-rank results over the whole set (SURVEY.md §8e;
examples.py:37-91).  Cases: two ranks; four ranks over a job not divisible by
four; four ranks over three reports, so rank 0 holds none
(SweepMerge.total(have_results=False) and an empty prep_init / fold).  Only
the transport differs from the driver's 8-GPU run: gloo gathers host copies
where RCCL gathers over xGMI (tests/test_gpu_merge.py covers RCCL at one
rank)."""
import os
import random
import socket

import pytest

from conftest import PKG_ROOT, ROOT

pytestmark = pytest.mark.gpu

BITS, SEED = 10, 77
# (ranks, reports, threshold): even split; uneven split; a rank with no reports
CASES = [(2, 600, 12), (4, 601, 12), (4, 3, 1)]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _population(N):
    rng = random.Random(SEED)
    pool = [tuple(bool(rng.getrandbits(1)) for _ in range(BITS)) for _ in range(12)]
    alphas = [pool[min(int(rng.paretovariate(1.0)) - 1, len(pool) - 1)] for _ in range(N)]
    weights = [int(rng.random() < 0.9) for _ in range(N)]
    return (alphas, weights, rng.randbytes(16 * N), rng.randbytes(16 * N), rng.randbytes(32), pool)


def _reports(m, ctx, N, lo, hi):
    (alphas, weights, nonces, rands, _vk, _pool) = _population(N)
    rs = m.RAND_SIZE
    # rands for RAND_SIZE bytes per report, derived from the population stream
    rand_all = (rands * ((rs * N) // len(rands) + 1))[:rs * N]
    nc = nonces[16 * lo:16 * hi]
    (pub, in0, in1) = m.shard_batch(ctx, alphas[lo:hi], weights[lo:hi], nc, rand_all[rs * lo:rs * hi])
    return m.reports_upload(nc, pub, in0, in1)


def _agg_param(pool):
    return (BITS - 1, tuple(sorted(set(pool[:6]))), True)


def _worker(rank, world, port, N, thresh, q):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, PKG_ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import mastic_amd
        from mastic_amd.heavy_hitters import compute_heavy_hitters
        from mastic_amd.merge import SweepMerge, aggregate_to_tensor, merge_agg_shares
        m = mastic_amd.MasticCount(BITS)
        m.set_memory_budget(2 << 30)  # the ranks share one GPU
        ctx = b"two-ranks"
        lo, hi = N * rank // world, N * (rank + 1) // world
        dev = _reports(m, ctx, N, lo, hi)
        (_a, _w, _n, _r, vk, pool) = _population(N)
        trace = []
        hh = compute_heavy_hitters(m, ctx, {"default": thresh}, dev, verify_key=vk, trace=trace,
                                   merge=SweepMerge(m, dist))
        # the C2 bench step: one agg param, this rank's agg share folded in HBM, gathered, merged
        ap = _agg_param(pool)
        enc = m.encode_agg_param(ap)
        m.prep_init_device(dev, vk, ctx, 0, enc)
        n_elems = len(ap[1]) * (1 + m.OUTPUT_LEN)
        merged = merge_agg_shares(m, aggregate_to_tensor(m, 0, n_elems), dist).cpu().numpy().tobytes()
        q.put((rank, hi - lo, hh, [(t.level, t.prefixes, t.agg_result) for t in trace], merged))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,N,thresh", CASES, ids=["2x600", "4x601", "4x3-empty-rank"])
def test_ranks_on_one_gpu_match_single_rank(world, N, thresh):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import torch.multiprocessing as mp
    ctx_mp = mp.get_context("spawn")
    q = ctx_mp.Queue()
    port = _free_port()
    procs = [ctx_mp.Process(target=_worker, args=(r, world, port, N, thresh, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict((r, rest) for (r, *rest) in (q.get(timeout=240) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert sum(got[r][0] for r in range(world)) == N
    if N < world:
        assert got[0][0] == 0, "the case must give rank 0 no reports"
    # single rank over all reports
    import mastic_amd
    from mastic_amd.heavy_hitters import compute_heavy_hitters
    m = mastic_amd.MasticCount(BITS)
    ctx = b"two-ranks"
    dev = _reports(m, ctx, N, 0, N)
    (alphas, weights, _n, _r, vk, pool) = _population(N)
    trace = []
    hh = compute_heavy_hitters(m, ctx, {"default": thresh}, dev, verify_key=vk, trace=trace)
    want_trace = [(t.level, t.prefixes, t.agg_result) for t in trace]
    ap = _agg_param(pool)
    enc = m.encode_agg_param(ap)
    m.prep_init_device(dev, vk, ctx, 0, enc)
    want_agg = m.aggregate_device(0, enc, raw=True)
    # the heavy hitters are the plaintext ones (talks/func.py:49-80 semantics)
    tot = {}
    for (a, w) in zip(alphas, weights):
        tot[a] = tot.get(a, 0) + w
    assert sorted(hh) == sorted(a for (a, w) in tot.items() if w >= thresh)
    for r in range(world):
        (_n_r, hh_r, trace_r, merged_r) = got[r]
        assert hh_r == hh
        assert trace_r == want_trace
        assert merged_r == want_agg
