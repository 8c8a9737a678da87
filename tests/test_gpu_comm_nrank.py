"""The library's N-rank collective path on one GPU: N processes, each with its
own Mastic contexts on cuda:0, form communicators through the MASTIC_RCCL_LIB
test hook bound to tests/host/fake_rccl.cpp (a shared-memory stand-in for the
eight RCCL calls the library makes; RCCL itself refuses two ranks on one
device).  So everything above the transport -- mastic_comm_init's threaded
init, the agreement round, the data all-gather on the ctx's stream, the GF(p)
fold of every rank's shares, the bounded waits and the abort -- runs at N = 2
and 3 exactly as on the driver's multi-GPU node (include/mastic_hip.h, failure
model):

* merge_host / allgather_fold in Field64 and Field128 = the field sum of every
  rank's shares (Mastic.merge, poc/mastic.py:390-397);
* the heavy-hitters sweep over a report set split N ways, merged per level by
  CommMerge (mastic_aggregate_merged), and one aggregate_merged step = the
  single-rank results over all reports (examples.py:37-91);
* calls that disagree on the share geometry: EINVAL on every rank;
* an injected ENOMEM on rank 1's staging buffer: every rank returns ENOMEM,
  no shares move, and the repeated call merges correctly on all;
* a rank that skips a call: its peers return ETIMEDOUT after the bound and
  then EHIP (communicator aborted, no world-1 fallback); the late rank times
  out too; every process exits normally."""
import os
import random

import pytest

from conftest import PKG_ROOT, ROOT

pytestmark = pytest.mark.gpu

BITS, SEED, TIMEOUT_MS = 10, 91, 4000
# (ranks, reports, threshold); the last: rank 0 holds no reports (CommMerge.total(have_results=False))
CASES = [(2, 600, 12), (3, 601, 12), (3, 450, 9), (3, 2, 1)]


def _fake_rccl():
    sys_path = os.path.join(ROOT, "tests", "host", "_build", "libfake_rccl.so")
    if not os.path.exists(sys_path):
        pytest.fail("tests/host/_build/libfake_rccl.so is missing: run __graft_entry__.build() first")
    return sys_path


def _population(N):
    rng = random.Random(SEED)
    pool = [tuple(bool(rng.getrandbits(1)) for _ in range(BITS)) for _ in range(12)]
    alphas = [pool[min(int(rng.paretovariate(1.0)) - 1, len(pool) - 1)] for _ in range(N)]
    weights = [int(rng.random() < 0.9) for _ in range(N)]
    return (alphas, weights, rng.randbytes(16 * N), rng.randbytes(16 * N), rng.randbytes(32), pool)


def _reports(m, ctx, N, lo, hi):
    (alphas, weights, nonces, rands, _vk, _pool) = _population(N)
    rs = m.RAND_SIZE
    rand_all = (rands * ((rs * N) // len(rands) + 1))[:rs * N]
    nc = nonces[16 * lo:16 * hi]
    (pub, in0, in1) = m.shard_batch(ctx, alphas[lo:hi], weights[lo:hi], nc, rand_all[rs * lo:rs * hi])
    return m.reports_upload(nc, pub, in0, in1)


def _agg_param(pool):
    return (BITS - 1, tuple(sorted(set(pool[:6]))), True)


def _shares(F, seed, n_local, n_elems):
    rng = random.Random(seed)
    return [[F(rng.randrange(F.MODULUS)) for _ in range(n_elems)] for _ in range(n_local)]


def _code(fn):
    """The library's return code of a call (0 = success)."""
    from mastic_amd._lib import MasticError
    try:
        fn()
        return 0
    except ValueError:
        return -22
    except MasticError as e:
        return e.code


def _worker(rank, world, N, thresh, fake, idq, q):
    import faulthandler
    import sys
    import time
    # a hang shows up as every thread's stack on stderr, then the rank exits
    faulthandler.dump_traceback_later(70, exit=True)

    def say(msg):
        print("[rank %d %.1f s] %s" % (rank, time.time() - t_start, msg), file=sys.stderr, flush=True)
    t_start = time.time()
    sys.path.insert(0, ROOT)
    sys.path.insert(0, PKG_ROOT)
    os.environ["MASTIC_RCCL_LIB"] = fake  # read on the library's first communicator call
    if world >= 3:
        # Three processes on one GPU with HIP's default 4 hardware queues each
        # (plus the library's high-priority sponge streams): in 5 of 8 runs one
        # rank's stream stalled after a cross-stream event wait, right after its
        # status all-gather (its peers then timed out and aborted, as designed),
        # and 2 of 3 with SDMA copies off (HSA_ENABLE_SDMA=0); with one hardware
        # queue per process 9 of 9 runs passed.  Deployment is one process per
        # GPU; the rehearsal gives each rank one queue.
        os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("NRANK_HW_QUEUES", "1")  # (override: experiments)
    import torch
    torch.cuda.set_device(0)
    say("torch up")
    import mastic_amd
    from mastic_amd.heavy_hitters import compute_heavy_hitters
    from mastic_amd.merge import CommMerge
    from oracle.field import Field64, Field128
    out = {}
    m = mastic_amd.MasticCount(BITS)
    m.set_memory_budget(2 << 30)  # the ranks share one GPU
    mh = mastic_amd.Mastic(5, "Histogram", length=3, chunk_length=2)
    mh.set_memory_budget(1 << 30)
    if rank == 0:
        ids = [mastic_amd.Mastic.comm_unique_id() for _ in range(2)]
        for _ in range(world - 1):
            idq.put(ids)
    else:
        ids = idq.get(timeout=120)
    say("ids")
    m.comm_init(world, rank, ids[0], timeout_ms=TIMEOUT_MS)
    mh.comm_init(world, rank, ids[1], timeout_ms=TIMEOUT_MS)
    out["info"] = (m.comm_info(), mh.comm_info())
    say("communicators up")

    # 1. host and device share merges, both fields (the two communicators interleave)
    side = torch.cuda.Stream() if rank % 2 else None  # the caller's stream: torch's default or a side stream
    stream = (side or torch.cuda.current_stream()).cuda_stream
    for (name, mm, F) in (("f64", m, Field64), ("f128", mh, Field128)):
        n_el = 37
        raw = b"".join(F.encode_vec(s) for s in _shares(F, 1000 * rank + len(name), 2, n_el))
        out[name + "_host"] = mm.merge_host(raw, 2, n_el)
        with torch.cuda.stream(side or torch.cuda.current_stream()):
            dev = torch.frombuffer(bytearray(raw), dtype=torch.uint8).cuda()
            res = torch.empty(n_el * F.ENCODED_SIZE, dtype=torch.uint8, device="cuda")
        mm.allgather_fold(dev.data_ptr(), 2, n_el, res.data_ptr(), stream)
        out[name + "_agf"] = res.cpu().numpy().tobytes()
        say(name + " merges done")

    # 2. the split sweep (CommMerge per level) and one aggregate_merged step
    ctx = b"n-ranks"
    lo, hi = N * rank // world, N * (rank + 1) // world
    reps = _reports(m, ctx, N, lo, hi) if hi > lo else []  # a rank without reports
    (_a, _w, _n, _r, vk, pool) = _population(N)
    trace = []
    out["hh"] = compute_heavy_hitters(m, ctx, {"default": thresh}, reps, verify_key=vk, trace=trace,
                                      merge=CommMerge(m))
    out["trace"] = [(t.level, t.prefixes, t.agg_result) for t in trace]
    ap = _agg_param(pool)
    n_ap = len(ap[1]) * (1 + m.OUTPUT_LEN)
    if hi > lo:
        m.prep_init_device(reps, vk, ctx, 0, m.encode_agg_param(ap))
        out["agg"] = m.aggregate_merged((0,), n_ap)
    else:
        out["agg"] = m.aggregate_merged((0,), n_ap, zeros=True)  # agg_init's zeros, same collective
    out["n_reports"] = hi - lo
    say("sweep and step done")

    # 3. calls that disagree on the geometry
    n_bad = 5 + (rank == world - 1)
    out["mismatch"] = _code(lambda: m.merge_host(bytes(8 * n_bad), 1, n_bad))

    # 4. an injected ENOMEM on rank 1's staging buffer, then the same call again
    n_big = 100000
    big = Field64.encode_vec(_shares(Field64, 7000 + rank, 1, n_big)[0])
    if rank == 1:
        m.set_test_hooks(fail_allocs=1)
    out["enomem"] = _code(lambda: m.merge_host(big, 1, n_big))
    if rank == 1:
        out["enomem_hook_used"] = m.set_test_hooks(fail_allocs=0) == 0
    out["big"] = m.merge_host(big, 1, n_big)
    say("agreed failures done")

    # 5. the last rank skips a call: its peers time out, then see the abort
    mh.comm_destroy()
    t0 = time.time()
    if rank == world - 1:
        time.sleep(1.5 * TIMEOUT_MS / 1000)
        out["late"] = _code(lambda: m.merge_host(bytes(8), 1, 1))
    else:
        out["timeout"] = _code(lambda: m.merge_host(bytes(8), 1, 1))
        out["timeout_s"] = time.time() - t0
        out["after_abort"] = _code(lambda: m.merge_host(bytes(8), 1, 1))
    m.comm_destroy()
    out["info_end"] = m.comm_info()
    say("done")
    q.put((rank, out))


@pytest.mark.parametrize("world,N,thresh", CASES, ids=["2x600", "3x601", "3x450", "3x2-empty-rank"])
def test_n_ranks_on_one_gpu_through_the_library_comm(world, N, thresh):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    fake = _fake_rccl()
    import torch.multiprocessing as mp
    ctx_mp = mp.get_context("spawn")
    (idq, q) = (ctx_mp.Queue(), ctx_mp.Queue())
    procs = [ctx_mp.Process(target=_worker, args=(r, world, N, thresh, fake, idq, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        got = dict(q.get(timeout=100) for _ in range(world))
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.exitcode is None:
                p.kill()
    assert [p.exitcode for p in procs] == [0] * world

    from oracle.field import Field64, Field128
    for r in range(world):
        assert got[r]["info"] == ((world, r), (world, r))
    # 1. merges = the field sum of every rank's shares
    for (name, F) in (("f64", Field64), ("f128", Field128)):
        want = [F(0)] * 37
        for r in range(world):
            for s in _shares(F, 1000 * r + len(name), 2, 37):
                want = [a + b for (a, b) in zip(want, s)]
        for r in range(world):
            assert got[r][name + "_host"] == F.encode_vec(want), (name, r)
            assert got[r][name + "_agf"] == F.encode_vec(want), (name, r)
    # 2. the split sweep and step = the single-rank run over all reports
    import mastic_amd
    from mastic_amd.heavy_hitters import compute_heavy_hitters
    m = mastic_amd.MasticCount(BITS)
    ctx = b"n-ranks"
    reps = _reports(m, ctx, N, 0, N)
    (alphas, weights, _n, _r, vk, pool) = _population(N)
    trace = []
    hh = compute_heavy_hitters(m, ctx, {"default": thresh}, reps, verify_key=vk, trace=trace)
    tot = {}
    for (a, w) in zip(alphas, weights):
        tot[a] = tot.get(a, 0) + w
    assert sorted(hh) == sorted(a for (a, w) in tot.items() if w >= thresh) and hh
    ap = _agg_param(pool)
    enc = m.encode_agg_param(ap)
    m.prep_init_device(reps, vk, ctx, 0, enc)
    want_agg = m.aggregate_device(0, enc, raw=True)
    assert sum(got[r]["n_reports"] for r in range(world)) == N
    if N < world:
        assert got[0]["n_reports"] == 0, "the case must give rank 0 no reports"
    for r in range(world):
        assert got[r]["hh"] == hh
        assert got[r]["trace"] == [(t.level, t.prefixes, t.agg_result) for t in trace]
        assert got[r]["agg"] == want_agg
    # 3. / 4. agreed failures, then a correct merge
    want_big = [Field64(0)] * 100000
    for r in range(world):
        want_big = [a + b for (a, b) in zip(want_big, _shares(Field64, 7000 + r, 1, 100000)[0])]
    for r in range(world):
        assert got[r]["mismatch"] == -22, r
        assert got[r]["enomem"] == -12, r
        assert got[r]["big"] == Field64.encode_vec(want_big), r
    assert got[1]["enomem_hook_used"]
    # 5. a rank that never joins: ETIMEDOUT after the bound, then EHIP (aborted)
    for r in range(world - 1):
        assert got[r]["timeout"] == -110, r
        assert TIMEOUT_MS / 1000 * 0.9 <= got[r]["timeout_s"] < TIMEOUT_MS / 1000 + 20, got[r]["timeout_s"]
        assert got[r]["after_abort"] == -5, r
    assert got[world - 1]["late"] == -110
    for r in range(world):
        assert got[r]["info_end"] == (1, 0)
