"""The multi-GPU merge path on one GPU (Mastic.merge,
poc/mastic.py:390-397): the on-GPU GF(p) fold of gathered agg shares
(``mastic_fold_shares``) against the oracle's field sum with elements that
wrap mod p, the device-resident agg share (``mastic_aggregate_device``),
report-batch views, and the sweep's device merge over a 1-rank RCCL group."""
import random
import socket

import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _share_bytes(field, rng, n, near_p):
    vals = []
    for _ in range(n):
        if near_p and rng.random() < 0.7:
            vals.append(field(field.MODULUS - 1 - rng.randrange(16)))
        else:
            vals.append(field(rng.randrange(field.MODULUS)))
    return vals


@pytest.mark.parametrize("circuit,kw", [("Count", dict(bits=4)),
                                        ("Histogram", dict(bits=4, length=3, chunk_length=2))],
                         ids=["Field64", "Field128"])
@pytest.mark.parametrize("n_shares", [1, 3, 8])
def test_fold_shares_matches_field_sum(torch_cuda, circuit, kw, n_shares):
    torch = torch_cuda
    import mastic_amd
    from mastic_amd.merge import fold_on_gpu
    from oracle.field import Field64, Field128
    kw = dict(kw)
    bits = kw.pop("bits")
    m = mastic_amd.Mastic(bits, circuit, **kw)
    F = Field64 if m.field.ENCODED_SIZE == 8 else Field128
    rng = random.Random(n_shares * 31 + m.field.ENCODED_SIZE)
    n_elems = 300  # > one 256-thread workgroup
    shares = [_share_bytes(F, rng, n_elems, near_p=True) for _ in range(n_shares)]
    raw = b"".join(F.encode_vec(s) for s in shares)
    dev = torch.frombuffer(bytearray(raw), dtype=torch.uint8).cuda()
    merged = fold_on_gpu(m, dev, n_shares, n_elems).cpu().numpy().tobytes()
    want = [F(0)] * n_elems
    for s in shares:
        want = [a + b for (a, b) in zip(want, s)]
    assert merged == F.encode_vec(want)
    # the sums wrapped: some raw integer sums exceed p
    if n_shares > 1:
        assert any(sum(s[e].int() for s in shares) >= F.MODULUS for e in range(n_elems))


def _shard(m, rng, n, ctx):
    alphas = [tuple(bool(rng.getrandbits(1)) for _ in range(m.BITS)) for _ in range(n)]
    weights = [rng.randrange(m.max_measurement + 1) if m.circuit == "Sum" else rng.randrange(2) for _ in range(n)]
    nonces = bytes(rng.getrandbits(8) for _ in range(16 * n))
    rands = bytes(rng.getrandbits(8) for _ in range(m.RAND_SIZE * n))
    return alphas, weights, nonces, rands


def test_aggregate_device_and_views(torch_cuda):
    """Agg share folded into a device buffer equals the host-returned one; a
    view of a resident batch gives the same prep shares as the same reports
    uploaded on their own; slice agg shares merged on the GPU equal the whole
    batch's agg share."""
    torch = torch_cuda
    import mastic_amd
    from mastic_amd.merge import aggregate_to_tensor, fold_on_gpu
    rng = random.Random(3)
    m = mastic_amd.MasticSum(6, 9)
    ctx = b"merge"
    (alphas, weights, nonces, rands) = _shard(m, rng, 150, ctx)
    (pub, in0, in1) = m.shard_batch(ctx, alphas, weights, nonces, rands)
    allr = m.reports_upload(nonces, pub, in0, in1)
    cand = tuple(sorted(set(a for a in alphas[:40])))
    ap = (5, cand, True)
    enc = m.encode_agg_param(ap)
    vk = bytes(16)
    n_elems = len(cand) * (1 + m.OUTPUT_LEN)
    m.prep_init_device(allr, vk, ctx, 0, enc)
    whole = m.aggregate_device(0, enc, raw=True)
    dev = aggregate_to_tensor(m, 0, n_elems)
    assert dev.cpu().numpy().tobytes() == whole
    # views: reports 50..149 in slices of 50
    ps_sz, is_sz = m.public_share_size(), m.input_share_size(0)
    parts = []
    for first in (0, 50, 100):
        v = allr.view(first, 50)
        m.prep_init_device(v, vk, ctx, 0, enc)
        (ps_v, _js, _o, st) = m.prep_result(v, 0, enc)
        assert list(st) == [0] * 50
        (ps_u, _js2, _o2, _st2) = m.prep_init_batch(vk, ctx, 0, enc, nonces[16 * first:16 * (first + 50)],
                                                    pub[ps_sz * first:ps_sz * (first + 50)],
                                                    in0[is_sz * first:is_sz * (first + 50)])
        assert ps_v == ps_u
        m.prep_init_device(v, vk, ctx, 0, enc)
        parts.append(aggregate_to_tensor(m, 0, n_elems))
    merged = fold_on_gpu(m, torch.cat(parts), 3, n_elems)
    assert merged.cpu().numpy().tobytes() == whole
    with pytest.raises(ValueError):
        allr.view(100, 51)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_sweep_device_merge_one_rank_rccl(torch_cuda):
    """compute_heavy_hitters with the device merge (both agg shares folded in
    HBM, one RCCL all-gather per level, GF(p) fold of 2 x world shares) over a
    1-rank RCCL group gives the same trace as the single-rank host unshard."""
    torch = torch_cuda
    import os
    import torch.distributed as dist
    import mastic_amd
    from mastic_amd.heavy_hitters import compute_heavy_hitters
    from mastic_amd.merge import SweepMerge
    rng = random.Random(4)
    m = mastic_amd.MasticCount(8)
    ctx = b"rccl"
    pool = [tuple(bool(rng.getrandbits(1)) for _ in range(8)) for _ in range(5)]
    n = 200
    meas = [(pool[min(int(rng.paretovariate(1.0)) - 1, 4)], rng.randrange(2)) for _ in range(n)]
    (alphas, weights) = zip(*meas)
    nonces = rng.randbytes(16 * n)
    rands = rng.randbytes(m.RAND_SIZE * n)
    (pub, in0, in1) = m.shard_batch(ctx, list(alphas), list(weights), nonces, rands)
    dev = m.reports_upload(nonces, pub, in0, in1)
    vk = rng.randbytes(16)
    t_host = []
    hh_host = compute_heavy_hitters(m, ctx, {"default": 10}, dev, verify_key=vk, trace=t_host)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        t_dev = []
        hh_dev = compute_heavy_hitters(m, ctx, {"default": 10}, dev, verify_key=vk, trace=t_dev,
                                       merge=SweepMerge(m, dist))
    finally:
        dist.destroy_process_group()
    assert hh_dev == hh_host and hh_host
    assert [(t.level, t.prefixes, t.agg_result) for t in t_dev] == [(t.level, t.prefixes, t.agg_result)
                                                                     for t in t_host]


def test_decide_results_on_device_matches_host_decide(torch_cuda):
    """mastic_decide_results (both aggregators' results decided in HBM) gives
    the same codes as decide_batch on the downloaded prep shares, and its
    accept mask folds in the query status and the joint-rand confirmation
    (a corrupted peer joint-rand part is rejected)."""
    import mastic_amd
    from mastic_amd.heavy_hitters import joint_rand_confirmed
    rng = random.Random(6)
    m = mastic_amd.MasticHistogram(5, 6, 2)
    ctx = b"decide"
    n = 70
    alphas = [tuple(bool(rng.getrandbits(1)) for _ in range(5)) for _ in range(n)]
    weights = [rng.randrange(6) for _ in range(n)]
    nonces = rng.randbytes(16 * n)
    rands = rng.randbytes(m.RAND_SIZE * n)
    (pub, in0, in1) = m.shard_batch(ctx, alphas, weights, nonces, rands)
    isz = m.input_share_size(0)
    in0 = bytearray(in0)
    in0[isz * 3 + isz - 1] ^= 0x01  # report 3: leader's peer joint-rand part
    dev = m.reports_upload(nonces, pub, bytes(in0), in1)
    vk = rng.randbytes(16)
    for ap in [(0, ((False,), (True,)), True), (4, tuple(sorted(set(alphas)))[:9], False)]:
        enc = m.encode_agg_param(ap)
        for a in range(2):
            m.prep_init_device(dev, vk, ctx, a, enc)
        (acc, codes) = m.decide_results(ctx, n)
        sh = [m.prep_result(dev, a, enc) for a in range(2)]
        (msgs, valid) = m.decide_batch(ctx, enc, sh[0][0], sh[1][0])
        assert list(codes) == list(valid)
        want = (valid == 1) & (sh[0][3] == 0) & (sh[1][3] == 0)
        if ap[2]:
            want &= joint_rand_confirmed(msgs, sh[0][1], sh[1][1], n)
            assert not want[3]
        assert list(acc == 1) == list(want)


def test_aggregate_device_waits_for_callers_stream(torch_cuda):
    """mastic_aggregate_device writes a buffer that the caller prepared on its
    own stream: queue a long busy kernel and then a fill of the buffer on
    torch's current stream, fold into it, and the fold must land after the
    fill (the library orders itself after that stream by an event)."""
    torch = torch_cuda
    import mastic_amd
    from mastic_amd.merge import aggregate_to_tensor
    rng = random.Random(8)
    m = mastic_amd.MasticSum(6, 9)
    ctx = b"order"
    (alphas, weights, nonces, rands) = _shard(m, rng, 130, ctx)
    (pub, in0, in1) = m.shard_batch(ctx, alphas, weights, nonces, rands)
    reps = m.reports_upload(nonces, pub, in0, in1)
    cand = tuple(sorted(set(alphas[:30])))
    enc = m.encode_agg_param((5, cand, True))
    n_elems = len(cand) * (1 + m.OUTPUT_LEN)
    m.prep_init_device(reps, bytes(16), ctx, 0, enc)
    want = m.aggregate_device(0, enc, raw=True)
    for _ in range(3):
        out = torch.empty(n_elems * m.field.ENCODED_SIZE, dtype=torch.uint8, device="cuda")
        torch.cuda._sleep(50_000_000)  # ~20 ms of busy work ahead of the fill on torch's stream
        out.fill_(0xA5)
        aggregate_to_tensor(m, 0, n_elems, out=out)
        assert out.cpu().numpy().tobytes() == want


@pytest.mark.parametrize("circuit,kw,n", [("Count", dict(bits=8), 20000),
                                          ("Histogram", dict(bits=6, length=3, chunk_length=2), 9000)],
                         ids=["Field64", "Field128"])
def test_aggregate_split_fold_matches_field_sum(torch_cuda, circuit, kw, n):
    """agg_update over many reports and few output elements (a sweep level)
    runs as a report-chunked fold plus a mod-p merge of the chunk partials
    (aggregate_impl); it equals the field sum of the out shares of the valid
    reports (mastic.py:384-388), with and without a validity mask."""
    import numpy as np
    import mastic_amd
    kw = dict(kw)
    bits = kw.pop("bits")
    m = mastic_amd.Mastic(bits, circuit, **kw)
    rng = random.Random(n + bits)
    ctx = b"split-fold"
    vals = [rng.randrange(2 ** bits) for _ in range(n)]
    alphas = b"".join((v << (8 - bits)).to_bytes(1, "big") for v in vals)
    if circuit == "Count":
        meas = [rng.randrange(2) for _ in range(n)]
    else:
        meas = [rng.randrange(kw["length"]) for _ in range(n)]
    betas = b"".join(m.field.encode_vec(m.encode_measurement(x)) for x in meas)
    dev = m.reports_shard(ctx, alphas, betas, rng.randbytes(16 * n), rng.randbytes(m.RAND_SIZE * n))
    cand = tuple(sorted(set(tuple(bool((v >> (bits - 1 - i)) & 1) for i in range(3)) for v in vals[:50])))
    enc = m.encode_agg_param((2, cand, True))
    vk = bytes(range(16))
    p = m.field.MODULUS
    enc_sz = m.field.ENCODED_SIZE
    rows = len(cand) * (1 + m.OUTPUT_LEN)
    valid = np.array([rng.random() < 0.8 for _ in range(n)], dtype=np.uint8)
    for agg_id in range(2):
        m.prep_init_device(dev, vk, ctx, agg_id, enc)
        (_ps, _js, out, st) = m.prep_result(dev, agg_id, enc, want_out_shares=True)
        assert list(st) == [0] * n
        el = [int.from_bytes(out[i:i + enc_sz], "little") for i in range(0, len(out), enc_sz)]
        per = [el[r * rows:(r + 1) * rows] for r in range(n)]
        for mask in (None, valid):
            want = [0] * rows
            for r in range(n):
                if mask is None or mask[r]:
                    want = [a + b for (a, b) in zip(want, per[r])]
            want = b"".join((w % p).to_bytes(enc_sz, "little") for w in want)
            assert m.aggregate_device(agg_id, enc, mask, raw=True) == want
