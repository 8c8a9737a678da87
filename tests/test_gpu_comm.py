"""The library-owned RCCL communicator (include/mastic_hip.h: mastic_comm_*,
mastic_allgather_fold, mastic_merge_host, mastic_aggregate_merged; SURVEY.md
§8b "the ctx owns device buffers and RCCL comms", §8e) at world 1 on one GPU:
ncclCommInitRank with one rank, the all-gather on the ctx's stream, then the
GF(p) fold.  Every result equals the single-GPU forms (mastic_aggregate,
mastic_fold_shares) and the field sum (Mastic.merge, poc/mastic.py:390-397).
RCCL refuses two ranks on one device, so the library's world > 1 path runs
on one GPU through a shared-memory RCCL stand-in (tests/test_gpu_comm_nrank.py)
and with real RCCL on the driver's 8-GPU node; tests/test_multirank_cpu.py and
tests/test_split_cpu.py cover the multi-rank host logic over gloo."""
import random

import numpy as np
import pytest

from test_gpu_merge import _share_bytes, torch_cuda  # noqa: F401

pytestmark = pytest.mark.gpu


def _field_sum(F, shares):
    want = [F(0)] * len(shares[0])
    for s in shares:
        want = [a + b for (a, b) in zip(want, s)]
    return F.encode_vec(want)


@pytest.mark.parametrize("circuit,kw", [("Sum", dict(bits=6, max_measurement=9)),
                                        ("Histogram", dict(bits=5, length=3, chunk_length=2))],
                         ids=["Field64", "Field128"])
def test_world1_comm_equals_single_gpu_forms(torch_cuda, circuit, kw):
    torch = torch_cuda
    import mastic_amd
    from mastic_amd.merge import CommMerge, fold_on_gpu
    from oracle.field import Field64, Field128
    kw = dict(kw)
    bits = kw.pop("bits")
    m = mastic_amd.Mastic(bits, circuit, **kw)
    F = Field64 if m.field.ENCODED_SIZE == 8 else Field128
    assert m.comm_info() == (1, 0)
    m.comm_init(1, 0, m.comm_unique_id())
    assert m.comm_info() == (1, 0)
    with pytest.raises(ValueError):
        m.comm_init(1, 0, m.comm_unique_id())  # one communicator per ctx

    # all-gather + fold of device shares == mastic_fold_shares == the field sum
    rng = random.Random(5 + m.field.ENCODED_SIZE)
    n_elems = 301
    shares = [_share_bytes(F, rng, n_elems, near_p=True) for _ in range(3)]
    raw = b"".join(F.encode_vec(s) for s in shares)
    dev = torch.frombuffer(bytearray(raw), dtype=torch.uint8).cuda()
    out = torch.empty(n_elems * m.field.ENCODED_SIZE, dtype=torch.uint8, device="cuda")
    m.allgather_fold(dev.data_ptr(), 3, n_elems, out.data_ptr(), torch.cuda.current_stream().cuda_stream)
    want = _field_sum(F, shares)
    assert out.cpu().numpy().tobytes() == want
    assert fold_on_gpu(m, dev, 3, n_elems).cpu().numpy().tobytes() == want
    assert m.merge_host(raw, 3, n_elems) == want

    # agg_update + merge of prep_init results in HBM == mastic_aggregate
    ctx = b"comm-world1"
    n = 70
    alphas = [tuple(bool(rng.getrandbits(1)) for _ in range(bits)) for _ in range(n)]
    if circuit == "Sum":
        weights = [rng.randrange(kw["max_measurement"] + 1) for _ in range(n)]
    else:
        weights = [rng.randrange(kw["length"]) for _ in range(n)]
    nonces = b"".join(bytes([i]) * 16 for i in range(n))
    (pub, in0, in1) = m.shard_batch(ctx, alphas, weights, nonces, rng.randbytes(m.RAND_SIZE * n))
    reps = m.reports_upload(nonces, pub, in0, in1)
    cand = tuple(sorted(set(a[:4] for a in alphas)))
    ap = (3, cand, False)
    n_el = len(cand) * (1 + m.OUTPUT_LEN)
    vk = bytes(range(16))
    for a in range(2):
        m.prep_init_device(reps, vk, ctx, a, ap)
    valid = np.array([rng.random() < 0.75 for _ in range(n)], dtype=np.uint8)
    for mask in (None, valid):
        single = [m.aggregate_device(a, ap, mask, raw=True) for a in range(2)]
        assert m.aggregate_merged((0,), n_el, mask) == single[0]
        assert m.aggregate_merged((1,), n_el, mask) == single[1]
        both = m.aggregate_merged((0, 1), n_el, mask)
        assert both == _field_sum(F, [F.decode_vec(s) for s in single])
        # the collector's merge of both shares: the agg result of the plaintext
        assert CommMerge(m).total(n_el, mask) == both
    assert m.aggregate_merged((0, 1), n_el, zeros=True) == bytes(n_el * m.field.ENCODED_SIZE)
    with pytest.raises(ValueError):
        m.aggregate_merged((0,), n_el + 1)  # length must match the last prep_init
    m.comm_destroy()
    assert m.comm_info() == (1, 0)
    # without a communicator the same call is the world-1 merge
    assert m.aggregate_merged((0,), n_el) == m.aggregate_device(0, ap, raw=True)


def test_sweep_through_comm_merge_equals_local_sweep(torch_cuda):
    """compute_heavy_hitters with the library's communicator merging every
    level (CommMerge: fold, all-gather, GF(p) merge in one call) gives the
    same per-level aggregates and heavy hitters as the single-GPU sweep."""
    import mastic_amd
    from mastic_amd.heavy_hitters import compute_heavy_hitters
    from mastic_amd.merge import CommMerge
    rng = random.Random(9)
    m = mastic_amd.MasticSum(8, 7)
    ctx = b"comm-sweep"
    n = 400
    pool = [tuple(bool(rng.getrandbits(1)) for _ in range(8)) for _ in range(6)]
    alphas = [pool[min(int(rng.paretovariate(1.0)) - 1, 5)] for _ in range(n)]
    weights = [rng.randrange(8) for _ in range(n)]
    nonces = rng.randbytes(16 * n)
    (pub, in0, in1) = m.shard_batch(ctx, alphas, weights, nonces, rng.randbytes(m.RAND_SIZE * n))
    reps = m.reports_upload(nonces, pub, in0, in1)
    vk = bytes(16)
    (t_local, t_comm) = ([], [])
    hh_local = compute_heavy_hitters(m, ctx, {"default": 60}, reps, verify_key=vk, trace=t_local)
    m.comm_init(1, 0, m.comm_unique_id())
    hh_comm = compute_heavy_hitters(m, ctx, {"default": 60}, reps, verify_key=vk, merge=CommMerge(m))
    assert hh_comm == hh_local and hh_local
    compute_heavy_hitters(m, ctx, {"default": 60}, reps, verify_key=vk, trace=t_comm, merge=CommMerge(m))
    assert [(lv.level, lv.prefixes, lv.agg_result) for lv in t_comm] == \
        [(lv.level, lv.prefixes, lv.agg_result) for lv in t_local]


def _two_agg_results(m, rng, ctx, n=70):
    """Both aggregators' prep_init of n random Mastic(6, Sum 9) reports."""
    alphas = [tuple(bool(rng.getrandbits(1)) for _ in range(6)) for _ in range(n)]
    weights = [rng.randrange(10) for _ in range(n)]
    nonces = b"".join(bytes([i]) * 16 for i in range(n))
    (pub, in0, in1) = m.shard_batch(ctx, alphas, weights, nonces, rng.randbytes(m.RAND_SIZE * n))
    reps = m.reports_upload(nonces, pub, in0, in1)
    cand = tuple(sorted(set(a[:4] for a in alphas)))
    ap = (3, cand, False)
    for a in range(2):
        m.prep_init_device(reps, bytes(range(16)), ctx, a, ap)
    return reps, ap, len(cand) * (1 + m.OUTPUT_LEN)


def test_collective_local_failure_returns_cleanly(torch_cuda):
    """A rank-local failure inside a collective call (an injected ENOMEM on a
    staging buffer) is reported after the agreement round and leaves the
    communicator usable: the next call merges correctly.  At world 1 the
    agreement round is this rank alone; the same code path at N ranks makes
    every peer return the failing rank's code instead of blocking in the
    all-gather (include/mastic_hip.h, failure model)."""
    import mastic_amd
    from mastic_amd._lib import MasticError
    torch = torch_cuda
    rng = random.Random(61)
    m = mastic_amd.Mastic(6, "Sum", max_measurement=9)
    m.comm_init(1, 0, m.comm_unique_id(), timeout_ms=20000)
    (_reps, ap, n_el) = _two_agg_results(m, rng, b"comm-enomem")
    want = m.aggregate_device(0, ap, raw=True)
    # fresh ctx: the first merge must allocate its staging buffers
    m.set_test_hooks(fail_allocs=1)
    with pytest.raises(MasticError) as ei:
        m.aggregate_merged((0,), n_el)
    assert ei.value.code == -12
    assert m.set_test_hooks(fail_allocs=0) == 0  # the injected failure was used
    assert m.aggregate_merged((0,), n_el) == want
    # the device-buffer form: a larger share forces a new gather buffer
    n_big = 4 * n_el + 1000
    dev = torch.zeros(3 * n_big * 8, dtype=torch.uint8, device="cuda")
    out = torch.empty(n_big * 8, dtype=torch.uint8, device="cuda")
    m.set_test_hooks(fail_allocs=1)
    with pytest.raises(MasticError) as ei:
        m.allgather_fold(dev.data_ptr(), 3, n_big, out.data_ptr(), torch.cuda.current_stream().cuda_stream)
    assert ei.value.code == -12
    m.set_test_hooks(fail_allocs=0)
    m.allgather_fold(dev.data_ptr(), 3, n_big, out.data_ptr(), torch.cuda.current_stream().cuda_stream)
    assert not out.any().item()
    # argument errors are agreed on too, and leave the communicator usable
    with pytest.raises(ValueError):
        m.aggregate_merged((0,), n_el + 1)
    assert m.aggregate_merged((0, 1), 0) == b""
    assert m.aggregate_merged((0,), n_el) == want
    assert m.comm_info() == (1, 0)
    m.comm_destroy()


_TIMEOUT_SCRIPT = r"""
import os, sys, time
sys.path.insert(0, %(pkg)r)
import mastic_amd
from mastic_amd._lib import MasticError
m = mastic_amd.Mastic(6, "Sum", max_measurement=9)
t0 = time.time()
try:
    m.comm_init(2, 0, m.comm_unique_id(), timeout_ms=3000)   # rank 1 never joins
    print("RESULT joined", flush=True)
except MasticError as e:
    print("RESULT code=%%d after=%%.1f msg=%%s" %% (e.code, time.time() - t0, e), flush=True)
print("INFO", m.comm_info(), flush=True)
m.comm_init(1, 0, m.comm_unique_id(), timeout_ms=3000)     # the ctx can join another communicator
print("INFO2", m.comm_info(), m.merge_host(bytes(16), 2, 1).hex(), flush=True)
m.comm_destroy()
del m
sys.stdout.flush()
print("EXITING", flush=True)
"""


def test_comm_init_without_peers_times_out(torch_cuda):
    """mastic_comm_init for 2 ranks with no second rank: RCCL's init (which
    blocks in its bootstrap until every rank joins) runs on a library thread
    and the call returns MASTIC_ETIMEDOUT after the ctx's bound instead of
    blocking forever; the ctx is world 1 again and can join another
    communicator, and the process still exits normally with the abandoned
    init pending.  Runs in its own process, bounded."""
    import subprocess
    import sys
    from conftest import PKG_ROOT
    p = subprocess.Popen([sys.executable, "-u", "-c", _TIMEOUT_SCRIPT % {"pkg": PKG_ROOT}], stdout=subprocess.PIPE,
                         stderr=subprocess.STDOUT, text=True)
    try:
        out, _ = p.communicate(timeout=100)
    except subprocess.TimeoutExpired:
        p.kill()
        out, _ = p.communicate()
        raise AssertionError("probe did not finish:\n" + out[-3000:])
    assert p.returncode == 0, out[-3000:]
    line = [ln for ln in out.splitlines() if ln.startswith("RESULT")][0]
    assert "code=-110" in line, out
    after = float(line.split("after=")[1].split()[0])
    assert 2.5 <= after < 30, line
    assert "INFO (1, 0)" in out
    assert "INFO2 (1, 0) " + "00" * 8 in out
    assert "EXITING" in out
