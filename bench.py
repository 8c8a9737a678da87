"""Benchmark: VIDPF report x prefix evaluations/sec for Mastic prep_init +
aggregate on MI355X (BASELINE.json metric).  Default config C2 (the metric's headline):
Mastic(BITS=32, Sum max=255), 10k candidate prefixes at level 31, weight
check on, leader side (agg_id 0).

A step = one pass of the hot path over one batch of reports resident in HBM:
prep_init (VIDPF level walk, binder sponges, eval proof, FLP query) + the
aggregate fold of all out shares; with N > 1 ranks also the RCCL all-gather
of the per-rank agg shares and the on-GPU mod-p merge.  Reports are sharded
over ranks (independent units, weak scaling).

    python bench.py [--gpus N --steps K --warmup W --config c2|c3|c4|c5 --reports R --prefixes P]
    (N > 1: launched by torch.distributed.run, one rank per GPU)
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "draft-mouris-cfrg-mastic_amd"))

METRIC = "VIDPF report x prefix evals/sec at 1/2/4/8 GPUs; % of int-VALU peak"
# Fixed op-cost convention: int32 ops
AES_BLOCK_OPS = 340
KECCAK_OPS = 3720
FIELD_ADD_OPS = 4
# int32 VALU peak: 256 CUs x 4 SIMD x 32 lanes x 2.4 GHz (MI355X_MICROARCH.md)
VALU_PEAK_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12
# full-rate int32 VALU throughput measured on an MI355X at the clock it holds under load
# (v_bitop3_b32, 8 waves/SIMD: tools/valu_peak.hip, profiles/r01_v9_valu_peak.json)
VALU_MEASURED_TOPS = 67.9
HBM_PEAK_GBS = 8000.0


# BASELINE.json configs measured on one GPU (C1 is the reference's CPU-sized
# sweep; it is a parity case, tests/test_gpu_configs.py).  Each entry: Mastic
# constructor, level, candidate prefixes, default reports per rank per step.
CONFIGS = {
    "c2": dict(circuit="Sum", kw=dict(bits=32, max_measurement=255), prefixes=10000, reports=16384,
               total=1000000, full_job=True,
               desc="C2: Mastic(BITS=32, Sum max=255) prep_init+aggregate, level 31"),
    "c3": dict(circuit="Count", kw=dict(bits=256), prefixes=128, reports=16384,
               desc="C3: Mastic(BITS=256, Count) prep_init+aggregate at level 255 of the threshold-pruned "
                    "sweep (128 surviving candidates, the Zipf(1.1)/0.05% frontier)"),
    "c1sweep": dict(circuit="Count", kw=dict(bits=16), prefixes=0, reports=1000, sweep=True, pool=128, zipf=1.2,
                    weight_p=0.9, threshold=10,
                    desc="C1: Mastic(BITS=16, Count) weighted heavy hitters, full 16-level sweep (Zipf(1.2) over "
                         "128 random 16-bit strings, weights Bernoulli(0.9), threshold 10), both aggregators per "
                         "level: the reference's CPU-sized case"),
    "c3sweep": dict(circuit="Count", kw=dict(bits=256), prefixes=0, reports=65536, sweep=True, pool=2 ** 20, zipf=1.1,
                    weight_p=1.0, threshold=None, spec_sample=8192, spec_every=8,
                    desc="C3: Mastic(BITS=256, Count) weighted heavy hitters, full 256-level threshold-pruned "
                         "sweep (Zipf(1.1) over 2^20 random 256-bit strings, threshold 0.05% of all reports), "
                         "both aggregators per level; run with --steps 1 --warmup 0"),
    "c2sweep": dict(circuit="Sum", kw=dict(bits=32, max_measurement=255), prefixes=0, reports=1000000, sweep=True,
                    pool="c2", zipf=1.1, threshold_frac=0.0005, spec_sample=65536,
                    desc="north_star: Mastic(BITS=32, Sum max=255) (C2's VDAF) weighted heavy hitters over 1M "
                         "reports, full 32-level threshold-pruned sweep (alphas Zipf(1.1) over C2's 10k random "
                         "32-bit attributes, weights uniform 0..255, threshold 0.05% of the expected total "
                         "weight), both aggregators per level, weight check at level 0; run with --steps 1 "
                         "--warmup 0"),
    "c4": dict(circuit="Histogram", kw=dict(bits=64, length=64, chunk_length=8), prefixes=1000, reports=16384,
               desc="C4: Mastic(BITS=64, Histogram length=64 chunk 8, Field128) prep_init+aggregate, level 63"),
    "c5": dict(circuit="SumVec", kw=dict(bits=32, length=1024, sum_vec_bits=1, chunk_length=32), prefixes=100,
               reports=16384,
               desc="C5: Mastic(BITS=32, SumVec length=1024 bits=1 chunk 32, Field128) prep_init+aggregate, "
                    "level 31"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS),
                    help="BASELINE config (c2 = the metric's headline config)")
    ap.add_argument("--reports", type=int, default=0, help="reports per rank per step (0 = config default)")
    ap.add_argument("--prefixes", type=int, default=0, help="candidate prefixes (0 = config default)")
    ap.add_argument("--total-reports", type=int, default=0,
                    help="reports resident in HBM per rank; steps walk distinct --reports slices of them "
                         "(0 = config default: 1M for c2)")
    ap.add_argument("--pool-reports", type=int, default=0,
                    help="distinct reports resident per rank (0 = all of --total-reports); a larger job cycles "
                         "through the pool slice by slice (SURVEY §8d: C5's cycled pool of 2^16 reports)")
    ap.add_argument("--full-job", type=int, default=-1,
                    help="also time prep_init+aggregate over all resident reports (-1 = config default)")
    ap.add_argument("--agg-id", type=int, default=0)
    ap.add_argument("--cpu-baseline", type=int, default=1, help="0 disables the CPU baseline leg")
    ap.add_argument("--cpu-procs", type=int, default=0,
                    help="CPU baseline pool size (0 = every CPU this process may use, see cpu_pool_size)")
    ap.add_argument("--launch-probe", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--frontier-cache", type=int, default=1,
                    help="sweep configs: keep each level's binder inputs in HBM (Mastic.set_frontier_cache)")
    ap.add_argument("--split", type=int, default=0,
                    help="sweep configs: --reports is the JOB's report count, divided over the ranks (strong "
                         "scaling; thresholds from the job total); c2: the resident reports of the full_job leg")
    ap.add_argument("--virtual-ranks", type=int, default=1,
                    help="sweep configs, one GPU: time rank 0's share of a K-way split job (the other ranks' "
                         "aggregates added in plaintext per level), to predict K-GPU strong scaling")
    ap.add_argument("--north-star", type=int, default=1,
                    help="c2: after the headline, the north_star job (1M-report full 32-level c2sweep, split over "
                         "the ranks) under a north_star key; 0 skips it")
    ap.add_argument("--memory-budget-gb", type=float, default=0,
                    help="HBM budget per context (0 = the library default, 75%% of free HBM); rehearsals with "
                         "several ranks sharing one GPU give each rank a slice")
    ap.add_argument("--lib", default="",
                    help="A/B tools only: bind this build of libmastic_hip (e.g. an experiment-knobs build) "
                         "instead of the shipped one; the JSON line then names it under 'library'")
    ap.add_argument("--standalone", type=int, default=1,
                    help="after the timed region, one more step (c2) / sweep (sweep configs) with every binder-sponge "
                         "launch running alone (Mastic.set_serial_sponges): the sponge kernels' and the level "
                         "kernel's own rooflines; 0 skips it")
    ap.add_argument("--north-star-reports", type=int, default=0,
                    help="job size of the north_star leg (0 = the 1M of BASELINE.json; smaller only for rehearsals)")
    return ap.parse_args()


def _attrs(rng, bits, n_prefixes):
    """n distinct random bits-bit attributes, sorted, as MSB-first byte rows."""
    if bits == 32:  # the C2 stream of earlier rounds (uint32 draws)
        attrs = np.unique(rng.integers(0, 2 ** 32, size=n_prefixes, dtype=np.uint64).astype(np.uint32))
        while len(attrs) < n_prefixes:
            attrs = np.unique(np.concatenate([attrs, rng.integers(0, 2 ** 32, size=n_prefixes - len(attrs),
                                                                  dtype=np.uint64).astype(np.uint32)]))
        return np.sort(attrs).astype(">u4").view(np.uint8).reshape(-1, 4)
    ab = (bits + 7) // 8
    rows = np.unique(rng.integers(0, 256, size=(n_prefixes, ab), dtype=np.uint8), axis=0)
    return rows  # np.unique sorts rows lexicographically (= MSB-first path order)


def synth(m, cfg, rank, n_reports, n_prefixes, seed):
    """Synthetic inputs: random attributes, alphas uniform over
    them, weights per the circuit, distinct random nonces per report."""
    rng = np.random.default_rng(seed)
    attrs = _attrs(rng, cfg["kw"]["bits"], n_prefixes)
    rrng = np.random.default_rng(seed * 1000003 + rank)
    alphas = attrs[rrng.integers(0, len(attrs), size=n_reports)]
    betas = encode_betas(m, cfg, n_reports, rrng)
    nonces = rrng.integers(0, 256, size=16 * n_reports, dtype=np.uint8).tobytes()
    rands = rrng.integers(0, 256, size=m.RAND_SIZE * n_reports, dtype=np.uint8).tobytes()
    return attrs, alphas.tobytes(), betas, nonces, rands


def encode_betas(m, cfg, n, rrng):
    """Valid.encode of random measurements, encode_vec'd (ENC bytes LE per element)."""
    c = cfg["circuit"]
    dt = "<u8"
    if c == "Sum":  # Sum(255): b = 8, offset 0 -> bits(w) || bits(w)
        w = rrng.integers(0, 256, size=n)
        bits = ((w[:, None] >> np.arange(8)) & 1).astype(dt)
        return np.concatenate([bits, bits], axis=1).tobytes()
    if c == "Count":
        return (rrng.random(n) < 0.9).astype(dt).tobytes()
    if c == "Histogram":
        e = np.zeros((n, m.length, 2), dtype=dt)
        e[np.arange(n), rrng.integers(0, m.length, size=n), 0] = 1
        return e.tobytes()
    # SumVec bits=1: one field element per bit
    e = np.zeros((n, m.length, 2), dtype=dt)
    e[:, :, 0] = rrng.integers(0, 2, size=(n, m.length))
    return e.tobytes()


def agg_param_bytes(level, attrs):
    return level.to_bytes(2, "big") + len(attrs).to_bytes(4, "big") + attrs.tobytes() + b"\x01"


# ---------------------------------------------------------------- CPU baseline
def _cpu_worker(job):
    (spec, enc_ap, nonce, pub, ins, vk, ctx, agg_id) = job
    o = _oracle_mastic(*spec)
    ap = o.decode_agg_param(enc_ap)
    cws = o.vidpf.decode_public_share(pub)
    isd = o.decode_input_share(agg_id, ins)
    t = time.perf_counter()
    (_st, sh) = o.prep_init(vk, ctx, agg_id, ap, nonce, cws, isd)
    dt = time.perf_counter() - t
    return (dt, o.test_vec_encode_prep_share(sh))


def _oracle_mastic(circuit, kw):
    sys.path.insert(0, ROOT)
    from oracle import mastic as om
    kw = dict(kw)
    bits = kw.pop("bits")
    if circuit == "Sum":
        return om.MasticSum(bits, kw["max_measurement"])
    if circuit == "Count":
        return om.MasticCount(bits)
    if circuit == "Histogram":
        return om.MasticHistogram(bits, kw["length"], kw["chunk_length"])
    return om.MasticSumVec(bits, kw["length"], kw["sum_vec_bits"], kw["chunk_length"])


def native_cpu_point(m, cfg, enc_ap, reps, vk, ctx, agg_id, threads, n_prefixes, budget_s=12.0):
    """The native multithreaded CPU baseline (oracle/native_prep.c: AES-NI,
    64-bit Keccak, one thread per report range; the FLP query in the Python
    oracle): prep_init of the same workload's reports on the host, as many
    per thread as fill a ~budget_s wall-time sample (one report per thread
    first, to size it), its prep shares checked against the GPU's.  The
    value is the C part's rate (VIDPF, binders, eval proof; the FLP query is
    <1 % of the work and runs in Python here); the rate including the Python
    FLP is reported beside it."""
    sys.path.insert(0, ROOT)
    from oracle.native import has_aesni, prep_init_native
    o = _oracle_mastic(cfg["circuit"], cfg["kw"])
    ap = o.decode_agg_param(enc_ap)
    psz = m.prep_share_size(ap[2])
    # calibration: one report per thread (not counted)
    n1 = min(threads, reps.n)
    (rn, pub, in0, in1) = reps.view(0, n1).download()
    t1 = {}
    prep_init_native(o, vk, ctx, agg_id, ap, rn, pub, in0 if agg_id == 0 else in1, threads, times=t1)
    per_thread = int(max(2, min(64, budget_s / max(t1["native_c_s"], 1e-3))))
    nn = min(per_thread * threads, reps.n)
    (rn, pub, in0, in1) = reps.view(0, nn).download()
    ins = in0 if agg_id == 0 else in1
    tm = {}
    t = time.perf_counter()
    (shares, _outs) = prep_init_native(o, vk, ctx, agg_id, ap, rn, pub, ins, threads, times=tm)
    wall = time.perf_counter() - t
    (gps, _js, _o, _st) = m.prep_init_batch(vk, ctx, agg_id, enc_ap, rn, pub, ins, want_out_shares=False)
    parity = all(gps[psz * i:psz * (i + 1)] == shares[i] for i in range(nn))
    return {
        "value": nn * n_prefixes / tm["native_c_s"],
        "unit": "report*prefix/s",
        "cores": threads,
        "kind": "port",
        "value_with_python_flp": nn * n_prefixes / wall,
        "impl": "native C (oracle/native_prep.c): AES-NI %s, 64-bit Keccak-p, pthreads; FLP query in the Python "
                "oracle (timed separately)" % ("on" if has_aesni() else "off (byte-wise AES)"),
        "sample": "%d reports x %d prefixes on %d threads (%d per thread): C part %.2f s, + Python FLP %.2f s; "
                  "GPU/CPU prep shares bit-identical: %s" % (nn, n_prefixes, threads, per_thread,
                                                            tm["native_c_s"], tm["flp_py_s"], parity),
        "parity": parity,
    }


def cpu_baseline(jobs, procs):
    import multiprocessing as mp
    t = time.perf_counter()
    if procs == 1:
        res = [_cpu_worker(j) for j in jobs]
    else:
        with mp.get_context("spawn").Pool(procs) as pool:
            res = pool.map(_cpu_worker, jobs)
    wall = time.perf_counter() - t
    return wall, res


def max_over_ranks(dist, torch, x):
    """The MAX over ranks of a host float (the timed regions): a device
    tensor through RCCL, a host one through a gloo rehearsal group."""
    if dist is None:
        return x
    on_gpu = dist.get_backend() != "gloo"
    tt = torch.tensor([x], dtype=torch.float64, device="cuda" if on_gpu else "cpu")
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    return float(tt.item())


def lib_comm_init(m, dist, world, rank, timeout_ms=0):
    """Join m's ctx to the library's own RCCL communicator: rank 0 creates the
    id (mastic_comm_unique_id), the gloo control group broadcasts it, every
    rank calls mastic_comm_init_timeout (collective; a peer that never joins
    ends in ETIMEDOUT after the library's bound instead of a hang), and the
    ranks agree on the outcome over gloo.  There is no fallback: if any rank's
    init failed, every rank raises SystemExit(3) (the run exits non-zero; the
    gloo merge exists only as the MASTIC_BENCH_BACKEND=gloo rehearsal)."""
    import torch

    def bcast(obj):
        box = [obj]
        dist.broadcast_object_list(box, src=0)
        return box[0]

    err = None
    uid = None
    if rank == 0:
        try:
            uid = m.comm_unique_id()
        except Exception as e:  # noqa: BLE001 -- rank 0 could not create the id: every rank learns it
            err = e
    uid = bytes(bcast(uid or b""))
    dist.barrier()  # every rank is at its init: none waits on a peer still generating data
    ok = 1
    if err is None and not uid:
        err = RuntimeError("rank 0 could not create the communicator id")
    if err is None and os.environ.get("MASTIC_BENCH_COMM_FAIL_RANK") == str(rank):
        # tests/test_gpu_bench_2rank.py: a rank whose init fails (the exit path end to end)
        err = RuntimeError("injected by MASTIC_BENCH_COMM_FAIL_RANK")
    if err is None:
        try:
            m.comm_init(world, rank, uid, timeout_ms)
        except Exception as e:  # noqa: BLE001 -- reported below, on every rank
            err = e
    if err is not None:
        ok = 0
        print("bench.py rank %d: mastic_comm_init failed (%s)" % (rank, err), file=sys.stderr, flush=True)
    flag = torch.tensor([ok], dtype=torch.int32)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    if int(flag.item()) == 1:
        return True
    if ok:
        m.comm_destroy()
    print("bench.py rank %d: a rank could not join the library's RCCL communicator; exiting (no silent fallback "
          "to another merge path)" % rank, file=sys.stderr, flush=True)
    raise SystemExit(3)


def device_desc(local):
    """This rank's GPU for the bench line's comm record."""
    import torch
    d = {"local_rank": local}
    try:
        props = torch.cuda.get_device_properties(local)
        d["name"] = props.name
        for k in ("pci_bus_id", "pci_device_id", "pci_domain_id", "uuid"):
            if hasattr(props, k):
                d[k] = str(getattr(props, k))
    except Exception as e:  # noqa: BLE001 -- descriptive only
        d["error"] = str(e)
    return d


def comm_record(dist, world, rank, lib_comm, m=None, desc=None):
    """The merge path of a bench line: which transport carried the ranks' agg
    shares, how many ranks the library's communicator saw, and every rank's
    device (gathered over the control group).  desc: this rank's device
    record (default: device_desc of LOCAL_RANK)."""
    if desc is None:
        desc = device_desc(int(os.environ.get("MASTIC_BENCH_DEVICE", os.environ.get("LOCAL_RANK", "0"))))
    desc = dict(desc, rank=rank)
    if dist is None:
        return {"backend": "none", "nranks": 1, "devices": [desc], "path": "single process: no merge"}
    devs = [None] * world
    dist.all_gather_object(devs, desc)
    if lib_comm:
        stand_in = os.environ.get("MASTIC_RCCL_LIB")  # the library's test hook (tests/host/fake_rccl.cpp)
        return {"backend": "rccl-stand-in" if stand_in else "rccl", "nranks": int(m.comm_info()[0]), "devices": devs,
                "path": "library-owned RCCL communicator: mastic_aggregate_merged / mastic_allgather_fold "
                        "(agreement round, ncclAllGather, GF(p) fold on the GPU)"
                        + (" -- transport: %s (MASTIC_RCCL_LIB rehearsal, ranks sharing one GPU)" % stand_in
                           if stand_in else "")}
    return {"backend": "gloo-rehearsal", "nranks": world, "devices": devs,
            "path": "MASTIC_BENCH_BACKEND=gloo: host copies all-gathered over gloo, GF(p) fold on the GPU "
                    "(ranks sharing one GPU)"}


# ---------------------------------------------------------------- sweeps
def sweep_population(cfg, bits, kw, seed, n, stream):
    """Synthetic sweep reports: alphas Zipf over a pool of
    attributes, weights per circuit, random nonces and randomness.  Returns
    (alphas uint8 [n, ceil(bits/8)], weights int64 [n], betas, nonces, rands)."""
    if cfg.get("pool") == "c2":  # the C2 attribute set (same draws as bench --config c2)
        pool = _attrs(np.random.default_rng(seed), bits, 10000)
    else:
        pool = np.random.default_rng(seed).integers(0, 256, size=(cfg["pool"], bits // 8), dtype=np.uint8)
    rrng = np.random.default_rng(stream)
    ranks = rrng.zipf(cfg["zipf"], size=n)
    while (ranks > len(pool)).any():
        bad = ranks > len(pool)
        ranks[bad] = rrng.zipf(cfg["zipf"], size=int(bad.sum()))
    alphas = pool[ranks - 1]
    if cfg["circuit"] == "Sum":  # weights uniform 0..max
        w = rrng.integers(0, kw["max_measurement"] + 1, size=n)
        nb = int(kw["max_measurement"]).bit_length()
        off = 2 ** nb - 1 - kw["max_measurement"]
        betas = np.concatenate([(w[:, None] >> np.arange(nb)) & 1, ((w + off)[:, None] >> np.arange(nb)) & 1],
                               axis=1).astype("<u8")
    else:
        w = (rrng.random(n) < cfg["weight_p"]).astype(np.int64)
        betas = w.astype("<u8")
    nonces = rrng.integers(0, 256, size=16 * n, dtype=np.uint8)
    return alphas, w, betas, nonces, rrng


def split_bounds(n_job, parts):
    """Report ranges of a job split over `parts` ranks (strong scaling):
    contiguous, sizes differing by at most one, covering the job."""
    return [(n_job * i // parts, n_job * (i + 1) // parts) for i in range(parts)]


def sweep_threshold(cfg, kw, n_job):
    """0.05 % of the job's expected total weight (Sum) / of its reports
    (Count), identical on every rank; C1 has a fixed threshold."""
    if cfg["circuit"] == "Sum":
        return max(1, int(np.ceil(cfg["threshold_frac"] * n_job * kw["max_measurement"] / 2)))
    return cfg["threshold"] or max(1, int(np.ceil(0.0005 * n_job)))


def prefix_sums(alphas, w, level, prefixes):
    """Plaintext per-candidate [reports, weight] of a set of reports at a sweep
    level (talks/func.py:49-80): the aggregate the collector unshards, as the
    integer pairs of Count/Sum's (counter, truncated weight) output."""
    L = level + 1
    ab = alphas.shape[1]
    val = np.zeros(len(alphas), dtype=np.uint64)
    for j in range((L + 7) // 8):
        val = (val << np.uint64(8)) | alphas[:, j].astype(np.uint64)
    val >>= np.uint64(8 * ((L + 7) // 8) - L)
    pv = np.array([int("".join("1" if b else "0" for b in p), 2) for p in prefixes], dtype=np.uint64)
    order = np.argsort(pv)
    idx = np.searchsorted(pv[order], val)
    idx_c = np.minimum(idx, len(pv) - 1)
    hit = pv[order][idx_c] == val
    cnt = np.bincount(order[idx_c[hit]], minlength=len(pv))
    ws = np.bincount(order[idx_c[hit]], weights=w[hit], minlength=len(pv))
    del ab
    return cnt.astype(np.int64), ws.astype(np.int64)


class VirtualRanksMerge:
    """One rank of a K-way split job on a single GPU (bench.py --virtual-ranks
    K): the per-level merge adds the plaintext aggregate of the other K-1
    ranks' reports to this rank's GPU agg shares, so the candidate trajectory,
    and with it this rank's GPU work per level, is exactly that of rank 0 of a
    real K-GPU run (only the RCCL all-gather of a few KB is missing).  Count
    and Sum only (aggregate = [reports, weight] per candidate)."""

    def __init__(self, m, rest_alphas, rest_w):
        self.m = m
        self.rest_alphas = rest_alphas
        self.rest_w = rest_w
        self.cur = None
        # the other ranks' per-level aggregates by (level, candidates): computed
        # in the warmup sweep, looked up in the timed one (same trajectory), so
        # the host-side plaintext work stays out of the timed region
        self.rest = {}

    def begin_level(self, level, prefixes):
        self.cur = (level, prefixes)

    def total(self, n_elems, valid=None, have_results=True):
        import torch
        from mastic_amd.merge import aggregate_to_tensor, fold_on_gpu
        m = self.m
        enc = m.field.ENCODED_SIZE
        if n_elems == 0:
            return b""
        if have_results:
            local = torch.empty(2 * n_elems * enc, dtype=torch.uint8, device="cuda")
            for agg_id in range(2):
                aggregate_to_tensor(m, agg_id, n_elems, valid, out=local[agg_id * n_elems * enc:])
            merged = np.frombuffer(fold_on_gpu(m, local, 2, n_elems).cpu().numpy().tobytes(), dtype="<u8")
        else:
            # this rank's share has no reports left (as SweepMerge: zero shares)
            merged = np.zeros(n_elems, dtype="<u8")
        key = (self.cur[0], tuple(self.cur[1]))
        rest = self.rest.get(key)
        if rest is None:
            (cnt, ws) = prefix_sums(self.rest_alphas, self.rest_w, key[0], key[1])
            rest = self.rest[key] = np.stack([cnt, ws], axis=1).reshape(-1).astype(np.uint64)
        p = m.field.MODULUS
        return np.array([(int(a) + int(b)) % p for (a, b) in zip(merged.tolist(), rest.tolist())],
                        dtype="<u8").tobytes()


def run_sweep(args, cfg, world, rank, local, dist, torch, split=None, steps=None, warmup=None, n_job=None,
              with_cpu=None, emit=True, m=None):
    """The reference's heavy-hitters driver (examples.py:37-91,
    mastic_amd.heavy_hitters) over HBM-resident reports: both aggregators'
    prep_init, the decide and the fold at every level, each level's agg shares
    merged over RCCL before pruning.  A step = one full level sweep.  Units =
    sum over levels and aggregators of reports x candidate prefixes.

    Weak scaling (default): every rank sweeps its own `--reports` reports.
    Strong scaling (split, the north_star job): the job's reports (generated
    identically on every rank) are divided over the ranks; thresholds use the
    job total.  --virtual-ranks K (one GPU): rank 0's share of a K-way split,
    the other ranks' aggregates added in plaintext (VirtualRanksMerge)."""
    from mastic_amd import Mastic
    from mastic_amd.heavy_hitters import compute_heavy_hitters
    from mastic_amd.merge import CommMerge, merge_field_shares

    split = args.split if split is None else split
    steps = args.steps if steps is None else steps
    warmup = args.warmup if warmup is None else warmup
    do_cpu = args.cpu_baseline if with_cpu is None else with_cpu
    kw = dict(cfg["kw"])
    bits = kw.pop("bits")
    if m is None:
        m = Mastic(bits, cfg["circuit"], device=local, **kw)
    budget_gb = args.memory_budget_gb or cfg.get("memory_budget_gb")
    if budget_gb:
        m.set_memory_budget(int(budget_gb * 2 ** 30))
    ctx = b"mastic-mi355x-bench"
    seed = 0x4D41 + int(cfg.get("seed_digit", args.config[1]))
    vr = getattr(args, "virtual_ranks", 1) or 1
    if vr > 1 and (world > 1 or cfg["circuit"] not in ("Count", "Sum")):
        raise SystemExit("--virtual-ranks: one process, Count or Sum")
    n_req = n_job or args.reports or cfg["reports"]
    if split or vr > 1:
        n_job = n_req
        (alphas_job, w_job, betas_job, nonces_job, rrng) = sweep_population(cfg, bits, kw, seed, n_job,
                                                                             seed * 1000003)
        rands_job = rrng.integers(0, 256, size=m.RAND_SIZE * n_job, dtype=np.uint8)
        (lo, hi) = split_bounds(n_job, max(world, vr))[rank]
        n_rep = hi - lo
        alphas, w = alphas_job[lo:hi], w_job[lo:hi]
        betas = betas_job[lo:hi].tobytes()
        nonces = nonces_job[16 * lo:16 * hi].tobytes()
        rands = rands_job[m.RAND_SIZE * lo:m.RAND_SIZE * hi].tobytes()
        del betas_job, nonces_job, rands_job
    else:
        n_rep = n_req
        n_job = n_rep * world
        (alphas, w, betas, nonces, rrng) = sweep_population(cfg, bits, kw, seed, n_rep, seed * 1000003 + rank)
        betas = betas.tobytes()
        nonces = nonces.tobytes()
        rands = rrng.integers(0, 256, size=m.RAND_SIZE * n_rep, dtype=np.uint8).tobytes()
        alphas_job, w_job = (alphas, w) if world == 1 else (None, None)
    threshold = sweep_threshold(cfg, kw, n_job)
    t_sh = time.perf_counter()
    reps = m.reports_shard(ctx, alphas.tobytes(), betas, nonces, rands)
    m.synchronize()
    shard_s = time.perf_counter() - t_sh
    del betas, nonces, rands
    vk = np.random.default_rng(0x4D41).integers(0, 256, size=16, dtype=np.uint8).tobytes()  # gen_rand(16)
    thresholds = {"default": threshold}
    if vr > 1:
        merge = VirtualRanksMerge(m, alphas_job[n_rep:], w_job[n_rep:])
    elif dist and getattr(args, "lib_comm", False) and lib_comm_init(m, dist, world, rank):
        merge = CommMerge(m)
    else:
        merge = merge_field_shares(m, dist) if dist else None
    comm = comm_record(dist, world, rank, isinstance(merge, CommMerge), m) if vr == 1 else {
        "backend": "none (virtual ranks)", "nranks": 1, "devices": [], "path": "VirtualRanksMerge: the other "
        "ranks' aggregates added in plaintext"}

    cached_levels = []
    phases = {}
    # cpu_parity_cached: the leader prep shares of the CPU leg's sample reports
    # at its sample levels, as the warmup sweep (frontier cache on, the timed
    # path) computed them; the CPU leg replays the same reports and levels in
    # the oracle (spec-literal) and compares
    procs = cpu_pool_size(args.cpu_procs)
    check_levels = set(range(0, bits, max(1, bits // 8))[:8])
    captured = {}
    want_capture = rank == 0 and world == 1 and do_cpu and warmup > 0

    def capture(level, enc, dev):
        if level in check_levels:
            (ps, _js, _o, _st) = m.prep_result(dev, 0, enc)
            psz = m.prep_share_size(level == 0)
            captured[level] = [ps[psz * i:psz * (i + 1)] for i in range(min(procs, dev.n))]

    def step(trace, timing, hook=None):
        cached_levels.clear()
        return compute_heavy_hitters(m, ctx, thresholds, reps, verify_key=vk, trace=trace, merge=merge,
                                     timing=timing, frontier_cache=bool(args.frontier_cache),
                                     cached_levels=cached_levels, phase_times=phases if timing is not None else None,
                                     level_hook=hook)

    captured_hits = []
    for i in range(warmup):
        step(None, None, capture if (want_capture and i == 0) else None)
        if want_capture and i == 0:
            captured_hits = sorted(set(cached_levels) & set(captured))
        if rank == 0:
            print("[sweep] warmup %d done" % (i + 1), file=sys.stderr, flush=True)
    m.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    traces, timing = [], []
    hh = None
    for i in range(steps):
        tr = []
        hh = step(tr, timing)
        traces.append(tr)
        if rank == 0:
            print("[sweep] step %d done" % (i + 1), file=sys.stderr, flush=True)
    m.synchronize()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    dt = time.perf_counter() - t0
    dt_local = dt
    (free_b, total_b) = torch.cuda.mem_get_info()
    hbm_used = (total_b - free_b) / 1e9  # whole device, arena and frontier cache included
    dt = max_over_ranks(dist, torch, dt)
    # the same sweep once more with every binder-sponge launch running alone
    # (results identical; its trajectory is the timed sweep's): the sponge
    # kernels' and the level kernel's own rates, beside the co-running ones
    timing_alone = None
    if getattr(args, "standalone", 1):
        m.set_serial_sponges(True)
        timing_alone = []
        step(None, timing_alone)
        m.set_serial_sponges(False)
        m.synchronize()
        if dist:
            dist.barrier()

    # units: reports x candidates of both aggregators at every level, over the job
    # (the ranks' shares sum to the job; a virtual rank reports its own share)
    n_units = n_rep if vr > 1 else (n_job if split else n_rep * world)
    units = sum(2 * n_units * len(lv.prefixes) for tr in traces for lv in tr)
    # plaintext check: the heavy hitters are exactly the attributes whose total
    # weight reaches the threshold (every prefix of one has at least its
    # weight), and sampled levels' aggregates equal the plaintext prefix sums
    # (talks/func.py:49-80); with the job's reports on this rank
    plain_ok = None
    if alphas_job is not None:
        keys, inv = np.unique(alphas_job, axis=0, return_inverse=True)
        tot = np.bincount(inv.ravel(), weights=w_job)
        want = set(bytes(k) for (k, t) in zip(keys, tot) if t >= threshold)
        got = set(np.packbits(np.array(p, dtype=bool)).tobytes() for p in hh)
        plain_ok = got == want
        for lv in traces[0][::max(1, len(traces[0]) // 6)]:
            if lv.prefixes and lv.level < 64:
                (_cnt, ws) = prefix_sums(alphas_job, w_job, lv.level, lv.prefixes)
                plain_ok = plain_ok and ws.tolist() == list(lv.agg_result)
    # node evaluations actually performed: a level served from the frontier cache evaluates
    # only its new tree level (both children of every distinct length-L prefix)
    hit = set(cached_levels)
    nodes = 0
    for lv in traces[0]:
        if not lv.prefixes:
            continue
        if lv.level in hit:
            nodes += 2 * len(set(p[:lv.level] for p in lv.prefixes))
        else:
            nodes += m.tree_stats((lv.level, tuple(lv.prefixes), lv.level == 0))[0]
    nodes *= 2 * n_rep * steps  # both aggregators, this rank
    aes_per_node = 1 + (16 + m.VALUE_LEN * m.field.ENCODED_SIZE + 15) // 16
    dom_ops = aes_per_node * AES_BLOCK_OPS + 2 * m.VALUE_LEN * FIELD_ADD_OPS + KECCAK_OPS
    dom_ms = sum(t[0] + t[2] for t in timing)
    n_launch = sum(t[1] for t in timing)
    achieved = nodes * dom_ops / (dom_ms / 1e3) / 1e12 if dom_ms > 0 else 0.0
    # per level of the first timed sweep (both aggregators): where the level
    # kernel's time goes.  A frontier-cache hit also recomputes each parent's
    # convert stream (its seed and payload, aes_per_node - 1 blocks) from the
    # cached convert seed: executed, but not algorithmic work (SURVEY §8d
    # counts a minimal evaluation), so `frac` leaves it out and
    # `frac_executed` counts it
    per_level = {"level": [], "hit": [], "candidates": [], "nodes_per_report": [], "level_kernel_ms": [],
                 "absorb_ms": [], "frac": [], "frac_executed": []}
    rec_ops = 0
    ab_perms = 0.0  # binder-sponge Keccak-p of the first timed sweep, both aggregators
    wl_b = m.VALUE_LEN * m.field.ENCODED_SIZE
    ti = 0
    for lv in traces[0]:
        if not lv.prefixes or ti + 1 >= len(timing):
            continue
        hit_l = lv.level in hit
        parents = len(set(p[:lv.level] for p in lv.prefixes)) if lv.level > 0 else 1
        nl = 2 * parents if hit_l else m.tree_stats((lv.level, tuple(lv.prefixes), lv.level == 0))[0]
        ms = timing[ti][0] + timing[ti][2] + timing[ti + 1][0] + timing[ti + 1][2]
        per_level["level"].append(lv.level)
        per_level["hit"].append(hit_l)
        per_level["candidates"].append(len(lv.prefixes))
        per_level["nodes_per_report"].append(nl)
        per_level["level_kernel_ms"].append(round(ms, 2))
        per_level["absorb_ms"].append(round(timing[ti][4] + timing[ti + 1][4], 2))
        per_level["frac"].append(round(2 * n_rep * nl * dom_ops / (ms / 1e3) / 1e12 / VALU_PEAK_TOPS, 3)
                                 if ms > 0 else None)
        rec_l = 2 * n_rep * parents * (aes_per_node - 1) * AES_BLOCK_OPS if hit_l else 0
        per_level["frac_executed"].append(
            round((2 * n_rep * nl * dom_ops + rec_l) / (ms / 1e3) / 1e12 / VALU_PEAK_TOPS, 3) if ms > 0 else None)
        if hit_l:
            rec_ops += 2 * n_rep * parents * (aes_per_node - 1) * AES_BLOCK_OPS
            # a hit absorbs its new level's proofs and level L-1's parents' differences
            ab_perms += 2 * n_rep * (32 * nl + wl_b * parents) / 168.0
        else:
            ab_perms += 2 * n_rep * (32 * nl + wl_b * (nl // 2 - 1)) / 168.0
        ti += 2
    rec_ops *= steps
    achieved_exec = (nodes * dom_ops + rec_ops) / (dom_ms / 1e3) / 1e12 if dom_ms > 0 else 0.0
    widths = [len(lv.prefixes) for lv in traces[0]]
    if split:
        scaling, workload = "strong", "%s; the job's %d reports split %d-way (%d on this rank)" % (
            cfg["desc"], n_job, world, n_rep)
    elif vr > 1:
        scaling, workload = "strong", "%s; rank 0 of a virtual %d-way split of %d reports (%d reports), the other "             "ranks' aggregates added in plaintext" % (cfg["desc"], vr, n_job, n_rep)
    else:
        scaling, workload = "weak", "%s, %d reports per rank" % (cfg["desc"], n_rep)
    out = {
        "metric": METRIC,
        "value": units / dt,
        "unit": "report*prefix/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": warmup,
        "ms_per_step": dt * 1e3 / steps,
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic",
        "config": {
            "workload": workload,
            "reports_per_step": n_units,
            "reports_this_rank": n_rep,
            "job_reports": n_job,
            "threshold": thresholds["default"],
            "levels": len(traces[0]),
            "max_candidates_per_level": max(widths),
            "sum_candidates_over_levels": sum(widths),
            "heavy_hitters": len(hh),
            "heavy_hitters_equal_plaintext": plain_ok,
            "frontier_cache": bool(args.frontier_cache),
            "levels_evaluated_from_cache": len(cached_levels),
            "node_evals_per_step": nodes // steps,
            "field": "Field64" if m.field.ENCODED_SIZE == 8 else "Field128",
            "shard_s": shard_s,
            "hbm_used_gb_after": hbm_used,
            "parallelism": "reports split %d-way, per-level agg-share all-gather + GPU fold" % world,
        },
        "comm": comm,
        "roofline": {
            "kernel": "k_eval_aes<F64> (+ node-proof waves, + k_node_proof for the last level)",
            "bound": "valu",
            "achieved": achieved,
            "peak": VALU_PEAK_TOPS,
            "unit": "Tops/s (int32)",
            "frac": achieved / VALU_PEAK_TOPS,
            "peak_measured": VALU_MEASURED_TOPS,
            "frac_of_measured_peak": achieved / VALU_MEASURED_TOPS,
            "traffic": None,
            "launches": n_launch,
            "avg_launch_ms": dom_ms / max(n_launch, 1),
            "ops_per_node": dom_ops,
            "frac_executed": achieved_exec / VALU_PEAK_TOPS,
            "frac_executed_note": "also counts the frontier-cache hits' parent convert-stream recompute (%d AES "
                                  "blocks per parent), which the cache trades for 20 B per cached node" % (
                                      aes_per_node - 1),
        },
        "per_level": per_level,
        "roofline_absorb": {
            "kernel": "k_absorb (1 lane per sponge, chunks >= 65,536 reports) / k_absorb_pair",
            "keccak_perms_per_sweep": ab_perms,
            "achieved": ab_perms * KECCAK_OPS / (sum(per_level["absorb_ms"]) / 1e3) / 1e12
            if sum(per_level["absorb_ms"]) > 0 else 0.0,
            "peak": VALU_PEAK_TOPS, "unit": "Tops/s (int32)",
            "frac": (ab_perms * KECCAK_OPS / (sum(per_level["absorb_ms"]) / 1e3) / 1e12 / VALU_PEAK_TOPS)
            if sum(per_level["absorb_ms"]) > 0 else 0.0,
            "note": "Keccak-p of the one-hot and payload binders over the summed duration of the sponge launches "
                    "(which run beside the level kernels in the timed sweep; `standalone`: alone)",
        },
        "breakdown_ms_per_step": {
            # every algorithmic op of the AES and Keccak kernels (level kernels: nodes x ops per
            # node; binder sponges: their Keccak-p) over the sweep's wall time (host gaps included)
            # (this rank's work over the job's wall time: per-GPU utilisation)
            "frac_int_valu_whole_sweep": (nodes * dom_ops + ab_perms * steps * KECCAK_OPS) / dt / 1e12
            / VALU_PEAK_TOPS,
            "eval_aes_plus_proofs": dom_ms / steps,
            "absorb": sum(t[4] for t in timing) / steps,
            "prep_init_total": sum(t[6] for t in timing) / steps,
            "wall_this_rank": dt_local * 1e3 / steps,
            "host_phases_ms": {k: v * 1e3 / steps for (k, v) in phases.items()},
        },
    }
    if timing_alone:
        ab_alone_ms = sum(x[4] for x in timing_alone)
        lk_alone_ms = sum(x[0] + x[2] for x in timing_alone)
        nodes_one = nodes // steps
        out["roofline_absorb"]["standalone"] = {
            "frac": ab_perms * KECCAK_OPS / (ab_alone_ms / 1e3) / 1e12 / VALU_PEAK_TOPS if ab_alone_ms > 0 else None,
            "sponge_ms": ab_alone_ms,
            "level_kernel_frac_alone": nodes_one * dom_ops / (lk_alone_ms / 1e3) / 1e12 / VALU_PEAK_TOPS
            if lk_alone_ms > 0 else None,
            "level_kernel_ms_alone": lk_alone_ms,
            "what": "one more sweep (same trajectory) with every binder-sponge launch running alone "
                    "(Mastic.set_serial_sponges: the level kernels wait for it); frac = the same Keccak-p over the "
                    "summed sponge-launch durations; level_kernel_frac_alone = the level kernel without sponges "
                    "beside it",
        }
    out["rates"] = {
        "with_frontier_cache" if args.frontier_cache else "spec_literal": units / dt,
        "unit": "report*prefix/s (both aggregators' prep_init + decide + fold per level, whole sweep)",
    }
    if args.frontier_cache and cfg.get("spec_sample"):
        # spec-literal rate: every level's prep_init evaluates
        # its whole tree, as the reference does; the same per-level body on a
        # bounded sample of the reports with the timed sweep's candidate lists
        m.set_frontier_cache(False)
        ns = min(cfg["spec_sample"], n_rep)
        sample = reps.view(0, ns)
        lvls = [lv for lv in traces[0] if lv.prefixes][::cfg.get("spec_every", 1)]
        m.synchronize()
        if dist:
            dist.barrier()
        t2 = time.perf_counter()
        su = 0
        for lv in lvls:
            enc = m.encode_agg_param((lv.level, tuple(lv.prefixes), lv.level == 0))
            for agg_id in range(2):
                m.prep_init_device(sample, vk, ctx, agg_id, enc)
            sh = [m.prep_result(sample, agg_id, enc) for agg_id in range(2)]
            (_msgs, valid) = m.decide_batch(ctx, enc, sh[0][0], sh[1][0])
            for agg_id in range(2):
                m.aggregate_device(agg_id, enc, valid == 1, raw=True)
            su += 2 * ns * len(lv.prefixes)
        m.synchronize()
        if dist:
            dist.barrier()
        t_spec = time.perf_counter() - t2
        t_spec = max_over_ranks(dist, torch, t_spec)
        out["rates"]["spec_literal_sampled"] = su * world / t_spec
        out["rates"]["spec_literal_sample"] = "%d reports per rank, %d of the sweep's levels (every %d-th), its " \
            "candidate lists, frontier cache off: each level evaluates its whole tree" % (
                ns, len(lvls), cfg.get("spec_every", 1))
        del sample
    if rank == 0 and world == 1 and do_cpu:
        # oracle prep_init (leader) of one report per process at 8 levels spread over the sweep,
        # with the GPU trace's candidate prefixes: a bounded sample of the same workload
        lvls = [lv for lv in traces[0] if lv.prefixes and lv.level in check_levels]
        (rn, pub, in0, _in1) = reps.view(0, procs).download()
        ps, isz = m.sizes.public_share_size, m.sizes.input_share_size[0]
        spec = (cfg["circuit"], cfg["kw"])
        jobs = []
        for i in range(procs):
            for lv in lvls:
                enc_ap = m.encode_agg_param((lv.level, tuple(lv.prefixes), lv.level == 0))
                jobs.append((spec, enc_ap, rn[16 * i:16 * (i + 1)], pub[ps * i:ps * (i + 1)],
                             in0[isz * i:isz * (i + 1)], vk, ctx, 0))
        wall, res = cpu_baseline(jobs, procs)
        # the same reports at the same levels through the GPU path (leader
        # prep_init of the resident reports with the sweep's candidate lists):
        # the oracle replays part of the timed workload bit for bit
        m.set_frontier_cache(False)
        gpu_ps = []
        for lv in lvls:
            enc_ap = m.encode_agg_param((lv.level, tuple(lv.prefixes), lv.level == 0))
            (gps, _js, _o, _st) = m.prep_init_batch(vk, ctx, 0, enc_ap, rn[:16 * procs], pub[:ps * procs],
                                                    in0[:isz * procs], want_out_shares=False)
            psz = m.prep_share_size(lv.level == 0)
            gpu_ps.append([gps[psz * i:psz * (i + 1)] for i in range(procs)])
        parity = all(res[i * len(lvls) + k][1] == gpu_ps[k][i] for i in range(procs) for k in range(len(lvls)))
        if captured:
            # the timed path itself (frontier cache on, sponges resumed from
            # cached states at the hit levels) against the oracle
            out["cpu_parity_cached"] = all(
                lv.level in captured and res[i * len(lvls) + k][1] == captured[lv.level][i]
                for i in range(procs) for (k, lv) in enumerate(lvls))
            out["cpu_parity_cached_levels"] = {
                "levels": [lv.level for lv in lvls], "of_which_frontier_cache_hits": captured_hits,
                "reports": procs,
                "what": "leader prep shares of the warmup sweep (frontier cache on) vs the oracle's spec-literal "
                        "prep_init of the same reports and candidate lists"}
        cu = procs * sum(len(lv.prefixes) for lv in lvls)
        out["cpu_baseline"] = {
            "value": cu / wall,
            "unit": "report*prefix/s",
            "cores": procs,
            "kind": "port",
            "single_process_value": cu / sum(r[0] for r in res),
            "sample": "%d reports (one per process, spawn pool of %d) x leader prep_init at levels %s of the "
                      "sweep with the GPU run's candidate prefixes; poc-faithful Python oracle with C "
                      "AES/TurboSHAKE; GPU/CPU prep shares bit-identical: %s" % (
                          procs, procs, [lv.level for lv in lvls], parity),
        }
        out["cpu_baseline"].update(cpu_host_info())
        out["cpu_parity"] = parity
        # the native multithreaded CPU point at the same levels, on as many
        # reports as fill a ~10 s sample of its C part (sized from a first
        # pass over 8 reports per thread, which is not counted)
        sys.path.insert(0, ROOT)
        from oracle.native import has_aesni, prep_init_native
        o = _oracle_mastic(cfg["circuit"], cfg["kw"])
        nn = min(8 * procs, reps.n)
        (nrn, npub, nin0, _nin1) = reps.view(0, nn).download()
        cal = {}
        for lv in lvls:
            prep_init_native(o, vk, ctx, 0, (lv.level, tuple(lv.prefixes), lv.level == 0), nrn, npub, nin0, procs,
                             times=cal)
        # (capped at 8,192 reports: the level-0 weight check runs the FLP query in Python, ~1 ms each)
        nn = int(min(reps.n, 8192, max(nn, nn * 10.0 / max(cal["native_c_s"], 1e-3))))
        (nrn, npub, nin0, _nin1) = reps.view(0, nn).download()
        nat_t, nat_u, nat_ok, nat_times = 0.0, 0, True, {}
        for lv in lvls:
            ap = (lv.level, tuple(lv.prefixes), lv.level == 0)
            t = time.perf_counter()
            (nsh, _o) = prep_init_native(o, vk, ctx, 0, ap, nrn, npub, nin0, procs, times=nat_times)
            nat_t += time.perf_counter() - t
            nat_u += nn * len(lv.prefixes)
            enc_ap = m.encode_agg_param(ap)
            (gps, _js, _o2, _st) = m.prep_init_batch(vk, ctx, 0, enc_ap, nrn, npub, nin0, want_out_shares=False)
            psz = m.prep_share_size(ap[2])
            nat_ok = nat_ok and all(gps[psz * i:psz * (i + 1)] == nsh[i] for i in range(nn))
        out["cpu_baseline"]["native"] = {
            "value": nat_u / nat_times["native_c_s"], "unit": "report*prefix/s", "cores": procs, "kind": "port",
            "value_with_python_flp": nat_u / nat_t,
            "impl": "native C (oracle/native_prep.c): AES-NI %s, 64-bit Keccak-p, pthreads; FLP query in the "
                    "Python oracle (timed separately)" % ("on" if has_aesni() else "off"),
            "sample": "%d reports x leader prep_init at levels %s (the sweep's candidate lists) on %d threads, "
                      "C part %.2f s (+ Python FLP %.2f s); GPU/CPU prep shares bit-identical: %s" % (
                          nn, [lv.level for lv in lvls], procs, nat_times["native_c_s"], nat_times["flp_py_s"],
                          nat_ok),
            "parity": nat_ok,
        }
    del reps
    if rank == 0 and emit:
        if args.lib:
            out["library"] = "alternate build (A/B only): " + args.lib
        print(json.dumps(out))
    if dist and emit:
        dist.destroy_process_group()
    return out


# ---------------------------------------------------------------- launch
def launch_command(argv, n_gpus, port):
    """The torch.distributed.run command that re-runs this script with one
    rank per GPU (as the driver launches it for N > 1)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n_gpus),
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)


def maybe_relaunch(args, argv):
    """--gpus N without a launcher: start N ranks through torch.distributed.run
    as a child process (before anything touches the GPU) and return its exit
    code; under a launcher, --gpus must equal WORLD_SIZE."""
    world = os.environ.get("WORLD_SIZE")
    if world is None:
        if args.gpus > 1:
            import socket
            import subprocess
            s = socket.socket()
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
            s.close()
            return subprocess.call(launch_command(argv, args.gpus, port))
        return None
    if int(world) != args.gpus:
        raise SystemExit("bench.py: --gpus %d but WORLD_SIZE=%s (launch one rank per GPU)" % (args.gpus, world))
    return None


def cpu_pool_size(requested):
    """Worker processes for the CPU baseline: the host's CPUs this process may
    use (affinity), capped by OMP_NUM_THREADS when the box sets it (its CPU
    share; os.cpu_count() there counts the whole machine) and by --cpu-procs."""
    n = os.cpu_count() or 1
    try:
        n = min(n, len(os.sched_getaffinity(0)))
    except AttributeError:
        pass
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    try:  # cgroup v2 CPU quota
        (q, period) = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(int(q) / int(period))))
    except (OSError, ValueError):
        pass
    if requested > 0:
        n = min(n, requested)
    return max(1, n)


def cpu_host_info():
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = None
    quota = None
    try:  # cgroup v2 CPU quota: the CPUs this lease is granted (e.g. "1600000 100000" = 16)
        (q, period) = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        quota = None if q == "max" else int(q) / int(period)
    except (OSError, ValueError):
        pass
    return {"cpu_model": model, "host_cpu_count": os.cpu_count(), "affinity_cpus": aff,
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS"), "cgroup_cpu_quota": quota,
            "cpu_share_note": "pool = min(affinity, OMP_NUM_THREADS, cgroup quota): the CPUs this lease grants "
                              "(the GPU box sets OMP_NUM_THREADS to its CPU share; os.cpu_count() counts the "
                              "whole machine)"}


# ---------------------------------------------------------------- main
def main():
    args = parse()
    if args.launch_probe:  # tests: report the rank layout and exit (no GPU)
        # one write per line (atomic on a pipe): the ranks share the launcher's stdout
        os.write(1, (json.dumps({"rank": int(os.environ.get("RANK", "0")),
                                 "world": int(os.environ.get("WORLD_SIZE", "1")), "gpus": args.gpus}) + "\n").encode())
        return 0
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    dist = None
    # under torch.distributed.run (the driver's N > 1 launch; also at one rank) the ranks form a
    # process group, even of one
    if "WORLD_SIZE" in os.environ:
        import torch.distributed as dist
        # The control plane (barriers, the max over ranks, the communicator id)
        # runs over gloo; the data path's all-gather of agg shares runs on the
        # library's own RCCL communicator (mastic_comm_init, one per Mastic
        # ctx).  MASTIC_BENCH_BACKEND=gloo / MASTIC_BENCH_DEVICE=0: a rehearsal
        # of the N-rank run with every rank on one GPU (tests; RCCL refuses two
        # ranks on one device), whose shares then move through gloo.
        backend = os.environ.get("MASTIC_BENCH_BACKEND", "nccl")
        local = int(os.environ.get("MASTIC_BENCH_DEVICE", local))
        torch.cuda.set_device(local)
        dist.init_process_group("gloo")
        args.lib_comm = backend == "nccl"
    if args.lib:
        from mastic_amd import _lib
        _lib.load(args.lib)
    from mastic_amd import Mastic
    from mastic_amd.merge import aggregate_to_tensor, fold_on_gpu, merge_agg_shares

    cfg = CONFIGS[args.config]
    lib_comm = getattr(args, "lib_comm", False)
    n_rep = args.reports or cfg["reports"]
    if cfg.get("sweep"):
        run_sweep(args, cfg, world, rank, local, dist, torch)
        return 0
    n_pre = args.prefixes or cfg["prefixes"]
    n_total = max(args.total_reports or cfg.get("total", n_rep), n_rep)
    n_job = n_total * world
    if args.split:
        # --split: the resident reports are the JOB's, divided over the ranks
        # (the full_job leg is then strong scaling)
        n_job = n_total
        (lo, hi) = split_bounds(n_job, world)[rank]
        if hi - lo < 1:
            raise SystemExit("--split: %d resident reports leave rank %d none" % (n_job, rank))
        # a rank's steps run within its own share of the job, so value (job
        # reports x prefixes / wall) counts exactly the reports processed
        n_rep = min(n_rep, hi - lo)
        n_total = hi - lo
    kw = dict(cfg["kw"])
    bits = kw.pop("bits")
    m = Mastic(bits, cfg["circuit"], device=local, **kw)
    if args.memory_budget_gb:
        m.set_memory_budget(int(args.memory_budget_gb * 2 ** 30))
    if lib_comm:
        lib_comm = lib_comm_init(m, dist, world, rank)
    comm = comm_record(dist, world, rank, lib_comm, m)
    ctx = b"mastic-mi355x-bench"
    seed = 0x4D41 + int(args.config[1])
    # distinct reports resident in HBM: all of them, or a pool the job cycles through
    n_res = n_total
    if args.pool_reports and args.pool_reports < n_total:
        n_res = max(n_rep, args.pool_reports // n_rep * n_rep)
    attrs, alpha_b, betas, nonces, rands = synth(m, cfg, rank, n_res, n_pre, seed)
    vk = np.random.default_rng(0x4D41).integers(0, 256, size=32, dtype=np.uint8).tobytes()
    enc_ap = agg_param_bytes(bits - 1, attrs)
    # the whole job's reports resident in HBM (GPU shard); each step runs the
    # hot path over the next distinct n_rep-report slice of them
    t_sh = time.perf_counter()
    reps_all = m.reports_shard(ctx, alpha_b, betas, nonces, rands)
    m.synchronize()
    shard_s = time.perf_counter() - t_sh
    del alpha_b, betas, nonces, rands
    slices = [reps_all.view(i * n_rep, n_rep) for i in range(n_res // n_rep)]
    (nodes, interior, _maxl) = m.tree_stats(enc_ap)
    n_elems = len(attrs) * (1 + m.OUTPUT_LEN)

    def step(reps):
        m.prep_init_device(reps, vk, ctx, args.agg_id, enc_ap)
        if dist is not None and lib_comm:
            # agg share folded into HBM, all-gathered over the library's RCCL
            # communicator and merged mod p on the GPU, in one call
            return m.aggregate_merged((args.agg_id,), n_elems)
        if world > 1:
            return merge_agg_shares(m, aggregate_to_tensor(m, args.agg_id, n_elems), dist)
        return m.aggregate_device(args.agg_id, enc_ap, raw=True)

    for i in range(args.warmup):
        step(slices[-1 - (i % len(slices))])
    m.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    aes_ms = proof_ms = absorb_ms = total_ms = 0.0
    n_launch = 0
    for k in range(args.steps):
        step(slices[k % len(slices)])
        (ea, na_, ep, _np, eb, _nb, t) = m.last_timing3()
        aes_ms += ea
        proof_ms += ep
        absorb_ms += eb
        n_launch += na_
        total_ms += t
    m.synchronize()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    dt = time.perf_counter() - t0
    dt = max_over_ranks(dist, torch, dt)

    alone = None
    if getattr(args, "standalone", 1):
        # one more step with every binder-sponge launch running alone (results
        # identical): the sponge kernel's and the level kernel's own rates
        m.set_serial_sponges(True)
        step(slices[0])
        alone = m.last_timing3()
        m.set_serial_sponges(False)
        m.synchronize()
        if dist:
            dist.barrier()
    units = n_rep * len(attrs) * args.steps * world
    value = units / dt
    # roofline of the dominant kernel: algorithmic int32 ops (fixed convention).
    # k_eval_aes runs each level's AES (extend, convert: 1 + ceil(VL*ENC/16) blocks, payload
    # adds) and, in its proof waves, the previous level's node proofs (one Keccak-p per node);
    # the last level's proofs run in k_node_proof, so the pair is timed together.
    aes_per_node = 1 + (16 + m.VALUE_LEN * m.field.ENCODED_SIZE + 15) // 16
    aes_ops_node = aes_per_node * AES_BLOCK_OPS + 2 * m.VALUE_LEN * FIELD_ADD_OPS
    node_units = nodes * n_rep * args.steps
    fname = "F64" if m.field.ENCODED_SIZE == 8 else "F128"
    dom = "k_eval_aes<%s> (+ node-proof waves, + k_node_proof for the last level)" % fname
    dom_ms = aes_ms + proof_ms
    dom_ops = aes_ops_node + KECCAK_OPS
    achieved = node_units * dom_ops / (dom_ms / 1e3) / 1e12 if dom_ms > 0 else 0.0
    # binder sponges: one-hot 32 B/node, payload VL*ENC B/interior node
    absorb_perms = (32 * nodes + m.VALUE_LEN * m.field.ENCODED_SIZE * interior) / 168.0
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "report*prefix/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic",
        "config": {
            "workload": "%s, %d reports resident per rank, each step a distinct %d-report slice x %d "
                        "prefixes, weight check, agg_id %d" % (cfg["desc"], n_total, n_rep, len(attrs), args.agg_id),
            "reports_per_step": n_rep * world,
            "prefixes": len(attrs),
            "nodes_per_report": nodes,
            "work_bytes_per_report": m.work_bytes(enc_ap),
            "field": "Field64" if fname == "F64" else "Field128",
            "parallelism": "reports sharded %d-way" % world,
        },
        "comm": comm,
        "roofline": {
            "kernel": dom,
            "bound": "valu",
            "achieved": achieved,
            "peak": VALU_PEAK_TOPS,
            "unit": "Tops/s (int32)",
            "frac": achieved / VALU_PEAK_TOPS,
            "peak_measured": VALU_MEASURED_TOPS,
            "frac_of_measured_peak": achieved / VALU_MEASURED_TOPS,
            "traffic": None,
            "launches": n_launch,
            "avg_launch_ms": dom_ms / max(n_launch, 1),
            "ops_per_node": dom_ops,
        },
        "breakdown_ms_per_step": {
            "eval_aes": aes_ms / args.steps,
            "node_proof_last_level": proof_ms / args.steps,
            "absorb": absorb_ms / args.steps,
            "prep_init_total": total_ms / args.steps,
            "frac_int_valu_whole_step": (node_units * (aes_ops_node + KECCAK_OPS) + absorb_perms * n_rep *
                                         args.steps * KECCAK_OPS) / (dt * 1e12) / VALU_PEAK_TOPS,
            "absorb_keccak_perms_per_report": absorb_perms,
        },
    }
    # the binder sponges' own roofline (verdict r04 item 4): their Keccak-p per
    # step under the fixed convention over the summed duration of their launches
    # (latency-bound chains at this batch size: the launches stay resident
    # beside the level kernel for most of the step)
    ab_perms = absorb_perms * n_rep * args.steps
    ab_ach = ab_perms * KECCAK_OPS / (absorb_ms / 1e3) / 1e12 if absorb_ms > 0 else 0.0
    standalone = None
    if alone is not None:
        (a_ea, _a_na, a_ep, _a_np, a_eb, _a_nb, _a_t) = alone
        standalone = {
            "frac": absorb_perms * n_rep * KECCAK_OPS / (a_eb / 1e3) / 1e12 / VALU_PEAK_TOPS if a_eb > 0 else None,
            "sponge_ms": a_eb,
            "level_kernel_frac_alone": nodes * n_rep * (aes_ops_node + KECCAK_OPS) / ((a_ea + a_ep) / 1e3) / 1e12
            / VALU_PEAK_TOPS if a_ea + a_ep > 0 else None,
            "level_kernel_ms_alone": a_ea + a_ep,
            "what": "one more step with every binder-sponge launch running alone (Mastic.set_serial_sponges: the "
                    "level kernels wait for it); frac = the step's Keccak-p over the summed sponge-launch "
                    "durations; at this batch the sponges are one dependent chain per report (%d waves for the "
                    "chip's 1,024 SIMDs), i.e. latency-bound, and hidden under the level kernel in the timed "
                    "steps" % ((n_rep * 2 * 2 + 63) // 64),
        }
    out["roofline_absorb"] = {
        "standalone": standalone,
        "kernel": "k_absorb_pair (2 lanes per sponge)" if n_rep < 65536 else "k_absorb (1 lane per sponge)",
        "keccak_perms_per_report": absorb_perms,
        "achieved": ab_ach, "peak": VALU_PEAK_TOPS, "unit": "Tops/s (int32)", "frac": ab_ach / VALU_PEAK_TOPS,
        "ms_per_step": absorb_ms / args.steps,
        "note": "one-hot 32 B per node + payload VL*ENC B per interior node, / 168 B per Keccak-p[1600,12] "
                "(3,720 ops); the timed steps run the sponges beside the level kernel, so `frac` is their share "
                "of the step's VALU; `standalone` times them alone",
    }
    # HBM bytes per launch of the dominant kernel from the PMC passes (profiles/eval_traffic.json),
    # when they were measured at this exact workload
    traffic_file = os.path.join(ROOT, "profiles", "eval_traffic.json")
    if os.path.exists(traffic_file):
        same = [tr for tr in json.load(open(traffic_file)).get("entries", [])
                if tr["config"] == args.config and tr["prefixes"] == len(attrs)]
        exact = [tr for tr in same if tr["reports"] == n_rep]
        if exact or same:
            # the level kernel moves a fixed number of bytes per report-node, so a PMC pass at another
            # batch size scales linearly; the line says which one it is
            tr = exact[0] if exact else min(same, key=lambda e: abs(e["reports"] - n_rep))
            scale = n_rep / tr["reports"]
            out["roofline"]["traffic"] = tr["hbm_bytes_per_launch"] * scale
            out["roofline"]["traffic_unit"] = "bytes per launch"
            out["roofline"]["traffic_per_step"] = (tr["hbm_read_bytes_per_step"] + tr["hbm_write_bytes_per_step"]) * scale
            out["roofline"]["traffic_source"] = (
                "PMC FETCH_SIZE/WRITE_SIZE at this batch size" if exact else
                "PMC FETCH_SIZE/WRITE_SIZE at %d reports per step, scaled by reports" % tr["reports"])
    # HBM bytes per step, two references (DESIGN.md §4 "HBM traffic"): SURVEY §8d's
    # algorithmic bytes (inputs and outputs only: correction words, input share,
    # prep share) and the floor of the level-synchronous schedule, whose level
    # buffers (child seeds, proofs, frontier payloads, payload differences) must
    # round-trip HBM because the BFS-ordered binders need a whole level at once
    wl_b = m.VALUE_LEN * m.field.ENCODED_SIZE
    alg = (bits * (16 + wl_b + 32) + (2 * bits + 7) // 8 + m.sizes.input_share_size[args.agg_id]
           + m.prep_share_size(True))
    floor = nodes * (20 + 10 + 32 + 20) + interior * (3 * wl_b)
    out["roofline"]["algorithmic_bytes_per_step"] = alg * n_rep
    out["roofline"]["level_buffer_floor_per_step"] = floor * n_rep

    full = cfg.get("full_job", False) if args.full_job < 0 else bool(args.full_job)
    if full and n_total > n_rep:
        # the whole resident batch: every slice (the tail too) through prep_init
        # + fold, the per-slice agg shares merged on the GPU into the job's
        # agg share (out shares of 1M x 10k prefixes = 160 GB cannot be
        # materialised at once, so the job is necessarily sliced)
        bounds = [(i, min(n_rep, n_total - i)) for i in range(0, n_total, n_rep)]
        tail = reps_all.view(0, bounds[-1][1]) if bounds[-1][1] != n_rep else None
        m.synchronize()
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        parts = []
        t_last = t1
        for (j, (first, cnt)) in enumerate(bounds):
            v = slices[j % len(slices)] if cnt == n_rep else tail
            m.prep_init_device(v, vk, ctx, args.agg_id, enc_ap)
            parts.append(aggregate_to_tensor(m, args.agg_id, n_elems))
            if rank == 0 and time.perf_counter() - t_last > 30:  # progress for long jobs (C4/C5 sizes)
                t_last = time.perf_counter()
                print("[full_job] %d / %d slices, %.0f s" % (j + 1, len(bounds), t_last - t1), file=sys.stderr,
                      flush=True)
        job = fold_on_gpu(m, torch.cat(parts), len(parts), n_elems)
        if dist is not None and lib_comm:
            merged = torch.empty_like(job)
            m.allgather_fold(job.data_ptr(), 1, n_elems, merged.data_ptr(), torch.cuda.current_stream().cuda_stream)
            job = merged
        elif world > 1:
            job = merge_agg_shares(m, job, dist)
        m.synchronize()
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        wall = time.perf_counter() - t1
        wall = max_over_ranks(dist, torch, wall)
        out["full_job"] = {
            "reports_per_rank": n_total,
            "job_reports": n_job,
            "scaling": "strong" if args.split else "weak",
            "prefixes": len(attrs),
            "wall_s": wall,
            "value": n_job * len(attrs) / wall,
            "unit": "report*prefix/s",
            "slices": len(bounds),
            "distinct_reports_resident": n_res,
            "what": "prep_init (leader) + fold of every report of the job, %d slices of <= %d, slice agg shares "
                    "merged mod p on the GPU (mastic_fold_shares%s)" % (
                        len(bounds), n_rep, "; ranks' shares: mastic_allgather_fold" if lib_comm else ""),
        }
    out["config"]["resident_reports_per_rank"] = n_res
    (free_b, total_b) = torch.cuda.mem_get_info()
    out["config"]["hbm_used_gb_after"] = (total_b - free_b) / 1e9
    out["config"]["shard_s"] = shard_s

    if rank == 0 and world == 1 and args.cpu_baseline:
        procs = cpu_pool_size(args.cpu_procs)
        (rn, pub, in0, in1) = reps_all.view(0, procs).download()
        ps = m.sizes.public_share_size
        isz = m.sizes.input_share_size[args.agg_id]
        ins = in0 if args.agg_id == 0 else in1
        spec = (cfg["circuit"], cfg["kw"])
        jobs = [(spec, enc_ap, rn[16 * i:16 * (i + 1)], pub[ps * i:ps * (i + 1)], ins[isz * i:isz * (i + 1)], vk, ctx,
                 args.agg_id) for i in range(procs)]
        wall, res = cpu_baseline(jobs, procs)
        # the same reports through the GPU path: parity of the timed workload
        (gps, _js, _out, _st) = m.prep_init_batch(vk, ctx, args.agg_id, enc_ap, rn[:16 * procs],
                                                  pub[:ps * procs], ins[:isz * procs], want_out_shares=False)
        psz = m.prep_share_size(True)
        parity = all(gps[psz * i:psz * (i + 1)] == res[i][1] for i in range(procs))
        per_report = sum(r[0] for r in res) / len(res)
        out["cpu_baseline"] = {
            "value": procs * len(attrs) / wall,
            "unit": "report*prefix/s",
            "cores": procs,
            "kind": "port",
            "single_process_value": len(attrs) / per_report,
            "sample": "%d reports x %d prefixes, one per process (multiprocessing spawn pool of %d = the CPUs "
                      "this process may use); poc-faithful Python oracle with C AES/TurboSHAKE; %.1f s per "
                      "report per core; GPU/CPU prep shares bit-identical: %s"
                      % (procs, len(attrs), procs, per_report, parity),
        }
        out["cpu_baseline"].update(cpu_host_info())
        out["cpu_parity"] = parity
        nat = native_cpu_point(m, cfg, enc_ap, reps_all, vk, ctx, args.agg_id, procs, len(attrs))
        nat["gpu_over_native_cpu"] = out["value"] / nat["value"]
        out["cpu_baseline"]["native"] = nat
    ns = None
    if args.config == "c2" and args.north_star:
        # the north_star job (BASELINE.json): bit-exact prep_init + aggregate for
        # 1M reports x a full 32-bit prefix-level sweep, i.e. the reference's
        # heavy-hitters driver (examples.py:37-91) over the c2sweep population,
        # the job's 1M reports split over the ranks (strong scaling).  The C2
        # context (its ~120 GB work arena) is released first.
        import gc
        slices = reps_all = tail = v = None  # noqa: F841
        m = None
        gc.collect()
        ns_cfg = CONFIGS["c2sweep"]
        try:
            ns = run_sweep(args, ns_cfg, world, rank, local, dist, torch, split=True, steps=1, warmup=1,
                           n_job=args.north_star_reports or ns_cfg["reports"], emit=False)
        except Exception as e:  # keep the headline line; report the failed leg in it
            import traceback
            traceback.print_exc()
            ns = None
            out["north_star"] = {"error": "%s: %s" % (type(e).__name__, e)}
    if args.config == "c2" and args.north_star and ns is not None:
        nc = ns["config"]
        out["north_star"] = {
            "workload": nc["workload"],
            "job_reports": nc["job_reports"],
            "n_gpus": world,
            "scaling": "strong",
            "wall_s": ns["ms_per_step"] / 1e3,
            "value": ns["value"],
            "unit": ns["unit"],
            "rate_kind": "frontier cache on (both aggregators' prep_init + decide + fold per level)",
            "spec_literal_sampled": ns["rates"].get("spec_literal_sampled"),
            "spec_literal_sample": ns["rates"].get("spec_literal_sample"),
            "levels": nc["levels"],
            "levels_evaluated_from_cache": nc["levels_evaluated_from_cache"],
            "sum_candidates_over_levels": nc["sum_candidates_over_levels"],
            "threshold": nc["threshold"],
            "heavy_hitters": nc["heavy_hitters"],
            "heavy_hitters_equal_plaintext": nc["heavy_hitters_equal_plaintext"],
            "frac": ns["roofline"]["frac"],
            "frac_executed": ns["roofline"]["frac_executed"],
            "frac_int_valu_whole_sweep": ns["breakdown_ms_per_step"]["frac_int_valu_whole_sweep"],
            "roofline_absorb": ns["roofline_absorb"],
            "roofline_kernel": ns["roofline"]["kernel"],
            "per_level": ns["per_level"],
            "breakdown_ms": ns["breakdown_ms_per_step"],
            "comm": ns["comm"],
        }
        if "cpu_baseline" in ns:
            cb = ns["cpu_baseline"]
            out["north_star"]["cpu_baseline"] = {k: cb[k] for k in ("value", "unit", "cores", "kind",
                                                                    "single_process_value", "sample")}
            out["north_star"]["cpu_parity"] = ns.get("cpu_parity")
            out["north_star"]["cpu_parity_cached"] = ns.get("cpu_parity_cached")
            out["north_star"]["cpu_parity_cached_levels"] = ns.get("cpu_parity_cached_levels")
            # like for like: the CPU leg evaluates whole trees (spec-literal, no
            # cache), so the spec-literal GPU rate is the comparable one; the
            # cached rate's ratio is kept beside it, labelled
            lit = ns["rates"].get("spec_literal_sampled")
            if lit:
                out["north_star"]["speedup_spec_literal_vs_cpu_pool"] = lit / cb["value"]
                out["north_star"]["speedup_spec_literal_vs_cpu_core"] = lit / cb["single_process_value"]
            out["north_star"]["speedup_cached_vs_cpu_pool"] = ns["value"] / cb["value"]
            out["north_star"]["speedup_cached_vs_cpu_core"] = ns["value"] / cb["single_process_value"]
            if "native" in cb:
                out["north_star"]["cpu_baseline"]["native"] = cb["native"]
                if lit:
                    out["north_star"]["speedup_spec_literal_vs_native_cpu"] = lit / cb["native"]["value"]
    if rank == 0:
        if args.lib:
            out["library"] = "alternate build (A/B only): " + args.lib
        print(json.dumps(out))
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    _args = parse()
    _rc = maybe_relaunch(_args, sys.argv[1:])
    if _rc is not None:
        sys.exit(_rc)
    try:
        _rc = main() or 0
    except SystemExit as _e:
        if _e.code != 3:
            raise
        # a rank could not join the communicator (lib_comm_init): leave at once,
        # without the interpreter's teardown (an abandoned RCCL init may still
        # sit in its bootstrap on a library thread)
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(3)
    sys.exit(_rc)
