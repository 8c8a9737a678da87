"""Weighted heavy-hitters level sweep.

Mirrors the reference driver ``compute_heavy_hitters`` (poc/examples.py:37-91)
and ``get_threshold`` (poc/examples.py:26-34): walk the prefix tree level by
level, keep the children of every candidate whose aggregate reaches its
threshold, report the surviving full-length prefixes.

Differences from the reference loop, all in how the work is batched, not in
what is computed:
  * the reports are uploaded to HBM once and every level runs as one batched
    ``prep_init`` per aggregator (GPU), one ``decide_batch`` and one GPU fold
    per aggregator, instead of a Python loop over reports;
  * a report that fails verification at some level (the reference would raise
    at ``prep_shares_to_prep``) is dropped from that level's aggregate and
    from every later level, which is what a deployed aggregator does.  With
    only honest reports the output is identical to the reference's.
  * multi-GPU: every rank sweeps its own shard of
    the reports and passes ``merge`` (e.g. :func:`mastic_amd.merge.merge_field_shares`:
    RCCL all-gather + GPU mod-p fold), so each level's pruning decision is
    taken on the job-wide aggregate and all ranks walk the same frontier.
"""
import time

import numpy as np

from .vdaf import Mastic


def get_threshold(thresholds, prefix):
    """poc/examples.py:26-34: the threshold of the longest proper prefix of
    ``prefix`` listed in ``thresholds`` (the prefix itself excluded), else
    ``thresholds['default']``."""
    if len(thresholds) == 1:  # only 'default' (common case: skips the O(len) walk)
        return thresholds['default']
    for level in reversed(range(len(prefix) - 1)):
        if prefix[:level + 1] in thresholds:
            return thresholds[prefix[:level + 1]]
    return thresholds['default']


def _encode_reports(mastic: Mastic, reports):
    nonces = b"".join(r[0] for r in reports)
    pubs = b"".join(mastic.encode_public_share(r[1]) for r in reports)
    in0 = b"".join(mastic.test_vec_encode_input_share(r[2][0]) for r in reports)
    in1 = b"".join(mastic.test_vec_encode_input_share(r[2][1]) for r in reports)
    return (nonces, pubs, in0, in1)


def _child_packed(packed: bytes, level: int, bit: bool) -> bytes:
    """MSB-first packing (vidpf.py:33-39) of ``prefix + (bit,)`` from the
    packing of the length-``level`` ``prefix``."""
    if level % 8 == 0:
        packed += b"\x00"
    if bit:
        packed = packed[:-1] + bytes([packed[-1] | (0x80 >> (level % 8))])
    return packed


def _unshard_raw(mastic: Mastic, raw_shares, num_measurements):
    """``mastic.unshard`` (mastic.py:399-411) on encode_vec agg shares (the
    two aggregators', or one already-merged total), summed as integers mod p
    (same result, without a field object per share element; Field64 in
    numpy: 2^64 = 2^32 - 1 mod p)."""
    f = mastic.field
    enc = f.ENCODED_SIZE
    p = f.MODULUS
    k = 1 + mastic.OUTPUT_LEN
    if enc == 8:
        acc = None
        for r in raw_shares:
            v = np.frombuffer(r, dtype="<u8")
            if v.size and int(v.max()) >= p:
                raise ValueError("encoded element out of range")
            if acc is None:
                acc = v.copy()
                continue
            t = acc + v  # wraps mod 2^64
            t += (t < acc).astype(np.uint64) * np.uint64(0xFFFFFFFF)
            acc = np.where(t >= np.uint64(p), t - np.uint64(p), t)
        ints = [] if acc is None else acc.tolist()
    else:
        vecs = [[int.from_bytes(r[i:i + enc], "little") for i in range(0, len(r), enc)] for r in raw_shares]
        for v in vecs:
            if v and max(v) >= p:
                raise ValueError("encoded element out of range")
        ints = [sum(col) % p for col in zip(*vecs)]
    if mastic.circuit in ("Count", "Sum"):  # Mastic.decode_result: the one output element
        return ints[1::k]
    return [ints[i + 1:i + k] for i in range(0, len(ints), k)]


def _unpack_prefix(packed: bytes, length: int):
    """The tuple of bools of an MSB-first packed prefix (vidpf.py:33-39)."""
    return tuple(bool((packed[i // 8] >> (7 - i % 8)) & 1) for i in range(length))


def joint_rand_confirmed(msgs: bytes, jr_seeds_0: bytes, jr_seeds_1: bytes, n: int):
    """Per report: ``prep_next``'s joint-rand confirmation (mastic.py:369-375)
    for both aggregators -- the prep message (the seed recomputed from both
    parts, ``prep_shares_to_prep``) equals each aggregator's own seed."""
    if n == 0:
        return np.ones(0, dtype=bool)
    m = np.frombuffer(msgs, np.uint8, count=32 * n).reshape(n, 32)
    j0 = np.frombuffer(jr_seeds_0, np.uint8, count=32 * n).reshape(n, 32)
    j1 = np.frombuffer(jr_seeds_1, np.uint8, count=32 * n).reshape(n, 32)
    return (m == j0).all(axis=1) & (m == j1).all(axis=1)


class SweepLevel:
    """What one level of the sweep did (for callers that want the trace)."""

    def __init__(self, level, prefixes, agg_result, n_valid):
        self.level = level
        self.prefixes = prefixes
        self.agg_result = agg_result
        self.n_valid = n_valid


def compute_heavy_hitters(mastic: Mastic, ctx: bytes, thresholds, reports, verify_key: bytes = None,
                          trace=None, merge=None, timing=None, frontier_cache=None, cached_levels=None,
                          phase_times=None, level_hook=None):
    """poc/examples.py:37-91 on the GPU.

    ``reports`` is either the reference's list of
    ``(nonce, public_share, input_shares)`` tuples or a device-resident
    :class:`~mastic_amd.vdaf.Reports` batch holding both input shares
    (``Mastic.reports_shard`` / ``reports_upload``).  ``verify_key`` defaults
    to 16 fresh random bytes, as in the reference (examples.py:38).  If ``trace`` is a list, one
    :class:`SweepLevel` per level is appended to it.  ``merge`` maps this
    rank's agg share (list of field elements) to the job-wide one (all
    ranks call it at every level, in the same order).  If ``timing`` is a
    list, ``mastic.last_timing3()`` of every prep_init is appended to it.
    ``frontier_cache`` (True/False) switches the GPU frontier cache
    (``Mastic.set_frontier_cache``): each level then evaluates only its new
    tree level when the previous level's tree is unchanged; if
    ``cached_levels`` is a list, the levels that took that path are appended.
    If ``phase_times`` is a dict, the host wall time of each phase of a level
    (enqueueing both prep_inits, decide, aggregate + merge, unshard + prune) is
    accumulated into it (seconds).  ``level_hook(level, enc_agg_param, reports)``
    (if given) runs after each level's decide, while both aggregators' prep_init
    results of the level are still in HBM (e.g. to read sampled prep shares).
    """
    def clock(phase, t0):
        if phase_times is not None:
            t1 = time.perf_counter()
            phase_times[phase] = phase_times.get(phase, 0.0) + t1 - t0
            return t1
        return t0

    if frontier_cache is not None:
        mastic.set_frontier_cache(frontier_cache)
    if verify_key is None:
        import os
        verify_key = os.urandom(16)  # gen_rand(16), examples.py:38
    if isinstance(reports, (list, tuple)):
        if len(reports) == 0:
            dev = None
        else:
            dev = mastic.reports_upload(*_encode_reports(mastic, reports))
    else:
        dev = reports
    n = 0 if dev is None else dev.n
    alive = np.ones(n, dtype=bool)

    prefixes = [(False,), (True,)]
    fast = isinstance(mastic, Mastic)
    packed = [b"\x00", b"\x80"]  # MSB-first packings of ``prefixes`` (fast path)
    # lazy: the candidates only as packings (no bool tuples per level) when
    # nothing asks for the tuples: no trace, one default threshold, and no
    # merge that needs the level's candidates or field-object shares
    lazy = (fast and trace is None and len(thresholds) == 1
            and (merge is None or (hasattr(merge, "total") and not hasattr(merge, "begin_level"))))
    if lazy:
        prefixes = None
        th = thresholds['default']
    prev_agg_params = []
    heavy_hitters = []
    bits = mastic.vidpf.BITS
    for level in range(bits):
        n_cand = len(packed) if lazy else len(prefixes)
        agg_param = (level, () if lazy else tuple(prefixes), level == 0)
        assert mastic.is_valid(agg_param, prev_agg_params)
        # encoded once per level (the batch calls take the bytes); the fast
        # path extends the parents' packings instead of re-packing every bit
        if fast:
            enc = (level.to_bytes(2, "big") + n_cand.to_bytes(4, "big") + b"".join(packed)
                   + bytes([int(level == 0)]))
        else:
            enc = mastic.encode_agg_param(agg_param)

        device_merge = fast and merge is not None and hasattr(merge, "total")
        if merge is not None and hasattr(merge, "begin_level"):
            merge.begin_level(level, prefixes)  # merges that need the level's candidates
        n_elems = n_cand * (1 + mastic.OUTPUT_LEN) if device_merge else 0
        raw = agg_shares = None
        tp = time.perf_counter() if phase_times is not None else 0.0
        if n and n_cand:
            # both aggregators' prep_init are queued before either result is
            # fetched, so the host work of the second overlaps the GPU run of
            # the first (stream-ordered; results and timings are per agg_id)
            for agg_id in range(2):
                mastic.prep_init_device(dev, verify_key, ctx, agg_id, enc)
                if cached_levels is not None and agg_id == 0 and frontier_cache and mastic.last_prep_was_cached():
                    cached_levels.append(level)
            tp = clock("prep_init_enqueue", tp)
            if fast:
                # both aggregators' prep_shares_to_prep + prep_next on the GPU:
                # the prep shares stay in HBM, only the accept mask comes back
                (accept, _codes) = mastic.decide_results(ctx, n)
                alive &= accept == 1
                tp = clock("decide_wait", tp)
                if timing is not None:
                    for agg_id in range(2):
                        mastic.select_timing(agg_id)
                        timing.append(mastic.last_timing3())
                tp = time.perf_counter() if phase_times is not None else 0.0
            else:
                shares = []
                for agg_id in range(2):
                    shares.append(mastic.prep_result(dev, agg_id, enc))
                    if timing is not None:
                        timing.append(mastic.last_timing3())
                (msgs, valid) = mastic.decide_batch(ctx, enc, shares[0][0], shares[1][0])
                alive &= (valid == 1) & (shares[0][3] == 0) & (shares[1][3] == 0)
                if level == 0 and mastic.JOINT_RAND_LEN > 0:
                    # prep_next (mastic.py:364-377, called at examples.py:67): each
                    # aggregator's joint-rand seed must equal the prep message
                    alive &= joint_rand_confirmed(msgs, shares[0][1], shares[1][1], n)
            if level_hook is not None:
                level_hook(level, enc, dev)
            mask = alive.astype(np.uint8)
            if device_merge:
                # both shares folded, gathered and merged in HBM (one RCCL call)
                raw = [merge.total(n_elems, mask)]
            elif fast and merge is None:
                raw = [mastic.aggregate_device(agg_id, enc, mask, raw=True) for agg_id in range(2)]
            else:
                agg_shares = [mastic.aggregate_device(agg_id, enc, mask) for agg_id in range(2)]
        elif device_merge:
            raw = [merge.total(n_elems, have_results=False)]  # same collectives on every rank
        elif lazy:
            # no reports: agg_init's zeros for every candidate (the lazy agg
            # param carries no prefix tuples for agg_init to count)
            raw = [bytes(n_cand * (1 + mastic.OUTPUT_LEN) * mastic.field.ENCODED_SIZE)]
        else:
            agg_shares = [mastic.agg_init(agg_param) for _ in range(2)]
        tp = clock("aggregate_merge", tp)
        if raw is not None:
            agg_result = _unshard_raw(mastic, raw, int(alive.sum()))
        else:
            if merge is not None:
                agg_shares = [merge(a) for a in agg_shares]
            agg_result = mastic.unshard(agg_param, agg_shares, int(alive.sum()))
        prev_agg_params.append(agg_param)
        if trace is not None:
            trace.append(SweepLevel(level, list(prefixes), agg_result, int(alive.sum())))

        if lazy:
            if level < bits - 1:
                next_packed = []
                for (pk, count) in zip(packed, agg_result):
                    if count >= th:
                        next_packed.append(_child_packed(pk, level + 1, False))
                        next_packed.append(_child_packed(pk, level + 1, True))
                packed = next_packed
                clock("unshard_prune", tp)
            else:
                heavy_hitters = [_unpack_prefix(pk, bits) for (pk, count) in zip(packed, agg_result) if count >= th]
        elif level < bits - 1:
            next_prefixes = []
            next_packed = []
            for (i, (prefix, count)) in enumerate(zip(prefixes, agg_result)):
                if count >= get_threshold(thresholds, prefix):
                    next_prefixes.append(prefix + (False,))
                    next_prefixes.append(prefix + (True,))
                    if fast:
                        next_packed.append(_child_packed(packed[i], level + 1, False))
                        next_packed.append(_child_packed(packed[i], level + 1, True))
            prefixes = next_prefixes
            packed = next_packed
            clock("unshard_prune", tp)
        else:
            for (prefix, count) in zip(prefixes, agg_result):
                if count >= get_threshold(thresholds, prefix):
                    heavy_hitters.append(prefix)
    return heavy_hitters
