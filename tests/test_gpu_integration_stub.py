"""The reference-side binding (integration/poc/mastic_hip.py, INTEGRATION.md
§3) actually run: the file a poc maintainer would drop next to
``poc/mastic.py``, driven with poc-shaped ``Mastic`` objects.  ``/root/reference``
is not on the GPU box, so the poc-shaped restatement under ``oracle/`` stands
in for ``poc/mastic.py`` (same class names, attributes and wire encoders,
mastic.py:52-614); it encodes the inputs and runs the CPU steps the poc keeps
(prep_next, unshard), while prep_init, prep_shares_to_prep and the aggregation
fold go through the stub to the GPU.  Everything is checked against the
reference's golden vectors (tests/golden/, byte copies of test_vec/mastic)."""
import importlib.util
import json
import os

import pytest

from conftest import ROOT, golden_files

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def stub():
    from mastic_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.fail("libmastic_hip.so missing: build() was not run")
    spec = importlib.util.spec_from_file_location(
        "mastic_hip_stub", os.path.join(ROOT, "integration", "poc", "mastic_hip.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod, mod.load(_lib.LIB_PATH)


def _reports(m, tv, agg_id=None):
    """The report tuples a poc driver holds (examples.py:12-23): decoded objects."""
    return [(bytes.fromhex(r["nonce"]),
             m.vidpf.decode_public_share(bytes.fromhex(r["public_share"])),
             [m.decode_input_share(a, bytes.fromhex(r["input_shares"][a])) for a in range(2)])
            for r in tv["prep"]]


def _run_loop(gpu, m, vk, ctx, ap, reports):
    """examples.py:49-74 with the per-report calls replaced by the stub's
    batches: prep_init of both aggregators, prep_shares_to_prep, the poc's
    own prep_next, agg_update as the GPU fold, then the poc's unshard."""
    (states, shares) = ([], [])
    for agg_id in range(2):
        res = gpu.prep_init_batch(vk, ctx, agg_id, ap, [(r[0], r[1], r[2][agg_id]) for r in reports])
        states.append([st for (st, _sh) in res])
        shares.append([sh for (_st, sh) in res])
    (prep_msgs, failures) = gpu.prep_shares_to_prep_batch(ctx, ap, list(zip(shares[0], shares[1])))
    valid = []
    out_shares = [[], []]
    for i in range(len(reports)):
        ok = failures[i] is None
        if ok:
            try:
                for agg_id in range(2):
                    out_shares[agg_id].append(m.prep_next(ctx, states[agg_id][i], prep_msgs[i]))
            except Exception:
                ok = False
        valid.append(ok)
    agg_shares = [gpu.aggregate(agg_id, ap, valid) for agg_id in range(2)]
    agg_result = m.unshard(ap, agg_shares, sum(valid))
    return (states, shares, prep_msgs, failures, valid, out_shares, agg_shares, agg_result)


@pytest.mark.parametrize("path", golden_files(), ids=os.path.basename)
def test_stub_runs_the_poc_aggregator_loop(stub, path):
    """The whole per-level loop of examples.py:49-74 through the stub on a
    golden vector: prep shares, prep states (truncated out shares and
    joint-rand seeds, mastic.py:311-318), prep messages, out shares, agg
    shares and the agg result all equal the reference's vector."""
    from oracle import mastic as poc_mastic
    (mod, lib) = stub
    tv = json.load(open(path))
    m = poc_mastic.from_test_vec(tv)  # the poc-shaped Mastic the maintainer's code holds
    gpu = mod.MasticHip(lib, m)
    ctx = bytes.fromhex(tv["ctx"])
    vk = bytes.fromhex(tv["verify_key"])
    ap = m.decode_agg_param(bytes.fromhex(tv["agg_param"]))
    (states, shares, prep_msgs, failures, valid, out_shares, agg_shares, agg_result) = \
        _run_loop(gpu, m, vk, ctx, ap, _reports(m, tv))
    for (i, r) in enumerate(tv["prep"]):
        for agg_id in range(2):
            assert m.test_vec_encode_prep_share(shares[agg_id][i]).hex() == r["prep_shares"][0][agg_id]
            # the vectors list each out-share element's encoding
            assert [m.field.encode_vec([x]).hex() for x in states[agg_id][i][0]] == r["out_shares"][agg_id]
            assert [m.field.encode_vec([x]).hex() for x in out_shares[agg_id][i]] == r["out_shares"][agg_id]
        assert m.test_vec_encode_prep_msg(prep_msgs[i]).hex() == r["prep_messages"][0]
        assert failures[i] is None
    assert valid == [True] * len(tv["prep"])
    assert [m.test_vec_encode_agg_share(a).hex() for a in agg_shares] == tv["agg_shares"]
    assert agg_result == tv["agg_result"]
    # the states are what the poc's own prep_init returns for the same report
    r0 = _reports(m, tv)[0]
    for agg_id in range(2):
        (ost, osh) = m.prep_init(vk, ctx, agg_id, ap, r0[0], r0[1], r0[2][agg_id])
        assert [x.int() for x in ost[0]] == [x.int() for x in states[agg_id][0][0]]
        assert ost[1] == states[agg_id][0][1]
        assert m.test_vec_encode_prep_share(osh) == m.test_vec_encode_prep_share(shares[agg_id][0])
    gpu.close()


@pytest.mark.parametrize("path", [p for p in golden_files() if "Sum_0" in p or "Histogram" in p],
                         ids=os.path.basename)
def test_stub_loop_rejects_a_tampered_report(stub, path):
    """A report whose helper key was tampered with fails the stub's
    prep_shares_to_prep with the poc's 'VIDPF verification failed' and is
    left out of the GPU fold: the agg result is the honest reports'."""
    from oracle import mastic as poc_mastic
    (mod, lib) = stub
    tv = json.load(open(path))
    m = poc_mastic.from_test_vec(tv)
    gpu = mod.MasticHip(lib, m)
    ctx = bytes.fromhex(tv["ctx"])
    vk = bytes.fromhex(tv["verify_key"])
    ap = m.decode_agg_param(bytes.fromhex(tv["agg_param"]))
    reports = _reports(m, tv)
    (key, proof_share, seed, peer_part) = reports[0][2][1]
    reports[0][2][1] = (bytes([key[0] ^ 1]) + key[1:], proof_share, seed, peer_part)
    (_st, _sh, _msgs, failures, valid, _outs, agg_shares, agg_result) = _run_loop(gpu, m, vk, ctx, ap, reports)
    assert str(failures[0]) == "VIDPF verification failed"
    assert valid == [False] + [True] * (len(reports) - 1)
    honest = _reports(m, tv)[1:]
    (_st2, _sh2, _m2, f2, v2, _o2, agg2, res2) = _run_loop(gpu, m, vk, ctx, ap, honest)
    assert all(f is None for f in f2) and all(v2)
    assert [m.test_vec_encode_agg_share(a) for a in agg_shares] == [m.test_vec_encode_agg_share(a) for a in agg2]
    assert agg_result == res2
    gpu.close()


def test_stub_raises_value_error_with_the_library_text(stub):
    """The poc's ValueError cases come back as ValueError carrying the
    library's message (mastic_last_error bound with restype c_char_p)."""
    from oracle import mastic as poc_mastic
    (mod, lib) = stub
    tv = json.load(open(golden_files()[0]))
    m = poc_mastic.from_test_vec(tv)
    gpu = mod.MasticHip(lib, m)
    r = tv["prep"][0]
    rep = (bytes.fromhex(r["nonce"]), m.vidpf.decode_public_share(bytes.fromhex(r["public_share"])),
           m.decode_input_share(0, bytes.fromhex(r["input_shares"][0])))
    bits = m.vidpf.BITS
    bad_level = (bits, ((False,) * (bits + 1),), True)  # level past BITS - 1 (mastic.py:219-220)
    with pytest.raises(ValueError) as e:
        gpu.prep_init_batch(bytes(32), b"ctx", 0, bad_level, [rep])
    assert str(e.value) and not str(e.value).isdigit()
    gpu.close()
