"""Pin the CPU oracle against the reference's own golden vectors.

``tests/golden/Mastic*.json`` are byte-identical copies of the reference's
``test_vec/mastic/*.json`` (written by ``poc/gen_test_vec.py:23-242`` through
``vdaf_poc.test_utils.gen_test_vec_for_vdaf``).  Every field is replayed:
public share, both input shares (client ``shard``), both prep shares
(``prep_init``), the prep message (``prep_shares_to_prep``), both out shares
(``prep_next``), both agg shares (``agg_update``) and the agg result
(``unshard``).  No test in the reference reads these files back; this one does.
"""
import json
import os

import pytest

from conftest import golden_files
from oracle.mastic import from_test_vec


@pytest.mark.parametrize("path", golden_files(), ids=os.path.basename)
def test_reference_vector(path):
    tv = json.load(open(path))
    m = from_test_vec(tv)
    ctx = bytes.fromhex(tv["ctx"])
    vk = bytes.fromhex(tv["verify_key"])
    ap = m.decode_agg_param(bytes.fromhex(tv["agg_param"]))
    assert m.encode_agg_param(ap).hex() == tv["agg_param"]
    assert tv["shares"] == 2
    agg = [m.agg_init(ap), m.agg_init(ap)]
    for rep in tv["prep"]:
        nonce = bytes.fromhex(rep["nonce"])
        rand = bytes.fromhex(rep["rand"])
        assert len(rand) == m.RAND_SIZE
        meas = (tuple(rep["measurement"][0]), rep["measurement"][1])
        (cws, ins) = m.shard(ctx, meas, nonce, rand)
        enc_ps = m.test_vec_encode_public_share(cws)
        assert enc_ps.hex() == rep["public_share"]
        # the decoder round-trips
        assert m.test_vec_encode_public_share(m.vidpf.decode_public_share(enc_ps)) == enc_ps
        for a in range(2):
            enc = m.test_vec_encode_input_share(ins[a])
            assert enc.hex() == rep["input_shares"][a]
            assert m.decode_input_share(a, enc) == ins[a]
        states, shares = [], []
        for a in range(2):
            (st, sh) = m.prep_init(vk, ctx, a, ap, nonce, cws, ins[a])
            states.append(st)
            shares.append(sh)
            enc = m.test_vec_encode_prep_share(sh)
            assert enc.hex() == rep["prep_shares"][0][a]
            assert m.decode_prep_share(ap[2], enc) == sh
        msg = m.prep_shares_to_prep(ctx, ap, shares)
        assert m.test_vec_encode_prep_msg(msg).hex() == rep["prep_messages"][0]
        for a in range(2):
            out = m.prep_next(ctx, states[a], msg)
            assert [m.field.encode_vec([x]).hex() for x in out] == rep["out_shares"][a]
            agg[a] = m.agg_update(ap, agg[a], out)
    for a in range(2):
        assert m.test_vec_encode_agg_share(agg[a]).hex() == tv["agg_shares"][a]
    assert m.unshard(ap, agg, len(tv["prep"])) == tv["agg_result"]
