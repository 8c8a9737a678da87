"""The reference-side binding (integration/poc/mastic_hip.py, INTEGRATION.md
§3) actually run: the file a poc maintainer would drop next to
``poc/mastic.py``, driven with poc-shaped ``Mastic`` objects.  ``/root/reference``
is not on the GPU box, so the poc-shaped restatement under ``oracle/`` stands
in for ``poc/mastic.py`` (same class names, attributes and wire encoders,
mastic.py:52-614); it only encodes the inputs here, the prep shares come from
the GPU and are checked against the reference's golden vectors
(tests/golden/, byte copies of test_vec/mastic)."""
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


@pytest.mark.parametrize("path", golden_files(), ids=os.path.basename)
def test_stub_reproduces_golden_prep_shares(stub, path):
    from oracle import mastic as poc_mastic
    (mod, lib) = stub
    tv = json.load(open(path))
    m = poc_mastic.from_test_vec(tv)  # the poc-shaped Mastic the maintainer's code holds
    gpu = mod.MasticHip(lib, m)
    ctx = bytes.fromhex(tv["ctx"])
    vk = bytes.fromhex(tv["verify_key"])
    ap = m.decode_agg_param(bytes.fromhex(tv["agg_param"]))
    for agg_id in range(2):
        # the report tuples a poc driver holds (examples.py:12-23): decoded objects
        reports = [(bytes.fromhex(r["nonce"]),
                    m.vidpf.decode_public_share(bytes.fromhex(r["public_share"])),
                    m.decode_input_share(agg_id, bytes.fromhex(r["input_shares"][agg_id])))
                   for r in tv["prep"]]
        got = gpu.prep_init_batch(vk, ctx, agg_id, ap, reports)
        assert [s.hex() for s in got] == [r["prep_shares"][0][agg_id] for r in tv["prep"]]
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
