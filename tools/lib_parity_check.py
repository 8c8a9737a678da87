"""Debug / A-B helper (GPU box): bind a given build of the library and check
its prep shares against the reference's golden vectors (tests/golden), the
same comparison tests/test_gpu_parity.py makes with the in-tree build.

    python3 tools/lib_parity_check.py build/libmastic_<tag>.so

Prints one line per vector and exits non-zero on any mismatch.  Not part of
the product."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "draft-mouris-cfrg-mastic_amd"), os.path.join(ROOT, "tests")]


def main():
    from mastic_amd import _lib
    _lib.load(os.path.abspath(sys.argv[1]))
    import mastic_amd
    from conftest import golden_files
    bad = 0
    for path in golden_files():
        tv = json.load(open(path))
        m = mastic_amd.from_test_vec(tv)
        ctx = bytes.fromhex(tv["ctx"])
        vk = bytes.fromhex(tv["verify_key"])
        ap = m.decode_agg_param(bytes.fromhex(tv["agg_param"]))
        reps = tv["prep"]
        nonces = b"".join(bytes.fromhex(r["nonce"]) for r in reps)
        pub = b"".join(bytes.fromhex(r["public_share"]) for r in reps)
        for a in range(2):
            ins = b"".join(bytes.fromhex(r["input_shares"][a]) for r in reps)
            (ps, _js, _out, _st) = m.prep_init_batch(vk, ctx, a, ap, nonces, pub, ins)
            ok = ps == b"".join(bytes.fromhex(r["prep_shares"][0][a]) for r in reps)
            bad += not ok
            print("%-28s agg %d ctx %dB: %s" % (os.path.basename(path), a, len(ctx), "ok" if ok else "MISMATCH"))
    print("mismatches:", bad)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
