"""CPU oracle for the Mastic prep_init + aggregate path — TEST INFRASTRUCTURE.

This package is the checker, never the product.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import it.  The product (``draft-mouris-cfrg-mastic_amd/``) never imports,
links or executes anything from here.

What it restates
----------------
* ``poc/dst.py``, ``poc/vidpf.py`` and ``poc/mastic.py`` of the reference
  (jimouris/draft-mouris-cfrg-mastic @ 2025-02-27), function by function, with
  the same per-report / per-node control flow (``oracle/vidpf.py``,
  ``oracle/mastic.py``, ``oracle/dst.py``).
* The un-vendored dependency ``vdaf_poc`` pinned at tag
  ``draft-irtf-cfrg-vdaf-13`` (``poc/requirements.txt:4``): ``field``
  (Field64/Field128), ``xof`` (XofTurboShake128, XofFixedKeyAes128),
  ``flp_bbcggi19`` (FlpBBCGGI19 + Count/Sum/SumVec/Histogram/MultihotCountVec),
  ``common`` and ``idpf_bbcggi21.pack_bits`` (``oracle/field.py``,
  ``oracle/xof.py``, ``oracle/flp.py``, ``oracle/common.py``).  Their source is
  not in the container; the restatement follows the published vdaf-13
  algorithms and is pinned byte-for-byte by the reference's own golden
  vectors ``test_vec/mastic/*.json`` (copied as data to ``tests/golden/``).
* pycryptodomex's C AES-128 and TurboSHAKE128 are replaced by our own C in
  ``oracle/prims.c`` (FIPS-197 / RFC 9861), loaded with ctypes.

Parity is pinned: ``tests/test_oracle_vectors.py`` reproduces every field of
all nine reference vectors.
"""
