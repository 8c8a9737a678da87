"""MI355X-native batched Mastic aggregator.

Drop-in for the reference's ``Mastic`` API (jimouris/draft-mouris-cfrg-mastic,
``poc/mastic.py``) whose prep_init / decide / aggregate / shard run as
hand-written gfx950 HIP kernels behind the C ABI in ``include/mastic_hip.h``.
"""
from ._lib import LIB_PATH, MasticError, build  # noqa: F401
from .field import Field64, Field128  # noqa: F401
from .vdaf import (Mastic, MasticCount, MasticHistogram, MasticMultihotCountVec,  # noqa: F401
                   MasticSum, MasticSumVec, from_test_vec)
