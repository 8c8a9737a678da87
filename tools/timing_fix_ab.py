"""A/B of the round-5 last_timing fix (47221e6), run once on the GPU box:
the scenario of tests/test_gpu_queued_calls.py::test_hit_timing_with_busy_sponge_stream
(a single-chunk frontier-cache hit whose sponge-stream timing marks are held
back by the sponge-delay test hook, then mastic_last_timing3 with no
synchronize) through the -DMASTIC_EXPERIMENT_KNOBS build, with
MASTIC_DBG_TIMING_NOWAIT=1 (last_timing3 as before the fix: no wait on the
marks) and =0 (as shipped).  Expected: the first fails with "device not
ready", the second returns finite times.

  python tools/timing_fix_ab.py            # builds build/libmastic_knobs.so on the CPU side first
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "draft-mouris-cfrg-mastic_amd")
KNOBS = os.path.join(ROOT, "build", "libmastic_knobs.so")

SCENARIO = r"""
import random, sys
sys.path.insert(0, %(pkg)r); sys.path.insert(0, %(tests)r)
from mastic_amd import _lib
_lib.load(%(lib)r)
import mastic_amd
from test_gpu_frontier_cache import _reports
CTX = b"timing-fix-ab"
rng = random.Random(95)
m = mastic_amd.MasticCount(8)
(alphas, weights, nonces, rands) = _reports(m, rng, 128, 5)
(pub, in0, in1) = m.shard_batch(CTX, alphas, weights, nonces, rands)
dev = m.reports_upload(nonces, pub, in0, in1)
m.set_frontier_cache(True)
m.prep_init_device(dev, bytes(16), CTX, 0, (0, ((False,), (True,)), False))
m.synchronize()
m.set_test_sponge_delay(400000)
m.prep_init_device(dev, bytes(16), CTX, 0, (1, ((False, False), (False, True), (True, False), (True, True)), False))
assert m.last_prep_was_cached()
try:
    print("RESULT ok", m.last_timing3())
except Exception as e:
    print("RESULT failed:", e)
m.synchronize()
"""


def main():
    if "--build" in sys.argv or not os.path.exists(KNOBS):
        sys.path.insert(0, PKG)
        from mastic_amd import _lib
        _lib.build(out=KNOBS, defines=("MASTIC_EXPERIMENT_KNOBS",), force=True)
        if "--build" in sys.argv:
            return 0
    code = SCENARIO % {"pkg": PKG, "tests": os.path.join(ROOT, "tests"), "lib": KNOBS}
    for nowait in ("1", "0"):
        env = dict(os.environ, MASTIC_DBG_TIMING_NOWAIT=nowait)
        r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
        res = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT")]
        print("MASTIC_DBG_TIMING_NOWAIT=%s (%s): %s" % (
            nowait, "last_timing3 as before 47221e6" if nowait == "1" else "as shipped",
            res[0] if res else "no result, rc %d: %s" % (r.returncode, r.stderr[-500:])), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
