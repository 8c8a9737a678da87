"""Probe (GPU box): mastic_comm_init for 2 ranks with no second rank, traced
(MASTIC_TRACE_COMM=1): which init path RCCL takes and whether the timeout
and ncclCommAbort return.  Prints a progress line per step."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "draft-mouris-cfrg-mastic_amd"))
os.environ["MASTIC_TRACE_COMM"] = "1"
import mastic_amd  # noqa: E402
from mastic_amd._lib import MasticError  # noqa: E402

m = mastic_amd.Mastic(6, "Sum", max_measurement=9)
print("ctx ok", flush=True)
uid = m.comm_unique_id()
print("uid ok", flush=True)
t0 = time.time()
try:
    m.comm_init(2, 0, uid, timeout_ms=3000)
    print("RESULT joined", flush=True)
except MasticError as e:
    print("RESULT code=%d after=%.1f msg=%s" % (e.code, time.time() - t0, e), flush=True)
print("INFO", m.comm_info(), flush=True)
m.comm_init(1, 0, m.comm_unique_id(), timeout_ms=3000)
print("INFO2", m.comm_info(), m.merge_host(bytes(16), 2, 1).hex(), flush=True)
