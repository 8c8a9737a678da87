"""bench.py's N > 1 merge path on CPU (gloo, world size 2), with a stand-in
for the Mastic ctx's communicator entry points (no GPU here):

* ``lib_comm_init`` has no silent fallback: if any rank's
  ``mastic_comm_init`` fails -- or rank 0 cannot create the id -- EVERY rank
  exits non-zero (SystemExit 3), none switches to another merge path, and a
  rank whose own init succeeded releases its communicator first;
* when every rank joins, the bench line's ``comm`` record names the RCCL
  backend, the rank count the library's communicator reports and every
  rank's device; the gloo rehearsal is labelled as such.

The library side (agreement round, bounded waits) is covered on the GPU by
tests/test_gpu_comm.py."""
import os
import socket
import sys

import torch.multiprocessing as mp

from conftest import PKG_ROOT, ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _FakeComm:
    """The ctx entry points lib_comm_init / comm_record use."""

    def __init__(self, world, fail_init=False, fail_id=False):
        self.world = world
        self.fail_init = fail_init
        self.fail_id = fail_id
        self.inited = None
        self.destroyed = False

    def comm_unique_id(self):
        if self.fail_id:
            raise RuntimeError("ncclGetUniqueId failed")
        return bytes(range(128))

    def comm_init(self, nranks, rank, uid, timeout_ms=0):
        if self.fail_init:
            raise RuntimeError("RCCL init: unhandled system error")
        assert len(uid) == 128 and uid == bytes(range(128))
        self.inited = (nranks, rank)

    def comm_info(self):
        return self.inited or (1, 0)

    def comm_destroy(self):
        self.destroyed = True
        self.inited = None


def _worker(rank, world, port, mode, out_q):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, PKG_ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    m = _FakeComm(world, fail_init=(mode == "fail_rank1" and rank == 1), fail_id=(mode == "fail_id"))
    res = {"rank": rank}
    try:
        res["joined"] = bench.lib_comm_init(m, dist, world, rank)
        res["comm"] = bench.comm_record(dist, world, rank, True, m, desc={"local_rank": rank, "name": "stand-in"})
        res["rehearsal"] = bench.comm_record(dist, world, rank, False, m, desc={"local_rank": 0})
    except SystemExit as e:
        res["exit"] = e.code
    res["destroyed"] = m.destroyed
    out_q.put(res)
    dist.destroy_process_group()


def _run(mode, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, mode, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(world):
        r = q.get(timeout=180)
        got[r["rank"]] = r
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return got


def test_comm_record_when_every_rank_joins():
    got = _run("ok")
    for rank in range(2):
        assert got[rank]["joined"] is True
        c = got[rank]["comm"]
        assert c["backend"] == "rccl" and c["nranks"] == 2
        assert [d["rank"] for d in c["devices"]] == [0, 1]
        assert [d["local_rank"] for d in c["devices"]] == [0, 1]
        r = got[rank]["rehearsal"]
        assert r["backend"] == "gloo-rehearsal" and r["nranks"] == 2


def test_failed_init_on_one_rank_exits_every_rank_nonzero():
    got = _run("fail_rank1")
    for rank in range(2):
        assert got[rank].get("exit") == 3, got[rank]
        assert "comm" not in got[rank]
    # the rank whose own init succeeded released its communicator before exiting
    assert got[0]["destroyed"] is True
    assert got[1]["destroyed"] is False


def test_failed_unique_id_exits_every_rank_nonzero():
    got = _run("fail_id")
    for rank in range(2):
        assert got[rank].get("exit") == 3, got[rank]


def test_comm_record_single_process():
    sys.path.insert(0, ROOT)
    import bench
    c = bench.comm_record(None, 1, 0, False, desc={"local_rank": 0})
    assert c["backend"] == "none" and c["nranks"] == 1 and c["devices"][0]["rank"] == 0
